"""The bench's stdout line, kept small enough for the driver to parse.

The driver keeps only the last few KB of a bench's stdout, so a line that
grows past that (round 3: 29.8 KB) is not parsed at all.  ``bench.py`` and
``distributed.bench_distributed`` therefore print a compact line — the
required keys, a compact ``roofline`` and ``cpu_baseline``, one short object
per extra workload — and write everything else to a detail file
(``gpurun_out/bench_detail.json`` by default).  ``fit`` drops optional keys,
least important first, until the line is under ``LINE_BUDGET`` bytes.
"""
from __future__ import annotations

import json
import os
import sys
from typing import Dict, Iterable, Optional

LINE_BUDGET = 6000  # bytes; the driver parsed a 9.0 KB tail in round 2, not 29.8 KB in round 3

REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")


def sig(v, digits: int = 4):
    """Round floats (recursively) to `digits` significant digits."""
    if isinstance(v, float):
        if v != v or v in (float("inf"), float("-inf")):
            return None
        return float(f"{v:.{digits}g}")
    if isinstance(v, dict):
        return {k: sig(x, digits) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [sig(x, digits) for x in v]
    return v


def write_detail(obj: Dict, path: Optional[str]) -> Optional[str]:
    """The full-detail JSON to `path`; returns the path written (None if it
    could not be written: the line must never fail for this)."""
    if not path:
        return None
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(obj, f, indent=1, default=str)
        rel = os.path.relpath(os.path.abspath(path))
        return path if rel.startswith("..") else rel
    except OSError as exc:
        print(f"[bench] detail file not written: {exc}", file=sys.stderr, flush=True)
        return None


def fit(line: Dict, drop_order: Iterable[str], budget: int = LINE_BUDGET) -> Dict:
    """Drop optional top-level keys in `drop_order` until json.dumps(line)
    fits `budget` bytes.  Required keys are never dropped."""
    line = dict(line)
    for key in drop_order:
        if len(json.dumps(line)) <= budget:
            break
        if key not in REQUIRED:
            line.pop(key, None)
    n = len(json.dumps(line))
    if n > budget:  # cannot happen with the keys above; say so rather than print a long line
        line = {k: line[k] for k in REQUIRED if k in line}
        line["truncated"] = f"compact line was {n} B > {budget} B; see the detail file"
    return line


def _get(d, *path):
    for p in path:
        if not isinstance(d, dict) or p not in d:
            return None
        d = d[p]
    return d


def _roofline(r: Dict) -> Dict:
    fab = r.get("fabric") or {}
    l2 = r.get("l2") or {}
    return {"bound": r["bound"], "achieved": r["achieved"], "peak": r["peak"], "unit": r["unit"],
            "frac": r["frac"], "traffic": r.get("traffic"), "kernel": r.get("kernel"),
            "kernel_ms": r.get("kernel_ms"),
            "algorithmic_bytes_per_launch": r.get("algorithmic_bytes_per_launch"),
            "algorithmic_model": "compulsory bytes: col 4/edge, rowptr+schedule 8/row, Wh table "
                                 "once, s_dst 4H/row, output 4C/row (DESIGN.md §5)",
            "frac_8d": r.get("frac_8d"), "achieved_8d": r.get("achieved_8d"),
            "model_8d": "SURVEY.md §8(d): (4 + 4HF + 4H) B/edge + (4 + 4H + 4C) B/row, every "
                        "gather as if from HBM (> 1: rows re-read from L2 / Infinity Cache)",
            "traffic_x_algorithmic": fab.get("x_compulsory"), "l2_hit": fab.get("l2_hit_rate"),
            "l2_gather_ceiling_frac": l2.get("frac_of_gather_ceiling")}


def _workload(w: Dict, cpu: Optional[Dict]) -> Dict:
    r = w.get("roofline") or {}
    fab = r.get("fabric") or {}
    d = {"value": w["value"], "ms": w["ms_per_step"], "edge_ms": _get(w, "edge_kernel", "ms"),
         "project_ms": _get(w, "projection", "ms"), "hbm_frac": r.get("frac"),
         "fabric_x": fab.get("x_compulsory"), "l2_hit": fab.get("l2_hit_rate"),
         "l2_gather_frac": _get(r, "l2", "frac_of_gather_ceiling"),
         "project_kernel": _get(w, "projection", "kernel"),
         "in_step": {k: v for k, v in (w.get("phases_in_step_ms") or {}).items() if k != "what"}
                    or None}
    if cpu:
        d["cpu_value"] = cpu.get("value")
    tr = w.get("training")
    if tr:
        d["train_step_ms"] = tr.get("train_step_ms")
        d["train_x_eval"] = tr.get("x_eval_forward")
    if "vs_uniform_reddit" in w:
        d["vs_uniform"] = w["vs_uniform_reddit"]
    return d


def compact_single(result: Dict, detail_path: Optional[str]) -> Dict:
    """The N = 1 line: required keys, roofline, cpu_baseline, one short object
    per extra workload, the per-P compute bounds of the emulated partition."""
    line = {k: result[k] for k in REQUIRED if k in result}
    line["roofline"] = _roofline(result["roofline"])
    cb = result.get("cpu_baseline")
    if cb:
        host = cb.get("host") or {}
        line["cpu_baseline"] = {"value": cb["value"], "unit": cb["unit"], "cores": cb["cores"],
                                "kind": cb["kind"], "sample": cb.get("sample"),
                                "host": f"{host.get('model')}, {host.get('physical_cores')} "
                                        f"physical cores, cgroup quota "
                                        f"{host.get('cgroup_cpu_quota')}"}
    line["breakdown_ms"] = result.get("breakdown_ms")
    pj = result.get("projection")
    if pj:
        line["projection"] = {k: pj.get(k) for k in ("kernel", "bound", "achieved", "peak",
                                                       "unit", "frac", "hbm_frac",
                                                       "mfma_busy_frac_pmc")}
    cpus = result.get("cpu_baselines") or {}
    line["workloads"] = {nm: _workload(w, cpus.get(nm))
                         for nm, w in (result.get("workloads") or {}).items()}
    ns = _get(result, "workloads", "reddit", "north_star")
    if ns:
        line["north_star_reddit"] = {"target": ns["target_edges_per_s"], "value": ns["value"],
                                     "met": ns["met"]}
    emu = {}
    for wl, d in (result.get("multi_gpu_emulated") or {}).items():
        if not isinstance(d, dict):
            continue
        emu[wl] = {k: {"proj": v.get("max_project_ms"), "edge": v.get("max_edge_passes_ms"),
                       "compute": v.get("max_compute_ms"),
                       "bound": v.get("compute_only_speedup_bound"),
                       "bound_eager": v.get("compute_only_speedup_bound_eager")}
                   for k, v in d.items() if isinstance(v, dict)}
    if emu:
        line["multi_gpu_emulated"] = emu
        line["multi_gpu_emulated_what"] = ("per-rank GPU ms of the node-partitioned step on one "
                                           "GPU (graph-replayed launches), max over ranks; bound "
                                           "= 1-GPU step / max compute (collective excluded); "
                                           "bound_eager: the same with eager launches")
    tr = result.get("training")
    if tr:
        line["training"] = {"step_ms": tr.get("train_step_ms"),
                            "graph_step_ms": tr.get("train_step_graph_ms"),
                            "x_eval": tr.get("x_eval_forward")}
    if result.get("pmc_error"):
        line["pmc_error"] = str(result["pmc_error"])[:200]
    line["detail"] = detail_path
    line = sig(line)
    return fit(line, ("multi_gpu_emulated_what", "training", "projection", "north_star_reddit",
                      "multi_gpu_emulated", "breakdown_ms", "workloads", "pmc_error"))


def compact_dist(res: Dict, detail_path: Optional[str]) -> Dict:
    """The N > 1 line: required keys plus the headline's one-GPU comparison,
    its phase times, and one short object per extra workload."""
    line = {k: res[k] for k in REQUIRED if k in res}
    head = res.get("headline_detail") or {}

    def phases(d):
        if not d:
            return None
        return {"strategy": d.get("strategy"), "launch": d.get("launch", "eager"),
                "value": d.get("value"),
                "ms": d.get("ms_per_step"), "collective_ms": d.get("collective_ms"),
                "project_ms": d.get("project_ms_max_over_ranks"),
                "edge_ms": d.get("edge_passes_ms_max_over_ranks"),
                "recv_bytes": d.get("collective_bytes_received_per_rank"),
                "speedup": d.get("speedup_vs_one_gpu"),
                "check_max_abs_diff": _get(d, "check", "max_abs_diff_vs_one_gpu")}

    line["one_gpu_value"] = _get(res, "one_gpu_same_workload", "value")
    line["speedup_vs_one_gpu"] = res.get("speedup_vs_one_gpu")
    line["headline"] = phases(head)
    line["replicate"] = phases(res.get("replicate"))

    def graph(d):
        g = (d or {}).get("graph")
        if not g:
            return None
        return {"ok": g.get("ok"), "value": g.get("value"), "ms": g.get("ms_per_step"),
                "eager_value": _get(d, "eager", "value"), "error": g.get("error")}
    line["graph"] = graph(head)
    line["strategy_trials_ms"] = head.get("strategy_trials_ms")
    wls = {}
    for nm, w in (res.get("workloads") or {}).items():
        wls[nm] = {"value": w.get("value"), "ms": w.get("ms_per_step"),
                   "strategy": w.get("strategy"), "launch": w.get("launch", "eager"),
                   "graph": graph(w), "one_gpu_value": _get(w, "one_gpu", "value"),
                   "speedup": w.get("speedup_vs_one_gpu"),
                   "collective_ms": w.get("collective_ms"),
                   "collective_bytes_received_per_rank":
                       w.get("collective_bytes_received_per_rank"),
                   "replicate": phases(w.get("replicate"))}
    line["workloads"] = wls
    weak = res.get("ppi_blocks_data_parallel")
    if weak:
        line["ppi_blocks_data_parallel"] = {"value": weak.get("value"),
                                            "ms": weak.get("ms_per_step"), "scaling": "weak"}
    line["detail"] = detail_path
    line = sig(line)
    return fit(line, ("strategy_trials_ms", "ppi_blocks_data_parallel", "replicate",
                      "headline", "workloads"))
