// MI355X GAT edge kernel: segmented softmax + aggregation over the CSR by
// target (GAT.py:53-67).  Kernels k_edge_fwd, k_edge_grp, k_edge_merge_wg; C-ABI
// gat_edge_aggregate*, gat_edge_merge, gat_layer_forward.

#include "gat_common.h"

#include <type_traits>

namespace {

// ---------------------------------------------------------------------------
// Edge kernel: one wavefront (= one 64-thread workgroup) per target row.
//
// For each chunk of C in-edges of row r:
//   score phase  lane (k, h) slots: e = LeakyReLU(s_dst[r,h] + s_src[col_k,h]),
//                chunk max per head by xor-shuffle, online rescale of (m, l),
//                p = exp(e - m) staged in LDS.
//   gather phase LPE lanes per edge, each a float4 of the source's Wh row
//                (one 256 B coalesced row read per edge at HF = 64),
//                acc += p[head] * Wh.  U steps in flight per lane.
// Row end: acc reduced across edge slots, divided by (l + 1e-16) (PyG
// softmax's epsilon), concat -> +bias, mean -> head mean via LDS, +bias.
// Optional lse[r,h] = m + log(l) for the backward pass.
// ---------------------------------------------------------------------------
// LPE (lanes per edge, a power of two <= 64) is a run-time argument: this
// kernel serves the shapes the lane-group kernel cannot (F % 4 != 0, head
// means of odd widths), where one instance per head-count class is enough.
template <int HP>
__global__ __launch_bounds__(64) void k_edge_fwd(
    const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ order,
    int row_begin, int row_end,
    const float* __restrict__ Wh, int ld_wh, const float* __restrict__ Ss, int ld_s,
    const float* __restrict__ s_dst,
    int H, int F, int HF, int concat, int act, float slope, const float* __restrict__ bias,
    float* __restrict__ out, int ld_out, float* __restrict__ lse, DropArgs drop_arg,
    float* __restrict__ y_heads, int LPE) {
    const DropArgs drop = resolve_drop(drop_arg);
    constexpr int C = (512 / HP) < kWave ? (512 / HP) : kWave;  // edges per chunk
    constexpr int R = C * HP / kWave;                          // score slots per lane
    constexpr int U = 4;                                       // gather steps in flight
    const int EPI = kWave / LPE;                               // edges per gather step
    __shared__ int col_s[C];
    __shared__ float p_s[C * HP];
    __shared__ float hv_s[HP];
    __shared__ float y_s[kWave * 4];

    const int lane = threadIdx.x;
    const int pos = row_begin + blockIdx.x;
    if (pos >= row_end) return;
    const int r = order != nullptr ? order[pos] : pos;
    const int e0 = rowptr[r], e1 = rowptr[r + 1];

    const int hs = lane & (HP - 1);
    const bool hs_ok = hs < H;
    const float sd = hs_ok ? s_dst[(size_t)r * H + hs] : 0.f;
    float m_run = -INFINITY, l_run = 0.f;

    const int c = lane & (LPE - 1);
    const int slot = lane / LPE;
    const bool c_ok = 4 * c < HF;
    const int coff = c_ok ? 4 * c : 0;
    int hq[4];
    bool cq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int f = 4 * c + q;
        cq[q] = f < HF;
        hq[q] = cq[q] ? f / F : 0;
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};

    for (int base = e0; base < e1; base += C) {
        const int nk = min(C, e1 - base);
        if (lane < nk) col_s[lane] = col[base + lane];
        __syncthreads();

        float ev[R];
        float mloc = -INFINITY;
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int k = (lane + kWave * q) / HP;
            const bool valid = k < nk && hs_ok;
            const int j = col_s[k < nk ? k : nk - 1];
            const float z = sd + Ss[(size_t)j * ld_s + (hs_ok ? hs : 0)];
            float e = act == GAT_ACT_HEAD_SOFTMAX ? head_softmax<HP>(z, valid)
                                                  : score_act(act, z, slope);
            e = valid ? e : -INFINITY;
            ev[q] = e;
            mloc = fmaxf(mloc, e);
        }
#pragma unroll
        for (int off = HP; off < kWave; off <<= 1) mloc = fmaxf(mloc, __shfl_xor(mloc, off));
        const float m_new = fmaxf(m_run, mloc);
        const float scale = hs_ok ? expf(m_run - m_new) : 1.f;
        l_run *= scale;
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const float p = (ev[q] == -INFINITY) ? 0.f : expf(ev[q] - m_new);
            l_run += p;  // the softmax denominator never sees the dropout
            float pd = p;
            if (drop.thresh != 0u && p != 0.f)
                pd = p * drop_factor(drop, base + (lane + kWave * q) / HP, hs, H);
            p_s[lane + kWave * q] = pd;
        }
        if (lane < HP) hv_s[lane] = scale;
        m_run = m_new;
        __syncthreads();

        acc.x *= hv_s[hq[0]];
        acc.y *= hv_s[hq[1]];
        acc.z *= hv_s[hq[2]];
        acc.w *= hv_s[hq[3]];

        for (int k0 = 0; k0 < nk; k0 += EPI * U) {
            f32x4 v[U];
            f32x4 pv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int k = k0 + u * EPI + slot;
                const bool ok = k < nk;
                const int kk = ok ? k : nk - 1;
                const int j = col_s[kk];
                v[u] = *reinterpret_cast<const f32x4*>(Wh + (size_t)j * ld_wh + coff);
                const float* pr = p_s + kk * HP;
                const float g = ok ? 1.f : 0.f;
                pv[u] = f32x4{pr[hq[0]] * g, pr[hq[1]] * g, pr[hq[2]] * g, pr[hq[3]] * g};
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc += pv[u] * v[u];
        }
        __syncthreads();
    }

#pragma unroll
    for (int off = HP; off < kWave; off <<= 1) l_run += __shfl_xor(l_run, off);
    for (int off = LPE; off < kWave; off <<= 1) {
        acc.x += __shfl_xor(acc.x, off);
        acc.y += __shfl_xor(acc.y, off);
        acc.z += __shfl_xor(acc.z, off);
        acc.w += __shfl_xor(acc.w, off);
    }
    if (lane < HP) hv_s[lane] = 1.f / (l_run + 1e-16f);
    if (lse != nullptr && lane < H) lse[(size_t)r * H + lane] = m_run + logf(l_run);
    __syncthreads();
    float y[4] = {acc.x * hv_s[hq[0]], acc.y * hv_s[hq[1]], acc.z * hv_s[hq[2]],
                  acc.w * hv_s[hq[3]]};
    if (y_heads != nullptr && slot == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (cq[q]) y_heads[(size_t)r * HF + 4 * c + q] = y[q];
    }
    if (concat) {
        if (slot == 0 && c_ok) {
            float* o = out + (size_t)r * ld_out + 4 * c;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (cq[q]) o[q] = y[q] + bias[4 * c + q];
        }
    } else {
        if (slot == 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (cq[q]) y_s[4 * c + q] = y[q];
        }
        __syncthreads();
        for (int f = lane; f < F; f += kWave) {
            float s = 0.f;
            for (int h = 0; h < H; ++h) s += y_s[h * F + f];
            out[(size_t)r * ld_out + f] = s / (float)H + bias[f];
        }
    }
}

// ---------------------------------------------------------------------------
// Edge kernel, lane-group variant (F % 4V == 0): G = next_pow2(HF/4)/V lanes
// per target row, each lane owning V float4s (4V columns of ONE head), 64/G
// rows per wave, one row per group.
//
// Each lane runs its head's online softmax in registers, so the hot loop has
// no LDS traffic, no barriers and no cross-lane reductions beyond the score's.
// Per chunk of U in-edges: one coalesced col load (software-pipelined: the
// next chunk's indices are in flight while this chunk gathers), U broadcasts
// by shuffle, then U*V independent Wh float4 gathers in flight per lane and
// one rescale per chunk.
// FUSED: the source score s_src[j,h] = Wh[j,h].a1_h + c1_h is recomputed from
// the gathered row (4V FMAs + a DPP sum over the head's F/4V lanes) instead
// of being gathered — one VMEM instruction and up to a cache line less per
// edge.  Softmax runs in log2 units: e' = LeakyReLU(z) * log2(e), p = 2^(e'-m').
// row_order (optional): target rows in descending in-degree order, so the
// rows sharing a wave have near-equal lengths and the heaviest start first.
// Head mean (concat=False, F/4V a power of two) is an xor-butterfly.
//
// Rows are described by an EdgeRows: the edge range of a row is
// [eb[i], ee[i]) with i = the row id (eb = rowptr, ee = rowptr + 1 for the
// plain forward) or, by_pos, the schedule position.  A row may be a SEGMENT
// of a target row's in-edges, with the online-softmax state (m in log2 units,
// l, un-normalised acc) carried in memory:
//   * multi-GPU passes (distributed.py): pass c covers the sources that arrived
//     with all-gather chunk c, loading the state pass c-1 stored;
//   * hub rows (degree skew): the segments of one long row run in parallel as
//     separate "virtual rows", and k_edge_merge_wg combines their states.
// ---------------------------------------------------------------------------

// KINK (training forward, recompute backward): also the per-head "kink sums"
//   Q[i,h] = sum_j A_ij L'(z_ij) Wh[j,h]   and   R[i,h] = sum_j alpha_ij L'(z_ij)
// (A = dropped coefficient, alpha = undropped, L' = 1 for z > 0 else slope).  The
// backward's dL/ds_dst[i,h] = sum_j alpha_ij L'_ij (drop_ij dy_i.Wh_j - delta_i)
// is then dy_i.Q_i - delta_i R_i: an elementwise kernel (k_bwd_table) instead of
// a second pass over every in-edge (k_bwd_targets).  Q and R cost one more
// accumulator per float4 and no gathers: the loop already holds Wh_j and p_ij.
// S = 2 or 4 (short rows, few rows per launch): S lane groups per row, group
// g walking chunks g, g + S, g + 2S, ... of the row's in-edges; at the end each
// lane merges its online-softmax state with its partners' (lane ^ G, then
// lane ^ 2G): M = max(m, m'), l = l 2^(m-M) + l' 2^(m'-M), acc likewise (the
// hub merge, in registers).  The chain of dependent chunk loads per row is S
// times shorter and a launch has S times the waves.  Only group 0 stores.
// Not with KINK or PIPE.
// HL (> 0): the head's lane count F/4V as a constant (the launcher
// instantiates it for the HF = 64 lane groups), so the per-edge score sums
// compile without branches; 0: read from F at run time.
// XF (> 0): the small-Fin fused forward (fin == XF <= 4): each gathered source's
// x row is projected in registers (Wh_j = x_j W^T + b for the lane's four
// columns, the fp32 FMA chain in k order, then + b, as GAT.py:43) and the
// target's s_dst is formed the same way from x_i; the kernel reads no Wh
// table.  At CIFAR's Fin = 3 a gathered edge is 12 B of x instead of a 128-B
// or 256-B Wh row, and the projection launch disappears.
template <int N>
struct XRow {  // one x row of the small-Fin form: N floats, 4-B aligned
    float v[N];
};

// RC (> 0; U = 4, quad-broadcast ids, S = 1, not PIPE): a row's col values are
// loaded 8 chunks at a time, one load per lane and register for 8 / (G / 4)
// chunks (chunk t's four ids in quad t % (G/4) of the group), instead of one
// chunk ahead: the col stream comes from HBM, and its per-chunk round trip
// was the walk's critical path at short rows (tools/edge_bisect.hip: a
// memory-only PPI walk 24.4 -> 21.4 us).  Same chunks, ids and order:
// results are bitwise the one-chunk-ahead form's.
// LEAN (eval, rows < 1024 edges: GAT_HINT_SHORT): no Kahan sums and no dropout
// code, so the registers they hold go to RC = 2's second chunk in flight.
// RC = 2 (LEAN only): the row-batched ids AND the gathers one chunk ahead.
template <int G, int U, int V, bool FUSED, bool PIPE = false, bool KINK = false, int S = 1,
          int HL = 0, int XF = 0, int RC = 0, bool LEAN = false>
__global__ __launch_bounds__(256) void k_edge_grp(
    const EdgeRows er, const int* __restrict__ col, const int* __restrict__ order,
    int row_begin, int row_end,
    const float* __restrict__ Wh, int ld_wh, const float* __restrict__ Ss, int ld_s,
    const float* __restrict__ a_src, const float* __restrict__ c_src,
    const float* __restrict__ s_dst, int H, int F, int HF, int concat, float slope,
    const float* __restrict__ bias, float* __restrict__ out, int ld_out,
    float* __restrict__ lse, DropArgs drop_arg, float* __restrict__ y_heads,
    int nslices, int slice_w, long long slice_stride, float* __restrict__ q_heads,
    float* __restrict__ r_heads, int store_wt, XProjArgs xp) {
    const DropArgs drop = resolve_drop(drop_arg);
    static_assert(S == 1 || ((S == 2 || S == 4) && !KINK && !PIPE && G * S <= kWave), "split rows");
    static_assert(XF == 0 || (V == 1 && FUSED && !KINK && !PIPE && S == 1), "small-Fin form");
    static_assert(RC == 0 || (U == 4 && G >= 4 && S == 1 && !PIPE), "row-batched col values");
    static_assert(!LEAN || (!KINK && XF == 0), "lean: the eval forward");
    static_assert(RC != 2 || LEAN, "pipelined row-batched ids: lean only");
    // col values held per lane per chunk.  Groups of >= 4 lanes: every quad of
    // the group holds the chunk's indices (lane c: edges (c & 3) + 4t), so the
    // source ids are broadcast by DPP within the quad instead of LDS permutes
    constexpr bool QB = G >= 4 && U % 4 == 0;
    constexpr int CL = QB ? U / 4 : (U + G - 1) / G;
    const int lane = threadIdx.x & 63;
    const int c = lane & (G - 1);
    const int gbase = lane & ~(G - 1);
    const int cstep = QB ? 4 : G;        // col slot stride per held value
    const int cfirst = QB ? (c & 3) : c;  // this lane's first col slot
    // sliced node table (nslices > 1): block b works on column slice b % nslices,
    // so with round-robin block placement one XCD gathers from one slice plane
    // only — an [N, slice_w] plane small enough to stay in that XCD's L2
    const int sl = nslices > 1 ? (int)(blockIdx.x % (unsigned)nslices) : 0;
    const unsigned blk = nslices > 1 ? blockIdx.x / (unsigned)nslices : blockIdx.x;
    const int pos = row_begin + (int)((blk * (size_t)blockDim.x + threadIdx.x) / (G * S));
    if (pos >= row_end) return;
    const int half = S > 1 ? (lane / G) & (S - 1) : 0;  // S > 1: which chunks of the row
    const int r = order != nullptr ? order[pos] : pos;
    const int sw = nslices > 1 ? slice_w : HF;  // columns this block's groups own
    const bool c_ok = 4 * V * c < sw;
    const int loff = c_ok ? 4 * V * c : 0;      // column within the slice
    const int coff = sl * slice_w + loff;       // column of the layer output
    const float* __restrict__ Whs = Wh + (size_t)sl * (size_t)slice_stride + loff;
    const int h = coff / F;
    f32x4 a4[V];
    float c1 = 0.f;
#pragma unroll
    for (int q = 0; q < V; ++q) a4[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (FUSED) {
        // a1 pre-scaled by log2(e): the recomputed score comes out in log2 units
        if (c_ok) {
#pragma unroll
            for (int q = 0; q < V; ++q)
                a4[q] = *reinterpret_cast<const f32x4*>(a_src + coff + 4 * q) * kLog2e;
        }
        c1 = c_src[h];
    }
    // XF (= fin): the lane's four columns of W and b (zero past HF)
    float wl[4][XF > 0 ? XF : 1], bl[4];
    if constexpr (XF > 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int cc = c_ok ? coff + q : 0;
            bl[q] = c_ok ? xp.b[cc] : 0.f;
#pragma unroll
            for (int k = 0; k < XF; ++k) {
                const float wv = xp.w[(size_t)cc * XF + k];
                wl[q][k] = c_ok ? wv : 0.f;
            }
        }
    }
    // x_j W^T + b for the lane's columns: the row's XF floats in ONE load
    // (global_load_dwordx<XF>; per-element loads made the kernel load-issue
    // bound), then the fp32 FMA chain in k order
    auto xproj = [&](int j) {
        f32x4 wh = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (XF > 0) {
            const XRow<XF> xr = *reinterpret_cast<const XRow<XF>*>(xp.x + (size_t)j * XF);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float t = 0.f;
#pragma unroll
                for (int k = 0; k < XF; ++k) t = __builtin_fmaf(xr.v[k], wl[q][k], t);
                wh[q] = t + bl[q];
            }
        }
        return wh;
    };
    const int si = er.by_pos ? pos : r;  // segment / state index
    const int e0 = er.eb[si], e1 = er.ee[si];
    const bool kahan = !LEAN && e1 - e0 >= 1024;
    const bool dropping = !LEAN && drop.thresh != 0u;  // kernel-uniform: a scalar branch
    // the target's share of every score, in log2 units (LeakyReLU is positively
    // homogeneous: LReLU(z) log2e = LReLU(z log2e)); + c1 when s_src is recomputed
    float sdv;
    if constexpr (XF > 0) {
        // s_dst[i, h] = Wh_i . a2_h + c2_h from the target's own x row
        const f32x4 whi = xproj(r);
        const f32x4 a2v = c_ok ? *reinterpret_cast<const f32x4*>(xp.a_dst + coff)
                               : f32x4{0.f, 0.f, 0.f, 0.f};
        const float t = whi.x * a2v.x + whi.y * a2v.y + whi.z * a2v.z + whi.w * a2v.w;
        sdv = group_sum16(t, HL > 0 ? HL : F / 4) + xp.c_dst[h];
    } else {
        sdv = s_dst[(size_t)r * H + h];
    }
    const float sd = (sdv + c1) * kLog2e;
    float m = -INFINITY, l = 0.f;  // running max in log2 units
    // rows of >= 1024 edges keep Kahan-compensated running sums (lc, cmp) over
    // per-chunk partial sums: a 10k-edge hub row otherwise accumulates more fp32
    // error than the reference's own.  Shorter rows add directly (cheaper).
    // (the kink sums Q, R get the same compensation on those rows: the backward
    // forms ds_dst = dy.Q - delta R, a difference of two large sums)
    f32x4 acc[V], cmp[V], accq[V], cmpq[V];
    float lc = 0.f, racc = 0.f, rc = 0.f;
#pragma unroll
    for (int q = 0; q < V; ++q) acc[q] = cmp[q] = accq[q] = cmpq[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (er.load && half == 0) {  // continue a row whose earlier segments a previous pass ran
        m = er.st_ml[(size_t)si * 2 * H + h];
        l = er.st_ml[(size_t)si * 2 * H + H + h];
        if (c_ok) {
#pragma unroll
            for (int q = 0; q < V; ++q)
                acc[q] = *reinterpret_cast<const f32x4*>(er.st_acc + (size_t)si * er.ld_st + coff + 4 * q);
        }
    }

    // col indices are software-pipelined: chunk k+U's are in flight while
    // chunk k gathers (loads unconditional, clamped to the row's last edge)
    int cv[CL];
#pragma unroll
    // an empty row (possible only through a caller-built CSR: gat_csr_build adds a
    // self-loop to every row) loads nothing and stores the bias
    for (int t = 0; t < CL; ++t)
        cv[t] = e1 > e0 ? col[min(e0 + half * U + cfirst + t * cstep, e1 - 1)] : 0;
    // gathers of one chunk: source ids broadcast from the group's col values
    auto fetch = [&](const int (&cc)[CL], f32x4 (&v)[U][V], float (&s)[U]) {
        int j[U];
        if constexpr (QB) {
#pragma unroll
            for (int u = 0; u < U; u += 4) {
                j[u + 0] = quad_bcast<0>(cc[u / 4]);
                j[u + 1] = quad_bcast<1>(cc[u / 4]);
                j[u + 2] = quad_bcast<2>(cc[u / 4]);
                j[u + 3] = quad_bcast<3>(cc[u / 4]);
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) j[u] = __shfl(cc[u / G], gbase + (u % G));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (XF > 0) {
                v[u][0] = xproj(j[u]);
            } else {
                const float* row = Whs + (size_t)j[u] * ld_wh;
#pragma unroll
                for (int q = 0; q < V; ++q) v[u][q] = *reinterpret_cast<const f32x4*>(row + 4 * q);
                if constexpr (!FUSED) s[u] = Ss[(size_t)j[u] * ld_s + h];
            }
        }
    };
    // scores, online softmax and accumulation of one gathered chunk
    auto consume = [&](int k, f32x4 (&v)[U][V], float (&s)[U]) {
        const int nk = min(U, e1 - k);
        if constexpr (FUSED) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                // two-lane packed partial sums (v_pk_fma_f32 on the row's own
                // register pairs, no operand shuffling)
                f32x2 d2 = f32x2{0.f, 0.f};
#pragma unroll
                for (int q = 0; q < V; ++q) {
                    d2 += f32x2{v[u][q].x, v[u][q].y} * f32x2{a4[q].x, a4[q].y};
                    d2 += f32x2{v[u][q].z, v[u][q].w} * f32x2{a4[q].z, a4[q].w};
                }
                s[u] = d2.x + d2.y;
            }
            const int hl = HL > 0 ? HL : F / (4 * V);  // lanes per head
            if (hl > 1) {
                if (hl <= 16) {  // the head's lanes sit in one 16-lane DPP row
#pragma unroll
                    for (int u = 0; u < U; ++u) s[u] = group_sum16(s[u], hl);
                } else {
                    for (int off = 1; off < hl; off <<= 1)
#pragma unroll
                        for (int u = 0; u < U; ++u) s[u] += __shfl_xor(s[u], off);
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) s[u] *= kLog2e;  // gathered s_src: natural units
        }
        float emax = -INFINITY;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float z = sd + s[u];  // log2 units
            s[u] = u < nk ? fmaxf(z, z * slope) : -INFINITY;  // slope in [0, 1]
            emax = fmaxf(emax, s[u]);
        }
        const float m_new = fmaxf(m, emax);
        const float scale = __builtin_amdgcn_exp2f(m - m_new);
        l *= scale;
#pragma unroll
        for (int q = 0; q < V; ++q) acc[q] *= scale;
        if constexpr (KINK) {
            racc *= scale;
#pragma unroll
            for (int q = 0; q < V; ++q) accq[q] *= scale;
        }
        // kink sums of one edge (s[u] = LReLU(z) log2e has the sign of z), into
        // (rr, qq): the running sums, or a Kahan row's chunk partials
        auto kink = [&](int u, float p, float pa, float& rr, f32x4 (&qq)[V]) {
            if constexpr (KINK) {
                const float lk = s[u] > 0.f ? 1.f : slope;
                rr += p * lk;
                const float pq = pa * lk;
#pragma unroll
                for (int q = 0; q < V; ++q) qq[q] += pq * v[u][q];
            }
        };
        // (dropout is kernel-uniform: one branch per chunk, not one per edge)
        auto plain = [&](auto drc) {
            constexpr bool DR = decltype(drc)::value;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float p = __builtin_amdgcn_exp2f(s[u] - m_new);
                l += p;  // the softmax denominator never sees the dropout
                float pa = p;
                if constexpr (DR) pa = p * drop_factor(drop, k + u, h, H);
#pragma unroll
                for (int q = 0; q < V; ++q) acc[q] += pa * v[u][q];
                kink(u, p, pa, racc, accq);
            }
        };
        if constexpr (LEAN) {
            plain(std::false_type{});
        } else if (!kahan) {
            if (dropping) plain(std::true_type{});
            else plain(std::false_type{});
        } else {
            lc *= scale;
#pragma unroll
            for (int q = 0; q < V; ++q) cmp[q] *= scale;
            float ls = 0.f, rs = 0.f;
            f32x4 cs[V], qs[V];
#pragma unroll
            for (int q = 0; q < V; ++q) cs[q] = qs[q] = f32x4{0.f, 0.f, 0.f, 0.f};
            if constexpr (KINK) {
                rc *= scale;
#pragma unroll
                for (int q = 0; q < V; ++q) cmpq[q] *= scale;
            }
            auto chunk_sums = [&](auto drc) {
                constexpr bool DR = decltype(drc)::value;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const float p = __builtin_amdgcn_exp2f(s[u] - m_new);
                    ls += p;
                    float pa = p;
                    if constexpr (DR) pa = p * drop_factor(drop, k + u, h, H);
#pragma unroll
                    for (int q = 0; q < V; ++q) cs[q] += pa * v[u][q];
                    kink(u, p, pa, rs, qs);
                }
            };
            if (dropping) chunk_sums(std::true_type{});
            else chunk_sums(std::false_type{});
            // Kahan: add the chunk sums into the running sums
            auto kahan_add = [](float& sum, float& c, float part) {
                const float y = part - c;
                const float t = sum + y;
                c = (t - sum) - y;
                sum = t;
            };
            auto kahan_add4 = [](f32x4& sum, f32x4& c, f32x4 part) {
                const f32x4 y = part - c;
                const f32x4 t = sum + y;
                c = (t - sum) - y;
                sum = t;
            };
            kahan_add(l, lc, ls);
#pragma unroll
            for (int q = 0; q < V; ++q) kahan_add4(acc[q], cmp[q], cs[q]);
            if constexpr (KINK) {
                kahan_add(racc, rc, rs);
#pragma unroll
                for (int q = 0; q < V; ++q) kahan_add4(accq[q], cmpq[q], qs[q]);
            }
        }
        m = m_new;
    };
    if constexpr (PIPE) {
        // gathers software-pipelined one chunk ahead: chunk k+U's rows are in
        // flight while chunk k is scored and accumulated.  Two register sets
        // (A, B) in a loop unrolled by two chunks, so no buffer is copied (a
        // copy of the prefetched rows waits for them: the pipelining would be
        // lost), and every fetch is unconditional (past the row's end the
        // clamped ids repeat its last edge: gathered, unused; a conditional
        // fetch leaves the waitcnt pass unable to count the loads in flight).
        auto col_at = [&](int k0, int (&cc)[CL]) {
#pragma unroll
            for (int t = 0; t < CL; ++t) cc[t] = col[min(k0 + cfirst + t * cstep, e1 - 1)];
        };
        f32x4 va[U][V], vb[U][V];
        float sa[U], sb[U];
        int cb[CL];
        fetch(cv, va, sa);  // (an empty row: cv = 0, row 0 gathered, unused)
#pragma unroll
        for (int t = 0; t < CL; ++t) cb[t] = e1 > e0 ? col[min(e0 + U + cfirst + t * cstep, e1 - 1)] : 0;
        for (int k = e0; k < e1; k += 2 * U) {
            int ca2[CL], cb2[CL];
            col_at(k + 2 * U, ca2);
            fetch(cb, vb, sb);
            consume(k, va, sa);
            col_at(k + 3 * U, cb2);
            fetch(ca2, va, sa);
            if (k + U < e1) consume(k + U, vb, sb);
#pragma unroll
            for (int t = 0; t < CL; ++t) cb[t] = cb2[t];
        }
    } else if constexpr (RC == 2) {
        // the ids as RC = 1, and the gathers one chunk ahead: chunk t+1's rows
        // are in flight while chunk t is scored and accumulated.  The wave
        // walks the chunk count of its longest row (wave-uniform, so the
        // prefetch branch is scalar); consume() is spelled out in both arms of
        // that branch, so the wait for chunk t's rows counts chunk t+1's loads
        // (a shared join would wait for all of them).  Groups whose row is
        // shorter gather clamped ids (their last edge) and skip consume (an
        // empty row keeps m = -inf, l = 0, acc = 0).
        constexpr int NQ = G / 4, R = 8 / NQ > 0 ? 8 / NQ : 1, NB = NQ * R;
        const int qd = (c >> 2) & (NQ - 1), pq = c & 3;
        int nchw = (e1 - e0 + U - 1) / U;
#pragma unroll
        for (int off = G; off < kWave; off <<= 1) nchw = max(nchw, __shfl_xor(nchw, off));
        nchw = __builtin_amdgcn_readfirstlane(nchw);
        f32x4 va[U][V], vb[U][V];
        float sa[U], sb[U];
        for (int i0 = 0; i0 < nchw; i0 += NB) {
            const int b0 = e0 + i0 * U;
            int cr[R];
#pragma unroll
            for (int q = 0; q < R; ++q)
                cr[q] = col[min(b0 + U * (NQ * q + qd) + pq, max(e1 - 1, 0))];
            auto ids = [&](int t, int (&cc)[CL]) {
                if constexpr (NQ == 1) cc[0] = cr[t];
                else cc[0] = __shfl(cr[t / NQ], gbase + 4 * (t % NQ) + pq);
            };
            const int nb = min(NB, nchw - i0);  // wave-uniform chunks in this batch
            {
                int cc[CL];
                ids(0, cc);
                fetch(cc, va, sa);
            }
#pragma unroll
            for (int t = 0; t < NB; t += 2) {  // chunk t in set A, chunk t+1 in set B
                if (t >= nb) break;
                const int ka = b0 + U * t, kb = ka + U;
                if (t + 1 < nb) {
                    int cc[CL];
                    ids(t + 1, cc);
                    fetch(cc, vb, sb);
                    if (ka < e1) consume(ka, va, sa);
                } else {
                    if (ka < e1) consume(ka, va, sa);
                    break;
                }
                if (t + 2 < nb) {
                    int cc[CL];
                    ids(t + 2, cc);
                    fetch(cc, va, sa);
                    if (kb < e1) consume(kb, vb, sb);
                } else {
                    if (kb < e1) consume(kb, vb, sb);
                    break;
                }
            }
        }
    } else if constexpr (RC > 0) {
        // ids of up to 8 chunks per round trip (see RC above)
        constexpr int NQ = G / 4, R = 8 / NQ > 0 ? 8 / NQ : 1, NB = NQ * R;
        const int qd = (c >> 2) & (NQ - 1), pq = c & 3;
        for (int b0 = e0; b0 < e1; b0 += NB * U) {
            int cr[R];
#pragma unroll
            for (int q = 0; q < R; ++q) cr[q] = col[min(b0 + U * (NQ * q + qd) + pq, e1 - 1)];
#pragma unroll
            for (int t = 0; t < NB; ++t) {
                const int k = b0 + U * t;
                if (k >= e1) break;
                int cc[CL];
                // chunk t's ids into this lane's quad (then broadcast inside it)
                if constexpr (NQ == 1) cc[0] = cr[t];
                else cc[0] = __shfl(cr[t / NQ], gbase + 4 * (t % NQ) + pq);
                f32x4 v[U][V];
                float s[U];
                fetch(cc, v, s);
                consume(k, v, s);
            }
        }
    } else {
        for (int k = e0 + half * U; k < e1; k += S * U) {
            int cn[CL];
#pragma unroll
            for (int t = 0; t < CL; ++t) cn[t] = col[min(k + S * U + cfirst + t * cstep, e1 - 1)];
            f32x4 v[U][V];
            float s[U];
            fetch(cv, v, s);
            consume(k, v, s);
#pragma unroll
            for (int t = 0; t < CL; ++t) cv[t] = cn[t];
        }
    }
    if constexpr (S > 1) {
        // merge the S groups' states by an xor butterfly over the groups (both
        // partners of a step end with the same values: a + b == b + a exactly);
        // the Kahan compensation is applied first
        if (kahan) {
            l -= lc;
            lc = 0.f;
#pragma unroll
            for (int q = 0; q < V; ++q) {
                acc[q] -= cmp[q];
                cmp[q] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
#pragma unroll
        for (int off = G; off < G * S; off <<= 1) {
            const float mp = __shfl_xor(m, off), lp = __shfl_xor(l, off);
            const float mm = fmaxf(m, mp);
            // an empty group (a row shorter than its chunk) has m = -inf, adds 0
            const float so = m == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m - mm);
            const float sp = mp == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mp - mm);
            l = l * so + lp * sp;
#pragma unroll
            for (int q = 0; q < V; ++q) {
                f32x4 ap;
                ap.x = __shfl_xor(acc[q].x, off);
                ap.y = __shfl_xor(acc[q].y, off);
                ap.z = __shfl_xor(acc[q].z, off);
                ap.w = __shfl_xor(acc[q].w, off);
                acc[q] = acc[q] * so + ap * sp;
            }
            m = mm;
        }
        if (half != 0) return;
    }

    if (pos < er.store_lt) {  // a segment: hand the state on (the row is not finished)
        if (c_ok) {
#pragma unroll
            for (int q = 0; q < V; ++q)
                *reinterpret_cast<f32x4*>(er.st_acc + (size_t)si * er.ld_st + coff + 4 * q) =
                    kahan ? acc[q] - cmp[q] : acc[q];
            if ((coff % F) == 0) {
                er.st_ml[(size_t)si * 2 * H + h] = m;
                er.st_ml[(size_t)si * 2 * H + H + h] = kahan ? l - lc : l;
            }
        }
        return;
    }
    const float inv = 1.f / (l + 1e-16f);
    if (lse != nullptr && c_ok && (coff % F) == 0)
        lse[(size_t)r * H + h] = (m + log2f(l)) * kLn2;  // natural-log units
    if (y_heads != nullptr && c_ok) {
#pragma unroll
        for (int q = 0; q < V; ++q)
            *reinterpret_cast<f32x4*>(y_heads + (size_t)r * HF + coff + 4 * q) = acc[q] * inv;
    }
    if constexpr (KINK) {
        if (c_ok) {
#pragma unroll
            for (int q = 0; q < V; ++q)
                *reinterpret_cast<f32x4*>(q_heads + (size_t)r * HF + coff + 4 * q) =
                    (kahan ? accq[q] - cmpq[q] : accq[q]) * inv;
            if ((coff % F) == 0) r_heads[(size_t)r * H + h] = (kahan ? racc - rc : racc) * inv;
        }
    }
    if (concat) {
        if (c_ok) {
#pragma unroll
            for (int q = 0; q < V; ++q) {
                const f32x4 b = *reinterpret_cast<const f32x4*>(bias + coff + 4 * q);
                store_out4(out, (size_t)r * ld_out + coff + 4 * q, acc[q] * inv + b, store_wt);
            }
        }
    } else {
        f32x4 y[V];
#pragma unroll
        for (int q = 0; q < V; ++q) y[q] = c_ok ? acc[q] * inv : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int off = G / 2; off >= 1; off >>= 1) {
            if (off < F / (4 * V)) break;
#pragma unroll
            for (int q = 0; q < V; ++q) {
                y[q].x += __shfl_xor(y[q].x, off);
                y[q].y += __shfl_xor(y[q].y, off);
                y[q].z += __shfl_xor(y[q].z, off);
                y[q].w += __shfl_xor(y[q].w, off);
            }
        }
        if (4 * V * c < F) {
            const float hh = (float)H;
#pragma unroll
            for (int q = 0; q < V; ++q) {
                const int f0 = 4 * V * c + 4 * q;
                const size_t o = (size_t)r * ld_out + f0;
                store_out1(out, o + 0, y[q].x / hh + bias[f0 + 0], store_wt);
                store_out1(out, o + 1, y[q].y / hh + bias[f0 + 1], store_wt);
                store_out1(out, o + 2, y[q].z / hh + bias[f0 + 2], store_wt);
                store_out1(out, o + 3, y[q].w / hh + bias[f0 + 3], store_wt);
            }
        }
    }
}


// ---------------------------------------------------------------------------
// Merge of split hub rows (degree skew).  A target row with more in-edges
// than one lane group should walk serially is cut into segments that run as
// separate virtual rows of k_edge_grp (EdgeRows by_pos + store), in parallel;
// hub k's segment states are virtual rows [vptr[k], vptr[k+1]) (through
// vslot when given: segment j's state at vslot[j], the schedule position the
// segment ran at).  Per head:
//   M = max_s m_s,  L = sum_s l_s 2^(m_s - M),  y = sum_s acc_s 2^(m_s - M) / (L + 1e-16)
// which is the segmented softmax of PyG utils.softmax (GAT.py:60) regrouped.
// A hub's segments are spread over a 256-thread workgroup (round 5: a
// one-wave-per-hub merge walking all of a hub's segments in one lane per head
// / column, three dependent loops of one load each, took 120 us at power-law
// Reddit, set by the longest hubs' load chains).  Thread t takes segments
// s0 + g, s0 + g + ng, ... (g = t / H or t / HF), and the per-group partial
// maxima / sums are combined in LDS in group order (deterministic).
__global__ __launch_bounds__(256) void k_edge_merge_wg(
    const int* __restrict__ hub_rows, const int* __restrict__ vptr,
    const int* __restrict__ vslot, int n_hub,
    const float* __restrict__ st_acc, int ld_st, const float* __restrict__ st_ml, int H, int F,
    int HF, int concat, const float* __restrict__ bias, float* __restrict__ out, int ld_out,
    float* __restrict__ lse, float* __restrict__ y_heads) {
    __shared__ float red[256];
    __shared__ float Ms[GAT_MAX_HEADS], Ls[GAT_MAX_HEADS], ys[GAT_MAX_HF];
    const int k = blockIdx.x;
    if (k >= n_hub) return;
    const int t = threadIdx.x;
    const int r = hub_rows[k], s0 = vptr[k], s1 = vptr[k + 1];
#define SLOT(sg) (vslot != nullptr ? vslot[sg] : (sg))
    // per-head max and sum: head h = t % H, segment group g = t / H of ng
    const int ng = 256 / H, h = t % H, g = t / H;
    const bool hact = g < ng;
    float m = -INFINITY;
    if (hact)
        for (int sg = s0 + g; sg < s1; sg += ng)
            m = fmaxf(m, st_ml[(size_t)SLOT(sg) * 2 * H + h]);
    red[t] = m;
    __syncthreads();
    if (t < H) {
        float M = -INFINITY;
        for (int q = 0; q < ng; ++q) M = fmaxf(M, red[q * H + t]);
        Ms[t] = M;
    }
    __syncthreads();
    float l = 0.f;
    if (hact) {
        const float M = Ms[h];
        for (int sg = s0 + g; sg < s1; sg += ng) {
            const size_t o = (size_t)SLOT(sg) * 2 * H;
            const float ms = st_ml[o + h];
            if (ms != -INFINITY) l += st_ml[o + H + h] * __builtin_amdgcn_exp2f(ms - M);
        }
    }
    red[t] = l;
    __syncthreads();
    if (t < H) {
        float L = 0.f;
        for (int q = 0; q < ng; ++q) L += red[q * H + t];
        Ls[t] = L;
        if (lse != nullptr) lse[(size_t)r * H + t] = (Ms[t] + log2f(L)) * kLn2;
    }
    __syncthreads();
    // columns: column c = t % HF, segment group gc = t / HF of ngc
    const int ngc = 256 / HF, c = t % HF, gc = t / HF;
    float a = 0.f;
    if (gc < ngc) {
        const int hh = c / F;
        const float M = Ms[hh];
        for (int sg = s0 + gc; sg < s1; sg += ngc) {
            const int sl = SLOT(sg);
            const float ms = st_ml[(size_t)sl * 2 * H + hh];
            if (ms != -INFINITY) a += st_acc[(size_t)sl * ld_st + c] * __builtin_amdgcn_exp2f(ms - M);
        }
    }
    red[t] = a;
    __syncthreads();
    if (t < HF) {
        float A = 0.f;
        for (int q = 0; q < ngc; ++q) A += red[q * HF + t];
        const float y = A / (Ls[t / F] + 1e-16f);
        if (y_heads != nullptr) y_heads[(size_t)r * HF + t] = y;
        if (concat) out[(size_t)r * ld_out + t] = y + bias[t];
        else ys[t] = y;
    }
    if (!concat) {
        __syncthreads();
        if (t < F) {
            float sum = 0.f;
            for (int q = 0; q < H; ++q) sum += ys[q * F + t];
            out[(size_t)r * ld_out + t] = sum / (float)H + bias[t];
        }
    }
#undef SLOT
}

}  // namespace

// ---------------------------------------------------------------------------
// Which k_edge_grp instances exist (the dispatch below maps every request onto
// one of them; the round-5 library carried 261 instances, most reachable only
// through A/B knobs):
//   * the "fast" lane groups G = 4, 8, 16 at V = 1 and G = 4, 8 at V = 2 — the
//     reference's HF = 32 / 64 rows and 128-B plane rows — with heads of 4 or 8
//     columns per lane group (hl = 1, 2 as a constant, HL): U = 4 (row-batched
//     col values RC where rows average >= 16 in-edges), 8 and 16; two or four
//     lane groups per row for small launches (S, G = 8 / 16, V = 1, U <= 8);
//     the pipelined long-row kernel (V = 2, U = 16); the kink-sum training
//     forward on HF = 64 (G = 16 at V = 1, G = 8 at V = 2);
//   * other head widths on those groups (hl read at run time): U = 8 only;
//   * every other lane group (HF = 4, 8, 128, 256; G = 16 at V = 2): U = 8;
//   * the gathered-score form (head lanes not a power of two): V = 1, U = 8;
//   * the small-Fin fused forward (XF): G = 8 / 16, hl 1 / 2, U = 4, fin 1-4.
// The row-batched col form (RC) for rows of >= 16 in-edges on average (PPI:
// edge kernel 26.3 -> 25.2 us, same box, profiles/r05/edge_ab_rowcol_ppi.json);
// rows of 2-3 chunks (arxiv, CIFAR) keep the one-chunk-ahead loads, which
// there measured faster (arxiv 54.0 vs 55.9 us, CIFAR H=8 18.8 vs 20.2;
// profiles/r05/edge_ab_rowcol_ungated_*.json).  GAT_EDGE_ROWCOL=0 (knob):
// never.  (Gathers one chunk ahead on top of it, round 6: 26.1 vs 25.1 us at
// PPI, 100 VGPRs; profiles/r06/edge_ab_rc_pipelined_ppi.json; removed.)
// ---------------------------------------------------------------------------
// 0: one chunk ahead; 1: row-batched ids; 2: + the gathers one chunk ahead,
// lean (the default where GAT_HINT_SHORT holds and the launch is an eval
// forward; else 1).  PPI edge kernel, same box, graph-timed: 26.45 / 25.25 /
// 25.00 us and 25.59 / 25.15 us for 1 / 2 in a second run; the lean row-batched
// form without the gathers ahead (64 VGPRs, 8 waves per SIMD) 25.96 / 25.91 us
// (profiles/r06/edge_ab_lean_ppi.json).
static int rowcol_for(int edges_per_row_hint) {
    const char* v = knob("GAT_EDGE_ROWCOL");
    const int m = v == nullptr ? 2 : std::max(0, std::min(2, std::atoi(v)));
    return edges_per_row_hint >= 16 ? m : 0;
}

constexpr bool fast_group(int g, int v) { return (g == 4 || g == 8 || g == 16) && (v == 1 || g <= 8); }

// one launch of the fused kernel with the head's lane count as a constant
// (hl = 1 or 2) or read at run time (HL = 0)
template <int G, int U, int V, bool PIPE, bool KINK, int S, int RC, bool LEAN = false,
          class... A>
static void launch_hl(int hl, dim3 grid, dim3 block, hipStream_t st, A... a) {
    if constexpr (fast_group(G, V)) {
        if (hl == 1) {
            hipLaunchKernelGGL((k_edge_grp<G, U, V, true, PIPE, KINK, S, 1, 0, RC, LEAN>), grid,
                               block, 0, st, a...);
            return;
        }
        if (hl == 2) {
            hipLaunchKernelGGL((k_edge_grp<G, U, V, true, PIPE, KINK, S, 2, 0, RC, LEAN>), grid,
                               block, 0, st, a...);
            return;
        }
    }
    if constexpr (!LEAN)
        hipLaunchKernelGGL((k_edge_grp<G, U, V, true, PIPE, KINK, S, 0, 0, RC>), grid, block, 0,
                           st, a...);
}

// the fused kernel on a fast lane group; u, rc, pipe and split as the
// dispatch resolved them (edge_aggregate_impl)
template <int G, int V, bool KINK, class... A>
static void launch_fast(int u, int rc, int pipe, int split, int hl, dim3 grid, dim3 block,
                        hipStream_t st, A... a) {
    constexpr bool kink_ok = (G == 16 && V == 1) || (G == 8 && V == 2);
    if constexpr (!KINK || kink_ok) {
        constexpr bool splittable = !KINK && V == 1 && (G == 8 || G == 16);
        if (u == 4) {
            if constexpr (splittable) {
                if (split == 2) return launch_hl<G, 4, V, false, false, 2, 0>(hl, dim3(grid.x * 2), block, st, a...);
                if (split == 4) return launch_hl<G, 4, V, false, false, 4, 0>(hl, dim3(grid.x * 4), block, st, a...);
            }
            if constexpr (G != 4) {  // (row-batched ids: G = 8, 16)
                if constexpr (!KINK && V == 1) {
                    if (rc == 2) return launch_hl<G, 4, V, false, false, 1, 2, true>(hl, grid, block, st, a...);
                }
                if (rc) return launch_hl<G, 4, V, false, KINK, 1, 1>(hl, grid, block, st, a...);
            }
            return launch_hl<G, 4, V, false, KINK, 1, 0>(hl, grid, block, st, a...);
        }
        if (u == 8) {
            if constexpr (splittable) {
                if (split == 2) return launch_hl<G, 8, V, false, false, 2, 0>(hl, dim3(grid.x * 2), block, st, a...);
                if (split == 4) return launch_hl<G, 8, V, false, false, 4, 0>(hl, dim3(grid.x * 4), block, st, a...);
            }
            return launch_hl<G, 8, V, false, KINK, 1, 0>(hl, grid, block, st, a...);
        }
        if constexpr (V == 2 && !KINK) {
            if (pipe) return launch_hl<G, 16, V, true, false, 1, 0>(hl, grid, block, st, a...);
        }
        launch_hl<G, 16, V, false, KINK, 1, 0>(hl, grid, block, st, a...);
    }
}

// the small-Fin fused forward (XF = fin, 1-4): G = 8 or 16, hl 1 or 2, U = 4
template <int G, int HL, class... A>
static void launch_xf(int xf, dim3 grid, dim3 block, hipStream_t st, A... a) {
    switch (xf) {
        case 1: hipLaunchKernelGGL((k_edge_grp<G, 4, 1, true, false, false, 1, HL, 1>), grid, block, 0, st, a...); break;
        case 2: hipLaunchKernelGGL((k_edge_grp<G, 4, 1, true, false, false, 1, HL, 2>), grid, block, 0, st, a...); break;
        case 3: hipLaunchKernelGGL((k_edge_grp<G, 4, 1, true, false, false, 1, HL, 3>), grid, block, 0, st, a...); break;
        default: hipLaunchKernelGGL((k_edge_grp<G, 4, 1, true, false, false, 1, HL, 4>), grid, block, 0, st, a...); break;
    }
}

// the shapes the small-Fin fused forward (XF) takes: fin 1-4, heads of 4 or 8
// columns (hl = 1, 2 at V = 1), lane groups of 8 or 16 (HF 17-64), LeakyReLU
// with a slope in [0, 1]
static bool xf_shape_ok(int fin, int heads, int f, float slope) {
    if (fin <= 0 || fin > 4 || heads <= 0 || f <= 0 || f % 4 != 0) return false;
    const int hf = heads * f, hl = f / 4, g = next_pow2((hf + 3) / 4);
    return hf <= GAT_MAX_HF && heads <= GAT_MAX_HEADS && (hl == 1 || hl == 2) &&
           (g == 8 || g == 16) && slope >= 0.f && slope <= 1.f;
}

// gat_layer_forward's choice (GAT_EDGE_XPROJ=0, knob: never fuse)
static bool xproj_takes(int n, int fin, int heads, int f, float slope) {
    const char* v = knob("GAT_EDGE_XPROJ");
    return n > 0 && (v == nullptr || std::atoi(v) != 0) && xf_shape_ok(fin, heads, f, slope);
}

extern "C" {

int gat_layer_forward_fuses(int n, int fin, int heads, int f, int concat, float negative_slope) {
    (void)concat;  // (a head mean of heads of 4 or 8 columns fuses too)
    return xproj_takes(n, fin, heads, f, negative_slope) ? 1 : 0;
}

static int edge_aggregate_impl(const EdgeRows er, const int* col, const int* row_order,
                               int row_begin, int row_end, const float* wh, int ld_wh,
                               const float* s_src, int ld_s, const float* a_src,
                               const float* c_src, const float* s_dst, int heads, int f,
                               int concat, int act, float negative_slope, const float* bias,
                               float* out, float* lse, float* y_heads, DropArgs drop,
                               int edges_per_row_hint, void* stream, int nslices = 1,
                               long long slice_stride = 0, float* q_heads = nullptr,
                               float* r_heads = nullptr, const XProjArgs* xp = nullptr) {
    if (act < GAT_ACT_LEAKY_RELU || act > GAT_ACT_HEAD_SOFTMAX) return GAT_EINVAL;
    if (heads <= 0 || f <= 0 || row_begin < 0 || row_end < row_begin || nslices <= 0)
        return GAT_EINVAL;
    const int hf = heads * f;
    if (hf > GAT_MAX_HF || heads > GAT_MAX_HEADS) return GAT_EUNSUPPORTED;
    const bool sliced = nslices > 1;
    if (sliced) {
        // slice planes of ld_wh = hf / nslices columns, whole heads or whole
        // float4 groups of one head; concat + fused LeakyReLU score only
        if (hf % nslices != 0 || ld_wh != hf / nslices || (ld_wh & 3) || slice_stride <= 0)
            return GAT_EINVAL;
        if (!concat || s_src != nullptr || act != GAT_ACT_LEAKY_RELU || lse != nullptr ||
            y_heads != nullptr)
            return GAT_EUNSUPPORTED;
    } else if (ld_wh < round_up4(hf) || (ld_wh & 3)) {
        return GAT_EINVAL;
    }
    const int slice_w = sliced ? ld_wh : round_up4(hf);
    // write-through output stores: only for the final (eval) output, which the
    // next kernel reads, not for the training forward's extra tensors
    const int store_wt = (lse == nullptr && q_heads == nullptr) ? 1 : 0;
    if (s_src != nullptr && ld_s < heads) return GAT_EINVAL;
    const bool have_a = a_src != nullptr && c_src != nullptr;
    if (s_src == nullptr && !have_a) return GAT_EINVAL;
    const int rows = row_end - row_begin;
    if (rows == 0) return GAT_OK;
    hipStream_t st = (hipStream_t)stream;
    const int ld_out = concat ? hf : f;
    // the lane-group kernel computes LeakyReLU as max(z, slope*z)
    const bool slope_ok = act == GAT_ACT_LEAKY_RELU && negative_slope >= 0.f &&
                          negative_slope <= 1.f;
    // V float4s per lane (one head per lane needs f % 4V == 0): fewer, fuller
    // waves; GAT_EDGE_V overrides
    // long rows (Reddit scale) take two float4s per lane: half the lanes per row,
    // twice the rows per wave (tools/tune_edge.py: Reddit 3.34 -> 3.23 ms; PPI and
    // arxiv are no faster with V = 2)
    // GAT_HINT_LOCAL (OR'd into the hint): sources lie near their targets in node
    // order (batched small graphs, kNN), so a wave's rows share source rows;
    // narrow row-major rows then take two float4s per lane (16 rows per wave at
    // HF = 32: CIFAR batch 11.6 -> 8.6 us; a uniform graph gains nothing)
    const bool local_hint = edges_per_row_hint > 0 && (edges_per_row_hint & GAT_HINT_LOCAL);
    const bool short_hint = edges_per_row_hint > 0 && (edges_per_row_hint & GAT_HINT_SHORT);
    edges_per_row_hint &= ~(GAT_HINT_LOCAL | GAT_HINT_SHORT);
    int vv = edges_per_row_hint >= 128 ? 2 : 1;
    if (local_hint && !sliced && round_up4(hf) <= 32) vv = 2;
    if (const char* ev = knob("GAT_EDGE_V")) vv = std::atoi(ev) >= 2 ? 2 : 1;
    if (xp != nullptr) vv = 1;  // the small-Fin form: four columns per lane
    while (vv > 1 && f % (4 * vv) != 0) vv >>= 1;
    // fused source score: the head's lanes must form an aligned power-of-two
    // block; otherwise (concat only) the gathered-score form at V = 1
    if (vv > 1 && !(next_pow2(f / (4 * vv)) == f / (4 * vv) && have_a)) vv = 1;
    const int hl = f / (4 * vv);  // lanes per head
    const bool pow2_hl = (f % (4 * vv) == 0) && next_pow2(hl) == hl;
    const int gcols = sliced ? slice_w : hf;  // columns one lane group owns
    const int g = next_pow2((gcols + 4 * vv - 1) / (4 * vv));
    const bool grp_ok = (f % 4 == 0) && (concat || pow2_hl) && slope_ok && g <= kWave;
    const bool fused = grp_ok && pow2_hl && have_a;
    if (s_src == nullptr && !fused) return GAT_EUNSUPPORTED;
    const bool kink = q_heads != nullptr;
    const bool kink_grp = (g == 16 && vv == 1) || (g == 8 && vv == 2);
    if (kink && (!fused || sliced || r_heads == nullptr || lse == nullptr || y_heads == nullptr ||
                 er.by_pos || er.load || er.store_lt > 0 || !kink_grp))
        return GAT_EUNSUPPORTED;
    // a slice holds whole heads (the fused score sums a head inside one group)
    if (sliced && (!fused || slice_w % f != 0)) return GAT_EUNSUPPORTED;
    if (grp_ok) {
        // edges per chunk: short rows want short chunks (less padding), long rows
        // more loads in flight; GAT_EDGE_U overrides
        // (tools/tune_edge.py: PPI, ~28 per row, 36.9 us at U = 8 -> 33.1 us at U = 4)
        int u = edges_per_row_hint <= 0 ? 8 : edges_per_row_hint <= 32 ? 4
              : edges_per_row_hint <= 64 ? 8 : 16;
        if (const char* eu = knob("GAT_EDGE_U")) u = std::atoi(eu) >= 16 ? 16 : std::atoi(eu) <= 4 ? 4 : 8;
        const long long threads = (long long)rows * g;
        const long long blocks = ((threads + 255) / 256) * nslices;
        if (blocks >= (1LL << 31)) return GAT_EUNSUPPORTED;
        const dim3 grid((unsigned)blocks), block(256);
        // gathers pipelined one chunk ahead for long rows (U = 16, V = 2: one
        // wave per SIMD at 360 registers, but 64 row gathers in flight per
        // lane; tools/slice_probe.py, Reddit scale 2.60 -> 1.99 ms); shorter
        // rows keep more, shallower waves (PPI 30.5 -> 32.9 us pipelined)
        // Not for the multi-GPU segment passes (rows' edges split over the
        // all-gather chunks, the state carried between passes): there the
        // one-wave-per-SIMD pipelined kernel exposes each pass's row prologue
        // (Reddit at P = 8, 3 passes: 342 us pipelined vs 287 us not; one
        // unsplit pass 252 vs 292; tools/emu_probe.py, profiles/r04/emu_reddit_p8.json)
        const bool seg_pass = !er.by_pos && (er.load || er.store_lt > 0);
        int pipe = (u == 16 && vv == 2 && !seg_pass) ? 1 : 0;
        if (const char* ep = knob("GAT_EDGE_PIPE")) pipe = std::atoi(ep) != 0 && u == 16 && vv == 2;
        // not the training forward (kink sums, dropout, lse / y): there the
        // gathers one chunk ahead cost more than they hide (Reddit training
        // step 8.45 -> 8.35 ms without, profiles/r06/train_ab_fwd_nopipe_reddit.json)
        if (kink) pipe = 0;
        // two lane groups per row (the grid doubles inside launch_fast); the
        // kink-sum forward and the pipelined kernel keep one group.  Segment
        // passes (er.load / store_lt: hub segments, the sharded chunk passes) DO
        // take S = 2/4: the carried (m, l, acc) state is loaded into group 0,
        // merged across the groups in registers, and stored by group 0.
        // Default: launches of fewer than ~4 waves per SIMD (a rank's share of a
        // small graph: PPI at P = 4 / 8 edge passes 14.2 -> 11.3 / 13.3 -> 9.0 us,
        // tools/emu_probe.py) — there the per-row chain of dependent chunk loads
        // is exposed; larger launches hide it and the split only adds work (full
        // PPI 27.8 -> 30.8 us, arxiv 54.2 -> 61.2 us).  Four groups under ~2
        // waves per SIMD (PPI at P = 8: 9.0 -> 8.2 us; at P = 4 it is 13.6).
        // Rows of fewer than ~3 chunks per group gain nothing from a split (arxiv
        // at P = 8, 8 edges per row: 10.9 us whole, 12.0 / 15.8 split 2 / 4).
        // GAT_EDGE_SPLIT (knob) forces 1, 2 or 4.
        const long long waves = (long long)rows * g * nslices / kWave;
        const int chunks = edges_per_row_hint > 0 ? edges_per_row_hint / u : 1 << 20;
        int split = (waves < 2048 && chunks >= 6) ? 4 : (waves < 4096 && chunks >= 3) ? 2 : 1;
        if (const char* es = knob("GAT_EDGE_SPLIT")) {
            split = std::atoi(es);
            if (split != 2 && split != 4) split = 1;
        }
        if (kink || pipe) split = 1;
        if ((long long)blocks * split >= (1LL << 31)) split = 1;
        int rc = rowcol_for(edges_per_row_hint);
        // the lean forms: eval, whole rows or hub-free schedules, rows < 1024
        const bool lean_ok = short_hint && !kink && lse == nullptr && y_heads == nullptr &&
                             drop.thresh == 0u && vv == 1;
        if (rc >= 2 && !lean_ok) rc = 1;
        // the instances that exist (see above): everything off the fast lane
        // groups, other head widths and the gathered-score form run U = 8, one
        // group per row, no row-batched ids, no pipelining
        const bool fast = fused && fast_group(g, vv) && (hl == 1 || hl == 2);
        if (!fast) {
            u = 8;
            split = 1;
            pipe = 0;
        }
        if (vv == 2 && u == 8) u = 4;  // V = 2 below U = 16: local narrow rows
        if (u != 4 || g == 4) rc = 0;
        const XProjArgs xpa = xp != nullptr ? *xp : XProjArgs{nullptr, nullptr, nullptr, nullptr,
                                                              nullptr, 0};
#define GAT_GRP_KARGS                                                                         \
    er, col, row_order, row_begin, row_end, wh, ld_wh, s_src, ld_s, a_src, c_src, s_dst,   \
        heads, f, hf, concat, negative_slope, bias, out, ld_out, lse, drop, y_heads, nslices,  \
        slice_w, slice_stride, q_heads, r_heads, store_wt, xpa
        if (xp != nullptr) {
            // the small-Fin fused forward: no Wh table, one lane group per row
            if (!(fused && vv == 1 && !kink && !sliced &&
                  xf_shape_ok(xp->fin, heads, f, negative_slope) && xp->x != nullptr &&
                  xp->w != nullptr && xp->b != nullptr && xp->a_dst != nullptr &&
                  xp->c_dst != nullptr))
                return GAT_EUNSUPPORTED;
            const int xf = xp->fin;
            if (g == 8) {
                if (hl == 1) launch_xf<8, 1>(xf, grid, block, st, GAT_GRP_KARGS);
                else launch_xf<8, 2>(xf, grid, block, st, GAT_GRP_KARGS);
            } else {
                if (hl == 1) launch_xf<16, 1>(xf, grid, block, st, GAT_GRP_KARGS);
                else launch_xf<16, 2>(xf, grid, block, st, GAT_GRP_KARGS);
            }
            return status_of(hipGetLastError());
        }
        if (!fused) {
            // gathered source scores (V = 1, U = 8)
#define GAT_GRP_GATHER(G)                                                                     \
    case G:                                                                                   \
        hipLaunchKernelGGL((k_edge_grp<G, 8, 1, false>), grid, block, 0, st, GAT_GRP_KARGS);  \
        break;
            switch (g) {
                GAT_GRP_GATHER(1) GAT_GRP_GATHER(2) GAT_GRP_GATHER(4) GAT_GRP_GATHER(8)
                GAT_GRP_GATHER(16) GAT_GRP_GATHER(32) GAT_GRP_GATHER(64)
                default: return GAT_EUNSUPPORTED;
            }
#undef GAT_GRP_GATHER
            return status_of(hipGetLastError());
        }
        if (fast) {
            if (vv == 1) {
                if (g == 4) launch_fast<4, 1, false>(u, rc, pipe, split, hl, grid, block, st, GAT_GRP_KARGS);
                else if (g == 8) launch_fast<8, 1, false>(u, rc, pipe, split, hl, grid, block, st, GAT_GRP_KARGS);
                else if (kink) launch_fast<16, 1, true>(u, rc, pipe, split, hl, grid, block, st, GAT_GRP_KARGS);
                else launch_fast<16, 1, false>(u, rc, pipe, split, hl, grid, block, st, GAT_GRP_KARGS);
            } else {
                if (g == 4) launch_fast<4, 2, false>(u, rc, pipe, split, hl, grid, block, st, GAT_GRP_KARGS);
                else if (kink) launch_fast<8, 2, true>(u, rc, pipe, split, hl, grid, block, st, GAT_GRP_KARGS);
                else launch_fast<8, 2, false>(u, rc, pipe, split, hl, grid, block, st, GAT_GRP_KARGS);
            }
            return status_of(hipGetLastError());
        }
        // run-time head width, U = 8, one group per row
#define GAT_GRP_SLOW(G, VV)                                                                   \
    if (kink)                                                                                 \
        hipLaunchKernelGGL((k_edge_grp<G, 8, VV, true, false, (G == 16 && VV == 1) ||          \
                                                              (G == 8 && VV == 2)>),          \
                           grid, block, 0, st, GAT_GRP_KARGS);                                \
    else                                                                                      \
        hipLaunchKernelGGL((k_edge_grp<G, 8, VV, true>), grid, block, 0, st, GAT_GRP_KARGS)
        if (vv == 2) {
            switch (g) {
                case 1: GAT_GRP_SLOW(1, 2); break;
                case 2: GAT_GRP_SLOW(2, 2); break;
                case 4: GAT_GRP_SLOW(4, 2); break;
                case 8: GAT_GRP_SLOW(8, 2); break;
                case 16: GAT_GRP_SLOW(16, 2); break;
                case 32: GAT_GRP_SLOW(32, 2); break;
                default: return GAT_EUNSUPPORTED;
            }
        } else {
            switch (g) {
                case 1: GAT_GRP_SLOW(1, 1); break;
                case 2: GAT_GRP_SLOW(2, 1); break;
                case 4: GAT_GRP_SLOW(4, 1); break;
                case 8: GAT_GRP_SLOW(8, 1); break;
                case 16: GAT_GRP_SLOW(16, 1); break;
                case 32: GAT_GRP_SLOW(32, 1); break;
                case 64: GAT_GRP_SLOW(64, 1); break;
                default: return GAT_EUNSUPPORTED;
            }
        }
#undef GAT_GRP_SLOW
#undef GAT_GRP_KARGS
        return status_of(hipGetLastError());
    }
    // the generic kernel runs whole CSR rows only
    if (kink) return GAT_EUNSUPPORTED;
    if (er.by_pos || er.load || er.store_lt > 0 || er.ee != er.eb + 1) return GAT_EUNSUPPORTED;
    const int* rowptr = er.eb;
    const int lpe = next_pow2((round_up4(hf) + 3) / 4);
    const int hp = next_pow2(heads);
    if (lpe > kWave) return GAT_EUNSUPPORTED;
    const dim3 grid(rows), block(kWave);
#define GAT_EDGE_LAUNCH(P)                                                                   \
    hipLaunchKernelGGL((k_edge_fwd<P>), grid, block, 0, st, rowptr, col, row_order,          \
                       row_begin, row_end, wh, ld_wh, s_src, ld_s, s_dst, heads, f, hf,      \
                       concat, act, negative_slope, bias, out, ld_out, lse, drop, y_heads,   \
                       lpe)
    switch (hp) {
        case 1: GAT_EDGE_LAUNCH(1); break;
        case 2: GAT_EDGE_LAUNCH(2); break;
        case 4: GAT_EDGE_LAUNCH(4); break;
        case 8: GAT_EDGE_LAUNCH(8); break;
        case 16: GAT_EDGE_LAUNCH(16); break;
        case 32: GAT_EDGE_LAUNCH(32); break;
        case 64: GAT_EDGE_LAUNCH(64); break;
        default: return GAT_EUNSUPPORTED;
    }
#undef GAT_EDGE_LAUNCH
    return status_of(hipGetLastError());
}

int gat_edge_aggregate(const int* rowptr, const int* col, const int* row_order, int row_begin,
                       int row_end, const float* wh, int ld_wh, const float* s_src, int ld_s,
                       const float* a_src, const float* c_src, const float* s_dst, int heads,
                       int f, int concat, float negative_slope, const float* bias, float* out,
                       float* lse, int edges_per_row_hint, void* stream) {
    return edge_aggregate_impl(rows_of_csr(rowptr), col, row_order, row_begin, row_end, wh, ld_wh, s_src,
                               ld_s, a_src, c_src, s_dst, heads, f, concat, GAT_ACT_LEAKY_RELU,
                               negative_slope, bias, out, lse, nullptr, make_drop(0.f, 0ull),
                               edges_per_row_hint, stream);
}

int gat_edge_aggregate_sliced(const int* rowptr, const int* col, const int* row_order,
                              int row_begin, int row_end, const float* wh, int n_table,
                              int slices, const float* a_src, const float* c_src,
                              const float* s_dst, int heads, int f, float negative_slope,
                              const float* bias, float* out, int edges_per_row_hint,
                              void* stream) {
    if (slices <= 1 || heads <= 0 || f <= 0 || n_table <= 0 || (heads * f) % slices != 0)
        return GAT_EINVAL;
    if (a_src == nullptr || c_src == nullptr) return GAT_EINVAL;
    const int sw = heads * f / slices;
    return edge_aggregate_impl(rows_of_csr(rowptr), col, row_order, row_begin, row_end, wh, sw, nullptr, 0,
                               a_src, c_src, s_dst, heads, f, 1, GAT_ACT_LEAKY_RELU,
                               negative_slope, bias, out, nullptr, nullptr, make_drop(0.f, 0ull),
                               edges_per_row_hint, stream, slices, (long long)n_table * sw);
}

int gat_edge_aggregate_ex(const int* rowptr, const int* col, const int* row_order, int row_begin,
                          int row_end, const float* wh, int ld_wh, const float* s_src, int ld_s,
                          const float* a_src, const float* c_src, const float* s_dst, int heads,
                          int f, int concat, int score_act, float act_param, float dropout_p,
                          unsigned long long seed, const unsigned long long* seed_dev,
                          const float* bias, float* out, float* lse, float* y_heads,
                          int edges_per_row_hint, void* stream) {
    if (!(dropout_p >= 0.f && dropout_p <= 1.f)) return GAT_EINVAL;
    return edge_aggregate_impl(rows_of_csr(rowptr), col, row_order, row_begin, row_end, wh, ld_wh, s_src,
                               ld_s, a_src, c_src, s_dst, heads, f, concat, score_act, act_param,
                               bias, out, lse, y_heads, make_drop(dropout_p, seed, seed_dev),
                               edges_per_row_hint, stream);
}

int gat_edge_aggregate_train(const int* rowptr, const int* col, const int* row_order,
                             int row_begin, int row_end, const float* wh, int ld_wh,
                             const float* a_src, const float* c_src, const float* s_dst,
                             int heads, int f, int concat, float negative_slope, float dropout_p,
                             unsigned long long seed, const unsigned long long* seed_dev,
                             const float* bias, float* out, float* lse, float* y_heads,
                             float* q_heads, float* r_heads, int edges_per_row_hint,
                             void* stream) {
    if (!(dropout_p >= 0.f && dropout_p <= 1.f)) return GAT_EINVAL;
    if (row_end > row_begin && (a_src == nullptr || c_src == nullptr || lse == nullptr ||
                                y_heads == nullptr || q_heads == nullptr || r_heads == nullptr))
        return GAT_EINVAL;
    // GAT_BWD_KINK=0 (A/B knob): refuse, so that the caller takes the
    // gat_edge_aggregate_ex + gat_bwd_targets path
    if (const char* v = knob("GAT_BWD_KINK"))
        if (std::atoi(v) == 0) return GAT_EUNSUPPORTED;
    return edge_aggregate_impl(rows_of_csr(rowptr), col, row_order, row_begin, row_end, wh, ld_wh,
                               nullptr, 0, a_src, c_src, s_dst, heads, f, concat,
                               GAT_ACT_LEAKY_RELU, negative_slope, bias, out, lse, y_heads,
                               make_drop(dropout_p, seed, seed_dev), edges_per_row_hint, stream,
                               1, 0, q_heads, r_heads);
}

int gat_edge_aggregate_seg(const int* seg_begin, const int* seg_end, int seg_by_pos,
                           const int* col, const int* row_order, int row_begin, int row_end,
                           const float* wh, int ld_wh, int n_table, int slices,
                           const float* a_src, const float* c_src, const float* s_dst, int heads,
                           int f, int concat, float negative_slope, float* st_acc, float* st_ml,
                           int flags, int store_rows, const float* bias, float* out,
                           int edges_per_row_hint, void* stream);

// The eval forward in one call (gat_project[_sliced] into a caller-owned table,
// then gat_edge_aggregate_seg over a scheduled CSR copy, rows by position):
// the host enqueue of a small graph's forward is one C-ABI call, not two.
int gat_layer_forward(const float* x, int n, int fin, const float* w, const float* b,
                      const float* a_src, const float* c_src, const float* a_dst,
                      const float* c_dst, int heads, int f, int slices, float* wh, float* s_src,
                      float* s_dst, const int* seg_begin, const int* seg_end, const int* col,
                      const int* row_order, int concat, float negative_slope, const float* bias,
                      float* out, int edges_per_row_hint, void* stream) {
    if (heads <= 0 || f <= 0 || slices <= 0 || n < 0) return GAT_EINVAL;
    const int hf = heads * f, hfp = round_up4(hf);
    int rc;
    // small Fin (<= 4: CIFAR's 3): the projection fused into the edge kernel,
    // which gathers x rows instead of Wh rows (k_edge_grp<..., XF>); wh, s_src
    // and s_dst are then not written.  GAT_EDGE_XPROJ=0 (A/B knob): project, then
    // aggregate.  Shapes it does not take (GAT_EUNSUPPORTED, nothing launched)
    // take the two-kernel path below.
    if (x != nullptr && xproj_takes(n, fin, heads, f, negative_slope)) {
        if (seg_begin == nullptr || seg_end == nullptr || a_src == nullptr || c_src == nullptr)
            return GAT_EINVAL;
        EdgeRows er;
        er.eb = seg_begin;
        er.ee = seg_end;
        er.st_acc = nullptr;
        er.st_ml = nullptr;
        er.ld_st = hfp;
        er.by_pos = 1;
        er.load = 0;
        er.store_lt = 0;
        const XProjArgs xp{x, w, b, a_dst, c_dst, fin};
        rc = edge_aggregate_impl(er, col, row_order, 0, n, x, hfp, nullptr, 0, a_src, c_src,
                                 nullptr, heads, f, concat, GAT_ACT_LEAKY_RELU, negative_slope,
                                 bias, out, nullptr, nullptr, make_drop(0.f, 0ull),
                                 edges_per_row_hint, stream, 1, 0, nullptr, nullptr, &xp);
        if (rc != GAT_EUNSUPPORTED) return rc;
    }
    if (slices > 1)
        rc = gat_project_sliced(x, n, fin, w, b, a_src, c_src, a_dst, c_dst, heads, f, slices, wh,
                                n, nullptr, heads, s_dst, stream);
    else
        rc = gat_project(x, n, fin, w, b, a_src, c_src, a_dst, c_dst, heads, f, wh, hfp, s_src,
                         heads, s_dst, stream);
    if (rc != GAT_OK) return rc;
    return gat_edge_aggregate_seg(seg_begin, seg_end, 1, col, row_order, 0, n, wh,
                                  slices > 1 ? hf / slices : hfp, n, slices, a_src, c_src, s_dst,
                                  heads, f, concat, negative_slope, nullptr, nullptr, 0, 0, bias,
                                  out, edges_per_row_hint, stream);
}

int gat_edge_aggregate_seg(const int* seg_begin, const int* seg_end, int seg_by_pos,
                           const int* col, const int* row_order, int row_begin, int row_end,
                           const float* wh, int ld_wh, int n_table, int slices,
                           const float* a_src, const float* c_src, const float* s_dst, int heads,
                           int f, int concat, float negative_slope, float* st_acc, float* st_ml,
                           int flags, int store_rows, const float* bias, float* out,
                           int edges_per_row_hint, void* stream) {
    if (seg_begin == nullptr || seg_end == nullptr || a_src == nullptr || c_src == nullptr)
        return GAT_EINVAL;
    if (heads <= 0 || f <= 0 || slices <= 0 || (flags & ~(GAT_SEG_LOAD | GAT_SEG_STORE)))
        return GAT_EINVAL;
    const int hf = heads * f;
    if ((flags != 0) && (st_acc == nullptr || st_ml == nullptr)) return GAT_EINVAL;
    EdgeRows er;
    er.eb = seg_begin;
    er.ee = seg_end;
    er.st_acc = st_acc;
    er.st_ml = st_ml;
    er.ld_st = round_up4(hf);
    er.by_pos = seg_by_pos != 0;
    er.load = (flags & GAT_SEG_LOAD) != 0;
    // GAT_SEG_STORE: every row stores its state; else, by position, the rows at
    // positions < store_rows do (split hub segments ahead of whole rows)
    er.store_lt = (flags & GAT_SEG_STORE) ? 0x7fffffff : (seg_by_pos ? store_rows : 0);
    if (store_rows < 0 || (store_rows > 0 && !seg_by_pos)) return GAT_EINVAL;
    if (er.store_lt > 0 && (st_acc == nullptr || st_ml == nullptr)) return GAT_EINVAL;
    if (slices > 1) {
        if (n_table <= 0 || hf % slices != 0) return GAT_EINVAL;
        const int sw = hf / slices;
        return edge_aggregate_impl(er, col, row_order, row_begin, row_end, wh, sw, nullptr, 0,
                                   a_src, c_src, s_dst, heads, f, concat, GAT_ACT_LEAKY_RELU,
                                   negative_slope, bias, out, nullptr, nullptr,
                                   make_drop(0.f, 0ull), edges_per_row_hint, stream, slices,
                                   (long long)n_table * sw);
    }
    return edge_aggregate_impl(er, col, row_order, row_begin, row_end, wh, ld_wh, nullptr, 0,
                               a_src, c_src, s_dst, heads, f, concat, GAT_ACT_LEAKY_RELU,
                               negative_slope, bias, out, nullptr, nullptr, make_drop(0.f, 0ull),
                               edges_per_row_hint, stream);
}

int gat_edge_merge(const int* hub_rows, const int* seg_ptr, int n_hub, const float* st_acc,
                   const float* st_ml, int heads, int f, int concat, const float* bias,
                   float* out, float* lse, float* y_heads, void* stream) {
    return gat_edge_merge_ex(hub_rows, seg_ptr, nullptr, n_hub, st_acc, st_ml, heads, f, concat,
                             bias, out, lse, y_heads, stream);
}

int gat_edge_merge_ex(const int* hub_rows, const int* seg_ptr, const int* seg_slot, int n_hub,
                      const float* st_acc, const float* st_ml, int heads, int f, int concat,
                      const float* bias, float* out, float* lse, float* y_heads, void* stream) {
    if (heads <= 0 || f <= 0 || n_hub < 0) return GAT_EINVAL;
    const int hf = heads * f;
    if (hf > GAT_MAX_HF || heads > GAT_MAX_HEADS) return GAT_EUNSUPPORTED;
    if (n_hub == 0) return GAT_OK;
    if (hub_rows == nullptr || seg_ptr == nullptr || st_acc == nullptr || st_ml == nullptr ||
        bias == nullptr || out == nullptr)
        return GAT_EINVAL;
    hipLaunchKernelGGL(k_edge_merge_wg, dim3(n_hub), dim3(256), 0, (hipStream_t)stream,
                           hub_rows, seg_ptr, seg_slot, n_hub, st_acc, round_up4(hf), st_ml, heads,
                           f, hf, concat, bias, out, concat ? hf : f, lse, y_heads);
    return status_of(hipGetLastError());
}

}  // extern "C"
