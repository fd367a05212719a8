#pragma once
// MI355X (gfx950) GAT attention layer: HIP kernels + C-ABI — shared helpers.
//
// The library is five translation units that include this header:
//   gat_abi.hip       ABI version, table layout, the knob snapshot
//   gat_project.hip   projection + score epilogue (gat_project*)
//   gat_edge.hip      fused edge kernel, hub merge, gat_layer_forward
//   gat_csr.hip       CSR / CSC builds (gat_csr_build, gat_csc_build)
//   gat_backward.hip  recompute backward, weight and input gradients
//
// Replaces the hot path of danieldritter/ATMLGraphAttentionNetworks
// GraphAttentionLayer.forward (GAT.py:37-67) and the PyG pieces it calls:
//   gat_csr_build       <- utils.add_self_loops (GAT.py:38) + propagate's
//                          grouping of edges by edge_index[1] (GAT.py:53)
//   gat_project         <- the per-head Linear loop + attention Linears
//                          (GAT.py:42-52), one fp32 MFMA GEMM with a fused
//                          score epilogue
//   gat_edge_aggregate  <- propagate/message/softmax/aggregate + bias
//                          (GAT.py:53-67, PyG utils.softmax, aggr='add')
//
// Data layout in HBM (see DESIGN.md "Data layout"):
//   Wh[n_nodes][ld_wh] fp32, one row per SOURCE node, Wh = x W^T + b,
//       head-major (column h*F+f), zero-padded to round_up(HF, 4) columns;
//       ld_wh % 4 == 0 so every row is 16-B aligned (HF = 64: one 256-B row =
//       exactly two 128-B lines per gathered edge).
//   s_src[n_nodes] at stride ld_s (>= H): Wh_h . a1_h + c1_h (source term).
//       Default layout: its own compact [N][H] array (PPI: 1.4 MB, L2-resident).
//       Packed layout (one all-gather for multi-GPU): s_src = Wh + s_off with
//       ld_s = ld_wh (gat_table_layout).
//   s_dst[n_nodes][H] fp32 (target term, read once per row)
//   CSR by target: rowptr int32 [n+1], col int32 [E+n]; within a row the
//   sources ascend (one stable radix sort of (target, source) keys over the
//   input edges plus the appended self-loops; duplicates keep input order).
//   The segmented softmax and the sum are order-independent up to fp32
//   rounding, which the 1e-5 parity bar covers.
//
// Everything is fp32 (parity bar 1e-5 vs the reference's fp32 CPU path).
// No CUDA shims, no hipify, no multi-backend code: gfx950 only.

#include <hip/hip_runtime.h>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <type_traits>

#include "../../include/gat_amd.h"

// Kernel-choice knobs (tests and A/B measurement; not part of the ABI),
// snapshotted from the environment at the first launch (gat_abi.hip).
namespace gat_detail __attribute__((visibility("hidden"))) {
const char* knob(const char* name);
void snapshot_knobs();
bool kernel_choice(const char* env, const char* slow);
}  // namespace gat_detail
using namespace gat_detail;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kWave = 64;

__device__ __forceinline__ float leaky(float z, float slope) {
    // torch.nn.LeakyReLU: z > 0 ? z : z * slope
    return z > 0.f ? z : z * slope;
}

// Score activations (GAT.py:30 LeakyReLU; run_act_func_experiment.py:111
// LogSigmoid, Tanh, Softmax — the last with torch's implicit dim=1 on the
// [E', H] scores, i.e. a softmax across the heads of each edge).
__device__ __forceinline__ float score_act(int act, float z, float param) {
    if (act == GAT_ACT_LOG_SIGMOID) return fminf(z, 0.f) - log1pf(expf(-fabsf(z)));
    if (act == GAT_ACT_TANH) return tanhf(z);
    return leaky(z, param);
}

// d act / dz for the elementwise activations
__device__ __forceinline__ float score_act_grad(int act, float z, float param) {
    if (act == GAT_ACT_LOG_SIGMOID) return 1.f / (1.f + expf(z));  // sigmoid(-z)
    if (act == GAT_ACT_TANH) {
        const float t = tanhf(z);
        return 1.f - t * t;
    }
    return z > 0.f ? 1.f : param;
}

// softmax over the HP consecutive lanes holding one edge's heads
template <int HP>
__device__ __forceinline__ float head_softmax(float z, bool valid) {
    float m = valid ? z : -INFINITY;
#pragma unroll
    for (int off = 1; off < HP; off <<= 1) m = fmaxf(m, __shfl_xor(m, off));
    const float p = valid ? expf(z - m) : 0.f;
    float sum = p;
#pragma unroll
    for (int off = 1; off < HP; off <<= 1) sum += __shfl_xor(sum, off);
    return valid ? p / sum : 0.f;
}

template <int HP>
__device__ __forceinline__ float head_sum(float v) {
#pragma unroll
    for (int off = 1; off < HP; off <<= 1) v += __shfl_xor(v, off);
    return v;
}

__host__ __device__ constexpr int round_up4(int v) { return (v + 3) & ~3; }

// Attention dropout (GAT.py:61, F.dropout on the softmax coefficients, training
// only).  The keep decision for (CSR edge position k, head h) is a pure function
// of (seed, k, h) — a counter-based hash — so the backward pass regenerates the
// forward's mask without storing it.  keep <=> mix(seed, k*H + h) >= thresh,
// thresh = round(p * 2^32); kept coefficients are scaled by 1/(1-p).
// oracle.dropout_factors restates the hash in numpy (tests/test_gpu_training.py
// checks forward and gradients against it).
struct DropArgs {
    unsigned thresh;   // 0: no dropout
    float scale;       // 1 / (1 - p)
    unsigned seed_lo, seed_hi;
    const unsigned long long* seed_ptr;  // if set, the seed is read from device memory
};

// The seed may live in device memory (gat_dropout_seed_next), so that a
// captured HIP graph draws a fresh mask on every replay.
__device__ __forceinline__ DropArgs resolve_drop(DropArgs d) {
    if (d.seed_ptr != nullptr) {
        const unsigned long long sv = *d.seed_ptr;
        d.seed_lo = (unsigned)sv;
        d.seed_hi = (unsigned)(sv >> 32);
    }
    return d;
}

__host__ __device__ __forceinline__ unsigned mix32(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// multiplier applied to a coefficient: scale if kept, 0 if dropped
__device__ __forceinline__ float drop_factor(const DropArgs& d, long long k, int h, int H) {
    const unsigned long long idx = (unsigned long long)k * (unsigned)H + (unsigned)h;
    const unsigned a = mix32((unsigned)idx ^ d.seed_lo);
    const unsigned b = mix32((unsigned)(idx >> 32) + d.seed_hi);
    return mix32(a ^ b) >= d.thresh ? d.scale : 0.f;
}

inline DropArgs make_drop(float p, unsigned long long seed,
                   const unsigned long long* seed_dev = nullptr) {
    DropArgs d;
    d.seed_ptr = seed_dev;
    double t = std::floor((double)p * 4294967296.0 + 0.5);
    if (t < 0.0) t = 0.0;
    if (t > 4294967295.0) t = 4294967295.0;
    d.thresh = (unsigned)t;
    // p >= 1 drops everything (F.dropout returns zeros)
    d.scale = p <= 0.f ? 1.f : p >= 1.f ? 0.f : 1.f / (1.f - p);
    d.seed_lo = (unsigned)seed;
    d.seed_hi = (unsigned)(seed >> 32);
    return d;
}

inline int next_pow2(int v) {
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}

// ---------------------------------------------------------------------------
// Cross-lane sums with DPP (a VALU modifier: no LDS round trip).  Sums over
// aligned groups of w lanes, w a power of two <= 16, within each 16-lane row:
// quad_perm [1,0,3,2] (xor 1), quad_perm [2,3,0,1] (xor 2), then
// row_half_mirror / row_mirror, which pair each quad (8-group) with the other
// one of its 8-group (16-row) — enough for a sum.
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// lane k of each quad, to all four lanes of the quad (DPP quad_perm [k,k,k,k])
template <int K>
__device__ __forceinline__ int quad_bcast(int v) {
    return __builtin_amdgcn_update_dpp(0, v, K * 0x55, 0xF, 0xF, false);
}

__device__ __forceinline__ float group_sum16(float v, int w) {
    if (w >= 2) v += dpp_mov<0xB1>(v);
    if (w >= 4) v += dpp_mov<0x4E>(v);
    if (w >= 8) v += dpp_mov<0x141>(v);
    if (w >= 16) v += dpp_mov<0x140>(v);
    return v;
}

// ---------------------------------------------------------------------------
// Explicitly fused float4 arithmetic.  With contraction left to the backend
// (-ffp-contract=fast), an unrolled `a.x*b.x + a.y*b.y + ...` is fused
// differently per unrolled instance once the SLP vectorizer packs some of the
// products into v_pk_mul (fma(x, x', y*y') + z*z' + w*w' for one edge,
// fma(w, w', fma(z, z', fma(y, y', x*x'))) for the next), so two kernels with
// the same source expression round differently.  Kernels that promise bitwise
// equal results to each other spell the order out with these.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float dot4(f32x4 a, f32x4 b) {
    return __builtin_fmaf(a.w, b.w, __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x)));
}

// acc + s * v, element by element, one rounding each
__device__ __forceinline__ f32x4 fma4(float s, f32x4 v, f32x4 acc) {
    return f32x4{__builtin_fmaf(s, v.x, acc.x), __builtin_fmaf(s, v.y, acc.y),
                 __builtin_fmaf(s, v.z, acc.z), __builtin_fmaf(s, v.w, acc.w)};
}

// ---------------------------------------------------------------------------
// Write-through (sc1) stores for a kernel's final outputs.  The bytes go to
// memory as they are stored, so the kernel ends with no dirty L2 lines: the
// dependent kernel's start does not wait for an L2 write-back of them
// (MI355X_MICROARCH.md, persistent-kernel price list, row 'boundary':
// + B / 6 TB/s for B dirty bytes left by the predecessor).  Buffer stores from
// a wave-uniform base (a kernel argument) with 32-bit byte offsets; an element
// past 2 GiB from the base takes a plain store.
// ---------------------------------------------------------------------------
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr size_t kWtMaxOff = 0x7FFFFFF0u;

// wt: 0 plain store; 1 write-through (sc1; the final outputs).  (Round 3
// measured plain, sc0, sc1, nt and nt + sc1 stores; sc1 won: DESIGN.md §3.1.)
__device__ __forceinline__ void store_out4(float* base, size_t idx, f32x4 v, int wt) {
    const size_t off = idx * sizeof(float);
    if (wt && off < kWtMaxOff) {
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7FFFFFFF, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsrc, (int)off, 0, 16);
    } else {
        *reinterpret_cast<f32x4*>(base + idx) = v;
    }
}

__device__ __forceinline__ void store_out1(float* base, size_t idx, float v, int wt) {
    const size_t off = idx * sizeof(float);
    if (wt && off < kWtMaxOff) {
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7FFFFFFF, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsrc, (int)off, 0, 16);
    } else {
        base[idx] = v;
    }
}

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// Small-Fin fused forward (gat_layer_forward with fin <= 8): the edge kernel
// gathers the source's x row (fin floats) instead of its Wh row and projects it
// in registers; no Wh table, no projection launch.
struct XProjArgs {
    const float* x;      // [n, fin]
    const float* w;      // [heads*f, fin]
    const float* b;      // [heads*f]
    const float* a_dst;  // [heads*f]
    const float* c_dst;  // [heads]
    int fin;
};

struct EdgeRows {
    const int* eb;     // segment begin (CSR position), indexed by row id or position
    const int* ee;     // segment end
    float* st_acc;     // carried state: un-normalised accumulators [.., ld_st]
    float* st_ml;      // carried state: per head (m in log2 units, l) as [.., 2H]
    int ld_st;         // floats per st_acc row
    int by_pos;        // eb/ee/state indexed by schedule position (else by row id)
    int load;          // start from the stored state
    int store_lt;      // positions < store_lt store the state instead of the output
};

inline EdgeRows rows_of_csr(const int* rowptr) {
    EdgeRows e;
    e.eb = rowptr;
    e.ee = rowptr + 1;
    e.st_acc = nullptr;
    e.st_ml = nullptr;
    e.ld_st = 0;
    e.by_pos = 0;
    e.load = 0;
    e.store_lt = 0;
    return e;
}

constexpr size_t kAlign = 256;
inline size_t align_up(size_t v) { return (v + kAlign - 1) / kAlign * kAlign; }

inline int grid_for(long long work, int block, int cap = 256 * 16) {
    long long g = (work + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

inline int status_of(hipError_t e) { return e == hipSuccess ? GAT_OK : (int)e; }

}  // namespace
