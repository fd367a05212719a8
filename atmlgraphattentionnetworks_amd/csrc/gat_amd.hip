// MI355X (gfx950) GAT attention layer: HIP kernels + C-ABI.
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
#include <rocprim/device/device_radix_sort.hpp>

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <type_traits>

#include "../../include/gat_amd.h"

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

DropArgs make_drop(float p, unsigned long long seed,
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

int next_pow2(int v) {
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}

// ---------------------------------------------------------------------------
// Projection: Wh = X W^T + b, s_src / s_dst fused in the epilogue.
// Replaces GAT.py:42-52 (H small Linear GEMMs + 2H attention Linears).
//
// One 256-thread workgroup (4 waves) owns 64 node rows x ALL NT*16 output
// columns; each wave owns 16 rows as NT accumulators of
// v_mfma_f32_16x16x4_f32 (exact fp32: a k-ordered fma chain).  Per 64-deep
// K tile the W tile [NT*16 x 64] is staged once in LDS for the 4 waves, and
// each wave loads its X fragments straight to registers (every X row is read
// once) — one load round per tile, a single round for Fin <= 64.
// Epilogue, on the accumulators: + Linear bias, Wh stores, then the two
// attention dot products per head — xor-shuffles across the head's F lanes
// when F | 16 or 16 | F (SHFL), else through an LDS copy of the tile.
// ---------------------------------------------------------------------------
template <int NT, bool SHFL>
__global__ __launch_bounds__(256) void k_project(
    const float* __restrict__ X, int n, int fin,
    const float* __restrict__ W, const float* __restrict__ bW,
    const float* __restrict__ a1, const float* __restrict__ c1,
    const float* __restrict__ a2, const float* __restrict__ c2,
    int H, int F, int HF, float* __restrict__ Wh, int ld_wh, float* __restrict__ Ss, int ld_s,
    float* __restrict__ s_dst) {
    constexpr int BK = 64, KS = BK / 4, BN = NT * 16;
    constexpr int WL = BN * BK / 256;      // W-tile elements per thread
    constexpr int WB = WL < 16 ? WL : 16;  // loads kept in flight per batch
    constexpr int WS = BK + 2;  // 16x16x4 B-fragment reads are conflict-free at this stride
    constexpr int OS = BN + 1;
    constexpr int LDS = (BN * WS > 64 * OS) ? BN * WS : 64 * OS;
    __shared__ float smem[LDS];

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int cl = lane & 15, kq = lane >> 4;
    const int row0 = blockIdx.x * 64 + w * 16;
    const int ar = row0 + cl;
    const float* xr = X + (size_t)(ar < n ? ar : (n > 0 ? n - 1 : 0)) * fin;
    const float xs = ar < n ? 1.f : 0.f;

    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int hfp = round_up4(HF);
    for (int k0 = 0; k0 < fin; k0 += BK) {
        // W tile -> LDS: batches of WB independent loads, then their stores
        // (a plain idx loop would wait on every load before its ds_write)
#pragma unroll
        for (int b0 = 0; b0 < WL; b0 += WB) {
            float wv[WB];
#pragma unroll
            for (int q = 0; q < WB; ++q) {
                // unconditional load from a clamped address times a 0/1 mask:
                // a guarded load compiles to a branch + vmcnt(0) per element
                const int idx = tid + (b0 + q) * 256;
                const int nn = idx / BK, gk = k0 + idx % BK;
                wv[q] = W[(size_t)min(nn, HF - 1) * fin + min(gk, fin - 1)] *
                        ((nn < HF && gk < fin) ? 1.f : 0.f);
            }
#pragma unroll
            for (int q = 0; q < WB; ++q) {
                const int idx = tid + (b0 + q) * 256;
                smem[(idx / BK) * WS + idx % BK] = wv[q];
            }
        }
        float xa[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            // value used unconditionally (x 0/1 mask), so the load is never
            // sunk into a branch with its own vmcnt(0); padded k: x * 0
            const int kk = k0 + 4 * s + kq;
            xa[s] = xr[min(kk, fin - 1)] * (kk < fin ? xs : 0.f);
        }
        __syncthreads();
        const int ksteps = min(KS, (fin - k0 + 3) / 4);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            if (s < ksteps) {  // wave-uniform
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    const float b = smem[(t * 16 + cl) * WS + 4 * s + kq];
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[s], b, acc[t], 0, 0, 0);
                }
            }
        }
        __syncthreads();
    }

    // accumulator map: column t*16 + cl, rows (lane >> 4) * 4 + i of the wave's 16
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int cc = t * 16 + cl;
        const float bb = cc < HF ? bW[cc] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float v = acc[t][i] + bb;  // Linear bias inside Wh (GAT.py:43)
            acc[t][i] = v;
            const int rr = row0 + (lane >> 4) * 4 + i;
            if (rr < n && cc < hfp) Wh[(size_t)rr * ld_wh + cc] = v;
        }
    }

    if constexpr (SHFL) {
        if (F <= 16) {  // head = F consecutive lanes of one tile: reduce tile by tile
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int cc = t * 16 + cl;
                const float w1 = cc < HF ? a1[cc] : 0.f, w2 = cc < HF ? a2[cc] : 0.f;
                float p1[4], p2[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    p1[i] = acc[t][i] * w1;
                    p2[i] = acc[t][i] * w2;
                }
                for (int off = 1; off < F; off <<= 1)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        p1[i] += __shfl_xor(p1[i], off);
                        p2[i] += __shfl_xor(p2[i], off);
                    }
                const int h = cc / F;
                if ((cl & (F - 1)) == 0 && h < H) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int rr = row0 + (lane >> 4) * 4 + i;
                        if (rr >= n) continue;
                        Ss[(size_t)rr * ld_s + h] = p1[i] + c1[h];
                        s_dst[(size_t)rr * H + h] = p2[i] + c2[h];
                    }
                }
            }
        } else {  // 16 | F: head h spans tiles [h*F/16, (h+1)*F/16)
            const int tph = F / 16;
            float p1[4] = {0.f, 0.f, 0.f, 0.f}, p2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int cc = t * 16 + cl;
                const float w1 = cc < HF ? a1[cc] : 0.f, w2 = cc < HF ? a2[cc] : 0.f;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    p1[i] += acc[t][i] * w1;
                    p2[i] += acc[t][i] * w2;
                }
                if ((t + 1) % tph == 0) {  // last tile of head h
                    const int h = t / tph;
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        for (int off = 1; off < 16; off <<= 1) {
                            p1[i] += __shfl_xor(p1[i], off);
                            p2[i] += __shfl_xor(p2[i], off);
                        }
                    if (cl == 0 && h < H) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int rr = row0 + (lane >> 4) * 4 + i;
                            if (rr >= n) continue;
                            Ss[(size_t)rr * ld_s + h] = p1[i] + c1[h];
                            s_dst[(size_t)rr * H + h] = p2[i] + c2[h];
                        }
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) p1[i] = p2[i] = 0.f;
                }
            }
        }
    } else {
        // any F: the wave's 16 x BN tile through LDS, one (row, head) per lane-iteration
        float* Os = smem + w * 16 * OS;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) Os[((lane >> 4) * 4 + i) * OS + t * 16 + cl] = acc[t][i];
        __syncthreads();
        for (int idx = lane; idx < 16 * H; idx += kWave) {
            const int rl = idx / H, h = idx % H;
            const int rr = row0 + rl;
            if (rr >= n) continue;
            float v1 = 0.f, v2 = 0.f;
            for (int f = 0; f < F; ++f) {
                const float v = Os[rl * OS + h * F + f];
                v1 = fmaf(v, a1[h * F + f], v1);
                v2 = fmaf(v, a2[h * F + f], v2);
            }
            Ss[(size_t)rr * ld_s + h] = v1 + c1[h];
            s_dst[(size_t)rr * H + h] = v2 + c2[h];
        }
    }
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

// ---------------------------------------------------------------------------
// Projection, software-pipelined K loop (Fin > 64).  fp32 MFMA throughput
// (157 TF) bounds a [N, Fin] x [Fin, 64] projection at large Fin (Reddit:
// 18 GFLOP -> 115 us).
//   * block = 128 rows x BN (<= 64) columns; wave w owns rows [32w, 32w+32)
//     as two 16-row groups, so every W fragment read from LDS feeds two MFMAs;
//   * per 64-wide K chunk, x [128 x 64] and W [BN x 64] are staged through
//     LDS with fully coalesced loads, and chunk c+1's loads are in flight in
//     registers while chunk c's 16 k-steps x 8 MFMAs run; two barriers per
//     chunk.
// Per-element overhead (measured against a one-float-per-lane version of the
// same schedule):
//   * x and W chunks load LW floats per lane (LW = 4 when fin % 4 == 0, 2 when
//     fin % 2 == 0) and land in LDS with one ds_write per load — 4x fewer
//     address computations, loads and LDS writes than one float per lane;
//     W rows padded to 68 floats (conflict-free B-fragment reads);
//   * the attention Linears (GAT.py:44-45) reduce over the head's F lanes by
//     DPP (no LDS permutes), and lane i of the head's group stores row i;
//   * Wh goes back through an LDS output tile: each thread stores one fixed
//     float4 column of 8 rows (coalesced rows, row-major or sliced planes).
// ---------------------------------------------------------------------------
template <int NT, int LW>
__global__ __launch_bounds__(256) void k_project_pipe2(
    const float* __restrict__ X, int n, int fin,
    const float* __restrict__ W, const float* __restrict__ bW,
    const float* __restrict__ a1, const float* __restrict__ c1,
    const float* __restrict__ a2, const float* __restrict__ c2,
    int H, int F, int HF, float* __restrict__ Wh, int ld_wh, float* __restrict__ Ss, int ld_s,
    float* __restrict__ s_dst, int slice_w, long long slice_stride) {
    constexpr int BK = 64, KS = BK / 4, BN = NT * 16, BM = 128;
    constexpr int XS = BK + 4, WS = BK + 4, OS = BN + 4;
    constexpr int XL = BM * BK / (256 * LW);  // x loads per thread per chunk
    constexpr int WL = BN * BK / (256 * LW);  // W loads per thread per chunk
    static_assert(OS <= XS, "the output tile reuses the x tile");
    using vec = typename std::conditional<LW == 4, f32x4,
                typename std::conditional<LW == 2, f32x2, float>::type>::type;
    __shared__ __attribute__((aligned(16))) float wsm[BN * WS];
    __shared__ __attribute__((aligned(16))) float xsm[BM * XS];

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int cl = lane & 15, kq = lane >> 4;
    const int blk0 = blockIdx.x * BM;
    const int row0 = blk0 + w * 32;
    f32x4 acc[2][NT];
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[g][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    vec xn[XL], wn[WL];
    auto load_chunk = [&](int k0) {
        // element e = (tid + 256 q) * LW -> row e / 64, k e % 64: consecutive
        // lanes read consecutive LW-float groups of one row (coalesced).  An LW
        // group is wholly below or wholly at/after fin (LW divides fin); groups
        // past fin and rows past n load clamped, in-bounds addresses (their
        // products meet zeroed W at the LDS write, or feed unstored rows).
#pragma unroll
        for (int q = 0; q < XL; ++q) {
            const int e = (tid + 256 * q) * LW;
            const int r = min(blk0 + e / BK, n - 1);
            const int k = min(k0 + e % BK, fin - LW);
            xn[q] = *reinterpret_cast<const vec*>(X + (size_t)r * fin + k);
        }
#pragma unroll
        for (int q = 0; q < WL; ++q) {
            const int e = (tid + 256 * q) * LW;
            const int nn = min(e / BK, HF - 1);
            const int k = min(k0 + e % BK, fin - LW);
            wn[q] = *reinterpret_cast<const vec*>(W + (size_t)nn * fin + k);
        }
    };
    load_chunk(0);
    for (int k0 = 0; k0 < fin; k0 += BK) {
        __syncthreads();  // the previous chunk's fragment reads are done
#pragma unroll
        for (int q = 0; q < XL; ++q) {
            const int e = (tid + 256 * q) * LW;
            *reinterpret_cast<vec*>(xsm + (e / BK) * XS + e % BK) = xn[q];
        }
#pragma unroll
        for (int q = 0; q < WL; ++q) {
            const int e = (tid + 256 * q) * LW;
            const bool ok = e / BK < HF && k0 + e % BK < fin;
            *reinterpret_cast<vec*>(wsm + (e / BK) * WS + e % BK) = ok ? wn[q] : vec{};
        }
        __syncthreads();
        if (k0 + BK < fin) load_chunk(k0 + BK);  // in flight during this chunk's MFMAs
        const int ksteps = min(KS, (fin - k0 + 3) / 4);
        const float* xa0 = xsm + (w * 32 + cl) * XS + kq;
        const float* xa1 = xa0 + 16 * XS;
#pragma unroll
        for (int st = 0; st < KS; ++st) {
            if (st < ksteps) {  // block-uniform
                const float a0 = xa0[4 * st], a1v = xa1[4 * st];
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    const float b = wsm[(t * 16 + cl) * WS + 4 * st + kq];
                    acc[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b, acc[0][t], 0, 0, 0);
                    acc[1][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1v, b, acc[1][t], 0, 0, 0);
                }
            }
        }
    }
    __syncthreads();  // x/W tiles dead: the x tile becomes the output tile

    const int hfp = round_up4(HF);
    const int lf = 31 - __builtin_clz((unsigned)F);  // F is a power of two <= 16
    float* Os = xsm;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int cc = t * 16 + cl;
        const float bb = cc < HF ? bW[cc] : 0.f;
        const float w1 = cc < HF ? a1[cc] : 0.f, w2 = cc < HF ? a2[cc] : 0.f;
        const int h = cc >> lf, li = cl & (F - 1);
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            float p1[4], p2[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float v = acc[g][t][i] + bb;  // Linear bias inside Wh (GAT.py:43)
                Os[(w * 32 + 16 * g + kq * 4 + i) * OS + cc] = cc < HF ? v : 0.f;
                p1[i] = group_sum16(v * w1, F);
                p2[i] = group_sum16(v * w2, F);
            }
            // lane li (< 4) of the head's F lanes stores row kq*4 + li's sums
            if (li < 4 && li < F && h < H) {
                const float v1 = li == 0 ? p1[0] : li == 1 ? p1[1] : li == 2 ? p1[2] : p1[3];
                const float v2 = li == 0 ? p2[0] : li == 1 ? p2[1] : li == 2 ? p2[2] : p2[3];
                const int rr = row0 + 16 * g + kq * 4 + li;
                if (rr < n) {
                    if (Ss != nullptr) Ss[(size_t)rr * ld_s + h] = v1 + c1[h];
                    s_dst[(size_t)rr * H + h] = v2 + c2[h];
                }
            }
            if (F < 4 && li == 0 && h < H) {  // heads narrower than 4 lanes: rows F..3
#pragma unroll
                for (int i = 1; i < 4; ++i) {
                    const int rr = row0 + 16 * g + kq * 4 + i;
                    if (i >= F && rr < n) {
                        if (Ss != nullptr) Ss[(size_t)rr * ld_s + h] = p1[i] + c1[h];
                        s_dst[(size_t)rr * H + h] = p2[i] + c2[h];
                    }
                }
            }
        }
    }
    __syncthreads();
    // Wh stores: thread owns float4 column c4 (plane offset computed once) of
    // rows tid / C4 + (256 / C4) * j
    constexpr int C4 = NT * 4;
    static_assert(256 % C4 == 0, "NT must divide 16");
    const int col = 4 * (tid % C4);
    if (col < hfp) {
        const int g = col / slice_w;
        float* dst = Wh + (size_t)g * (size_t)slice_stride + (col - g * slice_w);
        const int rows = min(BM, n - blk0);
        for (int r = tid / C4; r < rows; r += 256 / C4)
            *reinterpret_cast<f32x4*>(dst + (size_t)(blk0 + r) * ld_wh) =
                *reinterpret_cast<const f32x4*>(Os + r * OS + col);
    }
}

// ---------------------------------------------------------------------------
// Direct projection epilogue (the projection kernels' DIRECT form).  The MFMA
// operands are swapped (A = W fragment, B = x fragment), so the accumulators
// hold Wh^T: lane l (kq = l >> 4) has Wh[row][16t + 4kq .. +4] of its tile
// row, four consecutive columns.  Wh leaves as float4s straight from the
// registers; each head's scores s = Wh_h.a_h + c_h (GAT.py:44-45) are xor
// sums over the head's F/4 lanes.  For 8 heads of 8 (every reference
// configuration's first layer) a row's eight scores are gathered into one lane
// by two shuffles and stored as float4s: one contiguous 512-B run per wave
// instead of four instructions of scattered 4-B stores (PPI projection 8.2 ->
// 7.5 us).  Parameters: per column bs (Linear bias), a1s, a2s; per head c1s,
// c2s (16-B aligned, typically in LDS).
// ---------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ void proj_direct_epilogue(
    const f32x4 (&acc)[NT], int row, int n, int kq, const float* bs, const float* a1s,
    const float* a2s, const float* c1s, const float* c2s, int H, int F, int HF,
    float* __restrict__ Wh, int ld_wh, float* __restrict__ Ss, int ld_s,
    float* __restrict__ s_dst, int slice_w, long long slice_stride, int store_wt) {
    const int hfp = round_up4(HF);
    const int hl = F >> 2;  // lanes (kq) per head: 1, 2 or 4
    if constexpr (NT == 4) {
        if (H == 8 && F == 8) {
            // after the pair sums, lanes kq 0/1 hold head 2t and kq 2/3 head
            // 2t + 1 of tile t; lane kq 0 (kq 1) gathers heads 0-3 (4-7) of its
            // row from its kq ^ 2 partner
            float s1[NT], s2[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int c0 = 16 * t + 4 * kq;
                const f32x4 v = acc[t] + *reinterpret_cast<const f32x4*>(bs + c0);
                const f32x4 q1 = *reinterpret_cast<const f32x4*>(a1s + c0);
                const f32x4 q2 = *reinterpret_cast<const f32x4*>(a2s + c0);
                const float p1 = v.x * q1.x + v.y * q1.y + v.z * q1.z + v.w * q1.w;
                const float p2 = v.x * q2.x + v.y * q2.y + v.z * q2.z + v.w * q2.w;
                s1[t] = p1 + __shfl_xor(p1, 16);
                s2[t] = p2 + __shfl_xor(p2, 16);
                if (row < n) {
                    const int g = c0 / slice_w;
                    store_out4(Wh, (size_t)g * (size_t)slice_stride + (size_t)row * ld_wh +
                                       (c0 - g * slice_w), v, store_wt);
                }
            }
            float o1[NT], o2[NT];  // the kq ^ 2 partner's heads (2t + 1 for kq < 2)
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                o1[t] = __shfl_xor(s1[t], 32);
                o2[t] = __shfl_xor(s2[t], 32);
            }
            if (kq < 2 && row < n) {
                // kq 0: heads 0-3 = tiles 0, 1; kq 1: heads 4-7 = tiles 2, 3
                const f32x4 cs2 = *reinterpret_cast<const f32x4*>(c2s + 4 * kq);
                store_out4(s_dst, (size_t)row * 8 + 4 * kq,
                           f32x4{kq ? s2[2] : s2[0], kq ? o2[2] : o2[0],
                                 kq ? s2[3] : s2[1], kq ? o2[3] : o2[1]} + cs2, store_wt);
                if (Ss != nullptr) {
                    const f32x4 cs1 = *reinterpret_cast<const f32x4*>(c1s + 4 * kq);
                    const f32x4 v1 = f32x4{kq ? s1[2] : s1[0], kq ? o1[2] : o1[0],
                                           kq ? s1[3] : s1[1], kq ? o1[3] : o1[1]} + cs1;
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        store_out1(Ss, (size_t)row * ld_s + 4 * kq + i, v1[i], store_wt);
                }
            }
            return;
        }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int c0 = 16 * t + 4 * kq;
        const f32x4 v = acc[t] + *reinterpret_cast<const f32x4*>(bs + c0);
        const f32x4 q1 = *reinterpret_cast<const f32x4*>(a1s + c0);
        const f32x4 q2 = *reinterpret_cast<const f32x4*>(a2s + c0);
        float p1 = v.x * q1.x + v.y * q1.y + v.z * q1.z + v.w * q1.w;
        float p2 = v.x * q2.x + v.y * q2.y + v.z * q2.z + v.w * q2.w;
        if (hl >= 2) {
            p1 += __shfl_xor(p1, 16);
            p2 += __shfl_xor(p2, 16);
        }
        if (hl >= 4) {
            p1 += __shfl_xor(p1, 32);
            p2 += __shfl_xor(p2, 32);
        }
        if (row < n && c0 < hfp) {
            const int g = c0 / slice_w;  // slice_w % 4 == 0: one plane per float4
            store_out4(Wh, (size_t)g * (size_t)slice_stride + (size_t)row * ld_wh +
                               (c0 - g * slice_w), v, store_wt);
            if ((kq & (hl - 1)) == 0 && c0 < HF) {
                const int h = c0 / F;
                if (Ss != nullptr) store_out1(Ss, (size_t)row * ld_s + h, p1 + c1s[h], store_wt);
                store_out1(s_dst, (size_t)row * H + h, p2 + c2s[h], store_wt);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Projection on the bf16 matrix cores with split operands (Fin > 64: arxiv,
// Reddit).  gfx950's fp32 MFMA runs at the fp32 vector rate (1/16 of bf16), so
// the fp32 kernel above is MFMA-bound at Reddit scale (18 GFLOP: 115 us at
// peak).  Here every fp32 operand is split EXACTLY into three bf16 terms by
// round-to-nearest (x = x1 + x2 + x3: x1 = bf16(x), x2 = bf16(x - x1),
// x3 = x - x1 - x2, which has <= 8 significant bits, so bf16(x3) is exact),
// and x.w = sum over the six products x_i w_j with i + j <= 4 (bf16 x bf16
// products are exact in fp32).  The dropped terms x2 w3 + x3 w2 + x3 w3 are
// below 2^-24 |x w| each: fp32 rounding level, like the fp32 MFMA's own k-ordered
// chain.  Six v_mfma_f32_16x16x32_bf16 (16 cycles each) replace eight
// v_mfma_f32_16x16x4_f32 (32 cycles each) per 32-deep k step: 2.7x the
// product rate.  x1.w1 accumulates in `acc`, the five correction products in
// `cor` (summed at the end), so the small terms are not rounded against the
// large running sum at every step.
//
// Block: 64 rows x BN columns, one 16-row group per wave; 64-deep K chunks
// through LDS as k_project_pipe2, but with TWO chunks' loads in flight (a
// register double buffer): with the MFMA phase 2.7x shorter, one chunk in
// flight left the loads exposed (the 128-row, one-ahead form of this kernel
// ran Reddit in 196 us, 2.9 TB/s of x).
// x stays fp32 in LDS and each lane splits its own A fragment (8 consecutive k
// of one row) after reading it — every x element is split exactly once; W is
// split once per chunk at the LDS write, into three bf16 planes the waves
// share.  Fragment maps (cdna_hip_programming.md §3): lane l holds
// A[row l&15][k 8(l>>4)..+8] and B[k 8(l>>4)..+8][col l&15]; C/D as the fp32
// form (col l&15, rows 4(l>>4)+i), so the epilogue is k_project_pipe2's.
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// exact three-way bf16 split of a float pair (round to nearest at each level)
__device__ __forceinline__ void split3_pair(f32x2 v, bf16x2& p1, bf16x2& p2, bf16x2& p3) {
    p1 = __builtin_convertvector(v, bf16x2);
    const f32x2 r1 = v - __builtin_convertvector(p1, f32x2);
    p2 = __builtin_convertvector(r1, bf16x2);
    const f32x2 r2 = r1 - __builtin_convertvector(p2, f32x2);
    p3 = __builtin_convertvector(r2, bf16x2);
}

__device__ __forceinline__ void split3_x8(f32x4 a, f32x4 b, bf16x8& h1, bf16x8& h2, bf16x8& h3) {
    bf16x2 p1[4], p2[4], p3[4];
    split3_pair(f32x2{a.x, a.y}, p1[0], p2[0], p3[0]);
    split3_pair(f32x2{a.z, a.w}, p1[1], p2[1], p3[1]);
    split3_pair(f32x2{b.x, b.y}, p1[2], p2[2], p3[2]);
    split3_pair(f32x2{b.z, b.w}, p1[3], p2[3], p3[3]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        h1[2 * i] = p1[i][0];
        h1[2 * i + 1] = p1[i][1];
        h2[2 * i] = p2[i][0];
        h2[2 * i + 1] = p2[i][1];
        h3[2 * i] = p3[i][0];
        h3[2 * i + 1] = p3[i][1];
    }
}

template <int NT, int LW, int RG, int PD>
__global__ __launch_bounds__(256) void k_project_x3(
    const float* __restrict__ X, int n, int fin,
    const float* __restrict__ W, const float* __restrict__ bW,
    const float* __restrict__ a1, const float* __restrict__ c1,
    const float* __restrict__ a2, const float* __restrict__ c2,
    int H, int F, int HF, float* __restrict__ Wh, int ld_wh, float* __restrict__ Ss, int ld_s,
    float* __restrict__ s_dst, int slice_w, long long slice_stride, int store_wt) {
    // RG 16-row groups per wave, 4 waves: BM = 64 RG rows per block
    constexpr int BK = 64, BN = NT * 16, NTH = 256, BM = 64 * RG;
    constexpr int XS = BK + 4, WSB = BK + 8, OS = BN + 4;
    constexpr int XL = BM * BK / (NTH * LW);  // x loads per thread per chunk
    constexpr int WL = BN * BK / (NTH * LW) > 0 ? BN * BK / (NTH * LW) : 1;  // W loads
    static_assert(BN * BK % (NTH * LW) == 0 || BN * BK < NTH * LW, "W chunk split");
    static_assert(OS <= XS, "the output tile reuses the x tile");
    using vec = typename std::conditional<LW == 4, f32x4,
                typename std::conditional<LW == 2, f32x2, float>::type>::type;
    __shared__ __attribute__((aligned(16))) __bf16 wsb[3][BN * WSB];
    __shared__ __attribute__((aligned(16))) float xsm[BM * XS];

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int cl = lane & 15, kq = lane >> 4;
    const int blk0 = blockIdx.x * BM;
    const int row0 = blk0 + w * 16 * RG;  // wave w owns rows [16 RG w, 16 RG (w + 1))
    f32x4 acc[RG][NT], cor[RG][NT];
#pragma unroll
    for (int g = 0; g < RG; ++g)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[g][t] = cor[g][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    // PD chunks of loads in flight (PD = 2: a register double buffer,
    // statically indexed)
    vec xa_[XL], wa_[WL], xb_[PD == 2 ? XL : 1], wb_[PD == 2 ? WL : 1];
    auto load_chunk = [&](int k0, vec (&xn)[XL], vec (&wn)[WL]) {
        // element e = (tid + 256 q) * LW -> row e / 64, k e % 64 (coalesced rows);
        // clamped, in-bounds addresses past n / fin (zeroed W meets them)
#pragma unroll
        for (int q = 0; q < XL; ++q) {
            const int e = (tid + NTH * q) * LW;
            const int r = min(blk0 + e / BK, n - 1);
            const int k = min(k0 + e % BK, fin - LW);
            xn[q] = *reinterpret_cast<const vec*>(X + (size_t)r * fin + k);
        }
#pragma unroll
        for (int q = 0; q < WL; ++q) {
            const int e = (tid + NTH * q) * LW;
            const int nn = min(e / BK, HF - 1);  // (e past the chunk: a clamped dummy)
            const int k = min(k0 + e % BK, fin - LW);
            wn[q] = *reinterpret_cast<const vec*>(W + (size_t)nn * fin + k);
        }
    };
    // x chunk to LDS as fp32; W chunk split into three bf16 planes
    auto stage = [&](int k0, const vec (&xn)[XL], const vec (&wn)[WL]) {
#pragma unroll
        for (int q = 0; q < XL; ++q) {
            const int e = (tid + NTH * q) * LW;
            *reinterpret_cast<vec*>(xsm + (e / BK) * XS + e % BK) = xn[q];
        }
#pragma unroll
        for (int q = 0; q < WL; ++q) {
            const int e = (tid + NTH * q) * LW;
            const bool ok = e / BK < HF && k0 + e % BK < fin && e < BN * BK;
            const int o = min(e / BK, BN - 1) * WSB + e % BK;
            if constexpr (LW == 1) {
                bf16x2 p1, p2, p3;
                split3_pair(f32x2{ok ? wn[q] : 0.f, 0.f}, p1, p2, p3);
                wsb[0][o] = p1[0];
                wsb[1][o] = p2[0];
                wsb[2][o] = p3[0];
            } else if constexpr (LW == 2) {
                bf16x2 p1, p2, p3;
                split3_pair(ok ? wn[q] : f32x2{0.f, 0.f}, p1, p2, p3);
                *reinterpret_cast<bf16x2*>(&wsb[0][o]) = p1;
                *reinterpret_cast<bf16x2*>(&wsb[1][o]) = p2;
                *reinterpret_cast<bf16x2*>(&wsb[2][o]) = p3;
            } else {
                const f32x4 v = ok ? wn[q] : f32x4{0.f, 0.f, 0.f, 0.f};
                bf16x2 p1a, p2a, p3a, p1b, p2b, p3b;
                split3_pair(f32x2{v.x, v.y}, p1a, p2a, p3a);
                split3_pair(f32x2{v.z, v.w}, p1b, p2b, p3b);
                *reinterpret_cast<bf16x4*>(&wsb[0][o]) = bf16x4{p1a[0], p1a[1], p1b[0], p1b[1]};
                *reinterpret_cast<bf16x4*>(&wsb[1][o]) = bf16x4{p2a[0], p2a[1], p2b[0], p2b[1]};
                *reinterpret_cast<bf16x4*>(&wsb[2][o]) = bf16x4{p3a[0], p3a[1], p3b[0], p3b[1]};
            }
        }
    };
    auto compute = [&](int k0) {
        const int ksteps = min(BK / 32, (fin - k0 + 31) / 32);
#pragma unroll
        for (int s = 0; s < BK / 32; ++s) {
            if (s < ksteps) {  // block-uniform
                // A fragments of the wave's row groups split once; B fragments one
                // column tile at a time, each feeding RG row groups
                bf16x8 x1[RG], x2[RG], x3[RG];
#pragma unroll
                for (int g = 0; g < RG; ++g) {
                    const float* xa = xsm + (w * 16 * RG + 16 * g + cl) * XS + 32 * s + 8 * kq;
                    split3_x8(*reinterpret_cast<const f32x4*>(xa),
                              *reinterpret_cast<const f32x4*>(xa + 4), x1[g], x2[g], x3[g]);
                }
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    const int o = (t * 16 + cl) * WSB + 32 * s + 8 * kq;
                    const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(&wsb[0][o]);
                    const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(&wsb[1][o]);
                    const bf16x8 b3 = *reinterpret_cast<const bf16x8*>(&wsb[2][o]);
#pragma unroll
                    for (int g = 0; g < RG; ++g) {
                        acc[g][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1[g], b1, acc[g][t], 0, 0, 0);
                        cor[g][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1[g], b2, cor[g][t], 0, 0, 0);
                        cor[g][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x2[g], b1, cor[g][t], 0, 0, 0);
                        cor[g][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1[g], b3, cor[g][t], 0, 0, 0);
                        cor[g][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x2[g], b2, cor[g][t], 0, 0, 0);
                        cor[g][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x3[g], b1, cor[g][t], 0, 0, 0);
                    }
                }
            }
        }
    };
    // chunk c's loads were issued two chunks earlier.  Every load is
    // unconditional (chunks past fin load the last chunk again, unused): a
    // conditional load makes the compiler's vmcnt bookkeeping assume the worst
    // at the join and wait for ALL loads in flight, the prefetch included.
    const int klast = (fin - 1) / BK * BK;  // first k of the last chunk
    // (sched_barrier: the two chunks' loads stay in issue order, so the oldest
    // 16 are one chunk and the stage waits for that chunk alone)
    load_chunk(0, xa_, wa_);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PD == 1) {  // one chunk in flight (fewer registers, more waves)
        for (int k0 = 0; k0 < fin; k0 += BK) {
            __syncthreads();
            stage(k0, xa_, wa_);
            __syncthreads();
            load_chunk(min(k0 + BK, klast), xa_, wa_);
            compute(k0);
        }
    } else {
    load_chunk(min(BK, klast), xb_, wb_);
    __builtin_amdgcn_sched_barrier(0);
    for (int k0 = 0; k0 < fin; k0 += 2 * BK) {
        __syncthreads();  // the previous chunk's fragment reads are done
        stage(k0, xa_, wa_);
        __syncthreads();
        load_chunk(min(k0 + 2 * BK, klast), xa_, wa_);
        compute(k0);
        __syncthreads();
        stage(k0 + BK, xb_, wb_);  // past fin: zero W (ok is false), no k-steps
        __syncthreads();
        load_chunk(min(k0 + 3 * BK, klast), xb_, wb_);
        compute(k0 + BK);
    }
    }
    __syncthreads();  // x/W tiles dead: the x tile becomes the output tile
#pragma unroll
    for (int g = 0; g < RG; ++g)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[g][t] += cor[g][t];

    const int hfp = round_up4(HF);
    const int lf = 31 - __builtin_clz((unsigned)F);  // F is a power of two <= 16
    float* Os = xsm;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int cc = t * 16 + cl;
        const float bb = cc < HF ? bW[cc] : 0.f;
        const float w1 = cc < HF ? a1[cc] : 0.f, w2 = cc < HF ? a2[cc] : 0.f;
        const int h = cc >> lf, li = cl & (F - 1);
#pragma unroll
        for (int g = 0; g < RG; ++g) {
            float p1[4], p2[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float v = acc[g][t][i] + bb;  // Linear bias inside Wh (GAT.py:43)
                Os[(w * 16 * RG + 16 * g + kq * 4 + i) * OS + cc] = cc < HF ? v : 0.f;
                p1[i] = group_sum16(v * w1, F);
                p2[i] = group_sum16(v * w2, F);
            }
            // lane li (< 4) of the head's F lanes stores row kq*4 + li's sums
            if (li < 4 && li < F && h < H) {
                const float v1 = li == 0 ? p1[0] : li == 1 ? p1[1] : li == 2 ? p1[2] : p1[3];
                const float v2 = li == 0 ? p2[0] : li == 1 ? p2[1] : li == 2 ? p2[2] : p2[3];
                const int rr = row0 + 16 * g + kq * 4 + li;
                if (rr < n) {
                    if (Ss != nullptr) store_out1(Ss, (size_t)rr * ld_s + h, v1 + c1[h], store_wt);
                    store_out1(s_dst, (size_t)rr * H + h, v2 + c2[h], store_wt);
                }
            }
            if (F < 4 && li == 0 && h < H) {  // heads narrower than 4 lanes: rows F..3
#pragma unroll
                for (int i = 1; i < 4; ++i) {
                    const int rr = row0 + 16 * g + kq * 4 + i;
                    if (i >= F && rr < n) {
                        if (Ss != nullptr) store_out1(Ss, (size_t)rr * ld_s + h, p1[i] + c1[h], store_wt);
                        store_out1(s_dst, (size_t)rr * H + h, p2[i] + c2[h], store_wt);
                    }
                }
            }
        }
    }
    __syncthreads();
    constexpr int C4 = NT * 4;
    static_assert(NTH % C4 == 0, "NT must divide 16");
    const int col = 4 * (tid % C4);
    if (col < hfp) {
        const int g = col / slice_w;
        const size_t base = (size_t)g * (size_t)slice_stride + (col - g * slice_w);
        const int rows = min(BM, n - blk0);
        for (int r = tid / C4; r < rows; r += NTH / C4)
            store_out4(Wh, base + (size_t)(blk0 + r) * ld_wh,
                       *reinterpret_cast<const f32x4*>(Os + r * OS + col), store_wt);
    }
}

// ---------------------------------------------------------------------------
// Projection for Fin <= 128 (PPI's 50, ogbn-arxiv's 128): W resident in LDS,
// x streamed straight into MFMA fragments.
//
// With the whole K range small, W [HF, Fin] split into its three bf16 planes
// (k_project_x3's exact split) fits in LDS (arxiv: 3 x 64 x 136 bf16 = 52 KB),
// so each workgroup splits W ONCE and its waves then loop over 16-row tiles of
// x independently: no per-chunk W reloads or splits (with 64-row blocks W
// cost as many loads as x at arxiv), no x staging through LDS and no
// workgroup barriers in the loop.  Lane l loads its A fragments
// x[row l&15][k 8(l>>4)..+8] directly (each x byte read once; a row's 4 lanes
// x 2 loads fill its 128-B lines), splits them as soon as they land, and
// issues the next tile's loads before this tile's MFMAs, so a tile's loads
// are in flight during the previous tile's MFMAs and epilogue.  The epilogue
// (bias, fused scores by DPP, Wh rows through a per-wave LDS tile for
// coalesced float4 stores, row-major or column planes) is k_project_x3's.
// ---------------------------------------------------------------------------
template <int NT, int LW, int KS>
__global__ __launch_bounds__(256, 2) void k_project_wres(
    const float* __restrict__ X, int n, int fin,
    const float* __restrict__ W, const float* __restrict__ bW,
    const float* __restrict__ a1, const float* __restrict__ c1,
    const float* __restrict__ a2, const float* __restrict__ c2,
    int H, int F, int HF, float* __restrict__ Wh, int ld_wh, float* __restrict__ Ss, int ld_s,
    float* __restrict__ s_dst, int slice_w, long long slice_stride, int store_wt) {
    constexpr int BN = NT * 16, KP = KS * 32;  // padded K
    constexpr int WSB = KP + 8, OS = BN + 4;
    constexpr int NL = 8 / LW;                  // loads per 8-float fragment
    using vec = typename std::conditional<LW == 4, f32x4,
                typename std::conditional<LW == 2, f32x2, float>::type>::type;
    __shared__ __attribute__((aligned(16))) __bf16 wsb[3][BN * WSB];
    __shared__ __attribute__((aligned(16))) float osm[4][16 * OS];

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int cl = lane & 15, kq = lane >> 4;
    const int tiles = (n + 15) / 16;
    const int tstride = gridDim.x * 4;
    int tile = blockIdx.x * 4 + w;
    // x fragments of one tile: KS k-steps x NL loads (rows past n clamp to n-1,
    // k past fin to fin-LW: in bounds, and they meet zero W)
    vec xr[KS][NL];
    auto load_tile = [&](int tl) {
        const int r = min(tl * 16 + cl, n - 1);
        const float* xrow = X + (size_t)r * fin;
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int q = 0; q < NL; ++q) {
                const int k = min(32 * s + 8 * kq + LW * q, fin - LW);
                xr[s][q] = *reinterpret_cast<const vec*>(xrow + k);
            }
    };
    // the first tile's x loads go out before W's, so that the HBM latency of
    // the one overlaps the W split (both are waited for at the split below)
    load_tile(min(tile, tiles - 1));
    // W split into three bf16 planes, zero past HF columns and past fin.  All
    // of a thread's W loads are unconditional LW-wide loads at clamped
    // addresses, issued together: a guarded scalar load per element made the
    // split a chain of L2 round trips, one per loop iteration.
    {
        constexpr int WQ = (BN * KP + 256 * LW - 1) / (256 * LW);
        vec wv[WQ];
#pragma unroll
        for (int q = 0; q < WQ; ++q) {
            const int e = (tid + 256 * q) * LW;  // KP % 32 == 0: e..e+LW-1 share a row
            const int c = min(e / KP, HF - 1), k = min(e % KP, fin - LW);
            wv[q] = *reinterpret_cast<const vec*>(W + (size_t)c * fin + k);
        }
#pragma unroll
        for (int q = 0; q < WQ; ++q) {
            const int e = (tid + 256 * q) * LW;
            if (e < BN * KP) {
                const int c = e / KP, k = e % KP;
                const bool ok = c < HF && k < fin;  // fin % LW == 0: the whole vector
                const int o = c * WSB + k;
                if constexpr (LW == 1) {
                    bf16x2 p1, p2, p3;
                    split3_pair(f32x2{ok ? wv[q] : 0.f, 0.f}, p1, p2, p3);
                    wsb[0][o] = p1[0];
                    wsb[1][o] = p2[0];
                    wsb[2][o] = p3[0];
                } else if constexpr (LW == 2) {
                    bf16x2 p1, p2, p3;
                    split3_pair(ok ? wv[q] : f32x2{0.f, 0.f}, p1, p2, p3);
                    *reinterpret_cast<bf16x2*>(&wsb[0][o]) = p1;
                    *reinterpret_cast<bf16x2*>(&wsb[1][o]) = p2;
                    *reinterpret_cast<bf16x2*>(&wsb[2][o]) = p3;
                } else {
                    const f32x4 v = ok ? wv[q] : f32x4{0.f, 0.f, 0.f, 0.f};
                    bf16x2 p1a, p2a, p3a, p1b, p2b, p3b;
                    split3_pair(f32x2{v.x, v.y}, p1a, p2a, p3a);
                    split3_pair(f32x2{v.z, v.w}, p1b, p2b, p3b);
                    *reinterpret_cast<bf16x4*>(&wsb[0][o]) = bf16x4{p1a[0], p1a[1], p1b[0], p1b[1]};
                    *reinterpret_cast<bf16x4*>(&wsb[1][o]) = bf16x4{p2a[0], p2a[1], p2b[0], p2b[1]};
                    *reinterpret_cast<bf16x4*>(&wsb[2][o]) = bf16x4{p3a[0], p3a[1], p3b[0], p3b[1]};
                }
            }
        }
    }
    __syncthreads();

    const int hfp = round_up4(HF);
    const int lf = 31 - __builtin_clz((unsigned)F);  // F is a power of two <= 16
    float bb[NT], w1[NT], w2[NT];
    // (and c1/c2 per head: epilogue parameters stay in registers, since a global
    // load inside the tile loop would wait, vmcnt being in order, for the next
    // tile's x loads in flight)
    float cs1[NT], cs2[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int cc = t * 16 + cl;
        bb[t] = cc < HF ? bW[cc] : 0.f;
        w1[t] = cc < HF ? a1[cc] : 0.f;
        w2[t] = cc < HF ? a2[cc] : 0.f;
        const int h = min(cc >> lf, H - 1);
        cs1[t] = c1[h];
        cs2[t] = c2[h];
    }
    float* Os = osm[w];
    for (; tile < tiles; tile += tstride) {
        // split this tile's fragments (frees xr), then start the next tile's loads
        bf16x8 x1[KS], x2[KS], x3[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            float f[8];
#pragma unroll
            for (int q = 0; q < NL; ++q)
#pragma unroll
                for (int j = 0; j < LW; ++j) {
                    if constexpr (LW == 1) f[q] = xr[s][q];
                    else f[q * LW + j] = xr[s][q][j];
                }
            split3_x8(f32x4{f[0], f[1], f[2], f[3]}, f32x4{f[4], f[5], f[6], f[7]}, x1[s],
                      x2[s], x3[s]);
        }
        // unconditional (the last tile re-loads itself, unused): a conditional
        // load would make the compiler wait for every older store at the loop top
        load_tile(min(tile + tstride, tiles - 1));
        f32x4 acc[NT], cor[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = cor[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int o = (t * 16 + cl) * WSB + 32 * s + 8 * kq;
                const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(&wsb[0][o]);
                const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(&wsb[1][o]);
                const bf16x8 b3 = *reinterpret_cast<const bf16x8*>(&wsb[2][o]);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1[s], b1, acc[t], 0, 0, 0);
                cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1[s], b2, cor[t], 0, 0, 0);
                cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x2[s], b1, cor[t], 0, 0, 0);
                cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1[s], b3, cor[t], 0, 0, 0);
                cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x2[s], b2, cor[t], 0, 0, 0);
                cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x3[s], b1, cor[t], 0, 0, 0);
            }
        }
        const int row0 = tile * 16;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int cc = t * 16 + cl;
            const int h = cc >> lf, li = cl & (F - 1);
            float p1[4], p2[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float v = acc[t][i] + cor[t][i] + bb[t];  // Linear bias (GAT.py:43)
                Os[(kq * 4 + i) * OS + cc] = cc < HF ? v : 0.f;
                p1[i] = group_sum16(v * w1[t], F);
                p2[i] = group_sum16(v * w2[t], F);
            }
            if (li < 4 && li < F && h < H) {
                const float v1 = li == 0 ? p1[0] : li == 1 ? p1[1] : li == 2 ? p1[2] : p1[3];
                const float v2 = li == 0 ? p2[0] : li == 1 ? p2[1] : li == 2 ? p2[2] : p2[3];
                const int rr = row0 + kq * 4 + li;
                if (rr < n) {
                    if (Ss != nullptr) store_out1(Ss, (size_t)rr * ld_s + h, v1 + cs1[t], store_wt);
                    store_out1(s_dst, (size_t)rr * H + h, v2 + cs2[t], store_wt);
                }
            }
            if (F < 4 && li == 0 && h < H) {  // heads narrower than 4 lanes: rows F..3
#pragma unroll
                for (int i = 1; i < 4; ++i) {
                    const int rr = row0 + kq * 4 + i;
                    if (i >= F && rr < n) {
                        if (Ss != nullptr)
                            store_out1(Ss, (size_t)rr * ld_s + h, p1[i] + cs1[t], store_wt);
                        store_out1(s_dst, (size_t)rr * H + h, p2[i] + cs2[t], store_wt);
                    }
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        // Wh rows of the tile: float4 columns, 16 rows (row-major or planes)
        constexpr int C4 = BN / 4;
#pragma unroll
        for (int idx = lane; idx < 16 * C4; idx += 64) {
            const int r = idx / C4, col = 4 * (idx % C4);
            if (col < hfp && row0 + r < n) {
                const int g = col / slice_w;
                store_out4(Wh, (size_t)g * (size_t)slice_stride + (size_t)(row0 + r) * ld_wh +
                                   (col - g * slice_w),
                           *reinterpret_cast<const f32x4*>(Os + r * OS + col), store_wt);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ---------------------------------------------------------------------------
// Projection, whole-K variant (fin <= 64): the workgroup's 64 X rows are one
// contiguous 64*fin*4-byte chunk of HBM, and W [HF, fin] is contiguous too, so
// both are staged into LDS with fully coalesced float4 loads (16x fewer
// memory requests than per-row fragment loads) and the MFMAs read their A/B
// fragments from LDS.  The output tile goes back through LDS so that Wh rows
// leave as coalesced float4 stores and each (row, head) score is one short
// dot product per thread.  Two barriers per workgroup, no K loop.
// ---------------------------------------------------------------------------
// LDS layout of k_project_wk: [X tile | W tile] (reused for the output tile
// after the MFMAs), then the epilogue parameters [b | a1 | a2 (BN each) |
// c1 | c2 (64 each)] from this offset (floats).
__host__ __device__ inline int wk_param_offset(int fin, int nt) {
    const int tiles = ((64 * fin + 3) & ~3) + nt * 16 * fin;
    const int out = 64 * (nt * 16 + 4);
    return ((tiles > out ? tiles : out) + 3) & ~3;
}

__host__ __device__ inline int wk_lds_floats(int fin, int nt) {
    return wk_param_offset(fin, nt) + 3 * nt * 16 + 128;
}

// DIRECT (F in {4, 8, 16}): the MFMA operands are swapped (A = W fragment,
// B = x fragment), so the accumulator holds C^T: lane l has Wh[row l&15]
// [16t + 4(l>>4) .. +4], four consecutive columns of one row.  The epilogue
// then stores float4s straight from the accumulators and forms each head's
// scores by a DPP/xor sum over the F/4 lanes of the head: no output tile in
// LDS, no third barrier, no index divisions (PPI: tools/proj_floor.hip
// measured the projection's VALU count as what bounds it after the loads).
template <int NT, bool DIRECT = false>
__global__ __launch_bounds__(256) void k_project_wk(
    const float* __restrict__ X, int n, int fin,
    const float* __restrict__ W, const float* __restrict__ bW,
    const float* __restrict__ a1, const float* __restrict__ c1,
    const float* __restrict__ a2, const float* __restrict__ c2,
    int H, int F, int HF, float* __restrict__ Wh, int ld_wh,
    float* __restrict__ Ss, int ld_s, float* __restrict__ s_dst,
    int slice_w, long long slice_stride, int store_wt) {
    constexpr int BM = 64, BN = NT * 16;
    constexpr int OS = BN + 4;  // output-tile stride: float4-aligned rows, no write conflicts
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int cl = lane & 15, kq = lane >> 4;
    const int row0 = blockIdx.x * BM;
    const int rows = min(BM, n - row0);
    const int xs_n = round_up4(BM * fin);  // X tile floats (16-B aligned W tile after it)
    float* Xs = smem;
    float* Ws = smem + xs_n;
    // epilogue parameters in their own LDS region (past the X/W tiles and the
    // output tile): loaded now, with the tiles, instead of after the MFMAs
    float* Ps = smem + wk_param_offset(fin, NT);
    float* bs = Ps;
    float* a1s = Ps + BN;
    float* a2s = Ps + 2 * BN;
    float* c1s = Ps + 3 * BN;
    float* c2s = c1s + 64;
    if (tid < BN) {
        const bool ok = tid < HF;
        const int cc = ok ? tid : 0;
        const float bv = bW[cc], av1 = a1[cc], av2 = a2[cc];
        bs[tid] = ok ? bv : 0.f;
        a1s[tid] = ok ? av1 : 0.f;
        a2s[tid] = ok ? av2 : 0.f;
    }
    if (tid < H) {
        const float v1 = c1[tid], v2 = c2[tid];
        c1s[tid] = v1;
        c2s[tid] = v2;
    }

    // X rows [row0, row0+rows) are one contiguous chunk (row0*fin*4 = 256*b*fin bytes:
    // 16-B aligned) and W [HF, fin] another.  Each thread issues ALL its float4
    // loads first (fixed count, clamped addresses: a load->ds_write loop with a
    // runtime trip count waits on every load), then writes LDS.
    {
        constexpr int XIT = BM * 64 / 1024, WIT = BN * 64 / 1024;  // fin <= 64
        const float* xg = X + (size_t)row0 * fin;
        const int xc = rows * fin, xc4 = xc & ~3;
        const int wc = HF * fin, wc4 = wc & ~3;
        f32x4 xv[XIT], wv[WIT];
#pragma unroll
        for (int it = 0; it < XIT; ++it)
            xv[it] = *reinterpret_cast<const f32x4*>(xg + min(tid * 4 + it * 1024, max(xc4 - 4, 0)));
#pragma unroll
        for (int it = 0; it < WIT; ++it)
            wv[it] = *reinterpret_cast<const f32x4*>(W + min(tid * 4 + it * 1024, max(wc4 - 4, 0)));
#pragma unroll
        for (int it = 0; it < XIT; ++it) {
            const int i = tid * 4 + it * 1024;
            if (i < xc4) *reinterpret_cast<f32x4*>(Xs + i) = xv[it];
        }
#pragma unroll
        for (int it = 0; it < WIT; ++it) {
            const int i = tid * 4 + it * 1024;
            if (i < wc4) *reinterpret_cast<f32x4*>(Ws + i) = wv[it];
        }
        for (int i = xc4 + tid; i < BM * fin; i += 256) Xs[i] = i < xc ? xg[i] : 0.f;
        for (int i = wc4 + tid; i < BN * fin; i += 256) Ws[i] = i < wc ? W[i] : 0.f;
    }
    __syncthreads();

    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* xa = Xs + (w * 16 + cl) * fin + kq;
    const float* wb = Ws + cl * fin + kq;
    const int ks = fin / 4;
    int s = 0;
    for (; s + 4 <= ks; s += 4) {  // 4 full k-steps per iteration: LDS reads batched
        float a[4], bq[4][NT];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a[u] = xa[4 * (s + u)];
#pragma unroll
            for (int t = 0; t < NT; ++t) bq[u][t] = wb[t * 16 * fin + 4 * (s + u)];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int t = 0; t < NT; ++t)
                acc[t] = DIRECT
                    ? __builtin_amdgcn_mfma_f32_16x16x4f32(bq[u][t], a[u], acc[t], 0, 0, 0)
                    : __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], bq[u][t], acc[t], 0, 0, 0);
    }
    for (; s < ks; ++s) {
        const float a = xa[4 * s];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const float b = wb[t * 16 * fin + 4 * s];
            acc[t] = DIRECT ? __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, acc[t], 0, 0, 0)
                            : __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
        }
    }
    if (fin & 3) {  // last partial k-step
        const bool ok = 4 * ks + kq < fin;
        const float a = ok ? xa[4 * ks] : 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const float b = ok ? wb[t * 16 * fin + 4 * ks] : 0.f;
            acc[t] = DIRECT ? __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, acc[t], 0, 0, 0)
                            : __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
        }
    }
    if constexpr (DIRECT) {
        proj_direct_epilogue<NT>(acc, row0 + w * 16 + cl, n, kq, bs, a1s, a2s, c1s, c2s, H, F,
                                 HF, Wh, ld_wh, Ss, ld_s, s_dst, slice_w, slice_stride,
                                 store_wt);
        return;
    }
    __syncthreads();  // X/W tiles dead: reuse LDS for the output tile

    float* Os = smem;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int cc = t * 16 + cl;
        const float bb = bs[cc];  // Linear bias inside Wh (GAT.py:43); 0 past HF
#pragma unroll
        for (int i = 0; i < 4; ++i) Os[(w * 16 + kq * 4 + i) * OS + cc] = acc[t][i] + bb;
    }
    __syncthreads();
    // Wh stores: slice-major so consecutive lanes fill one slice plane's rows
    // (unsliced: slice_w >= hfp, one slice, the plain row-major order)
    const int hfp = round_up4(HF), c4n = hfp / 4;
    const int cs4 = (slice_w < hfp ? slice_w : hfp) / 4;  // float4s per slice row
    for (int idx = tid; idx < rows * c4n; idx += 256) {
        const int g = idx / (rows * cs4), rem = idx - g * rows * cs4;
        const int r = rem / cs4, q = rem - r * cs4;
        const int c4 = g * cs4 + q;
        f32x4 v = *reinterpret_cast<const f32x4*>(Os + r * OS + 4 * c4);
        if (4 * c4 + 3 >= HF) {  // zero the pad columns [HF, hfp)
            if (4 * c4 + 0 >= HF) v.x = 0.f;
            if (4 * c4 + 1 >= HF) v.y = 0.f;
            if (4 * c4 + 2 >= HF) v.z = 0.f;
            if (4 * c4 + 3 >= HF) v.w = 0.f;
        }
        store_out4(Wh, (size_t)g * (size_t)slice_stride + (size_t)(row0 + r) * ld_wh + 4 * q, v,
                   store_wt);
    }
    // attention Linears on the fp32 Wh (GAT.py:44-45): s = Wh_h . a_h + c_h
    for (int idx = tid; idx < rows * H; idx += 256) {
        const int r = idx / H, h = idx - r * H;
        const float* o = Os + r * OS + h * F;
        const float* p1 = a1s + h * F;
        const float* p2 = a2s + h * F;
        float v1 = 0.f, v2 = 0.f;
        for (int f = 0; f < F; ++f) {
            v1 = fmaf(o[f], p1[f], v1);
            v2 = fmaf(o[f], p2[f], v2);
        }
        if (Ss != nullptr) store_out1(Ss, (size_t)(row0 + r) * ld_s + h, v1 + c1s[h], store_wt);
        store_out1(s_dst, (size_t)(row0 + r) * H + h, v2 + c2s[h], store_wt);
    }
}

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
template <int LPE, int HP>
__global__ __launch_bounds__(64) void k_edge_fwd(
    const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ order,
    int row_begin, int row_end,
    const float* __restrict__ Wh, int ld_wh, const float* __restrict__ Ss, int ld_s,
    const float* __restrict__ s_dst,
    int H, int F, int HF, int concat, int act, float slope, const float* __restrict__ bias,
    float* __restrict__ out, int ld_out, float* __restrict__ lse, DropArgs drop_arg,
    float* __restrict__ y_heads) {
    const DropArgs drop = resolve_drop(drop_arg);
    constexpr int C = (512 / HP) < kWave ? (512 / HP) : kWave;  // edges per chunk
    constexpr int R = C * HP / kWave;                          // score slots per lane
    constexpr int EPI = kWave / LPE;                           // edges per gather step
    constexpr int U = (EPI >= 16) ? 2 : 4;                     // gather steps in flight
    __shared__ int col_s[C];
    __shared__ float p_s[C * HP];
    __shared__ float hv_s[HP];
    __shared__ float y_s[LPE * 4];

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
#pragma unroll
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
//     separate "virtual rows", and k_edge_merge combines their states.
// ---------------------------------------------------------------------------
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

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

EdgeRows rows_of_csr(const int* rowptr) {
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

// KINK (training forward, recompute backward): also the per-head "kink sums"
//   Q[i,h] = sum_j A_ij L'(z_ij) Wh[j,h]   and   R[i,h] = sum_j alpha_ij L'(z_ij)
// (A = dropped coefficient, alpha = undropped, L' = 1 for z > 0 else slope).  The
// backward's dL/ds_dst[i,h] = sum_j alpha_ij L'_ij (drop_ij dy_i.Wh_j - delta_i)
// is then dy_i.Q_i - delta_i R_i: an elementwise kernel (k_bwd_table) instead of
// a second pass over every in-edge (k_bwd_targets).  Q and R cost one more
// accumulator per float4 and no gathers: the loop already holds Wh_j and p_ij.
// S = 2 (short rows, few rows per launch): TWO lane groups per row, each
// walking every other chunk of the row's in-edges (half 0 chunks 0, 2, 4, ...,
// half 1 chunks 1, 3, ...); at the end each lane merges its online-softmax
// state with its partner's (lane ^ G): M = max(m, m'), l = l 2^(m-M) + l'
// 2^(m'-M), acc likewise (the hub merge, in registers).  The chain of
// dependent chunk loads per row halves and a launch has twice the waves.
// Only half 0 stores.  Not with KINK or PIPE.
template <int G, int U, int V, bool FUSED, bool PIPE = false, bool KINK = false, int S = 1>
__global__ __launch_bounds__(256) void k_edge_grp(
    const EdgeRows er, const int* __restrict__ col, const int* __restrict__ order,
    int row_begin, int row_end,
    const float* __restrict__ Wh, int ld_wh, const float* __restrict__ Ss, int ld_s,
    const float* __restrict__ a_src, const float* __restrict__ c_src,
    const float* __restrict__ s_dst, int H, int F, int HF, int concat, float slope,
    const float* __restrict__ bias, float* __restrict__ out, int ld_out,
    float* __restrict__ lse, DropArgs drop_arg, float* __restrict__ y_heads,
    int nslices, int slice_w, long long slice_stride, float* __restrict__ q_heads,
    float* __restrict__ r_heads, int store_wt) {
    const DropArgs drop = resolve_drop(drop_arg);
    static_assert(S == 1 || (S == 2 && !KINK && !PIPE && G * S <= kWave), "split rows");
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
    const int half = S == 2 ? (lane / G) & 1 : 0;  // S = 2: which chunks of the row
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
    const int si = er.by_pos ? pos : r;  // segment / state index
    const int e0 = er.eb[si], e1 = er.ee[si];
    const bool kahan = e1 - e0 >= 1024;
    const bool dropping = drop.thresh != 0u;  // kernel-uniform: a scalar branch
    // the target's share of every score, in log2 units (LeakyReLU is positively
    // homogeneous: LReLU(z) log2e = LReLU(z log2e)); + c1 when s_src is recomputed
    const float sd = (s_dst[(size_t)r * H + h] + c1) * kLog2e;
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
            const float* row = Whs + (size_t)j[u] * ld_wh;
#pragma unroll
            for (int q = 0; q < V; ++q) v[u][q] = *reinterpret_cast<const f32x4*>(row + 4 * q);
            if constexpr (!FUSED) s[u] = Ss[(size_t)j[u] * ld_s + h];
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
            const int hl = F / (4 * V);  // lanes per head
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
        if (!kahan) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float p = __builtin_amdgcn_exp2f(s[u] - m_new);
                l += p;  // the softmax denominator never sees the dropout
                float pa = p;
                if (dropping) pa = p * drop_factor(drop, k + u, h, H);
#pragma unroll
                for (int q = 0; q < V; ++q) acc[q] += pa * v[u][q];
                kink(u, p, pa, racc, accq);
            }
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
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const float p = __builtin_amdgcn_exp2f(s[u] - m_new);
                ls += p;
                float pa = p;
                if (dropping) pa = p * drop_factor(drop, k + u, h, H);
#pragma unroll
                for (int q = 0; q < V; ++q) cs[q] += pa * v[u][q];
                kink(u, p, pa, rs, qs);
            }
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
        // gathers software-pipelined one chunk ahead too: chunk k+U's rows are
        // in flight while chunk k is scored and accumulated (col two ahead)
        f32x4 vc[U][V];
        float sc[U];
        fetch(cv, vc, sc);
        int cn[CL];
#pragma unroll
        for (int t = 0; t < CL; ++t) cn[t] = e1 > e0 ? col[min(e0 + U + cfirst + t * cstep, e1 - 1)] : 0;
        for (int k = e0; k < e1; k += U) {
            int cnn[CL];
#pragma unroll
            for (int t = 0; t < CL; ++t) cnn[t] = col[min(k + 2 * U + cfirst + t * cstep, e1 - 1)];
            f32x4 vn[U][V];
            float sn[U];
            if (k + U < e1) fetch(cn, vn, sn);
            consume(k, vc, sc);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                sc[u] = sn[u];
#pragma unroll
                for (int q = 0; q < V; ++q) vc[u][q] = vn[u][q];
            }
#pragma unroll
            for (int t = 0; t < CL; ++t) cn[t] = cnn[t];
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
    if constexpr (S == 2) {
        // merge the two halves' states (both halves end with the same values:
        // a + b == b + a exactly); the Kahan compensation is applied first
        if (kahan) {
            l -= lc;
            lc = 0.f;
#pragma unroll
            for (int q = 0; q < V; ++q) {
                acc[q] -= cmp[q];
                cmp[q] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
        const float mp = __shfl_xor(m, G), lp = __shfl_xor(l, G);
        const float mm = fmaxf(m, mp);
        // an empty half (fewer than U + 1 edges) has m = -inf and contributes 0
        const float so = m == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m - mm);
        const float sp = mp == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mp - mm);
        l = l * so + lp * sp;
#pragma unroll
        for (int q = 0; q < V; ++q) {
            f32x4 ap;
            ap.x = __shfl_xor(acc[q].x, G);
            ap.y = __shfl_xor(acc[q].y, G);
            ap.z = __shfl_xor(acc[q].z, G);
            ap.w = __shfl_xor(acc[q].w, G);
            acc[q] = acc[q] * so + ap * sp;
        }
        m = mm;
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
// hub k's segment states are virtual rows [vptr[k], vptr[k+1]).  Per head:
//   M = max_s m_s,  L = sum_s l_s 2^(m_s - M),  y = sum_s acc_s 2^(m_s - M) / (L + 1e-16)
// which is the segmented softmax of PyG utils.softmax (GAT.py:60) regrouped.
// One wave per hub row; the segment loop is short (<= a few hundred).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_edge_merge(
    const int* __restrict__ hub_rows, const int* __restrict__ vptr, int n_hub,
    const float* __restrict__ st_acc, int ld_st, const float* __restrict__ st_ml, int H, int F,
    int HF, int concat, const float* __restrict__ bias, float* __restrict__ out, int ld_out,
    float* __restrict__ lse, float* __restrict__ y_heads) {
    __shared__ float Ms[GAT_MAX_HEADS], Ls[GAT_MAX_HEADS], ys[GAT_MAX_HF];
    const int k = blockIdx.x;
    if (k >= n_hub) return;
    const int lane = threadIdx.x;
    const int r = hub_rows[k], s0 = vptr[k], s1 = vptr[k + 1];
    for (int h = lane; h < H; h += kWave) {
        float M = -INFINITY;
        for (int sg = s0; sg < s1; ++sg) M = fmaxf(M, st_ml[(size_t)sg * 2 * H + h]);
        float L = 0.f;
        for (int sg = s0; sg < s1; ++sg) {
            const float ms = st_ml[(size_t)sg * 2 * H + h];
            if (ms != -INFINITY) L += st_ml[(size_t)sg * 2 * H + H + h] * __builtin_amdgcn_exp2f(ms - M);
        }
        Ms[h] = M;
        Ls[h] = L;
        if (lse != nullptr) lse[(size_t)r * H + h] = (M + log2f(L)) * kLn2;
    }
    __syncthreads();
    for (int cc = lane; cc < HF; cc += kWave) {
        const int h = cc / F;
        const float M = Ms[h];
        float a = 0.f;
        for (int sg = s0; sg < s1; ++sg) {
            const float ms = st_ml[(size_t)sg * 2 * H + h];
            if (ms != -INFINITY) a += st_acc[(size_t)sg * ld_st + cc] * __builtin_amdgcn_exp2f(ms - M);
        }
        const float y = a / (Ls[h] + 1e-16f);
        if (y_heads != nullptr) y_heads[(size_t)r * HF + cc] = y;
        if (concat) out[(size_t)r * ld_out + cc] = y + bias[cc];
        else ys[cc] = y;
    }
    if (!concat) {
        __syncthreads();
        for (int f = lane; f < F; f += kWave) {
            float sum = 0.f;
            for (int h = 0; h < H; ++h) sum += ys[h * F + f];
            out[(size_t)r * ld_out + f] = sum / (float)H + bias[f];
        }
    }
}

// ---------------------------------------------------------------------------
// CSR-by-target build with the self-loops added.  One stable radix sort of
// 64-bit keys (target << b | source) over the E input edges plus the N loops:
// rows are grouped by target and, within a row, sources ascend.  Sorted
// sources make the rows the edge kernel runs together (similar in-degree,
// by the degree schedule) sweep the node table in step, which turns part of
// the random Wh gathers into L2 hits (Reddit scale: 3.81 -> 3.43 ms).
// Duplicate (target, source) pairs — multi-edges, a pre-existing self-loop
// next to the added one — stay in input order (stable sort).
// ---------------------------------------------------------------------------
__global__ void k_csr_prepare(const long long* __restrict__ ei, long long E, int n,
                              unsigned kb, unsigned long long* __restrict__ keys,
                              int* __restrict__ err) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < E + n; k += stride) {
        unsigned long long s, d;
        if (k < E) {
            const long long ss = ei[k], dd = ei[E + k];
            const bool ok = ss >= 0 && ss < n && dd >= 0 && dd < n;
            if (!ok) atomicOr(err, 1);
            s = ok ? (unsigned long long)ss : 0ull;
            d = ok ? (unsigned long long)dd : 0ull;
        } else {
            s = d = (unsigned long long)(k - E);  // the added self-loop of node k - E
        }
        keys[k] = (d << kb) | s;
    }
}

__global__ void k_csr_rowptr(const unsigned long long* __restrict__ sorted_keys, long long nnz,
                             int n, unsigned kb, int* __restrict__ rowptr) {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i > n) return;
    // lower_bound over the target field
    long long lo = 0, hi = nnz;
    while (lo < hi) {
        const long long mid = (lo + hi) >> 1;
        if ((long long)(sorted_keys[mid] >> kb) < i) lo = mid + 1; else hi = mid;
    }
    rowptr[i] = (int)lo;
}

__global__ void k_csr_col(const unsigned long long* __restrict__ sorted_keys, long long nnz,
                          unsigned kb, int* __restrict__ col) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    const unsigned long long mask = (1ull << kb) - 1ull;
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < nnz; k += stride)
        col[k] = (int)(sorted_keys[k] & mask);
}

__global__ void k_degree_keys(const int* __restrict__ rowptr, int n, unsigned* __restrict__ keys,
                              int* __restrict__ rows) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
        keys[i] = (unsigned)(rowptr[i + 1] - rowptr[i]);
        rows[i] = (int)i;
    }
}

// ---------------------------------------------------------------------------
// CSC (edges grouped by SOURCE) over the CSR's edge positions, for the
// backward pass: the gradient of a source row gathers over its out-edges.
//   csc_ptr[j]       first CSC slot of source j
//   csc_dst[c]       target row of the edge in CSC slot c
//   csc_eid[c]       CSR position of the edge in CSC slot c
//   csr_to_csc[k]    CSC slot of CSR position k
// Built by a stable radix sort of (col[k], k): within a source, edges keep
// CSR order, so every reduction over them is deterministic.  The target row
// of a CSR position is found by binary search in rowptr (L2-resident) rather
// than gathered from a per-edge array.
// ---------------------------------------------------------------------------
__global__ void k_csc_keys(long long nnz, const int* __restrict__ col,
                           unsigned* __restrict__ keys, int* __restrict__ vals) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < nnz; k += stride) {
        keys[k] = (unsigned)col[k];
        vals[k] = (int)k;
    }
}

__global__ void k_csc_ptr(const unsigned* __restrict__ sorted_keys, long long nnz, int n,
                          int* __restrict__ csc_ptr) {
    const long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (j > n) return;
    long long lo = 0, hi = nnz;
    while (lo < hi) {
        const long long mid = (lo + hi) >> 1;
        if (sorted_keys[mid] < (unsigned)j) lo = mid + 1; else hi = mid;
    }
    csc_ptr[j] = (int)lo;
}

__global__ void k_csc_fill(const int* __restrict__ sorted_vals, const int* __restrict__ rowptr,
                           int n, long long nnz, int* __restrict__ csc_dst,
                           int* __restrict__ csr_to_csc) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x; c < nnz; c += stride) {
        const int k = sorted_vals[c];
        // the row holding CSR position k: last i with rowptr[i] <= k
        int lo = 0, hi = n - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (rowptr[mid] <= k) lo = mid; else hi = mid - 1;
        }
        csc_dst[c] = lo;
        if (csr_to_csc != nullptr) csr_to_csc[k] = (int)c;
    }
}

// ---------------------------------------------------------------------------
// Backward, pass 1: one wave per TARGET row i (CSR), lanes over (edge, head)
// slots as in k_edge_fwd's score phase.  With dy = dL/dy_heads[i] (concat: the
// row of g; mean: g[i]/H for every head), y = the forward's normalised
// per-head aggregation and alpha = exp(e - lse):
//   delta_h   = dy_h . y_h
//   dA        = drop * (dy_h . Wh[j]_h)            (A = alpha * drop, drop = keep/(1-p) or 0)
//   de        = alpha * (dA - delta_h)              softmax backward
//   dz        = de * (z > 0 ? 1 : slope)            LeakyReLU backward
//   ds_dst[i] = sum_edges dz
// and stores (A, dz) per (edge, head) — interleaved, one 8H-byte record per
// edge — at the edge's CSC slot, so pass 2 reads them contiguously.
// Algorithmic bytes per edge: 4 (col) + 4 (csr_to_csc) + 4H (s_src) + 4HF (Wh
// row) + 8H (A, dz); per row: 4HF (g) + 4HF (y) + 8H (s_dst, lse) + 4H.
// ---------------------------------------------------------------------------
template <int HP>
__global__ __launch_bounds__(64) void k_edge_bwd_rows(
    const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ order,
    int row_begin, int row_end, const int* __restrict__ csr_to_csc,
    const float* __restrict__ Wh, int ld_wh, const float* __restrict__ Ss, int ld_s,
    const float* __restrict__ s_dst, const float* __restrict__ lse,
    const float* __restrict__ y_heads, const float* __restrict__ g, int H, int F, int HF,
    int concat, int act, float slope, DropArgs drop_arg, float* __restrict__ ds_dst,
    float2* __restrict__ az_out) {
    const DropArgs drop = resolve_drop(drop_arg);
    constexpr int C = (512 / HP) < kWave ? (512 / HP) : kWave;
    constexpr int R = C * HP / kWave;
    __shared__ float dy_s[GAT_MAX_HF];
    __shared__ float delta_s[HP];
    __shared__ int col_s[C];
    __shared__ int slot_s[C];

    const int lane = threadIdx.x;
    const int pos = row_begin + blockIdx.x;
    if (pos >= row_end) return;
    const int r = order != nullptr ? order[pos] : pos;
    const int e0 = rowptr[r], e1 = rowptr[r + 1];
    const float inv_h = 1.f / (float)H;
    for (int c = lane; c < HF; c += kWave)
        dy_s[c] = concat ? g[(size_t)r * HF + c] : g[(size_t)r * F + (c % F)] * inv_h;
    __syncthreads();
    if (lane < H) {
        float d = 0.f;
        const float* yr = y_heads + (size_t)r * HF + lane * F;
        for (int f = 0; f < F; ++f) d = fmaf(dy_s[lane * F + f], yr[f], d);
        delta_s[lane] = d;
    }
    __syncthreads();
    const int hs = lane & (HP - 1);
    const bool hs_ok = hs < H;
    const float sd = hs_ok ? s_dst[(size_t)r * H + hs] : 0.f;
    const float ls = hs_ok ? lse[(size_t)r * H + hs] : 0.f;
    const float dl = hs_ok ? delta_s[hs] : 0.f;
    const float* dyh = dy_s + (hs_ok ? hs : 0) * F;
    float dsd = 0.f;
    for (int base = e0; base < e1; base += C) {
        const int nk = min(C, e1 - base);
        if (lane < nk) {
            col_s[lane] = col[base + lane];
            slot_s[lane] = csr_to_csc[base + lane];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int k = (lane + kWave * q) / HP;
            const bool valid = k < nk && hs_ok;
            const int j = col_s[k < nk ? k : nk - 1];
            const float z = sd + Ss[(size_t)j * ld_s + (hs_ok ? hs : 0)];
            const bool hsm = act == GAT_ACT_HEAD_SOFTMAX;
            const float ev = hsm ? head_softmax<HP>(z, valid) : score_act(act, z, slope);
            float de = 0.f, a = 0.f, dm = 1.f;
            if (valid) {
                a = expf(ev - ls);
                const float* wr = Wh + (size_t)j * ld_wh + hs * F;
                float da = 0.f;
                for (int f = 0; f < F; ++f) da = fmaf(dyh[f], wr[f], da);
                if (drop.thresh != 0u) dm = drop_factor(drop, base + k, hs, H);
                de = a * (dm * da - dl);
            }
            float dz;
            if (hsm) {  // d softmax_h: e_h (de_h - sum_h' e_h' de_h')
                const float sum = head_sum<HP>(ev * de);
                dz = ev * (de - sum);
            } else {
                dz = de * score_act_grad(act, z, slope);
            }
            if (valid) {
                dsd += dz;
                az_out[(size_t)slot_s[k] * H + hs] = make_float2(a * dm, dz);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int off = HP; off < kWave; off <<= 1) dsd += __shfl_xor(dsd, off);
    if (lane < H) ds_dst[(size_t)r * H + lane] = dsd;
}

// ---------------------------------------------------------------------------
// Backward, pass 1, lane-group variant (LeakyReLU, F/4 a power of two): the
// k_edge_grp layout — G lanes per target row, each lane one float4 of one
// head — so each in-edge costs one coalesced Wh-row gather, the source score
// is recomputed from it (fused, as in the forward) and the two per-head dot
// products (s_src and dA = dy . Wh[j]) are DPP sums over the head's lanes.
// No LDS, no barriers; col and csr_to_csc loads software-pipelined.
// Same results as k_edge_bwd_rows up to fp32 rounding.
// ---------------------------------------------------------------------------
template <int G, int U>
__global__ __launch_bounds__(256) void k_edge_bwd_grp(
    const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ order,
    int row_begin, int row_end, const int* __restrict__ csr_to_csc,
    const float* __restrict__ Wh, int ld_wh, const float* __restrict__ a_src,
    const float* __restrict__ c_src, const float* __restrict__ s_dst,
    const float* __restrict__ lse, const float* __restrict__ y_heads,
    const float* __restrict__ g, int H, int F, int HF, int concat, float slope, DropArgs drop_arg,
    float* __restrict__ ds_dst, float2* __restrict__ az_out) {
    const DropArgs drop = resolve_drop(drop_arg);
    constexpr int CL = (U + G - 1) / G;
    const int lane = threadIdx.x & 63;
    const int c = lane & (G - 1);
    const int gbase = lane & ~(G - 1);
    const int pos = row_begin + (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / G);
    if (pos >= row_end) return;
    const int r = order != nullptr ? order[pos] : pos;
    const bool c_ok = 4 * c < HF;
    const int coff = c_ok ? 4 * c : 0;
    const int h = coff / F;
    const int hl = F / 4;  // lanes per head
    const bool leader = c_ok && (coff % F) == 0;
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
    const f32x4 a4 = c_ok ? *reinterpret_cast<const f32x4*>(a_src + coff) : zero4;
    const float c1 = c_src[h];
    f32x4 dy = zero4, yv = zero4;
    if (c_ok) {
        if (concat) {
            dy = *reinterpret_cast<const f32x4*>(g + (size_t)r * HF + coff);
        } else {
            dy = *reinterpret_cast<const f32x4*>(g + (size_t)r * F + (coff % F));
            dy *= 1.f / (float)H;
        }
        yv = *reinterpret_cast<const f32x4*>(y_heads + (size_t)r * HF + coff);
    }
    auto hsum = [&](float v) {
        if (hl <= 16) return group_sum16(v, hl);
        for (int off = 1; off < hl; off <<= 1) v += __shfl_xor(v, off);
        return v;
    };
    const float dl = hsum(dy.x * yv.x + dy.y * yv.y + dy.z * yv.z + dy.w * yv.w);
    const float sd = s_dst[(size_t)r * H + h] + c1;
    const float ls2 = lse[(size_t)r * H + h] * kLog2e;
    const int e0 = rowptr[r], e1 = rowptr[r + 1];
    float dsd = 0.f;
    int cv[CL], sv[CL];
#pragma unroll
    for (int t = 0; t < CL; ++t) {
        const int kk = min(e0 + c + t * G, e1 - 1);
        cv[t] = e1 > e0 ? col[kk] : 0;
        sv[t] = e1 > e0 ? csr_to_csc[kk] : 0;
    }
    for (int k = e0; k < e1; k += U) {
        const int nk = min(U, e1 - k);
        int cn[CL], sn[CL];
#pragma unroll
        for (int t = 0; t < CL; ++t) {
            const int kk = min(k + U + c + t * G, e1 - 1);
            cn[t] = col[kk];
            sn[t] = csr_to_csc[kk];
        }
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = __shfl(cv[u / G], gbase + (u % G));
            v[u] = *reinterpret_cast<const f32x4*>(Wh + (size_t)j * ld_wh + coff);
        }
        float ss[U], da[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ss[u] = v[u].x * a4.x + v[u].y * a4.y + v[u].z * a4.z + v[u].w * a4.w;
            da[u] = v[u].x * dy.x + v[u].y * dy.y + v[u].z * dy.z + v[u].w * dy.w;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ss[u] = hsum(ss[u]);
            da[u] = hsum(da[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int slot = __shfl(sv[u / G], gbase + (u % G));
            const float z = sd + ss[u];
            const float a = __builtin_amdgcn_exp2f(fmaxf(z, z * slope) * kLog2e - ls2);
            const float dm = drop.thresh != 0u ? drop_factor(drop, k + u, h, H) : 1.f;
            const float de = a * (dm * da[u] - dl);
            const float dz = z > 0.f ? de : de * slope;
            if (u < nk) {
                dsd += dz;
                if (leader) az_out[(size_t)slot * H + h] = make_float2(a * dm, dz);
            }
        }
#pragma unroll
        for (int t = 0; t < CL; ++t) {
            cv[t] = cn[t];
            sv[t] = sn[t];
        }
    }
    if (leader) ds_dst[(size_t)r * H + h] = dsd;
}

// ---------------------------------------------------------------------------
// Recompute backward (LeakyReLU, F/4 a power of two): no per-edge state.
//
// Pass 1, per TARGET row i (k_edge_grp layout): delta_h = dy_h . y_h, then over
// the in-edges the same recomputation as k_edge_bwd_grp, accumulating only
// ds_dst[i].  Writes one row of the target table
//   T[i] = [ g_i (ldg, 0-padded to 4) | per head (s_dst, lse, delta, 0) ]
// so pass 2 gathers everything it needs about a target with two float4 loads
// per lane.  Per edge: 4 (col) + 4HF (Wh row) bytes, as the forward.
// ---------------------------------------------------------------------------
template <int G, int U>
__global__ __launch_bounds__(256) void k_bwd_targets(
    const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ order,
    int row_begin, int row_end, const float* __restrict__ Wh, int ld_wh,
    const float* __restrict__ a_src, const float* __restrict__ c_src,
    const float* __restrict__ s_dst, const float* __restrict__ lse,
    const float* __restrict__ y_heads, const float* __restrict__ g, int H, int F, int HF,
    int concat, float slope, DropArgs drop_arg, float* __restrict__ ds_dst,
    float* __restrict__ T, int ld_t) {
    const DropArgs drop = resolve_drop(drop_arg);
    constexpr int CL = (U + G - 1) / G;
    const int lane = threadIdx.x & 63;
    const int c = lane & (G - 1);
    const int gbase = lane & ~(G - 1);
    const int pos = row_begin + (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / G);
    if (pos >= row_end) return;
    const int r = order != nullptr ? order[pos] : pos;
    const bool c_ok = 4 * c < HF;
    const int coff = c_ok ? 4 * c : 0;
    const int h = coff / F;
    const int hl = F / 4;
    const bool leader = c_ok && (coff % F) == 0;
    const int ldg = concat ? HF : F;
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
    const f32x4 a4 = c_ok ? *reinterpret_cast<const f32x4*>(a_src + coff) : zero4;
    const float c1 = c_src[h];
    f32x4 g4 = zero4, yv = zero4;
    const bool g_ok = c_ok && (concat || coff < F);
    if (c_ok) {
        g4 = *reinterpret_cast<const f32x4*>(g + (size_t)r * ldg + (concat ? coff : coff % F));
        yv = *reinterpret_cast<const f32x4*>(y_heads + (size_t)r * HF + coff);
    }
    const f32x4 dy = concat ? g4 : g4 * (1.f / (float)H);
    auto hsum = [&](float v) {
        if (hl <= 16) return group_sum16(v, hl);
        for (int off = 1; off < hl; off <<= 1) v += __shfl_xor(v, off);
        return v;
    };
    const float dl = hsum(dy.x * yv.x + dy.y * yv.y + dy.z * yv.z + dy.w * yv.w);
    const float sdv = s_dst[(size_t)r * H + h];
    const float lsv = lse[(size_t)r * H + h];
    const float sd = sdv + c1;
    const float ls2 = lsv * kLog2e;
    const int e0 = rowptr[r], e1 = rowptr[r + 1];
    float dsd = 0.f;
    int cv[CL];
#pragma unroll
    for (int t = 0; t < CL; ++t) cv[t] = e1 > e0 ? col[min(e0 + c + t * G, e1 - 1)] : 0;
    for (int k = e0; k < e1; k += U) {
        const int nk = min(U, e1 - k);
        int cn[CL];
#pragma unroll
        for (int t = 0; t < CL; ++t) cn[t] = col[min(k + U + c + t * G, e1 - 1)];
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = __shfl(cv[u / G], gbase + (u % G));
            v[u] = *reinterpret_cast<const f32x4*>(Wh + (size_t)j * ld_wh + coff);
        }
        float ss[U], da[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ss[u] = hsum(v[u].x * a4.x + v[u].y * a4.y + v[u].z * a4.z + v[u].w * a4.w);
            da[u] = hsum(v[u].x * dy.x + v[u].y * dy.y + v[u].z * dy.z + v[u].w * dy.w);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float z = sd + ss[u];
            const float a = __builtin_amdgcn_exp2f(fmaxf(z, z * slope) * kLog2e - ls2);
            const float dm = drop.thresh != 0u ? drop_factor(drop, k + u, h, H) : 1.f;
            const float de = a * (dm * da[u] - dl);
            const float dz = z > 0.f ? de : de * slope;
            dsd += u < nk ? dz : 0.f;
        }
#pragma unroll
        for (int t = 0; t < CL; ++t) cv[t] = cn[t];
    }
    float* tr = T + (size_t)r * ld_t;
    if (g_ok) *reinterpret_cast<f32x4*>(tr + coff) = g4;
    if (leader) {
        ds_dst[(size_t)r * H + h] = dsd;
        *reinterpret_cast<f32x4*>(tr + round_up4(ldg) + 4 * h) = f32x4{sdv, lsv, dl, 0.f};
    }
}

// ---------------------------------------------------------------------------
// Pass 1 without edges (after the kink-sum forward, k_edge_grp<..., KINK>):
// per target row i and head h, with dy = dL/dy_h and delta = dy . y,
//   ds_dst[i,h] = dy . Q[i,h] - delta R[i,h]
// (= sum_j alpha_ij L'(z_ij) (drop_ij dy . Wh_j - delta), the sum k_bwd_targets
// walks the in-edges for), and the target table row exactly as k_bwd_targets
// writes it.  G lanes per row (G = next_pow2(HF/4)), one float4 of one head each.
// Per row: 4 ldg (g) + 8 HF (y, Q) + 12 H bytes read, 4 ld_t + 4 H written.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_bwd_table(
    int n, int G, const float* __restrict__ s_dst, const float* __restrict__ lse,
    const float* __restrict__ y_heads, const float* __restrict__ q_heads,
    const float* __restrict__ r_heads, const float* __restrict__ g, int H, int F, int HF,
    int concat, float* __restrict__ ds_dst, float* __restrict__ T, int ld_t) {
    const int lane = threadIdx.x & 63;
    const int c = lane & (G - 1);
    const long long r = (blockIdx.x * (long long)blockDim.x + threadIdx.x) / G;
    if (r >= n) return;  // whole groups (G divides 64)
    const bool c_ok = 4 * c < HF;
    const int coff = c_ok ? 4 * c : 0;
    const int h = coff / F;
    const int hl = F / 4;
    const bool leader = c_ok && (coff % F) == 0;
    const int ldg = concat ? HF : F;
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
    f32x4 g4 = zero4, yv = zero4, qv = zero4;
    const bool g_ok = c_ok && (concat || coff < F);
    if (c_ok) {
        g4 = *reinterpret_cast<const f32x4*>(g + r * ldg + (concat ? coff : coff % F));
        yv = *reinterpret_cast<const f32x4*>(y_heads + r * HF + coff);
        qv = *reinterpret_cast<const f32x4*>(q_heads + r * HF + coff);
    }
    const f32x4 dy = concat ? g4 : g4 * (1.f / (float)H);
    auto hsum = [&](float v) {
        if (hl <= 16) return group_sum16(v, hl);
        for (int off = 1; off < hl; off <<= 1) v += __shfl_xor(v, off);
        return v;
    };
    const float dl = hsum(dy.x * yv.x + dy.y * yv.y + dy.z * yv.z + dy.w * yv.w);
    const float dq = hsum(dy.x * qv.x + dy.y * qv.y + dy.z * qv.z + dy.w * qv.w);
    float* tr = T + r * ld_t;
    if (g_ok) *reinterpret_cast<f32x4*>(tr + coff) = g4;
    if (leader) {
        ds_dst[r * H + h] = dq - dl * r_heads[r * H + h];
        *reinterpret_cast<f32x4*>(tr + round_up4(ldg) + 4 * h) =
            f32x4{s_dst[r * H + h], lse[r * H + h], dl, 0.f};
    }
}

// ---------------------------------------------------------------------------
// Pass 2, per SOURCE row j (lane-group layout over the CSC): lane owns one
// float4 of Wh[j] (one head).  Per out-edge j -> i (slot e, CSR position
// k = csc_eid[e]): gather T[i] (the lane's g float4 + its head's
// (s_dst, lse, delta)), recompute
//   z = s_dst[i] + s_src[j], A = drop * exp(LReLU(z) - lse[i]),
//   dA = drop * (dy_i . Wh[j]) (DPP head sum), dz = A_undropped (dA - delta) LReLU'(z)
// and accumulate dWh[j] += A dy_i, ds_src[j] += dz.  Rows are strided over a
// fixed grid; each lane keeps its rows' contributions to da1/da2/dc1/dc2/db/
// dbias in registers, the wave's groups are combined by xor-shuffles and the
// wave writes one partial row [da1 | da2 | dc1 | dc2 | db | dbias] (summed by
// gat_sum_partials; deterministic).
// Per edge: 4 (csc_dst) + 4 (csc_eid, with dropout) + 4 ldg + 16 H bytes.
// ---------------------------------------------------------------------------
template <int G, int U>
__global__ __launch_bounds__(256) void k_bwd_sources(
    const int* __restrict__ csc_ptr, const int* __restrict__ csc_dst,
    const int* __restrict__ csc_eid, int n, const float* __restrict__ Wh, int ld_wh,
    const float* __restrict__ T, int ld_t, const float* __restrict__ ds_dst,
    const float* __restrict__ a_src, const float* __restrict__ c_src,
    const float* __restrict__ a_dst, int H, int F, int HF, int concat, float slope,
    DropArgs drop_arg, float* __restrict__ dwh, int ld_dwh, float* __restrict__ part) {
    const DropArgs drop = resolve_drop(drop_arg);
    constexpr int CL = (U + G - 1) / G;
    const int lane = threadIdx.x & 63;
    const int c = lane & (G - 1);
    const int gbase = lane & ~(G - 1);
    const int groups = (gridDim.x * blockDim.x) / G;
    const int gid = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / G);
    const bool c_ok = 4 * c < HF;
    const int coff = c_ok ? 4 * c : 0;
    const int h = coff / F;
    const int hl = F / 4;
    const bool leader = c_ok && (coff % F) == 0;
    const int ldg = concat ? HF : F;
    const int toff = round_up4(ldg) + 4 * h;
    const int goff = concat ? coff : coff % F;
    const bool g_ok = c_ok && (concat || coff < F);
    const float gs = concat ? 1.f : 1.f / (float)H;
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
    const f32x4 a1 = c_ok ? *reinterpret_cast<const f32x4*>(a_src + coff) : zero4;
    const f32x4 a2 = c_ok ? *reinterpret_cast<const f32x4*>(a_dst + coff) : zero4;
    const float c1 = c_src[h];
    auto hsum = [&](float v) {
        if (hl <= 16) return group_sum16(v, hl);
        for (int off = 1; off < hl; off <<= 1) v += __shfl_xor(v, off);
        return v;
    };
    f32x4 pa1 = zero4, pa2 = zero4, pdb = zero4, pbias = zero4;
    float pc1 = 0.f, pc2 = 0.f;
    const bool use_drop = drop.thresh != 0u;
    for (int j = gid; j < n; j += groups) {
        const f32x4 w4 = c_ok ? *reinterpret_cast<const f32x4*>(Wh + (size_t)j * ld_wh + coff)
                              : zero4;
        const float ssrc = hsum(w4.x * a1.x + w4.y * a1.y + w4.z * a1.z + w4.w * a1.w) + c1;
        const int b0 = csc_ptr[j], b1 = csc_ptr[j + 1];
        f32x4 acc = zero4;
        float dss = 0.f;
        int iv[CL], kv[CL];
#pragma unroll
        for (int t = 0; t < CL; ++t) {
            const int bb = max(min(b0 + c + t * G, b1 - 1), 0);
            iv[t] = csc_dst[bb];
            kv[t] = use_drop ? csc_eid[bb] : 0;
        }
        for (int b = b0; b < b1; b += U) {
            const int nb = min(U, b1 - b);
            int in_[CL], kn[CL];
#pragma unroll
            for (int t = 0; t < CL; ++t) {
                const int bb = min(b + U + c + t * G, b1 - 1);
                in_[t] = csc_dst[bb];
                kn[t] = use_drop ? csc_eid[bb] : 0;
            }
            f32x4 gv[U], tv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = __shfl(iv[u / G], gbase + (u % G));
                const float* tr = T + (size_t)i * ld_t;
                gv[u] = g_ok || !concat ? *reinterpret_cast<const f32x4*>(tr + goff) : zero4;
                tv[u] = *reinterpret_cast<const f32x4*>(tr + toff);
            }
            float da[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                da[u] = hsum(gv[u].x * w4.x + gv[u].y * w4.y + gv[u].z * w4.z + gv[u].w * w4.w);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int kpos = __shfl(kv[u / G], gbase + (u % G));
                const float z = tv[u].x + ssrc;
                // (e - lse) <= 0: the hardware exp2 on a log2e-scaled argument, as
                // the forward's softmax (v_exp_f32; expf's range reduction costs
                // ~10 more VALU per edge and head)
                const float a = __builtin_amdgcn_exp2f((fmaxf(z, z * slope) - tv[u].y) * kLog2e);
                const float dm = use_drop ? drop_factor(drop, kpos, h, H) : 1.f;
                const float de = a * (dm * da[u] * gs - tv[u].z);
                const float dz = z > 0.f ? de : de * slope;
                const float w = u < nb ? a * dm : 0.f;
                acc += w * gv[u];
                dss += u < nb ? dz : 0.f;
            }
#pragma unroll
            for (int t = 0; t < CL; ++t) {
                iv[t] = in_[t];
                kv[t] = kn[t];
            }
        }
        const float dsd = ds_dst[(size_t)j * H + h];
        const f32x4 d = acc * gs + dss * a1 + dsd * a2;
        if (c_ok) *reinterpret_cast<f32x4*>(dwh + (size_t)j * ld_dwh + coff) = d;
        pa1 += dss * w4;
        pa2 += dsd * w4;
        pdb += c_ok ? d : zero4;
        if (g_ok) pbias += *reinterpret_cast<const f32x4*>(T + (size_t)j * ld_t + goff);
        if (leader) {
            pc1 += dss;
            pc2 += dsd;
        }
    }
    // combine the wave's 64/G groups (same columns in every group)
#pragma unroll
    for (int off = G; off < kWave; off <<= 1) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            pa1[q] += __shfl_xor(pa1[q], off);
            pa2[q] += __shfl_xor(pa2[q], off);
            pdb[q] += __shfl_xor(pdb[q], off);
            pbias[q] += __shfl_xor(pbias[q], off);
        }
        pc1 += __shfl_xor(pc1, off);
        pc2 += __shfl_xor(pc2, off);
    }
    if (lane >= G) return;
    const int wave = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave);
    float* pw = part + (size_t)wave * (3 * HF + 2 * H + ldg);
    if (c_ok) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            pw[coff + q] = pa1[q];
            pw[HF + coff + q] = pa2[q];
            pw[2 * HF + 2 * H + coff + q] = pdb[q];
        }
    }
    if (g_ok) {
#pragma unroll
        for (int q = 0; q < 4; ++q) pw[3 * HF + 2 * H + goff + q] = pbias[q];
    }
    if (leader) {
        pw[2 * HF + h] = pc1;
        pw[2 * HF + H + h] = pc2;
    }
}

// ---------------------------------------------------------------------------
// Backward, pass 2: one wave per SOURCE row j (CSC, grid-stride), lanes over
// the HF columns (CQ per lane).  Over j's out-edges (target i, slot c):
//   dWh[j]    = sum_c A[c,h] * dy[i]_h            (message backward)
//   ds_src[j] = sum_c dz[c]
// then the score terms s_src = Wh.a1 + c1, s_dst = Wh.a2 + c2 fold in:
//   dWh_total[j] = dWh[j] + ds_src[j,h] a1_h + ds_dst[j,h] a2_h
// and each wave accumulates its rows' contributions to da1/da2 (ds * Wh),
// dc1/dc2 (ds), db (= sum of dWh_total rows, the projection bias gradient)
// and dbias (= sum of grad_out rows) in registers, written once as per-wave
// partials part[w] = [da1 (HF) | da2 (HF) | dc1 (H) | dc2 (H) | db (HF) |
// dbias (ldg)] — summed by the caller; no float atomics, so the result is
// run-to-run deterministic.
// Algorithmic bytes per edge: 4 (csc_dst) + 4HF (g row, concat; 4F mean)
// + 8H (A, dz); per row: 4HF (Wh) + 4HF (dWh) + 8H.
// ---------------------------------------------------------------------------
template <int CQ, int HP>
__global__ __launch_bounds__(64) void k_src_bwd(
    const int* __restrict__ csc_ptr, const int* __restrict__ csc_dst, int n,
    const float* __restrict__ Wh, int ld_wh, const float* __restrict__ g,
    const float2* __restrict__ az, const float* __restrict__ ds_dst, const float* __restrict__ a1, const float* __restrict__ a2,
    int H, int F, int HF, int concat, float* __restrict__ dwh, int ld_dwh,
    float* __restrict__ ds_src, float* __restrict__ part) {
    __shared__ float dss_s[HP];
    const int lane = threadIdx.x;
    const int w = blockIdx.x;
    const int nw = gridDim.x;
    const float inv_h = 1.f / (float)H;
    int cc[CQ], hq[CQ], gq[CQ];
    bool okq[CQ];
    float a1v[CQ], a2v[CQ], pa1[CQ], pa2[CQ], pdb[CQ], pbias[CQ];
#pragma unroll
    for (int q = 0; q < CQ; ++q) {
        const int c = lane + kWave * q;
        okq[q] = c < HF;
        cc[q] = okq[q] ? c : 0;
        hq[q] = cc[q] / F;
        gq[q] = concat ? cc[q] : cc[q] - hq[q] * F;  // column of g feeding column c
        a1v[q] = okq[q] ? a1[cc[q]] : 0.f;
        a2v[q] = okq[q] ? a2[cc[q]] : 0.f;
        pa1[q] = 0.f;
        pa2[q] = 0.f;
        pdb[q] = 0.f;
        pbias[q] = 0.f;
    }
    const int ldg = concat ? HF : F;
    const float gs = concat ? 1.f : inv_h;
    const bool h_ok = lane < H;
    float pc1 = 0.f, pc2 = 0.f;
    constexpr int UE = 4;
    for (int j = w; j < n; j += nw) {
        const int b0 = csc_ptr[j], b1 = csc_ptr[j + 1];
        float acc[CQ];
#pragma unroll
        for (int q = 0; q < CQ; ++q) acc[q] = 0.f;
        float dss = 0.f;
        for (int b = b0; b < b1; b += UE) {
            int iu[UE], su[UE];
            float gate[UE];
#pragma unroll
            for (int u = 0; u < UE; ++u) {
                su[u] = min(b + u, b1 - 1);
                gate[u] = (b + u < b1) ? 1.f : 0.f;
                iu[u] = csc_dst[su[u]];
            }
            float gv[UE][CQ], av[UE][CQ], zv[UE];
#pragma unroll
            for (int u = 0; u < UE; ++u) {
#pragma unroll
                for (int q = 0; q < CQ; ++q) {
                    gv[u][q] = g[(size_t)iu[u] * ldg + gq[q]];
                    av[u][q] = az[(size_t)su[u] * H + hq[q]].x;
                }
                zv[u] = h_ok ? az[(size_t)su[u] * H + lane].y : 0.f;
            }
#pragma unroll
            for (int u = 0; u < UE; ++u) {
#pragma unroll
                for (int q = 0; q < CQ; ++q) acc[q] = fmaf(gate[u] * av[u][q], gv[u][q], acc[q]);
                dss = fmaf(gate[u], zv[u], dss);
            }
        }
        if (h_ok) {
            dss_s[lane] = dss;
            if (ds_src != nullptr) ds_src[(size_t)j * H + lane] = dss;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < CQ; ++q) {
            if (okq[q]) {
                const float hsrc = dss_s[hq[q]];
                const float hdst = ds_dst[(size_t)j * H + hq[q]];
                const float whv = Wh[(size_t)j * ld_wh + cc[q]];
                const float d = fmaf(hdst, a2v[q], fmaf(hsrc, a1v[q], acc[q] * gs));
                dwh[(size_t)j * ld_dwh + cc[q]] = d;
                pa1[q] = fmaf(hsrc, whv, pa1[q]);
                pa2[q] = fmaf(hdst, whv, pa2[q]);
                pdb[q] += d;
            }
            if (cc[q] < ldg && okq[q]) pbias[q] += g[(size_t)j * ldg + cc[q]];
        }
        if (h_ok) {
            pc1 += dss;
            pc2 += ds_dst[(size_t)j * H + lane];
        }
        __syncthreads();
    }
    float* pw = part + (size_t)w * (3 * HF + 2 * H + ldg);
#pragma unroll
    for (int q = 0; q < CQ; ++q) {
        if (okq[q]) {
            pw[cc[q]] = pa1[q];
            pw[HF + cc[q]] = pa2[q];
            pw[2 * HF + 2 * H + cc[q]] = pdb[q];
            if (cc[q] < ldg) pw[3 * HF + 2 * H + cc[q]] = pbias[q];
        }
    }
    if (h_ok) {
        pw[2 * HF + lane] = pc1;
        pw[2 * HF + H + lane] = pc2;
    }
}

// ---------------------------------------------------------------------------
// Weight gradient of the projection: dW[HF, Fin] = dWh^T x, a contraction
// over all N rows (K = N), which library GEMM heuristics handle poorly (one
// 165 us hipBLASLt call at PPI shape).  Split-K on fp32 MFMA 16x16x4: block
// (fin tile of 64, row chunk s, hf tile of 64); wave w owns hf rows
// [16w, 16w+16) of the tile and all four 16-wide fin sub-tiles, so per 4 rows
// a lane issues 1 dWh + 4 x loads and 4 MFMAs.  Operands come straight from
// global memory (each row is read by one block: no reuse for LDS to exploit).
// part[s] = the chunk's [HF, Fin] partial; k_wgrad_reduce sums the chunks in
// a fixed order (deterministic).
// Algorithmic bytes: 4 N (HF + Fin) reads + 4 S HF Fin partials.
// LW > 1: the four 16-column sub-tiles are interleaved so that a lane's four x
// values of a row are LW adjacent floats (sub-tile t, lane column ii holds
// fin column j0 + LW ii + (t % LW) + 16 LW (t / LW)): one float2 / float4 load
// instead of four scalar ones (the B columns of an MFMA may be any 16 columns;
// the store maps them back).  The kernel is bound by load instructions.
// ---------------------------------------------------------------------------
template <int LW>
__global__ __launch_bounds__(256) void k_wgrad(const float* __restrict__ dwh, int ld_dwh,
                                               const float* __restrict__ x, int n, int fin,
                                               int hf, int rows_per_chunk,
                                               float* __restrict__ part) {
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int j0 = blockIdx.x * 64;
    const int s = blockIdx.y;
    const int i0 = blockIdx.z * 64 + wv * 16;
    const int r0 = s * rows_per_chunk;
    const int r1 = min(n, r0 + rows_per_chunk);
    const int kk = lane >> 4, ii = lane & 15;
    const int icol = i0 + ii;
    const bool i_ok = icol < hf;
    const float amask = i_ok ? 1.f : 0.f;
    const int ic = i_ok ? icol : 0;
    // column of sub-tile t held by this lane
    auto jcol = [&](int t) {
        return LW == 1 ? j0 + 16 * t + ii : j0 + LW * ii + (t % LW) + 16 * LW * (t / LW);
    };
    constexpr int NLD = 4 / LW;  // x loads per row
    int jc[NLD];
#pragma unroll
    for (int q = 0; q < NLD; ++q) jc[q] = min(jcol(q * LW), fin - LW);  // in bounds; unused past fin
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int UR = 4;  // 4-row MFMA steps in flight
    for (int r = r0; r < r1; r += 4 * UR) {
        float av[UR], bv[UR][4];
#pragma unroll
        for (int u = 0; u < UR; ++u) {
            const int row = r + 4 * u + kk;
            const bool ok = row < r1;
            const int rr = ok ? row : r1 - 1;
            av[u] = dwh[(size_t)rr * ld_dwh + ic] * (ok ? amask : 0.f);
            const float* xr = x + (size_t)rr * fin;
#pragma unroll
            for (int q = 0; q < NLD; ++q) {
                if constexpr (LW == 4) {
                    const f32x4 v = *reinterpret_cast<const f32x4*>(xr + jc[q]);
                    bv[u][0] = v.x; bv[u][1] = v.y; bv[u][2] = v.z; bv[u][3] = v.w;
                } else if constexpr (LW == 2) {
                    const f32x2 v = *reinterpret_cast<const f32x2*>(xr + jc[q]);
                    bv[u][2 * q] = v.x; bv[u][2 * q + 1] = v.y;
                } else {
                    bv[u][q] = xr[jc[q]];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < UR; ++u)
#pragma unroll
            for (int t = 0; t < 4; ++t)
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u][t], acc[t], 0, 0, 0);
    }
    // C[i][j]: j = lane & 15, i = 4 * (lane >> 4) + q
    float* ps = part + (size_t)s * hf * fin;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int j = jcol(t);
        if (j >= fin) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = i0 + 4 * kk + q;
            if (i < hf) ps[(size_t)i * fin + j] = acc[t][q];
        }
    }
}

// out[b * width + e] = sum_c part[c * width + e] over rows c of row block
// b = blockIdx.y ([b * rows_per_block, ...) ∩ [0, rows)): 16 columns x 16 row
// groups per block, 4 independent loads in flight per thread, then a fixed
// order combine in LDS (deterministic).  Sums the per-chunk / per-wave
// partials of k_wgrad and k_src_bwd.
// ---------------------------------------------------------------------------
// Input gradient of the projection: dx[n, fin] = dWh[n, hf] W[hf, fin] (the x
// side of GAT.py:42-48's Linear layers; replaces the hipBLASLt GEMM).  fp32
// MFMA (v_mfma_f32_16x16x4_f32, exact fp32 products) with the operands swapped
// so the accumulator holds dx^T tiles: lane l ends with dx[row l&15][c + 4(l>>4)
// .. +4], four consecutive columns of one row.  The K = hf sum runs as KL
// k-steps per lane (lane kq owns k in [KL kq, KL kq + KL): every lane's dWh
// fragment is one contiguous run of its row, loaded once); W^T is staged per
// 64-column block in LDS (row stride KP + 1: conflict-free fragment reads).
// A workgroup owns 64 rows (one 16-row tile per wave) and walks all fin
// columns, so dWh is read once and W (hf x fin, L2-resident) once per
// workgroup.
// ---------------------------------------------------------------------------
template <int KL>
__global__ __launch_bounds__(256) void k_dx(const float* __restrict__ dwh, int ld_dwh, int hf,
                                            int n, const float* __restrict__ W, int fin,
                                            float* __restrict__ dx, int ld_dx) {
    constexpr int KP = 4 * KL, WS = KP + 1;
    __shared__ float wt[64 * WS];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int cl = lane & 15, kq = lane >> 4;
    const int row = blockIdx.x * 64 + w * 16 + cl;
    const int kb = KL * kq;
    float b[KL];
    {
        const float* src = dwh + (size_t)min(row, n - 1) * ld_dwh;
#pragma unroll
        for (int s = 0; s < KL; ++s) b[s] = kb + s < hf ? src[min(kb + s, hf - 1)] : 0.f;
    }
    const bool pair = (ld_dx % 2) == 0 && (reinterpret_cast<uintptr_t>(dx) & 7) == 0;
    for (int c0 = 0; c0 < fin; c0 += 64) {
        __syncthreads();  // the previous block's fragment reads are done
        for (int i = tid; i < 64 * KP; i += 256) {
            const int c = i & 63, k = i >> 6;  // a wave reads 64 consecutive columns of W row k
            wt[c * WS + k] = (k < hf && c0 + c < fin) ? W[(size_t)k * fin + c0 + c] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            if (c0 + 16 * t >= fin) break;  // block-uniform
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
            const float* a = wt + (16 * t + cl) * WS + kb;
#pragma unroll
            for (int s = 0; s < KL; ++s)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], acc, 0, 0, 0);
            const int col = c0 + 16 * t + 4 * kq;
            if (row < n) {
                float* d = dx + (size_t)row * ld_dx + col;
                if (col + 3 < fin && pair) {
                    *reinterpret_cast<f32x2*>(d) = f32x2{acc.x, acc.y};
                    *reinterpret_cast<f32x2*>(d + 2) = f32x2{acc.z, acc.w};
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (col + r < fin) d[r] = acc[r];
                }
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_colsum(const float* __restrict__ part, int rows,
                                                long long width, float* __restrict__ out,
                                                int rows_per_block) {
    __shared__ float red[16][17];
    const int col = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const long long e = blockIdx.x * 16LL + col;
    const long long ec = e < width ? e : width - 1;
    const int rb0 = blockIdx.y * rows_per_block;
    part += (size_t)rb0 * width;
    out += (size_t)blockIdx.y * width;
    rows = min(rows - rb0, rows_per_block);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int c = grp;
    for (; c + 48 < rows; c += 64) {
        s0 += part[(size_t)c * width + ec];
        s1 += part[(size_t)(c + 16) * width + ec];
        s2 += part[(size_t)(c + 32) * width + ec];
        s3 += part[(size_t)(c + 48) * width + ec];
    }
    for (; c < rows; c += 16) s0 += part[(size_t)c * width + ec];
    red[grp][col] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (grp == 0 && e < width) {
        float t = 0.f;
#pragma unroll
        for (int g = 0; g < 16; ++g) t += red[g][col];
        out[e] = t;
    }
}

int wgrad_chunks(int n, int fin, int hf) {
    const int ftiles = (fin + 63) / 64, htiles = (hf + 63) / 64;
    int by_rows = (n + 255) / 256;
    int by_fill = (2048 + ftiles * htiles - 1) / (ftiles * htiles);
    int c = by_rows < by_fill ? by_rows : by_fill;
    return c < 1 ? 1 : c;
}

// counter -> seed: splitmix64 of the counter value, then counter += 1
__global__ void k_seed_next(unsigned long long* __restrict__ counter,
                            unsigned long long* __restrict__ seed_out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const unsigned long long v = counter[0];
    counter[0] = v + 1ull;
    unsigned long long z = v + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    seed_out[0] = z ^ (z >> 31);
}

constexpr size_t kAlign = 256;
size_t align_up(size_t v) { return (v + kAlign - 1) / kAlign * kAlign; }

unsigned key_bits(int n) {
    unsigned b = 1;
    while (b < 31 && (1u << b) < (unsigned)n) ++b;
    return b;
}

size_t radix_tmp_bytes(long long E, int n) {
    size_t tmp = 0;
    unsigned* k = nullptr;
    int* v = nullptr;
    const hipError_t e = rocprim::radix_sort_pairs(nullptr, tmp, k, k, v, v, (size_t)E, 0u, key_bits(n));
    return e == hipSuccess ? tmp : 0;
}

size_t degree_sort_tmp_bytes(int n) {
    size_t tmp = 0;
    unsigned* k = nullptr;
    int* v = nullptr;
    const hipError_t e = rocprim::radix_sort_pairs_desc(nullptr, tmp, k, k, v, v,
                                                        (size_t)(n > 0 ? n : 1), 0u, 32u);
    return e == hipSuccess ? tmp : 0;
}

inline int grid_for(long long work, int block, int cap = 256 * 16) {
    long long g = (work + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

int status_of(hipError_t e) { return e == hipSuccess ? GAT_OK : (int)e; }

// Kernel-choice knobs for A/B measurement (tools/, tests; not part of the
// ABI).  The environment is read ONCE, at the first launch, into a snapshot;
// gat_tuning_reload() re-reads it (for the tools and tests that switch
// variants within one process).  The specialised kernels are the default
// wherever the shape allows them.
const char* const kKnobNames[] = {
    "GAT_PROJ_KERNEL", "GAT_PROJ_WK_MAX", "GAT_EDGE_LDS",  "GAT_EDGE_V",   "GAT_EDGE_U",
    "GAT_EDGE_PIPE",   "GAT_EDGE_SCORE",  "GAT_EDGE_KERNEL", "GAT_BWD_LDS", "GAT_BWD_U",
    "GAT_BWD_KERNEL",  "GAT_BWD_WAVES",   "GAT_HUB_SEG",     "GAT_PROJ_X3",
    "GAT_PROJ_BM",     "GAT_PROJ_WRES",   "GAT_PROJ_WRES_WGS", "GAT_BWD_KINK",
    "GAT_WGRAD_LW",    "GAT_STORE_WT",    "GAT_PROJ_WK_DIRECT", "GAT_EDGE_SPLIT"};
constexpr int kNumKnobs = (int)(sizeof(kKnobNames) / sizeof(kKnobNames[0]));

struct KnobSnapshot {
    bool set[kNumKnobs];
    char val[kNumKnobs][32];
};
KnobSnapshot g_knobs;
bool g_knobs_ready = false;

void snapshot_knobs() {
    for (int i = 0; i < kNumKnobs; ++i) {
        const char* v = std::getenv(kKnobNames[i]);
        g_knobs.set[i] = v != nullptr;
        g_knobs.val[i][0] = '\0';
        if (v != nullptr) {
            std::strncpy(g_knobs.val[i], v, sizeof(g_knobs.val[i]) - 1);
            g_knobs.val[i][sizeof(g_knobs.val[i]) - 1] = '\0';
        }
    }
    g_knobs_ready = true;
}

const char* knob(const char* name) {
    if (!g_knobs_ready) snapshot_knobs();
    for (int i = 0; i < kNumKnobs; ++i)
        if (std::strcmp(kKnobNames[i], name) == 0) return g_knobs.set[i] ? g_knobs.val[i] : nullptr;
    return nullptr;
}

// GAT_STORE_WT (A/B knob): 1 = final outputs stored write-through (sc1), 0 = plain
int store_wt_on() {
    const char* v = knob("GAT_STORE_WT");
    return v != nullptr ? (std::atoi(v) != 0) : 1;
}

bool kernel_choice(const char* env, const char* slow) {
    const char* v = knob(env);
    return !(v != nullptr && std::strcmp(v, slow) == 0);
}

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

int gat_abi_version(void) { return GAT_ABI_VERSION; }

int gat_tuning_reload(void) {
    snapshot_knobs();
    return GAT_OK;
}

int gat_table_layout(int heads, int f, int* ld, int* s_off) {
    if (heads <= 0 || f <= 0 || ld == nullptr || s_off == nullptr) return GAT_EINVAL;
    const int hf = heads * f;
    *s_off = round_up4(hf);
    *ld = *s_off + round_up4(heads);
    return GAT_OK;
}

// slices == 1: Wh row-major [n, ld_wh].  slices > 1: `slices` planes of
// [n, ld_wh = hf / slices] at wh + g * n * ld_wh (only the whole-K and the
// pipelined kernels write that layout).
static int project_impl(const float* x, int n, int fin, const float* w, const float* b,
                        const float* a_src, const float* c_src, const float* a_dst,
                        const float* c_dst, int heads, int f, int slices, float* wh, int ld_wh,
                        float* s_src, int ld_s, float* s_dst, void* stream, int n_table = 0) {
    if (n < 0 || fin < 0 || heads <= 0 || f <= 0 || slices <= 0) return GAT_EINVAL;
    const int hf = heads * f;
    if (hf > GAT_MAX_HF || heads > GAT_MAX_HEADS) return GAT_EUNSUPPORTED;
    const bool sliced = slices > 1;
    if (sliced) {
        if (hf % slices != 0 || ((hf / slices) & 3) || ld_wh != hf / slices || ld_s < heads)
            return GAT_EINVAL;
    } else if (ld_wh < round_up4(hf) || (ld_wh & 3) || ld_s < heads) {
        return GAT_EINVAL;
    }
    if (sliced && n_table < n) return GAT_EINVAL;
    if (n == 0) return GAT_OK;
    const int slice_w = sliced ? ld_wh : round_up4(hf);
    const long long slice_stride = sliced ? (long long)n_table * ld_wh : 0;
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((n + 63) / 64), block(256);
    const int nt = (hf + 15) / 16;
    const int store_wt = store_wt_on();  // Wh / scores stored write-through
    // GAT_PROJ_KERNEL (A/B knob, tools/tests): "wk" (whole K in LDS; the
    // default for fin <= 64), "pipe" (pipelined K loop; the default for larger
    // fin), "tiled" / "lds" (K-tiled fallback, shuffle / LDS epilogue)
    const char* pk = sliced ? nullptr : knob("GAT_PROJ_KERNEL");
    const bool pow2_f = next_pow2(f) == f;
    const size_t wk_lds = (size_t)wk_lds_floats(fin, nt) * sizeof(float);
    const bool aligned16 = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) |
                             reinterpret_cast<uintptr_t>(wh)) & 15) == 0;
    // W-resident kernel for 64 < fin <= 128 (k_project_wres: arxiv 44.4 -> 38.4 us
    // against k_project_x3; at PPI's fin 50 the whole-K fp32 k_project_wk stays
    // faster, 10.4 vs 12.5 us: 1.4 tiles per wave do not amortise the W split).
    // GAT_PROJ_WRES (A/B knob): 0 never, 1 for every fin <= 128.
    bool wres = fin > 64;
    if (const char* v = knob("GAT_PROJ_WRES")) wres = std::atoi(v) != 0;
    if (pk != nullptr && std::strcmp(pk, "wres") != 0) wres = false;
    if (wres && fin > 0 && fin <= 128 && (nt == 1 || nt == 2 || nt == 4) && pow2_f && f <= 16) {
        // x and W are both read LW floats at a time
        const uintptr_t xa = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w);
        const int lw = (fin % 4 == 0 && (xa & 15) == 0) ? 4 : (fin % 2 == 0 && (xa & 7) == 0) ? 2 : 1;
        const int ks = fin <= 32 ? 1 : fin <= 64 ? 2 : 4;
        const long long tiles = (n + 15) / 16;
        // persistent beyond the workgroups one CU holds at once (each wave loops
        // over tiles): 3 per CU for K <= 64 (45 KB of LDS, <= 168 VGPRs), else 2
        int wg_cu = ks <= 2 ? 3 : 2;
        if (const char* v = knob("GAT_PROJ_WRES_WGS")) wg_cu = std::max(1, std::atoi(v));
        const int grid_w = (int)std::min<long long>((tiles + 3) / 4, 256LL * wg_cu);
#define GAT_WRES(NTV, LWV, KSV)                                                               \
    hipLaunchKernelGGL((k_project_wres<NTV, LWV, KSV>), dim3(grid_w), dim3(256), 0, st, x, n, \
                       fin, w, b, a_src, c_src, a_dst, c_dst, heads, f, hf, wh, ld_wh, s_src,  \
                       ld_s, s_dst, slice_w, slice_stride, store_wt)
#define GAT_WRES_KS(NTV, LWV)                                          \
    switch (ks) {                                                      \
        case 1: GAT_WRES(NTV, LWV, 1); break;                          \
        case 2: GAT_WRES(NTV, LWV, 2); break;                          \
        default: GAT_WRES(NTV, LWV, 4); break;                         \
    }
#define GAT_WRES_LW(NTV)                                               \
    if (lw == 4) { GAT_WRES_KS(NTV, 4) }                               \
    else if (lw == 2) { GAT_WRES_KS(NTV, 2) }                          \
    else { GAT_WRES_KS(NTV, 1) }
        if (nt == 1) { GAT_WRES_LW(1) }
        else if (nt == 2) { GAT_WRES_LW(2) }
        else { GAT_WRES_LW(4) }
#undef GAT_WRES_LW
#undef GAT_WRES_KS
#undef GAT_WRES
        return status_of(hipGetLastError());
    }
    int wk_max = 64;  // GAT_PROJ_WK_MAX (A/B knob): largest fin for the whole-K kernel
    if (const char* v = knob("GAT_PROJ_WK_MAX")) wk_max = std::atoi(v);
    const bool wk_ok = fin > 0 && fin <= wk_max && aligned16 && wk_lds <= 160 * 1024 &&
                       (pk == nullptr || std::strcmp(pk, "wk") == 0);
    if (wk_ok) {
        // the direct epilogue for heads of 4, 8 or 16 columns (GAT_PROJ_WK_DIRECT=0:
        // the LDS output tile, A/B knob)
        bool direct = f == 4 || f == 8 || f == 16;
        if (const char* v = knob("GAT_PROJ_WK_DIRECT")) direct = direct && std::atoi(v) != 0;
#define GAT_WK_CASE(NT)                                                                       \
    case NT:                                                                                  \
        if (direct)                                                                           \
            hipLaunchKernelGGL((k_project_wk<NT, true>), grid, block, wk_lds, st, x, n, fin,  \
                               w, b, a_src, c_src, a_dst, c_dst, heads, f, hf, wh, ld_wh,     \
                               s_src, ld_s, s_dst, slice_w, slice_stride, store_wt);          \
        else                                                                                  \
            hipLaunchKernelGGL((k_project_wk<NT>), grid, block, wk_lds, st, x, n, fin, w, b,  \
                               a_src, c_src, a_dst, c_dst, heads, f, hf, wh, ld_wh, s_src,    \
                               ld_s, s_dst, slice_w, slice_stride, store_wt);                 \
        break;
        switch (nt) {
            GAT_WK_CASE(1) GAT_WK_CASE(2) GAT_WK_CASE(3) GAT_WK_CASE(4)
            GAT_WK_CASE(5) GAT_WK_CASE(6) GAT_WK_CASE(7) GAT_WK_CASE(8)
            GAT_WK_CASE(9) GAT_WK_CASE(10) GAT_WK_CASE(11) GAT_WK_CASE(12)
            GAT_WK_CASE(13) GAT_WK_CASE(14) GAT_WK_CASE(15) GAT_WK_CASE(16)
            default: return GAT_EUNSUPPORTED;
        }
#undef GAT_WK_CASE
        return status_of(hipGetLastError());
    }
    // pipelined K loop for large fin (F a power of two dividing 16, HF in
    // {16, 32, 64}, i.e. nt in {1, 2, 4}); LW floats per lane where fin allows
    const bool force_pipe = pk != nullptr && std::strcmp(pk, "pipe") == 0;
    const bool pipe_ok = (fin > 64 || force_pipe) && fin > 0 &&
                         (nt == 1 || nt == 2 || nt == 4) && pow2_f && f <= 16 &&
                         (long long)n * fin < (1LL << 31) && (pk == nullptr || force_pipe);
    if (pipe_ok) {
        const dim3 gp((n + 127) / 128), bp(256);
        const uintptr_t xa = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w);
        const int lw = (fin % 4 == 0 && (xa & 15) == 0) ? 4 : (fin % 2 == 0 && (xa & 7) == 0) ? 2 : 1;
        // split-bf16 matrix cores (k_project_x3) unless GAT_PROJ_X3=0 (A/B knob:
        // the fp32-MFMA k_project_pipe2)
        bool x3 = true;
#ifdef GAT_AB_KERNELS
        if (const char* v = knob("GAT_PROJ_X3")) x3 = std::atoi(v) != 0;
#endif
        // rows per block (GAT_PROJ_BM A/B knob: 64 = one 16-row group per wave,
        // 128 = two, sharing every B fragment)
        // tools/proj_ab.py: 4-float x rows (arxiv) prefer 64 rows per block with two
        // chunks in flight, 2-float rows (Reddit's 602) 128 rows sharing B
        // fragments with one chunk in flight
        int bm = lw == 4 ? 64 : 128;
        if (const char* v = knob("GAT_PROJ_BM")) bm = std::atoi(v);
#ifdef GAT_AB_KERNELS
#define GAT_PIPE2_FP32(NT, LWV)                                                                \
        hipLaunchKernelGGL((k_project_pipe2<NT, LWV>), gp, bp, 0, st, x, n, fin, w, b, a_src, \
                           c_src, a_dst, c_dst, heads, f, hf, wh, ld_wh, s_src, ld_s, s_dst,  \
                           slice_w, slice_stride)
#else
#define GAT_PIPE2_FP32(NT, LWV) (void)gp
#endif
#define GAT_PIPE2(NT, LWV)                                                                     \
    if (x3 && bm == 128)                                                                       \
        hipLaunchKernelGGL((k_project_x3<NT, LWV, 2, 1>), dim3((n + 127) / 128), bp, 0, st,    \
                           x, n, fin, w, b, a_src, c_src, a_dst, c_dst, heads, f, hf, wh,     \
                           ld_wh, s_src, ld_s, s_dst, slice_w, slice_stride, store_wt);       \
    else if (x3)                                                                               \
        hipLaunchKernelGGL((k_project_x3<NT, LWV, 1, 2>), dim3((n + 63) / 64), bp, 0, st, x, n, \
                           fin, w, b, a_src,                                                  \
                           c_src, a_dst, c_dst, heads, f, hf, wh, ld_wh, s_src, ld_s, s_dst,  \
                           slice_w, slice_stride, store_wt);                                  \
    else                                                                                       \
        GAT_PIPE2_FP32(NT, LWV)
#define GAT_PIPE2_LW(NT)                                  \
    if (lw == 4) { GAT_PIPE2(NT, 4); }                    \
    else if (lw == 2) { GAT_PIPE2(NT, 2); }               \
    else { GAT_PIPE2(NT, 1); }
        if (nt == 1) { GAT_PIPE2_LW(1) }
        else if (nt == 2) { GAT_PIPE2_LW(2) }
        else { GAT_PIPE2_LW(4) }
#undef GAT_PIPE2_LW
#undef GAT_PIPE2
#undef GAT_PIPE2_FP32
        return status_of(hipGetLastError());
    }
    if (sliced) return GAT_EUNSUPPORTED;  // the kernels below write row-major Wh only
    const bool shfl = ((f <= 16 && 16 % f == 0) || (f % 16 == 0)) &&
                      !(pk != nullptr && std::strcmp(pk, "lds") == 0);
#define GAT_PROJ_CASE(NT)                                                                   \
    case NT:                                                                                \
        if (shfl)                                                                           \
            hipLaunchKernelGGL((k_project<NT, true>), grid, block, 0, st, x, n, fin, w, b,   \
                               a_src, c_src, a_dst, c_dst, heads, f, hf, wh, ld_wh, s_src,  \
                               ld_s, s_dst);                                                \
        else                                                                                \
            hipLaunchKernelGGL((k_project<NT, false>), grid, block, 0, st, x, n, fin, w, b,  \
                               a_src, c_src, a_dst, c_dst, heads, f, hf, wh, ld_wh, s_src,  \
                               ld_s, s_dst);                                                \
        break;
    switch (nt) {
        GAT_PROJ_CASE(1) GAT_PROJ_CASE(2) GAT_PROJ_CASE(3) GAT_PROJ_CASE(4)
        GAT_PROJ_CASE(5) GAT_PROJ_CASE(6) GAT_PROJ_CASE(7) GAT_PROJ_CASE(8)
        GAT_PROJ_CASE(9) GAT_PROJ_CASE(10) GAT_PROJ_CASE(11) GAT_PROJ_CASE(12)
        GAT_PROJ_CASE(13) GAT_PROJ_CASE(14) GAT_PROJ_CASE(15) GAT_PROJ_CASE(16)
        default: return GAT_EUNSUPPORTED;
    }
#undef GAT_PROJ_CASE
    return status_of(hipGetLastError());
}

int gat_project(const float* x, int n, int fin, const float* w, const float* b,
                const float* a_src, const float* c_src, const float* a_dst, const float* c_dst,
                int heads, int f, float* wh, int ld_wh, float* s_src, int ld_s, float* s_dst,
                void* stream) {
    return project_impl(x, n, fin, w, b, a_src, c_src, a_dst, c_dst, heads, f, 1, wh, ld_wh,
                        s_src, ld_s, s_dst, stream);
}

int gat_project_sliced(const float* x, int n, int fin, const float* w, const float* b,
                       const float* a_src, const float* c_src, const float* a_dst,
                       const float* c_dst, int heads, int f, int slices, float* wh, int n_table,
                       float* s_src, int ld_s, float* s_dst, void* stream) {
    if (slices <= 0 || heads <= 0 || f <= 0 || (heads * f) % slices != 0) return GAT_EINVAL;
    if (s_src == nullptr) ld_s = heads;  // the sliced edge kernel recomputes s_src
    return project_impl(x, n, fin, w, b, a_src, c_src, a_dst, c_dst, heads, f, slices, wh,
                        heads * f / slices, s_src, ld_s, s_dst, stream, n_table);
}

}  // extern "C"

// Fused lane-group edge kernel, optionally with the gathers pipelined one
// chunk ahead (GAT_EDGE_PIPE A/B knob): instantiated for the (U, V) pairs the
// default schedule uses.
template <int G, int U, int V, bool KINK = false, class... A>
static void launch_edge_fused(int pipe, int split, dim3 grid, dim3 block, hipStream_t st,
                              A... a) {
    // GAT_EDGE_LDS (A/B knob): dynamic LDS bytes per block, unused by the
    // kernel — caps the blocks resident per CU (160 KB / bytes)
    size_t lds = 0;
    if (const char* el = knob("GAT_EDGE_LDS")) lds = (size_t)std::atol(el);
    // the pipelined form is instantiated for the pair the default schedule
    // pipelines (U = 16, V = 2: Reddit-scale rows); elsewhere the knob is ignored
    if constexpr (V == 2 && U == 16) {
        if (pipe) {
            hipLaunchKernelGGL((k_edge_grp<G, U, V, true, true, KINK>), grid, block, lds, st, a...);
            return;
        }
    }
    // two lane groups per row (S = 2, GAT_EDGE_SPLIT): instantiated for the
    // short-row lane groups of HF = 64 (G = 8: 2-plane table; G = 16: row-major)
    if constexpr (!KINK && V == 1 && U <= 8 && (G == 8 || G == 16)) {
        if (split == 2) {
            hipLaunchKernelGGL((k_edge_grp<G, U, V, true, false, false, 2>),
                               dim3(grid.x * 2), block, lds, st, a...);
            return;
        }
    }
    hipLaunchKernelGGL((k_edge_grp<G, U, V, true, false, KINK>), grid, block, lds, st, a...);
}

// the kink-sum forward is instantiated for the lane groups of HF = 64 heads
// (G = 16 at V = 1, G = 8 at V = 2); kink_grp_ok says which launch it serves
static bool kink_grp_ok(int g, int v) { return (g == 16 && v == 1) || (g == 8 && v == 2); }

template <int G, int U, int V, class... A>
static void launch_edge_kink(int pipe, dim3 grid, dim3 block, hipStream_t st, A... a) {
    if constexpr ((G == 16 && V == 1) || (G == 8 && V == 2))
        launch_edge_fused<G, U, V, true>(pipe, 1, grid, block, st, a...);
}

extern "C" {

static int edge_aggregate_impl(const EdgeRows er, const int* col, const int* row_order,
                               int row_begin, int row_end, const float* wh, int ld_wh,
                               const float* s_src, int ld_s, const float* a_src,
                               const float* c_src, const float* s_dst, int heads, int f,
                               int concat, int act, float negative_slope, const float* bias,
                               float* out, float* lse, float* y_heads, DropArgs drop,
                               int edges_per_row_hint, void* stream, int nslices = 1,
                               long long slice_stride = 0, float* q_heads = nullptr,
                               float* r_heads = nullptr) {
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
    const int store_wt = (lse == nullptr && q_heads == nullptr) ? store_wt_on() : 0;
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
    edges_per_row_hint &= ~GAT_HINT_LOCAL;
    int vv = edges_per_row_hint >= 128 ? 2 : 1;
    if (local_hint && !sliced && round_up4(hf) <= 32) vv = 2;
    if (const char* ev = knob("GAT_EDGE_V")) vv = std::atoi(ev) >= 2 ? 2 : 1;

    while (vv > 1 && f % (4 * vv) != 0) vv >>= 1;
    const int hl = f / (4 * vv);  // lanes per head
    const bool pow2_hl = (f % (4 * vv) == 0) && next_pow2(hl) == hl;
    const int gcols = sliced ? slice_w : hf;  // columns one lane group owns
    const int g = next_pow2((gcols + 4 * vv - 1) / (4 * vv));
    const bool grp_ok = (f % 4 == 0) && (concat || pow2_hl) && slope_ok;
    // fused source score: the head's lanes must form an aligned power-of-two block
    bool fused = grp_ok && pow2_hl && have_a;
    if (fused && s_src != nullptr) fused = kernel_choice("GAT_EDGE_SCORE", "gather");
    if (s_src == nullptr && !fused) return GAT_EUNSUPPORTED;
    const bool kink = q_heads != nullptr;
    if (kink && (!fused || sliced || r_heads == nullptr || lse == nullptr || y_heads == nullptr ||
                 er.by_pos || er.load || er.store_lt > 0))
        return GAT_EUNSUPPORTED;
    // a slice holds whole heads (the fused score sums a head inside one group)
    if (sliced && (!fused || slice_w % f != 0)) return GAT_EUNSUPPORTED;
    if (grp_ok && (s_src == nullptr || kernel_choice("GAT_EDGE_KERNEL", "generic"))) {
        // edges per chunk: short rows want short chunks (less padding), long rows
        // more loads in flight; GAT_EDGE_U overrides
        // (tools/tune_edge.py: PPI, ~28 per row, 36.9 us at U = 8 -> 33.1 us at U = 4)
        int u = edges_per_row_hint <= 0 ? 8 : edges_per_row_hint <= 32 ? 4
              : edges_per_row_hint <= 64 ? 8 : 16;
        if (const char* eu = knob("GAT_EDGE_U")) u = std::atoi(eu);
        const long long threads = (long long)rows * g;
        const long long blocks = ((threads + 255) / 256) * nslices;
        if (blocks >= (1LL << 31)) return GAT_EUNSUPPORTED;
        const dim3 grid((unsigned)blocks), block(256);
        // gathers pipelined one chunk ahead for long rows (U = 16, V = 2: one
        // wave per SIMD at 360 registers, but 64 row gathers in flight per
        // lane; tools/slice_probe.py, Reddit scale 2.60 -> 1.99 ms); shorter
        // rows keep more, shallower waves (PPI 30.5 -> 32.9 us pipelined)
        int pipe = (u == 16 && vv == 2) ? 1 : 0;
        if (const char* ep = knob("GAT_EDGE_PIPE")) pipe = std::atoi(ep);
        // two lane groups per row (the grid doubles inside launch_edge_fused):
        // GAT_EDGE_SPLIT = 2 (A/B knob); rows that run segment passes (er.load /
        // store_lt) and the kink-sum forward keep one group
        // Default: launches of fewer than ~4 waves per SIMD (a rank's share of a
        // small graph: PPI at P = 4 / 8 edge passes 14.4 -> 11.3 / 13.4 -> 9.4 us,
        // tools/emu_probe.py) — there the per-row chain of dependent chunk loads
        // is exposed; larger launches hide it and the split only adds work (full
        // PPI 27.8 -> 30.8 us, arxiv 54.2 -> 61.2 us).
        const long long waves = (long long)rows * g * nslices / kWave;
        int split = waves < 4096 ? 2 : 1;
        if (const char* es = knob("GAT_EDGE_SPLIT")) split = std::atoi(es) == 2 ? 2 : 1;
        if (kink || pipe) split = 1;
        if ((long long)blocks * split >= (1LL << 31)) split = 1;
        if (kink && !kink_grp_ok(g, vv)) return GAT_EUNSUPPORTED;
#define GAT_GRP_KARGS                                                                         \
    er, col, row_order, row_begin, row_end, wh, ld_wh, s_src, ld_s, a_src, c_src, s_dst,   \
        heads, f, hf, concat, negative_slope, bias, out, ld_out, lse, drop, y_heads, nslices,  \
        slice_w, slice_stride, q_heads, r_heads, store_wt
#define GAT_GRP_LAUNCH(G, UU, VV)                                                     \
    if (kink)                                                                         \
        launch_edge_kink<G, UU, VV>(pipe, grid, block, st, GAT_GRP_KARGS);             \
    else if (fused)                                                                   \
        launch_edge_fused<G, UU, VV>(pipe, split, grid, block, st, GAT_GRP_KARGS);     \
    else                                                                              \
        hipLaunchKernelGGL((k_edge_grp<G, UU, VV, false>), grid, block, 0, st, GAT_GRP_KARGS)
#define GAT_GRP_U(G, VV)                                                              \
    if (u == 4) { GAT_GRP_LAUNCH(G, 4, VV); }                                         \
    else if (u == 16) { GAT_GRP_LAUNCH(G, 16, VV); }                                  \
    else { GAT_GRP_LAUNCH(G, 8, VV); }
#define GAT_GRP_G32(VV)                               \
        case 1: GAT_GRP_U(1, VV) break;               \
        case 2: GAT_GRP_U(2, VV) break;               \
        case 4: GAT_GRP_U(4, VV) break;               \
        case 8: GAT_GRP_U(8, VV) break;               \
        case 16: GAT_GRP_U(16, VV) break;             \
        case 32: GAT_GRP_U(32, VV) break;
        // V = 2 owns <= 256 / 8 = 32 lanes per row: no G = 64 instance
        if (vv == 2) {
            switch (g) {
                GAT_GRP_G32(2)
                default: return GAT_EUNSUPPORTED;
            }
        } else {
            switch (g) {
                GAT_GRP_G32(1)
                case 64: GAT_GRP_U(64, 1) break;
                default: return GAT_EUNSUPPORTED;
            }
        }
#undef GAT_GRP_G32
#undef GAT_GRP_U
#undef GAT_GRP_LAUNCH
#undef GAT_GRP_KARGS
        return status_of(hipGetLastError());
    }
    // the generic kernel runs whole CSR rows only
    if (kink) return GAT_EUNSUPPORTED;
    if (er.by_pos || er.load || er.store_lt > 0 || er.ee != er.eb + 1) return GAT_EUNSUPPORTED;
    const int* rowptr = er.eb;
    const int lpe = next_pow2((round_up4(hf) + 3) / 4);
    const int hp = next_pow2(heads);
    const dim3 grid(rows), block(kWave);
#define GAT_EDGE_LAUNCH(L, P)                                                                \
    hipLaunchKernelGGL((k_edge_fwd<L, P>), grid, block, 0, st, rowptr, col, row_order,       \
                       row_begin,                                                            \
                       row_end, wh, ld_wh, s_src, ld_s, s_dst, heads, f, hf, concat, act,    \
                       negative_slope, bias, out, ld_out, lse, drop, y_heads)
#define GAT_EDGE_HP(L)                                                                       \
    switch (hp) {                                                                            \
        case 1: GAT_EDGE_LAUNCH(L, 1); break;                                                \
        case 2: GAT_EDGE_LAUNCH(L, 2); break;                                                \
        case 4: GAT_EDGE_LAUNCH(L, 4); break;                                                \
        case 8: GAT_EDGE_LAUNCH(L, 8); break;                                                \
        case 16: GAT_EDGE_LAUNCH(L, 16); break;                                              \
        case 32: GAT_EDGE_LAUNCH(L, 32); break;                                              \
        case 64: GAT_EDGE_LAUNCH(L, 64); break;                                              \
        default: return GAT_EUNSUPPORTED;                                                    \
    }
    switch (lpe) {
        case 1: GAT_EDGE_HP(1) break;
        case 2: GAT_EDGE_HP(2) break;
        case 4: GAT_EDGE_HP(4) break;
        case 8: GAT_EDGE_HP(8) break;
        case 16: GAT_EDGE_HP(16) break;
        case 32: GAT_EDGE_HP(32) break;
        case 64: GAT_EDGE_HP(64) break;
        default: return GAT_EUNSUPPORTED;
    }
#undef GAT_EDGE_HP
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
    if (heads <= 0 || f <= 0 || n_hub < 0) return GAT_EINVAL;
    const int hf = heads * f;
    if (hf > GAT_MAX_HF || heads > GAT_MAX_HEADS) return GAT_EUNSUPPORTED;
    if (n_hub == 0) return GAT_OK;
    if (hub_rows == nullptr || seg_ptr == nullptr || st_acc == nullptr || st_ml == nullptr ||
        bias == nullptr || out == nullptr)
        return GAT_EINVAL;
    hipLaunchKernelGGL(k_edge_merge, dim3(n_hub), dim3(kWave), 0, (hipStream_t)stream, hub_rows,
                       seg_ptr, n_hub, st_acc, round_up4(hf), st_ml, heads, f, hf, concat, bias,
                       out, concat ? hf : f, lse, y_heads);
    return status_of(hipGetLastError());
}

size_t csr_key_sort_tmp_bytes(long long nnz, int n) {
    size_t tmp = 0;
    unsigned long long* k = nullptr;
    const unsigned kb = key_bits(n);
    const hipError_t e = rocprim::radix_sort_keys(nullptr, tmp, k, k, (size_t)nnz, 0u, 2 * kb);
    return e == hipSuccess ? tmp : 0;
}

int gat_dropout_seed_next(unsigned long long* counter, unsigned long long* seed_out,
                          void* stream) {
    if (counter == nullptr || seed_out == nullptr) return GAT_EINVAL;
    hipLaunchKernelGGL(k_seed_next, dim3(1), dim3(64), 0, (hipStream_t)stream, counter, seed_out);
    return status_of(hipGetLastError());
}

int gat_csr_workspace_size(long long num_edges, int num_nodes, size_t* bytes) {
    if (num_edges < 0 || num_nodes < 0 || bytes == nullptr) return GAT_EINVAL;
    if (num_edges + num_nodes > 0x7fffffffLL) return GAT_EUNSUPPORTED;
    long long nnz = num_edges + num_nodes;
    if (nnz < 1) nnz = 1;
    const size_t t1 = csr_key_sort_tmp_bytes(nnz, num_nodes > 0 ? num_nodes : 1);
    const size_t t2 = degree_sort_tmp_bytes(num_nodes);
    const size_t kb = align_up((size_t)nnz * 8);
    const size_t nb = align_up((size_t)(num_nodes > 0 ? num_nodes : 1) * 4);
    const size_t a = 2 * kb;                       // keys in / out
    const size_t b = 4 * nb;                       // degree-sort buffers
    *bytes = (a > b ? a : b) + align_up(t1 > t2 ? t1 : t2);
    return GAT_OK;
}

int gat_csr_build(const long long* edge_index, long long num_edges, int num_nodes, int* rowptr,
                  int* col, int* row_order, void* workspace, size_t workspace_bytes,
                  int* error_flag, void* stream) {
    if (num_edges < 0 || num_nodes < 0 || error_flag == nullptr) return GAT_EINVAL;
    size_t need = 0;
    int rc = gat_csr_workspace_size(num_edges, num_nodes, &need);
    if (rc != GAT_OK) return rc;
    if (workspace_bytes < need) return GAT_EWORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(error_flag, 0, sizeof(int), st);
    if (e != hipSuccess) return status_of(e);
    if (num_nodes == 0) {
        if (num_edges > 0) {
            // every edge is out of range when there are no nodes
            e = hipMemsetAsync(error_flag, 0x01, 1, st);
            if (e != hipSuccess) return status_of(e);
        }
        return status_of(hipMemsetAsync(rowptr, 0, sizeof(int), st));
    }
    const long long nnz = num_edges + num_nodes;
    const unsigned kb = key_bits(num_nodes);
    const size_t keyb = align_up((size_t)nnz * 8);
    const size_t nb = align_up((size_t)num_nodes * 4);
    const size_t region = 2 * keyb > 4 * nb ? 2 * keyb : 4 * nb;
    char* ws = (char*)workspace;
    unsigned long long* keys_in = (unsigned long long*)ws;
    unsigned long long* keys_out = (unsigned long long*)(ws + keyb);
    void* tmp = ws + region;
    size_t tmp_bytes = need - region;
    hipLaunchKernelGGL(k_csr_prepare, dim3(grid_for(nnz, 256)), dim3(256), 0, st, edge_index,
                       num_edges, num_nodes, kb, keys_in, error_flag);
    e = rocprim::radix_sort_keys(tmp, tmp_bytes, keys_in, keys_out, (size_t)nnz, 0u, 2 * kb, st);
    if (e != hipSuccess) return status_of(e);
    hipLaunchKernelGGL(k_csr_rowptr, dim3((num_nodes + 1 + 255) / 256), dim3(256), 0, st,
                       keys_out, nnz, num_nodes, kb, rowptr);
    hipLaunchKernelGGL(k_csr_col, dim3(grid_for(nnz, 256)), dim3(256), 0, st, keys_out, nnz, kb,
                       col);
    if (row_order != nullptr) {
        // rows by descending in-degree (stable): the edge kernel's schedule
        unsigned* dkeys_in = (unsigned*)ws;
        int* dvals_in = (int*)(ws + nb);
        unsigned* dkeys_out = (unsigned*)(ws + 2 * nb);
        hipLaunchKernelGGL(k_degree_keys, dim3(grid_for(num_nodes, 256)), dim3(256), 0, st,
                           rowptr, num_nodes, dkeys_in, dvals_in);
        tmp_bytes = need - region;
        e = rocprim::radix_sort_pairs_desc(tmp, tmp_bytes, dkeys_in, dkeys_out, dvals_in,
                                           row_order, (size_t)num_nodes, 0u, 32u, st);
        if (e != hipSuccess) return status_of(e);
    }
    return status_of(hipGetLastError());
}

int gat_csc_workspace_size(long long nnz, int num_nodes, size_t* bytes) {
    if (nnz < 0 || num_nodes < 0 || bytes == nullptr) return GAT_EINVAL;
    if (nnz > 0x7fffffffLL) return GAT_EUNSUPPORTED;
    const size_t eb = align_up((size_t)(nnz > 0 ? nnz : 1) * 4);
    *bytes = 4 * eb + align_up(radix_tmp_bytes(nnz, num_nodes > 0 ? num_nodes : 1));
    return GAT_OK;
}

int gat_csc_build(const int* rowptr, const int* col, int num_nodes, long long nnz, int* csc_ptr,
                  int* csc_dst, int* csc_eid, int* csr_to_csc, void* workspace,
                  size_t workspace_bytes, void* stream) {
    if (num_nodes < 0 || nnz < 0) return GAT_EINVAL;
    size_t need = 0;
    int rc = gat_csc_workspace_size(nnz, num_nodes, &need);
    if (rc != GAT_OK) return rc;
    if (workspace_bytes < need) return GAT_EWORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    if (num_nodes == 0) return GAT_OK;
    if (nnz == 0) return status_of(hipMemsetAsync(csc_ptr, 0, sizeof(int) * (num_nodes + 1), st));
    const size_t eb = align_up((size_t)nnz * 4);
    char* ws = (char*)workspace;
    unsigned* keys_in = (unsigned*)ws;
    int* vals_in = (int*)(ws + eb);
    unsigned* keys_out = (unsigned*)(ws + 2 * eb);
    int* vals_out = csc_eid != nullptr ? csc_eid : (int*)(ws + 3 * eb);
    void* tmp = ws + 4 * eb;
    hipLaunchKernelGGL(k_csc_keys, dim3(grid_for(nnz, 256)), dim3(256), 0, st, nnz, col, keys_in,
                       vals_in);
    size_t tmp_bytes = need - 4 * eb;
    hipError_t e = rocprim::radix_sort_pairs(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out,
                                             (size_t)nnz, 0u, key_bits(num_nodes), st);
    if (e != hipSuccess) return status_of(e);
    hipLaunchKernelGGL(k_csc_ptr, dim3((num_nodes + 1 + 255) / 256), dim3(256), 0, st, keys_out,
                       nnz, num_nodes, csc_ptr);
    hipLaunchKernelGGL(k_csc_fill, dim3(grid_for(nnz, 256)), dim3(256), 0, st, vals_out, rowptr,
                       num_nodes, nnz, csc_dst, csr_to_csc);
    return status_of(hipGetLastError());
}

int gat_bwd_table_layout(int heads, int f, int concat, int* ld_t) {
    if (heads <= 0 || f <= 0 || ld_t == nullptr) return GAT_EINVAL;
    *ld_t = round_up4(concat ? heads * f : f) + 4 * heads;
    return GAT_OK;
}

// edges per chunk of the recompute backward kernels: the forward's thresholds;
// GAT_BWD_U overrides (A/B knob)
// GAT_BWD_LDS (A/B knob): dynamic LDS bytes per block for the recompute
// backward kernels, unused by them — caps the blocks resident per CU
static size_t bwd_lds_bytes() {
    const char* v = knob("GAT_BWD_LDS");
    return v != nullptr ? (size_t)std::atol(v) : 0;
}

static int bwd_unroll(int hint) {
    hint &= ~GAT_HINT_LOCAL;
    int u = hint <= 0 ? 8 : hint <= 32 ? 4 : hint <= 64 ? 8 : 16;
    if (const char* v = knob("GAT_BWD_U")) {
        const int x = std::atoi(v);
        u = (x == 4 || x == 16) ? x : 8;
    }
    return u;
}

static bool bwd_recompute_ok(int heads, int f, float slope, const float* wh, int ld_wh) {
    // GAT_BWD_KERNEL=stored|generic (A/B knob): force the stored-coefficient path
    if (const char* v = knob("GAT_BWD_KERNEL"))
        if (std::strcmp(v, "stored") == 0 || std::strcmp(v, "generic") == 0) return false;
    const int hl = f / 4;
    return heads * f <= GAT_MAX_HF && heads <= GAT_MAX_HEADS && f % 4 == 0 &&
           next_pow2(hl) == hl && slope >= 0.f && slope <= 1.f && (ld_wh & 3) == 0 &&
           (reinterpret_cast<uintptr_t>(wh) & 15) == 0;
}

int gat_bwd_targets(const int* rowptr, const int* col, const int* row_order, int row_begin,
                    int row_end, const float* wh, int ld_wh, const float* a_src,
                    const float* c_src, const float* s_dst, const float* lse,
                    const float* y_heads, const float* grad_out, int heads, int f, int concat,
                    float negative_slope, float dropout_p, unsigned long long seed,
                    const unsigned long long* seed_dev, float* ds_dst, float* table, int ld_t,
                    int edges_per_row_hint, void* stream) {
    if (heads <= 0 || f <= 0 || row_begin < 0 || row_end < row_begin) return GAT_EINVAL;
    if (!(dropout_p >= 0.f && dropout_p <= 1.f)) return GAT_EINVAL;
    int need_ld = 0;
    gat_bwd_table_layout(heads, f, concat, &need_ld);
    if (ld_t < need_ld || (ld_t & 3)) return GAT_EINVAL;
    if (!bwd_recompute_ok(heads, f, negative_slope, wh, ld_wh)) return GAT_EUNSUPPORTED;
    const int rows = row_end - row_begin;
    if (rows == 0) return GAT_OK;
    hipStream_t st = (hipStream_t)stream;
    const DropArgs drop = make_drop(dropout_p, seed, seed_dev);
    const int hf = heads * f;
    const int g = next_pow2(hf / 4);
    int u = bwd_unroll(edges_per_row_hint);
    const long long threads = (long long)rows * g;
    const dim3 grid((unsigned)((threads + 255) / 256)), block(256);
    const size_t bwd_lds = bwd_lds_bytes();
#define GAT_BT(G, UU)                                                                         \
    hipLaunchKernelGGL((k_bwd_targets<G, UU>), grid, block, bwd_lds, st, rowptr, col, row_order,    \
                       row_begin, row_end, wh, ld_wh, a_src, c_src, s_dst, lse, y_heads,      \
                       grad_out, heads, f, hf, concat, negative_slope, drop, ds_dst, table,   \
                       ld_t)
#define GAT_BT_U(G)                      \
    case G:                              \
        if (u == 4) { GAT_BT(G, 4); }    \
        else if (u == 16) { GAT_BT(G, 16); } \
        else { GAT_BT(G, 8); }           \
        break;
    switch (g) {
        GAT_BT_U(1) GAT_BT_U(2) GAT_BT_U(4) GAT_BT_U(8) GAT_BT_U(16) GAT_BT_U(32) GAT_BT_U(64)
        default: return GAT_EUNSUPPORTED;
    }
#undef GAT_BT_U
#undef GAT_BT
    return status_of(hipGetLastError());
}

int gat_bwd_table(const float* s_dst, const float* lse, const float* y_heads,
                  const float* q_heads, const float* r_heads, const float* grad_out,
                  int num_nodes, int heads, int f, int concat, float* ds_dst, float* table,
                  int ld_t, void* stream) {
    if (num_nodes < 0 || heads <= 0 || f <= 0) return GAT_EINVAL;
    if (num_nodes > 0 && (s_dst == nullptr || lse == nullptr || y_heads == nullptr || q_heads == nullptr ||
        r_heads == nullptr || grad_out == nullptr || ds_dst == nullptr || table == nullptr))
        return GAT_EINVAL;
    int need_ld = 0;
    gat_bwd_table_layout(heads, f, concat, &need_ld);
    if (ld_t < need_ld || (ld_t & 3)) return GAT_EINVAL;
    const int hf = heads * f;
    const int hl = f / 4;
    if (hf > GAT_MAX_HF || heads > GAT_MAX_HEADS || f % 4 != 0 || next_pow2(hl) != hl)
        return GAT_EUNSUPPORTED;
    // GAT_BWD_KERNEL=stored|generic forces the stored-coefficient backward, as
    // gat_bwd_targets honours it
    if (const char* v = knob("GAT_BWD_KERNEL"))
        if (std::strcmp(v, "stored") == 0 || std::strcmp(v, "generic") == 0) return GAT_EUNSUPPORTED;
    if (num_nodes == 0) return GAT_OK;
    const int g = next_pow2(hf / 4);
    const long long threads = (long long)num_nodes * g;
    hipLaunchKernelGGL(k_bwd_table, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, num_nodes, g, s_dst, lse, y_heads, q_heads, r_heads,
                       grad_out, heads, f, hf, concat, ds_dst, table, ld_t);
    return status_of(hipGetLastError());
}

int gat_bwd_sources_parts(int num_nodes, int heads, int f, int* num_parts) {
    if (num_nodes < 0 || heads <= 0 || f <= 0 || num_parts == nullptr) return GAT_EINVAL;
    const int g = next_pow2((heads * f + 3) / 4);
    const long long waves = ((long long)num_nodes * g + kWave - 1) / kWave;
    long long cap = 65536;  // GAT_BWD_WAVES overrides (A/B knob)
    if (const char* v = knob("GAT_BWD_WAVES")) cap = std::atoll(v) > 0 ? std::atoll(v) : cap;
    long long w = waves < cap ? waves : cap;
    w = (w + 3) / 4 * 4;  // whole 256-thread blocks
    *num_parts = (int)(w < 4 ? 4 : w);
    return GAT_OK;
}

int gat_bwd_sources(const int* csc_ptr, const int* csc_dst, const int* csc_eid, int num_nodes,
                    const float* wh, int ld_wh, const float* table, int ld_t,
                    const float* ds_dst, const float* a_src, const float* c_src,
                    const float* a_dst, int heads, int f, int concat, float negative_slope,
                    float dropout_p, unsigned long long seed, const unsigned long long* seed_dev,
                    float* dwh, int ld_dwh, float* partials, int num_parts,
                    int edges_per_row_hint, void* stream) {
    if (heads <= 0 || f <= 0 || num_nodes < 0 || num_parts <= 0 || (num_parts & 3))
        return GAT_EINVAL;
    if (!(dropout_p >= 0.f && dropout_p <= 1.f)) return GAT_EINVAL;
    const int hf = heads * f;
    if (ld_dwh < hf || (ld_dwh & 3)) return GAT_EINVAL;
    if (!bwd_recompute_ok(heads, f, negative_slope, wh, ld_wh)) return GAT_EUNSUPPORTED;
    if (dropout_p > 0.f && csc_eid == nullptr) return GAT_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const DropArgs drop = make_drop(dropout_p, seed, seed_dev);
    const int g = next_pow2(hf / 4);
    int u = bwd_unroll(edges_per_row_hint);
    const dim3 grid(num_parts / 4), block(256);
    const size_t bwd_lds = bwd_lds_bytes();
#define GAT_BS(G, UU)                                                                         \
    hipLaunchKernelGGL((k_bwd_sources<G, UU>), grid, block, bwd_lds, st, csc_ptr, csc_dst, csc_eid,  \
                       num_nodes, wh, ld_wh, table, ld_t, ds_dst, a_src, c_src, a_dst, heads, \
                       f, hf, concat, negative_slope, drop, dwh, ld_dwh, partials)
#define GAT_BS_U(G)                      \
    case G:                              \
        if (u == 4) { GAT_BS(G, 4); }    \
        else if (u == 16) { GAT_BS(G, 16); } \
        else { GAT_BS(G, 8); }           \
        break;
    switch (g) {
        GAT_BS_U(1) GAT_BS_U(2) GAT_BS_U(4) GAT_BS_U(8) GAT_BS_U(16) GAT_BS_U(32) GAT_BS_U(64)
        default: return GAT_EUNSUPPORTED;
    }
#undef GAT_BS_U
#undef GAT_BS
    return status_of(hipGetLastError());
}

int gat_edge_backward_rows(const int* rowptr, const int* col, const int* row_order,
                           int row_begin, int row_end, const int* csr_to_csc, const float* wh,
                           int ld_wh, const float* s_src, int ld_s, const float* a_src,
                           const float* c_src, const float* s_dst, const float* lse,
                           const float* y_heads, const float* grad_out, int heads, int f,
                           int concat, int score_act, float act_param, float dropout_p,
                           unsigned long long seed, const unsigned long long* seed_dev,
                           float* ds_dst, float* az_csc, int edges_per_row_hint, void* stream) {
    if (score_act < GAT_ACT_LEAKY_RELU || score_act > GAT_ACT_HEAD_SOFTMAX) return GAT_EINVAL;
    if (heads <= 0 || f <= 0 || row_begin < 0 || row_end < row_begin) return GAT_EINVAL;
    const int hf = heads * f;
    if (hf > GAT_MAX_HF || heads > GAT_MAX_HEADS) return GAT_EUNSUPPORTED;
    if (ld_wh < hf || ld_s < heads) return GAT_EINVAL;
    if (!(dropout_p >= 0.f && dropout_p <= 1.f)) return GAT_EINVAL;
    const int rows = row_end - row_begin;
    if (rows == 0) return GAT_OK;
    hipStream_t st = (hipStream_t)stream;
    const DropArgs drop = make_drop(dropout_p, seed, seed_dev);
    float2* az = reinterpret_cast<float2*>(az_csc);
    const int hl = f / 4;
    const bool grp_ok = score_act == GAT_ACT_LEAKY_RELU && act_param >= 0.f && act_param <= 1.f &&
                        f % 4 == 0 && next_pow2(hl) == hl && a_src != nullptr &&
                        c_src != nullptr && (ld_wh & 3) == 0 &&
                        kernel_choice("GAT_BWD_KERNEL", "generic");
    if (grp_ok) {
        const int g = next_pow2(hf / 4);
        const int hint = edges_per_row_hint & ~GAT_HINT_LOCAL;
        const int u = hint > 0 && hint <= 12 ? 4 : 8;
        const long long threads = (long long)rows * g;
        const dim3 grid((unsigned)((threads + 255) / 256)), block(256);
#define GAT_BWD_GRP(G, UU)                                                                    \
    hipLaunchKernelGGL((k_edge_bwd_grp<G, UU>), grid, block, 0, st, rowptr, col, row_order,   \
                       row_begin, row_end, csr_to_csc, wh, ld_wh, a_src, c_src, s_dst, lse,   \
                       y_heads, grad_out, heads, f, hf, concat, act_param, drop, ds_dst, az)
#define GAT_BWD_GRP_U(G)                       \
    case G:                                    \
        if (u == 4) { GAT_BWD_GRP(G, 4); }     \
        else { GAT_BWD_GRP(G, 8); }            \
        break;
        switch (g) {
            GAT_BWD_GRP_U(1) GAT_BWD_GRP_U(2) GAT_BWD_GRP_U(4) GAT_BWD_GRP_U(8)
            GAT_BWD_GRP_U(16) GAT_BWD_GRP_U(32) GAT_BWD_GRP_U(64)
            default: return GAT_EUNSUPPORTED;
        }
#undef GAT_BWD_GRP_U
#undef GAT_BWD_GRP
        return status_of(hipGetLastError());
    }
    if (s_src == nullptr) return GAT_EINVAL;
    const dim3 grid(rows), block(kWave);
#define GAT_BWD_ROWS(P)                                                                       \
    case P:                                                                                   \
        hipLaunchKernelGGL((k_edge_bwd_rows<P>), grid, block, 0, st, rowptr, col, row_order,  \
                           row_begin, row_end, csr_to_csc, wh, ld_wh, s_src, ld_s, s_dst, lse, \
                           y_heads, grad_out, heads, f, hf, concat, score_act, act_param,     \
                           drop, ds_dst, az);                                                 \
        break;
    switch (next_pow2(heads)) {
        GAT_BWD_ROWS(1) GAT_BWD_ROWS(2) GAT_BWD_ROWS(4) GAT_BWD_ROWS(8)
        GAT_BWD_ROWS(16) GAT_BWD_ROWS(32) GAT_BWD_ROWS(64)
        default: return GAT_EUNSUPPORTED;
    }
#undef GAT_BWD_ROWS
    return status_of(hipGetLastError());
}

int gat_src_backward(const int* csc_ptr, const int* csc_dst, int num_nodes, const float* wh,
                     int ld_wh, const float* grad_out, const float* az_csc,
                     const float* ds_dst, const float* a_src,
                     const float* a_dst, int heads, int f, int concat, float* dwh, int ld_dwh,
                     float* ds_src, float* partials, int num_parts, void* stream) {
    if (heads <= 0 || f <= 0 || num_nodes < 0 || num_parts <= 0) return GAT_EINVAL;
    const int hf = heads * f;
    if (hf > GAT_MAX_HF || heads > GAT_MAX_HEADS) return GAT_EUNSUPPORTED;
    if (ld_wh < hf || ld_dwh < hf) return GAT_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid(num_parts), block(kWave);
    const int cq = (hf + kWave - 1) / kWave;
#define GAT_SRC_LAUNCH(CQ, P)                                                                 \
    hipLaunchKernelGGL((k_src_bwd<CQ, P>), grid, block, 0, st, csc_ptr, csc_dst, num_nodes,   \
                       wh, ld_wh, grad_out, reinterpret_cast<const float2*>(az_csc), ds_dst,   \
                       a_src, a_dst, heads, f,                                                 \
                       hf, concat, dwh, ld_dwh, ds_src, partials)
#define GAT_SRC_HP(CQ)                                               \
    switch (next_pow2(heads)) {                                      \
        case 1: GAT_SRC_LAUNCH(CQ, 1); break;                        \
        case 2: GAT_SRC_LAUNCH(CQ, 2); break;                        \
        case 4: GAT_SRC_LAUNCH(CQ, 4); break;                        \
        case 8: GAT_SRC_LAUNCH(CQ, 8); break;                        \
        case 16: GAT_SRC_LAUNCH(CQ, 16); break;                      \
        case 32: GAT_SRC_LAUNCH(CQ, 32); break;                      \
        case 64: GAT_SRC_LAUNCH(CQ, 64); break;                      \
        default: return GAT_EUNSUPPORTED;                            \
    }
    switch (cq) {
        case 1: GAT_SRC_HP(1) break;
        case 2: GAT_SRC_HP(2) break;
        case 3: GAT_SRC_HP(3) break;
        case 4: GAT_SRC_HP(4) break;
        default: return GAT_EUNSUPPORTED;
    }
#undef GAT_SRC_HP
#undef GAT_SRC_LAUNCH
    return status_of(hipGetLastError());
}

int gat_weight_grad_workspace_size(int num_nodes, int fin, int hf, size_t* bytes) {
    if (num_nodes < 0 || fin <= 0 || hf <= 0 || bytes == nullptr) return GAT_EINVAL;
    *bytes = (size_t)wgrad_chunks(num_nodes, fin, hf) * hf * fin * sizeof(float);
    return GAT_OK;
}

int gat_weight_grad(const float* x, int num_nodes, int fin, const float* dwh, int ld_dwh, int hf,
                    float* dw, void* workspace, size_t workspace_bytes, void* stream) {
    if (num_nodes < 0 || fin <= 0 || hf <= 0 || ld_dwh < hf) return GAT_EINVAL;
    size_t need = 0;
    int rc = gat_weight_grad_workspace_size(num_nodes, fin, hf, &need);
    if (rc != GAT_OK) return rc;
    if (workspace_bytes < need) return GAT_EWORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    if (num_nodes == 0) return status_of(hipMemsetAsync(dw, 0, sizeof(float) * hf * fin, st));
    const int chunks = wgrad_chunks(num_nodes, fin, hf);
    const int rows = (num_nodes + chunks - 1) / chunks;
    float* part = (float*)workspace;
    const dim3 grid((fin + 63) / 64, chunks, (hf + 63) / 64), block(256);
    // x rows read LW floats at a time where fin and x's alignment allow
    // (GAT_WGRAD_LW A/B knob caps it)
    const uintptr_t xa = reinterpret_cast<uintptr_t>(x);
    int lw = (fin % 4 == 0 && (xa & 15) == 0) ? 4 : (fin % 2 == 0 && (xa & 7) == 0) ? 2 : 1;
    if (const char* v = knob("GAT_WGRAD_LW")) lw = std::min(lw, std::max(1, std::atoi(v)));
    if (lw == 4)
        hipLaunchKernelGGL(k_wgrad<4>, grid, block, 0, st, dwh, ld_dwh, x, num_nodes, fin, hf,
                           rows, part);
    else if (lw == 2)
        hipLaunchKernelGGL(k_wgrad<2>, grid, block, 0, st, dwh, ld_dwh, x, num_nodes, fin, hf,
                           rows, part);
    else
        hipLaunchKernelGGL(k_wgrad<1>, grid, block, 0, st, dwh, ld_dwh, x, num_nodes, fin, hf,
                           rows, part);
    const long long count = (long long)hf * fin;
    hipLaunchKernelGGL(k_colsum, dim3((unsigned)((count + 15) / 16)), dim3(256), 0, st, part,
                       chunks, count, dw, chunks);
    return status_of(hipGetLastError());
}

int gat_input_grad(const float* dwh, int ld_dwh, int num_nodes, int hf, const float* w,
                   int fin, float* dx, int ld_dx, void* stream) {
    if (num_nodes < 0 || fin <= 0 || hf <= 0 || ld_dwh < hf || ld_dx < fin) return GAT_EINVAL;
    if (hf > 128) return GAT_EUNSUPPORTED;
    if (num_nodes == 0) return GAT_OK;
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((num_nodes + 63) / 64), block(256);
    // K = hf padded with zeros to 4 KL
    const int kl = hf <= 8 ? 2 : hf <= 16 ? 4 : hf <= 32 ? 8 : hf <= 64 ? 16 : 32;
#define GAT_DX(KLV)                                                                            \
    hipLaunchKernelGGL(k_dx<KLV>, grid, block, 0, st, dwh, ld_dwh, hf, num_nodes, w, fin, dx, \
                       ld_dx)
    switch (kl) {
        case 2: GAT_DX(2); break;
        case 4: GAT_DX(4); break;
        case 8: GAT_DX(8); break;
        case 16: GAT_DX(16); break;
        default: GAT_DX(32); break;
    }
#undef GAT_DX
    return status_of(hipGetLastError());
}

int gat_sum_partials_workspace_size(int num_parts, long long width, size_t* bytes) {
    if (num_parts <= 0 || width <= 0 || bytes == nullptr) return GAT_EINVAL;
    *bytes = num_parts > 256 ? (size_t)((num_parts + 255) / 256) * width * sizeof(float) : 0;
    return GAT_OK;
}

int gat_sum_partials(const float* partials, int num_parts, long long width, float* out,
                     void* workspace, size_t workspace_bytes, void* stream) {
    size_t need = 0;
    const int rc = gat_sum_partials_workspace_size(num_parts, width, &need);
    if (rc != GAT_OK) return rc;
    if (workspace_bytes < need) return GAT_EWORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    const dim3 gx((unsigned)((width + 15) / 16));
    if (num_parts <= 256) {
        hipLaunchKernelGGL(k_colsum, gx, dim3(256), 0, st, partials, num_parts, width, out,
                           num_parts);
        return status_of(hipGetLastError());
    }
    // two stages: sums of 256-row blocks, then of the block sums (fixed order)
    const int blocks = (num_parts + 255) / 256;
    float* tmp = (float*)workspace;
    hipLaunchKernelGGL(k_colsum, dim3(gx.x, blocks), dim3(256), 0, st, partials, num_parts,
                       width, tmp, 256);
    hipLaunchKernelGGL(k_colsum, gx, dim3(256), 0, st, tmp, blocks, width, out, blocks);
    return status_of(hipGetLastError());
}

}  // extern "C"
