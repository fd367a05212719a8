// MI355X GAT projection: Wh = x W^T + b with the attention scores fused in the
// epilogue (GAT.py:42-52).  Kernels k_project, k_project_x3 (+ k_split_w),
// k_project_wres(_d), k_project_wk; C-ABI gat_project, gat_project_sliced,
// gat_project_chunked, gat_project_ex.

#include "gat_common.h"

namespace {

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
            // value used unconditionally (a select), so the load is never sunk
            // into a branch with its own vmcnt(0); padded k and rows past n: 0
            // (a select, not x * 0: an infinite x would give NaN)
            const int kk = k0 + 4 * s + kq;
            const float v = xr[min(kk, fin - 1)];
            xa[s] = (kk < fin && xs != 0.f) ? v : 0.f;
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
                        if (Ss != nullptr) Ss[(size_t)rr * ld_s + h] = p1[i] + c1[h];
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
                            if (Ss != nullptr) Ss[(size_t)rr * ld_s + h] = p1[i] + c1[h];
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
            if (Ss != nullptr) Ss[(size_t)rr * ld_s + h] = v1 + c1[h];
            s_dst[(size_t)rr * H + h] = v2 + c2[h];
        }
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
// through LDS (as round 2's fp32-MFMA k_project_pipe2, removed in round 6:
// 229-233 us at Reddit), with TWO chunks' loads in flight (a register double
// buffer) where rows are 4-float aligned: with the MFMA phase 2.7x shorter,
// one chunk in flight left the loads exposed (the 128-row, one-ahead form of
// this kernel ran Reddit in 196 us, 2.9 TB/s of x).
// x stays fp32 in LDS and each lane splits its own A fragment (8 consecutive k
// of one row) after reading it — every x element is split exactly once; W is
// split once per chunk at the LDS write, into three bf16 planes the waves
// share.  Fragment maps (cdna_hip_programming.md §3): lane l holds
// A[row l&15][k 8(l>>4)..+8] and B[k 8(l>>4)..+8][col l&15]; C/D as the fp32
// form (col l&15, rows 4(l>>4)+i).
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

// acc + cor of the split form.  For an infinite x element the split gives
// x1 = x and x2 = x - x1 = NaN, so the correction sum is NaN while acc (x1.w1)
// already holds what the reference's fp32 sum gives (+-Inf, or NaN for Inf*0
// and Inf - Inf, which acc reproduces term for term): keep acc when it is
// infinite.  Finite x: acc + cor, unchanged.
__device__ __forceinline__ float split_sum(float a, float c) {
    return __builtin_isinf(a) ? a : a + c;
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

// Row chunks (gridDim.y > 1, gat_project_chunked): blockIdx.y = c projects rows
// [c crows, (c + 1) crows) of x into the Wh block that starts cjump floats
// further per chunk (a rank's chunk slots of the multi-GPU node table, one
// launch for all of them); s_dst and s_src rows stay contiguous.
#define GAT_ROW_CHUNKS()                                                          \
    if (gridDim.y > 1) {                                                          \
        const int cy_ = (int)blockIdx.y;                                          \
        X += (size_t)cy_ * (size_t)crows * (size_t)fin;                           \
        Wh += (size_t)cy_ * (size_t)cjump;                                        \
        s_dst += (size_t)cy_ * (size_t)crows * (size_t)H;                         \
        if (Ss != nullptr) Ss += (size_t)cy_ * (size_t)crows * (size_t)ld_s;      \
        n = min(crows, n - cy_ * crows);                                          \
        if (n <= 0) return;                                                       \
    }

// W [HF, fin] split exactly into three bf16 planes [3][BN][KP] (KP =
// round_up(fin, 64), zero past HF and fin): the pre-split operand of
// k_project_x3<..., PS = true>.  One thread per 8 consecutive k of a column.
__global__ __launch_bounds__(256) void k_split_w(const float* __restrict__ W, int HF, int fin,
                                                int BN, int KP, __bf16* __restrict__ out) {
    const int per_row = KP / 8;
    const int u = blockIdx.x * 256 + threadIdx.x;
    if (u >= BN * per_row) return;
    const int c = u / per_row, k = (u % per_row) * 8;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (c < HF && k + j < fin) ? W[(size_t)c * fin + k + j] : 0.f;
    bf16x8 h1, h2, h3;
    split3_x8(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}, h1, h2, h3);
    const size_t o = (size_t)c * KP + k, plane = (size_t)BN * KP;
    *reinterpret_cast<bf16x8*>(out + o) = h1;
    *reinterpret_cast<bf16x8*>(out + plane + o) = h2;
    *reinterpret_cast<bf16x8*>(out + 2 * plane + o) = h3;
}

// bytes of the pre-split W planes for (hf, fin): 0 where k_project_x3 does not
// take them (fin <= 128, or column tiles other than 2 or 4)
inline size_t wsplit_bytes(int hf, int fin) {
    const int nt = (hf + 15) / 16;
    if (fin <= 128 || (nt != 2 && nt != 4)) return 0;
    return (size_t)3 * (size_t)(nt * 16) * (size_t)((fin + 63) / 64 * 64) * 2;
}

// PS (pre-split W): W points at the three bf16 planes gat_project_ex's
// k_split_w wrote into the caller's workspace, [3][BN][KP] with KP =
// round_up(fin, 64), zero past HF and fin: each chunk's W tile is copied into
// LDS as it is (six 16-B loads per thread at BN = 64) instead of being loaded
// as fp32 and split by every workgroup (the split was ~1/3 of the loop's VALU
// work, which bounds this kernel at Reddit scale).
template <int NT, int LW, int RG, int PD, int MINB = 1, bool PS = false>
__global__ __launch_bounds__(256, MINB) void k_project_x3(
    const float* __restrict__ X, int n, int fin,
    const float* __restrict__ W, const float* __restrict__ bW,
    const float* __restrict__ a1, const float* __restrict__ c1,
    const float* __restrict__ a2, const float* __restrict__ c2,
    int H, int F, int HF, float* __restrict__ Wh, int ld_wh, float* __restrict__ Ss, int ld_s,
    float* __restrict__ s_dst, int slice_w, long long slice_stride, int store_wt, int crows,
    long long cjump) {
    GAT_ROW_CHUNKS();
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
    if (blk0 >= n) return;  // a row chunk shorter than the grid (gat_project_chunked)
    const int row0 = blk0 + w * 16 * RG;  // wave w owns rows [16 RG w, 16 RG (w + 1))
    f32x4 acc[RG][NT], cor[RG][NT];
#pragma unroll
    for (int g = 0; g < RG; ++g)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[g][t] = cor[g][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    // PS: the W tile in 16-B pieces of the pre-split planes
    constexpr int WQ = PS ? 3 * BN * BK / (NTH * 8) : WL;
    static_assert(!PS || (3 * BN * BK) % (NTH * 8) == 0, "pre-split W tile split");
    using wvec = typename std::conditional<PS, u32x4, vec>::type;
    // PD chunks of loads in flight (PD = 2: a register double buffer,
    // statically indexed)
    vec xa_[XL], xb_[PD == 2 ? XL : 1];
    wvec wa_[WQ], wb_[PD == 2 ? WQ : 1];
    // element e = (tid + 256 q) * LW -> row e / 64, k e % 64 (coalesced rows);
    // clamped, in-bounds addresses past n / fin (zeroed W meets them).  The
    // addresses are recomputed per chunk, not hoisted into per-load registers:
    // hoisted offsets (and epilogue parameters loaded before the loop) took
    // Reddit's k_project_x3<4, 2, 1, 1> from 156 to 184 VGPRs, 3 -> 2 waves per
    // SIMD, 205 -> 226 us (profiles/r05/proj_x3_ab.json)
    const int kp = (fin + BK - 1) / BK * BK;  // PS: padded K of the planes
    auto load_chunk = [&](int k0, vec (&xn)[XL], wvec (&wn)[WQ]) {
#pragma unroll
        for (int q = 0; q < XL; ++q) {
            const int e = (tid + NTH * q) * LW;
            const int r = min(blk0 + e / BK, n - 1);
            const int k = min(k0 + e % BK, fin - LW);
            xn[q] = *reinterpret_cast<const vec*>(X + (size_t)r * fin + k);
        }
#pragma unroll
        for (int q = 0; q < WQ; ++q) {
            if constexpr (PS) {
                // 16-B piece u of the chunk's tile: plane u / (8 BN), column
                // (u / 8) % BN, k 8 (u % 8) .. +8 (bf16 elements)
                const int u = tid + NTH * q;
                wn[q] = *reinterpret_cast<const u32x4*>(
                    reinterpret_cast<const __bf16*>(W) +
                    ((size_t)((u / (8 * BN)) * BN + (u / 8) % BN) * kp + 8 * (u % 8) + k0));
            } else {
                const int e = (tid + NTH * q) * LW;
                const int nn = min(e / BK, HF - 1);  // (e past the chunk: a clamped dummy)
                const int k = min(k0 + e % BK, fin - LW);
                wn[q] = *reinterpret_cast<const vec*>(W + (size_t)nn * fin + k);
            }
        }
    };
    // x chunk to LDS as fp32; W chunk split into three bf16 planes
    auto stage = [&](int k0, const vec (&xn)[XL], const wvec (&wn)[WQ]) {
        // k past fin (the tail chunk): the clamped loads hold real x of this row,
        // which must not meet the zeroed W (an infinite x would give Inf * 0 = NaN).
        // Whole chunks (block-uniform, a scalar branch) skip the selects.
        const bool full = k0 + BK <= fin;
        if (full) {
#pragma unroll
            for (int q = 0; q < XL; ++q) {
                const int e = (tid + NTH * q) * LW;
                *reinterpret_cast<vec*>(xsm + (e / BK) * XS + e % BK) = xn[q];
            }
        } else {
#pragma unroll
            for (int q = 0; q < XL; ++q) {
                const int e = (tid + NTH * q) * LW;
                vec v = xn[q];
                if constexpr (LW == 4) {
                    // fin % 4 != 0 (8-B aligned rows): the load for position p was
                    // clamped to fin - 4; its elements d = p - (fin - 4) on are
                    // this position's, and elements past fin are zero
                    const int p = k0 + e % BK, d = p - min(p, fin - 4);
                    if (d == 1) v = f32x4{v.y, v.z, v.w, 0.f};
                    else if (d == 2) v = f32x4{v.z, v.w, 0.f, 0.f};
                    else if (d == 3) v = f32x4{v.w, 0.f, 0.f, 0.f};
                    else if (d != 0) v = f32x4{0.f, 0.f, 0.f, 0.f};
                    const int rem = fin - p;  // elements of this row from p on
                    if (rem < 4) {
                        if (rem <= 0) v.x = 0.f;
                        if (rem <= 1) v.y = 0.f;
                        if (rem <= 2) v.z = 0.f;
                        v.w = 0.f;
                    }
                }
                *reinterpret_cast<vec*>(xsm + (e / BK) * XS + e % BK) =
                    k0 + e % BK < fin ? v : vec{};
            }
        }
        if constexpr (PS) {
#pragma unroll
            for (int q = 0; q < WQ; ++q) {
                const int u = tid + NTH * q;
                *reinterpret_cast<u32x4*>(&wsb[u / (8 * BN)][((u / 8) % BN) * WSB + 8 * (u % 8)]) =
                    wn[q];
            }
            return;
        } else {
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
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[g][t][i] = split_sum(acc[g][t][i], cor[g][t][i]);

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
    float* __restrict__ s_dst, int slice_w, long long slice_stride, int store_wt, int crows,
    long long cjump) {
    GAT_ROW_CHUNKS();
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
            for (int q = 0; q < NL; ++q) {
                // k past fin (clamped loads of this row's real x) meets zero W:
                // zero it, so an infinite x cannot give Inf * 0 = NaN
                const bool kin = 32 * s + 8 * kq + LW * q < fin;
#pragma unroll
                for (int j = 0; j < LW; ++j) {
                    if constexpr (LW == 1) f[q] = kin ? xr[s][q] : 0.f;
                    else f[q * LW + j] = kin ? xr[s][q][j] : 0.f;
                }
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
                const float v = split_sum(acc[t][i], cor[t][i]) + bb[t];  // + bias (GAT.py:43)
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
// k_project_wres with the direct epilogue (heads of 4, 8 or 16 columns), for
// three workgroups / waves per SIMD instead of two.  k_project_wres holds two
// per CU at arxiv's K = 128: 69.6 KB of LDS (W planes 52 KB + a 17 KB output
// tile per wave) and 199 VGPRs; its SQ counters (profiles/r03/sq_counters_arxiv
// .txt) show the waves 44% of their life waiting, 18% issuing VALU.  Here:
//  - the MFMA operands are swapped (A = W fragment, B = x fragment), so a lane
//    holds four consecutive columns of one row and the Wh float4s and the
//    fused scores leave from registers (proj_direct_epilogue, as k_project_wk):
//    no output tile, no LDS round trip, no wave barrier;
//  - the epilogue parameters sit in LDS (1.3 KB), not in 20 VGPRs;
//  - a tile's x fragments are split one k-step at a time, the next tile's loads
//    for that k-step issued right after (12 live bf16x8 VGPRs instead of 48).
// LDS 53.5 KB and <= 168 VGPRs: three workgroups per CU.  Same products and
// split-sum as k_project_wres (outputs within 1e-6 of it: the MFMA's operand
// roles differ).  The default for those heads (arxiv 40.3 -> 31.7 us).
// ---------------------------------------------------------------------------
template <int NT, int LW, int KS>
__global__ __launch_bounds__(256, 3) void k_project_wres_d(
    const float* __restrict__ X, int n, int fin,
    const float* __restrict__ W, const float* __restrict__ bW,
    const float* __restrict__ a1, const float* __restrict__ c1,
    const float* __restrict__ a2, const float* __restrict__ c2,
    int H, int F, int HF, float* __restrict__ Wh, int ld_wh, float* __restrict__ Ss, int ld_s,
    float* __restrict__ s_dst, int slice_w, long long slice_stride, int store_wt, int crows,
    long long cjump) {
    GAT_ROW_CHUNKS();
    constexpr int BN = NT * 16, KP = KS * 32;  // padded K
    constexpr int WSB = KP + 8;
    constexpr int NL = 8 / LW;                  // loads per 8-float fragment
    using vec = typename std::conditional<LW == 4, f32x4,
                typename std::conditional<LW == 2, f32x2, float>::type>::type;
    __shared__ __attribute__((aligned(16))) __bf16 wsb[3][BN * WSB];
    __shared__ __attribute__((aligned(16))) float prm[3 * BN + 128];
    float* bs = prm;
    float* a1s = prm + BN;
    float* a2s = prm + 2 * BN;
    float* c1s = prm + 3 * BN;
    float* c2s = c1s + 64;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int cl = lane & 15, kq = lane >> 4;
    const int tiles = (n + 15) / 16;
    const int tstride = gridDim.x * 4;
    int tile = blockIdx.x * 4 + w;
    vec xr[KS][NL];
    auto load_step = [&](const float* xrow, int s) {
#pragma unroll
        for (int q = 0; q < NL; ++q) {
            const int k = min(32 * s + 8 * kq + LW * q, fin - LW);
            xr[s][q] = *reinterpret_cast<const vec*>(xrow + k);
        }
    };
    {
        const float* xrow = X + (size_t)min(min(tile, tiles - 1) * 16 + cl, n - 1) * fin;
#pragma unroll
        for (int s = 0; s < KS; ++s) load_step(xrow, s);
    }
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
    {  // W split into three bf16 planes, as k_project_wres
        constexpr int WQ = (BN * KP + 256 * LW - 1) / (256 * LW);
        vec wv[WQ];
#pragma unroll
        for (int q = 0; q < WQ; ++q) {
            const int e = (tid + 256 * q) * LW;
            const int c = min(e / KP, HF - 1), k = min(e % KP, fin - LW);
            wv[q] = *reinterpret_cast<const vec*>(W + (size_t)c * fin + k);
        }
#pragma unroll
        for (int q = 0; q < WQ; ++q) {
            const int e = (tid + 256 * q) * LW;
            if (e < BN * KP) {
                const int c = e / KP, k = e % KP;
                const bool ok = c < HF && k < fin;
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

    for (; tile < tiles; tile += tstride) {
        // the next tile's row (the last tile re-loads itself, unused: every load
        // is unconditional, see k_project_wres)
        const float* xnext =
            X + (size_t)min(min(tile + tstride, tiles - 1) * 16 + cl, n - 1) * fin;
        f32x4 acc[NT], cor[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = cor[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            bf16x8 x1, x2, x3;
            {
                float f[8];
#pragma unroll
                for (int q = 0; q < NL; ++q) {
                    // k past fin (clamped loads of this row's real x) meets zero W
                    const bool kin = 32 * s + 8 * kq + LW * q < fin;
#pragma unroll
                    for (int j = 0; j < LW; ++j) {
                        if constexpr (LW == 1) f[q] = kin ? xr[s][q] : 0.f;
                        else f[q * LW + j] = kin ? xr[s][q][j] : 0.f;
                    }
                }
                split3_x8(f32x4{f[0], f[1], f[2], f[3]}, f32x4{f[4], f[5], f[6], f[7]}, x1, x2, x3);
            }
            load_step(xnext, s);  // xr[s] is free: the next tile's k-step s
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                int o = (t * 16 + cl) * WSB + 32 * s + 8 * kq;
                // opaque per iteration: the W fragments are the same for every
                // tile, and hoisted out of the tile loop they would hold
                // KS x NT x 3 x 4 = 192 VGPRs at arxiv (spilled under the bound)
                asm volatile("" : "+v"(o));
                const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(&wsb[0][o]);
                const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(&wsb[1][o]);
                const bf16x8 b3 = *reinterpret_cast<const bf16x8*>(&wsb[2][o]);
                // swapped operands: the accumulator holds Wh^T (lane: row cl,
                // columns 16t + 4kq .. +4)
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1, x1, acc[t], 0, 0, 0);
                cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b2, x1, cor[t], 0, 0, 0);
                cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1, x2, cor[t], 0, 0, 0);
                cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b3, x1, cor[t], 0, 0, 0);
                cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b2, x2, cor[t], 0, 0, 0);
                cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1, x3, cor[t], 0, 0, 0);
            }
        }
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[t][i] = split_sum(acc[t][i], cor[t][i]);
        proj_direct_epilogue<NT>(acc, tile * 16 + cl, n, kq, bs, a1s, a2s, c1s, c2s, H, F, HF, Wh,
                                 ld_wh, Ss, ld_s, s_dst, slice_w, slice_stride, store_wt);
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
    int slice_w, long long slice_stride, int store_wt, int crows,
    long long cjump) {
    GAT_ROW_CHUNKS();
    constexpr int BM = 64, BN = NT * 16;
    constexpr int OS = BN + 4;  // output-tile stride: float4-aligned rows, no write conflicts
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int cl = lane & 15, kq = lane >> 4;
    const int row0 = blockIdx.x * BM;
    if (row0 >= n) return;  // a row chunk shorter than the grid (gat_project_chunked)
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

// k_project_x3 on pre-split W (instantiated for 2 and 4 column tiles only).  It
// reads x as float4s for every even fin whose rows are 8-B aligned (Reddit's
// 602: half the rows start 8 B into a 16-B unit; the loads need only dword
// alignment), the last k chunk's clamped loads shifted into place in `stage`:
// Reddit 191.7 -> 186.3 us, a P = 8 rank's share 30.9 -> 30.1 us, bitwise equal
// outputs (profiles/r06/proj_ab_x3_float4_reddit.json); two chunks in flight
// there: 216.6 us
template <int NT, int LW, class... A>
static void launch_x3_presplit(dim3 grid, dim3 block, hipStream_t st, A... a) {
    if constexpr (NT == 2 || NT == 4)
        hipLaunchKernelGGL((k_project_x3<NT, LW, 1, 1, 1, true>), grid, block, 0, st, a...);
}

}  // namespace

extern "C" {

// slices == 1: Wh row-major [n, ld_wh].  slices > 1: `slices` planes of
// [n, ld_wh = hf / slices] at wh + g * n * ld_wh (only the whole-K and the
// pipelined kernels write that layout).
static int project_impl(const float* x, int n, int fin, const float* w, const float* b,
                        const float* a_src, const float* c_src, const float* a_dst,
                        const float* c_dst, int heads, int f, int slices, float* wh, int ld_wh,
                        float* s_src, int ld_s, float* s_dst, void* stream, int n_table = 0,
                        int crows = 0, long long cjump = 0, void* ws = nullptr,
                        size_t ws_bytes = 0) {
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
    if (sliced && n_table < (crows > 0 ? std::min(crows, n) : n)) return GAT_EINVAL;
    if (n == 0) return GAT_OK;
    // row chunks (gat_project_chunked): ny launches' worth of rows in one grid
    if (crows < 0 || (crows > 0 && (crows % 64 != 0 || !sliced))) return GAT_EINVAL;
    const int ny = crows > 0 ? (n + crows - 1) / crows : 1;
    const int nr = crows > 0 ? std::min(crows, n) : n;  // rows per grid slice
    const int slice_w = sliced ? ld_wh : round_up4(hf);
    const long long slice_stride = sliced ? (long long)n_table * ld_wh : 0;
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((nr + 63) / 64, ny), block(256);
    const int nt = (hf + 15) / 16;
    const int store_wt = 1;  // Wh / scores stored write-through (sc1)
    const bool pow2_f = next_pow2(f) == f;
    const size_t wk_lds = (size_t)wk_lds_floats(fin, nt) * sizeof(float);
    const bool aligned16 = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) |
                             reinterpret_cast<uintptr_t>(wh)) & 15) == 0;
    // x and W read LW floats at a time where fin and the pointers allow
    const uintptr_t xwa = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w);
    const int lw = (fin % 4 == 0 && (xwa & 15) == 0) ? 4 : (fin % 2 == 0 && (xwa & 7) == 0) ? 2 : 1;
    // W-resident kernel for 64 < fin <= 128 (k_project_wres: arxiv 44.4 -> 38.4 us
    // against k_project_x3; at PPI's fin 50 the whole-K fp32 k_project_wk stays
    // faster, 10.4 vs 12.5 us: 1.4 tiles per wave do not amortise the W split)
    if (fin > 64 && fin <= 128 && (nt == 1 || nt == 2 || nt == 4) && pow2_f && f <= 16) {
        const long long tiles = (nr + 15) / 16;
        // the direct-epilogue form (heads of 4, 8 or 16 columns), three
        // workgroups per CU: arxiv 40.3 -> 31.7 us, a P = 8 rank's 21k rows
        // 11.4 -> 9.9 us, same box (profiles/r05/proj_wres_direct.json);
        // k_project_wres (output tile in LDS, two per CU) for heads of 1 or 2
        const bool wdir = f == 4 || f == 8 || f == 16;
        const int wg_cu = wdir ? 3 : 2;
        const int grid_w = (int)std::max<long long>(
            1, std::min<long long>((tiles + 3) / 4, 256LL * wg_cu / ny));
#define GAT_WRES(NTV, LWV)                                                                  \
    if (wdir)                                                                               \
        hipLaunchKernelGGL((k_project_wres_d<NTV, LWV, 4>), dim3(grid_w, ny), dim3(256), 0, \
                           st, x, n, fin, w, b, a_src, c_src, a_dst, c_dst, heads, f, hf, wh, \
                           ld_wh, s_src, ld_s, s_dst, slice_w, slice_stride, store_wt, crows, \
                           cjump);                                                          \
    else                                                                                    \
        hipLaunchKernelGGL((k_project_wres<NTV, LWV, 4>), dim3(grid_w, ny), dim3(256), 0,   \
                           st, x, n, fin, w, b, a_src, c_src, a_dst, c_dst, heads, f, hf, wh, \
                           ld_wh, s_src, ld_s, s_dst, slice_w, slice_stride, store_wt, crows, \
                           cjump)
#define GAT_WRES_LW(NTV)                                               \
    if (lw == 4) { GAT_WRES(NTV, 4); }                                 \
    else if (lw == 2) { GAT_WRES(NTV, 2); }                            \
    else { GAT_WRES(NTV, 1); }
        if (nt == 1) { GAT_WRES_LW(1) }
        else if (nt == 2) { GAT_WRES_LW(2) }
        else { GAT_WRES_LW(4) }
#undef GAT_WRES_LW
#undef GAT_WRES
        return status_of(hipGetLastError());
    }
    // whole K in LDS (fin <= 64: its staging loads cover 64 x 64 floats of X and W)
    if (fin > 0 && fin <= 64 && aligned16 && wk_lds <= 160 * 1024) {
        // the direct epilogue for heads of 4, 8 or 16 columns
        const bool direct = f == 4 || f == 8 || f == 16;
#define GAT_WK_CASE(NT)                                                                       \
    case NT:                                                                                  \
        if (direct)                                                                           \
            hipLaunchKernelGGL((k_project_wk<NT, true>), grid, block, wk_lds, st, x, n, fin,  \
                               w, b, a_src, c_src, a_dst, c_dst, heads, f, hf, wh, ld_wh,     \
                               s_src, ld_s, s_dst, slice_w, slice_stride, store_wt, crows,    \
                               cjump);                                                        \
        else                                                                                  \
            hipLaunchKernelGGL((k_project_wk<NT>), grid, block, wk_lds, st, x, n, fin, w, b,  \
                               a_src, c_src, a_dst, c_dst, heads, f, hf, wh, ld_wh, s_src,    \
                               ld_s, s_dst, slice_w, slice_stride, store_wt, crows, cjump);   \
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
    // split-bf16 matrix cores, K-chunked, for large fin (F a power of two
    // dividing 16, HF in {16, 32, 64}, i.e. nt in {1, 2, 4}):
    //   * 4-float x rows (arxiv-like): 64-row blocks, two chunks in flight;
    //   * 2-float rows (Reddit's 602): 64-row blocks, one chunk in flight
    //     (tools/proj_bench.py: Reddit 204 -> 201 us, a P = 8 rank's 29k rows
    //     34.4 -> 29.1 us: twice the blocks fill the CUs; profiles/r04/proj_ab.json;
    //     re-measured against the other block shapes in round 5: 190.9 vs
    //     207-242 us, profiles/r05/proj_x3v_reddit.json), on W pre-split once
    //     per call into bf16 planes (k_split_w) when the caller passes the
    //     workspace (gat_project_ex): Reddit 200 -> 190 us, same box
    //     (profiles/r05/proj_presplit_ab.json);
    //   * 1-float rows: 128-row blocks sharing every B fragment, one chunk.
    if (fin > 64 && (nt == 1 || nt == 2 || nt == 4) && pow2_f && f <= 16 &&
        (long long)n * fin < (1LL << 31)) {
        const dim3 bp(256);
        const size_t need = wsplit_bytes(hf, fin);
        const bool presplit = lw == 2 && (nt == 2 || nt == 4) && ws != nullptr && need > 0 &&
                              ws_bytes >= need && (reinterpret_cast<uintptr_t>(ws) & 15) == 0;
        if (presplit) {
            const int bn = nt * 16, kpad = (fin + 63) / 64 * 64;
            const int units = bn * (kpad / 8);
            hipLaunchKernelGGL(k_split_w, dim3((units + 255) / 256), dim3(256), 0, st, w, hf, fin, bn,
                               kpad, reinterpret_cast<__bf16*>(ws));
        }
#define GAT_X3(NT, LWV, RGV, PDV, MB, BMV)                                                    \
    hipLaunchKernelGGL((k_project_x3<NT, LWV, RGV, PDV, MB>), dim3((nr + BMV - 1) / BMV, ny), bp, \
                       0, st, x, n, fin, w, b, a_src, c_src, a_dst, c_dst, heads, f, hf, wh,   \
                       ld_wh, s_src, ld_s, s_dst, slice_w, slice_stride, store_wt, crows,     \
                       cjump)
#define GAT_X3_NT(NT)                                                                          \
    if (lw == 4) { GAT_X3(NT, 4, 1, 2, 1, 64); }                                               \
    else if (lw == 2 && presplit)                                                              \
        launch_x3_presplit<NT, 4>(dim3((nr + 63) / 64, ny), bp, st, x, n, fin,                 \
                                  reinterpret_cast<const float*>(ws), b, a_src, c_src, a_dst,  \
                                  c_dst, heads, f, hf, wh, ld_wh, s_src, ld_s, s_dst, slice_w, \
                                  slice_stride, store_wt, crows, cjump);                       \
    else if (lw == 2) { GAT_X3(NT, 2, 1, 1, 1, 64); }                                          \
    else { GAT_X3(NT, 1, 2, 1, 1, 128); }
        if (nt == 1) { GAT_X3_NT(1) }
        else if (nt == 2) { GAT_X3_NT(2) }
        else { GAT_X3_NT(4) }
#undef GAT_X3_NT
#undef GAT_X3
        return status_of(hipGetLastError());
    }
    if (sliced || ny > 1) return GAT_EUNSUPPORTED;  // the kernels below: row-major Wh, no chunks
    // K-tiled fallback (unaligned x or W, other head widths): a shuffle
    // epilogue where F divides 16 or is a multiple of 16, else an LDS one
    const bool shfl = (f <= 16 && 16 % f == 0) || (f % 16 == 0);
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

int gat_project_chunked(const float* x, int n, int fin, const float* w, const float* b,
                        const float* a_src, const float* c_src, const float* a_dst,
                        const float* c_dst, int heads, int f, int slices, float* wh,
                        int plane_rows, int chunk_rows, long long chunk_stride, float* s_dst,
                        void* stream) {
    if (slices <= 1 || heads <= 0 || f <= 0 || (heads * f) % slices != 0 || chunk_rows <= 0 ||
        plane_rows < chunk_rows || chunk_stride < (long long)slices * plane_rows * (heads * f / slices))
        return GAT_EINVAL;
    return project_impl(x, n, fin, w, b, a_src, c_src, a_dst, c_dst, heads, f, slices, wh,
                        heads * f / slices, nullptr, heads, s_dst, stream, plane_rows, chunk_rows,
                        chunk_stride);
}

int gat_project_workspace_size(int fin, int heads, int f, size_t* bytes) {
    if (bytes == nullptr || fin < 0 || heads <= 0 || f <= 0) return GAT_EINVAL;
    *bytes = wsplit_bytes(heads * f, fin);
    return GAT_OK;
}

int gat_project_ex(const float* x, int n, int fin, const float* w, const float* b,
                   const float* a_src, const float* c_src, const float* a_dst, const float* c_dst,
                   int heads, int f, int slices, float* wh, int ld_wh_or_n_table, float* s_src,
                   int ld_s, float* s_dst, int chunk_rows, long long chunk_stride,
                   void* workspace, size_t workspace_bytes, void* stream) {
    if (slices <= 0 || heads <= 0 || f <= 0 || (heads * f) % slices != 0 || chunk_rows < 0)
        return GAT_EINVAL;
    if (chunk_rows > 0 && (slices <= 1 || ld_wh_or_n_table < chunk_rows ||
                           chunk_stride < (long long)slices * ld_wh_or_n_table * (heads * f / slices)))
        return GAT_EINVAL;
    if (slices == 1)
        return project_impl(x, n, fin, w, b, a_src, c_src, a_dst, c_dst, heads, f, 1, wh,
                            ld_wh_or_n_table, s_src, ld_s, s_dst, stream, 0, 0, 0, workspace,
                            workspace_bytes);
    if (s_src == nullptr) ld_s = heads;
    return project_impl(x, n, fin, w, b, a_src, c_src, a_dst, c_dst, heads, f, slices, wh,
                        heads * f / slices, s_src, ld_s, s_dst, stream, ld_wh_or_n_table,
                        chunk_rows, chunk_stride, workspace, workspace_bytes);
}

}  // extern "C"
