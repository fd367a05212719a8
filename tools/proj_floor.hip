// Projection floor probe (PPI shape by default): how long must a kernel that
// reads x [N, fin] and writes the two-plane Wh table + s_dst take on this GPU,
// and how do the library's projection and a register-tile prototype compare?
// Standalone HIP program linked against the in-tree libgat_amd.so.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/proj_floor.hip \
//       -Iinclude -Latmlgraphattentionnetworks_amd -lgat_amd \
//       -Wl,-rpath,'$ORIGIN/../atmlgraphattentionnetworks_amd' -o tools/proj_floor
//   tools/proj_floor [n] [fin]
//
// Every kernel is timed two ways: R launches back to back (hipEvents around
// the loop), and R times behind a "pollute" kernel that, like the edge kernel
// before the next step's projection, reads the Wh table and writes an
// output of the same size (time of the pair minus time of pollute alone).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gat_amd.h"

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void st_wt4(float* base, size_t idx, f32x4 v) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7FFFFFFF, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsrc,
                                           (int)(idx * 4), 0, 16);
}
__device__ __forceinline__ void st_wt1(float* base, size_t idx, float v) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7FFFFFFF, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsrc, (int)(idx * 4), 0, 16);
}

// ---- floors -----------------------------------------------------------------
// read n4_in float4s, write n4_out float4s (write-through), grid-stride
__global__ __launch_bounds__(256) void k_copy(const f32x4* __restrict__ in, long n4_in,
                                              float* __restrict__ out, long n4_out, int wt) {
    const long t = blockIdx.x * 256L + threadIdx.x, s = gridDim.x * 256L;
    const long m = n4_in > n4_out ? n4_in : n4_out;
    for (long i = t; i < m; i += s) {
        f32x4 v = i < n4_in ? in[i] : f32x4{0.f, 0.f, 0.f, 0.f};
        if (i < n4_out) {
            if (wt) st_wt4(out, 4 * i, v);
            else reinterpret_cast<f32x4*>(out)[i] = v;
        }
    }
}

// the edge kernel's footprint: read the table, write an output of its size
__global__ __launch_bounds__(256) void k_pollute(const f32x4* __restrict__ tab, long n4,
                                                 float* __restrict__ out) {
    const long t = blockIdx.x * 256L + threadIdx.x, s = gridDim.x * 256L;
    for (long i = t; i < n4; i += s) st_wt4(out, 4 * i, tab[(i * 7919) % n4] * 1.0001f);
}

// store-policy variants: AUX = the buffer instruction's cache-policy bits
// (gfx950: sc0 = 1, nt = 2, sc1 = 16)
template <int AUX>
__global__ __launch_bounds__(256) void k_copy_aux(const f32x4* __restrict__ in, long n4_in,
                                                  float* __restrict__ out, long n4_out) {
    const long t = blockIdx.x * 256L + threadIdx.x, s = gridDim.x * 256L;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0x7FFFFFFF, 0x00020000);
    for (long i = t; i < n4_out; i += s) {
        const f32x4 v = in[i % n4_in];
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsrc, (int)(16 * i), 0, AUX);
    }
}
// pollute with a load policy on the table reads
template <int LAUX>
__global__ __launch_bounds__(256) void k_pollute_aux(const float* __restrict__ tab, long n4,
                                                     float* __restrict__ out) {
    const long t = blockIdx.x * 256L + threadIdx.x, s = gridDim.x * 256L;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(tab), (short)0, 0x7FFFFFFF, 0x00020000);
    for (long i = t; i < n4; i += s) {
        const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(16 * ((i * 7919) % n4)), 0, LAUX);
        st_wt4(out, 4 * i, __builtin_bit_cast(f32x4, u) * 1.0001f);
    }
}

// ---- register-tile prototype ------------------------------------------------
__device__ __forceinline__ void split3_pair(f32x2 v, bf16x2& p1, bf16x2& p2, bf16x2& p3) {
    p1 = __builtin_convertvector(v, bf16x2);
    const f32x2 r1 = v - __builtin_convertvector(p1, f32x2);
    p2 = __builtin_convertvector(r1, bf16x2);
    const f32x2 r2 = r1 - __builtin_convertvector(p2, f32x2);
    p3 = __builtin_convertvector(r2, bf16x2);
}
__device__ __forceinline__ void split3_8(const float* f, bf16x8& h1, bf16x8& h2, bf16x8& h3) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        bf16x2 p1, p2, p3;
        split3_pair(f32x2{f[2 * i], f[2 * i + 1]}, p1, p2, p3);
        h1[2 * i] = p1[0];
        h1[2 * i + 1] = p1[1];
        h2[2 * i] = p2[0];
        h2[2 * i + 1] = p2[1];
        h3[2 * i] = p3[0];
        h3[2 * i + 1] = p3[1];
    }
}

// C' = W x^T per 16-row tile on the split-bf16 matrix cores: A = W fragment
// (lane: output column 16t + (l&15), k in [KL kq, KL kq + KL) over the KS
// k-steps), B = x fragment (lane: row l&15, the same k).  Lane l then holds
// Wh[row l&15][16t + 4kq .. +4]: one float4 store per 16-column block.
// W: staged once per workgroup in LDS (coalesced), each wave reads its
// fragments and keeps them split in registers.  x: each wave's 16-row tile is
// contiguous in HBM, loaded coalesced (float4) one tile ahead into registers,
// written to a wave-private LDS tile, fragments read back from there.
// MODE (ablation): bit 0 no s_dst stores, bit 1 no Wh stores, bit 2 plain
// (not write-through) stores, bit 3 no MFMA (x sums stand in), bit 4 the
// output tile and scores go through a wave-private LDS tile so that Wh and
// s_dst leave as whole coalesced rows (a 16-row tile of one plane is
// contiguous in HBM)
template <int NT, int KS, int LR, int MODE = 0>
__global__ __launch_bounds__(256, 2) void k_proj_rt(
    const float* __restrict__ X, int n, int fin, const float* __restrict__ W,
    const float* __restrict__ bW, const float* __restrict__ a1, const float* __restrict__ c1,
    const float* __restrict__ a2, const float* __restrict__ c2, int H, int F, int HF,
    float* __restrict__ Wh, int slice_w, long slice_stride, float* __restrict__ s_dst) {
    constexpr int KL = KS * 8;        // k values per lane
    constexpr int KP = KS * 32;       // padded K
    constexpr int XQ = 2 * KS;        // float4 loads per lane per tile (16 rows x <= KP)
    constexpr int XS = 16 * KP + KP;  // floats per wave-private x tile (+ read overhang)
    using rvec = typename std::conditional<LR == 2, f32x2, float>::type;
    __shared__ __attribute__((aligned(16))) float xs_all[4][XS];
    __shared__ __attribute__((aligned(16))) float ws[16 * NT * KP + KP];
    constexpr int OS = 16 * NT + 4;
    __shared__ __attribute__((aligned(16))) float os_all[4][16 * OS + 16 * 16];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int cl = lane & 15, kq = lane >> 4;
    const int tiles = (n + 15) / 16;
    const int tstride = gridDim.x * 4;
    int tile = blockIdx.x * 4 + w;
    const int kb = KL * kq;
    float* xs = xs_all[w];

    // this wave's first tile: 16 rows = one contiguous run of 16*fin floats
    // (the last tile may be short: clamp inside the array)
    const long xtot4 = ((long)n * fin) / 4;  // whole float4s in x (fin*n % 4 tail below)
    f32x4 xr[XQ];
    auto load_tile = [&](int tl) {
        const long base4 = (long)tl * 16 * fin / 4;  // 16*fin*tl floats: 16-B aligned
#pragma unroll
        for (int q = 0; q < XQ; ++q)
            xr[q] = reinterpret_cast<const f32x4*>(X)[min(base4 + lane + 64 * q, xtot4 - 1)];
    };
    load_tile(min(tile, tiles - 1));
    // W [HF, fin] into LDS, coalesced; rows past HF and k past fin read as zero below
    {
        const int wn = HF * fin, wn4 = wn / 4;
        for (int i = tid; i < wn4; i += 256)
            reinterpret_cast<f32x4*>(ws)[i] = reinterpret_cast<const f32x4*>(W)[i];
        for (int i = 4 * wn4 + tid; i < wn; i += 256) ws[i] = W[i];
    }
    __syncthreads();
    bf16x8 w1[NT][KS], w2[NT][KS], w3[NT][KS];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int c = 16 * t + cl;
        const bool cok = c < HF;
        const float* wr = ws + (cok ? c : 0) * fin + kb;
        float v[KL];
#pragma unroll
        for (int k = 0; k < KL; ++k) v[k] = (cok && kb + k < fin) ? wr[k] : 0.f;
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) split3_8(&v[8 * s2], w1[t][s2], w2[t][s2], w3[t][s2]);
    }
    f32x4 bb[NT], p2v[NT];
    float cs2[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int cc = min(16 * t + 4 * kq + i, HF - 1);
            const bool ok = 16 * t + 4 * kq + i < HF;
            bb[t][i] = ok ? bW[cc] : 0.f;
            p2v[t][i] = ok ? a2[cc] : 0.f;
        }
        cs2[t] = c2[min((16 * t + 4 * kq) / F, H - 1)];
    }
    const int hl = F / 4;  // kq lanes per head (F in {4, 8, 16})

    for (; tile < tiles; tile += tstride) {
        // this tile to the wave's LDS tile (as laid out in HBM: row stride fin)
#pragma unroll
        for (int q = 0; q < XQ; ++q)
            if (lane + 64 * q < 4 * fin) reinterpret_cast<f32x4*>(xs)[lane + 64 * q] = xr[q];
        load_tile(min(tile + tstride, tiles - 1));  // next tile, in flight under this one
        __builtin_amdgcn_wave_barrier();
        float f[KL];
        const float* xrow = xs + cl * fin + kb;
#pragma unroll
        for (int k = 0; k < KL; k += LR) {
            rvec v = *reinterpret_cast<const rvec*>(xrow + k);
            if constexpr (LR == 1) f[k] = v;
            else { f[k] = v.x; f[k + 1] = v.y; }
        }
#pragma unroll
        for (int k = 0; k < KL; ++k) f[k] = kb + k < fin ? f[k] : 0.f;
        __builtin_amdgcn_wave_barrier();
        bf16x8 x1[KS], x2[KS], x3[KS];
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) split3_8(&f[8 * s2], x1[s2], x2[s2], x3[s2]);
        f32x4 acc[NT], cor[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = cor[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr ((MODE & 8) != 0) {
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int k = 0; k < KL; ++k) acc[t][k & 3] += f[k];
        } else
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2)
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[t][s2], x1[s2], acc[t], 0, 0, 0);
                cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2[t][s2], x1[s2], cor[t], 0, 0, 0);
                cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[t][s2], x2[s2], cor[t], 0, 0, 0);
                cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w3[t][s2], x1[s2], cor[t], 0, 0, 0);
                cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2[t][s2], x2[s2], cor[t], 0, 0, 0);
                cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[t][s2], x3[s2], cor[t], 0, 0, 0);
            }
        const int row = tile * 16 + cl;
        const bool rok = row < n;
        if constexpr ((MODE & 16) != 0) {
            float* os = os_all[w];
            float* sc = os + 16 * OS;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const f32x4 v = acc[t] + cor[t] + bb[t];
                const int c0 = 16 * t + 4 * kq;
                float p2 = v.x * p2v[t].x + v.y * p2v[t].y + v.z * p2v[t].z + v.w * p2v[t].w;
                for (int o = 16; o < 16 * hl; o <<= 1) p2 += __shfl_xor(p2, o);
                *reinterpret_cast<f32x4*>(os + cl * OS + c0) = v;
                if (c0 < HF && (kq & (hl - 1)) == 0) sc[cl * H + c0 / F] = p2 + cs2[t];
            }
            __builtin_amdgcn_wave_barrier();
            const int row0 = tile * 16;
            const int sw4 = slice_w >> 2, lsw = 31 - __builtin_clz((unsigned)sw4);
            const int planes = (HF + slice_w - 1) / slice_w;
            for (int g = 0; g < planes; ++g)
                for (int q = lane; q < 16 * sw4; q += 64) {
                    const int r = q >> lsw, c4 = q & (sw4 - 1);
                    if (row0 + r < n)
                        st_wt4(Wh, (size_t)g * slice_stride + (size_t)(row0 + r) * slice_w + 4 * c4,
                               *reinterpret_cast<const f32x4*>(os + r * OS + g * slice_w + 4 * c4));
                }
            // s_dst rows of the tile: 16 * H contiguous floats (H % 4 == 0 here)
            const int h4 = H >> 2;
            for (int q = lane; q < 16 * h4; q += 64) {
                const int r = q / h4, c4 = q - r * h4;
                if (row0 + r < n)
                    st_wt4(s_dst, (size_t)(row0 + r) * H + 4 * c4,
                           *reinterpret_cast<const f32x4*>(sc + r * H + 4 * c4));
            }
            __builtin_amdgcn_wave_barrier();
            continue;
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const f32x4 v = acc[t] + cor[t] + bb[t];
            const int c0 = 16 * t + 4 * kq;
            float p2 = v.x * p2v[t].x + v.y * p2v[t].y + v.z * p2v[t].z + v.w * p2v[t].w;
            for (int o = 16; o < 16 * hl; o <<= 1) p2 += __shfl_xor(p2, o);
            if (rok && c0 < HF) {
                const int g = c0 / slice_w;
                const size_t o = (size_t)g * slice_stride + (size_t)row * slice_w + (c0 - g * slice_w);
                if constexpr ((MODE & 2) == 0) {
                    if constexpr ((MODE & 4) != 0) *reinterpret_cast<f32x4*>(Wh + o) = v;
                    else st_wt4(Wh, o, v);
                }
                if constexpr ((MODE & 1) == 0) {
                    if ((kq & (hl - 1)) == 0) {
                        if constexpr ((MODE & 4) != 0) s_dst[(size_t)row * H + c0 / F] = p2 + cs2[t];
                        else st_wt1(s_dst, (size_t)row * H + c0 / F, p2 + cs2[t]);
                    }
                }
            }
        }
    }
}

// One-shot workgroup of 64 rows (4 waves x 16-row tiles), as the library's
// k_project_wk, but on the split-bf16 matrix cores: the x tile (fp32) and W
// go to LDS with coalesced float4 loads; W is split ONCE per workgroup into
// three bf16 planes [col][KP + 8]; each wave reads its x fragments (fp32,
// zeroed past fin, split in registers) and the W planes' fragments, 6 MFMA
// per (16-col tile, 32-deep k step).  Output straight from the accumulators
// (lane: row l&15, 4 consecutive columns).
template <int NT, int KS>
__global__ __launch_bounds__(256) void k_proj_wk3(
    const float* __restrict__ X, int n, int fin, const float* __restrict__ W,
    const float* __restrict__ bW, const float* __restrict__ a2, const float* __restrict__ c2,
    int H, int F, int HF, float* __restrict__ Wh, int slice_w, long slice_stride,
    float* __restrict__ s_dst) {
    constexpr int KP = 32 * KS, WSB = KP + 8, BN = 16 * NT;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    __bf16* wsb = reinterpret_cast<__bf16*>(smem);            // [3][BN][WSB]
    float* xs = smem + (3 * BN * WSB) / 2;                       // [64][fin] (+KP overhang)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int cl = lane & 15, kq = lane >> 4;
    const int row0 = blockIdx.x * 64;
    const int rows = min(64, n - row0);
    // x rows [row0, row0 + rows): one contiguous run; W [HF, fin] another
    {
        const int xc = rows * fin, xc4 = xc >> 2;
        const float* xg = X + (size_t)row0 * fin;  // 64*fin*4*b bytes: 16-B aligned
        constexpr int XIT = 64 * KP / 4 / 256;     // fin <= KP
        f32x4 xv[XIT];
#pragma unroll
        for (int it = 0; it < XIT; ++it)
            xv[it] = reinterpret_cast<const f32x4*>(xg)[min(tid + 256 * it, max(xc4 - 1, 0))];
        // W: each thread splits 4 consecutive k of one column per step
        constexpr int WIT = BN * KP / 4 / 256;
        f32x4 wv[WIT];
#pragma unroll
        for (int it = 0; it < WIT; ++it) {
            const int e = 4 * (tid + 256 * it), c = e / KP, k = e % KP;
            const float* src = W + (size_t)min(c, HF - 1) * fin;
#pragma unroll
            for (int j = 0; j < 4; ++j) wv[it][j] = src[min(k + j, fin - 1)];
        }
#pragma unroll
        for (int it = 0; it < XIT; ++it)
            if (tid + 256 * it < xc4) reinterpret_cast<f32x4*>(xs)[tid + 256 * it] = xv[it];
        for (int i = 4 * xc4 + tid; i < xc; i += 256) xs[i] = xg[i];
#pragma unroll
        for (int it = 0; it < WIT; ++it) {
            const int e = 4 * (tid + 256 * it), c = e / KP, k = e % KP;
            f32x4 v = wv[it];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (c < HF && k + j < fin) ? v[j] : 0.f;
            bf16x2 p1a, p2a, p3a, p1b, p2b, p3b;
            split3_pair(f32x2{v.x, v.y}, p1a, p2a, p3a);
            split3_pair(f32x2{v.z, v.w}, p1b, p2b, p3b);
            const int o = c * WSB + k;
            typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
            *reinterpret_cast<bf16x4*>(wsb + o) = bf16x4{p1a[0], p1a[1], p1b[0], p1b[1]};
            *reinterpret_cast<bf16x4*>(wsb + BN * WSB + o) = bf16x4{p2a[0], p2a[1], p2b[0], p2b[1]};
            *reinterpret_cast<bf16x4*>(wsb + 2 * BN * WSB + o) = bf16x4{p3a[0], p3a[1], p3b[0], p3b[1]};
        }
    }
    __syncthreads();
    const int r = w * 16 + cl;
    bf16x8 x1[KS], x2[KS], x3[KS];
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) {
        float f[8];
        const int k0 = 32 * s2 + 8 * kq;
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = k0 + j < fin ? xs[r * fin + k0 + j] : 0.f;
        split3_8(f, x1[s2], x2[s2], x3[s2]);
    }
    f32x4 acc[NT], cor[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = cor[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int o = (16 * t + cl) * WSB + 32 * s2 + 8 * kq;
            const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(wsb + o);
            const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(wsb + BN * WSB + o);
            const bf16x8 b3 = *reinterpret_cast<const bf16x8*>(wsb + 2 * BN * WSB + o);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1, x1[s2], acc[t], 0, 0, 0);
            cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b2, x1[s2], cor[t], 0, 0, 0);
            cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1, x2[s2], cor[t], 0, 0, 0);
            cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b3, x1[s2], cor[t], 0, 0, 0);
            cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b2, x2[s2], cor[t], 0, 0, 0);
            cor[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1, x3[s2], cor[t], 0, 0, 0);
        }
    const int row = row0 + r;
    const int hl = F / 4;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int c0 = 16 * t + 4 * kq;
        f32x4 bb, p2v;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool ok = c0 + i < HF;
            bb[i] = ok ? bW[min(c0 + i, HF - 1)] : 0.f;
            p2v[i] = ok ? a2[min(c0 + i, HF - 1)] : 0.f;
        }
        const f32x4 v = acc[t] + cor[t] + bb;
        float p2 = v.x * p2v.x + v.y * p2v.y + v.z * p2v.z + v.w * p2v.w;
        for (int o = 16; o < 16 * hl; o <<= 1) p2 += __shfl_xor(p2, o);
        if (row < n && c0 < HF) {
            const int g = c0 / slice_w;
            st_wt4(Wh, (size_t)g * slice_stride + (size_t)row * slice_w + (c0 - g * slice_w), v);
            if ((kq & (hl - 1)) == 0)
                st_wt1(s_dst, (size_t)row * H + c0 / F, p2 + c2[min(c0 / F, H - 1)]);
        }
    }
}

// ---- harness -----------------------------------------------------------------
static float time_loop(hipStream_t st, int reps, auto&& body) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 5; ++i) body();
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(a, st));
    for (int i = 0; i < reps; ++i) body();
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms * 1e3f / reps;  // us per iteration
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 44906;
    const int fin = argc > 2 ? atoi(argv[2]) : 50;
    const int H = 8, F = 8, HF = 64, slices = 2, sw = HF / slices;
    const int reps = 200;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    float *x, *w, *b, *a1, *c1, *a2, *c2, *wh, *wh2, *sd, *sd2, *pol_out, *cp_out;
    const size_t nx = (size_t)n * fin, nwh = (size_t)n * HF;
    CK(hipMalloc(&x, nx * 4));
    CK(hipMalloc(&w, HF * fin * 4));
    CK(hipMalloc(&b, HF * 4));
    CK(hipMalloc(&a1, HF * 4));
    CK(hipMalloc(&a2, HF * 4));
    CK(hipMalloc(&c1, H * 4));
    CK(hipMalloc(&c2, H * 4));
    CK(hipMalloc(&wh, nwh * 4));
    CK(hipMalloc(&wh2, nwh * 4));
    CK(hipMalloc(&sd, (size_t)n * H * 4));
    CK(hipMalloc(&sd2, (size_t)n * H * 4));
    CK(hipMalloc(&pol_out, nwh * 4));
    CK(hipMalloc(&cp_out, (nwh + (size_t)n * H) * 4));
    {
        std::vector<float> h(nx);
        srand(1);
        auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
        for (auto& v : h) v = rnd();
        CK(hipMemcpy(x, h.data(), nx * 4, hipMemcpyHostToDevice));
        std::vector<float> hw(HF * fin);
        for (auto& v : hw) v = rnd() * 0.2f;
        CK(hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
        std::vector<float> hv(HF);
        for (auto* p : {b, a1, a2}) {
            for (auto& v : hv) v = rnd();
            CK(hipMemcpy(p, hv.data(), HF * 4, hipMemcpyHostToDevice));
        }
        for (auto* p : {c1, c2}) {
            for (int i = 0; i < H; ++i) hv[i] = rnd();
            CK(hipMemcpy(p, hv.data(), H * 4, hipMemcpyHostToDevice));
        }
    }
    const long tab4 = (long)nwh / 4;
    float* pol_tab = wh;  // the table pollute reads (wh: as the edge kernel does)
    auto pollute = [&] { k_pollute<<<2048, 256, 0, st>>>((const f32x4*)pol_tab, tab4, pol_out); };
    auto lib_to = [&](float* dst) {
        return [&, dst] {
            int rc = gat_project_sliced(x, n, fin, w, b, a1, c1, a2, c2, H, F, slices, dst, n,
                                        nullptr, 0, sd, st);
            if (rc) { fprintf(stderr, "gat_project_sliced rc=%d\n", rc); exit(1); }
        };
    };
    auto lib = lib_to(wh);
    const long in4 = (long)nx / 4, out4 = (long)(nwh + (size_t)n * H) / 4;
    auto copy_rw = [&] { k_copy<<<2048, 256, 0, st>>>((const f32x4*)x, in4, cp_out, out4, 1); };
    auto copy_r = [&] { k_copy<<<2048, 256, 0, st>>>((const f32x4*)x, in4, cp_out, 0, 1); };
    auto copy_w = [&] { k_copy<<<2048, 256, 0, st>>>((const f32x4*)x, 0, cp_out, out4, 1); };
    auto copy_rw_wh = [&] { k_copy<<<2048, 256, 0, st>>>((const f32x4*)x, in4, wh, tab4, 1); };
    auto copy_0 = [&] { k_copy<<<1, 256, 0, st>>>((const f32x4*)x, 0, cp_out, 0, 1); };
    const int tiles = (n + 15) / 16;
    auto rt = [&](int wgs) {
        return [&, wgs] {
            if (fin % 2 == 0)
                k_proj_rt<4, 2, 2><<<wgs, 256, 0, st>>>(x, n, fin, w, b, a1, c1, a2, c2, H, F, HF,
                                                         wh2, sw, (long)n * sw, sd2);
            else
                k_proj_rt<4, 2, 1><<<wgs, 256, 0, st>>>(x, n, fin, w, b, a1, c1, a2, c2, H, F, HF,
                                                         wh2, sw, (long)n * sw, sd2);
        };
    };
    // parity of the prototype against the library
    lib();
    k_proj_wk3<4, 2><<<(n + 63) / 64, 256, (3 * 64 * 72) * 2 + (64 * 64 + 64) * 4, st>>>(x, n, fin, w, b, a2, c2, H, F, HF, wh2, sw, (long)n * sw, sd2);
    CK(hipStreamSynchronize(st));
    {
        std::vector<float> A(nwh), B(nwh), SA((size_t)n * H), SB((size_t)n * H);
        CK(hipMemcpy(A.data(), wh, nwh * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(B.data(), wh2, nwh * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(SA.data(), sd, SA.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(SB.data(), sd2, SB.size() * 4, hipMemcpyDeviceToHost));
        double dw = 0, ds = 0, mw = 0;
        for (size_t i = 0; i < nwh; ++i) {
            dw = fmax(dw, fabs(A[i] - B[i]));
            mw = fmax(mw, fabs(A[i]));
        }
        for (size_t i = 0; i < SA.size(); ++i) ds = fmax(ds, fabs(SA[i] - SB[i]));
        printf("{\"parity\": {\"max_abs_wh\": %.3g, \"max_abs_diff_wh\": %.3g, "
               "\"max_abs_diff_sdst\": %.3g},\n", mw, dw, ds);
    }
    const double mb_in = nx * 4 / 1e6, mb_out = (nwh + (size_t)n * H) * 4 / 1e6;
    printf(" \"shape\": {\"n\": %d, \"fin\": %d, \"x_MB\": %.2f, \"out_MB\": %.2f},\n", n, fin,
           mb_in, mb_out);
    const float t_pol = time_loop(st, reps, pollute);
    printf(" \"pollute_us\": %.2f,\n \"results\": {\n", t_pol);
    struct V { const char* name; std::function<void()> f; };
    std::vector<V> vs = {{"empty_1wg", copy_0}, {"copy_read_x", copy_r}, {"copy_write_out", copy_w},
                         {"copy_rw", copy_rw}, {"copy_rw_into_polluted_table", copy_rw_wh},
                         {"lib_project", lib}, {"lib_project_other_table", lib_to(wh2)}};
    const int rt_grids[] = {256, 512, 768, (tiles + 3) / 4};
    for (int wgs : rt_grids) vs.push_back({nullptr, rt(wgs)});
#define RT_MODE(M, NM)                                                                          \
    vs.push_back({NM, [&] {                                                                     \
        k_proj_rt<4, 2, 2, M><<<512, 256, 0, st>>>(x, n, fin, w, b, a1, c1, a2, c2, H, F, HF,   \
                                                   wh2, sw, (long)n * sw, sd2);                \
    }});
    RT_MODE(1, "rt512_no_sdst") RT_MODE(2, "rt512_no_wh") RT_MODE(3, "rt512_no_stores")
    RT_MODE(4, "rt512_plain_stores") RT_MODE(8, "rt512_no_mfma") RT_MODE(11, "rt512_loads_only")
    RT_MODE(16, "rt512_lds_epilogue")
    const size_t wk3_lds = (3 * 64 * 72) * 2 + (64 * 64 + 64) * 4;
    vs.push_back({"wk3", [&] { k_proj_wk3<4, 2><<<(n + 63) / 64, 256, wk3_lds, st>>>(x, n, fin, w, b, a2, c2, H, F, HF, wh2, sw, (long)n * sw, sd2); }});
    vs.push_back({"rt256_lds_epilogue", [&] { k_proj_rt<4, 2, 2, 16><<<256, 256, 0, st>>>(x, n, fin, w, b, a1, c1, a2, c2, H, F, HF, wh2, sw, (long)n * sw, sd2); }});
    vs.push_back({"rt768_lds_epilogue", [&] { k_proj_rt<4, 2, 2, 16><<<768, 256, 0, st>>>(x, n, fin, w, b, a1, c1, a2, c2, H, F, HF, wh2, sw, (long)n * sw, sd2); }});
    vs.push_back({"rt384_lds_epilogue", [&] { k_proj_rt<4, 2, 2, 16><<<384, 256, 0, st>>>(x, n, fin, w, b, a1, c1, a2, c2, H, F, HF, wh2, sw, (long)n * sw, sd2); }});
#undef RT_MODE
    for (size_t i = 0; i < vs.size(); ++i) {
        char nm[64];
        const char* name = vs[i].name;
        if (!name) {
            snprintf(nm, sizeof nm, "rt_wg%d", rt_grids[i - 7]);
            name = nm;
        }
        auto f = vs[i].f;
        const float alone = time_loop(st, reps, f);
        const float pair = time_loop(st, reps, [&] { pollute(); f(); });
        printf("  \"%s\": {\"alone_us\": %.2f, \"after_pollute_us\": %.2f}%s\n", name, alone,
               pair - t_pol, i + 1 < vs.size() ? "," : "");
    }
    // store policies for a copy into the table pollute read
    {
        auto run = [&](const char* nm, auto kern) {
            const float tp = time_loop(st, reps, pollute);
            const float pair = time_loop(st, reps, [&] { pollute(); kern(); });
            printf("  ,\"%s\": {\"after_pollute_us\": %.2f}\n", nm, pair - tp);
        };
        run("copy_into_table_plain", [&] { k_copy_aux<0><<<2048, 256, 0, st>>>((const f32x4*)x, in4, wh, tab4); });
        run("copy_into_table_sc1", [&] { k_copy_aux<16><<<2048, 256, 0, st>>>((const f32x4*)x, in4, wh, tab4); });
        run("copy_into_table_nt", [&] { k_copy_aux<2><<<2048, 256, 0, st>>>((const f32x4*)x, in4, wh, tab4); });
        run("copy_into_table_sc0", [&] { k_copy_aux<1><<<2048, 256, 0, st>>>((const f32x4*)x, in4, wh, tab4); });
        run("copy_into_table_sc0sc1", [&] { k_copy_aux<17><<<2048, 256, 0, st>>>((const f32x4*)x, in4, wh, tab4); });
        run("copy_into_table_sc1nt", [&] { k_copy_aux<18><<<2048, 256, 0, st>>>((const f32x4*)x, in4, wh, tab4); });
        run("copy_into_table_sc0sc1nt", [&] { k_copy_aux<19><<<2048, 256, 0, st>>>((const f32x4*)x, in4, wh, tab4); });
        // pollute's table loads with a policy, then the sc1 copy into that table
        auto run2 = [&](const char* nm, auto pol) {
            const float tp = time_loop(st, reps, pol);
            const float pair = time_loop(st, reps, [&] { pol(); k_copy_aux<16><<<2048, 256, 0, st>>>((const f32x4*)x, in4, wh, tab4); });
            const float pair2 = time_loop(st, reps, [&] { pol(); lib(); });
            printf("  ,\"%s\": {\"pollute_us\": %.2f, \"copy_after_us\": %.2f, \"lib_after_us\": %.2f}\n", nm, tp, pair - tp, pair2 - tp);
        };
        run2("pollute_loads_plain", [&] { k_pollute_aux<0><<<2048, 256, 0, st>>>(wh, tab4, pol_out); });
        run2("pollute_loads_nt", [&] { k_pollute_aux<2><<<2048, 256, 0, st>>>(wh, tab4, pol_out); });
        run2("pollute_loads_sc0", [&] { k_pollute_aux<1><<<2048, 256, 0, st>>>(wh, tab4, pol_out); });
        run2("pollute_loads_sc1", [&] { k_pollute_aux<16><<<2048, 256, 0, st>>>(wh, tab4, pol_out); });
        run2("pollute_loads_sc0sc1", [&] { k_pollute_aux<17><<<2048, 256, 0, st>>>(wh, tab4, pol_out); });
        // ping-pong: two tables alternate (lib writes T0, pollute reads T0, lib writes T1, ...)
        {
            auto lib1 = lib_to(wh2);
            auto pol1 = [&] { k_pollute<<<2048, 256, 0, st>>>((const f32x4*)wh2, tab4, pol_out); };
            const float tp = time_loop(st, reps, pollute);
            const float pp = time_loop(st, reps, [&] { lib(); pollute(); lib1(); pol1(); });
            const float same = time_loop(st, reps, [&] { lib(); pollute(); });
            printf("  ,\"pingpong\": {\"lib_after_us\": %.2f, \"same_table_lib_after_us\": %.2f}\n", pp / 2 - tp, same - tp);
        }
    }
    // the library projection behind a pollute kernel that reads ANOTHER table
    pol_tab = wh2;
    {
        const float tp = time_loop(st, reps, pollute);
        const float pair = time_loop(st, reps, [&] { pollute(); lib(); });
        printf("  ,\"lib_project_pollute_reads_other\": {\"after_pollute_us\": %.2f}\n", pair - tp);
    }
    printf(" }\n}\n");
    return 0;
}
