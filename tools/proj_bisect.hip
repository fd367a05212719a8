// PPI projection bisection: the library's k_project_wk (via gat_project_sliced,
// the eval forward's 2-plane table) against probe kernels with its grid (64
// rows per 256-thread workgroup) that add its pieces one at a time:
//   copy       each workgroup streams its 64 x rows in (coalesced float4) and
//              64 Wh rows + s_dst out: the one-pass floor of the grid
//   lds        x and W tiles staged through LDS as k_project_wk does (one
//              barrier), each lane sums its fragments (VALU), direct stores
//   mfma       lds + the fp32 MFMA loop of k_project_wk (13 k-steps x 4 tiles)
//   mfma_direct_loads  the same MFMAs on fragments each lane loads from global
//              memory itself (x rows, W from L1/L2): no LDS, no barrier
//   mfma_wave_lds_x_direct_w  x rows staged per wave in its own LDS region
//              (coalesced, no workgroup barrier), W fragments from L1/L2
//   mfma_wave_lds_x_fragment_w  the same with W pre-arranged in fragment order
//              (16 coalesced float4 loads per lane)
// Timed in interleaved rounds.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/proj_bisect.hip \
//       -Latmlgraphattentionnetworks_amd -lgat_amd \
//       -Wl,-rpath,'$ORIGIN/../atmlgraphattentionnetworks_amd' -o tools/proj_bisect
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <random>
#include <vector>

#include "../include/gat_amd.h"

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int FIN = 50, HF = 64, BM = 64, PW = 32, H = 8;

// MODE 0 copy, 1 lds, 2 mfma
template <int MODE>
__global__ __launch_bounds__(256) void k_probe(const float* __restrict__ X, int n,
                                               const float* __restrict__ W,
                                               float* __restrict__ Wh, float* __restrict__ s_dst,
                                               const f32x4* __restrict__ Wf) {
    __shared__ __attribute__((aligned(16))) float smem[BM * FIN + HF * FIN + 8];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int cl = lane & 15, kq = lane >> 4;
    const int row0 = blockIdx.x * BM;
    const int rows = min(BM, n - row0);
    const float* xg = X + (size_t)row0 * FIN;
    const int xc = rows * FIN, xc4 = xc & ~3;
    f32x4 xv[4];
    if constexpr (MODE < 3) {
#pragma unroll
        for (int it = 0; it < 4; ++it)
            xv[it] = *reinterpret_cast<const f32x4*>(xg + min(tid * 4 + it * 1024, max(xc4 - 4, 0)));
    }
    f32x4 acc[4];
    if constexpr (MODE == 3) {
        // no LDS: each lane loads its own A fragments (x[row][4s + kq]) and
        // B fragments (W[16t + cl][4s + kq]) from global memory / L1
        const int rrow = min(row0 + w * 16 + cl, n - 1);
        const float* xr = X + (size_t)rrow * FIN + kq;
        const float* wr = W + (size_t)cl * FIN + kq;
        float av[FIN / 4], bv[4][FIN / 4];
#pragma unroll
        for (int s = 0; s < FIN / 4; ++s) av[s] = xr[4 * s];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int s = 0; s < FIN / 4; ++s) bv[t][s] = wr[t * 16 * FIN + 4 * s];
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < FIN / 4; ++s)
#pragma unroll
            for (int t = 0; t < 4; ++t)
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(bv[t][s], av[s], acc[t], 0, 0, 0);
    } else if constexpr (MODE == 4 || MODE == 5) {
        // x: the wave's own 16 rows (one contiguous 3.2-KB run) staged in a
        // wave-private LDS region (no workgroup barrier); W fragments loaded by
        // each lane from global memory (L1/L2-resident 12.8 KB)
        float* Xw = smem + w * (16 * FIN + 4);
        const int wrow0 = row0 + w * 16;
        const int wrows = max(0, min(16, n - wrow0));
        const float* xw = X + (size_t)wrow0 * FIN;
        const int wc4 = (wrows * FIN) & ~3;
        f32x4 xq[4];
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int i = lane * 4 + it * 256;
            xq[it] = *reinterpret_cast<const f32x4*>(xw + min(i, max(wc4 - 4, 0)));
        }
        float bv[4][16];
        if constexpr (MODE == 5) {
            // W fragments pre-arranged [t][q][lane] float4 (s = 4q .. 4q+3):
            // 16 coalesced 1-KB wave loads
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const f32x4 v = Wf[(t * 4 + q) * 64 + lane];
                    bv[t][4 * q + 0] = v.x;
                    bv[t][4 * q + 1] = v.y;
                    bv[t][4 * q + 2] = v.z;
                    bv[t][4 * q + 3] = v.w;
                }
        } else {
            const float* wr = W + (size_t)cl * FIN + kq;
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int s = 0; s < FIN / 4; ++s) bv[t][s] = wr[t * 16 * FIN + 4 * s];
        }
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int i = lane * 4 + it * 256;
            if (i < wc4) *reinterpret_cast<f32x4*>(Xw + i) = xq[it];
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes landed
        __builtin_amdgcn_wave_barrier();
        const float* xa = Xw + cl * FIN + kq;
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < FIN / 4; ++s) {
            const float a = xa[4 * s];
#pragma unroll
            for (int t = 0; t < 4; ++t)
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(bv[t][s], a, acc[t], 0, 0, 0);
        }
    } else if constexpr (MODE == 0) {
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = xv[t];
    } else {
        float* Xs = smem;
        float* Ws = smem + BM * FIN;
        f32x4 wv[4];
#pragma unroll
        for (int it = 0; it < 4; ++it)
            wv[it] = *reinterpret_cast<const f32x4*>(W + min(tid * 4 + it * 1024, HF * FIN - 4));
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int i = tid * 4 + it * 1024;
            if (i < xc4) *reinterpret_cast<f32x4*>(Xs + i) = xv[it];
            if (i < HF * FIN) *reinterpret_cast<f32x4*>(Ws + i) = wv[it];
        }
        __syncthreads();
        const float* xa = Xs + (w * 16 + cl) * FIN + kq;
        const float* wb = Ws + cl * FIN + kq;
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int s = 0; s < FIN / 4; ++s) {
            const float a = xa[4 * s];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float b = wb[t * 16 * FIN + 4 * s];
                if constexpr (MODE == 2)
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, acc[t], 0, 0, 0);
                else
                    acc[t] += f32x4{a, b, a * b, a + b};
            }
        }
    }
    // direct stores as the library's epilogue: lane (cl, kq) has row cl of the
    // wave's 16, columns 16t + 4kq .. +4 of tile t; plane = column / 32
    const int row = row0 + w * 16 + cl;
    if (row < n) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int c0 = 16 * t + 4 * kq;
            const int g = c0 / PW;
            *reinterpret_cast<f32x4*>(Wh + (size_t)g * n * PW + (size_t)row * PW + (c0 - g * PW)) = acc[t];
        }
        if (kq < 2)
            *reinterpret_cast<f32x4*>(s_dst + (size_t)row * H + 4 * kq) = acc[0] + acc[1];
    }
}

int main() {
    const int n = 44906;
    std::mt19937 rng(3);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<float> x((size_t)n * FIN), w(HF * FIN), b(HF), a(HF), c(H);
    for (auto& v : x) v = nd(rng);
    for (auto& v : w) v = nd(rng) * 0.1f;
    for (auto& v : b) v = nd(rng) * 0.1f;
    for (auto& v : a) v = nd(rng) * 0.1f;
    for (auto& v : c) v = nd(rng) * 0.1f;
    float *d_x, *d_w, *d_b, *d_a, *d_c, *d_wh[2], *d_sd;
    CK(hipMalloc(&d_x, x.size() * 4));
    CK(hipMalloc(&d_w, w.size() * 4));
    CK(hipMalloc(&d_b, HF * 4));
    CK(hipMalloc(&d_a, HF * 4));
    CK(hipMalloc(&d_c, H * 4));
    for (int i = 0; i < 2; ++i) CK(hipMalloc(&d_wh[i], (size_t)n * HF * 4));
    CK(hipMalloc(&d_sd, (size_t)n * H * 4));
    CK(hipMemcpy(d_x, x.data(), x.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_w, w.data(), w.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_b, b.data(), HF * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_a, a.data(), HF * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_c, c.data(), H * 4, hipMemcpyHostToDevice));
    // W fragments pre-arranged for MODE 5: [t][q][lane] float4, lane (cl, kq)
    // gets W[16t + cl][4(4q + i) + kq], i = 0..3 (zero past fin)
    f32x4* d_wf;
    {
        std::vector<float> wf(4 * 4 * 64 * 4, 0.f);
        for (int t = 0; t < 4; ++t)
            for (int q = 0; q < 4; ++q)
                for (int l = 0; l < 64; ++l)
                    for (int i = 0; i < 4; ++i) {
                        const int k = 4 * (4 * q + i) + (l >> 4);
                        if (k < FIN) wf[(((t * 4 + q) * 64) + l) * 4 + i] = w[(16 * t + (l & 15)) * FIN + k];
                    }
        CK(hipMalloc(&d_wf, wf.size() * 4));
        CK(hipMemcpy(d_wf, wf.data(), wf.size() * 4, hipMemcpyHostToDevice));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int blocks = (n + BM - 1) / BM;
    std::vector<std::pair<const char*, std::function<void()>>> vars;
    vars.push_back({"library_k_project_wk", [&]() {
                        const int rc = gat_project_sliced(d_x, n, FIN, d_w, d_b, d_a, d_c, d_a, d_c,
                                                          H, 8, 2, d_wh[0], n, nullptr, H, d_sd,
                                                          nullptr);
                        if (rc != 0) {
                            fprintf(stderr, "library rc %d\n", rc);
                            exit(1);
                        }
                    }});
#define PROBE(NAME, MODE)                                                                       \
    vars.push_back({NAME, [&]() {                                                                \
                        hipLaunchKernelGGL((k_probe<MODE>), dim3(blocks), dim3(256), 0, 0, d_x, n, \
                                           d_w, d_wh[1], d_sd, d_wf);                            \
                    }});
    PROBE("copy", 0)
    PROBE("lds", 1)
    PROBE("mfma", 2)
    PROBE("mfma_direct_loads", 3)
    PROBE("mfma_wave_lds_x_direct_w", 4)
    PROBE("mfma_wave_lds_x_fragment_w", 5)
    std::vector<std::vector<float>> t(vars.size());
    for (auto& v : vars)
        for (int i = 0; i < 3; ++i) v.second();
    CK(hipDeviceSynchronize());
    for (int r = 0; r < 11; ++r)
        for (size_t k = 0; k < vars.size(); ++k) {
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < 20; ++i) vars[k].second();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[k].push_back(ms * 1e3f / 20);
        }
    printf("{\n \"shape\": {\"n\": %d, \"fin\": %d, \"hf\": %d, \"planes\": 2},\n", n, FIN, HF);
    printf(" \"note\": \"median us of 11 interleaved rounds of 20 back-to-back launches\"");
    for (size_t k = 0; k < vars.size(); ++k) {
        std::sort(t[k].begin(), t[k].end());
        printf(",\n \"%s_us\": %.2f", vars[k].first, t[k][5]);
    }
    printf("\n}\n");
    return 0;
}
