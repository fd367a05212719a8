// Reddit-shape bisection: the library's pipelined edge kernel (k_edge_grp,
// 2 column planes, 4 lanes x 2 float4 per 128-B plane row, 16 edges per chunk,
// gathers one chunk ahead, ids two chunks ahead) against a memory-only walk
// with the same loop structure (the gathered rows summed, no softmax), with
// and without its output stores.  Interleaved timing.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/edge_bisect_long.hip \
//       -Latmlgraphattentionnetworks_amd -lgat_amd \
//       -Wl,-rpath,'$ORIGIN/../atmlgraphattentionnetworks_amd' -o tools/edge_bisect_long
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

constexpr int G = 4, U = 16, H = 8, F = 8, PW = 32, NP = 2;

// MODE 0: walk + output store; 1: walk, no output store (sentinel only)
template <int MODE>
__global__ __launch_bounds__(256) void k_walk(const int* __restrict__ sb, const int* __restrict__ se,
                                              const int* __restrict__ col, int n,
                                              const float* __restrict__ wh, long long plane_stride,
                                              float* __restrict__ out) {
    const int lane = threadIdx.x & 63, c = lane & (G - 1), gbase = lane & ~(G - 1);
    const int sl = (int)(blockIdx.x & 1);
    const unsigned blk = blockIdx.x >> 1;
    const int pos = (int)((blk * 256u + threadIdx.x) / G);
    if (pos >= n) return;
    const int e0 = sb[pos], e1 = se[pos];
    const float* __restrict__ W = wh + sl * plane_stride + 8 * c;
    // a chunk's 16 ids: lane c holds ids c + 4t, t = 0..3
    auto ids = [&](int k, int (&cc)[4]) {
#pragma unroll
        for (int t = 0; t < 4; ++t) cc[t] = col[min(k + c + 4 * t, e1 - 1)];
    };
    auto fetch = [&](const int (&cc)[4], f32x4 (&v)[U][2]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = __shfl(cc[u / 4], gbase + (u % 4));
            const float* r = W + (size_t)j * PW;
            v[u][0] = *reinterpret_cast<const f32x4*>(r);
            v[u][1] = *reinterpret_cast<const f32x4*>(r + 4);
        }
    };
    f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    auto consume = [&](int k, f32x4 (&v)[U][2]) {
        const int nk = min(U, e1 - k);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (u < nk) {
                acc0 += v[u][0];
                acc1 += v[u][1];
            }
    };
    f32x4 va[U][2], vb[U][2];
    int ca[4], cb[4];
    ids(e0, ca);
    ids(e0 + U, cb);
    fetch(ca, va);
    for (int k = e0; k < e1; k += 2 * U) {
        int ca2[4], cb2[4];
        ids(k + 2 * U, ca2);
        fetch(cb, vb);
        consume(k, va);
        ids(k + 3 * U, cb2);
        fetch(ca2, va);
        if (k + U < e1) consume(k + U, vb);
#pragma unroll
        for (int t = 0; t < 4; ++t) cb[t] = cb2[t];
    }
    if (MODE == 0 || acc0.x == 12345.f) {
        float* o = out + (size_t)pos * 64 + sl * PW + 8 * c;
        *reinterpret_cast<f32x4*>(o) = acc0;
        *reinterpret_cast<f32x4*>(o + 4) = acc1;
    }
}

int main() {
    const int n = 232965;
    std::mt19937 rng(11);
    std::binomial_distribution<int> bd(1964, 0.25);  // ~491 in-edges + the self-loop
    std::vector<int> deg(n);
    long long E = 0;
    for (int i = 0; i < n; ++i) {
        deg[i] = 1 + bd(rng);
        E += deg[i];
    }
    std::sort(deg.begin(), deg.end(), std::greater<int>());
    std::vector<int> sb(n), se(n), order(n), col(E);
    std::uniform_int_distribution<int> ud(0, n - 1);
    long long p = 0;
    for (int i = 0; i < n; ++i) {
        sb[i] = (int)p;
        for (int k = 0; k < deg[i]; ++k) col[p + k] = ud(rng);
        std::sort(col.begin() + p, col.begin() + p + deg[i]);
        p += deg[i];
        se[i] = (int)p;
        order[i] = i;
    }
    int *d_sb, *d_se, *d_col, *d_order;
    float *d_wh, *d_a, *d_c, *d_sd, *d_bias, *d_out;
    CK(hipMalloc(&d_sb, n * 4));
    CK(hipMalloc(&d_se, n * 4));
    CK(hipMalloc(&d_order, n * 4));
    CK(hipMalloc(&d_col, E * 4));
    CK(hipMalloc(&d_wh, (size_t)n * 64 * 4));
    CK(hipMalloc(&d_a, 64 * 4));
    CK(hipMalloc(&d_c, 8 * 4));
    CK(hipMalloc(&d_sd, (size_t)n * 8 * 4));
    CK(hipMalloc(&d_bias, 64 * 4));
    CK(hipMalloc(&d_out, (size_t)n * 64 * 4));
    CK(hipMemcpy(d_sb, sb.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_se, se.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_order, order.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_col, col.data(), E * 4, hipMemcpyHostToDevice));
    {
        std::normal_distribution<float> nd(0.f, 1.f);
        std::vector<float> t((size_t)n * 64);
        for (auto& v : t) v = nd(rng) * 0.3f;
        CK(hipMemcpy(d_wh, t.data(), t.size() * 4, hipMemcpyHostToDevice));
        std::vector<float> a(64), cc(8, 0.1f), sd((size_t)n * 8), b(64, 0.f);
        for (auto& v : a) v = nd(rng) * 0.3f;
        for (auto& v : sd) v = nd(rng) * 0.3f;
        CK(hipMemcpy(d_a, a.data(), 64 * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_c, cc.data(), 8 * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_sd, sd.data(), sd.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_bias, b.data(), 64 * 4, hipMemcpyHostToDevice));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const long long plane_stride = (long long)n * PW;
    const int blocks = ((n * G + 255) / 256) * NP;
    std::vector<std::pair<const char*, std::function<void()>>> vars;
    vars.push_back({"library_k_edge_grp", [&]() {
                        const int rc = gat_edge_aggregate_seg(
                            d_sb, d_se, 1, d_col, d_order, 0, n, d_wh, PW, n, NP, d_a, d_c, d_sd, H,
                            F, 1, 0.2f, nullptr, nullptr, 0, 0, d_bias, d_out, (int)(E / n), nullptr);
                        if (rc != 0) {
                            fprintf(stderr, "library rc %d\n", rc);
                            exit(1);
                        }
                    }});
    vars.push_back({"walk", [&]() {
                        hipLaunchKernelGGL((k_walk<0>), dim3(blocks), dim3(256), 0, 0, d_sb, d_se,
                                           d_col, n, d_wh, plane_stride, d_out);
                    }});
    vars.push_back({"walk_nostore", [&]() {
                        hipLaunchKernelGGL((k_walk<1>), dim3(blocks), dim3(256), 0, 0, d_sb, d_se,
                                           d_col, n, d_wh, plane_stride, d_out);
                    }});
    std::vector<std::vector<float>> t(vars.size());
    for (auto& v : vars)
        for (int i = 0; i < 2; ++i) v.second();
    CK(hipDeviceSynchronize());
    for (int r = 0; r < 7; ++r)
        for (size_t k = 0; k < vars.size(); ++k) {
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < 3; ++i) vars[k].second();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[k].push_back(ms / 3);
        }
    printf("{\n \"shape\": {\"n\": %d, \"E\": %lld, \"planes\": 2, \"G\": %d, \"U\": %d},\n", n, E, G, U);
    printf(" \"note\": \"median ms of 7 interleaved rounds of 3 launches\"");
    for (size_t k = 0; k < vars.size(); ++k) {
        std::sort(t[k].begin(), t[k].end());
        printf(",\n \"%s_ms\": %.4f", vars[k].first, t[k][3]);
    }
    printf(",\n \"request_bytes\": %.0f\n}\n", (double)E * 2 * 128);
    return 0;
}
