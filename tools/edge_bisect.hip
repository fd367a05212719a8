// PPI edge-kernel bisection: the library's k_edge_grp over a PPI-shaped
// scheduled CSR (2 column planes, 8 lanes per 128-B plane row, 4 edges per
// chunk) against probe kernels that keep its memory pattern and add its
// pieces one at a time, to find where the time beyond the pure gathers goes
// (tools/line_gather_ceiling: 2-plane random 128-B gathers run at ~21 TB/s of
// requests; the library kernel at ~12.5 TB/s).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/edge_bisect.hip \
//       -Latmlgraphattentionnetworks_amd -lgat_amd \
//       -Wl,-rpath,'$ORIGIN/../atmlgraphattentionnetworks_amd' -o tools/edge_bisect
//   tools/edge_bisect                 (prints one JSON object)
//
// Probes (one lane group of 8 lanes per (row, plane), workgroup b on plane b % 2):
//   gather      row bounds by schedule position, col chunk, 4 gathers, sum
//   gather_pf   + the next chunk's col loads issued before this chunk's gathers
//   softmax     gather_pf + the fused score, LeakyReLU and online softmax
//   persist     softmax with each lane group walking several rows (grid-stride),
//               the next row's bounds loaded during the current row
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <functional>
#include <cstdlib>
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
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#ifdef SHAPE_ARXIV  // ogbn-arxiv shape: row-major 256-B rows, ~8 in-edges per row
constexpr int G = 16, U = 4, H = 8, F = 8, PW = 64, NP = 1, NROWS = 169343, DEG_TRIALS = 28;
#else  // PPI shape: two 128-B column planes, ~28 in-edges per row
constexpr int G = 8, U = 4, H = 8, F = 8, PW = 32, NP = 2, NROWS = 44906, DEG_TRIALS = 108;
#endif
constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ float pair_sum(float v) {  // sum over lanes l, l ^ 1
    return v + __shfl_xor(v, 1);
}

// MODE 0 gather, 1 gather_pf, 2 softmax, 3 gather_pf without the output store
// (kept only for a sentinel value), 4 gather_pf with hashed source ids (no col
// stream), 5 gathers with each row's col values loaded 8 chunks at a time,
// 6 = 5 + the softmax, 7 = 6 with write-through output stores, 8 = 6 with the
// target row read through the order array; PERSIST: grid-stride over positions
template <int MODE, bool PERSIST>
__global__ __launch_bounds__(256) void k_probe(const int* __restrict__ sb, const int* __restrict__ se,
                                               const int* __restrict__ col, int n,
                                               const float* __restrict__ wh, long long plane_stride,
                                               const float* __restrict__ a_src,
                                               const float* __restrict__ s_dst,
                                               float* __restrict__ out, const int* __restrict__ order) {
    const int lane = threadIdx.x & 63, c = lane & (G - 1), gbase = lane & ~(G - 1);
    const int sl = NP > 1 ? (int)(blockIdx.x & 1) : 0;
    const unsigned blk = NP > 1 ? blockIdx.x >> 1 : blockIdx.x;
    const unsigned nblk = NP > 1 ? gridDim.x >> 1 : gridDim.x;
    const int g_first = (int)((blk * 256u + threadIdx.x) / G);
    const int g_stride = PERSIST ? (int)(nblk * 256u / G) : n;
    const float* __restrict__ W = wh + sl * plane_stride + 4 * c;
    const int coff = sl * PW + 4 * c, h = coff / F;
    const f32x4 a4 = *reinterpret_cast<const f32x4*>(a_src + coff) * kLog2e;
    int pos = g_first;
    if (pos >= n) return;
    int e0 = sb[pos], e1 = se[pos];
    for (;;) {
        const int nxt = pos + g_stride;
        int ne0 = 0, ne1 = 0;
        if (PERSIST && nxt < n) {  // the next row's bounds, in flight during this row
            ne0 = sb[nxt];
            ne1 = se[nxt];
        }
        const float sd = s_dst[(size_t)pos * H + h] * kLog2e;
        float m = -INFINITY, l = 0.f;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (MODE >= 5) {
            // the row's col values for 8 chunks at a time, loaded at once: chunk t's
            // 4 ids sit in quad (t & 1) of the group, register t >> 1
            const int q = (c >> 2) & 1, pq = c & 3;
            // MODE 8: target row through the order array (identity here), as the
            // library's scheduled CSR reads s_dst[order[pos]]
            const int orow = MODE == 8 ? order[pos] : pos;
            const float sdr = MODE == 8 ? s_dst[(size_t)orow * H + h] * kLog2e : sd;
            for (int b0 = e0; b0 < e1; b0 += 8 * U) {
                int cr[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) cr[r] = col[min(b0 + U * (2 * r + q) + pq, e1 - 1)];
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const int k = b0 + U * t;
                    if (k >= e1) break;
                    int j[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) j[u] = __shfl(cr[t >> 1], gbase + 4 * (t & 1) + u);
                    f32x4 v[U];
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        v[u] = *reinterpret_cast<const f32x4*>(W + (size_t)j[u] * PW);
                    const int nk = min(U, e1 - k);
                    if constexpr (MODE == 5) {
#pragma unroll
                        for (int u = 0; u < U; ++u)
                            if (u < nk) acc += v[u];
                    } else {
                        float s[U];
                        float emax = -INFINITY;
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            float d = v[u].x * a4.x + v[u].y * a4.y + v[u].z * a4.z + v[u].w * a4.w;
                            d = pair_sum(d);
                            const float z = sdr + d;
                            s[u] = u < nk ? fmaxf(z, z * 0.2f) : -INFINITY;
                            emax = fmaxf(emax, s[u]);
                        }
                        const float mn = fmaxf(m, emax);
                        const float sc = __builtin_amdgcn_exp2f(m - mn);
                        l *= sc;
                        acc *= sc;
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const float p = __builtin_amdgcn_exp2f(s[u] - mn);
                            l += p;
                            acc += p * v[u];
                        }
                        m = mn;
                    }
                }
            }
            if constexpr (MODE >= 6) acc *= 1.f / (l + 1e-16f);
            if constexpr (MODE == 7) {
                // write-through 16-B store, as the library's store_out4
                const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0x7FFFFFFF, 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc), rsrc,
                                                       (int)(((size_t)orow * 64 + coff) * 4), 0, 16);
            } else {
                *reinterpret_cast<f32x4*>(out + (size_t)orow * 64 + coff) = acc;
            }
            if (!PERSIST) break;
            pos = nxt;
            if (pos >= n) break;
            e0 = ne0;
            e1 = ne1;
            continue;
        }
        // lane c holds col slot (c & 3) of the chunk
        int cv = MODE == 4 ? (int)(((unsigned)(e0 + (c & 3)) * 2654435761u >> 7) % (unsigned)n)
                           : col[min(e0 + (c & 3), e1 - 1)];
        for (int k = e0; k < e1; k += U) {
            int cn = 0;
            if (MODE == 4)
                cn = (int)(((unsigned)(k + U + (c & 3)) * 2654435761u >> 7) % (unsigned)n);
            else if (MODE >= 1)
                cn = col[min(k + U + (c & 3), e1 - 1)];
            int j[U];
#pragma unroll
            for (int u = 0; u < U; ++u) j[u] = __shfl(cv, (lane & ~3) + u);
            f32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const f32x4*>(W + (size_t)j[u] * PW);
            const int nk = min(U, e1 - k);
            if (MODE != 2) {
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (u < nk) acc += v[u];
            } else {
                float s[U];
                float emax = -INFINITY;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    float d = v[u].x * a4.x + v[u].y * a4.y + v[u].z * a4.z + v[u].w * a4.w;
                    d = pair_sum(d);
                    const float z = sd + d;
                    s[u] = u < nk ? fmaxf(z, z * 0.2f) : -INFINITY;
                    emax = fmaxf(emax, s[u]);
                }
                const float mn = fmaxf(m, emax);
                const float sc = __builtin_amdgcn_exp2f(m - mn);
                l *= sc;
                acc *= sc;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const float p = __builtin_amdgcn_exp2f(s[u] - mn);
                    l += p;
                    acc += p * v[u];
                }
                m = mn;
            }
            if (MODE >= 1) cv = cn;
            else cv = col[min(k + U + (c & 3), e1 - 1)];
        }
        const float inv = MODE == 2 ? 1.f / (l + 1e-16f) : 1.f;
        if (MODE != 3 || acc.x == 12345.f)
            *reinterpret_cast<f32x4*>(out + (size_t)pos * 64 + coff) = acc * inv;
        if (!PERSIST) break;
        pos = nxt;
        if (pos >= n) break;
        e0 = ne0;
        e1 = ne1;
    }
    (void)gbase;
}

int main() {
    const int n = NROWS;
    std::mt19937 rng(5);
    std::vector<int> deg(n);
    long long E = 0;
    std::binomial_distribution<int> bd(DEG_TRIALS, 0.25);  // in-edges + the self-loop
    for (int i = 0; i < n; ++i) {
        deg[i] = 1 + bd(rng);
        E += deg[i];
    }
    std::sort(deg.begin(), deg.end(), std::greater<int>());  // schedule: descending degree
    std::vector<int> sb(n), se(n), col(E), order(n);
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
        std::vector<float> a(64), c(8, 0.1f), sd((size_t)n * 8), b(64, 0.f);
        for (auto& v : a) v = nd(rng) * 0.3f;
        for (auto& v : sd) v = nd(rng) * 0.3f;
        CK(hipMemcpy(d_a, a.data(), 64 * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_c, c.data(), 8 * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_sd, sd.data(), sd.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_bias, b.data(), 64 * 4, hipMemcpyHostToDevice));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const long long plane_stride = (long long)n * PW;
    // the same rows with their sources in random order (each row's multiset
    // unchanged), and fresh uniformly random sources (unsorted)
    int *d_colr, *d_colu;
    CK(hipMalloc(&d_colr, E * 4));
    CK(hipMalloc(&d_colu, E * 4));
    {
        std::vector<int> colr = col;
        for (int i = 0; i < n; ++i) std::shuffle(colr.begin() + sb[i], colr.begin() + se[i], rng);
        CK(hipMemcpy(d_colr, colr.data(), E * 4, hipMemcpyHostToDevice));
        std::vector<int> colu(E);
        for (auto& v : colu) v = ud(rng);
        CK(hipMemcpy(d_colu, colu.data(), E * 4, hipMemcpyHostToDevice));
    }
    const int blocks = ((n * G + 255) / 256) * NP;
    std::vector<std::pair<const char*, std::function<void()>>> vars;
    auto lib_on = [&](const int* cp) {
        return [=]() {
            const int rc = gat_edge_aggregate_seg(d_sb, d_se, 1, cp, d_order, 0, n, d_wh, PW, n, NP,
                                                  d_a, d_c, d_sd, H, F, 1, 0.2f, nullptr, nullptr,
                                                  0, 0, d_bias, d_out, (int)(E / n), nullptr);
            if (rc != 0) {
                fprintf(stderr, "library rc %d\n", rc);
                exit(1);
            }
        };
    };
    vars.push_back({"library_k_edge_grp", lib_on(d_col)});
#define PROBE(NAME, MODE, PERS, GRID, CP)                                                         \
    vars.push_back({NAME, [=]() {                                                                 \
                        hipLaunchKernelGGL((k_probe<MODE, PERS>), dim3(GRID), dim3(256), 0, 0,     \
                                           d_sb, d_se, CP, n, d_wh, plane_stride, d_a, d_sd,        \
                                           d_out, d_order);                                         \
                    }});
    PROBE("gather", 0, false, blocks, d_col)
    PROBE("gather_pf", 1, false, blocks, d_col)
    PROBE("softmax", 2, false, blocks, d_col)
    PROBE("persist_24w", 2, true, 1536, d_col)
    PROBE("gather_persist_32w", 1, true, 2048, d_col)
    PROBE("gather_pf_nostore", 3, false, blocks, d_col)
    PROBE("gather_pf_hashcol", 4, false, blocks, d_col)
    PROBE("gather_rowcol", 5, false, blocks, d_col)
    PROBE("softmax_rowcol", 6, false, blocks, d_col)
    PROBE("softmax_rowcol_wtstore", 7, false, blocks, d_col)
    PROBE("softmax_rowcol_order", 8, false, blocks, d_col)
    vars.push_back({"unsorted_library_k_edge_grp", lib_on(d_colr)});
    PROBE("unsorted_gather_pf", 1, false, blocks, d_colr)
    PROBE("fresh_random_gather_pf", 1, false, blocks, d_colu)
    // interleaved rounds: every variant timed once per round (20 launches), medians
    std::vector<std::vector<float>> t(vars.size());
    for (auto& v : vars)
        for (int i = 0; i < 3; ++i) v.second();
    CK(hipDeviceSynchronize());
    for (int r = 0; r < 11; ++r) {
        for (size_t k = 0; k < vars.size(); ++k) {
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < 20; ++i) vars[k].second();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[k].push_back(ms * 1e3f / 20);
        }
    }
    printf("{\n \"shape\": {\"n\": %d, \"E\": %lld, \"planes\": %d, \"G\": %d, \"U\": %d},\n",
           n, E, NP, G, U);
    printf(" \"note\": \"median us of 11 interleaved rounds of 20 launches each\",\n");
    for (size_t k = 0; k < vars.size(); ++k) {
        std::sort(t[k].begin(), t[k].end());
        printf(" \"%s_us\": %.2f,\n", vars[k].first, t[k][5]);
    }
    const double req = (double)E * 2 * 128;
    printf(" \"request_bytes\": %.0f\n}\n", req);
    return 0;
}
