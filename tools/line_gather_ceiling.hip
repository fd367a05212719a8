// Random-row gather ceilings on one MI355X: how fast can the chip gather
// uniformly random 128-B (or 256-B) rows of a table of a given size?  The edge
// kernel's gathers are such rows (a 128-B plane row per edge and plane at PPI
// and Reddit), so these rates are the ceilings its time is judged against:
// L2-resident (a table that fits an XCD's 4 MB L2), Infinity-Cache-resident
// (past L2, inside 256 MB) and HBM (past the Infinity Cache), and the PPI
// layout itself (2 column planes of 5.75 MB, workgroup b on plane b % 2, so an
// XCD gathers from one plane under round-robin placement).
// Memory behaviour only: every lane sums what it loads; no index array (row ids
// are hashed from the request number, so no index traffic).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/line_gather_ceiling.hip -o tools/line_gather_ceiling
//   tools/line_gather_ceiling            (prints one JSON object)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// G lanes (16 B each) per row; K rows in flight per lane group per iteration.
// Request r of plane p reads row hash(r) % rows of that plane.
template <int G, int K>
__global__ __launch_bounds__(256) void k_gather(const f32x4* __restrict__ tab, long long plane_f4,
                                                int planes, unsigned rows, long long requests,
                                                unsigned seed, float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int c = lane & (G - 1);
    const int p = planes > 1 ? (int)(blockIdx.x % (unsigned)planes) : 0;
    const unsigned blk = planes > 1 ? blockIdx.x / (unsigned)planes : blockIdx.x;
    const unsigned nblk = planes > 1 ? gridDim.x / (unsigned)planes : gridDim.x;
    const long long groups = (long long)nblk * (256 / G);
    const long long g0 = (long long)blk * (256 / G) + threadIdx.x / G;
    const f32x4* __restrict__ base = tab + (long long)p * plane_f4 + c;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    for (long long r = g0 * K; r < requests; r += groups * K) {
        f32x4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const unsigned row = hash32((unsigned)(r + k) ^ seed) % rows;
            v[k] = base[(long long)row * G];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) acc += v[k];
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

struct Case {
    const char* name;
    double table_mb;
    int row_bytes;
    int planes;
};

int main() {
    const Case cases[] = {
        {"l2_2MB_128B", 2.0, 128, 1},
        {"ppi_planes_2x5.75MB_128B", 11.5, 128, 2},
        {"table_11.5MB_128B", 11.5, 128, 1},
        {"reddit_planes_2x30MB_128B", 60.0, 128, 2},
        {"mall_64MB_128B", 64.0, 128, 1},
        {"mall_200MB_128B", 200.0, 128, 1},
        {"hbm_2GB_128B", 2048.0, 128, 1},
        {"l2_2MB_256B", 2.0, 256, 1},
        {"table_11.5MB_256B", 11.5, 256, 1},
        {"arxiv_43MB_256B", 43.0, 256, 1},
        {"mall_200MB_256B", 200.0, 256, 1},
    };
    const size_t max_bytes = (size_t)2048 << 20;
    f32x4* tab;
    CK(hipMalloc(&tab, max_bytes));
    CK(hipMemset(tab, 0, max_bytes));
    const int blocks = 256 * 8 * 2;  // 16 waves... per CU at most; grid-stride
    float* out;
    CK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(float)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("{\n \"note\": \"uniformly random rows, hashed ids, K = 8 rows in flight per lane group, "
           "%d blocks of 256; GB/s of requested row bytes (median of 5 launches)\",\n", blocks);
    const int ncases = sizeof(cases) / sizeof(cases[0]);
    for (int ci = 0; ci < ncases; ++ci) {
        const Case& cs = cases[ci];
        const size_t bytes = (size_t)(cs.table_mb * 1048576.0) / 256 * 256;
        const size_t plane_bytes = bytes / cs.planes / cs.row_bytes * cs.row_bytes;
        const unsigned rows = (unsigned)(plane_bytes / cs.row_bytes);
        const long long requests = 1LL << 24;  // per plane group: 16M rows
        const long long plane_f4 = (long long)(plane_bytes / 16);
        auto launch = [&](unsigned seed) {
            if (cs.row_bytes == 128)
                hipLaunchKernelGGL((k_gather<8, 8>), dim3(blocks), dim3(256), 0, 0, tab, plane_f4,
                                   cs.planes, rows, requests, seed, out);
            else
                hipLaunchKernelGGL((k_gather<16, 8>), dim3(blocks), dim3(256), 0, 0, tab,
                                   plane_f4, cs.planes, rows, requests, seed, out);
        };
        launch(1);
        CK(hipDeviceSynchronize());
        std::vector<float> ms;
        for (int it = 0; it < 5; ++it) {
            CK(hipEventRecord(e0, 0));
            launch(100 + it);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double med = ms[2];
        const double req_bytes = (double)requests * cs.planes * cs.row_bytes;
        printf(" \"%s\": {\"table_MB\": %.1f, \"row_B\": %d, \"planes\": %d, \"ms\": %.4f, "
               "\"GBps\": %.0f}%s\n",
               cs.name, cs.table_mb, cs.row_bytes, cs.planes, med, req_bytes / (med * 1e-3) / 1e9,
               ci + 1 < ncases ? "," : "");
        fflush(stdout);
    }
    // in-flight depth at the PPI plane layout: K rows per lane group with all
    // waves resident (B blocks of 4 waves, grid-stride), the edge kernel's
    // register budget at ~6 waves per SIMD holding K = 4 rows per lane group
    {
        const size_t bytes = (size_t)(11.5 * 1048576.0) / 256 * 256;
        const size_t plane_bytes = bytes / 2 / 128 * 128;
        const unsigned rows = (unsigned)(plane_bytes / 128);
        const long long requests = 1LL << 24;
        printf(",\n \"depth_ppi_planes\": {");
        const int bl[] = {512, 1024, 1536, 2048};
        bool first = true;
        for (int b : bl) {
            for (int K : {1, 2, 4, 8, 16}) {
                auto launch = [&](unsigned seed) {
                    switch (K) {
                        case 1: hipLaunchKernelGGL((k_gather<8, 1>), dim3(b), dim3(256), 0, 0, tab, (long long)(plane_bytes / 16), 2, rows, requests, seed, out); break;
                        case 2: hipLaunchKernelGGL((k_gather<8, 2>), dim3(b), dim3(256), 0, 0, tab, (long long)(plane_bytes / 16), 2, rows, requests, seed, out); break;
                        case 4: hipLaunchKernelGGL((k_gather<8, 4>), dim3(b), dim3(256), 0, 0, tab, (long long)(plane_bytes / 16), 2, rows, requests, seed, out); break;
                        case 8: hipLaunchKernelGGL((k_gather<8, 8>), dim3(b), dim3(256), 0, 0, tab, (long long)(plane_bytes / 16), 2, rows, requests, seed, out); break;
                        default: hipLaunchKernelGGL((k_gather<8, 16>), dim3(b), dim3(256), 0, 0, tab, (long long)(plane_bytes / 16), 2, rows, requests, seed, out); break;
                    }
                };
                launch(7);
                CK(hipDeviceSynchronize());
                std::vector<float> ms;
                for (int it = 0; it < 5; ++it) {
                    CK(hipEventRecord(e0, 0));
                    launch(200 + it);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float t;
                    CK(hipEventElapsedTime(&t, e0, e1));
                    ms.push_back(t);
                }
                std::sort(ms.begin(), ms.end());
                const double req = (double)requests * 2 * 128;
                printf("%s\n  \"waves_per_cu_%d_K%d\": %.0f", first ? "" : ",", b * 4 / 256, K,
                       req / (ms[2] * 1e-3) / 1e9);
                first = false;
                fflush(stdout);
            }
        }
        printf("\n }\n");
    }
    printf("}\n");
    CK(hipFree(tab));
    CK(hipFree(out));
    return 0;
}
