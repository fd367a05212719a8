// Backward source-pass gather probe (Reddit scale): how fast can a per-source
// walk over the out-edges (CSC, targets ascending) gather a per-target record
// in different table layouts?  Memory behaviour only: each lane accumulates a
// product of what it loads, no softmax recompute.  Standalone HIP program.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bwd_gather_probe.hip -o tools/bwd_gather_probe
//   tools/bwd_gather_probe [n] [deg]
//
// Layouts (per target i, HF = 64 columns of g plus (s_dst, lse, delta, 0) for 8 heads):
//   row    [n][96] floats (384 B): the library's table today; 16 lanes per source
//          row, each loads its g float4 and its head's record float4 per edge
//   planes4 [4][n][32] floats (128 B): plane p = g columns 16p..16p+15 and the
//          records of heads 2p, 2p+1; workgroup b works on plane b % 4 (so an XCD
//          gathers from one plane under round-robin placement); 8 lanes per
//          (source, plane): 4 g lanes, 2 record lanes, 2 idle
//   planes2 [2][n][64] floats (256 B): plane p = g columns 32p..32p+31 + the
//          records of heads 4p..4p+3; 16 lanes per (source, plane)
#include <hip/hip_runtime.h>

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

// stratified ascending targets: t_k = floor((k + u) n / deg), u ~ U[0,1) hashed
__global__ void k_make_csc(int n, int deg, int* __restrict__ ptr, int* __restrict__ dst) {
    const long i = blockIdx.x * 256L + threadIdx.x;
    const long total = (long)n * deg;
    if (i <= n && i < (long)n + 1) {
        if (i <= n) ptr[i] = (int)(i * deg);
    }
    for (long e = i; e < total; e += (long)gridDim.x * 256) {
        const int k = (int)(e % deg);
        unsigned h = (unsigned)e * 2654435761u;
        h ^= h >> 15;
        h *= 0x2c1b3c6du;
        h ^= h >> 12;
        const float u = (h & 0xFFFFFF) / 16777216.f;
        int t = (int)(((double)k + u) * n / deg);
        dst[e] = t < n ? t : n - 1;
    }
}

template <int G, int U>
__global__ __launch_bounds__(256) void k_row(const int* __restrict__ ptr, const int* __restrict__ dst,
                                             int n, const float* __restrict__ T, int ld,
                                             float* __restrict__ out) {
    const int lane = threadIdx.x & 63, c = lane & (G - 1), gbase = lane & ~(G - 1);
    const int groups = gridDim.x * 256 / G;
    const int gid = (blockIdx.x * 256 + threadIdx.x) / G;
    const int h = c / 2;  // head of this lane's g float4 (F = 8)
    f32x4 tot = {0.f, 0.f, 0.f, 0.f};
    for (int j = gid; j < n; j += groups) {
        const int b0 = ptr[j], b1 = ptr[j + 1];
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int b = b0; b < b1; b += U) {
            int iv = dst[min(b + c, b1 - 1)];
            f32x4 gv[U], tv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = __shfl(iv, gbase + (u % G));
                const float* tr = T + (size_t)i * ld;
                gv[u] = *reinterpret_cast<const f32x4*>(tr + 4 * c);
                tv[u] = *reinterpret_cast<const f32x4*>(tr + 64 + 4 * h);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc += (b + u < b1 ? tv[u].x : 0.f) * gv[u];
        }
        tot += acc;
    }
    if (tot.x == 1234.5f) out[blockIdx.x] = tot.y;  // keep the loads
}

// planes: workgroup b on plane b % P, PL lanes per (source, plane) each loading
// one float4 of the plane row (lanes past the row's float4s idle)
template <int P, int PL, int U, int W4, int RS>
__global__ __launch_bounds__(256) void k_planes(const int* __restrict__ ptr,
                                                const int* __restrict__ dst, int n,
                                                const float* __restrict__ T,
                                                float* __restrict__ out) {
    const int lane = threadIdx.x & 63, c = lane & (PL - 1), gbase = lane & ~(PL - 1);
    const int pl = blockIdx.x % P;
    const int blk = blockIdx.x / P;
    const int groups = (gridDim.x / P) * 256 / PL;
    const int gid = (blk * 256 + threadIdx.x) / PL;
    const float* Tp = T + (size_t)pl * n * RS;
    const bool act = c < W4;
    f32x4 tot = {0.f, 0.f, 0.f, 0.f};
    for (int j = gid; j < n; j += groups) {
        const int b0 = ptr[j], b1 = ptr[j + 1];
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int b = b0; b < b1; b += U) {
            int iv[(U + PL - 1) / PL];
#pragma unroll
            for (int t = 0; t < (U + PL - 1) / PL; ++t) iv[t] = dst[min(b + c + t * PL, b1 - 1)];
            f32x4 gv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = __shfl(iv[u / PL], gbase + (u % PL));
                gv[u] = act ? *reinterpret_cast<const f32x4*>(Tp + (size_t)i * RS + 4 * c)
                            : f32x4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc += (b + u < b1 ? 1.f : 0.f) * gv[u];
        }
        tot += acc;
    }
    if (tot.x == 1234.5f) out[blockIdx.x] = tot.y;
}

static float time_it(hipStream_t st, int reps, auto&& f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(a, st));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 232965;
    const int deg = argc > 2 ? atoi(argv[2]) : 493;
    const long nnz = (long)n * deg;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    int *ptr, *dst;
    float *T, *out;
    CK(hipMalloc(&ptr, (n + 1) * 4));
    CK(hipMalloc(&dst, nnz * 4));
    CK(hipMalloc(&T, (size_t)n * 96 * 4 + (size_t)n * 128 * 4));
    CK(hipMalloc(&out, 1 << 20));
    k_make_csc<<<4096, 256, 0, st>>>(n, deg, ptr, dst);
    CK(hipMemsetAsync(T, 0, (size_t)n * (96 + 128) * 4, st));
    CK(hipStreamSynchronize(st));
    const double edges = (double)nnz;
    printf("{\"n\": %d, \"deg\": %d, \"nnz\": %ld, \"results\": {\n", n, deg, nnz);
    const int reps = 5;
    auto rep = [&](const char* name, float ms, double bytes_per_edge, bool last = false) {
        printf("  \"%s\": {\"ms\": %.3f, \"G_edges_per_s\": %.1f, \"line_TBps\": %.2f}%s\n", name,
               ms, edges / (ms * 1e-3) / 1e9, edges * bytes_per_edge / (ms * 1e-3) / 1e12,
               last ? "" : ",");
    };
    for (int waves : {16384, 32768, 65536}) {
        const int grid = waves / 4;
        char nm[64];
        snprintf(nm, sizeof nm, "row384_U16_w%d", waves);
        rep(nm, time_it(st, reps, [&] { k_row<16, 16><<<grid, 256, 0, st>>>(ptr, dst, n, T, 96, out); }), 384);
    }
    for (int waves : {16384, 65536}) {
        const int grid = (waves / 4 / 4) * 4;
        char nm[64];
        snprintf(nm, sizeof nm, "planes4_128B_U16_w%d", waves);
        rep(nm, time_it(st, reps, [&] { k_planes<4, 8, 16, 6, 32><<<grid, 256, 0, st>>>(ptr, dst, n, T, out); }), 512);
        snprintf(nm, sizeof nm, "planes4_128B_U8_w%d", waves);
        rep(nm, time_it(st, reps, [&] { k_planes<4, 8, 8, 6, 32><<<grid, 256, 0, st>>>(ptr, dst, n, T, out); }), 512);
        snprintf(nm, sizeof nm, "planes2_256B_U16_w%d", waves);
        rep(nm, time_it(st, reps, [&] { k_planes<2, 16, 16, 12, 64><<<(waves / 4 / 2) * 2, 256, 0, st>>>(ptr, dst, n, T, out); }), 512);
        snprintf(nm, sizeof nm, "planes1_384B_U16_w%d", waves);
        rep(nm, time_it(st, reps, [&] { k_planes<1, 32, 16, 24, 96><<<waves / 4, 256, 0, st>>>(ptr, dst, n, T, out); }), 384);
    }
    // the forward's table for comparison: 2 planes of 128-B rows (32 floats)
    rep("fwd_planes2_128B_U16_w32768", time_it(st, reps, [&] { k_planes<2, 8, 16, 8, 32><<<8192, 256, 0, st>>>(ptr, dst, n, T, out); }), 256, true);
    printf("}}\n");
    return 0;
}
