// MI355X GAT graph builds: CSR by target with self-loops (GAT.py:38, 53) and
// its CSC transpose for the backward pass.

#include "gat_common.h"
#include <rocprim/device/device_radix_sort.hpp>

namespace {

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

// rows by descending in-degree, ties by ascending row id (the order of a
// stable descending sort): one 64-bit key ((2^kd - 1 - degree) << kb | row),
// sorted ascending by the same u64 radix sort as the CSR keys (one sort
// instantiation in the library instead of three)
__global__ void k_degree_keys(const int* __restrict__ rowptr, int n, unsigned kb, unsigned kd,
                              unsigned long long* __restrict__ keys) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    const unsigned long long top = (1ull << kd) - 1ull;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride) {
        const unsigned long long deg = (unsigned long long)(rowptr[i + 1] - rowptr[i]);
        keys[i] = ((top - deg) << kb) | (unsigned long long)i;
    }
}

__global__ void k_low_bits(const unsigned long long* __restrict__ keys, long long n, unsigned kb,
                           int* __restrict__ out) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    const unsigned long long mask = (1ull << kb) - 1ull;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = (int)(keys[i] & mask);
}

// ---------------------------------------------------------------------------
// CSC (edges grouped by SOURCE) over the CSR's edge positions, for the
// backward pass: the gradient of a source row gathers over its out-edges.
//   csc_ptr[j]       first CSC slot of source j
//   csc_dst[c]       target row of the edge in CSC slot c
//   csc_eid[c]       CSR position of the edge in CSC slot c
//   csr_to_csc[k]    CSC slot of CSR position k
// Built by one radix sort of 64-bit keys (col[k] << kn | k), k < 2^kn: within
// a source, edges keep CSR order, so every reduction over them is
// deterministic.  The target row of a CSR position is found by binary search
// in rowptr (L2-resident) rather than gathered from a per-edge array.
// ---------------------------------------------------------------------------
__global__ void k_csc_keys(long long nnz, const int* __restrict__ col, unsigned kn,
                           unsigned long long* __restrict__ keys) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < nnz; k += stride)
        keys[k] = ((unsigned long long)(unsigned)col[k] << kn) | (unsigned long long)k;
}

__global__ void k_csc_ptr(const unsigned long long* __restrict__ sorted_keys, long long nnz,
                          int n, unsigned kn, int* __restrict__ csc_ptr) {
    const long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (j > n) return;
    long long lo = 0, hi = nnz;
    while (lo < hi) {
        const long long mid = (lo + hi) >> 1;
        if ((long long)(sorted_keys[mid] >> kn) < j) lo = mid + 1; else hi = mid;
    }
    csc_ptr[j] = (int)lo;
}

__global__ void k_csc_fill(const unsigned long long* __restrict__ sorted_keys, unsigned kn,
                           const int* __restrict__ rowptr, int n, long long nnz,
                           int* __restrict__ csc_eid, int* __restrict__ csc_dst,
                           int* __restrict__ csr_to_csc) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    const unsigned long long mask = (1ull << kn) - 1ull;
    for (long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x; c < nnz; c += stride) {
        const int k = (int)(sorted_keys[c] & mask);
        if (csc_eid != nullptr) csc_eid[c] = k;
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

// bits to hold values in [0, n)
unsigned key_bits(long long n) {
    unsigned b = 1;
    while (b < 40 && (1ll << b) < n) ++b;
    return b;
}

// temporary storage of the library's one radix sort (u64 keys) for `count`
// keys of `bits` bits
size_t key_sort_tmp_bytes(long long count, unsigned bits) {
    size_t tmp = 0;
    unsigned long long* k = nullptr;
    const hipError_t e = rocprim::radix_sort_keys(nullptr, tmp, k, k, (size_t)(count > 0 ? count : 1),
                                                  0u, bits);
    return e == hipSuccess ? tmp : 0;
}

// ---------------------------------------------------------------------------
// Staggered row walks (gat_csr_rotate, gat_csr_schedule, gat_csc_rotate).  A row's
// entries are sorted ascending (sources in a CSR row, targets in a CSC row);
// the walk for schedule position p starts at the row's first entry >= start(p)
// and wraps around: out[o + j] = in[b + (j + rot) mod d], rot = the number of
// entries below start (a binary search).  One wave per row, lanes over its
// entries (coalesced reads and writes).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int count_below(const int* __restrict__ v, int d, int x) {
    int lo = 0, hi = d;  // first index with v[i] >= x
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (v[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ int walk_start(long long p, long long stride, int n) {
    return stride > 0 ? (int)((p * stride) % (long long)n) : 0;
}

// rows at schedule positions p (row order[p], or p), written at out_off[p]
// (the scheduled copy) or at the row's own CSR offset (out_off == nullptr)
__global__ void k_rotate_rows(const int* __restrict__ rowptr, const int* __restrict__ in,
                              const int* __restrict__ order, int n, long long stride,
                              int max_degree, const int* __restrict__ out_off,
                              int* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const long long waves = (long long)gridDim.x * (blockDim.x >> 6);
    for (long long p = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); p < n;
         p += waves) {
        const int r = order != nullptr ? order[p] : (int)p;
        const int b = rowptr[r], d = rowptr[r + 1] - b;
        const int o = out_off != nullptr ? out_off[p] : b;
        const bool turn = stride > 0 && (max_degree <= 0 || d <= max_degree);
        const int rot = turn ? count_below(in + b, d, walk_start(p, stride, n)) : 0;
        for (int j = lane; j < d; j += 64) {
            int jj = j + rot;
            if (jj >= d) jj -= d;
            out[o + j] = in[b + jj];
        }
    }
}

// the scheduled copy's segment bounds: deg_in_order[p] = degree of row order[p]
__global__ void k_sched_degrees(const int* __restrict__ rowptr, const int* __restrict__ order,
                                int n, int* __restrict__ deg) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) {
        const int r = order[p];
        deg[p] = rowptr[r + 1] - rowptr[r];
    }
}

__global__ void k_sched_ends(const int* __restrict__ seg_b, int n, int* __restrict__ seg_e) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) seg_e[p] += seg_b[p];  // seg_e held the degrees
}

// a CSC row (source j, schedule position j) rotated: targets and edge ids
// together, and the CSR-position -> CSC-slot map re-inverted
__global__ void k_rotate_csc(const int* __restrict__ ptr, const int* __restrict__ dst,
                             const int* __restrict__ eid, int n, long long stride,
                             int* __restrict__ out_dst, int* __restrict__ out_eid,
                             int* __restrict__ out_c2c) {
    const int lane = threadIdx.x & 63;
    const long long waves = (long long)gridDim.x * (blockDim.x >> 6);
    for (long long j = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); j < n;
         j += waves) {
        const int b = ptr[j], d = ptr[j + 1] - b;
        const int rot = stride > 0 ? count_below(dst + b, d, walk_start(j, stride, n)) : 0;
        for (int t = lane; t < d; t += 64) {
            int tt = t + rot;
            if (tt >= d) tt -= d;
            out_dst[b + t] = dst[b + tt];
            if (eid != nullptr) {
                const int k = eid[b + tt];
                out_eid[b + t] = k;
                if (out_c2c != nullptr) out_c2c[k] = b + t;
            }
        }
    }
}

// exclusive scan of n ints (the scheduled copy's segment starts): 1024 per
// block (256 threads x 4), the block totals scanned by one block with a carry,
// then added back.  Small (n = the node count) and run once per graph.
__device__ __forceinline__ int block_excl_scan256(int v, int* sh) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        const int a = t >= off ? sh[t - off] : 0;
        __syncthreads();
        sh[t] += a;
        __syncthreads();
    }
    const int incl = sh[t];
    __syncthreads();
    return incl - v;
}

__global__ __launch_bounds__(256) void k_scan_blocks(const int* __restrict__ in, int n,
                                                     int* __restrict__ out,
                                                     int* __restrict__ block_sums) {
    __shared__ int sh[256];
    const long long base = (long long)blockIdx.x * 1024 + threadIdx.x * 4;
    int v[4], t = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[i] = base + i < n ? in[base + i] : 0;
        t += v[i];
    }
    int run = block_excl_scan256(t, sh);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (base + i < n) out[base + i] = run;
        run += v[i];
    }
    if (threadIdx.x == 255) block_sums[blockIdx.x] = run;
}

__global__ __launch_bounds__(256) void k_scan_sums(int* __restrict__ sums, int nb) {
    __shared__ int sh[256];
    int carry = 0;
    for (int c0 = 0; c0 < nb; c0 += 256) {
        const int i = c0 + threadIdx.x;
        const int v = i < nb ? sums[i] : 0;
        const int ex = block_excl_scan256(v, sh);
        if (i < nb) sums[i] = carry + ex;
        if (threadIdx.x == 255) sh[0] = ex + v;  // this chunk's total
        __syncthreads();
        carry += sh[0];
        __syncthreads();
    }
}

__global__ void k_scan_add(int* __restrict__ out, int n, const int* __restrict__ sums) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] += sums[i / 1024];
}

inline unsigned row_grid(long long rows) {  // 4 waves per block, capped grid
    const long long blocks = (rows + 3) / 4;
    return (unsigned)(blocks < 65536 ? (blocks > 0 ? blocks : 1) : 65536);
}

}  // namespace

extern "C" {

int gat_csr_workspace_size(long long num_edges, int num_nodes, size_t* bytes) {
    if (num_edges < 0 || num_nodes < 0 || bytes == nullptr) return GAT_EINVAL;
    if (num_edges + num_nodes > 0x7fffffffLL) return GAT_EUNSUPPORTED;
    long long nnz = num_edges + num_nodes;
    if (nnz < 1) nnz = 1;
    const int n = num_nodes > 0 ? num_nodes : 1;
    const unsigned kb = key_bits(n), kd = key_bits(nnz + 1);
    const size_t t1 = key_sort_tmp_bytes(nnz, 2 * kb);
    const size_t t2 = key_sort_tmp_bytes(n, kb + kd);
    const size_t a = 2 * align_up((size_t)nnz * 8);  // keys in / out (edges)
    const size_t b = 2 * align_up((size_t)n * 8);    // keys in / out (rows)
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
    const unsigned kb = key_bits(num_nodes), kd = key_bits(nnz + 1);
    const size_t keyb = align_up((size_t)nnz * 8);
    const size_t nb = align_up((size_t)num_nodes * 8);
    const size_t region = 2 * keyb > 2 * nb ? 2 * keyb : 2 * nb;
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
        // rows by descending in-degree (ties by row id): the edge kernel's schedule
        unsigned long long* dkeys_in = (unsigned long long*)ws;
        unsigned long long* dkeys_out = (unsigned long long*)(ws + nb);
        hipLaunchKernelGGL(k_degree_keys, dim3(grid_for(num_nodes, 256)), dim3(256), 0, st,
                           rowptr, num_nodes, kb, kd, dkeys_in);
        tmp_bytes = need - region;
        e = rocprim::radix_sort_keys(tmp, tmp_bytes, dkeys_in, dkeys_out, (size_t)num_nodes, 0u,
                                     kb + kd, st);
        if (e != hipSuccess) return status_of(e);
        hipLaunchKernelGGL(k_low_bits, dim3(grid_for(num_nodes, 256)), dim3(256), 0, st,
                           dkeys_out, (long long)num_nodes, kb, row_order);
    }
    return status_of(hipGetLastError());
}

int gat_csc_workspace_size(long long nnz, int num_nodes, size_t* bytes) {
    if (nnz < 0 || num_nodes < 0 || bytes == nullptr) return GAT_EINVAL;
    if (nnz > 0x7fffffffLL) return GAT_EUNSUPPORTED;
    const size_t eb = align_up((size_t)(nnz > 0 ? nnz : 1) * 8);
    const unsigned bits = key_bits(num_nodes > 0 ? num_nodes : 1) + key_bits(nnz > 0 ? nnz : 1);
    *bytes = 2 * eb + align_up(key_sort_tmp_bytes(nnz, bits));
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
    const size_t eb = align_up((size_t)nnz * 8);
    const unsigned kn = key_bits(nnz), bits = key_bits(num_nodes) + kn;
    char* ws = (char*)workspace;
    unsigned long long* keys_in = (unsigned long long*)ws;
    unsigned long long* keys_out = (unsigned long long*)(ws + eb);
    void* tmp = ws + 2 * eb;
    hipLaunchKernelGGL(k_csc_keys, dim3(grid_for(nnz, 256)), dim3(256), 0, st, nnz, col, kn,
                       keys_in);
    size_t tmp_bytes = need - 2 * eb;
    hipError_t e = rocprim::radix_sort_keys(tmp, tmp_bytes, keys_in, keys_out, (size_t)nnz, 0u,
                                            bits, st);
    if (e != hipSuccess) return status_of(e);
    hipLaunchKernelGGL(k_csc_ptr, dim3((num_nodes + 1 + 255) / 256), dim3(256), 0, st, keys_out,
                       nnz, num_nodes, kn, csc_ptr);
    hipLaunchKernelGGL(k_csc_fill, dim3(grid_for(nnz, 256)), dim3(256), 0, st, keys_out, kn,
                       rowptr, num_nodes, nnz, csc_eid, csc_dst, csr_to_csc);
    return status_of(hipGetLastError());
}

int gat_csr_rotate(const int* rowptr, const int* col, const int* row_order, int num_nodes,
                   int stride, int max_degree, int* out_col, void* stream) {
    if (num_nodes < 0 || stride < 0 || rowptr == nullptr || out_col == nullptr) return GAT_EINVAL;
    if (num_nodes == 0) return GAT_OK;
    if (row_order == nullptr) return GAT_EINVAL;  // (col, out_col: NULL with no entries)
    hipLaunchKernelGGL(k_rotate_rows, dim3(row_grid(num_nodes)), dim3(256), 0,
                       (hipStream_t)stream, rowptr, col, row_order, num_nodes, (long long)stride,
                       max_degree, nullptr, out_col);
    return status_of(hipGetLastError());
}

int gat_csr_schedule_workspace_size(int num_nodes, size_t* bytes) {
    if (num_nodes < 0 || bytes == nullptr) return GAT_EINVAL;
    const size_t nb = ((size_t)num_nodes + 1023) / 1024;  // block totals of the scan
    *bytes = align_up((nb > 0 ? nb : 1) * sizeof(int));
    return GAT_OK;
}

int gat_csr_schedule(const int* rowptr, const int* col, const int* row_order, int num_nodes,
                     int stagger, int* seg_begin, int* seg_end, int* out_col, void* workspace,
                     size_t workspace_bytes, void* stream) {
    if (num_nodes < 0 || stagger < 0) return GAT_EINVAL;
    size_t need = 0;
    int rc = gat_csr_schedule_workspace_size(num_nodes, &need);
    if (rc != GAT_OK) return rc;
    if (workspace_bytes < need) return GAT_EWORKSPACE;
    if (num_nodes == 0) return GAT_OK;
    if (rowptr == nullptr || row_order == nullptr || seg_begin == nullptr || seg_end == nullptr)
        return GAT_EINVAL;  // (col, out_col: NULL with no entries)
    hipStream_t st = (hipStream_t)stream;
    const unsigned g = (unsigned)((num_nodes + 255) / 256);
    hipLaunchKernelGGL(k_sched_degrees, dim3(g), dim3(256), 0, st, rowptr, row_order, num_nodes,
                       seg_end);
    const int nb = (num_nodes + 1023) / 1024;
    int* sums = (int*)workspace;
    hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(256), 0, st, seg_end, num_nodes, seg_begin,
                       sums);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(256), 0, st, sums, nb);
    hipLaunchKernelGGL(k_scan_add, dim3(g), dim3(256), 0, st, seg_begin, num_nodes, sums);
    hipLaunchKernelGGL(k_sched_ends, dim3(g), dim3(256), 0, st, seg_begin, num_nodes, seg_end);
    hipLaunchKernelGGL(k_rotate_rows, dim3(row_grid(num_nodes)), dim3(256), 0, st, rowptr, col,
                       row_order, num_nodes, (long long)stagger, 0, seg_begin, out_col);
    return status_of(hipGetLastError());
}

int gat_csc_rotate(const int* csc_ptr, const int* csc_dst, const int* csc_eid, int num_nodes,
                   int stride, int* out_dst, int* out_eid, int* out_csr_to_csc, void* stream) {
    if (num_nodes < 0 || stride < 0) return GAT_EINVAL;
    if (num_nodes == 0) return GAT_OK;
    if (csc_ptr == nullptr) return GAT_EINVAL;  // (csc_dst, out_dst: NULL with no entries)
    if ((csc_eid == nullptr) != (out_eid == nullptr)) return GAT_EINVAL;
    if (out_csr_to_csc != nullptr && csc_eid == nullptr) return GAT_EINVAL;
    hipLaunchKernelGGL(k_rotate_csc, dim3(row_grid(num_nodes)), dim3(256), 0, (hipStream_t)stream,
                       csc_ptr, csc_dst, csc_eid, num_nodes, (long long)stride, out_dst, out_eid,
                       out_csr_to_csc);
    return status_of(hipGetLastError());
}

}  // extern "C"
