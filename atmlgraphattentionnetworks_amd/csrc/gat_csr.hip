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

}  // extern "C"
