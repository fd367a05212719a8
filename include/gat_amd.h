/*
 * gat_amd.h — C-ABI of the MI355X (gfx950) GAT attention-layer library
 * (libgat_amd.so, built from the HIP sources in atmlgraphattentionnetworks_amd/csrc).
 *
 * Drop-in boundary for the hot path of danieldritter/ATMLGraphAttentionNetworks:
 * GraphAttentionLayer.forward(x, edge_index), GAT.py:37-67, and the PyG calls it
 * makes.  The reference is pure Python (it has no FFI of its own); the host side
 * above this ABI is the Python module atmlgraphattentionnetworks_amd.GraphAttentionLayer,
 * which keeps the reference's constructor, attributes and state_dict, and binds
 * these symbols with ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - Every pointer is a DEVICE pointer owned by the caller; the library never
 *    allocates or frees (CSR build takes a caller workspace sized by
 *    gat_csr_workspace_size).
 *  - `stream` is a hipStream_t passed as void* (torch's current stream).
 *    All work is enqueued on it; nothing synchronises the host.
 *  - Return value: GAT_OK (0), a negative GAT_E* code for bad arguments, or a
 *    positive hipError_t from the launch.  No exceptions cross the ABI.
 *  - Stateless and reentrant; safe to call concurrently on different devices
 *    or streams.
 *  - fp32 everywhere for features; int32 CSR indices; int64 edge_index input
 *    (the reference's LongTensor).
 */
#ifndef GAT_AMD_H_
#define GAT_AMD_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GAT_ABI_VERSION 12

#define GAT_OK 0
#define GAT_EINVAL (-1)       /* malformed arguments (negative sizes, bad layout) */
#define GAT_EUNSUPPORTED (-2) /* shape outside the kernels' range (see limits)    */
#define GAT_EWORKSPACE (-3)   /* workspace smaller than gat_csr_workspace_size      */

#define GAT_MAX_HEADS 64 /* num_heads                    */

/* Score activations (the attention_relu module, GAT.py:30 / run_act_func_experiment.py:111) */
#define GAT_ACT_LEAKY_RELU 0   /* LeakyReLU(act_param), the reference default 0.2          */
#define GAT_ACT_LOG_SIGMOID 1  /* LogSigmoid                                                */
#define GAT_ACT_TANH 2         /* Tanh                                                      */
#define GAT_ACT_HEAD_SOFTMAX 3 /* Softmax(dim=1) on the [E', heads] scores: across heads    */
#define GAT_MAX_HF 256   /* num_heads * output_channels  */

/* ABI version of the loaded library (== GAT_ABI_VERSION). */
int gat_abi_version(void);

/*
 * Re-read the GAT_* kernel-choice environment variables (A/B knobs used by
 * tools/ and the tests; never needed for correct results).  The library reads
 * them once, at its first launch; this call takes a new snapshot.  Not safe
 * to call while another thread launches through the library.
 */
int gat_tuning_reload(void);

/*
 * Packed node-table layout for (heads, f): row stride `ld` floats and column
 * `s_off` where s_src starts, for callers that keep Wh and s_src in ONE buffer
 * (e.g. to all-gather both with a single collective): pass wh = table,
 * ld_wh = ld, s_src = table + s_off, ld_s = ld.  Row n =
 * [Wh[n] (heads*f) | 0-pad | s_src[n] (heads) | 0-pad], both parts 16-B aligned.
 */
int gat_table_layout(int heads, int f, int* ld, int* s_off);

/*
 * Dense head projection with fused attention scores.
 * Replaces GAT.py:42-52 (per head h: ws[h](x), attentions1[h](.), attentions2[h](.),
 * then stack/transpose).
 *   x      [n, fin]       row-major
 *   w      [heads*f, fin] = cat_h ws[h].weight          (GAT.py:20)
 *   b      [heads*f]      = cat_h ws[h].bias
 *   a_src  [heads*f]      = cat_h attentions1[h].weight  (GAT.py:21, source term)
 *   c_src  [heads]        = cat_h attentions1[h].bias
 *   a_dst, c_dst          = the same for attentions2     (GAT.py:22, target term)
 * Writes, for rows [0, n):
 *   wh     [n, ld_wh]  Wh = x W^T + b, head-major (column h*f + k): the
 *                      reference's stack/transpose [N,H,F] view (GAT.py:49-50)
 *                      made contiguous; columns [heads*f, round_up(heads*f, 4))
 *                      zeroed; ld_wh % 4 == 0, ld_wh >= round_up(heads*f, 4)
 *   s_src  [n, ld_s]   Wh_h . a_src_h + c_src_h   (ld_s >= heads); may be NULL
 *                      (not written): the fused-score edge kernels recompute
 *                      it from the Wh rows they gather
 *   s_dst  [n, heads]  Wh_h . a_dst_h + c_dst_h
 * Non-finite inputs: a row of x holding +/-Inf or NaN affects that row only;
 * every output the fp32 reference makes non-finite is non-finite here too, but
 * where the reference gives +/-Inf the split-bf16 kernels (fin > 64) may give
 * NaN (the exact bf16 split of an infinity is not defined).
 */
int gat_project(const float* x, int n, int fin, const float* w, const float* b,
                const float* a_src, const float* c_src, const float* a_dst, const float* c_dst,
                int heads, int f, float* wh, int ld_wh, float* s_src, int ld_s, float* s_dst,
                void* stream);

/*
 * Fused per-edge score + LeakyReLU + segmented softmax + attention-weighted
 * aggregation + concat/head-mean + bias.
 * Replaces GAT.py:53-67 (PyG propagate/__collect__, message, utils.softmax,
 * aggregate aggr='add') and GAT.py:54 (+ bias).
 *   rowptr/col   CSR by target (gat_csr_build); col holds source row ids into wh/s_src
 *   row_order    optional [rows] permutation of target rows (gat_csr_build's
 *                degree order); the kernel processes rows row_order[row_begin ..
 *                row_end) — or rows row_begin .. row_end when NULL.  Only the
 *                schedule changes; every row's result is the same.
 *   wh           as written by gat_project (or an all-gathered copy)
 *   s_src, ld_s  the source term per node, as written by gat_project; may be NULL
 *                when a_src/c_src are given
 *   a_src, c_src the attentions1 parameters (gat_project's a_src/c_src); when given,
 *                the library may recompute s_src[j] from the gathered Wh[j] row
 *                instead of gathering it (same value up to fp32 rounding); may be
 *                NULL when s_src is given
 *   s_dst        [rows, heads], indexed by target row
 *   bias         [heads*f] if concat else [f]
 *   out          [rows, heads*f] if concat else [rows, f], indexed by target row
 *   lse          optional [rows, heads] = max + log(sum exp) per (row, head)
 *                (natural log; for the backward pass); may be NULL
 *   edges_per_row_hint  average in-degree (E'/rows) or 0 if unknown: picks the
 *                edge-chunk length, never affects results; GAT_HINT_LOCAL and
 *                GAT_HINT_SHORT may be OR'd in (every entry point taking a hint
 *                accepts them)
 * GAT_EUNSUPPORTED if s_src is NULL and the shape needs it (f % 4 != 0, or
 * f/4 not a power of two, or negative_slope outside [0, 1]).
 */
/* Scheduling hint bit: the graph's sources lie near their targets in node order
 * (block-diagonal batches of small graphs, kNN graphs), so rows processed
 * together share source rows.  Never affects results. */
#define GAT_HINT_LOCAL (1 << 30)
/* Scheduling hint bit (ABI 11): every row or segment the call walks has fewer
 * than 1024 in-edges, so the edge kernels may drop the Kahan-compensated sums
 * they keep for longer rows (which shorter rows never use).  Never affects
 * results when it holds. */
#define GAT_HINT_SHORT (1 << 29)

int gat_edge_aggregate(const int* rowptr, const int* col, const int* row_order, int row_begin,
                       int row_end, const float* wh, int ld_wh, const float* s_src, int ld_s,
                       const float* a_src, const float* c_src, const float* s_dst, int heads,
                       int f, int concat, float negative_slope, const float* bias, float* out,
                       float* lse, int edges_per_row_hint, void* stream);

/*
 * Sliced node table: the same projection (GAT.py:42-52) and edge aggregation
 * (GAT.py:53-67, +bias GAT.py:54) as gat_project / gat_edge_aggregate, with Wh
 * stored as `slices` column planes instead of row-major rows.  Plane g holds
 * columns [g*sw, (g+1)*sw) of every node, sw = heads*f/slices, as a row-major
 * [n_table, sw] array at wh + g*n_table*sw.  The edge kernel runs one plane per
 * workgroup (consecutive workgroups take consecutive planes), so with the
 * hardware's round-robin workgroup placement each XCD gathers from one plane,
 * which is 1/slices of the table and can stay resident in that XCD's L2.
 * Results equal the row-major entry points' (same arithmetic, same order).
 *
 * gat_project_sliced: as gat_project with ld_wh = sw (heads*f % slices == 0,
 *   sw % 4 == 0), writing rows [0, n) of planes of n_table >= n rows (wh may
 *   point at row r0 of the first plane: a rank's slot of a table the
 *   multi-GPU path all-gathers plane by plane).  s_src may be NULL (not
 *   written: the sliced edge kernel recomputes it).  GAT_EUNSUPPORTED for shapes whose projection
 *   kernel writes row-major only (fin > 64 needs f a power of two <= 16 and
 *   heads*f <= 64).
 * gat_edge_aggregate_sliced: concat only, LeakyReLU slope in [0, 1], sw % f == 0
 *   (whole heads per plane), f % 4 == 0 and f/4 a power of two; the source
 *   score is recomputed from the gathered plane row (a_src, c_src required).
 *   n_table = rows of each plane (the n passed to gat_project_sliced).
 */
int gat_project_sliced(const float* x, int n, int fin, const float* w, const float* b,
                       const float* a_src, const float* c_src, const float* a_dst,
                       const float* c_dst, int heads, int f, int slices, float* wh, int n_table,
                       float* s_src, int ld_s, float* s_dst, void* stream);
/*
 * gat_project_chunked (ABI 8): gat_project_sliced for the rows of one rank of
 * the multi-GPU node table, all of its all-gather chunks in ONE launch.  Rows
 * [c*chunk_rows, (c+1)*chunk_rows) of x (n rows in total) go to planes of
 * plane_rows rows starting at wh + c*chunk_stride floats (the table block of
 * chunk c; plane g at + g*plane_rows*sw); s_dst stays one contiguous [n, heads]
 * array; s_src is not written.  chunk_rows % 64 == 0, plane_rows >= chunk_rows,
 * chunk_stride >= slices*plane_rows*sw.  Replaces a per-chunk loop of
 * gat_project_sliced calls, each of which pays a whole block's latency (a
 * 9.7k-row chunk of the Reddit shape: ~30 us per launch for 1/3 of the rows).
 * Results are identical to those calls'.
 */
int gat_project_chunked(const float* x, int n, int fin, const float* w, const float* b,
                        const float* a_src, const float* c_src, const float* a_dst,
                        const float* c_dst, int heads, int f, int slices, float* wh,
                        int plane_rows, int chunk_rows, long long chunk_stride, float* s_dst,
                        void* stream);
/*
 * gat_project_ex (ABI 8): every projection layout in one entry point, with an
 * optional caller-owned workspace.  slices == 1: Wh row-major with ld_wh =
 * ld_wh_or_n_table (as gat_project; s_src [n, ld_s] or NULL).  slices
 * > 1: planes of n_table = ld_wh_or_n_table rows (as gat_project_sliced; s_src
 * may be NULL), and with chunk_rows > 0 the row chunks of gat_project_chunked
 * (chunk_stride floats apart).  workspace (16-B aligned, workspace_bytes >=
 * gat_project_workspace_size's bytes) lets the Fin > 128 kernel split W into
 * bf16 planes once per call instead of once per workgroup; NULL (or a smaller
 * buffer) runs the same kernels as the other entry points.  Results are
 * identical either way (the split is exact).
 * gat_project_workspace_size: the bytes for (fin, heads, f): 0 where the
 * projection takes no workspace (fin <= 128, or heads*f not in (16, 64]).
 */
int gat_project_workspace_size(int fin, int heads, int f, size_t* bytes);
int gat_project_ex(const float* x, int n, int fin, const float* w, const float* b,
                   const float* a_src, const float* c_src, const float* a_dst, const float* c_dst,
                   int heads, int f, int slices, float* wh, int ld_wh_or_n_table, float* s_src,
                   int ld_s, float* s_dst, int chunk_rows, long long chunk_stride,
                   void* workspace, size_t workspace_bytes, void* stream);
int gat_edge_aggregate_sliced(const int* rowptr, const int* col, const int* row_order,
                              int row_begin, int row_end, const float* wh, int n_table,
                              int slices, const float* a_src, const float* c_src,
                              const float* s_dst, int heads, int f, float negative_slope,
                              const float* bias, float* out, int edges_per_row_hint,
                              void* stream);

/*
 * Segmented edge aggregation: the same arithmetic as gat_edge_aggregate /
 * gat_edge_aggregate_sliced (GAT.py:53-67, + bias GAT.py:54), over a SEGMENT
 * of each row's in-edges, with the online-softmax state carried in memory.
 * Replaces nothing new in the reference: it is the same segmented softmax
 * (PyG utils.softmax, GAT.py:60) and scatter-add (aggr='add'), regrouped so
 * that (a) the multi-GPU forward can run one pass per all-gather chunk while
 * the next chunk is in flight, and (b) one very long row (a hub) can be cut
 * into segments that run in parallel and are combined by gat_edge_merge.
 *   seg_begin/seg_end  CSR positions: the segment of row i is
 *                [seg_begin[k], seg_end[k]) with k = i, or k = the schedule
 *                position (row_order index) when seg_by_pos != 0; state rows
 *                are indexed by the same k
 *   wh, ld_wh    slices == 1: row-major Wh-only table [.., ld_wh]
 *   wh, n_table  slices > 1: column planes as gat_edge_aggregate_sliced
 *                (plane g at wh + g * n_table * heads*f/slices)
 *   st_acc       [.., round_up(heads*f, 4)] un-normalised accumulators
 *   st_ml        [.., 2*heads]: per head, the running max (log2 units) then the sum
 *   flags        GAT_SEG_LOAD: start from the stored state (else from empty);
 *                GAT_SEG_STORE: every row stores its state (else writes the
 *                normalised row, + bias, to out)
 *   store_rows   with seg_by_pos and without GAT_SEG_STORE: the rows at schedule
 *                positions < store_rows store their state (the segments of
 *                split hub rows, scheduled first) and the others write their
 *                output; 0 otherwise
 * LeakyReLU with slope in [0, 1], f % 4 == 0, f/4 a power of two (the fused
 * source score: a_src, c_src required); concat or head mean (slices == 1).
 */
#define GAT_SEG_LOAD 1
#define GAT_SEG_STORE 2
int gat_edge_aggregate_seg(const int* seg_begin, const int* seg_end, int seg_by_pos,
                           const int* col, const int* row_order, int row_begin, int row_end,
                           const float* wh, int ld_wh, int n_table, int slices,
                           const float* a_src, const float* c_src, const float* s_dst, int heads,
                           int f, int concat, float negative_slope, float* st_acc, float* st_ml,
                           int flags, int store_rows, const float* bias, float* out,
                           int edges_per_row_hint, void* stream);

/*
 * Combine split hub rows: hub k (target row hub_rows[k]) has segment states
 * [seg_ptr[k], seg_ptr[k+1]) in st_acc / st_ml (written by
 * gat_edge_aggregate_seg with seg_by_pos and GAT_SEG_STORE).  Writes the row's
 * output (+ bias; concat or head mean), and optionally lse [.., heads] and
 * y_heads [.., heads*f] as gat_edge_aggregate_ex does.
 */
int gat_edge_merge(const int* hub_rows, const int* seg_ptr, int n_hub, const float* st_acc,
                   const float* st_ml, int heads, int f, int concat, const float* bias,
                   float* out, float* lse, float* y_heads, void* stream);

/*
 * gat_edge_merge_ex (ABI 9): as gat_edge_merge, with the segment states
 * addressed through seg_slot [seg_ptr[n_hub]] (segment j of the hub order at
 * state row seg_slot[j]; NULL: j itself).  For schedules that do not run a
 * hub's segments at adjacent positions (segments ordered by source range, so
 * that concurrently running segments gather from the same part of the
 * table).  The segments are combined in seg_ptr order either way, so the
 * output does not depend on the schedule.
 */
int gat_edge_merge_ex(const int* hub_rows, const int* seg_ptr, const int* seg_slot, int n_hub,
                      const float* st_acc, const float* st_ml, int heads, int f, int concat,
                      const float* bias, float* out, float* lse, float* y_heads, void* stream);

/*
 * The eval forward in one call: gat_project (slices == 1: row-major Wh at
 * ld = round_up(heads*f, 4), s_src [n, heads] if not NULL: the edge kernel
 * recomputes it, so callers pass NULL) or gat_project_sliced (slices > 1,
 * n_table = n, s_src unused), then gat_edge_aggregate_seg over a scheduled CSR
 * copy (seg_by_pos = 1: position p covers col[seg_begin[p] .. seg_end[p]) of
 * target row_order[p]; rows 0 .. n).  Replaces GAT.py:37-67 + GAT.py:54 for a
 * graph whose self-loops are already in the CSR.  Returns the first failing
 * call's status (GAT_EUNSUPPORTED from the projection launches nothing).
 * ABI 10: with 0 < fin <= 4 the projection is fused into the edge kernel (one
 * launch that gathers x rows and projects them in registers) wherever that
 * kernel takes the shape (heads*f of 32 or 64 in heads of 4 or 8 columns;
 * gat_layer_forward_fuses says which); wh, s_src and s_dst are then scratch
 * the call does not write.  Results are the two-launch path's up to fp32
 * rounding.
 */
int gat_layer_forward(const float* x, int n, int fin, const float* w, const float* b,
                      const float* a_src, const float* c_src, const float* a_dst,
                      const float* c_dst, int heads, int f, int slices, float* wh, float* s_src,
                      float* s_dst, const int* seg_begin, const int* seg_end, const int* col,
                      const int* row_order, int concat, float negative_slope, const float* bias,
                      float* out, int edges_per_row_hint, void* stream);

/*
 * gat_layer_forward_fuses (ABI 11): 1 when gat_layer_forward with these
 * arguments launches the fused small-Fin kernel (one launch, no Wh table),
 * 0 when it launches the projection and then the edge kernel.  A pure
 * function of the shape (and the library's knob snapshot); launches nothing.
 * For callers that account for the launches (the benchmark).
 */
int gat_layer_forward_fuses(int n, int fin, int heads, int f, int concat, float negative_slope);

/* Workspace bytes gat_csr_build needs for (num_edges, num_nodes). */
int gat_csr_workspace_size(long long num_edges, int num_nodes, size_t* bytes);

/*
 * COO -> CSR by target with the N self-loops appended.
 * Replaces torch_geometric.utils.add_self_loops (GAT.py:38) and the grouping of
 * edges by edge_index[1] that PyG's propagate/softmax/scatter perform (GAT.py:53,60).
 *   edge_index [2, num_edges] int64 (row 0 = source, row 1 = target)
 *   rowptr     [num_nodes + 1] int32,  col [num_edges + num_nodes] int32
 *   row_order  optional [num_nodes] int32: rows by descending in-degree (stable),
 *              the schedule gat_edge_aggregate takes; may be NULL
 * Within a row, sources ascend; equal (target, source) pairs — multi-edges, a
 * pre-existing self-loop beside the added one — keep cat([edge_index, loops])
 * order.  Existing self-loops and multi-edges are kept, as add_self_loops keeps
 * them.  (Only the summation order depends on the order within a row.)
 * *error_flag (device int) is set non-zero if any index is outside [0, num_nodes).
 */
int gat_csr_build(const long long* edge_index, long long num_edges, int num_nodes, int* rowptr,
                  int* col, int* row_order, void* workspace, size_t workspace_bytes,
                  int* error_flag, void* stream);

/* ---------------------------------------------------------------------------
 * Training: forward with attention dropout, and the backward pass.
 * Together these replace autograd through GAT.py:37-67 (the reference trains
 * the layer with loss.backward(), run_inductive.py / run_*_experiment.py).
 * ------------------------------------------------------------------------- */

/*
 * gat_edge_aggregate generalised: any score activation, attention dropout, and
 * the tensors the backward needs.  Replaces GAT.py:53-67 in training mode,
 * including GAT.py:61 (F.dropout on the attention coefficients), and the
 * activation experiment's layer (run_act_func_experiment.py:13-74).
 *   score_act  GAT_ACT_*; act_param is the LeakyReLU slope (ignored otherwise).
 *              Only LeakyReLU with slope in [0, 1] uses the lane-group kernel.
 *   dropout_p  in [0, 1]; coefficient (CSR position k, head h) is kept iff
 *              hash(seed, k*heads + h) >= round(dropout_p * 2^32) and then scaled
 *              by 1/(1 - dropout_p); the softmax denominator is not dropped.
 *              The mask is a pure function of (seed, k, h): the backward
 *              regenerates it from the same seed.
 *   seed_dev   optional device pointer: when set, the seed is read from it at run
 *              time (gat_dropout_seed_next), so a captured HIP graph draws a
 *              fresh mask on every replay; `seed` is then ignored.
 *   lse        optional [rows, heads]: log-sum-exp per (row, head)
 *   y_heads    optional [rows, heads*f]: per-head aggregation sum_k A_k Wh[j_k]
 *              (after dropout, before head mean and bias)
 * Other arguments as gat_edge_aggregate.
 */
int gat_edge_aggregate_ex(const int* rowptr, const int* col, const int* row_order, int row_begin,
                          int row_end, const float* wh, int ld_wh, const float* s_src, int ld_s,
                          const float* a_src, const float* c_src, const float* s_dst, int heads,
                          int f, int concat, int score_act, float act_param, float dropout_p,
                          unsigned long long seed, const unsigned long long* seed_dev,
                          const float* bias, float* out, float* lse, float* y_heads,
                          int edges_per_row_hint, void* stream);

/*
 * Training forward for the recompute backward (LeakyReLU with slope in [0, 1],
 * heads*f = 64 lane groups; GAT_EUNSUPPORTED otherwise -- then use
 * gat_edge_aggregate_ex + gat_bwd_targets).  As gat_edge_aggregate_ex with
 * score_act = GAT_ACT_LEAKY_RELU (s_src recomputed from the gathered Wh row), and
 * also the per-head kink sums the backward needs for dL/ds_dst:
 *   q_heads  [rows, heads*f]: Q[i,h] = sum_j A_ij L'(z_ij) Wh[j,h]
 *   r_heads  [rows, heads]:   R[i,h] = sum_j alpha_ij L'(z_ij)
 * with A the dropped and alpha the undropped coefficient, L' = 1 for z > 0 and
 * negative_slope otherwise.  lse and y_heads are required.  Replaces
 * GAT.py:53-67 in training mode; gat_bwd_table then replaces gat_bwd_targets.
 */
int gat_edge_aggregate_train(const int* rowptr, const int* col, const int* row_order,
                             int row_begin, int row_end, const float* wh, int ld_wh,
                             const float* a_src, const float* c_src, const float* s_dst,
                             int heads, int f, int concat, float negative_slope, float dropout_p,
                             unsigned long long seed, const unsigned long long* seed_dev,
                             const float* bias, float* out, float* lse, float* y_heads,
                             float* q_heads, float* r_heads, int edges_per_row_hint,
                             void* stream);

/*
 * Device-side dropout seeds: *seed_out = splitmix64(*counter); *counter += 1, on
 * `stream`.  Pass seed_out as `seed_dev` to the forward and to the backward of the
 * same call.  Inside a captured HIP graph each replay advances the counter, so
 * every replay draws a new mask.
 */
int gat_dropout_seed_next(unsigned long long* counter, unsigned long long* seed_out,
                          void* stream);

/* ---------------------------------------------------------------------------
 * Staggered row walks (ABI 12).  The edge entry points take a row's in-edges
 * in any order; walking each row from its first source at or after a start
 * that advances with the row's schedule position, and wrapping around, keeps
 * the rows that run together from all gathering the same table lines at once
 * (PPI edge kernel 3-4% faster, Reddit layer 2.6%).  All three are stateless
 * device passes on `stream` over rows whose entries ascend (gat_csr_build's
 * col, gat_csc_build's csc_dst); position p's start is (p * stride) mod N.
 * ------------------------------------------------------------------------- */

/* out_col [nnz]: col with row row_order[p] rotated for start (p * stride) mod N,
 * in CSR order (rowptr still indexes it).  The module's eval forward walks it at
 * stride 2 when rows average >= 64 in-edges.  stride = 0 copies col; rows of more
 * than max_degree entries (> 0) are copied unrotated (the module passes its hub
 * threshold: hub segments are scheduled by the first source they gather). */
int gat_csr_rotate(const int* rowptr, const int* col, const int* row_order, int num_nodes,
                   int stride, int max_degree, int* out_col, void* stream);

/* Workspace bytes gat_csr_schedule needs (a device scan). */
int gat_csr_schedule_workspace_size(int num_nodes, size_t* bytes);

/* The scheduled CSR copy: position p holds row row_order[p]'s entries at
 * [seg_begin[p], seg_end[p]) of out_col, positions contiguous in order (the
 * seg_begin/seg_end/col arguments of gat_edge_aggregate_seg and
 * gat_layer_forward with seg_by_pos = 1).  stagger = 0: each row as in col;
 * stagger = s > 0: rotated for start (p * s) mod N (the module uses 1 when rows
 * average 16-63 in-edges). */
int gat_csr_schedule(const int* rowptr, const int* col, const int* row_order, int num_nodes,
                     int stagger, int* seg_begin, int* seg_end, int* out_col, void* workspace,
                     size_t workspace_bytes, void* stream);

/* The CSC with source j's slots rotated for start (j * stride) mod N: csc_dst
 * and csc_eid (optional) permuted together, and out_csr_to_csc (optional,
 * needs csc_eid) the inverse of the permuted eid.  The module's backward uses
 * stride 8 when rows average >= 64 in-edges (gradients equal up to fp32
 * summation order).  In all three the entry arrays may be NULL when the graph
 * has no entries. */
int gat_csc_rotate(const int* csc_ptr, const int* csc_dst, const int* csc_eid, int num_nodes,
                   int stride, int* out_dst, int* out_eid, int* out_csr_to_csc, void* stream);

/* Workspace bytes gat_csc_build needs for nnz = E + N CSR entries. */
int gat_csc_workspace_size(long long nnz, int num_nodes, size_t* bytes);

/*
 * Transpose of the CSR (edges grouped by SOURCE), for the backward pass.
 *   rowptr/col  from gat_csr_build; nnz = rowptr[num_nodes]
 *   csc_ptr     [num_nodes + 1] int32: first CSC slot of each source node
 *   csc_dst     [nnz] int32: target row of the edge in each CSC slot
 *   csc_eid     optional [nnz] int32: CSR position of the edge in each CSC slot
 *               (gat_bwd_sources needs it when dropout is on)
 *   csr_to_csc  optional [nnz] int32: CSC slot of each CSR position
 *               (gat_edge_backward_rows needs it)
 * Within a source, slots follow CSR order (stable), so reductions over them are
 * deterministic.
 */
int gat_csc_build(const int* rowptr, const int* col, int num_nodes, long long nnz, int* csc_ptr,
                  int* csc_dst, int* csc_eid, int* csr_to_csc, void* workspace,
                  size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Backward, recompute form (LeakyReLU with slope in [0, 1], f % 4 == 0 and f/4 a
 * power of two; GAT_EUNSUPPORTED otherwise — then use gat_edge_backward_rows +
 * gat_src_backward).  No per-edge intermediate is stored: pass 2 recomputes each
 * edge's coefficient from a per-target table written by pass 1.
 * ------------------------------------------------------------------------- */

/* Row stride (floats) of the target table: round_up(ldg, 4) + 4*heads,
 * ldg = heads*f if concat else f. */
int gat_bwd_table_layout(int heads, int f, int concat, int* ld_t);

/*
 * Pass 1, per TARGET row: dL/ds_dst and the target table
 *   table[i] = [grad_out[i] (ldg) | pad | per head (s_dst, lse, delta, 0)],
 * delta = dy_h . y_h.  Inputs as gat_edge_backward_rows (a_src/c_src required).
 */
int gat_bwd_targets(const int* rowptr, const int* col, const int* row_order, int row_begin,
                    int row_end, const float* wh, int ld_wh, const float* a_src,
                    const float* c_src, const float* s_dst, const float* lse,
                    const float* y_heads, const float* grad_out, int heads, int f, int concat,
                    float negative_slope, float dropout_p, unsigned long long seed,
                    const unsigned long long* seed_dev, float* ds_dst, float* table, int ld_t,
                    int edges_per_row_hint, void* stream);

/*
 * Pass 1 without an edge loop, after gat_edge_aggregate_train: per TARGET row
 *   ds_dst[i,h] = dy_h . q_heads[i,h] - delta_h r_heads[i,h],  delta_h = dy_h . y_h
 * (the same sum gat_bwd_targets walks the in-edges for) and the same target
 * table as gat_bwd_targets.  All nodes, rows in node order.
 */
int gat_bwd_table(const float* s_dst, const float* lse, const float* y_heads,
                  const float* q_heads, const float* r_heads, const float* grad_out,
                  int num_nodes, int heads, int f, int concat, float* ds_dst, float* table,
                  int ld_t, void* stream);

/* Number of partial rows gat_bwd_sources writes for this shape (a multiple of 4). */
int gat_bwd_sources_parts(int num_nodes, int heads, int f, int* num_parts);

/*
 * Pass 2, per SOURCE row (over the CSC): dwh (as gat_src_backward) and the
 * partials [num_parts, 3*heads*f + 2*heads + ldg] in gat_src_backward's layout.
 *   table, ld_t   from gat_bwd_targets; ds_dst from gat_bwd_targets
 *   csc_eid       required when dropout_p > 0 (the mask is keyed on CSR positions)
 *   num_parts     from gat_bwd_sources_parts
 */
int gat_bwd_sources(const int* csc_ptr, const int* csc_dst, const int* csc_eid, int num_nodes,
                    const float* wh, int ld_wh, const float* table, int ld_t,
                    const float* ds_dst, const float* a_src, const float* c_src,
                    const float* a_dst, int heads, int f, int concat, float negative_slope,
                    float dropout_p, unsigned long long seed, const unsigned long long* seed_dev,
                    float* dwh, int ld_dwh, float* partials, int num_parts,
                    int edges_per_row_hint, void* stream);

/*
 * Backward pass 1, per TARGET row (softmax + LeakyReLU + dropout backward).
 *   grad_out   dL/d(layer output) [rows, heads*f] (concat) or [rows, f] (mean)
 *   lse, y_heads  as written by gat_edge_aggregate_ex (same activation, seed, dropout_p)
 *   s_src      as written by gat_project
 *   a_src, c_src  optional (the attentions1 parameters): with LeakyReLU and f/4 a
 *              power of two the library recomputes s_src from the gathered Wh row
 *   edges_per_row_hint  as for gat_edge_aggregate
 * Writes:
 *   ds_dst     [rows, heads]     dL/ds_dst
 *   az_csc     [nnz, heads, 2]   per edge and head, at the edge's CSC slot:
 *                                (A, dz) = (coefficient used in the forward, after
 *                                dropout; dL/d(s_dst[i] + s_src[j]))
 */
int gat_edge_backward_rows(const int* rowptr, const int* col, const int* row_order,
                           int row_begin, int row_end, const int* csr_to_csc, const float* wh,
                           int ld_wh, const float* s_src, int ld_s, const float* a_src,
                           const float* c_src, const float* s_dst, const float* lse,
                           const float* y_heads, const float* grad_out, int heads, int f,
                           int concat, int score_act, float act_param, float dropout_p,
                           unsigned long long seed, const unsigned long long* seed_dev,
                           float* ds_dst, float* az_csc, int edges_per_row_hint, void* stream);

/*
 * Backward pass 2, per SOURCE row: message backward plus the score terms.
 *   dwh[j]     = sum_{edges j->i} alpha * dy[i]  +  ds_src[j,h] a_src_h + ds_dst[j,h] a_dst_h
 *                ([num_nodes, ld_dwh], columns [0, heads*f)) = dL/dWh
 *   ds_src     optional [num_nodes, heads] = dL/ds_src
 *   partials   [num_parts, 3*heads*f + 2*heads + ldg] (ldg = heads*f if concat else f):
 *              per-part sums of [ds_src*Wh (da_src) | ds_dst*Wh (da_dst) | ds_src (dc_src) |
 *              ds_dst (dc_dst) | dwh rows (d of gat_project's b) | grad_out rows (dbias)];
 *              the caller sums them over parts (deterministic, no atomics).
 *   num_parts  >= 1; rows are strided over parts (a good value: min(num_nodes, 8192))
 */
int gat_src_backward(const int* csc_ptr, const int* csc_dst, int num_nodes, const float* wh,
                     int ld_wh, const float* grad_out, const float* az_csc,
                     const float* ds_dst, const float* a_src,
                     const float* a_dst, int heads, int f, int concat, float* dwh, int ld_dwh,
                     float* ds_src, float* partials, int num_parts, void* stream);

/* Workspace bytes gat_weight_grad needs. */
int gat_weight_grad_workspace_size(int num_nodes, int fin, int hf, size_t* bytes);

/*
 * Weight gradient of gat_project: dw[hf, fin] = dwh^T x (hf = heads*f), the
 * gradient of cat_h ws[h].weight (GAT.py:20).  Split-K fp32 MFMA over the node
 * rows with a fixed-order reduction (deterministic).
 *   x    [num_nodes, fin], dwh [num_nodes, ld_dwh] (gat_src_backward's dwh)
 */
int gat_weight_grad(const float* x, int num_nodes, int fin, const float* dwh, int ld_dwh, int hf,
                    float* dw, void* workspace, size_t workspace_bytes, void* stream);

/*
 * Input gradient of gat_project: dx[num_nodes, fin] = dwh[num_nodes, hf] w[hf, fin]
 * (the x side of cat_h ws[h], GAT.py:42-48; replaces the reference autograd's
 * mm through each head's Linear).  fp32 matrix cores, exact fp32 products;
 * every row's sum runs in one fixed order (deterministic).  hf <= 128
 * (GAT_EUNSUPPORTED beyond).
 *   dwh  [num_nodes, ld_dwh] (gat_bwd_sources' / gat_src_backward's dwh)
 *   w    the packed projection weight [hf, fin] (gat_project's w)
 *   dx   [num_nodes, ld_dx], ld_dx >= fin
 */
int gat_input_grad(const float* dwh, int ld_dwh, int num_nodes, int hf, const float* w,
                   int fin, float* dx, int ld_dx, void* stream);

/* Workspace bytes gat_sum_partials needs (0 for num_parts <= 256). */
int gat_sum_partials_workspace_size(int num_parts, long long width, size_t* bytes);

/*
 * out[e] = sum over p of partials[p * width + e] (fixed summation order, so
 * deterministic): reduces gat_src_backward's per-part partials.
 */
int gat_sum_partials(const float* partials, int num_parts, long long width, float* out,
                     void* workspace, size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GAT_AMD_H_ */
