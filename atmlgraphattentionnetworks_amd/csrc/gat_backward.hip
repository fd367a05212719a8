// MI355X GAT backward: recompute edge backward, source pass, weight and input
// gradients, dropout seeds (training path of GAT.py:37-67).

#include "gat_common.h"

#include <utility>

namespace {

// ---------------------------------------------------------------------------
// Backward, pass 1: one wave per TARGET row i (CSR), lanes over (edge, head)
// slots as in k_edge_fwd's score phase.  With dy = dL/dy_heads[i] (concat: the
// row of g; mean: g[i]/H for every head), y = the forward's normalised
// per-head aggregation and alpha = exp(e - lse):
//   delta_h   = dy_h . y_h
//   dA        = drop * (dy_h . Wh[j]_h)            (A = alpha * drop, drop = keep/(1-p) or 0)
//   de        = alpha * (dA - delta_h)              softmax backward
//   dz        = de * (z > 0 ? 1 : slope)            LeakyReLU backward
//   ds_dst[i] = sum_edges dz
// and stores (A, dz) per (edge, head) — interleaved, one 8H-byte record per
// edge — at the edge's CSC slot, so pass 2 reads them contiguously.
// Algorithmic bytes per edge: 4 (col) + 4 (csr_to_csc) + 4H (s_src) + 4HF (Wh
// row) + 8H (A, dz); per row: 4HF (g) + 4HF (y) + 8H (s_dst, lse) + 4H.
// ---------------------------------------------------------------------------
template <int HP>
__global__ __launch_bounds__(64) void k_edge_bwd_rows(
    const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ order,
    int row_begin, int row_end, const int* __restrict__ csr_to_csc,
    const float* __restrict__ Wh, int ld_wh, const float* __restrict__ Ss, int ld_s,
    const float* __restrict__ s_dst, const float* __restrict__ lse,
    const float* __restrict__ y_heads, const float* __restrict__ g, int H, int F, int HF,
    int concat, int act, float slope, DropArgs drop_arg, float* __restrict__ ds_dst,
    float2* __restrict__ az_out) {
    const DropArgs drop = resolve_drop(drop_arg);
    constexpr int C = (512 / HP) < kWave ? (512 / HP) : kWave;
    constexpr int R = C * HP / kWave;
    __shared__ float dy_s[GAT_MAX_HF];
    __shared__ float delta_s[HP];
    __shared__ int col_s[C];
    __shared__ int slot_s[C];

    const int lane = threadIdx.x;
    const int pos = row_begin + blockIdx.x;
    if (pos >= row_end) return;
    const int r = order != nullptr ? order[pos] : pos;
    const int e0 = rowptr[r], e1 = rowptr[r + 1];
    const float inv_h = 1.f / (float)H;
    for (int c = lane; c < HF; c += kWave)
        dy_s[c] = concat ? g[(size_t)r * HF + c] : g[(size_t)r * F + (c % F)] * inv_h;
    __syncthreads();
    if (lane < H) {
        float d = 0.f;
        const float* yr = y_heads + (size_t)r * HF + lane * F;
        for (int f = 0; f < F; ++f) d = fmaf(dy_s[lane * F + f], yr[f], d);
        delta_s[lane] = d;
    }
    __syncthreads();
    const int hs = lane & (HP - 1);
    const bool hs_ok = hs < H;
    const float sd = hs_ok ? s_dst[(size_t)r * H + hs] : 0.f;
    const float ls = hs_ok ? lse[(size_t)r * H + hs] : 0.f;
    const float dl = hs_ok ? delta_s[hs] : 0.f;
    const float* dyh = dy_s + (hs_ok ? hs : 0) * F;
    float dsd = 0.f;
    for (int base = e0; base < e1; base += C) {
        const int nk = min(C, e1 - base);
        if (lane < nk) {
            col_s[lane] = col[base + lane];
            slot_s[lane] = csr_to_csc[base + lane];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int k = (lane + kWave * q) / HP;
            const bool valid = k < nk && hs_ok;
            const int j = col_s[k < nk ? k : nk - 1];
            const float z = sd + Ss[(size_t)j * ld_s + (hs_ok ? hs : 0)];
            const bool hsm = act == GAT_ACT_HEAD_SOFTMAX;
            const float ev = hsm ? head_softmax<HP>(z, valid) : score_act(act, z, slope);
            float de = 0.f, a = 0.f, dm = 1.f;
            if (valid) {
                a = expf(ev - ls);
                const float* wr = Wh + (size_t)j * ld_wh + hs * F;
                float da = 0.f;
                for (int f = 0; f < F; ++f) da = fmaf(dyh[f], wr[f], da);
                if (drop.thresh != 0u) dm = drop_factor(drop, base + k, hs, H);
                de = a * (dm * da - dl);
            }
            float dz;
            if (hsm) {  // d softmax_h: e_h (de_h - sum_h' e_h' de_h')
                const float sum = head_sum<HP>(ev * de);
                dz = ev * (de - sum);
            } else {
                dz = de * score_act_grad(act, z, slope);
            }
            if (valid) {
                dsd += dz;
                az_out[(size_t)slot_s[k] * H + hs] = make_float2(a * dm, dz);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int off = HP; off < kWave; off <<= 1) dsd += __shfl_xor(dsd, off);
    if (lane < H) ds_dst[(size_t)r * H + lane] = dsd;
}

// ---------------------------------------------------------------------------
// Backward, pass 1, lane-group variant (LeakyReLU, F/4 a power of two): the
// k_edge_grp layout — G lanes per target row, each lane one float4 of one
// head — so each in-edge costs one coalesced Wh-row gather, the source score
// is recomputed from it (fused, as in the forward) and the two per-head dot
// products (s_src and dA = dy . Wh[j]) are DPP sums over the head's lanes.
// No LDS, no barriers; col and csr_to_csc loads software-pipelined.
// Same results as k_edge_bwd_rows up to fp32 rounding.
// ---------------------------------------------------------------------------
template <int G, int U>
__global__ __launch_bounds__(256) void k_edge_bwd_grp(
    const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ order,
    int row_begin, int row_end, const int* __restrict__ csr_to_csc,
    const float* __restrict__ Wh, int ld_wh, const float* __restrict__ a_src,
    const float* __restrict__ c_src, const float* __restrict__ s_dst,
    const float* __restrict__ lse, const float* __restrict__ y_heads,
    const float* __restrict__ g, int H, int F, int HF, int concat, float slope, DropArgs drop_arg,
    float* __restrict__ ds_dst, float2* __restrict__ az_out) {
    const DropArgs drop = resolve_drop(drop_arg);
    constexpr int CL = (U + G - 1) / G;
    const int lane = threadIdx.x & 63;
    const int c = lane & (G - 1);
    const int gbase = lane & ~(G - 1);
    const int pos = row_begin + (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / G);
    if (pos >= row_end) return;
    const int r = order != nullptr ? order[pos] : pos;
    const bool c_ok = 4 * c < HF;
    const int coff = c_ok ? 4 * c : 0;
    const int h = coff / F;
    const int hl = F / 4;  // lanes per head
    const bool leader = c_ok && (coff % F) == 0;
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
    const f32x4 a4 = c_ok ? *reinterpret_cast<const f32x4*>(a_src + coff) : zero4;
    const float c1 = c_src[h];
    f32x4 dy = zero4, yv = zero4;
    if (c_ok) {
        if (concat) {
            dy = *reinterpret_cast<const f32x4*>(g + (size_t)r * HF + coff);
        } else {
            dy = *reinterpret_cast<const f32x4*>(g + (size_t)r * F + (coff % F));
            dy *= 1.f / (float)H;
        }
        yv = *reinterpret_cast<const f32x4*>(y_heads + (size_t)r * HF + coff);
    }
    auto hsum = [&](float v) {
        if (hl <= 16) return group_sum16(v, hl);
        for (int off = 1; off < hl; off <<= 1) v += __shfl_xor(v, off);
        return v;
    };
    const float dl = hsum(dy.x * yv.x + dy.y * yv.y + dy.z * yv.z + dy.w * yv.w);
    const float sd = s_dst[(size_t)r * H + h] + c1;
    const float ls2 = lse[(size_t)r * H + h] * kLog2e;
    const int e0 = rowptr[r], e1 = rowptr[r + 1];
    float dsd = 0.f;
    int cv[CL], sv[CL];
#pragma unroll
    for (int t = 0; t < CL; ++t) {
        const int kk = min(e0 + c + t * G, e1 - 1);
        cv[t] = e1 > e0 ? col[kk] : 0;
        sv[t] = e1 > e0 ? csr_to_csc[kk] : 0;
    }
    for (int k = e0; k < e1; k += U) {
        const int nk = min(U, e1 - k);
        int cn[CL], sn[CL];
#pragma unroll
        for (int t = 0; t < CL; ++t) {
            const int kk = min(k + U + c + t * G, e1 - 1);
            cn[t] = col[kk];
            sn[t] = csr_to_csc[kk];
        }
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = __shfl(cv[u / G], gbase + (u % G));
            v[u] = *reinterpret_cast<const f32x4*>(Wh + (size_t)j * ld_wh + coff);
        }
        float ss[U], da[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ss[u] = v[u].x * a4.x + v[u].y * a4.y + v[u].z * a4.z + v[u].w * a4.w;
            da[u] = v[u].x * dy.x + v[u].y * dy.y + v[u].z * dy.z + v[u].w * dy.w;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ss[u] = hsum(ss[u]);
            da[u] = hsum(da[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int slot = __shfl(sv[u / G], gbase + (u % G));
            const float z = sd + ss[u];
            const float a = __builtin_amdgcn_exp2f(fmaxf(z, z * slope) * kLog2e - ls2);
            const float dm = drop.thresh != 0u ? drop_factor(drop, k + u, h, H) : 1.f;
            const float de = a * (dm * da[u] - dl);
            const float dz = z > 0.f ? de : de * slope;
            if (u < nk) {
                dsd += dz;
                if (leader) az_out[(size_t)slot * H + h] = make_float2(a * dm, dz);
            }
        }
#pragma unroll
        for (int t = 0; t < CL; ++t) {
            cv[t] = cn[t];
            sv[t] = sn[t];
        }
    }
    if (leader) ds_dst[(size_t)r * H + h] = dsd;
}

// ---------------------------------------------------------------------------
// Recompute backward (LeakyReLU, F/4 a power of two): no per-edge state.
//
// Pass 1, per TARGET row i (k_edge_grp layout): delta_h = dy_h . y_h, then over
// the in-edges the same recomputation as k_edge_bwd_grp, accumulating only
// ds_dst[i].  Writes one row of the target table
//   T[i] = [ g_i (ldg, 0-padded to 4) | per head (s_dst, lse, delta, 0) ]
// so pass 2 gathers everything it needs about a target with two float4 loads
// per lane.  Per edge: 4 (col) + 4HF (Wh row) bytes, as the forward.
// ---------------------------------------------------------------------------
template <int G, int U>
__global__ __launch_bounds__(256) void k_bwd_targets(
    const int* __restrict__ rowptr, const int* __restrict__ col, const int* __restrict__ order,
    int row_begin, int row_end, const float* __restrict__ Wh, int ld_wh,
    const float* __restrict__ a_src, const float* __restrict__ c_src,
    const float* __restrict__ s_dst, const float* __restrict__ lse,
    const float* __restrict__ y_heads, const float* __restrict__ g, int H, int F, int HF,
    int concat, float slope, DropArgs drop_arg, float* __restrict__ ds_dst,
    float* __restrict__ T, int ld_t) {
    const DropArgs drop = resolve_drop(drop_arg);
    constexpr int CL = (U + G - 1) / G;
    const int lane = threadIdx.x & 63;
    const int c = lane & (G - 1);
    const int gbase = lane & ~(G - 1);
    const int pos = row_begin + (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / G);
    if (pos >= row_end) return;
    const int r = order != nullptr ? order[pos] : pos;
    const bool c_ok = 4 * c < HF;
    const int coff = c_ok ? 4 * c : 0;
    const int h = coff / F;
    const int hl = F / 4;
    const bool leader = c_ok && (coff % F) == 0;
    const int ldg = concat ? HF : F;
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
    const f32x4 a4 = c_ok ? *reinterpret_cast<const f32x4*>(a_src + coff) : zero4;
    const float c1 = c_src[h];
    f32x4 g4 = zero4, yv = zero4;
    const bool g_ok = c_ok && (concat || coff < F);
    if (c_ok) {
        g4 = *reinterpret_cast<const f32x4*>(g + (size_t)r * ldg + (concat ? coff : coff % F));
        yv = *reinterpret_cast<const f32x4*>(y_heads + (size_t)r * HF + coff);
    }
    const f32x4 dy = concat ? g4 : g4 * (1.f / (float)H);
    auto hsum = [&](float v) {
        if (hl <= 16) return group_sum16(v, hl);
        for (int off = 1; off < hl; off <<= 1) v += __shfl_xor(v, off);
        return v;
    };
    const float dl = hsum(dy.x * yv.x + dy.y * yv.y + dy.z * yv.z + dy.w * yv.w);
    const float sdv = s_dst[(size_t)r * H + h];
    const float lsv = lse[(size_t)r * H + h];
    const float sd = sdv + c1;
    const float ls2 = lsv * kLog2e;
    const int e0 = rowptr[r], e1 = rowptr[r + 1];
    float dsd = 0.f;
    int cv[CL];
#pragma unroll
    for (int t = 0; t < CL; ++t) cv[t] = e1 > e0 ? col[min(e0 + c + t * G, e1 - 1)] : 0;
    for (int k = e0; k < e1; k += U) {
        const int nk = min(U, e1 - k);
        int cn[CL];
#pragma unroll
        for (int t = 0; t < CL; ++t) cn[t] = col[min(k + U + c + t * G, e1 - 1)];
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = __shfl(cv[u / G], gbase + (u % G));
            v[u] = *reinterpret_cast<const f32x4*>(Wh + (size_t)j * ld_wh + coff);
        }
        float ss[U], da[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ss[u] = hsum(v[u].x * a4.x + v[u].y * a4.y + v[u].z * a4.z + v[u].w * a4.w);
            da[u] = hsum(v[u].x * dy.x + v[u].y * dy.y + v[u].z * dy.z + v[u].w * dy.w);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float z = sd + ss[u];
            const float a = __builtin_amdgcn_exp2f(fmaxf(z, z * slope) * kLog2e - ls2);
            const float dm = drop.thresh != 0u ? drop_factor(drop, k + u, h, H) : 1.f;
            const float de = a * (dm * da[u] - dl);
            const float dz = z > 0.f ? de : de * slope;
            dsd += u < nk ? dz : 0.f;
        }
#pragma unroll
        for (int t = 0; t < CL; ++t) cv[t] = cn[t];
    }
    float* tr = T + (size_t)r * ld_t;
    if (g_ok) *reinterpret_cast<f32x4*>(tr + coff) = g4;
    if (leader) {
        ds_dst[(size_t)r * H + h] = dsd;
        *reinterpret_cast<f32x4*>(tr + round_up4(ldg) + 4 * h) = f32x4{sdv, lsv, dl, 0.f};
    }
}

// ---------------------------------------------------------------------------
// Pass 1 without edges (after the kink-sum forward, k_edge_grp<..., KINK>):
// per target row i and head h, with dy = dL/dy_h and delta = dy . y,
//   ds_dst[i,h] = dy . Q[i,h] - delta R[i,h]
// (= sum_j alpha_ij L'(z_ij) (drop_ij dy . Wh_j - delta), the sum k_bwd_targets
// walks the in-edges for), and the target table row exactly as k_bwd_targets
// writes it.  G lanes per row (G = next_pow2(HF/4)), one float4 of one head each.
// Per row: 4 ldg (g) + 8 HF (y, Q) + 12 H bytes read, 4 ld_t + 4 H written.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_bwd_table(
    int n, int G, const float* __restrict__ s_dst, const float* __restrict__ lse,
    const float* __restrict__ y_heads, const float* __restrict__ q_heads,
    const float* __restrict__ r_heads, const float* __restrict__ g, int H, int F, int HF,
    int concat, float* __restrict__ ds_dst, float* __restrict__ T, int ld_t) {
    const int lane = threadIdx.x & 63;
    const int c = lane & (G - 1);
    const long long r = (blockIdx.x * (long long)blockDim.x + threadIdx.x) / G;
    if (r >= n) return;  // whole groups (G divides 64)
    const bool c_ok = 4 * c < HF;
    const int coff = c_ok ? 4 * c : 0;
    const int h = coff / F;
    const int hl = F / 4;
    const bool leader = c_ok && (coff % F) == 0;
    const int ldg = concat ? HF : F;
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
    f32x4 g4 = zero4, yv = zero4, qv = zero4;
    const bool g_ok = c_ok && (concat || coff < F);
    if (c_ok) {
        g4 = *reinterpret_cast<const f32x4*>(g + r * ldg + (concat ? coff : coff % F));
        yv = *reinterpret_cast<const f32x4*>(y_heads + r * HF + coff);
        qv = *reinterpret_cast<const f32x4*>(q_heads + r * HF + coff);
    }
    const f32x4 dy = concat ? g4 : g4 * (1.f / (float)H);
    auto hsum = [&](float v) {
        if (hl <= 16) return group_sum16(v, hl);
        for (int off = 1; off < hl; off <<= 1) v += __shfl_xor(v, off);
        return v;
    };
    const float dl = hsum(dy.x * yv.x + dy.y * yv.y + dy.z * yv.z + dy.w * yv.w);
    const float dq = hsum(dy.x * qv.x + dy.y * qv.y + dy.z * qv.z + dy.w * qv.w);
    float* tr = T + r * ld_t;
    if (g_ok) *reinterpret_cast<f32x4*>(tr + coff) = g4;
    if (leader) {
        ds_dst[r * H + h] = dq - dl * r_heads[r * H + h];
        *reinterpret_cast<f32x4*>(tr + round_up4(ldg) + 4 * h) =
            f32x4{s_dst[r * H + h], lse[r * H + h], dl, 0.f};
    }
}

// ---------------------------------------------------------------------------
// Pass 2, per SOURCE row j (lane-group layout over the CSC): lane owns one
// float4 of Wh[j] (one head).  Per out-edge j -> i (slot e, CSR position
// k = csc_eid[e]): gather T[i] (the lane's g float4 + its head's
// (s_dst, lse, delta)), recompute
//   z = s_dst[i] + s_src[j], A = drop * exp(LReLU(z) - lse[i]),
//   dA = drop * (dy_i . Wh[j]) (DPP head sum), dz = A_undropped (dA - delta) LReLU'(z)
// and accumulate dWh[j] += A dy_i, ds_src[j] += dz.  Rows are strided over a
// fixed grid; each lane keeps its rows' contributions to da1/da2/dc1/dc2/db/
// dbias in registers, the wave's groups are combined by xor-shuffles and the
// wave writes one partial row [da1 | da2 | dc1 | dc2 | db | dbias] (summed by
// gat_sum_partials; deterministic).
// Per edge: 4 (csc_dst) + 4 (csc_eid, with dropout) + 4 ldg + 16 H bytes.
// ---------------------------------------------------------------------------
template <int G, int U>
__global__ __launch_bounds__(256) void k_bwd_sources(
    const int* __restrict__ csc_ptr, const int* __restrict__ csc_dst,
    const int* __restrict__ csc_eid, int n, const float* __restrict__ Wh, int ld_wh,
    const float* __restrict__ T, int ld_t, const float* __restrict__ ds_dst,
    const float* __restrict__ a_src, const float* __restrict__ c_src,
    const float* __restrict__ a_dst, int H, int F, int HF, int concat, float slope,
    DropArgs drop_arg, float* __restrict__ dwh, int ld_dwh, float* __restrict__ part) {
    const DropArgs drop = resolve_drop(drop_arg);
    constexpr int CL = (U + G - 1) / G;
    const int lane = threadIdx.x & 63;
    const int c = lane & (G - 1);
    const int gbase = lane & ~(G - 1);
    const int groups = (gridDim.x * blockDim.x) / G;
    const int gid = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / G);
    const bool c_ok = 4 * c < HF;
    const int coff = c_ok ? 4 * c : 0;
    const int h = coff / F;
    const int hl = F / 4;
    const bool leader = c_ok && (coff % F) == 0;
    const int ldg = concat ? HF : F;
    const int toff = round_up4(ldg) + 4 * h;
    const int goff = concat ? coff : coff % F;
    const bool g_ok = c_ok && (concat || coff < F);
    const float gs = concat ? 1.f : 1.f / (float)H;
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
    const f32x4 a1 = c_ok ? *reinterpret_cast<const f32x4*>(a_src + coff) : zero4;
    const f32x4 a2 = c_ok ? *reinterpret_cast<const f32x4*>(a_dst + coff) : zero4;
    const float c1 = c_src[h];
    auto hsum = [&](float v) {
        if (hl <= 16) return group_sum16(v, hl);
        for (int off = 1; off < hl; off <<= 1) v += __shfl_xor(v, off);
        return v;
    };
    f32x4 pa1 = zero4, pa2 = zero4, pdb = zero4, pbias = zero4;
    float pc1 = 0.f, pc2 = 0.f;
    const bool use_drop = drop.thresh != 0u;
    for (int j = gid; j < n; j += groups) {
        const f32x4 w4 = c_ok ? *reinterpret_cast<const f32x4*>(Wh + (size_t)j * ld_wh + coff)
                              : zero4;
        const float ssrc = hsum(dot4(w4, a1)) + c1;
        const int b0 = csc_ptr[j], b1 = csc_ptr[j + 1];
        f32x4 acc = zero4;
        float dss = 0.f;
        int iv[CL], kv[CL];
#pragma unroll
        for (int t = 0; t < CL; ++t) {
            const int bb = max(min(b0 + c + t * G, b1 - 1), 0);
            iv[t] = csc_dst[bb];
            kv[t] = use_drop ? csc_eid[bb] : 0;
        }
        for (int b = b0; b < b1; b += U) {
            const int nb = min(U, b1 - b);
            int in_[CL], kn[CL];
#pragma unroll
            for (int t = 0; t < CL; ++t) {
                const int bb = min(b + U + c + t * G, b1 - 1);
                in_[t] = csc_dst[bb];
                kn[t] = use_drop ? csc_eid[bb] : 0;
            }
            f32x4 gv[U], tv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = __shfl(iv[u / G], gbase + (u % G));
                const float* tr = T + (size_t)i * ld_t;
                gv[u] = g_ok || !concat ? *reinterpret_cast<const f32x4*>(tr + goff) : zero4;
                tv[u] = *reinterpret_cast<const f32x4*>(tr + toff);
            }
            float da[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                da[u] = hsum(dot4(gv[u], w4));
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int kpos = __shfl(kv[u / G], gbase + (u % G));
                const float z = tv[u].x + ssrc;
                // (e - lse) <= 0: the hardware exp2 on a log2e-scaled argument, as
                // the forward's softmax (v_exp_f32; expf's range reduction costs
                // ~10 more VALU per edge and head)
                const float a = __builtin_amdgcn_exp2f((fmaxf(z, z * slope) - tv[u].y) * kLog2e);
                const float dm = use_drop ? drop_factor(drop, kpos, h, H) : 1.f;
                const float de = a * __builtin_fmaf(dm * da[u], gs, -tv[u].z);
                const float dz = z > 0.f ? de : de * slope;
                const float w = u < nb ? a * dm : 0.f;
                acc = fma4(w, gv[u], acc);
                dss += u < nb ? dz : 0.f;
            }
#pragma unroll
            for (int t = 0; t < CL; ++t) {
                iv[t] = in_[t];
                kv[t] = kn[t];
            }
        }
        const float dsd = ds_dst[(size_t)j * H + h];
        const f32x4 d = fma4(dsd, a2, fma4(dss, a1, acc * gs));
        if (c_ok) *reinterpret_cast<f32x4*>(dwh + (size_t)j * ld_dwh + coff) = d;
        pa1 = fma4(dss, w4, pa1);
        pa2 = fma4(dsd, w4, pa2);
        pdb += c_ok ? d : zero4;
        if (g_ok) pbias += *reinterpret_cast<const f32x4*>(T + (size_t)j * ld_t + goff);
        if (leader) {
            pc1 += dss;
            pc2 += dsd;
        }
    }
    // combine the wave's 64/G groups (same columns in every group)
#pragma unroll
    for (int off = G; off < kWave; off <<= 1) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            pa1[q] += __shfl_xor(pa1[q], off);
            pa2[q] += __shfl_xor(pa2[q], off);
            pdb[q] += __shfl_xor(pdb[q], off);
            pbias[q] += __shfl_xor(pbias[q], off);
        }
        pc1 += __shfl_xor(pc1, off);
        pc2 += __shfl_xor(pc2, off);
    }
    if (lane >= G) return;
    const int wave = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave);
    float* pw = part + (size_t)wave * (3 * HF + 2 * H + ldg);
    if (c_ok) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            pw[coff + q] = pa1[q];
            pw[HF + coff + q] = pa2[q];
            pw[2 * HF + 2 * H + coff + q] = pdb[q];
        }
    }
    if (g_ok) {
#pragma unroll
        for (int q = 0; q < 4; ++q) pw[3 * HF + 2 * H + goff + q] = pbias[q];
    }
    if (leader) {
        pw[2 * HF + h] = pc1;
        pw[2 * HF + H + h] = pc2;
    }
}

// ---------------------------------------------------------------------------
// Pass 2, straight-line form for HF = 64 with 16 lanes per source row (every
// lane one float4 of one head: the reference's training configurations 8x8
// and 4x16).  The same arithmetic in the same order as k_bwd_sources (both
// spell their fused operations out: dot4 / fma4 / fmaf, gat_common.h), so the
// results are bitwise equal, but:
//  - the head's lane count HL = F/4 and dropout are template parameters, so
//    the edge loop has no branches, and every load is unconditional (in
//    k_bwd_sources the guarded loads and the runtime head-sum width split a
//    chunk into ~80 basic blocks, and the waitcnt pass, unable to count the
//    loads in flight across them, made each chunk wait for the id prefetch
//    it had just issued: a full memory latency per 16 edges);
//  - a chunk's target ids go to the row's lanes by DPP row_newbcast (a VALU
//    modifier) instead of ds_bpermute round trips through the LDS unit;
//  - the chunk's table gathers are issued before the next chunk's id loads
//    (sched_barrier), so the next chunk's wait covers only loads a chunk old.
// ---------------------------------------------------------------------------
template <int K>
__device__ __forceinline__ int row_bcast(int v) {
    return __builtin_amdgcn_update_dpp(0, v, 0x150 + K, 0xF, 0xF, false);
}

// f(integral_constant<int, 0>) ... f(integral_constant<int, N - 1>), in order
template <class Fn, int... Is>
__device__ __forceinline__ void static_for_impl(Fn&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class Fn>
__device__ __forceinline__ void static_for(Fn&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <int U, int HL, bool DROP>
__global__ __launch_bounds__(256) void k_bwd_sources_sl(
    const int* __restrict__ csc_ptr, const int* __restrict__ csc_dst,
    const int* __restrict__ csc_eid, int n, const float* __restrict__ Wh, int ld_wh,
    const float* __restrict__ T, int ld_t, const float* __restrict__ ds_dst,
    const float* __restrict__ a_src, const float* __restrict__ c_src,
    const float* __restrict__ a_dst, int H, int F, int HF, int concat, float slope,
    DropArgs drop_arg, float* __restrict__ dwh, int ld_dwh, float* __restrict__ part) {
    constexpr int G = 16;
    static_assert(U == 8 || U == 16, "one id per lane per chunk");
    const DropArgs drop = resolve_drop(drop_arg);
    const int lane = threadIdx.x & 63;
    const int c = lane & (G - 1);
    const int groups = (gridDim.x * blockDim.x) / G;
    const int gid = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / G);
    const int coff = 4 * c;  // HF == 64: every lane holds a float4
    const int h = c / HL;    // coff / F
    const bool leader = c % HL == 0;
    const int ldg = concat ? HF : F;
    const int toff = round_up4(ldg) + 4 * h;
    const int goff = concat ? coff : 4 * (c % HL);  // (coff % F)
    const bool g_ok = concat || coff < F;
    const float gs = concat ? 1.f : 1.f / (float)H;
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
    const f32x4 a1 = *reinterpret_cast<const f32x4*>(a_src + coff);
    const f32x4 a2 = *reinterpret_cast<const f32x4*>(a_dst + coff);
    const float c1 = c_src[h];
    const auto rs_dst = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(csc_dst), (short)0,
                                                          0x7FFFFFFF, 0x00020000);
    const auto rs_eid = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int*>(DROP ? csc_eid : csc_dst), (short)0, 0x7FFFFFFF, 0x00020000);
    f32x4 pa1 = zero4, pa2 = zero4, pdb = zero4, pbias = zero4;
    float pc1 = 0.f, pc2 = 0.f;
    for (int j = gid; j < n; j += groups) {
        const f32x4 w4 = *reinterpret_cast<const f32x4*>(Wh + (size_t)j * ld_wh + coff);
        const float ssrc = group_sum16(dot4(w4, a1), HL) + c1;
        const int b0 = csc_ptr[j], b1 = csc_ptr[j + 1];
        f32x4 acc = zero4;
        float dss = 0.f;
        int iv, kv = 0;
        {
            const int bb = max(min(b0 + c, b1 - 1), 0);
            iv = csc_dst[bb];
            if constexpr (DROP) kv = csc_eid[bb];
        }
        for (int b = b0; b < b1; b += U) {
            const int nb = min(U, b1 - b);
            f32x4 gv[U], tv[U];
            static_for<U>([&](auto uc) {
                constexpr int u = decltype(uc)::value;
                const float* tr = T + (size_t)row_bcast<u>(iv) * ld_t;
                gv[u] = *reinterpret_cast<const f32x4*>(tr + goff);
                tv[u] = *reinterpret_cast<const f32x4*>(tr + toff);
            });
            const int kc = kv;
            __builtin_amdgcn_sched_barrier(0);
            {  // the next chunk's ids (past the row: its last edge again, unused).
               // Buffer loads: a phi of this load and the row's first (a plain
               // load) would be folded into one load at the loop top, which
               // undoes the prefetch (byte offsets < 2^31: checked at launch)
                const int bb = min(b + U + c, b1 - 1);
                iv = (int)__builtin_amdgcn_raw_buffer_load_b32(rs_dst, bb * 4, 0, 0);
                if constexpr (DROP) kv = (int)__builtin_amdgcn_raw_buffer_load_b32(rs_eid, bb * 4, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);  // (the arithmetic below stays after them)
            float da[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                da[u] = group_sum16(dot4(gv[u], w4), HL);
            static_for<U>([&](auto uc) {
                constexpr int u = decltype(uc)::value;
                const float z = tv[u].x + ssrc;
                const float a = __builtin_amdgcn_exp2f((fmaxf(z, z * slope) - tv[u].y) * kLog2e);
                float dm = 1.f;
                if constexpr (DROP) dm = drop_factor(drop, row_bcast<u>(kc), h, H);
                const float de = a * __builtin_fmaf(dm * da[u], gs, -tv[u].z);
                const float dz = z > 0.f ? de : de * slope;
                const float w = u < nb ? a * dm : 0.f;
                acc = fma4(w, gv[u], acc);
                dss += u < nb ? dz : 0.f;
            });
        }
        const float dsd = ds_dst[(size_t)j * H + h];
        const f32x4 d = fma4(dsd, a2, fma4(dss, a1, acc * gs));
        *reinterpret_cast<f32x4*>(dwh + (size_t)j * ld_dwh + coff) = d;
        pa1 = fma4(dss, w4, pa1);
        pa2 = fma4(dsd, w4, pa2);
        pdb += d;
        if (g_ok) pbias += *reinterpret_cast<const f32x4*>(T + (size_t)j * ld_t + goff);
        if (leader) {
            pc1 += dss;
            pc2 += dsd;
        }
    }
#pragma unroll
    for (int off = G; off < kWave; off <<= 1) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            pa1[q] += __shfl_xor(pa1[q], off);
            pa2[q] += __shfl_xor(pa2[q], off);
            pdb[q] += __shfl_xor(pdb[q], off);
            pbias[q] += __shfl_xor(pbias[q], off);
        }
        pc1 += __shfl_xor(pc1, off);
        pc2 += __shfl_xor(pc2, off);
    }
    if (lane >= G) return;
    const int wave = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kWave);
    float* pw = part + (size_t)wave * (3 * HF + 2 * H + ldg);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        pw[coff + q] = pa1[q];
        pw[HF + coff + q] = pa2[q];
        pw[2 * HF + 2 * H + coff + q] = pdb[q];
    }
    if (g_ok) {
#pragma unroll
        for (int q = 0; q < 4; ++q) pw[3 * HF + 2 * H + goff + q] = pbias[q];
    }
    if (leader) {
        pw[2 * HF + h] = pc1;
        pw[2 * HF + H + h] = pc2;
    }
}

// ---------------------------------------------------------------------------
// Backward, pass 2: one wave per SOURCE row j (CSC, grid-stride), lanes over
// the HF columns (CQ per lane).  Over j's out-edges (target i, slot c):
//   dWh[j]    = sum_c A[c,h] * dy[i]_h            (message backward)
//   ds_src[j] = sum_c dz[c]
// then the score terms s_src = Wh.a1 + c1, s_dst = Wh.a2 + c2 fold in:
//   dWh_total[j] = dWh[j] + ds_src[j,h] a1_h + ds_dst[j,h] a2_h
// and each wave accumulates its rows' contributions to da1/da2 (ds * Wh),
// dc1/dc2 (ds), db (= sum of dWh_total rows, the projection bias gradient)
// and dbias (= sum of grad_out rows) in registers, written once as per-wave
// partials part[w] = [da1 (HF) | da2 (HF) | dc1 (H) | dc2 (H) | db (HF) |
// dbias (ldg)] — summed by the caller; no float atomics, so the result is
// run-to-run deterministic.
// Algorithmic bytes per edge: 4 (csc_dst) + 4HF (g row, concat; 4F mean)
// + 8H (A, dz); per row: 4HF (Wh) + 4HF (dWh) + 8H.
// ---------------------------------------------------------------------------
template <int CQ, int HP>
__global__ __launch_bounds__(64) void k_src_bwd(
    const int* __restrict__ csc_ptr, const int* __restrict__ csc_dst, int n,
    const float* __restrict__ Wh, int ld_wh, const float* __restrict__ g,
    const float2* __restrict__ az, const float* __restrict__ ds_dst, const float* __restrict__ a1, const float* __restrict__ a2,
    int H, int F, int HF, int concat, float* __restrict__ dwh, int ld_dwh,
    float* __restrict__ ds_src, float* __restrict__ part) {
    __shared__ float dss_s[HP];
    const int lane = threadIdx.x;
    const int w = blockIdx.x;
    const int nw = gridDim.x;
    const float inv_h = 1.f / (float)H;
    int cc[CQ], hq[CQ], gq[CQ];
    bool okq[CQ];
    float a1v[CQ], a2v[CQ], pa1[CQ], pa2[CQ], pdb[CQ], pbias[CQ];
#pragma unroll
    for (int q = 0; q < CQ; ++q) {
        const int c = lane + kWave * q;
        okq[q] = c < HF;
        cc[q] = okq[q] ? c : 0;
        hq[q] = cc[q] / F;
        gq[q] = concat ? cc[q] : cc[q] - hq[q] * F;  // column of g feeding column c
        a1v[q] = okq[q] ? a1[cc[q]] : 0.f;
        a2v[q] = okq[q] ? a2[cc[q]] : 0.f;
        pa1[q] = 0.f;
        pa2[q] = 0.f;
        pdb[q] = 0.f;
        pbias[q] = 0.f;
    }
    const int ldg = concat ? HF : F;
    const float gs = concat ? 1.f : inv_h;
    const bool h_ok = lane < H;
    float pc1 = 0.f, pc2 = 0.f;
    constexpr int UE = 4;
    for (int j = w; j < n; j += nw) {
        const int b0 = csc_ptr[j], b1 = csc_ptr[j + 1];
        float acc[CQ];
#pragma unroll
        for (int q = 0; q < CQ; ++q) acc[q] = 0.f;
        float dss = 0.f;
        for (int b = b0; b < b1; b += UE) {
            int iu[UE], su[UE];
            float gate[UE];
#pragma unroll
            for (int u = 0; u < UE; ++u) {
                su[u] = min(b + u, b1 - 1);
                gate[u] = (b + u < b1) ? 1.f : 0.f;
                iu[u] = csc_dst[su[u]];
            }
            float gv[UE][CQ], av[UE][CQ], zv[UE];
#pragma unroll
            for (int u = 0; u < UE; ++u) {
#pragma unroll
                for (int q = 0; q < CQ; ++q) {
                    gv[u][q] = g[(size_t)iu[u] * ldg + gq[q]];
                    av[u][q] = az[(size_t)su[u] * H + hq[q]].x;
                }
                zv[u] = h_ok ? az[(size_t)su[u] * H + lane].y : 0.f;
            }
#pragma unroll
            for (int u = 0; u < UE; ++u) {
#pragma unroll
                for (int q = 0; q < CQ; ++q) acc[q] = fmaf(gate[u] * av[u][q], gv[u][q], acc[q]);
                dss = fmaf(gate[u], zv[u], dss);
            }
        }
        if (h_ok) {
            dss_s[lane] = dss;
            if (ds_src != nullptr) ds_src[(size_t)j * H + lane] = dss;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < CQ; ++q) {
            if (okq[q]) {
                const float hsrc = dss_s[hq[q]];
                const float hdst = ds_dst[(size_t)j * H + hq[q]];
                const float whv = Wh[(size_t)j * ld_wh + cc[q]];
                const float d = fmaf(hdst, a2v[q], fmaf(hsrc, a1v[q], acc[q] * gs));
                dwh[(size_t)j * ld_dwh + cc[q]] = d;
                pa1[q] = fmaf(hsrc, whv, pa1[q]);
                pa2[q] = fmaf(hdst, whv, pa2[q]);
                pdb[q] += d;
            }
            if (cc[q] < ldg && okq[q]) pbias[q] += g[(size_t)j * ldg + cc[q]];
        }
        if (h_ok) {
            pc1 += dss;
            pc2 += ds_dst[(size_t)j * H + lane];
        }
        __syncthreads();
    }
    float* pw = part + (size_t)w * (3 * HF + 2 * H + ldg);
#pragma unroll
    for (int q = 0; q < CQ; ++q) {
        if (okq[q]) {
            pw[cc[q]] = pa1[q];
            pw[HF + cc[q]] = pa2[q];
            pw[2 * HF + 2 * H + cc[q]] = pdb[q];
            if (cc[q] < ldg) pw[3 * HF + 2 * H + cc[q]] = pbias[q];
        }
    }
    if (h_ok) {
        pw[2 * HF + lane] = pc1;
        pw[2 * HF + H + lane] = pc2;
    }
}

// ---------------------------------------------------------------------------
// Weight gradient of the projection: dW[HF, Fin] = dWh^T x, a contraction
// over all N rows (K = N), which library GEMM heuristics handle poorly (one
// 165 us hipBLASLt call at PPI shape).  Split-K on fp32 MFMA 16x16x4: block
// (fin tile of 64, row chunk s, hf tile of 64); wave w owns hf rows
// [16w, 16w+16) of the tile and all four 16-wide fin sub-tiles, so per 4 rows
// a lane issues 1 dWh + 4 x loads and 4 MFMAs.  Operands come straight from
// global memory (each row is read by one block: no reuse for LDS to exploit).
// part[s] = the chunk's [HF, Fin] partial; k_wgrad_reduce sums the chunks in
// a fixed order (deterministic).
// Algorithmic bytes: 4 N (HF + Fin) reads + 4 S HF Fin partials.
// LW > 1: the four 16-column sub-tiles are interleaved so that a lane's four x
// values of a row are LW adjacent floats (sub-tile t, lane column ii holds
// fin column j0 + LW ii + (t % LW) + 16 LW (t / LW)): one float2 / float4 load
// instead of four scalar ones (the B columns of an MFMA may be any 16 columns;
// the store maps them back).  The kernel is bound by load instructions.
// ---------------------------------------------------------------------------
template <int LW>
__global__ __launch_bounds__(256) void k_wgrad(const float* __restrict__ dwh, int ld_dwh,
                                               const float* __restrict__ x, int n, int fin,
                                               int hf, int rows_per_chunk,
                                               float* __restrict__ part) {
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int j0 = blockIdx.x * 64;
    const int s = blockIdx.y;
    const int i0 = blockIdx.z * 64 + wv * 16;
    const int r0 = s * rows_per_chunk;
    const int r1 = min(n, r0 + rows_per_chunk);
    const int kk = lane >> 4, ii = lane & 15;
    const int icol = i0 + ii;
    const bool i_ok = icol < hf;
    const float amask = i_ok ? 1.f : 0.f;
    const int ic = i_ok ? icol : 0;
    // column of sub-tile t held by this lane
    auto jcol = [&](int t) {
        return LW == 1 ? j0 + 16 * t + ii : j0 + LW * ii + (t % LW) + 16 * LW * (t / LW);
    };
    constexpr int NLD = 4 / LW;  // x loads per row
    int jc[NLD];
#pragma unroll
    for (int q = 0; q < NLD; ++q) jc[q] = min(jcol(q * LW), fin - LW);  // in bounds; unused past fin
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int UR = 4;  // 4-row MFMA steps in flight
    for (int r = r0; r < r1; r += 4 * UR) {
        float av[UR], bv[UR][4];
#pragma unroll
        for (int u = 0; u < UR; ++u) {
            const int row = r + 4 * u + kk;
            const bool ok = row < r1;
            const int rr = ok ? row : r1 - 1;
            av[u] = dwh[(size_t)rr * ld_dwh + ic] * (ok ? amask : 0.f);
            const float* xr = x + (size_t)rr * fin;
#pragma unroll
            for (int q = 0; q < NLD; ++q) {
                if constexpr (LW == 4) {
                    const f32x4 v = *reinterpret_cast<const f32x4*>(xr + jc[q]);
                    bv[u][0] = v.x; bv[u][1] = v.y; bv[u][2] = v.z; bv[u][3] = v.w;
                } else if constexpr (LW == 2) {
                    const f32x2 v = *reinterpret_cast<const f32x2*>(xr + jc[q]);
                    bv[u][2 * q] = v.x; bv[u][2 * q + 1] = v.y;
                } else {
                    bv[u][q] = xr[jc[q]];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < UR; ++u)
#pragma unroll
            for (int t = 0; t < 4; ++t)
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u][t], acc[t], 0, 0, 0);
    }
    // C[i][j]: j = lane & 15, i = 4 * (lane >> 4) + q
    float* ps = part + (size_t)s * hf * fin;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int j = jcol(t);
        if (j >= fin) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = i0 + 4 * kk + q;
            if (i < hf) ps[(size_t)i * fin + j] = acc[t][q];
        }
    }
}

// ---------------------------------------------------------------------------
// Input gradient of the projection: dx[n, fin] = dWh[n, hf] W[hf, fin] (the x
// side of GAT.py:42-48's Linear layers; replaces the hipBLASLt GEMM).  fp32
// MFMA (v_mfma_f32_16x16x4_f32, exact fp32 products) with the operands swapped
// so the accumulator holds dx^T tiles: lane l ends with dx[row l&15][c + 4(l>>4)
// .. +4], four consecutive columns of one row.  The K = hf sum runs as KL
// k-steps per lane (lane kq owns k in [KL kq, KL kq + KL): every lane's dWh
// fragment is one contiguous run of its row, loaded once); W^T is staged per
// 64-column block in LDS (row stride KP + 1: conflict-free fragment reads).
// A workgroup owns 64 rows (one 16-row tile per wave) and walks all fin
// columns, so dWh is read once and W (hf x fin, L2-resident) once per
// workgroup.
// ---------------------------------------------------------------------------
template <int KL>
__global__ __launch_bounds__(256) void k_dx(const float* __restrict__ dwh, int ld_dwh, int hf,
                                            int n, const float* __restrict__ W, int fin,
                                            float* __restrict__ dx, int ld_dx) {
    constexpr int KP = 4 * KL, WS = KP + 1;
    __shared__ float wt[64 * WS];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int cl = lane & 15, kq = lane >> 4;
    const int row = blockIdx.x * 64 + w * 16 + cl;
    const int kb = KL * kq;
    float b[KL];
    {
        const float* src = dwh + (size_t)min(row, n - 1) * ld_dwh;
#pragma unroll
        for (int s = 0; s < KL; ++s) b[s] = kb + s < hf ? src[min(kb + s, hf - 1)] : 0.f;
    }
    const bool pair = (ld_dx % 2) == 0 && (reinterpret_cast<uintptr_t>(dx) & 7) == 0;
    for (int c0 = 0; c0 < fin; c0 += 64) {
        __syncthreads();  // the previous block's fragment reads are done
        for (int i = tid; i < 64 * KP; i += 256) {
            const int c = i & 63, k = i >> 6;  // a wave reads 64 consecutive columns of W row k
            wt[c * WS + k] = (k < hf && c0 + c < fin) ? W[(size_t)k * fin + c0 + c] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            if (c0 + 16 * t >= fin) break;  // block-uniform
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
            const float* a = wt + (16 * t + cl) * WS + kb;
#pragma unroll
            for (int s = 0; s < KL; ++s)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], acc, 0, 0, 0);
            const int col = c0 + 16 * t + 4 * kq;
            if (row < n) {
                float* d = dx + (size_t)row * ld_dx + col;
                if (col + 3 < fin && pair) {
                    *reinterpret_cast<f32x2*>(d) = f32x2{acc.x, acc.y};
                    *reinterpret_cast<f32x2*>(d + 2) = f32x2{acc.z, acc.w};
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (col + r < fin) d[r] = acc[r];
                }
            }
        }
    }
}

// out[b * width + e] = sum_c part[c * width + e] over rows c of row block
// b = blockIdx.y ([b * rows_per_block, ...) ∩ [0, rows)): 16 columns x 16 row
// groups per block, 4 independent loads in flight per thread, then a fixed
// order combine in LDS (deterministic).  Sums the per-chunk / per-wave
// partials of k_wgrad and k_src_bwd.
__global__ __launch_bounds__(256) void k_colsum(const float* __restrict__ part, int rows,
                                                long long width, float* __restrict__ out,
                                                int rows_per_block) {
    __shared__ float red[16][17];
    const int col = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const long long e = blockIdx.x * 16LL + col;
    const long long ec = e < width ? e : width - 1;
    const int rb0 = blockIdx.y * rows_per_block;
    part += (size_t)rb0 * width;
    out += (size_t)blockIdx.y * width;
    rows = min(rows - rb0, rows_per_block);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int c = grp;
    for (; c + 48 < rows; c += 64) {
        s0 += part[(size_t)c * width + ec];
        s1 += part[(size_t)(c + 16) * width + ec];
        s2 += part[(size_t)(c + 32) * width + ec];
        s3 += part[(size_t)(c + 48) * width + ec];
    }
    for (; c < rows; c += 16) s0 += part[(size_t)c * width + ec];
    red[grp][col] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (grp == 0 && e < width) {
        float t = 0.f;
#pragma unroll
        for (int g = 0; g < 16; ++g) t += red[g][col];
        out[e] = t;
    }
}

int wgrad_chunks(int n, int fin, int hf) {
    const int ftiles = (fin + 63) / 64, htiles = (hf + 63) / 64;
    int by_rows = (n + 255) / 256;
    int by_fill = (2048 + ftiles * htiles - 1) / (ftiles * htiles);
    int c = by_rows < by_fill ? by_rows : by_fill;
    return c < 1 ? 1 : c;
}

// counter -> seed: splitmix64 of the counter value, then counter += 1
__global__ void k_seed_next(unsigned long long* __restrict__ counter,
                            unsigned long long* __restrict__ seed_out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const unsigned long long v = counter[0];
    counter[0] = v + 1ull;
    unsigned long long z = v + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    seed_out[0] = z ^ (z >> 31);
}

}  // namespace

extern "C" {

int gat_dropout_seed_next(unsigned long long* counter, unsigned long long* seed_out,
                          void* stream) {
    if (counter == nullptr || seed_out == nullptr) return GAT_EINVAL;
    hipLaunchKernelGGL(k_seed_next, dim3(1), dim3(64), 0, (hipStream_t)stream, counter, seed_out);
    return status_of(hipGetLastError());
}

int gat_bwd_table_layout(int heads, int f, int concat, int* ld_t) {
    if (heads <= 0 || f <= 0 || ld_t == nullptr) return GAT_EINVAL;
    *ld_t = round_up4(concat ? heads * f : f) + 4 * heads;
    return GAT_OK;
}

// edges per chunk of the recompute backward kernels: the forward's thresholds
static int bwd_unroll(int hint) {
    hint &= ~(GAT_HINT_LOCAL | GAT_HINT_SHORT);
    return hint <= 0 ? 8 : hint <= 32 ? 4 : hint <= 64 ? 8 : 16;
}

static bool bwd_recompute_ok(int heads, int f, float slope, const float* wh, int ld_wh) {
    // GAT_BWD_KERNEL=stored|generic (A/B knob): force the stored-coefficient path
    if (const char* v = knob("GAT_BWD_KERNEL"))
        if (std::strcmp(v, "stored") == 0 || std::strcmp(v, "generic") == 0) return false;
    const int hl = f / 4;
    return heads * f <= GAT_MAX_HF && heads <= GAT_MAX_HEADS && f % 4 == 0 &&
           next_pow2(hl) == hl && slope >= 0.f && slope <= 1.f && (ld_wh & 3) == 0 &&
           (reinterpret_cast<uintptr_t>(wh) & 15) == 0;
}

int gat_bwd_targets(const int* rowptr, const int* col, const int* row_order, int row_begin,
                    int row_end, const float* wh, int ld_wh, const float* a_src,
                    const float* c_src, const float* s_dst, const float* lse,
                    const float* y_heads, const float* grad_out, int heads, int f, int concat,
                    float negative_slope, float dropout_p, unsigned long long seed,
                    const unsigned long long* seed_dev, float* ds_dst, float* table, int ld_t,
                    int edges_per_row_hint, void* stream) {
    if (heads <= 0 || f <= 0 || row_begin < 0 || row_end < row_begin) return GAT_EINVAL;
    if (!(dropout_p >= 0.f && dropout_p <= 1.f)) return GAT_EINVAL;
    int need_ld = 0;
    gat_bwd_table_layout(heads, f, concat, &need_ld);
    if (ld_t < need_ld || (ld_t & 3)) return GAT_EINVAL;
    if (!bwd_recompute_ok(heads, f, negative_slope, wh, ld_wh)) return GAT_EUNSUPPORTED;
    const int rows = row_end - row_begin;
    if (rows == 0) return GAT_OK;
    hipStream_t st = (hipStream_t)stream;
    const DropArgs drop = make_drop(dropout_p, seed, seed_dev);
    const int hf = heads * f;
    const int g = next_pow2(hf / 4);
    int u = bwd_unroll(edges_per_row_hint);
    const long long threads = (long long)rows * g;
    const dim3 grid((unsigned)((threads + 255) / 256)), block(256);
    #define GAT_BT(G, UU)                                                                         \
    hipLaunchKernelGGL((k_bwd_targets<G, UU>), grid, block, 0, st, rowptr, col, row_order,    \
                       row_begin, row_end, wh, ld_wh, a_src, c_src, s_dst, lse, y_heads,      \
                       grad_out, heads, f, hf, concat, negative_slope, drop, ds_dst, table,   \
                       ld_t)
    // (the kink-sum table, gat_bwd_table, is the default where the forward can
    // form the sums: this pass serves the other head widths, at U = 8)
    (void)u;
#define GAT_BT_U(G)                      \
    case G:                              \
        GAT_BT(G, 8);                    \
        break;
    switch (g) {
        GAT_BT_U(1) GAT_BT_U(2) GAT_BT_U(4) GAT_BT_U(8) GAT_BT_U(16) GAT_BT_U(32) GAT_BT_U(64)
        default: return GAT_EUNSUPPORTED;
    }
#undef GAT_BT_U
#undef GAT_BT
    return status_of(hipGetLastError());
}

int gat_bwd_table(const float* s_dst, const float* lse, const float* y_heads,
                  const float* q_heads, const float* r_heads, const float* grad_out,
                  int num_nodes, int heads, int f, int concat, float* ds_dst, float* table,
                  int ld_t, void* stream) {
    if (num_nodes < 0 || heads <= 0 || f <= 0) return GAT_EINVAL;
    if (num_nodes > 0 && (s_dst == nullptr || lse == nullptr || y_heads == nullptr || q_heads == nullptr ||
        r_heads == nullptr || grad_out == nullptr || ds_dst == nullptr || table == nullptr))
        return GAT_EINVAL;
    int need_ld = 0;
    gat_bwd_table_layout(heads, f, concat, &need_ld);
    if (ld_t < need_ld || (ld_t & 3)) return GAT_EINVAL;
    const int hf = heads * f;
    const int hl = f / 4;
    if (hf > GAT_MAX_HF || heads > GAT_MAX_HEADS || f % 4 != 0 || next_pow2(hl) != hl)
        return GAT_EUNSUPPORTED;
    // GAT_BWD_KERNEL=stored|generic forces the stored-coefficient backward, as
    // gat_bwd_targets honours it
    if (const char* v = knob("GAT_BWD_KERNEL"))
        if (std::strcmp(v, "stored") == 0 || std::strcmp(v, "generic") == 0) return GAT_EUNSUPPORTED;
    if (num_nodes == 0) return GAT_OK;
    const int g = next_pow2(hf / 4);
    const long long threads = (long long)num_nodes * g;
    hipLaunchKernelGGL(k_bwd_table, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, num_nodes, g, s_dst, lse, y_heads, q_heads, r_heads,
                       grad_out, heads, f, hf, concat, ds_dst, table, ld_t);
    return status_of(hipGetLastError());
}

int gat_bwd_sources_parts(int num_nodes, int heads, int f, int* num_parts) {
    if (num_nodes < 0 || heads <= 0 || f <= 0 || num_parts == nullptr) return GAT_EINVAL;
    const int g = next_pow2((heads * f + 3) / 4);
    const long long waves = ((long long)num_nodes * g + kWave - 1) / kWave;
    const long long cap = 65536;
    long long w = waves < cap ? waves : cap;
    w = (w + 3) / 4 * 4;  // whole 256-thread blocks
    *num_parts = (int)(w < 4 ? 4 : w);
    return GAT_OK;
}

int gat_bwd_sources(const int* csc_ptr, const int* csc_dst, const int* csc_eid, int num_nodes,
                    const float* wh, int ld_wh, const float* table, int ld_t,
                    const float* ds_dst, const float* a_src, const float* c_src,
                    const float* a_dst, int heads, int f, int concat, float negative_slope,
                    float dropout_p, unsigned long long seed, const unsigned long long* seed_dev,
                    float* dwh, int ld_dwh, float* partials, int num_parts,
                    int edges_per_row_hint, void* stream) {
    if (heads <= 0 || f <= 0 || num_nodes < 0 || num_parts <= 0 || (num_parts & 3))
        return GAT_EINVAL;
    if (!(dropout_p >= 0.f && dropout_p <= 1.f)) return GAT_EINVAL;
    const int hf = heads * f;
    if (ld_dwh < hf || (ld_dwh & 3)) return GAT_EINVAL;
    if (!bwd_recompute_ok(heads, f, negative_slope, wh, ld_wh)) return GAT_EUNSUPPORTED;
    if (dropout_p > 0.f && csc_eid == nullptr) return GAT_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const DropArgs drop = make_drop(dropout_p, seed, seed_dev);
    const int g = next_pow2(hf / 4);
    int u = bwd_unroll(edges_per_row_hint);
    const dim3 grid(num_parts / 4), block(256);
    #define GAT_BS(G, UU)                                                                         \
    hipLaunchKernelGGL((k_bwd_sources<G, UU>), grid, block, 0, st, csc_ptr, csc_dst, csc_eid,  \
                       num_nodes, wh, ld_wh, table, ld_t, ds_dst, a_src, c_src, a_dst, heads, \
                       f, hf, concat, negative_slope, drop, dwh, ld_dwh, partials)
    // every chunk length for the HF = 32 / 64 lane groups (G = 8, 16); U = 8
    // for the other widths
#define GAT_BS_U(G)                                      \
    case G:                                              \
        if constexpr (G == 8 || G == 16) {               \
            if (u == 4) { GAT_BS(G, 4); }                \
            else if (u == 16) { GAT_BS(G, 16); }         \
            else { GAT_BS(G, 8); }                       \
        } else {                                         \
            GAT_BS(G, 8);                                \
        }                                                \
        break;
    // the straight-line kernel for HF = 64 (the default; GAT_BWD_SL=0 is the A/B
    // knob back to k_bwd_sources): Reddit training step 8.79 -> 8.55 ms, PPI
    // 0.568 -> 0.556 ms, same box, bitwise equal gradients
    // (profiles/r05/train_ab_sl_*.json)
    // (its id prefetch takes buffer loads of 31-bit byte offsets: E' < 2^29,
    // judged from the edges-per-row hint, floor(E'/N))
    const long long hint = edges_per_row_hint & ~(GAT_HINT_LOCAL | GAT_HINT_SHORT);
    bool sl = hf == 64 && (u == 8 || u == 16) && (f == 4 || f == 8 || f == 16) && hint > 0 &&
              (hint + 1) * (long long)num_nodes < (1LL << 29);
    {
        const char* v = knob("GAT_BWD_SL");
        sl = sl && (v == nullptr || std::atoi(v) != 0);
    }
    if (sl) {
        const bool dr = drop.thresh != 0u;
#define GAT_BSL(UU, HLV, DR)                                                                   \
    hipLaunchKernelGGL((k_bwd_sources_sl<UU, HLV, DR>), grid, block, 0, st, csc_ptr, csc_dst, \
                       csc_eid, num_nodes, wh, ld_wh, table, ld_t, ds_dst, a_src, c_src, a_dst,   \
                       heads, f, hf, concat, negative_slope, drop, dwh, ld_dwh, partials)
#define GAT_BSL_HL(UU, HLV) \
    if (dr) { GAT_BSL(UU, HLV, true); } else { GAT_BSL(UU, HLV, false); }
#define GAT_BSL_U(UU)                                   \
    if (f == 4) { GAT_BSL_HL(UU, 1) }                    \
    else if (f == 8) { GAT_BSL_HL(UU, 2) }               \
    else { GAT_BSL_HL(UU, 4) }
        if (u == 16) { GAT_BSL_U(16) }
        else { GAT_BSL_U(8) }
#undef GAT_BSL_U
#undef GAT_BSL_HL
#undef GAT_BSL
        return status_of(hipGetLastError());
    }
    switch (g) {
        GAT_BS_U(1) GAT_BS_U(2) GAT_BS_U(4) GAT_BS_U(8) GAT_BS_U(16) GAT_BS_U(32) GAT_BS_U(64)
        default: return GAT_EUNSUPPORTED;
    }
#undef GAT_BS_U
#undef GAT_BS
    return status_of(hipGetLastError());
}

int gat_edge_backward_rows(const int* rowptr, const int* col, const int* row_order,
                           int row_begin, int row_end, const int* csr_to_csc, const float* wh,
                           int ld_wh, const float* s_src, int ld_s, const float* a_src,
                           const float* c_src, const float* s_dst, const float* lse,
                           const float* y_heads, const float* grad_out, int heads, int f,
                           int concat, int score_act, float act_param, float dropout_p,
                           unsigned long long seed, const unsigned long long* seed_dev,
                           float* ds_dst, float* az_csc, int edges_per_row_hint, void* stream) {
    if (score_act < GAT_ACT_LEAKY_RELU || score_act > GAT_ACT_HEAD_SOFTMAX) return GAT_EINVAL;
    if (heads <= 0 || f <= 0 || row_begin < 0 || row_end < row_begin) return GAT_EINVAL;
    const int hf = heads * f;
    if (hf > GAT_MAX_HF || heads > GAT_MAX_HEADS) return GAT_EUNSUPPORTED;
    if (ld_wh < hf || ld_s < heads) return GAT_EINVAL;
    if (!(dropout_p >= 0.f && dropout_p <= 1.f)) return GAT_EINVAL;
    const int rows = row_end - row_begin;
    if (rows == 0) return GAT_OK;
    hipStream_t st = (hipStream_t)stream;
    const DropArgs drop = make_drop(dropout_p, seed, seed_dev);
    float2* az = reinterpret_cast<float2*>(az_csc);
    const int hl = f / 4;
    const bool grp_ok = score_act == GAT_ACT_LEAKY_RELU && act_param >= 0.f && act_param <= 1.f &&
                        f % 4 == 0 && next_pow2(hl) == hl && a_src != nullptr &&
                        c_src != nullptr && (ld_wh & 3) == 0 &&
                        kernel_choice("GAT_BWD_KERNEL", "generic");
    if (grp_ok) {
        const int g = next_pow2(hf / 4);
        const int hint = edges_per_row_hint & ~(GAT_HINT_LOCAL | GAT_HINT_SHORT);
        const int u = hint > 0 && hint <= 12 ? 4 : 8;
        const long long threads = (long long)rows * g;
        const dim3 grid((unsigned)((threads + 255) / 256)), block(256);
#define GAT_BWD_GRP(G, UU)                                                                    \
    hipLaunchKernelGGL((k_edge_bwd_grp<G, UU>), grid, block, 0, st, rowptr, col, row_order,   \
                       row_begin, row_end, csr_to_csc, wh, ld_wh, a_src, c_src, s_dst, lse,   \
                       y_heads, grad_out, heads, f, hf, concat, act_param, drop, ds_dst, az)
        (void)u;  // (the knob-only stored path for LeakyReLU: U = 8)
#define GAT_BWD_GRP_U(G)                       \
    case G:                                    \
        GAT_BWD_GRP(G, 8);                     \
        break;
        switch (g) {
            GAT_BWD_GRP_U(1) GAT_BWD_GRP_U(2) GAT_BWD_GRP_U(4) GAT_BWD_GRP_U(8)
            GAT_BWD_GRP_U(16) GAT_BWD_GRP_U(32) GAT_BWD_GRP_U(64)
            default: return GAT_EUNSUPPORTED;
        }
#undef GAT_BWD_GRP_U
#undef GAT_BWD_GRP
        return status_of(hipGetLastError());
    }
    if (s_src == nullptr) return GAT_EINVAL;
    const dim3 grid(rows), block(kWave);
#define GAT_BWD_ROWS(P)                                                                       \
    case P:                                                                                   \
        hipLaunchKernelGGL((k_edge_bwd_rows<P>), grid, block, 0, st, rowptr, col, row_order,  \
                           row_begin, row_end, csr_to_csc, wh, ld_wh, s_src, ld_s, s_dst, lse, \
                           y_heads, grad_out, heads, f, hf, concat, score_act, act_param,     \
                           drop, ds_dst, az);                                                 \
        break;
    switch (next_pow2(heads)) {
        GAT_BWD_ROWS(1) GAT_BWD_ROWS(2) GAT_BWD_ROWS(4) GAT_BWD_ROWS(8)
        GAT_BWD_ROWS(16) GAT_BWD_ROWS(32) GAT_BWD_ROWS(64)
        default: return GAT_EUNSUPPORTED;
    }
#undef GAT_BWD_ROWS
    return status_of(hipGetLastError());
}

int gat_src_backward(const int* csc_ptr, const int* csc_dst, int num_nodes, const float* wh,
                     int ld_wh, const float* grad_out, const float* az_csc,
                     const float* ds_dst, const float* a_src,
                     const float* a_dst, int heads, int f, int concat, float* dwh, int ld_dwh,
                     float* ds_src, float* partials, int num_parts, void* stream) {
    if (heads <= 0 || f <= 0 || num_nodes < 0 || num_parts <= 0) return GAT_EINVAL;
    const int hf = heads * f;
    if (hf > GAT_MAX_HF || heads > GAT_MAX_HEADS) return GAT_EUNSUPPORTED;
    if (ld_wh < hf || ld_dwh < hf) return GAT_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid(num_parts), block(kWave);
    const int cq = (hf + kWave - 1) / kWave;
#define GAT_SRC_LAUNCH(CQ, P)                                                                 \
    hipLaunchKernelGGL((k_src_bwd<CQ, P>), grid, block, 0, st, csc_ptr, csc_dst, num_nodes,   \
                       wh, ld_wh, grad_out, reinterpret_cast<const float2*>(az_csc), ds_dst,   \
                       a_src, a_dst, heads, f,                                                 \
                       hf, concat, dwh, ld_dwh, ds_src, partials)
#define GAT_SRC_HP(CQ)                                               \
    switch (next_pow2(heads)) {                                      \
        case 1: GAT_SRC_LAUNCH(CQ, 1); break;                        \
        case 2: GAT_SRC_LAUNCH(CQ, 2); break;                        \
        case 4: GAT_SRC_LAUNCH(CQ, 4); break;                        \
        case 8: GAT_SRC_LAUNCH(CQ, 8); break;                        \
        case 16: GAT_SRC_LAUNCH(CQ, 16); break;                      \
        case 32: GAT_SRC_LAUNCH(CQ, 32); break;                      \
        case 64: GAT_SRC_LAUNCH(CQ, 64); break;                      \
        default: return GAT_EUNSUPPORTED;                            \
    }
    switch (cq) {
        case 1: GAT_SRC_HP(1) break;
        case 2: GAT_SRC_HP(2) break;
        case 3: GAT_SRC_HP(3) break;
        case 4: GAT_SRC_HP(4) break;
        default: return GAT_EUNSUPPORTED;
    }
#undef GAT_SRC_HP
#undef GAT_SRC_LAUNCH
    return status_of(hipGetLastError());
}

int gat_weight_grad_workspace_size(int num_nodes, int fin, int hf, size_t* bytes) {
    if (num_nodes < 0 || fin <= 0 || hf <= 0 || bytes == nullptr) return GAT_EINVAL;
    *bytes = (size_t)wgrad_chunks(num_nodes, fin, hf) * hf * fin * sizeof(float);
    return GAT_OK;
}

int gat_weight_grad(const float* x, int num_nodes, int fin, const float* dwh, int ld_dwh, int hf,
                    float* dw, void* workspace, size_t workspace_bytes, void* stream) {
    if (num_nodes < 0 || fin <= 0 || hf <= 0 || ld_dwh < hf) return GAT_EINVAL;
    size_t need = 0;
    int rc = gat_weight_grad_workspace_size(num_nodes, fin, hf, &need);
    if (rc != GAT_OK) return rc;
    if (workspace_bytes < need) return GAT_EWORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    if (num_nodes == 0) return status_of(hipMemsetAsync(dw, 0, sizeof(float) * hf * fin, st));
    const int chunks = wgrad_chunks(num_nodes, fin, hf);
    const int rows = (num_nodes + chunks - 1) / chunks;
    float* part = (float*)workspace;
    const dim3 grid((fin + 63) / 64, chunks, (hf + 63) / 64), block(256);
    // x rows read LW floats at a time where fin and x's alignment allow
    const uintptr_t xa = reinterpret_cast<uintptr_t>(x);
    const int lw = (fin % 4 == 0 && (xa & 15) == 0) ? 4 : (fin % 2 == 0 && (xa & 7) == 0) ? 2 : 1;
    if (lw == 4)
        hipLaunchKernelGGL(k_wgrad<4>, grid, block, 0, st, dwh, ld_dwh, x, num_nodes, fin, hf,
                           rows, part);
    else if (lw == 2)
        hipLaunchKernelGGL(k_wgrad<2>, grid, block, 0, st, dwh, ld_dwh, x, num_nodes, fin, hf,
                           rows, part);
    else
        hipLaunchKernelGGL(k_wgrad<1>, grid, block, 0, st, dwh, ld_dwh, x, num_nodes, fin, hf,
                           rows, part);
    const long long count = (long long)hf * fin;
    hipLaunchKernelGGL(k_colsum, dim3((unsigned)((count + 15) / 16)), dim3(256), 0, st, part,
                       chunks, count, dw, chunks);
    return status_of(hipGetLastError());
}

int gat_input_grad(const float* dwh, int ld_dwh, int num_nodes, int hf, const float* w,
                   int fin, float* dx, int ld_dx, void* stream) {
    if (num_nodes < 0 || fin <= 0 || hf <= 0 || ld_dwh < hf || ld_dx < fin) return GAT_EINVAL;
    if (hf > 128) return GAT_EUNSUPPORTED;
    if (num_nodes == 0) return GAT_OK;
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((num_nodes + 63) / 64), block(256);
    // K = hf padded with zeros to 4 KL
    const int kl = hf <= 8 ? 2 : hf <= 16 ? 4 : hf <= 32 ? 8 : hf <= 64 ? 16 : 32;
#define GAT_DX(KLV)                                                                            \
    hipLaunchKernelGGL(k_dx<KLV>, grid, block, 0, st, dwh, ld_dwh, hf, num_nodes, w, fin, dx, \
                       ld_dx)
    switch (kl) {
        case 2: GAT_DX(2); break;
        case 4: GAT_DX(4); break;
        case 8: GAT_DX(8); break;
        case 16: GAT_DX(16); break;
        default: GAT_DX(32); break;
    }
#undef GAT_DX
    return status_of(hipGetLastError());
}

int gat_sum_partials_workspace_size(int num_parts, long long width, size_t* bytes) {
    if (num_parts <= 0 || width <= 0 || bytes == nullptr) return GAT_EINVAL;
    *bytes = num_parts > 256 ? (size_t)((num_parts + 255) / 256) * width * sizeof(float) : 0;
    return GAT_OK;
}

int gat_sum_partials(const float* partials, int num_parts, long long width, float* out,
                     void* workspace, size_t workspace_bytes, void* stream) {
    size_t need = 0;
    const int rc = gat_sum_partials_workspace_size(num_parts, width, &need);
    if (rc != GAT_OK) return rc;
    if (workspace_bytes < need) return GAT_EWORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    const dim3 gx((unsigned)((width + 15) / 16));
    if (num_parts <= 256) {
        hipLaunchKernelGGL(k_colsum, gx, dim3(256), 0, st, partials, num_parts, width, out,
                           num_parts);
        return status_of(hipGetLastError());
    }
    // two stages: sums of 256-row blocks, then of the block sums (fixed order)
    const int blocks = (num_parts + 255) / 256;
    float* tmp = (float*)workspace;
    hipLaunchKernelGGL(k_colsum, dim3(gx.x, blocks), dim3(256), 0, st, partials, num_parts,
                       width, tmp, 256);
    hipLaunchKernelGGL(k_colsum, gx, dim3(256), 0, st, tmp, blocks, width, out, blocks);
    return status_of(hipGetLastError());
}

}  // extern "C"
