// GNN message passing of gnn_utils.py:5-74 on a destination-sorted CSR graph.
//
//   P      = x . W1'^T            one MFMA GEMM, W1 [H][2F] read as [2H][F] (row stride F), so
//                                 P[v][2q] = W1[q,:F].x_v (target part), P[v][2q+1] = W1[q,F:].x_v
//   alpha  = sigmoid(w2 . relu(P[d][2q] + P[s][2q+1] + b1) + b2)      attn_score_kernel
//   agg[d] = sum_e (alpha_e / sum alpha) x[src_e]                      aggregate kernels (HBM-bound)
//   x'[d]  = x_d + sigmoid(Wg[x_d;agg_d]+bg) * (Wu2 relu(Wu1[x_d;agg_d]+bu1)+bu2)   3 GEMMs,
//            the concatenation [x_d;agg_d] is never materialised (A/A2 K-split + row gather),
//            the gated residual is the last GEMM's epilogue.
#include <stdlib.h>

#include "az_common.h"

namespace az {
int gemm_f32(const az_gemm_desc* d, hipStream_t s);
bool gnn_layer_fusable(const az_graph* g, int F, int H);
bool gnn_layer_band_ok(const az_graph* g, int F, int H);
size_t gnn_layer_band_ws_bytes();
int gnn_layer_band(const az_graph* g, const float* x, const az_gnn_layer_w* w, float* x_out,
                   void* ws, hipStream_t s, const float* const* ot = nullptr);
size_t gnn_layer_fused_ws_bytes(int V);
int gnn_layer_fused(const az_graph* g, const float* x, const az_gnn_layer_w* w, float* x_out,
                    void* ws, size_t ws_bytes, hipStream_t s);
int gnn_layer_fused_kernel_launch(const az_graph* g, const float* x, const float* Ps,
                                  const az_gnn_layer_w* w, float* x_out, hipStream_t s);
int gnn_layer_source_projection(const az_graph* g, const float* x, const az_gnn_layer_w* w,
                                float* Ps, void* ws, size_t ws_bytes, hipStream_t s);

__device__ __forceinline__ int xcd_remap(int b, int n) {
  // give every XCD (blocks b, b+8, ...) one contiguous run of destinations so the
  // neighbour rows a destination gathers are mostly resident in that XCD's L2
  return (n & 7) == 0 ? (b & 7) * (n >> 3) + (b >> 3) : b;
}

// 16 lanes per edge.  P rows interleave (target, source) projections per hidden unit q.
__global__ __launch_bounds__(256) void attn_score_kernel(int E, const int* __restrict__ edge_dst,
                                                        const int* __restrict__ col,
                                                        const float* __restrict__ P, int ldp,
                                                        int H, const float* __restrict__ b1,
                                                        const float* __restrict__ w2,
                                                        const float* __restrict__ b2,
                                                        float* __restrict__ alpha) {
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int e = (blk * 256 + threadIdx.x) >> 4;
  const int l = threadIdx.x & 15;
  if (e >= E) return;  // whole 16-lane groups exit together
  const int d = edge_dst[e], s = col[e];
  const float* pd = P + (size_t)d * ldp;
  const float* ps = P + (size_t)s * ldp;
  float acc = 0.f;
  for (int m = l; m < H / 2; m += 16) {
    const f32x4 t = *reinterpret_cast<const f32x4*>(pd + 4 * m);
    const f32x4 u = *reinterpret_cast<const f32x4*>(ps + 4 * m);
    float h0 = t[0] + u[1] + b1[2 * m];
    float h1 = t[2] + u[3] + b1[2 * m + 1];
    h0 = h0 > 0.f ? h0 : 0.f;
    h1 = h1 > 0.f ? h1 : 0.f;
    acc = fmaf(h0, w2[2 * m], acc);
    acc = fmaf(h1, w2[2 * m + 1], acc);
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 16);
  if (l == 0) alpha[e] = sigmoidf_ref(acc + b2[0]);
}

// Segmented weighted reduce.  LPR lanes own one destination row; each lane covers NV
// float4 column slices per pass (F == 4*LPR*NV exactly for the grid shapes, a loop otherwise).
// Dependent-load chain per destination: rowptr -> (col, alpha) -> x rows; for degree <= 4 (the
// grid) all of a destination's col/alpha loads are issued together, then all its x rows.
template <int LPR, int NV>
__global__ __launch_bounds__(256) void aggregate_lanes_kernel(
    int D, int identity, const int* __restrict__ dst_rows, const int* __restrict__ rowptr,
    const int* __restrict__ col, const float* __restrict__ alpha, const float* __restrict__ x,
    int ldx, int F, float* __restrict__ agg, int ldagg) {
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int i = (blk * 256 + threadIdx.x) / LPR;
  const int l = threadIdx.x % LPR;
  if (i >= D) return;
  const int d = identity ? i : dst_rows[i];
  const int e0 = rowptr[d], e1 = rowptr[d + 1];
  const int deg = e1 - e0;
  if (deg <= 4) {
    int s[4];
    float a[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[j] = j < deg ? col[e0 + j] : 0;
      a[j] = j < deg ? alpha[e0 + j] : 0.f;
    }
    float S = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < deg) S += a[j];
    const bool norm = S > 0.f;
    float w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = norm ? a[j] / S : a[j];
    for (int f0 = l * 4; f0 < F; f0 += LPR * 4 * NV) {
      f32x4 v[4][NV];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < NV; ++q) {
          const int f = f0 + q * LPR * 4;
          v[j][q] = (j < deg && f < F) ? *reinterpret_cast<const f32x4*>(x + (size_t)s[j] * ldx + f)
                                       : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        const int f = f0 + q * LPR * 4;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (j < deg)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[c] = fmaf(w[j], v[j][q][c], acc[c]);
        if (f < F) *reinterpret_cast<f32x4*>(agg + (size_t)d * ldagg + f) = acc;
      }
    }
    return;
  }
  float S = 0.f;
  for (int e = e0; e < e1; ++e) S += alpha[e];
  const bool norm = S > 0.f;
  for (int f = l * 4; f < F; f += LPR * 4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    int e = e0;
    for (; e + 4 <= e1; e += 4) {
      int s[4];
      float w[4];
      f32x4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[j] = col[e + j];
        w[j] = norm ? alpha[e + j] / S : alpha[e + j];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = *reinterpret_cast<const f32x4*>(x + (size_t)s[j] * ldx + f);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = fmaf(w[j], v[j][c], acc[c]);
    }
    for (; e < e1; ++e) {
      const float w = norm ? alpha[e] / S : alpha[e];
      const f32x4 v = *reinterpret_cast<const f32x4*>(x + (size_t)col[e] * ldx + f);
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = fmaf(w, v[c], acc[c]);
    }
    *reinterpret_cast<f32x4*>(agg + (size_t)d * ldagg + f) = acc;
  }
}

// High in-degree form (the reference's star: one destination, N-1 sources, F = 3136): the
// lanes kernel would give one destination to one wave walking all its edges serially.  Here
// block (destination i, 256-column chunk c) splits the destination's edges over its 4 waves in
// contiguous quarters; each wave keeps its quarter's weighted float4 sums, the quarters are
// added in wave order through LDS (deterministic), and sum(alpha) comes from a wave reduction.
__global__ __launch_bounds__(256) void aggregate_wide_kernel(
    int identity, const int* __restrict__ dst_rows, const int* __restrict__ rowptr,
    const int* __restrict__ col, const float* __restrict__ alpha, const float* __restrict__ x,
    int ldx, int F, float* __restrict__ agg, int ldagg) {
  __shared__ f32x4 part[4][64];
  const int i = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int d = identity ? i : dst_rows[i];
  const int e0 = rowptr[d], e1 = rowptr[d + 1];
  const int deg = e1 - e0;
  float S = 0.f;
  for (int e = e0 + lane; e < e1; e += 64) S += alpha[e];
  S = wave_sum(S);
  const bool norm = S > 0.f;
  const int f = blockIdx.y * 256 + lane * 4;
  const int q = (deg + 3) / 4;
  const int eb = e0 + wave * q, ee = min(e1, eb + q);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (f < F) {
    int e = eb;
    for (; e + 4 <= ee; e += 4) {
      int sc[4];
      float w[4];
      f32x4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sc[j] = col[e + j];
        w[j] = norm ? alpha[e + j] / S : alpha[e + j];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = *reinterpret_cast<const f32x4*>(x + (size_t)sc[j] * ldx + f);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = fmaf(w[j], v[j][c], acc[c]);
    }
    for (; e < ee; ++e) {
      const float w = norm ? alpha[e] / S : alpha[e];
      const f32x4 v = *reinterpret_cast<const f32x4*>(x + (size_t)col[e] * ldx + f);
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = fmaf(w, v[c], acc[c]);
    }
  }
  part[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && f < F) {
    f32x4 r = part[0][lane];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const f32x4 t = part[w][lane];
#pragma unroll
      for (int c = 0; c < 4; ++c) r[c] += t[c];
    }
    *reinterpret_cast<f32x4*>(agg + (size_t)d * ldagg + f) = r;
  }
}

// Max in-degree <= 4 (the synthetic grid), F = 64: 8 lanes x 2 float4 per destination row; a lane
// group owns DPT consecutive destinations and issues all their index loads, then all their
// neighbour-row loads, before any math.  NT: agg written with non-temporal stores.
template <int LPR, int NV, int DPT, bool NT>
__global__ __launch_bounds__(256) void aggregate_small_kernel(
    int D, int identity, const int* __restrict__ dst_rows, const int* __restrict__ rowptr,
    const int* __restrict__ col, const float* __restrict__ alpha, const float* __restrict__ x,
    int ldx, int F, float* __restrict__ agg, int ldagg) {
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int grp = (blk * 256 + threadIdx.x) / LPR;
  const int l = threadIdx.x % LPR;
  const int i0 = grp * DPT;
  if (i0 >= D) return;
  int d[DPT], e0[DPT], deg[DPT];
#pragma unroll
  for (int t = 0; t < DPT; ++t) {
    const int i = min(i0 + t, D - 1);
    d[t] = identity ? i : dst_rows[i];
    e0[t] = rowptr[d[t]];
    deg[t] = rowptr[d[t] + 1] - e0[t];
  }
  int sc[DPT][4];
  float a[DPT][4];
#pragma unroll
  for (int t = 0; t < DPT; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sc[t][j] = j < deg[t] ? col[e0[t] + j] : 0;
      a[t][j] = j < deg[t] ? alpha[e0[t] + j] : 0.f;
    }
  f32x4 v[DPT][4][NV];
#pragma unroll
  for (int t = 0; t < DPT; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        const int f = l * 4 + q * LPR * 4;
        v[t][j][q] = (j < deg[t] && f < F)
                         ? *reinterpret_cast<const f32x4*>(x + (size_t)sc[t][j] * ldx + f)
                         : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
  for (int t = 0; t < DPT; ++t) {
    if (i0 + t >= D) break;
    float S = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < deg[t]) S += a[t][j];
    for (int j = 4; j < deg[t]; ++j) S += alpha[e0[t] + j];   // in-degree above 4 (never dropped)
    const bool norm = S > 0.f;
    float w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = norm ? a[t][j] / S : a[t][j];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int f = l * 4 + q * LPR * 4;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (j < deg[t])
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[c] = fmaf(w[j], v[t][j][q][c], acc[c]);
      for (int j = 4; j < deg[t]; ++j) {     // a caller whose max_deg understates the graph
        const float aj = alpha[e0[t] + j];
        const float wj = norm ? aj / S : aj;
        if (f < F) {
          const f32x4 xj = *reinterpret_cast<const f32x4*>(x + (size_t)col[e0[t] + j] * ldx + f);
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[c] = fmaf(wj, xj[c], acc[c]);
        }
      }
      if (f < F) {
        f32x4* dst = reinterpret_cast<f32x4*>(agg + (size_t)d[t] * ldagg + f);
        if constexpr (NT) __builtin_nontemporal_store(acc, dst);
        else *dst = acc;
      }
    }
  }
}

// Attention scores AND the aggregation of one destination in one pass, for the grid (in-degree
// <= 4, F = 64, H = 128): 16 lanes per destination.  The destination's P row (its target
// halves) is read once for all its edges instead of once per edge, the scores never round-trip
// through HBM before the aggregation reads them, and one launch replaces two.  Every
// arithmetic step is attn_score_kernel's (lane l owns hidden pairs m = l, l+16, l+32, l+48,
// the same fmaf order and 16-lane xor reduction) and aggregate_small_kernel's (sum of alpha and
// the weighted sum in edge order), so alpha and agg are bit-identical to the two-kernel path.
__global__ __launch_bounds__(256) void attn_aggregate_small_kernel(
    int D, int identity, const int* __restrict__ dst_rows, const int* __restrict__ rowptr,
    const int* __restrict__ col, const float* __restrict__ P, int ldp,
    const float* __restrict__ b1, const float* __restrict__ w2, const float* __restrict__ b2,
    const float* __restrict__ x, int ldx, float* __restrict__ alpha, float* __restrict__ agg,
    int ldagg) {
  constexpr int H = 128, F = 64;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int i = (blk * 256 + threadIdx.x) >> 4;
  const int l = threadIdx.x & 15;
  if (i >= D) return;  // whole 16-lane groups exit together
  const int d = identity ? i : dst_rows[i];
  const int e0 = rowptr[d];
  const int deg = rowptr[d + 1] - e0;
  int sc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) sc[j] = j < deg ? col[e0 + j] : d;
  // every load issued before any math: target chunks, neighbour chunks, neighbour x rows
  f32x4 t[4], u[4][4], xv[4];
  const float* pd = P + (size_t)d * ldp;
#pragma unroll
  for (int k = 0; k < 4; ++k) t[k] = *reinterpret_cast<const f32x4*>(pd + 4 * (l + 16 * k));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float* ps = P + (size_t)sc[j] * ldp;
#pragma unroll
    for (int k = 0; k < 4; ++k) u[j][k] = *reinterpret_cast<const f32x4*>(ps + 4 * (l + 16 * k));
    xv[j] = *reinterpret_cast<const f32x4*>(x + (size_t)sc[j] * ldx + 4 * l);
  }
  float bb[8], ww[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int m = l + 16 * k;
    bb[2 * k] = b1[2 * m];
    bb[2 * k + 1] = b1[2 * m + 1];
    ww[2 * k] = w2[2 * m];
    ww[2 * k + 1] = w2[2 * m + 1];
  }
  const float bias2 = b2[0];
  float a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float h0 = t[k][0] + u[j][k][1] + bb[2 * k];
      float h1 = t[k][2] + u[j][k][3] + bb[2 * k + 1];
      h0 = h0 > 0.f ? h0 : 0.f;
      h1 = h1 > 0.f ? h1 : 0.f;
      acc = fmaf(h0, ww[2 * k], acc);
      acc = fmaf(h1, ww[2 * k + 1], acc);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 16);
    a[j] = sigmoidf_ref(acc + bias2);
  }
  if (l < deg && l < 4) {   // lane j writes edge j's score
    const float aj = l == 0 ? a[0] : (l == 1 ? a[1] : (l == 2 ? a[2] : a[3]));
    alpha[e0 + l] = aj;
  }
  // in-degree above 4 (a caller's az_graph.max_deg understating the graph): the remaining
  // edges' scores from global memory, in CSR order -- slower, never dropped
  auto alpha_far = [&](int q) {
    const float* ps = P + (size_t)col[e0 + q] * ldp;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const f32x4 uq = *reinterpret_cast<const f32x4*>(ps + 4 * (l + 16 * k));
      float h0 = t[k][0] + uq[1] + bb[2 * k];
      float h1 = t[k][2] + uq[3] + bb[2 * k + 1];
      h0 = h0 > 0.f ? h0 : 0.f;
      h1 = h1 > 0.f ? h1 : 0.f;
      acc = fmaf(h0, ww[2 * k], acc);
      acc = fmaf(h1, ww[2 * k + 1], acc);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 16);
    return sigmoidf_ref(acc + bias2);
  };
  float S = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (j < deg) S += a[j];
  for (int q = 4; q < deg; ++q) {
    const float aq = alpha_far(q);
    if (l == 0) alpha[e0 + q] = aq;
    S += aq;
  }
  const bool norm = S > 0.f;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (j < deg) {
      const float w = norm ? a[j] / S : a[j];
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = fmaf(w, xv[j][c], acc[c]);
    }
  for (int q = 4; q < deg; ++q) {
    const float aq = alpha_far(q);
    const float w = norm ? aq / S : aq;
    const f32x4 xq = *reinterpret_cast<const f32x4*>(x + (size_t)col[e0 + q] * ldx + 4 * l);
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = fmaf(w, xq[c], acc[c]);
  }
  (void)H;
  (void)F;
  __builtin_nontemporal_store(acc, reinterpret_cast<f32x4*>(agg + (size_t)d * ldagg + 4 * l));
}

template <int LPR, int NV>
static void launch_aggregate(const az_graph* g, int identity, const float* x, int ldx, int F,
                             const float* alpha, float* agg, int ldagg, hipStream_t s) {
  const long threads = (long)g->D * LPR;
  const int blocks = (int)((threads + 255) / 256);
  hipLaunchKernelGGL((aggregate_lanes_kernel<LPR, NV>), dim3(blocks), dim3(256), 0, s, g->D,
                     identity, g->dst_rows, g->rowptr, g->col, alpha, x, ldx, F, agg, ldagg);
}

int aggregate(const az_graph* g, const float* x, int ldx, int F, const float* alpha, float* agg,
              int ldagg, hipStream_t s) {
  if (g->D == 0) return AZ_OK;
  const int identity = (g->D == g->V) ? 1 : 0;
  // few destinations with many in-edges each (the star of a training batch): spread every
  // destination's edges over a block instead of walking them in one wave
  if ((long)g->D * F < 65536 && g->E >= 16L * g->D) {
    hipLaunchKernelGGL(aggregate_wide_kernel, dim3(g->D, (F + 255) / 256), dim3(256), 0, s,
                       identity, g->dst_rows, g->rowptr, g->col, alpha, x, ldx, F, agg, ldagg);
    return check_launch("aggregate_wide_kernel");
  }
  static const char* env = tuning_env("AZ_AGG_CFG");   // tuning experiments only
  const int cfg = env ? atoi(env) : 0;
  if (g->max_deg > 0 && g->max_deg <= 4 && F == 64 && cfg != 9) {
    // the grid: non-temporal agg stores keep the gathered x rows resident in L2 / Infinity
    // Cache instead of the stream of outputs (tools/agg_sweep.py: 67 -> 42 us on the 512-grid
    // shard, unchanged at 4096 grids where x alone exceeds the 256 MB cache)
    const int dpt = cfg == 2 ? 2 : 1;
    const long groups = ((long)g->D + dpt - 1) / dpt;
    const int blocks = (int)((groups * 8 + 255) / 256);
    if (dpt == 2)
      hipLaunchKernelGGL((aggregate_small_kernel<8, 2, 2, true>), dim3(blocks), dim3(256), 0, s,
                         g->D, identity, g->dst_rows, g->rowptr, g->col, alpha, x, ldx, F, agg,
                         ldagg);
    else
      hipLaunchKernelGGL((aggregate_small_kernel<8, 2, 1, true>), dim3(blocks), dim3(256), 0, s,
                         g->D, identity, g->dst_rows, g->rowptr, g->col, alpha, x, ldx, F, agg,
                         ldagg);
    return check_launch("aggregate_small_kernel");
  }
  if (F <= 32) launch_aggregate<8, 1>(g, identity, x, ldx, F, alpha, agg, ldagg, s);
  else if (F <= 64) launch_aggregate<8, 2>(g, identity, x, ldx, F, alpha, agg, ldagg, s);
  else if (F <= 128) launch_aggregate<16, 2>(g, identity, x, ldx, F, alpha, agg, ldagg, s);
  else launch_aggregate<64, 1>(g, identity, x, ldx, F, alpha, agg, ldagg, s);
  return check_launch("aggregate_lanes_kernel");
}

int attn_score(const az_graph* g, const float* P, int ldp, int H, const float* b1,
               const float* w2, const float* b2, float* alpha, hipStream_t s) {
  if (g->E == 0) return AZ_OK;
  const int blocks = (int)(((long)g->E * 16 + 255) / 256);
  hipLaunchKernelGGL(attn_score_kernel, dim3(blocks), dim3(256), 0, s, g->E, g->edge_dst, g->col,
                     P, ldp, H, b1, w2, b2, alpha);
  return check_launch("attn_score_kernel");
}

static int check_graph(const az_graph* g) {
  AZ_REQUIRE(g && g->V >= 0 && g->E >= 0 && g->D >= 0 && g->D <= g->V, AZ_EINVAL,
             "az_graph: bad sizes");
  AZ_REQUIRE(g->rowptr && (g->E == 0 || (g->col && g->edge_dst)) && (g->D == 0 || g->dst_rows),
             AZ_EINVAL, "az_graph: null arrays");
  return AZ_OK;
}

static size_t align256(size_t b) { return (b + 255) & ~size_t(255); }

constexpr size_t kSplitWsBytes = size_t(40) << 20;  // stream-K partial slots for the layer GEMMs

struct LayerWs {
  float *P, *alpha, *agg, *gate, *u1, *u;
  void* split;
};

static LayerWs carve(void* ws, int V, int E, int D, int F, int H) {
  char* p = static_cast<char*>(ws);
  LayerWs w;
  w.P = reinterpret_cast<float*>(p); p += align256((size_t)V * 2 * H * 4);
  w.alpha = reinterpret_cast<float*>(p); p += align256((size_t)E * 4);
  w.agg = reinterpret_cast<float*>(p); p += align256((size_t)V * F * 4);
  w.gate = reinterpret_cast<float*>(p); p += align256((size_t)D * F * 4);
  w.u1 = reinterpret_cast<float*>(p); p += align256((size_t)D * F * 4);
  w.u = reinterpret_cast<float*>(p); p += align256((size_t)D * F * 4);
  w.split = p;
  return w;
}

// Activations the backward pass reads back from a forward workspace (az_backward.hip).
struct FwdSaved {
  const float *P, *alpha, *agg, *gate, *u1, *u;
};
FwdSaved fwd_saved(const void* ws, int V, int E, int D, int F, int H) {
  LayerWs L = carve(const_cast<void*>(ws), V, E, D, F, H);
  return FwdSaved{L.P, L.alpha, L.agg, L.gate, L.u1, L.u};
}

// GNNLayer's gated node update (gnn_utils.py:18-28 gate / update_net, :67-74) for the D
// destinations (rows dst_rows, or every row when D == V): c = [x_d ; agg_d],
// gate = sigmoid(Wg c + bg), u1 = relu(Wu1 c + bu1), u = Wu2 u1 + bu2 (kept, pre-gate, for the
// backward pass), x_out[d] = x[d] + gate * u.  Rows of x_out outside the destinations are the
// caller's (az_gnn_layer_fwd / az_gnn_node_update_fwd copy x there first).
int node_update(const float* x, const float* agg, int V, int F, int D, const int* dst_rows,
                const float* gate_w, const float* gate_b, const float* upd_w1,
                const float* upd_b1, const float* upd_w2, const float* upd_b2, float* x_out,
                float* gate, float* u1, float* u, void* split, size_t split_bytes,
                hipStream_t s) {
  int rc;
  az_gemm_desc c = {};
  c.M = D; c.N = F; c.K = 2 * F;
  c.A = x; c.lda = F; c.a_kmajor = 1; c.A2 = agg; c.lda2 = F; c.K0 = F;
  c.a_rows = (D == V) ? nullptr : dst_rows;
  c.b_kmajor = 1; c.ldb = 2 * F; c.ldc = F;
  c.ws = split; c.ws_bytes = split_bytes;
  c.B = gate_w; c.bias = gate_b; c.act = AZ_ACT_SIGMOID; c.C = gate;
  if ((rc = gemm_f32(&c, s))) return rc;
  c.B = upd_w1; c.bias = upd_b1; c.act = AZ_ACT_RELU; c.C = u1;
  if ((rc = gemm_f32(&c, s))) return rc;
  az_gemm_desc o = {};
  o.M = D; o.N = F; o.K = F;
  o.A = u1; o.lda = F; o.a_kmajor = 1;
  o.B = upd_w2; o.ldb = F; o.b_kmajor = 1; o.bias = upd_b2;
  o.R = x; o.ldr = F; o.G = gate; o.ldg = F;
  o.C2 = u; o.ldc2 = F;  // pre-gate update, kept for the backward pass
  o.C = x_out; o.ldc = F; o.c_rows = (D == V) ? nullptr : dst_rows;
  o.ws = split; o.ws_bytes = split_bytes;
  return gemm_f32(&o, s);
}

}  // namespace az

using namespace az;

extern "C" int az_gnn_attn_score_fwd(const az_graph* g, const float* P, int ldp, int H,
                                     const float* b1, const float* w2, const float* b2,
                                     float* alpha, void* stream) {
  int rc = check_graph(g);
  if (rc) return rc;
  AZ_REQUIRE(H > 0 && H % 2 == 0 && ldp % 4 == 0 && ldp >= 2 * H && aligned16(P), AZ_EINVAL,
             "az_gnn_attn_score_fwd: P needs [V][>=2H] rows, 16B aligned");
  AZ_REQUIRE(b1 && w2 && b2 && alpha, AZ_EINVAL, "az_gnn_attn_score_fwd: null");
  return attn_score(g, P, ldp, H, b1, w2, b2, alpha, as_stream(stream));
}

extern "C" int az_gnn_aggregate_fwd(const az_graph* g, const float* x, int ldx, int F,
                                    const float* alpha, float* agg, int ldagg, void* stream) {
  int rc = check_graph(g);
  if (rc) return rc;
  AZ_REQUIRE(F > 0 && F % 4 == 0 && ldx % 4 == 0 && ldagg % 4 == 0 && aligned16(x) &&
                 aligned16(agg),
             AZ_EINVAL, "az_gnn_aggregate_fwd: F, strides %%4 and 16B alignment required");
  AZ_REQUIRE(alpha || g->E == 0, AZ_EINVAL, "az_gnn_aggregate_fwd: null alpha");
  return aggregate(g, x, ldx, F, alpha, agg, ldagg, as_stream(stream));
}

extern "C" size_t az_gnn_layer_ws_bytes(int V, int E, int D, int F, int H) {
  return align256((size_t)V * 2 * H * 4) + align256((size_t)E * 4) + align256((size_t)V * F * 4) +
         align256((size_t)D * F * 4) * 3 + kSplitWsBytes;
}

extern "C" int az_gnn_layer_fwd(const az_graph* g, const float* x, int F, int H,
                                const az_gnn_layer_w* w, float* x_out, void* ws, size_t ws_bytes,
                                void* stream) {
  int rc = check_graph(g);
  if (rc) return rc;
  AZ_REQUIRE(x && x_out && w && ws && x != x_out, AZ_EINVAL, "az_gnn_layer_fwd: bad pointers");
  AZ_REQUIRE(F % 16 == 0 && H % 4 == 0, AZ_EINVAL, "az_gnn_layer_fwd: F%%16, H%%4 required");
  AZ_REQUIRE(ws_bytes >= az_gnn_layer_ws_bytes(g->V, g->E, g->D, F, H), AZ_EINVAL,
             "az_gnn_layer_fwd: workspace too small");
  hipStream_t s = as_stream(stream);
  LayerWs L = carve(ws, g->V, g->E, g->D, F, H);
  if (g->D < g->V) {
    if (hipMemcpyAsync(x_out, x, (size_t)g->V * F * 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
      return check_launch("hipMemcpyAsync");
  }
  if (g->D == 0) return AZ_OK;
  // 1. attention projections for every node: P = x . W1'^T (W1 read as [2H][F])
  az_gemm_desc d = {};
  d.M = g->V; d.N = 2 * H; d.K = F;
  d.A = x; d.lda = F; d.a_kmajor = 1;
  d.B = w->att_w1; d.ldb = F; d.b_kmajor = 1;
  d.C = L.P; d.ldc = 2 * H;
  d.ws = L.split; d.ws_bytes = kSplitWsBytes;
  if ((rc = gemm_f32(&d, s))) return rc;
  // 2. per-edge attention weights, 3. normalised aggregation (one fused pass on the grid)
  static const bool no_fuse = tuning_env("AZ_GNN_NOFUSE") != nullptr;   // A/B experiments
  if (!no_fuse && g->max_deg > 0 && g->max_deg <= 4 && F == 64 && H == 128) {
    const int identity = (g->D == g->V) ? 1 : 0;
    const int blocks = (int)(((long)g->D * 16 + 255) / 256);
    hipLaunchKernelGGL(attn_aggregate_small_kernel, dim3(blocks), dim3(256), 0, s, g->D, identity,
                       g->dst_rows, g->rowptr, g->col, L.P, 2 * H, w->att_b1, w->att_w2,
                       w->att_b2, x, F, L.alpha, L.agg, F);
    if ((rc = check_launch("attn_aggregate_small_kernel"))) return rc;
  } else {
    if ((rc = attn_score(g, L.P, 2 * H, H, w->att_b1, w->att_w2, w->att_b2, L.alpha, s)))
      return rc;
    if ((rc = aggregate(g, x, F, F, L.alpha, L.agg, F, s))) return rc;
  }
  // 4.-5. the gated node update of the D destinations
  return node_update(x, L.agg, g->V, F, g->D, g->dst_rows, w->gate_w, w->gate_b, w->upd_w1,
                     w->upd_b1, w->upd_w2, w->upd_b2, x_out, L.gate, L.u1, L.u, L.split,
                     kSplitWsBytes, s);
}

extern "C" size_t az_gnn_node_update_ws_bytes(int D, int F) {
  (void)D;
  (void)F;
  return kSplitWsBytes;
}

extern "C" int az_gnn_node_update_fwd(const float* x, const float* agg, int V, int F, int D,
                                      const int* dst_rows, const float* gate_w,
                                      const float* gate_b, const float* upd_w1,
                                      const float* upd_b1, const float* upd_w2,
                                      const float* upd_b2, float* x_out, float* save, void* ws,
                                      size_t ws_bytes, void* stream) {
  AZ_REQUIRE(V >= 0 && D >= 0 && D <= V && F > 0 && F % 16 == 0, AZ_EINVAL,
             "az_gnn_node_update_fwd: V=%d D=%d F=%d (D <= V, F %% 16)", V, D, F);
  if (V == 0) return AZ_OK;
  AZ_REQUIRE(x && agg && x_out && save && ws && x != x_out && (D == V || dst_rows), AZ_EINVAL,
             "az_gnn_node_update_fwd: bad pointers");
  AZ_REQUIRE(gate_w && gate_b && upd_w1 && upd_b1 && upd_w2 && upd_b2, AZ_EINVAL,
             "az_gnn_node_update_fwd: null weight");
  AZ_REQUIRE(ws_bytes >= az_gnn_node_update_ws_bytes(D, F), AZ_EINVAL,
             "az_gnn_node_update_fwd: workspace too small");
  hipStream_t s = as_stream(stream);
  if (D < V &&
      hipMemcpyAsync(x_out, x, (size_t)V * F * 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return check_launch("hipMemcpyAsync");
  if (D == 0) return AZ_OK;
  const size_t DF = (size_t)D * F;
  return node_update(x, agg, V, F, D, dst_rows, gate_w, gate_b, upd_w1, upd_b1, upd_w2, upd_b2,
                     x_out, save, save + DF, save + 2 * DF, ws, ws_bytes, s);
}

extern "C" size_t az_gnn_layer_infer_ws_bytes(const az_graph* g, int F, int H) {
  if (!g) return 0;
  if (gnn_layer_band_ok(g, F, H)) return gnn_layer_band_ws_bytes();
  return gnn_layer_fusable(g, F, H) ? gnn_layer_fused_ws_bytes(g->V)
                                    : az_gnn_layer_ws_bytes(g->V, g->E, g->D, F, H);
}

extern "C" int az_gnn_layer_infer(const az_graph* g, const float* x, int F, int H,
                                  const az_gnn_layer_w* w, float* x_out, void* ws,
                                  size_t ws_bytes, void* stream) {
  int rc = check_graph(g);
  if (rc) return rc;
  if (gnn_layer_band_ok(g, F, H)) {
    AZ_REQUIRE(x && w && x_out && x_out != x && ws, AZ_EINVAL,
               "az_gnn_layer_infer: null pointer or x_out aliasing x");
    AZ_REQUIRE(ws_bytes >= gnn_layer_band_ws_bytes(), AZ_EINVAL,
               "az_gnn_layer_infer: workspace too small");
    return gnn_layer_band(g, x, w, x_out, ws, as_stream(stream));
  }
  if (!gnn_layer_fusable(g, F, H))
    return az_gnn_layer_fwd(g, x, F, H, w, x_out, ws, ws_bytes, stream);
  AZ_REQUIRE(x && x_out && w && ws && x != x_out, AZ_EINVAL, "az_gnn_layer_infer: bad pointers");
  AZ_REQUIRE(aligned16(x) && aligned16(x_out) && aligned16(ws), AZ_EINVAL,
             "az_gnn_layer_infer: x, x_out, ws need 16B alignment");
  AZ_REQUIRE(w->att_w1 && w->att_b1 && w->att_w2 && w->att_b2 && w->upd_w1 && w->upd_b1 &&
                 w->upd_w2 && w->upd_b2 && w->gate_w && w->gate_b,
             AZ_EINVAL, "az_gnn_layer_infer: null weight");
  AZ_REQUIRE(ws_bytes >= az_gnn_layer_infer_ws_bytes(g, F, H), AZ_EINVAL,
             "az_gnn_layer_infer: workspace too small");
  hipStream_t s = as_stream(stream);
  if (g->D < g->V) {
    if (hipMemcpyAsync(x_out, x, (size_t)g->V * F * 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
      return check_launch("hipMemcpyAsync");
  }
  return gnn_layer_fused(g, x, w, x_out, ws, ws_bytes, s);
}

extern "C" size_t az_gnn_layer_ot_infer_ws_bytes(const az_graph* g, int F, int H) {
  if (!g) return 0;
  if (gnn_layer_band_ok(g, F, H)) return gnn_layer_band_ws_bytes();
  // the layer's output and output_transform's hidden activations, then the layer's workspace
  const size_t act = ((size_t)g->V * F * 4 + 255) / 256 * 256;
  return 2 * act + az_gnn_layer_infer_ws_bytes(g, F, H) + kSplitWsBytes;
}

extern "C" int az_gnn_layer_ot_infer(const az_graph* g, const float* x, int F, int H,
                                     const az_gnn_layer_w* w, const float* ot_w0,
                                     const float* ot_b0, const float* ot_w2, const float* ot_b2,
                                     float* y, void* ws, size_t ws_bytes, void* stream) {
  int rc = check_graph(g);
  if (rc) return rc;
  AZ_REQUIRE(x && w && y && y != x && ws && ot_w0 && ot_b0 && ot_w2 && ot_b2, AZ_EINVAL,
             "az_gnn_layer_ot_infer: null pointer or y aliasing x");
  AZ_REQUIRE(ws_bytes >= az_gnn_layer_ot_infer_ws_bytes(g, F, H), AZ_EINVAL,
             "az_gnn_layer_ot_infer: workspace too small");
  if (gnn_layer_band_ok(g, F, H)) {
    const float* const ot[4] = {ot_w0, ot_b0, ot_w2, ot_b2};
    return gnn_layer_band(g, x, w, y, ws, as_stream(stream), ot);
  }
  const size_t act = ((size_t)g->V * F * 4 + 255) / 256 * 256;
  float* layer_out = static_cast<float*>(ws);
  float* hidden = reinterpret_cast<float*>(static_cast<char*>(ws) + act);
  char* rest = static_cast<char*>(ws) + 2 * act;
  const size_t rest_bytes = ws_bytes - 2 * act;
  if ((rc = az_gnn_layer_infer(g, x, F, H, w, layer_out, rest, rest_bytes, stream))) return rc;
  return az_mlp2_fwd(layer_out, g->V, F, ot_w0, ot_b0, ot_w2, ot_b2, hidden, y, rest,
                     rest_bytes, stream);
}

extern "C" int az_gnn_source_proj_fwd(const az_graph* g, const float* x, int F, int H,
                                      const az_gnn_layer_w* w, float* Ps, void* ws,
                                      size_t ws_bytes, void* stream) {
  int rc = check_graph(g);
  if (rc) return rc;
  AZ_REQUIRE(gnn_layer_fusable(g, F, H), AZ_EINVAL,
             "az_gnn_source_proj_fwd: only the fused shapes (F 64, H 128, in-degree <= 4)");
  AZ_REQUIRE(x && w && w->att_w1 && Ps && aligned16(x) && aligned16(Ps), AZ_EINVAL,
             "az_gnn_source_proj_fwd: bad pointers");
  return gnn_layer_source_projection(g, x, w, Ps, ws, ws_bytes, as_stream(stream));
}

extern "C" int az_gnn_layer_fused_fwd(const az_graph* g, const float* x, const float* Ps, int F,
                                      int H, const az_gnn_layer_w* w, float* x_out,
                                      void* stream) {
  int rc = check_graph(g);
  if (rc) return rc;
  AZ_REQUIRE(gnn_layer_fusable(g, F, H), AZ_EINVAL,
             "az_gnn_layer_fused_fwd: only F 64, H 128, in-degree <= 4");
  AZ_REQUIRE(x && Ps && x_out && w && x != x_out && aligned16(x) && aligned16(Ps) &&
                 aligned16(x_out),
             AZ_EINVAL, "az_gnn_layer_fused_fwd: bad pointers");
  AZ_REQUIRE(w->att_w1 && w->att_b1 && w->att_w2 && w->att_b2 && w->upd_w1 && w->upd_b1 &&
                 w->upd_w2 && w->upd_b2 && w->gate_w && w->gate_b,
             AZ_EINVAL, "az_gnn_layer_fused_fwd: null weight");
  hipStream_t s = as_stream(stream);
  if (g->D < g->V) {
    if (hipMemcpyAsync(x_out, x, (size_t)g->V * F * 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
      return check_launch("hipMemcpyAsync");
  }
  return gnn_layer_fused_kernel_launch(g, x, Ps, w, x_out, s);
}

extern "C" int az_mlp2_fwd(const float* x, int M, int F, const float* w0, const float* b0,
                           const float* w2, const float* b2, float* hidden, float* y, void* ws,
                           size_t ws_bytes, void* stream) {
  AZ_REQUIRE(x && w0 && b0 && w2 && b2 && hidden && y, AZ_EINVAL, "az_mlp2_fwd: null");
  hipStream_t s = as_stream(stream);
  az_gemm_desc d = {};
  d.M = M; d.N = F; d.K = F;
  d.A = x; d.lda = F; d.a_kmajor = 1;
  d.B = w0; d.ldb = F; d.b_kmajor = 1; d.bias = b0; d.act = AZ_ACT_RELU;
  d.C = hidden; d.ldc = F;
  d.ws = ws; d.ws_bytes = ws ? ws_bytes : 0;
  int rc = gemm_f32(&d, s);
  if (rc) return rc;
  d.A = hidden; d.B = w2; d.bias = b2; d.act = AZ_ACT_NONE; d.C = y;
  return gemm_f32(&d, s);
}
