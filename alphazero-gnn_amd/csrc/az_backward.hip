// Backward pass of the hot path (Connect4GNN.py:140-197 / TicTacToeGNN.py:206-264):
// losses -> heads -> [output_transform -> GNN layers] -> conv trunk, all deterministic
// (fixed-order reductions, no float atomics).  Dense products go through az_gemm_f32.
#include <stdlib.h>

#include <algorithm>

#include "az_common.h"

namespace az {
int gemm_f32(const az_gemm_desc* d, hipStream_t s);

// Forward-workspace views (az_gnn.hip carve()): what az_gnn_layer_fwd kept for us.
struct FwdSaved {
  const float *P, *alpha, *agg, *gate, *u1, *u;
};
FwdSaved fwd_saved(const void* ws, int V, int E, int D, int F, int H);

// ------------------------------------------------------------------------------ losses
// l_pi = -sum(pi * logp) / Bn ; l_v = sum((z - v)^2) / Bn     (Connect4GNN.py:150-152)
// d l / d logits_j = (softmax_j * sum_a pi_a - pi_j) / Bn     (log_softmax backward)
// d l / d pre_v    = -2 (z - v) / Bn * (1 - v^2)              (tanh backward on its output)
__global__ __launch_bounds__(256) void heads_loss_bwd_kernel(
    const float* __restrict__ logp, const float* __restrict__ v, const float* __restrict__ tpi,
    const float* __restrict__ tv, int B, int A, float inv_bn, float* __restrict__ dlog,
    float* __restrict__ dvpre, float* __restrict__ lrow) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  if (row >= B) return;
  float spi = 0.f, lp = 0.f;
  for (int a = 0; a < A; ++a) spi += tpi[(size_t)row * A + a];
  for (int a = 0; a < A; ++a) {
    const float l = logp[(size_t)row * A + a], t = tpi[(size_t)row * A + a];
    dlog[(size_t)row * A + a] = (expf(l) * spi - t) * inv_bn;
    lp = fmaf(t, l, lp);
  }
  const float vv = v[row], d = tv[row] - vv;
  dvpre[row] = -2.f * d * inv_bn * (1.f - vv * vv);
  if (lrow) {
    lrow[2 * row] = -lp * inv_bn;
    lrow[2 * row + 1] = d * d * inv_bn;
  }
}

// ------------------------------------------------------------------------------ heads bwd
// One wave per 256-column slice of K (lane = float4).  Rows are swept in order:
//   dwp[a][k] = sum_b dlog[b][a] hp[b][k]       dwv[k] = sum_b dvpre[b] hv[b][k]
//   dhp[b][k] = sum_a dlog[b][a] wp[a][k] (+ dvpre[b] wv[k] when dhv == dhp)
template <int AMAX>
__global__ __launch_bounds__(64) void heads_bwd_kernel(
    const float* __restrict__ dlog, const float* __restrict__ dvpre, const float* hp, int ldhp,
    const float* hv, int ldhv, int B, int K, const float* __restrict__ wp, int A,
    const float* __restrict__ wv, float* dwp, float* dwv, float* dhp, int lddhp, float* dhv,
    int lddhv) {
  const int lane = threadIdx.x;
  const int k = blockIdx.x * 256 + lane * 4;
  if (k >= K) return;
  const bool same_in = (hp == hv && ldhp == ldhv);
  const bool fused_out = (dhp == dhv);
  f32x4 w[AMAX], wvv = {0.f, 0.f, 0.f, 0.f};
  f32x4 gw[AMAX], gv = {0.f, 0.f, 0.f, 0.f};
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int a = 0; a < AMAX; ++a) {
    w[a] = (dhp && a < A) ? *reinterpret_cast<const f32x4*>(wp + (size_t)a * K + k) : z;
    gw[a] = z;
  }
  if (dhv) wvv = *reinterpret_cast<const f32x4*>(wv + k);
  for (int b = 0; b < B; ++b) {
    float dl[AMAX];
#pragma unroll
    for (int a = 0; a < AMAX; ++a) dl[a] = a < A ? dlog[(size_t)b * A + a] : 0.f;
    const float dv = dvpre[b];
    if (dwp) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(hp + (size_t)b * ldhp + k);
      const f32x4 y = same_in ? x : *reinterpret_cast<const f32x4*>(hv + (size_t)b * ldhv + k);
#pragma unroll
      for (int a = 0; a < AMAX; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) gw[a][c] = fmaf(dl[a], x[c], gw[a][c]);
#pragma unroll
      for (int c = 0; c < 4; ++c) gv[c] = fmaf(dv, y[c], gv[c]);
    }
    if (dhp) {
      f32x4 o = z;
#pragma unroll
      for (int a = 0; a < AMAX; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) o[c] = fmaf(dl[a], w[a][c], o[c]);
      if (fused_out) {
#pragma unroll
        for (int c = 0; c < 4; ++c) o[c] = fmaf(dv, wvv[c], o[c]);
      } else if (dhv) {
        f32x4 ov;
#pragma unroll
        for (int c = 0; c < 4; ++c) ov[c] = dv * wvv[c];
        *reinterpret_cast<f32x4*>(dhv + (size_t)b * lddhv + k) = ov;
      }
      *reinterpret_cast<f32x4*>(dhp + (size_t)b * lddhp + k) = o;
    }
  }
  if (dwp) {
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
      if (a < A) *reinterpret_cast<f32x4*>(dwp + (size_t)a * K + k) = gw[a];
    *reinterpret_cast<f32x4*>(dwv + k) = gv;
  }
}

// ------------------------------------------------------------------------------ column sums
// out[j] = beta*out[j] + sum_i X[i][j], two fixed-order passes (bias gradients).
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ X, int R,
                                                            int C, int ldx, int rows_per,
                                                            float* __restrict__ part) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int ch = blockIdx.y;
  if (j >= C) return;
  const int r0 = ch * rows_per, r1 = min(R, r0 + rows_per);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int r = r0;
  for (; r + 4 <= r1; r += 4) {
    s0 += X[(size_t)r * ldx + j];
    s1 += X[(size_t)(r + 1) * ldx + j];
    s2 += X[(size_t)(r + 2) * ldx + j];
    s3 += X[(size_t)(r + 3) * ldx + j];
  }
  for (; r < r1; ++r) s0 += X[(size_t)r * ldx + j];
  part[(size_t)ch * C + j] = (s0 + s1) + (s2 + s3);
}

// out[j] = beta*out[j] + sum_c part[c*stride + j] for j < ncols (fixed order over chunks)
__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ part,
                                                          int nch, int stride, int ncols,
                                                          float beta, float* __restrict__ out) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= ncols) return;
  float s = 0.f;
  for (int c = 0; c < nch; ++c) s += part[(size_t)c * stride + j];
  out[j] = (beta != 0.f ? beta * out[j] : 0.f) + s;
}

static int colsum_chunks(int R) { return std::max(1, std::min((R + 1023) / 1024, 1024)); }

int colsum(const float* X, int R, int C, int ldx, float* out, float beta, float* part,
           hipStream_t s) {
  const int nch = colsum_chunks(R);
  const int rows_per = (R + nch - 1) / nch;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((C + 255) / 256, nch), dim3(256), 0, s, X, R, C,
                     ldx, rows_per, part);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((C + 255) / 256), dim3(256), 0, s, part, nch, C, C,
                     beta, out);
  return check_launch("colsum");
}

// ------------------------------------------------------------------------------ dropout
// Counter-based keep mask (splitmix64 of seed, element index): keep with prob 1-p.
// Applied like F.dropout: y = x * (keep / (1-p)) (Connect4Net.py:52).
__device__ __forceinline__ uint32_t mix32(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (uint32_t)(x >> 32);
}

__global__ __launch_bounds__(256) void dropout_mask_kernel(uint8_t* __restrict__ mask, long n,
                                                          uint64_t seed, uint32_t thresh) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    mask[i] = mix32(seed * 0x100000001B3ull ^ (uint64_t)i) >= thresh ? 1 : 0;
}

__global__ __launch_bounds__(256) void mask_scale_kernel(const float* __restrict__ x,
                                                        const uint8_t* __restrict__ mask,
                                                        float scale, long n,
                                                        float* __restrict__ y) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    y[i] = mask[i] ? x[i] * scale : 0.f;
}

// ------------------------------------------------------------------------------ conv trunk bwd
// dz[b*HW + p][c] = dy[b][c*HW + p] * (mask ? mask*scale : 1) * (y > 0)
// (ReLU + optional dropout backward, NCHW -> position-major for the im2col GEMMs)
__global__ __launch_bounds__(256) void nchw_drelu_to_pm_kernel(
    const float* __restrict__ dy, const float* __restrict__ y, const uint8_t* __restrict__ mask,
    float scale, int B, int C, int HW, float* __restrict__ dz) {
  const long total = (long)B * C * HW;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = i % C;
    const long bp = i / C;
    const int p = bp % HW;
    const long b = bp / HW;
    const long src = (b * C + c) * HW + p;
    float g = dy[src];
    if (mask) g = mask[src] ? g * scale : 0.f;
    dz[i] = y[src] > 0.f ? g : 0.f;
  }
}

// cols[(b*Ho + y)*Wo + x][c*9 + kh*3 + kw] = in[b][c][y+kh-pad][x+kw-pad] (0 outside), row
// stride ldc >= C*9 (tail zero-filled).
template <bool IN_I8>
__global__ __launch_bounds__(256) void im2col3x3_kernel(const void* __restrict__ in_, int B, int C,
                                                       int H, int W, int pad, int ldc,
                                                       float* __restrict__ cols) {
  const int Ho = H + 2 * pad - 2, Wo = W + 2 * pad - 2;
  const long total = (long)B * Ho * Wo * ldc;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int k = i % ldc;
    const long r = i / ldc;
    float v = 0.f;
    if (k < C * 9) {
      const int x = r % Wo, y = (r / Wo) % Ho;
      const long b = r / ((long)Wo * Ho);
      const int c = k / 9, kh = (k % 9) / 3, kw = k % 3;
      const int yi = y + kh - pad, xi = x + kw - pad;
      if (yi >= 0 && yi < H && xi >= 0 && xi < W) {
        const long ii = ((b * C + c) * H + yi) * W + xi;
        v = IN_I8 ? (float)static_cast<const int8_t*>(in_)[ii] : static_cast<const float*>(in_)[ii];
      }
    }
    cols[i] = v;
  }
}

// dz_prev[(b*H + y)*W + x][c] = (sum_{kh,kw} dcols[(b, y-kh+pad, x-kw+pad)][c*9+kh*3+kw])
//                               * (a_prev[b][c][y][x] > 0)            (position-major out)
__global__ __launch_bounds__(256) void col2im3x3_drelu_kernel(const float* __restrict__ dcols,
                                                             int ldc, const float* __restrict__ a,
                                                             int B, int C, int H, int W, int pad,
                                                             float* __restrict__ dz) {
  const int Ho = H + 2 * pad - 2, Wo = W + 2 * pad - 2;
  const long total = (long)B * H * W * C;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = i % C;
    const long r = i / C;
    const int x = r % W, y = (r / W) % H;
    const long b = r / ((long)W * H);
    float s = 0.f;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int yo = y - kh + pad;
      if (yo < 0 || yo >= Ho) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int xo = x - kw + pad;
        if (xo < 0 || xo >= Wo) continue;
        s += dcols[((b * Ho + yo) * Wo + xo) * ldc + c * 9 + kh * 3 + kw];
      }
    }
    dz[i] = a[((b * C + c) * H + y) * W + x] > 0.f ? s : 0.f;
  }
}

// ------------------------------------------------------------------------------ GNN layer bwd
// gate/update elementwise: du = dout[d] * g ; dgpre = dout[d] * u * g * (1 - g)
__global__ __launch_bounds__(256) void gnn_gate_bwd_kernel(const float* __restrict__ dout, int D,
                                                          int F, const int* __restrict__ rows,
                                                          const float* __restrict__ g,
                                                          const float* __restrict__ u,
                                                          float* __restrict__ du,
                                                          float* __restrict__ dgpre) {
  const long total = (long)D * F;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int j = i % F;
    const long r = i / F;
    const long d = rows ? rows[r] : r;
    const float o = dout[d * F + j], gg = g[i];
    du[i] = o * gg;
    dgpre[i] = o * u[i] * gg * (1.f - gg);
  }
}

// dx[dst_r] += dc[r][0:F]; dagg[r] = dc[r][F:2F] stays in place (compact rows).
__global__ __launch_bounds__(256) void gnn_dc_scatter_kernel(const float* __restrict__ dc, int D,
                                                            int F, const int* __restrict__ rows,
                                                            float* __restrict__ dx) {
  const long total = (long)D * F;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int j = i % F;
    const long r = i / F;
    const long d = rows ? rows[r] : r;
    dx[d * F + j] += dc[r * 2 * F + j];
  }
}

// One wave per destination (compact index r, node d): for each in-edge e (source s)
//   dw_e = dagg_r . x_s ; S = sum alpha ; a' = alpha/S
//   dalpha_e = (dw_e - sum_e' a'_e' dw_e') / S          (normalisation backward, S > 0)
//   dsc_e = dalpha_e * alpha_e * (1 - alpha_e)           (sigmoid backward)
// writes dsc[e] and the normalised weight an[e] = a'_e (for the source-side scatter).
// Lane l keeps dw of edges e0 + l + 64 j (j < 4) in registers: in-degree <= 256.
__global__ __launch_bounds__(256) void gnn_agg_bwd_edges_kernel(
    int D, const int* __restrict__ rows, const int* __restrict__ rowptr,
    const int* __restrict__ col, const float* __restrict__ alpha, const float* __restrict__ x,
    int F, const float* __restrict__ dc, float* __restrict__ dsc, float* __restrict__ an) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= D) return;
  const int d = rows ? rows[r] : r;
  const int e0 = rowptr[d], e1 = rowptr[d + 1];
  const float* dagg = dc + (size_t)r * 2 * F + F;
  float S = 0.f;
  for (int e = e0; e < e1; ++e) S += alpha[e];
  const bool norm = S > 0.f;
  float swd = 0.f;
  float my0 = 0.f, my1 = 0.f, my2 = 0.f, my3 = 0.f;
  for (int e = e0; e < e1; ++e) {
    const float* xs = x + (size_t)col[e] * F;
    float p = 0.f;
    for (int f = lane * 4; f < F; f += 256) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(dagg + f);
      const f32x4 b = *reinterpret_cast<const f32x4*>(xs + f);
      p = fmaf(a[0], b[0], fmaf(a[1], b[1], fmaf(a[2], b[2], fmaf(a[3], b[3], p))));
    }
    p = wave_sum(p);
    const float w = norm ? alpha[e] / S : alpha[e];
    swd = fmaf(w, p, swd);
    const int o = e - e0;
    if ((o & 63) == lane) {
      const int j = o >> 6;
      if (j == 0) my0 = p;
      else if (j == 1) my1 = p;
      else if (j == 2) my2 = p;
      else my3 = p;
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = e0 + lane + 64 * j;
    if (e < e1) {
      const float dwv = j == 0 ? my0 : (j == 1 ? my1 : (j == 2 ? my2 : my3));
      const float a = alpha[e];
      const float da = norm ? (dwv - swd) / S : dwv;
      dsc[e] = da * a * (1.f - a);
      an[e] = norm ? a / S : a;
    }
  }
}

// High in-degree form of gnn_agg_bwd_edges_kernel (the star: one destination, N-1 edges,
// F = 3136), in two passes so the per-edge dot products run in parallel:
//  1. one wave per edge: p_e = dagg[dst(e)] . x[src(e)]  -> dsc[e] (scratch)
//  2. one wave per destination: S = sum alpha, swd = sum_e w_e p_e (wave reductions), then
//     dsc[e] = (norm ? (p_e - swd) / S : p_e) * a (1 - a),  an[e] = norm ? a / S : a.
__global__ __launch_bounds__(256) void gnn_agg_bwd_dots_kernel(
    int E, const int* __restrict__ edge_dst, const int* __restrict__ dst_index,
    const int* __restrict__ col, const float* __restrict__ x, int F,
    const float* __restrict__ dc, float* __restrict__ pdot) {
  const int e = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (e >= E) return;
  const int d = edge_dst[e];
  const int r = dst_index ? dst_index[d] : d;
  const float* dagg = dc + (size_t)r * 2 * F + F;
  const float* xs = x + (size_t)col[e] * F;
  float p = 0.f;
  for (int f = lane * 4; f < F; f += 256) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(dagg + f);
    const f32x4 b = *reinterpret_cast<const f32x4*>(xs + f);
    p = fmaf(a[0], b[0], fmaf(a[1], b[1], fmaf(a[2], b[2], fmaf(a[3], b[3], p))));
  }
  p = wave_sum(p);
  if (lane == 0) pdot[e] = p;
}

__global__ __launch_bounds__(256) void gnn_agg_bwd_finish_kernel(
    int D, const int* __restrict__ rows, const int* __restrict__ rowptr,
    const float* __restrict__ alpha, float* __restrict__ dsc, float* __restrict__ an) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= D) return;
  const int d = rows ? rows[r] : r;
  const int e0 = rowptr[d], e1 = rowptr[d + 1];
  float S = 0.f;
  for (int e = e0 + lane; e < e1; e += 64) S += alpha[e];
  S = wave_sum(S);
  const bool norm = S > 0.f;
  float swd = 0.f;
  for (int e = e0 + lane; e < e1; e += 64) swd = fmaf(norm ? alpha[e] / S : alpha[e], dsc[e], swd);
  swd = wave_sum(swd);
  for (int e = e0 + lane; e < e1; e += 64) {
    const float a = alpha[e], pe = dsc[e];
    const float da = norm ? (pe - swd) / S : pe;
    dsc[e] = da * a * (1.f - a);
    an[e] = norm ? a / S : a;
  }
}

// One wave per node v:
//   dP[v][2q]   = sum_{e: dst(e)=v} dpre_e[q]     dP[v][2q+1] = sum_{e: src(e)=v} dpre_e[q]
//   dpre_e[q]   = dsc_e * w2[q] * (P[dst][2q] + P[src][2q+1] + b1[q] > 0)
//   dx[v]      += sum_{e: src(e)=v} an_e * dagg[dst(e)]
__global__ __launch_bounds__(256) void gnn_attn_bwd_nodes_kernel(
    int V, int H, const int* __restrict__ rowptr, const int* __restrict__ col,
    const int* __restrict__ edge_dst, const int* __restrict__ src_rowptr,
    const int* __restrict__ src_edges, const int* __restrict__ dst_index,
    const float* __restrict__ P, const float* __restrict__ b1, const float* __restrict__ w2,
    const float* __restrict__ dsc, const float* __restrict__ an, const float* __restrict__ dc,
    int F, float* __restrict__ dP, float* __restrict__ dx) {
  const int v = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (v >= V) return;
  const float* Pv = P + (size_t)v * 2 * H;
  for (int q = lane; q < H; q += 64) {
    const float pt = Pv[2 * q], ps_v = Pv[2 * q + 1], bb = b1[q], ww = w2[q];
    float gt = 0.f, gs = 0.f;
    for (int e = rowptr[v]; e < rowptr[v + 1]; ++e) {          // v as destination
      const float pre = pt + P[(size_t)col[e] * 2 * H + 2 * q + 1] + bb;
      if (pre > 0.f) gt = fmaf(dsc[e], ww, gt);
    }
    for (int j = src_rowptr[v]; j < src_rowptr[v + 1]; ++j) {   // v as source
      const int e = src_edges[j];
      const float pre = P[(size_t)edge_dst[e] * 2 * H + 2 * q] + ps_v + bb;
      if (pre > 0.f) gs = fmaf(dsc[e], ww, gs);
    }
    dP[(size_t)v * 2 * H + 2 * q] = gt;
    dP[(size_t)v * 2 * H + 2 * q + 1] = gs;
  }
  for (int f = lane * 4; f < F; f += 256) {
    f32x4 acc = *reinterpret_cast<const f32x4*>(dx + (size_t)v * F + f);
    for (int j = src_rowptr[v]; j < src_rowptr[v + 1]; ++j) {
      const int e = src_edges[j];
      const int r = dst_index[edge_dst[e]];
      const f32x4 g = *reinterpret_cast<const f32x4*>(dc + (size_t)r * 2 * F + F + f);
      const float w = an[e];
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = fmaf(w, g[c], acc[c]);
    }
    *reinterpret_cast<f32x4*>(dx + (size_t)v * F + f) = acc;
  }
}

// attention parameter gradients over edge chunks (stage 1; stage 2 = colsum_final):
//   part[ch][q] = sum_e dsc_e relu(pre_e[q])            (w2 grad)
//   part[ch][H+q] = sum_e dsc_e w2[q] 1(pre_e[q] > 0)   (b1 grad)
//   part[ch][2H] = sum_e dsc_e                          (b2 grad)
__global__ __launch_bounds__(256) void gnn_attn_param_partial_kernel(
    int E, int H, int per, const int* __restrict__ col, const int* __restrict__ edge_dst,
    const float* __restrict__ P, const float* __restrict__ b1, const float* __restrict__ w2,
    const float* __restrict__ dsc, float* __restrict__ part) {
  const int ch = blockIdx.x;
  const int e0 = ch * per, e1 = min(E, e0 + per);
  for (int q = threadIdx.x; q <= H; q += 256) {
    float gw = 0.f, gb = 0.f, g2 = 0.f;
    for (int e = e0; e < e1; ++e) {
      const float ds = dsc[e];
      if (q == H) {
        g2 += ds;
        continue;
      }
      const float pre = P[(size_t)edge_dst[e] * 2 * H + 2 * q] + P[(size_t)col[e] * 2 * H + 2 * q + 1] + b1[q];
      if (pre > 0.f) {
        gw = fmaf(ds, pre, gw);
        gb = fmaf(ds, w2[q], gb);
      }
    }
    if (q < H) {
      part[(size_t)ch * (2 * H + 1) + q] = gw;
      part[(size_t)ch * (2 * H + 1) + H + q] = gb;
    } else {
      part[(size_t)ch * (2 * H + 1) + 2 * H] = g2;
    }
  }
}

static size_t align256(size_t b) { return (b + 255) & ~size_t(255); }

static int grid_for(long n) { return (int)std::min<long>((n + 255) / 256, 8192); }

}  // namespace az

using namespace az;

// ================================================================================ C-ABI
extern "C" int az_heads_loss_bwd(const float* logp, const float* v, const float* target_pi,
                                 const float* target_v, int B, int A, int B_norm, float* dlogits,
                                 float* dvpre, float* loss_rows, void* stream) {
  AZ_REQUIRE(B >= 0 && A > 0 && B_norm > 0, AZ_EINVAL, "az_heads_loss_bwd: bad shape");
  if (B == 0) return AZ_OK;
  AZ_REQUIRE(logp && v && target_pi && target_v && dlogits && dvpre, AZ_EINVAL,
             "az_heads_loss_bwd: null");
  hipLaunchKernelGGL(heads_loss_bwd_kernel, dim3((B + 255) / 256), dim3(256), 0,
                     as_stream(stream), logp, v, target_pi, target_v, B, A, 1.f / (float)B_norm,
                     dlogits, dvpre, loss_rows);
  return check_launch("heads_loss_bwd_kernel");
}

extern "C" int az_heads_bwd(const float* dlogits, const float* dvpre, const float* hp, int ldhp,
                            const float* hv, int ldhv, int B, int K, const float* wp, int A,
                            const float* wv, float* dwp, float* dbp, float* dwv, float* dbv,
                            float* dhp, int lddhp, float* dhv, int lddhv, void* ws,
                            size_t ws_bytes, void* stream) {
  AZ_REQUIRE(B >= 0 && K > 0 && K % 4 == 0 && A > 0 && A <= 32, AZ_EINVAL,
             "az_heads_bwd: bad shape");
  if (B == 0) return AZ_OK;
  AZ_REQUIRE(dlogits && dvpre && wp && wv, AZ_EINVAL, "az_heads_bwd: null");
  AZ_REQUIRE(!dwp || (hp && hv && dwv && dbp && dbv && ws), AZ_EINVAL,
             "az_heads_bwd: weight grads need hp, hv, dwv, dbp, dbv and ws");
  AZ_REQUIRE(!dhp || dhv, AZ_EINVAL, "az_heads_bwd: dhp needs dhv (pass dhv == dhp to sum)");
  AZ_REQUIRE(!dwp || ws_bytes >= (size_t)colsum_chunks(B) * (A + 1) * 4, AZ_EINVAL,
             "az_heads_bwd: workspace too small");
  hipStream_t s = as_stream(stream);
  dim3 g((K + 255) / 256), b(64);
  if (A <= 8)
    hipLaunchKernelGGL(heads_bwd_kernel<8>, g, b, 0, s, dlogits, dvpre, hp, ldhp, hv, ldhv, B, K,
                       wp, A, wv, dwp, dwv, dhp, lddhp, dhv, lddhv);
  else if (A <= 16)
    hipLaunchKernelGGL(heads_bwd_kernel<16>, g, b, 0, s, dlogits, dvpre, hp, ldhp, hv, ldhv, B, K,
                       wp, A, wv, dwp, dwv, dhp, lddhp, dhv, lddhv);
  else
    hipLaunchKernelGGL(heads_bwd_kernel<32>, g, b, 0, s, dlogits, dvpre, hp, ldhp, hv, ldhv, B, K,
                       wp, A, wv, dwp, dwv, dhp, lddhp, dhv, lddhv);
  int rc = check_launch("heads_bwd_kernel");
  if (rc || !dwp) return rc;
  float* part = static_cast<float*>(ws);
  if ((rc = colsum(dlogits, B, A, A, dbp, 0.f, part, s))) return rc;
  return colsum(dvpre, B, 1, 1, dbv, 0.f, part, s);
}

extern "C" size_t az_colsum_ws_bytes(int R, int C) {
  return (size_t)colsum_chunks(R) * (size_t)C * 4;
}

extern "C" int az_colsum(const float* X, int R, int C, int ldx, float* out, float beta, void* ws,
                         size_t ws_bytes, void* stream) {
  AZ_REQUIRE(R >= 0 && C > 0 && ldx >= C && X && out && ws, AZ_EINVAL, "az_colsum: bad args");
  AZ_REQUIRE(ws_bytes >= az_colsum_ws_bytes(R, C), AZ_EINVAL, "az_colsum: workspace too small");
  return colsum(X, R, C, ldx, out, beta, static_cast<float*>(ws), as_stream(stream));
}

extern "C" int az_dropout_mask(uint8_t* mask, int64_t n, double p, uint64_t seed, void* stream) {
  AZ_REQUIRE(mask && n >= 0 && p >= 0.0 && p < 1.0, AZ_EINVAL, "az_dropout_mask: bad args");
  if (n == 0) return AZ_OK;
  const uint32_t thresh = (uint32_t)std::min(4294967295.0, p * 4294967296.0);
  hipLaunchKernelGGL(dropout_mask_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), mask,
                     (long)n, seed, thresh);
  return check_launch("dropout_mask_kernel");
}

extern "C" int az_mask_scale(const float* x, const uint8_t* mask, float scale, int64_t n,
                             float* y, void* stream) {
  AZ_REQUIRE(x && mask && y && n >= 0, AZ_EINVAL, "az_mask_scale: bad args");
  if (n == 0) return AZ_OK;
  hipLaunchKernelGGL(mask_scale_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), x, mask,
                     scale, (long)n, y);
  return check_launch("mask_scale_kernel");
}

extern "C" int az_nchw_drelu_to_pm(const float* dy, const float* y, const uint8_t* mask,
                                   float scale, int B, int C, int HW, float* dz, void* stream) {
  AZ_REQUIRE(dy && y && dz && B >= 0 && C > 0 && HW > 0, AZ_EINVAL, "az_nchw_drelu_to_pm: bad args");
  const long n = (long)B * C * HW;
  if (n == 0) return AZ_OK;
  hipLaunchKernelGGL(nchw_drelu_to_pm_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream),
                     dy, y, mask, scale, B, C, HW, dz);
  return check_launch("nchw_drelu_to_pm_kernel");
}

extern "C" int az_im2col3x3(const void* in, int in_int8, int B, int C, int H, int W, int pad,
                            int ldc, float* cols, void* stream) {
  AZ_REQUIRE(in && cols && B >= 0 && C > 0 && ldc >= C * 9 && (pad == 0 || pad == 1), AZ_EINVAL,
             "az_im2col3x3: bad args");
  const long n = (long)B * (H + 2 * pad - 2) * (W + 2 * pad - 2) * ldc;
  if (n == 0) return AZ_OK;
  if (in_int8)
    hipLaunchKernelGGL(im2col3x3_kernel<true>, dim3(grid_for(n)), dim3(256), 0, as_stream(stream),
                       in, B, C, H, W, pad, ldc, cols);
  else
    hipLaunchKernelGGL(im2col3x3_kernel<false>, dim3(grid_for(n)), dim3(256), 0, as_stream(stream),
                       in, B, C, H, W, pad, ldc, cols);
  return check_launch("im2col3x3_kernel");
}

extern "C" int az_col2im3x3_drelu(const float* dcols, int ldc, const float* a, int B, int C, int H,
                                  int W, int pad, float* dz, void* stream) {
  AZ_REQUIRE(dcols && a && dz && B >= 0 && C > 0 && ldc >= C * 9 && (pad == 0 || pad == 1),
             AZ_EINVAL, "az_col2im3x3_drelu: bad args");
  const long n = (long)B * H * W * C;
  if (n == 0) return AZ_OK;
  hipLaunchKernelGGL(col2im3x3_drelu_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream),
                     dcols, ldc, a, B, C, H, W, pad, dz);
  return check_launch("col2im3x3_drelu_kernel");
}

// ------------------------------------------------------------------------------ GNN layer bwd
struct BwdWs {
  float *du, *dg, *du1, *dc, *dw, *dsc, *an, *dP, *part;
  void* split;
};
constexpr size_t kBwdSplitBytes = size_t(40) << 20;

static BwdWs carve_bwd(void* ws, int V, int E, int D, int F, int H) {
  char* p = static_cast<char*>(ws);
  BwdWs w;
  w.du = reinterpret_cast<float*>(p); p += align256((size_t)D * F * 4);
  w.dg = reinterpret_cast<float*>(p); p += align256((size_t)D * F * 4);
  w.du1 = reinterpret_cast<float*>(p); p += align256((size_t)D * F * 4);
  w.dc = reinterpret_cast<float*>(p); p += align256((size_t)D * 2 * F * 4);
  w.dw = reinterpret_cast<float*>(p); p += align256((size_t)E * 4);
  w.dsc = reinterpret_cast<float*>(p); p += align256((size_t)E * 4);
  w.an = reinterpret_cast<float*>(p); p += align256((size_t)E * 4);
  w.dP = reinterpret_cast<float*>(p); p += align256((size_t)V * 2 * H * 4);
  w.part = reinterpret_cast<float*>(p);
  p += align256((size_t)std::max(colsum_chunks(std::max(D, V)) * (size_t)std::max(2 * F, 2 * H + 1),
                                 (size_t)1024 * (2 * H + 1)) * 4);
  w.split = p;
  return w;
}

// The node update's backward (az_gnn_node_update_bwd, and az_gnn_layer_bwd's first half):
// from dout (rows of the D destinations) and the forward's gate / u1 / u, the six parameter
// gradients and dc = d[x_d ; agg_d] ([D][2F], compact destination rows).  Scratch du, dg, du1
// ([D][F] each), part (colsum partials), split (GEMM split-K room).
static int node_update_bwd(const float* x, const float* agg, int D, int F, const int* rows,
                           const float* gate_w, const float* upd_w1, const float* upd_w2,
                           const float* gate, const float* u1, const float* u,
                           const float* dout, float* d_gate_w, float* d_gate_b, float* d_upd_w1,
                           float* d_upd_b1, float* d_upd_w2, float* d_upd_b2, float* du,
                           float* dg, float* du1, float* dc, float* part, void* split,
                           size_t split_bytes, hipStream_t s) {
  int rc;
  const long DF = (long)D * F;
  hipLaunchKernelGGL(gnn_gate_bwd_kernel, dim3(grid_for(DF)), dim3(256), 0, s, dout, D, F, rows,
                     gate, u, du, dg);
  if ((rc = check_launch("gnn_gate_bwd_kernel"))) return rc;

  az_gemm_desc d = {};
  // du1pre = (du . Wu2) * (u1 > 0)
  d.M = D; d.N = F; d.K = F;
  d.A = du; d.lda = F; d.a_kmajor = 1;
  d.B = upd_w2; d.ldb = F; d.b_kmajor = 0;
  d.act = AZ_ACT_DRELU; d.G = u1; d.ldg = F;
  d.C = du1; d.ldc = F; d.ws = split; d.ws_bytes = split_bytes;
  if ((rc = gemm_f32(&d, s))) return rc;
  // dWu2 = du^T u1 ; dbu2 = colsum(du)
  d = {};
  d.M = F; d.N = F; d.K = D;
  d.A = du; d.lda = F; d.a_kmajor = 0;
  d.B = u1; d.ldb = F; d.b_kmajor = 0;
  d.C = d_upd_w2; d.ldc = F; d.ws = split; d.ws_bytes = split_bytes;
  if ((rc = gemm_f32(&d, s))) return rc;
  if ((rc = colsum(du, D, F, F, d_upd_b2, 0.f, part, s))) return rc;
  // dW{u1,g} = d{u1,g}pre^T [x_dst | agg_dst] (two column halves) ; biases
  const float* pre_in[2] = {du1, dg};
  float* wout[2] = {d_upd_w1, d_gate_w};
  float* bout[2] = {d_upd_b1, d_gate_b};
  for (int t = 0; t < 2; ++t) {
    for (int half = 0; half < 2; ++half) {
      d = {};
      d.M = F; d.N = F; d.K = D;
      d.A = pre_in[t]; d.lda = F; d.a_kmajor = 0;
      d.B = half == 0 ? x : agg; d.ldb = F; d.b_kmajor = 0; d.b_rows = rows;
      d.C = wout[t] + half * F; d.ldc = 2 * F; d.ws = split; d.ws_bytes = split_bytes;
      if ((rc = gemm_f32(&d, s))) return rc;
    }
    if ((rc = colsum(pre_in[t], D, F, F, bout[t], 0.f, part, s))) return rc;
  }
  // dc = du1pre . Wu1 + dgpre . Wg      [D][2F]
  d = {};
  d.M = D; d.N = 2 * F; d.K = F;
  d.A = du1; d.lda = F; d.a_kmajor = 1;
  d.B = upd_w1; d.ldb = 2 * F; d.b_kmajor = 0;
  d.C = dc; d.ldc = 2 * F; d.ws = split; d.ws_bytes = split_bytes;
  if ((rc = gemm_f32(&d, s))) return rc;
  d.A = dg; d.B = gate_w; d.beta = 1.f;
  return gemm_f32(&d, s);
}

// dagg[dst_r] = dc[r][F:2F] (the agg half of dc, onto the destination rows)
__global__ __launch_bounds__(256) void gnn_dc_agg_scatter_kernel(const float* __restrict__ dc,
                                                                int D, int F,
                                                                const int* __restrict__ rows,
                                                                float* __restrict__ dagg) {
  const long total = (long)D * F;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int j = i % F;
    const long r = i / F;
    const long d = rows ? rows[r] : r;
    dagg[d * F + j] = dc[r * 2 * F + F + j];
  }
}

extern "C" size_t az_gnn_layer_bwd_ws_bytes(int V, int E, int D, int F, int H) {
  return align256((size_t)D * F * 4) * 3 + align256((size_t)D * 2 * F * 4) +
         align256((size_t)E * 4) * 3 + align256((size_t)V * 2 * H * 4) +
         align256((size_t)std::max(colsum_chunks(std::max(D, V)) * (size_t)std::max(2 * F, 2 * H + 1),
                                   (size_t)1024 * (2 * H + 1)) * 4) +
         kBwdSplitBytes;
}


extern "C" int az_gnn_layer_bwd(const az_graph* g, const float* x, int F, int H,
                                const az_gnn_layer_w* w, const void* fwd_ws, const float* dout,
                                float* dx, const az_gnn_layer_grads* gr, void* ws,
                                size_t ws_bytes, void* stream) {
  AZ_REQUIRE(g && x && w && fwd_ws && dout && dx && gr && ws, AZ_EINVAL, "az_gnn_layer_bwd: null");
  AZ_REQUIRE(g->E == 0 || (g->src_rowptr && g->src_edges && g->dst_index), AZ_EINVAL,
             "az_gnn_layer_bwd: graph needs src_rowptr/src_edges/dst_index");
  AZ_REQUIRE(g->max_deg <= 256, AZ_EINVAL, "az_gnn_layer_bwd: in-degree %d > 256", g->max_deg);
  AZ_REQUIRE(F % 16 == 0 && H % 4 == 0 && H <= 1024, AZ_EINVAL, "az_gnn_layer_bwd: F%%16, H%%4");
  AZ_REQUIRE(ws_bytes >= az_gnn_layer_bwd_ws_bytes(g->V, g->E, g->D, F, H), AZ_EINVAL,
             "az_gnn_layer_bwd: workspace too small");
  hipStream_t s = as_stream(stream);
  const int V = g->V, E = g->E, D = g->D;
  const int* rows = (D == V) ? nullptr : g->dst_rows;
  const FwdSaved sv = fwd_saved(fwd_ws, V, E, D, F, H);
  BwdWs L = carve_bwd(ws, V, E, D, F, H);
  int rc;
  // identity path: every row passes dout straight through (out[v] = x[v] + ...)
  if (hipMemcpyAsync(dx, dout, (size_t)V * F * 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return check_launch("hipMemcpyAsync");
  if (D == 0) {
    hipMemsetAsync(gr->att_w1, 0, (size_t)H * 2 * F * 4, s);
    hipMemsetAsync(gr->att_b1, 0, (size_t)H * 4, s);
    hipMemsetAsync(gr->att_w2, 0, (size_t)H * 4, s);
    hipMemsetAsync(gr->att_b2, 0, 4, s);
    hipMemsetAsync(gr->upd_w1, 0, (size_t)F * 2 * F * 4, s);
    hipMemsetAsync(gr->upd_b1, 0, (size_t)F * 4, s);
    hipMemsetAsync(gr->upd_w2, 0, (size_t)F * F * 4, s);
    hipMemsetAsync(gr->upd_b2, 0, (size_t)F * 4, s);
    hipMemsetAsync(gr->gate_w, 0, (size_t)F * 2 * F * 4, s);
    hipMemsetAsync(gr->gate_b, 0, (size_t)F * 4, s);
    return check_launch("hipMemsetAsync");
  }
  const long DF = (long)D * F;
  if ((rc = node_update_bwd(x, sv.agg, D, F, rows, w->gate_w, w->upd_w1, w->upd_w2, sv.gate,
                            sv.u1, sv.u, dout, gr->gate_w, gr->gate_b, gr->upd_w1, gr->upd_b1,
                            gr->upd_w2, gr->upd_b2, L.du, L.dg, L.du1, L.dc, L.part, L.split,
                            kBwdSplitBytes, s)))
    return rc;
  hipLaunchKernelGGL(gnn_dc_scatter_kernel, dim3(grid_for(DF)), dim3(256), 0, s, L.dc, D, F, rows,
                     dx);
  if ((rc = check_launch("gnn_dc_scatter_kernel"))) return rc;
  // aggregation + attention backward
  if (E > 0 && E >= 16L * D) {
    // few destinations with many in-edges (the training star): per-edge dots in parallel
    hipLaunchKernelGGL(gnn_agg_bwd_dots_kernel, dim3((E + 3) / 4), dim3(256), 0, s, E,
                       g->edge_dst, D == V ? nullptr : g->dst_index, g->col, x, F, L.dc, L.dsc);
    if ((rc = check_launch("gnn_agg_bwd_dots_kernel"))) return rc;
    hipLaunchKernelGGL(gnn_agg_bwd_finish_kernel, dim3((D + 3) / 4), dim3(256), 0, s, D, rows,
                       g->rowptr, sv.alpha, L.dsc, L.an);
    if ((rc = check_launch("gnn_agg_bwd_finish_kernel"))) return rc;
  } else if (E > 0) {
    hipLaunchKernelGGL(gnn_agg_bwd_edges_kernel, dim3((D + 3) / 4), dim3(256), 0, s, D, rows,
                       g->rowptr, g->col, sv.alpha, x, F, L.dc, L.dsc, L.an);
    if ((rc = check_launch("gnn_agg_bwd_edges_kernel"))) return rc;
  }
  hipLaunchKernelGGL(gnn_attn_bwd_nodes_kernel, dim3((V + 3) / 4), dim3(256), 0, s, V, H,
                     g->rowptr, g->col, g->edge_dst, g->src_rowptr, g->src_edges, g->dst_index,
                     sv.P, w->att_b1, w->att_w2, L.dsc, L.an, L.dc, F, L.dP, dx);
  if ((rc = check_launch("gnn_attn_bwd_nodes_kernel"))) return rc;
  // dW1' = dP^T x  (W1 [H][2F] viewed as [2H][F]) ; dx += dP . W1'
  az_gemm_desc d = {};
  d.M = 2 * H; d.N = F; d.K = V;
  d.A = L.dP; d.lda = 2 * H; d.a_kmajor = 0;
  d.B = x; d.ldb = F; d.b_kmajor = 0;
  d.C = gr->att_w1; d.ldc = F; d.ws = L.split; d.ws_bytes = kBwdSplitBytes;
  if ((rc = gemm_f32(&d, s))) return rc;
  d = {};
  d.M = V; d.N = F; d.K = 2 * H;
  d.A = L.dP; d.lda = 2 * H; d.a_kmajor = 1;
  d.B = w->att_w1; d.ldb = F; d.b_kmajor = 0;
  d.beta = 1.f; d.C = dx; d.ldc = F; d.ws = L.split; d.ws_bytes = kBwdSplitBytes;
  if ((rc = gemm_f32(&d, s))) return rc;
  // w2, b1, b2 gradients
  const int nch = std::max(1, std::min((E + 1023) / 1024, 1024));
  const int per = E > 0 ? (E + nch - 1) / nch : 1;
  hipLaunchKernelGGL(gnn_attn_param_partial_kernel, dim3(nch), dim3(256), 0, s, E, H, per, g->col,
                     g->edge_dst, sv.P, w->att_b1, w->att_w2, L.dsc, L.part);
  if ((rc = check_launch("gnn_attn_param_partial_kernel"))) return rc;
  hipLaunchKernelGGL(colsum_final_kernel, dim3((H + 255) / 256), dim3(256), 0, s, L.part, nch,
                     2 * H + 1, H, 0.f, gr->att_w2);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((H + 255) / 256), dim3(256), 0, s, L.part + H, nch,
                     2 * H + 1, H, 0.f, gr->att_b1);
  hipLaunchKernelGGL(colsum_final_kernel, dim3(1), dim3(256), 0, s, L.part + 2 * H, nch, 2 * H + 1,
                     1, 0.f, gr->att_b2);
  return check_launch("attn param grads");
}

// ------------------------------------------------------------------------------ node update bwd
static size_t node_update_bwd_part_bytes(int D, int F) {
  return align256((size_t)colsum_chunks(D) * (size_t)F * 4);
}

extern "C" size_t az_gnn_node_update_bwd_ws_bytes(int D, int F) {
  return align256((size_t)D * F * 4) * 3 + align256((size_t)D * 2 * F * 4) +
         node_update_bwd_part_bytes(D, F) + kBwdSplitBytes;
}

extern "C" int az_gnn_node_update_bwd(const float* x, const float* agg, int V, int F, int D,
                                      const int* dst_rows, const float* gate_w,
                                      const float* upd_w1, const float* upd_w2,
                                      const float* save, const float* dout, float* dx,
                                      float* dagg, float* d_gate_w, float* d_gate_b,
                                      float* d_upd_w1, float* d_upd_b1, float* d_upd_w2,
                                      float* d_upd_b2, void* ws, size_t ws_bytes, void* stream) {
  AZ_REQUIRE(V >= 0 && D >= 0 && D <= V && F > 0 && F % 16 == 0, AZ_EINVAL,
             "az_gnn_node_update_bwd: V=%d D=%d F=%d (D <= V, F %% 16)", V, D, F);
  if (V == 0) return AZ_OK;
  AZ_REQUIRE(x && agg && save && dout && dx && dagg && ws && (D == V || dst_rows), AZ_EINVAL,
             "az_gnn_node_update_bwd: bad pointers");
  AZ_REQUIRE(gate_w && upd_w1 && upd_w2 && d_gate_w && d_gate_b && d_upd_w1 && d_upd_b1 &&
                 d_upd_w2 && d_upd_b2,
             AZ_EINVAL, "az_gnn_node_update_bwd: null weight / gradient");
  AZ_REQUIRE(ws_bytes >= az_gnn_node_update_bwd_ws_bytes(D, F), AZ_EINVAL,
             "az_gnn_node_update_bwd: workspace too small");
  hipStream_t s = as_stream(stream);
  // identity path: every row passes dout straight through (x_out[v] = x[v] + ...)
  if (hipMemcpyAsync(dx, dout, (size_t)V * F * 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return check_launch("hipMemcpyAsync");
  if (D == 0) {
    hipMemsetAsync(d_upd_w1, 0, (size_t)F * 2 * F * 4, s);
    hipMemsetAsync(d_upd_b1, 0, (size_t)F * 4, s);
    hipMemsetAsync(d_upd_w2, 0, (size_t)F * F * 4, s);
    hipMemsetAsync(d_upd_b2, 0, (size_t)F * 4, s);
    hipMemsetAsync(d_gate_w, 0, (size_t)F * 2 * F * 4, s);
    hipMemsetAsync(d_gate_b, 0, (size_t)F * 4, s);
    return check_launch("hipMemsetAsync");
  }
  const int* rows = (D == V) ? nullptr : dst_rows;
  const size_t DF = (size_t)D * F;
  char* p = static_cast<char*>(ws);
  float* du = reinterpret_cast<float*>(p); p += align256(DF * 4);
  float* dg = reinterpret_cast<float*>(p); p += align256(DF * 4);
  float* du1 = reinterpret_cast<float*>(p); p += align256(DF * 4);
  float* dc = reinterpret_cast<float*>(p); p += align256(2 * DF * 4);
  float* part = reinterpret_cast<float*>(p); p += node_update_bwd_part_bytes(D, F);
  int rc;
  if ((rc = node_update_bwd(x, agg, D, F, rows, gate_w, upd_w1, upd_w2, save, save + DF,
                            save + 2 * DF, dout, d_gate_w, d_gate_b, d_upd_w1, d_upd_b1, d_upd_w2,
                            d_upd_b2, du, dg, du1, dc, part, p, kBwdSplitBytes, s)))
    return rc;
  hipLaunchKernelGGL(gnn_dc_scatter_kernel, dim3(grid_for((long)DF)), dim3(256), 0, s, dc, D, F,
                     rows, dx);
  if ((rc = check_launch("gnn_dc_scatter_kernel"))) return rc;
  hipLaunchKernelGGL(gnn_dc_agg_scatter_kernel, dim3(grid_for((long)DF)), dim3(256), 0, s, dc, D,
                     F, rows, dagg);
  return check_launch("gnn_dc_agg_scatter_kernel");
}

// ------------------------------------------------------------------------------ mlp2 bwd
extern "C" int az_mlp2_bwd(const float* x, int M, int F, const float* w0, const float* w2,
                           const float* hidden, const float* dy, float* dx, float* dw0, float* db0,
                           float* dw2, float* db2, float* dh, void* ws, size_t ws_bytes,
                           void* stream) {
  AZ_REQUIRE(x && w0 && w2 && hidden && dy && dw0 && db0 && dw2 && db2 && dh && ws, AZ_EINVAL,
             "az_mlp2_bwd: null");
  AZ_REQUIRE(ws_bytes >= az_colsum_ws_bytes(M, F), AZ_EINVAL, "az_mlp2_bwd: workspace too small");
  hipStream_t s = as_stream(stream);
  float* part = static_cast<float*>(ws);
  void* split = static_cast<char*>(ws) + align256(az_colsum_ws_bytes(M, F));
  const size_t split_bytes = ws_bytes - align256(az_colsum_ws_bytes(M, F));
  int rc;
  az_gemm_desc d = {};
  // dW2 = dy^T h ; db2 = colsum(dy)
  d.M = F; d.N = F; d.K = M;
  d.A = dy; d.lda = F; d.a_kmajor = 0;
  d.B = hidden; d.ldb = F; d.b_kmajor = 0;
  d.C = dw2; d.ldc = F; d.ws = split; d.ws_bytes = split_bytes;
  if ((rc = gemm_f32(&d, s))) return rc;
  if ((rc = colsum(dy, M, F, F, db2, 0.f, part, s))) return rc;
  // dh = (dy . W2) * (h > 0)
  d = {};
  d.M = M; d.N = F; d.K = F;
  d.A = dy; d.lda = F; d.a_kmajor = 1;
  d.B = w2; d.ldb = F; d.b_kmajor = 0;
  d.act = AZ_ACT_DRELU; d.G = hidden; d.ldg = F;
  d.C = dh; d.ldc = F; d.ws = split; d.ws_bytes = split_bytes;
  if ((rc = gemm_f32(&d, s))) return rc;
  // dW0 = dh^T x ; db0 = colsum(dh)
  d = {};
  d.M = F; d.N = F; d.K = M;
  d.A = dh; d.lda = F; d.a_kmajor = 0;
  d.B = x; d.ldb = F; d.b_kmajor = 0;
  d.C = dw0; d.ldc = F; d.ws = split; d.ws_bytes = split_bytes;
  if ((rc = gemm_f32(&d, s))) return rc;
  if ((rc = colsum(dh, M, F, F, db0, 0.f, part, s))) return rc;
  if (!dx) return AZ_OK;
  // dx = dh . W0
  d = {};
  d.M = M; d.N = F; d.K = F;
  d.A = dh; d.lda = F; d.a_kmajor = 1;
  d.B = w0; d.ldb = F; d.b_kmajor = 0;
  d.C = dx; d.ldc = F; d.ws = split; d.ws_bytes = split_bytes;
  return gemm_f32(&d, s);
}
