// Policy/value heads of one board row computed by one workgroup (shared by the trunk, heads and
// GEMV translation units).  Connect4GNN.py:48-57: log_softmax(x wp^T + bp), tanh(y wv^T + bv).
#pragma once

#include "az_common.h"

namespace az {

constexpr int HEADS_KC = 256;         // K columns per chunk (64 lanes x float4)
constexpr int HEADS_ROWS_MAXC = 64;   // chunks a one-block row may have: K <= 16384

// Heads of rows x[0..B) run by extra blocks of another launch (gemv_side_heads).
struct SideHeads {
  const float* x; int ldx; int K; int B;
  const float* wp; const float* bp; int A; const float* wv; const float* bv;
  float* logp; float* pi; float* v;
};

// One row's heads with all NW waves of the block (NW * 64 threads): xr / yr may point into LDS
// (the fused trunk) or HBM; part is [HEADS_ROWS_MAXC][AMAX+1] and sm [AMAX+1] floats of LDS.
// Wave w forms the partials of chunks w, w + NW, ... with heads_partial_kernel's arithmetic (two
// chunks' loads issued together) and the chunk sums run in chunk order, so the result does not
// depend on NW.  Ends with a barrier: the caller may reuse part / sm for the next row.
template <int AMAX, int NW, bool SC1 = false>   // SC1: xr / yr stored by other blocks
__device__ __forceinline__ void heads_row_block(const float* xr, const float* yr, int K,
                                                const float* __restrict__ wp, int A,
                                                const float* __restrict__ wv,
                                                const float* __restrict__ bp,
                                                const float* __restrict__ bv, int row,
                                                float* __restrict__ logp, float* __restrict__ pi,
                                                float* __restrict__ v, float* part, float* sm) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nchunks = (K + HEADS_KC - 1) / HEADS_KC;
  constexpr int LOGV = AMAX == 8 ? 3 : (AMAX == 16 ? 4 : 5);
  constexpr int PW = AMAX + 1;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  for (int c0 = wave; c0 < nchunks; c0 += 2 * NW) {
    f32x4 xs[2], ys[2], w[2][AMAX + 1];
    bool kin[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = min(c0 + NW * j, nchunks - 1);
      const int k = c * HEADS_KC + lane * 4;
      kin[j] = k < K;
      const int kc = kin[j] ? k : 0;
      if constexpr (SC1) {
        xs[j] = ld4_sc1(xr, kc * 4, K * 4);
        ys[j] = ld4_sc1(yr, kc * 4, K * 4);
      } else {
        xs[j] = *reinterpret_cast<const f32x4*>(xr + kc);
        ys[j] = *reinterpret_cast<const f32x4*>(yr + kc);
      }
#pragma unroll
      for (int a = 0; a < AMAX; ++a)
        w[j][a] = *reinterpret_cast<const f32x4*>(wp + (size_t)min(a, A - 1) * K + kc);
      w[j][AMAX] = *reinterpret_cast<const f32x4*>(wv + kc);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = c0 + NW * j;
      if (c >= nchunks) break;
#pragma unroll
      for (int a = 0; a < AMAX; ++a) w[j][a] = (a < A && kin[j]) ? w[j][a] : z;
      w[j][AMAX] = kin[j] ? w[j][AMAX] : z;
      const f32x4 x = kin[j] ? xs[j] : z, y = kin[j] ? ys[j] : z;
      float pv[AMAX];
#pragma unroll
      for (int a = 0; a < AMAX; ++a)
        pv[a] = fmaf(x[3], w[j][a][3], fmaf(x[2], w[j][a][2], fmaf(x[1], w[j][a][1], x[0] * w[j][a][0])));
      const float ps = wave_multi_sum<AMAX>(pv);
      const float vs = wave_sum_x(fmaf(y[3], w[j][AMAX][3], fmaf(y[2], w[j][AMAX][2],
                                fmaf(y[1], w[j][AMAX][1], y[0] * w[j][AMAX][0]))));
      const int a = lane >> (6 - LOGV);
      if ((lane & ((1 << (6 - LOGV)) - 1)) == 0 && a < A) part[c * PW + a] = ps;
      if (lane == 0) part[c * PW + A] = vs;
    }
  }
  __syncthreads();
  const int W = A + 1;
  if (threadIdx.x < W) {
    float s = 0.f;
    for (int c = 0; c < nchunks; ++c) s += part[c * PW + threadIdx.x];
    sm[threadIdx.x] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float l[AMAX];
    float mx = -INFINITY;
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
      if (a < A) {
        l[a] = sm[a] + bp[a];
        mx = fmaxf(mx, l[a]);
      }
    float se = 0.f;
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
      if (a < A) se += expf(l[a] - mx);
    const float lse = logf(se);
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
      if (a < A) {
        const float o = (l[a] - mx) - lse;
        logp[(size_t)row * A + a] = o;
        if (pi) pi[(size_t)row * A + a] = expf(o);
      }
    v[row] = tanhf(sm[A] + bv[0]);
  }
  __syncthreads();
}

// heads_row_block split at its chunk boundary, for a row whose chunks are computed by different
// workgroups (c4_leaf_kernel): one wave forms chunk c's partial sums -- heads_row_block's
// per-chunk arithmetic, operand for operand -- into dst[0 .. A) (policy) and dst[A] (value) ...
template <int AMAX, bool SC1 = false>   // SC1: xr / yr read, dst written, across blocks
__device__ __forceinline__ void heads_chunk_part(const float* xr, const float* yr, int K,
                                                 const float* __restrict__ wp, int A,
                                                 const float* __restrict__ wv, int c, float* dst) {
  const int lane = threadIdx.x & 63;
  constexpr int LOGV = AMAX == 8 ? 3 : (AMAX == 16 ? 4 : 5);
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  const int k = c * HEADS_KC + lane * 4;
  const bool kin = k < K;
  const int kc = kin ? k : 0;
  const f32x4 xs = SC1 ? ld4_sc1(xr, kc * 4, K * 4) : *reinterpret_cast<const f32x4*>(xr + kc);
  const f32x4 ys = SC1 ? ld4_sc1(yr, kc * 4, K * 4) : *reinterpret_cast<const f32x4*>(yr + kc);
  f32x4 w[AMAX + 1];
#pragma unroll
  for (int a = 0; a < AMAX; ++a) w[a] = *reinterpret_cast<const f32x4*>(wp + (size_t)min(a, A - 1) * K + kc);
  w[AMAX] = *reinterpret_cast<const f32x4*>(wv + kc);
#pragma unroll
  for (int a = 0; a < AMAX; ++a) w[a] = (a < A && kin) ? w[a] : z;
  w[AMAX] = kin ? w[AMAX] : z;
  const f32x4 x = kin ? xs : z, y = kin ? ys : z;
  float pv[AMAX];
#pragma unroll
  for (int a = 0; a < AMAX; ++a)
    pv[a] = fmaf(x[3], w[a][3], fmaf(x[2], w[a][2], fmaf(x[1], w[a][1], x[0] * w[a][0])));
  const float ps = wave_multi_sum<AMAX>(pv);
  const float vs = wave_sum_x(fmaf(y[3], w[AMAX][3], fmaf(y[2], w[AMAX][2],
                            fmaf(y[1], w[AMAX][1], y[0] * w[AMAX][0]))));
  const int a = lane >> (6 - LOGV);
  if constexpr (SC1) {
    if ((lane & ((1 << (6 - LOGV)) - 1)) == 0 && a < A) st_sc1(dst + a, ps);
    if (lane == 0) st_sc1(dst + A, vs);
  } else {
    if ((lane & ((1 << (6 - LOGV)) - 1)) == 0 && a < A) dst[a] = ps;
    if (lane == 0) dst[A] = vs;
  }
}

// ... and the whole block sums a row's chunk partials (part [nchunks][AMAX + 1]) in chunk order
// and runs heads_row_block's log_softmax / exp / tanh (sm: AMAX + 1 floats of LDS).
template <int AMAX, bool SC1 = false>   // SC1: part stored by other blocks
__device__ __forceinline__ void heads_finalize_row(const float* part, int nchunks, int A,
                                                   const float* __restrict__ bp,
                                                   const float* __restrict__ bv, int row,
                                                   float* __restrict__ logp,
                                                   float* __restrict__ pi, float* __restrict__ v,
                                                   float* sm) {
  constexpr int PW = AMAX + 1;
  const int W = A + 1;
  if ((int)threadIdx.x < W) {
    float s = 0.f;
    if constexpr (SC1) {
      // the chunks' partials all in flight at once (buffer loads, sc1), then summed in order
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(part), 0, nchunks * PW * 4, 0x00020000);
      for (int c0 = 0; c0 < nchunks; c0 += 16) {
        float t[16];
#pragma unroll
        for (int j = 0; j < 16; ++j)
          t[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                               rs, ((c0 + j) * PW + threadIdx.x) * 4, 0, 16));
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (c0 + j < nchunks) s += t[j];
      }
    } else {
      for (int c = 0; c < nchunks; ++c) s += part[c * PW + threadIdx.x];
    }
    sm[threadIdx.x] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float l[AMAX];
    float mx = -INFINITY;
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
      if (a < A) {
        l[a] = sm[a] + bp[a];
        mx = fmaxf(mx, l[a]);
      }
    float se = 0.f;
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
      if (a < A) se += expf(l[a] - mx);
    const float lse = logf(se);
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
      if (a < A) {
        const float o = (l[a] - mx) - lse;
        logp[(size_t)row * A + a] = o;
        if (pi) pi[(size_t)row * A + a] = expf(o);
      }
    v[row] = tanhf(sm[A] + bv[0]);
  }
  __syncthreads();
}

}  // namespace az
