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
template <int AMAX, int NW>
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
      xs[j] = *reinterpret_cast<const f32x4*>(xr + kc);
      ys[j] = *reinterpret_cast<const f32x4*>(yr + kc);
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
      const float vs = wave_sum(fmaf(y[3], w[j][AMAX][3], fmaf(y[2], w[j][AMAX][2],
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

}  // namespace az
