// Band-mode inference GNNLayer (gnn_utils.py:5-74) for node-ordered graphs whose in-edges stay
// near the diagonal -- every source s of a destination d has |s - d| <= 32, which the synthetic
// 32x32 grid in row-major order is (config 5: sources d +- 1, d +- 32) -- with F = 64 node
// features and H = 128 attention hidden units.  ONE launch per layer (+ a 3 us weight split):
//
//   per tile of 64 consecutive destination nodes [d0, d0 + 64), one 512-thread block per CU,
//   persistent over a contiguous run of tiles:
//     A  Pt = X[d0, d0+64) W1[:, :F]^T           (waves 0-3)   } x3 MFMAs: fp32 operands as three
//        Ps = X[d0+32, d0+96) W1[:, F:]^T         (waves 4-7)   } bf16 terms, six products
//     B  alpha_e = sigmoid(w2 . relu(Pt[d] + Ps[s] + b1) + b2), agg_d = sum_e alpha_e / S x_s
//        (8 lanes per destination, edges in CSR order, S = sum alpha > 0: gnn_utils.py:48-65)
//     C  [gate | u1] = [x_d ; agg_d] [Wg ; Wu1]^T + b   (K split over the two wave halves)
//     D  x_out[d] = x_d + gate * (u1 Wu2^T + bu2)       (gnn_utils.py:67-71)
//
//   x and the SOURCE half of the attention projection live in a 128-row ring in LDS covering the
//   tile's window [d0 - 32, d0 + 96): each tile adds 64 new rows (their x and Ps) and drops 64,
//   so every node's x is read from HBM once and its Ps computed once per block run -- the
//   separate Ps projection GEMM (and its 268 MB write + gather at 512 grids) is gone.  Nothing
//   but x_out leaves the CU.  The weights (three bf16 planes, split once per launch) stream
//   from L2.
//
// Edges are never dropped: a destination with any in-degree is aggregated completely, and a
// source outside the window (a graph that is not banded as the caller claimed) takes a slow
// path from global memory (its Ps on the VALU from the fp32 weights) -- slower, never wrong.
#include <stdlib.h>

#include "az_common.h"
#include "az_x3.h"

namespace az {
namespace {

constexpr int BF = 64;        // node features
constexpr int BH = 128;       // attention hidden units
constexpr int BT = 64;        // destinations per tile
constexpr int BR = 32;        // band radius the window covers
constexpr int RING = 128;     // window rows = BT + 2 BR (node n lives in slot n & 127)
constexpr int BNT = 512;      // threads: 8 waves, one block per CU
constexpr int XS = 68;        // row strides (floats) = 4 (mod 64): the 32-row MFMA fragment reads
constexpr int PSS = 132;      //   (lane: row lane & 31, 16 B at k 8 (lane >> 5)) are conflict free
constexpr int AS = 68;

// weight planes [3][WTOT] bf16 in MFMA-fragment order: a matrix W [N][K] (nn.Linear [out][in])
// is stored as (N / 32) x (K / 16) blocks of 512 bf16, block (nb, ks) holding the B operand of
// one v_mfma_f32_32x32x16_bf16 step lane by lane (lane l: row 32 nb + (l & 31), k = 16 ks +
// 8 (l >> 5) .. + 7), so a wave reads its fragment as ONE contiguous 1 KB (row-major planes
// made every lane touch its own cache line: 4x the L2 traffic)
constexpr int W1_OFF = 0;                    // attention.0    [128][128]
constexpr int WC_OFF = BH * 2 * BF;          // [gate.0 ; update_net.0]  [128][128]
constexpr int WU2_OFF = WC_OFF + 2 * BF * 2 * BF;   // update_net.2 [64][64]
constexpr int WTOT = WU2_OFF + BF * BF;
constexpr int FRAG = 512;                    // bf16 per fragment block

// offset of W[n][k .. k + 7] (k % 8 == 0) in a fragment-ordered matrix of K columns
__host__ __device__ constexpr int frag_off(int n, int k, int K) {
  return ((n >> 5) * (K >> 4) + (k >> 4)) * FRAG + ((n & 31) + 32 * ((k >> 3) & 1)) * 8;
}

struct BandW {
  const unsigned short* planes;              // [3][WTOT]
  const float *w1, *b1, *w2, *b2, *gb, *ub1, *ub2;
};

__device__ __forceinline__ float relu(float v) { return v > 0.f ? v : 0.f; }

// 8 consecutive weights -> their three bf16 planes
__global__ __launch_bounds__(256) void band_split_weights(const float* __restrict__ w1,
                                                          const float* __restrict__ gw,
                                                          const float* __restrict__ uw1,
                                                          const float* __restrict__ uw2,
                                                          unsigned short* __restrict__ planes) {
  const int i = (blockIdx.x * 256 + threadIdx.x) * 8;   // element of [W1 | Wg ; Wu1 | Wu2]
  if (i >= WTOT) return;
  const float* src;
  int dst;
  if (i < WC_OFF) {                       // W1 [128][128]
    src = w1 + i;
    dst = W1_OFF + frag_off(i >> 7, i & 127, 2 * BF);
  } else if (i < WU2_OFF) {               // [Wg ; Wu1] [128][128]
    const int j = i - WC_OFF;
    src = j < BF * 2 * BF ? gw + j : uw1 + (j - BF * 2 * BF);
    dst = WC_OFF + frag_off(j >> 7, j & 127, 2 * BF);
  } else {                                // Wu2 [64][64]
    const int j = i - WU2_OFF;
    src = uw2 + j;
    dst = WU2_OFF + frag_off(j >> 6, j & 63, BF);
  }
  const f32x4 x0 = *reinterpret_cast<const f32x4*>(src);
  const f32x4 x1 = *reinterpret_cast<const f32x4*>(src + 4);
  u32x4 o[3];
  split3(x0, x1, o);
#pragma unroll
  for (int pl = 0; pl < 3; ++pl)
    *reinterpret_cast<u32x4*>(planes + (size_t)pl * WTOT + dst) = o[pl];
}

// acc[mb] += A[32 rows of m-block mb][K = 16 KS] . W[32 rows][K]^T on x3 MFMAs.  arow[mb]: this
// lane's A row in LDS (fp32) at k = 8 (lane >> 5); w: plane 0 of the first fragment block
// (frag_off(n0, k0, K) + 8 lane; the KS blocks of one row block are consecutive).  Every B
// fragment is requested before the first MFMA (L2 latency); A is split per step.
template <int MB, int KS>
__device__ __forceinline__ void x3_rows(f32x16 (&acc)[MB], const float* const (&arow)[MB],
                                        const unsigned short* __restrict__ w, int abl = 0) {
  bf16x8 b[KS][3];
  if (abl & 16) {                         // tuning ablation: no weight loads
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) b[ks][pl] = bf16x8{};
  } else {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        b[ks][pl] = *reinterpret_cast<const bf16x8*>(w + (size_t)pl * WTOT + FRAG * ks);
  }
  if (abl & 32) return;                   // tuning ablation: no A reads / split / MFMAs
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(arow[mb] + 16 * ks);
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(arow[mb] + 16 * ks + 4);
      u32x4 o[3];
      split3(x0, x1, o);
      const bf16x8 a[3] = {__builtin_bit_cast(bf16x8, o[0]), __builtin_bit_cast(bf16x8, o[1]),
                           __builtin_bit_cast(bf16x8, o[2])};
      acc[mb] = mfma6_32x32x16(a, b[ks], acc[mb]);
    }
}

// row of register r of a 32x32 MFMA accumulator (column = lane & 31)
__device__ __forceinline__ int acc_row(int r, int lane) {
  return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}

}  // namespace

__global__ __launch_bounds__(BNT, 1) void gnn_layer_band_kernel(
    int V, const int* __restrict__ rowptr, const int* __restrict__ col,
    const float* __restrict__ x, BandW W, float* __restrict__ x_out, int ntiles, int per,
    int abl) {
  __shared__ __attribute__((aligned(16))) float XR[RING * XS];   // x rows of the window
  __shared__ __attribute__((aligned(16))) float PSR[RING * PSS]; // Ps rows of the window
  __shared__ __attribute__((aligned(16))) float PT[BT * PSS];    // Pt; then C partials; then u1
  __shared__ __attribute__((aligned(16))) float AG[BT * AS];     // agg; then gate
  __shared__ __attribute__((aligned(16))) float B1W2[2 * BH];
  __shared__ int DEG[BT];
  __shared__ int RPS[2][BT + 1];          // rowptr of the tile's destinations (+1), prefetched
  __shared__ int CLS[2][BNT];             // the tile's sources (col), when it has <= 512 edges
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 31, hk = 8 * (lane >> 5);
  const int t0 = blockIdx.x * per, t1 = min(ntiles, t0 + per);
  if (t0 >= t1) return;                   // uniform per block
  if (tid < BH) {
    B1W2[tid] = W.b1[tid];
    B1W2[BH + tid] = W.w2[tid];
  }
  const float b2 = W.b2[0];

  // 64 x rows [r0, r0 + 64) <-> the ring: thread = (row tid >> 3, 8 floats at 8 (tid & 7))
  auto load_rows = [&](int r0, f32x4 (&v)[2]) {
    const int n = r0 + (tid >> 3), c = (tid & 7) * 8;
    if (n >= 0 && n < V) {
      v[0] = *reinterpret_cast<const f32x4*>(x + (size_t)n * BF + c);
      v[1] = *reinterpret_cast<const f32x4*>(x + (size_t)n * BF + c + 4);
    } else {
      v[0] = v[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store_rows = [&](int r0, const f32x4 (&v)[2]) {
    const int n = r0 + (tid >> 3), c = (tid & 7) * 8;
    float* d = XR + (n & (RING - 1)) * XS + c;
    *reinterpret_cast<f32x4*>(d) = v[0];
    *reinterpret_cast<f32x4*>(d + 4) = v[1];
  };
  // Ps rows [r0, r0 + 64) into the ring (waves 4-7: wave = n-block, both m-blocks)
  auto ps_rows = [&](int r0) {
    const int nb = wave - 4;
    f32x16 acc[2];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mb][r] = 0.f;
    const float* const arow[2] = {XR + ((r0 + lr) & (RING - 1)) * XS + hk,
                                  XR + ((r0 + 32 + lr) & (RING - 1)) * XS + hk};
    x3_rows<2, 4>(acc, arow, W.planes + W1_OFF + frag_off(32 * nb, BF, 2 * BF) + 8 * lane,
                  (abl & 1) ? (abl | 32) : abl);
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        PSR[((r0 + 32 * mb + acc_row(r, lane)) & (RING - 1)) * PSS + 32 * nb + lr] = acc[mb][r];
  };

  // prologue: the first tile's window [d0 - 32, d0 + 96) and the Ps of its first 64 rows
  {
    const int d0 = t0 * BT;
    f32x4 v[2];
    load_rows(d0 - BR, v);
    store_rows(d0 - BR, v);
    load_rows(d0 + BR, v);
    store_rows(d0 + BR, v);
    if (tid <= BT) RPS[t0 & 1][tid] = rowptr[min(d0 + tid, V)];
    __syncthreads();
    const int eb = RPS[t0 & 1][0], ne = RPS[t0 & 1][BT] - eb;
    if (tid < ne && ne <= BNT) CLS[t0 & 1][tid] = col[eb + tid];
    if (wave >= 4) ps_rows(d0 - BR);
  }

  // edge-phase lane roles: destination i (8 lanes), hidden units 4j + 32c (+0..3), features 8j..
  const int ei = tid >> 3, ej = tid & 7;
  __syncthreads();

  for (int tile = t0; tile < t1; ++tile) {
    const int d0 = tile * BT;
    const int lo = d0 - BR;               // the window: nodes [lo, lo + RING)
    const bool has_next = tile + 1 < t1;
    const int cur = tile & 1, nxt = cur ^ 1;
    f32x4 nextx[2];                       // the next tile's new rows [d0 + 96, d0 + 160)
    if (has_next) load_rows(d0 + BT + BR, nextx);
    int rpn = 0, cln = 0;                 // the next tile's rowptr (tid <= 64), then its col
    if (has_next && tid <= BT) rpn = rowptr[min(d0 + BT + tid, V)];

    // ---- A: Pt (waves 0-3: wave = n-block) | Ps of rows [d0 + 32, d0 + 96) (waves 4-7)
    if (wave < 4) {
      f32x16 acc[2];
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mb][r] = 0.f;
      const float* const arow[2] = {XR + ((d0 + lr) & (RING - 1)) * XS + hk,
                                    XR + ((d0 + 32 + lr) & (RING - 1)) * XS + hk};
      x3_rows<2, 4>(acc, arow, W.planes + W1_OFF + frag_off(32 * wave, 0, 2 * BF) + 8 * lane,
                    (abl & 1) ? (abl | 32) : abl);
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          PT[(32 * mb + acc_row(r, lane)) * PSS + 32 * wave + lr] = acc[mb][r];
    } else {
      ps_rows(d0 + BR);
    }
    __syncthreads();

    // ---- B: attention scores and normalised aggregation (gnn_utils.py:48-65)
    if (abl & 2) {                        // tuning ablation: no edge phase
      if (tid < BT) DEG[tid] = 0;
    } else {
      const int d = d0 + ei;
      const int eb = RPS[cur][0], ne = RPS[cur][BT] - eb;
      const int e0 = RPS[cur][ei], deg = RPS[cur][ei + 1] - e0;   // 0 past V
      const bool staged = ne <= BNT;
      auto col_of = [&](int q) { return staged ? CLS[cur][e0 - eb + q] : col[e0 + q]; };
      f32x4 pt[4], bb[4], ww[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        pt[c] = *reinterpret_cast<const f32x4*>(PT + ei * PSS + 4 * ej + 32 * c);
        bb[c] = *reinterpret_cast<const f32x4*>(B1W2 + 4 * ej + 32 * c);
        ww[c] = *reinterpret_cast<const f32x4*>(B1W2 + BH + 4 * ej + 32 * c);
      }
      auto alpha_of = [&](int s) {
        float acc = 0.f;
        if ((unsigned)(s - lo) < (unsigned)RING) {
          const float* ps = PSR + (s & (RING - 1)) * PSS + 4 * ej;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const f32x4 p = *reinterpret_cast<const f32x4*>(ps + 32 * c);
#pragma unroll
            for (int u = 0; u < 4; ++u) acc = fmaf(relu(pt[c][u] + p[u] + bb[c][u]), ww[c][u], acc);
          }
        } else {    // source outside the window: its Ps from global memory, on the VALU
          const float* xs = x + (size_t)s * BF;
#pragma unroll 1
          for (int q = 0; q < 16; ++q) {
            const int c = q >> 2, u = q & 3;
            const float* wr = W.w1 + (size_t)(4 * ej + 32 * c + u) * (2 * BF) + BF;
            float p = 0.f;
#pragma unroll 4
            for (int k = 0; k < BF; ++k) p = fmaf(wr[k], xs[k], p);
            const float hb = B1W2[4 * ej + 32 * c + u], hw = B1W2[BH + 4 * ej + 32 * c + u];
            const float ht = PT[ei * PSS + 4 * ej + 32 * c + u];
            acc = fmaf(relu(ht + p + hb), hw, acc);
          }
        }
#pragma unroll
        for (int o = 4; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 8);
        return sigmoidf_ref(acc + b2);
      };
      auto x_of = [&](int s, f32x4 (&v)[2]) {
        const float* src = (unsigned)(s - lo) < (unsigned)RING ? XR + (s & (RING - 1)) * XS
                                                               : x + (size_t)s * BF;
        v[0] = *reinterpret_cast<const f32x4*>(src + 8 * ej);
        v[1] = *reinterpret_cast<const f32x4*>(src + 8 * ej + 4);
      };
      int src[4];
      float a[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) src[q] = q < deg ? col_of(q) : d;
      float S = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        a[q] = 0.f;
        if (q < deg) {
          a[q] = alpha_of(src[q]);
          S += a[q];
        }
      }
#pragma unroll 1
      for (int q = 4; q < deg; ++q) S += alpha_of(col_of(q));
      const bool norm = S > 0.f;
      f32x4 g0 = {0.f, 0.f, 0.f, 0.f}, g1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q < deg) {
          const float wq = norm ? a[q] / S : a[q];
          f32x4 v[2];
          x_of(src[q], v);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            g0[c] = fmaf(wq, v[0][c], g0[c]);
            g1[c] = fmaf(wq, v[1][c], g1[c]);
          }
        }
#pragma unroll 1
      for (int q = 4; q < deg; ++q) {
        const int s = col_of(q);
        const float aq = alpha_of(s);
        const float wq = norm ? aq / S : aq;
        f32x4 v[2];
        x_of(s, v);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          g0[c] = fmaf(wq, v[0][c], g0[c]);
          g1[c] = fmaf(wq, v[1][c], g1[c]);
        }
      }
      *reinterpret_cast<f32x4*>(AG + ei * AS + 8 * ej) = g0;
      *reinterpret_cast<f32x4*>(AG + ei * AS + 8 * ej + 4) = g1;
      if (ej == 0) DEG[ei] = deg;
    }
    __syncthreads();

    // ---- C: [gate | u1] over [x_d ; agg]: waves 0-3 the x_d half of K, 4-7 the agg half;
    //      wave & 3 = 32-column quarter of the 128 outputs (0-1 gate, 2-3 u1)
    {
      const int nq = wave & 3, kh = wave >> 2;
      f32x16 acc[2];
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mb][r] = 0.f;
      const float* arow[2];
      if (kh == 0) {
        arow[0] = XR + ((d0 + lr) & (RING - 1)) * XS + hk;
        arow[1] = XR + ((d0 + 32 + lr) & (RING - 1)) * XS + hk;
      } else {
        arow[0] = AG + lr * AS + hk;
        arow[1] = AG + (32 + lr) * AS + hk;
      }
      const float* const ar[2] = {arow[0], arow[1]};
      x3_rows<2, 4>(acc, ar, W.planes + WC_OFF + frag_off(32 * nq, BF * kh, 2 * BF) + 8 * lane,
                    (abl & 4) ? (abl | 32) : abl);
      // the agg half's partials -> PT (accumulator layout), summed by the partner wave in order
      float* part = PT + nq * 2048 + lane;
      if (kh == 1) {
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
          for (int r = 0; r < 16; ++r) part[(mb * 16 + r) * 64] = acc[mb][r];
      }
      if (has_next && tid <= BT) RPS[nxt][tid] = rpn;
      __syncthreads();
      if (has_next) {                     // the next tile's sources, in flight during D
        const int nb0 = RPS[nxt][0], nn = RPS[nxt][BT] - nb0;
        if (tid < nn && nn <= BNT) cln = col[nb0 + tid];
      }
      if (kh == 0) {
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[mb][r] += part[(mb * 16 + r) * 64];
      }
      __syncthreads();                    // partials read: PT and AG are free
      if (kh == 0) {
        const int n = 32 * nq + lr;       // output column: gate (n < 64) or u1 (n - 64)
        if (nq < 2) {
          const float bias = W.gb[n];
#pragma unroll
          for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              AG[(32 * mb + acc_row(r, lane)) * AS + n] = sigmoidf_ref(acc[mb][r] + bias);
        } else {
          const float bias = W.ub1[n - BF];
#pragma unroll
          for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              PT[(32 * mb + acc_row(r, lane)) * PSS + (n - BF)] = relu(acc[mb][r] + bias);
        }
      }
    }
    __syncthreads();

    // ---- D: x_out = x_d + gate * (u1 Wu2^T + bu2)  (waves 0-3: 32 x 32 each)
    if (wave < 4) {
      const int mb = wave >> 1, nb = wave & 1;
      f32x16 acc[1];
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[0][r] = 0.f;
      const float* const arow[1] = {PT + (32 * mb + lr) * PSS + hk};
      x3_rows<1, 4>(acc, arow, W.planes + WU2_OFF + frag_off(32 * nb, 0, BF) + 8 * lane,
                    (abl & 8) ? (abl | 32) : abl);
      const int n = 32 * nb + lr;
      const float ub = W.ub2[n];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 32 * mb + acc_row(r, lane);
        const int d = d0 + row;
        if (d < V) {
          const float xd = XR[(d & (RING - 1)) * XS + n];
          x_out[(size_t)d * BF + n] =
              DEG[row] > 0 ? xd + AG[row * AS + n] * (acc[0][r] + ub) : xd;
        }
      }
    }
    __syncthreads();                      // x_d rows read: their slots take the next rows
    if (has_next) {
      store_rows(d0 + BT + BR, nextx);
      CLS[nxt][tid] = cln;
    }
    __syncthreads();
  }
}

// Host side -----------------------------------------------------------------------------------
bool gnn_layer_band_ok(const az_graph* g, int F, int H) {
  return F == BF && H == BH && g->V > 0 && g->band > 0 && g->band <= BR;
}

size_t gnn_layer_band_ws_bytes() { return ((size_t)3 * WTOT * 2 + 255) / 256 * 256; }

int gnn_layer_band(const az_graph* g, const float* x, const az_gnn_layer_w* w, float* x_out,
                   void* ws, hipStream_t s) {
  unsigned short* planes = static_cast<unsigned short*>(ws);
  hipLaunchKernelGGL(band_split_weights, dim3((WTOT / 8 + 255) / 256), dim3(256), 0, s,
                     w->att_w1, w->gate_w, w->upd_w1, w->upd_w2, planes);
  int rc = check_launch("band_split_weights");
  if (rc) return rc;
  static int cus = 0;                     // queried once per process
  if (cus <= 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      cus = n;
    else
      cus = 256;
  }
  const int ntiles = (g->V + BT - 1) / BT;
  const int per = (ntiles + cus - 1) / cus;
  const int blocks = (ntiles + per - 1) / per;
  const BandW bw = {planes, w->att_w1, w->att_b1, w->att_w2, w->att_b2, w->gate_b, w->upd_b1,
                    w->upd_b2};
  int abl = 0;
#ifdef AZ_TUNING   // timing ablations (results wrong by design): AZ_BAND_ABL bits 1 / 2 / 4 / 8 =
                   // no phase A / B / C / D math, 16 = no weight loads
  static const char* env_abl = tuning_env("AZ_BAND_ABL");
  abl = env_abl ? atoi(env_abl) : 0;
#endif
  hipLaunchKernelGGL(gnn_layer_band_kernel, dim3(blocks), dim3(BNT), 0, s, g->V, g->rowptr, g->col,
                     x, bw, x_out, ntiles, per, abl);
  return check_launch("gnn_layer_band_kernel");
}

}  // namespace az
