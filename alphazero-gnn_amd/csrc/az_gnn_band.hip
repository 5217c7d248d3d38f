// Band-mode inference GNNLayer (gnn_utils.py:5-74) for node-ordered graphs whose in-edges stay
// near the diagonal -- every source s of a destination d has |s - d| <= 32, which the synthetic
// 32x32 grid in row-major order is (config 5: sources d +- 1, d +- 32) -- with F = 64 node
// features and H = 128 attention hidden units.  ONE launch per layer (+ a 3 us weight split):
//
//   per tile of 64 consecutive destination nodes [d0, d0 + 64), one 512-thread block per CU,
//   persistent over a contiguous run of tiles:
//     A  Pt = X[d0, d0+64) W1[:, :F]^T           (waves 0-3)   } fp16-form MFMAs: fp32 operands,
//        Ps = X[d0+32, d0+96) W1[:, F:]^T         (waves 4-7)   } row-scaled, as two fp16 terms
//                                                                  (az_x3.h), three products
//     B  alpha_e = sigmoid(w2 . relu(Pt[d] + Ps[s] + b1) + b2), agg_d = sum_e alpha_e / S x_s
//        (8 lanes per destination, edges in CSR order, S = sum alpha > 0: gnn_utils.py:48-65)
//     C  [gate | u1] = [x_d ; agg_d] [Wg ; Wu1]^T + b   (K split over the two wave halves)
//     D  x_out[d] = x_d + gate * (u1 Wu2^T + bu2)       (gnn_utils.py:67-71)
//
//   x and the SOURCE half of the attention projection live in a 128-row ring in LDS covering the
//   tile's window [d0 - 32, d0 + 96): each tile adds 64 new rows (their x and Ps) and drops 64,
//   so every node's x is read from HBM once and its Ps computed once per block run -- the
//   separate Ps projection GEMM (and its 268 MB write + gather at 512 grids) is gone.  Nothing
//   but x_out leaves the CU.  The weights (two fp16 planes in MFMA fragment order, each row scaled
//   by its power of two, split once per launch) stream from L2.
//
//   MFMA operands that come from LDS are stored ALREADY split: x rows enter the ring as the two
//   fp16 planes of x s (s the row's power-of-two scale, 1/s kept per ring slot), and each
//   destination's agg is written as its two planes over its own (consumed) Pt row.  The
//   aggregation takes its sources from the planes ((h + l) / s, within 2^-22 |x|); the residual
//   x + gate * u2 reads x itself (global memory, L2-resident: the rows entered the ring a tile
//   earlier), so a destination without in-edges gets x bit for bit (gnn_utils.py:35-36).
//   update_net.0's output (u1) and output_transform's operands (x_out, h) become fp16 planes in
//   place in PT, each row with its own scale.  Every GEMM's accumulators are multiplied back by
//   1 / (s_row s_w) (exact) before use.
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
constexpr int PSS = 132;      // Pt / agg-plane / [gate | u1] row stride (floats), = 4 (mod 64)
constexpr int PSRS = 128;     // Ps ring row stride: every row starts on bank 0, and the two
                              // destinations of a 16-lane read group take opposite halves
constexpr int XRS = 2 * BF;   // ring row: two planes of 64 fp16 (256 B), 16-B chunks swizzled

// weight planes [2][WTOT] fp16 in MFMA-fragment order: a matrix W [N][K] (nn.Linear [out][in])
// is stored as (N / 32) x (K / 16) blocks of 512 fp16, block (nb, ks) holding the B operand of
// one v_mfma_f32_32x32x16_f16 step lane by lane (lane l: row 32 nb + (l & 31), k = 16 ks +
// 8 (l >> 5) .. + 7), so a wave reads its fragment as ONE contiguous 1 KB (row-major planes
// made every lane touch its own cache line: 4x the L2 traffic)
constexpr int W1_OFF = 0;                    // attention.0    [128][128]
constexpr int WC_OFF = BH * 2 * BF;          // [gate.0 ; update_net.0]  [128][128]
constexpr int WU2_OFF = WC_OFF + 2 * BF * 2 * BF;   // update_net.2 [64][64]
constexpr int OT0_OFF = WU2_OFF + BF * BF;  // output_transform.0 [64][64] (fused tail, OT)
constexpr int OT2_OFF = OT0_OFF + BF * BF;   // output_transform.2 [64][64]
constexpr int WLAYER = OT0_OFF;              // the layer's own weights
constexpr int WTOT = OT2_OFF + BF * BF;      // plane stride
constexpr int FRAG = 512;                    // fp16 per fragment block
// 1 / s of every weight row (after the planes): W1 rows, [Wg ; Wu1] rows, Wu2, OT.0, OT.2
constexpr int WI_W1 = 0, WI_WC = 128, WI_WU2 = 256, WI_OT0 = 320, WI_OT2 = 384, WI_N = 448;

// offset of W[n][k .. k + 7] (k % 8 == 0) in a fragment-ordered matrix of K columns
__host__ __device__ constexpr int frag_off(int n, int k, int K) {
  return ((n >> 5) * (K >> 4) + (k >> 4)) * FRAG + ((n & 31) + 32 * ((k >> 3) & 1)) * 8;
}

struct BandW {
  const unsigned short* planes;              // [2][WTOT]
  const float* winv;                         // [WI_N] 1 / s per weight row
  const float *w1, *b1, *w2, *b2, *gb, *ub1, *ub2;
  const float *ob0, *ob2;                    // output_transform biases (OT only)
};

__device__ __forceinline__ float relu(float v) { return v > 0.f ? v : 0.f; }

// 1 / (1 + e^-v) with the hardware exp2 and reciprocal (~1 ulp each) instead of expf and an IEEE
// division: a few instructions instead of ~20, within 3e-7 relative of torch.sigmoid -- far
// inside the 2e-6 the layer is held to against the training path (tests/test_gpu_kernels.py).
// Below v = -80 the result nears fp32's denormal range, which the reciprocal flushes to zero:
// there the exact form (torch's 1 / (1 + exp(-v)): denormal, then 0 below -88.7), because a
// destination whose every score is that small is still normalised by S > 0 (gnn_utils.py:58).
__device__ __forceinline__ float sigmoid_fast(float v) {
  if (v < -80.f) return 1.f / (1.f + expf(-v));
  return __builtin_amdgcn_rcpf(1.f + __expf(-v));
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, false));
}

// sum over each aligned group of 8 lanes, the same bits in every lane of the group: quad_perm
// [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror -- three DPP adds (no LDS round trip, where
// __shfl_xor with width 8 is a ds_bpermute and a wait per step)
__device__ __forceinline__ float sum8(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  return v + dpp<0x141>(v);
}

// the same for the maximum (row scales of the fp16 planes)
__device__ __forceinline__ float max8(float v) {
  v = fmaxf(v, dpp<0xB1>(v));
  v = fmaxf(v, dpp<0x4E>(v));
  return fmaxf(v, dpp<0x141>(v));
}

__device__ __forceinline__ float absmax8(const f32x4 (&v)[2]) {
  float m = 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < 4; ++e) m = fmaxf(m, fabsf(v[h][e]));
  return m;
}

// 8 consecutive weights of one row -> their two fp16 planes, the row scaled by its power of two
// (max |w s| in [2^13, 2^14): every thread reads its row's <= 128 weights for the maximum); the
// row's first chunk also stores 1 / s in winv
__global__ __launch_bounds__(256) void band_split_weights(const float* __restrict__ w1,
                                                          const float* __restrict__ gw,
                                                          const float* __restrict__ uw1,
                                                          const float* __restrict__ uw2,
                                                          const float* __restrict__ ow0,
                                                          const float* __restrict__ ow2,
                                                          unsigned short* __restrict__ planes,
                                                          float* __restrict__ winv, int n) {
  const int i = (blockIdx.x * 256 + threadIdx.x) * 8;   // element of [W1 | Wg ; Wu1 | Wu2 | ..]
  if (i >= n) return;
  const float* src;
  int dst, len, wrow, pos;
  if (i < WC_OFF) {                       // W1 [128][128]
    src = w1 + i;
    dst = W1_OFF + frag_off(i >> 7, i & 127, 2 * BF);
    len = 2 * BF;
    wrow = WI_W1 + (i >> 7);
    pos = i & 127;
  } else if (i < WU2_OFF) {               // [Wg ; Wu1] [128][128]
    const int j = i - WC_OFF;
    src = j < BF * 2 * BF ? gw + j : uw1 + (j - BF * 2 * BF);
    dst = WC_OFF + frag_off(j >> 7, j & 127, 2 * BF);
    len = 2 * BF;
    wrow = WI_WC + (j >> 7);
    pos = j & 127;
  } else {                                // Wu2, then output_transform.0 / .2: [64][64] each
    const int m = (i - WU2_OFF) / (BF * BF), j = (i - WU2_OFF) % (BF * BF);
    src = (m == 0 ? uw2 : m == 1 ? ow0 : ow2) + j;
    dst = WU2_OFF + m * BF * BF + frag_off(j >> 6, j & 63, BF);
    len = BF;
    wrow = WI_WU2 + m * BF + (j >> 6);
    pos = j & 63;
  }
  const float* row = src - pos;
  float mx = 0.f;
  for (int k = 0; k < len; k += 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(row + k);
    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
  }
  float inv;
  const float sc = h3_scale(mx, 14, &inv);
  if (pos == 0) winv[wrow] = inv;
  const f32x4 x0 = *reinterpret_cast<const f32x4*>(src);
  const f32x4 x1 = *reinterpret_cast<const f32x4*>(src + 4);
  u32x4 o[2];
  split2s(x0, x1, sc, o);
#pragma unroll
  for (int pl = 0; pl < 2; ++pl)
    *reinterpret_cast<u32x4*>(planes + (size_t)pl * WTOT + dst) = o[pl];
}

// acc[mb] += A[32 rows of m-block mb][K = 16 KS] . W[32 rows][K]^T on fp16-form MFMAs, both
// operands as two fp16 planes.  a(mb, ks, pl) -> this lane's A fragment (plane pl of step ks); w:
// plane 0 of the first weight fragment block (frag_off(n0, k0, K) + 8 lane; the KS blocks of a
// row block are consecutive).
// this lane's weight fragments of KS k steps (2 planes each), requested from L2: issued a phase
// ahead of their MFMAs, so no GEMM of the tile starts by waiting for its weights.  Buffer loads
// off one descriptor: the lane part (16 B x lane) is the only VGPR, the fragment block's offset
// `w` (fp16 elements, wave-uniform) rides in an SGPR -- flat pointers per fragment would hold
// 16 VGPRs of addresses per weight set across the whole tile loop.
template <int KS, int ABL = 0>
__device__ __forceinline__ void load_w(bf16x8 (&b)[KS][2], __amdgpu_buffer_rsrc_t planes,
                                       int lane_off, int w) {
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int pl = 0; pl < 2; ++pl) {
      if constexpr ((ABL & 16) != 0) {
        b[ks][pl] = bf16x8{};             // tuning ablation: no weight loads
      } else {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
            planes, lane_off, 2 * (w + pl * WTOT + FRAG * ks), 0);
        b[ks][pl] = __builtin_bit_cast(bf16x8, v);
      }
    }
}

// acc[mb] += A . W^T with the weight fragments already in registers (load_w)
template <int MB, int KS, int ABL, typename AFrag>
__device__ __forceinline__ void h3_mfma(f32x16 (&acc)[MB], const AFrag& afrag,
                                        const bf16x8 (&b)[KS][2]) {
  if constexpr ((ABL & 32) != 0) return;  // tuning ablation: no A reads / MFMAs
  // A fragments one k step ahead of their MFMAs (LDS latency behind the previous step's)
  bf16x8 a[2][MB][2];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) afrag(mb, 0, a[0][mb]);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (ks + 1 < KS) {
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) afrag(mb, ks + 1, a[(ks + 1) & 1][mb]);
    }
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[mb] = mfma3_32x32x16_f16(a[ks & 1][mb], b[ks], acc[mb]);
  }
}

// row of register r of a 32x32 MFMA accumulator (column = lane & 31)
__device__ __forceinline__ int acc_row(int r, int lane) {
  return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}

// ring row `slot`, plane pl, 16-B chunk c (8 features) -> fp16 offset; the row's 16 chunk
// positions (both planes) are XOR-swizzled by the low 4 bits of slot with its bit pairs swapped
// (s1 s0 s3 s2), a bijection of slot mod 16:
//  * the 16 rows a 16-lane group of an MFMA fragment read touches (one plane, one chunk) land on
//    16 distinct 16-B bank positions of the 256-B row stride;
//  * the edge phase's source reads -- 4 destinations per 16-lane group, each reading 4 chunks of
//    its source, the sources of consecutive destinations in consecutive slots -- are conflict-free
//    too once each destination's lanes take their chunks in the order ej ^ x_chunk_flip(ei) (the
//    plain slot & 15 swizzle put two destinations of a group on the same 4 positions: 2-way
//    conflicts on every x read, 4.2e6 of the layer's 4.7e6 conflict cycles per launch, PMC r05i)
__device__ __forceinline__ int xr_swz(int slot) {
  return ((slot & 3) << 2) | ((slot >> 2) & 3);
}
__device__ __forceinline__ int xr_off(int slot, int pl, int c) {
  return slot * XRS + ((((pl << 3) | c) ^ xr_swz(slot)) << 3);
}
// the chunk order of destination ei's 8 lanes in the edge phase (searched with the swizzle above:
// flip the chunk's bit 2 for destinations 1 and 2 of every 4)
__device__ __forceinline__ int x_chunk_flip(int ei) { return ((ei + 1) & 2) << 1; }

// The edge phase's Pt / Ps / w2 reads (16-B chunks of 128 hidden units, 4 per lane, 16-lane
// read groups of 4 destinations x 4 lanes).  Ps rows (stride 128 floats) put chunk h on bank
// position h mod 16, Pt rows (stride PSS = 33 chunks) on (row + h) mod 16.  With the Pt of
// destination i in row i, no assignment of chunks to lanes is conflict-free for both (the 16
// positions of a group sum to 8 mod 16 in Ps, to 8 + 4 (4 e + 6) = 0 mod 16 in Pt for rows e ..
// e + 3).  So phase A stores destination i's Pt in row pt_row(i) (i's low 3 bits (b2 b1 b0) ->
// (b1 b0 b2): the group's 4 rows are 0, 2, 4, 6 apart), and lane (i, j) takes at step c the
// chunk h_chunk: the 4 destinations of a group use 4 different residues mod 4 at every step
// ((i + c) & 3; shifted by 2 (i & 3) in Pt still 4 different ones) and their lanes the 4
// multiples of 4 -- conflict-free in both (a row's agg planes go to row i: every Pt row of the
// wave is read before any agg write, so the permutation stays inside the wave's 8 rows).
__device__ __forceinline__ int pt_row(int i) { return (i & ~7) | ((i & 3) << 1) | ((i >> 2) & 1); }
__device__ __forceinline__ int h_chunk(int ei, int ej, int c) { return ((ei + c) & 3) + 4 * ej; }
// the row passes (split_pass, the residual, the y copy-out: 8 threads per row, 2 float4 reads
// each at PT stride 33 chunks): thread c of row i takes 8-float group row_chunk(i, c), rotated
// by one for rows 2, 3 (mod 4) -- plain c put rows i and i + 2 of a 16-lane group on the same
// bank positions (2-way conflicts on every read)
__device__ __forceinline__ int row_chunk(int i, int c) { return (c - ((i >> 1) & 1)) & 7; }

// the accumulator rows of register r relative to the lane's first (acc_row(r, lane) - acc_row(0,
// lane)), and an opaque copy of a lane's base offset: the per-register stores then use base +
// constant (the DS immediate offset) instead of 16 loop-invariant addresses hoisted out of the
// tile loop (which spill at 256 VGPRs)
__device__ __forceinline__ constexpr int acc_drow(int r) { return (r & 3) + 8 * (r >> 2); }
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

__device__ __forceinline__ void zero(f32x16& a) {
#pragma unroll
  for (int r = 0; r < 16; ++r) a[r] = 0.f;
}

}  // namespace

#ifdef AZ_TUNING
// ABL & 256 (tuning build): wall-clock stamps of block 0's waves 0 and 4 at the phase boundaries
// of its first 64 tiles, [wave group][tile][event] (tools/band_trace.py)
constexpr int BT_EV = 12, BT_TILES = 64;
__device__ unsigned long long g_band_trace[2 * BT_TILES * BT_EV];
#define BSTAMP(ev)                                                                            \
  do {                                                                                        \
    if constexpr ((ABL & 256) != 0)                                                           \
      if (blockIdx.x == 0 && lane == 0 && (wave & 3) == 0 && tile - t0 < BT_TILES)            \
        g_band_trace[((wave >> 2) * BT_TILES + (tile - t0)) * BT_EV + (ev)] = wall_clock64(); \
  } while (0)
#else
#define BSTAMP(ev) do {} while (0)
#endif

// ABL != 0 only in the tuning build: timing ablations, results wrong by design (bits 1 / 2 / 4 /
// 8 = no phase A / B / C / D math, 16 = no weight loads, 64 = no x_out stores, 128 = no x loads)
// OT: the layer is the network's last -- output_transform (gnn_utils.py:101-105,115: Linear +
// ReLU + Linear, every row) runs on the tile in LDS and only its output y is stored.
template <int ABL, bool OT>
__global__ __launch_bounds__(BNT, 1) void gnn_layer_band_kernel(
    int V, int E, const int* __restrict__ rowptr, const int* __restrict__ col,
    const float* __restrict__ x, BandW W, float* __restrict__ x_out, int ntiles, int per) {
  __shared__ __attribute__((aligned(16))) unsigned short XR[RING * XRS];  // x planes (ring)
  __shared__ __attribute__((aligned(16))) float PSR[RING * PSRS]; // Ps rows of the window
  __shared__ __attribute__((aligned(16))) float PT[BT * PSS];     // Pt -> agg planes ->
                                                                   // C partials -> [gate | u1]
  __shared__ __attribute__((aligned(16))) float B1W2[2 * BH];
  __shared__ float BS[5 * BF];            // biases: gate.0 | update_net.0 | update_net.2 | OT .0 | .2
  __shared__ int DEG[BT];
  __shared__ int RPS[2][BT + 1];          // rowptr of the tile's destinations (+1), prefetched
  __shared__ int CLS[2][BNT];             // the tile's sources (col), when it has <= 512 edges
  __shared__ float XSI[RING];             // 1 / s of each ring row's fp16 planes
  __shared__ float AGSI[BT];              // 1 / s of each destination's agg planes
  __shared__ float RSI[BT];               // 1 / s of each row's u1 (D) / x_out (E) / h (F) planes
  // update_net.2's two fp16 planes (fragment order), copied once per block: phase D reads its B
  // fragments here, so waves 0-3 request the next phase's weights from L2 a phase earlier and
  // the four D waves no longer fetch the same fragments twice
  __shared__ __attribute__((aligned(16))) unsigned short WU2L[2 * BF * BF];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 31, hc = lane >> 5;          // fragment row, k half (8-element chunk)
  const int t0 = blockIdx.x * per, t1 = min(ntiles, t0 + per);
  if (t0 >= t1) return;                   // uniform per block
  if (tid < BH) {
    B1W2[tid] = W.b1[tid];
    B1W2[BH + tid] = W.w2[tid];
  }
  if (tid < 5 * BF) {
    const int m = tid / BF, j = tid % BF;
    const float* b = m == 0 ? W.gb : m == 1 ? W.ub1 : m == 2 ? W.ub2 : m == 3 ? W.ob0 : W.ob2;
    BS[tid] = (OT || m < 3) ? b[j] : 0.f;
  }
  const float b2 = W.b2[0];

  // 64 x rows [r0, r0 + 64) -> the ring as planes: thread = (row tid >> 3, features 8 (tid & 7))
  // (every load is unconditional -- clamped address, result masked -- so the compiler can count
  // the loads in flight instead of draining all of them at the next wait)
  auto load_rows = [&](int r0, f32x4 (&v)[2]) {
    const int n = r0 + (tid >> 3), c = (tid & 7) * 8;
    const size_t nc = (size_t)min(max(n, 0), V - 1) * BF + c;
    v[0] = *reinterpret_cast<const f32x4*>(x + nc);
    v[1] = *reinterpret_cast<const f32x4*>(x + nc + 4);
    if (n < 0 || n >= V) v[0] = v[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto store_rows = [&](int r0, const f32x4 (&v)[2]) {
    const int slot = (r0 + (tid >> 3)) & (RING - 1);
    float inv;
    const float sc = h3_scale(max8(absmax8(v)), 14, &inv);   // the row's 8 threads agree
    u32x4 o[2];
    split2s(v[0], v[1], sc, o);
#pragma unroll
    for (int pl = 0; pl < 2; ++pl)
      *reinterpret_cast<u32x4*>(XR + xr_off(slot, pl, tid & 7)) = o[pl];
    if ((tid & 7) == 0) XSI[slot] = inv;
  };
  // x of a ring row, features 8c .. 8c + 7, from its two fp16 planes and 1 / s: (h + l) / s is
  // within 2^-22 |x| (2^-39 of the row maximum below l's normal range) -- the aggregation's
  // sources; the residual reads x itself from global memory
  auto x_planes = [](const u32x4& h, const u32x4& l, float inv, f32x4 (&v)[2]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // the dwords go through scalars: __builtin_bit_cast of an ext-vector ELEMENT (h[q])
      // compiles to a bit cast of element 0 for every q on this toolchain (ROCm 7.2 clang)
      const unsigned hq = h[q], lq = l[q];
      const f16x2 hh = __builtin_bit_cast(f16x2, hq), ll = __builtin_bit_cast(f16x2, lq);
      v[q >> 1][2 * (q & 1)] = ((float)hh[0] + (float)ll[0]) * inv;
      v[q >> 1][2 * (q & 1) + 1] = ((float)hh[1] + (float)ll[1]) * inv;
    }
  };
  auto x_ring = [&](int slot, int c, f32x4 (&v)[2]) {
    x_planes(*reinterpret_cast<const u32x4*>(XR + xr_off(slot, 0, c)),
             *reinterpret_cast<const u32x4*>(XR + xr_off(slot, 1, c)), XSI[slot], v);
  };
  // A fragments straight from the ring planes: rows r0 + 32 mb + (lane & 31)
  auto ring_frag = [&](int r0) {
    return [=](int mb, int ks, bf16x8 (&a)[2]) {
      const int slot = (r0 + 32 * mb + lr) & (RING - 1);
#pragma unroll
      for (int pl = 0; pl < 2; ++pl)
        a[pl] = *reinterpret_cast<const bf16x8*>(XR + xr_off(slot, pl, 2 * ks + hc));
    };
  };
  // A row segment of PT (64 floats from column col0: u1, h) -> its two fp16 planes IN PLACE
  // (plane pl at fp16 offset 64 pl of the segment, 16-B chunk c), scaled by the row's power of
  // two, 1 / s into RSI -- per row, not per tile, so rows of very different magnitudes keep
  // their own precision.  Thread = (row tid >> 3, chunk tid & 7): a row's 8 threads sit in one
  // wave and read their chunks before any of them writes (the row maximum needs all of them).
  auto split_pass = [&](int col0) {
    const int i = tid >> 3, c = row_chunk(i, tid & 7);
    float* const rowp = PT + i * PSS + col0;
    f32x4 v[2];
    v[0] = *reinterpret_cast<const f32x4*>(rowp + 8 * c);
    v[1] = *reinterpret_cast<const f32x4*>(rowp + 8 * c + 4);
    float inv;
    const float sc = h3_scale(max8(absmax8(v)), 14, &inv);
    u32x4 t[2];
    split2s(v[0], v[1], sc, t);
    unsigned short* pp = reinterpret_cast<unsigned short*>(rowp);
    *reinterpret_cast<u32x4*>(pp + 8 * c) = t[0];
    *reinterpret_cast<u32x4*>(pp + BF + 8 * c) = t[1];
    if (c == 0) RSI[i] = inv;
  };
  // A fragments from such planes: rows 32 mb + (lane & 31) of the segment at column col0
  auto plane_frag = [&](int mb, int col0) {
    return [=](int, int ks, bf16x8 (&a)[2]) {
      const unsigned short* row =
          reinterpret_cast<const unsigned short*>(PT + (32 * mb + lr) * PSS + col0);
#pragma unroll
      for (int pl = 0; pl < 2; ++pl)
        a[pl] = *reinterpret_cast<const bf16x8*>(row + pl * BF + 8 * (2 * ks + hc));
    };
  };
  // Each wave's weight fragments for the GEMM of the NEXT phase are requested as soon as the
  // current phase's MFMAs are issued (bw is one register set, reloaded after its last use): they
  // arrive behind the barriers and the edge phase instead of at the head of each GEMM.
  //   A  attention.0: waves 0-3 the target half (n-block = wave), 4-7 the source half
  //   C  [gate ; update_net.0]: n quarter wave & 3, K half wave >> 2
  //   D  update_net.2 (waves 0-3: n-block wave & 1); OT: output_transform.0 / .2 likewise
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(W.planes), 0, 2 * WTOT * 2, 0x00020000);
  const int wl = 16 * lane;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int wA = W1_OFF + frag_off(32 * (wv & 3), wv < 4 ? 0 : BF, 2 * BF);
  // C's column quarter of a wave: the agg-half waves (4-7) take the quarters of the x-half waves
  // on the other SIMDs' partner (quarter ^ 2), so each SIMD (waves w, w + 4) finishes one gate
  // quarter (sigmoid: two transcendentals per element) and one update_net.0 quarter (ReLU)
  const int cq = (wv & 3) ^ (wv < 4 ? 0 : 2);
  const int wC = WC_OFF + frag_off(32 * cq, BF * (wv >> 2), 2 * BF);
  const int wD = WU2_OFF + frag_off(32 * (wv & 1), 0, BF);
  bf16x8 bw[4][2];
  constexpr int AAB = (ABL & 1) ? (ABL | 32) : ABL;
  load_w<4, ABL>(bw, wr, wl, wA);

  // Ps rows [r0, r0 + 64) into the ring (waves 4-7: wave = n-block, both m-blocks; bw = wA)
  auto ps_rows = [&](int r0) {
    const int nb = wave - 4;
    f32x16 acc[2];
    zero(acc[0]);
    zero(acc[1]);
    h3_mfma<2, 4, AAB>(acc, ring_frag(r0), bw);
    const float wi = W.winv[WI_W1 + 32 * nb + lr];   // attention.0 row (hidden unit) scale
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int slot = (r0 + 32 * mb + acc_row(r, lane)) & (RING - 1);
        PSR[slot * PSRS + 32 * nb + lr] = acc[mb][r] * (XSI[slot] * wi);
      }
  };

  // prologue: the first tile's window [d0 - 32, d0 + 96) and the Ps of its first 64 rows
  {
#pragma unroll
    for (int j = tid; j < 2 * BF * BF / 8; j += BNT) {   // 16-B chunks of the two Wu2 planes
      const int pl = j / (BF * BF / 8), o = (j % (BF * BF / 8)) * 8;
      *reinterpret_cast<u32x4*>(WU2L + pl * BF * BF + o) =
          *reinterpret_cast<const u32x4*>(W.planes + (size_t)pl * WTOT + WU2_OFF + o);
    }
    const int d0 = t0 * BT;
    f32x4 v[2];
    load_rows(d0 - BR, v);
    store_rows(d0 - BR, v);
    load_rows(d0 + BR, v);
    store_rows(d0 + BR, v);
    if (tid <= BT) {                      // both parities: the unconditional prefetch reads
      RPS[t0 & 1][tid] = rowptr[min(d0 + tid, V)];         // RPS[nxt] even with no next tile
      RPS[(t0 + 1) & 1][tid] = rowptr[min(d0 + BT + tid, V)];
    }
    __syncthreads();
    const int eb = RPS[t0 & 1][0], ne = RPS[t0 & 1][BT] - eb;
    if (tid < ne && ne <= BNT) CLS[t0 & 1][tid] = col[eb + tid];
    if (wave >= 4) {                      // the window's first 128 rows; later tiles' new
      ps_rows(d0 - BR);                   // rows get theirs in the previous tile's phase D
      ps_rows(d0 + BR);
    }
  }

  // edge-phase lane roles: destination i (8 lanes), hidden units 4j + 32c (+0..3), features 8j..
  const int ei = tid >> 3, ej = tid & 7;
  __syncthreads();

  for (int tile = t0; tile < t1; ++tile) {
    BSTAMP(0);
    const int d0 = tile * BT;
    const int lo = d0 - BR;               // the window: nodes [lo, lo + RING)
    const bool has_next = tile + 1 < t1;
    const int cur = tile & 1, nxt = cur ^ 1;
    // prefetch, issued at the start of the edge phase and stored at the end of the tile: the
    // next tile's new x rows [d0 + 96, d0 + 160), its sources (col, from its rowptr staged a
    // tile earlier) and the rowptr of the tile after it
    f32x4 nextx[2];
    int cln = 0, rp2 = 0;
    auto prefetch = [&]() {               // unconditional (clamped) loads, see load_rows
      if constexpr ((ABL & 128) != 0) nextx[0] = nextx[1] = f32x4{0.f, 0.f, 0.f, 0.f};
      else load_rows(d0 + BT + BR, nextx);
      cln = col[max(0, min(RPS[nxt][0] + tid, E - 1))];
      rp2 = rowptr[min(d0 + 2 * BT + min(tid, BT), V)];
    };

    // ---- A: Pt (waves 0-3: wave = n-block); the Ps of the window's new rows [d0 + 32, d0 + 96)
    //      were computed by waves 4-7 during the previous tile's phase D
    if (wave < 4) {
      f32x16 acc[2];
      zero(acc[0]);
      zero(acc[1]);
      h3_mfma<2, 4, AAB>(acc, ring_frag(d0), bw);
      const float b1n = B1W2[32 * wave + lr];     // attention.0's bias, folded into Pt
      const float wi = W.winv[WI_W1 + 32 * wave + lr];
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = 32 * mb + acc_row(r, lane);
          const int prow = 32 * mb + 8 * (r >> 2) + ((r & 3) << 1) + hc;   // pt_row(row)
          PT[prow * PSS + 32 * wave + lr] = acc[mb][r] * (XSI[(d0 + row) & (RING - 1)] * wi) + b1n;
        }
    }
    BSTAMP(1);
    __syncthreads();
    BSTAMP(2);

    // ---- B: attention scores and normalised aggregation (gnn_utils.py:48-65); each
    //      destination's agg replaces its Pt row, as three planes.  The prefetch goes out first:
    //      this phase issues no other global load, so its HBM latency hides behind the edge
    //      math (the vector-memory counter retires in order: issued before a GEMM's weight
    //      loads, it would hold up that GEMM's first MFMA)
    prefetch();
    if constexpr ((ABL & 2) != 0) {       // tuning ablation: no edge phase
      if (tid < BT) DEG[tid] = 0;
    } else {
      const int d = d0 + ei;
      const int eb = RPS[cur][0], ne = RPS[cur][BT] - eb;
      const int e0 = RPS[cur][ei], deg = RPS[cur][ei + 1] - e0;   // 0 past V
      // the edge math, once for staged sources (LDS) and once for a tile with > 512 edges
      // (global col): two instantiations, so neither load is a generic (flat) one that would
      // make the compiler drain the prefetch before it
      // fast: every destination of this wave has deg <= 4 and all its sources inside the window
      // (any banded graph, the grid) -- no global loads and no loops in that instantiation, so
      // nothing in it has to wait for the prefetch (a global load on a rarely taken path shares
      // its destination registers with the LDS path and makes the compiler wait vmcnt there too)
      auto edges = [&](auto col_of, auto fast) {
        constexpr bool FAST = decltype(fast)::value;
        // lane: hidden units 4 h_chunk(ei, ej, c) (+0..3), c = 0..3 (conflict-free with Pt in
        // row pt_row(ei): see h_chunk)
        int hk[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) hk[c] = 4 * h_chunk(ei, ej, c);
        const float* const ptrow = PT + pt_row(ei) * PSS;
        f32x4 pt[4], ww[4];                 // Pt + b1, w2
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          pt[c] = *reinterpret_cast<const f32x4*>(ptrow + hk[c]);
          ww[c] = *reinterpret_cast<const f32x4*>(B1W2 + BH + hk[c]);
        }
        auto alpha_of = [&](int s) {
          float acc = 0.f;
          if (FAST || (unsigned)(s - lo) < (unsigned)RING) {
            // two interleaved partial sums (even / odd hidden unit): the adds and FMAs go out
            // as packed v_pk_add_f32 / v_pk_fma_f32, half the instructions of the scalar chain
            const float* ps = PSR + (s & (RING - 1)) * PSRS;
            f32x2 acc2 = {0.f, 0.f};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const f32x4 p = *reinterpret_cast<const f32x4*>(ps + hk[c]);
#pragma unroll
              for (int u = 0; u < 4; u += 2) {
                f32x2 t = f32x2{pt[c][u], pt[c][u + 1]} + f32x2{p[u], p[u + 1]};
                t = f32x2{relu(t.x), relu(t.y)};
                acc2 = __builtin_elementwise_fma(t, f32x2{ww[c][u], ww[c][u + 1]}, acc2);
              }
            }
            acc = acc2.x + acc2.y;
          } else {    // source outside the window: its Ps from global memory, on the VALU
            const float* xs = x + (size_t)s * BF;
#pragma unroll 1
            for (int q = 0; q < 16; ++q) {
              const int u = q & 3, h = 4 * h_chunk(ei, ej, q >> 2) + u;
              const float* wr = W.w1 + (size_t)h * (2 * BF) + BF;
              float p = 0.f;
#pragma unroll 4
              for (int k = 0; k < BF; ++k) p = fmaf(wr[k], xs[k], p);
              acc = fmaf(relu(ptrow[h] + p), B1W2[BH + h], acc);
            }
          }
          return sigmoid_fast(sum8(acc) + b2);
        };
        // this lane's feature chunk of the aggregation (ej in a destination-dependent order, so
        // the x reads of a 16-lane group hit 16 distinct bank positions: xr_off)
        const int ec = ej ^ x_chunk_flip(ei);
        auto x_of = [&](int s, f32x4 (&v)[2]) {
          if (FAST || (unsigned)(s - lo) < (unsigned)RING) {
            x_ring(s & (RING - 1), ec, v);
          } else {
            v[0] = *reinterpret_cast<const f32x4*>(x + (size_t)s * BF + 8 * ec);
            v[1] = *reinterpret_cast<const f32x4*>(x + (size_t)s * BF + 8 * ec + 4);
          }
        };
        int src[4];
        float a[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) src[q] = q < deg ? col_of(q) : d;
        // FAST: the four edges straight-line, a missing edge (q >= deg) scored on the
        // destination's own row and given weight 0 (S + 0 and g + 0 * x are exact for finite x):
        // all 16 Ps reads go out before the first use, and the four score reductions and
        // sigmoids interleave instead of each edge waiting behind its own branch and LDS reads
        float S = 0.f;
        if constexpr (FAST) {
          f32x4 p[4][4];
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int c = 0; c < 4; ++c)
              p[q][c] = *reinterpret_cast<const f32x4*>(PSR + (src[q] & (RING - 1)) * PSRS +
                                                        hk[c]);
          float z[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            f32x2 acc2 = {0.f, 0.f};
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
              for (int u = 0; u < 4; u += 2) {
                f32x2 t = f32x2{pt[c][u], pt[c][u + 1]} + f32x2{p[q][c][u], p[q][c][u + 1]};
                t = f32x2{relu(t.x), relu(t.y)};
                acc2 = __builtin_elementwise_fma(t, f32x2{ww[c][u], ww[c][u + 1]}, acc2);
              }
            z[q] = acc2.x + acc2.y;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) z[q] = sum8(z[q]);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float aq = sigmoid_fast(z[q] + b2);
            a[q] = q < deg ? aq : 0.f;
            S += a[q];
          }
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            a[q] = 0.f;
            if (q < deg) {
              a[q] = alpha_of(src[q]);
              S += a[q];
            }
          }
        }
        if constexpr (!FAST) {
#pragma unroll 1
          for (int q = 4; q < deg; ++q) S += alpha_of(col_of(q));
        }
        // alpha / S as alpha * (1 / S): one IEEE division per destination instead of one per
        // edge (<= 1.5 ulp apart; the layer is held to 2e-6 of the training path); a tiny S
        // (1 / S would overflow: every alpha near fp32's denormal range) divides per edge
        const bool norm = S > 0.f;
        const float rS = norm ? 1.f / S : 1.f;
        const bool tiny = norm && S < 0x1p-100f;
        f32x4 g[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
        if constexpr (FAST) {
          u32x4 xp[4][2];                   // the four sources' planes, all reads in flight
          float xi[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
#pragma unroll
            for (int pl = 0; pl < 2; ++pl)
              xp[q][pl] = *reinterpret_cast<const u32x4*>(XR + xr_off(src[q] & (RING - 1), pl, ec));
            xi[q] = XSI[src[q] & (RING - 1)];
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float wq = tiny ? a[q] / S : a[q] * rS;
            f32x4 v[2];
            x_planes(xp[q][0], xp[q][1], xi[q], v);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              g[0][c] = fmaf(wq, v[0][c], g[0][c]);
              g[1][c] = fmaf(wq, v[1][c], g[1][c]);
            }
          }
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (q < deg) {
              const float wq = tiny ? a[q] / S : a[q] * rS;
              f32x4 v[2];
              x_of(src[q], v);
#pragma unroll
              for (int c = 0; c < 4; ++c) {
                g[0][c] = fmaf(wq, v[0][c], g[0][c]);
                g[1][c] = fmaf(wq, v[1][c], g[1][c]);
              }
            }
        }
#pragma unroll 1
        for (int q = FAST ? deg : 4; q < deg; ++q) {
          const int s = col_of(q);
          const float aq = alpha_of(s);
          const float wq = tiny ? aq / S : aq * rS;
          f32x4 v[2];
          x_of(s, v);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            g[0][c] = fmaf(wq, v[0][c], g[0][c]);
            g[1][c] = fmaf(wq, v[1][c], g[1][c]);
          }
        }
        // the group's 8 lanes read their Pt row above (same wave, in order): the row now takes
        // agg's two fp16 planes (scaled by the row's power of two), plane pl at byte 128 pl,
        // 16-B chunk ec
        float ainv;
        const float asc = h3_scale(max8(absmax8(g)), 14, &ainv);
        u32x4 o[2];
        split2s(g[0], g[1], asc, o);
        unsigned short* arow = reinterpret_cast<unsigned short*>(PT + ei * PSS);
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) *reinterpret_cast<u32x4*>(arow + pl * BF + 8 * ec) = o[pl];
        if (ej == 0) AGSI[ei] = ainv;
      };
      bool ok = deg <= 4 && ne <= BNT;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q < deg && ne <= BNT)
          ok = ok && (unsigned)(CLS[cur][e0 - eb + q] - lo) < (unsigned)RING;
      if (__builtin_amdgcn_ballot_w64(!ok) == 0)      // wave-uniform
        edges([&](int q) { return CLS[cur][e0 - eb + q]; }, std::true_type{});
      else if (ne <= BNT)
        edges([&](int q) { return CLS[cur][e0 - eb + q]; }, std::false_type{});
      else
        edges([&](int q) { return col[e0 + q]; }, std::false_type{});
      if (ej == 0) DEG[ei] = deg;
    }
    load_w<4, ABL>(bw, wr, wl, wC);
    BSTAMP(3);
    __syncthreads();
    BSTAMP(4);

    // ---- C: [gate | u1] over [x_d ; agg]: waves 0-3 the x_d half of K (ring planes), 4-7 the
    //      agg half (planes in the Pt rows); wave & 3 = 32-column quarter (0-1 gate, 2-3 u1)
    {
      const int nq = cq, kh = wave >> 2;
      f32x16 acc[2];
      zero(acc[0]);
      zero(acc[1]);
      constexpr int CAB = (ABL & 4) ? (ABL | 32) : ABL;
      if (kh == 0) {
        h3_mfma<2, 4, CAB>(acc, ring_frag(d0), bw);
        load_w<4, ABL>(bw, wr, wl, OT ? wD + (OT0_OFF - WU2_OFF) : wA);   // D's come from LDS
      } else {
        h3_mfma<2, 4, CAB>(acc, [&](int mb, int ks, bf16x8 (&a)[2]) {
          const unsigned short* row = reinterpret_cast<const unsigned short*>(PT + (32 * mb + lr) * PSS);
#pragma unroll
          for (int pl = 0; pl < 2; ++pl)
            a[pl] = *reinterpret_cast<const bf16x8*>(row + pl * BF + 8 * (2 * ks + hc));
        }, bw);
        load_w<4, ABL>(bw, wr, wl, wA);           // waves 4-7 are idle until the next tile's phase A
      }
      {   // each K half back to fp32 units with its own row scales (x_d's / agg's) before the sum
        const float wi = W.winv[WI_WC + 32 * nq + lr];
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = 32 * mb + acc_row(r, lane);
            acc[mb][r] *= (kh == 0 ? XSI[(d0 + row) & (RING - 1)] : AGSI[row]) * wi;
          }
      }
      BSTAMP(5);
      // the two K halves' partials meet in the Ps ring's dead half (accumulator layout, 16 rows
      // per quarter): the slots of rows [d0 - 32, d0 + 32), read for the last time in phase B and
      // written next by the next tile's phase A -- so no barrier is needed before the partials
      // are stored, nor between reading them and storing [gate | u1] over the agg planes in PT.
      // Each wave of a pair keeps m-block kh, hands the other to its partner, and finishes its
      // own (sum = x_d half + agg half either way round: fp32 addition commutes)
      float* part = PSR + ((d0 - BR + 16 * nq) & (RING - 1)) * PSRS + lane;
      f32x16 mine;
      if (kh == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) part[(16 + r) * 64] = acc[1][r];
        mine = acc[0];
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) part[r * 64] = acc[0][r];
        mine = acc[1];
      }
      __syncthreads();                    // partials stored; every wave's agg-plane reads done
      BSTAMP(6);
#pragma unroll
      for (int r = 0; r < 16; ++r) mine[r] += part[(kh * 16 + r) * 64];
      const int n = 32 * nq + lr;         // output column: gate (n < 64) or u1 (n - 64)
      const float bias = BS[n];         // gate.0 (n < 64) | update_net.0
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = mine[r] + bias;
        PT[(32 * kh + acc_row(r, lane)) * PSS + n] = nq < 2 ? sigmoid_fast(v) : relu(v);
      }
      // the next tile's new x rows [d0 + 96, d0 + 160) into the ring: their slots (rows
      // [d0 - 32, d0 + 32)) were read for the last time by this phase's MFMAs, before the
      // barrier above
      if (has_next) store_rows(d0 + BT + BR, nextx);
    }
    __syncthreads();
    BSTAMP(7);

    // ---- D: x_out = x_d + gate * (u1 Wu2^T + bu2)  (waves 0-3: 32 x 32 each; u1 split here).
    //      Each MFMA wave replaces its gate elements in PT by gate * u2 (every element has one
    //      owner); then all 8 waves apply the residual row by row: a thread per (row, 8 features)
    //      adds x (global) to the products and stores x_out as two float4s (the MFMA layout would
    //      need 16 scattered 4-byte loads and stores per lane, on half the waves).  Meanwhile
    //      waves 4-7 compute the next tile's Ps rows into the ring's dead slots.
    // the residual's x rows, requested now (L2: they entered the ring a tile ago) and used after
    // the u2 barrier: x_out is x + gate * u2 with x itself, not its fp16 planes
    const int ri = tid >> 3, rc = row_chunk(ri, tid & 7);   // row, features 8 rc .. 8 rc + 7
    f32x4 xres[2];
    {
      const size_t xo = (size_t)min(d0 + ri, V - 1) * BF + 8 * rc;
      xres[0] = *reinterpret_cast<const f32x4*>(x + xo);
      xres[1] = *reinterpret_cast<const f32x4*>(x + xo + 4);
    }
    split_pass(BF);                       // u1 -> its fp16 planes, a scale per row
    __syncthreads();
    if (wave < 4) {
      const int mb = wave >> 1, nb = wave & 1;
      f32x16 acc[1];
      zero(acc[0]);
      bf16x8 bd[4][2];                    // update_net.2's fragments of this wave, from LDS
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
          bd[ks][pl] = *reinterpret_cast<const bf16x8*>(WU2L + pl * BF * BF + (wD - WU2_OFF) +
                                                         FRAG * ks + 8 * lane);
      h3_mfma<1, 4, (ABL & 8) ? (ABL | 32) : ABL>(acc, plane_frag(mb, BF), bd);
      const int n = 32 * nb + lr;
      const float ub = BS[2 * BF + n];
      const float wi = W.winv[WI_WU2 + n];
      const int r0 = opaque(32 * mb + acc_row(0, lane));
      float* const pg = PT + r0 * PSS + n;
#pragma unroll
      for (int r = 0; r < 16; ++r)                                    // gate * u2
        pg[acc_drow(r) * PSS] *= acc[0][r] * (RSI[r0 + acc_drow(r)] * wi) + ub;
    } else if (has_next) {
      ps_rows(d0 + BT + BR);              // the next tile's new rows (their x stored in C)
    }
    __syncthreads();                      // gate * u2 complete
    {
      const int i = ri, c = rc;
      const f32x4* gp = reinterpret_cast<const f32x4*>(PT + i * PSS + 8 * c);   // gate * u2
      const bool upd = DEG[i] > 0;
      f32x4 o[2];
      if (!upd) {                         // no in-edges: x itself, bit for bit (gnn_utils.py:35)
        o[0] = xres[0];
        o[1] = xres[1];
      } else {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 gu = gp[h];
#pragma unroll
          for (int e = 0; e < 4; ++e) o[h][e] = xres[h][e] + gu[e];
        }
      }
      if constexpr (OT) {                 // x_out's fp16 planes (phase E's A), scaled per row,
        float inv;                        // in place of the gate * u2 row the group just read
        const float sc = h3_scale(max8(absmax8(o)), 14, &inv);
        u32x4 t[2];
        split2s(o[0], o[1], sc, t);
        unsigned short* pp = reinterpret_cast<unsigned short*>(PT + i * PSS);
        *reinterpret_cast<u32x4*>(pp + 8 * c) = t[0];
        *reinterpret_cast<u32x4*>(pp + BF + 8 * c) = t[1];
        if (c == 0) RSI[i] = inv;
      } else {
        const int d = d0 + i;
        if (d < V) {
          if constexpr ((ABL & 64) == 0) {
            *reinterpret_cast<f32x4*>(x_out + (size_t)d * BF + 8 * c) = o[0];
            *reinterpret_cast<f32x4*>(x_out + (size_t)d * BF + 8 * c + 4) = o[1];
          } else if (o[0][0] == 12345.f) {
            x_out[0] = o[0][0];
          }
        }
      }
    }
    BSTAMP(8);
    if constexpr (OT) {
      // ---- E: h = relu(x_out W0^T + b0) -> PT[:, 64:128] (u1's planes, free once every wave's
      //      D MFMAs are done);  F: y = h W2^T + b2 -> HBM  (waves 0-3, 32 x 32 each; x_out's and
      //      h's fp16 planes scaled per row)
      __syncthreads();
      const int mb = (wave >> 1) & 1, nb = wave & 1, n = 32 * nb + lr;
      f32x16 acc[1];
      if (wave < 4) {
        zero(acc[0]);
        h3_mfma<1, 4, ABL>(acc, plane_frag(mb, 0), bw);
        load_w<4, ABL>(bw, wr, wl, wD + (OT2_OFF - WU2_OFF));
        const float bias = BS[3 * BF + n];
        const float wi = W.winv[WI_OT0 + n];
        const int r0 = opaque(32 * mb + acc_row(0, lane));
        float* const pe = PT + r0 * PSS + BF + n;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          pe[acc_drow(r) * PSS] = relu(acc[0][r] * (RSI[r0 + acc_drow(r)] * wi) + bias);
      }
      __syncthreads();                    // h complete; E's reads of x_out's scales done
      split_pass(BF);                     // h -> its fp16 planes, a scale per row
      __syncthreads();
      if (wave < 4) {
        zero(acc[0]);
        h3_mfma<1, 4, ABL>(acc, plane_frag(mb, BF), bw);
        load_w<4, ABL>(bw, wr, wl, wA);
        const float bias = BS[4 * BF + n];
        const float wi = W.winv[WI_OT2 + n];
        const int r0 = opaque(32 * mb + acc_row(0, lane));
        float* const pf = PT + r0 * PSS + n;
#pragma unroll
        for (int r = 0; r < 16; ++r)      // y over x_out's rows in PT (read by E, before F)
          pf[acc_drow(r) * PSS] = acc[0][r] * (RSI[r0 + acc_drow(r)] * wi) + bias;
      }
    }
    if constexpr (OT) __syncthreads();    // F's y rows in PT complete
    if constexpr (OT) {                   // y leaves row by row, two float4 per thread
      const int i = tid >> 3, c = row_chunk(i, tid & 7), d = d0 + i;
      if (d < V) {
        const float* src = PT + i * PSS + 8 * c;
        *reinterpret_cast<f32x4*>(x_out + (size_t)d * BF + 8 * c) = *reinterpret_cast<const f32x4*>(src);
        *reinterpret_cast<f32x4*>(x_out + (size_t)d * BF + 8 * c + 4) =
            *reinterpret_cast<const f32x4*>(src + 4);
      }
    }
    BSTAMP(9);
    if (has_next) CLS[nxt][tid] = cln;    // used only when the next tile has <= 512 edges
    if (tile + 2 < t1 && tid <= BT) RPS[cur][tid] = rp2;   // tile + 2 has this tile's parity
    __syncthreads();
    BSTAMP(10);
  }
}

// Host side -----------------------------------------------------------------------------------
bool gnn_layer_band_ok(const az_graph* g, int F, int H) {
  return F == BF && H == BH && g->V > 0 && g->band > 0 && g->band <= BR;
}

constexpr size_t band_planes_bytes() { return ((size_t)2 * WTOT * 2 + 255) / 256 * 256; }
size_t gnn_layer_band_ws_bytes() { return band_planes_bytes() + ((size_t)WI_N * 4 + 255) / 256 * 256; }

// One eval-mode GNNLayer on a band graph; with `ot` (output_transform.{0,2}.{weight,bias}: w0,
// b0, w2, b2) the layer is the network's last and x_out receives output_transform's output.
int gnn_layer_band(const az_graph* g, const float* x, const az_gnn_layer_w* w, float* x_out,
                   void* ws, hipStream_t s, const float* const* ot) {
  unsigned short* planes = static_cast<unsigned short*>(ws);
  float* winv = reinterpret_cast<float*>(static_cast<char*>(ws) + band_planes_bytes());
  const int n = ot ? WTOT : WLAYER;
  hipLaunchKernelGGL(band_split_weights, dim3((n / 8 + 255) / 256), dim3(256), 0, s,
                     w->att_w1, w->gate_w, w->upd_w1, w->upd_w2, ot ? ot[0] : nullptr,
                     ot ? ot[2] : nullptr, planes, winv, n);
  int rc = check_launch("band_split_weights");
  if (rc) return rc;
  static int cus = 0;                     // queried once per process
  if (cus <= 0) {
    int dev = 0, nc = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&nc, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        nc > 0)
      cus = nc;
    else
      cus = 256;
  }
  const int ntiles = (g->V + BT - 1) / BT;
  const int per = (ntiles + cus - 1) / cus;
  const int blocks = (ntiles + per - 1) / per;
  const BandW bw = {planes, winv, w->att_w1, w->att_b1, w->att_w2, w->att_b2, w->gate_b,
                    w->upd_b1, w->upd_b2, ot ? ot[1] : nullptr, ot ? ot[3] : nullptr};
#define AZ_BAND(A_)                                                                          \
  do {                                                                                       \
    if (ot)                                                                                  \
      hipLaunchKernelGGL((gnn_layer_band_kernel<A_, true>), dim3(blocks), dim3(BNT), 0, s,   \
                         g->V, g->E, g->rowptr, g->col, x, bw, x_out, ntiles, per);          \
    else                                                                                     \
      hipLaunchKernelGGL((gnn_layer_band_kernel<A_, false>), dim3(blocks), dim3(BNT), 0, s,  \
                         g->V, g->E, g->rowptr, g->col, x, bw, x_out, ntiles, per);          \
  } while (0)
#ifdef AZ_TUNING   // timing ablations (tools/gpu_band_abl.sh): AZ_BAND_ABL=<bits>
  static const char* env_abl = tuning_env("AZ_BAND_ABL");
  switch (env_abl ? atoi(env_abl) : 0) {
    case 1: AZ_BAND(1); break;
    case 2: AZ_BAND(2); break;
    case 4: AZ_BAND(4); break;
    case 8: AZ_BAND(8); break;
    case 16: AZ_BAND(16); break;
    case 15: AZ_BAND(15); break;
    case 31: AZ_BAND(31); break;
    case 223: AZ_BAND(223); break;
    case 256: AZ_BAND(256); break;
    default: AZ_BAND(0); break;
  }
#else
  AZ_BAND(0);
#endif
#undef AZ_BAND
  return check_launch("gnn_layer_band_kernel");
}

#ifdef AZ_TUNING
// tools/band_trace.py: the last traced launch's stamps (synchronous)
extern "C" int az_tuning_band_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_band_trace), sizeof(g_band_trace)) == hipSuccess
             ? (int)(sizeof(g_band_trace) / 8)
             : -1;
}
#endif

}  // namespace az
