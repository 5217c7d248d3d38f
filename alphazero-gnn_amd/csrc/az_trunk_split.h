// The Connect4 trunk's conv2 core in the fp16 split form, and the trunk in its latency form (one
// (board, quarter of the output channels) per block): shared by az_trunk.hip (c4_trunk_tile,
// c4_trunk_split_kernel) and az_gemm.hip (the batch-1 leaf kernel, c4_leaf_kernel), which cannot
// call across translation units (-fno-gpu-rdc).
//
// conv2 (Connect4Net.py:44-45) is an implicit GEMM: rows = (board, position), 64 output
// channels, K = 288 in (tap, ci) order.  It runs on v_mfma_f32_16x16x32_f16 in the h3 form of
// az_x3.h: conv1's output (ReLU'd) is scaled per board by a power of two (the board's largest
// value into [2^13, 2^14)) and split into two fp16 planes, conv2's weights per output channel the
// same way, and every 32-channel tap step is the three products ah*bl + al*bh + ah*bh -- a
// sixteenth of the f32 MFMA's cycles per product, three products: ~5x fewer MFMA cycles than the
// exact-f32 chain it replaces (v_mfma_f32_16x16x4_f32, 18,432 cycles per SIMD at 2 boards per
// block).  Each product is exact in fp32; the split keeps 22 bits of each operand relative to its
// board's / channel's maximum (az_x3.h), far inside the 1e-5 the features are held to.  Every
// kernel that computes a trunk row uses the same planes, the same taps in the same order and the
// same three MFMAs, so a board's features do not depend on the kernel or its batch (bit-identical
// across c4_trunk_kernel<NB>, the split form and the leaf kernel).
#pragma once
#include "az_common.h"
#include "az_trunk_rows.h"
#include "az_x3.h"

namespace az {

typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// conv2's fp32 weights staged in LDS (when no fragment-ordered copy is given): row co at stride
// W2S_STRIDE floats.  Stride = 2 (mod 32) makes the fragment reads (lane: co = 16 consecutive
// rows, ci = 2 values 9 floats apart per 32-lane half) hit 32 distinct ds_read_b32 banks.
constexpr int W2S_STRIDE = 290;
constexpr int W2S_FLOATS = 64 * W2S_STRIDE;

// conv1's output in LDS as the two fp16 planes: board b at 16-B unit C1_UNITS_PER_BOARD * b,
// padded 9x9 position pp at + 9 pp; channels 8g .. 8g + 7 of the high plane at + g, of the low
// plane at + 4 + g (unit 8 is padding).  The conv2 rows are taken in the order of
// az_trunk_rows.h (tools/gen_trunk_rows.py), which makes every A-fragment read conflict-free.
constexpr int C1_FLOATS_PER_BOARD = C1_UNITS_PER_BOARD * 4;
constexpr int C1_UNITS_PER_POS = 9;

// unit offset of tap t (3x3, row-major) relative to the output position's unit
__device__ __forceinline__ constexpr int c1_tap_units(int t) {
  return C1_UNITS_PER_POS * ((t / 3) * 9 + (t % 3));
}

// tile row table of NB boards per block
template <int NB>
__device__ __forceinline__ const uint16_t* trunk_rows() {
  if constexpr (NB == 1) return TROW1;
  else if constexpr (NB == 2) return TROW2;
  else if constexpr (NB == 3) return TROW3;
  else if constexpr (NB == 4) return TROW4;
  else if constexpr (NB == 5) return TROW5;
  else if constexpr (NB == 6) return TROW6;
  else if constexpr (NB == 7) return TROW7;
  else return TROW8;
}

// the unit of row entry e (b * 49 + p) at tap 0, lane group h (channels 8h .. 8h + 7)
__device__ __forceinline__ int c1_row_unit(int e, int h) {
  const int b = e / 49, p = e - 49 * b;
  return C1_UNITS_PER_BOARD * b + C1_UNITS_PER_POS * ((p / 7) * 9 + (p % 7)) + h;
}

// conv1 (Connect4Net.py:42-43) of channels 8g .. 8g + 7 at padded position pp of one board (bd:
// its padded 9x9 cells, w1s: the 288 weights then the 32 biases): the taps' fmaf chain, the
// bias, ReLU; 0 on the padding ring
__device__ __forceinline__ void conv1_octet(const float* w1s, const float* bd, int pp, int g,
                                            float (&v)[8]) {
  const int px = pp / 9, py = pp % 9;
  const bool in = px >= 1 && px <= 7 && py >= 1 && py <= 7;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int ci = 8 * g + j;
    float s = 0.f;
    if (in) {
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
          s = fmaf(w1s[ci * 9 + kh * 3 + kw], bd[(px - 1 + kh) * 9 + (py - 1 + kw)], s);
      s += w1s[32 * 9 + ci];
      s = s > 0.f ? s : 0.f;
    }
    v[j] = s;
  }
}

__device__ __forceinline__ float octet_max(const float (&v)[8]) {
  float m = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) m = fmaxf(m, v[j]);
  return m;
}

// the octet's two planes (scaled by sc) into the board's image
__device__ __forceinline__ void c1_store(float* c1b, int pp, int g, const float (&v)[8], float sc) {
  u32x4 o[2];
  split2s(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}, sc, o);
  u32x4* u = reinterpret_cast<u32x4*>(c1b) + C1_UNITS_PER_POS * pp + g;
  u[0] = o[0];
  u[4] = o[1];
}

// this lane's conv2 weights (breg[tap * 8 + j] = w2[co][8h + j][tap]) -> the fp16 planes of its 9
// B fragments, row co scaled by its power of two (the max over the 4 lanes that hold co: lanes
// ^ 16, ^ 32); returns 1 / scale
__device__ __forceinline__ float w2_planes(const float (&breg)[72], bf16x8 (&bh)[9],
                                           bf16x8 (&bl)[9]) {
  float m = 0.f;
#pragma unroll
  for (int s = 0; s < 72; ++s) m = fmaxf(m, fabsf(breg[s]));
  m = fmaxf(m, __shfl_xor(m, 16));
  m = fmaxf(m, __shfl_xor(m, 32));
  float inv;
  const float sc = h3_scale(m, H3_TA, &inv);
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    u32x4 o[2];
    split2s(f32x4{breg[8 * t], breg[8 * t + 1], breg[8 * t + 2], breg[8 * t + 3]},
            f32x4{breg[8 * t + 4], breg[8 * t + 5], breg[8 * t + 6], breg[8 * t + 7]}, sc, o);
    bh[t] = __builtin_bit_cast(bf16x8, o[0]);
    bl[t] = __builtin_bit_cast(bf16x8, o[1]);
  }
  return inv;
}

// one 32-channel tap step: acc += ah*bl + al*bh + ah*bh (smallest first)
__device__ __forceinline__ f32x4v conv2_step(const u32x4& ah, const u32x4& al, const bf16x8& bh,
                                             const bf16x8& bl, f32x4v acc) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  const h8 a0 = __builtin_bit_cast(h8, ah), a1 = __builtin_bit_cast(h8, al);
  const h8 b0 = __builtin_bit_cast(h8, bh), b1 = __builtin_bit_cast(h8, bl);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b1, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b0, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b0, acc, 0, 0, 0);
}

struct TrunkSplitSmem {
  __attribute__((aligned(16))) float w2s[17 * W2S_STRIDE];   // + pad row
  float bd[81 + 1];
  __attribute__((aligned(16))) float c1[C1_FLOATS_PER_BOARD];
  float w1s[32 * 9 + 32 + 1];
  int c1max;                              // the board's largest conv1 value (float bits, >= 0)
};

// Latency form of the trunk for a handful of boards (the arena's leaf + speculative children,
// B <= 8): block (b, q) computes output channels [16q, 16q + 16) of board b, so one board's
// trunk is spread over 4 CUs and each block stages a quarter of conv2's weights (18 KB instead
// of 74 KB).  Every block computes the board's whole conv1 (its scale is the board's maximum);
// the four waves take the four row tiles of az_trunk_rows.h (NB = 1): the same planes, taps and
// MFMAs as c4_trunk_tile, so the output is bit-identical to c4_trunk_kernel<NB>.  256 threads.
template <bool SC1 = false>   // SC1: write-through feature stores (handed to other blocks)
__device__ __forceinline__ void c4_trunk_split_block(
    const int8_t* __restrict__ boards, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2, float* __restrict__ feat, int b,
    int q, TrunkSplitSmem& sm) {
  constexpr int P = 49, PP = 81, CI = 32;
  const int tid = threadIdx.x;
  float* w2s = sm.w2s;
  float* bd = sm.bd;
  float* c1 = sm.c1;
  float* w1s = sm.w1s;
  const int lane = tid & 63, mt = tid >> 6;            // wave = row tile (4 x 16 rows >= 49)
  const int h = lane >> 4, c16 = lane & 15;
  const int co = q * 16 + c16;
  // all prologue loads in flight before the first wait (see c4_trunk_tile), then the stores
  constexpr int NW2 = (16 * 72 + 255) / 256;
  f32x4v wst[NW2];
  const f32x4v* w2q = reinterpret_cast<const f32x4v*>(w2 + (size_t)q * 16 * 288);
#pragma unroll
  for (int j = 0; j < NW2; ++j) wst[j] = w2q[min(tid + 256 * j, 16 * 72 - 1)];
  const int px = tid / 9, py = tid % 9;
  const bool inside = tid < PP && px >= 1 && px <= 7 && py >= 1 && py <= 7;
  const int8_t bv = boards[(size_t)b * P + (inside ? (px - 1) * 7 + (py - 1) : 0)];
  const float w1a = w1[tid];                                   // tid < 256 < CI * 9
  const int e1 = min(tid + 256, CI * 9 + CI - 1);
  const float w1b = e1 < CI * 9 ? w1[e1] : b1[e1 - CI * 9];
  const float bias = b2[co];
  const uint16_t* const rows = trunk_rows<1>();
  const uint16_t erow = rows[16 * mt + c16];                    // this lane's A row
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < NW2; ++j) {   // unguarded: lanes past the 1152 float4 write the pad row
    const int i = min(tid + 256 * j, 16 * 72);
    float* d = w2s + (i / 72) * W2S_STRIDE + (i % 72) * 4;
    d[0] = wst[j][0]; d[1] = wst[j][1]; d[2] = wst[j][2]; d[3] = wst[j][3];
  }
  bd[min(tid, PP)] = inside ? (float)bv : 0.f;   // unguarded (pad slot): keeps the load early
  w1s[tid] = w1a;
  w1s[min(tid + 256, CI * 9 + CI)] = w1b;          // unguarded (pad slot)
  if (tid == 0) sm.c1max = 0;
  __syncthreads();
  float breg[72];   // step tap * 8 + j takes channel 8h + j
#pragma unroll
  for (int s = 0; s < 72; ++s) {
    const int tap = s >> 3, ci = 8 * h + (s & 7);
    breg[s] = w2s[c16 * W2S_STRIDE + ci * 9 + (tap / 3) * 3 + (tap % 3)];
  }
  bf16x8 bh[9], bl[9];
  const float iw = w2_planes(breg, bh, bl);
  // conv1: 81 positions x 4 channel octets = 324 items over 256 threads, kept in registers
  // until the board's maximum (its plane scale) is known
  float v0[8], v1[8];
  const int i1 = tid + 256;
  conv1_octet(w1s, bd, tid >> 2, tid & 3, v0);
  if (i1 < PP * 4) conv1_octet(w1s, bd, i1 >> 2, i1 & 3, v1);
  else
#pragma unroll
    for (int j = 0; j < 8; ++j) v1[j] = 0.f;
  const float m = fmaxf(octet_max(v0), octet_max(v1));
  if (m > 0.f) atomicMax(&sm.c1max, __float_as_int(m));
  __syncthreads();
  float ia;
  const float sa = h3_scale(__int_as_float(sm.c1max), H3_TA, &ia);
  c1_store(c1, tid >> 2, tid & 3, v0, sa);
  if (i1 < PP * 4) c1_store(c1, i1 >> 2, i1 & 3, v1, sa);
  __syncthreads();
  const u32x4* const c1u = reinterpret_cast<const u32x4*>(c1);
  const int u0 = c1_row_unit(erow & 0x7fff, h);
  f32x4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int u = u0 + c1_tap_units(tap);
    acc = conv2_step(c1u[u], c1u[u + 4], bh[tap], bl[tap], acc);
  }
  const float os = ia * iw;                // both powers of two: exact
  if constexpr (SC1) {
    // the block's 16 channels x 49 positions are ONE contiguous, 16-B aligned run of 784 floats
    // (feat[b][16q * 49 ..]): staged in LDS (conv1's planes are no longer read) and written
    // through as 196 16-B stores instead of 784 dword ones (each an own fabric write when
    // write-through)
    __syncthreads();                                 // every wave is done reading c1
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = rows[16 * mt + 4 * h + r];
      if (!(e & 0x8000)) {
        const float v = acc[r] * os + bias;
        c1[c16 * P + e] = v > 0.f ? v : 0.f;
      }
    }
    __syncthreads();
    if (tid < 16 * P / 4) {
      float* dst = feat + (size_t)b * 3136 + (size_t)q * 16 * P;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 16 * P * 4, 0x00020000);
      const f32x4v v = *reinterpret_cast<const f32x4v*>(c1 + tid * 4);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rs, tid * 16, 0, 16);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = rows[16 * mt + 4 * h + r];
      if (!(e & 0x8000)) {
        const float v = acc[r] * os + bias;
        feat[(size_t)b * 3136 + co * P + e] = v > 0.f ? v : 0.f;
      }
    }
  }
}

}  // namespace az
