// fp32 on the bf16 matrix cores ("x3"): the exact three-term bf16 split of fp32 operands and the
// six-product MFMA step, shared by gemm_x3 (az_gemm.hip) and the band-mode GNN layer
// (az_gnn_band.hip).  Every fp32 x = h + m + l with h = rne(x), m = rne(x - h), l = rne(x - h - m)
// (|m| <= 2^-8 |x|, |l| <= 2^-16 |x|; all 24 significand bits kept), and a*b is the sum of the
// six leading cross products ah*bl + al*bh + am*bm + ah*bm + am*bh + ah*bh, each exact in fp32.
// Operands must be finite and below the bf16 maximum (~3.39e38): an infinite x (or one that
// rounds to an infinite h) leaves a NaN residual, so the product is NaN where an fp32 GEMM gives
// +-inf.  Network weights and activations on this path are finite; a non-finite operand is an
// upstream fault in either case.
#pragma once
#include "az_common.h"

namespace az {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// two floats -> one dword of two bf16 (round to nearest even; v_cvt_pk_bf16_f32, low = a)
__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
  const bf16x2 h = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, h);
}

// 8 consecutive floats -> three planes of 8 bf16 (element j in bits 16j.. of the 128-bit word):
// per pair one v_cvt_pk_bf16_f32 per plane, the residual from the packed halves (shift / mask).
// The two residuals of a pair are formed by different (exact) instructions, a - h and
// fma(h, -1, b), so the compiler does not pack them into v_pk_add_f32, which costs extra
// cycles beside MFMAs (MI355X_MICROARCH.md, filler prices).
__device__ __forceinline__ void split3(const f32x4& x0, const f32x4& x1, u32x4 (&o)[3]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float a = q < 2 ? x0[2 * q] : x1[2 * q - 4];
    const float b = q < 2 ? x0[2 * q + 1] : x1[2 * q - 3];
    const unsigned h = pk_bf16(a, b);
    const float ra = a - __uint_as_float(h << 16);
    const float rb = __builtin_fmaf(__uint_as_float(h & 0xFFFF0000u), -1.f, b);
    const unsigned m = pk_bf16(ra, rb);
    const float sa = ra - __uint_as_float(m << 16);
    const float sb = __builtin_fmaf(__uint_as_float(m & 0xFFFF0000u), -1.f, rb);
    o[0][q] = h;
    o[1][q] = m;
    o[2][q] = pk_bf16(sa, sb);
  }
}


// ---------------------------------------------------------------------------------------------
// fp32 on the fp16 matrix cores ("h3"): an fp32 x times its row's power-of-two scale s (so the
// row's largest |x s| lies in [2^13, 2^14)) is split into two fp16 terms h = rne(x s),
// l = rne(x s - h) (x s - h is exact in fp32); |x s - h - l| <= 2^-22 |x s| while l is a normal
// fp16, and <= 2^-25 absolutely below that, i.e. <= 2^-39 of the row's largest |x s|.  a*b is the
// sum of the three products ah*bl + al*bh + ah*bh (each exact in fp32); the dropped al*bl is
// <= 2^-22 |a s_a||b s_b|.  Per product that is <= 3 * 2^-22 |a||b| (+ the 2^-39 floors), an order
// of magnitude below the fp32 accumulation's own rounding over K = 3136 products
// (tests/test_gpu_kernels.py x3_bound).  v_mfma_f32_32x32x16_f16 runs at the bf16 rate: half the
// MFMAs of the six-product bf16 form and two LDS planes instead of three.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned pk_f16(float a, float b) {
  const f16x2 h = {(_Float16)a, (_Float16)b};
  return __builtin_bit_cast(unsigned, h);
}

// 8 consecutive floats of one row, scaled by s -> two planes of 8 fp16 (element j in bits 16j..)
__device__ __forceinline__ void split2s(const f32x4& x0, const f32x4& x1, float s, u32x4 (&o)[2]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float a = (q < 2 ? x0[2 * q] : x1[2 * q - 4]) * s;
    const float b = (q < 2 ? x0[2 * q + 1] : x1[2 * q - 3]) * s;
    const unsigned h = pk_f16(a, b);
    const f16x2 hh = __builtin_bit_cast(f16x2, h);
    o[0][q] = h;
    o[1][q] = pk_f16(a - (float)hh[0], b - (float)hh[1]);
  }
}

// The same fp16 terms three deep: h, m = rne(x s - h), l = rne(x s - h - m) (both differences
// exact in fp32).  (h + m) + l rebuilds x s exactly while l is a normal fp16 (|x s| >= 2^8 for
// |x s| < 2^15), and within 2^-25 absolutely below that; h, m are the two-term split above.
__device__ __forceinline__ void split3h(const f32x4& x0, const f32x4& x1, float s, u32x4 (&o)[3]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float a = (q < 2 ? x0[2 * q] : x1[2 * q - 4]) * s;
    const float b = (q < 2 ? x0[2 * q + 1] : x1[2 * q - 3]) * s;
    const unsigned h = pk_f16(a, b);
    const f16x2 hh = __builtin_bit_cast(f16x2, h);
    const float ra = a - (float)hh[0], rb = b - (float)hh[1];
    const unsigned m = pk_f16(ra, rb);
    const f16x2 mm = __builtin_bit_cast(f16x2, m);
    o[0][q] = h;
    o[1][q] = m;
    o[2][q] = pk_f16(ra - (float)mm[0], rb - (float)mm[1]);
  }
}

// power-of-two scale s with max |x s| in [2^(T-1), 2^T) for a row / tile maximum m (1 when m is 0
// or not finite), and its inverse
__device__ __forceinline__ float h3_scale(float m, int T, float* inv) {
  int e = 0;
  if (m > 0.f && m <= 3.4e38f) {
    int ex;
    (void)frexpf(m, &ex);
    e = min(120, max(-120, T - ex));
  }
  *inv = ldexpf(1.f, -e);
  return ldexpf(1.f, e);
}

// acc += A . B over one 16-k step of v_mfma_f32_32x32x16_f16, both operands as their two fp16
// terms (bit patterns in bf16x8 registers: a[0] = h, a[1] = l), the dropped l*l smallest;
// smallest first
__device__ __forceinline__ f32x16 mfma3_32x32x16_f16(const bf16x8 (&a)[2], const bf16x8 (&b)[2],
                                                    f32x16 t) {
  const f16x8 ah = __builtin_bit_cast(f16x8, a[0]), al = __builtin_bit_cast(f16x8, a[1]);
  const f16x8 bh = __builtin_bit_cast(f16x8, b[0]), bl = __builtin_bit_cast(f16x8, b[1]);
  t = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, t, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, t, 0, 0, 0);
}

// acc += A . B over one 16-k step of v_mfma_f32_32x32x16_bf16 with both operands as three bf16
// planes (a[0..2] = h, m, l of A's fragment, b[0..2] of B's), the dropped terms smallest first
__device__ __forceinline__ f32x16 mfma6_32x32x16(const bf16x8 (&a)[3], const bf16x8 (&b)[3],
                                                  f32x16 t) {
  t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], t, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], t, 0, 0, 0);
}

// A's rows are scaled into [2^13, 2^14) (fp16 max 65504); W's into [2^9, 2^10): W's scales are
// cached between weight updates (az_gemm.hip) and stay safe while the weights grow up to 64x.
constexpr int H3_TA = 14, H3_TW = 10;

// The P2 GEMM's fp16 planes are stored row-interleaved per 32-k step, [rows][K / 32][2][32]:
// one row's two planes for one k step form one 128-B line, so every LDS-DMA piece of a stage
// (8 rows x 128 B) moves whole lines.  With the planes apart ([2][rows][K]) a piece was 16 rows
// x 64 B, half of each line it touched: the stage fill alone took 0.93 us per 48-KB stage with
// two stages in flight against 0.60 for whole lines, above the stage's ~0.73 us of MFMA
// (profiles/r06/dma_pattern/).  Element offset of the 8-element chunk ch (k = 8 ch .. 8 ch + 7)
// of row r, plane pl, in a matrix of K columns (K % 32 == 0).
__host__ __device__ __forceinline__ size_t p2_chunk(size_t r, int ch, int pl, int K) {
  return r * 2 * (size_t)K + (size_t)(ch >> 2) * 64 + pl * 32 + (ch & 3) * 8;
}

// An A operand already in the P2 GEMM's form, made by whoever produced A (the Connect4 trunk,
// the fused split-K reduce of the GEMM before): planes = the two fp16 planes of x * s in the
// p2_chunk layout (split2s), sc = [2][M] (s, then 1 / s) with s = h3_scale(max_k |x|, H3_TA) --
// exactly what h3_split_rows_kernel would write, so the GEMM's bits do not depend on who split A.
struct PreSplitA {
  const unsigned short* planes;
  const float* sc;
};

// The policy / value heads taken straight from a P2 GEMM's tiles (az_linear_heads_fwd /
// az_transform_heads_fwd without y, az_c4_eval_fwd).  The heads are linear in
// y = x W^T + b (Connect4GNN.py:48-57: fc_policy / fc_value read y itself), so instead of storing
// its part of y, each block leaves the dot products of its tile's columns (+ b in the first k
// split) with the heads' weight rows: part[row][t][9], t = n_tile * splits + split, slot a < A the
// policy row a, slot 8 the value row.  heads_tiles_finalize_kernel sums the t in order, adds the
// heads' biases and runs log_softmax / exp / tanh.  y is never written: 12.8 MB less traffic per
// B = 512 call than the split-K slabs and the heads pass that re-read them.
// The stream-K form (gemm_x3_csk) writes one slot per wave instead: t = (64-column block) x
// max_pieces + piece, and its finalize reads each tile's piece count from the plan.
constexpr int HEADS_TILE_SLOTS = 9;
struct HeadsEpi {
  const float* wp;   // fc_policy.weight [A][N]
  const float* wv;   // fc_value.weight [N]
  int A;             // <= 8
  float* part;       // [M][P][HEADS_TILE_SLOTS]
  int mp;            // stream-K: slots per 64-column block (max pieces); 0: split-K form
  // the finalize's operands (launched by the GEMM's dispatch, which knows P)
  const float* bp;   // fc_policy.bias [A]
  const float* bv;   // fc_value.bias [1]
  float* logp;       // [M][A]
  float* pi;         // [M][A] (may be null)
  float* v;          // [M]
};

}  // namespace az
