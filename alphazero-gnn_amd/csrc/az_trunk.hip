// Board trunks and policy/value heads.
//
// c4_trunk: Connect4Net conv1 -> ReLU -> conv2 -> ReLU -> flatten (connect4/Connect4Net.py:42-49)
// fused in one launch.  A 512-thread workgroup takes NB boards:
//   1. boards (int8) -> zero-padded 9x9 fp32 tiles in LDS
//   2. conv1 (1->32, 9 MACs/output) on the VALU into a zero-padded [NB][32][9][9] LDS image
//   3. conv2 as an implicit GEMM on MFMA 16x16x4 f32:  rows = (board, position) flattened
//      (NB*49), cols = 64 output channels, K = 288 ordered (tap, ci = 8h + j) so that the 8
//      A-fragments of a tap are TWO ds_read_b128 per lane (conv1's output is laid out
//      [board][position][channel]).  Each wave owns a 16-channel column tile and keeps its 72
//      weight fragments in VGPRs for the whole launch.
//   4. bias + ReLU epilogue into an LDS copy of the NB NCHW-flattened feature rows, written to
//      HBM as contiguous float4 rows.
#include <stdlib.h>

#include <algorithm>
#include "az_common.h"
#include "az_heads.h"
#include "az_trunk_split.h"
#include "az_x3.h"

namespace az {

// LDS the kernel hands to c4_trunk_tile: (unregistered weights only) conv2's weights while they
// are read into registers, then (NB <= 4) the NB*3136-float output staging tile, or (NB > 4, no
// staging) conv1's output.  REGW (registered weights: the fragment-ordered copy is loaded straight
// into registers) drops the 74 KB staging room, so NB <= 3 fits two blocks per CU.
//
// Round 5 ran two blocks per CU and got WRONG rows, nondeterministically, in blocks sharing a CU.
// Round 6 found the cause (tools/trunk_selfcheck_probe.py, profiles/r06/trunk_packed_fp32/):
// conv1's packed-FP32 fma chain (v_pk_fma_f32, two channels per instruction, the low operand
// register written by the VALU instruction just before) returned a wrong LOW element in lanes
// 48-63 -- the wave's last quarter -- only while another workgroup's waves shared the SIMD.
// The conv1 image was then stored from those values (each thread's re-derivation of its item
// disagreed with itself in exactly that element).  Every kernel is now compiled without
// packed-FP32 code (azhip/build.py NO_PK_F32; tests/test_lib_abi.py asserts none is left), and
// with it the probe finds no mismatch in 12 runs at two blocks per CU.
#ifdef AZ_TRUNK_SELFCHECK
__device__ unsigned* g_trunk_chk;   // residency experiment log (az_debug_trunk_chk)
#endif

template <int NB, bool REGW>
constexpr int trunk_union_floats() {
  constexpr int after = NB <= 4 ? NB * 3136 : NB * C1_FLOATS_PER_BOARD;
  return REGW || after >= W2S_FLOATS ? after : W2S_FLOATS;
}

// occupancy asked of the compiler (waves per SIMD): two 8-wave blocks per CU where their LDS fits
// (REGW, NB <= 3: <= 76 KB per block), else no constraint
template <int NB, bool REGW>
constexpr int trunk_waves_per_eu() { return REGW && NB <= 3 ? 4 : 1; }
template <int NB, bool REGW>
constexpr int trunk_blocks_per_cu() { return REGW && NB <= 3 ? 2 : 1; }

// The standard heads (Connect4Net.py:48-57: log_softmax(feat wp^T + bp), tanh(feat wv^T + bv)) of
// the block's feature rows, for predict_both batches whose trunk stages its rows in LDS.
struct TrunkHeads {
  const float* wp; const float* bp; int A; const float* wv; const float* bv;
  float* logp; float* pi; float* v;
};

// heads_rowsw_kernel's arithmetic on rows already in LDS (ob: nb rows of 3136 floats): wave w takes
// chunks w, w + 8, ... (256 columns each, the chunk's head weights loaded once for all nb rows),
// the same per-(row, chunk) fma chains and wave reductions, the chunk partials summed in chunk
// order from 0, then the same log_softmax / exp / tanh -- so the outputs are az_heads_fwd's bits.
template <int NB>
__device__ __forceinline__ void trunk_rows_heads(const float* ob, int nb, int b0,
                                                 const TrunkHeads& hd) {
  constexpr int AMAX = 8, PW = AMAX + 1, K = 3136, NCH = (K + HEADS_KC - 1) / HEADS_KC;
  __shared__ float part[NB][NCH][PW];
  __shared__ float hsm[NB][PW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int A = hd.A;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  // Wave w takes chunks w and w + 8 (13 chunks, 8 waves), both chunks' weight loads issued up
  // front.  The NB boards of a chunk are formed and reduced with no control flow between them
  // (rows past nb use zeros and are not stored), so their exchange chains overlap instead of
  // running board after board.  Each (row, chunk) partial is still the same fma chain and the
  // same wave_multi_sum / wave sum, so the bits are az_heads_fwd's.
  static_assert(NCH <= 16, "two chunks per wave");
  auto load_w = [&](int c, f32x4 (&w)[AMAX + 1], bool& kin, int& kc) {
    const int k = c * HEADS_KC + lane * 4;
    kin = k < K;
    kc = kin ? k : 0;
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
      w[a] = *reinterpret_cast<const f32x4*>(hd.wp + (size_t)min(a, A - 1) * K + kc);
    w[AMAX] = *reinterpret_cast<const f32x4*>(hd.wv + kc);
  };
  auto chunk = [&](int c, f32x4 (&w)[AMAX + 1], bool kin, int kc) {
#pragma unroll
    for (int a = 0; a < AMAX; ++a) w[a] = (a < A && kin) ? w[a] : z;
    w[AMAX] = kin ? w[AMAX] : z;
    float ps[NB], vs[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const f32x4 x = kin && b < nb ? *reinterpret_cast<const f32x4*>(ob + b * K + kc) : z;
      float pv[AMAX];
#pragma unroll
      for (int a = 0; a < AMAX; ++a)
        pv[a] = fmaf(x[3], w[a][3], fmaf(x[2], w[a][2], fmaf(x[1], w[a][1], x[0] * w[a][0])));
      ps[b] = wave_multi_sum<AMAX>(pv);
      vs[b] = wave_sum_x(
          fmaf(x[3], w[AMAX][3], fmaf(x[2], w[AMAX][2], fmaf(x[1], w[AMAX][1], x[0] * w[AMAX][0]))));
    }
    const int a = lane >> 3;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (b < nb && (lane & 7) == 0 && a < A) part[b][c][a] = ps[b];
      if (b < nb && lane == 0) part[b][c][A] = vs[b];
    }
  };
  f32x4 w0[AMAX + 1], w1[AMAX + 1];
  bool kin0, kin1 = false;
  int kc0, kc1 = 0;
  const bool two = wave + 8 < NCH;
  load_w(wave, w0, kin0, kc0);
  if (two) load_w(wave + 8, w1, kin1, kc1);
  chunk(wave, w0, kin0, kc0);
  if (two) chunk(wave + 8, w1, kin1, kc1);
  __syncthreads();
  if (tid < NB * PW) {
    const int b = tid / PW, a = tid % PW;
    if (b < nb && a <= A) {
      float s = 0.f;
      for (int c = 0; c < NCH; ++c) s += part[b][c][a];
      hsm[b][a] = s;
    }
  }
  __syncthreads();
  if (tid < nb) {
    const int row = b0 + tid;
    float l[AMAX];
    float mx = -INFINITY;
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
      if (a < A) {
        l[a] = hsm[tid][a] + hd.bp[a];
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
        hd.logp[(size_t)row * A + a] = o;
        if (hd.pi) hd.pi[(size_t)row * A + a] = expf(o);
      }
    hd.v[row] = tanhf(hsm[tid][A] + hd.bv[0]);
  }
}

// The trunk of one 512-thread block (boards blockIdx.x*NB ...).  `un` is LDS of
// trunk_union_floats<NB, REGW>() floats: conv2's weights are staged there with coalesced float4 loads
// (each lane then reads its 72 fragments from LDS -- one pass over the 74 KB per block instead of
// 72 scattered 4-byte loads per lane in all 8 waves), and with NB <= 4 the feature rows are then
// assembled in it (still there on return).
// apl / asc (NB <= 4 only; may be null): the feature rows also leave as the P2 GEMM's A operand
// for output_transform.0 (PreSplitA: two fp16 planes in the p2_chunk layout and scales [2][B], the bits
// h3_split_rows_kernel would make of feat), so that GEMM needs no split launch of its own.
// REGW: w2f (non-null) is conv2's weights already in fragment order (az_gemm.hip conv2_frags,
// cached per weight generation): each lane loads its 72 weights as 18 coalesced float4 loads,
// issued first, and the LDS staging of w2 (its bank-conflicted scalar stores and reads, a barrier)
// is skipped; the registers hold the same values, so the bits are the same.  !REGW: w2f unused.
template <int NB, bool HEADS = false, bool REGW = false>
__device__ __forceinline__ void c4_trunk_tile(const int8_t* __restrict__ boards, int B,
                                              const float* __restrict__ w1,
                                              const float* __restrict__ b1,
                                              const float* __restrict__ w2,
                                              const float* __restrict__ b2,
                                              float* __restrict__ feat, float* un,
                                              unsigned short* __restrict__ apl = nullptr,
                                              float* __restrict__ asc = nullptr,
                                              const float* __restrict__ w2f = nullptr,
                                              const TrunkHeads* hd = nullptr) {
  static_assert(!HEADS || NB <= 4, "HEADS: the rows staged in LDS");
  float* const ob = un;
  constexpr int P = 49, PP = 81, CI = 32;
  constexpr int NT = TTILES[NB];          // 16-row tiles (az_trunk_rows.h order)
  // STAGE: the output tile is assembled in LDS in NCHW-flatten order and written as whole
  // float4 rows (the MFMA layout puts 16 channels 49 floats apart on consecutive lanes, so
  // direct stores scatter 4-byte writes); NB = 8 lacks the LDS for it
  constexpr bool STAGE = NB <= 4;
  __shared__ float bd[NB * PP + 1];
  // conv1's output planes (az_trunk_split.h): own LDS when the output is staged (NB <= 4), else
  // in `un` once conv2's weights have moved to registers
  __shared__ __attribute__((aligned(16))) float c1s[STAGE ? NB * C1_FLOATS_PER_BOARD : 4];
  float* const c1 = STAGE ? c1s : un;
  __shared__ float w1s[CI * 9 + CI + 1];   // conv1 weights, bias, pad: one round trip, then LDS
  __shared__ float c1wmax[NB][8];          // each board's largest conv1 value, per wave
  __shared__ float c1inv[NB];              // ... its planes' 1 / scale
  const int tid = threadIdx.x;
  const int b0 = blockIdx.x * NB;
  const int nb = min(NB, B - b0);
  const int lane = tid & 63, wave = tid >> 6;
  const int nt = wave & 3, mh = wave >> 2;
  const int h = lane >> 4, c16 = lane & 15;
  const int co = nt * 16 + c16;
  const uint16_t* const rows = trunk_rows<NB>();
  // Every global load of the prologue is issued before the first one is waited for (conv2's
  // 9 float4 per thread, the boards, conv1's weights, the bias), then the LDS stores: as a
  // load -> store loop each iteration waited for its own round trip (11 in a row).
  // conv2's weights -> LDS (row co = 288 floats = 72 float4, so no float4 crosses a row), or
  // straight into the fragment registers from the fragment-ordered copy
  constexpr int NW2 = 64 * 72 / 512;
  f32x4v wst[NW2];
  float breg[72];   // step s = tap * 8 + j takes channel ci = 8h + j of tap (lane group h)
  if constexpr (REGW) {
#pragma unroll
    for (int q = 0; q < 18; ++q) {
      const f32x4v v = reinterpret_cast<const f32x4v*>(w2f)[(nt * 18 + q) * 64 + lane];
#pragma unroll
      for (int e = 0; e < 4; ++e) breg[4 * q + e] = v[e];
    }
  } else {
#pragma unroll
    for (int j = 0; j < NW2; ++j) wst[j] = reinterpret_cast<const f32x4v*>(w2)[tid + 512 * j];
  }
  constexpr int NBD = (NB * PP + 511) / 512;
  int8_t bdv[NBD];
  bool bdin[NBD];
#pragma unroll
  for (int j = 0; j < NBD; ++j) {
    const int i = tid + 512 * j;
    const int b = i / PP, pp = i % PP, px = pp / 9, py = pp % 9;
    bdin[j] = i < NB * PP && b < nb && px >= 1 && px <= 7 && py >= 1 && py <= 7;
    bdv[j] = boards[bdin[j] ? (size_t)(b0 + b) * P + (px - 1) * 7 + (py - 1) : (size_t)b0 * P];
  }
  const float w1v = tid < CI * 9 ? w1[tid] : b1[min(tid - CI * 9, CI - 1)];
  const float bias = b2[co];
  __builtin_amdgcn_sched_barrier(0);   // no load sinks into the guarded stores below
  if constexpr (!REGW) {
#pragma unroll
    for (int j = 0; j < NW2; ++j) {
      const int i = tid + 512 * j;
      float* d = un + (i / 72) * W2S_STRIDE + (i % 72) * 4;
      d[0] = wst[j][0]; d[1] = wst[j][1]; d[2] = wst[j][2]; d[3] = wst[j][3];
    }
  }
#pragma unroll
  for (int j = 0; j < NBD; ++j)   // unguarded (past-the-end lanes hit bd's pad slot): a guarded
    bd[min(tid + 512 * j, NB * PP)] = bdin[j] ? (float)bdv[j] : 0.f;   // use sinks the load
  w1s[min(tid, CI * 9 + CI)] = w1v;     // unguarded: lanes past the 320 weights hit the pad
  __syncthreads();
  if constexpr (!REGW) {
#pragma unroll
    for (int s = 0; s < 72; ++s) {
      const int tap = s >> 3, ci = 8 * h + (s & 7);
      breg[s] = un[co * W2S_STRIDE + ci * 9 + (tap / 3) * 3 + (tap % 3)];
    }
  }
  bf16x8 bh[9], bl[9];
  const float iw = w2_planes(breg, bh, bl);
  if constexpr (!STAGE && !REGW) __syncthreads();   // conv1's output overwrites the weights in `un`
  // conv1: (board, padded position, channel octet) items, kept in registers until each board's
  // maximum (its plane scale) is known
  constexpr int NI = NB * PP * 4, NIT = (NI + 511) / 512;
  float cv[NIT][8];
  float cm[NB];                            // this lane's maximum per board, then the wave's
#pragma unroll
  for (int b = 0; b < NB; ++b) cm[b] = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int i = tid + 512 * it;
    if (i < NI) {
      const int b = i / (PP * 4), r = i - b * (PP * 4);
      conv1_octet(w1s, bd + b * PP, r >> 2, r & 3, cv[it]);
      const float m = octet_max(cv[it]);
#pragma unroll
      for (int q = 0; q < NB; ++q)
        if (q == b) cm[q] = fmaxf(cm[q], m);
    }
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cm[b] = fmaxf(cm[b], __shfl_xor(cm[b], o));
    if (lane == 0) c1wmax[b][wave] = cm[b];
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int i = tid + 512 * it;
    if (i < NI) {
      const int b = i / (PP * 4), r = i - b * (PP * 4);
      float mx = c1wmax[b][0];
#pragma unroll
      for (int w = 1; w < 8; ++w) mx = fmaxf(mx, c1wmax[b][w]);
      float inv;
      const float sa = h3_scale(mx, H3_TA, &inv);
      c1_store(c1 + b * C1_FLOATS_PER_BOARD, r >> 2, r & 3, cv[it], sa);
      if (r == 0) c1inv[b] = inv;
    }
  }
  __syncthreads();
#ifdef AZ_TRUNK_SELFCHECK
  // residency experiment: every thread re-derives conv1 item i (conv1_octet + the split, the
  // same arithmetic) and compares the two 16-B units of the image in LDS; mismatches are logged
  // to g_trunk_chk (vector atomics only): [0] = count, then 8 words per entry
  auto c1_check = [&](int phase, int i) {
    if (i >= NI || !g_trunk_chk) return;
    const int b = i / (PP * 4), r = i - b * (PP * 4);
    float v[8], v2[8];
    conv1_octet(w1s, bd + b * PP, r >> 2, r & 3, v);
    asm volatile("" ::: "memory");
    conv1_octet(w1s, bd + b * PP, r >> 2, r & 3, v2);
    float mx = c1wmax[b][0];
    for (int w = 1; w < 8; ++w) mx = fmaxf(mx, c1wmax[b][w]);
    float inv;
    const float sa = h3_scale(mx, H3_TA, &inv);
    u32x4 o[2];
    split2s(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}, sa, o);
    const u32x4* u = reinterpret_cast<const u32x4*>(c1 + b * C1_FLOATS_PER_BOARD) +
                     C1_UNITS_PER_POS * (r >> 2) + (r & 3);
    const u32x4 x0 = u[0], x1 = u[4];
    int nbad = 0, nconv = 0;
    for (int e = 0; e < 4; ++e) nbad += (x0[e] != o[0][e]) + (x1[e] != o[1][e]);
    for (int e = 0; e < 8; ++e) nconv += __float_as_uint(v[e]) != __float_as_uint(v2[e]);
    if (nbad || nconv) {
      const unsigned k = atomicAdd(g_trunk_chk, 1u);
      if (k < 2048) {
        unsigned* d = g_trunk_chk + 64 + 48 * k;
        d[0] = blockIdx.x; d[1] = tid; d[2] = i; d[3] = phase;
        d[4] = nbad; d[5] = nconv;
        d[6] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));   // HW_ID
        d[7] = __float_as_uint(sa);
        for (int e = 0; e < 4; ++e) {
          d[8 + e] = x0[e]; d[12 + e] = x1[e];
          d[16 + e] = o[0][e]; d[20 + e] = o[1][e];
        }
        for (int e = 0; e < 8; ++e) {
          d[24 + e] = __float_as_uint(v[e]);
          d[32 + e] = __float_as_uint(v2[e]);
        }
      }
    }
  };
#pragma unroll
  for (int it = 0; it < NIT; ++it) c1_check(0, tid + 512 * it);       // own item
  c1_check(1, (tid + 192) % (NIT * 512));                           // another wave's item
#endif

  // the wave's row tiles go in pairs (mt, mt + 2) with their two MFMA chains interleaved: each
  // chain keeps its own k order (same sums as one tile at a time), but the pipeline now has two
  // independent accumulators to alternate between instead of stalling on one
  const u32x4* const c1u = reinterpret_cast<const u32x4*>(c1);
  auto a_unit = [&](int mt) { return mt < NT ? c1_row_unit(rows[16 * mt + c16] & 0x7fff, h) : h; };
  // bm: each board's max feature (>= 0 after the ReLU) over this lane's stores, for the A split
  float bm[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) bm[b] = 0.f;
  auto store_tile = [&](int mt, const f32x4v& acc) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = rows[16 * mt + h * 4 + r];
      const int b = (e & 0x7fff) / P, p = (e & 0x7fff) - P * ((e & 0x7fff) / P);
      if (!(e & 0x8000) && b < nb) {
        const float v = acc[r] * (c1inv[b] * iw) + bias;
        const float o = v > 0.f ? v : 0.f;
        if constexpr (STAGE) {
          ob[b * 3136 + co * P + p] = o;
#pragma unroll
          for (int q = 0; q < NB; ++q)
            if (q == b) bm[q] = fmaxf(bm[q], o);
        } else {
          feat[(size_t)(b0 + b) * 3136 + co * P + p] = o;
        }
      }
    }
  };
  for (int mt = mh; mt < NT; mt += 4) {
    const int u0 = a_unit(mt), u1 = a_unit(mt + 2);
    f32x4v acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int off = c1_tap_units(tap);
      const u32x4 ah0 = c1u[u0 + off], al0 = c1u[u0 + off + 4];
      const u32x4 ah1 = c1u[u1 + off], al1 = c1u[u1 + off + 4];
      acc0 = conv2_step(ah0, al0, bh[tap], bl[tap], acc0);
      acc1 = conv2_step(ah1, al1, bh[tap], bl[tap], acc1);
    }
    store_tile(mt, acc0);
    if (mt + 2 < NT) store_tile(mt + 2, acc1);
  }
  if constexpr (STAGE) {
    // each board's max feature, one per wave (max is exact: any order gives the value
    // h3_split_rows_kernel computes from feat)
    __shared__ float wmax[NB][8];
    if (apl) {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) bm[b] = fmaxf(bm[b], __shfl_xor(bm[b], o));
        if (lane == 0) wmax[b][wave] = bm[b];
      }
    }
    __syncthreads();
#ifdef AZ_TRUNK_SELFCHECK
#pragma unroll
    for (int it = 0; it < NIT; ++it) c1_check(2, tid + 512 * it);     // the image at the end
#endif
    // feat may be null when apl is not: the caller's GEMM then reads only the planes
    f32x4v* dst = feat ? reinterpret_cast<f32x4v*>(feat + (size_t)b0 * 3136) : nullptr;
    const f32x4v* src = reinterpret_cast<const f32x4v*>(ob);
    if (!apl) {
      for (int i = tid; i < nb * 784; i += 512) dst[i] = src[i];
      return;
    }
    for (int ch = tid; ch < nb * 392; ch += 512) {     // 8-float chunks: fp32 row + two planes
      const int b = ch / 392, c = ch - b * 392;
      float mx = wmax[b][0];
#pragma unroll
      for (int w = 1; w < 8; ++w) mx = fmaxf(mx, wmax[b][w]);
      float inv;
      const float sc = h3_scale(mx, H3_TA, &inv);
      const f32x4v lo = src[2 * ch], hi = src[2 * ch + 1];
      if (dst) {
        dst[2 * ch] = lo;
        dst[2 * ch + 1] = hi;
      }
      u32x4 o[2];
      split2s(__builtin_bit_cast(f32x4, lo), __builtin_bit_cast(f32x4, hi), sc, o);
      *reinterpret_cast<u32x4*>(apl + p2_chunk(b0 + b, c, 0, 3136)) = o[0];
      *reinterpret_cast<u32x4*>(apl + p2_chunk(b0 + b, c, 1, 3136)) = o[1];
      if (c == 0) {
        asc[b0 + b] = sc;
        asc[B + b0 + b] = inv;
      }
    }
    if constexpr (HEADS) trunk_rows_heads<NB>(ob, nb, b0, *hd);   // ob is final since the barrier
  }
}

// REGW selects the registered-weights form (w2f non-null; `un` without the weight staging room)
#define AZ_TRUNK_LB(NB_, REGW_)                                                                  \
  __attribute__((amdgpu_flat_work_group_size(1, 512),                                            \
                 amdgpu_waves_per_eu(trunk_waves_per_eu<NB_, REGW_>())))
template <int NB, bool REGW = false>
__global__ AZ_TRUNK_LB(NB, REGW) void c4_trunk_kernel(const int8_t* __restrict__ boards, int B,
                                                      const float* __restrict__ w1,
                                                      const float* __restrict__ b1,
                                                      const float* __restrict__ w2,
                                                      const float* __restrict__ b2,
                                                      float* __restrict__ feat,
                                                      const float* __restrict__ w2f = nullptr) {
  __shared__ __attribute__((aligned(16))) float un[trunk_union_floats<NB, REGW>()];
  c4_trunk_tile<NB, false, REGW>(boards, B, w1, b1, w2, b2, feat, un, nullptr, nullptr, w2f);
}

// c4_trunk_kernel that also writes feat's rows as output_transform.0's pre-split A (NB <= 4)
// HEADS: also the standard heads of the rows (predict_both above the one-launch trunk + heads size)
template <int NB, bool HEADS = false, bool REGW = false>
__global__ AZ_TRUNK_LB(NB, REGW) void c4_trunk_split_a_kernel(
    const int8_t* __restrict__ boards, int B, const float* __restrict__ w1,
    const float* __restrict__ b1, const float* __restrict__ w2, const float* __restrict__ b2,
    float* __restrict__ feat, unsigned short* __restrict__ apl, float* __restrict__ asc,
    const float* __restrict__ w2f = nullptr, TrunkHeads hd = {}) {
  static_assert(NB <= 4, "the A split reads the LDS staging tile");
  __shared__ __attribute__((aligned(16))) float un[trunk_union_floats<NB, REGW>()];
  c4_trunk_tile<NB, HEADS, REGW>(boards, B, w1, b1, w2, b2, feat, un, apl, asc, w2f, &hd);
}

// Generic 3x3 conv + ReLU, one thread per output (TicTacToe trunks: tiny, latency-bound).
template <bool IN_I8>
__global__ __launch_bounds__(256) void conv3x3_relu_kernel(const void* __restrict__ in_, int B,
                                                          int Cin, int H, int W,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ b, int Cout,
                                                          int pad, float* __restrict__ out) {
  const int Ho = H + 2 * pad - 2, Wo = W + 2 * pad - 2;
  const long total = (long)B * Cout * Ho * Wo;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int xo = idx % Wo, yo = (idx / Wo) % Ho, co = (idx / ((long)Wo * Ho)) % Cout;
    const long bi = idx / ((long)Wo * Ho * Cout);
    float s = 0.f;
    for (int ci = 0; ci < Cin; ++ci) {
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int yi = yo + kh - pad;
        if (yi < 0 || yi >= H) continue;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int xi = xo + kw - pad;
          if (xi < 0 || xi >= W) continue;
          const long ii = ((bi * Cin + ci) * H + yi) * W + xi;
          const float iv = IN_I8 ? (float)static_cast<const int8_t*>(in_)[ii]
                                 : static_cast<const float*>(in_)[ii];
          s = fmaf(w[((co * Cin + ci) * 3 + kh) * 3 + kw], iv, s);
        }
      }
    }
    s += b[co];
    out[idx] = s > 0.f ? s : 0.f;
  }
}

// Heads in two deterministic passes (no weight re-reads per row):
//  1. heads_partial_kernel: block (chunk c of 256 K-columns, group of rows).  Each thread owns
//     one float4 column slice of the chunk and keeps the A+1 weight slices for it in VGPRs;
//     every wave sweeps rows, reduces its 64 lanes and writes part[c][row][0..A].
//  2. heads_finalize_kernel: sum the chunks in order, add biases, log_softmax / exp / tanh.
constexpr int HEADS_ROWS = 16;       // rows per block (4 per wave)

template <int AMAX>
__global__ __launch_bounds__(256) void heads_partial_kernel(
    const float* __restrict__ hp, int ldhp, const float* __restrict__ hv, int ldhv, int B, int K,
    const float* __restrict__ wp, int A, const float* __restrict__ wv, float* __restrict__ part) {
  const int c = blockIdx.x;                 // K chunk
  const int r0 = blockIdx.y * HEADS_ROWS;   // row group
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int k = c * HEADS_KC + lane * 4;
  const bool kin = k < K;
  const int kc = kin ? k : 0;
  // every load is unconditional (addresses clamped into valid memory) and issued before any
  // value is masked: a select or branch next to a load makes hipcc drain vmcnt there, which
  // serialised the weight / row round trips of this latency-bound kernel (hv == hp, as for
  // Connect4, just re-reads the same lines from cache)
  constexpr int RPW = HEADS_ROWS / 4;
  f32x4 xs[RPW], ys[RPW];
  if (hv == hp && ldhv == ldhp) {           // Connect4: both heads read the same rows (uniform)
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int row = min(r0 + wave + 4 * i, B - 1);
      xs[i] = *reinterpret_cast<const f32x4*>(hp + (size_t)row * ldhp + kc);
      ys[i] = xs[i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int row = min(r0 + wave + 4 * i, B - 1);
      xs[i] = *reinterpret_cast<const f32x4*>(hp + (size_t)row * ldhp + kc);
      ys[i] = *reinterpret_cast<const f32x4*>(hv + (size_t)row * ldhv + kc);
    }
  }
  f32x4 w[AMAX + 1];
#pragma unroll
  for (int a = 0; a < AMAX; ++a)
    w[a] = *reinterpret_cast<const f32x4*>(wp + (size_t)min(a, A - 1) * K + kc);
  w[AMAX] = *reinterpret_cast<const f32x4*>(wv + kc);
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int a = 0; a < AMAX; ++a) w[a] = (a < A && kin) ? w[a] : z;
  w[AMAX] = kin ? w[AMAX] : z;
  constexpr int LOGV = AMAX == 8 ? 3 : (AMAX == 16 ? 4 : 5);
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int row = r0 + wave + 4 * i;
    if (row >= B) break;
    const f32x4 x = kin ? xs[i] : z, y = kin ? ys[i] : z;
    float* out = part + ((size_t)c * B + row) * (A + 1);
    float pv[AMAX];
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
      pv[a] = fmaf(x[3], w[a][3], fmaf(x[2], w[a][2], fmaf(x[1], w[a][1], x[0] * w[a][0])));
    const float ps = wave_multi_sum<AMAX>(pv);        // policy logit (lane >> (6-LOGV))
    const float vs = wave_sum_x(
        fmaf(y[3], w[AMAX][3], fmaf(y[2], w[AMAX][2], fmaf(y[1], w[AMAX][1], y[0] * w[AMAX][0]))));
    const int a = lane >> (6 - LOGV);
    if ((lane & ((1 << (6 - LOGV)) - 1)) == 0 && a < A) out[a] = ps;
    if (lane == 0) out[A] = vs;
  }
}

// output_transform's second GEMM (gnn_utils.py:115) left as S split-K slabs, reduced here and
// fed straight into the heads' first pass (Connect4GNN.py:48-57): block (chunk c of 256
// columns, 16 rows) as heads_partial_kernel; each lane sums its float4 of the S slabs in slab
// order and adds the bias -- the arithmetic of splitk_reduce_kernel -- stores y, and forms the
// same per-chunk dot products, so y, logp, pi and v are bit-identical to the unfused path while
// y is never re-read from HBM.
// ROWS rows per block (ROWS / 4 per wave): fewer rows per block = more blocks in flight for the
// same bytes (the per-(chunk,row) arithmetic, hence the result, does not depend on ROWS).
template <int AMAX, int S, int ROWS = HEADS_ROWS>
__global__ __launch_bounds__(256) void splitk_heads_partial_kernel(
    const float* __restrict__ slab, int B, int K, const float* __restrict__ bias,
    float* __restrict__ y, const float* __restrict__ wp, int A, const float* __restrict__ wv,
    float* __restrict__ part) {
  const int c = blockIdx.x;
  const int r0 = blockIdx.y * ROWS;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int k = c * HEADS_KC + lane * 4;
  const bool kin = k < K;
  const int kc = kin ? k : 0;
  const size_t plane = (size_t)B * K;
  constexpr int RPW = ROWS / 4;
  // all loads unconditional (clamped addresses) and issued before any masking, as in
  // heads_partial_kernel: slabs (S x RPW float4 per lane), then weights and bias
  f32x4 sv[RPW][S];
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const size_t off = (size_t)min(r0 + wave + 4 * i, B - 1) * K + kc;
#pragma unroll
    for (int q = 0; q < S; ++q) sv[i][q] = *reinterpret_cast<const f32x4*>(slab + q * plane + off);
  }
  f32x4 w[AMAX + 1];
#pragma unroll
  for (int a = 0; a < AMAX; ++a)
    w[a] = *reinterpret_cast<const f32x4*>(wp + (size_t)min(a, A - 1) * K + kc);
  w[AMAX] = *reinterpret_cast<const f32x4*>(wv + kc);
  const f32x4 bb = *reinterpret_cast<const f32x4*>(bias + kc);
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int a = 0; a < AMAX; ++a) w[a] = (a < A && kin) ? w[a] : z;
  w[AMAX] = kin ? w[AMAX] : z;
  constexpr int LOGV = AMAX == 8 ? 3 : (AMAX == 16 ? 4 : 5);
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int row = r0 + wave + 4 * i;
    if (row >= B) break;
    f32x4 x;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < S; ++q) t += sv[i][q][e];
      x[e] = kin ? t + bb[e] : 0.f;
    }
    if (kin) *reinterpret_cast<f32x4*>(y + (size_t)row * K + k) = x;
    float* out = part + ((size_t)c * B + row) * (A + 1);
    float pv[AMAX];
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
      pv[a] = fmaf(x[3], w[a][3], fmaf(x[2], w[a][2], fmaf(x[1], w[a][1], x[0] * w[a][0])));
    const float ps = wave_multi_sum<AMAX>(pv);
    const float vs = wave_sum_x(
        fmaf(x[3], w[AMAX][3], fmaf(x[2], w[AMAX][2], fmaf(x[1], w[AMAX][1], x[0] * w[AMAX][0]))));
    const int a = lane >> (6 - LOGV);
    if ((lane & ((1 << (6 - LOGV)) - 1)) == 0 && a < A) out[a] = ps;
    if (lane == 0) out[A] = vs;
  }
}

// 16 rows x 16 lanes per block: lane (row, a) sums value a's chunk partials in chunk order (the
// same order as a serial loop, so the result does not depend on the launch shape), then one
// thread per row applies log_softmax / exp / tanh.
constexpr int FIN_ROWS = 16;

template <int AMAX>
__global__ __launch_bounds__(256) void heads_finalize_kernel(const float* __restrict__ part,
                                                            int nchunks, int B, int A,
                                                            const float* __restrict__ bp,
                                                            const float* __restrict__ bv,
                                                            float* __restrict__ logp,
                                                            float* __restrict__ pi,
                                                            float* __restrict__ v) {
  __shared__ float sm[FIN_ROWS][AMAX + 1];
  const int r = threadIdx.x >> 4, cl = threadIdx.x & 15;
  const int row = blockIdx.x * FIN_ROWS + r;
  const int W = A + 1;
  if (row < B)
    for (int a = cl; a < W; a += 16) {
      // chunk partials summed in chunk order; the first 16 loads are issued together
      float vals[16];
#pragma unroll
      for (int c = 0; c < 16; ++c)
        vals[c] = c < nchunks ? part[((size_t)c * B + row) * W + a] : 0.f;
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c)
        if (c < nchunks) s += vals[c];
      for (int c = 16; c < nchunks; ++c) s += part[((size_t)c * B + row) * W + a];
      sm[r][a] = s;
    }
  __syncthreads();
  if (cl != 0 || row >= B) return;
  float l[AMAX];
  float mx = -INFINITY;
#pragma unroll
  for (int a = 0; a < AMAX; ++a)
    if (a < A) {
      l[a] = sm[r][a] + bp[a];
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
  v[row] = tanhf(sm[r][A] + bv[0]);
}

// Small batches (B <= HEADS_ROWS_MAXB, the batch-1 MCTS leaf): both passes in ONE launch, one
// 512-thread block per row.  Wave w forms the chunk partials of chunks w, w+8, ... with exactly
// heads_partial_kernel's arithmetic (two chunks' loads issued together), parks them in LDS, and
// the finalize arithmetic of heads_finalize_kernel follows in the same block -- so logp, pi and v
// are bit-identical to the two-launch path, minus one launch and the partials' HBM round trip.
constexpr int HEADS_ROWS_MAXB = 32;

template <int AMAX>
__global__ __launch_bounds__(512) void heads_rows_kernel(
    const float* __restrict__ hp, int ldhp, const float* __restrict__ hv, int ldhv, int K,
    const float* __restrict__ wp, int A, const float* __restrict__ wv,
    const float* __restrict__ bp, const float* __restrict__ bv, float* __restrict__ logp,
    float* __restrict__ pi, float* __restrict__ v) {
  __shared__ float part[HEADS_ROWS_MAXC * (AMAX + 1)];
  __shared__ float sm[AMAX + 1];
  const int row = blockIdx.x;
  heads_row_block<AMAX, 8>(hp + (size_t)row * ldhp, hv + (size_t)row * ldhv, K, wp, A, wv, bp, bv,
                        row, logp, pi, v, part, sm);
}

// output_transform.2's split-K slabs reduced and both head passes in ONE launch, one 512-thread
// block per row: the row x = sum of the S slabs (in slab order, from 0.f) + bias -- the arithmetic
// of splitk_heads_partial_kernel -- is staged in LDS (and stored as y), then heads_row_block forms
// the chunk partials and the finalize as heads_rows_kernel does.  Bit-identical to
// splitk_heads_partial_kernel + heads_finalize_kernel, minus that launch and the partials' round
// trip.  K <= SPLITK_ROWS_MAXK.
constexpr int SPLITK_ROWS_MAXK = 4096;

template <int AMAX, int S>
__global__ __launch_bounds__(512) void splitk_heads_rows_kernel(
    const float* __restrict__ slab, int B, int K, const float* __restrict__ bias,
    float* __restrict__ y, const float* __restrict__ wp, int A, const float* __restrict__ wv,
    const float* __restrict__ bp, const float* __restrict__ bv, float* __restrict__ logp,
    float* __restrict__ pi, float* __restrict__ v) {
  __shared__ __attribute__((aligned(16))) float xr[SPLITK_ROWS_MAXK];
  __shared__ float part[HEADS_ROWS_MAXC * (AMAX + 1)];
  __shared__ float sm[AMAX + 1];
  const int row = blockIdx.x;
  const size_t plane = (size_t)B * K;
  const float* src = slab + (size_t)row * K;
  const int K4 = K / 4;
  constexpr int IT = SPLITK_ROWS_MAXK / 4 / 512;
  f32x4 sv[IT][S];
#pragma unroll
  for (int it = 0; it < IT; ++it) {                  // every slab load issued before the adds
    const int k4 = min(it * 512 + (int)threadIdx.x, K4 - 1);
#pragma unroll
    for (int q = 0; q < S; ++q)
      sv[it][q] = *reinterpret_cast<const f32x4*>(src + q * plane + (size_t)k4 * 4);
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int k4 = it * 512 + (int)threadIdx.x;
    if (k4 >= K4) break;
    const f32x4 bb = *reinterpret_cast<const f32x4*>(bias + (size_t)k4 * 4);
    f32x4 x;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < S; ++q) t += sv[it][q][e];
      x[e] = t + bb[e];
    }
    *reinterpret_cast<f32x4*>(xr + k4 * 4) = x;
    if (y) *reinterpret_cast<f32x4*>(y + (size_t)row * K + k4 * 4) = x;
  }
  __syncthreads();
  heads_row_block<AMAX, 8>(xr, xr, K, wp, A, wv, bp, bv, row, logp, pi, v, part, sm);
}

// The same in one launch with R rows per block and one wave per 256-column chunk (blockDim =
// 64 * nchunks <= 1024): wave c loads its chunk's head weights ONCE into registers and reuses
// them for the block's R rows (the one-row-per-block kernel re-reads 113 KB of weights per row);
// every slab load of the R rows is issued before the first add.  Per (row, chunk) arithmetic and
// chunk-order finalize exactly as splitk_heads_partial_kernel + heads_finalize_kernel.
// Body of the R-rows-per-block heads kernels: wave c owns chunk c (blockDim = 64 * nchunks),
// keeps that chunk's head weights in registers for the block's R rows, and gets the rows' x / y
// float4s from load(i, kc, x, y) (all of them issued before the first FMA); then the chunk-order
// finalize for the R rows.
template <int AMAX, int R, typename Load>
__device__ __forceinline__ void heads_rowsw_body(int B, int K, const float* __restrict__ wp,
                                                 int A, const float* __restrict__ wv,
                                                 const float* __restrict__ bp,
                                                 const float* __restrict__ bv,
                                                 float* __restrict__ logp, float* __restrict__ pi,
                                                 float* __restrict__ v, Load load) {
  constexpr int PW = AMAX + 1;
  __shared__ float part[R][16][PW];
  __shared__ float sm[R][PW];
  const int lane = threadIdx.x & 63, c = threadIdx.x >> 6;
  const int nchunks = blockDim.x >> 6;
  const int r0 = blockIdx.x * R;
  const int k = c * HEADS_KC + lane * 4;
  const bool kin = k < K;
  const int kc = kin ? k : 0;
  f32x4 xs[R], ys[R];
  load(r0, kc, kin, k, xs, ys);
  f32x4 w[AMAX + 1];
#pragma unroll
  for (int a = 0; a < AMAX; ++a)
    w[a] = *reinterpret_cast<const f32x4*>(wp + (size_t)min(a, A - 1) * K + kc);
  w[AMAX] = *reinterpret_cast<const f32x4*>(wv + kc);
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int a = 0; a < AMAX; ++a) w[a] = (a < A && kin) ? w[a] : z;
  w[AMAX] = kin ? w[AMAX] : z;
  constexpr int LOGV = AMAX == 8 ? 3 : (AMAX == 16 ? 4 : 5);
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int row = r0 + i;
    if (row >= B) break;
    const f32x4 x = kin ? xs[i] : z, y = kin ? ys[i] : z;
    float pv[AMAX];
#pragma unroll
    for (int a = 0; a < AMAX; ++a)
      pv[a] = fmaf(x[3], w[a][3], fmaf(x[2], w[a][2], fmaf(x[1], w[a][1], x[0] * w[a][0])));
    const float ps = wave_multi_sum<AMAX>(pv);
    const float vs = wave_sum_x(
        fmaf(y[3], w[AMAX][3], fmaf(y[2], w[AMAX][2], fmaf(y[1], w[AMAX][1], y[0] * w[AMAX][0]))));
    const int a = lane >> (6 - LOGV);
    if ((lane & ((1 << (6 - LOGV)) - 1)) == 0 && a < A) part[i][c][a] = ps;
    if (lane == 0) part[i][c][A] = vs;
  }
  __syncthreads();
  const int W = A + 1;
  if (threadIdx.x < R * PW) {
    const int i = threadIdx.x / PW, a = threadIdx.x % PW;
    if (a < W) {
      float s = 0.f;
      for (int cc = 0; cc < nchunks; ++cc) s += part[i][cc][a];
      sm[i][a] = s;
    }
  }
  __syncthreads();
  if (threadIdx.x < R) {
    const int i = threadIdx.x, row = r0 + i;
    if (row < B) {
      float l[AMAX];
      float mx = -INFINITY;
#pragma unroll
      for (int a = 0; a < AMAX; ++a)
        if (a < A) {
          l[a] = sm[i][a] + bp[a];
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
      v[row] = tanhf(sm[i][A] + bv[0]);
    }
  }
}

template <int AMAX, int S, int R>
__global__ __launch_bounds__(1024) void splitk_heads_rowsw_kernel(
    const float* __restrict__ slab, int B, int K, const float* __restrict__ bias,
    float* __restrict__ y, const float* __restrict__ wp, int A, const float* __restrict__ wv,
    const float* __restrict__ bp, const float* __restrict__ bv, float* __restrict__ logp,
    float* __restrict__ pi, float* __restrict__ v) {
  const size_t plane = (size_t)B * K;
  heads_rowsw_body<AMAX, R>(B, K, wp, A, wv, bp, bv, logp, pi, v,
                            [&](int r0, int kc, bool kin, int k, f32x4 (&xs)[R], f32x4 (&ys)[R]) {
    f32x4 sv[R][S];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const size_t off = (size_t)min(r0 + i, B - 1) * K + kc;
#pragma unroll
      for (int q = 0; q < S; ++q) sv[i][q] = *reinterpret_cast<const f32x4*>(slab + q * plane + off);
    }
    const f32x4 bb = *reinterpret_cast<const f32x4*>(bias + kc);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      f32x4 x;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < S; ++q) t += sv[i][q][e];
        x[e] = kin ? t + bb[e] : 0.f;
      }
      if (kin && r0 + i < B) *reinterpret_cast<f32x4*>(y + (size_t)(r0 + i) * K + k) = x;
      xs[i] = x;
      ys[i] = x;
    }
  });
}

// Plain heads (x = hp rows, y = hv rows) with the same body: az_heads_fwd for B > 32, A <= 8.
template <int AMAX, int R>
__global__ __launch_bounds__(1024) void heads_rowsw_kernel(
    const float* __restrict__ hp, int ldhp, const float* __restrict__ hv, int ldhv, int B, int K,
    const float* __restrict__ wp, int A, const float* __restrict__ wv,
    const float* __restrict__ bp, const float* __restrict__ bv, float* __restrict__ logp,
    float* __restrict__ pi, float* __restrict__ v) {
  heads_rowsw_body<AMAX, R>(B, K, wp, A, wv, bp, bv, logp, pi, v,
                            [&](int r0, int kc, bool, int, f32x4 (&xs)[R], f32x4 (&ys)[R]) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int row = min(r0 + i, B - 1);
      xs[i] = *reinterpret_cast<const f32x4*>(hp + (size_t)row * ldhp + kc);
      ys[i] = *reinterpret_cast<const f32x4*>(hv + (size_t)row * ldhv + kc);
    }
  });
}

__global__ __launch_bounds__(256) void c4_trunk_split_kernel(
    const int8_t* __restrict__ boards, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2, float* __restrict__ feat) {
  __shared__ TrunkSplitSmem sm;
  c4_trunk_split_block(boards, w1, b1, w2, b2, feat, blockIdx.x, blockIdx.y, sm);
}

// Connect4 trunk + policy/value heads in ONE launch for small batches (the batch-1 MCTS leaf):
// c4_trunk_kernel's body, then each of the block's boards runs heads_row_block on its feature
// row straight from the LDS staging tile -- same values and arithmetic as az_c4_trunk_fwd +
// az_heads_fwd, so every output is bit-identical to that pair.
template <int NB>
__global__ __launch_bounds__(512) void c4_trunk_heads_kernel(
    const int8_t* __restrict__ boards, int B, const float* __restrict__ w1,
    const float* __restrict__ b1, const float* __restrict__ w2, const float* __restrict__ b2,
    float* __restrict__ feat, const float* __restrict__ wp, const float* __restrict__ bp, int A,
    const float* __restrict__ wv, const float* __restrict__ bv, float* __restrict__ logp,
    float* __restrict__ pi, float* __restrict__ v) {
  __shared__ __attribute__((aligned(16))) float ob[trunk_union_floats<NB, false>()];
  __shared__ float part[HEADS_ROWS_MAXC * 9];
  __shared__ float sm[9];
  c4_trunk_tile<NB>(boards, B, w1, b1, w2, b2, feat, ob);
  const int b0 = blockIdx.x * NB, nb = min(NB, B - b0);
  for (int b = 0; b < nb; ++b)
    heads_row_block<8, 8>(ob + b * 3136, ob + b * 3136, 3136, wp, A, wv, bp, bv, b0 + b, logp, pi, v,
                       part, sm);
}

}  // namespace az

using namespace az;

namespace az {
const float* conv2_frags(const float* w2, hipStream_t s);   // az_gemm.hip

// The Connect4 trunk launch (az_c4_trunk_fwd); apl / asc non-null: when the chosen NB stages its
// output in LDS (NB <= 4: B <= 1,024 on 256 CUs) the rows also leave as output_transform.0's
// pre-split A (c4_trunk_split_a_kernel) and *split is set; otherwise *split stays false.
static int c4_trunk_launch(const int8_t* boards, int B, const float* conv1_w,
                           const float* conv1_b, const float* conv2_w, const float* conv2_b,
                           float* feat, unsigned short* apl, float* asc, bool* split,
                           hipStream_t s, const TrunkHeads* heads = nullptr,
                           bool* heads_done = nullptr, bool feat_optional = false) {
  static const char* env = tuning_env("AZ_TRUNK_NB");   // tuning experiments only
  // boards per block from a fitted time model (below; every NB is bit-identical); when the caller
  // wants output_transform.0's A pre-split (apl), NB > 4 pays the separate split pass (~3.8 ns
  // per board).  Registered weights: B = 512 -> 2 (12.2 us), 1,024 -> 2, 1,576 -> 2 (28.7 us;
  // 33.2 at one block per CU in round 5), 3,150 -> 3 (44.3 us; 62.7), 4,096 -> 3 (51.7 us; 68.2)
  static int cus = 0;
  if (cus <= 0) {
    int dev = 0, n = 0;
    cus = (hipGetDevice(&dev) == hipSuccess &&
           hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
           n > 0) ? n : 256;
  }
  // conv2's weights in fragment order when they are registered (cached per weight generation):
  // the REGW kernels, whose smaller LDS puts two blocks on a CU for NB <= 3
  static const bool no_frag = tuning_env("AZ_TRUNK_NO_W2F") != nullptr;   // A/B experiments
  const float* w2f = B > 8 && !no_frag ? conv2_frags(conv2_w, s) : nullptr;
  const bool regw = w2f != nullptr;
  int nbk = 0;
  if (B > 8) {
    // t = a(NB) + b(NB) x k, k = ceil(blocks / CUs) blocks per CU.  Registered weights (REGW,
    // two blocks per CU for NB <= 3): refitted to profiles/r06/trunk_nb_sweep.txt; unregistered
    // (one block per CU, conv2 staged through LDS): the round-5 fit
    static const float ra[9] = {0.f, 4.3f, 5.f, 7.3f, 2.5f, 1.5f, 0.f, 0.f, 0.5f};
    static const float rb[9] = {0.f, 4.1f, 5.95f, 7.3f, 14.3f, 22.f, 26.f, 29.7f, 32.5f};
    static const float ua[9] = {0.f, 2.f, 2.6f, 3.7f, 3.5f, 3.f, 0.f, 0.f, 0.f};
    static const float ub[9] = {0.f, 7.6f, 10.8f, 11.8f, 15.5f, 22.f, 26.f, 30.5f, 33.f};
    const float* ta = regw ? ra : ua;
    const float* tb = regw ? rb : ub;
    float best = 0.f;
    for (int nb = 1; nb <= 8; ++nb) {
      const long k = ((long)(B + nb - 1) / nb + cus - 1) / cus;
      const float t = ta[nb] + (float)k * tb[nb] + (apl && nb > 4 ? 0.0038f * B : 0.f);
      if (nb == 1 || t < best) best = t, nbk = nb;
    }
  }
  // the split-A form without heads (the batched predict_with_gnn) above one round of 256 blocks
  // and up to two blocks per CU: one board per block measured 1.3 us faster per B = 512 step
  // than the model's NB = 2 (97.5 vs 98.8 us, tools/gpu_r06_nb_sweep.sh; the kernels alone are
  // within 0.3 us: profiles/r06/trunk_nb/)
  if (regw && apl && asc && !heads && B > cus && B <= 2 * cus) nbk = 1;
  if (env) nbk = atoi(env);
  const bool sa = apl && asc && nbk >= 1 && nbk <= 4;
  if (split) *split = sa;
  // the standard heads ride along when the rows are staged in LDS (the split-A kernel)
  const bool hk = sa && heads && heads->A >= 1 && heads->A <= 8;
  if (heads_done) *heads_done = hk;
  // feat_optional: the caller's GEMM takes the pre-split operand for certain and nothing else
  // reads feat unless the standard heads do -- the split-A kernel then skips the fp32 rows
  float* const feat_sa = feat_optional && sa && (!heads || hk) ? nullptr : feat;
#ifdef AZ_TUNING   // AZ_TRUNK_DYN_LDS=<bytes>: extra (unused) LDS per block, to limit residency
  static const char* env_dyn = tuning_env("AZ_TRUNK_DYN_LDS");
  const size_t dyn = env_dyn ? (size_t)atol(env_dyn) : 0;
#else
  constexpr size_t dyn = 0;
#endif
#define AZ_TRUNK_RW(NB_, RW_)                                                                    \
  if (hk) hipLaunchKernelGGL((c4_trunk_split_a_kernel<NB_, true, RW_>),                          \
                             dim3((B + NB_ - 1) / NB_), dim3(512), dyn, s, boards, B, conv1_w,  \
                             conv1_b, conv2_w, conv2_b, feat_sa, apl, asc, w2f, *heads);         \
  else if (sa) hipLaunchKernelGGL((c4_trunk_split_a_kernel<NB_, false, RW_>),                    \
                                  dim3((B + NB_ - 1) / NB_), dim3(512), dyn, s, boards, B,      \
                                  conv1_w, conv1_b, conv2_w, conv2_b, feat_sa, apl, asc, w2f,   \
                                  TrunkHeads{});                                                 \
  else hipLaunchKernelGGL((c4_trunk_kernel<NB_, RW_>), dim3((B + NB_ - 1) / NB_), dim3(512),    \
                          dyn, s, boards, B, conv1_w, conv1_b, conv2_w, conv2_b, feat, w2f);
#define AZ_TRUNK(NB_)                                                                            \
  if (regw) { AZ_TRUNK_RW(NB_, true) } else { AZ_TRUNK_RW(NB_, false) }
#define AZ_TRUNK_BIG(NB_)                                                                        \
  if (regw) hipLaunchKernelGGL((c4_trunk_kernel<NB_, true>), dim3((B + NB_ - 1) / NB_),         \
                               dim3(512), dyn, s, boards, B, conv1_w, conv1_b, conv2_w, conv2_b, \
                               feat, w2f);                                                       \
  else hipLaunchKernelGGL((c4_trunk_kernel<NB_, false>), dim3((B + NB_ - 1) / NB_), dim3(512),  \
                          dyn, s, boards, B, conv1_w, conv1_b, conv2_w, conv2_b, feat, nullptr);
  switch (nbk) {
    case 8: AZ_TRUNK_BIG(8) break;
    case 7: AZ_TRUNK_BIG(7) break;
    case 6: AZ_TRUNK_BIG(6) break;
    case 5: AZ_TRUNK_BIG(5) break;
    case 4: AZ_TRUNK(4) break;
    case 3: AZ_TRUNK(3) break;
    case 2: AZ_TRUNK(2) break;
    case 0:   // latency form: 4 blocks per board (bit-identical)
      hipLaunchKernelGGL(c4_trunk_split_kernel, dim3(B, 4), dim3(256), 0, s, boards, conv1_w,
                         conv1_b, conv2_w, conv2_b, feat);
      break;
    default: AZ_TRUNK(1)
  }
#undef AZ_TRUNK
#undef AZ_TRUNK_RW
#undef AZ_TRUNK_BIG
  return check_launch("c4_trunk_kernel");
}
}  // namespace az

#ifdef AZ_TRUNK_SELFCHECK
extern "C" int az_debug_trunk_chk(void* log) {   // residency experiment library only
  return hipMemcpyToSymbol(HIP_SYMBOL(g_trunk_chk), &log, sizeof(log)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int az_c4_trunk_fwd(const int8_t* boards, int B, const float* conv1_w,
                               const float* conv1_b, const float* conv2_w, const float* conv2_b,
                               float* feat, void* stream) {
  AZ_REQUIRE(B >= 0, AZ_EINVAL, "az_c4_trunk_fwd: B=%d", B);
  if (B == 0) return AZ_OK;
  AZ_REQUIRE(boards && conv1_w && conv1_b && conv2_w && conv2_b && feat, AZ_EINVAL,
             "az_c4_trunk_fwd: null pointer");
  return c4_trunk_launch(boards, B, conv1_w, conv1_b, conv2_w, conv2_b, feat, nullptr, nullptr,
                         nullptr, as_stream(stream));
}

extern "C" int az_conv3x3_relu_fwd(const void* in, int in_int8, int B, int Cin, int H, int W,
                                   const float* w, const float* b, int Cout, int pad, float* out,
                                   void* stream) {
  AZ_REQUIRE(B >= 0 && Cin > 0 && Cout > 0 && H >= 3 - 2 * pad && W >= 3 - 2 * pad &&
                 (pad == 0 || pad == 1),
             AZ_EINVAL, "az_conv3x3_relu_fwd: bad shape");
  if (B == 0) return AZ_OK;
  AZ_REQUIRE(in && w && b && out, AZ_EINVAL, "az_conv3x3_relu_fwd: null pointer");
  AZ_REQUIRE(!in_int8 || Cin == 1, AZ_EINVAL, "az_conv3x3_relu_fwd: int8 input needs Cin=1");
  const long total = (long)B * Cout * (H + 2 * pad - 2) * (W + 2 * pad - 2);
  const int blocks = (int)std::min<long>((total + 255) / 256, 8192);
  hipStream_t s = as_stream(stream);
  if (in_int8)
    hipLaunchKernelGGL(conv3x3_relu_kernel<true>, dim3(blocks), dim3(256), 0, s, in, B, Cin, H, W,
                       w, b, Cout, pad, out);
  else
    hipLaunchKernelGGL(conv3x3_relu_kernel<false>, dim3(blocks), dim3(256), 0, s, in, B, Cin, H,
                       W, w, b, Cout, pad, out);
  return check_launch("conv3x3_relu_kernel");
}

namespace az {
int gemv1_with_side_heads(const az_gemm_desc* d, const SideHeads* h, hipStream_t s);
int c4_leaf_fwd(const az_c4_eval* e, const int8_t* boards, int B, float* pi, float* v, float* gpi,
                float* gv, hipStream_t s);
int gemm_f32(const az_gemm_desc* d, hipStream_t s);
int gemm_f32_partial(const az_gemm_desc* d, hipStream_t s, int* splits_out, const PreSplitA* pre,
                     const HeadsEpi* he = nullptr, bool* heads_done = nullptr);
int splitk_reduce(const az_gemm_desc* d, int splits, hipStream_t s);
bool gemm_p2_certain(const az_gemm_desc* d, hipStream_t s);
int splitk_reduce_split(const az_gemm_desc* d, int splits, unsigned short* planes, float* sc,
                        hipStream_t s, bool write_c = true);
bool gemm_p2_weights(const float* w, int n, int k, int ld);
const float* conv2_frags(const float* w2, hipStream_t s);

static size_t align256(size_t b) { return (b + 255) & ~size_t(255); }

// The B x F pre-split-A region at the END of a transform_heads / c4_eval workspace: two fp16
// planes [2][B][F] and scales [2][B] (PreSplitA), written by the trunk for output_transform.0 and
// then by output_transform.0's fused reduce for output_transform.2.
struct PreRegion {
  unsigned short* planes;
  float* sc;
  size_t bytes;   // taken from the end of the workspace (0: no region)
};
static size_t pre_region_bytes(int B, int F) {
  return align256((size_t)4 * B * F) + align256((size_t)8 * B) + 256;
}
static PreRegion pre_region(void* ws, size_t ws_bytes, int B, int F, size_t reserved) {
  const size_t need = pre_region_bytes(B, F);
  if (!ws || ws_bytes < reserved + need) return {nullptr, nullptr, 0};
  char* base = static_cast<char*>(ws) + (ws_bytes - need + 255) / 256 * 256;
  return {reinterpret_cast<unsigned short*>(base),
          reinterpret_cast<float*>(base + align256((size_t)4 * B * F)), need};
}
}  // namespace az

extern "C" size_t az_heads_ws_bytes(int B, int K, int A) {
  return (size_t)((K + HEADS_KC - 1) / HEADS_KC) * (size_t)B * (size_t)(A + 1) * 4;
}

template <int AMAX>
static void launch_heads(const float* hp, int ldhp, const float* hv, int ldhv, int B, int K,
                         const float* wp, const float* bp, int A, const float* wv,
                         const float* bv, float* logp, float* pi, float* v, float* part,
                         hipStream_t s) {
  const int nchunks = (K + HEADS_KC - 1) / HEADS_KC;
  static const bool two_pass = tuning_env("AZ_HEADS_TWOPASS") != nullptr;   // A/B experiments
  if (B <= HEADS_ROWS_MAXB && nchunks <= HEADS_ROWS_MAXC && !two_pass) {
    hipLaunchKernelGGL(heads_rows_kernel<AMAX>, dim3(B), dim3(512), 0, s, hp, ldhp, hv, ldhv, K,
                       wp, A, wv, bp, bv, logp, pi, v);
    return;
  }
  static const char* env_r = tuning_env("AZ_HEADS_R");   // tuning sweeps (tools/heads_sweep.py)
  // R rows per block, one wave per chunk holding that chunk's head weights for all R rows: a
  // block re-reads the 113 KB of head weights, so R grows with B while the grid still covers
  // the CUs (2 at B = 512: 256 blocks; 4 from the self-play rounds' B ~ 1,600: ~400)
  int R = B > 768 ? 4 : 2;      // r03m: B = 1,576 21.4 vs 24.2 us, B = 4,096 41.6 vs 47.8
  if (env_r) R = atoi(env_r);
  if (AMAX == 8 && nchunks <= 16 && !two_pass && B <= 8192 && (R == 2 || R == 4 || R == 8)) {
    // one launch (splitk_heads_rowsw_kernel's body); above B = 8192 the two-pass form's
    // 16-row weight reuse wins (B = 65,536: rowsw at R = 2 took 735 us vs ~0.3 ms)
    const dim3 blk(64 * nchunks);
    if (R == 2)
      hipLaunchKernelGGL((heads_rowsw_kernel<8, 2>), dim3((B + 1) / 2), blk, 0, s, hp, ldhp, hv,
                         ldhv, B, K, wp, A, wv, bp, bv, logp, pi, v);
    else if (R == 4)
      hipLaunchKernelGGL((heads_rowsw_kernel<8, 4>), dim3((B + 3) / 4), blk, 0, s, hp, ldhp, hv,
                         ldhv, B, K, wp, A, wv, bp, bv, logp, pi, v);
    else
      hipLaunchKernelGGL((heads_rowsw_kernel<8, 8>), dim3((B + 7) / 8), blk, 0, s, hp, ldhp, hv,
                         ldhv, B, K, wp, A, wv, bp, bv, logp, pi, v);
    return;
  }
  dim3 g(nchunks, (B + HEADS_ROWS - 1) / HEADS_ROWS);
  hipLaunchKernelGGL(heads_partial_kernel<AMAX>, g, dim3(256), 0, s, hp, ldhp, hv, ldhv, B, K, wp,
                     A, wv, part);
  hipLaunchKernelGGL(heads_finalize_kernel<AMAX>, dim3((B + FIN_ROWS - 1) / FIN_ROWS), dim3(256),
                     0, s, part, nchunks, B, A, bp, bv, logp, pi, v);
}

extern "C" int az_heads_fwd(const float* hp, int ldhp, const float* hv, int ldhv, int B, int K,
                            const float* wp, const float* bp, int A, const float* wv,
                            const float* bv, float* logp, float* pi, float* v, void* ws,
                            size_t ws_bytes, void* stream) {
  AZ_REQUIRE(B >= 0 && K > 0 && K % 4 == 0 && A > 0 && A <= 32, AZ_EINVAL,
             "az_heads_fwd: bad shape B=%d K=%d A=%d", B, K, A);
  if (B == 0) return AZ_OK;
  AZ_REQUIRE(hp && hv && wp && bp && wv && bv && logp && v && ws, AZ_EINVAL, "az_heads_fwd: null");
  AZ_REQUIRE(ws_bytes >= az_heads_ws_bytes(B, K, A), AZ_EINVAL, "az_heads_fwd: workspace too small");
  AZ_REQUIRE(aligned16(hp) && aligned16(hv) && aligned16(wp) && aligned16(wv) && ldhp % 4 == 0 &&
                 ldhv % 4 == 0,
             AZ_EINVAL, "az_heads_fwd: operands need 16B alignment");
  hipStream_t s = as_stream(stream);
  float* part = static_cast<float*>(ws);
  if (A <= 8)
    launch_heads<8>(hp, ldhp, hv, ldhv, B, K, wp, bp, A, wv, bv, logp, pi, v, part, s);
  else if (A <= 16)
    launch_heads<16>(hp, ldhp, hv, ldhv, B, K, wp, bp, A, wv, bv, logp, pi, v, part, s);
  else
    launch_heads<32>(hp, ldhp, hv, ldhv, B, K, wp, bp, A, wv, bv, logp, pi, v, part, s);
  return check_launch("heads_kernels");
}

extern "C" int az_c4_trunk_heads_fwd(const int8_t* boards, int B, const float* conv1_w,
                                     const float* conv1_b, const float* conv2_w,
                                     const float* conv2_b, const float* wp, const float* bp, int A,
                                     const float* wv, const float* bv, float* feat, float* logp,
                                     float* pi, float* v, void* ws, size_t ws_bytes,
                                     void* stream) {
  AZ_REQUIRE(B >= 0 && A > 0 && A <= 32, AZ_EINVAL, "az_c4_trunk_heads_fwd: B=%d A=%d", B, A);
  if (B == 0) return AZ_OK;
  AZ_REQUIRE(boards && conv1_w && conv1_b && conv2_w && conv2_b && wp && bp && wv && bv && feat &&
                 logp && v,
             AZ_EINVAL, "az_c4_trunk_heads_fwd: null pointer");
  AZ_REQUIRE(aligned16(feat) && aligned16(wp) && aligned16(wv), AZ_EINVAL,
             "az_c4_trunk_heads_fwd: operands need 16B alignment");
  static const bool split = tuning_env("AZ_TRUNK_HEADS_SPLIT") != nullptr;   // A/B experiments
  static const char* fused_nb = tuning_env("AZ_TRUNK_HEADS_FUSED");        // A/B: any B, NB 1/2
  if (fused_nb && A <= 8) {
    if (atoi(fused_nb) == 2)
      hipLaunchKernelGGL(c4_trunk_heads_kernel<2>, dim3((B + 1) / 2), dim3(512), 0,
                         as_stream(stream), boards, B, conv1_w, conv1_b, conv2_w, conv2_b, feat,
                         wp, bp, A, wv, bv, logp, pi, v);
    else
      hipLaunchKernelGGL(c4_trunk_heads_kernel<1>, dim3(B), dim3(512), 0, as_stream(stream),
                         boards, B, conv1_w, conv1_b, conv2_w, conv2_b, feat, wp, bp, A, wv, bv,
                         logp, pi, v);
    return check_launch("c4_trunk_heads_kernel");
  }
  // one launch up to B = 320 (profiles/r03t_trunk_heads_probe.jsonl, bit-identical: B = 64
  // 17.2 vs 19.9 us for trunk + heads, 256 17.1 vs 23.8; at 512 the two launches win, 25.5 vs
  // 28.9): the self-play lanes' shrinking batches as their games finish
  constexpr int TRUNK_HEADS_MAXB = 320;
  if (B <= TRUNK_HEADS_MAXB && A <= 8 && !split) {
    hipLaunchKernelGGL(c4_trunk_heads_kernel<1>, dim3(B), dim3(512), 0, as_stream(stream), boards,
                       B, conv1_w, conv1_b, conv2_w, conv2_b, feat, wp, bp, A, wv, bv, logp, pi,
                       v);
    return check_launch("c4_trunk_heads_kernel");
  }
  int rc = az_c4_trunk_fwd(boards, B, conv1_w, conv1_b, conv2_w, conv2_b, feat, stream);
  if (rc) return rc;
  return az_heads_fwd(feat, 3136, feat, 3136, B, 3136, wp, bp, A, wv, bv, logp, pi, v, ws,
                      ws_bytes, stream);
}


extern "C" size_t az_transform_heads_ws_bytes(int B, int F, int A) {
  // the heads' chunk partials, then room for 8 split-K slabs of the [B][F] GEMM outputs, the
  // GEMM's A operand as two fp16 planes (the fp16 form on pre-split planes, az_gemm.hip) and
  // A's row scales, and the pre-split-A region (pre_region) at the end
  // (+ [B][F] scratch for y when the caller passes y = NULL and the GEMM's shape has no heads
  // epilogue)
  return align256(az_heads_ws_bytes(B, F, A)) + (size_t)8 * B * F * 4 +
         align256((size_t)4 * B * F) + align256((size_t)8 * B) + 256 +
         az::pre_region_bytes(B, F) + align256((size_t)4 * B * F);
}

template <int S>
static void launch_splitk_heads(const float* slab, int B, int K, const float* bias, float* y,
                                const float* wp, int A, const float* wv, float* part,
                                hipStream_t s) {
  // 4 rows per block (one per wave): 1,664 blocks at B = 512 instead of 416 with 16 rows, so
  // 4x the slab loads in flight: 12.1 -> 9.0 us (tools/heads_rows_probe.sh on MI355X).
  // AZ_SPLITK_HEADS_ROWS = 8 / 16 selects the other shapes for A/B runs.
  static const char* env_rows = tuning_env("AZ_SPLITK_HEADS_ROWS");
  const int rows = env_rows ? atoi(env_rows) : 4;
  if (rows == 4 || rows == 8) {
    dim3 g((K + HEADS_KC - 1) / HEADS_KC, (B + rows - 1) / rows);
    if (rows == 4)
      hipLaunchKernelGGL((splitk_heads_partial_kernel<8, S, 4>), g, dim3(256), 0, s, slab, B, K,
                         bias, y, wp, A, wv, part);
    else
      hipLaunchKernelGGL((splitk_heads_partial_kernel<8, S, 8>), g, dim3(256), 0, s, slab, B, K,
                         bias, y, wp, A, wv, part);
    return;
  }
  dim3 g((K + HEADS_KC - 1) / HEADS_KC, (B + HEADS_ROWS - 1) / HEADS_ROWS);
  hipLaunchKernelGGL((splitk_heads_partial_kernel<8, S>), g, dim3(256), 0, s, slab, B, K, bias, y,
                     wp, A, wv, part);
}

namespace az {
// az_linear_heads_fwd with x optionally already in the P2 GEMM's form (pre, may be null)
static int linear_heads_impl(const float* x, int B, int F, const float* w, const float* b,
                             const float* wp, const float* bp, int A, const float* wv,
                             const float* bv, float* y, float* logp, float* pi, float* v,
                             void* ws, size_t ws_bytes, void* stream, const PreSplitA* pre) {
  AZ_REQUIRE(B >= 0 && F > 0 && F % 4 == 0 && A > 0 && A <= 32, AZ_EINVAL,
             "az_linear_heads_fwd: bad shape B=%d F=%d A=%d", B, F, A);
  if (B == 0) return AZ_OK;
  AZ_REQUIRE(x && w && b && wp && bp && wv && bv && logp && v && ws, AZ_EINVAL,
             "az_linear_heads_fwd: null pointer");
  const size_t part_bytes = align256(az_heads_ws_bytes(B, F, A));
  AZ_REQUIRE(ws_bytes >= part_bytes, AZ_EINVAL, "az_linear_heads_fwd: workspace too small");
  AZ_REQUIRE(aligned16(x) && (!y || aligned16(y)) && aligned16(wp) && aligned16(wv) &&
                 aligned16(b) && aligned16(ws),
             AZ_EINVAL, "az_linear_heads_fwd: operands need 16B alignment");
  hipStream_t s = as_stream(stream);
  // y == NULL: the caller wants only the heads.  The GEMM then hands its tiles' head dot
  // products to heads_tiles_finalize_kernel when it can (az_x3.h HeadsEpi); the other shapes
  // form y in a [B][F] scratch at the workspace's end
  const bool want_y = y != nullptr;
  if (!want_y) {
    const size_t yb = align256((size_t)4 * B * F);
    AZ_REQUIRE(ws_bytes >= part_bytes + yb + 256, AZ_EINVAL,
               "az_linear_heads_fwd: workspace too small for y = NULL");
    ws_bytes = (ws_bytes - yb) / 256 * 256;
    y = reinterpret_cast<float*>(static_cast<char*>(ws) + ws_bytes);
  }
  float* part = static_cast<float*>(ws);
  void* slabs = static_cast<char*>(ws) + part_bytes;
  int rc;
  // y = x W^T + b, its split-K reduction fused into the heads' first pass
  az_gemm_desc d = {};
  d.M = B; d.N = F; d.K = F;
  d.A = x; d.lda = F; d.a_kmajor = 1;
  d.B = w; d.ldb = F; d.b_kmajor = 1; d.bias = b; d.act = AZ_ACT_NONE;
  d.C = y; d.ldc = F;
  d.ws = slabs; d.ws_bytes = ws_bytes - part_bytes;
  int S = 1;
  // the tile partials [B][P][9] (P <= ceil(F / 128) * 8) at the start of the slab region
  const size_t tiles_bytes = (size_t)B * ((F + 127) / 128) * 8 * HEADS_TILE_SLOTS * 4;
  // (the stream-K form's slots: 49 column blocks x its max pieces, <= 8 for these shapes)
  const HeadsEpi he{wp, wv, A, static_cast<float*>(slabs), 0, bp, bv, logp, pi, v};
  bool heads_done = false;
  static const bool no_tiles = tuning_env("AZ_NO_HEADS_TILES") != nullptr;   // A/B experiments
  const bool try_tiles = !want_y && !no_tiles && A <= 8 && 2 * tiles_bytes <= d.ws_bytes;
  if ((rc = gemm_f32_partial(&d, s, &S, pre, try_tiles ? &he : nullptr, &heads_done))) return rc;
  if (heads_done) return AZ_OK;   // the GEMM's dispatch also ran the heads' finalize
  const float* sl = static_cast<const float*>(slabs);
  // one launch: splitk_heads_rowsw_kernel (AZ_SPLITK_HEADS_MODE = rows / chunks select the
  // one-row-per-block kernel / chunk partials + finalize for A/B runs)
  static const char* env_mode = tuning_env("AZ_SPLITK_HEADS_MODE");
  const char mode = env_mode ? env_mode[0] : 'w';   // w: rowsw, r: rows, c: chunks + finalize
  const bool rows_mode = mode != 'c' && F <= SPLITK_ROWS_MAXK &&
                         (F + HEADS_KC - 1) / HEADS_KC <= HEADS_ROWS_MAXC;
  const int nch = (F + HEADS_KC - 1) / HEADS_KC;
  // rows per block: 1 (512 blocks at B = 512, 1.2-2 us faster per call than 2 rows at B = 256 ..
  // 4,096 in the fused step: profiles/r04x/heads_rows_ab.jsonl; the same bits for any R)
  static const char* env_r = tuning_env("AZ_SPLITK_HEADS_R");   // rows per block, A/B runs
  const int R = env_r ? atoi(env_r) : 1;
  if (S > 1 && A <= 8 && S <= 8 && rows_mode && mode == 'w' && nch <= 16 &&
      (R == 1 || R == 2 || R == 4)) {
    const dim3 g((B + R - 1) / R), blk(64 * nch);
    switch (S * 8 + R) {
#define AZ_SKW(SS, RR) case SS * 8 + RR: hipLaunchKernelGGL((splitk_heads_rowsw_kernel<8, SS, RR>), g, \
                           blk, 0, s, sl, B, F, b, y, wp, A, wv, bp, bv, logp, pi, v); break;
      AZ_SKW(2, 1) AZ_SKW(3, 1) AZ_SKW(4, 1) AZ_SKW(5, 1) AZ_SKW(6, 1) AZ_SKW(7, 1) AZ_SKW(8, 1)
#ifdef AZ_TUNING   // 2 and 4 rows per block (AZ_SPLITK_HEADS_R): 2 measured equal or slower
      AZ_SKW(2, 2) AZ_SKW(3, 2) AZ_SKW(4, 2) AZ_SKW(5, 2) AZ_SKW(6, 2) AZ_SKW(7, 2) AZ_SKW(8, 2)
      AZ_SKW(2, 4) AZ_SKW(3, 4) AZ_SKW(4, 4) AZ_SKW(5, 4) AZ_SKW(6, 4) AZ_SKW(7, 4) AZ_SKW(8, 4)
#endif
#undef AZ_SKW
    }
    return check_launch("splitk_heads_rowsw_kernel");
  }
  if (S > 1 && A <= 8 && S <= 8 && rows_mode) {
    switch (S) {
#define AZ_SKR(SS) case SS: hipLaunchKernelGGL((splitk_heads_rows_kernel<8, SS>), dim3(B), dim3(512), \
                                              0, s, sl, B, F, b, y, wp, A, wv, bp, bv, logp, pi, v); break;
      AZ_SKR(2) AZ_SKR(3) AZ_SKR(4) AZ_SKR(5) AZ_SKR(6) AZ_SKR(7)
      default: AZ_SKR(8)
#undef AZ_SKR
    }
    return check_launch("splitk_heads_rows_kernel");
  }
  if (S > 1 && A <= 8 && S <= 8) {
    switch (S) {
      case 2: launch_splitk_heads<2>(sl, B, F, b, y, wp, A, wv, part, s); break;
      case 3: launch_splitk_heads<3>(sl, B, F, b, y, wp, A, wv, part, s); break;
      case 4: launch_splitk_heads<4>(sl, B, F, b, y, wp, A, wv, part, s); break;
      case 5: launch_splitk_heads<5>(sl, B, F, b, y, wp, A, wv, part, s); break;
      case 6: launch_splitk_heads<6>(sl, B, F, b, y, wp, A, wv, part, s); break;
      case 7: launch_splitk_heads<7>(sl, B, F, b, y, wp, A, wv, part, s); break;
      default: launch_splitk_heads<8>(sl, B, F, b, y, wp, A, wv, part, s); break;
    }
    if ((rc = check_launch("splitk_heads_partial_kernel"))) return rc;
    hipLaunchKernelGGL(heads_finalize_kernel<8>, dim3((B + FIN_ROWS - 1) / FIN_ROWS), dim3(256), 0,
                       s, part, (F + HEADS_KC - 1) / HEADS_KC, B, A, bp, bv, logp, pi, v);
    return check_launch("heads_finalize_kernel");
  }
  if (S > 1 && (rc = splitk_reduce(&d, S, s))) return rc;
  return az_heads_fwd(y, F, y, F, B, F, wp, bp, A, wv, bv, logp, pi, v, part, part_bytes, stream);
}

// az_transform_heads_fwd with x optionally pre-split (pre_x: the trunk wrote it into the
// workspace's pre_region).  When output_transform.0 leaves split-K slabs and output_transform.2
// takes the P2 path, the slabs' reduce also writes hidden's planes into pre_region
// (splitk_reduce_split), so neither GEMM launches a split of its own; every output is bit-identical
// to the unfused sequence (same planes, same products, same reduce arithmetic).
static int transform_heads_impl(const float* x, int B, int F, const float* w0, const float* b0,
                                const float* w2, const float* b2, const float* wp,
                                const float* bp, int A, const float* wv, const float* bv,
                                float* hidden, float* y, float* logp, float* pi, float* v,
                                void* ws, size_t ws_bytes, void* stream, const PreSplitA* pre_x,
                                bool hidden_scratch = false) {
  const size_t part_bytes = align256(az_heads_ws_bytes(B, F, A > 0 ? A : 1));
  AZ_REQUIRE(ws_bytes >= part_bytes, AZ_EINVAL, "az_transform_heads_fwd: workspace too small");
  hipStream_t s = as_stream(stream);
  static const bool no_fuse = tuning_env("AZ_NO_PRESPLIT") != nullptr;   // A/B experiments
  // the region is reserved whenever the caller's pre_x lives in it (the same address: pre_region
  // depends only on ws, ws_bytes, B, F)
  const PreRegion R = pre_x || (!no_fuse && gemm_p2_weights(w2, F, F, F))
                          ? pre_region(ws, ws_bytes, B, F, part_bytes + (size_t)B * F * 8)
                          : PreRegion{nullptr, nullptr, 0};
  AZ_REQUIRE(!pre_x || pre_x->planes == R.planes, AZ_EINVAL,
             "az_transform_heads_fwd: pre-split A outside the workspace's region");
  // hidden = relu(x W0^T + b0)   (output_transform.0 + ReLU); slabs after the heads' partials
  az_gemm_desc d = {};
  d.M = B; d.N = F; d.K = F;
  d.A = x; d.lda = F; d.a_kmajor = 1;
  d.B = w0; d.ldb = F; d.b_kmajor = 1; d.bias = b0; d.act = AZ_ACT_RELU;
  d.C = hidden; d.ldc = F;
  d.ws = static_cast<char*>(ws) + part_bytes;
  d.ws_bytes = ws_bytes - part_bytes - R.bytes;
  int S = 1, rc;
  if ((rc = gemm_f32_partial(&d, s, &S, pre_x))) return rc;
  PreSplitA pre_h{nullptr, nullptr};
  if (S > 1) {
    // hidden_scratch (az_c4_eval_fwd's e->hidden): the fp32 hidden rows are skipped when
    // output_transform.2 certainly takes the reduce's planes -- gemm_p2_certain on the
    // descriptor linear_heads_impl builds (y NULL: its scratch y at the workspace's end)
    bool write_c = true;
    if (R.planes && hidden_scratch && A > 0 && A <= 32) {
      size_t wsb = ws_bytes - R.bytes;
      const size_t part2 = align256(az_heads_ws_bytes(B, F, A));
      const size_t yb = y ? 0 : align256((size_t)4 * B * F);
      if (wsb >= part2 + yb + 256) {
        wsb = y ? wsb : (wsb - yb) / 256 * 256;
        az_gemm_desc d2 = {};
        d2.M = B; d2.N = F; d2.K = F;
        d2.A = hidden; d2.lda = F; d2.a_kmajor = 1;
        d2.B = w2; d2.ldb = F; d2.b_kmajor = 1; d2.bias = b2; d2.act = AZ_ACT_NONE;
        d2.ws = static_cast<char*>(ws) + part2;
        d2.ws_bytes = wsb - part2;
        write_c = !gemm_p2_certain(&d2, s);
      }
    }
    rc = R.planes ? splitk_reduce_split(&d, S, R.planes, R.sc, s, write_c) : 0;
    if (rc < 0) return rc;
    if (rc == 1) pre_h = {R.planes, R.sc};
    else if ((rc = splitk_reduce(&d, S, s))) return rc;
  }
  // y = hidden W2^T + b2 (output_transform.2) and the heads
  return linear_heads_impl(hidden, B, F, w2, b2, wp, bp, A, wv, bv, y, logp, pi, v, ws,
                           ws_bytes - R.bytes, stream, pre_h.planes ? &pre_h : nullptr);
}
}  // namespace az

extern "C" int az_linear_heads_fwd(const float* x, int B, int F, const float* w, const float* b,
                                   const float* wp, const float* bp, int A, const float* wv,
                                   const float* bv, float* y, float* logp, float* pi, float* v,
                                   void* ws, size_t ws_bytes, void* stream) {
  return az::linear_heads_impl(x, B, F, w, b, wp, bp, A, wv, bv, y, logp, pi, v, ws, ws_bytes,
                               stream, nullptr);
}

extern "C" int az_transform_heads_fwd(const float* x, int B, int F, const float* w0,
                                      const float* b0, const float* w2, const float* b2,
                                      const float* wp, const float* bp, int A, const float* wv,
                                      const float* bv, float* hidden, float* y, float* logp,
                                      float* pi, float* v, void* ws, size_t ws_bytes,
                                      void* stream) {
  AZ_REQUIRE(B >= 0 && F > 0 && F % 4 == 0, AZ_EINVAL,
             "az_transform_heads_fwd: bad shape B=%d F=%d", B, F);
  if (B == 0) return AZ_OK;
  AZ_REQUIRE(x && w0 && b0 && hidden && ws, AZ_EINVAL, "az_transform_heads_fwd: null pointer");
  AZ_REQUIRE(aligned16(x) && aligned16(hidden) && aligned16(ws), AZ_EINVAL,
             "az_transform_heads_fwd: operands need 16B alignment");
  return transform_heads_impl(x, B, F, w0, b0, w2, b2, wp, bp, A, wv, bv, hidden, y, logp, pi, v,
                              ws, ws_bytes, stream, nullptr);
}

extern "C" int az_c4_eval_fwd(const az_c4_eval* e, const int8_t* boards, int B, float* pi,
                              float* v, float* gpi, float* gv, void* stream) {
  AZ_REQUIRE(e && B >= 0 && B <= e->max_B, AZ_EINVAL, "az_c4_eval_fwd: B=%d max_B=%d", B,
             e ? e->max_B : 0);
  if (B == 0) return AZ_OK;
  AZ_REQUIRE(boards && e->feat, AZ_EINVAL, "az_c4_eval_fwd: null boards / feat");
  int rc;
  static const bool side = tuning_env("AZ_EVAL_NO_SIDE") == nullptr;   // A/B experiments
  if (B <= 8 && v && gv && e->sync) {        // one launch (c4_leaf_kernel) when it applies
    rc = c4_leaf_fwd(e, boards, B, pi, v, gpi, gv, as_stream(stream));
    if (rc != 0) return rc < 0 ? rc : AZ_OK;
  }
  if (B <= 8 && v && gv && side && e->ot0_w && e->hidden && e->y && e->glogp) {
    // batch 1 and small speculative batches: the trunk in its latency form (4 blocks per
    // board), the standard heads ride along with output_transform.0 (extra blocks of the same
    // launch, off the trunk -> GEMV -> GEMV -> heads chain); same kernels' arithmetic, same bits
    if ((rc = az_c4_trunk_fwd(boards, B, e->conv1_w, e->conv1_b, e->conv2_w, e->conv2_b, e->feat,
                              stream)))
      return rc;
    az_gemm_desc d = {};
    d.M = B; d.N = 3136; d.K = 3136;
    d.A = e->feat; d.lda = 3136; d.a_kmajor = 1;
    d.B = e->ot0_w; d.ldb = 3136; d.b_kmajor = 1; d.bias = e->ot0_b; d.act = AZ_ACT_RELU;
    d.C = e->hidden; d.ldc = 3136;
    const SideHeads h = {e->feat, 3136, 3136, B, e->fc_policy_w, e->fc_policy_b, e->A,
                         e->fc_value_w, e->fc_value_b, e->logp, pi, v};
    rc = gemv1_with_side_heads(&d, &h, as_stream(stream));
    if (rc < 0) return rc;
    if (rc == 1)
      return az_linear_heads_fwd(e->hidden, B, 3136, e->ot2_w, e->ot2_b, e->fc_policy_w,
                                 e->fc_policy_b, e->A, e->fc_value_w, e->fc_value_b, e->y,
                                 e->glogp, gpi, gv, e->ws, e->ws_bytes, stream);
    // shapes not covered: the general sequence below (re-runs the trunk, harmless)
  }
  // the GNN tail (predict_with_gnn batches, and predict_both above the one-launch trunk + heads
  // size): the trunk also writes feat's rows as output_transform.0's pre-split A into the
  // workspace's pre_region when that GEMM takes the P2 path (c4_trunk_launch decides by its
  // NB), so the GEMM launches no split of its own; the standard heads (predict_both) then read
  // feat as before -- the same kernels, the same bits
  constexpr int TRUNK_HEADS_ONE_LAUNCH = 320;   // az_c4_trunk_heads_fwd's one-launch limit
  PreRegion R{nullptr, nullptr, 0};
  bool split = false;
  // the fp32 scratch rows (e->feat, e->hidden) a certain pre-split hand-off never reads are not
  // written; AZ_EVAL_KEEP_FEAT (tuning build) writes them for A/B runs
  static const bool keep_feat = tuning_env("AZ_EVAL_KEEP_FEAT") != nullptr;
  static const bool no_fuse = tuning_env("AZ_NO_PRESPLIT") != nullptr;   // A/B experiments
  static const bool no_both = tuning_env("AZ_NO_PRESPLIT_BOTH") != nullptr;
  if (gv && (!v || (B > TRUNK_HEADS_ONE_LAUNCH && !no_both)) && !no_fuse && e->ot0_w &&
      aligned16(e->ws) &&
      gemm_p2_weights(e->ot0_w, 3136, 3136, 3136))
    R = pre_region(e->ws, e->ws_bytes, B, 3136,
                   align256(az_heads_ws_bytes(B, 3136, e->A)) + (size_t)B * 3136 * 8);
  if (v && !R.planes) {
    rc = az_c4_trunk_heads_fwd(boards, B, e->conv1_w, e->conv1_b, e->conv2_w, e->conv2_b,
                               e->fc_policy_w, e->fc_policy_b, e->A, e->fc_value_w, e->fc_value_b,
                               e->feat, e->logp, pi, v, e->ws, e->ws_bytes, stream);
  } else {
    // predict_both: the split-A trunk computes the standard heads from its LDS rows
    // (trunk_rows_heads: az_heads_fwd's bits), else they run after it as az_c4_trunk_heads_fwd
    // does above 320 rows
    static const bool no_th = tuning_env("AZ_NO_TRUNK_HEADS") != nullptr;   // A/B experiments
    const TrunkHeads th{e->fc_policy_w, e->fc_policy_b, e->A, e->fc_value_w, e->fc_value_b,
                        e->logp, pi, v};
    bool heads_done = false;
    const bool want_th = v && e->logp && e->fc_policy_w && e->fc_policy_b && e->fc_value_w &&
                         e->fc_value_b && !no_th && aligned16(e->fc_policy_w) &&
                         aligned16(e->fc_value_w);
    // e->feat stays unwritten when output_transform.0 certainly takes the trunk's pre-split
    // operand (gemm_p2_certain on the descriptor transform_heads_impl builds below) and the
    // standard heads, if wanted, come from the trunk's LDS rows
    bool feat_opt = false;
    if (R.planes && gv && e->ot0_w && e->ot0_b && e->hidden && (!v || want_th) && !keep_feat) {
      const size_t part_bytes = align256(az_heads_ws_bytes(B, 3136, e->A > 0 ? e->A : 1));
      az_gemm_desc d = {};
      d.M = B; d.N = 3136; d.K = 3136;
      d.A = e->feat; d.lda = 3136; d.a_kmajor = 1;
      d.B = e->ot0_w; d.ldb = 3136; d.b_kmajor = 1; d.bias = e->ot0_b; d.act = AZ_ACT_RELU;
      d.C = e->hidden; d.ldc = 3136;
      d.ws = static_cast<char*>(e->ws) + part_bytes;
      d.ws_bytes = e->ws_bytes > part_bytes + R.bytes ? e->ws_bytes - part_bytes - R.bytes : 0;
      feat_opt = gemm_p2_certain(&d, as_stream(stream));
    }
    rc = c4_trunk_launch(boards, B, e->conv1_w, e->conv1_b, e->conv2_w, e->conv2_b, e->feat,
                         R.planes, R.sc, &split, as_stream(stream), want_th ? &th : nullptr,
                         &heads_done, feat_opt);
    if (!rc && v && !heads_done)
      rc = az_heads_fwd(e->feat, 3136, e->feat, 3136, B, 3136, e->fc_policy_w, e->fc_policy_b,
                        e->A, e->fc_value_w, e->fc_value_b, e->logp, pi, v, e->ws, e->ws_bytes,
                        stream);
  }
  if (rc || !gv) return rc;
  AZ_REQUIRE(e->ot0_w && e->ot0_b && e->ot2_w && e->ot2_b && e->hidden && e->y && e->glogp,
             AZ_EINVAL, "az_c4_eval_fwd: GNN tail requested without its weights / scratch");
  AZ_REQUIRE(aligned16(e->feat) && aligned16(e->hidden) && aligned16(e->ws), AZ_EINVAL,
             "az_c4_eval_fwd: scratch needs 16B alignment");
  const PreSplitA pre{R.planes, R.sc};
  // y (the transform's output) is not an output of the evaluator: the heads come from the
  // GEMM's tiles (az_x3.h HeadsEpi) wherever its shape allows
  return transform_heads_impl(e->feat, B, 3136, e->ot0_w, e->ot0_b, e->ot2_w, e->ot2_b,
                              e->fc_policy_w, e->fc_policy_b, e->A, e->fc_value_w, e->fc_value_b,
                              e->hidden, nullptr, e->glogp, gpi, gv, e->ws, e->ws_bytes, stream,
                              split ? &pre : nullptr, !keep_feat);
}
