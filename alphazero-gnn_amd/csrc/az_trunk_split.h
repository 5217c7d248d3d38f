// The Connect4 trunk in its latency form, one (board, quarter of the output channels) per block:
// shared by az_trunk.hip (c4_trunk_split_kernel) and az_gemm.hip (the batch-1 leaf kernel,
// c4_leaf_kernel), which cannot call across translation units (-fno-gpu-rdc).
#pragma once
#include "az_common.h"

namespace az {

typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// conv2's weights in LDS: row co at stride W2S_STRIDE floats.  Stride = 2 (mod 32) makes the
// conv2 fragment reads (lane: co = 16 consecutive rows, ci = 2 values 9 floats apart per 32-lane
// half) hit 32 distinct ds_read_b32 banks.
constexpr int W2S_STRIDE = 290;
constexpr int W2S_FLOATS = 64 * W2S_STRIDE;

// conv1's output in LDS: [board][padded 9x9 position][channel], rows of C1S floats.  A lane of
// conv2's MFMA chain (row = position, lane group h = 16-lane quarter) reads the 8 channels
// 8h .. 8h+7 of one position as two ds_read_b128, which feed 8 MFMA steps (the k order of a tap
// is ci = 8h + j, j = 0..7).  C1S = 36 (32 channels + 4 pad): 16 consecutive rows of a
// quarter then start on 16 distinct 4-bank groups.
constexpr int C1S = 36;
constexpr int C1_FLOATS_PER_BOARD = 81 * C1S;

struct TrunkSplitSmem {
  __attribute__((aligned(16))) float w2s[17 * W2S_STRIDE];   // + pad row
  float bd[81 + 1];
  __attribute__((aligned(16))) float c1[C1_FLOATS_PER_BOARD];
  float w1s[32 * 9 + 32 + 1];
};

// Latency form of the trunk for a handful of boards (the arena's leaf + speculative children,
// B <= 8): block (b, q) computes output channels [16q, 16q + 16) of board b, so one board's
// trunk is spread over 4 CUs and each block stages a quarter of conv2's weights (18 KB instead
// of 74 KB).  Every feature value is the same MFMA chain as c4_trunk_tile's (same operands,
// same k order, same bias + ReLU), so the output is bit-identical to c4_trunk_kernel<1>.
// 256 threads.
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
  const int lane = tid & 63, mt = tid >> 6;            // wave = m-tile (4 x 16 rows >= 49)
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
  __syncthreads();
  float breg[72];   // c4_trunk_tile's k order: step tap * 8 + j takes channel 8h + j
#pragma unroll
  for (int s = 0; s < 72; ++s) {
    const int tap = s >> 3, ci = 8 * h + (s & 7);
    breg[s] = w2s[c16 * W2S_STRIDE + ci * 9 + (tap / 3) * 3 + (tap % 3)];
  }
  for (int i = tid; i < CI * PP; i += 256) {
    const int pp = i / CI, ci = i % CI, px = pp / 9, py = pp % 9;
    float v = 0.f;
    if (px >= 1 && px <= 7 && py >= 1 && py <= 7) {
      float s = 0.f;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
          s = fmaf(w1s[ci * 9 + kh * 3 + kw], bd[(px - 1 + kh) * 9 + (py - 1 + kw)], s);
      s += w1s[CI * 9 + ci];
      v = s > 0.f ? s : 0.f;
    }
    c1[pp * C1S + ci] = v;
  }
  __syncthreads();
  const int i = mt * 16 + c16;
  const float* a0 = c1 + (i < P ? ((i / 7) * 9 + (i % 7)) * C1S : 0) + 8 * h;
  f32x4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int off = ((tap / 3) * 9 + (tap % 3)) * C1S;
    const f32x4v x = *reinterpret_cast<const f32x4v*>(a0 + off);
    const f32x4v y = *reinterpret_cast<const f32x4v*>(a0 + off + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(j < 4 ? x[j] : y[j - 4], breg[tap * 8 + j], acc,
                                                 0, 0, 0);
  }
  if constexpr (SC1) {
    // the block's 16 channels x 49 positions are ONE contiguous, 16-B aligned run of 784 floats
    // (feat[b][16q * 49 ..]): staged in LDS (conv1's tile is no longer read) and written through
    // as 196 16-B stores instead of 784 dword ones (each an own fabric write when write-through)
    __syncthreads();                                 // every wave is done reading c1
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int p = mt * 16 + h * 4 + r;
      if (p < P) {
        const float v = acc[r] + bias;
        c1[c16 * P + p] = v > 0.f ? v : 0.f;
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
      const int p = mt * 16 + h * 4 + r;
      if (p < P) {
        const float v = acc[r] + bias;
        feat[(size_t)b * 3136 + co * P + p] = v > 0.f ? v : 0.f;
      }
    }
  }
}

}  // namespace az
