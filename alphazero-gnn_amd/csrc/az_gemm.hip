// fp32 GEMM on gfx950 MFMA (v_mfma_f32_32x32x2_f32) with fused epilogues, plus a
// weight-streaming GEMV for M <= 8 (batch-1 predict, the star's row-0 update).
//
// Tile kernel: 256 threads = 4 waves as 2x2, BM x BN block tile (128x128 or 64x64), BK = 32,
// register-staged double-buffered LDS, optional split-K with a deterministic slab reduce when
// the tile grid alone cannot fill the 256 CUs.  Both operands are kept K-contiguous in LDS
// ([row][k], stride 36 floats: conflict-free ds_read_b128 for the 16-lane groups) so each lane
// fetches 4 k-values
// of its A row / B column with one ds_read_b128 and feeds 4 MFMAs; the k order inside an
// 8-k group is permuted (lane half h owns k = 4h..4h+3, MFMA t sums k = t and 4+t), which
// changes only the fp32 summation order.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <type_traits>
#include <utility>
#include <unordered_map>
#include <vector>

#include "az_common.h"
#include "az_x3.h"
#include "az_heads.h"
#include "az_trunk_split.h"

namespace az {

struct GemmArgs {
  int M, N, K;
  const float* A; int lda;
  const float* A2; int lda2; int K0;
  const int* a_rows;
  const float* B; int ldb;
  const int* b_rows;
  const float* bias; int act;
  const float* R; int ldr;
  const float* G; int ldg;
  float beta;
  float* C; int ldc;
  const int* c_rows;
  float* C2; int ldc2;
  // split-K: block (tile, s) covers k in [s*kc, min(K, (s+1)*kc)) and writes raw partial sums
  // to slab[s][M][N]; splitk_reduce_kernel sums the slabs in s order (deterministic) and runs
  // the epilogue.
  int splits, kc;
  float* slab;
  int vec_epi;  // host-checked: N, every leading dimension % 4 == 0 and 16-B aligned C/C2/R/G,
                // so whole float4 rows can leave through epilogue_store4
  int ablate;   // timing experiments only (AZ_GEMM_ABLATE, glds2): 1 = no DMA after the first
                // tile, 2 = no barrier in the k loop; results are then wrong
  // gemm_x3 with A already split (x3_split_kernel): three bf16 planes [3][M][K] at apl
  const unsigned short* apl;
  size_t apl_plane;   // elements per plane (M * K)
  // gemm_p3: W already split too, three bf16 planes [3][N][K] at bpl (row stride K)
  const unsigned short* bpl;
  size_t bpl_plane;   // elements per plane (N * K)
  // gemm_x3 in its fp16 form (H3): per-row power-of-two scales of A ([2][M]: s, then 1/s) and of
  // W ([2][N]), row_scale_kernel
  const float* sa;
  const float* sw;
  // gemm_p3 HEADS: the heads' dot products per tile row instead of C / slabs (az_x3.h HeadsEpi)
  HeadsEpi he;
  int heads_done;   // host side: launch_x3 ran the HEADS form (no C, no slabs written)
};

__device__ __forceinline__ void epilogue_store(const GemmArgs& p, int row, int col, float acc) {
  if (row >= p.M || col >= p.N) return;
  float v = acc + (p.bias ? p.bias[col] : 0.f);
  if (p.act == AZ_ACT_DRELU) {
    v = p.G[(size_t)row * p.ldg + col] > 0.f ? v : 0.f;
  } else {
    v = apply_act(v, p.act);
  }
  if (p.C2) p.C2[(size_t)row * p.ldc2 + col] = v;
  const int cr = p.c_rows ? p.c_rows[row] : row;
  if (p.R) v = p.R[(size_t)cr * p.ldr + col] + (p.G ? p.G[(size_t)row * p.ldg + col] : 1.f) * v;
  float* dst = p.C + (size_t)cr * p.ldc + col;
  if (p.beta != 0.f) v += p.beta * *dst;
  *dst = v;
}

// epilogue_store for 4 consecutive columns (col % 4 == 0, col + 4 <= N, p.vec_epi): one float4
// load / store per operand instead of four scalar ones.
__device__ __forceinline__ void epilogue_store4(const GemmArgs& p, int row, int col, f32x4 v) {
  if (row >= p.M || col >= p.N) return;
  if (p.bias) {
    const f32x4 b = *reinterpret_cast<const f32x4*>(p.bias + col);
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] += b[c];
  }
  if (p.act == AZ_ACT_DRELU) {
    const f32x4 g = *reinterpret_cast<const f32x4*>(p.G + (size_t)row * p.ldg + col);
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = g[c] > 0.f ? v[c] : 0.f;
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = apply_act(v[c], p.act);
  }
  if (p.C2) *reinterpret_cast<f32x4*>(p.C2 + (size_t)row * p.ldc2 + col) = v;
  const int cr = p.c_rows ? p.c_rows[row] : row;
  if (p.R) {
    const f32x4 r = *reinterpret_cast<const f32x4*>(p.R + (size_t)cr * p.ldr + col);
    f32x4 g = {1.f, 1.f, 1.f, 1.f};
    if (p.G) g = *reinterpret_cast<const f32x4*>(p.G + (size_t)row * p.ldg + col);
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = r[c] + g[c] * v[c];
  }
  f32x4* dst = reinterpret_cast<f32x4*>(p.C + (size_t)cr * p.ldc + col);
  if (p.beta != 0.f) {
    const f32x4 o = *dst;
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] += p.beta * o[c];
  }
  *dst = v;
}

// Loaders.  Every per-thread row pointer is resolved ONCE before the K loop, each load in the
// loop is unconditional (rows past M/N are clamped to row 0: they only feed outputs that are
// never stored) and the K-tail mask is applied when the staged registers are written to LDS,
// after the MFMA block of the previous tile.  A branch or a select on a loaded value next to
// the load makes hipcc wait vmcnt(0) right there, which serialises the prefetch
// (cdna_hip_programming.md §5 item 4(c)).
template <int ROWS, int BK, int NT>
struct KMajorSlots {
  static constexpr int NF4 = ROWS * BK / 4 / NT;
  const float* p0[NF4];   // row pointer in segment 0 (A or B)
  const float* p1[NF4];   // row pointer in segment 1 (A2, pre-offset by -K0), k >= K0
  int kq[NF4];
};

template <int ROWS, int BK, int NT, bool IS_A>
__device__ __forceinline__ void init_kmajor(const GemmArgs& p, int r0, int nrows,
                                            KMajorSlots<ROWS, BK, NT>& sl) {
  constexpr int F4_PER_ROW = BK / 4;
#pragma unroll
  for (int q = 0; q < KMajorSlots<ROWS, BK, NT>::NF4; ++q) {
    const int idx = threadIdx.x + q * NT;
    const int gr = r0 + idx / F4_PER_ROW;
    const int cr = gr < nrows ? gr : 0;
    sl.kq[q] = (idx % F4_PER_ROW) * 4;
    if (IS_A) {
      const int ar = p.a_rows ? p.a_rows[cr] : cr;
      sl.p0[q] = p.A + (size_t)ar * p.lda;
      sl.p1[q] = p.A2 ? p.A2 + (size_t)ar * p.lda2 - p.K0 : sl.p0[q];
    } else {
      sl.p0[q] = p.B + (size_t)cr * p.ldb;
      sl.p1[q] = sl.p0[q];
    }
  }
}

template <int ROWS, int BK, int NT>
__device__ __forceinline__ void load_kmajor(const KMajorSlots<ROWS, BK, NT>& sl, int k0, int kend,
                                            int K0, f32x4 (&reg)[ROWS * BK / 4 / NT]) {
#pragma unroll
  for (int q = 0; q < KMajorSlots<ROWS, BK, NT>::NF4; ++q) {
    const int k = k0 + sl.kq[q];
    const int kk = k < kend ? k : 0;
    reg[q] = *reinterpret_cast<const f32x4*>((kk >= K0 ? sl.p1[q] : sl.p0[q]) + kk);
  }
}

template <int ROWS, int BK, int NT, int LDK>
__device__ __forceinline__ void store_kmajor(float* lds, const f32x4 (&reg)[ROWS * BK / 4 / NT],
                                             int k0, int kend) {
  constexpr int NF4 = ROWS * BK / 4 / NT;
  constexpr int F4_PER_ROW = BK / 4;
#pragma unroll
  for (int q = 0; q < NF4; ++q) {
    const int idx = threadIdx.x + q * NT;
    const int row = idx / F4_PER_ROW, kq = idx % F4_PER_ROW;
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<f32x4*>(lds + row * LDK + kq * 4) = (k0 + kq * 4 < kend) ? reg[q] : z;
  }
}

// Operand contiguous along its M/N dimension: element (k, i) at base[row(k)*ld + i] with
// row(k) = rows ? rows[k] : k (row gather for weight gradients of gathered destinations).
template <int ROWS, int BK, int NT>
__device__ __forceinline__ void load_mnmajor(const float* base, int ld, const int* rows, int r0,
                                             int k0, int kend, int nrows,
                                             f32x4 (&reg)[ROWS * BK / 4 / NT]) {
  constexpr int NF4 = ROWS * BK / 4 / NT;
  constexpr int PER_K = ROWS / 4;
#pragma unroll
  for (int q = 0; q < NF4; ++q) {
    const int idx = threadIdx.x + q * NT;
    const int kr = idx / PER_K, mq = idx % PER_K;
    const int gr = r0 + mq * 4, k = k0 + kr;
    const int kk = k < kend ? k : 0;
    const int rk = rows ? rows[kk] : kk;
    reg[q] = *reinterpret_cast<const f32x4*>(base + (size_t)rk * ld + (gr < nrows ? gr : 0));
  }
}

template <int ROWS, int BK, int NT, int LDK>
__device__ __forceinline__ void store_mnmajor(float* lds, const f32x4 (&reg)[ROWS * BK / 4 / NT],
                                              int k0, int kend) {
  constexpr int NF4 = ROWS * BK / 4 / NT;
  constexpr int PER_K = ROWS / 4;
#pragma unroll
  for (int q = 0; q < NF4; ++q) {
    const int idx = threadIdx.x + q * NT;
    const int kr = idx / PER_K, mq = idx % PER_K;
    const bool ok = k0 + kr < kend;
#pragma unroll
    for (int e = 0; e < 4; ++e) lds[(mq * 4 + e) * LDK + kr] = ok ? reg[q][e] : 0.f;
  }
}

// Bijective XCD-aware remap for any grid size: hardware deals blocks round-robin over the 8
// XCDs (b -> XCD b % 8); XCD x gets the contiguous id range [start(x), start(x) + count(x)).
__device__ __forceinline__ int xcd_swizzle(int bid, int nwg) {
  const int xcd = bid & 7, local = bid >> 3;
  const int base = nwg >> 3, rem = nwg & 7;
  return xcd * base + min(xcd, rem) + local;
}

// (m tile, n tile, split) of swizzled id `bid`.  Up to 8 m tiles: m fastest (the tiles of one W
// panel adjacent).  More (large M, no split): groups of 4 m tiles, m fastest inside a group and
// the group's n tiles in turn, so an XCD's ~32 resident blocks are 4 m x 8 n tiles -- W panels
// re-read per group of 4 m tiles instead of A panels per n tile (M = 65,536 x 3136: the m-fastest
// order re-fetched every 3.2 MB A panel for each of the 25 n tiles, 22 GB per call; L2 hit 0.33)
__device__ __forceinline__ void tile_of(int bid, int mt_n, int nt_n, int& mt, int& nt, int& sp) {
  const int tiles = mt_n * nt_n;
  sp = bid / tiles;
  const int t = bid - sp * tiles;
  if (mt_n <= 8) {
    mt = t % mt_n;
    nt = t / mt_n;
    return;
  }
  constexpr int GM = 4;
  const int per = GM * nt_n, g = t / per, r = t - g * per;
  const int gm = min(GM, mt_n - g * GM);     // the last group may be ragged
  mt = g * GM + r % gm;
  nt = r / gm;
}

// Tile epilogue shared by the tile kernels.  A wave owns the TI x TJ MF x MF accumulators of
// its sub-tile at (r0, c0).  No split: the fused epilogue straight from the accumulators.
// Split-K: the raw partial goes to slab[sp] and splitk_reduce_kernel sums the slabs in s order.
// (An in-launch reduction by each tile's last-arriving block -- agent-scope release/acquire
// around a ticket counter -- was measured 1.8x slower here: a tile's 5 slabs are 320 KB, far
// above the few tens of KB where one block's serial combine beats a separate launch;
// cdna_hip_programming.md §5 "In-launch split-K reduction".)
// WAVE_LOCAL: only some of the block's waves run the epilogue (gemm_x3ws: the producer waves
// have left), each in its own stage region, so the block barriers become wave-local LDS waits.
template <int MF, int TI, int TJ, bool WAVE_LOCAL = false, class Acc>
__device__ __forceinline__ void tile_epilogue(const GemmArgs& p, Acc (&acc)[TI][TJ], int r0,
                                              int c0, int sp, float* stage = nullptr) {
  // Each wave stages through its own LDS region, so only the first wait needs the block (the k
  // loop's last LDS reads, other waves' included, must be done before the region is written);
  // the per-chunk waits are wave-local: a __syncthreads there is also a release fence that drains
  // every outstanding global store (s_waitcnt vmcnt(0)) -- twice per 32-column chunk, with every
  // block of a one-round grid storing at once (MI355X, tools/gpu_p3_abl.sh: 15 of 41 us at
  // M = 512, 158 of 594 at M = 8,192 were this epilogue)
  auto sync_first = [] {
    if constexpr (WAVE_LOCAL) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else __syncthreads();
  };
  auto sync = [] { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
  constexpr int NACC = MF == 32 ? 16 : 4;
  constexpr int WM = TI * MF, WN = TJ * MF;
  const int lane = threadIdx.x & 63;
  auto row_in = [&](int i, int r) {
    return i * MF + (MF == 32 ? (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5) : 4 * (lane >> 4) + r);
  };
  const int cl = lane & (MF - 1);
  const bool skip = (p.ablate & 4) != 0;
  const size_t plane = (size_t)p.M * p.N;
  float* slab = p.splits > 1 ? p.slab + (size_t)sp * plane : nullptr;
  if (stage != nullptr && p.vec_epi && WN % 32 == 0) {
    // Row-contiguous stores through the wave's LDS region (the MFMA layout scatters 4-byte
    // stores over 2-4 rows per instruction): each 32-column chunk of the wave tile is written
    // to LDS [WM][36] and read back as float4 rows, 8 lanes per 128-B row segment.
    constexpr int LD = 36, CH = 32 / MF;   // MFMA column tiles per 32-column chunk
    sync_first();                           // the k loop's last LDS reads are done everywhere
#pragma unroll
    for (int cc = 0; cc < WN / 32; ++cc) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int jj = 0; jj < CH; ++jj)
#pragma unroll
          for (int r = 0; r < NACC; ++r)
            stage[row_in(i, r) * LD + jj * MF + cl] = acc[i][cc * CH + jj][r];
      sync();
#pragma unroll
      for (int it = 0; it < WM / 8; ++it) {
        const int idx = it * 64 + lane, rl = idx >> 3, c4 = (idx & 7) * 4;
        const f32x4 v = *reinterpret_cast<const f32x4*>(stage + rl * LD + c4);
        const int row = r0 + rl, col = c0 + cc * 32 + c4;
        if (skip && v[0] == v[0]) continue;
        if (slab) {
          if (row < p.M && col < p.N) *reinterpret_cast<f32x4*>(slab + (size_t)row * p.N + col) = v;
        } else {
          epilogue_store4(p, row, col, v);
        }
      }
      sync();
    }
    return;
  }
  if (!slab) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < NACC; ++r)
          if (!skip || acc[i][j][r] != acc[i][j][r])
            epilogue_store(p, r0 + row_in(i, r), c0 + j * MF + cl, acc[i][j][r]);
    return;
  }
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < NACC; ++r) {
        const int row = r0 + row_in(i, r), col = c0 + j * MF + cl;
        if (row < p.M && col < p.N && (!skip || acc[i][j][r] != acc[i][j][r]))
          slab[(size_t)row * p.N + col] = acc[i][j][r];
      }
}

// The heads' weights (and y's bias) a HEADS tile's wave needs, loaded before the k loop so their
// latency hides under it: chunk cc (32 columns from c0 + 32 cc), slot a (policy rows a < A, slot
// 8 the value row), half h: lane l holds column c0 + 32 cc + 16 h + (l & 15).  The epilogue gives
// every lane the weight of column c with a DPP row_share:(c & 15) operand -- no LDS, no scalar
// loads in the epilogue.
template <int TJ>
struct HeadsRegs {
  float w[TJ][HEADS_TILE_SLOTS][2];
  float b[TJ][2];
};
template <int TJ>
__device__ __forceinline__ void heads_preload(const GemmArgs& p, int c0, HeadsRegs<TJ>& hr) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int cc = 0; cc < TJ; ++cc)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int col = c0 + cc * 32 + 16 * h + (lane & 15);
      const bool in = c0 + cc * 32 < p.N;         // N % 32 == 0: whole chunks
      const int cl = in ? col : 0;
#pragma unroll
      for (int a = 0; a < HEADS_TILE_SLOTS; ++a) {
        const bool use = in && (a == 8 || a < p.he.A);
        const float* src = a < 8 ? p.he.wp + (size_t)min(a, max(p.he.A - 1, 0)) * p.N : p.he.wv;
        hr.w[cc][a][h] = use ? src[cl] : 0.f;
      }
      hr.b[cc][h] = in && p.bias ? p.bias[cl] : 0.f;
    }
}

// acc + bcast(w) * x and x + bcast(b), bcast = lane C of each 16-lane row (DPP row_newbcast, the
// gfx950 row_share) as the operand modifier of the VALU op itself: one instruction each.  The
// first use of a weight register per chunk waits 2 cycles (s_nop 1): a VALU write of a VGPR that a
// DPP operand reads needs 2 wait states, and the register may have been copied just before.
template <int C>
__device__ __forceinline__ float fma_share(float acc, float w, float x) {
  if constexpr (C == 0)
    asm("s_nop 1\n\tv_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc) : "v"(w), "v"(x), "i"(C));
  else
    asm("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc) : "v"(w), "v"(x), "i"(C));
  return acc;
}
template <int C>
__device__ __forceinline__ float add_share(float x, float b) {
  if constexpr (C == 0)
    asm("s_nop 1\n\tv_add_f32_dpp %0, %1, %0 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
        : "+v"(x) : "v"(b), "i"(C));
  else
    asm("v_add_f32_dpp %0, %1, %0 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
        : "+v"(x) : "v"(b), "i"(C));
  return x;
}

// The HEADS epilogue of a 64-row wave tile (gemm_p3 / gemm_x3 / gemm_x3_csk HEADS; az_x3.h
// HeadsEpi): per row, the dot products of the wave's WN columns of the tile (+ the bias in k split
// / piece 0) with the 8 policy rows and the value row, in column order.
//   split-K form (p.he.mp == 0): the WGN waves sharing the rows are added in wave order through
//     LDS and the block's row results leave as part[row][nt * splits + sp][0..8] -- every wave
//     reaches the block barrier; comb: [WGM][64][9] floats;
//   stream-K form (p.he.mp > 0): each wave writes its own slot part[row][(c0 / 64) mp + sp].
// stage: the wave's [64][36] region.
template <int TI, int TJ, int WGM, int WGN>
__device__ __forceinline__ void heads_tile_epilogue(const GemmArgs& p, f32x16 (&acc)[TI][TJ],
                                                    const HeadsRegs<TJ>& hr, int r0, int c0,
                                                    int nt, int sp, int wm, int wn, float* stage,
                                                    float* comb) {
  constexpr int WM = TI * 32, LD = 36, HS = HEADS_TILE_SLOTS;
  static_assert(WM == 64, "one row per lane");
  const int lane = threadIdx.x & 63;
  float part[HS];
#pragma unroll
  for (int a = 0; a < HS; ++a) part[a] = 0.f;
#pragma unroll
  for (int cc = 0; cc < TJ; ++cc) {
    if (c0 + cc * 32 >= p.N) break;          // N % 32 == 0 (host-checked): whole chunks only
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        stage[(i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * LD + (lane & 31)] =
            acc[i][cc][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // wave-local: own region
    f32x4 x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = *reinterpret_cast<const f32x4*>(stage + lane * LD + 4 * q);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // read before the next chunk's stores
    if (sp == 0) {
      static_for<32>([&](auto C) {
        constexpr int c = decltype(C)::value;
        x[c >> 2][c & 3] = add_share<c & 15>(x[c >> 2][c & 3], hr.b[cc][c >> 4]);
      });
    }
    static_for<32>([&](auto C) {
      constexpr int c = decltype(C)::value;
#pragma unroll
      for (int a = 0; a < HS; ++a)
        part[a] = fma_share<c & 15>(part[a], hr.w[cc][a][c >> 4], x[c >> 2][c & 3]);
    });
  }
  const int row = r0 + lane;
  if (p.he.mp > 0) {                         // stream-K: one slot per wave
    if (row < p.M && c0 < p.N) {
      const int P = (p.N >> 6) * p.he.mp;
      float* dst = p.he.part + ((size_t)row * P + (c0 >> 6) * p.he.mp + sp) * HS;
#pragma unroll
      for (int a = 0; a < HS; ++a) dst[a] = part[a];
    }
    return;
  }
  // the WGN waves of this row group: wave order, through LDS
  if (wn > 0) {
#pragma unroll
    for (int a = 0; a < HS; ++a) comb[((wn - 1) * WGM + wm) * 64 * HS + lane * HS + a] = part[a];
  }
  __syncthreads();
  if (wn == 0) {
    for (int w = 1; w < WGN; ++w)
#pragma unroll
      for (int a = 0; a < HS; ++a) part[a] += comb[((w - 1) * WGM + wm) * 64 * HS + lane * HS + a];
    if (row < p.M) {
      const int P = ((p.N + WGN * 64 - 1) / (WGN * 64)) * p.splits;
      float* dst = p.he.part + ((size_t)row * P + nt * p.splits + sp) * HS;
#pragma unroll
      for (int a = 0; a < HS; ++a) dst[a] = part[a];
    }
  }
}

// Waves arranged WGM x WGN; each wave computes a (BM/WGM) x (BN/WGN) sub-tile as TI x TJ
// 32x32 MFMA accumulators.
template <int BM, int BN, int BK, int WGM, int WGN, bool A_KM, bool B_KM>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_f32_mfma(GemmArgs p) {
  constexpr int NT = 64 * WGM * WGN;
  constexpr int LDK = BK + 4;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TI = WM / 32, TJ = WN / 32;
  constexpr int AF4 = BM * BK / 4 / NT, BF4 = BN * BK / 4 / NT;
  static_assert(TI >= 1 && TJ >= 1 && AF4 >= 1 && BF4 >= 1, "bad tile");
  __shared__ __attribute__((aligned(16))) float As[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDK];

  const int mt_n = (p.M + BM - 1) / BM, nt_n = (p.N + BN - 1) / BN;
  const int nwg = mt_n * nt_n * p.splits;
  // consecutive ids share (split, B panel): keep them on one XCD so the weight slice is
  // fetched into that XCD's L2 once and re-read from there by the M tiles.
  const int bid = xcd_swizzle(blockIdx.x, nwg);
  const int mt = bid % mt_n, nt = (bid / mt_n) % nt_n, sp = bid / (mt_n * nt_n);
  const int m0 = mt * BM, n0 = nt * BN;
  const int kbeg = sp * p.kc, kend = min(p.K, kbeg + p.kc);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WGN, wn = wave % WGN;

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  f32x4 ra[AF4], rb[BF4];
  KMajorSlots<BM, BK, NT> sa;
  KMajorSlots<BN, BK, NT> sb;
  if constexpr (A_KM) init_kmajor<BM, BK, NT, true>(p, m0, p.M, sa);
  if constexpr (B_KM) init_kmajor<BN, BK, NT, false>(p, n0, p.N, sb);
  auto load = [&](int k0) {
    if constexpr (A_KM) load_kmajor<BM, BK, NT>(sa, k0, kend, p.K0, ra);
    else load_mnmajor<BM, BK, NT>(p.A, p.lda, nullptr, m0, k0, kend, p.M, ra);
    if constexpr (B_KM) load_kmajor<BN, BK, NT>(sb, k0, kend, p.K, rb);
    else load_mnmajor<BN, BK, NT>(p.B, p.ldb, p.b_rows, n0, k0, kend, p.N, rb);
  };
  auto store = [&](int buf, int k0) {
    if constexpr (A_KM) store_kmajor<BM, BK, NT, LDK>(As[buf], ra, k0, kend);
    else store_mnmajor<BM, BK, NT, LDK>(As[buf], ra, k0, kend);
    if constexpr (B_KM) store_kmajor<BN, BK, NT, LDK>(Bs[buf], rb, k0, kend);
    else store_mnmajor<BN, BK, NT, LDK>(Bs[buf], rb, k0, kend);
  };

  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk > 0) {
    load(kbeg);
    store(0, kbeg);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load(kbeg + (kt + 1) * BK);
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      f32x4 a[TI], b[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i)
        a[i] = *reinterpret_cast<const f32x4*>(
            &As[cur][(wm * WM + i * 32 + (lane & 31)) * LDK + g * 8 + (lane >> 5) * 4]);
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        b[j] = *reinterpret_cast<const f32x4*>(
            &Bs[cur][(wn * WN + j * 32 + (lane & 31)) * LDK + g * 8 + (lane >> 5) * 4]);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][t], b[j][t], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store(cur ^ 1, kbeg + (kt + 1) * BK);
    __syncthreads();
  }

  tile_epilogue<32, TI, TJ>(p, acc, m0 + wm * WM, n0 + wn * WN, sp);
}

// ------------------------------------------------------------------------------ LDS-DMA tile
// Both operands K-major with no row gather / concatenation (the forward Linear layers).  Tiles
// of BM x BK and BN x BK floats go global -> LDS with global_load_lds_dwordx4 (no VGPR round
// trip): one wave-instruction fills 8 rows x 128 B.  The LDS image is unpadded, [row][32 k],
// with the 16-B chunk index XOR-swizzled by (row >> 1) & 7 -- applied on the per-lane GLOBAL
// address, since the LDS destination of a DMA is lane-linear -- so the fragment reads
// (ds_read_b128, 16 lanes = 16 consecutive rows at one k chunk) hit 16 distinct bank groups.
// Two LDS buffers: tile t+1 is in flight while tile t feeds the MFMAs; one barrier per tile.
// Rows past M/N read row 0 and k past the range reads k = 0 of the same row (valid memory,
// finite values); the A tail of a partial last tile is zeroed in LDS before use.
template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_f32_glds(GemmArgs p) {
  constexpr int BK = 32;
  constexpr int NT = 64 * WGM * WGN, NW = NT / 64;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TI = WM / 32, TJ = WN / 32;
  constexpr int APC = BM / 8 / NW, BPC = BN / 8 / NW;   // 8-row pieces per wave
  static_assert(TI >= 1 && TJ >= 1 && APC >= 1 && BPC >= 1, "bad tile");
  __shared__ __attribute__((aligned(1024))) float smem[2 * (BM + BN) * BK];

  const int mt_n = (p.M + BM - 1) / BM, nt_n = (p.N + BN - 1) / BN;
  const int nwg = mt_n * nt_n * p.splits;
  const int bid = xcd_swizzle(blockIdx.x, nwg);
  const int mt = bid % mt_n, nt = (bid / mt_n) % nt_n, sp = bid / (mt_n * nt_n);
  const int m0 = mt * BM, n0 = nt * BN;
  const int kbeg = sp * p.kc, kend = min(p.K, kbeg + p.kc);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WGN, wn = wave % WGN;

  // per-lane DMA sources: piece q of this wave covers rows (q*NW + wave)*8 .. +8
  const int lrow = lane >> 3, pch = lane & 7;
  const float* asrc[APC];
  const float* bsrc[BPC];
  int akq[APC], bkq[BPC];
#pragma unroll
  for (int q = 0; q < APC; ++q) {
    const int r = (q * NW + wave) * 8 + lrow;
    const int gr = m0 + r < p.M ? m0 + r : 0;
    asrc[q] = p.A + (size_t)gr * p.lda;
    akq[q] = (pch ^ ((r >> 1) & 7)) * 4;
  }
#pragma unroll
  for (int q = 0; q < BPC; ++q) {
    const int r = (q * NW + wave) * 8 + lrow;
    const int gr = n0 + r < p.N ? n0 + r : 0;
    bsrc[q] = p.B + (size_t)gr * p.ldb;
    bkq[q] = (pch ^ ((r >> 1) & 7)) * 4;
  }
  auto issue = [&](int buf, int k0) {
    float* As = smem + buf * (BM + BN) * BK;
    float* Bs = As + BM * BK;
#pragma unroll
    for (int q = 0; q < APC; ++q) {
      const int k = k0 + akq[q];
      const float* src = asrc[q] + (k < p.K ? k : 0);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)src,
          (__attribute__((address_space(3))) void*)(As + (q * NW + wave) * 8 * BK), 16, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < BPC; ++q) {
      const int k = k0 + bkq[q];
      const float* src = bsrc[q] + (k < p.K ? k : 0);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)src,
          (__attribute__((address_space(3))) void*)(Bs + (q * NW + wave) * 8 * BK), 16, 0, 0);
    }
  };
  // zero A's k >= kend columns of a partial tile.  Rows were DMA'd by other waves: every wave
  // has waited for its own DMAs (vmcnt(0)) before this point, and the barrier makes all of them
  // complete before any zero is written over them.
  auto zero_tail = [&](int buf, int k0) {
    if (k0 + BK <= kend) return;
    __syncthreads();
    float* As = smem + buf * (BM + BN) * BK;
    for (int idx = threadIdx.x; idx < BM * 8; idx += NT) {
      const int r = idx >> 3, lc = idx & 7;
      if (k0 + lc * 4 >= kend) {
        // kend is a multiple of 4 (K % 4 == 0 and kc % BK == 0)
        *reinterpret_cast<f32x4*>(As + r * BK + ((lc ^ ((r >> 1) & 7)) * 4)) =
            f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk > 0) {
    issue(0, kbeg);
    __builtin_amdgcn_s_waitcnt(0);
    zero_tail(0, kbeg);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) issue(cur ^ 1, kbeg + (kt + 1) * BK);
    const float* As = smem + cur * (BM + BN) * BK;
    const float* Bs = As + BM * BK;
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      f32x4 a[TI], b[TJ];
      const int lc = g * 2 + (lane >> 5);
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int r = wm * WM + i * 32 + (lane & 31);
        a[i] = *reinterpret_cast<const f32x4*>(As + r * BK + ((lc ^ ((r >> 1) & 7)) * 4));
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int r = wn * WN + j * 32 + (lane & 31);
        b[j] = *reinterpret_cast<const f32x4*>(Bs + r * BK + ((lc ^ ((r >> 1) & 7)) * 4));
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][t], b[j][t], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      __builtin_amdgcn_s_waitcnt(0);
      zero_tail(cur ^ 1, kbeg + (kt + 1) * BK);
    }
    __syncthreads();
  }

  tile_epilogue<32, TI, TJ>(p, acc, m0 + wm * WM, n0 + wn * WN, sp,
                            (NW * WM * 36 <= (int)(sizeof(smem) / 4)) ? smem + wave * (WM * 36)
                                                                       : nullptr);
}

// Multi-stage LDS-DMA tile: NBUF buffers, tile t+NBUF-1 is issued while tile t is consumed, so
// NBUF-1 tiles of DMA are in flight across each barrier.  No __syncthreads() in the loop (its
// fence would drain the DMAs, vmcnt(0)): a counted `s_waitcnt vmcnt(N)` retires exactly the
// oldest tile, then a raw s_barrier publishes it to every wave (cdna_hip_programming.md §5,
// "Pipelining across barriers").  The LDS image is [row][BK] with the 16-B chunk XOR-swizzled
// by the row bits that would otherwise put a 16-lane ds_read_b128 group on one bank set.
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int BK>
__device__ __forceinline__ int swz(int r) {
  // chunks per row = BK/4; rows per 256-B bank row = 256 / (BK*4)
  if constexpr (BK == 32) return (r >> 1) & 7;
  else if constexpr (BK == 16) return (r >> 2) & 3;
  else return (r >> 0) & 15;   // BK = 64
}

template <int BM, int BN, int BK, int NBUF, int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_f32_glds_pipe(GemmArgs p) {
  constexpr int NT = 64 * WGM * WGN, NW = NT / 64;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TI = WM / 32, TJ = WN / 32;
  constexpr int CPR = BK / 4;                    // 16-B chunks per row
  constexpr int RPP = 64 / CPR;                  // rows per 1-KB wave piece
  constexpr int APC = BM / RPP / NW, BPC = BN / RPP / NW;
  constexpr int DPT = APC + BPC;                 // DMAs per thread per tile
  constexpr int TILE = (BM + BN) * BK;
  static_assert(TI >= 1 && TJ >= 1 && APC >= 1 && BPC >= 1 && NBUF >= 2, "bad tile");
  static_assert(DPT * (NBUF - 2) <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(1024))) float smem[NBUF * TILE];

  const int mt_n = (p.M + BM - 1) / BM, nt_n = (p.N + BN - 1) / BN;
  const int nwg = mt_n * nt_n * p.splits;
  const int bid = xcd_swizzle(blockIdx.x, nwg);
  const int mt = bid % mt_n, nt = (bid / mt_n) % nt_n, sp = bid / (mt_n * nt_n);
  const int m0 = mt * BM, n0 = nt * BN;
  const int kbeg = sp * p.kc, kend = min(p.K, kbeg + p.kc);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WGN, wn = wave % WGN;

  const int lrow = lane / CPR, pch = lane % CPR;
  const float* asrc[APC];
  const float* bsrc[BPC];
  int akq[APC], bkq[BPC];
#pragma unroll
  for (int q = 0; q < APC; ++q) {
    const int r = (q * NW + wave) * RPP + lrow;
    const int gr = m0 + r < p.M ? m0 + r : 0;
    asrc[q] = p.A + (size_t)gr * p.lda;
    akq[q] = (pch ^ swz<BK>(r)) * 4;
  }
#pragma unroll
  for (int q = 0; q < BPC; ++q) {
    const int r = (q * NW + wave) * RPP + lrow;
    const int gr = n0 + r < p.N ? n0 + r : 0;
    bsrc[q] = p.B + (size_t)gr * p.ldb;
    bkq[q] = (pch ^ swz<BK>(r)) * 4;
  }
  auto issue = [&](int buf, int k0) {
    float* As = smem + buf * TILE;
    float* Bs = As + BM * BK;
#pragma unroll
    for (int q = 0; q < APC; ++q) {
      const int k = k0 + akq[q];
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(asrc[q] + (k < p.K ? k : 0)),
          (__attribute__((address_space(3))) void*)(As + (q * NW + wave) * RPP * BK), 16, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < BPC; ++q) {
      const int k = k0 + bkq[q];
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(bsrc[q] + (k < p.K ? k : 0)),
          (__attribute__((address_space(3))) void*)(Bs + (q * NW + wave) * RPP * BK), 16, 0, 0);
    }
  };

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = (kend - kbeg + BK - 1) / BK;
#pragma unroll
  for (int t = 0; t < NBUF - 1; ++t)
    if (t < nk) issue(t, kbeg + t * BK);
  for (int kt = 0; kt < nk; ++kt) {
    // tiles issued so far: min(nk, kt + NBUF - 1); retire tile kt, keep the later ones flying
    const int later = min(nk, kt + NBUF - 1) - kt - 1;
    if constexpr (NBUF >= 4) {
      if (later >= 2) wait_vm<DPT * 2>();
      else if (later == 1) wait_vm<DPT>();
      else wait_vm<0>();
    } else if constexpr (NBUF == 3) {
      if (later >= 1) wait_vm<DPT>();
      else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    lds_barrier();
    const int cur = kt % NBUF;
    const int k0 = kbeg + kt * BK;
    if (k0 + BK > kend) {                        // partial last tile: zero A's k >= kend
      float* As = smem + cur * TILE;
      for (int idx = threadIdx.x; idx < BM * CPR; idx += NT) {
        const int r = idx / CPR, lc = idx % CPR;
        if (k0 + lc * 4 >= kend)
          *reinterpret_cast<f32x4*>(As + r * BK + ((lc ^ swz<BK>(r)) * 4)) =
              f32x4{0.f, 0.f, 0.f, 0.f};
      }
      lds_barrier();
    }
    if (kt + NBUF - 1 < nk) issue((kt + NBUF - 1) % NBUF, kbeg + (kt + NBUF - 1) * BK);
    const float* As = smem + cur * TILE;
    const float* Bs = As + BM * BK;
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      f32x4 a[TI], b[TJ];
      const int lc = g * 2 + (lane >> 5);
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int r = wm * WM + i * 32 + (lane & 31);
        a[i] = *reinterpret_cast<const f32x4*>(As + r * BK + ((lc ^ swz<BK>(r)) * 4));
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int r = wn * WN + j * 32 + (lane & 31);
        b[j] = *reinterpret_cast<const f32x4*>(Bs + r * BK + ((lc ^ swz<BK>(r)) * 4));
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][t], b[j][t], acc[i][j], 0, 0, 0);
    }
  }

  tile_epilogue<32, TI, TJ>(p, acc, m0 + wm * WM, n0 + wn * WN, sp,
                            (NW * WM * 36 <= (int)(sizeof(smem) / 4)) ? smem + wave * (WM * 36)
                                                                       : nullptr);
}

// LDS-DMA tile, v2: the same LDS image and DMA schedule as gemm_f32_glds, but every wave reads
// ALL of its fragments for the k-tile (16 ds_read_b128) before the first MFMA, so the LDS
// latency of later fragment groups hides behind the MFMAs of earlier ones (the compiler counts
// lgkmcnt down group by group) instead of draining once per group.  MF selects the MFMA shape:
//   MF = 32: v_mfma_f32_32x32x2_f32, lane l holds A[row l&31][4 k of chunk 2g + (l>>5)]
//   MF = 16: v_mfma_f32_16x16x4_f32, lane l holds A[row l&15][4 k of chunk 4g + (l>>4)]
// Element t of the 4-k fragment feeds MFMA t, so the k order inside a group is permuted (only
// the fp32 summation order changes).  The 16x16 shape is the lower-energy one per FLOP
// (cdna_hip_programming.md §5.4 rule 28: the chip holds a higher clock on it).
//
// NB = 3 (IL = false only): a three-buffer LDS ring.  Tile kt + 2 is issued right after the
// barrier that retires tile kt, so each DMA has two k-tiles of MFMA time to land instead of
// one, and the wait before a tile is a counted vmcnt (the next tile's pieces stay in flight);
// one barrier per k-tile.  256x128: 144 KB of LDS, one block per CU.
template <int BM, int BN, int WGM, int WGN, int MF, bool IL, int NB = 2, bool ST = false>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_f32_glds2(GemmArgs p) {
  static_assert(NB == 2 || (NB == 3 && !IL), "three-buffer ring without interleaved issue");
  static_assert(!ST || NB == 3, "the stagger needs the three-buffer ring");
  constexpr int BK = 32;
  constexpr int NT = 64 * WGM * WGN, NW = NT / 64;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TI = WM / MF, TJ = WN / MF;
  constexpr int NG = MF == 32 ? BK / 8 : BK / 16;     // fragment groups per k-tile
  constexpr int LSH = MF == 32 ? 5 : 4;                // lane >> LSH = chunk within a group
  constexpr int APC = BM / 8 / NW, BPC = BN / 8 / NW;
  using acc_t = typename std::conditional<MF == 32, f32x16, f32x4>::type;
  constexpr int NACC = MF == 32 ? 16 : 4;
  static_assert(TI >= 1 && TJ >= 1 && APC >= 1 && BPC >= 1, "bad tile");
  __shared__ __attribute__((aligned(1024))) float smem[NB * (BM + BN) * BK];

  const int mt_n = (p.M + BM - 1) / BM, nt_n = (p.N + BN - 1) / BN;
  const int nwg = mt_n * nt_n * p.splits;
  const int bid = xcd_swizzle(blockIdx.x, nwg);
  const int mt = bid % mt_n, nt = (bid / mt_n) % nt_n, sp = bid / (mt_n * nt_n);
  const int m0 = mt * BM, n0 = nt * BN;
  const int kbeg = sp * p.kc, kend = min(p.K, kbeg + p.kc);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WGN, wn = wave % WGN;

  const int lrow = lane >> 3, pch = lane & 7;
  const float* asrc[APC];
  const float* bsrc[BPC];
  int akq[APC], bkq[BPC];
#pragma unroll
  for (int q = 0; q < APC; ++q) {
    const int r = (q * NW + wave) * 8 + lrow;
    const int gr = m0 + r < p.M ? m0 + r : 0;
    asrc[q] = p.A + (size_t)gr * p.lda;
    akq[q] = (pch ^ ((r >> 1) & 7)) * 4;
  }
#pragma unroll
  for (int q = 0; q < BPC; ++q) {
    const int r = (q * NW + wave) * 8 + lrow;
    const int gr = n0 + r < p.N ? n0 + r : 0;
    bsrc[q] = p.B + (size_t)gr * p.ldb;
    bkq[q] = (pch ^ ((r >> 1) & 7)) * 4;
  }
  auto issue = [&](int buf, int k0) {
    float* As = smem + buf * (BM + BN) * BK;
    float* Bs = As + BM * BK;
#pragma unroll
    for (int q = 0; q < APC; ++q) {
      const int k = k0 + akq[q];
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(asrc[q] + (k < p.K ? k : 0)),
          (__attribute__((address_space(3))) void*)(As + (q * NW + wave) * 8 * BK), 16, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < BPC; ++q) {
      const int k = k0 + bkq[q];
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(bsrc[q] + (k < p.K ? k : 0)),
          (__attribute__((address_space(3))) void*)(Bs + (q * NW + wave) * 8 * BK), 16, 0, 0);
    }
  };
  // one 1-KB DMA piece: q < APC is A piece q, else B piece q - APC
  auto issue_piece = [&](int buf, int k0, int q) {
    float* As = smem + buf * (BM + BN) * BK;
    float* Bs = As + BM * BK;
    if (q < APC) {
      const int k = k0 + akq[q];
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(asrc[q] + (k < p.K ? k : 0)),
          (__attribute__((address_space(3))) void*)(As + (q * NW + wave) * 8 * BK), 16, 0, 0);
    } else {
      const int qb = q - APC;
      const int k = k0 + bkq[qb];
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(bsrc[qb] + (k < p.K ? k : 0)),
          (__attribute__((address_space(3))) void*)(Bs + (qb * NW + wave) * 8 * BK), 16, 0, 0);
    }
  };
  auto zero_tail = [&](int buf, int k0) {
    if (k0 + BK <= kend) return;
    __syncthreads();
    float* As = smem + buf * (BM + BN) * BK;
    for (int idx = threadIdx.x; idx < BM * 8; idx += NT) {
      const int r = idx >> 3, lc = idx & 7;
      if (k0 + lc * 4 >= kend)
        *reinterpret_cast<f32x4*>(As + r * BK + ((lc ^ ((r >> 1) & 7)) * 4)) =
            f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };

  acc_t acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < NACC; ++r) acc[i][j][r] = 0.f;

  // per-lane fragment row offsets (in floats) and swizzle keys, fixed for the whole loop
  int aoff[TI], boff[TJ], akey[TI], bkey[TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i) {
    const int r = wm * WM + i * MF + (lane & (MF - 1));
    aoff[i] = r * BK;
    akey[i] = (r >> 1) & 7;
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int r = wn * WN + j * MF + (lane & (MF - 1));
    boff[j] = BM * BK + r * BK;
    bkey[j] = (r >> 1) & 7;
  }

  const int nk = (kend - kbeg + BK - 1) / BK;
  if constexpr (NB == 3) {
    constexpr int DPT = APC + BPC;                   // DMA pieces per lane per tile
    // ST: waves NW/2.. (the SIMD partners of waves 0..NW/2-1) run half a k-tile behind: they
    // carry the fragments of the tile's last group across the barrier and start each tile with
    // those MFMAs while their partners wait on their first LDS reads
    // (MI355X_MICROARCH.md, "two waves that run the same program ... try a stagger").  The
    // accumulation order of every wave is unchanged: results are bit-identical.
    const bool hi = ST && wave >= NW / 2;
    f32x4 a[NG][TI], b[NG][TJ];
    auto read = [&](const float* S, int g) {
      const int lc = g * (64 >> LSH) + (lane >> LSH);
#pragma unroll
      for (int i = 0; i < TI; ++i)
        a[g][i] = *reinterpret_cast<const f32x4*>(S + aoff[i] + ((lc ^ akey[i]) * 4));
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        b[g][j] = *reinterpret_cast<const f32x4*>(S + boff[j] + ((lc ^ bkey[j]) * 4));
    };
    auto mfma = [&](int g, int t) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          if constexpr (MF == 32)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[g][i][t], b[g][j][t], acc[i][j],
                                                             0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[g][i][t], b[g][j][t], acc[i][j],
                                                             0, 0, 0);
        }
    };
    if (nk > 0) issue(0, kbeg);
    if (nk > 1) issue(1, kbeg + BK);
    for (int kt = 0; kt < nk; ++kt) {
      // raw barriers only: __syncthreads()' fence would drain the next tile's DMA (vmcnt(0))
      if (kt + 1 < nk) wait_vm<DPT>();               // tile kt landed, tile kt + 1 in flight
      else wait_vm<0>();
      lds_barrier();                                 // ... for every wave; tile kt - 1 retired
      const int cur = kt % 3;
      const int k0 = kbeg + kt * BK;
      if (k0 + BK > kend) {                          // partial last tile: zero A's k >= kend
        float* As = smem + cur * (BM + BN) * BK;
        for (int idx = threadIdx.x; idx < BM * 8; idx += NT) {
          const int r = idx >> 3, lc = idx & 7;
          if (k0 + lc * 4 >= kend)
            *reinterpret_cast<f32x4*>(As + r * BK + ((lc ^ ((r >> 1) & 7)) * 4)) =
                f32x4{0.f, 0.f, 0.f, 0.f};
        }
        lds_barrier();
      }
      if (kt + 2 < nk) issue((kt + 2) % 3, k0 + 2 * BK);   // overwrites tile kt - 1's buffer
      const float* S = smem + cur * (BM + BN) * BK;
      if (!hi) {
        read(S, 0);
#pragma unroll
        for (int g = 0; g < NG; ++g)
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            mfma(g, t);
            if (t == 0 && g + 1 < NG) {
              __builtin_amdgcn_sched_barrier(0);
              read(S, g + 1);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
      } else {
        if (kt > 0) {                                // tile kt - 1's last group, from registers
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            mfma(NG - 1, t);
            if (t == 0) {
              __builtin_amdgcn_sched_barrier(0);
              read(S, 0);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
        } else {
          read(S, 0);
        }
#pragma unroll
        for (int g = 0; g < NG - 1; ++g)
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            mfma(g, t);
            if (t == 0) {
              __builtin_amdgcn_sched_barrier(0);
              read(S, g + 1);                        // group NG - 1 rides across the barrier
              __builtin_amdgcn_sched_barrier(0);
            }
          }
      }
    }
    if (hi && nk > 0) {
#pragma unroll
      for (int t = 0; t < 4; ++t) mfma(NG - 1, t);
    }
    lds_barrier();                                   // the epilogue reuses the LDS
    tile_epilogue<MF, TI, TJ>(p, acc, m0 + wm * WM, n0 + wn * WN, sp,
                              (NW * WM * 36 <= (int)(sizeof(smem) / 4)) ? smem + wave * (WM * 36)
                                                                         : nullptr);
    return;
  }
  if (nk > 0) {
    issue(0, kbeg);
    __builtin_amdgcn_s_waitcnt(0);
    zero_tail(0, kbeg);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk && !(p.ablate & 1);
    if (!IL && more) issue(cur ^ 1, kbeg + (kt + 1) * BK);
    const float* S = smem + cur * (BM + BN) * BK;
    f32x4 a[NG][TI], b[NG][TJ];
    auto read = [&](int g) {
      const int lc = g * (64 >> LSH) + (lane >> LSH);
#pragma unroll
      for (int i = 0; i < TI; ++i)
        a[g][i] = *reinterpret_cast<const f32x4*>(S + aoff[i] + ((lc ^ akey[i]) * 4));
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        b[g][j] = *reinterpret_cast<const f32x4*>(S + boff[j] + ((lc ^ bkey[j]) * 4));
    };
    // group g+1's fragments are read right after the first quarter of group g's MFMAs, so
    // their LDS latency hides behind the other three quarters; sched_barrier pins the order
    // (the scheduler would otherwise sink the reads behind all MFMAs to save registers) and
    // keeps at most two groups of reads outstanding (lgkmcnt counts to 15).
    read(0);
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            if constexpr (MF == 32)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[g][i][t], b[g][j][t], acc[i][j],
                                                               0, 0, 0);
            else
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[g][i][t], b[g][j][t], acc[i][j],
                                                               0, 0, 0);
          }
        if (t == 0 && g + 1 < NG) {
          __builtin_amdgcn_sched_barrier(0);
          read(g + 1);
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (IL) {
          // IL: the next tile's DMA pieces are spread over the first half of the MFMA steps
          // (one DMA issue stalls the wave for ~60-180 cycles; beside MFMAs it hides)
          constexpr int STEPS = NG * 4 / 2, PER = (APC + BPC + STEPS - 1) / STEPS;
          const int st = g * 4 + t;
          if (st < STEPS && more) {
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < PER; ++u)
              if (st * PER + u < APC + BPC) issue_piece(cur ^ 1, kbeg + (kt + 1) * BK, st * PER + u);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    if (more) {
      __builtin_amdgcn_s_waitcnt(0);
      zero_tail(cur ^ 1, kbeg + (kt + 1) * BK);
    }
    if (!(p.ablate & 2)) __syncthreads();
  }

  tile_epilogue<MF, TI, TJ>(p, acc, m0 + wm * WM, n0 + wn * WN, sp,
                            (NW * WM * 36 <= (int)(sizeof(smem) / 4)) ? smem + wave * (WM * 36)
                                                                       : nullptr);
}

// ---------------------------------------------------------------------------------------------
// fp32 GEMM on the bf16 matrix cores ("x3").  Every fp32 operand element x is split into three
// bf16 terms x = h + m + l, each rounded to nearest even (h = rne(x), m = rne(x - h),
// l = rne(x - h - m); |m| <= 2^-8 |x|, |l| <= 2^-16 |x|, and the three hold all 24 significand
// bits of x), and every product a*b is the sum of the six leading cross terms
//   ah*bl + al*bh + am*bm + ah*bm + am*bh + ah*bh
// on v_mfma_f32_32x32x16_bf16 (a bf16 x bf16 product is exact in fp32; sums are fp32).  The
// three dropped terms am*bl + al*bm + al*bl are below 2^-23 |a||b|, the size of one fp32
// rounding of the product, so the result keeps fp32 accuracy (tests/test_gpu_kernels.py holds
// it to the same 1e-6 * sum|a*b| bound as the fp32 MFMA path and compares both errors).  Cost:
// 6 x 32 cycles per 16 k against 8 x 64 for v_mfma_f32_32x32x2_f32, i.e. 2.67x the fp32 MFMA
// rate (MI355X_MICROARCH.md constants: 32x32x16 bf16 issues every 32 cycles per SIMD).
//
// Register-staged tile: each thread loads 8-k segments (two float4) of A and W rows, splits them
// after the current tile's MFMAs and writes the three planes to the other LDS buffer (one
// ds_write_b128 per plane); one barrier per 32-k tile.  LDS image per plane: [row][32 bf16]
// (64 B rows), 16-B chunk c stored at c ^ ((row >> 2) & 3), which makes the MFMA operand reads
// (lane: row lane & 31, chunk 2s + (lane >> 5)) conflict-free for every ds_read_b128 lane group.
// ABL (tuning build only, timing ablations whose results are wrong by design): 1 = every tile's
// loads from the split's first four tiles (L2-resident), 2 = no MFMA, 4 = no split (raw bits)
// APL: A comes as three bf16 planes split once by x3_split_kernel (p.apl, row stride K, K % 32
// == 0): the tile copies them into the LDS image without any VALU, only W is split here.
// MF = 16 (tuning build): v_mfma_f32_16x16x32_bf16 blocks, one k step per 32-k tile (lane l
// holds row l & 15, k chunk l >> 4), against two 32x32x16 steps for MF = 32.
template <int BM, int BN, int WGM, int WGN, int MF = 32, int PL = 3>
constexpr int x3_smem_bytes() {
  constexpr int NW = WGM * WGN, WM = BM / WGM;
  constexpr int BUF = PL * (BM + BN) * 64, STAGE = NW * WM * 36 * 4;
  return 2 * BUF > STAGE ? 2 * BUF : STAGE;
}

// One (tile, k range) of gemm_x3: C tile (mt, nt) over k in [kbeg, kend); sp = the split-K
// slab it writes when p.splits > 1 (raw partial sums), else the fused epilogue.
// FLEX (stream-K tail rows): the tile shape is chosen at run time from the 384 LDS rows of the
// 256 x 128 / 8-wave body: bma = 256 (256 x 128, waves 4 x 2) or bma = 128 (128 x 256, waves
// 2 x 4); every wave keeps its 64 x 64 sub-tile, so the loop, its MFMAs and its LDS traffic are
// the same, and only the loader's row split, the fragment row offsets and the epilogue origin
// change (all computed once, before the k loop).  mt / nt count tiles of that shape.
//
// H3: the fp16 form (see az_x3.h split2s): every operand row scaled by its power-of-two factor
// (p.sa / p.sw, from row_scale_kernel), split into two fp16 terms, a*b as the three products
// ah*bl + al*bh + ah*bh on v_mfma_f32_32x32x16_f16 (two LDS planes instead of three, half the
// MFMAs), and the accumulators multiplied back by 1 / (sa[row] sw[col]) (exact) before the
// epilogue.
template <int BM, int BN, int WGM, int WGN, bool MASK, int ABL = 0, bool APL = false, int MF = 32,
          bool FLEX = false, bool H3 = false, bool HEADS = false>
__device__ __forceinline__ void gemm_x3_body(const GemmArgs& p, char* smem, int mt, int nt,
                                             int sp, int kbeg, int kend, int bma = BM) {
  static_assert(!APL || !MASK, "pre-split A needs whole 32-k tiles");
  static_assert(!H3 || (!APL && ABL == 0 && MF == 32), "H3: the product form only");
  static_assert(!FLEX || (BM == 256 && BN == 128 && WGM == 4 && WGN == 2 && MF == 32 && !APL),
                "FLEX reshapes the 256 x 128 8-wave tile");
  constexpr int BK = 32;
  constexpr int NT = 64 * WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TI = WM / MF, TJ = WN / MF;
  constexpr int NSTEP = MF == 32 ? 2 : 1;
  using acc_t = typename std::conditional<MF == 32, f32x16, f32x4>::type;
  constexpr int NACC = MF == 32 ? 16 : 4;
  constexpr int ASEG = BM * 4 / NT, BSEG = BN * 4 / NT, NSEG = ASEG + BSEG;
  static_assert(TI >= 1 && TJ >= 1 && ASEG >= 1 && BSEG >= 1 && (BM * 4) % NT == 0 &&
                (BN * 4) % NT == 0, "bad x3 tile");
  constexpr int PL = H3 ? 2 : 3;                 // operand planes (fp16 h, l / bf16 h, m, l)
  constexpr int PLANE = (BM + BN) * 64;          // bytes of one 16-bit plane (A rows, then W rows)
  constexpr int BUF = PL * PLANE;
  const int tbm = FLEX ? bma : BM, tbn = FLEX ? BM + BN - bma : BN;
  const int wgn = FLEX ? tbn / WN : WGN;
  const int m0 = mt * tbm, n0 = nt * tbn;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / wgn, wn = wave % wgn;

  // loader: segment q covers image row (tid + q NT) >> 2 (A rows first, then W rows),
  // k = 8 * (idx & 3) ..+7
  const float* src[NSEG];
  int soff[NSEG], sk[NSEG];
  float ssc[H3 ? NSEG : 1];                      // H3: the segment's row scale
#pragma unroll
  for (int q = 0; q < NSEG; ++q) {
    const int idx = threadIdx.x + q * NT;
    const int row = idx >> 2, c = idx & 3;
    const bool isa = FLEX ? row < tbm : q < ASEG;
    if (isa) {
      const int gr = m0 + row < p.M ? m0 + row : 0;     // clamped rows feed outputs never stored
      src[q] = p.A + (size_t)gr * p.lda;
      if constexpr (H3) ssc[q] = p.sa[gr];
    } else {
      const int r = row - tbm;
      const int gr = n0 + r < p.N ? n0 + r : 0;
      src[q] = p.B + (size_t)gr * p.ldb;
      if constexpr (H3) ssc[q] = p.sw[gr];
    }
    soff[q] = row * 64 + ((c ^ ((row >> 2) & 3)) << 4);
    sk[q] = c * 8;
  }
  struct Regs {
    f32x4 f[NSEG][2];                 // fp32 segments (A's only when !APL)
    u32x4 pa[APL ? ASEG : 1][3];      // A's three bf16 planes when APL
  };
  // every load is unconditional (k clamped in bounds); k >= kend is zeroed at the split
  auto gload = [&](Regs& ld, int k0) {
    if constexpr ((ABL & 1) != 0) k0 = kbeg + (k0 - kbeg) % (4 * BK);
#pragma unroll
    for (int q = 0; q < NSEG; ++q) {
      const int k = k0 + sk[q];
      if constexpr (APL) {
        if (q < ASEG) {
          const int r = (threadIdx.x + q * NT) >> 2;
          const size_t off = (size_t)min(m0 + r, p.M - 1) * p.K + (k < p.K ? k : 0);
#pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            ld.pa[q][pl] = *reinterpret_cast<const u32x4*>(p.apl + pl * p.apl_plane + off);
          continue;
        }
      }
      ld.f[q][0] = *reinterpret_cast<const f32x4*>(src[q] + (k < p.K ? k : 0));
      ld.f[q][1] = *reinterpret_cast<const f32x4*>(src[q] + (k + 4 < p.K ? k + 4 : 0));
    }
  };
  auto split_store = [&](const Regs& ld, int buf, int k0, int q, auto mask) {
    char* base = smem + buf * BUF;
    u32x4 o[3];
    if constexpr (APL) {
      if (q < ASEG) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          *reinterpret_cast<u32x4*>(base + pl * PLANE + soff[q]) = ld.pa[q][pl];
        return;
      }
    }
    if constexpr (H3) {
      u32x4 o2[2];
      if constexpr (decltype(mask)::value) {
        const int k = k0 + sk[q];
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        split2s(k < kend ? ld.f[q][0] : z, k + 4 < kend ? ld.f[q][1] : z, ssc[q], o2);
      } else {
        split2s(ld.f[q][0], ld.f[q][1], ssc[q], o2);
      }
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) *reinterpret_cast<u32x4*>(base + pl * PLANE + soff[q]) = o2[pl];
      return;
    }
    if constexpr (decltype(mask)::value) {
      const int k = k0 + sk[q];
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      split3(k < kend ? ld.f[q][0] : z, k + 4 < kend ? ld.f[q][1] : z, o);
    } else if constexpr ((ABL & 4) != 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[0][e] = __float_as_uint(ld.f[q][0][e]);
        o[1][e] = __float_as_uint(ld.f[q][1][e]);
        o[2][e] = o[0][e];
      }
    } else {
      split3(ld.f[q][0], ld.f[q][1], o);
    }
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<u32x4*>(base + pl * PLANE + soff[q]) = o[pl];
  };

  acc_t acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < NACC; ++r) acc[i][j][r] = 0.f;

  int aoff[TI], akey[TI], boff[TJ], bkey[TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i) {
    const int row = wm * WM + i * MF + (lane & (MF - 1));
    aoff[i] = row * 64;
    akey[i] = (row >> 2) & 3;
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int row = tbm + wn * WN + j * MF + (lane & (MF - 1));
    boff[j] = row * 64;
    bkey[j] = (row >> 2) & 3;
  }
  const int hk = MF == 32 ? lane >> 5 : lane >> 4;
  struct Frags { bf16x8 a[PL][TI], b[PL][TJ]; };
  auto read = [&](Frags& f, const char* S, int s) {
    const int c = MF == 32 ? 2 * s + hk : hk;
#pragma unroll
    for (int pl = 0; pl < PL; ++pl) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
        f.a[pl][i] = *reinterpret_cast<const bf16x8*>(S + pl * PLANE + aoff[i] + ((c ^ akey[i]) << 4));
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        f.b[pl][j] = *reinterpret_cast<const bf16x8*>(S + pl * PLANE + boff[j] + ((c ^ bkey[j]) << 4));
    }
  };
  auto mfma6 = [&](const Frags& f, int i, int j) {
    if constexpr ((ABL & 2) != 0) {
      acc[i][j][0] += __builtin_bit_cast(float, __builtin_bit_cast(u32x4, f.a[0][i])[0] ^
                                                    __builtin_bit_cast(u32x4, f.b[0][j])[0]);
      return;
    }
    acc_t t = acc[i][j];
    if constexpr (H3) {
      // fp16 terms (h = plane 0, l = plane 1), the dropped al*bl smallest; smallest first
      const f16x8 ah = __builtin_bit_cast(f16x8, f.a[0][i]), al = __builtin_bit_cast(f16x8, f.a[PL - 1][i]);
      const f16x8 bh = __builtin_bit_cast(f16x8, f.b[0][j]), bl = __builtin_bit_cast(f16x8, f.b[PL - 1][j]);
      t = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, t, 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, t, 0, 0, 0);
    } else if constexpr (MF == 32) {
      t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[0][i], f.b[2][j], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[2][i], f.b[0][j], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[1][i], f.b[1][j], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[0][i], f.b[1][j], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[1][i], f.b[0][j], t, 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[0][i], f.b[0][j], t, 0, 0, 0);
    } else {
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[0][i], f.b[2][j], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[2][i], f.b[0][j], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[1][i], f.b[1][j], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[0][i], f.b[1][j], t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[1][i], f.b[0][j], t, 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[0][i], f.b[0][j], t, 0, 0, 0);
    }
  };

  // One 32-k tile: tile kt + 2's global loads first, step 0's fragments and its first MFMA
  // group, step 1's fragment reads, then the remaining groups of both steps with tile kt + 1's
  // split + LDS stores (its registers were loaded one tile earlier) pinned between them, so the
  // conversion VALU issues while earlier MFMAs run.  `nxt` holds tile kt + 1, `fut` receives
  // tile kt + 2; MASK zeroes k >= kend (only the last tile can be partial).
  Frags fz;
  if constexpr ((ABL & 8) != 0) read(fz, smem, 0);
  constexpr int NG = TI * TJ;
  auto body = [&](auto mask, int kt, const Regs& nxt, Regs& fut) {
    const char* S = smem + (kt & 1) * BUF;
    if constexpr ((ABL & 8) == 0) gload(fut, kbeg + (kt + 2) * BK);
    Frags f0, f1;
    if constexpr ((ABL & 8) != 0) {          // MFMA-only ablation: no loads, split or LDS reads
      f0 = fz;
      f1 = fz;
#pragma unroll
      for (int g = 0; g < NSTEP * NG; ++g) {
        if (g < NG) mfma6(f0, g / TJ, g % TJ);
        else mfma6(f1, (g - NG) / TJ, (g - NG) % TJ);
      }
      __syncthreads();
      return;
    }
    read(f0, S, 0);
#pragma unroll
    for (int g = 0; g < NSTEP * NG; ++g) {
      if (g < NG) mfma6(f0, g / TJ, g % TJ);
      else mfma6(f1, (g - NG) / TJ, (g - NG) % TJ);
      if (g == 0 && NSTEP == 2) {
        __builtin_amdgcn_sched_barrier(0);
        read(f1, S, 1);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int q = 0; q < NSEG; ++q)
        if (q * NSTEP * NG / NSEG == g) {
          __builtin_amdgcn_sched_barrier(0);
          split_store(nxt, (kt + 1) & 1, kbeg + (kt + 1) * BK, q, mask);
          __builtin_amdgcn_sched_barrier(0);
        }
    }
    __syncthreads();
  };
  // MASK = false when every split's k range is whole 32-k tiles (K % 32 == 0, e.g. 3136): no
  // k >= kend selects in the split
  auto step = [&](int kt, const Regs& nxt, Regs& fut) {
    body(std::integral_constant<bool, MASK>{}, kt, nxt, fut);
  };

  HeadsRegs<TJ> hregs;                 // HEADS: the heads' weights, loaded before the loop
  if constexpr (HEADS) heads_preload<TJ>(p, n0 + wn * WN, hregs);
  const int nk = (kend - kbeg + BK - 1) / BK;
  Regs r0, r1;
  gload(r0, kbeg);
  gload(r1, kbeg + BK);
#pragma unroll
  for (int q = 0; q < NSEG; ++q) split_store(r0, 0, kbeg, q, std::integral_constant<bool, MASK>{});
  __syncthreads();
  for (int kt = 0; kt < nk; kt += 2) {
    step(kt, r1, r0);                 // tile kt + 1 in r1, tile kt + 2 -> r0
    if (kt + 1 < nk) step(kt + 1, r0, r1);
  }
  if constexpr (H3) {
    // back to the operands' units: acc(row, col) / (sa[row] sw[col]), powers of two (exact);
    // the inverses sit after the scales (p.sa + M, p.sw + N)
    float iw[TJ];
#pragma unroll
    for (int j = 0; j < TJ; ++j)
      iw[j] = p.sw[p.N + min(n0 + wn * WN + j * MF + (lane & (MF - 1)), p.N - 1)];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int r = 0; r < NACC; ++r) {
        const int row = m0 + wm * WM + i * MF + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const float ia = p.sa[p.M + min(row, p.M - 1)];
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j][r] *= ia * iw[j];
      }
  }
  if constexpr (HEADS) {     // the same epilogue as gemm_p3's: the same bits for the same planes
    static_assert(H3 && MF == 32 && WN == 64 && TI == 2, "heads epilogue: fp16 tiles");
    __syncthreads();         // the k loop's last LDS reads are done everywhere
    float* f = reinterpret_cast<float*>(smem);
    heads_tile_epilogue<TI, TJ, WGM, WGN>(p, acc, hregs, m0 + wm * WM, n0 + wn * WN, nt, sp, wm,
                                          wn, f + wave * (WM * 36), f + WGM * WGN * WM * 36);
    return;
  }
  tile_epilogue<MF, TI, TJ>(p, acc, m0 + wm * WM, n0 + wn * WN, sp,
                            reinterpret_cast<float*>(smem) + wave * (WM * 36));
}

template <int BM, int BN, int WGM, int WGN, bool MASK, int ABL = 0, bool APL = false, int MF = 32,
          bool H3 = false, bool HEADS = false>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_x3(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[x3_smem_bytes<BM, BN, WGM, WGN, MF, H3 ? 2 : 3>()];
  static_assert(!HEADS || x3_smem_bytes<BM, BN, WGM, WGN, MF, H3 ? 2 : 3>() >=
                              (WGM * WGN * 64 * 36 + WGM * (WGN - 1) * 64 * HEADS_TILE_SLOTS) * 4,
                "heads epilogue: stage + comb must fit");
  const int mt_n = (p.M + BM - 1) / BM, nt_n = (p.N + BN - 1) / BN;
  const int nwg = mt_n * nt_n * p.splits;
  int mt, nt, sp;
  tile_of(xcd_swizzle(blockIdx.x, nwg), mt_n, nt_n, mt, nt, sp);
  const int kbeg = sp * p.kc, kend = min(p.K, kbeg + p.kc);
  gemm_x3_body<BM, BN, WGM, WGN, MASK, ABL, APL, MF, false, H3, HEADS>(p, smem, mt, nt, sp, kbeg,
                                                                       kend);
}

// Stream-K form of gemm_x3 for grids whose tile count does not fill the chip in whole rounds
// (M ~ 600 .. 2,000 at N = 3,136: 100 .. 200 tiles of 256 x 128 on 256 CUs).  The tiles' k-steps
// (KT 32-k steps per tile, tiles in (mt fastest, nt) order) are cut into B contiguous ranges of
// equal cost, one per block: a block finishes the tail of one tile and starts the next.  A step
// costs 2 units, or SkPlan::wt for the last, partial row of m-tiles (1 = half: an experiment in
// which the waves of a tail tile whose rows all lie past M skipped their MFMAs -- measured
// slower, r03m: a tail step costs a full step at one MFMA wave per SIMD, and the blocks given
// more tail steps became the critical path; wt = 2 in the product).  A range that
// covers a whole tile writes C through the fused epilogue; a piece of a tile writes its raw
// partial sums to slab[piece] (piece = the block's index among the tile's blocks), and
// streamk_fixup4_kernel sums a split tile's pieces in piece order (deterministic) and runs the
// epilogue.
struct SkPlan {
  int mt_n, KT, wt;     // m-tiles, k-steps per tile, cost of a last-row step (1 or 2)
  long C;               // total cost units
  int B;                // blocks
};

// cost units before k-step k of tile t
__host__ __device__ __forceinline__ long sk_unit(const SkPlan& q, long t, int k) {
  const long full_rows_done = t / q.mt_n;            // the last-row tiles before t
  const long before = (t - full_rows_done) * 2L * q.KT + full_rows_done * (long)q.wt * q.KT;
  return before + (long)k * ((int)(t % q.mt_n) == q.mt_n - 1 ? q.wt : 2);
}
// the block that runs k-step k of tile t
__host__ __device__ __forceinline__ int sk_block(const SkPlan& q, long t, int k) {
  return (int)(sk_unit(q, t, k) * q.B / q.C);
}
// block b's first k-step (flattened t * KT + k): the first whose cost position u satisfies
// u * B / C >= b, i.e. u >= ceil(b * C / B)
__device__ __forceinline__ long sk_first(const SkPlan& q, int b) {
  const long u = ((long)b * q.C + q.B - 1) / q.B;
  const long G = (long)(q.mt_n - 1) * 2 * q.KT + (long)q.wt * q.KT;   // one n-tile column
  const long g = u / G, r = u - g * G;
  long mt, k;
  if (r < (long)(q.mt_n - 1) * 2 * q.KT) {
    mt = r / (2L * q.KT);
    k = (r - mt * 2L * q.KT + 1) / 2;
  } else {
    mt = q.mt_n - 1;
    k = (r - (long)(q.mt_n - 1) * 2 * q.KT + q.wt - 1) / q.wt;
  }
  return (g * q.mt_n + mt) * q.KT + k;       // k == KT rolls over to the next tile's step 0
}

template <int BM, int BN, int WGM, int WGN, bool MASK>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_x3_sk(GemmArgs p, SkPlan q) {
  __shared__ __attribute__((aligned(1024))) char smem[x3_smem_bytes<BM, BN, WGM, WGN>()];
  const int b = xcd_swizzle(blockIdx.x, q.B);
  const int KT = q.KT, mt_n = q.mt_n;
  long i0 = sk_first(q, b);
  const long i1 = b + 1 < q.B ? sk_first(q, b + 1) : (long)mt_n * ((p.N + BN - 1) / BN) * KT;
  while (i0 < i1) {
    const int t = (int)(i0 / KT);
    const int k0 = (int)(i0 - (long)t * KT);
    const int k1 = (int)min((long)KT, k0 + (i1 - i0));
    GemmArgs g = p;
    int sp = 0;
    if (k0 == 0 && k1 == KT) {
      g.splits = 1;                       // the whole tile: fused epilogue into C
    } else {
      g.splits = 2;                       // a piece: raw partials into slab[piece]
      sp = b - sk_block(q, t, 0);
    }
    gemm_x3_body<BM, BN, WGM, WGN, MASK>(g, smem, t % mt_n, t / mt_n, sp, 32 * k0,
                                         min(p.K, 32 * k1));
    i0 += k1 - k0;
    if (i0 < i1) __syncthreads();         // the next segment's prologue reuses the LDS
  }
}

#ifdef AZ_TUNING   // round 3's stream-K (gemm_x3_sk, gemm_p3_sk): A/B runs only
// Sums the pieces of every tile gemm_x3_sk / gemm_p3_sk split (slab[0 .. np), np = the tile's
// block count) and runs the epilogue on them; whole tiles were written by their block.  float4
// per lane.
__global__ __launch_bounds__(256) void streamk_fixup4_kernel(GemmArgs p, int BM, int BN, SkPlan q) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const int n4 = p.N >> 2;
  if (idx >= (long)p.M * n4) return;
  const int row = (int)(idx / n4), col = (int)(idx % n4) * 4;
  const long t = (long)(col / BN) * q.mt_n + row / BM;
  const int bf = sk_block(q, t, 0), bl = sk_block(q, t, q.KT - 1);
  if (bf == bl) return;
  const size_t plane = (size_t)p.M * p.N, off = (size_t)row * p.N + col;
  f32x4 v = *reinterpret_cast<const f32x4*>(p.slab + off);
  for (int s = 1; s <= bl - bf; ++s) {
    const f32x4 u = *reinterpret_cast<const f32x4*>(p.slab + s * plane + off);
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] += u[c];
  }
  epilogue_store4(p, row, col, v);
}

#endif

// The stream-K plan for a BM x BN tile grid on B blocks (host); weighted: the last row of
// m-tiles costs half when at most 128 of its rows are real (see gemm_x3_sk; not used).
static SkPlan sk_plan(int M, int N, int K, int BM, int BN, int B, bool weighted) {
  SkPlan q;
  q.mt_n = (M + BM - 1) / BM;
  q.KT = (K + 31) / 32;
  const int rows_last = M - (q.mt_n - 1) * BM;
  q.wt = weighted && rows_last < BM && rows_last <= BM / 2 ? 1 : 2;
  const long nt_n = (N + BN - 1) / BN;
  q.C = nt_n * ((long)(q.mt_n - 1) * 2 * q.KT + (long)q.wt * q.KT);
  q.B = B;
  return q;
}
// the most pieces any tile of plan q is cut into (slabs needed)
static int sk_max_pieces(const SkPlan& q, int N, int BN) {
  const long tiles = (long)q.mt_n * ((N + BN - 1) / BN);
  int mx = 1;
  for (long t = 0; t < tiles; ++t)
    mx = std::max(mx, sk_block(q, t, q.KT - 1) - sk_block(q, t, 0) + 1);
  return mx;
}

// ---------------------------------------------------------------------------------------------
// Cycled stream-K ("csk"): gemm_x3_sk with the tile order and the block -> XCD placement chosen
// for L2 reuse, and a short tile for a mostly padded last m-row.
//
// gemm_x3_sk walks the whole (tile, k) sequence with B equal ranges, so the blocks that need the
// same A panel (same m-tile) or W panel (same n-tile) at the same k run 16-36 k-steps apart: on
// one XCD that is ~25 MB of other loads in between, far beyond its 4 MB L2, and every k-slab of
// A and W is fetched again from the Infinity Cache by each of its consumers (980 MB per dispatch
// at the self-play shapes against ~86 MB algorithmic, L2 hit 0.29; r03x).
//
// Here the tiles are grouped into CYCLES, macro tiles of am x an tiles (slot f = fm + am * fn
// holds tile (cm * am + fm, cn * an + fn) of cycle (cm, cn)), and every cycle's am * an * KT
// k-steps are cut the same way into b equal ranges, one per block.  Block r of every cycle thus
// runs the same (slot, k) sequence at the same time: in phase.  Logical block ids run r-major,
// cycle fastest, so the in-phase blocks of all cycles are neighbours on one XCD; at slot f they
// hold a 2-D set of tiles (every cm, every cn), in which each A k-slab is read by the cycles
// along n and each W k-slab by the cycles along m at the same k, out of that XCD's L2.
// Measured (tools/csk_probe.py, profiles/r04a_csk.jsonl): M = 1,536 with am x an = 1 x 5 on 240
// blocks runs 62 steps per block in 200 us, gemm_x3_sk 58 steps on 256 blocks in 203 us:
// 3.22 vs 3.49 us per step.
//
// A last m-row with at most 128 real rows runs 128 x 256 tiles instead of mostly padded
// 256 x 128 ones (the FLEX body: the same waves, MFMAs and LDS image, half the rows, twice the
// columns): half the steps, in cycles of its own (`at` wide tiles each, bt blocks per cycle).
// Pieces of a tile (a slot split between blocks) write raw partials to slab[r - first block of
// the slot] and csk_fixup4_kernel sums them in that order: deterministic.
struct CskPlan {
  int mt_n, nt_n, KT;  // 256 x 128 tile grid, 32-k steps per tile
  int am, an;          // macro tile of a full cycle (am | full m-rows, an | nt_n)
  int cm;              // cycles along m (full rows / am); along n: nt_n / an
  int tail;            // 1: the last m-row runs 128 x 256 tiles
  int at, ct;          // wide tiles per tail cycle, tail cycles (at * ct = ceil(N / 256))
  int bf, bt;          // blocks per full / tail cycle
  int Cf, Ct;          // full / tail cycles
  int B;               // blocks: Cf * bf + Ct * bt
};

// the block of a b-block cycle of W steps that runs cycle step u (ranges [r W / b, (r+1) W / b))
__host__ __device__ __forceinline__ int csk_block_of(int u, int b, int W) {
  return ((u + 1) * b - 1) / W;
}

template <int BM, int BN, int WGM, int WGN, bool H3 = false, int NBUF = 2>
constexpr int p3_smem_bytes() {
  constexpr int NW = WGM * WGN, WM = BM / WGM;
  constexpr int BUF = (H3 ? 2 : 3) * (BM + BN) * 64, STAGE = NW * WM * 36 * 4;
  return NBUF * BUF > STAGE ? NBUF * BUF : STAGE;
}

#ifdef AZ_P3_STAMPS
// timing-experiment library only (tools/p3_stamp_probe.py): lane 0 of every wave of a gemm_p3
// block records s_memrealtime (100 MHz) at fixed points -- [block][wave][72]: 0 body start,
// 1 prologue issued, 2 + 2 kt before stage kt's wait, 3 + 2 kt after its barrier, 66 loop end,
// 67 epilogue end, 68 / 69 s_memtime at start / end, 70 HW_ID, 71 XCC_ID
__device__ unsigned long long* g_p3_stamps;
#endif
// gemm_p3_body (below): the tile on operands already split into planes, LDS-DMA only
template <int BM, int BN, int WGM, int WGN, bool H3 = false, bool FLEX = false, int NBUF = 2,
          int ABL = 0, bool HEADS = false>
__device__ __forceinline__ void gemm_p3_body(const GemmArgs& p, char* smem, int mt, int nt,
                                             int sp, int kbeg, int kend, int bma = BM);

// P2: the fp16 form on pre-split planes (p.apl: A's two planes from h3_split_rows_kernel, p.bpl:
// W's, cached per weight generation), every stage global -> LDS by LDS-DMA; same products in the
// same order as the in-tile split, so the same bits.
// RING (P2 only): the pre-split tile's LDS-DMA ring depth, 3 in the product (two stages in
// flight: the whole-line stage fill then takes 0.60 us per stage against the MFMA's ~0.73)
template <bool MASK, bool H3, bool P2 = false, bool HEADS = false, int RING = 3>
__global__ __launch_bounds__(512) void gemm_x3_csk(GemmArgs p, CskPlan q) {
  static_assert(!P2 || (H3 && !MASK), "P2: the fp16 form on whole 32-k tiles");
  static_assert(!HEADS || (H3 && !MASK), "HEADS: the fp16 form on whole 32-k tiles");
  constexpr int SMEM = P2 ? p3_smem_bytes<256, 128, 4, 2, true, RING>()
                          : x3_smem_bytes<256, 128, 4, 2, 32, H3 ? 2 : 3>();
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  const int L = xcd_swizzle(blockIdx.x, q.B);
  int r, b, am, an, mt0, nt0, bma;
  if (L < q.Cf * q.bf) {                  // r-major, cycle fastest: in-phase blocks adjacent
    r = L / q.Cf;
    const int c = L - r * q.Cf, cn = c / q.cm;
    b = q.bf;
    am = q.am;
    an = q.an;
    mt0 = (c - cn * q.cm) * q.am;
    nt0 = cn * q.an;
    bma = 256;
  } else {
    const int l = L - q.Cf * q.bf;
    r = l / q.Ct;
    b = q.bt;
    am = 1;
    an = q.at;
    mt0 = (q.mt_n - 1) * 2;               // in 128-row units
    nt0 = (l - r * q.Ct) * q.at;          // in 256-column units
    bma = 128;
  }
  const int W = am * an * q.KT;           // <= 256 x 98 steps: int arithmetic throughout
  int i0 = r * W / b;
  const int i1 = (r + 1) * W / b;
  while (i0 < i1) {
    const int f = i0 / q.KT;
    const int k0 = i0 - f * q.KT;
    const int k1 = min(q.KT, k0 + (i1 - i0));
    GemmArgs g = p;
    int sp = 0;
    if (k0 == 0 && k1 == q.KT) {
      g.splits = 1;                       // the whole tile: fused epilogue into C
    } else {
      g.splits = 2;                       // a piece: raw partials into slab[piece]
      sp = r - csk_block_of(f * q.KT, b, W);
    }
    // HEADS: every piece leaves its heads' dot products in slot (column block, piece sp)
    const int fn = f / am;
    int mt_i = mt0 + (f - fn * am), bma_i = bma;   // opaque per segment: keeps the body's
    asm volatile("" : "+s"(mt_i), "+s"(bma_i));    // address setup in the loop (hoisted, it spills)
    if constexpr (P2)
      gemm_p3_body<256, 128, 4, 2, true, true, RING, 0, HEADS>(g, smem, mt_i, nt0 + fn, sp,
                                                              32 * k0, min(p.K, 32 * k1), bma_i);
    else
      gemm_x3_body<256, 128, 4, 2, MASK, 0, false, 32, true, H3, HEADS>(
          g, smem, mt_i, nt0 + fn, sp, 32 * k0, min(p.K, 32 * k1), bma_i);
    i0 += k1 - k0;
    if (i0 < i1) __syncthreads();         // the next segment's prologue reuses the LDS
  }
}

// Sums the pieces of every tile gemm_x3_csk split, in piece (= k) order, and runs the epilogue;
// whole tiles were written by their block.  float4 per lane.
__global__ __launch_bounds__(256) void csk_fixup4_kernel(GemmArgs p, CskPlan q) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const int n4 = p.N >> 2;
  if (idx >= (long)p.M * n4) return;
  const int row = (int)(idx / n4), col = (int)(idx % n4) * 4;
  const int mt = row >> 8;
  const bool tail = q.tail && mt == q.mt_n - 1;
  int f, b, W;
  if (tail) {
    f = (col >> 8) % q.at;
    b = q.bt;
    W = q.at * q.KT;
  } else {
    f = mt % q.am + q.am * ((col >> 7) % q.an);
    b = q.bf;
    W = q.am * q.an * q.KT;
  }
  const int bf = csk_block_of(f * q.KT, b, W), bl = csk_block_of((f + 1) * q.KT - 1, b, W);
  if (bf == bl) return;
  const size_t plane = (size_t)p.M * p.N, off = (size_t)row * p.N + col;
  f32x4 v = *reinterpret_cast<const f32x4*>(p.slab + off);
  for (int s = 1; s <= bl - bf; ++s) {
    const f32x4 u = *reinterpret_cast<const f32x4*>(p.slab + s * plane + off);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] += u[e];
  }
  epilogue_store4(p, row, col, v);
}

static int csk_max_pieces(const CskPlan& q) {
  int mx = 1;
  for (int t = 0; t < 2; ++t) {
    const int b = t ? q.bt : q.bf, per = t ? q.at : q.am * q.an;
    if (b <= 0 || per <= 0) continue;
    const int W = per * q.KT;
    for (int f = 0; f < per; ++f)
      mx = std::max(mx, csk_block_of((f + 1) * q.KT - 1, b, W) - csk_block_of(f * q.KT, b, W) + 1);
  }
  return mx;
}

// Fills the derived fields of a plan from (am, an, bf) and the tail's (at, bt); false if the
// plan does not tile this M x N or needs more than `cus` blocks.
static bool csk_make(int M, int N, int K, int cus, int am, int an, int bf, int at, int bt,
                     CskPlan& q) {
  q = CskPlan{};
  q.mt_n = (M + 255) / 256;
  q.nt_n = (N + 127) / 128;
  q.KT = (K + 31) / 32;
  const int ntw = (N + 255) / 256, rows_last = M - (q.mt_n - 1) * 256;
  q.tail = at > 0 ? 1 : 0;
  if (q.tail && (q.mt_n < 2 || rows_last > 128 || ntw % at || bt < 1)) return false;
  const int rows_full = q.mt_n - q.tail;
  if (am < 1 || an < 1 || bf < 1 || rows_full % am || q.nt_n % an) return false;
  q.am = am;
  q.an = an;
  q.cm = rows_full / am;
  q.bf = bf;
  q.Cf = q.cm * (q.nt_n / an);
  q.at = at;
  q.ct = q.tail ? ntw / at : 0;
  q.bt = q.tail ? bt : 0;
  q.Ct = q.ct;
  q.B = q.Cf * q.bf + q.Ct * q.bt;
  return q.B >= 1 && q.B <= cus;
}

// Chooses the plan for an M x N x K GEMM on `cus` CUs: every (am, an) macro tile and block count
// bf for the full rows, the fastest (at, bt) for a wide-tile tail row in the CUs left.  A cycle
// of `per` tiles on b blocks takes ceil(per KT / b) steps (the wide tile's step costs what the
// 256 x 128 one's does), the launch the slowest cycle.  The per-step cost grows with the k-slab
// bytes each block fetches past the XCD's L2: (ua * 32 KB + un * 16 KB) / (ua * un) for the ua
// m-tiles x un n-tiles that the in-phase blocks on one XCD hold at a slot (an estimate; 48 KB
// when nothing is shared).  Fitted to tools/csk_probe.py at M = 1,536 .. 4,096
// (profiles/r04a_csk.jsonl): a step costs ~1 + miss_cost x (KB - 9) / 39 relative to a fully
// shared one, miss_cost ~0.1 (3.16 vs 3.53 us per step at M = 1,536, 2.80 vs 3.08 at 4,096).
constexpr double CSK_MISS_COST = 0.12;
static bool csk_plan(int M, int N, int K, int cus, double miss_cost, CskPlan& out) {
  const int mt_n = (M + 255) / 256, nt_n = (N + 127) / 128, KT = (K + 31) / 32;
  const int ntw = (N + 255) / 256;
  const int rows_last = M - (mt_n - 1) * 256;
  const int tail = mt_n > 1 && rows_last <= 128 ? 1 : 0;
  const int rows_full = mt_n - tail;
  double best = 1e30;
  bool found = false;
  for (int am = 1; am <= rows_full; ++am) {
    if (rows_full % am) continue;
    for (int an = 1; an <= nt_n; ++an) {
      if (nt_n % an) continue;
      const int Cm = rows_full / am, Cn = nt_n / an, Cf = Cm * Cn;
      const int W = am * an * KT;
      // in-phase cycles on one XCD: up to 32 / (cycles per XCD) of them, m-fastest
      const int on_xcd = std::min(Cf, 32);
      const int ua = std::min(Cm, on_xcd), un = (on_xcd + Cm - 1) / Cm;
      const double miss_kb = (ua * 32.0 + un * 16.0) / (double)(ua * un);
      const double step = 1.0 + miss_cost * std::max(0.0, std::min(1.0, (miss_kb - 9.0) / 39.0));
      for (int bf = 1; Cf * bf <= cus && W / bf >= 8; ++bf) {   // >= 8 steps per block
        const int tf = (W + bf - 1) / bf;
        int at = 0, bt = 0, tt = 0;
        if (tail) {
          // the tail row: per cycle width, the fewest blocks that finish within tf, else all
          // the CUs left; the earliest finish, ties to the narrower cycles (more in phase)
          const int room = cus - Cf * bf;
          int tt_best = 1 << 30;
          for (int a = 1; a <= ntw; ++a) {
            if (ntw % a || room < ntw / a) continue;
            const int ct = ntw / a, Wt = a * KT;
            const int b = std::min(room / ct, (Wt + tf - 1) / tf);
            const int t = std::max(tf, (Wt + b - 1) / b);
            if (t < tt_best) {
              tt_best = t;
              at = a;
              bt = b;
            }
          }
          if (!at) break;
          tt = tt_best;
        }
        const double cost = std::max(tf, tt) * step;
        CskPlan q;
        if (cost < best - 1e-9 && csk_make(M, N, K, cus, am, an, bf, at, bt, q)) {
          best = cost;
          out = q;
          found = true;
        }
      }
    }
  }
  return found;
}

// csk_plan memoised per shape: the search walks up to ~10^4 (am, an, bf, at) candidates, up to
// ~1 ms of host time per call.  A plan depends on M only through its 256-row tile count and
// whether the last tile row has <= 128 rows (csk_plan / csk_make keep no M), so that pair is the
// key: the lock-step self-play's shrinking batches (a new M nearly every round once games end)
// then hit the memo instead of re-running the search for every M (~1 ms of host time per round,
// measured in tools/sp_pipeline_probe.py's timeline)
static bool csk_plan_cached(int M, int N, int K, int cus, double miss_cost, CskPlan& out) {
  struct Key {
    int M, N, K, cus;
    double miss;
    bool operator==(const Key& o) const {
      return M == o.M && N == o.N && K == o.K && cus == o.cus && miss == o.miss;
    }
  };
  struct Hash {
    size_t operator()(const Key& k) const {
      return std::hash<long long>()(((long long)k.M << 40) ^ ((long long)k.N << 20) ^ k.K ^
                                    ((long long)k.cus << 52));
    }
  };
  static std::mutex mu;
  static std::unordered_map<Key, std::pair<bool, CskPlan>, Hash> memo;
  const int mt_n = (M + 255) / 256, rows_last = M - (mt_n - 1) * 256;
  const int mkey = 2 * mt_n + (mt_n > 1 && rows_last <= 128 ? 1 : 0);   // the plan's M classes
  const Key key{mkey, N, K, cus, miss_cost};
  {
    std::lock_guard<std::mutex> lk(mu);
    const auto it = memo.find(key);
    if (it != memo.end()) {
      out = it->second.second;
      return it->second.first;
    }
  }
  CskPlan q{};
  const bool ok = csk_plan(M, N, K, cus, miss_cost, q);
  std::lock_guard<std::mutex> lk(mu);
  if (memo.size() > 65536) memo.clear();
  memo.emplace(key, std::make_pair(ok, q));
  out = q;
  return ok;
}

// gemm_x3's fp16 form on operands that are ALREADY split ("p3", the product's P2 GEMM): A's and
// W's row-scaled values as two fp16 planes each in the p2_chunk layout of az_x3.h (A from
// h3_split_rows_kernel / the trunk / the fused split-K reduce, W cached per weight generation),
// K % 32 == 0.  Nothing is converted in the tile: each 32-k stage ((BM + BN) rows x 128 B = 48 KB
// for 256 x 128) goes global -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KB = 8 whole 128-B
// lines per wave-instruction, no VGPR round trip, no VALU, no ds_write), in a ring of NBUF
// stages with one raw barrier per stage.  The LDS image is [row][8 units of 16 B], unit u stored
// at slot u ^ ((row >> 1) & 7) (the swizzle applied on the global address, since a DMA's LDS
// destination is lane-linear).  Three fp16 products per step (ah bl, al bh, ah bh), the
// accumulators unscaled by 1 / (sa sw) before the epilogue: the same products in the same order
// as gemm_x3's in-tile fp16 split, so the same bits for the same split-K partition.

// FLEX (the cycled stream-K tail): bma = 256 (256 x 128 tile) or 128 (128 x 256), as gemm_x3_body.
// NBUF = 3: a three-stage ring (stage kt + 2 issued while stage kt computes), one barrier per
// stage as with two; the fp16 256 x 128 ring is 3 x 48 KB.
// ABL (tuning-build timing ablations, results wrong by design): 1 = no epilogue stores,
// 2 = no MFMAs, 4 = no DMA (stale LDS)
template <int BM, int BN, int WGM, int WGN, bool H3, bool FLEX, int NBUF, int ABL, bool HEADS>
__device__ __forceinline__ void gemm_p3_body(const GemmArgs& p, char* smem, int mt, int nt,
                                             int sp, int kbeg, int kend, int bma) {
  static_assert(NBUF == 2 || NBUF == 3, "p3 ring: 2 or 3 stages");
  static_assert(!FLEX || (BM == 256 && BN == 128 && WGM == 4 && WGN == 2), "FLEX: 256 x 128");
  static_assert(H3, "p3: the fp16 form's two planes (p2_chunk layout)");
  constexpr int PL = 2;
  constexpr int BK = 32;
  constexpr int NT = 64 * WGM * WGN, NW = NT / 64;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TI = WM / 32, TJ = WN / 32;
  constexpr int ROWS = BM + BN;
  constexpr int BUF = ROWS * 128;                  // [ROWS][2 planes x 32 k]: 128 B per row
  constexpr int PIECES = ROWS / 8;                 // 1-KB DMA pieces per stage, 8 rows each
  static_assert(ROWS % 8 == 0 && PIECES % NW == 0 && TI >= 1 && TJ >= 1, "bad p3 tile");
  constexpr int PPW = PIECES / NW;
  const int tbm = FLEX ? bma : BM, tbn = FLEX ? BM + BN - bma : BN;
  const int wgn = FLEX ? tbn / WN : WGN;
  const int m0 = mt * tbm, n0 = nt * tbn;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / wgn, wn = wave % wgn;

  // piece q * NW + wave covers image rows 8 piece .. + 7, each row one whole 128-B line of the
  // p2_chunk layout (8 units of 16 B: plane 0's four k chunks, then plane 1's); lane l lands at
  // byte 16 l of the piece: row 8 piece + (l >> 3), unit slot l & 7 = logical unit
  // (l & 7) ^ key(row), key = (row >> 1) & 7 -- any 16 rows r..r+15 (r % 16 == 0) then put one
  // unit on 16 distinct 16-B slots of the 256-B bank row, so the fragment reads are conflict-free
  const unsigned short* src[PPW];
#pragma unroll
  for (int q = 0; q < PPW; ++q) {
    const int r = (q * NW + wave) * 8 + (lane >> 3);
    const int u = (lane & 7) ^ ((r >> 1) & 7);
    if (r < tbm) {
      const int gr = min(m0 + r, p.M - 1);
      src[q] = p.apl + (size_t)gr * 2 * p.K + 8 * u;
    } else {
      const int gr = min(n0 + r - tbm, p.N - 1);
      src[q] = p.bpl + (size_t)gr * 2 * p.K + 8 * u;
    }
  }
  auto issue_one = [&](int buf, int k0, int q) {   // k0 % 32 == 0: step k0 / 32 at element 2 k0
    if constexpr ((ABL & 4) != 0) return;
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(src[q] + 2 * k0),
        (__attribute__((address_space(3))) void*)(smem + buf * BUF + (q * NW + wave) * 1024),
        16, 0, 0);
  };
  auto issue = [&](int buf, int k0) {
#pragma unroll
    for (int q = 0; q < PPW; ++q) issue_one(buf, k0, q);
  };

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  int aoff[TI], akey[TI], boff[TJ], bkey[TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i) {
    const int row = wm * WM + i * 32 + (lane & 31);
    aoff[i] = row * 128;
    akey[i] = (row >> 1) & 7;
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int row = tbm + wn * WN + j * 32 + (lane & 31);
    boff[j] = row * 128;
    bkey[j] = (row >> 1) & 7;
  }
  const int hk = lane >> 5;
  struct Frags { bf16x8 a[PL][TI], b[PL][TJ]; };
  auto read = [&](Frags& f, const char* S, int s) {
    const int c = 2 * s + hk;          // k chunk of this half of the wave; unit 4 pl + c
#pragma unroll
    for (int pl = 0; pl < PL; ++pl) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
        f.a[pl][i] = *reinterpret_cast<const bf16x8*>(S + aoff[i] + (((4 * pl + c) ^ akey[i]) << 4));
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        f.b[pl][j] = *reinterpret_cast<const bf16x8*>(S + boff[j] + (((4 * pl + c) ^ bkey[j]) << 4));
    }
  };
  auto mfma6 = [&](const Frags& f, int i, int j) {
    f32x16 t = acc[i][j];
    if constexpr ((ABL & 2) != 0) {       // keep the fragment reads live, no MFMA
      acc[i][j][0] += __builtin_bit_cast(float, __builtin_bit_cast(u32x4, f.a[0][i])[0]) +
                      __builtin_bit_cast(float, __builtin_bit_cast(u32x4, f.b[0][j])[0]) +
                      __builtin_bit_cast(float, __builtin_bit_cast(u32x4, f.a[PL - 1][i])[1]) +
                      __builtin_bit_cast(float, __builtin_bit_cast(u32x4, f.b[PL - 1][j])[1]);
      return;
    }
    if constexpr (H3) {
      const f16x8 ah = __builtin_bit_cast(f16x8, f.a[0][i]), al = __builtin_bit_cast(f16x8, f.a[PL - 1][i]);
      const f16x8 bh = __builtin_bit_cast(f16x8, f.b[0][j]), bl = __builtin_bit_cast(f16x8, f.b[PL - 1][j]);
      t = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, t, 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, t, 0, 0, 0);
      return;
    }
    t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[0][i], f.b[PL - 1][j], t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[PL - 1][i], f.b[0][j], t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[1][i], f.b[1][j], t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[0][i], f.b[1][j], t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[1][i], f.b[0][j], t, 0, 0, 0);
    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[0][i], f.b[0][j], t, 0, 0, 0);
  };
  constexpr int NG = TI * TJ;
  HeadsRegs<TJ> hregs;                 // HEADS: the heads' weights, loaded before the loop
  if constexpr (HEADS) heads_preload<TJ>(p, n0 + wn * WN, hregs);
  const int nk = (kend - kbeg) / BK;
#ifdef AZ_P3_STAMPS
  unsigned long long* const stp = (g_p3_stamps && !FLEX && lane == 0)
                                      ? g_p3_stamps + ((size_t)blockIdx.x * NW + wave) * 72
                                      : nullptr;
  auto stamp = [&](int slot) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if (stp) stp[slot] = t;
  };
  if (stp) {
    stp[68] = __builtin_amdgcn_s_memtime();
    stp[70] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));
    stp[71] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((32 - 1) << 11));
  }
  stamp(0);
#else
  auto stamp = [](int) {};
#endif
  if (nk > 0) issue(0, kbeg);
  if (NBUF == 3 && nk > 1) issue(1, kbeg + BK);
  stamp(1);
  int cur = 0;             // kt % NBUF
  for (int kt = 0; kt < nk; ++kt) {
    if (kt < 32) stamp(2 + 2 * kt);
    if (NBUF == 3 && kt + 1 < nk) wait_vm<PPW>();   // stage kt + 1's pieces may still fly
    else wait_vm<0>();     // this wave's pieces of stage kt have landed
    lds_barrier();         // ... everyone's; and every wave is done reading stage kt - 1
    if (kt < 32) stamp(3 + 2 * kt);
    // stage kt + NBUF - 1 goes into stage kt - 1's buffer, free since the barrier.  Its pieces
    // leave one by one between this stage's MFMA groups (piece q after group 2 NG q / PPW): all
    // 48 of a CU's pieces issued together at the barrier kept both waves of every SIMD waiting
    // for memory-issue room while their MFMA pipe idled
    const bool more = kt + NBUF - 1 < nk;
    const int nb = cur == 0 ? NBUF - 1 : cur - 1;   // (kt + NBUF - 1) % NBUF
    const int kn = kbeg + (kt + NBUF - 1) * BK;
    const char* S = smem + cur * BUF;
    cur = cur + 1 == NBUF ? 0 : cur + 1;
    Frags f0, f1;
    read(f0, S, 0);
#pragma unroll
    for (int g = 0; g < 2 * NG; ++g) {
      if (g < NG) mfma6(f0, g / TJ, g % TJ);
      else mfma6(f1, (g - NG) / TJ, (g - NG) % TJ);
      if (g == 0) {
        __builtin_amdgcn_sched_barrier(0);
        read(f1, S, 1);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int q = 0; q < PPW; ++q)
        if (q * 2 * NG / PPW == g && more) {
          __builtin_amdgcn_sched_barrier(0);
          issue_one(nb, kn, q);
          __builtin_amdgcn_sched_barrier(0);
        }
    }
  }
  stamp(66);
  if constexpr (H3) {
    float iw[TJ];
#pragma unroll
    for (int j = 0; j < TJ; ++j)
      iw[j] = p.sw[p.N + min(n0 + wn * WN + j * 32 + (lane & 31), p.N - 1)];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const float ia = p.sa[p.M + min(row, p.M - 1)];
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j][r] *= ia * iw[j];
      }
    __syncthreads();           // the epilogue's staging reuses the stage buffers
  }
  if constexpr ((ABL & 1) != 0) {        // no stores unless a sentinel appears (every
    float t = 0.f;                         // accumulator stays live: no MFMA is dead code)
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) t += acc[i][j][r];
    if (t == 12345.f) p.C[0] = t;
    return;
  }
  if constexpr (HEADS) {
    static_assert(H3 && WN == 64 && TI == 2, "heads epilogue: the P2 tiles");
    float* f = reinterpret_cast<float*>(smem);
    heads_tile_epilogue<TI, TJ, WGM, WGN>(p, acc, hregs, m0 + wm * WM, n0 + wn * WN, nt, sp, wm,
                                          wn, f + wave * (WM * 36), f + NW * WM * 36);
#ifdef AZ_P3_STAMPS
    stamp(67);
    if (stp) stp[69] = __builtin_amdgcn_s_memtime();
#endif
    return;
  }
  tile_epilogue<32, TI, TJ>(p, acc, m0 + wm * WM, n0 + wn * WN, sp,
                            reinterpret_cast<float*>(smem) + wave * (WM * 36));
#ifdef AZ_P3_STAMPS
  stamp(67);
  if (stp) stp[69] = __builtin_amdgcn_s_memtime();
#endif
}

template <int BM, int BN, int WGM, int WGN, bool H3 = false, int NBUF = 2, int ABL = 0,
          bool HEADS = false>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_p3(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[p3_smem_bytes<BM, BN, WGM, WGN, H3, NBUF>()];
  static_assert(!HEADS || p3_smem_bytes<BM, BN, WGM, WGN, H3, NBUF>() >=
                              (WGM * WGN * 64 * 36 + WGM * (WGN - 1) * 64 * HEADS_TILE_SLOTS) * 4,
                "heads epilogue: stage + comb must fit the stage buffers");
  const int mt_n = (p.M + BM - 1) / BM, nt_n = (p.N + BN - 1) / BN;
  const int nwg = mt_n * nt_n * p.splits;
  int mt, nt, sp;
  tile_of(xcd_swizzle(blockIdx.x, nwg), mt_n, nt_n, mt, nt, sp);
  const int kbeg = sp * p.kc, kend = min(p.K, kbeg + p.kc);
  gemm_p3_body<BM, BN, WGM, WGN, H3, false, NBUF, ABL, HEADS>(p, smem, mt, nt, sp, kbeg, kend,
                                                              BM);
}

// gemm_x3 as a two-group ping-pong ("x3pp").  The timing ablations of gemm_x3 (tools/gemm_sweep.py
// x3, tuning tiles 7-11) showed its MFMAs and its other work do not overlap: M = 4096 takes
// 518 us, 219 us of it without any MFMA and ~200 us of MFMA alone; the loads are not the
// bound (L2-resident loads: 503 us).  Both waves of a SIMD reach the same phase together after
// every barrier.  Here the 8 waves (4 x 2, 64 x 64 each) form two groups of one wave per SIMD,
// G0 = waves 0-3 and G1 = waves 4-7, and each 32-k tile t is two phases split by block
// barriers:
//   P1(t): G0 runs tile t's 48 MFMAs from fragments already in registers; G1 reads tile t's
//          fragments, splits its share of tile t + 1 into LDS and issues its loads for t + 2;
//   P2(t): G1 runs tile t's MFMAs; G0 reads tile t + 1's fragments, splits its share of tile
//          t + 2 and issues its loads for t + 3.
// So each SIMD's MFMA pipe alternates between its two waves while the other one does the LDS /
// VALU / load work.  LDS: the planes of tiles t and t + 1 (the same double-buffered image as
// gemm_x3); tile t + 2's shares overwrite tile t's buffer only after both groups have read it.
// Same split and product order as gemm_x3.
template <int BM, int BN, bool MASK>
__global__ __launch_bounds__(512) void gemm_x3pp(GemmArgs p) {
  constexpr int BK = 32, WGM = 4, WGN = 2, NT = 512;
  constexpr int WM = BM / WGM, WN = BN / WGN, TI = WM / 32, TJ = WN / 32;
  constexpr int ASEG = BM * 4 / NT, BSEG = BN * 4 / NT, NSEG = ASEG + BSEG;
  static_assert(TI >= 1 && TJ >= 1 && ASEG >= 1 && BSEG >= 1 && (BM * 4) % NT == 0 &&
                (BN * 4) % NT == 0, "bad x3pp tile");
  constexpr int PLANE = (BM + BN) * 64, BUF = 3 * PLANE;
  constexpr int STAGE = 8 * WM * 36 * 4;
  constexpr int SMEM = 2 * BUF > STAGE ? 2 * BUF : STAGE;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const int mt_n = (p.M + BM - 1) / BM, nt_n = (p.N + BN - 1) / BN;
  const int nwg = mt_n * nt_n * p.splits;
  const int bid = xcd_swizzle(blockIdx.x, nwg);
  const int mt = bid % mt_n, nt = (bid / mt_n) % nt_n, sp = bid / (mt_n * nt_n);
  const int m0 = mt * BM, n0 = nt * BN;
  const int kbeg = sp * p.kc, kend = min(p.K, kbeg + p.kc);
  const int nk = (kend - kbeg + BK - 1) / BK;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const bool g1 = __builtin_amdgcn_readfirstlane(wave) >= 4;

  const float* src[NSEG];
  int soff[NSEG], sk[NSEG];
#pragma unroll
  for (int q = 0; q < NSEG; ++q) {
    const bool isa = q < ASEG;
    const int idx = threadIdx.x + (isa ? q : q - ASEG) * NT;
    const int r = idx >> 2, c = idx & 3;
    if (isa) {
      const int gr = m0 + r < p.M ? m0 + r : 0;     // clamped rows feed outputs never stored
      src[q] = p.A + (size_t)gr * p.lda;
    } else {
      const int gr = n0 + r < p.N ? n0 + r : 0;
      src[q] = p.B + (size_t)gr * p.ldb;
    }
    const int row = isa ? r : BM + r;
    soff[q] = row * 64 + ((c ^ ((row >> 2) & 3)) << 4);
    sk[q] = c * 8;
  }
  f32x4 ld[NSEG][2];
  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < NSEG; ++q) {
      const int k = k0 + sk[q];
      ld[q][0] = *reinterpret_cast<const f32x4*>(src[q] + (k < p.K ? k : 0));
      ld[q][1] = *reinterpret_cast<const f32x4*>(src[q] + (k + 4 < p.K ? k + 4 : 0));
    }
  };
  // buffer indices are compile-time (B = 0 / 1) so the LDS addresses are a few per-lane bases
  // plus immediate offsets, not a hoisted copy per buffer
  auto split_store = [&](auto B, int k0) {
    char* base = smem + decltype(B)::value * BUF;
#pragma unroll
    for (int q = 0; q < NSEG; ++q) {
      u32x4 o[3];
      if constexpr (MASK) {
        const int k = k0 + sk[q];
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        split3(k < kend ? ld[q][0] : z, k + 4 < kend ? ld[q][1] : z, o);
      } else {
        split3(ld[q][0], ld[q][1], o);
      }
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        *reinterpret_cast<u32x4*>(base + pl * PLANE + soff[q]) = o[pl];
    }
  };

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  int aoff[TI], akey[TI], boff[TJ], bkey[TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i) {
    const int row = wm * WM + i * 32 + (lane & 31);
    aoff[i] = row * 64;
    akey[i] = (row >> 2) & 3;
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int row = BM + wn * WN + j * 32 + (lane & 31);
    boff[j] = row * 64;
    bkey[j] = (row >> 2) & 3;
  }
  const int hk = lane >> 5;
  bf16x8 fa[2][3][TI], fb[2][3][TJ];        // both k steps of one tile
  auto read = [&](auto B) {
    const char* S = smem + decltype(B)::value * BUF;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 2 * s + hk;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
          fa[s][pl][i] = *reinterpret_cast<const bf16x8*>(S + pl * PLANE + aoff[i] + ((c ^ akey[i]) << 4));
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          fb[s][pl][j] = *reinterpret_cast<const bf16x8*>(S + pl * PLANE + boff[j] + ((c ^ bkey[j]) << 4));
      }
    }
  };
  auto mfma_tile = [&]() {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          f32x16 t = acc[i][j];
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][0][i], fb[s][2][j], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][2][i], fb[s][0][j], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][1][i], fb[s][1][j], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][0][i], fb[s][1][j], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][1][i], fb[s][0][j], t, 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][0][i], fb[s][0][j], t, 0, 0, 0);
        }
  };
  // memory phase of a wave: its fragments of the tile in buffer RB, its share of tile wr
  // (registers loaded one tile earlier) into buffer 1 - RB, then its loads for tile wr + 1
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  auto mem_phase = [&](auto RB, int wr) {
    using WB = std::integral_constant<int, 1 - decltype(RB)::value>;
    read(RB);
    split_store(WB{}, kbeg + wr * BK);
    gload(kbeg + (wr + 1) * BK);
  };
  // one tile t held in buffer E = t & 1: G0's MFMAs while G1 reads it and writes tile t + 1,
  // then G1's MFMAs while G0 reads tile t + 1 and writes tile t + 2.  Each group runs its own
  // copy of the loop (the same two barriers per tile), so the accumulators never merge across a
  // role branch and stay in place.
  auto tile_g0 = [&](auto E, int t) {
    using NE = std::integral_constant<int, 1 - decltype(E)::value>;
    mfma_tile();
    __syncthreads();
    mem_phase(NE{}, t + 2);
    __syncthreads();
  };
  auto tile_g1 = [&](auto E, int t) {
    mem_phase(E, t + 1);
    __syncthreads();
    mfma_tile();
    __syncthreads();
  };

  // prologue: tile 0 complete (all shares); G0's share of tile 1 written and its loads for tile 2
  // issued; G1's loads for tile 1 in registers; G0 holds tile 0's fragments
  gload(kbeg);
  split_store(B0{}, kbeg);
  gload(kbeg + BK);
  if (!g1) {
    split_store(B1{}, kbeg + BK);
    gload(kbeg + 2 * BK);
    __syncthreads();
    read(B0{});
    for (int t = 0; t < nk; t += 2) {
      tile_g0(B0{}, t);
      if (t + 1 < nk) tile_g0(B1{}, t + 1);
    }
  } else {
    __syncthreads();
    for (int t = 0; t < nk; t += 2) {
      tile_g1(B0{}, t);
      if (t + 1 < nk) tile_g1(B1{}, t + 1);
    }
  }
  tile_epilogue<32, TI, TJ>(p, acc, m0 + wm * WM, n0 + wn * WN, sp,
                            reinterpret_cast<float*>(smem) + wave * (WM * 36));
}

// gemm_x3 with specialised waves ("x3ws"): WGM x WGN consumer waves (the product tile: 4 x 2
// waves of 64 x 64) only read the bf16 planes from LDS and issue MFMAs; 4 producer waves (one per
// SIMD) only load the fp32 tiles, split them and write the planes.  The split's VALU and the
// global-load waits then run in the producer wave beside the consumers' MFMA stream instead of
// between its MFMA groups (gemm_x3 at 2 waves per SIMD: MFMA busy 0.40, half of the wave-cycles
// waiting; MI355X PMC, profiles/r02m_*).  12 waves = 3 per SIMD: 168 VGPRs each, which both
// roles fit (a 4 + 4 wave form with 128 x 64 consumer tiles spills at 256).  Same LDS image,
// split and product order as gemm_x3; one block barrier per 32-k tile: consumers read buffer
// kt & 1 while producers fill buffer (kt + 1) & 1 from registers loaded one tile earlier.
template <int BM, int BN, int WGM, int WGN, bool MASK>
__global__ __launch_bounds__(64 * (WGM * WGN + 4)) void gemm_x3ws(GemmArgs p) {
  constexpr int BK = 32, NC = WGM * WGN;       // consumer waves; 4 producer waves after them
  constexpr int WM = BM / WGM, WN = BN / WGN, TI = WM / 32, TJ = WN / 32;
  constexpr int NPT = 256;                        // producer threads
  constexpr int NSEG = (BM + BN) * 4 / NPT;       // 8-k segments per producer thread and tile
  static_assert((BM + BN) * 4 % NPT == 0 && TI >= 1 && TJ >= 1, "bad x3ws tile");
  constexpr int PLANE = (BM + BN) * 64, BUF = 3 * PLANE;
  constexpr int STAGE = NC * WM * 36 * 4;
  constexpr int SMEM = 2 * BUF > STAGE ? 2 * BUF : STAGE;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const int mt_n = (p.M + BM - 1) / BM, nt_n = (p.N + BN - 1) / BN;
  const int nwg = mt_n * nt_n * p.splits;
  const int bid = xcd_swizzle(blockIdx.x, nwg);
  const int mt = bid % mt_n, nt = (bid / mt_n) % nt_n, sp = bid / (mt_n * nt_n);
  const int m0 = mt * BM, n0 = nt * BN;
  const int kbeg = sp * p.kc, kend = min(p.K, kbeg + p.kc);
  const int nk = (kend - kbeg + BK - 1) / BK;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool producer = __builtin_amdgcn_readfirstlane(wave) >= NC;

  if (producer) {
    const int pt = threadIdx.x - 64 * NC;
    const float* src[NSEG];
    int soff[NSEG], sk[NSEG];
#pragma unroll
    for (int q = 0; q < NSEG; ++q) {
      const int idx = pt + q * NPT;
      const int row = idx >> 2, c = idx & 3;
      if (row < BM) {
        const int gr = m0 + row < p.M ? m0 + row : 0;   // clamped rows feed unstored outputs
        src[q] = p.A + (size_t)gr * p.lda;
      } else {
        const int gr = n0 + row - BM < p.N ? n0 + row - BM : 0;
        src[q] = p.B + (size_t)gr * p.ldb;
      }
      soff[q] = row * 64 + ((c ^ ((row >> 2) & 3)) << 4);
      sk[q] = c * 8;
    }
    using Regs = f32x4[NSEG][2];
    auto gload = [&](Regs& ld, int k0) {
#pragma unroll
      for (int q = 0; q < NSEG; ++q) {
        const int k = k0 + sk[q];
        ld[q][0] = *reinterpret_cast<const f32x4*>(src[q] + (k < p.K ? k : 0));
        ld[q][1] = *reinterpret_cast<const f32x4*>(src[q] + (k + 4 < p.K ? k + 4 : 0));
      }
    };
    auto split_store = [&](const Regs& ld, int buf, int k0) {
      char* base = smem + buf * BUF;
#pragma unroll
      for (int q = 0; q < NSEG; ++q) {
        u32x4 o[3];
        if constexpr (MASK) {
          const int k = k0 + sk[q];
          const f32x4 z = {0.f, 0.f, 0.f, 0.f};
          split3(k < kend ? ld[q][0] : z, k + 4 < kend ? ld[q][1] : z, o);
        } else {
          split3(ld[q][0], ld[q][1], o);
        }
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          *reinterpret_cast<u32x4*>(base + pl * PLANE + soff[q]) = o[pl];
      }
    };
    Regs r0, r1;
    gload(r0, kbeg);
    gload(r1, kbeg + BK);
    split_store(r0, 0, kbeg);
    __syncthreads();
    // tile kt: tile kt + 2's loads issued, tile kt + 1 (loaded one tile ago) split into the
    // other buffer, then the barrier that hands it to the consumers
    for (int kt = 0; kt < nk; kt += 2) {
      gload(r0, kbeg + (kt + 2) * BK);
      split_store(r1, (kt + 1) & 1, kbeg + (kt + 1) * BK);
      __syncthreads();
      if (kt + 1 < nk) {
        gload(r1, kbeg + (kt + 3) * BK);
        split_store(r0, kt & 1, kbeg + (kt + 2) * BK);
        __syncthreads();
      }
    }
    return;
  }

  const int wm = wave / WGN, wn = wave % WGN;
  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  int aoff[TI], akey[TI], boff[TJ], bkey[TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i) {
    const int row = wm * WM + i * 32 + (lane & 31);
    aoff[i] = row * 64;
    akey[i] = (row >> 2) & 3;
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int row = BM + wn * WN + j * 32 + (lane & 31);
    boff[j] = row * 64;
    bkey[j] = (row >> 2) & 3;
  }
  const int hk = lane >> 5;
  // fragments per unit u = (k step s, row block i): A's three planes of row block i, and W's
  // three planes of all TJ column blocks (held for the whole step); the next unit's fragments
  // are read while this unit's MFMAs run (double buffers indexed by the unrolled unit parity:
  // 72 VGPRs of fragments beside the 128 of accumulators, within the 256 of two waves per SIMD)
  bf16x8 fa[2][3], fb[2][3][TJ];
  auto rd_a = [&](bf16x8 (&d)[3], const char* S, int s, int i) {
    const int c = 2 * s + hk;
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      d[pl] = *reinterpret_cast<const bf16x8*>(S + pl * PLANE + aoff[i] + ((c ^ akey[i]) << 4));
  };
  auto rd_b = [&](bf16x8 (&d)[3][TJ], const char* S, int s, int j) {
    const int c = 2 * s + hk;
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      d[pl][j] = *reinterpret_cast<const bf16x8*>(S + pl * PLANE + boff[j] + ((c ^ bkey[j]) << 4));
  };
  auto mfma6 = [&](const bf16x8 (&A)[3], const bf16x8 (&B)[3][TJ], int i, int j) {
    f32x16 t = acc[i][j];
    t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[2][j], t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[2], B[0][j], t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[1][j], t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[1][j], t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[0][j], t, 0, 0, 0);
    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[0][j], t, 0, 0, 0);
  };
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const char* S = smem + (kt & 1) * BUF;
#pragma unroll
    for (int j = 0; j < TJ; ++j) rd_b(fb[0], S, 0, j);
    rd_a(fa[0], S, 0, 0);
#pragma unroll
    for (int u = 0; u < 2 * TI; ++u) {
      const int s = u / TI, i = u % TI;
      const int s1 = (u + 1) / TI, i1 = (u + 1) % TI;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        mfma6(fa[u & 1], fb[s], i, j);
        // after column block j's MFMAs: the next unit's A fragments (once), and at the step
        // change step 1's W fragments of column block j, whose step-0 copy just died
        if (u + 1 < 2 * TI) {
          __builtin_amdgcn_sched_barrier(0);
          if (j == 0) rd_a(fa[(u + 1) & 1], S, s1, i1);
          if (s1 != s) rd_b(fb[s1], S, s1, j);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    __syncthreads();
  }
  tile_epilogue<32, TI, TJ, true>(p, acc, m0 + wm * WM, n0 + wn * WN, sp,
                                  reinterpret_cast<float*>(smem) + wave * (WM * 36));
}

#ifdef AZ_TUNING   // gemm_x3 APL experiment only
// A [M][K] (row stride lda) -> three bf16 planes [3][M][K] (plane stride `plane` elements), the
// same split3 as gemm_x3's in-tile split, so a GEMM on the planes gives the same bits; one 8-k
// segment per thread (K % 8 == 0)
__global__ __launch_bounds__(256) void x3_split_kernel(const float* __restrict__ A, int lda, int M,
                                                       int K, unsigned short* __restrict__ out,
                                                       size_t plane) {
  const long idx = blockIdx.x * 256L + threadIdx.x;
  const int segs = K >> 3;
  if (idx >= (long)M * segs) return;
  const int r = (int)(idx / segs), c = (int)(idx % segs);
  const float* s = A + (size_t)r * lda + c * 8;
  u32x4 o[3];
  split3(*reinterpret_cast<const f32x4*>(s), *reinterpret_cast<const f32x4*>(s + 4), o);
  unsigned short* d = out + (size_t)r * K + c * 8;
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<u32x4*>(d + pl * plane) = o[pl];
}

#endif

__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmArgs p) {
  const long total = (long)p.M * p.N;
  const size_t plane = (size_t)p.M * p.N;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    float s = 0.f;
    for (int k = 0; k < p.splits; ++k) s += p.slab[k * plane + idx];
    epilogue_store(p, (int)(idx / p.N), (int)(idx % p.N), s);
  }
}

// splitk_reduce_kernel for p.vec_epi shapes: one float4 of the output per lane, its S slab
// float4s loaded before the first add (S known at compile time), summed in slab order from 0.f
// exactly as above, then epilogue_store4; one pass, no grid-stride loop.
template <int S>
__global__ __launch_bounds__(256) void splitk_reduce4_kernel(GemmArgs p) {
  const long i4 = blockIdx.x * 256L + threadIdx.x;
  const long total4 = (long)p.M * p.N / 4;
  if (i4 >= total4) return;
  const size_t plane = (size_t)p.M * p.N;
  f32x4 v[S];
#pragma unroll
  for (int k = 0; k < S; ++k) v[k] = *reinterpret_cast<const f32x4*>(p.slab + k * plane + i4 * 4);
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < S; ++k)
#pragma unroll
    for (int c = 0; c < 4; ++c) s[c] += v[k][c];
  const long e = i4 * 4;
  epilogue_store4(p, (int)(e / p.N), (int)(e % p.N), s);
}

// ------------------------------------------------------------------------------ GEMV
// C[M<=8][N] = epi(A[M][K] . W[N][K]^T): each wave owns GV_ROWS output columns and streams
// their weight rows from HBM (float4, GV_ROWS*KC/256 loads in flight per lane); A is staged
// through LDS in KC-wide chunks and shared by the block's 4 waves.
constexpr int GV_ROWS = 2;
constexpr int GV_KC = 1024;

template <int MR>
__global__ __launch_bounds__(256) void gemv_f32(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) float As[MR * GV_KC];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n_base = (blockIdx.x * 4 + wave) * GV_ROWS;
  float acc[MR][GV_ROWS];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int r = 0; r < GV_ROWS; ++r) acc[m][r] = 0.f;

  for (int kc = 0; kc < p.K; kc += GV_KC) {
    const int klen = min(GV_KC, p.K - kc);
    __syncthreads();
    for (int idx = threadIdx.x; idx < MR * (GV_KC / 4); idx += 256) {
      const int m = idx / (GV_KC / 4), k4 = (idx % (GV_KC / 4)) * 4;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      const int k = kc + k4;
      if (m < p.M && k4 < klen) {
        const int ar = p.a_rows ? p.a_rows[m] : m;
        const float* src = (p.A2 && k >= p.K0) ? p.A2 + (size_t)ar * p.lda2 + (k - p.K0)
                                               : p.A + (size_t)ar * p.lda + k;
        v = *reinterpret_cast<const f32x4*>(src);
      }
      *reinterpret_cast<f32x4*>(&As[m * GV_KC + k4]) = v;
    }
    __syncthreads();
    // unconditional loads: rows past N are clamped to row 0 (never stored), k past the chunk
    // re-reads the chunk start and meets zeros in the staged A
    f32x4 w[GV_ROWS][GV_KC / 256];
#pragma unroll
    for (int r = 0; r < GV_ROWS; ++r) {
      const int n = n_base + r < p.N ? n_base + r : 0;
#pragma unroll
      for (int s = 0; s < GV_KC / 256; ++s) {
        const int k4 = (lane + 64 * s) * 4;
        w[r][s] = *reinterpret_cast<const f32x4*>(p.B + (size_t)n * p.ldb + kc + (k4 < klen ? k4 : 0));
      }
    }
#pragma unroll
    for (int s = 0; s < GV_KC / 256; ++s) {
      const int k4 = (lane + 64 * s) * 4;
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(&As[m * GV_KC + k4]);
#pragma unroll
        for (int r = 0; r < GV_ROWS; ++r)
          acc[m][r] = fmaf(a[0], w[r][s][0], fmaf(a[1], w[r][s][1],
                      fmaf(a[2], w[r][s][2], fmaf(a[3], w[r][s][3], acc[m][r]))));
      }
    }
  }
  float mine = 0.f;  // lane m*GV_ROWS + r keeps the reduced sum of output (m, n_base + r)
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int r = 0; r < GV_ROWS; ++r) {
      const float s = wave_sum(acc[m][r]);
      if (lane == m * GV_ROWS + r) mine = s;
    }
  if (lane < MR * GV_ROWS) {
    const int m = lane / GV_ROWS, r = lane % GV_ROWS;
    if (m < p.M) epilogue_store(p, m, n_base + r, mine);
  }
}

// Staging of MG rows of A (zero-padded to S*256 floats each) for the whole-K GEMVs, split into
// a load phase and an LDS-store phase so that every load of the block is in flight before the
// first one is waited for: with the loads issued ahead of the weight stream, the store phase
// waits for A alone (vmcnt is in order), and no load sits next to a branch.
template <int MG, int S, bool SC1 = false>   // SC1: A's rows were stored by other blocks
struct RowStage {
  static constexpr int T = MG * S * 64;          // float4 slots
  static constexpr int NI = (T + 255) / 256;     // per thread
  f32x4 v[NI];
  __device__ __forceinline__ void load(const GemmArgs& p, int m0) {
    int ar[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i)
      ar[i] = min(m0 + min((int)threadIdx.x + 256 * i, T - 1) / (S * 64), p.M - 1);
    if (p.a_rows) {                                // gathered rows: all index loads, one wait
#pragma unroll
      for (int i = 0; i < NI; ++i) ar[i] = p.a_rows[ar[i]];
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int idx = min((int)threadIdx.x + 256 * i, T - 1);
      const int k = (idx % (S * 64)) * 4;
      const int kc = k < p.K ? k : 0;
      if constexpr (SC1) {                         // no A2 / gathered rows on this path
        v[i] = ld4_sc1(p.A, (ar[i] * p.lda + kc) * 4, p.M * p.lda * 4);
        continue;
      }
      const float* src = (p.A2 && kc >= p.K0) ? p.A2 + (size_t)ar[i] * p.lda2 + (kc - p.K0)
                                              : p.A + (size_t)ar[i] * p.lda + kc;
      v[i] = *reinterpret_cast<const f32x4*>(src);
    }
  }
  __device__ __forceinline__ void store(const GemmArgs& p, int m0, float* As) const {
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int idx = (int)threadIdx.x + 256 * i;
      if (T % 256 == 0 || idx < T) {
        const int m = idx / (S * 64), k = (idx % (S * 64)) * 4;
        const bool ok = m0 + m < p.M && k < p.K;
        *reinterpret_cast<f32x4*>(&As[m * S * 256 + k]) = ok ? v[i] : z;
      }
    }
  }
};

// Whole-K GEMV for K <= 256*S (the batch-1 predict shapes): A's MR rows are staged in LDS once
// (zero-padded to 256*S), then each wave issues ALL S float4 loads of its R weight rows before
// the first FMA -- one HBM round trip per wave instead of one per KC chunk.  Loads past K
// re-read the row start and meet zeros in the staged A; rows past N are clamped to row 0 and
// never stored.
// WF (the batch-1 leaf kernel): the weight rows are loaded FIRST, then pre() runs (a wait for the
// producer of A, true = go on) and only then A is staged -- same arithmetic.
struct NoPre {
  __device__ bool operator()() const { return true; }
};

// SC1 (with WF): A is read with sc1 loads and C written through with sc1 stores (bias and
// activation only: epilogue_store's arithmetic for an epilogue without C2 / R / G / beta).
template <int MR, int S, int R, bool WF = false, class Pre = NoPre, bool SC1 = false>
__device__ __forceinline__ bool gemv_full_block(const GemmArgs& p, int bid, float* As,
                                                Pre pre = Pre{}) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n_base = (bid * 4 + wave) * R;
  RowStage<MR, S, SC1> st;
  if constexpr (!WF) st.load(p, 0);
  f32x4 w[R][S];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int n = n_base + r < p.N ? n_base + r : 0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int k4 = (lane + 64 * s) * 4;
      w[r][s] = *reinterpret_cast<const f32x4*>(p.B + (size_t)n * p.ldb + (k4 < p.K ? k4 : 0));
    }
  }
  __builtin_amdgcn_sched_barrier(0);        // keep the weight stream issued before A's wait
  if constexpr (WF) {
    if (!pre()) return false;
    st.load(p, 0);
  }
  st.store(p, 0, As);
  __syncthreads();
  float acc[MR][R];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int r = 0; r < R; ++r) acc[m][r] = 0.f;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int k4 = (lane + 64 * s) * 4;
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(&As[m * S * 256 + k4]);
#pragma unroll
      for (int r = 0; r < R; ++r)
        acc[m][r] = fmaf(a[0], w[r][s][0], fmaf(a[1], w[r][s][1],
                    fmaf(a[2], w[r][s][2], fmaf(a[3], w[r][s][3], acc[m][r]))));
    }
  }
  float mine = 0.f;  // lane m*R + r keeps the reduced sum of output (m, n_base + r)
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float t = wave_sum(acc[m][r]);
      if (lane == m * R + r) mine = t;
    }
  if (lane < MR * R) {
    const int m = lane / R, r = lane % R;
    if (m < p.M && n_base + r < p.N) {
      if constexpr (SC1) {
        const int col = n_base + r;
        st_sc1(p.C + (size_t)m * p.ldc + col,
               apply_act(mine + (p.bias ? p.bias[col] : 0.f), p.act));
      } else {
        epilogue_store(p, m, n_base + r, mine);
      }
    }
  }
  return true;
}

template <int MR, int S, int R>
__global__ __launch_bounds__(256) void gemv_full(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) float As[MR * S * 256];
  gemv_full_block<MR, S, R>(p, blockIdx.x, As);
}

// gemv_full for 3 <= M <= 8 with S = 13 (K = 3136: output_transform on a speculative arena
// batch, mcts_native.ArenaPlayer), where MR = 4 / 8 rows of A would not fit gemv_full's LDS
// budget: the wave's R weight rows are loaded ONCE into registers, then the rows of A go through
// LDS MG at a time.  Every output is the same lane-strided fmaf chain + wave_sum as gemv_full,
// so a row's result does not depend on M (bit-identical to the batch-1 launch).
template <int S, int R, int MG, bool WF = false, class Pre = NoPre, bool SC1 = false>
__device__ __forceinline__ bool gemv_rows_block(const GemmArgs& p, int bid, float* As,
                                                Pre pre = Pre{}) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n_base = (bid * 4 + wave) * R;
  RowStage<MG, S, SC1> st;
  if constexpr (!WF) st.load(p, 0);
  f32x4 w[R][S];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int n = n_base + r < p.N ? n_base + r : 0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int k4 = (lane + 64 * s) * 4;
      w[r][s] = *reinterpret_cast<const f32x4*>(p.B + (size_t)n * p.ldb + (k4 < p.K ? k4 : 0));
    }
  }
  __builtin_amdgcn_sched_barrier(0);        // keep the weight stream issued before A's wait
  if constexpr (WF) {
    if (!pre()) return false;
    st.load(p, 0);
  }
  st.store(p, 0, As);
  for (int m0 = 0; m0 < p.M; m0 += MG) {
    __syncthreads();                        // this group's A is in LDS
    const bool more = m0 + MG < p.M;
    if (more) st.load(p, m0 + MG);          // the next group's loads fly under this group's FMAs
    float acc[MG][R];
#pragma unroll
    for (int m = 0; m < MG; ++m)
#pragma unroll
      for (int r = 0; r < R; ++r) acc[m][r] = 0.f;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int k4 = (lane + 64 * s) * 4;
#pragma unroll
      for (int m = 0; m < MG; ++m) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(&As[m * S * 256 + k4]);
#pragma unroll
        for (int r = 0; r < R; ++r)
          acc[m][r] = fmaf(a[0], w[r][s][0], fmaf(a[1], w[r][s][1],
                      fmaf(a[2], w[r][s][2], fmaf(a[3], w[r][s][3], acc[m][r]))));
      }
    }
    float mine = 0.f;  // lane m*R + r keeps the reduced sum of output (m0 + m, n_base + r)
#pragma unroll
    for (int m = 0; m < MG; ++m)
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const float t = wave_sum(acc[m][r]);
        if (lane == m * R + r) mine = t;
      }
    if (more) {
      __syncthreads();                      // every wave is done reading this group
      st.store(p, m0 + MG, As);
    }
    if (lane < MG * R) {
      const int m = m0 + lane / R, r = lane % R;
      if (m < p.M && n_base + r < p.N) {
        if constexpr (SC1) {
          const int col = n_base + r;
          st_sc1(p.C + (size_t)m * p.ldc + col,
                 apply_act(mine + (p.bias ? p.bias[col] : 0.f), p.act));
        } else {
          epilogue_store(p, m, n_base + r, mine);
        }
      }
    }
  }
  return true;
}

template <int S, int R, int MG>
__global__ __launch_bounds__(256) void gemv_rows(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) float As[MG * S * 256];
  gemv_rows_block<S, R, MG>(p, blockIdx.x, As);
}

// gemv_full / gemv_rows (M <= 8) plus B extra blocks that run the policy/value heads of rows of
// `side.x` --
// the batch-1 leaf's standard heads ride along with output_transform.0 instead of lengthening
// the launch chain (they only need the trunk's features, which the GEMV reads too).
template <int S, int R, int MK>
__global__ __launch_bounds__(256) void gemv_side_heads(GemmArgs p, SideHeads h, int nblk) {
  // MK: 1 / 2 = gemv_full_block with that many rows, 3 = gemv_rows_block (3..8 rows, 2 per group)
  __shared__ __attribute__((aligned(16))) float As[(MK == 1 ? 1 : 2) * S * 256];
  __shared__ float part[HEADS_ROWS_MAXC * 9];
  __shared__ float sm[9];
  // the heads blocks come FIRST in the grid: a block's start follows its index, and the heads'
  // serial chunk passes are the launch's longest path (last in the grid they ended it ~4.7 us
  // after the GEMV blocks: 12.5 vs 7.8 us, r03h kernel stats)
  if ((int)blockIdx.x >= h.B) {
    const int b = blockIdx.x - h.B;
    if constexpr (MK == 3) gemv_rows_block<S, R, 2>(p, b, As);
    else gemv_full_block<MK, S, R>(p, b, As);
  } else {
    const int row = blockIdx.x;
    heads_row_block<8, 4>(h.x + (size_t)row * h.ldx, h.x + (size_t)row * h.ldx, h.K, h.wp, h.A,
                          h.wv, h.bp, h.bv, row, h.logp, h.pi, h.v, part, sm);
  }
}

// --------------------------------------------------------------------- the batch-1 leaf kernel
// az_c4_eval_fwd for B <= 2 boards (the MCTS leaf, MCTS.py:169-173, and the arena's two-row
// speculative batches; 3-8 rows are faster as four launches) in ONE launch instead of four (trunk, output_transform.0 + standard heads,
// output_transform.2, GNN heads): every stage is the same device code as in the separate
// launches -- so every output is bit-identical to them -- and the stages hand over through
// device-scope counters:
//   blocks [0, 4B)            the trunk (c4_trunk_split_block), then signal "trunk";
//   blocks [4B, 5B)           the standard heads of one board behind "trunk"; signal "std";
//   the next ng = 392 blocks  8 columns of output_transform.0 -- their weight rows loaded into
//                             registers FIRST, under the trunk, then the features staged behind
//                             "trunk" -- signal "g1"; then the same 8 columns of
//                             output_transform.2 (weights loaded right away, hidden behind
//                             "g1"); the last block of each 256-column head chunk (ticket)
//                             forms the chunk's head partials, the last chunk (ticket)
//                             finalizes the GNN heads and zeroes every counter for the next
//                             launch.
// All blocks must be resident at once (a waiting block holds its CU): launch bounds of 2 blocks
// per CU (no spills), the launcher checks the occupancy first, workgroups are
// dispatched in index order (producers first), and every wait gives up after 20 ms, setting *err
// (host-visible) -- the caller then discards the outputs, zeroes the counters and uses the
// four-launch path.  (A first form with separate blocks for the second GEMV, both weight streams
// under the trunk, 4 blocks per CU and 1-2 rows only, measured the same 29 us at one row:
// r03n_leaf_ab, the stage chain is the bound, not the weight stream.)
struct HeadsTail {
  const float* wp; const float* bp; int A; const float* wv; const float* bv;
  float* logp; float* pi; float* v;
  float* part;        // [B][chunks][9] device scratch
};

struct LeafArgs {
  const int8_t* boards; int B;
  const float *w1, *b1, *w2, *b2;     // conv1 / conv2
  float* feat;
  GemmArgs g1, g2;                    // output_transform.0 (+ ReLU), output_transform.2
  SideHeads sh;                       // standard heads of feat
  HeadsTail ht;                       // GNN heads of g2.C
  int* sync;                          // [4 + chunks] device counters: zero on entry, left zero
  int* err;                           // host-visible: 1 = a wait timed out, outputs invalid
  int ng;                             // GEMV blocks per GEMV (8 output columns each)
  unsigned long long* trace;          // tuning build (AZ_LEAF_TRACE): [event][min, max] stamps
};

// Timing probe of the tuning build: the earliest and latest 100 MHz wall-clock stamp of each
// event over the blocks that pass it (tools/leaf_probe.py); compiled out of the product.
enum LeafEv { LE_START, LE_TRUNK, LE_G1_WEIGHTS, LE_G1_GO, LE_G1_DONE, LE_G2_WEIGHTS, LE_G2_GO,
              LE_G2_DONE, LE_CHUNK, LE_FINAL, LE_STD, LE_N };
__device__ __forceinline__ void leaf_stamp(const LeafArgs& a, int ev) {
#ifdef AZ_TUNING
  if (a.trace && threadIdx.x == 0) {
    const unsigned long long t = wall_clock64();
    atomicMin(&a.trace[2 * ev], t);
    atomicMax(&a.trace[2 * ev + 1], t);
  }
#else
  (void)a;
  (void)ev;
#endif
}

constexpr uint64_t kLeafTimeoutTicks = 2000000;   // 20 ms of the 100 MHz wall clock
// sync layout (ints): the two counters hundreds of blocks poll -- trunk done, output_transform.0
// done -- are kept in kLeafRep replicas, each on a 128-B line of its own, so the polls spread
// over many L2 channels instead of hammering one (MI355X_MICROARCH.md hand-off table, row 2:
// each producer adds to every replica with ONE wave instruction, a consumer polls one replica);
// then the standard-heads counter, the chunk-done ticket and the per-chunk tickets, one line each.
constexpr int kLeafRep = 32, kLeafLine = 32;
constexpr int kSyncTrunk = 0, kSyncG1 = kLeafRep * kLeafLine;
constexpr int kSyncStd = 2 * kLeafRep * kLeafLine, kSyncChunks = kSyncStd + kLeafLine;
constexpr int kSyncTicket0 = kSyncChunks + kLeafLine;   // + c * kLeafLine for chunk c
constexpr int kSyncInts = kSyncTicket0 + 16 * kLeafLine;   // 16 chunks at most (K <= 4096)

// wait until *ctr >= target: thread 0 polls with sc1 loads (the block parks at the barrier);
// the handed-off bytes are then read with sc1 loads only (no acquire fence: see st_sc1)
__device__ __forceinline__ bool leaf_wait(int* ctr, int target, int* err, int* flag) {
  if (threadIdx.x == 0) {
    int ok = 1;
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      // ~0.25 us between polls: hundreds of blocks polling one line back to back slow the
      // chip's memory traffic -- the weight streams this kernel overlaps (MI355X_MICROARCH.md:
      // "255 pollers cut chip bandwidth 37-71 %")
      __builtin_amdgcn_s_sleep(4);
      if (wall_clock64() - t0 > kLeafTimeoutTicks) {
        ok = 0;
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    *flag = ok;
  }
  __syncthreads();
  return *flag != 0;
}

// every wave's write-through stores have completed, then ONE lane counts the block (rep: in
// every replica, lane l of wave 0 adding to replica l)
__device__ __forceinline__ void leaf_signal(int* ctr, bool rep = false) {
  drain_stores();
  __syncthreads();
  if (rep ? threadIdx.x < kLeafRep : threadIdx.x == 0)
    __hip_atomic_fetch_add(ctr + threadIdx.x * kLeafLine, 1, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
// the replica of a replicated counter this block polls
__device__ __forceinline__ int* leaf_rep(int* ctr) {
  return ctr + (blockIdx.x % kLeafRep) * kLeafLine;
}

// leaf_signal that tells the block whether it was the total-th (last) to arrive
__device__ __forceinline__ bool leaf_ticket(int* ctr, int total, int* flag) {
  drain_stores();
  __syncthreads();
  if (threadIdx.x == 0)
    *flag = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == total - 1;
  __syncthreads();
  return *flag != 0;
}

template <int MK>
__global__ __launch_bounds__(256, 2) void c4_leaf_kernel(LeafArgs a) {   // <= 256 VGPRs
  constexpr int S = 13, R = 2;
  static_assert(MK == 1 || MK == 2, "one or two rows");
  __shared__ union {
    TrunkSplitSmem trunk;
    float As[MK * S * 256];
    struct { float part[HEADS_ROWS_MAXC * 9]; float sm[9]; } hd;
  } sm;
  __shared__ int flag;
  const int nt = 4 * a.B, id = blockIdx.x;
  leaf_stamp(a, LE_START);
  if (id < nt) {
    c4_trunk_split_block<true>(a.boards, a.w1, a.b1, a.w2, a.b2, a.feat, id >> 2, id & 3,
                               sm.trunk);
    leaf_signal(a.sync + kSyncTrunk, true);
    leaf_stamp(a, LE_TRUNK);
    return;
  }
  if (id < nt + a.B) {
    const int row = id - nt;
    if (leaf_wait(leaf_rep(a.sync + kSyncTrunk), nt, a.err, &flag))
      heads_row_block<8, 4, true>(a.sh.x + (size_t)row * a.sh.ldx, a.sh.x + (size_t)row * a.sh.ldx,
                            a.sh.K, a.sh.wp, a.sh.A, a.sh.wv, a.sh.bp, a.sh.bv, row, a.sh.logp,
                            a.sh.pi, a.sh.v, sm.hd.part, sm.hd.sm);
    leaf_signal(a.sync + kSyncStd);
    leaf_stamp(a, LE_STD);
    return;
  }
  // the GEMV blocks: 8 columns of output_transform.0, then the same 8 of output_transform.2
  const int g = id - nt - a.B;
  auto gemv = [&](const GemmArgs& p, int* ctr, int target, bool second) {
    auto pre = [&] {
#ifdef AZ_TUNING
      if (a.trace) {                     // the weights have landed (vmcnt is in order)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        leaf_stamp(a, second ? LE_G2_WEIGHTS : LE_G1_WEIGHTS);
      }
#endif
      const bool go = leaf_wait(ctr, target, a.err, &flag);
      leaf_stamp(a, second ? LE_G2_GO : LE_G1_GO);
      return go;
    };
    return gemv_full_block<MK, S, R, true, decltype(pre), true>(p, g, sm.As, pre);
  };
  const bool ok1 = gemv(a.g1, leaf_rep(a.sync + kSyncTrunk), nt, false);
  leaf_signal(a.sync + kSyncG1, true);
  leaf_stamp(a, LE_G1_DONE);
  __syncthreads();                       // the staging LDS is reused by the second GEMV
  const bool ok = gemv(a.g2, leaf_rep(a.sync + kSyncG1), a.ng, true) && ok1;
  leaf_stamp(a, LE_G2_DONE);
  const int nch = (a.g2.N + HEADS_KC - 1) / HEADS_KC;
  constexpr int PER = HEADS_KC / (4 * R);           // GEMV blocks per head chunk
  const int c = g / PER;
  if (!leaf_ticket(a.sync + kSyncTicket0 + c * kLeafLine, min(PER, a.ng - c * PER), &flag))
    return;
  const int wave = threadIdx.x >> 6;
  if (ok) {
    for (int r = wave; r < a.B; r += 4) {
      const float* yr = a.g2.C + (size_t)r * a.g2.ldc;
      heads_chunk_part<8, true>(yr, yr, a.g2.N, a.ht.wp, a.ht.A, a.ht.wv, c,
                                a.ht.part + ((size_t)r * nch + c) * 9);
    }
  }
  leaf_stamp(a, LE_CHUNK);
  if (!leaf_ticket(a.sync + kSyncChunks, nch, &flag)) return;
  if (ok) {
    for (int r = 0; r < a.B; ++r)
      heads_finalize_row<8, true>(a.ht.part + (size_t)r * nch * 9, nch, a.ht.A, a.ht.bp, a.ht.bv, r,
                            a.ht.logp, a.ht.pi, a.ht.v, sm.hd.sm);
  }
  leaf_wait(a.sync + kSyncStd, a.B, a.err, &flag);   // the standard heads' waits are over too
  for (int i = threadIdx.x; i < kSyncInts; i += 256) a.sync[i] = 0;
  leaf_stamp(a, LE_FINAL);
}

#ifdef AZ_TUNING
static unsigned long long* g_leaf_trace = nullptr;
#endif

// --------------------------------------------------------------------- K-sliced row panels
// C = epi(A . W^T) for mid-size M (the B = 512 output_transform: 512 x 3136 x 3136).  A tile
// grid cannot fill 256 CUs there without split-K, whose slabs cost a 32 MB write + re-read and
// a reduce launch per call.  Here block (mb, nb) owns 32 rows x one column panel over the WHOLE
// K (16 x 16 blocks for that shape: one per CU, no slabs):
//   - column panels are 16*CT wide except the first n_narrow, which are 16 narrower (3136 =
//     12 x 192 + 4 x 208); every block computes CT sub-tiles, so a narrow panel's last one
//     overlaps its neighbour (computed, not stored) and no row of W is ever out of range -- the
//     lanes need no clamps, hence one base pointer each instead of 15;
//   - its KW waves split K into KW contiguous slices; each wave streams its A and W fragments
//     straight from L2 into registers (double-buffered: the next step's loads fly under this
//     step's MFMAs), so the loop has no LDS traffic and no barriers;
//   - MFMA (h, t) of a step takes k = 16h + 4g + t in lane group g for both operands (a
//     bijection of the step's k values);
//   - the partial tiles meet in LDS and are summed in wave order (deterministic), then bias /
//     activation and float4 stores.
// One wave's share of a gemm_kslice block: NC column sub-tiles starting at sub-tile cs0, the
// 32 rows, k steps [it0, it1) of 32; the partial tile goes to LDS slot `slot` (row stride SP).
template <int NC, int SP>
__device__ __forceinline__ void kslice_wave(const GemmArgs& p, int m0, int n0, int cs0, int it0,
                                            int it1, float* slot) {
  constexpr int RT = 2;
  const int lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  // buffer loads: one 32-bit per-lane byte offset per operand plus a wave-uniform SGPR offset
  // per 16-row sub-tile (no hoisted 64-bit addresses)
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.A), 0, p.M * p.lda * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.B), 0, p.N * p.ldb * 4, 0x00020000);
  const int va = ((m0 + c16) * p.lda + 4 * g) * 4;               // host: M % 32 == 0
  const int vb = ((n0 + cs0 * 16 + c16) * p.ldb + 4 * g) * 4;    // rows < N by the panel layout
  const int sa = 16 * p.lda * 4, sb = 16 * p.ldb * 4;
  f32x4 acc[RT][NC];
#pragma unroll
  for (int rs = 0; rs < RT; ++rs)
#pragma unroll
    for (int cs = 0; cs < NC; ++cs) acc[rs][cs] = f32x4{0.f, 0.f, 0.f, 0.f};
  // step `it` covers k in [32 it, 32 it + 32); lane group g holds k = 16h + 4g .. +3 of half h
  auto load = [&](f32x4 (&a)[RT][2], f32x4 (&b)[NC][2], int it) {
    const int k = it * 32;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int rs = 0; rs < RT; ++rs)
        a[rs][h] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, va + (k + 16 * h) * 4, rs * sa, 0));
#pragma unroll
      for (int cs = 0; cs < NC; ++cs)
        b[cs][h] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rb, vb + (k + 16 * h) * 4, cs * sb, 0));
    }
  };
  // MFMA (h, t) of a step takes k = 16h + 4g + t in lane group g for both operands
  auto mma = [&](const f32x4 (&a)[RT][2], const f32x4 (&b)[NC][2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int rs = 0; rs < RT; ++rs)
#pragma unroll
          for (int cs = 0; cs < NC; ++cs)
            acc[rs][cs] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rs][h][t], b[cs][h][t],
                                                               acc[rs][cs], 0, 0, 0);
  };
  f32x4 a0[RT][2], b0[NC][2], a1[RT][2], b1[NC][2];
  int it = it0;
  if (it < it1) load(a0, b0, it);
  // sched_barrier: the next step's loads stay issued BEFORE this step's MFMAs (left alone, the
  // scheduler sinks them behind the MFMAs and the prefetch distance collapses)
  for (; it + 1 < it1; it += 2) {
    load(a1, b1, it + 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    if (it + 2 < it1) load(a0, b0, it + 2);
    __builtin_amdgcn_sched_barrier(0);
    mma(a1, b1);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (it < it1) mma(a0, b0);
#pragma unroll
  for (int rs = 0; rs < RT; ++rs)
#pragma unroll
    for (int cs = 0; cs < NC; ++cs)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        slot[(rs * 16 + 4 * g + r) * SP + (cs0 + cs) * 16 + c16] = acc[rs][cs][r];
}

// 512 threads: wave w takes K slice w & 3 (of 4) and column half w >> 2 (sub-tiles 0..CT0-1 or
// CT0..CT0+CT1-1); the two waves of a SIMD (w, w + 4) hold CT0 + CT1 sub-tiles between them, so
// every SIMD does the same MFMA work and has two waves to issue it.
template <int CT0, int CT1>
__global__ __launch_bounds__(512) void gemm_kslice(GemmArgs p, int n_narrow) {
  constexpr int CT = CT0 + CT1;
  constexpr int SP = 16 * CT + 4;           // partial-tile row stride: conflict-free writes
  __shared__ __attribute__((aligned(16))) float part[4 * 32 * SP];
  const int wave = threadIdx.x >> 6;
  // XCD-aware placement (1-D grid, block id b runs on XCD b % 8): each XCD owns nb / 8 whole
  // column panels and all row blocks of them, so a W panel is fetched into ONE L2 and shared by
  // the row blocks there (host: nb % 8 == 0)
  const int mb = p.M / 32, nb = gridDim.x / mb;
  const int per = nb / 8, j = blockIdx.x >> 3;
  const int by = (blockIdx.x & 7) * per + j % per, bx = j / per;
  const int m0 = bx * 32;
  const int n0 = by < n_narrow ? by * (16 * CT - 16)
                               : n_narrow * (16 * CT - 16) + (by - n_narrow) * 16 * CT;
  const int cw = by < n_narrow ? 16 * CT - 16 : 16 * CT;      // columns this block stores
  const int nit = p.K / 32;                 // host: K % 32 == 0
  const int ks = wave & 3;
  const int it0 = nit * ks / 4, it1 = nit * (ks + 1) / 4;
  float* slot = part + ks * 32 * SP;
  if (wave < 4) kslice_wave<CT0, SP>(p, m0, n0, 0, it0, it1, slot);
  else kslice_wave<CT1, SP>(p, m0, n0, CT0, it0, it1, slot);
  __syncthreads();
  const int c4n = cw / 4;
  for (int i = threadIdx.x; i < 32 * c4n; i += 512) {
    const int row = i / c4n, c4 = (i % c4n) * 4;
    const float* q = part + row * SP + c4;
    f32x4 v = *reinterpret_cast<const f32x4*>(q);
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const f32x4 u = *reinterpret_cast<const f32x4*>(q + w * 32 * SP);
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] += u[c];
    }
    epilogue_store4(p, m0 + row, n0 + c4, v);
  }
}

// gemm_kslice<7, 6> covers the shape when 16 column panels of 192 / 208 columns tile N exactly
// and 32-row blocks x 16 panels make one round of 256 blocks (M = 512, N = 3072 .. 3328: the
// B = 512 output_transform).  Returns the number of narrow (192) panels, or -1.
static int kslice_narrow(const GemmArgs& a) {
  if (a.M != 512 || a.K % 32 != 0 || a.K < 1024 || a.lda % 4 != 0 || a.ldb % 4 != 0 || !a.vec_epi)
    return -1;
  const int nb = 16;
  if (a.N % 16 != 0 || a.N < 192 * nb || a.N > 208 * nb) return -1;
  return nb - (a.N - 192 * nb) / 16;        // 208 x (nb - n) + 192 x n = N
}

// ------------------------------------------------------------------------ tall-skinny GEMM
// C[M][N] = epi(A[M][K] . W[N][K]^T) for the grid-graph layers: M ~ 10^5..10^6 rows, K in
// {64, 128}, N in {64, 128, 256}.  A tile kernel with K <= 128 spends most of each block on its
// prologue / epilogue (2 k-tiles of work per block; 2.2 TB/s on the 524288 x 256 x 64
// projection).  Here each 256-thread block is persistent over 64-row strips:
//   - W is resident in LDS, rows padded to K+1 floats (stride = 1 mod 32: the 16 columns x 2
//     k-groups of one ds_read_b32 half-wave land on 32 distinct banks);
//   - A goes straight from HBM to registers: the K axis is permuted so that lane group
//     g = lane >> 4 owns k in [g*K/4, (g+1)*K/4) and MFMA step j (16x16x4 f32) takes k = g*K/4 + j,
//     i.e. each lane reads K/4 CONTIGUOUS floats of its row (K/16 float4 loads, every row's
//     K floats covered by the 4 groups: full lines);
//   - the next strip's A is loaded while the current one is multiplied, and the outputs leave
//     in the MFMA layout as 16-float (64 B) row segments per 16 lanes, the two halves of a
//     128-B line coming from consecutive tiles of the same lanes.
// Concatenated inputs [A | A2] need K0 = a multiple of K/4 (a whole k-group per source).
// NW waves per block share one LDS copy of W (N = 256: W is 66.5 KB, so 8-wave blocks give
// 16 waves per CU where 4-wave blocks gave 8); N is covered in NP column passes that reuse the
// strip's A registers (NT/NP accumulator tiles live at a time: fewer VGPRs, more waves).
template <int N, int K, int NW, int NP>
__global__ __launch_bounds__(64 * NW) void gemm_tall(GemmArgs p, int nstrips) {
  constexpr int KS = K + 1;            // padded W row (floats)
  constexpr int KG = K / 4;            // k per lane group
  constexpr int NT = N / 16 / NP;      // 16x16 output tiles per pass
  constexpr int NV = KG / 4;           // float4 loads per lane per strip
  constexpr int BM = 16 * NW;          // rows per strip
  __shared__ float Ws[N * KS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  // W -> LDS (once per block)
  for (int i = threadIdx.x; i < N * K / 4; i += 64 * NW) {
    const int n = i / (K / 4), k = (i % (K / 4)) * 4;
    const f32x4 w = *reinterpret_cast<const f32x4*>(p.B + (size_t)n * p.ldb + k);
    float* d = Ws + n * KS + k;
    d[0] = w[0]; d[1] = w[1]; d[2] = w[2]; d[3] = w[3];
  }
  // this lane's A source for a strip: row strip*BM + wave*16 + c, k in [g*KG, g*KG + KG)
  const int kg0 = g * KG;
  const bool from2 = p.A2 != nullptr && kg0 >= p.K0;
  const float* abase = from2 ? p.A2 + (kg0 - p.K0) : p.A + kg0;
  const int lda = from2 ? p.lda2 : p.lda;
  auto load_a = [&](int strip, f32x4 (&a)[NV]) {
    int row = strip * BM + wave * 16 + c;
    row = row < p.M ? row : p.M - 1;              // clamped (never stored)
    const f32x4* src = reinterpret_cast<const f32x4*>(abase + (size_t)row * lda);
#pragma unroll
    for (int v = 0; v < NV; ++v) a[v] = src[v];
  };
  f32x4 acur[NV], anext[NV];
  int strip = blockIdx.x;
  if (strip < nstrips) load_a(strip, acur);
  __syncthreads();
  for (; strip < nstrips; strip += gridDim.x) {
    const int nxt = strip + gridDim.x;
    if (nxt < nstrips) load_a(nxt, anext);
    const int rbase = strip * BM + wave * 16 + 4 * g;   // lane's rows: rbase + r, r = 0..3
#pragma unroll 1
    for (int h = 0; h < NP; ++h) {
      f32x4 acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      // B fragments of step j + 1 are read while step j's MFMAs run; the sched_barrier keeps
      // the compiler from hoisting every step's LDS reads to the top (VGPR pressure)
      const float* wcol = Ws + (h * NT * 16 + c) * KS + kg0;
      float bcur[NT], bnext[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) bcur[t] = wcol[t * 16 * KS];
#pragma unroll
      for (int j = 0; j < KG; ++j) {
        if (j + 1 < KG) {
#pragma unroll
          for (int t = 0; t < NT; ++t) bnext[t] = wcol[t * 16 * KS + j + 1];
        }
        const float av = acur[j >> 2][j & 3];
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bcur[t], acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NT; ++t) bcur[t] = bnext[t];
        __builtin_amdgcn_sched_barrier(0);
      }
      if (p.ablate & 4) {               // timing experiment: keep the sums live, no stores
        float t0 = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) t0 += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
        if (t0 == 1234.5f) p.C[0] = t0;
        continue;
      }
      // epilogue: lane holds C[rbase + r][col], col = (h*NT + t)*16 + c; a row's tiles are
      // stored back to back, so both 64-B halves of each 128-B line leave together
      float bias[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) bias[t] = p.bias ? p.bias[(h * NT + t) * 16 + c] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbase + r;
        if (row >= p.M) break;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int col = (h * NT + t) * 16 + c;
          float v = apply_act(acc[t][r] + bias[t], p.act);
          if (p.C2) p.C2[(size_t)row * p.ldc2 + col] = v;
          if (p.R)
            v = p.R[(size_t)row * p.ldr + col] + (p.G ? p.G[(size_t)row * p.ldg + col] : 1.f) * v;
          float* dst = p.C + (size_t)row * p.ldc + col;
          if (p.beta != 0.f) v += p.beta * *dst;
          *dst = v;
        }
      }
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) acur[v] = anext[v];
  }
}

// Launches gemm_tall when the shape is one it covers; false otherwise (nothing launched).
static bool launch_tall(const GemmArgs& a, hipStream_t s) {
  static const bool off = tuning_env("AZ_GEMM_NOTALL") != nullptr;   // A/B experiments
  if (off || a.M < 16384 || a.a_rows || a.b_rows || a.c_rows || a.act == AZ_ACT_DRELU)
    return false;
  if (!((a.K == 64 || a.K == 128) && (a.N == 64 || a.N == 128 || a.N == 256))) return false;
  if (a.A2 && (a.K0 % (a.K / 4) != 0 || a.lda2 % 4 != 0)) return false;
  if (a.lda % 4 != 0 || a.ldb % 4 != 0) return false;
#define AZ_TALL(NN, KK, NW, NP)                                                               \
  if (a.N == NN && a.K == KK) {                                                              \
    const int nstrips = (a.M + 16 * NW - 1) / (16 * NW);                                     \
    hipLaunchKernelGGL((gemm_tall<NN, KK, NW, NP>), dim3(std::min(nstrips, 1024)),           \
                       dim3(64 * NW), 0, s, a, nstrips);                                     \
    return true;                                                                             \
  }
  AZ_TALL(64, 64, 4, 1) AZ_TALL(64, 128, 4, 1) AZ_TALL(128, 64, 8, 2) AZ_TALL(128, 128, 8, 2)
  AZ_TALL(256, 64, 8, 2)
#undef AZ_TALL
  return false;
}

struct TileCfg { int bm, bn, bk, wgm, wgn; };
// register-staged: 0: 64x64x32 (4 waves 2x2)   1: 128x128x32 (4 waves 2x2)   2: 64x64x64
// 3: 128x64x32 (4 waves 2x2)  4: 128x128x32 (8 waves 2x4)   5: 256x128x32 (8 waves 4x2)
// LDS-DMA (K-major A and B only): 6: 128x128x32 (4 waves 2x2)  7: 64x64x32  8: 128x64x32
// 9: 128x128x32 (8 waves 2x4)
// multi-stage LDS-DMA: 10: 128x128x16 x4 buffers  11: 128x128x32 x3  12: 128x64x32 x3
// 13: 128x128x16 x3  14: 128x64x16 x4
// LDS-DMA v2 (fragments of the whole k-tile read up front): 15: 128x128 mfma32  16: 128x128
// mfma16  17: 128x64 mfma16  18: 128x64 mfma32  19: 128x128 mfma16 (8 waves 2x4)
// v2 + DMA issue interleaved with the MFMAs: 20: 128x128 mfma32  21: 128x128 mfma16
// 22: 128x64 mfma16
// 8-wave 1-block-per-CU tiles (6 DMA pieces per 64 MFMAs instead of 8): 23: 256x128 (glds)
// 24: 256x128 (v2, mfma16)  25: 128x256 (v2, mfma16)  26/27: 256x128 interleaved DMA issue
// (mfma16 / mfma32)  28: 256x128 (v2, mfma32)
static const TileCfg kCfgs[] = {{64, 64, 32, 2, 2},  {128, 128, 32, 2, 2}, {64, 64, 64, 2, 2},
                                {128, 64, 32, 2, 2}, {128, 128, 32, 2, 4}, {256, 128, 32, 4, 2},
                                {128, 128, 32, 2, 2}, {64, 64, 32, 2, 2},  {128, 64, 32, 2, 2},
                                {128, 128, 32, 2, 4}, {128, 128, 16, 2, 2}, {128, 128, 32, 2, 2},
                                {128, 64, 32, 2, 2},  {128, 128, 16, 2, 2}, {128, 64, 16, 2, 2},
                                {128, 128, 32, 2, 2}, {128, 128, 32, 2, 2}, {128, 64, 32, 2, 2},
                                {128, 64, 32, 2, 2},  {128, 128, 32, 2, 4}, {128, 128, 32, 2, 2},
                                {128, 128, 32, 2, 2}, {128, 64, 32, 2, 2},  {256, 128, 32, 4, 2},
                                {256, 128, 32, 4, 2}, {128, 256, 32, 2, 4}, {256, 128, 32, 4, 2},
                                {256, 128, 32, 4, 2}, {256, 128, 32, 4, 2}, {256, 128, 32, 4, 2},
                                {256, 128, 32, 4, 2}, {256, 128, 32, 4, 2}, {256, 128, 32, 4, 2}};
constexpr int kNumCfgs = 33;

template <int BM, int BN, int BK, int WGM, int WGN>
static void launch_tile(const GemmArgs& a, bool akm, bool bkm, hipStream_t s) {
  const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN) * a.splits;
  dim3 g(nwg), b(64 * WGM * WGN);
  if (akm && bkm) hipLaunchKernelGGL((gemm_f32_mfma<BM, BN, BK, WGM, WGN, true, true>), g, b, 0, s, a);
  else if (akm) hipLaunchKernelGGL((gemm_f32_mfma<BM, BN, BK, WGM, WGN, true, false>), g, b, 0, s, a);
  else if (bkm) hipLaunchKernelGGL((gemm_f32_mfma<BM, BN, BK, WGM, WGN, false, true>), g, b, 0, s, a);
  else hipLaunchKernelGGL((gemm_f32_mfma<BM, BN, BK, WGM, WGN, false, false>), g, b, 0, s, a);
}

template <int BM, int BN, int WGM, int WGN>
static void launch_glds(const GemmArgs& a, hipStream_t s) {
  const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN) * a.splits;
  hipLaunchKernelGGL((gemm_f32_glds<BM, BN, WGM, WGN>), dim3(nwg), dim3(64 * WGM * WGN), 0, s, a);
}

template <int BM, int BN, int BK, int NBUF>
static void launch_pipe(const GemmArgs& a, hipStream_t s) {
  const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN) * a.splits;
  hipLaunchKernelGGL((gemm_f32_glds_pipe<BM, BN, BK, NBUF, 2, 2>), dim3(nwg), dim3(256), 0, s, a);
}

template <int BM, int BN, int WGM, int WGN, int MF, bool IL = false, int NB = 2, bool ST = false>
static void launch_glds2(const GemmArgs& a, hipStream_t s) {
  const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN) * a.splits;
  hipLaunchKernelGGL((gemm_f32_glds2<BM, BN, WGM, WGN, MF, IL, NB, ST>), dim3(nwg),
                     dim3(64 * WGM * WGN), 0, s, a);
}

static void launch_cfg(int cfg, const GemmArgs& a, bool akm, bool bkm, hipStream_t s) {
  // the product dispatch uses configs 0, 6, 8 and 24 (gemm_f32_partial); every other tile is a
  // measured-slower experiment, compiled only into the tuning build
  switch (cfg) {
    case 24: launch_glds2<256, 128, 4, 2, 16>(a, s); break;
    case 6: launch_glds<128, 128, 2, 2>(a, s); break;
    case 8: launch_glds<128, 64, 2, 2>(a, s); break;
#ifdef AZ_TUNING
    case 15: launch_glds2<128, 128, 2, 2, 32>(a, s); break;
    case 16: launch_glds2<128, 128, 2, 2, 16>(a, s); break;
    case 17: launch_glds2<128, 64, 2, 2, 16>(a, s); break;
    case 18: launch_glds2<128, 64, 2, 2, 32>(a, s); break;
    case 19: launch_glds2<128, 128, 2, 4, 16>(a, s); break;
    case 23: launch_glds<256, 128, 4, 2>(a, s); break;
    case 25: launch_glds2<128, 256, 2, 4, 16>(a, s); break;
    case 26: launch_glds2<256, 128, 4, 2, 16, true>(a, s); break;
    case 27: launch_glds2<256, 128, 4, 2, 32, true>(a, s); break;
    case 28: launch_glds2<256, 128, 4, 2, 32>(a, s); break;
    case 29: launch_glds2<256, 128, 4, 2, 16, false, 3>(a, s); break;
    case 30: launch_glds2<256, 128, 4, 2, 32, false, 3>(a, s); break;
    case 31: launch_glds2<256, 128, 4, 2, 16, false, 3, true>(a, s); break;
    case 32: launch_glds2<256, 128, 4, 2, 32, false, 3, true>(a, s); break;
    case 20: launch_glds2<128, 128, 2, 2, 32, true>(a, s); break;
    case 21: launch_glds2<128, 128, 2, 2, 16, true>(a, s); break;
    case 22: launch_glds2<128, 64, 2, 2, 16, true>(a, s); break;
    case 10: launch_pipe<128, 128, 16, 4>(a, s); break;
    case 11: launch_pipe<128, 128, 32, 3>(a, s); break;
    case 12: launch_pipe<128, 64, 32, 3>(a, s); break;
    case 13: launch_pipe<128, 128, 16, 3>(a, s); break;
    case 14: launch_pipe<128, 64, 16, 4>(a, s); break;
    case 7: launch_glds<64, 64, 2, 2>(a, s); break;
    case 9: launch_glds<128, 128, 2, 4>(a, s); break;
    case 1: launch_tile<128, 128, 32, 2, 2>(a, akm, bkm, s); break;
    case 2: launch_tile<64, 64, 64, 2, 2>(a, akm, bkm, s); break;
    case 3: launch_tile<128, 64, 32, 2, 2>(a, akm, bkm, s); break;
    case 4: launch_tile<128, 128, 32, 2, 4>(a, akm, bkm, s); break;
    case 5: launch_tile<256, 128, 32, 4, 2>(a, akm, bkm, s); break;
#endif
    default: launch_tile<64, 64, 32, 2, 2>(a, akm, bkm, s); break;
  }
}

template <int MR, int S, int R>
static bool try_gemv_full(const GemmArgs& a, hipStream_t s) {
  if constexpr (MR * S <= 32) {
    if (a.K > 256 * S) return false;
    const int nblk = (a.N + 4 * R - 1) / (4 * R);
    hipLaunchKernelGGL((gemv_full<MR, S, R>), dim3(nblk), dim3(256), 0, s, a);
    return true;
  }
  return false;
}

// whole-K kernel when A's rows fit 32 KB of LDS (S = ceil(K/256) rounded up to an
// instantiated width); AZ_GEMV_R=1 selects one weight row per wave instead of two
template <int MR>
static bool launch_gemv_full(const GemmArgs& a, hipStream_t s) {
#ifdef AZ_TUNING
  static const bool r1 = [] { const char* e = tuning_env("AZ_GEMV_R"); return e && atoi(e) == 1; }();
  if (r1)
    return try_gemv_full<MR, 1, 1>(a, s) || try_gemv_full<MR, 2, 1>(a, s) ||
           try_gemv_full<MR, 4, 1>(a, s) || try_gemv_full<MR, 8, 1>(a, s) ||
           try_gemv_full<MR, 13, 1>(a, s) || try_gemv_full<MR, 16, 1>(a, s);
#endif
  return try_gemv_full<MR, 1, 2>(a, s) || try_gemv_full<MR, 2, 2>(a, s) ||
         try_gemv_full<MR, 4, 2>(a, s) || try_gemv_full<MR, 8, 2>(a, s) ||
         try_gemv_full<MR, 13, 2>(a, s) || try_gemv_full<MR, 16, 2>(a, s);
}

static void launch_gemv(const GemmArgs& a, hipStream_t s) {
  static const bool chunked = tuning_env("AZ_GEMV_CHUNKED") != nullptr;   // A/B experiments
  if (!chunked && a.M >= 3 && a.K > 256 * 8 && a.K <= 256 * 13) {
#ifdef AZ_TUNING   // AZ_GEMV_ROWS=<MG><R>: rows per LDS group, weight rows per wave (A/B runs)
    static const char* env_rows = tuning_env("AZ_GEMV_ROWS");
    const int v = env_rows ? atoi(env_rows) : 22;
    switch (v) {
      case 42: hipLaunchKernelGGL((gemv_rows<13, 2, 4>), dim3((a.N + 7) / 8), dim3(256), 0, s, a); return;
      case 82: hipLaunchKernelGGL((gemv_rows<13, 2, 8>), dim3((a.N + 7) / 8), dim3(256), 0, s, a); return;
      case 41: hipLaunchKernelGGL((gemv_rows<13, 1, 4>), dim3((a.N + 3) / 4), dim3(256), 0, s, a); return;
      case 44: hipLaunchKernelGGL((gemv_rows<13, 4, 4>), dim3((a.N + 15) / 16), dim3(256), 0, s, a); return;
      case 12: hipLaunchKernelGGL((gemv_rows<13, 2, 1>), dim3((a.N + 7) / 8), dim3(256), 0, s, a); return;
      default: break;
    }
#endif
    // 2 rows per LDS group: 10.6 us at M = 3..4, 14.6 at M = 8 vs 16.4 / 25.2 with 4-row groups
    // and 9.9 / 15.7 with 1 (tools/gemv_probe.py on MI355X)
    hipLaunchKernelGGL((gemv_rows<13, 2, 2>), dim3((a.N + 7) / 8), dim3(256), 0, s, a);
    return;
  }
  if (!chunked) {
    bool done = false;
    switch (a.M) {
      case 1: done = launch_gemv_full<1>(a, s); break;
      case 2: done = launch_gemv_full<2>(a, s); break;
      case 3: case 4: done = launch_gemv_full<4>(a, s); break;
      default: done = launch_gemv_full<8>(a, s); break;
    }
    if (done) return;
  }
  const int nblk = (a.N + 4 * GV_ROWS - 1) / (4 * GV_ROWS);
  switch (a.M) {
    case 1: hipLaunchKernelGGL(gemv_f32<1>, dim3(nblk), dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL(gemv_f32<2>, dim3(nblk), dim3(256), 0, s, a); break;
    case 3: case 4: hipLaunchKernelGGL(gemv_f32<4>, dim3(nblk), dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL(gemv_f32<8>, dim3(nblk), dim3(256), 0, s, a); break;
  }
}

// Pick the block tile and the split-K factor: aim for ~2 blocks per CU (512) on the 256 CUs,
// keep >= 4 BK steps per split, and only split when the caller's workspace holds the slabs.
static void plan(GemmArgs& a, int bm, int bn, int bk, size_t ws_bytes) {
  const long tiles = (long)((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
  int S = 1;
  static const char* env_split = tuning_env("AZ_GEMM_SPLITS");
  if (env_split && a.slab) {
    S = std::max(1, atoi(env_split));
  } else if (tiles < 1024 && a.slab) {
    // measured on MI355X (tools/gemm_sweep.py): M=512 x 3136^2 best at S=3 (1176 blocks),
    // M=64 at S=4..8; keep >= 4 BK steps per split
    S = (int)std::min<long>(std::min<long>((1024 + tiles - 1) / tiles, 8), a.K / (bk * 4));
  }
  while (S > 1 && (size_t)S * a.M * a.N * 4 > ws_bytes) --S;
  if (S < 1) S = 1;
  a.splits = S;
  a.kc = S > 1 ? ((a.K + S - 1) / S + bk - 1) / bk * bk : a.K;
  if (S > 1) a.splits = (a.K + a.kc - 1) / a.kc;
}

// Split factor for the 128x128 LDS-DMA tile when its grid alone is small.  At most 2 blocks fit
// a CU (64 KB of LDS each), so the launch runs in ceil(blocks / 256) block-rounds per CU, each
// as long as one split's k-tiles; two co-resident blocks hide each other's latency (~1.1x,
// measured), and every extra split costs an M x N slab written and re-read.  The model
// reproduces the MI355X sweep ranking (tools/gemm_sweep.py glds: M=512 -> S=5, M=256 -> S=5).
static int glds_splits(const GemmArgs& a, long tiles, size_t ws_bytes) {
  const int bk = 32;
  int best = 1;
  double best_cost = 1e30;
  for (int S = 1; S <= 16; ++S) {
    const long kc = ((a.K + S - 1) / S + bk - 1) / bk * bk;
    if (S > 1 && (kc < 4 * bk || (size_t)S * a.M * a.N * 4 > ws_bytes || !a.slab)) break;
    const long splits = (a.K + kc - 1) / kc;
    const long nwg = tiles * splits;
    const long rounds = (nwg + 255) / 256;
    double cost = (double)rounds * (double)(kc / bk) / (nwg > 256 ? 1.1 : 1.0);
    // slab round trip (S x M x N x 8 B at ~5 TB/s) in units of one k-tile (~2 us)
    if (splits > 1) cost += (double)splits * a.M * a.N * 8.0 / 5e12 / 2e-6;
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = (int)splits;
    }
  }
  return best;
}

// Split factor for the 256x128 8-wave tile (96 KB of LDS: one block per CU): the largest S with
// tiles * S <= 256 CUs, used only when that grid fills >= 85 % of the CUs, each split keeps
// >= 8 k-tiles and the S slabs fit the workspace; 0 = do not use this tile.
static int splits_256x128(int M, int N, int K, size_t ws_bytes) {
  const long tiles = (long)((M + 255) / 256) * ((N + 127) / 128);
  if (tiles >= 256) return 0;
  const int S = (int)std::min<long>(256 / tiles, 8);
  if (tiles * S < 218) return 0;   // >= 85 % of the CUs (M = 768: 225 blocks, 158 vs 178 us)
  if (S > 1 && ((long)K / S < 8 * 32 || (size_t)S * M * N * 4 > ws_bytes)) return 0;
  return S;
}

// ---------------------------------------------------------------------------------------------
// Row scales of the fp16 form (H3, az_x3.h split2s): one 256-thread block per row, s[r] = 2^e
// with max_k |X[r][k]| * s in [2^(T-1), 2^T) (s = 1 for an all-zero or non-finite row: a NaN / inf
// then reaches the outputs as in fp32), out[rows + r] = 1 / s (exact).  e is kept within +-120 so
// s and 1/s are normal floats.  Every lane issues its (up to 4) float4 loads of a 4096-column
// chunk before the first maximum: one HBM round trip per chunk (a wave per row walking the row
// one float4 per lane at a time took 5.7 us at M = 512, K = 3136 -- 13 dependent round trips).
__global__ __launch_bounds__(256) void row_scale_kernel(const float* __restrict__ X, int rows,
                                                        int cols, int ld, int T,
                                                        float* __restrict__ out) {
  __shared__ float wm[4];
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  if (r >= rows) return;
  const float* x = X + (size_t)r * ld;
  float m = 0.f;
  const int c4 = (reinterpret_cast<uintptr_t>(x) & 15) == 0 ? cols & ~3 : 0;
  constexpr int U = 4;
  for (int c0 = tid * 4; c0 < c4; c0 += 256 * 4 * U) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + u * 256 * 4;
      v[u] = c < c4 ? *reinterpret_cast<const f32x4*>(x + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u][0]), fabsf(v[u][1])), fmaxf(fabsf(v[u][2]), fabsf(v[u][3]))));
  }
  for (int c = c4 + tid; c < cols; c += 256) m = fmaxf(m, fabsf(x[c]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if (lane == 0) wm[tid >> 6] = m;
  __syncthreads();
  if (tid == 0) {
    m = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
    int e = 0;
    if (m > 0.f && m <= 3.4e38f) {
      int ex;
      (void)frexpf(m, &ex);
      e = min(120, max(-120, T - ex));
    }
    out[r] = ldexpf(1.f, e);
    out[rows + r] = ldexpf(1.f, -e);
  }
}

// A row's power-of-two scale (as row_scale_kernel: sc[r] = s, sc[rows + r] = 1 / s) AND its two fp16
// planes (split2s of x s, in the p2_chunk layout of az_x3.h), one 256-thread block per row, the
// row read once when cols <= 4096 (8-float chunks in registers): the P2 GEMM's operands.
// cols % 32 == 0 and 16-B aligned rows (the caller checks).
__global__ __launch_bounds__(256) void h3_split_rows_kernel(const float* __restrict__ X, int rows,
                                                            int cols, int ld, int T,
                                                            unsigned short* __restrict__ out,
                                                            float* __restrict__ sc) {
  __shared__ float wm[4];
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  if (r >= rows) return;
  const float* x = X + (size_t)r * ld;
  const int nch = cols >> 3;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  f32x4 v[2][2];
  float m = 0.f;
  auto amax = [](const f32x4& a, const f32x4& b) {
    return fmaxf(fmaxf(fmaxf(fabsf(a[0]), fabsf(a[1])), fmaxf(fabsf(a[2]), fabsf(a[3]))),
                 fmaxf(fmaxf(fabsf(b[0]), fabsf(b[1])), fmaxf(fabsf(b[2]), fabsf(b[3]))));
  };
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int ch = tid + 256 * u;
    v[u][0] = ch < nch ? *reinterpret_cast<const f32x4*>(x + 8 * ch) : z;
    v[u][1] = ch < nch ? *reinterpret_cast<const f32x4*>(x + 8 * ch + 4) : z;
    m = fmaxf(m, amax(v[u][0], v[u][1]));
  }
  for (int ch = tid + 512; ch < nch; ch += 256)      // rows longer than 4096
    m = fmaxf(m, amax(*reinterpret_cast<const f32x4*>(x + 8 * ch),
                      *reinterpret_cast<const f32x4*>(x + 8 * ch + 4)));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if (lane == 0) wm[tid >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
  int e = 0;
  if (m > 0.f && m <= 3.4e38f) {
    int ex;
    (void)frexpf(m, &ex);
    e = min(120, max(-120, T - ex));
  }
  const float s = ldexpf(1.f, e);
  if (tid == 0) {
    sc[r] = s;
    sc[rows + r] = ldexpf(1.f, -e);
  }
  auto put = [&](int ch, const f32x4& a, const f32x4& b) {
    u32x4 o[2];
    split2s(a, b, s, o);
    *reinterpret_cast<u32x4*>(out + p2_chunk(r, ch, 0, cols)) = o[0];
    *reinterpret_cast<u32x4*>(out + p2_chunk(r, ch, 1, cols)) = o[1];
  };
#pragma unroll
  for (int u = 0; u < 2; ++u)
    if (tid + 256 * u < nch) put(tid + 256 * u, v[u][0], v[u][1]);
  for (int ch = tid + 512; ch < nch; ch += 256)
    put(ch, *reinterpret_cast<const f32x4*>(x + 8 * ch), *reinterpret_cast<const f32x4*>(x + 8 * ch + 4));
}

// The split-K reduce of a GEMM whose C is the next GEMM's A, fused with that GEMM's A split (the
// output_transform.0 -> .2 hand-off, gnn_utils.py:115): one block per row; each lane's
// 8-column chunk(s) are summed over the S slabs in slab order from 0.f, then bias and activation
// -- splitk_reduce4_kernel's arithmetic, so C's bits are unchanged -- and stored; the row's max
// |C| (one block reduction) gives the scale, and the chunks, still in registers, leave as the two
// fp16 planes + scales h3_split_rows_kernel would make of C (out: the p2_chunk layout, sc [2][M]).
// N % 32 == 0, N <= 4096, bias / activation epilogue only, 16-B aligned rows (splitk_reduce_split).
template <int S, int U>
__global__ __launch_bounds__(512) void splitk_reduce_split_kernel(GemmArgs p,
                                                                  unsigned short* __restrict__ out,
                                                                  float* __restrict__ sc) {
  __shared__ float wm[8];
  const int T = blockDim.x;          // U chunks per thread, stride T
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int nch = p.N >> 3;
  const size_t plane = (size_t)p.M * p.N;
  const float* sl = p.slab + (size_t)r * p.N;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  f32x4 x[U][S][2], bb[U][2];
#pragma unroll
  for (int u = 0; u < U; ++u) {               // every load issued before the first add
    const int c = 8 * min(tid + T * u, nch - 1);
#pragma unroll
    for (int q = 0; q < S; ++q) {
      x[u][q][0] = *reinterpret_cast<const f32x4*>(sl + q * plane + c);
      x[u][q][1] = *reinterpret_cast<const f32x4*>(sl + q * plane + c + 4);
    }
    bb[u][0] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + c) : z;
    bb[u][1] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + c + 4) : z;
  }
  f32x4 v[U][2];
  float m = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < S; ++q) t += x[u][q][h][e];
        if (p.bias) t += bb[u][h][e];
        v[u][h][e] = apply_act(t, p.act);
      }
    const int ch = tid + T * u;
    if (ch < nch) {
      if (p.C) {                                  // null: the caller needs only the planes
        float* dst = p.C + (size_t)r * p.ldc + 8 * ch;
        *reinterpret_cast<f32x4*>(dst) = v[u][0];
        *reinterpret_cast<f32x4*>(dst + 4) = v[u][1];
      }
      m = fmaxf(m, fmaxf(fmaxf(fmaxf(fabsf(v[u][0][0]), fabsf(v[u][0][1])),
                               fmaxf(fabsf(v[u][0][2]), fabsf(v[u][0][3]))),
                         fmaxf(fmaxf(fabsf(v[u][1][0]), fabsf(v[u][1][1])),
                               fmaxf(fabsf(v[u][1][2]), fabsf(v[u][1][3])))));
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if (lane == 0) wm[tid >> 6] = m;
  __syncthreads();
  m = wm[0];
  for (int w = 1; w < (T >> 6); ++w) m = fmaxf(m, wm[w]);
  float inv;
  const float s = h3_scale(m, H3_TA, &inv);
  if (tid == 0) {
    sc[r] = s;
    sc[p.M + r] = inv;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int ch = tid + T * u;
    if (ch < nch) {
      u32x4 o[2];
      split2s(v[u][0], v[u][1], s, o);
      *reinterpret_cast<u32x4*>(out + p2_chunk(r, ch, 0, p.N)) = o[0];
      *reinterpret_cast<u32x4*>(out + p2_chunk(r, ch, 1, p.N)) = o[1];
    }
  }
}


// W row-scale cache: weights change only between calls that say so (az_weights_changed, which
// az_adam_f32 also calls; the Python parameter store calls it on every load / copy), so a
// weight matrix's scales are computed once per weight update.  Each entry has two buffers: a
// recompute writes the other one and synchronises its stream before publishing it, so a GEMM
// launched earlier on another stream keeps reading consistent scales, and one launched later on
// any stream sees finished ones.
static std::atomic<long> g_wgen{1};
struct WScaleEntry {
  const float* w;
  int n, k, ld;
  long gen;                    // generation buf[cur] (the in-tile GEMM's row scales) is from
  float* buf[2];
  int cur;
  unsigned short* planes[2];   // the P2 GEMM's W planes [2][n][k] (nullptr until first asked)
  float* pbuf[2];              // their row scales: a double buffer of its own, so a recompute
  int pcur;                    // of one kind never overwrites the other kind's live buffer
  long pgen;                   // generation planes[pcur] / pbuf[pcur] were split at
  float* frags[2];             // conv2's weights in the trunk's MFMA fragment order (conv2_frags)
  int fcur;
  long fgen;
};

static std::mutex g_wmu;
static std::vector<WScaleEntry> g_wcache;

// the entry of (w, n, k, ld), created on first use (caller holds g_wmu); nullptr when out of memory
static WScaleEntry* wcache_entry(const float* w, int n, int k, int ld) {
  for (auto& x : g_wcache)
    if (x.w == w && x.n == n && x.k == k && x.ld == ld) return &x;
  WScaleEntry x{w, n, k, ld, 0, {nullptr, nullptr}, 1, {nullptr, nullptr}, {nullptr, nullptr},
                1, 0, {nullptr, nullptr}, 1, 0};
  if (hipMalloc(&x.buf[0], (size_t)8 * n * sizeof(float)) != hipSuccess) return nullptr;
  x.buf[1] = x.buf[0] + 2 * n;
  x.pbuf[0] = x.buf[0] + 4 * n;
  x.pbuf[1] = x.buf[0] + 6 * n;
  g_wcache.push_back(x);
  return &g_wcache.back();
}

// Parameter storage the caller registered (az_weights_register): only weights inside it are
// cached -- anywhere else a pointer says nothing about the values behind it (a freed tensor's
// memory can hold the next one), so their scales are computed per call and the pre-split planes
// are not used.
static std::mutex g_regmu;
static std::vector<std::pair<uintptr_t, uintptr_t>> g_regs;

static bool weights_registered(const float* w, int n, int k, int ld) {
  const uintptr_t b = reinterpret_cast<uintptr_t>(w);
  const uintptr_t e = b + ((size_t)(n - 1) * ld + k) * sizeof(float);
  std::lock_guard<std::mutex> lk(g_regmu);
  for (const auto& r : g_regs)
    if (b >= r.first && e <= r.second) return true;
  return false;
}

}  // namespace az
extern "C" int az_weights_changed(void) {
  az::g_wgen.fetch_add(1);
  return AZ_OK;
}
extern "C" int az_weights_register(const void* base, size_t bytes) {
  AZ_REQUIRE(base && bytes > 0, AZ_EINVAL, "az_weights_register: null / empty range");
  {
    std::lock_guard<std::mutex> lk(az::g_regmu);
    const uintptr_t b = reinterpret_cast<uintptr_t>(base);
    az::g_regs.emplace_back(b, b + bytes);
  }
  return az_weights_changed();           // a reused range must not meet old cache entries
}
extern "C" int az_weights_unregister(const void* base) {
  std::vector<std::pair<uintptr_t, uintptr_t>> gone;
  {
    std::lock_guard<std::mutex> lk(az::g_regmu);
    const uintptr_t b = reinterpret_cast<uintptr_t>(base);
    for (size_t i = 0; i < az::g_regs.size();)
      if (az::g_regs[i].first == b) {
        gone.push_back(az::g_regs[i]);
        az::g_regs.erase(az::g_regs.begin() + i);
      } else {
        ++i;
      }
  }
  // free the cache entries (row scales + fp16 planes: 8 N K bytes per weight, 79 MB for a
  // 3136 x 3136 one) of weights inside the range, once no launched GEMM can still read them
  if (!gone.empty()) {
    std::lock_guard<std::mutex> lk(az::g_wmu);
    bool synced = false;
    for (size_t i = 0; i < az::g_wcache.size();) {
      const uintptr_t w = reinterpret_cast<uintptr_t>(az::g_wcache[i].w);
      bool inside = false;
      for (const auto& r : gone) inside |= w >= r.first && w < r.second;
      if (!inside) {
        ++i;
        continue;
      }
      if (!synced) {
        AZ_REQUIRE(hipDeviceSynchronize() == hipSuccess, AZ_EDEVICE,
                   "az_weights_unregister: hipDeviceSynchronize failed");
        synced = true;
      }
      (void)hipFree(az::g_wcache[i].buf[0]);
      if (az::g_wcache[i].planes[0]) (void)hipFree(az::g_wcache[i].planes[0]);
      if (az::g_wcache[i].frags[0]) (void)hipFree(az::g_wcache[i].frags[0]);
      az::g_wcache.erase(az::g_wcache.begin() + i);
    }
  }
  return az_weights_changed();
}
namespace az {

static const float* w_row_scales(const float* w, int n, int k, int ld, hipStream_t s) {
  if (!weights_registered(w, n, k, ld)) return nullptr;   // the caller computes them per call
  const long gen = g_wgen.load();
  std::lock_guard<std::mutex> lk(g_wmu);
  WScaleEntry* e = wcache_entry(w, n, k, ld);
  if (!e) return nullptr;
  if (e->gen == gen) return e->buf[e->cur];
  const int nxt = e->cur ^ 1;
  hipLaunchKernelGGL(row_scale_kernel, dim3(n), dim3(256), 0, s, w, n, k, ld, H3_TW,
                     e->buf[nxt]);
  if (hipStreamSynchronize(s) != hipSuccess) return nullptr;
  e->cur = nxt;
  e->gen = gen;
  return e->buf[nxt];
}

// W's fp16 planes and scales for the P2 GEMM, cached like the scales above (two buffers, the
// recompute synchronises its stream before publishing); nullptr when memory is short.
static const unsigned short* w_planes(const float* w, int n, int k, int ld, hipStream_t s,
                                      const float** scales) {
  if (!weights_registered(w, n, k, ld)) return nullptr;
  const long gen = g_wgen.load();
  std::lock_guard<std::mutex> lk(g_wmu);
  WScaleEntry* e = wcache_entry(w, n, k, ld);
  if (!e) return nullptr;
  if (!e->planes[0]) {
    const size_t one = (size_t)2 * n * k;
    if (hipMalloc(&e->planes[0], 2 * one * sizeof(unsigned short)) != hipSuccess) {
      e->planes[0] = nullptr;
      return nullptr;
    }
    e->planes[1] = e->planes[0] + one;
    e->pgen = 0;
  }
  if (e->pgen == gen) {
    *scales = e->pbuf[e->pcur];
    return e->planes[e->pcur];
  }
  const int nxt = e->pcur ^ 1;
  hipLaunchKernelGGL(h3_split_rows_kernel, dim3(n), dim3(256), 0, s, w, n, k, ld, H3_TW,
                     e->planes[nxt], e->pbuf[nxt]);
  if (hipStreamSynchronize(s) != hipSuccess) return nullptr;
  e->pcur = nxt;
  e->pgen = gen;
  *scales = e->pbuf[nxt];
  return e->planes[nxt];
}

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, false));
}

// The heads from a GEMM's tile partials (az_x3.h HeadsEpi; the GEMM added the bias b of y in its
// first k split / piece): one wave per row sums the row's slots in a fixed order -- split-K form:
// lane t takes slots t, t + 64, ... in turn; stream-K form (CSK): lane t takes 64-column block t
// and its pieces in k order (their count from the plan, as csk_fixup4_kernel) -- then one
// butterfly over the lanes for all 9 values at once, so the bits do not depend on the launch
// shape; then the heads' biases and log_softmax / exp / tanh as heads_finalize_kernel.
template <bool CSK>
__global__ __launch_bounds__(256) void heads_tiles_finalize_kernel(HeadsEpi he, int M, int N,
                                                                   int P, CskPlan q) {
  constexpr int HS = HEADS_TILE_SLOTS;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);   // one row per wave
  const float* src = he.part + (size_t)min(row, M - 1) * P * HS;
  float s[16];
#pragma unroll
  for (int a = 0; a < 16; ++a) s[a] = 0.f;
  if constexpr (CSK) {
    // the row's P * HS slot values (contiguous) staged in LDS by coalesced loads first: read in
    // place, lane cb's pieces sit P * HS / 49 floats from its neighbour's, so every load
    // instruction touched ~49 cache lines (41 us per M = 3,150 launch, PMC-free trace r05m)
    extern __shared__ float hstage[];
    float* const st = hstage + (threadIdx.x >> 6) * P * HS;
    const int n = P * HS;
    for (int i0 = 0; i0 < n; i0 += 8 * 64) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + 64 * u + lane;
        t[u] = i < n ? src[i] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + 64 * u + lane;
        if (i < n) st[i] = t[u];
      }
    }
    __syncthreads();
    if (row >= M) return;
    const int cb = lane, col = 64 * cb;
    if (col < N) {
      const int mt = row >> 8;
      int f, b, W;
      if (q.tail && mt == q.mt_n - 1) {
        f = (col >> 8) % q.at;
        b = q.bt;
        W = q.at * q.KT;
      } else {
        f = mt % q.am + q.am * ((col >> 7) % q.an);
        b = q.bf;
        W = q.am * q.an * q.KT;
      }
      const int np = csk_block_of((f + 1) * q.KT - 1, b, W) - csk_block_of(f * q.KT, b, W) + 1;
      // the pieces in k order
      for (int pc = 0; pc < np; ++pc)
#pragma unroll
        for (int a = 0; a < HS; ++a) s[a] += st[(cb * he.mp + pc) * HS + a];
    }
  } else {
    if (row >= M) return;
    for (int t = lane; t < P; t += 64)
#pragma unroll
      for (int a = 0; a < HS; ++a) s[a] += src[(size_t)t * HS + a];
  }
  // the lane sums: DPP adds within each 16-lane row (quad_perm [1,0,3,2], [2,3,0,1],
  // row_half_mirror, row_mirror: no LDS), then the four row sums in row order (readlane)
#pragma unroll
  for (int a = 0; a < HS; ++a) {
    float v = s[a];
    v += dpp_mov<0xB1>(v);
    v += dpp_mov<0x4E>(v);
    v += dpp_mov<0x141>(v);
    v += dpp_mov<0x140>(v);
    s[a] = (__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0)) +
            __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16)) +
            __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32)) +
            __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48)));
  }
  if (lane != 0) return;
  const int A = he.A;
  float l[8];
  float mx = -INFINITY;
#pragma unroll
  for (int a = 0; a < 8; ++a)
    if (a < A) {
      l[a] = s[a] + he.bp[a];
      mx = fmaxf(mx, l[a]);
    }
  float se = 0.f;
#pragma unroll
  for (int a = 0; a < 8; ++a)
    if (a < A) se += expf(l[a] - mx);
  const float lse = logf(se);
#pragma unroll
  for (int a = 0; a < 8; ++a)
    if (a < A) {
      const float o = (l[a] - mx) - lse;
      he.logp[(size_t)row * A + a] = o;
      if (he.pi) he.pi[(size_t)row * A + a] = expf(o);
    }
  he.v[row] = tanhf(s[8] + he.bv[0]);
}

// The Connect4 trunk's conv2 weights ([64][32][3][3]) in the order its MFMA fragments use them
// (az_trunk.hip c4_trunk_tile): frag[nt][q][lane][e] = w2[co][ci][tap] for step s = 4q + e
// = tap * 8 + j, co = 16 nt + (lane & 15), ci = 8 (lane >> 4) + j.  A wave then loads its 72
// weights as 18 coalesced 1-KB float4 loads instead of staging the 74 KB through LDS.
__global__ __launch_bounds__(256) void c4_w2_frag_kernel(const float* __restrict__ w2,
                                                         float* __restrict__ frag) {
  const int i = blockIdx.x * 256 + threadIdx.x;       // 4 * 18 * 64 * 4 = 18,432 values
  if (i >= 18432) return;
  const int e = i & 3, lane = (i >> 2) & 63, q = (i >> 8) % 18, nt = i / (18 * 256);
  const int st = 4 * q + e, tap = st >> 3, j = st & 7;
  const int co = 16 * nt + (lane & 15), ci = 8 * (lane >> 4) + j;
  frag[i] = w2[co * 288 + ci * 9 + tap];
}

// conv2_frags: the fragment-ordered copy of registered conv2 weights, cached per weight
// generation like w_planes (double buffer, the recompute synchronises its stream before
// publishing); nullptr for unregistered weights or when memory is short (the trunk then stages
// the weights through LDS itself: the same values, the same bits).
const float* conv2_frags(const float* w2, hipStream_t s) {
  if (!weights_registered(w2, 64, 288, 288)) return nullptr;
  const long gen = g_wgen.load();
  std::lock_guard<std::mutex> lk(g_wmu);
  WScaleEntry* e = wcache_entry(w2, 64, 288, 288);
  if (!e) return nullptr;
  if (!e->frags[0]) {
    if (hipMalloc(&e->frags[0], (size_t)2 * 18432 * sizeof(float)) != hipSuccess) {
      e->frags[0] = nullptr;
      return nullptr;
    }
    e->frags[1] = e->frags[0] + 18432;
    e->fgen = 0;
  }
  if (e->fgen == gen) return e->frags[e->fcur];
  const int nxt = e->fcur ^ 1;
  hipLaunchKernelGGL(c4_w2_frag_kernel, dim3(72), dim3(256), 0, s, w2, e->frags[nxt]);
  if (hipStreamSynchronize(s) != hipSuccess) return nullptr;
  e->fcur = nxt;
  e->fgen = gen;
  return e->frags[nxt];
}

// the split-K HEADS tiles' finalize (P = 128-column tiles x k splits)
static void launch_heads_finalize(GemmArgs& a, hipStream_t s) {
  const int P = (a.N + 127) / 128 * a.splits;
  // one wave (one row) per block: the M = 512 rows over every CU rather than 128 of them
  // (6.01 -> 5.11 us per launch, profiles/r06/finalize_ab); staging the row's slots through
  // LDS by coalesced loads first, as the stream-K form does, measured 6.57 us
  hipLaunchKernelGGL(heads_tiles_finalize_kernel<false>, dim3(a.M), dim3(64), 0, s, a.he, a.M,
                     a.N, P, CskPlan{});
  a.heads_done = 1;
}

// gemm_x3 launch for a K-major A and W (no A2 / gathered rows), M > 64: 256x128 (8 waves) above
// M = 256, else 128x128 (4 waves); split-K so the grid nears one block per CU (measured on
// MI355X, tools/gemm_sweep.py x3: M = 512 75 us vs 103 us for the fp32 MFMA tile, M = 800 147 vs
// 185, M = 4096 516 vs 767).  Tuning build: AZ_GEMM_X3=0 keeps the fp32 MFMA tiles, 1..4 forces
// a tile, AZ_GEMM_SPLITS the split.  Sets a.splits / a.kc; false = not launched.
static bool launch_x3(GemmArgs& a, size_t ws_bytes, hipStream_t s, const PreSplitA* pre) {
  static const char* env = tuning_env("AZ_GEMM_X3");
  static const char* env_split = tuning_env("AZ_GEMM_SPLITS");
  // the fp16 form (H3) for the product tiles when the workspace can hold A's row scales (taken
  // from its end, after every split-K slab); tuning build: AZ_GEMM_PREC=x3 keeps the bf16 form
  static const char* env_prec = tuning_env("AZ_GEMM_PREC");
  // A's scales [2][M] and, for weights outside registered parameter storage, W's [2][N]
  const size_t sa_bytes = ((size_t)2 * (a.M + a.N) * sizeof(float) + 255) / 256 * 256;
  bool h3 = !(env_prec && strcmp(env_prec, "x3") == 0) && a.slab && ws_bytes >= sa_bytes + 256;
  if (h3) ws_bytes = (ws_bytes - sa_bytes) / 256 * 256;
  float* const sa_buf = h3 ? reinterpret_cast<float*>(reinterpret_cast<char*>(a.slab) + ws_bytes)
                           : nullptr;
  float* const sw_buf = h3 ? sa_buf + 2 * a.M : nullptr;
  // P2 (product dispatch, whole 32-k tiles): A split once per call into its two fp16 planes
  // (h3_split_rows_kernel, also its row scales) in the workspace before the scales, W's planes
  // cached per weight generation (w_planes); the tile then moves both by LDS-DMA with no VALU --
  // 8-12 % faster tiles than splitting in the tile, bit-identical (tools/p2h_probe.py)
  const bool whole_k = a.K % 32 == 0;
  // a caller that already holds A's planes and scales (PreSplitA: the trunk / the fused split-K
  // reduce of the layer before) needs no room for them here
  const bool have_pre = pre && pre->planes && pre->sc && aligned16(pre->planes);
  const size_t p2a_bytes = have_pre ? 0 : ((size_t)4 * a.M * a.K + 255) / 256 * 256;
  bool p2 = h3 && !tuning_env("AZ_GEMM_X3") && !tuning_env("AZ_GEMM_SPLITS") &&
            !tuning_env("AZ_GEMM_NOP2") && whole_k && a.lda % 4 == 0 && a.ldb % 4 == 0 &&
            aligned16(a.A) && aligned16(a.B) && ws_bytes >= p2a_bytes + 256 &&
            weights_registered(a.B, a.N, a.K, a.ldb);
  unsigned short* apl_buf = nullptr;
  if (p2 && !have_pre) {
    ws_bytes = (ws_bytes - p2a_bytes) / 256 * 256;
    apl_buf = reinterpret_cast<unsigned short*>(reinterpret_cast<char*>(a.slab) + ws_bytes);
  }
  auto p2_prep = [&]() {
    const float* sw = nullptr;
    const unsigned short* wpl = w_planes(a.B, a.N, a.K, a.ldb, s, &sw);
    if (!wpl) return false;
    if (have_pre) {
      a.apl = pre->planes;
      a.sa = pre->sc;
    } else {
      hipLaunchKernelGGL(h3_split_rows_kernel, dim3(a.M), dim3(256), 0, s, a.A, a.M, a.K, a.lda,
                         H3_TA, apl_buf, sa_buf);
      a.apl = apl_buf;
      a.sa = sa_buf;
    }
    a.apl_plane = (size_t)a.M * a.K;
    a.bpl = wpl;
    a.bpl_plane = (size_t)a.N * a.K;
    a.sw = sw;
    return true;
  };
  // A's row scales and W's (cached) just before the launch that uses them
  auto h3_scales = [&]() {
    const float* sw = w_row_scales(a.B, a.N, a.K, a.ldb, s);
    if (!sw) {                          // not cacheable: this call's own W scales
      hipLaunchKernelGGL(row_scale_kernel, dim3(a.N), dim3(256), 0, s, a.B, a.N, a.K, a.ldb,
                         H3_TW, sw_buf);
      sw = sw_buf;
    }
    hipLaunchKernelGGL(row_scale_kernel, dim3(a.M), dim3(256), 0, s, a.A, a.M, a.K,
                       a.lda, H3_TA, sa_buf);
    a.sa = sa_buf;
    a.sw = sw;
    return true;
  };
  int tile = env ? atoi(env) : 0;
  if (env && tile == 0) return false;
  if (!env && a.M <= 64) return false;  // tools/gemm_sweep.py x3: fp32 tiles win to M = 64 (27 vs 31 us)
  // 7..11: gemm_x3<256,128> timing ablations (ABL 1, 2, 4, 5, 3), K % 32 == 0 only
  const int bms[17] = {0, 256, 128, 128, 256, 256, 256, 256, 256, 256, 256, 256, 256, 256, 256, 256, 256};
  const int bns[17] = {0, 128, 128, 64, 128, 128, 128, 128, 128, 128, 128, 128, 128, 128, 128, 128, 128};
  if (tile < 1 || tile > 16 || (((tile >= 7 && tile <= 11) || tile >= 13) && a.K % 32 != 0)) {
    tile = a.M > 256 ? 1 : 2;
  }
  const int bm = bms[tile], bn = bns[tile];
  const long tiles = (long)((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
  int S = 1;
  if (env_split) {
    S = std::max(1, atoi(env_split));
  } else if (tiles < 256) {
    S = (int)std::min<long>(256 / tiles, 8);
  }
  while (S > 1 && (!a.slab || (size_t)S * a.M * a.N * 4 > ws_bytes || a.K / S < 8 * 32)) --S;
  a.splits = S;
  a.kc = S > 1 ? ((a.K + S - 1) / S + 31) / 32 * 32 : a.K;
  if (S > 1) a.splits = (a.K + a.kc - 1) / a.kc;
  const dim3 grid((unsigned)(tiles * a.splits));
  const bool whole = a.K % 32 == 0;   // kc is a multiple of 32 too: no partial k tile anywhere
  // Stream-K (gemm_x3_sk) for the 256 x 128 tile when the split-K grid leaves CUs idle (below
  // 90 % of its last round: M = 800 -> 200 blocks, M = 1,576 -> 175): one block per CU, equal
  // k-iteration ranges, split tiles summed by streamk_fixup4_kernel.  C is complete on return
  // (a.splits = 1).  Product dispatch only (the tuning overrides keep the split-K forms).
  if (!env && !env_split && tile == 1 && a.vec_epi && a.slab && tiles >= 64) {
    static int cus = 0;
    if (cus <= 0) {
      int dev = 0, n = 0;
      cus = (hipGetDevice(&dev) == hipSuccess &&
             hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
             n > 0) ? n : 256;
    }
    const long blocks = tiles * a.splits;
    const long rounds = (blocks + cus - 1) / cus;
    const int KT = (a.K + 31) / 32;
    const long I = tiles * (long)KT;
    const int B = (int)std::min<long>(cus, I);
    const long per = I / B;
    if ((double)blocks / (double)(rounds * cus) < 0.9 && per >= 8) {
      // cycled stream-K (gemm_x3_csk).  Tuning build: AZ_CSK = "off" runs round 3's gemm_x3_sk,
      // "am,an,bf,at,bt" forces a plan (csk_make), AZ_CSK_MISS sets the planner's miss cost,
      // AZ_CSK_PRINT prints the plan
      CskPlan cq{};
      bool use_csk = true, ok = false;
#ifdef AZ_TUNING
      bool forced = false;
      static const char* env_csk = tuning_env("AZ_CSK");
      static const char* env_miss = tuning_env("AZ_CSK_MISS");
      int am = 0, an = 0, bf = 0, at = 0, bt = 0;
      use_csk = !env_csk || strcmp(env_csk, "off") != 0;
      if (use_csk && env_csk && sscanf(env_csk, "%d,%d,%d,%d,%d", &am, &an, &bf, &at, &bt) == 5) {
        forced = true;
        ok = csk_make(a.M, a.N, a.K, cus, am, an, bf, at, bt, cq);
      }
      if (use_csk && !forced)
        ok = csk_plan_cached(a.M, a.N, a.K, cus, env_miss ? atof(env_miss) : CSK_MISS_COST, cq);
      if (ok && tuning_env("AZ_CSK_PRINT"))
        fprintf(stderr, "csk M=%d: am=%d an=%d cycles=%d bf=%d tail=%d at=%d ct=%d bt=%d B=%d pieces=%d\n",
                a.M, cq.am, cq.an, cq.Cf, cq.bf, cq.tail, cq.at, cq.ct, cq.bt, cq.B, csk_max_pieces(cq));
#else
      ok = csk_plan_cached(a.M, a.N, a.K, cus, CSK_MISS_COST, cq);
#endif
      const int mp = use_csk && ok ? csk_max_pieces(cq) : 0;
#ifdef AZ_TUNING
      static const char* env_cring = tuning_env("AZ_P3_RING");
      const int csk_ring = env_cring ? atoi(env_cring) : 3;
#else
      constexpr int csk_ring = 3;
#endif
      // the finalize gives each lane one whole 64-column block of a row: N % 64 == 0, N <= 4,096
      if (use_csk && ok && a.he.part && whole && (p2 || h3) && a.N % 64 == 0 && a.N <= 64 * 64 &&
          (size_t)a.M * (a.N / 64) * mp * HEADS_TILE_SLOTS * 4 * 2 <= ws_bytes &&
          (size_t)4 * (a.N / 64) * mp * HEADS_TILE_SLOTS * 4 <= 65536) {   // finalize's LDS
        // the heads from the pieces (az_x3.h HeadsEpi, stream-K slots): no fix-up, no C
        if (p2) p2 = p2_prep();
        if (!p2) h3 = h3_scales();
        a.he.mp = mp;
        if (p2 && csk_ring == 2)
          hipLaunchKernelGGL((gemm_x3_csk<false, true, true, true, 2>), dim3(cq.B), dim3(512), 0, s, a, cq);
        else if (p2) hipLaunchKernelGGL((gemm_x3_csk<false, true, true, true>), dim3(cq.B), dim3(512), 0, s, a, cq);
        else hipLaunchKernelGGL((gemm_x3_csk<false, true, false, true>), dim3(cq.B), dim3(512), 0, s, a, cq);
        const int P = (a.N / 64) * mp;
        hipLaunchKernelGGL(heads_tiles_finalize_kernel<true>, dim3((a.M + 3) / 4), dim3(256),
                           (size_t)4 * P * HEADS_TILE_SLOTS * sizeof(float), s, a.he, a.M, a.N,
                           P, cq);
        a.splits = 1;
        a.heads_done = 1;
        return true;
      }
      if (use_csk && ok && mp * (size_t)a.M * a.N * 4 <= ws_bytes) {
        if (p2) p2 = p2_prep();
        if (!p2 && h3) h3 = h3_scales();
        if (p2 && csk_ring == 2)
          hipLaunchKernelGGL((gemm_x3_csk<false, true, true, false, 2>), dim3(cq.B), dim3(512), 0, s, a, cq);
        else if (p2) hipLaunchKernelGGL((gemm_x3_csk<false, true, true>), dim3(cq.B), dim3(512), 0, s, a, cq);
        else if (h3 && whole) hipLaunchKernelGGL((gemm_x3_csk<false, true>), dim3(cq.B), dim3(512), 0, s, a, cq);
        else if (h3) hipLaunchKernelGGL((gemm_x3_csk<true, true>), dim3(cq.B), dim3(512), 0, s, a, cq);
        else if (whole) hipLaunchKernelGGL((gemm_x3_csk<false, false>), dim3(cq.B), dim3(512), 0, s, a, cq);
        else hipLaunchKernelGGL((gemm_x3_csk<true, false>), dim3(cq.B), dim3(512), 0, s, a, cq);
        const long n4 = (long)a.M * (a.N / 4);
        hipLaunchKernelGGL(csk_fixup4_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s,
                           a, cq);
        a.splits = 1;
        return true;
      }
#ifdef AZ_TUNING
      const SkPlan q = sk_plan(a.M, a.N, a.K, 256, 128, B, false);
      if ((size_t)sk_max_pieces(q, a.N, 128) * a.M * a.N * 4 <= ws_bytes) {
        if (whole) hipLaunchKernelGGL((gemm_x3_sk<256, 128, 4, 2, false>), dim3(B), dim3(512), 0, s, a, q);
        else hipLaunchKernelGGL((gemm_x3_sk<256, 128, 4, 2, true>), dim3(B), dim3(512), 0, s, a, q);
        const long n4 = (long)a.M * (a.N / 4);
        hipLaunchKernelGGL(streamk_fixup4_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0,
                           s, a, 256, 128, q);
        a.splits = 1;
        return true;
      }
#endif
    }
  }
#ifdef AZ_TUNING
  // A split once into bf16 planes (x3_split_kernel) in the workspace after the slabs, only W
  // split in the tile (AZ_GEMM_X3APL=1): measured slower -- M = 512 82.8 vs 75.0 us incl. the
  // split launch, M = 4096 557 vs 514 (1.5x the A bytes through L2, no clock gain)
  static const char* env_apl = tuning_env("AZ_GEMM_X3APL");
  const bool want_apl = env_apl && atoi(env_apl) != 0;
  const size_t slab_bytes = a.splits > 1 ? ((size_t)a.splits * a.M * a.N * 4 + 255) / 256 * 256 : 0;
  const size_t apl_bytes = (size_t)3 * a.M * a.K * 2;
  if (want_apl && tile == 1 && whole && a.lda % 4 == 0 && a.slab &&
      slab_bytes + apl_bytes <= ws_bytes) {
    unsigned short* pl = reinterpret_cast<unsigned short*>(reinterpret_cast<char*>(a.slab) + slab_bytes);
    const long segs = (long)a.M * (a.K / 8);
    hipLaunchKernelGGL(x3_split_kernel, dim3((unsigned)((segs + 255) / 256)), dim3(256), 0, s,
                       a.A, a.lda, a.M, a.K, pl, (size_t)a.M * a.K);
    a.apl = pl;
    a.apl_plane = (size_t)a.M * a.K;
    hipLaunchKernelGGL((gemm_x3<256, 128, 4, 2, false, 0, true>), grid, dim3(512), 0, s, a);
    return true;
  }
#endif
#define AZ_X3(BM_, BN_, WM_, WN_)                                                              \
  if (whole) hipLaunchKernelGGL((gemm_x3<BM_, BN_, WM_, WN_, false>), grid, dim3(64 * WM_ * WN_), \
                                0, s, a);                                                      \
  else hipLaunchKernelGGL((gemm_x3<BM_, BN_, WM_, WN_, true>), grid, dim3(64 * WM_ * WN_), 0, s, a);
#define AZ_H3(BM_, BN_, WM_, WN_)                                                              \
  if (whole) hipLaunchKernelGGL((gemm_x3<BM_, BN_, WM_, WN_, false, 0, false, 32, true>), grid,  \
                                dim3(64 * WM_ * WN_), 0, s, a);                                \
  else hipLaunchKernelGGL((gemm_x3<BM_, BN_, WM_, WN_, true, 0, false, 32, true>), grid,         \
                          dim3(64 * WM_ * WN_), 0, s, a);
  if (p2 && (tile == 1 || tile == 2) && p2_prep()) {
    // the 256 x 128 tile's LDS-DMA ring: 3 stages (two in flight) in the product; the tuning
    // build's AZ_P3_RING=2 keeps round 5's double buffer for A/B runs (same bits)
    static const char* env_ring = tuning_env("AZ_P3_RING");
    const int ring = env_ring ? atoi(env_ring) : 3;
    static const char* env_abl = tuning_env("AZ_P3_ABL");
    const int abl = env_abl ? atoi(env_abl) : 0;
    if (false) {
    }
#ifdef AZ_TUNING
    else if (tile == 1 && abl == 1)
      hipLaunchKernelGGL((gemm_p3<256, 128, 4, 2, true, 3, 1>), grid, dim3(512), 0, s, a);
    else if (tile == 1 && abl == 2)
      hipLaunchKernelGGL((gemm_p3<256, 128, 4, 2, true, 3, 2>), grid, dim3(512), 0, s, a);
    else if (tile == 1 && abl == 4)
      hipLaunchKernelGGL((gemm_p3<256, 128, 4, 2, true, 3, 4>), grid, dim3(512), 0, s, a);
    else if (tile == 1 && abl == 5)
      hipLaunchKernelGGL((gemm_p3<256, 128, 4, 2, true, 3, 5>), grid, dim3(512), 0, s, a);
    else if (tile == 1 && abl == 6)
      hipLaunchKernelGGL((gemm_p3<256, 128, 4, 2, true, 3, 6>), grid, dim3(512), 0, s, a);
    else if (tile == 1 && tuning_env("AZ_P3_WIDE")) {
      // 256 x 256 tiles (waves 4 x 2 of 64 x 128): 2/3 of the 256 x 128 tile's DMA bytes per
      // flop; AZ_P3_WIDE_SPLITS = its split-K (default: none)
      static const char* env_ws = tuning_env("AZ_P3_WIDE_SPLITS");
      int S = env_ws ? atoi(env_ws) : 1;
      while (S > 1 && (!a.slab || (size_t)S * a.M * a.N * 4 > ws_bytes)) --S;
      a.kc = S > 1 ? ((a.K + S - 1) / S + 31) / 32 * 32 : a.K;
      a.splits = S > 1 ? (a.K + a.kc - 1) / a.kc : 1;
      const dim3 gw((unsigned)(((a.M + 255) / 256) * ((a.N + 255) / 256) * a.splits));
      hipLaunchKernelGGL((gemm_p3<256, 256, 4, 2, true>), gw, dim3(512), 0, s, a);
    }
    else if (tile == 1 && ring == 2) {
      if (a.he.part) {
        hipLaunchKernelGGL((gemm_p3<256, 128, 4, 2, true, 2, 0, true>), grid, dim3(512), 0, s, a);
        launch_heads_finalize(a, s);
      } else {
        hipLaunchKernelGGL((gemm_p3<256, 128, 4, 2, true, 2>), grid, dim3(512), 0, s, a);
      }
    }
#endif
    else if (a.he.part) {
      if (tile == 1)
        hipLaunchKernelGGL((gemm_p3<256, 128, 4, 2, true, 3, 0, true>), grid, dim3(512), 0, s, a);
      else
        hipLaunchKernelGGL((gemm_p3<128, 128, 2, 2, true, 2, 0, true>), grid, dim3(256), 0, s, a);
      launch_heads_finalize(a, s);
    }
    else if (tile == 1) hipLaunchKernelGGL((gemm_p3<256, 128, 4, 2, true, 3>), grid, dim3(512), 0, s, a);
    else hipLaunchKernelGGL((gemm_p3<128, 128, 2, 2, true>), grid, dim3(256), 0, s, a);
    return true;
  }
  if (h3 && (tile == 1 || tile == 2) && h3_scales()) {
    if (a.he.part && whole) {     // the heads from the tiles, as on the P2 tiles (same bits)
      if (tile == 1)
        hipLaunchKernelGGL((gemm_x3<256, 128, 4, 2, false, 0, false, 32, true, true>), grid,
                           dim3(512), 0, s, a);
      else
        hipLaunchKernelGGL((gemm_x3<128, 128, 2, 2, false, 0, false, 32, true, true>), grid,
                           dim3(256), 0, s, a);
      launch_heads_finalize(a, s);
      return true;
    }
    if (tile == 1) { AZ_H3(256, 128, 4, 2) }
    else { AZ_H3(128, 128, 2, 2) }
    return true;
  }
  switch (tile) {
    case 1: AZ_X3(256, 128, 4, 2) break;
#ifdef AZ_TUNING
    case 3: AZ_X3(128, 64, 2, 1) break;
    case 4: AZ_X3(256, 128, 2, 2) break;
    // wave-specialised x3 (measured no faster: M = 512 84 vs 78 us, M = 4096 541 vs 518)
    case 5:
      if (whole) hipLaunchKernelGGL((gemm_x3ws<256, 128, 4, 2, false>), grid, dim3(768), 0, s, a);
      else hipLaunchKernelGGL((gemm_x3ws<256, 128, 4, 2, true>), grid, dim3(768), 0, s, a);
      break;
    case 12:
      if (whole) hipLaunchKernelGGL((gemm_x3pp<256, 128, false>), grid, dim3(512), 0, s, a);
      else hipLaunchKernelGGL((gemm_x3pp<256, 128, true>), grid, dim3(512), 0, s, a);
      break;
    case 7: hipLaunchKernelGGL((gemm_x3<256, 128, 4, 2, false, 1>), grid, dim3(512), 0, s, a); break;
    case 8: hipLaunchKernelGGL((gemm_x3<256, 128, 4, 2, false, 2>), grid, dim3(512), 0, s, a); break;
    case 9: hipLaunchKernelGGL((gemm_x3<256, 128, 4, 2, false, 4>), grid, dim3(512), 0, s, a); break;
    case 10: hipLaunchKernelGGL((gemm_x3<256, 128, 4, 2, false, 5>), grid, dim3(512), 0, s, a); break;
    case 11: hipLaunchKernelGGL((gemm_x3<256, 128, 4, 2, false, 3>), grid, dim3(512), 0, s, a); break;
    case 13: hipLaunchKernelGGL((gemm_x3<256, 128, 4, 2, false, 8>), grid, dim3(512), 0, s, a); break;
    case 14:   // 16x16x32 MFMA blocks
      if (whole) hipLaunchKernelGGL((gemm_x3<256, 128, 4, 2, false, 0, false, 16>), grid, dim3(512), 0, s, a);
      else hipLaunchKernelGGL((gemm_x3<256, 128, 4, 2, true, 0, false, 16>), grid, dim3(512), 0, s, a);
      break;
    case 6:   // 4 consumer waves with 128 x 64 wave tiles (two waves per SIMD)
      if (whole) hipLaunchKernelGGL((gemm_x3ws<256, 128, 2, 2, false>), grid, dim3(512), 0, s, a);
      else hipLaunchKernelGGL((gemm_x3ws<256, 128, 2, 2, true>), grid, dim3(512), 0, s, a);
      break;
#endif
    default: AZ_X3(128, 128, 2, 2) break;
  }
#undef AZ_X3
  return true;
}

// True when the 256x128 grid is >= 4 rounds of one block per CU and its last round is >= 95 %
// full (wave quantisation otherwise costs the 8-wave tile its edge: M = 8,192 / 16,384).
static bool full_waves_256x128(int M, int N) {
  const long tiles = (long)((M + 255) / 256) * ((N + 127) / 128);
  const long rounds = (tiles + 255) / 256;
  return rounds >= 4 && (double)tiles / (double)(rounds * 256) >= 0.95;
}

// The GEMM without its split-K reduction: when the plan splits K, the raw partial sums are left
// in d->ws as slabs [*splits_out][M][N] and C is NOT written (the caller reduces them, e.g.
// fused with its consumer: az_transform_heads_fwd); otherwise C is written and *splits_out = 1.
int gemm_f32_partial(const az_gemm_desc* d, hipStream_t s, int* splits_out, const PreSplitA* pre,
                     const HeadsEpi* he, bool* heads_done) {
  *splits_out = 1;
  if (heads_done) *heads_done = false;
  AZ_REQUIRE(d != nullptr, AZ_EINVAL, "az_gemm_f32: null descriptor");
  AZ_REQUIRE(d->M >= 0 && d->N >= 0 && d->K >= 0, AZ_EINVAL, "az_gemm_f32: negative size");
  if (d->M == 0 || d->N == 0) return AZ_OK;
  AZ_REQUIRE(d->A && d->B && d->C, AZ_EINVAL, "az_gemm_f32: null A/B/C");
  const bool akm = d->a_kmajor != 0, bkm = d->b_kmajor != 0;
  AZ_REQUIRE(!(akm || bkm) || d->K % 4 == 0, AZ_EINVAL,
             "az_gemm_f32: K=%d must be a multiple of 4 for a K-major operand", d->K);
  AZ_REQUIRE(d->lda % 4 == 0 && aligned16(d->A), AZ_EINVAL, "az_gemm_f32: A needs lda%%4==0, 16B alignment");
  AZ_REQUIRE(d->ldb % 4 == 0 && aligned16(d->B), AZ_EINVAL, "az_gemm_f32: B needs ldb%%4==0, 16B alignment");
  if (d->A2) {
    AZ_REQUIRE(akm, AZ_EINVAL, "az_gemm_f32: A2 needs a K-major A");
    AZ_REQUIRE(d->K0 % 4 == 0 && d->K0 > 0 && d->K0 < d->K, AZ_EINVAL,
               "az_gemm_f32: K0 must be a multiple of 4 inside (0,K)");
    AZ_REQUIRE(d->lda2 % 4 == 0 && aligned16(d->A2), AZ_EINVAL, "az_gemm_f32: A2 needs lda2%%4==0, 16B alignment");
  }
  AZ_REQUIRE(!d->a_rows || akm, AZ_EINVAL, "az_gemm_f32: a_rows needs a K-major A");
  AZ_REQUIRE(!d->b_rows || !bkm, AZ_EINVAL, "az_gemm_f32: b_rows needs an N-major B");
  AZ_REQUIRE(akm || (d->M + 3) / 4 * 4 <= d->lda, AZ_EINVAL,
             "az_gemm_f32: M-major A needs round_up(M,4) <= lda");
  AZ_REQUIRE(bkm || (d->N + 3) / 4 * 4 <= d->ldb, AZ_EINVAL,
             "az_gemm_f32: N-major B needs round_up(N,4) <= ldb");
  AZ_REQUIRE(d->act >= 0 && d->act <= AZ_ACT_DRELU, AZ_EINVAL, "az_gemm_f32: bad act %d", d->act);
  AZ_REQUIRE(d->act != AZ_ACT_DRELU || d->G, AZ_EINVAL, "az_gemm_f32: DRELU needs G");
  AZ_REQUIRE(!(d->act == AZ_ACT_DRELU && d->R), AZ_EINVAL, "az_gemm_f32: DRELU excludes R");

  GemmArgs a = {};
  a.M = d->M; a.N = d->N; a.K = d->K;
  a.A = d->A; a.lda = d->lda; a.A2 = d->A2; a.lda2 = d->lda2; a.K0 = d->A2 ? d->K0 : d->K;
  a.a_rows = d->a_rows; a.B = d->B; a.ldb = d->ldb; a.b_rows = d->b_rows;
  a.bias = d->bias; a.act = d->act; a.R = d->R; a.ldr = d->ldr; a.G = d->G; a.ldg = d->ldg;
  a.beta = d->beta; a.C = d->C; a.ldc = d->ldc; a.c_rows = d->c_rows;
  a.C2 = d->C2; a.ldc2 = d->ldc2;
  a.slab = static_cast<float*>(d->ws);
  a.splits = 1; a.kc = d->K;
  static const char* env_abl = tuning_env("AZ_GEMM_ABLATE");
  a.ablate = env_abl ? atoi(env_abl) : 0;
  static const bool no_vec = tuning_env("AZ_GEMM_NOVEC") != nullptr;   // A/B experiments
  a.vec_epi = !no_vec && d->N % 4 == 0 && d->ldc % 4 == 0 && aligned16(d->C) &&
              (!d->C2 || (d->ldc2 % 4 == 0 && aligned16(d->C2))) &&
              (!d->R || (d->ldr % 4 == 0 && aligned16(d->R))) &&
              (!d->G || (d->ldg % 4 == 0 && aligned16(d->G))) && (!d->bias || aligned16(d->bias));

  if (d->M <= 8 && akm && bkm && !d->C2 && d->act != AZ_ACT_DRELU) {
    launch_gemv(a, s);
    return check_launch("gemv_f32");
  }
  if (akm && bkm && launch_tall(a, s)) return check_launch("gemm_tall");
  // gemm_kslice: measured slower than the split-K tile so far (111 vs 103 us at M = 512), so
  // only the tuning build runs it, on request (AZ_GEMM_KSLICE=1, tools/gemm_sweep.py kslice)
  static const bool use_kslice = tuning_env("AZ_GEMM_KSLICE") != nullptr;
  if (akm && bkm && use_kslice && !d->A2 && !d->a_rows && !d->b_rows && !d->C2 && !d->R &&
      !d->G && d->beta == 0.f && d->act != AZ_ACT_DRELU && aligned16(d->A) && aligned16(d->B)) {
    const int nn = kslice_narrow(a);
    if (nn >= 0) {
      const dim3 grid(a.M / 32 * 16);
      hipLaunchKernelGGL((gemm_kslice<7, 6>), grid, dim3(512), 0, s, a, nn);
      return check_launch("gemm_kslice");
    }
  }
  const bool glds_ok = akm && bkm && !d->A2 && !d->a_rows;
  // the heads from the tiles (az_x3.h HeadsEpi): only a plain y = x W^T + b, whole 32-column
  // chunks, A <= 8; launch_x3 takes it on its P2 split-K tiles and says so in a.heads_done
  if (he && he->part && he->A <= 8 && d->N % 32 == 0 && d->act == AZ_ACT_NONE && !d->R &&
      !d->G && !d->C2 && d->beta == 0.f && !d->c_rows && (!d->bias || aligned16(d->bias)))
    a.he = *he;
  if (glds_ok && d->M > 8 && d->K >= 1024 && d->N >= 256 && launch_x3(a, d->ws_bytes, s, pre)) {
    *splits_out = a.splits;
    if (heads_done) *heads_done = a.heads_done != 0;
    return check_launch("gemm_x3");
  }
  a.he = HeadsEpi{};
  // tile choice (tuning override for experiments: AZ_GEMM_CFG=<index into kCfgs>)
  static const char* env_cfg = tuning_env("AZ_GEMM_CFG");
  int cfg = 0;
  int s256 = 0;   // split factor when the 256x128 8-wave tile packs the chip (one block per CU)
  if (env_cfg) {
    cfg = std::min(std::max(atoi(env_cfg), 0), kNumCfgs - 1);
    if (cfg >= 6 && !glds_ok) cfg = 0;
  } else if (glds_ok && d->M > 256 && (s256 = splits_256x128(d->M, d->N, d->K, d->ws_bytes)) > 0) {
    // 256x128 tile, 8 waves, one block per CU, K split so the grid fills >= 85 % of the CUs
    // (tools/gemm_sweep.py glds on MI355X, M = 512: 106 us vs 113 us for 128x128 x 5)
    cfg = 24;
  } else if (glds_ok && d->N >= 1024 && d->K >= 1024 && full_waves_256x128(d->M, d->N)) {
    // large M whose 256x128 grid is (nearly) whole rounds of 256 blocks: the 8-wave tile's
    // steady state wins (tools/gemm_sweep.py bigm, M = 65,536: 130 vs 109 TFLOP/s for 128x64)
    cfg = 24;
  } else if (glds_ok && d->M > 128) {
    // LDS-DMA tiles (tools/gemm_sweep.py glds on MI355X): 128x64 once the grid fills the chip,
    // 128x128 + split-K below that
    const long t128 = (long)((d->M + 127) / 128) * ((d->N + 127) / 128);
    cfg = t128 >= 256 ? 8 : 6;
  } else {
    cfg = 0;  // register-staged 64x64x32: gathered / concatenated operands, small M
  }
  static const char* env_ring = tuning_env("AZ_GEMM_RING");   // experiment: 3-buffer 256x128
  if (cfg == 24 && env_ring) {
    const int r = atoi(env_ring);
    cfg = r == 3 ? 29 : r == 4 ? 31 : r == 5 ? 30 : r == 6 ? 32 : 24;
  }
  const TileCfg& tc = kCfgs[cfg];
  plan(a, tc.bm, tc.bn, tc.bk, d->ws_bytes);
  const bool is128 = tc.bm == 128 && tc.bn == 128 && cfg >= 6;
  if (s256 > 0 && !tuning_env("AZ_GEMM_SPLITS")) {
    a.splits = s256;
    a.kc = s256 > 1 ? ((a.K + s256 - 1) / s256 + 31) / 32 * 32 : a.K;
    if (s256 > 1) a.splits = (a.K + a.kc - 1) / a.kc;
  } else if (is128 && !tuning_env("AZ_GEMM_SPLITS")) {
    const int S = glds_splits(a, (long)((a.M + 127) / 128) * ((a.N + 127) / 128), d->ws_bytes);
    a.splits = S;
    a.kc = S > 1 ? ((a.K + S - 1) / S + 31) / 32 * 32 : a.K;
    if (S > 1) a.splits = (a.K + a.kc - 1) / a.kc;
  }
  launch_cfg(cfg, a, akm, bkm, s);
  *splits_out = a.splits;
  return check_launch("gemm_f32_mfma");
}

// Sums the split-K slabs a gemm_f32_partial call left in d->ws (in slab order) and applies d's
// epilogue into d->C.
int splitk_reduce(const az_gemm_desc* d, int splits, hipStream_t s) {
  GemmArgs a = {};
  a.M = d->M; a.N = d->N;
  a.bias = d->bias; a.act = d->act; a.R = d->R; a.ldr = d->ldr; a.G = d->G; a.ldg = d->ldg;
  a.beta = d->beta; a.C = d->C; a.ldc = d->ldc; a.c_rows = d->c_rows;
  a.C2 = d->C2; a.ldc2 = d->ldc2;
  a.slab = static_cast<float*>(d->ws);
  a.splits = splits;
  const long total = (long)a.M * a.N;
  static const bool no_vec = tuning_env("AZ_GEMM_NOVEC") != nullptr;   // A/B experiments
  const bool vec = !no_vec && d->N % 4 == 0 && d->ldc % 4 == 0 && aligned16(d->C) &&
                   (!d->C2 || (d->ldc2 % 4 == 0 && aligned16(d->C2))) &&
                   (!d->R || (d->ldr % 4 == 0 && aligned16(d->R))) &&
                   (!d->G || (d->ldg % 4 == 0 && aligned16(d->G))) &&
                   (!d->bias || aligned16(d->bias)) && aligned16(d->ws);
  if (vec && splits >= 2 && splits <= 8) {
    // float4 per lane: 38.7 MB at M = 512, N = 3136, S = 5 in one pass (the scalar
    // grid-stride kernel took 10.6 us for it)
    const int blocks = (int)((total / 4 + 255) / 256);
    switch (splits) {
      case 2: hipLaunchKernelGGL(splitk_reduce4_kernel<2>, dim3(blocks), dim3(256), 0, s, a); break;
      case 3: hipLaunchKernelGGL(splitk_reduce4_kernel<3>, dim3(blocks), dim3(256), 0, s, a); break;
      case 4: hipLaunchKernelGGL(splitk_reduce4_kernel<4>, dim3(blocks), dim3(256), 0, s, a); break;
      case 5: hipLaunchKernelGGL(splitk_reduce4_kernel<5>, dim3(blocks), dim3(256), 0, s, a); break;
      case 6: hipLaunchKernelGGL(splitk_reduce4_kernel<6>, dim3(blocks), dim3(256), 0, s, a); break;
      case 7: hipLaunchKernelGGL(splitk_reduce4_kernel<7>, dim3(blocks), dim3(256), 0, s, a); break;
      default: hipLaunchKernelGGL(splitk_reduce4_kernel<8>, dim3(blocks), dim3(256), 0, s, a); break;
    }
    return check_launch("splitk_reduce4_kernel");
  }
  const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, s, a);
  return check_launch("splitk_reduce_kernel");
}

// splitk_reduce, and C's rows split for a P2 GEMM that takes C as its A (PreSplitA{planes, sc}:
// planes [2][M][N] fp16, sc [2][M]); C's bits are splitk_reduce's.  Returns 1 when launched, 0 when
// the shapes / epilogue do not qualify (nothing launched: the caller reduces the usual way), or a
// negative AZ_E* code.
int splitk_reduce_split(const az_gemm_desc* d, int splits, unsigned short* planes, float* sc,
                        hipStream_t s, bool write_c) {
  if (!(splits >= 2 && splits <= 8 && d->N % 32 == 0 && d->N <= 4096 && d->M > 0 && !d->C2 &&
        !d->R && !d->G && !d->c_rows && d->beta == 0.f &&
        (d->act == AZ_ACT_NONE || d->act == AZ_ACT_RELU) && d->ldc % 4 == 0 && aligned16(d->C) &&
        (!d->bias || aligned16(d->bias)) && aligned16(d->ws) && planes && sc &&
        aligned16(planes)))
    return 0;
  GemmArgs a = {};
  a.M = d->M; a.N = d->N;
  a.bias = d->bias; a.act = d->act; a.C = write_c ? d->C : nullptr; a.ldc = d->ldc;
  a.slab = static_cast<float*>(d->ws);
  a.splits = splits;
  // one 8-column chunk per thread (N = 3,136: 7 waves; 8.5 -> 8.35 us per M = 512 launch against
  // two chunks on 4 waves, profiles/r06/reduce_ab)
  const int T = (d->N / 8 + 63) / 64 * 64;
  switch (splits) {
#define AZ_RS(SS) case SS: hipLaunchKernelGGL((splitk_reduce_split_kernel<SS, 1>), dim3(a.M), dim3(T), \
                                             0, s, a, planes, sc); break;
    AZ_RS(2) AZ_RS(3) AZ_RS(4) AZ_RS(5) AZ_RS(6) AZ_RS(7) default: AZ_RS(8)
#undef AZ_RS
  }
  const int rc = check_launch("splitk_reduce_split_kernel");
  return rc == AZ_OK ? 1 : rc;
}

#ifdef AZ_P3_STAMPS
}  // namespace az
extern "C" int az_debug_p3_stamps(void* buf) {   // timing-experiment library only
  return hipMemcpyToSymbol(HIP_SYMBOL(az::g_p3_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
}
namespace az {
#endif

// Whether az_gemm_f32(d), given a PreSplitA of its A, takes the P2 tiles and so never reads
// d->A: gemm_f32_partial's and launch_x3's conditions for that path (product dispatch: M > 64,
// K-major 32-k operands, the workspace for the scales, registered W) and W's planes in the cache
// (w_planes, which fills it now if needed: the later p2_prep of the same call then returns them)
bool gemm_p2_certain(const az_gemm_desc* d, hipStream_t s) {
  if (!(d->a_kmajor && d->b_kmajor && !d->A2 && !d->a_rows && !d->b_rows && d->M > 64 &&
        d->K >= 1024 && d->N >= 256 && d->K % 32 == 0 && d->lda % 4 == 0 && d->ldb % 4 == 0 &&
        aligned16(d->A) && aligned16(d->B) && d->ws && d->act != AZ_ACT_DRELU))
    return false;
  if (tuning_env("AZ_GEMM_X3") || tuning_env("AZ_GEMM_SPLITS") || tuning_env("AZ_GEMM_NOP2") ||
      tuning_env("AZ_GEMM_PREC") || tuning_env("AZ_GEMM_KSLICE"))
    return false;
  const size_t sa_bytes = ((size_t)2 * (d->M + d->N) * sizeof(float) + 255) / 256 * 256;
  if (d->ws_bytes < sa_bytes + 512) return false;
  if (!weights_registered(d->B, d->N, d->K, d->ldb)) return false;
  const float* sw = nullptr;
  return w_planes(d->B, d->N, d->K, d->ldb, s, &sw) != nullptr;
}

// Whether a GEMM with weight w (n x k, row stride ld) takes the P2 path's cached weight planes,
// i.e. whether splitting its A ahead of the call (PreSplitA) can pay off.
bool gemm_p2_weights(const float* w, int n, int k, int ld) {
  return k % 32 == 0 && weights_registered(w, n, k, ld);
}

// gemv_side_heads for the batch-1 leaf and small speculative batches: d must be M <= 8 (the
// same per-row arithmetic as gemv for that M) with K-major operands, a plain
// bias/activation epilogue and 3072 < K <= 3328 (output_transform.0 at F = 3136), and h at most
// 8 actions; returns 1 when launched, 0 when the shapes do not qualify (nothing launched), or
// a negative AZ_E* code.
int gemv1_with_side_heads(const az_gemm_desc* d, const SideHeads* h, hipStream_t s) {
  if (!(d->M >= 1 && d->M <= 8 && d->a_kmajor && d->b_kmajor && !d->A2 && !d->a_rows && !d->C2 &&
        !d->R &&
        !d->G && d->act != AZ_ACT_DRELU && d->K > 3072 && d->K <= 3328 && d->K % 4 == 0 &&
        d->lda % 4 == 0 && d->ldb % 4 == 0 && aligned16(d->A) && aligned16(d->B) &&
        h->A >= 1 && h->A <= 8 && h->K % 4 == 0 && h->ldx % 4 == 0 &&
        (h->K + HEADS_KC - 1) / HEADS_KC <= HEADS_ROWS_MAXC && aligned16(h->x) &&
        aligned16(h->wp) && aligned16(h->wv)))
    return 0;
  GemmArgs a = {};
  a.M = d->M; a.N = d->N; a.K = d->K;
  a.A = d->A; a.lda = d->lda; a.K0 = d->K;
  a.B = d->B; a.ldb = d->ldb;
  a.bias = d->bias; a.act = d->act; a.beta = d->beta; a.C = d->C; a.ldc = d->ldc;
  a.splits = 1; a.kc = d->K;
  const int nblk = (a.N + 4 * 2 - 1) / (4 * 2);
  const dim3 grid(nblk + h->B), blk(256);
  if (a.M == 1) hipLaunchKernelGGL((gemv_side_heads<13, 2, 1>), grid, blk, 0, s, a, *h, nblk);
  else if (a.M == 2) hipLaunchKernelGGL((gemv_side_heads<13, 2, 2>), grid, blk, 0, s, a, *h, nblk);
  else hipLaunchKernelGGL((gemv_side_heads<13, 2, 3>), grid, blk, 0, s, a, *h, nblk);
  const int rc = check_launch("gemv_side_heads");
  return rc == AZ_OK ? 1 : rc;
}

// The batch <= 2 leaf of az_c4_eval_fwd as ONE c4_leaf_kernel launch (see there).  Returns 1
// when launched, 0 when it does not apply (shapes, no counters, or the grid would not be
// resident at once on this device), or a negative AZ_E* code.
int c4_leaf_fwd(const az_c4_eval* e, const int8_t* boards, int B, float* pi, float* v, float* gpi,
                float* gv, hipStream_t s) {
  const int F = 3136, nch = (F + HEADS_KC - 1) / HEADS_KC;
  // 1-2 rows: 3 or more take the four launches, faster there (tools/leaf_rows_probe.py, r03p:
  // 1 row 39.8 vs 45.6 us, 2 rows 44.8 vs 47.9, 3 rows 53.8 vs 50.6, 8 rows 75.0 vs 58.4)
  if (!(e->sync && e->err && B >= 1 && B <= 2 && v && gv && e->A >= 1 && e->A <= 8 &&
        e->ot0_w && e->ot0_b && e->ot2_w && e->ot2_b && e->hidden && e->y && e->glogp && e->ws &&
        e->ws_bytes >= (size_t)B * nch * 9 * 4 && aligned16(e->feat) && aligned16(e->hidden) &&
        aligned16(e->y) && aligned16(e->ot0_w) && aligned16(e->ot2_w) &&
        aligned16(e->fc_policy_w) && aligned16(e->fc_value_w)))
    return 0;
  static_assert(kSyncInts <= 4096, "az_c4_eval.sync holds 4096 ints");
  const int mk = B;
  const int ng = F / 8;
  const int grid = 4 * B + B + ng;
  static int cap[4] = {-1, -1, -1, -1};
  if (cap[mk] < 0) {
    int dev = 0, cus = 0, nb = 0;
    const void* k = mk == 1 ? reinterpret_cast<const void*>(&c4_leaf_kernel<1>)
                            : reinterpret_cast<const void*>(&c4_leaf_kernel<2>);
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 256, 0) != hipSuccess)
      cap[mk] = 0;
    else
      cap[mk] = nb * cus;
  }
  if (grid > cap[mk]) return 0;
  LeafArgs a = {};
  a.boards = boards; a.B = B;
  a.w1 = e->conv1_w; a.b1 = e->conv1_b; a.w2 = e->conv2_w; a.b2 = e->conv2_b;
  a.feat = e->feat;
  auto gemv_args = [&](const float* A, const float* W, const float* bias, int act, float* C) {
    GemmArgs g = {};
    g.M = B; g.N = F; g.K = F;
    g.A = A; g.lda = F; g.K0 = F; g.B = W; g.ldb = F;
    g.bias = bias; g.act = act; g.C = C; g.ldc = F;
    g.splits = 1; g.kc = F;
    return g;
  };
  a.g1 = gemv_args(e->feat, e->ot0_w, e->ot0_b, AZ_ACT_RELU, e->hidden);
  a.g2 = gemv_args(e->hidden, e->ot2_w, e->ot2_b, AZ_ACT_NONE, e->y);
  a.sh = {e->feat, F, F, B, e->fc_policy_w, e->fc_policy_b, e->A, e->fc_value_w, e->fc_value_b,
          e->logp, pi, v};
  a.ht = {e->fc_policy_w, e->fc_policy_b, e->A, e->fc_value_w, e->fc_value_b, e->glogp, gpi, gv,
          static_cast<float*>(e->ws)};
  a.sync = e->sync; a.err = e->err; a.ng = ng;
#ifdef AZ_TUNING
  static const bool trace = tuning_env("AZ_LEAF_TRACE") != nullptr;
  if (trace) {
    if (!g_leaf_trace && hipMalloc(&g_leaf_trace, 2 * LE_N * 8) != hipSuccess) return 0;
    unsigned long long init[2 * LE_N];
    for (int i = 0; i < LE_N; ++i) { init[2 * i] = ~0ull; init[2 * i + 1] = 0; }
    if (hipMemcpy(g_leaf_trace, init, sizeof(init), hipMemcpyHostToDevice) != hipSuccess) return 0;
    a.trace = g_leaf_trace;
  }
#endif
  if (mk == 1) hipLaunchKernelGGL(c4_leaf_kernel<1>, dim3(grid), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(c4_leaf_kernel<2>, dim3(grid), dim3(256), 0, s, a);
  const int rc = check_launch("c4_leaf_kernel");
  return rc == AZ_OK ? 1 : rc;
}

#ifdef AZ_TUNING
// tools/leaf_probe.py: the last traced launch's [event][min, max] stamps (synchronous)
extern "C" int az_tuning_leaf_trace(unsigned long long* out) {
  if (!g_leaf_trace) return -1;
  return hipMemcpy(out, g_leaf_trace, 2 * LE_N * 8, hipMemcpyDeviceToHost) == hipSuccess ? LE_N : -1;
}
#endif

int gemm_f32(const az_gemm_desc* d, hipStream_t s) {
  int splits = 1;
  int rc = gemm_f32_partial(d, s, &splits, nullptr, nullptr, nullptr);
  if (rc || splits <= 1) return rc;
  return splitk_reduce(d, splits, s);
}

}  // namespace az

extern "C" int az_gemm_f32(const az_gemm_desc* d, void* stream) {
  return az::gemm_f32(d, az::as_stream(stream));
}

// The MFMA products per fp32 product az_gemm_f32 uses for a plain K-major M x N x K GEMM with
// ws_bytes of workspace (the dispatch rules of gemm_f32 / launch_x3, product build): 3 = the
// fp16 form (h3), 6 = the bf16 form (x3), 1 = an fp32 MFMA tile, 0 = the fp32 GEMV (M <= 8).
extern "C" int az_gemm_form(int M, int N, int K, size_t ws_bytes) {
  if (M <= 8) return 0;
  if (!(M > 64 && K >= 1024 && N >= 256)) return 1;
  const size_t sa_bytes = ((size_t)2 * M * sizeof(float) + 255) / 256 * 256;
  return ws_bytes >= sa_bytes + 256 ? 3 : 6;
}
