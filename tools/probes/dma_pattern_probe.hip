// Probe: how fast one CU's LDS-DMA (global_load_lds_dwordx4) fills the gemm_p3 stage image,
// by the shape of each 1-KB piece.  Every block of the M = 512 headline grid (2 x 25 tiles of
// 256 x 128, split-K 5 = 250 blocks, xcd_swizzle + tile_of order as az_gemm.hip) streams its 20
// stages of (256 + 128) rows x 2 fp16 planes x 32 k (48 KB) into a double-buffered LDS ring,
// one raw barrier per stage, no MFMA: the DMA alone, at the operands' real L2 sharing.
//   mode 0: the product's pieces: 16 rows x 64 B of ONE plane (planes stored [2][rows][K])
//   mode 1: full lines: 8 rows x 128 B = both planes' 64 B of a row (planes interleaved per 32-k
//           step, [rows][K/32][2][32]); the same bytes into the same LDS buffer size
//   mode 2: 1 KB contiguous per piece (the bytes of mode 0, no row structure): the ceiling
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/dma_pattern_probe tools/probes/dma_pattern_probe.hip
//   depth 1: one stage in flight (the product's ring); depth 2: two (a three-buffer ring)
//   dma_pattern_probe [iters]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

constexpr int M = 512, N = 3136, K = 3136, BM = 256, BN = 128, ROWS = BM + BN;
constexpr int KT = K / 32, SPLITS = 5, KC = (KT + SPLITS - 1) / SPLITS;   // 20 stages per block
constexpr int NW = 8, PIECES = 2 * ROWS / 16, PPW = PIECES / NW;         // 48 pieces, 6 per wave
constexpr int BUF = 2 * ROWS * 64;                                        // 48 KB

__device__ __forceinline__ int xcd_swizzle(int bid, int nwg) {
  const int xcd = bid & 7, local = bid >> 3;
  const int base = nwg >> 3, rem = nwg & 7;
  return xcd * base + min(xcd, rem) + local;
}

template <int MODE, int DEPTH>
__global__ __launch_bounds__(512) void fill(const unsigned short* __restrict__ apl,
                                            const unsigned short* __restrict__ bpl,
                                            unsigned* sink) {
  __shared__ __attribute__((aligned(1024))) char smem[(DEPTH + 1) * BUF];
  const int mt_n = M / BM, nt_n = (N + BN - 1) / BN, tiles = mt_n * nt_n;
  const int bid = xcd_swizzle(blockIdx.x, tiles * SPLITS);
  const int sp = bid / tiles, t = bid - sp * tiles, mt = t % mt_n, nt = t / mt_n;
  const int k0 = sp * KC, nk = min(KT, k0 + KC) - k0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned short* src[PPW];
  int stride[PPW];
#pragma unroll
  for (int q = 0; q < PPW; ++q) {
    const int piece = q * NW + wave;
    if (MODE == 0) {            // plane-major image rows, 4 lanes per 64-B row slice
      const int R = piece * 16 + (lane >> 2), pl = R / ROWS, r = R % ROWS;
      const int c = (lane & 3) ^ ((r >> 2) & 3);
      const unsigned short* base = r < BM ? apl + (size_t)pl * M * K + (size_t)(mt * BM + r) * K
                                          : bpl + (size_t)pl * N * K +
                                                (size_t)min(nt * BN + r - BM, N - 1) * K;
      src[q] = base + 8 * c;
    } else if (MODE == 1) {     // row-major image of 128-B rows (both planes), 8 lanes per row
      const int r = piece * 8 + (lane >> 3), u = (lane & 7) ^ ((r >> 1) & 7);
      const unsigned short* base = r < BM ? apl + (size_t)(mt * BM + r) * 2 * K
                                          : bpl + (size_t)min(nt * BN + r - BM, N - 1) * 2 * K;
      src[q] = base + 8 * u;    // + 64 fp16 per 32-k step
    } else {                    // contiguous 1 KB: A as [mt][kt][32 KB], W as [nt][kt][16 KB]
      src[q] = piece < 32 ? apl + ((size_t)mt * KT * 32 + piece) * 512 + 8 * lane
                          : bpl + ((size_t)nt * KT * 16 + piece - 32) * 512 + 8 * lane;
    }
    stride[q] = MODE == 0 ? 32 : MODE == 1 ? 64 : (piece < 32 ? 32 * 512 : 16 * 512);
  }
  auto issue = [&](int buf, int kt) {
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
      const size_t off = (size_t)stride[q] * kt;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(src[q] + off),
          (__attribute__((address_space(3))) void*)(smem + buf * BUF + (q * NW + wave) * 1024), 16,
          0, 0);
    }
  };
  for (int d = 0; d < DEPTH; ++d) issue(d, k0 + d);
  unsigned acc = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt landed; with DEPTH 2 stage kt + 1's pieces may still fly
    if (DEPTH == 2 && kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + DEPTH < nk) issue((kt + DEPTH) % (DEPTH + 1), k0 + kt + DEPTH);
    acc += reinterpret_cast<const unsigned*>(smem + (kt % (DEPTH + 1)) * BUF)[threadIdx.x];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  const size_t abytes = (size_t)2 * M * K * 2, bbytes = (size_t)2 * 3200 * K * 2;   // 25 tiles of W rows
  unsigned short *a, *b;
  unsigned* sink;
  CK(hipMalloc(&a, abytes));
  CK(hipMalloc(&b, bbytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(a, 1, abytes));
  CK(hipMemset(b, 1, bbytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int blocks = 2 * 25 * SPLITS;
  const double bytes = (double)blocks * KC * BUF;   // ~ every block's 20 stages
  for (int rep = 0; rep < 3; ++rep)
    for (int mode = 0; mode < 6; ++mode) {
      auto launch = [&]() {
        switch (mode) {
          case 0: hipLaunchKernelGGL((fill<0, 1>), dim3(blocks), dim3(512), 0, 0, a, b, sink); break;
          case 1: hipLaunchKernelGGL((fill<1, 1>), dim3(blocks), dim3(512), 0, 0, a, b, sink); break;
          case 2: hipLaunchKernelGGL((fill<2, 1>), dim3(blocks), dim3(512), 0, 0, a, b, sink); break;
          case 3: hipLaunchKernelGGL((fill<0, 2>), dim3(blocks), dim3(512), 0, 0, a, b, sink); break;
          case 4: hipLaunchKernelGGL((fill<1, 2>), dim3(blocks), dim3(512), 0, 0, a, b, sink); break;
          default: hipLaunchKernelGGL((fill<2, 2>), dim3(blocks), dim3(512), 0, 0, a, b, sink);
        }
      };
      for (int i = 0; i < 20; ++i) launch();
      CK(hipEventRecord(e0));
      for (int i = 0; i < iters; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = 1e3 * ms / iters;
      printf("rep %d mode %d depth %d: %.2f us per launch, %.2f us per stage, %.1f GB/s per block, %.2f TB/s\n",
             rep, mode % 3, 1 + mode / 3, us, us / KC, bytes / blocks / (us * 1e-6) / 1e9, bytes / (us * 1e-6) / 1e12);
    }
  return 0;
}
