// Microbenchmark: the GEMM inner loop alone (fragments re-read from LDS with ds_read_b128, f32
// MFMA into TI x TJ accumulators per wave) on RANDOM operands, for several wave-tile shapes and
// 1 or 2 waves per SIMD.  TFLOP/s on random data includes the clock the chip holds under the
// loop (MI355X_MICROARCH.md "DVFS give-back"): fewer LDS bytes per MFMA = less energy per FLOP.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ inline float hashf(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return (float)(x & 0xffffff) / 8388608.0f - 1.0f;
}

// wave tile (TI*MF) x (TJ*MF), 4 waves per block, LDS image [rows][32 k] swizzled like the GEMM
template <int MF, int TI, int TJ>
__global__ __launch_bounds__(256) void tile_loop(float* out, int iters) {
  constexpr int RA = 2 * TI * MF, RB = 2 * TJ * MF;   // 2x2 waves
  __shared__ __attribute__((aligned(1024))) float L[(RA + RB) * 32];
  for (int i = threadIdx.x; i < (RA + RB) * 32; i += 256) L[i] = hashf(i * 2654435761u + blockIdx.x);
  __syncthreads();
  using acc_t = typename std::conditional<MF == 32, f32x16, f32x4>::type;
  constexpr int NACC = MF == 32 ? 16 : 4;
  constexpr int LSH = MF == 32 ? 5 : 4;
  constexpr int NG = MF == 32 ? 4 : 2;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave >> 1, wn = wave & 1;
  acc_t acc[TI][TJ];
  for (int i = 0; i < TI; ++i) for (int j = 0; j < TJ; ++j) for (int r = 0; r < NACC; ++r) acc[i][j][r] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      f32x4 a[TI], b[TJ];
      const int lc = g * (64 >> LSH) + (lane >> LSH);
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int r = wm * TI * MF + i * MF + (lane & (MF - 1));
        a[i] = *reinterpret_cast<const f32x4*>(&L[r * 32 + ((lc ^ ((r >> 1) & 7)) * 4)]);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int r = RA + wn * TJ * MF + j * MF + (lane & (MF - 1));
        b[j] = *reinterpret_cast<const f32x4*>(&L[r * 32 + ((lc ^ ((r >> 1) & 7)) * 4)]);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            if constexpr (MF == 32)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][t], b[j][t], acc[i][j], 0, 0, 0);
            else
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][t], b[j][t], acc[i][j], 0, 0, 0);
          }
    }
  }
  float s = 0.f;
  for (int i = 0; i < TI; ++i) for (int j = 0; j < TJ; ++j) for (int r = 0; r < NACC; ++r) s += acc[i][j][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MF, int TI, int TJ>
static void run(int blocks, int iters, float* out) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((tile_loop<MF, TI, TJ>), dim3(blocks), dim3(256), 0, 0, out, iters);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL((tile_loop<MF, TI, TJ>), dim3(blocks), dim3(256), 0, 0, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1); ms /= 10;
  const double flop = (double)blocks * 4 * iters * 32.0 * (TI * MF) * (TJ * MF) * 2.0;
  printf("mfma%dx%d wave tile %3dx%-3d  %d w/SIMD  %.3f ms  %.1f TFLOP/s  LDS B/MFMA %d\n", MF, MF,
         TI * MF, TJ * MF, blocks / 256, ms, flop / ms / 1e9, (TI + TJ) * 1024 * (MF == 32 ? 4 : 2) / (TI * TJ * 16 / (MF == 32 ? 1 : 1) * (MF == 32 ? 1 : 2)));
}

int main() {
  float* out;
  (void)hipMalloc(&out, 4096 * 256 * 4);
  const int it = 1500;
  for (int w = 1; w <= 2; ++w) {
    run<32, 2, 2>(256 * w, it, out);
    run<32, 4, 2>(256 * w, it / 2, out);
    run<32, 4, 4>(256 * w, it / 4, out);
    run<16, 4, 4>(256 * w, it, out);
    run<16, 8, 4>(256 * w, it / 2, out);
    run<16, 8, 8>(256 * w, it / 4, out);
  }
  (void)hipFree(out);
  return 0;
}
