// Microbenchmark: sustained v_mfma_f32_32x32x2_f32 / 16x16x4 issue rate per SIMD on gfx950,
// operands in registers vs re-read from LDS with ds_read_b128, 1 or 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma32_regs(float* out, int iters, float seed) {
  f32x16 acc[NACC];
  for (int i = 0; i < NACC; ++i) for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  float a = seed * threadIdx.x, b = seed + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
    a += 1e-7f; b -= 1e-7f;
  }
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) for (int r = 0; r < 16; ++r) s += acc[i][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int NACC>
__global__ __launch_bounds__(256) void mfma16_regs(float* out, int iters, float seed) {
  f32x4 acc[NACC];
  for (int i = 0; i < NACC; ++i) for (int r = 0; r < 4; ++r) acc[i][r] = 0.f;
  float a = seed * threadIdx.x, b = seed + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
    a += 1e-7f; b -= 1e-7f;
  }
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) for (int r = 0; r < 4; ++r) s += acc[i][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// 2x2 accumulators of 32x32, operands re-read from LDS each 8-k group (the GEMM inner loop)
__global__ __launch_bounds__(256) void mfma32_lds(float* out, int iters, float seed) {
  __shared__ __attribute__((aligned(16))) float L[2][128 * 36];
  for (int i = threadIdx.x; i < 2 * 128 * 36; i += 256) (&L[0][0])[i] = seed * i;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave >> 1, wn = wave & 1;
  f32x16 acc[2][2];
  for (int i = 0; i < 2; ++i) for (int j = 0; j < 2; ++j) for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = *reinterpret_cast<const f32x4*>(&L[0][(wm * 64 + i * 32 + (lane & 31)) * 36 + g * 8 + (lane >> 5) * 4]);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = *reinterpret_cast<const f32x4*>(&L[1][(wn * 64 + j * 32 + (lane & 31)) * 36 + g * 8 + (lane >> 5) * 4]);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][t], b[j][t], acc[i][j], 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int i = 0; i < 2; ++i) for (int j = 0; j < 2; ++j) for (int r = 0; r < 16; ++r) s += acc[i][j][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <typename K>
static void run(const char* name, K kern, int blocks, int iters, int mfma_per_iter, float* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-3f);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-3f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
  const double mfmas_per_simd = (double)blocks * 4 / 1024.0 * iters * mfma_per_iter;  // 1024 SIMDs
  const double cyc = ms * 1e-3 * 2.4e9;
  printf("%-28s blocks=%5d  %.3f ms  ~%.1f cycles per MFMA per SIMD (at 2.4 GHz)\n", name, blocks, ms,
         cyc / mfmas_per_simd);
}

int main() {
  float* out;
  hipMalloc(&out, 4096 * 256 * 4);
  const int it = 20000;
  run("32x32x2 regs, 4 acc, 1w/SIMD", mfma32_regs<4>, 256, it, 4, out);
  run("32x32x2 regs, 8 acc, 1w/SIMD", mfma32_regs<8>, 256, it / 2, 8, out);
  run("32x32x2 regs, 4 acc, 2w/SIMD", mfma32_regs<4>, 512, it, 4, out);
  run("32x32x2 regs, 1 acc, 1w/SIMD", mfma32_regs<1>, 256, it, 1, out);
  run("16x16x4 regs, 4 acc, 1w/SIMD", mfma16_regs<4>, 256, it, 4, out);
  run("16x16x4 regs, 8 acc, 2w/SIMD", mfma16_regs<8>, 512, it / 2, 8, out);
  run("32x32x2 LDS-fed 2x2, 1w/SIMD", mfma32_lds, 256, 2000, 64, out);
  run("32x32x2 LDS-fed 2x2, 2w/SIMD", mfma32_lds, 512, 2000, 64, out);
  hipFree(out);
  return 0;
}
