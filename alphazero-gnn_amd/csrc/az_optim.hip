// Adam over one flat fp32 parameter buffer: one HBM-streaming pass over p, g, m, v
// (16 B/lane loads and stores, 28 bytes moved per parameter).
#include <math.h>

#include <stdlib.h>

#include <algorithm>
#include "az_common.h"

namespace az {

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float b1c,
                                          float b2, float b2c, float neg_step, float bc2_sqrt,
                                          float eps) {
  // torch.optim.Adam (foreach=False/True, non-capturable):
  //   exp_avg.lerp_(grad, 1-beta1); exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1-beta2)
  //   denom = exp_avg_sq.sqrt() / bias_correction2_sqrt + eps
  //   param.addcdiv_(exp_avg, denom, value=-step_size)
  m = m + b1c * (g - m);
  v = v * b2 + b2c * g * g;
  const float denom = sqrtf(v) / bc2_sqrt + eps;
  p = p + neg_step * m / denom;
}

// U float4s per stream per thread, all loads issued before any math (4*U 16-B loads in
// flight per lane); blocks = ceil(n4 / (256*U)), no grid-stride loop.
template <int U>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ m, float* __restrict__ v,
                                                  long n4, long n, float b1c, float b2, float b2c,
                                                  float neg_step, float bc2_sqrt, float eps) {
  const long base = blockIdx.x * (256L * U) + threadIdx.x;
  f32x4 pp[U], gg[U], mm[U], vv[U];
  if (n4 > 0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = min(base + u * 256L, n4 - 1);
      pp[u] = reinterpret_cast<const f32x4*>(p)[i];
      gg[u] = reinterpret_cast<const f32x4*>(g)[i];
      mm[u] = reinterpret_cast<const f32x4*>(m)[i];
      vv[u] = reinterpret_cast<const f32x4*>(v)[i];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long i = base + u * 256L;
    if (i >= n4) break;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float pc = pp[u][c], mc = mm[u][c], vc = vv[u][c];
      adam_elem(pc, gg[u][c], mc, vc, b1c, b2, b2c, neg_step, bc2_sqrt, eps);
      pp[u][c] = pc; mm[u][c] = mc; vv[u][c] = vc;
    }
    reinterpret_cast<f32x4*>(p)[i] = pp[u];
    reinterpret_cast<f32x4*>(m)[i] = mm[u];
    reinterpret_cast<f32x4*>(v)[i] = vv[u];
  }
  // scalar tail (n % 4 elements), block 0 only
  if (blockIdx.x == 0)
    for (long i = n4 * 4 + threadIdx.x; i < n; i += 256)
      adam_elem(p[i], g[i], m[i], v[i], b1c, b2, b2c, neg_step, bc2_sqrt, eps);
}

}  // namespace az

using namespace az;

extern "C" int az_adam_f32(float* p, const float* g, float* m, float* v, int64_t n, double lr,
                           double beta1, double beta2, double eps, int step, void* stream) {
  AZ_REQUIRE(n >= 0 && step >= 1, AZ_EINVAL, "az_adam_f32: n=%lld step=%d", (long long)n, step);
  if (n == 0) return AZ_OK;
  AZ_REQUIRE(p && g && m && v, AZ_EINVAL, "az_adam_f32: null");
  AZ_REQUIRE(aligned16(p) && aligned16(g) && aligned16(m) && aligned16(v), AZ_EINVAL,
             "az_adam_f32: buffers need 16B alignment");
  az_weights_changed();   // the GEMMs' cached weight scales (az_gemm.hip) are stale now
  const double bc1 = 1.0 - pow(beta1, step);
  const double bc2 = 1.0 - pow(beta2, step);
  const double step_size = lr / bc1;
  const double bc2_sqrt = sqrt(bc2);
  const long n4 = n / 4;
  static const int env_u = [] {
    const char* e = tuning_env("AZ_ADAM_U");
    return e ? atoi(e) : 0;
  }();
  const int U = env_u == 1 || env_u == 2 || env_u == 4 || env_u == 8 ? env_u : 4;
  const long blocks = std::max<long>(1, (n4 + 256L * U - 1) / (256L * U));
  AZ_REQUIRE(blocks < (1L << 31), AZ_EINVAL, "az_adam_f32: n=%lld too large", (long long)n);
  const float a0 = (float)(1.0 - beta1), a1 = (float)beta2, a2 = (float)(1.0 - beta2),
              a3 = (float)(-step_size), a4 = (float)bc2_sqrt, a5 = (float)eps;
  hipStream_t st = as_stream(stream);
  if (n4 == 0) {
    hipLaunchKernelGGL(adam_kernel<1>, dim3(1), dim3(256), 0, st, p, g, m, v, 0L, (long)n, a0, a1,
                       a2, a3, a4, a5);
  } else if (U == 1) {
    hipLaunchKernelGGL(adam_kernel<1>, dim3(blocks), dim3(256), 0, st, p, g, m, v, n4, (long)n, a0,
                       a1, a2, a3, a4, a5);
  } else if (U == 2) {
    hipLaunchKernelGGL(adam_kernel<2>, dim3(blocks), dim3(256), 0, st, p, g, m, v, n4, (long)n, a0,
                       a1, a2, a3, a4, a5);
  } else if (U == 8) {
    hipLaunchKernelGGL(adam_kernel<8>, dim3(blocks), dim3(256), 0, st, p, g, m, v, n4, (long)n, a0,
                       a1, a2, a3, a4, a5);
  } else {
    hipLaunchKernelGGL(adam_kernel<4>, dim3(blocks), dim3(256), 0, st, p, g, m, v, n4, (long)n, a0,
                       a1, a2, a3, a4, a5);
  }
  return check_launch("adam_kernel");
}

// SURVEY.md §8b's name for the optimizer entry point: the same arguments, the same kernel.
extern "C" int az_adam_step(float* p, const float* g, float* m, float* v, int64_t n, double lr,
                            double beta1, double beta2, double eps, int step, void* stream) {
  return az_adam_f32(p, g, m, v, n, lr, beta1, beta2, eps, step, stream);
}
