// Adam over one flat fp32 parameter buffer: one HBM-streaming pass over p, g, m, v
// (16 B/lane loads and stores, 28 bytes moved per parameter).
#include <math.h>

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

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ m, float* __restrict__ v,
                                                  long n4, long n, float b1c, float b2, float b2c,
                                                  float neg_step, float bc2_sqrt, float eps) {
  const long stride = (long)gridDim.x * 256;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += stride) {
    f32x4 pp = reinterpret_cast<f32x4*>(p)[i];
    const f32x4 gg = reinterpret_cast<const f32x4*>(g)[i];
    f32x4 mm = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float pc = pp[c], mc = mm[c], vc = vv[c];
      adam_elem(pc, gg[c], mc, vc, b1c, b2, b2c, neg_step, bc2_sqrt, eps);
      pp[c] = pc; mm[c] = mc; vv[c] = vc;
    }
    reinterpret_cast<f32x4*>(p)[i] = pp;
    reinterpret_cast<f32x4*>(m)[i] = mm;
    reinterpret_cast<f32x4*>(v)[i] = vv;
  }
  // scalar tail
  for (long i = n4 * 4 + blockIdx.x * 256L + threadIdx.x; i < n; i += stride)
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
  const double bc1 = 1.0 - pow(beta1, step);
  const double bc2 = 1.0 - pow(beta2, step);
  const double step_size = lr / bc1;
  const double bc2_sqrt = sqrt(bc2);
  const long n4 = n / 4;
  const int blocks = (int)std::min<long>((n4 + 255) / 256 + 1, 256L * 8);
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), p, g, m, v, n4,
                     (long)n, (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2),
                     (float)(-step_size), (float)bc2_sqrt, (float)eps);
  return check_launch("adam_kernel");
}
