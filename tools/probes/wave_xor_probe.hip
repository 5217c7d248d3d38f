// Bitwise check of az_common.h's VALU lane exchanges (DPP / v_permlane*_swap) against the
// __shfl_xor (ds_bpermute) forms they replace: xor_lane<M>, swap_add<M>, wave_sum_x and
// wave_multi_sum<8 / 16 / 1> on random data (random exponents and signs, so any change of
// association shows).  Prints mismatch counts; exit 1 on any.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/wave_xor_probe tools/probes/wave_xor_probe.hip
#include "../../alphazero-gnn_amd/csrc/az_common.h"

using namespace az;

template <int NV>
__device__ float multi_sum_ref(float (&v)[NV]) {   // round 5's wave_multi_sum
  const int lane = threadIdx.x & 63;
  int m = 32;
  for (int n = NV; n > 1; n >>= 1, m >>= 1) {
    const bool hi = (lane & m) != 0;
    for (int i = 0; i < n / 2; ++i) {
      const float keep = hi ? v[i + n / 2] : v[i];
      const float send = hi ? v[i] : v[i + n / 2];
      v[i] = keep + __shfl_xor(send, m, 64);
    }
  }
  float r = v[0];
  for (; m > 0; m >>= 1) r += __shfl_xor(r, m, 64);
  return r;
}

__global__ void probe(const float* in, unsigned* bad) {
  const int lane = threadIdx.x & 63;
  const float* x = in + blockIdx.x * 64 * 32;
  float a = x[lane], b = x[64 + lane];
  unsigned nb = 0;
  auto cmp = [&](float p, float q) { nb += __float_as_uint(p) != __float_as_uint(q); };
  cmp(xor_lane<1>(a), __shfl_xor(a, 1, 64));
  cmp(xor_lane<2>(a), __shfl_xor(a, 2, 64));
  cmp(xor_lane<4>(a), __shfl_xor(a, 4, 64));
  cmp(xor_lane<8>(a), __shfl_xor(a, 8, 64));
  const bool h32 = lane & 32, h16 = lane & 16;
  cmp(swap_add<32>(a, b), (h32 ? b : a) + __shfl_xor(h32 ? a : b, 32, 64));
  cmp(swap_add<16>(a, b), (h16 ? b : a) + __shfl_xor(h16 ? a : b, 16, 64));
  cmp(wave_sum_x(a), wave_sum(a));
  float v8[8], r8[8], v16[16], r16[16], v1[1], r1[1];
  for (int i = 0; i < 8; ++i) v8[i] = r8[i] = x[64 * (2 + i) + lane];
  for (int i = 0; i < 16; ++i) v16[i] = r16[i] = x[64 * (10 + i) + lane];
  v1[0] = r1[0] = b;
  cmp(wave_multi_sum<8>(v8), multi_sum_ref<8>(r8));
  cmp(wave_multi_sum<16>(v16), multi_sum_ref<16>(r16));
  cmp(wave_multi_sum<1>(v1), multi_sum_ref<1>(r1));
  if (nb) atomicAdd(bad, nb);
}

int main() {
  const int blocks = 4096, n = blocks * 64 * 32;
  float* h = (float*)malloc(n * sizeof(float));
  unsigned s = 12345;
  for (int i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    const float m = (float)((s >> 8) & 0xffff) / 65536.f + 0.5f;
    const int e = (int)((s >> 24) & 31) - 16;
    h[i] = ((s & 1) ? -1.f : 1.f) * ldexpf(m, e);
  }
  float* d;
  unsigned* bad;
  if (hipMalloc(&d, n * sizeof(float)) || hipMalloc(&bad, 4)) return 2;
  hipMemcpy(d, h, n * sizeof(float), hipMemcpyHostToDevice);
  hipMemset(bad, 0, 4);
  hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, 0, d, bad);
  unsigned hb = 0;
  if (hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  printf("wave_xor_probe: %d waves x 10 checks, %u bitwise mismatches\n", blocks * 4, hb);
  return hb ? 1 : 0;
}
