// Shared helpers for the gfx950 kernels of libaz_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/az_hip.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace az {

// Error reporting: every entry point returns AZ_OK or an AZ_E* code and leaves a message
// retrievable with az_last_error() (thread-local).
void set_error(const char* fmt, ...);
int check_launch(const char* what);

enum Act { ACT_NONE = AZ_ACT_NONE, ACT_RELU = AZ_ACT_RELU, ACT_SIGMOID = AZ_ACT_SIGMOID,
           ACT_TANH = AZ_ACT_TANH };

__device__ __forceinline__ float sigmoidf_ref(float x) {
  // torch.sigmoid on fp32: 1 / (1 + exp(-x))
  return 1.0f / (1.0f + expf(-x));
}

__device__ __forceinline__ float apply_act(float v, int act) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? v : 0.f;
    case ACT_SIGMOID: return sigmoidf_ref(v);
    case ACT_TANH: return tanhf(v);
    default: return v;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Sum NV per-lane values (NV a power of two <= 64) over the 64 lanes at once: each halving step
// exchanges the half of the values a lane does not keep (xor 32, 16, ...), so NV values cost
// NV-1 + (6 - log2 NV) shuffles instead of 6 NV.  Returns the sum of value index
// lane >> (6 - log2 NV) (every lane of that group holds it).
template <int NV>
__device__ __forceinline__ float wave_multi_sum(float (&v)[NV]) {
  static_assert(NV >= 1 && NV <= 64 && (NV & (NV - 1)) == 0, "NV must be a power of two");
  const int lane = threadIdx.x & 63;
  int m = 32;
#pragma unroll
  for (int n = NV; n > 1; n >>= 1, m >>= 1) {
    const bool hi = (lane & m) != 0;
#pragma unroll
    for (int i = 0; i < n / 2; ++i) {
      const float keep = hi ? v[i + n / 2] : v[i];
      const float send = hi ? v[i] : v[i + n / 2];
      v[i] = keep + __shfl_xor(send, m, 64);
    }
  }
  float r = v[0];
#pragma unroll
  for (; m > 0; m >>= 1) r += __shfl_xor(r, m, 64);
  return r;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// A/B-experiment switches (AZ_GEMM_CFG, AZ_SPLITK_HEADS_MODE, ...) are read only by the tuning
// build (-DAZ_TUNING -> libaz_hip_tuning.so, used by tools/ and the kernel-variant test): the
// product library never consults the environment and runs its fixed, measured dispatch.
#ifdef AZ_TUNING
inline const char* tuning_env(const char* name) { return getenv(name); }
#else
inline const char* tuning_env(const char*) { return nullptr; }
#endif

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace az

#define AZ_REQUIRE(cond, code, ...)      \
  do {                                   \
    if (!(cond)) {                       \
      az::set_error(__VA_ARGS__);        \
      return (code);                     \
    }                                    \
  } while (0)
