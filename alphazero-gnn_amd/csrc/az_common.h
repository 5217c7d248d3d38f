// Shared helpers for the gfx950 kernels of libaz_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <type_traits>

#include "../../include/az_hip.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace az {

// Error reporting: every entry point returns AZ_OK or an AZ_E* code and leaves a message
// retrievable with az_last_error() (thread-local).
void set_error(const char* fmt, ...);
int check_launch(const char* what);

// f(std::integral_constant<int, I>) for I = 0 .. N-1, unrolled at compile time (for intrinsics
// that need the index as a constant, e.g. a DPP control)
template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

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

// Bytes handed between the workgroups of ONE launch (c4_leaf_kernel; MI355X_MICROARCH.md,
// "Hand-offs measured with sc1 loads", row 1): the producer stores them write-through (sc1),
// every storing wave waits for its stores (vmcnt(0)) before its block counts itself, and EVERY
// load of them is an sc1 load, which bypasses the CU's L1 (another CU's stores never refresh
// it) -- no agent-scope fence (buffer_wbl2 / buffer_inv, several us each at 4 blocks per CU).
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16 bytes at byte offset `off` of the wave-uniform `base` (`bytes` addressable from base)
__device__ __forceinline__ f32x4 ld4_sc1(const float* base, int off, int bytes) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, bytes, 0x00020000);
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

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
