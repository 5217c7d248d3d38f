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

// Exact lane-xor exchanges on the VALU instead of the LDS crossbar (ds_bpermute, what __shfl_xor
// compiles to: ~1 LDS round trip per step).  Full waves only (every lane active: the DPP forms
// keep a lane's own value where the partner is inactive).  M = 32 / 16: v_permlane32_swap /
// v_permlane16_swap exchange half-waves / alternate 16-lane rows; M = 8: DPP row_ror:8;
// M = 4: two DPP row shifts written into alternate 4-lane banks; M = 2, 1: DPP quad_perm.
template <int M>
__device__ __forceinline__ float xor_lane(float v) {
  static_assert(M == 1 || M == 2 || M == 4 || M == 8, "DPP forms: M <= 8");
  const int x = __float_as_int(v);
  int r;
  if constexpr (M == 8) {
    r = __builtin_amdgcn_update_dpp(x, x, 0x128, 0xf, 0xf, false);       // row_ror:8
  } else if constexpr (M == 4) {
    const int t = __builtin_amdgcn_update_dpp(x, x, 0x114, 0xf, 0xa, false);  // row_shr:4 -> banks 1, 3
    r = __builtin_amdgcn_update_dpp(t, x, 0x104, 0xf, 0x5, false);       // row_shl:4 -> banks 0, 2
  } else if constexpr (M == 2) {
    r = __builtin_amdgcn_update_dpp(x, x, 0x4e, 0xf, 0xf, false);        // quad_perm [2,3,0,1]
  } else {
    r = __builtin_amdgcn_update_dpp(x, x, 0xb1, 0xf, 0xf, false);        // quad_perm [1,0,3,2]
  }
  return __int_as_float(r);
}

// The half-wave (M = 32) or row (M = 16) exchange of a pair: lanes whose bit M is clear keep
// `lo` and receive the partner's `lo`; lanes with it set keep `hi` and receive the partner's
// `hi`; the sum of what a lane keeps and receives, in an order that is bitwise the same as
// keep + __shfl_xor(send, M) (IEEE addition is commutative).
template <int M>
__device__ __forceinline__ float swap_add(float lo, float hi) {
  static_assert(M == 16 || M == 32, "permlane swaps: M = 16, 32");
  const unsigned a = __float_as_uint(lo), b = __float_as_uint(hi);
  const auto r = M == 32 ? __builtin_amdgcn_permlane32_swap(a, b, false, false)
                         : __builtin_amdgcn_permlane16_swap(a, b, false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// v + v of lane ^ M, bitwise as v + __shfl_xor(v, M) (full waves)
template <int M>
__device__ __forceinline__ float xor_add(float v) {
  if constexpr (M >= 16) return swap_add<M>(v, v);
  else return v + xor_lane<M>(v);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// wave_sum on the VALU exchanges (bitwise the same result; full waves only)
__device__ __forceinline__ float wave_sum_x(float v) {
  v = xor_add<32>(v);
  v = xor_add<16>(v);
  v = xor_add<8>(v);
  v = xor_add<4>(v);
  v = xor_add<2>(v);
  return xor_add<1>(v);
}

// Sum NV per-lane values (NV a power of two <= 64) over the 64 lanes at once: each halving step
// exchanges the half of the values a lane does not keep (xor 32, 16, ...), so NV values cost
// NV-1 + (6 - log2 NV) exchanges instead of 6 NV.  Returns the sum of value index
// lane >> (6 - log2 NV) (every lane of that group holds it).  The exchanges are the VALU forms
// above (full waves only); the sums are bitwise those of keep + __shfl_xor(send, m).
template <int NV>
__device__ __forceinline__ float wave_multi_sum(float (&v)[NV]) {
  static_assert(NV >= 1 && NV <= 64 && (NV & (NV - 1)) == 0, "NV must be a power of two");
  constexpr int LOG = NV >= 64 ? 6 : NV >= 32 ? 5 : NV >= 16 ? 4 : NV >= 8 ? 3 : NV >= 4 ? 2
                      : NV >= 2 ? 1 : 0;
  const int lane = threadIdx.x & 63;
  static_for<LOG>([&](auto st) {               // halving step at m = 32 >> st
    constexpr int m = 32 >> st.value, n = NV >> st.value;
    if constexpr (m >= 16) {
#pragma unroll
      for (int i = 0; i < n / 2; ++i) v[i] = swap_add<m>(v[i], v[i + n / 2]);
    } else {
      const bool hi = (lane & m) != 0;
#pragma unroll
      for (int i = 0; i < n / 2; ++i) {
        const float keep = hi ? v[i + n / 2] : v[i];
        const float send = hi ? v[i] : v[i + n / 2];
        v[i] = keep + xor_lane<m>(send);
      }
    }
  });
  float r = v[0];
  static_for<6 - LOG>([&](auto st) { r = xor_add<(32 >> (LOG + st.value))>(r); });
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
