// Probe: where the hardware puts each workgroup's LDS when two share a CU.  Every block of a
// 512-thread kernel with the trunk's static LDS size (c4_trunk_kernel<1> in the two-per-CU layout:
// 25,888 B, + optional dynamic LDS) records its HW_ID (XCC / SE / SA / CU / SIMD / wave slot) and
// LDS_ALLOC hardware registers, then fills its whole LDS with its block id and, after a delay that
// keeps the co-resident blocks alive together, checks that every word still holds its own id.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/lds_alloc_probe tools/probes/lds_alloc_probe.hip
//   lds_alloc_probe [blocks] [dyn_bytes]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <map>
#include <vector>

constexpr int STATIC_FLOATS = 25888 / 4;

__global__ __launch_bounds__(512) void probe(unsigned* rec, unsigned* bad, int dyn_floats,
                                             long long spin) {
  __shared__ __attribute__((aligned(16))) float st[STATIC_FLOATS];
  extern __shared__ float dy[];
  const unsigned id = blockIdx.x;
  typedef float f4 __attribute__((ext_vector_type(4)));
  const float fid = __uint_as_float(id);
  for (int i = threadIdx.x; i < STATIC_FLOATS / 4; i += 512)   // 16-B stores, as the trunk's
    reinterpret_cast<f4*>(st)[i] = f4{fid, fid, fid, fid};
  for (int i = threadIdx.x; i < dyn_floats; i += 512) dy[i] = __uint_as_float(id);
  __syncthreads();
  const long long t0 = clock64();
  while (clock64() - t0 < spin) __builtin_amdgcn_s_sleep(2);
  __syncthreads();
  unsigned nb = 0;
  for (int i = threadIdx.x; i < STATIC_FLOATS / 4; i += 512) {
    const f4 v = reinterpret_cast<const f4*>(st)[i];
    for (int e = 0; e < 4; ++e) nb += __float_as_uint(v[e]) != id;
  }
  for (int i = threadIdx.x; i < dyn_floats; i += 512) nb += __float_as_uint(dy[i]) != id;
  bad[(size_t)id * 512 + threadIdx.x] = nb;   // per thread, summed on the host
  if (threadIdx.x == 0 || threadIdx.x == 448) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID
    const unsigned lds = __builtin_amdgcn_s_getreg((31 << 11) | 6);    // HW_REG_LDS_ALLOC
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
    const int slot = threadIdx.x ? 1 : 0;
    rec[(id * 2 + slot) * 3 + 0] = hw;
    rec[(id * 2 + slot) * 3 + 1] = lds;
    rec[(id * 2 + slot) * 3 + 2] = xcc;
  }
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 512;
  const int dyn = argc > 2 ? atoi(argv[2]) : 0;
  unsigned *rec, *bad;
  (void)hipMalloc(&rec, (size_t)blocks * 6 * 4);
  (void)hipMalloc(&bad, (size_t)blocks * 512 * 4);
  (void)hipMemset(rec, 0, (size_t)blocks * 6 * 4);
  (void)hipMemset(bad, 0, (size_t)blocks * 512 * 4);
  hipLaunchKernelGGL(probe, dim3(blocks), dim3(512), dyn, 0, rec, bad, dyn / 4, 200000LL);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
  std::vector<unsigned> r((size_t)blocks * 6), bt((size_t)blocks * 512), b(blocks, 0);
  (void)hipMemcpy(r.data(), rec, r.size() * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(bt.data(), bad, bt.size() * 4, hipMemcpyDeviceToHost);
  for (size_t i = 0; i < bt.size(); ++i) b[i / 512] += bt[i];
  // HW_ID (gfx9): wave_id [3:0], simd_id [5:4], pipe [7:6], cu_id [11:8], sh_id [12], se_id [15:13]
  std::map<unsigned, std::vector<int>> per_cu;
  long nbad = 0;
  for (int i = 0; i < blocks; ++i) {
    const unsigned hw = r[i * 6], xcc = r[i * 6 + 2] & 0xf;
    const unsigned cu = (xcc << 16) | (hw & 0xff00);
    per_cu[cu].push_back(i);
    nbad += b[i];
  }
  int shown = 0, shared = 0;
  for (auto& kv : per_cu) {
    if (kv.second.size() > 1) ++shared;
    if (kv.second.size() > 1 && shown < 6) {
      ++shown;
      printf("cu %05x:", kv.first);
      for (int i : kv.second)
        printf("  blk %d lds_alloc 0x%08x/0x%08x simd %u wave %u bad %u", i, r[i * 6 + 1],
               r[i * 6 + 4], (r[i * 6] >> 4) & 3, r[i * 6] & 15, b[i]);
      printf("\n");
    }
  }
  printf("blocks %d dyn %d: %zu CUs used, %d with >1 block, words overwritten by another block: %ld\n",
         blocks, dyn, per_cu.size(), shared, nbad);
  return 0;
}
