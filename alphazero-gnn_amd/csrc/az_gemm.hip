// fp32 GEMM on gfx950 MFMA (v_mfma_f32_32x32x2_f32) with fused epilogues, plus a
// weight-streaming GEMV for M <= 8 (batch-1 predict, the star's row-0 update).
//
// Tile kernel: 256 threads = 4 waves as 2x2, BM x BN block tile, BK = 16, register-staged
// double-buffered LDS.  Both operands are kept K-contiguous in LDS ([row][k], stride 20
// floats: conflict-free ds_read_b128 for 16-lane groups) so each lane fetches 4 k-values
// of its A row / B column with one ds_read_b128 and feeds 4 MFMAs; the k order inside an
// 8-k group is permuted (lane half h owns k = 4h..4h+3, MFMA t sums k = t and 4+t), which
// changes only the fp32 summation order.
#include "az_common.h"

namespace az {

struct GemmArgs {
  int M, N, K;
  const float* A; int lda;
  const float* A2; int lda2; int K0;
  const int* a_rows;
  const float* B; int ldb;
  const float* bias; int act;
  const float* R; int ldr;
  const float* G; int ldg;
  float beta;
  float* C; int ldc;
  const int* c_rows;
};

constexpr int BK = 16;
constexpr int LDK = BK + 4;

__device__ __forceinline__ void epilogue_store(const GemmArgs& p, int row, int col, float acc) {
  if (row >= p.M || col >= p.N) return;
  float v = acc + (p.bias ? p.bias[col] : 0.f);
  v = apply_act(v, p.act);
  const int cr = p.c_rows ? p.c_rows[row] : row;
  if (p.R) v = p.R[(size_t)cr * p.ldr + col] + (p.G ? p.G[(size_t)row * p.ldg + col] : 1.f) * v;
  float* dst = p.C + (size_t)cr * p.ldc + col;
  if (p.beta != 0.f) v += p.beta * *dst;
  *dst = v;
}

// Load one BK-deep slice of a K-major operand (rows x BK, row-major along k) as float4s.
template <int ROWS, bool IS_A>
__device__ __forceinline__ void load_kmajor(const GemmArgs& p, int r0, int k0, int nrows,
                                            f32x4 (&reg)[ROWS * BK / 4 / 256]) {
  constexpr int NF4 = ROWS * BK / 4 / 256;
#pragma unroll
  for (int q = 0; q < NF4; ++q) {
    const int idx = threadIdx.x + q * 256;
    const int row = idx >> 2, kq = idx & 3;
    const int gr = r0 + row, k = k0 + kq * 4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (gr < nrows && k < p.K) {
      if (IS_A) {
        const int ar = p.a_rows ? p.a_rows[gr] : gr;
        const float* src = (p.A2 && k >= p.K0) ? p.A2 + (size_t)ar * p.lda2 + (k - p.K0)
                                               : p.A + (size_t)ar * p.lda + k;
        v = *reinterpret_cast<const f32x4*>(src);
      } else {
        v = *reinterpret_cast<const f32x4*>(p.B + (size_t)gr * p.ldb + k);
      }
    }
    reg[q] = v;
  }
}

template <int ROWS>
__device__ __forceinline__ void store_kmajor(float* lds, const f32x4 (&reg)[ROWS * BK / 4 / 256]) {
  constexpr int NF4 = ROWS * BK / 4 / 256;
#pragma unroll
  for (int q = 0; q < NF4; ++q) {
    const int idx = threadIdx.x + q * 256;
    const int row = idx >> 2, kq = idx & 3;
    *reinterpret_cast<f32x4*>(lds + row * LDK + kq * 4) = reg[q];
  }
}

// Operand stored contiguous along its M/N dimension: element (k, i) at base[k*ld + i].
template <int ROWS>
__device__ __forceinline__ void load_mnmajor(const float* base, int ld, int r0, int k0, int nrows,
                                             int K, f32x4 (&reg)[ROWS * BK / 4 / 256]) {
  constexpr int NF4 = ROWS * BK / 4 / 256;
  constexpr int PER_K = ROWS / 4;
#pragma unroll
  for (int q = 0; q < NF4; ++q) {
    const int idx = threadIdx.x + q * 256;
    const int kr = idx / PER_K, mq = idx % PER_K;
    const int gr = r0 + mq * 4, k = k0 + kr;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (k < K && gr < nrows) v = *reinterpret_cast<const f32x4*>(base + (size_t)k * ld + gr);
    reg[q] = v;
  }
}

template <int ROWS>
__device__ __forceinline__ void store_mnmajor(float* lds, const f32x4 (&reg)[ROWS * BK / 4 / 256]) {
  constexpr int NF4 = ROWS * BK / 4 / 256;
  constexpr int PER_K = ROWS / 4;
#pragma unroll
  for (int q = 0; q < NF4; ++q) {
    const int idx = threadIdx.x + q * 256;
    const int kr = idx / PER_K, mq = idx % PER_K;
#pragma unroll
    for (int e = 0; e < 4; ++e) lds[(mq * 4 + e) * LDK + kr] = reg[q][e];
  }
}

template <int BM, int BN, bool A_KM, bool B_KM>
__global__ __launch_bounds__(256) void gemm_f32_mfma(GemmArgs p) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TI = WM / 32, TJ = WN / 32;
  constexpr int AF4 = BM * BK / 4 / 256, BF4 = BN * BK / 4 / 256;
  __shared__ __attribute__((aligned(16))) float As[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDK];

  const int mt_n = (p.M + BM - 1) / BM, nt_n = (p.N + BN - 1) / BN;
  const int nwg = mt_n * nt_n;
  int bid = blockIdx.x;
  // XCD-aware remap (blocks b, b+8 share an XCD): give each XCD a contiguous run of tile ids,
  // consecutive ids share the B (weight) panel -> weight panel re-reads hit that XCD's L2.
  if ((nwg & 7) == 0) bid = (bid & 7) * (nwg >> 3) + (bid >> 3);
  const int mt = bid % mt_n, nt = bid / mt_n;
  const int m0 = mt * BM, n0 = nt * BN;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  f32x4 ra[AF4], rb[BF4];
  auto load = [&](int k0) {
    if constexpr (A_KM) load_kmajor<BM, true>(p, m0, k0, p.M, ra);
    else load_mnmajor<BM>(p.A, p.lda, m0, k0, p.M, p.K, ra);
    if constexpr (B_KM) load_kmajor<BN, false>(p, n0, k0, p.N, rb);
    else load_mnmajor<BN>(p.B, p.ldb, n0, k0, p.N, p.K, rb);
  };
  auto store = [&](int buf) {
    if constexpr (A_KM) store_kmajor<BM>(As[buf], ra); else store_mnmajor<BM>(As[buf], ra);
    if constexpr (B_KM) store_kmajor<BN>(Bs[buf], rb); else store_mnmajor<BN>(Bs[buf], rb);
  };

  const int nk = (p.K + BK - 1) / BK;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load((kt + 1) * BK);
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      f32x4 a[TI], b[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i)
        a[i] = *reinterpret_cast<const f32x4*>(
            &As[cur][(wm * WM + i * 32 + (lane & 31)) * LDK + g * 8 + (lane >> 5) * 4]);
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        b[j] = *reinterpret_cast<const f32x4*>(
            &Bs[cur][(wn * WN + j * 32 + (lane & 31)) * LDK + g * 8 + (lane >> 5) * 4]);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][t], b[j][t], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int col = n0 + wn * WN + j * 32 + (lane & 31);
        epilogue_store(p, row, col, acc[i][j][r]);
      }
}

// ------------------------------------------------------------------------------ GEMV
// C[M<=8][N] = epi(A[M][K] . W[N][K]^T): each wave owns GV_ROWS output columns and streams
// their weight rows from HBM (float4, GV_ROWS*KC/256 loads in flight per lane); A is staged
// through LDS in KC-wide chunks and shared by the block's 4 waves.
constexpr int GV_ROWS = 2;
constexpr int GV_KC = 1024;

template <int MR>
__global__ __launch_bounds__(256) void gemv_f32(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) float As[MR * GV_KC];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n_base = (blockIdx.x * 4 + wave) * GV_ROWS;
  float acc[MR][GV_ROWS];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int r = 0; r < GV_ROWS; ++r) acc[m][r] = 0.f;

  for (int kc = 0; kc < p.K; kc += GV_KC) {
    const int klen = min(GV_KC, p.K - kc);
    __syncthreads();
    for (int idx = threadIdx.x; idx < MR * (GV_KC / 4); idx += 256) {
      const int m = idx / (GV_KC / 4), k4 = (idx % (GV_KC / 4)) * 4;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      const int k = kc + k4;
      if (m < p.M && k4 < klen) {
        const int ar = p.a_rows ? p.a_rows[m] : m;
        const float* src = (p.A2 && k >= p.K0) ? p.A2 + (size_t)ar * p.lda2 + (k - p.K0)
                                               : p.A + (size_t)ar * p.lda + k;
        v = *reinterpret_cast<const f32x4*>(src);
      }
      *reinterpret_cast<f32x4*>(&As[m * GV_KC + k4]) = v;
    }
    __syncthreads();
    f32x4 w[GV_ROWS][GV_KC / 256];
#pragma unroll
    for (int r = 0; r < GV_ROWS; ++r) {
      const int n = n_base + r;
#pragma unroll
      for (int s = 0; s < GV_KC / 256; ++s) {
        const int k4 = (lane + 64 * s) * 4;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (n < p.N && k4 < klen)
          v = *reinterpret_cast<const f32x4*>(p.B + (size_t)n * p.ldb + kc + k4);
        w[r][s] = v;
      }
    }
#pragma unroll
    for (int s = 0; s < GV_KC / 256; ++s) {
      const int k4 = (lane + 64 * s) * 4;
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(&As[m * GV_KC + k4]);
#pragma unroll
        for (int r = 0; r < GV_ROWS; ++r)
          acc[m][r] = fmaf(a[0], w[r][s][0], fmaf(a[1], w[r][s][1],
                      fmaf(a[2], w[r][s][2], fmaf(a[3], w[r][s][3], acc[m][r]))));
      }
    }
  }
  float mine = 0.f;  // lane m*GV_ROWS + r keeps the reduced sum of output (m, n_base + r)
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int r = 0; r < GV_ROWS; ++r) {
      const float s = wave_sum(acc[m][r]);
      if (lane == m * GV_ROWS + r) mine = s;
    }
  if (lane < MR * GV_ROWS) {
    const int m = lane / GV_ROWS, r = lane % GV_ROWS;
    if (m < p.M) epilogue_store(p, m, n_base + r, mine);
  }
}

template <int BM, int BN>
static void launch_tile(const GemmArgs& a, bool akm, bool bkm, hipStream_t s) {
  const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  if (akm && bkm) hipLaunchKernelGGL((gemm_f32_mfma<BM, BN, true, true>), dim3(nwg), dim3(256), 0, s, a);
  else if (akm) hipLaunchKernelGGL((gemm_f32_mfma<BM, BN, true, false>), dim3(nwg), dim3(256), 0, s, a);
  else if (bkm) hipLaunchKernelGGL((gemm_f32_mfma<BM, BN, false, true>), dim3(nwg), dim3(256), 0, s, a);
  else hipLaunchKernelGGL((gemm_f32_mfma<BM, BN, false, false>), dim3(nwg), dim3(256), 0, s, a);
}

static void launch_gemv(const GemmArgs& a, hipStream_t s) {
  const int nblk = (a.N + 4 * GV_ROWS - 1) / (4 * GV_ROWS);
  switch (a.M) {
    case 1: hipLaunchKernelGGL(gemv_f32<1>, dim3(nblk), dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL(gemv_f32<2>, dim3(nblk), dim3(256), 0, s, a); break;
    case 3: case 4: hipLaunchKernelGGL(gemv_f32<4>, dim3(nblk), dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL(gemv_f32<8>, dim3(nblk), dim3(256), 0, s, a); break;
  }
}

int gemm_f32(const az_gemm_desc* d, hipStream_t s) {
  AZ_REQUIRE(d != nullptr, AZ_EINVAL, "az_gemm_f32: null descriptor");
  AZ_REQUIRE(d->M >= 0 && d->N >= 0 && d->K >= 0, AZ_EINVAL, "az_gemm_f32: negative size");
  if (d->M == 0 || d->N == 0) return AZ_OK;
  AZ_REQUIRE(d->A && d->B && d->C, AZ_EINVAL, "az_gemm_f32: null A/B/C");
  AZ_REQUIRE(d->K % 4 == 0, AZ_EINVAL, "az_gemm_f32: K=%d must be a multiple of 4", d->K);
  const bool akm = d->a_kmajor != 0, bkm = d->b_kmajor != 0;
  AZ_REQUIRE(d->lda % 4 == 0 && aligned16(d->A), AZ_EINVAL, "az_gemm_f32: A needs lda%%4==0, 16B alignment");
  AZ_REQUIRE(d->ldb % 4 == 0 && aligned16(d->B), AZ_EINVAL, "az_gemm_f32: B needs ldb%%4==0, 16B alignment");
  if (d->A2) {
    AZ_REQUIRE(akm, AZ_EINVAL, "az_gemm_f32: A2 needs a K-major A");
    AZ_REQUIRE(d->K0 % 16 == 0 && d->K0 > 0 && d->K0 < d->K, AZ_EINVAL, "az_gemm_f32: K0 must be a multiple of 16 inside (0,K)");
    AZ_REQUIRE(d->lda2 % 4 == 0 && aligned16(d->A2), AZ_EINVAL, "az_gemm_f32: A2 needs lda2%%4==0, 16B alignment");
  }
  AZ_REQUIRE(!d->a_rows || akm, AZ_EINVAL, "az_gemm_f32: a_rows needs a K-major A");
  AZ_REQUIRE(akm || d->M % 4 == 0, AZ_EINVAL, "az_gemm_f32: M-major A needs M%%4==0");
  AZ_REQUIRE(bkm || d->N % 4 == 0, AZ_EINVAL, "az_gemm_f32: N-major B needs N%%4==0");
  AZ_REQUIRE(d->act >= 0 && d->act <= 3, AZ_EINVAL, "az_gemm_f32: bad act %d", d->act);

  GemmArgs a;
  a.M = d->M; a.N = d->N; a.K = d->K;
  a.A = d->A; a.lda = d->lda; a.A2 = d->A2; a.lda2 = d->lda2; a.K0 = d->A2 ? d->K0 : d->K;
  a.a_rows = d->a_rows; a.B = d->B; a.ldb = d->ldb;
  a.bias = d->bias; a.act = d->act; a.R = d->R; a.ldr = d->ldr; a.G = d->G; a.ldg = d->ldg;
  a.beta = d->beta; a.C = d->C; a.ldc = d->ldc; a.c_rows = d->c_rows;

  if (d->M <= 8 && akm && bkm) {
    launch_gemv(a, s);
    return check_launch("gemv_f32");
  }
  const long t128 = (long)((d->M + 127) / 128) * ((d->N + 127) / 128);
  if (t128 >= 240) launch_tile<128, 128>(a, akm, bkm, s);
  else launch_tile<64, 64>(a, akm, bkm, s);
  return check_launch("gemm_f32_mfma");
}

}  // namespace az

extern "C" int az_gemm_f32(const az_gemm_desc* d, void* stream) {
  return az::gemm_f32(d, az::as_stream(stream));
}
