// bf16 MFMA GEMM for TWO workgroups per CU: 256 x 128 tiles, 4 waves, BK = 32, 3-stage LDS-DMA ring.
//
//   C[m][n] = Σ_k A(m,k) · B(n,k)        fp32 accumulate, v_mfma_f32_16x16x32_bf16
//
// Why a second GEMM body next to gemm2 (one 8-wave 256 x 256 workgroup per CU): gemm2's epilogue (bias /
// GELU / dropout math, two bf16 outputs, derivative products, column sums) runs with nothing else on the CU,
// and a K = 768 tile has only 12 K-steps of MFMA work to amortise it — the FFN1 forward (GELU + GELU' out)
// and the FFN2 dgrad (× GELU', bias-gradient column sums) run at 700-800 TFLOP/s against ~1,050 for the
// plain-store tile. Here each CU holds two independent 4-wave workgroups (72 KiB LDS and <= 256 VGPRs each,
// __launch_bounds__(256, 2)): while one workgroup is in its epilogue or prologue, its partner's waves — one
// on every SIMD — keep the matrix pipes busy (MI355X_MICROARCH.md "Two waves per SIMD": MFMA and VALU of
// different waves co-issue). The same residency hides the barrier / LDS-read bubbles of the transposing
// (TT) weight-gradient main loop, which gemm2 runs at ~37 % MFMA-busy.
//
// Wave tile 128 x 64 (acc[8][4] of 16 x 16 blocks, the layout of gemm2's 256-wide tile, so the bf16 epilogue
// of gemm_common.h is shared). Waves 2 (M) x 2 (N).
//
// LDS images (source-swizzled LDS-DMA, lane-linear destination, cdna_hip_programming.md §5.4 rule 21):
//   k-contiguous operand  [rows][32 k], 64-B rows, 16-B chunk c at position c ^ ((-(row >> 2)) & 3):
//     fragments by ds_read_b128, conflict-free for the b128 lane groups (tools/lds_banks.py model);
//   k-strided operand     [32 k][R], R = 256 or 128 (512-B / 256-B rows), chunk ^ f2(k) as gemm2, fragments
//     by ds_read_b64_tr_b16 (conflict-free at both widths).
//
// Pipeline: stages t, t+1 in flight while t is consumed; ONE barrier per K-step:
//   vmcnt(6)  -> stage t landed (6 DMA wave-instructions per stage per wave)
//   s_barrier -> stage t visible to every wave; every wave done reading stage t-1's buffer
//   DMA stage t+2 into that buffer, read stage t's fragments, 32 MFMAs.
#include "gemm_common.h"

#include <stdlib.h>

#include <algorithm>

namespace hsd {
namespace g3 {

constexpr int BM = 256, BN = 128, BK = 32, NSTAGE = 3;
constexpr int TA = BM * BK, TB = BN * BK, STAGE = TA + TB;  // elements
constexpr int GA = 4, GB = 2;                               // DMA wave-instructions per wave per stage
constexpr int DMA_PER_STAGE = GA + GB;

__device__ __forceinline__ int swz(int row) { return (-(row >> 2)) & 3; }
__device__ __forceinline__ int f2(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;

// DMA wave-instruction `g` (1 KiB) of a [R rows][32 k] (L = 0) or [32 k][R] (L = 1) image.
template <int L, int R>
__device__ __forceinline__ void dma(bf16_t* img, const bf16_t* __restrict__ X, int64_t ld, int r0, int Rmax, int k0,
                                    int g, int lane) {
  const bf16_t* src;
  if constexpr (L == 0) {
    const int row = g * 16 + (lane >> 2);
    const int c = (lane & 3) ^ swz(row);
    const int rr = min(r0 + row, Rmax - 1);
    src = X + (int64_t)rr * ld + k0 + c * 8;
  } else {
    constexpr int LPR = R / 8;           // lanes per k-row (16-B chunks per row): 32 or 16
    constexpr int RPI = 64 / LPR;        // k-rows per instruction: 2 or 4
    const int krow = g * RPI + lane / LPR;
    const int lc = (lane % LPR) ^ f2(krow);
    const int cc = min(r0 + lc * 8, Rmax - 8);
    src = X + (int64_t)(k0 + krow) * ld + cc;
  }
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)(img + g * 512), 16, 0, 0);
}

// 16x16x32 fragment: lane l holds row rbase + (l & 15), k = 8 (l >> 4) + 0..7
template <int L, int R>
__device__ __forceinline__ bf16x8 frag(const bf16_t* img, int rbase, int lane) {
  if constexpr (L == 0) {
    const int row = rbase + (lane & 15);
    const int ch = lane >> 4;
    return *reinterpret_cast<const bf16x8*>(img + row * BK + ((ch ^ swz(row)) << 3));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int k = 8 * g + q, k2 = k + 4;
    const int m = rbase + 4 * p;
    bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_bf16x4_t*)(img + k * R + (((m >> 3) ^ f2(k)) << 3) + (m & 7)));
    bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_bf16x4_t*)(img + k2 * R + (((m >> 3) ^ f2(k2)) << 3) + (m & 7)));
    bf16x8 r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  }
}

template <int N>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int LA, int LB, int EPI>
__global__ __launch_bounds__(256, 2) void gemm3_kernel(G2Params p) {
  p.dp = resolve_seed(p.dp);
  constexpr bool F32OUT = EPI == E2_F32_ATOMIC || EPI == E2_F32_SLAB;
  __shared__ __attribute__((aligned(16))) bf16_t smem[NSTAGE * STAGE];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap (gemm2): blocks an XCD runs together get consecutive (split-major) indices
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int split = v / p.ntiles, wg = v % p.ntiles;
  const int m0 = (wg / p.tiles_n) * BM, n0 = (wg % p.tiles_n) * BN;
  const int kbeg = split * p.kps;
  const int kend = min(p.K, kbeg + p.kps);
  const int nt = (kend - kbeg) / BK;
  HSD_DASSERT(v < nwg && m0 < p.M && n0 < p.N && (kend - kbeg) % BK == 0 && nt >= 1);

  auto dma_stage = [&](int s, int k0) {
    bf16_t* st = smem + s * STAGE;
#pragma unroll
    for (int q = 0; q < GA; ++q) dma<LA, BM>(st, p.A, p.lda, m0, p.M, k0, wave * GA + q, lane);
#pragma unroll
    for (int q = 0; q < GB; ++q) dma<LB, BN>(st + TA, p.B, p.ldb, n0, p.N, k0, wave * GB + q, lane);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int arow = wm * 128, bcol = wn * 64;
  dma_stage(0, kbeg);
  if (nt > 1) dma_stage(1, kbeg + BK);
  int cs = 0;  // stage holding K-step t
  for (int t = 0; t < nt; ++t) {
    if (t + 1 < nt) vmcnt<DMA_PER_STAGE>();
    else vmcnt<0>();
    G2_BARRIER();
    const int ns = cs == 0 ? 2 : cs - 1;  // (t + 2) % 3: the buffer every wave finished reading at step t - 1
    if (t + 2 < nt) dma_stage(ns, kbeg + (t + 2) * BK);
    const bf16_t* cA = smem + cs * STAGE;
    const bf16_t* cB = cA + TA;
    bf16x8 fa[8], fb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = frag<LB, BN>(cB, bcol + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = frag<LA, BM>(cA, arow + 16 * i, lane);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    cs = cs == 2 ? 0 : cs + 1;
  }
  // every wave past its last LDS read before the epilogue reuses the stages as staging space
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  G2_BARRIER();

  const int mw = m0 + arow, nw = n0 + bcol;
  if constexpr (F32OUT) {
    const int q4 = lane >> 4, lr = lane & 15;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mw + 16 * i + lr;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nw + 16 * j + 4 * q4;
        if (n >= p.N) continue;
        if constexpr (EPI == E2_F32_ATOMIC) {
          float* c = reinterpret_cast<float*>(p.C) + (int64_t)m * p.ldc + n;
          atomicAdd(c + 0, acc[i][j][0]);
          atomicAdd(c + 1, acc[i][j][1]);
          atomicAdd(c + 2, acc[i][j][2]);
          atomicAdd(c + 3, acc[i][j][3]);
        } else {
          float* c = reinterpret_cast<float*>(p.C) + (int64_t)split * p.M * p.N + (int64_t)m * p.N + n;
          *reinterpret_cast<f32x4*>(c) = acc[i][j];
        }
      }
    }
  } else {
    // wave-private [64][64] staging slices (8 KiB each) inside the now idle operand stages
    g2::epilogue_bf16<EPI, 256>(acc, p, smem, wave, lane, mw, nw);
  }
}

__global__ __launch_bounds__(256) void slab_reduce3_kernel(const float* __restrict__ ws, float* __restrict__ C,
                                                          int64_t ldc, int M, int N, int splits) {
  const int64_t n4 = (int64_t)M * N / 4;
  const int64_t plane = (int64_t)M * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i * 4;
    f32x4 s = *reinterpret_cast<const f32x4*>(ws + e);
    for (int k = 1; k < splits; ++k) s += *reinterpret_cast<const f32x4*>(ws + k * plane + e);
    const int64_t m = e / N, n = e % N;
    f32x4* c = reinterpret_cast<f32x4*>(C + m * ldc + n);
    *c = *c + s;
  }
}

}  // namespace g3

// staging slices of the bf16 epilogue: 4 waves x 8 KiB must fit the operand stages
static_assert(4 * 64 * 64 <= g3::NSTAGE * g3::STAGE, "gemm3 epilogue staging");

bool gemm3_supported(int la, int lb, int epi, int M, int N, int K) {
  if (K % g3::BK || M < 1 || N % g3::BN) return false;
  if (la == 0 && lb == 0) return epi_bf16_out(epi);
  if (la == 1 && lb == 1) return (epi == E2_F32_ATOMIC || epi == E2_F32_SLAB) && M % 8 == 0;
  return false;
}

// splits for the TT wgrad: fill two workgroups per CU with >= 8 K-steps each
int gemm3_wgrad_splits(int M, int N, int K) {
  const int tiles = ((M + g3::BM - 1) / g3::BM) * (N / g3::BN);
  int s = 512 / tiles;
  if (s < 1) s = 1;
  const int kt = K / g3::BK;
  while (s > 1 && kt / s < 8) --s;
  return s;
}

template <int LA, int LB, int EPI>
static void g3_launch(const G2Params& p0, int splits, hipStream_t st) {
  G2Params p = p0;
  const int tiles_m = (p.M + g3::BM - 1) / g3::BM;
  p.tiles_n = p.N / g3::BN;
  if (splits < 1) splits = 1;
  int kps = (p.K + splits - 1) / splits;
  kps = (kps + g3::BK - 1) / g3::BK * g3::BK;
  splits = (p.K + kps - 1) / kps;
  p.kps = kps;
  p.ntiles = tiles_m * p.tiles_n;
  hipLaunchKernelGGL((g3::gemm3_kernel<LA, LB, EPI>), dim3(p.ntiles * splits), dim3(256), 0, st, p);
  HSD_CHECK_LAUNCH();
}

void launch_gemm3(int la, int lb, int epi, const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, int M, int N,
                  int K, void* C, int64_t ldc, const bf16_t* bias, const bf16_t* aux, int64_t ldaux, bf16_t* C2,
                  double p_drop, uint64_t seed, int splits, float* ws, float* dbias, hipStream_t st) {
  G2Params p{};
  p.dbias = dbias;
  p.A = A; p.lda = lda; p.B = B; p.ldb = ldb; p.M = M; p.N = N; p.K = K; p.C = C; p.ldc = ldc;
  p.bias = bias; p.aux = aux; p.ldaux = ldaux; p.C2 = C2;
  p.dp = make_dropout(p_drop, seed);
  if (!gemm3_supported(la, lb, epi, M, N, K)) abort();
  if (la == 0 && lb == 0) {
    switch (epi) {
      case E2_STORE: g3_launch<0, 0, E2_STORE>(p, 1, st); return;
      case E2_BIAS: g3_launch<0, 0, E2_BIAS>(p, 1, st); return;
      case E2_BIAS_GELU: g3_launch<0, 0, E2_BIAS_GELU>(p, 1, st); return;
      case E2_BIAS_DROP_RES: g3_launch<0, 0, E2_BIAS_DROP_RES>(p, 1, st); return;
      case E2_RES: g3_launch<0, 0, E2_RES>(p, 1, st); return;
      case E2_DGELU: g3_launch<0, 0, E2_DGELU>(p, 1, st); return;
      case E2_BIAS_GELU_D: g3_launch<0, 0, E2_BIAS_GELU_D>(p, 1, st); return;
      case E2_MUL: g3_launch<0, 0, E2_MUL>(p, 1, st); return;
      default: abort();
    }
  }
  if (splits <= 0) splits = gemm3_wgrad_splits(M, N, K);
  if (epi == E2_F32_SLAB && splits > 1 && ws != nullptr) {
    G2Params q = p;
    q.C = ws;
    g3_launch<1, 1, E2_F32_SLAB>(q, splits, st);
    int kps = (K + splits - 1) / splits;
    kps = (kps + g3::BK - 1) / g3::BK * g3::BK;
    const int real = (K + kps - 1) / kps;
    const int64_t n4 = (int64_t)M * N / 4;
    const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
    hipLaunchKernelGGL(g3::slab_reduce3_kernel, dim3(blocks), dim3(256), 0, st, ws, reinterpret_cast<float*>(C), ldc,
                       M, N, real);
    HSD_CHECK_LAUNCH();
  } else {
    g3_launch<1, 1, E2_F32_ATOMIC>(p, splits, st);
  }
}

}  // namespace hsd
