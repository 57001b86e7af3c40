// bf16 MFMA GEMM with ONE wave per SIMD: 256 x 256 tiles, 4 waves (2 x 2) of 128 x 128, BK = 32, 4-stage
// LDS-DMA ring, ONE barrier per K-step.
//
//   C[m][n] = Σ_k A(m,k) · B(n,k)        fp32 accumulate, v_mfma_f32_16x16x32_bf16
//
// Why next to gemm2 (8 waves of 128 x 64, four barrier-separated MFMA phases per 64-deep K-tile): a 128 x 128
// wave tile reads 2/3 of gemm2's LDS bytes per MFMA (16 fragments per 64 MFMAs instead of 12 per 32), and
// with one wave per SIMD nothing but the wave's own program order decides when its matrix pipe is fed —
// no partner-wave arbitration, no 8-barrier-per-K-tile rendezvous (rocprofv3 PMC on gemm2: MFMA busy
// 37-49 %, waves parked at s_waitcnt / s_barrier 33-43 % of their cycles). The price is that the wave
// itself must keep LDS reads and LDS-DMA issue in flight behind its MFMAs: fragments of step t+1 are read
// while step t's 64 MFMAs run (two register sets), and stages t+1..t+3 are in flight (4-stage ring).
//
// Register budget (one wave per SIMD -> up to 512 per lane): 256 accumulators (acc[8][8] of 16 x 16
// blocks, the layout gemm_common.h's bf16 epilogue takes at WN = 128) + 2 x 64 fragment registers.
//
// LDS images (source-swizzled LDS-DMA, lane-linear destination — cdna_hip_programming.md rule 21): each
// operand stage is [256 rows][32 k] bf16 (64-B rows), 16-B chunk c stored at c ^ ((-(row >> 2)) & 3)
// (gemm3.hip's image: conflict-free for the ds_read_b128 lane groups, tools/lds_banks.py).
//
// Pipeline (K-step t consumes stage t % 4):
//   s_waitcnt vmcnt(8)  -> this wave's DMA of step t+1 landed (8 DMA wave-instructions per step per wave)
//   s_barrier           -> step t+1 visible to every wave; every wave done with step t-1's stage
//   DMA step t+3 into step t-1's stage; read step t+1's fragments; 64 MFMAs on step t's fragments.
#include "gemm_common.h"

#include <stdlib.h>

namespace hsd {
namespace g4 {

constexpr int BM = 256, BN = 256, BK = 32, NSTAGE = 4;
constexpr int TA = BM * BK, TB = BN * BK, STAGE = TA + TB;  // elements per stage (32 KiB)
constexpr int GA = 4, GB = 4;                               // DMA wave-instructions per wave per stage
constexpr int G = GA + GB;

__device__ __forceinline__ int swz(int row) { return (-(row >> 2)) & 3; }

// DMA wave-instruction g (1 KiB = 16 rows x 64 B) of a [256 rows][32 k] image
__device__ __forceinline__ void dma(bf16_t* img, const bf16_t* __restrict__ X, int64_t ld, int r0, int Rmax, int k0,
                                    int g, int lane) {
  const int row = g * 16 + (lane >> 2);
  const int c = (lane & 3) ^ swz(row);
  const int rr = min(r0 + row, Rmax - 1);
  const bf16_t* src = X + (int64_t)rr * ld + k0 + c * 8;
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)(img + g * 512), 16, 0, 0);
}

// 16x16x32 fragment: lane l holds row rbase + (l & 15), k = 8 (l >> 4) + 0..7
__device__ __forceinline__ bf16x8 frag(const bf16_t* img, int rbase, int lane) {
  const int row = rbase + (lane & 15);
  const int ch = lane >> 4;
  return *reinterpret_cast<const bf16x8*>(img + row * BK + ((ch ^ swz(row)) << 3));
}

template <int N>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

#define G4_BARRIER()                       \
  do {                                     \
    asm volatile("" ::: "memory");         \
    __builtin_amdgcn_sched_barrier(0);     \
    __builtin_amdgcn_s_barrier();          \
    __builtin_amdgcn_sched_barrier(0);     \
    asm volatile("" ::: "memory");         \
  } while (0)

template <int EPI, int SCHED>
__global__ __launch_bounds__(256, 1) void gemm4_kernel(G2Params p) {
  p.dp = resolve_seed(p.dp);
  __shared__ __attribute__((aligned(16))) bf16_t smem[NSTAGE * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap (gemm2.hip): the tiles one XCD runs together are neighbours -> shared panels in L2
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tm = wg / p.tiles_n, tn = wg % p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nt = p.K / BK;
  HSD_DASSERT(wg < nwg && m0 < p.M && n0 < p.N && p.K % BK == 0 && nt >= 1);

  auto dma_step = [&](int t) {
    bf16_t* st = smem + (t & (NSTAGE - 1)) * STAGE;
    const int k0 = t * BK;
#pragma unroll
    for (int q = 0; q < GA; ++q) dma(st, p.A, p.lda, m0, p.M, k0, wave * GA + q, lane);
#pragma unroll
    for (int q = 0; q < GB; ++q) dma(st + TA, p.B, p.ldb, n0, p.N, k0, wave * GB + q, lane);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int arow = wm * 128, bcol = wn * 128;
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];

  // prologue: steps 0, 1, 2 in flight; step 0 landed -> its fragments
  dma_step(0);
  if (nt > 1) dma_step(1);
  if (nt > 2) dma_step(2);
  if (nt > 2) vmcnt<2 * G>();
  else if (nt > 1) vmcnt<G>();
  else vmcnt<0>();
  G4_BARRIER();
#pragma unroll
  for (int i = 0; i < 8; ++i) fa0[i] = frag(smem, arow + 16 * i, lane);
#pragma unroll
  for (int j = 0; j < 8; ++j) fb0[j] = frag(smem + TA, bcol + 16 * j, lane);

  // one K-step: wait for step t+1, publish, DMA t+3, read t+1 into (FAn, FBn), MFMAs on (FAc, FBc).
  // FULL: steady state (steps t+1..t+3 exist) -> branch-free body the scheduling hints apply to.
#define G4_STEP(FULL, FAc, FBc, FAn, FBn)                                                                   \
  {                                                                                                         \
    const bool h1 = FULL || t + 1 < nt, h2 = FULL || t + 2 < nt, h3 = FULL || t + 3 < nt;                  \
    if (h2) vmcnt<G>();                                                                                     \
    else vmcnt<0>();                                                                                        \
    G4_BARRIER();                                                                                           \
    if (h3 && !(SCHED == 3 && FULL)) dma_step(t + 3);                                                       \
    if (h1 && !(SCHED == 3 && FULL)) {                                                                      \
      const bf16_t* ns = smem + ((t + 1) & (NSTAGE - 1)) * STAGE;                                           \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) FAn[i] = frag(ns, arow + 16 * i, lane);                 \
      _Pragma("unroll") for (int j = 0; j < 8; ++j) FBn[j] = frag(ns + TA, bcol + 16 * j, lane);            \
    }                                                                                                       \
    if constexpr (SCHED == 3 && FULL) {                                                                     \
      /* 8 fenced groups: {fragment reads A_g, B_g of step t+1, DMA piece g of step t+3, 8 MFMAs row-block g} */ \
      const bf16_t* ns = smem + ((t + 1) & (NSTAGE - 1)) * STAGE;                                           \
      bf16_t* ds = smem + ((t + 3) & (NSTAGE - 1)) * STAGE;                                                 \
      const int k3 = (t + 3) * BK;                                                                          \
      _Pragma("unroll") for (int g = 0; g < 8; ++g) {                                                       \
        FAn[g] = frag(ns, arow + 16 * g, lane);                                                             \
        FBn[g] = frag(ns + TA, bcol + 16 * g, lane);                                                        \
        if (g < GA) dma(ds, p.A, p.lda, m0, p.M, k3, wave * GA + g, lane);                                  \
        else dma(ds + TA, p.B, p.ldb, n0, p.N, k3, wave * GB + (g - GA), lane);                             \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) acc[g][j] =                                           \
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(FBc[j], FAc[g], acc[g][j], 0, 0, 0);                    \
        __builtin_amdgcn_sched_barrier(0);                                                                  \
      }                                                                                                     \
    } else {                                                                                                \
    if constexpr (SCHED == 1) __builtin_amdgcn_s_setprio(1);                                                \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) _Pragma("unroll") for (int j = 0; j < 8; ++j) acc[i][j] = \
        __builtin_amdgcn_mfma_f32_16x16x32_bf16(FBc[j], FAc[i], acc[i][j], 0, 0, 0);                        \
    if constexpr (SCHED == 1) __builtin_amdgcn_s_setprio(0);                                                \
    }                                                                                                       \
    if constexpr (SCHED == 2 && FULL) {                                                                     \
      /* interleave: a DMA wave-instruction and two fragment reads per 8 MFMAs */                           \
      _Pragma("unroll") for (int g = 0; g < 8; ++g) {                                                       \
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                                  \
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);                                                  \
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);                                                  \
      }                                                                                                     \
    }                                                                                                       \
  }

  int t = 0;
  for (; t + 4 < nt; t += 2) {  // steps t, t+1 both with t+3 / t+4 present
    G4_STEP(true, fa0, fb0, fa1, fb1)
    ++t;
    G4_STEP(true, fa1, fb1, fa0, fb0)
    --t;
  }
  // tail: at most 4 steps left
  for (; t < nt; t += 2) {
    G4_STEP(false, fa0, fb0, fa1, fb1)
    ++t;
    if (t < nt) G4_STEP(false, fa1, fb1, fa0, fb0)
    --t;
  }
#undef G4_STEP

  // epilogue: the LDS ring becomes the bf16 staging area (every wave past its last fragment read)
  vmcnt<0>();
  G4_BARRIER();
  constexpr bool F32OUT = EPI == E2_F32_ATOMIC || EPI == E2_F32_SLAB;
  static_assert(!F32OUT, "gemm4: bf16 epilogues only");
  g2::epilogue_bf16<EPI, 512>(acc, p, smem, wave, lane, m0 + arow, n0 + bcol);
}

}  // namespace g4

bool gemm4_supported(int la, int lb, int epi, int M, int N, int K) {
  if (la != 0 || lb != 0) return false;
  if (!epi_bf16_out(epi)) return false;
  // fused bias-gradient column sums need gemm2's 8-column-per-lane epilogue layout
  return M >= 1 && N % 256 == 0 && K % 32 == 0 && K >= 32;
}

static int gemm4_sched() {
  const char* e = getenv("HSD_G4_SCHED");
  return e ? atoi(e) : 0;
}

template <int EPI>
static void g4_launch(const G2Params& p0, hipStream_t st) {
  G2Params p = p0;
  const int tiles_m = (p.M + g4::BM - 1) / g4::BM;
  p.tiles_n = p.N / g4::BN;
  p.ntiles = tiles_m * p.tiles_n;
  p.kps = p.K;
  const int s = gemm4_sched();
  if (s == 1) hipLaunchKernelGGL((g4::gemm4_kernel<EPI, 1>), dim3(p.ntiles), dim3(256), 0, st, p);
  else if (s == 3) hipLaunchKernelGGL((g4::gemm4_kernel<EPI, 3>), dim3(p.ntiles), dim3(256), 0, st, p);
  else if (s == 2) hipLaunchKernelGGL((g4::gemm4_kernel<EPI, 2>), dim3(p.ntiles), dim3(256), 0, st, p);
  else hipLaunchKernelGGL((g4::gemm4_kernel<EPI, 0>), dim3(p.ntiles), dim3(256), 0, st, p);
  HSD_CHECK_LAUNCH();
}

void launch_gemm4(int epi, const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, int M, int N, int K, bf16_t* C,
                  int64_t ldc, const bf16_t* bias, const bf16_t* aux, int64_t ldaux, bf16_t* C2, double p_drop,
                  uint64_t seed, hipStream_t st) {
  if (!gemm4_supported(0, 0, epi, M, N, K)) abort();
  G2Params p{};
  p.A = A; p.lda = lda; p.B = B; p.ldb = ldb; p.M = M; p.N = N; p.K = K; p.C = C; p.ldc = ldc;
  p.bias = bias; p.aux = aux; p.ldaux = ldaux; p.C2 = C2;
  p.dp = make_dropout(p_drop, seed);
  switch (epi) {
    case E2_STORE: g4_launch<E2_STORE>(p, st); return;
    case E2_BIAS: g4_launch<E2_BIAS>(p, st); return;
    case E2_BIAS_GELU: g4_launch<E2_BIAS_GELU>(p, st); return;
    case E2_BIAS_DROP_RES: g4_launch<E2_BIAS_DROP_RES>(p, st); return;
    case E2_RES: g4_launch<E2_RES>(p, st); return;
    case E2_DGELU: g4_launch<E2_DGELU>(p, st); return;
    case E2_BIAS_GELU_D: g4_launch<E2_BIAS_GELU_D>(p, st); return;
    case E2_MUL: g4_launch<E2_MUL>(p, st); return;
    default: abort();
  }
}

}  // namespace hsd
