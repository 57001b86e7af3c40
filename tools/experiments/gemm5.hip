// Experimental bf16 NT GEMM, one wave per SIMD (4 waves of 128 x 128), 256 x 256 x 64 tiles, with the loop
// structure of a register-prefetch pipeline (one fragment set per k-half with FIXED roles, so the register
// allocator never has to swap accumulators or fragments between loop iterations — the failure of gemm4):
//
//   F0 = fragments of k-half 0, F1 = fragments of k-half 1 (16 x bf16x8 each), two LDS stages (LDS-DMA).
//   iteration t:  [64 MFMAs on F0(t)]  +  reads F1(t)                       (stage t)
//                 lgkmcnt(0), vmcnt(0), s_barrier   -> stage t free, tile t+1 landed and visible
//                 [64 MFMAs on F1(t)]  +  DMA tile t+2 -> stage t  +  reads F0(t+1)  (stage t+1)
#include "gemm_common.h"

#include <stdlib.h>

namespace hsd {
namespace g5 {

constexpr int BM = 256, BK = 64;
constexpr int TA = BM * BK;
constexpr int GA = 8;  // A DMA wave-instructions per wave per stage (1 KiB each)

__device__ __forceinline__ int f1(int row) { return (row >> 1) & 7; }

// DMA wave-instruction g (8 rows x 128 B) of a [256 rows][64 k] image, 16-B chunk c at c ^ f1(row)
__device__ __forceinline__ void dma(bf16_t* img, const bf16_t* __restrict__ X, int64_t ld, int r0, int Rmax, int k0,
                                    int g, int lane) {
  const int row = g * 8 + (lane >> 3);
  const int lc = (lane & 7) ^ f1(row);
  const int rr = min(r0 + row, Rmax - 1);
  const bf16_t* src = X + (int64_t)rr * ld + k0 + lc * 8;
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)(img + g * 512), 16, 0, 0);
}

// 16x16x32 fragment of k-half ks: lane l holds row rbase + (l & 15), k = 32 ks + 8 (l >> 4) + 0..7
__device__ __forceinline__ bf16x8 frag(const bf16_t* img, int rbase, int ks, int lane) {
  const int row = rbase + (lane & 15);
  const int ch = (lane >> 4) + 4 * ks;
  return *reinterpret_cast<const bf16x8*>(img + row * 64 + ((ch ^ f1(row)) << 3));
}

template <int N>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

#define G5_BARRIER()                       \
  do {                                     \
    asm volatile("" ::: "memory");         \
    __builtin_amdgcn_sched_barrier(0);     \
    __builtin_amdgcn_s_barrier();          \
    __builtin_amdgcn_sched_barrier(0);     \
    asm volatile("" ::: "memory");         \
  } while (0)

template <int EPI, int SCHED, int WN>
__global__ __launch_bounds__(256, 1) void gemm5_kernel(G2Params p) {
  constexpr int BN = 2 * WN, NJ = WN / 16;
  constexpr int STAGE = TA + BN * BK;
  constexpr int GB = BN / 32;  // B DMA wave-instructions per wave per stage
  p.dp = resolve_seed(p.dp);
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tm = wg / p.tiles_n, tn = wg % p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  HSD_DASSERT(p.N % BN == 0);
  const int nt = p.K / BK;
  const int arow = wm * 128, bcol = wn * WN;

  auto dma_tile = [&](int t, bf16_t* st) {
    const int k0 = t * BK;
#pragma unroll
    for (int q = 0; q < GA; ++q) dma(st, p.A, p.lda, m0, p.M, k0, wave * GA + q, lane);
#pragma unroll
    for (int q = 0; q < GB; ++q) dma(st + TA, p.B, p.ldb, n0, p.N, k0, wave * GB + q, lane);
  };

  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // B fragments of one k-half for all 8 column blocks (32 VGPRs, two sets); A fragments streamed one row
  // block ahead (2 x 4 VGPRs) — 80 fragment registers instead of 128, so the accumulators keep their AGPRs.
  bf16x8 b0[NJ], b1[NJ], aa, ab;

  dma_tile(0, smem);
  if (nt > 1) dma_tile(1, smem + STAGE);
  if (nt > 1) vmcnt<GA + GB>();
  else vmcnt<0>();
  G5_BARRIER();
#pragma unroll
  for (int j = 0; j < NJ; ++j) b0[j] = frag(smem + TA, bcol + 16 * j, 0, lane);
  aa = frag(smem, arow, 0, lane);

  for (int t = 0; t < nt; ++t) {
    const bf16_t* cs = smem + (t & 1) * STAGE;
    bf16_t* ns = smem + ((t + 1) & 1) * STAGE;
    // half 0 on (A rows streamed, b0); reads b1 of this tile; A of half 1 starts streaming
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i < 7) ab = frag(cs, arow + 16 * (i + 1), 0, lane);
      else ab = frag(cs, arow, 1, lane);
      if (i < NJ) b1[i] = frag(cs + TA, bcol + 16 * i, 1, lane);
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[j], aa, acc[i][j], 0, 0, 0);
      aa = ab;
      if constexpr (SCHED == 1) __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    vmcnt<0>();
    G5_BARRIER();
    if (t + 2 < nt) dma_tile(t + 2, const_cast<bf16_t*>(cs));
    // half 1 on (A rows streamed, b1); reads b0 of the next tile; A of its half 0 starts streaming
    const bool more = t + 1 < nt;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i < 7) ab = frag(cs, arow + 16 * (i + 1), 1, lane);
      else if (more) ab = frag(ns, arow, 0, lane);
      if (more && i < NJ) b0[i] = frag(ns + TA, bcol + 16 * i, 0, lane);
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], aa, acc[i][j], 0, 0, 0);
      aa = ab;
      if constexpr (SCHED == 1) __builtin_amdgcn_sched_barrier(0);
    }
  }
  vmcnt<0>();
  G5_BARRIER();
  g2::epilogue_bf16<EPI, 4 * WN>(acc, p, smem, wave, lane, m0 + arow, n0 + bcol);
}

}  // namespace g5

static int gemm5_sched() {
  const char* e = getenv("HSD_G5_SCHED");
  return e ? atoi(e) : 0;
}

void launch_gemm5(int epi, const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, int M, int N, int K, bf16_t* C,
                  int64_t ldc, const bf16_t* bias, const bf16_t* aux, int64_t ldaux, bf16_t* C2, double p_drop,
                  uint64_t seed, hipStream_t st) {
  const int wn = getenv("HSD_G5_WN") ? atoi(getenv("HSD_G5_WN")) : 96;
  if (N % (2 * wn) || K % 64) abort();
  G2Params p{};
  p.A = A; p.lda = lda; p.B = B; p.ldb = ldb; p.M = M; p.N = N; p.K = K; p.C = C; p.ldc = ldc;
  p.bias = bias; p.aux = aux; p.ldaux = ldaux; p.C2 = C2;
  p.dp = make_dropout(p_drop, seed);
  p.tiles_n = N / (2 * wn);
  p.ntiles = ((M + 255) / 256) * p.tiles_n;
  p.kps = K;
  if (epi != E2_STORE) abort();
  if (wn == 128) {
    if (gemm5_sched() == 1) hipLaunchKernelGGL((g5::gemm5_kernel<E2_STORE, 1, 128>), dim3(p.ntiles), dim3(256), 0, st, p);
    else hipLaunchKernelGGL((g5::gemm5_kernel<E2_STORE, 0, 128>), dim3(p.ntiles), dim3(256), 0, st, p);
  } else {
    if (gemm5_sched() == 1) hipLaunchKernelGGL((g5::gemm5_kernel<E2_STORE, 1, 96>), dim3(p.ntiles), dim3(256), 0, st, p);
    else hipLaunchKernelGGL((g5::gemm5_kernel<E2_STORE, 0, 96>), dim3(p.ntiles), dim3(256), 0, st, p);
  }
}

}  // namespace hsd
