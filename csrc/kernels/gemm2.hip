// bf16 MFMA GEMM, 256-row tiles, 8-phase-style schedule (cdna_hip_programming.md §5 "256² 8-phase
// template": T1 XCD remap, T2 source-swizzled LDS images, T3/T4 phase interleave with counted vmcnt
// across raw s_barriers, T5 s_setprio around the MFMA clusters).
//
//   C[m][n] = Σ_k A(m,k) · B(n,k)        fp32 accumulate, v_mfma_f32_16x16x32_bf16
//
// Operand layouts (template LA / LB):
//   0 = k-contiguous   A[M][K] / B[N][K]  -> LDS image [rows][64 k], 128-B rows, 16-B chunk ^ ((row>>1)&7),
//                                            fragments by ds_read_b128
//   1 = k-strided      A[K][M] / B[K][N]  -> LDS image [64 k][256], 512-B rows,
//                                            16-B chunk ^ 2·((k&3) | ((k>>3)&1)<<2), fragments by the
//                                            transposing ds_read_b64_tr_b16
// (both images bank-conflict-free for their fragment reads: tools/lds_banks.py model).
//
// Uses in the BERT step:
//   forward  Y  = X · Wᵀ    NT  (LA=0, LB=0)   bf16 out + fused epilogue
//   dgrad    dX = dY · W    NT with Wᵀ stored [K][N] -> B(n,k) = Wᵀ[n][k]  (LA=0, LB=0)
//   wgrad    dW += dYᵀ · X  TT  (LA=1, LB=1)   fp32 out, split-K over tokens into slabs + reduce
//
// Block = 512 threads = 8 waves as 2 (M) x 4 (N); tile 256 x BN x 64; wave tile 128 x BN/4.
// Per K-tile a wave runs 4 phases over its output quadrants (A rows 0-63 / 64-127 of the wave,
// B cols first / second half): P1 reads A-sub0 + B-sub0, P2 B-sub1, P3 A-sub1, P4 no reads. The
// next K-tile's LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave instruction) is spread over
// P4(prev) / P1 / P2 / P3 into the other LDS stage and retired by ONE counted vmcnt at the end of P4.
#include "gemm2_dev.h"
// DMA slots of K-tile t+2 issued in P4 of K-tile t (of G = 7-8 per wave) by the staggered 4-phase loop (bf16 NT / TT):
// 4 measured best (tools/gpu_tree_gemm_ab.sh, profiles/dma_depth_d0_ab_r5.log: vs 2, every headline GEMM 0.3-6.9 %
// faster and the step +1.9 %; 3, 5 and 6 slower than 4)
#ifndef G2_D0
#define G2_D0 4
#endif
// the same for the fp8 persistent NT / TT kernels (gemm8pk, gemm8tt)
#ifndef G8_D0
#define G8_D0 4
#endif
#include <stdlib.h>

#include <cmath>

namespace hsd {

namespace g2 {

// Staggered 4-phase main loop (SYNC 4 / 5 / 7) over nt K-tiles from kbeg, shared by gemm2_kernel and the persistent
// gemm2pk_kernel. PRO: issue the prologue (tile 0 whole + D0 slots of tile 1 -> stage 0 / 1, retire tile 0, first
// barrier) here; without it the caller has done exactly that (the persistent kernel, under the previous tile's
// epilogue). Enters with every wave at the same barrier count; leaves the same way.
template <int LA, int LB, int BN, int SYNC, int G, int D0, bool PRO, class DMA>
__device__ __forceinline__ void mainloop_staggered(f32x4 (&acc)[8][BN / 64], bf16_t* smem, const DMA& dma_slot,
                                                   int nt, int kbeg, int wm, int arow, int bcol, int lane) {
  constexpr int WN = BN / 4, NREP = WN / 16, NB0 = 2, NB1 = NREP - NB0;
  constexpr int TA = BM * 64, STAGE = TA + BN * 64;
  bf16x8 fa[4][2], fb0[NB0][2], fb1[NB1][2];
  // Staggered 4-phase schedule (cdna_hip_programming.md §5 "256² 8-phase template"; MI355X_MICROARCH.md
  // "Two waves per SIMD" item 9): the wave groups wm = 0 / 1 — one wave of each on every SIMD — run ONE
  // barrier apart, so on every SIMD one wave's MFMA cluster overlaps the other wave's LDS reads and DMA
  // issue. Each phase is   reads (+ DMA issue) -> lgkmcnt(0) -> barrier -> MFMA cluster -> barrier.
  // * lgkmcnt(0) before the barrier: a group one barrier behind has COMPLETED (not just issued) the reads
  //   of the phase it is in, so the P4 DMA into the current stage (tile t+2) cannot overwrite live data.
  // * the counted vmcnt sits before P4's FIRST barrier (one barrier earlier than the unstaggered form), so
  //   the lagging group's DMAs of tile t+1 have landed before the leading group reads them in P1(t+1).
  // Tile t+1's DMA: SYNC 4 issues it in P1 / P2 (two MFMA phases to land), SYNC 5 spreads it over
  // P1 / P2 / P3 (2 pieces per phase, fewer issue stalls per phase); D0 slots of tile t+2 go out in P4.
#ifndef G2_STATIC_PRIO
#define G2_STATIC_PRIO 1
#endif
  constexpr bool kStaticPrio = G2_STATIC_PRIO;
  constexpr int E1 = SYNC != 5 ? D0 + (G - D0 + 1) / 2 : D0 + 2;
  constexpr int E2 = SYNC != 5 ? G : (D0 + 4 < G ? D0 + 4 : G);
#define G2_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
#define G2_CLUSTER(ACC_I0, FA, FB, NBX, J0)                                                                  \
  if constexpr (!kStaticPrio) __builtin_amdgcn_s_setprio(1);                                                 \
  _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) _Pragma("unroll") for (int i = 0; i < 4; ++i)               \
      _Pragma("unroll") for (int j = 0; j < NBX; ++j) acc[ACC_I0 + i][J0 + j] =                                \
          __builtin_amdgcn_mfma_f32_16x16x32_bf16(FB[j][ks], FA[i][ks], acc[ACC_I0 + i][J0 + j], 0, 0, 0);     \
  if constexpr (!kStaticPrio) __builtin_amdgcn_s_setprio(0);
  if constexpr (PRO) {
#pragma unroll
    for (int q = 0; q < G; ++q) dma_slot(q, smem, kbeg);
    if (nt > 1) {
#pragma unroll
      for (int q = 0; q < D0; ++q) dma_slot(q, smem + STAGE, kbeg + BK);
      vmcnt<D0>();
    } else {
      vmcnt<0>();
    }
    G2_BARRIER();
  }
  // static priority (MI355X_MICROARCH.md 'Two waves per SIMD' item 4): the second-dispatched half (waves 4-7, the
  // lagging group) at prio 1 for the whole loop instead of per-cluster flips. G2_STATIC_PRIO=0: per-cluster flips.
  if constexpr (kStaticPrio) {
    if (wm == 1) __builtin_amdgcn_s_setprio(1);
  }
  if (wm == 1) G2_BARRIER();
  for (int t = 0; t < nt; ++t) {
    const bf16_t* cA = smem + (t & 1) * STAGE;
    const bf16_t* cB = cA + TA;
    bf16_t* nS = smem + ((t + 1) & 1) * STAGE;
    const bool n1 = t + 1 < nt, n2 = t + 2 < nt;
    const int k1 = kbeg + (t + 1) * BK, k2 = kbeg + (t + 2) * BK;
    // P1: A-sub0 + B-sub0 reads, first part of tile t+1's DMA
#pragma unroll
    for (int j = 0; j < NB0; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fb0[j][ks] = frag<LB>(cB, bcol + 16 * j, ks, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fa[i][ks] = frag<LA>(cA, arow + 16 * i, ks, lane);
    if (n1) {
#pragma unroll
      for (int q = D0; q < E1; ++q) dma_slot(q, nS, k1);
    }
    G2_LGKM0();
    G2_BARRIER();
    G2_CLUSTER(0, fa, fb0, NB0, 0)
    G2_BARRIER();
    // P2: B-sub1 reads, more of tile t+1's DMA
#pragma unroll
    for (int j = 0; j < NB1; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fb1[j][ks] = frag<LB>(cB, bcol + 16 * (NB0 + j), ks, lane);
    if (n1) {
#pragma unroll
      for (int q = E1; q < E2; ++q) dma_slot(q, nS, k1);
    }
    G2_LGKM0();
    G2_BARRIER();
    G2_CLUSTER(0, fa, fb1, NB1, NB0)
    G2_BARRIER();
    // P3: A-sub1 reads (+ the rest of tile t+1's DMA, SYNC 5)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fa[i][ks] = frag<LA>(cA, arow + 64 + 16 * i, ks, lane);
    if (n1) {
#pragma unroll
      for (int q = E2; q < G; ++q) dma_slot(q, nS, k1);
    }
    G2_LGKM0();
    G2_BARRIER();
    G2_CLUSTER(4, fa, fb1, NB1, NB0)
    G2_BARRIER();
    // P4: no reads; D0 slots of tile t+2 into this stage; retire tile t+1
    if (n2) {
#pragma unroll
      for (int q = 0; q < D0; ++q) dma_slot(q, const_cast<bf16_t*>(cA), k2);
      vmcnt<D0>();
    } else {
      vmcnt<0>();
    }
    G2_BARRIER();
    G2_CLUSTER(4, fa, fb0, NB0, 0)
    G2_BARRIER();
  }
  if (wm == 0) G2_BARRIER();
  if constexpr (kStaticPrio) __builtin_amdgcn_s_setprio(0);
#undef G2_CLUSTER
#undef G2_LGKM0
}

template <int LA, int LB, int EPI, int BN, int SYNC, bool SEG = false>
__global__ __launch_bounds__(512, 1) void gemm2_kernel(G2Params p) {
  p.dp = resolve_seed(p.dp);
  constexpr int WN = BN / 4;       // wave tile columns
  constexpr int NREP = WN / 16;    // 16-col MFMA blocks per wave
  constexpr int NB0 = 2;           // B-sub0 blocks (cols 0..31 of the wave)
  constexpr int NB1 = NREP - NB0;  // B-sub1 blocks
  static_assert(NREP == 3 || NREP == 4, "BN 192 or 256");
  static_assert(LB == 0 || BN == 256, "k-strided B needs BN 256");
  constexpr int TA = BM * 64, TB = BN * 64, STAGE = TA + TB;
  constexpr int GA = 4;                              // DMA instructions per wave per stage for A
  constexpr int GB = (LB == 0) ? BN / 64 : 4;        // ... for B
  constexpr int G = GA + GB;                         // 8 (BN 256) or 7 (BN 192)
  // slots of tile t+2 issued in P4 of tile t (the rest in P1-P3 of t+1); SYNC 6 / 7 = SYNC 0 / 4 with the
  // WHOLE next-next tile issued in P4, so every DMA has a full K-tile of MFMAs to land
  constexpr int D0 = (SYNC == 6 || SYNC == 7) ? G : G2_D0;
  constexpr bool F32OUT = EPI == E2_F32_ATOMIC || EPI == E2_F32_SLAB;

  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  // 1-D grid over (split, tile), XCD-aware bijective remap: the blocks an XCD runs together get
  // consecutive (split-major) indices, i.e. the same K-range (token window for the TT wgrad) and
  // neighbouring tiles (shared A row panels / B column panels) -> L2 reuse inside the XCD.
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int split = v / p.ntiles, wg = v % p.ntiles;
  const int tm = wg / p.tiles_n, tn = wg % p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = split * p.kps;
  const int kend = min(p.K, kbeg + p.kps);
  const int nt = (kend - kbeg) / BK;
  HSD_DASSERT(v < nwg && m0 < p.M && n0 < p.N && kbeg < p.K && (kend - kbeg) % BK == 0);

  // any k-strided operand: every DMA of the kernel is inline asm (a builtin DMA beside the transposing reads draws
  // hipcc's vmcnt(0) drain, see dma_lds_asm); k-contiguous-only (NT) kernels keep the builtin
  constexpr bool ASM = LA == 1 || LB == 1;
  uint32_t aoff[ASM ? G : 1];
  if constexpr (ASM) {
#pragma unroll
    for (int q = 0; q < G; ++q)
      aoff[q] = q < GA ? lane_off<LA>(p.lda, m0, p.M, wave * GA + q, lane)
                       : lane_off<LB>(p.ldb, n0, p.N, wave * GB + (q - GA), lane);
  }
  // LDS byte address of smem (one generic -> LDS conversion; stage / slot offsets are plain integer adds)
  const uint32_t smem_lds = (uint32_t)(size_t)(__attribute__((address_space(3))) bf16_t*)smem;
  const SegSel<SEG> segsel(p);
  auto dma_slot = [&](int q, bf16_t* stage, int k0) {
    const bf16_t* Ap;
    const bf16_t* Bp;
    const int kk = segsel.map(k0, Ap, Bp);
    if constexpr (ASM) {
      const uint32_t st = smem_lds + (uint32_t)(stage - smem) * 2u;
      if (q < GA) dma_lds_asm(asm_base<LA>(Ap, p.lda, m0, kk), aoff[q], st + (wave * GA + q) * 1024u);
      else dma_lds_asm(asm_base<LB>(Bp, p.ldb, n0, kk), aoff[q], st + (TA + (wave * GB + (q - GA)) * 512) * 2u);
    } else {
      if (q < GA) dma<LA, BM>(stage, Ap, p.lda, m0, p.M, kk, wave * GA + q, lane);
      else dma<LB, BN>(stage + TA, Bp, p.ldb, n0, p.N, kk, wave * GB + (q - GA), lane);
    }
  };

  f32x4 acc[8][NREP];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NREP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int arow = wm * 128;
  const int bcol = wn * WN;
  bf16x8 fa[4][2], fb0[NB0][2], fb1[NB1][2];
  if constexpr (SYNC == 0 || SYNC == 6) {
    // prologue: tile 0 whole, first D0 slots of tile 1
  #pragma unroll
    for (int q = 0; q < G; ++q) dma_slot(q, smem, kbeg);
    if (nt > 1) {
  #pragma unroll
      for (int q = 0; q < D0; ++q) dma_slot(q, smem + STAGE, kbeg + BK);
      vmcnt<D0>();
    } else {
      vmcnt<0>();
    }
    G2_BARRIER();


    for (int t = 0; t < nt; ++t) {
      const bf16_t* cA = smem + (t & 1) * STAGE;
      const bf16_t* cB = cA + TA;
      bf16_t* nS = smem + ((t + 1) & 1) * STAGE;
      const bool n1 = t + 1 < nt, n2 = t + 2 < nt;
      const int k1 = kbeg + (t + 1) * BK, k2 = kbeg + (t + 2) * BK;

      // ---------------- P1: A-sub0, B-sub0
  #pragma unroll
      for (int j = 0; j < NB0; ++j)
  #pragma unroll
        for (int ks = 0; ks < 2; ++ks) fb0[j][ks] = frag<LB>(cB, bcol + 16 * j, ks, lane);
  #pragma unroll
      for (int i = 0; i < 4; ++i)
  #pragma unroll
        for (int ks = 0; ks < 2; ++ks) fa[i][ks] = frag<LA>(cA, arow + 16 * i, ks, lane);
      if (n1) {
  #pragma unroll
        for (int q = D0; q < (D0 + 2 < G ? D0 + 2 : G); ++q) dma_slot(q, nS, k1);
      }
      G2_BARRIER();
      __builtin_amdgcn_s_setprio(1);
  #pragma unroll
      for (int ks = 0; ks < 2; ++ks)
  #pragma unroll
        for (int i = 0; i < 4; ++i)
  #pragma unroll
          for (int j = 0; j < NB0; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[j][ks], fa[i][ks], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      G2_BARRIER();

      // ---------------- P2: B-sub1
  #pragma unroll
      for (int j = 0; j < NB1; ++j)
  #pragma unroll
        for (int ks = 0; ks < 2; ++ks) fb1[j][ks] = frag<LB>(cB, bcol + 16 * (NB0 + j), ks, lane);
      if (n1) {
  #pragma unroll
        for (int q = D0 + 2; q < (D0 + 4 < G ? D0 + 4 : G); ++q) dma_slot(q, nS, k1);
      }
      G2_BARRIER();
      __builtin_amdgcn_s_setprio(1);
  #pragma unroll
      for (int ks = 0; ks < 2; ++ks)
  #pragma unroll
        for (int i = 0; i < 4; ++i)
  #pragma unroll
          for (int j = 0; j < NB1; ++j)
            acc[i][NB0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[j][ks], fa[i][ks], acc[i][NB0 + j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      G2_BARRIER();

      // ---------------- P3: A-sub1
  #pragma unroll
      for (int i = 0; i < 4; ++i)
  #pragma unroll
        for (int ks = 0; ks < 2; ++ks) fa[i][ks] = frag<LA>(cA, arow + 64 + 16 * i, ks, lane);
      if (n1) {
  #pragma unroll
        for (int q = D0 + 4; q < G; ++q) dma_slot(q, nS, k1);
      }
      G2_BARRIER();
      __builtin_amdgcn_s_setprio(1);
  #pragma unroll
      for (int ks = 0; ks < 2; ++ks)
  #pragma unroll
        for (int i = 0; i < 4; ++i)
  #pragma unroll
          for (int j = 0; j < NB1; ++j)
            acc[4 + i][NB0 + j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[j][ks], fa[i][ks], acc[4 + i][NB0 + j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      G2_BARRIER();

      // ---------------- P4: registers only; first D0 slots of tile t+2 into this (now free) stage
      if (n2) {
  #pragma unroll
        for (int q = 0; q < D0; ++q) dma_slot(q, const_cast<bf16_t*>(cA), k2);
      }
      __builtin_amdgcn_s_setprio(1);
  #pragma unroll
      for (int ks = 0; ks < 2; ++ks)
  #pragma unroll
        for (int i = 0; i < 4; ++i)
  #pragma unroll
          for (int j = 0; j < NB0; ++j)
            acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[j][ks], fa[i][ks], acc[4 + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if (n2) vmcnt<D0>();
      else vmcnt<0>();
      G2_BARRIER();
    }
  } else if constexpr (SYNC == 2) {
    // Software-pipelined LDS reads, one barrier per K-tile placed MID-tile: after the last reads of
    // stage t (A-sub1) every wave meets, tile t+1 (DMA'd a full tile earlier) becomes visible, tile
    // t+2's DMA goes into stage t, and A-sub0 of tile t+1 is read underneath the A-sub1 MFMAs.
    // Separate registers for A-sub0 / A-sub1 let each read overlap the previous group's MFMAs.
    bf16x8 fa1[4][2];
#define G2_SB() __builtin_amdgcn_sched_barrier(0)
#define G2_MMA(ACC_I0, FA, FB, NBX, J0)                                                                      \
  _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) _Pragma("unroll") for (int i = 0; i < 4; ++i)               \
      _Pragma("unroll") for (int j = 0; j < NBX; ++j) acc[ACC_I0 + i][J0 + j] =                                \
          __builtin_amdgcn_mfma_f32_16x16x32_bf16(FB[j][ks], FA[i][ks], acc[ACC_I0 + i][J0 + j], 0, 0, 0);
#pragma unroll
    for (int q = 0; q < G; ++q) dma_slot(q, smem, kbeg);
    if (nt > 1) {
#pragma unroll
      for (int q = 0; q < G; ++q) dma_slot(q, smem + STAGE, kbeg + BK);
      vmcnt<G>();
    } else {
      vmcnt<0>();
    }
    G2_BARRIER();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fa[i][ks] = frag<LA>(smem, arow + 16 * i, ks, lane);
    for (int t = 0; t < nt; ++t) {
      const bf16_t* cA = smem + (t & 1) * STAGE;
      const bf16_t* cB = cA + TA;
      const bf16_t* nA = smem + ((t + 1) & 1) * STAGE;
#pragma unroll
      for (int j = 0; j < NB0; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fb0[j][ks] = frag<LB>(cB, bcol + 16 * j, ks, lane);
      G2_SB();
#pragma unroll
      for (int j = 0; j < NB1; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fb1[j][ks] = frag<LB>(cB, bcol + 16 * (NB0 + j), ks, lane);
      G2_SB();
      G2_MMA(0, fa, fb0, NB0, 0)
      G2_SB();
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fa1[i][ks] = frag<LA>(cA, arow + 64 + 16 * i, ks, lane);
      G2_SB();
      G2_MMA(0, fa, fb1, NB1, NB0)
      G2_SB();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      vmcnt<0>();
      G2_BARRIER();
      if (t + 2 < nt) {
#pragma unroll
        for (int q = 0; q < G; ++q) dma_slot(q, const_cast<bf16_t*>(cA), kbeg + (t + 2) * BK);
      }
      if (t + 1 < nt) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) fa[i][ks] = frag<LA>(nA, arow + 16 * i, ks, lane);
      }
      G2_SB();
      G2_MMA(4, fa1, fb1, NB1, NB0)
      G2_MMA(4, fa1, fb0, NB0, 0)
      G2_SB();
    }
    vmcnt<0>();
    G2_BARRIER();
#undef G2_MMA
#undef G2_SB
  } else if constexpr (SYNC == 4 || SYNC == 5 || SYNC == 7) {
    mainloop_staggered<LA, LB, BN, SYNC, G, D0, true>(acc, smem, dma_slot, nt, kbeg, wm, arow, bcol, lane);
  } else {
    // ONE barrier per K-tile: tile t+1's DMA (into the other stage, free since the previous barrier) is
    // issued in two halves at the start of P1 / P2 and retired by vmcnt(0) before the end-of-tile
    // barrier; the four phases run without barriers so the two waves of a SIMD drift and overlap
    // each other's LDS reads with MFMAs.
#pragma unroll
    for (int q = 0; q < G; ++q) dma_slot(q, smem, kbeg);
    vmcnt<0>();
    G2_BARRIER();
    for (int t = 0; t < nt; ++t) {
      const bf16_t* cA = smem + (t & 1) * STAGE;
      const bf16_t* cB = cA + TA;
      bf16_t* nS = smem + ((t + 1) & 1) * STAGE;
      const bool n1 = t + 1 < nt;
      const int k1 = kbeg + (t + 1) * BK;
      if (n1) {
#pragma unroll
        for (int q = 0; q < G / 2; ++q) dma_slot(q, nS, k1);
      }
#pragma unroll
      for (int j = 0; j < NB0; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fb0[j][ks] = frag<LB>(cB, bcol + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fa[i][ks] = frag<LA>(cA, arow + 16 * i, ks, lane);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NB0; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[j][ks], fa[i][ks], acc[i][j], 0, 0, 0);
      if (n1) {
#pragma unroll
        for (int q = G / 2; q < G; ++q) dma_slot(q, nS, k1);
      }
#pragma unroll
      for (int j = 0; j < NB1; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fb1[j][ks] = frag<LB>(cB, bcol + 16 * (NB0 + j), ks, lane);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NB1; ++j)
            acc[i][NB0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[j][ks], fa[i][ks], acc[i][NB0 + j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fa[i][ks] = frag<LA>(cA, arow + 64 + 16 * i, ks, lane);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int j = 0; j < NB1; ++j)
            acc[4 + i][NB0 + j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[j][ks], fa[i][ks], acc[4 + i][NB0 + j], 0, 0, 0);
#pragma unroll
          for (int j = 0; j < NB0; ++j)
            acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[j][ks], fa[i][ks], acc[4 + i][j], 0, 0, 0);
        }
      vmcnt<0>();
      G2_BARRIER();
    }
  }

  // ================================================================ epilogue
  // acc[i][j] = D[n][m] block: lane l holds m = 16i + (l&15), n = 16j + 4(l>>4) + r (r = 0..3)
  const int mw = m0 + arow, nw = n0 + bcol;
  const int q4 = lane >> 4, lr = lane & 15;
  if constexpr (F32OUT) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mw + 16 * i + lr;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < NREP; ++j) {
        const int n = nw + 16 * j + 4 * q4;
        if (n >= p.N) continue;
        if constexpr (EPI == E2_F32_ATOMIC) {
          float* c = reinterpret_cast<float*>(p.C) + (int64_t)m * p.ldc + n;
          atomicAdd(c + 0, acc[i][j][0]);
          atomicAdd(c + 1, acc[i][j][1]);
          atomicAdd(c + 2, acc[i][j][2]);
          atomicAdd(c + 3, acc[i][j][3]);
        } else if (p.accum_direct) {
          f32x4* c = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.C) + (int64_t)m * p.ldc + n);
          *c = *c + acc[i][j];
        } else {
          float* c = reinterpret_cast<float*>(p.C) + (int64_t)split * p.M * p.N + (int64_t)m * p.N + n;
          *reinterpret_cast<f32x4*>(c) = acc[i][j];
        }
      }
    }
  } else {
    epilogue_bf16<EPI, BN>(acc, p, smem, wave, lane, mw, nw);
  }
}

// Persistent NT GEMM (k-contiguous A and B, bf16 epilogues, no split-K): grid = min(tiles, CUs), one workgroup per
// CU walking tiles v = bid, bid + grid, ... through the same XCD-aware remap as gemm2_kernel (grid is a multiple of
// 8, so tile L and workgroup bid share an XCD). Main loop = gemm2_kernel's SYNC 4 schedule, unchanged. What changes
// is the seam between tiles: a one-shot kernel pays, per tile, the new workgroup's prologue (address setup + the
// first K-tile's DMA round trip, ~1-2 us at HBM latency under load) AFTER the previous workgroup's stores drained.
// Here the next tile's prologue DMA (K-tile 0 into stage 0, D0 slots of K-tile 1 into stage 1) is issued right after
// the main loop, BEFORE the epilogue, and lands while the epilogue stages and stores the finished tile through its
// own 32 KiB LDS area (32-row passes; 2 x 64 KiB operand stages + 32 KiB = the whole 160 KiB).
// Ordering rules (gfx9-family vector-memory counter: loads AND stores retire in issue order -- hipcc itself emits
// counted vmcnt waits with stores outstanding):
// * the epilogue's bias and first-pass residual loads are issued BEFORE the DMA, so waiting on them never waits on
//   the DMA; later passes' residual loads do -- by then the DMA has had a pass to land;
// * the DMA is inline asm (invisible to hipcc), so hipcc's wait for an epilogue LDS store cannot turn into a drain;
// * after the epilogue, vmcnt<D0 + stores issued since> + barrier retires the next tile's K-tile 0 for every wave
//   while the epilogue's stores are still in flight (they drain under the next tile's first K-tile).
template <int EPI, int BN>
__global__ __launch_bounds__(512, 1) void gemm2pk_kernel(G2Params p) {
  p.dp = resolve_seed(p.dp);
  static_assert(epi_bf16_out(EPI), "bf16 epilogues");
  constexpr int WN = BN / 4, NREP = WN / 16;
  constexpr int TA = BM * 64, STAGE = TA + BN * 64;
  constexpr int GA = 4, GB = BN / 64, G = GA + GB, D0 = G2_D0;
  constexpr int PB = 2;                                  // 32-row epilogue passes
  constexpr int STG = 8 * 16 * PB * epi_srow<BN>();      // epilogue staging, elements
  constexpr int ITER = epi_iter<BN, PB>();
  constexpr int NST = (8 / PB) * ITER * (epi_two_out(EPI) ? 2 : 1);  // epilogue stores per wave, all rows inside M
  static_assert(D0 + NST <= 63, "vmcnt field");
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * STAGE + STG];
  static_assert(sizeof(smem) <= 160 * 1024, "LDS");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int ntiles = p.ntiles, q8 = ntiles >> 3, r8 = ntiles & 7;
  const int nt = p.K / BK;
  HSD_DASSERT(p.K % BK == 0 && nt >= 1 && (gridDim.x == (unsigned)ntiles || gridDim.x % 8 == 0));
  auto tile_of = [&](int L, int& m0, int& n0) {
    const int xcd = L & 7;
    const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (L >> 3);
    m0 = (v / p.tiles_n) * BM;
    n0 = (v % p.tiles_n) * BN;
  };
  const uint32_t smem_lds = (uint32_t)(size_t)(__attribute__((address_space(3))) bf16_t*)smem;
  uint32_t aoff[G];
  int m0, n0;
  auto set_tile = [&](int L) {
    tile_of(L, m0, n0);
#pragma unroll
    for (int q = 0; q < G; ++q)
      aoff[q] = q < GA ? lane_off<0>(p.lda, m0, p.M, wave * GA + q, lane)
                       : lane_off<0>(p.ldb, n0, p.N, wave * GB + (q - GA), lane);
  };
  auto dma_slot = [&](int q, bf16_t* stage, int k0) {
    const uint32_t st = smem_lds + (uint32_t)(stage - smem) * 2u;
    if (q < GA) dma_lds_asm(asm_base<0>(p.A, p.lda, m0, k0), aoff[q], st + (wave * GA + q) * 1024u);
    else dma_lds_asm(asm_base<0>(p.B, p.ldb, n0, k0), aoff[q], st + (TA + (wave * GB + (q - GA)) * 512) * 2u);
  };
  auto prologue = [&]() {
#pragma unroll
    for (int q = 0; q < G; ++q) dma_slot(q, smem, 0);
    if (nt > 1) {
#pragma unroll
      for (int q = 0; q < D0; ++q) dma_slot(q, smem + STAGE, BK);
    }
  };

  const int arow = wm * 128, bcol = wn * WN;
  // tile walk: static (L = blockIdx.x, +gridDim.x, ...) or claimed from the launch's tile queue (p.tq; gemm_common.h
  // tq_*). The claimed index reaches every wave through one LDS word in stage 1 at byte 2048 (A slot 2 of wave 0):
  // no DMA is in flight when it is written (before the first prologue / after the last K-tile's vmcnt<0>), and the
  // next DMA into those bytes is issued in P1 of the next main loop, after the seam barrier every wave passes after
  // reading it.
  int* const tq = p.tq;
  const int xg = tq != nullptr ? tq_xcc() : 0;
  uint32_t dead = 0;  // wave 0 lane 0: XCD groups seen exhausted
  int* const bcast = reinterpret_cast<int*>(smem + STAGE + 1024);
  int L = blockIdx.x;
  if (tq != nullptr) {
    if (wave == 0 && lane == 0) *bcast = tq_claim(tq, xg, dead, ntiles);
    __syncthreads();
    L = __builtin_amdgcn_readfirstlane(*bcast);  // wave-uniform: tile addresses stay scalar
    if (L >= ntiles) {
      if (wave == 0 && lane == 0) tq_exit(tq);
      return;
    }
  }
  set_tile(L);
  prologue();
  vmcnt<0>();
  G2_BARRIER();
  f32x4 acc[8][NREP];
  for (int it = 0;; ++it) {
    // claim the NEXT tile now (wave 0 lane 0, own XCD group): the atomic returns under this tile's main loop
    int pre = 0;
    if (tq != nullptr && wave == 0 && lane == 0 && !(dead & (1u << xg))) pre = tq_fetch(tq, xg);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NREP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    mainloop_staggered<0, 0, BN, 4, G, D0, false>(acc, smem, dma_slot, nt, 0, wm, arow, bcol, lane);
    uint64_t ts0 = 0, ts1 = 0;
    if (p.diag) ts0 = __builtin_amdgcn_s_memtime();
    if (tq != nullptr) {
      if (wave == 0 && lane == 0) {
        int Ln = dead & (1u << xg) ? ntiles : xg + 8 * pre;
        if (Ln >= ntiles) {
          dead |= 1u << xg;
          Ln = tq_claim(tq, xg, dead, ntiles);
        }
        *bcast = Ln;
      }
      __syncthreads();  // nothing in flight here: the main loop ended with vmcnt<0>
      L = __builtin_amdgcn_readfirstlane(*bcast);  // wave-uniform: tile addresses stay scalar
    } else {
      L += gridDim.x;
    }
    const int mw = m0 + arow, nw = n0 + bcol;
    f32x4 bv[NREP];
    u32x4 xv0[ITER];
    epi_bias_regs<EPI, BN>(bv, p, lane, nw);
    epi_aux_regs<EPI, BN, PB>(xv0, p, lane, mw, nw, 0);
    const bool more = L < ntiles;
    if (more) {
      set_tile(L);
      prologue();
    }
    epilogue_bf16<EPI, BN, 8, PB, true>(acc, p, smem + 2 * STAGE, wave, lane, mw, nw, bv, xv0);
    if (p.diag) ts1 = __builtin_amdgcn_s_memtime();
    // diagnostic stamps (wave 0): main loop end, epilogue end, seam end, real time -- tools/seam_probe.py
    auto stamp = [&](uint64_t ts2) {
      if (p.diag && wave == 0 && lane == 0) {
        unsigned long long* d = p.diag + ((int64_t)blockIdx.x * 64 + min(it, 63)) * 4;
        d[0] = ts0; d[1] = ts1; d[2] = ts2; d[3] = __builtin_amdgcn_s_memrealtime();
      }
    };
    if (!more) {
      stamp(ts1);
      if (tq != nullptr && wave == 0 && lane == 0) tq_exit(tq);
      break;
    }
    // retire the next tile's K-tile 0 (the oldest G DMAs of this wave) without draining the epilogue's stores:
    // a wave whose 128 rows are all inside M issued at least NST stores after the DMAs (more with the column-sum
    // atomics); a wave on the M edge counts none
    if (mw + 128 <= p.M) {
      if (nt > 1) vmcnt<D0 + NST>();
      else vmcnt<NST>();
    } else {
      if (nt > 1) vmcnt<D0>();
      else vmcnt<0>();
    }
    G2_BARRIER();
    if (p.diag) stamp(__builtin_amdgcn_s_memtime());
  }
}

// ------------------------------------------------------------------------------------------------
// fp8 persistent NT GEMM (gemm8pk): gemm2pk with v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales, twice the bf16
// MFMA rate). A K-tile of 128 fp8 values is the same 128-B row as 64 bf16 values, so an fp8 [M][K] operand is handled
// as a "bf16" [M][K/2] one: same LDS images, DMA slots (inline asm), staggered 4-phase schedule, tile walk, seam and
// epilogues. Per K-tile a wave issues 32 MFMAs of 32 cycles (bf16: 64 of 16) and reads 24 x 16 B per lane (same).
typedef __attribute__((ext_vector_type(8))) int i32x8;

// 16x16x128 fragment: lane l holds row rbase + (l&15) and the 16-B chunks (l>>4) and (l>>4)+4 of the 128-B K-tile
// row as its instruction k slots 32(l>>4) .. +31. A and B use the same chunk -> slot assignment, so the product is the
// same sum. Chunks (g, g+4) rather than the contiguous (2g, 2g+1): with the f1 swizzle the contiguous pair put two
// lanes of every ds_read_b128 lane group on the same banks (2-way, 43-48 % SQ_LDS_BANK_CONFLICT per
// profiles/r6/pmc_gemm8_r6.tsv); (g, g+4) is conflict-free in the gfx950 lane-group model (tools/lds_banks.py)
__device__ __forceinline__ i32x8 frag8(const bf16_t* img, int rbase, int lane) {
  const int row = rbase + (lane & 15);
  const int c0 = lane >> 4;
  const bf16_t* r = img + row * 64;
  const u32x4 lo = *reinterpret_cast<const u32x4*>(r + ((c0 ^ f1(row)) << 3));
  const u32x4 hi = *reinterpret_cast<const u32x4*>(r + (((c0 + 4) ^ f1(row)) << 3));
  i32x8 v;
  v[0] = (int)lo[0]; v[1] = (int)lo[1]; v[2] = (int)lo[2]; v[3] = (int)lo[3];
  v[4] = (int)hi[0]; v[5] = (int)hi[1]; v[6] = (int)hi[2]; v[7] = (int)hi[3];
  return v;
}

// fp8 k-strided operand image (the TT weight gradient reads dY8 [T][M] and X8 [T][N] as written, tokens = k):
// [128 tokens][256 B] per operand per stage (the same 32 KiB as a k-contiguous image), 16-B chunk c of token row k
// stored at chunk c ^ s8t(k). A 16x16x128 fragment is four transposing reads (ds_read_b64_tr_b8): in 16-lane group g,
// lane i addresses token row 32g + 8r + (i>>1), bytes 8(i&1) .. +7 of the fragment's 16 columns, and receives column
// i's 8 tokens, so lane l holds column rbase + (l&15), tokens 32(l>>4) .. +31 (in some fixed order that is the same
// for A and B: the product does not depend on it). s8t: the 16 rows a half-wave reads (groups g, g+1: rows k0..k0+7
// and k0+32..k0+39) land in 16 distinct chunks = all 64 banks; s8t(k + 8r) = s8t(k) for the four reads of a lane.
__device__ __forceinline__ int s8t(int k) { return (k & 7) | (((k >> 5) & 1) << 3); }

typedef __attribute__((ext_vector_type(2))) int i32x2;
typedef __attribute__((address_space(3))) i32x2 lds_i32x2_t;

__device__ __forceinline__ i32x8 frag8t(const bf16_t* img, int rbase, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int k = 32 * g + (i >> 1);
  const char* a = reinterpret_cast<const char*>(img) + k * 256 + ((((rbase >> 4) ^ s8t(k))) << 4) + 8 * (i & 1);
  i32x8 v;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const i32x2 t = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_i32x2_t*)(a + r * 8 * 256));
    v[2 * r] = t[0];
    v[2 * r + 1] = t[1];
  }
  return v;
}

// per-lane byte offset of DMA slot gs (0..31) of an fp8 k-strided image: token rows 4gs .. 4gs+3, the lane's LDS
// chunk (lane & 15) holds logical chunk (lane & 15) ^ s8t(row)
__device__ __forceinline__ uint32_t lane_off8t(int64_t ld, int gs, int lane) {
  const int row = 4 * gs + (lane >> 4);
  return (uint32_t)((int64_t)row * ld + 16 * ((lane & 15) ^ s8t(row)));
}

template <int LT>
__device__ __forceinline__ i32x8 frag8x(const bf16_t* img, int rbase, int lane) {
  if constexpr (LT == 0) return frag8(img, rbase, lane);
  else return frag8t(img, rbase, lane);
}

// FB / FA: formats of the B / A operands (0 = e4m3, 1 = e5m2); B is the instruction's first operand (D[n][m])
template <int FB, int FA>
__device__ __forceinline__ f32x4 mma8(const i32x8& b, const i32x8& a, const f32x4& c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b, a, c, FB, FA, 0, 0, 0, 0);
}

// mainloop_staggered (SYNC 4, prologue issued by the caller) with fp8 fragments: one MFMA per (i, j) per K-tile.
// LT 0: k-contiguous images (NT), 1: k-strided images (TT, frag8t)
template <int BN, int G, int D0, int FA, int FB, int LT = 0, class DMA>
__device__ __forceinline__ void mainloop_staggered8(f32x4 (&acc)[8][BN / 64], bf16_t* smem, const DMA& dma_slot,
                                                    int nt, int wm, int arow, int bcol, int lane) {
  constexpr int WN = BN / 4, NREP = WN / 16, NB0 = 2, NB1 = NREP - NB0;
  constexpr int TA = BM * 64, STAGE = TA + BN * 64;
  constexpr int E1 = D0 + (G - D0 + 1) / 2;
  i32x8 fa[4], fb0[NB0], fb1[NB1];
#define G8_CLUSTER(ACC_I0, FB_, NBX, J0)                                                                     \
  if constexpr (!G2_STATIC_PRIO) __builtin_amdgcn_s_setprio(1);                                             \
  _Pragma("unroll") for (int i = 0; i < 4; ++i) _Pragma("unroll") for (int j = 0; j < NBX; ++j)              \
      acc[ACC_I0 + i][J0 + j] = mma8<FB, FA>(FB_[j], fa[i], acc[ACC_I0 + i][J0 + j]);                        \
  if constexpr (!G2_STATIC_PRIO) __builtin_amdgcn_s_setprio(0);
  if constexpr (G2_STATIC_PRIO) {  // static priority of the lagging group, as in mainloop_staggered
    if (wm == 1) __builtin_amdgcn_s_setprio(1);
  }
  if (wm == 1) G2_BARRIER();
  for (int t = 0; t < nt; ++t) {
    const bf16_t* cA = smem + (t & 1) * STAGE;
    const bf16_t* cB = cA + TA;
    bf16_t* nS = smem + ((t + 1) & 1) * STAGE;
    const bool n1 = t + 1 < nt, n2 = t + 2 < nt;
    const int k1 = (t + 1) * BK, k2 = (t + 2) * BK;
    // P1: A-sub0 + B-sub0, first part of tile t+1's DMA
#pragma unroll
    for (int j = 0; j < NB0; ++j) fb0[j] = frag8x<LT>(cB, bcol + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag8x<LT>(cA, arow + 16 * i, lane);
    if (n1) {
#pragma unroll
      for (int q = D0; q < E1; ++q) dma_slot(q, nS, k1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G2_BARRIER();
    G8_CLUSTER(0, fb0, NB0, 0)
    G2_BARRIER();
    // P2: B-sub1, rest of tile t+1's DMA
#pragma unroll
    for (int j = 0; j < NB1; ++j) fb1[j] = frag8x<LT>(cB, bcol + 16 * (NB0 + j), lane);
    if (n1) {
#pragma unroll
      for (int q = E1; q < G; ++q) dma_slot(q, nS, k1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G2_BARRIER();
    G8_CLUSTER(0, fb1, NB1, NB0)
    G2_BARRIER();
    // P3: A-sub1
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag8x<LT>(cA, arow + 64 + 16 * i, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G2_BARRIER();
    G8_CLUSTER(4, fb1, NB1, NB0)
    G2_BARRIER();
    // P4: no reads; D0 slots of tile t+2 into this stage; retire tile t+1
    if (n2) {
#pragma unroll
      for (int q = 0; q < D0; ++q) dma_slot(q, const_cast<bf16_t*>(cA), k2);
      vmcnt<D0>();
    } else {
      vmcnt<0>();
    }
    G2_BARRIER();
    G8_CLUSTER(4, fb0, NB0, 0)
    G2_BARRIER();
  }
  if (wm == 0) G2_BARRIER();
  if constexpr (G2_STATIC_PRIO) __builtin_amdgcn_s_setprio(0);
#undef G8_CLUSTER
}

// p.A / p.B: fp8 [M][K] / [N][K] viewed as bf16 [..][K/2] (p.K, p.lda, p.ldb in bf16 units); sa / sb: device
// dequantisation scalars
// Q8: the epilogue also writes the output's fp8 copy (the next fp8 GEMM's operand). Its stores and amax atomics come
// after the next tile's DMA like the bf16 stores; the seam's counted wait still uses NST (bf16 stores only), which is
// conservative: fewer outstanding operations allowed than were issued after the DMA.
template <int EPI, int BN, int FA, int FB, bool Q8 = false>
__global__ __launch_bounds__(512, 1) void gemm8pk_kernel(G2Params p, const float* __restrict__ sa,
                                                         const float* __restrict__ sb) {
  p.dp = resolve_seed(p.dp);
  static_assert(epi_bf16_out(EPI), "bf16 epilogues");
  constexpr int WN = BN / 4, NREP = WN / 16;
  constexpr int TA = BM * 64, STAGE = TA + BN * 64;
  constexpr int GA = 4, GB = BN / 64, G = GA + GB, D0 = G8_D0;
  constexpr int PB = 2;
  constexpr int STG = 8 * 16 * PB * epi_srow<BN>();
  constexpr int ITER = epi_iter<BN, PB>();
  constexpr int NST = (8 / PB) * ITER * (epi_two_out(EPI) ? 2 : 1);
  static_assert(D0 + NST <= 63, "vmcnt field");
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * STAGE + STG];
  static_assert(sizeof(smem) <= 160 * 1024, "LDS");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int ntiles = p.ntiles, q8 = ntiles >> 3, r8 = ntiles & 7;
  const int nt = p.K / BK;
  const float dq = sa[0] * sb[0];
  HSD_DASSERT(p.K % BK == 0 && nt >= 1 && (gridDim.x == (unsigned)ntiles || gridDim.x % 8 == 0));
  const uint32_t smem_lds = (uint32_t)(size_t)(__attribute__((address_space(3))) bf16_t*)smem;
  uint32_t aoff[G];
  int m0, n0;
  auto set_tile = [&](int L) {
    const int xcd = L & 7;
    const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (L >> 3);
    m0 = (v / p.tiles_n) * BM;
    n0 = (v % p.tiles_n) * BN;
#pragma unroll
    for (int q = 0; q < G; ++q)
      aoff[q] = q < GA ? lane_off<0>(p.lda, m0, p.M, wave * GA + q, lane)
                       : lane_off<0>(p.ldb, n0, p.N, wave * GB + (q - GA), lane);
  };
  auto dma_slot = [&](int q, bf16_t* stage, int k0) {
    const uint32_t st = smem_lds + (uint32_t)(stage - smem) * 2u;
    if (q < GA) dma_lds_asm(asm_base<0>(p.A, p.lda, m0, k0), aoff[q], st + (wave * GA + q) * 1024u);
    else dma_lds_asm(asm_base<0>(p.B, p.ldb, n0, k0), aoff[q], st + (TA + (wave * GB + (q - GA)) * 512) * 2u);
  };
  auto prologue = [&]() {
#pragma unroll
    for (int q = 0; q < G; ++q) dma_slot(q, smem, 0);
    if (nt > 1) {
#pragma unroll
      for (int q = 0; q < D0; ++q) dma_slot(q, smem + STAGE, BK);
    }
  };

  const int arow = wm * 128, bcol = wn * WN;
  // tile walk: static or claimed from p.tq, exactly as gemm2pk_kernel (broadcast word in stage 1 at byte 2048)
  int* const tq = p.tq;
  const int xg = tq != nullptr ? tq_xcc() : 0;
  uint32_t dead = 0;
  int* const bcast = reinterpret_cast<int*>(smem + STAGE + 1024);
  int L = blockIdx.x;
  if (tq != nullptr) {
    if (wave == 0 && lane == 0) *bcast = tq_claim(tq, xg, dead, ntiles);
    __syncthreads();
    L = __builtin_amdgcn_readfirstlane(*bcast);  // wave-uniform: tile addresses stay scalar
    if (L >= ntiles) {
      if (wave == 0 && lane == 0) tq_exit(tq);
      return;
    }
  }
  set_tile(L);
  prologue();
  vmcnt<0>();
  G2_BARRIER();
  f32x4 acc[8][NREP];
  for (;;) {
    int pre = 0;
    if (tq != nullptr && wave == 0 && lane == 0 && !(dead & (1u << xg))) pre = tq_fetch(tq, xg);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NREP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    mainloop_staggered8<BN, G, D0, FA, FB>(acc, smem, dma_slot, nt, wm, arow, bcol, lane);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NREP; ++j) acc[i][j] *= dq;
    if (tq != nullptr) {
      if (wave == 0 && lane == 0) {
        int Ln = dead & (1u << xg) ? ntiles : xg + 8 * pre;
        if (Ln >= ntiles) {
          dead |= 1u << xg;
          Ln = tq_claim(tq, xg, dead, ntiles);
        }
        *bcast = Ln;
      }
      __syncthreads();
      L = __builtin_amdgcn_readfirstlane(*bcast);  // wave-uniform: tile addresses stay scalar
    } else {
      L += gridDim.x;
    }
    const int mw = m0 + arow, nw = n0 + bcol;
    f32x4 bv[NREP];
    u32x4 xv0[ITER];
    epi_bias_regs<EPI, BN>(bv, p, lane, nw);
    epi_aux_regs<EPI, BN, PB>(xv0, p, lane, mw, nw, 0);
    const bool more = L < ntiles;
    if (more) {
      set_tile(L);
      prologue();
    }
    epilogue_bf16<EPI, BN, 8, PB, true, Q8>(acc, p, smem + 2 * STAGE, wave, lane, mw, nw, bv, xv0);
    if (!more) {
      if (tq != nullptr && wave == 0 && lane == 0) tq_exit(tq);
      break;
    }
    if (mw + 128 <= p.M) {
      if (nt > 1) vmcnt<D0 + NST>();
      else vmcnt<NST>();
    } else {
      if (nt > 1) vmcnt<D0>();
      else vmcnt<0>();
    }
    G2_BARRIER();
  }
}

// fp8 TT weight gradient (gemm8tt): dW[M][N] += sa·sb · Σ_t dY8[t][M] · X8[t][N], the fp8 copies the producers
// already write for the fp8 forward / dgrad GEMMs (no transposed copies: both operands are staged as written, tokens
// as the k rows of fp8 k-strided images, and transposed on the way out of LDS by ds_read_b64_tr_b8). One-shot grid over
// (K-split, tile) with gemm2_kernel's XCD-aware remap, 256 x 256 tiles of 8 waves, K-tiles of 128 tokens, the
// staggered 4-phase schedule of gemm8pk; fp32 partials [split][M][N] (dequantised) summed into dW by
// slab_reduce_kernel. M, N multiples of 256, token splits multiples of 128.
template <int FA, int FB>
__global__ __launch_bounds__(512, 1) void gemm8tt_kernel(G2Params p, const float* __restrict__ sa,
                                                         const float* __restrict__ sb) {
  constexpr int BN = 256, NREP = 4;
  constexpr int TA = BM * 64, STAGE = TA + BN * 64;
  constexpr int GA = 4, GB = 4, G = GA + GB, D0 = G8_D0;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int split = v / p.ntiles, wg = v % p.ntiles;
  const int m0 = (wg / p.tiles_n) * BM, n0 = (wg % p.tiles_n) * BN;
  const int kbeg = split * p.kps;  // tokens
  const int nt = (min(p.K, kbeg + p.kps) - kbeg) / 128;
  HSD_DASSERT(v < nwg && m0 + BM <= p.M && n0 + BN <= p.N && nt >= 1);
  const uint8_t* A8 = reinterpret_cast<const uint8_t*>(p.A) + (int64_t)kbeg * p.lda + m0;
  const uint8_t* B8 = reinterpret_cast<const uint8_t*>(p.B) + (int64_t)kbeg * p.ldb + n0;
  uint32_t aoff[G];
#pragma unroll
  for (int q = 0; q < G; ++q)
    aoff[q] = q < GA ? lane_off8t(p.lda, wave * GA + q, lane) : lane_off8t(p.ldb, wave * GB + (q - GA), lane);
  const uint32_t smem_lds = (uint32_t)(size_t)(__attribute__((address_space(3))) bf16_t*)smem;
  // k0: the main loop's K offset in bf16 units (BK = 64 per K-tile) = half the token offset
  auto dma_slot = [&](int q, bf16_t* stage, int k0) {
    const int64_t tok = 2 * (int64_t)k0;
    const uint32_t st = smem_lds + (uint32_t)(stage - smem) * 2u;
    if (q < GA)
      dma_lds_asm(reinterpret_cast<const bf16_t*>(A8 + tok * p.lda), aoff[q], st + (wave * GA + q) * 1024u);
    else
      dma_lds_asm(reinterpret_cast<const bf16_t*>(B8 + tok * p.ldb), aoff[q],
                  st + (TA + (wave * GB + (q - GA)) * 512) * 2u);
  };
#pragma unroll
  for (int q = 0; q < G; ++q) dma_slot(q, smem, 0);
  if (nt > 1) {
#pragma unroll
    for (int q = 0; q < D0; ++q) dma_slot(q, smem + STAGE, BK);
  }
  vmcnt<0>();
  G2_BARRIER();
  f32x4 acc[8][NREP];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NREP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int arow = wm * 128, bcol = wn * (BN / 4);
  mainloop_staggered8<BN, G, D0, FA, FB, 1>(acc, smem, dma_slot, nt, wm, arow, bcol, lane);
  // acc[i][j]: lane l holds m = 16i + (l&15), n = 16j + 4(l>>4) .. +3 of the wave tile
  const float dq = sa[0] * sb[0];
  float* ws = reinterpret_cast<float*>(p.C) + (int64_t)split * p.M * p.N;
  const int q4 = lane >> 4, lr = lane & 15;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + arow + 16 * i + lr;
#pragma unroll
    for (int j = 0; j < NREP; ++j) {
      const int n = n0 + bcol + 16 * j + 4 * q4;
      *reinterpret_cast<f32x4*>(ws + (int64_t)m * p.N + n) = acc[i][j] * dq;
    }
  }
}

// main_grad[i] += Σ_s ws[s][i]   (float4 lanes, grid-stride); assign: C = Σ_s ws[s] (the split-K fp32 NT output)
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ ws, float* __restrict__ C,
                                                          int64_t ldc, int M, int N, int splits, int assign) {
  const int64_t n4 = (int64_t)M * N / 4;
  const int64_t plane = (int64_t)M * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i * 4;
    f32x4 s = *reinterpret_cast<const f32x4*>(ws + e);
    for (int k = 1; k < splits; ++k) s += *reinterpret_cast<const f32x4*>(ws + k * plane + e);
    const int64_t m = e / N, n = e % N;
    f32x4* c = reinterpret_cast<f32x4*>(C + m * ldc + n);
    *c = assign ? s : *c + s;
  }
}

// Split-K NT (small tile counts, gemm2_nt_splits): the main loop wrote fp32 partials [splits][M][N]
// (E2_F32_SLAB); this pass sums them in split order and runs the SAME per-chunk epilogue math as the fused
// epilogue (epi_chunk on bf16(acc + bias)), so every epilogue kind, its dropout sites and the fused bias-gradient
// column sums behave exactly as in the one-pass kernel (up to the fp32 summation order of the K-splits).
// Block = 8 16-B column chunks (64 columns) x 32 row lanes; `rpb` rows per block.
template <int EPI>
__global__ __launch_bounds__(256) void splitk_epi_kernel(const float* __restrict__ ws, int splits, int rpb,
                                                         G2Params p) {
  p.dp = resolve_seed(p.dp);
  const int tid = threadIdx.x, lane = tid & 63;
  const int c8 = tid & 7, rl = tid >> 3;
  const int nb = blockIdx.x * 64;
  const int n = nb + c8 * 8;
  const int m0 = blockIdx.y * rpb;
  const int m1 = min(p.M, m0 + rpb);
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (n < p.N) {
    f32x4 b0 = {0.f, 0.f, 0.f, 0.f}, b1 = {0.f, 0.f, 0.f, 0.f};
    if constexpr (epi_bias(EPI)) {
      const u32x4 b = *reinterpret_cast<const u32x4*>(p.bias + n);
      b0 = f32x4{lo_bf(b.x), hi_bf(b.x), lo_bf(b.y), hi_bf(b.y)};
      b1 = f32x4{lo_bf(b.z), hi_bf(b.z), lo_bf(b.w), hi_bf(b.w)};
    }
    const int64_t plane = (int64_t)p.M * p.N;
    bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
    const uint32_t cw = epi_col_word<EPI>(n, p);
    for (int m = m0 + rl; m < m1; m += 32) {
      const float* w = ws + (int64_t)m * p.N + n;
      f32x4 a0 = *reinterpret_cast<const f32x4*>(w);
      f32x4 a1 = *reinterpret_cast<const f32x4*>(w + 4);
      for (int sp = 1; sp < splits; ++sp) {
        a0 += *reinterpret_cast<const f32x4*>(w + sp * plane);
        a1 += *reinterpret_cast<const f32x4*>(w + sp * plane + 4);
      }
      if constexpr (epi_bias(EPI)) {
        a0 += b0;
        a1 += b1;
      }
      const u32x2 lo = pack4(a0), hi = pack4(a1);
      u32x4 o = {lo.x, lo.y, hi.x, hi.y}, o2;
      u32x4 x = {0, 0, 0, 0};
      if constexpr (epi_aux(EPI)) x = *reinterpret_cast<const u32x4*>(p.aux + (int64_t)m * p.ldaux + n);
      epi_chunk<EPI>(o, o2, x, m, n, p, csum,
                     EPI == E2_BIAS_DROP_RES && p.dp.enabled ? drop_row((uint32_t)m, p.dp.key) ^ cw : 0u);
      if constexpr (EPI == E2_STORE_RDOT) rdot_group(o, x, m, n, p, c8 == 0, true);  // 8 lanes of one row, all in
      st16(C + (int64_t)m * p.ldc + n, o, p.nt_store);
      if constexpr (epi_two_out(EPI)) st16(p.C2 + (int64_t)m * p.ldc + n, o2, p.nt_store);
    }
  }
  if constexpr (EPI == E2_DGELU || EPI == E2_MUL) {
    if (p.dbias != nullptr) colsum_flush(csum, p.dbias, nb, p.N, lane);  // every lane: shuffles inside
  }
}

// ------------------------------------------------------------------------------------------------
// gemm2s: GEMM on 128 x 128 tiles for grids the 256 x 256 kernel cannot fill (small token counts: the
// reference's per-rank batch of 8 x 512 tokens, serving batches). 4 waves (2 x 2), 64 x 64 wave tiles of
// v_mfma_f32_16x16x32_bf16, BK 64, NSTG 32-KiB LDS stages, the same swizzled LDS images (k-contiguous rows for NT;
// 128-wide k-strided rows + transposing reads for the TT wgrad) and epilogues as gemm2. With one workgroup per CU
// (<= 256 tiles) each SIMD runs ONE wave, so HBM latency is hidden by depth, not by occupancy: tiles t+1 .. t+NSTG-2
// are in flight while tile t computes, retired by a counted vmcnt. The DMAs are inline asm issued right after the
// barrier that frees their stage, so hipcc does not drain them with vmcnt(0) before the current tile's LDS reads (a
// builtin DMA into a runtime-indexed stage makes hipcc assume aliasing).
// TT (fp32 out): one split accumulates into C (unique owner, C += acc); split-K writes [split][M][N] slabs for
// slab_reduce_kernel.
constexpr int SBM = 128, SBN = 128;

template <int L>
__device__ __forceinline__ void dma_asm(bf16_t* img, const bf16_t* __restrict__ X, int64_t ld, int r0, int Rmax,
                                        int k0, int g, int lane) {
  const bf16_t* src;
  if constexpr (L == 0) {
    const int row = g * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ f1(row);
    const int rr = min(r0 + row, Rmax - 1);
    src = X + (int64_t)rr * ld + k0 + lc * 8;
  } else {
    // [64 k][128] image: 4 k-rows of 256 B per wave instruction
    const int krow = g * 4 + (lane >> 4);
    const int lc = (lane & 15) ^ f2(krow);
    const int cc = min(r0 + lc * 8, Rmax - 8);
    src = X + (int64_t)(k0 + krow) * ld + cc;
  }
  const uint32_t lds = (uint32_t)__builtin_amdgcn_readfirstlane(
      (int)(uint32_t)(size_t)(__attribute__((address_space(3))) bf16_t*)(img + g * 512));
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds)
               : "memory");
}

// wait until at most `left` (wave-uniform) K-tiles of DMA (PER instructions per wave each) are still in flight
template <int NSTG, int PER>
__device__ __forceinline__ void wait_tiles(int left) {
  if constexpr (NSTG >= 4) {
    if (left >= 2) { vmcnt<2 * PER>(); return; }
  }
  if constexpr (NSTG >= 3) {
    if (left >= 1) { vmcnt<PER>(); return; }
  }
  vmcnt<0>();
}

// KW = 2: 8 waves, two per SIMD -- wave groups kg = 0 / 1 take the first / second 32 k of every K-tile for the same
// 2 x 2 arrangement of 64 x 64 wave tiles (a K-split inside the workgroup), so on each SIMD one wave's MFMAs run
// while the other's LDS reads are in flight; group 1 hands its partial tile to group 0 through LDS (64 KiB after
// the 32 KiB epilogue staging: NSTG 3 or 4) and group 0 runs the epilogue. KW = 1: 4 waves, one per SIMD.
template <int LA, int LB, int EPI, int NSTG, int KW = 1, bool SEG = false>
__global__ __launch_bounds__(256 * KW, (NSTG <= 2 && KW == 1) ? 2 : 1) void gemm2s_kernel(G2Params p) {
  static_assert(NSTG >= 2 && NSTG <= 4, "2-4 stages");
  static_assert(KW == 1 || (KW == 2 && NSTG >= 3), "the in-workgroup K-split needs the 3rd stage's LDS for its handoff");
  static_assert(LA == 0 ? (epi_bf16_out(EPI) || EPI == E2_F32_SLAB) : (LB == 1 && EPI == E2_F32_SLAB),
                "NT / NT with k-strided B: bf16 epilogues or split-K slabs; TT: fp32");
  p.dp = resolve_seed(p.dp);
  constexpr int TA = SBM * 64, STAGE = TA + SBN * 64;  // elements
  __shared__ __attribute__((aligned(16))) bf16_t smem[NSTG * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = KW == 2 ? wave >> 2 : 0;
  const int w4 = wave & 3;
  const int wm = w4 >> 1, wn = w4 & 1;
  // 1-D grid over (split, tile), XCD-aware bijective remap (as gemm2): the tiles one XCD runs are neighbours
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int split = v / p.ntiles, wg = v % p.ntiles;
  const int tm = wg / p.tiles_n, tn = wg % p.tiles_n;
  const int m0 = tm * SBM, n0 = tn * SBN;
  const int kbeg = split * p.kps;
  const int nt = (min(p.K, kbeg + p.kps) - kbeg) / BK;
  HSD_DASSERT(v < nwg && m0 < p.M && n0 < p.N && kbeg < p.K && p.kps % BK == 0 && p.K % BK == 0);

  // 16 DMA wave-instructions per operand image per stage, DW + DW per wave
  constexpr int DW = 4 / KW;
  const SegSel<SEG> segsel(p);
  auto dma_tile = [&](bf16_t* stage, int k0) {
    const bf16_t* Ap;
    const bf16_t* Bp;
    const int kk = segsel.map(k0, Ap, Bp);
#pragma unroll
    for (int q = 0; q < DW; ++q) dma_asm<LA>(stage, Ap, p.lda, m0, p.M, kk, wave * DW + q, lane);
#pragma unroll
    for (int q = 0; q < DW; ++q) dma_asm<LB>(stage + TA, Bp, p.ldb, n0, p.N, kk, wave * DW + q, lane);
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int arow = wm * 64, bcol = wn * 64;

#pragma unroll
  for (int s = 0; s < NSTG - 1; ++s)
    if (s < nt) dma_tile(smem + s * STAGE, kbeg + s * BK);
  int rs = 0, ws = NSTG - 1;
  for (int t = 0; t < nt; ++t) {
    const bf16_t* cA = smem + rs * STAGE;
    const bf16_t* cB = cA + TA;
    // tile t landed (this wave's part) and every wave's part visible; every wave finished reading tile t-1,
    // whose stage tile t+NSTG-1 now refills
    wait_tiles<NSTG, 2 * DW>(min(NSTG - 2, nt - 1 - t));
    G2_BARRIER();
    if (t + NSTG - 1 < nt) dma_tile(smem + ws * STAGE, kbeg + (t + NSTG - 1) * BK);
#pragma unroll
    for (int kk = 0; kk < 2 / KW; ++kk) {
      const int ks = KW == 1 ? kk : kg;
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag<LA, SBM>(cA, arow + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag<LB, SBN>(cB, bcol + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    rs = rs == NSTG - 1 ? 0 : rs + 1;
    ws = ws == NSTG - 1 ? 0 : ws + 1;
  }
  if constexpr (KW == 2) {
    // every wave done with the operand stages; group 1's partial tile -> LDS [32 KiB, 96 KiB) -> group 0
    G2_BARRIER();
    f32x4* red = reinterpret_cast<f32x4*>(smem + 16384) + w4 * (16 * 64);
    if (kg == 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[(i * 4 + j) * 64 + lane] = acc[i][j];
    }
    G2_BARRIER();
    if (kg == 1) return;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] += red[(i * 4 + j) * 64 + lane];
  }
  const int mw = m0 + arow, nw = n0 + bcol;
  if constexpr (EPI == E2_F32_SLAB) {
    // acc[i][j]: lane l holds m = 16i + (l&15), n = 16j + 4(l>>4) + r. One TT split (or one NT split with
    // accum_direct: the fp32 step's dgrad into the residual gradient) accumulates into C; NT otherwise writes its slab
    // (split 0 of one split: C itself, ldc == N).
    const bool direct = (LA == 1 || p.accum_direct) && nwg == p.ntiles;
    const int q4 = lane >> 4, lr = lane & 15;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mw + 16 * i + lr;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nw + 16 * j + 4 * q4;
        if (direct) {
          f32x4* c = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.C) + (int64_t)m * p.ldc + n);
          *c = *c + acc[i][j];
        } else {
          float* c = reinterpret_cast<float*>(p.C) + (int64_t)split * p.M * p.N + (int64_t)m * p.N + n;
          *reinterpret_cast<f32x4*>(c) = acc[i][j];
        }
      }
    }
  } else {
    // every wave done with the operand images: they become the epilogue staging (4 x 8 KiB slices)
    if constexpr (KW == 1) G2_BARRIER();
    epilogue_bf16<EPI, 256, 4>(acc, p, smem, w4, lane, mw, nw);
  }
}

}  // namespace g2

// Main-loop schedule (interleaved rounds in one process, random operands, T = 131072 tokens): the staggered 4-phase
// form (SYNC 4) is the fastest on both layouts. NT (forward / dgrad): +5-10 % over one-barrier-per-K-tile SYNC 1 on
// every BERT shape (tools/gemm_probe.py, profiles/gemm_probe_r1_sync.json). TT (weight gradients), once its LDS-DMA
// stopped draining every K-tile (dma_lds_asm): 1,018-1,134 TFLOP/s vs 920-1,065 for SYNC 7 and 979-1,074 for SYNC 0
// on the four bert-base weights (tools/tt_probe.py, profiles/tt_probe_r3_sync_splits.json). HSD_G2_SYNC overrides
// for A/B runs; the bf16 epilogue stores are non-temporal (st16nt).
static int g2_sync_mode(int la, int K) {
  const int e = HSD_KNOB("HSD_G2_SYNC", kKnobUnset);
  (void)la;
  return e != kKnobUnset ? e : 4;
}

template <int LA, int LB, int EPI, int BN, bool SEG = false>
static void g2_launch(const G2Params& p0, int splits, hipStream_t st) {
  G2Params p = p0;
  const int tiles_m = (p.M + g2::BM - 1) / g2::BM;
  p.tiles_n = (p.N + BN - 1) / BN;
  if (splits < 1) splits = 1;
  int kps = (p.K + splits - 1) / splits;
  kps = (kps + g2::BK - 1) / g2::BK * g2::BK;
  splits = (p.K + kps - 1) / kps;
  p.kps = kps;
  p.ntiles = tiles_m * p.tiles_n;
  dim3 grid(p.ntiles * splits);
  if constexpr (SEG) {
    hipLaunchKernelGGL((g2::gemm2_kernel<LA, LB, EPI, BN, 4, true>), grid, dim3(512), 0, st, p);
    HSD_CHECK_LAUNCH();
    return;
  }
  const int mode = g2_sync_mode(LA, p.K);
  if (mode == 1) hipLaunchKernelGGL((g2::gemm2_kernel<LA, LB, EPI, BN, 1>), grid, dim3(512), 0, st, p);
  else if (mode == 2) hipLaunchKernelGGL((g2::gemm2_kernel<LA, LB, EPI, BN, 2>), grid, dim3(512), 0, st, p);
  else if (mode == 4) hipLaunchKernelGGL((g2::gemm2_kernel<LA, LB, EPI, BN, 4>), grid, dim3(512), 0, st, p);
  else if (mode == 5) hipLaunchKernelGGL((g2::gemm2_kernel<LA, LB, EPI, BN, 5>), grid, dim3(512), 0, st, p);
  else if (mode == 6) hipLaunchKernelGGL((g2::gemm2_kernel<LA, LB, EPI, BN, 6>), grid, dim3(512), 0, st, p);
  else if (mode == 7) hipLaunchKernelGGL((g2::gemm2_kernel<LA, LB, EPI, BN, 7>), grid, dim3(512), 0, st, p);
  else hipLaunchKernelGGL((g2::gemm2_kernel<LA, LB, EPI, BN, 0>), grid, dim3(512), 0, st, p);
  HSD_CHECK_LAUNCH();
}

// Persistent NT kernel (gemm2pk_kernel): for grids of more than one round of workgroups (a one-round grid has no tile
// seam to hide). Measured on the bert-base B=1024 NT GEMMs (tools/env_ab_gemm.py, profiles/persist_ab_r3.log): 1-6 %
// faster on every one, bit-identical outputs; the headline step 80.8 -> 79.3 ms. HSD_G2_PERSIST=0 turns it off.
static int g2_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return 256;
    n = prop.multiProcessorCount;
  }
  return n;
}

// Tile-queue ring of the persistent kernels (gemm_common.h tq_*): one 9-counter slot per launch, 256 slots per device,
// zeroed once; every launch leaves its slot zeroed (the last workgroup resets it). Launches on one stream reuse a slot
// only 256 launches later; persistent GEMMs run on the compute stream only (the weight-gradient side stream runs the
// TT kernels), so no two co-running launches share a slot. (The static tile walk, p.tq = nullptr, measured 71-78 %
// slower on the QKV forward with CUs held by a co-running kernel: profiles/contention_ab_r4.jsonl.)
static int* g2_tq_slot(hipStream_t st) {
  constexpr int kSlots = 256;
  static int* base[64] = {};
  static unsigned next = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) abort();
  if (base[dev] == nullptr) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
      fprintf(stderr, "gemm2: first persistent GEMM launch inside a graph capture (tile queue not allocated)\n");
      abort();
    }
    int* b = nullptr;
    if (hipMalloc(&b, sizeof(int) * kTqInts * kSlots) != hipSuccess) abort();
    if (hipMemset(b, 0, sizeof(int) * kTqInts * kSlots) != hipSuccess) abort();
    base[dev] = b;
  }
  return base[dev] + (size_t)(next++ % kSlots) * kTqInts;
}

static bool g2_persist(int tiles) {
  if (!HSD_KNOB("HSD_G2_PERSIST", 1)) return false;
  return tiles > (g2_num_cus() & ~7);
}

template <int EPI, int BN>
static void g2pk_launch(const G2Params& p0, hipStream_t st) {
  G2Params p = p0;
  const int tiles_m = (p.M + g2::BM - 1) / g2::BM;
  p.tiles_n = (p.N + BN - 1) / BN;
  p.ntiles = tiles_m * p.tiles_n;
  p.kps = p.K;
  if (p.K % g2::BK) abort();
  const int grid = std::min(p.ntiles, g2_num_cus() & ~7);
  p.tq = g2_tq_slot(st);
  hipLaunchKernelGGL((g2::gemm2pk_kernel<EPI, BN>), dim3(grid), dim3(512), 0, st, p);
  HSD_CHECK_LAUNCH();
}

template <int EPI, int BN, int FA>
static void g8pk_launch(const G2Params& p0, const float* sa, const float* sb, hipStream_t st) {
  G2Params p = p0;
  const int tiles_m = (p.M + g2::BM - 1) / g2::BM;
  p.tiles_n = (p.N + BN - 1) / BN;
  p.ntiles = tiles_m * p.tiles_n;
  p.kps = p.K;
  const int grid = p.ntiles > (g2_num_cus() & ~7) ? (g2_num_cus() & ~7) : p.ntiles;
  p.tq = g2_tq_slot(st);
  if (p.q8 != nullptr) {
    // fp8 output copies: the FFN epilogues whose outputs feed the next fp8 GEMM (GELU -> FFN2 forward, GELU'
    // product -> FFN1 dgrad)
    if constexpr (EPI == E2_BIAS_GELU_D || EPI == E2_BIAS_GELU || EPI == E2_MUL || EPI == E2_DGELU)
      hipLaunchKernelGGL((g2::gemm8pk_kernel<EPI, BN, FA, 0, true>), dim3(grid), dim3(512), 0, st, p, sa, sb);
    else
      abort();
  } else {
    hipLaunchKernelGGL((g2::gemm8pk_kernel<EPI, BN, FA, 0>), dim3(grid), dim3(512), 0, st, p, sa, sb);
  }
  HSD_CHECK_LAUNCH();
}

// fp8 NT GEMM on the persistent kernel (gemm8.hip's launch_gemm8 routes here): A8 [M][K], B8 [N][K] bytes, K % 128 == 0,
// even leading dimensions; fa: A format (0 e4m3, 1 e5m2), B e4m3.
void launch_gemm8pk(int epi, int bn, const G2Params& p0, int fa, const float* sa, const float* sb, hipStream_t st) {
  G2Params p = p0;
  p.nt_store = 1;  // non-temporal epilogue stores (profiles/store_policy_r3.log)
  p.K /= 2;
  p.lda /= 2;
  p.ldb /= 2;
#define G8PK(E)                                                                   \
  case E:                                                                         \
    if (bn == 256) {                                                              \
      if (fa == 0) g8pk_launch<E, 256, 0>(p, sa, sb, st);                         \
      else g8pk_launch<E, 256, 1>(p, sa, sb, st);                                 \
    } else {                                                                      \
      if (fa == 0) g8pk_launch<E, 192, 0>(p, sa, sb, st);                         \
      else g8pk_launch<E, 192, 1>(p, sa, sb, st);                                 \
    }                                                                             \
    return;
  switch (epi) {
    G8PK(E2_STORE)
    G8PK(E2_BIAS)
    G8PK(E2_BIAS_GELU)
    G8PK(E2_BIAS_DROP_RES)
    G8PK(E2_RES)
    G8PK(E2_DGELU)
    G8PK(E2_BIAS_GELU_D)
    G8PK(E2_MUL)
    case E2_STORE_RDOT:  // 64-column wave tiles (one head per 8-lane group): BN 256
      if (fa == 0) g8pk_launch<E2_STORE_RDOT, 256, 0>(p, sa, sb, st);
      else g8pk_launch<E2_STORE_RDOT, 256, 1>(p, sa, sb, st);
      return;
    default: abort();
  }
#undef G8PK
}

// Tile width for a bf16-output NT GEMM: minimise (rounds of 256 CUs) x (per-tile cost ∝ BN + c).
int gemm2_pick_bn(int M, int N) {
  const int tm = (M + 255) / 256;
  int best = 0;
  double best_cost = 1e30;
  for (int bn : {256, 192}) {
    if (N % bn) continue;
    const int blocks = tm * (N / bn);
    const int rounds = (blocks + 255) / 256;
    const double cost = rounds * (bn + 64.0);
    if (cost < best_cost) { best_cost = cost; best = bn; }
  }
  return best;
}

// K-splits for a bf16-output NT GEMM. A 256 x 256 tile grid that leaves more than half of the 256 CUs idle
// (the reference's own per-rank batch: bert-large, B = 8, S = 512 -> M = 4096: 64 tiles on the H-wide GEMMs)
// is split over K into fp32 slabs plus one reduce-and-epilogue pass, keeping >= 8 K-tiles per split.
// HSD_G2_SPLITK=0 disables, =n forces n.
constexpr int SBN_HOST = 128;
bool gemm2s_use(int M, int N, int K);

int gemm2_nt_splits(int M, int N, int K) {
  const int e = HSD_KNOB("HSD_G2_SPLITK", kKnobUnset);
  const int kt = K / 64;
  if (e != kKnobUnset) return std::max(1, std::min(e, kt));
  if (gemm2s_use(M, N, K)) {
    // 128 x 128 tiles: split only grids that leave more than half of the CUs idle (serving batches: B = 1 has 6-24
    // tiles, each a latency-bound chain of 12-48 K-steps), >= 2 K-tiles per split
    const int tiles = ((M + 127) / 128) * (N / 128);
    if (tiles * 2 > 256) return 1;
    int s = 256 / tiles;
    while (s > 1 && kt / s < 2) --s;
    return s;
  }
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  if (tiles * 2 > 256) return 1;
  int s = 256 / tiles;
  while (s > 1 && kt / s < 8) --s;
  return s;
}

// gemm2s (128 x 128 tiles) for NT grids that 256 x 256 tiles leave mostly idle. HSD_G2_SMALL=0 disables,
// =1 forces it for every shape it supports.
bool gemm2s_use(int M, int N, int K) {
  if (N % SBN_HOST != 0 || K % 64 != 0) return false;
  const int e = HSD_KNOB("HSD_G2_SMALL", kKnobUnset);
  if (e != kKnobUnset) return e != 0;
  // long K (>= 16,384: the MLM head's dgrad over the ~50k-word table): the 256 x 256 kernel with K-splits filling the
  // CUs beats 128 x 128 tiles at one split -- 4,928 x 1,024 x 50,432: 446 us at 3 splits vs 770 us
  // (tools/mlm_dgrad_probe.py, profiles/mlm_dgrad_probe_r4.jsonl)
  if (K >= 16384) return false;
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  return tiles * 2 <= 256;
}

// Weight-gradient plan: 256 x 256 tiles (gemm2, split-K slabs) or 128 x 128 tiles (gemm2s TT), and the K-split
// count, by a cost model fitted to tools/wgrad_ab.py on MI355X (24 BERT shapes x T = 4096 / 8192 / 16384; it
// picks the faster path on all 24, profiles/wgrad_ab_r2.json): us = rounds x (a·K-tiles per split + b) + c·MB of
// slab / C traffic, rounds = ceil(workgroups / 256) (one workgroup per CU on both). HSD_G2_SMALL_TT=0 / 1 forces
// the tile size (the split count is still chosen by the model); >= 2 K-tiles per split.
struct WgradPlan {
  bool small;
  int splits;
};

static double wgrad_cost(int M, int N, int K, int s, bool small) {
  const int tile = small ? 128 : 256;
  const double tiles = (double)((M + tile - 1) / tile) * ((N + tile - 1) / tile);
  const int kt_all = K / 64;
  const int kt = (kt_all + s - 1) / s;
  const int real = (kt_all + kt - 1) / kt;
  const double rounds = std::ceil(tiles * real / 256.0);
  const double mb = ((real > 1 ? 8.0 * real : 0.0) + 8.0) * M * N / 1e6;
  return small ? rounds * (0.658 * kt + 5.02) + 0.176 * mb : rounds * (1.637 * kt + 15.9) + 0.0847 * mb;
}

static WgradPlan wgrad_plan(int M, int N, int K) {
  const int force = HSD_KNOB("HSD_G2_SMALL_TT", -1);
  const bool can_small = N % SBN_HOST == 0 && M % 8 == 0 && K % 64 == 0 && force != 0;
  const bool can_big = N % 256 == 0 && force != 1;
  // small steps (<= 8,192 tokens), whose weight gradients run on the side stream under the backward: the fewest K-splits
  // of the 128 x 128 kernel that still give 384 workgroups, so a weight gradient takes no more CUs and slab traffic
  // than it needs beside the critical path (the latency cost model below minimises its own time instead). Measured
  // (profiles/wgrad_min_grid_ab_r4.log): bert-large S=512 B=8 504-505 -> 524-526 seq/s, bert-base B=64 +1.8 % at a
  // 192-workgroup target; re-swept in round 6 with the optimizer slices behind the weight-gradient forks
  // (profiles/r6/bl8_knob_sweep_r6.log, profiles/r6/wgrad_min_grid_small_steps_r6.log): 384 is +1.2-1.4 % at
  // bert-large B = 8 (552.6-554.2 vs 546.4-547.7) and ahead at bert-base B = 32 too; 256, 512 and 768 are 2 % slower.
  // Both are 4,096-token steps: below that (the graph-replayed small batches) the measured 192 stays.
  // HSD_WGRAD_MIN_GRID sets the workgroup target (0 = the cost model at every size).
  const int grid_knob = HSD_KNOB("HSD_WGRAD_MIN_GRID", kKnobUnset);
  const int min_grid = grid_knob != kKnobUnset ? grid_knob : (K <= 8192 ? (K >= 4096 ? 384 : 192) : 0);
  if (min_grid > 0 && can_small) {
    const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
    int sp = 1;
    while (tiles * sp < min_grid && sp < 32 && (K / 64) / (sp + 1) >= 2) ++sp;
    return WgradPlan{true, sp};
  }
  const int min_kt = 2;
  const int kt_all = K / 64;
  WgradPlan best{can_small && !can_big, 1};
  double best_cost = 1e30;
  for (int small = 0; small < 2; ++small) {
    if (small ? !can_small : !can_big) continue;
    for (int sp = 1; sp <= 32 && (sp == 1 || kt_all / sp >= min_kt); ++sp) {
      const double c = wgrad_cost(M, N, K, sp, small);
      if (c < best_cost) { best_cost = c; best = WgradPlan{small != 0, sp}; }
    }
  }
  return best;
}

bool gemm2st_use(int M, int N, int K) { return wgrad_plan(M, N, K).small; }

// LDS stages of gemm2s: 2 -> two workgroups per CU, 3 -> one with a deeper DMA prefetch. A grid that fits one
// workgroup per CU takes 3 stages, a larger one 2 (tools/nt_ab.py, profiles/nt_ab_r2.jsonl: at T = 8192 the 384-tile
// bert-base GEMMs run 19-49 us at 2 stages vs 26-68 us at 3; at <= 256 tiles 3 stages are equal or up to 5 % faster).
// HSD_G2S_STAGES (2-4) overrides.
static int g2s_stages(int grid) {
  const int e = HSD_KNOB("HSD_G2S_STAGES", kKnobUnset);
  const int v = e != kKnobUnset ? e : (grid <= 256 ? 3 : 2);
  return v < 2 ? 2 : (v > 4 ? 4 : v);
}

// gemm2s workgroup for grids of one workgroup per CU (3 stages): 8 waves with the in-workgroup K-split (2 waves per
// SIMD, default) or 4 (one per SIMD). Measured end to end (profiles/g2s_kw2_ab_r4.log, interleaved x2): bert-large
// S = 512 B = 8 488 -> 500-502 seq/s, bert-base B = 32 5,581-5,666 -> 5,723-5,734. HSD_G2S_KW = 1 / 2 overrides.
static int g2s_kw(int grid) {
  const int e = HSD_KNOB("HSD_G2S_KW", kKnobUnset);
  if (e != kKnobUnset) return e == 2 ? 2 : 1;
  (void)grid;
  return 2;
}

template <int LA, int LB, int EPI, bool SEG = false>
static void g2s_launch(const G2Params& q, int grid, hipStream_t st) {
  const int ns = g2s_stages(grid);
  if constexpr (SEG) {
    if (ns == 2) hipLaunchKernelGGL((g2::gemm2s_kernel<LA, LB, EPI, 2, 1, true>), dim3(grid), dim3(256), 0, st, q);
    else hipLaunchKernelGGL((g2::gemm2s_kernel<LA, LB, EPI, 3, 2, true>), dim3(grid), dim3(512), 0, st, q);
    HSD_CHECK_LAUNCH();
    return;
  }
  if (ns == 2) hipLaunchKernelGGL((g2::gemm2s_kernel<LA, LB, EPI, 2>), dim3(grid), dim3(256), 0, st, q);
  else if (ns == 3 && g2s_kw(grid) == 2)
    hipLaunchKernelGGL((g2::gemm2s_kernel<LA, LB, EPI, 3, 2>), dim3(grid), dim3(512), 0, st, q);
  else if (ns == 3) hipLaunchKernelGGL((g2::gemm2s_kernel<LA, LB, EPI, 3>), dim3(grid), dim3(256), 0, st, q);
  else hipLaunchKernelGGL((g2::gemm2s_kernel<LA, LB, EPI, 4>), dim3(grid), dim3(256), 0, st, q);
  HSD_CHECK_LAUNCH();
}

bool gemm2_supported(int la, int lb, int epi, int M, int N, int K) {
  if (K % 64 || M < 1 || N % 8) return false;
  if (epi == E2_STORE_RDOT && (la != 0 || N % 256)) return false;
  if (la == 0 && epi == E2_F32_SLAB) return N % 256 == 0;  // fp32-output NT, one pass (launch_gemm2)
  if (la == 0 && lb == 0) return epi_bf16_out(epi) && gemm2_pick_bn(M, N) != 0;
  if (la == 0 && lb == 1) return epi_bf16_out(epi) && (N % 256 == 0 || gemm2s_use(M, N, K));
  if (la == 1 && lb == 1)
    return (epi == E2_F32_ATOMIC || epi == E2_F32_SLAB) && M % 8 == 0 &&
           (N % 256 == 0 || (epi == E2_F32_SLAB && gemm2st_use(M, N, K)));
  return false;
}

// K-splits of the fp32-output NT GEMM (the fp32 step's split-product forward / dgrad): a 256 x 256 grid of at most
// half the CUs (bert-large B = 8: M = 4,096 tokens, N = 1,024 -> 64 workgroups on 256 CUs) is split over K until it
// fills the chip, keeping >= 8 K-tiles per split. HSD_F32NT_SPLITS: 1 = off, n = force n.
int gemm2_f32nt_splits(int M, int N, int K) {
  const int force = HSD_KNOB("HSD_F32NT_SPLITS", 0);
  if (force > 0) return std::max(1, std::min(force, K / 64));
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const int cus = g2_num_cus();
  if (2 * tiles > cus) return 1;
  return std::max(1, std::min(cus / tiles, K / (64 * 8)));
}

// K-splits of the TT wgrad (wgrad_plan)
int gemm2_wgrad_splits(int M, int N, int K) {
  return wgrad_plan(M, N, K).splits;
}

// NT-shaped GEMM (bf16 out, fused epilogues): B k-contiguous (LB = 0: B[N][K], e.g. the stored Wᵀ for dgrad) or
// k-strided (LB = 1: B[K][N], the dgrad reading W[N_out][K_in] directly, no Wᵀ copy). 128 x 128 tiles for grids the
// 256 x 256 kernel leaves mostly idle, split-K slabs + one reduce-and-epilogue pass for the smallest grids.
template <int LB>
static void launch_nt(const G2Params& p, int epi, int M, int N, int K, int splits, float* ws, float* dbias,
                      hipStream_t st) {
  if (splits <= 1 && gemm2s_use(M, N, K)) {
    G2Params q = p;
    q.tiles_n = N / g2::SBN;
    q.ntiles = ((M + g2::SBM - 1) / g2::SBM) * q.tiles_n;
    q.kps = K;
#define G2_SMALL(E)                   \
  case E:                             \
    g2s_launch<0, LB, E>(q, q.ntiles, st); \
    break;
    switch (epi) {
      G2_SMALL(E2_STORE)
      G2_SMALL(E2_BIAS)
      G2_SMALL(E2_BIAS_GELU)
      G2_SMALL(E2_BIAS_DROP_RES)
      G2_SMALL(E2_RES)
      G2_SMALL(E2_DGELU)
      G2_SMALL(E2_BIAS_GELU_D)
      G2_SMALL(E2_MUL)
      G2_SMALL(E2_STORE_RDOT)
      default: abort();
    }
#undef G2_SMALL
    return;
  }
  if (splits > 1) {
    if (ws == nullptr || !epi_bf16_out(epi)) abort();
    G2Params q = p;
    q.C = ws;
    q.dbias = nullptr;
    int kps = (K + splits - 1) / splits;
    kps = (kps + 63) / 64 * 64;
    const int real = (K + kps - 1) / kps;
    if (gemm2s_use(M, N, K)) {
      q.tiles_n = N / g2::SBN;
      q.ntiles = ((M + g2::SBM - 1) / g2::SBM) * q.tiles_n;
      q.kps = kps;
      g2s_launch<0, LB, E2_F32_SLAB>(q, q.ntiles * real, st);
    } else {
      g2_launch<0, LB, E2_F32_SLAB, 256>(q, splits, st);
    }
    const int gx = (N + 63) / 64;
    const int gy_want = std::max(1, 2048 / gx);
    int rpb = (M + gy_want - 1) / gy_want;
    rpb = (rpb + 31) / 32 * 32;
    const dim3 grid(gx, (M + rpb - 1) / rpb);
#define G2_SK(E)                                                                                          \
  case E:                                                                                                 \
    hipLaunchKernelGGL(g2::splitk_epi_kernel<E>, grid, dim3(256), 0, st, (const float*)ws, real, rpb, p); \
    break;
    switch (epi) {
      G2_SK(E2_STORE)
      G2_SK(E2_BIAS)
      G2_SK(E2_BIAS_GELU)
      G2_SK(E2_BIAS_DROP_RES)
      G2_SK(E2_RES)
      G2_SK(E2_DGELU)
      G2_SK(E2_BIAS_GELU_D)
      G2_SK(E2_MUL)
      G2_SK(E2_STORE_RDOT)
      default: abort();
    }
#undef G2_SK
    HSD_CHECK_LAUNCH();
    return;
  }
  {
    int bn = LB == 1 || epi == E2_STORE_RDOT ? 256 : gemm2_pick_bn(M, N);  // k-strided B images are 256 wide
    if (dbias != nullptr) {
      if ((epi != E2_DGELU && epi != E2_MUL) || N % 256) abort();  // fused column sums: 8 columns per lane (BN 256)
      bn = 256;
    }
    const bool pk = LB == 0 && g2_persist((M + 255) / 256 * (N / bn));
#define G2_NT(E)                                                     \
  case E:                                                            \
    if (pk) {                                                        \
      if (bn == 256) g2pk_launch<E, 256>(p, st);                     \
      else g2pk_launch<E, 192>(p, st);                               \
    } else if (bn == 256 || LB == 1) {                               \
      g2_launch<0, LB, E, 256>(p, 1, st);                            \
    } else {                                                         \
      g2_launch<0, LB, E, LB == 1 ? 256 : 192>(p, 1, st);            \
    }                                                                \
    return;
    switch (epi) {
      G2_NT(E2_STORE)
      G2_NT(E2_BIAS)
      G2_NT(E2_BIAS_GELU)
      G2_NT(E2_BIAS_DROP_RES)
      G2_NT(E2_RES)
      G2_NT(E2_DGELU)
      G2_NT(E2_BIAS_GELU_D)
      G2_NT(E2_MUL)
      case E2_STORE_RDOT:  // 64-column wave tiles only (one head per 8-lane group): BN 256
        if (pk) g2pk_launch<E2_STORE_RDOT, 256>(p, st);
        else g2_launch<0, LB, E2_STORE_RDOT, 256>(p, 1, st);
        return;
      default: abort();
    }
#undef G2_NT
  }
}

static unsigned long long* g_diag = nullptr;
void gemm2_set_diag(void* p) { g_diag = (unsigned long long*)p; }

void launch_gemm2(int la, int lb, int epi, const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, int M, int N,
                  int K, void* C, int64_t ldc, const bf16_t* bias, const bf16_t* aux, int64_t ldaux, bf16_t* C2,
                  double p_drop, uint64_t seed, int splits, float* ws, float* dbias, hipStream_t st, float* rd,
                  int rd_seq) {
  G2Params p{};
  p.dbias = dbias;
  p.rd = rd;
  p.rd_seq = rd_seq;
  if (epi == E2_STORE_RDOT && (rd == nullptr || rd_seq <= 0 || M % rd_seq || N % 64)) abort();
  p.diag = g_diag;
  p.nt_store = 1;  // non-temporal epilogue stores (profiles/store_policy_r3.log)
  p.A = A; p.lda = lda; p.B = B; p.ldb = ldb; p.M = M; p.N = N; p.K = K; p.C = C; p.ldc = ldc;
  p.bias = bias; p.aux = aux; p.ldaux = ldaux; p.C2 = C2;
  p.dp = make_dropout(p_drop, seed);
  if (la == 0 && epi == E2_F32_SLAB) {
    // fp32 output [M][N] (ldc == N): the split-product GEMMs of the fp32 step (fp32.hip, ops/hip32.py). splits > 1
    // (gemm2_f32nt_splits: grids that would leave most CUs idle): K-split fp32 slabs in ws, then C = Σ slabs
    if (ldc != N || (splits > 1 && ws == nullptr)) abort();
    G2Params q = p;
    if (splits > 1) q.C = ws;
    if (lb == 0) g2_launch<0, 0, E2_F32_SLAB, 256>(q, splits, st);
    else g2_launch<0, 1, E2_F32_SLAB, 256>(q, splits, st);
    if (splits > 1) {
      int kps = (K + splits - 1) / splits;
      kps = (kps + 63) / 64 * 64;
      const int real = (K + kps - 1) / kps;
      const int64_t n4 = (int64_t)M * N / 4;
      const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
      hipLaunchKernelGGL(g2::slab_reduce_kernel, dim3(blocks), dim3(256), 0, st, ws, reinterpret_cast<float*>(C), ldc,
                         M, N, real, 1);
      HSD_CHECK_LAUNCH();
    }
    return;
  }
  if (la == 0 && lb == 0) {
    launch_nt<0>(p, epi, M, N, K, splits, ws, dbias, st);
  } else if (la == 1 && lb == 1) {
    if (splits <= 0) splits = gemm2_wgrad_splits(M, N, K);
    if (epi == E2_F32_SLAB && gemm2st_use(M, N, K) && (splits == 1 || ws != nullptr)) {
      G2Params q = p;
      q.tiles_n = N / g2::SBN;
      q.ntiles = ((M + g2::SBM - 1) / g2::SBM) * q.tiles_n;
      int kps = (K + splits - 1) / splits;
      kps = (kps + 63) / 64 * 64;
      const int real = (K + kps - 1) / kps;
      q.kps = kps;
      if (real > 1) q.C = ws;
      g2s_launch<1, 1, E2_F32_SLAB>(q, q.ntiles * real, st);
      if (real > 1) {
        const int64_t n4 = (int64_t)M * N / 4;
        int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
        hipLaunchKernelGGL(g2::slab_reduce_kernel, dim3(blocks), dim3(256), 0, st, ws, reinterpret_cast<float*>(C),
                           ldc, M, N, real, 0);
        HSD_CHECK_LAUNCH();
      }
    } else if (epi == E2_F32_SLAB && splits > 1 && ws != nullptr) {
      G2Params q = p;
      q.C = ws;
      g2_launch<1, 1, E2_F32_SLAB, 256>(q, splits, st);
      int kps = (K + splits - 1) / splits;
      kps = (kps + 63) / 64 * 64;
      const int real = (K + kps - 1) / kps;
      const int64_t n4 = (int64_t)M * N / 4;
      int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
      hipLaunchKernelGGL(g2::slab_reduce_kernel, dim3(blocks), dim3(256), 0, st, ws, reinterpret_cast<float*>(C), ldc,
                         M, N, real, 0);
      HSD_CHECK_LAUNCH();
    } else if (epi == E2_F32_SLAB && splits <= 1 && ldc % 4 == 0 && !HSD_KNOB("HSD_G2_TT_ATOMIC", 0)) {
      // one K-split: every output element has one owner -> C += acc in place instead of fp32 atomics (the tied MLM
      // decoder weight gradient: Vp x H = 51.6 M atomics per roberta-large step; HSD_G2_TT_ATOMIC=1 = the old path)
      G2Params q = p;
      q.accum_direct = 1;
      g2_launch<1, 1, E2_F32_SLAB, 256>(q, 1, st);
    } else {
      g2_launch<1, 1, E2_F32_ATOMIC, 256>(p, splits, st);
    }
  } else if (la == 0 && lb == 1) {
    launch_nt<1>(p, epi, M, N, K, splits, ws, dbias, st);
  } else {
    abort();
  }
}

// ---- segmented-K fp32-output GEMMs (the fp32 step's split products) ------------------------------------------------
// C[M][N] (fp32) = Σ_{s<3} A_s · B_s over segments of Kseg (G2Params seg): la = 0, lb = 0 / 1: the NT forward / dgrad
// (C written, or C += with `accumulate`: the fp32 blocks' residual gradient + dgrad in place; split-K slabs + one reduce
// for small grids, gemm2_f32nt_splits), la = lb = 1: the TT weight gradient (C += ..., wgrad_plan's tile size and
// K-splits). Kseg % 64 == 0.
// the fp32 forward / dgrad on 128 x 128 tiles (gemm2s, one K-split) for grids that 256 x 256 tiles leave mostly idle
// (gemm2s_use) and K < 6,144, instead of 256 x 256 tiles split over K into slabs plus a reduce pass. bert-large T = 4,096
// (tools/seg_vs_cat.py, profiles/r6/seg_vs_cat_r6e.log): N 1,024 at K 3 x 1,024: 32.4 / 34.8 us (fwd / dgrad) vs 44.4 /
// 45.2 on slabs; at K 3 x 3,072 and 3 x 4,096 the slabs win (81.6 vs 91.2, 96.6 vs 111.8, 99.3 vs 124.5 us).
// HSD_SEG_NT_SMALL=0: always the slabs.
static bool seg_nt_small(int M, int N, int K) {
  return HSD_KNOB("HSD_SEG_NT_SMALL", 1) && K < 6144 && gemm2s_use(M, N, K);
}

bool gemm2_seg_supported(int la, int lb, int M, int N, int Kseg) {
  if (Kseg % 64 || Kseg <= 0) return false;
  if (la == 0) return (lb == 0 || lb == 1) && gemm2_supported(0, lb, E2_F32_SLAB, M, N, 3 * Kseg);
  return la == 1 && lb == 1 && gemm2_supported(1, 1, E2_F32_SLAB, M, N, 3 * Kseg);
}

int64_t gemm2_seg_ws_numel(int la, int lb, int M, int N, int Kseg) {
  const int K = 3 * Kseg;
  if (la == 0 && seg_nt_small(M, N, K)) return 0;
  int sp = la == 0 ? gemm2_f32nt_splits(M, N, K) : wgrad_plan(M, N, K).splits;
  if (sp <= 1) return 0;
  int kps = (K + sp - 1) / sp;
  kps = (kps + 63) / 64 * 64;
  return (int64_t)((K + kps - 1) / kps) * M * N;
}

void launch_gemm2_seg(int la, int lb, const bf16_t* const A[3], int64_t lda, const bf16_t* const B[3], int64_t ldb,
                      int M, int N, int Kseg, float* C, int64_t ldc, float* ws, hipStream_t st, bool accumulate) {
  if (!gemm2_seg_supported(la, lb, M, N, Kseg) || ldc % 4) abort();
  G2Params p{};
  p.nt_store = 1;
  p.A = A[0]; p.lda = lda; p.B = B[0]; p.ldb = ldb; p.M = M; p.N = N; p.K = 3 * Kseg; p.C = C; p.ldc = ldc;
  p.seg = Kseg;
  for (int s = 0; s < 3; ++s) {
    p.segA[s] = A[s];
    p.segB[s] = B[s];
  }
  const int K = 3 * Kseg;
  auto reduce = [&](int real, int assign) {
    const int64_t n4 = (int64_t)M * N / 4;
    const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
    hipLaunchKernelGGL(g2::slab_reduce_kernel, dim3(blocks), dim3(256), 0, st, ws, C, ldc, M, N, real, assign);
    HSD_CHECK_LAUNCH();
  };
  auto real_of = [&](int sp) {
    int kps = (K + sp - 1) / sp;
    kps = (kps + 63) / 64 * 64;
    return (K + kps - 1) / kps;
  };
  if (la == 0) {
    if (ldc != N) abort();
    if (seg_nt_small(M, N, K)) {
      // 128 x 128 tiles, one K-split: the grid fills the CUs without slabs or a reduce pass; each output element has
      // one owner (written, or C += acc with `accumulate`)
      G2Params q = p;
      q.tiles_n = N / g2::SBN;
      q.ntiles = ((M + g2::SBM - 1) / g2::SBM) * q.tiles_n;
      q.kps = K;
      q.accum_direct = accumulate ? 1 : 0;
      if (lb == 0) g2s_launch<0, 0, E2_F32_SLAB, true>(q, q.ntiles, st);
      else g2s_launch<0, 1, E2_F32_SLAB, true>(q, q.ntiles, st);
      return;
    }
    const int sp = gemm2_f32nt_splits(M, N, K);
    if (sp > 1 && ws == nullptr) abort();
    G2Params q = p;
    if (sp > 1) q.C = ws;
    else q.accum_direct = accumulate ? 1 : 0;  // one split: each element has one owner (C += acc in place)
    if (lb == 0) g2_launch<0, 0, E2_F32_SLAB, 256, true>(q, sp, st);
    else g2_launch<0, 1, E2_F32_SLAB, 256, true>(q, sp, st);
    if (sp > 1) reduce(real_of(sp), accumulate ? 0 : 1);
    return;
  }
  const WgradPlan plan = wgrad_plan(M, N, K);
  const int real = real_of(plan.splits);
  if (real > 1 && ws == nullptr) abort();
  G2Params q = p;
  if (plan.small) {
    q.tiles_n = N / g2::SBN;
    q.ntiles = ((M + g2::SBM - 1) / g2::SBM) * q.tiles_n;
    int kps = (K + plan.splits - 1) / plan.splits;
    q.kps = (kps + 63) / 64 * 64;
    if (real > 1) q.C = ws;  // one split: the kernel accumulates into C (unique owner per element)
    g2s_launch<1, 1, E2_F32_SLAB, true>(q, q.ntiles * real, st);
  } else if (real > 1) {
    q.C = ws;
    g2_launch<1, 1, E2_F32_SLAB, 256, true>(q, plan.splits, st);
  } else {
    q.accum_direct = 1;
    g2_launch<1, 1, E2_F32_SLAB, 256, true>(q, 1, st);
  }
  if (real > 1) reduce(real, 0);
}

// ---- fp8 TT weight gradient (g2::gemm8tt_kernel) ----------------------------------------------------------------------
bool gemm8_wgrad_supported(int M, int N, int T) { return M % 256 == 0 && N % 256 == 0 && T % 128 == 0 && T >= 128; }

// K-splits: wgrad_plan's cost model for the 256-tile kernel with one fp8 K-tile (128 tokens: the bytes and MFMA cycles
// of one bf16 K-tile of 64) per bf16 K-tile
int gemm8_wgrad_splits(int M, int N, int T) {
  const int kt_all = T / 128;
  int best = 1;
  double best_cost = 1e30;
  for (int sp = 1; sp <= 32 && (sp == 1 || kt_all / sp >= 2); ++sp) {
    const double c = wgrad_cost(M, N, T / 2, sp, false);
    if (c < best_cost) { best_cost = c; best = sp; }
  }
  return best;
}

// token splits actually launched for `splits` requested (each a multiple of 128 tokens); the workspace holds that
// many [M][N] fp32 slabs
static int g8tt_kps(int T, int splits) {
  int kps = (T + splits - 1) / splits;
  return (kps + 127) / 128 * 128;
}
int64_t gemm8_wgrad_ws_numel(int M, int N, int T, int splits) {
  if (splits <= 0) splits = gemm8_wgrad_splits(M, N, T);
  const int kps = g8tt_kps(T, splits);
  return (int64_t)((T + kps - 1) / kps) * M * N;
}

// C[M][N] (fp32, ldc) += sdy·sx · dY8ᵀ · X8: dY8 [T][M] (ldd bytes, format fdy), X8 [T][N] (ldx bytes, e4m3)
void launch_gemm8_wgrad(const uint8_t* dy, int64_t ldd, int fdy, const float* sdy, const uint8_t* x, int64_t ldx,
                        int fx, const float* sx, int M, int N, int T, float* C, int64_t ldc, int splits, float* ws,
                        hipStream_t st) {
  if (!gemm8_wgrad_supported(M, N, T) || fx != 0 || (fdy != 0 && fdy != 1) || ws == nullptr) abort();
  if (splits <= 0) splits = gemm8_wgrad_splits(M, N, T);
  G2Params p{};
  p.A = reinterpret_cast<const bf16_t*>(dy); p.lda = ldd;
  p.B = reinterpret_cast<const bf16_t*>(x); p.ldb = ldx;
  p.M = M; p.N = N; p.K = T; p.C = ws; p.ldc = N;
  p.kps = g8tt_kps(T, splits);
  const int real = (T + p.kps - 1) / p.kps;
  p.tiles_n = N / 256;
  p.ntiles = (M / 256) * p.tiles_n;
  const dim3 grid(p.ntiles * real);
  if (fdy == 0) hipLaunchKernelGGL((g2::gemm8tt_kernel<0, 0>), grid, dim3(512), 0, st, p, sdy, sx);
  else hipLaunchKernelGGL((g2::gemm8tt_kernel<1, 0>), grid, dim3(512), 0, st, p, sdy, sx);
  HSD_CHECK_LAUNCH();
  const int64_t n4 = (int64_t)M * N / 4;
  const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
  hipLaunchKernelGGL(g2::slab_reduce_kernel, dim3(blocks), dim3(256), 0, st, ws, C, ldc, M, N, real, 0);
  HSD_CHECK_LAUNCH();
}

}  // namespace hsd
