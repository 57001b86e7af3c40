// gemm2pd: persistent NT GEMM whose epilogue runs UNDER the next tile's main loop.
//
// Why (profiles/store_probe_r4.jsonl, tools/store_probe.cpp): one CU alone stores at ~130 GB/s, but when all 256 CUs
// store at once the chip delivers ~5.9 TB/s = 23 GB/s per CU. The 256 x 256 persistent kernel (gemm2pk) runs every
// CU's epilogue at the same moment, after the tile's MFMAs: the FFN1 forward's 256 KiB of GELU / GELU' stores per
// tile take ~20k cycles + a ~10k seam against a 33k-cycle main loop (profiles/seam_probe_r3.log). Spread over the
// main loop the same bytes need ~2 TB/s. A 256 x 256 tile's output does not fit anywhere while the next tile
// accumulates (LDS: 2 x 64 KiB operand stages; registers: 238-249 of 256), so this kernel uses 128 x 256 tiles:
//
// * 8 waves as 2 (M) x 4 (N), 64 x 64 wave tiles: 64 accumulator registers. At the tile's last K-tile each wave packs
//   bf16(acc + bias) into 32 registers (the DEFERRED tile) and starts the next tile at once -- no seam, no drain.
// * during K-tiles 0..7 of the next tile each wave runs one "piece" of the deferred epilogue in its read phase (P2),
//   while its SIMD partner (the other wave group, one barrier behind) runs MFMAs: a 16-row pass through a 2 KiB
//   wave-private LDS slice (written every second piece), one 16-B chunk per lane through the epilogue math (GELU +
//   GELU' for FFN1) and its stores. The VALU work of a piece fits under the partner's MFMA cluster.
// * operands: 3-stage LDS ring of 48 KiB (A 128 x 64, B 256 x 64, source-swizzled LDS-DMA images as gemm2), the DMA of
//   stream K-tile s + 2 issued during K-tile s (the stream runs across tile boundaries, so the next tile's first
//   K-tiles are already in flight when a tile ends); 3 x 48 + 16 KiB staging = 160 KiB.
// * every vector-memory op in the loop is counted by hand: DMA slots (inline asm), the pieces' stores (always issued;
//   rows past M go to an out-of-range buffer offset that the hardware drops), and one wait per K-tile,
//   vmcnt(S(s-1) + G + S(s)), retires K-tile s + 1 without waiting for any store.
// * bias: 8 B per lane per tile, loaded at the tile's start, used at its end (the wait hipcc puts there counts the
//   pieces' stores issued since, so the load has long landed).
// Outputs are bit-identical to gemm2pk / gemm2 (same fragments, same K order per element, same epilogue math):
// tests/test_gpu_gemm.py::test_gemm2_deferred_epilogue_matches_persistent.
#include "gemm2_dev.h"

namespace hsd {
namespace g2 {
namespace pd {

constexpr int BMD = 128, BND = 256, NSTG = 3;
constexpr int TA = BMD * 64, TB = BND * 64, STAGE = TA + TB;  // elements
constexpr int GA = 2, GB = 4, G = GA + GB, G1 = 3;              // DMA slots per wave per K-tile (G1 in P1)
constexpr int SROWS = 16;
constexpr int STG = 8 * SROWS * 64;  // staging elements (8 waves x one 16-row pass)
constexpr int NPIECE = 8;            // pieces per deferred tile: 64 rows x 8 chunks / 64 lanes
constexpr int BIAS_KT = NPIECE;      // K-tile of the bias DMA; retired by K-tile BIAS_KT + 2's wait -> nt >= 11

template <int EPI>
constexpr int stores_per_piece() { return epi_two_out(EPI) ? 2 : 1; }

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm2pd_kernel(G2Params p) {
  static_assert(EPI == E2_STORE || EPI == E2_BIAS || EPI == E2_BIAS_GELU || EPI == E2_BIAS_GELU_D,
                "epilogues without an aux operand");
  constexpr int SP = stores_per_piece<EPI>();
  static_assert(2 * SP + G <= 10, "vmcnt_rt range");
  __shared__ __attribute__((aligned(16))) bf16_t smem[NSTG * STAGE + STG];
  static_assert(sizeof(smem) <= 160 * 1024, "LDS");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int ntiles = p.ntiles, q8 = ntiles >> 3, r8 = ntiles & 7;
  const int nt = p.K / BK;
  const int grid = gridDim.x, bid = blockIdx.x;
  const int my_tiles = (ntiles - bid + grid - 1) / grid;
  const int total = my_tiles * nt;  // K-tiles of this workgroup's stream
  HSD_DASSERT(p.K % BK == 0 && nt >= BIAS_KT + 3 && bid < ntiles && grid % 8 == 0);
  // tile order: the XCD-aware remap gives each XCD's 32 workgroups 32 consecutive indices v per round; in groups of
  // group_m row tiles those are group_m rows x 32/group_m columns (8 x 4: 8 A panels + 4 B panels = 3.1 MB, inside
  // the XCD's 4 MB L2; row-major: ~3 A panels + all 12 B panels of the FFN weight = 5 MB)
  const int tiles_m = ntiles / p.tiles_n;
  auto tile_of = [&](int j, int& m0, int& n0) {
    const int L = bid + j * grid;
    const int xcd = L & 7;
    const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (L >> 3);
    int tm, tn;
    if (p.group_m > 0) {
      const int per = p.group_m * p.tiles_n;
      const int g = v / per, first = g * p.group_m;
      const int gs = min(tiles_m - first, p.group_m);
      const int w = v - g * per;
      tm = first + w % gs;
      tn = w / gs;
    } else {
      tm = v / p.tiles_n;
      tn = v % p.tiles_n;
    }
    m0 = tm * BMD;
    n0 = tn * BND;
  };
  const uint32_t smem_lds = (uint32_t)(size_t)(__attribute__((address_space(3))) bf16_t*)smem;

  // ---- DMA stream state: the tile / K-tile of the next K-tile to issue
  int dj = 0, dk = 0, dm0, dn0;
  uint32_t aoff[G];
  auto dma_tile = [&]() {
    tile_of(dj, dm0, dn0);
#pragma unroll
    for (int q = 0; q < G; ++q)
      aoff[q] = q < GA ? lane_off<0>(p.lda, dm0, p.M, wave * GA + q, lane)
                       : lane_off<0>(p.ldb, dn0, p.N, wave * GB + (q - GA), lane);
  };
  // slots [q0, q1) of the current DMA K-tile into its stage (stream index s_dma % 3)
  auto dma_part = [&](int s_dma, int q0, int q1) {
    const uint32_t st = smem_lds + (uint32_t)((s_dma % NSTG) * STAGE) * 2u;
    const int k0 = dk * BK;
#pragma unroll
    for (int q = 0; q < G; ++q) {
      if (q < q0 || q >= q1) continue;
      if (q < GA) dma_lds_asm(asm_base<0>(p.A, p.lda, dm0, k0), aoff[q], st + (wave * GA + q) * 1024u);
      else dma_lds_asm(asm_base<0>(p.B, p.ldb, dn0, k0), aoff[q], st + (TA + (wave * GB + (q - GA)) * 512) * 2u);
    }
  };
  auto dma_advance = [&]() {
    if (++dk == nt) {
      dk = 0;
      ++dj;
      if (dj < my_tiles) dma_tile();
    }
  };

  // ---- deferred tile: bf16(acc + bias) of the last finished tile, its coordinates
  u32x2 y[4][4];
  int ym0 = 0, yn0 = 0;
  bf16_t* const stg = smem + NSTG * STAGE + wave * (SROWS * 64);
  const int q4 = lane >> 4, lr = lane & 15;
  auto piece = [&](int k) {
    const int pass = k >> 1, half = k & 1;
    if (half == 0) {
      // the pass's 16 rows into the wave's staging slice, 8-B slots XOR-swizzled by row. The passes leave y[0] in
      // order and the blocks rotate down (register moves): y is never indexed at run time (a run-time index sends
      // the array to scratch, and a scratch load's vmcnt(0) would drain the operand DMA every piece)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = ((4 * j + q4) ^ lr) << 2;
        *reinterpret_cast<u32x2*>(stg + lr * 64 + col) = y[0][j];
      }
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) y[i][j] = y[i + 1][j];
      __builtin_amdgcn_wave_barrier();
    }
    const int idx = lane + 64 * half;
    const int row = idx >> 3, c8 = idx & 7;
    const u32x4 t = *reinterpret_cast<const u32x4*>(stg + row * 64 + ((c8 ^ (row >> 1)) << 3));
    u32x4 o = (row & 1) ? u32x4{t.z, t.w, t.x, t.y} : t, o2;
    const int mw = ym0 + wm * 64;
    const int m = mw + pass * 16 + row, n = yn0 + wn * 64 + c8 * 8;
    float csum[8];
    epi_chunk<EPI>(o, o2, u32x4{0, 0, 0, 0}, m, n, p, csum);
    // rows past M: the buffer range ends at row M, so the hardware drops those stores whole while they are still
    // issued (the vm counter sees exactly SP stores per piece). Range = (M - mw) rows of ldc elements (0 when the
    // wave's 64 rows all lie past M); the row offset of an in-range store is < 64 rows.
    const int vrows = max(0, min(64, p.M - mw));
    const uint32_t nb = (uint32_t)((int64_t)(vrows > 0 ? vrows - 1 : 0) * p.ldc * 2 + (vrows > 0 ? (int64_t)p.N * 2 : 0));
    const uint32_t bo = (uint32_t)(((int64_t)(m - mw) * p.ldc + n) * 2);
    bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
    st16nt(wave_rsrc_n(C + (int64_t)mw * p.ldc, nb), bo, o);
    if constexpr (SP == 2) st16nt(wave_rsrc_n(p.C2 + (int64_t)mw * p.ldc, nb), bo, o2);
  };

  // ---- compute stream
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int cj = 0, ck = 0;  // compute tile / K-tile
  int cm0, cn0;
  tile_of(0, cm0, cn0);
  // the compute tile's bias: the wave's 64 columns (128 B) LDS-DMA'd by lanes 0..7 into the start of its staging
  // slice in K-tile BIAS_KT, when no piece uses the slice; counted like the pieces' stores, retired by the waits of
  // the K-tiles after it and read at the tile's end. (A vector load into registers made hipcc, which cannot count
  // K-tiles across the loop back-edge, wait vmcnt(0) at the tile boundary and drain the operand DMA.)
  const uint32_t stg_lds = smem_lds + (uint32_t)(NSTG * STAGE + wave * (SROWS * 64)) * 2u;
  dma_tile();
  // prologue: stream K-tiles 0 and 1 (my_tiles >= 1 and nt >= 8, so both exist)
  dma_part(0, 0, G);
  dma_advance();
  dma_part(1, 0, G);
  dma_advance();
  vmcnt<G>();
  G2_BARRIER();
  if (wm == 1) G2_BARRIER();  // stagger: group 1 runs one barrier behind for the whole stream
  const int arow = wm * 64, bcol = wn * 64;
  int s_prev = 0;
  for (int s = 0; s < total; ++s) {
    const bf16_t* cA = smem + (s % NSTG) * STAGE;
    const bf16_t* cB = cA + TA;
    const bool dma_on = s + 2 < total;
    const bool has_piece = cj > 0 && ck < NPIECE;
    const bool bias_dma = epi_bias(EPI) && ck == BIAS_KT;
    const int s_cur = has_piece ? SP : (bias_dma ? 1 : 0);
    bf16x8 fa[4][2], fb[2][2];
    // P1: A (all four row blocks) + B cols 0..31, first DMA slots of stream K-tile s + 2
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fb[j][ks] = frag<0>(cB, bcol + 16 * j, ks, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fa[i][ks] = frag<0>(cA, arow + 16 * i, ks, lane);
    if (dma_on) dma_part(s + 2, 0, G1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G2_BARRIER();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][ks], fa[i][ks], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    G2_BARRIER();
    // P2: B cols 32..63, the rest of the DMA, one deferred-epilogue piece, retire stream K-tile s + 1
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fb[j][ks] = frag<0>(cB, bcol + 32 + 16 * j, ks, lane);
    if (dma_on) {
      dma_part(s + 2, G1, G);
      dma_advance();
    }
    if (has_piece) piece(ck);
    if (bias_dma) {
      if (lane < 8) {
        const uint64_t ba = (uint64_t)(p.bias + cn0 + bcol);
        const bf16_t* bp = (const bf16_t*)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(ba >> 32)) << 32) |
                                           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)ba));
        dma_lds_asm(bp, (uint32_t)lane * 16u, stg_lds);
      }
    }
    vmcnt_rt(s_prev + (dma_on ? G : 0) + s_cur);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    G2_BARRIER();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][ks], fa[i][ks], acc[i][2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    G2_BARRIER();
    s_prev = s_cur;
    if (++ck == nt) {
      // tile boundary: bf16(acc + bias) -> the deferred registers (its pieces of the previous tile all ran in K-tiles
      // 0..7 of this one), next tile
      f32x4 bv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (epi_bias(EPI)) {
          const u32x2 b = *reinterpret_cast<const u32x2*>(stg + 16 * j + 4 * q4);
          bv[j] = f32x4{lo_bf(b.x), hi_bf(b.x), lo_bf(b.y), hi_bf(b.y)};
        } else {
          bv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f32x4 v = acc[i][j];
          if constexpr (epi_bias(EPI)) v += bv[j];
          y[i][j] = pack4(v);
          acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      ym0 = cm0;
      yn0 = cn0;
      ck = 0;
      if (++cj < my_tiles) tile_of(cj, cm0, cn0);
    }
  }
  if (wm == 0) G2_BARRIER();
  // the last tile's epilogue has no main loop to hide under
#pragma unroll 1
  for (int k = 0; k < NPIECE; ++k) piece(k);
  vmcnt<0>();
}

}  // namespace pd
}  // namespace g2

bool gemm2pd_supported(int epi, int M, int N, int K) {
  return (epi == E2_STORE || epi == E2_BIAS || epi == E2_BIAS_GELU || epi == E2_BIAS_GELU_D) && N % 256 == 0 &&
         K % 64 == 0 && K / 64 >= g2::pd::BIAS_KT + 3 && M >= 1;
}

// grid: one workgroup per CU (multiple of 8), at most one per tile. bias is read by 128-B scalar loads per wave
// (aligned: n0 and the wave offset are multiples of 64 columns).
void launch_gemm2pd(int epi, const G2Params& p0, int num_cus, hipStream_t st) {
  G2Params p = p0;
  const int tiles_m = (p.M + g2::pd::BMD - 1) / g2::pd::BMD;
  p.tiles_n = p.N / g2::pd::BND;
  p.ntiles = tiles_m * p.tiles_n;
  p.kps = p.K;
  p.group_m = HSD_KNOB("HSD_G2_GROUP", 8);
  int grid = num_cus & ~7;
  if (p.ntiles < grid) grid = p.ntiles & ~7;
  if (grid < 8) abort();  // tiny grids: the caller keeps gemm2pk / gemm2
  switch (epi) {
    case E2_STORE: hipLaunchKernelGGL(g2::pd::gemm2pd_kernel<E2_STORE>, dim3(grid), dim3(512), 0, st, p); break;
    case E2_BIAS: hipLaunchKernelGGL(g2::pd::gemm2pd_kernel<E2_BIAS>, dim3(grid), dim3(512), 0, st, p); break;
    case E2_BIAS_GELU:
      hipLaunchKernelGGL(g2::pd::gemm2pd_kernel<E2_BIAS_GELU>, dim3(grid), dim3(512), 0, st, p);
      break;
    case E2_BIAS_GELU_D:
      hipLaunchKernelGGL(g2::pd::gemm2pd_kernel<E2_BIAS_GELU_D>, dim3(grid), dim3(512), 0, st, p);
      break;
    default: abort();
  }
  HSD_CHECK_LAUNCH();
}

}  // namespace hsd
