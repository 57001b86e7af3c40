// bf16 MFMA GEMM with fused epilogues for the BERT training step.
//
//   C[m][n] = Σ_k A(m,k) · B(k,n)      fp32 accumulate, v_mfma_f32_32x32x16_bf16
//
// Operand layouts (template LA / LB) cover all three training GEMMs without any transpose pass:
//   forward  Y = X·Wᵀ     : A = X  [M][K]  (LA=0, k-contiguous)   B = W  [N][K] (LB=0, k-contiguous)
//   dgrad    dX = dY·W    : A = dY [M][N'] (LA=0)                  B = W  [N'][K'] (LB=1, n-contiguous)
//   wgrad    dW += dYᵀ·X  : A = dY [T][N]  (LA=1, m-contiguous)    B = X  [T][K] (LB=1, n-contiguous)
// k-contiguous tiles are staged as [rows][64 k] (128-B rows) and read with ds_read_b128;
// k-strided tiles as [64 k][128 rows] (256-B rows) and read with the gfx950 transposing
// ds_read_b64_tr_b16 — both LDS images XOR-swizzled to be bank-conflict-free for their reads AND the
// staging writes (tools/lds_banks.py).
//
// Tile 128x128x64, 256 threads = 4 waves (2x2, 64x64 per wave = 2x2 MFMA 32x32 blocks), LDS double
// buffer (64 KiB) with register-staged global loads issued one K-tile ahead (T14: issue early, write
// late), one barrier per K-tile. XCD-aware bijective block->tile remap so the blocks that share an A
// row-panel run on the same XCD/L2 (cdna_hip_programming.md T1).
//
// Epilogues (bf16 outputs are written with m on the MFMA lane so each lane stores 4 consecutive n):
//   STORE, BIAS, BIAS_GELU (pre-activation + activation), BIAS_DROP_RES (dropout + residual: the
//   post-LN block input z), RES (dgrad + residual-gradient add), DGELU (dgrad × gelu'(pre-act)),
//   F32_ATOMIC (wgrad straight into the fp32 main_grad buffer; split-K partials add atomically —
//   n on the lane so every atomic wave instruction is two contiguous 128-B row segments).
#include "common.h"
#include <stdlib.h>

namespace hsd {

enum Epi : int { EPI_STORE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_BIAS_DROP_RES = 3, EPI_RES = 4, EPI_DGELU = 5,
                 EPI_F32_ATOMIC = 6 };

struct GemmParams {
  const bf16_t* A;
  int64_t lda;
  const bf16_t* B;
  int64_t ldb;
  int M, N, K;
  void* C;
  int64_t ldc;
  const bf16_t* bias;
  const bf16_t* aux;
  int64_t ldaux;
  bf16_t* C2;
  DropoutParams dp;
  int kps;      // K elements per split (multiple of 64)
  int tiles_m, tiles_n;
};

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_ELEMS = 128 * 64;  // one operand tile (either image)

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;

__device__ __forceinline__ int swz0(int row) {  // [rows][64] image: chunk ^ brev3((row>>1)&7)
  const int t = (row >> 1) & 7;
  return ((t & 1) << 2) | (t & 2) | ((t >> 2) & 1);
}
__device__ __forceinline__ int off0(int row, int chunk) { return row * 64 + ((chunk ^ swz0(row)) << 3); }
__device__ __forceinline__ int swz1(int krow) { return (((krow & 1) << 1) | ((krow >> 1) & 1)) << 2; }
template <int R = 128>
__device__ __forceinline__ int off1(int krow, int col) {  // [64 k][R] image, col = element column
  return krow * R + ((((col >> 3) ^ swz1(krow))) << 3) + (col & 7);
}

// fragment (8 consecutive-k bf16 for lane row r = lane&31, k = 16ks + 8h + j) of rows [rbase, rbase+32)
template <int L, int R = 128>
__device__ __forceinline__ bf16x8 frag(const bf16_t* tile, int rbase, int ks, int lane) {
  if constexpr (L == 0) {
    const int r = lane & 31, h = lane >> 5;
    return *reinterpret_cast<const bf16x8*>(tile + off0(rbase + r, 2 * ks + h));
  } else {
    const int g = lane >> 4, i = lane & 15, h = g >> 1, q = i >> 2, p = i & 3;
    const int col = rbase + 16 * (g & 1) + 4 * p;
    const int k0 = 16 * ks + 8 * h + q;
    bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4_t*)(tile + off1<R>(k0, col)));
    bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4_t*)(tile + off1<R>(k0 + 4, col)));
    bf16x8 r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  }
}

// stage one operand tile: rows [r0, r0+128) x k [k0, k0+64) of a matrix with `R` rows, k < kend
template <int L>
__device__ __forceinline__ void gload(u32x4 (&st)[4], const bf16_t* __restrict__ X, int64_t ld, int r0, int R, int k0,
                                      int kend, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    int row, kk;
    if constexpr (L == 0) {
      row = c >> 3;
      kk = (c & 7) * 8;
      const bool ok = (r0 + row < R) && (k0 + kk < kend);
      st[i] = ok ? *reinterpret_cast<const u32x4*>(X + (int64_t)(r0 + row) * ld + k0 + kk) : u32x4{0, 0, 0, 0};
    } else {
      kk = c >> 4;
      row = (c & 15) * 8;
      const bool ok = (k0 + kk < kend) && (r0 + row < R);
      st[i] = ok ? *reinterpret_cast<const u32x4*>(X + (int64_t)(k0 + kk) * ld + r0 + row) : u32x4{0, 0, 0, 0};
    }
  }
}

template <int L>
__device__ __forceinline__ void swrite(bf16_t* tile, const u32x4 (&st)[4], int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    if constexpr (L == 0) {
      *reinterpret_cast<u32x4*>(tile + off0(c >> 3, c & 7)) = st[i];
    } else {
      *reinterpret_cast<u32x4*>(tile + off1(c >> 4, (c & 15) * 8)) = st[i];
    }
  }
}


// One 32x32 accumulator block. SWAP: D[n][m] (m on the lane, regs walk n); else D[m][n] (n on the lane).
template <int EPI, bool SWAP>
__device__ __forceinline__ void epi_block(const f32x16& a, int mb, int nb, int lane, const GemmParams& p) {
  const int r = lane & 31, h = lane >> 5;
  if constexpr (!SWAP) {
    float* C = reinterpret_cast<float*>(p.C);
    const int n = nb + r;
    if (n >= p.N) return;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int m = mb + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (m < p.M) atomicAdd(C + (int64_t)m * p.ldc + n, a[reg]);
    }
  } else {
    bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
    const int m = mb + r;
    if (m >= p.M) return;
    constexpr bool kBias = EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_DROP_RES;
    constexpr bool kAux = EPI == EPI_BIAS_DROP_RES || EPI == EPI_RES || EPI == EPI_DGELU;
    // phase 1: issue every load of the block (bias / residual / pre-activation) before any store
    u32x2 bw[4], xw[4];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const int n = min(nb + 8 * q4 + 4 * h, p.N - 4);
      if constexpr (kBias) bw[q4] = *reinterpret_cast<const u32x2*>(p.bias + n);
      if constexpr (kAux) xw[q4] = *reinterpret_cast<const u32x2*>(p.aux + (int64_t)m * p.ldaux + n);
    }
    // phase 2: math + stores
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const int n = nb + 8 * q4 + 4 * h;
      if (n >= p.N) continue;
      float v[4] = {a[4 * q4], a[4 * q4 + 1], a[4 * q4 + 2], a[4 * q4 + 3]};
      const int64_t co = (int64_t)m * p.ldc + n;
      if constexpr (kBias) {
        v[0] += lo_bf(bw[q4].x); v[1] += hi_bf(bw[q4].x); v[2] += lo_bf(bw[q4].y); v[3] += hi_bf(bw[q4].y);
      }
      u32x2 o;
      if constexpr (EPI == EPI_BIAS_GELU) {
        o.x = pack_bf2(v[0], v[1]);
        o.y = pack_bf2(v[2], v[3]);
        *reinterpret_cast<u32x2*>(C + co) = o;  // pre-activation (saved for backward)
        u32x2 g;
        g.x = pack_bf2(gelu_erf(lo_bf(o.x)), gelu_erf(hi_bf(o.x)));
        g.y = pack_bf2(gelu_erf(lo_bf(o.y)), gelu_erf(hi_bf(o.y)));
        *reinterpret_cast<u32x2*>(p.C2 + co) = g;
        continue;
      } else if constexpr (EPI == EPI_BIAS_DROP_RES) {
        // y = bf16(acc + b); z = bf16(y * keep * scale + residual): ONE rounding of the sum, exactly as gemm2 / gemm8's
        // E2_BIAS_DROP_RES (gemm_common.h epi_chunk), so a dropout + residual site gives the same bits on every path
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = bf2f(f2bf(v[e]));
        if (p.dp.enabled) {
          uint32_t b0, b1;
          dropout_bits4((uint32_t)m, (uint32_t)n, p.dp, b0, b1);  // mask row m of width N, n % 4 == 0
          v[0] = __builtin_fmaf(v[0], keep_factor(b0, 0, p.dp), lo_bf(xw[q4].x));
          v[1] = __builtin_fmaf(v[1], keep_factor(b0, 1, p.dp), hi_bf(xw[q4].x));
          v[2] = __builtin_fmaf(v[2], keep_factor(b1, 0, p.dp), lo_bf(xw[q4].y));
          v[3] = __builtin_fmaf(v[3], keep_factor(b1, 1, p.dp), hi_bf(xw[q4].y));
        } else {
          v[0] += lo_bf(xw[q4].x); v[1] += hi_bf(xw[q4].x); v[2] += lo_bf(xw[q4].y); v[3] += hi_bf(xw[q4].y);
        }
      } else if constexpr (EPI == EPI_RES) {
        v[0] += lo_bf(xw[q4].x); v[1] += hi_bf(xw[q4].x); v[2] += lo_bf(xw[q4].y); v[3] += hi_bf(xw[q4].y);
      } else if constexpr (EPI == EPI_DGELU) {
        v[0] = bf2f(f2bf(v[0])) * gelu_erf_grad(lo_bf(xw[q4].x));
        v[1] = bf2f(f2bf(v[1])) * gelu_erf_grad(hi_bf(xw[q4].x));
        v[2] = bf2f(f2bf(v[2])) * gelu_erf_grad(lo_bf(xw[q4].y));
        v[3] = bf2f(f2bf(v[3])) * gelu_erf_grad(hi_bf(xw[q4].y));
      }
      o.x = pack_bf2(v[0], v[1]);
      o.y = pack_bf2(v[2], v[3]);
      *reinterpret_cast<u32x2*>(C + co) = o;
    }
  }
}

// ================================================================================================
// v2 main loop: direct global->LDS DMA (global_load_lds_dwordx4, 1 KiB per wave instruction, swizzle
// applied on the SOURCE address so the LDS image stays lane-linear — cdna_hip_programming.md rule 21),
// 8 waves, BMxBNx64 tiles, 2 LDS stages, next stage's DMA in flight across the raw s_barrier with a
// counted vmcnt (never a drain to 0 inside the loop).
template <int L, int R>
__device__ __forceinline__ void dma_tile(bf16_t* tile, const bf16_t* __restrict__ X, int64_t ld, int r0, int Rmax,
                                         int k0, int wave, int lane) {
  constexpr int PER_WAVE = R / 64;  // 1-KiB instructions per wave
#pragma unroll
  for (int j = 0; j < PER_WAVE; ++j) {
    const int g = wave * PER_WAVE + j;
    int row, lc;
    const bf16_t* src;
    if constexpr (L == 0) {  // [R rows][64 k], 8 rows per KiB
      row = g * 8 + (lane >> 3);
      lc = (lane & 7) ^ swz0(row);
      const int rr = min(r0 + row, Rmax - 1);
      src = X + (int64_t)rr * ld + k0 + lc * 8;
    } else {  // [64 k][R cols], 512/R k-rows per KiB
      constexpr int RPK = 512 / R;
      row = g * RPK + (lane * 8) / R;
      const int pc = ((lane * 8) % R) >> 3;
      lc = pc ^ swz1(row);
      const int cc = min(r0 + lc * 8, Rmax - 8);
      src = X + (int64_t)(k0 + row) * ld + cc;
    }
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(tile + g * 512), 16, 0, 0);
  }
}

// piece j (0..R/64-1) of this wave's share of one operand tile
template <int L, int R, int NWV = 8>
__device__ __forceinline__ void dma_piece(int j, bf16_t* tile, const bf16_t* __restrict__ X, int64_t ld, int r0,
                                          int Rmax, int k0, int wave, int lane) {
  constexpr int PER_WAVE = R / 8 / NWV;  // R/8 one-KiB pieces per tile
  const int g = wave * PER_WAVE + j;
  const bf16_t* src;
  if constexpr (L == 0) {
    const int row = g * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ swz0(row);
    const int rr = min(r0 + row, Rmax - 1);
    src = X + (int64_t)rr * ld + k0 + lc * 8;
  } else {
    constexpr int RPK = 512 / R;
    const int row = g * RPK + (lane * 8) / R;
    const int pc = ((lane * 8) % R) >> 3;
    const int lc = pc ^ swz1(row);
    const int cc = min(r0 + lc * 8, Rmax - 8);
    src = X + (int64_t)(k0 + row) * ld + cc;
  }
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)(tile + g * 512), 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int LA, int LB, int EPI, int BM_, int BN_, int WM, int WN, int NS>
__global__ __launch_bounds__(512, 1) void gemm_dma_kernel(GemmParams p) {
  p.dp = resolve_seed(p.dp);
  constexpr bool SWAP = EPI != EPI_F32_ATOMIC;
  constexpr int TA = BM_ * 64, TB = BN_ * 64, STAGE = TA + TB;
  constexpr int MB = BM_ / WM / 32, NB = BN_ / WN / 32;
  constexpr int G = BM_ / 64 + BN_ / 64;  // DMA instructions per wave per stage
  static_assert(WM * WN == 8, "8 waves");
  static_assert(LA == 0 || BM_ == 128 || BM_ == 256, "k-strided tiles are 128 or 256 wide");
  static_assert(LB == 0 || BN_ == 128 || BN_ == 256, "k-strided tiles are 128 or 256 wide");
  static_assert(NS >= 2 && NS <= 4, "2..4 LDS stages");
  __shared__ __attribute__((aligned(16))) bf16_t smem[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;

  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tm = wg / p.tiles_n, tn = wg % p.tiles_n;
  const int m0 = tm * BM_, n0 = tn * BN_;
  const int kbeg = blockIdx.y * p.kps;
  const int kend = min(p.K, kbeg + p.kps);
  const int nt = (kend - kbeg) / BK;

  f32x16 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x16{};

  // prologue: NS-1 stages in flight
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) {
    if (s < nt) {
      dma_tile<LA, BM_>(smem + s * STAGE, p.A, p.lda, m0, p.M, kbeg + s * BK, wave, lane);
      dma_tile<LB, BN_>(smem + s * STAGE + TA, p.B, p.ldb, n0, p.N, kbeg + s * BK, wave, lane);
    }
  }
  // Main loop, ONE barrier per K-tile: at the top of iteration t the outstanding DMA stages are
  // t .. t+NS-2; wait until stage t landed (counted vmcnt), barrier (stage t visible to every wave AND
  // every wave finished reading stage t-1, whose buffer stage t+NS-1 now overwrites), then compute
  // stage t while the DMA pieces of stage t+NS-1 are issued between the MFMA groups.
  constexpr int GA = BM_ / 64;
  int slot = 0;
  for (int t = 0; t < nt; ++t) {
    const int newer = min(NS - 2, nt - 1 - t);  // stages issued after t and still possibly in flight
    if constexpr (NS >= 4) { if (newer == 2) wait_vmcnt<2 * G>(); }
    if constexpr (NS >= 3) { if (newer == 1) wait_vmcnt<G>(); }
    if (newer == 0) wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    const int ahead = t + NS - 1;
    const bool issue = ahead < nt;
    int nslot = slot + NS - 1;
    nslot = nslot >= NS ? nslot - NS : nslot;
    bf16_t* nA = smem + nslot * STAGE;
    const int kn = kbeg + ahead * BK;
    const bf16_t* tA = smem + slot * STAGE;
    const bf16_t* tB = tA + TA;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 fa[MB], fb[NB];
#pragma unroll
      for (int i = 0; i < MB; ++i) fa[i] = frag<LA, BM_>(tA, wm * (BM_ / WM) + 32 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < NB; ++j) fb[j] = frag<LB, BN_>(tB, wn * (BN_ / WN) + 32 * j, ks, lane);
      if (issue) {
#pragma unroll
        for (int j = 0; j < G; ++j) {
          if ((j * 4) / G == ks) {
            if (j < GA) dma_piece<LA, BM_>(j, nA, p.A, p.lda, m0, p.M, kn, wave, lane);
            else dma_piece<LB, BN_>(j - GA, nA + TA, p.B, p.ldb, n0, p.N, kn, wave, lane);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          if constexpr (SWAP) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
          else acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
    }
    slot = slot + 1 == NS ? 0 : slot + 1;
  }
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
      epi_block<EPI, SWAP>(acc[i][j], m0 + wm * (BM_ / WM) + 32 * i, n0 + wn * (BN_ / WN) + 32 * j, lane, p);
}

template <int LA, int LB, int EPI, int BM_, int BN_, int WM, int WN, int NS = 2>
static void gemm_dma_launch(const GemmParams& p0, int splits, hipStream_t st) {
  GemmParams p = p0;
  p.tiles_m = (p.M + BM_ - 1) / BM_;
  p.tiles_n = (p.N + BN_ - 1) / BN_;
  if (splits < 1) splits = 1;
  int kps = (p.K + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  splits = (p.K + kps - 1) / kps;
  p.kps = kps;
  dim3 grid(p.tiles_m * p.tiles_n, splits);
  hipLaunchKernelGGL((gemm_dma_kernel<LA, LB, EPI, BM_, BN_, WM, WN, NS>), grid, dim3(512), 0, st, p);
  HSD_CHECK_LAUNCH();
}

template <int LA, int LB, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_kernel(GemmParams p) {
  p.dp = resolve_seed(p.dp);
  constexpr bool SWAP = EPI != EPI_F32_ATOMIC;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * 2 * TILE_ELEMS];  // [stage][A|B][tile]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // ---- XCD-aware bijective remap of the flat tile index (split index = blockIdx.y)
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tm = wg / p.tiles_n, tn = wg % p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.y * p.kps;
  const int kend = min(p.K, kbeg + p.kps);
  const int nt = (kend - kbeg + BK - 1) / BK;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  u32x4 sa[4], sb[4];
  gload<LA>(sa, p.A, p.lda, m0, p.M, kbeg, kend, tid);
  gload<LB>(sb, p.B, p.ldb, n0, p.N, kbeg, kend, tid);
  swrite<LA>(smem, sa, tid);
  swrite<LB>(smem + TILE_ELEMS, sb, tid);
  __syncthreads();

  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < nt;
    if (more) {
      gload<LA>(sa, p.A, p.lda, m0, p.M, kbeg + (t + 1) * BK, kend, tid);
      gload<LB>(sb, p.B, p.ldb, n0, p.N, kbeg + (t + 1) * BK, kend, tid);
    }
    const bf16_t* tA = smem + cur * 2 * TILE_ELEMS;
    const bf16_t* tB = tA + TILE_ELEMS;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 fa0 = frag<LA>(tA, wm * 64, ks, lane);
      bf16x8 fa1 = frag<LA>(tA, wm * 64 + 32, ks, lane);
      bf16x8 fb0 = frag<LB>(tB, wn * 64, ks, lane);
      bf16x8 fb1 = frag<LB>(tB, wn * 64 + 32, ks, lane);
      if constexpr (SWAP) {  // D[n][m]: m on the lane
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb0, fa0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb0, fa1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb1, fa0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb1, fa1, acc[1][1], 0, 0, 0);
      } else {  // D[m][n]: n on the lane
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa0, fb0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa0, fb1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa1, fb0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa1, fb1, acc[1][1], 0, 0, 0);
      }
    }
    if (more) {
      bf16_t* nA = smem + (cur ^ 1) * 2 * TILE_ELEMS;
      swrite<LA>(nA, sa, tid);
      swrite<LB>(nA + TILE_ELEMS, sb, tid);
    }
    __syncthreads();
  }

  // ------------------------------------------------------------------ epilogue
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if constexpr (SWAP) epi_block<EPI, true>(acc[i][j], m0 + wm * 64 + 32 * j, n0 + wn * 64 + 32 * i, lane, p);
      else epi_block<EPI, false>(acc[i][j], m0 + wm * 64 + 32 * i, n0 + wn * 64 + 32 * j, lane, p);
    }
}

template <int LA, int LB, int EPI>
static void gemm_launch(const GemmParams& p0, int splits, hipStream_t st) {
  GemmParams p = p0;
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (p.N + BN - 1) / BN;
  if (splits < 1) splits = 1;
  int kps = (p.K + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  splits = (p.K + kps - 1) / kps;
  p.kps = kps;
  dim3 grid(p.tiles_m * p.tiles_n, splits);
  hipLaunchKernelGGL((gemm_kernel<LA, LB, EPI>), grid, dim3(256), 0, st, p);
  HSD_CHECK_LAUNCH();
}


// Public entry: layouts + epilogue chosen at run time.
void launch_gemm(int la, int lb, int epi, const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, int M, int N,
                 int K, void* C, int64_t ldc, const bf16_t* bias, const bf16_t* aux, int64_t ldaux, bf16_t* C2,
                 double p_drop, uint64_t seed, int splits, hipStream_t st) {
  GemmParams p{};
  p.A = A; p.lda = lda; p.B = B; p.ldb = ldb; p.M = M; p.N = N; p.K = K; p.C = C; p.ldc = ldc;
  p.bias = bias; p.aux = aux; p.ldaux = ldaux; p.C2 = C2;
  p.dp = make_dropout(p_drop, seed);
  // the v2 (LDS-DMA) kernel where the shape tiles it; the v1 register-staged kernel for the rest (K % 64, tiny M / N)
  const bool dma = (K % 64 == 0) && (M >= 128) && (N >= 128);
  if (dma) {
    if (epi == EPI_F32_ATOMIC) {
      if (la == 1 && lb == 1) { gemm_dma_launch<1, 1, EPI_F32_ATOMIC, 256, 128, 4, 2>(p, splits, st); return; }
      if (la == 0 && lb == 0) { gemm_dma_launch<0, 0, EPI_F32_ATOMIC, 256, 128, 4, 2>(p, splits, st); return; }
      if (la == 0 && lb == 1) { gemm_dma_launch<0, 1, EPI_F32_ATOMIC, 256, 128, 4, 2>(p, splits, st); return; }
    } else if (la == 0 && lb == 0) {
      switch (epi) {
        case EPI_STORE: gemm_dma_launch<0, 0, EPI_STORE, 256, 192, 4, 2>(p, 1, st); return;
        case EPI_BIAS: gemm_dma_launch<0, 0, EPI_BIAS, 256, 192, 4, 2>(p, 1, st); return;
        case EPI_BIAS_GELU: gemm_dma_launch<0, 0, EPI_BIAS_GELU, 256, 192, 4, 2>(p, 1, st); return;
        case EPI_BIAS_DROP_RES: gemm_dma_launch<0, 0, EPI_BIAS_DROP_RES, 256, 192, 4, 2>(p, 1, st); return;
        default: break;
      }
    } else if (la == 0 && lb == 1) {
      switch (epi) {
        case EPI_STORE: gemm_dma_launch<0, 1, EPI_STORE, 256, 128, 4, 2>(p, 1, st); return;
        case EPI_RES: gemm_dma_launch<0, 1, EPI_RES, 256, 128, 4, 2>(p, 1, st); return;
        case EPI_DGELU: gemm_dma_launch<0, 1, EPI_DGELU, 256, 128, 4, 2>(p, 1, st); return;
        default: break;
      }
    }
  }
  if (epi == EPI_F32_ATOMIC) {
    if (la == 1 && lb == 1) gemm_launch<1, 1, EPI_F32_ATOMIC>(p, splits, st);
    else if (la == 0 && lb == 0) gemm_launch<0, 0, EPI_F32_ATOMIC>(p, splits, st);
    else if (la == 0 && lb == 1) gemm_launch<0, 1, EPI_F32_ATOMIC>(p, splits, st);
    else abort();
    return;
  }
  if (la == 0 && lb == 0) {
    switch (epi) {
      case EPI_STORE: gemm_launch<0, 0, EPI_STORE>(p, 1, st); break;
      case EPI_BIAS: gemm_launch<0, 0, EPI_BIAS>(p, 1, st); break;
      case EPI_BIAS_GELU: gemm_launch<0, 0, EPI_BIAS_GELU>(p, 1, st); break;
      case EPI_BIAS_DROP_RES: gemm_launch<0, 0, EPI_BIAS_DROP_RES>(p, 1, st); break;
      default: abort();
    }
  } else if (la == 0 && lb == 1) {
    switch (epi) {
      case EPI_STORE: gemm_launch<0, 1, EPI_STORE>(p, 1, st); break;
      case EPI_RES: gemm_launch<0, 1, EPI_RES>(p, 1, st); break;
      case EPI_DGELU: gemm_launch<0, 1, EPI_DGELU>(p, 1, st); break;
      default: abort();
    }
  } else {
    abort();
  }
}

}  // namespace hsd
