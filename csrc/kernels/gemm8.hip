// fp8 MFMA GEMM for the NT products (forward Y = X·Wᵀ, dgrad dX = dY·W with Wᵀ stored), SURVEY.md §2.10
// K19 / BASELINE.json config "roberta-large MLM ... fp8 weights (CDNA4 fp8 MFMA path)":
//
//   C[m][n] = epilogue( sa·sb · Σ_k A8(m,k) · B8(n,k) )     A8 [M][K], B8 [N][K] fp8 (OCP e4m3 / e5m2)
//
// v_mfma_f32_16x16x128_f8f6f4 (unit block scales): twice the bf16 MFMA rate, and a K-tile of 128 fp8
// values is the same 128-B row as gemm2's 64 bf16 values, so the LDS images (16-B chunk ^ (row>>1)&7,
// filled by global_load_lds with the swizzle on the source address), the tile shape (256 x BN, 8 waves
// as 2 x 4, wave tile 128 x BN/4), the one-barrier-per-K-tile schedule, the XCD-aware grid and the bf16
// epilogues (gemm_common.h) are gemm2's — each K-tile just carries twice the K. A lane's fragment is
// 32 consecutive k (two 16-B chunks) of one row; A and B use the same k assignment, so the product is
// independent of the instruction's internal k order.
// sa / sb are device scalars (1 / quantisation scale of each operand, fp8.hip): no host round trip.
#include "gemm_common.h"
#include <stdlib.h>

namespace hsd {
namespace g8 {

using g2::BM;
using g2::f1;
constexpr int BK = 128;  // fp8 elements (bytes) per K-tile row

typedef __attribute__((ext_vector_type(8))) int i32x8;

// one 1-KiB DMA wave instruction `g` of a [rows][128 B] image (8 rows x 8 chunks per instruction)
__device__ __forceinline__ void dma8(bf16_t* img, const uint8_t* __restrict__ X, int64_t ld, int r0, int Rmax, int k0,
                                     int g, int lane) {
  const int row = g * 8 + (lane >> 3);
  const int lc = (lane & 7) ^ f1(row);
  const int rr = min(r0 + row, Rmax - 1);
  const uint8_t* src = X + (int64_t)rr * ld + k0 + lc * 16;
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)(img + g * 512), 16, 0, 0);
}

// 16x16x128 fragment: lane l holds row rbase + (l&15), k = 32(l>>4) .. +31 (chunks 2(l>>4), 2(l>>4)+1)
__device__ __forceinline__ i32x8 frag8(const bf16_t* img, int rbase, int lane) {
  const int row = rbase + (lane & 15);
  const int c0 = 2 * (lane >> 4);
  const bf16_t* r = img + row * 64;
  const u32x4 lo = *reinterpret_cast<const u32x4*>(r + ((c0 ^ f1(row)) << 3));
  const u32x4 hi = *reinterpret_cast<const u32x4*>(r + (((c0 + 1) ^ f1(row)) << 3));
  i32x8 v;
  v[0] = (int)lo[0]; v[1] = (int)lo[1]; v[2] = (int)lo[2]; v[3] = (int)lo[3];
  v[4] = (int)hi[0]; v[5] = (int)hi[1]; v[6] = (int)hi[2]; v[7] = (int)hi[3];
  return v;
}

// FB / FA: formats of the B-matrix / A-matrix operands (0 = e4m3, 1 = e5m2); the B fragment is the
// instruction's first operand (D[n][m] orientation, as in gemm2)
template <int FB, int FA>
__device__ __forceinline__ f32x4 mma8(const i32x8& b, const i32x8& a, const f32x4& c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b, a, c, FB, FA, 0, 0, 0, 0);
}

template <int EPI, int BN, int FA, int FB>
__global__ __launch_bounds__(512, 1) void gemm8_kernel(G2Params p, const float* __restrict__ sa,
                                                       const float* __restrict__ sb) {
  p.dp = resolve_seed(p.dp);
  constexpr int WN = BN / 4;
  constexpr int NREP = WN / 16;
  constexpr int NB0 = 2;
  constexpr int NB1 = NREP - NB0;
  static_assert(NREP == 3 || NREP == 4, "BN 192 or 256");
  constexpr int TA = BM * 64, TB = BN * 64, STAGE = TA + TB;  // bf16 units (= 128 B rows)
  constexpr int GA = 4, GB = BN / 64, G = GA + GB;

  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const uint8_t* A8 = reinterpret_cast<const uint8_t*>(p.A);
  const uint8_t* B8 = reinterpret_cast<const uint8_t*>(p.B);

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tm = wg / p.tiles_n, tn = wg % p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nt = p.K / BK;
  HSD_DASSERT(wg < p.ntiles && m0 < p.M && n0 < p.N && p.K % BK == 0);

  auto dma_slot = [&](int q, bf16_t* stage, int k0) {
    if (q < GA) dma8(stage, A8, p.lda, m0, p.M, k0, wave * GA + q, lane);
    else dma8(stage + TA, B8, p.ldb, n0, p.N, k0, wave * GB + (q - GA), lane);
  };

  f32x4 acc[8][NREP];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NREP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int arow = wm * 128;
  const int bcol = wn * WN;
  i32x8 fa[4], fb0[NB0], fb1[NB1];
  // one barrier per K-tile (gemm2 SYNC 1): tile t+1's DMA goes into the other stage in two halves
#pragma unroll
  for (int q = 0; q < G; ++q) dma_slot(q, smem, 0);
  g2::vmcnt<0>();
  G2_BARRIER();
  for (int t = 0; t < nt; ++t) {
    const bf16_t* cA = smem + (t & 1) * STAGE;
    const bf16_t* cB = cA + TA;
    bf16_t* nS = smem + ((t + 1) & 1) * STAGE;
    const bool n1 = t + 1 < nt;
    const int k1 = (t + 1) * BK;
    if (n1) {
#pragma unroll
      for (int q = 0; q < G / 2; ++q) dma_slot(q, nS, k1);
    }
#pragma unroll
    for (int j = 0; j < NB0; ++j) fb0[j] = frag8(cB, bcol + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag8(cA, arow + 16 * i, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NB0; ++j) acc[i][j] = mma8<FB, FA>(fb0[j], fa[i], acc[i][j]);
    if (n1) {
#pragma unroll
      for (int q = G / 2; q < G; ++q) dma_slot(q, nS, k1);
    }
#pragma unroll
    for (int j = 0; j < NB1; ++j) fb1[j] = frag8(cB, bcol + 16 * (NB0 + j), lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NB1; ++j) acc[i][NB0 + j] = mma8<FB, FA>(fb1[j], fa[i], acc[i][NB0 + j]);
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag8(cA, arow + 64 + 16 * i, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < NB1; ++j) acc[4 + i][NB0 + j] = mma8<FB, FA>(fb1[j], fa[i], acc[4 + i][NB0 + j]);
#pragma unroll
      for (int j = 0; j < NB0; ++j) acc[4 + i][j] = mma8<FB, FA>(fb0[j], fa[i], acc[4 + i][j]);
    }
    g2::vmcnt<0>();
    G2_BARRIER();
  }

  // dequantise, then gemm2's bf16 epilogue
  const float s = sa[0] * sb[0];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NREP; ++j) acc[i][j] *= s;
  g2::epilogue_bf16<EPI, BN>(acc, p, smem, wave, lane, m0 + arow, n0 + bcol);
}

}  // namespace g8

int gemm2_pick_bn(int M, int N);
void launch_gemm8pk(int epi, int bn, const G2Params& p, int fa, const float* sa, const float* sb, hipStream_t st);

bool gemm8_supported(int epi, int M, int N, int K) {
  if (epi == E2_STORE_RDOT && N % 256) return false;  // 256-wide tiles: one 64-column head per 8-lane group
  return K % g8::BK == 0 && M >= 1 && N % 8 == 0 && epi_bf16_out(epi) && gemm2_pick_bn(M, N) != 0;
}

template <int EPI, int BN, int FA, int FB>
static void g8_launch(const G2Params& p0, const float* sa, const float* sb, hipStream_t st) {
  G2Params p = p0;
  const int tiles_m = (p.M + g2::BM - 1) / g2::BM;
  p.tiles_n = (p.N + BN - 1) / BN;
  p.kps = p.K;
  p.ntiles = tiles_m * p.tiles_n;
  hipLaunchKernelGGL((g8::gemm8_kernel<EPI, BN, FA, FB>), dim3(p.ntiles), dim3(512), 0, st, p, sa, sb);
  HSD_CHECK_LAUNCH();
}

// A8 [M][K] (lda), B8 [N][K] (ldb) fp8; fa / fb: 0 = e4m3, 1 = e5m2; sa / sb: device dequant scalars.
void launch_gemm8(int epi, const uint8_t* A, int64_t lda, int fa, const float* sa, const uint8_t* B, int64_t ldb,
                  int fb, const float* sb, int M, int N, int K, bf16_t* C, int64_t ldc, const bf16_t* bias,
                  const bf16_t* aux, int64_t ldaux, bf16_t* C2, double p_drop, uint64_t seed, float* dbias,
                  hipStream_t st, uint8_t* q8, const float* q8_amax, float* q8_sinv, float* q8_track, int q8_fmt,
                  float* rd, int rd_seq) {
  if (!gemm8_supported(epi, M, N, K)) abort();
  G2Params p{};
  p.rd = rd;
  p.rd_seq = rd_seq;
  if (epi == E2_STORE_RDOT && (rd == nullptr || rd_seq <= 0 || M % rd_seq || lda % 2 || ldb % 2)) abort();
  p.q8 = q8; p.q8_amax = q8_amax; p.q8_sinv = q8_sinv; p.q8_track = q8_track; p.q8_fmt = q8_fmt;
  p.A = reinterpret_cast<const bf16_t*>(A); p.lda = lda;
  p.B = reinterpret_cast<const bf16_t*>(B); p.ldb = ldb;
  p.M = M; p.N = N; p.K = K; p.C = C; p.ldc = ldc;
  p.bias = bias; p.aux = aux; p.ldaux = ldaux; p.C2 = C2;
  p.dp = make_dropout(p_drop, seed);
  p.dbias = dbias;
  int bn = epi == E2_STORE_RDOT ? 256 : gemm2_pick_bn(M, N);
  if (dbias != nullptr) {
    if ((epi != E2_DGELU && epi != E2_MUL) || N % 256) abort();
    bn = 256;
  }
  // formats: activations / weights e4m3, gradients (dgrad A operand) e4m3 or e5m2
  if (fb != 0) abort();
  // default: the persistent staggered-schedule kernel (gemm2.hip gemm8pk_kernel); HSD_G8_LEGACY=1: this file's
  // one-barrier-per-K-tile kernel (A/B reference)
  {
    if ((!HSD_KNOB("HSD_G8_LEGACY", 0) || epi == E2_STORE_RDOT) && lda % 2 == 0 && ldb % 2 == 0) {
      launch_gemm8pk(epi, bn, p, fa, sa, sb, st);
      return;
    }
  }
  if (q8 != nullptr) abort();  // fp8 output copies: persistent kernel only
#define G8_E(E)                                                              \
  case E:                                                                    \
    if (bn == 256) {                                                         \
      if (fa == 0) g8_launch<E, 256, 0, 0>(p, sa, sb, st);                   \
      else g8_launch<E, 256, 1, 0>(p, sa, sb, st);                           \
    } else {                                                                 \
      if (fa == 0) g8_launch<E, 192, 0, 0>(p, sa, sb, st);                   \
      else g8_launch<E, 192, 1, 0>(p, sa, sb, st);                           \
    }                                                                        \
    return;
  switch (epi) {
    G8_E(E2_STORE)
    G8_E(E2_BIAS)
    G8_E(E2_BIAS_GELU)
    G8_E(E2_BIAS_DROP_RES)
    G8_E(E2_RES)
    G8_E(E2_DGELU)
    G8_E(E2_BIAS_GELU_D)
    G8_E(E2_MUL)
    default: abort();
  }
#undef G8_E
}

}  // namespace hsd
