// fp8 MFMA GEMM for the NT products (forward Y = X·Wᵀ, dgrad dX = dY·W with Wᵀ stored), SURVEY.md §2.10
// K19 / BASELINE.json config "roberta-large MLM ... fp8 weights (CDNA4 fp8 MFMA path)":
//
//   C[m][n] = epilogue( sa·sb · Σ_k A8(m,k) · B8(n,k) )     A8 [M][K], B8 [N][K] fp8 (OCP e4m3 / e5m2)
//
// This file holds the host side: shape support and the launch. The kernel is gemm2.hip's persistent
// staggered-schedule gemm8pk_kernel (v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales: twice the bf16 MFMA
// rate; a K-tile of 128 fp8 values is the same 128-B row as gemm2's 64 bf16 values, so it shares gemm2's swizzled
// LDS images, tiles, XCD-aware grid and bf16 epilogues, gemm_common.h). The round-2 one-barrier kernel that used to
// live here as an A/B reference (HSD_G8_LEGACY) is gone; tests/test_gpu_fp8.py checks the kernel against the fp32
// product of the dequantised operands instead.
// sa / sb are device scalars (1 / quantisation scale of each operand, fp8.hip): no host round trip.
#include "gemm_common.h"
#include <stdlib.h>

namespace hsd {

constexpr int kG8BK = 128;  // fp8 elements (bytes) per K-tile row

int gemm2_pick_bn(int M, int N);
void launch_gemm8pk(int epi, int bn, const G2Params& p, int fa, const float* sa, const float* sb, hipStream_t st);

bool gemm8_supported(int epi, int M, int N, int K) {
  if (epi == E2_STORE_RDOT && N % 256) return false;  // 256-wide tiles: one 64-column head per 8-lane group
  return K % kG8BK == 0 && M >= 1 && N % 8 == 0 && epi_bf16_out(epi) && gemm2_pick_bn(M, N) != 0;
}

// A8 [M][K] (lda), B8 [N][K] (ldb) fp8; fa / fb: 0 = e4m3, 1 = e5m2; sa / sb: device dequant scalars.
void launch_gemm8(int epi, const uint8_t* A, int64_t lda, int fa, const float* sa, const uint8_t* B, int64_t ldb,
                  int fb, const float* sb, int M, int N, int K, bf16_t* C, int64_t ldc, const bf16_t* bias,
                  const bf16_t* aux, int64_t ldaux, bf16_t* C2, double p_drop, uint64_t seed, float* dbias,
                  hipStream_t st, uint8_t* q8, const float* q8_amax, float* q8_sinv, float* q8_track, int q8_fmt,
                  float* rd, int rd_seq, int q8_only) {
  if (!gemm8_supported(epi, M, N, K)) abort();
  // the kernel's LDS-DMA reads 2-B aligned rows (every fp8 operand of the step: [rows][K] with K % 128 == 0)
  if (lda % 2 || ldb % 2) abort();
  G2Params p{};
  p.rd = rd;
  p.rd_seq = rd_seq;
  if (epi == E2_STORE_RDOT && (rd == nullptr || rd_seq <= 0 || M % rd_seq)) abort();
  p.q8 = q8; p.q8_amax = q8_amax; p.q8_sinv = q8_sinv; p.q8_track = q8_track; p.q8_fmt = q8_fmt;
  p.q8_only = q8 != nullptr && q8_only;
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
  launch_gemm8pk(epi, bn, p, fa, sa, sb, st);
}

}  // namespace hsd
