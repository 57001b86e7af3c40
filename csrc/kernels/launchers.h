// Host-side launch functions of the gfx950 kernels (implemented in csrc/kernels/*.hip).
// Every launcher is stream-ordered and allocation-free, so callers may capture it into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hsd {
typedef uint16_t bf16_t;
struct DropoutParams;

// adam.hip
void launch_adam(float* p, float* m, float* v, void* g, bool grad_bf16, bf16_t* out_bf16,
                 const uint8_t* decay, int64_t n, float step, float eps, float b1, float b2, float gscale,
                 float lr_wd, const float* coef, hipStream_t stream,
                 bf16_t* out_lo = nullptr, bool zero_grad = false);

}  // namespace hsd

namespace hsd {
// layernorm.hip
void launch_ln_fwd(const bf16_t* y, const bf16_t* res, const bf16_t* gamma, const bf16_t* beta, bf16_t* z,
                   bf16_t* out, float* mean, float* rstd, int rows, int H, float eps, double p, uint64_t seed,
                   hipStream_t st);
void launch_ln_fwd_q8(const bf16_t* y, const bf16_t* gamma, const bf16_t* beta, bf16_t* out, float* mean, float* rstd,
                      int rows, int H, float eps, uint8_t* q8, const float* amax_in, float* sinv, float* amax_track,
                      hipStream_t st);
void launch_ln_bwd_q8(const bf16_t* dout, const bf16_t* z, const float* mean, const float* rstd, const bf16_t* gamma,
                      bf16_t* dz, bf16_t* dy, const bf16_t* dres_add, float* dgamma, float* dbeta, float* dbias,
                      int rows, int H, double p, uint64_t seed, uint8_t* q8, const float* amax_in, float* sinv,
                      float* amax_track, int qfmt, hipStream_t st, bool q8_only = false);
void launch_ln_bwd(const bf16_t* dout, const bf16_t* z, const float* mean, const float* rstd, const bf16_t* gamma,
                   bf16_t* dz, bf16_t* dy, const bf16_t* dres_add, float* dgamma, float* dbeta, float* dbias,
                   int rows, int H, double p, uint64_t seed, hipStream_t st);
// embedding.hip
void launch_embed_fwd(const int64_t* ids, const int64_t* pos_ids, const int64_t* type_ids, const bf16_t* word,
                      const bf16_t* pos, const bf16_t* type, const bf16_t* gamma, const bf16_t* beta, bf16_t* out,
                      float* mean, float* rstd, int rows, int H, float eps, double p, uint64_t seed, hipStream_t st,
                      uint8_t* q8 = nullptr, const float* amax_in = nullptr, float* sinv = nullptr,
                      float* amax_track = nullptr);  // q8: the output's fp8 copy (as launch_ln_fwd_q8)
void launch_embed_bwd(const bf16_t* dout, const int64_t* ids, const int64_t* pos_ids, const int64_t* type_ids,
                      const bf16_t* word, const bf16_t* pos, const bf16_t* type, const bf16_t* gamma,
                      const float* mean, const float* rstd, float* gword, float* gpos, float* gtype, float* ggamma,
                      float* gbeta, int B, int S, int H, int pos_is_arange, double p, uint64_t seed, hipStream_t st);
// elementwise.hip
void launch_gelu_fwd(const bf16_t* y, bf16_t* g, int64_t n, hipStream_t st);
void launch_gelu_bwd_colsum(const bf16_t* dg, const bf16_t* y, bf16_t* da, float* dbias, int rows, int N,
                            hipStream_t st);
void launch_colsum(const bf16_t* x, float* dbias, int rows, int N, hipStream_t st);
// the 32 mask bits of column pair cp of row `row` of a dropout site with 64-bit `seed` (common.h), on the host
uint32_t dropout_pair_bits_host(uint64_t seed, uint32_t row, uint32_t cp);
void launch_dropout(const bf16_t* x, bf16_t* out, int64_t n, int W, double p, uint64_t seed, hipStream_t st);
void launch_mask_bias(const void* mask, bool i64, float* out, int64_t n, hipStream_t st);
// C[N][K] (fp32, ldc) += dy[T][N]ᵀ · x[T][K] for small T (K % 4 == 0)
void launch_small_wgrad(const bf16_t* dy, int64_t ldy, const bf16_t* x, int64_t ldx, float* C, int64_t ldc, int T,
                        int N, int K, hipStream_t st);
// xent.hip: fused softmax cross-entropy (+ gradient, + argmax-correct count); stats = {Σloss, correct}
void launch_xent(const void* logits, bool bf16, const int64_t* labels, void* dlogits, float* stats,
                 const float* n_valid, int rows, int V, int64_t ld, hipStream_t st);
// gradient wire casts (comm_engine 16-bit compression): to16: dst16 = src32 * scale; else dst32 = src16 * scale.
// half: fp16, else bf16. n % 4 == 0, 16-B aligned fp32 side.
void launch_wire_cast(const void* src, void* dst, int64_t n, bool to16, bool half, float scale, hipStream_t st);
// desc: int64 [n][5] = {src, dst, rows, cols, first_tile}; rows, cols multiples of 4
void launch_transpose_many(const int64_t* desc, int n, int total_tiles, hipStream_t st);
// cls_head.hip: fused sequence-classification head after the dense GEMM (act, dropout, classifier, CE, accuracy)
int cls_head_blocks(int R);
void launch_cls_head_fwd(const bf16_t* pre, int64_t ld_pre, const bf16_t* W2, const bf16_t* b2, const int64_t* labels,
                         bf16_t* t_out, bf16_t* logits, float* partials, float* stats, int R, int H, int C, int act,
                         double p, uint64_t seed, hipStream_t st);
void launch_cls_head_bwd(const bf16_t* t_in, const bf16_t* W2, const bf16_t* logits, const int64_t* labels,
                         const float* stats, const float* dloss, bf16_t* dpre, float* dW2, float* db2, int R, int H,
                         int C, int act, double p, uint64_t seed, hipStream_t st);
// attention.hip
bool attn_streaming(int S);
// kmask (optional, streaming S > 128 kernels: attn_keep_mask_supported): the forward writes its dropout keep bits
// ([B*heads][S/32][S] u32, attentionS.hip header), the backward reads them instead of re-hashing every (query, key) pair
bool attn_keep_mask_supported(int S);
int64_t attn_keep_mask_numel(int B, int S, int heads);
void launch_attn_fwd(const bf16_t* qkv, const float* mask, bf16_t* out, float* lse2, int B, int S, int heads,
                     double p, uint64_t seed, hipStream_t st, uint32_t* kmask = nullptr);
// attentionS.hip fp8 variants (S > 128 streaming kernels only: attn_streaming(S) && S > 128)
void launch_attnS_fwd_q8(const bf16_t* qkv, const float* mask, bf16_t* out, float* lse2, int B, int S, int heads,
                         double p, uint64_t seed, uint8_t* q8, const float* amax_in, float* sinv, float* amax_track,
                         hipStream_t st, uint32_t* kmask = nullptr);
void launch_attnS_bwd_q8(const bf16_t* qkv, const float* mask, const bf16_t* o, const bf16_t* dout, const float* lse2,
                         bf16_t* dqkv, float* delta_ws, float* dbias, int B, int S, int heads, double p, uint64_t seed,
                         uint8_t* q8, const float* amax_in, float* sinv, float* amax_track, int qfmt, hipStream_t st,
                         const uint32_t* kmask = nullptr, bool delta_ready = false, bool q8_only = false);
// dbias (optional): fp32 [3H] += column sums of dqkv (the fused QKV bias gradient)
void launch_attn_bwd(const bf16_t* qkv, const float* mask, const bf16_t* o, const bf16_t* dout, const float* lse2,
                     bf16_t* dqkv, float* dq_acc, float* dbias, int B, int S, int heads, double p, uint64_t seed,
                     hipStream_t st, const uint32_t* kmask = nullptr, bool delta_ready = false);
}  // namespace hsd

namespace hsd {
// gemm.hip — la: 0 A[M][K], 1 A[K][M];  lb: 0 B[N][K], 1 B[K][N];  epi: see gemm.hip Epi
void launch_gemm(int la, int lb, int epi, const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, int M, int N,
                 int K, void* C, int64_t ldc, const bf16_t* bias, const bf16_t* aux, int64_t ldaux, bf16_t* C2,
                 double p_drop, uint64_t seed, int splits, hipStream_t st);
// gemm2.hip — 256-row-tile 8-phase MFMA GEMM: (0,0) NT bf16 out with epilogues 0..5; (1,1) TT fp32 out
// (epi 6 = atomics, 7 = split-K slabs in `ws` [splits][M][N] + reduce into C)
// device step seed for dropout (common.h g_dropout_dev_seed); nullptr = off
void set_dropout_dev_seed(const uint32_t* p);
// HSD_* knobs are cached per generation (common.h HSD_KNOB); this re-reads them at their next use
void refresh_env_knobs();
// fp32.hip: the fp32 (reference precision) step -- split-product operands for the bf16 MFMA GEMMs, fp32 epilogues,
// LayerNorm, embeddings, streaming attention, classification head (ops/hip32.py)
void launch_split3(const float* x, bf16_t* out, int64_t R, int64_t C, int pat, bool rows, hipStream_t st,
                   bf16_t* out2 = nullptr, int pat2 = 0);
void launch_epi32(float* y, const float* bias, const float* aux, float* out, int64_t M, int N, int kind, double p,
                  uint64_t seed, hipStream_t st, bf16_t* hi = nullptr, bf16_t* lo = nullptr);
void launch_dropout32(const float* x, float* out, int64_t n, int W, double p, uint64_t seed, hipStream_t st,
                      bf16_t* hi = nullptr, bf16_t* lo = nullptr);
void launch_colsum32(const float* x, float* dbias, int M, int N, hipStream_t st);
void launch_ln32_fwd(const float* x, const float* g, const float* b, float* out, float* mean, float* rstd, int R,
                     int H, float eps, hipStream_t st, bf16_t* hi = nullptr, bf16_t* lo = nullptr);
void launch_ln32_bwd(const float* dy, const float* x, const float* mean, const float* rstd, const float* g, float* dx,
                     float* dg, float* db, int R, int H, hipStream_t st);
void launch_embed32_gather(const int64_t* ids, const int64_t* pids, const int64_t* tids, const float* word,
                           const float* pos, const float* type, float* x, int R, int H, hipStream_t st);
void launch_embed32_scatter(const float* dx, const int64_t* ids, const int64_t* pids, const int64_t* tids,
                            float* gword, float* gpos, float* gtype, int R, int H, hipStream_t st);
void launch_attn32_fwd(const float* qkv, const float* mask, float* out, float* lse, int B, int S, int heads, double p,
                       uint64_t seed, hipStream_t st);
void launch_attn32_bwd(const float* qkv, const float* mask, const float* o, const float* dout, const float* lse,
                       float* dqkv, float* delta, int B, int S, int heads, double p, uint64_t seed, hipStream_t st);
void launch_attn32_delta(const float* o, const float* dout, float* delta, int B, int S, int heads, hipStream_t st);
// fp32 attention on split bf16 MFMA products (attention32m.hip)
bool attn32m_supported(int S, int head_dim);
void launch_split2(const float* x, bf16_t* hi, bf16_t* lo, int64_t n, hipStream_t st);
void launch_attn32m_fwd(const bf16_t* qkv_hi, const bf16_t* qkv_lo, const float* mask, float* out, float* lse2, int B,
                        int S, int heads, double p, uint64_t seed, hipStream_t st);
void launch_attn32m_bwd(const bf16_t* qkv_hi, const bf16_t* qkv_lo, const bf16_t* do_hi, const bf16_t* do_lo,
                        const float* mask, const float* lse2, const float* delta, float* dqkv, int B, int S, int heads,
                        double p, uint64_t seed, hipStream_t st);
void launch_cls32_fwd(const float* pre, const float* W2, const float* b2, const int64_t* labels, float* t_out,
                      float* logits, float* stats, int R, int H, int C, int act, double p, uint64_t seed,
                      hipStream_t st);
void launch_cls32_bwd(const float* pre, const float* t_in, const float* W2, const float* logits,
                      const int64_t* labels, const float* dloss, float* dpre, float* dW2, float* db2, int R, int H,
                      int C, int act, double p, uint64_t seed, hipStream_t st);
// contention emulation: `blocks` workgroups holding one whole CU each (160 KiB LDS) for `usec` us
void launch_cu_hog(int blocks, double usec, hipStream_t st);

// fp8 (gemm8.hip / fp8.hip)
bool gemm8_supported(int epi, int M, int N, int K);
void launch_gemm8(int epi, const uint8_t* A, int64_t lda, int fa, const float* sa, const uint8_t* B, int64_t ldb,
                  int fb, const float* sb, int M, int N, int K, bf16_t* C, int64_t ldc, const bf16_t* bias,
                  const bf16_t* aux, int64_t ldaux, bf16_t* C2, double p_drop, uint64_t seed, float* dbias,
                  hipStream_t st, uint8_t* q8 = nullptr, const float* q8_amax = nullptr, float* q8_sinv = nullptr,
                  float* q8_track = nullptr, int q8_fmt = 0, float* rd = nullptr, int rd_seq = 0,
                  int q8_only = 0);
void launch_fp8_quant(const bf16_t* x, int64_t n, float* amax, uint8_t* q, float* sinv, int fmt, bool compute_amax,
                      float* amax_track, hipStream_t st);
void launch_fp8_quant_many(const int64_t* amax_desc, int n_amax, int amax_blocks, const int64_t* quant_desc,
                           int n_quant, int quant_blocks_total, float* amax, float* sinv, int fmt, hipStream_t st);
int fp8_elems_per_block();
void attn_set_force_generic(bool on);
// gemm2.hip: segmented-K fp32-output GEMMs over bf16 hi / lo operand halves (the fp32 step's split products)
bool gemm2_seg_supported(int la, int lb, int M, int N, int Kseg);
int64_t gemm2_seg_ws_numel(int la, int lb, int M, int N, int Kseg);
void launch_gemm2_seg(int la, int lb, const bf16_t* const A[3], int64_t lda, const bf16_t* const B[3], int64_t ldb,
                      int M, int N, int Kseg, float* C, int64_t ldc, float* ws, hipStream_t st, bool accumulate = false);  // tests: every S on the tiled generic attention kernels
void attn128_set_diag(void* p);  // diagnostic phase stamps of the S=128 attention backward ([B*heads][8] u64)
void gemm2_set_diag(void* p);  // diagnostic timestamps of the persistent NT kernel ([grid][64][4] u64), nullptr = off
void launch_gemm2(int la, int lb, int epi, const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, int M, int N,
                  int K, void* C, int64_t ldc, const bf16_t* bias, const bf16_t* aux, int64_t ldaux, bf16_t* C2,
                  double p_drop, uint64_t seed, int splits, float* ws, float* dbias, hipStream_t st,
                  float* rd = nullptr, int rd_seq = 0);
bool gemm2_supported(int la, int lb, int epi, int M, int N, int K);
int gemm2_wgrad_splits(int M, int N, int K);
int gemm2_f32nt_splits(int M, int N, int K);
// fp8 TT weight gradient (gemm2.hip gemm8tt_kernel + slab_reduce): C[M][N] (fp32) += sdy·sx · dY8ᵀ · X8
bool gemm8_wgrad_supported(int M, int N, int T);
int gemm8_wgrad_splits(int M, int N, int T);
int64_t gemm8_wgrad_ws_numel(int M, int N, int T, int splits);
void launch_gemm8_wgrad(const uint8_t* dy, int64_t ldd, int fdy, const float* sdy, const uint8_t* x, int64_t ldx,
                        int fx, const float* sx, int M, int N, int T, float* C, int64_t ldc, int splits, float* ws,
                        hipStream_t st);
int gemm2_nt_splits(int M, int N, int K);
}  // namespace hsd
