// Fused sequence-classification head (SURVEY.md §2.10 K15 + K16): everything after the pooler / pre-classifier
// dense GEMM, in one forward and one backward kernel.
//
//   reference: scripts/train.py:117-118 — TFAutoModelForSequenceClassification's head + SparseCategoricalCrossentropy
//   (from_logits), SparseCategoricalAccuracy; HF modeling_bert.py BertPooler (tanh) -> dropout -> classifier,
//   RobertaClassificationHead (tanh), DistilBERT pre_classifier (relu).
//
//   forward   t       = act(pre)                      pre = x·W1ᵀ + b1 (gemm2, bias epilogue), act = tanh | relu
//             d       = bf16(t · keep · 1/(1-p))      the hash dropout of ops/rng.py (element e = row·H + h)
//             logits  = bf16(d·W2ᵀ + b2)              C <= 4 classes: a per-row GEMV, reduced across the wave
//             loss    = mean over rows with label != -100 of (logsumexp(logits) - logits[label]); correct = argmax hits
//   backward  g       = (softmax(logits) - onehot(label)) · dloss / n_valid         (0 on ignored rows)
//             dpre    = (g·W2 · keep · 1/(1-p)) · act'(t)          bf16, feeds the dense layer's dgrad / wgrad / colsum
//             dW2    += gᵀ·d,  db2 += Σ g                          fp32 straight into main_grad (one atomic per element
//                                                                  per 16-row block)
//
// One wave per row; lanes own 8-element (16-B) chunks of the row, chunk c = lane + 64·i. Block = 4 waves x 4 rows.
// The forward writes per-block partial sums {loss, correct, n_valid}; cls_stats_kernel (one block) reduces them
// into stats = {mean loss, correct, n_valid, loss sum} — no memset, no atomics, deterministic.
#include "common.h"
#include "launchers.h"

namespace hsd {
namespace cls {

constexpr int ROWS_PER_WAVE = 4;
constexpr int ROWS_PER_BLOCK = 4 * ROWS_PER_WAVE;
constexpr int MAXC = 4;
constexpr int MAX_CHUNKS = 2;  // H <= 1024 (8 elements x 64 lanes x 2)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float act_fwd(float x, int act) { return act == 0 ? tanhf(x) : fmaxf(x, 0.0f); }

// act'(.) from the stored activation t: tanh' = 1 - t², relu' = [t > 0]
__device__ __forceinline__ float act_bwd(float t, int act) { return act == 0 ? 1.0f - t * t : (t > 0.0f ? 1.0f : 0.0f); }

__device__ __forceinline__ void unpack8(const u32x4& w, float (&v)[8]) {
  v[0] = lo_bf(w.x); v[1] = hi_bf(w.x); v[2] = lo_bf(w.y); v[3] = hi_bf(w.y);
  v[4] = lo_bf(w.z); v[5] = hi_bf(w.z); v[6] = lo_bf(w.w); v[7] = hi_bf(w.w);
}

__device__ __forceinline__ u32x4 pack8(const float (&v)[8]) {
  return u32x4{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7])};
}

// keep factors of the 8 elements from column h0 (h0 % 8 == 0) of row `row` ([R][H] site, mask rows of width H)
__device__ __forceinline__ void keep8(int row, int h0, const DropoutParams& dp, float (&kf)[8]) {
  const uint32_t x = dropout_row((uint32_t)row, dp) ^ drop_col((uint32_t)h0 >> 1);
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // (h0 / 2) % 4 == 0: pair h0 / 2 + j = h0 / 2 ^ j
    const uint32_t b = drop_fin(x ^ drop_col((uint32_t)j));
    kf[2 * j] = keep_factor(b, 0, dp);
    kf[2 * j + 1] = keep_factor(b, 1, dp);
  }
}

template <int C>
__global__ __launch_bounds__(256) void cls_fwd_kernel(const bf16_t* __restrict__ pre, int64_t ld_pre,
                                                      const bf16_t* __restrict__ W2, const bf16_t* __restrict__ b2,
                                                      const int64_t* __restrict__ labels, bf16_t* __restrict__ t_out,
                                                      bf16_t* __restrict__ logits, float* __restrict__ partials, int R,
                                                      int H, int act, DropoutParams dp) {
  dp = resolve_seed(dp);
  __shared__ float red[4][3];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = H >> 3;
  float loss_sum = 0.f, correct = 0.f, nvalid = 0.f;
  for (int rr = 0; rr < ROWS_PER_WAVE; ++rr) {
    const int row = blockIdx.x * ROWS_PER_BLOCK + wave * ROWS_PER_WAVE + rr;
    if (row >= R) break;
    float dot[C];
#pragma unroll
    for (int c = 0; c < C; ++c) dot[c] = 0.f;
#pragma unroll
    for (int i = 0; i < MAX_CHUNKS; ++i) {
      const int ch = lane + 64 * i;
      if (ch >= nch) break;
      const int h0 = ch * 8;
      float v[8];
      unpack8(*reinterpret_cast<const u32x4*>(pre + (int64_t)row * ld_pre + h0), v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = bf2f(f2bf(act_fwd(v[k], act)));  // the bf16 activation the backward sees
      *reinterpret_cast<u32x4*>(t_out + (int64_t)row * H + h0) = pack8(v);
      if (dp.enabled) {  // bf16(t · keep · scale)
        float kf[8];
        keep8(row, h0, dp, kf);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = bf2f(f2bf(v[k] * kf[k]));
      }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        float w[8];
        unpack8(*reinterpret_cast<const u32x4*>(W2 + (int64_t)c * H + h0), w);
#pragma unroll
        for (int k = 0; k < 8; ++k) dot[c] = fmaf(v[k], w[k], dot[c]);
      }
    }
    float lg[C];
#pragma unroll
    for (int c = 0; c < C; ++c) lg[c] = bf2f(f2bf(wave_sum(dot[c]) + bf2f(b2[c])));
    if (lane == 0) {
#pragma unroll
      for (int c = 0; c < C; ++c) logits[(int64_t)row * C + c] = f2bf(lg[c]);
      const int64_t lab = labels != nullptr ? labels[row] : -100;
      if (lab >= 0 && lab < C) {
        float m = lg[0];
        int am = 0;
#pragma unroll
        for (int c = 1; c < C; ++c)
          if (lg[c] > m) { m = lg[c]; am = c; }  // first maximum, as torch.argmax
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) s += __expf(lg[c] - m);
        loss_sum += __logf(s) + m - lg[lab];
        correct += am == lab ? 1.f : 0.f;
        nvalid += 1.f;
      }
    }
  }
  if (lane == 0) {
    red[wave][0] = loss_sum;
    red[wave][1] = correct;
    red[wave][2] = nvalid;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int k = threadIdx.x;
    partials[(int64_t)blockIdx.x * 4 + k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
  }
}

// stats = {loss_sum / max(n_valid, 1), correct, n_valid, loss_sum}
__global__ __launch_bounds__(256) void cls_stats_kernel(const float* __restrict__ partials, int nblk,
                                                        float* __restrict__ stats) {
  __shared__ float red[4][3];
  float s[3] = {0.f, 0.f, 0.f};
  for (int b = threadIdx.x; b < nblk; b += blockDim.x) {
#pragma unroll
    for (int k = 0; k < 3; ++k) s[k] += partials[(int64_t)b * 4 + k];
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 3; ++k) s[k] = wave_sum(s[k]);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 3; ++k) red[wave][k] = s[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float t[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) t[k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
    stats[0] = t[0] / fmaxf(t[2], 1.0f);
    stats[1] = t[1];
    stats[2] = t[2];
    stats[3] = t[0];
  }
}

template <int C>
__global__ __launch_bounds__(256) void cls_bwd_kernel(const bf16_t* __restrict__ t_in, const bf16_t* __restrict__ W2,
                                                      const bf16_t* __restrict__ logits, const int64_t* __restrict__ labels,
                                                      const float* __restrict__ stats, const float* __restrict__ dloss,
                                                      bf16_t* __restrict__ dpre, float* __restrict__ dW2,
                                                      float* __restrict__ db2, int R, int H, int act, DropoutParams dp) {
  static_assert(C <= MAXC, "classes");
  dp = resolve_seed(dp);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = H >> 3;
  const float scale = dloss[0] / fmaxf(stats[2], 1.0f);
  float aw[C][MAX_CHUNKS][8];  // this lane's dW2 partial sums over the block's rows
  float ab[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    ab[c] = 0.f;
#pragma unroll
    for (int i = 0; i < MAX_CHUNKS; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) aw[c][i][k] = 0.f;
  }
  for (int rr = 0; rr < ROWS_PER_WAVE; ++rr) {
    const int row = blockIdx.x * ROWS_PER_BLOCK + wave * ROWS_PER_WAVE + rr;
    if (row >= R) break;
    const int64_t lab = labels[row];
    float g[C];
    if (lab >= 0 && lab < C) {
      float lg[C], m = -3.0e38f;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        lg[c] = bf2f(logits[(int64_t)row * C + c]);
        m = fmaxf(m, lg[c]);
      }
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        lg[c] = __expf(lg[c] - m);
        s += lg[c];
      }
      const float inv = 1.0f / s;
#pragma unroll
      for (int c = 0; c < C; ++c) g[c] = (lg[c] * inv - (c == lab ? 1.f : 0.f)) * scale;
    } else {
#pragma unroll
      for (int c = 0; c < C; ++c) g[c] = 0.f;
    }
#pragma unroll
    for (int c = 0; c < C; ++c) ab[c] += g[c];
#pragma unroll
    for (int i = 0; i < MAX_CHUNKS; ++i) {
      const int ch = lane + 64 * i;
      if (ch >= nch) break;
      const int h0 = ch * 8;
      const int64_t e0 = (int64_t)row * H + h0;
      float t[8], dd[8];
      unpack8(*reinterpret_cast<const u32x4*>(t_in + e0), t);
#pragma unroll
      for (int k = 0; k < 8; ++k) dd[k] = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        float w[8];
        unpack8(*reinterpret_cast<const u32x4*>(W2 + (int64_t)c * H + h0), w);
#pragma unroll
        for (int k = 0; k < 8; ++k) dd[k] = fmaf(g[c], w[k], dd[k]);
      }
      float o[8], kf[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
      if (dp.enabled) keep8(row, h0, dp, kf);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float keep = kf[k];
        const float dv = bf2f(f2bf(t[k] * keep));  // the dropped activation (classifier input)
#pragma unroll
        for (int c = 0; c < C; ++c) aw[c][i][k] = fmaf(g[c], dv, aw[c][i][k]);
        o[k] = dd[k] * keep * act_bwd(t[k], act);
      }
      *reinterpret_cast<u32x4*>(dpre + e0) = pack8(o);
    }
  }
  // dW2 / db2: this lane's partial sums -> main_grad (fp32 atomics; 4 waves of a block add their own partials)
#pragma unroll
  for (int i = 0; i < MAX_CHUNKS; ++i) {
    const int ch = lane + 64 * i;
    if (ch >= nch) break;
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int k = 0; k < 8; ++k) atomicAdd(dW2 + (int64_t)c * H + ch * 8 + k, aw[c][i][k]);
  }
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < C; ++c) atomicAdd(db2 + c, ab[c]);
  }
}

}  // namespace cls

int cls_head_blocks(int R) { return (R + cls::ROWS_PER_BLOCK - 1) / cls::ROWS_PER_BLOCK; }

void launch_cls_head_fwd(const bf16_t* pre, int64_t ld_pre, const bf16_t* W2, const bf16_t* b2, const int64_t* labels,
                         bf16_t* t_out, bf16_t* logits, float* partials, float* stats, int R, int H, int C, int act,
                         double p, uint64_t seed, hipStream_t st) {
  const int nblk = cls_head_blocks(R);
  const DropoutParams dp = make_dropout(p, seed);
#define CLS_F(CC)                                                                                                 \
  case CC:                                                                                                        \
    hipLaunchKernelGGL(cls::cls_fwd_kernel<CC>, dim3(nblk), dim3(256), 0, st, pre, ld_pre, W2, b2, labels, t_out, \
                       logits, partials, R, H, act, dp);                                                          \
    break;
  switch (C) {
    CLS_F(1) CLS_F(2) CLS_F(3) CLS_F(4)
    default: abort();
  }
#undef CLS_F
  HSD_CHECK_LAUNCH();
  hipLaunchKernelGGL(cls::cls_stats_kernel, dim3(1), dim3(256), 0, st, (const float*)partials, nblk, stats);
  HSD_CHECK_LAUNCH();
}

void launch_cls_head_bwd(const bf16_t* t_in, const bf16_t* W2, const bf16_t* logits, const int64_t* labels,
                         const float* stats, const float* dloss, bf16_t* dpre, float* dW2, float* db2, int R, int H,
                         int C, int act, double p, uint64_t seed, hipStream_t st) {
  const int nblk = cls_head_blocks(R);
  const DropoutParams dp = make_dropout(p, seed);
#define CLS_B(CC)                                                                                             \
  case CC:                                                                                                    \
    hipLaunchKernelGGL(cls::cls_bwd_kernel<CC>, dim3(nblk), dim3(256), 0, st, t_in, W2, logits, labels, stats, \
                       dloss, dpre, dW2, db2, R, H, act, dp);                                                 \
    break;
  switch (C) {
    CLS_B(1) CLS_B(2) CLS_B(3) CLS_B(4)
    default: abort();
  }
#undef CLS_B
  HSD_CHECK_LAUNCH();
}

}  // namespace hsd
