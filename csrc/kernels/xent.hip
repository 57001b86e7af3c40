// Fused softmax cross-entropy for the task heads (reference loss
// SparseCategoricalCrossentropy(from_logits=True), SUM_OVER_BATCH_SIZE, scripts/train.py:118):
//
//   loss  = Σ_valid (logsumexp(x_r) - x_r[y_r]) / n_valid          (labels == -100 ignored, HF MLM)
//   dx_r  = (softmax(x_r) - onehot(y_r)) / n_valid                 (written in the same launch)
//   correct += [argmax(x_r) == y_r]                                (accuracy metric)
//
// One wave per row, any vocabulary size: pass 1 streams the row with 16-B loads keeping a per-lane
// online (max, Σexp) pair and argmax, wave-reduced; pass 2 re-reads the row and writes the gradient.
// The 2-way classifier (V = 2) and the 50265-way RoBERTa MLM decoder use the same kernel, so the MLM
// head never materialises a separate probability tensor.
#include "common.h"

namespace hsd {

template <bool kBF16>
__device__ __forceinline__ float ld1(const void* x, int64_t i) {
  if constexpr (kBF16) return bf2f(reinterpret_cast<const bf16_t*>(x)[i]);
  else return reinterpret_cast<const float*>(x)[i];
}
template <bool kBF16>
__device__ __forceinline__ void st1(void* x, int64_t i, float v) {
  if constexpr (kBF16) reinterpret_cast<bf16_t*>(x)[i] = f2bf(v);
  else reinterpret_cast<float*>(x)[i] = v;
}

// one 16-B load: 8 bf16 or 4 fp32 values from element index i (16-B aligned)
template <bool kBF16>
__device__ __forceinline__ void ldvec(const void* __restrict__ x, int64_t i, float (&v)[kBF16 ? 8 : 4]) {
  if constexpr (kBF16) {
    const u32x4 w = *reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16_t*>(x) + i);
#pragma unroll
    for (int k = 0; k < 4; ++k) { v[2 * k] = lo_bf(w[k]); v[2 * k + 1] = hi_bf(w[k]); }
  } else {
    const f32x4 w = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(x) + i);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = w[k];
  }
}

template <bool kBF16>
__global__ __launch_bounds__(256) void xent_kernel(const void* __restrict__ logits, const int64_t* __restrict__ labels,
                                                   void* __restrict__ dlogits, float* __restrict__ stats,
                                                   const float* __restrict__ n_valid, int rows, int V, int64_t ld) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t base = (int64_t)row * ld;
  const int64_t y = labels[row];
  const bool valid = y >= 0 && y < V;
  float m = -INFINITY, s = 0.f, best = -INFINITY;
  int besti = 0;
  // vector path: 8 bf16 (or 4 fp32) per 16-B load over the 16-B-aligned part of the row, scalar tail. XU 16-B loads
  // per lane are issued before any is used: one wave per row holds XU KiB in flight instead of 1 (the MLM head's
  // 4,928 x 50,432 logits were latency-bound at one load per wave)
  constexpr int VEC = kBF16 ? 8 : 4;
  constexpr int XU = 4;
  const bool vec = (ld % VEC) == 0;
  const int Vv = vec ? V - V % VEC : 0;
  auto consume = [&](const float (&v)[VEC], int j) {
    float cm = v[0];
#pragma unroll
    for (int k = 1; k < VEC; ++k) cm = fmaxf(cm, v[k]);
    const float nm = fmaxf(m, cm);
    s = s * __expf(m - nm);
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      s += __expf(v[k] - nm);
      if (v[k] > best) { best = v[k]; besti = j + k; }
    }
    m = nm;
  };
  int j0 = lane * VEC;
  for (; j0 + (XU - 1) * 64 * VEC < Vv; j0 += XU * 64 * VEC) {
    float v[XU][VEC];
#pragma unroll
    for (int u = 0; u < XU; ++u) ldvec<kBF16>(logits, base + j0 + u * 64 * VEC, v[u]);
#pragma unroll
    for (int u = 0; u < XU; ++u) consume(v[u], j0 + u * 64 * VEC);
  }
  for (; j0 < Vv; j0 += 64 * VEC) {
    float v[VEC];
    ldvec<kBF16>(logits, base + j0, v);
    consume(v, j0);
  }
  for (int j = Vv + lane; j < V; j += 64) {
    const float v = ld1<kBF16>(logits, base + j);
    const float nm = fmaxf(m, v);
    s = s * __expf(m - nm) + __expf(v - nm);
    m = nm;
    if (v > best || (v == best && j < besti)) { best = v; besti = j; }
  }
  // wave reduction of (m, s) and argmax (lowest index on ties, like torch.argmax)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(besti, o, 64);
    if (ob > best || (ob == best && oi < besti)) { best = ob; besti = oi; }
  }
  const float lse = m + __logf(s);
  const float inv_n = 1.0f / fmaxf(*n_valid, 1.0f);
  if (lane == 0 && valid) {
    atomicAdd(stats + 0, lse - ld1<kBF16>(logits, base + y));
    atomicAdd(stats + 1, besti == (int)y ? 1.0f : 0.0f);
  }
  if (dlogits) {
    // gradient over the whole padded row: columns >= V (a padded vocabulary) get exact zeros
    const float scale = valid ? inv_n : 0.f;
    if (vec) {
      auto emit = [&](const float (&v)[VEC], int j) {
        float g[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          const int jj = j + k;
          g[k] = jj < V ? scale * (__expf(v[k] - lse) - (jj == y ? 1.0f : 0.0f)) : 0.0f;
        }
        if constexpr (kBF16) {
          *reinterpret_cast<u32x4*>(reinterpret_cast<bf16_t*>(dlogits) + base + j) =
              u32x4{pack_bf2(g[0], g[1]), pack_bf2(g[2], g[3]), pack_bf2(g[4], g[5]), pack_bf2(g[6], g[7])};
        } else {
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(dlogits) + base + j) = f32x4{g[0], g[1], g[2], g[3]};
        }
      };
      // 16-B loads (the padded columns beyond V read the padding, which is then zeroed), XU in flight per lane
      int j = lane * VEC;
      for (; j + (XU - 1) * 64 * VEC < ld; j += XU * 64 * VEC) {
        float v[XU][VEC];
#pragma unroll
        for (int u = 0; u < XU; ++u) ldvec<kBF16>(logits, base + j + u * 64 * VEC, v[u]);
#pragma unroll
        for (int u = 0; u < XU; ++u) emit(v[u], j + u * 64 * VEC);
      }
      for (; j < ld; j += 64 * VEC) {
        float v[VEC];
        ldvec<kBF16>(logits, base + j, v);
        emit(v, j);
      }
    } else {
      for (int j = lane; j < ld; j += 64) {
        const float g = j < V ? scale * (__expf(ld1<kBF16>(logits, base + j) - lse) - (j == y ? 1.0f : 0.0f)) : 0.0f;
        st1<kBF16>(dlogits, base + j, g);
      }
    }
  }
}

// stats[0] += Σ loss terms, stats[1] += correct; n_valid: device scalar (number of non-ignored rows)
// ld: row stride of logits / dlogits (>= V; a padded vocabulary's extra columns are ignored and get zero gradient)
void launch_xent(const void* logits, bool bf16, const int64_t* labels, void* dlogits, float* stats,
                 const float* n_valid, int rows, int V, int64_t ld, hipStream_t st) {
  const int blocks = (rows + 3) / 4;
  if (blocks == 0) return;
  if (bf16) hipLaunchKernelGGL(xent_kernel<true>, dim3(blocks), dim3(256), 0, st, logits, labels, dlogits, stats, n_valid, rows, V, ld);
  else hipLaunchKernelGGL(xent_kernel<false>, dim3(blocks), dim3(256), 0, st, logits, labels, dlogits, stats, n_valid, rows, V, ld);
  HSD_CHECK_LAUNCH();
}

}  // namespace hsd
