// Memory-bound elementwise kernels (16-B vector IO, grid-stride, 2048-block cap —
// cdna_hip_programming.md Guideline 11/13).
//
//  * bias_gelu_fwd : g = gelu_erf(y)  (y = GEMM output incl. bias; y is kept for backward)
//  * gelu_bwd_colsum: da = dg * gelu'(y)   and   dbias += Σ_rows da   (fused bias-grad reduction)
//  * colsum        : dbias += Σ_rows x   (fp32 atomics, one per column per block)
//  * dropout_fwd/bwd: out = x * keep * scale (hash RNG, ops/rng.py)
#include "common.h"

namespace hsd {

__global__ __launch_bounds__(256) void gelu_fwd_kernel(const bf16_t* __restrict__ y, bf16_t* __restrict__ g, int64_t n8) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    u32x4 w = reinterpret_cast<const u32x4*>(y)[i];
    u32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = pack_bf2(gelu_erf(lo_bf(w[k])), gelu_erf(hi_bf(w[k])));
    reinterpret_cast<u32x4*>(g)[i] = o;
  }
}

// block: 256 threads; thread t owns columns [8t, 8t+8) of a 2048-column group (blockIdx.y);
// blockIdx.x walks `rows_per_block` rows.
template <bool kGelu>
__global__ __launch_bounds__(256) void colsum_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ y,
                                                     bf16_t* __restrict__ out, float* __restrict__ dbias, int rows,
                                                     int N, int rows_per_block) {
  const int col = (blockIdx.y * 256 + threadIdx.x) * 8;
  if (col >= N) return;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int r = r0; r < r1; ++r) {
    size_t off = (size_t)r * N + col;
    u32x4 w = *reinterpret_cast<const u32x4*>(x + off);
    if constexpr (kGelu) {
      u32x4 yy = *reinterpret_cast<const u32x4*>(y + off);
      u32x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float a = lo_bf(w[k]) * gelu_erf_grad(lo_bf(yy[k]));
        float b = hi_bf(w[k]) * gelu_erf_grad(hi_bf(yy[k]));
        o[k] = pack_bf2(a, b);
        acc[2 * k] += lo_bf(o[k]);
        acc[2 * k + 1] += hi_bf(o[k]);
      }
      *reinterpret_cast<u32x4*>(out + off) = o;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[2 * k] += lo_bf(w[k]);
        acc[2 * k + 1] += hi_bf(w[k]);
      }
    }
  }
  if (dbias) {
#pragma unroll
    for (int k = 0; k < 8; ++k) atomicAdd(dbias + col + k, acc[k]);
  }
}

__global__ __launch_bounds__(256) void dropout_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ out, int64_t n4,
                                                      DropoutParams dp) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    u32x2 w = reinterpret_cast<const u32x2*>(x)[i];
    uint32_t pair0 = (uint32_t)(i * 2);
    uint32_t b0 = dropout_bits(pair0, dp.seed_lo, dp.seed_hi);
    uint32_t b1 = dropout_bits(pair0 + 1, dp.seed_lo, dp.seed_hi);
    u32x2 o;
    o.x = pack_bf2(lo_bf(w.x) * keep_factor(b0, 0, dp), hi_bf(w.x) * keep_factor(b0, 1, dp));
    o.y = pack_bf2(lo_bf(w.y) * keep_factor(b1, 0, dp), hi_bf(w.y) * keep_factor(b1, 1, dp));
    reinterpret_cast<u32x2*>(out)[i] = o;
  }
}

static inline int grid_for(int64_t n, int per_thread_vecs_div = 1) {
  int64_t b = (n + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

void launch_gelu_fwd(const bf16_t* y, bf16_t* g, int64_t n, hipStream_t st) {
  int64_t n8 = n / 8;  // caller guarantees n % 8 == 0
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(grid_for(n8)), dim3(256), 0, st, y, g, n8);
  HSD_CHECK_LAUNCH();
}

static void colsum_launch(bool gelu, const bf16_t* x, const bf16_t* y, bf16_t* out, float* dbias, int rows, int N,
                          hipStream_t st) {
  int gy = (N + 2047) / 2048;
  // aim for ~1024 blocks total
  int want_x = max(1, 1024 / gy);
  int rpb = max(16, (rows + want_x - 1) / want_x);
  int gx = (rows + rpb - 1) / rpb;
  if (gelu)
    hipLaunchKernelGGL((colsum_kernel<true>), dim3(gx, gy), dim3(256), 0, st, x, y, out, dbias, rows, N, rpb);
  else
    hipLaunchKernelGGL((colsum_kernel<false>), dim3(gx, gy), dim3(256), 0, st, x, y, out, dbias, rows, N, rpb);
  HSD_CHECK_LAUNCH();
}

void launch_gelu_bwd_colsum(const bf16_t* dg, const bf16_t* y, bf16_t* da, float* dbias, int rows, int N,
                            hipStream_t st) {
  colsum_launch(true, dg, y, da, dbias, rows, N, st);
}

void launch_colsum(const bf16_t* x, float* dbias, int rows, int N, hipStream_t st) {
  colsum_launch(false, x, nullptr, nullptr, dbias, rows, N, st);
}

void launch_dropout(const bf16_t* x, bf16_t* out, int64_t n, double p, uint64_t seed, hipStream_t st) {
  DropoutParams dp = make_dropout(p, seed);
  int64_t n4 = n / 4;  // caller guarantees n % 4 == 0
  hipLaunchKernelGGL(dropout_kernel, dim3(grid_for(n4)), dim3(256), 0, st, x, out, n4, dp);
  HSD_CHECK_LAUNCH();
}

}  // namespace hsd
