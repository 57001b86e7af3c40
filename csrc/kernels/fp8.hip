// fp8 (OCP e4m3fn / e5m2 — gfx950 formats, not the MI300 fnuz ones) per-tensor quantisation for the fp8
// GEMM path (BASELINE.json config "roberta-large MLM ... fp8"):
//
//   amax  = max |x|                                  (block reduce + one atomicMax per block)
//   q     = sat_fmt(x · s),  s = FMT_MAX / amax       (16-B loads, 8 values -> 8 bytes per lane)
//   sinv  = 1 / s                                      (the GEMM epilogue multiplies acc by sinv_a·sinv_b)
//
// Everything stays on the device (amax / sinv are device scalars): no host synchronisation. Activations
// and gradients use DELAYED scaling — the scale comes from the amax the same site saw in the previous
// step and the quantising pass records this step's amax on the fly — so a tensor is read once; only a
// site's first use (no history yet) runs the separate amax pass ("current" scaling). The *_many
// variants batch all weight matrices of the model (W and its stored transpose share one amax) into one
// launch each after every optimizer step.
#include "fp8_common.h"

namespace hsd {

__device__ __forceinline__ float block_max(float v) {
  __shared__ float red[16];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r = fmaxf(r, red[i]);
  return r;  // valid in thread 0
}

__device__ __forceinline__ float absmax_range(const bf16_t* __restrict__ x, int64_t beg, int64_t end, int64_t stride) {
  float m = 0.f;
  int64_t i = beg;
  for (; i + 3 * stride + 8 <= end; i += 4 * stride) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const u32x4*>(x + i + u * stride);
#pragma unroll
    for (int u = 0; u < 4; ++u) m = absmax8(v[u], m);
  }
  for (; i < end; i += stride) {
    if (i + 8 <= end) {
      m = absmax8(*reinterpret_cast<const u32x4*>(x + i), m);
    } else {
      for (int64_t j = i; j < end; ++j) m = fmaxf(m, fabsf(bf2f(x[j])));
    }
  }
  return m;
}

// quantise [beg, end) (thread's first element `beg`, `stride` between a thread's vectors); four 16-B
// loads are issued before any is used so each thread keeps 64 B in flight. Returns max |x| seen.
template <int FMT>
__device__ __forceinline__ float quant_range(const bf16_t* __restrict__ x, uint8_t* __restrict__ q, int64_t beg,
                                             int64_t end, int64_t stride, float s) {
  float m = 0.f;
  int64_t i = beg;
  for (; i + 3 * stride + 8 <= end; i += 4 * stride) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const u32x4*>(x + i + u * stride);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      m = absmax8(v[u], m);
      *reinterpret_cast<u32x2*>(q + i + u * stride) = quant8<FMT>(v[u], s);
    }
  }
  for (; i < end; i += stride) {
    if (i + 8 <= end) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(x + i);
      m = absmax8(v, m);
      *reinterpret_cast<u32x2*>(q + i) = quant8<FMT>(v, s);
    } else {
      for (int64_t j = i; j < end; ++j) {
        m = fmaxf(m, fabsf(bf2f(x[j])));
        q[j] = (uint8_t)(cvt4<FMT>(bf2f(x[j]) * s, 0.f, 0.f, 0.f) & 0xFF);
      }
    }
  }
  return m;
}

// ---- single tensor -----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void amax_kernel(const bf16_t* __restrict__ x, int64_t n, float* __restrict__ amax) {
  const int64_t stride = (int64_t)gridDim.x * 256 * 8;
  const float m = block_max(absmax_range(x, ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8, n, stride));
  if (threadIdx.x == 0) atomic_max_pos(amax, m);
}

// scale from amax_in; amax_track (optional) accumulates this tensor's amax for the next step's scale
template <int FMT>
__global__ __launch_bounds__(256) void quant_kernel(const bf16_t* __restrict__ x, int64_t n,
                                                    const float* __restrict__ amax_in, uint8_t* __restrict__ q,
                                                    float* __restrict__ sinv, float* __restrict__ amax_track) {
  const float s = fmt_scale(FMT, *amax_in);
  if (blockIdx.x == 0 && threadIdx.x == 0) *sinv = 1.0f / s;
  const int64_t stride = (int64_t)gridDim.x * 256 * 8;
  const float m = quant_range<FMT>(x, q, ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8, n, stride, s);
  if (amax_track != nullptr) {
    const float bm = block_max(m);
    if (threadIdx.x == 0) atomic_max_pos(amax_track, bm);
  }
}

// ---- batched (weights) -------------------------------------------------------------------------
// desc rows: {src, dst (quant only), numel, amax index, first block}; blocks of tensor t: [first_t, first_t+1)
constexpr int kElemsPerBlock = 256 * 8 * 8;

__device__ __forceinline__ int find_tensor(const int64_t* desc, int nt, int ncol, int blk) {
  int lo = 0, hi = nt - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (desc[mid * ncol + 4] <= blk) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__global__ __launch_bounds__(256) void amax_many_kernel(const int64_t* __restrict__ desc, int nt,
                                                        float* __restrict__ amax) {
  const int t = find_tensor(desc, nt, 5, blockIdx.x);
  const int64_t* d = desc + t * 5;
  const bf16_t* x = reinterpret_cast<const bf16_t*>(d[0]);
  const int64_t n = d[2];
  const int64_t b0 = ((int64_t)blockIdx.x - d[4]) * kElemsPerBlock;
  const int64_t end = b0 + kElemsPerBlock < n ? b0 + kElemsPerBlock : n;
  const float m = block_max(absmax_range(x, b0 + threadIdx.x * 8, end, 256 * 8));
  if (threadIdx.x == 0) atomic_max_pos(amax + d[3], m);
}

template <int FMT>
__global__ __launch_bounds__(256) void quant_many_kernel(const int64_t* __restrict__ desc, int nt,
                                                         const float* __restrict__ amax, float* __restrict__ sinv) {
  const int t = find_tensor(desc, nt, 5, blockIdx.x);
  const int64_t* d = desc + t * 5;
  const bf16_t* x = reinterpret_cast<const bf16_t*>(d[0]);
  uint8_t* q = reinterpret_cast<uint8_t*>(d[1]);
  const int64_t n = d[2];
  const float s = fmt_scale(FMT, amax[d[3]]);
  if (blockIdx.x == d[4] && threadIdx.x == 0) sinv[d[3]] = 1.0f / s;
  const int64_t b0 = ((int64_t)blockIdx.x - d[4]) * kElemsPerBlock;
  const int64_t end = b0 + kElemsPerBlock < n ? b0 + kElemsPerBlock : n;
  (void)quant_range<FMT>(x, q, b0 + threadIdx.x * 8, end, 256 * 8, s);
}

// ---- host --------------------------------------------------------------------------------------
// ~2 resident blocks per SIMD-set of 256 CUs, each thread >= 4 vectors
static int quant_blocks(int64_t n) {
  const int64_t b = (n + 256 * 8 * 4 - 1) / (256 * 8 * 4);
  return (int)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

// compute_amax: first run the amax pass into `amax` (which must then be zeroed by the caller); the
// scale is taken from `amax`; amax_track (optional, atomicMax) records this tensor's amax.
void launch_fp8_quant(const bf16_t* x, int64_t n, float* amax, uint8_t* q, float* sinv, int fmt, bool compute_amax,
                      float* amax_track, hipStream_t st) {
  if (n <= 0) return;
  const int blocks = quant_blocks(n);
  if (compute_amax) {
    hipLaunchKernelGGL(amax_kernel, dim3(blocks), dim3(256), 0, st, x, n, amax);
    HSD_CHECK_LAUNCH();
  }
  if (fmt == 0) hipLaunchKernelGGL(quant_kernel<0>, dim3(blocks), dim3(256), 0, st, x, n, amax, q, sinv, amax_track);
  else hipLaunchKernelGGL(quant_kernel<1>, dim3(blocks), dim3(256), 0, st, x, n, amax, q, sinv, amax_track);
  HSD_CHECK_LAUNCH();
}

// amax_desc / quant_desc: device int64 [n][5]; block offsets built by the caller with kElemsPerBlock
void launch_fp8_quant_many(const int64_t* amax_desc, int n_amax, int amax_blocks, const int64_t* quant_desc,
                           int n_quant, int quant_blocks_total, float* amax, float* sinv, int fmt, hipStream_t st) {
  if (n_amax > 0) {
    hipLaunchKernelGGL(amax_many_kernel, dim3(amax_blocks), dim3(256), 0, st, amax_desc, n_amax, amax);
    HSD_CHECK_LAUNCH();
  }
  if (n_quant > 0) {
    if (fmt == 0)
      hipLaunchKernelGGL(quant_many_kernel<0>, dim3(quant_blocks_total), dim3(256), 0, st, quant_desc, n_quant, amax, sinv);
    else
      hipLaunchKernelGGL(quant_many_kernel<1>, dim3(quant_blocks_total), dim3(256), 0, st, quant_desc, n_quant, amax, sinv);
    HSD_CHECK_LAUNCH();
  }
}

int fp8_elems_per_block() { return kElemsPerBlock; }

}  // namespace hsd
