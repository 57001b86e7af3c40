// One LayerNorm row in the 16-B lane layout (bf16 in, fp32 two-pass statistics, bf16 out): lane owns the 8-column
// chunks c = lane + 64 i (i < NC8, c < H / 8). Shared by the standalone LayerNorm forward (layernorm.hip
// ln_fwd_plain16_kernel) and the LayerNorm tail of the persistent dropout + residual GEMM (gemm2.hip gemm2pk_kernel
// LNF), so both write identical bits.
#pragma once
#include "common.h"
#include "fp8_common.h"

namespace hsd {

template <int NC8, bool Q8>
__device__ __forceinline__ void ln_row16(const u32x4 (&yw)[NC8], const u32x4 (&gw)[NC8], const u32x4 (&bw)[NC8],
                                         int row, int H, int lane, float eps, bf16_t* __restrict__ out,
                                         float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                         uint8_t* __restrict__ q8 = nullptr, float qs = 0.f, float* qm = nullptr) {
  const int n8 = H >> 3;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NC8; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) s += lo_bf(yw[i][k]) + hi_bf(yw[i][k]);
  const float mean = wave_sum(s) / (float)H;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NC8; ++i) {
    if (lane + 64 * i < n8) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float d0 = lo_bf(yw[i][k]) - mean, d1 = hi_bf(yw[i][k]) - mean;
        ss += d0 * d0;
        ss += d1 * d1;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(ss) / (float)H + eps);
#pragma unroll
  for (int i = 0; i < NC8; ++i) {
    const int c = lane + 64 * i;
    if (c < n8) {
      u32x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        o[k] = pack_bf2((lo_bf(yw[i][k]) - mean) * rstd * lo_bf(gw[i][k]) + lo_bf(bw[i][k]),
                        (hi_bf(yw[i][k]) - mean) * rstd * hi_bf(gw[i][k]) + hi_bf(bw[i][k]));
      *reinterpret_cast<u32x4*>(out + (size_t)row * H + 8 * c) = o;
      if constexpr (Q8) {
        *qm = absmax8(o, *qm);
        *reinterpret_cast<u32x2*>(q8 + (size_t)row * H + 8 * c) = quant8<0>(o, qs);
      }
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// gamma / beta chunks of the lane (zero beyond H)
template <int NC8>
__device__ __forceinline__ void ln_params16(const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ beta, int H,
                                            int lane, u32x4 (&gw)[NC8], u32x4 (&bw)[NC8]) {
#pragma unroll
  for (int i = 0; i < NC8; ++i) {
    const int c = lane + 64 * i;
    gw[i] = bw[i] = u32x4{0, 0, 0, 0};
    if (c < (H >> 3)) {
      gw[i] = *reinterpret_cast<const u32x4*>(gamma + 8 * c);
      bw[i] = *reinterpret_cast<const u32x4*>(beta + 8 * c);
    }
  }
}

// the row's chunks of the lane (zero beyond H)
template <int NC8>
__device__ __forceinline__ void ln_load16(const bf16_t* __restrict__ y, int row, int H, int lane, u32x4 (&yw)[NC8]) {
#pragma unroll
  for (int i = 0; i < NC8; ++i) {
    const int c = lane + 64 * i;
    yw[i] = u32x4{0, 0, 0, 0};
    if (c < (H >> 3)) yw[i] = *reinterpret_cast<const u32x4*>(y + (size_t)row * H + 8 * c);
  }
}

}  // namespace hsd
