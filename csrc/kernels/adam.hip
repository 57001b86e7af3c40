// Fused Adam / AdamW over the flat parameter store (optim/adam.py).
//
// Replaces TF's ResourceApplyAdam, launched once per variable (393 launches for bert-large,
// SURVEY.md §2.10 K17), with ONE launch over flat buffers: 16-B vector IO on master/m/v/grad,
// DP 1/N (and grad-accum 1/k) folded into `grad_scale`, decoupled weight decay gated per
// 64-element block (segments are 64-aligned, so a block never straddles two parameters), and the
// bf16 compute copy written in the same pass (no separate cast kernel).
//
//   m = b1 m + (1-b1) g ;  v = b2 v + (1-b2) g² ;  θ = θ(1 - lr·wd·mask) - step·m/(√v + eps)
#include "common.h"

namespace hsd {

template <bool kGradBf16, bool kWriteBf16>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, float* __restrict__ m,
                                                   float* __restrict__ v, const void* __restrict__ g_,
                                                   bf16_t* __restrict__ out, const uint8_t* __restrict__ decay,
                                                   int64_t n4, float step, float eps, float b1, float b2,
                                                   float gscale, float lr_wd) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 g;
    if constexpr (kGradBf16) {
      u32x2 w = reinterpret_cast<const u32x2*>(g_)[i];
      g = f32x4{lo_bf(w.x), hi_bf(w.x), lo_bf(w.y), hi_bf(w.y)};
    } else {
      g = reinterpret_cast<const f32x4*>(g_)[i];
    }
    f32x4 pp = reinterpret_cast<f32x4*>(p)[i];
    f32x4 mm = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
    float wdf = 1.0f;
    if (decay != nullptr && lr_wd != 0.0f) wdf = decay[(i * 4) >> 6] ? (1.0f - lr_wd) : 1.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gk = g[k] * gscale;
      mm[k] = b1 * mm[k] + (1.0f - b1) * gk;
      vv[k] = b2 * vv[k] + (1.0f - b2) * gk * gk;
      pp[k] = pp[k] * wdf - step * mm[k] / (sqrtf(vv[k]) + eps);
    }
    reinterpret_cast<f32x4*>(p)[i] = pp;
    reinterpret_cast<f32x4*>(m)[i] = mm;
    reinterpret_cast<f32x4*>(v)[i] = vv;
    if constexpr (kWriteBf16) {
      u32x2 o;
      o.x = pack_bf2(pp[0], pp[1]);
      o.y = pack_bf2(pp[2], pp[3]);
      reinterpret_cast<u32x2*>(out)[i] = o;
    }
  }
}

void launch_adam(float* p, float* m, float* v, const void* g, bool grad_bf16, bf16_t* out_bf16,
                 const uint8_t* decay, int64_t n, float step, float eps, float b1, float b2, float gscale,
                 float lr_wd, hipStream_t stream) {
  int64_t n4 = n / 4;  // n is a multiple of 1024 (FlatParamStore)
  int threads = 256;
  int64_t blocks = (n4 + threads - 1) / threads;
  if (blocks > 256 * 16) blocks = 256 * 16;  // grid-stride: 16 blocks/CU over 256 CUs
#define HSD_ADAM(GB, WB)                                                                          \
  hipLaunchKernelGGL((adam_kernel<GB, WB>), dim3((unsigned)blocks), dim3(threads), 0, stream, p, m, v, g, \
                     out_bf16, decay, n4, step, eps, b1, b2, gscale, lr_wd)
  if (grad_bf16) {
    if (out_bf16) HSD_ADAM(true, true); else HSD_ADAM(true, false);
  } else {
    if (out_bf16) HSD_ADAM(false, true); else HSD_ADAM(false, false);
  }
#undef HSD_ADAM
  HSD_CHECK_LAUNCH();
}

}  // namespace hsd
