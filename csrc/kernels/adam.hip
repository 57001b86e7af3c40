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

#include <stdlib.h>

namespace hsd {

template <bool kGradBf16, bool kWriteBf16>
__device__ __forceinline__ f32x4 load_grad(const void* __restrict__ g_, int64_t i) {
  if constexpr (kGradBf16) {
    const u32x2 w = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(g_) + i);
    return f32x4{lo_bf(w.x), hi_bf(w.x), lo_bf(w.y), hi_bf(w.y)};
  } else {
    return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g_) + i);
  }
}

// kLo (fp32 compute, ops/hip32.py): `out` / `out_lo` receive the bf16 hi / lo halves of the updated weight (hi =
// bf16(θ), lo = bf16(θ - hi), exactly split2's), which the split-product GEMMs read directly -- the weights are split
// once per optimizer step instead of at every use in forward and backward.
// zero_g: the kernel also clears the gradient it consumed (16-B stores of the slot it just read), so the next step
// needs no separate memset pass over the whole gradient buffer ahead of its forward (optim/adam.py: set by the
// Trainer's eager steps; the store then skips its zero_grad once).
// U chunks of 4 elements per thread per trip, all U x 4 loads issued before the first use (a one-chunk trip
// leaves ~4 loads in flight per thread, too few to cover HBM latency at the occupancy a CU holds). Every
// byte is touched once per step, so loads and stores are non-temporal (no L2 / MALL pollution).
template <bool kGradBf16, bool kWriteBf16, int U, bool kLo = false>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, float* __restrict__ m,
                                                   float* __restrict__ v, void* __restrict__ g_,
                                                   bf16_t* __restrict__ out, const uint8_t* __restrict__ decay,
                                                   int64_t n4, float step, float eps, float b1, float b2,
                                                   float gscale, float lr_wd, const float* __restrict__ coef,
                                                   bf16_t* __restrict__ out_lo, int zero_g) {
  if (coef != nullptr) {  // HIP-graph replays: this step's scalars live on the device (train/graph.py)
    step = coef[0];
    eps = coef[1];
    gscale = coef[2];
    lr_wd = coef[3];
  }
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n4; i0 += stride * U) {
    f32x4 g[U], pp[U], mm[U], vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < n4) {
        g[u] = load_grad<kGradBf16, kWriteBf16>(g_, i);
        pp[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p) + i);
        mm[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(m) + i);
        vv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(v) + i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= n4) break;
      float wdf = 1.0f;
      if (decay != nullptr && lr_wd != 0.0f) wdf = decay[(i * 4) >> 6] ? (1.0f - lr_wd) : 1.0f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float gk = g[u][k] * gscale;
        mm[u][k] = b1 * mm[u][k] + (1.0f - b1) * gk;
        vv[u][k] = b2 * vv[u][k] + (1.0f - b2) * gk * gk;
        pp[u][k] = pp[u][k] * wdf - step * mm[u][k] / (sqrtf(vv[u][k]) + eps);
      }
      __builtin_nontemporal_store(pp[u], reinterpret_cast<f32x4*>(p) + i);
      __builtin_nontemporal_store(mm[u], reinterpret_cast<f32x4*>(m) + i);
      __builtin_nontemporal_store(vv[u], reinterpret_cast<f32x4*>(v) + i);
      if (zero_g) {
        if constexpr (kGradBf16) __builtin_nontemporal_store(u32x2{0u, 0u}, reinterpret_cast<u32x2*>(g_) + i);
        else __builtin_nontemporal_store(f32x4{0.f, 0.f, 0.f, 0.f}, reinterpret_cast<f32x4*>(g_) + i);
      }
      if constexpr (kWriteBf16) {
        u32x2 o;
        o.x = pack_bf2(pp[u][0], pp[u][1]);
        o.y = pack_bf2(pp[u][2], pp[u][3]);
        reinterpret_cast<u32x2*>(out)[i] = o;
        if constexpr (kLo) {
          u32x2 l;
          l.x = pack_bf2(pp[u][0] - lo_bf(o.x), pp[u][1] - hi_bf(o.x));
          l.y = pack_bf2(pp[u][2] - lo_bf(o.y), pp[u][3] - hi_bf(o.y));
          reinterpret_cast<u32x2*>(out_lo)[i] = l;
        }
      }
    }
  }
}

void launch_adam(float* p, float* m, float* v, void* g, bool grad_bf16, bf16_t* out_bf16,
                 const uint8_t* decay, int64_t n, float step, float eps, float b1, float b2, float gscale,
                 float lr_wd, const float* coef, hipStream_t stream, bf16_t* out_lo, bool zero_grad) {
  const int zg = zero_grad ? 1 : 0;
  int64_t n4 = n / 4;  // n is a multiple of 1024 (FlatParamStore)
  int threads = 256;
  int64_t blocks = (n4 + threads - 1) / threads;
  if (blocks > 256 * 8) blocks = 256 * 8;  // grid-stride: 8 blocks (32 waves) per CU over 256 CUs
  // two 16-B chunks per thread per trip (1 and 4 measured slower: profiles/bench_adam_r2.json)
#define HSD_ADAM(GB, WB)                                                                                            \
  hipLaunchKernelGGL((adam_kernel<GB, WB, 2>), dim3((unsigned)blocks), dim3(threads), 0, stream, p, m, v, g,      \
                     out_bf16, decay, n4, step, eps, b1, b2, gscale, lr_wd, coef, nullptr, zg)
  if (out_lo != nullptr) {
    if (out_bf16 == nullptr) abort();
    if (grad_bf16)
      hipLaunchKernelGGL((adam_kernel<true, true, 2, true>), dim3((unsigned)blocks), dim3(threads), 0, stream, p, m, v,
                         g, out_bf16, decay, n4, step, eps, b1, b2, gscale, lr_wd, coef, out_lo, zg);
    else
      hipLaunchKernelGGL((adam_kernel<false, true, 2, true>), dim3((unsigned)blocks), dim3(threads), 0, stream, p, m,
                         v, g, out_bf16, decay, n4, step, eps, b1, b2, gscale, lr_wd, coef, out_lo, zg);
    HSD_CHECK_LAUNCH();
    return;
  }
  if (grad_bf16) {
    if (out_bf16) HSD_ADAM(true, true); else HSD_ADAM(true, false);
  } else {
    if (out_bf16) HSD_ADAM(false, true); else HSD_ADAM(false, false);
  }
#undef HSD_ADAM
  HSD_CHECK_LAUNCH();
}

}  // namespace hsd
