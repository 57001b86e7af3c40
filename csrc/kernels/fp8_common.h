// fp8 (OCP e4m3fn / e5m2, gfx950) element helpers shared by the standalone quantiser (fp8.hip) and the producers
// that write an fp8 copy of their output in the same pass (layernorm.hip: LN forward / backward), so a fused and a
// standalone quantisation of the same bf16 tensor give the same bytes.
#pragma once
#include "common.h"

namespace hsd {

// an fp8 copy a producer kernel writes next to its bf16 output: q = sat(x / amax_in * FMT_MAX) with the site's
// delayed-scaling amax, sinv = amax_in / FMT_MAX (for the GEMM epilogue), this pass's max |x| into amax_track
struct Q8Out {
  uint8_t* q;
  const float* amax_in;
  float* sinv;
  float* amax_track;
  int only;  // 1: the producer skips the bf16 values this fp8 copy duplicates (the LN backward's dy)
};

constexpr float kE4M3Max = 448.0f, kE5M2Max = 57344.0f;

__device__ __forceinline__ void atomic_max_pos(float* addr, float v) {
  // non-negative floats order like their bit patterns; skip the (same-address, serialising) atomic when a
  // larger value is already there — after the first few blocks almost every block skips it
  if (v > __hip_atomic_load(addr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    atomicMax(reinterpret_cast<unsigned int*>(addr), __float_as_uint(v));
}

// max(m, |8 bf16 values|)
__device__ __forceinline__ float absmax8(const u32x4& v, float m) {
#pragma unroll
  for (int k = 0; k < 4; ++k) m = fmaxf(m, fmaxf(fabsf(lo_bf(v[k])), fabsf(hi_bf(v[k]))));
  return m;
}
template <int FMT>
__device__ __forceinline__ uint32_t cvt4(float a, float b, float c, float d) {
  constexpr float mx = FMT == 0 ? kE4M3Max : kE5M2Max;
  a = fminf(fmaxf(a, -mx), mx);
  b = fminf(fmaxf(b, -mx), mx);
  c = fminf(fmaxf(c, -mx), mx);
  d = fminf(fmaxf(d, -mx), mx);
  int r;
  if constexpr (FMT == 0) {
    r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    r = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
  } else {
    r = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
    r = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, r, true);
  }
  return (uint32_t)r;
}

template <int FMT>
__device__ __forceinline__ u32x2 quant8(const u32x4& v, float s) {
  u32x2 o;
  o.x = cvt4<FMT>(lo_bf(v[0]) * s, hi_bf(v[0]) * s, lo_bf(v[1]) * s, hi_bf(v[1]) * s);
  o.y = cvt4<FMT>(lo_bf(v[2]) * s, hi_bf(v[2]) * s, lo_bf(v[3]) * s, hi_bf(v[3]) * s);
  return o;
}

__device__ __forceinline__ float fmt_scale(int fmt, float amax) {
  return (fmt == 0 ? kE4M3Max : kE5M2Max) / fmaxf(amax, 1e-12f);
}

// per-wave max |x| -> one atomic per wave into amax_track (non-negative float order = bit order)
__device__ __forceinline__ void wave_amax_track(float m, float* amax_track) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) atomic_max_pos(amax_track, m);
}

}  // namespace hsd
