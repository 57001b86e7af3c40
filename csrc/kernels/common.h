// Shared device helpers for the gfx950 (CDNA4) kernels.
//
// * bf16 is carried as raw 16-bit words (`bf16_t`); conversions go through the compiler's
//   f32->bf16 cast (v_cvt_pk_bf16_f32 on gfx950, RNE, NaN-preserving — MI355X_MICROARCH.md
//   'Correctness boundaries').
// * 16-byte vector types for every memory-bound kernel (cdna_hip_programming.md Guideline 13).
// * wave64 reductions (never 32-lane warp idioms).
// * the counter-based dropout hash, bit-identical to ops/rng.py.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stdlib.h>

namespace hsd {

// ---- host-side A/B knobs (HSD_* environment variables) --------------------------------
// Read once per knob generation, not per launch: launch paths call HSD_KNOB(name, default) (a cached int; the
// default when unset). refresh_env_knobs() (bound as _C.refresh_env, called by tests that flip a knob in-process)
// bumps the generation so every knob is re-read at its next use.
inline int g_env_gen = 0;
#define HSD_KNOB(NAME, DFLT)                                 \
  ([]() -> int {                                             \
    static int v_ = 0, gen_ = -1;                            \
    if (gen_ != ::hsd::g_env_gen) {                          \
      const char* e_ = getenv(NAME);                         \
      v_ = e_ ? atoi(e_) : (DFLT);                           \
      gen_ = ::hsd::g_env_gen;                               \
    }                                                        \
    return v_;                                               \
  }())
constexpr int kKnobUnset = -0x7fffffff;  // HSD_KNOB default meaning "not set"

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) short bf16x8;   // MFMA A/B fragment (8 bf16)
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<bf16_t*>(&b);
}

// two floats -> packed bf16x2 in one u32 (lo = a, hi = b)
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}
__device__ __forceinline__ float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_bf(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }

// ---- lane exchanges inside 8-lane groups on DPP (one VALU op each; __shfl_xor is a ds_bpermute: an LDS round trip
// whose lgkmcnt wait serialises dependent chains, e.g. the attention backward's per-key-pair dropout hash exchange)
__device__ __forceinline__ uint32_t dpp_xor1(uint32_t v) {  // lane l <- lane l^1 (quad_perm [1,0,3,2])
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ float dpp_xor1(float v) { return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false)); }
__device__ __forceinline__ float dpp_xor2(float v) {  // lane l <- lane l^2 (quad_perm [2,3,0,1])
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_half_mirror(float v) {  // lane l <- lane 7-l within each 8-lane group
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));
}
// sum over each aligned group of 8 lanes, every lane gets its group's total (same value in all 8 lanes, and the same
// additions pairwise as the xor-1/2/4 butterfly: bit-identical to it)
__device__ __forceinline__ float sum8_dpp(float v) {
  v += dpp_xor1(v);
  v += dpp_xor2(v);
  return v + dpp_half_mirror(v);
}

// sum over the 8 lanes {l & 7 + 8 j}: lane-bit 3 by DPP row_ror:8, bits 4 and 5 by the gfx950 permlane swaps (each swap
// of v with itself returns both halves of the xor-16 / xor-32 pair); the same pairwise additions as the xor-8/16/32
// butterfly, so bit-identical to it, with no LDS round trip
__device__ __forceinline__ float sum_stride8(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, false));
  auto p16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(p16[0]) + __uint_as_float(p16[1]);
  auto p32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(p32[0]) + __uint_as_float(p32[1]);
}

// pair reductions across the two 32-lane halves (lane l with l ^ 32) on one permlane32 swap
__device__ __forceinline__ float sum_xor32(float v) {
  auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ float max_xor32(float v) {
  auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}

// ---- wave64 reductions ---------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- dropout hash (ops/rng.py) -------------------------------------------------------
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
// 32-bit key of a dropout site's 64-bit seed (mixed ONCE per site / kernel, not per element)
__host__ __device__ __forceinline__ uint32_t dropout_key(uint32_t seed_lo, uint32_t seed_hi) {
  return mix32(seed_lo ^ mix32(seed_hi));
}
// 32 random bits for element pair j: lo16 -> element 2j, hi16 -> element 2j+1. ONE lowbias32 round per pair
// (a bijection of j ^ key, so no two pairs of a site collide): the attention kernels hash every (query, key)
// pair, and a second per-pair round cost ~15 % of their time at p = 0.1 (tools/attn_one.py).
__device__ __forceinline__ uint32_t dropout_bits_k(uint32_t pair, uint32_t key) { return mix32(pair ^ key); }

struct DropoutParams {
  uint32_t seed_lo, seed_hi;
  uint32_t key;     // dropout_key(seed_lo, seed_hi), device step seed folded in by resolve_seed
  uint32_t thr;     // keep iff bits16 >= thr
  float scale;      // 1/(1-p)
  int enabled;
  // optional device-side step seed XORed into (seed_lo, seed_hi): lets a captured HIP graph replay with
  // fresh dropout masks every step (the per-site host seeds are baked into the graph)
  const uint32_t* dev_seed;
};

// process-wide device step seed (uint32 [2]) picked up by every make_dropout (null = off)
inline const uint32_t* g_dropout_dev_seed = nullptr;

__host__ inline DropoutParams make_dropout(double p, uint64_t seed) {
  DropoutParams d;
  d.seed_lo = (uint32_t)(seed & 0xFFFFFFFFull);
  d.seed_hi = (uint32_t)(seed >> 32);
  d.key = dropout_key(d.seed_lo, d.seed_hi);
  double t = p * 65536.0;
  d.thr = (uint32_t)(t + 0.5);
  d.scale = p > 0.0 ? (float)(1.0 / (1.0 - p)) : 1.0f;
  d.enabled = p > 0.0 ? 1 : 0;
  d.dev_seed = g_dropout_dev_seed;
  return d;
}

// fold the device step seed into the params ONCE per kernel (kernels call this on entry), so the per-element
// hash below reads no memory
__device__ __forceinline__ DropoutParams resolve_seed(DropoutParams d) {
  if (d.dev_seed != nullptr) {
    d.seed_lo ^= d.dev_seed[0];
    d.seed_hi ^= d.dev_seed[1];
    d.key = dropout_key(d.seed_lo, d.seed_hi);
    d.dev_seed = nullptr;
  }
  return d;
}

__device__ __forceinline__ uint32_t dropout_bits(uint32_t pair, const DropoutParams& d) {
  uint32_t key = d.key;
  if (d.dev_seed != nullptr) key = dropout_key(d.seed_lo ^ d.dev_seed[0], d.seed_hi ^ d.dev_seed[1]);
  return dropout_bits_k(pair, key);
}

// keep factor (0 or scale) for element `e` given its pair's bits
__device__ __forceinline__ float keep_factor(uint32_t bits, int e, const DropoutParams& d) {
  uint32_t b16 = (e & 1) ? (bits >> 16) : (bits & 0xFFFFu);
  return b16 >= d.thr ? d.scale : 0.0f;
}

// Exact-erf GELU (HF "gelu") with erf from Abramowitz & Stegun 7.1.26 (|err| <= 1.5e-7, far below bf16
// resolution): one v_rcp_f32 + one v_exp_f32 + ~12 FMA-class ops instead of libm erff's piecewise
// polynomial — the GELU epilogues of the FFN GEMMs are VALU-bound (cdna_hip_programming.md §5.4 rule 28).
//   z = |x|/√2,  t = 1/(1 + p·z),  erf(z) = 1 - P(t)·e^{-z²}
//   gelu(x)  = max(x, 0) - ½|x|·P·E                 with E = e^{-x²/2}
//   gelu'(x) = ½(1+erf(x/√2)) + x·E/√(2π)
struct GeluParts {
  float pe;  // P(t)·E
  float e;   // E
};
__device__ __forceinline__ GeluParts gelu_parts(float x) {
  const float a = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.23164189784f /* p/√2 */, a, 1.0f));
  float P = fmaf(t, 1.061405429f, -1.453152027f);
  P = fmaf(t, P, 1.421413741f);
  P = fmaf(t, P, -0.284496736f);
  P = fmaf(t, P, 0.254829592f);
  P *= t;
  const float e = __builtin_amdgcn_exp2f(x * x * -0.72134752044f /* -½·log2(e) */);
  return {P * e, e};
}
__device__ __forceinline__ float gelu_erf(float x) {
  const GeluParts g = gelu_parts(x);
  return fmaf(-0.5f * fabsf(x), g.pe, fmaxf(x, 0.0f));
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const GeluParts g = gelu_parts(x);
  const float half_1p_erf = x >= 0.0f ? fmaf(-0.5f, g.pe, 1.0f) : 0.5f * g.pe;
  return fmaf(x * 0.3989422804014327f, g.e, half_1p_erf);
}

// gelu(x) and gelu'(x) from one set of erf parts (the FFN forward keeps gelu' for the backward)
__device__ __forceinline__ void gelu_and_grad(float x, float& g, float& dg) {
  const GeluParts q = gelu_parts(x);
  const float half_1p_erf = x >= 0.0f ? fmaf(-0.5f, q.pe, 1.0f) : 0.5f * q.pe;
  g = x * half_1p_erf;
  dg = fmaf(x * 0.3989422804014327f, q.e, half_1p_erf);
}

// Two elements per call on packed f32 math (v_pk_fma_f32 / v_pk_mul_f32: two lanes' worth of FMA per issue;
// only v_rcp / v_exp stay scalar) for the VALU-bound GELU epilogue of the FFN1 GEMM; same FMAs, same results
// as gelu_and_grad.
__device__ __forceinline__ void gelu_and_grad2(f32x2 x, f32x2& g, f32x2& dg) {
  const f32x2 a = {fabsf(x.x), fabsf(x.y)};
  const f32x2 den = __builtin_elementwise_fma(a, f32x2{0.23164189784f, 0.23164189784f}, f32x2{1.0f, 1.0f});
  const f32x2 t = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  f32x2 P = __builtin_elementwise_fma(t, f32x2{1.061405429f, 1.061405429f}, f32x2{-1.453152027f, -1.453152027f});
  P = __builtin_elementwise_fma(t, P, f32x2{1.421413741f, 1.421413741f});
  P = __builtin_elementwise_fma(t, P, f32x2{-0.284496736f, -0.284496736f});
  P = __builtin_elementwise_fma(t, P, f32x2{0.254829592f, 0.254829592f});
  P = P * t;
  const f32x2 q = x * x * f32x2{-0.72134752044f, -0.72134752044f};
  const f32x2 e = {__builtin_amdgcn_exp2f(q.x), __builtin_amdgcn_exp2f(q.y)};
  const f32x2 pe = P * e;
  const f32x2 pos = __builtin_elementwise_fma(f32x2{-0.5f, -0.5f}, pe, f32x2{1.0f, 1.0f});
  const f32x2 neg = f32x2{0.5f, 0.5f} * pe;
  const f32x2 h = {x.x >= 0.0f ? pos.x : neg.x, x.y >= 0.0f ? pos.y : neg.y};
  g = x * h;
  dg = __builtin_elementwise_fma(x * f32x2{0.3989422804014327f, 0.3989422804014327f}, e, h);
}

}  // namespace hsd

// Debug build (HSD_DEBUG=1 python -m ..._build, loaded as _C_debug when HSD_DEBUG=1 at run time;
// SURVEY.md §5 'bounds-check debug builds'): every launch is followed by a device synchronisation so a
// fault is reported at the kernel that caused it, and HSD_DASSERT device checks are compiled in.
#ifdef HSD_DEBUG
#define HSD_CHECK_LAUNCH()                                                                    \
  do {                                                                                        \
    hipError_t e__ = hipGetLastError();                                                       \
    if (e__ == hipSuccess) e__ = hipDeviceSynchronize();                                      \
    if (e__ != hipSuccess) {                                                                  \
      fprintf(stderr, "HIP error %s after launch at %s:%d\n", hipGetErrorString(e__), __FILE__, __LINE__); \
      abort();                                                                                \
    }                                                                                         \
  } while (0)
#define HSD_DASSERT(c)                                                                        \
  do {                                                                                        \
    if (!(c)) {                                                                               \
      printf("HSD_DASSERT(%s) failed at %s:%d block (%d,%d) thread %d\n", #c, __FILE__, __LINE__, \
             (int)blockIdx.x, (int)blockIdx.y, (int)threadIdx.x);                             \
      __builtin_trap();                                                                       \
    }                                                                                         \
  } while (0)
#else
#define HSD_CHECK_LAUNCH()                                                                    \
  do {                                                                                        \
    hipError_t e__ = hipGetLastError();                                                       \
    if (e__ != hipSuccess) {                                                                  \
      fprintf(stderr, "HIP launch error %s at %s:%d\n", hipGetErrorString(e__), __FILE__, __LINE__); \
      abort();                                                                                \
    }                                                                                         \
  } while (0)
#define HSD_DASSERT(c) \
  do {                 \
  } while (0)
#endif
