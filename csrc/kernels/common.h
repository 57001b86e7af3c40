// Shared device helpers for the gfx950 (CDNA4) kernels.
//
// * bf16 is carried as raw 16-bit words (`bf16_t`); conversions go through the compiler's
//   f32->bf16 cast (v_cvt_pk_bf16_f32 on gfx950, RNE, NaN-preserving — MI355X_MICROARCH.md
//   'Correctness boundaries').
// * 16-byte vector types for every memory-bound kernel (cdna_hip_programming.md Guideline 13).
// * wave64 reductions (never 32-lane warp idioms).
// * the counter-based dropout mask (row word x column-pair word), bit-identical to ops/rng.py.
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

// two floats -> packed bf16x2 in one u32 (lo = a, hi = b): ONE v_cvt_pk_bf16_f32 with both sources (RNE, as f2bf).
// Built from two f2bf calls the compiler emitted two single-source converts + a shift + an SDWA or per pair -- about
// one extra VALU instruction per element in every bf16 epilogue.
typedef __bf16 bf16x2_native __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2_native));
}
__device__ __forceinline__ float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_bf(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }
// four fp32 values -> their bf16 hi = bf16(v) and lo = bf16(v - hi) halves at group i (8 B each): the split-product
// GEMMs' operand halves, written by the producing kernel (split2_kernel's arithmetic, bit for bit)
__device__ __forceinline__ void store_halves4(bf16_t* hi, bf16_t* lo, int64_t i, const float v0, const float v1,
                                              const float v2, const float v3) {
  u32x2 h, l;
  h.x = pack_bf2(v0, v1);
  h.y = pack_bf2(v2, v3);
  l.x = pack_bf2(v0 - lo_bf(h.x), v1 - hi_bf(h.x));
  l.y = pack_bf2(v2 - lo_bf(h.y), v3 - hi_bf(h.y));
  reinterpret_cast<u32x2*>(hi)[i] = h;
  reinterpret_cast<u32x2*>(lo)[i] = l;
}

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

// Σ over 8 bf16 pairs of (a·b): the attention backward's delta row partials -- ONE definition for the delta kernel and
// the out-projection dgrad epilogue that writes the same rows (E2_STORE_RDOT), so both give identical bits
__device__ __forceinline__ float dot8_bf16(const u32x4& a, const u32x4& b) {
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) acc += lo_bf(a[k]) * lo_bf(b[k]) + hi_bf(a[k]) * hi_bf(b[k]);
  return acc;
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

// ---- dropout mask (ops/rng.py, bit-identical) ------------------------------------------
// A dropout site is viewed as [rows, W] (W = its last dimension: the hidden size for [tokens, H] activations, S for
// the [B, heads, S, S] attention probabilities). Element (r, c) takes 16 bits of the 32-bit word of its column pair
// cp = c >> 1 of row r (lo16 -> even column, hi16 -> odd column):
//     bits(r, cp) = fin(R(r) ^ C(cp))
//     R(r)   = mix32(r ^ key)          lowbias32, ONE per row (attention: per lane; LN: per wave; GEMM epilogue: per chunk)
//     C(cp)  = clmul32(cp, kDropC)     GF(2)-linear, so C(a ^ b) = C(a) ^ C(b): a kernel folds its lane / tile offsets into
//                                      one register and each register offset is a compile-time literal
//     fin(x) = y ^ (y >> 16), y = x * kDropM
// Per element pair that is one XOR, one multiply and one XOR (the round-4 hash was two lowbias32 multiplies, three
// xor-shifts and the pair-index arithmetic per pair). Statistics (tools/rng_quality.py, tests/test_rng.py): keep rate
// within 3 sigma of 1 - p over 1e8 draws, no correlation between neighbouring rows / columns / pair halves / strides, 2x2
// block patterns chi-square consistent with independence. Trade-off of the linear column word: two rows whose row
// words differ by C(d) (0 < d < W/2) carry the same mask with the column pairs permuted by XOR d; a row pair hits one of
// those W/2 - 1 differences with probability (W/2 - 1) / 2^32, the rate of a random function
// (tests/test_rng.py::test_cross_row_twin_masks_occur_at_the_random_function_rate), and a twin keeps exactly as many
// elements as its partner.
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
constexpr uint32_t kDropC = 0x6D2B79F5u;
constexpr uint32_t kDropM = 0x9E3779B1u;
// C(cp): carry-less product of the column-pair index with kDropC (constexpr: literal offsets fold at compile time)
__host__ __device__ constexpr uint32_t drop_col(uint32_t cp) {
  uint32_t o = 0;
  for (int i = 0; i < 32; ++i)
    if ((kDropC >> i) & 1u) o ^= cp << i;
  return o;
}
// R(r): the row word (the site key folded in)
__host__ __device__ __forceinline__ uint32_t drop_row(uint32_t row, uint32_t key) { return mix32(row ^ key); }
// the pair's 32 bits from x = R(r) ^ C(cp)
__host__ __device__ __forceinline__ uint32_t drop_fin(uint32_t x) {
  const uint32_t y = x * kDropM;
  return y ^ (y >> 16);
}

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
// mask below reads no memory
__device__ __forceinline__ DropoutParams resolve_seed(DropoutParams d) {
  if (d.dev_seed != nullptr) {
    d.seed_lo ^= d.dev_seed[0];
    d.seed_hi ^= d.dev_seed[1];
    d.key = dropout_key(d.seed_lo, d.seed_hi);
    d.dev_seed = nullptr;
  }
  return d;
}

__device__ __forceinline__ uint32_t dropout_key_of(const DropoutParams& d) {
  if (d.dev_seed != nullptr) return dropout_key(d.seed_lo ^ d.dev_seed[0], d.seed_hi ^ d.dev_seed[1]);
  return d.key;
}

// the row word of row `row` of a site (R(r))
__device__ __forceinline__ uint32_t dropout_row(uint32_t row, const DropoutParams& d) {
  return drop_row(row, dropout_key_of(d));
}

// bits of column pair `cp` given its row word (generic path: C(cp) computed at run time when cp is not a literal)
__device__ __forceinline__ uint32_t dropout_bits_rc(uint32_t rw, uint32_t cp) { return drop_fin(rw ^ drop_col(cp)); }

// bits of element pair (row, cp) from scratch (one-off uses: heads, tails)
__device__ __forceinline__ uint32_t dropout_bits2(uint32_t row, uint32_t cp, const DropoutParams& d) {
  return dropout_bits_rc(dropout_row(row, d), cp);
}

// the two pairs of 4 consecutive elements from column c0 (c0 % 4 == 0) of row `row`: pairs c0/2 (even) and c0/2 ^ 1
__device__ __forceinline__ void dropout_bits4(uint32_t row, uint32_t c0, const DropoutParams& d, uint32_t& b0,
                                              uint32_t& b1) {
  const uint32_t x = dropout_row(row, d) ^ drop_col(c0 >> 1);
  b0 = drop_fin(x);
  b1 = drop_fin(x ^ drop_col(1));
}

// keep factor (0 or scale) for element `e` given its pair's bits
__device__ __forceinline__ float keep_factor(uint32_t bits, int e, const DropoutParams& d) {
  uint32_t b16 = (e & 1) ? (bits >> 16) : (bits & 0xFFFFu);
  return b16 >= d.thr ? d.scale : 0.0f;
}
// keep predicates of the two elements of a pair
__device__ __forceinline__ bool keep_lo(uint32_t bits, uint32_t thr) { return (bits & 0xFFFFu) >= thr; }
__device__ __forceinline__ bool keep_hi(uint32_t bits, uint32_t thr) { return (bits >> 16) >= thr; }

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
  // |x| rides on two scalar FMAs as a source modifier (a packed FMA has no |.| modifier: it took two v_and first)
  const f32x2 den = {fmaf(0.23164189784f, fabsf(x.x), 1.0f), fmaf(0.23164189784f, fabsf(x.y), 1.0f)};
  const f32x2 t = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  f32x2 P = __builtin_elementwise_fma(t, f32x2{1.061405429f, 1.061405429f}, f32x2{-1.453152027f, -1.453152027f});
  P = __builtin_elementwise_fma(t, P, f32x2{1.421413741f, 1.421413741f});
  P = __builtin_elementwise_fma(t, P, f32x2{-0.284496736f, -0.284496736f});
  P = __builtin_elementwise_fma(t, P, f32x2{0.254829592f, 0.254829592f});
  P = P * t;
  const f32x2 q = x * x * f32x2{-0.72134752044f, -0.72134752044f};
  const f32x2 e = {__builtin_amdgcn_exp2f(q.x), __builtin_amdgcn_exp2f(q.y)};
  const f32x2 pe = P * e;
  // ½(1 + erf(x/√2)) = ½ + sign(x)·(½ - ½·P·E): one packed FMA, two sign copies (v_bfi_b32) and one packed add, in
  // place of two candidates + two compares + two selects
  const f32x2 u = __builtin_elementwise_fma(f32x2{-0.5f, -0.5f}, pe, f32x2{0.5f, 0.5f});
  const f32x2 h = f32x2{copysignf(u.x, x.x), copysignf(u.y, x.y)} + f32x2{0.5f, 0.5f};
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
