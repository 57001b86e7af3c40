// fp32 attention on the bf16 matrix cores: split products (the fp32 step, ops/hip32.py; the reference's precision,
// scripts/train.py:113-123 compiles with no mixed-precision policy). S = 128 .. 1024 (multiple of 128), head_dim 64.
//
// Every fp32 operand x is carried as two bf16 tensors x = hi + lo (hi = bf16(x), lo = bf16(x - hi): |x - hi - lo| <=
// 2^-17 |x|), and each product of the attention is the three-term split product
//     a·b ≈ ah·bh + al·bh + ah·bl        (the dropped al·bl is <= 2^-16 of each term)
// on v_mfma_f32_32x32x16_bf16 with fp32 accumulation -- the scheme of the fp32 GEMMs (ops/hip32.py split3). The
// softmax (max, exp2, row sums), the dropout mask (ops/rng.py, re-hashed: no keep bits) and every accumulation stay
// fp32; the probabilities P and the score gradient dS are split on the fly (pack8_split) for the P·V, Pᵀ·dO, dSᵀ·Q
// and dS·K products. Against the round-4 fp32 attention on the vector ALUs (attn32_* in fp32.hip: 1 wave per SIMD,
// one FMA per MAC) this is 3 MFMAs per bf16-MFMA-equivalent on 4 waves per SIMD.
//
// The three kernels mirror attentionS.hip (same lane / register layouts, same swizzled [64][64] images), with the
// streamed operand pair doubled into hi / lo images and TWO LDS stages (the tile t + 1 DMA lands under tile t):
// * forward (queries on lanes, K/V streamed): online softmax, O and lse2 (fp32 out);
// * backward dK/dV (keys on lanes, Q/dO streamed), backward dQ (queries on lanes, K/V streamed); delta = rowsum(dO∘O)
//   is the fp32 pre-pass of fp32.hip (attn32_delta).
#include "attn_common.h"

namespace hsd {
namespace a32m {

using namespace attn;
constexpr int kMaxS = 1024;
constexpr int TILE = 64 * D;  // one [64][64] bf16 image

// 64 rows x 64 cols starting at src0 into a [64][64] image: 8 DMA instructions, 2 per wave (attentionS.hip dma_tile)
__device__ __forceinline__ void dma_tile(bf16_t* img, const bf16_t* __restrict__ src0, int64_t ld, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int g = wave * 2 + i;
    const int row = g * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ swz(row);
    const bf16_t* src = src0 + (int64_t)row * ld + lc * 8;
    const uint32_t dst = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)(uint32_t)(size_t)(__attribute__((address_space(3))) bf16_t*)(img + g * 512));
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(dst)
                 : "memory");
  }
}

// every wave's DMA of the current tile landed; every wave done with the stage the next DMA overwrites
__device__ __forceinline__ void tile_sync() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <typename T>
__device__ __forceinline__ void settle(const T& v) {
  asm volatile("" ::"v"(v));
}

// hi / lo bf16 fragments of 8 fp32 accumulator values (registers 8s .. 8s+7): hi = bf16(x), lo = bf16(x - hi)
__device__ __forceinline__ void pack8_split(const f32x16& acc, int s, bf16x8& hi, bf16x8& lo) {
  u32x4 h, l;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float a = acc[8 * s + 2 * j], b = acc[8 * s + 2 * j + 1];
    h[j] = pack_bf2(a, b);
    l[j] = pack_bf2(a - lo_bf(h[j]), b - hi_bf(h[j]));
  }
  hi = __builtin_bit_cast(bf16x8, h);
  lo = __builtin_bit_cast(bf16x8, l);
}

__device__ __forceinline__ f32x16 mma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// ah·bh + al·bh + ah·bl
__device__ __forceinline__ f32x16 mma3(const bf16x8& ah, const bf16x8& al, const bf16x8& bh, const bf16x8& bl,
                                       f32x16 c) {
  c = mma(ah, bh, c);
  c = mma(al, bh, c);
  return mma(ah, bl, c);
}

// acc (32 rows on the lane x 64 d in registers: d = 32 blk + (reg & 3) + 8 (reg >> 2) + 4 hf) * scale -> fp32 rows of
// dst (row stride ld): four 16-B stores per accumulator
__device__ __forceinline__ void store_rows32(const f32x16& a0, const f32x16& a1, float scale, float* __restrict__ dst,
                                             int64_t ld, int lane) {
  const int r = lane & 31, h = lane >> 5;
  float* row = dst + (int64_t)r * ld + 4 * h;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    *reinterpret_cast<f32x4*>(row + 8 * g) =
        f32x4{a0[4 * g] * scale, a0[4 * g + 1] * scale, a0[4 * g + 2] * scale, a0[4 * g + 3] * scale};
    *reinterpret_cast<f32x4*>(row + 32 + 8 * g) =
        f32x4{a1[4 * g] * scale, a1[4 * g + 1] * scale, a1[4 * g + 2] * scale, a1[4 * g + 3] * scale};
  }
}

// ------------------------------------------------------------------------------------------------ forward
template <bool DROP>
__global__ __launch_bounds__(256, 2) void attn32m_fwd_kernel(const bf16_t* __restrict__ qh_all,
                                                             const bf16_t* __restrict__ ql_all,
                                                             const float* __restrict__ mask, float* __restrict__ out,
                                                             float* __restrict__ lse2, int S, int heads, float sl2,
                                                             DropoutParams dp) {
  dp = resolve_seed(dp);
  // 2 stages x [Kh Kl Vh Vl] + mask bias
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * 4 * TILE + 2 * kMaxS];
  float* mb_s = reinterpret_cast<float*>(lds + 2 * 4 * TILE);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int bh = blockIdx.y, b = bh / heads, hh = bh % heads;
  const int H = heads * D, ld = 3 * H;
  const int64_t boff = (int64_t)b * S * ld + hh * D;
  const bf16_t* bh_ = qh_all + boff;
  const bf16_t* bl_ = ql_all + boff;
  const int q0 = blockIdx.x * 128 + wave * 32;
  const int q = q0 + r;
  const int nt = S / 64;
  auto dma = [&](int stg, int kt) {
    bf16_t* st = lds + stg * 4 * TILE;
    const int64_t off = (int64_t)kt * 64 * ld;
    dma_tile(st, bh_ + off + H, ld, wave, lane);
    dma_tile(st + TILE, bl_ + off + H, ld, wave, lane);
    dma_tile(st + 2 * TILE, bh_ + off + 2 * H, ld, wave, lane);
    dma_tile(st + 3 * TILE, bl_ + off + 2 * H, ld, wave, lane);
  };
  dma(0, 0);
  bf16x8 qh[4], ql[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qh[s] = *reinterpret_cast<const bf16x8*>(bh_ + (int64_t)q * ld + 16 * s + 8 * hf);
    ql[s] = *reinterpret_cast<const bf16x8*>(bl_ + (int64_t)q * ld + 16 * s + 8 * hf);
  }
  for (int k = tid; k < S; k += 256) mb_s[k] = mask ? fmaxf(mask[(int64_t)b * S + k] * kLog2e, -1e30f) : 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    settle(qh[s]);
    settle(ql[s]);
  }
  f32x16 o0 = {}, o1 = {};
  float m = -INFINITY, l = 0.f;
  // dropout (attentionS.hip forward): row word of (bh, q) with the hf term folded in, C(32 kt) by readlane
  uint32_t xq = 0, ctile = 0;
  if constexpr (DROP) {
    xq = dropout_row((uint32_t)(bh * S + q), dp) ^ drop_col(2u * (uint32_t)hf);
    ctile = drop_col(32u * (uint32_t)lane);
  }
#pragma unroll 1
  for (int kt = 0; kt < nt; ++kt) {
    tile_sync();  // tile kt landed (the only DMA in flight); every wave is done with tile kt - 1's stage
    if (kt + 1 < nt) dma((kt + 1) & 1, kt + 1);
    const bf16_t* Kh = lds + (kt & 1) * 4 * TILE;
    const bf16_t* Kl = Kh + TILE;
    const bf16_t* Vh = Kh + 2 * TILE;
    const bf16_t* Vl = Kh + 3 * TILE;
    f32x16 st[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      st[kb] = f32x16{};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int o = toff(kb * 32 + r, 16 * s + 8 * hf);
        st[kb] = mma3(*reinterpret_cast<const bf16x8*>(Kh + o), *reinterpret_cast<const bf16x8*>(Kl + o), qh[s], ql[s],
                      st[kb]);
      }
    }
    float mx = m;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const f32x4 mb = *reinterpret_cast<const f32x4*>(mb_s + kt * 64 + kb * 32 + 8 * g4 + 4 * hf);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x = fmaf(st[kb][4 * g4 + e], sl2, mb[e]);
          st[kb][4 * g4 + e] = x;
          mx = fmaxf(mx, x);
        }
      }
    mx = max_xor32(mx);
    const float alpha = __builtin_amdgcn_exp2f(m - mx);
    m = mx;
    float ls = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const float p = __builtin_amdgcn_exp2f(st[kb][reg] - mx);
        ls += p;
        st[kb][reg] = p;
      }
    l = fmaf(l, alpha, ls);
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      o0[reg] *= alpha;
      o1[reg] *= alpha;
    }
    if constexpr (DROP) {
      const uint32_t xt = xq ^ (uint32_t)__builtin_amdgcn_readlane((int)ctile, kt);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int reg = 0; reg < 16; reg += 2) {
          const uint32_t bits = drop_fin(xt ^ drop_col((uint32_t)(16 * kb + 4 * (reg >> 2) + ((reg >> 1) & 1))));
          st[kb][reg] = keep_lo(bits, dp.thr) ? st[kb][reg] : 0.f;
          st[kb][reg + 1] = keep_hi(bits, dp.thr) ? st[kb][reg + 1] : 0.f;
        }
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 ph, pl;
        pack8_split(st[kb], s, ph, pl);
        o0 = mma3(trA(Vh, kb * 32, s, 0, lane), trA(Vl, kb * 32, s, 0, lane), ph, pl, o0);
        o1 = mma3(trA(Vh, kb * 32, s, 1, lane), trA(Vl, kb * 32, s, 1, lane), ph, pl, o1);
      }
  }
  l = sum_xor32(l);
  if (hf == 0) lse2[(int64_t)bh * S + q] = m + __log2f(l);
  const float oscale = (DROP ? dp.scale : 1.0f) / l;
  store_rows32(o0, o1, oscale, out + ((int64_t)b * S + q0) * H + hh * D, H, lane);
}

// ------------------------------------------------------------------------------------------------ backward dK, dV
template <bool DROP>
__global__ __launch_bounds__(256, 2) void attn32m_bwd_kv_kernel(const bf16_t* __restrict__ qh_all,
                                                                const bf16_t* __restrict__ ql_all,
                                                                const bf16_t* __restrict__ doh_all,
                                                                const bf16_t* __restrict__ dol_all,
                                                                const float* __restrict__ mask,
                                                                const float* __restrict__ lse2,
                                                                const float* __restrict__ delta,
                                                                float* __restrict__ dqkv, int S, int heads, float sl2,
                                                                float scale, DropoutParams dp) {
  dp = resolve_seed(dp);
  // 2 stages x [Qh Ql dOh dOl] | lse | delta | dropout row words
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * 4 * TILE + 6 * kMaxS];
  float* lse_s = reinterpret_cast<float*>(lds + 2 * 4 * TILE);
  float* del_s = lse_s + kMaxS;
  uint32_t* rw_s = reinterpret_cast<uint32_t*>(del_s + kMaxS);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int bh = blockIdx.y, b = bh / heads, hh = bh % heads;
  const int H = heads * D, ld = 3 * H;
  const int64_t boff = (int64_t)b * S * ld + hh * D;
  const int64_t doff = (int64_t)b * S * H + hh * D;
  const int k0 = blockIdx.x * 128 + wave * 32;
  const int key = k0 + r;
  const int nt = S / 64;
  auto dma = [&](int stg, int qt) {
    bf16_t* st = lds + stg * 4 * TILE;
    dma_tile(st, qh_all + boff + (int64_t)qt * 64 * ld, ld, wave, lane);
    dma_tile(st + TILE, ql_all + boff + (int64_t)qt * 64 * ld, ld, wave, lane);
    dma_tile(st + 2 * TILE, doh_all + doff + (int64_t)qt * 64 * H, H, wave, lane);
    dma_tile(st + 3 * TILE, dol_all + doff + (int64_t)qt * 64 * H, H, wave, lane);
  };
  dma(0, 0);
  bf16x8 kh[4], kl[4], vh[4], vl[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int64_t o = boff + (int64_t)key * ld + 16 * s + 8 * hf;
    kh[s] = *reinterpret_cast<const bf16x8*>(qh_all + o + H);
    kl[s] = *reinterpret_cast<const bf16x8*>(ql_all + o + H);
    vh[s] = *reinterpret_cast<const bf16x8*>(qh_all + o + 2 * H);
    vl[s] = *reinterpret_cast<const bf16x8*>(ql_all + o + 2 * H);
  }
  const float kb2 = mask ? fmaxf(mask[(int64_t)b * S + key] * kLog2e, -1e30f) : 0.f;
  for (int i = tid; i < S; i += 256) {
    lse_s[i] = lse2[(int64_t)bh * S + i];
    del_s[i] = delta[(int64_t)bh * S + i];
    if (DROP) rw_s[i] = dropout_row((uint32_t)(bh * S + i), dp);
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    settle(kh[s]);
    settle(kl[s]);
    settle(vh[s]);
    settle(vl[s]);
  }
  settle(kb2);
  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
  const bool odd = (lane & 1) != 0;
  // dropout: the 32-bit word of (query, key pair) is shared by lanes l, l ^ 1: the even lane computes query qi0's, the
  // odd lane query qi0 + 1's, and they swap (one DPP move)
  const uint32_t ck = drop_col((uint32_t)key >> 1);
  const int qsel = 4 * hf + (odd ? 1 : 0);
#pragma unroll 1
  for (int qt = 0; qt < nt; ++qt) {
    tile_sync();
    if (qt + 1 < nt) dma((qt + 1) & 1, qt + 1);
    const bf16_t* Qh = lds + (qt & 1) * 4 * TILE;
    const bf16_t* Ql = Qh + TILE;
    const bf16_t* dOh = Qh + 2 * TILE;
    const bf16_t* dOl = Qh + 3 * TILE;
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      f32x16 sacc = {}, dpacc = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int o = toff(qs * 32 + r, 16 * s + 8 * hf);
        sacc = mma3(*reinterpret_cast<const bf16x8*>(Qh + o), *reinterpret_cast<const bf16x8*>(Ql + o), kh[s], kl[s],
                    sacc);
        dpacc = mma3(*reinterpret_cast<const bf16x8*>(dOh + o), *reinterpret_cast<const bf16x8*>(dOl + o), vh[s],
                     vl[s], dpacc);
      }
      // rows: query qi = (reg & 3) + 8 (reg >> 2) + 4 hf of the sub-block; column (lane): key
      f32x16 pd, ds;
#pragma unroll
      for (int reg = 0; reg < 16; reg += 2) {
        const int qi0 = qt * 64 + qs * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * hf;
        const f32x2 lse = *reinterpret_cast<const f32x2*>(lse_s + qi0);
        const f32x2 del = *reinterpret_cast<const f32x2*>(del_s + qi0);
        const float p0 = __builtin_amdgcn_exp2f(fmaf(sacc[reg], sl2, kb2) - lse[0]);
        const float p1 = __builtin_amdgcn_exp2f(fmaf(sacc[reg + 1], sl2, kb2) - lse[1]);
        float f0 = 1.f, f1 = 1.f;
        if constexpr (DROP) {
          const uint32_t bits = drop_fin(rw_s[qt * 64 + qs * 32 + (reg & 3) + 8 * (reg >> 2) + qsel] ^ ck);
          const uint32_t other = dpp_xor1(bits);
          f0 = keep_factor(odd ? other : bits, key & 1, dp);
          f1 = keep_factor(odd ? bits : other, key & 1, dp);
        }
        pd[reg] = p0 * f0;
        pd[reg + 1] = p1 * f1;
        ds[reg] = p0 * fmaf(dpacc[reg], f0, -del[0]);
        ds[reg + 1] = p1 * fmaf(dpacc[reg + 1], f1, -del[1]);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 ph, pl, sh, sl;
        pack8_split(pd, s, ph, pl);
        pack8_split(ds, s, sh, sl);
        dv0 = mma3(trA(dOh, qs * 32, s, 0, lane), trA(dOl, qs * 32, s, 0, lane), ph, pl, dv0);
        dv1 = mma3(trA(dOh, qs * 32, s, 1, lane), trA(dOl, qs * 32, s, 1, lane), ph, pl, dv1);
        dk0 = mma3(trA(Qh, qs * 32, s, 0, lane), trA(Ql, qs * 32, s, 0, lane), sh, sl, dk0);
        dk1 = mma3(trA(Qh, qs * 32, s, 1, lane), trA(Ql, qs * 32, s, 1, lane), sh, sl, dk1);
      }
    }
  }
  float* rowbase = dqkv + ((int64_t)b * S + k0) * ld + hh * D;
  store_rows32(dv0, dv1, 1.0f, rowbase + 2 * H, ld, lane);
  store_rows32(dk0, dk1, scale, rowbase + H, ld, lane);
}

// ------------------------------------------------------------------------------------------------ backward dQ
template <bool DROP>
__global__ __launch_bounds__(256, 2) void attn32m_bwd_q_kernel(const bf16_t* __restrict__ qh_all,
                                                               const bf16_t* __restrict__ ql_all,
                                                               const bf16_t* __restrict__ doh_all,
                                                               const bf16_t* __restrict__ dol_all,
                                                               const float* __restrict__ mask,
                                                               const float* __restrict__ lse2,
                                                               const float* __restrict__ delta,
                                                               float* __restrict__ dqkv, int S, int heads, float sl2,
                                                               float scale, DropoutParams dp) {
  dp = resolve_seed(dp);
  // 2 stages x [Kh Kl Vh Vl] | mask bias
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * 4 * TILE + 2 * kMaxS];
  float* mb_s = reinterpret_cast<float*>(lds + 2 * 4 * TILE);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int bh = blockIdx.y, b = bh / heads, hh = bh % heads;
  const int H = heads * D, ld = 3 * H;
  const int64_t boff = (int64_t)b * S * ld + hh * D;
  const int64_t doff = (int64_t)b * S * H + hh * D;
  const int q0 = blockIdx.x * 128 + wave * 32;
  const int q = q0 + r;
  const int nt = S / 64;
  auto dma = [&](int stg, int kt) {
    bf16_t* st = lds + stg * 4 * TILE;
    const int64_t off = boff + (int64_t)kt * 64 * ld;
    dma_tile(st, qh_all + off + H, ld, wave, lane);
    dma_tile(st + TILE, ql_all + off + H, ld, wave, lane);
    dma_tile(st + 2 * TILE, qh_all + off + 2 * H, ld, wave, lane);
    dma_tile(st + 3 * TILE, ql_all + off + 2 * H, ld, wave, lane);
  };
  dma(0, 0);
  bf16x8 qh[4], ql[4], dh[4], dl[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int64_t o = boff + (int64_t)q * ld + 16 * s + 8 * hf;
    const int64_t od = doff + (int64_t)q * H + 16 * s + 8 * hf;
    qh[s] = *reinterpret_cast<const bf16x8*>(qh_all + o);
    ql[s] = *reinterpret_cast<const bf16x8*>(ql_all + o);
    dh[s] = *reinterpret_cast<const bf16x8*>(doh_all + od);
    dl[s] = *reinterpret_cast<const bf16x8*>(dol_all + od);
  }
  const float lse_q = lse2[(int64_t)bh * S + q];
  const float del_q = delta[(int64_t)bh * S + q];
  for (int k = tid; k < S; k += 256) mb_s[k] = mask ? fmaxf(mask[(int64_t)b * S + k] * kLog2e, -1e30f) : 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    settle(qh[s]);
    settle(ql[s]);
    settle(dh[s]);
    settle(dl[s]);
  }
  settle(lse_q);
  settle(del_q);
  f32x16 dq0 = {}, dq1 = {};
  uint32_t xq = 0, ctile = 0;
  if constexpr (DROP) {
    xq = dropout_row((uint32_t)(bh * S + q), dp) ^ drop_col(2u * (uint32_t)hf);
    ctile = drop_col(32u * (uint32_t)lane);
  }
#pragma unroll 1
  for (int kt = 0; kt < nt; ++kt) {
    tile_sync();
    if (kt + 1 < nt) dma((kt + 1) & 1, kt + 1);
    const bf16_t* Kh = lds + (kt & 1) * 4 * TILE;
    const bf16_t* Kl = Kh + TILE;
    const bf16_t* Vh = Kh + 2 * TILE;
    const bf16_t* Vl = Kh + 3 * TILE;
    const uint32_t xt = DROP ? xq ^ (uint32_t)__builtin_amdgcn_readlane((int)ctile, kt) : 0u;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      // Sᵀ[key][q] = K·Qᵀ, dPᵀ[key][q] = V·dOᵀ (query on the lane, key in the registers)
      f32x16 sacc = {}, dpacc = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int o = toff(kb * 32 + r, 16 * s + 8 * hf);
        sacc = mma3(*reinterpret_cast<const bf16x8*>(Kh + o), *reinterpret_cast<const bf16x8*>(Kl + o), qh[s], ql[s],
                    sacc);
        dpacc = mma3(*reinterpret_cast<const bf16x8*>(Vh + o), *reinterpret_cast<const bf16x8*>(Vl + o), dh[s], dl[s],
                     dpacc);
      }
      f32x16 ds;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int kk = kt * 64 + kb * 32 + 8 * g4 + 4 * hf;  // keys kk .. kk+3 in regs 4g4 .. 4g4+3
        const f32x4 mb = *reinterpret_cast<const f32x4*>(mb_s + kk);
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const int reg = 4 * g4 + e;
          const float p0 = __builtin_amdgcn_exp2f(fmaf(sacc[reg], sl2, mb[e]) - lse_q);
          const float p1 = __builtin_amdgcn_exp2f(fmaf(sacc[reg + 1], sl2, mb[e + 1]) - lse_q);
          float f0 = 1.f, f1 = 1.f;
          if constexpr (DROP) {
            const uint32_t bits = drop_fin(xt ^ drop_col((uint32_t)(16 * kb + 4 * g4 + (e >> 1))));
            f0 = keep_factor(bits, 0, dp);
            f1 = keep_factor(bits, 1, dp);
          }
          ds[reg] = p0 * fmaf(dpacc[reg], f0, -del_q);
          ds[reg + 1] = p1 * fmaf(dpacc[reg + 1], f1, -del_q);
        }
      }
      // dQᵀ[d][q] += Σ_key Kᵀ[d][key] dSᵀ[key][q]
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 sh, sl;
        pack8_split(ds, s, sh, sl);
        dq0 = mma3(trA(Kh, kb * 32, s, 0, lane), trA(Kl, kb * 32, s, 0, lane), sh, sl, dq0);
        dq1 = mma3(trA(Kh, kb * 32, s, 1, lane), trA(Kl, kb * 32, s, 1, lane), sh, sl, dq1);
      }
    }
  }
  store_rows32(dq0, dq1, scale, dqkv + ((int64_t)b * S + q0) * ld + hh * D, ld, lane);
}

// fp32 x [n] -> hi = bf16(x), lo = bf16(x - hi)
__global__ __launch_bounds__(256) void split2_kernel(const float* __restrict__ x, bf16_t* __restrict__ hi,
                                                     bf16_t* __restrict__ lo, int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    store_halves4(hi, lo, i, v[0], v[1], v[2], v[3]);
  }
}

}  // namespace a32m

bool attn32m_supported(int S, int head_dim) {
  return head_dim == attn::D && S % 128 == 0 && S >= 128 && S <= a32m::kMaxS;
}

void launch_split2(const float* x, bf16_t* hi, bf16_t* lo, int64_t n, hipStream_t st) {
  if (n % 4) abort();
  const int64_t n4 = n / 4;
  const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 4096);
  hipLaunchKernelGGL(a32m::split2_kernel, dim3(blocks), dim3(256), 0, st, x, hi, lo, n4);
  HSD_CHECK_LAUNCH();
}

void launch_attn32m_fwd(const bf16_t* qkv_hi, const bf16_t* qkv_lo, const float* mask, float* out, float* lse2, int B,
                        int S, int heads, double p, uint64_t seed, hipStream_t st) {
  if (!attn32m_supported(S, attn::D)) abort();
  DropoutParams dp = make_dropout(p, seed);
  const float sl2 = attn::kLog2e / sqrtf((float)attn::D);
  const dim3 grid(S / 128, B * heads);
  if (dp.enabled)
    hipLaunchKernelGGL(a32m::attn32m_fwd_kernel<true>, grid, dim3(256), 0, st, qkv_hi, qkv_lo, mask, out, lse2, S, heads,
                       sl2, dp);
  else
    hipLaunchKernelGGL(a32m::attn32m_fwd_kernel<false>, grid, dim3(256), 0, st, qkv_hi, qkv_lo, mask, out, lse2, S,
                       heads, sl2, dp);
  HSD_CHECK_LAUNCH();
}

// delta: fp32 [B*heads*S] = rowsum(dO∘O) (launch_attn32_delta, fp32.hip)
void launch_attn32m_bwd(const bf16_t* qkv_hi, const bf16_t* qkv_lo, const bf16_t* do_hi, const bf16_t* do_lo,
                        const float* mask, const float* lse2, const float* delta, float* dqkv, int B, int S, int heads,
                        double p, uint64_t seed, hipStream_t st) {
  if (!attn32m_supported(S, attn::D)) abort();
  DropoutParams dp = make_dropout(p, seed);
  const float sl2 = attn::kLog2e / sqrtf((float)attn::D);
  const float scale = 1.0f / sqrtf((float)attn::D);
  const dim3 grid(S / 128, B * heads);
  if (dp.enabled) {
    hipLaunchKernelGGL(a32m::attn32m_bwd_kv_kernel<true>, grid, dim3(256), 0, st, qkv_hi, qkv_lo, do_hi, do_lo, mask,
                       lse2, delta, dqkv, S, heads, sl2, scale, dp);
    HSD_CHECK_LAUNCH();
    hipLaunchKernelGGL(a32m::attn32m_bwd_q_kernel<true>, grid, dim3(256), 0, st, qkv_hi, qkv_lo, do_hi, do_lo, mask,
                       lse2, delta, dqkv, S, heads, sl2, scale, dp);
  } else {
    hipLaunchKernelGGL(a32m::attn32m_bwd_kv_kernel<false>, grid, dim3(256), 0, st, qkv_hi, qkv_lo, do_hi, do_lo, mask,
                       lse2, delta, dqkv, S, heads, sl2, scale, dp);
    HSD_CHECK_LAUNCH();
    hipLaunchKernelGGL(a32m::attn32m_bwd_q_kernel<false>, grid, dim3(256), 0, st, qkv_hi, qkv_lo, do_hi, do_lo, mask,
                       lse2, delta, dqkv, S, heads, sl2, scale, dp);
  }
  HSD_CHECK_LAUNCH();
}

}  // namespace hsd
