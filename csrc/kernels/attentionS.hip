// Flash attention for S = 256 .. 1024 (multiple of 128), head_dim 64 — the long-sequence configs of
// SURVEY.md §2.10 (bert-large / roberta-large at max_seq_length 512; K4-K7 forward, K14 backward).
// S == 128 keeps the single-workgroup kernels of attention128.hip.
//
// All three kernels use one workgroup = 4 waves = 128 rows of one (batch, head), the wave's 32 rows on
// the MFMA lanes (v_mfma_f32_32x32x16_bf16), and stream the other operand pair through LDS in 64-row
// tiles: global_load_lds DMA into a 3-stage ring of [64][64] swizzled images (attn_common.h), one raw
// barrier per tile, the DMAs of tiles t+1 and t+2 in flight while tile t is multiplied.
//
// * forward (queries on lanes, K/V streamed): online softmax in the log2 domain; Oᵀ += Vᵀ·Pᵀ with the
//   Sᵀ accumulator as the B operand; O staged to 128-B row stores; lse2 saved for the backward.
// * backward dK/dV (keys on lanes, Q/dO streamed): P recomputed from lse2, dVᵀ += dOᵀ·P̃, dKᵀ += Qᵀ·dS,
//   k/v bias gradients as column sums of the stored rows.
// * backward dQ (queries on lanes, K/V streamed): Sᵀ and dPᵀ recomputed, dQᵀ += Kᵀ·dSᵀ, q bias gradient.
//   Splitting dQ into its own pass (instead of fp32 atomics across key blocks) keeps every output
//   written exactly once and deterministic, at the price of recomputing S and dP (7 instead of 5
//   GEMM-equivalents) — the MFMA work is cheap next to the atomics traffic it replaces.
// * delta[q] = Σ_d dO·O is a separate bandwidth kernel (every key block needs all of it).
// * keep mask (optional, kmask): the forward writes its dropout keep bits, [S/32][S] words per (batch, head), bit i
//   of word (qb, key) = keep(query 32 qb + i, key) (one wave ballot per key register), and both backward passes read
//   them (preloaded into LDS) instead of re-hashing every (query, key) pair: the dK/dV pass (keys on lanes) takes
//   its key's word of each query block, the dQ pass (queries on lanes) bit (q mod 32) of the words of its keys.
// Dropout / mask / lse conventions are identical to attention.hip / attention128.hip.
#include "attn_common.h"


namespace hsd {
namespace aS {

using namespace attn;
constexpr int kMaxS = 1024;
constexpr int TILE = 64 * D;  // one [64][64] bf16 image

constexpr int NSTG = 3;       // LDS stages per streamed operand: tiles t+1 and t+2 in flight while t is used

// 64 rows x 64 cols starting at src0 into a [64][64] image: 8 DMA instructions, 2 per wave.
// Issued as inline asm (cdna_hip_programming.md "Operands and clobbers" LDS-DMA recipe) so that hipcc does not
// track it: with the builtin, hipcc cannot prove that the stage being written (a runtime ring index) differs
// from the stage being read, and waits vmcnt(0) before the first ds_read_b64_tr_b16 after every DMA, which
// drains the prefetch. Completion is counted by hand in tile_barrier (4 wave-instructions per tile).
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

// Wait until this wave's DMA of the tile about to be used has landed (the newer `inflight` tiles of two operands,
// 4 DMA wave-instructions per tile, may stay in flight), then a raw barrier: every wave's part is visible and
// every wave is done with the stage the next DMA overwrites. Never __syncthreads() here: its fence would wait
// for vmcnt(0) and drain the prefetch (cdna_hip_programming.md §5 "Pipelining across barriers").
// Register operands loaded by plain global loads before the loop must be COMPLETE before the loop: while an
// LDS-DMA is in flight, hipcc waits vmcnt(0) at the first use of any pending plain load, and for a use inside
// the loop that wait would run every iteration and drain the prefetch. A fake use right after the loads moves
// that one wait to the prologue.
template <typename T>
__device__ __forceinline__ void settle(const T& v) {
  asm volatile("" ::"v"(v));
}

// lane L of v <- the wave-uniform x (one v_writelane_b32: no per-lane select masks held in SGPRs)
__device__ int llvm_writelane(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ void put_lane(uint32_t& v, int lane, uint32_t x) {
  v = (uint32_t)llvm_writelane((int)x, lane, (int)v);
}

template <int INFLIGHT, int EXTRA = 0>
__device__ __forceinline__ void tile_barrier() {
  // EXTRA: younger vector-memory ops issued since the in-flight tiles' DMA (the forward's keep-mask stores)
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(4 * INFLIGHT + EXTRA) : "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ------------------------------------------------------------------------------------------------
// KM: the keep bits are written (kmask non-null), a compile-time choice so the per-register ballots carry no branch
template <bool DROP, bool KM = false>
__global__ __launch_bounds__(256, 2) void attnS_fwd_kernel(const bf16_t* __restrict__ qkv,
                                                           const float* __restrict__ mask, bf16_t* __restrict__ out,
                                                           float* __restrict__ lse2, int S, int heads, float sl2,
                                                           DropoutParams dp, Q8Out q8o, uint32_t* __restrict__ kmask) {
  dp = resolve_seed(dp);
  // [K0 K1 K2 | V0 V1 V2 | mask bias]; after the loop K0|K1 is the output staging
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * NSTG * TILE + 2 * kMaxS];
  bf16_t* Kb = lds;
  bf16_t* Vb = lds + NSTG * TILE;
  float* mb_s = reinterpret_cast<float*>(lds + 2 * NSTG * TILE);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int bh = blockIdx.y, b = bh / heads, hh = bh % heads;
  const int H = heads * D, ld = 3 * H;
  const bf16_t* base = qkv + (int64_t)b * S * ld + hh * D;
  const int q0 = blockIdx.x * 128 + wave * 32;
  const int q = q0 + r;
  const int nt = S / 64;
  HSD_DASSERT(S % 64 == 0 && S <= kMaxS && q < S);

  dma_tile(Kb, base + H, ld, wave, lane);
  dma_tile(Vb, base + 2 * H, ld, wave, lane);
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(base + (int64_t)q * ld + 16 * s + 8 * hf);
  for (int k = tid; k < S; k += 256) mb_s[k] = mask ? fmaxf(mask[(int64_t)b * S + k] * kLog2e, -1e30f) : 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) settle(qf[s]);
  if (nt > 1) {
    dma_tile(Kb + TILE, base + 64 * ld + H, ld, wave, lane);
    dma_tile(Vb + TILE, base + 64 * ld + 2 * H, ld, wave, lane);
  }

  f32x16 o0 = {}, o1 = {};
  float m = -INFINITY, l = 0.f;
  // dropout: mask row bh S + q, column pair key / 2 = 32 kt + 16 kb + 4 (reg >> 2) + (reg >> 1 & 1) + 2 hf (disjoint
  // bits). One row word per lane with the hf term folded in; C(32 kt) from lane kt of a per-kernel table (one
  // readlane per tile); each register's C(...) is a literal. P is kept or zeroed, the 1/(1-p) scale rides on 1/l.
  uint32_t xq = 0, ctile = 0;
  if constexpr (DROP) {
    xq = dropout_row((uint32_t)(bh * S + q), dp) ^ drop_col(2u * (uint32_t)hf);
    ctile = drop_col(32u * (uint32_t)lane);  // lane kt: C(32 kt), kt < S / 64 <= 16
  }
  constexpr bool km_on = DROP && KM;
  // keep-mask words of this wave: key-major [bh][q0 / 32][key], query-major [bh][kt][q][hf] (header)
  uint32_t* const km_k = km_on ? kmask + ((int64_t)bh * (S / 32) + q0 / 32) * S : nullptr;
  auto tile = [&](const int stg, const int kt) {
    // the previous tile's keep-mask store is younger than tile kt + 1's DMA: counted, not waited for
    if (kt + 1 < nt) {
      if (km_on && kt > 0) tile_barrier<1, 1>();
      else tile_barrier<1>();
    } else {
      if (km_on && kt > 0) tile_barrier<0, 1>();
      else tile_barrier<0>();
    }
    const bf16_t* Ks = Kb + stg * TILE;
    const bf16_t* Vs = Vb + stg * TILE;
    if (kt + 2 < nt) {
      const int s2 = stg == 0 ? 2 : stg - 1;
      const int64_t off = (int64_t)(kt + 2) * 64 * ld;
      dma_tile(Kb + s2 * TILE, base + off + H, ld, wave, lane);
      dma_tile(Vb + s2 * TILE, base + off + 2 * H, ld, wave, lane);
    }
    // Sᵀ[key][q] for the tile's 2 key blocks of 32
    f32x16 st[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      st[kb] = f32x16{};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(Ks + toff(kb * 32 + r, 16 * s + 8 * hf));
        st[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[s], st[kb], 0, 0, 0);
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
      uint32_t wk = 0;  // keep-mask word of key 64 kt + lane (the wave's 32 queries)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int reg = 0; reg < 16; reg += 2) {
          // key = kt*64 + kb*32 + (reg & 3) + 8 (reg >> 2) + 4 hf
          const uint32_t bits = drop_fin(xt ^ drop_col((uint32_t)(16 * kb + 4 * (reg >> 2) + ((reg >> 1) & 1))));
          const bool k0 = keep_lo(bits, dp.thr), k1 = keep_hi(bits, dp.thr);
          st[kb][reg] = k0 ? st[kb][reg] : 0.f;
          st[kb][reg + 1] = k1 ? st[kb][reg + 1] : 0.f;
          if constexpr (km_on) {
            // the wave's keep bits of this register's two keys per half-wave -> lanes (tile keys) kl, kl + 4, ...
            // (the ballot of the very compare the selects above use: the lane mask v_cmp already wrote)
            const unsigned long long m0 = __builtin_amdgcn_ballot_w64(k0), m1 = __builtin_amdgcn_ballot_w64(k1);
            const int kl = kb * 32 + (reg & 3) + 8 * (reg >> 2);  // tile key of `reg` on lanes 0-31
            put_lane(wk, kl, (uint32_t)m0);
            put_lane(wk, kl + 4, (uint32_t)(m0 >> 32));
            put_lane(wk, kl + 1, (uint32_t)m1);
            put_lane(wk, kl + 5, (uint32_t)(m1 >> 32));
          }
        }
      if constexpr (km_on) km_k[kt * 64 + lane] = wk;
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pb = pack8(st[kb], s);
        o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(Vs, kb * 32, s, 0, lane), pb, o0, 0, 0, 0);
        o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(Vs, kb * 32, s, 1, lane), pb, o1, 0, 0, 0);
      }
  };
#pragma unroll 1
  for (int t = 0, stg = 0; t < nt; ++t, stg = stg == NSTG - 1 ? 0 : stg + 1) tile(stg, t);
  l = sum_xor32(l);
  if (hf == 0) lse2[(int64_t)bh * S + q] = m + __log2f(l);
  __syncthreads();  // K images no longer read: reuse as staging
  const float oscale = (DROP ? dp.scale : 1.0f) / l;  // the dropout scale of the kept probabilities
  if (q8o.q != nullptr) {  // fp8 e4m3 copy of the output for the fp8 out-projection GEMM (delayed scaling)
    const float qs = fmt_scale(0, *q8o.amax_in);
    if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) *q8o.sinv = 1.0f / qs;
    float qm = 0.f;
    const int64_t off = ((int64_t)b * S + q0) * H + hh * D;
    store_rows(Kb + wave * 32 * D, o0, o1, oscale, out + off, H, lane, nullptr, q8o.q + off, 0, qs, &qm);
    wave_amax_track(qm, q8o.amax_track);
    return;
  }
  store_rows(Kb + wave * 32 * D, o0, o1, oscale, out + ((int64_t)b * S + q0) * H + hh * D, H, lane);
}

// ------------------------------------------------------------------------------------------------
// delta[bh*S + s] = Σ_d dO[b*S+s][h*64+d] · O[b*S+s][h*64+d]. One workgroup per (32 tokens, b·head): 8 threads
// per token (16 B each of O and dO, one 128-B line per token), so each wave stores 8 consecutive deltas and the
// workgroup one contiguous 128-B run (the old token-major mapping scattered one 4-B store per head, S·4 B apart).
__global__ __launch_bounds__(256) void attnS_delta_kernel(const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout,
                                                          float* __restrict__ delta, int S, int heads) {
  const int bh = blockIdx.y;
  const int b = bh / heads, hh = bh - b * heads;
  const int s = blockIdx.x * 32 + (threadIdx.x >> 3);  // S % 128 == 0 (attnS_supported)
  const int c = threadIdx.x & 7;
  const int64_t off = (((int64_t)b * S + s) * heads + hh) * D + c * 8;
  const u32x4 ov = *reinterpret_cast<const u32x4*>(o + off);
  const u32x4 dv = *reinterpret_cast<const u32x4*>(dout + off);
  const float acc = sum8_dpp(dot8_bf16(dv, ov));
  if (c == 0) delta[(int64_t)bh * S + s] = acc;
}

// ------------------------------------------------------------------------------------------------
template <bool DROP, bool KM = false>
__global__ __launch_bounds__(256, 2) void attnS_bwd_kv_kernel(const bf16_t* __restrict__ qkv,
                                                              const float* __restrict__ mask,
                                                              const bf16_t* __restrict__ dout,
                                                              const float* __restrict__ lse2,
                                                              const float* __restrict__ delta,
                                                              bf16_t* __restrict__ dqkv, float* __restrict__ dbias,
                                                              int S, int heads, float sl2, float scale,
                                                              DropoutParams dp, Q8Out q8o, int qfmt,
                                                              const uint32_t* __restrict__ kmask) {
  dp = resolve_seed(dp);
  // [Q0 Q1 Q2 | dO0 dO1 dO2 | lse | delta | k/v bias partials | keep-mask words]; after the loop Q0|Q1 is the output
  // staging
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * NSTG * TILE + 4 * kMaxS + 2 * 2 * 4 * D + 2 * (kMaxS / 32) * 128];
  bf16_t* Qb = lds;
  bf16_t* dOb = lds + NSTG * TILE;
  float* lse_s = reinterpret_cast<float*>(lds + 2 * NSTG * TILE);
  float* del_s = lse_s + kMaxS;
  float* bsum = del_s + kMaxS;  // [2 (k,v)][4 waves][64]
  uint32_t* km_s = reinterpret_cast<uint32_t*>(bsum + 2 * 4 * D);  // [S/32 query blocks][this block's 128 keys]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int bh = blockIdx.y, b = bh / heads, hh = bh % heads;
  const int H = heads * D, ld = 3 * H;
  const bf16_t* base = qkv + (int64_t)b * S * ld + hh * D;
  const bf16_t* dobase = dout + (int64_t)b * S * H + hh * D;
  const int k0 = blockIdx.x * 128 + wave * 32;
  const int key = k0 + r;
  const int nt = S / 64;
  HSD_DASSERT(S % 64 == 0 && S <= kMaxS && key < S);

  dma_tile(Qb, base, ld, wave, lane);
  dma_tile(dOb, dobase, H, wave, lane);
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = *reinterpret_cast<const bf16x8*>(base + (int64_t)key * ld + H + 16 * s + 8 * hf);
    vf[s] = *reinterpret_cast<const bf16x8*>(base + (int64_t)key * ld + 2 * H + 16 * s + 8 * hf);
  }
  const float kb2 = mask ? fmaxf(mask[(int64_t)b * S + key] * kLog2e, -1e30f) : 0.f;
  for (int i = tid; i < S; i += 256) {
    lse_s[i] = lse2[(int64_t)bh * S + i];
    del_s[i] = delta[(int64_t)bh * S + i];
  }
  constexpr bool km_on = DROP && KM;  // the forward's keep bits are read (compile-time: no per-register branch)
  if constexpr (km_on) {
    const uint32_t* src = kmask + (int64_t)bh * (S / 32) * S + blockIdx.x * 128;
    for (int i = tid; i < (S / 32) * 128; i += 256) km_s[i] = src[(int64_t)(i >> 7) * S + (i & 127)];
  } else if (DROP) {
    // re-hashing: the dropout row words R(bh S + q) of every query, in the keep-mask slot
    for (int i = tid; i < S; i += 256) km_s[i] = dropout_row((uint32_t)(bh * S + i), dp);
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    settle(kf[s]);
    settle(vf[s]);
  }
  settle(kb2);
  if (nt > 1) {
    dma_tile(Qb + TILE, base + 64 * ld, ld, wave, lane);
    dma_tile(dOb + TILE, dobase + 64 * H, H, wave, lane);
  }

  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
  const bool odd = (lane & 1) != 0;
  // dropout (re-hashing): mask row bh S + query, column pair key / 2 -- one 32-bit word for lanes l and l ^ 1: the
  // even lane computes query qi0's, the odd lane query qi0 + 1's, and they swap (one DPP move)
  const uint32_t ck = drop_col((uint32_t)key >> 1);
  const int qsel = 4 * hf + (odd ? 1 : 0);
  auto tile = [&](const int stg, const int qt) {

    if (qt + 1 < nt) tile_barrier<1>();
    else tile_barrier<0>();
    const bf16_t* Qs = Qb + stg * TILE;
    const bf16_t* dOs = dOb + stg * TILE;
    if (qt + 2 < nt) {
      const int s2 = stg == 0 ? 2 : stg - 1;
      dma_tile(Qb + s2 * TILE, base + (int64_t)(qt + 2) * 64 * ld, ld, wave, lane);
      dma_tile(dOb + s2 * TILE, dobase + (int64_t)(qt + 2) * 64 * H, H, wave, lane);
    }
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      f32x16 sacc = {}, dpacc = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 aq = *reinterpret_cast<const bf16x8*>(Qs + toff(qs * 32 + r, 16 * s + 8 * hf));
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aq, kf[s], sacc, 0, 0, 0);
        const bf16x8 ad = *reinterpret_cast<const bf16x8*>(dOs + toff(qs * 32 + r, 16 * s + 8 * hf));
        dpacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ad, vf[s], dpacc, 0, 0, 0);
      }
      // rows: query qi = (reg&3) + 8(reg>>2) + 4hf of the sub-block; col (lane): key
      f32x16 pd, ds;
      // this query block's keep bits of the lane's key, shifted to the lane's rows (4 hf)
      const uint32_t kmw = km_on ? km_s[(qt * 2 + qs) * 128 + wave * 32 + r] >> (4 * hf) : 0u;
#pragma unroll
      for (int reg = 0; reg < 16; reg += 2) {
        const int qi0 = qt * 64 + qs * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * hf;  // rows qi0, qi0 + 1
        const f32x2 lse = *reinterpret_cast<const f32x2*>(lse_s + qi0);
        const f32x2 del = *reinterpret_cast<const f32x2*>(del_s + qi0);
        const float p0 = __builtin_amdgcn_exp2f(fmaf(sacc[reg], sl2, kb2) - lse[0]);
        const float p1 = __builtin_amdgcn_exp2f(fmaf(sacc[reg + 1], sl2, kb2) - lse[1]);
        float f0 = 1.f, f1 = 1.f;
        if constexpr (DROP) {
          if constexpr (km_on) {
            const int pos = (reg & 3) + 8 * (reg >> 2);
            f0 = __uint_as_float((uint32_t)__builtin_amdgcn_sbfe((int)kmw, pos, 1) & __float_as_uint(dp.scale));
            f1 = __uint_as_float((uint32_t)__builtin_amdgcn_sbfe((int)kmw, pos + 1, 1) & __float_as_uint(dp.scale));
          } else {
            // keys 2j, 2j+1 (lanes l, l^1) share one hash per query row: the even lane hashes row qi0,
            // the odd lane row qi0 + 1, then they swap
            const uint32_t bits = drop_fin(km_s[qt * 64 + qs * 32 + (reg & 3) + 8 * (reg >> 2) + qsel] ^ ck);
            const uint32_t other = dpp_xor1(bits);
            f0 = keep_factor(odd ? other : bits, key & 1, dp);
            f1 = keep_factor(odd ? bits : other, key & 1, dp);
          }
        }
        pd[reg] = p0 * f0;
        pd[reg + 1] = p1 * f1;
        ds[reg] = p0 * fmaf(dpacc[reg], f0, -del[0]);
        ds[reg + 1] = p1 * fmaf(dpacc[reg + 1], f1, -del[1]);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pb = pack8(pd, s);
        const bf16x8 sb = pack8(ds, s);
        dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(dOs, qs * 32, s, 0, lane), pb, dv0, 0, 0, 0);
        dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(dOs, qs * 32, s, 1, lane), pb, dv1, 0, 0, 0);
        dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(Qs, qs * 32, s, 0, lane), sb, dk0, 0, 0, 0);
        dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(Qs, qs * 32, s, 1, lane), sb, dk1, 0, 0, 0);
      }
    }
  };
#pragma unroll 1
  for (int t = 0, stg = 0; t < nt; ++t, stg = stg == NSTG - 1 ? 0 : stg + 1) tile(stg, t);
  __syncthreads();  // Q images no longer read: reuse as staging
  bf16_t* stg_w = Qb + wave * 32 * D;
  const int64_t roff = ((int64_t)b * S + k0) * ld + hh * D;
  bf16_t* rowbase = dqkv + roff;
  // fp8 copy of dqkv (the fp8 QKV dgrad's A operand; delayed scaling, format qfmt)
  uint8_t* q8b = q8o.q != nullptr ? q8o.q + roff : nullptr;
  float qs = 0.f, qm = 0.f;
  if (q8b != nullptr) qs = fmt_scale(qfmt, *q8o.amax_in);
  store_rows(stg_w, dv0, dv1, 1.0f, rowbase + 2 * H, ld, lane, dbias ? bsum + (4 + wave) * D : nullptr,
             q8b ? q8b + 2 * H : nullptr, qfmt, qs, &qm, q8o.only != 0);
  store_rows(stg_w, dk0, dk1, scale, rowbase + H, ld, lane, dbias ? bsum + wave * D : nullptr,
             q8b ? q8b + H : nullptr, qfmt, qs, &qm, q8o.only != 0);
  if (q8b != nullptr) wave_amax_track(qm, q8o.amax_track);
  if (dbias) {
    __syncthreads();
    if (tid < 2 * D) {
      const int which = tid / D, c = tid % D;
      const float* p = bsum + which * 4 * D + c;
      atomicAdd(dbias + (1 + which) * H + hh * D + c, p[0] + p[D] + p[2 * D] + p[3 * D]);
    }
  }
}

// ------------------------------------------------------------------------------------------------
template <bool DROP, bool KM = false>
__global__ __launch_bounds__(256, 2) void attnS_bwd_q_kernel(const bf16_t* __restrict__ qkv,
                                                             const float* __restrict__ mask,
                                                             const bf16_t* __restrict__ dout,
                                                             const float* __restrict__ lse2,
                                                             const float* __restrict__ delta,
                                                             bf16_t* __restrict__ dqkv, float* __restrict__ dbias,
                                                             int S, int heads, float sl2, float scale,
                                                             DropoutParams dp, Q8Out q8o, int qfmt,
                                                             const uint32_t* __restrict__ kmask) {
  dp = resolve_seed(dp);
  // [K0 K1 K2 | V0 V1 V2 | mask bias | q bias partials | keep-mask words]; after the loop K0|K1 is the output staging
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * NSTG * TILE + 2 * kMaxS + 2 * 4 * D + 2 * 4 * kMaxS];
  bf16_t* Kb = lds;
  bf16_t* Vb = lds + NSTG * TILE;
  float* mb_s = reinterpret_cast<float*>(lds + 2 * NSTG * TILE);
  float* bsum = mb_s + kMaxS;  // [4 waves][64]
  uint32_t* km_s = reinterpret_cast<uint32_t*>(bsum + 4 * D);  // [4 waves' query blocks][S keys]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int bh = blockIdx.y, b = bh / heads, hh = bh % heads;
  const int H = heads * D, ld = 3 * H;
  const bf16_t* base = qkv + (int64_t)b * S * ld + hh * D;
  const int q0 = blockIdx.x * 128 + wave * 32;
  const int q = q0 + r;
  const int nt = S / 64;
  HSD_DASSERT(S % 64 == 0 && S <= kMaxS && q < S);

  dma_tile(Kb, base + H, ld, wave, lane);
  dma_tile(Vb, base + 2 * H, ld, wave, lane);
  bf16x8 qf[4], df[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = *reinterpret_cast<const bf16x8*>(base + (int64_t)q * ld + 16 * s + 8 * hf);
    df[s] = *reinterpret_cast<const bf16x8*>(dout + ((int64_t)b * S + q) * H + hh * D + 16 * s + 8 * hf);
  }
  const float lse_q = lse2[(int64_t)bh * S + q];
  const float del_q = delta[(int64_t)bh * S + q];
  for (int k = tid; k < S; k += 256) mb_s[k] = mask ? fmaxf(mask[(int64_t)b * S + k] * kLog2e, -1e30f) : 0.f;
  constexpr bool km_on = DROP && KM;  // the forward's keep bits are read (compile-time: no per-register branch)
  if constexpr (km_on) {
    const uint32_t* src = kmask + ((int64_t)bh * (S / 32) + blockIdx.x * 4) * S;  // the 4 query blocks, contiguous
    for (int i = tid; i < 4 * S; i += 256) km_s[i] = src[i];
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    settle(qf[s]);
    settle(df[s]);
  }
  settle(lse_q);
  settle(del_q);
  if (nt > 1) {
    dma_tile(Kb + TILE, base + 64 * ld + H, ld, wave, lane);
    dma_tile(Vb + TILE, base + 64 * ld + 2 * H, ld, wave, lane);
  }

  f32x16 dq0 = {}, dq1 = {};
  // dropout (re-hashing): as the forward -- row word of (bh, q) with the hf term folded in, C(32 kt) by readlane
  uint32_t xq = 0, ctile = 0;
  if (DROP && !km_on) {
    xq = dropout_row((uint32_t)(bh * S + q), dp) ^ drop_col(2u * (uint32_t)hf);
    ctile = drop_col(32u * (uint32_t)lane);
  }
  auto tile = [&](const int stg, const int kt) {

    if (kt + 1 < nt) tile_barrier<1>();
    else tile_barrier<0>();
    const bf16_t* Ks = Kb + stg * TILE;
    const bf16_t* Vs = Vb + stg * TILE;
    if (kt + 2 < nt) {
      const int s2 = stg == 0 ? 2 : stg - 1;
      const int64_t off = (int64_t)(kt + 2) * 64 * ld;
      dma_tile(Kb + s2 * TILE, base + off + H, ld, wave, lane);
      dma_tile(Vb + s2 * TILE, base + off + 2 * H, ld, wave, lane);
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      // Sᵀ[key][q] = K·Qᵀ, dPᵀ[key][q] = V·dOᵀ (query on the lane, key in the registers)
      f32x16 sacc = {}, dpacc = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 ak = *reinterpret_cast<const bf16x8*>(Ks + toff(kb * 32 + r, 16 * s + 8 * hf));
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ak, qf[s], sacc, 0, 0, 0);
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(Vs + toff(kb * 32 + r, 16 * s + 8 * hf));
        dpacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, df[s], dpacc, 0, 0, 0);
      }
      f32x16 ds;
      const uint32_t xt = DROP && !km_on ? xq ^ (uint32_t)__builtin_amdgcn_readlane((int)ctile, kt) : 0u;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int kk = kt * 64 + kb * 32 + 8 * g4 + 4 * hf;  // keys kk .. kk+3 in regs 4g4 .. 4g4+3
        const f32x4 mb = *reinterpret_cast<const f32x4*>(mb_s + kk);
        // keep-mask words of keys kk .. kk+3 for this wave's query block: bit r = this lane's query
        const u32x4 kw4 = km_on ? *reinterpret_cast<const u32x4*>(km_s + wave * S + kk) : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const int reg = 4 * g4 + e;
          const float p0 = __builtin_amdgcn_exp2f(fmaf(sacc[reg], sl2, mb[e]) - lse_q);
          const float p1 = __builtin_amdgcn_exp2f(fmaf(sacc[reg + 1], sl2, mb[e + 1]) - lse_q);
          float f0 = 1.f, f1 = 1.f;
          if constexpr (DROP) {
            if constexpr (km_on) {
              f0 = __uint_as_float((uint32_t)__builtin_amdgcn_sbfe((int)kw4[e], r, 1) & __float_as_uint(dp.scale));
              f1 = __uint_as_float((uint32_t)__builtin_amdgcn_sbfe((int)kw4[e + 1], r, 1) & __float_as_uint(dp.scale));
            } else {
              const uint32_t bits = drop_fin(xt ^ drop_col((uint32_t)(16 * kb + 4 * g4 + (e >> 1))));
              f0 = keep_factor(bits, 0, dp);
              f1 = keep_factor(bits, 1, dp);
            }
          }
          ds[reg] = p0 * fmaf(dpacc[reg], f0, -del_q);
          ds[reg + 1] = p1 * fmaf(dpacc[reg + 1], f1, -del_q);
        }
      }
      // dQᵀ[d][q] += Σ_key Kᵀ[d][key] dSᵀ[key][q]
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 sb = pack8(ds, s);
        dq0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(Ks, kb * 32, s, 0, lane), sb, dq0, 0, 0, 0);
        dq1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(Ks, kb * 32, s, 1, lane), sb, dq1, 0, 0, 0);
      }
    }
  };
#pragma unroll 1
  for (int t = 0, stg = 0; t < nt; ++t, stg = stg == NSTG - 1 ? 0 : stg + 1) tile(stg, t);
  __syncthreads();  // K images no longer read: reuse as staging
  const int64_t qoff = ((int64_t)b * S + q0) * ld + hh * D;
  float qs = 0.f, qm = 0.f;
  if (q8o.q != nullptr) {
    qs = fmt_scale(qfmt, *q8o.amax_in);
    if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) *q8o.sinv = 1.0f / qs;
  }
  store_rows(Kb + wave * 32 * D, dq0, dq1, scale, dqkv + qoff, ld, lane, dbias ? bsum + wave * D : nullptr,
             q8o.q != nullptr ? q8o.q + qoff : nullptr, qfmt, qs, &qm, q8o.only != 0);
  if (q8o.q != nullptr) wave_amax_track(qm, q8o.amax_track);
  if (dbias) {
    __syncthreads();
    if (tid < D) atomicAdd(dbias + hh * D + tid, bsum[tid] + bsum[D + tid] + bsum[2 * D + tid] + bsum[3 * D + tid]);
  }
}

}  // namespace aS

bool attnS_supported(int S, int head_dim) {
  return head_dim == attn::D && S % 128 == 0 && S >= 256 && S <= aS::kMaxS;
}

void launch_attnS_fwd(const bf16_t* qkv, const float* mask, bf16_t* out, float* lse2, int B, int S, int heads,
                      double p, uint64_t seed, hipStream_t st, Q8Out q8o, uint32_t* kmask) {
  DropoutParams dp = make_dropout(p, seed);
  const float sl2 = attn::kLog2e / sqrtf((float)attn::D);
  if (dp.enabled && kmask != nullptr)
    hipLaunchKernelGGL((aS::attnS_fwd_kernel<true, true>), dim3(S / 128, B * heads), dim3(256), 0, st, qkv, mask, out,
                       lse2, S, heads, sl2, dp, q8o, kmask);
  else if (dp.enabled)
    hipLaunchKernelGGL((aS::attnS_fwd_kernel<true, false>), dim3(S / 128, B * heads), dim3(256), 0, st, qkv, mask, out,
                       lse2, S, heads, sl2, dp, q8o, (uint32_t*)nullptr);
  else
    hipLaunchKernelGGL(aS::attnS_fwd_kernel<false>, dim3(S / 128, B * heads), dim3(256), 0, st, qkv, mask, out, lse2, S,
                       heads, sl2, dp, q8o, (uint32_t*)nullptr);
  HSD_CHECK_LAUNCH();
}

// delta_ws: fp32 [B*heads*S] scratch; delta_ready: it already holds the delta rows (written by the out-projection
// dgrad's E2_STORE_RDOT epilogue, ops/hip.py), so the delta pass is skipped
void launch_attnS_bwd(const bf16_t* qkv, const float* mask, const bf16_t* o, const bf16_t* dout, const float* lse2,
                      bf16_t* dqkv, float* delta_ws, float* dbias, int B, int S, int heads, double p, uint64_t seed,
                      hipStream_t st, Q8Out q8o, int qfmt, const uint32_t* kmask, bool delta_ready) {
  DropoutParams dp = make_dropout(p, seed);
  const float sl2 = attn::kLog2e / sqrtf((float)attn::D);
  const float scale = 1.0f / sqrtf((float)attn::D);
  if (!delta_ready) {
    hipLaunchKernelGGL(aS::attnS_delta_kernel, dim3(S / 32, B * heads), dim3(256), 0, st, o, dout, delta_ws, S, heads);
    HSD_CHECK_LAUNCH();
  }
  if (dp.enabled && kmask != nullptr) {
    hipLaunchKernelGGL((aS::attnS_bwd_kv_kernel<true, true>), dim3(S / 128, B * heads), dim3(256), 0, st, qkv, mask,
                       dout, lse2, delta_ws, dqkv, dbias, S, heads, sl2, scale, dp, q8o, qfmt, kmask);
    HSD_CHECK_LAUNCH();
    hipLaunchKernelGGL((aS::attnS_bwd_q_kernel<true, true>), dim3(S / 128, B * heads), dim3(256), 0, st, qkv, mask,
                       dout, lse2, delta_ws, dqkv, dbias, S, heads, sl2, scale, dp, q8o, qfmt, kmask);
  } else if (dp.enabled) {
    hipLaunchKernelGGL((aS::attnS_bwd_kv_kernel<true, false>), dim3(S / 128, B * heads), dim3(256), 0, st, qkv, mask,
                       dout, lse2, delta_ws, dqkv, dbias, S, heads, sl2, scale, dp, q8o, qfmt, nullptr);
    HSD_CHECK_LAUNCH();
    hipLaunchKernelGGL((aS::attnS_bwd_q_kernel<true, false>), dim3(S / 128, B * heads), dim3(256), 0, st, qkv, mask,
                       dout, lse2, delta_ws, dqkv, dbias, S, heads, sl2, scale, dp, q8o, qfmt, nullptr);
  } else {
    hipLaunchKernelGGL(aS::attnS_bwd_kv_kernel<false>, dim3(S / 128, B * heads), dim3(256), 0, st, qkv, mask, dout,
                       lse2, delta_ws, dqkv, dbias, S, heads, sl2, scale, dp, q8o, qfmt, nullptr);
    HSD_CHECK_LAUNCH();
    hipLaunchKernelGGL(aS::attnS_bwd_q_kernel<false>, dim3(S / 128, B * heads), dim3(256), 0, st, qkv, mask, dout,
                       lse2, delta_ws, dqkv, dbias, S, heads, sl2, scale, dp, q8o, qfmt, nullptr);
  }
  HSD_CHECK_LAUNCH();
}

// fp8 variants for the fp8 GEMM path (ops/hip.py): the forward also writes the output's e4m3 copy (the out-projection
// GEMM's A operand), the backward dqkv's copy in format qfmt (the QKV dgrad's A operand); delayed-scaling sites
void launch_attnS_fwd_q8(const bf16_t* qkv, const float* mask, bf16_t* out, float* lse2, int B, int S, int heads,
                         double p, uint64_t seed, uint8_t* q8, const float* amax_in, float* sinv, float* amax_track,
                         hipStream_t st, uint32_t* kmask) {
  launch_attnS_fwd(qkv, mask, out, lse2, B, S, heads, p, seed, st, Q8Out{q8, amax_in, sinv, amax_track}, kmask);
}

void launch_attnS_bwd_q8(const bf16_t* qkv, const float* mask, const bf16_t* o, const bf16_t* dout, const float* lse2,
                         bf16_t* dqkv, float* delta_ws, float* dbias, int B, int S, int heads, double p, uint64_t seed,
                         uint8_t* q8, const float* amax_in, float* sinv, float* amax_track, int qfmt, hipStream_t st,
                         const uint32_t* kmask, bool delta_ready, bool q8_only) {
  launch_attnS_bwd(qkv, mask, o, dout, lse2, dqkv, delta_ws, dbias, B, S, heads, p, seed, st,
                   Q8Out{q8, amax_in, sinv, amax_track, q8_only ? 1 : 0}, qfmt, kmask, delta_ready);
}

}  // namespace hsd
