// Flash-style fused self-attention for head_dim 64 on CDNA4 MFMA (v_mfma_f32_32x32x16_bf16).
// SURVEY.md §2.10 K4-K7 (forward) and K14 (backward); replaces TF's BatchMatMul + Softmax + dropout
// + BatchMatMul chain (S x S probabilities never touch HBM).
//
// Input  qkv [B*S, 3H] (the fused QKV GEMM output; q | k | v, head h at columns h*64), additive key
// mask bias [B, S] (0 / finfo.min, like HF's extended mask), dropout on the probabilities indexed as
// element ((b*heads + h)*S + q)*S + key of the site tensor (ops/rng.py).
//
// Forward: one workgroup = 4 waves = 128 queries of one (b, h); wave = 32 queries held on the MFMA
// lane ("swapped" QKᵀ: Sᵀ = K·Qᵀ, so each lane owns one query row and the softmax row-reduction is
// in-register + one lane^32 exchange — cdna_hip_programming.md T12 idea). K/V tiles of 64 keys are
// staged in LDS with an XOR swizzle that is conflict-free for both ds_read_b128 row reads and
// ds_read_b64_tr_b16 transposed reads (tools/lds_banks.py). P stays in registers: the Sᵀ accumulator
// is directly the B operand of Oᵀ = Vᵀ·Pᵀ (§3 'An accumulator tile as the next MFMA's operand').
// Saves lse2 = m + log2(l) (log2 domain, scores pre-scaled by log2(e)/√d) for the backward.
//
// Backward: one workgroup = 4 waves = 128 keys of one (b, h); wave = 32 keys on the lane, dKᵀ/dVᵀ
// accumulated in registers across all query blocks (no cross-workgroup sums for dK/dV); dS crosses
// LDS once for dQ. dQ is written directly when one workgroup covers all keys (S <= 128) and
// accumulated with fp32 atomics otherwise.
#include "common.h"
#include "fp8_common.h"
#include <stdlib.h>

namespace hsd {

constexpr int kD = 64;
constexpr float kLog2e = 1.4426950408889634f;

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

__device__ __forceinline__ int swz(int row) {  // bit-reverse of (row>>1)&7 : dual b128 / tr16 conflict-free
  const int t = (row >> 1) & 7;
  return ((t & 1) << 2) | (t & 2) | ((t >> 2) & 1);
}
// element offset of (row, col) in a [rows][64] bf16 LDS tile
__device__ __forceinline__ int toff(int row, int col) { return row * 64 + ((((col >> 3) ^ swz(row))) << 3) + (col & 7); }

__device__ __forceinline__ bf16x4 tr_read(const bf16_t* lds_base, int elem_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(lds_base + elem_off));
}

__device__ __forceinline__ bf16x8 cat8(bf16x4 a, bf16x4 b) {
  bf16x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

__device__ __forceinline__ bf16x8 pack8(const f32x16& acc, int s) {
  const u32x4 w = {pack_bf2(acc[8 * s], acc[8 * s + 1]), pack_bf2(acc[8 * s + 2], acc[8 * s + 3]),
                   pack_bf2(acc[8 * s + 4], acc[8 * s + 5]), pack_bf2(acc[8 * s + 6], acc[8 * s + 7])};
  return __builtin_bit_cast(bf16x8, w);
}

// A-operand (transposed) fragment for Oᵀ-style products: rows (keys/queries) of a [rows][64] tile taken
// in the accumulator's permuted k order: element j <-> row rb + 16s + 8(j>>2) + 4h + (j&3), column c.
__device__ __forceinline__ bf16x8 trA(const bf16_t* tile, int rb, int s, int colblk, int lane) {
  const int g = lane >> 4, i = lane & 15, h = g >> 1;
  const int q = i >> 2, p = i & 3;
  const int col = colblk * 32 + 16 * (g & 1) + 4 * p;
  const int r0 = rb + 16 * s + 4 * h + q;
  return cat8(tr_read(tile, toff(r0, col)), tr_read(tile, toff(r0 + 8, col)));
}

__device__ __forceinline__ float mask_bias2(const float* mask, int b, int S, int key) {
  if (key >= S) return -INFINITY;
  if (!mask) return 0.f;
  return fmaxf(mask[(size_t)b * S + key] * kLog2e, -1e30f);
}

// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void attn_fwd_kernel(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                                                       bf16_t* __restrict__ out, float* __restrict__ lse2,
                                                       int S, int heads, float sl2, DropoutParams dp) {
  dp = resolve_seed(dp);
  __shared__ __attribute__((aligned(16))) bf16_t Ks[64 * kD];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[64 * kD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hf = lane >> 5;
  const int bh = blockIdx.y, b = bh / heads, hh = bh % heads;
  const int H = heads * kD, ld = 3 * H;
  const int q = blockIdx.x * 128 + wave * 32 + r;
  const int qc = min(q, S - 1);
  const bf16_t* base = qkv + (size_t)b * S * ld;

  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(base + (size_t)qc * ld + hh * kD + 16 * s + 8 * hf);

  f32x16 o0 = {}, o1 = {};
  float m = -INFINITY, l = 0.f;
  const int ntiles = (S + 63) / 64;
  for (int kt = 0; kt < ntiles; ++kt) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i, row = c >> 3, ch = c & 7;
      const int key = kt * 64 + row;
      u32x4 kv = {0, 0, 0, 0}, vv = {0, 0, 0, 0};
      if (key < S) {
        const bf16_t* src = base + (size_t)key * ld + hh * kD + ch * 8;
        kv = *reinterpret_cast<const u32x4*>(src + H);
        vv = *reinterpret_cast<const u32x4*>(src + 2 * H);
      }
      *reinterpret_cast<u32x4*>(Ks + toff(row, ch * 8)) = kv;
      *reinterpret_cast<u32x4*>(Vs + toff(row, ch * 8)) = vv;
    }
    __syncthreads();
    f32x16 st[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      st[kb] = f32x16{};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8 a = *reinterpret_cast<const bf16x8*>(Ks + toff(kb * 32 + r, 16 * s + 8 * hf));
        st[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[s], st[kb], 0, 0, 0);
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int key = kt * 64 + kb * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * hf;
        float x = st[kb][reg] * sl2 + mask_bias2(mask, b, S, key);
        st[kb][reg] = x;
        mx = fmaxf(mx, x);
      }
    mx = max_xor32(mx);
    const float mn = fmaxf(m, mx);
    const float alpha = exp2f(m - mn);  // m = -inf on the first tile -> 0
    float ls = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        float p = exp2f(st[kb][reg] - mn);
        ls += p;
        st[kb][reg] = p;
      }
    ls = sum_xor32(ls);
    l = l * alpha + ls;
    m = mn;
    o0 *= alpha;
    o1 *= alpha;
    if (dp.enabled) {
      // mask row bh S + qc, column pair key / 2 = 32 kt + 16 kb + 4 (reg >> 2) + (reg >> 1 & 1) + 2 hf (disjoint bits)
      const uint32_t xt = dropout_row((uint32_t)(bh * S + qc), dp) ^ drop_col(32u * (uint32_t)kt + 2u * (uint32_t)hf);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int reg = 0; reg < 16; reg += 2) {
          const uint32_t bits = drop_fin(xt ^ drop_col((uint32_t)(16 * kb + 4 * (reg >> 2) + ((reg >> 1) & 1))));
          st[kb][reg] *= keep_factor(bits, 0, dp);
          st[kb][reg + 1] *= keep_factor(bits, 1, dp);
        }
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pb = pack8(st[kb], s);
        o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(Vs, kb * 32, s, 0, lane), pb, o0, 0, 0, 0);
        o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(Vs, kb * 32, s, 1, lane), pb, o1, 0, 0, 0);
      }
  }
  if (q < S) {
    const float inv = 1.0f / l;
    bf16_t* dst = out + ((size_t)b * S + q) * H + hh * kD;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int d = 8 * i + 4 * hf;
      u32x2 w0, w1;
      w0.x = pack_bf2(o0[4 * i] * inv, o0[4 * i + 1] * inv);
      w0.y = pack_bf2(o0[4 * i + 2] * inv, o0[4 * i + 3] * inv);
      w1.x = pack_bf2(o1[4 * i] * inv, o1[4 * i + 1] * inv);
      w1.y = pack_bf2(o1[4 * i + 2] * inv, o1[4 * i + 3] * inv);
      *reinterpret_cast<u32x2*>(dst + d) = w0;
      *reinterpret_cast<u32x2*>(dst + 32 + d) = w1;
    }
    if (hf == 0) lse2[(size_t)bh * S + q] = m + log2f(l);
  }
}

// ------------------------------------------------------------------------------------------------
// dSt image: [128 keys][32 queries] bf16, 64-B rows, swizzle chunk ^ ((row>>2)&3)
__device__ __forceinline__ int soff(int row, int col) { return row * 32 + ((((col >> 3) ^ ((row >> 2) & 3))) << 3) + (col & 7); }

__global__ __launch_bounds__(256) void attn_bwd_kernel(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                                                       const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout,
                                                       const float* __restrict__ lse2, bf16_t* __restrict__ dqkv,
                                                       float* __restrict__ dq_acc, int S, int heads, float sl2,
                                                       float scale, DropoutParams dp) {
  dp = resolve_seed(dp);
  __shared__ __attribute__((aligned(16))) bf16_t Qs[32 * kD];
  __shared__ __attribute__((aligned(16))) bf16_t dOs[32 * kD];
  __shared__ __attribute__((aligned(16))) bf16_t Kall[128 * kD];
  __shared__ __attribute__((aligned(16))) bf16_t dSt[128 * 32];
  __shared__ float lse_s[32], del_s[32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hf = lane >> 5;
  const int bh = blockIdx.y, b = bh / heads, hh = bh % heads;
  const int H = heads * kD, ld = 3 * H;
  const int kbase = blockIdx.x * 128;
  const int key = kbase + wave * 32 + r;
  const int kc = min(key, S - 1);
  const uint32_t ck = drop_col((uint32_t)kc >> 1);  // dropout column word of this lane's key
  const bf16_t* base = qkv + (size_t)b * S * ld;

  // per-wave K and V B-fragments (key on the lane)
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = *reinterpret_cast<const bf16x8*>(base + (size_t)kc * ld + H + hh * kD + 16 * s + 8 * hf);
    vf[s] = *reinterpret_cast<const bf16x8*>(base + (size_t)kc * ld + 2 * H + hh * kD + 16 * s + 8 * hf);
  }
  // all 128 keys of this workgroup into LDS (for dQ)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i, row = c >> 3, ch = c & 7;
    const int kk = kbase + row;
    u32x4 kv = {0, 0, 0, 0};
    if (kk < S) kv = *reinterpret_cast<const u32x4*>(base + (size_t)kk * ld + H + hh * kD + ch * 8);
    *reinterpret_cast<u32x4*>(Kall + toff(row, ch * 8)) = kv;
  }
  const float kb2 = mask_bias2(mask, b, S, key);
  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
  const bool single = S <= 128;
  const int nqb = (S + 31) / 32;
  for (int qb = 0; qb < nqb; ++qb) {
    __syncthreads();
    {
      // Q / dO tiles (32 rows x 8 chunks = 256 chunks: one per thread), lse, delta = rowsum(dO*O)
      const int row = tid >> 3, ch = tid & 7;
      const int qq = qb * 32 + row;
      u32x4 qv = {0, 0, 0, 0}, dv = {0, 0, 0, 0}, ov = {0, 0, 0, 0};
      if (qq < S) {
        qv = *reinterpret_cast<const u32x4*>(base + (size_t)qq * ld + hh * kD + ch * 8);
        const size_t oo = ((size_t)b * S + qq) * H + hh * kD + ch * 8;
        dv = *reinterpret_cast<const u32x4*>(dout + oo);
        ov = *reinterpret_cast<const u32x4*>(o + oo);
      }
      *reinterpret_cast<u32x4*>(Qs + toff(row, ch * 8)) = qv;
      *reinterpret_cast<u32x4*>(dOs + toff(row, ch * 8)) = dv;
      float part = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) part += lo_bf(dv[k]) * lo_bf(ov[k]) + hi_bf(dv[k]) * hi_bf(ov[k]);
      part = sum8_dpp(part);
      if (ch == 0) {
        del_s[row] = part;
        lse_s[row] = qq < S ? lse2[(size_t)bh * S + qq] : 0.f;
      }
    }
    __syncthreads();
    f32x16 sacc = {}, dpacc = {};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 aq = *reinterpret_cast<const bf16x8*>(Qs + toff(r, 16 * s + 8 * hf));
      sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aq, kf[s], sacc, 0, 0, 0);
      bf16x8 ad = *reinterpret_cast<const bf16x8*>(dOs + toff(r, 16 * s + 8 * hf));
      dpacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ad, vf[s], dpacc, 0, 0, 0);
    }
    // sacc/dpacc: col = key (lane), row qi = (reg&3) + 8*(reg>>2) + 4*hf
    f32x16 pd, ds;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int qi = (reg & 3) + 8 * (reg >> 2) + 4 * hf;
      const int qq = qb * 32 + qi;
      float p = (qq < S) ? exp2f(sacc[reg] * sl2 + kb2 - lse_s[qi]) : 0.f;
      float kf_ = 1.0f;
      if (dp.enabled) {
        kf_ = keep_factor(drop_fin(dropout_row((uint32_t)(bh * S + min(qq, S - 1)), dp) ^ ck), kc & 1, dp);
      }
      pd[reg] = p * kf_;
      ds[reg] = p * (dpacc[reg] * kf_ - del_s[qi]);
    }
    // dVᵀ += dOᵀ · Pd ; dKᵀ += Qᵀ · dS   (B operands straight from the accumulators)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 pb = pack8(pd, s);
      bf16x8 sb = pack8(ds, s);
      dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(dOs, 0, s, 0, lane), pb, dv0, 0, 0, 0);
      dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(dOs, 0, s, 1, lane), pb, dv1, 0, 0, 0);
      dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(Qs, 0, s, 0, lane), sb, dk0, 0, 0, 0);
      dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(Qs, 0, s, 1, lane), sb, dk1, 0, 0, 0);
    }
    // dS -> LDS as [key][q] (4 consecutive q per register quad)
    {
      const int krow = wave * 32 + r;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        u32x2 w;
        w.x = pack_bf2(ds[4 * i], ds[4 * i + 1]);
        w.y = pack_bf2(ds[4 * i + 2], ds[4 * i + 3]);
        *reinterpret_cast<u32x2*>(dSt + soff(krow, 8 * i + 4 * hf)) = w;
      }
    }
    __syncthreads();
    if (wave < 2) {
      // dQᵀ[d][q] = Σ_key Kᵀ[d][key] · dSᵀ[key][q] over the 128 keys; wave w = d-block w
      f32x16 dq = {};
      const int g = lane >> 4, i = lane & 15, h = g >> 1, qd = i >> 2, p = i & 3;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int r0 = 16 * s + 4 * h + qd;
        const int colk = wave * 32 + 16 * (g & 1) + 4 * p;
        bf16x8 a = cat8(tr_read(Kall, toff(r0, colk)), tr_read(Kall, toff(r0 + 8, colk)));
        const int colq = 16 * (g & 1) + 4 * p;
        bf16x8 bb = cat8(tr_read(dSt, soff(r0, colq)), tr_read(dSt, soff(r0 + 8, colq)));
        dq = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bb, dq, 0, 0, 0);
      }
      // dq: col = q (lane&31), rows d = wave*32 + (reg&3) + 8*(reg>>2) + 4*hf
      const int qq = qb * 32 + r;
      if (qq < S) {
        if (single) {
          bf16_t* dst = dqkv + ((size_t)b * S + qq) * ld + hh * kD + wave * 32;
#pragma unroll
          for (int ii = 0; ii < 4; ++ii) {
            u32x2 w;
            w.x = pack_bf2(dq[4 * ii] * scale, dq[4 * ii + 1] * scale);
            w.y = pack_bf2(dq[4 * ii + 2] * scale, dq[4 * ii + 3] * scale);
            *reinterpret_cast<u32x2*>(dst + 8 * ii + 4 * hf) = w;
          }
        } else {
          float* dst = dq_acc + ((size_t)b * S + qq) * H + hh * kD + wave * 32;
#pragma unroll
          for (int reg = 0; reg < 16; ++reg) atomicAdd(dst + (reg & 3) + 8 * (reg >> 2) + 4 * hf, dq[reg] * scale);
        }
      }
    }
  }
  if (key < S) {
    bf16_t* dk = dqkv + ((size_t)b * S + key) * ld + H + hh * kD;
    bf16_t* dvp = dqkv + ((size_t)b * S + key) * ld + 2 * H + hh * kD;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int d = 8 * i + 4 * hf;
      u32x2 w;
      w.x = pack_bf2(dk0[4 * i] * scale, dk0[4 * i + 1] * scale);
      w.y = pack_bf2(dk0[4 * i + 2] * scale, dk0[4 * i + 3] * scale);
      *reinterpret_cast<u32x2*>(dk + d) = w;
      w.x = pack_bf2(dk1[4 * i] * scale, dk1[4 * i + 1] * scale);
      w.y = pack_bf2(dk1[4 * i + 2] * scale, dk1[4 * i + 3] * scale);
      *reinterpret_cast<u32x2*>(dk + 32 + d) = w;
      w.x = pack_bf2(dv0[4 * i], dv0[4 * i + 1]);
      w.y = pack_bf2(dv0[4 * i + 2], dv0[4 * i + 3]);
      *reinterpret_cast<u32x2*>(dvp + d) = w;
      w.x = pack_bf2(dv1[4 * i], dv1[4 * i + 1]);
      w.y = pack_bf2(dv1[4 * i + 2], dv1[4 * i + 3]);
      *reinterpret_cast<u32x2*>(dvp + 32 + d) = w;
    }
  }
}

// dq_acc (fp32 [T, H]) -> dqkv q-columns (bf16), for S > 128
__global__ __launch_bounds__(256) void dq_convert_kernel(const float* __restrict__ acc, bf16_t* __restrict__ dqkv, int T,
                                                         int H) {
  const int64_t n4 = (int64_t)T * H / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const int64_t e = i * 4, t = e / H, c = e % H;
    f32x4 v = reinterpret_cast<const f32x4*>(acc)[i];
    u32x2 w;
    w.x = pack_bf2(v[0], v[1]);
    w.y = pack_bf2(v[2], v[3]);
    *reinterpret_cast<u32x2*>(dqkv + t * 3 * H + c) = w;
  }
}

bool attn128_supported(int S, int head_dim);
void launch_attn128_fwd(const bf16_t* qkv, const float* mask, bf16_t* out, float* lse2, int B, int heads, double p,
                        uint64_t seed, hipStream_t st);
void launch_attn128_bwd(const bf16_t* qkv, const float* mask, const bf16_t* o, const bf16_t* dout, const float* lse2,
                        bf16_t* dqkv, float* dbias, int B, int heads, double p, uint64_t seed, hipStream_t st);
void launch_colsum(const bf16_t* x, float* dbias, int rows, int N, hipStream_t st);
bool attnS_supported(int S, int head_dim);
void launch_attnS_fwd(const bf16_t* qkv, const float* mask, bf16_t* out, float* lse2, int B, int S, int heads,
                      double p, uint64_t seed, hipStream_t st, Q8Out q8o, uint32_t* kmask);
void launch_attnS_bwd(const bf16_t* qkv, const float* mask, const bf16_t* o, const bf16_t* dout, const float* lse2,
                      bf16_t* dqkv, float* delta_ws, float* dbias, int B, int S, int heads, double p, uint64_t seed,
                      hipStream_t st, Q8Out q8o, int qfmt, const uint32_t* kmask, bool delta_ready);

// Tests only (attn_set_force_generic, tests/test_gpu_ops.py): route every S to the tiled generic kernels below, the
// independent implementation the S = 128 / streaming kernels are checked against. Not an environment knob.
static bool g_attn_force_generic = false;
void attn_set_force_generic(bool on) { g_attn_force_generic = on; }

// S in 256..1024 (multiple of 128) runs the streaming kernels of attentionS.hip; its backward takes
// an fp32 [B*heads*S] scratch (no zeroing) where the generic kernel takes a zeroed [B*S, H] dq accumulator.
bool attn_streaming(int S) { return attnS_supported(S, kD) && !g_attn_force_generic; }

// the streaming (S > 128) kernels only: at S = 128 the one-workgroup forward is memory-bound with four workgroups per
// CU, and writing the bits cost it more (+27 us at bert-base B = 1024, plus a lost workgroup per CU) than the
// backward saved (-26 us; profiles/attn_keep_mask_ab_r4.log)
bool attn_keep_mask_supported(int S) { return attn_streaming(S); }
// words of the keep mask per launch: [B*heads][S/32 query blocks][S keys]
int64_t attn_keep_mask_numel(int B, int S, int heads) {
  return attn_keep_mask_supported(S) ? (int64_t)B * heads * (S / 32) * S : 0;
}

void launch_attn_fwd(const bf16_t* qkv, const float* mask, bf16_t* out, float* lse2, int B, int S, int heads,
                     double p, uint64_t seed, hipStream_t st, uint32_t* kmask) {
  if (attn128_supported(S, kD) && !g_attn_force_generic) {
    launch_attn128_fwd(qkv, mask, out, lse2, B, heads, p, seed, st);
    return;
  }
  if (attn_streaming(S)) {
    launch_attnS_fwd(qkv, mask, out, lse2, B, S, heads, p, seed, st, Q8Out{}, kmask);
    return;
  }
  DropoutParams dp = make_dropout(p, seed);
  const float sl2 = kLog2e / sqrtf((float)kD);
  dim3 grid((S + 127) / 128, B * heads);
  hipLaunchKernelGGL(attn_fwd_kernel, grid, dim3(256), 0, st, qkv, mask, out, lse2, S, heads, sl2, dp);
  HSD_CHECK_LAUNCH();
}

void launch_attn_bwd(const bf16_t* qkv, const float* mask, const bf16_t* o, const bf16_t* dout, const float* lse2,
                     bf16_t* dqkv, float* dq_acc, float* dbias, int B, int S, int heads, double p, uint64_t seed,
                     hipStream_t st, const uint32_t* kmask, bool delta_ready) {
  if (attn128_supported(S, kD) && !g_attn_force_generic) {
    launch_attn128_bwd(qkv, mask, o, dout, lse2, dqkv, dbias, B, heads, p, seed, st);
    return;
  }
  if (attn_streaming(S)) {
    launch_attnS_bwd(qkv, mask, o, dout, lse2, dqkv, dq_acc, dbias, B, S, heads, p, seed, st, Q8Out{}, 0, kmask,
                     delta_ready);
    return;
  }
  DropoutParams dp = make_dropout(p, seed);
  const float sl2 = kLog2e / sqrtf((float)kD);
  const float scale = 1.0f / sqrtf((float)kD);
  dim3 grid((S + 127) / 128, B * heads);
  hipLaunchKernelGGL(attn_bwd_kernel, grid, dim3(256), 0, st, qkv, mask, o, dout, lse2, dqkv, dq_acc, S, heads, sl2,
                     scale, dp);
  HSD_CHECK_LAUNCH();
  if (S > 128) {
    const int T = B * S, H = heads * kD;
    int64_t n4 = (int64_t)T * H / 4;
    int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
    hipLaunchKernelGGL(dq_convert_kernel, dim3(blocks), dim3(256), 0, st, dq_acc, dqkv, T, H);
    HSD_CHECK_LAUNCH();
  }
  if (dbias) launch_colsum(dqkv, dbias, B * S, 3 * heads * kD, st);
}

}  // namespace hsd
