// Self-attention for S == 128, head_dim 64 (the headline BERT-base seq-128 config; SURVEY.md §2.10
// K4-K7 forward, K14 backward): ONE workgroup per (batch, head) holds the whole 128x128 problem, so
// Q/K/V/dO are read from HBM exactly once and probabilities never leave registers; the forward synchronises
// once after the operand DMA, the backward once per query block (below) plus its phase changes.
//
// * operands are staged HBM -> LDS with global_load_lds_dwordx4 (1 KiB per wave instruction) into
//   [128][64] bf16 images whose 16-B chunks are XOR-swizzled (chunk ^ bitrev3((row>>1)&7)) — the
//   swizzle is applied to the per-lane SOURCE address so the DMA destination stays lane-linear
//   (cdna_hip_programming.md rule 21); the image is conflict-free for ds_read_b128 row reads AND
//   ds_read_b64_tr_b16 transposed reads.
// * forward: wave w owns queries 32w..32w+31 on the MFMA lanes ("swapped" Sᵀ = K·Qᵀ), all 128 keys in
//   its 64 accumulator registers -> exact (not online) softmax in registers, Oᵀ = Vᵀ·Pᵀ with the
//   accumulator as the B operand, O staged through a wave-private LDS slice to 128-B row stores.
// * backward: wave w owns keys 32w..32w+31 on the lanes; loops over 4 query blocks recomputing P from
//   the saved log-sum-exp, accumulates dKᵀ, dVᵀ in registers, writes dS once, then dQᵀ = Kᵀ·dSᵀ with wave w
//   owning queries 32w..32w+31. The dS of query block qb ([128 key][32 q], 64-B rows, 8-B units swizzled by key) is
//   written over the Q / dO rows of that block once every wave is past it (one barrier per block), K has its own
//   slot (re-read per block instead of held in VGPRs): 52.5 KiB of LDS and 168 VGPRs, three workgroups per CU (the
//   round-4 [128 key][128 q] dS image took 68.5 KiB, two per CU: 422 -> 371-376 us, profiles/attn128_bwd_v3_ab_r5.log).
//   The dropout hash of
//   a key pair is computed once per lane pair and exchanged (keys sit on adjacent lanes here).
// Dropout / mask / lse conventions are identical to attention.hip (ops/rng.py site indexing).
#include "attn_common.h"

namespace hsd {
namespace a128 {

constexpr int S = 128;
using namespace attn;

// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 4) void attn128_fwd_kernel(const bf16_t* __restrict__ qkv,
                                                             const float* __restrict__ mask, bf16_t* __restrict__ out,
                                                             float* __restrict__ lse2, int heads, float sl2,
                                                             DropoutParams dp) {
  dp = resolve_seed(dp);
  // [K | V | mask bias]; the output staging reuses K's slot after a barrier, so the 33 KiB footprint lets four
  // workgroups share a CU (122 VGPRs: four waves per SIMD) for more memory-level parallelism
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * S * D + 2 * S];
  bf16_t* Ks = lds;
  bf16_t* Vs = lds + S * D;
  bf16_t* stg_all = lds;
  float* mbias = reinterpret_cast<float*>(lds + 2 * S * D);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int bh = blockIdx.x, b = bh / heads, hh = bh % heads;
  const int H = heads * D, ld = 3 * H;
  const bf16_t* base = qkv + (int64_t)b * S * ld + hh * D;

  // K, V -> LDS (8 DMA instructions per wave), Q fragments -> registers, mask bias -> LDS
  dma_img(Ks, base + H, ld, wave * 4, 4, lane);
  dma_img(Vs, base + 2 * H, ld, wave * 4, 4, lane);
  const int q = wave * 32 + r;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(base + (int64_t)q * ld + 16 * s + 8 * hf);
  if (tid < S) mbias[tid] = mask ? fmaxf(mask[(int64_t)b * S + tid] * kLog2e, -1e30f) : 0.f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // Sᵀ[key][q]: 4 key blocks of 32
  f32x16 st[4];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    st[kb] = f32x16{};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(Ks + toff(kb * 32 + r, 16 * s + 8 * hf));
      st[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[s], st[kb], 0, 0, 0);
    }
  }
  // exact softmax over the 128 keys of this query (64 in-lane + the partner half-wave)
  float mx = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 mb = *reinterpret_cast<const f32x4*>(mbias + kb * 32 + 8 * g4 + 4 * hf);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = fmaf(st[kb][4 * g4 + e], sl2, mb[e]);
        st[kb][4 * g4 + e] = x;
        mx = fmaxf(mx, x);
      }
    }
  mx = max_xor32(mx);
  float l = 0.f;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const float p = __builtin_amdgcn_exp2f(st[kb][reg] - mx);
      l += p;
      st[kb][reg] = p;
    }
  l = sum_xor32(l);
  float oscale = 1.0f / l;
  if (dp.enabled) {
    // mask row bh S + q, column pair key / 2 = 16 kb + 4 (reg >> 2) + (reg >> 1 & 1) + 2 hf (disjoint bits): one row
    // word per lane, the hf term folded in, each register's C(...) a literal. P is kept or zeroed (the 1/(1-p) scale
    // rides on the output normalisation)
    const uint32_t xq = dropout_row((uint32_t)(bh * S + q), dp) ^ drop_col(2u * (uint32_t)hf);
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int reg = 0; reg < 16; reg += 2) {
        const uint32_t bits = drop_fin(xq ^ drop_col((uint32_t)(16 * kb + 4 * (reg >> 2) + ((reg >> 1) & 1))));
        st[kb][reg] = keep_lo(bits, dp.thr) ? st[kb][reg] : 0.f;
        st[kb][reg + 1] = keep_hi(bits, dp.thr) ? st[kb][reg + 1] : 0.f;
      }
    oscale *= dp.scale;
  }
  // Oᵀ[d][q] = Σ_key Vᵀ[d][key] Pᵀ[key][q]
  f32x16 o0 = {}, o1 = {};
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 pb = pack8(st[kb], s);
      o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(Vs, kb * 32, s, 0, lane), pb, o0, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(Vs, kb * 32, s, 1, lane), pb, o1, 0, 0, 0);
    }
  if (hf == 0) lse2[(int64_t)bh * S + q] = mx + __log2f(l);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // every wave's K reads done: K's slot becomes the output staging
  asm volatile("" ::: "memory");
  store_rows(stg_all + wave * 32 * D, o0, o1, oscale, out + ((int64_t)b * S + wave * 32) * H + hh * D, H, lane);
}

// ------------------------------------------------------------------------------------------------
// dS block image: the dS of query block qb, [128 keys][32 queries] bf16, lives in the dead rows of that block in the
// Q image (keys 0-63) and the dO image (keys 64-127): 64-B rows, 8-B unit u of key row k stored at u ^ ((k >> 1) & 7) --
// conflict-free for the b64 writes (16 consecutive keys per lane group) and for the dQ phase's tr reads (4 whole rows
// per 32 lanes)
__device__ __forceinline__ int dsoff(int key, int qc) {
  const int k = key & 63;
  return k * 32 + ((((qc >> 2) ^ (k >> 1)) & 7) << 2) + (qc & 3);
}

// dS of query block qb is written (one barrier per block) over the Q / dO rows of that block, which no wave reads
// again; K gets its own slot, written from the registers at the start, and serves as the output staging after the dQ
// phase: 52.5 KiB and <= 168 VGPRs, three workgroups (twelve waves) per CU.
template <bool DROP>
__global__ __launch_bounds__(256, 3) void attn128_bwd_kernel(const bf16_t* __restrict__ qkv,
                                                             const float* __restrict__ mask,
                                                             const bf16_t* __restrict__ o,
                                                             const bf16_t* __restrict__ dout,
                                                             const float* __restrict__ lse2,
                                                             bf16_t* __restrict__ dqkv, float* __restrict__ dbias,
                                                             int heads, float sl2, float scale, DropoutParams dp,
                                                             unsigned long long* __restrict__ diag) {
  dp = resolve_seed(dp);
  // diagnostic phase stamps (attn128_set_diag, tools/attn_phase_probe.py): start, operands landed, delta done, loop
  // done, dK / dV stored, end, and the real-time clock at start / end
  unsigned long long ts[6] = {0, 0, 0, 0, 0, 0}, rt0 = 0;
  if (diag) {
    ts[0] = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  // [Q | dO | K | lse | delta | bias-grad partials]; dS blocks go over dead Q / dO rows, K's slot is the output
  // staging after the dQ phase
  constexpr int kImg = 3 * S * D;
  __shared__ __attribute__((aligned(16))) bf16_t lds[kImg + 4 * S + 2 * 3 * 4 * D + 2 * S];
  bf16_t* Qs = lds;
  bf16_t* dOs = lds + S * D;
  bf16_t* dSt = lds + 2 * S * D;  // K's slot
  float* lse_s = reinterpret_cast<float*>(lds + kImg);
  float* del_s = lse_s + S;
  float* bsum = del_s + S;  // [3 (q,k,v)][4 waves][64]
  uint32_t* rw_s = reinterpret_cast<uint32_t*>(bsum + 3 * 4 * D);  // dropout row words R(bh S + q) of the 128 queries
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int bh = blockIdx.x, b = bh / heads, hh = bh % heads;
  const int H = heads * D, ld = 3 * H;
  const bf16_t* base = qkv + (int64_t)b * S * ld + hh * D;
  const bf16_t* obase = o + (int64_t)b * S * H + hh * D;
  const bf16_t* dobase = dout + (int64_t)b * S * H + hh * D;

  dma_img(Qs, base, ld, wave * 4, 4, lane);
  dma_img(dOs, dobase, H, wave * 4, 4, lane);
  const int key = wave * 32 + r;
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = *reinterpret_cast<const bf16x8*>(base + (int64_t)key * ld + H + 16 * s + 8 * hf);
    vf[s] = *reinterpret_cast<const bf16x8*>(base + (int64_t)key * ld + 2 * H + 16 * s + 8 * hf);
  }
  const float kb2 = mask ? fmaxf(mask[(int64_t)b * S + key] * kLog2e, -1e30f) : 0.f;
  // delta[q] = Σ_d dO[q][d]·O[q][d]: thread handles rows (tid>>3) + 32i, chunk tid&7. O comes from global memory
  // (loads issued here, under the DMA); dO from its LDS image once the DMA has landed -- dO is read from HBM once
  // (it used to be read a second time for this pre-pass: 16 of the 144 KiB a (batch, head) moves)
  u32x4 ov[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (tid >> 3) + 32 * i, c = tid & 7;
    ov[i] = *reinterpret_cast<const u32x4*>(obase + (int64_t)row * H + c * 8);
  }
  if (tid < S) lse_s[tid] = lse2[(int64_t)bh * S + tid];
  if constexpr (DROP) {
    if (tid < S) rw_s[tid] = dropout_row((uint32_t)(bh * S + tid), dp);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // K -> its own slot now (dQ phase operand); visible to every wave after the barriers below
#pragma unroll
  for (int s = 0; s < 4; ++s) *reinterpret_cast<bf16x8*>(dSt + toff(key, 16 * s + 8 * hf)) = kf[s];
  __syncthreads();
  if (diag) ts[1] = __builtin_amdgcn_s_memtime();
  {
    float part[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (tid >> 3) + 32 * i, c = tid & 7;
      const u32x4 dv = *reinterpret_cast<const u32x4*>(dOs + toff(row, c * 8));
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) acc += lo_bf(dv[k]) * lo_bf(ov[i][k]) + hi_bf(dv[k]) * hi_bf(ov[i][k]);
      part[i] = sum8_dpp(acc);
    }
    if ((tid & 7) == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) del_s[(tid >> 3) + 32 * i] = part[i];
    }
  }
  __syncthreads();
  if (diag) ts[2] = __builtin_amdgcn_s_memtime();

  f32x16 dk0 = {}, dk1 = {}, dv0 = {}, dv1 = {};
  const bool odd = (lane & 1) != 0;
  // per-lane LDS offsets of the query-block-0 fragments; block qb adds qb * 32 rows (the images' swizzles
  // depend on row bits 1..3 only, so they are the same for every block)
  int off_row[4], off_tr[2][2][2];
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) off_row[s4] = toff(r, 16 * s4 + 8 * hf);
  {
    const int g = lane >> 4, i = lane & 15, h = g >> 1, q = i >> 2, pp = i & 3;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int col = cb * 32 + 16 * (g & 1) + 4 * pp;
        const int r0 = 16 * s2 + 4 * h + q;
        off_tr[s2][cb][0] = toff(r0, col);
        off_tr[s2][cb][1] = toff(r0 + 8, col);
      }
  }
  // dropout: mask row bh S + query, column pair key / 2 -- the same 32-bit word for lanes l and l ^ 1 (keys 2j, 2j + 1):
  // the even lane computes query qi0's word, the odd lane query qi0 + 1's, and they swap (one DPP move)
  const uint32_t ck = drop_col((uint32_t)key >> 1);
  const int qsel = 4 * hf + (odd ? 1 : 0);
  // the previous block's packed dS, written after the next block's barrier
  u32x2 dsw[4];
  bf16_t* const dsb = key < 64 ? Qs : dOs;  // region of this wave's keys (wave-uniform)
  auto put_ds = [&](int blk) {
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<u32x2*>(dsb + blk * 32 * 64 + dsoff(key, 8 * i + 4 * hf)) = dsw[i];
  };
#pragma unroll 1
  for (int qb = 0; qb < 4; ++qb) {
    if (qb > 0) {
      __syncthreads();  // every wave is past block qb - 1: its Q / dO rows are dead
      put_ds(qb - 1);
    }
    const int qoff = qb * 32 * 64;  // element offset of the block's first row in a [rows][64] image
    f32x16 sacc = {}, dpacc = {};
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const bf16x8 aq = *reinterpret_cast<const bf16x8*>(Qs + qoff + off_row[s4]);
      // K fragments re-read from K's slot (16 VGPRs fewer across the loop)
      const bf16x8 kq = *reinterpret_cast<const bf16x8*>(dSt + toff(key, 16 * s4 + 8 * hf));
      sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aq, kq, sacc, 0, 0, 0);
      const bf16x8 ad = *reinterpret_cast<const bf16x8*>(dOs + qoff + off_row[s4]);
      dpacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ad, vf[s4], dpacc, 0, 0, 0);
    }
    // rows: query qi = (reg&3) + 8(reg>>2) + 4hf of the block; col (lane): key
    f32x16 pd, ds;
#pragma unroll
    for (int reg = 0; reg < 16; reg += 2) {
      const int qi0 = qb * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * hf;  // rows qi0, qi0 + 1
      const f32x2 lse = *reinterpret_cast<const f32x2*>(lse_s + qi0);
      const f32x2 del = *reinterpret_cast<const f32x2*>(del_s + qi0);
      const float p0 = __builtin_amdgcn_exp2f(fmaf(sacc[reg], sl2, kb2) - lse[0]);
      const float p1 = __builtin_amdgcn_exp2f(fmaf(sacc[reg + 1], sl2, kb2) - lse[1]);
      float k0 = 1.f, k1 = 1.f;
      if constexpr (DROP) {
        const uint32_t bits = drop_fin(rw_s[qb * 32 + (reg & 3) + 8 * (reg >> 2) + qsel] ^ ck);
        const uint32_t other = dpp_xor1(bits);
        const uint32_t b0 = odd ? other : bits;   // hash of row qi0
        const uint32_t b1 = odd ? bits : other;   // hash of row qi0 + 1
        k0 = keep_factor(b0, key & 1, dp);
        k1 = keep_factor(b1, key & 1, dp);
      }
      pd[reg] = p0 * k0;
      pd[reg + 1] = p1 * k1;
      ds[reg] = p0 * fmaf(dpacc[reg], k0, -del[0]);
      ds[reg + 1] = p1 * fmaf(dpacc[reg + 1], k1, -del[1]);
    }
    // dVᵀ += dOᵀ·Pd, dKᵀ += Qᵀ·dS  (accumulators as B operands, rows of the images in the same order)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pb = pack8(pd, s2);
      const bf16x8 sb = pack8(ds, s2);
      auto tr = [&](const bf16_t* img, int cb) {
        return cat8(tr_read(img, qoff + off_tr[s2][cb][0]), tr_read(img, qoff + off_tr[s2][cb][1]));
      };
      dv0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr(dOs, 0), pb, dv0, 0, 0, 0);
      dv1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr(dOs, 1), pb, dv1, 0, 0, 0);
      dk0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr(Qs, 0), sb, dk0, 0, 0, 0);
      dk1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr(Qs, 1), sb, dk1, 0, 0, 0);
    }
    // dS, packed: held until the next block's barrier
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      dsw[i].x = pack_bf2(ds[4 * i], ds[4 * i + 1]);
      dsw[i].y = pack_bf2(ds[4 * i + 2], ds[4 * i + 3]);
    }
  }
  {
    __syncthreads();  // every wave is past block 3
    put_ds(3);
    __syncthreads();  // every dS written
    if (diag) ts[3] = __builtin_amdgcn_s_memtime();
    // dQᵀ[d][q] = Σ_key Kᵀ[d][key] dSᵀ[key][q], wave w: queries 32w..32w+31 = dS block w
    f32x16 dq0 = {}, dq1 = {};
    {
      const int g = lane >> 4, i = lane & 15, h = g >> 1, q = i >> 2, pp = i & 3;
      const int col = 16 * (g & 1) + 4 * pp;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const bf16_t* blk = (kb < 2 ? Qs : dOs) + wave * 32 * 64;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int r0 = kb * 32 + 16 * s + 4 * h + q;
          const bf16x8 bs = cat8(tr_read(blk, dsoff(r0, col)), tr_read(blk, dsoff(r0 + 8, col)));
          dq0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(dSt, kb * 32, s, 0, lane), bs, dq0, 0, 0, 0);
          dq1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(dSt, kb * 32, s, 1, lane), bs, dq1, 0, 0, 0);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's K / dS reads done: K's slot becomes the output staging
    asm volatile("" ::: "memory");
    if (diag) ts[4] = __builtin_amdgcn_s_memtime();
    bf16_t* stg = dSt + wave * 32 * D;
    bf16_t* rowbase = dqkv + ((int64_t)b * S + wave * 32) * ld + hh * D;
    float* bs_w = dbias ? bsum + wave * D : nullptr;
    store_rows(stg, dv0, dv1, 1.0f, rowbase + 2 * H, ld, lane, dbias ? bs_w + 2 * 4 * D : nullptr);
    store_rows(stg, dk0, dk1, scale, rowbase + H, ld, lane, dbias ? bs_w + 4 * D : nullptr);
    store_rows(stg, dq0, dq1, scale, rowbase, ld, lane, bs_w);
  }
  if (dbias) {
    // qkv bias gradient: column sums of this (batch, head)'s dQ | dK | dV, one atomic per column
    __syncthreads();
    if (tid < 3 * D) {
      const int which = tid / D, c = tid % D;
      const float* b = bsum + which * 4 * D + c;
      atomicAdd(dbias + which * H + hh * D + c, b[0] + b[D] + b[2 * D] + b[3 * D]);
    }
  }
  if (diag) {
    ts[5] = __builtin_amdgcn_s_memtime();
    const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
      unsigned long long* d = diag + (int64_t)blockIdx.x * 8;
#pragma unroll
      for (int i = 0; i < 6; ++i) d[i] = ts[i];
      d[6] = rt0;
      d[7] = rt1;
    }
  }
}

}  // namespace a128

bool attn128_supported(int S, int head_dim) { return S == a128::S && head_dim == a128::D; }

static unsigned long long* g_a128_diag = nullptr;
void attn128_set_diag(void* p) { g_a128_diag = (unsigned long long*)p; }

void launch_attn128_fwd(const bf16_t* qkv, const float* mask, bf16_t* out, float* lse2, int B, int heads, double p,
                        uint64_t seed, hipStream_t st) {
  DropoutParams dp = make_dropout(p, seed);
  const float sl2 = a128::kLog2e / sqrtf((float)a128::D);
  hipLaunchKernelGGL(a128::attn128_fwd_kernel, dim3(B * heads), dim3(256), 0, st, qkv, mask, out, lse2, heads, sl2, dp);
  HSD_CHECK_LAUNCH();
}

void launch_attn128_bwd(const bf16_t* qkv, const float* mask, const bf16_t* o, const bf16_t* dout, const float* lse2,
                        bf16_t* dqkv, float* dbias, int B, int heads, double p, uint64_t seed, hipStream_t st) {
  DropoutParams dp = make_dropout(p, seed);
  const float sl2 = a128::kLog2e / sqrtf((float)a128::D);
  const float scale = 1.0f / sqrtf((float)a128::D);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(B * heads), dim3(256), 0, st, qkv, mask, o, dout, lse2, dqkv, dbias, heads, sl2,
                       scale, dp, g_a128_diag);
  };
  if (dp.enabled) go(a128::attn128_bwd_kernel<true>);
  else go(a128::attn128_bwd_kernel<false>);
  HSD_CHECK_LAUNCH();
}

}  // namespace hsd
