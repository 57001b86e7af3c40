// Shared pieces of the MFMA GEMMs (gemm2.hip bf16, gemm8.hip fp8): epilogue kinds, launch parameters,
// the barrier / counted-wait helpers and the bf16-output epilogue (wave-private LDS staging, 16-B row
// stores, fused bias / GELU / dropout+residual / derivative products / bias-gradient column sums).
#pragma once
#include "common.h"
#include "fp8_common.h"

namespace hsd {

// E2_BIAS_GELU_D: C = gelu'(y), C2 = gelu(y) (y = acc + bias) — the FFN1 forward keeps the GELU DERIVATIVE
// for backward, so the FFN2 dgrad epilogue is a plain product (E2_MUL: C = bf16(acc) * aux) instead of
// re-evaluating erf/exp per element.
// E2_STORE_RDOT: C = bf16(acc), plus the attention backward's delta rows rd[(b·heads + h)·S + s] = Σ_{64 columns of head h}
// C·aux over row m = b·S + s (aux = the attention output O, heads = N / 64): the out-projection dgrad writes dO AND the
// row dots the streaming attention backward would otherwise recompute in a separate pass (re-reading dO and O)
enum Epi2 : int { E2_STORE = 0, E2_BIAS = 1, E2_BIAS_GELU = 2, E2_BIAS_DROP_RES = 3, E2_RES = 4, E2_DGELU = 5,
                  E2_F32_ATOMIC = 6, E2_F32_SLAB = 7, E2_BIAS_GELU_D = 8, E2_MUL = 9, E2_STORE_RDOT = 10 };

__host__ __device__ constexpr bool epi_bias(int e) { return e == E2_BIAS || e == E2_BIAS_GELU || e == E2_BIAS_DROP_RES || e == E2_BIAS_GELU_D; }
__host__ __device__ constexpr bool epi_aux(int e) {
  return e == E2_BIAS_DROP_RES || e == E2_RES || e == E2_DGELU || e == E2_MUL || e == E2_STORE_RDOT;
}
__host__ __device__ constexpr bool epi_two_out(int e) { return e == E2_BIAS_GELU || e == E2_BIAS_GELU_D; }
__host__ __device__ constexpr bool epi_bf16_out(int e) {
  return e <= E2_DGELU || e == E2_BIAS_GELU_D || e == E2_MUL || e == E2_STORE_RDOT;
}

struct G2Params {
  const bf16_t* A;
  int64_t lda;
  const bf16_t* B;
  int64_t ldb;
  int M, N, K;
  void* C;  // bf16 [M][ldc], or fp32 (atomic: [M][ldc]; slab: [splits][M][N])
  int64_t ldc;
  const bf16_t* bias;
  const bf16_t* aux;
  int64_t ldaux;
  bf16_t* C2;
  DropoutParams dp;
  int kps;  // K elements per split (multiple of 64)
  int tiles_n;
  int ntiles;    // tiles_m * tiles_n
  float* dbias;  // E2_DGELU: optional fp32 column sums of the output (the bias gradient), BN 256 only
  int nt_store;  // bf16 epilogues: non-temporal stores (always 1 in the step; plain stores measured slower)
  unsigned long long* diag;  // persistent NT kernel, diagnostic: per-workgroup seam timestamps (gemm2_set_diag)
  // optional fp8 copy of the bf16 output (C2 for two-output epilogues, else C) for the next fp8 GEMM: q8 [M][ldc]
  // bytes, format q8_fmt, delayed scaling from *q8_amax; 1/scale into *q8_sinv, this output's amax into *q8_track
  uint8_t* q8;
  const float* q8_amax;
  float* q8_sinv;
  float* q8_track;
  int q8_fmt;
  // Q8 epilogues: 1 = the fp8 copy is the output's only consumer-visible form; the bf16 output it duplicates (C2 of the
  // two-output GELU epilogue, else C) is not stored (its consumers all take the fp8 copy: ops/hip.py, the FFN block)
  int q8_only;
  // persistent kernels: dynamic tile queue (tq_* below; one ring slot per launch), nullptr = static tile walk
  int* tq;
  // E2_F32_SLAB with one K-split: C[m][n] += acc in place (ldc; each element has one owner) instead of a slab
  int accum_direct;
  // E2_STORE_RDOT: fp32 [M / rd_seq · N / 64][rd_seq] row dots (rd_seq = the attention's sequence length)
  float* rd;
  int rd_seq;
  // segmented K (SEG kernels; the fp32 step's split products, ops/hip32.py): K = 3 · seg, and a K-tile at k0 of segment
  // s = k0 / seg reads segA[s] / segB[s] at k0 - s · seg (the leading dimensions lda / ldb are shared), so
  // [xh | xh | xl] · [wh | wl | wh]ᵀ runs over the bf16 hi / lo halves of each operand as they are stored -- no
  // concatenated three-block copies (seg % 64 == 0: a K-tile never straddles two segments)
  int seg;
  const bf16_t* segA[3];
  const bf16_t* segB[3];
};

// wave-uniform copy of a kernel-argument pointer (readfirstlane'd halves: SGPRs, as wave_rsrc below)
__device__ __forceinline__ const bf16_t* uniform_ptr(const bf16_t* ptr) {
  const uint64_t a = (uint64_t)ptr;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return reinterpret_cast<const bf16_t*>(((uint64_t)hi << 32) | lo);
}

// Operand bases and the segment-local k0 of a K-tile. The six segment pointers are copied out of the parameter
// struct ONCE, into scalar locals: indexing G2Params' arrays inside the main loop made hipcc keep the whole struct in
// scratch memory and reload it per DMA (a 2.2x slower main loop). SEG = false: p.A / p.B, k0 unchanged.
template <bool SEG>
struct SegSel {
  const bf16_t *a0, *a1, *a2, *b0, *b1, *b2;
  int seg;
  __device__ __forceinline__ explicit SegSel(const G2Params& p) {
    if constexpr (SEG) {
      a0 = uniform_ptr(p.segA[0]); a1 = uniform_ptr(p.segA[1]); a2 = uniform_ptr(p.segA[2]);
      b0 = uniform_ptr(p.segB[0]); b1 = uniform_ptr(p.segB[1]); b2 = uniform_ptr(p.segB[2]);
      seg = __builtin_amdgcn_readfirstlane(p.seg);
    } else {
      a0 = a1 = a2 = p.A;
      b0 = b1 = b2 = p.B;
      seg = 0;
    }
  }
  __device__ __forceinline__ int map(int k0, const bf16_t*& A, const bf16_t*& B) const {
    if constexpr (!SEG) {
      A = a0;
      B = b0;
      return k0;
    } else {
      // masked adds, not `s == 0 ? a0 : ...`: hipcc turns a select of the six members into a dynamically indexed load
      // of this object, then promotes the object to LDS (a ds_write of the six pointers in the prologue and a
      // ds_read_b64 in front of every DMA of the main loop, queued behind the fragment reads: ~45 % slower GEMMs)
      const bool s1 = k0 >= seg, s2 = k0 >= 2 * seg;
      const uint64_t m1 = 0 - (uint64_t)(s1 && !s2), m2 = 0 - (uint64_t)s2;
      A = reinterpret_cast<const bf16_t*>((uint64_t)a0 + ((((uint64_t)a1 - (uint64_t)a0)) & m1) +
                                          ((((uint64_t)a2 - (uint64_t)a0)) & m2));
      B = reinterpret_cast<const bf16_t*>((uint64_t)b0 + ((((uint64_t)b1 - (uint64_t)b0)) & m1) +
                                          ((((uint64_t)b2 - (uint64_t)b0)) & m2));
      return k0 - ((int)s1 + (int)s2) * seg;
    }
  }
};

// E2_STORE_RDOT: the 8 lanes holding the 8 chunks (64 columns = one head) of row m reduce their chunk dots; the first
// writes the head's delta. Called by every lane of the group (DPP), `store` false for rows past M.
__device__ __forceinline__ void rdot_group(const u32x4& o, const u32x4& x, int m, int n, const G2Params& p, bool lead,
                                           bool store) {
  const float d = sum8_dpp(dot8_bf16(o, x));
  if (lead && store) {
    const int b = m / p.rd_seq, s = m - b * p.rd_seq;
    p.rd[((int64_t)b * (p.N >> 6) + (n >> 6)) * p.rd_seq + s] = d;
  }
}

// ---- dynamic tile queue of the persistent NT GEMMs (gemm2pk / gemm8pk) ----------------------------------------------
// A persistent workgroup that starts late (its CU held by a co-running RCCL kernel or optimizer slice) must not own a
// fixed share of the tiles, or the GEMM's tail grows by the delay. Tiles are claimed instead: 8 counters, one per XCD
// group (tile L belongs to group L & 7, which the XCD-aware remap maps to that group's contiguous tile range, so a
// workgroup claiming from the counter of the XCD it runs on keeps its L2 locality); a workgroup whose own group is
// exhausted steals from the others. Counters are relaxed agent-scope atomics (they hand out indices, no data: no
// acquire/release needed). The last workgroup to leave resets the slot for the next launch that uses it (the exit
// counter reaches gridDim.x only after every claim of the launch has returned), so no memset node per launch.
// Layout: 9 counters 128 B apart (8 claim counters + the exit counter).
constexpr int kTqStride = 32;
constexpr int kTqInts = 9 * kTqStride;

__device__ __forceinline__ int tq_xcc() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 7;
}

__device__ __forceinline__ int tq_fetch(int* q, int g) {
  return __hip_atomic_fetch_add(q + g * kTqStride, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// blocking claim: own group first, then the others not yet seen exhausted (`dead` bit mask); ntiles = none left
__device__ __forceinline__ int tq_claim(int* q, int g, uint32_t& dead, int ntiles) {
  for (int k = 0; k < 8; ++k) {
    const int gg = (g + k) & 7;
    if (dead & (1u << gg)) continue;
    const int L = gg + 8 * tq_fetch(q, gg);
    if (L < ntiles) return L;
    dead |= 1u << gg;
  }
  return ntiles;
}

__device__ __forceinline__ void tq_exit(int* q) {
  if (__hip_atomic_fetch_add(q + 8 * kTqStride, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
      (int)gridDim.x - 1) {
#pragma unroll
    for (int g = 0; g <= 8; ++g) __hip_atomic_store(q + g * kTqStride, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Buffer descriptor over `ptr` (wave-uniform: built from readfirstlane'd halves so hipcc keeps it in SGPRs).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void* ptr) {
  const uint64_t a = (uint64_t)ptr;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, 0x7FFFFFFF, 0x00020000);
}

// 16-B non-temporal buffer store (cache policy nt). The bf16 GEMM epilogues store through it: plain stores
// allocate the output lines in the XCD's 4 MiB L2 and evict the A / B panels the CU's next tiles stream from it;
// with nt the T x 3072 x 768 GEMM (FFN1 shape) runs 583 -> 494 us and T x 768 x 768 147 -> 125 us
// (tools/store_policy_probe.py, profiles/store_policy_r3.log). hipcc's __builtin_nontemporal_store emits a plain
// global_store on gfx950, hence the buffer form.
__device__ __forceinline__ void st16nt(__amdgpu_buffer_rsrc_t r, uint32_t off, const u32x4& v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 2);
}

__device__ __forceinline__ void st16(bf16_t* dst, const u32x4& v, int nt) {
  if (nt) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst));
  else *reinterpret_cast<u32x4*>(dst) = v;
}

namespace g2 {

constexpr int BM = 256;
#ifndef G2_AUX_NO_PREFETCH
#define G2_AUX_NO_PREFETCH 0
#endif

__device__ __forceinline__ int f1(int row) { return (row >> 1) & 7; }

#define G2_BARRIER()                       \
  do {                                     \
    asm volatile("" ::: "memory");         \
    __builtin_amdgcn_sched_barrier(0);     \
    __builtin_amdgcn_s_barrier();          \
    __builtin_amdgcn_sched_barrier(0);     \
    asm volatile("" ::: "memory");         \
  } while (0)

template <int N>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ u32x2 pack4(const f32x4& v) {
  u32x2 o;
  o.x = pack_bf2(v[0], v[1]);
  o.y = pack_bf2(v[2], v[3]);
  return o;
}


// Epilogue math for one 16-B chunk (8 consecutive n of row m) of the staged bf16(acc [+ bias]) tile `o`;
// `x` is the aux chunk. Returns the primary output in `o` and (two-output epilogues) the second in `o2`.
// `xw`: the dropout word R(m) ^ C(n / 2) of the chunk's row m and column n (E2_BIAS_DROP_RES; the caller keeps the
// column word in a register across rows and gets the row word from a lane that hashed it -- epilogue_bf16)
template <int EPI>
__device__ __forceinline__ void epi_chunk(u32x4& o, u32x4& o2, const u32x4& x, int m, int n, const G2Params& p,
                                          float (&csum)[8], uint32_t xw = 0u) {
  if constexpr (EPI == E2_BIAS_GELU) {
    o2.x = pack_bf2(gelu_erf(lo_bf(o.x)), gelu_erf(hi_bf(o.x)));
    o2.y = pack_bf2(gelu_erf(lo_bf(o.y)), gelu_erf(hi_bf(o.y)));
    o2.z = pack_bf2(gelu_erf(lo_bf(o.z)), gelu_erf(hi_bf(o.z)));
    o2.w = pack_bf2(gelu_erf(lo_bf(o.w)), gelu_erf(hi_bf(o.w)));
  } else if constexpr (EPI == E2_BIAS_GELU_D) {
    float v[8] = {lo_bf(o.x), hi_bf(o.x), lo_bf(o.y), hi_bf(o.y), lo_bf(o.z), hi_bf(o.z), lo_bf(o.w), hi_bf(o.w)};
    float a[8], d[8];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      f32x2 ga, gd;
      gelu_and_grad2(f32x2{v[e], v[e + 1]}, ga, gd);
      a[e] = ga.x; a[e + 1] = ga.y; d[e] = gd.x; d[e + 1] = gd.y;
    }
    o.x = pack_bf2(d[0], d[1]); o.y = pack_bf2(d[2], d[3]); o.z = pack_bf2(d[4], d[5]); o.w = pack_bf2(d[6], d[7]);
    o2.x = pack_bf2(a[0], a[1]); o2.y = pack_bf2(a[2], a[3]); o2.z = pack_bf2(a[4], a[5]); o2.w = pack_bf2(a[6], a[7]);
  } else if constexpr (EPI == E2_BIAS_DROP_RES) {
    // z = bf16(y · keep · scale + residual), y = bf16(acc + bias): one rounding of the sum (the dropped value is not
    // rounded to bf16 on its own -- a pack / unpack pair per element less, and no less accurate)
    // rounded once, as fma(y, keep ? scale : 0, residual) -- the same expression as gemm.hip's epi_block, so a site gives
    // the same bits on every kernel path
    float v[8] = {lo_bf(o.x), hi_bf(o.x), lo_bf(o.y), hi_bf(o.y), lo_bf(o.z), hi_bf(o.z), lo_bf(o.w), hi_bf(o.w)};
    const float r[8] = {lo_bf(x.x), hi_bf(x.x), lo_bf(x.y), hi_bf(x.y), lo_bf(x.z), hi_bf(x.z), lo_bf(x.w), hi_bf(x.w)};
    if (p.dp.enabled) {
      // mask row m (width N), pairs n / 2 + e = n / 2 ^ e (n % 8 == 0)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t b = drop_fin(xw ^ drop_col((uint32_t)e));
        v[2 * e] = __builtin_fmaf(v[2 * e], keep_lo(b, p.dp.thr) ? p.dp.scale : 0.f, r[2 * e]);
        v[2 * e + 1] = __builtin_fmaf(v[2 * e + 1], keep_hi(b, p.dp.thr) ? p.dp.scale : 0.f, r[2 * e + 1]);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += r[e];
    }
    o.x = pack_bf2(v[0], v[1]);
    o.y = pack_bf2(v[2], v[3]);
    o.z = pack_bf2(v[4], v[5]);
    o.w = pack_bf2(v[6], v[7]);
  } else if constexpr (EPI == E2_RES) {
    o.x = pack_bf2(lo_bf(o.x) + lo_bf(x.x), hi_bf(o.x) + hi_bf(x.x));
    o.y = pack_bf2(lo_bf(o.y) + lo_bf(x.y), hi_bf(o.y) + hi_bf(x.y));
    o.z = pack_bf2(lo_bf(o.z) + lo_bf(x.z), hi_bf(o.z) + hi_bf(x.z));
    o.w = pack_bf2(lo_bf(o.w) + lo_bf(x.w), hi_bf(o.w) + hi_bf(x.w));
  } else if constexpr (EPI == E2_DGELU || EPI == E2_MUL) {
    if constexpr (EPI == E2_DGELU) {
      o.x = pack_bf2(lo_bf(o.x) * gelu_erf_grad(lo_bf(x.x)), hi_bf(o.x) * gelu_erf_grad(hi_bf(x.x)));
      o.y = pack_bf2(lo_bf(o.y) * gelu_erf_grad(lo_bf(x.y)), hi_bf(o.y) * gelu_erf_grad(hi_bf(x.y)));
      o.z = pack_bf2(lo_bf(o.z) * gelu_erf_grad(lo_bf(x.z)), hi_bf(o.z) * gelu_erf_grad(hi_bf(x.z)));
      o.w = pack_bf2(lo_bf(o.w) * gelu_erf_grad(lo_bf(x.w)), hi_bf(o.w) * gelu_erf_grad(hi_bf(x.w)));
    } else {
      o.x = pack_bf2(lo_bf(o.x) * lo_bf(x.x), hi_bf(o.x) * hi_bf(x.x));
      o.y = pack_bf2(lo_bf(o.y) * lo_bf(x.y), hi_bf(o.y) * hi_bf(x.y));
      o.z = pack_bf2(lo_bf(o.z) * lo_bf(x.z), hi_bf(o.z) * hi_bf(x.z));
      o.w = pack_bf2(lo_bf(o.w) * lo_bf(x.w), hi_bf(o.w) * hi_bf(x.w));
    }
    csum[0] += lo_bf(o.x); csum[1] += hi_bf(o.x); csum[2] += lo_bf(o.y); csum[3] += hi_bf(o.y);
    csum[4] += lo_bf(o.z); csum[5] += hi_bf(o.z); csum[6] += lo_bf(o.w); csum[7] += hi_bf(o.w);
  }
}

template <int EPI>
__device__ __forceinline__ uint32_t epi_col_word(int n, const G2Params& p) {
  if constexpr (EPI == E2_BIAS_DROP_RES) return p.dp.enabled ? drop_col((uint32_t)n >> 1) : 0u;
  return 0u;
}

// column sums of 8 columns per lane, lanes with equal (lane & 7) hold the same columns: reduce + atomics
__device__ __forceinline__ void colsum_flush(float (&csum)[8], float* dbias, int nw, int N, int lane) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    csum[e] = sum_stride8(csum[e]);
  }
  if (lane < 8 && nw + lane * 8 < N) {
#pragma unroll
    for (int e = 0; e < 8; ++e) atomicAdd(dbias + nw + lane * 8 + e, csum[e]);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) csum[e] = 0.f;
}

// bf16-output epilogue of a 256 x BN tile held as acc[8][BN/64] (acc[i][j] = D[n][m] block: lane l holds
// m = 16i + (l&15), n = 16j + 4(l>>4) + r), staged through the wave's [16·PB][SROW] slice of `smem`.
// MB = 16-row MFMA blocks per wave (8: the 128-row wave tiles of the 256 x BN kernels; 4: the 64-row wave tiles
// of gemm2s_kernel). PB = 16-row MFMA blocks per staging pass (4: 64-row passes; 2: 32-row passes -- the
// persistent kernel's staging area beside its two operand stages).
// PRE: the bias registers (epi_bias_regs) and the first pass's residual chunks (epi_aux_regs, h = 0) were loaded by
// the caller -- the persistent kernel loads them BEFORE it issues the next tile's LDS-DMA, so waiting for them does
// not wait for that DMA (vector-memory counters retire loads in order).
template <int BN, int PB>
constexpr int epi_iter() { return 16 * PB * (BN / 32) / 64; }
template <int BN>
constexpr int epi_srow() { return BN / 4 == 64 ? 64 : BN / 4 + 8; }

template <int EPI, int BN>
__device__ __forceinline__ void epi_bias_regs(f32x4 (&bv)[BN / 64], const G2Params& p, int lane, int nw) {
  if constexpr (epi_bias(EPI)) {
#pragma unroll
    for (int j = 0; j < BN / 64; ++j) {
      const int n = min(nw + 16 * j + 4 * (lane >> 4), p.N - 4);
      const u32x2 b = *reinterpret_cast<const u32x2*>(p.bias + n);
      bv[j] = f32x4{lo_bf(b.x), hi_bf(b.x), lo_bf(b.y), hi_bf(b.y)};
    }
  }
}

template <int EPI, int BN, int PB, int NIT>
__device__ __forceinline__ void epi_aux_regs(u32x4 (&xv)[NIT], const G2Params& p, int lane, int mw, int nw, int h) {
  static_assert(NIT == epi_iter<BN, PB>(), "one chunk per lane per 64 chunks of a pass");
  constexpr int CPR = BN / 32;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    if constexpr (epi_aux(EPI)) {
      const int idx = lane + 64 * it;
      const int row = idx / CPR, c8 = idx % CPR;
      const int m = min(mw + 16 * PB * h + row, p.M - 1);
      xv[it] = *reinterpret_cast<const u32x4*>(p.aux + (int64_t)m * p.ldaux + nw + c8 * 8);
    } else {
      xv[it] = u32x4{0, 0, 0, 0};
    }
  }
}

// Q8: also the output's fp8 copy (G2Params q8 fields; fp8 persistent kernel only)
template <int EPI, int BN, int MB = 8, int PB = 4, bool PRE = false, bool Q8 = false>
__device__ __forceinline__ void epilogue_bf16(f32x4 (&acc)[MB][BN / 64], const G2Params& p, bf16_t* smem, int wave,
                                              int lane, int mw, int nw, const f32x4* bv_pre = nullptr,
                                              const u32x4* xv_pre = nullptr) {
  static_assert(MB == 4 || MB == 8, "64 or 128 rows per wave");
  static_assert(PB == 2 || PB == 4, "32- or 64-row staging passes");
  constexpr int WN = BN / 4, NREP = WN / 16;
  const int q4 = lane >> 4, lr = lane & 15;
  // stage bf16(acc [+ bias]) through a wave-private LDS slice ([16·PB rows][SROW]), then write whole
  // rows with 16-B lanes: each lane owns 8 consecutive n of one m.
  // WN = 64 (BN 256): unpadded 128-B rows whose 8-B slots are XOR-swizzled by (row & 15) -- the 16 lanes of a
  // ds_write_b64 group (16 rows, one slot) then cover all 32 banks, and a ds_read_b128 of chunk c8 finds its
  // two halves in chunk c8 ^ ((row & 15) >> 1), swapped when row is odd (both conflict-free; the padded
  // [64][72] image measured 12 % LDS bank-conflict cycles, tools/pmc_gemm2.sh). Other widths keep the pad.
  constexpr bool kSwz = WN == 64;
  constexpr int SROW = epi_srow<BN>();
  constexpr int CPR = WN / 8;  // 16-B chunks per row
  constexpr bool kBias = epi_bias(EPI);
  constexpr int ITER = epi_iter<BN, PB>();
  bf16_t* stg = smem + wave * (16 * PB * SROW);
  f32x4 bv[NREP];
  if constexpr (PRE) {
#pragma unroll
    for (int j = 0; j < NREP; ++j) bv[j] = bv_pre[j];
  } else {
    epi_bias_regs<EPI, BN>(bv, p, lane, nw);
  }
  bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
  // stores: non-temporal buffer stores off the wave's first row (st16nt); p.nt_store = 0: plain
  const __amdgpu_buffer_rsrc_t rc = wave_rsrc(C + (int64_t)mw * p.ldc);
  const __amdgpu_buffer_rsrc_t rc2 = wave_rsrc(epi_two_out(EPI) ? p.C2 + (int64_t)mw * p.ldc : C);
  constexpr bool kColsum = (EPI == E2_DGELU || EPI == E2_MUL) && CPR == 8;
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float qs = 0.f, qm = 0.f;
  if constexpr (Q8) qs = fmt_scale(p.q8_fmt, *p.q8_amax);
  const bool q8_only = Q8 && __builtin_amdgcn_readfirstlane(p.q8_only) != 0;
  // aux (residual / GELU' operand) chunks of the NEXT pass are loaded right after this pass's staging writes, i.e.
  // BEFORE this pass's stores: the vector-memory counter retires loads and stores in issue order, so a load issued
  // after the previous pass's stores made its consumer wait for all of them (s_waitcnt vmcnt(0) per pass)
  constexpr bool kAuxPf = epi_aux(EPI) && !G2_AUX_NO_PREFETCH;
  // dropout: the column word of the lane's chunk column is the same in every pass when CPR divides 64 (hoisted); the
  // row words of a pass's 16·PB rows are hashed once, one row per lane, and each chunk takes its row's word from that
  // lane (ds_bpermute: an LDS-pipe move, not 9 VALU instructions of lowbias32 per chunk)
  constexpr bool kColFixed = 64 % CPR == 0;
  constexpr bool kDrop = EPI == E2_BIAS_DROP_RES;
  const bool drop_on = kDrop && p.dp.enabled;
  const uint32_t cw = kColFixed ? epi_col_word<EPI>(nw + (lane % CPR) * 8, p) : 0u;
  u32x4 xnext[ITER];
#pragma unroll
  for (int h = 0; h < MB / PB; ++h) {
#pragma unroll
    for (int i = 0; i < PB; ++i)
#pragma unroll
      for (int j = 0; j < NREP; ++j) {
        f32x4 v = acc[PB * h + i][j];
        if constexpr (kBias) v += bv[j];
        const int row = 16 * i + lr;
        const int col = kSwz ? (((4 * j + q4) ^ (row & 15)) << 2) : 16 * j + 4 * q4;
        *reinterpret_cast<u32x2*>(stg + row * SROW + col) = pack4(v);
      }
    __builtin_amdgcn_wave_barrier();
    u32x4 sv[ITER], xv[ITER];
    if constexpr (kAuxPf) {
      if (h > 0) {
#pragma unroll
        for (int it = 0; it < ITER; ++it) xv[it] = xnext[it];
      }
      if (h + 1 < MB / PB) epi_aux_regs<EPI, BN, PB>(xnext, p, lane, mw, nw, h + 1);
    }
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int idx = lane + 64 * it;
      const int row = idx / CPR, c8 = idx % CPR;
      if constexpr (kSwz) {
        const int hs = row & 15;
        const u32x4 t = *reinterpret_cast<const u32x4*>(stg + row * SROW + ((c8 ^ (hs >> 1)) << 3));
        sv[it] = (hs & 1) ? u32x4{t.z, t.w, t.x, t.y} : t;
      } else {
        sv[it] = *reinterpret_cast<const u32x4*>(stg + row * SROW + c8 * 8);
      }
    }
    if (PRE && h == 0) {
#pragma unroll
      for (int it = 0; it < ITER; ++it) xv[it] = xv_pre[it];
    } else if (!kAuxPf || h == 0) {
      epi_aux_regs<EPI, BN, PB>(xv, p, lane, mw, nw, h);
    }
    uint32_t rw_lane = 0u;  // R(row `lane` of this pass)
    if (kDrop && drop_on && kColFixed) rw_lane = drop_row((uint32_t)(mw + 16 * PB * h + lane), p.dp.key);
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int idx = lane + 64 * it;
      const int row = idx / CPR, c8 = idx % CPR;
      const int m = mw + 16 * PB * h + row;
      const int n = nw + c8 * 8;
      uint32_t xw = 0u;
      if (kDrop && drop_on) {
        xw = kColFixed ? (uint32_t)__builtin_amdgcn_ds_bpermute(4 * row, (int)rw_lane) ^ cw
                       : drop_row((uint32_t)m, p.dp.key) ^ epi_col_word<EPI>(n, p);
      }
      if constexpr (EPI == E2_STORE_RDOT) {
        static_assert(CPR == 8, "row dots: 8 chunks (one 64-column head) per row");
        rdot_group(sv[it], xv[it], m, n, p, c8 == 0, m < p.M);
      }
      if (m >= p.M) continue;
      const int64_t co = (int64_t)m * p.ldc + n;
      u32x4 o = sv[it], o2;
      epi_chunk<EPI>(o, o2, xv[it], m, n, p, csum, xw);
      // Q8 with q8_only: the bf16 twin of the fp8 copy is not written (o2 of a two-output epilogue, else o)
      const bool st_o = !(Q8 && !epi_two_out(EPI) && q8_only);
      const bool st_o2 = !(Q8 && q8_only);
      if (p.nt_store) {
        const uint32_t bo = (uint32_t)(((int64_t)(m - mw) * p.ldc + n) * 2);
        if (st_o) st16nt(rc, bo, o);
        if constexpr (epi_two_out(EPI)) if (st_o2) st16nt(rc2, bo, o2);
      } else {
        if (st_o) st16(C + co, o, 0);
        if constexpr (epi_two_out(EPI)) if (st_o2) st16(p.C2 + co, o2, 0);
      }
      if constexpr (Q8) {
        const u32x4 src = epi_two_out(EPI) ? o2 : o;
        qm = absmax8(src, qm);
        *reinterpret_cast<u32x2*>(p.q8 + co) = p.q8_fmt == 0 ? quant8<0>(src, qs) : quant8<1>(src, qs);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  if constexpr (kColsum) {
    if (p.dbias != nullptr) colsum_flush(csum, p.dbias, nw, p.N, lane);
  }
  if constexpr (Q8) {
    wave_amax_track(qm, p.q8_track);
    if (blockIdx.x == 0 && threadIdx.x == 0) *p.q8_sinv = 1.0f / qs;
  }
}

}  // namespace g2
}  // namespace hsd
