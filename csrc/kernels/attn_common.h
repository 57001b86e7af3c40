// Shared device helpers of the flash-attention kernels (attention128.hip, attentionS.hip): the
// [rows][64] bf16 operand image (XOR-swizzled 16-B chunks, filled by LDS-DMA with the swizzle on the
// source address), transposed fragment reads (ds_read_b64_tr_b16), accumulator-as-operand packing and
// the wave-private staging used for 128-B row stores. head_dim is 64.
#pragma once
#include "common.h"
#include "fp8_common.h"

namespace hsd {
namespace attn {

constexpr int D = 64;
constexpr float kLog2e = 1.4426950408889634f;

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

__device__ __forceinline__ int swz(int row) {
  const int t = (row >> 1) & 7;
  return ((t & 1) << 2) | (t & 2) | ((t >> 2) & 1);
}
// element offset of (row, col) in a [rows][64] bf16 image
__device__ __forceinline__ int toff(int row, int col) { return row * 64 + (((col >> 3) ^ swz(row)) << 3) + (col & 7); }
// [128][128] dS image
__device__ __forceinline__ int fS(int row) { return 4 * ((row & 3) ^ ((row >> 4) & 3)) + ((row >> 2) & 3); }
__device__ __forceinline__ int soff(int row, int col) { return row * 128 + (((col >> 3) ^ fS(row)) << 3) + (col & 7); }
// wave-private [32][64] output staging slice
__device__ __forceinline__ int stoff(int row, int col) { return row * 64 + (((col >> 3) ^ ((row >> 1) & 7)) << 3) + (col & 7); }

__device__ __forceinline__ bf16x4 tr_read(const bf16_t* base, int elem_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(base + elem_off));
}
__device__ __forceinline__ bf16x8 cat8(bf16x4 a, bf16x4 b) {
  bf16x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}
__device__ __forceinline__ bf16x8 pack8(const f32x16& acc, int s) {
  // four two-source v_cvt_pk_bf16_f32 (pack_bf2), not eight single converts + shifts / ors
  const u32x4 w = {pack_bf2(acc[8 * s], acc[8 * s + 1]), pack_bf2(acc[8 * s + 2], acc[8 * s + 3]),
                   pack_bf2(acc[8 * s + 4], acc[8 * s + 5]), pack_bf2(acc[8 * s + 6], acc[8 * s + 7])};
  return __builtin_bit_cast(bf16x8, w);
}
// Transposed A operand from a [rows][64] image: rows rb + 16s + 8(j>>2) + 4h + (j&3) (the accumulator's
// permuted k order), columns colblk*32 + (lane & 31).
__device__ __forceinline__ bf16x8 trA(const bf16_t* img, int rb, int s, int colblk, int lane) {
  const int g = lane >> 4, i = lane & 15, h = g >> 1, q = i >> 2, p = i & 3;
  const int col = colblk * 32 + 16 * (g & 1) + 4 * p;
  const int r0 = rb + 16 * s + 4 * h + q;
  return cat8(tr_read(img, toff(r0, col)), tr_read(img, toff(r0 + 8, col)));
}
// Same from the [128][128] dS image (columns cb + (lane & 31)).
__device__ __forceinline__ bf16x8 trS(const bf16_t* img, int rb, int s, int cb, int lane) {
  const int g = lane >> 4, i = lane & 15, h = g >> 1, q = i >> 2, p = i & 3;
  const int col = cb + 16 * (g & 1) + 4 * p;
  const int r0 = rb + 16 * s + 4 * h + q;
  return cat8(tr_read(img, soff(r0, col)), tr_read(img, soff(r0 + 8, col)));
}

// DMA rows [0,128) x 64 cols of a qkv / [T][H] column block into a [128][64] image: 16 instructions,
// wave w issues instructions w*per .. (w+1)*per-1.
__device__ __forceinline__ void dma_img(bf16_t* img, const bf16_t* __restrict__ src0, int64_t ld, int first, int count,
                                        int lane) {
  for (int g = first; g < first + count; ++g) {
    const int row = g * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ swz(row);
    const bf16_t* src = src0 + (int64_t)row * ld + lc * 8;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(img + g * 512), 16, 0, 0);
  }
}

// acc (32 rows on the lane x 64 d in regs: d = 32*blk + (reg&3) + 8(reg>>2) + 4h) * scale -> bf16 rows
// of `dst` (row stride ld) through the wave-private staging slice `stg` ([32][64]).
// q8dst (optional): the rows' fp8 copy (format qfmt, scale qs; same element offsets as dst), max |x| into *qm
__device__ __forceinline__ void store_rows(bf16_t* stg, const f32x16& a0, const f32x16& a1, float scale,
                                           bf16_t* __restrict__ dst, int64_t ld, int lane,
                                           float* colsum_lds = nullptr, uint8_t* __restrict__ q8dst = nullptr,
                                           int qfmt = 0, float qs = 0.f, float* qm = nullptr, bool q8only = false) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    u32x2 w0, w1;
    w0.x = pack_bf2(a0[4 * i] * scale, a0[4 * i + 1] * scale);
    w0.y = pack_bf2(a0[4 * i + 2] * scale, a0[4 * i + 3] * scale);
    w1.x = pack_bf2(a1[4 * i] * scale, a1[4 * i + 1] * scale);
    w1.y = pack_bf2(a1[4 * i + 2] * scale, a1[4 * i + 3] * scale);
    *reinterpret_cast<u32x2*>(stg + stoff(r, 8 * i + 4 * h)) = w0;
    *reinterpret_cast<u32x2*>(stg + stoff(r, 32 + 8 * i + 4 * h)) = w1;
  }
  __builtin_amdgcn_wave_barrier();
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int row = (lane >> 3) + 8 * it, c = lane & 7;
    const u32x4 v = *reinterpret_cast<const u32x4*>(stg + stoff(row, c * 8));
    // q8only: the fp8 copy is the only form the consumers read (the bf16 row is not stored)
    if (!(q8only && q8dst != nullptr)) *reinterpret_cast<u32x4*>(dst + (int64_t)row * ld + c * 8) = v;
    if (q8dst != nullptr) {
      *qm = absmax8(v, *qm);
      *reinterpret_cast<u32x2*>(q8dst + (int64_t)row * ld + c * 8) = qfmt == 0 ? quant8<0>(v, qs) : quant8<1>(v, qs);
    }
    if (colsum_lds) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        cs[2 * k] += lo_bf(v[k]);
        cs[2 * k + 1] += hi_bf(v[k]);
      }
    }
  }
  if (colsum_lds) {
    // lanes with equal (lane & 7) hold the same 8 columns: reduce over lane bits 3..5
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      cs[e] = sum_stride8(cs[e]);
    }
    if (lane < 8) {
#pragma unroll
      for (int e = 0; e < 8; ++e) colsum_lds[lane * 8 + e] = cs[e];
    }
  }
  __builtin_amdgcn_wave_barrier();
}


}  // namespace attn
}  // namespace hsd
