// Device helpers shared by the bf16 MFMA GEMM kernels (gemm2.hip): LDS-DMA slots of the operand tile
// images (builtin and inline-asm forms) and the 16x16x32 fragment reads. Image layouts: gemm2.hip header.
#pragma once
#include "gemm_common.h"

namespace hsd {
namespace g2 {

constexpr int BK = 64;

__device__ __forceinline__ int f2(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;

// One 1-KiB LDS-DMA wave instruction `g` of an operand tile image (see header for the images).
template <int L, int R>
__device__ __forceinline__ void dma(bf16_t* img, const bf16_t* __restrict__ X, int64_t ld, int r0, int Rmax, int k0,
                                    int g, int lane) {
  const bf16_t* src;
  if constexpr (L == 0) {
    const int row = g * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ f1(row);
    const int rr = min(r0 + row, Rmax - 1);
    src = X + (int64_t)rr * ld + k0 + lc * 8;
  } else {
    static_assert(R == 256, "k-strided images are 256 wide");
    const int krow = g * 2 + (lane >> 5);
    const int lc = (lane & 31) ^ f2(krow);
    const int cc = min(r0 + lc * 8, Rmax - 8);
    src = X + (int64_t)(k0 + krow) * ld + cc;
  }
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)(img + g * 512), 16, 0, 0);
}

// DMA of kernels with a k-strided operand (TT weight gradients, NT dgrad reading W directly): inline asm, a per-lane byte offset computed once per workgroup and a scalar
// (SGPR) base per K-tile. With the builtin, hipcc does not tell the transposing LDS reads (ds_read_b64_tr_b16) apart
// from the LDS-DMA destination and drains EVERY DMA (s_waitcnt vmcnt(0)) before the first read of each K-tile, so
// tile t+2's DMA had one MFMA phase to land instead of a K-tile. The asm DMA is invisible to hipcc's wait
// bookkeeping; the kernel's counted vmcnt<N>() waits retire it.
// Per-lane byte offset of DMA slot g from the operand's per-K-tile scalar base (asm_base): k-strided images
// (L = 1, base X + k0·ld) and k-contiguous images (L = 0, base X + r0·ld + k0; rows clamped to the matrix).
template <int L>
__device__ __forceinline__ uint32_t lane_off(int64_t ld, int r0, int Rmax, int g, int lane) {
  if constexpr (L == 1) {
    const int krow = g * 2 + (lane >> 5);
    const int lc = (lane & 31) ^ f2(krow);
    const int cc = min(r0 + lc * 8, Rmax - 8);
    return (uint32_t)(((int64_t)krow * ld + cc) * 2);
  } else {
    const int row = g * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ f1(row);
    const int rr = min(row, Rmax - 1 - r0);
    return (uint32_t)(((int64_t)rr * ld + lc * 8) * 2);
  }
}

template <int L>
__device__ __forceinline__ const bf16_t* asm_base(const bf16_t* X, int64_t ld, int r0, int k0) {
  if constexpr (L == 1) return X + (int64_t)k0 * ld;
  else return X + (int64_t)r0 * ld + k0;
}

__device__ __forceinline__ void dma_lds_asm(const bf16_t* sbase_in, uint32_t voff, uint32_t lds_addr) {
  const uint32_t lds = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds_addr);
  // the base is wave-uniform by construction; say so (folded away where the compiler already proves it)
  const uint64_t ba = (uint64_t)sbase_in;
  const bf16_t* sbase = (const bf16_t*)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(ba >> 32)) << 32) |
                                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)ba));
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds)
               : "memory");
}

// 16x16x32 operand fragment: lane l holds rows (rbase + (l&15)), k = 32·ks + 8·(l>>4) + 0..7
template <int L, int W = 256>
__device__ __forceinline__ bf16x8 frag(const bf16_t* img, int rbase, int ks, int lane) {
  if constexpr (L == 0) {
    const int row = rbase + (lane & 15);
    const int ch = (lane >> 4) + 4 * ks;
    return *reinterpret_cast<const bf16x8*>(img + row * 64 + ((ch ^ f1(row)) << 3));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int k = 32 * ks + 8 * g + q;
    const int m = rbase + 4 * p;
    const int k2 = k + 4;
    bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_bf16x4_t*)(img + k * W + (((m >> 3) ^ f2(k)) << 3) + (m & 7)));
    bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_bf16x4_t*)(img + k2 * W + (((m >> 3) ^ f2(k2)) << 3) + (m & 7)));
    bf16x8 r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  }
}

}  // namespace g2
}  // namespace hsd
