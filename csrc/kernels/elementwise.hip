// Memory-bound elementwise kernels (16-B vector IO, grid-stride, 2048-block cap —
// cdna_hip_programming.md Guideline 11/13).
//
//  * bias_gelu_fwd : g = gelu_erf(y)  (y = GEMM output incl. bias; y is kept for backward)
//  * gelu_bwd_colsum: da = dg * gelu'(y)   and   dbias += Σ_rows da   (fused bias-grad reduction)
//  * colsum        : dbias += Σ_rows x   (fp32 atomics, one per column per block)
//  * dropout_fwd/bwd: out = x * keep * scale (hash RNG, ops/rng.py)
#include "common.h"

namespace hsd {

__global__ __launch_bounds__(256) void gelu_fwd_kernel(const bf16_t* __restrict__ y, bf16_t* __restrict__ g, int64_t n8) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    u32x4 w = reinterpret_cast<const u32x4*>(y)[i];
    u32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = pack_bf2(gelu_erf(lo_bf(w[k])), gelu_erf(hi_bf(w[k])));
    reinterpret_cast<u32x4*>(g)[i] = o;
  }
}

// Column sums (bias gradients). Block = 256 threads = 64 column chunks (8 columns each, 512 columns)
// x 4 row groups; each thread walks rows rg, rg+4, ... of the block's row range with 4 rows' loads in
// flight, then the 4 row groups are reduced through LDS -> one atomic per column per block.
// kGelu: also writes da = dg * gelu'(y) (the FFN1 dgrad input) and sums da instead of x.
template <bool kGelu>
__global__ __launch_bounds__(256) void colsum_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ y,
                                                     bf16_t* __restrict__ out, float* __restrict__ dbias, int rows,
                                                     int N, int rows_per_block) {
  __shared__ float red[4][512 + 8];
  const int cc = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int col = blockIdx.x * 512 + cc * 8;
  const bool active = col < N;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (active) {
    for (int rb = r0 + rg; rb < r1; rb += 16) {
      u32x4 w[4], yy[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = rb + 4 * u;
        if (r < r1) {
          w[u] = *reinterpret_cast<const u32x4*>(x + (size_t)r * N + col);
          if constexpr (kGelu) yy[u] = *reinterpret_cast<const u32x4*>(y + (size_t)r * N + col);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = rb + 4 * u;
        if (r >= r1) continue;
        if constexpr (kGelu) {
          u32x4 o;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            o[k] = pack_bf2(lo_bf(w[u][k]) * gelu_erf_grad(lo_bf(yy[u][k])),
                            hi_bf(w[u][k]) * gelu_erf_grad(hi_bf(yy[u][k])));
            acc[2 * k] += lo_bf(o[k]);
            acc[2 * k + 1] += hi_bf(o[k]);
          }
          *reinterpret_cast<u32x4*>(out + (size_t)r * N + col) = o;
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            acc[2 * k] += lo_bf(w[u][k]);
            acc[2 * k + 1] += hi_bf(w[u][k]);
          }
        }
      }
    }
  }
  if (dbias == nullptr) return;
#pragma unroll
  for (int k = 0; k < 8; ++k) red[rg][cc * 8 + k] = acc[k];
  __syncthreads();
  // 256 threads x 2 columns each
  for (int c = threadIdx.x; c < 512; c += 256) {
    const int gc = blockIdx.x * 512 + c;
    if (gc < N) atomicAdd(dbias + gc, red[0][c] + red[1][c] + red[2][c] + red[3][c]);
  }
}

__global__ __launch_bounds__(256) void dropout_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ out, int64_t n4,
                                                      int W, DropoutParams dp) {
  dp = resolve_seed(dp);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    u32x2 w = reinterpret_cast<const u32x2*>(x)[i];
    // 4 elements of one row (W % 4 == 0): column pairs cp0 (even) and cp0 + 1 = cp0 ^ 1
    const int64_t row = (i * 4) / W;
    const uint32_t cp0 = (uint32_t)((i * 4 - row * W) >> 1);
    const uint32_t xw = drop_row((uint32_t)row, dp.key) ^ drop_col(cp0);
    const uint32_t b0 = drop_fin(xw), b1 = drop_fin(xw ^ drop_col(1));
    u32x2 o;
    o.x = pack_bf2(lo_bf(w.x) * keep_factor(b0, 0, dp), hi_bf(w.x) * keep_factor(b0, 1, dp));
    o.y = pack_bf2(lo_bf(w.y) * keep_factor(b1, 0, dp), hi_bf(w.y) * keep_factor(b1, 1, dp));
    reinterpret_cast<u32x2*>(out)[i] = o;
  }
}

static inline int grid_for(int64_t n, int per_thread_vecs_div = 1) {
  int64_t b = (n + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

void launch_gelu_fwd(const bf16_t* y, bf16_t* g, int64_t n, hipStream_t st) {
  int64_t n8 = n / 8;  // caller guarantees n % 8 == 0
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(grid_for(n8)), dim3(256), 0, st, y, g, n8);
  HSD_CHECK_LAUNCH();
}

static void colsum_launch(bool gelu, const bf16_t* x, const bf16_t* y, bf16_t* out, float* dbias, int rows, int N,
                          hipStream_t st) {
  const int gx = (N + 511) / 512;
  // ~2048 blocks (8 per CU); rows per block a multiple of 16 (4 row groups x 4 rows in flight)
  int want_y = max(1, 2048 / gx);
  int rpb = max(16, (rows + want_y - 1) / want_y);
  rpb = (rpb + 15) / 16 * 16;
  const int gy = (rows + rpb - 1) / rpb;
  if (gelu)
    hipLaunchKernelGGL((colsum_kernel<true>), dim3(gx, gy), dim3(256), 0, st, x, y, out, dbias, rows, N, rpb);
  else
    hipLaunchKernelGGL((colsum_kernel<false>), dim3(gx, gy), dim3(256), 0, st, x, y, out, dbias, rows, N, rpb);
  HSD_CHECK_LAUNCH();
}

void launch_gelu_bwd_colsum(const bf16_t* dg, const bf16_t* y, bf16_t* da, float* dbias, int rows, int N,
                            hipStream_t st) {
  colsum_launch(true, dg, y, da, dbias, rows, N, st);
}

void launch_colsum(const bf16_t* x, float* dbias, int rows, int N, hipStream_t st) {
  colsum_launch(false, x, nullptr, nullptr, dbias, rows, N, st);
}

// C[n][k] += Σ_t dy[t][n] · x[t][k]  (bf16 in, fp32 C) for token counts below one 64-token K-tile: the weight gradient of
// the classification head's dense layer at small batches (the reference's own B = 8), where gemm2's TT path does not
// tile. One thread per 4 consecutive k; the dy element is a wave-wide broadcast, the x row chunk an 8-B load.
__global__ __launch_bounds__(256) void small_wgrad_kernel(const bf16_t* __restrict__ dy, int64_t ldy,
                                                          const bf16_t* __restrict__ x, int64_t ldx, float* __restrict__ C,
                                                          int64_t ldc, int T, int N, int K) {
  const int64_t n4 = (int64_t)N * (K / 4);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(i / (K / 4));
    const int k = (int)(i % (K / 4)) * 4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < T; ++t) {
      const float d = bf2f(dy[(int64_t)t * ldy + n]);
      const u32x2 w = *reinterpret_cast<const u32x2*>(x + (int64_t)t * ldx + k);
      acc[0] = fmaf(d, lo_bf(w.x), acc[0]);
      acc[1] = fmaf(d, hi_bf(w.x), acc[1]);
      acc[2] = fmaf(d, lo_bf(w.y), acc[2]);
      acc[3] = fmaf(d, hi_bf(w.y), acc[3]);
    }
    f32x4* c = reinterpret_cast<f32x4*>(C + (int64_t)n * ldc + k);
    *c = *c + acc;
  }
}

void launch_small_wgrad(const bf16_t* dy, int64_t ldy, const bf16_t* x, int64_t ldx, float* C, int64_t ldc, int T,
                        int N, int K, hipStream_t st) {
  const int64_t n4 = (int64_t)N * (K / 4);
  hipLaunchKernelGGL(small_wgrad_kernel, dim3(grid_for(n4)), dim3(256), 0, st, dy, ldy, x, ldx, C, ldc, T, N, K);
  HSD_CHECK_LAUNCH();
}

// additive key-padding bias of attention: out = (1 - mask) * FLT_MIN (ops/reference.py key_mask_bias, bit for bit)
template <typename T>
__global__ __launch_bounds__(256) void mask_bias_kernel(const T* __restrict__ m, float* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (1.0f - (float)m[i]) * -3.4028234663852886e+38f;
}

void launch_mask_bias(const void* mask, bool i64, float* out, int64_t n, hipStream_t st) {
  if (i64) hipLaunchKernelGGL(mask_bias_kernel<int64_t>, dim3(grid_for(n)), dim3(256), 0, st, (const int64_t*)mask, out, n);
  else hipLaunchKernelGGL(mask_bias_kernel<int32_t>, dim3(grid_for(n)), dim3(256), 0, st, (const int32_t*)mask, out, n);
  HSD_CHECK_LAUNCH();
}

uint32_t dropout_pair_bits_host(uint64_t seed, uint32_t row, uint32_t cp) {
  const DropoutParams d = make_dropout(0.1, seed);
  return drop_fin(drop_row(row, d.key) ^ drop_col(cp));
}

void launch_dropout(const bf16_t* x, bf16_t* out, int64_t n, int W, double p, uint64_t seed, hipStream_t st) {
  DropoutParams dp = make_dropout(p, seed);
  int64_t n4 = n / 4;  // caller guarantees n % 4 == 0
  hipLaunchKernelGGL(dropout_kernel, dim3(grid_for(n4)), dim3(256), 0, st, x, out, n4, W, dp);
  HSD_CHECK_LAUNCH();
}

}  // namespace hsd

namespace hsd {

// Batched bf16 transpose for the dgrad weights: dst_i [cols][rows] = src_i [rows][cols]ᵀ for every matrix
// of a descriptor table {src, dst, rows, cols, first_tile} (int64 x 5, device memory), one launch for
// all of them after the optimizer step. Block = 256 threads = one 64x64 tile.
// Full tiles (the common case: every BERT weight dimension is a multiple of 64): 16-B global loads and stores, the
// tile staged through LDS as 16-B chunks (one ds_write_b128 per chunk) with the chunk index XOR-swizzled by the row
// block, so the column gathers (8 lanes = 8 row blocks of one column) hit 8 different chunk positions — conflict-free;
// each 8-lane group stores one 128-B output row. Edge tiles (dimensions multiple of 4 only): 8-B element path.
__global__ __launch_bounds__(256) void transpose_many_kernel(const int64_t* __restrict__ desc, int n) {
  __shared__ __attribute__((aligned(16))) u32x4 t16[64 * 8 + 16];  // + 16: the edge path's 64 x 66 bf16 tile
  const int bid = blockIdx.x;
  int mi = 0;
  while (mi + 1 < n && desc[(mi + 1) * 5 + 4] <= bid) ++mi;
  const bf16_t* src = reinterpret_cast<const bf16_t*>(desc[mi * 5 + 0]);
  bf16_t* dst = reinterpret_cast<bf16_t*>(desc[mi * 5 + 1]);
  const int rows = (int)desc[mi * 5 + 2], cols = (int)desc[mi * 5 + 3];
  const int t = bid - (int)desc[mi * 5 + 4];
  const int tcols = (cols + 63) / 64;
  const int r0 = (t / tcols) * 64, c0 = (t % tcols) * 64;
  const int tid = threadIdx.x;
  const bool full = r0 + 64 <= rows && c0 + 64 <= cols && (rows & 7) == 0 && (cols & 7) == 0;
  if (full) {
    u32x4 v[2];
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int q = tid + 256 * it, r = q >> 3, cc = q & 7;
      v[it] = *reinterpret_cast<const u32x4*>(src + (int64_t)(r0 + r) * cols + c0 + 8 * cc);
    }
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int q = tid + 256 * it, r = q >> 3, cc = q & 7;
      t16[r * 8 + (cc ^ ((r >> 3) & 7))] = v[it];
    }
    __syncthreads();
    const uint16_t* th = reinterpret_cast<const uint16_t*>(t16);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int q = tid + 256 * it, rg = q & 7, c = q >> 3;  // output row c (input column), input rows 8 rg .. 8 rg + 7
      const int pc = (c >> 3) ^ rg;                         // swizzled chunk of column c in row block rg
      uint32_t w[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = th[(rg * 8 + j) * 64 + pc * 8 + (c & 7)];
      u32x4 o;
      o.x = w[0] | (w[1] << 16);
      o.y = w[2] | (w[3] << 16);
      o.z = w[4] | (w[5] << 16);
      o.w = w[6] | (w[7] << 16);
      *reinterpret_cast<u32x4*>(dst + (int64_t)(c0 + c) * rows + r0 + 8 * rg) = o;
    }
    return;
  }
  bf16_t(*tile)[66] = reinterpret_cast<bf16_t(*)[66]>(t16);  // 64 x 66 bf16 = 8,448 B
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int r = (tid >> 4) + 16 * it, c = (tid & 15) * 4;
    if (r0 + r < rows && c0 + c + 3 < cols) {
      const u32x2 v = *reinterpret_cast<const u32x2*>(src + (int64_t)(r0 + r) * cols + c0 + c);
      tile[r][c] = (bf16_t)(v.x & 0xFFFF); tile[r][c + 1] = (bf16_t)(v.x >> 16);
      tile[r][c + 2] = (bf16_t)(v.y & 0xFFFF); tile[r][c + 3] = (bf16_t)(v.y >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int c = (tid >> 4) + 16 * it, r = (tid & 15) * 4;  // output row c (= input col), 4 input rows
    if (c0 + c < cols && r0 + r + 3 < rows) {
      u32x2 o;
      o.x = (uint32_t)tile[r][c] | ((uint32_t)tile[r + 1][c] << 16);
      o.y = (uint32_t)tile[r + 2][c] | ((uint32_t)tile[r + 3][c] << 16);
      *reinterpret_cast<u32x2*>(dst + (int64_t)(c0 + c) * rows + r0 + r) = o;
    }
  }
}

void launch_transpose_many(const int64_t* desc, int n, int total_tiles, hipStream_t st) {
  if (n <= 0 || total_tiles <= 0) return;
  hipLaunchKernelGGL(transpose_many_kernel, dim3(total_tiles), dim3(256), 0, st, desc, n);
  HSD_CHECK_LAUNCH();
}

// Gradient wire casts of the RCCL engine's 16-bit compression (comm_engine.cpp; Horovod's hvd.Compression.fp16 /
// bf16): to16: w = 16-bit(g · scale); from16: g = float(w) · scale. One pass each, 16-B loads and
// 8-B stores, where the ATen form was a scaled fp32 temporary + a cast copy (and back: a copy + an in-place mul).
// fp16: round-to-nearest-even via the hardware cvt; bf16: the shared RNE pack.
template <bool kHalf>
__global__ __launch_bounds__(256) void wire_to16_kernel(const float* __restrict__ g, uint16_t* __restrict__ w,
                                                        int64_t n4, float scale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const f32x4 v = reinterpret_cast<const f32x4*>(g)[i] * scale;
    u32x2 o;
    if constexpr (kHalf) {
      const _Float16 a = (_Float16)v[0], b = (_Float16)v[1], c = (_Float16)v[2], d = (_Float16)v[3];
      o.x = (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
      o.y = (uint32_t)__builtin_bit_cast(uint16_t, c) | ((uint32_t)__builtin_bit_cast(uint16_t, d) << 16);
    } else {
      o.x = pack_bf2(v[0], v[1]);
      o.y = pack_bf2(v[2], v[3]);
    }
    reinterpret_cast<u32x2*>(w)[i] = o;
  }
}

template <bool kHalf>
__global__ __launch_bounds__(256) void wire_from16_kernel(const uint16_t* __restrict__ w, float* __restrict__ g,
                                                          int64_t n4, float scale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const u32x2 v = reinterpret_cast<const u32x2*>(w)[i];
    f32x4 o;
    if constexpr (kHalf) {
      o[0] = (float)__builtin_bit_cast(_Float16, (uint16_t)(v.x & 0xFFFF));
      o[1] = (float)__builtin_bit_cast(_Float16, (uint16_t)(v.x >> 16));
      o[2] = (float)__builtin_bit_cast(_Float16, (uint16_t)(v.y & 0xFFFF));
      o[3] = (float)__builtin_bit_cast(_Float16, (uint16_t)(v.y >> 16));
    } else {
      o = f32x4{lo_bf(v.x), hi_bf(v.x), lo_bf(v.y), hi_bf(v.y)};
    }
    reinterpret_cast<f32x4*>(g)[i] = o * scale;
  }
}

static int wire_blocks(int64_t n4) { return (int)std::min<int64_t>(2048, std::max<int64_t>(1, (n4 + 255) / 256)); }

void launch_wire_cast(const void* src, void* dst, int64_t n, bool to16, bool half, float scale, hipStream_t st) {
  if (n <= 0) return;
  if (n % 4 != 0) {
    fprintf(stderr, "launch_wire_cast: n %% 4 != 0 (%lld)\n", (long long)n);
    abort();
  }
  const int64_t n4 = n / 4;
  if (to16) {
    if (half) hipLaunchKernelGGL(wire_to16_kernel<true>, dim3(wire_blocks(n4)), dim3(256), 0, st, (const float*)src, (uint16_t*)dst, n4, scale);
    else hipLaunchKernelGGL(wire_to16_kernel<false>, dim3(wire_blocks(n4)), dim3(256), 0, st, (const float*)src, (uint16_t*)dst, n4, scale);
  } else {
    if (half) hipLaunchKernelGGL(wire_from16_kernel<true>, dim3(wire_blocks(n4)), dim3(256), 0, st, (const uint16_t*)src, (float*)dst, n4, scale);
    else hipLaunchKernelGGL(wire_from16_kernel<false>, dim3(wire_blocks(n4)), dim3(256), 0, st, (const uint16_t*)src, (float*)dst, n4, scale);
  }
  HSD_CHECK_LAUNCH();
}

void set_dropout_dev_seed(const uint32_t* p) { g_dropout_dev_seed = p; }

void refresh_env_knobs() { ++g_env_gen; }

// Contention emulation (tools/contention_ab.py): `blocks` workgroups that each hold a whole CU (all 160 KiB of LDS,
// so no other 160-KiB workgroup -- the persistent GEMMs -- can share it) for `usec` microseconds, then exit. Stands
// in for the RCCL all-reduce kernels (one workgroup per channel) that a data-parallel step runs beside its backward
// GEMMs. Waits on the 100 MHz constant clock (s_memrealtime) with s_sleep between polls; every wave exits.
__global__ __launch_bounds__(64) void cu_hog_kernel(uint64_t ticks, float* sink) {
  __shared__ float hog_lds[160 * 1024 / 4];
  hog_lds[threadIdx.x] = (float)threadIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  __syncthreads();
  if (sink != nullptr) sink[threadIdx.x] = hog_lds[(threadIdx.x * 37) & 63];
}

void launch_cu_hog(int blocks, double usec, hipStream_t st) {
  if (blocks <= 0 || usec <= 0.0) return;
  hipLaunchKernelGGL(cu_hog_kernel, dim3(blocks), dim3(64), 0, st, (uint64_t)(usec * 100.0), (float*)nullptr);
  HSD_CHECK_LAUNCH();
}

}  // namespace hsd
