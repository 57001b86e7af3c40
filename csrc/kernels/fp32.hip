// fp32 step kernels: the reference's own precision (TF 2.4 Keras with no mixed-precision policy,
// /root/reference/scripts/train.py:113-123) on hand-written gfx950 kernels (ops/hip32.py drives them; VERDICT r3
// 'missing 2'). Every tensor is fp32 in HBM; statistics and accumulations are fp32.
//
// * GEMMs (ops/hip32.py) run on the bf16 MFMA kernels as 3-term split products: x = hi + lo with hi = bf16(x),
//   lo = bf16(x - hi) (|x - hi - lo| <= 2^-17 |x|), and A·Bᵀ ≈ Ah·Bhᵀ + Ah·Blᵀ + Al·Bhᵀ (the dropped Al·Blᵀ is
//   <= 2^-16 of each product) summed in fp32 by ONE GEMM over the concatenated K: [Ah|Ah|Al]·[Bh|Bl|Bh]ᵀ.
//   split3 below writes those concatenations; the GEMM epilogues (bias, GELU, dropout + residual) are fp32
//   element passes here.
// * LayerNorm forward / backward, one wave per row, two-pass statistics in fp32.
// * embedding gather-add and its scatter-add backward (fp32 atomics).
// * attention: streaming fp32 (online softmax, exact fp32 FMAs on the VALU: gfx950's fp32 MFMA rate equals the
//   fp32 VALU rate, MI355X_MICROARCH.md 'Peak FP32 (matrix)'), one query per lane, K/V tiles broadcast from LDS;
//   backward as three passes (dQ: queries on lanes; dV and dK: keys on lanes) so no gradient needs atomics.
// * the sequence-classification head's activation, dropout, classifier, cross-entropy and accuracy.
// Dropout masks come from the shared counter hash (common.h / ops/rng.py) with the same element indexing as the bf16
// kernels and the torch reference, so fp32 runs draw the reference's masks bit for bit.
#include "common.h"

namespace hsd {
namespace f32k {

// ------------------------------------------------------------------------------------------------ split3
// out = 3 blocks of x [R][C], block b = lo(x) if (pat >> b) & 1 else hi(x); blocks side by side along the columns
// (out [R][3C]) or stacked along the rows (out [3R][C]). C % 4 == 0; V = 8 elements per step (16-B stores) when
// C % 8 == 0. The (row, column) of a thread's element group advance incrementally by the grid stride: one 64-bit
// division per thread instead of a 64-bit division and remainder per step (those dominated the kernel's VALU).
// out2 (optional): a second copy in the row-stacked layout [3R][C] with pattern pat2, written from the same read (the
// incoming gradient of a linear layer feeds both its dgrad, column blocks, and its weight gradient, row blocks)
template <int V>
__global__ __launch_bounds__(256) void split3_kernel(const float* __restrict__ x, bf16_t* __restrict__ out, int64_t R,
                                                     int64_t C, int pat, int rows, bf16_t* __restrict__ out2,
                                                     int pat2) {
  const int64_t cvn = C / V, n = R * cvn;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t r = i / cvn, cv = i - r * cvn;
  const int64_t sr = stride / cvn, sc = stride - sr * cvn;
  for (; i < n; i += stride) {
    const int64_t c = cv * V;
    uint32_t hw[V / 2], lw[V / 2];
#pragma unroll
    for (int q = 0; q < V / 4; ++q) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(x + r * C + c + 4 * q);
      float h[4], l[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        h[e] = bf2f(f2bf(v[e]));
        l[e] = v[e] - h[e];
      }
      hw[2 * q] = pack_bf2(h[0], h[1]);
      hw[2 * q + 1] = pack_bf2(h[2], h[3]);
      lw[2 * q] = pack_bf2(l[0], l[1]);
      lw[2 * q + 1] = pack_bf2(l[2], l[3]);
    }
#pragma unroll
    for (int bb = 0; bb < 3; ++bb) {
      const int64_t off = rows ? ((int64_t)bb * R + r) * C + c : r * 3 * C + (int64_t)bb * C + c;
      const uint32_t* w = ((pat >> bb) & 1) ? lw : hw;
      if constexpr (V == 8) {
        *reinterpret_cast<u32x4*>(out + off) = u32x4{w[0], w[1], w[2], w[3]};
      } else {
        *reinterpret_cast<u32x2*>(out + off) = u32x2{w[0], w[1]};
      }
    }
    if (out2 != nullptr) {
#pragma unroll
      for (int bb = 0; bb < 3; ++bb) {
        const int64_t off = ((int64_t)bb * R + r) * C + c;
        const uint32_t* w = ((pat2 >> bb) & 1) ? lw : hw;
        if constexpr (V == 8) {
          *reinterpret_cast<u32x4*>(out2 + off) = u32x4{w[0], w[1], w[2], w[3]};
        } else {
          *reinterpret_cast<u32x2*>(out2 + off) = u32x2{w[0], w[1]};
        }
      }
    }
    cv += sc;
    r += sr;
    if (cv >= cvn) {
      cv -= cvn;
      ++r;
    }
  }
}

// ------------------------------------------------------------------------------------------------ epilogues
// y [M][N] (the GEMM's fp32 accumulation, modified in place where noted), bias [N]:
//   0: out = y + bias
//   1: y = y + bias (the pre-activation, kept for backward), out = gelu_erf(y)
//   2: out = dropout(y + bias) + res          (dropout element index m·N + n)
//   3: out = y + res                          (dgrad + residual gradient)
//   4: out = y · gelu'(aux)                   (dgrad through GELU; aux = saved pre-activation)
// hi / lo (optional): out's bf16 halves for the next split-product GEMM (no split2 pass); out may then be null (the
// fp32 value is not needed: the QKV projection's output, the GELU output)
__global__ __launch_bounds__(256) void epi32_kernel(float* __restrict__ y, const float* __restrict__ bias,
                                                    const float* __restrict__ aux, float* __restrict__ out,
                                                    int64_t M, int N, int kind, DropoutParams dp,
                                                    bf16_t* __restrict__ hi, bf16_t* __restrict__ lo) {
  dp = resolve_seed(dp);
  const int64_t n4 = M * N / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int N4 = N / 4;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  // row m / column n0 of group i, advanced by the grid stride (no 64-bit division per step, as split3_kernel)
  int64_t m = i / N4;
  int c4 = (int)(i - m * N4);
  const int64_t sr = stride / N4;
  const int sc = (int)(stride - sr * N4);
  for (; i < n4; i += stride) {
    const int n0 = 4 * c4;
    f32x4 v = reinterpret_cast<const f32x4*>(y)[i];
    if (bias != nullptr) v += *reinterpret_cast<const f32x4*>(bias + n0);
    f32x4 o;
    if (kind == 0) {
      o = v;
    } else if (kind == 1) {
      reinterpret_cast<f32x4*>(y)[i] = v;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = 0.5f * v[e] * (1.0f + erff(v[e] * 0.70710678118654752f));
    } else if (kind == 2) {
      if (dp.enabled) {
        uint32_t b0, b1;
        dropout_bits4((uint32_t)m, (uint32_t)n0, dp, b0, b1);
        v[0] *= keep_factor(b0, 0, dp);
        v[1] *= keep_factor(b0, 1, dp);
        v[2] *= keep_factor(b1, 0, dp);
        v[3] *= keep_factor(b1, 1, dp);
      }
      o = v + reinterpret_cast<const f32x4*>(aux)[i];
    } else if (kind == 3) {
      o = v + reinterpret_cast<const f32x4*>(aux)[i];
    } else {
      const f32x4 a = reinterpret_cast<const f32x4*>(aux)[i];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = a[e];
        const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
        o[e] = v[e] * (cdf + x * 0.3989422804014327f * expf(-0.5f * x * x));
      }
    }
    if (out != nullptr) reinterpret_cast<f32x4*>(out)[i] = o;
    if (hi != nullptr) store_halves4(hi, lo, i, o[0], o[1], o[2], o[3]);
    c4 += sc;
    m += sr;
    if (c4 >= N4) {
      c4 -= N4;
      ++m;
    }
  }
}

// out = x · keep (mask rows of width W = the last dimension, W % 4 == 0), in place allowed; hi / lo (optional): out's
// bf16 halves
__global__ __launch_bounds__(256) void dropout32_kernel(const float* __restrict__ x, float* out, int64_t n4, int W,
                                                        DropoutParams dp, bf16_t* __restrict__ hi,
                                                        bf16_t* __restrict__ lo) {
  dp = resolve_seed(dp);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int W4 = W / 4;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  int64_t row = i / W4;
  int c4 = (int)(i - row * W4);
  const int64_t sr = stride / W4;
  const int sc = (int)(stride - sr * W4);
  for (; i < n4; i += stride) {
    f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    uint32_t b0, b1;
    dropout_bits4((uint32_t)row, (uint32_t)(4 * c4), dp, b0, b1);
    v[0] *= keep_factor(b0, 0, dp);
    v[1] *= keep_factor(b0, 1, dp);
    v[2] *= keep_factor(b1, 0, dp);
    v[3] *= keep_factor(b1, 1, dp);
    reinterpret_cast<f32x4*>(out)[i] = v;
    if (hi != nullptr) store_halves4(hi, lo, i, v[0], v[1], v[2], v[3]);
    c4 += sc;
    row += sr;
    if (c4 >= W4) {
      c4 -= W4;
      ++row;
    }
  }
}

// column sums: dbias[n] += Σ_m x[m][n]. Block: 64 columns x 4 row groups; one atomic per column per block (N % 4 != 0)
__global__ __launch_bounds__(256) void colsum32_scalar_kernel(const float* __restrict__ x, float* __restrict__ dbias,
                                                              int M, int N, int rows_per_block) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), rg = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float acc = 0.f;
  if (c < N)
    for (int r = r0 + rg; r < r1; r += 4) acc += x[(int64_t)r * N + c];
  red[rg][threadIdx.x & 63] = acc;
  __syncthreads();
  if (rg == 0 && c < N) atomicAdd(dbias + c, red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                                                 red[3][threadIdx.x]);
}

// N % 4 == 0: block = 256 columns x 4 row groups, >= 256 rows per block: every block ends with
// 256 column atomics on the same addresses, so few long blocks win (4096 x 1024: 51 us at 4 rows, 5.6 at 256;
// profiles/colsum32_rows_r5.log)
__global__ __launch_bounds__(256) void colsum32_kernel(const float* __restrict__ x, float* __restrict__ dbias, int M,
                                                       int N, int rows_per_block) {
  // 16-B column chunks (4 columns per lane, 256 per block row group), four rows' loads in flight per lane
  __shared__ f32x4 red[4][64];
  const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = (blockIdx.x * 64 + lane) * 4;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(M, r0 + rows_per_block);
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  if (c < N) {
    const float* xc = x + c;
    int r = r0 + rg;
    for (; r + 12 < r1; r += 16) {
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(xc + (int64_t)r * N);
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(xc + (int64_t)(r + 4) * N);
      const f32x4 a2 = *reinterpret_cast<const f32x4*>(xc + (int64_t)(r + 8) * N);
      const f32x4 a3 = *reinterpret_cast<const f32x4*>(xc + (int64_t)(r + 12) * N);
      acc += (a0 + a1) + (a2 + a3);
    }
    for (; r < r1; r += 4) acc += *reinterpret_cast<const f32x4*>(xc + (int64_t)r * N);
  }
  red[rg][lane] = acc;
  __syncthreads();
  if (rg == 0 && c < N) {
    const f32x4 t = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
#pragma unroll
    for (int e = 0; e < 4; ++e) atomicAdd(dbias + c + e, t[e]);
  }
}

// ------------------------------------------------------------------------------------------------ LayerNorm
// one wave per row; lane owns columns lane*4 + 256j (H % 4 == 0, H <= 1024): NJ = ceil(H / 256) float4 chunks
template <int NJ>
__global__ __launch_bounds__(256) void ln32_fwd_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                       const float* __restrict__ b, float* __restrict__ out,
                                                       float* __restrict__ mean, float* __restrict__ rstd, int R,
                                                       int H, float eps, bf16_t* __restrict__ hi,
                                                       bf16_t* __restrict__ lo) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const float* xr = x + (int64_t)row * H;
  f32x4 v[NJ];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane * 4 + 256 * j;
    v[j] = c < H ? *reinterpret_cast<const f32x4*>(xr + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    s += v[j][0] + v[j][1] + v[j][2] + v[j][3];
  }
  const float mu = wave_sum(s) / (float)H;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane * 4 + 256 * j;
    if (c < H)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[j][e] - mu;
        q += d * d;
      }
  }
  const float rs = rsqrtf(wave_sum(q) / (float)H + eps);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane * 4 + 256 * j;
    if (c < H) {
      const f32x4 gg = *reinterpret_cast<const f32x4*>(g + c), bb = *reinterpret_cast<const f32x4*>(b + c);
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (v[j][e] - mu) * rs * gg[e] + bb[e];
      *reinterpret_cast<f32x4*>(out + (int64_t)row * H + c) = o;
      if (hi != nullptr) store_halves4(hi, lo, ((int64_t)row * H + c) / 4, o[0], o[1], o[2], o[3]);
    }
  }
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// dx = rstd·(dy·g − mean(dy·g) − x̂·mean(dy·g·x̂)); dgamma += Σ dy·x̂, dbeta += Σ dy (per-lane partials over the
// rows a wave walks, one atomic per column per wave). dx may alias dy.
template <int NJ>
__global__ __launch_bounds__(256) void ln32_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                       const float* __restrict__ mean, const float* __restrict__ rstd,
                                                       const float* __restrict__ g, float* dx,
                                                       float* __restrict__ dg, float* __restrict__ db, int R, int H,
                                                       int rows_per_wave) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int r0 = w * rows_per_wave, r1 = min(R, r0 + rows_per_wave);
  f32x4 pg[NJ], pb[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) pg[j] = pb[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int row = r0; row < r1; ++row) {
    const float mu = mean[row], rs = rstd[row];
    f32x4 xh[NJ], dyg[NJ], dyv[NJ];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = lane * 4 + 256 * j;
      if (c < H) {
        const f32x4 xv = *reinterpret_cast<const f32x4*>(x + (int64_t)row * H + c);
        dyv[j] = *reinterpret_cast<const f32x4*>(dy + (int64_t)row * H + c);
        const f32x4 gg = *reinterpret_cast<const f32x4*>(g + c);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          xh[j][e] = (xv[e] - mu) * rs;
          dyg[j][e] = dyv[j][e] * gg[e];
          s1 += dyg[j][e];
          s2 += dyg[j][e] * xh[j][e];
        }
        pg[j] += dyv[j] * xh[j];
        pb[j] += dyv[j];
      }
    }
    s1 = wave_sum(s1) / (float)H;
    s2 = wave_sum(s2) / (float)H;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = lane * 4 + 256 * j;
      if (c < H) {
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = rs * (dyg[j][e] - s1 - xh[j][e] * s2);
        *reinterpret_cast<f32x4*>(dx + (int64_t)row * H + c) = o;
      }
    }
  }
  // γ/β partials: the block's 4 waves are summed in LDS first, then one atomic per column per BLOCK (per-wave atomics
  // put thousands of waves on the same H addresses: 237 us per bert-large layer at 4096 rows, kernel_stats_r5_fp32)
  __shared__ float red[2][4][NJ * 256];
  const int wv = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[0][wv][256 * j + lane * 4 + e] = r0 < r1 ? pg[j][e] : 0.f;
      red[1][wv][256 * j + lane * 4 + e] = r0 < r1 ? pb[j][e] : 0.f;
    }
  __syncthreads();
  for (int c = threadIdx.x; c < H; c += 256) {
    const float sg = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    const float sb = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
    atomicAdd(dg + c, sg);
    atomicAdd(db + c, sb);
  }
}

// ------------------------------------------------------------------------------------------------ embeddings
// x[r] = word[ids[r]] + pos[pos_ids[r]] (+ type[type_ids[r]]); one wave per row
__global__ __launch_bounds__(256) void embed32_gather_kernel(const int64_t* __restrict__ ids,
                                                             const int64_t* __restrict__ pids,
                                                             const int64_t* __restrict__ tids,
                                                             const float* __restrict__ word,
                                                             const float* __restrict__ pos,
                                                             const float* __restrict__ type, float* __restrict__ x,
                                                             int R, int H) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const float* wr = word + ids[row] * (int64_t)H;
  const float* pr = pos + pids[row] * (int64_t)H;
  const float* tr = type != nullptr ? type + (tids != nullptr ? tids[row] : 0) * (int64_t)H : nullptr;
  for (int c = lane * 4; c < H; c += 256) {
    f32x4 v = *reinterpret_cast<const f32x4*>(wr + c) + *reinterpret_cast<const f32x4*>(pr + c);
    if (tr != nullptr) v += *reinterpret_cast<const f32x4*>(tr + c);
    *reinterpret_cast<f32x4*>(x + (int64_t)row * H + c) = v;
  }
}

// table gradients: gword[ids[r]] += dx[r], gpos[pos_ids[r]] += dx[r], gtype[type_ids[r]] += dx[r]
__global__ __launch_bounds__(256) void embed32_scatter_kernel(const float* __restrict__ dx,
                                                              const int64_t* __restrict__ ids,
                                                              const int64_t* __restrict__ pids,
                                                              const int64_t* __restrict__ tids,
                                                              float* __restrict__ gword, float* __restrict__ gpos,
                                                              float* __restrict__ gtype, int R, int H) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  float* gw = gword + ids[row] * (int64_t)H;
  float* gp = gpos != nullptr ? gpos + pids[row] * (int64_t)H : nullptr;
  float* gt = gtype != nullptr ? gtype + (tids != nullptr ? tids[row] : 0) * (int64_t)H : nullptr;
  for (int c = lane; c < H; c += 64) {
    const float v = dx[(int64_t)row * H + c];
    atomicAdd(gw + c, v);
    if (gp != nullptr) atomicAdd(gp + c, v);
    if (gt != nullptr) atomicAdd(gt + c, v);
  }
}

// ------------------------------------------------------------------------------------------------ attention
// qkv [B·S][3H] (q | k | v, head h at columns h·64), out [B·S][H]; mask: additive key bias [B][S] or null;
// lse [B·heads·S] = log2-domain log-sum-exp of the scaled scores (log2(e)/√d · q·k + log2(e)·mask).
// One query per lane, 64 queries per block (one wave), keys in tiles of KT through LDS (broadcast reads).
constexpr int AD = 64, KT = 32, CH = 4;
constexpr float kLog2e32 = 1.4426950408889634f;

__global__ __launch_bounds__(64) void attn32_fwd_kernel(const float* __restrict__ qkv, const float* __restrict__ mask,
                                                        float* __restrict__ out, float* __restrict__ lse, int S,
                                                        int heads, float sl2, DropoutParams dp) {
  dp = resolve_seed(dp);
  __shared__ __attribute__((aligned(16))) float Ks[KT][AD], Vs[KT][AD];
  __shared__ float mb[KT];
  const int lane = threadIdx.x;
  const int bh = blockIdx.x, b = bh / heads, h = bh % heads;
  const int H = heads * AD, ld = 3 * H;
  const int q = blockIdx.y * 64 + lane;
  const bool valid = q < S;
  const float* base = qkv + (int64_t)b * S * ld + h * AD;
  float qv[AD], o[AD];
#pragma unroll
  for (int d = 0; d < AD; d += 4) {
    const f32x4 t = valid ? *reinterpret_cast<const f32x4*>(base + (int64_t)q * ld + d) : f32x4{0.f, 0.f, 0.f, 0.f};
    qv[d] = t[0] * sl2; qv[d + 1] = t[1] * sl2; qv[d + 2] = t[2] * sl2; qv[d + 3] = t[3] * sl2;
    o[d] = o[d + 1] = o[d + 2] = o[d + 3] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  // dropout row word of (bh, q): mask row bh S + q, column pair key / 2 (ops/rng.py)
  const uint32_t rw = dropout_row((uint32_t)(bh * S + q), dp);
  for (int k0 = 0; k0 < S; k0 += KT) {
    __syncthreads();
    // stage K / V rows k0 .. k0 + KT (64 lanes x 8 float4 each per matrix)
    for (int i = lane; i < KT * AD / 4; i += 64) {
      const int kr = i / (AD / 4), c = (i % (AD / 4)) * 4;
      const bool in = k0 + kr < S;
      const float* kp = base + (int64_t)(k0 + kr) * ld;
      *reinterpret_cast<f32x4*>(&Ks[kr][c]) = in ? *reinterpret_cast<const f32x4*>(kp + H + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f32x4*>(&Vs[kr][c]) = in ? *reinterpret_cast<const f32x4*>(kp + 2 * H + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (lane < KT) {
      const int k = k0 + lane;
      mb[lane] = k < S ? (mask != nullptr ? fmaxf(mask[(int64_t)b * S + k] * kLog2e32, -1e30f) : 0.f) : -INFINITY;
    }
    __syncthreads();
    // chunks of CH keys: scores, one online-softmax rescale, probabilities, P·V (compile-time register indices)
#pragma unroll 1
    for (int j0 = 0; j0 < KT; j0 += CH) {
      float s[CH];
      float mx = m;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        float acc = 0.f;
#pragma unroll
        for (int d = 0; d < AD; d += 4) {
          const f32x4 kk = *reinterpret_cast<const f32x4*>(&Ks[j0 + j][d]);
          acc = fmaf(qv[d], kk[0], acc);
          acc = fmaf(qv[d + 1], kk[1], acc);
          acc = fmaf(qv[d + 2], kk[2], acc);
          acc = fmaf(qv[d + 3], kk[3], acc);
        }
        s[j] = acc + mb[j0 + j];
        mx = fmaxf(mx, s[j]);
      }
      const float corr = exp2f(m - mx);  // m = -inf before the first chunk: 0
      l *= corr;
#pragma unroll
      for (int d = 0; d < AD; ++d) o[d] *= corr;
      m = mx;
      // (k0 + j0) / 2 is a multiple of CH / 2 (powers of two): C((k0 + j0 + j) / 2) = C((k0 + j0) / 2) ^ C(j / 2)
      const uint32_t xc = dp.enabled ? rw ^ drop_col((uint32_t)(k0 + j0) >> 1) : 0u;
#pragma unroll
      for (int j = 0; j < CH; j += 2) {
        float p0 = exp2f(s[j] - m), p1 = exp2f(s[j + 1] - m);
        l += p0 + p1;
        if (dp.enabled) {
          const uint32_t bits = drop_fin(xc ^ drop_col((uint32_t)j >> 1));
          p0 *= keep_factor(bits, 0, dp);
          p1 *= keep_factor(bits, 1, dp);
        }
#pragma unroll
        for (int d = 0; d < AD; d += 4) {
          const f32x4 v0 = *reinterpret_cast<const f32x4*>(&Vs[j0 + j][d]);
          const f32x4 v1 = *reinterpret_cast<const f32x4*>(&Vs[j0 + j + 1][d]);
#pragma unroll
          for (int e = 0; e < 4; ++e) o[d + e] = fmaf(p1, v1[e], fmaf(p0, v0[e], o[d + e]));
        }
      }
    }
  }
  if (!valid) return;
  const float inv = 1.0f / l;
  float* op = out + ((int64_t)b * S + q) * H + h * AD;
#pragma unroll
  for (int d = 0; d < AD; d += 4)
    *reinterpret_cast<f32x4*>(op + d) = f32x4{o[d] * inv, o[d + 1] * inv, o[d + 2] * inv, o[d + 3] * inv};
  lse[(int64_t)bh * S + q] = m + __log2f(l);
}

// delta[bh·S + q] = Σ_d dO[q][d]·O[q][d]
__global__ __launch_bounds__(256) void attn32_delta_kernel(const float* __restrict__ o, const float* __restrict__ dout,
                                                           float* __restrict__ delta, int B, int S, int heads) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // (b, h, q) flattened as bh·S + q
  if (i >= B * heads * S) return;
  const int q = i % S, bh = i / S, b = bh / heads, h = bh % heads;
  const int64_t off = ((int64_t)b * S + q) * heads * AD + h * AD;
  float acc = 0.f;
#pragma unroll
  for (int d = 0; d < AD; d += 4) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(o + off + d), g = *reinterpret_cast<const f32x4*>(dout + off + d);
    acc += a[0] * g[0] + a[1] * g[1] + a[2] * g[2] + a[3] * g[3];
  }
  delta[i] = acc;
}

// dQ pass: one query per lane; dq = scale · Σ_k ds_qk · k,  ds = p · (keep · dO·v − delta)
__global__ __launch_bounds__(64) void attn32_dq_kernel(const float* __restrict__ qkv, const float* __restrict__ mask,
                                                       const float* __restrict__ dout, const float* __restrict__ lse,
                                                       const float* __restrict__ delta, float* __restrict__ dqkv,
                                                       int S, int heads, float sl2, float scale, DropoutParams dp) {
  dp = resolve_seed(dp);
  __shared__ __attribute__((aligned(16))) float Ks[KT][AD], Vs[KT][AD];
  __shared__ float mb[KT];
  const int lane = threadIdx.x;
  const int bh = blockIdx.x, b = bh / heads, h = bh % heads;
  const int H = heads * AD, ld = 3 * H;
  const int q = blockIdx.y * 64 + lane;
  const bool valid = q < S;
  const float* base = qkv + (int64_t)b * S * ld + h * AD;
  float qv[AD], dov[AD], dq[AD];
#pragma unroll
  for (int d = 0; d < AD; d += 4) {
    const f32x4 t = valid ? *reinterpret_cast<const f32x4*>(base + (int64_t)q * ld + d) : f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 g = valid ? *reinterpret_cast<const f32x4*>(dout + ((int64_t)b * S + q) * H + h * AD + d)
                          : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      qv[d + e] = t[e] * sl2;
      dov[d + e] = g[e];
      dq[d + e] = 0.f;
    }
  }
  const float ls = valid ? lse[(int64_t)bh * S + q] : 0.f;
  const float dl = valid ? delta[(int64_t)bh * S + q] : 0.f;
  const uint32_t rw = dropout_row((uint32_t)(bh * S + q), dp);
  for (int k0 = 0; k0 < S; k0 += KT) {
    __syncthreads();
    for (int i = lane; i < KT * AD / 4; i += 64) {
      const int kr = i / (AD / 4), c = (i % (AD / 4)) * 4;
      const bool in = k0 + kr < S;
      const float* kp = base + (int64_t)(k0 + kr) * ld;
      *reinterpret_cast<f32x4*>(&Ks[kr][c]) = in ? *reinterpret_cast<const f32x4*>(kp + H + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f32x4*>(&Vs[kr][c]) = in ? *reinterpret_cast<const f32x4*>(kp + 2 * H + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (lane < KT) {
      const int k = k0 + lane;
      mb[lane] = k < S ? (mask != nullptr ? fmaxf(mask[(int64_t)b * S + k] * kLog2e32, -1e30f) : 0.f) : -INFINITY;
    }
    __syncthreads();
#pragma unroll 1
    for (int j = 0; j < KT; j += 2) {
      float sd[2], dp2[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float a = 0.f, c = 0.f;
#pragma unroll
        for (int d = 0; d < AD; d += 4) {
          const f32x4 kk = *reinterpret_cast<const f32x4*>(&Ks[j + u][d]);
          const f32x4 vv = *reinterpret_cast<const f32x4*>(&Vs[j + u][d]);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            a = fmaf(qv[d + e], kk[e], a);
            c = fmaf(dov[d + e], vv[e], c);
          }
        }
        sd[u] = a + mb[j + u];
        dp2[u] = c;
      }
      float k0f = 1.f, k1f = 1.f;
      if (dp.enabled) {
        const uint32_t bits = dropout_bits_rc(rw, (uint32_t)(k0 + j) >> 1);
        k0f = keep_factor(bits, 0, dp);
        k1f = keep_factor(bits, 1, dp);
      }
      const float p0 = exp2f(sd[0] - ls), p1 = exp2f(sd[1] - ls);
      const float ds0 = p0 * fmaf(dp2[0], k0f, -dl), ds1 = p1 * fmaf(dp2[1], k1f, -dl);
#pragma unroll
      for (int d = 0; d < AD; d += 4) {
        const f32x4 ka = *reinterpret_cast<const f32x4*>(&Ks[j][d]);
        const f32x4 kb = *reinterpret_cast<const f32x4*>(&Ks[j + 1][d]);
#pragma unroll
        for (int e = 0; e < 4; ++e) dq[d + e] = fmaf(ds1, kb[e], fmaf(ds0, ka[e], dq[d + e]));
      }
    }
  }
  if (!valid) return;
  float* op = dqkv + ((int64_t)b * S + q) * ld + h * AD;
#pragma unroll
  for (int d = 0; d < AD; d += 4)
    *reinterpret_cast<f32x4*>(op + d) = f32x4{dq[d] * scale, dq[d + 1] * scale, dq[d + 2] * scale, dq[d + 3] * scale};
}

// dK / dV passes: one key per lane, queries in tiles through LDS.
//   DV: dv_k = Σ_q p_qk · keep_qk · dO_q            (registers: k, dv)
//   DK: dk_k = scale · Σ_q ds_qk · q_q                (registers: k, v, dk)
template <bool DV>
__global__ __launch_bounds__(64) void attn32_dkv_kernel(const float* __restrict__ qkv, const float* __restrict__ mask,
                                                        const float* __restrict__ dout, const float* __restrict__ lse,
                                                        const float* __restrict__ delta, float* __restrict__ dqkv,
                                                        int S, int heads, float sl2, float scale, DropoutParams dp) {
  dp = resolve_seed(dp);
  __shared__ __attribute__((aligned(16))) float Qs[KT][AD], Gs[KT][AD];
  __shared__ float lse_s[KT], del_s[KT];
  const int lane = threadIdx.x;
  const int bh = blockIdx.x, b = bh / heads, h = bh % heads;
  const int H = heads * AD, ld = 3 * H;
  const int k = blockIdx.y * 64 + lane;
  const bool valid = k < S;
  const float* base = qkv + (int64_t)b * S * ld + h * AD;
  const float kbias = valid ? (mask != nullptr ? fmaxf(mask[(int64_t)b * S + k] * kLog2e32, -1e30f) : 0.f) : -INFINITY;
  float kv[AD], vv[DV ? 1 : AD], acc[AD];
#pragma unroll
  for (int d = 0; d < AD; d += 4) {
    const f32x4 t = valid ? *reinterpret_cast<const f32x4*>(base + (int64_t)k * ld + H + d) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      kv[d + e] = t[e];
      acc[d + e] = 0.f;
    }
    if constexpr (!DV) {
      const f32x4 u = valid ? *reinterpret_cast<const f32x4*>(base + (int64_t)k * ld + 2 * H + d)
                            : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) vv[d + e] = u[e];
    }
  }
  // dropout mask of (q, k): row bh S + q (the row word is wave-uniform per query), column pair k / 2, element k & 1
  const uint32_t kc = drop_col((uint32_t)k >> 1);
  for (int q0 = 0; q0 < S; q0 += KT) {
    __syncthreads();
    for (int i = lane; i < KT * AD / 4; i += 64) {
      const int qr = i / (AD / 4), c = (i % (AD / 4)) * 4;
      const bool in = q0 + qr < S;
      *reinterpret_cast<f32x4*>(&Qs[qr][c]) =
          in ? *reinterpret_cast<const f32x4*>(base + (int64_t)(q0 + qr) * ld + c) * sl2 : f32x4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f32x4*>(&Gs[qr][c]) =
          in ? *reinterpret_cast<const f32x4*>(dout + ((int64_t)b * S + q0 + qr) * H + h * AD + c)
             : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (lane < KT) {
      const bool in = q0 + lane < S;
      lse_s[lane] = in ? lse[(int64_t)bh * S + q0 + lane] : INFINITY;  // out-of-range queries: p = 0
      del_s[lane] = in ? delta[(int64_t)bh * S + q0 + lane] : 0.f;
    }
    __syncthreads();
#pragma unroll 1
    for (int i = 0; i < KT; ++i) {
      float a = 0.f, c = 0.f;
#pragma unroll
      for (int d = 0; d < AD; d += 4) {
        const f32x4 qq = *reinterpret_cast<const f32x4*>(&Qs[i][d]);
#pragma unroll
        for (int e = 0; e < 4; ++e) a = fmaf(qq[e], kv[d + e], a);
        if constexpr (!DV) {
          const f32x4 gg = *reinterpret_cast<const f32x4*>(&Gs[i][d]);
#pragma unroll
          for (int e = 0; e < 4; ++e) c = fmaf(gg[e], vv[d + e], c);
        }
      }
      const float p = exp2f(a + kbias - lse_s[i]);
      float kf = 1.f;
      if (dp.enabled) {
        kf = keep_factor(drop_fin(dropout_row((uint32_t)(bh * S + q0 + i), dp) ^ kc), k & 1, dp);
      }
      if constexpr (DV) {
        const float w = p * kf;
#pragma unroll
        for (int d = 0; d < AD; d += 4) {
          const f32x4 gg = *reinterpret_cast<const f32x4*>(&Gs[i][d]);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[d + e] = fmaf(w, gg[e], acc[d + e]);
        }
      } else {
        const float ds = p * fmaf(c, kf, -del_s[i]);
#pragma unroll
        for (int d = 0; d < AD; d += 4) {
          const f32x4 qq = *reinterpret_cast<const f32x4*>(&Qs[i][d]);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[d + e] = fmaf(ds, qq[e], acc[d + e]);
        }
      }
    }
  }
  if (!valid) return;
  // DK: Qs held q · sl2 = q · log2(e)/√d; dk = (1/√d) Σ ds q = Σ ds (q·sl2) / log2(e)
  const float f = DV ? 1.0f : scale / sl2;
  float* op = dqkv + ((int64_t)b * S + k) * ld + (DV ? 2 * H : H) + h * AD;
#pragma unroll
  for (int d = 0; d < AD; d += 4)
    *reinterpret_cast<f32x4*>(op + d) = f32x4{acc[d] * f, acc[d + 1] * f, acc[d + 2] * f, acc[d + 3] * f};
}

// ------------------------------------------------------------------------------------------------ cls head
// rows r < R of pre [R][H] (pooler pre-activation): t = dropout(act(pre)) (saved), logits = t·W2ᵀ + b2 [R][C],
// stats[0] += Σ CE, stats[1] += Σ correct (argmax == label). One wave per row; C <= 8.
__global__ __launch_bounds__(64) void cls32_fwd_kernel(const float* __restrict__ pre, const float* __restrict__ W2,
                                                       const float* __restrict__ b2, const int64_t* __restrict__ labels,
                                                       float* __restrict__ t_out, float* __restrict__ logits,
                                                       float* __restrict__ stats, int R, int H, int C, int act,
                                                       DropoutParams dp) {
  dp = resolve_seed(dp);
  const int r = blockIdx.x, lane = threadIdx.x;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int c0 = lane * 2; c0 < H; c0 += 128) {
    float t[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float x = pre[(int64_t)r * H + c0 + e];
      t[e] = act == 0 ? tanhf(x) : fmaxf(x, 0.f);
    }
    if (dp.enabled) {
      const uint32_t bits = dropout_bits2((uint32_t)r, (uint32_t)c0 >> 1, dp);
      t[0] *= keep_factor(bits, 0, dp);
      t[1] *= keep_factor(bits, 1, dp);
    }
    t_out[(int64_t)r * H + c0] = t[0];
    t_out[(int64_t)r * H + c0 + 1] = t[1];
    for (int c = 0; c < C; ++c) acc[c] += t[0] * W2[(int64_t)c * H + c0] + t[1] * W2[(int64_t)c * H + c0 + 1];
  }
  float lg[8];
  for (int c = 0; c < C; ++c) lg[c] = wave_sum(acc[c]) + b2[c];
  if (lane == 0) {
    float mx = -INFINITY;
    int am = 0;
    for (int c = 0; c < C; ++c) {
      logits[(int64_t)r * C + c] = lg[c];
      if (lg[c] > mx) { mx = lg[c]; am = c; }
    }
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += expf(lg[c] - mx);
    const int y = (int)labels[r];
    atomicAdd(stats, logf(se) + mx - lg[y]);
    atomicAdd(stats + 1, am == y ? 1.f : 0.f);
  }
}

// dlogits = (softmax − onehot) · dloss / R; dW2 += dlogitsᵀ·t, db2 += Σ dlogits; dpre = (dlogits·W2) · keep · act'(pre)
__global__ __launch_bounds__(64) void cls32_bwd_kernel(const float* __restrict__ pre, const float* __restrict__ t_in,
                                                       const float* __restrict__ W2, const float* __restrict__ logits,
                                                       const int64_t* __restrict__ labels,
                                                       const float* __restrict__ dloss, float* __restrict__ dpre,
                                                       float* __restrict__ dW2, float* __restrict__ db2, int R, int H,
                                                       int C, int act, DropoutParams dp) {
  dp = resolve_seed(dp);
  const int r = blockIdx.x, lane = threadIdx.x;
  float mx = -INFINITY;
  for (int c = 0; c < C; ++c) mx = fmaxf(mx, logits[(int64_t)r * C + c]);
  float se = 0.f;
  for (int c = 0; c < C; ++c) se += expf(logits[(int64_t)r * C + c] - mx);
  const int y = (int)labels[r];
  const float g = dloss[0] / (float)R;
  float dl[8];
  for (int c = 0; c < C; ++c) dl[c] = (expf(logits[(int64_t)r * C + c] - mx) / se - (c == y ? 1.f : 0.f)) * g;
  if (lane < C) atomicAdd(db2 + lane, dl[lane]);
  for (int c0 = lane * 2; c0 < H; c0 += 128) {
    float kf[2] = {1.f, 1.f};
    if (dp.enabled) {
      const uint32_t bits = dropout_bits2((uint32_t)r, (uint32_t)c0 >> 1, dp);
      kf[0] = keep_factor(bits, 0, dp);
      kf[1] = keep_factor(bits, 1, dp);
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int c1 = c0 + e;
      const float t = t_in[(int64_t)r * H + c1];
      float dt = 0.f;
      for (int c = 0; c < C; ++c) {
        atomicAdd(dW2 + (int64_t)c * H + c1, dl[c] * t);
        dt += dl[c] * W2[(int64_t)c * H + c1];
      }
      const float x = pre[(int64_t)r * H + c1];
      float da;
      if (act == 0) {
        const float th = tanhf(x);
        da = 1.f - th * th;
      } else {
        da = x > 0.f ? 1.f : 0.f;
      }
      dpre[(int64_t)r * H + c1] = dt * kf[e] * da;
    }
  }
}

}  // namespace f32k

static int ew_blocks(int64_t n) { return (int)std::min<int64_t>(2048, std::max<int64_t>(1, (n + 255) / 256)); }

void launch_split3(const float* x, bf16_t* out, int64_t R, int64_t C, int pat, bool rows, hipStream_t st,
                   bf16_t* out2, int pat2) {
  if (C % 4) abort();
  if (C % 8 == 0)
    hipLaunchKernelGGL(f32k::split3_kernel<8>, dim3(ew_blocks(R * C / 8)), dim3(256), 0, st, x, out, R, C, pat,
                       rows ? 1 : 0, out2, pat2);
  else
    hipLaunchKernelGGL(f32k::split3_kernel<4>, dim3(ew_blocks(R * C / 4)), dim3(256), 0, st, x, out, R, C, pat,
                       rows ? 1 : 0, out2, pat2);
  HSD_CHECK_LAUNCH();
}

void launch_epi32(float* y, const float* bias, const float* aux, float* out, int64_t M, int N, int kind, double p,
                  uint64_t seed, hipStream_t st, bf16_t* hi, bf16_t* lo) {
  if (N % 4 || (hi == nullptr) != (lo == nullptr) || (out == nullptr && (hi == nullptr || kind > 1))) abort();
  hipLaunchKernelGGL(f32k::epi32_kernel, dim3(ew_blocks(M * N / 4)), dim3(256), 0, st, y, bias, aux, out, M, N, kind,
                     make_dropout(kind == 2 ? p : 0.0, seed), hi, lo);
  HSD_CHECK_LAUNCH();
}

void launch_dropout32(const float* x, float* out, int64_t n, int W, double p, uint64_t seed, hipStream_t st,
                      bf16_t* hi, bf16_t* lo) {
  if (n % 4 || W % 4 || W <= 0 || (hi == nullptr) != (lo == nullptr)) abort();
  hipLaunchKernelGGL(f32k::dropout32_kernel, dim3(ew_blocks(n / 4)), dim3(256), 0, st, x, out, n / 4, W,
                     make_dropout(p, seed), hi, lo);
  HSD_CHECK_LAUNCH();
}

void launch_colsum32(const float* x, float* dbias, int M, int N, hipStream_t st) {
  if (N % 4 == 0) {
    const int gx = (N + 255) / 256;
    const int min_rows = 256;
    const int gy = std::max(1, std::min(std::min(1024, 2048 / gx), (M + min_rows - 1) / min_rows));
    const int rpb = (M + gy - 1) / gy;
    hipLaunchKernelGGL(f32k::colsum32_kernel, dim3(gx, (M + rpb - 1) / rpb), dim3(256), 0, st, x, dbias, M, N, rpb);
    HSD_CHECK_LAUNCH();
    return;
  }
  const int gx = (N + 63) / 64;
  const int gy = std::max(1, std::min(1024, 2048 / gx));
  const int rpb = (M + gy - 1) / gy;
  hipLaunchKernelGGL(f32k::colsum32_scalar_kernel, dim3(gx, (M + rpb - 1) / rpb), dim3(256), 0, st, x, dbias, M, N,
                     rpb);
  HSD_CHECK_LAUNCH();
}

void launch_ln32_fwd(const float* x, const float* g, const float* b, float* out, float* mean, float* rstd, int R,
                     int H, float eps, hipStream_t st, bf16_t* hi, bf16_t* lo) {
  if (H % 4 || H > 1024 || (hi == nullptr) != (lo == nullptr)) abort();
  const dim3 grid((R + 3) / 4);
#define LN32F(NJ) \
  hipLaunchKernelGGL(f32k::ln32_fwd_kernel<NJ>, grid, dim3(256), 0, st, x, g, b, out, mean, rstd, R, H, eps, hi, lo)
  if (H <= 256) LN32F(1);
  else if (H <= 512) LN32F(2);
  else LN32F(4);
#undef LN32F
  HSD_CHECK_LAUNCH();
}

void launch_ln32_bwd(const float* dy, const float* x, const float* mean, const float* rstd, const float* g, float* dx,
                     float* dg, float* db, int R, int H, hipStream_t st) {
  if (H % 4 || H > 1024) abort();
  const int rpw = std::max(1, (R + 1023) / 1024);  // <= 256 blocks of 4 waves: <= 256 atomics per column
  const int waves = (R + rpw - 1) / rpw;
  const dim3 grid((waves + 3) / 4);
  if (H <= 256) hipLaunchKernelGGL(f32k::ln32_bwd_kernel<1>, grid, dim3(256), 0, st, dy, x, mean, rstd, g, dx, dg, db, R, H, rpw);
  else if (H <= 512) hipLaunchKernelGGL(f32k::ln32_bwd_kernel<2>, grid, dim3(256), 0, st, dy, x, mean, rstd, g, dx, dg, db, R, H, rpw);
  else hipLaunchKernelGGL(f32k::ln32_bwd_kernel<4>, grid, dim3(256), 0, st, dy, x, mean, rstd, g, dx, dg, db, R, H, rpw);
  HSD_CHECK_LAUNCH();
}

void launch_embed32_gather(const int64_t* ids, const int64_t* pids, const int64_t* tids, const float* word,
                           const float* pos, const float* type, float* x, int R, int H, hipStream_t st) {
  if (H % 4) abort();
  hipLaunchKernelGGL(f32k::embed32_gather_kernel, dim3((R + 3) / 4), dim3(256), 0, st, ids, pids, tids, word, pos,
                     type, x, R, H);
  HSD_CHECK_LAUNCH();
}

void launch_embed32_scatter(const float* dx, const int64_t* ids, const int64_t* pids, const int64_t* tids,
                            float* gword, float* gpos, float* gtype, int R, int H, hipStream_t st) {
  hipLaunchKernelGGL(f32k::embed32_scatter_kernel, dim3((R + 3) / 4), dim3(256), 0, st, dx, ids, pids, tids, gword,
                     gpos, gtype, R, H);
  HSD_CHECK_LAUNCH();
}

static float attn32_sl2() { return f32k::kLog2e32 / sqrtf((float)f32k::AD); }

void launch_attn32_fwd(const float* qkv, const float* mask, float* out, float* lse, int B, int S, int heads, double p,
                       uint64_t seed, hipStream_t st) {
  if (S % 2) abort();
  hipLaunchKernelGGL(f32k::attn32_fwd_kernel, dim3(B * heads, (S + 63) / 64), dim3(64), 0, st, qkv, mask, out, lse, S,
                     heads, attn32_sl2(), make_dropout(p, seed));
  HSD_CHECK_LAUNCH();
}

// delta: fp32 [B·heads·S] workspace
void launch_attn32_bwd(const float* qkv, const float* mask, const float* o, const float* dout, const float* lse,
                       float* dqkv, float* delta, int B, int S, int heads, double p, uint64_t seed, hipStream_t st) {
  if (S % 2) abort();
  const float sl2 = attn32_sl2(), scale = 1.0f / sqrtf((float)f32k::AD);
  const DropoutParams dp = make_dropout(p, seed);
  const int n = B * heads * S;
  hipLaunchKernelGGL(f32k::attn32_delta_kernel, dim3((n + 255) / 256), dim3(256), 0, st, o, dout, delta, B, S, heads);
  const dim3 grid(B * heads, (S + 63) / 64);
  hipLaunchKernelGGL(f32k::attn32_dq_kernel, grid, dim3(64), 0, st, qkv, mask, dout, lse, delta, dqkv, S, heads, sl2,
                     scale, dp);
  hipLaunchKernelGGL(f32k::attn32_dkv_kernel<true>, grid, dim3(64), 0, st, qkv, mask, dout, lse, delta, dqkv, S, heads,
                     sl2, scale, dp);
  hipLaunchKernelGGL(f32k::attn32_dkv_kernel<false>, grid, dim3(64), 0, st, qkv, mask, dout, lse, delta, dqkv, S,
                     heads, sl2, scale, dp);
  HSD_CHECK_LAUNCH();
}

void launch_attn32_delta(const float* o, const float* dout, float* delta, int B, int S, int heads, hipStream_t st) {
  const int n = B * heads * S;
  hipLaunchKernelGGL(f32k::attn32_delta_kernel, dim3((n + 255) / 256), dim3(256), 0, st, o, dout, delta, B, S, heads);
  HSD_CHECK_LAUNCH();
}

void launch_cls32_fwd(const float* pre, const float* W2, const float* b2, const int64_t* labels, float* t_out,
                      float* logits, float* stats, int R, int H, int C, int act, double p, uint64_t seed,
                      hipStream_t st) {
  if (C > 8 || H % 2) abort();
  hipLaunchKernelGGL(f32k::cls32_fwd_kernel, dim3(R), dim3(64), 0, st, pre, W2, b2, labels, t_out, logits, stats, R, H,
                     C, act, make_dropout(p, seed));
  HSD_CHECK_LAUNCH();
}

void launch_cls32_bwd(const float* pre, const float* t_in, const float* W2, const float* logits,
                      const int64_t* labels, const float* dloss, float* dpre, float* dW2, float* db2, int R, int H,
                      int C, int act, double p, uint64_t seed, hipStream_t st) {
  if (C > 8 || H % 2) abort();
  hipLaunchKernelGGL(f32k::cls32_bwd_kernel, dim3(R), dim3(64), 0, st, pre, t_in, W2, logits, labels, dloss, dpre,
                     dW2, db2, R, H, C, act, make_dropout(p, seed));
  HSD_CHECK_LAUNCH();
}

}  // namespace hsd
