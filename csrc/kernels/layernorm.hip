// LayerNorm with the BERT post-LN block tail fused in.
//
// forward : z = dropout(y) + residual   (y = GEMM output incl. bias)
//           out = (z - mean) * rstd * gamma + beta       (fp32 statistics, eps 1e-12 / 1e-5)
//           saves z (bf16) + mean/rstd (fp32) for backward
// backward: dz   = rstd * (g - mean(g) - xhat * mean(g * xhat)),   g = dout * gamma
//           dy   = dz * keep * scale          (gradient into the GEMM output, dropout regenerated)
//           dgamma += Σ dout * xhat ; dbeta += Σ dout ; dbias += Σ dy   (fp32 atomics into main_grad,
//           after a per-block register/LDS reduction — one atomic per column per block)
//
// One wave64 per row; each lane owns columns {4·(lane + 64·i)} (8-byte vector IO), so column
// partial sums for the weight/bias gradients accumulate in registers across the rows a block
// walks, with no atomics until the block ends.
#include "common.h"
#include "ln_common.h"
#include "fp8_common.h"
#include <stdlib.h>
#include <algorithm>

namespace hsd {

constexpr int kLnWaves = 4;

template <int NCH>  // 4-element chunks per lane: ceil(H / 256)
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16_t* __restrict__ y, const bf16_t* __restrict__ res,
                                                     const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ beta,
                                                     bf16_t* __restrict__ z_out, bf16_t* __restrict__ out,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int rows, int H, float eps, DropoutParams dp) {
  dp = resolve_seed(dp);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kLnWaves + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nq = H >> 2;  // 4-element chunks in the row
  // dropout: mask row `row`, pairs 2c and 2c + 1 of chunk c = lane + 64 i: C(2c) = C(2 lane) ^ C(128 i)
  const uint32_t xr = dp.enabled ? dropout_row((uint32_t)row, dp) ^ drop_col(2u * (uint32_t)lane) : 0u;
  float v[NCH][4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    int c = lane + 64 * i;
    if (c < nq) {
      size_t off = (size_t)row * H + 4 * c;
      u32x2 w = *reinterpret_cast<const u32x2*>(y + off);
      float a[4] = {lo_bf(w.x), hi_bf(w.x), lo_bf(w.y), hi_bf(w.y)};
      if (dp.enabled) {
        const uint32_t x = xr ^ drop_col(128u * (uint32_t)i);
        const uint32_t b0 = drop_fin(x), b1 = drop_fin(x ^ drop_col(1));
        a[0] *= keep_factor(b0, 0, dp);
        a[1] *= keep_factor(b0, 1, dp);
        a[2] *= keep_factor(b1, 0, dp);
        a[3] *= keep_factor(b1, 1, dp);
      }
      if (res) {
        u32x2 r = *reinterpret_cast<const u32x2*>(res + off);
        a[0] += lo_bf(r.x); a[1] += hi_bf(r.x); a[2] += lo_bf(r.y); a[3] += hi_bf(r.y);
      }
      // round z to bf16 now: backward recomputes xhat from the stored bf16 z
      u32x2 zw;
      zw.x = pack_bf2(a[0], a[1]);
      zw.y = pack_bf2(a[2], a[3]);
      if (z_out) *reinterpret_cast<u32x2*>(z_out + off) = zw;
      v[i][0] = lo_bf(zw.x); v[i][1] = hi_bf(zw.x); v[i][2] = lo_bf(zw.y); v[i][3] = hi_bf(zw.y);
      s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
    } else {
      v[i][0] = v[i][1] = v[i][2] = v[i][3] = 0.f;
    }
  }
  const float mean = wave_sum(s) / (float)H;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    int c = lane + 64 * i;
    if (c < nq) {
#pragma unroll
      for (int k = 0; k < 4; ++k) { float d = v[i][k] - mean; ss += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(ss) / (float)H + eps);
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    int c = lane + 64 * i;
    if (c < nq) {
      size_t off = (size_t)row * H + 4 * c;
      u32x2 gw = *reinterpret_cast<const u32x2*>(gamma + 4 * c);
      u32x2 bw = *reinterpret_cast<const u32x2*>(beta + 4 * c);
      float g[4] = {lo_bf(gw.x), hi_bf(gw.x), lo_bf(gw.y), hi_bf(gw.y)};
      float b[4] = {lo_bf(bw.x), hi_bf(bw.x), lo_bf(bw.y), hi_bf(bw.y)};
      u32x2 o;
      o.x = pack_bf2((v[i][0] - mean) * rstd * g[0] + b[0], (v[i][1] - mean) * rstd * g[1] + b[1]);
      o.y = pack_bf2((v[i][2] - mean) * rstd * g[2] + b[2], (v[i][3] - mean) * rstd * g[3] + b[3]);
      *reinterpret_cast<u32x2*>(out + off) = o;
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Plain LayerNorm forward for the encoder's LN tails (z = dropout(y) + residual already comes out of the GEMM
// epilogue, so no residual / dropout / z here): every wave walks `rpw` consecutive rows with the NEXT row's
// 16-B loads in flight while the current row reduces. 5.1 TB/s at T = 131072, H = 768 against 3.6 TB/s for the
// one-row-per-wave kernel above with its 8-B lanes (tools/bench_ln.py, profiles/bench_ln_r2.json). Needs
// H % 8 == 0. Q8: also the output's fp8 copy (launch_ln_fwd_q8).
template <int NC8, bool Q8>
__global__ __launch_bounds__(256) void ln_fwd_plain16_kernel(const bf16_t* __restrict__ y,
                                                             const bf16_t* __restrict__ gamma,
                                                             const bf16_t* __restrict__ beta, bf16_t* __restrict__ out,
                                                             float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                             int rows, int H, int rpw, float eps, Q8Out q8o) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r0 = (blockIdx.x * kLnWaves + wave) * rpw;
  const int r1 = min(rows, r0 + rpw);
  // fp8 copy of the output (Q8: e4m3, delayed scaling from q8o.amax_in; this pass's amax into q8o.amax_track)
  float qs = 0.f, qm = 0.f;
  if constexpr (Q8) {
    qs = fmt_scale(0, *q8o.amax_in);
    if (blockIdx.x == 0 && threadIdx.x == 0) *q8o.sinv = 1.0f / qs;
  }
  if (r0 >= r1) return;
  u32x4 gw[NC8], bw[NC8];
  ln_params16<NC8>(gamma, beta, H, lane, gw, bw);
  auto process = [&](int row, const u32x4(&yw)[NC8]) {
    ln_row16<NC8, Q8>(yw, gw, bw, row, H, lane, eps, out, mean_out, rstd_out, q8o.q, qs, &qm);
  };
  u32x4 ya[NC8], yb[NC8];
  ln_load16<NC8>(y, r0, H, lane, ya);
  for (int r = r0; r < r1; r += 2) {
    const bool more = r + 1 < r1;
    if (more) ln_load16<NC8>(y, r + 1, H, lane, yb);
    process(r, ya);
    if (!more) break;
    if (r + 2 < r1) ln_load16<NC8>(y, r + 2, H, lane, ya);
    process(r + 1, yb);
  }
  if constexpr (Q8) wave_amax_track(qm, q8o.amax_track);
}

// Block = 4 waves; block walks `rows_per_block` rows (wave-strided, TWO rows in flight per wave so the
// second row's loads overlap the first row's reductions) accumulating column partials in registers.
template <int NCH>
__device__ __forceinline__ void ln_bwd_load(const bf16_t* __restrict__ dout, const bf16_t* __restrict__ z, int row,
                                            int H, int lane, u32x2 (&zw)[NCH], u32x2 (&dw)[NCH]) {
  const int nq = H >> 2;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + 64 * i;
    if (c < nq) {
      const size_t off = (size_t)row * H + 4 * c;
      zw[i] = *reinterpret_cast<const u32x2*>(z + off);
      dw[i] = *reinterpret_cast<const u32x2*>(dout + off);
    } else {
      zw[i] = u32x2{0, 0};
      dw[i] = u32x2{0, 0};
    }
  }
}

// QF >= 0: also dy's fp8 copy (QF = format) into q8 with scale qs, max |dy| into qm
template <int NCH, int QF = -1>
__device__ __forceinline__ void ln_bwd_row(const u32x2 (&zw)[NCH], const u32x2 (&dw)[NCH], float mean, float rstd,
                                           const float (&gam)[NCH][4], int row, int H, int lane,
                                           bf16_t* __restrict__ dz_out, bf16_t* __restrict__ dy_out,
                                           const bf16_t* __restrict__ dres_add, const DropoutParams& dp,
                                           float (&acc_g)[NCH][4], float (&acc_b)[NCH][4], float (&acc_db)[NCH][4],
                                           uint8_t* __restrict__ q8 = nullptr, float qs = 0.f, float* qm = nullptr,
                                           bool q8only = false) {
  const int nq = H >> 2;
  float xh[NCH][4], g[NCH][4];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const float zz[4] = {lo_bf(zw[i].x), hi_bf(zw[i].x), lo_bf(zw[i].y), hi_bf(zw[i].y)};
    const float d[4] = {lo_bf(dw[i].x), hi_bf(dw[i].x), lo_bf(dw[i].y), hi_bf(dw[i].y)};
    const bool ok = lane + 64 * i < nq;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      xh[i][k] = ok ? (zz[k] - mean) * rstd : 0.f;
      g[i][k] = d[k] * gam[i][k];
      s1 += g[i][k];
      s2 += g[i][k] * xh[i][k];
      acc_g[i][k] += d[k] * xh[i][k];
      acc_b[i][k] += d[k];
    }
  }
  s1 = wave_sum(s1) / (float)H;
  s2 = wave_sum(s2) / (float)H;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + 64 * i;
    if (c >= nq) continue;
    const size_t off = (size_t)row * H + 4 * c;
    float dz[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) dz[k] = rstd * (g[i][k] - s1 - xh[i][k] * s2);
    if (dres_add) {
      u32x2 r = *reinterpret_cast<const u32x2*>(dres_add + off);
      dz[0] += lo_bf(r.x); dz[1] += hi_bf(r.x); dz[2] += lo_bf(r.y); dz[3] += hi_bf(r.y);
    }
    u32x2 o;
    o.x = pack_bf2(dz[0], dz[1]);
    o.y = pack_bf2(dz[2], dz[3]);
    if (dz_out) *reinterpret_cast<u32x2*>(dz_out + off) = o;
    if (dy_out) {
      float dy[4] = {dz[0], dz[1], dz[2], dz[3]};
      if (dp.enabled) {
        // mask row `row`, pairs 2c and 2c + 1: C(2c) = C(2 lane) ^ C(128 i) (C(2 lane) is loop-invariant: hoisted)
        const uint32_t x = dropout_row((uint32_t)row, dp) ^ drop_col(2u * (uint32_t)lane) ^ drop_col(128u * (uint32_t)i);
        const uint32_t b0 = drop_fin(x), b1 = drop_fin(x ^ drop_col(1));
        dy[0] *= keep_factor(b0, 0, dp);
        dy[1] *= keep_factor(b0, 1, dp);
        dy[2] *= keep_factor(b1, 0, dp);
        dy[3] *= keep_factor(b1, 1, dp);
      }
      u32x2 yo;
      yo.x = pack_bf2(dy[0], dy[1]);
      yo.y = pack_bf2(dy[2], dy[3]);
      if (!(QF >= 0 && q8only)) *reinterpret_cast<u32x2*>(dy_out + off) = yo;
      // bias grad sums the bf16-rounded dy that the dgrad GEMM consumes
      acc_db[i][0] += lo_bf(yo.x); acc_db[i][1] += hi_bf(yo.x);
      acc_db[i][2] += lo_bf(yo.y); acc_db[i][3] += hi_bf(yo.y);
      if constexpr (QF >= 0) {
        const float a0 = lo_bf(yo.x), a1 = hi_bf(yo.x), a2 = lo_bf(yo.y), a3 = hi_bf(yo.y);
        *qm = fmaxf(*qm, fmaxf(fmaxf(fabsf(a0), fabsf(a1)), fmaxf(fabsf(a2), fabsf(a3))));
        *reinterpret_cast<uint32_t*>(q8 + off) = cvt4<QF>(a0 * qs, a1 * qs, a2 * qs, a3 * qs);
      }
    }
  }
}

// Single pass: every wave walks `rpw` consecutive rows (next row's loads in flight while the current
// row reduces), keeps dgamma / dbeta / dbias column partials in registers, and the block reduces its 4
// waves' partials through LDS into one fp32 atomic per column per block. Reads dout, z once; writes
// dz, dy once (the round-1 split rows + columns passes read dout / z twice: 170 -> ~120 us at the headline shape).
template <int NCH, int QF>
__global__ __launch_bounds__(256) void ln_bwd_fused_kernel(const bf16_t* __restrict__ dout,
                                                           const bf16_t* __restrict__ z,
                                                           const float* __restrict__ mean_in,
                                                           const float* __restrict__ rstd_in,
                                                           const bf16_t* __restrict__ gamma, bf16_t* __restrict__ dz_out,
                                                           bf16_t* __restrict__ dy_out,
                                                           const bf16_t* __restrict__ dres_add,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                           float* __restrict__ dbias, int rows, int H, int rpw,
                                                           DropoutParams dp, Q8Out q8o) {
  dp = resolve_seed(dp);
  float qs = 0.f, qm = 0.f;
  bool q8only = false;  // dy's bf16 values skipped: its consumers all take the fp8 copy (ops/hip.py _ln_bwd)
  if constexpr (QF >= 0) {
    qs = fmt_scale(QF, *q8o.amax_in);
    q8only = q8o.only != 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) *q8o.sinv = 1.0f / qs;
  }
  __shared__ float red[kLnWaves][3][NCH * 256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nq = H >> 2;
  const int r0 = (blockIdx.x * kLnWaves + wave) * rpw;
  const int r1 = min(rows, r0 + rpw);
  float gam[NCH][4], ag[NCH][4], ab[NCH][4], ad[NCH][4];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + 64 * i;
#pragma unroll
    for (int k = 0; k < 4; ++k) gam[i][k] = ag[i][k] = ab[i][k] = ad[i][k] = 0.f;
    if (c < nq) {
      const u32x2 gw = *reinterpret_cast<const u32x2*>(gamma + 4 * c);
      gam[i][0] = lo_bf(gw.x); gam[i][1] = hi_bf(gw.x); gam[i][2] = lo_bf(gw.y); gam[i][3] = hi_bf(gw.y);
    }
  }
  if (r0 < r1) {
    u32x2 za[NCH], da[NCH], zb[NCH], db[NCH];
    ln_bwd_load<NCH>(dout, z, r0, H, lane, za, da);
    float mu = mean_in[r0], rs = rstd_in[r0];
    for (int r = r0; r < r1; r += 2) {
      const bool more = r + 1 < r1;
      float mu2 = 0.f, rs2 = 0.f;
      if (more) {
        ln_bwd_load<NCH>(dout, z, r + 1, H, lane, zb, db);
        mu2 = mean_in[r + 1];
        rs2 = rstd_in[r + 1];
      }
      ln_bwd_row<NCH, QF>(za, da, mu, rs, gam, r, H, lane, dz_out, dy_out, dres_add, dp, ag, ab, ad, q8o.q, qs, &qm,
                          q8only);
      if (!more) break;
      const bool more2 = r + 2 < r1;
      if (more2) {
        ln_bwd_load<NCH>(dout, z, r + 2, H, lane, za, da);
        mu = mean_in[r + 2];
        rs = rstd_in[r + 2];
      }
      ln_bwd_row<NCH, QF>(zb, db, mu2, rs2, gam, r + 1, H, lane, dz_out, dy_out, dres_add, dp, ag, ab, ad, q8o.q, qs,
                          &qm, q8only);
    }
  }
  if constexpr (QF >= 0) wave_amax_track(qm, q8o.amax_track);
#pragma unroll
  for (int i = 0; i < NCH; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int col = 4 * (lane + 64 * i) + k;
      red[wave][0][col] = ag[i][k];
      red[wave][1][col] = ab[i][k];
      red[wave][2][col] = ad[i][k];
    }
  __syncthreads();
  for (int c = threadIdx.x; c < H; c += 256) {
    atomicAdd(dgamma + c, red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c]);
    atomicAdd(dbeta + c, red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c]);
    if (dbias && dy_out) atomicAdd(dbias + c, red[0][2][c] + red[1][2][c] + red[2][2][c] + red[3][2][c]);
  }
}

template <int NCH>
static void ln_fwd_t(const bf16_t* y, const bf16_t* res, const bf16_t* gamma, const bf16_t* beta, bf16_t* z,
                     bf16_t* out, float* mean, float* rstd, int rows, int H, float eps, const DropoutParams& dp,
                     hipStream_t st) {
  if (res == nullptr && z == nullptr && !dp.enabled && H % 8 == 0 && H <= 1024) {
    // 2 rows per wave (the next row's loads in flight while one reduces): best at the HBM-bound headline shape
    // (131072 x 768: 75 us vs 81 us at 16 rows per wave); every setting is equal once the tensors fit the MALL
    // (tools/bench_ln_rpw.py, profiles/bench_ln_rpw_r2.jsonl)
    const int rpw = 2;
    const int waves = (rows + rpw - 1) / rpw;
    const int blocks = (waves + kLnWaves - 1) / kLnWaves;
    if (H <= 512)
      hipLaunchKernelGGL((ln_fwd_plain16_kernel<1, false>), dim3(blocks), dim3(256), 0, st, y, gamma, beta, out, mean,
                         rstd, rows, H, rpw, eps, Q8Out{});
    else
      hipLaunchKernelGGL((ln_fwd_plain16_kernel<2, false>), dim3(blocks), dim3(256), 0, st, y, gamma, beta, out, mean,
                         rstd, rows, H, rpw, eps, Q8Out{});
    return;
  }
  dim3 grid((rows + kLnWaves - 1) / kLnWaves);
  hipLaunchKernelGGL((ln_fwd_kernel<NCH>), grid, dim3(256), 0, st, y, res, gamma, beta, z, out, mean, rstd, rows,
                     H, eps, dp);
}

void launch_ln_fwd(const bf16_t* y, const bf16_t* res, const bf16_t* gamma, const bf16_t* beta, bf16_t* z,
                   bf16_t* out, float* mean, float* rstd, int rows, int H, float eps, double p, uint64_t seed,
                   hipStream_t st) {
  DropoutParams dp = make_dropout(p, seed);
  int nch = (H / 4 + 63) / 64;
  if (nch <= 1) ln_fwd_t<1>(y, res, gamma, beta, z, out, mean, rstd, rows, H, eps, dp, st);
  else if (nch <= 2) ln_fwd_t<2>(y, res, gamma, beta, z, out, mean, rstd, rows, H, eps, dp, st);
  else if (nch <= 3) ln_fwd_t<3>(y, res, gamma, beta, z, out, mean, rstd, rows, H, eps, dp, st);
  else if (nch <= 4) ln_fwd_t<4>(y, res, gamma, beta, z, out, mean, rstd, rows, H, eps, dp, st);
  else if (nch <= 8) ln_fwd_t<8>(y, res, gamma, beta, z, out, mean, rstd, rows, H, eps, dp, st);
  else abort();
  HSD_CHECK_LAUNCH();
}

template <int NCH>
static void ln_bwd_t(const bf16_t* dout, const bf16_t* z, const float* mean, const float* rstd, const bf16_t* gamma,
                     bf16_t* dz, bf16_t* dy, const bf16_t* dres_add, float* dgamma, float* dbeta, float* dbias,
                     int rows, int H, const DropoutParams& dp, hipStream_t st, const Q8Out& q8o = Q8Out{},
                     int qfmt = -1) {
  // ~16 rows per wave at the headline's 131072 rows: 2048 waves = 8 per CU, a few thousand column atomics per
  // block; at least 4 rows per wave (a floor of 2 for small row counts, twice the waves and the column atomics,
  // measured 1-2 % slower end to end at bert-large B = 8 and bert-base B = 32: profiles/small_tiles_r2.log; other
  // floors: profiles/ln_bwd_rpw_r5.log)
  const int min_rpw = 4;
  const int rpw = std::max(min_rpw, (rows + 2047) / 2048);
  const int waves = (rows + rpw - 1) / rpw;
  const int blocks = (waves + kLnWaves - 1) / kLnWaves;
  // dbias sums the gradient that enters the GEMM: dy (or dz, which equals dy when there is no dropout)
  bf16_t* ysink = dy ? dy : nullptr;
  if (qfmt == 0)
    hipLaunchKernelGGL((ln_bwd_fused_kernel<NCH, 0>), dim3(blocks), dim3(256), 0, st, dout, z, mean, rstd, gamma, dz,
                       ysink, dres_add, dgamma, dbeta, dbias, rows, H, rpw, dp, q8o);
  else if (qfmt == 1)
    hipLaunchKernelGGL((ln_bwd_fused_kernel<NCH, 1>), dim3(blocks), dim3(256), 0, st, dout, z, mean, rstd, gamma, dz,
                       ysink, dres_add, dgamma, dbeta, dbias, rows, H, rpw, dp, q8o);
  else
    hipLaunchKernelGGL((ln_bwd_fused_kernel<NCH, -1>), dim3(blocks), dim3(256), 0, st, dout, z, mean, rstd, gamma, dz,
                       ysink, dres_add, dgamma, dbeta, dbias, rows, H, rpw, dp, q8o);
}

// LayerNorm forward (no residual / dropout) that also writes the output's fp8 e4m3 copy for the next fp8 GEMM
// (ops/hip.py: the LN at the end of a block quantises for the next block's first GEMM), H % 8 == 0, H <= 1024.
void launch_ln_fwd_q8(const bf16_t* y, const bf16_t* gamma, const bf16_t* beta, bf16_t* out, float* mean, float* rstd,
                      int rows, int H, float eps, uint8_t* q8, const float* amax_in, float* sinv, float* amax_track,
                      hipStream_t st) {
  const int rpw = 2;
  const int waves = (rows + rpw - 1) / rpw;
  const int blocks = (waves + kLnWaves - 1) / kLnWaves;
  const Q8Out q{q8, amax_in, sinv, amax_track};
  if (H <= 512)
    hipLaunchKernelGGL((ln_fwd_plain16_kernel<1, true>), dim3(blocks), dim3(256), 0, st, y, gamma, beta, out, mean,
                       rstd, rows, H, rpw, eps, q);
  else
    hipLaunchKernelGGL((ln_fwd_plain16_kernel<2, true>), dim3(blocks), dim3(256), 0, st, y, gamma, beta, out, mean,
                       rstd, rows, H, rpw, eps, q);
  HSD_CHECK_LAUNCH();
}

// LN backward (fused single-pass kernel) that also writes dy's fp8 copy (qfmt 0 = e4m3, 1 = e5m2) for the fp8
// dgrad GEMM that consumes dy; dy must be materialised (dy != nullptr)
void launch_ln_bwd_q8(const bf16_t* dout, const bf16_t* z, const float* mean, const float* rstd, const bf16_t* gamma,
                      bf16_t* dz, bf16_t* dy, const bf16_t* dres_add, float* dgamma, float* dbeta, float* dbias,
                      int rows, int H, double p, uint64_t seed, uint8_t* q8, const float* amax_in, float* sinv,
                      float* amax_track, int qfmt, hipStream_t st, bool q8_only) {
  DropoutParams dp = make_dropout(p, seed);
  // dy's bf16 values may be skipped only when dz is its own buffer (no dropout: dz IS dy, the residual gradient)
  if (q8_only && dz == nullptr) abort();
  const Q8Out q{q8, amax_in, sinv, amax_track, q8_only ? 1 : 0};
  int nch = (H / 4 + 63) / 64;
  if (nch <= 1) ln_bwd_t<1>(dout, z, mean, rstd, gamma, dz, dy, dres_add, dgamma, dbeta, dbias, rows, H, dp, st, q, qfmt);
  else if (nch <= 2) ln_bwd_t<2>(dout, z, mean, rstd, gamma, dz, dy, dres_add, dgamma, dbeta, dbias, rows, H, dp, st, q, qfmt);
  else if (nch <= 3) ln_bwd_t<3>(dout, z, mean, rstd, gamma, dz, dy, dres_add, dgamma, dbeta, dbias, rows, H, dp, st, q, qfmt);
  else if (nch <= 4) ln_bwd_t<4>(dout, z, mean, rstd, gamma, dz, dy, dres_add, dgamma, dbeta, dbias, rows, H, dp, st, q, qfmt);
  else abort();
  HSD_CHECK_LAUNCH();
}

void launch_ln_bwd(const bf16_t* dout, const bf16_t* z, const float* mean, const float* rstd, const bf16_t* gamma,
                   bf16_t* dz, bf16_t* dy, const bf16_t* dres_add, float* dgamma, float* dbeta, float* dbias,
                   int rows, int H, double p, uint64_t seed, hipStream_t st) {
  DropoutParams dp = make_dropout(p, seed);
  int nch = (H / 4 + 63) / 64;
  if (nch <= 1) ln_bwd_t<1>(dout, z, mean, rstd, gamma, dz, dy, dres_add, dgamma, dbeta, dbias, rows, H, dp, st);
  else if (nch <= 2) ln_bwd_t<2>(dout, z, mean, rstd, gamma, dz, dy, dres_add, dgamma, dbeta, dbias, rows, H, dp, st);
  else if (nch <= 3) ln_bwd_t<3>(dout, z, mean, rstd, gamma, dz, dy, dres_add, dgamma, dbeta, dbias, rows, H, dp, st);
  else if (nch <= 4) ln_bwd_t<4>(dout, z, mean, rstd, gamma, dz, dy, dres_add, dgamma, dbeta, dbias, rows, H, dp, st);
  else abort();
  HSD_CHECK_LAUNCH();
}

}  // namespace hsd
