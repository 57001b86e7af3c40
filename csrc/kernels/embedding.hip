// Embedding gather + add + LayerNorm + dropout, and its backward.
//
// forward : e = word[id] + pos[pos_id] + type[type_id];  out = dropout(LN(e))   -> saves mean/rstd
// backward: recompute e by re-gathering (cheaper than storing it), LN backward, then
//           word_grad[id] += de      (fp32 atomics, 256-B-contiguous per wave instruction)
//           pos_grad / type_grad     (reduced in registers per block first: each block owns ONE
//                                     position and walks the batch, so the position row gets one
//                                     atomic per block and the type rows are not hammered by
//                                     every token — MI355X_MICROARCH.md 'Global float atomics',
//                                     one-row contention is 14x slower)
//           dgamma / dbeta           (register partials, one atomic per column per block)
#include "common.h"
#include "fp8_common.h"

#include <stdlib.h>

namespace hsd {

template <int NCH>
__device__ __forceinline__ void gather_row(float (&e)[NCH][4], const bf16_t* __restrict__ w, const bf16_t* __restrict__ p,
                                           const bf16_t* __restrict__ t, int64_t wid_, int64_t pid, int64_t tid, int H,
                                           int lane) {
  const int nq = H >> 2;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    int c = lane + 64 * i;
    if (c < nq) {
      u32x2 a = *reinterpret_cast<const u32x2*>(w + wid_ * H + 4 * c);
      u32x2 b = *reinterpret_cast<const u32x2*>(p + pid * H + 4 * c);
      e[i][0] = lo_bf(a.x) + lo_bf(b.x);
      e[i][1] = hi_bf(a.x) + hi_bf(b.x);
      e[i][2] = lo_bf(a.y) + lo_bf(b.y);
      e[i][3] = hi_bf(a.y) + hi_bf(b.y);
      if (t) {
        u32x2 d = *reinterpret_cast<const u32x2*>(t + tid * H + 4 * c);
        e[i][0] += lo_bf(d.x); e[i][1] += hi_bf(d.x); e[i][2] += lo_bf(d.y); e[i][3] += hi_bf(d.y);
      }
    } else {
      e[i][0] = e[i][1] = e[i][2] = e[i][3] = 0.f;
    }
  }
}

template <int NCH>
__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ ids, const int64_t* __restrict__ pos_ids,
                                                        const int64_t* __restrict__ type_ids, const bf16_t* __restrict__ word,
                                                        const bf16_t* __restrict__ pos, const bf16_t* __restrict__ type,
                                                        const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ beta,
                                                        bf16_t* __restrict__ out, float* __restrict__ mean_out,
                                                        float* __restrict__ rstd_out, int rows, int H, float eps,
                                                        DropoutParams dp, Q8Out q8o) {
  dp = resolve_seed(dp);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  // q8o.q: the output's fp8 e4m3 copy for the first encoder layer's fp8 QKV GEMM (delayed scaling, as the LayerNorm
  // forward's q8 path: scale from q8o.amax_in, this pass's max |x| into q8o.amax_track)
  float qs = 0.f, qm = 0.f;
  if (q8o.q != nullptr) {
    qs = fmt_scale(0, *q8o.amax_in);
    if (blockIdx.x == 0 && threadIdx.x == 0) *q8o.sinv = 1.0f / qs;
  }
  if (row >= rows) return;
  const int nq = H >> 2;
  float e[NCH][4];
  gather_row<NCH>(e, word, pos, type, ids[row], pos_ids[row], type ? type_ids[row] : 0, H, lane);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) s += e[i][0] + e[i][1] + e[i][2] + e[i][3];
  const float mean = wave_sum(s) / (float)H;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i)
    if (lane + 64 * i < nq)
#pragma unroll
      for (int k = 0; k < 4; ++k) { float d = e[i][k] - mean; ss += d * d; }
  const float rstd = rsqrtf(wave_sum(ss) / (float)H + eps);
  // dropout: mask row `row`, column pairs 2c and 2c + 1 of chunk c = lane + 64 i: C(2c) = C(2 lane) ^ C(128 i)
  const uint32_t xr = dp.enabled ? dropout_row((uint32_t)row, dp) ^ drop_col(2u * (uint32_t)lane) : 0u;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    int c = lane + 64 * i;
    if (c < nq) {
      size_t off = (size_t)row * H + 4 * c;
      u32x2 gw = *reinterpret_cast<const u32x2*>(gamma + 4 * c);
      u32x2 bw = *reinterpret_cast<const u32x2*>(beta + 4 * c);
      float o[4] = {(e[i][0] - mean) * rstd * lo_bf(gw.x) + lo_bf(bw.x), (e[i][1] - mean) * rstd * hi_bf(gw.x) + hi_bf(bw.x),
                    (e[i][2] - mean) * rstd * lo_bf(gw.y) + lo_bf(bw.y), (e[i][3] - mean) * rstd * hi_bf(gw.y) + hi_bf(bw.y)};
      if (dp.enabled) {
        // dropout is applied to the bf16-rounded LN output (matches the reference op order)
        const uint32_t x = xr ^ drop_col(128u * (uint32_t)i);
        const uint32_t b0 = drop_fin(x), b1 = drop_fin(x ^ drop_col(1));
        o[0] = bf2f(f2bf(o[0])) * keep_factor(b0, 0, dp);
        o[1] = bf2f(f2bf(o[1])) * keep_factor(b0, 1, dp);
        o[2] = bf2f(f2bf(o[2])) * keep_factor(b1, 0, dp);
        o[3] = bf2f(f2bf(o[3])) * keep_factor(b1, 1, dp);
      }
      u32x2 w;
      w.x = pack_bf2(o[0], o[1]);
      w.y = pack_bf2(o[2], o[3]);
      *reinterpret_cast<u32x2*>(out + off) = w;
      if (q8o.q != nullptr) {  // from the stored bf16 values: the same bytes as the standalone quantiser
        const float v0 = lo_bf(w.x), v1 = hi_bf(w.x), v2 = lo_bf(w.y), v3 = hi_bf(w.y);
        qm = fmaxf(qm, fmaxf(fmaxf(fabsf(v0), fabsf(v1)), fmaxf(fabsf(v2), fabsf(v3))));
        *reinterpret_cast<uint32_t*>(q8o.q + off) = cvt4<0>(v0 * qs, v1 * qs, v2 * qs, v3 * qs);
      }
    }
  }
  if (q8o.q != nullptr) wave_amax_track(qm, q8o.amax_track);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// grid: (S positions) x (batch chunks). Block = 4 waves; wave w handles batch rows b = chunk*bpc + w, +4, ...
// Element mapping in the backward is e = lane + 64*i (NE = H/64 elements per lane) so each fp32 atomic
// wave instruction into the word-gradient row is 256 contiguous bytes (full atomic rate,
// MI355X_MICROARCH.md 'Global float atomics' access-shape row).
template <int NE>
__global__ __launch_bounds__(256) void embed_bwd_kernel(const bf16_t* __restrict__ dout, const int64_t* __restrict__ ids,
                                                        const int64_t* __restrict__ pos_ids, const int64_t* __restrict__ type_ids,
                                                        const bf16_t* __restrict__ word, const bf16_t* __restrict__ pos,
                                                        const bf16_t* __restrict__ type, const bf16_t* __restrict__ gamma,
                                                        const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                                                        float* __restrict__ gword, float* __restrict__ gpos,
                                                        float* __restrict__ gtype, float* __restrict__ ggamma,
                                                        float* __restrict__ gbeta, int B, int S, int H, int bpc,
                                                        int pos_is_arange, DropoutParams dp) {
  dp = resolve_seed(dp);
  __shared__ float red[4][4][NE * 64];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int s = blockIdx.x;
  const int b0 = blockIdx.y * bpc;
  const int b1 = min(B, b0 + bpc);
  float gam[NE], acc_g[NE], acc_b[NE], acc_p[NE], acc_t0[NE];
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    const int e = lane + 64 * i;
    acc_g[i] = acc_b[i] = acc_p[i] = acc_t0[i] = 0.f;
    gam[i] = e < H ? bf2f(gamma[e]) : 0.f;
  }
  for (int b = b0 + wid; b < b1; b += 4) {
    const int row = b * S + s;
    const int64_t id = ids[row], pid = pos_ids[row];
    const int64_t tid = type ? type_ids[row] : 0;
    const float mean = mean_in[row], rstd = rstd_in[row];
    // dropout: mask row `row`, element e = lane + 64 i in column pair e / 2: C(e / 2) = C(lane / 2) ^ C(32 i)
    const uint32_t xr = dp.enabled ? dropout_row((uint32_t)row, dp) ^ drop_col((uint32_t)lane >> 1) : 0u;
    float xh[NE], g[NE], d[NE];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = lane + 64 * i;
      if (e < H) {
        float ev = bf2f(word[id * H + e]) + bf2f(pos[pid * H + e]);
        if (type) ev += bf2f(type[tid * H + e]);
        const size_t off = (size_t)row * H + e;
        float dv = bf2f(dout[off]);
        if (dp.enabled) dv *= keep_factor(drop_fin(xr ^ drop_col(32u * (uint32_t)i)), lane & 1, dp);
        d[i] = dv;
        xh[i] = (ev - mean) * rstd;
        g[i] = dv * gam[i];
        s1 += g[i];
        s2 += g[i] * xh[i];
        acc_g[i] += dv * xh[i];
        acc_b[i] += dv;
      } else {
        d[i] = xh[i] = g[i] = 0.f;
      }
    }
    s1 = wave_sum(s1) / (float)H;
    s2 = wave_sum(s2) / (float)H;
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = lane + 64 * i;
      if (e >= H) continue;
      const float de = rstd * (g[i] - s1 - xh[i] * s2);
      atomicAdd(gword + id * H + e, de);
      if (pos_is_arange) acc_p[i] += de;
      else atomicAdd(gpos + pid * H + e, de);
      if (gtype) {
        if (tid == 0) acc_t0[i] += de;
        else atomicAdd(gtype + tid * H + e, de);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NE; ++i) {
    red[wid][0][lane + 64 * i] = acc_g[i];
    red[wid][1][lane + 64 * i] = acc_b[i];
    red[wid][2][lane + 64 * i] = acc_p[i];
    red[wid][3][lane + 64 * i] = acc_t0[i];
  }
  __syncthreads();
  float* dst = wid == 0 ? ggamma : wid == 1 ? gbeta : wid == 2 ? (pos_is_arange ? gpos + (size_t)s * H : nullptr) : gtype;
  if (dst) {
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = lane + 64 * i;
      if (e < H) atomicAdd(dst + e, red[0][wid][e] + red[1][wid][e] + red[2][wid][e] + red[3][wid][e]);
    }
  }
}

// 16-B backward (H % 8 == 0): each lane owns 8 consecutive columns per chunk for the row loads (dout and the
// re-gathered word / position / type rows), the LN backward runs in that
// layout, and the embedding gradient de goes through a wave-private LDS row so the fp32 atomics into the
// word-gradient row are issued in the lane + 64 i layout (256 contiguous bytes per wave instruction — the full
// atomic rate). The scalar kernel above loads 2 B per lane per element.
template <int NC8, int NE>  // NE: atomic-layout elements per lane, H <= 64 * NE
__global__ __launch_bounds__(256, 2) void embed_bwd16_kernel(const bf16_t* __restrict__ dout, const int64_t* __restrict__ ids,
                                                          const int64_t* __restrict__ pos_ids,
                                                          const int64_t* __restrict__ type_ids,
                                                          const bf16_t* __restrict__ word, const bf16_t* __restrict__ pos,
                                                          const bf16_t* __restrict__ type, const bf16_t* __restrict__ gamma,
                                                          const float* __restrict__ mean_in,
                                                          const float* __restrict__ rstd_in, float* __restrict__ gword,
                                                          float* __restrict__ gpos, float* __restrict__ gtype,
                                                          float* __restrict__ ggamma, float* __restrict__ gbeta, int B,
                                                          int S, int H, int bpc, int pos_is_arange, DropoutParams dp) {
  dp = resolve_seed(dp);
  __shared__ __attribute__((aligned(16))) float lds[4][NC8 * 512];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int n8 = H >> 3;
  const int s = blockIdx.x;
  const int b0 = blockIdx.y * bpc;
  const int b1 = min(B, b0 + bpc);
  float* wl = lds[wid];
  float gam[NC8][8], acc_g[NC8][8], acc_b[NC8][8], acc_p[NE], acc_t0[NE];
#pragma unroll
  for (int i = 0; i < NC8; ++i) {
    const int c = lane + 64 * i;
    u32x4 gw = u32x4{0, 0, 0, 0};
    if (c < n8) gw = *reinterpret_cast<const u32x4*>(gamma + 8 * c);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      gam[i][2 * k] = lo_bf(gw[k]);
      gam[i][2 * k + 1] = hi_bf(gw[k]);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc_g[i][k] = acc_b[i][k] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < NE; ++i) acc_p[i] = acc_t0[i] = 0.f;

  struct Row {
    u32x4 d[NC8], w[NC8], p[NC8], t[NC8];
    int64_t id, pid, tid;
    float mean, rstd;
  };
  auto load = [&](int b, Row& r) {
    const int row = b * S + s;
    r.id = ids[row];
    r.pid = pos_ids[row];
    r.tid = type ? type_ids[row] : 0;
    r.mean = mean_in[row];
    r.rstd = rstd_in[row];
#pragma unroll
    for (int i = 0; i < NC8; ++i) {
      const int c = lane + 64 * i;
      r.d[i] = r.w[i] = r.p[i] = r.t[i] = u32x4{0, 0, 0, 0};
      if (c < n8) {
        r.d[i] = *reinterpret_cast<const u32x4*>(dout + (size_t)row * H + 8 * c);
        r.w[i] = *reinterpret_cast<const u32x4*>(word + r.id * H + 8 * c);
        r.p[i] = *reinterpret_cast<const u32x4*>(pos + r.pid * H + 8 * c);
        if (type) r.t[i] = *reinterpret_cast<const u32x4*>(type + r.tid * H + 8 * c);
      }
    }
  };
  auto process = [&](int b, const Row& r) {
    const int row = b * S + s;
    // dropout: mask row `row`, pairs 4c + k of chunk c = lane + 64 i: C(4c + k) = C(4 lane) ^ C(256 i) ^ C(k)
    const uint32_t xr = dp.enabled ? dropout_row((uint32_t)row, dp) ^ drop_col(4u * (uint32_t)lane) : 0u;
    float xh[NC8][8], g[NC8][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NC8; ++i) {
      const int c = lane + 64 * i;
      const bool ok = c < n8;
      const size_t off0 = (size_t)row * H + 8 * c;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint32_t bits = 0;
        if (dp.enabled) bits = drop_fin(xr ^ drop_col(256u * (uint32_t)i) ^ drop_col((uint32_t)k));
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e = 2 * k + h;
          const float ev = (h ? hi_bf(r.w[i][k]) + hi_bf(r.p[i][k]) + hi_bf(r.t[i][k])
                              : lo_bf(r.w[i][k]) + lo_bf(r.p[i][k]) + lo_bf(r.t[i][k]));
          float dv = h ? hi_bf(r.d[i][k]) : lo_bf(r.d[i][k]);
          if (dp.enabled) dv *= keep_factor(bits, h, dp);
          xh[i][e] = ok ? (ev - r.mean) * r.rstd : 0.f;
          g[i][e] = dv * gam[i][e];
          s1 += g[i][e];
          s2 += g[i][e] * xh[i][e];
          acc_g[i][e] += dv * xh[i][e];
          acc_b[i][e] += dv;
        }
      }
    }
    s1 = wave_sum(s1) / (float)H;
    s2 = wave_sum(s2) / (float)H;
#pragma unroll
    for (int i = 0; i < NC8; ++i) {
      const int c = lane + 64 * i;
      if (c < n8) {
        f32x4 lo, hi;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          lo[e] = r.rstd * (g[i][e] - s1 - xh[i][e] * s2);
          hi[e] = r.rstd * (g[i][4 + e] - s1 - xh[i][4 + e] * s2);
        }
        *reinterpret_cast<f32x4*>(wl + 8 * c) = lo;
        *reinterpret_cast<f32x4*>(wl + 8 * c + 4) = hi;
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = lane + 64 * i;
      if (e < H) {
        const float de = wl[e];
        atomicAdd(gword + r.id * H + e, de);
        if (pos_is_arange) acc_p[i] += de;
        else atomicAdd(gpos + r.pid * H + e, de);
        if (gtype) {
          if (r.tid == 0) acc_t0[i] += de;
          else atomicAdd(gtype + r.tid * H + e, de);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  };
  for (int b = b0 + wid; b < b1; b += 4) {
    Row r;
    load(b, r);
    process(b, r);
  }
  // block reduction of the four column partials through the (now free) LDS rows; one atomic per column
#pragma unroll
  for (int which = 0; which < 4; ++which) {
    __syncthreads();
    if (which < 2) {
#pragma unroll
      for (int i = 0; i < NC8; ++i) {
        const int c = lane + 64 * i;
        if (c < n8) {
#pragma unroll
          for (int e = 0; e < 8; ++e) wl[8 * c + e] = which == 0 ? acc_g[i][e] : acc_b[i][e];
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const int e = lane + 64 * i;
        if (e < H) wl[e] = which == 2 ? acc_p[i] : acc_t0[i];
      }
    }
    __syncthreads();
    float* dst = which == 0 ? ggamma : which == 1 ? gbeta : which == 2 ? (pos_is_arange ? gpos + (size_t)s * H : nullptr)
                                                                          : gtype;
    if (dst) {
      for (int c = threadIdx.x; c < H; c += 256) atomicAdd(dst + c, lds[0][c] + lds[1][c] + lds[2][c] + lds[3][c]);
    }
  }
}

template <int NCH>
static void embed_fwd_t(const int64_t* ids, const int64_t* pos_ids, const int64_t* type_ids, const bf16_t* word,
                        const bf16_t* pos, const bf16_t* type, const bf16_t* gamma, const bf16_t* beta, bf16_t* out,
                        float* mean, float* rstd, int rows, int H, float eps, const DropoutParams& dp, hipStream_t st,
                        const Q8Out& q8o) {
  hipLaunchKernelGGL((embed_fwd_kernel<NCH>), dim3((rows + 3) / 4), dim3(256), 0, st, ids, pos_ids, type_ids, word, pos,
                     type, gamma, beta, out, mean, rstd, rows, H, eps, dp, q8o);
}

void launch_embed_fwd(const int64_t* ids, const int64_t* pos_ids, const int64_t* type_ids, const bf16_t* word,
                      const bf16_t* pos, const bf16_t* type, const bf16_t* gamma, const bf16_t* beta, bf16_t* out,
                      float* mean, float* rstd, int rows, int H, float eps, double p, uint64_t seed, hipStream_t st,
                      uint8_t* q8, const float* amax_in, float* sinv, float* amax_track) {
  DropoutParams dp = make_dropout(p, seed);
  const Q8Out q8o{q8, amax_in, sinv, amax_track};
  int nch = (H / 4 + 63) / 64;
  if (nch <= 1) embed_fwd_t<1>(ids, pos_ids, type_ids, word, pos, type, gamma, beta, out, mean, rstd, rows, H, eps, dp, st, q8o);
  else if (nch <= 2) embed_fwd_t<2>(ids, pos_ids, type_ids, word, pos, type, gamma, beta, out, mean, rstd, rows, H, eps, dp, st, q8o);
  else if (nch <= 3) embed_fwd_t<3>(ids, pos_ids, type_ids, word, pos, type, gamma, beta, out, mean, rstd, rows, H, eps, dp, st, q8o);
  else if (nch <= 4) embed_fwd_t<4>(ids, pos_ids, type_ids, word, pos, type, gamma, beta, out, mean, rstd, rows, H, eps, dp, st, q8o);
  else abort();
  HSD_CHECK_LAUNCH();
}

template <int NE>
static void embed_bwd_t(const bf16_t* dout, const int64_t* ids, const int64_t* pos_ids, const int64_t* type_ids,
                        const bf16_t* word, const bf16_t* pos, const bf16_t* type, const bf16_t* gamma,
                        const float* mean, const float* rstd, float* gword, float* gpos, float* gtype, float* ggamma,
                        float* gbeta, int B, int S, int H, int pos_is_arange, const DropoutParams& dp, hipStream_t st) {
  // enough blocks to fill 256 CUs: S * chunks >= ~2048
  int chunks = max(1, min(B, (2048 + S - 1) / S));
  int bpc = (B + chunks - 1) / chunks;
  chunks = (B + bpc - 1) / bpc;
  hipLaunchKernelGGL((embed_bwd_kernel<NE>), dim3(S, chunks), dim3(256), 0, st, dout, ids, pos_ids, type_ids, word,
                     pos, type, gamma, mean, rstd, gword, gpos, gtype, ggamma, gbeta, B, S, H, bpc, pos_is_arange, dp);
}

void launch_embed_bwd(const bf16_t* dout, const int64_t* ids, const int64_t* pos_ids, const int64_t* type_ids,
                      const bf16_t* word, const bf16_t* pos, const bf16_t* type, const bf16_t* gamma,
                      const float* mean, const float* rstd, float* gword, float* gpos, float* gtype, float* ggamma,
                      float* gbeta, int B, int S, int H, int pos_is_arange, double p, uint64_t seed, hipStream_t st) {
  DropoutParams dp = make_dropout(p, seed);
  if (H % 8 == 0 && H <= 1024) {  // 16-B kernel (957 -> 414 us vs the round-1 scalar one, kept for other H)
    // ~512 blocks (at least one per position): every block ends with 3-4 x H column atomics
    // (gamma / beta / position / type partials) on the same H addresses, so fewer, longer blocks win: 512 measured
    // best or within 3 % of best at all four shapes of tools/embed_bwd_probe.py (2048 before: bert-large B = 8
    // 81 -> 35 us, bert-base B = 32 120 -> 34 us, B = 1024 421 -> 393 us; profiles/embed_bwd_blocks_r5.log)
    const int target = 512;
    int chunks = max(1, min(B, (target + S - 1) / S));
    int bpc = (B + chunks - 1) / chunks;
    chunks = (B + bpc - 1) / bpc;
#define HSD_EB16(NC8, NE)                                                                                      \
  hipLaunchKernelGGL((embed_bwd16_kernel<NC8, NE>), dim3(S, chunks), dim3(256), 0, st, dout, ids, pos_ids, type_ids, \
                     word, pos, type, gamma, mean, rstd, gword, gpos, gtype, ggamma, gbeta, B, S, H, bpc,             \
                     pos_is_arange, dp)
    if (H <= 512) HSD_EB16(1, 8);
    else if (H <= 768) HSD_EB16(2, 12);
    else HSD_EB16(2, 16);
#undef HSD_EB16
    HSD_CHECK_LAUNCH();
    return;
  }
  const int ne = (H + 63) / 64;
  if (ne <= 1) embed_bwd_t<1>(dout, ids, pos_ids, type_ids, word, pos, type, gamma, mean, rstd, gword, gpos, gtype, ggamma, gbeta, B, S, H, pos_is_arange, dp, st);
  else if (ne <= 2) embed_bwd_t<2>(dout, ids, pos_ids, type_ids, word, pos, type, gamma, mean, rstd, gword, gpos, gtype, ggamma, gbeta, B, S, H, pos_is_arange, dp, st);
  else if (ne <= 12) embed_bwd_t<12>(dout, ids, pos_ids, type_ids, word, pos, type, gamma, mean, rstd, gword, gpos, gtype, ggamma, gbeta, B, S, H, pos_is_arange, dp, st);
  else if (ne <= 16) embed_bwd_t<16>(dout, ids, pos_ids, type_ids, word, pos, type, gamma, mean, rstd, gword, gpos, gtype, ggamma, gbeta, B, S, H, pos_is_arange, dp, st);
  else abort();
  HSD_CHECK_LAUNCH();
}

}  // namespace hsd
