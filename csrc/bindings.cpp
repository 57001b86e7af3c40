// Python bindings for the gfx950 kernels: argument validation + current-HIP-stream launch.
// Compiled into huggingface_sagemaker_tensorflow_distributed_amd/_C.so by _build.py (hipcc).
#include <torch/extension.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include "kernels/launchers.h"

namespace hsd {
void register_comm(pybind11::module& m);
}

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

// ---- host-cheap stream ordering (ops/hip.py weight-gradient side stream, optimizer slices): one event from a
// per-thread ring per fork, no Python stream objects / context managers on the per-layer backward path.
// The events order streams of ONE device, so they skip the system-scope fence (hipEventDisableSystemFence): a default
// event's record made the next kernel on the recording stream wait for a system-scope release, a 6-12 us bubble per
// fork on a busy stream (bert-large B = 8: ~8 forks per layer, tools/timeline.py). HSD_EVENT_SYSFENCE=1: the old events.
static hipEvent_t ring_event() {
  constexpr int kRing = 64;
  thread_local hipEvent_t ring[kRing] = {};
  thread_local int next = 0;
  hipEvent_t& e = ring[next];
  next = (next + 1) % kRing;
  if (e == nullptr) {
    const char* env = getenv("HSD_EVENT_SYSFENCE");
    const unsigned flags = hipEventDisableTiming | ((env && atoi(env)) ? 0u : (unsigned)hipEventDisableSystemFence);
    TORCH_CHECK(hipEventCreateWithFlags(&e, flags) == hipSuccess, "hipEventCreate");
  }
  return e;
}

// dst waits for the work queued on src so far (0 = the current stream)
void stream_wait(int64_t dst_ptr, int64_t src_ptr) {
  hipStream_t dst = dst_ptr ? reinterpret_cast<hipStream_t>(dst_ptr) : cur_stream();
  hipStream_t src = src_ptr ? reinterpret_cast<hipStream_t>(src_ptr) : cur_stream();
  hipEvent_t e = ring_event();
  TORCH_CHECK(hipEventRecord(e, src) == hipSuccess, "hipEventRecord");
  TORCH_CHECK(hipStreamWaitEvent(dst, e, 0) == hipSuccess, "hipStreamWaitEvent");
}

#define CHECK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define CHECK_DTYPE(x, d) TORCH_CHECK((x).scalar_type() == (d), #x " has wrong dtype")
#define BF(x) reinterpret_cast<hsd::bf16_t*>((x).data_ptr())
#define CBF(x) reinterpret_cast<const hsd::bf16_t*>((x).data_ptr())

void adam_step(torch::Tensor p, torch::Tensor m, torch::Tensor v, torch::Tensor g, c10::optional<torch::Tensor> out,
               c10::optional<torch::Tensor> decay, double step, double eps, double b1, double b2, double gscale,
               double lr_wd, c10::optional<torch::Tensor> coef, c10::optional<torch::Tensor> out_lo, bool zero_grad) {
  CHECK_CUDA(p); CHECK_CONTIG(p); CHECK_DTYPE(p, torch::kFloat32);
  TORCH_CHECK(!zero_grad || g.is_contiguous(), "adam zero_grad: contiguous gradient");
  CHECK_DTYPE(m, torch::kFloat32); CHECK_DTYPE(v, torch::kFloat32);
  TORCH_CHECK(p.numel() == m.numel() && p.numel() == v.numel() && p.numel() == g.numel(), "size mismatch");
  TORCH_CHECK(p.numel() % 64 == 0, "flat buffer (or slice) must be a multiple of 64 elements");
  bool gbf = g.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(gbf || g.scalar_type() == torch::kFloat32, "grad must be fp32 or bf16");
  hsd::bf16_t* o = nullptr;
  if (out.has_value()) {
    CHECK_DTYPE(*out, torch::kBFloat16);
    TORCH_CHECK(out->numel() == p.numel(), "out size");
    o = BF(*out);
  }
  const uint8_t* dm = nullptr;
  if (decay.has_value()) {
    TORCH_CHECK(decay->numel() * 64 >= p.numel(), "decay mask too small");
    dm = decay->data_ptr<uint8_t>();
  }
  const float* dcoef = nullptr;  // fp32 [4] on the device: (step, eps, grad_scale, lr*wd) override the scalars
  if (coef.has_value()) {
    CHECK_CUDA(*coef); CHECK_DTYPE(*coef, torch::kFloat32);
    TORCH_CHECK(coef->numel() >= 4, "coef: fp32 [4]");
    dcoef = coef->data_ptr<float>();
  }
  hsd::bf16_t* lo = nullptr;  // fp32 compute: `out` / `out_lo` = the bf16 hi / lo halves of the updated weights
  if (out_lo.has_value()) {
    CHECK_DTYPE(*out_lo, torch::kBFloat16);
    TORCH_CHECK(o != nullptr && out_lo->numel() == p.numel() && out_lo->is_contiguous(), "out_lo needs out, same size");
    lo = BF(*out_lo);
  }
  hsd::launch_adam(p.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), g.data_ptr(), gbf, o, dm,
                   p.numel(), (float)step, (float)eps, (float)b1, (float)b2, (float)gscale, (float)lr_wd,
                   dcoef, cur_stream(), lo, zero_grad);
}

#define OPT_BF(o) ((o).has_value() ? reinterpret_cast<hsd::bf16_t*>((o)->data_ptr()) : nullptr)
#define OPT_F(o) ((o).has_value() ? (o)->data_ptr<float>() : nullptr)
#define OPT_I64(o) ((o).has_value() ? (o)->data_ptr<int64_t>() : nullptr)

void check_bf16(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == torch::kBFloat16, name,
              " must be a contiguous bf16 GPU tensor");
}
void check_f32(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == torch::kFloat32, name,
              " must be a contiguous fp32 GPU tensor");
}

// y [rows,H] (+ residual) -> z (saved), out, mean, rstd
void ln_fwd(torch::Tensor y, c10::optional<torch::Tensor> res, torch::Tensor gamma, torch::Tensor beta,
            c10::optional<torch::Tensor> z, torch::Tensor out, torch::Tensor mean, torch::Tensor rstd, double eps,
            double p, int64_t seed) {
  check_bf16(y, "y"); check_bf16(out, "out"); check_bf16(gamma, "gamma"); check_bf16(beta, "beta");
  check_f32(mean, "mean"); check_f32(rstd, "rstd");
  const int H = (int)y.size(-1);
  const int rows = (int)(y.numel() / H);
  TORCH_CHECK(H % 4 == 0 && H <= 2048, "LayerNorm width must be a multiple of 4 and <= 2048");
  TORCH_CHECK(gamma.numel() == H && beta.numel() == H && mean.numel() >= rows && rstd.numel() >= rows, "ln shapes");
  if (res.has_value()) { check_bf16(*res, "res"); TORCH_CHECK(res->numel() == y.numel(), "res shape"); }
  if (z.has_value()) { check_bf16(*z, "z"); TORCH_CHECK(z->numel() == y.numel(), "z shape"); }
  hsd::launch_ln_fwd(CBF(y), res.has_value() ? CBF(*res) : nullptr, CBF(gamma), CBF(beta), OPT_BF(z), BF(out),
                     mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, H, (float)eps, p, (uint64_t)seed,
                     cur_stream());
}

// LN forward + the output's fp8 e4m3 copy (delayed scaling: amax_in = the site's previous amax, fp32 [1]; sinv fp32 [1]
// written; amax_track fp32 [1] accumulates this tensor's amax)
void ln_fwd_q8(torch::Tensor y, torch::Tensor gamma, torch::Tensor beta, torch::Tensor out, torch::Tensor mean,
               torch::Tensor rstd, double eps, torch::Tensor q8, torch::Tensor amax_in, torch::Tensor sinv,
               torch::Tensor amax_track) {
  check_bf16(y, "y"); check_bf16(out, "out"); check_bf16(gamma, "gamma"); check_bf16(beta, "beta");
  check_f32(mean, "mean"); check_f32(rstd, "rstd");
  check_f32(amax_in, "amax_in"); check_f32(sinv, "sinv"); check_f32(amax_track, "amax_track");
  CHECK_CUDA(q8); CHECK_CONTIG(q8); CHECK_DTYPE(q8, torch::kUInt8);
  const int H = (int)y.size(-1);
  const int rows = (int)(y.numel() / H);
  TORCH_CHECK(H % 8 == 0 && H <= 1024, "ln_fwd_q8: H % 8 == 0 and H <= 1024");
  TORCH_CHECK(gamma.numel() == H && beta.numel() == H && mean.numel() >= rows && rstd.numel() >= rows, "ln shapes");
  TORCH_CHECK(q8.numel() == y.numel() && out.numel() == y.numel(), "q8 / out shape");
  hsd::launch_ln_fwd_q8(CBF(y), CBF(gamma), CBF(beta), BF(out), mean.data_ptr<float>(), rstd.data_ptr<float>(), rows,
                        H, (float)eps, q8.data_ptr<uint8_t>(), amax_in.data_ptr<float>(), sinv.data_ptr<float>(),
                        amax_track.data_ptr<float>(), cur_stream());
}

void ln_bwd(torch::Tensor dout, torch::Tensor z, torch::Tensor mean, torch::Tensor rstd, torch::Tensor gamma,
            c10::optional<torch::Tensor> dz, c10::optional<torch::Tensor> dy, c10::optional<torch::Tensor> dres_add,
            torch::Tensor dgamma, torch::Tensor dbeta, c10::optional<torch::Tensor> dbias, double p, int64_t seed) {
  check_bf16(dout, "dout"); check_bf16(z, "z"); check_bf16(gamma, "gamma");
  check_f32(mean, "mean"); check_f32(rstd, "rstd"); check_f32(dgamma, "dgamma"); check_f32(dbeta, "dbeta");
  const int H = (int)z.size(-1);
  const int rows = (int)(z.numel() / H);
  TORCH_CHECK(dout.numel() == z.numel() && H % 4 == 0 && H <= 1024, "ln_bwd shapes (H <= 1024)");
  TORCH_CHECK(dgamma.numel() == H && dbeta.numel() == H, "dgamma/dbeta shape");
  if (dz.has_value()) { check_bf16(*dz, "dz"); TORCH_CHECK(dz->numel() == z.numel(), "dz shape"); }
  if (dy.has_value()) { check_bf16(*dy, "dy"); TORCH_CHECK(dy->numel() == z.numel(), "dy shape"); }
  if (dres_add.has_value()) { check_bf16(*dres_add, "dres_add"); TORCH_CHECK(dres_add->numel() == z.numel(), "dres"); }
  if (dbias.has_value()) { check_f32(*dbias, "dbias"); TORCH_CHECK(dbias->numel() == H, "dbias shape"); }
  hsd::launch_ln_bwd(CBF(dout), CBF(z), mean.data_ptr<float>(), rstd.data_ptr<float>(), CBF(gamma), OPT_BF(dz),
                     OPT_BF(dy), dres_add.has_value() ? CBF(*dres_add) : nullptr, dgamma.data_ptr<float>(),
                     dbeta.data_ptr<float>(), OPT_F(dbias), rows, H, p, (uint64_t)seed, cur_stream());
}

// ln_bwd + dy's fp8 copy (qfmt 0 e4m3 / 1 e5m2) for the fp8 dgrad GEMM; dy required
void ln_bwd_q8(torch::Tensor dout, torch::Tensor z, torch::Tensor mean, torch::Tensor rstd, torch::Tensor gamma,
               c10::optional<torch::Tensor> dz, torch::Tensor dy, torch::Tensor dgamma, torch::Tensor dbeta,
               c10::optional<torch::Tensor> dbias, double p, int64_t seed, torch::Tensor q8, torch::Tensor amax_in,
               torch::Tensor sinv, torch::Tensor amax_track, int64_t qfmt, bool q8_only) {
  check_bf16(dout, "dout"); check_bf16(z, "z"); check_bf16(gamma, "gamma"); check_bf16(dy, "dy");
  TORCH_CHECK(!q8_only || (dz.has_value() && p > 0), "ln_bwd_q8 q8_only: dz must be its own buffer (dropout on)");
  check_f32(mean, "mean"); check_f32(rstd, "rstd"); check_f32(dgamma, "dgamma"); check_f32(dbeta, "dbeta");
  check_f32(amax_in, "amax_in"); check_f32(sinv, "sinv"); check_f32(amax_track, "amax_track");
  CHECK_CUDA(q8); CHECK_CONTIG(q8); CHECK_DTYPE(q8, torch::kUInt8);
  const int H = (int)z.size(-1);
  const int rows = (int)(z.numel() / H);
  TORCH_CHECK(dout.numel() == z.numel() && dy.numel() == z.numel() && q8.numel() == z.numel(), "ln_bwd_q8 shapes");
  TORCH_CHECK(H % 4 == 0 && H <= 1024 && (qfmt == 0 || qfmt == 1), "ln_bwd_q8: H % 4 == 0, H <= 1024, qfmt 0/1");
  TORCH_CHECK(dgamma.numel() == H && dbeta.numel() == H, "dgamma/dbeta shape");
  if (dz.has_value()) { check_bf16(*dz, "dz"); TORCH_CHECK(dz->numel() == z.numel(), "dz shape"); }
  if (dbias.has_value()) { check_f32(*dbias, "dbias"); TORCH_CHECK(dbias->numel() == H, "dbias shape"); }
  hsd::launch_ln_bwd_q8(CBF(dout), CBF(z), mean.data_ptr<float>(), rstd.data_ptr<float>(), CBF(gamma), OPT_BF(dz),
                        BF(dy), nullptr, dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), OPT_F(dbias), rows, H, p,
                        (uint64_t)seed, q8.data_ptr<uint8_t>(), amax_in.data_ptr<float>(), sinv.data_ptr<float>(),
                        amax_track.data_ptr<float>(), (int)qfmt, cur_stream(), q8_only);
}

void embed_fwd(torch::Tensor ids, torch::Tensor pos_ids, c10::optional<torch::Tensor> type_ids, torch::Tensor word,
               torch::Tensor pos, c10::optional<torch::Tensor> type, torch::Tensor gamma, torch::Tensor beta,
               torch::Tensor out, torch::Tensor mean, torch::Tensor rstd, double eps, double p, int64_t seed,
               c10::optional<torch::Tensor> q8, c10::optional<torch::Tensor> amax_in, c10::optional<torch::Tensor> sinv,
               c10::optional<torch::Tensor> amax_track) {
  TORCH_CHECK(ids.scalar_type() == torch::kInt64 && pos_ids.scalar_type() == torch::kInt64, "ids must be int64");
  TORCH_CHECK(ids.is_contiguous() && pos_ids.is_contiguous(), "ids contiguous");
  check_bf16(word, "word"); check_bf16(pos, "pos"); check_bf16(out, "out");
  const int H = (int)word.size(1);
  const int rows = (int)ids.numel();
  TORCH_CHECK(H % 4 == 0 && H <= 1024 && out.numel() == (int64_t)rows * H, "embed shapes");
  TORCH_CHECK(type.has_value() == type_ids.has_value(), "type table and ids go together");
#ifdef HSD_DEBUG
  // the kernels index the tables with these ids unchecked
  auto in_range = [](const torch::Tensor& t, int64_t n) {
    return t.numel() == 0 || (t.min().item<int64_t>() >= 0 && t.max().item<int64_t>() < n);
  };
  TORCH_CHECK(in_range(ids, word.size(0)), "HSD_DEBUG: input id out of vocabulary range");
  TORCH_CHECK(in_range(pos_ids, pos.size(0)), "HSD_DEBUG: position id out of range");
  if (type_ids.has_value()) TORCH_CHECK(in_range(*type_ids, type->size(0)), "HSD_DEBUG: token type id out of range");
#endif
  if (q8.has_value()) {  // the output's fp8 copy (the first layer's fp8 QKV GEMM): as ln_fwd_q8
    CHECK_CUDA(*q8); CHECK_CONTIG(*q8); CHECK_DTYPE(*q8, torch::kUInt8);
    TORCH_CHECK(q8->numel() == out.numel() && amax_in.has_value() && sinv.has_value() && amax_track.has_value(),
                "embed_fwd q8 arguments");
    check_f32(*amax_in, "amax_in"); check_f32(*sinv, "sinv"); check_f32(*amax_track, "amax_track");
  }
  hsd::launch_embed_fwd(ids.data_ptr<int64_t>(), pos_ids.data_ptr<int64_t>(), OPT_I64(type_ids), CBF(word),
                        CBF(pos), type.has_value() ? CBF(*type) : nullptr, CBF(gamma), CBF(beta), BF(out),
                        mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, H, (float)eps, p, (uint64_t)seed,
                        cur_stream(), q8.has_value() ? q8->data_ptr<uint8_t>() : nullptr, OPT_F(amax_in), OPT_F(sinv),
                        OPT_F(amax_track));
}

void embed_bwd(torch::Tensor dout, torch::Tensor ids, torch::Tensor pos_ids, c10::optional<torch::Tensor> type_ids,
               torch::Tensor word, torch::Tensor pos, c10::optional<torch::Tensor> type, torch::Tensor gamma,
               torch::Tensor mean, torch::Tensor rstd, torch::Tensor gword, torch::Tensor gpos,
               c10::optional<torch::Tensor> gtype, torch::Tensor ggamma, torch::Tensor gbeta, int64_t B, int64_t S,
               bool pos_is_arange, double p, int64_t seed) {
  check_bf16(dout, "dout");
  check_f32(gword, "gword"); check_f32(gpos, "gpos"); check_f32(ggamma, "ggamma"); check_f32(gbeta, "gbeta");
  const int H = (int)word.size(1);
  TORCH_CHECK(ids.numel() == B * S && dout.numel() == B * S * H, "embed_bwd shapes");
  TORCH_CHECK(gword.numel() == word.numel() && gpos.numel() == pos.numel(), "grad table shapes");
  hsd::launch_embed_bwd(CBF(dout), ids.data_ptr<int64_t>(), pos_ids.data_ptr<int64_t>(), OPT_I64(type_ids),
                        CBF(word), CBF(pos), type.has_value() ? CBF(*type) : nullptr, CBF(gamma),
                        mean.data_ptr<float>(), rstd.data_ptr<float>(), gword.data_ptr<float>(),
                        gpos.data_ptr<float>(), OPT_F(gtype), ggamma.data_ptr<float>(), gbeta.data_ptr<float>(),
                        (int)B, (int)S, H, pos_is_arange ? 1 : 0, p, (uint64_t)seed, cur_stream());
}

void gelu_fwd(torch::Tensor y, torch::Tensor g) {
  check_bf16(y, "y"); check_bf16(g, "g");
  TORCH_CHECK(y.numel() == g.numel() && y.numel() % 8 == 0, "gelu shapes");
  hsd::launch_gelu_fwd(CBF(y), BF(g), y.numel(), cur_stream());
}

void gelu_bwd_colsum(torch::Tensor dg, torch::Tensor y, torch::Tensor da, c10::optional<torch::Tensor> dbias) {
  check_bf16(dg, "dg"); check_bf16(y, "y"); check_bf16(da, "da");
  const int N = (int)y.size(-1);
  const int rows = (int)(y.numel() / N);
  TORCH_CHECK(N % 8 == 0 && dg.numel() == y.numel() && da.numel() == y.numel(), "gelu_bwd shapes");
  if (dbias.has_value()) { check_f32(*dbias, "dbias"); TORCH_CHECK(dbias->numel() == N, "dbias"); }
  hsd::launch_gelu_bwd_colsum(CBF(dg), CBF(y), BF(da), OPT_F(dbias), rows, N, cur_stream());
}

void colsum(torch::Tensor x, torch::Tensor dbias) {
  check_bf16(x, "x"); check_f32(dbias, "dbias");
  const int N = (int)x.size(-1);
  const int rows = (int)(x.numel() / N);
  TORCH_CHECK(N % 8 == 0 && dbias.numel() == N, "colsum shapes");
  hsd::launch_colsum(CBF(x), dbias.data_ptr<float>(), rows, N, cur_stream());
}

void dropout(torch::Tensor x, torch::Tensor out, double p, int64_t seed) {
  check_bf16(x, "x"); check_bf16(out, "out");
  // the mask's row width is the last dimension (ops/rng.py); 4-element vectors never straddle a row
  const int64_t W = x.dim() ? x.size(-1) : 1;
  TORCH_CHECK(x.numel() == out.numel() && W % 4 == 0, "dropout shapes");
  hsd::launch_dropout(CBF(x), BF(out), x.numel(), (int)W, p, (uint64_t)seed, cur_stream());
}

static uint32_t* keep_mask_ptr(const c10::optional<torch::Tensor>& km, int64_t B, int64_t S, int64_t heads) {
  if (!km.has_value()) return nullptr;
  CHECK_CUDA(*km); CHECK_CONTIG(*km); CHECK_DTYPE(*km, torch::kInt32);
  TORCH_CHECK(km->numel() > 0 && km->numel() == hsd::attn_keep_mask_numel((int)B, (int)S, (int)heads),
              "attention keep mask (attn_keep_mask_numel)");
  return reinterpret_cast<uint32_t*>(km->data_ptr<int32_t>());
}

void attn_fwd(torch::Tensor qkv, c10::optional<torch::Tensor> mask, torch::Tensor out, torch::Tensor lse2, int64_t B,
              int64_t S, int64_t heads, double p, int64_t seed, c10::optional<torch::Tensor> kmask) {
  check_bf16(qkv, "qkv"); check_bf16(out, "out"); check_f32(lse2, "lse2");
  TORCH_CHECK(qkv.size(-1) == 3 * heads * 64, "attention requires head_dim 64");
  TORCH_CHECK(qkv.numel() == B * S * 3 * heads * 64 && out.numel() == B * S * heads * 64, "attn shapes");
  TORCH_CHECK(lse2.numel() == B * heads * S, "lse shape");
  TORCH_CHECK(S % 2 == 0, "sequence length must be even");
  if (mask.has_value()) { check_f32(*mask, "mask"); TORCH_CHECK(mask->numel() == B * S, "mask shape"); }
  hsd::launch_attn_fwd(CBF(qkv), OPT_F(mask), BF(out), lse2.data_ptr<float>(), (int)B, (int)S, (int)heads, p,
                       (uint64_t)seed, cur_stream(), keep_mask_ptr(kmask, B, S, heads));
}

void attn_bwd(torch::Tensor qkv, c10::optional<torch::Tensor> mask, torch::Tensor o, torch::Tensor dout,
              torch::Tensor lse2, torch::Tensor dqkv, c10::optional<torch::Tensor> dq_acc, int64_t B, int64_t S,
              int64_t heads, double p, int64_t seed, c10::optional<torch::Tensor> dbias,
              c10::optional<torch::Tensor> kmask, bool delta_ready) {
  check_bf16(qkv, "qkv"); check_bf16(o, "o"); check_bf16(dout, "dout"); check_bf16(dqkv, "dqkv");
  TORCH_CHECK(!delta_ready || (S > 128 && hsd::attn_streaming((int)S) && dq_acc.has_value()),
              "attn_bwd delta_ready: streaming attention with the delta rows in dq_acc");
  check_f32(lse2, "lse2");
  TORCH_CHECK(qkv.size(-1) == 3 * heads * 64 && dqkv.numel() == qkv.numel(), "attn_bwd shapes");
  TORCH_CHECK(o.numel() == B * S * heads * 64 && dout.numel() == o.numel(), "attn_bwd o shapes");
  TORCH_CHECK(S <= 128 || dq_acc.has_value(), "S > 128 needs an fp32 workspace (attn_bwd_ws_numel)");
  if (dq_acc.has_value()) {
    check_f32(*dq_acc, "dq_acc");
    TORCH_CHECK(dq_acc->numel() == (hsd::attn_streaming((int)S) ? B * heads * S : o.numel()), "dq_acc workspace size");
  }
  if (mask.has_value()) { check_f32(*mask, "mask"); TORCH_CHECK(mask->numel() == B * S, "mask shape"); }
  if (dbias.has_value()) { check_f32(*dbias, "dbias"); TORCH_CHECK(dbias->numel() == 3 * heads * 64, "dbias shape"); }
  hsd::launch_attn_bwd(CBF(qkv), OPT_F(mask), CBF(o), CBF(dout), lse2.data_ptr<float>(), BF(dqkv), OPT_F(dq_acc),
                       OPT_F(dbias), (int)B, (int)S, (int)heads, p, (uint64_t)seed, cur_stream(),
                       keep_mask_ptr(kmask, B, S, heads), delta_ready);
}

// attention + fp8 copy of its output (forward: e4m3 of the context; backward: dqkv in format qfmt), S > 128 streaming
// kernels only (attn_q8_supported); amax_in / sinv / amax_track: fp32 [1] delayed-scaling site slots
static void check_q8(const torch::Tensor& q8, int64_t numel, const torch::Tensor& a, const torch::Tensor& s,
                     const torch::Tensor& t) {
  CHECK_CUDA(q8); CHECK_CONTIG(q8); CHECK_DTYPE(q8, torch::kUInt8);
  TORCH_CHECK(q8.numel() == numel, "q8 shape");
  check_f32(a, "amax_in"); check_f32(s, "sinv"); check_f32(t, "amax_track");
}

void attn_fwd_q8(torch::Tensor qkv, c10::optional<torch::Tensor> mask, torch::Tensor out, torch::Tensor lse2, int64_t B,
                 int64_t S, int64_t heads, double p, int64_t seed, torch::Tensor q8, torch::Tensor amax_in,
                 torch::Tensor sinv, torch::Tensor amax_track, c10::optional<torch::Tensor> kmask) {
  check_bf16(qkv, "qkv"); check_bf16(out, "out"); check_f32(lse2, "lse2");
  TORCH_CHECK(S > 128 && hsd::attn_streaming((int)S), "attn_fwd_q8: streaming attention (S > 128) only");
  TORCH_CHECK(qkv.size(-1) == 3 * heads * 64, "attention requires head_dim 64");
  TORCH_CHECK(qkv.numel() == B * S * 3 * heads * 64 && out.numel() == B * S * heads * 64, "attn shapes");
  TORCH_CHECK(lse2.numel() == B * heads * S, "lse shape");
  if (mask.has_value()) { check_f32(*mask, "mask"); TORCH_CHECK(mask->numel() == B * S, "mask shape"); }
  check_q8(q8, out.numel(), amax_in, sinv, amax_track);
  hsd::launch_attnS_fwd_q8(CBF(qkv), OPT_F(mask), BF(out), lse2.data_ptr<float>(), (int)B, (int)S, (int)heads, p,
                           (uint64_t)seed, q8.data_ptr<uint8_t>(), amax_in.data_ptr<float>(), sinv.data_ptr<float>(),
                           amax_track.data_ptr<float>(), cur_stream(), keep_mask_ptr(kmask, B, S, heads));
}

void attn_bwd_q8(torch::Tensor qkv, c10::optional<torch::Tensor> mask, torch::Tensor o, torch::Tensor dout,
                 torch::Tensor lse2, torch::Tensor dqkv, torch::Tensor ws, int64_t B, int64_t S, int64_t heads, double p,
                 int64_t seed, c10::optional<torch::Tensor> dbias, torch::Tensor q8, torch::Tensor amax_in,
                 torch::Tensor sinv, torch::Tensor amax_track, int64_t qfmt, c10::optional<torch::Tensor> kmask,
                 bool delta_ready, bool q8_only) {
  check_bf16(qkv, "qkv"); check_bf16(o, "o"); check_bf16(dout, "dout"); check_bf16(dqkv, "dqkv");
  check_f32(lse2, "lse2"); check_f32(ws, "ws");
  TORCH_CHECK(S > 128 && hsd::attn_streaming((int)S), "attn_bwd_q8: streaming attention (S > 128) only");
  TORCH_CHECK(qkv.size(-1) == 3 * heads * 64 && dqkv.numel() == qkv.numel(), "attn_bwd shapes");
  TORCH_CHECK(o.numel() == B * S * heads * 64 && dout.numel() == o.numel(), "attn_bwd o shapes");
  TORCH_CHECK(ws.numel() == B * heads * S, "ws size");
  TORCH_CHECK(qfmt == 0 || qfmt == 1, "qfmt");
  if (mask.has_value()) { check_f32(*mask, "mask"); TORCH_CHECK(mask->numel() == B * S, "mask shape"); }
  if (dbias.has_value()) { check_f32(*dbias, "dbias"); TORCH_CHECK(dbias->numel() == 3 * heads * 64, "dbias shape"); }
  check_q8(q8, dqkv.numel(), amax_in, sinv, amax_track);
  hsd::launch_attnS_bwd_q8(CBF(qkv), OPT_F(mask), CBF(o), CBF(dout), lse2.data_ptr<float>(), BF(dqkv),
                           ws.data_ptr<float>(), OPT_F(dbias), (int)B, (int)S, (int)heads, p, (uint64_t)seed,
                           q8.data_ptr<uint8_t>(), amax_in.data_ptr<float>(), sinv.data_ptr<float>(),
                           amax_track.data_ptr<float>(), (int)qfmt, cur_stream(), keep_mask_ptr(kmask, B, S, heads),
                           delta_ready, q8_only);
}

// C[M,N] (+)= A·B with fused epilogue. la=0: A [M,K]; la=1: A [K,M]. lb=0: B [N,K]; lb=1: B [K,N].
void gemm(torch::Tensor A, torch::Tensor B, torch::Tensor C, int64_t la, int64_t lb, int64_t epi,
          c10::optional<torch::Tensor> bias, c10::optional<torch::Tensor> aux, c10::optional<torch::Tensor> C2,
          double p, int64_t seed, int64_t splits) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && C.is_cuda(), "gemm operands must be GPU tensors");
  TORCH_CHECK(A.scalar_type() == torch::kBFloat16 && B.scalar_type() == torch::kBFloat16, "gemm inputs must be bf16");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "gemm operands must be 2-D");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && C.stride(1) == 1, "gemm operands need unit inner stride");
  const int64_t M = la == 0 ? A.size(0) : A.size(1);
  const int64_t K = la == 0 ? A.size(1) : A.size(0);
  const int64_t N = lb == 0 ? B.size(0) : B.size(1);
  const int64_t KB = lb == 0 ? B.size(1) : B.size(0);
  TORCH_CHECK(K == KB, "gemm K mismatch");
  TORCH_CHECK(C.size(0) == M && C.size(1) == N, "gemm C shape");
  TORCH_CHECK(M % 8 == 0 && N % 8 == 0 && K % 8 == 0, "gemm dims must be multiples of 8");
  TORCH_CHECK(A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0 && C.stride(0) % 4 == 0, "gemm leading dims alignment");
  const bool f32out = epi == 6;
  TORCH_CHECK(C.scalar_type() == (f32out ? torch::kFloat32 : torch::kBFloat16), "gemm C dtype");
  if (epi == 1 || epi == 2 || epi == 3) {
    TORCH_CHECK(bias.has_value() && bias->numel() == N && bias->scalar_type() == torch::kBFloat16 &&
                bias->is_contiguous(), "gemm bias");
  }
  if (epi == 3 || epi == 4 || epi == 5) {
    TORCH_CHECK(aux.has_value() && aux->dim() == 2 && aux->size(0) == M && aux->size(1) == N &&
                aux->stride(1) == 1 && aux->scalar_type() == torch::kBFloat16, "gemm aux");
  }
  if (epi == 2) {
    TORCH_CHECK(C2.has_value() && C2->sizes() == C.sizes() && C2->strides() == C.strides() &&
                C2->scalar_type() == torch::kBFloat16, "gemm C2");
  }
  TORCH_CHECK(epi == 6 || splits == 1, "split-K only with the fp32 atomic epilogue");
  hsd::launch_gemm((int)la, (int)lb, (int)epi, CBF(A), A.stride(0), CBF(B), B.stride(0), (int)M, (int)N, (int)K,
                   C.data_ptr(), C.stride(0), bias.has_value() ? CBF(*bias) : nullptr,
                   aux.has_value() ? CBF(*aux) : nullptr, aux.has_value() ? aux->stride(0) : 0,
                   C2.has_value() ? BF(*C2) : nullptr, p, (uint64_t)seed, (int)splits, cur_stream());
}

// gemm2: la=lb=0 -> NT (A [M,K], B [N,K]) bf16 C with epilogue 0..5;
//        la=lb=1 -> TT (A [K,M], B [K,N]) fp32 C += A^T B, epi 6 atomics / 7 slabs in ws.
// fp8 per-tensor quantisation: q = sat(x · FMT_MAX / amax), sinv = amax / FMT_MAX (device scalars)
void fp8_quant(torch::Tensor x, torch::Tensor amax, torch::Tensor q, torch::Tensor sinv, int64_t fmt,
               bool compute_amax, c10::optional<torch::Tensor> amax_track) {
  check_bf16(x, "x");
  check_f32(amax, "amax"); check_f32(sinv, "sinv");
  TORCH_CHECK(q.is_cuda() && q.scalar_type() == torch::kUInt8 && q.is_contiguous() && q.numel() == x.numel(),
              "fp8_quant q: contiguous uint8 of x's size");
  TORCH_CHECK(fmt == 0 || fmt == 1, "fmt: 0 = e4m3, 1 = e5m2");
  TORCH_CHECK(amax.numel() >= 1 && sinv.numel() >= 1, "fp8_quant scalars");
  float* trk = nullptr;
  if (amax_track.has_value()) {
    check_f32(*amax_track, "amax_track");
    trk = amax_track->data_ptr<float>();
  }
  hsd::launch_fp8_quant(CBF(x), x.numel(), amax.data_ptr<float>(), q.data_ptr<uint8_t>(), sinv.data_ptr<float>(),
                        (int)fmt, compute_amax, trk, cur_stream());
}

void fp8_quant_many(torch::Tensor amax_desc, int64_t amax_blocks, torch::Tensor quant_desc, int64_t quant_blocks,
                    torch::Tensor amax, torch::Tensor sinv, int64_t fmt) {
  TORCH_CHECK(amax_desc.is_cuda() && amax_desc.scalar_type() == torch::kInt64 && amax_desc.dim() == 2 &&
              amax_desc.size(1) == 5 && amax_desc.is_contiguous(), "amax_desc int64 [n][5]");
  TORCH_CHECK(quant_desc.is_cuda() && quant_desc.scalar_type() == torch::kInt64 && quant_desc.dim() == 2 &&
              quant_desc.size(1) == 5 && quant_desc.is_contiguous(), "quant_desc int64 [n][5]");
  check_f32(amax, "amax"); check_f32(sinv, "sinv");
  TORCH_CHECK(fmt == 0 || fmt == 1, "fmt");
  hsd::launch_fp8_quant_many(amax_desc.data_ptr<int64_t>(), (int)amax_desc.size(0), (int)amax_blocks,
                             quant_desc.data_ptr<int64_t>(), (int)quant_desc.size(0), (int)quant_blocks,
                             amax.data_ptr<float>(), sinv.data_ptr<float>(), (int)fmt, cur_stream());
}

// C = epilogue(sa·sb · A8 · B8ᵀ): A8 [M][K], B8 [N][K] uint8 (fp8 bits), same epilogue codes as gemm2 (bf16 out)
// q8 (optional): uint8 [M][N] fp8 copy of the bf16 output (C2 for two-output epilogues, else C) in format q8fmt,
// delayed scaling from q8_amax[0]; q8_sinv[0] = 1/scale; q8_track[0] accumulates the output's amax
void gemm8(torch::Tensor A, int64_t fa, torch::Tensor sa, torch::Tensor B, int64_t fb, torch::Tensor sb,
           torch::Tensor C, int64_t epi, c10::optional<torch::Tensor> bias, c10::optional<torch::Tensor> aux,
           c10::optional<torch::Tensor> C2, double p, int64_t seed, c10::optional<torch::Tensor> dbias,
           c10::optional<torch::Tensor> q8, c10::optional<torch::Tensor> q8_amax, c10::optional<torch::Tensor> q8_sinv,
           c10::optional<torch::Tensor> q8_track, int64_t q8fmt, c10::optional<torch::Tensor> rd, int64_t rd_seq,
           bool q8_only) {
  uint8_t* q8p = nullptr;
  float *q8s = nullptr, *q8t = nullptr;
  const float* q8a = nullptr;
  if (q8.has_value()) {
    TORCH_CHECK(q8_amax.has_value() && q8_sinv.has_value() && q8_track.has_value(), "gemm8 q8: amax / sinv / track");
    check_q8(*q8, C.numel(), *q8_amax, *q8_sinv, *q8_track);
    TORCH_CHECK(C.is_contiguous(), "gemm8 q8: contiguous C");
    TORCH_CHECK(q8fmt == 0 || q8fmt == 1, "gemm8 q8 format");
    q8p = q8->data_ptr<uint8_t>(); q8a = q8_amax->data_ptr<float>(); q8s = q8_sinv->data_ptr<float>();
    q8t = q8_track->data_ptr<float>();
  }
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && C.is_cuda(), "gemm8 operands must be GPU tensors");
  TORCH_CHECK(A.scalar_type() == torch::kUInt8 && B.scalar_type() == torch::kUInt8, "gemm8 inputs: uint8 fp8 bits");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "gemm8 operands must be 2-D");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && C.stride(1) == 1, "gemm8 unit inner stride");
  const int64_t M = A.size(0), K = A.size(1), N = B.size(0);
  TORCH_CHECK(B.size(1) == K, "gemm8 K mismatch");
  TORCH_CHECK(C.size(0) == M && C.size(1) == N && C.scalar_type() == torch::kBFloat16, "gemm8 C");
  TORCH_CHECK(hsd::gemm8_supported((int)epi, (int)M, (int)N, (int)K), "gemm8: unsupported shape/epilogue");
  TORCH_CHECK(A.stride(0) % 16 == 0 && B.stride(0) % 16 == 0 && C.stride(0) % 8 == 0, "gemm8 leading dims alignment");
  TORCH_CHECK(fa == 0 || fa == 1, "gemm8 fa");
  TORCH_CHECK(fb == 0, "gemm8: weights (B) are e4m3");
  check_f32(sa, "sa"); check_f32(sb, "sb");
  if (epi == 1 || epi == 2 || epi == 3 || epi == 8) {
    TORCH_CHECK(bias.has_value() && bias->numel() == N && bias->scalar_type() == torch::kBFloat16 &&
                bias->is_contiguous(), "gemm8 bias");
  }
  if (epi == 3 || epi == 4 || epi == 5 || epi == 9 || epi == 10) {
    TORCH_CHECK(aux.has_value() && aux->dim() == 2 && aux->size(0) == M && aux->size(1) == N &&
                aux->stride(1) == 1 && aux->stride(0) % 8 == 0 && aux->scalar_type() == torch::kBFloat16, "gemm8 aux");
  }
  if (epi == 2 || epi == 8) {
    TORCH_CHECK(C2.has_value() && C2->sizes() == C.sizes() && C2->strides() == C.strides() &&
                C2->scalar_type() == torch::kBFloat16, "gemm8 C2");
  }
  float* dbp = nullptr;
  if (dbias.has_value()) {
    TORCH_CHECK((epi == 5 || epi == 9) && N % 256 == 0, "gemm8 fused dbias: DGELU / MUL epilogue with N % 256 == 0");
    check_f32(*dbias, "dbias");
    TORCH_CHECK(dbias->numel() == N, "dbias size");
    dbp = dbias->data_ptr<float>();
  }
  float* rdp = nullptr;
  if (epi == 10) {
    TORCH_CHECK(rd.has_value() && rd_seq > 0 && M % rd_seq == 0, "gemm8 row dots: rd and the sequence length");
    check_f32(*rd, "rd");
    TORCH_CHECK(rd->numel() == M * (N / 64), "gemm8 row dots: rd size");
    rdp = rd->data_ptr<float>();
  }
  hsd::launch_gemm8((int)epi, A.data_ptr<uint8_t>(), A.stride(0), (int)fa, sa.data_ptr<float>(), B.data_ptr<uint8_t>(),
                    B.stride(0), (int)fb, sb.data_ptr<float>(), (int)M, (int)N, (int)K, BF(C), C.stride(0),
                    bias.has_value() ? CBF(*bias) : nullptr, aux.has_value() ? CBF(*aux) : nullptr,
                    aux.has_value() ? aux->stride(0) : 0, C2.has_value() ? BF(*C2) : nullptr, p, (uint64_t)seed, dbp,
                    cur_stream(), q8p, q8a, q8s, q8t, (int)q8fmt, rdp, (int)rd_seq, q8_only ? 1 : 0);
}

// C[M][N] fp32 += sdy·sx · dY8ᵀ · X8 (fp8 TT weight gradient): dY8 uint8 [T][M] (format fdy), X8 uint8 [T][N] (e4m3),
// ws fp32 >= gemm8_wgrad_ws_numel; stream_ptr 0 = the current stream (else e.g. the weight-gradient side stream)
void gemm8_wgrad(int64_t stream_ptr, torch::Tensor dy, int64_t fdy, torch::Tensor sdy, torch::Tensor x, int64_t fx,
                 torch::Tensor sx, torch::Tensor C, int64_t splits, torch::Tensor ws) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && C.is_cuda() && ws.is_cuda(), "gemm8_wgrad: GPU tensors");
  TORCH_CHECK(dy.scalar_type() == torch::kUInt8 && x.scalar_type() == torch::kUInt8, "gemm8_wgrad: uint8 fp8 bits");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && C.dim() == 2, "gemm8_wgrad: 2-D operands");
  TORCH_CHECK(dy.stride(1) == 1 && x.stride(1) == 1 && C.stride(1) == 1, "gemm8_wgrad: unit inner stride");
  const int64_t T = dy.size(0), M = dy.size(1), N = x.size(1);
  TORCH_CHECK(x.size(0) == T, "gemm8_wgrad: token count mismatch");
  TORCH_CHECK(C.size(0) == M && C.size(1) == N && C.scalar_type() == torch::kFloat32, "gemm8_wgrad: C fp32 [M][N]");
  TORCH_CHECK(hsd::gemm8_wgrad_supported((int)M, (int)N, (int)T), "gemm8_wgrad: unsupported shape");
  TORCH_CHECK(dy.stride(0) % 16 == 0 && x.stride(0) % 16 == 0 && C.stride(0) % 4 == 0, "gemm8_wgrad: leading dims");
  TORCH_CHECK(fdy == 0 || fdy == 1, "gemm8_wgrad: fdy");
  TORCH_CHECK(fx == 0, "gemm8_wgrad: activations (X8) are e4m3");
  check_f32(sdy, "sdy"); check_f32(sx, "sx"); check_f32(ws, "ws");
  TORCH_CHECK(ws.numel() >= hsd::gemm8_wgrad_ws_numel((int)M, (int)N, (int)T, (int)splits), "gemm8_wgrad: workspace");
  hipStream_t st = stream_ptr ? reinterpret_cast<hipStream_t>(stream_ptr) : cur_stream();
  hsd::launch_gemm8_wgrad(dy.data_ptr<uint8_t>(), dy.stride(0), (int)fdy, sdy.data_ptr<float>(), x.data_ptr<uint8_t>(),
                          x.stride(0), (int)fx, sx.data_ptr<float>(), (int)M, (int)N, (int)T, C.data_ptr<float>(),
                          C.stride(0), (int)splits, ws.data_ptr<float>(), st);
}

// device step seed for dropout (uint32/int32 [2] GPU tensor, kept alive by the caller), None = off
void set_dropout_device_seed(c10::optional<torch::Tensor> t) {
  if (!t.has_value()) {
    hsd::set_dropout_dev_seed(nullptr);
    return;
  }
  TORCH_CHECK(t->is_cuda() && t->numel() >= 2 && t->element_size() == 4 && t->is_contiguous(),
              "device seed: contiguous 32-bit GPU tensor of >= 2 elements");
  hsd::set_dropout_dev_seed(reinterpret_cast<const uint32_t*>(t->data_ptr()));
}

void gemm2(torch::Tensor A, torch::Tensor B, torch::Tensor C, int64_t la, int64_t lb, int64_t epi,
           c10::optional<torch::Tensor> bias, c10::optional<torch::Tensor> aux, c10::optional<torch::Tensor> C2,
           double p, int64_t seed, int64_t splits, c10::optional<torch::Tensor> ws,
           c10::optional<torch::Tensor> dbias, c10::optional<torch::Tensor> rd, int64_t rd_seq) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && C.is_cuda(), "gemm2 operands must be GPU tensors");
  TORCH_CHECK(A.scalar_type() == torch::kBFloat16 && B.scalar_type() == torch::kBFloat16, "gemm2 inputs must be bf16");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "gemm2 operands must be 2-D");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && C.stride(1) == 1, "gemm2 operands need unit inner stride");
  TORCH_CHECK(la == lb || (la == 0 && lb == 1), "gemm2 layouts: NT (0,0), NT with B = W[K][N] (0,1) or TT (1,1)");
  const int64_t M = la == 0 ? A.size(0) : A.size(1);
  const int64_t K = la == 0 ? A.size(1) : A.size(0);
  const int64_t N = lb == 0 ? B.size(0) : B.size(1);
  const int64_t KB = lb == 0 ? B.size(1) : B.size(0);
  TORCH_CHECK(K == KB, "gemm2 K mismatch");
  TORCH_CHECK(C.size(0) == M && C.size(1) == N, "gemm2 C shape");
  TORCH_CHECK(hsd::gemm2_supported((int)la, (int)lb, (int)epi, (int)M, (int)N, (int)K), "gemm2: unsupported shape/epilogue");
  TORCH_CHECK(A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0 && C.stride(0) % 8 == 0, "gemm2 leading dims alignment");
  const bool f32out = epi == 6 || epi == 7;
  TORCH_CHECK(C.scalar_type() == (f32out ? torch::kFloat32 : torch::kBFloat16), "gemm2 C dtype");
  if (epi == 1 || epi == 2 || epi == 3 || epi == 8) {
    TORCH_CHECK(bias.has_value() && bias->numel() == N && bias->scalar_type() == torch::kBFloat16 &&
                bias->is_contiguous(), "gemm2 bias");
  }
  if (epi == 3 || epi == 4 || epi == 5 || epi == 9 || epi == 10) {
    TORCH_CHECK(aux.has_value() && aux->dim() == 2 && aux->size(0) == M && aux->size(1) == N &&
                aux->stride(1) == 1 && aux->stride(0) % 8 == 0 && aux->scalar_type() == torch::kBFloat16, "gemm2 aux");
  }
  if (epi == 2 || epi == 8) {
    TORCH_CHECK(C2.has_value() && C2->sizes() == C.sizes() && C2->strides() == C.strides() &&
                C2->scalar_type() == torch::kBFloat16, "gemm2 C2");
  }
  float* wsp = nullptr;
  int sp = (int)splits;
  if (f32out && sp <= 0) sp = hsd::gemm2_wgrad_splits((int)M, (int)N, (int)K);
  if (epi == 7) {
    TORCH_CHECK(C.is_contiguous() || C.stride(0) % 4 == 0, "gemm2 slab C");
    TORCH_CHECK(ws.has_value() && ws->scalar_type() == torch::kFloat32 && ws->is_contiguous() &&
                ws->numel() >= (int64_t)sp * M * N, "gemm2 slab workspace too small");
    wsp = ws->data_ptr<float>();
  }
  torch::Tensor nt_ws;
  if (!f32out) {
    // NT bf16 output: splits <= 0 = automatic (gemm2_nt_splits), 1 = one pass, > 1 = split-K slabs + epilogue pass
    if (sp <= 0) sp = la == 0 ? hsd::gemm2_nt_splits((int)M, (int)N, (int)K) : 1;
    TORCH_CHECK(la == 0 || sp == 1, "gemm2: split-K bf16 output is NT only");
    if (sp > 1) {
      nt_ws = torch::empty({(int64_t)sp * M * N}, A.options().dtype(torch::kFloat32));
      wsp = nt_ws.data_ptr<float>();
    }
  }
  float* dbp = nullptr;
  if (dbias.has_value()) {
    TORCH_CHECK((epi == 5 || epi == 9) && N % 256 == 0, "gemm2 fused dbias: DGELU / MUL epilogue with N % 256 == 0");
    check_f32(*dbias, "dbias");
    TORCH_CHECK(dbias->numel() == N, "dbias size");
    dbp = dbias->data_ptr<float>();
  }
  float* rdp = nullptr;
  if (epi == 10) {
    // delta rows of the attention backward: [M / rd_seq][N / 64][rd_seq] fp32
    TORCH_CHECK(rd.has_value() && rd_seq > 0 && M % rd_seq == 0, "gemm2 row dots: rd and the sequence length");
    check_f32(*rd, "rd");
    TORCH_CHECK(rd->numel() == M * (N / 64), "gemm2 row dots: rd size");
    rdp = rd->data_ptr<float>();
  }
  hsd::launch_gemm2((int)la, (int)lb, (int)epi, CBF(A), A.stride(0), CBF(B), B.stride(0), (int)M, (int)N, (int)K,
                    C.data_ptr(), C.stride(0), bias.has_value() ? CBF(*bias) : nullptr,
                    aux.has_value() ? CBF(*aux) : nullptr, aux.has_value() ? aux->stride(0) : 0,
                    C2.has_value() ? BF(*C2) : nullptr, p, (uint64_t)seed, sp, wsp, dbp, cur_stream(), rdp, (int)rd_seq);
}

// ---- fp32 step (fp32.hip, ops/hip32.py) ---------------------------------------------------------------------------
// C [M][N] fp32 = A [M][K] · Bᵀ (lb 0: B [N][K]; lb 1: B [K][N]), bf16 operands (the split-product concatenations)
void gemm2_f32nt(torch::Tensor A, torch::Tensor B, torch::Tensor C, int64_t lb) {
  check_bf16(A, "A"); check_bf16(B, "B"); check_f32(C, "C");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2 && (lb == 0 || lb == 1), "gemm2_f32nt: 2-D operands");
  const int64_t M = A.size(0), K = A.size(1);
  const int64_t N = lb == 0 ? B.size(0) : B.size(1), KB = lb == 0 ? B.size(1) : B.size(0);
  TORCH_CHECK(K == KB && C.size(0) == M && C.size(1) == N, "gemm2_f32nt shapes");
  TORCH_CHECK(hsd::gemm2_supported(0, (int)lb, 7, (int)M, (int)N, (int)K), "gemm2_f32nt: unsupported shape");
  TORCH_CHECK(C.is_contiguous(), "gemm2_f32nt: contiguous C");
  const int sp = hsd::gemm2_f32nt_splits((int)M, (int)N, (int)K);
  torch::Tensor ws;
  if (sp > 1) ws = torch::empty({(int64_t)sp * M * N}, C.options());  // K-split slabs (stream-ordered pool)
  hsd::launch_gemm2(0, (int)lb, 7, CBF(A), A.stride(0), CBF(B), B.stride(0), (int)M, (int)N, (int)K, C.data_ptr(),
                    C.stride(0), nullptr, nullptr, 0, nullptr, 0.0, 0, sp, sp > 1 ? ws.data_ptr<float>() : nullptr,
                    nullptr, cur_stream());
}

// Segmented-K split-product GEMM (gemm2.hip launch_gemm2_seg): C = Σ_s A[s] · B[s] over three K segments of the bf16
// hi / lo halves (same shapes and strides within A and within B). la = 0: NT, A [M][K], B [N][K] (lb 0) or [K][N]
// (lb 1), C [M][N] fp32 written; la = lb = 1: TT weight gradient, A [T][M], B [T][N], C [M][N] fp32 accumulated.
void gemm2_seg(std::vector<torch::Tensor> A, std::vector<torch::Tensor> B, torch::Tensor C, int64_t la, int64_t lb,
               bool accumulate) {
  TORCH_CHECK(A.size() == 3 && B.size() == 3, "gemm2_seg: three A and three B segments");
  for (int s = 0; s < 3; ++s) {
    TORCH_CHECK(A[s].is_cuda() && B[s].is_cuda() && A[s].scalar_type() == torch::kBFloat16 &&
                B[s].scalar_type() == torch::kBFloat16 && A[s].dim() == 2 && B[s].dim() == 2 &&
                A[s].stride(1) == 1 && B[s].stride(1) == 1, "gemm2_seg: 2-D bf16 GPU segments, unit inner stride");
    TORCH_CHECK(A[s].sizes() == A[0].sizes() && A[s].stride(0) == A[0].stride(0) && B[s].sizes() == B[0].sizes() &&
                B[s].stride(0) == B[0].stride(0), "gemm2_seg: segments of one operand share shape and stride");
  }
  check_f32(C, "C");
  TORCH_CHECK(C.dim() == 2 && (la == 0 ? (lb == 0 || lb == 1) : lb == 1), "gemm2_seg layouts: (0,0), (0,1), (1,1)");
  const int64_t M = la == 0 ? A[0].size(0) : A[0].size(1);
  const int64_t Kseg = la == 0 ? A[0].size(1) : A[0].size(0);
  const int64_t N = lb == 0 ? B[0].size(0) : B[0].size(1);
  const int64_t KB = lb == 0 ? B[0].size(1) : B[0].size(0);
  TORCH_CHECK(Kseg == KB && C.size(0) == M && C.size(1) == N, "gemm2_seg shapes");
  TORCH_CHECK(hsd::gemm2_seg_supported((int)la, (int)lb, (int)M, (int)N, (int)Kseg), "gemm2_seg: unsupported shape");
  TORCH_CHECK(A[0].stride(0) % 8 == 0 && B[0].stride(0) % 8 == 0, "gemm2_seg leading dims alignment");
  const int64_t wsn = hsd::gemm2_seg_ws_numel((int)la, (int)lb, (int)M, (int)N, (int)Kseg);
  torch::Tensor ws;
  if (wsn > 0) ws = torch::empty({wsn}, C.options());  // K-split slabs (stream-ordered pool)
  const hsd::bf16_t* a[3] = {CBF(A[0]), CBF(A[1]), CBF(A[2])};
  const hsd::bf16_t* b[3] = {CBF(B[0]), CBF(B[1]), CBF(B[2])};
  hsd::launch_gemm2_seg((int)la, (int)lb, a, A[0].stride(0), b, B[0].stride(0), (int)M, (int)N, (int)Kseg,
                        C.data_ptr<float>(), C.stride(0), wsn > 0 ? ws.data_ptr<float>() : nullptr, cur_stream(),
                        accumulate);
}

bool gemm2_seg_supported(int64_t la, int64_t lb, int64_t M, int64_t N, int64_t Kseg) {
  return hsd::gemm2_seg_supported((int)la, (int)lb, (int)M, (int)N, (int)Kseg);
}

void split3(torch::Tensor x, torch::Tensor out, int64_t pat, bool rows) {
  check_f32(x, "x"); check_bf16(out, "out");
  TORCH_CHECK(x.dim() == 2 && x.size(1) % 4 == 0 && out.numel() == 3 * x.numel(), "split3 shapes");
  TORCH_CHECK(rows ? (out.size(0) == 3 * x.size(0) && out.size(1) == x.size(1))
                   : (out.size(0) == x.size(0) && out.size(1) == 3 * x.size(1)), "split3 out shape");
  hsd::launch_split3(x.data_ptr<float>(), BF(out), x.size(0), x.size(1), (int)pat, rows, cur_stream());
}

// both layouts from one read: out_cols [R][3C] (pattern pat_cols) and out_rows [3R][C] (pattern pat_rows)
void split3_dual(torch::Tensor x, torch::Tensor out_cols, int64_t pat_cols, torch::Tensor out_rows, int64_t pat_rows) {
  check_f32(x, "x"); check_bf16(out_cols, "out_cols"); check_bf16(out_rows, "out_rows");
  TORCH_CHECK(x.dim() == 2 && x.size(1) % 4 == 0, "split3_dual x");
  TORCH_CHECK(out_cols.size(0) == x.size(0) && out_cols.size(1) == 3 * x.size(1), "split3_dual out_cols shape");
  TORCH_CHECK(out_rows.size(0) == 3 * x.size(0) && out_rows.size(1) == x.size(1), "split3_dual out_rows shape");
  hsd::launch_split3(x.data_ptr<float>(), BF(out_cols), x.size(0), x.size(1), (int)pat_cols, false, cur_stream(),
                     BF(out_rows), (int)pat_rows);
}

// optional bf16 halves of an fp32 output (hi = bf16(v), lo = bf16(v - hi)): both or neither, contiguous, numel n
static void check_halves(const c10::optional<torch::Tensor>& hi, const c10::optional<torch::Tensor>& lo, int64_t n) {
  TORCH_CHECK(hi.has_value() == lo.has_value(), "halves: hi and lo together");
  if (!hi.has_value()) return;
  check_bf16(*hi, "hi"); check_bf16(*lo, "lo");
  TORCH_CHECK(hi->numel() == n && lo->numel() == n, "halves: numel");
}

// out (optional with halves for kinds 0 / 1: the fp32 output is then not written), hi / lo: out's bf16 halves
void epi32(torch::Tensor y, c10::optional<torch::Tensor> bias, c10::optional<torch::Tensor> aux,
           c10::optional<torch::Tensor> out, int64_t kind, double p, int64_t seed, c10::optional<torch::Tensor> hi,
           c10::optional<torch::Tensor> lo) {
  check_f32(y, "y");
  if (out.has_value()) { check_f32(*out, "out"); TORCH_CHECK(y.sizes() == out->sizes(), "epi32 out shape"); }
  TORCH_CHECK(out.has_value() || (hi.has_value() && kind <= 1), "epi32: out needed");
  TORCH_CHECK(y.dim() == 2 && y.size(1) % 4 == 0, "epi32 shapes");
  check_halves(hi, lo, y.numel());
  if (bias.has_value()) { check_f32(*bias, "bias"); TORCH_CHECK(bias->numel() == y.size(1), "epi32 bias"); }
  if (kind >= 2) { TORCH_CHECK(aux.has_value(), "epi32 aux"); check_f32(*aux, "aux"); TORCH_CHECK(aux->sizes() == y.sizes(), "aux"); }
  hsd::launch_epi32(y.data_ptr<float>(), OPT_F(bias), OPT_F(aux), OPT_F(out), y.size(0), (int)y.size(1), (int)kind,
                    p, (uint64_t)seed, cur_stream(), OPT_BF(hi), OPT_BF(lo));
}

void dropout32(torch::Tensor x, torch::Tensor out, double p, int64_t seed, c10::optional<torch::Tensor> hi,
               c10::optional<torch::Tensor> lo) {
  check_f32(x, "x"); check_f32(out, "out");
  const int64_t W = x.dim() ? x.size(-1) : 1;
  TORCH_CHECK(x.numel() == out.numel() && W % 4 == 0, "dropout32 sizes");
  check_halves(hi, lo, x.numel());
  hsd::launch_dropout32(x.data_ptr<float>(), out.data_ptr<float>(), x.numel(), (int)W, p, (uint64_t)seed, cur_stream(),
                        OPT_BF(hi), OPT_BF(lo));
}

void colsum32(torch::Tensor x, torch::Tensor dbias) {
  check_f32(x, "x"); check_f32(dbias, "dbias");
  TORCH_CHECK(x.dim() == 2 && dbias.numel() == x.size(1), "colsum32 shapes");
  hsd::launch_colsum32(x.data_ptr<float>(), dbias.data_ptr<float>(), (int)x.size(0), (int)x.size(1), cur_stream());
}

void ln32_fwd(torch::Tensor x, torch::Tensor g, torch::Tensor b, torch::Tensor out, torch::Tensor mean,
              torch::Tensor rstd, double eps, c10::optional<torch::Tensor> hi, c10::optional<torch::Tensor> lo) {
  check_f32(x, "x"); check_f32(g, "g"); check_f32(b, "b"); check_f32(out, "out"); check_f32(mean, "mean");
  check_f32(rstd, "rstd");
  const int64_t R = x.size(0), H = x.size(1);
  TORCH_CHECK(x.dim() == 2 && H % 4 == 0 && H <= 1024 && g.numel() == H && b.numel() == H && mean.numel() == R &&
              rstd.numel() == R && out.sizes() == x.sizes(), "ln32_fwd shapes");
  check_halves(hi, lo, x.numel());
  hsd::launch_ln32_fwd(x.data_ptr<float>(), g.data_ptr<float>(), b.data_ptr<float>(), out.data_ptr<float>(),
                       mean.data_ptr<float>(), rstd.data_ptr<float>(), (int)R, (int)H, (float)eps, cur_stream(),
                       OPT_BF(hi), OPT_BF(lo));
}

void ln32_bwd(torch::Tensor dy, torch::Tensor x, torch::Tensor mean, torch::Tensor rstd, torch::Tensor g,
              torch::Tensor dx, torch::Tensor dg, torch::Tensor db) {
  check_f32(dy, "dy"); check_f32(x, "x"); check_f32(mean, "mean"); check_f32(rstd, "rstd"); check_f32(g, "g");
  check_f32(dx, "dx"); check_f32(dg, "dg"); check_f32(db, "db");
  const int64_t R = x.size(0), H = x.size(1);
  TORCH_CHECK(dy.sizes() == x.sizes() && dx.sizes() == x.sizes() && H % 4 == 0 && H <= 1024 && dg.numel() == H &&
              db.numel() == H && mean.numel() == R, "ln32_bwd shapes");
  hsd::launch_ln32_bwd(dy.data_ptr<float>(), x.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                       g.data_ptr<float>(), dx.data_ptr<float>(), dg.data_ptr<float>(), db.data_ptr<float>(), (int)R,
                       (int)H, cur_stream());
}

void embed32_gather(torch::Tensor ids, torch::Tensor pids, c10::optional<torch::Tensor> tids, torch::Tensor word,
                    torch::Tensor pos, c10::optional<torch::Tensor> type, torch::Tensor x) {
  CHECK_DTYPE(ids, torch::kInt64); CHECK_DTYPE(pids, torch::kInt64); CHECK_CONTIG(ids); CHECK_CONTIG(pids);
  check_f32(word, "word"); check_f32(pos, "pos"); check_f32(x, "x");
  const int64_t R = ids.numel(), H = word.size(1);
  TORCH_CHECK(pids.numel() == R && x.size(0) == R && x.size(1) == H && pos.size(1) == H && H % 4 == 0, "embed32 shapes");
  if (tids.has_value()) { CHECK_DTYPE(*tids, torch::kInt64); CHECK_CONTIG(*tids); TORCH_CHECK(tids->numel() == R, "tids"); }
  if (type.has_value()) check_f32(*type, "type");
  hsd::launch_embed32_gather(ids.data_ptr<int64_t>(), pids.data_ptr<int64_t>(), OPT_I64(tids), word.data_ptr<float>(),
                             pos.data_ptr<float>(), OPT_F(type), x.data_ptr<float>(), (int)R, (int)H, cur_stream());
}

void embed32_scatter(torch::Tensor dx, torch::Tensor ids, torch::Tensor pids, c10::optional<torch::Tensor> tids,
                     torch::Tensor gword, c10::optional<torch::Tensor> gpos, c10::optional<torch::Tensor> gtype) {
  check_f32(dx, "dx"); check_f32(gword, "gword");
  CHECK_DTYPE(ids, torch::kInt64); CHECK_DTYPE(pids, torch::kInt64);
  const int64_t R = ids.numel(), H = dx.size(1);
  TORCH_CHECK(dx.size(0) == R && gword.size(1) == H, "embed32_scatter shapes");
  if (gpos.has_value()) check_f32(*gpos, "gpos");
  if (gtype.has_value()) check_f32(*gtype, "gtype");
  hsd::launch_embed32_scatter(dx.data_ptr<float>(), ids.data_ptr<int64_t>(), pids.data_ptr<int64_t>(), OPT_I64(tids),
                              gword.data_ptr<float>(), OPT_F(gpos), OPT_F(gtype), (int)R, (int)H, cur_stream());
}

void attn32_fwd(torch::Tensor qkv, c10::optional<torch::Tensor> mask, torch::Tensor out, torch::Tensor lse, int64_t B,
                int64_t S, int64_t heads, double p, int64_t seed) {
  check_f32(qkv, "qkv"); check_f32(out, "out"); check_f32(lse, "lse");
  TORCH_CHECK(qkv.size(0) == B * S && qkv.size(1) == 3 * heads * 64 && out.size(0) == B * S &&
              out.size(1) == heads * 64 && lse.numel() == B * heads * S && S % 2 == 0, "attn32_fwd shapes (head dim 64)");
  if (mask.has_value()) { check_f32(*mask, "mask"); TORCH_CHECK(mask->numel() == B * S, "mask"); }
  hsd::launch_attn32_fwd(qkv.data_ptr<float>(), OPT_F(mask), out.data_ptr<float>(), lse.data_ptr<float>(), (int)B,
                         (int)S, (int)heads, p, (uint64_t)seed, cur_stream());
}

void attn32_bwd(torch::Tensor qkv, c10::optional<torch::Tensor> mask, torch::Tensor o, torch::Tensor dout,
                torch::Tensor lse, torch::Tensor dqkv, torch::Tensor delta, int64_t B, int64_t S, int64_t heads, double p,
                int64_t seed) {
  check_f32(qkv, "qkv"); check_f32(o, "o"); check_f32(dout, "dout"); check_f32(lse, "lse"); check_f32(dqkv, "dqkv");
  check_f32(delta, "delta");
  TORCH_CHECK(qkv.sizes() == dqkv.sizes() && o.sizes() == dout.sizes() && o.size(0) == B * S &&
              o.size(1) == heads * 64 && lse.numel() == B * heads * S && delta.numel() >= B * heads * S, "attn32_bwd shapes");
  if (mask.has_value()) { check_f32(*mask, "mask"); TORCH_CHECK(mask->numel() == B * S, "mask"); }
  hsd::launch_attn32_bwd(qkv.data_ptr<float>(), OPT_F(mask), o.data_ptr<float>(), dout.data_ptr<float>(),
                         lse.data_ptr<float>(), dqkv.data_ptr<float>(), delta.data_ptr<float>(), (int)B, (int)S,
                         (int)heads, p, (uint64_t)seed, cur_stream());
}

// fp32 attention on split bf16 MFMA products (attention32m.hip): qkv / dout carried as hi + lo bf16 pairs
void split2(torch::Tensor x, torch::Tensor hi, torch::Tensor lo) {
  check_f32(x, "x"); check_bf16(hi, "hi"); check_bf16(lo, "lo");
  TORCH_CHECK(x.numel() == hi.numel() && x.numel() == lo.numel() && x.numel() % 4 == 0, "split2 sizes");
  hsd::launch_split2(x.data_ptr<float>(), BF(hi), BF(lo), x.numel(), cur_stream());
}

void attn32m_fwd(torch::Tensor qh, torch::Tensor ql, c10::optional<torch::Tensor> mask, torch::Tensor out,
                 torch::Tensor lse, int64_t B, int64_t S, int64_t heads, double p, int64_t seed) {
  check_bf16(qh, "qkv_hi"); check_bf16(ql, "qkv_lo"); check_f32(out, "out"); check_f32(lse, "lse");
  TORCH_CHECK(hsd::attn32m_supported((int)S, 64), "attn32m_fwd: S must be a multiple of 128 in [128, 1024]");
  TORCH_CHECK(qh.sizes() == ql.sizes() && qh.size(0) == B * S && qh.size(1) == 3 * heads * 64 && out.size(0) == B * S &&
              out.size(1) == heads * 64 && lse.numel() == B * heads * S, "attn32m_fwd shapes (head dim 64)");
  if (mask.has_value()) { check_f32(*mask, "mask"); TORCH_CHECK(mask->numel() == B * S, "mask"); }
  hsd::launch_attn32m_fwd(CBF(qh), CBF(ql), OPT_F(mask), out.data_ptr<float>(), lse.data_ptr<float>(), (int)B, (int)S,
                          (int)heads, p, (uint64_t)seed, cur_stream());
}

void attn32m_bwd(torch::Tensor qh, torch::Tensor ql, torch::Tensor doh, torch::Tensor dol,
                 c10::optional<torch::Tensor> mask, torch::Tensor o, torch::Tensor dout, torch::Tensor lse,
                 torch::Tensor dqkv, torch::Tensor delta, int64_t B, int64_t S, int64_t heads, double p, int64_t seed) {
  check_bf16(qh, "qkv_hi"); check_bf16(ql, "qkv_lo"); check_bf16(doh, "dout_hi"); check_bf16(dol, "dout_lo");
  check_f32(o, "o"); check_f32(dout, "dout"); check_f32(lse, "lse"); check_f32(dqkv, "dqkv"); check_f32(delta, "delta");
  TORCH_CHECK(hsd::attn32m_supported((int)S, 64), "attn32m_bwd: S must be a multiple of 128 in [128, 1024]");
  TORCH_CHECK(qh.sizes() == ql.sizes() && qh.sizes() == dqkv.sizes() && doh.sizes() == dol.sizes() &&
              doh.sizes() == o.sizes() && o.sizes() == dout.sizes() && o.size(0) == B * S && o.size(1) == heads * 64 &&
              lse.numel() == B * heads * S && delta.numel() >= B * heads * S, "attn32m_bwd shapes");
  if (mask.has_value()) { check_f32(*mask, "mask"); TORCH_CHECK(mask->numel() == B * S, "mask"); }
  hsd::launch_attn32_delta(o.data_ptr<float>(), dout.data_ptr<float>(), delta.data_ptr<float>(), (int)B, (int)S,
                           (int)heads, cur_stream());
  hsd::launch_attn32m_bwd(CBF(qh), CBF(ql), CBF(doh), CBF(dol), OPT_F(mask), lse.data_ptr<float>(),
                          delta.data_ptr<float>(), dqkv.data_ptr<float>(), (int)B, (int)S, (int)heads, p,
                          (uint64_t)seed, cur_stream());
}

void cls32_fwd(torch::Tensor pre, torch::Tensor W2, torch::Tensor b2, torch::Tensor labels, torch::Tensor t_out,
               torch::Tensor logits, torch::Tensor stats, int64_t act, double p, int64_t seed) {
  check_f32(pre, "pre"); check_f32(W2, "W2"); check_f32(b2, "b2"); check_f32(t_out, "t_out"); check_f32(logits, "logits");
  check_f32(stats, "stats"); CHECK_DTYPE(labels, torch::kInt64); CHECK_CONTIG(labels);
  const int64_t R = pre.size(0), H = pre.size(1), C = W2.size(0);
  TORCH_CHECK(W2.size(1) == H && b2.numel() == C && C <= 8 && labels.numel() == R && t_out.sizes() == pre.sizes() &&
              logits.size(0) == R && logits.size(1) == C && stats.numel() >= 2 && H % 2 == 0, "cls32_fwd shapes");
  hsd::launch_cls32_fwd(pre.data_ptr<float>(), W2.data_ptr<float>(), b2.data_ptr<float>(), labels.data_ptr<int64_t>(),
                        t_out.data_ptr<float>(), logits.data_ptr<float>(), stats.data_ptr<float>(), (int)R, (int)H,
                        (int)C, (int)act, p, (uint64_t)seed, cur_stream());
}

void cls32_bwd(torch::Tensor pre, torch::Tensor t, torch::Tensor W2, torch::Tensor logits, torch::Tensor labels,
               torch::Tensor dloss, torch::Tensor dpre, torch::Tensor dW2, torch::Tensor db2, int64_t act, double p,
               int64_t seed) {
  check_f32(pre, "pre"); check_f32(t, "t"); check_f32(W2, "W2"); check_f32(logits, "logits"); check_f32(dloss, "dloss");
  check_f32(dpre, "dpre"); check_f32(dW2, "dW2"); check_f32(db2, "db2");
  const int64_t R = pre.size(0), H = pre.size(1), C = W2.size(0);
  TORCH_CHECK(dpre.sizes() == pre.sizes() && dW2.sizes() == W2.sizes() && db2.numel() == C && C <= 8, "cls32_bwd shapes");
  hsd::launch_cls32_bwd(pre.data_ptr<float>(), t.data_ptr<float>(), W2.data_ptr<float>(), logits.data_ptr<float>(),
                        labels.data_ptr<int64_t>(), dloss.data_ptr<float>(), dpre.data_ptr<float>(),
                        dW2.data_ptr<float>(), db2.data_ptr<float>(), (int)R, (int)H, (int)C, (int)act, p,
                        (uint64_t)seed, cur_stream());
}

// gemm2 on an explicit stream (the weight-gradient side stream): no Python stream context per call
void gemm2_on(int64_t stream_ptr, torch::Tensor A, torch::Tensor B, torch::Tensor C, int64_t la, int64_t lb, int64_t epi,
              c10::optional<torch::Tensor> bias, c10::optional<torch::Tensor> aux, c10::optional<torch::Tensor> C2,
              double p, int64_t seed, int64_t splits, c10::optional<torch::Tensor> ws,
              c10::optional<torch::Tensor> dbias) {
  c10::hip::HIPStreamGuard guard(
      c10::hip::getStreamFromExternal(reinterpret_cast<hipStream_t>(stream_ptr), A.get_device()));
  gemm2(A, B, C, la, lb, epi, bias, aux, C2, p, seed, splits, ws, dbias, c10::nullopt, 0);
}

// logits [R, V] (bf16 | fp32), labels int64 [R] (-100 = ignore); stats fp32 [2] += {Σ loss, correct};
// dlogits (optional, same dtype/shape) = (softmax - onehot) / n_valid
// logits [rows][ld] (unit inner stride), the first V columns scored (V = 0: all); dlogits same shape / strides
void xent(torch::Tensor logits, torch::Tensor labels, c10::optional<torch::Tensor> dlogits, torch::Tensor stats,
          torch::Tensor n_valid, int64_t V) {
  TORCH_CHECK(logits.is_cuda() && logits.dim() == 2 && logits.stride(1) == 1, "xent logits");
  const bool bf = logits.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(bf || logits.scalar_type() == torch::kFloat32, "xent logits dtype");
  TORCH_CHECK(labels.scalar_type() == torch::kInt64 && labels.is_contiguous() && labels.numel() == logits.size(0),
              "xent labels");
  const int64_t ld = logits.size(0) > 1 ? logits.stride(0) : logits.size(1);
  TORCH_CHECK(ld == logits.size(1), "xent: rows must be dense (the padding is the columns beyond V)");
  if (V <= 0) V = logits.size(1);
  TORCH_CHECK(V <= logits.size(1), "xent V");
  check_f32(stats, "stats");
  check_f32(n_valid, "n_valid");
  TORCH_CHECK(stats.numel() >= 2 && n_valid.numel() == 1, "xent stats");
  void* dl = nullptr;
  if (dlogits.has_value()) {
    TORCH_CHECK(dlogits->sizes() == logits.sizes() && dlogits->scalar_type() == logits.scalar_type() &&
                dlogits->is_contiguous(), "xent dlogits");
    dl = dlogits->data_ptr();
  }
  hsd::launch_xent(logits.data_ptr(), bf, labels.data_ptr<int64_t>(), dl, stats.data_ptr<float>(),
                   n_valid.data_ptr<float>(), (int)logits.size(0), (int)V, ld, cur_stream());
}

// fused classification head (cls_head.hip). pre [R][H] bf16 (row stride ld), W2 [C][H], b2 [C] bf16, labels int64 [R]
// (or none: logits only); t_out [R][H], logits [R][C] bf16; partials fp32 [cls_head_blocks(R)][4]; stats fp32 [4]
void cls_head_fwd(torch::Tensor pre, torch::Tensor W2, torch::Tensor b2, c10::optional<torch::Tensor> labels,
                  torch::Tensor t_out, torch::Tensor logits, torch::Tensor partials, torch::Tensor stats, int64_t act,
                  double p, int64_t seed) {
  TORCH_CHECK(pre.is_cuda() && pre.dim() == 2 && pre.stride(1) == 1 && pre.stride(0) % 8 == 0 &&
              pre.scalar_type() == torch::kBFloat16, "cls_head pre");
  const int64_t R = pre.size(0), H = pre.size(1), C = W2.size(0);
  TORCH_CHECK(H % 8 == 0 && H <= 1024 && C >= 1 && C <= 4, "cls_head: H % 8 == 0, H <= 1024, 1 <= classes <= 4");
  TORCH_CHECK(W2.is_contiguous() && W2.size(1) == H && W2.scalar_type() == torch::kBFloat16, "cls_head W2");
  TORCH_CHECK(b2.is_contiguous() && b2.numel() == C && b2.scalar_type() == torch::kBFloat16, "cls_head b2");
  TORCH_CHECK(t_out.is_contiguous() && t_out.sizes() == pre.sizes() && t_out.scalar_type() == torch::kBFloat16, "cls t");
  TORCH_CHECK(logits.is_contiguous() && logits.size(0) == R && logits.size(1) == C &&
              logits.scalar_type() == torch::kBFloat16, "cls_head logits");
  check_f32(partials, "partials");
  check_f32(stats, "stats");
  TORCH_CHECK(partials.numel() >= 4 * (int64_t)hsd::cls_head_blocks((int)R) && stats.numel() >= 4, "cls_head stats");
  const int64_t* lab = nullptr;
  if (labels.has_value()) {
    TORCH_CHECK(labels->scalar_type() == torch::kInt64 && labels->is_contiguous() && labels->numel() == R, "labels");
    lab = labels->data_ptr<int64_t>();
  }
  TORCH_CHECK(act == 0 || act == 1, "cls_head act: 0 tanh, 1 relu");
  hsd::launch_cls_head_fwd(CBF(pre), pre.stride(0), CBF(W2), CBF(b2), lab, BF(t_out), BF(logits),
                           partials.data_ptr<float>(), stats.data_ptr<float>(), (int)R, (int)H, (int)C, (int)act, p,
                           (uint64_t)seed, cur_stream());
}

void cls_head_bwd(torch::Tensor t, torch::Tensor W2, torch::Tensor logits, torch::Tensor labels, torch::Tensor stats,
                  torch::Tensor dloss, torch::Tensor dpre, torch::Tensor dW2, torch::Tensor db2, int64_t act, double p,
                  int64_t seed) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.is_contiguous() && t.scalar_type() == torch::kBFloat16, "cls t");
  const int64_t R = t.size(0), H = t.size(1), C = W2.size(0);
  TORCH_CHECK(H % 8 == 0 && H <= 1024 && C >= 1 && C <= 4, "cls_head shape");
  TORCH_CHECK(W2.is_contiguous() && W2.size(1) == H && W2.scalar_type() == torch::kBFloat16, "cls_head W2");
  TORCH_CHECK(logits.is_contiguous() && logits.size(0) == R && logits.size(1) == C &&
              logits.scalar_type() == torch::kBFloat16, "cls_head logits");
  TORCH_CHECK(labels.scalar_type() == torch::kInt64 && labels.is_contiguous() && labels.numel() == R, "labels");
  check_f32(stats, "stats");
  check_f32(dloss, "dloss");
  TORCH_CHECK(dpre.is_contiguous() && dpre.sizes() == t.sizes() && dpre.scalar_type() == torch::kBFloat16, "dpre");
  check_f32(dW2, "dW2");
  check_f32(db2, "db2");
  TORCH_CHECK(dW2.numel() == C * H && db2.numel() == C, "cls_head grads");
  hsd::launch_cls_head_bwd(CBF(t), CBF(W2), CBF(logits), labels.data_ptr<int64_t>(), stats.data_ptr<float>(),
                           dloss.data_ptr<float>(), BF(dpre), dW2.data_ptr<float>(), db2.data_ptr<float>(), (int)R,
                           (int)H, (int)C, (int)act, p, (uint64_t)seed, cur_stream());
}

// C [N][K] fp32 += dy [T][N]ᵀ · x [T][K] for small T (row strides allowed; unit inner strides)
void small_wgrad(torch::Tensor dy, torch::Tensor x, torch::Tensor C) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0), "small_wgrad");
  TORCH_CHECK(dy.scalar_type() == torch::kBFloat16 && x.scalar_type() == torch::kBFloat16 && dy.stride(1) == 1 &&
              x.stride(1) == 1 && x.stride(0) % 4 == 0, "small_wgrad inputs");
  TORCH_CHECK(C.scalar_type() == torch::kFloat32 && C.dim() == 2 && C.size(0) == dy.size(1) && C.size(1) == x.size(1) &&
              C.stride(1) == 1 && C.stride(0) % 4 == 0 && x.size(1) % 4 == 0, "small_wgrad C");
  hsd::launch_small_wgrad(CBF(dy), dy.stride(0), CBF(x), x.stride(0), C.data_ptr<float>(), C.stride(0),
                          (int)dy.size(0), (int)dy.size(1), (int)x.size(1), cur_stream());
}

void mask_bias(torch::Tensor mask, torch::Tensor out) {
  TORCH_CHECK(mask.is_cuda() && mask.is_contiguous() &&
              (mask.scalar_type() == torch::kInt64 || mask.scalar_type() == torch::kInt32), "mask_bias mask");
  check_f32(out, "mask_bias out");
  TORCH_CHECK(out.numel() == mask.numel(), "mask_bias shape");
  hsd::launch_mask_bias(mask.data_ptr(), mask.scalar_type() == torch::kInt64, out.data_ptr<float>(), mask.numel(),
                        cur_stream());
}

int64_t cls_head_blocks(int64_t R) { return hsd::cls_head_blocks((int)R); }

// stream-ordered zero fill (hipMemsetAsync): gradient buffers and scatter targets without an at::native fill kernel
void memset0(torch::Tensor x) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "memset0: contiguous GPU tensor");
  const auto err = hipMemsetAsync(x.data_ptr(), 0, x.numel() * x.element_size(), cur_stream());
  TORCH_CHECK(err == hipSuccess, "hipMemsetAsync failed");
}

void transpose_many(torch::Tensor desc, int64_t total_tiles) {
  TORCH_CHECK(desc.is_cuda() && desc.scalar_type() == torch::kInt64 && desc.dim() == 2 && desc.size(1) == 5 &&
              desc.is_contiguous(), "transpose_many: int64 [n, 5] device descriptor table");
  hsd::launch_transpose_many(desc.data_ptr<int64_t>(), (int)desc.size(0), (int)total_tiles, cur_stream());
}

int64_t gemm2_splits(int64_t M, int64_t N, int64_t K) { return hsd::gemm2_wgrad_splits((int)M, (int)N, (int)K); }
int64_t gemm2_nt_splits(int64_t M, int64_t N, int64_t K) { return hsd::gemm2_nt_splits((int)M, (int)N, (int)K); }
void attn128_set_diag(c10::optional<at::Tensor> buf) {
  hsd::attn128_set_diag(buf.has_value() ? buf->data_ptr() : nullptr);
}
void gemm2_set_diag(c10::optional<at::Tensor> buf) {
  hsd::gemm2_set_diag(buf.has_value() ? buf->data_ptr() : nullptr);
}

bool gemm2_supported(int64_t la, int64_t lb, int64_t epi, int64_t M, int64_t N, int64_t K) {
  return hsd::gemm2_supported((int)la, (int)lb, (int)epi, (int)M, (int)N, (int)K);
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 HIP kernels for huggingface_sagemaker_tensorflow_distributed_amd";
  hsd::register_comm(m);
  m.def("adam_step", &adam_step, py::arg("p"), py::arg("m"), py::arg("v"), py::arg("g"), py::arg("out"),
        py::arg("decay"), py::arg("step"), py::arg("eps"), py::arg("b1"), py::arg("b2"), py::arg("gscale"),
        py::arg("lr_wd"), py::arg("coef") = py::none(), py::arg("out_lo") = py::none(), py::arg("zero_grad") = false);
  m.def("ln_fwd_q8", &ln_fwd_q8);
  m.def("stream_wait", &stream_wait);
  m.def("gemm2_on", &gemm2_on);
  m.def("ln_bwd_q8", &ln_bwd_q8, py::arg("dout"), py::arg("z"), py::arg("mean"), py::arg("rstd"), py::arg("gamma"),
        py::arg("dz"), py::arg("dy"), py::arg("dgamma"), py::arg("dbeta"), py::arg("dbias"), py::arg("p"),
        py::arg("seed"), py::arg("q8"), py::arg("amax_in"), py::arg("sinv"), py::arg("amax_track"), py::arg("qfmt"),
        py::arg("q8_only") = false);
  m.def("attn_fwd_q8", &attn_fwd_q8, py::arg("qkv"), py::arg("mask"), py::arg("out"), py::arg("lse2"), py::arg("B"),
        py::arg("S"), py::arg("heads"), py::arg("p"), py::arg("seed"), py::arg("q8"), py::arg("amax_in"),
        py::arg("sinv"), py::arg("amax_track"), py::arg("kmask") = py::none());
  m.def("attn_bwd_q8", &attn_bwd_q8, py::arg("qkv"), py::arg("mask"), py::arg("o"), py::arg("dout"), py::arg("lse2"),
        py::arg("dqkv"), py::arg("ws"), py::arg("B"), py::arg("S"), py::arg("heads"), py::arg("p"), py::arg("seed"),
        py::arg("dbias"), py::arg("q8"), py::arg("amax_in"), py::arg("sinv"), py::arg("amax_track"), py::arg("qfmt"),
        py::arg("kmask") = py::none(), py::arg("delta_ready") = false, py::arg("q8_only") = false);
  m.def("attn_q8_supported", [](int64_t S) { return S > 128 && hsd::attn_streaming((int)S); });
  m.def("ln_fwd", &ln_fwd);
  m.def("ln_bwd", &ln_bwd);
  m.def("embed_fwd", &embed_fwd, py::arg("ids"), py::arg("pos_ids"), py::arg("type_ids"), py::arg("word"),
        py::arg("pos"), py::arg("type"), py::arg("gamma"), py::arg("beta"), py::arg("out"), py::arg("mean"),
        py::arg("rstd"), py::arg("eps"), py::arg("p"), py::arg("seed"), py::arg("q8") = py::none(),
        py::arg("amax_in") = py::none(), py::arg("sinv") = py::none(), py::arg("amax_track") = py::none());
  m.def("embed_bwd", &embed_bwd);
  m.def("gelu_fwd", &gelu_fwd);
  m.def("gelu_bwd_colsum", &gelu_bwd_colsum);
  m.def("colsum", &colsum);
  m.def("dropout", &dropout);
  m.def("set_dropout_device_seed", &set_dropout_device_seed);
  m.def("cu_hog", [](int64_t blocks, double usec) { hsd::launch_cu_hog((int)blocks, usec, cur_stream()); },
        "contention emulation: hold `blocks` whole CUs for `usec` us on the current stream");
  m.def("gemm2_f32nt", &gemm2_f32nt);
  m.def("gemm2_seg", &gemm2_seg, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("la"), py::arg("lb"),
        py::arg("accumulate") = false);
  m.def("gemm2_seg_supported", &gemm2_seg_supported);
  m.def("split3", &split3);
  m.def("split3_dual", &split3_dual);
  m.def("epi32", &epi32, py::arg("y"), py::arg("bias"), py::arg("aux"), py::arg("out"), py::arg("kind"), py::arg("p"),
        py::arg("seed"), py::arg("hi") = py::none(), py::arg("lo") = py::none());
  m.def("dropout32", &dropout32, py::arg("x"), py::arg("out"), py::arg("p"), py::arg("seed"),
        py::arg("hi") = py::none(), py::arg("lo") = py::none());
  m.def("colsum32", &colsum32);
  m.def("ln32_fwd", &ln32_fwd, py::arg("x"), py::arg("g"), py::arg("b"), py::arg("out"), py::arg("mean"),
        py::arg("rstd"), py::arg("eps"), py::arg("hi") = py::none(), py::arg("lo") = py::none());
  m.def("ln32_bwd", &ln32_bwd);
  m.def("embed32_gather", &embed32_gather);
  m.def("embed32_scatter", &embed32_scatter);
  m.def("attn32_fwd", &attn32_fwd);
  m.def("attn32_bwd", &attn32_bwd);
  m.def("split2", &split2);
  m.def("attn32m_supported", [](int64_t S) { return hsd::attn32m_supported((int)S, 64); });
  m.def("attn32m_fwd", &attn32m_fwd);
  m.def("attn32m_bwd", &attn32m_bwd);
  m.def("cls32_fwd", &cls32_fwd);
  m.def("cls32_bwd", &cls32_bwd);
  m.def("refresh_env", &hsd::refresh_env_knobs, "re-read the HSD_* launch knobs (cached per generation)");
  // the kernels' dropout mask definition evaluated on the host (common.h): tests pin ops/rng.py to it bit for bit
  m.def("dropout_pair_bits", [](int64_t seed, int64_t row, int64_t cp) -> int64_t {
    return (int64_t)hsd::dropout_pair_bits_host((uint64_t)seed, (uint32_t)row, (uint32_t)cp);
  });
  m.def("fp8_quant", &fp8_quant, py::arg("x"), py::arg("amax"), py::arg("q"), py::arg("sinv"), py::arg("fmt"),
        py::arg("compute_amax"), py::arg("amax_track") = py::none());
  m.def("fp8_quant_many", &fp8_quant_many);
  m.def("fp8_elems_per_block", &hsd::fp8_elems_per_block);
  m.def("gemm8", &gemm8, py::arg("A"), py::arg("fa"), py::arg("sa"), py::arg("B"), py::arg("fb"), py::arg("sb"),
        py::arg("C"), py::arg("epi"), py::arg("bias") = py::none(), py::arg("aux") = py::none(),
        py::arg("C2") = py::none(), py::arg("p") = 0.0, py::arg("seed") = 0, py::arg("dbias") = py::none(),
        py::arg("q8") = py::none(), py::arg("q8_amax") = py::none(),
        py::arg("q8_sinv") = py::none(), py::arg("q8_track") = py::none(), py::arg("q8fmt") = 0,
        py::arg("rd") = py::none(), py::arg("rd_seq") = 0, py::arg("q8_only") = false);
  m.def("gemm8_supported", &hsd::gemm8_supported);
  m.def("attn_fwd", &attn_fwd, py::arg("qkv"), py::arg("mask"), py::arg("out"), py::arg("lse2"), py::arg("B"),
        py::arg("S"), py::arg("heads"), py::arg("p"), py::arg("seed"), py::arg("kmask") = py::none());
  m.def("attn_keep_mask_supported", &hsd::attn_keep_mask_supported);
  m.def("attn_keep_mask_numel", &hsd::attn_keep_mask_numel);
  // backward workspace for S > 128: (numel, must_be_zeroed)
  m.def("attn_bwd_ws", [](int64_t B, int64_t S, int64_t heads) {
    if (S <= 128) return std::make_pair<int64_t, bool>(0, false);
    if (hsd::attn_streaming((int)S)) return std::make_pair<int64_t, bool>(B * heads * S, false);
    return std::make_pair<int64_t, bool>(B * S * heads * 64, true);
  });
  m.def("attn_bwd", &attn_bwd, py::arg("qkv"), py::arg("mask"), py::arg("o"), py::arg("dout"), py::arg("lse2"),
        py::arg("dqkv"), py::arg("dq_acc"), py::arg("B"), py::arg("S"), py::arg("heads"), py::arg("p"), py::arg("seed"),
        py::arg("dbias") = py::none(), py::arg("kmask") = py::none(), py::arg("delta_ready") = false);
  m.def("gemm", &gemm);
  m.def("gemm2", &gemm2, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("la"), py::arg("lb"), py::arg("epi"),
        py::arg("bias"), py::arg("aux"), py::arg("C2"), py::arg("p"), py::arg("seed"), py::arg("splits"), py::arg("ws"),
        py::arg("dbias"), py::arg("rd") = py::none(), py::arg("rd_seq") = 0);
  m.def("gemm2_splits", &gemm2_splits);
  m.def("gemm8_wgrad", &gemm8_wgrad);
  m.def("gemm8_wgrad_supported", [](int64_t M, int64_t N, int64_t T) {
    return hsd::gemm8_wgrad_supported((int)M, (int)N, (int)T);
  });
  m.def("gemm8_wgrad_ws_numel", [](int64_t M, int64_t N, int64_t T, int64_t splits) {
    return hsd::gemm8_wgrad_ws_numel((int)M, (int)N, (int)T, (int)splits);
  });
  m.def("gemm2_nt_splits", &gemm2_nt_splits);
  m.def("gemm2_supported", &gemm2_supported);
  m.def("gemm2_set_diag", &gemm2_set_diag);
  m.def("attn128_set_diag", &attn128_set_diag);
  m.def("attn_set_force_generic", &hsd::attn_set_force_generic);
  m.def("transpose_many", &transpose_many);
  m.def("xent", &xent, py::arg("logits"), py::arg("labels"), py::arg("dlogits"), py::arg("stats"),
        py::arg("n_valid"), py::arg("V") = 0);
  m.def("cls_head_fwd", &cls_head_fwd);
  m.def("cls_head_bwd", &cls_head_bwd);
  m.def("cls_head_blocks", &cls_head_blocks);
  m.def("memset0", &memset0);
  m.def("small_wgrad", &small_wgrad);
  m.def("mask_bias", &mask_bias);
}
