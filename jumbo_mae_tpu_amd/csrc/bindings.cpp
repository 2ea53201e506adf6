// PyTorch bindings of the jumbo_mae_tpu_amd HIP kernels.
// Kernels live in *.hip translation units with a plain pointer + hipStream_t interface; this file
// only validates tensors, allocates outputs with the caching allocator and launches on the
// current HIP stream (so everything is HIP-graph capturable).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include "jm_api.h"

// ---- kernel entry points (see *.hip)
int jm_layernorm_fwd(const float* x, long sB, long sT, int B, int T, int D, const float* gamma, const float* beta,
                     float eps, void* y, int out_bf16, float* mean, float* rstd, hipStream_t st, uint16_t* y2 = nullptr);
int jm_layernorm_bwd(const void* dy, int dy_bf16, const float* x, long sB, long sT, int B, int T, int D,
                     const float* mean, const float* rstd, const float* gamma, float* dx_ptr, long oB, long oT,
                     const float* dres, long rB, long rT, float* dgamma, float* dbeta, int accum_params, float* ws,
                     const JmLnRes* res, hipStream_t st, const uint16_t* hx = nullptr,
                     const float* beta = nullptr);
int jm_layernorm_bwd_blocks(int rows, int D);
// debug build (-DJM_DEBUG): first failing soft-check line per kernel translation unit (0 = none;
// reading clears it); always 0 in the release build
int jm_debug_line_attention();
int jm_debug_line_dropout();
int jm_debug_line_augment();
int jm_rrc_resize(const uint8_t* src, const int64_t* tab, int B, int S, uint8_t* tmp, int tmp_rows_max, uint8_t* out,
                  hipStream_t st);
int jm_rrc_kmax();
int jm_dropout_apply(const void* x, void* y, long n, int bf16, const int64_t* seed, uint32_t thr, float scale,
                     hipStream_t st);
int jm_gelu_drop(const uint16_t* h, uint16_t* g, uint16_t* gp, long n, const int64_t* seed, uint32_t thr, float scale,
                 hipStream_t st);
int jm_softmax_dropout_fwd(const float* z, float* p, float* pd, long rows, int S, const int64_t* seed, uint32_t thr,
                           float scale, hipStream_t st);
int jm_softmax_dropout_bwd(const float* dpd, const float* p, float* dz, long rows, int S, const int64_t* seed,
                           uint32_t thr, float scale, hipStream_t st);
int jm_debug_line_elementwise();
int jm_debug_line_gemm();
int jm_debug_line_gemm_tn();
int jm_debug_line_layernorm();
int jm_debug_line_mae();
int jm_debug_line_optim();
void jm_debug_selftest(int v, hipStream_t st);
int jm_residual_ln_fwd(const float* x, long sB, long sT, const uint16_t* y, const float* scale, const float* mask,
                       float* x1, long oB, long oT, uint16_t* h, float* mean, float* rstd, int B, int T, int T0,
                       int D, const float* gamma, const float* beta, float eps, hipStream_t st, int R0 = 0,
                       JmDrop drop = JmDrop{nullptr, 0u, 1.f, 0});
int jm_gelu_fwd(const uint16_t* h, uint16_t* a, long n, hipStream_t st);
long jm_rowcol_ws_floats(int M, int N, int nacc);
int jm_gelu_bwd(const uint16_t* h, const uint16_t* da, uint16_t* dh, float* bias_grad, int M, int N, hipStream_t st,
                int deriv, float* ws);
int jm_colsum_bf16(const uint16_t* x, float* acc, int M, int N, hipStream_t st, float* ws);
int jm_splitk_reduce_add(const float* part, float* g, long n, int S, hipStream_t st, int store = 0);
int jm_colsum_add_f32(const float* x, long ld, int rows, long n, float* g, hipStream_t st);
int jm_zero_ranges(float* base, const long long* desc, int n, long long blocks, hipStream_t st);
int jm_transpose_bf16(const uint16_t* src, uint16_t* dst, int R, int C, hipStream_t st);
int jm_transpose_bf16_batch(const long long* desc, int n, int tiles, hipStream_t st);
int jm_residual_fwd(const float* x, long sB, long sT, int B, int T, int D, const uint16_t* y, const float* scale,
                    const float* mask, float* out, long oB, long oT, hipStream_t st, JmDrop drop);
int jm_residual_bwd(const float* dout, long dB, long dT, const uint16_t* y, const float* scale, const float* mask,
                    float* dscale, uint16_t* dy, int B, int T, int D, float* dbias, long yB, long yT, hipStream_t st,
                    JmDrop drop, float* ws);
int jm_attn_fwd(const uint16_t* qkv, uint16_t* o, float* lse, int B, int S, int H, int hd, const int64_t* dseed,
                uint32_t dthr, float dscale, hipStream_t st);
int jm_attn_bwd(const uint16_t* qkv, const uint16_t* o, const uint16_t* dO, const float* lse, uint16_t* dqkv, int B,
                int S, int H, int hd, float* dbias_part, const int64_t* dseed, uint32_t dthr, float dscale,
                hipStream_t st);
int jm_attn_max_seq();
int jm_attn_bwd_part_rows(int B, int S, int hd);
int jm_attn_bwd_long(const uint16_t* qkv, const uint16_t* o, const uint16_t* dO, const float* lse, uint16_t* dqkv,
                     float* delta, int B, int S, int H, int hd, hipStream_t st);
void jm_opt_sumsq(const float* x, const int* chunks, int nchunks, float* out, float* cpart, hipStream_t st);
void jm_zero_f32(float* p, long n, hipStream_t st);
void jm_opt_adamw(float* p, const float* g, float* mu, float* nu, uint16_t* shadow, const int* chunks, int nchunks,
                  const float* meta, const float* hyper, const float* gnorm_sq, hipStream_t st);
void jm_opt_lamb_phase1(const float* p, const float* g, float* mu, float* nu, float* u, const int* chunks, int nchunks,
                        const float* meta, const float* hyper, const float* gnorm_sq, float* norms, float* cpart,
                        hipStream_t st);
void jm_opt_lars_norms(const float* p, const float* g, const int* chunks, int nchunks, const float* hyper,
                       const float* gnorm_sq, float* norms, float* cpart, hipStream_t st);
void jm_opt_apply_trust(float* p, const float* u_or_g, float* trace, uint16_t* shadow, const int* chunks, int nchunks,
                        const float* meta, const float* hyper, const float* norms, const float* gnorm_sq, int mode,
                        float momentum, float trust_coef, hipStream_t st);
void jm_opt_sgd(float* p, const float* g, float* trace, uint16_t* shadow, const int* chunks, int nchunks,
                const float* meta, const float* hyper, const float* gnorm_sq, float momentum, hipStream_t st);
int jm_splitk_reduce_bf16(const float* part, int S, long n, int N, const float* bias, uint16_t* out, hipStream_t st);
int jm_splitk_reduce_f32(const float* part, int S, int M, int N, const float* bias, const float* add, long add_ld,
                         float* out, hipStream_t st);
int jm_gemm_nt(const uint16_t* A, long lda, const uint16_t* B, long ldb, int M, int N, int K, int epi,
               const GemmEpi& ep, hipStream_t st);
int jm_gemm_nt_tiles(int M, int N, int K, int epi, long lda);
int jm_gemm_nt_colpart_rows(int M, int N, int K, int epi, long lda);
int jm_gemm_nt_tail_plan(int M, int N, int K, int epi, long lda, int* tail_r, long* ws_floats);
void jm_gemm_test_force(int path, int rows);
int jm_gemm_tn_plan(int M, int N, int K, int* S_out);
int jm_gemm_tn_group_plan(const TnGroup& grp, int M, int* S_out);
int jm_gemm_tn_group(TnGroup grp, int M, int sps, int S, hipStream_t st, int store);
int jm_gemm_tn(const uint16_t* A, long lda, const uint16_t* B, long ldb, int M, int N, int K, int sps, int S,
               float* G, long ldo, float* partial, hipStream_t st, int store);
struct TnSegs {  // gemm_tn.hip layout
  const uint16_t* a[64];
  const uint16_t* b[64];
  int rows;
  int n;
};
int jm_gemm_tn_group_seg(TnGroup grp, const TnSegs& segs, int sps, int S, hipStream_t st, int store);
int jm_gemm_tn_seg(const TnSegs& segs, long lda, long ldb, int N, int K, int sps, int S, float* G, long ldo,
                   float* partial, hipStream_t st, int store);
int jm_patchify_normalize(const uint8_t* img, float* out, int B, int H, int W, int p, hipStream_t st);
int jm_gather_patches(const uint8_t* img, const int* ids, long idsB, uint16_t* out, int B, int K, int H, int W, int p,
                      hipStream_t st);
int jm_embed_finish(const uint16_t* e, const float* pos, const int* ids, long idsB, const float* cls, float* out,
                    int B, int C, int K, int D, hipStream_t st);
int jm_mask_ids(const float* noise, int R, int N, int keep, int64_t* shuffle, int64_t* restore, int* keep32,
                int* restore32, float* mask, hipStream_t st);
int jm_unshuffle_fwd(const uint16_t* y, const float* tok, const int* restore, long rsB, const float* pos, float* out,
                     int B, int C, int K, int N, int d, hipStream_t st);
int jm_unshuffle_bwd_blocks(int B, int C, int N, int rows_per_block);
int jm_unshuffle_bwd(const float* dout, const int* restore, long rsB, uint16_t* dy, float* part, int B, int C, int K,
                     int N, int d, int rows_per_block, hipStream_t st);
int jm_mix_patches(const uint8_t* img, const int* perm, const float* prm, const int* box, uint16_t* out, int B, int H,
                   int W, int p, hipStream_t st);
int jm_patch_mse_fwd(const uint16_t* pred, long ldp, const uint8_t* img, float* mse, long rows, int N, int H, int W,
                     int p, int norm_pix, hipStream_t st);
int jm_patch_mse_bwd(const uint16_t* pred, long ldp, const uint8_t* img, const float* dmse, uint16_t* dpred, long rows,
                     int N, int H, int W, int p, int norm_pix, hipStream_t st);

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define CHECK_DT(x, d) TORCH_CHECK((x).scalar_type() == (d), #x " has wrong dtype")

const uint16_t* bf(const torch::Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
uint16_t* bfm(torch::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }
uint16_t* bfp(const torch::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }
const float* fopt(const c10::optional<torch::Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr;
}
float* fopt_m(c10::optional<torch::Tensor>& t) { return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr; }

void check_rc(int rc, const char* what) { TORCH_CHECK(rc == 0, what, ": unsupported shape (rc=", rc, ")"); }

// dropout: keep threshold on 16 hash bits (common.h drop_keep) and the 1/keep scale of a drop
// rate in [0, 1)
static std::pair<uint32_t, float> keep_params(double rate) {
  TORCH_CHECK(rate >= 0.0 && rate < 1.0, "dropout rate must be in [0, 1)");
  const double keep = 1.0 - rate;
  return {(uint32_t)std::llround(keep * 65536.0), (float)(1.0 / keep)};
}

static void check_seed(const torch::Tensor& seed, const torch::Tensor& like) {
  TORCH_CHECK(seed.scalar_type() == torch::kInt64 && seed.numel() == 1 && seed.device() == like.device(),
              "dropout seed: int64 [1] on the data's device");
}

// Dense-output dropout descriptor for the residual kernels: seed null / rate 0 = none; ioff = the
// element offset of y's view within the branch tensor the mask indexes
JmDrop make_drop(const c10::optional<torch::Tensor>& seed, double rate, const torch::Tensor& like, int64_t ioff) {
  if (!seed.has_value() || !seed->defined() || rate <= 0.0) return JmDrop{nullptr, 0u, 1.f, 0};
  check_seed(*seed, like);
  const auto kp = keep_params(rate);
  return JmDrop{seed->data_ptr<int64_t>(), kp.first, kp.second, (long)ioff};
}

// ------------------------------------------------------------------------------ layernorm
// also_bf16 (fp32 output only): a bf16 copy of y written by the same pass, returned 4th
std::vector<torch::Tensor> layernorm_fwd(torch::Tensor x, torch::Tensor gamma, torch::Tensor beta, double eps,
                                         py::object out_dtype, bool also_bf16) {
  CHECK_CUDA(x);
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1, "x must be [B,T,D] with contiguous last dim");
  CHECK_DT(x, torch::kFloat32);
  CHECK_CONTIG(gamma);
  CHECK_CONTIG(beta);
  const auto odt = torch::python::detail::py_object_to_dtype(out_dtype);
  const int B = x.size(0), T = x.size(1), D = x.size(2);
  auto y = torch::empty({(long)B * T, D}, x.options().dtype(odt));
  auto mean = torch::empty({(long)B * T}, x.options());
  auto rstd = torch::empty({(long)B * T}, x.options());
  TORCH_CHECK(odt == torch::kBFloat16 || odt == torch::kFloat32, "out dtype must be bf16/fp32");
  TORCH_CHECK(!also_bf16 || odt == torch::kFloat32, "also_bf16 needs an fp32 output");
  torch::Tensor y2;
  if (also_bf16) y2 = torch::empty({(long)B * T, D}, x.options().dtype(torch::kBFloat16));
  check_rc(jm_layernorm_fwd(x.data_ptr<float>(), x.stride(0), x.stride(1), B, T, D, gamma.data_ptr<float>(),
                            beta.data_ptr<float>(), (float)eps, y.data_ptr(), odt == torch::kBFloat16,
                            mean.data_ptr<float>(), rstd.data_ptr<float>(), stream(), also_bf16 ? bfm(y2) : nullptr),
           "layernorm_fwd");
  if (also_bf16) return {y, mean, rstd, y2};
  return {y, mean, rstd};
}

// res_*: optional fused residual backward of the consumer of dx (see JmLnRes); returns [dx] or
// [dx, dy_res] (dy_res written into res_out, a [B, T - T0, D] view, or a new [B*(T-T0), D] tensor)
std::vector<torch::Tensor> layernorm_bwd(torch::Tensor dy, torch::Tensor x, torch::Tensor mean, torch::Tensor rstd,
                                         torch::Tensor gamma, torch::Tensor dgamma, torch::Tensor dbeta, bool accum,
                                         c10::optional<torch::Tensor> dres, c10::optional<torch::Tensor> out,
                                         c10::optional<torch::Tensor> res_y, c10::optional<torch::Tensor> res_scale,
                                         c10::optional<torch::Tensor> res_mask, c10::optional<torch::Tensor> res_dscale,
                                         c10::optional<torch::Tensor> res_dbias, int64_t res_T0,
                                         c10::optional<torch::Tensor> res_out, c10::optional<torch::Tensor> res_seed,
                                         double res_rate, int64_t res_ioff, c10::optional<torch::Tensor> hx,
                                         c10::optional<torch::Tensor> beta) {
  CHECK_CONTIG(dy);
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1, "x must be [B,T,D]");
  const int B = x.size(0), T = x.size(1), D = x.size(2);
  TORCH_CHECK(dy.numel() == (long)B * T * D, "dy shape");
  torch::Tensor dx;
  if (out.has_value() && out->defined()) {
    dx = *out;
    TORCH_CHECK(dx.dim() == 3 && dx.size(0) == B && dx.size(1) == T && dx.size(2) == D && dx.stride(2) == 1, "out view");
  } else {
    dx = torch::empty({B, T, D}, x.options());
  }
  const float* rp = nullptr;
  long rB = 0, rT = 0;
  if (dres.has_value() && dres->defined()) {
    TORCH_CHECK(dres->dim() == 3 && dres->size(0) == B && dres->size(1) == T && dres->stride(2) == 1, "dres view");
    rp = dres->data_ptr<float>();
    rB = dres->stride(0);
    rT = dres->stride(1);
  }
  const bool dyb = dy.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(dyb || dy.scalar_type() == torch::kFloat32, "dy dtype");
  const bool has_res = res_y.has_value() && res_y->defined();
  JmLnRes res{};
  torch::Tensor dyr;
  if (has_res) {
    const int Tr = T - (int)res_T0;
    TORCH_CHECK(res_T0 >= 0 && Tr > 0, "res_T0");
    const auto& y = *res_y;
    CHECK_DT(y, torch::kBFloat16);
    long yB, yT;
    if (y.dim() == 3) {  // [B, Tr, D] view
      TORCH_CHECK(y.size(0) == B && y.size(1) == Tr && y.size(2) == D && y.stride(2) == 1, "res_y view");
      yB = y.stride(0);
      yT = y.stride(1);
    } else {
      TORCH_CHECK(y.is_contiguous() && y.numel() == (long)B * Tr * D, "res_y shape");
      yB = (long)Tr * D;
      yT = D;
    }
    if (res_out.has_value() && res_out->defined()) {  // same view layout as y (e.g. rows of a shared buffer)
      dyr = *res_out;
      CHECK_DT(dyr, torch::kBFloat16);
      TORCH_CHECK(dyr.sizes() == y.sizes() && dyr.strides() == y.strides(), "res_out must match res_y's view");
    } else {
      TORCH_CHECK(y.is_contiguous(), "res_y view needs res_out");
      dyr = torch::empty_like(y);
    }
    res = JmLnRes{bf(y), bfm(dyr), yB, yT, fopt(res_scale), fopt(res_mask), (int)res_T0, fopt_m(res_dscale),
                  fopt_m(res_dbias), make_drop(res_seed, res_rate, y, res_ioff)};
  }
  const uint16_t* hxp = nullptr;
  const float* betap = nullptr;
  if (hx.has_value() && hx->defined()) {  // the forward's bf16 LN output, rows like dy
    CHECK_DT((*hx), torch::kBFloat16);
    CHECK_CONTIG((*hx));
    TORCH_CHECK(hx->numel() == (long)B * T * D, "hx shape");
    TORCH_CHECK(beta.has_value() && beta->defined() && beta->numel() == D, "hx needs beta [D]");
    CHECK_DT((*beta), torch::kFloat32);
    hxp = bf(*hx);
    betap = beta->data_ptr<float>();
  }
  const int NP = has_res ? 4 : 2;
  auto ws = torch::empty({(accum || has_res) ? (long)jm_layernorm_bwd_blocks(B * T, D) * NP * D : 1}, x.options());
  check_rc(jm_layernorm_bwd(dy.data_ptr(), dyb, x.data_ptr<float>(), x.stride(0), x.stride(1), B, T, D,
                            mean.data_ptr<float>(), rstd.data_ptr<float>(), gamma.data_ptr<float>(),
                            dx.data_ptr<float>(), dx.stride(0), dx.stride(1), rp, rB, rT, dgamma.data_ptr<float>(),
                            dbeta.data_ptr<float>(), accum, ws.data_ptr<float>(), has_res ? &res : nullptr,
                            stream(), hxp, betap),
           "layernorm_bwd");
  if (has_res) return {dx, dyr};
  return {dx};
}

// ------------------------------------------------------------------------------ elementwise
torch::Tensor gelu_fwd(torch::Tensor h) {
  CHECK_CONTIG(h);
  CHECK_DT(h, torch::kBFloat16);
  auto a = torch::empty_like(h);
  check_rc(jm_gelu_fwd(bf(h), bfm(a), h.numel(), stream()), "gelu_fwd");
  return a;
}

// deriv: h holds the saved gelu'(pre-activation) (EPI_GELU_D forward) -> dh = da * h
// partial-row workspace of the column-reducing elementwise kernels (their fixed-order bias /
// scale gradient sums); a caching-allocator temporary on the current stream
static torch::Tensor rowcol_ws(const torch::Tensor& like, int M, int N, int nacc) {
  const long n = jm_rowcol_ws_floats(M, N, nacc);
  return torch::empty({n > 0 ? n : 1}, like.options().dtype(torch::kFloat32));
}

torch::Tensor gelu_bwd(torch::Tensor h, torch::Tensor da, c10::optional<torch::Tensor> bias_grad, bool deriv) {
  CHECK_CONTIG(h);
  CHECK_CONTIG(da);
  CHECK_DT(h, torch::kBFloat16);
  CHECK_DT(da, torch::kBFloat16);
  const int N = h.size(-1);
  const int M = h.numel() / N;
  auto dh = torch::empty_like(h);
  float* bg = fopt_m(bias_grad);
  torch::Tensor ws;
  if (bg) ws = rowcol_ws(h, M, N, 1);
  check_rc(jm_gelu_bwd(bf(h), bf(da), bfm(dh), bg, M, N, stream(), deriv ? 1 : 0, bg ? ws.data_ptr<float>() : nullptr),
           "gelu_bwd");
  return dh;
}

void colsum(torch::Tensor x, torch::Tensor acc) {
  CHECK_CONTIG(x);
  CHECK_DT(x, torch::kBFloat16);
  const int N = x.size(-1);
  const int M = x.numel() / N;
  auto ws = rowcol_ws(x, M, N, 1);
  check_rc(jm_colsum_bf16(bf(x), acc.data_ptr<float>(), M, N, stream(), ws.data_ptr<float>()), "colsum");
}

void splitk_reduce_add(torch::Tensor part, torch::Tensor g) {
  CHECK_CONTIG(part);
  TORCH_CHECK(g.is_contiguous() && g.numel() * part.size(0) == part.numel(), "splitk_reduce_add shapes");
  check_rc(jm_splitk_reduce_add(part.data_ptr<float>(), g.data_ptr<float>(), g.numel(), part.size(0), stream()),
           "splitk_reduce_add");
}

// g += x.sum(0) for a 2-D fp32 view with unit column stride (any row stride), no torch reduce
void colsum_add_f32(torch::Tensor x, torch::Tensor g) {
  CHECK_CUDA(x);
  CHECK_DT(x, torch::kFloat32);
  CHECK_DT(g, torch::kFloat32);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && g.is_contiguous() && g.numel() == x.size(1),
              "colsum_add_f32: x [rows, n] with unit column stride, g [n]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(g.data_ptr()) % 16 == 0,
              "colsum_add_f32: 16-byte aligned operands");
  check_rc(jm_colsum_add_f32(x.data_ptr<float>(), x.stride(0), x.size(0), x.size(1), g.data_ptr<float>(), stream()),
           "colsum_add_f32");
}

torch::Tensor residual_fwd(torch::Tensor x, torch::Tensor y, c10::optional<torch::Tensor> scale,
                           c10::optional<torch::Tensor> mask, c10::optional<torch::Tensor> out_opt,
                           c10::optional<torch::Tensor> seed, double rate, int64_t ioff) {
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1, "x must be [B,T,D]");
  CHECK_DT(x, torch::kFloat32);
  CHECK_CONTIG(y);
  CHECK_DT(y, torch::kBFloat16);
  const int B = x.size(0), T = x.size(1), D = x.size(2);
  torch::Tensor out;
  if (out_opt.has_value() && out_opt->defined()) {
    out = *out_opt;
    TORCH_CHECK(out.dim() == 3 && out.size(0) == B && out.size(1) == T && out.size(2) == D && out.stride(2) == 1,
                "out view");
  } else {
    out = torch::empty({B, T, D}, x.options());
  }
  check_rc(jm_residual_fwd(x.data_ptr<float>(), x.stride(0), x.stride(1), B, T, D, bf(y), fopt(scale), fopt(mask),
                           out.data_ptr<float>(), out.stride(0), out.stride(1), stream(),
                           make_drop(seed, rate, y, ioff)),
           "residual_fwd");
  return out;
}

// y / out: contiguous [B*T, D] or [B, T, D] views (out must then share y's strides; out given
// with y absent: its own strides)
torch::Tensor residual_bwd(torch::Tensor dout, c10::optional<torch::Tensor> y, c10::optional<torch::Tensor> scale,
                           c10::optional<torch::Tensor> mask, c10::optional<torch::Tensor> dscale, py::object ydtype,
                           c10::optional<torch::Tensor> dbias, c10::optional<torch::Tensor> out,
                           c10::optional<torch::Tensor> seed, double rate, int64_t ioff) {
  TORCH_CHECK(dout.dim() == 3 && dout.stride(2) == 1, "dout must be a [B,T,D] view");
  CHECK_DT(dout, torch::kFloat32);
  const int B = dout.size(0), T = dout.size(1), D = dout.size(2);
  const auto odt = torch::python::detail::py_object_to_dtype(ydtype);
  TORCH_CHECK(odt == torch::kBFloat16, "residual_bwd: y must be bf16");
  const bool has_y = y.has_value() && y->defined();
  auto strides_of = [&](const torch::Tensor& t, long& sb, long& st_) {
    if (t.dim() == 3) {
      TORCH_CHECK(t.size(0) == B && t.size(1) == T && t.size(2) == D && t.stride(2) == 1, "residual_bwd view");
      sb = t.stride(0);
      st_ = t.stride(1);
    } else {
      TORCH_CHECK(t.is_contiguous() && t.numel() == (long)B * T * D, "residual_bwd shape");
      sb = (long)T * D;
      st_ = D;
    }
  };
  long yB = (long)T * D, yT = D;
  if (has_y) strides_of(*y, yB, yT);
  torch::Tensor dy;
  if (out.has_value() && out->defined()) {
    dy = *out;
    CHECK_DT(dy, odt);
    long oB, oT;
    strides_of(dy, oB, oT);
    if (has_y) {
      TORCH_CHECK(oB == yB && oT == yT, "residual_bwd: out must share y's strides");
    } else {
      yB = oB;
      yT = oT;
    }
  } else {
    TORCH_CHECK(yB == (long)T * D && yT == D, "residual_bwd: a strided y needs out");
    dy = torch::empty({(long)B * T, D}, dout.options().dtype(odt));
  }
  torch::Tensor ws;
  const bool sums = (dscale && dscale->defined()) || (dbias && dbias->defined());
  if (sums) ws = rowcol_ws(dout, B * T, D, 2);
  check_rc(jm_residual_bwd(dout.data_ptr<float>(), dout.stride(0), dout.stride(1), has_y ? bf(*y) : nullptr,
                           fopt(scale), fopt(mask), fopt_m(dscale), bfm(dy), B, T, D, fopt_m(dbias), yB, yT,
                           stream(), make_drop(seed, rate, dout, ioff), sums ? ws.data_ptr<float>() : nullptr),
           "residual_bwd");
  return dy;
}

// ------------------------------------------------------------------------------ attention
// seed (int64 [1] on the device) with rate > 0: dropout on the attention probabilities (mask:
// common.h drop_keep at ((b H + h) S + q) SE + k, the backward regenerates it from the same seed)
static std::tuple<const int64_t*, uint32_t, float> attn_drop(const c10::optional<torch::Tensor>& seed, double rate,
                                                             const torch::Tensor& like, int S) {
  if (!seed.has_value() || !seed->defined() || rate <= 0.0) return {nullptr, 0u, 1.f};
  check_seed(*seed, like);
  TORCH_CHECK(S <= jm_attn_max_seq(), "attention dropout: S <= ", jm_attn_max_seq(), " (whole-sequence kernels)");
  const auto kp = keep_params(rate);
  return {seed->data_ptr<int64_t>(), kp.first, kp.second};
}

std::vector<torch::Tensor> attn_fwd(torch::Tensor qkv, int64_t heads, c10::optional<torch::Tensor> seed, double rate) {
  CHECK_CONTIG(qkv);
  CHECK_DT(qkv, torch::kBFloat16);
  const int B = qkv.size(0), S = qkv.size(1), D3 = qkv.size(2);
  const int D = D3 / 3, hd = D / heads;
  auto o = torch::empty({B, S, D}, qkv.options());
  auto lse = torch::empty({B, (long)heads, S}, qkv.options().dtype(torch::kFloat32));
  const auto dr = attn_drop(seed, rate, qkv, S);
  check_rc(jm_attn_fwd(bf(qkv), bfm(o), lse.data_ptr<float>(), B, S, heads, hd, std::get<0>(dr), std::get<1>(dr),
                       std::get<2>(dr), stream()),
           "attn_fwd");
  return {o, lse};
}

// dbias (optional, fp32 [3D]) += column sums of dqkv (the QKV Dense bias gradient), taken from
// the kernel's fp32 accumulators as per-sample partials and reduced here.
torch::Tensor attn_bwd(torch::Tensor dO, torch::Tensor qkv, torch::Tensor o, torch::Tensor lse, int64_t heads,
                       c10::optional<torch::Tensor> dbias, c10::optional<torch::Tensor> seed, double rate) {
  CHECK_CONTIG(dO);
  CHECK_CONTIG(qkv);
  CHECK_CONTIG(o);
  CHECK_DT(dO, torch::kBFloat16);
  const int B = qkv.size(0), S = qkv.size(1), D3 = qkv.size(2);
  const int D = D3 / 3, hd = D / heads;
  auto dqkv = torch::empty_like(qkv);
  const auto dr = attn_drop(seed, rate, qkv, S);
  if (S > jm_attn_max_seq()) {  // tile-streamed kernels; the caller reduces the bias gradient
    TORCH_CHECK(!dbias, "attn_bwd: no fused bias gradient for S > ", jm_attn_max_seq());
    auto delta = torch::empty({B, (long)heads, S}, qkv.options().dtype(torch::kFloat32));
    check_rc(jm_attn_bwd_long(bf(qkv), bf(o), bf(dO), lse.data_ptr<float>(), bfm(dqkv), delta.data_ptr<float>(), B,
                              S, heads, hd, stream()),
             "attn_bwd (long)");
    return dqkv;
  }
  torch::Tensor part;
  const int rows = jm_attn_bwd_part_rows(B, S, hd);
  if (dbias) {
    TORCH_CHECK(dbias->is_contiguous() && dbias->scalar_type() == torch::kFloat32 && dbias->numel() == D3,
                "attn_bwd: dbias must be contiguous fp32 [3D]");
    part = torch::empty({rows, D3}, qkv.options().dtype(torch::kFloat32));
  }
  float* pp = dbias ? part.data_ptr<float>() : nullptr;
  check_rc(jm_attn_bwd(bf(qkv), bf(o), bf(dO), lse.data_ptr<float>(), bfm(dqkv), B, S, heads, hd, pp, std::get<0>(dr),
                       std::get<1>(dr), std::get<2>(dr), stream()),
           "attn_bwd");
  if (dbias) check_rc(jm_splitk_reduce_add(pp, dbias->data_ptr<float>(), D3, rows, stream()), "attn_bwd dbias");
  return dqkv;
}

// ------------------------------------------------------------------------------ optimizer
int nch(const torch::Tensor& chunks) { return chunks.size(0); }
const int* chp(const torch::Tensor& chunks) { return chunks.data_ptr<int>(); }
uint16_t* shadow_ptr(c10::optional<torch::Tensor>& s) {
  return (s.has_value() && s->defined()) ? reinterpret_cast<uint16_t*>(s->data_ptr()) : nullptr;
}

// per-chunk partial sums of the norm kernels (summed per segment in chunk order: deterministic)
torch::Tensor chunk_part(const torch::Tensor& like, const torch::Tensor& chunks, int nc) {
  return torch::empty({(long)nch(chunks) * nc + 1}, like.options().dtype(torch::kFloat32));
}

void opt_sumsq(torch::Tensor x, torch::Tensor chunks, torch::Tensor out) {
  auto cp = chunk_part(x, chunks, 1);
  jm_opt_sumsq(x.data_ptr<float>(), chp(chunks), nch(chunks), out.data_ptr<float>(), cp.data_ptr<float>(), stream());
}

void opt_adamw(torch::Tensor p, torch::Tensor g, torch::Tensor mu, torch::Tensor nu, c10::optional<torch::Tensor> shadow,
               torch::Tensor chunks, torch::Tensor meta, torch::Tensor hyper, torch::Tensor gnorm_sq) {
  jm_opt_adamw(p.data_ptr<float>(), g.data_ptr<float>(), mu.data_ptr<float>(), nu.data_ptr<float>(),
               shadow_ptr(shadow), chp(chunks), nch(chunks), meta.data_ptr<float>(), hyper.data_ptr<float>(),
               gnorm_sq.data_ptr<float>(), stream());
}

void opt_lamb_phase1(torch::Tensor p, torch::Tensor g, torch::Tensor mu, torch::Tensor nu, torch::Tensor u,
                     torch::Tensor chunks, torch::Tensor meta, torch::Tensor hyper, torch::Tensor gnorm_sq,
                     torch::Tensor norms) {
  auto cp = chunk_part(p, chunks, 2);
  jm_opt_lamb_phase1(p.data_ptr<float>(), g.data_ptr<float>(), mu.data_ptr<float>(), nu.data_ptr<float>(),
                     u.data_ptr<float>(), chp(chunks), nch(chunks), meta.data_ptr<float>(), hyper.data_ptr<float>(),
                     gnorm_sq.data_ptr<float>(), norms.data_ptr<float>(), cp.data_ptr<float>(), stream());
}

void opt_lars_norms(torch::Tensor p, torch::Tensor g, torch::Tensor chunks, torch::Tensor hyper,
                    torch::Tensor gnorm_sq, torch::Tensor norms) {
  auto cp = chunk_part(p, chunks, 2);
  jm_opt_lars_norms(p.data_ptr<float>(), g.data_ptr<float>(), chp(chunks), nch(chunks), hyper.data_ptr<float>(),
                    gnorm_sq.data_ptr<float>(), norms.data_ptr<float>(), cp.data_ptr<float>(), stream());
}

void opt_apply_trust(torch::Tensor p, torch::Tensor u_or_g, c10::optional<torch::Tensor> trace,
                     c10::optional<torch::Tensor> shadow, torch::Tensor chunks, torch::Tensor meta, torch::Tensor hyper,
                     torch::Tensor norms, torch::Tensor gnorm_sq, int64_t mode, double momentum, double trust_coef) {
  jm_opt_apply_trust(p.data_ptr<float>(), u_or_g.data_ptr<float>(), fopt_m(trace), shadow_ptr(shadow), chp(chunks),
                     nch(chunks), meta.data_ptr<float>(), hyper.data_ptr<float>(), norms.data_ptr<float>(),
                     gnorm_sq.data_ptr<float>(), (int)mode, (float)momentum, (float)trust_coef, stream());
}

void opt_sgd(torch::Tensor p, torch::Tensor g, torch::Tensor trace, c10::optional<torch::Tensor> shadow,
             torch::Tensor chunks, torch::Tensor meta, torch::Tensor hyper, torch::Tensor gnorm_sq, double momentum) {
  jm_opt_sgd(p.data_ptr<float>(), g.data_ptr<float>(), trace.data_ptr<float>(), shadow_ptr(shadow), chp(chunks),
             nch(chunks), meta.data_ptr<float>(), hyper.data_ptr<float>(), gnorm_sq.data_ptr<float>(),
             (float)momentum, stream());
}

// ------------------------------------------------------------------------------ MAE
torch::Tensor patchify_normalize(torch::Tensor img, int64_t p) {
  CHECK_CONTIG(img);
  CHECK_DT(img, torch::kUInt8);
  const int B = img.size(0), H = img.size(2), W = img.size(3);
  TORCH_CHECK(img.size(1) == 3, "expects 3 channels");
  const int n = (H / p) * (W / p);
  auto out = torch::empty({B, n, (long)p * p * 3}, img.options().dtype(torch::kFloat32));
  check_rc(jm_patchify_normalize(img.data_ptr<uint8_t>(), out.data_ptr<float>(), B, H, W, p, stream()),
           "patchify_normalize");
  return out;
}

// Index tensors: int32, 1-D (shared permutation, batch stride 0) or 2-D [B, n] (per sample).
long ids_bstride(const torch::Tensor& ids) {
  CHECK_DT(ids, torch::kInt32);
  CHECK_CONTIG(ids);
  TORCH_CHECK(ids.dim() == 1 || ids.dim() == 2, "ids must be 1-D or 2-D");
  return ids.dim() == 1 ? 0 : ids.size(1);
}

torch::Tensor gather_patches(torch::Tensor img, torch::Tensor ids_keep, int64_t p) {
  CHECK_CONTIG(img);
  CHECK_DT(img, torch::kUInt8);
  TORCH_CHECK(img.size(1) == 3, "expects 3 channels");
  const long sb = ids_bstride(ids_keep);
  const int B = img.size(0), H = img.size(2), W = img.size(3);
  const int K = ids_keep.size(-1);
  TORCH_CHECK(ids_keep.dim() == 1 || ids_keep.size(0) == B, "ids_keep batch mismatch");
  auto out = torch::empty({(long)B * K, 3 * p * p}, img.options().dtype(torch::kBFloat16));
  check_rc(jm_gather_patches(img.data_ptr<uint8_t>(), ids_keep.data_ptr<int>(), sb, bfp(out), B, K, H, W, p, stream()),
           "gather_patches");
  return out;
}

torch::Tensor embed_finish(torch::Tensor e, c10::optional<torch::Tensor> pos, torch::Tensor ids_keep, torch::Tensor cls,
                           int64_t B) {
  CHECK_CONTIG(e);
  CHECK_DT(e, torch::kBFloat16);
  CHECK_CONTIG(cls);
  CHECK_DT(cls, torch::kFloat32);
  const long sb = ids_bstride(ids_keep);
  const int K = ids_keep.size(-1), D = e.size(1), C = cls.numel() / D;
  TORCH_CHECK(e.size(0) == B * K, "embed_finish: e rows");
  const float* pp = nullptr;
  if (pos) {
    CHECK_CONTIG((*pos));
    CHECK_DT((*pos), torch::kFloat32);
    TORCH_CHECK(pos->size(-1) == D, "pos dim");
    pp = pos->data_ptr<float>();
  }
  auto out = torch::empty({B, C + K, D}, e.options().dtype(torch::kFloat32));
  check_rc(jm_embed_finish(bfp(e), pp, ids_keep.data_ptr<int>(), sb, cls.data_ptr<float>(), out.data_ptr<float>(), B, C,
                           K, D, stream()),
           "embed_finish");
  return out;
}

torch::Tensor unshuffle_fwd(torch::Tensor y, torch::Tensor tok, torch::Tensor ids_restore, torch::Tensor pos,
                            int64_t C) {
  CHECK_CONTIG(y);
  CHECK_DT(y, torch::kBFloat16);
  CHECK_CONTIG(tok);
  CHECK_CONTIG(pos);
  CHECK_DT(tok, torch::kFloat32);
  CHECK_DT(pos, torch::kFloat32);
  const long sb = ids_bstride(ids_restore);
  const int B = y.size(0), d = y.size(2), K = y.size(1) - C, N = pos.size(0);
  TORCH_CHECK(ids_restore.size(-1) == N && tok.numel() == d && pos.size(1) == d, "unshuffle_fwd shapes");
  auto out = torch::empty({B, C + N, d}, y.options().dtype(torch::kFloat32));
  check_rc(jm_unshuffle_fwd(bfp(y), tok.data_ptr<float>(), ids_restore.data_ptr<int>(), sb, pos.data_ptr<float>(),
                            out.data_ptr<float>(), B, C, K, N, d, stream()),
           "unshuffle_fwd");
  return out;
}

// t[:] = 0 by the kernel the store-mode gradients use in front of an accumulating reduce (graph tests)
void zero_f32(torch::Tensor t) {
  CHECK_CUDA(t);
  CHECK_CONTIG(t);
  CHECK_DT(t, torch::kFloat32);
  jm_zero_f32(t.data_ptr<float>(), t.numel(), stream());
}

// random-masking ids from noise [N] or [R, N] fp32 -> (ids_shuffle i64, ids_restore i64, keep32 i32
// [.., keep], restore32 i32, mask f32), each shaped like the noise (keep32: last dim keep)
std::vector<torch::Tensor> mask_ids(torch::Tensor noise, int64_t keep) {
  CHECK_CUDA(noise);
  CHECK_CONTIG(noise);
  CHECK_DT(noise, torch::kFloat32);
  TORCH_CHECK(noise.dim() == 1 || noise.dim() == 2, "mask_ids: noise [N] or [R, N]");
  const int N = noise.size(-1), R = noise.dim() == 1 ? 1 : noise.size(0);
  TORCH_CHECK(N <= 1024 && keep >= 0 && keep <= N, "mask_ids: N <= 1024, 0 <= keep <= N");
  auto i64 = noise.options().dtype(torch::kInt64), i32 = noise.options().dtype(torch::kInt32);
  auto shuffle = torch::empty(noise.sizes(), i64), restore = torch::empty(noise.sizes(), i64);
  auto restore32 = torch::empty(noise.sizes(), i32), mask = torch::empty(noise.sizes(), noise.options());
  auto ks = noise.sizes().vec();
  ks.back() = keep;
  auto keep32 = torch::empty(ks, i32);
  check_rc(jm_mask_ids(noise.data_ptr<float>(), R, N, (int)keep, shuffle.data_ptr<int64_t>(),
                       restore.data_ptr<int64_t>(), keep32.data_ptr<int>(), restore32.data_ptr<int>(),
                       mask.data_ptr<float>(), stream()),
           "mask_ids");
  return {shuffle, restore, keep32, restore32, mask};
}

// -> (dy bf16 [B, C+K, d], d mask_token fp32 [d])
std::vector<torch::Tensor> unshuffle_bwd(torch::Tensor dout, torch::Tensor ids_restore, int64_t C, int64_t K) {
  CHECK_CONTIG(dout);
  CHECK_DT(dout, torch::kFloat32);
  const long sb = ids_bstride(ids_restore);
  const int B = dout.size(0), N = dout.size(1) - C, d = dout.size(2);
  TORCH_CHECK(ids_restore.size(-1) == N, "unshuffle_bwd shapes");
  const int rpb = 64;
  const int nb = jm_unshuffle_bwd_blocks(B, C, N, rpb);
  auto dy = torch::empty({B, C + K, d}, dout.options().dtype(torch::kBFloat16));
  auto part = torch::empty({nb, d}, dout.options());
  check_rc(jm_unshuffle_bwd(dout.data_ptr<float>(), ids_restore.data_ptr<int>(), sb, bfp(dy), part.data_ptr<float>(), B,
                            C, K, N, d, rpb, stream()),
           "unshuffle_bwd");
  return {dy, part};  // [nb, d] fp32 partials: the caller adds their column sums (colsum_add_f32)
}

// finetune input: [B*N, 3p^2] bf16 normalized patches of the (Mixup / CutMix) blended batch
torch::Tensor mix_patches(torch::Tensor img, c10::optional<torch::Tensor> perm, c10::optional<torch::Tensor> prm,
                          c10::optional<torch::Tensor> box, int64_t p) {
  CHECK_CONTIG(img);
  CHECK_DT(img, torch::kUInt8);
  TORCH_CHECK(img.size(1) == 3, "mix_patches: 3 channels");
  const int B = img.size(0), H = img.size(2), W = img.size(3);
  const int* pp = nullptr;
  const float* pr = nullptr;
  const int* bx = nullptr;
  if (prm) {
    TORCH_CHECK(perm && box, "mix_patches: prm needs perm and box");
    CHECK_DT((*perm), torch::kInt32);
    CHECK_DT((*prm), torch::kFloat32);
    CHECK_DT((*box), torch::kInt32);
    TORCH_CHECK(perm->numel() == B && prm->numel() >= 2 && box->numel() == 4, "mix_patches: param sizes");
    pp = perm->data_ptr<int>();
    pr = prm->data_ptr<float>();
    bx = box->data_ptr<int>();
  }
  auto out = torch::empty({(long)B * (H / p) * (W / p), 3 * p * p}, img.options().dtype(torch::kBFloat16));
  check_rc(jm_mix_patches(img.data_ptr<uint8_t>(), pp, pr, bx, bfp(out), B, H, W, p, stream()), "mix_patches");
  return out;
}

// pred: bf16 [B*N, P3] (row stride may exceed P3); -> per-patch MSE fp32 [B*N]
torch::Tensor patch_mse_fwd(torch::Tensor pred, torch::Tensor img, int64_t p, bool norm_pix) {
  CHECK_DT(pred, torch::kBFloat16);
  TORCH_CHECK(pred.stride(1) == 1, "pred rows must be contiguous");
  CHECK_CONTIG(img);
  CHECK_DT(img, torch::kUInt8);
  const int H = img.size(2), W = img.size(3), N = (H / p) * (W / p);
  TORCH_CHECK(pred.size(0) == img.size(0) * N && pred.size(1) == 3 * p * p, "patch_mse_fwd shapes");
  auto mse = torch::empty({pred.size(0)}, pred.options().dtype(torch::kFloat32));
  check_rc(jm_patch_mse_fwd(bfp(pred), pred.stride(0), img.data_ptr<uint8_t>(), mse.data_ptr<float>(), pred.size(0), N,
                            H, W, p, norm_pix, stream()),
           "patch_mse_fwd");
  return mse;
}

torch::Tensor patch_mse_bwd(torch::Tensor pred, torch::Tensor img, torch::Tensor dmse, int64_t p, bool norm_pix) {
  CHECK_DT(pred, torch::kBFloat16);
  TORCH_CHECK(pred.stride(1) == 1, "pred rows must be contiguous");
  CHECK_CONTIG(img);
  CHECK_CONTIG(dmse);
  CHECK_DT(dmse, torch::kFloat32);
  const int H = img.size(2), W = img.size(3), N = (H / p) * (W / p);
  TORCH_CHECK(dmse.numel() == pred.size(0) && pred.size(0) == img.size(0) * N, "patch_mse_bwd shapes");
  auto dpred = torch::empty({pred.size(0), pred.size(1)}, pred.options());
  check_rc(jm_patch_mse_bwd(bfp(pred), pred.stride(0), img.data_ptr<uint8_t>(), dmse.data_ptr<float>(), bfp(dpred),
                            pred.size(0), N, H, W, p, norm_pix, stream()),
           "patch_mse_bwd");
  return dpred;
}

}  // namespace

// ------------------------------------------------------------------------------ GEMM
// C[M, N] = A[M, K] . B[N, K]^T (+ bias) in bf16 (fp32 accumulate); gelu=true also returns
// gelu(C) (the pre-activation C is what the backward needs).  A / B rows may be strided.
// tail split (gemm.hip jm_gemm_nt_tail_plan): workspace for the split-K partials of the last,
// partly filled wave of output tiles; returns the number of tail tiles (0 = plain launch)
int attach_tail(GemmEpi& ep, torch::Tensor& ws, int M, int N, int K, int epi, const torch::Tensor& like) {
  int r = 0;
  long n = 0;
  const int S = jm_gemm_nt_tail_plan(M, N, K, epi, like.stride(0), &r, &n);
  if (S < 2) return 0;
  ws = torch::empty({n}, like.options().dtype(torch::kFloat32));
  ep.tail = ws.data_ptr<float>();
  ep.tail_S = S;
  ep.t_count = r;
  return r;
}

// gelu_deriv (with gelu): returns {gelu'(h) as uint8 codes (common.h gd_code), gelu(h)} instead of
// {h, gelu(h)} (EPI_GELU_D); with dropout the codes are those of the kept gelu'(h) unscaled (0 where
// dropped) and gemm_nt_dgelu applies 1 / keep when it decodes them
std::vector<torch::Tensor> gemm_nt(torch::Tensor A, torch::Tensor B, c10::optional<torch::Tensor> bias, bool gelu,
                                   bool gelu_only, bool gelu_deriv, c10::optional<torch::Tensor> seed, double rate) {
  CHECK_DT(A, torch::kBFloat16);
  CHECK_DT(B, torch::kBFloat16);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(1), "gemm_nt: A [M,K], B [N,K]");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1, "gemm_nt: K must be contiguous");
  const int M = A.size(0), N = B.size(0), K = A.size(1);
  TORCH_CHECK(!gelu_deriv || N % 8 == 0, "gemm_nt: gelu_deriv needs N % 8 == 0");
  auto out = torch::empty({M, N}, gelu_deriv ? A.options().dtype(torch::kUInt8) : A.options());
  torch::Tensor out2;
  GemmEpi ep{nullptr, gelu_deriv ? nullptr : bfm(out), N, nullptr, nullptr, nullptr, nullptr, 1};
  if (gelu_deriv) ep.dq = out.data_ptr<uint8_t>();
  if (bias) {
    TORCH_CHECK(bias->is_contiguous() && bias->scalar_type() == torch::kFloat32 && bias->numel() == N, "gemm_nt bias");
    ep.bias = bias->data_ptr<float>();
  }
  if (gelu && !gelu_only) {
    out2 = torch::empty({M, N}, A.options());
    ep.out2 = bfm(out2);
  }
  TORCH_CHECK(!gelu_deriv || (gelu && !gelu_only), "gemm_nt: gelu_deriv needs gelu and not gelu_only");
  const int epi = gelu_only ? 4 : (gelu_deriv ? 6 : (gelu ? 1 : 0));
  if (seed.has_value() && seed->defined() && rate > 0.0) {  // FF hidden dropout in the GELU_D epilogue
    TORCH_CHECK(epi == 6, "gemm_nt: dropout only with gelu_deriv");
    check_seed(*seed, A);
    const auto kp = keep_params(rate);
    ep.dseed = seed->data_ptr<int64_t>();
    ep.dthr = kp.first;
    ep.dscale = kp.second;
  }
  torch::Tensor ws;
  attach_tail(ep, ws, M, N, K, epi, A);
  check_rc(jm_gemm_nt(bf(A), A.stride(0), bf(B), B.stride(0), M, N, K, epi, ep, stream()), "gemm_nt");
  if (gelu && !gelu_only) return {out, out2};
  return {out};
}

// split-K: C[M, N] = A[M, K] . B[N, K]^T (+ bias) in bf16 via S fp32 partial products
// add (optional fp32 [M, N] view, unit column stride): the result is returned in fp32 as
// A.B^T (+ bias) + add, summed in the split-K reduction
torch::Tensor gemm_nt_splitk(torch::Tensor A, torch::Tensor B, c10::optional<torch::Tensor> bias, int64_t splits,
                             c10::optional<torch::Tensor> add) {
  CHECK_DT(A, torch::kBFloat16);
  CHECK_DT(B, torch::kBFloat16);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(1), "gemm_nt_splitk: A [M,K], B [N,K]");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1, "gemm_nt_splitk: K must be contiguous");
  const int M = A.size(0), N = B.size(0), K = A.size(1);
  auto out = torch::empty({M, N}, A.options());
  auto part = torch::empty({splits, (long)M * N}, A.options().dtype(torch::kFloat32));
  GemmEpi ep{nullptr, bfm(out), N, nullptr, nullptr, nullptr, part.data_ptr<float>(), (int)splits};
  check_rc(jm_gemm_nt(bf(A), A.stride(0), bf(B), B.stride(0), M, N, K, 3, ep, stream()), "gemm_nt_splitk");
  const float* bp = nullptr;
  if (bias) {
    TORCH_CHECK(bias->is_contiguous() && bias->scalar_type() == torch::kFloat32 && bias->numel() == N, "bias");
    bp = bias->data_ptr<float>();
  }
  if (add) {
    CHECK_CUDA(*add);
    CHECK_DT(*add, torch::kFloat32);
    TORCH_CHECK(add->dim() == 2 && add->size(0) == M && add->size(1) == N && add->stride(1) == 1,
                "gemm_nt_splitk: add must be fp32 [M, N] with unit column stride");
    auto out32 = torch::empty({M, N}, A.options().dtype(torch::kFloat32));
    check_rc(jm_splitk_reduce_f32(part.data_ptr<float>(), (int)splits, M, N, bp, add->data_ptr<float>(),
                                  add->stride(0), out32.data_ptr<float>(), stream()),
             "gemm_nt_splitk reduce f32");
    return out32;
  }
  check_rc(jm_splitk_reduce_bf16(part.data_ptr<float>(), (int)splits, (long)M * N, N, bp, bfm(out), stream()),
           "gemm_nt_splitk reduce");
  return out;
}

// C[M, N] = A[M, K] . B[N, K]^T in fp32 (EPI_PARTIAL with one split: the accumulators stored as
// they are) -- short-reduction weight gradients in NT form (ops/prims.py wgrad)
torch::Tensor gemm_nt_f32(torch::Tensor A, torch::Tensor B) {
  CHECK_DT(A, torch::kBFloat16);
  CHECK_DT(B, torch::kBFloat16);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(1), "gemm_nt_f32: A [M,K], B [N,K]");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1, "gemm_nt_f32: K must be contiguous");
  const int M = A.size(0), N = B.size(0), K = A.size(1);
  auto out = torch::empty({M, N}, A.options().dtype(torch::kFloat32));
  GemmEpi ep{nullptr, nullptr, N, nullptr, nullptr, nullptr, out.data_ptr<float>(), 1};
  check_rc(jm_gemm_nt(bf(A), A.stride(0), bf(B), B.stride(0), M, N, K, 3, ep, stream()), "gemm_nt_f32");
  return out;
}

// dh[M, N] = (A[M, K] . B[N, K]^T) * gelu'(pre[M, N]) -- FF2 data gradient through the GELU,
// B = W2^T; dbias (fp32 [N], optional) += column sums of dh (the FF1 bias gradient).
// deriv: ``pre`` holds the saved gelu'(h) as uint8 codes (EPI_GELU_D forward): the epilogue decodes
// and multiplies (EPI_DMUL); ``rate`` > 0: the forward's FF hidden dropout rate (codes of the unscaled
// kept derivative), 1 / keep applied with the decode
torch::Tensor gemm_nt_dgelu(torch::Tensor A, torch::Tensor B, torch::Tensor pre, c10::optional<torch::Tensor> dbias,
                            bool deriv, double rate) {
  CHECK_DT(A, torch::kBFloat16);
  CHECK_DT(B, torch::kBFloat16);
  CHECK_DT(pre, deriv ? torch::kUInt8 : torch::kBFloat16);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(1), "gemm_nt_dgelu: A [M,K], B [N,K]");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1, "gemm_nt_dgelu: K must be contiguous");
  const int M = A.size(0), N = B.size(0), K = A.size(1);
  TORCH_CHECK(pre.is_contiguous() && pre.size(0) == M && pre.size(1) == N, "gemm_nt_dgelu: pre [M,N]");
  auto out = torch::empty({M, N}, A.options());
  torch::Tensor part;
  GemmEpi ep{nullptr, bfm(out), N, nullptr, deriv ? nullptr : bf(pre), nullptr, nullptr, 1};
  if (deriv) {
    ep.dqa = pre.data_ptr<uint8_t>();
    ep.dqs = (rate > 0.0 ? keep_params(rate).second : 1.f) / 195.f;  // common.h GD_Q
  }
  torch::Tensor ws;
  const int epi = deriv ? 7 : 2;
  const int r = attach_tail(ep, ws, M, N, K, epi, A);
  int nM = jm_gemm_nt_colpart_rows(M, N, K, epi, A.stride(0));
  if (dbias) {
    TORCH_CHECK(dbias->is_contiguous() && dbias->scalar_type() == torch::kFloat32 && dbias->numel() == N,
                "gemm_nt_dgelu dbias");
    // tail tiles: their entries of the nM per-row-tile rows stay zero; the finish kernel writes
    // 8 extra rows per tail tile
    part = r ? torch::zeros({nM + 8 * r, N}, A.options().dtype(torch::kFloat32))
             : torch::empty({nM, N}, A.options().dtype(torch::kFloat32));
    ep.colpart = part.data_ptr<float>();
    nM += 8 * r;
  }
  check_rc(jm_gemm_nt(bf(A), A.stride(0), bf(B), B.stride(0), M, N, K, epi, ep, stream()), "gemm_nt_dgelu");
  if (dbias) check_rc(jm_splitk_reduce_add(part.data_ptr<float>(), dbias->data_ptr<float>(), N, nM, stream()),
                      "gemm_nt_dgelu dbias");
  return out;
}

// ---------------------------------------------------------------- augment (csrc/augment.hip)
// Pillow-exact RandomResizedCrop (bicubic) + flip of a batch of decoded crop windows on the device
// (data/loader.py DeviceAugment): src = concatenated HWC uint8 windows, tab = [B, 13] int64
// descriptors (csrc/augment.hip); tmp_bytes / tmp_rows_max from the host copy of the table.
torch::Tensor rrc_resize(torch::Tensor src, torch::Tensor tab, int64_t size, int64_t tmp_bytes, int64_t tmp_rows_max) {
  CHECK_CUDA(src);
  CHECK_CUDA(tab);
  CHECK_DT(src, torch::kUInt8);
  CHECK_DT(tab, torch::kInt64);
  TORCH_CHECK(src.dim() == 1 && src.is_contiguous(), "rrc_resize: src must be a flat uint8 buffer");
  TORCH_CHECK(tab.dim() == 2 && tab.size(1) == 13 && tab.is_contiguous(), "rrc_resize: tab [B, 13] int64");
  TORCH_CHECK(size > 0 && size <= 4096 && tmp_bytes > 0 && tmp_rows_max > 0, "rrc_resize: bad sizes");
  const int B = tab.size(0);
  auto out = torch::empty({B, 3, size, size}, src.options());
  auto tmp = torch::empty({tmp_bytes}, src.options());
  check_rc(jm_rrc_resize(src.data_ptr<uint8_t>(), tab.data_ptr<int64_t>(), B, (int)size, tmp.data_ptr<uint8_t>(),
                         (int)tmp_rows_max, out.data_ptr<uint8_t>(), stream()),
           "rrc_resize");
  return out;
}

// ---------------------------------------------------------------- dropout (csrc/dropout.hip)

// y = x * keep(seed, i) / keep  (bf16 or fp32, contiguous, numel % 8 == 0); also its own backward
torch::Tensor dropout_apply(torch::Tensor x, torch::Tensor seed, double rate) {
  CHECK_CONTIG(x);
  check_seed(seed, x);
  TORCH_CHECK(x.scalar_type() == torch::kBFloat16 || x.scalar_type() == torch::kFloat32, "dropout: bf16 / fp32");
  TORCH_CHECK(x.numel() % 8 == 0, "dropout: numel % 8");
  auto [thr, scale] = keep_params(rate);
  auto y = torch::empty_like(x);
  check_rc(jm_dropout_apply(x.data_ptr(), y.data_ptr(), x.numel(), x.scalar_type() == torch::kBFloat16,
                            seed.data_ptr<int64_t>(), thr, scale, stream()),
           "dropout_apply");
  return y;
}

// rows of fp32 logits [..., S] -> (softmax p (saved for the backward), dropped p * mask / keep)
// x *= keep(seed, i) / keep in place (bf16 or fp32, contiguous, numel % 8 == 0): the fused
// blocks' Dense-output dropout (forward on the branch output, backward on its gradient)
void dropout_apply_(torch::Tensor x, torch::Tensor seed, double rate) {
  CHECK_CUDA(x);
  check_seed(seed, x);
  TORCH_CHECK(x.is_contiguous() && x.numel() % 8 == 0, "dropout_apply_: contiguous, numel % 8 == 0");
  TORCH_CHECK(x.scalar_type() == torch::kBFloat16 || x.scalar_type() == torch::kFloat32, "dropout: bf16 / fp32");
  const auto kp = keep_params(rate);
  check_rc(jm_dropout_apply(x.data_ptr(), x.data_ptr(), x.numel(), x.scalar_type() == torch::kBFloat16,
                            seed.data_ptr<int64_t>(), kp.first, kp.second, stream()),
           "dropout_apply_");
}

// FF hidden dropout: (g, gp) masked in place (pair = the fused epilogue's gelu(h), gelu'(h)), or
// from the pre-activation h: returns (gelu(h) m, gelu'(h) m)
std::vector<torch::Tensor> gelu_drop(torch::Tensor a, c10::optional<torch::Tensor> b, torch::Tensor seed, double rate) {
  CHECK_CONTIG(a);
  CHECK_DT(a, torch::kBFloat16);
  check_seed(seed, a);
  TORCH_CHECK(a.numel() % 8 == 0, "gelu_drop: numel % 8");
  const auto kp = keep_params(rate);
  if (b.has_value() && b->defined()) {
    CHECK_CONTIG((*b));
    TORCH_CHECK(b->sizes() == a.sizes() && b->scalar_type() == torch::kBFloat16, "gelu_drop: (g, gp) pair");
    check_rc(jm_gelu_drop(nullptr, bfm(a), bfm(*b), a.numel(), seed.data_ptr<int64_t>(), kp.first, kp.second,
                          stream()),
             "gelu_drop");
    return {a, *b};
  }
  auto g = torch::empty_like(a), gp = torch::empty_like(a);
  check_rc(jm_gelu_drop(bf(a), bfm(g), bfm(gp), a.numel(), seed.data_ptr<int64_t>(), kp.first, kp.second, stream()),
           "gelu_drop");
  return {g, gp};
}

std::vector<torch::Tensor> softmax_dropout_fwd(torch::Tensor z, torch::Tensor seed, double rate) {
  CHECK_CONTIG(z);
  CHECK_DT(z, torch::kFloat32);
  check_seed(seed, z);
  auto [thr, scale] = keep_params(rate);
  const int S = z.size(-1);
  auto p = torch::empty_like(z);
  auto pd = torch::empty_like(z);
  check_rc(jm_softmax_dropout_fwd(z.data_ptr<float>(), p.data_ptr<float>(), pd.data_ptr<float>(), z.numel() / S, S,
                                  seed.data_ptr<int64_t>(), thr, scale, stream()),
           "softmax_dropout_fwd");
  return {p, pd};
}

torch::Tensor softmax_dropout_bwd(torch::Tensor dpd, torch::Tensor p, torch::Tensor seed, double rate) {
  CHECK_CONTIG(dpd);
  CHECK_CONTIG(p);
  CHECK_DT(dpd, torch::kFloat32);
  CHECK_DT(p, torch::kFloat32);
  TORCH_CHECK(dpd.sizes() == p.sizes(), "softmax_dropout_bwd shapes");
  check_seed(seed, p);
  auto [thr, scale] = keep_params(rate);
  const int S = p.size(-1);
  auto dz = torch::empty_like(p);
  check_rc(jm_softmax_dropout_bwd(dpd.data_ptr<float>(), p.data_ptr<float>(), dz.data_ptr<float>(), p.numel() / S, S,
                                  seed.data_ptr<int64_t>(), thr, scale, stream()),
           "softmax_dropout_bwd");
  return dz;
}

// dst [C, R] = src [R, C]^T (bf16, both contiguous)
void transpose_bf16(torch::Tensor src, torch::Tensor dst) {
  CHECK_CONTIG(src);
  CHECK_CONTIG(dst);
  CHECK_DT(src, torch::kBFloat16);
  CHECK_DT(dst, torch::kBFloat16);
  TORCH_CHECK(src.dim() == 2 && dst.dim() == 2 && dst.size(0) == src.size(1) && dst.size(1) == src.size(0),
              "transpose_bf16 shapes");
  check_rc(jm_transpose_bf16(bf(src), bfm(dst), src.size(0), src.size(1), stream()), "transpose_bf16");
}

// all transposed weight copies of a step in one launch: desc int64 [n, 6] on the device
// ({src, dst, R, C, first tile, tiles along C}, built by ParamStore.refresh_transposes)
void transpose_bf16_batch(torch::Tensor desc, int64_t tiles) {
  CHECK_CONTIG(desc);
  TORCH_CHECK(desc.is_cuda() && desc.scalar_type() == torch::kInt64 && desc.dim() == 2 && desc.size(1) == 6,
              "transpose_bf16_batch: desc int64 [n, 6] on the device");
  check_rc(jm_transpose_bf16_batch(reinterpret_cast<const long long*>(desc.data_ptr<int64_t>()), (int)desc.size(0),
                                   (int)tiles, stream()),
           "transpose_bf16_batch");
}

// weight gradient G[N, K] += dy[M, N]^T . x[M, K] on the TN MFMA kernel (split over M, fp32
// partial tiles reduced into G); returns the number of M splits used
// store: g = dy^T . x (g's old contents ignored: its first contribution of the step)
int64_t gemm_tn_wgrad(torch::Tensor dy, torch::Tensor x, torch::Tensor g, bool store) {
  CHECK_DT(dy, torch::kBFloat16);
  CHECK_DT(x, torch::kBFloat16);
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0), "gemm_tn_wgrad: dy [M,N], x [M,K]");
  TORCH_CHECK(dy.stride(1) == 1 && x.stride(1) == 1, "gemm_tn_wgrad: rows must be contiguous");
  const int M = dy.size(0), N = dy.size(1), K = x.size(1);
  TORCH_CHECK(g.is_contiguous() && g.scalar_type() == torch::kFloat32 && g.numel() == (long)N * K, "gemm_tn_wgrad g");
  int S = 1;
  const int sps = jm_gemm_tn_plan(M, N, K, &S);
  torch::Tensor part;
  const int SP = S;  // fp32 partial slices, reduced into g
  if (S > 1) part = torch::empty({SP, (long)N * K}, g.options());
  const int done = jm_gemm_tn(bf(dy), dy.stride(0), bf(x), x.stride(0), M, N, K, sps, S, g.data_ptr<float>(), K,
                              S > 1 ? part.data_ptr<float>() : nullptr, stream(), store);
  check_rc(done, "gemm_tn_wgrad");
  if (S > 1)
    check_rc(jm_splitk_reduce_add(part.data_ptr<float>(), g.data_ptr<float>(), (long)N * K, SP, stream(), store),
             "gemm_tn_wgrad reduce");
  return S;
}

// g[N, K] += sum_i dys[i]^T xs[i]: the reduction rows are the concatenation of the per-layer
// blocks (all [rows, N] / [rows, K], same strides), read in place (no torch.cat copy)
int64_t gemm_tn_wgrad_seg(std::vector<torch::Tensor> dys, std::vector<torch::Tensor> xs, torch::Tensor g, bool store) {
  TORCH_CHECK(!dys.empty() && dys.size() == xs.size() && dys.size() <= 32, "gemm_tn_wgrad_seg: 1..32 blocks");
  const auto& d0 = dys[0];
  const auto& x0 = xs[0];
  const int rows = d0.size(0), N = d0.size(1), K = x0.size(1);
  TnSegs segs{};
  segs.rows = rows;
  segs.n = (int)dys.size();
  for (size_t i = 0; i < dys.size(); ++i) {
    CHECK_DT(dys[i], torch::kBFloat16);
    CHECK_DT(xs[i], torch::kBFloat16);
    TORCH_CHECK(dys[i].dim() == 2 && xs[i].dim() == 2 && dys[i].size(0) == rows && xs[i].size(0) == rows &&
                    dys[i].size(1) == N && xs[i].size(1) == K,
                "gemm_tn_wgrad_seg: block shapes differ");
    TORCH_CHECK(dys[i].stride(1) == 1 && xs[i].stride(1) == 1 && dys[i].stride(0) == d0.stride(0) &&
                    xs[i].stride(0) == x0.stride(0),
                "gemm_tn_wgrad_seg: block strides differ");
    segs.a[i] = bf(dys[i]);
    segs.b[i] = bf(xs[i]);
  }
  TORCH_CHECK(g.is_contiguous() && g.scalar_type() == torch::kFloat32 && g.numel() == (long)N * K, "gemm_tn_wgrad_seg g");
  const int M = rows * segs.n;
  int S = 1;
  const int sps = jm_gemm_tn_plan(M, N, K, &S);
  torch::Tensor part;
  const int SP = S;
  if (S > 1) part = torch::empty({SP, (long)N * K}, g.options());
  const int done = jm_gemm_tn_seg(segs, d0.stride(0), x0.stride(0), N, K, sps, S, g.data_ptr<float>(), K,
                                  S > 1 ? part.data_ptr<float>() : nullptr, stream(), store);
  check_rc(done, "gemm_tn_wgrad_seg");
  if (S > 1)
    check_rc(jm_splitk_reduce_add(part.data_ptr<float>(), g.data_ptr<float>(), (long)N * K, SP, stream(), store),
             "gemm_tn_wgrad_seg reduce");
  return S;
}

// g_p[N_p, K_p] += dys[p]^T . xs[p] for up to 4 problems over the same M rows in ONE grid (e.g. a
// layer's FF1 + FF2 or QKV + Wo weight gradients): fewer M splits per problem than separate
// launches -> fewer fp32 partial slices to write and reduce; returns the split count
// One-split grouped launches store into every G or accumulate into every G (one kernel variant):
// with mixed store flags the store problems' G are zeroed first and all accumulate.  Returns the
// launch's store mode.
int group_stores(const std::vector<bool>& stores, const std::vector<torch::Tensor>& gs, int S, int n) {
  if (S > 1 || stores.empty()) return 0;
  int ns = 0;
  for (int p = 0; p < n; ++p) ns += p < (int)stores.size() && stores[p];
  if (ns == n) return 1;
  for (int p = 0; p < n; ++p)
    if (p < (int)stores.size() && stores[p])
      jm_zero_f32(gs[p].data_ptr<float>(), gs[p].numel(), stream());
  return 0;
}

// stores[p]: g_p = its product (first contribution of the step) instead of +=
int64_t gemm_tn_wgrad_group(std::vector<torch::Tensor> dys, std::vector<torch::Tensor> xs,
                            std::vector<torch::Tensor> gs, std::vector<bool> stores) {
  const int n = (int)dys.size();
  TORCH_CHECK(n >= 1 && n <= 4 && (int)xs.size() == n && (int)gs.size() == n, "gemm_tn_wgrad_group: 1..4 problems");
  const int M = dys[0].size(0);
  TnGroup grp{};
  grp.n = n;
  long total = 0;
  for (int p = 0; p < n; ++p) {
    const auto &dy = dys[p], &x = xs[p], &g = gs[p];
    CHECK_DT(dy, torch::kBFloat16);
    CHECK_DT(x, torch::kBFloat16);
    TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == M && x.size(0) == M,
                "gemm_tn_wgrad_group: dy [M,N_p], x [M,K_p] with one M");
    TORCH_CHECK(dy.stride(1) == 1 && x.stride(1) == 1, "gemm_tn_wgrad_group: rows must be contiguous");
    const int N = dy.size(1), K = x.size(1);
    TORCH_CHECK(N % 256 == 0 && K % 256 == 0, "gemm_tn_wgrad_group: N, K multiples of 256");
    TORCH_CHECK(g.is_contiguous() && g.scalar_type() == torch::kFloat32 && g.numel() == (long)N * K && g.is_cuda(),
                "gemm_tn_wgrad_group g");
    grp.a[p] = bf(dy);
    grp.b[p] = bf(x);
    grp.lda[p] = dy.stride(0);
    grp.ldb[p] = x.stride(0);
    grp.N[p] = N;
    grp.K[p] = K;
    total += (long)N * K;
  }
  int S = 1;
  const int sps = jm_gemm_tn_group_plan(grp, M, &S);
  torch::Tensor part;
  long off = 0;
  if (S > 1) part = torch::empty({(long)S * total}, gs[0].options());
  for (int p = 0; p < n; ++p) {
    grp.out[p] = S > 1 ? part.data_ptr<float>() + off : gs[p].data_ptr<float>();
    off += (long)S * grp.N[p] * grp.K[p];
  }
  const int all_store = group_stores(stores, gs, S, n);
  check_rc(jm_gemm_tn_group(grp, M, sps, S, stream(), all_store), "gemm_tn_wgrad_group");
  if (S > 1)
    for (int p = 0; p < n; ++p)
      check_rc(jm_splitk_reduce_add(grp.out[p], gs[p].data_ptr<float>(), (long)grp.N[p] * grp.K[p], S, stream(),
                                    p < (int)stores.size() && stores[p]),
               "gemm_tn_wgrad_group reduce");
  return S;
}

// g_p[N_p, K_p] += sum_i dys[p][i]^T xs[p][i] for two problems whose reduction rows are the same
// per-layer blocks (the shared jumbo MLP's W1 and W2 gradients over all layers), one grid
int64_t gemm_tn_wgrad_seg_group(std::vector<std::vector<torch::Tensor>> dys, std::vector<std::vector<torch::Tensor>> xs,
                                std::vector<torch::Tensor> gs, std::vector<bool> stores) {
  const int np = (int)dys.size();
  TORCH_CHECK(np >= 1 && np <= 2 && (int)xs.size() == np && (int)gs.size() == np, "gemm_tn_wgrad_seg_group: 1-2 problems");
  const int nb = (int)dys[0].size();
  TORCH_CHECK(nb >= 1 && nb <= 32, "gemm_tn_wgrad_seg_group: 1..32 blocks");
  const int rows = dys[0][0].size(0);
  TnSegs segs{};
  segs.rows = rows;
  segs.n = nb;
  TnGroup grp{};
  grp.n = np;
  long total = 0;
  for (int p = 0; p < np; ++p) {
    TORCH_CHECK((int)dys[p].size() == nb && (int)xs[p].size() == nb, "gemm_tn_wgrad_seg_group: block counts differ");
    const auto &d0 = dys[p][0], &x0 = xs[p][0];
    const int N = d0.size(1), K = x0.size(1);
    for (int i = 0; i < nb; ++i) {
      const auto &d = dys[p][i], &x = xs[p][i];
      CHECK_DT(d, torch::kBFloat16);
      CHECK_DT(x, torch::kBFloat16);
      TORCH_CHECK(d.dim() == 2 && x.dim() == 2 && d.size(0) == rows && x.size(0) == rows && d.size(1) == N &&
                      x.size(1) == K && d.stride(1) == 1 && x.stride(1) == 1 && d.stride(0) == d0.stride(0) &&
                      x.stride(0) == x0.stride(0),
                  "gemm_tn_wgrad_seg_group: block shapes / strides differ");
      segs.a[32 * p + i] = bf(d);
      segs.b[32 * p + i] = bf(x);
    }
    const auto& g = gs[p];
    TORCH_CHECK(g.is_contiguous() && g.scalar_type() == torch::kFloat32 && g.numel() == (long)N * K,
                "gemm_tn_wgrad_seg_group g");
    grp.lda[p] = d0.stride(0);
    grp.ldb[p] = x0.stride(0);
    grp.N[p] = N;
    grp.K[p] = K;
    total += (long)N * K;
  }
  int S = 1;
  const int sps = jm_gemm_tn_group_plan(grp, rows * nb, &S);
  torch::Tensor part;
  if (S > 1) part = torch::empty({(long)S * total}, gs[0].options());
  long off = 0;
  for (int p = 0; p < np; ++p) {
    grp.out[p] = S > 1 ? part.data_ptr<float>() + off : gs[p].data_ptr<float>();
    off += (long)S * grp.N[p] * grp.K[p];
  }
  const int all_store = group_stores(stores, gs, S, np);
  check_rc(jm_gemm_tn_group_seg(grp, segs, sps, S, stream(), all_store), "gemm_tn_wgrad_seg_group");
  if (S > 1)
    for (int p = 0; p < np; ++p)
      check_rc(jm_splitk_reduce_add(grp.out[p], gs[p].data_ptr<float>(), (long)grp.N[p] * grp.K[p], S, stream(),
                                    p < (int)stores.size() && stores[p]),
               "gemm_tn_wgrad_seg_group reduce");
  return S;
}

// zero the (offset, count) float ranges of ``base`` listed in desc (int64 [n, 2] on the device)
void zero_ranges(torch::Tensor base, torch::Tensor desc, int64_t blocks) {
  CHECK_CONTIG(base);
  CHECK_DT(base, torch::kFloat32);
  TORCH_CHECK(desc.is_cuda() && desc.scalar_type() == torch::kInt64 && desc.dim() == 2 && desc.size(1) == 2,
              "zero_ranges: desc int64 [n, 2] on the device");
  check_rc(jm_zero_ranges(base.data_ptr<float>(), reinterpret_cast<const long long*>(desc.data_ptr<int64_t>()),
                          (int)desc.size(0), blocks, stream()),
           "zero_ranges");
}

// x1 = x + mask*scale*y ([B,T,D] fp32, fresh contiguous); h / mean / rstd = LN of rows t >= T0
std::vector<torch::Tensor> residual_ln_fwd(torch::Tensor x, torch::Tensor y, c10::optional<torch::Tensor> scale,
                                           c10::optional<torch::Tensor> mask, torch::Tensor gamma,
                                           torch::Tensor beta, double eps, int64_t T0, int64_t R0,
                                           c10::optional<torch::Tensor> out, c10::optional<torch::Tensor> seed,
                                           double rate) {
  CHECK_CUDA(x);
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1, "x must be [B,T,D] with contiguous last dim");
  CHECK_DT(x, torch::kFloat32);
  CHECK_DT(y, torch::kBFloat16);
  CHECK_CONTIG(y);
  const int B = x.size(0), T = x.size(1), D = x.size(2);
  TORCH_CHECK(R0 >= 0 && R0 < T, "residual_ln_fwd: R0");
  TORCH_CHECK(y.numel() == (long)B * (T - R0) * D, "residual_ln_fwd: y must be [B*(T-R0), D]");
  TORCH_CHECK(T0 >= 0 && T0 < T, "residual_ln_fwd: T0");
  TORCH_CHECK(R0 == 0 || out.has_value(), "residual_ln_fwd: R0 > 0 needs out (its rows t < R0 are inputs)");
  torch::Tensor x1;
  if (out) {
    CHECK_DT(*out, torch::kFloat32);
    TORCH_CHECK(out->dim() == 3 && out->size(0) == B && out->size(1) == T && out->size(2) == D && out->stride(2) == 1,
                "residual_ln_fwd: out must be [B,T,D] with contiguous last dim");
    x1 = *out;
  } else {
    x1 = torch::empty({B, T, D}, x.options());
  }
  const long R = (long)B * (T - T0);
  auto h = torch::empty({R, D}, y.options());
  auto mean = torch::empty({R}, x.options());
  auto rstd = torch::empty({R}, x.options());
  check_rc(jm_residual_ln_fwd(x.data_ptr<float>(), x.stride(0), x.stride(1), bf(y), fopt(scale), fopt(mask),
                              x1.data_ptr<float>(), x1.stride(0), x1.stride(1), bfm(h), mean.data_ptr<float>(),
                              rstd.data_ptr<float>(), B, T, T0, D, gamma.data_ptr<float>(), beta.data_ptr<float>(),
                              (float)eps, stream(), (int)R0, make_drop(seed, rate, y, 0)),
           "residual_ln_fwd");
  return {x1, h, mean, rstd};
}

py::dict debug_lines() {
  py::dict d;
  const std::pair<const char*, int (*)()> tus[] = {
      {"attention", jm_debug_line_attention}, {"dropout", jm_debug_line_dropout},
      {"augment", jm_debug_line_augment},
      {"elementwise", jm_debug_line_elementwise},
      {"gemm", jm_debug_line_gemm},           {"gemm_tn", jm_debug_line_gemm_tn},
      {"layernorm", jm_debug_line_layernorm}, {"mae", jm_debug_line_mae},
      {"optim", jm_debug_line_optim}};
  for (const auto& t : tus) {
    const int line = t.second();
    if (line) d[t.first] = line;
  }
  return d;
}

void debug_selftest(int v) { jm_debug_selftest(v, stream()); }

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "jumbo_mae_tpu_amd CDNA4 (gfx950) HIP kernels";
  m.def("layernorm_fwd", &layernorm_fwd, py::arg("x"), py::arg("gamma"), py::arg("beta"), py::arg("eps"),
        py::arg("out_dtype"), py::arg("also_bf16") = false);
  m.def("layernorm_bwd", &layernorm_bwd, py::arg("dy"), py::arg("x"), py::arg("mean"), py::arg("rstd"),
        py::arg("gamma"), py::arg("dgamma"), py::arg("dbeta"), py::arg("accum"), py::arg("dres") = py::none(),
        py::arg("out") = py::none(), py::arg("res_y") = py::none(), py::arg("res_scale") = py::none(),
        py::arg("res_mask") = py::none(), py::arg("res_dscale") = py::none(), py::arg("res_dbias") = py::none(),
        py::arg("res_T0") = 0, py::arg("res_out") = py::none(), py::arg("res_seed") = py::none(),
        py::arg("res_rate") = 0.0, py::arg("res_ioff") = 0, py::arg("hx") = py::none(), py::arg("beta") = py::none());
  m.def("gelu_fwd", &gelu_fwd);
  m.def("dropout_apply", &dropout_apply);
  m.def("dropout_apply_", &dropout_apply_);
  m.def("rrc_resize", &rrc_resize, py::arg("src"), py::arg("tab"), py::arg("size"), py::arg("tmp_bytes"),
        py::arg("tmp_rows_max"));
  m.def("rrc_kmax", &jm_rrc_kmax);
  m.def("gelu_drop", &gelu_drop, py::arg("a"), py::arg("b") = py::none(), py::arg("seed"), py::arg("rate"));
  m.def("softmax_dropout_fwd", &softmax_dropout_fwd);
  m.def("softmax_dropout_bwd", &softmax_dropout_bwd);
  m.def("gelu_bwd", &gelu_bwd, py::arg("h"), py::arg("da"), py::arg("bias_grad") = py::none(),
        py::arg("deriv") = false);
  m.def("colsum", &colsum);
  m.def("splitk_reduce_add", &splitk_reduce_add);
  m.def("residual_ln_fwd", &residual_ln_fwd, py::arg("x"), py::arg("y"), py::arg("scale"), py::arg("mask"),
        py::arg("gamma"), py::arg("beta"), py::arg("eps"), py::arg("T0"), py::arg("R0") = 0,
        py::arg("out") = py::none(), py::arg("seed") = py::none(), py::arg("rate") = 0.0);
  m.def("transpose_bf16", &transpose_bf16);
  m.def("residual_fwd", &residual_fwd, py::arg("x"), py::arg("y"), py::arg("scale"), py::arg("mask"),
        py::arg("out") = py::none(), py::arg("seed") = py::none(), py::arg("rate") = 0.0, py::arg("ioff") = 0);
  m.def("residual_bwd", &residual_bwd, py::arg("dout"), py::arg("y"), py::arg("scale"), py::arg("mask"),
        py::arg("dscale"), py::arg("ydtype"), py::arg("dbias") = py::none(), py::arg("out") = py::none(),
        py::arg("seed") = py::none(), py::arg("rate") = 0.0, py::arg("ioff") = 0);
  m.def("attn_fwd", &attn_fwd, py::arg("qkv"), py::arg("heads"), py::arg("seed") = py::none(), py::arg("rate") = 0.0);
  m.def("attn_bwd", &attn_bwd, py::arg("dO"), py::arg("qkv"), py::arg("o"), py::arg("lse"), py::arg("heads"),
        py::arg("dbias") = py::none(), py::arg("seed") = py::none(), py::arg("rate") = 0.0);
  m.def("attn_max_seq", &jm_attn_max_seq);
  m.def("gemm_tn_wgrad", &gemm_tn_wgrad, py::arg("dy"), py::arg("x"), py::arg("g"), py::arg("store") = false);
  m.def("gemm_tn_wgrad_seg", &gemm_tn_wgrad_seg, py::arg("dys"), py::arg("xs"), py::arg("g"), py::arg("store") = false);
  m.def("zero_ranges", &zero_ranges, "zero float ranges of a flat buffer (one launch)");
  m.def("colsum_add_f32", &colsum_add_f32, "g += x.sum(0) for a row-strided fp32 [rows, n] view");
  m.def("gemm_tn_wgrad_seg_group", &gemm_tn_wgrad_seg_group, py::arg("dys"), py::arg("xs"), py::arg("gs"),
        py::arg("stores") = std::vector<bool>{}, "grouped segmented weight gradients (<= 2 problems)");
  m.def("gemm_tn_wgrad_group", &gemm_tn_wgrad_group, py::arg("dys"), py::arg("xs"), py::arg("gs"),
        py::arg("stores") = std::vector<bool>{}, "grouped weight gradients over one M (<= 4 problems)");
  m.def("gemm_test_force", &jm_gemm_test_force, py::arg("path"), py::arg("rows") = 0,
        "numerics tests only: NT GEMM kernel path 0 = by shape, 1 = 64-deep main loop everywhere, "
        "2 = 4-phase kernels at every M without tail split (rows = forced tile height)");
  m.def("gemm_nt_tiles", &jm_gemm_nt_tiles, py::arg("M"), py::arg("N"), py::arg("K") = 1024, py::arg("epi") = 0,
        py::arg("lda") = 0, "output tiles (workgroups before split-K) of an NT launch");
  m.def("transpose_bf16_batch", &transpose_bf16_batch);
  m.def("gemm_nt_splitk", &gemm_nt_splitk, py::arg("A"), py::arg("B"), py::arg("bias") = py::none(),
        py::arg("splits") = 8, py::arg("add") = py::none());
  m.def("gemm_nt_dgelu", &gemm_nt_dgelu, py::arg("A"), py::arg("B"), py::arg("pre"), py::arg("dbias") = py::none(),
        py::arg("deriv") = false, py::arg("rate") = 0.0);
  m.def("gemm_nt_f32", &gemm_nt_f32, py::arg("A"), py::arg("B"));
  m.def("gemm_nt", &gemm_nt, py::arg("A"), py::arg("B"), py::arg("bias") = py::none(), py::arg("gelu") = false,
        py::arg("gelu_only") = false, py::arg("gelu_deriv") = false, py::arg("seed") = py::none(),
        py::arg("rate") = 0.0);
  m.def("opt_sumsq", &opt_sumsq);
  m.def("opt_adamw", &opt_adamw);
  m.def("opt_lamb_phase1", &opt_lamb_phase1);
  m.def("opt_lars_norms", &opt_lars_norms);
  m.def("opt_apply_trust", &opt_apply_trust);
  m.def("opt_sgd", &opt_sgd);
  m.def("patchify_normalize", &patchify_normalize);
  m.def("gather_patches", &gather_patches);
  m.def("embed_finish", &embed_finish);
  m.def("zero_f32", &zero_f32, "fp32 zero fill kernel (the store-mode gradients' pre-reduce fill)");
  m.def("mask_ids", &mask_ids, "random-masking permutation ids + mask from noise (one workgroup per row)");
  m.def("unshuffle_fwd", &unshuffle_fwd);
  m.def("unshuffle_bwd", &unshuffle_bwd);
  m.def("patch_mse_fwd", &patch_mse_fwd);
  m.def("mix_patches", &mix_patches);
  m.def("patch_mse_bwd", &patch_mse_bwd);
  m.def("debug_lines", &debug_lines);
  m.def("debug_selftest", &debug_selftest);
#ifdef JM_DEBUG
  m.attr("debug_build") = true;
#else
  m.attr("debug_build") = false;
#endif
}
