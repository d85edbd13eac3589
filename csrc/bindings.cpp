// torch.ops.p2p.* registrations for the HIP/CDNA4 kernels (gfx950).
//
// Host-side responsibilities kept in C++: argument checking, output / workspace
// allocation through PyTorch's caching allocator (so every op is hipGraph-capturable --
// no hipMalloc, no sync), GEMM tile and split-K selection, and launching on the current
// HIP stream.  Autograd, weight-layout caching and channel padding live in
// p2p_pytorch_amd/ops/hip.py.
//
// Tensor convention: activations are bf16 NCHW-shaped tensors in channels_last memory
// (i.e. NHWC bytes) with C % 8 == 0 (16-B channel chunks); weights are pre-laid-out bf16
// GEMM operands produced by weight_prep; master weights / grads / optimizer state fp32.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "conv.h"
#include "knobs.h"

// fp8 layers the stride-2 halo kernel takes (P2P_S2T_F8, read per call): bit 0 the e4m3
// ConvT forward, bit 1 the e5m2 input gradient (extended epilogue)
static int s2t_f8_mask() {   // (read per call: tests/test_fp8_gpu.py pins both variants on)
  constexpr int kDefault = 1;   // input gradient off: B=256 fp8 8955 (both) vs 9087 (forward only), profiles/bench_fp8_r4fb.jsonl
  const char* v = std::getenv("P2P_S2T_F8");
  return v ? std::atoi(v) & 3 : kDefault;
}

extern "C" {
long p2p_sn_ws_floats(int h, int wd);
int p2p_sn_power_iter(const float* W, int h, int wd, float* u, float* v, float* sigma, float* ws,
                      float* scale, hipStream_t st);
int p2p_sn_wgrad_blocks(long n);
int p2p_sn_wgrad(const float* G, const float* W, const float* u, const float* v, const float* scale, int h,
                 int wd, float* part, float* out, int accumulate, hipStream_t st);
long p2p_norm_ws_floats(int N, int HW, int C);
int p2p_norm_fwd_partials(const void* x, int N, int HW, int C, int nchunks, const float* partials,
                          float eps, const float* gamma, const float* beta, const float* prelu_w,
                          int act, float* mean, float* rstd, float* run_mean, float* run_var,
                          float momentum, void* y, void* q, int* qsite, int qfmt, const void* res,
                          hipStream_t st);
int p2p_norm_fwd(const void* x, int N, int HW, int C, float eps, const float* gamma,
                 const float* beta, const float* prelu_w, int act, float* mean, float* rstd,
                 float* run_mean, float* run_var, float momentum, float* ws, void* y,
                 void* q, int* qsite, int qfmt, const void* res, hipStream_t st);
int p2p_norm_apply(const void* x, int N, int HW, int C, const float* mean, const float* rstd,
                   const float* gamma, const float* beta, const float* prelu_w, int act, void* y,
                   const void* res, hipStream_t st);
int p2p_norm_bwd(const void* x, const void* dy, int N, int HW, int C, const float* mean,
                 const float* rstd, const float* gamma, const float* beta, int act,
                 const float* prelu_w, float* dprelu, float* dgamma, float* dbeta, float* ws, void* dx,
                 float* dsum, void* q, int* qsite, int qfmt, int frozen, hipStream_t st);
int p2p_norm_bwd_partials(const void* x, const void* dy, int N, int HW, int C, int nchunks,
                          const float* partials, const float* mean, const float* rstd,
                          const float* gamma, const float* beta, int act, const float* prelu_w, float* dgamma,
                          float* dbeta, float* coef, void* dx, float* dsum, void* q, int* qsite, int qfmt,
                          hipStream_t st);
int p2p_act(const void* a, const void* b, long n, int act, int mode, void* out, hipStream_t st);
int p2p_dropout(const void* x, long n, float p, const int64_t* seed, unsigned salt, void* y,
                hipStream_t st);
int p2p_misc_nblocks(long n);
int p2p_prelu_fwd(const void* x, long n, const float* w, void* y, hipStream_t st);
int p2p_prelu_bwd(const void* x, const void* dy, long n, const float* w, void* dx, float* ws, float* gw,
                  int accumulate, hipStream_t st);
int p2p_tv_fwd(const void* x, int N, int H, int W, int C, float* ws, float* out, hipStream_t st);
int p2p_tv_bwd(const void* x, int N, int H, int W, int C, const float* gout, void* dx, hipStream_t st);
int p2p_quantize(const void* x, long n, int bits, void* y, hipStream_t st);
int p2p_quantize_unshuffle(const void* x, int N, int H, int W, int C, int bits, int r, void* y, void* yu, int Cp,
                           hipStream_t st);
int p2p_metrics_ws(int C, int H, int W);
int p2p_image_metrics(const void* a, const void* b, int dtype, const long* strides, int N, int C, int H, int W,
                      int shift, double data_range, double* ws, hipStream_t st);
int p2p_avgpool3s2(const void* x, int N, int H, int W, int C, int OH, int OW, void* y, int bwd, hipStream_t st);
int p2p_maxpool2(const void* x, const void* gy, int N, int H, int W, int C, void* out, hipStream_t st);
int p2p_l2norm(const void* x, const void* gy, long P, int C, float eps, const void* res, void* out, int r, int IH,
               int IW, hipStream_t st);
int p2p_pixel_shuffle(const void* in, int N, int OH, int OW, int OC, int r, int dir, void* out,
                      hipStream_t st);
int p2p_weight_prep_pairs(int count, const float* const* w, void* const* out0, void* const* out1,
                          const int* A, const int* B, const int* T, const int* Xa, const int* Xb,
                          int* const* site, hipStream_t st);
int p2p_m32_enabled();
int p2p_set_m32(int on);
long p2p_wgrad_reduce_extra(int splits, long slab);
int p2p_oob_counts(unsigned int* out4, int reset);
int p2p_oob_selftest(void* scratch, hipStream_t st);
int p2p_conv_fwd_m32(const p2p::ConvFwdArgs* a, int mode, int variant, hipStream_t st);
int p2p_conv_m32_rows(const p2p::ConvFwdArgs* a, int mode, int variant);
int p2p_dgrad_c1(const void* dy, int dyC, int N, int H, int W, const float* w, int KH, int KW, int pad, int OH,
                 int OW, int Cp, const float* alpha, void* dx, hipStream_t st);
int p2p_up2_dgrad_image(const float* w, int Cout, int Cin, int Xp, int Yp, void* out, hipStream_t st);
int p2p_col_weight(const void* w, int T, int C, int Cv, int Cvp, int Ncol, void* out, hipStream_t st);
int p2p_vec_pad(const float* x, int n, float fill, int nout, float* out, hipStream_t st);
int p2p_pad_fold(const void* dxp, int N, int H, int W, int C, int pad, int up, int reflect,
                 const void* xb, int act, const void* res, void* dx, hipStream_t st);
int p2p_fold_band_nb_blocks();
int p2p_fold_band(const void* fb, int N, int H, int W, int C, int pad, int edge, const void* xb, int act, void* dx,
                  float* nb_ws, long nb_plane, int nb_chunk0, const void* nb_x, const float* nb_mean,
                  const float* nb_rstd, const float* nb_gamma, const float* nb_beta, const float* nb_prelu,
                  int nb_act, hipStream_t st);
int p2p_pad_channels(const void* a, int Ca, const void* b, int Cb, long P, int Co, void* out,
                     hipStream_t st);
int p2p_slice_channels(const void* in, int Ci, int c0, long P, int C, void* out, hipStream_t st);
int p2p_colsum_blocks(long M, int C);
int p2p_colsum(const void* x, long M, int C, float scale, int accumulate, float* ws, float* out, int Cout,
               hipStream_t st);
int p2p_loss_blocks(long n);
int p2p_loss_fwd(const void* a, const void* b, int is_f32, long n, int kind, float t, float scale,
                 float* ws, float* out, hipStream_t st);
int p2p_loss_bwd(const void* a, const void* b, int is_f32, long n, int kind, float t, float scale,
                 const float* gout, void* ga, void* gb, hipStream_t st);
int p2p_adam_max_tensors();
int p2p_union_weight(const float* w, int CinT, int CoutT, int co_off, int nv, int Nrows, int Cpad,
                     const float* bias, void* out, float* bias_out, hipStream_t st);
int p2p_sum_partials(const float* ws, int nb, float scale, float* out, hipStream_t st);
int p2p_sum_long(const float* ws, long n, float scale, float* part, float* out, hipStream_t st);
int p2p_rowsum_blocks(long R);
long p2p_s2t_dbg_bytes();
int p2p_s2t_dbg_read(void* dst, long bytes);
int p2p_rowsum_f32(const float* ws, long R, int C, float* tmp, float* out, hipStream_t st);
int p2p_lincomb(const float* a, const float* b, float wa, float wb, float c, long n, float* out, hipStream_t st);
int p2p_i64_add(long long* t, long long v, long n, hipStream_t st);
int p2p_lincomb_n(const float* const* p, const float* w, int n, float* out, hipStream_t st);
int p2p_scale_n(const float* g, const float* w, int n, float* out, hipStream_t st);
int p2p_guard_flag(const float* const* v, int n, float* flag, float* counter, hipStream_t st);
int p2p_adam(int count, float* const* p, const float* const* g, float* const* m, float* const* v,
             const long* n, const float* lr, const float* step, const float* skip, float b1, float b2,
             float eps, float wd, hipStream_t st);
}

namespace {

using at::Tensor;
using c10::optional;

hipStream_t cur_stream(const Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void check_act(const Tensor& t, const char* name, bool allow_fp8 = false) {
  TORCH_CHECK(t.is_cuda(), name, ": expected a GPU tensor");
  const auto dt = t.scalar_type();
  TORCH_CHECK(dt == at::kBFloat16 || (allow_fp8 && (dt == at::kFloat8_e4m3fn || dt == at::kFloat8_e5m2)), name,
              ": expected bf16", allow_fp8 ? " or fp8" : "", ", got ", dt);
  TORCH_CHECK(t.dim() == 4, name, ": expected NCHW-shaped tensor");
  TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), name,
              ": expected channels_last (NHWC) memory");
  TORCH_CHECK(t.size(1) % 8 == 0, name, ": channels must be a multiple of 8, got ", t.size(1));
}

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, ": HIP launch failed: ", hipGetErrorString((hipError_t)rc));
}

// 4 KB of zeros per device: the padding source of the global_load_lds conv variant
const void* zero_page(const Tensor& like) {
  static std::vector<Tensor> pages(64);
  const int d = like.device().index();
  if (!pages[d].defined()) pages[d] = at::zeros({4096}, like.options().dtype(at::kByte));
  return pages[d].data_ptr();
}


// conv kernel variant: P2P_CONV_VARIANT = v1 (register-staged) | g2 | g3 | g4 (LDS-DMA
// rings) | unset = auto: g4 (256x128 tile, 8 waves, 3-stage ring) for Cout > 64, g2
// (128x64, 2-stage) below -- the per-layer winners of tools/conv_bench.py on MI355X
// (profiles/conv_variants_r1.jsonl).
// glds tile variant: 4 = 256x128 3-stage (one 144 KB block per CU), 2 = 128-row 2-stage
// (two blocks per CU).  A GEMM with only a few K tiles (packed 8-channel inputs / dgrads
// of the image layers) spends most of a block's life in prologue and epilogue, which only
// overlap across blocks when two fit on a CU.
// 5 = 256x256 2-stage (Cout > 128 only; 8 waves of 128x64 -> a quarter less LDS fragment
// traffic and half the A re-reads per MFMA of variant 4).
// Auto: 5 when it still yields >= 256 tiles (one per CU; measured: it wins on every such
// U-Net / PatchGAN layer and loses below, profiles/conv_layers_r1d.jsonl), else 4 / 2.
int conv_variant(int64_t Cout, int64_t kmax, int64_t tiles256 = 0) {
  const char* v = std::getenv("P2P_CONV_VARIANT");   // per call: tests force tiles per case
  if (v && v[0] == 'v') return 1;
  const int v4 = (Cout > 64 && kmax > 256) ? 4 : 2;
  const bool big = Cout > 128 && kmax > 256;
  if (v && v[0] == 'g' && v[1] >= '2' && v[1] <= '4') return v[1] - '0';
  if (v && v[0] == 'g' && v[1] == '5') return big ? 5 : v4;
  if (v && v[0] == 'g' && v[1] == '6') return (Cout <= 64 && kmax > 256) ? 6 : ((big && tiles256 >= 256) ? 5 : v4);
  if (v && v[0] == 'g' && v[1] == '8') {   // g8: 256x64 for N <= 64; g89: also 256x128 for N <= 128
    if (Cout <= 64 && kmax > 256) return 8;
    if (v[2] == '9' && Cout <= 128 && kmax > 256) return 9;
  }
  if (v && v[0] == 'g' && v[1] == '9' && Cout > 64 && Cout <= 128 && kmax > 256) return 9;
  return (big && tiles256 >= 256) ? 5 : v4;
}

void check_site(const Tensor& site) {
  TORCH_CHECK(site.is_cuda() && site.scalar_type() == at::kInt && site.numel() >= 4 && site.is_contiguous(),
              "fp8: a scale site is a contiguous int32 GPU tensor of 4 words");
}

Tensor empty_nhwc(int64_t N, int64_t C, int64_t H, int64_t W, const Tensor& like) {
  return at::empty({N, C, H, W}, like.options().memory_format(at::MemoryFormat::ChannelsLast));
}

// ------------------------------------------------------------------ conv fwd / dgrad
std::vector<Tensor> conv_fwd(const Tensor& x1, const optional<Tensor>& x2, const Tensor& w,
                             const optional<Tensor>& bias, int64_t mode, int64_t KH, int64_t KW,
                             int64_t stride, int64_t pad, int64_t reflect, int64_t up,
                             int64_t act_in, int64_t OH, int64_t OW, int64_t Cout, int64_t act_out,
                             int64_t Csplit, const optional<Tensor>& xb1,
                             const optional<Tensor>& xb2, int64_t act_bwd, int64_t Cvalid,
                             bool want_stats, const optional<Tensor>& qs_x1,
                             const optional<Tensor>& qs_x2, const optional<Tensor>& qs_w,
                             const optional<Tensor>& y_qsite, int64_t y_qfmt,
                             const optional<Tensor>& res, const optional<Tensor>& alpha,
                             const optional<Tensor>& nb_x, const optional<Tensor>& nb_mean,
                             const optional<Tensor>& nb_rstd, const optional<Tensor>& nb_gamma,
                             const optional<Tensor>& nb_beta, int64_t nb_act, int64_t nb_half, bool nb_batch,
                             bool nb_colsum, bool nb_gate, int64_t fold_H, int64_t fold_W, int64_t fold_p,
                             int64_t fold_edge, const optional<Tensor>& nb_prelu) {
  check_act(x1, "conv_fwd x1", true);
  // fp8 operands: x e4m3 (activations) or e5m2 (gradients), weight image e4m3, each with
  // an fp8 scale site (csrc/fp8.hip); outputs stay bf16
  const int fp8 = x1.scalar_type() == at::kFloat8_e4m3fn ? 1 : (x1.scalar_type() == at::kFloat8_e5m2 ? 2 : 0);
  const Tensor obf = fp8 ? at::empty({0}, x1.options().dtype(at::kBFloat16)) : x1;
  const int64_t N = x1.size(0), H = x1.size(2), W = x1.size(3);
  int64_t C2 = 0;
  if (x2) {
    check_act(*x2, "conv_fwd x2", true);
    TORCH_CHECK(x2->scalar_type() == x1.scalar_type(), "conv_fwd: concat halves must share a dtype");
    TORCH_CHECK(x2->size(0) == N && x2->size(2) == H && x2->size(3) == W, "conv_fwd: concat shape");
    C2 = x2->size(1);
  }
  const int64_t C1 = x1.size(1), C = C1 + C2;
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == (fp8 ? at::kFloat8_e4m3fn : at::kBFloat16) && w.is_contiguous(),
              "conv_fwd: weight (bf16, or e4m3 with fp8 activations)");
  if (fp8) {
    auto site_ok = [](const optional<Tensor>& t) {
      return t.has_value() && t->is_cuda() && t->scalar_type() == at::kInt && t->numel() >= 4 && t->is_contiguous();
    };
    TORCH_CHECK(site_ok(qs_x1) && site_ok(qs_w) && (!x2 || site_ok(qs_x2)), "conv_fwd: fp8 needs scale sites");
  }
  TORCH_CHECK(w.numel() >= Cout * KH * KW * C, "conv_fwd: weight too small for the GEMM view");
  TORCH_CHECK(Cout % 8 == 0 && Csplit % 8 == 0 && Csplit > 0 && Csplit <= Cout, "conv_fwd: Cout/Csplit");
  TORCH_CHECK(mode == 0 || mode == 1, "conv_fwd: mode");
  TORCH_CHECK(up == 1 || up == 2, "conv_fwd: upsample must be 1 or 2");
  TORCH_CHECK(mode == 0 || (up == 1 && reflect == 0), "conv_fwd: CONVT mode has no pad/upsample folds");
  if (reflect) TORCH_CHECK(pad < H * up && pad < W * up, "conv_fwd: reflect pad too large");
  if (bias) TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() >= Cout, "conv_fwd: bias");
  // pad fold of an input gradient computed on a padded grid (conv.h fold_buf): y1, xb1 and
  // res are real-grid (fold_H x fold_W) tensors.  Reflect: a MODE-1 dgrad onto the reflect-
  // padded grid; edge: the MODE-0 4x4 stride-2 dgrad of nearest-x2 + reflect-1 (ops/hip.py)
  const bool fold = fold_p > 0;
  if (fold)
    TORCH_CHECK(((mode == 1 && pad == 0 && !fold_edge) || (mode == 0 && fold_edge && fold_p <= 2)) && up == 1 &&
                    !reflect && !x2 && Csplit == Cout && !want_stats && !y_qsite && (!nb_x || nb_batch) &&
                    !nb_colsum &&
                    OH == fold_H + 2 * fold_p && OW == fold_W + 2 * fold_p,
                "conv_fwd: fold geometry");
  const int64_t RH = fold ? fold_H : OH, RW = fold ? fold_W : OW;
  if (act_bwd) {
    TORCH_CHECK(xb1.has_value(), "conv_fwd: act_bwd needs xb1");
    check_act(*xb1, "xb1");
    TORCH_CHECK(xb1->size(1) == Csplit && xb1->size(2) == RH && xb1->size(3) == RW, "xb1 shape");
    if (Csplit < Cout && xb2.has_value()) {   // no xb2: the second half is not gated
      check_act(*xb2, "xb2");
      TORCH_CHECK(xb2->size(1) == Cout - Csplit, "xb2 shape");
    }
  }
  Tensor y1 = empty_nhwc(N, Csplit, RH, RW, obf);
  Tensor fbuf;   // fold: the padded-grid gradient (only its frame is written in the epilogue route)
  if (fold) fbuf = empty_nhwc(N, Cout, OH, OW, obf);
  Tensor y2;
  if (Csplit < Cout) y2 = empty_nhwc(N, Cout - Csplit, OH, OW, obf);

  p2p::ConvFwdArgs a{};
  a.x1 = x1.data_ptr();
  a.x2 = x2 ? x2->data_ptr() : nullptr;
  a.C1 = (int)C1;
  a.C2 = (int)C2;
  a.C = (int)C;
  a.N = (int)N;
  a.H = (int)H;
  a.W = (int)W;
  a.up = (int)up;
  a.KH = (int)KH;
  a.KW = (int)KW;
  a.stride = (int)stride;
  a.pad = (int)pad;
  a.reflect = (int)reflect;
  a.act_in = (int)act_in;
  a.OH = (int)OH;
  a.OW = (int)OW;
  a.Cout = (int)Cout;
  a.w = w.data_ptr();
  a.bias = bias ? bias->data_ptr<float>() : nullptr;
  if (alpha)
    TORCH_CHECK(alpha->is_cuda() && alpha->scalar_type() == at::kFloat && alpha->numel() == 1,
                "conv_fwd: alpha must be a 1-element fp32 GPU tensor");
  a.alpha = alpha ? alpha->data_ptr<float>() : nullptr;
  a.act_out = (int)act_out;
  a.y1 = y1.data_ptr();
  a.y2 = y2.defined() ? y2.data_ptr() : nullptr;
  a.Csplit = (int)Csplit;
  a.xb1 = act_bwd ? xb1->data_ptr() : nullptr;
  a.xb2 = (act_bwd && Csplit < Cout && xb2) ? xb2->data_ptr() : nullptr;
  a.act_bwd = (int)act_bwd;
  a.res1 = nullptr;
  if (res) {
    check_act(*res, "conv_fwd res");
    TORCH_CHECK(Csplit == Cout && res->size(0) == N && res->size(1) == Cout && res->size(2) == RH &&
                    res->size(3) == RW,
                "conv_fwd: res must match the (unsplit) output");
    a.res1 = res->data_ptr();
  }
  a.ws = nullptr;
  a.splits = 1;
  a.zero = zero_page(x1);
  a.stats = nullptr;
  a.stats_nchunks = 0;
  a.fp8 = fp8;
  a.qs_x1 = fp8 ? qs_x1->data_ptr<int>() : nullptr;
  a.qs_x2 = (fp8 && x2) ? qs_x2->data_ptr<int>() : nullptr;
  a.qs_w = fp8 ? qs_w->data_ptr<int>() : nullptr;
  a.q_out = nullptr;
  a.q_site = nullptr;
  a.q_fmt = 0;

  hipStream_t st = cur_stream(x1);
  // ---- tiny-Cout "col" path: dense GEMM over the input pixels (N = taps x Cvalid) + col2im
  const int64_t Cv = Cvalid > 0 ? Cvalid : Cout;
  if (Cout <= 16 && Cv <= 16 && Csplit == Cout && !reflect && up == 1 && C1 % 64 == 0 &&
      C2 % 64 == 0 && !fold) {
    TORCH_CHECK(!fp8, "conv_fwd: fp8 is not supported on the tiny-Cout col path");
    TORCH_CHECK(!res, "conv_fwd: no residual on the tiny-Cout col path");
    TORCH_CHECK(!alpha, "conv_fwd: no alpha on the tiny-Cout col path");
    // col[i][t*Cvp + co]: each tap's outputs padded to Cvp (4 / 8 / 16) so col2im reads
    // one aligned vector per tap
    const int64_t T = KH * KW;
    const int64_t Cvp = Cv <= 2 ? Cv : (Cv <= 4 ? 4 : (Cv <= 8 ? 8 : 16));
    const int64_t Ncol = ((T * Cvp + 7) / 8) * 8;
    Tensor wv = at::empty({Ncol, C}, w.options());
    TORCH_CHECK(w.is_contiguous() && w.scalar_type() == at::kBFloat16 && w.numel() >= Cout * T * C,
                "conv_fwd(col): bf16 weight image [Cout][T][C]");
    check_rc(p2p_col_weight(w.data_ptr(), (int)T, (int)C, (int)Cv, (int)Cvp, (int)Ncol, wv.data_ptr(), st),
             "conv_fwd(col weight)");
    Tensor col = empty_nhwc(N, Ncol, H, W, obf);
    p2p::ConvFwdArgs g = a;
    g.KH = g.KW = 1;
    g.stride = 1;
    g.pad = 0;
    g.OH = (int)H;
    g.OW = (int)W;
    g.Cout = (int)Ncol;
    g.Csplit = (int)Ncol;
    g.w = wv.data_ptr();
    g.bias = nullptr;
    g.act_out = 0;
    g.act_bwd = 0;
    g.xb1 = g.xb2 = nullptr;
    g.y1 = col.data_ptr();
    g.y2 = nullptr;
    int grc = -2;
    // Ncol <= 32 (the PatchGAN logits: 16 taps x 1 channel): the 256x32 glds tile streams
    // the wide input once at full rate (the register-staged 256x16 kernel ran at ~1/3 of it)
    if (act_in == 0 || act_in == 1)
      grc = p2p_conv_fwd_glds(&g, 0, Ncol > 32 ? conv_variant(Ncol, C) : 7, st);
    if (grc == -2) {
      const int gbn = Ncol <= 16 ? 16 : (Ncol <= 32 ? 32 : (Ncol <= 64 ? 64 : 128));
      const int gbm = gbn <= 32 ? 256 : 128;
      grc = p2p_conv_fwd(&g, 0, gbm, gbn, st);
    }
    check_rc(grc, "conv_fwd(col gemm)");
    check_rc(p2p_col2im((int)mode, col.data_ptr(), (int)Ncol, (int)N, (int)H, (int)W, (int)OH, (int)OW,
                        (int)KH, (int)KW, (int)stride, (int)pad, (int)Cv, (int)Cout, a.bias,
                        (int)act_out, act_bwd ? xb1->data_ptr() : nullptr, (int)act_bwd, y1.data_ptr(),
                        st),
             "col2im");
    return {y1};
  }

  // ---- tile choice: N-tile from Cout, M-tile from the largest parity class
  const int classes = mode == 0 ? 1 : (int)(stride * stride);
  int64_t mmax = 0;
  int64_t kmax = 0;
  for (int c = 0; c < classes; ++c) {
    int64_t hq = OH, wq = OW, taps = KH * KW;
    if (mode == 1) {
      const int ry = c / (int)stride, rx = c % (int)stride;
      hq = OH > ry ? (OH - ry + stride - 1) / stride : 0;
      wq = OW > rx ? (OW - rx + stride - 1) / stride : 0;
      const int ky0 = (int)((ry + pad) % stride), kx0 = (int)((rx + pad) % stride);
      const int64_t tj = ky0 < KH ? (KH - ky0 + stride - 1) / stride : 0;
      const int64_t ti = kx0 < KW ? (KW - kx0 + stride - 1) / stride : 0;
      taps = tj * ti;
    }
    mmax = std::max(mmax, N * hq * wq);
    kmax = std::max(kmax, taps * C);
  }
  const int variant = conv_variant(Cout, kmax, ((mmax + 255) / 256) * ((Cout + 255) / 256) * classes);
  const bool glds_ok = variant > 1 && Cout > 32 && (act_in == 0 || act_in == 1);
  int bm, bn;
  if (glds_ok) {
    bn = variant == 5 ? 256 : (Cout > 64 ? 128 : 64);
    bm = (variant == 4 || variant == 5 || variant == 6 || variant == 8 || variant == 9) ? 256 : 128;
  } else if (Cout <= 16) {
    bn = 16;
    bm = mmax >= 4096 ? 256 : 64;
  } else if (Cout <= 32) {
    bn = 32;
    bm = 256;
  } else if (Cout <= 64) {
    bn = 64;
    bm = mmax >= 8192 ? 128 : 64;
  } else {
    bn = 128;
    bm = mmax >= 16384 ? 128 : 64;
  }
  const int64_t tiles = ((mmax + bm - 1) / bm) * ((Cout + bn - 1) / bn) * classes;
  const int64_t ktiles = (kmax + (fp8 ? 127 : 63)) / (fp8 ? 128 : 64);
  int splits = 1;
  if (tiles < 256 && ktiles >= 8) {
    splits = (int)std::min<int64_t>((512 + tiles - 1) / tiles, ktiles / 4);
    splits = std::max(1, std::min(splits, 32));
    // no empty split: the kernel gives split s the k tiles [s*kps, (s+1)*kps), and every
    // split's slab must be written whole (it is not zero-filled)
    for (int it = 0; it < 4; ++it) {
      const int64_t kps = (ktiles + splits - 1) / splits;
      splits = (int)((ktiles + kps - 1) / kps);
    }
  }
  // stride-2 4x4 transposed convs onto 32x32 / 64x64 grids (U-Net decoder ConvT, every 4x4
  // s2 conv's input gradient): the class-shared halo kernel (csrc/conv_s2t.hip).  Its tiles
  // are BM = 128 rows of one class, which fixes the stats / partial chunk layout below.
  // 32- and 64-wide grids with K = 4 taps x C <= 1024 (C = 512, U-Net d3 / d6 ConvT, runs
  // at 830+ TF/s on the 256x128 implicit-GEMM tile; profiles/kernel_experiments_r4.md).
  // fp8 (e4m3 activations / e5m2 gradients): the same layers on 128-channel chunks (the
  // 128-B halo pixel of the bf16 kernel); no input activation on gradients, no extended
  // epilogue on activations (as the implicit-GEMM fp8 tiles)
  const int64_t s2t_chc = fp8 ? 128 : 64;
  const bool s2t_ok = mode == 1 && splits == 1 && KH == 4 && KW == 4 && stride == 2 && pad == 1 &&
                      !reflect && up == 1 && OH == 2 * H && OW == 2 * W &&
                      W == 64 &&
                      (H * W) % 128 == 0 && Cout % 64 == 0 && C1 % s2t_chc == 0 && C2 % s2t_chc == 0 &&
                      C1 + C2 >= s2t_chc && C1 + C2 <= 256 &&
                      (act_in == 0 || (act_in == 1 && act_bwd == 0 && !res)) && act_out <= 2 &&
                      (fp8 != 2 || act_in == 0) && (fp8 != 1 || (!act_bwd && !res)) &&
                      (!fp8 || (s2t_f8_mask() & (int)fp8)) && std::getenv("P2P_NO_S2T") == nullptr;
  if (s2t_ok) bm = 128;
  // the 512 x 128 m32 tile: its fused-statistics / norm-partial chunks are 512 rows (one
  // predicate with the kernel's own routing, conv_fwd_m32.hip p2p_conv_m32_rows)
  if (!s2t_ok && glds_ok && splits == 1 && p2p_m32_enabled() && p2p_conv_m32_rows(&a, (int)mode, variant) == 512)
    bm = 512;
  if (P2P_KNOB_ONCE("P2P_ROUTE_LOG"))   // routing trace (tools): one line per conv call
    fprintf(stderr, "[route] mode %d N %ld C %ld+%ld %ldx%ld -> %ld %ldx%ld k%d s%d p%d act_in %d act_bwd %d res %d "
            "fp8 %d splits %d s2t %d bm %d bn %d tiles %ld\n", (int)mode, (long)N, (long)C1, (long)C2, (long)H,
            (long)W, (long)Cout, (long)OH, (long)OW, (int)KH, (int)stride, (int)pad, (int)act_in, (int)act_bwd,
            res ? 1 : 0, (int)fp8, splits, (int)s2t_ok, (int)bm, (int)bn, (long)tiles);
  Tensor ws;
  if (splits > 1) {
    // per-split fp32 slabs (plain stores, no zero fill) summed in split order by
    // conv_finalize: deterministic, and no atomics
    a.det = 1;
    ws = at::empty({splits, N * OH * OW, Cout}, obf.options().dtype(at::kFloat));
    a.ws = ws.data_ptr<float>();
    a.splits = splits;
  }
  // fused norm statistics: only on the glds path with whole tiles inside one image/class
  Tensor stats;
  if (want_stats && (glds_ok || s2t_ok) && splits == 1 && Csplit == Cout && act_out == 0 && !act_bwd) {
    bool ok = true;
    int64_t hwq = OH * OW;
    if (mode == 1) {
      ok = OH % stride == 0 && OW % stride == 0;
      hwq = (OH / stride) * (OW / stride);
    }
    ok = ok && hwq % bm == 0;
    if (ok) {
      const int64_t nch = classes * (hwq / bm);
      stats = at::empty({2, N, nch, Cout}, x1.options().dtype(at::kFloat));
      a.stats = stats.data_ptr<float>();
      a.stats_nchunks = (int)nch;
    }
  }
  // fused norm-backward partials (dgrad epilogue): half nb_half (1 = channels [0, Csplit),
  // 2 = [Csplit, Cout)) is the gradient of a norm's output; same tile constraints as stats
  Tensor nbp;
  a.nb_ws = nullptr;
  // the packed-image halo kernel (below) beats the generic tile with fused partials: keep it
  const bool pk8_halo = mode == 0 && !fp8 && C1 == 8 && C2 == 0 && KH == 4 && KW == 4 && stride == 2 && pad == 1 &&
                        (Cout == 64 || Cout == 128) && std::getenv("P2P_NO_HALO") == nullptr;
  // affine / PReLU norms: batch norm only, on the implicit-GEMM tiles (the s2t kernel has its
  // own partial code, non-affine only; the halo kernels none -- keep their routes).  Never with a
  // pad fold: the fold dgrads' partials (round 5, opt-in) measured slower than the norm's own
  // pass and were removed in round 6 (profiles/kernel_experiments_r5.md section 12)
  const bool nb_ext = nb_gamma || nb_prelu;
  const bool nb_halo = KH == 9 || (KH == 3 && C1 == 64 && Cout <= 32);
  const int64_t nb_band = 0;
  if ((nb_x || nb_colsum) && nb_half && (glds_ok || s2t_ok) && splits == 1 && fp8 != 1 && !want_stats && !fold &&
      !pk8_halo && (!nb_ext || (nb_batch && !nb_colsum && !s2t_ok && !nb_halo && nb_band >= 0 && nb_half == 1 &&
                                Csplit == Cout))) {
    const int64_t c0 = nb_half == 1 ? 0 : Csplit;
    const int64_t nC = nb_half == 1 ? Csplit : Cout - Csplit;
    bool ok = nC > 0 && nC % 8 == 0 && (nb_half == 1 || Csplit < Cout);
    int64_t hwq = OH * OW;
    if (mode == 1) {
      ok = ok && OH % stride == 0 && OW % stride == 0;
      hwq = (OH / stride) * (OW / stride);
    }
    // batch-norm extension: flat tiles over all images (every class N * hwq pixels)
    const bool flat = nb_ext;
    const int64_t tiles_cls = (N * hwq + bm - 1) / bm;
    ok = ok && (flat || hwq % bm == 0);
    if (ok && !nb_colsum) {
      check_act(*nb_x, "conv_fwd nb_x");
      TORCH_CHECK(nb_x->size(0) == N && nb_x->size(1) == nC && nb_x->size(2) == RH && nb_x->size(3) == RW,
                  "conv_fwd: nb_x must match the gradient half");
      const int64_t groups = nb_batch ? 1 : N;
      TORCH_CHECK(nb_mean && nb_rstd && nb_mean->numel() == groups * nC && nb_rstd->numel() == groups * nC &&
                      nb_mean->scalar_type() == at::kFloat && nb_rstd->scalar_type() == at::kFloat,
                  "conv_fwd: nb mean / rstd");
    }
    if (ok) {
      if (nb_gamma) TORCH_CHECK(nb_beta && nb_gamma->numel() == nC && nb_beta->numel() == nC, "conv_fwd: nb affine");
      if (nb_prelu)
        TORCH_CHECK(nb_prelu->numel() == 1 && nb_prelu->scalar_type() == at::kFloat && nb_prelu->is_cuda(),
                    "conv_fwd: nb_prelu must be a 1-element fp32 GPU tensor");
      const int64_t planes = nb_prelu ? 3 : 2;
      const int64_t nch = flat ? classes * tiles_cls + std::max<int64_t>(nb_band, 0) : classes * (hwq / bm);
      nbp = flat ? at::empty({planes, 1, nch, nC}, x1.options().dtype(at::kFloat))
                 : at::empty({2, N, nch, nC}, x1.options().dtype(at::kFloat));
      a.nb_colsum = nb_colsum ? 1 : 0;
      a.nb_x = nb_colsum ? nullptr : nb_x->data_ptr();
      a.nb_mean = nb_colsum ? nullptr : nb_mean->data_ptr<float>();
      a.nb_rstd = nb_colsum ? nullptr : nb_rstd->data_ptr<float>();
      a.nb_gamma = nb_gamma ? nb_gamma->data_ptr<float>() : nullptr;
      a.nb_beta = nb_gamma ? nb_beta->data_ptr<float>() : nullptr;
      a.nb_prelu = nb_prelu ? nb_prelu->data_ptr<float>() : nullptr;
      a.nb_act = (int)nb_act;
      a.nb_gate = (nb_gate && !nb_colsum && nb_act == 0 && !nb_gamma && !nb_prelu) ? 1 : 0;
      a.nb_batch = nb_batch ? 1 : 0;
      a.nb_c0 = (int)c0;
      a.nb_C = (int)nC;
      a.nb_nchunks = (int)nch;
      a.nb_flat = flat ? 1 : 0;
      a.nb_tiles_cls = (int)tiles_cls;
      a.nb_planes = (int)planes;
      a.nb_ws = nbp.data_ptr<float>();
    }
  }
  // fp8 shadow of y (the next conv's operand) from the epilogue: plain single-output GEMMs
  Tensor yq;
  if (y_qsite && splits == 1 && Csplit == Cout && !act_bwd) {
    check_site(*y_qsite);
    yq = at::empty_like(y1, y1.options().dtype(y_qfmt == 0 ? at::kFloat8_e4m3fn : at::kFloat8_e5m2),
                        at::MemoryFormat::ChannelsLast);
    a.q_out = yq.data_ptr();
    a.q_site = y_qsite->data_ptr<int>();
    a.q_fmt = (int)y_qfmt;
  }
  // stride-1 9x9 convs with 8-32 input channels and <= 32 outputs (family R's full-res
  // layers): the halo-tile direct conv (csrc/halo_kxk.hip); MODE 1 stride 1 = flipped taps
  const bool halo_geo = (KH == 9 && KW == 9 && (C1 == 8 || C1 == 16 || C1 == 32) && Cout <= 32) ||
                        (KH == 3 && KW == 3 && C1 == 64 && Cout <= 32);
  const bool halo_cond = !fp8 && C2 == 0 && halo_geo && stride == 1 && Csplit == Cout && act_in == 0 &&
                         act_bwd == 0 && !a.res1 && !a.q_out && !a.stats && !a.nb_ws && !a.alpha &&
                         (mode == 0 || (up == 1 && !reflect && pad <= KH - 1)) &&
                         std::getenv("P2P_NO_HALO") == nullptr;
  // reflect fold: in the implicit-GEMM epilogue or the halo kernel's store loop (interior
  // pixels straight into y1, the frame folded by fold_band); the split-K route writes the whole
  // padded grid and pad_fold folds it afterwards (gate and skip gradient applied there)
  bool fold_late = false;
  if (fold) {
    const int64_t bw = fold_edge ? 1 : fold_p;   // band rows / columns per side (elementwise.hip fold_band)
    // (the halo kernel folds in its store loop too: interior to y1, frame to fold_buf)
    fold_late = splits > 1 || fold_H < 2 * bw + 2 || fold_W < 2 * bw + 2;
    if (fold_late) {
      a.y1 = fbuf.data_ptr();
      a.xb1 = nullptr;
      a.act_bwd = 0;
      a.res1 = nullptr;
    } else {
      a.fold_buf = fbuf.data_ptr();
      a.fold_H = (int)fold_H;
      a.fold_W = (int)fold_W;
      a.fold_p = (int)fold_p;
    }
  }
  int rc = -2;
  // packed 8-channel image convs (4x4 s2 p1): the halo-tile kernel (csrc/halo_pk8.hip)
  if (mode == 0 && !fp8 && C1 == 8 && C2 == 0 && KH == 4 && KW == 4 && stride == 2 && pad == 1 && !reflect &&
      up == 1 && act_in == 0 && splits == 1 && !a.stats && !a.nb_ws && !a.res1 && !a.alpha && (Cout == 64 || Cout == 128) &&
      std::getenv("P2P_NO_HALO") == nullptr) {
    p2p::HaloPk8Args h{};
    h.x = static_cast<const __bf16*>(x1.data_ptr());
    h.Hi = (int)H;
    h.Wi = (int)W;
    h.Ho = (int)OH;
    h.Wo = (int)OW;
    h.w = static_cast<const __bf16*>(w.data_ptr());
    h.bias = a.bias;
    h.Cout = (int)Cout;
    h.act_out = (int)act_out;
    h.y1 = static_cast<__bf16*>(a.y1);
    h.y2 = static_cast<__bf16*>(a.y2);
    h.Csplit = (int)Csplit;
    h.xb1 = static_cast<const __bf16*>(a.xb1);
    h.xb2 = static_cast<const __bf16*>(a.xb2);
    h.zero = static_cast<const __bf16*>(a.zero);
    h.tiles_x = (int)((OW + 15) / 16);
    h.tiles_y = (int)((OH + 15) / 16);
    h.ntiles = (int)N * h.tiles_x * h.tiles_y;
    h.q = static_cast<uint8_t*>(a.q_out);
    h.q_site = a.q_site;
    h.q_fmt = a.q_fmt;
    const bool gate_ok = act_bwd == 0 || act_bwd == 1;
    if (gate_ok && (act_bwd == 0 || Cout == 128) && OH == (H + 2 - 4) / 2 + 1 && OW == (W + 2 - 4) / 2 + 1) {
      if (act_bwd == 0) h.xb1 = h.xb2 = nullptr;
      int dev = 0, cus = 256;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      const int per_cu = Cout == 128 ? 1 : 2;   // halo_pk8.hip launch bounds
      rc = p2p_halo_pk8(&h, std::max(1, std::min(h.ntiles, per_cu * cus)), st);
    }
  }
  if (rc == -2 && halo_cond) {
    p2p::HaloKArgs h{};
    h.x = static_cast<const __bf16*>(x1.data_ptr());
    h.C = (int)C1;
    h.N = (int)N;
    h.H = (int)H;
    h.W = (int)W;
    h.up = (int)up;
    h.pad = mode == 0 ? (int)pad : (int)(KH - 1 - pad);
    h.reflect = (int)reflect;
    h.flip = mode == 1 ? 1 : 0;
    h.OH = (int)OH;
    h.OW = (int)OW;
    h.w = static_cast<const __bf16*>(w.data_ptr());
    h.bias = a.bias;
    h.Cout = (int)Cout;
    h.act_out = (int)act_out;
    h.y = static_cast<__bf16*>(a.y1);
    h.zero = static_cast<const __bf16*>(a.zero);
    h.tiles_x = (int)((OW + 15) / 16);
    h.tiles_y = (int)((OH + 15) / 16);
    h.ntiles = (int)N * h.tiles_x * h.tiles_y;
    h.fold_buf = static_cast<__bf16*>(a.fold_buf);
    h.fold_H = a.fold_H;
    h.fold_W = a.fold_W;
    h.fold_p = a.fold_p;
    if (OH == H * up + 2 * h.pad - KH + 1 && OW == W * up + 2 * h.pad - KW + 1) {
      int dev = 0, cus = 256;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      rc = p2p_halo_kxk(&h, (int)KH, std::max(1, std::min(h.ntiles, cus)), st);
      if (rc == 0) splits = 1;   // no split-K partials to finalize: the halo kernel wrote y
    }
  }
  if (rc == -2 && s2t_ok) {
    rc = p2p_conv_s2t(&a, st);
    TORCH_CHECK(rc != -2, "conv_fwd: the s2t kernel refused a geometry the host accepted");
  }
  // the 32x32x16 MFMA tiles (conv_fwd_m32.hip) take the 256-row bf16 FASTK layers first
  // (fp8: the 32x32x64 f8f6f4 tiles since round 6; P2P_M32_F8=0 -- read per call, the tests A/B
  // it -- keeps fp8 on the 16x16x128 glds tiles)
  const char* m32f8 = fp8 ? std::getenv("P2P_M32_F8") : nullptr;
  const bool m32_f8_on = !(m32f8 && m32f8[0] == '0');
  if (rc == -2 && glds_ok && (!fp8 || m32_f8_on) && p2p_m32_enabled())
    rc = p2p_conv_fwd_m32(&a, (int)mode, variant, st);
  if (rc == -2 && glds_ok) rc = p2p_conv_fwd_glds(&a, (int)mode, variant, st);
  if (rc == -2 && a.stats) {  // glds refused after all: no fused statistics
    a.stats = nullptr;
    stats = Tensor();
  }
  if (rc == -2 && a.nb_ws) {  // the register-staged kernel shares the epilogue, but keep it simple
    a.nb_ws = nullptr;
    nbp = Tensor();
  }
  TORCH_CHECK(!(fp8 && rc == -2), "conv_fwd: no fp8 kernel for this geometry (Cout ", Cout, ", C1 ", C1, ", C2 ",
              C2, ", act_in ", act_in, ")");
  if (rc == -2) {
    // register-staged kernel: its own tile table
    int vbm = bm, vbn = bn;
    if (glds_ok) {
      vbn = Cout > 64 ? 128 : 64;
      vbm = 128;
    }
    rc = p2p_conv_fwd(&a, (int)mode, vbm, vbn, st);
  }
  check_rc(rc, "conv_fwd");
  if (splits > 1) check_rc(p2p_conv_finalize(&a, st), "conv_finalize");
  if (fold) {
    const void* xg = act_bwd ? xb1->data_ptr() : nullptr;
    if (fold_late)
      check_rc(p2p_pad_fold(fbuf.data_ptr(), (int)N, (int)fold_H, (int)fold_W, (int)Cout, (int)fold_p, 1,
                            fold_edge ? 2 : 1, xg,
                            (int)act_bwd, res ? res->data_ptr() : nullptr, y1.data_ptr(), st),
               "conv_fwd(pad_fold)");
    else
      check_rc(p2p_fold_band(fbuf.data_ptr(), (int)N, (int)fold_H, (int)fold_W, (int)Cout, (int)fold_p,
                             (int)fold_edge, xg, (int)act_bwd, y1.data_ptr(), a.nb_ws,
                             a.nb_ws ? (long)a.nb_nchunks * a.nb_C : 0L,
                             a.nb_ws ? a.nb_nchunks - p2p_fold_band_nb_blocks() : 0, a.nb_x, a.nb_mean, a.nb_rstd,
                             a.nb_gamma, a.nb_beta, a.nb_prelu, a.nb_act, st),
               "conv_fwd(fold_band)");
  }
  std::vector<Tensor> out{y1};
  if (y2.defined()) out.push_back(y2);
  if (stats.defined()) out.push_back(stats);
  if (nbp.defined()) out.push_back(nbp);  // dgrad calls only (no stats / fp8 shadow there)
  if (yq.defined()) out.push_back(yq);   // always last (fp8 dtype)
  return out;
}

// ------------------------------------------------------------------ packed-image layers
// GEMM operand (bf16 [Nrows][9][Cpad]) + bias (fp32 [Nrows]) of the 3x3 union conv that
// computes a 4x4 stride-2 pad-1 transposed conv onto a 3-channel image (csrc/image.hip)
std::vector<Tensor> union_weight(const Tensor& w, int64_t co_off, int64_t nv, int64_t Nrows, int64_t Cpad,
                                 const optional<Tensor>& bias) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.is_contiguous() && w.dim() == 4 &&
                  w.size(2) == 4 && w.size(3) == 4,
              "union_weight: fp32 contiguous [CinT][CoutT][4][4] weight");
  TORCH_CHECK(nv >= 1 && nv <= 4 && Nrows >= 16 && Cpad >= w.size(0) && Cpad % 8 == 0 &&
                  co_off + nv <= w.size(1),
              "union_weight: geometry");
  if (bias) TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() >= co_off + nv, "union_weight: bias");
  Tensor img = at::empty({Nrows, 3, 3, Cpad}, w.options().dtype(at::kBFloat16));
  Tensor bu = at::empty({Nrows}, w.options());
  check_rc(p2p_union_weight(w.data_ptr<float>(), (int)w.size(0), (int)w.size(1), (int)co_off, (int)nv, (int)Nrows,
                            (int)Cpad, bias ? bias->data_ptr<float>() : nullptr, img.data_ptr(),
                            bu.data_ptr<float>(), cur_stream(w)),
           "union_weight");
  return {img, bu};
}

// The union GEMM over the [N][H][W] grid of x1 (| x2), writing the packed [N][2H][2W][8]
// image ``out`` through the depth-to-space epilogue (conv.h ``d2s``): mode 1 = image forward
// (returns the device scalar lam_scale * sum|fake - pk_a[3..5]|), mode 2 = head gradient.
Tensor conv_d2s(const Tensor& x1, const optional<Tensor>& x2, const Tensor& w, const Tensor& bias, int64_t act_in,
                int64_t act_out, int64_t mode, Tensor out, const Tensor& pk_a, const optional<Tensor>& pk_f,
                double scale, const optional<Tensor>& wscale) {
  check_act(x1, "conv_d2s x1");
  check_act(pk_a, "conv_d2s pk_a");
  check_act(out, "conv_d2s out");
  const int64_t N = x1.size(0), H = x1.size(2), W = x1.size(3);
  int64_t C2 = 0;
  if (x2) {
    check_act(*x2, "conv_d2s x2");
    TORCH_CHECK(x2->size(0) == N && x2->size(2) == H && x2->size(3) == W, "conv_d2s: concat shape");
    C2 = x2->size(1);
  }
  const int64_t C1 = x1.size(1), C = C1 + C2;
  TORCH_CHECK(C1 % 64 == 0 && C2 % 64 == 0 && C1 <= 1024 && C2 <= 1024, "conv_d2s: channel groups of 64");
  const int64_t nrows = w.numel() / (9 * C);
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.numel() == nrows * 9 * C &&
                  (nrows == 16 || nrows == 32),
              "conv_d2s: union weight [16|32][3][3][C]");
  TORCH_CHECK(bias.scalar_type() == at::kFloat && bias.numel() == nrows, "conv_d2s: union bias");
  TORCH_CHECK(mode == 1 || mode == 2, "conv_d2s: mode");
  TORCH_CHECK(act_in == 0 || act_in == 1, "conv_d2s: input act none / relu");
  for (const Tensor* t : {static_cast<const Tensor*>(&out), &pk_a}) {
    TORCH_CHECK(t->size(0) == N && t->size(1) == 8 && t->size(2) == 2 * H && t->size(3) == 2 * W,
                "conv_d2s: packed image tensors must be [N][8][2H][2W]");
  }
  if (mode == 2) {
    TORCH_CHECK(pk_f.has_value(), "conv_d2s: head gradient needs pk_f");
    check_act(*pk_f, "conv_d2s pk_f");
    TORCH_CHECK(pk_f->sizes() == out.sizes(), "conv_d2s: pk_f shape");
  }
  const float* wsc = nullptr;
  if (wscale) {
    TORCH_CHECK(mode == 2 && wscale->is_cuda() && wscale->scalar_type() == at::kFloat && wscale->numel() == 1,
                "conv_d2s: wscale is a 1-element fp32 device tensor (head gradient only)");
    wsc = wscale->data_ptr<float>();
  }
  hipStream_t st = cur_stream(x1);
  if (nrows == 16) {
    // halo-tile kernel: persistent blocks (one per CU) over 16x16 tiles of the input grid
    p2p::HaloArgs h{};
    h.x1 = static_cast<const __bf16*>(x1.data_ptr());
    h.x2 = x2 ? static_cast<const __bf16*>(x2->data_ptr()) : nullptr;
    h.C1 = (int)C1;
    h.C2 = (int)C2;
    h.N = (int)N;
    h.H = (int)H;
    h.W = (int)W;
    h.w = static_cast<const __bf16*>(w.data_ptr());
    h.bias = bias.data_ptr<float>();
    h.act_out = (int)act_out;
    h.mode = (int)mode;
    h.out = static_cast<__bf16*>(out.data_ptr());
    h.pk_a = static_cast<const __bf16*>(pk_a.data_ptr());
    h.pk_f = mode == 2 ? static_cast<const __bf16*>(pk_f->data_ptr()) : nullptr;
    h.scale = (float)scale;
    h.wscale = wsc;
    h.zero = static_cast<const __bf16*>(zero_page(x1));
    h.tiles_x = (int)((W + 15) / 16);
    h.tiles_y = (int)((H + 15) / 16);
    h.ntiles = (int)N * h.tiles_x * h.tiles_y;
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int blocks = std::max(1, std::min(h.ntiles, cus));
    Tensor part;
    if (mode == 1) {   // every block (each owns >= 1 tile) writes its partial
      part = at::empty({blocks}, x1.options().dtype(at::kFloat));
      h.l1_part = part.data_ptr<float>();
    }
    const int rc = p2p_halo_union(&h, act_in == 1 ? 1 : 0, blocks, st);
    TORCH_CHECK(rc != -2, "conv_d2s: no halo kernel for C1 ", C1, " C2 ", C2);
    check_rc(rc, "conv_d2s(halo)");
    if (mode == 1) {
      Tensor l1 = at::empty({}, x1.options().dtype(at::kFloat));
      check_rc(p2p_sum_partials(h.l1_part, blocks, (float)scale, l1.data_ptr<float>(), st), "conv_d2s l1");
      return l1;
    }
    return out;
  }
  p2p::ConvFwdArgs a{};
  a.x1 = x1.data_ptr();
  a.x2 = x2 ? x2->data_ptr() : nullptr;
  a.C1 = (int)C1;
  a.C2 = (int)C2;
  a.C = (int)C;
  a.N = (int)N;
  a.H = (int)H;
  a.W = (int)W;
  a.up = 1;
  a.KH = a.KW = 3;
  a.stride = 1;
  a.pad = 1;
  a.act_in = (int)act_in;
  a.OH = (int)H;
  a.OW = (int)W;
  a.Cout = 32;
  a.Csplit = 32;
  a.w = w.data_ptr();
  a.bias = bias.data_ptr<float>();
  a.act_out = (int)act_out;
  a.y1 = out.data_ptr();
  a.splits = 1;
  a.zero = zero_page(x1);
  a.d2s = (int)mode;
  a.pk_a = pk_a.data_ptr();
  a.pk_f = mode == 2 ? pk_f->data_ptr() : nullptr;
  a.d2s_scale = (float)scale;
  a.d2s_w = wsc;
  const int64_t blocks = (N * H * W + 255) / 256;
  Tensor part, l1;
  if (mode == 1) {
    part = at::zeros({blocks}, x1.options().dtype(at::kFloat));
    a.l1_part = part.data_ptr<float>();
  }
  const int rc = p2p_conv_fwd_glds(&a, 0, 7, st);
  TORCH_CHECK(rc != -2, "conv_d2s: no union-GEMM kernel for this geometry");
  check_rc(rc, "conv_d2s");
  if (mode == 1) {
    l1 = at::empty({}, x1.options().dtype(at::kFloat));
    check_rc(p2p_sum_partials(a.l1_part, (int)blocks, (float)scale, l1.data_ptr<float>(), st), "conv_d2s l1");
    return l1;
  }
  return out;
}

// ------------------------------------------------------------------ conv wgrad
// fp8 (qs_p / qs_q given): p / q are OCP fp8 shadows (p_fmt / q_fmt 0 = e4m3, 1 = e5m2) with
// their scale sites; returns false (nothing launched) when the fp8 kernel does not take the
// geometry -- the caller then runs the bf16 path.  bf16 always returns true.
bool conv_wgrad(const Tensor& p1, const optional<Tensor>& p2, int64_t p_act, const Tensor& q1,
                const optional<Tensor>& q2, int64_t q_act, int64_t KH, int64_t KW, int64_t stride,
                int64_t pad, int64_t reflect, int64_t up, Tensor dw, double scale,
                int64_t accumulate, int64_t flip, const optional<Tensor>& qs_p,
                const optional<Tensor>& qs_q, int64_t p_fmt, int64_t q_fmt, const optional<Tensor>& qs_p2,
                const optional<Tensor>& qs_q2) {
  const bool f8 = qs_p.has_value() || qs_q.has_value();
  TORCH_CHECK(!f8 || (qs_p && qs_q && !flip && p1.element_size() == 1 && q1.element_size() == 1 &&
                      (!p2 || p2->element_size() == 1) && (!q2 || q2->element_size() == 1)),
              "conv_wgrad fp8: both operands fp8 with both scale sites");
  if (f8) {
    check_site(*qs_p);
    check_site(*qs_q);
  }
  check_act(p1, "conv_wgrad p1", f8);
  check_act(q1, "conv_wgrad q1", f8);
  const int64_t N = p1.size(0), OH = p1.size(2), OW = p1.size(3);
  int64_t R2 = 0, C2 = 0;
  if (p2) {
    check_act(*p2, "conv_wgrad p2", f8);
    TORCH_CHECK(p2->size(0) == N && p2->size(2) == OH && p2->size(3) == OW, "wgrad p concat shape");
    R2 = p2->size(1);
  }
  const int64_t H = q1.size(2), W = q1.size(3);
  TORCH_CHECK(q1.size(0) == N, "conv_wgrad: batch mismatch");
  if (q2) {
    check_act(*q2, "conv_wgrad q2", f8);
    TORCH_CHECK(q2->size(0) == N && q2->size(2) == H && q2->size(3) == W, "wgrad q concat shape");
    C2 = q2->size(1);
  }
  const int64_t R = p1.size(1) + R2, C = q1.size(1) + C2;
  TORCH_CHECK(dw.is_cuda() && dw.scalar_type() == at::kFloat && dw.is_contiguous() && dw.dim() == 4,
              "conv_wgrad: dw must be contiguous fp32 [R][C][KH][KW]");
  // flip: dw is [C][R][KH][KW] with flipped taps (stride-1 conv wgrad in transposed form)
  const int64_t Rr = flip ? dw.size(1) : dw.size(0), Cr = flip ? dw.size(0) : dw.size(1);
  TORCH_CHECK(Rr <= R && Cr <= C && dw.size(2) == KH && dw.size(3) == KW, "conv_wgrad: dw shape");
  // the conv geometry over q must produce the p grid
  const int64_t Hu = H * up, Wu = W * up;
  TORCH_CHECK((Hu + 2 * pad - KH) / stride + 1 == OH && (Wu + 2 * pad - KW) / stride + 1 == OW,
              "conv_wgrad: geometry mismatch");
  p2p::ConvWgradArgs a{};
  a.p1 = p1.data_ptr();
  a.p2 = p2 ? p2->data_ptr() : nullptr;
  a.R1 = (int)p1.size(1);
  a.R2 = (int)R2;
  a.R = (int)R;
  a.p_act = (int)p_act;
  a.q1 = q1.data_ptr();
  a.q2 = q2 ? q2->data_ptr() : nullptr;
  a.C1 = (int)q1.size(1);
  a.C2 = (int)C2;
  a.C = (int)C;
  a.N = (int)N;
  a.H = (int)H;
  a.W = (int)W;
  a.up = (int)up;
  a.KH = (int)KH;
  a.KW = (int)KW;
  a.stride = (int)stride;
  a.pad = (int)pad;
  a.reflect = (int)reflect;
  a.q_act = (int)q_act;
  a.OH = (int)OH;
  a.OW = (int)OW;
  a.M = (int)(N * OH * OW);
  a.Kq = (int)(KH * KW * C);
  a.zero = zero_page(p1);
  hipStream_t st = cur_stream(p1);
  if (f8) {
    a.f8 = 1;
    a.p_fmt = (int)p_fmt;
    a.q_fmt = (int)q_fmt;
    a.qs_p = qs_p->data_ptr<int>();
    a.qs_q = qs_q->data_ptr<int>();
    if (qs_p2) {
      check_site(*qs_p2);
      a.qs_p2 = qs_p2->data_ptr<int>();
    }
    if (qs_q2) {
      check_site(*qs_q2);
      a.qs_q2 = qs_q2->data_ptr<int>();
    }
    int tr = 0, tq = 0;
    if (!p2p_conv_wgrad_f8_tile(&a, &tr, &tq) || !((p_fmt == 1 && q_fmt == 0) || (p_fmt == 0 && q_fmt == 1)))
      return false;
    const int64_t tiles = ((R + tr - 1) / tr) * ((a.Kq + tq - 1) / tq);
    const int64_t stages = ((int64_t)a.M + 127) / 128;
    int64_t splits = std::max<int64_t>(1, 512 / std::max<int64_t>(tiles, 1));
    splits = std::min<int64_t>(splits, std::max<int64_t>(1, stages / 8));
    const int64_t slab = R * (int64_t)a.Kq;
    splits = std::max<int64_t>(1, std::min<int64_t>(splits, (64ll << 20) / std::max<int64_t>(slab, 1)));
    a.splits = (int)splits;
    Tensor ws = at::empty({splits * slab + p2p_wgrad_reduce_extra((int)splits, slab)}, p1.options().dtype(at::kFloat));
    a.ws = ws.data_ptr<float>();
    check_rc(p2p_conv_wgrad(&a, st), "conv_wgrad(fp8)");
    check_rc(p2p_wgrad_reduce(a.ws, a.splits, a.R, a.KH, a.KW, a.C, (int)Rr, (int)Cr, dw.data_ptr<float>(),
                              (float)scale, (int)accumulate, 0, st),
             "wgrad_reduce(fp8)");
    return true;
  }
  // 9x9 stride-1 layers with 16 / 32 input and <= 32 output channels: halo-tile wgrad
  // (csrc/halo_wgrad.hip), one fp32 slab per persistent block
  const bool halo_geo = (KH == 9 && KW == 9 && (C == 16 || C == 32) && (R <= 16 || (C == 16 && R == 32))) ||
                        (KH == 3 && KW == 3 && C == 64 && R <= 32);
  if (!p2 && !q2 && p_act == 0 && q_act == 0 && halo_geo && stride == 1 && !flip && R % 8 == 0 &&
      std::getenv("P2P_NO_HALO") == nullptr) {
    p2p::HaloWArgs h{};
    h.gy = static_cast<const __bf16*>(p1.data_ptr());
    h.x = static_cast<const __bf16*>(q1.data_ptr());
    h.R = (int)R;
    h.C = (int)C;
    h.N = (int)N;
    h.H = (int)H;
    h.W = (int)W;
    h.up = (int)up;
    h.pad = (int)pad;
    h.reflect = (int)reflect;
    h.OH = (int)OH;
    h.OW = (int)OW;
    h.zero = static_cast<const __bf16*>(a.zero);
    h.tiles_x = (int)((OW + 15) / 16);
    h.tiles_y = (int)((OH + 15) / 16);
    h.ntiles = (int)N * h.tiles_x * h.tiles_y;
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int blocks = std::max(1, std::min(h.ntiles, cus));
    Tensor ws = at::empty({(int64_t)blocks * R * a.Kq + p2p_wgrad_reduce_extra(blocks, R * a.Kq)},
                          p1.options().dtype(at::kFloat));
    h.ws = ws.data_ptr<float>();
    const int rc = p2p_halo_wgrad(&h, (int)KH, blocks, st);
    if (rc != -2) {
      check_rc(rc, "conv_wgrad(halo)");
      check_rc(p2p_wgrad_reduce(h.ws, blocks, (int)R, (int)KH, (int)KW, (int)C, (int)Rr, (int)Cr, dw.data_ptr<float>(),
                                (float)scale, (int)accumulate, 0, st),
               "wgrad_reduce(halo)");
      return true;
    }
  }
  int wbr = 128, wbq = 128;
  p2p_conv_wgrad_tile(&a, &wbr, &wbq);
  const int64_t tiles = ((R + wbr - 1) / wbr) * ((a.Kq + wbq - 1) / wbq);
  const int64_t stages = ((int64_t)a.M + 63) / 64;
  // >= P2P_WGRAD_BLOCKS blocks (default 512: 2 waves of 256 CUs); every split keeps >= 8
  // reduction stages (pipeline depth 3)
  const char* wbv = std::getenv("P2P_WGRAD_BLOCKS");   // (per call: A/B of the split target)
  const int64_t wblocks = wbv ? std::max<int64_t>(1, std::atoll(wbv)) : 512;
  int64_t splits = std::max<int64_t>(1, wblocks / std::max<int64_t>(tiles, 1));
  splits = std::min<int64_t>(splits, std::max<int64_t>(1, stages / 8));
  // bound the fp32 slab workspace to ~256 MB
  const int64_t slab = R * (int64_t)a.Kq;
  splits = std::max<int64_t>(1, std::min<int64_t>(splits, (64ll << 20) / std::max<int64_t>(slab, 1)));
  a.splits = (int)splits;
  Tensor ws = at::empty({splits * slab + p2p_wgrad_reduce_extra((int)splits, slab)}, p1.options().dtype(at::kFloat));
  a.ws = ws.data_ptr<float>();
  check_rc(p2p_conv_wgrad(&a, st), "conv_wgrad");
  check_rc(p2p_wgrad_reduce(a.ws, a.splits, a.R, a.KH, a.KW, a.C, flip ? (int)Cr : (int)Rr,
                            flip ? (int)Rr : (int)Cr, dw.data_ptr<float>(), (float)scale,
                            (int)accumulate, (int)flip, st),
           "wgrad_reduce");
  return true;
}

// ------------------------------------------------------------------ weight prep
Tensor weight_prep(const Tensor& w, int64_t swap, int64_t Xp, int64_t Yp,
                   const optional<Tensor>& scale) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.is_contiguous() && w.dim() == 4,
              "weight_prep: fp32 contiguous 4-D weight");
  const int64_t A = w.size(0), B = w.size(1), KH = w.size(2), KW = w.size(3);
  TORCH_CHECK(Xp >= (swap ? B : A) && Yp >= (swap ? A : B), "weight_prep: padding too small");
  Tensor out = at::empty({Xp, KH, KW, Yp}, w.options().dtype(at::kBFloat16));
  check_rc(p2p_weight_prep(w.data_ptr<float>(), (int)A, (int)B, (int)KH, (int)KW, (int)swap, (int)Xp,
                           (int)Yp, scale ? scale->data_ptr<float>() : nullptr, out.data_ptr(),
                           cur_stream(w)),
           "weight_prep");
  return out;
}

// out[:x.numel()] = x, out[x.numel():] = fill (fp32 vectors; out may be shorter: a copy)
void vec_pad_into(const Tensor& x, Tensor out, double fill) {
  TORCH_CHECK(x.is_cuda() && out.is_cuda() && x.scalar_type() == at::kFloat && out.scalar_type() == at::kFloat &&
                  x.is_contiguous() && out.is_contiguous(), "vec_pad_into: contiguous fp32 vectors");
  if (out.numel() == 0) return;
  check_rc(p2p_vec_pad(x.data_ptr<float>(), (int)x.numel(), (float)fill, (int)out.numel(), out.data_ptr<float>(),
                       cur_stream(out)),
           "vec_pad_into");
}

// runtime A/B switch of the 32x32x16 conv tiles (returns the previous setting)
int64_t set_m32(int64_t on) { return p2p_set_m32((int)on); }

// P2P_BOUNDS_ASSERT build (csrc/bounds.h): [enabled, failed checks, largest site id, last bad
// index, its limit] summed over every translation unit's device counters (reset when asked)
// launches one deliberately out-of-range check (site 99) on the scratch tensor's stream
void oob_selftest(Tensor scratch) {
  TORCH_CHECK(scratch.is_cuda() && scratch.scalar_type() == at::kInt && scratch.numel() >= 1, "oob_selftest: int32 scratch");
  check_rc(p2p_oob_selftest(scratch.data_ptr(), cur_stream(scratch)), "oob_selftest");
}

std::vector<int64_t> oob_counts(bool reset) {
  unsigned int v[4] = {0, 0, 0, 0};
  const int on = p2p_oob_counts(v, reset ? 1 : 0);
  return {on, v[0], v[1], v[2], v[3]};
}

// input-gradient image of a nearest-x2 + reflect-1 3x3 conv: [Xp][4][4][Yp] bf16 (misc.hip)
Tensor up2_dgrad_image(const Tensor& w, int64_t Xp, int64_t Yp) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.is_contiguous() && w.dim() == 4 &&
                  w.size(2) == 3 && w.size(3) == 3,
              "up2_dgrad_image: fp32 contiguous [Cout][Cin][3][3] weight");
  const int64_t Cout = w.size(0), Cin = w.size(1);
  TORCH_CHECK(Xp >= Cin && Yp >= Cout, "up2_dgrad_image: padding too small");
  Tensor out = at::empty({Xp, 4, 4, Yp}, w.options().dtype(at::kBFloat16));
  check_rc(p2p_up2_dgrad_image(w.data_ptr<float>(), (int)Cout, (int)Cin, (int)Xp, (int)Yp, out.data_ptr(),
                               cur_stream(w)),
           "up2_dgrad_image");
  return out;
}

// all weight images of a network in one launch per WP_MAX tensors
// both images of each weight (T <= 16) in one launch: returns [out0_0, out1_0, out0_1, ...]
// sites (optional): e4m3 images instead of bf16, scaled by the current-scaling site
// sites[site_idx[i]] (int32 [n][4], amax in word 0 -- csrc/fp8.hip)
std::vector<Tensor> weight_prep_pairs(at::TensorList ws, at::IntArrayRef xa, at::IntArrayRef xb,
                                      const optional<Tensor>& sites, at::OptionalIntArrayRef site_idx) {
  const size_t n = ws.size();
  TORCH_CHECK(xa.size() == n && xb.size() == n, "weight_prep_pairs: list sizes");
  const bool f8 = sites.has_value();
  if (f8)
    TORCH_CHECK(site_idx.has_value() && site_idx->size() == n && sites->scalar_type() == at::kInt &&
                    sites->dim() == 2 && sites->size(1) == 4 && sites->is_contiguous(),
                "weight_prep_pairs: fp8 sites");
  const auto odt = f8 ? at::kFloat8_e4m3fn : at::kBFloat16;
  std::vector<int*> S;
  std::vector<Tensor> outs;
  outs.reserve(2 * n);
  std::vector<const float*> W;
  std::vector<void*> O0, O1;
  std::vector<int> A, B, T, XA, XB;
  auto flush = [&]() {
    if (W.empty()) return;
    check_rc(p2p_weight_prep_pairs((int)W.size(), W.data(), O0.data(), O1.data(), A.data(), B.data(),
                                   T.data(), XA.data(), XB.data(), f8 ? S.data() : nullptr,
                                   cur_stream(ws[0])),
             "weight_prep_pairs");
    W.clear(); O0.clear(); O1.clear(); A.clear(); B.clear(); T.clear(); XA.clear(); XB.clear(); S.clear();
  };
  for (size_t i = 0; i < n; ++i) {
    const Tensor& w = ws[i];
    TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.is_contiguous() && w.dim() == 4,
                "weight_prep_pairs: fp32 contiguous 4-D weights");
    const int64_t a = w.size(0), b = w.size(1), kh = w.size(2), kw = w.size(3);
    TORCH_CHECK(kh * kw <= 16 && xa[i] >= a && xb[i] >= b && xa[i] % 2 == 0 && xb[i] % 2 == 0,
                "weight_prep_pairs: T <= 16, even padded sizes");
    Tensor o0 = at::empty({xa[i], kh, kw, xb[i]}, w.options().dtype(odt));
    Tensor o1 = at::empty({xb[i], kh, kw, xa[i]}, w.options().dtype(odt));
    if (f8) {
      const int64_t si = (*site_idx)[i];
      TORCH_CHECK(si >= 0 && si < sites->size(0), "weight_prep_pairs: site index");
      S.push_back(sites->data_ptr<int>() + 4 * si);
    }
    outs.push_back(o0);
    outs.push_back(o1);
    W.push_back(w.data_ptr<float>());
    O0.push_back(o0.data_ptr());
    O1.push_back(o1.data_ptr());
    A.push_back((int)a);
    B.push_back((int)b);
    T.push_back((int)(kh * kw));
    XA.push_back((int)xa[i]);
    XB.push_back((int)xb[i]);
    if (W.size() == 24) flush();
  }
  flush();
  return outs;
}

std::vector<Tensor> weight_prep_multi(at::TensorList ws, at::IntArrayRef swap, at::IntArrayRef xp,
                                      at::IntArrayRef yp) {
  const size_t n = ws.size();
  TORCH_CHECK(swap.size() == n && xp.size() == n && yp.size() == n, "weight_prep_multi: list sizes");
  std::vector<Tensor> outs;
  outs.reserve(n);
  const int maxT = p2p_weight_prep_max();
  std::vector<const float*> W;
  std::vector<void*> O;
  std::vector<int> A, B, T, S, X, Y;
  auto flush = [&]() {
    if (W.empty()) return;
    check_rc(p2p_weight_prep_multi((int)W.size(), W.data(), O.data(), A.data(), B.data(), T.data(),
                                   S.data(), X.data(), Y.data(), cur_stream(ws[0])),
             "weight_prep_multi");
    W.clear(); O.clear(); A.clear(); B.clear(); T.clear(); S.clear(); X.clear(); Y.clear();
  };
  for (size_t i = 0; i < n; ++i) {
    const Tensor& w = ws[i];
    TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.is_contiguous() && w.dim() == 4,
                "weight_prep_multi: fp32 contiguous 4-D weights");
    const int64_t a = w.size(0), b = w.size(1), kh = w.size(2), kw = w.size(3);
    TORCH_CHECK(xp[i] >= (swap[i] ? b : a) && yp[i] >= (swap[i] ? a : b), "weight_prep_multi: padding");
    Tensor out = at::empty({xp[i], kh, kw, yp[i]}, w.options().dtype(at::kBFloat16));
    outs.push_back(out);
    W.push_back(w.data_ptr<float>());
    O.push_back(out.data_ptr());
    A.push_back((int)a);
    B.push_back((int)b);
    T.push_back((int)(kh * kw));
    S.push_back((int)swap[i]);
    X.push_back((int)xp[i]);
    Y.push_back((int)yp[i]);
    if ((int)W.size() == maxT) flush();
  }
  flush();
  return outs;
}

// ------------------------------------------------------------------ norms
// batch=false: instance norm (groups n x c); batch=true: batch norm (groups c)
std::vector<Tensor> norm_fwd(const Tensor& x, double eps, const optional<Tensor>& gamma,
                             const optional<Tensor>& beta, const optional<Tensor>& prelu_w,
                             int64_t act, const optional<Tensor>& run_mean,
                             const optional<Tensor>& run_var, double momentum, bool batch,
                             const optional<Tensor>& partials, const optional<Tensor>& qsite,
                             const optional<Tensor>& q_out, int64_t qfmt, const optional<Tensor>& res) {
  check_act(x, "norm_fwd x");
  // res: residual added before the activation (same shape / layout as x)
  if (res) {
    check_act(*res, "norm_fwd res");
    TORCH_CHECK(res->sizes() == x.sizes(), "norm_fwd: residual shape");
    TORCH_CHECK(!prelu_w, "norm_fwd: residual with the fused PReLU is unsupported");
  }
  const void* resp = res ? res->data_ptr() : nullptr;
  // optional fp8 shadow of y written by the apply pass (q_out: same shape, fp8, NHWC)
  void* qp = nullptr;
  int* qs = nullptr;
  if (q_out) {
    TORCH_CHECK(qsite && q_out->numel() == x.numel() && q_out->element_size() == 1 &&
                    q_out->is_contiguous(at::MemoryFormat::ChannelsLast),
                "norm_fwd: fp8 shadow output");
    check_site(*qsite);
    qp = q_out->data_ptr();
    qs = qsite->data_ptr<int>();
  }
  const int64_t N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  TORCH_CHECK(C <= 2048, "norm_fwd: C > 2048 unsupported");
  const int gN = batch ? 1 : (int)N;
  const int gHW = batch ? (int)(N * HW) : (int)HW;
  Tensor mean = at::empty({gN, C}, x.options().dtype(at::kFloat));
  Tensor rstd = at::empty({gN, C}, x.options().dtype(at::kFloat));
  if (partials) {
    // [2][N][nch][C] from the producing conv's epilogue (BN: all N*nch chunks of one group)
    TORCH_CHECK(partials->dim() == 4 && partials->size(0) == 2 && partials->size(1) == N &&
                    partials->size(3) == C && partials->scalar_type() == at::kFloat,
                "norm_fwd: partials shape");
    const int nch = (int)(batch ? N * partials->size(2) : partials->size(2));
    Tensor y = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
    check_rc(p2p_norm_fwd_partials(x.data_ptr(), gN, gHW, (int)C, nch, partials->data_ptr<float>(),
                                   (float)eps, gamma ? gamma->data_ptr<float>() : nullptr,
                                   beta ? beta->data_ptr<float>() : nullptr,
                                   prelu_w ? prelu_w->data_ptr<float>() : nullptr, (int)act,
                                   mean.data_ptr<float>(), rstd.data_ptr<float>(),
                                   run_mean ? run_mean->data_ptr<float>() : nullptr,
                                   run_var ? run_var->data_ptr<float>() : nullptr, (float)momentum,
                                   y.data_ptr(), qp, qs, (int)qfmt, resp, cur_stream(x)),
             "norm_fwd(partials)");
    return {y, mean, rstd};
  }
  Tensor ws = at::empty({p2p_norm_ws_floats(gN, gHW, (int)C)}, x.options().dtype(at::kFloat));
  Tensor y = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  check_rc(p2p_norm_fwd(x.data_ptr(), gN, gHW, (int)C, (float)eps,
                        gamma ? gamma->data_ptr<float>() : nullptr,
                        beta ? beta->data_ptr<float>() : nullptr,
                        prelu_w ? prelu_w->data_ptr<float>() : nullptr, (int)act,
                        mean.data_ptr<float>(), rstd.data_ptr<float>(),
                        run_mean ? run_mean->data_ptr<float>() : nullptr,
                        run_var ? run_var->data_ptr<float>() : nullptr, (float)momentum,
                        ws.data_ptr<float>(), y.data_ptr(), qp, qs, (int)qfmt, resp, cur_stream(x)),
           "norm_fwd");
  return {y, mean, rstd};
}

Tensor norm_apply(const Tensor& x, const Tensor& mean, const Tensor& rstd,
                  const optional<Tensor>& gamma, const optional<Tensor>& beta,
                  const optional<Tensor>& prelu_w, int64_t act, bool batch, const optional<Tensor>& res) {
  check_act(x, "norm_apply x");
  if (res) {
    check_act(*res, "norm_apply res");
    TORCH_CHECK(res->sizes() == x.sizes() && !prelu_w, "norm_apply: residual shape / PReLU");
  }
  const int64_t N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  Tensor y = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  check_rc(p2p_norm_apply(x.data_ptr(), batch ? 1 : (int)N, batch ? (int)(N * HW) : (int)HW, (int)C,
                          mean.data_ptr<float>(), rstd.data_ptr<float>(),
                          gamma ? gamma->data_ptr<float>() : nullptr,
                          beta ? beta->data_ptr<float>() : nullptr,
                          prelu_w ? prelu_w->data_ptr<float>() : nullptr, (int)act, y.data_ptr(),
                          res ? res->data_ptr() : nullptr, cur_stream(x)),
           "norm_apply");
  return y;
}

// act: the ReLU / LeakyReLU fused by the forward (recomputed from x, no extra pass);
// dsum: optional [C] fp32 output = column sums of dx (bias grad of the producing conv).
Tensor norm_bwd(const Tensor& x, const Tensor& dy, const Tensor& mean, const Tensor& rstd,
                const optional<Tensor>& gamma, const optional<Tensor>& beta, int64_t act,
                const optional<Tensor>& dgamma, const optional<Tensor>& dbeta, bool need_dx,
                bool batch, const optional<Tensor>& dsum, const optional<Tensor>& qsite,
                const optional<Tensor>& q_out, int64_t qfmt, const optional<Tensor>& prelu_w,
                const optional<Tensor>& dprelu, const optional<Tensor>& partials, bool frozen) {
  check_act(x, "norm_bwd x");
  TORCH_CHECK(!frozen || (!partials && !dsum), "norm_bwd: frozen statistics take no partials / dsum");
  if (prelu_w)
    TORCH_CHECK(prelu_w->numel() == 1 && prelu_w->scalar_type() == at::kFloat && prelu_w->is_cuda(),
                "norm_bwd: prelu_w must be a 1-element fp32 GPU tensor");
  if (dprelu)
    TORCH_CHECK(prelu_w && dprelu->numel() == 1 && dprelu->scalar_type() == at::kFloat,
                "norm_bwd: dprelu needs prelu_w and a 1-element fp32 tensor");
  check_act(dy, "norm_bwd dy");
  void* qp = nullptr;
  int* qs = nullptr;
  if (q_out && need_dx) {
    TORCH_CHECK(qsite && q_out->numel() == x.numel() && q_out->element_size() == 1 &&
                    q_out->is_contiguous(at::MemoryFormat::ChannelsLast),
                "norm_bwd: fp8 shadow output");
    check_site(*qsite);
    qp = q_out->data_ptr();
    qs = qsite->data_ptr<int>();
  }
  const int64_t N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  const int gN = batch ? 1 : (int)N;
  const int gHW = batch ? (int)(N * HW) : (int)HW;
  if (dsum) TORCH_CHECK(dsum->numel() == C && dsum->scalar_type() == at::kFloat, "norm_bwd: dsum");
  Tensor dx;
  if (need_dx) dx = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  if (partials) {
    // [2][N][nch][C] sum(d) / sum(d * xhat) from the consumer conv's dgrad epilogue; batch
    // norm may come flat ([P][1][nch][C], tiles over all images) and with a shared-slope PReLU
    // as a third plane of sum(dz * z * [z <= 0]) -- the slope gradient is its total
    const int64_t planes = partials->dim() == 4 ? partials->size(0) : 0;
    TORCH_CHECK(partials->dim() == 4 && (planes == 2 || (planes == 3 && prelu_w && batch)) &&
                    (partials->size(1) == N || (batch && partials->size(1) == 1)) && partials->size(3) == C &&
                    partials->scalar_type() == at::kFloat && partials->is_contiguous() && (!prelu_w || planes == 3),
                "norm_bwd: partials shape");
    const int nch = (int)(batch ? partials->size(1) * partials->size(2) : partials->size(2));
    Tensor coef = at::empty({3 * gN * C}, x.options().dtype(at::kFloat));
    if (dprelu) {
      const long plane = (long)nch * C;   // batch: gN = 1
      Tensor part = at::empty({256}, x.options().dtype(at::kFloat));
      check_rc(p2p_sum_long(partials->data_ptr<float>() + 2 * plane, plane, 1.f, part.data_ptr<float>(),
                            dprelu->data_ptr<float>(), cur_stream(x)),
               "norm_bwd(partials: dprelu)");
    }
    check_rc(p2p_norm_bwd_partials(x.data_ptr(), dy.data_ptr(), gN, gHW, (int)C, nch, partials->data_ptr<float>(),
                                   mean.data_ptr<float>(), rstd.data_ptr<float>(),
                                   gamma ? gamma->data_ptr<float>() : nullptr,
                                   beta ? beta->data_ptr<float>() : nullptr, (int)act,
                                   prelu_w ? prelu_w->data_ptr<float>() : nullptr,
                                   dgamma ? dgamma->data_ptr<float>() : nullptr,
                                   dbeta ? dbeta->data_ptr<float>() : nullptr, coef.data_ptr<float>(),
                                   need_dx ? dx.data_ptr() : nullptr,
                                   (need_dx && dsum) ? dsum->data_ptr<float>() : nullptr, qp, qs, (int)qfmt,
                                   cur_stream(x)),
             "norm_bwd(partials)");
    return dx;
  }
  Tensor ws = at::empty({p2p_norm_ws_floats(gN, gHW, (int)C)}, x.options().dtype(at::kFloat));
  check_rc(p2p_norm_bwd(x.data_ptr(), dy.data_ptr(), gN, gHW, (int)C, mean.data_ptr<float>(),
                        rstd.data_ptr<float>(), gamma ? gamma->data_ptr<float>() : nullptr,
                        beta ? beta->data_ptr<float>() : nullptr, (int)act,
                        prelu_w ? prelu_w->data_ptr<float>() : nullptr,
                        dprelu ? dprelu->data_ptr<float>() : nullptr,
                        dgamma ? dgamma->data_ptr<float>() : nullptr,
                        dbeta ? dbeta->data_ptr<float>() : nullptr, ws.data_ptr<float>(),
                        need_dx ? dx.data_ptr() : nullptr,
                        (need_dx && dsum) ? dsum->data_ptr<float>() : nullptr, qp, qs, (int)qfmt,
                        frozen ? 1 : 0, cur_stream(x)),
           "norm_bwd");
  return dx;
}

// ------------------------------------------------------------------ elementwise
Tensor act(const Tensor& a, const optional<Tensor>& b, int64_t act, int64_t mode) {
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == at::kBFloat16, "act: bf16 GPU tensor");
  const auto mf = a.is_contiguous(at::MemoryFormat::ChannelsLast) && a.dim() == 4
                      ? at::MemoryFormat::ChannelsLast
                      : at::MemoryFormat::Contiguous;
  TORCH_CHECK(a.is_contiguous(mf), "act: dense input");
  if (b) TORCH_CHECK(b->is_contiguous(mf) && b->sizes() == a.sizes(), "act: b layout");
  Tensor out = at::empty_like(a, a.options().memory_format(mf));
  check_rc(p2p_act(a.data_ptr(), b ? b->data_ptr() : nullptr, a.numel(), (int)act, (int)mode,
                   out.data_ptr(), cur_stream(a)),
           "act");
  return out;
}

Tensor dropout(const Tensor& x, double p, const Tensor& seed, int64_t salt) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.numel() % 8 == 0, "dropout: x");
  TORCH_CHECK(seed.scalar_type() == at::kLong && seed.is_cuda(), "dropout: seed must be a GPU int64");
  const auto mf = x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast)
                      ? at::MemoryFormat::ChannelsLast
                      : at::MemoryFormat::Contiguous;
  TORCH_CHECK(x.is_contiguous(mf), "dropout: dense input");
  Tensor y = at::empty_like(x, x.options().memory_format(mf));
  check_rc(p2p_dropout(x.data_ptr(), x.numel(), (float)p, seed.data_ptr<int64_t>(), (unsigned)salt,
                       y.data_ptr(), cur_stream(x)),
           "dropout");
  return y;
}

// ------------------------------------------------------------------ family-R fringe ops
static void check_nhwc(const Tensor& x, const char* what) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4, what, ": bf16 4-D CUDA");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), what, ": NHWC (channels_last) input");
}

Tensor prelu_fwd(const Tensor& x, const Tensor& w) {
  check_nhwc(x, "prelu");
  TORCH_CHECK(w.numel() == 1 && w.scalar_type() == at::kFloat, "prelu: one fp32 slope");
  Tensor y = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  check_rc(p2p_prelu_fwd(x.data_ptr(), x.numel(), w.data_ptr<float>(), y.data_ptr(), cur_stream(x)), "prelu");
  return y;
}

std::vector<Tensor> prelu_bwd(const Tensor& x, const Tensor& gy, const Tensor& w, bool need_x) {
  check_nhwc(x, "prelu_bwd x");
  check_nhwc(gy, "prelu_bwd gy");
  Tensor gx;
  if (need_x) gx = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor ws = at::empty({p2p_misc_nblocks(x.numel())}, x.options().dtype(at::kFloat));
  Tensor gw = at::empty({1}, x.options().dtype(at::kFloat));
  check_rc(p2p_prelu_bwd(x.data_ptr(), gy.data_ptr(), x.numel(), w.data_ptr<float>(),
                         need_x ? gx.data_ptr() : nullptr, ws.data_ptr<float>(), gw.data_ptr<float>(), 0,
                         cur_stream(x)),
           "prelu_bwd");
  if (!need_x) return {gw};
  return {gw, gx};
}

Tensor tv_fwd(const Tensor& x) {
  check_nhwc(x, "tv");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  Tensor ws = at::empty({p2p_misc_nblocks(x.numel())}, x.options().dtype(at::kFloat));
  Tensor out = at::empty({}, x.options().dtype(at::kFloat));
  check_rc(p2p_tv_fwd(x.data_ptr(), N, H, W, C, ws.data_ptr<float>(), out.data_ptr<float>(), cur_stream(x)),
           "tv");
  return out;
}

// per-image (PSNR, SSIM) of two [N, C, H, W] image batches (any strides, fp32 or bf16):
// returns float64 [N, 2]
Tensor image_metrics(const Tensor& a, const Tensor& b, bool shift, double data_range) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.dim() == 4 && a.sizes() == b.sizes(),
              "image_metrics: two 4-D CUDA tensors of one shape");
  TORCH_CHECK(a.scalar_type() == b.scalar_type() &&
                  (a.scalar_type() == at::kFloat || a.scalar_type() == at::kBFloat16),
              "image_metrics: fp32 or bf16 inputs of one dtype");
  const int N = (int)a.size(0), C = (int)a.size(1), H = (int)a.size(2), W = (int)a.size(3);
  TORCH_CHECK(H >= 7 && W >= 7, "image_metrics: images of at least 7x7 (SSIM window)");
  const long st[8] = {(long)a.stride(0), (long)a.stride(1), (long)a.stride(2), (long)a.stride(3),
                      (long)b.stride(0), (long)b.stride(1), (long)b.stride(2), (long)b.stride(3)};
  Tensor ws = at::empty({N, p2p_metrics_ws(C, H, W), 2}, a.options().dtype(at::kDouble));
  check_rc(p2p_image_metrics(a.data_ptr(), b.data_ptr(), a.scalar_type() == at::kBFloat16 ? 1 : 0, st, N, C, H,
                             W, shift ? 1 : 0, data_range, ws.data_ptr<double>(), cur_stream(a)),
           "image_metrics");
  Tensor sums = ws.sum(1);  // fixed-order reduction of the per-tile partials
  Tensor mse = sums.select(1, 1) / ((double)C * H * W);
  Tensor psnr = (255.0 * 255.0 / mse).log10() * 10.0;
  Tensor ssim = sums.select(1, 0) / ((double)C * (H - 6) * (W - 6));
  return at::stack({psnr, ssim}, 1);
}

Tensor tv_bwd(const Tensor& x, const Tensor& gout) {
  check_nhwc(x, "tv_bwd");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  Tensor g = gout.to(at::kFloat).reshape({1}).contiguous();
  Tensor gx = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  check_rc(p2p_tv_bwd(x.data_ptr(), N, H, W, C, g.data_ptr<float>(), gx.data_ptr(), cur_stream(x)), "tv_bwd");
  return gx;
}

Tensor quantize(const Tensor& x, int64_t bits) {
  check_nhwc(x, "quantize");
  TORCH_CHECK(bits >= 1 && bits <= 16, "quantize: bits");
  Tensor y = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  check_rc(p2p_quantize(x.data_ptr(), x.numel(), (int)bits, y.data_ptr(), cur_stream(x)), "quantize");
  return y;
}

// quantise + pixel-unshuffle(r) in one pass: [y (x's shape), yu (N, cp, H/r, W/r)] with yu's
// channels [C*r*r, cp) zero (a pad-8 conv input, no channel-pad pass)
std::vector<Tensor> quantize_unshuffle(const Tensor& x, int64_t bits, int64_t r, int64_t cp) {
  check_nhwc(x, "quantize_unshuffle");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(bits >= 1 && bits <= 16 && r >= 1 && H % r == 0 && W % r == 0 && cp >= C * r * r,
              "quantize_unshuffle: bits / r / cp");
  Tensor y = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor yu = empty_nhwc(N, cp, H / r, W / r, x);
  check_rc(p2p_quantize_unshuffle(x.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)bits, (int)r, y.data_ptr(),
                                  yu.data_ptr(), (int)cp, cur_stream(x)),
           "quantize_unshuffle");
  return {y, yu};
}

// bwd = 0: x (N,C,H,W) -> pooled; bwd = 1: x = gy (N,C,OH,OW) -> gx (N,C,H,W)
Tensor avgpool3s2(const Tensor& x, int64_t bwd, int64_t H, int64_t W) {
  check_nhwc(x, "avgpool3s2");
  const int64_t N = x.size(0), C = x.size(1);
  int64_t h = x.size(2), w = x.size(3);
  if (!bwd) {
    H = h;
    W = w;
  }
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  if (bwd) TORCH_CHECK(h == OH && w == OW, "avgpool3s2 bwd: geometry");
  Tensor y = bwd ? empty_nhwc(N, C, H, W, x) : empty_nhwc(N, C, OH, OW, x);
  check_rc(p2p_avgpool3s2(x.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)OH, (int)OW, y.data_ptr(),
                          (int)bwd, cur_stream(x)),
           "avgpool3s2");
  return y;
}

// input gradient of a stride-1 conv with one output channel (csrc/dgrad_c1.hip): gy is the
// output gradient padded to C8 channels (channel 0 live), w the fp32 master weight
// [1][Cp][KH][KW]; dX [N][Cp][OH][OW] NHWC, times the optional device scalar alpha (SN 1/sigma)
Tensor dgrad_c1(const Tensor& gy, const Tensor& w, int64_t pad, int64_t OH, int64_t OW,
                const optional<Tensor>& alpha) {
  check_nhwc(gy, "dgrad_c1 gy");
  const int64_t N = gy.size(0), C8 = gy.size(1), H = gy.size(2), W = gy.size(3);
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.is_contiguous() && w.dim() == 4 && w.size(0) == 1,
              "dgrad_c1: fp32 master weight [1][Cin][KH][KW]");
  const int64_t Cp = w.size(1), KH = w.size(2), KW = w.size(3);
  TORCH_CHECK(OH + 2 * pad - KH + 1 == H && OW + 2 * pad - KW + 1 == W,
              "dgrad_c1: (OH, OW) must be the stride-1 conv's input size");
  if (alpha) TORCH_CHECK(alpha->is_cuda() && alpha->scalar_type() == at::kFloat && alpha->numel() == 1, "dgrad_c1: alpha");
  Tensor dx = empty_nhwc(N, Cp, OH, OW, gy);
  const int rc = p2p_dgrad_c1(gy.data_ptr(), (int)C8, (int)N, (int)H, (int)W, w.data_ptr<float>(), (int)KH, (int)KW,
                              (int)pad, (int)OH, (int)OW, (int)Cp, alpha ? alpha->data_ptr<float>() : nullptr,
                              dx.data_ptr(), cur_stream(gy));
  TORCH_CHECK(rc != -2, "dgrad_c1: geometry not covered (16 taps, Cin / 8 a power of two <= 64)");
  check_rc(rc, "dgrad_c1");
  return dx;
}

Tensor maxpool2(const Tensor& x, const optional<Tensor>& gy) {
  check_nhwc(x, "maxpool2");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  Tensor out = gy ? empty_nhwc(N, C, H, W, x) : empty_nhwc(N, C, H / 2, W / 2, x);
  if (gy) check_nhwc(*gy, "maxpool2 gy");
  check_rc(p2p_maxpool2(x.data_ptr(), gy ? gy->data_ptr() : nullptr, (int)N, (int)H, (int)W, (int)C,
                        out.data_ptr(), cur_stream(x)),
           "maxpool2");
  return out;
}

// shuffle > 1: x is the pre-PixelShuffle tensor (C*r*r, H, W); the forward's output / the
// backward's gy are the shuffled (C, H*r, W*r) one, the backward's dx is x-shaped again
Tensor l2norm(const Tensor& x, const optional<Tensor>& gy, double eps, const optional<Tensor>& res, int64_t shuffle) {
  check_nhwc(x, "l2norm");
  const int64_t r = shuffle;
  TORCH_CHECK(r >= 1 && x.size(1) % (r * r) == 0, "l2norm: channels % shuffle^2");
  const int64_t N = x.size(0), C = x.size(1) / (r * r), IH = x.size(2), IW = x.size(3);
  if (gy) {
    check_nhwc(*gy, "l2norm gy");
    TORCH_CHECK(gy->size(0) == N && gy->size(1) == C && gy->size(2) == IH * r && gy->size(3) == IW * r,
                "l2norm: gy must be the (shuffled) output's shape");
  }
  if (res) {
    check_nhwc(*res, "l2norm res");
    TORCH_CHECK(!gy && res->size(0) == N && res->size(1) == C && res->size(2) == IH * r && res->size(3) == IW * r,
                "l2norm: res must match the output (forward only)");
  }
  Tensor out = gy ? at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast))
                  : empty_nhwc(N, C, IH * r, IW * r, x);
  check_rc(p2p_l2norm(x.data_ptr(), gy ? gy->data_ptr() : nullptr, N * IH * r * IW * r, (int)C, (float)eps,
                      res ? res->data_ptr() : nullptr, out.data_ptr(), (int)r, (int)IH, (int)IW, cur_stream(x)),
           "l2norm");
  return out;
}

// dir 0: unshuffle (C,H,W) -> (C*r*r, H/r, W/r); dir 1: shuffle (C,H,W) -> (C/(r*r), H*r, W*r)
Tensor pixel_shuffle(const Tensor& x, int64_t r, int64_t dir) {
  check_nhwc(x, "pixel_shuffle");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  int64_t OC, OH, OW;
  if (dir == 0) {
    TORCH_CHECK(H % r == 0 && W % r == 0, "pixel_unshuffle: H, W % r");
    OC = C * r * r;
    OH = H / r;
    OW = W / r;
  } else {
    TORCH_CHECK(C % (r * r) == 0, "pixel_shuffle: C % r^2");
    OC = C / (r * r);
    OH = H * r;
    OW = W * r;
  }
  Tensor out = empty_nhwc(N, OC, OH, OW, x);
  check_rc(p2p_pixel_shuffle(x.data_ptr(), (int)N, (int)OH, (int)OW, (int)OC, (int)r, (int)dir, out.data_ptr(),
                             cur_stream(x)),
           "pixel_shuffle");
  return out;
}

// pad_fold: gradient of a virtual reflect/zero-padded + nearest-upsampled input -> real input
Tensor pad_fold(const Tensor& dxp, int64_t H, int64_t W, int64_t pad, int64_t up, int64_t reflect,
                const optional<Tensor>& xb, int64_t act, const optional<Tensor>& res) {
  TORCH_CHECK(dxp.is_cuda() && dxp.scalar_type() == at::kBFloat16 && dxp.dim() == 4, "pad_fold: dxp");
  TORCH_CHECK(dxp.is_contiguous(at::MemoryFormat::ChannelsLast), "pad_fold: NHWC input");
  const int64_t N = dxp.size(0), C = dxp.size(1);
  TORCH_CHECK(C % 8 == 0, "pad_fold: C % 8");
  TORCH_CHECK(dxp.size(2) == H * up + 2 * pad && dxp.size(3) == W * up + 2 * pad, "pad_fold: geometry");
  TORCH_CHECK(!act || (xb && xb->is_contiguous(at::MemoryFormat::ChannelsLast) && xb->size(1) == C),
              "pad_fold: xb");
  if (res)
    TORCH_CHECK(res->scalar_type() == at::kBFloat16 && res->is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    res->size(0) == N && res->size(1) == C && res->size(2) == H && res->size(3) == W,
                "pad_fold: res must match dx");
  Tensor dx = empty_nhwc(N, C, H, W, dxp);
  check_rc(p2p_pad_fold(dxp.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)pad, (int)up, (int)reflect,
                        act ? xb->data_ptr() : nullptr, (int)act, res ? res->data_ptr() : nullptr, dx.data_ptr(),
                        cur_stream(dxp)),
           "pad_fold");
  return dx;
}

// pad_channels: NHWC a (Ca) [+ b (Cb)] -> Co channels, zero filled
Tensor pad_channels(const Tensor& a, const optional<Tensor>& b, int64_t Co) {
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == at::kBFloat16 && a.dim() == 4, "pad_channels: a");
  Tensor ac = a.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor bc;
  int64_t Cb = 0;
  if (b) {
    bc = b->contiguous(at::MemoryFormat::ChannelsLast);
    Cb = bc.size(1);
  }
  TORCH_CHECK(ac.size(1) + Cb <= Co, "pad_channels: Co too small");
  Tensor out = empty_nhwc(a.size(0), Co, a.size(2), a.size(3), a);
  check_rc(p2p_pad_channels(ac.data_ptr(), (int)ac.size(1), bc.defined() ? bc.data_ptr() : nullptr,
                            (int)Cb, a.size(0) * a.size(2) * a.size(3), (int)Co, out.data_ptr(),
                            cur_stream(a)),
           "pad_channels");
  return out;
}

// pad_channels_into: the same into a caller-provided NHWC view (a batch slice of a bigger
// packed tensor: the two halves of the fused D batch are packed straight into one buffer)
void pad_channels_into(const Tensor& a, const optional<Tensor>& b, const Tensor& out) {
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == at::kBFloat16 && a.dim() == 4, "pad_channels_into: a");
  check_act(out, "pad_channels_into out");
  Tensor ac = a.contiguous(at::MemoryFormat::ChannelsLast);
  Tensor bc;
  int64_t Cb = 0;
  if (b) {
    bc = b->contiguous(at::MemoryFormat::ChannelsLast);
    TORCH_CHECK(bc.size(0) == a.size(0) && bc.size(2) == a.size(2) && bc.size(3) == a.size(3),
                "pad_channels_into: b shape");
    Cb = bc.size(1);
  }
  const int64_t Co = out.size(1);
  TORCH_CHECK(out.size(0) == a.size(0) && out.size(2) == a.size(2) && out.size(3) == a.size(3) &&
                  ac.size(1) + Cb <= Co && Co % 8 == 0,
              "pad_channels_into: out shape");
  check_rc(p2p_pad_channels(ac.data_ptr(), (int)ac.size(1), bc.defined() ? bc.data_ptr() : nullptr,
                            (int)Cb, a.size(0) * a.size(2) * a.size(3), (int)Co, out.data_ptr(),
                            cur_stream(a)),
           "pad_channels_into");
}

Tensor slice_channels(const Tensor& x, int64_t c0, int64_t C) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4, "slice_channels: x");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "slice_channels: NHWC input");
  TORCH_CHECK(c0 + C <= x.size(1), "slice_channels: range");
  Tensor out = empty_nhwc(x.size(0), C, x.size(2), x.size(3), x);
  check_rc(p2p_slice_channels(x.data_ptr(), (int)x.size(1), (int)c0, x.size(0) * x.size(2) * x.size(3),
                              (int)C, out.data_ptr(), cur_stream(x)),
           "slice_channels");
  return out;
}

// out[c] (+)= scale * sum over all pixels of x[..., c]   (bias gradient)
// ------------------------------------------------------------------ spectral norm (csrc/sn.hip)
// one power iteration on W [h][wd] (fp32): v <- l2n(W^T u), u <- l2n(W v) in place; returns
// sigma = u . (W v) as a 0-dim fp32 tensor
Tensor sn_power_iter(const Tensor& w, Tensor u, Tensor v) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.is_contiguous() && w.dim() == 2,
              "sn_power_iter: fp32 contiguous [h][wd] weight");
  const int64_t h = w.size(0), wd = w.size(1);
  TORCH_CHECK(u.scalar_type() == at::kFloat && u.is_contiguous() && u.numel() == h, "sn_power_iter: u");
  TORCH_CHECK(v.scalar_type() == at::kFloat && v.is_contiguous() && v.numel() == wd, "sn_power_iter: v");
  Tensor ws = at::empty({p2p_sn_ws_floats((int)h, (int)wd)}, w.options());
  Tensor sigma = at::empty({}, w.options());
  check_rc(p2p_sn_power_iter(w.data_ptr<float>(), (int)h, (int)wd, u.data_ptr<float>(), v.data_ptr<float>(),
                             sigma.data_ptr<float>(), ws.data_ptr<float>(), nullptr, cur_stream(w)),
           "sn_power_iter");
  return sigma;
}

// one power iteration, returning 1 / sigma (the conv epilogues' scale; no autograd here --
// sn_wgrad carries the sigma path of the weight gradient)
Tensor sn_scale(const Tensor& w, Tensor u, Tensor v) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.is_contiguous() && w.dim() == 2,
              "sn_scale: fp32 contiguous [h][wd] weight");
  const int64_t h = w.size(0), wd = w.size(1);
  TORCH_CHECK(u.scalar_type() == at::kFloat && u.is_contiguous() && u.numel() == h, "sn_scale: u");
  TORCH_CHECK(v.scalar_type() == at::kFloat && v.is_contiguous() && v.numel() == wd, "sn_scale: v");
  Tensor ws = at::empty({p2p_sn_ws_floats((int)h, (int)wd) + 1}, w.options());
  Tensor scale = at::empty({1}, w.options());
  check_rc(p2p_sn_power_iter(w.data_ptr<float>(), (int)h, (int)wd, u.data_ptr<float>(), v.data_ptr<float>(),
                             ws.data_ptr<float>() + p2p_sn_ws_floats((int)h, (int)wd), ws.data_ptr<float>(),
                             scale.data_ptr<float>(), cur_stream(w)),
           "sn_scale");
  return scale;
}

// dL/dW_bar of a spectral-norm conv from its conv weight gradient G (see csrc/sn.hip)
// acc: add this gradient into acc (a later contribution of the same backward) and return it
Tensor sn_wgrad(const Tensor& G, const Tensor& w, const Tensor& u, const Tensor& v, const Tensor& scale,
                const optional<Tensor>& acc) {
  TORCH_CHECK(G.is_cuda() && G.scalar_type() == at::kFloat && G.is_contiguous(), "sn_wgrad: G fp32 contiguous");
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.numel() == G.numel(), "sn_wgrad: W like G");
  const int64_t h = u.numel(), wd = v.numel();
  TORCH_CHECK(h * wd == G.numel() && u.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat &&
                  u.is_contiguous() && v.is_contiguous(), "sn_wgrad: u / v");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.numel() == 1, "sn_wgrad: scale");
  Tensor part = at::empty({p2p_sn_wgrad_blocks(h * wd)}, G.options());
  if (acc) TORCH_CHECK(acc->is_cuda() && acc->scalar_type() == at::kFloat && acc->is_contiguous() &&
                       acc->numel() == G.numel(), "sn_wgrad: acc fp32 contiguous like G");
  Tensor out = acc ? *acc : at::empty_like(G);
  check_rc(p2p_sn_wgrad(G.data_ptr<float>(), w.data_ptr<float>(), u.data_ptr<float>(), v.data_ptr<float>(),
                        scale.data_ptr<float>(), (int)h, (int)wd, part.data_ptr<float>(), out.data_ptr<float>(),
                        acc ? 1 : 0, cur_stream(G)),
           "sn_wgrad");
  return out;
}

// ------------------------------------------------------------------ fp8 (csrc/fp8.hip)

Tensor fp8_quant(const Tensor& x, Tensor site, int64_t fmt, int64_t use_cur) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16, "fp8_quant: bf16 input");
  TORCH_CHECK(x.is_contiguous() || x.is_contiguous(at::MemoryFormat::ChannelsLast), "fp8_quant: dense input");
  TORCH_CHECK(x.numel() % 8 == 0, "fp8_quant: numel % 8");
  TORCH_CHECK(fmt == 0 || fmt == 1, "fp8_quant: fmt 0 (e4m3) or 1 (e5m2)");
  check_site(site);
  Tensor q = at::empty_like(x, x.options().dtype(fmt == 0 ? at::kFloat8_e4m3fn : at::kFloat8_e5m2),
                            at::MemoryFormat::Preserve);
  check_rc(p2p_fp8_quant(x.data_ptr(), x.numel(), site.data_ptr<int>(), (int)use_cur, (int)fmt, q.data_ptr(),
                         cur_stream(x)),
           "fp8_quant");
  return q;
}

void fp8_amax(const Tensor& x, Tensor site, int64_t slot) {
  TORCH_CHECK(x.is_cuda() && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat), "fp8_amax: input");
  TORCH_CHECK(x.is_contiguous() || x.is_contiguous(at::MemoryFormat::ChannelsLast), "fp8_amax: dense input");
  TORCH_CHECK(slot >= 0 && slot < 4, "fp8_amax: slot");
  check_site(site);
  check_rc(p2p_fp8_amax(x.data_ptr(), x.scalar_type() == at::kFloat, x.numel(), site.data_ptr<int>(), (int)slot,
                        cur_stream(x)),
           "fp8_amax");
}

// amax of every fp32 tensor x[i] -> sites[idx[i]][0] (pre-zeroed by the caller)
void fp8_amax_multi(at::TensorList xs, Tensor sites, at::IntArrayRef idx) {
  TORCH_CHECK(xs.size() == idx.size(), "fp8_amax_multi: list sizes");
  TORCH_CHECK(sites.is_cuda() && sites.scalar_type() == at::kInt && sites.is_contiguous() && sites.dim() == 2 &&
                  sites.size(1) == 4,
              "fp8_amax_multi: int32 [n][4] pool");
  constexpr int MAXT = 48;
  size_t i0 = 0;
  while (i0 < xs.size()) {
    const size_t cnt = std::min<size_t>(MAXT, xs.size() - i0);
    std::vector<const float*> xp(cnt);
    std::vector<long> n(cnt);
    std::vector<int*> sp(cnt);
    for (size_t i = 0; i < cnt; ++i) {
      const Tensor& t = xs[i0 + i];
      TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), "fp8_amax_multi: fp32 input");
      TORCH_CHECK(idx[i0 + i] >= 0 && idx[i0 + i] < sites.size(0), "fp8_amax_multi: site index");
      xp[i] = t.data_ptr<float>();
      n[i] = t.numel();
      sp[i] = sites.data_ptr<int>() + 4 * idx[i0 + i];
    }
    check_rc(p2p_fp8_amax_multi((int)cnt, xp.data(), n.data(), sp.data(), cur_stream(sites)), "fp8_amax_multi");
    i0 += cnt;
  }
}

// word `word` of the first n sites of a [.][4] int32 pool (or of one [4] site) := 0
void fp8_word_zero(Tensor sites, int64_t n, int64_t word) {
  TORCH_CHECK(sites.is_cuda() && sites.scalar_type() == at::kInt && sites.is_contiguous() && sites.numel() >= 4 * n &&
                  word >= 0 && word < 4,
              "fp8_word_zero: int32 [n][4] sites");
  check_rc(p2p_fp8_word_zero(sites.data_ptr<int>(), (int)n, (int)word, cur_stream(sites)), "fp8_word_zero");
}

void fp8_roll(Tensor sites) {
  TORCH_CHECK(sites.is_cuda() && sites.scalar_type() == at::kInt && sites.is_contiguous() && sites.numel() % 4 == 0,
              "fp8_roll: int32 [n][4] pool");
  check_rc(p2p_fp8_roll(sites.data_ptr<int>(), (int)(sites.numel() / 4), cur_stream(sites)), "fp8_roll");
}

Tensor fp8_dequant(const Tensor& q, const Tensor& site) {
  const auto dt = q.scalar_type();
  TORCH_CHECK(q.is_cuda() && (dt == at::kFloat8_e4m3fn || dt == at::kFloat8_e5m2), "fp8_dequant: fp8 input");
  TORCH_CHECK(q.is_contiguous() || q.is_contiguous(at::MemoryFormat::ChannelsLast), "fp8_dequant: dense input");
  check_site(site);
  Tensor y = at::empty_like(q, q.options().dtype(at::kBFloat16), at::MemoryFormat::Preserve);
  check_rc(p2p_fp8_dequant(q.data_ptr(), q.numel(), site.data_ptr<int>(), dt == at::kFloat8_e5m2 ? 1 : 0,
                           y.data_ptr(), cur_stream(q)),
           "fp8_dequant");
  return y;
}

void colsum(const Tensor& x, Tensor out, double scale, bool accumulate) {
  check_act(x, "colsum x");
  const int64_t C = x.size(1), M = x.numel() / C;
  TORCH_CHECK(C <= 2048, "colsum: C > 2048");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.numel() <= C && out.is_contiguous(),
              "colsum: out");
  const int nb = p2p_colsum_blocks(M, (int)C);
  Tensor ws = at::empty({(int64_t)nb * C}, x.options().dtype(at::kFloat));
  // padded channels (out.numel() < C): the kernel writes the leading out.numel() only
  check_rc(p2p_colsum(x.data_ptr(), M, (int)C, (float)scale, accumulate ? 1 : 0, ws.data_ptr<float>(),
                      out.data_ptr<float>(), (int)out.numel(), cur_stream(x)),
           "colsum");
}

// ------------------------------------------------------------------ losses
Tensor loss_fwd(const Tensor& a, const optional<Tensor>& b, int64_t kind, double t, double scale) {
  TORCH_CHECK(a.is_cuda() && (a.scalar_type() == at::kBFloat16 || a.scalar_type() == at::kFloat),
              "loss_fwd: a");
  TORCH_CHECK(a.is_contiguous() || a.is_contiguous(at::MemoryFormat::ChannelsLast), "loss_fwd: dense a");
  if (b) {
    TORCH_CHECK(b->scalar_type() == a.scalar_type() && b->sizes() == a.sizes() &&
                    b->strides() == a.strides(), "loss_fwd: b must match a");
  }
  const int nb = p2p_loss_blocks(a.numel());
  Tensor ws = at::empty({nb}, a.options().dtype(at::kFloat));
  Tensor out = at::empty({}, a.options().dtype(at::kFloat));
  check_rc(p2p_loss_fwd(a.data_ptr(), b ? b->data_ptr() : nullptr, a.scalar_type() == at::kFloat,
                        a.numel(), (int)kind, (float)t, (float)scale, ws.data_ptr<float>(),
                        out.data_ptr<float>(), cur_stream(a)),
           "loss_fwd");
  return out;
}

std::vector<Tensor> loss_bwd(const Tensor& a, const optional<Tensor>& b, int64_t kind, double t,
                             double scale, const Tensor& gout, bool need_a, bool need_b) {
  TORCH_CHECK(gout.scalar_type() == at::kFloat && gout.numel() == 1, "loss_bwd: gout");
  Tensor gout_c = gout.contiguous();
  Tensor ga, gb;
  if (need_a) ga = at::empty_like(a);
  if (need_b) gb = at::empty_like(a);
  check_rc(p2p_loss_bwd(a.data_ptr(), b ? b->data_ptr() : nullptr, a.scalar_type() == at::kFloat,
                        a.numel(), (int)kind, (float)t, (float)scale, gout_c.data_ptr<float>(),
                        need_a ? ga.data_ptr() : nullptr, need_b ? gb.data_ptr() : nullptr,
                        cur_stream(a)),
           "loss_bwd");
  return {ga, gb};
}

// ------------------------------------------------------------------ small-tensor helpers
// out = wa * a + wb * b + c over fp32 tensors of one shape (the step's scalar bookkeeping)
Tensor lincomb(const Tensor& a, const optional<Tensor>& b, double wa, double wb, double c) {
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == at::kFloat && a.is_contiguous(), "lincomb: a fp32 contiguous");
  TORCH_CHECK(!b || (b->scalar_type() == at::kFloat && b->is_contiguous() && b->numel() == a.numel()),
              "lincomb: b like a");
  Tensor out = at::empty_like(a);
  check_rc(p2p_lincomb(a.data_ptr<float>(), b ? b->data_ptr<float>() : nullptr, (float)wa, (float)wb, (float)c,
                       a.numel(), out.data_ptr<float>(), cur_stream(a)),
           "lincomb");
  return out;
}

// in place: t = wa * t + wb * b + c
void lincomb_(Tensor t, const optional<Tensor>& b, double wa, double wb, double c) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), "lincomb_: t fp32 contiguous");
  TORCH_CHECK(!b || (b->scalar_type() == at::kFloat && b->is_contiguous() && b->numel() == t.numel()),
              "lincomb_: b like t");
  check_rc(p2p_lincomb(t.data_ptr<float>(), b ? b->data_ptr<float>() : nullptr, (float)wa, (float)wb, (float)c,
                       t.numel(), t.data_ptr<float>(), cur_stream(t)),
           "lincomb_");
}

void i64_add_(Tensor t, int64_t v) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kLong && t.is_contiguous(), "i64_add_: int64 contiguous");
  check_rc(p2p_i64_add(reinterpret_cast<long long*>(t.data_ptr<int64_t>()), (long long)v, t.numel(), cur_stream(t)),
           "i64_add_");
}

// sum_i w_i * t_i over up to 16 one-element fp32 tensors (a composed loss) -> 0-d tensor
Tensor lincomb_n(at::TensorList ts, at::ArrayRef<double> ws) {
  TORCH_CHECK(!ts.empty() && ts.size() <= 16 && ts.size() == ws.size(), "lincomb_n: 1..16 terms, one weight each");
  std::vector<const float*> p;
  std::vector<float> w;
  for (size_t i = 0; i < ts.size(); ++i) {
    TORCH_CHECK(ts[i].is_cuda() && ts[i].scalar_type() == at::kFloat && ts[i].numel() == 1, "lincomb_n: fp32 scalars");
    p.push_back(ts[i].data_ptr<float>());
    w.push_back((float)ws[i]);
  }
  Tensor out = at::empty({}, ts[0].options());
  check_rc(p2p_lincomb_n(p.data(), w.data(), (int)p.size(), out.data_ptr<float>(), cur_stream(ts[0])), "lincomb_n");
  return out;
}

// [n] = w_i * g (the n-term sum's backward)
Tensor scale_n(const Tensor& g, at::ArrayRef<double> ws) {
  TORCH_CHECK(g.is_cuda() && g.scalar_type() == at::kFloat && g.numel() == 1 && ws.size() >= 1 && ws.size() <= 16,
              "scale_n: fp32 scalar, 1..16 weights");
  std::vector<float> w(ws.begin(), ws.end());
  Tensor gc = g.contiguous();
  Tensor out = at::empty({(int64_t)w.size()}, g.options());
  check_rc(p2p_scale_n(gc.data_ptr<float>(), w.data(), (int)w.size(), out.data_ptr<float>(), cur_stream(g)),
           "scale_n");
  return out;
}

// column sums of an fp32 [..., C] partial-sum image (rows in fixed order)
// timeline probe of the s2t kernel (P2P_S2T_DEBUG=1): int64 [blocks][tiles][4] on the host
Tensor s2t_debug() {
  (void)hipDeviceSynchronize();
  const long n = p2p_s2t_dbg_bytes() / 8;
  Tensor out = at::empty({n}, at::TensorOptions().dtype(at::kLong));
  check_rc(p2p_s2t_dbg_read(out.data_ptr(), n * 8), "s2t_debug");
  return out;
}

Tensor rowsum(const Tensor& ws) {
  TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.dim() >= 1,
              "rowsum: fp32 contiguous");
  const int64_t C = ws.size(-1);
  const int64_t R = ws.numel() / std::max<int64_t>(C, 1);
  Tensor out = at::empty({C}, ws.options());
  Tensor tmp = at::empty({(int64_t)p2p_rowsum_blocks(R) * C}, ws.options());
  check_rc(p2p_rowsum_f32(ws.data_ptr<float>(), R, (int)C, tmp.data_ptr<float>(), out.data_ptr<float>(),
                          cur_stream(ws)),
           "rowsum");
  return out;
}

// ------------------------------------------------------------------ optimizer
void adam(at::TensorList p, at::TensorList g, at::TensorList m, at::TensorList v, const Tensor& lr,
          const Tensor& step, double b1, double b2, double eps, double wd, const optional<Tensor>& skip) {
  const size_t n = p.size();
  TORCH_CHECK(!skip || skip->scalar_type() == at::kFloat, "adam: skip flag fp32");
  TORCH_CHECK(g.size() == n && m.size() == n && v.size() == n, "adam: list sizes");
  TORCH_CHECK(lr.scalar_type() == at::kFloat && step.scalar_type() == at::kFloat, "adam: lr/step fp32");
  const int maxT = p2p_adam_max_tensors();
  std::vector<float*> P, M, V;
  std::vector<const float*> G;
  std::vector<long> Nn;
  hipStream_t st = n ? cur_stream(p[0]) : nullptr;
  auto flush = [&]() {
    if (P.empty()) return;
    check_rc(p2p_adam((int)P.size(), P.data(), G.data(), M.data(), V.data(), Nn.data(),
                      lr.data_ptr<float>(), step.data_ptr<float>(), skip ? skip->data_ptr<float>() : nullptr,
                      (float)b1, (float)b2, (float)eps,
                      (float)wd, st),
             "adam");
    P.clear(); G.clear(); M.clear(); V.clear(); Nn.clear();
  };
  for (size_t i = 0; i < n; ++i) {
    TORCH_CHECK(p[i].scalar_type() == at::kFloat && p[i].is_contiguous() && g[i].is_contiguous() &&
                    m[i].is_contiguous() && v[i].is_contiguous() && g[i].scalar_type() == at::kFloat,
                "adam: fp32 contiguous tensors");
    TORCH_CHECK(p[i].numel() == g[i].numel() && p[i].numel() < (1ll << 31), "adam: sizes");
    P.push_back(p[i].data_ptr<float>());
    G.push_back(g[i].data_ptr<float>());
    M.push_back(m[i].data_ptr<float>());
    V.push_back(v[i].data_ptr<float>());
    Nn.push_back((long)p[i].numel());
    if ((int)P.size() == maxT) flush();
  }
  flush();
}

}  // namespace

// NaN / Inf guard: fp32 flag (1 = some loss is not finite) and counter += flag, one launch
Tensor guard_flag(const std::vector<Tensor>& losses, const optional<Tensor>& counter) {
  TORCH_CHECK(!losses.empty() && losses.size() <= 8, "guard_flag: 1..8 loss scalars");
  const float* v[8] = {};
  for (size_t i = 0; i < losses.size(); ++i) {
    TORCH_CHECK(losses[i].is_cuda() && losses[i].scalar_type() == at::kFloat && losses[i].numel() == 1,
                "guard_flag: fp32 one-element GPU tensors");
    v[i] = losses[i].data_ptr<float>();
  }
  if (counter)
    TORCH_CHECK(counter->is_cuda() && counter->scalar_type() == at::kFloat && counter->numel() == 1,
                "guard_flag: counter is a one-element fp32 GPU tensor");
  Tensor flag = at::empty({}, losses[0].options());
  check_rc(p2p_guard_flag(v, (int)losses.size(), flag.data_ptr<float>(),
                          counter ? counter->data_ptr<float>() : nullptr, cur_stream(losses[0])),
           "guard_flag");
  return flag;
}

TORCH_LIBRARY(p2p, m) {
  m.def("conv_fwd(Tensor x1, Tensor? x2, Tensor w, Tensor? bias, int mode, int KH, int KW, int stride, "
        "int pad, int reflect, int up, int act_in, int OH, int OW, int Cout, int act_out, int Csplit, "
        "Tensor? xb1, Tensor? xb2, int act_bwd, int Cvalid=0, bool want_stats=False, Tensor? qs_x1=None, "
        "Tensor? qs_x2=None, Tensor? qs_w=None, Tensor(a!)? y_qsite=None, int y_qfmt=0, Tensor? res=None, "
        "Tensor? alpha=None, Tensor? nb_x=None, Tensor? nb_mean=None, Tensor? nb_rstd=None, "
        "Tensor? nb_gamma=None, Tensor? nb_beta=None, int nb_act=0, int nb_half=0, bool nb_batch=False, "
        "bool nb_colsum=False, bool nb_gate=False, int fold_H=0, int fold_W=0, int fold_p=0, int fold_edge=0, "
        "Tensor? nb_prelu=None) -> Tensor[]");
  m.def("fp8_quant(Tensor x, Tensor(a!) site, int fmt, int use_cur=0) -> Tensor");
  m.def("sn_power_iter(Tensor w, Tensor(a!) u, Tensor(b!) v) -> Tensor");
  m.def("sn_scale(Tensor w, Tensor(a!) u, Tensor(b!) v) -> Tensor");
  m.def("sn_wgrad(Tensor G, Tensor w, Tensor u, Tensor v, Tensor scale, Tensor(a!)? acc=None) -> Tensor");
  m.def("fp8_amax(Tensor x, Tensor(a!) site, int slot) -> ()");
  m.def("fp8_roll(Tensor(a!) sites) -> ()");
  m.def("fp8_word_zero(Tensor(a!) sites, int n, int word) -> ()");
  m.def("fp8_amax_multi(Tensor[] x, Tensor(a!) sites, int[] idx) -> ()");
  m.def("fp8_dequant(Tensor q, Tensor site) -> Tensor");
  m.def("conv_wgrad(Tensor p1, Tensor? p2, int p_act, Tensor q1, Tensor? q2, int q_act, int KH, int KW, "
        "int stride, int pad, int reflect, int up, Tensor(a!) dw, float scale, int accumulate, "
        "int flip=0, Tensor? qs_p=None, Tensor? qs_q=None, int p_fmt=0, int q_fmt=0, Tensor? qs_p2=None, "
        "Tensor? qs_q2=None) -> bool");
  m.def("weight_prep(Tensor w, int swap, int Xp, int Yp, Tensor? scale) -> Tensor");
  m.def("up2_dgrad_image(Tensor w, int Xp, int Yp) -> Tensor");
  m.def("oob_selftest(Tensor scratch) -> ()");
  m.def("vec_pad_into(Tensor x, Tensor(a!) out, float fill) -> ()");
  m.def("set_m32(int on) -> int", set_m32);
  m.def("oob_counts(bool reset) -> int[]", oob_counts);   // no tensor arguments: a catch-all kernel
  m.def("union_weight(Tensor w, int co_off, int nv, int Nrows, int Cpad, Tensor? bias) -> Tensor[]");
  m.def("conv_d2s(Tensor x1, Tensor? x2, Tensor w, Tensor bias, int act_in, int act_out, int mode, "
        "Tensor(a!) out, Tensor pk_a, Tensor? pk_f, float scale, Tensor? wscale=None) -> Tensor");
  m.def("prelu_fwd(Tensor x, Tensor w) -> Tensor");
  m.def("prelu_bwd(Tensor x, Tensor gy, Tensor w, bool need_x) -> Tensor[]");
  m.def("tv_fwd(Tensor x) -> Tensor");
  m.def("tv_bwd(Tensor x, Tensor gout) -> Tensor");
  m.def("quantize(Tensor x, int bits) -> Tensor");
  m.def("quantize_unshuffle(Tensor x, int bits, int r, int cp) -> Tensor[]");
  m.def("image_metrics(Tensor a, Tensor b, bool shift, float data_range) -> Tensor");
  m.def("avgpool3s2(Tensor x, int bwd, int H, int W) -> Tensor");
  m.def("maxpool2(Tensor x, Tensor? gy) -> Tensor");
  m.def("dgrad_c1(Tensor gy, Tensor w, int pad, int OH, int OW, Tensor? alpha=None) -> Tensor");
  m.def("l2norm(Tensor x, Tensor? gy, float eps, Tensor? res=None, int shuffle=1) -> Tensor");
  m.def("pixel_shuffle(Tensor x, int r, int dir) -> Tensor");
  m.def("pad_fold(Tensor dxp, int H, int W, int pad, int up, int reflect, Tensor? xb, int act, "
        "Tensor? res=None) -> Tensor");
  m.def("weight_prep_pairs(Tensor[] w, int[] xa, int[] xb, Tensor(a!)? sites=None, int[]? site_idx=None) -> Tensor[]");
  m.def("weight_prep_multi(Tensor[] w, int[] swap, int[] xp, int[] yp) -> Tensor[]");
  m.def("norm_fwd(Tensor x, float eps, Tensor? gamma, Tensor? beta, Tensor? prelu_w, int act, "
        "Tensor(a!)? run_mean, Tensor(b!)? run_var, float momentum, bool batch, Tensor? partials=None, "
        "Tensor(c!)? qsite=None, Tensor(d!)? q_out=None, int qfmt=0, Tensor? res=None) -> Tensor[]");
  m.def("norm_apply(Tensor x, Tensor mean, Tensor rstd, Tensor? gamma, Tensor? beta, Tensor? prelu_w, "
        "int act, bool batch, Tensor? res=None) -> Tensor");
  m.def("norm_bwd(Tensor x, Tensor dy, Tensor mean, Tensor rstd, Tensor? gamma, Tensor? beta, int act, "
        "Tensor(a!)? dgamma, Tensor(b!)? dbeta, bool need_dx, bool batch, Tensor(c!)? dsum, "
        "Tensor(d!)? qsite=None, Tensor(e!)? q_out=None, int qfmt=0, Tensor? prelu_w=None, "
        "Tensor(f!)? dprelu=None, Tensor? partials=None, bool frozen=False) -> Tensor");
  m.def("act(Tensor a, Tensor? b, int act, int mode) -> Tensor");
  m.def("dropout(Tensor x, float p, Tensor seed, int salt) -> Tensor");
  m.def("pad_channels(Tensor a, Tensor? b, int Co) -> Tensor");
  m.def("pad_channels_into(Tensor a, Tensor? b, Tensor(a!) out) -> ()");
  m.def("slice_channels(Tensor x, int c0, int C) -> Tensor");
  m.def("colsum(Tensor x, Tensor(a!) out, float scale, bool accumulate) -> ()");
  m.def("lincomb(Tensor a, Tensor? b, float wa, float wb, float c) -> Tensor");
  m.def("lincomb_(Tensor(a!) t, Tensor? b, float wa, float wb, float c) -> ()");
  m.def("i64_add_(Tensor(a!) t, int v) -> ()");
  m.def("rowsum(Tensor ws) -> Tensor");
  m.def("s2t_debug() -> Tensor", &s2t_debug);
  m.def("lincomb_n(Tensor[] ts, float[] ws) -> Tensor");
  m.def("scale_n(Tensor g, float[] ws) -> Tensor");
  m.def("guard_flag(Tensor[] losses, Tensor(a!)? counter) -> Tensor");
  m.def("loss_fwd(Tensor a, Tensor? b, int kind, float t, float scale) -> Tensor");
  m.def("loss_bwd(Tensor a, Tensor? b, int kind, float t, float scale, Tensor gout, bool need_a, "
        "bool need_b) -> Tensor[]");
  m.def("adam(Tensor(a!)[] p, Tensor[] g, Tensor(b!)[] m, Tensor(c!)[] v, Tensor lr, Tensor step, "
        "float b1, float b2, float eps, float wd, Tensor? skip=None) -> ()");
}

TORCH_LIBRARY_IMPL(p2p, CUDA, m) {
  m.impl("conv_fwd", conv_fwd);
  m.impl("guard_flag", guard_flag);
  m.impl("fp8_quant", fp8_quant);
  m.impl("sn_power_iter", sn_power_iter);
  m.impl("sn_scale", sn_scale);
  m.impl("sn_wgrad", sn_wgrad);
  m.impl("fp8_amax", fp8_amax);
  m.impl("fp8_roll", fp8_roll);
  m.impl("fp8_word_zero", fp8_word_zero);
  m.impl("fp8_amax_multi", fp8_amax_multi);
  m.impl("fp8_dequant", fp8_dequant);
  m.impl("conv_wgrad", conv_wgrad);
  m.impl("weight_prep", weight_prep);
  m.impl("up2_dgrad_image", up2_dgrad_image);
  m.impl("oob_selftest", oob_selftest);
  m.impl("vec_pad_into", vec_pad_into);
  m.impl("union_weight", union_weight);
  m.impl("conv_d2s", conv_d2s);
  m.impl("weight_prep_multi", weight_prep_multi);
  m.impl("weight_prep_pairs", weight_prep_pairs);
  m.impl("norm_fwd", norm_fwd);
  m.impl("norm_apply", norm_apply);
  m.impl("norm_bwd", norm_bwd);
  m.impl("act", act);
  m.impl("dropout", dropout);
  m.impl("pad_channels", pad_channels);
  m.impl("pad_channels_into", pad_channels_into);
  m.impl("pad_fold", pad_fold);
  m.impl("prelu_fwd", prelu_fwd);
  m.impl("prelu_bwd", prelu_bwd);
  m.impl("tv_fwd", tv_fwd);
  m.impl("tv_bwd", tv_bwd);
  m.impl("quantize", quantize);
  m.impl("quantize_unshuffle", quantize_unshuffle);
  m.impl("image_metrics", image_metrics);
  m.impl("avgpool3s2", avgpool3s2);
  m.impl("maxpool2", maxpool2);
  m.impl("dgrad_c1", dgrad_c1);
  m.impl("l2norm", l2norm);
  m.impl("pixel_shuffle", pixel_shuffle);
  m.impl("slice_channels", slice_channels);
  m.impl("colsum", colsum);
  m.impl("lincomb", lincomb);
  m.impl("lincomb_", lincomb_);
  m.impl("i64_add_", i64_add_);
  m.impl("rowsum", rowsum);
  m.impl("lincomb_n", lincomb_n);
  m.impl("scale_n", scale_n);
  m.impl("loss_fwd", loss_fwd);
  m.impl("loss_bwd", loss_bwd);
  m.impl("adam", adam);
}
