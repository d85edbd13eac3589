// Argument blocks shared between the conv kernels and the host bindings.
#pragma once
#include <hip/hip_runtime.h>

namespace p2p {

// Implicit-GEMM convolution forward.  MODE 0 (CONV): gathered im2col over a NHWC input
// with stride / zero-or-reflect pad / nearest upsample / virtual concat / input act.
// MODE 1 (CONVT): transposed conv by sub-pixel decomposition -- one GEMM per output
// parity class, each with only the taps that hit that class (no zero-stuffing).
// Also used for conv dgrad (CONVT on dY with the transposed weight) and ConvT dgrad
// (CONV on dY).
struct ConvFwdArgs {
  const void* x1;  // NHWC bf16 [N][H][W][C1]
  const void* x2;  // NHWC bf16 [N][H][W][C2] (virtual concat), may be null
  int C1, C2, C;   // C = C1 + C2, all % 8 == 0
  int N, H, W;     // input spatial size (before upsample)
  int up;          // nearest upsample factor (1 or 2), CONV only
  int KH, KW, stride, pad, reflect;
  int act_in;      // activation applied to the input in the loader
  int OH, OW, Cout;
  const void* w;   // bf16 [Cout][KH][KW][C]
  const float* bias;  // [Cout] or null
  const float* alpha; // device scalar multiplying the accumulator before the bias (null = 1):
                      // spectral norm's 1 / sigma without materialising W / sigma
  int act_out;
  void* y1;        // bf16 output, channels [0, Csplit): NHWC with ld = Csplit
  void* y2;        // bf16 output, channels [Csplit, Cout): ld = Cout - Csplit (may be null)
  int Csplit;
  const void* xb1; // dgrad epilogue: multiply by act'(xb) (same channel split as y)
  const void* xb2;
  int act_bwd;
  const void* res1; // dgrad epilogue: + res1 (bf16, y1's layout) after the act' gate -- the
                    // other consumer's gradient of a tensor read twice (U-Net skips)
  float* ws;       // split-K fp32 accumulator [N*OH*OW][Cout] (pre-zeroed) when splits > 1
  int splits;
  int det;         // deterministic split-K: per-split slabs ws[split][N*OH*OW][Cout] (plain
                   // stores), summed in split order by the finalize -- bitwise repeatable
  const void* zero;  // >= 16 zero bytes in global memory (global_load_lds padding source)
  // Normalisation statistics fused into the epilogue (null = off): every BM-row tile (all
  // rows inside one image and one parity class -- host-checked) writes the per-channel
  // (mean, M2) of its bf16 outputs to stats[{0,1}][n][chunk][Cout], chunk = class * (Hq*Wq
  // / BM) + tile-in-class; the norm then only merges them (norm.hip finalize).
  float* stats;
  int stats_nchunks;  // chunks per image
  // fp8 operands (0 = bf16): 1 = x e4m3, 2 = x e5m2 (gradients); weights always e4m3.
  // qs_*: fp8 scale sites (csrc/fp8.hip) whose word [2] is the E8M0 dequant exponent.
  int fp8;
  const int* qs_x1;
  const int* qs_x2;
  const int* qs_w;
  // optional fp8 shadow of the (bf16) output, written by the epilogue in the same pass:
  // q_out [N*OH*OW][Cout] bytes, q_site its scale site, q_fmt 0 = e4m3 / 1 = e5m2
  void* q_out;
  int* q_site;
  int q_fmt;
  // Depth-to-space packed-image epilogue (0 = off).  The stride-2 4x4 pad-1 transposed conv
  // onto a small image is computed as a 3x3 pad-1 "union" conv over its input grid: GEMM
  // column n = cls * 4 + j (cls = ry * 2 + rx the output parity class, j < 3 the image
  // channel), so one GEMM row (grid position q) yields the 2x2 output pixels 2q + (ry, rx).
  // y1 is then a packed [N][2*OH][2*OW][8] bf16 image (16 B per pixel).
  //  1: image forward -- pixel = (pk_a[0..2], y[0..2], 0, 0): the pair (A | fake) written in
  //     place; per-block sum of |y - pk_a[3..5]| into l1_part[block] (the L1 term)
  //  2: head gradient -- pixel = ((g + d2s_scale * sign(f - b)) * (1 - f^2), 0...) with
  //     g the GEMM value, f = pk_f[3 + j] (tanh output), b = pk_a[3 + j] (target): the
  //     pre-tanh gradient of the generator's last layer, in slots 0..2
  int d2s;
  const void* pk_a;
  const void* pk_f;
  float d2s_scale;
  const float* d2s_w;   // mode 2: device multiplier of the sign term (dL/dl1; null = 1)
  float* l1_part;
  // Norm-backward partial sums fused into a dgrad epilogue (null nb_ws = off): the output
  // channels [nb_c0, nb_c0 + nb_C) are the gradient dz of a norm's output z = act(xhat*g + b)
  // (xhat = (x - mean) * rstd, x = nb_x [N][OH][OW][nb_C]); every BM-row tile (one image /
  // parity class, host-checked like ``stats``) writes sum(d) and sum(d * xhat), d = dz *
  // act'(z), per channel to nb_ws[{0,1}][n][chunk][nb_C] -- the norm backward's partial pass.
  const void* nb_x;
  const float* nb_mean;   // [N][nb_C] (instance) or [nb_C] (batch, nb_batch = 1)
  const float* nb_rstd;
  const float* nb_gamma;  // affine norms (batch norm only: the host checks): z = xhat * g + b
  const float* nb_beta;
  int nb_act, nb_batch, nb_c0, nb_C, nb_nchunks;
  float* nb_ws;
  int nb_colsum;    // 1: plain column sums sum(dz) of the half (the bias gradient of the conv
                    // that produced it), no norm input read: nb_ws[0] only, nb_x / stats unused
  int nb_gate;      // the act' gate of the nb half reads the norm's output, which IS xhat (non-affine,
                    // no fused act): compute the gate from the xhat the partials already form,
                    // instead of loading that output again (one operand stream fewer)
  // Pad fold of an input gradient computed on a padded grid OH x OW = (fold_H + 2p) x
  // (fold_W + 2p) (fold_buf null = off): an interior output pixel is stored straight into the
  // real input's gradient y1 [N][fold_H][fold_W] (act' gate and parked skip gradient as
  // usual); a pixel of the p-wide frame goes, raw, to fold_buf [N][OH][OW] -- only the frame
  // of which is ever written -- and elementwise.hip fold_band adds it (gated) onto the band
  // pixels it pads (reflect: the mirrored ones; edge: the replicated border) afterwards.
  // Reflect-pad dgrads (MODE 1 onto the padded grid) and the nearest-x2 + reflect-1 dgrad
  // (MODE 0, 4x4 stride 2 over dY onto the edge-padded grid).  Unsplit single-output GEMMs.
  void* fold_buf;
  int fold_H, fold_W, fold_p;
  // batch-norm partials over a whole batch (nb_batch): nb_flat = 1 -> chunk = class *
  // nb_tiles_cls + m0 / BM over ALL images (tiles may straddle images: a fold's padded grid),
  // planes [nb_planes][nb_nchunks][nb_C]; nb_prelu (device slope, shared-slope PReLU): the
  // gate slope, and a third plane of sum(dz * z * [z <= 0]) (the slope gradient's terms)
  const float* nb_prelu;
  int nb_flat, nb_tiles_cls, nb_planes;
};

// Weight gradient: C[R][Kq] = sum_m P[m][R] * im2col(Q)[m][Kq], written to per-split
// fp32 slabs ws[split][R][Kq] and reduced (deterministically) by wgrad_reduce.
struct ConvWgradArgs {
  // P: plain NHWC rows (optionally virtual concat + activation); rows m enumerate the
  // OUTPUT pixels of the CONV geometry below (N*OH*OW).
  const void* p1;
  const void* p2;
  int R1, R2, R;   // R = R1 + R2 (% 8 == 0)
  int p_act;
  // Q: gathered with the CONV geometry (like ConvFwdArgs MODE 0)
  const void* q1;
  const void* q2;
  int C1, C2, C;
  int N, H, W, up, KH, KW, stride, pad, reflect;
  int q_act;
  int OH, OW;
  float* ws;       // [splits][R][KH*KW*C]
  int splits;
  int M;           // N*OH*OW
  int Kq;          // KH*KW*C
  const void* zero;  // zero page for the global_load_lds variant
  // fp8 operands (f8 = 1): P and Q are 1-byte OCP fp8 tensors (p_fmt / q_fmt: 0 = e4m3,
  // 1 = e5m2) with per-tensor E8M0 dequant exponents in word 2 of their scale sites
  int f8;
  int p_fmt, q_fmt;
  const int* qs_p;    // P (first concat half)
  const int* qs_q;    // Q (first concat half)
  const int* qs_p2;   // second concat halves' sites (null = the first half's)
  const int* qs_q2;
};

// Halo-tile union conv (csrc/halo_conv.hip): the conv_d2s GEMM with a resident 16-column
// weight and 18x18 halo tiles of the input grid staged once per 64-channel chunk.
struct HaloArgs {
  const __bf16* x1;
  const __bf16* x2;
  int C1, C2;          // NHWC channel counts, multiples of 64 (C1 + C2 <= 128)
  int N, H, W;         // input (q) grid
  const __bf16* w;     // union image [16][9][C1 + C2]
  const float* bias;   // [16]
  int act_out;         // tanh (image forward) / none
  int mode;            // d2s mode: 1 image forward, 2 head gradient
  __bf16* out;         // packed [N][2H][2W][8]
  const __bf16* pk_a;
  const __bf16* pk_f;
  float scale;
  const float* wscale; // mode 2: device multiplier of the sign term (dL/dl1; null = 1)
  float* l1_part;      // [blocks] (mode 1)
  const __bf16* zero;
  int tiles_x, tiles_y, ntiles;
};

// Halo-tile packed-image conv (csrc/halo_pk8.hip): 4x4 s2 p1 over [N][Hi][Wi][8] bf16,
// Cout 64 (bias + act) or 128 (optionally the ReLU gate of a dgrad, split output).
struct HaloPk8Args {
  const __bf16* x;
  int Hi, Wi, Ho, Wo;
  const __bf16* w;     // [Cout][16][8] weight image
  const float* bias;   // [Cout] or null
  int Cout, act_out;
  __bf16* y1;          // channels [0, Csplit), ld Csplit
  __bf16* y2;          // channels [Csplit, Cout), ld Cout - Csplit
  int Csplit;
  const __bf16* xb1;   // ReLU-gate inputs (same split), null = no gate
  const __bf16* xb2;
  const __bf16* zero;
  int tiles_x, tiles_y, ntiles;
  uint8_t* q;          // optional fp8 shadow of the (Cout 64, unsplit) output, null = off
  int* q_site;
  int q_fmt;
};

// Halo-tile direct conv for stride-1 KxK convs with few channels (csrc/halo_kxk.hip): input
// C in {8, 16, 32}, Cout <= 32 (multiple of 8), reflect / zero pad, nearest upsample, and
// flip = 1 for a stride-1 transposed conv (taps reversed; the host passes pad = K - 1 - p).
struct HaloKArgs {
  const __bf16* x;     // NHWC [N][H][W][C]
  int C, N, H, W, up, pad, reflect, flip;
  int OH, OW;
  const __bf16* w;     // [Cout][K*K][C] weight image
  const float* bias;   // [Cout] or null
  int Cout, act_out;
  __bf16* y;           // NHWC [N][OH][OW][Cout]  (with a fold: the real grid [N][fold_H][fold_W])
  const __bf16* zero;
  int tiles_x, tiles_y, ntiles;
  // reflect-pad fold of an input gradient on the padded grid (as ConvFwdArgs.fold_buf): interior
  // pixels go straight to y on the real grid, the p-wide frame raw to fold_buf [N][OH][OW]
  // (elementwise.hip fold_band adds it onto the band afterwards); null = plain store
  __bf16* fold_buf;
  int fold_H, fold_W, fold_p;
};

// Halo-tile weight gradient of the same 9x9 stride-1 layers (csrc/halo_wgrad.hip): per-block
// fp32 slabs ws[block][R][K*K*C] (summed by p2p_wgrad_reduce).
struct HaloWArgs {
  const __bf16* gy;    // NHWC [N][OH][OW][R]  (R in {8, 16, 32})
  const __bf16* x;     // NHWC [N][H][W][C]    (C in {16, 32})
  int R, C, N, H, W, up, pad, reflect;
  int OH, OW;
  float* ws;
  const __bf16* zero;
  int tiles_x, tiles_y, ntiles;
};

}  // namespace p2p

extern "C" {
int p2p_halo_wgrad(const p2p::HaloWArgs* a, int KS, int blocks, hipStream_t st);
int p2p_halo_kxk(const p2p::HaloKArgs* a, int KS, int blocks, hipStream_t st);
int p2p_halo_pk8(const p2p::HaloPk8Args* a, int blocks, hipStream_t st);
int p2p_halo_union(const p2p::HaloArgs* a, int relu, int blocks, hipStream_t st);
int p2p_conv_fwd(const p2p::ConvFwdArgs* a, int mode, int bm, int bn, hipStream_t stream);
int p2p_conv_finalize(const p2p::ConvFwdArgs* a, hipStream_t stream);
// global_load_lds pipelined variant (FAST layers, BN in {64, 128}); returns -2 if the
// configuration is not supported so the caller can fall back to p2p_conv_fwd.
int p2p_conv_fwd_glds(const p2p::ConvFwdArgs* a, int mode, int variant, hipStream_t stream);
// stride-2 4x4 pad-1 transposed convs (MODE 1) onto 32x32 / 64x64 grids on the class-shared
// halo kernel (conv_s2t.hip); -2 = geometry not covered
int p2p_conv_s2t(const p2p::ConvFwdArgs* a, hipStream_t stream);
int p2p_conv_wgrad(const p2p::ConvWgradArgs* a, hipStream_t stream);
int p2p_fp8_quant(const void* x, long n, int* site, int use_cur, int fmt, void* q, hipStream_t st);
int p2p_fp8_amax(const void* x, int is_f32, long n, int* site, int slot, hipStream_t st);
int p2p_fp8_roll(int* sites, int nsites, hipStream_t st);
int p2p_fp8_word_zero(int* sites, int nsites, int word, hipStream_t st);
int p2p_fp8_amax_multi(int count, const float* const* x, const long* n, int* const* site, hipStream_t st);
int p2p_fp8_dequant(const void* q, long n, const int* site, int fmt, void* y, hipStream_t st);
int p2p_conv_wgrad_tile_rows(int R);
int p2p_conv_wgrad_tile(const p2p::ConvWgradArgs* a, int* tile_r, int* tile_q);
int p2p_conv_wgrad_f8_tile(const p2p::ConvWgradArgs* a, int* tile_r, int* tile_q);
int p2p_wgrad_reduce(const float* ws, int splits, int R, int KH, int KW, int C, int Rr, int Cr,
                     float* dw, float scale, int accumulate, int flip, hipStream_t stream);
int p2p_col2im(int mode, const void* col, int ldc, int N, int H, int W, int OH, int OW, int KH, int KW,
               int s, int p, int Cv, int Coutp, const float* bias, int act_out, const void* xb,
               int act_bwd, void* y, hipStream_t stream);
int p2p_weight_prep_max();
int p2p_weight_prep_multi(int count, const float* const* w, void* const* out, const int* A, const int* B,
                          const int* T, const int* swap, const int* Xp, const int* Yp,
                          hipStream_t stream);
int p2p_weight_prep(const float* w, int A, int B, int KH, int KW, int swap, int Xp, int Yp,
                    const float* scale, void* out, hipStream_t stream);
}
