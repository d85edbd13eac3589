// Implicit-GEMM convolution / transposed convolution on CDNA4 bf16 MFMA (gfx950).
//
// GEMM view: C[M][N] = A[M][K] * B[K][N] with M = output pixels (NHWC rows), N = output
// channels, K = taps x input channels.  A is gathered on the fly (im2col never exists in
// memory); B is the bf16 weight image [Cout][KH][KW][Cin] so each output channel's K run
// is contiguous (see weight_prep at the end of this file).
//
//  * 256 threads = 4 wave64s arranged WM x WN; each wave owns a (BM/WM) x (BN/WN) block
//    of 16x16 accumulators fed by v_mfma_f32_16x16x32_bf16.
//  * BK = 64: each K-tile is two 32-deep MFMA steps.  Double-buffered LDS with register
//    staging: the next tile's global loads are issued before the current tile's MFMAs and
//    written to the other LDS buffer after them, one barrier per K-tile.
//  * LDS tiles are [rows][64] bf16 (128-B rows) with the 16-B chunk index XOR-swizzled
//    by (row>>1)&7 so the 16 rows a ds_read_b128 lane-group touches land on 16 distinct
//    16-B slots (conflict-free fragment reads and row writes).
//  * Loader cost is what bounds an implicit GEMM on CDNA4 (one wave64 VALU op = 2 cycles
//    of a SIMD that also issues the MFMAs), so it is kept to ~10 VALU ops per 16-B chunk:
//      - FAST path (every channel group a multiple of 64, i.e. all U-Net / PatchGAN
//        layers but the first): a 64-deep K tile never straddles a tap, so (tap, ci, src)
//        are wave-uniform scalars per tile; each thread keeps its rows' (image base, y0,
//        x0) and only adds the tap offset + one bounds test.
//      - general path (C = 8 / 16 / 24 ...: packed image inputs): per-thread tap split by
//        magic-number division, no hardware divide anywhere.
//      - the input activation is folded in as a packed int16 max for ReLU (4 ops / 16 B);
//        LeakyReLU is stored pre-applied by its producer (norm / epilogue) instead.
//  * Folded into the gather: zero / reflection padding, nearest upsample (src = dst >> 1)
//    and a virtual channel concat of two tensors (the U-Net skip) -- none materialised.
//  * CONVT (MODE 1) = sub-pixel decomposition: blockIdx.z selects the output parity class
//    (ry, rx); only the ceil(K/s)^2 taps that hit the class are iterated, so a 4x4 s2
//    transposed conv costs 4 taps per output pixel instead of 16 with 3/4 zeros.  MODE 1
//    also serves conv dgrad (dY * W^T) and MODE 0 serves convT dgrad.
//  * Epilogue: bias + output activation in registers, the tile staged through LDS as
//    bf16 (fits inside the 64 KB pipeline buffers: 2 workgroups / CU), then 16-B stores
//    with the optional act'(x) multiply of dgrad and a channel split into two tensors
//    (gradient of a virtual concat).  Split-K (tiny-M bottleneck layers) accumulates
//    fp32 atomics straight from the accumulators, finished by conv_finalize_kernel.
//  * Workgroup ids are remapped XCD-aware so the n-tiles of one m-tile share an L2.
#include "conv_dev.h"

namespace p2p {

template <int BM, int BN>
struct FwdSmem {
  static constexpr int pipe = 2 * (BM + BN) * BK * 2;
  static constexpr int epi = BM * (BN + 8) * 2 + 2 * 256 * 4;  // + stats scratch
  static constexpr int bytes = pipe > epi ? pipe : epi;
};

template <int BM, int BN, int WM, int WN, int MODE, bool FAST>
__global__ void __launch_bounds__(256) conv_fwd_kernel(ConvFwdArgs a) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  constexpr int AROWS = BM / 32;                      // A rows loaded per thread
  constexpr int BROWS = BN >= 32 ? BN / 32 : 1;       // B rows loaded per thread
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* As = reinterpret_cast<bf16*>(smem);
  bf16* Bs = As + 2 * BM * BK;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;

  const int cls = blockIdx.z / a.splits;
  const int split = blockIdx.z % a.splits;
  const ClassGeom g = class_geom<MODE>(a, cls);
  const int ntiles = (a.Cout + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / ntiles, nt = bid % ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  if (m0 >= g.Mc) return;

  const int ktiles = (g.Kc + BK - 1) / BK;
  const int kps = (ktiles + a.splits - 1) / a.splits;
  const int kt0 = split * kps;
  const int kt1 = min(ktiles, kt0 + kps);
  if (kt0 >= kt1 && a.splits > 1) return;

  const bf16* __restrict__ x1 = static_cast<const bf16*>(a.x1);
  const bf16* __restrict__ x2 = static_cast<const bf16*>(a.x2);
  const bf16* __restrict__ w = static_cast<const bf16*>(a.w);
  const int C = a.C, C1 = a.C1, C2 = a.C2;
  const int kc = tid & 7;  // this thread's 16-B chunk within a 64-wide K tile
  const int ush = a.up == 2 ? 1 : 0;
  const int Hu = a.H << ush, Wu = a.W << ush;

  // ---- per-thread A rows (fixed over the K loop): image base pixel, y0, x0
  int r_img[AROWS], r_y[AROWS], r_x[AROWS];
  const int HWq = g.Hq * g.Wq;
  const FastDiv fd_hwq = make_fastdiv((uint32_t)HWq), fd_wq = make_fastdiv((uint32_t)g.Wq);
#pragma unroll
  for (int i = 0; i < AROWS; ++i) {
    const int m = m0 + (tid >> 3) + 32 * i;
    const int mm = m < g.Mc ? m : 0;
    const int n = (int)fdiv((uint32_t)mm, fd_hwq);
    const int r = mm - n * HWq;
    const int qy = (int)fdiv((uint32_t)r, fd_wq);
    const int qx = r - qy * g.Wq;
    r_img[i] = n * a.H * a.W;
    if (MODE == 0) {
      r_y[i] = qy * a.stride - a.pad;
      r_x[i] = qx * a.stride - a.pad;
    } else {
      r_y[i] = qy + g.dy;
      r_x[i] = qx + g.dx;
    }
    if (m >= g.Mc) r_y[i] = -(1 << 28);  // forces the bounds test to fail (zero row)
  }
  const FastDiv fd_c = make_fastdiv((uint32_t)C), fd_ti = make_fastdiv((uint32_t)g.Ti);
  const long wrow = (MODE == 0) ? (long)g.Kc : (long)a.KH * a.KW * C;  // weight row stride

  u32x4 ra[AROWS], rb[BROWS];

  // gather one 16-B chunk of row i at tap (t_y, t_x) from src + channel offset cio
  auto gather = [&](int i, int t_y, int t_x, const bf16* src, int cs, int cio) -> u32x4 {
    u32x4 v = zero_u32x4();
    int iy, ix;
    bool inb;
    if (MODE == 0) {
      int uy = r_y[i] + t_y, ux = r_x[i] + t_x;
      if (a.reflect && r_y[i] > -(1 << 27)) {
        uy = reflect_idx(uy, Hu);
        ux = reflect_idx(ux, Wu);
      }
      inb = (unsigned)uy < (unsigned)Hu && (unsigned)ux < (unsigned)Wu;
      iy = uy >> ush;
      ix = ux >> ush;
    } else {
      iy = r_y[i] - t_y;
      ix = r_x[i] - t_x;
      inb = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
    }
    if (inb) {
      const int pix = r_img[i] + iy * a.W + ix;
      v = *reinterpret_cast<const u32x4*>(src + (long)pix * cs + cio);
      v = act_chunk(v, a.act_in);
    }
    return v;
  };

  auto load_tile = [&](int kt) {
    const int k0 = kt * BK;
    if constexpr (FAST) {
      // wave-uniform: the whole 64-deep tile is one tap and one source tensor
      const int tap = (int)fdiv((uint32_t)k0, fd_c);
      const int ci0 = k0 - tap * C;
      const int t_y = (int)fdiv((uint32_t)tap, fd_ti);
      const int t_x = tap - t_y * g.Ti;
      const bool s1 = ci0 < C1;
      const bf16* src = s1 ? x1 : x2;
      const int cs = s1 ? C1 : C2;
      const int cio = (s1 ? ci0 : ci0 - C1) + kc * 8;
#pragma unroll
      for (int i = 0; i < AROWS; ++i) ra[i] = gather(i, t_y, t_x, src, cs, cio);
      long woff;
      if (MODE == 0) {
        woff = k0 + kc * 8;
      } else {
        const int ky = g.ky0 + a.stride * t_y, kx = g.kx0 + a.stride * t_x;
        woff = (long)(ky * a.KW + kx) * C + ci0 + kc * 8;
      }
#pragma unroll
      for (int i = 0; i < BROWS; ++i) {
        const int row = (tid >> 3) + 32 * i;
        const int co = n0 + row;
        u32x4 v = zero_u32x4();
        if (row < BN && co < a.Cout) v = *reinterpret_cast<const u32x4*>(w + co * wrow + woff);
        rb[i] = v;
      }
    } else {
      const int k = k0 + kc * 8;
      const bool kok = k < g.Kc;
      int tap = 0, ci = 0, t_y = 0, t_x = 0;
      if (kok) {
        tap = (int)fdiv((uint32_t)k, fd_c);
        ci = k - tap * C;
        t_y = (int)fdiv((uint32_t)tap, fd_ti);
        t_x = tap - t_y * g.Ti;
      }
      const bool s1 = ci < C1;
      const bf16* src = s1 ? x1 : x2;
      const int cs = s1 ? C1 : C2;
      const int cio = s1 ? ci : ci - C1;
#pragma unroll
      for (int i = 0; i < AROWS; ++i) ra[i] = kok ? gather(i, t_y, t_x, src, cs, cio) : zero_u32x4();
      long woff;
      if (MODE == 0) {
        woff = k;
      } else {
        const int ky = g.ky0 + a.stride * t_y, kx = g.kx0 + a.stride * t_x;
        woff = (long)(ky * a.KW + kx) * C + ci;
      }
#pragma unroll
      for (int i = 0; i < BROWS; ++i) {
        const int row = (tid >> 3) + 32 * i;
        const int co = n0 + row;
        u32x4 v = zero_u32x4();
        if (kok && row < BN && co < a.Cout) v = *reinterpret_cast<const u32x4*>(w + co * wrow + woff);
        rb[i] = v;
      }
    }
  };

  auto store_tile = [&](int buf) {
    bf16* A = As + buf * BM * BK;
    bf16* B = Bs + buf * BN * BK;
#pragma unroll
    for (int i = 0; i < AROWS; ++i) {
      const int row = (tid >> 3) + 32 * i;
      *reinterpret_cast<u32x4*>(A + swz(row, kc)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BROWS; ++i) {
      const int row = (tid >> 3) + 32 * i;
      if (row < BN) *reinterpret_cast<u32x4*>(B + swz(row, kc)) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kt0 < kt1) {
    load_tile(kt0);
    store_tile(0);
    __syncthreads();
  }
  int buf = 0;
  for (int kt = kt0; kt < kt1; ++kt) {
    const bool more = kt + 1 < kt1;
    if (more) load_tile(kt + 1);
    const bf16* A = As + buf * BM * BK;
    const bf16* B = Bs + buf * BN * BK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + (lane >> 4);
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * TM * 16 + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(A + swz(row, chunk));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * TN * 16 + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(B + swz(row, chunk));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) store_tile(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  conv_epilogue<BM, BN, WM, WN, MODE, 256>(a, g, acc, m0, n0, smem, fd_hwq, fd_wq);
}

// split-K finish: ws [P][Cout] fp32 -> bias / act / act' / channel split -> bf16
__global__ void __launch_bounds__(256) conv_finalize_kernel(ConvFwdArgs a, long P) {
  const long nchunks = P * (a.Cout / 8);
  for (long c = blockIdx.x * 256L + threadIdx.x; c < nchunks; c += (long)gridDim.x * 256) {
    const long pix = c / (a.Cout / 8);
    const int co = (int)(c - pix * (a.Cout / 8)) * 8;
    f32x4 v0 = *reinterpret_cast<const f32x4*>(a.ws + pix * a.Cout + co);
    f32x4 v1 = *reinterpret_cast<const f32x4*>(a.ws + pix * a.Cout + co + 4);
    if (a.det) {  // per-split slabs, summed in split order
      for (int s = 1; s < a.splits; ++s) {
        const float* w = a.ws + (long)s * P * a.Cout + pix * a.Cout + co;
        v0 += *reinterpret_cast<const f32x4*>(w);
        v1 += *reinterpret_cast<const f32x4*>(w + 4);
      }
    }
    float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    if (a.alpha) {
      const float al = a.alpha[0];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= al;
    }
    if (a.bias) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += a.bias[co + j];
    }
    if (a.act_out) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = act_fwd(v[j], a.act_out);
    }
    const bool first = co < a.Csplit;
    const int ld = first ? a.Csplit : a.Cout - a.Csplit;
    const int cof = first ? co : co - a.Csplit;
    const bf16* xb = static_cast<const bf16*>(first ? a.xb1 : a.xb2);
    if (a.act_bwd && xb) {
      bf16x8 xv = *reinterpret_cast<const bf16x8*>(xb + pix * ld + cof);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= act_grad_from_input((float)xv[j], a.act_bwd);
    }
    if (a.res1 && first) {
      const bf16x8 rv = *reinterpret_cast<const bf16x8*>(static_cast<const bf16*>(a.res1) + pix * ld + cof);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (float)(bf16)v[j] + (float)rv[j];
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
    bf16* y = static_cast<bf16*>(first ? a.y1 : a.y2);
    *reinterpret_cast<bf16x8*>(y + pix * ld + cof) = o;
  }
}

template <int BM, int BN, int WM, int WN, int MODE, bool FAST>
static int launch_fwd(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int smem = FwdSmem<BM, BN>::bytes;
  static std::atomic<uint64_t> attr_mask{0};
  smem_attr_once(reinterpret_cast<const void*>(&conv_fwd_kernel<BM, BN, WM, WN, MODE, FAST>), smem, attr_mask);
  int classes = MODE == 0 ? 1 : a.stride * a.stride;
  long mmax = 0;
  for (int c = 0; c < classes; ++c) {
    long hq, wq;
    if (MODE == 0) {
      hq = a.OH;
      wq = a.OW;
    } else {
      int ry = c / a.stride, rx = c % a.stride;
      hq = a.OH > ry ? (a.OH - ry + a.stride - 1) / a.stride : 0;
      wq = a.OW > rx ? (a.OW - rx + a.stride - 1) / a.stride : 0;
    }
    long mc = (long)a.N * hq * wq;
    mmax = mc > mmax ? mc : mmax;
  }
  const long mtiles = (mmax + BM - 1) / BM;
  const long ntiles = (a.Cout + BN - 1) / BN;
  dim3 grid((unsigned)(mtiles * ntiles), 1, (unsigned)(classes * a.splits));
  hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, WM, WN, MODE, FAST>), grid, dim3(256), smem, st, a);
  return (int)hipGetLastError();
}

template <int MODE, bool FAST>
static int dispatch_fwd2(const ConvFwdArgs& a, int bm, int bn, hipStream_t st) {
  if (bm == 128 && bn == 128) return launch_fwd<128, 128, 2, 2, MODE, FAST>(a, st);
  if (bm == 128 && bn == 64) return launch_fwd<128, 64, 2, 2, MODE, FAST>(a, st);
  if (bm == 64 && bn == 128) return launch_fwd<64, 128, 2, 2, MODE, FAST>(a, st);
  if (bm == 64 && bn == 64) return launch_fwd<64, 64, 2, 2, MODE, FAST>(a, st);
  if (bm == 256 && bn == 32) return launch_fwd<256, 32, 4, 1, MODE, FAST>(a, st);
  if (bm == 256 && bn == 16) return launch_fwd<256, 16, 4, 1, MODE, FAST>(a, st);
  if (bm == 64 && bn == 16) return launch_fwd<64, 16, 4, 1, MODE, FAST>(a, st);
  return -1;
}

template <int MODE>
static int dispatch_fwd(const ConvFwdArgs& a, int bm, int bn, hipStream_t st) {
  const bool fast = (a.C1 % BK == 0) && (a.C2 % BK == 0);
  return fast ? dispatch_fwd2<MODE, true>(a, bm, bn, st) : dispatch_fwd2<MODE, false>(a, bm, bn, st);
}

}  // namespace p2p

extern "C" int p2p_conv_fwd(const p2p::ConvFwdArgs* a, int mode, int bm, int bn, hipStream_t st) {
  return mode == 0 ? p2p::dispatch_fwd<0>(*a, bm, bn, st) : p2p::dispatch_fwd<1>(*a, bm, bn, st);
}


// ---------------------------------------------------------------------------------------
// Weight preparation: fp32 master weight [A][B][KH][KW] (PyTorch Conv2d: [Cout][Cin][..],
// ConvTranspose2d: [Cin][Cout][..]) -> bf16 GEMM operand [X][KH][KW][Yp] with X = A, Y = B
// (swap = 0) or X = B, Y = A (swap = 1), zero-padded to Xp rows / Yp channels, optionally
// scaled by a device scalar (1/sigma of spectral norm).  The four operand images:
//   conv fwd   swap 0    conv dgrad (CONVT mode on dY)   swap 1
//   convT fwd  swap 1    convT dgrad (CONV mode on dY)   swap 0
namespace p2p {
__global__ void __launch_bounds__(256) weight_prep_kernel(const float* __restrict__ w, int A, int B,
                                                          int KH, int KW, int swap, int Xp, int Yp,
                                                          const float* __restrict__ scale,
                                                          bf16* __restrict__ out) {
  const int T = KH * KW;
  const long total = (long)Xp * T * Yp;
  const float s = scale ? scale[0] : 1.f;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int y = (int)(e % Yp);
    const long r = e / Yp;
    const int t = (int)(r % T);
    const int x = (int)(r / T);
    const int a = swap ? y : x, b = swap ? x : y;
    float v = 0.f;
    if (a < A && b < B) v = w[((long)a * B + b) * T + t] * s;
    out[e] = (bf16)v;
  }
}
}  // namespace p2p

extern "C" int p2p_weight_prep(const float* w, int A, int B, int KH, int KW, int swap, int Xp, int Yp,
                               const float* scale, void* out, hipStream_t st) {
  const long total = (long)Xp * KH * KW * Yp;
  long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(p2p::weight_prep_kernel, dim3((unsigned)blocks), dim3(256), 0, st, w, A, B, KH, KW,
                     swap, Xp, Yp, scale, static_cast<p2p::bf16*>(out));
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// col2im for the tiny-Cout "col" path (U-Net head, PatchGAN logits, first-layer dgrad):
// the dense GEMM col[i][t*Cv + co] = sum_ci x[i][ci] w[co][t][ci] ran over the INPUT
// pixels (N = taps x Cv, no MFMA lanes wasted on padded output channels); here every
// output pixel gathers its taps:
//   MODE 0 (conv):  input i = o*s - p + t            (if inside the image)
//   MODE 1 (convT): input i = (o + p - t) / s        (if divisible and inside)
// then bias, output activation, optional act'(xb) (dgrad) and zero padded channels.
namespace p2p {
// one thread per output pixel; only the taps that hit it are visited (MODE 1: the
// ceil(K/s)^2 taps of its parity class, found arithmetically -- no per-tap divisibility
// loop).  Each tap's values are CVP (4 / 8 / 16, >= Cv, zero-padded by the GEMM) contiguous
// bf16 in col, read as one 8 / 16 / 32-byte vector per tap.
__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// ACT >= 0: the output activation as a compile-time code (no per-element switch); -1: runtime
template <int MODE, int CVP, int ACT>
__global__ void __launch_bounds__(256) col2im_kernel(const bf16* __restrict__ col, int ldc, int N, int H,
                                                     int W, int OH, int OW, int KH, int KW, int s, int p,
                                                     int Cv, int Coutp, const float* __restrict__ bias,
                                                     int act_out, const bf16* __restrict__ xb, int act_bwd,
                                                     bf16* __restrict__ y) {
  constexpr int NW = CVP / 2;  // 32-bit words per tap
  const long total = (long)N * OH * OW;
  for (long o = blockIdx.x * 256L + threadIdx.x; o < total; o += (long)gridDim.x * 256) {
    const int ox = (int)(o % OW);
    const long t1 = o / OW;
    const int oy = (int)(t1 % OH);
    const int n = (int)(t1 / OH);
    float acc[CVP];
#pragma unroll
    for (int j = 0; j < CVP; ++j) acc[j] = 0.f;
    int ky = 0, kx0 = 0, kstep = 1;
    if (MODE == 1) {
      ky = (oy + p) % s;
      kx0 = (ox + p) % s;
      kstep = s;
    }
    for (; ky < KH; ky += kstep) {
      const int iy = MODE == 0 ? oy * s - p + ky : (oy + p - ky) / s;
      if ((unsigned)iy >= (unsigned)H) continue;
      for (int kx = kx0; kx < KW; kx += kstep) {
        const int ix = MODE == 0 ? ox * s - p + kx : (ox + p - kx) / s;
        if ((unsigned)ix >= (unsigned)W) continue;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(
            col + ((long)(n * H + iy) * W + ix) * ldc + (ky * KW + kx) * CVP);
        if constexpr (CVP == 1) {
          acc[0] += (float)*reinterpret_cast<const bf16*>(src);
          continue;
        }
        uint32_t wv[NW > 0 ? NW : 1];
        if constexpr (NW == 1) {
          wv[0] = src[0];
        } else if constexpr (NW == 2) {
          const uint2 v = *reinterpret_cast<const uint2*>(src);
          wv[0] = v.x;
          wv[1] = v.y;
        } else {
#pragma unroll
          for (int q = 0; q < NW / 4; ++q) {
            const uint4 v = *reinterpret_cast<const uint4*>(src + 4 * q);
            wv[4 * q] = v.x;
            wv[4 * q + 1] = v.y;
            wv[4 * q + 2] = v.z;
            wv[4 * q + 3] = v.w;
          }
        }
#pragma unroll
        for (int q = 0; q < NW; ++q) {
          acc[2 * q] += bf_lo(wv[q]);
          acc[2 * q + 1] += bf_hi(wv[q]);
        }
      }
    }
    for (int g0 = 0; g0 < Coutp; g0 += 8) {
      uint4 xv = make_uint4(0, 0, 0, 0);
      if (act_bwd) xv = *reinterpret_cast<const uint4*>(xb + o * Coutp + g0);
      const uint32_t xw[4] = {xv.x, xv.y, xv.z, xv.w};
      uint32_t ow[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v2[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int co = g0 + 2 * q + h;
          float v = 0.f;
#pragma unroll
          for (int k = 0; k < CVP; ++k)
            if (k == co && co < Cv) v = act_fwd(acc[k] + (bias ? bias[co] : 0.f), ACT >= 0 ? ACT : act_out);
          if (act_bwd) v *= act_grad_from_input(h ? bf_hi(xw[q]) : bf_lo(xw[q]), act_bwd);
          v2[h] = v;
        }
        const uint32_t lo = __builtin_bit_cast(uint16_t, (bf16)v2[0]);
        const uint32_t hi = __builtin_bit_cast(uint16_t, (bf16)v2[1]);
        ow[q] = lo | (hi << 16);
      }
      *reinterpret_cast<uint4*>(y + o * Coutp + g0) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
    }
  }
}
}  // namespace p2p

extern "C" int p2p_col2im(int mode, const void* col, int ldc, int N, int H, int W, int OH, int OW, int KH,
                          int KW, int s, int p, int Cv, int Coutp, const float* bias, int act_out,
                          const void* xb, int act_bwd, void* y, hipStream_t st) {
  const long total = (long)N * OH * OW;
  long blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  if (blocks < 1) blocks = 1;
  const p2p::bf16* c = static_cast<const p2p::bf16*>(col);
  const p2p::bf16* x = static_cast<const p2p::bf16*>(xb);
  p2p::bf16* o = static_cast<p2p::bf16*>(y);
  const int cvp = Cv <= 2 ? Cv : (Cv <= 4 ? 4 : (Cv <= 8 ? 8 : 16));
  if (Cv > 16 || Cv < 1 || ldc % cvp) return -1;
#define P2P_COL2IM_A(M, V, A)                                                                            \
  hipLaunchKernelGGL((p2p::col2im_kernel<M, V, A>), dim3((unsigned)blocks), dim3(256), 0, st, c, ldc, N, H, W, \
                     OH, OW, KH, KW, s, p, Cv, Coutp, bias, act_out, x, act_bwd, o)
#define P2P_COL2IM(M, V)                                           \
  do {                                                             \
    if (act_out == p2p::ACT_NONE) P2P_COL2IM_A(M, V, p2p::ACT_NONE); \
    else if (act_out == p2p::ACT_TANH) P2P_COL2IM_A(M, V, p2p::ACT_TANH); \
    else P2P_COL2IM_A(M, V, -1);                                   \
  } while (0)
  if (mode == 0) {
    if (cvp == 1) P2P_COL2IM(0, 1);
    else if (cvp == 2) P2P_COL2IM(0, 2);
    else if (cvp == 4) P2P_COL2IM(0, 4);
    else if (cvp == 8) P2P_COL2IM(0, 8);
    else P2P_COL2IM(0, 16);
  } else {
    if (cvp == 1) P2P_COL2IM(1, 1);
    else if (cvp == 2) P2P_COL2IM(1, 2);
    else if (cvp == 4) P2P_COL2IM(1, 4);
    else if (cvp == 8) P2P_COL2IM(1, 8);
    else P2P_COL2IM(1, 16);
  }
#undef P2P_COL2IM
#undef P2P_COL2IM_A
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Multi-tensor weight preparation: every conv of a network in ONE launch (blockIdx.y =
// tensor, descriptors in the kernel-argument block), instead of one small launch per
// layout per layer.
namespace p2p {
constexpr int WP_MAX = 24;
struct WPrepList {
  const float* w[WP_MAX];
  bf16* out[WP_MAX];
  int A[WP_MAX], B[WP_MAX], T[WP_MAX], swap[WP_MAX], Xp[WP_MAX], Yp[WP_MAX];
  int count;
};

// One thread per (x, y-pair) of the image: it reads the two source rows w[a][b][0..T)
// (contiguous fp32 runs) and writes the T taps as packed bf16 pairs, so for every tap a
// wave stores 256 contiguous bytes (the element-per-thread form re-read each 64-B source
// line T times at stride T and issued 2-byte stores).
__global__ void __launch_bounds__(256) weight_prep_multi_kernel(WPrepList L) {
  const int t = blockIdx.y;
  const float* __restrict__ w = L.w[t];
  bf16* __restrict__ out = L.out[t];
  const int A = L.A[t], B = L.B[t], T = L.T[t], swap = L.swap[t], Yp = L.Yp[t];
  if (Yp & 1) {
    const long total = (long)L.Xp[t] * T * Yp;
    for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
      const int yv = (int)(e % Yp);
      const long r = e / Yp;
      const int tap = (int)(r % T);
      const int xv = (int)(r / T);
      const int a = swap ? yv : xv, b = swap ? xv : yv;
      float v = 0.f;
      if (a < A && b < B) v = w[((long)a * B + b) * T + tap];
      out[e] = (bf16)v;
    }
    return;
  }
  const int Yh = Yp >> 1;
  const long pairs = (long)L.Xp[t] * Yh;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < pairs; e += (long)gridDim.x * 256) {
    const int y0 = (int)(e % Yh) * 2;
    const int xv = (int)(e / Yh);
    const int a0 = swap ? y0 : xv, b0 = swap ? xv : y0;
    const int a1 = swap ? y0 + 1 : xv, b1 = swap ? xv : y0 + 1;
    const bool ok0 = a0 < A && b0 < B, ok1 = a1 < A && b1 < B;
    const float* r0 = w + ((long)a0 * B + b0) * T;
    const float* r1 = w + ((long)a1 * B + b1) * T;
    uint32_t* o = reinterpret_cast<uint32_t*>(out + (long)xv * T * Yp + y0);
    if (T == 16) {  // 4x4 kernels: two 64-B rows as 16-B vector loads
      float4 f0[4], f1[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f0[q] = ok0 ? reinterpret_cast<const float4*>(r0)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
        f1[q] = ok1 ? reinterpret_cast<const float4*>(r1)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      const float* a0 = reinterpret_cast<const float*>(f0);
      const float* a1 = reinterpret_cast<const float*>(f1);
#pragma unroll
      for (int tap = 0; tap < 16; ++tap) {
        const uint32_t lo = __builtin_bit_cast(uint16_t, (bf16)a0[tap]);
        const uint32_t hi = __builtin_bit_cast(uint16_t, (bf16)a1[tap]);
        o[(long)tap * Yh] = lo | (hi << 16);
      }
      continue;
    }
    for (int tap = 0; tap < T; ++tap) {
      const float v0 = ok0 ? r0[tap] : 0.f;
      const float v1 = ok1 ? r1[tap] : 0.f;
      const uint32_t lo = __builtin_bit_cast(uint16_t, (bf16)v0);
      const uint32_t hi = __builtin_bit_cast(uint16_t, (bf16)v1);
      o[(long)tap * Yh] = lo | (hi << 16);
    }
  }
}
}  // namespace p2p

extern "C" int p2p_conv_finalize(const p2p::ConvFwdArgs* a, hipStream_t st) {
  const long P = (long)a->N * a->OH * a->OW;
  const long nchunks = P * (a->Cout / 8);
  long blocks = (nchunks + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(p2p::conv_finalize_kernel, dim3((unsigned)blocks), dim3(256), 0, st, *a, P);
  return (int)hipGetLastError();
}

extern "C" int p2p_weight_prep_max() { return p2p::WP_MAX; }

// ---------------------------------------------------------------------------------------
// Both GEMM images of a weight in ONE pass (T = KH*KW <= 16): out0 [Xa][T][Xb] (w[a][b][t])
// and out1 [Xb][T][Xa] (w[b-major]) with Xa >= A, Xb >= B zero-padded.  A 32(a) x 32(b) x T
// block is read once with coalesced runs (each a-row's b x t slab is contiguous), staged
// as bf16 in LDS, and written out as 4-byte pairs along the contiguous axis of each image
// -- the transposed image no longer gathers across 64 KB-strided source rows.
namespace p2p {
constexpr int WPP_MAX = 24;
struct WPairList {
  const float* w[WPP_MAX];
  void* out0[WPP_MAX];
  void* out1[WPP_MAX];
  int* site[WPP_MAX];  // F8: per-tensor scale site (amax in [0], e8m0 published to [2])
  int A[WPP_MAX], B[WPP_MAX], T[WPP_MAX], Xa[WPP_MAX], Xb[WPP_MAX];
};

// element pair (lo at the lower address) -> bf16x2 (4 B) or e4m3x2 (2 B) store
template <bool F8>
__device__ __forceinline__ void store_pair(void* base, long idx, bf16 lo, bf16 hi, float qsc) {
  if constexpr (F8) {
    const float fm = 448.f;
    const float a = fminf(fmaxf((float)lo * qsc, -fm), fm), b = fminf(fmaxf((float)hi * qsc, -fm), fm);
    const int pk = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    *reinterpret_cast<uint16_t*>(static_cast<uint8_t*>(base) + idx) = (uint16_t)(pk & 0xffff);
  } else {
    const uint32_t l = __builtin_bit_cast(uint16_t, lo), h = __builtin_bit_cast(uint16_t, hi);
    *reinterpret_cast<uint32_t*>(static_cast<bf16*>(base) + idx) = l | (h << 16);
  }
}

// TT = 16: the 4x4-kernel fast path (all index math shifts, float4 source loads);
// TT = 0: any T <= 16 with runtime division.  F8: e4m3 images with the current-scaling
// power-of-two scale of the tensor's site (fp8 conv path, csrc/fp8.hip).
template <int TT, bool F8>
__global__ void __launch_bounds__(256) weight_prep_pair_kernel(WPairList L) {
  constexpr int TA = 32, TB = 32, TMAX = 16, TS = TMAX + 2;  // +2: breaks the 32-B row stride
  __shared__ bf16 tile[TA][TB][TS];
  const int k = blockIdx.y;
  const float* __restrict__ w = L.w[k];
  const int A = L.A[k], B = L.B[k], Xa = L.Xa[k], Xb = L.Xb[k];
  const int T = TT ? TT : L.T[k];
  if (TT && L.T[k] != TT) return;
  if (!TT && L.T[k] == 16) return;
  const int ta = (Xa + TA - 1) / TA, tb = (Xb + TB - 1) / TB;
  const int tid = threadIdx.x;
  float qsc = 0.f;
  if constexpr (F8) {
    const int e = fp8_exp(__int_as_float(L.site[k][0]), 0);
    if (blockIdx.x == 0 && tid == 0) L.site[k][2] = 127 - e;
    qsc = ldexpf(1.f, e);
  }
  for (int tile_id = blockIdx.x; tile_id < ta * tb; tile_id += gridDim.x) {
    const int a0 = (tile_id / tb) * TA, b0 = (tile_id % tb) * TB;
    if constexpr (TT == 16) {
      // per a-row the [b0, b0+32) x 16 run is 128 float4s
      for (int idx = tid; idx < TA * 128; idx += 256) {
        const int al = idx >> 7, bl = (idx >> 2) & 31, t4 = (idx & 3) * 4;
        const int a = a0 + al, b = b0 + bl;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (a < A && b < B) v = *reinterpret_cast<const float4*>(w + ((long)a * B + b) * 16 + t4);
        bf16* d = &tile[al][bl][t4];
        d[0] = (bf16)v.x;
        d[1] = (bf16)v.y;
        d[2] = (bf16)v.z;
        d[3] = (bf16)v.w;
      }
    } else {
      const int run = TB * T;
      for (int idx = tid; idx < TA * run; idx += 256) {
        const int al = idx / run, r = idx - al * run;
        const int bl = r / T, t = r - bl * T;
        const int a = a0 + al, b = b0 + bl;
        float v = 0.f;
        if (a < A && b < B) v = w[((long)a * B + b) * T + t];
        tile[al][bl][t] = (bf16)v;
      }
    }
    __syncthreads();
    // out0[a][t][b]: bf16 pairs along b
    const int n0 = TA * T * (TB / 2);
    for (int idx = tid; idx < n0; idx += 256) {
      int al, t, bl;
      if constexpr (TT == 16) {
        al = idx >> 8;
        t = (idx >> 4) & 15;
        bl = (idx & 15) * 2;
      } else {
        al = idx / (T * (TB / 2));
        const int r = idx - al * (T * (TB / 2));
        t = r / (TB / 2);
        bl = (r - t * (TB / 2)) * 2;
      }
      const int a = a0 + al, b = b0 + bl;
      if (a < Xa && b < Xb) store_pair<F8>(L.out0[k], ((long)a * T + t) * Xb + b, tile[al][bl][t], tile[al][bl + 1][t], qsc);
    }
    // out1[b][t][a]: bf16 pairs along a
    for (int idx = tid; idx < n0; idx += 256) {
      int bl, t, al;
      if constexpr (TT == 16) {
        bl = idx >> 8;
        t = (idx >> 4) & 15;
        al = (idx & 15) * 2;
      } else {
        bl = idx / (T * (TA / 2));
        const int r = idx - bl * (T * (TA / 2));
        t = r / (TA / 2);
        al = (r - t * (TA / 2)) * 2;
      }
      const int a = a0 + al, b = b0 + bl;
      if (b < Xb && a < Xa) store_pair<F8>(L.out1[k], ((long)b * T + t) * Xa + a, tile[al][bl][t], tile[al + 1][bl][t], qsc);
    }
    __syncthreads();
  }
}
}  // namespace p2p

extern "C" int p2p_weight_prep_pairs(int count, const float* const* w, void* const* out0, void* const* out1,
                                     const int* A, const int* B, const int* T, const int* Xa, const int* Xb,
                                     int* const* site, hipStream_t st) {
  using namespace p2p;
  if (count <= 0) return 0;
  if (count > WPP_MAX) return -1;
  WPairList L;
  int maxt = 1;
  const bool f8 = site != nullptr;
  for (int i = 0; i < count; ++i) {
    if (T[i] > 16 || (Xa[i] & 1) || (Xb[i] & 1)) return -1;
    L.w[i] = w[i];
    L.out0[i] = out0[i];
    L.out1[i] = out1[i];
    L.site[i] = f8 ? site[i] : nullptr;
    L.A[i] = A[i];
    L.B[i] = B[i];
    L.T[i] = T[i];
    L.Xa[i] = Xa[i];
    L.Xb[i] = Xb[i];
    const int tiles = ((Xa[i] + 31) / 32) * ((Xb[i] + 31) / 32);
    maxt = tiles > maxt ? tiles : maxt;
  }
  bool any16 = false, other = false;
  for (int i = 0; i < count; ++i) (T[i] == 16 ? any16 : other) = true;
  const dim3 grid((unsigned)(maxt < 2048 ? maxt : 2048), count);
  if (f8) {
    if (any16) hipLaunchKernelGGL((weight_prep_pair_kernel<16, true>), grid, dim3(256), 0, st, L);
    if (other) hipLaunchKernelGGL((weight_prep_pair_kernel<0, true>), grid, dim3(256), 0, st, L);
  } else {
    if (any16) hipLaunchKernelGGL((weight_prep_pair_kernel<16, false>), grid, dim3(256), 0, st, L);
    if (other) hipLaunchKernelGGL((weight_prep_pair_kernel<0, false>), grid, dim3(256), 0, st, L);
  }
  return (int)hipGetLastError();
}

// descriptors: w[i] fp32 [A][B][T], out[i] bf16 [Xp][T][Yp]
extern "C" int p2p_weight_prep_multi(int count, const float* const* w, void* const* out, const int* A,
                                     const int* B, const int* T, const int* swap, const int* Xp,
                                     const int* Yp, hipStream_t st) {
  using namespace p2p;
  if (count <= 0) return 0;
  if (count > WP_MAX) return -1;
  WPrepList L;
  L.count = count;
  long maxel = 0;
  for (int i = 0; i < count; ++i) {
    L.w[i] = w[i];
    L.out[i] = static_cast<bf16*>(out[i]);
    L.A[i] = A[i];
    L.B[i] = B[i];
    L.T[i] = T[i];
    L.swap[i] = swap[i];
    L.Xp[i] = Xp[i];
    L.Yp[i] = Yp[i];
    const long el = (Yp[i] & 1) ? (long)Xp[i] * T[i] * Yp[i] : (long)Xp[i] * (Yp[i] / 2);
    maxel = el > maxel ? el : maxel;
  }
  long bx = (maxel + 255) / 256;
  if (bx > 1024) bx = 1024;
  hipLaunchKernelGGL(weight_prep_multi_kernel, dim3((unsigned)bx, count), dim3(256), 0, st, L);
  return (int)hipGetLastError();
}
