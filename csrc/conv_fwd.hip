// Implicit-GEMM convolution / transposed convolution on CDNA4 bf16 MFMA (gfx950).
//
// GEMM view: C[M][N] = A[M][K] * B[K][N] with M = output pixels (NHWC rows), N = output
// channels, K = taps x input channels.  A is gathered on the fly (im2col never exists in
// memory); B is the bf16 weight stored [Cout][KH][KW][Cin] so each output channel's K
// run is contiguous.
//
//  * 256 threads = 4 wave64s arranged WM x WN; each wave owns a (BM/WM) x (BN/WN) block
//    of 16x16 accumulators fed by v_mfma_f32_16x16x32_bf16.
//  * BK = 64: each K-tile is two 32-deep MFMA steps.  Double-buffered LDS with register
//    staging: the next tile's global loads are issued before the current tile's MFMAs,
//    written to the other LDS buffer after them, one barrier per K-tile.
//  * LDS tiles are [rows][64] bf16 (128-B rows) with the 16-B chunk index XOR-swizzled
//    by (row>>1)&7 so the 16 rows a ds_read_b128 lane-group touches land on 16 distinct
//    16-B slots (conflict-free fragment reads, conflict-free 8-lane row writes).
//  * The loader folds: zero / reflection padding, nearest upsample (src = dst / up),
//    a virtual channel concat of two tensors (U-Net skip) and the input activation
//    (LeakyReLU for encoders, ReLU for decoders) -- none of those tensors is materialised.
//  * CONVT (MODE 1) = sub-pixel decomposition: blockIdx.z selects the output parity class
//    (ry, rx); only the ceil(K/s)^2 taps that hit the class are iterated, so a 4x4 s2
//    transposed conv costs 4 taps per output pixel instead of 16 with 3/4 zeros.
//  * Epilogue is staged through LDS as fp32 so every lane stores 16 contiguous bytes:
//    bias + output activation (tanh for the U-Net head) + optional act'(x) multiply for
//    dgrad (backward through the activation fused into the producing dgrad) + a channel
//    split into two tensors (gradient of a virtual concat).  Split-K (small-M layers at
//    the U-Net bottleneck) accumulates fp32 into a workspace, finished by
//    conv_finalize_kernel.
//  * Workgroup ids are remapped XCD-aware (blocks b, b+8 share an L2) so the n-tiles of
//    one m-tile run on one XCD and re-read the same activation panel from L2.
#include "common.h"
#include "conv.h"

namespace p2p {

constexpr int BK = 64;

__device__ __forceinline__ int swz(int row, int chunk) {  // element offset in a [rows][64] tile
  return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3);
}

struct ClassGeom {
  int ry, rx, ky0, kx0, dy, dx, Tj, Ti, Hq, Wq, Mc, Kc;
};

template <int MODE>
__device__ __forceinline__ ClassGeom class_geom(const ConvFwdArgs& a, int cls) {
  ClassGeom g;
  if (MODE == 0) {
    g.ry = g.rx = g.ky0 = g.kx0 = g.dy = g.dx = 0;
    g.Tj = a.KH;
    g.Ti = a.KW;
    g.Hq = a.OH;
    g.Wq = a.OW;
  } else {
    const int s = a.stride, p = a.pad;
    g.ry = cls / s;
    g.rx = cls % s;
    g.ky0 = (g.ry + p) % s;
    g.kx0 = (g.rx + p) % s;
    g.dy = (g.ry + p - g.ky0) / s;
    g.dx = (g.rx + p - g.kx0) / s;
    g.Tj = g.ky0 < a.KH ? (a.KH - g.ky0 + s - 1) / s : 0;
    g.Ti = g.kx0 < a.KW ? (a.KW - g.kx0 + s - 1) / s : 0;
    g.Hq = a.OH > g.ry ? (a.OH - g.ry + s - 1) / s : 0;
    g.Wq = a.OW > g.rx ? (a.OW - g.rx + s - 1) / s : 0;
  }
  g.Mc = a.N * g.Hq * g.Wq;
  g.Kc = g.Tj * g.Ti * a.C;
  return g;
}

template <int BM, int BN>
struct FwdSmem {
  static constexpr int pipe = 2 * (BM + BN) * BK * 2;
  static constexpr int epi = BM * (BN + 4) * 4;
  static constexpr int bytes = pipe > epi ? pipe : epi;
};

template <int BM, int BN, int WM, int WN, int MODE>
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

  // ---- per-thread A rows (fixed over the K loop)
  int a_ybase[AROWS], a_xbase[AROWS], a_nbase[AROWS];
  bool a_ok[AROWS];
  const int HWq = g.Hq * g.Wq;
#pragma unroll
  for (int i = 0; i < AROWS; ++i) {
    int m = m0 + (tid >> 3) + 32 * i;
    a_ok[i] = m < g.Mc;
    int mm = a_ok[i] ? m : 0;
    int n = mm / HWq;
    int r = mm - n * HWq;
    int qy = r / g.Wq;
    int qx = r - qy * g.Wq;
    a_nbase[i] = n * a.H;
    if (MODE == 0) {
      a_ybase[i] = qy * a.stride - a.pad;
      a_xbase[i] = qx * a.stride - a.pad;
    } else {
      a_ybase[i] = qy + g.dy;
      a_xbase[i] = qx + g.dx;
    }
  }
  const int ush = a.up == 2 ? 1 : 0;
  const int Hu = a.H << ush, Wu = a.W << ush;

  u32x4 ra[AROWS], rb[BROWS];

  auto load_tile = [&](int kt) {
    const int k = kt * BK + kc * 8;
    const bool kok = k < g.Kc;
    int tap = 0, ci = 0, t_y = 0, t_x = 0;
    if (kok) {
      tap = k / C;
      ci = k - tap * C;
      t_y = tap / g.Ti;
      t_x = tap - t_y * g.Ti;
    }
    const bool src1 = ci < C1;
    const bf16* src = src1 ? x1 : x2;
    const int cs = src1 ? C1 : C2;
    const int cio = src1 ? ci : ci - C1;
#pragma unroll
    for (int i = 0; i < AROWS; ++i) {
      u32x4 v = zero_u32x4();
      if (kok && a_ok[i]) {
        int iy, ix;
        bool inb;
        if (MODE == 0) {
          int uy = a_ybase[i] + t_y, ux = a_xbase[i] + t_x;
          if (a.reflect) {
            uy = reflect_idx(uy, Hu);
            ux = reflect_idx(ux, Wu);
            inb = true;
          } else {
            inb = (unsigned)uy < (unsigned)Hu && (unsigned)ux < (unsigned)Wu;
          }
          iy = uy >> ush;
          ix = ux >> ush;
        } else {
          iy = a_ybase[i] - t_y;
          ix = a_xbase[i] - t_x;
          inb = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
        }
        if (inb) {
          const long pix = (long)(a_nbase[i] + iy) * a.W + ix;
          v = *reinterpret_cast<const u32x4*>(src + pix * cs + cio);
          v = act8(v, a.act_in);
        }
      }
      ra[i] = v;
    }
    // B (weights)
    long woff = 0;
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
      if (kok && row < BN && co < a.Cout) {
        const long base = (MODE == 0) ? (long)co * g.Kc : (long)co * a.KH * a.KW * C;
        v = *reinterpret_cast<const u32x4*>(w + base + woff);
      }
      rb[i] = v;
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

  // ---- epilogue: stage fp32 tile in LDS, then 16-B stores
  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int LDC = BN + 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * TN * 16 + j * 16 + (lane & 15);
      const int rowb = wm * TM * 16 + i * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int r = 0; r < 4; ++r) Cs[(rowb + r) * LDC + col] = acc[i][j][r];
    }
  __syncthreads();

  const int s = a.stride;
  constexpr int CPR = BN / 8;  // 8-channel chunks per row
  for (int c = tid; c < BM * CPR; c += 256) {
    const int row = c / CPR, cc = c - row * CPR;
    const int m = m0 + row;
    const int co = n0 + cc * 8;
    if (m >= g.Mc || co >= a.Cout) continue;
    long pix;
    if (MODE == 0) {
      pix = m;
    } else {
      int n = m / HWq;
      int r = m - n * HWq;
      int qy = r / g.Wq;
      int qx = r - qy * g.Wq;
      pix = ((long)n * a.OH + qy * s + g.ry) * a.OW + qx * s + g.rx;
    }
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(Cs + row * LDC + cc * 8);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(Cs + row * LDC + cc * 8 + 4);
    float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    if (a.splits > 1) {
      float* dst = a.ws + pix * a.Cout + co;
#pragma unroll
      for (int j = 0; j < 8; ++j) atomicAdd(dst + j, v[j]);
      continue;
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
    if (a.act_bwd) {
      const bf16* xb = static_cast<const bf16*>(first ? a.xb1 : a.xb2);
      bf16x8 xv = *reinterpret_cast<const bf16x8*>(xb + pix * ld + cof);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= act_grad_from_input((float)xv[j], a.act_bwd);
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
    bf16* y = static_cast<bf16*>(first ? a.y1 : a.y2);
    *reinterpret_cast<bf16x8*>(y + pix * ld + cof) = o;
  }
}

// split-K finish: ws [P][Cout] fp32 -> bias / act / act' / channel split -> bf16
__global__ void __launch_bounds__(256) conv_finalize_kernel(ConvFwdArgs a, long P) {
  const long nchunks = P * (a.Cout / 8);
  for (long c = blockIdx.x * 256L + threadIdx.x; c < nchunks; c += (long)gridDim.x * 256) {
    const long pix = c / (a.Cout / 8);
    const int co = (int)(c - pix * (a.Cout / 8)) * 8;
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(a.ws + pix * a.Cout + co);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(a.ws + pix * a.Cout + co + 4);
    float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
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
    if (a.act_bwd) {
      const bf16* xb = static_cast<const bf16*>(first ? a.xb1 : a.xb2);
      bf16x8 xv = *reinterpret_cast<const bf16x8*>(xb + pix * ld + cof);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= act_grad_from_input((float)xv[j], a.act_bwd);
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
    bf16* y = static_cast<bf16*>(first ? a.y1 : a.y2);
    *reinterpret_cast<bf16x8*>(y + pix * ld + cof) = o;
  }
}

template <int BM, int BN, int WM, int WN, int MODE>
static int launch_fwd(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int smem = FwdSmem<BM, BN>::bytes;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_fwd_kernel<BM, BN, WM, WN, MODE>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set = true;
  }
  // max rows over classes
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
  hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, WM, WN, MODE>), grid, dim3(256), smem, st, a);
  return (int)hipGetLastError();
}

template <int MODE>
static int dispatch_fwd(const ConvFwdArgs& a, int bm, int bn, hipStream_t st) {
  if (bm == 128 && bn == 128) return launch_fwd<128, 128, 2, 2, MODE>(a, st);
  if (bm == 128 && bn == 64) return launch_fwd<128, 64, 2, 2, MODE>(a, st);
  if (bm == 64 && bn == 128) return launch_fwd<64, 128, 2, 2, MODE>(a, st);
  if (bm == 64 && bn == 64) return launch_fwd<64, 64, 2, 2, MODE>(a, st);
  if (bm == 256 && bn == 32) return launch_fwd<256, 32, 4, 1, MODE>(a, st);
  if (bm == 256 && bn == 16) return launch_fwd<256, 16, 4, 1, MODE>(a, st);
  if (bm == 64 && bn == 16) return launch_fwd<64, 16, 4, 1, MODE>(a, st);
  return -1;
}

}  // namespace p2p

extern "C" int p2p_conv_fwd(const p2p::ConvFwdArgs* a, int mode, int bm, int bn, hipStream_t st) {
  return mode == 0 ? p2p::dispatch_fwd<0>(*a, bm, bn, st) : p2p::dispatch_fwd<1>(*a, bm, bn, st);
}

extern "C" int p2p_conv_finalize(const p2p::ConvFwdArgs* a, hipStream_t st) {
  const long P = (long)a->N * a->OH * a->OW;
  const long nchunks = P * (a->Cout / 8);
  long blocks = (nchunks + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(p2p::conv_finalize_kernel, dim3((unsigned)blocks), dim3(256), 0, st, *a, P);
  return (int)hipGetLastError();
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
