// Family-R (compression GAN) fringe ops on bf16 NHWC tensors (gfx950): shared-scalar
// PReLU, anisotropic TV loss, the 3-bit quantiser, AvgPool(3, s2, p1, no-pad-count) of the
// multiscale discriminator, 2x2 max-pool (VGG19), per-pixel L2 normalisation over channels
// (compression network head) and pixel (un)shuffle.  All memory-bound: one thread per
// output element (or pixel), backward passes written as gathers so no atomics are needed
// and every result is bitwise reproducible; reductions are two-stage (block partials ->
// one finishing block, fixed order).
//   reference: networks.py:173-236 (C), :452 (PReLU), :732 (AvgPool), train.py:123-126
//   (TV), generate_dataset.py:29-34 (quantiser), torchvision VGG19 (max-pool).
#include "bounds.h"
#include "common.h"

namespace p2p {

static inline unsigned mgrid(long work) {
  long b = (work + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (unsigned)b;
}

__device__ __forceinline__ float block_sum256(float s, float* red) {
  s = warp_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// ------------------------------------------------------------------ PReLU (one slope)
__global__ void __launch_bounds__(256) prelu_fwd_kernel(const bf16* __restrict__ x, long n,
                                                        const float* __restrict__ w, bf16* __restrict__ y) {
  const float a = w[0];
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const float v = (float)x[e];
    y[e] = (bf16)(v > 0.f ? v : a * v);
  }
}

// dx = dy * (x > 0 ? 1 : a); ws[block] = sum dy * x * [x <= 0]
__global__ void __launch_bounds__(256) prelu_bwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                        long n, const float* __restrict__ w,
                                                        bf16* __restrict__ dx, float* __restrict__ ws) {
  const float a = w[0];
  float s = 0.f;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const float v = (float)x[e], g = (float)dy[e];
    if (dx) dx[e] = (bf16)(v > 0.f ? g : a * g);
    if (v <= 0.f) s += g * v;
  }
  __shared__ float red[4];
  const float t = block_sum256(s, red);
  if (threadIdx.x == 0) ws[blockIdx.x] = t;
}

__global__ void __launch_bounds__(256) sum_final_kernel(const float* __restrict__ ws, int nb, float scale,
                                                        int accumulate, float* __restrict__ out) {
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += 256) s += ws[i];
  __shared__ float red[4];
  const float t = block_sum256(s, red) * scale;
  if (threadIdx.x == 0) out[0] = accumulate ? out[0] + t : t;
}

// ------------------------------------------------------------------ TV loss
// mean|x[..., w] - x[..., w+1]| + mean|x[h, :] - x[h+1, :]|  over NHWC (N, H, W, C)
__global__ void __launch_bounds__(256) tv_partial_kernel(const bf16* __restrict__ x, int N, int H, int W, int C,
                                                         float ih, float iv, float* __restrict__ ws) {
  const long n = (long)N * H * W * C;
  float s = 0.f;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const long pix = e / C;
    const int w = (int)(pix % W);
    const int h = (int)((pix / W) % H);
    const float v = (float)x[e];
    if (w + 1 < W) s += fabsf(v - (float)x[e + C]) * ih;
    if (h + 1 < H) s += fabsf(v - (float)x[e + (long)W * C]) * iv;
  }
  __shared__ float red[4];
  const float t = block_sum256(s, red);
  if (threadIdx.x == 0) ws[blockIdx.x] = t;
}

__device__ __forceinline__ float sgnf(float d) { return d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f); }

__global__ void __launch_bounds__(256) tv_grad_kernel(const bf16* __restrict__ x, int N, int H, int W, int C,
                                                      float ih, float iv, const float* __restrict__ gout,
                                                      bf16* __restrict__ dx) {
  const long n = (long)N * H * W * C;
  const float g = gout[0];
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const long pix = e / C;
    const int w = (int)(pix % W);
    const int h = (int)((pix / W) % H);
    const float v = (float)x[e];
    float d = 0.f;
    if (w + 1 < W) d += sgnf(v - (float)x[e + C]) * ih;
    if (w > 0) d -= sgnf((float)x[e - C] - v) * ih;
    if (h + 1 < H) d += sgnf(v - (float)x[e + (long)W * C]) * iv;
    if (h > 0) d -= sgnf((float)x[e - (long)W * C] - v) * iv;
    dx[e] = (bf16)(g * d);
  }
}

// ------------------------------------------------------------------ quantiser
__global__ void __launch_bounds__(256) quantize_kernel(const bf16* __restrict__ x, long n, float m,
                                                       bf16* __restrict__ y) {
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const float v = fminf(fmaxf((float)x[e], 0.f), 1.f);
    y[e] = (bf16)(rintf(v * m) / m);
  }
}

// quantise + pixel-unshuffle(r) in one pass: besides y (x's layout) it writes the unshuffled,
// channel-padded copy yu [N][H/r][W/r][Cp], channel c*r*r + i*r + j = y[h*r+i][w*r+j][c], the
// pad channels zero -- the ExpandNetwork's head input (networks.py:457, 494-496), which then
// needs neither an unshuffle nor a channel-pad pass.  One thread per yu pixel.
__global__ void __launch_bounds__(256) quantize_unshuffle_kernel(const bf16* __restrict__ x, int N, int H, int W,
                                                                 int C, int r, float m, bf16* __restrict__ y,
                                                                 bf16* __restrict__ yu, int Cp) {
  const int OH = H / r, OW = W / r;
  const long np = (long)N * OH * OW;
  for (long p = blockIdx.x * 256L + threadIdx.x; p < np; p += (long)gridDim.x * 256) {
    const int ow = (int)(p % OW);
    const long t = p / OW;
    const int oh = (int)(t % OH);
    const long n = t / OH;
    bf16* o = yu + p * Cp;
    for (int c = C * r * r; c < Cp; ++c) o[c] = (bf16)0.f;
    for (int i = 0; i < r; ++i)
      for (int j = 0; j < r; ++j) {
        const long src = ((n * H + oh * r + i) * W + ow * r + j) * C;
        for (int c = 0; c < C; ++c) {
          const float v = fminf(fmaxf((float)x[src + c], 0.f), 1.f);
          const bf16 q = (bf16)(rintf(v * m) / m);
          y[src + c] = q;
          o[c * r * r + i * r + j] = q;
        }
      }
  }
}

// ------------------------------------------------------------------ AvgPool 3x3 s2 p1, count_include_pad=False
__device__ __forceinline__ int pool_count(int o, int n) {  // valid taps of window 2o-1 .. 2o+1
  const int lo = max(2 * o - 1, 0), hi = min(2 * o + 1, n - 1);
  return hi - lo + 1;
}

__global__ void __launch_bounds__(256) avgpool_fwd_kernel(const bf16* __restrict__ x, int N, int H, int W, int C,
                                                          int OH, int OW, bf16* __restrict__ y) {
  const long n = (long)N * OH * OW * C;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int c = (int)(e % C);
    const long p = e / C;
    const int ow = (int)(p % OW);
    const int oh = (int)((p / OW) % OH);
    const int b = (int)(p / ((long)OW * OH));
    float s = 0.f;
    for (int dy = -1; dy <= 1; ++dy) {
      const int ih = 2 * oh + dy;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int dx = -1; dx <= 1; ++dx) {
        const int iw = 2 * ow + dx;
        if ((unsigned)iw >= (unsigned)W) continue;
        s += (float)x[(((long)b * H + ih) * W + iw) * C + c];
      }
    }
    y[e] = (bf16)(s / (float)(pool_count(oh, H) * pool_count(ow, W)));
  }
}

__global__ void __launch_bounds__(256) avgpool_bwd_kernel(const bf16* __restrict__ gy, int N, int H, int W, int C,
                                                          int OH, int OW, bf16* __restrict__ gx) {
  const long n = (long)N * H * W * C;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int c = (int)(e % C);
    const long p = e / C;
    const int iw = (int)(p % W);
    const int ih = (int)((p / W) % H);
    const int b = (int)(p / ((long)W * H));
    float s = 0.f;
    // outputs whose window 2o-1..2o+1 contains i: o in [ceil((i-1)/2), floor((i+1)/2)]
    for (int oh = (ih > 0 ? ih : ih + 1) / 2; oh <= (ih + 1) / 2; ++oh) {
      if (oh >= OH) continue;
      for (int ow = (iw > 0 ? iw : iw + 1) / 2; ow <= (iw + 1) / 2; ++ow) {
        if (ow >= OW) continue;
        s += (float)gy[(((long)b * OH + oh) * OW + ow) * C + c] /
             (float)(pool_count(oh, H) * pool_count(ow, W));
      }
    }
    gx[e] = (bf16)s;
  }
}

// ------------------------------------------------------------------ MaxPool 2x2 s2
// PyTorch semantics: the gradient goes to the FIRST maximum of the window in row-major
// order (strict '>' scan; NaN wins).
__device__ __forceinline__ int max2x2_arg(const bf16* x, long base, long rowst, int C, float* mv) {
  int arg = 0;
  float m = (float)x[base];
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    const float v = (float)x[base + (k >> 1) * rowst + (k & 1) * C];
    if (v > m || v != v) {
      m = v;
      arg = k;
    }
  }
  *mv = m;
  return arg;
}

__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const bf16* __restrict__ x, int N, int H, int W, int C,
                                                          bf16* __restrict__ y) {
  const int OH = H / 2, OW = W / 2;
  const long n = (long)N * OH * OW * C;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int c = (int)(e % C);
    const long p = e / C;
    const int ow = (int)(p % OW);
    const int oh = (int)((p / OW) % OH);
    const int b = (int)(p / ((long)OW * OH));
    float m;
    max2x2_arg(x, (((long)b * H + 2 * oh) * W + 2 * ow) * C + c, (long)W * C, C, &m);
    y[e] = (bf16)m;
  }
}

__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ gy,
                                                          int N, int H, int W, int C, bf16* __restrict__ gx) {
  const int OH = H / 2, OW = W / 2;
  const long n = (long)N * H * W * C;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int c = (int)(e % C);
    const long p = e / C;
    const int iw = (int)(p % W);
    const int ih = (int)((p / W) % H);
    const int b = (int)(p / ((long)W * H));
    const int oh = ih >> 1, ow = iw >> 1;
    float g = 0.f;
    if (oh < OH && ow < OW) {
      float m;
      const int arg = max2x2_arg(x, (((long)b * H + 2 * oh) * W + 2 * ow) * C + c, (long)W * C, C, &m);
      if (arg == ((ih & 1) << 1 | (iw & 1))) g = (float)gy[(((long)b * OH + oh) * OW + ow) * C + c];
    }
    gx[e] = (bf16)g;
  }
}

// 8-channel vector variants (C % 8 == 0, even H and W -- every VGG pool): one thread per
// (output pixel, 8-channel chunk) reads its 2x2 window once (4 x 16-B loads); the backward
// writes all four input-gradient vectors from that one read of x and gy.  Same tie rule as
// max2x2_arg (first maximum in window order wins; NaN propagates).
__device__ __forceinline__ void max2x2_vec(const bf16* x, long base, long rowst, int C, float* m,
                                           int* arg) {
  float f[4][8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bf16x8 v = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(
                                                     x + base + (k >> 1) * rowst + (k & 1) * C));
#pragma unroll
    for (int j = 0; j < 8; ++j) f[k][j] = (float)v[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    m[j] = f[0][j];
    arg[j] = 0;
#pragma unroll
    for (int k = 1; k < 4; ++k)
      if (f[k][j] > m[j] || f[k][j] != f[k][j]) {
        m[j] = f[k][j];
        arg[j] = k;
      }
  }
}

__global__ void __launch_bounds__(256) maxpool_fwd_vec_kernel(const bf16* __restrict__ x, int N, int H, int W,
                                                              int C, bf16* __restrict__ y) {
  const int OH = H / 2, OW = W / 2, CG = C / 8;
  const long n = (long)N * OH * OW * CG;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int cg = (int)(e % CG);
    const long p = e / CG;
    const int ow = (int)(p % OW);
    const long bh = p / OW;   // b * OH + oh
    float m[8];
    int arg[8];
    max2x2_vec(x, ((bh * 2) * W + 2 * ow) * C + cg * 8, (long)W * C, C, m, arg);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)m[j];
    *reinterpret_cast<u32x4*>(y + p * C + cg * 8) = __builtin_bit_cast(u32x4, o);
  }
}

__global__ void __launch_bounds__(256) maxpool_bwd_vec_kernel(const bf16* __restrict__ x,
                                                              const bf16* __restrict__ gy, int N, int H,
                                                              int W, int C, bf16* __restrict__ gx) {
  const int OH = H / 2, OW = W / 2, CG = C / 8;
  const long n = (long)N * OH * OW * CG;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int cg = (int)(e % CG);
    const long p = e / CG;
    const int ow = (int)(p % OW);
    const long bh = p / OW;
    const long base = ((bh * 2) * W + 2 * ow) * C + cg * 8;
    float m[8];
    int arg[8];
    max2x2_vec(x, base, (long)W * C, C, m, arg);
    const bf16x8 g = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(gy + p * C + cg * 8));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = arg[j] == k ? g[j] : (bf16)0.f;
      *reinterpret_cast<u32x4*>(gx + base + (k >> 1) * (long)W * C + (k & 1) * C) = __builtin_bit_cast(u32x4, o);
    }
  }
}

// ------------------------------------------------------------------ L2 normalise over channels
// y = x / max(||x||, eps);  dx = (dy - y * <dy, y>) / max(||x||, eps)  (norm > eps),
// dx = dy / eps otherwise (F.normalize's clamp_min has zero gradient below eps).
// r > 1: x is the PRE-PixelShuffle tensor [N][IH][IW][C*r*r] and y / dy the shuffled one
// [N][IH*r][IW*r][C] (CompressionNetwork: conv s2 -> PixelShuffle(2) -> l2-normalise + x,
// networks.py:217-218, 233-236): output pixel (oh, ow) channel c reads x[oh/r][ow/r]
// [c*r*r + (oh%r)*r + ow%r] -- the shuffle is this pass's addressing, no pass of its own, and
// the backward writes dx in the pre-shuffle layout (the un-shuffle of the gradient, too).
struct L2Map {
  int r, IW, OW, OH, Cin;
  __device__ __forceinline__ long base(long p) const {   // x index of channel 0 of output pixel p
    if (r == 1) return p * Cin;
    const int ow = (int)(p % OW);
    const long t = p / OW;
    const int oh = (int)(t % OH);
    const long b = t / OH;
    return ((b * (OH / r) + oh / r) * IW + ow / r) * Cin + (oh % r) * r + ow % r;
  }
};

__global__ void __launch_bounds__(256) l2norm_fwd_kernel(const bf16* __restrict__ x, long P, int C, float eps,
                                                         const bf16* __restrict__ res, bf16* __restrict__ y,
                                                         L2Map mp) {
  const int cs = mp.r * mp.r;   // channel stride of the output's channels inside x
  for (long p = blockIdx.x * 256L + threadIdx.x; p < P; p += (long)gridDim.x * 256) {
    const long xb = mp.base(p);
    float s = 0.f;
    for (int c = 0; c < C; ++c) {
      const float v = (float)x[xb + c * cs];
      s += v * v;
    }
    const float inv = 1.f / fmaxf(sqrtf(s), eps);
    // res: the CompressionNetwork's residual input added in the same pass (networks.py:236)
    for (int c = 0; c < C; ++c)
      y[p * C + c] = (bf16)((float)x[xb + c * cs] * inv + (res ? (float)res[p * C + c] : 0.f));
  }
}

__global__ void __launch_bounds__(256) l2norm_bwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ gy,
                                                         long P, int C, float eps, bf16* __restrict__ gx,
                                                         L2Map mp) {
  const int cs = mp.r * mp.r;
  for (long p = blockIdx.x * 256L + threadIdx.x; p < P; p += (long)gridDim.x * 256) {
    const long xb = mp.base(p);
    float s = 0.f;
    for (int c = 0; c < C; ++c) {
      const float v = (float)x[xb + c * cs];
      s += v * v;
    }
    const float nrm = sqrtf(s);
    const float d = fmaxf(nrm, eps);
    float dot = 0.f;
    if (nrm > eps)
      for (int c = 0; c < C; ++c) dot += (float)gy[p * C + c] * (float)x[xb + c * cs];
    const float k = nrm > eps ? dot / (d * d * d) : 0.f;
    for (int c = 0; c < C; ++c)
      gx[xb + c * cs] = (bf16)((float)gy[p * C + c] / d - (float)x[xb + c * cs] * k);
  }
}

// ------------------------------------------------------------------ pixel (un)shuffle, NHWC
// unshuffle: out[n][h][w][c*r*r + i*r + j] = in[n][h*r+i][w*r+j][c]   (out H/r x W/r x C*r*r)
// shuffle is the inverse map.  dir 0 = unshuffle, 1 = shuffle; shapes are the OUTPUT's.
__global__ void __launch_bounds__(256) pixel_shuffle_kernel(const bf16* __restrict__ in, int N, int OH, int OW,
                                                            int OC, int r, int dir, bf16* __restrict__ out) {
  const long n = (long)N * OH * OW * OC;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int oc = (int)(e % OC);
    const long p = e / OC;
    const int ow = (int)(p % OW);
    const int oh = (int)((p / OW) % OH);
    const int b = (int)(p / ((long)OW * OH));
    long src;
    if (dir == 0) {  // input (OH*r, OW*r, OC/(r*r))
      const int C = OC / (r * r);
      const int c = oc / (r * r), ij = oc % (r * r), i = ij / r, j = ij % r;
      src = (((long)b * OH * r + oh * r + i) * (OW * r) + ow * r + j) * C + c;
    } else {         // input (OH/r, OW/r, OC*r*r)
      const int IH = OH / r, IW = OW / r, IC = OC * r * r;
      const int ih = oh / r, i = oh % r, iw = ow / r, j = ow % r;
      src = (((long)b * IH + ih) * IW + iw) * IC + oc * r * r + i * r + j;
    }
    out[e] = in[src];
  }
}


// ------------------------------------------------------------------ nearest-x2 + reflect-1 dgrad taps
// Input-gradient GEMM image of G.deconv{2,3} (UpsampleConvLayer, networks.py:408-423): the
// 3x3 kernel seen through nearest x2 + edge pad 1 is ONE 4x4 stride-2 conv over dY whose taps
// are phase sums of the 3x3 taps, W''[ci][co][a][b] = sum_kl M[a][k] M[b][l] w[co][ci][k][l]
// with M = ((0,0,1), (0,1,1), (1,1,0), (1,0,0)) -- i.e. per axis out = (w2, w1+w2, w0+w1, w0).
// Written straight into the bf16 [Xp][4][4][Yp] operand image (x = ci, y = co, zero padded):
// a device-only computation, so it is legal inside a hipGraph capture (no host tensor).
__device__ __forceinline__ float up2_axis(const float* v, int a, int stride) {
  // v[0], v[stride], v[2*stride] = taps 0, 1, 2 along one axis
  return a == 0 ? v[2 * stride] : a == 1 ? v[stride] + v[2 * stride] : a == 2 ? v[0] + v[stride] : v[0];
}

// out[i] = i < n ? x[i] : fill for i < nout (fp32): a norm's per-channel vectors padded to the
// 8-channel groups of the norm kernels (odd channel counts: family R's BN(3)) and copied back
__global__ void __launch_bounds__(256) vec_pad_kernel(const float* __restrict__ x, int n, float fill, int nout,
                                                      float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < nout) out[i] = i < n ? x[i] : fill;
}

// The tiny-Cout "col" GEMM's weight (bindings.cpp conv_fwd): out[t * Cvp + co][c] =
// w[co][t][c] for co < Cv, zero for the padded tap slots and rows (out is [Ncol][C]); one
// pass instead of a memset + a strided aten copy per call.
__global__ void __launch_bounds__(256) col_weight_kernel(const bf16* __restrict__ w, int T, int C, int Cv, int Cvp,
                                                         int Ncol, bf16* __restrict__ out) {
  const long total = (long)Ncol * C;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int row = (int)(e / C), c = (int)(e - (long)row * C);
    const int t = row / Cvp, co = row - t * Cvp;
    out[e] = (t < T && co < Cv) ? w[((long)co * T + t) * C + c] : (bf16)0.f;
  }
}

__global__ void __launch_bounds__(256) up2_dgrad_image_kernel(const float* __restrict__ w, int Cout, int Cin,
                                                              int Xp, int Yp, bf16* __restrict__ out) {
  const long total = (long)Xp * 16 * Yp;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int y = (int)(e % Yp);
    const long r = e / Yp;
    const int t = (int)(r % 16);
    const int x = (int)(r / 16);
    const int a = t >> 2, b = t & 3;
    float v = 0.f;
    if (x < Cin && y < Cout) {
      const float* k = w + ((long)y * Cin + x) * 9;   // w[co][ci][3][3]
      float rows[3];
#pragma unroll
      for (int l = 0; l < 3; ++l) rows[l] = up2_axis(k + l, a, 3);   // sum over k for column l
      v = up2_axis(rows, b, 1);
    }
    out[e] = (bf16)v;
  }
}

}  // namespace p2p

extern "C" {

int p2p_misc_nblocks(long n) { return (int)p2p::mgrid(n); }

int p2p_prelu_fwd(const void* x, long n, const float* w, void* y, hipStream_t st) {
  hipLaunchKernelGGL(p2p::prelu_fwd_kernel, dim3(p2p::mgrid(n)), dim3(256), 0, st,
                     static_cast<const p2p::bf16*>(x), n, w, static_cast<p2p::bf16*>(y));
  return (int)hipGetLastError();
}

// ws >= p2p_misc_nblocks(n) floats; gw: [1] fp32 (accumulated when accumulate != 0)
int p2p_prelu_bwd(const void* x, const void* dy, long n, const float* w, void* dx, float* ws, float* gw,
                  int accumulate, hipStream_t st) {
  const unsigned nb = p2p::mgrid(n);
  hipLaunchKernelGGL(p2p::prelu_bwd_kernel, dim3(nb), dim3(256), 0, st, static_cast<const p2p::bf16*>(x),
                     static_cast<const p2p::bf16*>(dy), n, w, static_cast<p2p::bf16*>(dx), ws);
  hipLaunchKernelGGL(p2p::sum_final_kernel, dim3(1), dim3(256), 0, st, ws, (int)nb, 1.f, accumulate, gw);
  return (int)hipGetLastError();
}

int p2p_tv_fwd(const void* x, int N, int H, int W, int C, float* ws, float* out, hipStream_t st) {
  const long n = (long)N * H * W * C;
  const unsigned nb = p2p::mgrid(n);
  const float ih = W > 1 ? 1.f / ((float)N * C * H * (W - 1)) : 0.f;
  const float iv = H > 1 ? 1.f / ((float)N * C * (H - 1) * W) : 0.f;
  hipLaunchKernelGGL(p2p::tv_partial_kernel, dim3(nb), dim3(256), 0, st, static_cast<const p2p::bf16*>(x), N, H,
                     W, C, ih, iv, ws);
  hipLaunchKernelGGL(p2p::sum_final_kernel, dim3(1), dim3(256), 0, st, ws, (int)nb, 1.f, 0, out);
  return (int)hipGetLastError();
}

int p2p_tv_bwd(const void* x, int N, int H, int W, int C, const float* gout, void* dx, hipStream_t st) {
  const long n = (long)N * H * W * C;
  const float ih = W > 1 ? 1.f / ((float)N * C * H * (W - 1)) : 0.f;
  const float iv = H > 1 ? 1.f / ((float)N * C * (H - 1) * W) : 0.f;
  hipLaunchKernelGGL(p2p::tv_grad_kernel, dim3(p2p::mgrid(n)), dim3(256), 0, st,
                     static_cast<const p2p::bf16*>(x), N, H, W, C, ih, iv, gout, static_cast<p2p::bf16*>(dx));
  return (int)hipGetLastError();
}

int p2p_quantize(const void* x, long n, int bits, void* y, hipStream_t st) {
  const float m = (float)((1 << bits) - 1);
  hipLaunchKernelGGL(p2p::quantize_kernel, dim3(p2p::mgrid(n)), dim3(256), 0, st,
                     static_cast<const p2p::bf16*>(x), n, m, static_cast<p2p::bf16*>(y));
  return (int)hipGetLastError();
}

int p2p_quantize_unshuffle(const void* x, int N, int H, int W, int C, int bits, int r, void* y, void* yu, int Cp,
                           hipStream_t st) {
  const float m = (float)((1 << bits) - 1);
  const long np = (long)N * (H / r) * (W / r);
  hipLaunchKernelGGL(p2p::quantize_unshuffle_kernel, dim3(p2p::mgrid(np)), dim3(256), 0, st,
                     static_cast<const p2p::bf16*>(x), N, H, W, C, r, m, static_cast<p2p::bf16*>(y),
                     static_cast<p2p::bf16*>(yu), Cp);
  return (int)hipGetLastError();
}

int p2p_avgpool3s2(const void* x, int N, int H, int W, int C, int OH, int OW, void* y, int bwd, hipStream_t st) {
  if (!bwd) {
    const long n = (long)N * OH * OW * C;
    hipLaunchKernelGGL(p2p::avgpool_fwd_kernel, dim3(p2p::mgrid(n)), dim3(256), 0, st,
                       static_cast<const p2p::bf16*>(x), N, H, W, C, OH, OW, static_cast<p2p::bf16*>(y));
  } else {  // x = gy (OH x OW), y = gx (H x W)
    const long n = (long)N * H * W * C;
    hipLaunchKernelGGL(p2p::avgpool_bwd_kernel, dim3(p2p::mgrid(n)), dim3(256), 0, st,
                       static_cast<const p2p::bf16*>(x), N, H, W, C, OH, OW, static_cast<p2p::bf16*>(y));
  }
  return (int)hipGetLastError();
}

int p2p_maxpool2(const void* x, const void* gy, int N, int H, int W, int C, void* out, hipStream_t st) {
  if (C % 8 == 0 && H % 2 == 0 && W % 2 == 0) {
    const long n = (long)N * (H / 2) * (W / 2) * (C / 8);
    if (!gy)
      hipLaunchKernelGGL(p2p::maxpool_fwd_vec_kernel, dim3(p2p::mgrid(n)), dim3(256), 0, st,
                         static_cast<const p2p::bf16*>(x), N, H, W, C, static_cast<p2p::bf16*>(out));
    else
      hipLaunchKernelGGL(p2p::maxpool_bwd_vec_kernel, dim3(p2p::mgrid(n)), dim3(256), 0, st,
                         static_cast<const p2p::bf16*>(x), static_cast<const p2p::bf16*>(gy), N, H, W, C,
                         static_cast<p2p::bf16*>(out));
    return (int)hipGetLastError();
  }
  if (!gy) {
    const long n = (long)N * (H / 2) * (W / 2) * C;
    hipLaunchKernelGGL(p2p::maxpool_fwd_kernel, dim3(p2p::mgrid(n)), dim3(256), 0, st,
                       static_cast<const p2p::bf16*>(x), N, H, W, C, static_cast<p2p::bf16*>(out));
  } else {
    const long n = (long)N * H * W * C;
    hipLaunchKernelGGL(p2p::maxpool_bwd_kernel, dim3(p2p::mgrid(n)), dim3(256), 0, st,
                       static_cast<const p2p::bf16*>(x), static_cast<const p2p::bf16*>(gy), N, H, W, C,
                       static_cast<p2p::bf16*>(out));
  }
  return (int)hipGetLastError();
}

// r > 1: x pre-PixelShuffle [N][IH][IW][C*r*r], P = N * IH*r * IW*r output pixels of C channels
int p2p_l2norm(const void* x, const void* gy, long P, int C, float eps, const void* res, void* out, int r, int IH,
               int IW, hipStream_t st) {
  const p2p::L2Map mp{r, IW, IW * r, IH * r, C * r * r};
  if (!gy)
    hipLaunchKernelGGL(p2p::l2norm_fwd_kernel, dim3(p2p::mgrid(P)), dim3(256), 0, st,
                       static_cast<const p2p::bf16*>(x), P, C, eps, static_cast<const p2p::bf16*>(res),
                       static_cast<p2p::bf16*>(out), mp);
  else
    hipLaunchKernelGGL(p2p::l2norm_bwd_kernel, dim3(p2p::mgrid(P)), dim3(256), 0, st,
                       static_cast<const p2p::bf16*>(x), static_cast<const p2p::bf16*>(gy), P, C, eps,
                       static_cast<p2p::bf16*>(out), mp);
  return (int)hipGetLastError();
}

int p2p_pixel_shuffle(const void* in, int N, int OH, int OW, int OC, int r, int dir, void* out,
                      hipStream_t st) {
  const long n = (long)N * OH * OW * OC;
  hipLaunchKernelGGL(p2p::pixel_shuffle_kernel, dim3(p2p::mgrid(n)), dim3(256), 0, st,
                     static_cast<const p2p::bf16*>(in), N, OH, OW, OC, r, dir, static_cast<p2p::bf16*>(out));
  return (int)hipGetLastError();
}

int p2p_vec_pad(const float* x, int n, float fill, int nout, float* out, hipStream_t st) {
  hipLaunchKernelGGL(p2p::vec_pad_kernel, dim3((nout + 255) / 256), dim3(256), 0, st, x, n, fill, nout, out);
  return (int)hipGetLastError();
}

int p2p_col_weight(const void* w, int T, int C, int Cv, int Cvp, int Ncol, void* out, hipStream_t st) {
  const long n = (long)Ncol * C;
  hipLaunchKernelGGL(p2p::col_weight_kernel, dim3(p2p::mgrid(n)), dim3(256), 0, st, static_cast<const p2p::bf16*>(w),
                     T, C, Cv, Cvp, Ncol, static_cast<p2p::bf16*>(out));
  return (int)hipGetLastError();
}

int p2p_up2_dgrad_image(const float* w, int Cout, int Cin, int Xp, int Yp, void* out, hipStream_t st) {
  if (Xp < Cin || Yp < Cout) return -2;
  const long n = (long)Xp * 16 * Yp;
  hipLaunchKernelGGL(p2p::up2_dgrad_image_kernel, dim3(p2p::mgrid(n)), dim3(256), 0, st, w, Cout, Cin, Xp, Yp,
                     static_cast<p2p::bf16*>(out));
  return (int)hipGetLastError();
}

}  // extern "C"

// ---------------------------------------------------------------- bounds-check registry
// (P2P_BOUNDS_ASSERT build: every translation unit that includes bounds.h registers the host
// reader of its own device counters here; see csrc/bounds.h)
namespace p2p {
// positive control of the counters: one index past the end (site 99); a no-op in the normal build
__global__ void oob_selftest_kernel(int* out) {
  if (P2P_OOB_OK(99, 1, 1, 1)) out[0] = 1;
}
}  // namespace p2p
extern "C" int p2p_oob_selftest(void* scratch, hipStream_t st) {
  hipLaunchKernelGGL(p2p::oob_selftest_kernel, dim3(1), dim3(1), 0, st, static_cast<int*>(scratch));
  return (int)hipGetLastError();
}
#ifdef P2P_BOUNDS_ASSERT
namespace p2p {
static OobReader g_oob_readers[64];
static int g_oob_nreaders = 0;
int oob_register(OobReader fn) {
  if (g_oob_nreaders < 64) g_oob_readers[g_oob_nreaders++] = fn;
  return g_oob_nreaders;
}
}  // namespace p2p
extern "C" int p2p_oob_counts(unsigned int* out4, int reset) {
  out4[0] = out4[1] = out4[2] = out4[3] = 0;
  (void)hipDeviceSynchronize();
  for (int i = 0; i < p2p::g_oob_nreaders; ++i) p2p::g_oob_readers[i](out4, reset != 0);
  return 1;
}
#else
extern "C" int p2p_oob_counts(unsigned int* out4, int) {
  out4[0] = out4[1] = out4[2] = out4[3] = 0;
  return 0;
}
#endif
