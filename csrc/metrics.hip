// Evaluation metrics on the device (gfx950): per-image PSNR and SSIM of two image batches
// in one pass, replacing the reference's host round trip (train.py:54-65 `ssim`/`psnr`
// through numpy + skimage, 4 D2H copies per image, :477-482).
//
// Semantics (skimage structural_similarity, 7x7 uniform window, sample covariance, mean
// over the valid window positions of every channel; PSNR = 10 log10(255^2 / MSE)) on the
// uint8 levels floor(clamp(255 * x, 0, 255)) the reference's tensor2np produces.
//
// The levels are integers, so every window moment (sum x, sum x^2, sum xy, ...) is an
// exact int32 (49 * 255^2 < 2^22): the 7x7 box sums are exact and separable (horizontal
// 7-sums into LDS, then vertical), and only the per-window SSIM ratio is evaluated in
// double -- the result matches the float64 skimage computation to ~1e-15.  Per-block
// partials go to a workspace reduced in a fixed order (bitwise reproducible).
//
// Tiling: one workgroup = one channel x 16 rows x 64 columns of window origins; it stages
// the 22 x 70 input levels (origins + 6-pixel halo) and owns the 16 x 64 input pixels of
// the same rectangle for the PSNR sum.
#include "common.h"

namespace p2p {

constexpr int MT_H = 16, MT_W = 64, MT_WIN = 7;
constexpr int MT_IH = MT_H + MT_WIN - 1, MT_IW = MT_W + MT_WIN - 1;

struct MetricArgs {
  const void* a;
  const void* b;
  long sn, sc, sh, sw;    // element strides (n, c, h, w) of a
  long tn, tc, th, tw;    // ... and of b
  int N, C, H, W, shift, tiles_h, tiles_w;
  double c1, c2;
  double* ws;             // [N][C * tiles_h * tiles_w][2] = (ssim sum, squared-error sum)
};

template <typename T>
__device__ __forceinline__ int level(T v, int shift) {
  float f = (float)v;
  if (shift) f = (f + 1.0f) * 0.5f;
  return (int)floorf(fminf(fmaxf(f * 255.0f, 0.0f), 255.0f));
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__global__ void __launch_bounds__(256) image_metrics_kernel(MetricArgs m) {
  __shared__ int lx[MT_IH][MT_IW], ly[MT_IH][MT_IW];
  __shared__ int hs[5][MT_IH][MT_W];
  __shared__ double red[2][4];
  const int tid = threadIdx.x;
  const int n = blockIdx.z, c = blockIdx.y / m.tiles_h, ty = blockIdx.y % m.tiles_h;
  const int r0 = ty * MT_H, c0 = blockIdx.x * MT_W;
  const T* A = static_cast<const T*>(m.a) + n * m.sn + c * m.sc;
  const T* B = static_cast<const T*>(m.b) + n * m.tn + c * m.tc;

  long sse = 0;
  for (int e = tid; e < MT_IH * MT_IW; e += 256) {
    const int i = e / MT_IW, j = e % MT_IW, y = r0 + i, x = c0 + j;
    int va = 0, vb = 0;
    if (y < m.H && x < m.W) {
      va = level(A[y * m.sh + x * m.sw], m.shift);
      vb = level(B[y * m.th + x * m.tw], m.shift);
      if (i < MT_H && j < MT_W) sse += (va - vb) * (va - vb);
    }
    lx[i][j] = va;
    ly[i][j] = vb;
  }
  __syncthreads();
  // horizontal 7-sums of x, y, x^2, y^2, xy (halo columns past W are zeros and only feed
  // origins that are not valid windows)
  for (int e = tid; e < MT_IH * MT_W; e += 256) {
    const int i = e / MT_W, j = e % MT_W;
    int s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0;
#pragma unroll
    for (int t = 0; t < MT_WIN; ++t) {
      const int u = lx[i][j + t], v = ly[i][j + t];
      s0 += u; s1 += v; s2 += u * u; s3 += v * v; s4 += u * v;
    }
    hs[0][i][j] = s0; hs[1][i][j] = s1; hs[2][i][j] = s2; hs[3][i][j] = s3; hs[4][i][j] = s4;
  }
  __syncthreads();
  const double inv = 1.0 / (MT_WIN * MT_WIN);
  const double cov = (double)(MT_WIN * MT_WIN) / (MT_WIN * MT_WIN - 1);
  double acc = 0.0;
  for (int e = tid; e < MT_H * MT_W; e += 256) {
    const int i = e / MT_W, j = e % MT_W;
    if (r0 + i > m.H - MT_WIN || c0 + j > m.W - MT_WIN) continue;
    int s[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < MT_WIN; ++t)
#pragma unroll
      for (int q = 0; q < 5; ++q) s[q] += hs[q][i + t][j];
    const double ux = s[0] * inv, uy = s[1] * inv;
    const double vx = cov * (s[2] * inv - ux * ux), vy = cov * (s[3] * inv - uy * uy);
    const double vxy = cov * (s[4] * inv - ux * uy);
    acc += ((2.0 * ux * uy + m.c1) * (2.0 * vxy + m.c2)) /
           ((ux * ux + uy * uy + m.c1) * (vx + vy + m.c2));
  }
  acc = wave_sum_d(acc);
  const double se = wave_sum_d((double)sse);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = acc;
    red[1][tid >> 6] = se;
  }
  __syncthreads();
  if (tid == 0) {
    const long blk = ((long)c * m.tiles_h + ty) * m.tiles_w + blockIdx.x;
    double* o = m.ws + ((long)n * m.C * m.tiles_h * m.tiles_w + blk) * 2;
    o[0] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    o[1] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
  }
}

}  // namespace p2p

// dtype: 0 = fp32, 1 = bf16.  strides[8] = (n, c, h, w) of a, then of b.
extern "C" int p2p_metrics_ws(int C, int H, int W) {
  return C * ((H + p2p::MT_H - 1) / p2p::MT_H) * ((W + p2p::MT_W - 1) / p2p::MT_W);
}

extern "C" int p2p_image_metrics(const void* a, const void* b, int dtype, const long* strides, int N, int C,
                                 int H, int W, int shift, double data_range, double* ws, hipStream_t st) {
  if (H < p2p::MT_WIN || W < p2p::MT_WIN || N < 1 || C < 1 || N > 65535) return -1;
  p2p::MetricArgs m{};
  m.a = a;
  m.b = b;
  m.sn = strides[0]; m.sc = strides[1]; m.sh = strides[2]; m.sw = strides[3];
  m.tn = strides[4]; m.tc = strides[5]; m.th = strides[6]; m.tw = strides[7];
  m.N = N; m.C = C; m.H = H; m.W = W; m.shift = shift;
  m.tiles_h = (H + p2p::MT_H - 1) / p2p::MT_H;
  m.tiles_w = (W + p2p::MT_W - 1) / p2p::MT_W;
  m.c1 = (0.01 * data_range) * (0.01 * data_range);
  m.c2 = (0.03 * data_range) * (0.03 * data_range);
  m.ws = ws;
  if ((long)C * m.tiles_h > 65535) return -1;
  const dim3 grid(m.tiles_w, C * m.tiles_h, N);
  if (dtype == 1)
    hipLaunchKernelGGL(p2p::image_metrics_kernel<p2p::bf16>, grid, dim3(256), 0, st, m);
  else
    hipLaunchKernelGGL(p2p::image_metrics_kernel<float>, grid, dim3(256), 0, st, m);
  return (int)hipGetLastError();
}
