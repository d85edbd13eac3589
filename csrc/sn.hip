// Spectral-norm power iteration (reference networks.py:525-549, SpectralNorm._update_u_v):
//   v = l2n(W^T u),  u = l2n(W v),  sigma = u . (W v),   l2n(x) = x / (||x|| + 1e-12)
// on the fp32 master W viewed as [h][wd] (h = out channels, wd = in*kh*kw), updating u / v
// in place.  Four short launches, every reduction in a fixed order (bitwise repeatable):
//   1. tpart[rc][c] = sum_{r in row chunk rc} W[r][c] u[r]     grid (wd/256, RC): coalesced rows
//   2. t[c] = sum_rc tpart[rc][c], per-block sum t^2           grid (wd/256)
//   3. v = t / (||t|| + eps)  (v written),  s[r] = W[r] . v  (one wave per row), per-block sum s^2
//   4. u = s / (||s|| + eps)  (u written),  sigma = u . s
// The gradient of sigma w.r.t. W is u v^T (u, v constants), applied by the autograd Function.
#include "common.h"

namespace p2p {

constexpr int SN_RC = 8;      // row chunks of pass 1
constexpr float SN_EPS = 1e-12f;

__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = warp_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  __syncthreads();
  return s;
}

__global__ void __launch_bounds__(256) sn_wtu_kernel(const float* __restrict__ W, int h, int wd,
                                                     const float* __restrict__ u, float* __restrict__ tpart) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int rc = blockIdx.y;
  const int r0 = (int)((long)h * rc / SN_RC), r1 = (int)((long)h * (rc + 1) / SN_RC);
  if (c >= wd) return;
  float acc = 0.f;
  for (int r = r0; r < r1; ++r) acc += W[(long)r * wd + c] * u[r];
  tpart[(long)rc * wd + c] = acc;
}

__global__ void __launch_bounds__(256) sn_tsum_kernel(const float* __restrict__ tpart, int wd, float* __restrict__ t,
                                                      float* __restrict__ part) {
  __shared__ float red[4];
  const int c = blockIdx.x * 256 + threadIdx.x;
  float v = 0.f;
  if (c < wd) {
#pragma unroll
    for (int rc = 0; rc < SN_RC; ++rc) v += tpart[(long)rc * wd + c];
    t[c] = v;
  }
  const float s = block_sum256(v * v, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ void __launch_bounds__(256) sn_wv_kernel(const float* __restrict__ W, int h, int wd,
                                                    const float* __restrict__ t, const float* __restrict__ tpart_sq,
                                                    int nt, float* __restrict__ v, float* __restrict__ s,
                                                    float* __restrict__ part) {
  __shared__ float red[4];
  float n2 = 0.f;
  for (int i = 0; i < nt; ++i) n2 += tpart_sq[i];
  const float inv = 1.f / (sqrtf(n2) + SN_EPS);
  if (blockIdx.x == 0)
    for (int c = threadIdx.x; c < wd; c += 256) v[c] = t[c] * inv;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = blockIdx.x * 4 + wid;
  float acc = 0.f;
  if (r < h) {
    const float* row = W + (long)r * wd;
    for (int c = lane; c < wd; c += 64) acc += row[c] * (t[c] * inv);
    acc = warp_sum(acc);
    if (lane == 0) s[r] = acc;
  }
  const float sq = block_sum256(lane == 0 && r < h ? acc * acc : 0.f, red);
  if (threadIdx.x == 0) part[blockIdx.x] = sq;
}

__global__ void __launch_bounds__(256) sn_finish_kernel(const float* __restrict__ s, int h,
                                                        const float* __restrict__ spart, int ns,
                                                        float* __restrict__ u, float* __restrict__ sigma,
                                                        float* __restrict__ scale) {
  __shared__ float red[4];
  float n2 = 0.f;
  for (int i = 0; i < ns; ++i) n2 += spart[i];
  const float inv = 1.f / (sqrtf(n2) + SN_EPS);
  float dot = 0.f;
  for (int r = threadIdx.x; r < h; r += 256) {
    const float ur = s[r] * inv;
    u[r] = ur;
    dot += ur * s[r];
  }
  dot = block_sum256(dot, red);
  if (threadIdx.x == 0) {
    sigma[0] = dot;
    if (scale) scale[0] = 1.f / dot;   // the conv epilogues' 1 / sigma
  }
}

// Fused weight_bar gradient of a spectral-norm conv y = conv(x, s * W), s = 1 / sigma,
// sigma = u^T W v (u, v constants): from the conv's weight gradient G = dL/d(sW),
//   dL/dW = s G - <G, W> s^2 u v^T
// (the direct term plus the one through sigma) -- one dot pass, one elementwise pass.
__global__ void __launch_bounds__(256) sn_dot_kernel(const float* __restrict__ G, const float* __restrict__ W,
                                                     long n, float* __restrict__ part) {
  __shared__ float red[4];
  float a = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) a += G[i] * W[i];
  a = block_sum256(a, red);
  if (threadIdx.x == 0) part[blockIdx.x] = a;
}

__global__ void __launch_bounds__(256) sn_grad_kernel(const float* __restrict__ G, const float* __restrict__ u,
                                                      const float* __restrict__ v, const float* __restrict__ scale,
                                                      const float* __restrict__ part, int np, int h, int wd,
                                                      float* __restrict__ out, int accumulate) {
  __shared__ float dsh;
  if (threadIdx.x == 0) {
    float d = 0.f;
    for (int i = 0; i < np; ++i) d += part[i];   // fixed order: bitwise repeatable
    dsh = d;
  }
  __syncthreads();
  const float sc = scale[0];
  const float k = dsh * sc * sc;
  const long n = (long)h * wd;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int r = (int)(i / wd);
    const int c = (int)(i - (long)r * wd);
    const float g = sc * G[i] - k * u[r] * v[c];
    out[i] = accumulate ? out[i] + g : g;   // accumulate: a later contribution of one backward
  }
}

}  // namespace p2p

extern "C" {
// workspace floats: SN_RC*wd (tpart) + wd (t) + nt + h (s) + ns
long p2p_sn_ws_floats(int h, int wd) {
  const int nt = (wd + 255) / 256, ns = (h + 3) / 4;
  return (long)p2p::SN_RC * wd + wd + nt + h + ns;
}

int p2p_sn_power_iter(const float* W, int h, int wd, float* u, float* v, float* sigma, float* ws,
                      float* scale, hipStream_t st) {
  using namespace p2p;
  const int nt = (wd + 255) / 256, ns = (h + 3) / 4;
  float* tpart = ws;
  float* t = tpart + (long)SN_RC * wd;
  float* tsq = t + wd;
  float* s = tsq + nt;
  float* ssq = s + h;
  hipLaunchKernelGGL(sn_wtu_kernel, dim3(nt, SN_RC), dim3(256), 0, st, W, h, wd, u, tpart);
  hipLaunchKernelGGL(sn_tsum_kernel, dim3(nt), dim3(256), 0, st, tpart, wd, t, tsq);
  hipLaunchKernelGGL(sn_wv_kernel, dim3(ns), dim3(256), 0, st, W, h, wd, t, tsq, nt, v, s, ssq);
  hipLaunchKernelGGL(sn_finish_kernel, dim3(1), dim3(256), 0, st, s, h, ssq, ns, u, sigma, scale);
  return (int)hipGetLastError();
}

int p2p_sn_wgrad_blocks(long n) {
  long b = (n + 4095) / 4096;
  return (int)(b < 1 ? 1 : (b > 256 ? 256 : b));
}

// part: p2p_sn_wgrad_blocks(h * wd) floats
int p2p_sn_wgrad(const float* G, const float* W, const float* u, const float* v, const float* scale, int h,
                 int wd, float* part, float* out, int accumulate, hipStream_t st) {
  using namespace p2p;
  const long n = (long)h * wd;
  const int nb = p2p_sn_wgrad_blocks(n);
  hipLaunchKernelGGL(sn_dot_kernel, dim3(nb), dim3(256), 0, st, G, W, n, part);
  hipLaunchKernelGGL(sn_grad_kernel, dim3(nb), dim3(256), 0, st, G, u, v, scale, part, nb, h, wd, out, accumulate);
  return (int)hipGetLastError();
}
}
