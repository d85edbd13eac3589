// Instance / batch normalisation over NHWC bf16 activations (gfx950).
//
// Both norms are the same three-kernel pipeline with a different reduction domain:
//   IN : one group per (sample n, channel c), reduced over the H*W pixels of n
//   BN : one group per channel, reduced over all N*H*W pixels  (host passes N=1, HW=N*H*W)
// Forward
//   1. norm_partial   grid (chunks, N): every block reduces a contiguous run of pixels of
//      one sample; each thread owns one 16-B channel chunk (8 channels, bf16x8 vector loads)
//      and accumulates shifted sums around a per-block pivot (the block's first pixel), so
//      E[x^2]-E[x]^2 cancellation never happens.  Block partials (mean_b, M2_b) -> workspace.
//   2. norm_finalize  one thread per (n, c): Chan's parallel merge of the block partials in
//      a fixed order (deterministic), biased variance, rstd; BN also updates running stats
//      with the unbiased variance (PyTorch semantics).
//   3. norm_apply     y = act((x - mean) * rstd * gamma + beta), 16-B loads/stores.
// Backward (dx = rstd*g*(dy - mean(dy) - xhat*mean(dy*xhat)), dgamma/dbeta for affine)
//   1. norm_bwd_partial : block partial sums of dy and dy*xhat (recomputed from x) -- ONE
//      pass serves dgamma/dbeta and dx (gamma is constant per channel, the finalize scales);
//      a fused shared-slope PReLU also reduces its slope gradient here
//   2. norm_bwd_finalize: per (n,c) coefficients; per-channel dgamma/dbeta (summed over n)
//   3. norm_bwd_apply   : dx = A*dy + B + Cc*xhat
#include "fp8_dev.h"
#include <cstdlib>

namespace p2p {

struct NormGeom {
  int N, HW, C;   // groups: N x C; pixels per group: HW
  int chunk;      // pixels per block
  int nchunks;    // blocks per sample
};

// streaming 16-B accesses of the apply passes (every byte touched once per pass)
__device__ __forceinline__ u32x4 ld_stream(const bf16* p) { return *reinterpret_cast<const u32x4*>(p); }
__device__ __forceinline__ void st_stream(bf16* p, u32x4 v) { *reinterpret_cast<u32x4*>(p) = v; }

__device__ __forceinline__ void unpack8(u32x4 v, float* f) {
  bf16x8 b = __builtin_bit_cast(bf16x8, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (float)b[j];
}

__device__ __forceinline__ u32x4 pack8(const float* f) {
  bf16x8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = (bf16)f[j];
  return __builtin_bit_cast(u32x4, b);
}

// ---------------------------------------------------------------- forward
// ws layout: [N][nchunks][C] mean_b, then [N][nchunks][C] M2_b
__global__ void __launch_bounds__(256) norm_partial_kernel(const bf16* __restrict__ x, NormGeom g,
                                                           float* __restrict__ ws) {
  const int n = blockIdx.y, cb = blockIdx.x;
  const int CP = g.C >> 3;
  const int RP = 256 / CP;           // pixel rows processed per pass
  const int tid = threadIdx.x;
  const int cg = tid % CP, tr = tid / CP;
  const int p0 = cb * g.chunk;
  const int p1 = min(g.HW, p0 + g.chunk);
  const bf16* base = x + (long)n * g.HW * g.C;
  float piv[8], s1[8], s2[8];
  {
    u32x4 v = *reinterpret_cast<const u32x4*>(base + (long)p0 * g.C + cg * 8);
    unpack8(v, piv);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  if (tr < RP) {
    auto acc1 = [&](u32x4 v) {
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = f[j] - piv[j];
        s1[j] += d;
        s2[j] += d * d;
      }
    };
    int p = p0 + tr;
    for (; p + 3 * RP < p1; p += 4 * RP) {   // 4 independent 16-B loads in flight
      u32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = *reinterpret_cast<const u32x4*>(base + (long)(p + u * RP) * g.C + cg * 8);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc1(v[u]);
    }
    for (; p < p1; p += RP) acc1(*reinterpret_cast<const u32x4*>(base + (long)p * g.C + cg * 8));
  }
  // block reduce over rows sharing a channel chunk: LDS [RP][C] x 2
  __shared__ float red1[2048], red2[2048];
  const int rows_red = 2048 / g.C;   // rows that fit in the LDS buffer at once
  // every thread with tr < RP contributes; fold rows tr >= rows_red in a loop
  for (int base_r = 0; base_r < RP; base_r += rows_red) {
    if (tr >= base_r && tr < base_r + rows_red && tr < RP) {
      const int r = tr - base_r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (base_r == 0) {
          red1[r * g.C + cg * 8 + j] = s1[j];
          red2[r * g.C + cg * 8 + j] = s2[j];
        } else {
          red1[r * g.C + cg * 8 + j] += s1[j];
          red2[r * g.C + cg * 8 + j] += s2[j];
        }
      }
    }
    __syncthreads();
  }
  const int rr = min(RP, rows_red);
  const int npx = p1 - p0;
  for (int c = tid; c < g.C; c += 256) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < rr; ++r) {
      a += red1[r * g.C + c];
      b += red2[r * g.C + c];
    }
    const float pv = (float)base[(long)p0 * g.C + c];
    const float inv = 1.f / (float)npx;
    const float mb = pv + a * inv;
    const float m2 = fmaxf(b - a * a * inv, 0.f);
    const long o = ((long)n * g.nchunks + cb) * g.C + c;
    ws[o] = mb;
    ws[(long)g.N * g.nchunks * g.C + o] = m2;
  }
}

// Chunk-partial reductions (finalize passes): one block per (CT-channel tile, group n);
// thread (j, c) = (tid / CT, tid % CT) merges chunks j, j+J, j+2J, ... of channel c0 + c in
// order, then the J partial results merge through LDS in a fixed tree -- deterministic, and
// parallel over chunks (BN has ~1-2k chunks per channel: a thread-per-channel serial merge
// cost 300 us per call on the family-R step).
// CT channels x J chunk-lanes per block: (32, 8) for instance norm (few chunks per group),
// (8, 32) when a group has hundreds of chunks (batch norm over N*H*W pixels)

// Chan's merge of (cnt, mean, M2) partials
__device__ __forceinline__ void chan_merge(float& cA, float& mA, float& qA, float cB, float mB, float qB) {
  const float tot = cA + cB;
  if (tot <= 0.f) return;
  const float d = mB - mA;
  mA += d * (cB / tot);
  qA += qB + d * d * (cA * cB / tot);
  cA = tot;
}

// stats: [N][C] mean, [N][C] rstd (fp32).  bn: running stats update (N == 1).
template <int FIN_CT, int FIN_J>
__global__ void __launch_bounds__(256) norm_finalize_kernel(const float* __restrict__ ws, NormGeom g,
                                                            float eps, float* __restrict__ mean_out,
                                                            float* __restrict__ rstd_out,
                                                            float* __restrict__ run_mean,
                                                            float* __restrict__ run_var,
                                                            float momentum) {
  __shared__ float sc[FIN_J][FIN_CT], sm[FIN_J][FIN_CT], sq[FIN_J][FIN_CT];
  const int n = blockIdx.y;
  const int cl = threadIdx.x % FIN_CT, j = threadIdx.x / FIN_CT;
  const int c = blockIdx.x * FIN_CT + cl;
  float cntA = 0.f, meanA = 0.f, M2A = 0.f;
  if (c < g.C) {
    const float* mb = ws + (long)n * g.nchunks * g.C + c;
    const float* m2 = mb + (long)g.N * g.nchunks * g.C;
    for (int b = j; b < g.nchunks; b += FIN_J)
      chan_merge(cntA, meanA, M2A, (float)min(g.chunk, g.HW - b * g.chunk), mb[(long)b * g.C], m2[(long)b * g.C]);
  }
  sc[j][cl] = cntA;
  sm[j][cl] = meanA;
  sq[j][cl] = M2A;
  __syncthreads();
  for (int w = FIN_J / 2; w > 0; w >>= 1) {
    if (j < w) {
      float cA = sc[j][cl], mA = sm[j][cl], qA = sq[j][cl];
      chan_merge(cA, mA, qA, sc[j + w][cl], sm[j + w][cl], sq[j + w][cl]);
      sc[j][cl] = cA;
      sm[j][cl] = mA;
      sq[j][cl] = qA;
    }
    __syncthreads();
  }
  if (j == 0 && c < g.C) {
    cntA = sc[0][cl];
    meanA = sm[0][cl];
    M2A = sq[0][cl];
    const int i = n * g.C + c;
    const float var = M2A / cntA;
    mean_out[i] = meanA;
    rstd_out[i] = rsqrtf(var + eps);
    if (run_mean) {
      const float unb = cntA > 1.f ? M2A / (cntA - 1.f) : var;
      run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * meanA;
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
    }
  }
}

// sums of the two [N][nchunks][C] partial planes over chunks (and, ngroups > 1, over the
// groups n0 .. n0+ngroups-1): block-parallel, fixed order
template <int FIN_CT, int FIN_J>
__device__ __forceinline__ void chunk_sums(const float* __restrict__ ws, const NormGeom& g, int n0, int ngroups,
                                           int c, int j, float& sa, float& sb, float (*ra)[FIN_CT],
                                           float (*rb)[FIN_CT], int cl) {
  sa = 0.f;
  sb = 0.f;
  if (c < g.C)
    for (int n = n0; n < n0 + ngroups; ++n) {
      const float* a = ws + (long)n * g.nchunks * g.C + c;
      const float* b = a + (long)g.N * g.nchunks * g.C;
      for (int k = j; k < g.nchunks; k += FIN_J) {
        sa += a[(long)k * g.C];
        sb += b[(long)k * g.C];
      }
    }
  ra[j][cl] = sa;
  rb[j][cl] = sb;
  __syncthreads();
  for (int w = FIN_J / 2; w > 0; w >>= 1) {
    if (j < w) {
      ra[j][cl] += ra[j + w][cl];
      rb[j][cl] += rb[j + w][cl];
    }
    __syncthreads();
  }
  sa = ra[0][cl];
  sb = rb[0][cl];
}

// The activation is a template parameter of the element-wise kernels: a runtime code,
// even a wave-uniform one, costs a compare + branch per element (measured on the conv
// epilogue: 6 % of the whole training step).  ACT_PRELU_T: the shared-slope PReLU.
constexpr int ACT_PRELU_T = 5;

template <typename F>
static void with_act(int act, F&& f) {
  switch (act) {
    case ACT_RELU: f(std::integral_constant<int, ACT_RELU>{}); break;
    case ACT_LRELU: f(std::integral_constant<int, ACT_LRELU>{}); break;
    case ACT_TANH: f(std::integral_constant<int, ACT_TANH>{}); break;
    case ACT_SIGMOID: f(std::integral_constant<int, ACT_SIGMOID>{}); break;
    case ACT_PRELU_T: f(std::integral_constant<int, ACT_PRELU_T>{}); break;
    default: f(std::integral_constant<int, ACT_NONE>{}); break;
  }
}

// y = act((x - mean) * rstd * gamma + beta [+ res]); mean/rstd indexed [n][c] (BN: n == 0
// always).  res (optional, x's shape): a residual added BEFORE the activation -- the family-R
// residual block's relu(BN(conv(.)) + x) in this one pass instead of an apply pass plus an
// add+act pass.  grid (chunks, N): each thread owns one 8-channel chunk (its 8 scale/shift
// pairs live in registers) and strides over the block's pixels.
template <int ACT>
__global__ void __launch_bounds__(256) norm_apply_kernel(const bf16* __restrict__ x, NormGeom g,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ rstd,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta,
                                                         const float* __restrict__ prelu_w,
                                                         bf16* __restrict__ y, Fp8Shadow sh,
                                                         const bf16* __restrict__ res) {
  const int n = blockIdx.y, cb = blockIdx.x;
  const int CP = g.C >> 3;
  const int RP = 256 / CP;
  const int tid = threadIdx.x;
  const int cg = tid % CP, tr = tid / CP;
  if (tr >= RP) return;
  const int p0 = cb * g.chunk;
  const int p1 = min(g.HW, p0 + g.chunk);
  float sc[8], sf[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cg * 8 + j;
    const float r = rstd[(long)n * g.C + c];
    const float gm = gamma ? gamma[c] : 1.f;
    sc[j] = r * gm;
    sf[j] = (gamma ? beta[c] : 0.f) - mean[(long)n * g.C + c] * r * gm;
  }
  const float pw = prelu_w ? prelu_w[0] : 0.f;
  const long base = (long)n * g.HW * g.C + cg * 8;
  // optional fp8 shadow of y (the next conv's operand) written in the same pass
  const float qsc = sh.q ? fp8_shadow_scale(sh) : 0.f;
  float qmax = 0.f;
  auto one = [&](u32x4 v, u32x4 rv, long off) {
    float f[8], r8[8];
    unpack8(v, f);
    if (res) unpack8(rv, r8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = f[j] * sc[j] + sf[j];
      if (res) t += r8[j];
      if constexpr (ACT == ACT_PRELU_T) t = t > 0.f ? t : pw * t;
      else t = act_fwd(t, ACT);
      f[j] = t;
    }
    const u32x4 o = pack8(f);
    st_stream(y + off, o);
    if (sh.q) {
      float r[8];
      unpack8(o, r);   // quantise the stored bf16 value: shadow == fp8(y) exactly
#pragma unroll
      for (int j = 0; j < 8; ++j) qmax = fmaxf(qmax, fabsf(r[j]));
      *reinterpret_cast<uint2*>(sh.q + off) = fp8_pack8(r, qsc, sh.fmt);
    }
  };
  const u32x4 zero4 = {0u, 0u, 0u, 0u};   // +0.0 bf16 x 8
  int p = p0 + tr;
  for (; p + 3 * RP < p1; p += 4 * RP) {
    u32x4 v[4], rv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      v[u] = ld_stream(x + base + (long)(p + u * RP) * g.C);
      rv[u] = res ? ld_stream(res + base + (long)(p + u * RP) * g.C) : zero4;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) one(v[u], rv[u], base + (long)(p + u * RP) * g.C);
  }
  for (; p < p1; p += RP)
    one(ld_stream(x + base + (long)p * g.C), res ? ld_stream(res + base + (long)p * g.C) : zero4,
        base + (long)p * g.C);
  if (sh.q) fp8_amax_commit(qmax, sh.site);
}

// ---------------------------------------------------------------- backward
// The forward may have fused an activation: y = act(z), z = xhat*gamma + beta.  For ReLU /
// LeakyReLU the backward recomputes z from x and the saved statistics, so the act' gate
// (dy_eff = dy * act'(z)) costs no extra pass over memory.  Tanh / sigmoid (family-R
// output layer only) go through the separate act kernel before this one.
__device__ __forceinline__ float act_gate(float z, int act, float pw) {
  if (act == ACT_RELU) return z > 0.f ? 1.f : 0.f;
  if (act == ACT_LRELU) return z > 0.f ? 1.f : LRELU_SLOPE;
  if (act == ACT_PRELU_T) return z > 0.f ? 1.f : pw;
  return 1.f;
}

// block reduction of per-thread [8]-channel partials over the RP pixel rows -> out[c]
__device__ __forceinline__ void block_rows_reduce(const float* s1, const float* s2, int C, int cg,
                                                  int tr, int RP, float* red1, float* red2,
                                                  float* out1, float* out2) {
  const int tid = threadIdx.x;
  const int rows_red = 2048 / C;
  for (int base_r = 0; base_r < RP; base_r += rows_red) {
    if (tr >= base_r && tr < base_r + rows_red && tr < RP) {
      const int r = tr - base_r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (base_r == 0) {
          red1[r * C + cg * 8 + j] = s1[j];
          if (s2) red2[r * C + cg * 8 + j] = s2[j];
        } else {
          red1[r * C + cg * 8 + j] += s1[j];
          if (s2) red2[r * C + cg * 8 + j] += s2[j];
        }
      }
    }
    __syncthreads();
  }
  const int rr = min(RP, rows_red);
  for (int c = tid; c < C; c += 256) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < rr; ++r) {
      a += red1[r * C + c];
      if (s2) b += red2[r * C + c];
    }
    out1[c] = a;
    if (s2) out2[c] = b;
  }
}

// ws: [N][nchunks][C] sum(dy_eff), [N][nchunks][C] sum(dy_eff * xhat); PReLU: pws[n][chunk]
// = sum(dy * z * [z <= 0]) over the block (the slope gradient, deterministic block order)
template <int ACT>
__global__ void __launch_bounds__(256) norm_bwd_partial_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ dy, NormGeom g,
    const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, const float* __restrict__ prelu_w, float* __restrict__ ws,
    float* __restrict__ pws) {
  const int n = blockIdx.y, cb = blockIdx.x;
  const int CP = g.C >> 3;
  const int RP = 256 / CP;
  const int tid = threadIdx.x;
  const int cg = tid % CP, tr = tid / CP;
  const int p0 = cb * g.chunk;
  const int p1 = min(g.HW, p0 + g.chunk);
  const long off = (long)n * g.HW * g.C + cg * 8;
  float mu[8], rs[8], ga[8], be[8], s1[8], s2[8];
  float s3 = 0.f;
  const float pw = ACT == ACT_PRELU_T ? prelu_w[0] : 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = mean[(long)n * g.C + cg * 8 + j];
    rs[j] = rstd[(long)n * g.C + cg * 8 + j];
    ga[j] = gamma ? gamma[cg * 8 + j] : 1.f;
    be[j] = gamma ? beta[cg * 8 + j] : 0.f;
    s1[j] = s2[j] = 0.f;
  }
  if (tr < RP) {
    auto acc2 = [&](u32x4 vx, u32x4 vd) {
      float fx[8], fd[8];
      unpack8(vx, fx);
      unpack8(vd, fd);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (fx[j] - mu[j]) * rs[j];
        const float z = xh * ga[j] + be[j];
        if constexpr (ACT == ACT_PRELU_T) s3 += z <= 0.f ? fd[j] * z : 0.f;
        const float d = fd[j] * act_gate(z, ACT, pw);
        s1[j] += d;
        s2[j] += d * xh;
      }
    };
    int p = p0 + tr;
    for (; p + 3 * RP < p1; p += 4 * RP) {
      u32x4 vx[4], vd[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        vx[u] = *reinterpret_cast<const u32x4*>(x + off + (long)(p + u * RP) * g.C);
        vd[u] = *reinterpret_cast<const u32x4*>(dy + off + (long)(p + u * RP) * g.C);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc2(vx[u], vd[u]);
    }
    for (; p < p1; p += RP)
      acc2(*reinterpret_cast<const u32x4*>(x + off + (long)p * g.C),
           *reinterpret_cast<const u32x4*>(dy + off + (long)p * g.C));
  }
  __shared__ float red1[2048], red2[2048];
  __shared__ float o1[2048], o2[2048];
  block_rows_reduce(s1, s2, g.C, cg, tr, RP, red1, red2, o1, o2);
  __syncthreads();
  for (int c = tid; c < g.C; c += 256) {
    const long o = ((long)n * g.nchunks + cb) * g.C + c;
    ws[o] = o1[c];
    ws[(long)g.N * g.nchunks * g.C + o] = o2[c];
  }
  if constexpr (ACT == ACT_PRELU_T) {
    // fixed-order block reduction of the slope partial: wave shuffles, then 4 wave sums
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s3 += __shfl_xor(s3, m);
    __syncthreads();
    if ((tid & 63) == 0) red1[tid >> 6] = s3;
    __syncthreads();
    if (tid == 0) pws[(long)n * g.nchunks + cb] = (red1[0] + red1[1]) + (red1[2] + red1[3]);
  }
}

// coef: [N][C] A, [N][C] B, [N][C] Cc  with dx = A*dy_eff + B + Cc*xhat
template <int FIN_CT, int FIN_J>
__global__ void __launch_bounds__(256) norm_bwd_finalize_kernel(const float* __restrict__ ws,
                                                                NormGeom g,
                                                                const float* __restrict__ rstd,
                                                                const float* __restrict__ gamma,
                                                                float* __restrict__ coef) {
  __shared__ float ra[FIN_J][FIN_CT], rb[FIN_J][FIN_CT];
  const int n = blockIdx.y;
  const int cl = threadIdx.x % FIN_CT, j = threadIdx.x / FIN_CT;
  const int c = blockIdx.x * FIN_CT + cl;
  float sdy, sdx;
  chunk_sums<FIN_CT, FIN_J>(ws, g, n, 1, c, j, sdy, sdx, ra, rb, cl);
  if (j != 0 || c >= g.C) return;
  const int i = n * g.C + c;
  const float r = rstd[i];
  const float inv = 1.f / (float)g.HW;
  const float ga = gamma ? gamma[c] : 1.f;
  const long NC = (long)g.N * g.C;
  coef[i] = r * ga;
  coef[NC + i] = -r * ga * sdy * inv;   // partial sums are of the un-scaled dy_eff
  coef[2 * NC + i] = -r * ga * sdx * inv;
}

// eval-mode (frozen statistics) backward: x -> xhat is a fixed affine map, so
// dx = rstd * gamma * dy_eff (no mean terms) -- the apply kernel with B = Cc = 0
__global__ void __launch_bounds__(256) norm_frozen_coef_kernel(int NC, int C, const float* __restrict__ rstd,
                                                               const float* __restrict__ gamma,
                                                               float* __restrict__ coef) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= NC) return;
  coef[i] = rstd[i] * (gamma ? gamma[i % C] : 1.f);
  coef[NC + i] = 0.f;
  coef[2 * NC + i] = 0.f;
}

// d(gamma) = sum(dy_eff * xhat), d(beta) = sum(dy_eff) over every group of the channel
// (stored, not accumulated: one launch per norm backward writes every channel once, so the
// caller hands uninitialised buffers -- no zero fill per norm)
template <int FIN_CT, int FIN_J>
__global__ void __launch_bounds__(256) norm_param_grad_kernel(const float* __restrict__ ws, NormGeom g,
                                                              float* __restrict__ dgamma,
                                                              float* __restrict__ dbeta) {
  __shared__ float ra[FIN_J][FIN_CT], rb[FIN_J][FIN_CT];
  const int cl = threadIdx.x % FIN_CT, j = threadIdx.x / FIN_CT;
  const int c = blockIdx.x * FIN_CT + cl;
  float sdy, sdx;
  chunk_sums<FIN_CT, FIN_J>(ws, g, 0, g.N, c, j, sdy, sdx, ra, rb, cl);
  if (j != 0 || c >= g.C) return;
  dgamma[c] = sdx;
  dbeta[c] = sdy;
}

// dx = A*dy_eff + B + Cc*xhat.  (The column sums of dx -- the bias gradient of the conv
// that produced x -- are exactly zero for a normalised group: sum_p dx = Cc * sum_p xhat = 0,
// so the host returns that exact zero instead of re-reading dx.)
template <int ACT>
__global__ void __launch_bounds__(256) norm_bwd_apply_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ dy, NormGeom g,
    const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, const float* __restrict__ prelu_w, const float* __restrict__ coef,
    bf16* __restrict__ dx, Fp8Shadow sh) {
  const int n = blockIdx.y, cb = blockIdx.x;
  const int CP = g.C >> 3;
  const int RP = 256 / CP;
  const int tid = threadIdx.x;
  const int cg = tid % CP, tr = tid / CP;
  if (tr >= RP) return;
  const int p0 = cb * g.chunk;
  const int p1 = min(g.HW, p0 + g.chunk);
  const long NC = (long)g.N * g.C;
  // per channel, folded once: z = x * zs + zb (the fused activation's input), and
  // dx = ca * dy_eff + k0 + k1 * x (= ca * dy_eff + c0 + cx * xhat): five registers per
  // channel instead of seven, two fewer VALU per element
  float ca[8], k0[8], k1[8], zs[8], zb[8];
  const float pw = ACT == ACT_PRELU_T ? prelu_w[0] : 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const long ci = (long)n * g.C + cg * 8 + j;
    const float mu = mean[ci], rs = rstd[ci];
    const float ga = gamma ? gamma[cg * 8 + j] : 1.f;
    const float be = gamma ? beta[cg * 8 + j] : 0.f;
    const float cx = coef[2 * NC + ci];
    ca[j] = coef[ci];
    k1[j] = cx * rs;
    k0[j] = coef[NC + ci] - k1[j] * mu;
    zs[j] = rs * ga;
    zb[j] = be - mu * zs[j];
  }
  const long base = (long)n * g.HW * g.C + cg * 8;
  // optional fp8 (e5m2) shadow of dx: the producing conv's dgrad operand
  const float qsc = sh.q ? fp8_shadow_scale(sh) : 0.f;
  float qmax = 0.f;
  auto one = [&](u32x4 vx, u32x4 vd, long off) {
    float fx[8], fd[8];
    unpack8(vx, fx);
    unpack8(vd, fd);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = ACT ? fd[j] * act_gate(fmaf(fx[j], zs[j], zb[j]), ACT, pw) : fd[j];
      fd[j] = fmaf(ca[j], d, fmaf(k1[j], fx[j], k0[j]));
    }
    const u32x4 o = pack8(fd);
    st_stream(dx + off, o);
    if (sh.q) {
      float r[8];
      unpack8(o, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) qmax = fmaxf(qmax, fabsf(r[j]));
      *reinterpret_cast<uint2*>(sh.q + off) = fp8_pack8(r, qsc, sh.fmt);
    }
  };
  int p = p0 + tr;
  for (; p + 3 * RP < p1; p += 4 * RP) {
    u32x4 vx[4], vd[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      vx[u] = ld_stream(x + base + (long)(p + u * RP) * g.C);
      vd[u] = ld_stream(dy + base + (long)(p + u * RP) * g.C);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) one(vx[u], vd[u], base + (long)(p + u * RP) * g.C);
  }
  for (; p < p1; p += RP)
    one(ld_stream(x + base + (long)p * g.C), ld_stream(dy + base + (long)p * g.C),
        base + (long)p * g.C);
  if (sh.q) fp8_amax_commit(qmax, sh.site);
}

// finalize-pass launches: many chunks per group -> 8 channels x 32 chunk-lanes per block;
// batch norm over N*H*W (thousands of chunks per channel) -> one channel x 256 chunk-lanes
// per block (the merge was latency-bound: 64 dependent merges per lane, 16 blocks busy)
static inline bool fin_wide(const NormGeom& g) { return g.nchunks >= 64; }
static inline bool fin_huge(const NormGeom& g) { return g.nchunks >= 512; }

// launch a finalize-style kernel with the (channels, chunk-lanes) split chosen by nchunks
#define P2P_FIN_LAUNCH(KERNEL, g, ny, st, ...)                                                            \
  do {                                                                                                   \
    if (fin_huge(g))                                                                                     \
      hipLaunchKernelGGL((KERNEL<1, 256>), dim3((g).C, ny), dim3(256), 0, st, __VA_ARGS__);              \
    else if (fin_wide(g))                                                                                \
      hipLaunchKernelGGL((KERNEL<8, 32>), dim3(((g).C + 7) / 8, ny), dim3(256), 0, st, __VA_ARGS__);     \
    else                                                                                                 \
      hipLaunchKernelGGL((KERNEL<32, 8>), dim3(((g).C + 31) / 32, ny), dim3(256), 0, st, __VA_ARGS__);   \
  } while (0)

static inline NormGeom make_geom(int N, int HW, int C) {
  NormGeom g;
  g.N = N;
  g.HW = HW;
  g.C = C;
  // ~2048 blocks of work: every thread walks `iters` pixels (4..64) of its 8-channel
  // column, RP = 256 / (C/8) columns' worth of pixel rows per pass
  const long total_px = (long)N * HW;
  const int RP = C >= 2048 ? 1 : 256 / (C >> 3);
  long iters = total_px / ((long)RP * 2048);
  iters = iters < 4 ? 4 : (iters > 64 ? 64 : iters);
  int chunk = (int)(RP * iters);
  if (chunk > HW) chunk = HW;
  g.chunk = chunk;
  g.nchunks = (HW + chunk - 1) / chunk;
  return g;
}

}  // namespace p2p

extern "C" {

int p2p_sum_partials(const float* ws, int nb, float scale, float* out, hipStream_t st);

// workspace floats needed by p2p_norm_fwd / p2p_norm_bwd (incl. the fused bias-grad partials)
long p2p_norm_ws_floats(int N, int HW, int C) {
  p2p::NormGeom g = p2p::make_geom(N, HW, C);
  return 2L * N * g.nchunks * C + 3L * N * C + (long)N * g.nchunks;
}

int p2p_norm_fwd(const void* x, int N, int HW, int C, float eps, const float* gamma,
                 const float* beta, const float* prelu_w, int act, float* mean, float* rstd,
                 float* run_mean, float* run_var, float momentum, float* ws, void* y,
                 void* q, int* qsite, int qfmt, const void* res, hipStream_t st) {
  using namespace p2p;
  NormGeom g = make_geom(N, HW, C);
  hipLaunchKernelGGL(norm_partial_kernel, dim3(g.nchunks, N), dim3(256), 0, st,
                     static_cast<const bf16*>(x), g, ws);
  P2P_FIN_LAUNCH(norm_finalize_kernel, g, N, st, ws, g, eps, mean, rstd, run_mean, run_var, momentum);
  if (y)
    with_act(prelu_w ? ACT_PRELU_T : act, [&](auto t) {
      hipLaunchKernelGGL((norm_apply_kernel<decltype(t)::value>), dim3(g.nchunks, N), dim3(256), 0, st,
                         static_cast<const bf16*>(x), g, mean, rstd, gamma, beta, prelu_w, static_cast<bf16*>(y),
                         Fp8Shadow{static_cast<uint8_t*>(q), qsite, qfmt}, static_cast<const bf16*>(res));
    });
  return (int)hipGetLastError();
}

// forward from per-chunk (mean, M2) partials produced by the conv epilogue (conv_dev.h):
// partials [2][N][nchunks][C], every chunk HW / nchunks pixels -- the read-only stats pass
// over x is gone; finalize merges, apply normalises.
int p2p_norm_fwd_partials(const void* x, int N, int HW, int C, int nchunks, const float* partials,
                          float eps, const float* gamma, const float* beta, const float* prelu_w,
                          int act, float* mean, float* rstd, float* run_mean, float* run_var,
                          float momentum, void* y, void* q, int* qsite, int qfmt, const void* res,
                          hipStream_t st) {
  using namespace p2p;
  if (nchunks <= 0 || HW % nchunks) return -1;
  NormGeom pg;
  pg.N = N;
  pg.HW = HW;
  pg.C = C;
  pg.chunk = HW / nchunks;
  pg.nchunks = nchunks;
  P2P_FIN_LAUNCH(norm_finalize_kernel, pg, N, st, partials, pg, eps, mean, rstd, run_mean, run_var, momentum);
  NormGeom g = make_geom(N, HW, C);
  with_act(prelu_w ? ACT_PRELU_T : act, [&](auto t) {
    hipLaunchKernelGGL((norm_apply_kernel<decltype(t)::value>), dim3(g.nchunks, N), dim3(256), 0, st,
                       static_cast<const bf16*>(x), g, mean, rstd, gamma, beta, prelu_w, static_cast<bf16*>(y),
                       Fp8Shadow{static_cast<uint8_t*>(q), qsite, qfmt}, static_cast<const bf16*>(res));
  });
  return (int)hipGetLastError();
}

// apply only (eval-mode BN with running stats: host passes mean/rstd computed from them)
int p2p_norm_apply(const void* x, int N, int HW, int C, const float* mean, const float* rstd,
                   const float* gamma, const float* beta, const float* prelu_w, int act, void* y,
                   const void* res, hipStream_t st) {
  using namespace p2p;
  NormGeom g = make_geom(N, HW, C);
  with_act(prelu_w ? ACT_PRELU_T : act, [&](auto t) {
    hipLaunchKernelGGL((norm_apply_kernel<decltype(t)::value>), dim3(g.nchunks, N), dim3(256), 0, st,
                       static_cast<const bf16*>(x), g, mean, rstd, gamma, beta, prelu_w, static_cast<bf16*>(y),
                       Fp8Shadow{nullptr, nullptr, 0}, static_cast<const bf16*>(res));
  });
  return (int)hipGetLastError();
}

// act: ReLU / LeakyReLU fused by the forward (0 = none); prelu_w: the fused shared-slope
// PReLU (its slope gradient -> *dprelu, written not accumulated); dsum (optional, [C] fp32):
// the column sums of dx (bias gradient of the producing conv), which are exactly zero.
int p2p_norm_bwd(const void* x, const void* dy, int N, int HW, int C, const float* mean,
                 const float* rstd, const float* gamma, const float* beta, int act,
                 const float* prelu_w, float* dprelu, float* dgamma, float* dbeta, float* ws, void* dx,
                 float* dsum, void* q, int* qsite, int qfmt, int frozen, hipStream_t st) {
  using namespace p2p;
  NormGeom g = make_geom(N, HW, C);
  float* coef = ws + 2L * N * g.nchunks * C;
  float* pws = coef + 3L * N * C;
  const bf16* xb = static_cast<const bf16*>(x);
  const bf16* db = static_cast<const bf16*>(dy);
  const int a = prelu_w ? ACT_PRELU_T : act;
  if (!dgamma && !dx && !dprelu) return 0;
  // frozen (eval-mode BN): the partial sums serve only the parameter / slope gradients
  if (!frozen || dgamma || dprelu) {
    with_act(a, [&](auto t) {
      hipLaunchKernelGGL((norm_bwd_partial_kernel<decltype(t)::value>), dim3(g.nchunks, N), dim3(256), 0, st, xb,
                         db, g, mean, rstd, gamma, beta, prelu_w, ws, pws);
    });
  }
  if (dprelu) {
    const int rc = p2p_sum_partials(pws, N * g.nchunks, 1.f, dprelu, st);
    if (rc) return rc;
  }
  if (dgamma) {
    if (fin_huge(g))
      hipLaunchKernelGGL((norm_param_grad_kernel<1, 256>), dim3(C), dim3(256), 0, st, ws, g, dgamma, dbeta);
    else if (fin_wide(g) || N > 8)
      hipLaunchKernelGGL((norm_param_grad_kernel<8, 32>), dim3((C + 7) / 8), dim3(256), 0, st, ws, g, dgamma, dbeta);
    else
      hipLaunchKernelGGL((norm_param_grad_kernel<32, 8>), dim3((C + 31) / 32), dim3(256), 0, st, ws, g, dgamma, dbeta);
  }
  if (dx) {
    if (frozen)
      hipLaunchKernelGGL(norm_frozen_coef_kernel, dim3((N * C + 255) / 256), dim3(256), 0, st, N * C, C, rstd, gamma,
                         coef);
    else
      P2P_FIN_LAUNCH(norm_bwd_finalize_kernel, g, N, st, ws, g, rstd, gamma, coef);
    with_act(a, [&](auto t) {
      hipLaunchKernelGGL((norm_bwd_apply_kernel<decltype(t)::value>), dim3(g.nchunks, N), dim3(256), 0, st, xb, db,
                         g, mean, rstd, gamma, beta, prelu_w, coef, static_cast<bf16*>(dx),
                         Fp8Shadow{static_cast<uint8_t*>(q), qsite, qfmt});
    });
    // a normalised group's dx sums to exactly zero (the producer's bias gradient); not so
    // under frozen statistics -- the caller computes that column sum itself
    if (dsum && !frozen) (void)hipMemsetAsync(dsum, 0, sizeof(float) * C, st);
  }
  return (int)hipGetLastError();
}

// backward from per-chunk partials [2][N][nchunks][C] of sum(d) / sum(d * xhat) produced by the
// consumer conv's dgrad epilogue (conv_dev.h nb_*): the partial pass over (x, dy) is gone;
// finalize (+ the affine parameter gradients) and apply as in p2p_norm_bwd.  coef: [3][N][C].
// prelu_w: the shared-slope PReLU of the forward (the apply pass gates with it; its slope
// gradient comes from the partials' third plane, summed by the caller)
int p2p_norm_bwd_partials(const void* x, const void* dy, int N, int HW, int C, int nchunks,
                          const float* partials, const float* mean, const float* rstd,
                          const float* gamma, const float* beta, int act, const float* prelu_w, float* dgamma,
                          float* dbeta, float* coef, void* dx, float* dsum, void* q, int* qsite, int qfmt,
                          hipStream_t st) {
  using namespace p2p;
  if (nchunks <= 0) return -1;   // (the backward's sums do not use the chunk size)
  NormGeom pg;
  pg.N = N;
  pg.HW = HW;
  pg.C = C;
  pg.chunk = HW / nchunks;
  pg.nchunks = nchunks;
  if (dgamma) {
    if (fin_huge(pg))
      hipLaunchKernelGGL((norm_param_grad_kernel<1, 256>), dim3(C), dim3(256), 0, st, partials, pg, dgamma, dbeta);
    else if (fin_wide(pg) || N > 8)
      hipLaunchKernelGGL((norm_param_grad_kernel<8, 32>), dim3((C + 7) / 8), dim3(256), 0, st, partials, pg, dgamma,
                         dbeta);
    else
      hipLaunchKernelGGL((norm_param_grad_kernel<32, 8>), dim3((C + 31) / 32), dim3(256), 0, st, partials, pg, dgamma,
                         dbeta);
  }
  if (dx) {
    P2P_FIN_LAUNCH(norm_bwd_finalize_kernel, pg, N, st, partials, pg, rstd, gamma, coef);
    NormGeom g = make_geom(N, HW, C);
    with_act(prelu_w ? ACT_PRELU_T : act, [&](auto t) {
      hipLaunchKernelGGL((norm_bwd_apply_kernel<decltype(t)::value>), dim3(g.nchunks, N), dim3(256), 0, st,
                         static_cast<const bf16*>(x), static_cast<const bf16*>(dy), g, mean, rstd, gamma, beta,
                         prelu_w, coef, static_cast<bf16*>(dx), Fp8Shadow{static_cast<uint8_t*>(q), qsite, qfmt});
    });
    if (dsum) (void)hipMemsetAsync(dsum, 0, sizeof(float) * C, st);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
