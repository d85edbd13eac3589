// Memory-bound helpers on bf16 NHWC tensors (gfx950): activations and their backward,
// counter-hash dropout, channel pad / slice (for C % 8 != 0 image tensors at the network
// fringe), per-channel column sums (bias gradients) and the fused GAN / reconstruction
// losses (forward value and input gradient, no target tensor ever materialised).
//
// Every vector path moves 16 B per lane (bf16x8) -- hipcc does not vectorise bf16.
// Reductions are two-stage (fixed-order block partials -> one finishing block), so every
// loss and bias gradient is bitwise reproducible run to run.
#include "bounds.h"
#include "common.h"

namespace p2p {

__device__ __forceinline__ void unpack8e(u32x4 v, float* f) {
  bf16x8 b = __builtin_bit_cast(bf16x8, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (float)b[j];
}

__device__ __forceinline__ u32x4 pack8e(const float* f) {
  bf16x8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = (bf16)f[j];
  return __builtin_bit_cast(u32x4, b);
}

static inline unsigned egrid(long work) {
  long b = (work + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (unsigned)b;
}

// y = act(x)                                           mode 0
// dx = dy * act'(x)   (relu / lrelu, from the input)    mode 1
// dx = dy * act'(y)   (tanh / sigmoid / relu, from the output)  mode 2
__global__ void __launch_bounds__(256) act_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b,
                                                  long n, int act, int mode, bf16* __restrict__ out) {
  const long n8 = n / 8;
  // scalar tail (numel % 8: e.g. a 1-channel PatchGAN logit map of odd size)
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) {
    const long i = n8 * 8 + threadIdx.x;
    const float fa = (float)a[i];
    float r;
    if (mode == 0) r = act_fwd(fa, act);
    else if (mode == 3) r = act_fwd(fa + (float)b[i], act);
    else if (mode == 1) r = fa * act_grad_from_input((float)b[i], act);
    else r = fa * act_grad_from_output((float)b[i], act);
    out[i] = (bf16)r;
  }
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n8; e += (long)gridDim.x * 256) {
    float fa[8], fb[8];
    unpack8e(*reinterpret_cast<const u32x4*>(a + e * 8), fa);
    if (mode != 0) unpack8e(*reinterpret_cast<const u32x4*>(b + e * 8), fb);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (mode == 0) fa[j] = act_fwd(fa[j], act);
      else if (mode == 3) fa[j] = act_fwd(fa[j] + fb[j], act);   // fused residual add
      else if (mode == 1) fa[j] = fa[j] * act_grad_from_input(fb[j], act);
      else fa[j] = fa[j] * act_grad_from_output(fb[j], act);
    }
    *reinterpret_cast<u32x4*>(out + e * 8) = pack8e(fa);
  }
}

// counter-based hash (PCG output permutation over a 32-bit state)
__device__ __forceinline__ uint32_t hash32(uint32_t v) {
  uint32_t s = v * 747796405u + 2891336453u;
  uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
  return (w >> 22u) ^ w;
}

// keep(i) = hash(seed, salt, i) >= p ; y = keep ? x / (1-p) : 0.  Same call with dy gives dx.
// seed is read from device memory so a captured hipGraph draws a new mask every replay.
__global__ void __launch_bounds__(256) dropout_kernel(const bf16* __restrict__ x, long n8, float p,
                                                      const int64_t* __restrict__ seed, uint32_t salt,
                                                      bf16* __restrict__ y) {
  const uint32_t s0 = hash32((uint32_t)seed[0] ^ hash32(salt * 0x9E3779B9u + 0x7F4A7C15u));
  const float scale = 1.f / (1.f - p);
  const uint32_t thr = (uint32_t)(p * 4294967296.0);
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n8; e += (long)gridDim.x * 256) {
    float f[8];
    unpack8e(*reinterpret_cast<const u32x4*>(x + e * 8), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t h = hash32(s0 ^ hash32((uint32_t)(e * 8 + j)));
      f[j] = h >= thr ? f[j] * scale : 0.f;
    }
    *reinterpret_cast<u32x4*>(y + e * 8) = pack8e(f);
  }
}

// out[p][0:Ca] = a[p][:], out[p][Ca:Ca+Cb] = b[p][:], out[p][Ca+Cb:Co] = 0   (NHWC, any C)
// one thread per pixel, 16-B stores of 8-channel chunks
__global__ void __launch_bounds__(256) pad_channels_kernel(const bf16* __restrict__ a, int Ca,
                                                           const bf16* __restrict__ b, int Cb,
                                                           long P, int Co, bf16* __restrict__ out) {
  for (long p = blockIdx.x * 256L + threadIdx.x; p < P; p += (long)gridDim.x * 256) {
    for (int c0 = 0; c0 < Co; c0 += 8) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        bf16 e = (bf16)0.f;
        if (c < Ca) e = a[p * Ca + c];
        else if (c < Ca + Cb) e = b[p * Cb + (c - Ca)];
        v[j] = e;
      }
      *reinterpret_cast<bf16x8*>(out + p * Co + c0) = v;
    }
  }
}

// dgrad of a conv whose input was reflect/zero padded by `pad` and nearest-upsampled by
// `up` inside the conv's gather (family-R ConvLayer / UpsampleConvLayer): the MODE-1 dgrad
// wrote the gradient of the VIRTUAL padded input dxp[N][Hp][Wp][C] (Hp = H*up + 2*pad);
// here every real input pixel sums the padded positions that read it (reflection maps up
// to 3 padded rows onto one, the upsample 2x2 up-pixels onto one), then the input
// activation's derivative is applied (act_bwd with the saved input xb).
// One thread per (pixel, 8-channel chunk).
__device__ __forceinline__ int fold_taps(int u, int pad, int Hu, int reflect, int* q) {
  int n = 0;
  if (reflect == 2) {   // replicate (edge) padding: the border pixel collects the whole frame side
    q[n++] = u + pad;
    if (u == 0)
      for (int j = 0; j < pad && n < 5; ++j) q[n++] = j;
    if (u == Hu - 1)
      for (int j = 0; j < pad && n < 5; ++j) q[n++] = Hu + pad + j;
    return n;
  }
  const int c[3] = {u + pad, pad - u, 2 * (Hu - 1) + pad - u};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int qq = c[i];
    if (qq < 0 || qq >= Hu + 2 * pad) continue;
    const int src = reflect ? reflect_idx(qq - pad, Hu) : qq - pad;
    if (src != u) continue;
    bool dup = false;
    for (int j = 0; j < n; ++j) dup = dup || q[j] == qq;
    if (!dup) q[n++] = qq;
  }
  return n;
}

__global__ void __launch_bounds__(256) pad_fold_kernel(const bf16* __restrict__ dxp, int N, int H, int W,
                                                       int C, int pad, int up, int reflect,
                                                       const bf16* __restrict__ xb, int act,
                                                       const bf16* __restrict__ res,
                                                       bf16* __restrict__ dx) {
  const int CP = C >> 3;
  const int Hu = H * up, Wu = W * up;
  const int Hp = Hu + 2 * pad, Wp = Wu + 2 * pad;
  const long total = (long)N * H * W * CP;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int cg = (int)(e % CP);
    const long pix = e / CP;
    const int x = (int)(pix % W);
    const long t = pix / W;
    const int y = (int)(t % H);
    const int n = (int)(t / H);
    int qy[6], qx[6];
    int ny = 0, nx = 0;
    for (int k = 0; k < up; ++k) {
      ny += fold_taps(y * up + k, pad, Hu, reflect, qy + ny);
      nx += fold_taps(x * up + k, pad, Wu, reflect, qx + nx);
    }
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int i = 0; i < ny; ++i)
      for (int k = 0; k < nx; ++k) {
        float f[8];
        unpack8e(*reinterpret_cast<const u32x4*>(dxp + (((long)n * Hp + qy[i]) * Wp + qx[k]) * C + cg * 8), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += f[j];
      }
    if (act) {
      float xf[8];
      unpack8e(*reinterpret_cast<const u32x4*>(xb + pix * C + cg * 8), xf);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= act_grad_from_input(xf[j], act);
    }
    if (res) {   // the other consumer's gradient of this input (residual blocks), after the gate
      float rf[8];
      unpack8e(*reinterpret_cast<const u32x4*>(res + pix * C + cg * 8), rf);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += rf[j];
    }
    if (P2P_OOB_OK(10, pix * C + cg * 8, 8, (long)N * H * W * C))
      *reinterpret_cast<u32x4*>(dx + pix * C + cg * 8) = pack8e(acc);
  }
}

// out[p][0:C] = in[p][c0:c0+C]   (in has Ci channels); one thread per pixel
__global__ void __launch_bounds__(256) slice_channels_kernel(const bf16* __restrict__ in, int Ci, int c0,
                                                             long P, int C, bf16* __restrict__ out) {
  for (long p = blockIdx.x * 256L + threadIdx.x; p < P; p += (long)gridDim.x * 256) {
    for (int c = 0; c < C; ++c) out[p * C + c] = in[p * Ci + c0 + c];
  }
}

// partial column sums of a [M][C] bf16 matrix: ws[block][C]  (C % 8 == 0, C <= 2048)
__global__ void __launch_bounds__(256) colsum_partial_kernel(const bf16* __restrict__ x, long M, int C,
                                                             long rows_per_block, float* __restrict__ ws) {
  const int CP = C >> 3;
  const int RP = 256 / CP;
  const int tid = threadIdx.x, cg = tid % CP, tr = tid / CP;
  const long m0 = blockIdx.x * rows_per_block;
  const long m1 = min(M, m0 + rows_per_block);
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  if (tr < RP) {
    for (long m = m0 + tr; m < m1; m += RP) {
      float f[8];
      unpack8e(*reinterpret_cast<const u32x4*>(x + m * C + cg * 8), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += f[j];
    }
  }
  __shared__ float red[2048];
  const int rows_red = 2048 / C;
  for (int base_r = 0; base_r < RP; base_r += rows_red) {
    if (tr >= base_r && tr < base_r + rows_red && tr < RP) {
      const int r = tr - base_r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (base_r == 0) red[r * C + cg * 8 + j] = s[j];
        else red[r * C + cg * 8 + j] += s[j];
      }
    }
    __syncthreads();
  }
  const int rr = min(RP, rows_red);
  for (int c = tid; c < C; c += 256) {
    float a = 0.f;
    for (int r = 0; r < rr; ++r) a += red[r * C + c];
    ws[(long)blockIdx.x * C + c] = a;
  }
}

// out[c] (+)= scale * sum_b ws[b][c]: G threads per channel, fixed-order LDS combine
template <int G>
__global__ void __launch_bounds__(256) colsum_final_kernel(const float* __restrict__ ws, int nb, int C,
                                                           float scale, int accumulate,
                                                           float* __restrict__ out, int Cout) {
  constexpr int EPB = 256 / G;
  const int le = threadIdx.x % EPB, sg = threadIdx.x / EPB;
  const int c = blockIdx.x * EPB + le;
  float a = 0.f;
  if (c < C)
    for (int b = sg; b < nb; b += G) a += ws[(long)b * C + c];
  __shared__ float red[256];
  red[threadIdx.x] = a;
  __syncthreads();
  if (sg != 0 || c >= Cout) return;   // Cout <= C: the leading channels of a padded gradient
  for (int q = 1; q < G; ++q) a += red[q * EPB + le];
  a *= scale;
  out[c] = accumulate ? out[c] + a : a;
}

// ---------------------------------------------------------------- losses
// kinds: 0 = mse vs const t, 1 = bce-with-logits vs const t, 2 = bce(prob) vs const t,
//        3 = l1(a, b), 4 = mse(a, b), 5 = mean(a), 6 = l1(a, b) whose gradient also carries
//        lrelu'(a) (a is a LeakyReLU output whose producer left its derivative to consumers),
//        7 = the same with relu'(a) (a ReLU output)
__device__ __forceinline__ float loss_elem(int kind, float a, float b, float t) {
  switch (kind) {
    case 0: { const float d = a - t; return d * d; }
    case 1: return fmaxf(a, 0.f) - a * t + log1pf(__expf(-fabsf(a)));
    case 2: {
      const float lp = fmaxf(logf(a), -100.f), lq = fmaxf(logf(1.f - a), -100.f);
      return -(t * lp + (1.f - t) * lq);
    }
    case 3:
    case 6:
    case 7: return fabsf(a - b);
    case 4: { const float d = a - b; return d * d; }
    default: return a;
  }
}

__device__ __forceinline__ float loss_grad(int kind, float a, float b, float t) {
  switch (kind) {
    case 0: return 2.f * (a - t);
    case 1: return 1.f / (1.f + __expf(-a)) - t;
    case 2: {
      const float den = fmaxf(a * (1.f - a), 1e-12f);
      return (a - t) / den;
    }
    case 3: { const float d = a - b; return d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f); }
    case 6: {
      const float d = a - b;
      return (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f)) * (a > 0.f ? 1.f : LRELU_SLOPE);
    }
    case 7: {   // a is a ReLU output: relu'(pre) = [a > 0]
      const float d = a - b;
      return a > 0.f ? (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f)) : 0.f;
    }
    case 4: return 2.f * (a - b);
    default: return 1.f;
  }
}

__device__ __forceinline__ float ldval(const void* p, long i, int is_f32) {
  return is_f32 ? static_cast<const float*>(p)[i] : (float)static_cast<const bf16*>(p)[i];
}

// partial sums of loss_elem over [0, n): one float per block
__global__ void __launch_bounds__(256) loss_partial_kernel(const void* __restrict__ a,
                                                           const void* __restrict__ b, int is_f32,
                                                           long n, int kind, float t,
                                                           float* __restrict__ ws) {
  float s = 0.f;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256)
    s += loss_elem(kind, ldval(a, e, is_f32), b ? ldval(b, e, is_f32) : 0.f, t);
  __shared__ float red[4];
  s = warp_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) ws[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(256) loss_final_kernel(const float* __restrict__ ws, int nb,
                                                         float scale, float* __restrict__ out) {
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += 256) s += ws[i];
  __shared__ float red[4];
  s = warp_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (red[0] + red[1] + red[2] + red[3]) * scale;
}

// first stage of a long sum: block b adds its contiguous segment (fixed order) -> part[b]
__global__ void __launch_bounds__(256) seg_sum_kernel(const float* __restrict__ ws, long n, long seg,
                                                      float* __restrict__ part) {
  const long lo = blockIdx.x * seg, hi = min(n, lo + seg);
  float s = 0.f;
  for (long i = lo + threadIdx.x; i < hi; i += 256) s += ws[i];
  __shared__ float red[4];
  s = warp_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ga = gout * scale * dloss/da (bf16 or fp32 like a); gb = -ga (l1 / mse pairs) if requested
__global__ void __launch_bounds__(256) loss_grad_kernel(const void* __restrict__ a,
                                                        const void* __restrict__ b, int is_f32, long n,
                                                        int kind, float t, float scale,
                                                        const float* __restrict__ gout,
                                                        void* __restrict__ ga, void* __restrict__ gb) {
  const float g = gout[0] * scale;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const float v = g * loss_grad(kind, ldval(a, e, is_f32), b ? ldval(b, e, is_f32) : 0.f, t);
    if (ga) {
      if (is_f32) static_cast<float*>(ga)[e] = v;
      else static_cast<bf16*>(ga)[e] = (bf16)v;
    }
    if (gb) {
      if (is_f32) static_cast<float*>(gb)[e] = -v;
      else static_cast<bf16*>(gb)[e] = (bf16)(-v);
    }
  }
}

// Vectorised loss kernels: 16-B loads (8 bf16 / 4 fp32 per thread per pass), kind and dtype
// as template parameters (the scalar kernels above remain for misaligned views).  Element
// partition per block is fixed by n -> deterministic partial sums.
template <int F32>
struct LossVec {
  static constexpr int V = F32 ? 4 : 8;
  __device__ static void load(const void* p, long v, float* f) {
    if constexpr (F32) {
      const float4 q = reinterpret_cast<const float4*>(p)[v];
      f[0] = q.x; f[1] = q.y; f[2] = q.z; f[3] = q.w;
    } else {
      unpack8e(reinterpret_cast<const u32x4*>(p)[v], f);
    }
  }
  __device__ static void store(void* p, long v, const float* f) {
    if constexpr (F32) reinterpret_cast<float4*>(p)[v] = make_float4(f[0], f[1], f[2], f[3]);
    else reinterpret_cast<u32x4*>(p)[v] = pack8e(f);
  }
};

template <int F32, int KIND, bool HAS_B>
__global__ void __launch_bounds__(256) loss_partial_vec_kernel(const void* __restrict__ a,
                                                               const void* __restrict__ b, long n,
                                                               float t, float* __restrict__ ws) {
  using L = LossVec<F32>;
  constexpr int V = L::V;
  const long nv = n / V;
  float s = 0.f;
  for (long v = blockIdx.x * 256L + threadIdx.x; v < nv; v += (long)gridDim.x * 256) {
    float fa[V], fb[V];
    L::load(a, v, fa);
    if constexpr (HAS_B) L::load(b, v, fb);
#pragma unroll
    for (int j = 0; j < V; ++j) s += loss_elem(KIND, fa[j], HAS_B ? fb[j] : 0.f, t);
  }
  if (blockIdx.x == 0 && threadIdx.x < n - nv * V) {
    const long e = nv * V + threadIdx.x;
    s += loss_elem(KIND, ldval(a, e, F32), HAS_B ? ldval(b, e, F32) : 0.f, t);
  }
  __shared__ float red[4];
  s = warp_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) ws[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

template <int F32, int KIND, bool HAS_B>
__global__ void __launch_bounds__(256) loss_grad_vec_kernel(const void* __restrict__ a,
                                                            const void* __restrict__ b, long n, float t,
                                                            float scale, const float* __restrict__ gout,
                                                            void* __restrict__ ga, void* __restrict__ gb) {
  using L = LossVec<F32>;
  constexpr int V = L::V;
  const float g = gout[0] * scale;
  const long nv = n / V;
  for (long v = blockIdx.x * 256L + threadIdx.x; v < nv; v += (long)gridDim.x * 256) {
    float fa[V], fb[V];
    L::load(a, v, fa);
    if constexpr (HAS_B) L::load(b, v, fb);
#pragma unroll
    for (int j = 0; j < V; ++j) fa[j] = g * loss_grad(KIND, fa[j], HAS_B ? fb[j] : 0.f, t);
    if (ga) L::store(ga, v, fa);
    if (gb) {
#pragma unroll
      for (int j = 0; j < V; ++j) fa[j] = -fa[j];
      L::store(gb, v, fa);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < n - nv * V) {
    const long e = nv * V + threadIdx.x;
    const float v = g * loss_grad(KIND, ldval(a, e, F32), HAS_B ? ldval(b, e, F32) : 0.f, t);
    if (ga) {
      if (F32) static_cast<float*>(ga)[e] = v;
      else static_cast<bf16*>(ga)[e] = (bf16)v;
    }
    if (gb) {
      if (F32) static_cast<float*>(gb)[e] = -v;
      else static_cast<bf16*>(gb)[e] = (bf16)(-v);
    }
  }
}

template <typename F>
static void with_loss(int is_f32, int kind, bool has_b, F&& f) {
  auto k2 = [&](auto f32) {
    switch (kind) {
      case 0: f(f32, std::integral_constant<int, 0>{}, std::false_type{}); break;
      case 1: f(f32, std::integral_constant<int, 1>{}, std::false_type{}); break;
      case 2: f(f32, std::integral_constant<int, 2>{}, std::false_type{}); break;
      case 3: f(f32, std::integral_constant<int, 3>{}, std::true_type{}); break;
      case 4: f(f32, std::integral_constant<int, 4>{}, std::true_type{}); break;
      case 6: f(f32, std::integral_constant<int, 6>{}, std::true_type{}); break;
      case 7: f(f32, std::integral_constant<int, 7>{}, std::true_type{}); break;
      default: f(f32, std::integral_constant<int, 5>{}, std::false_type{}); break;
    }
  };
  (void)has_b;
  if (is_f32) k2(std::integral_constant<int, 1>{});
  else k2(std::integral_constant<int, 0>{});
}

static inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace p2p

namespace p2p {
// Stride-1, no-upsample fold (the residual blocks' reflect-pad dgrads): one thread per (pixel,
// 4 chunks of 8 channels), the pixel's 1-4 source positions resolved once, 4 independent 16-B
// loads per source in flight, int32 indexing (host-checked sizes).
__global__ void __launch_bounds__(256) pad_fold_s1_kernel(const bf16* __restrict__ dxp, int N, int H, int W,
                                                          int C, int pad, int reflect,
                                                          const bf16* __restrict__ xb, int act,
                                                          const bf16* __restrict__ res,
                                                          bf16* __restrict__ dx) {
  const int CQ = C >> 5;   // groups of 4 chunks per pixel
  const int Hp = H + 2 * pad, Wp = W + 2 * pad;
  const int total = N * H * W * CQ;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
    const int cq = e % CQ;
    const int pix = e / CQ;
    const int x = pix % W;
    const int t = pix / W;
    const int y = t % H, n = t / H;
    int qy[3], qx[3], ny = 0, nx = 0;
    qy[ny++] = y + pad;
    qx[nx++] = x + pad;
    if (reflect) {
      if (y >= 1 && y <= pad) qy[ny++] = pad - y;                       // reflected top rows
      if (y >= H - 1 - pad && y <= H - 2) qy[ny++] = 2 * (H - 1) + pad - y;   // bottom rows
      if (x >= 1 && x <= pad) qx[nx++] = pad - x;
      if (x >= W - 1 - pad && x <= W - 2) qx[nx++] = 2 * (W - 1) + pad - x;
    }
    float acc[4][8];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
    for (int i = 0; i < ny; ++i)
      for (int k2 = 0; k2 < nx; ++k2) {
        const bf16* src = dxp + ((n * Hp + qy[i]) * Wp + qx[k2]) * C + cq * 32;
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = *reinterpret_cast<const u32x4*>(src + k * 8);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float f[8];
          unpack8e(v[k], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[k][j] += f[j];
        }
      }
    const int o = pix * C + cq * 32;
    if (act) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float xf[8];
        unpack8e(*reinterpret_cast<const u32x4*>(xb + o + k * 8), xf);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[k][j] *= act_grad_from_input(xf[j], act);
      }
    }
    if (res) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float rf[8];
        unpack8e(*reinterpret_cast<const u32x4*>(res + o + k * 8), rf);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[k][j] += rf[j];
      }
    }
    if (!P2P_OOB_OK(11, o, 32, N * H * W * C)) continue;
#pragma unroll
    for (int k = 0; k < 4; ++k) *reinterpret_cast<u32x4*>(dx + o + k * 8) = pack8e(acc[k]);
  }
}

// Frame half of the reflect-pad fold (conv.h fold_buf): the dgrad's epilogue already stored
// every interior pixel of the padded grid -- gated, + the parked skip gradient -- into dx; here
// each real pixel with a mirror image in the p-wide frame (rows / columns 1..p and
// H-1-p..H-2) adds the frame values that reflect onto it, times the same act' gate.  Band
// pixels only: 2p rows x W + (H - 2p) rows x 2p columns per image (host: H, W >= 2p + 2).
// edge = 1 (replicate pad, the nearest-x2 + reflect-1 dgrad): the band is the outermost row /
// column on each side, which collects all p frame rows / columns beyond it (host: p <= 4).
// nb.ws (batch norm fused into the dgrad epilogue, conv_dev.h nb_flat): the epilogue's
// partials counted each band pixel's PRE-fold value; this pass adds, per channel, the change of
// the partial sums d = dz * act'(z), d * xhat (and PReLU's dz * z * [z <= 0]) from the old to
// the new bf16 value of every pixel it rewrites -- block b's sums go to chunk nb.chunk0 + b in
// a fixed order (host: a fixed grid of NB_BAND_BLOCKS blocks), so the norm sees the folded dz.
struct NbBand {
  float* ws;
  long plane;
  int chunk0;
  const bf16* x;
  const float *mean, *rstd, *gamma, *beta, *prelu;
  int act;
};

template <bool NB>   // NB: the partial-sum corrections (their LDS only in that instance)
__global__ void __launch_bounds__(256) fold_band_kernel(const bf16* __restrict__ fb, int N, int H, int W, int C,
                                                        int pad, int edge, const bf16* __restrict__ xb, int act,
                                                        bf16* __restrict__ dx, NbBand nb) {
  float s1[8], s2[8], s3[8], zs[8], zc[8], rs[8], c1[8];
  const int cgt = threadIdx.x % (C >> 3);   // fixed per thread (host: 256 % (C / 8) == 0)
  const float slope = NB ? (nb.prelu ? *nb.prelu : (nb.act ? neg_slope(nb.act) : 1.f)) : 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s1[j] = s2[j] = s3[j] = 0.f;
    rs[j] = c1[j] = zs[j] = zc[j] = 0.f;
    if constexpr (NB) {
      const int c = cgt * 8 + j;
      rs[j] = nb.rstd[c];
      c1[j] = -nb.mean[c] * rs[j];
      const float ga = nb.gamma ? nb.gamma[c] : 1.f, be = nb.gamma ? nb.beta[c] : 0.f;
      zs[j] = rs[j] * ga;
      zc[j] = c1[j] * ga + be;
    }
  }
  const int CP = C >> 3;
  const int Hp = H + 2 * pad, Wp = W + 2 * pad;
  const int bw = edge ? 1 : pad;   // band rows / columns per side
  const int nrow = 2 * bw * W, per_img = nrow + (H - 2 * bw) * 2 * bw;
  const long total = (long)N * per_img * CP;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int cg = (int)(e % CP);
    const long t = e / CP;
    const int n = (int)(t / per_img);
    int k = (int)(t - (long)n * per_img), y, x;
    // band of a side: reflect -> indices 1..p / H-1-p..H-2, edge -> 0 / H-1
    const int b0 = edge ? 0 : 1;
    if (k < nrow) {   // a band row, every column
      const int r = k / W;
      x = k - r * W;
      y = r < bw ? b0 + r : H - b0 - bw + (r - bw);
    } else {          // another row, a band column
      k -= nrow;
      const int r = k / (2 * bw), c = k - r * 2 * bw;
      // the rows outside the bands, in order: reflect 0, p+1 .. H-2-p, H-1; edge 1 .. H-2
      y = edge ? 1 + r : (r == 0 ? 0 : (r == H - 2 * bw - 1 ? H - 1 : pad + r));
      x = c < bw ? b0 + c : W - b0 - bw + (c - bw);
    }
    int qy[9], qx[9], ny = 0, nx = 0;
    qy[ny++] = y + pad;
    qx[nx++] = x + pad;
    if (edge) {
      if (y == 0) for (int j = 0; j < pad; ++j) qy[ny++] = j;
      if (y == H - 1) for (int j = 0; j < pad; ++j) qy[ny++] = H + pad + j;
      if (x == 0) for (int j = 0; j < pad; ++j) qx[nx++] = j;
      if (x == W - 1) for (int j = 0; j < pad; ++j) qx[nx++] = W + pad + j;
    } else {
      if (y >= 1 && y <= pad) qy[ny++] = pad - y;
      if (y >= H - 1 - pad && y <= H - 2) qy[ny++] = 2 * (H - 1) + pad - y;
      if (x >= 1 && x <= pad) qx[nx++] = pad - x;
      if (x >= W - 1 - pad && x <= W - 2) qx[nx++] = 2 * (W - 1) + pad - x;
    }
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int i = 0; i < ny; ++i)
      for (int k2 = 0; k2 < nx; ++k2) {
        if (i == 0 && k2 == 0) continue;   // the interior pixel itself: already in dx
        const long fo = (((long)n * Hp + qy[i]) * Wp + qx[k2]) * C + cg * 8;
        if (!P2P_OOB_OK(13, fo, 8, (long)N * Hp * Wp * C) || (unsigned)qy[i] >= (unsigned)Hp ||
            (unsigned)qx[k2] >= (unsigned)Wp) {
          (void)P2P_OOB_OK(13, -1, 0, 0);
          continue;
        }
        float f[8];
        unpack8e(*reinterpret_cast<const u32x4*>(fb + fo), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += f[j];
      }
    const long o = (((long)n * H + y) * W + x) * C + cg * 8;
    if (!P2P_OOB_OK(12, o, 8, (long)N * H * W * C)) continue;
    if (act) {
      float xf[8];
      unpack8e(*reinterpret_cast<const u32x4*>(xb + o), xf);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= act_grad_from_input(xf[j], act);
    }
    float d[8];
    unpack8e(*reinterpret_cast<const u32x4*>(dx + o), d);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += d[j];
    const u32x4 nv = pack8e(acc);
    *reinterpret_cast<u32x4*>(dx + o) = nv;
    if constexpr (NB) {   // partial-sum change from the old to the new stored value
      float nf[8], xf[8];
      unpack8e(nv, nf);
      unpack8e(*reinterpret_cast<const u32x4*>(nb.x + o), xf);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float dd = nf[j] - d[j];
        const float xh = xf[j] * rs[j] + c1[j];
        const float z = xf[j] * zs[j] + zc[j];
        const float g = dd * (z > 0.f ? 1.f : slope);
        s1[j] += g;
        s2[j] += g * xh;
        s3[j] += z <= 0.f ? dd * z : 0.f;
      }
    }
  }
  if constexpr (NB) {
    // fixed-order block reduction per channel: the 256 / CP threads sharing a channel group
    __shared__ float red[3][256][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[0][threadIdx.x][j] = s1[j];
      red[1][threadIdx.x][j] = s2[j];
      red[2][threadIdx.x][j] = s3[j];
    }
    __syncthreads();
    const int CP = C >> 3;
    for (int c = threadIdx.x; c < C; c += 256) {
      float a1 = 0.f, a2 = 0.f, a3 = 0.f;
      for (int t = c >> 3; t < 256; t += CP) {
        a1 += red[0][t][c & 7];
        a2 += red[1][t][c & 7];
        a3 += red[2][t][c & 7];
      }
      const long oo = (long)(nb.chunk0 + blockIdx.x) * C + c;
      if (P2P_OOB_OK(14, oo, 1, nb.plane)) {
        nb.ws[oo] = a1;
        nb.ws[nb.plane + oo] = a2;
        if (nb.prelu) nb.ws[2 * nb.plane + oo] = a3;
      }
    }
  }
}
}  // namespace p2p

namespace p2p {
// NaN / Inf guard of a training step: flag = 1 if any of the n fp32 loss scalars is not finite
// (else 0), and the guard's device counter += flag -- one launch instead of the
// isfinite / not / any / max / add chain of aten kernels per optimizer step
struct GuardArgs {
  const float* v[8];
  int n;
};
__global__ void guard_flag_kernel(GuardArgs a, float* flag, float* counter) {
  if (threadIdx.x != 0) return;
  float bad = 0.f;
  for (int i = 0; i < a.n; ++i) {
    const float x = *a.v[i];
    if (!(fabsf(x) <= 3.402823466e38f)) bad = 1.f;   // NaN fails every comparison
  }
  *flag = bad;
  if (counter) *counter += bad;
}
}  // namespace p2p

// ---------------------------------------------------------------- small-tensor helpers
// The step's scalar bookkeeping (loss composition, the optimizer's step counter, the dropout
// seed) on HIP kernels instead of PyTorch elementwise ops: out = wa * a + wb * b + c.
__global__ void __launch_bounds__(256) lincomb_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                      float wa, float wb, float c, long n, float* out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float v = wa * a[i] + (b ? wb * b[i] : 0.f) + c;
  out[i] = v;
}

// n-term weighted sum of fp32 scalars (a loss composed of up to 16 weighted terms) and its
// backward (g * w_i into slot i): one launch each
struct LinList {
  const float* p[16];
  float w[16];
  int n;
};

__global__ void __launch_bounds__(64) lincomb_n_kernel(LinList l, float* out) {
  if (threadIdx.x != 0) return;
  float s = 0.f;
  for (int i = 0; i < l.n; ++i) s += l.w[i] * l.p[i][0];
  out[0] = s;
}

__global__ void __launch_bounds__(64) scale_n_kernel(const float* g, LinList l, float* out) {
  const int i = threadIdx.x;
  if (i < l.n) out[i] = l.w[i] * g[0];
}

// part[b][c] = sum of ws rows [b * rpb, (b + 1) * rpb) (column c per thread, rows in order)
__global__ void __launch_bounds__(256) rowsum_partial_kernel(const float* __restrict__ ws, long R, int C, long rpb,
                                                             float* __restrict__ part) {
  const long r0 = (long)blockIdx.x * rpb;
  const long r1 = r0 + rpb < R ? r0 + rpb : R;
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = 0.f;
    for (long r = r0; r < r1; ++r) a += ws[r * C + c];
    part[(long)blockIdx.x * C + c] = a;
  }
}

__global__ void __launch_bounds__(64) i64_add_kernel(long long* t, long long v, long n) {
  const long i = (long)blockIdx.x * 64 + threadIdx.x;
  if (i < n) t[i] += v;
}

extern "C" {

int p2p_act(const void* a, const void* b, long n, int act, int mode, void* out, hipStream_t st) {
  using namespace p2p;
  hipLaunchKernelGGL(act_kernel, dim3(egrid(n / 8 > 0 ? n / 8 : 1)), dim3(256), 0, st, static_cast<const bf16*>(a),
                     static_cast<const bf16*>(b), n, act, mode, static_cast<bf16*>(out));
  return (int)hipGetLastError();
}

int p2p_dropout(const void* x, long n, float p, const int64_t* seed, unsigned salt, void* y,
                hipStream_t st) {
  using namespace p2p;
  hipLaunchKernelGGL(dropout_kernel, dim3(egrid(n / 8)), dim3(256), 0, st, static_cast<const bf16*>(x),
                     n / 8, p, seed, (uint32_t)salt, static_cast<bf16*>(y));
  return (int)hipGetLastError();
}

int p2p_pad_channels(const void* a, int Ca, const void* b, int Cb, long P, int Co, void* out,
                     hipStream_t st) {
  using namespace p2p;
  hipLaunchKernelGGL(pad_channels_kernel, dim3(egrid(P)), dim3(256), 0, st,
                     static_cast<const bf16*>(a), Ca, static_cast<const bf16*>(b), Cb, P, Co,
                     static_cast<bf16*>(out));
  return (int)hipGetLastError();
}

int p2p_pad_fold(const void* dxp, int N, int H, int W, int C, int pad, int up, int reflect,
                 const void* xb, int act, const void* res, void* dx, hipStream_t st) {
  using namespace p2p;
  const long padded = (long)N * (H + 2 * pad) * (W + 2 * pad) * C;
  if (reflect == 2 && (up != 1 || pad > 2)) return -2;   // replicate: the edge dgrad's own frame only
  if (up == 1 && reflect != 2 && C % 32 == 0 && pad < H - 1 && pad < W - 1 && padded < (1L << 31)) {
    const long work = (long)N * H * W * (C / 32);
    long b = (work + 255) / 256;
    b = b > 8192 ? 8192 : (b < 1 ? 1 : b);
    hipLaunchKernelGGL(pad_fold_s1_kernel, dim3((unsigned)b), dim3(256), 0, st, static_cast<const bf16*>(dxp), N,
                       H, W, C, pad, reflect, static_cast<const bf16*>(xb), act, static_cast<const bf16*>(res),
                       static_cast<bf16*>(dx));
    return (int)hipGetLastError();
  }
  const long total = (long)N * H * W * (C / 8);
  hipLaunchKernelGGL(pad_fold_kernel, dim3(egrid(total)), dim3(256), 0, st, static_cast<const bf16*>(dxp), N,
                     H, W, C, pad, up, reflect, static_cast<const bf16*>(xb), act, static_cast<const bf16*>(res),
                     static_cast<bf16*>(dx));
  return (int)hipGetLastError();
}

// blocks of a fold_band pass that also corrects fused batch-norm partials (one chunk each)
int p2p_fold_band_nb_blocks() { return 256; }

// nb_ws: batch-norm partial planes [2 or 3][nchunks][C] (plane = nchunks * C floats) whose
// chunks [nb_chunk0, nb_chunk0 + p2p_fold_band_nb_blocks()) this pass writes (null = off)
int p2p_fold_band(const void* fb, int N, int H, int W, int C, int pad, int edge, const void* xb, int act, void* dx,
                  float* nb_ws, long nb_plane, int nb_chunk0, const void* nb_x, const float* nb_mean,
                  const float* nb_rstd, const float* nb_gamma, const float* nb_beta, const float* nb_prelu,
                  int nb_act, hipStream_t st) {
  using namespace p2p;
  const int bw = edge ? 1 : pad;
  if (C % 8 || pad < 1 || (edge && pad > 4) || H < 2 * bw + 2 || W < 2 * bw + 2) return -2;
  if (nb_ws && (256 % (C / 8) || !nb_x || !nb_mean || !nb_rstd)) return -2;
  const long total = (long)N * (2 * bw * W + (H - 2 * bw) * 2 * bw) * (C / 8);
  const NbBand nb{nb_ws, nb_plane, nb_chunk0, static_cast<const bf16*>(nb_x), nb_mean, nb_rstd, nb_gamma, nb_beta,
                  nb_prelu, nb_act};
  if (nb_ws)
    hipLaunchKernelGGL(fold_band_kernel<true>, dim3(p2p_fold_band_nb_blocks()), dim3(256), 0, st,
                       static_cast<const bf16*>(fb), N, H, W, C, pad, edge, static_cast<const bf16*>(xb), act,
                       static_cast<bf16*>(dx), nb);
  else
    hipLaunchKernelGGL(fold_band_kernel<false>, dim3(egrid(total)), dim3(256), 0, st, static_cast<const bf16*>(fb),
                       N, H, W, C, pad, edge, static_cast<const bf16*>(xb), act, static_cast<bf16*>(dx), nb);
  return (int)hipGetLastError();
}

int p2p_slice_channels(const void* in, int Ci, int c0, long P, int C, void* out, hipStream_t st) {
  using namespace p2p;
  hipLaunchKernelGGL(slice_channels_kernel, dim3(egrid(P)), dim3(256), 0, st,
                     static_cast<const bf16*>(in), Ci, c0, P, C, static_cast<bf16*>(out));
  return (int)hipGetLastError();
}

// workspace: colsum_blocks(M, C) * C floats
int p2p_colsum_blocks(long M, int C) {
  long b = (M + 511) / 512;
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  (void)C;
  return (int)b;
}

int p2p_colsum(const void* x, long M, int C, float scale, int accumulate, float* ws, float* out, int Cout,
               hipStream_t st) {
  using namespace p2p;
  const int nb = p2p_colsum_blocks(M, C);
  const long rpb = (M + nb - 1) / nb;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(nb), dim3(256), 0, st, static_cast<const bf16*>(x), M,
                     C, rpb, ws);
  // nb <= 1024 partials per channel: 32 threads per channel, <= 32 reads each
  hipLaunchKernelGGL(colsum_final_kernel<32>, dim3((C + 7) / 8), dim3(256), 0, st, ws, nb, C, scale,
                     accumulate, out, Cout);
  return (int)hipGetLastError();
}

int p2p_loss_blocks(long n) {
  long b = (n + 2047) / 2048;
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  return (int)b;
}

int p2p_loss_fwd(const void* a, const void* b, int is_f32, long n, int kind, float t, float scale,
                 float* ws, float* out, hipStream_t st) {
  using namespace p2p;
  const int nb = p2p_loss_blocks(n);
  const bool pair = kind == 3 || kind == 4 || kind == 6 || kind == 7;
  if (al16(a) && (!pair || (b && al16(b)))) {
    with_loss(is_f32, kind, pair, [&](auto f32, auto k, auto hb) {
      hipLaunchKernelGGL((loss_partial_vec_kernel<decltype(f32)::value, decltype(k)::value, decltype(hb)::value>),
                         dim3(nb), dim3(256), 0, st, a, b, n, t, ws);
    });
  } else {
    hipLaunchKernelGGL(loss_partial_kernel, dim3(nb), dim3(256), 0, st, a, b, is_f32, n, kind, t, ws);
  }
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(256), 0, st, ws, nb, scale, out);
  return (int)hipGetLastError();
}

int p2p_guard_flag(const float* const* v, int n, float* flag, float* counter, hipStream_t st) {
  using namespace p2p;
  if (n < 1 || n > 8) return -1;
  GuardArgs a{};
  for (int i = 0; i < n; ++i) a.v[i] = v[i];
  a.n = n;
  hipLaunchKernelGGL(guard_flag_kernel, dim3(1), dim3(64), 0, st, a, flag, counter);
  return (int)hipGetLastError();
}

// out[0] = scale * sum(ws[0..n)) for long n: 256 segment sums, then one block (both fixed
// order); part: 256 floats of workspace
int p2p_sum_long(const float* ws, long n, float scale, float* part, float* out, hipStream_t st) {
  using namespace p2p;
  const long seg = (n + 255) / 256;
  hipLaunchKernelGGL(seg_sum_kernel, dim3(256), dim3(256), 0, st, ws, n, seg > 0 ? seg : 1, part);
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(256), 0, st, part, 256, scale, out);
  return (int)hipGetLastError();
}

// out[0] = scale * sum(ws[0..nb)) in a fixed order (per-block partials -> scalar)
int p2p_sum_partials(const float* ws, int nb, float scale, float* out, hipStream_t st) {
  using namespace p2p;
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(256), 0, st, ws, nb, scale, out);
  return (int)hipGetLastError();
}

int p2p_loss_bwd(const void* a, const void* b, int is_f32, long n, int kind, float t, float scale,
                 const float* gout, void* ga, void* gb, hipStream_t st) {
  using namespace p2p;
  const bool pair = kind == 3 || kind == 4 || kind == 6 || kind == 7;
  if (al16(a) && (!pair || (b && al16(b))) && (!ga || al16(ga)) && (!gb || al16(gb))) {
    const long nv = n / (is_f32 ? 4 : 8);
    with_loss(is_f32, kind, pair, [&](auto f32, auto k, auto hb) {
      hipLaunchKernelGGL((loss_grad_vec_kernel<decltype(f32)::value, decltype(k)::value, decltype(hb)::value>),
                         dim3(egrid(nv > 0 ? nv : 1)), dim3(256), 0, st, a, b, n, t, scale, gout, ga, gb);
    });
  } else {
    hipLaunchKernelGGL(loss_grad_kernel, dim3(egrid(n)), dim3(256), 0, st, a, b, is_f32, n, kind, t, scale,
                       gout, ga, gb);
  }
  return (int)hipGetLastError();
}


// out[c] = sum_r ws[r][c] for an fp32 [R][C] partial-sum image (fixed order): rows split over
// up to 1024 blocks first (tmp: p2p_rowsum_tmp_floats(R, C)), then the partials combined
int p2p_rowsum_blocks(long R) {
  long b = (R + 31) / 32;
  return (int)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

int p2p_rowsum_f32(const float* ws, long R, int C, float* tmp, float* out, hipStream_t st) {
  using namespace p2p;
  if (R <= 0 || R > 0x7fffffff) return -1;
  if (R <= 64) {
    hipLaunchKernelGGL(colsum_final_kernel<32>, dim3((C + 7) / 8), dim3(256), 0, st, ws, (int)R, C, 1.f, 0, out, C);
    return (int)hipGetLastError();
  }
  const int nb = p2p_rowsum_blocks(R);
  const long rpb = (R + nb - 1) / nb;
  hipLaunchKernelGGL(rowsum_partial_kernel, dim3(nb), dim3(256), 0, st, ws, R, C, rpb, tmp);
  hipLaunchKernelGGL(colsum_final_kernel<32>, dim3((C + 7) / 8), dim3(256), 0, st, tmp, nb, C, 1.f, 0, out, C);
  return (int)hipGetLastError();
}

int p2p_lincomb(const float* a, const float* b, float wa, float wb, float c, long n, float* out, hipStream_t st) {
  using namespace p2p;
  hipLaunchKernelGGL(lincomb_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, b, wa, wb, c, n, out);
  return (int)hipGetLastError();
}

int p2p_i64_add(long long* t, long long v, long n, hipStream_t st) {
  using namespace p2p;
  hipLaunchKernelGGL(i64_add_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, t, v, n);
  return (int)hipGetLastError();
}

int p2p_lincomb_n(const float* const* p, const float* w, int n, float* out, hipStream_t st) {
  using namespace p2p;
  if (n < 1 || n > 16) return -1;
  LinList l{};
  for (int i = 0; i < n; ++i) {
    l.p[i] = p[i];
    l.w[i] = w[i];
  }
  l.n = n;
  hipLaunchKernelGGL(lincomb_n_kernel, dim3(1), dim3(64), 0, st, l, out);
  return (int)hipGetLastError();
}

int p2p_scale_n(const float* g, const float* w, int n, float* out, hipStream_t st) {
  using namespace p2p;
  if (n < 1 || n > 16) return -1;
  LinList l{};
  for (int i = 0; i < n; ++i) l.w[i] = w[i];
  l.n = n;
  hipLaunchKernelGGL(scale_n_kernel, dim3(1), dim3(64), 0, st, g, l, out);
  return (int)hipGetLastError();
}

}  // extern "C"
