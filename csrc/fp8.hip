// FP8 (OCP e4m3 / e5m2, gfx950) tensor quantisation with per-tensor power-of-two scales.
//
// Scaling recipe (MI355X-first): every fp8 tensor carries a *power-of-two* scale 2^k, so its
// dequantisation factor is an E8M0 byte (127 - k) that the conv kernels hand to the MFMA's
// own block-scale operands (v_mfma_scale_f32_16x16x128_f8f6f4 scale_a / scale_b): the
// dequant is free inside the matrix core, the two halves of a virtual concat can carry
// different scales, and the epilogue needs no multiply.
//
// A scale "site" is 4 int32 words in device memory:
//   [0] amax_ref  (float bits) -- the amax the scale is derived from
//   [1] amax_cur  (float bits) -- running amax of everything quantised this step (atomicMax)
//   [2] e8m0      (int)        -- dequant exponent byte of the last quantisation (read by convs)
//   [3] amax_last (float bits) -- previous step's amax_cur (2-step history window)
// Delayed scaling (activations, gradients): quantise with amax_ref of the previous steps,
// record amax_cur; p2p_fp8_roll (once per step, one launch for the whole pool) shifts the
// window.  Current scaling (weights): p2p_fp8_amax writes amax_ref of this very tensor first.
// Everything stays on the device (graph-capturable, no host sync).
#include "fp8_dev.h"

namespace p2p {

__device__ __forceinline__ float block_max(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  v = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) v = fmaxf(v, red[i]);
  return v;
}

// x: n bf16 (n % 8 == 0) -> q: n fp8 bytes, x * 2^k saturated to +-fmax (the hardware
// conversion returns NaN on overflow, so clamp first).  amax of |x| -> site[1].
template <int FMT>
__global__ void __launch_bounds__(256) fp8_quant_kernel(const bf16* __restrict__ x, long n8, int* site,
                                                        int use_cur, uint8_t* __restrict__ q) {
  __shared__ float red[4];
  const float ref = __int_as_float(site[use_cur ? 1 : 0]);
  const int k = fp8_exp(ref, FMT);
  const float sc = ldexpf(1.f, k), fm = fp8_max(FMT);
  float amax = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + i * 8);
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f[j] = (float)v[j];
      amax = fmaxf(amax, fabsf(f[j]));
      f[j] = fminf(fmaxf(f[j] * sc, -fm), fm);
    }
    uint2 o;
    o.x = cvt4(f[0], f[1], f[2], f[3], FMT);
    o.y = cvt4(f[4], f[5], f[6], f[7], FMT);
    *reinterpret_cast<uint2*>(q + i * 8) = o;
  }
  amax = block_max(amax, red);
  if (threadIdx.x == 0) {
    if (!use_cur) atomicMax(site + 1, __float_as_int(amax));
    if (blockIdx.x == 0) site[2] = 127 - k;
  }
}

// amax of |x| -> site[slot] (site[slot] pre-zeroed by the caller); bf16 or fp32 input,
// 16-B vector loads + scalar tail
template <typename T>
__global__ void __launch_bounds__(256) fp8_amax_kernel(const T* __restrict__ x, long n, int* site, int slot) {
  __shared__ float red[4];
  constexpr int V = 16 / sizeof(T);
  float amax = 0.f;
  const long nv = n / V;
  const long tid0 = (long)blockIdx.x * blockDim.x + threadIdx.x, stride = (long)gridDim.x * blockDim.x;
  for (long i = tid0; i < nv; i += stride) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(x + i * V);
    const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
    for (int j = 0; j < V; ++j) amax = fmaxf(amax, fabsf((float)e[j]));
  }
  for (long i = nv * V + tid0; i < n; i += stride) amax = fmaxf(amax, fabsf((float)x[i]));
  amax = block_max(amax, red);
  if (threadIdx.x == 0 && amax > 0.f) atomicMax(site + slot, __float_as_int(amax));
}

// multi-tensor amax of fp32 tensors (the weight masters: one launch per step for every
// fp8 weight site), blockIdx.y = tensor; site[0] pre-zeroed
constexpr int AMAX_MULTI = 48;
struct AmaxList {
  const float* x[AMAX_MULTI];
  long n[AMAX_MULTI];
  int* site[AMAX_MULTI];
};

__global__ void __launch_bounds__(256) fp8_amax_multi_kernel(AmaxList L) {
  __shared__ float red[4];
  const int t = blockIdx.y;
  const float* __restrict__ x = L.x[t];
  const long n = L.n[t];
  float amax = 0.f;
  const long nv = n / 4;
  const long tid0 = (long)blockIdx.x * blockDim.x + threadIdx.x, stride = (long)gridDim.x * blockDim.x;
  for (long i = tid0; i < nv; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    amax = fmaxf(fmaxf(amax, fmaxf(fabsf(v.x), fabsf(v.y))), fmaxf(fabsf(v.z), fabsf(v.w)));
  }
  for (long i = nv * 4 + tid0; i < n; i += stride) amax = fmaxf(amax, fabsf(x[i]));
  amax = block_max(amax, red);
  if (threadIdx.x == 0 && amax > 0.f) atomicMax(L.site[t], __float_as_int(amax));
}

__global__ void fp8_roll_kernel(int* sites, int nsites) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsites) return;
  int* s = sites + 4 * i;
  const float cur = __int_as_float(s[1]), last = __int_as_float(s[3]);
  const float m = fmaxf(cur, last);
  if (m > 0.f) s[0] = __float_as_int(m);
  s[3] = s[1];
  s[1] = 0;
}

// word `word` of sites [0, nsites) := 0 (a current-scaling weight site's amax before its
// per-step measurement; a HIP launch instead of an aten fill on a strided view)
__global__ void fp8_word_zero_kernel(int* sites, int nsites, int word) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nsites) sites[4 * i + word] = 0;
}

// fp8 -> bf16 with the site's dequant exponent (tests / debugging)
template <int FMT>
__global__ void fp8_dequant_kernel(const uint8_t* __restrict__ q, long n, const int* site, bf16* __restrict__ y) {
  const float sc = ldexpf(1.f, site[2] - 127);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const uint32_t b = q[i];
    float v;
    if (FMT == 0) {
      const int s = b >> 7, e = (b >> 3) & 15, m = b & 7;
      v = (e == 15 && m == 7) ? __builtin_nanf("") : (e == 0 ? ldexpf((float)m, -9) : ldexpf(1.f + m * 0.125f, e - 7));
      v = s ? -v : v;
    } else {
      const int s = b >> 7, e = (b >> 2) & 31, m = b & 3;
      v = e == 31 ? (m ? __builtin_nanf("") : __builtin_inff()) : (e == 0 ? ldexpf((float)m, -16) : ldexpf(1.f + m * 0.25f, e - 15));
      v = s ? -v : v;
    }
    y[i] = (bf16)(v * sc);
  }
}

static int grid_for(long work, int per_block) {
  long g = (work + per_block - 1) / per_block;
  if (g > 4096) g = 4096;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace p2p

extern "C" {
int p2p_fp8_quant(const void* x, long n, int* site, int use_cur, int fmt, void* q, hipStream_t st) {
  if (n % 8) return -1;
  const long n8 = n / 8;
  const int g = p2p::grid_for(n8, 256 * 4);
  if (fmt == 0)
    hipLaunchKernelGGL(p2p::fp8_quant_kernel<0>, dim3(g), dim3(256), 0, st, (const p2p::bf16*)x, n8, site, use_cur,
                       (uint8_t*)q);
  else
    hipLaunchKernelGGL(p2p::fp8_quant_kernel<1>, dim3(g), dim3(256), 0, st, (const p2p::bf16*)x, n8, site, use_cur,
                       (uint8_t*)q);
  return (int)hipGetLastError();
}

int p2p_fp8_amax(const void* x, int is_f32, long n, int* site, int slot, hipStream_t st) {
  const int g = p2p::grid_for(n, 256 * 8);
  if (is_f32)
    hipLaunchKernelGGL(p2p::fp8_amax_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)x, n, site, slot);
  else
    hipLaunchKernelGGL(p2p::fp8_amax_kernel<p2p::bf16>, dim3(g), dim3(256), 0, st, (const p2p::bf16*)x, n, site, slot);
  return (int)hipGetLastError();
}

int p2p_fp8_amax_multi(int count, const float* const* x, const long* n, int* const* site, hipStream_t st) {
  using namespace p2p;
  if (count <= 0) return 0;
  if (count > AMAX_MULTI) return -1;
  AmaxList L;
  long mx = 1;
  for (int i = 0; i < count; ++i) {
    if (((uintptr_t)x[i]) & 15) return -1;
    L.x[i] = x[i];
    L.n[i] = n[i];
    L.site[i] = site[i];
    mx = n[i] > mx ? n[i] : mx;
  }
  long g = (mx / 4 + 256 * 8 - 1) / (256 * 8);
  g = g < 1 ? 1 : (g > 256 ? 256 : g);
  hipLaunchKernelGGL(fp8_amax_multi_kernel, dim3((unsigned)g, count), dim3(256), 0, st, L);
  return (int)hipGetLastError();
}

int p2p_fp8_word_zero(int* sites, int nsites, int word, hipStream_t st) {
  if (nsites <= 0) return 0;
  hipLaunchKernelGGL(p2p::fp8_word_zero_kernel, dim3((nsites + 255) / 256), dim3(256), 0, st, sites, nsites, word);
  return (int)hipGetLastError();
}

int p2p_fp8_roll(int* sites, int nsites, hipStream_t st) {
  if (nsites <= 0) return 0;
  hipLaunchKernelGGL(p2p::fp8_roll_kernel, dim3((nsites + 255) / 256), dim3(256), 0, st, sites, nsites);
  return (int)hipGetLastError();
}

int p2p_fp8_dequant(const void* q, long n, const int* site, int fmt, void* y, hipStream_t st) {
  const int g = p2p::grid_for(n, 256 * 4);
  if (fmt == 0)
    hipLaunchKernelGGL(p2p::fp8_dequant_kernel<0>, dim3(g), dim3(256), 0, st, (const uint8_t*)q, n, site,
                       (p2p::bf16*)y);
  else
    hipLaunchKernelGGL(p2p::fp8_dequant_kernel<1>, dim3(g), dim3(256), 0, st, (const uint8_t*)q, n, site,
                       (p2p::bf16*)y);
  return (int)hipGetLastError();
}
}
