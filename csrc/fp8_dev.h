// Device helpers of the fp8 path shared by the quantiser (fp8.hip) and the producers that
// write an fp8 "shadow" of their bf16 output in the same pass (norm apply / norm backward /
// conv epilogue).  Scale sites: see fp8.hip.
#pragma once
#include "common.h"

namespace p2p {

__device__ __forceinline__ float fp8_max(int fmt) { return fmt == 0 ? 448.f : 57344.f; }

// k such that amax * 2^k <= fmax (largest such power of two); 0 when amax is 0 / not finite
__device__ __forceinline__ int fp8_exp(float amax, int fmt) {
  if (!(amax > 0.f) || !(amax < 3.0e38f)) return 0;
  int e;
  (void)frexpf(fp8_max(fmt) / amax, &e);  // fmax/amax = m * 2^e, m in [0.5, 1)
  int k = e - 1;
  return k < -120 ? -120 : (k > 120 ? 120 : k);
}

__device__ __forceinline__ uint32_t cvt4(float a, float b, float c, float d, int fmt) {
  int lo, hi;
  if (fmt == 0) {
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, lo, true);
  } else {
    lo = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
    hi = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, lo, true);
  }
  return (uint32_t)hi;
}

// 8 floats -> 8 fp8 bytes: x * sc saturated to +-fmax (the hardware conversion returns NaN
// on overflow, so clamp first)
__device__ __forceinline__ uint2 fp8_pack8(const float* f, float sc, int fmt) {
  const float fm = fp8_max(fmt);
  float g[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) g[j] = fminf(fmaxf(f[j] * sc, -fm), fm);
  uint2 o;
  o.x = cvt4(g[0], g[1], g[2], g[3], fmt);
  o.y = cvt4(g[4], g[5], g[6], g[7], fmt);
  return o;
}

// fused-shadow output descriptor: q == nullptr -> off
struct Fp8Shadow {
  uint8_t* q;
  int* site;
  int fmt;
};

// quantisation multiplier 2^k of a shadow (delayed scaling: amax_ref = site[0]); the
// first thread of the grid publishes the E8M0 dequant exponent for the consumers
__device__ __forceinline__ float fp8_shadow_scale(const Fp8Shadow& s) {
  const int k = fp8_exp(__int_as_float(s.site[0]), s.fmt);
  if (blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0) s.site[2] = 127 - k;
  return ldexpf(1.f, k);
}

// running amax of what was quantised -> site[1]: wave max, then an atomic only when the
// wave's max beats the value already there (thousands of waves hit the same word; after the
// first few the plain load filters almost all of them -- the unconditional per-wave atomic
// made a 64-channel 128x128 conv epilogue 7x slower)
__device__ __forceinline__ void fp8_amax_commit(float amax, int* site) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
  if ((threadIdx.x & 63) == 0 && amax > 0.f) {
    const int bits = __float_as_int(amax);
    if (bits > __atomic_load_n(site + 1, __ATOMIC_RELAXED)) atomicMax(site + 1, bits);
  }
}

}  // namespace p2p
