// Shared device helpers for the p2p_pytorch_amd HIP/CDNA4 (gfx950) kernels.
#pragma once
#include "knobs.h"
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

namespace p2p {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// activation codes shared with bindings.cpp / ops/hip.py
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_LRELU = 2, ACT_TANH = 3, ACT_SIGMOID = 4 };
constexpr float LRELU_SLOPE = 0.2f;

__device__ __forceinline__ float act_fwd(float v, int act) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? v : 0.f;
    case ACT_LRELU: return v > 0.f ? v : LRELU_SLOPE * v;
    case ACT_TANH: return tanhf(v);
    case ACT_SIGMOID: return 1.f / (1.f + __expf(-v));
    default: return v;
  }
}

// derivative of act expressed through the activation's INPUT x (relu / lrelu).  Branch-free
// in the per-element part: the negative-side slope depends only on the (wave-uniform) code,
// so it is computed once per unrolled block, and each element costs one compare + select
// instead of a scalar branch.
__device__ __forceinline__ float neg_slope(int act) {
  return act == ACT_RELU ? 0.f : (act == ACT_LRELU ? LRELU_SLOPE : 1.f);
}
__device__ __forceinline__ float act_grad_from_input(float x, int act) {
  return x > 0.f ? 1.f : neg_slope(act);
}

// derivative of act expressed through the activation's OUTPUT y (tanh / sigmoid / relu),
// branch-free (selects only)
__device__ __forceinline__ float act_grad_from_output(float y, int act) {
  const float pw = y > 0.f ? 1.f : neg_slope(act);
  const float t = act == ACT_TANH ? 1.f - y * y : y * (1.f - y);
  return act >= ACT_TANH ? t : pw;
}

__device__ __forceinline__ u32x4 zero_u32x4() { return u32x4{0u, 0u, 0u, 0u}; }

// apply relu / lrelu to 8 packed bf16 held in a 16-byte vector
__device__ __forceinline__ u32x4 act8(u32x4 v, int act) {
  if (act == ACT_NONE) return v;
  bf16x8 b = __builtin_bit_cast(bf16x8, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float f = (float)b[j];
    b[j] = (bf16)act_fwd(f, act);
  }
  return __builtin_bit_cast(u32x4, b);
}

__host__ __device__ __forceinline__ int reflect_idx(int i, int n) {
  // PyTorch ReflectionPad semantics (pad < n)
  i = i < 0 ? -i : i;
  return i >= n ? 2 * (n - 1) - i : i;
}

// Bijective XCD-aware remap of a linear workgroup id: blocks b and b+8 share an XCD
// (MI355X dispatches round-robin over 8 XCDs); give each XCD a contiguous range of
// logical tiles so tiles that share operand panels hit the same L2.
__host__ __device__ __forceinline__ int xcd_remap(int b, int nwg) {
  if (nwg < 16) return b;
  int q = nwg / 8, r = nwg % 8;
  int xcd = b % 8, loc = b / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// ReLU on 8 packed bf16: a bf16 is negative iff its int16 bit pattern is, so a packed
// signed int16 max with 0 is an exact ReLU (-0.0 -> +0.0): 4 v_pk_max_i16 per 16 bytes.
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t relu2(uint32_t w) {
  s16x2 s = __builtin_bit_cast(s16x2, w);
  s = __builtin_elementwise_max(s, (s16x2){0, 0});
  return __builtin_bit_cast(uint32_t, s);
}
// NB: spelled out per component.  hipcc (ROCm 7.2) miscompiles __builtin_bit_cast applied
// to a subscripted ext_vector element inside a loop (v[j]): it reads element 0 for every j.
__device__ __forceinline__ u32x4 relu8(u32x4 v) {
  u32x4 o;
  o.x = relu2(v.x);
  o.y = relu2(v.y);
  o.z = relu2(v.z);
  o.w = relu2(v.w);
  return o;
}

// activation of a loaded 16-B chunk: ReLU on the integer pipe, anything else through fp32
__device__ __forceinline__ u32x4 act_chunk(u32x4 v, int act) {
  if (act == ACT_NONE) return v;
  if (act == ACT_RELU) return relu8(v);
  return act8(v, act);
}

// Division by a loop-invariant divisor: q = (umulhi(n, mul) + n) >> shift, exact for
// n < 2^31 (Granlund-Montgomery).  Built from uniform values -> scalar registers.
struct FastDiv {
  uint32_t d, mul, shift;
};

__host__ __device__ __forceinline__ FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1u << s) < d) ++s;
  f.shift = s;
  f.mul = (uint32_t)((((1ull << 32) * ((1ull << s) - d)) / d) + 1ull);
  return f;
}

// (the 64-bit product's high word is v_mul_hi_u32 on the device; plain C++ on the host, so
// tests/native/host_checks.cpp runs this exact function under ASan/UBSan)
__host__ __device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return ((uint32_t)(((uint64_t)n * f.mul) >> 32) + n) >> f.shift;
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}


// Raise a kernel's dynamic-LDS limit once per DEVICE (the attribute is per device: a second
// GPU driven by the same process needs its own call).  ``mask``: one static per kernel
// instantiation at the call site, bit d = device d done.
inline void smem_attr_once(const void* fn, int smem, std::atomic<uint64_t>& mask) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  const uint64_t bit = 1ull << (dev & 63);
  if (mask.load(std::memory_order_relaxed) & bit) return;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  mask.fetch_or(bit, std::memory_order_relaxed);
}

}  // namespace p2p
