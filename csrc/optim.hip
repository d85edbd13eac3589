// Multi-tensor Adam (torch.optim.Adam semantics: L2 weight decay, bias-corrected) on fp32
// master weights, gfx950.  ONE launch updates up to MT_MAX tensors: the tensor list rides
// in the kernel-argument block (no device metadata buffer, no H2D copy, stable under
// hipGraph replay), each workgroup owns a 4096-element chunk of one tensor and moves it
// with float4 loads.  lr and the step counter are read from device memory so a captured
// step follows LR schedules and bias correction without re-capture.
#include "common.h"

namespace p2p {

constexpr int MT_MAX = 40;
constexpr int MT_CHUNK = 4096;

struct AdamList {
  float* p[MT_MAX];
  const float* g[MT_MAX];
  float* m[MT_MAX];
  float* v[MT_MAX];
  int n[MT_MAX];
  int chunk_start[MT_MAX + 1];  // prefix sum of chunks
  int count;
};

// skip_p (optional): a device flag set by the NaN/Inf guard -- when non-zero the whole
// update (parameters AND moments) is skipped, with no host round trip.
__global__ void __launch_bounds__(256) adam_kernel(AdamList L, const float* __restrict__ lr_p,
                                                   const float* __restrict__ step_p,
                                                   const float* __restrict__ skip_p, float b1, float b2,
                                                   float eps, float wd) {
  if (skip_p && skip_p[0] != 0.f) return;
  const int blk = blockIdx.x;
  int t = 0;
  while (t + 1 < L.count && L.chunk_start[t + 1] <= blk) ++t;
  const int c = blk - L.chunk_start[t];
  const int n = L.n[t];
  const int e0 = c * MT_CHUNK;
  const int e1 = min(n, e0 + MT_CHUNK);
  float* __restrict__ p = L.p[t];
  const float* __restrict__ g = L.g[t];
  float* __restrict__ m = L.m[t];
  float* __restrict__ v = L.v[t];
  const float lr = lr_p[0];
  const float step = step_p[0];
  const float bc1 = 1.f - powf(b1, step);
  const float bc2 = 1.f - powf(b2, step);
  const float step_size = lr / bc1;
  const float rbc2 = rsqrtf(bc2);
  const bool vec = ((n & 3) == 0);
  if (vec) {
    for (int e = e0 + threadIdx.x * 4; e < e1; e += 256 * 4) {
      f32x4 pp = *reinterpret_cast<const f32x4*>(p + e);
      f32x4 gg = *reinterpret_cast<const f32x4*>(g + e);
      f32x4 mm = *reinterpret_cast<const f32x4*>(m + e);
      f32x4 vv = *reinterpret_cast<const f32x4*>(v + e);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float gj = gg[j] + wd * pp[j];
        mm[j] = b1 * mm[j] + (1.f - b1) * gj;
        vv[j] = b2 * vv[j] + (1.f - b2) * gj * gj;
        const float den = sqrtf(vv[j]) * rbc2 + eps;
        pp[j] -= step_size * mm[j] / den;
      }
      *reinterpret_cast<f32x4*>(p + e) = pp;
      *reinterpret_cast<f32x4*>(m + e) = mm;
      *reinterpret_cast<f32x4*>(v + e) = vv;
    }
  } else {
    for (int e = e0 + threadIdx.x; e < e1; e += 256) {
      float gj = g[e] + wd * p[e];
      const float mj = b1 * m[e] + (1.f - b1) * gj;
      const float vj = b2 * v[e] + (1.f - b2) * gj * gj;
      m[e] = mj;
      v[e] = vj;
      p[e] -= step_size * mj / (sqrtf(vj) * rbc2 + eps);
    }
  }
}

}  // namespace p2p

extern "C" {

int p2p_adam_max_tensors() { return p2p::MT_MAX; }

int p2p_adam(int count, float* const* p, const float* const* g, float* const* m, float* const* v,
             const long* n, const float* lr, const float* step, const float* skip, float b1, float b2,
             float eps, float wd, hipStream_t st) {
  using namespace p2p;
  if (count <= 0) return 0;
  if (count > MT_MAX) return -1;
  AdamList L;
  L.count = count;
  int chunks = 0;
  for (int i = 0; i < count; ++i) {
    L.p[i] = p[i];
    L.g[i] = g[i];
    L.m[i] = m[i];
    L.v[i] = v[i];
    L.n[i] = (int)n[i];
    L.chunk_start[i] = chunks;
    chunks += (int)((n[i] + MT_CHUNK - 1) / MT_CHUNK);
  }
  L.chunk_start[count] = chunks;
  hipLaunchKernelGGL(adam_kernel, dim3(chunks), dim3(256), 0, st, L, lr, step, skip, b1, b2, eps, wd);
  return (int)hipGetLastError();
}

}  // extern "C"
