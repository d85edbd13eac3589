// Probe: operand lane map of v_mfma_scale_f32_16x16x128_f8f6f4 with e4m3 / e5m2 operands (unscaled;
// NB an unscaled product is blind to a consistent K permutation -- see mfma_fp8_scale.hip).
// Hypothesis H: lane l holds A[row l&15][k = 32*(l>>4) + j] (byte j of its 8 dwords) and
// B[k = 32*(l>>4) + j][col l&15]; C/D: col = l&15, row = 4*(l>>4) + r.
// Exact small-integer data, asymmetric B.  Prints PASS/FAIL per format.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstdint>
#include <vector>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

static float dec_e4m3(uint8_t c) {
  int s = c >> 7, e = (c >> 3) & 15, m = c & 7;
  if (e == 15 && m == 7) return NAN;
  float v = e == 0 ? std::ldexp((float)m / 8.f, -6) : std::ldexp(1.f + m / 8.f, e - 7);
  return s ? -v : v;
}
static float dec_e5m2(uint8_t c) {
  int s = c >> 7, e = (c >> 2) & 31, m = c & 3;
  if (e == 31) return NAN;
  float v = e == 0 ? std::ldexp((float)m / 4.f, -14) : std::ldexp(1.f + m / 4.f, e - 15);
  return s ? -v : v;
}
static uint8_t enc(float x, int fmt) {
  for (int c = 0; c < 256; ++c) {
    float d = fmt == 0 ? dec_e4m3((uint8_t)c) : dec_e5m2((uint8_t)c);
    if (d == x) return (uint8_t)c;
  }
  return 0;
}

template <int FMT>
__global__ void k(const uint8_t* A, const uint8_t* B, float* C) {
  const int l = threadIdx.x;
  v8i a, b;
  uint8_t* pa = reinterpret_cast<uint8_t*>(&a);
  uint8_t* pb = reinterpret_cast<uint8_t*>(&b);
  for (int j = 0; j < 32; ++j) {
    const int kk = 32 * (l >> 4) + j;
    pa[j] = A[(l & 15) * 128 + kk];
    pb[j] = B[kk * 16 + (l & 15)];
  }
  v4f acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, FMT, FMT, 0, 127, 0, 127);
  for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}

template <int FMT>
static bool run() {
  std::vector<uint8_t> A(16 * 128), B(128 * 16);
  std::vector<float> Af(16 * 128), Bf(128 * 16), ref(256, 0.f), out(256);
  for (int i = 0; i < 16; ++i)
    for (int kk = 0; kk < 128; ++kk) {
      float v = (float)(((i * 7 + kk * 3) % 9) - 4);
      Af[i * 128 + kk] = v;
      A[i * 128 + kk] = enc(v, FMT);
    }
  for (int kk = 0; kk < 128; ++kk)
    for (int j = 0; j < 16; ++j) {
      float v = (float)(((kk * 5 + j * 11 + kk / 7) % 7) - 3);
      Bf[kk * 16 + j] = v;
      B[kk * 16 + j] = enc(v, FMT);
    }
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j)
      for (int kk = 0; kk < 128; ++kk) ref[i * 16 + j] += Af[i * 128 + kk] * Bf[kk * 16 + j];
  uint8_t *dA, *dB;
  float* dC;
  (void)hipMalloc(&dA, A.size());
  (void)hipMalloc(&dB, B.size());
  (void)hipMalloc(&dC, 256 * 4);
  (void)hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k<FMT>, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  (void)hipMemcpy(out.data(), dC, 256 * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256; ++i) bad += out[i] != ref[i];
  printf("fmt %d: %s (%d/256 mismatches; out[0]=%g ref[0]=%g)\n", FMT, bad ? "FAIL" : "PASS", bad, out[0], ref[0]);
  (void)hipFree(dA);
  (void)hipFree(dB);
  (void)hipFree(dC);
  return bad == 0;
}

int main() {
  bool ok = run<0>();
  ok = run<1>() && ok;
  return ok ? 0 : 1;
}
