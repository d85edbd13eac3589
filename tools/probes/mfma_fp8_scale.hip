// Probe 2: (a) mixed e5m2 A x e4m3 B, (b) per-lane E8M0 scale operands of
// v_mfma_scale_f32_16x16x128_f8f6f4.  Layout under test: lane l (q = l>>4, row/col l&15)
// holds K [16q, 16q+16) in bytes 0-15 and K [64+16q, 64+16q+16) in bytes 16-31; the A / B
// scale of K block b = [32b, 32b+32) is the scale operand of lane group b.  (An earlier
// version put K [32q, 32q+32) in lane group q -- a consistent K permutation passes any
// unscaled test, and its scale check cancelled out: sa*sb was constant.)
// (c) v_cvt_pk_fp8_f32 / v_cvt_pk_bf8_f32 encodings (OCP) incl. rounding and overflow.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstdint>
#include <vector>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

static float dec(uint8_t c, int fmt) {
  if (fmt == 0) {
    int s = c >> 7, e = (c >> 3) & 15, m = c & 7;
    if (e == 15 && m == 7) return NAN;
    float v = e == 0 ? std::ldexp((float)m / 8.f, -6) : std::ldexp(1.f + m / 8.f, e - 7);
    return s ? -v : v;
  }
  int s = c >> 7, e = (c >> 2) & 31, m = c & 3;
  if (e == 31) return m ? NAN : (s ? -INFINITY : INFINITY);
  float v = e == 0 ? std::ldexp((float)m / 4.f, -14) : std::ldexp(1.f + m / 4.f, e - 15);
  return s ? -v : v;
}
static uint8_t enc(float x, int fmt) {
  for (int c = 0; c < 256; ++c)
    if (dec((uint8_t)c, fmt) == x) return (uint8_t)c;
  return 0;
}

__global__ void kmix(const uint8_t* A, const uint8_t* B, float* C) {
  const int l = threadIdx.x;
  v8i a, b;
  uint8_t* pa = reinterpret_cast<uint8_t*>(&a);
  uint8_t* pb = reinterpret_cast<uint8_t*>(&b);
  for (int j = 0; j < 32; ++j) {
    const int kk = j < 16 ? 16 * (l >> 4) + j : 64 + 16 * (l >> 4) + (j - 16);
    pa[j] = A[(l & 15) * 128 + kk];
    pb[j] = B[kk * 16 + (l & 15)];
  }
  const int sa = 127 + (l >> 4) - 1;        // 2^-1, 2^0, 2^1, 2^2 per K block
  const int sb = 127 - 2 * (l >> 4);        // 2^0, 2^-2, 2^-4, 2^-6 (products do not cancel)
  v4f acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 1, 0, 0, sa, 0, sb);
  for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}

__global__ void kcvt(const float* x, int n, uint8_t* q8, uint8_t* q5) {
  const int i = threadIdx.x;
  if (2 * i + 1 < n) {
    int r = __builtin_amdgcn_cvt_pk_fp8_f32(x[2 * i], x[2 * i + 1], 0, false);
    int s = __builtin_amdgcn_cvt_pk_bf8_f32(x[2 * i], x[2 * i + 1], 0, false);
    q8[2 * i] = r & 0xff;
    q8[2 * i + 1] = (r >> 8) & 0xff;
    q5[2 * i] = s & 0xff;
    q5[2 * i + 1] = (s >> 8) & 0xff;
  }
}

int main() {
  int fails = 0;
  {
    std::vector<uint8_t> A(16 * 128), B(128 * 16);
    std::vector<float> Af(16 * 128), Bf(128 * 16), ref(256, 0.f), out(256);
    for (int i = 0; i < 16; ++i)
      for (int kk = 0; kk < 128; ++kk) {
        float v = (float)(((i * 7 + kk * 3) % 9) - 4);
        Af[i * 128 + kk] = v;
        A[i * 128 + kk] = enc(v, 1);
      }
    for (int kk = 0; kk < 128; ++kk)
      for (int j = 0; j < 16; ++j) {
        float v = (float)(((kk * 5 + j * 11 + kk / 7) % 7) - 3);
        Bf[kk * 16 + j] = v;
        B[kk * 16 + j] = enc(v, 0);
      }
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j)
        for (int kk = 0; kk < 128; ++kk) {
          const int blk = kk / 32;
          ref[i * 16 + j] += Af[i * 128 + kk] * std::ldexp(1.f, blk - 1) * Bf[kk * 16 + j] * std::ldexp(1.f, -2 * blk);
        }
    uint8_t *dA, *dB;
    float* dC;
    (void)hipMalloc(&dA, A.size());
    (void)hipMalloc(&dB, B.size());
    (void)hipMalloc(&dC, 256 * 4);
    (void)hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(kmix, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    (void)hipMemcpy(out.data(), dC, 256 * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += out[i] != ref[i];
    printf("mixed e5m2 x e4m3 with per-lane scales: %s (%d bad; out0=%g ref0=%g)\n", bad ? "FAIL" : "PASS", bad,
           out[0], ref[0]);
    fails += bad != 0;
  }
  {
    std::vector<float> x = {0.f, 1.f, -1.f, 0.3f, 1.0625f, 1.1875f, 447.f, 448.f, 464.f, 500.f, 1000.f, -1e6f,
                            1e-3f, 2e-3f, 3e-9f, 57344.f, 61440.f, 1e5f, 0.0146484375f, 1.f / 1024.f};
    const int n = (int)x.size();
    float* dx;
    uint8_t *d8, *d5;
    (void)hipMalloc(&dx, n * 4);
    (void)hipMalloc(&d8, n);
    (void)hipMalloc(&d5, n);
    (void)hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(kcvt, dim3(1), dim3(64), 0, 0, dx, n, d8, d5);
    std::vector<uint8_t> q8(n), q5(n);
    (void)hipMemcpy(q8.data(), d8, n, hipMemcpyDeviceToHost);
    (void)hipMemcpy(q5.data(), d5, n, hipMemcpyDeviceToHost);
    for (int i = 0; i < n; ++i)
      printf("cvt %-12g -> e4m3 0x%02x (%g)   e5m2 0x%02x (%g)\n", x[i], q8[i], dec(q8[i], 0), q5[i], dec(q5[i], 1));
  }
  return fails;
}
