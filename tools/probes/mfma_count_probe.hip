// Counter calibration: kernels with an exactly known MFMA count, run under
//   rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE ...
// so tools/roofline.py can turn the raw counters into (a) FLOPs per MFMA instruction and
// (b) MFMA busy as a true fraction of the chip's SIMD-cycles.
//   k_bf16: every wave issues ITERS x 4 v_mfma_f32_16x16x32_bf16 (16 cycles each)
//   k_bf16_32: every wave issues ITERS x 4 v_mfma_f32_32x32x16_bf16 (32 cycles each)
//   k_fp8 : every wave issues ITERS x 4 v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3, 32 cycles)
// Grid: 2048 blocks x 256 threads (8 waves per CU on 256 CUs: 2 per SIMD), so the MFMA pipe of
// every SIMD is saturated and the expected busy fraction is ~1.  The probe prints the
// expected instruction counts; the counter pass supplies the rest.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

constexpr int ITERS = 4096;
constexpr int BLOCKS = 2048;
constexpr int THREADS = 256;

__global__ void __launch_bounds__(256) k_bf16(float* out, int seed) {
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (short)(0x3f80 + ((threadIdx.x + j + seed) & 7));
    b[j] = (short)(0x3f80 + ((threadIdx.x * 3 + j) & 7));
  }
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < ITERS; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c3, 0, 0, 0);
  }
  const f32x4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * THREADS + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

// 32x32x16 bf16 (the round-5 conv tiles): 32768 FLOPs, 32 cycles per instruction
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ void __launch_bounds__(256) k_bf16_32(float* out, int seed) {
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (short)(0x3f80 + ((threadIdx.x + j + seed) & 7));
    b[j] = (short)(0x3f80 + ((threadIdx.x * 3 + j) & 7));
  }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < ITERS; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
  }
  const f32x16 s = c0 + c1 + c2 + c3;
  float t = 0.f;
  for (int r = 0; r < 16; ++r) t += s[r];
  out[blockIdx.x * THREADS + threadIdx.x] = t;
}

__global__ void __launch_bounds__(256) k_fp8(float* out, int seed) {
  i32x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = 0x38383838 + ((threadIdx.x + j + seed) & 3);
    b[j] = 0x38383838 + ((threadIdx.x + 2 * j) & 3);
  }
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < ITERS; ++i) {
    c0 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c0, 0, 0, 0, 127, 0, 127);
    c1 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c1, 0, 0, 0, 127, 0, 127);
    c2 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c2, 0, 0, 0, 127, 0, 127);
    c3 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c3, 0, 0, 0, 127, 0, 127);
  }
  const f32x4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * THREADS + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

int main() {
  float* out;
  if (hipMalloc(&out, sizeof(float) * BLOCKS * THREADS) != hipSuccess) return 1;
  const double waves = (double)BLOCKS * THREADS / 64;
  const double n_mfma = waves * ITERS * 4;
  for (int rep = 0; rep < 3; ++rep) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_bf16, dim3(BLOCKS), dim3(THREADS), 0, 0, out, rep);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::printf("k_bf16 rep %d: %.3f ms, wave-MFMAs %.0f, FLOP %.4e (16384 per MFMA), %.1f TF/s\n", rep, ms,
                n_mfma, n_mfma * 16384.0, n_mfma * 16384.0 / ms / 1e9);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_bf16_32, dim3(BLOCKS), dim3(THREADS), 0, 0, out, rep);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::printf("k_bf16_32 rep %d: %.3f ms, wave-MFMAs %.0f, FLOP %.4e (32768 per MFMA), %.1f TF/s\n", rep, ms,
                n_mfma, n_mfma * 32768.0, n_mfma * 32768.0 / ms / 1e9);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_fp8, dim3(BLOCKS), dim3(THREADS), 0, 0, out, rep);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::printf("k_fp8  rep %d: %.3f ms, wave-MFMAs %.0f, FLOP %.4e (65536 per MFMA), %.1f TF/s\n", rep, ms,
                n_mfma, n_mfma * 65536.0, n_mfma * 65536.0 / ms / 1e9);
  }
  (void)hipFree(out);
  return 0;
}
