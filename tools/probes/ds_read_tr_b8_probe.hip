// Probe: semantics of ds_read_b64_tr_b8 on gfx950 (the 8-bit transposing LDS read), for the
// fp8 weight-gradient kernel (both MFMA operands k-transposed out of LDS).
// Hypothesis (by analogy with ds_read_b64_tr_b16, cdna_hip_programming.md T10): per group of
// 16 lanes, a block of 8 rows x 16 byte-columns; lane 2q+p supplies the address of row q,
// columns 8p..8p+7; lane i receives column i of the 8 rows, row q in byte q.
// LDS holds byte(row, col) = (row * 16 + col) & 0xff on a [32 rows][64 B] image.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k(uint64_t* out, int variant) {
  __shared__ __attribute__((aligned(16))) uint8_t img[32 * 64];
  const int l = threadIdx.x;
  for (int i = l; i < 32 * 64; i += 64) img[i] = (uint8_t)(((i / 64) * 16 + (i % 64)) & 0xff);
  __syncthreads();
  const int g = l >> 4, i = l & 15;
  int row, col;
  if (variant == 0) {            // hypothesis: lane 2q+p -> row q, cols 8p..8p+7 (+ group g: rows 8g..)
    row = 8 * g + (i >> 1);
    col = 8 * (i & 1);
  } else {                       // alternative: lane 8p+q -> row q, cols 8p..
    row = 8 * g + (i & 7);
    col = 8 * (i >> 3);
  }
  const uint32_t addr = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t*)(img + row * 64 + col));
  uint64_t v;
  asm volatile("ds_read_b64_tr_b8 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr));
  out[l] = v;
}

int main() {
  uint64_t* d;
  if (hipMalloc(&d, 64 * 8) != hipSuccess) return 1;
  uint64_t h[64];
  for (int variant = 0; variant < 2; ++variant) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, variant);
    (void)hipMemcpy(h, d, 64 * 8, hipMemcpyDeviceToHost);
    int ok = 0;
    for (int l = 0; l < 64; ++l) {
      const int g = l >> 4, i = l & 15;
      bool good = true;
      for (int q = 0; q < 8; ++q) {
        const int b = (int)((h[l] >> (8 * q)) & 0xff);
        if (b != (((8 * g + q) * 16 + i) & 0xff)) good = false;   // row 8g+q, column i
      }
      ok += good;
    }
    std::printf("variant %d: %d / 64 lanes match 'lane i <- column i of rows 8g..8g+7'\n", variant, ok);
    for (int l = 0; l < 20; ++l) {
      std::printf("  lane %2d:", l);
      for (int q = 0; q < 8; ++q) std::printf(" r%02d c%02d", (int)((h[l] >> (8 * q)) & 0xff) / 16,
                                              (int)((h[l] >> (8 * q)) & 0xff) % 16);
      std::printf("\n");
    }
  }
  (void)hipFree(d);
  return 0;
}
