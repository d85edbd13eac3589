// Probe: global_load_lds (LDS-DMA) staging throughput per CU, the suspected limiter of the
// implicit-GEMM conv kernels (profiles/kernel_experiments_r3.md).  One 512-thread block per
// CU (8 waves) streams 1 KiB-per-wave-instruction glds pieces (8 rows x 128 B, the conv
// kernels' A/B row shape) from a buffer into a 2-slot LDS ring, K-tile by K-tile, with
// optional MFMA work per tile; it reports bytes/s per CU and MFMA TF/s.
//   source: L2-resident (every block re-reads one 2 MiB window) or streamed (a 2 GiB sweep)
//   mode 0: all of a tile's glds issued in one burst, then the MFMAs (the LATE loop's shape)
//   mode 1: the glds interleaved in pairs between groups of MFMAs (the 8-phase shape)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// LOADS glds per thread per tile (64 KiB per tile at LOADS = 8), MF MFMAs per wave per tile
template <int LOADS, int MF, int MODE>
__global__ void __launch_bounds__(512) k(const uint8_t* src, size_t window, int tiles, float* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const size_t tile_bytes = (size_t)LOADS * 512 * 16;
  const size_t base = ((size_t)blockIdx.x * tile_bytes * tiles) % window;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (short)(0x3f80 + (lane & 7));
    b[j] = (short)(0x3f80 + (j & 3));
  }
  f32x4 acc[4] = {};
  auto issue = [&](int t, int slot, int lo, int hi) {
    const size_t off = (base + (size_t)t * tile_bytes) % window;
#pragma unroll
    for (int i = lo; i < hi; ++i) {
      const uint8_t* g = src + off + ((size_t)i * 512 + tid) * 16;
      char* d = lds + slot * (int)tile_bytes + (i * 512 + wid * 64) * 16;
      __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)d, 16, 0, 0);
    }
  };
  issue(0, 0, 0, LOADS);
  for (int t = 0; t < tiles; ++t) {
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    const int nslot = (t + 1) & 1;
    if (MODE == 0) {
      if (t + 1 < tiles) issue(t + 1, nslot, 0, LOADS);
#pragma unroll
      for (int m = 0; m < MF; ++m) acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[m & 3], 0, 0, 0);
    } else {
#pragma unroll
      for (int g = 0; g < LOADS / 2; ++g) {
        if (t + 1 < tiles) issue(t + 1, nslot, 2 * g, 2 * g + 2);
#pragma unroll
        for (int m = 0; m < MF / (LOADS / 2); ++m)
          acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[m & 3], 0, 0, 0);
      }
    }
    // keep a dependence on the staged bytes so nothing is dead
    a[0] ^= (short)lds[(t & 1) * tile_bytes + tid * 16];
  }
  const f32x4 s = acc[0] + acc[1] + acc[2] + acc[3];
  out[blockIdx.x * 512 + tid] = s[0] + s[1] + s[2] + s[3];
}

template <int LOADS, int MF, int MODE>
static void run(const uint8_t* src, size_t window, const char* tag, float* out) {
  constexpr int smem = 2 * LOADS * 512 * 16;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k<LOADS, MF, MODE>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  const int blocks = 256, tiles = 512;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((k<LOADS, MF, MODE>), dim3(blocks), dim3(512), smem, 0, src, window, tiles, out);
  (void)hipEventRecord(e0, 0);
  for (int r = 0; r < 3; ++r)
    hipLaunchKernelGGL((k<LOADS, MF, MODE>), dim3(blocks), dim3(512), smem, 0, src, window, tiles, out);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 3;
  const double bytes = (double)blocks * tiles * LOADS * 512 * 16;
  const double flop = (double)blocks * 8 * tiles * MF * 16384.0;
  std::printf("%-10s loads/thread/tile %d  MFMA/wave/tile %3d  mode %d: %7.3f ms  %6.1f GB/s per CU  %7.1f TF/s\n",
              tag, LOADS, MF, MODE, ms, bytes / ms / 1e6 / 256, flop / ms / 1e9);
}

int main() {
  const size_t big = (size_t)2 << 30;
  uint8_t* src;
  float* out;
  if (hipMalloc(&src, big) != hipSuccess || hipMalloc(&out, 256 * 512 * 4) != hipSuccess) return 1;
  (void)hipMemset(src, 1, big);
  for (int w = 0; w < 2; ++w) {
    const size_t window = w == 0 ? ((size_t)2 << 20) : big;
    const char* tag = w == 0 ? "L2-window" : "HBM-sweep";
    run<8, 0, 0>(src, window, tag, out);
    run<8, 64, 0>(src, window, tag, out);
    run<8, 64, 1>(src, window, tag, out);
    run<8, 128, 0>(src, window, tag, out);
    run<8, 128, 1>(src, window, tag, out);
    run<4, 32, 0>(src, window, tag, out);
    run<4, 32, 1>(src, window, tag, out);
  }
  (void)hipFree(src);
  (void)hipFree(out);
  return 0;
}
