// Input gradient of a stride-1 convolution with ONE output channel -- the PatchGAN logits conv
// (reference networks.py:781-784: 512 -> 1, 4x4, stride 1, pad 1; one per discriminator scale
// in the reference family) -- as a bandwidth kernel.
//
// Routed through the implicit-GEMM tiles, this input gradient ran K = 16 taps x 8 channels of
// a dY padded from 1 channel to the tiles' 8-channel granularity: 8x the useful MFMA work on a
// 128 x 128 tile at 9 % MFMA busy, 876 us per call at B = 1024 (1.4 % of the headline step,
// profiles/roofline_r6_final.md).  The useful work is 16 multiply-adds per output element:
//     dX[n][oy][ox][co] = alpha * sum_{ky,kx} dY[n][oy + p - ky][ox + p - kx][0] * W[co][ky][kx]
// (W rounded to bf16, as the GEMM path's weight image), so the kernel is bound by writing dX.
// A block stages the weights and its dY window once in LDS; a thread owns 8 consecutive
// output channels (its taps' weights in 8 x T fp32 registers) and walks the block's pixels;
// the TPP = Cp / 8 threads of one pixel read the same window values (LDS broadcast) and store
// one contiguous Cp x 2-byte row with 16-B stores.  Taps summed in ascending order in fp32.
// (Earlier versions read the weights straight from the strided bf16 GEMM image -- 8192
// cache-line requests per wave for 16 pixels, 6.4 ms per call -- and dY from global memory in
// the pixel loop -- a dependent load -> FMA chain per pixel, 4.0 ms: the GEMM took 1.7.)
#include "conv_dev.h"

namespace p2p {

// A block = RB output rows of one image x all Cp channels.  LDS: the weights transposed to
// [T][Cp] (a thread's 8 channels of one tap are 32 contiguous bytes) and rounded to bf16 like
// the GEMM path's weight image, and the block's dY window ((RB + KH - 1) x (OW + KW - 1), zero
// outside the image) -- the pixel loop then reads dY as LDS broadcasts, no global latency in it.
template <int T, int RB>
__global__ void __launch_bounds__(256) dgrad_c1_kernel(const bf16* __restrict__ dy, int dyC, int H, int W,
                                                      const float* __restrict__ w, int KW, int pad, int OH, int OW,
                                                      int Cp, const float* alpha, bf16* __restrict__ dx) {
  extern __shared__ float lds[];
  float* wl = lds;                 // [T][Cp]
  float* win = lds + T * Cp;       // [RB + KH - 1][OW + KW - 1]
  const int KH = T / KW;
  const int rblocks = (OH + RB - 1) / RB;
  const int n = blockIdx.x / rblocks, r0 = (blockIdx.x - n * rblocks) * RB;
  const int WX = OW + KW - 1, WY = RB + KH - 1;
  for (int i = threadIdx.x; i < T * Cp; i += 256) {
    const int co = i / T, t = i - co * T;
    wl[t * Cp + co] = (float)(bf16)w[i];
  }
  const int wy0 = r0 + pad - (KH - 1), wx0 = pad - (KW - 1);
  const bf16* dyn = dy + (long)n * H * W * dyC;
  for (int i = threadIdx.x; i < WY * WX; i += 256) {
    const int wy = i / WX, wx = i - (i / WX) * WX;
    const int iy = wy + wy0, ix = wx + wx0;
    win[i] = ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) ? (float)dyn[(iy * W + ix) * dyC] : 0.f;
  }
  __syncthreads();
  const int tpp = Cp >> 3;                     // threads per pixel (host: a power of two <= 64)
  const int chunk = threadIdx.x & (tpp - 1);
  const int lane_pix = threadIdx.x / tpp;
  const int ppp = 256 / tpp;                   // pixels per pass of the block
  float wr[T][8];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const float4 lo = *reinterpret_cast<const float4*>(wl + t * Cp + chunk * 8);
    const float4 hi = *reinterpret_cast<const float4*>(wl + t * Cp + chunk * 8 + 4);
    wr[t][0] = lo.x; wr[t][1] = lo.y; wr[t][2] = lo.z; wr[t][3] = lo.w;
    wr[t][4] = hi.x; wr[t][5] = hi.y; wr[t][6] = hi.z; wr[t][7] = hi.w;
  }
  const float al = alpha ? alpha[0] : 1.f;
  const int rows = OH - r0 < RB ? OH - r0 : RB;
  const int npx = rows * OW;
  bf16* dxn = dx + ((long)n * OH + r0) * OW * Cp + chunk * 8;
  for (int q = lane_pix; q < npx; q += ppp) {
    const int oy = q / OW, ox = q - (q / OW) * OW;   // oy relative to r0
    // window row of tap ky: oy + (KH - 1) - ky; column: ox + (KW - 1) - kx
    const float* wp = win + (oy + KH - 1) * WX + ox + KW - 1;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int ky = t / KW, kx = t - (t / KW) * KW;
      const float v = wp[-ky * WX - kx];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v * wr[t][j];
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)(acc[j] * al);
    if (P2P_OOB_OK(30, ((long)n * OH + r0) * OW * Cp + (long)q * Cp + chunk * 8, 8, (long)(n + 1) * OH * OW * Cp))
      *reinterpret_cast<bf16x8*>(dxn + (long)q * Cp) = o;
  }
}

}  // namespace p2p

// dY [N][H][W][dyC] (channel 0 live), w the fp32 master weight [Cp][KH][KW] (the conv's
// [1][Cin][KH][KW]), dX [N][OH][OW][Cp]; T = KH * KW = 16.  -2: geometry not covered.
extern "C" int p2p_dgrad_c1(const void* dy, int dyC, int N, int H, int W, const float* w, int KH, int KW, int pad,
                            int OH, int OW, int Cp, const float* alpha, void* dx, hipStream_t st) {
  using namespace p2p;
  constexpr int RB = 16;
  const int tpp = Cp / 8;
  if (KH * KW != 16 || KW < 1 || Cp % 8 || tpp > 64 || (tpp & (tpp - 1))) return -2;
  const size_t lds = (16 * (size_t)Cp + (size_t)(RB + KH - 1) * (OW + KW - 1)) * sizeof(float);
  if (lds > 64 * 1024) return -2;
  const long blocks = (long)N * ((OH + RB - 1) / RB);
  hipLaunchKernelGGL((dgrad_c1_kernel<16, RB>), dim3((unsigned)blocks), dim3(256), lds, st,
                     static_cast<const bf16*>(dy), dyC, H, W, w, KW, pad, OH, OW, Cp, alpha, static_cast<bf16*>(dx));
  return (int)hipGetLastError();
}
