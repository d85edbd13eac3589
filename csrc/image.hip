// Packed-image layers of the pix2pix step (the generator's last transposed conv and the
// discriminator's first conv's input gradient), MI355X-native:
//
// A stride-2, 4x4, pad-1 transposed conv onto a 3-channel image, out[2q + r] =
// sum_t x[q + t] W[k(r, t)], has four output parity classes r = (ry, rx) that each read a
// 2x2 window of the input grid; together they read the 3x3 window around q.  So the whole
// layer is ONE 3x3 pad-1 conv over the input grid with 4 classes x 3 channels = 12 (padded
// to 32) output columns -- a FASTK implicit GEMM (K = 9 x Cin) whose epilogue scatters each
// row's 4 x 3 values to the 2x2 output pixels (conv_dev.h, ``d2s``).  This replaces the
// tiny-Cout column GEMM (16 taps x Cout) + col2im + channel slicing, and lets the epilogue
// write the packed (A | fake) discriminator input and the L1 term directly.
//
// union_weight_kernel builds that GEMM's B operand from the fp32 transposed-conv weight
// [CinT][CoutT][4][4] (a conv's weight [Cout][Cin][4][4] read as a transposed conv gives its
// input gradient): row n = cls * 4 + j (j < nv) -> W[c][co_off + j][3 - 2uy + ry][3 - 2ux + rx]
// for the 9 union taps (uy, ux) (zero where the tap does not reach the class), k-order
// [tap][c] like every other weight image (conv_fwd.hip weight_prep).
#include "common.h"

namespace p2p {

__global__ void __launch_bounds__(256) union_weight_kernel(const float* __restrict__ w, int CinT, int CoutT,
                                                           int co_off, int nv, int Nrows, int Cpad,
                                                           const float* __restrict__ bias,
                                                           bf16* __restrict__ out, float* __restrict__ bias_out) {
  const int total = Nrows * 9 * Cpad;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
    const int c = e % Cpad;
    const int u = (e / Cpad) % 9;
    const int n = e / (Cpad * 9);
    const int cls = n >> 2, j = n & 3;
    float v = 0.f;
    if (cls < 4 && j < nv && c < CinT) {
      const int ry = cls >> 1, rx = cls & 1, uy = u / 3, ux = u % 3;
      const int ky = 3 - 2 * uy + ry, kx = 3 - 2 * ux + rx;
      const int co = co_off + j;
      if (ky >= 0 && ky < 4 && kx >= 0 && kx < 4 && co < CoutT)
        v = w[(((long)c * CoutT + co) * 4 + ky) * 4 + kx];
    }
    out[e] = (bf16)v;
    if (bias_out && u == 0 && c == 0) {
      const int co = co_off + j;
      bias_out[n] = (bias && cls < 4 && j < nv && co < CoutT) ? bias[co] : 0.f;
    }
  }
}

}  // namespace p2p

extern "C" int p2p_union_weight(const float* w, int CinT, int CoutT, int co_off, int nv, int Nrows, int Cpad,
                                const float* bias, void* out, float* bias_out, hipStream_t st) {
  const int total = Nrows * 9 * Cpad;
  const int blocks = (total + 255) / 256;
  hipLaunchKernelGGL(p2p::union_weight_kernel, dim3(blocks < 1024 ? blocks : 1024), dim3(256), 0, st, w, CinT,
                     CoutT, co_off, nv, Nrows, Cpad, bias, static_cast<p2p::bf16*>(out), bias_out);
  return (int)hipGetLastError();
}
