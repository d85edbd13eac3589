// Standalone check of p2p_halo_kxk against a CPU reference (build: hipcc -O3
// --offload-arch=gfx950 -I csrc tools/probes/halo_kxk_probe.hip csrc/halo_kxk.hip).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include "conv.h"

static float bf2f(__bf16 v) { return (float)v; }

int main(int argc, char** argv) {
  const int C = argc > 1 ? atoi(argv[1]) : 8, Cout = argc > 2 ? atoi(argv[2]) : 8;
  const int refl = argc > 3 ? atoi(argv[3]) : 0, up = argc > 4 ? atoi(argv[4]) : 1;
  const int N = 1, H = 20, W = 20, K = 9, pad = 4;
  const int OH = H * up, OW = W * up, VH = H * up, VW = W * up;
  std::vector<__bf16> x(N * H * W * C), w(Cout * K * K * C);
  srand(1);
  for (auto& v : x) v = (__bf16)((rand() % 17 - 8) / 8.f);
  for (auto& v : w) v = (__bf16)((rand() % 17 - 8) / 8.f);
  std::vector<float> ref(N * OH * OW * Cout, 0.f);
  for (int oy = 0; oy < OH; ++oy)
    for (int ox = 0; ox < OW; ++ox)
      for (int co = 0; co < Cout; ++co) {
        float s = 0.f;
        for (int ky = 0; ky < K; ++ky)
          for (int kx = 0; kx < K; ++kx) {
            int iy = oy - pad + ky, ix = ox - pad + kx;
            if (refl) {
              iy = iy < 0 ? -iy : (iy >= VH ? 2 * (VH - 1) - iy : iy);
              ix = ix < 0 ? -ix : (ix >= VW ? 2 * (VW - 1) - ix : ix);
            }
            if (iy < 0 || iy >= VH || ix < 0 || ix >= VW) continue;
            iy /= up;
            ix /= up;
            for (int c = 0; c < C; ++c) s += bf2f(x[(iy * W + ix) * C + c]) * bf2f(w[(co * K * K + ky * K + kx) * C + c]);
          }
        ref[(oy * OW + ox) * Cout + co] = s;
      }
  __bf16 *dx, *dw, *dy, *dz;
  hipMalloc(&dx, x.size() * 2);
  hipMalloc(&dw, w.size() * 2);
  hipMalloc(&dy, ref.size() * 2);
  hipMalloc(&dz, 256);
  hipMemset(dz, 0, 256);
  hipMemset(dy, 0, ref.size() * 2);
  hipMemcpy(dx, x.data(), x.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dw, w.data(), w.size() * 2, hipMemcpyHostToDevice);
  p2p::HaloKArgs a{};
  a.x = dx; a.C = C; a.N = N; a.H = H; a.W = W; a.up = up; a.pad = pad; a.reflect = refl; a.flip = 0;
  a.OH = OH; a.OW = OW; a.w = dw; a.bias = nullptr; a.Cout = Cout; a.act_out = 0; a.y = dy; a.zero = dz;
  a.tiles_x = (OW + 15) / 16; a.tiles_y = (OH + 15) / 16; a.ntiles = N * a.tiles_x * a.tiles_y;
  int rc = p2p_halo_kxk(&a, 9, a.ntiles, 0);
  hipError_t e = hipDeviceSynchronize();
  std::vector<__bf16> y(ref.size());
  hipMemcpy(y.data(), dy, y.size() * 2, hipMemcpyDeviceToHost);
  double md = 0, mr = 0;
  for (size_t i = 0; i < y.size(); ++i) {
    md = fmax(md, fabs(bf2f(y[i]) - ref[i]));
    mr = fmax(mr, fabs(ref[i]));
  }
  printf("C=%d Cout=%d rc=%d err=%s maxdiff=%g maxref=%g y0=%g ref0=%g\n", C, Cout, rc, hipGetErrorString(e), md, mr,
         bf2f(y[0]), ref[0]);
  return 0;
}
