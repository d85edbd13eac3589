// Halo-tile weight gradient for large-kernel, few-channel stride-1 convolutions (gfx950):
// the wgrad twin of csrc/halo_kxk.hip (family R's 9x9 full-resolution layers).
//
//   dW[co][t][ci] = sum_p dY[p][co] * Xv[p + off(t)][ci]      (Xv: padded / upsampled input)
//
// As a GEMM over the im2col matrix (conv_wgrad.hip) the 81 shifted copies of X are gathered
// from L2 for 8-32 output channels: ~9 TF/s on the 32 -> 3 layer.  Here a block owns a 16 x 16
// tile of dY pixels, stages that tile and its (16 + K - 1)^2 input halo ONCE per tile
// (global_load_lds, 2-stage ring), and every wave accumulates a fixed quarter of the taps for
// all channel pairs in registers across all the tiles it walks (persistent blocks).  The MFMA
// reduces over pixels, so both operands are read TRANSPOSED out of the pixel-major images with
// ds_read_b64_tr_b16 (4 pixels x 16 channels per 16-lane group, delivered channel-per-lane):
// the tap shift is a per-lane pixel offset and needs no alignment beyond 8 bytes.  Each block
// writes one fp32 slab [R][K*K*C]; wgrad_reduce (conv_wgrad.hip) sums the slabs in a fixed
// order into the PyTorch-layout gradient.
//
// Banking: a 32-lane half of a transposed read covers pixels P..P+3 and P+8..P+11; pixel
// slots (16 channels per pixel) or 16-B chunks (32 channels per pixel) are XOR-swizzled with
// pixel bit 3 so the two quads land on different banks.
#include "conv.h"
#include "common.h"

namespace p2p {

namespace {

__device__ __forceinline__ void glds16w(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(lds_wave_base), 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vmw() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ s16x4 tr_read(const char* lds_byte) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(lds_byte));
}

// 16-B unit index of (pixel, chunk) in an image with CH channels per pixel (16 or 32)
template <int CH>
__device__ __forceinline__ int wmask(int hp) {   // chunk XOR of a pixel (CH >= 32)
  if constexpr (CH == 64) return (((hp >> 1) & 1) << 1) | (((hp >> 3) & 1) << 2);
  else return ((hp >> 3) & 1) << 1;
}
template <int CH>
__device__ __forceinline__ int wunit(int hp, int c) {
  if constexpr (CH >= 32) return hp * (CH / 8) + (c ^ wmask<CH>(hp));
  else return (hp ^ (((hp >> 3) & 1) << 2)) * 2 + c;
}

}  // namespace

template <int KS, int CIN, int RL>
struct HaloW {
  static constexpr int KK = KS * KS;
  static constexpr int HT = 16;
  static constexpr int HP = HT + KS - 1;
  // LDS row stride (pixels): K-steps advance 2 rows, so 2 * HPS = 0 mod 16 leaves every
  // swizzle (pixel bits < 4) unchanged -- the read offsets are computed once per kernel
  static constexpr int HPS = (HP + 7) / 8 * 8;
  static constexpr int HPIX = HP * HPS;
  static constexpr int XCPP = CIN / 8;
  static constexpr int GCPP = RL / 8;
  static constexpr int XLD = (HPIX * XCPP + 255) / 256;
  static constexpr int GLD = 256 * GCPP / 256;
  static constexpr int XUNITS = XLD * 256;
  static constexpr int STAGE_UNITS = XUNITS + GLD * 256;
  static constexpr int STAGE_BYTES = STAGE_UNITS * 16;
  static constexpr int CB = CIN / 16, RB = RL / 16;
  static constexpr int ITEMS = KK * CB;          // (tap, 16-channel block) pairs
  static constexpr int IPW = (ITEMS + 3) / 4;    // items per wave: i = wid + 4u
};

template <int KS, int CIN, int RL>
__global__ void __launch_bounds__(256) halo_wgrad_kernel(HaloWArgs a) {
  using G = HaloW<KS, CIN, RL>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int my_tiles = (a.ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;

  // ---- per-lane staging units (fixed across tiles)
  int hy[G::XLD], hx[G::XLD], hc[G::XLD];
#pragma unroll
  for (int j = 0; j < G::XLD; ++j) {
    const int e = (j * 4 + wid) * 64 + lane;
    int hp, c;
    if constexpr (CIN >= 32) {
      hp = e / G::XCPP;
      c = (e % G::XCPP) ^ wmask<CIN>(hp);
    } else {
      const int slot = e >> 1;
      hp = slot ^ (((slot >> 3) & 1) << 2);   // the swizzle is an involution
      c = e & 1;
    }
    const int hxx = hp % G::HPS;
    hy[j] = hp < G::HPIX && hxx < G::HP ? hp / G::HPS : -100000;   // padding column: zero
    hx[j] = hxx;
    hc[j] = c;
  }
  int gp[G::GLD], gc[G::GLD];
#pragma unroll
  for (int j = 0; j < G::GLD; ++j) {
    const int e = (j * 4 + wid) * 64 + lane;
    if constexpr (RL == 32) {
      gp[j] = e >> 2;
      gc[j] = (e & 3) ^ wmask<32>(gp[j]);
    } else {
      const int slot = e >> 1;
      gp[j] = slot ^ (((slot >> 3) & 1) << 2);
      gc[j] = e & 1;
    }
  }
  const int VH = a.H * a.up, VW = a.W * a.up;
  const int tiles_img = a.tiles_x * a.tiles_y;
  auto tile_origin = [&](int k, int& n, int& oy0, int& ox0) {
    const int t = (int)blockIdx.x + k * (int)gridDim.x;
    n = t / tiles_img;
    const int r = t - n * tiles_img;
    oy0 = (r / a.tiles_x) * G::HT;
    ox0 = (r % a.tiles_x) * G::HT;
  };
  auto issue = [&](int it, int stage) {
    int n, oy0, ox0;
    tile_origin(it, n, oy0, ox0);
    bf16* dst = reinterpret_cast<bf16*>(smem + stage * G::STAGE_BYTES);
#pragma unroll
    for (int j = 0; j < G::XLD; ++j) {
      int iy = oy0 - a.pad + hy[j], ix = ox0 - a.pad + hx[j];
      if (a.reflect) {
        iy = iy < 0 ? -iy : (iy >= VH ? 2 * (VH - 1) - iy : iy);
        ix = ix < 0 ? -ix : (ix >= VW ? 2 * (VW - 1) - ix : ix);
      }
      const bool inb = hy[j] >= 0 && (unsigned)iy < (unsigned)VH && (unsigned)ix < (unsigned)VW;
      const int sy = a.up == 2 ? iy >> 1 : iy, sx = a.up == 2 ? ix >> 1 : ix;
      const bf16* g = inb ? a.x + ((long)(n * a.H + sy) * a.W + sx) * CIN + hc[j] * 8 : a.zero;
      glds16w(g, dst + (j * 4 + wid) * 64 * 8);
    }
#pragma unroll
    for (int j = 0; j < G::GLD; ++j) {
      const int oy = oy0 + (gp[j] >> 4), ox = ox0 + (gp[j] & 15);
      const bool inb = oy < a.OH && ox < a.OW && gc[j] * 8 < a.R;
      const bf16* g = inb ? a.gy + (((long)n * a.OH + oy) * a.OW + ox) * a.R + gc[j] * 8 : a.zero;
      glds16w(g, dst + (G::XUNITS + (j * 4 + wid) * 64) * 8);
    }
  };

  f32x4 acc[G::IPW][G::RB];
#pragma unroll
  for (int u = 0; u < G::IPW; ++u)
#pragma unroll
    for (int rb = 0; rb < G::RB; ++rb) acc[u][rb] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read lane roles: group g = lane / 16 takes k = 8g .. 8g + 7 of a 32-pixel
  // K-step (tile rows 2j + (g >> 1), columns 8 (g & 1) + 4 r + q, r = read 0 / 1);
  // lane 4q + p of the group addresses pixel q, channels 4p .. 4p + 3 of a 16-channel block
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int prow = g >> 1, pcol = 8 * (g & 1) + q;
  const int pch = (p >> 1), phalf = (p & 1) * 8;   // chunk within a 16-channel block, byte half

  // read offsets (bytes) of K-step 0; K-step j adds j * XSTEP / YSTEP (same swizzle)
  constexpr int XSTEP = 2 * G::HPS * G::XCPP * 16, YSTEP = 32 * G::GCPP * 16;
  int ax0[G::IPW], ax1[G::IPW];
#pragma unroll
  for (int u = 0; u < G::IPW; ++u) {
    const int item = min(wid + 4 * u, G::ITEMS - 1);
    const int t = item / G::CB, cb = item % G::CB;
    const int hp = prow * G::HPS + pcol + (t / KS) * G::HPS + (t % KS);
    ax0[u] = wunit<CIN>(hp, cb * 2 + pch) * 16 + phalf;
    ax1[u] = wunit<CIN>(hp + 4, cb * 2 + pch) * 16 + phalf;
  }
  int gy0[G::RB], gy1[G::RB];
#pragma unroll
  for (int rb = 0; rb < G::RB; ++rb) {
    const int gpx = prow * 16 + pcol;
    gy0[rb] = wunit<RL>(gpx, rb * 2 + pch) * 16 + phalf;
    gy1[rb] = wunit<RL>(gpx + 4, rb * 2 + pch) * 16 + phalf;
  }

  if (my_tiles > 0) issue(0, 0);
  for (int it = 0; it < my_tiles; ++it) {
    const int stage = it & 1;
    if (it + 1 < my_tiles) {
      issue(it + 1, stage ^ 1);
      wait_vmw<G::XLD + G::GLD>();
    } else {
      wait_vmw<0>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const char* X = smem + stage * G::STAGE_BYTES;
    const char* Y = X + G::XUNITS * 16;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bf16x8 bfr[G::RB];
#pragma unroll
      for (int rb = 0; rb < G::RB; ++rb) {
        const s16x4 b0 = tr_read(Y + gy0[rb] + j * YSTEP);
        const s16x4 b1 = tr_read(Y + gy1[rb] + j * YSTEP);
        bfr[rb] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int u = 0; u < G::IPW; ++u) {
        if (u == G::IPW - 1 && wid + 4 * u >= G::ITEMS) break;   // wave-uniform: EXEC stays full
        const s16x4 a0 = tr_read(X + ax0[u] + j * XSTEP);
        const s16x4 a1 = tr_read(X + ax1[u] + j * XSTEP);
        const bf16x8 af = __builtin_bit_cast(bf16x8, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int rb = 0; rb < G::RB; ++rb)
          acc[u][rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[rb], acc[u][rb], 0, 0, 0);
      }
    }
    __builtin_amdgcn_s_barrier();   // every wave done with this stage before it is refilled
  }

  // ---- this block's slab: ws[block][co][t * CIN + ci]
  float* slab = a.ws + (long)blockIdx.x * a.R * (G::KK * CIN);
  const int col = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int u = 0; u < G::IPW; ++u) {
    const int item = wid + 4 * u;
    if (item >= G::ITEMS) break;
    const int t = item / G::CB, cb = item % G::CB;
#pragma unroll
    for (int rb = 0; rb < G::RB; ++rb) {
      const int co = rb * 16 + col;
      if (co >= a.R) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        slab[(long)co * (G::KK * CIN) + t * CIN + cb * 16 + kq * 4 + r] = acc[u][rb][r];
    }
  }
}

template <int KS, int CIN, int RL>
static int launch_halo_wgrad(const HaloWArgs& a, int blocks, hipStream_t st) {
  using G = HaloW<KS, CIN, RL>;
  constexpr int smem = 2 * G::STAGE_BYTES;
  static_assert(smem <= 163840, "halo_wgrad: LDS budget");
  static std::atomic<uint64_t> attr_mask{0};
  smem_attr_once(reinterpret_cast<const void*>(&halo_wgrad_kernel<KS, CIN, RL>), smem, attr_mask);
  hipLaunchKernelGGL((halo_wgrad_kernel<KS, CIN, RL>), dim3(blocks), dim3(256), smem, st, a);
  return (int)hipGetLastError();
}

}  // namespace p2p

// returns -2 when the geometry is not covered (caller falls back to the GEMM wgrad)
extern "C" int p2p_halo_wgrad(const p2p::HaloWArgs* a, int KS, int blocks, hipStream_t st) {
  using namespace p2p;
  if (a->up != 1 && a->up != 2) return -2;
  if (a->reflect && (a->pad >= a->H * a->up || a->pad >= a->W * a->up)) return -2;
  if (KS == 9) {
    if (a->C == 32 && a->R <= 16) return launch_halo_wgrad<9, 32, 16>(*a, blocks, st);
    if (a->C == 16 && a->R <= 16) return launch_halo_wgrad<9, 16, 16>(*a, blocks, st);
    if (a->C == 16 && a->R == 32) return launch_halo_wgrad<9, 16, 32>(*a, blocks, st);
  }
  if (KS == 3 && a->C == 64) {
    if (a->R <= 16) return launch_halo_wgrad<3, 64, 16>(*a, blocks, st);
    if (a->R == 32) return launch_halo_wgrad<3, 64, 32>(*a, blocks, st);
  }
  return -2;
}
