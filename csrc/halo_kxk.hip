// Halo-tile direct conv for large-kernel, few-channel stride-1 convolutions (gfx950).
//
// Family R's full-resolution 9x9 layers -- the generator's first conv (12 -> 32 channels on
// the pixel-unshuffled, nearest-upsampled image, reflect pad 4), its last conv (32 -> 3,
// reflect pad 4) and that layer's input gradient (3 -> 32, a stride-1 transposed conv) --
// carry 0.25-1.3 kFLOP per output pixel but only 8-32 channels per operand.  As implicit
// GEMMs (conv_fwd.hip) every input pixel is gathered from L2 once per TAP (81x) for 8-32
// MACs per element: ~100 TF/s, 20 % of the family-R step.
//
// Here a block owns a 16 x 16 tile of outputs and stages its (16 + K - 1)^2 input halo ONCE
// (global_load_lds; reflect / zero pad and nearest upsample resolved in the per-lane source
// address), with the whole weight resident in LDS.  The MFMA K = 32 of one
// v_mfma_f32_16x16x32_bf16 is a "slice" of 32 / C taps x C channels: every lane gathers its
// 8-channel piece of the A fragment at its own tap's pixel offset in the halo image, so
// 8- and 16-channel inputs still fill the K dimension.  Persistent blocks walk the tiles with
// the next halo in flight (2-stage ring, counted vmcnt + raw s_barrier).
//
// LDS banking: both operands are read as 2 x ds_read_b64 per fragment (one 32-lane group per
// cycle pair).  A pixel's C / 8 16-B chunks are XOR-swizzled with pixel bits so 16 consecutive
// pixels x one chunk index cover the 16 slots of a 256-B bank row, and lanes with odd kq read
// their two 8-B halves in the opposite order (the matching B lanes do the same, so the k
// order inside the MFMA stays consistent): conflict-free for every tap shift.
#include "bounds.h"
#include "conv.h"
#include "common.h"

namespace p2p {

namespace {

__device__ __forceinline__ void glds16k(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(lds_wave_base), 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vmk() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// 8 bf16 of one 16-B LDS unit as two 8-B reads, halves swapped when `swap`
__device__ __forceinline__ bf16x8 lds_frag(const bf16* base_unit, bool swap) {
  const bf16x4* p = reinterpret_cast<const bf16x4*>(base_unit);
  const bf16x4 a = p[swap ? 1 : 0];
  const bf16x4 b = p[swap ? 0 : 1];
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// the same from a 32-bit LDS byte address (an opaque register: see the slice loop)
typedef __attribute__((address_space(3))) const bf16x4 lds_bf16x4;
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const void*)p));
}
__device__ __forceinline__ bf16x8 lds_frag_at(uint32_t addr, bool swap) {
  const lds_bf16x4* p = (const lds_bf16x4*)(uintptr_t)addr;
  const bf16x4 a = p[swap ? 1 : 0];
  const bf16x4 b = p[swap ? 0 : 1];
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

}  // namespace

template <int KS, int CIN>
struct HaloK {
  static constexpr int KK = KS * KS;
  // an MFMA K-slice is 32 / CIN taps (CIN <= 32) or 1/SPT of a tap (CIN = 32 * SPT)
  static constexpr int TPS = CIN <= 32 ? 32 / CIN : 1;
  static constexpr int SPT = CIN <= 32 ? 1 : CIN / 32;
  static constexpr int S = CIN <= 32 ? (KK + TPS - 1) / TPS : KK * SPT;   // K-slices
  static constexpr int CPP = CIN / 8;                // 16-B chunks per pixel
  static constexpr int LSH = CPP == 8 ? 1 : (CPP == 4 ? 2 : (CPP == 2 ? 3 : 4));   // log2(16 / CPP)
  static constexpr int HT = 16;
  static constexpr int HP = HT + KS - 1;             // halo edge
  // LDS row stride (pixels): a wave's 4 output rows are 4 apart, so 4 * HPS = 0 mod 16 keeps
  // the chunk swizzle (pixel bits < 4) identical on all four -- one address per K-slice
  static constexpr int HPS = (HP + 3) / 4 * 4;
  static constexpr int HPIX = HP * HPS;
  static constexpr int HUNITS = HPIX * CPP;
  static constexpr int HLD = (HUNITS + 255) / 256;   // glds per lane per stage
  static constexpr int STAGE_UNITS = HLD * 256;
  static constexpr int STAGE_BYTES = STAGE_UNITS * 16;
  __device__ static int aslot(int hp, int c) {
    return hp * CPP + (c ^ ((hp >> LSH) & (CPP - 1)));
  }
};

template <int KS, int CIN, int NBLK>
__global__ void __launch_bounds__(256) halo_kxk_kernel(HaloKArgs a) {
  using G = HaloK<KS, CIN>;
  constexpr int BUNITS = G::S * NBLK * 16 * 4;
  constexpr int BUNITS_PAD = (BUNITS + 255) / 256 * 256;
  constexpr int LDCS = NBLK * 16 + 8;                // epilogue staging row (bf16)
  constexpr int EPI_BYTES = 256 * LDCS * 2;
  constexpr bool EPI_IN_STAGE = EPI_BYTES <= G::STAGE_BYTES;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* As = reinterpret_cast<bf16*>(smem);                                 // 2 stages
  bf16* Bs = reinterpret_cast<bf16*>(smem + 2 * G::STAGE_BYTES);            // [S][NBLK][16][4 units]
  bf16* Ed = reinterpret_cast<bf16*>(smem + 2 * G::STAGE_BYTES + BUNITS_PAD * 16);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int my_tiles = (a.ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  if (my_tiles <= 0) return;

  // ---- resident weights: unit ((s * NBLK + nb) * 16 + n) * 4 + slot holds logical k-chunk
  // c = slot ^ ((n >> 2) & 3) of slice s: tap s * TPS + 8c / CIN, channels (8c % CIN) + 0..7
  // (CIN > 32: tap s / SPT, channels 8 * ((s % SPT) * 4 + c) + 0..7)
  for (int e0 = wid * 64; e0 < BUNITS_PAD; e0 += 256) {
    const int e = e0 + lane;
    const int n = (e >> 2) & 15, sn = e >> 6;
    const int nb = sn % NBLK, s = sn / NBLK;
    const int c = (e & 3) ^ ((n >> 2) & 3);
    const int t = CIN <= 32 ? s * G::TPS + (8 * c) / CIN : s / G::SPT;
    const int ch = CIN <= 32 ? (8 * c) % CIN : 8 * ((s % G::SPT) * 4 + c);
    const int co = nb * 16 + n;
    const int tw = a.flip ? G::KK - 1 - t : t;
    const bool ok = e < BUNITS && co < a.Cout && t < G::KK;
    glds16k(ok ? a.w + ((long)co * G::KK + tw) * CIN + ch : a.zero, Bs + e0 * 8);
  }

  // ---- per-lane halo units (fixed across tiles)
  int hy[G::HLD], hx[G::HLD], hc[G::HLD];
#pragma unroll
  for (int j = 0; j < G::HLD; ++j) {
    const int e = (j * 4 + wid) * 64 + lane;
    const int hp = e / G::CPP;
    const int hxx = hp % G::HPS;
    hy[j] = hp < G::HPIX && hxx < G::HP ? hp / G::HPS : -100000;   // padding column: zero
    hx[j] = hxx;
    hc[j] = (e % G::CPP) ^ ((hp >> G::LSH) & (G::CPP - 1));
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
    bf16* dst = As + stage * (G::STAGE_UNITS * 8);
#pragma unroll
    for (int j = 0; j < G::HLD; ++j) {
      int iy = oy0 - a.pad + hy[j], ix = ox0 - a.pad + hx[j];
      bool inb;
      if (a.reflect) {
        iy = iy < 0 ? -iy : (iy >= VH ? 2 * (VH - 1) - iy : iy);
        ix = ix < 0 ? -ix : (ix >= VW ? 2 * (VW - 1) - ix : ix);
      }
      inb = hy[j] >= 0 && (unsigned)iy < (unsigned)VH && (unsigned)ix < (unsigned)VW;
      const int sy = a.up == 2 ? iy >> 1 : iy, sx = a.up == 2 ? ix >> 1 : ix;
      const bf16* g = inb ? a.x + ((long)(n * a.H + sy) * a.W + sx) * CIN + hc[j] * 8 : a.zero;
      glds16k(g, dst + (j * 4 + wid) * 64 * 8);
    }
  };

  f32x4 acc[4][NBLK];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int nb = 0; nb < NBLK; ++nb) acc[i][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int px = lane & 15, kq = lane >> 4;
  const bool hswap = kq & 1;
  // this lane's tap within a slice and chunk within the tap
  const int tsub = CIN <= 32 ? kq / G::CPP : 0, csub0 = CIN <= 32 ? kq % G::CPP : kq;
  const int bslot = kq ^ ((px >> 2) & 3);
  // the wave's output rows are wid + 4i (i < 4): row i's A fragment sits ISTRIDE elements
  // after row 0's (same swizzle, see HPS)
  constexpr int ISTRIDE = 4 * G::HPS * G::CPP * 8;
  const int rowbase = wid * G::HPS + px;

  issue(0, 0);
  for (int it = 0; it < my_tiles; ++it) {
    const int stage = it & 1;
    if (it + 1 < my_tiles) {
      issue(it + 1, stage ^ 1);
      wait_vmk<G::HLD>();
    } else {
      wait_vmk<0>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const bf16* A = As + stage * (G::STAGE_UNITS * 8);
    // the lane's tap walks t = s * TPS + tsub incrementally (loop-carried: the compiler must
    // not hoist 81 per-slice offsets into registers across the tile loop)
    int dx = tsub % KS, toff = (tsub / KS) * G::HPS + tsub % KS, sub = 0;
    const bf16* bp = Bs + (px * 4 + bslot) * 8;
#pragma unroll 2
    for (int s = 0; s < G::S; ++s) {
      const int to = CIN > 32 || s * G::TPS + tsub < G::KK ? toff : 0;   // padding tap: zero weights
      const int csub = csub0 + sub * 4;
      // every fragment's address goes through its own opaque register: left visible, hipcc
      // pairs reads 512 B apart into ds_read2st64_b64, whose 16-lane / 32-bank service breaks
      // the 64-bank conflict-free layout above (6-7 conflict cycles per LDS instruction in the
      // round-5 family-R roofline); as separate ds_read_b64 they are conflict-free
      bf16x8 bfr[NBLK];
#pragma unroll
      for (int nb = 0; nb < NBLK; ++nb) {
        uint32_t bq = lds_u32(bp + nb * 16 * 4 * 8);
#ifndef P2P_HALO_NOLAUNDER   // (diagnostic build: the round-5 paired reads, for the A/B)
        asm volatile("" : "+v"(bq));
#endif
        bfr[nb] = lds_frag_at(bq, hswap);
      }
      const bf16* a0 = A + G::aslot(rowbase + to, csub) * 8;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint32_t aq = lds_u32(a0 + i * ISTRIDE);
#ifndef P2P_HALO_NOLAUNDER
        asm volatile("" : "+v"(aq));
#endif
        const bf16x8 af = lds_frag_at(aq, hswap);
#pragma unroll
        for (int nb = 0; nb < NBLK; ++nb)
          acc[i][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[nb], acc[i][nb], 0, 0, 0);
      }
      bp += NBLK * 16 * 4 * 8;
      if (CIN > 32 && ++sub < G::SPT) continue;
      sub = 0;
      dx += G::TPS;
      toff += G::TPS;
#pragma unroll
      for (int w = 0; w < (G::TPS + KS - 1) / KS; ++w)   // TPS may exceed KS (3x3, 8 ch)
        if (dx >= KS) {
          dx -= KS;
          toff += G::HPS - KS;
        }
    }
    __builtin_amdgcn_s_barrier();   // every wave done reading this stage
    // ---- epilogue: bias + act -> bf16 staging [256 px][LDCS] -> 16-B NHWC stores
    int n, oy0, ox0;
    tile_origin(it, n, oy0, ox0);
    bf16* Cs = EPI_IN_STAGE ? As + stage * (G::STAGE_UNITS * 8) : Ed;
#pragma unroll
    for (int nb = 0; nb < NBLK; ++nb) {
      const int co = nb * 16 + px;
      const float bj = (a.bias && co < a.Cout) ? a.bias[co] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = (wid + 4 * i) * 16 + kq * 4 + r;
          Cs[q * LDCS + co] = (bf16)act_fwd(acc[i][nb][r] + bj, a.act_out);
        }
        acc[i][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int upp = a.Cout / 8;             // 16-B units per output pixel
    for (int u = tid; u < 256 * upp; u += 256) {
      const int q = u / upp, k = u - q * upp;
      const int oy = oy0 + (q >> 4), ox = ox0 + (q & 15);
      if (oy < a.OH && ox < a.OW) {
        __bf16* dst = a.y + (((long)n * a.OH + oy) * a.OW + ox) * a.Cout + k * 8;
        if (a.fold_buf) {   // interior -> the real grid; frame -> fold_buf (fold_band folds it)
          const int iy = oy - a.fold_p, ix = ox - a.fold_p;
          if ((unsigned)iy < (unsigned)a.fold_H && (unsigned)ix < (unsigned)a.fold_W) {
            const long o = (((long)n * a.fold_H + iy) * a.fold_W + ix) * a.Cout + k * 8;
            dst = P2P_OOB_OK(4, o, 8, (long)a.N * a.fold_H * a.fold_W * a.Cout) ? a.y + o : nullptr;
          } else {
            const long o = (((long)n * a.OH + oy) * a.OW + ox) * a.Cout + k * 8;
            dst = P2P_OOB_OK(4, o, 8, (long)a.N * a.OH * a.OW * a.Cout) ? a.fold_buf + o : nullptr;
          }
        }
        if (dst) *reinterpret_cast<u32x4*>(dst) = *reinterpret_cast<const u32x4*>(Cs + q * LDCS + k * 8);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // staging read before the stage is re-filled
  }
}

template <int KS, int CIN, int NBLK>
static int launch_halo_kxk(const HaloKArgs& a, int blocks, hipStream_t st) {
  using G = HaloK<KS, CIN>;
  constexpr int BUNITS = G::S * NBLK * 16 * 4;
  constexpr int BUNITS_PAD = (BUNITS + 255) / 256 * 256;
  constexpr int EPI_BYTES = 256 * (NBLK * 16 + 8) * 2;
  constexpr int smem = 2 * G::STAGE_BYTES + BUNITS_PAD * 16 + (EPI_BYTES <= G::STAGE_BYTES ? 0 : EPI_BYTES);
  static_assert(smem <= 163840, "halo_kxk: LDS budget");
  static std::atomic<uint64_t> attr_mask{0};
  smem_attr_once(reinterpret_cast<const void*>(&halo_kxk_kernel<KS, CIN, NBLK>), smem, attr_mask);
  hipLaunchKernelGGL((halo_kxk_kernel<KS, CIN, NBLK>), dim3(blocks), dim3(256), smem, st, a);
  return (int)hipGetLastError();
}

}  // namespace p2p

// returns -2 when the geometry is not covered (caller falls back to the implicit GEMM)
extern "C" int p2p_halo_kxk(const p2p::HaloKArgs* a, int KS, int blocks, hipStream_t st) {
  using namespace p2p;
  if (a->Cout % 8 || a->Cout <= 0 || a->Cout > 64) return -2;
  if (a->up != 1 && a->up != 2) return -2;
  if (a->reflect && (a->pad >= a->H * a->up || a->pad >= a->W * a->up)) return -2;
  const int nblk = (a->Cout + 15) / 16;
  if (KS == 9) {
    if (nblk > 2) return -2;
    const bool wide = nblk == 2;
    switch (a->C) {
      case 32: return wide ? -2 : launch_halo_kxk<9, 32, 1>(*a, blocks, st);
      case 16: return wide ? launch_halo_kxk<9, 16, 2>(*a, blocks, st) : launch_halo_kxk<9, 16, 1>(*a, blocks, st);
      case 8: return wide ? launch_halo_kxk<9, 8, 2>(*a, blocks, st) : launch_halo_kxk<9, 8, 1>(*a, blocks, st);
      default: return -2;
    }
  }
  if (KS == 3) {
    // 64-channel inputs into <= 32 outputs (G.deconv2, VGG conv1_1's input gradient).  The
    // 8-channel image into 64 (VGG conv1_1) measured 1.6x slower than the implicit GEMM: its
    // 3 K-slices per tile leave the 64-channel epilogue stores exposed
    if (a->C == 64 && nblk == 1) return launch_halo_kxk<3, 64, 1>(*a, blocks, st);
    if (a->C == 64 && nblk == 2) return launch_halo_kxk<3, 64, 2>(*a, blocks, st);
    return -2;
  }
  return -2;
}
