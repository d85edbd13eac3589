// Implicit-GEMM conv / transposed conv, global_load_lds ("LDS-DMA") pipelined variant
// (gfx950).  Same GEMM view, tile geometry, LDS image and epilogue as conv_fwd.hip; what
// differs is the staging:
//  * every 16-B operand chunk goes global -> LDS with global_load_lds_dwordx4: no VGPR
//    staging, no ds_write instructions (13 cycles each on the shared store path), and the
//    im2col gather is just a per-lane source address.  Out-of-image taps read a zero page.
//  * the LDS image must be lane-linear per wave instruction (base + lane*16), so the
//    bank-conflict XOR swizzle moves to the SOURCE side: lane (row r, slot s) fetches
//    chunk s ^ ((r>>1)&7) -- the ds_read side keeps swz() (cdna_hip_programming.md rule 21).
//  * STAGES-deep ring: tile k+STAGES-1 is issued right after the barrier that retires
//    tile k, so STAGES-1 tiles of HBM/L2 latency are hidden behind MFMAs; counted
//    s_waitcnt vmcnt(LOADS*(STAGES-2)) + raw s_barrier (never __syncthreads in the loop:
//    its implicit vmcnt(0) would drain the ring).
//  * the input ReLU is applied to the A fragments after ds_read (packed int16 max).
// Only the FAST geometry (channel groups multiple of 64) with BN >= 32 rows per pass
// is handled; everything else falls back to conv_fwd.hip.
#include "conv_dev.h"

namespace p2p {

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void glds16(const void* g, bf16* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(lds_wave_base), 16, 0, 0);
}

// FASTK: every channel group a multiple of 64 (one tap per 64-deep K tile, wave-uniform);
// otherwise (packed 8 / 16 / 24-channel image inputs) each lane splits its own chunk's k
// into (tap, channel) and k >= Kc reads zeros.
template <int BM, int BN, int WM, int WN, int MODE, int STAGES, bool FASTK, bool RELU>
__global__ void __launch_bounds__(WM * WN * 64) conv_fwd_glds_kernel(ConvFwdArgs a) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  constexpr int RPP = NT / 8;            // tile rows covered per glds pass (8 lanes per row)
  constexpr int AROWS = BM / RPP;
  constexpr int BROWS = BN / RPP;
  constexpr int LOADS = AROWS + BROWS;   // glds instructions per thread per tile
  static_assert(BM % RPP == 0 && BN % RPP == 0, "every wave issues the same glds count");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* As = reinterpret_cast<bf16*>(smem);
  bf16* Bs = As + STAGES * BM * BK;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;

  const int cls = blockIdx.z / a.splits;
  const int split = blockIdx.z % a.splits;
  const ClassGeom g = class_geom<MODE>(a, cls);
  const int ntiles = (a.Cout + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / ntiles, nt = bid % ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  if (m0 >= g.Mc) return;

  const int ktiles = (g.Kc + BK - 1) / BK;
  const int kps = (ktiles + a.splits - 1) / a.splits;
  const int kt0 = split * kps;
  const int kt1 = min(ktiles, kt0 + kps);
  if (kt0 >= kt1 && a.splits > 1) return;

  const bf16* __restrict__ x1 = static_cast<const bf16*>(a.x1);
  const bf16* __restrict__ x2 = static_cast<const bf16*>(a.x2);
  const bf16* __restrict__ w = static_cast<const bf16*>(a.w);
  const bf16* zero = static_cast<const bf16*>(a.zero);
  const int C = a.C, C1 = a.C1, C2 = a.C2;
  const int slot = lane & 7;
  const int rsub = lane >> 3;            // row within this wave's 8-row glds group
  const int ush = a.up == 2 ? 1 : 0;
  const int Hu = a.H << ush, Wu = a.W << ush;

  // A rows of this lane: row_i = wid*8 + rsub + RPP*i
  int r_img[AROWS], r_y[AROWS], r_x[AROWS], r_c[AROWS];
  const int HWq = g.Hq * g.Wq;
  const FastDiv fd_hwq = make_fastdiv((uint32_t)HWq), fd_wq = make_fastdiv((uint32_t)g.Wq);
#pragma unroll
  for (int i = 0; i < AROWS; ++i) {
    const int row = wid * 8 + rsub + RPP * i;
    const int m = m0 + row;
    const int mm = m < g.Mc ? m : 0;
    const int n = (int)fdiv((uint32_t)mm, fd_hwq);
    const int r = mm - n * HWq;
    const int qy = (int)fdiv((uint32_t)r, fd_wq);
    const int qx = r - qy * g.Wq;
    r_img[i] = n * a.H * a.W;
    if (MODE == 0) {
      r_y[i] = qy * a.stride - a.pad;
      r_x[i] = qx * a.stride - a.pad;
    } else {
      r_y[i] = qy + g.dy;
      r_x[i] = qx + g.dx;
    }
    if (m >= g.Mc) r_y[i] = -(1 << 28);
    r_c[i] = (slot ^ ((row >> 1) & 7)) * 8;   // source-side swizzle
  }
  int b_off[BROWS];
  bool b_ok[BROWS];
  const long wrow = (MODE == 0) ? (long)g.Kc : (long)a.KH * a.KW * C;
#pragma unroll
  for (int i = 0; i < BROWS; ++i) {
    const int row = wid * 8 + rsub + RPP * i;
    const int co = n0 + row;
    b_ok[i] = co < a.Cout;
    b_off[i] = (slot ^ ((row >> 1) & 7)) * 8;
  }
  const FastDiv fd_c = make_fastdiv((uint32_t)C), fd_ti = make_fastdiv((uint32_t)g.Ti);
  // FASTK A-row pointers of the current channel segment (one tap x one source tensor):
  // formed once per segment, then advanced by BK per k-tile (out-of-image rows walk the
  // zero page, which covers a whole segment: host guarantees C1, C2 <= 1024).
  const bf16* a_ptr[AROWS];
  const bf16* b_base[BROWS];
#pragma unroll
  for (int i = 0; i < BROWS; ++i) {
    const int co = n0 + wid * 8 + rsub + RPP * i;
    b_base[i] = w + (long)(b_ok[i] ? co : 0) * wrow + b_off[i];
  }

  auto issue = [&](int kt, int stage) {
    const int k0 = kt * BK;
    bf16* Ast = As + stage * BM * BK;
    bf16* Bst = Bs + stage * BN * BK;
    if constexpr (FASTK) {
      const int tap = (int)fdiv((uint32_t)k0, fd_c);
      const int ci0 = k0 - tap * C;
      const int t_y = (int)fdiv((uint32_t)tap, fd_ti);
      const int t_x = tap - t_y * g.Ti;
      if (kt == kt0 || ci0 == 0 || ci0 == C1) {
        const bool s1 = ci0 < C1;
        const bf16* src = s1 ? x1 : x2;
        const int cs = s1 ? C1 : C2;
        const int cio = s1 ? ci0 : ci0 - C1;
#pragma unroll
        for (int i = 0; i < AROWS; ++i) {
          int iy, ix;
          bool inb;
          if (MODE == 0) {
            int uy = r_y[i] + t_y, ux = r_x[i] + t_x;
            if (a.reflect && r_y[i] > -(1 << 27)) {
              uy = reflect_idx(uy, Hu);
              ux = reflect_idx(ux, Wu);
            }
            inb = (unsigned)uy < (unsigned)Hu && (unsigned)ux < (unsigned)Wu;
            iy = uy >> ush;
            ix = ux >> ush;
          } else {
            iy = r_y[i] - t_y;
            ix = r_x[i] - t_x;
            inb = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
          }
          const long off = (long)(r_img[i] + iy * a.W + ix) * cs + cio + r_c[i];
          a_ptr[i] = inb ? src + off : zero;
        }
      } else {
#pragma unroll
        for (int i = 0; i < AROWS; ++i) a_ptr[i] += BK;
      }
#pragma unroll
      for (int i = 0; i < AROWS; ++i) glds16(a_ptr[i], Ast + (wid * 8 + RPP * i) * BK);
      long woff;
      if (MODE == 0) {
        woff = k0;
      } else {
        const int ky = g.ky0 + a.stride * t_y, kx = g.kx0 + a.stride * t_x;
        woff = (long)(ky * a.KW + kx) * C + ci0;
      }
#pragma unroll
      for (int i = 0; i < BROWS; ++i) {
        const bf16* gp = b_ok[i] ? b_base[i] + woff : zero;
        glds16(gp, Bst + (wid * 8 + RPP * i) * BK);
      }
    } else {
#pragma unroll
      for (int i = 0; i < AROWS; ++i) {
        const int k = k0 + r_c[i];
        const int tap = (int)fdiv((uint32_t)k, fd_c);
        const int ci = k - tap * C;
        const int t_y = (int)fdiv((uint32_t)tap, fd_ti);
        const int t_x = tap - t_y * g.Ti;
        const bool s1 = ci < C1;
        const bf16* src = s1 ? x1 : x2;
        const int cs = s1 ? C1 : C2;
        const int cio = s1 ? ci : ci - C1;
        int iy, ix;
        bool inb;
        if (MODE == 0) {
          int uy = r_y[i] + t_y, ux = r_x[i] + t_x;
          if (a.reflect && r_y[i] > -(1 << 27)) {
            uy = reflect_idx(uy, Hu);
            ux = reflect_idx(ux, Wu);
          }
          inb = (unsigned)uy < (unsigned)Hu && (unsigned)ux < (unsigned)Wu;
          iy = uy >> ush;
          ix = ux >> ush;
        } else {
          iy = r_y[i] - t_y;
          ix = r_x[i] - t_x;
          inb = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
        }
        inb = inb && k < g.Kc;
        const long off = (long)(r_img[i] + iy * a.W + ix) * cs + cio;
        const bf16* gp = inb ? src + off : zero;
        glds16(gp, Ast + (wid * 8 + RPP * i) * BK);
      }
#pragma unroll
      for (int i = 0; i < BROWS; ++i) {
        const int co = n0 + wid * 8 + rsub + RPP * i;
        const int k = k0 + b_off[i];
        long woff;
        if (MODE == 0) {
          woff = k;
        } else {
          const int tap = (int)fdiv((uint32_t)k, fd_c);
          const int ci = k - tap * C;
          const int t_y = (int)fdiv((uint32_t)tap, fd_ti);
          const int t_x = tap - t_y * g.Ti;
          const int ky = g.ky0 + a.stride * t_y, kx = g.kx0 + a.stride * t_x;
          woff = (long)(ky * a.KW + kx) * C + ci;
        }
        const bf16* gp = (b_ok[i] && k < g.Kc) ? w + co * wrow + woff : zero;
        glds16(gp, Bst + (wid * 8 + RPP * i) * BK);
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: STAGES-1 tiles in flight
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (kt0 + s < kt1) issue(kt0 + s, s);

  int stage = 0;
  for (int kt = kt0; kt < kt1; ++kt) {
    // retire tile kt (this wave's share), then the barrier makes every wave's share visible
    if (kt + STAGES - 2 < kt1) wait_vmcnt<LOADS * (STAGES - 2)>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + STAGES - 1 < kt1) {
      int ns = stage + STAGES - 1;
      if (ns >= STAGES) ns -= STAGES;
      issue(kt + STAGES - 1, ns);
    }
    const bf16* A = As + stage * BM * BK;
    const bf16* B = Bs + stage * BN * BK;
    // fragments of both 32-deep halves are read up front (double-buffered registers) so
    // the second half's LDS latency hides behind the first half's MFMAs
    bf16x8 af[2][TM], bfr[2][TN];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * TM * 16 + i * 16 + (lane & 15);
        af[kk][i] = *reinterpret_cast<const bf16x8*>(A + swz(row, chunk));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * TN * 16 + j * 16 + (lane & 15);
        bfr[kk][j] = *reinterpret_cast<const bf16x8*>(B + swz(row, chunk));
      }
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if constexpr (RELU) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[kk][i] = __builtin_bit_cast(bf16x8, relu8(__builtin_bit_cast(u32x4, af[kk][i])));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bfr[kk][j], acc[i][j], 0, 0, 0);
    }
    stage = stage + 1 == STAGES ? 0 : stage + 1;
  }
  __syncthreads();  // every wave done with the ring before the epilogue reuses the LDS
  conv_epilogue<BM, BN, WM, WN, MODE, NT>(a, g, acc, m0, n0, smem, fd_hwq, fd_wq);
}

template <int BM, int BN, int WM, int WN, int MODE, int STAGES, bool FASTK, bool RELU>
static int launch_glds(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int pipe = STAGES * (BM + BN) * BK * 2;
  constexpr int epi = BM * (BN + 8) * 2 + 2 * (WM * WN * 64) * 4;  // + stats scratch
  constexpr int smem = pipe > epi ? pipe : epi;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(
        reinterpret_cast<const void*>(&conv_fwd_glds_kernel<BM, BN, WM, WN, MODE, STAGES, FASTK, RELU>),
        hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set = true;
  }
  const int classes = MODE == 0 ? 1 : a.stride * a.stride;
  long mmax = 0;
  for (int c = 0; c < classes; ++c) {
    long hq = a.OH, wq = a.OW;
    if (MODE == 1) {
      const int ry = c / a.stride, rx = c % a.stride;
      hq = a.OH > ry ? (a.OH - ry + a.stride - 1) / a.stride : 0;
      wq = a.OW > rx ? (a.OW - rx + a.stride - 1) / a.stride : 0;
    }
    const long mc = (long)a.N * hq * wq;
    mmax = mc > mmax ? mc : mmax;
  }
  const long mtiles = (mmax + BM - 1) / BM;
  const long ntiles = (a.Cout + BN - 1) / BN;
  dim3 grid((unsigned)(mtiles * ntiles), 1, (unsigned)(classes * a.splits));
  hipLaunchKernelGGL((conv_fwd_glds_kernel<BM, BN, WM, WN, MODE, STAGES, FASTK, RELU>), grid, dim3(WM * WN * 64), smem,
                     st, a);
  return (int)hipGetLastError();
}

template <int MODE, bool FASTK, bool RELU>
static int dispatch_glds2(const ConvFwdArgs& a, int variant, hipStream_t st) {
  // variant: 2 = 2-stage 128-row tile, 3 = 3-stage 128-row tile, 4 = 3-stage 256x128 8 waves,
  // 5 = 2-stage 256x256 (8 waves of 128x64: half the LDS fragment traffic per MFMA of 4),
  // 6 = 2-stage 256x64 on 4 waves of 64x64 (N <= 64 layers)
  if (a.Cout > 128 && variant == 5) return launch_glds<256, 256, 2, 4, MODE, 2, FASTK, RELU>(a, st);
  if (a.Cout > 64) {
    if (variant == 5) return launch_glds<256, 128, 4, 2, MODE, 3, FASTK, RELU>(a, st);
    if (variant == 2) return launch_glds<128, 128, 2, 2, MODE, 2, FASTK, RELU>(a, st);
    if (variant == 3) return launch_glds<128, 128, 2, 2, MODE, 3, FASTK, RELU>(a, st);
    if (variant == 4) return launch_glds<256, 128, 4, 2, MODE, 3, FASTK, RELU>(a, st);
  } else if (a.Cout > 32) {
    if (variant == 6) return launch_glds<256, 64, 4, 1, MODE, 2, FASTK, RELU>(a, st);
    if (variant == 2) return launch_glds<128, 64, 2, 2, MODE, 2, FASTK, RELU>(a, st);
    if (variant == 3) return launch_glds<128, 64, 2, 2, MODE, 3, FASTK, RELU>(a, st);
    if (variant == 4) return launch_glds<256, 64, 4, 2, MODE, 3, FASTK, RELU>(a, st);
  }
  return -2;
}

template <int MODE>
static int dispatch_glds(const ConvFwdArgs& a, int variant, hipStream_t st) {
  const bool fastk = a.C1 % BK == 0 && a.C2 % BK == 0;
  if (a.act_in == ACT_RELU)
    return fastk ? dispatch_glds2<MODE, true, true>(a, variant, st) : dispatch_glds2<MODE, false, true>(a, variant, st);
  return fastk ? dispatch_glds2<MODE, true, false>(a, variant, st) : dispatch_glds2<MODE, false, false>(a, variant, st);
}

}  // namespace p2p

extern "C" int p2p_conv_fwd_glds(const p2p::ConvFwdArgs* a, int mode, int variant, hipStream_t st) {
  if (!a->zero) return -2;
  if (a->C1 > 1024 || a->C2 > 1024) return -2;  // zero-page walk bound (see a_ptr)
  if (a->act_in != p2p::ACT_NONE && a->act_in != p2p::ACT_RELU) return -2;
  return mode == 0 ? p2p::dispatch_glds<0>(*a, variant, st) : p2p::dispatch_glds<1>(*a, variant, st);
}
