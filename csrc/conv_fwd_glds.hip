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

__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(lds_wave_base), 16, 0, 0);
}

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i32x8 cat8(u32x4 lo, u32x4 hi) {
  return __builtin_shufflevector(__builtin_bit_cast(i32x4, lo), __builtin_bit_cast(i32x4, hi), 0, 1, 2, 3, 4, 5,
                                 6, 7);
}


// ReLU on 16 packed fp8 (e4m3 / e5m2: sign = bit 7 of each byte): zero the negative bytes
__device__ __forceinline__ uint32_t relu_fp8x4(uint32_t w) {
  const uint32_t neg = (w >> 7) & 0x01010101u;
  return w & ~(neg * 0xffu);
}
__device__ __forceinline__ u32x4 relu_fp8x16(u32x4 v) {
  u32x4 o;
  o.x = relu_fp8x4(v.x);
  o.y = relu_fp8x4(v.y);
  o.z = relu_fp8x4(v.z);
  o.w = relu_fp8x4(v.w);
  return o;
}

// FASTK: every channel group a multiple of 64 (one tap per 64-deep K tile, wave-uniform);
// otherwise (packed 8 / 16 / 24-channel image inputs) each lane splits its own chunk's k
// into (tap, channel) and k >= Kc reads zeros.
// F8 = 0: bf16 operands, v_mfma_f32_16x16x32_bf16 (two per 64-deep K tile).
// F8 = 1 / 2: fp8 operands -- A e4m3 / e5m2 (activations / gradients), B e4m3 (weights) --
// one v_mfma_scale_f32_16x16x128_f8f6f4 per 128-deep K tile.  The LDS image is byte-for-byte
// the bf16 one ([rows][128 B], 16-B chunks, same swizzle), so per K tile the staging, LDS
// traffic and MFMA cycles are unchanged while the tile carries twice the MACs.  Dequant:
// per-source power-of-two scales as the MFMA's E8M0 scale operands (csrc/fp8.hip).
// PK8 (non-FASTK, MODE 0, bf16): the packed 8-channel image inputs (C1 == 8, no second
// source, KW | 8) -- one 16-B chunk is exactly one tap, so a row's chunk keeps its tap offset
// (ty0 + kt * 8 / KW, tx) from tile to tile and the loader needs no per-tile divisions.
template <int BM, int BN, int WM, int WN, int MODE, int STAGES, bool FASTK, bool RELU, int F8, bool PK8 = false,
          bool EXT = false>
__global__ void __launch_bounds__(WM * WN * 64) conv_fwd_glds_kernel(ConvFwdArgs a) {
  static_assert(!PK8 || (!FASTK && MODE == 0 && F8 == 0), "PK8: packed bf16 image convs");
  using T = typename std::conditional<F8 != 0, uint8_t, bf16>::type;
  constexpr int EPC = 16 / (int)sizeof(T);  // elements per 16-B chunk
  constexpr int BKE = 8 * EPC;              // K elements per tile (128 B per row)
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  constexpr int RPP = NT / 8;            // tile rows covered per glds pass (8 lanes per row)
  constexpr int AROWS = BM / RPP;
  constexpr int BROWS = BN / RPP;
  constexpr int LOADS = AROWS + BROWS;   // glds instructions per thread per tile
  static_assert(BM % RPP == 0 && BN % RPP == 0, "every wave issues the same glds count");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* As = reinterpret_cast<T*>(smem);
  T* Bs = As + STAGES * BM * BKE;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;

  // MODE 1: the stride^2 parity classes of one (m, n) tile are adjacent block ids (class
  // fastest), so after the XCD remap they run together on one XCD and share the input rows
  // in its L2 -- class-major order re-read the whole input from HBM once per class
  const int classes = MODE == 1 ? a.stride * a.stride : 1;
  const int split = blockIdx.z;
  const int ntiles = (a.Cout + BN - 1) / BN;
  const int bid0 = xcd_remap(blockIdx.x, gridDim.x);
  const int cls = MODE == 1 ? bid0 % classes : 0;
  const int bid = MODE == 1 ? bid0 / classes : bid0;
  const ClassGeom g = class_geom<MODE>(a, cls);
  const int mt = bid / ntiles, nt = bid % ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  if (m0 >= g.Mc) return;

  const int ktiles = (g.Kc + BKE - 1) / BKE;
  const int kps = (ktiles + a.splits - 1) / a.splits;
  const int kt0 = split * kps;
  const int kt1 = min(ktiles, kt0 + kps);
  if (kt0 >= kt1 && a.splits > 1) return;

  const T* __restrict__ x1 = static_cast<const T*>(a.x1);
  const T* __restrict__ x2 = static_cast<const T*>(a.x2);
  const T* __restrict__ w = static_cast<const T*>(a.w);
  const T* zero = static_cast<const T*>(a.zero);
  const int C = a.C, C1 = a.C1, C2 = a.C2;
  // fp8: E8M0 dequant exponents of the two A sources and of the weights (fp8 scale sites)
  const int ex1 = (F8 && a.qs_x1) ? a.qs_x1[2] : 127;
  const int ex2 = (F8 && a.qs_x2) ? a.qs_x2[2] : 127;
  const int ew = (F8 && a.qs_w) ? a.qs_w[2] : 127;
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
    r_c[i] = (slot ^ ((row >> 1) & 7)) * EPC;   // source-side swizzle
  }
  int b_off[BROWS];
  bool b_ok[BROWS];
  const long wrow = (MODE == 0) ? (long)g.Kc : (long)a.KH * a.KW * C;
#pragma unroll
  for (int i = 0; i < BROWS; ++i) {
    const int row = wid * 8 + rsub + RPP * i;
    const int co = n0 + row;
    b_ok[i] = co < a.Cout;
    b_off[i] = (slot ^ ((row >> 1) & 7)) * EPC;
  }
  const FastDiv fd_c = make_fastdiv((uint32_t)C), fd_ti = make_fastdiv((uint32_t)g.Ti);
  // FASTK A-row pointers of the current channel segment (one tap x one source tensor):
  // formed once per segment, then advanced by BK per k-tile (out-of-image rows walk the
  // zero page, which covers a whole segment: host guarantees C1, C2 <= 1024).
  const T* a_ptr[AROWS];
  const T* b_base[BROWS];
#pragma unroll
  for (int i = 0; i < BROWS; ++i) {
    const int co = n0 + wid * 8 + rsub + RPP * i;
    b_base[i] = w + (long)(b_ok[i] ? co : 0) * wrow + b_off[i];
  }

  int pk_ty[PK8 ? AROWS : 1], pk_tx[PK8 ? AROWS : 1];
  const int pk_dty = PK8 ? 8 / g.Ti : 0;   // tap rows advanced per 8-tap K tile
  if constexpr (PK8) {
#pragma unroll
    for (int i = 0; i < AROWS; ++i) {
      const int c = r_c[i] / EPC;            // this row's chunk == tap within the tile
      pk_ty[i] = c / g.Ti;
      pk_tx[i] = c - pk_ty[i] * g.Ti;
    }
  }
  auto issue = [&](int kt, int stage) {
    const int k0 = kt * BKE;
    T* Ast = As + stage * BM * BKE;
    T* Bst = Bs + stage * BN * BKE;
    if constexpr (FASTK) {
      const int tap = (int)fdiv((uint32_t)k0, fd_c);
      const int ci0 = k0 - tap * C;
      const int t_y = (int)fdiv((uint32_t)tap, fd_ti);
      const int t_x = tap - t_y * g.Ti;
      if (kt == kt0 || ci0 == 0 || ci0 == C1) {
        const bool s1 = ci0 < C1;
        const T* src = s1 ? x1 : x2;
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
        for (int i = 0; i < AROWS; ++i) a_ptr[i] += BKE;
      }
#pragma unroll
      for (int i = 0; i < AROWS; ++i) glds16(a_ptr[i], Ast + (wid * 8 + RPP * i) * BKE);
      long woff;
      if (MODE == 0) {
        woff = k0;
      } else {
        const int ky = g.ky0 + a.stride * t_y, kx = g.kx0 + a.stride * t_x;
        woff = (long)(ky * a.KW + kx) * C + ci0;
      }
#pragma unroll
      for (int i = 0; i < BROWS; ++i) {
        const T* gp = b_ok[i] ? b_base[i] + woff : zero;
        glds16(gp, Bst + (wid * 8 + RPP * i) * BKE);
      }
    } else if constexpr (PK8) {
      const int ntaps = g.Kc >> 3;
#pragma unroll
      for (int i = 0; i < AROWS; ++i) {
        const int tap = kt * 8 + r_c[i] / EPC;
        const int t_y = pk_ty[i] + kt * pk_dty, t_x = pk_tx[i];
        int uy = r_y[i] + t_y, ux = r_x[i] + t_x;
        if (a.reflect && r_y[i] > -(1 << 27)) {
          uy = reflect_idx(uy, Hu);
          ux = reflect_idx(ux, Wu);
        }
        const bool inb = (unsigned)uy < (unsigned)Hu && (unsigned)ux < (unsigned)Wu && tap < ntaps;
        const long off = (long)(r_img[i] + (uy >> ush) * a.W + (ux >> ush)) * 8;
        glds16(inb ? x1 + off : zero, Ast + (wid * 8 + RPP * i) * BKE);
      }
#pragma unroll
      for (int i = 0; i < BROWS; ++i) {
        const int k = k0 + b_off[i];
        const T* gp = (b_ok[i] && k < g.Kc) ? b_base[i] - b_off[i] + k : zero;
        glds16(gp, Bst + (wid * 8 + RPP * i) * BKE);
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
        const T* src = s1 ? x1 : x2;
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
        const T* gp = inb ? src + off : zero;
        glds16(gp, Ast + (wid * 8 + RPP * i) * BKE);
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
        const T* gp = (b_ok[i] && k < g.Kc) ? w + co * wrow + woff : zero;
        glds16(gp, Bst + (wid * 8 + RPP * i) * BKE);
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr bool LATE = STAGES == 2 && F8 == 0;
  if constexpr (LATE) {
    // 2-slot ring with prefetch distance 2: each K tile's fragments are read into registers
    // up front (they already were), a second barrier then frees its slot, and tile kt + 2 is
    // issued into it BEFORE the MFMAs -- two K tiles of MFMA time cover each load instead of
    // one, with the same LDS (the 256x256 tile's vmcnt(0) per tile was exposed HBM latency)
    issue(kt0, 0);
    if (kt0 + 1 < kt1) issue(kt0 + 1, 1);
    int stage = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      if (kt + 1 < kt1) wait_vmcnt<LOADS>();   // tile kt landed; kt + 1 may still fly
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      const bf16* A = As + stage * BM * BK;
      const bf16* B = Bs + stage * BN * BK;
      // first 32-deep half: read and multiply; second half: read, then free the slot (every
      // wave's reads retired + barrier) and issue tile kt + 2 before its MFMAs -- only one
      // half's fragments are live across the issue (register budget of the 256x256 tile)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int chunk = kk * 4 + (lane >> 4);
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wn * TN * 16 + j * 16 + (lane & 15);
          bfr[j] = *reinterpret_cast<const bf16x8*>(B + swz(row, chunk));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * TM * 16 + i * 16 + (lane & 15);
          af[i] = *reinterpret_cast<const bf16x8*>(A + swz(row, chunk));
        }
        if (kk == 1) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();         // every wave holds its fragments: slot free
          __builtin_amdgcn_sched_barrier(0);
          if (kt + 2 < kt1) issue(kt + 2, stage);
        }
        if constexpr (RELU) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
            af[i] = __builtin_bit_cast(bf16x8, relu8(__builtin_bit_cast(u32x4, af[i])));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
      stage ^= 1;
    }
  } else {
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
      if constexpr (F8 != 0) {
        const T* A = As + stage * BM * BKE;
        const T* B = Bs + stage * BN * BKE;
        // this lane's 32-deep k block comes from one source tensor (host: C1 % 32 == 0):
        // its E8M0 dequant exponent is the MFMA's scale_a
        int sa = ex1;
        if (C2 > 0) {
          const int k = FASTK ? kt * BKE : kt * BKE + 32 * (lane >> 4);
          const int tap = (int)fdiv((uint32_t)k, fd_c);
          sa = (k - tap * C) < C1 ? ex1 : ex2;
        }
        // operand layout of the 16x16x128 f8 MFMA: lane group q = lane>>4 holds K [16q, 16q+16)
        // in its low 16 bytes and K [64+16q, 64+16q+16) in its high 16 bytes (LDS chunks q and
        // q+4), and its scale operand covers K block [32q, 32q+32) -- probes/mfma_fp8_scale.hip
        const int c0 = lane >> 4;
        i32x8 af[TM], bfr[TN];
  #pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * TM * 16 + i * 16 + (lane & 15);
          u32x4 lo = *reinterpret_cast<const u32x4*>(A + 2 * swz(row, c0));
          u32x4 hi = *reinterpret_cast<const u32x4*>(A + 2 * swz(row, c0 + 4));
          if constexpr (RELU) {
            lo = relu_fp8x16(lo);
            hi = relu_fp8x16(hi);
          }
          af[i] = cat8(lo, hi);
        }
  #pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wn * TN * 16 + j * 16 + (lane & 15);
          bfr[j] = cat8(*reinterpret_cast<const u32x4*>(B + 2 * swz(row, c0)),
                        *reinterpret_cast<const u32x4*>(B + 2 * swz(row, c0 + 4)));
        }
  #pragma unroll
        for (int i = 0; i < TM; ++i)
  #pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i][j], F8 - 1, 0, 0, sa,
                                                                         0, ew);
      } else {
      const bf16* A = As + stage * BM * BK;
      const bf16* B = Bs + stage * BN * BK;
      // fragments of both 32-deep halves are read up front (double-buffered registers) so
      // the second half's LDS latency hides behind the first half's MFMAs; per half the B
      // fragments come first (every MFMA row needs all of them)
      bf16x8 af[2][TM], bfr[2][TN];
  #pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int chunk = kk * 4 + (lane >> 4);
  #pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wn * TN * 16 + j * 16 + (lane & 15);
          bfr[kk][j] = *reinterpret_cast<const bf16x8*>(B + swz(row, chunk));
        }
  #pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * TM * 16 + i * 16 + (lane & 15);
          af[kk][i] = *reinterpret_cast<const bf16x8*>(A + swz(row, chunk));
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
      }
      stage = stage + 1 == STAGES ? 0 : stage + 1;
    }
  }
  __syncthreads();  // every wave done with the ring before the epilogue reuses the LDS
  conv_epilogue<BM, BN, WM, WN, MODE, NT, EXT>(a, g, acc, m0, n0, smem, fd_hwq, fd_wq);
}

template <int BM, int BN, int WM, int WN, int MODE, int STAGES, bool FASTK, bool RELU, int F8, bool PK8 = false,
          bool EXT = false>
static int launch_glds(const ConvFwdArgs& a, hipStream_t st) {
  if ((BM / WM / 16) * (BN / WN / 16) > 16 && a.splits > 1) return -2;   // no split-K epilogue in big wave tiles
  constexpr int pipe = STAGES * (BM + BN) * BK * 2;
  constexpr int epi = BM * (BN + 8) * 2 + 2 * (WM * WN * 64) * 4;  // + stats scratch
  constexpr int smem = pipe > epi ? pipe : epi;
  static std::atomic<uint64_t> attr_mask{0};
  smem_attr_once(reinterpret_cast<const void*>(&conv_fwd_glds_kernel<BM, BN, WM, WN, MODE, STAGES, FASTK, RELU, F8, PK8, EXT>), smem, attr_mask);
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
  dim3 grid((unsigned)(mtiles * ntiles * classes), 1, (unsigned)a.splits);
  hipLaunchKernelGGL((conv_fwd_glds_kernel<BM, BN, WM, WN, MODE, STAGES, FASTK, RELU, F8, PK8, EXT>), grid, dim3(WM * WN * 64), smem,
                     st, a);
  return (int)hipGetLastError();
}

template <int MODE, bool FASTK, bool RELU, int F8, bool PK8 = false, bool EXT = false>
static int dispatch_glds2(const ConvFwdArgs& a, int variant, hipStream_t st) {
  if constexpr (F8 != 0) {
    // fp8: the bf16 winners only (256x256 / 256x128 for wide layers, 128x64 below)
    if (a.Cout > 128 && variant == 5) return launch_glds<256, 256, 2, 4, MODE, 2, FASTK, RELU, F8, false, EXT>(a, st);
    if (a.Cout > 64) {
      if (variant == 2) return launch_glds<128, 128, 2, 2, MODE, 2, FASTK, RELU, F8, false, EXT>(a, st);
      return launch_glds<256, 128, 4, 2, MODE, 3, FASTK, RELU, F8, false, EXT>(a, st);
    }
    if (a.Cout > 32) return launch_glds<128, 64, 2, 2, MODE, 2, FASTK, RELU, F8, false, EXT>(a, st);
    return -2;
  } else {
  // variant: 2 = 2-stage 128-row tile, 3 = 3-stage 128-row tile, 4 = 3-stage 256x128 8 waves,
  // 5 = 2-stage 256x256 (8 waves of 128x64: half the LDS fragment traffic per MFMA of 4),
  // 6 = 2-stage 256x64 on 4 waves of 64x64 (N <= 64 layers)
  if constexpr (PK8) {   // image layers: K = taps x 8 is short -> the 2-block-per-CU 128-row tiles
    if (a.Cout > 64) return launch_glds<128, 128, 2, 2, MODE, 2, FASTK, RELU, F8, true>(a, st);
    if (a.Cout > 32) return launch_glds<128, 64, 2, 2, MODE, 2, FASTK, RELU, F8, true>(a, st);
    return -2;
  }
  if (a.Cout > 128 && variant == 5) return launch_glds<256, 256, 2, 4, MODE, 2, FASTK, RELU, F8, false, EXT>(a, st);
  // 7 = 256x32 on 4 waves of 64x32: the skinny union GEMMs of the packed-image layers
  // (d1 forward / c1 dgrad: 4 parity classes x 3 image channels, padded to 32 columns)
  if (variant == 7) {
    if constexpr (MODE == 0 && FASTK) {
      if (a.Cout <= 32) return launch_glds<256, 32, 4, 1, MODE, 2, FASTK, RELU, F8, false, EXT>(a, st);
    }
    return -2;
  }
  // 8 = 256x64 on 2 waves of 128x64, 9 = 256x128 on 4 waves of 128x64: the 256x256 tile's
  // per-wave operand reuse (384 B of LDS fragments per MFMA) for N = 64 / 128 layers
  if (variant == 8 && a.Cout <= 64) return launch_glds<256, 64, 2, 1, MODE, 2, FASTK, RELU, F8, false, EXT>(a, st);
  if (variant == 9 && a.Cout > 64 && a.Cout <= 128)
    return launch_glds<256, 128, 2, 2, MODE, 2, FASTK, RELU, F8, false, EXT>(a, st);
  if (a.Cout > 64) {
    if (variant == 5) return launch_glds<256, 128, 4, 2, MODE, 3, FASTK, RELU, F8, false, EXT>(a, st);
    if (variant == 2) return launch_glds<128, 128, 2, 2, MODE, 2, FASTK, RELU, F8, false, EXT>(a, st);
    if (variant == 3) return launch_glds<128, 128, 2, 2, MODE, 3, FASTK, RELU, F8, false, EXT>(a, st);
    if (variant == 4) return launch_glds<256, 128, 4, 2, MODE, 3, FASTK, RELU, F8, false, EXT>(a, st);
  } else if (a.Cout > 32) {
    if (variant == 6) return launch_glds<256, 64, 4, 1, MODE, 2, FASTK, RELU, F8, false, EXT>(a, st);
    if (variant == 2) return launch_glds<128, 64, 2, 2, MODE, 2, FASTK, RELU, F8, false, EXT>(a, st);
    if (variant == 3) return launch_glds<128, 64, 2, 2, MODE, 3, FASTK, RELU, F8, false, EXT>(a, st);
    if (variant == 4) return launch_glds<256, 64, 4, 2, MODE, 3, FASTK, RELU, F8, false, EXT>(a, st);
  }
  return -2;
  }
}

template <int MODE, int F8>
static int dispatch_glds(const ConvFwdArgs& a, int variant, hipStream_t st) {
  constexpr int BKE = F8 ? 2 * BK : BK;
  const bool fastk = a.C1 % BKE == 0 && a.C2 % BKE == 0;
  if (a.act_in == ACT_RELU) {
    if constexpr (F8 == 2) return -2;  // gradients (e5m2) never carry an input activation
    else
      return fastk ? dispatch_glds2<MODE, true, true, F8>(a, variant, st)
                   : dispatch_glds2<MODE, false, true, F8>(a, variant, st);
  }
  if constexpr (MODE == 0 && F8 == 0) {
    if (!fastk && a.C1 == 8 && a.C2 == 0 && a.KW <= 8 && 8 % a.KW == 0 && variant != 1)
      return dispatch_glds2<MODE, false, false, F8, true>(a, variant, st);
  }
  if constexpr (F8 != 1) {
    // dgrads (bf16 or e5m2 gradient operands) with an act' gate / parked skip gradient / fused
    // norm partials: the EXT epilogue
    if (a.nb_ws || (a.act_bwd || a.res1))
      return fastk ? dispatch_glds2<MODE, true, false, F8, false, true>(a, variant, st)
                   : dispatch_glds2<MODE, false, false, F8, false, true>(a, variant, st);
  }
  if (a.nb_ws) return -2;   // (fp8 / input-ReLU convs never carry fused norm partials)
  return fastk ? dispatch_glds2<MODE, true, false, F8>(a, variant, st)
               : dispatch_glds2<MODE, false, false, F8>(a, variant, st);
}

template <int F8>
static int dispatch_mode(const ConvFwdArgs& a, int mode, int variant, hipStream_t st) {
  return mode == 0 ? dispatch_glds<0, F8>(a, variant, st) : dispatch_glds<1, F8>(a, variant, st);
}

}  // namespace p2p

extern "C" int p2p_conv_fwd_glds(const p2p::ConvFwdArgs* a, int mode, int variant, hipStream_t st) {
  if (!a->zero) return -2;
  if (a->C1 > 1024 || a->C2 > 1024) return -2;  // zero-page walk bound (see a_ptr)
  if (a->act_in != p2p::ACT_NONE && a->act_in != p2p::ACT_RELU) return -2;
  if (a->fp8 == 0) return p2p::dispatch_mode<0>(*a, mode, variant, st);
  // fp8: every 32-deep k block of a lane inside one source tensor and one tap
  if (a->C1 % 32 || a->C2 % 32 || a->splits > 1 && a->ws == nullptr) return -2;
  if (a->fp8 == 1) return p2p::dispatch_mode<1>(*a, mode, variant, st);
  if (a->fp8 == 2) return p2p::dispatch_mode<2>(*a, mode, variant, st);
  return -2;
}
