// Implicit-GEMM conv / transposed conv on gfx950 v_mfma_f32_32x32x16_bf16, 256-row tiles.
//
// Same GEMM view, LDS image (source-side swizzled global_load_lds "LDS-DMA" staging, zero
// page for out-of-image taps) and fused epilogue as conv_fwd_glds.hip; what is new is the
// MFMA shape and the software pipeline around it (the 16x16x32 tiles
// sat at 37-48 % MFMA busy with every LDS fragment burst and every glds issue exposed).
//
//  * v_mfma_f32_32x32x16_bf16: half the MFMA instructions of 16x16x32 for the same FLOP,
//    32 issue cycles each -- an MFMA holds vector issue for 8 of its 32 cycles instead of
//    8 of 16, so the loader's VALU / glds issue and the fragment reads fit beside the
//    matrix pipe (MI355X_MICROARCH.md: per-instruction issue costs).
//  * k16-step pipeline with a 3-deep fragment register ring: the LDS reads of step t + 2
//    are in flight while step t's MFMAs run, and only the reads a step consumes are
//    waited for (counted lgkmcnt on inline-asm ds_read_b128, invisible to the compiler's
//    conservative LDS-DMA aliasing waits).
//  * ONE barrier per 64-deep K tile (the 16x16 kernel had two): before it every wave has
//    (a) retired all reads of the slot it is done with and (b) landed its share of the
//    next tile; after it the next tile's first fragments are read and the slot just freed
//    is refilled (tile kt + STAGES) with the glds interleaved between the MFMAs of the
//    tile's last two k16 steps.
//  * the loop is unrolled over lcm(3, STAGES) = 6 tiles, so the fragment-ring index and
//    the LDS slot of every step are compile-time constants (immediate offsets).
//
// Wave tiles: BN = 256 -> 8 waves of 128 x 64 (TM 4 x TN 2 MFMA blocks of 32 x 32),
// BN = 128 -> 8 waves of 64 x 64 (2 x 2) with a 3-slot ring (48 KB per slot).
// Covered: bf16 operands, FASTK geometry (both concat halves multiples of 64 channels),
// MODE 0 (conv) / MODE 1 (transposed conv as stride^2 parity classes), input ReLU, the
// plain and the EXT (act' gate / skip gradient / norm-backward partials) epilogues, no
// split-K.  Everything else returns -2 and stays on conv_fwd_glds.hip.
//   reference layers: the PatchGAN ladder (networks.py:764-784) and the U-Net encoder /
//   decoder of the north-star config (BASELINE.json) -- every 4x4 conv with >= 64 channels.
#include <atomic>
#include <cstdlib>

#include "conv_dev.h"

namespace p2p {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int N>
__device__ __forceinline__ void m32_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ uint32_t lds_byte_addr(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const void*)p));
}

template <int OFF>
__device__ __forceinline__ u32x4 ds_rd128(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  u32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

typedef int m32_i32x8 __attribute__((ext_vector_type(8)));
typedef int m32_i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ m32_i32x8 m32_cat8(u32x4 lo, u32x4 hi) {
  return __builtin_shufflevector(__builtin_bit_cast(m32_i32x4, lo), __builtin_bit_cast(m32_i32x4, hi), 0, 1, 2, 3, 4,
                                 5, 6, 7);
}
// ReLU on 16 packed fp8 bytes (e4m3: sign = bit 7 of each byte): zero the negative ones
__device__ __forceinline__ u32x4 m32_relu_fp8x16(u32x4 v) {
#pragma unroll
  for (int w = 0; w < 4; ++w) v[w] &= ~(((v[w] >> 7) & 0x01010101u) * 0xffu);
  return v;
}

// one k16 step's operands: TM A fragments (32 pixel rows x 16 k) and TN B fragments
template <int TM, int TN>
struct Frag {
  u32x4 a[TM];
  u32x4 b[TN];
};

// s_waitcnt lgkmcnt(N) that every use of the fragment registers must follow
template <int N, int TM, int TN>
__device__ __forceinline__ void frag_wait(Frag<TM, TN>& f) {
  static_assert(N >= 0 && N <= 15, "lgkmcnt range");
  if constexpr (TM == 4 && TN == 2) {
    asm volatile("s_waitcnt lgkmcnt(%6)"
                 : "+v"(f.a[0]), "+v"(f.a[1]), "+v"(f.a[2]), "+v"(f.a[3]), "+v"(f.b[0]), "+v"(f.b[1])
                 : "n"(N));
  } else {
    static_assert(TM == 2 && TN == 2, "wave tile");
    asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(f.a[0]), "+v"(f.a[1]), "+v"(f.b[0]), "+v"(f.b[1]) : "n"(N));
  }
}

// 16-B buffer_load ... lds (M0 = the wave's LDS destination).  Kept in a __device__ helper:
// called straight from the kernel's (host + device) lambdas, hipcc's host pass silently
// dropped the kernels' launch stubs (undefined symbols at dlopen).
__device__ __forceinline__ void bld16(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(lds), 16, voff, soff, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                           (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL), 0x00020000);
}

// bias + output activation in registers -> the bf16 tile in LDS (row stride LDC).  The MFMAs
// run with the operands swapped (weights = src A, pixels = src B), so the 32x32 accumulator
// holds D[pixel][channel] transposed: acc[i][j][4 g + e] = D[i*32 + (lane & 31)]
// [j*32 + 8 g + 4 (lane >> 5) + e] -- a lane owns 4 consecutive channels of one pixel per
// register quad and stages them with ONE ds_write_b64 (a quarter of the 2-B stores).
template <int TM, int TN, int LDC>
__device__ __forceinline__ void stage_tile32(const ConvFwdArgs& a, f32x16 (&acc)[TM][TN], bf16* Cs, int row0,
                                             int col0, int n0, int lane) {
  static_assert(LDC % 4 == 0, "8-B aligned staging rows");
  const float al = a.alpha ? a.alpha[0] : 1.f;
  const int h = lane >> 5, pr = lane & 31;
  auto stage = [&](auto act_tag) __attribute__((always_inline)) {
    constexpr int ACT = decltype(act_tag)::value;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int coll = col0 + j * 32 + 8 * q + 4 * h;
        const int col = n0 + coll;
        float bj[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) bj[e] = (a.bias && col + e < a.Cout) ? a.bias[col + e] : 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          bf16x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = (bf16)act_fwd(acc[i][j][4 * q + e] * al + bj[e], ACT);
          *reinterpret_cast<bf16x4*>(Cs + (row0 + i * 32 + pr) * LDC + coll) = v;
        }
      }
    }
  };
  switch (a.act_out) {
    case ACT_RELU: stage(std::integral_constant<int, ACT_RELU>{}); break;
    case ACT_LRELU: stage(std::integral_constant<int, ACT_LRELU>{}); break;
    case ACT_TANH: stage(std::integral_constant<int, ACT_TANH>{}); break;
    case ACT_SIGMOID: stage(std::integral_constant<int, ACT_SIGMOID>{}); break;
    default: stage(std::integral_constant<int, ACT_NONE>{}); break;
  }
}

}  // namespace

#ifdef P2P_M32_STAMPS
// diagnostic build only (tools/build_ext.py --define P2P_M32_STAMPS --out ...): per block,
// s_memtime at kernel start / after the prologue / after the K loop / at the end, and
// s_memrealtime at start and end -- written by lane 0 of wave 0 with vector stores into a
// buffer no output is computed from (tools/m32_stamps.py reads it back)
__device__ unsigned long long m32_stamps[65536 * 6];
#define M32_STAMP(i, v)                                                        \
  do {                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < 65536) m32_stamps[blockIdx.x * 6 + (i)] = (v); \
  } while (0)
#else
#define M32_STAMP(i, v) \
  do {                  \
  } while (0)
#endif

// BMT = 512 (round 6, BN = 128 only): 8 waves of 128 x 64 like the 256 x 256 tile -- the
// 256 x 128 tile's 64 x 64 wave tiles read 128 KB of fragments per 64-deep K tile for 1024
// MFMA cycles per SIMD (LDS-read bound at 128 B / clk / CU); 128 x 64 wave tiles read 192 KB
// for 2048.  Two 80 KB stages fill the 160 KB LDS.
template <int BN, int BMT = 256>
struct M32Geom {
  static constexpr int BM = BMT;
  static constexpr int WM = BN == 256 ? 2 : (BN == 64 ? 8 : 4);
  static constexpr int WN = 8 / WM;
  static constexpr int TM = BM / WM / 32;
  static constexpr int TN = BN / WN / 32;
  static constexpr int STAGES = (BN == 256 || BM == 512) ? 2 : 3;
  static constexpr int NT = 512;
  static constexpr int RPP = NT / 8;                // tile rows per glds pass (8 lanes per row)
  static constexpr int AROWS = BM / RPP;            // A glds per thread per tile
  static constexpr int BROWS = BN / RPP;
  static constexpr int LOADS = AROWS + BROWS;
  static constexpr int A_SLOT = BM * BK * 2;        // bytes per A slot
  static constexpr int B_SLOT = BN * BK * 2;
  static constexpr int PIPE = STAGES * (A_SLOT + B_SLOT);
  static constexpr int EPI = BM * (BN + 8) * 2 + 2 * NT * 4;
  static constexpr int SMEM = PIPE > EPI ? PIPE : EPI;
  static constexpr int NR = TM + TN;                // ds_read_b128 per k16 step
  static_assert(SMEM <= 160 * 1024, "LDS");
  static_assert(2 * NR <= 15, "two steps of reads within the lgkm counter");
};

// F8 (round 6): fp8 operands -- 1: e4m3 activations (forward / ConvT
// forward), 2: e5m2 gradients (input gradients, EXT epilogue) -- x e4m3 weights, on
// v_mfma_scale_f32_32x32x64_f8f6f4 with the per-tensor E8M0 exponents as its scale operands.
// The LDS image is byte-for-byte the bf16 one (a 128-B row = 128 fp8 k instead of 64 bf16 k),
// so staging, swizzle and fragment reads are unchanged: one fp8 k64 step is the union of the
// reads of two bf16 k16 steps (lane half h: chunks 4s + h and 4s + 2 + h), fed as the low /
// high 16 bytes of the 32-byte operand.  A and B take the same lane map, so the products pair
// whatever k order the instruction assigns inside the 32 bytes, and one per-tensor scale per
// operand makes the per-32-k scale blocks uniform.  Half the K tiles of the bf16 GEMM for the
// same MFMA cycles per tile: twice the FLOP per staged byte.
template <int BN, int MODE, bool RELU, bool EXT, int F8 = 0, int BMT = 256>
__global__ void __launch_bounds__(512) conv_fwd_m32_kernel(ConvFwdArgs a) {
  using G = M32Geom<BN, BMT>;
  static_assert(BMT == 256 || (BMT == 512 && (BN == 128 || BN == 64) && F8 == 0), "512-row tile: bf16, 64 / 128 columns");
  constexpr int ES = F8 ? 1 : 2;            // bytes per operand element
  constexpr int BKE = F8 ? 2 * BK : BK;     // operand elements per 128-B K tile row
  constexpr int BM = G::BM, WN = G::WN, TM = G::TM, TN = G::TN, STAGES = G::STAGES, NT = G::NT;
  constexpr int RPP = G::RPP, AROWS = G::AROWS, BROWS = G::BROWS, LOADS = G::LOADS;
  constexpr int NR = G::NR;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* As = reinterpret_cast<bf16*>(smem);                      // [STAGES][BM][64]
  bf16* Bs = reinterpret_cast<bf16*>(smem + STAGES * G::A_SLOT);  // [STAGES][BN][64]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: SALU glds bases
  const int wm = wid / WN, wn = wid % WN;

  const int classes = MODE == 1 ? a.stride * a.stride : 1;
  const int ntiles = (a.Cout + BN - 1) / BN;
  const int bid0 = xcd_remap(blockIdx.x, gridDim.x);
  const int cls = MODE == 1 ? bid0 % classes : 0;
  const int bid = MODE == 1 ? bid0 / classes : bid0;
  const ClassGeom g = class_geom<MODE>(a, cls);
  const int mt = bid / ntiles, nt = bid % ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  if (m0 >= g.Mc) return;
  const int kt1 = (g.Kc + BKE - 1) / BKE;   // no split-K: K tiles [0, kt1)
  // fp8: E8M0 dequant exponents of the two A sources and of the weights (fp8 scale sites)
  const int ex1 = (F8 && a.qs_x1) ? a.qs_x1[2] : 127;
  const int ex2 = (F8 && a.qs_x2) ? a.qs_x2[2] : 127;
  const int ew = (F8 && a.qs_w) ? a.qs_w[2] : 127;
  M32_STAMP(0, __builtin_amdgcn_s_memtime());
  M32_STAMP(4, __builtin_amdgcn_s_memrealtime());

  const int C = a.C, C1 = a.C1, C2 = a.C2;
  const int slot8 = lane & 7;
  const int rsub = lane >> 3;
  const int ush = a.up == 2 ? 1 : 0;
  const int Hu = a.H << ush, Wu = a.W << ush;
  const int HWq = g.Hq * g.Wq;
  const FastDiv fd_hwq = make_fastdiv((uint32_t)HWq), fd_wq = make_fastdiv((uint32_t)g.Wq);

  // ---- buffer-resource LDS-DMA (buffer_load_dwordx4 ... lds): 32-bit per-lane byte offsets
  // from a block-uniform base, and out-of-range offsets read ZERO -- the out-of-image taps,
  // padded GEMM rows and output channels beyond Cout need no zero page and no 64-bit
  // pointer per row.  The A base is the block's first image (a 256-row tile spans a few
  // images, so offsets stay far below 2^31 whatever the batch).
  constexpr uint32_t OOB = 0x80000000u;
  const int img0 = (int)fdiv((uint32_t)m0, fd_hwq);
  const long img_elems = (long)a.H * a.W;
  auto img_rsrc = [&](const void* base, int cs) __attribute__((always_inline)) {
    const long first = (long)img0 * img_elems * cs;
    return make_rsrc(static_cast<const char*>(base) + first * ES, ((long)a.N * img_elems * cs - first) * ES);
  };
  const auto rx1 = img_rsrc(a.x1, C1);
  const auto rx2 = img_rsrc(C2 > 0 ? a.x2 : a.x1, C2 > 0 ? C2 : C1);
  const long wrow = (MODE == 0) ? (long)g.Kc : (long)a.KH * a.KW * C;
  const auto rw = make_rsrc(a.w, a.Cout * wrow * ES);

  // ---- loader decode: A rows row_i = wid*8 + rsub + RPP*i (pixel of the block's first image
  // + y / x origin of its taps); the source-side swizzle (row >> 1) & 7 does not depend on i
  // per A row: the image offset and the tap origin (y, x) packed as two int16 (one register
  // instead of two); y = -16384 marks a padded row
  // 512-row tiles (host predicate p2p_conv_m32_rows: every parity class a multiple of 512
  // pixels, so a tile lies in one image and has no padded rows): no per-row image offset.
  // DERIVE: not even the per-row packed tap origins -- ONE register, the first row's in-image
  // index, and rows i (that + RPP i) re-derived per channel segment: more VALU per segment, 7
  // registers fewer.  The input-ReLU instances need it (their fragment masking spilled the
  // per-row layout inside the K loop); -DP2P_M32_DERIVE_ROWS (build-time A/B) takes it for all.
  constexpr bool ONE_IMG = BM == 512;
#ifdef P2P_M32_DERIVE_ROWS
  constexpr bool DERIVE = ONE_IMG;
#else
  constexpr bool DERIVE = ONE_IMG && RELU;
#endif
  int r_img[ONE_IMG ? 1 : AROWS], r_yx[DERIVE ? 1 : AROWS];
  r_img[0] = 0;
  if constexpr (DERIVE) {
    r_yx[0] = m0 + wid * 8 + rsub - img0 * HWq;
  } else {
#pragma unroll
    for (int i = 0; i < AROWS; ++i) {
      const int row = wid * 8 + rsub + RPP * i;
      const int m = m0 + row;
      const int mm = m < g.Mc ? m : 0;
      const int n = (int)fdiv((uint32_t)mm, fd_hwq);
      const int r = mm - n * HWq;
      const int qy = (int)fdiv((uint32_t)r, fd_wq);
      const int qx = r - qy * g.Wq;
      if constexpr (!ONE_IMG) r_img[i] = (n - img0) * a.H * a.W;
      int y0, x0;
      if (MODE == 0) {
        y0 = qy * a.stride - a.pad;
        x0 = qx * a.stride - a.pad;
      } else {
        y0 = qy + g.dy;
        x0 = qx + g.dx;
      }
      if (m >= g.Mc) y0 = -16384;
      r_yx[i] = (int)(((uint32_t)y0 << 16) | ((uint32_t)x0 & 0xffffu));
    }
  }
  // tap origin (y0, x0) and image offset of A row i
  auto row_origin = [&](int i, int& y0, int& x0, int& rimg) __attribute__((always_inline)) {
    if constexpr (DERIVE) {
      // opaque per call: keeps the compiler from hoisting the 8 rows' loop-invariant origins
      // out of the K loop (their registers are what this layout saves)
      int r0 = r_yx[0];
      asm volatile("" : "+v"(r0));
      const int r = r0 + RPP * i;
      const int qy = (int)fdiv((uint32_t)r, fd_wq);
      const int qx = r - qy * g.Wq;
      y0 = MODE == 0 ? qy * a.stride - a.pad : qy + g.dy;
      x0 = MODE == 0 ? qx * a.stride - a.pad : qx + g.dx;
    } else {
      y0 = r_yx[i] >> 16;
      x0 = (int)(int16_t)(r_yx[i] & 0xffff);
    }
    rimg = ONE_IMG ? 0 : r_img[i];
  };
  const int r_c = (slot8 ^ (((wid * 8 + rsub) >> 1) & 7)) * 8;
  uint32_t b_vo[BROWS];
#pragma unroll
  for (int i = 0; i < BROWS; ++i) {
    const int co = n0 + wid * 8 + rsub + RPP * i;
    b_vo[i] = co < a.Cout ? (uint32_t)(co * wrow * ES + r_c * 2) : OOB;
  }
  const FastDiv fd_c = make_fastdiv((uint32_t)C), fd_ti = make_fastdiv((uint32_t)g.Ti);
  uint32_t a_vo[AROWS];
  int a_soff = 0, w_soff = 0;
  bool a_first = true;

  // offsets of K tile kt (FASTK: one tap x one source tensor per 64-deep tile; the row
  // offsets are formed once per channel segment, later tiles of the segment only move the
  // uniform soffset by 128 B)
  auto prep = [&](int kt) __attribute__((always_inline)) {
    const int k0 = kt * BKE;
    const int tap = (int)fdiv((uint32_t)k0, fd_c);
    const int ci0 = k0 - tap * C;
    const int t_y = (int)fdiv((uint32_t)tap, fd_ti);
    const int t_x = tap - t_y * g.Ti;
    if (kt == 0 || ci0 == 0 || ci0 == C1) {
      const bool s1 = ci0 < C1;
      a_first = s1;
      const int cs = s1 ? C1 : C2;
      const int cio = s1 ? ci0 : ci0 - C1;
#pragma unroll
      for (int i = 0; i < AROWS; ++i) {
        int iy, ix, ry0, rx0, rimg;
        bool inb;
        row_origin(i, ry0, rx0, rimg);
        if (MODE == 0) {
          int uy = ry0 + t_y, ux = rx0 + t_x;
          if (a.reflect && ry0 > -8192) {
            uy = reflect_idx(uy, Hu);
            ux = reflect_idx(ux, Wu);
          }
          inb = (unsigned)uy < (unsigned)Hu && (unsigned)ux < (unsigned)Wu;
          iy = uy >> ush;
          ix = ux >> ush;
        } else {
          iy = ry0 - t_y;
          ix = rx0 - t_x;
          inb = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
        }
        a_vo[i] = inb ? (uint32_t)(((rimg + iy * a.W + ix) * cs + cio) * ES + r_c * 2) : OOB;
      }
      a_soff = 0;
    } else {
      a_soff += BK * 2;
    }
    if (MODE == 0) {
      w_soff = k0 * ES;
    } else {
      const int ky = g.ky0 + a.stride * t_y, kx = g.kx0 + a.stride * t_x;
      w_soff = ((ky * a.KW + kx) * C + ci0) * ES;
    }
  };
  // load number q (A rows first, then B rows) of the prepared tile into LDS slot SLOT
  auto fire = [&](auto slot_c, int q) __attribute__((always_inline)) {
    constexpr int SLOT = decltype(slot_c)::value;
    if (q < AROWS) {
      bld16(a_first ? rx1 : rx2, As + SLOT * (G::A_SLOT / 2) + (wid * 8 + RPP * q) * BK, a_vo[q], a_soff);
    } else {
      const int i = q - AROWS;
      bld16(rw, Bs + SLOT * (G::B_SLOT / 2) + (wid * 8 + RPP * i) * BK, b_vo[i], w_soff);
    }
  };
  // fp8: the E8M0 exponent of the A source of the tile in each LDS slot (a 128-deep tile never
  // straddles the concat halves: host-checked C1 % 128 == 0)
  int sa_slot[STAGES];
#pragma unroll
  for (int s = 0; s < STAGES; ++s) sa_slot[s] = ex1;
  auto issue_all = [&](auto slot_c, int kt) __attribute__((always_inline)) {
    prep(kt);
    if constexpr (F8 != 0) sa_slot[decltype(slot_c)::value] = a_first ? ex1 : ex2;
#pragma unroll
    for (int q = 0; q < LOADS; ++q) fire(slot_c, q);
  };

  // ---- per-lane LDS byte addresses of the k16 steps' fragments in slot 0
  //   lane l: row (l & 31) of a 32-row block, 16-B chunk 2s + (l >> 5) of the 64-deep tile
  uint32_t fa[4], fb[4];
  {
    const int ra = wm * TM * 32 + (lane & 31), rb = wn * TN * 32 + (lane & 31);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int chunk = 2 * s + (lane >> 5);
      fa[s] = lds_byte_addr(As + swz(ra, chunk));
      fb[s] = lds_byte_addr(Bs + swz(rb, chunk));
    }
  }
  using F = Frag<TM, TN>;
  auto read_step = [&](auto slot_c, auto s_c, F& f) __attribute__((always_inline)) {
    constexpr int SLOT = decltype(slot_c)::value, S = decltype(s_c)::value;
    const uint32_t ab = fa[S] + SLOT * G::A_SLOT, bb = fb[S] + SLOT * G::B_SLOT;
    // row block i is 32 rows = 4 KB further with the same XOR key ((row + 32) >> 1 & 7)
    f.a[0] = ds_rd128<0>(ab);
    f.a[1] = ds_rd128<4096>(ab);
    if constexpr (TM > 2) {
      f.a[2] = ds_rd128<8192>(ab);
      f.a[3] = ds_rd128<12288>(ab);
    }
    f.b[0] = ds_rd128<0>(bb);
    f.b[1] = ds_rd128<4096>(bb);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // one k16 step of MFMAs with glds Q0 .. Q0 + NQ - 1 of the refill tile spread over its
  // P = TM * TN MFMAs (after MFMA p: floor((p + 1) NQ / P) - floor(p NQ / P) of them, so every
  // glds index is a compile-time constant once the loops are unrolled)
  auto mma_step = [&](F& f, auto nq_c, auto q0_c, auto slot_c, bool refill) __attribute__((always_inline)) {
    constexpr int NQ = decltype(nq_c)::value, Q0 = decltype(q0_c)::value, P = TM * TN;
    static_assert(NQ <= 2 * P, "at most two glds per MFMA");
    if constexpr (RELU) {
#pragma unroll
      for (int i = 0; i < TM; ++i) f.a[i] = relu8(f.a[i]);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        // weights as src A, pixels as src B: the accumulator comes out pixel-major (stage_tile32)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, f.b[j]),
                                                             __builtin_bit_cast(bf16x8, f.a[i]), acc[i][j], 0, 0, 0);
        const int p = i * TN + j;
        if (NQ > 0 && refill) {
#pragma unroll
          for (int q = (p * NQ) / P; q < ((p + 1) * NQ) / P; ++q) {
            __builtin_amdgcn_sched_barrier(0);
            fire(slot_c, Q0 + q);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    }
  };
  // fp8: one k64 step = the fragments of two bf16 k16 steps (lo: chunks 4s + h, hi: 4s + 2 + h)
  // held as fixed lo / hi pairs (one 8-register MFMA operand each), with glds Q0 .. Q0 + NQ - 1
  // spread over its P MFMAs (up to two after an MFMA)
  struct F8Frag {
    u32x4 alo[TM], ahi[TM], blo[TN], bhi[TN];
  };
  auto read_f8 = [&](auto slot_c, auto s_c, F8Frag& f) __attribute__((always_inline)) {
    constexpr int SLOT = decltype(slot_c)::value, S = decltype(s_c)::value;
    const uint32_t a0 = fa[2 * S] + SLOT * G::A_SLOT, a1 = fa[2 * S + 1] + SLOT * G::A_SLOT;
    const uint32_t b0 = fb[2 * S] + SLOT * G::B_SLOT, b1 = fb[2 * S + 1] + SLOT * G::B_SLOT;
    f.alo[0] = ds_rd128<0>(a0);
    f.ahi[0] = ds_rd128<0>(a1);
    f.alo[1] = ds_rd128<4096>(a0);
    f.ahi[1] = ds_rd128<4096>(a1);
    if constexpr (TM > 2) {
      f.alo[2] = ds_rd128<8192>(a0);
      f.ahi[2] = ds_rd128<8192>(a1);
      f.alo[3] = ds_rd128<12288>(a0);
      f.ahi[3] = ds_rd128<12288>(a1);
    }
    f.blo[0] = ds_rd128<0>(b0);
    f.bhi[0] = ds_rd128<0>(b1);
    f.blo[1] = ds_rd128<4096>(b0);
    f.bhi[1] = ds_rd128<4096>(b1);
  };
  auto wait_f8 = [&](auto n_c, F8Frag& f) __attribute__((always_inline)) {
    constexpr int N = decltype(n_c)::value;
    static_assert(N >= 0 && N <= 15, "lgkmcnt range");
    if constexpr (TM == 4) {
      asm volatile("s_waitcnt lgkmcnt(%12)"
                   : "+v"(f.alo[0]), "+v"(f.alo[1]), "+v"(f.alo[2]), "+v"(f.alo[3]), "+v"(f.ahi[0]), "+v"(f.ahi[1]),
                     "+v"(f.ahi[2]), "+v"(f.ahi[3]), "+v"(f.blo[0]), "+v"(f.blo[1]), "+v"(f.bhi[0]), "+v"(f.bhi[1])
                   : "n"(N));
    } else {
      asm volatile("s_waitcnt lgkmcnt(%8)"
                   : "+v"(f.alo[0]), "+v"(f.alo[1]), "+v"(f.ahi[0]), "+v"(f.ahi[1]), "+v"(f.blo[0]), "+v"(f.blo[1]),
                     "+v"(f.bhi[0]), "+v"(f.bhi[1])
                   : "n"(N));
    }
  };
  // k64 step of MFMAs on f, streaming the NEXT step's fragments into f behind them (RD: A
  // fragment i is re-read once its MFMAs are issued, the B fragments after the last one): one
  // register set of 8-register operands (a second set spilled the 256-wide tile)
  auto mma_f8 = [&](F8Frag& f, auto nq_c, auto q0_c, auto slot_c, bool refill, int sa, auto rslot_c, auto rstep_c,
                    bool rd) __attribute__((always_inline)) {
    constexpr int NQ = decltype(nq_c)::value, Q0 = decltype(q0_c)::value, P = TM * TN;
    constexpr int RSLOT = decltype(rslot_c)::value, RS = decltype(rstep_c)::value;
    static_assert(NQ <= 2 * P, "at most two glds per MFMA");
    if constexpr (RELU) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        f.alo[i] = m32_relu_fp8x16(f.alo[i]);
        f.ahi[i] = m32_relu_fp8x16(f.ahi[i]);
      }
    }
    const uint32_t a0 = fa[2 * RS] + RSLOT * G::A_SLOT, a1 = fa[2 * RS + 1] + RSLOT * G::A_SLOT;
    const uint32_t b0 = fb[2 * RS] + RSLOT * G::B_SLOT, b1 = fb[2 * RS + 1] + RSLOT * G::B_SLOT;
    m32_i32x8 bv[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) bv[j] = m32_cat8(f.blo[j], f.bhi[j]);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const m32_i32x8 av = m32_cat8(f.alo[i], f.ahi[i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        // weights (e4m3) as src A, pixels (e4m3 / e5m2) as src B: pixel-major accumulator
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bv[j], av, acc[i][j], 0, F8 - 1, 0, ew, 0, sa);
        const int p = i * TN + j;
        if (NQ > 0 && refill) {
#pragma unroll
          for (int q = (p * NQ) / P; q < ((p + 1) * NQ) / P; ++q) {
            __builtin_amdgcn_sched_barrier(0);
            fire(slot_c, Q0 + q);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
      if (rd) {
        __builtin_amdgcn_sched_barrier(0);
        // ds offsets: row block i is 32 rows = 4 KB further (same XOR key)
        if (i == 0) { f.alo[0] = ds_rd128<0>(a0); f.ahi[0] = ds_rd128<0>(a1); }
        if (i == 1) { f.alo[1] = ds_rd128<4096>(a0); f.ahi[1] = ds_rd128<4096>(a1); }
        if (i == 2) { f.alo[2] = ds_rd128<8192>(a0); f.ahi[2] = ds_rd128<8192>(a1); }
        if (i == 3) { f.alo[3] = ds_rd128<12288>(a0); f.ahi[3] = ds_rd128<12288>(a1); }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (rd) {
      f.blo[0] = ds_rd128<0>(b0);
      f.bhi[0] = ds_rd128<0>(b1);
      f.blo[1] = ds_rd128<4096>(b0);
      f.bhi[1] = ds_rd128<4096>(b1);
    }
  };

  F fr[3];
  // ---- prologue: tiles 0 .. STAGES-1 in flight, tile 0 landed, its steps 0 / 1 being read
#pragma unroll
  for (int s = 0; s < STAGES; ++s) {
    if (s < kt1) {
      if (s == 0) issue_all(std::integral_constant<int, 0>{}, 0);
      if (s == 1) issue_all(std::integral_constant<int, 1>{}, 1);
      if (s == 2) issue_all(std::integral_constant<int, 2 % STAGES>{}, 2);
    }
  }
  {
    const int inflight = (kt1 < STAGES ? kt1 : STAGES) - 1;   // tiles issued after tile 0
    if (inflight >= 2) m32_vmcnt<2 * LOADS>();
    else if (inflight == 1) m32_vmcnt<LOADS>();
    else m32_vmcnt<0>();
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  F8Frag p8;
  if constexpr (F8 != 0) {
    read_f8(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, p8);
  } else {
    read_step(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, fr[0]);
    read_step(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{}, fr[1]);
  }
  M32_STAMP(1, __builtin_amdgcn_s_memtime());

  // ---- one 64-deep K tile; T = kt mod 6 (ring index R = T % 3, LDS slot T % STAGES)
  constexpr int QA = LOADS / 2, QB = LOADS - LOADS / 2;   // glds in steps 2 / 3
  auto tile = [&](auto t_c, int kt) __attribute__((always_inline)) {
    constexpr int T = decltype(t_c)::value;
    constexpr int R = T % 3;
    constexpr int SLOT = T % STAGES, NSLOT = (T + 1) % STAGES;
    using SC = std::integral_constant<int, SLOT>;
    using NC = std::integral_constant<int, NSLOT>;
    const bool more = kt + 1 < kt1;
    const bool refill = kt + STAGES < kt1;
    // step 0: read step 2 of this tile, run step 0
    read_step(SC{}, std::integral_constant<int, 2>{}, fr[(R + 2) % 3]);
    frag_wait<2 * NR>(fr[R]);
    __builtin_amdgcn_sched_barrier(0);
    mma_step(fr[R], std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, SC{}, false);
    __builtin_amdgcn_sched_barrier(0);
    // step 1: read step 3, run step 1
    read_step(SC{}, std::integral_constant<int, 3>{}, fr[R]);
    frag_wait<2 * NR>(fr[(R + 1) % 3]);
    __builtin_amdgcn_sched_barrier(0);
    mma_step(fr[(R + 1) % 3], std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, SC{}, false);
    __builtin_amdgcn_sched_barrier(0);
    // sync: all my reads of this slot retired, my share of tile kt + 1 landed
    frag_wait<0>(fr[(R + 2) % 3]);
    frag_wait<0>(fr[R]);
    if constexpr (STAGES == 3) {
      if (kt + 2 < kt1) m32_vmcnt<LOADS>();
      else m32_vmcnt<0>();
    } else {
      m32_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (refill) prep(kt + STAGES);   // loader address math (VALU) before the MFMAs it hides behind
    // step 2: read step 0 of tile kt + 1, run step 2 with the first glds of tile kt + STAGES
    if (more) read_step(NC{}, std::integral_constant<int, 0>{}, fr[(R + 1) % 3]);
    __builtin_amdgcn_sched_barrier(0);
    mma_step(fr[(R + 2) % 3], std::integral_constant<int, QA>{}, std::integral_constant<int, 0>{}, SC{}, refill);
    __builtin_amdgcn_sched_barrier(0);
    // step 3: read step 1 of tile kt + 1, run step 3 with the remaining glds
    if (more) read_step(NC{}, std::integral_constant<int, 1>{}, fr[(R + 2) % 3]);
    __builtin_amdgcn_sched_barrier(0);
    mma_step(fr[R], std::integral_constant<int, QB>{}, std::integral_constant<int, QA>{}, SC{}, refill);
    __builtin_amdgcn_sched_barrier(0);
  };
  // ---- fp8: one 128-deep K tile = two k64 steps on ONE operand register set p8 (entry: p8
  // holds step 0's reads, in flight); each step's MFMAs stream the next step's reads into p8.
  // Same barrier / refill structure as the bf16 tile: the slot's last reads are retired before
  // the barrier, the refill glds run behind the second step's MFMAs.
  auto tile_f8 = [&](auto t_c, int kt) __attribute__((always_inline)) {
    constexpr int T = decltype(t_c)::value;
    constexpr int SLOT = T % STAGES, NSLOT = (T + 1) % STAGES;
    using SC = std::integral_constant<int, SLOT>;
    using NC = std::integral_constant<int, NSLOT>;
    const bool refill = kt + STAGES < kt1;
    const int sa = sa_slot[SLOT];
    wait_f8(std::integral_constant<int, 0>{}, p8);
    __builtin_amdgcn_sched_barrier(0);
    mma_f8(p8, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, SC{}, false, sa, SC{},
           std::integral_constant<int, 1>{}, true);
    __builtin_amdgcn_sched_barrier(0);
    // sync: all my reads of this slot retired, my share of tile kt + 1 landed
    wait_f8(std::integral_constant<int, 0>{}, p8);
    if constexpr (STAGES == 3) {
      if (kt + 2 < kt1) m32_vmcnt<LOADS>();
      else m32_vmcnt<0>();
    } else {
      m32_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (refill) {
      prep(kt + STAGES);
      sa_slot[SLOT] = a_first ? ex1 : ex2;
    }
    // (the last tile reads the next slot anyway: unconditional reads keep one dataflow for p8; the
    // values are never used)
    mma_f8(p8, std::integral_constant<int, LOADS>{}, std::integral_constant<int, 0>{}, SC{}, refill, sa, NC{},
           std::integral_constant<int, 0>{}, true);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto run = [&](auto body) __attribute__((always_inline)) {
    for (int kt = 0;;) {
      body(std::integral_constant<int, 0>{}, kt);
      if (++kt >= kt1) break;
      body(std::integral_constant<int, 1>{}, kt);
      if (++kt >= kt1) break;
      body(std::integral_constant<int, 2>{}, kt);
      if (++kt >= kt1) break;
      body(std::integral_constant<int, 3>{}, kt);
      if (++kt >= kt1) break;
      body(std::integral_constant<int, 4>{}, kt);
      if (++kt >= kt1) break;
      body(std::integral_constant<int, 5>{}, kt);
      if (++kt >= kt1) break;
    }
  };
  if constexpr (F8 != 0) run(tile_f8);
  else run(tile);
  __syncthreads();  // every wave done with the ring before the epilogue reuses the LDS
  M32_STAMP(2, __builtin_amdgcn_s_memtime());

  bf16* Cs = reinterpret_cast<bf16*>(smem);
  constexpr int LDC = BN + 8;
  stage_tile32<TM, TN, LDC>(a, acc, Cs, wm * TM * 32, wn * TN * 32, n0, lane);
  __syncthreads();
  conv_epilogue_tail<BM, BN, MODE, NT, EXT>(a, g, m0, n0, Cs, reinterpret_cast<float*>(smem + BM * LDC * 2), smem,
                                            fd_hwq, fd_wq);
#ifdef P2P_M32_STAMPS
  __syncthreads();
  M32_STAMP(3, __builtin_amdgcn_s_memtime());
  M32_STAMP(5, __builtin_amdgcn_s_memrealtime());
#endif
}

template <int BN, int MODE, bool RELU, bool EXT, int F8 = 0, int BMT = 256>
static int launch_m32(const ConvFwdArgs& a, hipStream_t st) {
  using G = M32Geom<BN, BMT>;
  static std::atomic<uint64_t> attr_mask{0};
  smem_attr_once(reinterpret_cast<const void*>(&conv_fwd_m32_kernel<BN, MODE, RELU, EXT, F8, BMT>), G::SMEM,
                 attr_mask);
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
  const long mtiles = (mmax + G::BM - 1) / G::BM;
  const long ntiles = (a.Cout + BN - 1) / BN;
  dim3 grid((unsigned)(mtiles * ntiles * classes), 1, 1);
  hipLaunchKernelGGL((conv_fwd_m32_kernel<BN, MODE, RELU, EXT, F8, BMT>), grid, dim3(G::NT), G::SMEM, st, a);
  return (int)hipGetLastError();
}

// fp8 runs the 256 x 128 tile only (Cout 65..128): its 128-deep K tiles give it 175 FLOP per
// staged byte (the bf16 256 x 256 tile: 128), and a 256-wide fp8 m32 tile spills (the
// 8-register operands of 32x32x64 need ~24 registers per step more than two bf16 k16 steps)
template <int MODE>
static int dispatch_m32_f8(const ConvFwdArgs& a, hipStream_t st) {
  if (a.fp8 == 1) {   // e4m3 activations: plain epilogue, optional input ReLU
    if (a.nb_ws || a.act_bwd || a.res1) return -2;
    return a.act_in == ACT_RELU ? launch_m32<128, MODE, true, false, 1>(a, st)
                                : launch_m32<128, MODE, false, false, 1>(a, st);
  }
  if (a.fp8 == 2) {   // e5m2 gradients: no input activation; the EXT epilogue for gated dgrads
    if (a.act_in != ACT_NONE) return -2;
    if (a.nb_ws || (a.act_bwd || a.res1)) return launch_m32<128, MODE, false, true, 2>(a, st);
    return launch_m32<128, MODE, false, false, 2>(a, st);
  }
  return -2;
}

template <int BN, int MODE, int BMT = 256>
static int dispatch_m32_epi(const ConvFwdArgs& a, hipStream_t st) {
  if (a.act_in == ACT_RELU) return launch_m32<BN, MODE, true, false, 0, BMT>(a, st);
  if (a.nb_ws || (a.act_bwd || a.res1)) return launch_m32<BN, MODE, false, true, 0, BMT>(a, st);
  return launch_m32<BN, MODE, false, false, 0, BMT>(a, st);
}

}  // namespace p2p

// 1 (default) = the 32x32x16 tiles take the 256x256 / 256x128 bf16 FASTK convs; 0 = the
// round-4 16x16x32 tiles of conv_fwd_glds.hip.  Initialised once from P2P_M32, switchable at
// run time (torch.ops.p2p.set_m32) so one process can A/B both paths.
static std::atomic<int>& m32_flag() {
  static std::atomic<int> on{[] {
    const char* v = std::getenv("P2P_M32");
    return v ? (v[0] != '0' ? 1 : 0) : 1;
  }()};
  return on;
}
extern "C" int p2p_m32_enabled() { return m32_flag().load(std::memory_order_relaxed); }
extern "C" int p2p_set_m32(int on) { return m32_flag().exchange(on ? 1 : 0); }

#ifdef P2P_M32_STAMPS
extern "C" int p2p_m32_stamps(void* host_out, int nblocks) {
  if (nblocks > 65536) nblocks = 65536;
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(p2p::m32_stamps), (size_t)nblocks * 6 * 8, 0,
                                  hipMemcpyDeviceToHost);
}
#endif

// Rows of the m32 tile that p2p_conv_fwd_m32 would run for these arguments: 0 = not covered
// (-2 there), else 256 or 512.  The host sizes the fused-statistics / norm-partial chunks by
// it (conv_epilogue_tail: one chunk per BM rows), so this is THE routing predicate.
// 512 rows (bf16, variant 4: the 128-column tiles): every parity class a multiple of 512
// pixels and >= 256 blocks in the grid (one per CU; family R's B = 64 residual 3x3s have 512
// and gained 1 % on it), unless P2P_M32_BM (read per call: the tests and A/Bs pin it) says
// 256 or 512.
extern "C" int p2p_conv_m32_rows(const p2p::ConvFwdArgs* a, int mode, int variant) {
  using namespace p2p;
  if (a->splits > 1 || a->d2s) return 0;
  // FASTK: every 128-B K tile inside one tap and one source (64 bf16 / 128 fp8 channels)
  const int chc = a->fp8 ? 128 : 64;
  if (a->C1 % chc || a->C2 % chc || a->C1 > 1024 || a->C2 > 1024) return 0;
  if (a->fp8 && (!a->qs_x1 || !a->qs_w || (a->C2 && !a->qs_x2) || a->fp8 > 2)) return 0;
  if (a->act_in != ACT_NONE && a->act_in != ACT_RELU) return 0;
  if (a->fp8) {
    // Cout 65..128 only: there the 256 x 128 fp8 tile beats the 16x16x128 glds tile by 3-10 %
    // per layer; for Cout > 128 the glds 256 x 256 fp8 tile (A staged once for 256 columns)
    // is 10-20 % faster than two 128-wide m32 column tiles (profiles/kernel_experiments_r6.md)
    if ((variant != 4 && variant != 5) || a->Cout <= 64 || a->Cout > 128) return 0;
    if (a->fp8 == 1 && (a->nb_ws || a->act_bwd || a->res1)) return 0;
    if (a->fp8 == 2 && a->act_in != ACT_NONE) return 0;
    return 256;
  }
  if (variant == 5 && a->Cout > 128) return 256;
  // 33-64 output channels (variant 2, the glds 128 x 64 tile otherwise): only the 512 x 64
  // tile (8 waves of 64 x 64), under the same geometry conditions as the 512 x 128 one
  const bool c64 = variant == 2 && a->Cout > 32 && a->Cout <= 64 && a->KH * a->KW >= 4;
  if (!(variant == 4 && a->Cout > 64) && !c64) return 0;
  const int fallback = c64 ? 0 : 256;
  const char* env = std::getenv("P2P_M32_BM");
  const int pin = env ? std::atoi(env) : 0;
  if (pin == 256) return fallback;
  if (c64 && std::getenv("P2P_M32_C64") && std::getenv("P2P_M32_C64")[0] == '0') return 0;
  const int classes = mode == 0 ? 1 : a->stride * a->stride;
  long hwq = (long)a->OH * a->OW;
  if (mode == 1) {
    if (a->OH % a->stride || a->OW % a->stride) return fallback;
    hwq = (long)(a->OH / a->stride) * (a->OW / a->stride);
  }
  if (hwq % 512) return fallback;
  const long blocks = (long)a->N * hwq / 512 * ((a->Cout + 127) / 128) * classes;
  return (pin == 512 || blocks >= 256) ? 512 : fallback;
}

// variant 5 -> 256 x 256 tile (Cout > 128), 4 -> 256 x 128 or 512 x 128 (Cout > 64); -2 = not
// covered
extern "C" int p2p_conv_fwd_m32(const p2p::ConvFwdArgs* a, int mode, int variant, hipStream_t st) {
  using namespace p2p;
  const int rows = p2p_conv_m32_rows(a, mode, variant);
  if (rows == 0) return -2;
  if (a->fp8) return mode == 0 ? dispatch_m32_f8<0>(*a, st) : dispatch_m32_f8<1>(*a, st);
  // (the ReLU 256-wide variants spill a few loop-invariant epilogue values before the K loop; the loop itself is spill-free)
  if (variant == 5)
    return mode == 0 ? dispatch_m32_epi<256, 0>(*a, st) : dispatch_m32_epi<256, 1>(*a, st);
  if (rows == 512 && a->Cout <= 64)
    return mode == 0 ? dispatch_m32_epi<64, 0, 512>(*a, st) : dispatch_m32_epi<64, 1, 512>(*a, st);
  if (rows == 512)
    return mode == 0 ? dispatch_m32_epi<128, 0, 512>(*a, st) : dispatch_m32_epi<128, 1, 512>(*a, st);
  return mode == 0 ? dispatch_m32_epi<128, 0>(*a, st) : dispatch_m32_epi<128, 1>(*a, st);
}
