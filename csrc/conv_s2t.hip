// Stride-2 transposed conv (4x4, pad 1, OH = 2H) -- the U-Net decoder's ConvTranspose2d and
// the input gradient of every 4x4 stride-2 conv -- on a halo tile shared by the 4 parity
// classes (VERDICT r2 #1a).
//
// The implicit GEMM (conv_fwd_glds.hip MODE 1) runs one GEMM per output parity class: every
// class tile gathers its own im2col rows, so each input pixel is staged from L2 into LDS
// 16 times (4 classes x 4 taps) for a 64-column output -- these layers ran at 390-540 TF/s,
// bound by the L2 -> LDS staging rate (profiles/kernel_experiments_r3.md).  Here a block
// owns BM = 128 consecutive grid positions q (RH = 128 / W whole rows of the input grid,
// one image) and 64 output channels of ALL four classes: per 64-channel chunk it stages
// the (RH + 2) x (W + 2) input halo ONCE (global_load_lds, source-side swizzle, 2-stage
// ring), and wave c (= class (ry, rx)) reads the A fragments of its 2 x 2 taps out of that
// one LDS image at shifted pixel offsets.  8 waves: wave w computes class w & 3 for output
// channels 32 (w >> 2) .. + 32 (128 x 32 per wave: 64 accumulator registers, so two blocks
// fit a CU and one's epilogue overlaps the other's MFMAs).  A wave's B fragments (its
// class's 4 taps x 32 channels; the weights are L2-resident) go global -> VGPR (buffer
// loads) one k-step ahead.  Per wave and chunk: 64 ds_read_b128 + 16 buffer loads for 128
// MFMAs.
//
// Tap geometry (conv_dev.h class_geom, s = 2, p = 1): class (ry, rx) reads input row
// qy + dy - ty with kernel row ky = ky0 + 2 ty, ty in {0, 1}; ky0 = (ry + 1) % 2,
// dy = (ry + 1 - ky0) / 2 (columns alike).  Halo pixel (hy, hx) = input (qy0 - 1 + hy, hx - 1).
//
// Epilogue: each wave stages its 128 x 32 block into its class's LDS tile; then
// the whole block runs the shared GEMM epilogue tail (conv_dev.h) class by class -- bias,
// activation, statistics for a following norm, act' gate / skip gradient / norm-backward
// partials of a dgrad, fp8 shadow -- with exactly the per-class BM = 128 tile conventions
// of the implicit GEMM (stats / partial chunk index), so the host's buffers are the same.
//
// F8 = 1 / 2 (fp8 precision: x e4m3 / gradients e5m2, weights e4m3): the same kernel on a
// 128-channel chunk -- byte for byte the bf16 64-channel halo (128 B per pixel, same units,
// same swizzle) -- with one v_mfma_scale_f32_16x16x128_f8f6f4 per tap where bf16 issues two
// 16x16x32 MFMAs: its lane group q takes K [16q, 16q + 16) from LDS chunk q and
// [64 + 16q, ...) from chunk q + 4 -- the same two reads the two bf16 k-steps make -- and the
// per-source E8M0 exponents are its scale operands (csrc/fp8.hip sites).
#include "conv_dev.h"

namespace p2p {

namespace {

__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(lds_wave_base), 16, 0, 0);
}

// s_waitcnt vmcnt(N) through the builtin (not inline asm): the compiler's wait-count pass
// sees it, so registers loaded before the wait are known complete after it (with an asm
// wait it re-waits vmcnt(0) at the first use -- the chunk's fresh halo loads included)
typedef int s2t_i32x8 __attribute__((ext_vector_type(8)));
typedef int s2t_i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ s2t_i32x8 s2t_cat8(u32x4 lo, u32x4 hi) {
  return __builtin_shufflevector(__builtin_bit_cast(s2t_i32x4, lo), __builtin_bit_cast(s2t_i32x4, hi), 0, 1, 2, 3,
                                 4, 5, 6, 7);
}

// ReLU on 16 packed fp8 bytes (sign = bit 7): zero the negative ones
__device__ __forceinline__ u32x4 s2t_relu_fp8x16(u32x4 v) {
#pragma unroll
  for (int w = 0; w < 4; ++w) v[w] &= ~(((v[w] >> 7) & 0x01010101u) * 0xffu);
  return v;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | 0x70 | 0xF00 | (((N >> 4) & 3) << 14));
}

#ifndef S2T_F8PF
#define S2T_F8PF 0   // fp8: B one tap ahead (1 spills the accumulators at 128 VGPRs)
#endif
#ifndef S2T_PD
#define S2T_PD 1   // B prefetch distance in k-steps (2, 3: the register-ring experiment)
#endif
constexpr int BM = 128, BN = 64, NT = 512;
constexpr int TM = BM / 16, TN = 2;         // one wave = one class x 32 channels: 8 x 2 fragments
constexpr int LDC = BN + 8;

template <int W>
struct S2TGeom {
  static constexpr int RH = BM / W;                 // grid rows per tile
  // halo edge: W + 2 columns stored at a row pitch HW that is a multiple of 8 pixels, so
  // the swizzle key hp & 6 is the same for every fragment of a k-step (only their -1 column
  // shift changes it): a whole k-step's A reads are one base register + immediate offsets
  static constexpr int HWV = W + 2, HW = (W + 2 + 7) / 8 * 8, HH = RH + 2;
  static constexpr int HPIX = HH * HW;
  static constexpr int UNITS = HPIX * 8;            // 16-B units per 128-B chunk (64 bf16 / 128 fp8)
  static constexpr int HLD = (UNITS + NT - 1) / NT; // glds per lane per stage
  static constexpr int STAGE_BYTES = HLD * NT * 16;
  static constexpr int EPI_BYTES = 4 * BM * LDC * 2 + 2 * NT * 4;
  static constexpr int SMEM = 2 * STAGE_BYTES > EPI_BYTES ? 2 * STAGE_BYTES : EPI_BYTES;
  static_assert(SMEM <= 80 * 1024, "two blocks per CU");
};

}  // namespace

template <int W, bool RELU, bool EXT, int F8 = 0>
__global__ void __launch_bounds__(512, 4) conv_s2t_kernel(ConvFwdArgs a) {
  using G = S2TGeom<W>;
  constexpr int ES = F8 ? 1 : 2;      // bytes per operand element
  constexpr int CHC = 128 / ES;       // channels per 128-B halo chunk
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntiles_n = a.Cout / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / ntiles_n, nt = bid - mt * ntiles_n;
  const int m0 = mt * BM, n0 = nt * BN;
  const int HWq = a.H * a.W;
  const int img = m0 / HWq;
  const int qy0 = (m0 - img * HWq) / W;
  const int C = a.C1 + a.C2;
  const int nch = C / CHC;
  // fp8: E8M0 dequant exponents of the two sources and of the weight image
  const int ex1 = (F8 && a.qs_x1) ? a.qs_x1[2] : 127;
  const int ex2 = (F8 && a.qs_x2) ? a.qs_x2[2] : 127;
  const int ew = (F8 && a.qs_w) ? a.qs_w[2] : 127;

  char* ring = smem;
  // halo chunk ch -> ring stage: unit e = j * NT + tid holds logical 16-B chunk
  // (e & 7) ^ (hp & 6) of halo pixel hp = e >> 3 (source-side swizzle).  Unlike the im2col
  // tiles' (row >> 1) & 7 key, hp & 6 keeps every ds_read_b128 lane group conflict-free for
  // ANY fragment base pixel (the tap shifts move it by -1 / -HW): 16 consecutive pixels,
  // 8 of each parity, with the group's two k chunks in the pattern 0,0,1,1,1,1,0,0 map to 16
  // distinct bank quads (exhaustive check over bases and k steps; the old key: up to 4-way)
  // pixels outside the image (or beyond the halo) read the zero page.  Recomputed per issue
  // (a few VALU per unit, 2-4 issues per block) instead of holding 2 x HLD registers.
  auto issue = [&](int ch, int stage) {
    const bool s1 = ch * CHC < a.C1;
    const char* src = static_cast<const char*>(s1 ? a.x1 : a.x2);
    const int cs = s1 ? a.C1 : a.C2;
    const int coff = s1 ? ch * CHC : ch * CHC - a.C1;
    char* dst = ring + stage * G::STAGE_BYTES;
    // the per-lane unit geometry is loop-invariant: laundering tid keeps the compiler from
    // hoisting it out of the chunk loop into (spilled) registers
    int t = tid;
    asm volatile("" : "+v"(t));
#pragma unroll
    for (int j = 0; j < G::HLD; ++j) {
      const int e = j * NT + t;
      const int hp = e >> 3;
      const int hy = hp / G::HW, hx = hp - (hp / G::HW) * G::HW;
      const int iy = qy0 - 1 + hy, ix = hx - 1;
      const bool in = hp < G::HPIX && hx < G::HWV && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
      const int kc = (e & 7) ^ (hp & 6);
      const int pix = in ? (img * a.H + iy) * a.W + ix : 0;
      const char* g = src + ((long)pix * cs + coff) * ES + kc * 16;
      glds16(in ? g : static_cast<const char*>(a.zero), dst + (j * NT + wid * 64) * 16);
    }
  };

  // ---- this wave's class and its tap geometry (wave-uniform: scalar registers)
  const int cls_w = __builtin_amdgcn_readfirstlane(wid & 3);
  const int nh = __builtin_amdgcn_readfirstlane(wid >> 2);   // 32-channel half of the co tile
  const int ry = cls_w >> 1, rx = cls_w & 1;
  const int ky0 = (ry + 1) & 1, kx0 = (rx + 1) & 1;
  const int dy = (ry + 1 - ky0) >> 1, dx = (rx + 1 - kx0) >> 1;
  // B fragments by buffer loads: per-lane row offset (output channel n0 + (lane & 15), k block
  // 8 * (lane >> 4)) in voffset, the (tap, k-step, 16-column block) offset in soffset
  const int wrow = 16 * C * ES;   // bytes per output channel of the [Cout][4][4][C] image
  const auto wsrd = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0, a.Cout * wrow, 0x00020000);
  const int bvoff = (n0 + 32 * nh + (lane & 15)) * wrow + 16 * (lane >> 4);
  // A fragment rows: lane row r = lane & 15 of fragment i -> grid position p = 16 i + r
  //   (ly = p / W, qx = p % W); tap (ty, tx) reads halo pixel (ly + dy - ty + 1, qx + dx - tx + 1)
  //   = abase + (i / (W / 16)) * HW + 16 * (i % (W / 16)): one register, the rest immediate
  int abase = (dy + 1) * G::HW + (lane & 15) + dx + 1;
  const int kq = lane >> 4;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // B operand of k-step (ch, t, ks): t = ty * 2 + tx, ks = 64-B half of the chunk (bf16: the
  // 32-deep half; fp8: the high 16 bytes of each lane's 32-deep operand)
  auto loadB = [&](int ch, int t, int ks, u32x4 (&b)[TN]) __attribute__((always_inline)) {
    const int ky = ky0 + 2 * (t >> 1), kx = kx0 + 2 * (t & 1);
    const int so = ((ky * 4 + kx) * C + ch * CHC) * ES + ks * 64;
#pragma unroll
    for (int j = 0; j < TN; ++j)
      b[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wsrd, bvoff, so + j * 16 * wrow, 0));
  };

  if constexpr (F8 != 0) {
    // fp8: one k-step per tap (128 deep); both 64-B halves of its B operand one tap ahead
    // both halves land in one 8-register operand per fragment (no concatenation copies)
    auto loadB8 = [&](int ch, int t, s2t_i32x8 (&b)[TN]) __attribute__((always_inline)) {
      u32x4 lo[TN], hi[TN];
      loadB(ch, t, 0, lo);
      loadB(ch, t, 1, hi);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = s2t_cat8(lo[j], hi[j]);
    };
#if S2T_F8PF
    s2t_i32x8 bc[TN], bn[TN];
    loadB8(0, 0, bc);
#endif
    issue(0, 0);
    for (int ch = 0; ch < nch; ++ch) {
      const int stage = ch & 1;
      if (ch + 1 < nch) {
        issue(ch + 1, stage ^ 1);
        wait_vm<G::HLD>();
      } else {
        wait_vm<0>();
      }
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      const char* A = ring + stage * G::STAGE_BYTES;
      asm volatile("" : "+v"(abase));
      const int sa = ch * CHC < a.C1 ? ex1 : ex2;   // a chunk never straddles the sources
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#if S2T_F8PF
        if (t < 3) loadB8(ch, t + 1, bn);
        else if (ch + 1 < nch) loadB8(ch + 1, 0, bn);
#else
        s2t_i32x8 bc[TN];
        loadB8(ch, t, bc);
#endif
        const int toff = -(t >> 1) * G::HW - (t & 1);
        constexpr int FPR = W / 16;
        const int hp0 = abase + toff;
        const int offlo = (hp0 * 8 + (kq ^ (hp0 & 6))) * 16;
        const int offhi = (hp0 * 8 + ((kq + 4) ^ (hp0 & 6))) * 16;
        auto rd = [&](int i) __attribute__((always_inline)) {
          const int fo = ((i / FPR) * G::HW + 16 * (i % FPR)) * 128;
          u32x4 lo = *reinterpret_cast<const u32x4*>(A + offlo + fo);
          u32x4 hi = *reinterpret_cast<const u32x4*>(A + offhi + fo);
          if constexpr (RELU) {
            lo = s2t_relu_fp8x16(lo);
            hi = s2t_relu_fp8x16(hi);
          }
          return s2t_cat8(lo, hi);
        };
        s2t_i32x8 af[2];
        af[0] = rd(0);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          if (i + 1 < TM) af[(i + 1) & 1] = rd(i + 1);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i & 1], bc[j], acc[i][j], F8 - 1, 0, 0,
                                                                         sa, 0, ew);
        }
        __builtin_amdgcn_sched_group_barrier(0x020, 2 * TN, 0);   // the B prefetch first
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);        // A fragments 0 and 1
#pragma unroll
        for (int i = 0; i < TM - 2; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, TN, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * TN, 0);
#if S2T_F8PF
#pragma unroll
        for (int j = 0; j < TN; ++j) bc[j] = bn[j];
#endif
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  } else {
#if S2T_PD > 1
    // B ring: k-step st of a chunk uses bq[st & 3]; loads run PD k-steps ahead (8 k-steps per
    // chunk keep the ring index static across chunks) -- experiment (kernel_experiments_r3.md)
    constexpr int PD = S2T_PD;
    u32x4 bq[4][TN];
#pragma unroll
    for (int st = 0; st < PD; ++st) loadB(0, st >> 1, st & 1, bq[st]);
#else
    u32x4 bcur[TN], bnxt[TN];
    loadB(0, 0, 0, bcur);
#endif
    issue(0, 0);
    for (int ch = 0; ch < nch; ++ch) {
      const int stage = ch & 1;
      if (ch + 1 < nch) {
        issue(ch + 1, stage ^ 1);
        wait_vm<G::HLD>();
      } else {
        wait_vm<0>();
      }
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      const bf16* A = reinterpret_cast<const bf16*>(ring + stage * G::STAGE_BYTES);
      // the A addresses are loop-invariant per (tap, k-step, fragment): hoisted out of the chunk
      // loop they would pin 64 registers (and spill); laundering abase keeps them per step
      asm volatile("" : "+v"(abase));
#pragma unroll
      for (int st = 0; st < 8; ++st) {
        const int t = st >> 1, ks = st & 1;
        // prefetch the next k-step's B (the next chunk's first after the last) a whole k-step
        // of MFMAs ahead of its use; then A fragment i + 1 is read while fragment i's 4 MFMAs
        // run (sched_group_barrier pins that interleave: left alone the scheduler sinks the B
        // loads below the MFMAs and the next step waits vmcnt(0) on a full L2 round trip)
#if S2T_PD > 1
        if (st + PD < 8) loadB(ch, (st + PD) >> 1, (st + PD) & 1, bq[(st + PD) & 3]);
        else if (ch + 1 < nch) loadB(ch + 1, (st + PD - 8) >> 1, (st + PD - 8) & 1, bq[(st + PD) & 3]);
        u32x4 (&bcur)[TN] = bq[st & 3];
#else
        if (st < 7) loadB(ch, (st + 1) >> 1, (st + 1) & 1, bnxt);
        else if (ch + 1 < nch) loadB(ch + 1, 0, 0, bnxt);
#endif
        const int toff = -(t >> 1) * G::HW - (t & 1);
        const int kc = ks * 4 + kq;
        // fragment i sits (i / FPR) rows and 16 (i % FPR) pixels from fragment 0: both multiples
        // of 8 pixels, so the same swizzle key -- its address is an immediate offset
        constexpr int FPR = W / 16;
        const int hp0 = abase + toff;
        const int off0 = (hp0 * 8 + (kc ^ (hp0 & 6))) * 8;
        auto rd = [&](int i) __attribute__((always_inline)) {
          bf16x8 v = *reinterpret_cast<const bf16x8*>(A + off0 + ((i / FPR) * G::HW + 16 * (i % FPR)) * 64);
          if constexpr (RELU) v = __builtin_bit_cast(bf16x8, relu8(__builtin_bit_cast(u32x4, v)));
          return v;
        };
        bf16x8 af[2];
        af[0] = rd(0);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          if (i + 1 < TM) af[(i + 1) & 1] = rd(i + 1);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i & 1], __builtin_bit_cast(bf16x8, bcur[j]),
                                                                 acc[i][j], 0, 0, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x020, TN, 0);   // the B prefetch (VMEM reads) first
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);    // A fragments 0 and 1
#pragma unroll
        for (int i = 0; i < TM - 2; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, TN, 0); // fragment i's MFMAs
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // read fragment i + 2
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * TN, 0);
#if S2T_PD <= 1
#pragma unroll
        for (int j = 0; j < TN; ++j) bcur[j] = bnxt[j];
#endif
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();   // every wave done reading this stage before it is re-filled
    }
  }
  __syncthreads();

  // ---- epilogue: every wave stages its class tile, then the block stores class by class
  bf16* Cs0 = reinterpret_cast<bf16*>(smem);
  conv_stage_tile<TM, TN, LDC>(a, acc, Cs0 + cls_w * BM * LDC, 0, 32 * nh, n0, lane);
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem + 4 * BM * LDC * 2);
  const FastDiv fd_hwq = make_fastdiv((uint32_t)HWq), fd_wq = make_fastdiv((uint32_t)a.W);
#pragma unroll 1
  for (int cls = 0; cls < 4; ++cls) {
    const ClassGeom g = class_geom<1>(a, cls);
    bf16* Cs = Cs0 + cls * BM * LDC;
    conv_epilogue_tail<BM, BN, 1, NT, EXT>(a, g, m0, n0, Cs, red, reinterpret_cast<char*>(Cs), fd_hwq, fd_wq);
    __syncthreads();
  }
}

template <int W, bool RELU, bool EXT, int F8 = 0>
static int launch_s2t(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int smem = S2TGeom<W>::SMEM;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_s2t_kernel<W, RELU, EXT, F8>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const long mtiles = (long)a.N * a.H * a.W / BM;
  const long blocks = mtiles * (a.Cout / BN);
  hipLaunchKernelGGL((conv_s2t_kernel<W, RELU, EXT, F8>), dim3((unsigned)blocks), dim3(NT), smem, st, a);
  return (int)hipGetLastError();
}

template <int W>
static int dispatch_s2t_w(const ConvFwdArgs& a, bool ext, hipStream_t st) {
  const bool relu = a.act_in == ACT_RELU;
  if (ext) return relu ? -2 : launch_s2t<W, false, true>(a, st);
  return relu ? launch_s2t<W, true, false>(a, st) : launch_s2t<W, false, false>(a, st);
}

}  // namespace p2p

// Geometry gate (the host checks the same before choosing this path, see s2t_ok in
// bindings.cpp): returns -2 when not covered.  fp8: 64-wide grids, 128-channel chunks;
// activations (e4m3) as the ConvT forward with or without its input ReLU, gradients (e5m2)
// as input gradients with or without the extended epilogue.
extern "C" int p2p_conv_s2t(const p2p::ConvFwdArgs* a, hipStream_t st) {
  using namespace p2p;
  if (a->splits != 1 || a->d2s || a->KH != 4 || a->KW != 4 || a->stride != 2 || a->pad != 1 || a->up != 1 ||
      a->reflect)
    return -2;
  const int chc = a->fp8 ? 128 : 64;
  if (a->OH != 2 * a->H || a->OW != 2 * a->W || a->Cout % 64 || a->C1 % chc || a->C2 % chc || a->C1 + a->C2 < chc)
    return -2;
  if ((long)a->H * a->W % 128) return -2;
  if (a->act_in != ACT_NONE && a->act_in != ACT_RELU) return -2;
  const bool ext = a->nb_ws || ((a->act_bwd || a->res1) && !a->epi_serial);
  if (ext && a->act_in) return -2;
  if (a->fp8) {
    if (a->W != 64 || !a->qs_x1 || !a->qs_w || (a->C2 && !a->qs_x2)) return -2;
    if (a->fp8 == 1) {
      if (ext) return -2;
      return a->act_in == ACT_RELU ? launch_s2t<64, true, false, 1>(*a, st) : launch_s2t<64, false, false, 1>(*a, st);
    }
    if (a->act_in) return -2;
    return ext ? launch_s2t<64, false, true, 2>(*a, st) : launch_s2t<64, false, false, 2>(*a, st);
  }
  switch (a->W) {
    case 32: return dispatch_s2t_w<32>(*a, ext, st);
    case 64: return dispatch_s2t_w<64>(*a, ext, st);
    default: return -2;
  }
}
