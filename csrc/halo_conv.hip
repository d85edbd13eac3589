// Halo-tile direct conv for the 3x3 "union" GEMM of the packed-image layers (csrc/image.hip):
// the generator's last transposed conv (d1 forward, C = 128) and the discriminator's first
// conv's input gradient (head gradient, C = 64), both 16 GEMM columns (4 parity classes x 3
// image channels + 1 pad).
//
// As an implicit GEMM (conv_fwd_glds.hip, 256x32 tile) every input pixel is fetched from
// L2 into LDS once per TAP -- 9x -- for only 16-32 MACs per element: the L2 -> LDS path,
// not the MFMA, bounds it (~0.28 PF/s, 1.1 ms for d1 at B = 256).  Here a block owns a
// 16 x 16 block of the input grid and stages its 18 x 18 halo ONCE per 64-channel chunk
// (global_load_lds, source-side swizzle); the 9 taps read their A fragments out of that
// one LDS image at shifted pixel offsets.  The whole B operand (16 x 9 x C, <= 37 KB) stays
// resident.  Persistent blocks walk the tiles with the next (tile, chunk) halo in flight
// while the current one feeds the MFMAs (2-stage ring, counted vmcnt + raw s_barrier).
//
// LDS image of one stage: 16-B unit e = pixel * 8 + (kc ^ ((pixel >> 1) & 7)) holds
// channels [8 kc, 8 kc + 8) of halo pixel ``pixel`` (row-major 18 x 18): 16 consecutive
// pixels of a ds_read_b128 lane group hit 16 distinct bank slots (conv_dev.h swz()).
#include "conv_dev.h"

namespace p2p {

namespace {

constexpr int HT = 16;                  // q tile edge
constexpr int HP = HT + 2;              // halo edge
constexpr int HPIX = HP * HP;           // 324 halo pixels
constexpr int HUNITS = HPIX * 8;        // 16-B units per 64-channel chunk
constexpr int NTH = 512;                // 8 waves: 2 per SIMD at one block per CU (round 4:
                                        // 4 waves left a single wave per SIMD to hide every
                                        // halo and epilogue round trip of this memory-bound layer)
constexpr int NW = NTH / 64;
constexpr int RPW = HT / NW;            // q rows (16-pixel fragments) per wave
constexpr int HLD = (HUNITS + NTH - 1) / NTH;  // glds per lane per stage (6)
constexpr int STAGE_UNITS = HLD * NTH;
constexpr int STAGE_BYTES = STAGE_UNITS * 16;
constexpr int LDC = 24;                 // epilogue staging row (16 columns + pad)

__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(lds_wave_base), 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 16-B units of the resident weight operand, rounded up to whole block-wide glds rounds:
// the kernel's B loop writes exactly this many units and the launcher reserves exactly
// this many (the launcher rounded to 256 units while the 512-thread loop wrote
// up to the next 512-unit multiple -- 4 KB past the allocation per launch).
template <int NCH>
constexpr int b_units_pad() {
  return (9 * NCH * 16 * 8 + NTH - 1) / NTH * NTH;
}

template <int NCH>
constexpr int halo_smem_bytes() {
  return 2 * STAGE_BYTES + b_units_pad<NCH>() * 16;
}

}  // namespace


template <int NCH, bool RELU>
__global__ void __launch_bounds__(NTH) halo_union_kernel(HaloArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* As = reinterpret_cast<bf16*>(smem);                       // 2 stages
  bf16* Bs = reinterpret_cast<bf16*>(smem + 2 * STAGE_BYTES);     // [9][NCH][16][64]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int C = a.C1 + a.C2;
  const int my_tiles = (a.ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  if (my_tiles <= 0) return;
  const int total = my_tiles * NCH;

  // ---- resident B operand (waited together with the first stage)
  constexpr int BUNITS = 9 * NCH * 16 * 8;
  constexpr int BUNITS_PAD = b_units_pad<NCH>();   // whole block-wide glds rounds
#pragma unroll
  for (int e0 = wid * 64; e0 < BUNITS_PAD; e0 += NTH) {
    const int e = e0 + lane;
    const int n = (e >> 3) & 15, tc = e >> 7;
    const int tap = tc / NCH, ch = tc - tap * NCH;
    const int kc = (e & 7) ^ ((n >> 1) & 7);
    glds16(e < BUNITS ? a.w + (long)(n * 9 + tap) * C + ch * 64 + kc * 8 : a.zero, Bs + e0 * 8);
  }

  // ---- per-lane halo units (fixed across tiles): pixel row / col and logical chunk
  int hy[HLD], hx[HLD], kcs[HLD];
#pragma unroll
  for (int j = 0; j < HLD; ++j) {
    const int e = (j * NW + wid) * 64 + lane;
    const int hp = e >> 3;
    hy[j] = hp < HPIX ? hp / HP : -4096;   // beyond the halo: out of image -> zero page
    hx[j] = hp - (hp / HP) * HP;
    kcs[j] = (e & 7) ^ ((hp >> 1) & 7);
  }
  const int tiles_img = a.tiles_x * a.tiles_y;
  auto tile_origin = [&](int k, int& n, int& qy0, int& qx0) {
    const int t = (int)blockIdx.x + k * (int)gridDim.x;
    n = t / tiles_img;
    const int r = t - n * tiles_img;
    qy0 = (r / a.tiles_x) * HT;
    qx0 = (r % a.tiles_x) * HT;
  };
  auto issue = [&](int it, int stage) {
    int n, qy0, qx0;
    tile_origin(it / NCH, n, qy0, qx0);
    const int ch = it % NCH;
    const bool s1 = ch * 64 < a.C1;
    const bf16* src = s1 ? a.x1 : a.x2;
    const int cs = s1 ? a.C1 : a.C2;
    const int coff = s1 ? ch * 64 : ch * 64 - a.C1;
    bf16* dst = As + stage * (STAGE_UNITS * 8);
#pragma unroll
    for (int j = 0; j < HLD; ++j) {
      const int iy = qy0 - 1 + hy[j], ix = qx0 - 1 + hx[j];
      const bool inb = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
      const bf16* g = inb ? src + ((long)(n * a.H + iy) * a.W + ix) * cs + coff + kcs[j] * 8 : a.zero;
      glds16(g, dst + (j * NW + wid) * 64 * 8);
    }
  };

  f32x4 acc[RPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float l1 = 0.f;
  // mode 2: the L1 sign term's weight = scale x dL/dl1 (a device scalar written by autograd)
  const float l1w = a.scale * (a.mode == 2 && a.wscale ? *a.wscale : 1.f);
  const int px = lane & 15, kq = lane >> 4;
  // the depth-to-space epilogue's packed-image operands of the current tile, loaded when its
  // first chunk starts: their HBM latency runs behind the tile's MFMAs instead of after the
  // epilogue's barrier (round 6; the kernel streamed at 3.9-4.4 TB/s)
  constexpr int PQ = 1024 / NTH;   // output pixels per thread (256 q x 4 classes)
  long P[PQ];
  bool ok[PQ];
  bf16x8 ab[PQ], af[PQ];

  issue(0, 0);
  for (int it = 0; it < total; ++it) {
    const int stage = it & 1;
    if (it + 1 < total) {
      issue(it + 1, stage ^ 1);
      wait_vm<HLD>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const int ch = it % NCH;
    const bf16* A = As + stage * (STAGE_UNITS * 8);
    if (ch == 0) {
      int n, qy0, qx0;
      tile_origin(it / NCH, n, qy0, qx0);
      const int Ho = 2 * a.H, Wo = 2 * a.W;
#pragma unroll
      for (int q = 0; q < PQ; ++q) {
        const int item = tid + q * NTH, row = item >> 2, cls = item & 3;
        const int qy = qy0 + (row >> 4), qx = qx0 + (row & 15);
        ok[q] = qy < a.H && qx < a.W;
        P[q] = ((long)n * Ho + 2 * (ok[q] ? qy : 0) + (cls >> 1)) * Wo + 2 * (ok[q] ? qx : 0) + (cls & 1);
        ab[q] = *reinterpret_cast<const bf16x8*>(a.pk_a + P[q] * 8);
        if (a.mode == 2) af[q] = *reinterpret_cast<const bf16x8*>(a.pk_f + P[q] * 8);
      }
    }
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int uy = tap / 3, ux = tap % 3;
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const int kc = kh * 4 + kq;
        const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(
            Bs + (((tap * NCH + ch) * 16 + px) * 8 + (kc ^ ((px >> 1) & 7))) * 8);
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
          const int hp = (wid * RPW + i + uy) * HP + px + ux;
          bf16x8 af = *reinterpret_cast<const bf16x8*>(A + (hp * 8 + (kc ^ ((hp >> 1) & 7))) * 8);
          if constexpr (RELU) af = __builtin_bit_cast(bf16x8, relu8(__builtin_bit_cast(u32x4, af)));
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[i], 0, 0, 0);
        }
      }
    }
    __builtin_amdgcn_s_barrier();   // every wave done reading this stage
    if (ch == NCH - 1) {
      // ---- epilogue of the tile: bias + act into a bf16 tile in this stage's LDS, then the
      // depth-to-space packed stores (conv_dev.h d2s_pixel)
      int n, qy0, qx0;
      tile_origin(it / NCH, n, qy0, qx0);
      bf16* Cs = As + stage * (STAGE_UNITS * 8);
      const float bj = a.bias[px];
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        const int rowb = (wid * RPW + i) * 16 + kq * 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[i][r] + bj;
          Cs[(rowb + r) * LDC + px] = (bf16)(a.act_out == ACT_TANH ? tanhf(v) : v);
        }
        acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      // depth-to-space stores: 4 output pixels per thread (operands loaded at the tile start)
#pragma unroll
      for (int q = 0; q < PQ; ++q) {
        const int item = tid + q * NTH, row = item >> 2, cls = item & 3;
        if (!ok[q]) continue;
        const bf16* c = Cs + row * LDC + cls * 4;
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (bf16)0.f;
        if (a.mode == 1) {
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            o[j] = ab[q][j];
            o[3 + j] = c[j];
            l1 += fabsf((float)c[j] - (float)ab[q][3 + j]);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            const float f = (float)af[q][3 + j], b = (float)ab[q][3 + j];
            const float sg = (float)(f > b) - (float)(f < b);
            o[j] = (bf16)(((float)c[j] + l1w * sg) * (1.f - f * f));
          }
        }
        *reinterpret_cast<bf16x8*>(a.out + P[q] * 8) = o;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();   // staging read before the stage is re-filled
    }
  }
  if (a.mode == 1 && a.l1_part) {
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) l1 += __shfl_xor(l1, off);
    __syncthreads();
    if (lane == 0) red[wid] = l1;
    __syncthreads();
    if (tid == 0) {
      float t = 0.f;
      for (int w = 0; w < NW; ++w) t += red[w];
      a.l1_part[blockIdx.x] = t;
    }
  }
}

template <int NCH, bool RELU>
static int launch_halo(const HaloArgs& a, int blocks, hipStream_t st) {
  constexpr int smem = halo_smem_bytes<NCH>();
  static_assert(smem >= 2 * STAGE_BYTES + b_units_pad<NCH>() * 16 && smem <= 160 * 1024,
                "the B loop's padded writes stay inside the reserved LDS");
  static std::atomic<uint64_t> attr_mask{0};
  smem_attr_once(reinterpret_cast<const void*>(&halo_union_kernel<NCH, RELU>), smem, attr_mask);
  hipLaunchKernelGGL((halo_union_kernel<NCH, RELU>), dim3(blocks), dim3(NTH), smem, st, a);
  return (int)hipGetLastError();
}

}  // namespace p2p

// returns -2 when the geometry is not covered (caller falls back to the implicit GEMM)
extern "C" int p2p_halo_union(const p2p::HaloArgs* a, int relu, int blocks, hipStream_t st) {
  using namespace p2p;
  if (a->C1 % 64 || a->C2 % 64 || a->C1 + a->C2 > 128 || a->C1 + a->C2 < 64) return -2;
  const int nch = (a->C1 + a->C2) / 64;
  if (nch == 1) return relu ? launch_halo<1, true>(*a, blocks, st) : launch_halo<1, false>(*a, blocks, st);
  return relu ? launch_halo<2, true>(*a, blocks, st) : launch_halo<2, false>(*a, blocks, st);
}

extern "C" int p2p_halo_args_size() { return (int)sizeof(p2p::HaloArgs); }
