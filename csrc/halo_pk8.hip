// Halo-tile direct conv for the packed 8-channel image convs: 4x4, stride 2, pad 1 over a
// [N][Hi][Wi][8] bf16 input (16 B = one pixel = one tap of 8 channels) -- the generator's
// first conv (A | B pair, zero weights on B), the discriminator's first conv (2B and B
// batches) and the generator's last layer's input gradient (d1 dgrad, 128 channels split
// into the skip / up halves with the ReLU gate of its input).
//
// As an implicit GEMM these layers have K = 16 taps x 8 = 128 (two K tiles), so every tile
// pays the full load latency twice for a few MFMAs and every input pixel is fetched through
// L2 four times (once per output pixel whose window covers it).  Here a block owns a 16 x 16
// block of OUTPUT pixels and stages the 34 x 34 input halo ONCE (global_load_lds, 18.5 KB);
// each lane's A fragment for tap (ty, tx) is one ds_read_b128 of input pixel
// (2 py + ty, 2 px + tx).  The halo image keeps even and odd columns apart, so the 16 lanes
// of a read group (16 consecutive output columns = 16 input pixels two apart) read 16
// consecutive units: conflict-free.  The [Cout][16 taps][8] weight stays resident with its
// tap slot XORed by the row (16 rows x 16 slots -> distinct banks).  Persistent blocks walk
// the tiles with the next halo in flight behind the current tile's MFMAs and epilogue.
#include "conv_dev.h"

namespace p2p {

namespace {

constexpr int OT = 16;                   // output tile edge
constexpr int IH = 2 * OT + 2;           // input halo edge (34)
constexpr int HALF = IH / 2;             // 17 units per column-parity half-row
constexpr int HUN = IH * IH;             // 1156 units (pixels)
constexpr int NLD = (HUN + 255) / 256;   // glds per lane per stage (5)
constexpr int SUNITS = NLD * 256;

__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(lds_wave_base), 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// halo unit of input pixel (hy, hx): rows of [even columns | odd columns]
__device__ __forceinline__ int unit_of(int hy, int hx) { return (hy * 2 + (hx & 1)) * HALF + (hx >> 1); }

}  // namespace

// TN = 8 (128 channels) keeps 128 accumulators + 8 weight fragments live: one block per CU
// (512-register budget; at two blocks per CU it spills); TN = 4 runs two blocks per CU.
// QS: also write the e4m3 / e5m2 shadow of the output (fp8 precision: the next conv's operand)
//
// Round 4: the MFMA operands are swapped (weight = src A, halo pixels = src B), so a lane's
// accumulator holds 4 CONSECUTIVE output channels of one output pixel and the epilogue runs
// from registers -- bf16 conversion, all of the tile's ReLU-gate loads in flight at once,
// 8-byte stores -- instead of four 32-channel pieces staged through LDS behind barriers, each
// one HBM round trip (the GATE variant, the generator head's input gradient, ran at 3 TB/s).
template <int TN, int ACT, bool GATE, bool QS = false>
__global__ void __launch_bounds__(256, TN >= 8 ? 1 : 2) halo_pk8_kernel(HaloPk8Args a) {
  float qsc = 0.f, qmax = 0.f;
  if constexpr (QS) qsc = fp8_shadow_scale(Fp8Shadow{a.q, a.q_site, a.q_fmt});
  constexpr int NC = TN * 16;              // output channels of the block (== Cout)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* As = reinterpret_cast<bf16*>(smem);                               // 2 x SUNITS units
  bf16* Bs = As + 2 * SUNITS * 8;                                         // NC x 16 units
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int my_tiles = (a.ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  if (my_tiles <= 0) return;

  // ---- resident weight: unit (n, tap) at n * 16 + (tap ^ (n & 15))
  static_assert((NC * 16) % 256 == 0, "weight units per wave instruction");
#pragma unroll
  for (int e0 = wid * 64; e0 < NC * 16; e0 += 256) {
    const int e = e0 + lane;
    const int n = e >> 4, tap = (e & 15) ^ (n & 15);
    glds16(a.w + (long)n * 128 + tap * 8, Bs + e0 * 8);
  }

  // ---- per-lane halo units (fixed across tiles)
  int hy[NLD], hx[NLD];
#pragma unroll
  for (int j = 0; j < NLD; ++j) {
    const int e = (j * 4 + wid) * 64 + lane;   // lane-linear LDS unit
    const int row2 = e / HALF, c = e - row2 * HALF;
    hy[j] = e < HUN ? (row2 >> 1) : -4096;
    hx[j] = 2 * c + (row2 & 1);
  }
  const int tiles_img = a.tiles_x * a.tiles_y;
  auto origin = [&](int k, int& n, int& oy0, int& ox0) {
    const int t = (int)blockIdx.x + k * (int)gridDim.x;
    n = t / tiles_img;
    const int r = t - n * tiles_img;
    oy0 = (r / a.tiles_x) * OT;
    ox0 = (r % a.tiles_x) * OT;
  };
  auto issue = [&](int k, int stage) {
    int n, oy0, ox0;
    origin(k, n, oy0, ox0);
    bf16* dst = As + stage * SUNITS * 8;
    // laundered: the per-lane unit geometry must not be hoisted into (spilled) registers
    int w = wid;
    asm volatile("" : "+v"(w));
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const int iy = 2 * oy0 - 1 + hy[j], ix = 2 * ox0 - 1 + hx[j];
      const bool inb = (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
      glds16(inb ? a.x + ((long)(n * a.Hi + iy) * a.Wi + ix) * 8 : a.zero, dst + (j * 4 + w) * 64 * 8);
    }
  };

  const int px = lane & 15, kq = lane >> 4, g = lane >> 4;
  issue(0, 0);
  for (int k = 0; k < my_tiles; ++k) {
    const int stage = k & 1;
    if (k + 1 < my_tiles) {
      issue(k + 1, stage ^ 1);
      wait_vm<NLD>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    bf16* A = As + stage * SUNITS * 8;
    // the resident weight's fragments are the same for every tile: hoisted out of the tile
    // loop they would pin 16 taps x TN fragments of registers (and spill at two blocks per
    // CU) -- a per-tile laundered base keeps them per k-step LDS reads
    const bf16* Bt = Bs;
    asm volatile("" : "+v"(Bt));
    f32x4 acc[4][TN];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {           // 4 taps per 32-deep MFMA step
      const int tap = ks * 4 + kq, ty = tap >> 2, tx = tap & 3;
      bf16x8 bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = j * 16 + px;
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bt + (n * 16 + (tap ^ (n & 15))) * 8);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int py = wid * 4 + i;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(A + unit_of(2 * py + ty, 2 * px + tx) * 8);
#pragma unroll
        for (int j = 0; j < TN; ++j)   // weights = src A (rows = channels), pixels = src B
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af, acc[i][j], 0, 0, 0);
      }
      // one k-step's fragments live at a time (TN = 8: 128 accumulators + 48 fragment registers)
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();     // every wave done with this stage: the next tile's lands here

    // ---- register epilogue: acc[i][j][r] = channel 16 j + 4 g + r of output pixel
    // (oy0 + 4 wid + i, ox0 + px)
    int n, oy0, ox0;
    origin(k, n, oy0, ox0);
    const int ox = ox0 + px;
    uint2 v[4][TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float bj[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) bj[r] = a.bias ? a.bias[j * 16 + 4 * g + r] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float f[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) f[r] = act_fwd(acc[i][j][r] + bj[r], ACT);
        const bf16 b0 = (bf16)f[0], b1 = (bf16)f[1], b2 = (bf16)f[2], b3 = (bf16)f[3];
        v[i][j] = uint2{(uint32_t)__builtin_bit_cast(uint16_t, b0) | ((uint32_t)__builtin_bit_cast(uint16_t, b1) << 16),
                        (uint32_t)__builtin_bit_cast(uint16_t, b2) | ((uint32_t)__builtin_bit_cast(uint16_t, b3) << 16)};
      }
    }
    long pix[4];
    bool ok[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int oy = oy0 + wid * 4 + i;
      ok[i] = oy < a.Ho && ox < a.Wo;
      pix[i] = ((long)n * a.Ho + (ok[i] ? oy : 0)) * a.Wo + (ok[i] ? ox : 0);
    }
    if constexpr (GATE) {
      // ReLU' of the layer's input (dgrad of a ReLU-input conv): the gate loads of up to 4
      // channel columns (16 loads of 8 B per lane) in flight at once
      constexpr int JG = TN < 4 ? TN : 4;
#pragma unroll
      for (int j0 = 0; j0 < TN; j0 += JG) {
        uint2 xv[4][JG];
#pragma unroll
        for (int jj = 0; jj < JG; ++jj) {
          const int co = (j0 + jj) * 16 + 4 * g;
          const bool first = co < a.Csplit;        // a 16-channel column never straddles the split
          const int ld = first ? a.Csplit : NC - a.Csplit;
          const bf16* xb = first ? a.xb1 : a.xb2;
          const int cof = first ? co : co - a.Csplit;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            xv[i][jj] = (xb && ok[i]) ? *reinterpret_cast<const uint2*>(xb + pix[i] * ld + cof)
                                      : uint2{0x3f803f80u, 0x3f803f80u};
        }
#pragma unroll
        for (int jj = 0; jj < JG; ++jj)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t x0 = xv[i][jj].x, x1 = xv[i][jj].y;
            uint2& w = v[i][j0 + jj];
            w.x &= (((int16_t)(x0 & 0xffffu) > 0) ? 0xffffu : 0u) | (((int16_t)(x0 >> 16) > 0) ? 0xffff0000u : 0u);
            w.y &= (((int16_t)(x1 & 0xffffu) > 0) ? 0xffffu : 0u) | (((int16_t)(x1 >> 16) > 0) ? 0xffff0000u : 0u);
          }
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int co = j * 16 + 4 * g;
      const bool first = co < a.Csplit;
      const int ld = first ? a.Csplit : NC - a.Csplit;
      const int cof = first ? co : co - a.Csplit;
      bf16* yb = first ? a.y1 : a.y2;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (!ok[i]) continue;
        *reinterpret_cast<uint2*>(yb + pix[i] * ld + cof) = v[i][j];
        if constexpr (QS) {   // host: unsplit output (ld == Cout)
          const float fm = fp8_max(a.q_fmt);
          float f[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t w = r < 2 ? v[i][j].x : v[i][j].y;
            f[r] = __uint_as_float((r & 1) ? (w & 0xffff0000u) : (w << 16));
            qmax = fmaxf(qmax, fabsf(f[r]));
            f[r] = fminf(fmaxf(f[r] * qsc, -fm), fm);
          }
          *reinterpret_cast<uint32_t*>(a.q + pix[i] * ld + cof) = cvt4(f[0], f[1], f[2], f[3], a.q_fmt);
        }
      }
    }
  }
  if constexpr (QS) fp8_amax_commit(qmax, a.q_site);
}

template <int TN, int ACT, bool GATE, bool QS = false>
static int launch_pk8(const HaloPk8Args& a, int blocks, hipStream_t st) {
  constexpr int smem = (2 * SUNITS + TN * 16 * 16) * 16;
  static std::atomic<uint64_t> attr_mask{0};
  smem_attr_once(reinterpret_cast<const void*>(&halo_pk8_kernel<TN, ACT, GATE, QS>), smem, attr_mask);
  hipLaunchKernelGGL((halo_pk8_kernel<TN, ACT, GATE, QS>), dim3(blocks), dim3(256), smem, st, a);
  return (int)hipGetLastError();
}

}  // namespace p2p

// -2: geometry / epilogue not covered (the caller uses the implicit GEMM)
extern "C" int p2p_halo_pk8(const p2p::HaloPk8Args* a, int blocks, hipStream_t st) {
  using namespace p2p;
  const bool gate = a->xb1 != nullptr || a->xb2 != nullptr;
  if (a->Csplit % 32) return -2;   // epilogue pieces never straddle the split
  if (a->q && (a->Cout != 64 || gate || a->Csplit != a->Cout)) return -2;
  if (a->Cout == 64 && !gate && a->q) {
    if (a->act_out == ACT_LRELU) return launch_pk8<4, ACT_LRELU, false, true>(*a, blocks, st);
    if (a->act_out == ACT_RELU) return launch_pk8<4, ACT_RELU, false, true>(*a, blocks, st);
    return -2;
  }
  if (a->Cout == 64 && !gate) {
    if (a->act_out == ACT_LRELU) return launch_pk8<4, ACT_LRELU, false>(*a, blocks, st);
    if (a->act_out == ACT_NONE) return launch_pk8<4, ACT_NONE, false>(*a, blocks, st);
    if (a->act_out == ACT_RELU) return launch_pk8<4, ACT_RELU, false>(*a, blocks, st);
    return -2;
  }
  if (a->Csplit % 32) return -2;   // epilogue pieces never straddle the split
  if (a->Cout == 128 && a->act_out == ACT_NONE) {
    if (gate) return launch_pk8<8, ACT_NONE, true>(*a, blocks, st);
    return launch_pk8<8, ACT_NONE, false>(*a, blocks, st);
  }
  return -2;
}
