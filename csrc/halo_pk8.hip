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

// TN = 8 (128 channels) keeps 128 accumulators + 8 B fragments live: one block per CU
// (512-register budget, no spill); TN = 4 runs two blocks per CU
// QS: also write the e4m3 / e5m2 shadow of the output (fp8 precision: the next conv's operand)
template <int TN, int ACT, bool GATE, bool QS = false>
__global__ void __launch_bounds__(256, TN >= 8 ? 1 : 2) halo_pk8_kernel(HaloPk8Args a) {
  float qsc = 0.f, qmax = 0.f;
  if constexpr (QS) qsc = fp8_shadow_scale(Fp8Shadow{a.q, a.q_site, a.q_fmt});
  constexpr int NC = TN * 16;              // output channels of the block (== Cout)
  constexpr int PC = 32;                   // channels per epilogue piece
  constexpr int LDC = PC + 8;              // staging row (80 B: 16-B aligned, spread banks)
  static_assert(256 * LDC * 2 <= SUNITS * 16, "epilogue piece fits in one halo stage");
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
#pragma unroll
    for (int j = 0; j < NLD; ++j) {
      const int iy = 2 * oy0 - 1 + hy[j], ix = 2 * ox0 - 1 + hx[j];
      const bool inb = (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
      glds16(inb ? a.x + ((long)(n * a.Hi + iy) * a.Wi + ix) * 8 : a.zero, dst + (j * 4 + wid) * 64 * 8);
    }
  };

  const int px = lane & 15, kq = lane >> 4;
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
    // the epilogue's output pixels, and (GATE) the act' inputs of ALL its pieces, issued here:
    // their HBM latency runs behind the K loop instead of once per 32-channel piece after a
    // barrier (round 6: the 128-channel gated input gradient streamed at 3.1 TB/s)
    int n, oy0, ox0;
    origin(k, n, oy0, ox0);
    long pix[4];
    bool ok[4];
    u32x4 xg[GATE ? NC / PC : 1][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {               // 256 pixels x 4 chunks of 8 channels
      const int it = tid + q * 256, row = it >> 2;
      const int oy = oy0 + (row >> 4), ox = ox0 + (row & 15);
      ok[q] = oy < a.Ho && ox < a.Wo;
      pix[q] = ((long)n * a.Ho + (ok[q] ? oy : 0)) * a.Wo + (ok[q] ? ox : 0);
    }
    if constexpr (GATE) {
#pragma unroll
      for (int piece = 0; piece < NC / PC; ++piece) {
        const int co0 = piece * PC;
        const bool first = co0 < a.Csplit;
        const int ld = first ? a.Csplit : NC - a.Csplit;
        const int cof0 = first ? co0 : co0 - a.Csplit;
        const bf16* xb = first ? a.xb1 : a.xb2;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int it = tid + q * 256;
          xg[piece][q] = xb ? *reinterpret_cast<const u32x4*>(xb + pix[q] * ld + cof0 + (it & 3) * 8)
                            : u32x4{0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};
        }
      }
    }
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
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (n * 16 + (tap ^ (n & 15))) * 8);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int py = wid * 4 + i;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(A + unit_of(2 * py + ty, 2 * px + tx) * 8);
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();     // every wave done with this stage: it hosts the staging tile
    // ---- epilogue, 32 channels at a time: bias + act staged as bf16 in this stage's LDS,
    // then 16-B stores (the ReLU-gate inputs were loaded before the K loop)
    bf16* Cs = A;
#pragma unroll
    for (int piece = 0; piece < NC / PC; ++piece) {
#pragma unroll
      for (int j = piece * 2; j < piece * 2 + 2; ++j) {
        const int col = j * 16 + px;
        const float bj = a.bias ? a.bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rowb = wid * 64 + i * 16 + kq * 4;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(rowb + r) * LDC + (col - piece * PC)] = (bf16)act_fwd(acc[i][j][r] + bj, ACT);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      const int co0 = piece * PC;
      const bool first = co0 < a.Csplit;          // a piece never straddles the split (host)
      const int ld = first ? a.Csplit : NC - a.Csplit;
      const int cof0 = first ? co0 : co0 - a.Csplit;
      bf16* yb = first ? a.y1 : a.y2;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int it = tid + q * 256, row = it >> 2, cc = it & 3;
        if (!ok[q]) continue;
        u32x4 v = *reinterpret_cast<const u32x4*>(Cs + row * LDC + cc * 8);
        if constexpr (GATE) {   // ReLU' of the layer's input (dgrad of a ReLU-input conv)
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const uint32_t xw = xg[GATE ? piece : 0][q][w];
            uint32_t keep = 0;
            if ((int16_t)(xw & 0xffffu) > 0) keep |= 0xffffu;
            if ((int16_t)(xw >> 16) > 0) keep |= 0xffff0000u;
            v[w] &= keep;
          }
        }
        *reinterpret_cast<u32x4*>(yb + pix[q] * ld + cof0 + cc * 8) = v;
        if constexpr (QS) {   // host: unsplit output (ld == Cout)
          const bf16x8 vb = __builtin_bit_cast(bf16x8, v);
          float r[8];
#pragma unroll
          for (int w = 0; w < 8; ++w) {
            r[w] = (float)vb[w];
            qmax = fmaxf(qmax, fabsf(r[w]));
          }
          *reinterpret_cast<uint2*>(a.q + pix[q] * ld + cof0 + cc * 8) = fp8_pack8(r, qsc, a.q_fmt);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
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
