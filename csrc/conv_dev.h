// Device-side pieces shared by the implicit-GEMM conv kernels (conv_fwd.hip: register-
// staged; conv_fwd_glds.hip: global_load_lds multi-stage): tile geometry of the two GEMM
// modes, the LDS swizzle of the [rows][64] bf16 operand tiles, and the fused epilogue.
#pragma once
#include "bounds.h"
#include "conv.h"
#include "fp8_dev.h"

namespace p2p {

constexpr int BK = 64;

__device__ __forceinline__ int swz(int row, int chunk) {  // element offset in a [rows][64] tile
  return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3);
}

struct ClassGeom {
  int ry, rx, ky0, kx0, dy, dx, Tj, Ti, Hq, Wq, Mc, Kc;
};

template <int MODE>
__device__ __forceinline__ ClassGeom class_geom(const ConvFwdArgs& a, int cls) {
  ClassGeom g;
  if (MODE == 0) {
    g.ry = g.rx = g.ky0 = g.kx0 = g.dy = g.dx = 0;
    g.Tj = a.KH;
    g.Ti = a.KW;
    g.Hq = a.OH;
    g.Wq = a.OW;
  } else {
    const int s = a.stride, p = a.pad;
    g.ry = cls / s;
    g.rx = cls % s;
    g.ky0 = (g.ry + p) % s;
    g.kx0 = (g.rx + p) % s;
    g.dy = (g.ry + p - g.ky0) / s;
    g.dx = (g.rx + p - g.kx0) / s;
    g.Tj = g.ky0 < a.KH ? (a.KH - g.ky0 + s - 1) / s : 0;
    g.Ti = g.kx0 < a.KW ? (a.KW - g.kx0 + s - 1) / s : 0;
    g.Hq = a.OH > g.ry ? (a.OH - g.ry + s - 1) / s : 0;
    g.Wq = a.OW > g.rx ? (a.OW - g.rx + s - 1) / s : 0;
  }
  g.Mc = a.N * g.Hq * g.Wq;
  g.Kc = g.Tj * g.Ti * a.C;
  return g;
}

// One packed output pixel P of the depth-to-space epilogue (conv.h ``d2s``) from its three
// GEMM values c[0..2]: mode 1 writes (pk_a[0..2], c, 0, 0) and returns sum|c - pk_a[3..5]|;
// mode 2 writes ((c + scale * sign(f - b)) * (1 - f^2), 0 ...) with f = pk_f[3..5], b = pk_a[3..5]
// (scale already multiplied by the device weight dL/dl1 by the caller).
__device__ __forceinline__ float d2s_pixel(int mode, long P, const bf16* c, const bf16* pk_a, const bf16* pk_f,
                                           float scale, bf16* out) {
  const bf16x8 ab = *reinterpret_cast<const bf16x8*>(pk_a + P * 8);
  bf16x8 o;
#pragma unroll
  for (int q = 0; q < 8; ++q) o[q] = (bf16)0.f;
  float l1 = 0.f;
  if (mode == 1) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      o[j] = ab[j];
      o[3 + j] = c[j];
      l1 += fabsf((float)c[j] - (float)ab[3 + j]);
    }
  } else {
    const bf16x8 af = *reinterpret_cast<const bf16x8*>(pk_f + P * 8);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float f = (float)af[3 + j], b = (float)ab[3 + j];
      const float sg = (float)(f > b) - (float)(f < b);
      o[j] = (bf16)(((float)c[j] + scale * sg) * (1.f - f * f));
    }
  }
  *reinterpret_cast<bf16x8*>(out + P * 8) = o;
  return l1;
}

// Store loop of the EXT dgrad epilogue (see conv_epilogue): the bf16 tile is staged in Cs.
// Per output chunk: act'(x) gate, + the parked skip gradient, store, and -- for the channels
// of a norm's output (nb_*) -- sum(d) / sum(d * xhat) with d = dz * act'(xhat) (non-affine
// norms; the host only fuses those).  A thread's 8-channel chunk is fixed (NT % CPR == 0);
// its operand loads are issued two rows ahead so their latencies overlap.
template <int BM, int BN, int MODE, int NT, typename PixF>
__device__ __forceinline__ void conv_epilogue_ext(const ConvFwdArgs& a, const ClassGeom& g, int m0, int n0,
                                                  char* smem, const bf16* Cs, int LDC, int HWq, int s,
                                                  PixF&& out_pix) {
  constexpr int CPR = BN / 8;
  static_assert(NT % CPR == 0, "a thread's 8-channel chunk is fixed across the store loop");
  static_assert(64 % CPR == 0, "the lanes sharing a chunk lie in one wave");
  const int tid = threadIdx.x;
  const int co_t = n0 + (tid % CPR) * 8;
  const bool first_t = co_t < a.Csplit;
  const int ld_t = first_t ? a.Csplit : a.Cout - a.Csplit;
  const int cof_t = first_t ? co_t : co_t - a.Csplit;
  const bf16* xb_t = static_cast<const bf16*>(first_t ? a.xb1 : a.xb2);
  const bool res_t = a.res1 && first_t;    // host: res1 only with Csplit == Cout
  bf16* y_t = static_cast<bf16*>(first_t ? a.y1 : a.y2);
  const bf16* res_p = static_cast<const bf16*>(a.res1);
  const bf16* nbx_p = static_cast<const bf16*>(a.nb_x);
  const int nb_co = co_t - a.nb_c0;
  const bool nb_on = a.nb_ws != nullptr && nb_co >= 0 && nb_co < a.nb_C;
  const bool nb_x_on = nb_on && !a.nb_colsum;   // colsum mode: d = dz, xhat = 0 (rs = c1 = 0)
  const float nb_slope = a.nb_colsum ? 1.f : (a.nb_prelu ? *a.nb_prelu : (a.nb_act ? neg_slope(a.nb_act) : 1.f));
  const bool nb_p3 = a.nb_prelu != nullptr;   // third plane: the PReLU slope-gradient terms
  // act' gate (a null half is gated by its producer's backward): from the xhat of the nb
  // partials when the gated input is the norm's output itself (nb_gate), else loaded
  const bool gate_nb = a.act_bwd && xb_t && nb_x_on && a.nb_gate;
  const bool gate_t = a.act_bwd && xb_t && !gate_nb;
  const float gate_slope = gate_nb ? neg_slope(a.act_bwd) : 0.f;
  // xhat = x * rs + c1 (c1 = -mean * rstd); the gate's z = xhat * g + b = x * zs + zc
  float rs[8], c1[8], zs[8], zc[8], s1[8], s2[8], s3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    rs[j] = c1[j] = s1[j] = s2[j] = s3[j] = 0.f;
    if (nb_on && !a.nb_colsum) {
      const long si = a.nb_batch ? nb_co + j : (long)(m0 / HWq) * a.nb_C + nb_co + j;
      rs[j] = a.nb_rstd[si];
      c1[j] = -a.nb_mean[si] * rs[j];
    }
    const float ga = a.nb_gamma && nb_on ? a.nb_gamma[nb_co + j] : 1.f;
    const float be = a.nb_gamma && nb_on ? a.nb_beta[nb_co + j] : 0.f;
    zs[j] = rs[j] * ga;
    zc[j] = c1[j] * ga + be;
  }
  const u32x4 z4 = {0u, 0u, 0u, 0u};
  auto ld16 = [](const bf16* p) __attribute__((always_inline)) { return *reinterpret_cast<const u32x4*>(p); };
  auto finish = [&](int row, long pix, u32x4 xv, u32x4 rv, u32x4 nv) __attribute__((always_inline)) {
    u32x4 v = *reinterpret_cast<const u32x4*>(Cs + row * LDC + (tid % CPR) * 8);
    if (pix < 0) {   // fold frame pixel (no nb partials with a fold: host)
      if (P2P_OOB_OK(1, (-pix - 2) * a.Cout + co_t, 8, (long)a.N * a.OH * a.OW * a.Cout))
        *reinterpret_cast<u32x4*>(static_cast<bf16*>(a.fold_buf) + (-pix - 2) * a.Cout + co_t) = v;
      return;
    }
    if (gate_t) {
      if (a.act_bwd == ACT_RELU) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t xw = xv[q];
          uint32_t keep = 0;
          if ((int16_t)(xw & 0xffffu) > 0) keep |= 0xffffu;
          if ((int16_t)(xw >> 16) > 0) keep |= 0xffff0000u;
          v[q] &= keep;
        }
      } else {
        bf16x8 vb = __builtin_bit_cast(bf16x8, v);
        const bf16x8 xb8 = __builtin_bit_cast(bf16x8, xv);
#pragma unroll
        for (int q = 0; q < 8; ++q)
          vb[q] = (bf16)((float)vb[q] * act_grad_from_input((float)xb8[q], a.act_bwd));
        v = __builtin_bit_cast(u32x4, vb);
      }
    }
    if (gate_nb) {
      bf16x8 vb = __builtin_bit_cast(bf16x8, v);
      const bf16x8 xn = __builtin_bit_cast(bf16x8, nv);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float xh = (float)xn[q] * rs[q] + c1[q];
        vb[q] = (bf16)((float)vb[q] * (xh > 0.f ? 1.f : gate_slope));
      }
      v = __builtin_bit_cast(u32x4, vb);
    }
    if (res_t) {
      bf16x8 vb = __builtin_bit_cast(bf16x8, v);
      const bf16x8 rb = __builtin_bit_cast(bf16x8, rv);
#pragma unroll
      for (int q = 0; q < 8; ++q) vb[q] = (bf16)((float)vb[q] + (float)rb[q]);
      v = __builtin_bit_cast(u32x4, vb);
    }
    if (P2P_OOB_OK(2, pix * ld_t + cof_t, 8,
                   (long)a.N * (a.fold_buf ? (long)a.fold_H * a.fold_W : (long)a.OH * a.OW) * ld_t))
      *reinterpret_cast<u32x4*>(y_t + pix * ld_t + cof_t) = v;
    if (nb_on) {   // from the stored bf16 dz, as the unfused partial pass reads it
      const bf16x8 dz = __builtin_bit_cast(bf16x8, v);
      const bf16x8 xn = __builtin_bit_cast(bf16x8, nv);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float xv = (float)xn[q];
        const float xh = xv * rs[q] + c1[q];
        const float z = xv * zs[q] + zc[q];
        const float d = (float)dz[q] * (z > 0.f ? 1.f : nb_slope);
        s1[q] += d;
        s2[q] += d * xh;
        if (nb_p3) s3[q] += z <= 0.f ? (float)dz[q] * z : 0.f;
      }
    }
  };
  constexpr int IT = (BM * CPR) / NT;   // rows per thread
  constexpr int RSTEP = NT / CPR;
  // operand prefetch group: 2 rows in the small tiles (several blocks per CU: their registers
  // would cost occupancy), up to 8 in the 256-row tiles, which run one block per CU anyway
  // (their LDS ring) -- there each 2-row group was a serial HBM round trip per 256 x BN tile
  constexpr int PG = (BM >= 256 && IT % 8 == 0) ? 8 : ((BM >= 256 && IT % 4 == 0) ? 4 : 2);
  if constexpr (IT >= 2 && (BM * CPR) % NT == 0 && IT % 2 == 0) {
    if (co_t < a.Cout) {
      for (int g0 = 0; g0 < IT; g0 += PG) {
        long pixv[PG];
        u32x4 xv[PG], rv[PG], nv[PG];
#pragma unroll
        for (int u = 0; u < PG; ++u) {
          const int m = m0 + tid / CPR + (g0 + u) * RSTEP;
          pixv[u] = m < g.Mc ? out_pix(m) : -1;
          const bool ok = pixv[u] >= 0;
          xv[u] = (gate_t && ok) ? ld16(xb_t + pixv[u] * ld_t + cof_t) : z4;
          rv[u] = (res_t && ok) ? ld16(res_p + pixv[u] * ld_t + cof_t) : z4;
          nv[u] = (nb_x_on && ok) ? ld16(nbx_p + pixv[u] * a.nb_C + nb_co) : z4;
        }
#pragma unroll
        for (int u = 0; u < PG; ++u)
          if (pixv[u] != -1) finish(tid / CPR + (g0 + u) * RSTEP, pixv[u], xv[u], rv[u], nv[u]);
      }
    }
  } else {
    for (int c = tid; c < BM * CPR; c += NT) {
      const int row = c / CPR;
      const int m = m0 + row;
      if (m >= g.Mc || co_t >= a.Cout) continue;
      const long pix = out_pix(m);
      const bool ok = pix >= 0;
      finish(row, pix, (gate_t && ok) ? ld16(xb_t + pix * ld_t + cof_t) : z4,
             (res_t && ok) ? ld16(res_p + pix * ld_t + cof_t) : z4,
             (nb_x_on && ok) ? ld16(nbx_p + pix * a.nb_C + nb_co) : z4);
    }
  }
  if (a.nb_ws) {
    // per column: the NT / CPR threads sharing its chunk, summed in a fixed order -- first
    // across the lanes of a wave that share it (lane % CPR), then across the waves in LDS
    // (NT / 64 x CPR x 16 floats: fits in the staged tile it aliases)
#pragma unroll
    for (int off = CPR; off < 64; off <<= 1)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        s1[q] += __shfl_xor(s1[q], off);
        s2[q] += __shfl_xor(s2[q], off);
        if (nb_p3) s3[q] += __shfl_xor(s3[q], off);
      }
    __syncthreads();   // every thread is done with the staged tile
    float* red = reinterpret_cast<float*>(smem);
    const int lane = tid & 63, wid = tid >> 6;
    if (lane < CPR) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        red[(wid * CPR + lane) * 24 + q] = s1[q];
        red[(wid * CPR + lane) * 24 + 8 + q] = s2[q];
        red[(wid * CPR + lane) * 24 + 16 + q] = s3[q];
      }
    }
    __syncthreads();
    if (tid < BN) {
      const int cc = tid >> 3, q = tid & 7;
      const int co = n0 + tid - a.nb_c0;
      if (co >= 0 && co < a.nb_C) {
        float S1 = 0.f, S2 = 0.f, S3 = 0.f;
        for (int k = 0; k < NT / 64; ++k) {
          S1 += red[(k * CPR + cc) * 24 + q];
          S2 += red[(k * CPR + cc) * 24 + 8 + q];
          S3 += red[(k * CPR + cc) * 24 + 16 + q];
        }
        const int cls = g.ry * s + g.rx;
        long o, plane;
        if (a.nb_flat) {   // batch norm, tiles over all images (a fold's padded grid)
          o = ((long)cls * a.nb_tiles_cls + m0 / BM) * a.nb_C + co;
          plane = (long)a.nb_nchunks * a.nb_C;
        } else {
          const int img = m0 / HWq;
          const int chunk = cls * (HWq / BM) + (m0 - img * HWq) / BM;
          o = ((long)img * a.nb_nchunks + chunk) * a.nb_C + co;
          plane = (long)a.N * a.nb_nchunks * a.nb_C;
        }
        if (P2P_OOB_OK(3, o, 1, plane)) {
          a.nb_ws[o] = S1;
          a.nb_ws[plane + o] = S2;
          if (nb_p3) a.nb_ws[2 * plane + o] = S3;
        }
      }
    }
  }
}

// bias + output activation in registers -> the bf16 tile in LDS (row stride LDC): one wave's
// TM x TN fragment block at (row0, col0) of the tile.  The activation is dispatched ONCE per
// tile (compile-time body per code), not by a wave-uniform branch per accumulator element.
template <int TM, int TN, int LDC>
__device__ __forceinline__ void conv_stage_tile(const ConvFwdArgs& a, f32x4 (&acc)[TM][TN], bf16* Cs, int row0,
                                                int col0, int n0, int lane) {
  const float al = a.alpha ? a.alpha[0] : 1.f;
  auto stage = [&](auto act_tag) __attribute__((always_inline)) {
    constexpr int ACT = decltype(act_tag)::value;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int coll = col0 + j * 16 + (lane & 15);
      const int col = n0 + coll;
      const float bj = (a.bias && col < a.Cout) ? a.bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int rowb = row0 + i * 16 + (lane >> 4) * 4;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Cs[(rowb + r) * LDC + coll] = (bf16)act_fwd(acc[i][j][r] * al + bj, ACT);
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

// Everything after the staged bf16 tile (Cs, row stride BN + 8, visible to all NT threads):
// depth-to-space / statistics / the store loop with the act' gate, concat split, skip
// gradient, fp8 shadow (or the EXT loop with fused norm-backward partials).  red_stats:
// 2 * NT floats of scratch (d2s / stats); red_nb: NT * 16 floats that may alias Cs (EXT
// reuses it after a barrier).
template <int BM, int BN, int MODE, int NT, bool EXT = false>
__device__ __forceinline__ void conv_epilogue_tail(const ConvFwdArgs& a, const ClassGeom& g, int m0, int n0,
                                                   const bf16* Cs, float* red_stats, char* red_nb,
                                                   const FastDiv& fd_hwq, const FastDiv& fd_wq) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int HWq = g.Hq * g.Wq;
  const int s = a.stride;
  constexpr int LDC = BN + 8;
  // output pixel of GEMM row m; with a fold (conv.h fold_buf): the real-grid pixel of an
  // interior row, or -(padded pixel) - 2 for a frame row (-1 stays "no row")
  auto out_pix = [&](int m) __attribute__((always_inline)) -> long {
    if (MODE == 0 && !a.fold_buf) return m;
    const int n = (int)fdiv((uint32_t)m, fd_hwq);
    const int r = m - n * HWq;
    const int qy = (int)fdiv((uint32_t)r, fd_wq);
    const int qx = r - qy * g.Wq;
    const int oy = MODE == 0 ? qy : qy * s + g.ry, ox = MODE == 0 ? qx : qx * s + g.rx;
    if (a.fold_buf) {
      const int iy = oy - a.fold_p, ix = ox - a.fold_p;
      if ((unsigned)iy < (unsigned)a.fold_H && (unsigned)ix < (unsigned)a.fold_W)
        return ((long)n * a.fold_H + iy) * a.fold_W + ix;
      return -(((long)n * a.OH + oy) * a.OW + ox) - 2;
    }
    return ((long)n * a.OH + oy) * a.OW + ox;
  };

  if (a.d2s) {  // depth-to-space packed image (d1 forward / its head gradient)
    const int Ho = 2 * a.OH, Wo = 2 * a.OW;
    float l1 = 0.f;
    const float d2s_sc = a.d2s_scale * (a.d2s == 2 && a.d2s_w ? *a.d2s_w : 1.f);
    for (int it = tid; it < BM * 4; it += NT) {
      const int row = it >> 2, cls = it & 3;
      const int m = m0 + row;
      if (m >= g.Mc) continue;
      const int n = (int)fdiv((uint32_t)m, fd_hwq);
      const int r = m - n * HWq;
      const int qy = (int)fdiv((uint32_t)r, fd_wq);
      const int qx = r - qy * g.Wq;
      const long P = ((long)n * Ho + 2 * qy + (cls >> 1)) * Wo + 2 * qx + (cls & 1);
      l1 += d2s_pixel(a.d2s, P, Cs + row * LDC + cls * 4, static_cast<const bf16*>(a.pk_a),
                      static_cast<const bf16*>(a.pk_f), d2s_sc, static_cast<bf16*>(a.y1));
    }
    if (a.d2s == 1 && a.l1_part) {
      float* red = red_stats;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) l1 += __shfl_xor(l1, off);
      if (lane == 0) red[wid] = l1;
      __syncthreads();
      if (tid == 0) {
        float t = 0.f;
        for (int w = 0; w < NT / 64; ++w) t += red[w];
        a.l1_part[blockIdx.x] = t;
      }
    }
    return;
  }

  if (a.stats) {
    // per-column (mean, M2) of the tile's BM bf16 outputs, shifted by the tile's first row
    // (no E[x^2] - E[x]^2 cancellation); NT / BN threads per column, combined in LDS
    constexpr int TPC = NT / BN;
    static_assert(NT % BN == 0 && BM % TPC == 0, "stats partition");
    float* red = red_stats;
    const int col = tid % BN, part = tid / BN;
    const float piv = (float)Cs[col];
    float s1 = 0.f, s2 = 0.f;
    for (int r = part * (BM / TPC); r < (part + 1) * (BM / TPC); ++r) {
      const float d = (float)Cs[r * LDC + col] - piv;
      s1 += d;
      s2 += d * d;
    }
    red[tid] = s1;
    red[NT + tid] = s2;
    __syncthreads();
    const int co = n0 + col;
    if (part == 0 && co < a.Cout) {
      float S1 = 0.f, S2 = 0.f;
#pragma unroll
      for (int q = 0; q < TPC; ++q) {
        S1 += red[q * BN + col];
        S2 += red[NT + q * BN + col];
      }
      const float inv = 1.f / (float)BM;
      const int img = m0 / HWq;
      const int chunk = g.ry * s * (HWq / BM) + g.rx * (HWq / BM) + (m0 - img * HWq) / BM;
      const long o = ((long)img * a.stats_nchunks + chunk) * a.Cout + co;
      a.stats[o] = piv + S1 * inv;
      a.stats[(long)a.N * a.stats_nchunks * a.Cout + o] = fmaxf(S2 - S1 * S1 * inv, 0.f);
    }
  }

  if constexpr (!EXT) {
  constexpr int CPR = BN / 8;  // 8-channel chunks per row
  const Fp8Shadow qsh{static_cast<uint8_t*>(a.q_out), a.q_site, a.q_fmt};
  const float qsc = qsh.q ? fp8_shadow_scale(qsh) : 0.f;
  float qmax = 0.f;
  for (int c = tid; c < BM * CPR; c += NT) {
    const int row = c / CPR, cc = c - row * CPR;
    const int m = m0 + row;
    const int co = n0 + cc * 8;
    if (m >= g.Mc || co >= a.Cout) continue;
    const long pix = out_pix(m);
    u32x4 v = *reinterpret_cast<const u32x4*>(Cs + row * LDC + cc * 8);
    if (pix < 0) {   // fold frame pixel: raw, folded by fold_band (host: Csplit == Cout)
      if (P2P_OOB_OK(1, (-pix - 2) * a.Cout + co, 8, (long)a.N * a.OH * a.OW * a.Cout))
        *reinterpret_cast<u32x4*>(static_cast<bf16*>(a.fold_buf) + (-pix - 2) * a.Cout + co) = v;
      continue;
    }
    const bool first = co < a.Csplit;
    const int ld = first ? a.Csplit : a.Cout - a.Csplit;
    const int cof = first ? co : co - a.Csplit;
    const bf16* xb = static_cast<const bf16*>(first ? a.xb1 : a.xb2);
    if (a.act_bwd && xb) {   // a null half is gated by its producer's backward instead
      const u32x4 xv = *reinterpret_cast<const u32x4*>(xb + pix * ld + cof);
      if (a.act_bwd == ACT_RELU) {
        // zero the gradient where x <= 0 (bf16 sign / zero test on the int pipe)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t xw = xv[q];
          uint32_t keep = 0;
          if ((int16_t)(xw & 0xffffu) > 0) keep |= 0xffffu;
          if ((int16_t)(xw >> 16) > 0) keep |= 0xffff0000u;
          v[q] &= keep;
        }
      } else {
        bf16x8 vb = __builtin_bit_cast(bf16x8, v);
        const bf16x8 xb8 = __builtin_bit_cast(bf16x8, xv);
#pragma unroll
        for (int q = 0; q < 8; ++q)
          vb[q] = (bf16)((float)vb[q] * act_grad_from_input((float)xb8[q], a.act_bwd));
        v = __builtin_bit_cast(u32x4, vb);
      }
    }
    if (a.res1 && first) {   // host: res1 only with Csplit == Cout
      bf16x8 vb = __builtin_bit_cast(bf16x8, v);
      const bf16x8 rb = *reinterpret_cast<const bf16x8*>(static_cast<const bf16*>(a.res1) + pix * ld + cof);
#pragma unroll
      for (int q = 0; q < 8; ++q) vb[q] = (bf16)((float)vb[q] + (float)rb[q]);
      v = __builtin_bit_cast(u32x4, vb);
    }
    bf16* y = static_cast<bf16*>(first ? a.y1 : a.y2);
    if (P2P_OOB_OK(2, pix * ld + cof, 8,
                   (long)a.N * (a.fold_buf ? (long)a.fold_H * a.fold_W : (long)a.OH * a.OW) * ld))
      *reinterpret_cast<u32x4*>(y + pix * ld + cof) = v;
    if (qsh.q) {  // host: only with Csplit == Cout, no act_bwd
      const bf16x8 vb = __builtin_bit_cast(bf16x8, v);
      float r[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        r[q] = (float)vb[q];
        qmax = fmaxf(qmax, fabsf(r[q]));
      }
      *reinterpret_cast<uint2*>(qsh.q + pix * ld + cof) = fp8_pack8(r, qsc, qsh.fmt);
    }
  }
  if (qsh.q) fp8_amax_commit(qmax, qsh.site);
  } else {
    conv_epilogue_ext<BM, BN, MODE, NT>(a, g, m0, n0, red_nb, Cs, LDC, HWq, s, out_pix);
  }
}

// bias + output activation in registers, the bf16 tile staged through LDS, 16-B stores
// with the optional act'(x) multiply (dgrad) and the concat channel split; split-K tiles
// accumulate fp32 atomics instead.
// EXT (dgrad kernels with an act' gate, a parked skip gradient or fused norm-backward partials):
// the store loop prefetches those operands two rows at a time and accumulates the partials.  A
// separate instantiation: its registers would halve the occupancy of the plain store loop.
template <int BM, int BN, int WM, int WN, int MODE, int NT, bool EXT = false>
__device__ __forceinline__ void conv_epilogue(const ConvFwdArgs& a, const ClassGeom& g,
                                              f32x4 (&acc)[BM / WM / 16][BN / WN / 16], int m0,
                                              int n0, char* smem, const FastDiv& fd_hwq,
                                              const FastDiv& fd_wq) {
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int HWq = g.Hq * g.Wq;
  const int s = a.stride;
  auto out_pix = [&](int m) __attribute__((always_inline)) -> long {
    if (MODE == 0) return m;
    const int n = (int)fdiv((uint32_t)m, fd_hwq);
    const int r = m - n * HWq;
    const int qy = (int)fdiv((uint32_t)r, fd_wq);
    const int qx = r - qy * g.Wq;
    return ((long)n * a.OH + qy * s + g.ry) * a.OW + qx * s + g.rx;
  };

  // ---- split-K: fp32 atomics straight from the accumulators (tiny-M layers only).  Not
  // compiled into the big tiles (the host never splits them): its out_pix division loop
  // is not unrolled there, which made the compiler keep the accumulators in scratch.
  if constexpr (TM * TN <= 16) if (a.splits > 1) {
    float* wsb = a.det ? a.ws + (long)(blockIdx.z % a.splits) * a.N * a.OH * a.OW * a.Cout : a.ws;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn * TN * 16 + j * 16 + (lane & 15);
        const int rowb = m0 + wm * TM * 16 + i * 16 + (lane >> 4) * 4;
        if (col >= a.Cout) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = rowb + r;
          if (m < g.Mc) {
            if (a.det) wsb[out_pix(m) * a.Cout + col] = acc[i][j][r];
            else atomicAdd(a.ws + out_pix(m) * a.Cout + col, acc[i][j][r]);
          }
        }
      }
    return;
  }

  // ---- epilogue: bias + act in registers, bf16 tile staged in LDS, 16-B stores
  bf16* Cs = reinterpret_cast<bf16*>(smem);
  constexpr int LDC = BN + 8;
  conv_stage_tile<TM, TN, LDC>(a, acc, Cs, wm * TM * 16, wn * TN * 16, n0, lane);
  __syncthreads();
  conv_epilogue_tail<BM, BN, MODE, NT, EXT>(a, g, m0, n0, Cs, reinterpret_cast<float*>(smem + BM * LDC * 2), smem,
                                            fd_hwq, fd_wq);
}

}  // namespace p2p
