// Device-side index checks for the P2P_BOUNDS_ASSERT diagnostic build.
//
// `P2P_OOB_OK(site, first, count, limit)` is true when the element range
// [first, first + count) lies inside [0, limit). In the normal build it is the constant true
// and compiles away. In the diagnostic build (tools/build_ext.py --define P2P_BOUNDS_ASSERT
// --out ...), a failed check does three things:
//   * bumps a per-translation-unit device counter (vector atomics on a global word);
//   * records the site id and the offending index;
//   * makes the caller SKIP the access.
// A bad index therefore shows up as a count, not as a memory fault or a trap: a trap or
// fault can take the whole GPU host down, a skipped store cannot.
// `torch.ops.p2p.oob_counts()` sums every unit's counters on the host and resets them.
// tests/conftest.py checks that sum after every GPU test when P2P_BOUNDS_CHECK=1.
//
// Site ids:
//   1     fold epilogue frame store (conv_dev.h, both tails)
//   2     epilogue y store (conv_dev.h)
//   10-12 pad_fold / pad_fold_s1 / fold_band stores
//   13    fold_band frame loads
//   20    wgrad_reduce_t store
//   30    s2t register-epilogue stores
//   31    s2t register-epilogue gate / operand loads
#pragma once

#include <hip/hip_runtime.h>

#ifdef P2P_BOUNDS_ASSERT

namespace p2p {

// host registry of the per-unit readers (defined once, csrc/misc.hip)
typedef void (*OobReader)(unsigned int* out4, bool reset);
int oob_register(OobReader fn);

namespace {

// [0] failed checks, [1] largest site id seen, [2] low 32 bits of the last bad index,
// [3] its limit's low 32 bits
__device__ unsigned int g_oob[4];

__device__ __forceinline__ bool oob_ok(int site, long first, long count, long limit) {
  if (first >= 0 && first + count <= limit) return true;
  atomicAdd(&g_oob[0], 1u);
  atomicMax(&g_oob[1], (unsigned int)site);
  atomicExch(&g_oob[2], (unsigned int)first);
  atomicExch(&g_oob[3], (unsigned int)limit);
  return false;
}

void oob_read_unit(unsigned int* out4, bool reset) {
  unsigned int v[4] = {0, 0, 0, 0};
  (void)hipMemcpyFromSymbol(v, HIP_SYMBOL(g_oob), sizeof(v), 0, hipMemcpyDeviceToHost);
  out4[0] += v[0];
  if (v[1] > out4[1]) out4[1] = v[1];
  if (v[0]) {
    out4[2] = v[2];
    out4[3] = v[3];
  }
  if (reset) {
    const unsigned int z[4] = {0, 0, 0, 0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_oob), z, sizeof(z), 0, hipMemcpyHostToDevice);
  }
}

const int g_oob_registered = oob_register(&oob_read_unit);

}  // namespace
}  // namespace p2p

#define P2P_OOB_OK(site, first, count, limit) (::p2p::oob_ok((site), (long)(first), (long)(count), (long)(limit)))

#else

#define P2P_OOB_OK(site, first, count, limit) (true)

#endif
