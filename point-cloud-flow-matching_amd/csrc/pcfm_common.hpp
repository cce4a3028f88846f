// Shared helpers for the gfx950 kernels behind include/pcfm.h.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstddef>
#include <cstdint>
#include <cstdio>

#include "../../include/pcfm.h"

namespace pcfm {

// Thread-local last-error text (pcfm_last_error).
void set_error(const char* fmt, ...);

// Host-side argument check: returns PCFM_EINVAL with a message when !cond.
#define PCFM_CHECK_ARG(cond, ...)            \
  do {                                       \
    if (!(cond)) {                           \
      ::pcfm::set_error(__VA_ARGS__);        \
      return PCFM_EINVAL;                    \
    }                                        \
  } while (0)

// After a group of launches: map the sticky launch error to a return code.
int check_launch(const char* what);

// Every 64-bit index computation goes through size_t; kernels take int sizes
// that fit the reference's own int arithmetic.
inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

constexpr int kCUs = 256;           // MI355X: 8 XCDs x 32 CUs
constexpr int kLdsBytesMax = 160 * 1024;

// Raise the dynamic-LDS cap of one kernel to the gfx950 maximum once.
int allow_big_lds(const void* kernel);

// Whole-CU residency for a kernel whose block puts W waves on each SIMD: naming
// register v(512 / W - 1) in a clobber makes the kernel descriptor allocate
// 512 / W VGPRs per lane (granule 8), so the block's waves take every register
// of the CU's four SIMDs and no wave of another kernel (any kernel that needs
// more than 8 VGPRs) can be resident on the CU beside them.  Used by the
// LDS-DMA weight gradient ("co-residence").
#define PCFM_CLAIM_VGPRS(last) asm volatile("" ::: "v" #last)

// Split operands (bf16 hi / lo of an fp32 tensor, channels-last rows of C
// channels, C % 32 == 0) are stored interleaved per 32-channel group: row r
// holds [hi c0..c31 | lo c0..c31 | hi c32..c63 | lo c32..c63 | ...], so the
// hi and lo halves of one K-step of 32 channels share one 128-byte line (a
// step fetches whole lines, not halves of lines it reads the rest of 27 steps
// later).  Element offset of (row, channel c) in hi; its lo is 32 further.
__host__ __device__ inline size_t split_off(size_t row, int c, int C) {
  return row * 2 * (size_t)C + (size_t)(((c >> 5) << 6) + (c & 31));
}
constexpr int kSplitLo = 32;  // element offset of lo from hi

// Squared distance contract shared by every nearest-neighbour kernel and the
// oracle: dx = q - p;  d = fma(dz, dz, fma(dx, dx, dy*dy)).
// (This is how NVVM contracts the reference's `x*x + y*y + z*z`; pinned here
// explicitly so the order does not depend on the compiler.)
__device__ __forceinline__ float sqdist3(float dx, float dy, float dz) {
  return __builtin_fmaf(dz, dz, __builtin_fmaf(dx, dx, dy * dy));
}
__device__ __forceinline__ double sqdist3(double dx, double dy, double dz) {
  return __builtin_fma(dz, dz, __builtin_fma(dx, dx, dy * dy));
}

// Block index walked in reverse (a second pass over data a first pass just
// read in forward order finds its most recent rows in the Infinity Cache).
#ifndef PCFM_REV_APPLY
#define PCFM_REV_APPLY 1
#endif
__device__ __forceinline__ unsigned rev_order(unsigned i, unsigned n) {
  return PCFM_REV_APPLY ? n - 1 - i : i;
}

// Streamed (non-temporal) global accesses for outputs next read by another
// kernel and inputs read once; PCFM_NT=0 builds them as plain accesses
// (measurement / diagnosis switch).
#ifndef PCFM_NT
#define PCFM_NT 1
#endif
template <class T>
__device__ __forceinline__ void nt_st(T v, T* p) {
#if PCFM_NT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
template <class T>
__device__ __forceinline__ T nt_ld(const T* p) {
#if defined(PCFM_COHERENT_LD) && PCFM_COHERENT_LD
  // diagnosis switch: device-coherent (agent-scope) load, no stale cache line
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#elif PCFM_NT
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}

}  // namespace pcfm
