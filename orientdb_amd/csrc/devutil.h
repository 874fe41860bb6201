// devutil.h — device helpers shared by the gfx950 kernel files (kernels.hip, bfs.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "common.h"
#include "devtypes.h"
#include "kernels.h"

namespace omx {

// OMX_SYNC_LAUNCH=1: synchronise after every launch so an asynchronous fault names its kernel
bool sync_launches();
#define KCHECK(name)                                                                                    \
  do {                                                                                                  \
    hipError_t e_ = hipGetLastError();                                                                  \
    if (e_ == hipSuccess && sync_launches()) e_ = hipStreamSynchronize(s);                              \
    if (e_ != hipSuccess) fail(OMX_E_DEVICE, std::string("launch of ") + name + ": " + hipGetErrorString(e_)); \
  } while (0)

static inline unsigned nblocks(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

__device__ __forceinline__ bool bm_test(const uint64_t *bm, uint32_t v) { return (bm[v >> 6] >> (v & 63)) & 1ull; }

__device__ __forceinline__ uint32_t lane_prefix(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// wave-uniform copy of a 64-bit value (lane 0's); the compiler can then keep it in SGPRs
__device__ __forceinline__ uint64_t wave_bcast64(uint64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x), hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t adj_degree(const DAdj &a, uint32_t v) {
  uint64_t d = 0;
  for (int p = 0; p < a.n; ++p) d += a.p[p].rp[v + 1] - a.p[p].rp[v];
  return d;
}

// publish a host mailbox (kernels.h Mail): the payload stores become visible before the sequence word
__device__ __forceinline__ void mail_post(const Mail &m) {
  __threadfence_system();
  __hip_atomic_store(m.p + kMailSeq, m.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// block-wide exclusive scan of one u32 per thread (4 waves); returns the block total in *total
template <int B>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t *s_w, uint32_t *total) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    uint32_t y = __shfl_up(incl, off, 64);
    if (lane >= (uint32_t)off) incl += y;
  }
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  uint32_t woff = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < B / 64; ++w) {
    uint32_t t = s_w[w];
    woff += (w < (int)wave) ? t : 0;
    tot += t;
  }
  *total = tot;
  return woff + incl - x;
}

}  // namespace omx
