// wave.hpp — wave64 building blocks shared by the pair engines (query.hip: read walk, sweep.hip:
// position sweep): lane masks, DPP scans, scalar-cache loads, the length gate as integer ranges,
// and the LDS-staged edge output.
#pragma once
#include <hip/hip_runtime.h>

#include "fslr_hip.h"
#include "kernels.hpp"

namespace fslr {

__device__ __forceinline__ int lane_id() { return static_cast<int>(__lane_id()); }

__device__ __forceinline__ int mbcnt(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(m >> 32),
                                   __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(m), 0u));
}

// wave-uniform loads through the scalar cache (constant address space => s_load)
typedef const __attribute__((address_space(4))) int* const_i32_ptr;
__device__ __forceinline__ int2 sload2(const void* p, int i) {
  const_i32_ptr q = (const_i32_ptr)(p) + 2 * i;
  return make_int2(q[0], q[1]);
}
__device__ __forceinline__ int4 sload4(const void* p, int i) {
  const_i32_ptr q = (const_i32_ptr)(p) + 4 * i;
  return make_int4(q[0], q[1], q[2], q[3]);
}

// three consecutive dwords of a 16-B record, starting at dword `first`
__device__ __forceinline__ int3 load3(const int4* p, int k, int first) {
  const int* q = reinterpret_cast<const int*>(p + k) + first;
  return make_int3(q[0], q[1], q[2]);
}

// inclusive wave64 prefix sum on DPP: row_shr 1/2/4/8 inside each row of 16 lanes, then
// row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) — six VALU ops, no LDS round trips
__device__ __forceinline__ int wave_incl_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
  return x;
}

__device__ __forceinline__ int rdl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The gate of one read as integer ranges (exact: IEEE division is monotone, so the reference's
// double test fl(min/max) >= cut, cluster.py:178-183, holds on a contiguous range of the
// partner's value).  {lo, hi}: partner values x in [lo, hi] pass; lo < 0 marks v == 0, where
// x == 0 raises ZeroDivisionError and the passing range is [1, hi].
__device__ inline int2 ratio_range(int v, double cut) {
  constexpr int kTop = 0x7FFFFFFF;
  if (v == 0) return make_int2(-1, 0.0 >= cut ? kTop : 0);
  if (!(1.0 >= cut)) return make_int2(1, 0);
  const double dv = static_cast<double>(v);
  if (!(cut > 0.0)) return make_int2(0, kTop);      // every ratio >= 0 >= cut
  // smallest x <= v with fl(x / v) >= cut: start at the estimate, then walk with the exact test
  // (monotone, so the walks end at the true bound whatever the estimate; here they take 1-2 steps)
  int lo = static_cast<int>(fmin(fmax(ceil(cut * dv), 0.0), dv));
  while (lo > 0 && static_cast<double>(lo - 1) / dv >= cut) --lo;
  while (!(static_cast<double>(lo) / dv >= cut)) ++lo;
  // largest x >= v with fl(v / x) >= cut
  int hi = static_cast<int>(fmin(fmax(floor(dv / cut), dv), static_cast<double>(kTop)));
  while (hi < kTop && dv / static_cast<double>(hi + 1) >= cut) ++hi;
  while (!(dv / static_cast<double>(hi) >= cut)) --hi;
  return make_int2(lo, hi);
}

// a pair (a, b) whose evaluation raises ZeroDivisionError: listed in the error words (kernels.hpp
// kErrZdCount); the reference raises only if a loop reaches it, which the edge cap decides
__device__ __forceinline__ void raise_zd(int* err, bool zd, int a, int b) {
  if (zd) {
    const int k = atomicAdd(&err[kErrZdCount], 1);
    if (k < err[kErrZdCap]) reinterpret_cast<int2*>(err + kErrZdList)[k] = make_int2(a, b);
  }
}

constexpr unsigned kRankMask = 0x1FFFFFFu;     // read ranks < FSLR_MAX_READS = 2^25

// Wave-level edge staging in LDS (64-edge flushes, one global atomic each).  ES holds
// a << 39 | b << 14 | I << 7 | U.
struct EdgeOut {
  int2* edges;
  unsigned short* edge_iu;
  long long cap;
  unsigned long long* count;          // the global edge counter (own cache line)
  int* parent = nullptr;              // EdgeStageN: each flushed edge (a, b) also takes parent[b] down to a
                                      // (the union-find's pre-hook, SweepArgs::parent)
};

struct EdgeStage {
  unsigned long long* ES;
  int n;
  __device__ void flush(const EdgeOut& o, int nb, int lane) {
    wave_lds_sync();
    const bool act = lane < nb;
    const unsigned long long e = act ? ES[lane] : 0ull;
    const int rem = n - nb;
    const unsigned long long mv = lane < rem ? ES[nb + lane] : 0ull;
    wave_lds_sync();
    if (lane < rem) ES[lane] = mv;
    n = rem;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(o.count, static_cast<unsigned long long>(nb));
    base = __shfl(base, 0);
    const long long k = static_cast<long long>(base) + lane;
    if (act && k < o.cap) {
      o.edges[k] = make_int2(static_cast<int>(e >> 39), static_cast<int>((e >> 14) & kRankMask));
      o.edge_iu[k] = static_cast<unsigned short>(((e >> 7) & 127u) | ((e & 127u) << 8));
    }
  }
  // stage the lanes' edges (at most kWave staged between flushes); returns the number staged
  __device__ int put(const EdgeOut& o, bool edge, int a, int B, int I, int U, int lane) {
    const unsigned long long em = __ballot(edge);
    const int ne = __popcll(em);
    if (ne) {
      if (n + ne > kWave) flush(o, n, lane);
      if (edge)
        ES[n + mbcnt(em)] = (static_cast<unsigned long long>(a) << 39) | (static_cast<unsigned long long>(B) << 14) |
                            (static_cast<unsigned long long>(I) << 7) | static_cast<unsigned long long>(U);
      n += ne;
    }
    return ne;
  }
};

// Edge staging for kCap edges per wave (a multiple of 64): fewer flushes, so fewer contended
// atomics on the one edge counter (it saturates near 90 returning atomics per microsecond).
template <int kCap>
struct EdgeStageN {
  unsigned long long* ES;
  int n;
  __device__ void flush(const EdgeOut& o, int lane) {
    wave_lds_sync();
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(o.count, static_cast<unsigned long long>(n));
    base = __shfl(base, 0);
    for (int t = lane; t < n; t += kWave) {
      const unsigned long long e = ES[t];
      const long long k = static_cast<long long>(base) + t;
      if (k < o.cap) {
        o.edges[k] = make_int2(static_cast<int>(e >> 39), static_cast<int>((e >> 14) & kRankMask));
        o.edge_iu[k] = static_cast<unsigned short>(((e >> 7) & 127u) | ((e & 127u) << 8));
      }
      // the pre-hook here, batched with the flush's stores, rather than one atomic per edge as it is formed
      // (every later load of the wave waits behind its atomics: once per flush instead of once per group)
      if (o.parent) atomicMin(o.parent + ((e >> 14) & kRankMask), static_cast<int>(e >> 39));
    }
    wave_lds_sync();
    n = 0;
  }
  __device__ int put(const EdgeOut& o, bool edge, int a, int B, int I, int U, int lane) {
    const unsigned long long em = __ballot(edge);
    const int ne = __popcll(em);
    if (ne) {
      if (n + ne > kCap) flush(o, lane);
      if (edge)
        ES[n + mbcnt(em)] = (static_cast<unsigned long long>(a) << 39) | (static_cast<unsigned long long>(B) << 14) |
                            (static_cast<unsigned long long>(I) << 7) | static_cast<unsigned long long>(U);
      n += ne;
    }
    return ne;
  }
};

}  // namespace fslr
