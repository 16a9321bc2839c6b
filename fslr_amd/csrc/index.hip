// index.hip — the interval index (replaces build_interval_trees, cluster.py:124-130, and the
// superintervals IntervalMap it builds per chromosome).
//
// 1. keys: one thread per read writes, for each of its intervals, the sort key and the tag
//    read << 6 | j.  With the start-sorted `data` order given (cluster.py:114), the key is the
//    chromosome and the entries are placed at their data position: a single stable radix pass
//    then yields (chrom, start) order.  Without it, the key is (chrom << 32 | start).
// 2. scatter: per sorted position q the record {start, end, thr, tag} and the read's packed gate
//    fields {qlen2, nal | LB << 24 | haz << 31} (the pair gate reads them beside the hit)
// 3. inclusive max-scan of (chrom << 32 | end): per-chromosome prefix max of end (pmax)
// 4. scan ranges per interval, by galloping from q inside its chromosome:
//      n_fwd     = #{p > q : start_p <= end_q}        (all overlap: start_q <= start_p <= end_q)
//      bwd_begin = first p with pmax_p >= start_q     (p < q with pmax < start_q cannot overlap)
//    so a query interval's end-inclusive overlaps (superintervals search_values semantics,
//    SURVEY.md §8a A6) are exactly: q+1 .. q+n_fwd, plus p in [bwd_begin, q) with end_p >= start_q.
#include <hipcub/hipcub.hpp>

#include "kernels.hpp"

namespace fslr {
namespace {

template <bool kByData>
__global__ void k_keys(const int4* __restrict__ rmeta, const int4* __restrict__ iv, const int* __restrict__ data_pos,
                       int n, unsigned long long* __restrict__ keys64, unsigned* __restrict__ keys32,
                       int* __restrict__ vals) {
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
    const int4 m = rmeta[r];
    const int len = m.y & 0xffff;
    for (int j = 0; j < len; ++j) {
      const int k = m.x + j;
      const int4 rec = iv[k];
      if (kByData) {
        const int d = data_pos[k];
        keys32[d] = static_cast<unsigned>(rec.x);
        vals[d] = (r << 6) | j;
      } else {
        keys64[k] = (static_cast<unsigned long long>(rec.x) << 32) | static_cast<unsigned>(rec.y);
        vals[k] = (r << 6) | j;
      }
    }
  }
}

__global__ void k_scatter(const int* __restrict__ stags, const int4* __restrict__ iv,
                          const int4* __restrict__ rmeta, int ni, int4* __restrict__ idx4,
                          int2* __restrict__ idx_gate, int* __restrict__ s_start,
                          unsigned long long* __restrict__ endkey) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < ni; q += gridDim.x * blockDim.x) {
    const int rj = stags[q];
    const int4 m = rmeta[rj >> 6];
    const int4 rec = iv[m.x + (rj & 63)];
    idx4[q] = make_int4(rec.y, rec.z, rec.w, rj);
    // {qlen2, nal | LB << 24 | haz << 31}
    idx_gate[q] = make_int2(m.z, (m.w & 0xFFFFFF) | ((m.y & 0x7F) << 24) | (((m.y >> 16) & 1) << 31));
    s_start[q] = rec.y;
    endkey[q] = (static_cast<unsigned long long>(rec.x) << 32) | static_cast<unsigned>(rec.z);
  }
}

struct MaxU64 {
  __device__ __forceinline__ unsigned long long operator()(unsigned long long a, unsigned long long b) const {
    return a > b ? a : b;
  }
};

__global__ void k_ranges(const int* __restrict__ stags, const int4* __restrict__ rmeta,
                         const int* __restrict__ s_start, const unsigned long long* __restrict__ endkey,
                         const unsigned long long* __restrict__ pmaxkey, const int2* __restrict__ crange, int ni,
                         int4* __restrict__ iv_rng) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < ni; q += gridDim.x * blockDim.x) {
    const unsigned long long ek = endkey[q];
    const int2 cr = crange[static_cast<int>(ek >> 32)];
    const int s = s_start[q], e = static_cast<int>(static_cast<unsigned>(ek));
    // forward: first p in (q, cr.y) with start_p > e — gallop, then bisect
    int lo = q + 1, step = 1, hi = q + 1;
    while (hi < cr.y && s_start[hi] <= e) {
      lo = hi + 1;
      hi = q + 1 + step;
      step <<= 1;
    }
    if (hi > cr.y) hi = cr.y;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s_start[mid] <= e) lo = mid + 1; else hi = mid;
    }
    const int n_fwd = lo - q - 1;
    // backward: first p in [cr.x, q) with pmax_p >= s (pmax non-decreasing within the chromosome)
    hi = q;
    lo = q - 1;
    step = 1;
    while (lo >= cr.x && static_cast<int>(static_cast<unsigned>(pmaxkey[lo])) >= s) {
      hi = lo;
      lo = q - 1 - step;
      step <<= 1;
    }
    if (lo < cr.x) lo = cr.x; else lo = lo + 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (static_cast<int>(static_cast<unsigned>(pmaxkey[mid])) >= s) hi = mid; else lo = mid + 1;
    }
    const int rj = stags[q];
    iv_rng[rmeta[rj >> 6].x + (rj & 63)] = make_int4(q, n_fwd, lo, q - lo);
  }
}

__global__ void k_set_thr(const int* __restrict__ thr, int4* __restrict__ iv, const int4* __restrict__ iv_rng,
                          int4* __restrict__ idx4, int ni) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ni; k += gridDim.x * blockDim.x) {
    iv[k].w = thr[k];
    if (idx4) idx4[iv_rng[k].x].z = thr[k];
  }
}

int bits_for(int v) {
  int b = 1;
  while ((1 << b) <= v) ++b;
  return b;
}

}  // namespace

hipError_t index_temp_bytes(int ni, size_t* bytes, hipStream_t s) {
  size_t b1 = 0, b2 = 0, b3 = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, b1, static_cast<unsigned long long*>(nullptr),
                                                    static_cast<unsigned long long*>(nullptr),
                                                    static_cast<int*>(nullptr), static_cast<int*>(nullptr), ni, 0,
                                                    64, s);
  if (e != hipSuccess) return e;
  e = hipcub::DeviceRadixSort::SortPairs(nullptr, b3, static_cast<unsigned*>(nullptr),
                                         static_cast<unsigned*>(nullptr), static_cast<int*>(nullptr),
                                         static_cast<int*>(nullptr), ni, 0, 32, s);
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::InclusiveScan(nullptr, b2, static_cast<unsigned long long*>(nullptr),
                                        static_cast<unsigned long long*>(nullptr), MaxU64(), ni, s);
  if (e != hipSuccess) return e;
  *bytes = b1 > b2 ? b1 : b2;
  if (b3 > *bytes) *bytes = b3;
  return hipSuccess;
}

hipError_t launch_build_index(const IndexBufs& b, int n, int ni, int n_chroms, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  hipError_t e;
  size_t tb = b.temp_bytes;
  if (b.data_pos) {
    unsigned* k32 = reinterpret_cast<unsigned*>(b.keys);
    unsigned* k32b = reinterpret_cast<unsigned*>(b.keys2);
    k_keys<true><<<grid_for(n), 256, 0, s>>>(b.rmeta, b.iv, b.data_pos, n, nullptr, k32, b.vals);
    e = hipcub::DeviceRadixSort::SortPairs(b.temp, tb, k32, k32b, b.vals, b.vals2, ni, 0, bits_for(n_chroms), s);
  } else {
    k_keys<false><<<grid_for(n), 256, 0, s>>>(b.rmeta, b.iv, nullptr, n, b.keys, nullptr, b.vals);
    e = hipcub::DeviceRadixSort::SortPairs(b.temp, tb, b.keys, b.keys2, b.vals, b.vals2, ni, 0,
                                           32 + bits_for(n_chroms), s);
  }
  if (e != hipSuccess) return e;
  k_scatter<<<grid_for(ni), 256, 0, s>>>(b.vals2, b.iv, b.rmeta, ni, b.idx4, b.idx_gate, b.s_start, b.endkey);
  tb = b.temp_bytes;
  e = hipcub::DeviceScan::InclusiveScan(b.temp, tb, b.endkey, b.pmaxkey, MaxU64(), ni, s);
  if (e != hipSuccess) return e;
  k_ranges<<<grid_for(ni), 256, 0, s>>>(b.vals2, b.rmeta, b.s_start, b.endkey, b.pmaxkey, b.crange, ni, b.iv_rng);
  return hipGetLastError();
}

hipError_t launch_set_thr(const int* thr, int4* iv, const int4* iv_rng, int4* idx4, int ni, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  k_set_thr<<<grid_for(ni), 256, 0, s>>>(thr, iv, iv_rng, idx4, ni);
  return hipGetLastError();
}

}  // namespace fslr
