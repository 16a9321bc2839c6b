// index.hip — the interval index (replaces build_interval_trees, cluster.py:124-130, and the
// superintervals IntervalMap it builds per chromosome).
//
// 1. radix sort of (chrom << 32 | start) with the CSR interval id as value
// 2. scatter: per sorted position q the record {start, end, thr, read<<6|j}, a copy of the read's
//    rmeta record (so the pair gate needs no dependent gather), start; chromosome ranges
// 3. inclusive max-scan of (chrom << 32 | end): per-chromosome prefix max of end (pmax)
// 4. scan ranges per interval (binary searches inside its chromosome):
//      n_fwd     = #{p > q : start_p <= end_q}        (all overlap: start_q <= start_p <= end_q)
//      bwd_begin = first p with pmax_p >= start_q     (p < q with pmax < start_q cannot overlap)
//    so a query interval's end-inclusive overlaps (superintervals search_values semantics,
//    SURVEY.md §8a A6) are exactly: q+1 .. q+n_fwd, plus p in [bwd_begin, q) with end_p >= start_q.
#include <hipcub/hipcub.hpp>

#include "kernels.hpp"

namespace fslr {
namespace {

__global__ void k_fill_iv_read(const int4* __restrict__ rmeta, int n, int* __restrict__ iv_read) {
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
    const int4 m = rmeta[r];
    const int len = m.y & 0xffff;
    for (int k = 0; k < len; ++k) iv_read[m.x + k] = r;
  }
}

__global__ void k_make_keys(const int4* __restrict__ iv, int ni, unsigned long long* __restrict__ keys,
                            int* __restrict__ vals) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ni; k += gridDim.x * blockDim.x) {
    const int4 r = iv[k];
    keys[k] = (static_cast<unsigned long long>(r.x) << 32) | static_cast<unsigned>(r.y);
    vals[k] = k;
  }
}

__global__ void k_scatter(const unsigned long long* __restrict__ skeys, const int* __restrict__ svals,
                          const int4* __restrict__ iv, const int* __restrict__ iv_read,
                          const int4* __restrict__ rmeta, int ni, int4* __restrict__ idx4,
                          int4* __restrict__ idx_meta, int* __restrict__ s_start,
                          unsigned long long* __restrict__ endkey, int2* __restrict__ crange) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < ni; q += gridDim.x * blockDim.x) {
    const int k = svals[q];
    const int r = iv_read[k];
    const int4 m = rmeta[r];
    const int j = k - m.x;
    const int4 rec = iv[k];
    idx4[q] = make_int4(rec.y, rec.z, rec.w, (r << 6) | j);
    idx_meta[q] = m;
    s_start[q] = rec.y;
    endkey[q] = (static_cast<unsigned long long>(rec.x) << 32) | static_cast<unsigned>(rec.z);
    const int c = rec.x;
    if (q == 0 || static_cast<int>(skeys[q - 1] >> 32) != c) crange[c].x = q;
    if (q == ni - 1 || static_cast<int>(skeys[q + 1] >> 32) != c) crange[c].y = q + 1;
  }
}

struct MaxU64 {
  __device__ __forceinline__ unsigned long long operator()(unsigned long long a, unsigned long long b) const {
    return a > b ? a : b;
  }
};

__global__ void k_ranges(const unsigned long long* __restrict__ skeys, const int* __restrict__ svals,
                         const int* __restrict__ s_start, const int4* __restrict__ idx4,
                         const unsigned long long* __restrict__ pmaxkey, const int2* __restrict__ crange, int ni,
                         int4* __restrict__ iv_rng) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < ni; q += gridDim.x * blockDim.x) {
    const int c = static_cast<int>(skeys[q] >> 32);
    const int2 cr = crange[c];
    const int s = s_start[q], e = idx4[q].y;
    // forward: first p in (q, cr.y) with start_p > e
    int lo = q + 1, hi = cr.y;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s_start[mid] <= e) lo = mid + 1; else hi = mid;
    }
    const int n_fwd = lo - q - 1;
    // backward: first p in [cr.x, q) with pmax_p >= s (pmax is non-decreasing within the chromosome)
    lo = cr.x;
    hi = q;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (static_cast<int>(static_cast<unsigned>(pmaxkey[mid])) >= s) hi = mid; else lo = mid + 1;
    }
    iv_rng[svals[q]] = make_int4(q, n_fwd, lo, q - lo);
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
  size_t b1 = 0, b2 = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, b1, static_cast<unsigned long long*>(nullptr),
                                                    static_cast<unsigned long long*>(nullptr),
                                                    static_cast<int*>(nullptr), static_cast<int*>(nullptr), ni, 0,
                                                    64, s);
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::InclusiveScan(nullptr, b2, static_cast<unsigned long long*>(nullptr),
                                        static_cast<unsigned long long*>(nullptr), MaxU64(), ni, s);
  if (e != hipSuccess) return e;
  *bytes = b1 > b2 ? b1 : b2;
  return hipSuccess;
}

hipError_t launch_build_index(const IndexBufs& b, int n, int ni, int n_chroms, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(b.crange, 0, n_chroms * sizeof(int2), s);
  if (e != hipSuccess) return e;
  k_fill_iv_read<<<grid_for(n), 256, 0, s>>>(b.rmeta, n, b.iv_read);
  k_make_keys<<<grid_for(ni), 256, 0, s>>>(b.iv, ni, b.keys, b.vals);
  size_t tb = b.temp_bytes;
  e = hipcub::DeviceRadixSort::SortPairs(b.temp, tb, b.keys, b.keys2, b.vals, b.vals2, ni, 0,
                                         32 + bits_for(n_chroms), s);
  if (e != hipSuccess) return e;
  k_scatter<<<grid_for(ni), 256, 0, s>>>(b.keys2, b.vals2, b.iv, b.iv_read, b.rmeta, ni, b.idx4, b.idx_meta,
                                         b.s_start, b.endkey, b.crange);
  tb = b.temp_bytes;
  e = hipcub::DeviceScan::InclusiveScan(b.temp, tb, b.endkey, b.pmaxkey, MaxU64(), ni, s);
  if (e != hipSuccess) return e;
  k_ranges<<<grid_for(ni), 256, 0, s>>>(b.keys2, b.vals2, b.s_start, b.idx4, b.pmaxkey, b.crange, ni,
                                        b.iv_rng);
  return hipGetLastError();
}

hipError_t launch_set_thr(const int* thr, int4* iv, const int4* iv_rng, int4* idx4, int ni, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  k_set_thr<<<grid_for(ni), 256, 0, s>>>(thr, iv, iv_rng, idx4, ni);
  return hipGetLastError();
}

}  // namespace fslr
