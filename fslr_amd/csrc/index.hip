// index.hip — the interval index (replaces build_interval_trees, cluster.py:124-130, and the
// superintervals IntervalMap it builds per chromosome).
//
// Fast path (the start-sorted `data` list of cluster.py:114-121 is resident in HBM, one
// {start, end, thr, tag} record per data position, tag = read << 6 | j):
//   1. one stable radix pass on the chromosome carries the 16-B records: (chrom, start) order
//   2. per sorted position q (coalesced): the read's packed gate fields, start, (chrom, end) key
// General path (CSR only): radix sort of (chrom << 32 | start) → gather the records.
// Then, both paths:
//   3. inclusive max-scan of (chrom << 32 | end): per-chromosome prefix max of end (pmax)
//   4. scan ranges per interval, searched in an LDS window of starts / pmax around the block
//      (galloping out of the window in global memory when a range is longer):
//        n_fwd     = #{p > q : start_p <= end_q}        (all overlap: start_q <= start_p <= end_q)
//        bwd_begin = first p with pmax_p >= start_q     (p < q with pmax < start_q cannot overlap)
//      so a query interval's end-inclusive overlaps (superintervals search_values semantics,
//      SURVEY.md §8a A6) are exactly: q+1 .. q+n_fwd, plus p in [bwd_begin, q) with end_p >= start_q.
#include <hipcub/hipcub.hpp>

#include "kernels.hpp"

namespace fslr {
namespace {

constexpr int kRangeBlock = 256;
constexpr int kWin = 512;

__global__ void k_keys_csr(const int4* __restrict__ rmeta, const int4* __restrict__ iv, int n,
                           unsigned long long* __restrict__ keys64, int* __restrict__ vals) {
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
    const int4 m = rmeta[r];
    const int len = m.y & 0xffff;
    for (int j = 0; j < len; ++j) {
      const int k = m.x + j;
      const int4 rec = iv[k];
      keys64[k] = (static_cast<unsigned long long>(rec.x) << 32) | static_cast<unsigned>(rec.y);
      vals[k] = (r << 6) | j;
    }
  }
}

// general path: records from the CSR by tag
__global__ void k_gather_records(const int* __restrict__ stags, const int4* __restrict__ iv,
                                 const int4* __restrict__ rmeta, int ni, int4* __restrict__ idx4) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < ni; q += gridDim.x * blockDim.x) {
    const int rj = stags[q];
    const int4 rec = iv[rmeta[rj >> 6].x + (rj & 63)];
    idx4[q] = make_int4(rec.y, rec.z, rec.w, rj);
  }
}

// per sorted position: gate fields of the read, start, (chrom, end) key
template <bool kKey64>
__global__ void k_finish(const int4* __restrict__ idx4, const void* __restrict__ skeys,
                         const int4* __restrict__ rmeta, int ni, int2* __restrict__ idx_gate,
                         int* __restrict__ s_start, unsigned long long* __restrict__ endkey) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < ni; q += gridDim.x * blockDim.x) {
    const int4 rec = idx4[q];
    const int4 m = rmeta[rec.w >> 6];
    const unsigned c = kKey64 ? static_cast<unsigned>(static_cast<const unsigned long long*>(skeys)[q] >> 32)
                              : static_cast<const unsigned*>(skeys)[q];
    // {qlen2, nal | LB << 24 | haz << 31}
    idx_gate[q] = make_int2(m.z, (m.w & 0xFFFFFF) | ((m.y & 0x7F) << 24) | (((m.y >> 16) & 1) << 31));
    s_start[q] = rec.x;
    endkey[q] = (static_cast<unsigned long long>(c) << 32) | static_cast<unsigned>(rec.y);
  }
}

struct MaxU64 {
  __device__ __forceinline__ unsigned long long operator()(unsigned long long a, unsigned long long b) const {
    return a > b ? a : b;
  }
};

__device__ __forceinline__ int pmax_at(const unsigned long long* pmaxkey, int p) {
  return static_cast<int>(static_cast<unsigned>(pmaxkey[p]));
}

__global__ __launch_bounds__(kRangeBlock) void k_ranges(const int4* __restrict__ idx4, const int4* __restrict__ rmeta,
                                                        const int* __restrict__ s_start,
                                                        const unsigned long long* __restrict__ endkey,
                                                        const unsigned long long* __restrict__ pmaxkey,
                                                        const int2* __restrict__ crange, int ni,
                                                        int4* __restrict__ iv_rng) {
  __shared__ int w_st[kRangeBlock + 2 * kWin];   // starts of [w0, w1)
  __shared__ int w_pm[kRangeBlock + kWin];       // pmax of [w0, q0 + kRangeBlock)
  const int q0 = blockIdx.x * kRangeBlock;
  const int w0 = max(q0 - kWin, 0);
  const int w1 = min(q0 + kRangeBlock + kWin, ni);
  const int wp1 = min(q0 + kRangeBlock, ni);
  for (int t = threadIdx.x; t < w1 - w0; t += kRangeBlock) w_st[t] = s_start[w0 + t];
  for (int t = threadIdx.x; t < wp1 - w0; t += kRangeBlock) w_pm[t] = pmax_at(pmaxkey, w0 + t);
  __syncthreads();
  const int q = q0 + threadIdx.x;
  if (q >= ni) return;
  const unsigned long long ek = endkey[q];
  const int2 cr = crange[static_cast<int>(ek >> 32)];
  const int s = w_st[q - w0], e = static_cast<int>(static_cast<unsigned>(ek));
  // forward: first p in (q, cr.y) with start_p > e
  int hi_lim = min(cr.y, w1);
  int lo = q + 1, hi = hi_lim;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (w_st[mid - w0] <= e) lo = mid + 1; else hi = mid;
  }
  if (lo == hi_lim && hi_lim < cr.y) {   // range leaves the window: gallop on in global memory
    int step = 1;
    hi = lo;
    while (hi < cr.y && s_start[hi] <= e) {
      lo = hi + 1;
      hi = lo + step;
      step <<= 1;
    }
    if (hi > cr.y) hi = cr.y;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s_start[mid] <= e) lo = mid + 1; else hi = mid;
    }
  }
  const int n_fwd = lo - q - 1;
  // backward: first p in [cr.x, q) with pmax_p >= s (pmax non-decreasing inside a chromosome)
  const int lo_lim = max(cr.x, w0);
  lo = lo_lim;
  hi = q;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (w_pm[mid - w0] >= s) hi = mid; else lo = mid + 1;
  }
  if (lo == lo_lim && lo_lim > cr.x && lo < q) {   // may extend below the window
    hi = lo;
    int step = 1;
    int cand = lo - 1;
    while (cand >= cr.x && pmax_at(pmaxkey, cand) >= s) {
      hi = cand;
      cand = hi - step;
      step <<= 1;
    }
    lo = cand < cr.x ? cr.x : cand + 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (pmax_at(pmaxkey, mid) >= s) hi = mid; else lo = mid + 1;
    }
  }
  const int rj = idx4[q].w;
  iv_rng[rmeta[rj >> 6].x + (rj & 63)] = make_int4(q, n_fwd, lo, q - lo);
}

__global__ void k_set_thr(const int* __restrict__ thr, int4* __restrict__ iv, const int4* __restrict__ iv_rng,
                          int4* __restrict__ idx4, const int* __restrict__ data_pos, int4* __restrict__ drec,
                          int ni) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ni; k += gridDim.x * blockDim.x) {
    iv[k].w = thr[k];
    if (idx4) idx4[iv_rng[k].x].z = thr[k];
    if (drec) drec[data_pos[k]].z = thr[k];
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
                                         static_cast<unsigned*>(nullptr), static_cast<int4*>(nullptr),
                                         static_cast<int4*>(nullptr), ni, 0, 32, s);
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
  if (b.dchrom) {
    unsigned* k32 = reinterpret_cast<unsigned*>(b.keys2);
    e = hipcub::DeviceRadixSort::SortPairs(b.temp, tb, b.dchrom, k32, b.drec, b.idx4, ni, 0, bits_for(n_chroms), s);
    if (e != hipSuccess) return e;
    k_finish<false><<<grid_for(ni), 256, 0, s>>>(b.idx4, k32, b.rmeta, ni, b.idx_gate, b.s_start, b.endkey);
  } else {
    k_keys_csr<<<grid_for(n), 256, 0, s>>>(b.rmeta, b.iv, n, b.keys, b.vals);
    e = hipcub::DeviceRadixSort::SortPairs(b.temp, tb, b.keys, b.keys2, b.vals, b.vals2, ni, 0,
                                           32 + bits_for(n_chroms), s);
    if (e != hipSuccess) return e;
    k_gather_records<<<grid_for(ni), 256, 0, s>>>(b.vals2, b.iv, b.rmeta, ni, b.idx4);
    k_finish<true><<<grid_for(ni), 256, 0, s>>>(b.idx4, b.keys2, b.rmeta, ni, b.idx_gate, b.s_start, b.endkey);
  }
  tb = b.temp_bytes;
  e = hipcub::DeviceScan::InclusiveScan(b.temp, tb, b.endkey, b.pmaxkey, MaxU64(), ni, s);
  if (e != hipSuccess) return e;
  k_ranges<<<(ni + kRangeBlock - 1) / kRangeBlock, kRangeBlock, 0, s>>>(b.idx4, b.rmeta, b.s_start, b.endkey,
                                                                         b.pmaxkey, b.crange, ni, b.iv_rng);
  return hipGetLastError();
}

hipError_t launch_set_thr(const int* thr, int4* iv, const int4* iv_rng, int4* idx4, const int* data_pos,
                          int4* drec, int ni, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  k_set_thr<<<grid_for(ni), 256, 0, s>>>(thr, iv, iv_rng, idx4, data_pos, drec, ni);
  return hipGetLastError();
}

}  // namespace fslr
