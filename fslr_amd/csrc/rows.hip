// rows.hip — the clustering input built on the device from rows (fslr_set_reads_rows, capi.hip): the
// columnar CLI (fastcli.py) uploads keep_fillings' rows (cluster.py:14-31) and prepare_data's start
// order of them (cluster.py:109-121), and the device makes what the host used to: the `data` list
// after mask_sequences2 (cluster.py:89-106, as keep flags), the read ranks by first appearance in it
// and each read's interval list in data order (cluster.py:189-191: the CSR), the dense chromosome ids,
// and the folded overlap thresholds (calculate_overlap >= overlap, cluster.py:133-136; prep.py
// fold_overlap_threshold).  The packing and validation of fslr_set_reads (upload.hip) follow.
#include <hipcub/hipcub.hpp>

#include <cmath>

#include "fslr_hip.h"
#include "kernels.hpp"

namespace fslr {
namespace {

constexpr long long kMaxCoordL = 1ll << 30;

// the data list: rows order[d] whose keep flag is set (order's values checked in range)
__global__ void k_rows_flags(const long long* __restrict__ order, const unsigned char* __restrict__ keep, long long n,
                             int* __restrict__ ord32, unsigned char* __restrict__ flag, int* __restrict__ err) {
  for (long long d = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; d < n;
       d += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long r = order[d];
    const bool ok = r >= 0 && r < n;
    if (!ok) atomicOr(err, kRowsErrOrder);
    ord32[d] = ok ? static_cast<int>(r) : 0;
    flag[d] = ok && (!keep || keep[r]) ? 1 : 0;
  }
}

// first data position of every qname code (codes checked in range)
__global__ void k_rows_first(const int* __restrict__ sel, int m, const long long* __restrict__ qcode, long long n_codes,
                             int* __restrict__ first, int* __restrict__ err) {
  for (int d = blockIdx.x * blockDim.x + threadIdx.x; d < m; d += gridDim.x * blockDim.x) {
    const long long q = qcode[sel[d]];
    if (q < 0 || q >= n_codes) {
      atomicOr(err, kRowsErrCode);
      continue;
    }
    atomicMin(first + q, d);
  }
}

// a code out of range (flagged by k_rows_first) is read nowhere: it counts as no first appearance
__global__ void k_rows_isfirst(const int* __restrict__ sel, int m, const long long* __restrict__ qcode,
                               long long n_codes, const int* __restrict__ first, int* __restrict__ f) {
  for (int d = blockIdx.x * blockDim.x + threadIdx.x; d < m; d += gridDim.x * blockDim.x) {
    const long long q = qcode[sel[d]];
    f[d] = q >= 0 && q < n_codes && first[q] == d ? 1 : 0;
  }
}

// read rank of every data position (the scan of first appearances at its qname's first position), the
// qname code of every rank, and d as the value of the grouping sort
// (an out-of-range code, flagged before, takes rank 0: every write stays inside its array and the host
// reports kRowsErrCode after the build)
__global__ void k_rows_rank(const int* __restrict__ sel, int m, const long long* __restrict__ qcode, long long n_codes,
                            const int* __restrict__ first, const int* __restrict__ fscan, int* __restrict__ key,
                            int* __restrict__ val, long long* __restrict__ code_of_rank) {
  for (int d = blockIdx.x * blockDim.x + threadIdx.x; d < m; d += gridDim.x * blockDim.x) {
    const long long q = qcode[sel[d]];
    const bool ok = q >= 0 && q < n_codes;
    const int f = ok ? first[q] : d;
    const int r = ok ? fscan[f] : 0;
    key[d] = r;
    val[d] = d;
    if (ok && f == d) code_of_rank[r] = q;
  }
}

// CSR position k (sorted by rank, data order inside a read): the read offsets, the interval columns,
// the chromosomes present
__global__ void k_rows_csr(const int* __restrict__ rk, const int* __restrict__ perm, const int* __restrict__ sel, int m,
                           int n_reads, const long long* __restrict__ chrom, const long long* __restrict__ start,
                           const long long* __restrict__ end, const long long* __restrict__ aln, long long n_cids,
                           int* __restrict__ off, int* __restrict__ ch_raw, int* __restrict__ st32, int* __restrict__ en32,
                           long long* __restrict__ aln_k, int* __restrict__ dp, int* __restrict__ present,
                           int* __restrict__ err) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < m; k += gridDim.x * blockDim.x) {
    const int r = rk[k];
    if (k == 0 || rk[k - 1] != r) off[r] = k;
    if (k == m - 1) off[n_reads] = m;
    const int d = perm[k];
    const int row = sel[d];
    const long long c = chrom[row], s = start[row], e = end[row];
    int bad = 0;
    if (c < 0 || c >= n_cids) bad |= kRowsErrChrom;
    if (s < 0 || e < s || e >= kMaxCoordL) bad |= kRowsErrCoord;
    if (bad) atomicOr(err, bad);
    const int cc = bad & kRowsErrChrom ? 0 : static_cast<int>(c);
    ch_raw[k] = cc;
    if (!(bad & kRowsErrChrom) && !present[cc]) present[cc] = 1;    // a benign race: every writer stores 1
    st32[k] = bad & kRowsErrCoord ? 0 : static_cast<int>(s);
    en32[k] = bad & kRowsErrCoord ? 0 : static_cast<int>(e);
    aln_k[k] = aln[row];
    dp[k] = d;
  }
}

// per read: its gate values from its first interval (cluster.py:178-183 reads them per interval; they
// are per read in the reference's data), its length, and whether n_alignments varies inside it
__global__ void k_rows_reads(const int* __restrict__ off, int n_reads, const int* __restrict__ perm,
                             const int* __restrict__ sel, const long long* __restrict__ nal,
                             const long long* __restrict__ qlen2, int* __restrict__ q2_out, int* __restrict__ nal_out,
                             int* __restrict__ stat, int* __restrict__ err) {
  int mx = 0, varies = 0;
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n_reads; r += gridDim.x * blockDim.x) {
    const int o = off[r], e = off[r + 1];
    const int row0 = sel[perm[o]];
    const long long v = nal[row0], q = qlen2[row0];
    int bad = 0;
    if (v < 0 || v >= (1 << 24)) bad |= kRowsErrNal;
    if (q < 0 || q > 0x7FFFFFFFll) bad |= kRowsErrQlen;
    if (bad) atomicOr(err, bad);
    q2_out[r] = static_cast<int>(q < 0 ? 0 : q > 0x7FFFFFFFll ? 0x7FFFFFFF : q);
    nal_out[r] = static_cast<int>(bad & kRowsErrNal ? 0 : v);
    mx = max(mx, e - o);
    for (int k = o + 1; k < e && !varies; ++k) varies = nal[sel[perm[k]]] != v;
  }
  for (int s = 32; s > 0; s >>= 1) {
    mx = max(mx, __shfl_xor(mx, s));
    varies |= __shfl_xor(varies, s);
  }
  if ((threadIdx.x & 63) == 0) {
    if (mx) atomicMax(stat + 0, mx);
    if (varies) atomicOr(stat + 1, 1);
  }
}

// the least (or, p <= 0 with aln < 0, the greatest) integer overlap o with fl(o / aln) >= p — the
// integer form of calculate_overlap >= overlap (prep.py fold_overlap_threshold, same searches with the
// same correctly rounded IEEE divisions; include/fslr_hip.h for the encoding)
__device__ int fold_one(long long a, double p) {
  constexpr int kNever = 0x7FFFFFFF;
  if (a == 0) return FSLR_THR_ZERO_ALN;
  if (p != p) return kNever;                                   // NaN: nothing passes
  if (a > 0) {
    if (p <= 0.0) return 0;
    const double ap = static_cast<double>(a);
    long long t = static_cast<long long>(ceil(fmin(p * ap, 1099511627776.0)));
    if (t > kMaxCoordL + 2) return kNever;                     // no overlap below 2^30 reaches it
    for (int it = 0; it < 64; ++it) {
      const bool dec = t > 0 && static_cast<double>(t - 1) / ap >= p;
      const bool inc = !(static_cast<double>(t) / ap >= p);
      if (!dec && !inc) break;
      t = t - dec + inc;
    }
    return t >= kMaxCoordL ? kNever : static_cast<int>(t);
  }
  if (p > 0.0) return kNever;                                  // o / aln <= 0 < p
  const double an = static_cast<double>(-a), q = -p;
  long long h = static_cast<long long>(floor(fmin(q * an, 1099511627776.0)));
  if (h < kMaxCoordL) {
    for (int it = 0; it < 64; ++it) {
      const bool inc = static_cast<double>(h + 1) / an <= q;
      const bool dec = h > 0 && !(static_cast<double>(h) / an <= q);
      if (!inc && !dec) break;
      h = h + inc - dec;
    }
  }
  h = h < kMaxCoordL ? h : kMaxCoordL;
  return ~static_cast<int>(h);
}

__global__ void k_rows_fold(const long long* __restrict__ aln, int ni, double p, const int* __restrict__ ch_raw,
                            const int* __restrict__ dmap, int* __restrict__ thr, int* __restrict__ ch,
                            int* __restrict__ stat) {
  int mode = 0, zero = 0;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ni; k += gridDim.x * blockDim.x) {
    const int t = fold_one(aln[k], p);
    thr[k] = t;
    if (ch) ch[k] = dmap[ch_raw[k]];
    zero |= t == FSLR_THR_ZERO_ALN;
    mode |= t != FSLR_THR_ZERO_ALN && t < 1;
  }
  for (int s = 32; s > 0; s >>= 1) {
    mode |= __shfl_xor(mode, s);
    zero |= __shfl_xor(zero, s);
  }
  if ((threadIdx.x & 63) == 0) {
    if (mode) atomicOr(stat + 2, 1);
    if (zero) atomicOr(stat + 3, 1);
  }
}

__global__ void k_rows_zero(const int* __restrict__ thr, int ni, unsigned char* __restrict__ z) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ni; k += gridDim.x * blockDim.x)
    z[k] = thr[k] == FSLR_THR_ZERO_ALN;
}

__global__ void k_rows_fill(int* __restrict__ p, long long n, int v) {
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * blockDim.x)
    p[i] = v;
}

int bits_of(long long v) {
  int b = 1;
  while (b < 62 && (v >> b)) ++b;
  return b;
}

}  // namespace

// the data list and the read ranks: returns the list's length and the read count through host_out
// (synchronises).  Scratch comes from RowsWork.
hipError_t rows_rank(const RowsWork& w, long long n_rows, long long n_codes, const long long* order,
                     const unsigned char* keep, long long out[2], hipStream_t s) {
  out[0] = out[1] = 0;
  if (n_rows <= 0) return hipSuccess;
  k_rows_flags<<<grid_for(n_rows), 256, 0, s>>>(order, keep, n_rows, w.ord32, w.flag, w.err);
  size_t tb = w.temp_bytes;
  hipError_t e = hipcub::DeviceSelect::Flagged(w.temp, tb, w.ord32, w.flag, w.sel, w.nsel, static_cast<int>(n_rows), s);
  if (e != hipSuccess) return e;
  int m = 0;
  if ((e = hipMemcpyAsync(&m, w.nsel, sizeof(int), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
  out[0] = m;
  if (m == 0) return hipSuccess;
  k_rows_fill<<<grid_for(n_codes), 256, 0, s>>>(w.first, n_codes, 0x7FFFFFFF);
  k_rows_first<<<grid_for(m), 256, 0, s>>>(w.sel, m, w.qcode, n_codes, w.first, w.err);
  k_rows_isfirst<<<grid_for(m), 256, 0, s>>>(w.sel, m, w.qcode, n_codes, w.first, w.f);
  tb = w.temp_bytes;
  if ((e = hipcub::DeviceScan::ExclusiveSum(w.temp, tb, w.f, w.fscan, m, s)) != hipSuccess) return e;
  int last[2] = {0, 0};
  if ((e = hipMemcpyAsync(&last[0], w.fscan + m - 1, sizeof(int), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(&last[1], w.f + m - 1, sizeof(int), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
  out[1] = last[0] + last[1];
  k_rows_rank<<<grid_for(m), 256, 0, s>>>(w.sel, m, w.qcode, n_codes, w.first, w.fscan, w.key, w.val, w.code_of_rank);
  return hipGetLastError();
}

// scratch bytes of rows_rank / rows_csr's library calls for n rows
size_t rows_temp_bytes(long long n, hipStream_t s) {
  size_t a = 0, b = 0, c = 0;
  (void)hipcub::DeviceSelect::Flagged(nullptr, a, static_cast<int*>(nullptr), static_cast<unsigned char*>(nullptr),
                                      static_cast<int*>(nullptr), static_cast<int*>(nullptr), static_cast<int>(n), s);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, static_cast<int*>(nullptr), static_cast<int*>(nullptr),
                                         static_cast<int>(n), s);
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, c, static_cast<int*>(nullptr), static_cast<int*>(nullptr),
                                           static_cast<int*>(nullptr), static_cast<int*>(nullptr), static_cast<int>(n),
                                           0, 32, s);
  return std::max(a, std::max(b, c));
}

// group the data list by read rank (stable: data order inside a read) into the CSR columns
hipError_t rows_csr(const RowsWork& w, int m, int n_reads, long long n_cids, hipStream_t s) {
  size_t tb = w.temp_bytes;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(w.temp, tb, w.key, w.key_s, w.val, w.perm, m, 0,
                                                    bits_of(std::max(1, n_reads - 1)), s);
  if (e != hipSuccess) return e;
  if ((e = hipMemsetAsync(w.present, 0, static_cast<size_t>(n_cids) * sizeof(int), s)) != hipSuccess) return e;
  k_rows_csr<<<grid_for(m), 256, 0, s>>>(w.key_s, w.perm, w.sel, m, n_reads, w.chrom, w.start, w.end, w.aln, n_cids,
                                         w.off, w.ch_raw, w.st32, w.en32, w.aln_k, w.dp, w.present, w.err);
  k_rows_reads<<<grid_for(n_reads), 256, 0, s>>>(w.off, n_reads, w.perm, w.sel, w.nal, w.qlen2, w.q2, w.nal32,
                                                 w.stat, w.err);
  return hipGetLastError();
}

// the thresholds of overlap `p` in CSR order; with dmap also the dense chromosome ids.  stat[2] |= a
// threshold below 1 (the walk engine's general mode), stat[3] |= an aln_size == 0 interval
hipError_t rows_fold(const long long* aln_k, int ni, double p, const int* ch_raw, const int* dmap, int* thr, int* ch,
                     int* stat, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  k_rows_fold<<<grid_for(ni), 256, 0, s>>>(aln_k, ni, p, ch_raw, dmap, thr, ch, stat);
  return hipGetLastError();
}

hipError_t rows_zero_flags(const int* thr, int ni, unsigned char* z, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  k_rows_zero<<<grid_for(ni), 256, 0, s>>>(thr, ni, z);
  return hipGetLastError();
}

}  // namespace fslr
