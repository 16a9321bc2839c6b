// upload.hip — the device side of fslr_set_reads (capi.hip): the caller's CSR columns arrive as they are
// (one H2D copy each, no host packing) and are validated and packed here, including the start-sorted
// `data` list of prepare_data (cluster.py:109-121) the index is built from.
//
// Validation reports the input's first failure deterministically: every failing element offers
// (its index << 3 | code) to an atomicMin (err[0] for the intervals' columns, err[1] for the data
// order), so the lowest index wins whatever the schedule, with the check order of the host version
// (chromosome before coordinates for one interval; interval columns, then reads, then the data order).
#include <algorithm>

#include "fslr_hip.h"
#include "kernels.hpp"

namespace fslr {
namespace {

__global__ void k_up_iv(const int* __restrict__ chrom, const int* __restrict__ start, const int* __restrict__ end,
                        const int* __restrict__ thr, int ni, int n_chroms, int4* __restrict__ iv,
                        unsigned long long* __restrict__ err) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ni; k += gridDim.x * blockDim.x) {
    const int ch = chrom[k], s = start[k], e = end[k];
    int code = 0;
    if (ch < 0 || ch >= n_chroms) code = kUpErrChrom;
    else if (s < 0 || e < s || e >= kMaxCoord) code = kUpErrCoord;
    if (code) atomicMin(err, (static_cast<unsigned long long>(k) << 3) | static_cast<unsigned>(code));
    iv[k] = make_int4(ch, s, e, thr[k]);
  }
}

// intervals per chromosome: a block histogram in LDS (n_chroms <= kUpHistLds), else global atomics
__global__ __launch_bounds__(256) void k_up_chist(const int* __restrict__ chrom, int ni, int n_chroms,
                                                  unsigned long long* __restrict__ cnt) {
  __shared__ unsigned h[kUpHistLds];
  const bool lds = n_chroms <= kUpHistLds;
  if (lds)
    for (int i = threadIdx.x; i < n_chroms; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ni; k += gridDim.x * blockDim.x) {
    const int ch = chrom[k];
    if (ch < 0 || ch >= n_chroms) continue;
    if (lds) atomicAdd(&h[ch], 1u);
    else atomicAdd(cnt + ch, 1ull);
  }
  __syncthreads();
  if (lds)
    for (int i = threadIdx.x; i < n_chroms; i += blockDim.x)
      if (h[i]) atomicAdd(cnt + i, static_cast<unsigned long long>(h[i]));
}

// per read: {CSR offset, L | zero-aln flag << 16, qlen2, n_alignments} and its 1-byte length (read_off
// was validated on the host: every read has 1 .. FSLR_MAX_L intervals inside [0, ni))
__global__ void k_up_reads(const int* __restrict__ off, const int* __restrict__ qlen2, const int* __restrict__ nal,
                           const int* __restrict__ thr, int n, int4* __restrict__ rmeta,
                           unsigned char* __restrict__ rlen8) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int o = off[i], len = off[i + 1] - o;
    int flags = 0;
    for (int k = o; k < o + len; ++k) flags |= thr[k] == FSLR_THR_ZERO_ALN;
    rmeta[i] = make_int4(o, len | (flags << 16), qlen2[i], nal[i]);
    rlen8[i] = static_cast<unsigned char>(len);
  }
}

// the data order must be a permutation: inv[d] = k, a second k for one d (or d out of range) fails
__global__ void k_up_inv(const int* __restrict__ dp, int ni, int* __restrict__ inv, unsigned long long* __restrict__ err) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ni; k += gridDim.x * blockDim.x) {
    const int d = dp[k];
    if (d < 0 || d >= ni || atomicCAS(inv + d, -1, k) != -1)
      atomicMin(err + 1, (static_cast<unsigned long long>(k) << 3) | static_cast<unsigned>(kUpErrDataPos));
  }
}

// ... with non-decreasing starts along it
__global__ void k_up_sorted(const int* __restrict__ inv, const int* __restrict__ start, int ni,
                            unsigned long long* __restrict__ err) {
  for (int d = blockIdx.x * blockDim.x + threadIdx.x; d < ni; d += gridDim.x * blockDim.x) {
    const int k = inv[d];
    const int kp = d > 0 ? inv[d - 1] : 0;
    if (k < 0 || kp < 0 || (d > 0 && start[k] < start[kp]))
      atomicMin(err + 1, (static_cast<unsigned long long>(d) << 3) | static_cast<unsigned>(kUpErrDataPos));
  }
}

// the `data` list in its start-sorted order: chromosome, {start, end, thr, read << 6 | j} and the
// owning read's gate word (kernels.hpp idx_gate; the reference's IntervalItem carries qlen2 and
// n_alignments, cluster.py:10-11).  One thread per read, its intervals in CSR order.
__global__ void k_up_data(const int* __restrict__ off, const int* __restrict__ dp, const int4* __restrict__ iv,
                          const int4* __restrict__ rmeta, int n, int ni, unsigned* __restrict__ dch,
                          int4* __restrict__ drc, int2* __restrict__ dgt) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int4 m = rmeta[i];
    const int2 gate = make_int2(m.z, (m.w & 0xFFFFFF) | ((m.y & 0x7F) << 24) | (((m.y >> 16) & 1) << 31));
    const int o = off[i], e = off[i + 1];
    for (int k = o; k < e; ++k) {
      const int d = dp[k];
      if (d < 0 || d >= ni) continue;                  // flagged by k_up_inv; nothing written out of range
      const int4 v = iv[k];
      dch[d] = static_cast<unsigned>(v.x);
      drc[d] = make_int4(v.y, v.z, v.w, (i << 6) | (k - o));
      dgt[d] = gate;
    }
  }
}

__global__ void k_up_fill(int* __restrict__ p, int n, int v) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = v;
}

}  // namespace

hipError_t launch_upload_pack(const UploadArgs& a, hipStream_t s) {
  if (a.ni > 0) {
    k_up_iv<<<grid_for(a.ni), 256, 0, s>>>(a.chrom, a.start, a.end, a.thr, a.ni, a.n_chroms, a.iv, a.err);
    k_up_chist<<<std::min(grid_for(a.ni), 1024), 256, 0, s>>>(a.chrom, a.ni, a.n_chroms, a.chrom_cnt);
  }
  if (a.reads_ok && a.n > 0)
    k_up_reads<<<grid_for(a.n), 256, 0, s>>>(a.off, a.qlen2, a.nal, a.thr, a.n, a.rmeta, a.rlen8);
  if (a.dp && a.ni > 0) {
    k_up_fill<<<grid_for(a.ni), 256, 0, s>>>(a.inv, a.ni, -1);
    k_up_inv<<<grid_for(a.ni), 256, 0, s>>>(a.dp, a.ni, a.inv, a.err);
    k_up_sorted<<<grid_for(a.ni), 256, 0, s>>>(a.inv, a.start, a.ni, a.err);
    if (a.reads_ok && a.n > 0)
      k_up_data<<<grid_for(a.n), 256, 0, s>>>(a.off, a.dp, a.iv, a.rmeta, a.n, a.ni, a.dch, a.drc, a.dgt);
  }
  return hipGetLastError();
}

}  // namespace fslr
