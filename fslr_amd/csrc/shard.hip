// shard.hip — the multi-GPU split of the sweep engine.
//
// Every rank holds all reads (set_reads) but indexes only the chromosomes it owns: the first-fit
// match matrix of a read pair is block-diagonal by chromosome (an interval only meets intervals of
// its own chromosome, cluster.py:159-160), so the pair's intersection I is the sum of its
// per-chromosome matchings, and the match entries (a, b, i, j) each rank's sweep emits over its
// chromosomes are exactly the entries of the one-GPU sweep on them.  The entries are then routed
// to the rank owning read a (blocks of 2^shift ranks dealt round robin), which evaluates I, U and
// the edge for every pair whose first read it owns — each pair is evaluated by exactly one rank.
//
//  * k_own_flags / k_own_scatter: the owned chromosomes' data-order records, compacted stably
//    (the index build's input; the build itself is index.hip's, unchanged);
//  * k_part_count / k_part_scatter: match entries grouped by destination rank (counting sort over
//    <= 64 destinations, per-block LDS histograms, one scan).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "kernels.hpp"

namespace fslr {
namespace {

constexpr int kBlk = 256;

__global__ void k_own_flags(const unsigned* __restrict__ dchrom, unsigned long long owned, int ni,
                            int* __restrict__ flags) {
  for (int k = blockIdx.x * kBlk + threadIdx.x; k < ni; k += gridDim.x * kBlk)
    flags[k] = static_cast<int>((owned >> (dchrom[k] & 63u)) & 1ull);
}

__global__ void k_own_scatter(const unsigned* __restrict__ dchrom, const int4* __restrict__ drec,
                              const int2* __restrict__ dgate, const int* __restrict__ flags,
                              const int* __restrict__ offs, int ni, unsigned* __restrict__ fdchrom,
                              int4* __restrict__ fdrec, int2* __restrict__ fdgate) {
  for (int k = blockIdx.x * kBlk + threadIdx.x; k < ni; k += gridDim.x * kBlk) {
    if (!flags[k]) continue;
    const int o = offs[k];
    fdchrom[o] = dchrom[k];
    fdrec[o] = drec[k];
    fdgate[o] = dgate[k];
  }
}

// destination of an entry: its first read's block of 2^shift ranks, dealt round robin (low ranks
// have more higher-rank partners, so contiguous ranges would not balance the evaluation)
__device__ __forceinline__ int dest_of(unsigned long long e, int shift, int n_dest) {
  return static_cast<int>((e >> (39 + shift)) % static_cast<unsigned long long>(n_dest));
}

// per block b: counts of its chunk's entries per destination -> cnt[k * kPartBlocks + b]
__global__ void __launch_bounds__(kBlk) k_part_count(const unsigned long long* __restrict__ ent, long long n, int shift,
                                                     int n_dest, long long* __restrict__ cnt) {
  __shared__ int H[kMaxDest];
  if (threadIdx.x < kMaxDest) H[threadIdx.x] = 0;
  __syncthreads();
  const long long chunk = (n + kPartBlocks - 1) / kPartBlocks;
  const long long b0 = blockIdx.x * chunk, b1 = b0 + chunk < n ? b0 + chunk : n;
  for (long long k = b0 + threadIdx.x; k < b1; k += kBlk) atomicAdd(&H[dest_of(ent[k], shift, n_dest)], 1);
  __syncthreads();
  if (threadIdx.x < n_dest) cnt[static_cast<long long>(threadIdx.x) * kPartBlocks + blockIdx.x] = H[threadIdx.x];
}

__global__ void __launch_bounds__(kBlk) k_part_scatter(const unsigned long long* __restrict__ ent, long long n, int shift,
                                                       int n_dest, const long long* __restrict__ off,
                                                       unsigned long long* __restrict__ dst, long long dst_cap) {
  __shared__ unsigned long long P[kMaxDest];
  if (threadIdx.x < kMaxDest)
    P[threadIdx.x] = threadIdx.x < n_dest ? off[static_cast<long long>(threadIdx.x) * kPartBlocks + blockIdx.x] : 0;
  __syncthreads();
  const long long chunk = (n + kPartBlocks - 1) / kPartBlocks;
  const long long b0 = blockIdx.x * chunk, b1 = b0 + chunk < n ? b0 + chunk : n;
  for (long long k = b0 + threadIdx.x; k < b1; k += kBlk) {
    const unsigned long long e = ent[k];
    const long long o = static_cast<long long>(atomicAdd(&P[dest_of(e, shift, n_dest)], 1ull));
    if (o < dst_cap) dst[o] = e;
  }
}

// totals[k] = entries for destination k (from the scanned offsets and the last block's count)
__global__ void k_part_totals(const long long* __restrict__ cnt, const long long* __restrict__ off, int n_dest,
                              long long* __restrict__ totals) {
  const int k = threadIdx.x;
  if (k >= n_dest) return;
  const long long first = off[static_cast<long long>(k) * kPartBlocks];
  const long long last = static_cast<long long>(k) * kPartBlocks + kPartBlocks - 1;
  totals[k] = off[last] + cnt[last] - first;
}

}  // namespace

hipError_t launch_chrom_filter(const unsigned* dchrom, const int4* drec, const int2* dgate, unsigned long long owned,
                               int ni, unsigned* fdchrom, int4* fdrec, int2* fdgate, int* flags, int* offs,
                               void* temp, size_t temp_bytes, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  const int grid = static_cast<int>(std::min<long long>(4096, (ni + kBlk - 1) / kBlk));
  k_own_flags<<<grid, kBlk, 0, s>>>(dchrom, owned, ni, flags);
  size_t need = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, need, flags, offs, ni, s);
  if (e != hipSuccess) return e;
  if (need > temp_bytes) return hipErrorInvalidValue;
  e = hipcub::DeviceScan::ExclusiveSum(temp, need, flags, offs, ni, s);
  if (e != hipSuccess) return e;
  k_own_scatter<<<grid, kBlk, 0, s>>>(dchrom, drec, dgate, flags, offs, ni, fdchrom, fdrec, fdgate);
  return hipGetLastError();
}

size_t partition_temp_bytes(hipStream_t s) {
  size_t need = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, need, static_cast<long long*>(nullptr),
                                         static_cast<long long*>(nullptr), kMaxDest * kPartBlocks, s);
  return need;
}

hipError_t launch_partition_by_dest(const unsigned long long* ent, long long n, int shift, int n_dest,
                                    long long* scratch, void* temp, size_t temp_bytes, unsigned long long* dst,
                                    long long dst_cap, long long* totals, hipStream_t s) {
  long long* cnt = scratch;
  long long* off = scratch + static_cast<long long>(kMaxDest) * kPartBlocks;
  const int m = n_dest * kPartBlocks;
  k_part_count<<<kPartBlocks, kBlk, 0, s>>>(ent, n, shift, n_dest, cnt);
  size_t need = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, need, cnt, off, m, s);
  if (e != hipSuccess) return e;
  if (need > temp_bytes) return hipErrorInvalidValue;
  e = hipcub::DeviceScan::ExclusiveSum(temp, need, cnt, off, m, s);
  if (e != hipSuccess) return e;
  k_part_totals<<<1, kMaxDest, 0, s>>>(cnt, off, n_dest, totals);
  k_part_scatter<<<kPartBlocks, kBlk, 0, s>>>(ent, n, shift, n_dest, off, dst, dst_cap);
  return hipGetLastError();
}

}  // namespace fslr
