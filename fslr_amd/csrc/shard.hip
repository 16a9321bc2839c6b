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
//  * k_own_flags / k_own_scatter: the owned chromosomes' data-order records, compacted stably and
//    renumbered 0 .. k-1 in chromosome order (the index build's input; the build itself is
//    index.hip's: the counting sort for k <= 64 owned chromosomes, the radix pass beyond);
//  * the routing by destination is the grouping sort's bucket pass with bucket (a >> shift) % W,
//    reading the sweep's tile slots directly (sweep.hip launch_sweep_partition).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "kernels.hpp"

namespace fslr {
namespace {

constexpr int kBlk = 256;

__global__ void k_own_flags(const unsigned* __restrict__ dchrom, const int* __restrict__ lmap, int ni,
                            int* __restrict__ flags) {
  for (int k = blockIdx.x * kBlk + threadIdx.x; k < ni; k += gridDim.x * kBlk)
    flags[k] = lmap[dchrom[k]] >= 0;
}

__global__ void k_own_scatter(const unsigned* __restrict__ dchrom, const int4* __restrict__ drec,
                              const int2* __restrict__ dgate, const int* __restrict__ flags,
                              const int* __restrict__ lmap, const int* __restrict__ offs, int ni,
                              unsigned* __restrict__ fdchrom, int4* __restrict__ fdrec, int2* __restrict__ fdgate) {
  for (int k = blockIdx.x * kBlk + threadIdx.x; k < ni; k += gridDim.x * kBlk) {
    if (!flags[k]) continue;
    const int o = offs[k];
    fdchrom[o] = static_cast<unsigned>(lmap[dchrom[k]]);   // the rank's own chromosome numbering
    fdrec[o] = drec[k];
    fdgate[o] = dgate[k];
  }
}

}  // namespace

hipError_t launch_chrom_filter(const unsigned* dchrom, const int4* drec, const int2* dgate, const int* lmap, int ni,
                               unsigned* fdchrom, int4* fdrec, int2* fdgate, int* flags, int* offs, void* temp,
                               size_t temp_bytes, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  const int grid = static_cast<int>(std::min<long long>(4096, (ni + kBlk - 1) / kBlk));
  k_own_flags<<<grid, kBlk, 0, s>>>(dchrom, lmap, ni, flags);
  size_t need = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, need, flags, offs, ni, s);
  if (e != hipSuccess) return e;
  if (need > temp_bytes) return hipErrorInvalidValue;
  e = hipcub::DeviceScan::ExclusiveSum(temp, need, flags, offs, ni, s);
  if (e != hipSuccess) return e;
  k_own_scatter<<<grid, kBlk, 0, s>>>(dchrom, drec, dgate, flags, lmap, offs, ni, fdchrom, fdrec, fdgate);
  return hipGetLastError();
}

}  // namespace fslr
