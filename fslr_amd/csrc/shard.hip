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

// ---- the position split: a rank's contiguous range of sorted positions --------------------------
// per tile of 64 sorted positions: its pair tests (the sum of the forward counts, the sweep's cost)
// and the end of its forward window (max q + n_fwd(q) + 1: the records a rank sweeping the tile needs)
__global__ void k_tile_costs(const int* __restrict__ swin, int ni, long long* __restrict__ tests,
                             long long* __restrict__ reach) {
  const int nt = (ni + kWave - 1) / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  for (int t = (blockIdx.x * kBlk + threadIdx.x) >> 6; t < nt; t += (gridDim.x * kBlk) >> 6) {
    const int q = t * kWave + lane;
    const int nf = q < ni ? swin[q] : 0;
    long long sum = nf;
    int r = q < ni ? q + nf + 1 : 0;
    for (int o = 32; o > 0; o >>= 1) {
      sum += __shfl_xor(sum, o);
      r = max(r, __shfl_xor(r, o));
    }
    if (lane == 0) {
      tests[t] = sum;
      reach[t] = r;
    }
  }
}

// the data positions whose sorted position (qd, the data -> sorted map) lies in [lo, end)
__global__ void k_pos_flags(const int* __restrict__ qd, int ni, int lo, int end, int* __restrict__ flags) {
  for (int d = blockIdx.x * kBlk + threadIdx.x; d < ni; d += gridDim.x * kBlk) flags[d] = qd[d] >= lo && qd[d] < end;
}

__global__ void k_pos_sel(const int* __restrict__ flags, const int* __restrict__ offs, int ni, int* __restrict__ sel) {
  for (int d = blockIdx.x * kBlk + threadIdx.x; d < ni; d += gridDim.x * kBlk)
    if (flags[d]) sel[offs[d]] = d;
}

// the selected records in data order (so the counting sort by chromosome gives the global order
// restricted to the range), chromosomes renumbered by lmap
__global__ void k_pos_gather(const int* __restrict__ sel, int m, const unsigned* __restrict__ dchrom,
                             const int4* __restrict__ drec, const int2* __restrict__ dgate, const int* __restrict__ lmap,
                             unsigned* __restrict__ fdchrom, int4* __restrict__ fdrec, int2* __restrict__ fdgate) {
  for (int k = blockIdx.x * kBlk + threadIdx.x; k < m; k += gridDim.x * kBlk) {
    const int d = sel[k];
    fdchrom[k] = static_cast<unsigned>(lmap[dchrom[d]]);
    fdrec[k] = drec[d];
    fdgate[k] = dgate[d];
  }
}

}  // namespace

hipError_t launch_tile_costs(const int* swin, int ni, long long* tests, long long* reach, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  const long long nt = (ni + kWave - 1) / kWave;
  k_tile_costs<<<static_cast<int>(std::min<long long>(4096, (nt * kWave + kBlk - 1) / kBlk)), kBlk, 0, s>>>(swin, ni, tests,
                                                                                                        reach);
  return hipGetLastError();
}

// sel[0, end - lo) = the data positions of the sorted positions [lo, end), ascending
hipError_t launch_pos_select(const int* qd, int ni, int lo, int end, int* flags, int* offs, int* sel,
                             void* temp, size_t temp_bytes, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  const int grid = static_cast<int>(std::min<long long>(4096, (ni + kBlk - 1) / kBlk));
  k_pos_flags<<<grid, kBlk, 0, s>>>(qd, ni, lo, end, flags);
  size_t need = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, need, flags, offs, ni, s);
  if (e != hipSuccess) return e;
  if (need > temp_bytes) return hipErrorInvalidValue;
  e = hipcub::DeviceScan::ExclusiveSum(temp, need, flags, offs, ni, s);
  if (e != hipSuccess) return e;
  k_pos_sel<<<grid, kBlk, 0, s>>>(flags, offs, ni, sel);   // end - lo of them: the whole range
  return hipGetLastError();
}

hipError_t launch_pos_gather(const int* sel, int m, const unsigned* dchrom, const int4* drec, const int2* dgate,
                             const int* lmap, unsigned* fdchrom, int4* fdrec, int2* fdgate, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  const int grid = static_cast<int>(std::min<long long>(4096, (m + kBlk - 1) / kBlk));
  k_pos_gather<<<grid, kBlk, 0, s>>>(sel, m, dchrom, drec, dgate, lmap, fdchrom, fdrec, fdgate);
  return hipGetLastError();
}

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
