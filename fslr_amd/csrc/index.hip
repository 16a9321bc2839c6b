// index.hip — the interval index (replaces build_interval_trees, cluster.py:124-130, and the
// superintervals IntervalMap it builds per chromosome).
//
// Fast path (the start-sorted `data` list of cluster.py:114-121 is resident in HBM, one
// {start, end, thr, tag} record, gate word and CSR index per data position, tag = read << 6 | j):
//   1-2. a stable counting sort on the chromosome (<= 64 chromosomes: k_chrom_*; otherwise one
//        radix pass + k_finish) writes the records, gate words, starts and (chrom, end) keys at
//        their (chrom, start) positions and the CSR -> sorted position map
// General path (CSR only): radix sort of (chrom << 32 | start) → gather the records.
// Then, both paths:
//   3. per 256-position tile, the max of (chrom << 32 | end) (written by k_finish), and their
//      inclusive max-scan (one small block): the per-chromosome prefix max of end (pmax) at tile
//      granularity — pmax at any position is the previous tile's prefix and a scan inside the tile
//   4. scan ranges per interval, searched in an LDS window of starts / pmax around the block
//      (pmax rebuilt in LDS from the tile prefix; galloping out of the window in global memory
//      when a range is longer):
//        n_fwd     = #{p > q : start_p <= end_q}        (all overlap: start_q <= start_p <= end_q)
//        bwd_begin = first p with pmax_p >= start_q     (p < q with pmax < start_q cannot overlap)
//      so a query interval's end-inclusive overlaps (superintervals search_values semantics,
//      SURVEY.md §8a A6) are exactly: q+1 .. q+n_fwd, plus p in [bwd_begin, q) with end_p >= start_q.
#include <hipcub/hipcub.hpp>

#include "kernels.hpp"
#include "wave.hpp"

namespace fslr {
namespace {

constexpr int kRangeBlock = 256;        // threads of k_ranges
constexpr int kRangeSpan = 1024;        // sorted positions per k_ranges block (4 per thread)
constexpr int kTile = 256;              // pmax tiles (window edges are tile-aligned)
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

__device__ __forceinline__ unsigned long long max_u64(unsigned long long a, unsigned long long b) {
  return a > b ? a : b;
}

// per sorted position: gate fields of the read, start, (chrom, end) key; per tile of kTile
// positions (one block iteration): the max key
template <bool kKey64>
__global__ __launch_bounds__(kTile) void k_finish(const int4* __restrict__ idx4, const void* __restrict__ skeys,
                                                  const int4* __restrict__ rmeta, int ni, int2* __restrict__ idx_gate,
                                                  int* __restrict__ s_start, unsigned long long* __restrict__ endkey,
                                                  unsigned long long* __restrict__ tile_max, int* __restrict__ qpos,
                                                  int shard, int n_shards) {
  __shared__ unsigned long long wmax[kTile / 64];
  const int n_tiles = (ni + kTile - 1) / kTile;
  for (int t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    const int q = t * kTile + threadIdx.x;
    unsigned long long key = 0ull;
    if (q < ni) {
      const int4 rec = idx4[q];
      const int4 m = rmeta[rec.w >> 6];
      const unsigned c = kKey64 ? static_cast<unsigned>(static_cast<const unsigned long long*>(skeys)[q] >> 32)
                                : static_cast<const unsigned*>(skeys)[q];
      // {qlen2, nal | LB << 24 | haz << 31}
      idx_gate[q] = make_int2(m.z, (m.w & 0xFFFFFF) | ((m.y & 0x7F) << 24) | (((m.y >> 16) & 1) << 31));
      s_start[q] = rec.x;
      // CSR interval -> sorted position (the one scatter of the build; this shard's reads only)
      if (shard_owns(rec.w >> 6, shard, n_shards)) qpos[m.x + (rec.w & 63)] = q;
      key = (static_cast<unsigned long long>(c) << 32) | static_cast<unsigned>(rec.y);
      endkey[q] = key;
    }
    for (int o = 32; o > 0; o >>= 1) key = max_u64(key, __shfl_xor(key, o));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = key;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long mx = wmax[0];
      for (int w = 1; w < kTile / 64; ++w) mx = max_u64(mx, wmax[w]);
      tile_max[t] = mx;
    }
    __syncthreads();
  }
}

// ---- fused data-order path (n_chroms <= 64) --------------------------------------------------
// A stable counting sort on the chromosome, one block per tile of rounds x 1024 data positions.
// Within a round of 64 lanes, six ballots of the chromosome bits give every lane the mask of lanes
// sharing its chromosome (its rank among them) and lane l the count of chromosome l.
//   k_chrom_count    counts per (chromosome, tile)                      reads 4 B / interval
//   k_chrom_scan     exclusive scan per chromosome (one block each) + the chromosome's begin
//   k_chrom_scatter  q = run[c] + rank: writes idx4, idx_gate, start, (chrom, end) key and the
//                    data -> sorted position map          reads 28 B, writes 40 B / interval
//   k_qpos_gather    CSR -> sorted position map
// The result is the stable partition of the start-sorted `data` list by chromosome, i.e. the
// same (chrom, start) order, ties included, as the radix pass it replaces.
constexpr int kTileThreads = 1024;
constexpr int kTileWaves = kTileThreads / 64;
// a block tile is `rounds` rounds of kTileThreads data positions, sized so the grid fits the chip in
// one pass (two 16-wave blocks per CU): 519 tiles of 16 rounds at cfg3 left 7 blocks for a second pass
int chrom_rounds(int ni) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || cus < 1)
      cus = 256;
  }
  const long long subs = (static_cast<long long>(ni) + kTileThreads - 1) / kTileThreads;
  const long long slots = 2ll * cus;
  return static_cast<int>(std::max(4ll, (subs + slots - 1) / slots));
}
constexpr int kChromBits = 6;
constexpr int kMaxFusedChroms = 1 << kChromBits;

__device__ __forceinline__ unsigned long long lane_mask_lt() {
  return (1ull << (threadIdx.x & 63)) - 1ull;
}

__global__ __launch_bounds__(kTileThreads) void k_chrom_count(const unsigned* __restrict__ dchrom, int ni,
                                                              int ntl, int rounds, int* __restrict__ chist) {
  __shared__ int wc[kTileWaves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int tl = blockIdx.x;
  const int e0 = tl * rounds * kTileThreads;
  int cnt = 0;
  // kU rounds' loads in flight before their ballots (one load's latency per kU rounds, not per round)
  constexpr int kU = 8;
  for (int r0 = 0; r0 < rounds; r0 += kU) {
    unsigned cc[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int e = e0 + (r0 + u) * kTileThreads + threadIdx.x;
      cc[u] = r0 + u < rounds && e < ni ? dchrom[e] : 0u;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (r0 + u >= rounds) break;                 // block-uniform
      const int e = e0 + (r0 + u) * kTileThreads + threadIdx.x;
      const unsigned c = cc[u];
      unsigned long long m = __ballot(e < ni);
#pragma unroll
      for (int b = 0; b < kChromBits; ++b) {
        const unsigned long long bb = __ballot((c >> b) & 1u);
        m &= ((lane >> b) & 1) ? bb : ~bb;
      }
      cnt += __popcll(m);
    }
  }
  wc[w][lane] = cnt;
  __syncthreads();
  if (w == 0) {
    int t = 0;
    for (int k = 0; k < kTileWaves; ++k) t += wc[k][lane];
    chist[lane * ntl + tl] = t;
  }
}

__global__ __launch_bounds__(1024) void k_chrom_scan(int* __restrict__ chist, int nsub,
                                                     const int2* __restrict__ crange) {
  __shared__ int part[1024];
  int* row = chist + blockIdx.x * nsub;
  const int per = (nsub + 1023) / 1024;
  const int b = threadIdx.x * per, e = min(b + per, nsub);
  int sum = 0;
  for (int i = b; i < e; ++i) sum += row[i];
  part[threadIdx.x] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int v = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int acc = crange[blockIdx.x].x + (threadIdx.x ? part[threadIdx.x - 1] : 0);
  for (int i = b; i < e; ++i) {
    const int x = row[i];
    row[i] = acc;
    acc += x;
  }
}

// One block of 16 waves per tile of `rounds` x 1024 data positions, rounds of 1024 in data order.
// Per round each wave ranks its lanes within their chromosome (ballots), the waves' per-chromosome
// counts are prefixed in LDS, and every element lands at q = run[c] + (earlier waves' count of c)
// + rank.  A chromosome's run in a tile (~700 positions at 23 chromosomes) is written by one block,
// so its cache lines fill up in one L2; with 1024-position tiles per wave the runs were ~45 long,
// most lines were shared by waves on different XCDs and the stores cost 155 of 215 us.
// qd[e] = q is written in data order for the CSR -> sorted position gather.
// kFull = false (the sweep engine's lean index): the (chrom, end) key and the data -> sorted map are
// not written (k_ranges reads each position's end from its record): 52 instead of 68 B / interval
template <bool kFull>
__global__ __launch_bounds__(kTileThreads) void k_chrom_scatter(const unsigned* __restrict__ dchrom,
                                                              const int4* __restrict__ drec,
                                                              const int2* __restrict__ dgate,
                                                              const int* __restrict__ chist, int ni, int ntl,
                                                              int rounds, int4* __restrict__ idx4, int2* __restrict__ idx_gate,
                                                              int* __restrict__ s_start,
                                                              unsigned long long* __restrict__ endkey,
                                                              int* __restrict__ qd) {
  __shared__ int wc[kTileWaves][64];      // this round: count of chromosome l in wave w
  __shared__ int wp[kTileWaves][64];      // this round: count of chromosome l in waves < w
  __shared__ int runs[2][64];             // next sorted position of chromosome l (double buffered)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int tl = blockIdx.x;
  const int e0 = tl * rounds * kTileThreads;
  const unsigned long long lt = lane_mask_lt();
  if (threadIdx.x < 64) runs[0][threadIdx.x] = chist[threadIdx.x * ntl + tl];
  auto load = [&](int r, unsigned& c, int4& rec, int2& gate) {
    const int e = e0 + r * kTileThreads + threadIdx.x;
    c = 0u;
    rec = make_int4(0, 0, 0, 0);
    gate = make_int2(0, 0);
    if (e < ni) {
      c = dchrom[e];
      rec = drec[e];
      gate = dgate[e];
    }
  };
  unsigned c_n;
  int4 rec_n;
  int2 gate_n;
  load(0, c_n, rec_n, gate_n);
  for (int r = 0; r < rounds; ++r) {
    const unsigned c = c_n;
    const int4 rec = rec_n;
    const int2 gate = gate_n;
    const int e = e0 + r * kTileThreads + threadIdx.x;
    const bool valid = e < ni;
    if (r + 1 < rounds) load(r + 1, c_n, rec_n, gate_n);
    const unsigned long long v = __ballot(valid);
    unsigned long long mine = v, mylane = v;
#pragma unroll
    for (int b = 0; b < kChromBits; ++b) {
      const unsigned long long bb = __ballot((c >> b) & 1u);
      mine &= ((c >> b) & 1u) ? bb : ~bb;
      mylane &= ((lane >> b) & 1) ? bb : ~bb;
    }
    wc[w][lane] = __popcll(mylane);
    __syncthreads();
    {
      // thread (w, l): chromosome l's count in waves < w; the last wave also advances the run
      int pre = 0;
      for (int k = 0; k < w; ++k) pre += wc[k][lane];
      wp[w][lane] = pre;
      if (w == kTileWaves - 1) runs[(r + 1) & 1][lane] = runs[r & 1][lane] + pre + wc[w][lane];
    }
    __syncthreads();
    if (valid) {
      const int q = runs[r & 1][c] + wp[w][c] + __popcll(mine & lt);
      idx4[q] = rec;
      idx_gate[q] = gate;
      s_start[q] = rec.x;
      if constexpr (kFull) {
        endkey[q] = (static_cast<unsigned long long>(c) << 32) | static_cast<unsigned>(rec.y);
        qd[e] = q;
      }                                          // (lean: the end column is idx4's .y)
    }
  }
}

// CSR -> sorted position map as a gather: qpos[k] = qd[data_pos[k]], one wavefront per block of 64
// ranks (the query-shard unit), whose intervals are one contiguous CSR span; blocks of other shards
// are skipped.  Coalesced reads of data_pos and writes of qpos; the random 4-B reads of qd hit the
// caches, where the scatter it replaces (qpos[k] = q in sorted order) wrote 8.5M partial lines
// (150 us at 1M reads, now ~1/3 of that).
__global__ __launch_bounds__(256) void k_qpos_gather(const int4* __restrict__ rmeta, const int* __restrict__ data_pos,
                                                     const int* __restrict__ qd, int n, int ni, int shard,
                                                     int n_shards, int* __restrict__ qpos) {
  const int lane = threadIdx.x & 63;
  const int nblk = (n + 63) >> kShardShift;
  for (int blk = blockIdx.x * 4 + (threadIdx.x >> 6); blk < nblk; blk += gridDim.x * 4) {
    if (!shard_owns(blk << kShardShift, shard, n_shards)) continue;
    const int r0 = blk << kShardShift, r1 = min(r0 + 64, n);
    const int k0 = rmeta[r0].x;
    const int k1 = r1 < n ? rmeta[r1].x : ni;
    for (int kb = k0; kb < k1; kb += 4 * 64) {
      int d[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = kb + u * 64 + lane;
        d[u] = k < k1 ? data_pos[k] : -1;
      }
      int q[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) q[u] = d[u] >= 0 ? qd[d[u]] : 0;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (d[u] >= 0) qpos[kb + u * 64 + lane] = q[u];
    }
  }
}

// per tile of kTile sorted positions: the max (chrom, end) key
__global__ __launch_bounds__(kTile) void k_tile_max(const unsigned long long* __restrict__ endkey, int ni,
                                                    unsigned long long* __restrict__ tile_max) {
  __shared__ unsigned long long wmax[kTile / 64];
  const int n_tiles = (ni + kTile - 1) / kTile;
  for (int t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    const int q = t * kTile + threadIdx.x;
    unsigned long long key = q < ni ? endkey[q] : 0ull;
    for (int o = 32; o > 0; o >>= 1) key = max_u64(key, __shfl_xor(key, o));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = key;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long mx = wmax[0];
      for (int w = 1; w < kTile / 64; ++w) mx = max_u64(mx, wmax[w]);
      tile_max[t] = mx;
    }
    __syncthreads();
  }
}

// inclusive max-scan of the tile maxima in two levels: groups of 1024 tiles (one block each,
// coalesced) hold local inclusive prefixes and a group total; one block scans the group totals.
// The inclusive prefix of tile t is max(group_excl[t / 1024], tile_loc[t]).
constexpr int kGroup = 1024;

__global__ __launch_bounds__(kGroup) void k_tile_scan_local(const unsigned long long* __restrict__ tile_max, int nt,
                                                            unsigned long long* __restrict__ tile_loc,
                                                            unsigned long long* __restrict__ group_tot) {
  __shared__ unsigned long long part[kGroup];
  const int t = blockIdx.x * kGroup + threadIdx.x;
  part[threadIdx.x] = t < nt ? tile_max[t] : 0ull;
  __syncthreads();
  for (int o = 1; o < kGroup; o <<= 1) {
    const unsigned long long v = threadIdx.x >= o ? part[threadIdx.x - o] : 0ull;
    __syncthreads();
    part[threadIdx.x] = max_u64(part[threadIdx.x], v);
    __syncthreads();
  }
  if (t < nt) tile_loc[t] = part[threadIdx.x];
  if (threadIdx.x == kGroup - 1) group_tot[blockIdx.x] = part[kGroup - 1];
}

__global__ __launch_bounds__(kGroup) void k_group_scan(unsigned long long* __restrict__ group, int ng) {
  __shared__ unsigned long long part[kGroup];
  const int per = (ng + kGroup - 1) / kGroup;
  const int b = threadIdx.x * per, e = min(b + per, ng);
  unsigned long long m = 0ull;
  for (int i = b; i < e; ++i) m = max_u64(m, group[i]);
  part[threadIdx.x] = m;
  __syncthreads();
  for (int o = 1; o < kGroup; o <<= 1) {
    const unsigned long long v = threadIdx.x >= o ? part[threadIdx.x - o] : 0ull;
    __syncthreads();
    part[threadIdx.x] = max_u64(part[threadIdx.x], v);
    __syncthreads();
  }
  m = threadIdx.x > 0 ? part[threadIdx.x - 1] : 0ull;     // exclusive prefix of this thread's groups
  for (int i = b; i < e; ++i) {
    const unsigned long long tot = group[i];
    group[i] = m;                                           // in place: exclusive prefix per group
    m = max_u64(m, tot);
  }
}

struct TilePrefix {
  const unsigned long long* loc;
  const unsigned long long* group_excl;
  __device__ __forceinline__ unsigned long long incl(int t) const { return max_u64(group_excl[t / kGroup], loc[t]); }
};

// kBwd = false (the sweep engine, lean index): the sweep windows (swin) only, no pmax window and no
// rng_s; ends from the records (idx4 .y; endkey unused), the chromosome from its begin in crange
// (n_chroms <= 64)
template <bool kBwd>
__global__ __launch_bounds__(kRangeBlock) void k_ranges(const int4* __restrict__ idx4, int shard, int n_shards,
                                                        const int* __restrict__ s_start,
                                                        const unsigned long long* __restrict__ endkey,
                                                        TilePrefix tile_incl,
                                                        const int2* __restrict__ crange, int ni,
                                                        int2* __restrict__ rng_s, int* __restrict__ swin,
                                                        const int2* __restrict__ gate, int n_chroms = 0,
                                                        long long* __restrict__ tile_tests = nullptr) {
  __shared__ int w_st[kRangeSpan + 2 * kWin];    // starts of [w0, w1)
  __shared__ int w_pm[kBwd ? kRangeSpan + kWin : 1];   // pmax (end part) of [w0, q0 + kRangeSpan)
  __shared__ unsigned long long t_part[kBwd ? kRangeBlock : 1];
  __shared__ int c_beg[kBwd ? 1 : 64];
  const int q0 = blockIdx.x * kRangeSpan;
  if constexpr (!kBwd)
    if (threadIdx.x < 64) c_beg[threadIdx.x] = threadIdx.x < n_chroms ? crange[threadIdx.x].x : 0x7FFFFFFF;
  const int w0 = max(q0 - kWin, 0);              // tile-aligned
  const int w1 = min(q0 + kRangeSpan + kWin, ni);
  const int wp1 = min(q0 + kRangeSpan, ni);
  for (int t = threadIdx.x; t < w1 - w0; t += kRangeBlock) w_st[t] = s_start[w0 + t];
  // pmax over [w0, wp1): prefix of the tiles before w0, then a scan of the window's keys
  if constexpr (kBwd) {
    constexpr int kPer = (kRangeSpan + kWin) / kRangeBlock;   // consecutive keys per thread
    unsigned long long k[kPer];
    unsigned long long m = 0ull;
    for (int u = 0; u < kPer; ++u) {
      const int p = w0 + threadIdx.x * kPer + u;
      k[u] = p < wp1 ? endkey[p] : 0ull;
      m = max_u64(m, k[u]);
    }
    t_part[threadIdx.x] = m;
    __syncthreads();
    for (int o = 1; o < kRangeBlock; o <<= 1) {
      const unsigned long long v = threadIdx.x >= o ? t_part[threadIdx.x - o] : 0ull;
      __syncthreads();
      t_part[threadIdx.x] = max_u64(t_part[threadIdx.x], v);
      __syncthreads();
    }
    m = w0 > 0 ? tile_incl.incl(w0 / kTile - 1) : 0ull;
    if (threadIdx.x > 0) m = max_u64(m, t_part[threadIdx.x - 1]);
    for (int u = 0; u < kPer; ++u) {
      m = max_u64(m, k[u]);
      w_pm[threadIdx.x * kPer + u] = static_cast<int>(static_cast<unsigned>(m));
    }
  }
  __syncthreads();
  // the lean build: this thread's records and gate words loaded up front (4 positions, all loads in
  // flight together instead of one position's behind the previous one's searches)
  constexpr int kPerQ = kRangeSpan / kRangeBlock;
  int4 pre4[kPerQ];
  int2 preg[kPerQ];
  if constexpr (!kBwd) {
#pragma unroll
    for (int u = 0; u < kPerQ; ++u) {
      const int q = q0 + threadIdx.x + u * kRangeBlock;
      pre4[u] = q < wp1 ? idx4[q] : make_int4(0, 0, 0, 0);
      preg[u] = q < wp1 ? gate[q] : make_int2(0, 0);
    }
    // The lean build writes the sweep windows only (the walk engine, the cap replay and k_swin read
    // n_fwd from k_ranges<true>'s rng_s: ensure_bwd_ranges / ensure_walk_index): one search per
    // position, for the window's bound start_p <= end_q - thr_q (cluster.py:133-136), or the whole
    // forward range start_p <= end_q when q's read has qlen2 or n_alignments 0 (cluster.py:178-183).
    // With `tile_tests`, each wave's 64 positions are one 64-position tile of the sweep: the wave sums
    // their windows (the tile's pair tests, which the sweep's plan scans for its upper-bound slots).
#pragma unroll
    for (int u = 0; u < kPerQ; ++u) {
      const int q = q0 + threadIdx.x + u * kRangeBlock;
      const int4 rq = pre4[u];
      int m = 0;
      if (q < wp1 && (n_shards == 1 || shard_owns(rq.w >> 6, shard, n_shards))) {
        const int e = rq.y;
        int c = 0;                                   // the last chromosome beginning at or before q
#pragma unroll
        for (int b = 32; b > 0; b >>= 1)
          if (c + b < 64 && c_beg[c + b] <= q) c += b;
        const int2 cr = crange[c];
        const int2 gq = preg[u];
        const int key = gq.x != 0 && (gq.y & 0xFFFFFF) != 0 ? min(e, e - rq.z) : e;
        const int hi_lim = min(cr.y, w1);
        int lo = q + 1, hi = hi_lim;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (w_st[mid - w0] <= key) lo = mid + 1; else hi = mid;
        }
        if (lo == hi_lim && hi_lim < cr.y) {       // the window leaves the LDS span: gallop in global memory
          int step = 1;
          hi = lo;
          while (hi < cr.y && s_start[hi] <= key) {
            lo = hi + 1;
            hi = lo + step;
            step <<= 1;
          }
          if (hi > cr.y) hi = cr.y;
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_start[mid] <= key) lo = mid + 1; else hi = mid;
          }
        }
        m = lo - q - 1;
        swin[q] = m;
      }
      if (tile_tests) {
        const int tot = rdl(wave_incl_scan(m), kWave - 1);
        const int tq = q0 + (threadIdx.x & ~(kWave - 1)) + u * kRangeBlock;   // the wave's tile
        if ((threadIdx.x & (kWave - 1)) == 0 && tq < wp1) tile_tests[tq / kWave] = tot;
      }
    }
    return;
  }
#pragma unroll
  for (int u = 0; u < kPerQ; ++u) {
    const int q = q0 + threadIdx.x + u * kRangeBlock;
    if (q >= wp1) break;
    const int4 rq = kBwd ? make_int4(0, 0, 0, 0) : pre4[u];
    if (n_shards > 1 && !shard_owns((kBwd ? idx4[q].w : rq.w) >> 6, shard, n_shards)) continue;   // another shard's A side
    int c, e;
    if constexpr (kBwd) {
      const unsigned long long ek = endkey[q];
      c = static_cast<int>(ek >> 32);
      e = static_cast<int>(static_cast<unsigned>(ek));
    } else {
      e = rq.y;                                  // (its .z, the threshold, is the window's below)
      c = 0;                                     // the last chromosome beginning at or before q
#pragma unroll
      for (int b = 32; b > 0; b >>= 1)
        if (c + b < 64 && c_beg[c + b] <= q) c += b;
    }
    const int2 cr = crange[c];
    const int s = w_st[q - w0];
    // forward: first p in (q, cr.y) with start_p > e
    const int hi_lim = min(cr.y, w1);
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
    // the sweep's window (swin): p with start_p <= end_q - thr_q only, the pairs calculate_overlap can
    // pass from q's side (cluster.py:133-136: min(end) - start_p >= thr_q); the whole forward range
    // when q's read has qlen2 or n_alignments 0 (a ZeroDivisionError pair is any hit, cluster.py:178-183)
    if (swin) {
      const int2 gq = kBwd ? gate[q] : preg[u];
      int m = n_fwd;
      if (gq.x != 0 && (gq.y & 0xFFFFFF) != 0) {
        const int key = e - (kBwd ? idx4[q].z : rq.z);
        int a = q + 1, z = lo;                   // first p in (q, lo) with start_p > key
        if (z <= w1) {
          while (a < z) {
            const int mid = (a + z) >> 1;
            if (w_st[mid - w0] <= key) a = mid + 1; else z = mid;
          }
        } else {
          while (a < z) {
            const int mid = (a + z) >> 1;
            if (s_start[mid] <= key) a = mid + 1; else z = mid;
          }
        }
        m = a - q - 1;
      }
      swin[q] = m;
    }
    // backward: first p in [cr.x, q) with pmax_p >= s (pmax non-decreasing inside a chromosome)
    const int lo_lim = max(cr.x, w0);
    lo = lo_lim;
    hi = q;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (w_pm[mid - w0] >= s) hi = mid; else lo = mid + 1;
    }
    if (lo == lo_lim && lo_lim > cr.x && lo < q) {
      // the answer may lie below the window: first tile (from the chromosome's) whose inclusive
      // prefix reaches (c, s), then the first position inside it
      const unsigned long long key = (static_cast<unsigned long long>(c) << 32) | static_cast<unsigned>(s);
      int tb = cr.x / kTile, te = w0 / kTile;
      while (tb < te) {
        const int mid = (tb + te) >> 1;
        if (tile_incl.incl(mid) >= key) te = mid; else tb = mid + 1;
      }
      if (tb < w0 / kTile) {
        unsigned long long m = tb > 0 ? tile_incl.incl(tb - 1) : 0ull;
        int p = tb * kTile;
        for (; p < w0; ++p) {
          m = max_u64(m, endkey[p]);
          if (m >= key) break;
        }
        lo = max(p, cr.x);
      }
    }
    rng_s[q] = make_int2(n_fwd, lo);
  }
}

__global__ void k_set_thr(const int* __restrict__ thr, int4* __restrict__ iv, const int* __restrict__ qpos,
                          int4* __restrict__ idx4, const int* __restrict__ data_pos, int4* __restrict__ drec,
                          int ni) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ni; k += gridDim.x * blockDim.x) {
    iv[k].w = thr[k];
    if (idx4) idx4[qpos[k]].z = thr[k];
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
  // the chromosome filter's scan of the owned flags (launch_chrom_filter) shares this buffer
  e = hipcub::DeviceScan::ExclusiveSum(nullptr, b2, static_cast<int*>(nullptr), static_cast<int*>(nullptr), ni, s);
  if (e != hipSuccess) return e;
  *bytes = b1 > b2 ? b1 : b2;
  if (b3 > *bytes) *bytes = b3;
  return hipSuccess;
}

// the walk engine's part of the index (data-order path): the CSR -> sorted position map, the
// tile prefix of end, and the backward scan ranges
static hipError_t launch_walk_parts(const IndexBufs& b, int n, int ni, hipStream_t s, bool qpos_and_tiles) {
  if (qpos_and_tiles) {
    k_qpos_gather<<<grid_for((n + 63) / 64, 4), 256, 0, s>>>(b.rmeta, b.data_pos, b.vals, n, ni, b.shard, b.n_shards,
                                                              b.qpos);
    k_tile_max<<<grid_for(ni, kTile), kTile, 0, s>>>(b.endkey, ni, b.pmaxkey);
  }
  // pmaxkey: tile maxima [0, nt), local group prefixes [nt, 2 nt), group prefixes [2 nt, 2 nt + ng)
  const int nt = (ni + kTile - 1) / kTile, ng = (nt + kGroup - 1) / kGroup;
  unsigned long long *tmax = b.pmaxkey, *tloc = b.pmaxkey + nt, *grp = b.pmaxkey + 2 * nt;
  k_tile_scan_local<<<ng, kGroup, 0, s>>>(tmax, nt, tloc, grp);
  k_group_scan<<<1, kGroup, 0, s>>>(grp, ng);
  k_ranges<true><<<(ni + kRangeSpan - 1) / kRangeSpan, kRangeBlock, 0, s>>>(b.idx4, b.shard, b.n_shards, b.s_start,
                                                                            b.endkey, TilePrefix{tloc, grp}, b.crange,
                                                                            ni, b.rng_s, b.swin, b.idx_gate);
  return hipGetLastError();
}

hipError_t launch_index_bwd_ranges(const IndexBufs& b, int ni, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  k_tile_max<<<grid_for(ni, kTile), kTile, 0, s>>>(b.endkey, ni, b.pmaxkey);
  return launch_walk_parts(b, 0, ni, s, false);
}

hipError_t launch_index_walk_parts(const IndexBufs& b, int n, int ni, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  return launch_walk_parts(b, n, ni, s, true);
}

hipError_t launch_build_index(const IndexBufs& b, int n, int ni, int n_chroms, bool full, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  hipError_t e;
  size_t tb = b.temp_bytes;
  if (b.dchrom && n_chroms <= kMaxFusedChroms) {
    const int rounds = chrom_rounds(ni);
    const int ntl = static_cast<int>((static_cast<long long>(ni) + rounds * kTileThreads - 1) / (rounds * kTileThreads));
    k_chrom_count<<<ntl, kTileThreads, 0, s>>>(b.dchrom, ni, ntl, rounds, b.chist);
    k_chrom_scan<<<n_chroms, 1024, 0, s>>>(b.chist, ntl, b.crange);
    if (!full) {
      // the sweep engine's lean index: records, gate words, starts and ends, forward counts
      k_chrom_scatter<false><<<ntl, kTileThreads, 0, s>>>(b.dchrom, b.drec, b.dgate, b.chist, ni, ntl, rounds, b.idx4,
                                                          b.idx_gate, b.s_start, b.endkey, b.vals);
      k_ranges<false><<<(ni + kRangeSpan - 1) / kRangeSpan, kRangeBlock, 0, s>>>(
          b.idx4, b.shard, b.n_shards, b.s_start, nullptr,
          TilePrefix{nullptr, nullptr}, b.crange, ni, b.rng_s, b.swin, b.idx_gate, n_chroms, b.tile_tests);
      return hipGetLastError();
    }
    k_chrom_scatter<true><<<ntl, kTileThreads, 0, s>>>(b.dchrom, b.drec, b.dgate, b.chist, ni, ntl, rounds, b.idx4, b.idx_gate,
                                                       b.s_start, b.endkey, b.vals);
    return launch_walk_parts(b, n, ni, s, true);
  } else if (b.dchrom) {
    unsigned* k32 = reinterpret_cast<unsigned*>(b.keys2);
    e = hipcub::DeviceRadixSort::SortPairs(b.temp, tb, b.dchrom, k32, b.drec, b.idx4, ni, 0, bits_for(n_chroms), s);
    if (e != hipSuccess) return e;
    k_finish<false><<<grid_for(ni, kTile), kTile, 0, s>>>(b.idx4, k32, b.rmeta, ni, b.idx_gate, b.s_start, b.endkey,
                                                          b.pmaxkey, b.qpos, b.shard, b.n_shards);
  } else {
    k_keys_csr<<<grid_for(n), 256, 0, s>>>(b.rmeta, b.iv, n, b.keys, b.vals);
    e = hipcub::DeviceRadixSort::SortPairs(b.temp, tb, b.keys, b.keys2, b.vals, b.vals2, ni, 0,
                                           32 + bits_for(n_chroms), s);
    if (e != hipSuccess) return e;
    k_gather_records<<<grid_for(ni), 256, 0, s>>>(b.vals2, b.iv, b.rmeta, ni, b.idx4);
    k_finish<true><<<grid_for(ni, kTile), kTile, 0, s>>>(b.idx4, b.keys2, b.rmeta, ni, b.idx_gate, b.s_start, b.endkey,
                                                         b.pmaxkey, b.qpos, b.shard, b.n_shards);
  }
  return launch_walk_parts(b, n, ni, s, false);
}

// the sweep windows again after the thresholds changed in place (fslr_set_thresholds): the same search
// as k_ranges', over the start column in global memory
__global__ __launch_bounds__(256) void k_swin(const int4* __restrict__ idx4, const int2* __restrict__ gate,
                                              const int2* __restrict__ rng_s, const int* __restrict__ s_start, int ni,
                                              int* __restrict__ swin) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < ni; q += gridDim.x * blockDim.x) {
    const int n_fwd = rng_s[q].x;
    const int2 gq = gate[q];
    int m = n_fwd;
    if (gq.x != 0 && (gq.y & 0xFFFFFF) != 0) {
      const int4 r = idx4[q];
      const int key = r.y - r.z;
      int a = q + 1, z = q + 1 + n_fwd;
      while (a < z) {
        const int mid = (a + z) >> 1;
        if (s_start[mid] <= key) a = mid + 1; else z = mid;
      }
      m = a - q - 1;
    }
    swin[q] = m;
  }
}

// a lean index's (chrom, end) keys from its records' ends (the backward ranges need them, not the map)
__global__ __launch_bounds__(256) void k_endkey(const int4* __restrict__ idx4, const int2* __restrict__ crange,
                                                int n_chroms, int ni, unsigned long long* __restrict__ endkey) {
  __shared__ int c_beg[64];
  if (threadIdx.x < 64) c_beg[threadIdx.x] = threadIdx.x < n_chroms ? crange[threadIdx.x].x : 0x7FFFFFFF;
  __syncthreads();
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < ni; q += gridDim.x * blockDim.x) {
    int c = 0;
#pragma unroll
    for (int b = 32; b > 0; b >>= 1)
      if (c + b < 64 && c_beg[c + b] <= q) c += b;
    endkey[q] = (static_cast<unsigned long long>(c) << 32) | static_cast<unsigned>(idx4[q].y);
  }
}

hipError_t launch_index_swin(const IndexBufs& b, int ni, hipStream_t s) {
  if (ni <= 0 || !b.swin) return hipSuccess;
  k_swin<<<grid_for(ni), 256, 0, s>>>(b.idx4, b.idx_gate, b.rng_s, b.s_start, ni, b.swin);
  return hipGetLastError();
}

hipError_t launch_index_endkeys(const IndexBufs& b, int ni, int n_chroms, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  if (n_chroms > kMaxFusedChroms) return hipErrorInvalidValue;
  k_endkey<<<grid_for(ni), 256, 0, s>>>(b.idx4, b.crange, n_chroms, ni, b.endkey);
  return hipGetLastError();
}

hipError_t launch_index_rescatter(const IndexBufs& b, int ni, int n_chroms, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  if (!b.dchrom || n_chroms > kMaxFusedChroms) return hipErrorInvalidValue;
  const int rounds = chrom_rounds(ni);
  const int ntl = static_cast<int>((static_cast<long long>(ni) + rounds * kTileThreads - 1) / (rounds * kTileThreads));
  k_chrom_count<<<ntl, kTileThreads, 0, s>>>(b.dchrom, ni, ntl, rounds, b.chist);
  k_chrom_scan<<<n_chroms, 1024, 0, s>>>(b.chist, ntl, b.crange);
  k_chrom_scatter<true><<<ntl, kTileThreads, 0, s>>>(b.dchrom, b.drec, b.dgate, b.chist, ni, ntl, rounds, b.idx4, b.idx_gate,
                                                     b.s_start, b.endkey, b.vals);
  return hipGetLastError();
}

hipError_t launch_set_thr(const int* thr, int4* iv, const int* qpos, int4* idx4, const int* data_pos,
                          int4* drec, int ni, hipStream_t s) {
  if (ni <= 0) return hipSuccess;
  k_set_thr<<<grid_for(ni), 256, 0, s>>>(thr, iv, qpos, idx4, data_pos, drec, ni);
  return hipGetLastError();
}

}  // namespace fslr
