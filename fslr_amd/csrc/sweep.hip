// sweep.hip — the position-sweep pair engine: the driver of query_interval_trees (cluster.py:187-227)
// reorganised around the (chrom, start)-sorted index instead of the query reads.
//
// Every pair of end-inclusive overlapping intervals (the hits of superintervals' search_values,
// cluster.py:201) is q < p in sorted order with p in q + 1 .. q + n_fwd(q) (kernels.hpp: rng_s), so
// one forward sweep over the sorted positions meets each of them exactly once, in position order —
// consecutive positions share their windows, so the index streams through L1/L2 once instead of
// once per query read.  The rest of the reference's per-pair work is then:
//   1. k_sweep<2>: per overlapping interval pair of two different reads X != Y (A = min, B = max
//      rank): the pair gate different_lengths_or_alignments (:178-183, the integer ranges of
//      ratio_range), and calculate_overlap >= overlap (:133-136, folded thresholds: o >= max(thr)).
//      A pair that passes both is a match entry A << 39 | B << 14 | i << 7 | j (i, j: the intervals'
//      indices in their reads' lists, cluster.py:189-191), written at its 64-position tile's
//      upper-bound slot (the scan of the tiles' pair tests) — one pass, no global atomics — and
//      counted per coarse A bucket in the block's LDS histogram.
//   2. the entries are grouped by A: one scan of the sweep's [bucket][block] counts, k_sweep_scatter
//      (the sweep's tiles walked again in its own chunk order, LDS cursors), k_msd_pass2r (each
//      bucket by A's low bits, the bucket held in registers between its histogram and its scatter).
//   3. k_sweep_pairs: whole runs of one read A, up to 128 entries at a time, sorted by (run, B, i, j)
//      with a wave bitonic network; one lane per read pair: first-fit greedy (overall_jaccard_
//      similarity, :152-161) is the entry count unless two entries share a row or a column, where the
//      rows are walked in the reference's order (i ascending, lowest unused j).  Edge iff
//      U <= umax[I - 1] (:216-219).  A longer run goes through an LDS hash over its partners.
// A pair with overlapping intervals but no match entry is evaluated too — its I is 0 — so the
// edge set is the walk engine's E*, bit for bit.  The sweep does not count evaluated pairs (the
// reference's seen-set size): that is the walk engine's job (query.hip), which the parity tests
// and bench.py use for the counts.
// Scope: thresholds >= 1 (overlap > 0) and no aln_size == 0 interval; other inputs take the walk
// engine (capi.hip picks).
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "fslr_hip.h"
#include "kernels.hpp"
#include "wave.hpp"

namespace fslr {
namespace {

constexpr int kSwWaves = 4;
constexpr int kSwBlock = kSwWaves * kWave;
constexpr int kPairLimit = 64;             // long runs: insert while partners < limit (+64 per step <= 128)
constexpr int kPerPass = 40;               // entries per partner partition of a long run
constexpr int kWsFields = 4;               // per-wave statistics slots

__device__ __forceinline__ int entry_a(unsigned long long e) { return static_cast<int>(e >> 39); }
// lane masks: bits above / up to position h (0 <= h < 64)
__device__ __forceinline__ unsigned long long above(int h) { return h >= 63 ? 0ull : (~0ull << (h + 1)); }
__device__ __forceinline__ unsigned long long upto(int h) { return h >= 63 ? ~0ull : ((2ull << h) - 1); }

// same multiplier as the walk engine's partner partitions
__device__ __forceinline__ int part_of(int B, int npass) {
  return static_cast<int>(((static_cast<unsigned>(B) * 0x85EBCA6Bu) >> 8) % static_cast<unsigned>(npass));
}

// ---- 1. the sweep -------------------------------------------------------------------------------
// One wavefront per tile of 64 consecutive sorted positions (lane l holds q = q0 + l), tiles dealt in
// chunks of consecutive tiles, grid-stride over a resident grid.  The tile's forward ranges are
// flattened into an LDS map (item r -> its lane and p - q0), then walked 64 interval pairs per step,
// one per lane.
// The index records and gate words of positions [q0, q0 + kRing) sit in a per-wave LDS ring (slot
// p mod kRing): a tile's pairs have p in q0 + 1 .. q + n_fwd(q), so the p side of almost every pair
// test — and the q side — is an LDS read instead of a dependent gather through L1 / L2.  Moving to the
// next tile of a chunk loads only the 64 positions entering the ring (one coalesced record and gate
// load per lane: every position's 24 B cross HBM once per chunk); a pair beyond the ring (a tile whose
// forward window is longer) reads the index in global memory.
// kEmit = false counts the tile's entries (and the statistics); kEmit = true writes them.
constexpr int kRing = 128;                 // positions per wave in the LDS ring (64: +2 %, 256: +7 % step, profiles/r05/r5c)
static_assert(kRing >= kWave && (kRing & (kRing - 1)) == 0 && kRing < 1024, "ring size");
constexpr int kRingMask = kRing - 1;
constexpr int kMapCap = 1024;              // items per map segment (a longer tile takes several)
constexpr int kTileRun = 8;                // consecutive tiles per work item (two-pass fallback)
constexpr long long kTileCost = 256;       // a tile's fixed cost in pair tests (its ring load, header, map)

// One wave-instruction of keys (lanes with `act`, a contiguous prefix): equal keys on adjacent lanes
// form runs; the run's first lane adds its length to bin[key] (returning the base when `ret`), every
// lane gets base + its offset in the run.
template <bool kRet>
__device__ __forceinline__ int run_add(int* bin, int key, bool act, int lane) {
  const int prev = __shfl_up(key, 1);
  const bool head = act && (lane == 0 || prev != key);
  const unsigned long long hm = __ballot(head);
  const unsigned long long am = __ballot(act);
  const int n_act = __popcll(am);
  int base = 0;
  if (head) {
    const unsigned long long nx = hm & above(lane);
    const int len = (nx ? __builtin_ctzll(nx) : n_act) - lane;
    if (kRet) base = atomicAdd(&bin[key], len);
    else atomicAdd(&bin[key], len);
  }
  if (!kRet) return 0;
  const int my_head = 63 - __builtin_clzll(hm & upto(lane));   // lane 0 is a head when active
  return __shfl(base, act ? my_head : 0) + (lane - my_head);
}

constexpr int kHistMax = 1024;             // coarse A buckets the one-pass sweep counts (LDS)

// kMode 0: count the tile's entries (two-pass fallback), 1: write them at the tile's scanned offset
// (two-pass fallback), 2: one pass — write them at the tile's upper-bound slot (its forward-range
// total, the pair tests) and count them; k_compact then packs the tiles.
template <int kMode>
__global__ __launch_bounds__(kSwBlock) __attribute__((amdgpu_waves_per_eu(5))) void k_sweep(SweepArgs g) {
  constexpr bool kEmit = kMode != 0;
  constexpr bool kCount = kMode != 1;
  __shared__ int4 rr_all[kSwWaves][kRing];     // ring: index records {start, end, thr, read << 6 | j}
  __shared__ int2 rg_all[kSwWaves][kRing];     // ring: gate words {qlen2, nal | L << 24 | zero-aln << 31}
  __shared__ int4 qb_all[kSwWaves][kWave];     // lane's read's gate as integer ranges {qlo, qhi, nlo, nhi}
  __shared__ int off_all[kSwWaves][kWave];     // item r of lane k is position r + offv_k
  __shared__ unsigned char zf_all[kSwWaves][kWave];   // q's read has qlen2 == 0 (1) / n_alignments == 0 (2)
  __shared__ unsigned short map_all[kSwWaves][kMapCap];   // item -> lane | min(p - q0, kRing) << 6
  __shared__ unsigned long long st_all[kSwWaves][kEmit ? kWave : 1];
  __shared__ int hist_s[kMode == 2 ? kHistMax : 1];   // the block's entries per coarse A bucket
  unsigned long long* const dst = kMode == 2 ? g.ent_ub : g.ent;
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  const bool do_hist = kMode == 2 && g.hist_mat != nullptr;
  if (do_hist) {
    for (int i = threadIdx.x; i < g.hist_h; i += kSwBlock) hist_s[i] = 0;
    __syncthreads();
  }
  int4* RR = rr_all[wv];
  int2* RG = rg_all[wv];
  int4* QB = qb_all[wv];
  int* OFF = off_all[wv];
  unsigned char* ZF = zf_all[wv];
  unsigned short* MAP = map_all[wv];
  unsigned long long* ST = st_all[wv];
  unsigned long long w_tests = 0, w_hits = 0, w_ent = 0;
  const int nt = (g.nq + kWave - 1) / kWave;      // query tiles (the index may hold a halo beyond them)
  const int nw = gridDim.x * kSwWaves;
  const int wid = blockIdx.x * kSwWaves + wv;
  // tiles in chunks of up to kTileRun consecutive tiles per wave (a tile's forward window reaches
  // into the next tile, whose records the ring already holds), chunks dealt grid-stride; shorter
  // chunks when there are fewer than kTileRun tiles per wave of the grid (a rank's share of the
  // multi-GPU split), so every wave gets work: the sweep is latency bound
  // The one-pass sweep (kMode 2) instead gives each wave one contiguous range of tiles of equal cost
  // (pair tests + kTileCost per tile, k_wave_bounds): a tile's cost varies by orders of magnitude
  // with the local depth (a dense locus, one chromosome carrying most intervals), and chunks of equal
  // tile counts left the waves that drew dense chunks running long after the rest
#ifdef FSLR_SWEEP_CLOCK
  // measurement build: wave-clock sums (kMode 2) of the tile header, the item maps, the steps and the
  // tail into counters 68..71
  unsigned long long sck[4] = {0, 0, 0, 0};
  long long stk = clock64();
#define FSLR_SCK(k) do { if (kMode == 2) { const long long t_ = clock64(); sck[k] += t_ - stk; stk = t_; } } while (0)
#else
#define FSLR_SCK(k) do { } while (0)
#endif
  const int run = max(1, min(kTileRun, nt / nw));
  const int nchunks = kMode == 2 ? 1 : (nt + run - 1) / run;
  for (int chunk = kMode == 2 ? 0 : wid; chunk < nchunks; chunk += kMode == 2 ? 1 : nw) {
  const int tb = kMode == 2 ? g.wlo[wid] : chunk * run;
  const int te = kMode == 2 ? g.wlo[wid + 1] : min(nt, (chunk + 1) * run);
  for (int tile = tb; tile < te; ++tile) {
    const int q0 = tile * kWave;
    const int q = q0 + lane;
    const bool qv = q < g.nq;
    const int qc = qv ? q : q0;
    const bool first = tile == tb;
    const int nf = qv ? g.swin[qc] : 0;
    wave_lds_sync();                             // the previous tile's ring and map reads are done
    if (first) {
      // the chunk's first tile: positions [q0, q0 + kRing)
#pragma unroll
      for (int k = 0; k < kRing / kWave; ++k) {
        const int p = q0 + k * kWave + lane;
        if (p < g.ni) {
          RR[p & kRingMask] = g.idx4[p];
          RG[p & kRingMask] = g.idx_gate[p];
        }
      }
    } else {
      // the ring held [q0 - 64, q0 - 64 + kRing): the 64 positions entering it replace the last tile's
      const int p = q0 + kRing - kWave + lane;
      if (p < g.ni) {
        RR[p & kRingMask] = g.idx4[p];
        RG[p & kRingMask] = g.idx_gate[p];
      }
    }
    wave_lds_sync();
    const int4 rq = RR[qc & kRingMask];
    FSLR_BOUND(rq.w >> 6, g.n_reads);
    const int4 lbq = g.lb[rq.w >> 6];            // the gate of q's read as integer ranges
    const bool any_zero = __ballot(qv && (lbq.x < 0 || lbq.z < 0)) != 0ull;   // v == 0 (ZeroDivision)
    const int pre = wave_incl_scan(nf);
    const int ex = pre - nf;
    const bool fits = __ballot(qv && lane + nf >= kRing) == 0ull;   // every p of the tile in the ring
    const int T = rdl(pre, kWave - 1);
    // lower bounds with v == 0 (lo < 0: partner 0 raises, [1, hi] passes) folded to 1
    QB[lane] = make_int4(lbq.x < 0 ? 1 : lbq.x, lbq.y, lbq.z < 0 ? 1 : lbq.z, lbq.w);
    OFF[lane] = q + 1 - ex;
    ZF[lane] = static_cast<unsigned char>((lbq.x < 0 ? 1 : 0) | (lbq.z < 0 ? 2 : 0));
    long long out = 0;                           // kEmit: next entry slot of this tile
    if constexpr (kMode == 1) out = g.tile_off[tile];
    if constexpr (kMode == 2) {
      out = g.tile_ub[tile];
      if (out + T > g.ub_cap) {                  // the upper-bound buffer is too small: grow + rerun
        if (lane == 0) {
          atomicOr(g.err + kErrOverflow, 8);
          g.tile_cnt[tile] = 0;                  // the passes after the sweep read every tile's count
        }
        continue;
      }
    }
    int sn = 0, cnt = 0;                         // staged entries (kEmit) / entries of the tile
    // the staged entries to their slots (and, counting coarse buckets, into the block's histogram:
    // equal buckets on adjacent lanes take one LDS atomic)
    auto flush = [&]() __attribute__((always_inline)) {
      wave_lds_sync();
      const bool act = lane < sn;
      const unsigned long long v = act ? ST[lane] : 0ull;
      if (act) dst[out + lane] = v;
      if (do_hist) {
        const unsigned b = static_cast<unsigned>(v >> 39) >> g.hist_lo;
        run_add<false>(hist_s, static_cast<int>(g.hist_mod ? b % static_cast<unsigned>(g.hist_h) : b), act, lane);
      }
    };
    if constexpr (kCount) w_tests += static_cast<unsigned long long>(T);
    FSLR_SCK(3);
    for (int seg = 0; seg < T; seg += kMapCap) {
      const int se = min(T, seg + kMapCap);
      wave_lds_sync();
      for (int r = max(ex, seg); r < min(pre, se); ++r)
        MAP[r - seg] = static_cast<unsigned short>(lane | min(r - ex + lane + 1, kRing) << 6);
      wave_lds_sync();
      FSLR_SCK(1);
      // step operands: the mapped lane's gate ranges, q's record (ring), p's record and gate word
      // (ring; global beyond it)
      struct Step {
        int mi;
        int4 b4, a4, rp;
        int2 gp;
      };
      // kFits: every pair of the tile has its p in the ring (the usual case at cfg3), so the step
      // reads LDS only; otherwise (a deep locus: cfg5's ~50x coverage) it reads global memory only
      auto step_load = [&](auto fits_tag, int base, Step& t) __attribute__((always_inline)) {
        constexpr bool kFits = decltype(fits_tag)::value;
        const int r = base + lane;
        const unsigned md = r < se ? MAP[r - seg] : 0u;
        t.mi = static_cast<int>(md & 63u);
        const int d = static_cast<int>(md >> 6);
        t.b4 = QB[t.mi];
        t.a4 = RR[(q0 + t.mi) & kRingMask];
        if (kFits) {
          t.rp = RR[(q0 + d) & kRingMask];
          t.gp = RG[(q0 + d) & kRingMask];
        } else {
          // a deep tile (windows beyond the ring: every p from the index in global memory, as a
          // per-lane choice of address would make every load of the step a flat load)
          const int p = r < se ? r + OFF[t.mi] : q0;   // lanes past the segment read a valid position
          FSLR_BOUND(p, g.ni);
          t.rp = g.idx4[p];
          t.gp = g.idx_gate[p];
        }
      };
      // one step of 64 interval pairs; kZero: some q of the tile has qlen2 or n_alignments == 0
      // (only then can a pair raise ZeroDivisionError)
      auto step = [&](auto zero_tag, int base, const Step& t) __attribute__((always_inline)) {
        constexpr bool kZero = decltype(zero_tag)::value;
        const bool valid = base + lane < se;
        const int4 a4 = t.a4;
        const int X = a4.w >> 6, Y = t.rp.w >> 6;
        const bool hit = valid & (X != Y);
        // calculate_overlap >= overlap for both intervals: start_p >= start_q, start_p <= end_q
        const int o = min(a4.y, t.rp.y) - t.rp.x;
        const bool match = o >= max(a4.z, t.rp.z);
        // different_lengths_or_alignments: passes when either ratio is close (idx_gate word of p)
        const int q2 = t.gp.x, n2 = t.gp.y & 0xFFFFFF;
        const int qlo = t.b4.x, qhi = t.b4.y, nlo = t.b4.z, nhi = t.b4.w;
        const bool pq = (q2 >= qlo) & (q2 <= qhi);
        const bool lenok = pq | ((n2 >= nlo) & (n2 <= nhi));
        bool emit = hit & lenok & match;
        if constexpr (kZero) {
          const unsigned zf = ZF[t.mi];
          const bool zd = hit & ((((zf & 1u) != 0) & (q2 == 0)) | (!pq & ((zf & 2u) != 0) & (n2 == 0)));
          emit = emit & !zd;
          if (__ballot(zd)) raise_zd(g.err, zd, min(X, Y), max(X, Y));
        }
        const unsigned long long em = __ballot(emit);
        const int ne = __popcll(em);
        if constexpr (kCount) {
          w_hits += __popcll(__ballot(hit));
          cnt += ne;
        }
        if (kEmit && ne) {
          if (sn + ne > kWave) {
            flush();
            out += sn;
            sn = 0;
            wave_lds_sync();
          }
          if (emit) {
            // A << 39 | B << 14 | i << 7 | j as two dwords
            const int A = min(X, Y), B = max(X, Y);
            const int iq = a4.w & 63, jp = t.rp.w & 63;
            const unsigned ij = X < Y ? static_cast<unsigned>(iq << 7 | jp) : static_cast<unsigned>(jp << 7 | iq);
            const unsigned lo = (static_cast<unsigned>(B) << 14) | ij;
            const unsigned hi = (static_cast<unsigned>(A) << 7) | (static_cast<unsigned>(B) >> 18);
            ST[sn + mbcnt(em)] = (static_cast<unsigned long long>(hi) << 32) | lo;
          }
          sn += ne;
        }
      };
      auto run_steps = [&](auto zero_tag, auto fits_tag) __attribute__((always_inline)) {
        // LDS operands: other waves cover their latency
        for (int base = seg; base < se; base += kWave) {
          Step s0;
          step_load(fits_tag, base, s0);
          step(zero_tag, base, s0);
        }
      };
      if (fits) {
        if (any_zero) run_steps(std::true_type{}, std::true_type{});
        else run_steps(std::false_type{}, std::true_type{});
      } else {
        if (any_zero) run_steps(std::true_type{}, std::false_type{});
        else run_steps(std::false_type{}, std::false_type{});
      }
      FSLR_SCK(2);
    }
    if constexpr (kEmit) {
      if (sn > 0) flush();
    }
    if constexpr (kCount) {
      if (lane == 0) g.tile_cnt[tile] = cnt;
      w_ent += static_cast<unsigned long long>(cnt);
    }
    FSLR_SCK(0);                                 // (the tail, counted with the next tile's header)
  }
  }
#ifdef FSLR_SWEEP_CLOCK
  if (kMode == 2 && lane == 0)
    for (int k = 0; k < 4; ++k) atomicAdd(&g.counters[68 + k], sck[k]);
#endif
#undef FSLR_SCK
  if constexpr (kCount) {
    // statistics: plain stores into this wave's slots, summed by k_sweep_total / k_sum_slots
    const unsigned long long f = lane == 0 ? w_tests : lane == 1 ? w_hits : w_ent;
    if (lane < 3) g.wstat[static_cast<long long>(wid) * kWsFields + lane] = f;
  }
  if (do_hist) {
    __syncthreads();
    for (int i = threadIdx.x; i < g.hist_h; i += kSwBlock)
      g.hist_mat[static_cast<long long>(i) * gridDim.x + blockIdx.x] = hist_s[i];
  }
}

// Sum (fields 0..2) / max (field 3) of the per-wave slots [f0, f1) into counters / an err word: each
// block reduces a slice of waves, then one atomic per field and block (few blocks: no contention).
constexpr int kSumBlocks = 32;
__global__ __launch_bounds__(256) void k_sum_slots(const unsigned long long* __restrict__ ws, int nwaves, int f0,
                                                    int f1, int c0, int c1, int c2, unsigned long long* counters,
                                                    int* err_max) {
  __shared__ unsigned long long part[256][kWsFields];
  unsigned long long acc[kWsFields] = {0, 0, 0, 0};
  const int per = (nwaves + gridDim.x - 1) / gridDim.x;
  const int w0 = blockIdx.x * per, w1 = min(w0 + per, nwaves);
  for (int w = w0 + threadIdx.x; w < w1; w += 256)
    for (int f = f0; f < f1; ++f) {
      const unsigned long long x = ws[static_cast<long long>(w) * kWsFields + f];
      acc[f] = (f == 3) ? (acc[f] > x ? acc[f] : x) : acc[f] + x;
    }
  for (int f = 0; f < kWsFields; ++f) part[threadIdx.x][f] = acc[f];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o)
      for (int f = 0; f < kWsFields; ++f) {
        const unsigned long long x = part[threadIdx.x + o][f];
        part[threadIdx.x][f] = f == 3 ? (part[threadIdx.x][f] > x ? part[threadIdx.x][f] : x) : part[threadIdx.x][f] + x;
      }
    __syncthreads();
  }
  if (threadIdx.x < kWsFields) {
    const int f = threadIdx.x;
    const unsigned long long r = part[0][f];
    const int dst = f == 0 ? c0 : f == 1 ? c1 : c2;
    if (f < 3 && f >= f0 && f < f1 && dst >= 0 && r) atomicAdd(&counters[dst], r);
    if (f == 3 && f >= f0 && f < f1 && err_max && r) atomicMax(err_max, static_cast<int>(r));
  }
}

// entries of the count pass: last tile offset + last tile count; (one-pass) also the upper-bound
// total and the overflow flag, for the host.  n_dev (sync-free repeat query): the count for the
// grouping and pair kernels, clamped to the entry capacity cap (flag 16 when it did not fit: the
// query is then refused and rerun with a sync)
__global__ void k_total(const long long* __restrict__ off, const long long* __restrict__ cnt,
                        const long long* __restrict__ ub, const long long* __restrict__ tests, int* err, int nt,
                        long long* total, long long* n_dev, long long cap) {
  if (threadIdx.x == 0) {
    const long long t = off[nt - 1] + cnt[nt - 1];
    total[0] = t;
    total[1] = ub ? ub[nt - 1] + tests[nt - 1] : 0;
    if (n_dev) {
      n_dev[0] = t < cap ? t : cap;
      if (t > cap) atomicOr(&err[kErrOverflow], 16);
    }
    total[2] = err ? err[kErrOverflow] : 0;
  }
}

// one-pass sweep (kMode 2): the per-wave statistics summed into the counters (tests, hits, entries),
// the entry total and upper-bound total for the host, the clamped count for a sync-free query —
// one block in place of k_sum_slots, a scan of the tile counts and k_total
__global__ __launch_bounds__(1024) void k_sweep_total(const unsigned long long* __restrict__ ws, int nwaves,
                                                      const long long* __restrict__ ub,
                                                      const long long* __restrict__ tests, int nt,
                                                      unsigned long long* counters, int* err, long long* total,
                                                      long long* n_dev, long long cap, const int* __restrict__ mat,
                                                      int* __restrict__ off, int H, int P, long long* __restrict__ dtot) {
  __shared__ unsigned long long part[16][3];
  __shared__ int wsum[16];
  unsigned long long a0 = 0, a1 = 0, a2 = 0;
#pragma unroll 4
  for (int w = threadIdx.x; w < nwaves; w += 1024) {
    a0 += ws[static_cast<long long>(w) * kWsFields];
    a1 += ws[static_cast<long long>(w) * kWsFields + 1];
    a2 += ws[static_cast<long long>(w) * kWsFields + 2];
  }
  for (int o = 32; o > 0; o >>= 1) {
    a0 += __shfl_xor(a0, o);
    a1 += __shfl_xor(a1, o);
    a2 += __shfl_xor(a2, o);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    part[w][0] = a0;
    part[w][1] = a1;
    part[w][2] = a2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 16; ++k) {
      a0 += part[k][0];
      a1 += part[k][1];
      a2 += part[k][2];
    }
    counters[kSwTests] += a0;
    counters[kCand] += a1;
    counters[kMatchEntries] += a2;
    const long long t = static_cast<long long>(a2);
    total[0] = t;
    total[1] = ub[nt - 1] + tests[nt - 1];
    if (n_dev) {
      n_dev[0] = t < cap ? t : cap;
      if (t > cap) atomicOr(&err[kErrOverflow], 16);
    }
    total[2] = err[kErrOverflow];
  }
  if (mat) {
    // a small partition's [destination][block] counts: their exclusive scan and each destination's
    // total here (instead of a two-kernel device scan and a totals kernel)
    const int N = H * P;
    const int per = (N + 1023) / 1024;
    const int first = static_cast<int>(threadIdx.x) * per;
    // (up to kPerReg counts per thread — a W <= 8 partition — held in registers: their loads in flight
    // together and read once, not one dependent load per element and a second pass)
    constexpr int kPerReg = 16;
    int v[kPerReg];
    int loc = 0;
    if (per <= kPerReg) {
#pragma unroll
      for (int i = 0; i < kPerReg; ++i) v[i] = i < per && first + i < N ? mat[first + i] : 0;
#pragma unroll
      for (int i = 0; i < kPerReg; ++i) loc += v[i];
    } else {
      for (int i = 0; i < per && first + i < N; ++i) loc += mat[first + i];
    }
    const int inc = wave_incl_scan(loc);
    if (lane == kWave - 1) wsum[w] = inc;
    __syncthreads();
    int base = inc - loc;
    for (int x = 0; x < w; ++x) base += wsum[x];
    if (per <= kPerReg) {
#pragma unroll
      for (int i = 0; i < kPerReg; ++i) {
        if (i < per && first + i < N) off[first + i] = base;
        base += v[i];
      }
    } else {
      for (int i = 0; i < per && first + i < N; ++i) {
        off[first + i] = base;
        base += mat[first + i];
      }
    }
    __syncthreads();
    if (static_cast<int>(threadIdx.x) < H) {
      const long long k0 = static_cast<long long>(threadIdx.x) * P, k1 = k0 + P - 1;
      dtot[threadIdx.x] = static_cast<long long>(off[k1]) + mat[k1] - off[k0];
    }
  }
}

// pair tests of each tile: the sum of its positions' forward counts (an upper bound of its entries)
// wlo[w] = the first tile whose cost start (tile_ub[t] + t kTileCost, the exclusive cumulative cost)
// maps to wave w or later, cost scaled to nw waves: each tile writes the boundaries it crosses
__global__ __launch_bounds__(256) void k_wave_bounds(const long long* __restrict__ ub, const long long* __restrict__ tests,
                                                     int nt, int nw, int* __restrict__ wlo) {
  const long long total = ub[nt - 1] + tests[nt - 1] + static_cast<long long>(nt) * kTileCost;
  auto wave_of = [&](int t) -> int {
    const long long c = ub[t] + static_cast<long long>(t) * kTileCost;
    return total > 0 ? static_cast<int>(min(static_cast<long long>(nw - 1), c * nw / total)) : 0;
  };
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += gridDim.x * blockDim.x) {
    const int w = t == 0 ? 0 : wave_of(t);
    const int wp = t == 0 ? -1 : wave_of(t - 1);
    for (int x = wp + 1; x <= w; ++x) wlo[x] = t;
    if (t == nt - 1)
      for (int x = w + 1; x <= nw; ++x) wlo[x] = nt;
  }
}

__global__ __launch_bounds__(256) void k_tile_tests(const int* __restrict__ swin, int ni, long long* __restrict__ tests) {
  const int nt = (ni + kWave - 1) / kWave;
  const int lane = lane_id();
  for (int t = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < nt; t += (gridDim.x * blockDim.x) >> 6) {
    const int q = t * kWave + lane;
    int v = q < ni ? swin[q] : 0;
    v = wave_incl_scan(v);
    if (lane == kWave - 1) tests[t] = v;
  }
}

// pack each tile's entries from its upper-bound slot to its scanned offset (one wave per tile)
__global__ __launch_bounds__(256) void k_compact(const unsigned long long* __restrict__ src,
                                                 const long long* __restrict__ ub, const long long* __restrict__ off,
                                                 const long long* __restrict__ cnt, int nt,
                                                 unsigned long long* __restrict__ dst) {
  const int lane = lane_id();
  for (int t = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < nt; t += (gridDim.x * blockDim.x) >> 6) {
    const long long n = cnt[t], a = ub[t], b = off[t];
    for (long long k = lane; k < n; k += kWave) dst[b + k] = src[a + k];
  }
}

// ---- 3. pairs from the entries grouped by A ------------------------------------------------------
// Work item: a chunk of kChunk2 sorted entries; the runs (reads A) that start in it.  (Smaller chunks
// for a rank's small share measured slower: 112 vs 103 us mean, profiles/r05/r5l.)  Whole runs are
// taken a group of at most kStageE entries at a time (two per lane, in registers) and sorted by
// (run, B, i, j) with a wave-wide bitonic network: each read pair's entries become one segment, in
// the reference's row order.  Per segment (one lane each): I = its entry count unless two entries
// share a row (adjacent equal i) or a column (the segment's OR of column bits has fewer bits than
// entries) — then first-fit in the reference's order over the sorted segment (rows ascending, the
// lowest unused column, cluster.py:152-161).  A run longer than the stage is evaluated alone,
// streamed from HBM, through an LDS hash over its partners in partner partitions (pass k takes the
// partners with part(B) == k).
constexpr int kChunk2 = 512;               // a wave's work item: whole runs starting in it
constexpr int kStageE = 128;
constexpr int kHash2 = 128;
constexpr unsigned kEmpty = 0xFFFFFFFFu;
#ifndef FSLR_PAIR_EDGE_STAGE
#define FSLR_PAIR_EDGE_STAGE 256
#endif
constexpr int kPairEdgeStage = FSLR_PAIR_EDGE_STAGE;   // staged edges per wave (one atomic per flush)
static_assert(kPairEdgeStage >= kStageE, "a group's edges fit one flush");
// per-wave LDS shared by the two paths: the long-run hash (KEY, CNT: 4 B, RM, CM: 8 B per slot, the
// slot list) or the group's sorted keys, segment keys, column masks and heads
constexpr int kLongScr = kHash2 * (4 + 4 + 8 + 8) + 2 * (kPairLimit + kWave);
constexpr int kGroupScr = kStageE * (8 + 8 + 8) + 4 * (kStageE + 1);
constexpr int kScrWords = ((kLongScr > kGroupScr ? kLongScr : kGroupScr) + 15) / 16 * 2;   // 16-B rows

// lane ^ ST's value: DPP for strides 1 .. 8 (inside a 16-lane row: quad permutes, row shifts),
// ds_swizzle for 16 (inside 32 lanes), ds_bpermute for 32 — the short strides cost a VALU op, not an
// LDS round trip
template <int ST>
__device__ __forceinline__ unsigned xor_lane32(unsigned v, int lane) {
  if constexpr (ST == 1) {
    return static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0xB1, 0xF, 0xF, false));
  } else if constexpr (ST == 2) {
    return static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x4E, 0xF, 0xF, false));
  } else if constexpr (ST == 4 || ST == 8) {
    const int up = __builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x100 + ST, 0xF, 0xF, true);   // lane + ST
    const int dn = __builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x110 + ST, 0xF, 0xF, true);   // lane - ST
    return static_cast<unsigned>((lane & ST) ? dn : up);
  } else if constexpr (ST == 16) {
    return static_cast<unsigned>(__builtin_amdgcn_ds_swizzle(static_cast<int>(v), 0x401F));            // xor 16
  } else {
    return static_cast<unsigned>(__shfl_xor(static_cast<int>(v), ST));
  }
}

template <int ST>
__device__ __forceinline__ unsigned long long xor_lane(unsigned long long v, int lane) {
  const unsigned lo = xor_lane32<ST>(static_cast<unsigned>(v), lane);
  const unsigned hi = xor_lane32<ST>(static_cast<unsigned>(v >> 32), lane);
  return (static_cast<unsigned long long>(hi) << 32) | lo;
}

// one compare-exchange step of the bitonic network: keep the min (keep_min) or the max of the
// pair (lane, lane ^ ST)
template <int ST>
__device__ __forceinline__ unsigned long long bitonic_cx(unsigned long long v, bool keep_min, int lane) {
  const unsigned long long o = xor_lane<ST>(v, lane);
  return keep_min == (v < o) ? v : o;
}

// Bitonic sort of up to 128 keys, two per lane, element e = lane << 1 | slot (a: slot 0, b: slot 1):
// index bit 0 is in-lane (7 of the 28 stages exchange nothing), bits 1-4 are DPP lane exchanges and
// only bits 5 and 6 cross 16 lanes (3 LDS-permute stages instead of 5 with e = lane | slot << 6).  The network is a chain of 28 dependent stages, and a
// permute through LDS is its slowest link.  Sorted element e ends at lane e >> 1, slot e & 1.
template <int SIZE, int D>
__device__ __forceinline__ void bitonic_il_steps(unsigned long long& a, unsigned long long& b, int lane) {
  if constexpr (D >= 1) {
    const bool asc = ((lane << 1) & SIZE) == 0;
    if constexpr (D == 1) {
      const unsigned long long lo = a < b ? a : b, hi = a < b ? b : a;
      a = asc ? lo : hi;
      b = asc ? hi : lo;
    } else {
      const bool lower = (lane & (D >> 1)) == 0;
      a = bitonic_cx<D / 2>(a, lower == asc, lane);
      b = bitonic_cx<D / 2>(b, lower == asc, lane);
    }
    bitonic_il_steps<SIZE, D / 2>(a, b, lane);
  }
}

// ascending sort of N = 32, 64 or 128 elements in lanes [0, N / 2) (N < 128: lanes N / 2 .. 63 sort
// their own copies, which the caller discards): log2(N) (log2(N) + 1) / 2 dependent stages — 15 for
// 32 (all DPP), 21 for 64 (one ds_swizzle stride), 28 for 128 (three LDS permutes)
template <int N>
__device__ __forceinline__ void bitonic_il(unsigned long long& a, unsigned long long& b, int lane) {
  bitonic_il_steps<2, 1>(a, b, lane);
  bitonic_il_steps<4, 2>(a, b, lane);
  bitonic_il_steps<8, 4>(a, b, lane);
  bitonic_il_steps<16, 8>(a, b, lane);
  bitonic_il_steps<32, 16>(a, b, lane);
  if constexpr (N >= 64) bitonic_il_steps<64, 32>(a, b, lane);
  if constexpr (N >= 128) bitonic_il_steps<128, 64>(a, b, lane);
}

// group sort key: run (7 bits) << 39 | B << 14 | i << 7 | j; the segment key (run, B) is key >> 14
__device__ __forceinline__ unsigned long long group_key(unsigned long long e, int r) {
  return (static_cast<unsigned long long>(r) << 39) | (e & ((1ull << 39) - 1));
}

__global__ __launch_bounds__(kSwBlock) __attribute__((amdgpu_waves_per_eu(5))) void k_sweep_pairs(SweepArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned long long scr_all[kSwWaves][kScrWords];
  __shared__ int runa_all[kSwWaves][kStageE];                 // per run of the group: A | L_A << 25, edges formed
  __shared__ int runf_all[kSwWaves][kStageE];
  __shared__ uint2 rr_all[kSwWaves][kWave];                   // long runs' ordered path: row masks of one partner
  __shared__ unsigned long long es_all[kSwWaves][kPairEdgeStage];
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  unsigned long long* scr = scr_all[wv];
  // long-run path views
  unsigned* KEY = reinterpret_cast<unsigned*>(scr);           // B
  unsigned* CNT = KEY + kHash2;                               // entry count | L_B << 16 | conflict << 31
  uint2* RM = reinterpret_cast<uint2*>(CNT + kHash2);          // rows i of A used by the pair's entries
  uint2* CM = RM + kHash2;                                    // columns j of B
  unsigned short* MP = reinterpret_cast<unsigned short*>(CM + kHash2);
  // group path views
  unsigned long long* SK = scr;                               // the sorted keys
  unsigned long long* PK = SK + kStageE;                      // per segment: (run, B)
  unsigned long long* PJ = PK + kStageE;                      // per segment: OR of column bits
  int* PH = reinterpret_cast<int*>(PJ + kStageE);             // per segment: first position | row dup << 30
  int* RUNA = runa_all[wv];
  int* RUNF = runf_all[wv];
  uint2* RR = rr_all[wv];
  EdgeStageN<kPairEdgeStage> es{es_all[wv], 0};
  const EdgeOut eo{g.edges, g.edge_iu, g.edge_cap, &g.counters[kEdgeCount], g.parent};
  const int umax_v = g.umax[lane];
  const long long n = g.n_dev ? *g.n_dev : g.n_ent;
  const unsigned long long* E = g.ent_sorted;
  const unsigned char* RL = g.rlen8;
  const long long nchunks = (n + kChunk2 - 1) / kChunk2;
  const long long nw = static_cast<long long>(gridDim.x) * kSwWaves;
  const int wid = blockIdx.x * kSwWaves + wv;
  int w_maxfwd = 0;
  unsigned long long w_pairs = 0;
  auto a_at = [&](long long k) -> int {   // A of sorted entry k (wave-uniform, scalar cache)
    const_i32_ptr p = (const_i32_ptr)(E + k);
    return static_cast<int>(static_cast<unsigned>(p[1]) >> 7);
  };
  // first k in [k, lim) whose A differs from `a` (lim if none); lanes scan 64 entries per step
  auto next_run = [&](long long k, long long lim, int a) -> long long {
    for (; k < lim; k += kWave) {
      const long long t = k + lane;
      const bool diff = t < lim && entry_a(E[min(t, n - 1)]) != a;
      const unsigned long long m = __ballot(diff);
      if (m) return k + __builtin_ctzll(m);
    }
    return lim;
  };
  auto clear_hash = [&]() {
    for (int t = lane; t < kHash2; t += kWave) KEY[t] = kEmpty;
    wave_lds_sync();
  };
  // insert `key` (lanes with `mine`); returns the slot; isnew for the lane that created it
  auto insert = [&](bool mine, unsigned key, unsigned hseed, bool& isnew) -> int {
    unsigned h = (hseed * 2654435761u) >> 25;       // 7 bits: kHash2
    isnew = false;
    if (mine) {
      while (true) {
        unsigned cur = KEY[h];
        if (cur == kEmpty) {
          const unsigned old = atomicCAS(&KEY[h], kEmpty, key);
          if (old == kEmpty) { isnew = true; break; }
          cur = old;
        }
        if (cur == key) break;
        h = (h + 1) & (kHash2 - 1);
      }
    }
    return static_cast<int>(h);
  };
  // first-fit in the reference's order (cluster.py:152-161) from row masks in lanes i < LA
  auto ordered_I = [&](int LA) -> int {
    const uint2 rv = RR[lane];
    unsigned used_lo = 0u, used_hi = 0u;
    int Ic = 0;
    for (int ii = 0; ii < LA; ++ii) {
      const unsigned m_lo = static_cast<unsigned>(rdl(static_cast<int>(rv.x), ii)) & ~used_lo;
      const unsigned m_hi = static_cast<unsigned>(rdl(static_cast<int>(rv.y), ii)) & ~used_hi;
      if (m_lo) used_lo |= m_lo & (0u - m_lo);
      else if (m_hi) used_hi |= m_hi & (0u - m_hi);
      Ic += (m_lo | m_hi) != 0u;
    }
    return Ic;
  };
  // the pair's entry counts and masks (lanes with `mine`, slot h)
  auto record = [&](bool mine, int h, int i, int j) {
    if (mine) {
      const unsigned bi = 1u << (i & 31), bj = 1u << (j & 31);
      const unsigned oi = i < 32 ? atomicOr(&RM[h].x, bi) : atomicOr(&RM[h].y, bi);
      const unsigned oj = j < 32 ? atomicOr(&CM[h].x, bj) : atomicOr(&CM[h].y, bj);
      atomicAdd(&CNT[h], 1u);
      if ((oi & bi) | (oj & bj)) atomicOr(&CNT[h], 0x80000000u);
    }
  };

  // ---- a run longer than the stage: alone, streamed, in partner partitions ----
  auto long_run = [&](long long rs, long long re) {
    const int A = a_at(rs);
    FSLR_BOUND(rs, n);
    FSLR_BOUND(re - 1, n);
    FSLR_BOUND(A, g.n_reads);
    const int LA = RL[A];
    const long long len = re - rs;
    const int npass = len <= kPairLimit ? 1 : static_cast<int>((len + kPerPass - 1) / kPerPass);
#ifdef FSLR_PAIRS_HIST
    // measurement build: long runs' entries (45), their wave-steps over all partner passes (46), the
    // longest run (47)
    if (lane == 0) {
      atomicAdd(&g.counters[45], static_cast<unsigned long long>(len));
      atomicAdd(&g.counters[46], static_cast<unsigned long long>(npass) * ((len + kWave - 1) / kWave));
      atomicMax(&g.counters[47], static_cast<unsigned long long>(len));
    }
#endif
    int fwdA = 0;
    if (es.n > 0) es.flush(eo, lane);               // A's edges from an empty stage: one run (<= the stage)
    for (int pass = 0; pass < npass; ++pass) {
      clear_hash();
      int uniq = 0;
      bool full_any = false;
      for (long long b = rs; b < re; b += kWave) {
        const long long t = b + lane;
        const bool act = t < re;
        const unsigned long long e = act ? E[t] : 0ull;
        const int B = static_cast<int>((e >> 14) & kRankMask);
        const int i = static_cast<int>((e >> 7) & 127u), j = static_cast<int>(e & 127u);
        bool mine = act && (npass == 1 || part_of(B, npass) == pass);
        // insert while fewer than kPairLimit partners (+ 64 per step: at most kHash2 slots)
        const bool full = mine && uniq >= kPairLimit;
        full_any |= __ballot(full) != 0ull;
        mine = mine && !full;
        bool isnew;
        const int h = insert(mine, static_cast<unsigned>(B), static_cast<unsigned>(B), isnew);
        int lbn = 0;
        if (isnew) {
          CNT[h] = 0u;
          RM[h] = make_uint2(0u, 0u);
          CM[h] = make_uint2(0u, 0u);
          FSLR_BOUND(B, g.n_reads);
          lbn = RL[B];
        }
        const unsigned long long nm = __ballot(isnew);
        if (isnew) MP[uniq + mbcnt(nm)] = static_cast<unsigned short>(h);
        uniq += __popcll(nm);
        wave_lds_sync();
        record(mine, h, i, j);
        if (isnew) atomicOr(&CNT[h], static_cast<unsigned>(lbn) << 16);   // bits 16..22: L_B
      }
      if (full_any && lane == 0) atomicOr(g.err + kErrOverflow, 4);
      wave_lds_sync();
      for (int k0 = 0; k0 < uniq; k0 += kWave) {
        const bool act = k0 + lane < uniq;
        const int h = act ? static_cast<int>(MP[k0 + lane]) : 0;
        const int B = static_cast<int>(KEY[h]);
        const unsigned st = act ? CNT[h] : 0u;
        int I = static_cast<int>(st & 0xFFFFu);
        const int LB = static_cast<int>((st >> 16) & 127u);
        unsigned long long cm = __ballot(act && (st >> 31));
        while (cm) {
          const int c = __builtin_ctzll(cm);
          cm &= cm - 1;
          const int Bc = rdl(B, c);
          RR[lane] = make_uint2(0u, 0u);
          wave_lds_sync();
          for (long long b = rs; b < re; b += kWave) {
            const long long t = b + lane;
            const unsigned long long e = t < re ? E[t] : 0ull;
            if (t < re && static_cast<int>((e >> 14) & kRankMask) == Bc) {
              const int ii = static_cast<int>((e >> 7) & 127u), jj = static_cast<int>(e & 127u);
              if (jj < 32) atomicOr(&RR[ii].x, 1u << jj);
              else atomicOr(&RR[ii].y, 1u << (jj - 32));
            }
          }
          wave_lds_sync();
          const int Ic = ordered_I(LA);
          if (lane == c) I = Ic;
          wave_lds_sync();
        }
        const int U = LA + LB - I;
        const int um = __shfl(umax_v, max(I, 1) - 1);     // every lane reads (no && in front)
        const bool edge = act && I > 0 && U <= um;
        fwdA += es.put(eo, edge, A, B, I, U, lane);
        w_pairs += __popcll(__ballot(act));
      }
    }
    if (lane == 0) g.fwd[A] = fwdA;
    w_maxfwd = max(w_maxfwd, fwdA);
  };

  // ---- a run longer than the stage, bucketed (round 6): its partners hashed into P = ceil(len / 96)
  // buckets of at most kStageE entries — counted in LDS, scattered into the grouping's free buffer at the
  // run's own positions — and each bucket sorted by (B, i, j) and evaluated like a group (one run): two
  // streams over the run and P network sorts instead of one stream per 40-entry partner partition.
  // Returns false, having written nothing, when the run has more than 64 buckets or one bucket more than
  // kStageE entries (a pair of reads with that many matches): then the partition path above runs.
  auto long_run_buckets = [&](long long rs, long long re) -> bool {
    unsigned long long* S = g.pair_scr;
    const long long len = re - rs;
    const int P = static_cast<int>((len + 95) / 96);
    if (!S || P > kWave) return false;
    const int A = a_at(rs);
    FSLR_BOUND(A, g.n_reads);
    FSLR_BOUND(re - 1, n);
    auto bucket_of = [&](unsigned long long e) -> int {
      return static_cast<int>(((static_cast<unsigned>((e >> 14) & kRankMask) * 0x9E3779B1u) >> 8) % static_cast<unsigned>(P));
    };
    int* BC = RUNA;                                 // per bucket: entry count, then the scatter cursor
    int* BO = RUNF;
    wave_lds_sync();
    if (lane < P) BC[lane] = 0;
    wave_lds_sync();
    for (long long b = rs; b < re; b += kWave) {
      const long long t = b + lane;
      if (t < re) atomicAdd(&BC[bucket_of(E[t])], 1);
    }
    wave_lds_sync();
    const int cnt = lane < P ? BC[lane] : 0;
    int cmax = cnt;
    for (int o = 32; o > 0; o >>= 1) cmax = max(cmax, __shfl_xor(cmax, o));
    if (cmax > kStageE) return false;
    const int off = wave_incl_scan(cnt) - cnt;
    if (lane < P) BO[lane] = off;
    wave_lds_sync();
    for (long long b = rs; b < re; b += kWave) {
      const long long t = b + lane;
      if (t < re) {
        const unsigned long long e = E[t];
        const int p = atomicAdd(&BO[bucket_of(e)], 1);
        FSLR_BOUND(p, len);
        S[rs + p] = e;
      }
    }
    // the wave reads its own scattered entries back: its stores complete (no other CU touches these
    // positions, so no L1 on another CU can hold them and the workgroup scope is enough)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const int LA = RL[A];
#ifdef FSLR_PAIRS_HIST
    if (lane == 0) {                                // measurement build: bucketed runs (40), their entries (41)
      atomicAdd(&g.counters[40], 1ull);
      atomicAdd(&g.counters[41], static_cast<unsigned long long>(len));
    }
#endif
    int fwdA = 0;
    if (es.n > 0) es.flush(eo, lane);               // A's edges from an empty stage: one run (<= the stage)
    for (int kb = 0; kb < P; ++kb) {
      const int bo = rdl(off, kb), bc = rdl(cnt, kb);
      if (bc == 0) continue;
      const unsigned long long* Sb = S + rs + bo;
      const bool v0 = lane < bc, v1 = lane + kWave < bc;
      unsigned long long k0 = v0 ? (Sb[lane] & ((1ull << 39) - 1)) << 7 : ~0ull;
      unsigned long long k1 = v1 ? (Sb[kWave + lane] & ((1ull << 39) - 1)) << 7 : ~0ull;
      if (bc > kWave) {
        bitonic_il<128>(k0, k1, lane);
      } else if (bc > kWave / 2) {
        k1 = __shfl(k0, (lane + kWave / 2) & (kWave - 1));
        bitonic_il<64>(k0, k1, lane);
        if (lane >= kWave / 2) k0 = k1 = ~0ull;
      } else {
        k1 = __shfl(k0, (lane + kWave / 4) & (kWave - 1));
        bitonic_il<32>(k0, k1, lane);
        if (lane >= kWave / 4) k0 = k1 = ~0ull;
      }
      wave_lds_sync();                              // the previous bucket's reads are done
      reinterpret_cast<ulonglong2*>(SK)[lane] = make_ulonglong2(k0, k1);
      wave_lds_sync();
      k0 = SK[lane];
      k1 = SK[lane + kWave];
      const unsigned long long q0 = __shfl_up(k0, 1);
      const unsigned long long k0_63 = __shfl(k0, kWave - 1);
      const unsigned long long w1 = __shfl_up(k1, 1);
      const unsigned long long q1 = lane > 0 ? w1 : k0_63;
      // segments = partners B (key >> 21); a row repeated inside a segment sits next to itself
      const bool s0 = v0 && (lane == 0 || (k0 >> 21) != (q0 >> 21));
      const bool s1 = v1 && (k1 >> 21) != (q1 >> 21);
      const bool d0 = v0 && !s0 && (k0 >> 14) == (q0 >> 14);
      const bool d1 = v1 && !s1 && (k1 >> 14) == (q1 >> 14);
      int lb0 = 0, lb1 = 0;
      if (s0) lb0 = RL[(k0 >> 21) & kRankMask];
      if (s1) lb1 = RL[(k1 >> 21) & kRankMask];
      const unsigned long long S0 = __ballot(s0), S1 = __ballot(s1);
      const int ns0 = __popcll(S0), nseg = ns0 + __popcll(S1);
      const int g0 = __popcll(S0 & upto(lane)) - 1;
      const int g1 = ns0 + __popcll(S1 & upto(lane)) - 1;
      wave_lds_sync();
      if (s0) {
        PK[g0] = (k0 >> 21) | (static_cast<unsigned long long>(lb0) << 32);
        PJ[g0] = 0ull;
        PH[g0] = lane;
      }
      if (s1) {
        PK[g1] = (k1 >> 21) | (static_cast<unsigned long long>(lb1) << 32);
        PJ[g1] = 0ull;
        PH[g1] = lane + kWave;
      }
      if (lane == 0) PH[nseg] = bc;
      wave_lds_sync();
      if (v0) atomicOr(&PJ[g0], 1ull << ((k0 >> 7) & 63u));
      if (v1) atomicOr(&PJ[g1], 1ull << ((k1 >> 7) & 63u));
      if (d0) atomicOr(&PH[g0], 1 << 30);
      if (d1) atomicOr(&PH[g1], 1 << 30);
      wave_lds_sync();
      for (int k0s = 0; k0s < nseg; k0s += kWave) {
        const int p = k0s + lane;
        const bool act = p < nseg;
        int I = 0, B = 0, LB = 0;
        if (act) {
          const int hp = PH[p];
          const int h = hp & 0x3FFFFFFF, he = PH[p + 1] & 0x3FFFFFFF;
          const unsigned long long pk = PK[p];
          B = static_cast<int>(pk & kRankMask);
          LB = static_cast<int>(pk >> 32);
          I = he - h;
          if ((hp >> 30) || __popcll(PJ[p]) < I) {
            // a shared row or column: first-fit over the segment, rows ascending, lowest free column
            unsigned long long used = 0ull;
            int row = -1, Ic = 0;
            for (int q = h; q < he; ++q) {
              const unsigned long long key = SK[q];
              const int i = static_cast<int>((key >> 14) & 127u), j = static_cast<int>((key >> 7) & 63u);
              if (i == row) continue;
              if (!((used >> j) & 1ull)) {
                used |= 1ull << j;
                ++Ic;
                row = i;
              }
            }
            I = Ic;
          }
        }
        const int U = LA + LB - I;
        const int um = __shfl(umax_v, max(I, 1) - 1);   // every lane reads (no && in front)
        const bool edge = act && I > 0 && U <= um;
        fwdA += es.put(eo, edge, A, B, I, U, lane);
        w_pairs += __popcll(__ballot(act));
      }
    }
    if (lane == 0) g.fwd[A] = fwdA;
    w_maxfwd = max(w_maxfwd, fwdA);
    return true;
  };

  // the window of (up to) kStageE entries at s, and (lane 0) the entry after it (~0: none).  Vector
  // loads only: a scalar load in flight would hold every LDS wait (lgkmcnt) of the group behind it
  auto load_window = [&](long long s, unsigned long long& w0, unsigned long long& w1, unsigned long long& wn) {
    const int lim = static_cast<int>(min(static_cast<long long>(kStageE), n - s));
    w0 = lane < lim ? E[s + lane] : ~0ull;
    w1 = lane + kWave < lim ? E[s + kWave + lane] : ~0ull;
    wn = lane == 0 && s + lim < n ? E[s + lim] : ~0ull;
  };
#ifdef FSLR_PAIRS_HIST
  // measurement build: wave-clock sums per phase (counters 68..73: window and heads, sort, segment
  // setup, segment evaluation, tail, long runs)
  unsigned long long ck[6] = {0, 0, 0, 0, 0, 0};
  long long tck = clock64();
#define FSLR_PCK(k) do { const long long t_ = clock64(); ck[k] += t_ - tck; tck = t_; } while (0)
#else
#define FSLR_PCK(k) do { } while (0)
#endif
  for (long long c = wid; c < nchunks; c += nw) {
    const long long c0 = c * kChunk2, c1 = min(c0 + kChunk2, n);
    long long s = c0;
    if (s > 0) s = next_run(s, c1, a_at(s - 1));       // the run in progress belongs to the previous chunk
    unsigned long long e0 = ~0ull, e1 = ~0ull, en = ~0ull;
    if (s < c1) load_window(s, e0, e1, en);
    while (s < c1) {
      // the window [s, s + lim): two entries per lane, neighbours by shuffles
      const int lim = static_cast<int>(min(static_cast<long long>(kStageE), n - s));
      const unsigned long long en0 = static_cast<unsigned long long>(
          static_cast<unsigned>(__builtin_amdgcn_readfirstlane(static_cast<int>(en >> 32)))) << 32;
      const bool last_done = s + lim >= n ||
                             entry_a(en0) != entry_a(lim <= kWave ? __shfl(e0, lim - 1) : __shfl(e1, lim - 1 - kWave));
      // every lane shuffles (a source lane outside EXEC would read as 0), then selects
      const unsigned long long p0 = __shfl_up(e0, 1);
      const unsigned long long e0_63 = __shfl(e0, kWave - 1);
      const unsigned long long u1 = __shfl_up(e1, 1);
      const unsigned long long p1 = lane > 0 ? u1 : e0_63;
      const bool h0 = lane < lim && (lane == 0 || entry_a(e0) != entry_a(p0));
      const bool h1 = lane + kWave < lim && entry_a(e1) != entry_a(p1);
      const unsigned long long H0 = __ballot(h0), H1 = __ballot(h1);
      // owned heads: runs starting before c1
      const long long own = min(c1 - s, static_cast<long long>(lim));
      const unsigned long long O0 = own >= kWave ? ~0ull : ((1ull << own) - 1);
      const unsigned long long O1 = own <= kWave ? 0ull : own >= 2 * kWave ? ~0ull : ((1ull << (own - kWave)) - 1);
      const unsigned long long OH0 = H0 & O0, OH1 = H1 & O1;
      const int h_top = OH1 ? kWave + 63 - __builtin_clzll(OH1) : 63 - __builtin_clzll(OH0);   // OH0 has bit 0
      // the next head after h_top (owned or not) ends its run
      const unsigned long long A0 = h_top >= kWave ? 0ull : H0 & above(h_top);
      const unsigned long long A1 = h_top >= kWave ? H1 & above(h_top - kWave) : H1;
      int gend;
      if (A0) gend = __builtin_ctzll(A0);
      else if (A1) gend = kWave + __builtin_ctzll(A1);
      else gend = last_done ? lim : h_top;
#ifdef FSLR_PAIRS_HIST
      // measurement build: groups by size (8-entry bins, counters 48..63), long runs (42), the groups'
      // read pairs (43) and runs (44)
      if (lane == 0) atomicAdd(gend ? &g.counters[kSecBase + ((gend - 1) >> 3)] : &g.counters[42], 1ull);
#endif
      FSLR_PCK(0);
      if (gend == 0) {
        // the run at s does not fit the stage: alone
        const long long re = next_run(s + lim, n, entry_a(__shfl(e0, 0)));
#ifndef FSLR_PAIRS_NO_BUCKETS
        if (!long_run_buckets(s, re))
#endif
          long_run(s, re);
        FSLR_PCK(5);
        s = re;
        if (s < c1) load_window(s, e0, e1, en);
        continue;
      }
      // ---- the group [s, s + gend): whole runs, sorted by (run, B, i, j) ----
      const int r0 = __popcll(H0 & upto(lane)) - 1;                 // run (in the group) of entry lane
      const int r1 = __popcll(H0) + __popcll(H1 & upto(lane)) - 1;
      const bool v0 = lane < gend, v1 = lane + kWave < gend;
      const bool hv0 = h0 && v0, hv1 = h1 && v1;
      int la0 = 0, la1 = 0;
      if (hv0) FSLR_BOUND(entry_a(e0), g.n_reads);
      if (hv1) FSLR_BOUND(entry_a(e1), g.n_reads);
      if (hv0) la0 = RL[entry_a(e0)];                              // in flight during the sort
      if (hv1) la1 = RL[entry_a(e1)];
      unsigned long long k0 = v0 ? group_key(e0, r0) : ~0ull;
      unsigned long long k1 = v1 ? group_key(e1, r1) : ~0ull;
      // the group's network: the smallest of 32 / 64 / 128 elements that holds it (a group of <= 64
      // entries sits in k0; its upper half moves to lanes [0, 32) as the second slot)
      if (gend > kWave) {
        bitonic_il<128>(k0, k1, lane);
      } else if (gend > kWave / 2) {
        k1 = __shfl(k0, (lane + kWave / 2) & (kWave - 1));
        bitonic_il<64>(k0, k1, lane);
        if (lane >= kWave / 2) k0 = k1 = ~0ull;
      } else {
        k1 = __shfl(k0, (lane + kWave / 4) & (kWave - 1));
        bitonic_il<32>(k0, k1, lane);
        if (lane >= kWave / 4) k0 = k1 = ~0ull;
      }
      FSLR_PCK(1);
      // back to position p at lane p (k0) / p - 64 (k1) through the group's key array
      wave_lds_sync();                                             // the previous group's reads are done
      reinterpret_cast<ulonglong2*>(SK)[lane] = make_ulonglong2(k0, k1);
      wave_lds_sync();
      k0 = SK[lane];                                               // positions [0, gend) hold the group
      k1 = SK[lane + kWave];
      const unsigned long long q0 = __shfl_up(k0, 1);
      const unsigned long long k0_63 = __shfl(k0, kWave - 1);
      const unsigned long long w1 = __shfl_up(k1, 1);
      const unsigned long long q1 = lane > 0 ? w1 : k0_63;
      // segments = read pairs (run, B); a row repeated inside a segment sits next to itself
      const bool s0 = v0 && (lane == 0 || (k0 >> 14) != (q0 >> 14));
      const bool s1 = v1 && (k1 >> 14) != (q1 >> 14);
      const bool d0 = v0 && !s0 && (k0 >> 7) == (q0 >> 7);
      const bool d1 = v1 && !s1 && (k1 >> 7) == (q1 >> 7);
      int lb0 = 0, lb1 = 0;                                        // L_B of each segment, gathered by its head
      if (s0) FSLR_BOUND((k0 >> 14) & kRankMask, g.n_reads);
      if (s1) FSLR_BOUND((k1 >> 14) & kRankMask, g.n_reads);
      if (s0) lb0 = RL[(k0 >> 14) & kRankMask];
      if (s1) lb1 = RL[(k1 >> 14) & kRankMask];
      // the next window, in flight while this group is evaluated
      const long long sn = s + gend;
      unsigned long long n0 = ~0ull, n1 = ~0ull, nn = ~0ull;
      if (sn < c1) load_window(sn, n0, n1, nn);
      const unsigned long long S0 = __ballot(s0), S1 = __ballot(s1);
      const int ns0 = __popcll(S0), nseg = ns0 + __popcll(S1);
#ifdef FSLR_PAIRS_HIST
      if (lane == 0) {
        atomicAdd(&g.counters[43], static_cast<unsigned long long>(nseg));
        atomicAdd(&g.counters[44], static_cast<unsigned long long>(__popcll(H0 & (gend >= kWave ? ~0ull : (1ull << gend) - 1)) +
                                                                  __popcll(H1 & (gend <= kWave ? 0ull : gend >= 2 * kWave ? ~0ull : (1ull << (gend - kWave)) - 1))));
      }
#endif
      const int g0 = __popcll(S0 & upto(lane)) - 1;
      const int g1 = ns0 + __popcll(S1 & upto(lane)) - 1;
      wave_lds_sync();                                             // the previous group's reads are done
      if (hv0) {
        RUNA[r0] = static_cast<int>(static_cast<unsigned>(entry_a(e0)) | static_cast<unsigned>(la0) << 25);
        RUNF[r0] = 0;
      }
      if (hv1) {
        RUNA[r1] = static_cast<int>(static_cast<unsigned>(entry_a(e1)) | static_cast<unsigned>(la1) << 25);
        RUNF[r1] = 0;
      }
      if (s0) {
        PK[g0] = (k0 >> 14) | (static_cast<unsigned long long>(lb0) << 32);
        PJ[g0] = 0ull;
        PH[g0] = lane;
      }
      if (s1) {
        PK[g1] = (k1 >> 14) | (static_cast<unsigned long long>(lb1) << 32);
        PJ[g1] = 0ull;
        PH[g1] = lane + kWave;
      }
      if (lane == 0) PH[nseg] = gend;
      wave_lds_sync();
      if (v0) atomicOr(&PJ[g0], 1ull << (k0 & 63u));
      if (v1) atomicOr(&PJ[g1], 1ull << (k1 & 63u));
      if (d0) atomicOr(&PH[g0], 1 << 30);
      if (d1) atomicOr(&PH[g1], 1 << 30);
      wave_lds_sync();
      // the group's edges (at most one per segment) go out in one flush: each read's forward edges stay
      // one run of the edge list (the edge cap's replay walks those runs)
      FSLR_PCK(2);
      if (es.n + nseg > kPairEdgeStage) es.flush(eo, lane);
      for (int k0s = 0; k0s < nseg; k0s += kWave) {
        const int p = k0s + lane;
        const bool act = p < nseg;
        int I = 0, r = 0, B = 0, LB = 0;
        if (act) {
          const int hp = PH[p];
          const int h = hp & 0x3FFFFFFF, he = PH[p + 1] & 0x3FFFFFFF;
          const unsigned long long pk = PK[p];
          r = static_cast<int>((pk >> 25) & 127u);
          B = static_cast<int>(pk & kRankMask);
          LB = static_cast<int>(pk >> 32);
          I = he - h;
          if ((hp >> 30) || __popcll(PJ[p]) < I) {
            // a shared row or column: first-fit over the segment, rows ascending, lowest free column
            unsigned long long used = 0ull;
            int row = -1, Ic = 0;
            for (int k = h; k < he; ++k) {
              const unsigned long long key = SK[k];
              const int i = static_cast<int>((key >> 7) & 127u), j = static_cast<int>(key & 63u);
              if (i == row) continue;                              // this row already matched
              if (!((used >> j) & 1ull)) {
                used |= 1ull << j;
                ++Ic;
                row = i;
              }
            }
            I = Ic;
          }
        }
        const int ra = act ? RUNA[r] : 0;
        const int A = static_cast<int>(static_cast<unsigned>(ra) & kRankMask);
        const int U = static_cast<int>(static_cast<unsigned>(ra) >> 25) + LB - I;
        const int um = __shfl(umax_v, max(I, 1) - 1);     // every lane reads (no && in front)
        const bool edge = act && I > 0 && U <= um;
        es.put(eo, edge, A, B, I, U, lane);
        if (edge) atomicAdd(&RUNF[r], 1);
        w_pairs += __popcll(__ballot(act));
      }
      FSLR_PCK(3);
      wave_lds_sync();
      if (hv0) {
        const int f = RUNF[r0];
        g.fwd[entry_a(e0)] = f;
        w_maxfwd = max(w_maxfwd, f);
      }
      if (hv1) {
        const int f = RUNF[r1];
        g.fwd[entry_a(e1)] = f;
        w_maxfwd = max(w_maxfwd, f);
      }
      s = sn;
      e0 = n0;
      e1 = n1;
      en = nn;
      FSLR_PCK(4);
    }
  }
#ifdef FSLR_PAIRS_HIST
  if (lane == 0)
    for (int k = 0; k < 6; ++k) atomicAdd(&g.counters[68 + k], ck[k]);
#endif
#undef FSLR_PCK
  if (es.n > 0) es.flush(eo, lane);
  // statistics: plain stores into this wave's slots (field 2: matched pairs, field 3: max fwd)
  for (int o = 32; o > 0; o >>= 1) w_maxfwd = max(w_maxfwd, __shfl_xor(w_maxfwd, o));
  const unsigned long long f = lane == 2 ? w_pairs : static_cast<unsigned long long>(w_maxfwd);
  if (lane == 2 || lane == 3) g.wstat[static_cast<long long>(wid) * kWsFields + lane] = f;
}

// ---- 2. grouping by A: a two-level counting sort ---------------------------------------------------
// One GPU (mode 2): the sweep already counted its entries per coarse bucket (sweep_coarse_hist), so
// the grouping is one scan, k_sweep_scatter and k_msd_pass2r (group_by_a's first branch).  The
// passes below serve the rest: the two-pass fallback (mode 0), the caller's entries of
// fslr_sweep_evaluate (mode 3) and the multi-GPU partition (kMod).
// Pass 1 scatters the entries into H = 2^hb buckets of A's high bits with per-block LDS histograms,
// one scan over the [bucket][block] counts and LDS cursors; pass 2 groups each bucket by A's low bits
// in one workgroup (LDS histogram and cursors; the bucket, a few thousand entries, stays in L2
// between its two reads).  A read's entries arrive in runs (the sweep emits a position's partners
// together), so each wave adds one run's length with one atomic from the run's first lane.  Reads
// come out in ascending order (the union-find over the edges k_sweep_pairs writes in that order keeps
// its locality); inside a run the order is free (k_sweep_pairs hashes the partners).
// Two reads and one write per pass; pass 1 reads the sweep's upper-bound tile slots (no packing).
constexpr int kMsdMaxBlocks = 1024;       // pass-1 workgroups (at most)
#ifndef FSLR_MSD_THREADS
#define FSLR_MSD_THREADS 1024
#endif
#ifndef FSLR_MSD_HBMAX
#define FSLR_MSD_HBMAX 13
#endif
#ifndef FSLR_MSD_UNROLL
#define FSLR_MSD_UNROLL 8
#endif
constexpr int kMsdThreads = FSLR_MSD_THREADS;
constexpr int kMsdMaxH = 16384;            // buckets (LDS histogram of pass 1)
constexpr int kMsdMaxLo = 4096;            // in-bucket bins (LDS histogram of pass 2)
constexpr int kGrpInts = 2 * (1 << 22);    // [bucket][block] counts and their scan (H P <= 2^22)

constexpr int kMsdUnroll = FSLR_MSD_UNROLL;  // entries loaded per lane before their atomics

// kTiles: entries of tile t at src[ub[t] .. ub[t] + cnt[t]) (slots at or beyond n, the buffer's size,
// are not read: an overflowed sweep's result is discarded by the caller); else dense src[0, n) in
// contiguous block chunks.  kScatter = false: histogram.
// kMod: bucket (A >> lo_bits) % H (the multi-GPU destination of fslr_sweep_partition) instead of
// A >> lo_bits; scattered entries at positions >= cap are dropped (the caller sees the totals).
template <bool kTiles, bool kScatter, bool kMod = false>
__global__ __launch_bounds__(kMsdThreads) void k_msd_pass1(const unsigned long long* __restrict__ src, long long n,
                                                           const long long* __restrict__ ub,
                                                           const long long* __restrict__ cnt, int nt,
                                                           int lo_bits, int H, int* __restrict__ mat,
                                                           unsigned long long* __restrict__ dst,
                                                           long long cap = 0x7FFFFFFFFFFFFFFFll) {
  __shared__ int hist[kMsdMaxH];
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1), w = tid >> 6;
  const int P = gridDim.x;
  for (int i = tid; i < H; i += kMsdThreads) hist[i] = kScatter ? mat[i * P + blockIdx.x] : 0;
  __syncthreads();
  // a span [a, a + c) of consecutive entries: kMsdUnroll wave-loads in flight, then their runs
  auto span = [&](long long a, long long c) {
    for (long long k0 = 0; k0 < c; k0 += kMsdUnroll * kWave) {
      unsigned long long v[kMsdUnroll];
#pragma unroll
      for (int u = 0; u < kMsdUnroll; ++u) {
        const long long k = k0 + u * kWave + lane;
        v[u] = k < c ? src[a + k] : 0ull;
      }
#pragma unroll
      for (int u = 0; u < kMsdUnroll; ++u) {
        const long long k = k0 + u * kWave + lane;
        if (k0 + u * kWave >= c) break;                     // wave-uniform
        const bool act = k < c;
        const unsigned a_hi = static_cast<unsigned>(v[u] >> 39) >> lo_bits;
        const int d = static_cast<int>(kMod ? a_hi % static_cast<unsigned>(H) : a_hi);
        if (kScatter) {
          const int p = run_add<true>(hist, d, act, lane);
          if (act && p < cap) dst[p] = v[u];
        } else {
          run_add<false>(hist, d, act, lane);
        }
      }
    }
  };
  if (kTiles) {
    // groups of G consecutive tiles per wave (G <= 64, about one group per wave of the grid): lane l
    // holds tile g G + l's count and slot; the group's entries are walked as one dense range of
    // kMsdUnroll x 64 entries per step, each lane finding its tile by a binary search over the lanes
    const int nwave = P * (kMsdThreads / kWave);
    const int G = max(1, min(kWave, (nt + nwave - 1) / nwave));
    const int ngroups = (nt + G - 1) / G;
    for (int g = blockIdx.x * (kMsdThreads / kWave) + w; g < ngroups; g += nwave) {
      const int t = g * G + lane;
      const bool tv = lane < G && t < nt;
      const int c = tv ? static_cast<int>(cnt[t]) : 0;
      const long long u0 = tv ? ub[t] : 0;
      const int inc = wave_incl_scan(c);
      const int exc = inc - c;
      const int T = rdl(inc, kWave - 1);
      for (int k0 = 0; k0 < T; k0 += kMsdUnroll * kWave) {
        unsigned long long v[kMsdUnroll];
#pragma unroll
        for (int q = 0; q < kMsdUnroll; ++q) {
          const int kc = k0 + q * kWave;                    // chunk start (wave-uniform)
          const int k = kc + lane;
          // lane k's tile: the tile holding the chunk start, then the tiles starting inside the
          // chunk (usually 0-2 of them; a binary search over the lanes when there are many)
          int j = 63 - __builtin_clzll(__ballot(c > 0 && exc <= kc) | 1ull);
          const unsigned long long st = __ballot(c > 0 && exc > kc && exc < kc + kWave);
          if (__popcll(st) <= 4) {
            for (unsigned long long m = st; m; m &= m - 1) {
              const int jj = __builtin_ctzll(m);
              if (k >= rdl(exc, jj)) j = jj;
            }
          } else {
            int lo = 0, hi = kWave - 1;                     // largest lane j with exc[j] <= k
#pragma unroll
            for (int it = 0; it < 6; ++it) {
              const int mid = (lo + hi + 1) >> 1;
              if (__shfl(exc, mid) <= k) lo = mid; else hi = mid - 1;
            }
            j = lo;
          }
          const long long at = __shfl(u0, j) + (k - __shfl(exc, j));
          v[q] = k < T && at >= 0 && at < n ? src[at] : 0ull;   // n: the slot buffer's size
        }
#pragma unroll
        for (int q = 0; q < kMsdUnroll; ++q) {
          if (k0 + q * kWave >= T) break;                   // wave-uniform
          const bool act = k0 + q * kWave + lane < T;
          const unsigned a_hi = static_cast<unsigned>(v[q] >> 39) >> lo_bits;
          const int d = static_cast<int>(kMod ? a_hi % static_cast<unsigned>(H) : a_hi);
          if (kScatter) {
            const int p = run_add<true>(hist, d, act, lane);
            if (act && p < cap) dst[p] = v[q];
          } else {
            run_add<false>(hist, d, act, lane);
          }
        }
      }
    }
  } else {
    const long long chunk = (n + P - 1) / P;
    const long long b0 = blockIdx.x * chunk, b1 = min(n, b0 + chunk);
    // the block's chunk in wave-sized spans of 4 x 64 entries, dealt to its waves
    const long long step = kMsdUnroll * kWave;
    for (long long a = b0 + w * step; a < b1; a += (kMsdThreads / kWave) * step) span(a, min(step, b1 - a));
  }
  if (!kScatter) {
    __syncthreads();
    for (int i = tid; i < H; i += kMsdThreads) mat[i * P + blockIdx.x] = hist[i];
  }
}

// one workgroup per bucket: group [off[b P], off[(b + 1) P]) by the low lo_bits of A into dst
// (kBins >= 2^lo_bits LDS bins: 4096 for the counted grouping, 16384 for the sweep's coarse buckets
// of an input beyond 2^22 reads)
template <int kBins>
__global__ __launch_bounds__(256) void k_msd_pass2(const unsigned long long* __restrict__ src, long long n_host,
                                                   const long long* __restrict__ n_dev,
                                                   const int* __restrict__ off, int P, int H, int hb, int lo_bits,
                                                   unsigned long long* __restrict__ dst) {
  const long long n = n_dev ? *n_dev : n_host;
  __shared__ int hist[kBins];
  __shared__ int wsum[4];
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1), w = tid >> 6;
  const int nb = 1 << lo_bits;
  const int b = blockIdx.x;
  const long long s = min(static_cast<long long>(off[static_cast<long long>(b) * P]), n);
  const long long e = b + 1 < H ? min(static_cast<long long>(off[static_cast<long long>(b + 1) * P]), n) : n;
  if (e - s <= 1) {
    if (tid == 0 && e > s) dst[s] = src[s];
    return;
  }
  for (int i = tid; i < nb; i += 256) hist[i] = 0;
  __syncthreads();
  const unsigned mask = static_cast<unsigned>(nb - 1);
  auto key_of = [&](unsigned long long v) { return static_cast<int>(static_cast<unsigned>(v >> 39) & mask); };
  // each wave takes spans of 4 x 64 consecutive entries, loads first (runs stay on adjacent lanes)
  constexpr int kU2 = 4;
  for (long long a = s + w * (kU2 * kWave); a < e; a += 4 * kU2 * kWave) {
    int kv[kU2];
#pragma unroll
    for (int q = 0; q < kU2; ++q) {
      const long long k = a + q * kWave + lane;
      kv[q] = k < e ? key_of(src[k]) : 0;
    }
#pragma unroll
    for (int q = 0; q < kU2; ++q) {
      if (a + q * kWave >= e) break;
      run_add<false>(hist, kv[q], a + q * kWave + lane < e, lane);
    }
  }
  __syncthreads();
  // exclusive scan of hist: each thread owns a contiguous run of per = nb / 256 bins (or one bin)
  const int per = nb >= 256 ? nb / 256 : 1;
  const int first = tid * per;
  int loc = 0;
  if (first < nb)
    for (int i = 0; i < per; ++i) loc += hist[first + i];
  const int inc = wave_incl_scan(loc);
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int base = inc - loc;
  for (int x = 0; x < w; ++x) base += wsum[x];
  __syncthreads();
  if (first < nb) {
    int run = static_cast<int>(s) + base;          // positions fit 31 bits (n < 2^31)
    for (int i = 0; i < per; ++i) {
      const int c = hist[first + i];
      hist[first + i] = run;
      run += c;
    }
  }
  __syncthreads();
  for (long long a = s + w * (kU2 * kWave); a < e; a += 4 * kU2 * kWave) {
    unsigned long long v[kU2];
#pragma unroll
    for (int q = 0; q < kU2; ++q) {
      const long long k = a + q * kWave + lane;
      v[q] = k < e ? src[k] : 0ull;
    }
#pragma unroll
    for (int q = 0; q < kU2; ++q) {
      if (a + q * kWave >= e) break;
      const bool act = a + q * kWave + lane < e;
      const int p = run_add<true>(hist, act ? key_of(v[q]) : 0, act, lane);
      if (act) dst[p] = v[q];
    }
  }
}

// k_msd_pass2 for the sweep's coarse buckets (~16K entries at 1M reads): 1024 threads, the first
// kR x 1024 entries of the bucket held in registers between the histogram and the scatter (one HBM
// read instead of two); the rest, if any, read twice.
constexpr int kP2Threads = 1024;
template <int kBins, int kR>
__global__ __launch_bounds__(kP2Threads) void k_msd_pass2r(const unsigned long long* __restrict__ src, long long n_host,
                                                           const long long* __restrict__ n_dev,
                                                           const int* __restrict__ off, int P, int H, int lo_bits,
                                                           unsigned long long* __restrict__ dst) {
  const long long n = n_dev ? *n_dev : n_host;
  __shared__ int hist[kBins];
  __shared__ int wsum[kP2Threads / kWave];
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1), w = tid >> 6;
  const int nb = 1 << lo_bits;
  const int b = blockIdx.x;
  const long long s = min(static_cast<long long>(off[static_cast<long long>(b) * P]), n);
  const long long e = b + 1 < H ? min(static_cast<long long>(off[static_cast<long long>(b + 1) * P]), n) : n;
  if (e - s <= 1) {
    if (tid == 0 && e > s) dst[s] = src[s];
    return;
  }
  for (int i = tid; i < nb; i += kP2Threads) hist[i] = 0;
  const unsigned mask = static_cast<unsigned>(nb - 1);
  auto key_of = [&](unsigned long long v) { return static_cast<int>(static_cast<unsigned>(v >> 39) & mask); };
  unsigned long long v[kR];
#pragma unroll
  for (int q = 0; q < kR; ++q) {
    const long long k = s + static_cast<long long>(q) * kP2Threads + tid;
    v[q] = k < e ? src[k] : 0ull;
  }
  __syncthreads();
  // a wave's lanes hold consecutive entries: a run of one read adds with one atomic
#pragma unroll
  for (int q = 0; q < kR; ++q) {
    const long long k0 = s + static_cast<long long>(q) * kP2Threads + w * kWave;
    if (k0 >= e) break;                                   // wave-uniform
    run_add<false>(hist, key_of(v[q]), k0 + lane < e, lane);
  }
  for (long long k0 = s + static_cast<long long>(kR) * kP2Threads + w * kWave; k0 < e; k0 += kP2Threads) {
    const bool act = k0 + lane < e;
    run_add<false>(hist, act ? key_of(src[k0 + lane]) : 0, act, lane);
  }
  __syncthreads();
  // exclusive scan of hist: each thread owns a contiguous run of per = nb / 1024 bins (or one bin)
  const int per = nb >= kP2Threads ? nb / kP2Threads : 1;
  const int first = tid * per;
  int loc = 0;
  if (first < nb)
    for (int i = 0; i < per; ++i) loc += hist[first + i];
  const int inc = wave_incl_scan(loc);
  if (lane == kWave - 1) wsum[w] = inc;
  __syncthreads();
  int base = inc - loc;
  for (int x = 0; x < w; ++x) base += wsum[x];
  if (first < nb) {
    int run = static_cast<int>(s) + base;                 // positions fit 31 bits (n < 2^31)
    for (int i = 0; i < per; ++i) {
      const int c = hist[first + i];
      hist[first + i] = run;
      run += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kR; ++q) {
    const long long k0 = s + static_cast<long long>(q) * kP2Threads + w * kWave;
    if (k0 >= e) break;
    const bool act = k0 + lane < e;
    const int p = run_add<true>(hist, act ? key_of(v[q]) : 0, act, lane);
    if (act) dst[p] = v[q];
  }
  for (long long k0 = s + static_cast<long long>(kR) * kP2Threads + w * kWave; k0 < e; k0 += kP2Threads) {
    const bool act = k0 + lane < e;
    const unsigned long long x = act ? src[k0 + lane] : 0ull;
    const int p = run_add<true>(hist, act ? key_of(x) : 0, act, lane);
    if (act) dst[p] = x;
  }
}

// The one-pass sweep's tile slots into their coarse A buckets (k_sweep<2> counted them per block in
// hist_mat; off = the scan of those counts): block b walks the tiles its k_sweep<2> block swept (same
// grid, same wave ranges wlo), so its LDS cursors start at off[bucket][b].  Each group of <= 8
// consecutive tiles is one dense range: lane l holds tile l's count and slot, each loaded entry finds
// its tile among those lanes; 4 wave-loads are in flight before their cursor atomics.
__global__ __launch_bounds__(kSwBlock) void k_sweep_scatter(SweepArgs g, const int* __restrict__ off,
                                                            unsigned long long* __restrict__ dst, long long cap) {
  __shared__ int cur[kHistMax];
  for (int i = threadIdx.x; i < g.hist_h; i += kSwBlock) cur[i] = off[static_cast<long long>(i) * gridDim.x + blockIdx.x];
  __syncthreads();
  const int lane = lane_id();
  const int wid = blockIdx.x * kSwWaves + (threadIdx.x >> 6);
  const int tb = g.wlo[wid], te = g.wlo[wid + 1];   // the tiles this wave swept (k_sweep<2>)
  FSLR_BOUND(tb, te + 1);
  FSLR_BOUND(te, (g.nq + kWave - 1) / kWave + 1);
  constexpr int kU = 4;
  for (int t0 = tb; t0 < te; t0 += kTileRun) {
    const int run = min(kTileRun, te - t0);
    const int t = t0 + lane;
    const bool tv = lane < run;
    const int c = tv ? g.tile_cnt[t] : 0;
    const long long u0 = tv ? g.tile_ub[t] : 0;
    const int inc = wave_incl_scan(c);
    const int exc = inc - c;
    const int T = rdl(inc, kWave - 1);
    for (int k0 = 0; k0 < T; k0 += kU * kWave) {
      unsigned long long v[kU];
#pragma unroll
      for (int q = 0; q < kU; ++q) {
        const int k = k0 + q * kWave + lane;
        int j = 0;                                    // the last tile (lane < run) starting at or before k
#pragma unroll
        for (int l = 1; l < kTileRun; ++l)
          if (l < run && rdl(exc, l) <= k && rdl(c, l) > 0) j = l;
        const long long at = __shfl(u0, j) + (k - __shfl(exc, j));
        v[q] = k < T && at < g.ub_cap ? g.ent_ub[at] : 0ull;
      }
#pragma unroll
      for (int q = 0; q < kU; ++q) {
        if (k0 + q * kWave >= T) break;               // wave-uniform
        const bool act = k0 + q * kWave + lane < T;
        const unsigned bk = static_cast<unsigned>(v[q] >> 39) >> g.hist_lo;
        const int p = run_add<true>(cur, static_cast<int>(g.hist_mod ? bk % static_cast<unsigned>(g.hist_h) : bk), act,
                                    lane);
        if (act && p < cap) dst[p] = v[q];
      }
    }
  }
}

int bits_for(long long v) {
  int b = 1;
  while ((1ll << b) <= v) ++b;
  return b;
}

template <typename K>
int resident_blocks(K kernel) {
  int dev = 0, cus = 256, per_cu = 0;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kSwBlock, 0) != hipSuccess || per_cu < 1)
    per_cu = 4;
  return cus * per_cu;
}

template <typename K>
int resident_blocks_n(K kernel, int threads) {
  int dev = 0, cus = 256, per_cu = 0;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu < 1)
    per_cu = 1;
  return cus * per_cu;
}

int blocks_mode(int m) {
  static const int b0 = resident_blocks(k_sweep<0>), b1 = resident_blocks(k_sweep<1>), b2 = resident_blocks(k_sweep<2>);
  return m == 0 ? b0 : m == 1 ? b1 : b2;
}
int blocks_pairs() { static const int b = resident_blocks(k_sweep_pairs); return b; }
// the one-pass sweep's grid for nt tiles (k_wave_bounds, k_sweep<2> and k_sweep_scatter share it)
int sweep_blocks(int nt) { return std::max(1, std::min(blocks_mode(2), (nt + kSwWaves - 1) / kSwWaves)); }
int tiles_of(const SweepArgs& a) { return static_cast<int>((static_cast<long long>(a.nq) + kWave - 1) / kWave); }
// a partition's destination counts are scanned inside k_sweep_total when they are few (<= 64K)
bool dest_scan_fused(const SweepArgs& a, int blocks) {
  return a.hist_mat && a.hist_mod && a.dest_totals && static_cast<long long>(a.hist_h) * blocks <= 65536 &&
         a.hist_h <= 1024;
}

}  // namespace

int sweep_max_waves() {
  return std::max(std::max(blocks_mode(0), blocks_mode(1)), std::max(blocks_mode(2), blocks_pairs())) * kSwWaves;
}

size_t sweep_temp_bytes(long long ent_cap, long long ni, hipStream_t s) {
  size_t a = 0, b = 0, c = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, static_cast<int*>(nullptr), static_cast<int*>(nullptr),
                                         kGrpInts / 2, s);
  (void)hipcub::DeviceRadixSort::SortKeys(nullptr, a, static_cast<unsigned long long*>(nullptr),
                                          static_cast<unsigned long long*>(nullptr), static_cast<int>(ent_cap), 39,
                                          64, s);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, static_cast<long long*>(nullptr),
                                         static_cast<long long*>(nullptr), static_cast<int>((ni + kWave - 1) / kWave),
                                         s);
  return std::max(std::max(a, b), c);
}

hipError_t launch_sweep_plan(const SweepArgs& a, hipStream_t s) {
  const int nt = tiles_of(a);
  if (nt == 0) return hipSuccess;
  if (!a.tests_ready)
    k_tile_tests<<<grid_for(static_cast<long long>(nt) * kWave, 256, 4096), 256, 0, s>>>(a.swin, a.nq, a.tile_tests);
  size_t tb = a.temp_bytes;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(a.temp, tb, a.tile_tests, a.tile_ub, nt, s);
  if (e != hipSuccess) return e;
  const int nw = sweep_blocks(nt) * kSwWaves;
  if (!a.wlo || nw > a.wstat_waves) return hipErrorInvalidValue;
  k_wave_bounds<<<grid_for(nt, 256, 1024), 256, 0, s>>>(a.tile_ub, a.tile_tests, nt, nw, a.wlo);
  return hipGetLastError();
}

hipError_t launch_sweep_count(const SweepArgs& a0, int mode, long long* total_dev, hipStream_t s, long long* n_dev,
                              long long cap) {
  const SweepArgs& a = a0;
  const int nt = tiles_of(a);
  if (nt == 0) return hipMemsetAsync(total_dev, 0, 3 * sizeof(long long), s);
  const int blocks = mode == 2 ? sweep_blocks(nt) : std::min(blocks_mode(mode), (nt + kSwWaves - 1) / kSwWaves);
  if (blocks * kSwWaves > a.wstat_waves) return hipErrorInvalidValue;
  if (a.k0) (void)hipEventRecord(a.k0, s);
  if (mode == 2)
    k_sweep<2><<<blocks, kSwBlock, 0, s>>>(a);
  else
    k_sweep<0><<<blocks, kSwBlock, 0, s>>>(a);
  if (a.k1) (void)hipEventRecord(a.k1, s);
  if (mode == 2) {
    const bool fuse = dest_scan_fused(a, blocks);
    k_sweep_total<<<1, 1024, 0, s>>>(a.wstat, blocks * kSwWaves, a.tile_ub, a.tile_tests, nt, a.counters, a.err,
                                     total_dev, n_dev, cap, fuse ? a.hist_mat : nullptr, a.grp + kGrpInts / 2,
                                     a.hist_h, blocks, a.dest_totals);
    if (a.ev[1]) (void)hipEventRecord(a.ev[1], s);
    return hipGetLastError();
  }
  k_sum_slots<<<kSumBlocks, 256, 0, s>>>(a.wstat, blocks * kSwWaves, 0, 3, kSwTests, kCand, kMatchEntries,
                                         a.counters, nullptr);
  if (a.ev[1]) (void)hipEventRecord(a.ev[1], s);
  size_t tb = a.temp_bytes;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(a.temp, tb, a.tile_cnt, a.tile_off, nt, s);
  if (e != hipSuccess) return e;
  k_total<<<1, 64, 0, s>>>(a.tile_off, a.tile_cnt, mode == 2 ? a.tile_ub : nullptr, a.tile_tests, a.err, nt, total_dev,
                           n_dev, cap);
  return hipGetLastError();
}

hipError_t launch_sweep_dense(const SweepArgs& a, int mode, hipStream_t s) {
  const int nt = tiles_of(a);
  if (a.n_ent <= 0 || nt == 0) return hipSuccess;
  if (mode == 2) {
    // the tiles' places in `ent` (the one-pass sweep does not scan its tile counts)
    size_t tb = a.temp_bytes;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(a.temp, tb, a.tile_cnt, a.tile_off, nt, s);
    if (e != hipSuccess) return e;
    k_compact<<<grid_for(static_cast<long long>(nt) * kWave, 256, 8192), 256, 0, s>>>(a.ent_ub, a.tile_ub, a.tile_off,
                                                                                    a.tile_cnt, nt, a.ent);
  } else {
    const int be = std::min(blocks_mode(1), (nt + kSwWaves - 1) / kSwWaves);
    k_sweep<1><<<be, kSwBlock, 0, s>>>(a);
  }
  return hipGetLastError();
}

int grp_ints() { return kGrpInts; }

void sweep_dest_hist(SweepArgs& a, int n_dest, int shift) {
  const int nt = tiles_of(a);
  const long long P = sweep_blocks(nt);
  if (!a.grp || n_dest < 1 || n_dest > kHistMax || static_cast<long long>(n_dest) * P > kGrpInts / 2) {
    a.hist_mat = nullptr;
    return;
  }
  a.hist_mat = a.grp;
  a.hist_h = n_dest;
  a.hist_lo = shift;
  a.hist_mod = 1;
}

void sweep_coarse_hist(SweepArgs& a) {
  // at most kHistMax buckets; the rest of A's bits (<= 12) are pass 2's LDS bins.  Beyond 2^22 reads the
  // counted grouping runs instead: 16384-bin LDS histograms held pass 2 at two blocks per CU (cfg5:
  // 2.49 ms against 1.40 ms for the counted pass 2, profiles/r05/r5n)
  const int nbits = bits_for(std::max(1, a.n_reads - 1));
  const int hb = std::min(nbits, 10);
  const int nt = tiles_of(a);
  const long long P = sweep_blocks(nt);
  if (!a.grp || nbits - hb > 12 || (static_cast<long long>(1) << hb) * P > kGrpInts / 2) {
    a.hist_mat = nullptr;
    return;
  }
  a.hist_mat = a.grp;
  a.hist_h = 1 << hb;
  a.hist_lo = nbits - hb;
  a.hist_mod = 0;
}

// group the entries by A: from the tile slots (mode 2) or dense `src` into `mid`, then into `out`
static hipError_t group_by_a(const SweepArgs& a, int mode, const unsigned long long* src, unsigned long long* mid,
                             unsigned long long* out, hipStream_t s) {
  const long long n = a.n_ent;
  const int nt = tiles_of(a);
  if (mode == 2 && a.hist_mat) {
    // the sweep counted its entries per coarse bucket: scan, scatter, then each bucket by its low bits
    const int P = sweep_blocks(nt);                                   // the sweep's grid
    const int H = a.hist_h, lo = a.hist_lo;
    int* off = a.grp + kGrpInts / 2;
    size_t tb = a.temp_bytes;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(a.temp, tb, a.hist_mat, off, H * P, s);
    if (e != hipSuccess) return e;
    k_sweep_scatter<<<P, kSwBlock, 0, s>>>(a, off, mid, a.n_dev ? a.ent_cap : 0x7FFFFFFFFFFFFFFFll);
    k_msd_pass2r<kMsdMaxLo, 16><<<H, kP2Threads, 0, s>>>(mid, n, a.n_dev, off, P, H, lo, out);
    return hipGetLastError();
  }
  const int nbits = bits_for(std::max(1, a.n_reads - 1));
  // H = 2^hb buckets of ~4096 entries; P pass-1 workgroups with H P <= kGrpInts / 2 (pass 1 is
  // latency bound, so it wants waves in flight more than wide per-block histograms)
  int hb = 0;
  while (hb < FSLR_MSD_HBMAX && (n >> (12 + hb)) > 0) ++hb;
  hb = std::max(hb, nbits - 12);                            // low digit <= 12 bits (LDS bins)
  hb = std::min(hb, nbits);
  const int H = 1 << hb, lo = nbits - hb;
  // (a small entry set, e.g. one rank's share of the multi-GPU split, takes fewer blocks: about 8K
  // entries per block, so the [bucket][block] counts and their scan stay small)
  const int P = std::max(64, std::min({kMsdMaxBlocks, (1 << 21) / H, static_cast<int>((n + 8191) / 8192)}));
  int* mat = a.grp;
  int* off = a.grp + kGrpInts / 2;
  if (mode == 2) {
    k_msd_pass1<true, false><<<P, kMsdThreads, 0, s>>>(a.ent_ub, a.ub_cap, a.tile_ub, a.tile_cnt, nt, lo, H, mat, nullptr);
  } else {
    k_msd_pass1<false, false><<<P, kMsdThreads, 0, s>>>(src, n, nullptr, nullptr, 0, lo, H, mat, nullptr);
  }
  size_t tb = a.temp_bytes;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(a.temp, tb, mat, off, H * P, s);
  if (e != hipSuccess) return e;
  if (mode == 2) {
    k_msd_pass1<true, true><<<P, kMsdThreads, 0, s>>>(a.ent_ub, a.ub_cap, a.tile_ub, a.tile_cnt, nt, lo, H, off, mid,
                                                      a.n_dev ? a.ent_cap : 0x7FFFFFFFFFFFFFFFll);
  } else {
    k_msd_pass1<false, true><<<P, kMsdThreads, 0, s>>>(src, n, nullptr, nullptr, 0, lo, H, off, mid);
  }
  k_msd_pass2<kMsdMaxLo><<<H, 256, 0, s>>>(mid, n, mode == 2 ? a.n_dev : nullptr, off, P, H, hb, lo, out);
  return hipGetLastError();
}

// totals[k] = entries of destination k from the [k][block] counts and their scan
__global__ void k_dest_totals(const int* __restrict__ mat, const int* __restrict__ off, int H, int P,
                              long long* __restrict__ totals) {
  const int k = threadIdx.x;
  if (k >= H) return;
  const long long last = static_cast<long long>(k) * P + P - 1;
  totals[k] = static_cast<long long>(off[last]) + mat[last] - off[static_cast<long long>(k) * P];
}

hipError_t launch_sweep_partition(const SweepArgs& a, int mode, int shift, int n_dest, unsigned long long* dst,
                                  long long dst_cap, long long* totals, hipStream_t s) {
  if (n_dest < 1 || n_dest > kMsdMaxH) return hipErrorInvalidValue;
  int* mat = a.grp;
  int* off = a.grp + kGrpInts / 2;
  const int nt = tiles_of(a);
  // a rank whose index range is empty (more ranks than chromosomes, an empty position range): no sweep
  // ran, so the wave ranges, histograms and totals the scatter would read are last query's — no entries
  if (nt == 0) return hipMemsetAsync(totals, 0, static_cast<size_t>(n_dest) * sizeof(long long), s);
  if (mode == 2 && a.hist_mat && a.hist_mod && a.hist_h == n_dest && a.hist_lo == shift) {
    // the sweep counted its entries per destination: scan, totals, one scatter over its wave ranges
    const int P = sweep_blocks(nt);
    if (!(dest_scan_fused(a, P) && a.dest_totals == totals)) {   // else k_sweep_total scanned them
      size_t tb = a.temp_bytes;
      hipError_t e = hipcub::DeviceScan::ExclusiveSum(a.temp, tb, mat, off, n_dest * P, s);
      if (e != hipSuccess) return e;
      k_dest_totals<<<1, 64, 0, s>>>(mat, off, n_dest, P, totals);
    }
    k_sweep_scatter<<<P, kSwBlock, 0, s>>>(a, off, dst, dst_cap);
    return hipGetLastError();
  }
  const int P = kMsdMaxBlocks;
  const long long n = a.n_ent;
  if (mode == 2)
    k_msd_pass1<true, false, true><<<P, kMsdThreads, 0, s>>>(a.ent_ub, a.ub_cap, a.tile_ub, a.tile_cnt, nt, shift, n_dest,
                                                             mat, nullptr);
  else
    k_msd_pass1<false, false, true><<<P, kMsdThreads, 0, s>>>(a.ent, n, nullptr, nullptr, 0, shift, n_dest, mat,
                                                              nullptr);
  size_t tb = a.temp_bytes;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(a.temp, tb, mat, off, n_dest * P, s);
  if (e != hipSuccess) return e;
  k_dest_totals<<<1, 64, 0, s>>>(mat, off, n_dest, P, totals);
  if (mode == 2)
    k_msd_pass1<true, true, true><<<P, kMsdThreads, 0, s>>>(a.ent_ub, a.ub_cap, a.tile_ub, a.tile_cnt, nt, shift, n_dest,
                                                            off, dst, dst_cap);
  else
    k_msd_pass1<false, true, true><<<P, kMsdThreads, 0, s>>>(a.ent, n, nullptr, nullptr, 0, shift, n_dest, off, dst,
                                                             dst_cap);
  return hipGetLastError();
}

hipError_t launch_sweep_pairs(const SweepArgs& a0, int mode, hipStream_t s) {
  SweepArgs a = a0;
  if (a.ev[2]) (void)hipEventRecord(a.ev[2], s);
  const bool msd = a.grp && a.n_ent > 0 && a.n_ent < (1ll << 31);
  if (mode == 0 || (mode == 2 && !msd)) {
    hipError_t e = launch_sweep_dense(a, mode, s);          // dense entries in a.ent
    if (e != hipSuccess) return e;
  }
  if (a.ev[3]) (void)hipEventRecord(a.ev[3], s);
  unsigned long long* const ent0 = a.ent;
  unsigned long long* const sorted0 = a.ent_sorted;
  if (msd) {
    // mode 2: tile slots -> ent -> ent_sorted; mode 0: ent -> ent_sorted -> ent (the pair kernel
    // then reads ent); mode 3: the caller's entries -> ent_mid -> ent_sorted
    hipError_t e;
    if (mode == 2) {
      e = group_by_a(a, 2, nullptr, a.ent, a.ent_sorted, s);
    } else if (mode == 0) {
      e = group_by_a(a, 0, a.ent, a.ent_sorted, a.ent, s);
      a.ent_sorted = a.ent;
    } else {
      e = group_by_a(a, 3, a.ent, a.ent_mid, a.ent_sorted, s);
    }
    if (e != hipSuccess) return e;
  } else if (a.n_ent > 0) {
    size_t tb = a.temp_bytes;
    const int end_bit = 39 + bits_for(std::max(1, a.n_reads - 1));
    hipError_t e = hipcub::DeviceRadixSort::SortKeys(a.temp, tb, a.ent, a.ent_sorted, static_cast<int>(a.n_ent), 39,
                                                     std::min(end_bit, 64), s);
    if (e != hipSuccess) return e;
  }
  if (a.ev[4]) (void)hipEventRecord(a.ev[4], s);
  // the grouping's buffer the pair kernel does not read: its long runs are bucketed there (mode 2 and the
  // radix fallback: ent; mode 0: the original ent_sorted; mode 3: ent_mid, the caller's ent being input)
  a.pair_scr = mode == 3 ? (msd ? a.ent_mid : nullptr) : (a.ent_sorted == ent0 ? sorted0 : ent0);
  const long long chunks = (a.n_ent + kChunk2 - 1) / kChunk2;
  const int blocks = static_cast<int>(std::max(1ll, std::min<long long>(blocks_pairs(), (chunks + kSwWaves - 1) / kSwWaves)));
  if (blocks * kSwWaves > a.wstat_waves) return hipErrorInvalidValue;
  if (a.p0) (void)hipEventRecord(a.p0, s);
  k_sweep_pairs<<<blocks, kSwBlock, 0, s>>>(a);
  if (a.p1) (void)hipEventRecord(a.p1, s);
  k_sum_slots<<<kSumBlocks, 256, 0, s>>>(a.wstat, blocks * kSwWaves, 2, 4, -1, -1, kMatchedPairs, a.counters,
                                         a.err + 3);
  return hipGetLastError();
}

}  // namespace fslr
