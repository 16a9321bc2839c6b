// query.hip — the pair kernels: replace the driver of query_interval_trees (cluster.py:187-227)
// with its predicates different_lengths_or_alignments (:178-183), overall_jaccard_similarity
// (:140-170), calculate_overlap (:133-136) and the cutoff lookup (:216-219).
//
// query_kernel — one wavefront per query read A (grid-stride over ranks a in [a_begin, a_end));
// A's intervals live in lanes 0..LA-1 and are read with v_readlane / ds_bpermute.
//  1. candidate walk: A's scan ranges (kernels.hpp: rng_s) are flattened with a wave prefix sum
//     and walked 64 records per step, one record per lane; the next step's records (and the next
//     read's header) are loaded while the current step is processed.  Forward records are hits,
//     backward records hit iff end >= start_i.
//  2. dedupe: a hit on read B > A goes into a per-wave LDS hash set (epoch-tagged): the first
//     insertion is the one evaluation of (A, B), like the reference's seen-set (:205-208).
//  3. gate at first sight: B's packed read record sits beside the hit record (idx_gate), so
//     different_lengths_or_alignments is decided without a dependent gather (IEEE double ==
//     Python int/int true division).
//  4. match list: with every overlap threshold >= 1 (overlap > 0), a matching interval pair
//     overlaps, so it IS one of the hits: hits whose reciprocal overlap passes are appended to a
//     per-wave LDS list in A-major order (the walk never moves back in i).
//  5. first-fit greedy per matched partner, one lane each, straight from the list in the
//     reference's order (rows i of A ascending, lowest unused j of B) — no row of B is read.
//  6. edges (A, B, I, U) are staged in LDS and flushed 64 at a time (one global atomic per 64).
// Pairs that need B's rows — thresholds < 1 (overlap <= 0: matches need not overlap), an
// aln_size == 0 interval (exact ZeroDivisionError replay), a full match list, or more distinct
// partners than the hash holds (witness rule) — are appended to a deferred list for
// deferred_kernel, one lane per pair, which gathers A's and B's intervals.
#include "fslr_hip.h"
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "kernels.hpp"
#include "wave.hpp"

namespace fslr {
namespace {

constexpr int kWavesPerBlock = 4;
constexpr int kShardMask = (1 << kShardShift) - 1;   // kernels.hpp: kShardShift
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kStageCap = kWave;          // LDS staging of edges / deferred entries (flush before overflow)
constexpr int kChunk = 8;                 // query reads per work-queue ticket
constexpr int kDynamicMinReads = 64;      // work queues only when every wave has this many reads
constexpr int kHashBits = 9;
constexpr int kHashSize = 1 << kHashBits;
constexpr int kHashLimit = 320;           // insert while distinct partners < limit (load <= 75 %)
constexpr int kMatchCap = 192;            // match-list entries per query read
constexpr int kPassRecords = 512;         // walk records per partner partition (the hash holds 320)
constexpr unsigned kEpochShift = 25;      // key = epoch << 25 | B  (B < FSLR_MAX_READS = 2^25)
constexpr unsigned kEpochMax = 127;
constexpr unsigned kBMask = 0x1FFFFFFu;
// per-partner state (one word per hash slot)
constexpr unsigned kStLenOk = 1u;         // passed different_lengths_or_alignments
constexpr unsigned kStDefer = 2u;         // evaluated by deferred_kernel
constexpr unsigned kStMatch = 4u;         // has at least one matching interval pair
constexpr unsigned kStSpill = 8u;         // a match did not fit the match list
constexpr unsigned kStConflict = 16u;     // two matching pairs share a row or a column (ordered greedy)
// deferred entries: a << 39 | B << 14 | ic << 8 | jc << 2 | kind
constexpr unsigned kDefPair = 0u;         // unique lenOK pair: gather evaluation (replay if aln_size==0)
constexpr unsigned kDefWitness = 1u;      // candidate past the hash limit: witness rule, then as above

// FSLR_SECTION_PROF builds (make prof): per-wave cycle sums of the kernel's sections land in
// counters[kSecBase + k] — 0 read setup, 1 next-chunk map + loads, 2 hit + dedupe (absorbs the
// load wait), 3 gate + deferred puts, 4 match list, 5 next-read prefetch, 6 greedy + edges, 7 wave total
#ifdef FSLR_SECTION_PROF
#define SEC_NOW(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define SEC_ADD(k, t0) (sec[k] += __builtin_amdgcn_s_memtime() - (t0))
constexpr int kSections = 8;
#else
#define SEC_NOW(v) (void)0
#define SEC_ADD(k, t0) (void)0
#endif

// partner partition of read B (a multiplier independent of the hash slot's)
__device__ __forceinline__ int part_of(int B, int npass) {
  return static_cast<int>(((static_cast<unsigned>(B) * 0x85EBCA6Bu) >> 8) % static_cast<unsigned>(npass));
}

__global__ void k_len_bounds(const int4* __restrict__ rmeta, int a0, int a1, double qcut, double ncut,
                             int4* __restrict__ lb) {
  for (int a = a0 + blockIdx.x * blockDim.x + threadIdx.x; a < a1; a += gridDim.x * blockDim.x) {
    const int4 m = rmeta[a];
    const int2 q = ratio_range(m.z, qcut), n = ratio_range(m.w, ncut);
    lb[a] = make_int4(q.x, q.y, n.x, n.y);
  }
}

// Deferred-list appends, staged in LDS like the edges.
struct DeferStage {
  unsigned long long* DQ;
  int n;
  __device__ void flush(const QueryArgs& g, int nb, int lane) {
    wave_lds_sync();
    const bool act = lane < nb;
    const unsigned long long e = act ? DQ[lane] : 0ull;
    const int rem = n - nb;
    const unsigned long long mv = lane < rem ? DQ[nb + lane] : 0ull;
    wave_lds_sync();
    if (lane < rem) DQ[lane] = mv;
    n = rem;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(&g.counters[kDeferCount], static_cast<unsigned long long>(nb));
    base = __shfl(base, 0);
    const long long k = static_cast<long long>(base) + lane;
    if (act && k < g.defer_cap) g.defer[k] = e;
  }
  __device__ void put(const QueryArgs& g, bool p, int a, int B, int ic, int jc, unsigned kind, int lane) {
    const unsigned long long m = __ballot(p);
    if (!m) return;
    const int np = __popcll(m);
    if (n + np > kStageCap) flush(g, n, lane);
    if (p)
      DQ[n + mbcnt(m)] = (static_cast<unsigned long long>(a) << 39) | (static_cast<unsigned long long>(B) << 14) |
                         (static_cast<unsigned long long>(ic) << 8) | (static_cast<unsigned long long>(jc) << 2) |
                         kind;
    n += np;
  }
};

// kMulti = false: every query read of the shard; a read whose walk exceeds 1.5 pass_records records
// (more partners than the hash holds) is handed to the kMulti = true launch (fwd[a] = -1, listed
// by k_collect_heavy).
// kMulti = true: the handed-over reads, each in ceil(R / pass_records) partner partitions.
template <int kThrMode, bool kMulti>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6))) void query_kernel(QueryArgs g) {
  __shared__ unsigned hash_all[kWavesPerBlock][kHashSize];
  __shared__ unsigned state_all[kWavesPerBlock][kHashSize];
  __shared__ unsigned ml_all[kWavesPerBlock][kMatchCap];
  __shared__ unsigned short mp_all[kWavesPerBlock][kHashLimit + kWave];
  __shared__ unsigned long long es_all[kWavesPerBlock][kStageCap];
  __shared__ unsigned long long dq_all[kWavesPerBlock][kStageCap];
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  unsigned* H = hash_all[wv];
  unsigned* ST = state_all[wv];
  unsigned* ML = ml_all[wv];
  unsigned short* MP = mp_all[wv];     // partners (hash slots) with at least one match, first-match order
  EdgeStage es{es_all[wv], 0};
  const EdgeOut eo{g.edges, g.edge_iu, g.edge_cap, &g.counters[kEdgeCount]};
  DeferStage ds{dq_all[wv], 0};
  for (int k = lane; k < kHashSize; k += kWave) H[k] = 0u;
  unsigned epoch = 0;
  // edge iff U <= umax[I-1] (cluster.py:218-219 folded on the host); lane l holds umax[l]
  const int umax_v = g.umax[lane];
  // Read assignment.  Query reads are numbered by a virtual index v: one shard → rank a_begin + v;
  // a multi-GPU query shard owns blocks of 64 consecutive ranks dealt round robin (balanced: low ranks
  // have more higher-rank partners).  The first k_static * nwaves indices are dealt grid-stride
  // (wave w takes w, w + nwaves, ...); the rest is handed out in chunks of kChunk consecutive
  // indices from 8 work queues (counters on separate cache lines; queue x serves chunks 8 k + x),
  // own XCD's queue first, then the others'.  The queues even out waves that run slower than their
  // neighbours (issue arbitration by age, heavier reads): 1M reads, one shard: 1.78 → 1.52 ms.
  // A ticket's returned atomic is waited on at the wave's next load wait (vmcnt is in order), so
  // small shards, whose waves hold few reads, are dealt statically (launch_query sets k_static).
  // The next chunk is reserved when the current one starts, four reads ahead of its use.
  const int nwaves = gridDim.x * kWavesPerBlock;
  const int wid = blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
  const int a_hi = g.a_end;
  // kMulti: the list's length is only known on the device (written by the kMulti = false launch)
  const int nv = kMulti ? static_cast<int>(min(static_cast<long long>(g.counters[kHeavyCount]),
                                               static_cast<long long>(g.a_end)))
                        : g.nv;
  auto rank_of = [&](int v) {
    if (kMulti) return v < 0 || v >= nv ? a_hi : ((const_i32_ptr)(g.heavy))[v];
    return v < 0 ? a_hi
                 : g.a_begin + ((((v >> kShardShift) * g.n_shards + g.shard) << kShardShift) | (v & kShardMask));
  };
  const int k_static = g.k_static;
  const int v0 = k_static * nwaves;                           // first dynamic index
  const int nchunks = (nv - v0 + kChunk - 1) / kChunk;
  const int q_home = static_cast<int>(__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20)) & 7;   // XCC_ID
  unsigned long long* queues = g.counters + (kMulti ? kQueueBase2 : kQueueBase);
  auto reserve = [&](int q) -> int {       // ticket on queue q (wave-uniform)
    int k = 0;
    if (lane_id() == 0) k = static_cast<int>(atomicAdd(&queues[q * kQueueStride], 1ull));
    return __builtin_amdgcn_readfirstlane(k);
  };
  int ks = 0;                 // static indices taken
  int cur_c = -2;             // current dynamic chunk (-2: none yet, -1: all drained)
  int cur_i = kChunk;         // next v inside it
  int res_q = q_home;
  int res_k = k_static < 2 && nchunks > 0 ? reserve(q_home) : 0;
  // next virtual index, or -1 when every queue is drained
  auto pull = [&]() -> int {
    if (ks < k_static) {
      const int v = wid + nwaves * ks++;
      if (ks == k_static - 1 && nchunks > 0) res_k = reserve(q_home);
      return v;
    }
    while (true) {
      if (cur_c >= 0 && cur_i < kChunk) {
        const int v = v0 + cur_c * kChunk + cur_i++;
        if (v < nv) return v;
      }
      if (cur_c == -1 || nchunks <= 0) return -1;
      // take the reserved chunk; if its queue is drained, steal from the next queues
      int c = 8 * res_k + res_q;
      while (c >= nchunks && res_q != ((q_home + 7) & 7)) {
        res_q = (res_q + 1) & 7;
        res_k = reserve(res_q);
        c = 8 * res_k + res_q;
      }
      if (c >= nchunks) {
        cur_c = -1;
        return -1;
      }
      cur_c = c;
      cur_i = 0;
      res_k = reserve(res_q);
    }
  };
  int v = pull();
  unsigned long long w_eval = 0, w_jacc = 0, w_cand = 0, w_over = 0, w_ml = 0, w_mp = 0, w_walk = 0;
  // algorithmic bytes of evaluated pairs: 16 (LA + LB) + 32 each
  unsigned long long w_la_pairs = 0;
  unsigned l_lb = 0;
  int w_maxfwd = 0;
#ifdef FSLR_SECTION_PROF
  unsigned long long sec[kSections] = {};
  unsigned long long read_max = 0;
  int read_max_a = -1;
  unsigned long long it_sum[3] = {0, 0, 0};
  int it_k = 0;
#endif
  SEC_NOW(t_wave);
  // read pipeline: headers (scalar loads) three reads ahead, the sorted positions of a read's
  // intervals (qpos, coalesced) two ahead, its rows in the index one ahead — so a read's rows are
  // requested when the previous read starts, from positions that arrived one read earlier
  const int v_n = pull(), v_nn = pull();
  int v_nnn = pull();
  int a = rank_of(v);
  const int2* rm2 = reinterpret_cast<const int2*>(g.rmeta);     // {iv offset, len | flags << 16}
  auto hdr = [&](int r) { return r < a_hi ? sload2(rm2, 2 * r) : make_int2(0, 0); };
  auto qpos_of = [&](int r, int2 h) { return r < a_hi && lane < (h.y & 0xffff) ? g.qpos[h.x + lane] : 0; };
  // lane i of A: my = {start, end, thr} of interval i, rg = {q, n_fwd, bwd_begin} (kernels.hpp)
  auto rows = [&](int r, int2 h, int q, int3& m, int3& rr) {
    m = make_int3(0, 0, 0);
    rr = make_int3(0, 0, 0);
    if (r < a_hi && lane < (h.y & 0xffff)) {
      m = load3(g.idx4, q, 0);
      const int2 rs = g.rng_s[q];
      rr = make_int3(q, rs.x, rs.y);
    }
  };
  int a_next = rank_of(v_n), a_nn = rank_of(v_nn);
  int2 am = hdr(a), am_n = hdr(a_next), am_nn = hdr(a_nn);
  int3 my, rg;
  rows(a, am, qpos_of(a, am), my, rg);
  int qv_n = qpos_of(a_next, am_n);

  int v_4 = -1;
  for (; a < a_hi; a = a_next, a_next = a_nn, a_nn = rank_of(v_nnn), v_nnn = v_4) {
    SEC_NOW(t_s0);
#ifdef FSLR_SECTION_PROF
    const unsigned long long rt_s0 = __builtin_amdgcn_s_memrealtime();
#endif
    int3 my_next, rg_next;
    rows(a_next, am_n, qv_n, my_next, rg_next);
    const int qv_nn = qpos_of(a_nn, am_nn);
    const int2 am_nnn = hdr(rank_of(v_nnn));
    // the index four reads ahead: a work-queue atomic issued here completes behind the loads just
    // issued and the walk's first loads, instead of stalling the next wait on its own
    v_4 = pull();
    const int4 alb = sload4(g.lb, a);
    const int amy = am.y;
    const int LA = amy & 0xffff;
    const bool hazA = (static_cast<unsigned>(amy) >> 16) & 1u;
    // length gate of A as integer ranges (k_len_bounds)
    const int qlo = alb.x, qhi = alb.y, nlo = alb.z, nhi = alb.w;
    const bool qz = qlo < 0, nz = nlo < 0;
    const int qlo_e = qz ? 1 : qlo, nlo_e = nz ? 1 : nlo;

    const int cnt = rg.y + (rg.x - rg.z);   // n_fwd + n_bwd
    const int pre = wave_incl_scan(cnt);
    const int ex = pre - cnt;
    const int R = rdl(pre, kWave - 1);
    // interval i's records r in [ex, ex + cnt) are two runs of sorted positions:
    // forward r < bnd: p = r + off_f;  backward: p = r + off_b
    const int bnd = ex + rg.y, off_f = rg.x + 1 - ex, off_b = rg.z - rg.y - ex;
    int fwdA = 0;

    // record r of A's walk → (interval mi, sorted position p, forward?)
    auto map_record = [&](int base, int& mi, int& p, bool& fwd) {
      const int r = base + lane;
      const int i0 = __popcll(__ballot(lane < LA && pre <= base));
      mi = i0;
      for (int k = i0 + 1; k < LA; ++k) {
        const int exk = rdl(ex, k);
        if (exk >= base + kWave) break;
        if (r >= exk) mi = k;
      }
      const int bnd_i = __shfl(bnd, mi), of_i = __shfl(off_f, mi), ob_i = __shfl(off_b, mi);
      fwd = r < bnd_i;
      p = r + (fwd ? of_i : ob_i);
    };

    // Partner partitions: a read whose walk is longer than kPassRecords records may have more
    // distinct partners than the hash holds, so its walk is repeated npass times, pass k taking the
    // partners B with part(B) == k (each pair still evaluated exactly once, in one pass).  Dense
    // inputs (10M reads on the same genome: ~700 hits per read) would otherwise defer most
    // candidates to the witness path, one wavefront per candidate.
    // one pass of the walk + greedy over the partners of partition `pass` (kParts: of npass > 1)
    auto walk_pass = [&](auto multi, int pass, int npass) __attribute__((always_inline)) {
    constexpr bool kParts = decltype(multi)::value;
    if (++epoch > kEpochMax) {
      wave_lds_sync();
      for (int k = lane; k < kHashSize; k += kWave) H[k] = 0u;
      epoch = 1;
    }
    int uniq = 0, mln = 0, mpn = 0;
    int mi_c = 0, p_c = 0;
    bool fwd_c = false;
    int4 rec_c = make_int4(0, -1, 0, 0);
    int2 gt_c = make_int2(0, 0);
    if (R > 0) {
      map_record(0, mi_c, p_c, fwd_c);
      if (lane < R) {
        rec_c = g.idx4[p_c];
        gt_c = g.idx_gate[p_c];
      }
    }
    SEC_ADD(0, t_s0);
    for (int base = 0; base < R; base += kWave) {
      SEC_NOW(t_s1);
      const bool valid = base + lane < R;
      const int mi = mi_c;
      const bool fwd = fwd_c;
      const int4 rec = rec_c;
      const int2 gt = gt_c;
      // issue the next step's loads before working on this one
      if (base + kWave < R) {
        map_record(base + kWave, mi_c, p_c, fwd_c);
        rec_c = make_int4(0, -1, 0, 0);
        if (base + kWave + lane < R) {
          rec_c = g.idx4[p_c];
          gt_c = g.idx_gate[p_c];
        }
      }
      SEC_ADD(1, t_s1);
      SEC_NOW(t_s2);
      const int s_i = __shfl(my.x, mi), e_i = __shfl(my.y, mi), t_i = __shfl(my.z, mi);
      const bool hit = valid && (fwd || rec.y >= s_i);
      if (!kParts || pass == 0) w_cand += __popcll(__ballot(hit));
      const int B = rec.w >> 6;
      const bool cand = hit && B > a && (!kParts || part_of(B, npass) == pass);
      // ---- dedupe: per-wave LDS hash set of partners (the reference's seen-set) ----------
      const bool ins_mode = uniq < kHashLimit;
      bool isnew = false, over = false;
      unsigned h = (static_cast<unsigned>(B) * 2654435761u) >> (32 - kHashBits);
      if (cand) {
        const unsigned key = (epoch << kEpochShift) | static_cast<unsigned>(B);
        while (true) {
          unsigned cur = H[h];
          if ((cur >> kEpochShift) != epoch) {
            if (!ins_mode) { over = true; break; }
            const unsigned old = atomicCAS(&H[h], cur, key);
            if (old == cur) { isnew = true; break; }
            cur = old;
            if ((cur >> kEpochShift) != epoch) continue;
          }
          if (cur == key) break;    // B already seen for this A
          h = (h + 1) & (kHashSize - 1);
        }
      }
      const unsigned long long nm = __ballot(isnew);
      uniq += __popcll(nm);
      SEC_ADD(2, t_s2);
      if (g.mode == 1) continue;
      SEC_NOW(t_s3);
      // ---- gate at first sight (idx_gate: {qlen2, nal | LB << 24 | haz << 31}) -------------
      const int LB = (gt.y >> 24) & 127;
      const bool haz = hazA || (static_cast<unsigned>(gt.y) >> 31);
      const int q2 = gt.x, n2 = gt.y & 0xFFFFFF;
      const bool pq = q2 >= qlo_e && q2 <= qhi;
      const bool zd = isnew && ((qz && q2 == 0) || (!pq && nz && n2 == 0));
      const bool lenok = isnew && !zd && (pq || (n2 >= nlo_e && n2 <= nhi));
      raise_zd(g.err, zd, a, B);
      const bool defer = lenok && (kThrMode == 1 || haz);
      if (isnew) {
        ST[h] = (lenok ? kStLenOk : 0u) | (defer ? kStDefer : 0u) | (static_cast<unsigned>(LB) << 8);
        l_lb += static_cast<unsigned>(LB);
      }
      w_eval += __popcll(nm);
      w_la_pairs += static_cast<unsigned long long>(LA) * __popcll(nm);
      w_jacc += __popcll(__ballot(lenok));
      if (g.mode == 0) {
        ds.put(g, defer, a, B, 0, 0, kDefPair, lane);
        ds.put(g, over, a, B, mi, rec.w & 63, kDefWitness, lane);
      }
      w_over += __popcll(__ballot(over));
      wave_lds_sync();
      SEC_ADD(3, t_s3);
      SEC_NOW(t_s4);
      // ---- matching interval pairs → match list (A-major: i never decreases) -----------------
      if (kThrMode == 0) {
        const bool mt = cand && !over && (min(e_i, rec.y) - max(s_i, rec.x) >= max(t_i, rec.z));
        const unsigned long long mm = __ballot(mt);
        if (mm) {
          bool first = false;
          if (mt) {
            const int idx = mln + mbcnt(mm);
            unsigned old;
            if (idx < kMatchCap) {
              ML[idx] = h | (static_cast<unsigned>(mi) << kHashBits) |
                        (static_cast<unsigned>(rec.w & 63) << (kHashBits + 6));
              old = atomicOr(&ST[h], kStMatch);
            } else {
              old = atomicOr(&ST[h], kStMatch | kStSpill);
            }
            first = !(old & kStMatch);
          }
          const unsigned long long fm = __ballot(first);
          if (first) MP[mpn + mbcnt(fm)] = static_cast<unsigned short>(h);
          mpn += __popcll(fm);
          mln = min(mln + __popcll(mm), kMatchCap);
        }
      }
      SEC_ADD(4, t_s4);
    }
    SEC_NOW(t_s5);
    SEC_ADD(5, t_s5);
    SEC_NOW(t_s6);
    // ---- first-fit greedy from the match list, one lane per matched partner ----------------
    if (kThrMode == 0 && g.mode == 0 && mpn > 0) {
      wave_lds_sync();
      // Fast path: a partner none of whose matching interval pairs share a row i or a column j
      // keeps every pair under first-fit (each row has one candidate, nobody else wants it), so
      // I = its number of pairs.  One pass with lanes = list entries ORs each entry's i and j into
      // the partner's masks (scratch words after the list; partner index in ST bits 16..21) and
      // flags the partner when a bit was already set; only flagged partners run the ordered scan.
      const bool fast = mpn <= kWave && mln + 4 * mpn <= kMatchCap;
      unsigned* SM = ML + mln;
      if (fast) {
        if (lane < mpn) {
          const int hp = MP[lane];
          ST[hp] = (ST[hp] & 0xFFFFu) | (static_cast<unsigned>(lane) << 16);
          SM[4 * lane] = SM[4 * lane + 1] = SM[4 * lane + 2] = SM[4 * lane + 3] = 0u;
        }
        wave_lds_sync();
        for (int kb = 0; kb < mln; kb += kWave) {
          if (kb + lane < mln) {
            const unsigned e = ML[kb + lane];
            const unsigned hh = e & (kHashSize - 1);
            const unsigned i = (e >> kHashBits) & 63u, j = (e >> (kHashBits + 6)) & 63u;
            const unsigned p = (ST[hh] >> 16) & 63u;
            const unsigned bi = 1u << (i & 31u), bj = 1u << (j & 31u);
            const unsigned oi = atomicOr(&SM[4 * p + (i >> 5)], bi);
            const unsigned oj = atomicOr(&SM[4 * p + 2 + (j >> 5)], bj);
            if ((oi & bi) | (oj & bj)) atomicOr(&ST[hh], kStConflict);
          }
        }
        wave_lds_sync();
      }
      for (int k0 = 0; k0 < mpn; k0 += kWave) {
        const bool act = k0 + lane < mpn;
        const int h = act ? static_cast<int>(MP[k0 + lane]) : 0;
        const unsigned key = H[h];
        const unsigned st = act ? ST[h] : 0u;
        const bool hasm = act && (st & kStLenOk) && !(st & kStDefer);
        const bool spill = hasm && (st & kStSpill);
        const bool need = hasm && !spill;
        const int B = static_cast<int>(key & kBMask);
        const int LB = static_cast<int>((st >> 8) & 0xffu);
        int I = 0;
        bool ordered = need;
        if (fast) {
          ordered = need && (st & kStConflict);
          if (act) I = __popc(SM[4 * lane]) + __popc(SM[4 * lane + 1]);
        }
        if (__ballot(ordered)) {
          // reference order (cluster.py:152-161): rows i of A ascending, lowest unused j of B.  The
          // list is A-major, so the row index is wave-uniform along it: entries are read 64 per
          // LDS load and walked with readlane, each lane ORs the j of its own partner's entries
          // into the current row, and a row change settles every lane's row at once.
          unsigned used_lo = 0u, used_hi = 0u, row_lo = 0u, row_hi = 0u;
          int cur = -1, Io = 0;
          for (int kb = 0; kb < mln; kb += kWave) {
            const unsigned ev = kb + lane < mln ? ML[kb + lane] : 0u;
            const int ne = min(kWave, mln - kb);
            for (int t = 0; t < ne; ++t) {
              const unsigned e = static_cast<unsigned>(rdl(static_cast<int>(ev), t));
              const int i = static_cast<int>((e >> kHashBits) & 63u);
              if (i != cur) {
                const unsigned m_lo = row_lo & ~used_lo, m_hi = row_hi & ~used_hi;
                used_lo |= m_lo & (0u - m_lo);
                used_hi |= m_lo ? 0u : (m_hi & (0u - m_hi));
                Io += (m_lo | m_hi) != 0u;
                row_lo = row_hi = 0u;
                cur = i;
              }
              const unsigned j = (e >> (kHashBits + 6)) & 63u;
              const bool mine = static_cast<int>(e & (kHashSize - 1)) == h;
              if (j < 32u) row_lo |= mine ? (1u << j) : 0u;
              else row_hi |= mine ? (1u << (j - 32u)) : 0u;
            }
          }
          const unsigned m_lo = row_lo & ~used_lo, m_hi = row_hi & ~used_hi;
          Io += (m_lo | m_hi) != 0u;
          if (ordered) I = Io;
        }
        const int U = LA + LB - I;
        const bool pass = U <= __shfl(umax_v, max(I, 1) - 1);
        fwdA += es.put(eo, pass && need && I > 0, a, B, I, U, lane);
        ds.put(g, spill, a, B, 0, 0, kDefPair, lane);
      }
    }
    SEC_ADD(6, t_s6);
    w_ml += mln;
    w_mp += mpn;
    w_walk += static_cast<unsigned long long>(R);
    };
    // R (the walk's records) bounds the distinct partners; a read whose walk is more than 1.5
    // partitions long goes to the partitioned launch, which splits it into ~pass_records-record parts
    const int pr = g.pass_records;
    bool handed = false;
    if constexpr (!kMulti) {
      // to the partitioned launch: marked by fwd[a] = -1 (k_collect_heavy lists the marked reads;
      // a pointer and an atomic here cost the kernel registers it does not have)
      handed = pr > 0 && R > pr + (pr >> 1);
      if (!handed) walk_pass(std::false_type{}, 0, 1);
    } else {
      const int npass = pr > 0 ? max(1, (R + pr - 1) / pr) : 1;
      for (int pass = 0; pass < npass; ++pass) walk_pass(std::true_type{}, pass, npass);
    }
    if (lane == 0) g.fwd[a] = handed ? -1 : fwdA;
    w_maxfwd = max(w_maxfwd, fwdA);
#ifdef FSLR_SECTION_PROF
    {
      const unsigned long long dt = __builtin_amdgcn_s_memtime() - t_s0;
      if (dt > read_max) {
        read_max = dt;
        read_max_a = a;
      }
      it_sum[min(it_k, 2)] += dt;
      ++it_k;
      if (lane == 0 && g.diag) {
        g.diag[2 * a] = rt_s0;
        g.diag[2 * a + 1] = min(dt, 0xffffffffull) | (static_cast<unsigned long long>(__smid() & 0xffffu) << 32) |
                            (static_cast<unsigned long long>(min(it_k, 4095)) << 48);
      }
    }
#endif
    am = am_n;
    am_n = am_nn;
    am_nn = am_nnn;
    qv_n = qv_nn;
    my = my_next;
    rg = rg_next;
  }
  if (es.n > 0) es.flush(eo, es.n, lane);
  if (ds.n > 0) ds.flush(g, ds.n, lane);
  SEC_ADD(7, t_wave);
  unsigned long long l_bytes = l_lb;
  for (int o = 32; o > 0; o >>= 1) l_bytes += __shfl_xor(l_bytes, o);
  l_bytes = 16ull * (l_bytes + w_la_pairs) + 32ull * w_eval;
  // per-wave statistics: one plain 8-B store per lane into this wave's slot (kernels.hpp WaveStat)
  {
    const int wid = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    unsigned long long f = 0;
    f = lane == kWsEval ? w_eval : f;
    f = lane == kWsJacc ? w_jacc : f;
    f = lane == kWsCand ? w_cand : f;
    f = lane == kWsAlgoBytes ? l_bytes : f;
    f = lane == kWsOverflow ? w_over : f;
    f = lane == kWsMatchEntries ? w_ml : f;
    f = lane == kWsMatchedPairs ? w_mp : f;
    f = lane == kWsMaxFwd ? static_cast<unsigned long long>(w_maxfwd) : f;
    f = lane == kWsWalked ? w_walk : f;
#ifdef FSLR_SECTION_PROF
    for (int k = 0; k < kSections; ++k) f = lane == kWsBase + k ? sec[k] : f;
    f = lane == kWsBase + 8 ? read_max : f;
    f = lane == kWsBase + 9 ? static_cast<unsigned long long>(read_max_a) : f;
    f = lane == kWsBase + 10 ? sec[7] : f;
    f = lane == kWsBase + 11 ? sec[7] : f;
    f = lane == kWsBase + 12 ? 1ull : f;
    for (int k = 0; k < 3; ++k) f = lane == kWsBase + 13 + k ? it_sum[k] : f;
#endif
    if constexpr (!kMulti) {
      if (lane < kWsProf) g.wstat[static_cast<long long>(wid) * kWStride + lane] = f;
    } else if (w_cand != 0) {
      // the partitioned launch: few waves have work at typical densities, so those add their
      // statistics directly (no per-wave slots, no reduction launch)
      if (lane == kWsMaxFwd) {
        if (f) atomicMax(g.err + 3, static_cast<int>(f));
      } else if (lane < kWsBase && f) {
        const int dst = lane == kWsEval ? kEval : lane == kWsJacc ? kJacc : lane == kWsCand ? kCand
                      : lane == kWsAlgoBytes ? kAlgoBytes : lane == kWsOverflow ? kOverflow
                      : lane == kWsMatchEntries ? kMatchEntries : lane == kWsWalked ? kWalked : kMatchedPairs;
        atomicAdd(&g.counters[dst], f);
      }
    }
  }
}

// The reads query_kernel<., false> handed over (fwd == -1) as a list for query_kernel<., true>:
// one atomic per wave with marked reads; list order is irrelevant (work queues deal it).
__global__ __launch_bounds__(256) void k_collect_heavy(const int* __restrict__ fwd, int a0, int a1,
                                                       int* __restrict__ heavy,
                                                       unsigned long long* __restrict__ counters) {
  const int lane = threadIdx.x & 63;
  for (int b = a0 + (blockIdx.x * blockDim.x + threadIdx.x - lane); b < a1; b += gridDim.x * blockDim.x) {
    const int a = b + lane;
    const bool h = a < a1 && fwd[a] < 0;
    const unsigned long long m = __ballot(h);
    if (!m) continue;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(&counters[kHeavyCount], static_cast<unsigned long long>(__popcll(m)));
    base = __shfl(base, 0);
    if (h) heavy[base + mbcnt(m)] = a;
  }
}

// Sum of the per-wave statistics into the counters (after query_kernel).  Each block reduces a
// contiguous slice of waves (thread t: field t % 32, every 8th wave of the slice, so each thread
// has only a few loads in flight), combines its 8 partials in LDS and adds one atomic per field.
// A single block walking all 6144 waves was latency-bound (192 dependent loads per thread: 94 µs).
constexpr int kReduceBlock = 256;
constexpr int kReduceMaxBlocks = 64;
enum WsOp { kOpSum, kOpMax, kOpMinInv, kOpArgPacked };
__device__ __forceinline__ WsOp ws_op(int f) {
  if (f == kWsMaxFwd) return kOpMax;
#ifdef FSLR_SECTION_PROF
  if (f == kWsBase + 8 || f == kWsBase + 10) return kOpMax;
  if (f == kWsBase + 11) return kOpMinInv;       // stored as ~min (counters start at 0)
  if (f == kWsBase + 9) return kOpArgPacked;     // slowest read: min(cycles, 2^38) << 25 | rank
#endif
  return kOpSum;
}

__global__ __launch_bounds__(kReduceBlock) void k_reduce_wstat(const unsigned long long* __restrict__ ws, int nwaves,
                                                               unsigned long long* __restrict__ counters, int* err) {
  constexpr int kGroups = kReduceBlock / kWStride;
  __shared__ unsigned long long val[kGroups][kWStride];
  const int f = threadIdx.x % kWStride, grp = threadIdx.x / kWStride;
  const WsOp op = ws_op(f);
  const int per = (nwaves + gridDim.x - 1) / gridDim.x;
  const int w0 = blockIdx.x * per, w1 = min(w0 + per, nwaves);
  unsigned long long acc = 0ull;
  if (f < kWsProf) {
    for (int w = w0 + grp; w < w1; w += kGroups) {
      const unsigned long long* row = ws + static_cast<long long>(w) * kWStride;
      unsigned long long x = row[f];
      if (op == kOpMinInv) x = ~x;
      if (op == kOpArgPacked) x = (min(row[kWsBase + 8], (1ull << 38) - 1) << 25) | (x & ((1ull << 25) - 1));
      if (op == kOpSum) acc += x;
      else acc = acc > x ? acc : x;
    }
  }
  val[grp][f] = acc;
  __syncthreads();
  if (threadIdx.x >= kWsProf) return;
  const int fi = threadIdx.x;
  const WsOp o = ws_op(fi);
  unsigned long long r = val[0][fi];
  for (int g2 = 1; g2 < kGroups; ++g2) {
    const unsigned long long x = val[g2][fi];
    if (o == kOpSum) r += x;
    else r = r > x ? r : x;
  }
  if (fi == kWsMaxFwd) {
    if (r) atomicMax(err + 3, static_cast<int>(r));
  } else if (fi < kWsBase) {
    const int dst = fi == kWsEval ? kEval : fi == kWsJacc ? kJacc : fi == kWsCand ? kCand
                  : fi == kWsAlgoBytes ? kAlgoBytes : fi == kWsOverflow ? kOverflow
                  : fi == kWsMatchEntries ? kMatchEntries : fi == kWsWalked ? kWalked : kMatchedPairs;
    if (r) atomicAdd(&counters[dst], r);
  } else if (r) {
    if (o == kOpSum) atomicAdd(&counters[kSecBase + (fi - kWsBase)], r);
    else atomicMax(&counters[kSecBase + (fi - kWsBase)], r);
  }
}

// ------------------------------------------------------------------------------------------
// deferred_kernel: one wavefront per deferred entry (grid-stride over the list); B's intervals sit
// in lanes j, A's are broadcast a row at a time with readlane.
//   kDefPair     lenOK pair: first-fit greedy in the reference's order (cluster.py:152-161): for
//                each row i of A, the lowest unused j of B on the same chromosome that either
//                matches or — when an aln_size == 0 interval is involved — raises
//                ZeroDivisionError at the position the reference would (first such candidate).
//   kDefWitness  candidate (A, B, ic, jc) of a read past the hash limit: evaluated only if
//                (jc, ic) is the first overlapping interval pair in B-major order, which makes
//                exactly one candidate of each such pair the evaluator; then gate + as above.
// Forward degrees are added atomically on top of query_kernel's counts.
__global__ __launch_bounds__(256) void deferred_kernel(QueryArgs g) {
  __shared__ unsigned long long es_all[4][kStageCap];
  const int lane = lane_id();
  EdgeStage es{es_all[threadIdx.x >> 6], 0};
  const EdgeOut eo{g.edges, g.edge_iu, g.edge_cap, &g.counters[kEdgeCount]};
  const long long n_all = static_cast<long long>(g.counters[kDeferCount]);
  if (n_all > g.defer_cap && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(g.err + kErrOverflow, 1);
  const long long n = min(n_all, g.defer_cap);
  const int umax_v = g.umax[lane];
  unsigned long long w_eval = 0, w_jacc = 0, w_gather = 0, w_bytes = 0;
  const long long nw = static_cast<long long>(gridDim.x) * (blockDim.x >> 6);
  for (long long t = static_cast<long long>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6); t < n; t += nw) {
    const unsigned long long e = g.defer[t];
    const int a = static_cast<int>(e >> 39);
    const int B = static_cast<int>((e >> 14) & kBMask);
    const int ic = static_cast<int>((e >> 8) & 63u), jc = static_cast<int>((e >> 2) & 63u);
    const unsigned kind = static_cast<unsigned>(e & 3u);
    const int4 am = sload4(g.rmeta, a), bm = sload4(g.rmeta, B);
    const int LA = am.y & 0xffff, LB = bm.y & 0xffff;
    const bool haz = ((am.y | bm.y) >> 16) & 1;
    int4 ai = make_int4(-1, 0, 0, 0), bj = make_int4(-2, 0, 0, 0);
    if (lane < LA) ai = g.iv[am.x + lane];
    if (lane < LB) bj = g.iv[bm.x + lane];
    bool zd = false, lenok = kind == kDefPair, canon = lenok;
    if (kind == kDefWitness) {
      // lane j: does B's interval j overlap (end-inclusive, same chromosome) any of A's?
      unsigned long long ov = 0ull;
      for (int i = 0; i < LA; ++i) {
        const int c = rdl(ai.x, i), si = rdl(ai.y, i), ei = rdl(ai.z, i);
        ov |= static_cast<unsigned long long>(lane < LB && bj.x == c && min(ei, bj.z) >= max(si, bj.y)) << i;
      }
      const unsigned long long jm = __ballot(ov != 0ull);
      const int wj = jm ? __builtin_ctzll(jm) : -1;
      const unsigned long long ovw = wj >= 0 ? __shfl(ov, wj) : 0ull;
      const int wi = ovw ? __builtin_ctzll(ovw) : -1;
      canon = wj == jc && wi == ic;
      if (canon) {
        lenok = lengths_pass(am.z, bm.z, am.w, bm.w, g.qlen_cut, g.nal_cut, &zd);
        if (lane == 0) raise_zd(g.err, zd, a, B);
        ++w_eval;
        w_jacc += lenok;
        w_bytes += 16ull * static_cast<unsigned long long>(LA + LB) + 32ull;
      }
    }
    const bool work = canon && lenok && !zd && g.mode == 0;
    int I = 0;
    if (work) {
      ++w_gather;
      bool used = false;
      for (int i = 0; i < LA; ++i) {
        const int c = rdl(ai.x, i), si = rdl(ai.y, i), ei = rdl(ai.z, i), ti = rdl(ai.w, i);
        const bool cand = lane < LB && !used && bj.x == c;
        const bool zero = haz && cand && (ti == FSLR_THR_ZERO_ALN || bj.w == FSLR_THR_ZERO_ALN);
        const bool hit = cand && (zero || iv_match_general(si, ei, ti, bj.y, bj.z, bj.w));
        const unsigned long long hm = __ballot(hit);
        if (!hm) continue;
        const int j = __builtin_ctzll(hm);
        if (__shfl(static_cast<int>(zero), j)) { zd = true; break; }
        if (lane == j) used = true;
        ++I;
      }
      if (lane == 0) raise_zd(g.err, zd, a, B);
    }
    const int U = LA + LB - I;
    const bool pass = U <= __shfl(umax_v, max(I, 1) - 1);
    const bool edge = pass && work && !zd && I > 0;
    es.put(eo, edge && lane == 0, a, B, I, U, lane);
    if (edge && lane == 0) {
      const int old = atomicAdd(&g.fwd[a], 1);
      atomicMax(g.err + 3, old + 1);
    }
  }
  if (es.n > 0) es.flush(eo, es.n, lane);
  if (lane == 0) {
    if (w_bytes) atomicAdd(&g.counters[kAlgoBytes], w_bytes);
    if (w_eval) atomicAdd(&g.counters[kEval], w_eval);
    if (w_jacc) atomicAdd(&g.counters[kJacc], w_jacc);
    if (w_gather) atomicAdd(&g.counters[kGather], w_gather);
  }
}

// resident grid: waves walk the read ranks grid-stride, so launch exactly what fits on the chip
template <int kThrMode, bool kMulti>
int resident_blocks() {
  static int cached = 0;
  if (cached) return cached;
  int dev = 0, cus = 256, per_cu = 0;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, query_kernel<kThrMode, kMulti>, kBlock, 0) != hipSuccess ||
      per_cu < 1)
    per_cu = 4;
  cached = cus * per_cu;
  return cached;
}

}  // namespace

int query_max_waves() {
  const int b = std::max(std::max(resident_blocks<0, false>(), resident_blocks<1, false>()),
                         std::max(resident_blocks<0, true>(), resident_blocks<1, true>()));
  return b * kWavesPerBlock;
}

hipError_t launch_len_bounds(const int4* rmeta, int a0, int a1, double qcut, double ncut, int4* lb, hipStream_t s) {
  if (a1 > a0) k_len_bounds<<<grid_for(a1 - a0), 256, 0, s>>>(rmeta, a0, a1, qcut, ncut, lb);
  return hipGetLastError();
}

hipError_t launch_query(const QueryArgs& a_in, int thr_mode, hipStream_t s) {
  QueryArgs a = a_in;
  const long long span = static_cast<long long>(a.a_end) - a.a_begin;
  // virtual indices of this shard: its blocks of 64 ranks are k n_shards + shard (query_kernel)
  {
    const long long nb = (span + kShardMask) >> kShardShift;
    const long long m = nb > a.shard ? (nb - 1 - a.shard) / a.n_shards + 1 : 0;
    long long nv = m << kShardShift;
    if (m > 0 && a.shard + (m - 1) * a.n_shards == nb - 1 && (span & kShardMask)) nv -= kWave - (span & kShardMask);
    a.nv = static_cast<int>(nv);
  }
  const long long nq = a.nv;
  if (span > 0) {
    k_len_bounds<<<grid_for(span), 256, 0, s>>>(a.rmeta, a.a_begin, a.a_end, a.qlen_cut, a.nal_cut, a.lb);
    const long long nchunks = (nq + kChunk - 1) / kChunk;
    long long want = (nchunks + kWavesPerBlock - 1) / kWavesPerBlock;
#ifdef FSLR_SECTION_PROF
    if (const char* e = getenv("FSLR_QUERY_BLOCKS")) want = std::min(want, std::max(1ll, atoll(e)));
#endif
    const int cap = thr_mode == 0 ? resident_blocks<0, false>() : resident_blocks<1, false>();
    const int blocks = static_cast<int>(want < cap ? want : cap);
    if (blocks * kWavesPerBlock > a.wstat_waves) return hipErrorInvalidValue;   // capi sizes wstat
    if (blocks > 0) {
      // read assignment (query_kernel): work queues when every wave has many reads (the per-wave
      // imbalance of a static deal is then large and each ticket's atomic is amortised over
      // kChunk reads); a static grid-stride deal when the shard is small (multi-GPU shards)
      const long long nw = static_cast<long long>(blocks) * kWavesPerBlock;
      a.pass_records = kPassRecords;
      // FSLR_PASS_RECORDS (tests): 0 turns partner partitions off, so the hash-overflow (witness)
      // path is exercised at small sizes
      if (const char* e = getenv("FSLR_PASS_RECORDS")) a.pass_records = atoi(e);
      long long dyn_min = kDynamicMinReads;
      // FSLR_DYNAMIC_MIN_READS: lets the parity tests drive the work-queue path at small sizes
      if (const char* e = getenv("FSLR_DYNAMIC_MIN_READS")) dyn_min = std::max(0ll, atoll(e));
      a.k_static = nq >= dyn_min * nw ? 0 : static_cast<int>((nq + nw - 1) / nw);
      if (a.ev_k0) (void)hipEventRecord(a.ev_k0, s);
      if (thr_mode == 0)
        query_kernel<0, false><<<blocks, kBlock, 0, s>>>(a);
      else
        query_kernel<1, false><<<blocks, kBlock, 0, s>>>(a);
      if (a.ev_k1) (void)hipEventRecord(a.ev_k1, s);
      const int nwv = blocks * kWavesPerBlock;
      const int rb = std::min(kReduceMaxBlocks, (nwv + kWave - 1) / kWave);
      k_reduce_wstat<<<rb, kReduceBlock, 0, s>>>(a.wstat, nwv, a.counters, a.err);
      if (a.heavy != nullptr && a.pass_records > 0) {
        // the reads handed over (their number is on the device): a resident grid on work queues
        k_collect_heavy<<<grid_for(span), 256, 0, s>>>(a.fwd, a.a_begin, a.a_end, a.heavy, a.counters);
        const int hb = thr_mode == 0 ? resident_blocks<0, true>() : resident_blocks<1, true>();
        if (hb * kWavesPerBlock > a.wstat_waves) return hipErrorInvalidValue;
        a.k_static = 0;
        if (thr_mode == 0)
          query_kernel<0, true><<<hb, kBlock, 0, s>>>(a);
        else
          query_kernel<1, true><<<hb, kBlock, 0, s>>>(a);
      }
    }
  }
  // the deferred list's length is only known on the device: a fixed grid walks it
  deferred_kernel<<<2048, 256, 0, s>>>(a);
  return hipGetLastError();
}

}  // namespace fslr
