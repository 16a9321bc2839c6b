// query.hip — the pair kernel: replaces the driver of query_interval_trees (cluster.py:187-227)
// with its predicates different_lengths_or_alignments (:178-183), overall_jaccard_similarity
// (:140-170), calculate_overlap (:133-136) and the cutoff lookup (:216-219).
//
// One wavefront per query read A (grid-stride over ranks a in [a_begin, a_end)).  A's intervals
// live in lanes 0..LA-1 and are read wave-uniformly with v_readlane.
//
//  1. candidate walk — A's scan ranges (kernels.hpp: iv_rng) are flattened with a wave prefix
//     sum and walked 64 records per step, one record per lane (4-8 B loads, no wasted reads):
//     forward records are all hits, backward records hit iff end >= start_i.
//  2. dedupe — a hit on read B > A is inserted into a per-wave LDS hash set (epoch-tagged,
//     1024 slots); the first insertion of B is the one evaluation of (A, B), exactly like the
//     reference's seen-set (:205-208).  Reads with more than kHashLimit distinct partners
//     continue in lookup-only mode; partners not in the set are evaluated once by the witness
//     rule (the candidate whose (j, i) is the first overlapping interval pair in B-major order).
//  3. gate queue (LDS) → 64 pairs at a time: read B's record, apply the length / alignment-count
//     gate in IEEE double (bit-identical to Python's int/int true division).
//  4. eval queue (LDS) → 64 pairs at a time: each lane walks B's intervals four rows per load
//     group; per row j the 64-bit match mask M_j over A's intervals feeds the first-fit greedy
//     (m = M_j & free; take lowest).  First-fit greedy is symmetric in (l1, l2) (SURVEY §8a A8,
//     tests/test_oracle_golden.py::test_kat_jaccard_symmetric), so B-major = the reference's
//     A-major count.  Pairs holding an aln_size==0 interval replay the reference loop exactly to
//     raise ZeroDivisionError where the reference does.
//  5. edges (A, B, I, U) are appended with one atomic per wave batch; A's forward degree is the
//     wave's edge count.
#include "fslr_hip.h"
#include "kernels.hpp"

namespace fslr {
namespace {

constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kQueueCap = 2 * kWave;
constexpr int kHashBits = 9;
constexpr int kHashSize = 1 << kHashBits;
constexpr int kHashLimit = 320;           // insert while distinct partners < limit (load <= 75 %)
constexpr int kMatchCap = 256;            // match-list entries per query read
constexpr unsigned kEpochShift = 25;      // key = epoch << 25 | B  (B < FSLR_MAX_READS = 2^25)
constexpr unsigned kEpochMax = 127;
// per-partner state (one word per hash slot)
constexpr unsigned kStLenOk = 1u;         // passed different_lengths_or_alignments
constexpr unsigned kStHaz = 2u;           // holds an aln_size == 0 interval: exact replay
constexpr unsigned kStMatch = 4u;         // has at least one matching interval pair
constexpr unsigned kStSpill = 8u;         // a match did not fit the match list: gather evaluation

__device__ __forceinline__ int lane_id() { return static_cast<int>(__lane_id()); }

__device__ __forceinline__ int mbcnt(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(m >> 32),
                                   __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(m), 0u));
}

__device__ __forceinline__ int rdl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// interval accepts overlap o (fslr_hip.h: thr >= 0 ? o >= thr : o <= ~thr)
__device__ __forceinline__ bool thr_ok(int o, int t) { return t >= 0 ? o >= t : o <= ~t; }

// calculate_overlap(i1, i2) >= overlap (cluster.py:133-136), same chromosome already checked.
template <int kThrMode>
__device__ __forceinline__ bool iv_match(int sa, int ea, int ta, int sb, int eb, int tb) {
  const int o_raw = min(ea, eb) - max(sa, sb);
  if (kThrMode == 0) return o_raw >= max(ta, tb);   // every threshold >= 1: o_raw < 0 never passes
  const int o = max(o_raw, 0);
  return thr_ok(o, ta) && thr_ok(o, tb);
}

// different_lengths_or_alignments (cluster.py:178-183) → true = pair passes (not different);
// *zd = the reference would raise ZeroDivisionError (max == 0).
__device__ __forceinline__ bool lengths_pass(int q1, int q2, int n1, int n2, double qcut, double ncut, bool* zd) {
  int mn = min(q1, q2), mx = max(q1, q2);
  if (mx == 0) { *zd = true; return false; }
  if (static_cast<double>(mn) / static_cast<double>(mx) >= qcut) return true;
  mn = min(n1, n2);
  mx = max(n1, n2);
  if (mx == 0) { *zd = true; return false; }
  return static_cast<double>(mn) / static_cast<double>(mx) >= ncut;
}

template <int kThrMode>
__global__ __launch_bounds__(kBlock) void query_kernel(QueryArgs g) {
  __shared__ unsigned hash_all[kWavesPerBlock][kHashSize];
  __shared__ unsigned state_all[kWavesPerBlock][kHashSize];
  __shared__ unsigned ml_all[kWavesPerBlock][kMatchCap];
  __shared__ unsigned long long eq_all[kWavesPerBlock][kQueueCap];
  __shared__ unsigned short mp_all[kWavesPerBlock][kHashLimit + kWave];
  __shared__ unsigned long long es_all[kWavesPerBlock][kQueueCap];
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  unsigned* H = hash_all[wv];
  unsigned* ST = state_all[wv];
  unsigned* ML = ml_all[wv];
  unsigned short* MP = mp_all[wv];     // partners (hash slots) with at least one match, first-match order
  unsigned long long* ES = es_all[wv]; // staged edges: a << 39 | B << 14 | I << 7 | U
  int esn = 0;
  // edge iff U <= umax[I-1] (cluster.py:218-219 folded on the host); lane l holds umax[l]
  const int umax_v = g.umax[lane];
  // flush nb staged edges with one atomic (a single global counter per edge would serialise)
  auto flush_edges = [&](int nb) {
    wave_lds_sync();
    const bool act = lane < nb;
    const unsigned long long e = act ? ES[lane] : 0ull;
    const int rem = esn - nb;
    const unsigned long long mv = lane < rem ? ES[nb + lane] : 0ull;
    wave_lds_sync();
    if (lane < rem) ES[lane] = mv;
    esn = rem;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(&g.counters[kEdgeCount], static_cast<unsigned long long>(nb));
    base = __shfl(base, 0);
    const long long k = static_cast<long long>(base) + lane;
    if (act && k < g.edge_cap) {
      g.edges[k] = make_int2(static_cast<int>(e >> 39), static_cast<int>((e >> 14) & 0x1FFFFFFull));
      g.edge_iu[k] = static_cast<unsigned short>(((e >> 7) & 127u) | ((e & 127u) << 8));
    }
  };
  unsigned long long* EQ = eq_all[wv];
  for (int k = lane; k < kHashSize; k += kWave) H[k] = 0u;
  unsigned epoch = 0;
  const int nwaves = gridDim.x * kWavesPerBlock;
  unsigned long long w_eval = 0, w_jacc = 0, w_cand = 0, w_over = 0, w_gather = 0, w_ml = 0, w_mp = 0;
  unsigned long long l_bytes = 0;       // per lane: algorithmic bytes of evaluated pairs
  int w_maxfwd = 0;

  for (int a = g.a_begin + blockIdx.x * kWavesPerBlock + wv; a < g.a_end; a += nwaves) {
    if (++epoch > kEpochMax) {
      wave_lds_sync();
      for (int k = lane; k < kHashSize; k += kWave) H[k] = 0u;
      epoch = 1;
    }
    const int4 am = g.rmeta[a];
    const int offA = __builtin_amdgcn_readfirstlane(am.x);
    const int amy = __builtin_amdgcn_readfirstlane(am.y);
    const int LA = amy & 0xffff;
    const bool hazA = (static_cast<unsigned>(amy) >> 16) & 1u;
    const int q1 = __builtin_amdgcn_readfirstlane(am.z), n1 = __builtin_amdgcn_readfirstlane(am.w);
    int4 my = make_int4(-1, 0, 0, 0);
    int4 rg = make_int4(0, 0, 0, 0);
    if (lane < LA) {
      my = g.iv[offA + lane];
      rg = g.iv_rng[offA + lane];
    }
    const unsigned long long fullA = LA == 64 ? ~0ull : ((1ull << LA) - 1ull);
    const int cnt = rg.y + rg.w;
    int pre = cnt;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int t = __shfl_up(pre, o);
      if (lane >= o) pre += t;
    }
    const int ex = pre - cnt;
    const int R = rdl(pre, kWave - 1);
    int en = 0, uniq = 0, mln = 0, mpn = 0, fwdA = 0;

    auto raise_zd = [&](bool zd, int B) {
      if (zd && atomicCAS(g.err, 0, FSLR_ERR_ZERO_DIVISION) == 0) {
        g.err[1] = a;
        g.err[2] = B;
      }
    };

    auto emit = [&](bool edge, int B, int I, int U) {
      const unsigned long long em = __ballot(edge);
      const int ne = __popcll(em);
      if (ne) {
        if (edge)
          ES[esn + mbcnt(em)] = (static_cast<unsigned long long>(a) << 39) |
                                (static_cast<unsigned long long>(B) << 14) |
                                (static_cast<unsigned long long>(I) << 7) | static_cast<unsigned long long>(U);
        esn += ne;
        fwdA += ne;
        if (esn >= kWave) flush_edges(kWave);
      }
    };

    // U <= umax[I-1]  (I in 1..64 → lane I-1)
    auto passes = [&](int I, int U) { return U <= __shfl(umax_v, max(I, 1) - 1); };

    // exact replay of the reference's i-major loop (cluster.py:152-161) for pairs holding an
    // aln_size == 0 interval: ZeroDivisionError exactly when the reference divides by it
    auto replay = [&](int offB, int LB, bool* zd) {
      unsigned long long used = 0ull;
      int I = 0;
      for (int i = 0; i < LA && !*zd; ++i) {
        const int4 ai = g.iv[offA + i];
        for (int j = 0; j < LB; ++j) {
          if ((used >> j) & 1ull) continue;
          const int4 b = g.iv[offB + j];
          if (b.x != ai.x) continue;
          if (ai.w == FSLR_THR_ZERO_ALN || b.w == FSLR_THR_ZERO_ALN) { *zd = true; break; }
          const int o = max(min(ai.z, b.z) - max(ai.y, b.y), 0);
          if (thr_ok(o, ai.w) && thr_ok(o, b.w)) { used |= 1ull << j; ++I; break; }
        }
      }
      return I;
    };

    // gather evaluation: B's intervals are read four rows per load group; B-major first-fit
    // greedy on 64-bit match masks over A (symmetric to the reference's A-major count)
    auto eval_batch = [&](int nb) {
      wave_lds_sync();
      const bool act = lane < nb;
      const unsigned long long e = act ? EQ[lane] : 0ull;
      const int rem = en - nb;
      const unsigned long long mv = lane < rem ? EQ[nb + lane] : 0ull;
      wave_lds_sync();
      if (lane < rem) EQ[lane] = mv;
      en = rem;
      w_gather += nb;
      const unsigned lo = static_cast<unsigned>(e);
      const int B = static_cast<int>(lo & 0x1FFFFFFu);
      const int LB = act ? static_cast<int>((lo >> 25) & 63u) + 1 : 0;
      const bool haz = (lo >> 31) & 1u;
      const int offB = static_cast<int>(e >> 32);
      unsigned long long freeA = fullA;
      int I = 0;
      bool zd = false;
      if (!haz) {
        for (int j0 = 0; j0 < LB; j0 += 4) {
          int4 b[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) b[u] = (j0 + u < LB) ? g.iv[offB + j0 + u] : make_int4(-1, 0, -1, 0);
          unsigned long long M[4] = {0ull, 0ull, 0ull, 0ull};
          for (int i = 0; i < LA; ++i) {
            const int ci = rdl(my.x, i), si = rdl(my.y, i), ei = rdl(my.z, i), ti = rdl(my.w, i);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const bool mt = b[u].x == ci && iv_match<kThrMode>(si, ei, ti, b[u].y, b[u].z, b[u].w);
              M[u] |= static_cast<unsigned long long>(mt) << i;
            }
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const unsigned long long m = M[u] & freeA;
            if (m) { freeA ^= m & (~m + 1ull); ++I; }
          }
        }
      } else if (act) {
        I = replay(offB, LB, &zd);
      }
      raise_zd(act && zd, B);
      const int U = LA + LB - I;
      const bool edge = passes(I, U) && act && !zd && I > 0;
      emit(edge, B, I, U);
    };

    auto push_eval = [&](bool push, int B, int offB, int LB, bool haz) {
      const unsigned long long pm = __ballot(push);
      if (push) {
        const unsigned tag = static_cast<unsigned>(B) | (static_cast<unsigned>(LB - 1) << 25) |
                             (static_cast<unsigned>(haz) << 31);
        EQ[en + mbcnt(pm)] = (static_cast<unsigned long long>(static_cast<unsigned>(offB)) << 32) | tag;
      }
      en += __popcll(pm);
      if (en >= kWave) eval_batch(kWave);
    };

    // partners past the hash limit: witness rule (first overlapping pair in B-major order), in place
    auto witness_batch = [&](bool act, int B, int ic, int jc, int4 bm) {
      const int offB = bm.x;
      const int LB = act ? (bm.y & 0xffff) : 0;
      const bool haz = hazA || ((bm.y >> 16) & 1);
      bool zd = false;
      const bool lenok = act && lengths_pass(q1, bm.z, n1, bm.w, g.qlen_cut, g.nal_cut, &zd);
      const bool full = lenok && !haz && g.mode == 0;
      unsigned long long freeA = fullA;
      int I = 0;
      int state = act ? 0 : 2;   // 0 witness unknown, 1 canonical, 2 duplicate / idle
      for (int j = 0; j < LB; ++j) {
        const int4 b = g.iv[offB + j];
        unsigned long long O = 0ull, M = 0ull;
        for (int i = 0; i < LA; ++i) {
          const int ci = rdl(my.x, i), si = rdl(my.y, i), ei = rdl(my.z, i), ti = rdl(my.w, i);
          const bool same = b.x == ci;
          O |= static_cast<unsigned long long>(same && min(b.z, ei) >= max(b.y, si)) << i;
          M |= static_cast<unsigned long long>(same && iv_match<kThrMode>(si, ei, ti, b.y, b.z, b.w)) << i;
        }
        if (state == 0 && O != 0ull) state = (j == jc && __builtin_ctzll(O) == ic) ? 1 : 2;
        if (state == 2 || (state == 1 && !full)) break;
        const unsigned long long m = M & freeA;
        if (m) { freeA ^= m & (~m + 1ull); ++I; }
      }
      const bool canon = state == 1;
      if (canon && lenok && haz && g.mode == 0) I = replay(offB, LB, &zd);
      raise_zd(canon && zd, B);
      const unsigned long long cm = __ballot(canon);
      w_eval += __popcll(cm);
      w_gather += __popcll(cm);
      w_jacc += __popcll(__ballot(canon && lenok));
      if (canon) l_bytes += 16ull * static_cast<unsigned long long>(LA + LB) + 32ull;
      const int U = LA + LB - I;
      const bool edge = passes(I, U) && canon && lenok && !zd && g.mode == 0 && I > 0;
      emit(edge, B, I, U);
    };

    // ---- 1. candidate walk over A's flattened scan ranges -------------------------------
    for (int base = 0; base < R; base += kWave) {
      const int r = base + lane;
      const bool valid = r < R;
      const int i0 = __popcll(__ballot(lane < LA && pre <= base));
      int mi = i0;
      for (int k = i0 + 1; k < LA; ++k) {
        const int exk = rdl(ex, k);
        if (exk >= base + kWave) break;
        if (r >= exk) mi = k;
      }
      const int q_i = __shfl(rg.x, mi), nf_i = __shfl(rg.y, mi), bb_i = __shfl(rg.z, mi);
      const int ex_i = __shfl(ex, mi);
      const int s_i = __shfl(my.y, mi), e_i = __shfl(my.z, mi), t_i = __shfl(my.w, mi);
      const int loc = r - ex_i;
      const bool fwd = loc < nf_i;
      const int p = fwd ? q_i + 1 + loc : bb_i + (loc - nf_i);
      int4 rec = make_int4(0, -1, 0, 0);
      if (valid) rec = g.idx4[p];
      const bool hit = valid && (fwd || rec.y >= s_i);
      w_cand += __popcll(__ballot(hit));
      const int B = rec.w >> 6;
      const bool cand = hit && B > a;
      // ---- 2. dedupe: per-wave LDS hash set of partners (the reference's seen-set) -------
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
      if (g.mode == 1) continue;
      // ---- 3. gate at first sight: B's read record sits beside its interval record -------
      int4 bm = make_int4(0, 0, 0, 0);
      if (isnew || over) bm = g.idx_meta[p];
      const int LB = bm.y & 0xffff;
      const bool haz = hazA || ((bm.y >> 16) & 1);
      bool zd = false;
      const bool lenok = isnew && lengths_pass(q1, bm.z, n1, bm.w, g.qlen_cut, g.nal_cut, &zd);
      raise_zd(isnew && zd, B);
      if (isnew) {
        ST[h] = (lenok ? kStLenOk : 0u) | (haz ? kStHaz : 0u) | (static_cast<unsigned>(LB) << 8);
        l_bytes += 16ull * static_cast<unsigned long long>(LA + LB) + 32ull;
      }
      w_eval += __popcll(nm);
      w_jacc += __popcll(__ballot(lenok));
      wave_lds_sync();
      // pairs evaluated by gathering B's intervals: every pair under general thresholds,
      // aln_size == 0 replays
      push_eval(lenok && g.mode == 0 && (kThrMode == 1 || haz), B, bm.x, LB, haz);
      // ---- 4. matching interval pairs → match list (A-major order: i never decreases) -----
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
      const unsigned long long om = __ballot(over);
      if (om) {
        w_over += __popcll(om);
        witness_batch(over, B, mi, rec.w & 63, bm);
      }
    }
    // ---- 5. first-fit greedy from the match list, one lane per matched partner ------------
    if (kThrMode == 0 && g.mode == 0 && mpn > 0) {
      wave_lds_sync();
      for (int k0 = 0; k0 < mpn; k0 += kWave) {
        const bool act = k0 + lane < mpn;
        const int h = act ? static_cast<int>(MP[k0 + lane]) : 0;
        const unsigned key = H[h];
        const unsigned st = act ? ST[h] : 0u;
        const bool hasm = act && (st & kStLenOk) && !(st & kStHaz);
        const bool spill = hasm && (st & kStSpill);
        const bool need = hasm && !spill;
        const int B = static_cast<int>(key & 0x1FFFFFFu);
        const int LB = static_cast<int>((st >> 8) & 0xffu);
        int I = 0;
        if (__ballot(need)) {
          // reference order (cluster.py:152-161): rows i of A ascending, lowest unused j of B
          unsigned long long used = 0ull, rowm = 0ull;
          int cur = -1;
          for (int k = 0; k < mln; ++k) {
            const unsigned e = ML[k];
            if (need && static_cast<int>(e & (kHashSize - 1)) == h) {
              const int i = static_cast<int>((e >> kHashBits) & 63u);
              const int j = static_cast<int>((e >> (kHashBits + 6)) & 63u);
              if (i != cur) {
                const unsigned long long m = rowm & ~used;
                if (m) { used |= m & (~m + 1ull); ++I; }
                rowm = 0ull;
                cur = i;
              }
              rowm |= 1ull << j;
            }
          }
          const unsigned long long m = rowm & ~used;
          if (m) { used |= m & (~m + 1ull); ++I; }
        }
        const int U = LA + LB - I;
        const bool edge = passes(I, U) && need && I > 0;
        emit(edge, B, I, U);
        int4 bm = make_int4(0, 0, 0, 0);
        if (spill) bm = g.rmeta[B];
        push_eval(spill, B, bm.x, LB, false);
      }
    }
    while (en > 0) eval_batch(min(en, kWave));
    w_ml += mln;
    w_mp += mpn;
    if (lane == 0) g.fwd[a] = fwdA;
    w_maxfwd = max(w_maxfwd, fwdA);
  }
  if (esn > 0) flush_edges(esn);
  for (int o = 32; o > 0; o >>= 1) l_bytes += __shfl_xor(l_bytes, o);
  if (lane == 0) {
    if (l_bytes) atomicAdd(&g.counters[kAlgoBytes], l_bytes);
    if (w_eval) atomicAdd(&g.counters[kEval], w_eval);
    if (w_jacc) atomicAdd(&g.counters[kJacc], w_jacc);
    if (w_cand) atomicAdd(&g.counters[kCand], w_cand);
    if (w_over) atomicAdd(&g.counters[kOverflow], w_over);
    if (w_gather) atomicAdd(&g.counters[kGather], w_gather);
    if (w_ml) atomicAdd(&g.counters[kMatchEntries], w_ml);
    if (w_mp) atomicAdd(&g.counters[kMatchedPairs], w_mp);
    if (w_maxfwd) atomicMax(g.err + 3, w_maxfwd);
  }
}

}  // namespace

// resident grid: waves walk the read ranks grid-stride, so launch exactly what fits on the chip
template <int kThrMode>
int resident_blocks() {
  static int cached = 0;
  if (cached) return cached;
  int dev = 0, cus = 256, per_cu = 0;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, query_kernel<kThrMode>, kBlock, 0) != hipSuccess ||
      per_cu < 1)
    per_cu = 4;
  cached = cus * per_cu;
  return cached;
}

hipError_t launch_query(const QueryArgs& a, int thr_mode, hipStream_t s) {
  const long long nq = static_cast<long long>(a.a_end) - a.a_begin;
  if (nq <= 0) return hipSuccess;
  const long long want = (nq + kWavesPerBlock - 1) / kWavesPerBlock;
  if (thr_mode == 0) {
    const int cap = resident_blocks<0>();
    query_kernel<0><<<static_cast<int>(want < cap ? want : cap), kBlock, 0, s>>>(a);
  } else {
    const int cap = resident_blocks<1>();
    query_kernel<1><<<static_cast<int>(want < cap ? want : cap), kBlock, 0, s>>>(a);
  }
  return hipGetLastError();
}

}  // namespace fslr
