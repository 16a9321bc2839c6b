// cap.hip — the reference's per-query-read edge cap, replayed exactly (cluster.py:197-224).
//
// The reference's driver walks the reads in rank order; read x's loop visits, interval by
// interval (its `data` order), the superintervals hits of that interval (cluster.py:201) and
//   skips its own intervals (:203-204) and pairs already seen (:205-207), marks the pair seen
//   (:208), skips it on the length gate (:209-210) or when no interval pair matches (:216-217),
//   adds an edge when I/U >= cut(I) (:218-222), and leaves the current interval's hit list as
//   soon as its edge count reaches edge_threshold (:223-224) — only that inner loop: every later
//   interval still visits hits up to the next pair that passes the gate with I > 0.
// The pair kernels compute E* (every candidate pair evaluated).  E* is the reference's graph
// whenever no read has more than edge_threshold forward E* partners.  When one
// does, fslr_apply_edge_cap replays the reference's loops on the host for the reads that can
// reach the cap and rewrites the device edge list:
//   1. candidates T: in rank order, x joins T when fwd(x) + #{y in T, y < x, (y, x) in E*} >=
//      edge_threshold.  A read's loop breaks only if its edge count reaches the cap; the edges it
//      can form are its forward E* pairs plus E* pairs (y, x) that an earlier *breaking* read y
//      left unseen, so T contains every read that breaks.
//   2. k_hit_emit lists every hit of every interval of the reads in T from the device index (the
//      same end-inclusive overlaps the pair kernel walks); the host orders each interval's hits
//      the way the search returns them (descending (start, -end, data position) — the order of
//      the superintervals stand-in the golden fixtures were generated with; the library's own
//      order is undocumented, SURVEY.md §8c: parity is pinned to that stand-in order).
//   3. k_eval_pairs evaluates every distinct pair of those hit lists with the full predicate.
//   4. the host replays the loops of T in rank order; a pair (y, x), y < x, is unseen at x's loop
//      iff y broke before reaching it.  An E* pair is an edge iff the loop of its lower-rank read
//      or, failing that, of its higher-rank read reaches it.
// Edges are re-oriented as (the read whose loop formed it, the partner), like the reference's
// match set (:220); forward degrees become the edges formed in each read's own loop.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

#include "ctx.hpp"
#include "kernels.hpp"

namespace fslr {
namespace {

__device__ __forceinline__ int mbcnt64(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(m >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(m), 0u));
}

__global__ void k_hit_counts(const int* __restrict__ reads, int n, const int4* __restrict__ rmeta,
                             const int* __restrict__ qpos, const int2* __restrict__ rng_s,
                             long long* __restrict__ counts) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
    const int4 m = rmeta[reads[t]];
    const int len = m.y & 0xffff;
    long long c = 0;
    for (int i = 0; i < len; ++i) {
      const int q = qpos[m.x + i];
      const int2 rs = rng_s[q];
      c += static_cast<long long>(rs.x) + (q - rs.y) + 1;
    }
    counts[t] = c;
  }
}

// one wavefront per listed read; positions bwd_begin .. q + n_fwd of each interval, 64 per step
__global__ __launch_bounds__(256) void k_hit_emit(const int* __restrict__ reads, int n, const long long* __restrict__ off,
                                                  const int4* __restrict__ rmeta, const int* __restrict__ qpos,
                                                  const int2* __restrict__ rng_s, const int4* __restrict__ idx4,
                                                  int4* __restrict__ hits, int* __restrict__ nout) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int t = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < n; t += nw) {
    const int4 m = rmeta[reads[t]];
    const int len = m.y & 0xffff;
    const long long base = off[t];
    int w = 0;
    for (int i = 0; i < len; ++i) {
      const int q = qpos[m.x + i];
      const int2 rs = rng_s[q];
      const int s = idx4[q].x;
      const int hi = q + rs.x;
      for (int p0 = rs.y; p0 <= hi; p0 += 64) {
        const int p = p0 + lane;
        int4 rec = make_int4(0, -1, 0, 0);
        if (p <= hi) rec = idx4[p];
        const bool hit = p <= hi && (p >= q || rec.y >= s);
        const unsigned long long hm = __ballot(hit);
        if (hit) hits[base + w + mbcnt64(hm)] = make_int4(rec.w >> 6, i, rec.x, rec.y);
        w += __popcll(hm);
      }
    }
    if (lane == 0) nout[t] = w;
  }
}

// one wavefront per pair: B's intervals in lanes, A's rows broadcast (the deferred kernel's gather
// evaluation, query.hip), reporting the predicate's parts instead of appending an edge
__global__ __launch_bounds__(256) void k_eval_pairs(const int2* __restrict__ pairs, long long n,
                                                    const int4* __restrict__ rmeta, const int4* __restrict__ iv,
                                                    double qcut, double ncut, const int* __restrict__ umax,
                                                    int* __restrict__ flags) {
  const int lane = threadIdx.x & 63;
  const long long nw = static_cast<long long>(gridDim.x) * (blockDim.x >> 6);
  const int umax_v = umax[lane];
  for (long long t = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < n; t += nw) {
    const int2 pr = pairs[t];
    const int4 am = rmeta[pr.x], bm = rmeta[pr.y];
    const int LA = am.y & 0xffff, LB = bm.y & 0xffff;
    int4 ai = make_int4(-1, 0, 0, 0), bj = make_int4(-2, 0, 0, 0);
    if (lane < LA) ai = iv[am.x + lane];
    if (lane < LB) bj = iv[bm.x + lane];
    bool zd = false;
    const bool lenok = lengths_pass(am.z, bm.z, am.w, bm.w, qcut, ncut, &zd);
    int I = 0;
    if (lenok && !zd) {
      bool used = false;
      for (int i = 0; i < LA; ++i) {
        const int c = __builtin_amdgcn_readlane(ai.x, i), si = __builtin_amdgcn_readlane(ai.y, i);
        const int ei = __builtin_amdgcn_readlane(ai.z, i), ti = __builtin_amdgcn_readlane(ai.w, i);
        const bool cand = lane < LB && !used && bj.x == c;
        const bool zero = cand && (ti == FSLR_THR_ZERO_ALN || bj.w == FSLR_THR_ZERO_ALN);
        const bool hit = cand && (zero || iv_match_general(si, ei, ti, bj.y, bj.z, bj.w));
        const unsigned long long hm = __ballot(hit);
        if (!hm) continue;
        const int j = __builtin_ctzll(hm);
        if (__shfl(static_cast<int>(zero), j)) { zd = true; break; }
        if (lane == j) used = true;
        ++I;
      }
    }
    const int U = LA + LB - I;
    const bool edge = lenok && !zd && I > 0 && U <= __shfl(umax_v, max(I, 1) - 1);
    if (lane == 0)
      flags[t] = static_cast<int>(zd) | (static_cast<int>(lenok && !zd) << 1) | (static_cast<int>(edge) << 2) |
                 (I << 8) | (U << 20);
  }
}

}  // namespace

hipError_t launch_cap_hit_counts(const int* reads, int n, const int4* rmeta, const int* qpos, const int2* rng_s,
                                 long long* counts, hipStream_t s) {
  if (n > 0) k_hit_counts<<<grid_for(n), 256, 0, s>>>(reads, n, rmeta, qpos, rng_s, counts);
  return hipGetLastError();
}

hipError_t launch_cap_hit_emit(const int* reads, int n, const long long* off, const int4* rmeta, const int* qpos,
                               const int2* rng_s, const int4* idx4, int4* hits, int* nout, hipStream_t s) {
  if (n > 0) k_hit_emit<<<std::min(4096, (n + 3) / 4), 256, 0, s>>>(reads, n, off, rmeta, qpos, rng_s, idx4, hits, nout);
  return hipGetLastError();
}

hipError_t launch_eval_pairs(const int2* pairs, long long n, const int4* rmeta, const int4* iv, double qcut,
                             double ncut, const int* umax, int* flags, hipStream_t s) {
  if (n > 0)
    k_eval_pairs<<<static_cast<int>(std::min<long long>(8192, (n + 3) / 4)), 256, 0, s>>>(pairs, n, rmeta, iv, qcut,
                                                                                          ncut, umax, flags);
  return hipGetLastError();
}

}  // namespace fslr

using namespace fslr;

namespace {

// device scratch freed on every exit path
struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

constexpr int kFlagZd = 1, kFlagLenOk = 2, kFlagEdge = 4;

// f(begin, end) over [0, n) split across the host's cores
template <typename F>
void parallel_for(int n, F&& f) {
  const int hw = static_cast<int>(std::max(1u, std::thread::hardware_concurrency()));
  const int nth = std::max(1, std::min({hw, 16, n / 256}));
  if (nth == 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int k = 0; k < nth; ++k) {
    const int b = static_cast<int>(static_cast<long long>(n) * k / nth);
    const int e = static_cast<int>(static_cast<long long>(n) * (k + 1) / nth);
    th.emplace_back([&f, b, e] { f(b, e); });
  }
  for (auto& x : th) x.join();
}

// f(tid, begin, end) over [0, n) in `nth` contiguous ranges, one thread each (range k = thread k)
template <typename F>
void parallel_ranges(int64_t n, int nth, F&& f) {
  if (nth <= 1) {
    f(0, int64_t(0), n);
    return;
  }
  std::vector<std::thread> th;
  for (int k = 0; k < nth; ++k) {
    const int64_t b = n * k / nth, e = n * (k + 1) / nth;
    th.emplace_back([&f, k, b, e] { f(k, b, e); });
  }
  for (auto& x : th) x.join();
}

int host_threads(int64_t work) {
  const int hw = static_cast<int>(std::max(1u, std::thread::hardware_concurrency()));
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>({hw, 16, work / (1 << 16)})));
}

}  // namespace

extern "C" int fslr_apply_edge_cap(fslr_ctx* c, int32_t thr, fslr_cap_stats* out) {
  if (!c) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  fslr_cap_stats cs;
  std::memset(&cs, 0, sizeof(cs));
  unsigned long long ne_u = 0;
  int ew[4] = {};
  if (c->counters) {
    long long pk[3];
    if (int rc = peek_counts(c, pk)) return rc;
    ne_u = static_cast<unsigned long long>(pk[0]);
    ew[0] = static_cast<int>(pk[1]);
    ew[3] = static_cast<int>(pk[2]);
  } else {
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  if (ew[0] == FSLR_ERR_ZERO_DIVISION) return fail(c, FSLR_ERR_ZERO_DIVISION, "division by zero");
  const int64_t ne = static_cast<int64_t>(ne_u);
  if (ne > c->edge_cap) return fail(c, FSLR_ERR_STATE, "edge buffer overflowed; reserve and rerun the query");
  cs.max_fwd = ew[3];
  if (c->cap_stats.applied || ew[3] <= thr) {   // E* is the reference's graph (or already replayed)
    if (!c->cap_stats.applied) c->cap_stats = cs;
    if (out) *out = c->cap_stats;
    return FSLR_OK;
  }
  if (!c->last_full)
    return fail(c, FSLR_ERR_STATE, "the edge cap binds: its replay needs the last query to cover every read on "
                                   "one context (fslr_query over [0, n_reads))");
  if (int rc = ensure_walk_index(c)) return rc;       // the replayed loops walk qpos and the scan ranges
  const int64_t n = c->n;
  // FSLR_CAP_TIMING=1: host wall time per stage on stderr (diagnostics)
  const bool timing = std::getenv("FSLR_CAP_TIMING") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  auto stage = [&](const char* what) {
    if (!timing) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[cap] %-28s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(now - t_last).count());
    t_last = now;
  };
  // uninitialised host arrays (the D2H copies fill them; zero-filling 0.2 GB at cfg5 cost ~40 ms)
  std::unique_ptr<int[]> fwd_buf(new int[static_cast<size_t>(std::max<int64_t>(n, 1))]);
  std::unique_ptr<int2[]> edges_buf(new int2[static_cast<size_t>(std::max<int64_t>(ne, 1))]);
  std::unique_ptr<unsigned short[]> iu_buf(new unsigned short[static_cast<size_t>(std::max<int64_t>(ne, 1))]);
  int* const fwd = fwd_buf.get();
  int2* const edges = edges_buf.get();
  unsigned short* const iu = iu_buf.get();
  HIP_TRY(c, hipMemcpyAsync(fwd, c->fwd, n * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  if (ne) {
    HIP_TRY(c, hipMemcpyAsync(edges, c->edges, ne * sizeof(int2), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipMemcpyAsync(iu, c->edge_iu, ne * sizeof(unsigned short), hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));

  // forward adjacency of E* (edges are (a, b), a < b, from the pair kernels); rows are filled by
  // several threads, so a row's order is arbitrary (the closure below only counts over rows)
  const int nth_e = host_threads(ne);
  std::vector<int64_t> aoff(static_cast<size_t>(n) + 1, 0);
  std::vector<char> bad(static_cast<size_t>(nth_e), 0);
  parallel_ranges(ne, nth_e, [&](int tid, int64_t b, int64_t e) {
    for (int64_t k = b; k < e; ++k) {
      const int2 ed = edges[k];
      if (ed.x >= ed.y || ed.x < 0 || ed.y >= n) {
        bad[tid] = 1;
        return;
      }
      __atomic_fetch_add(&aoff[ed.x + 1], 1, __ATOMIC_RELAXED);
    }
  });
  for (char b : bad)
    if (b) return fail(c, FSLR_ERR_STATE, "edge list is not E* (a < b)");
  for (int64_t x = 0; x < n; ++x) aoff[x + 1] += aoff[x];
  std::vector<int> adj(static_cast<size_t>(ne));
  {
    std::vector<int64_t> fill(aoff.begin(), aoff.end() - 1);
    parallel_ranges(ne, nth_e, [&](int, int64_t b, int64_t e) {
      for (int64_t k = b; k < e; ++k)
        adj[__atomic_fetch_add(&fill[edges[k].x], 1, __ATOMIC_RELAXED)] = edges[k].y;
    });
  }
  stage("D2H fwd + edges, adjacency");
  // 1. candidate readers T (closure bound, rank order)
  std::vector<int> back(static_cast<size_t>(n), 0);
  std::vector<char> in_t(static_cast<size_t>(n), 0);
  std::vector<int> T;
  for (int64_t x = 0; x < n; ++x) {
    if (fwd[x] + back[x] < thr) continue;
    in_t[x] = 1;
    T.push_back(static_cast<int>(x));
    for (int64_t k = aoff[x]; k < aoff[x + 1]; ++k) ++back[adj[k]];
  }
  cs.candidates = static_cast<int64_t>(T.size());
  const int nt = static_cast<int>(T.size());

  stage("closure T");
  // 2. hit lists of the candidates from the device index
  DevBuf d_reads, d_cnt, d_hits, d_nout;
  HIP_TRY(c, hipMalloc(&d_reads.p, std::max(1, nt) * sizeof(int)));
  HIP_TRY(c, hipMalloc(&d_cnt.p, std::max(1, nt) * sizeof(long long)));
  HIP_TRY(c, hipMemcpyAsync(d_reads.p, T.data(), nt * sizeof(int), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, launch_cap_hit_counts(static_cast<int*>(d_reads.p), nt, c->rmeta, c->qpos, c->rng_s,
                                   static_cast<long long*>(d_cnt.p), c->stream));
  std::vector<long long> hoff(static_cast<size_t>(nt) + 1, 0);
  HIP_TRY(c, hipMemcpyAsync(hoff.data() + 1, d_cnt.p, nt * sizeof(long long), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  for (int t = 0; t < nt; ++t) hoff[t + 1] += hoff[t];
  const long long cap_hits = hoff[nt];
  HIP_TRY(c, hipMemcpyAsync(d_cnt.p, hoff.data(), nt * sizeof(long long), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipMalloc(&d_hits.p, std::max(1ll, cap_hits) * sizeof(int4)));
  HIP_TRY(c, hipMalloc(&d_nout.p, std::max(1, nt) * sizeof(int)));
  HIP_TRY(c, launch_cap_hit_emit(static_cast<int*>(d_reads.p), nt, static_cast<long long*>(d_cnt.p), c->rmeta,
                                 c->qpos, c->rng_s, c->idx4, static_cast<int4*>(d_hits.p),
                                 static_cast<int*>(d_nout.p), c->stream));
  std::vector<int4> hits(static_cast<size_t>(cap_hits));
  std::vector<int> nout(static_cast<size_t>(nt));
  if (cap_hits) HIP_TRY(c, hipMemcpyAsync(hits.data(), d_hits.p, cap_hits * sizeof(int4), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipMemcpyAsync(nout.data(), d_nout.p, nt * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));

  stage("hit lists (device) + D2H");
  // search order of each interval: the stand-in sorts by (start asc, end desc, data position asc)
  // and returns hits from the highest sorted position down.  Device positions of equal start are
  // in data order, so reading an interval's hits backwards is that order except inside runs of
  // equal start, which are stably re-sorted on (start asc, end desc) first.  seq: per read,
  // partners in visit order, -1 after each interval; own intervals dropped (cluster.py:203-204).
  // uq: per read, its distinct partners (sorted) — the pairs evaluated in step 3, flags aligned.
  std::vector<int64_t> soff(static_cast<size_t>(nt) + 1, 0), uoff(static_cast<size_t>(nt) + 1, 0);
  for (int t = 0; t < nt; ++t) {
    soff[t + 1] = soff[t] + nout[t] + 64;            // hits + one separator per interval (<= 64)
    uoff[t + 1] = uoff[t] + nout[t];
  }
  std::vector<int> seq(static_cast<size_t>(soff[nt]), -2);   // -2: unused tail of a read's slot
  std::vector<int> uq(static_cast<size_t>(uoff[nt]));
  std::vector<int> nuq(static_cast<size_t>(nt), 0);
  parallel_for(nt, [&](int t0, int t1) {
    std::vector<int> tmp;
    for (int t = t0; t < t1; ++t) {
      const int x = T[t];
      int4* h = hits.data() + hoff[t];
      const int cnt = nout[t];
      int64_t w = soff[t];
      tmp.clear();
      int g0 = 0;
      while (g0 < cnt) {
        int g1 = g0 + 1;
        bool ties = false;
        while (g1 < cnt && h[g1].y == h[g0].y) {
          ties |= h[g1].z == h[g1 - 1].z;
          ++g1;
        }
        if (ties)
          std::stable_sort(h + g0, h + g1, [](const int4& u, const int4& v) {
            return u.z != v.z ? u.z < v.z : u.w > v.w;
          });
        for (int k = g1 - 1; k >= g0; --k)
          if (h[k].x != x) {
            seq[w++] = h[k].x;
            tmp.push_back(h[k].x);
          }
        seq[w++] = -1;
        g0 = g1;
      }
      std::sort(tmp.begin(), tmp.end());
      tmp.erase(std::unique(tmp.begin(), tmp.end()), tmp.end());
      std::copy(tmp.begin(), tmp.end(), uq.begin() + uoff[t]);
      nuq[t] = static_cast<int>(tmp.size());
    }
  });
  for (int t = 0; t < nt; ++t) cs.hits += nout[t];
  std::vector<int4>().swap(hits);
  // compact the distinct partner lists (pairs of step 3, one per (read of T, partner))
  {
    int64_t w = 0;
    for (int t = 0; t < nt; ++t) {
      std::copy(uq.begin() + uoff[t], uq.begin() + uoff[t] + nuq[t], uq.begin() + w);
      uoff[t] = w;
      w += nuq[t];
    }
    uoff[nt] = w;
    uq.resize(static_cast<size_t>(w));
  }
  cs.pairs = static_cast<int64_t>(uq.size());

  stage("visit order + partner lists");
  // 3. the full predicate of every (read of T, partner) pair
  std::vector<int> flags(uq.size());
  if (!uq.empty()) {
    std::vector<int2> pv(uq.size());
    parallel_for(nt, [&](int t0, int t1) {
      for (int t = t0; t < t1; ++t)
        for (int64_t k = uoff[t]; k < uoff[t + 1]; ++k) pv[k] = make_int2(std::min(T[t], uq[k]), std::max(T[t], uq[k]));
    });
    DevBuf d_pairs, d_flags;
    HIP_TRY(c, hipMalloc(&d_pairs.p, pv.size() * sizeof(int2)));
    HIP_TRY(c, hipMalloc(&d_flags.p, pv.size() * sizeof(int)));
    HIP_TRY(c, hipMemcpyAsync(d_pairs.p, pv.data(), pv.size() * sizeof(int2), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, launch_eval_pairs(static_cast<int2*>(d_pairs.p), static_cast<long long>(pv.size()), c->rmeta, c->iv,
                                 c->last_qcut, c->last_ncut, c->umax, static_cast<int*>(d_flags.p), c->stream));
    HIP_TRY(c, hipMemcpyAsync(flags.data(), d_flags.p, flags.size() * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  std::vector<int> t_of(static_cast<size_t>(n), -1);
  for (int t = 0; t < nt; ++t) t_of[T[t]] = t;
  auto flag_of = [&](int x, int y) {   // x in T
    const int t = t_of[x];
    return flags[std::lower_bound(uq.begin() + uoff[t], uq.begin() + uoff[t + 1], y) - uq.begin()];
  };

  stage("pair predicates (device)");
  // 4. the loops of T in rank order
  std::vector<char> broke(static_cast<size_t>(n), 0);
  std::vector<int64_t> roff(static_cast<size_t>(nt) + 1, 0);   // reached partners of read T[t] (sorted)
  std::vector<int> reached;
  std::vector<int> stamp(static_cast<size_t>(n), -1);
  std::vector<int> own_edges(static_cast<size_t>(nt), 0);
  auto reached_by = [&](int y, int x) {   // did broken read y's loop reach x?
    const int t = t_of[y];
    return std::binary_search(reached.begin() + roff[t], reached.begin() + roff[t + 1], x);
  };
  for (int t = 0; t < nt; ++t) {
    const int x = T[t];
    int edges_x = 0;
    bool br = false;
    const size_t r0 = reached.size();
    for (int64_t k = soff[t]; k < soff[t + 1]; ++k) {
      const int y = seq[k];
      if (y == -2) break;                                      // end of this read's hits
      if (y < 0) continue;                                     // next interval
      if (stamp[y] == x) continue;                             // seen in this loop
      if (y < x && (!broke[y] || reached_by(y, x))) continue;  // seen in y's loop
      stamp[y] = x;
      reached.push_back(y);
      const int f = flag_of(x, y);
      if (f & kFlagZd) return fail(c, FSLR_ERR_ZERO_DIVISION, "division by zero");
      if (!(f & kFlagLenOk) || ((f >> 8) & 0xfff) == 0) continue;
      if (f & kFlagEdge) ++edges_x;
      if (edges_x >= thr) {
        br = true;
        while (k + 1 < soff[t + 1] && seq[k + 1] >= 0) ++k;   // leave this interval's hits
      }
    }
    own_edges[t] = edges_x;
    if (br) {
      broke[x] = 1;
      ++cs.capped;
      std::sort(reached.begin() + static_cast<int64_t>(r0), reached.end());
    } else {
      reached.resize(r0);                                      // reached everything: not stored
    }
    roff[t + 1] = static_cast<int64_t>(reached.size());
  }

  stage("replay loops");
  // E* pair (a, b) is an edge iff a's loop or, failing that, b's loop reaches it
  // (in parallel: per-range codes and counts, then each range compacts at its scanned offset, so the
  // kept edges stay in E* order)
  std::vector<unsigned char> who(static_cast<size_t>(ne));          // 0 a's loop, 1 b's loop, 2 none
  std::vector<int64_t> rkept(static_cast<size_t>(nth_e) + 1, 0), rdrop(static_cast<size_t>(nth_e), 0),
      rback(static_cast<size_t>(nth_e), 0);
  std::vector<int> formed(static_cast<size_t>(n), 0);
  parallel_ranges(ne, nth_e, [&](int tid, int64_t b0, int64_t e0) {
    int64_t kc = 0, dc = 0, bc = 0;
    for (int64_t k = b0; k < e0; ++k) {
      const int a = edges[k].x, b = edges[k].y;
      unsigned char w = 2;
      if (!broke[a] || reached_by(a, b)) w = 0;
      else if (!broke[b] || reached_by(b, a)) w = 1;
      who[k] = w;
      if (w == 2) {
        ++dc;
        continue;
      }
      ++kc;
      bc += w;
      __atomic_fetch_add(&formed[w == 0 ? a : b], 1, __ATOMIC_RELAXED);
    }
    rkept[tid + 1] = kc;
    rdrop[tid] = dc;
    rback[tid] = bc;
  });
  for (int k = 0; k < nth_e; ++k) {
    rkept[k + 1] += rkept[k];
    cs.dropped += rdrop[k];
    cs.backward += rback[k];
  }
  std::vector<int2> kept(static_cast<size_t>(rkept[nth_e]));
  std::vector<unsigned short> kept_iu(kept.size());
  parallel_ranges(ne, nth_e, [&](int tid, int64_t b0, int64_t e0) {
    int64_t w = rkept[tid];
    for (int64_t k = b0; k < e0; ++k) {
      if (who[k] == 2) continue;
      const int a = edges[k].x, b = edges[k].y;
      kept[w] = who[k] == 0 ? make_int2(a, b) : make_int2(b, a);
      kept_iu[w++] = iu[k];
    }
  });
  int max_fwd = 0;
  for (int64_t x = 0; x < n; ++x) {
    if (in_t[x] && formed[x] != own_edges[t_of[x]])
      return fail(c, FSLR_ERR_STATE, "edge cap replay: inconsistent edge count for read " + std::to_string(x));
    max_fwd = std::max(max_fwd, formed[x]);
  }
  cs.applied = 1;
  cs.max_fwd = max_fwd;

  stage("classify edges");
  // write the capped graph back: edges (former, partner), forward degree = edges formed per loop
  const unsigned long long nk = kept.size();
  if (nk) {
    HIP_TRY(c, hipMemcpyAsync(c->edges, kept.data(), nk * sizeof(int2), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->edge_iu, kept_iu.data(), nk * sizeof(unsigned short), hipMemcpyHostToDevice,
                              c->stream));
  }
  HIP_TRY(c, hipMemcpyAsync(c->counters + kEdgeCount, &nk, sizeof(nk), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->fwd, formed.data(), n * sizeof(int), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->errw + 3, &max_fwd, sizeof(int), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  stage("H2D capped graph");
  c->cap_stats = cs;
  if (out) *out = cs;
  return FSLR_OK;
}
