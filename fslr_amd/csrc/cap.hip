// cap.hip — the reference's per-query-read edge cap, replayed exactly on the device (cluster.py:197-224).
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
// does, the loops of the reads that can reach the cap are replayed:
//   1. candidates T: x joins T when fwd(x) + #{y in T, y < x, (y, x) in E*} >= edge_threshold (a
//      read's loop breaks only if its edge count reaches the cap; the edges it can form are its
//      forward E* pairs plus E* pairs (y, x) an earlier breaking read y left unseen).  Kleene
//      iteration from {fwd >= cap}: the rank-ordered definition has exactly one fixed point.
//   2. the visit sequence of every read of T: per interval, its hits in the search's order
//      (descending (start, -end, data position): the order of the superintervals stand-in the
//      golden fixtures were made with — the library's own order is undocumented),
//      the read's own intervals dropped (:203-204).  One wavefront per interval counts, then
//      writes its hits top-down; runs of equal start are re-ranked on (end, position).
//   3. slots: the distinct partners of each read of T (a radix sort of (t, partner) keys), with the
//      sequence position of each partner's first occurrence, and the full pair predicate of each
//      slot (k_cap_eval: length gate, first-fit, cut).
//   4. x's loop depends on an earlier read y of T only through (did y break, did y's loop reach x),
//      and only if y is one of x's partners: the loops are replayed per component of that
//      dependency graph (union-find over the slots), one wavefront per component, reads in rank
//      order.  Inside a loop, up to the break everything is visited, so the break is where the
//      prefix count of first-occurrence edges reaches the cap (a wave-wide scan); after it, each
//      later interval is walked to its first new counted pair.
//   5. an E* pair (a, b) is an edge iff a's loop or, failing that, b's loop reaches it; edges are
//      re-oriented as (the read whose loop formed it, partner) like the reference's match set
//      (:220); forward degrees become the edges formed per loop; each replayed loop's own count
//      must equal them (a consistency check).
// Multi-GPU: each rank holds the full E* list (fslr_cap_install_edges) but indexes
// only its chromosomes, so it writes the visit lists of the T intervals it owns (fslr_cap_local);
// the caller all-gathers them and every rank replays (fslr_cap_replay).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ctx.hpp"
#include "kernels.hpp"
#include "wave.hpp"

namespace fslr {
namespace {

constexpr int kInf = 0x7fffffff;
constexpr unsigned long long kKeyMask = (1ull << 25) - 1;   // read ranks < FSLR_MAX_READS
// per visit-sequence element (rec.y)
enum RecBits { kRFirst = 1, kRNonTBack = 2, kRBackT = 4, kREdge = 8, kRCounted = 16, kRZd = 32 };
// device error word
enum CapErr { kCapErrZd = 1, kCapErrState = 2 };
// device statistics words
enum CapStat { kStCapped = 0, kStDropped, kStBackward, kStMaxFwd, kStKept, kStWords = 8 };
// pinned host words (written by tiny kernels; one sync each)
enum CapHost { kHNt = 0, kHNti, kHNloc, kHNslots, kHNseq, kHErr, kHZd, kHStat = 8, kHWords = 16 };

// one value per block: the wavefronts' values combined in LDS, valid in thread 0 (call from every thread
// of the block; 256 threads).  A per-block atomic instead of one per wavefront: one hot word takes
// ~90 returning atomics per microsecond, so 150k wave atomics over a 10M-read pass cost ~0.2 ms
template <typename T, typename Op>
__device__ __forceinline__ T block_reduce256(T v, Op op) {
  __shared__ T ws[4];
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) v = op(op(ws[0], ws[1]), op(ws[2], ws[3]));
  return v;
}

__device__ __forceinline__ unsigned long long lanes_le(int lane) {
  return lane == 63 ? ~0ull : (2ull << lane) - 1ull;
}

// ---- 1. closure T ------------------------------------------------------------------------------
// state: 0 not in T, 1 joined in the last round (its forward edges not yet counted), 2 counted
__global__ void k_cap_init(const int* __restrict__ fwd, int n, int thr, int* __restrict__ state,
                           int* __restrict__ back) {
  for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < n; x += gridDim.x * blockDim.x) {
    state[x] = fwd[x] >= thr ? 1 : 0;
    back[x] = 0;
  }
}

__global__ void k_cap_back(const int2* __restrict__ edges, long long ne, const int* __restrict__ state,
                           int* __restrict__ back, const int* __restrict__ prev_chg) {
  if (!*prev_chg) return;                                         // converged in an earlier round
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < ne;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int2 e = edges[k];
    if (e.x >= 0 && state[e.x] == 1) atomicAdd(back + e.y, 1);     // a < 0: gathered padding
  }
}

__global__ void k_cap_join(const int* __restrict__ fwd, int n, int thr, int* __restrict__ state,
                           const int* __restrict__ back, const int* __restrict__ prev_chg, int* __restrict__ chg) {
  if (!*prev_chg) return;
  bool any = false;
  for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < n; x += gridDim.x * blockDim.x) {
    const int s = state[x];
    if (s == 1) {
      state[x] = 2;
    } else if (s == 0 && fwd[x] + back[x] >= thr) {
      state[x] = 1;
      any = true;
    }
  }
  if (__ballot(any) && (threadIdx.x & 63) == 0) atomicOr(chg, 1);
}

// The same fixed point by frontiers (the operator is monotone, so adding reads in any order as soon
// as they reach the cap ends at the same least fixed point): E* grouped by its lower read once, then
// each round walks only the forward edges of the reads that joined in the previous round.
__global__ void k_cap_adj_count(const int2* __restrict__ edges, long long ne, int* __restrict__ cnt) {
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < ne;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int a = edges[k].x;
    if (a >= 0) atomicAdd(cnt + a, 1);                              // a < 0: gathered padding
  }
}

__global__ void k_cap_adj_fill(const int2* __restrict__ edges, long long ne, const int* __restrict__ aoff,
                               int* __restrict__ cur, int* __restrict__ adj) {
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < ne;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int2 e = edges[k];
    if (e.x >= 0) adj[aoff[e.x] + atomicAdd(cur + e.x, 1)] = e.y;
  }
}

// the seeds: reads whose own forward degree reaches the cap (frontier 0)
__global__ void k_cap_seed(const int* __restrict__ fwd, int n, int thr, int* __restrict__ state,
                           int* __restrict__ back, int* __restrict__ fl, unsigned* __restrict__ fn,
                           int* __restrict__ tl, unsigned* __restrict__ tn) {
  const int lane = threadIdx.x & 63;
  for (int x0 = (blockIdx.x * blockDim.x + threadIdx.x) & ~63; x0 < n; x0 += gridDim.x * blockDim.x) {
    const int x = x0 + lane;
    const bool j = x < n && fwd[x] >= thr;
    if (x < n) {
      state[x] = j ? 1 : 0;
      back[x] = 0;
    }
    const unsigned long long m = __ballot(j);
    if (!m) continue;
    unsigned base = 0, tbase = 0;
    if (lane == 0) {
      base = atomicAdd(fn, static_cast<unsigned>(__popcll(m)));
      tbase = atomicAdd(tn, static_cast<unsigned>(__popcll(m)));
    }
    base = static_cast<unsigned>(__shfl(static_cast<int>(base), 0));
    tbase = static_cast<unsigned>(__shfl(static_cast<int>(tbase), 0));
    if (j) {
      fl[base + mbcnt(m)] = x;
      tl[tbase + mbcnt(m)] = x;                    // every member of T, in joining order
    }
  }
}


// one round, a wave's 64 frontier reads at a time with their forward rows spread over its lanes (two
// returning atomics in flight per lane; a read walking its own rows pays one memory round trip per
// row).  y joins on the one count that brings fwd(y) + back(y) to the cap: back grows by one per
// walked edge and a seed has fwd(y) >= thr already, so no flag word is needed.  kRows: the runs
// [a0[x], a1[x]) of the rows (gathered, sorted by lower read); else the adjacency a0 / adj
template <bool kRows>
__global__ void __launch_bounds__(256) k_cap_frontier_w(const int* __restrict__ a0, const int* __restrict__ a1,
                                                        const int2* __restrict__ rows, const int* __restrict__ adj,
                                                        const int* __restrict__ fwd, int thr, int* __restrict__ back,
                                                        const int* __restrict__ fin, const unsigned* __restrict__ fin_n,
                                                        int* __restrict__ fout, unsigned* __restrict__ fout_n,
                                                        int* __restrict__ tl, unsigned* __restrict__ tn, int n_reads,
                                                        long long n_rows) {
  const int nin = static_cast<int>(*fin_n);
  FSLR_BOUND(nin, n_reads + 1);                  // (an empty frontier is nin = 0)
  const int lane = threadIdx.x & 63;
  const int wave = static_cast<int>((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int nwaves = static_cast<int>((gridDim.x * blockDim.x) >> 6);
  for (int base = wave * 64; base < nin; base += nwaves * 64) {
    const int i = base + lane;
    int k0 = 0, len = 0;
    if (i < nin) {
      const int x = fin[i];
      FSLR_BOUND(x, n_reads);
      k0 = a0[x];
      len = (kRows ? a1[x] : a0[x + 1]) - k0;
      FSLR_BOUND(k0, n_rows + 1);
      FSLR_BOUND(k0 + len, n_rows + 1);
    }
    const int incl = wave_incl_scan(len);
    const int total = rdl(incl, 63);
    for (int r0 = 0; r0 < total; r0 += 128) {
      int y[2], fy[2], bk[2];
      bool on[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int r = r0 + u * 64 + lane;
        on[u] = r < total;
        int o = 0;                               // the lane holding row r: the first whose count exceeds r
#pragma unroll
        for (int st = 32; st > 0; st >>= 1)
          if (__shfl(incl, o + st - 1) <= r) o += st;
        const int k = __shfl(k0, o) + r - (__shfl(incl, o) - __shfl(len, o));
        if (on[u]) FSLR_BOUND(k, n_rows);
        y[u] = on[u] ? (kRows ? rows[k].y : adj[k]) : 0;
        if (on[u]) FSLR_BOUND(y[u], n_reads);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) fy[u] = on[u] ? fwd[y[u]] : 0;
#pragma unroll
      for (int u = 0; u < 2; ++u) bk[u] = on[u] ? atomicAdd(back + y[u], 1) + 1 : 0;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const bool join = on[u] && fy[u] + bk[u] == thr;
        const unsigned long long jm = __ballot(join);
        if (jm) {
          unsigned p0 = 0, p1 = 0;
          if (lane == 0) {
            p0 = atomicAdd(fout_n, static_cast<unsigned>(__popcll(jm)));
            p1 = atomicAdd(tn, static_cast<unsigned>(__popcll(jm)));
          }
          p0 = static_cast<unsigned>(__shfl(static_cast<int>(p0), 0));
          p1 = static_cast<unsigned>(__shfl(static_cast<int>(p1), 0));
          if (join) {
            fout[p0 + mbcnt(jm)] = y[u];
            tl[p1 + mbcnt(jm)] = y[u];
          }
        }
      }
    }
  }
}

__global__ void k_cap_fcnt_roll(unsigned* fcnt) {
  if (threadIdx.x == 0) {
    const unsigned v = fcnt[16];
    for (int k = 1; k < 32; ++k) fcnt[k] = 0;        // fcnt[32]: the T list's length
    fcnt[0] = v;
  }
}

// T in rank order: one scan of (1 << 32 | L) gives each member its index t and its first T-interval
// read x's interval count: rlen (reads of more than FSLR_MAX_L intervals, real-read space) or rmeta
__device__ __forceinline__ int read_len(const int4* __restrict__ rmeta, const int* __restrict__ rlen, int x) {
  return rlen ? rlen[x] : (rmeta[x].y & 0xffff);
}

__global__ void k_cap_tpack(const int* __restrict__ state, const int4* __restrict__ rmeta,
                            const int* __restrict__ rlen, int n, unsigned long long* __restrict__ v) {
  for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < n; x += gridDim.x * blockDim.x)
    v[x] = state[x] ? ((1ull << 32) | static_cast<unsigned>(read_len(rmeta, rlen, x))) : 0ull;
}

// T from the frontier closure's list (sorted by rank): the read of each t, its interval count
__global__ void k_cap_tfin(const int* __restrict__ T, int nt, const int4* __restrict__ rmeta,
                           const int* __restrict__ rlen, int* __restrict__ t_of, int* __restrict__ tlen) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t <= nt; t += gridDim.x * blockDim.x) {
    if (t == nt) {
      tlen[t] = 0;
      continue;
    }
    const int x = T[t];
    t_of[x] = t;
    tlen[t] = read_len(rmeta, rlen, x);
  }
}

// every read is a candidate (fslr_long_pairs: the pairs of every read's hits)
// every read (fslr_long_pairs), or a query shard's reads (blocks of 64 ranks dealt round robin)
__global__ void k_cap_all(int* __restrict__ state, int n, int shard, int n_shards) {
  for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < n; x += gridDim.x * blockDim.x)
    state[x] = shard_owns(x, shard, n_shards) ? 1 : 0;
}

__global__ void k_cap_tlist(const int* __restrict__ state, const unsigned long long* __restrict__ v,
                            const unsigned long long* __restrict__ vs, int n, int* __restrict__ T,
                            int* __restrict__ toff, int* __restrict__ t_of, long long* __restrict__ host) {
  for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < n; x += gridDim.x * blockDim.x) {
    const unsigned long long s = vs[x];
    if (state[x]) {
      const int t = static_cast<int>(s >> 32);
      T[t] = x;
      toff[t] = static_cast<int>(s & 0xffffffffu);
      t_of[x] = t;
    } else {
      t_of[x] = -1;
    }
    if (x == n - 1) {
      const unsigned long long tot = s + v[x];
      toff[tot >> 32] = static_cast<int>(tot & 0xffffffffu);
      host[kHNt] = static_cast<long long>(tot >> 32);
      host[kHNti] = static_cast<long long>(tot & 0xffffffffu);
    }
  }
}

// T-interval -> its read's index t
__global__ void k_cap_tread(const int* __restrict__ toff, int nt, int* __restrict__ tread) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += gridDim.x * blockDim.x)
    for (int j = toff[t]; j < toff[t + 1]; ++j) tread[j] = t;
}

// The index is over the uploaded reads; with reads of more than FSLR_MAX_L intervals those are
// virtual reads (fslr_set_long_reads): vreal / vbase map a virtual read and its interval j to the
// real read and its interval vbase + j.  Null maps: the identity.
__device__ __forceinline__ int real_of(const int* __restrict__ vreal, int v) { return vreal ? vreal[v] : v; }

// T-interval -> its position in this context's index (-1: a chromosome another rank indexes)
__global__ void k_cap_tq(const int4* __restrict__ idx4, int ni, const int* __restrict__ t_of,
                         const int* __restrict__ toff, const int* __restrict__ vreal, const int* __restrict__ vbase,
                         int* __restrict__ tq) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < ni; q += gridDim.x * blockDim.x) {
    const int tag = idx4[q].w;
    const int v = tag >> 6;
    const int t = t_of[real_of(vreal, v)];
    if (t >= 0) tq[toff[t] + (vbase ? vbase[v] : 0) + (tag & 63)] = q;
  }
}

// ... without reading the index: a binary search for the interval's start in its chromosome's range of
// the start column, then the run of equal starts (data order) for its record
__global__ void k_cap_tq_bs(const int* __restrict__ tread, const int* __restrict__ T, const int* __restrict__ toff,
                            int nti, const int4* __restrict__ rmeta, const int4* __restrict__ iv,
                            const int* __restrict__ fmap, const int2* __restrict__ crange,
                            const int* __restrict__ s_start, const int4* __restrict__ idx4, int* __restrict__ tq,
                            int* __restrict__ err) {
  for (int ti = blockIdx.x * blockDim.x + threadIdx.x; ti < nti; ti += gridDim.x * blockDim.x) {
    const int t = tread[ti];
    const int x = T[t];
    const int j = ti - toff[t];
    const int4 v = iv[rmeta[x].x + j];
    const int ch = fmap ? fmap[v.x] : v.x;         // a chromosome subset: its local number, -1 = not here
    if (ch < 0) {
      tq[ti] = -1;
      continue;
    }
    const int2 cr = crange[ch];
    int lo = cr.x, hi = cr.y;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s_start[mid] < v.y) lo = mid + 1; else hi = mid;
    }
    const int tag = (x << 6) | j;
    int q = -1;
    for (int p = lo; p < cr.y && s_start[p] == v.y; ++p)
      if (idx4[p].w == tag) {
        q = p;
        break;
      }
    tq[ti] = q;
    if (q < 0) atomicOr(err, kCapErrState);
  }
}

// ---- 2. visit sequences ------------------------------------------------------------------------
// One wavefront per T-interval (sorted position q): the hits are q + 1 .. q + n_fwd and those p in
// [bwd_begin, q) with end_p >= start_q (kernels.hpp rng_s), minus the read's own intervals.
// kEmit = false: icnt[ti] = their count; kEmit = true: their positions, highest first, at ioff[ti].
template <bool kEmit>
__global__ __launch_bounds__(256) void k_cap_hits(const int* __restrict__ tq, const int* __restrict__ tread,
                                                  const int* __restrict__ T, const int4* __restrict__ idx4,
                                                  const int2* __restrict__ rng_s, const int* __restrict__ vreal,
                                                  int nti, int* __restrict__ icnt, const int* __restrict__ ioff,
                                                  int* __restrict__ seqp) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int ti = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); ti < nti; ti += nw) {
    const int q = tq[ti];
    if (q < 0) {
      if (!kEmit && lane == 0) icnt[ti] = 0;
      continue;
    }
    const int x = T[tread[ti]];
    const int s = idx4[q].x;
    const int2 rg = rng_s[q];
    const int lo = rg.y, hi = q + rg.x;
    int w = 0;
    if (kEmit) {
      const int base = ioff[ti];
      for (int p0 = hi; p0 >= lo; p0 -= 64) {
        const int p = p0 - lane;
        bool hit = false;
        if (p >= lo) {
          const int4 r = idx4[p];
          hit = (p >= q || r.y >= s) && real_of(vreal, r.w >> 6) != x;
        }
        const unsigned long long hm = __ballot(hit);
        if (hit) seqp[base + w + mbcnt(hm)] = p;
        w += __popcll(hm);
      }
    } else {
      for (int p0 = lo; p0 <= hi; p0 += 64) {
        const int p = p0 + lane;
        bool hit = false;
        if (p <= hi) {
          const int4 r = idx4[p];
          hit = (p >= q || r.y >= s) && real_of(vreal, r.w >> 6) != x;
        }
        w += __popcll(__ballot(hit));
      }
      if (lane == 0) icnt[ti] = w;
    }
  }
}

// Positions -> partner reads in the search's order.  Inside a segment starts descend; a run of
// equal start holds exactly the hits of that run (its elements with end >= start_q, a prefix of the
// stand-in's (end desc, position asc) order), so each run's hits are re-ranked by (end asc,
// position desc).  One wavefront per T-interval.
__global__ __launch_bounds__(256) void k_cap_seq(const int* __restrict__ seqp, const int4* __restrict__ idx4,
                                                 const int* __restrict__ ioff, const int* __restrict__ vreal, int nti,
                                                 int* __restrict__ seq) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int ti = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); ti < nti; ti += nw) {
    const int b0 = ioff[ti], b1 = ioff[ti + 1];
    for (int k0 = b0; k0 < b1; k0 += 64) {
      const int k = k0 + lane;
      if (k >= b1) continue;
      const int p = seqp[k];
      const int4 r = idx4[p];
      const bool tied = (k > b0 && idx4[seqp[k - 1]].x == r.x) || (k + 1 < b1 && idx4[seqp[k + 1]].x == r.x);
      int dst = k;
      if (tied) {
        int bb = k;
        while (bb > b0 && idx4[seqp[bb - 1]].x == r.x) --bb;
        int rank = 0;
        for (int f = bb; f < b1; ++f) {
          const int pf = seqp[f];
          const int4 rf = idx4[pf];
          if (rf.x != r.x) break;
          rank += rf.y < r.y || (rf.y == r.y && pf > p);
        }
        dst = bb + rank;
      }
      seq[dst] = real_of(vreal, r.w >> 6);
    }
  }
}

// Multi-GPU: the ranks' gathered lists (rank w's list holds its T-intervals' segments in T-interval
// order) into one sequence.  loff = exclusive scan of the gathered counts (rank-major).
__global__ __launch_bounds__(256) void k_cap_assemble(const int* __restrict__ cnt_all, const int* __restrict__ loff,
                                                      const int* __restrict__ lists, long long pad, int world,
                                                      int nti, const int* __restrict__ ioff, int* __restrict__ seq) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int ti = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); ti < nti; ti += nw) {
    int dst = ioff[ti];
    for (int w = 0; w < world; ++w) {
      const long long i = static_cast<long long>(w) * nti + ti;
      const int cnt = cnt_all[i];
      if (!cnt) continue;
      const int* src = lists + w * pad + (loff[i] - loff[static_cast<long long>(w) * nti]);
      for (int k = lane; k < cnt; k += 64) seq[dst + k] = src[k];
      dst += cnt;
    }
  }
}

__global__ void k_cap_sum_counts(const int* __restrict__ cnt_all, int world, int nti, int* __restrict__ tot) {
  for (int ti = blockIdx.x * blockDim.x + threadIdx.x; ti <= nti; ti += gridDim.x * blockDim.x) {
    int s = 0;
    if (ti < nti)
      for (int w = 0; w < world; ++w) s += cnt_all[static_cast<long long>(w) * nti + ti];
    tot[ti] = s;
  }
}

// ---- 3. slots ----------------------------------------------------------------------------------
// sort keys (t << 25 | partner), values = sequence position; one wavefront per T-interval
__global__ __launch_bounds__(256) void k_cap_keys(const int* __restrict__ seq, const int* __restrict__ ioff,
                                                  const int* __restrict__ tread, int nti,
                                                  unsigned long long* __restrict__ key, int* __restrict__ val) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int ti = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); ti < nti; ti += nw) {
    const unsigned long long hi = static_cast<unsigned long long>(tread[ti]) << 25;
    for (int k = ioff[ti] + lane; k < ioff[ti + 1]; k += 64) {
      key[k] = hi | static_cast<unsigned>(seq[k]);
      val[k] = k;
    }
  }
}

// the segmented form: partners (32-bit) sorted inside each read's segment of the sequence (a few
// hundred hits) instead of (read, partner) keys over the whole sequence; then the keys rebuilt
__global__ __launch_bounds__(256) void k_cap_pkeys(const int* __restrict__ seq, int m, unsigned* __restrict__ key,
                                                   int* __restrict__ val) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < m; k += gridDim.x * blockDim.x) {
    key[k] = static_cast<unsigned>(seq[k]);
    val[k] = k;
  }
}

__global__ void k_cap_segb(const int* __restrict__ ioff, const int* __restrict__ toff, int nt, int* __restrict__ segb,
                           unsigned* __restrict__ segmax) {
  unsigned mx = 0;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t <= nt; t += gridDim.x * blockDim.x) {
    segb[t] = ioff[toff[t]];
    if (t < nt) mx = max(mx, static_cast<unsigned>(ioff[toff[t + 1]] - ioff[toff[t]]));
  }
  mx = block_reduce256(mx, [](unsigned x, unsigned y) { return max(x, y); });
  if (threadIdx.x == 0 && mx) atomicMax(segmax, mx);
}

// ... in LDS: one workgroup per read of T whose segment has (lo, CAP] hits, a bitonic sort of
// (partner << 32 | position) keys (positions ascending among equal partners, as the stable sorts)
template <int CAP>
__global__ __launch_bounds__(256) void k_cap_segsort(const int* __restrict__ seq, const int* __restrict__ segb, int nt,
                                                     int lo, unsigned* __restrict__ pkey2, int* __restrict__ sval2) {
  __shared__ unsigned long long buf[CAP];
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
    const int b = segb[t], n = segb[t + 1] - b;
    if (n <= lo || n > CAP) continue;                // another size class (workgroup-uniform)
    int P = 1;
    while (P < n) P <<= 1;
    for (int i = threadIdx.x; i < P; i += blockDim.x)
      buf[i] = i < n ? (static_cast<unsigned long long>(static_cast<unsigned>(seq[b + i])) << 32) |
                           static_cast<unsigned>(b + i)
                     : ~0ull;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = threadIdx.x; i < P; i += blockDim.x) {
          const int l = i ^ j;
          if (l > i) {
            const unsigned long long x = buf[i], y = buf[l];
            if ((x > y) == ((i & k) == 0)) {
              buf[i] = y;
              buf[l] = x;
            }
          }
        }
        __syncthreads();
      }
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const unsigned long long v = buf[i];
      pkey2[b + i] = static_cast<unsigned>(v >> 32);
      sval2[b + i] = static_cast<int>(static_cast<unsigned>(v));
    }
    __syncthreads();
  }
}
constexpr int kSegSmall = 1024, kSegBig = 8192;

__global__ __launch_bounds__(256) void k_cap_rekey(const unsigned* __restrict__ pkey, const int* __restrict__ segb,
                                                   int nt, unsigned long long* __restrict__ key) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int t = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < nt; t += nw) {
    const unsigned long long hi = static_cast<unsigned long long>(t) << 25;
    for (int k = segb[t] + lane; k < segb[t + 1]; k += 64) key[k] = hi | pkey[k];
  }
}

// each read of T's first slot (its sequence segment's first head; an empty segment: the next one's)
__global__ void k_cap_tsb(const int* __restrict__ hs, const int* __restrict__ head, const int* __restrict__ segb,
                          int nt, int m, int* __restrict__ tsb) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t <= nt; t += gridDim.x * blockDim.x) {
    const int k = segb[t];
    tsb[t] = k < m ? hs[k] : hs[m - 1] + head[m - 1];
  }
}

__global__ void k_cap_heads(const unsigned long long* __restrict__ key, int m, int* __restrict__ head) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < m; k += gridDim.x * blockDim.x)
    head[k] = k == 0 || key[k] != key[k - 1];
}

// stable sort: a run's first value is the partner's first occurrence in the read's sequence
__global__ void k_cap_slots(const unsigned long long* __restrict__ key, const int* __restrict__ val,
                            const int* __restrict__ head, const int* __restrict__ hs, int m,
                            int* __restrict__ slot_of, unsigned long long* __restrict__ ukey, int* __restrict__ fpos,
                            long long* __restrict__ host) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < m; k += gridDim.x * blockDim.x) {
    const int s = hs[k] + head[k] - 1;
    slot_of[val[k]] = s;
    if (head[k]) {
      ukey[s] = key[k];
      fpos[s] = val[k];
    }
    if (k == m - 1) host[kHNslots] = s + 1;
  }
}


__device__ __forceinline__ int row_at(const int4* __restrict__ rmeta, const int* __restrict__ off2, int r, int i) {
  return i < FSLR_MAX_L ? rmeta[r].x + i : off2[r] + (i - FSLR_MAX_L);
}

// one slot's first-fit on a wavefront (any lengths): B's intervals in lanes, 64 columns at a time
__device__ __forceinline__ void eval_wave(const int4* __restrict__ rmeta, const int4* __restrict__ iv,
                                          const int* __restrict__ off2, int a, int b, int LA, int LB, int lane,
                                          int* I_out, bool* zd_out) {
  const int4 bm = rmeta[b];
  const int nb = (LB + 63) >> 6;
  unsigned long long used = 0ull;
  int4 b0 = make_int4(-2, 0, 0, 0);                          // the first 64 columns stay in registers
  if (lane < LB) b0 = iv[bm.x + lane];
  int4 ai = make_int4(-1, 0, 0, 0);
  int I = 0;
  bool zd = false;
  for (int i = 0; i < LA && !zd; ++i) {
    if ((i & 63) == 0) ai = i + lane < LA ? iv[row_at(rmeta, off2, a, i + lane)] : make_int4(-1, 0, 0, 0);
    const int c = rdl(ai.x, i & 63), si = rdl(ai.y, i & 63), ei = rdl(ai.z, i & 63), ti = rdl(ai.w, i & 63);
    for (int cc = 0; cc < nb; ++cc) {
      const int jj = (cc << 6) + lane;
      int4 bj = b0;
      if (cc > 0) bj = jj < LB ? iv[row_at(rmeta, off2, b, jj)] : make_int4(-2, 0, 0, 0);
      const bool cand = jj < LB && !((used >> cc) & 1ull) && bj.x == c;
      const bool zero = cand && (ti == FSLR_THR_ZERO_ALN || bj.w == FSLR_THR_ZERO_ALN);
      const bool hit = cand && (zero || iv_match_general(si, ei, ti, bj.y, bj.z, bj.w));
      const unsigned long long hm = __ballot(hit);
      if (!hm) continue;
      const int j = __builtin_ctzll(hm);
      if (__shfl(static_cast<int>(zero), j)) {
        zd = true;
        break;
      }
      if (lane == j) used |= 1ull << cc;
      ++I;
      break;
    }
  }
  *I_out = I;
  *zd_out = zd;
}

// the same first-fit by one lane, for two reads of at most kLaneL intervals: rows ascending, the
// lowest unused column of the row's chromosome that matches (or raises)
constexpr int kLaneL = 16;
__device__ __forceinline__ void eval_lane(const int4* __restrict__ iv, int oa, int ob, int LA, int LB, int* I_out,
                                          bool* zd_out) {
  unsigned used = 0u;
  int I = 0;
  bool zd = false;
  for (int i = 0; i < LA && !zd; ++i) {
    const int4 ai = iv[oa + i];
    for (int j = 0; j < LB; ++j) {
      if ((used >> j) & 1u) continue;
      const int4 bj = iv[ob + j];
      if (bj.x != ai.x) continue;
      if (ai.w == FSLR_THR_ZERO_ALN || bj.w == FSLR_THR_ZERO_ALN) {
        zd = true;
        break;
      }
      if (iv_match_general(ai.y, ai.z, ai.w, bj.y, bj.z, bj.w)) {
        used |= 1u << j;
        ++I;
        break;
      }
    }
  }
  *I_out = I;
  *zd_out = zd;
}

// the full predicate of each slot's pair: the length gate, first-fit in the reference's order
// (rows ascending, the lowest unused column, cluster.py:152-161), the cut; ZeroDivisionError where
// the reference meets an aln_size == 0 interval (:133-136) or both reads' qlen2 / n_alignments are 0
// (:178-183).  A wavefront takes 64 consecutive slots, one per lane: pairs of two reads of at most
// kLaneL intervals are decided by their lane; the others one after the other by the whole wavefront
// (B's intervals in lanes, A's rows broadcast; any read length up to 4096 (long.hip checks it at
// upload): lane l keeps bit c
// of `used` for column 64 c + l; a real read's intervals are its first virtual read's and, beyond
// FSLR_MAX_L, the consecutive chunks starting at off2).
// flags: {zd | lenok << 1 | edge << 2, I | U << 16}
__global__ __launch_bounds__(256) void k_cap_eval(const unsigned long long* __restrict__ ukey, int ns,
                                                  const int* __restrict__ T, const int4* __restrict__ rmeta,
                                                  const int4* __restrict__ iv, const int* __restrict__ rlen,
                                                  const int* __restrict__ off2, double qcut, double ncut,
                                                  const int* __restrict__ umax, int n_umax, int2* __restrict__ flags) {
  const int lane = threadIdx.x & 63;
  const long long nw = static_cast<long long>(gridDim.x) * (blockDim.x >> 6);
  for (long long base = (static_cast<long long>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64; base < ns;
       base += nw * 64) {
    const long long sl = base + lane;
    const bool valid = sl < ns;
    int a = 0, b = 0, LA = 0, LB = 0;
    bool zd = false, lenok = false;
    if (valid) {
      const unsigned long long key = ukey[sl];
      const int x = T[key >> 25], y = static_cast<int>(key & kKeyMask);
      a = min(x, y);
      b = max(x, y);
      const int4 am = rmeta[a], bm = rmeta[b];
      LA = read_len(rmeta, rlen, a);
      LB = read_len(rmeta, rlen, b);
      lenok = lengths_pass(am.z, bm.z, am.w, bm.w, qcut, ncut, &zd);
    }
    const bool need = valid && lenok && !zd;
    const bool small = need && LA <= kLaneL && LB <= kLaneL;
    int I = 0;
    bool fzd = false;
    if (small) eval_lane(iv, rmeta[a].x, rmeta[b].x, LA, LB, &I, &fzd);
    // the larger pairs of these 64 slots: the whole wavefront, one pair after the other
    for (unsigned long long big = __ballot(need && !small); big; big &= big - 1) {
      const int c = __builtin_ctzll(big);
      int Ic = 0;
      bool zc = false;
      eval_wave(rmeta, iv, off2, rdl(a, c), rdl(b, c), rdl(LA, c), rdl(LB, c), lane, &Ic, &zc);
      if (lane == c) {
        I = Ic;
        fzd = zc;
      }
    }
    zd = zd || fzd;
    const int U = LA + LB - I;
    const bool edge = lenok && !zd && I > 0 && I <= n_umax && U <= umax[min(max(I, 1), n_umax) - 1];
    if (valid)
      flags[sl] = make_int2(static_cast<int>(zd) | (static_cast<int>(lenok && !zd) << 1) | (static_cast<int>(edge) << 2),
                            I | (U << 16));
  }
}

// slot of key k = t << 25 | partner among read t's slots [tsb[t], tsb[t + 1]) (ukey sorted; -1: none)
__device__ __forceinline__ int find_slot(const unsigned long long* __restrict__ ukey, const int* __restrict__ tsb,
                                         int t, unsigned long long k) {
  const int ns = tsb[t + 1];
  int lo = tsb[t], hi = ns;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (ukey[mid] < k) lo = mid + 1; else hi = mid;
  }
  return lo < ns && ukey[lo] == k ? lo : -1;
}

// per slot (x, y): for an earlier partner y of T, the slot of (y, x) (where y's loop records
// whether it reached x) and the union of x and y in the dependency graph
__global__ void k_cap_mirror(const unsigned long long* __restrict__ ukey, int ns, const int* __restrict__ tsb,
                             const int* __restrict__ T,
                             const int* __restrict__ t_of, int* __restrict__ mslot, int2* __restrict__ upairs,
                             int* __restrict__ err) {
  for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < ns; s += gridDim.x * blockDim.x) {
    const unsigned long long key = ukey[s];
    const int t = static_cast<int>(key >> 25), y = static_cast<int>(key & kKeyMask);
    const int x = T[t];
    const int ty = y < x ? t_of[y] : -1;
    int ms = -1;
    int2 up = make_int2(-1, -1);
    if (ty >= 0) {
      ms = find_slot(ukey, tsb, ty, (static_cast<unsigned long long>(ty) << 25) | static_cast<unsigned>(x));
      if (ms < 0) atomicOr(err, kCapErrState);          // hits are symmetric: cannot happen
      up = make_int2(t, ty);
    }
    mslot[s] = ms;
    upairs[s] = up;
  }
}

__global__ void k_cap_ckeys(const int* __restrict__ tpar, int nt, unsigned long long* __restrict__ ck) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += gridDim.x * blockDim.x)
    ck[t] = (static_cast<unsigned long long>(tpar[t]) << 25) | static_cast<unsigned>(t);
}

// the replay's static view of each sequence element: {slot, bits, mirror slot, T index of partner}
__global__ void k_cap_recs(const int* __restrict__ slot_of, const unsigned long long* __restrict__ ukey,
                           const int* __restrict__ fpos, const int2* __restrict__ flags, const int* __restrict__ mslot,
                           const int* __restrict__ T, const int* __restrict__ t_of, int m, int4* __restrict__ rec) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < m; k += gridDim.x * blockDim.x) {
    const int s = slot_of[k];
    const unsigned long long key = ukey[s];
    const int x = T[key >> 25], y = static_cast<int>(key & kKeyMask);
    const int2 fl = flags[s];
    const int f = fl.x;
    int bits = fpos[s] == k ? kRFirst : 0;
    int ty = -1;
    if (y < x) {
      ty = t_of[y];
      bits |= ty >= 0 ? kRBackT : kRNonTBack;     // a non-T earlier read never breaks: pair seen
    }
    if (f & 1) bits |= kRZd;
    if (f & 4) bits |= kREdge;
    if ((f & 2) && (fl.y & 0xffff) > 0) bits |= kRCounted;
    rec[k] = make_int4(s, bits, ty >= 0 ? mslot[s] : -1, ty);
  }
}

// ---- 4. the loops ------------------------------------------------------------------------------
// did the (finished) loop of T read ty reach its slot ms?  Everything up to its break position, plus
// what its post-break interval walks visited
__device__ __forceinline__ bool reached(const int* __restrict__ fpos, const unsigned char* vis2,
                                        const int* pbrk, int ms, int ty) {
  return fpos[ms] <= pbrk[ty] || vis2[ms];
}

__device__ bool replay_read(int t, int lane, int thr, const int* __restrict__ toff, const int* __restrict__ ioff,
                            const int4* __restrict__ rec, const int* __restrict__ fpos, unsigned char* vis2,
                            int* pbrk, int* own, int* err) {
  const int ti0 = toff[t], ti1 = toff[t + 1];
  const int sb = ioff[ti0], se = ioff[ti1];
  int edges = 0, P = kInf;
  // before the break every hit is visited: the first occurrence of each partner is its visit
  for (int k0 = sb; k0 < se; k0 += 64) {
    const int k = k0 + lane;
    bool e = false, cnt = false, zd = false;
    if (k < se) {
      const int4 r = rec[k];
      bool proc = (r.y & kRFirst) && !(r.y & kRNonTBack);
      if (proc && (r.y & kRBackT)) proc = !reached(fpos, vis2, pbrk, r.z, r.w);
      e = proc && (r.y & kREdge);
      cnt = proc && (r.y & kRCounted);
      zd = proc && (r.y & kRZd);
    }
    const unsigned long long em = __ballot(e);
    const int incl = edges + __popcll(em & lanes_le(lane));
    const unsigned long long bm = __ballot(cnt && incl >= thr);   // the check after a counted pair (:223)
    const unsigned long long zm = __ballot(zd);
    const int fb = bm ? __builtin_ctzll(bm) : 64;
    if (zm && __builtin_ctzll(zm) < fb) {
      if (lane == 0) atomicOr(err, kCapErrZd);
      return false;
    }
    if (bm) {
      P = k0 + fb;
      edges += __popcll(em & lanes_le(fb));
      break;
    }
    edges += __popcll(em);
  }
  if (P != kInf) {
    // the rest of the break's interval is left; each later interval is walked up to its first new
    // pair that passes the gate with I > 0 (:216-217 skip the check, :223 then breaks again)
    int ti = ti0;
    while (ioff[ti + 1] <= P) ++ti;
    for (++ti; ti < ti1; ++ti) {
      const int b0 = ioff[ti], b1 = ioff[ti + 1];
      for (int k0 = b0; k0 < b1; k0 += 64) {
        const int k = k0 + lane;
        bool proc = false, e = false, cnt = false, zd = false;
        int s = 0;
        if (k < b1) {
          const int4 r = rec[k];
          s = r.x;
          proc = !(r.y & kRNonTBack);
          if (proc && (r.y & kRBackT)) proc = !reached(fpos, vis2, pbrk, r.z, r.w);
          if (proc) proc = fpos[s] > P && !vis2[s];
          e = proc && (r.y & kREdge);
          cnt = proc && (r.y & kRCounted);
          zd = proc && (r.y & kRZd);
        }
        const unsigned long long cm = __ballot(cnt);
        const unsigned long long zm = __ballot(zd);
        const int stop = cm ? __builtin_ctzll(cm) : 64;
        if (zm && __builtin_ctzll(zm) < stop) {
          if (lane == 0) atomicOr(err, kCapErrZd);
          return false;
        }
        if (proc && lane <= stop) vis2[s] = 1;
        if (cm) {
          edges += static_cast<int>((__ballot(e) >> stop) & 1ull);
          break;
        }
      }
      // this walk's marks before the next interval's loads: the same wave reads them back, so the
      // stores only need to have landed (workgroup scope; an agent-scope fence per interval costs
      // microseconds, MI355X_MICROARCH.md)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
  }
  if (lane == 0) {
    pbrk[t] = P;
    own[t] = edges;
  }
  return true;
}

// one wavefront per component of the dependency graph (its head = its smallest t), reads in rank order
__global__ __launch_bounds__(256) void k_cap_replay(const unsigned long long* __restrict__ ck, int nt, int thr,
                                                    const int* __restrict__ toff, const int* __restrict__ ioff,
                                                    const int4* __restrict__ rec, const int* __restrict__ fpos,
                                                    unsigned char* vis2, int* pbrk, int* own, int* err) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int h = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); h < nt; h += nw) {
    const unsigned long long hk = ck[h];
    const int root = static_cast<int>(hk >> 25);
    if (static_cast<int>(hk & kKeyMask) != root) continue;
    for (int k = h; k < nt; ++k) {
      const unsigned long long kk = ck[k];
      if (static_cast<int>(kk >> 25) != root) break;
      if (!replay_read(static_cast<int>(kk & kKeyMask), lane, thr, toff, ioff, rec, fpos, vis2, pbrk, own, err))
        return;
      // this loop's results before a later read's loads (the same wave: workgroup scope)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
  }
}

// ---- 4'. the loops in dependency order (k_cap_replay_dag) ------------------------------------------
// x's loop needs only the finished loops of its earlier partners in T (replay_read reads their
// pbrk and the visit marks of their slots for x).  Those form a DAG in rank order, so a loop can
// run as soon as its last earlier T partner has finished: a ready queue instead of one wavefront
// per component, which keeps a large component's chain of loops from running one after the other.
// Slots of one t are contiguous in ukey (sorted by t, then partner): sbeg / send.
__global__ void k_cap_dag_bounds(const unsigned long long* __restrict__ ukey, int ns, int* __restrict__ sbeg,
                                 int* __restrict__ send) {
  for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < ns; s += gridDim.x * blockDim.x) {
    const int t = static_cast<int>(ukey[s] >> 25);
    if (s == 0 || static_cast<int>(ukey[s - 1] >> 25) != t) sbeg[t] = s;
    if (s == ns - 1 || static_cast<int>(ukey[s + 1] >> 25) != t) send[t] = s + 1;
  }
}

// earlier T partners per read (k_cap_mirror's upairs: (t, ty) for a partner ty of T before x)
__global__ void k_cap_dag_indeg(const int2* __restrict__ upairs, int ns, int* __restrict__ indeg) {
  for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < ns; s += gridDim.x * blockDim.x) {
    const int2 u = upairs[s];
    if (u.x >= 0) atomicAdd(indeg + u.x, 1);
  }
}

// the reads with no earlier T partner start the queue (rank order inside each wave)
__global__ void k_cap_dag_seed(const int* __restrict__ indeg, int nt, int* __restrict__ ready,
                               unsigned* __restrict__ qtail) {
  const int lane = threadIdx.x & 63;
  for (int t0 = (blockIdx.x * blockDim.x + threadIdx.x) & ~63; t0 < nt; t0 += gridDim.x * blockDim.x) {
    const int t = t0 + lane;
    const bool r = t < nt && indeg[t] == 0;
    const unsigned long long m = __ballot(r);
    if (!m) continue;
    unsigned base = 0;
    if (lane == 0) base = atomicAdd(qtail, static_cast<unsigned>(__popcll(m)));
    base = static_cast<unsigned>(__shfl(static_cast<int>(base), 0));
    if (r) ready[base + mbcnt(m)] = t;
  }
}

constexpr long long kDagSpinTicks = 50000000;   // s_memrealtime at 100 MHz: 0.5 s without a ready loop

// One wavefront per loop at a time: take the next queue position, wait for its read, replay it,
// then release the later T partners whose last earlier partner it was.  Every position below nt
// is filled exactly once (each read's in-degree reaches 0 once; the smallest unfinished rank always
// has every earlier partner done), and a wave leaves when the positions run out; a wave that sees
// no read arrive for kDagSpinTicks flags err[1] and leaves (the host then runs k_cap_replay).
__global__ __launch_bounds__(256) void k_cap_replay_dag(int nt, int thr, const int* __restrict__ T,
                                                        const int* __restrict__ t_of, const int* __restrict__ toff,
                                                        const int* __restrict__ ioff, const int4* __restrict__ rec,
                                                        const int* __restrict__ fpos,
                                                        const unsigned long long* __restrict__ ukey,
                                                        const int* __restrict__ sbeg, const int* __restrict__ send,
                                                        int* indeg, int* ready, unsigned* queue, unsigned char* vis2,
                                                        int* pbrk, int* own, int* err) {
  const int lane = threadIdx.x & 63;
  while (true) {
    unsigned k = 0;
    if (lane == 0) k = atomicAdd(queue, 1u);                     // queue[0]: next position to take
    k = static_cast<unsigned>(__shfl(static_cast<int>(k), 0));
    if (k >= static_cast<unsigned>(nt)) return;
    int t = __hip_atomic_load(ready + k, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    if (t < 0) {
      const long long t0 = wall_clock64();
      while (t < 0) {
        __builtin_amdgcn_s_sleep(4);
        t = __hip_atomic_load(ready + k, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (t < 0 && wall_clock64() - t0 > kDagSpinTicks) {
          if (lane == 0) atomicOr(err + 1, 1);
          return;
        }
      }
    }
    replay_read(t, lane, thr, toff, ioff, rec, fpos, vis2, pbrk, own, err);   // a ZeroDivisionError is in err
    __threadfence();                       // this loop's pbrk / own / visit marks before the releases
    const int x = T[t];
    for (int s0 = sbeg[t]; s0 < send[t]; s0 += 64) {
      const int s = s0 + lane;
      int t2 = -1;
      if (s < send[t]) {
        const int y = static_cast<int>(ukey[s] & kKeyMask);
        if (y > x) t2 = t_of[y];
      }
      // the release fence above orders this loop's results before the decrement; the lane that
      // takes the count to 0 acquires (every earlier partner's results) before it publishes t2
      if (t2 >= 0 && __hip_atomic_fetch_add(indeg + t2, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const unsigned slot = atomicAdd(queue + 1, 1u);                // queue[1]: next position to fill
        __hip_atomic_store(ready + slot, t2, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// ---- 5. the capped graph -----------------------------------------------------------------------
__device__ __forceinline__ bool loop_reaches(int x, int y, const int* __restrict__ t_of,
                                             const int* __restrict__ pbrk, const unsigned long long* __restrict__ ukey,
                                             const int* __restrict__ tsb, const int* __restrict__ fpos, const unsigned char* __restrict__ vis2,
                                             int* err) {
  const int t = t_of[x];
  if (t < 0 || pbrk[t] == kInf) return true;       // the loop never broke: it visited every hit
  const int s = find_slot(ukey, tsb, t, (static_cast<unsigned long long>(t) << 25) | static_cast<unsigned>(y));
  if (s < 0) {
    atomicOr(err, kCapErrState);
    return false;
  }
  return fpos[s] <= pbrk[t] || vis2[s];
}

// who: 0 formed in a's loop, 1 in b's, 2 in neither (dropped)
__global__ void k_cap_classify(const int2* __restrict__ edges, long long ne, const int* __restrict__ t_of,
                               const int* __restrict__ pbrk, const unsigned long long* __restrict__ ukey, const int* __restrict__ tsb,
                               const int* __restrict__ fpos, const unsigned char* __restrict__ vis2,
                               int* __restrict__ kflag, unsigned char* __restrict__ who, int* __restrict__ formed,
                               long long* __restrict__ stats, int* __restrict__ err) {
  long long drop = 0, bwd = 0;
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < ne;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int2 e = edges[k];
    int w = 2;
    if (loop_reaches(e.x, e.y, t_of, pbrk, ukey, tsb, fpos, vis2, err)) w = 0;
    else if (loop_reaches(e.y, e.x, t_of, pbrk, ukey, tsb, fpos, vis2, err)) w = 1;
    who[k] = static_cast<unsigned char>(w);
    kflag[k] = w != 2;
    // formed starts as the E* forward degrees (every edge in its lower read's loop): only an edge
    // formed in the higher read's loop, or dropped, moves a count (no atomic for the many others)
    if (w != 0) atomicSub(formed + e.x, 1);
    if (w == 1) atomicAdd(formed + e.y, 1);
    drop += w == 2;
    bwd += w == 1;
  }
  for (int o = 32; o > 0; o >>= 1) {
    drop += __shfl_xor(drop, o);
    bwd += __shfl_xor(bwd, o);
  }
  if ((threadIdx.x & 63) == 0) {
    if (drop) atomicAdd(reinterpret_cast<unsigned long long*>(stats + kStDropped), static_cast<unsigned long long>(drop));
    if (bwd) atomicAdd(reinterpret_cast<unsigned long long*>(stats + kStBackward), static_cast<unsigned long long>(bwd));
  }
}

// ---- 5'. one GPU, the edge list grouped by lower read (the sweep engine writes each read's forward
// edges as one run: its edge stage never splits a read).  The closure walks the runs (frontier), and
// only the rows of T's runs can change: they are classified in place, the dropped ones marked and
// the list closed up by moving the few surviving rows behind the new end into the holes before it.
// A read with two runs (another engine's order) flags the list: the full-list path runs instead.
// (gstart, gend zeroed: a read without edges has the empty run [0, 0); a run's end is never 0, so a
// second run of a read finds its end taken)
__global__ void k_cap_runs1(const int2* __restrict__ e, long long ne, int* __restrict__ gstart, int* __restrict__ gend,
                            int* __restrict__ flag) {
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < ne;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int a = e[k].x;
    const int prev = k ? e[k - 1].x : -1;
    const int next = k + 1 < ne ? e[k + 1].x : -1;
    if (prev != a) gstart[a] = static_cast<int>(k);
    if (next != a && atomicCAS(gend + a, 0, static_cast<int>(k + 1)) != 0) atomicOr(flag, 1);
  }
}

// one wavefront per read of T: its run's rows; re-oriented rows flipped in place, dropped rows marked
// (a = -1) and listed
__global__ __launch_bounds__(256) void k_cap_classify_runs(int2* __restrict__ edges, const int* __restrict__ gstart,
                                                           const int* __restrict__ gend, const int* __restrict__ T,
                                                           int nt, const int* __restrict__ t_of,
                                                           const int* __restrict__ pbrk,
                                                           const unsigned long long* __restrict__ ukey, const int* __restrict__ tsb,
                                                           const int* __restrict__ fpos,
                                                           const unsigned char* __restrict__ vis2,
                                                           int* __restrict__ formed, int* __restrict__ drops,
                                                           unsigned* __restrict__ ndrop, long long* __restrict__ stats,
                                                           int* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  long long drop = 0, bwd = 0;
  for (int t = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < nt; t += (gridDim.x * blockDim.x) >> 6) {
    const int a = T[t];
    if (pbrk[t] == kInf) continue;                   // the loop never broke: it formed all its edges
    const int k0 = gstart[a], k1 = gend[a];
    for (int kb = k0; kb < k1; kb += 64) {
      const int k = kb + lane;
      int w = 0;
      int2 e = make_int2(0, 0);
      if (k < k1) {
        e = edges[k];
        if (!loop_reaches(e.x, e.y, t_of, pbrk, ukey, tsb, fpos, vis2, err))
          w = loop_reaches(e.y, e.x, t_of, pbrk, ukey, tsb, fpos, vis2, err) ? 1 : 2;
      }
      if (w == 1) {
        edges[k] = make_int2(e.y, e.x);
        atomicAdd(formed + e.y, 1);
      }
      if (w) atomicSub(formed + e.x, 1);
      const unsigned long long dm = __ballot(w == 2);
      if (dm) {
        unsigned base = 0;
        if (lane == 0) base = atomicAdd(ndrop, static_cast<unsigned>(__popcll(dm)));
        base = static_cast<unsigned>(__shfl(static_cast<int>(base), 0));
        if (w == 2) {
          edges[k].x = -1;
          drops[base + mbcnt(dm)] = k;
        }
      }
      drop += w == 2;
      bwd += w == 1;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    drop += __shfl_xor(drop, o);
    bwd += __shfl_xor(bwd, o);
  }
  if (lane == 0) {
    if (drop) atomicAdd(reinterpret_cast<unsigned long long*>(stats + kStDropped), static_cast<unsigned long long>(drop));
    if (bwd) atomicAdd(reinterpret_cast<unsigned long long*>(stats + kStBackward), static_cast<unsigned long long>(bwd));
  }
}

// the holes: dropped rows before the new end ne - d; the survivors: unmarked rows from there on
__global__ void k_cap_holes(const int* __restrict__ drops, const unsigned* __restrict__ ndrop, long long ne,
                            int* __restrict__ holes, unsigned* __restrict__ nh) {
  const long long d = *ndrop;
  const long long keep = ne - d;
  const int lane = threadIdx.x & 63;
  for (long long i0 = (blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x) & ~63ll; i0 < d;
       i0 += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long i = i0 + lane;
    const int k = i < d ? drops[i] : 0;
    const bool h = i < d && k < keep;
    const unsigned long long m = __ballot(h);
    if (!m) continue;
    unsigned base = 0;
    if (lane == 0) base = atomicAdd(nh, static_cast<unsigned>(__popcll(m)));
    base = static_cast<unsigned>(__shfl(static_cast<int>(base), 0));
    if (h) holes[base + mbcnt(m)] = k;
  }
}

__global__ void k_cap_survivors(const int2* __restrict__ edges, const unsigned* __restrict__ ndrop, long long ne,
                                int* __restrict__ surv, unsigned* __restrict__ ns) {
  const long long keep = ne - static_cast<long long>(*ndrop);
  const int lane = threadIdx.x & 63;
  for (long long k0 = keep + ((blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x) & ~63ll); k0 < ne;
       k0 += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long k = k0 + lane;
    const bool v = k < ne && edges[k].x >= 0;
    const unsigned long long m = __ballot(v);
    if (!m) continue;
    unsigned base = 0;
    if (lane == 0) base = atomicAdd(ns, static_cast<unsigned>(__popcll(m)));
    base = static_cast<unsigned>(__shfl(static_cast<int>(base), 0));
    if (v) surv[base + mbcnt(m)] = static_cast<int>(k);
  }
}

// survivor i into hole i (as many of each); the edge count and the statistics for the host
__global__ void k_cap_fill(int2* __restrict__ edges, unsigned short* __restrict__ iu, const int* __restrict__ holes,
                           const int* __restrict__ surv, const unsigned* __restrict__ cnt, int* __restrict__ err) {
  const unsigned nh = cnt[0], nsv = cnt[1];
  if (blockIdx.x == 0 && threadIdx.x == 0 && nh != nsv) atomicOr(err, kCapErrState);
  const unsigned m = min(nh, nsv);
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
    const int h = holes[i], v = surv[i];
    edges[h] = edges[v];
    iu[h] = iu[v];
  }
}

__global__ void k_cap_commit_runs(const unsigned* __restrict__ ndrop, long long ne,
                                  unsigned long long* __restrict__ counters, int* __restrict__ errw,
                                  long long* __restrict__ stats, const int* __restrict__ err,
                                  long long* __restrict__ host, bool clear) {
  if (threadIdx.x != 0) return;
  const long long kept = ne - static_cast<long long>(*ndrop);
  stats[kStKept] = kept;
  counters[kEdgeCount] = static_cast<unsigned long long>(kept);
  if (clear) {                                       // the sharded replay: the query's flags are settled
    errw[0] = 0;
    errw[kErrOverflow] = 0;
  }
  errw[3] = static_cast<int>(stats[kStMaxFwd]);
  for (int k = 0; k < kStWords; ++k) host[kHStat + k] = stats[k];
  host[kHErr] = *err;
}

__global__ void k_cap_compact(const int2* __restrict__ edges, const unsigned short* __restrict__ iu, long long ne,
                              const unsigned char* __restrict__ who, const int* __restrict__ koff,
                              int2* __restrict__ oe, unsigned short* __restrict__ oiu) {
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < ne;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int w = who[k];
    if (w == 2) continue;
    const int2 e = edges[k];
    const int o = koff[k];
    oe[o] = w == 0 ? e : make_int2(e.y, e.x);
    oiu[o] = iu[k];
  }
}

// each replayed loop's own edge count must equal the edges classified as formed by it
__global__ void k_cap_check(const int* __restrict__ T, int nt, const int* __restrict__ own, const int* __restrict__ pbrk,
                            const int* __restrict__ formed, int n, long long* __restrict__ stats, int* __restrict__ err) {
  int capped = 0, mx = 0;
  const int m = max(n, nt);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
    if (i < nt) {
      if (formed[T[i]] != own[i]) atomicOr(err, kCapErrState);
      capped += pbrk[i] != kInf;
    }
    if (i < n) mx = max(mx, formed[i]);
  }
  capped = block_reduce256(capped, [](int x, int y) { return x + y; });
  mx = block_reduce256(mx, [](int x, int y) { return max(x, y); });
  if (threadIdx.x == 0) {
    if (capped) atomicAdd(reinterpret_cast<unsigned long long*>(stats + kStCapped), static_cast<unsigned long long>(capped));
    atomicMax(reinterpret_cast<long long*>(stats + kStMaxFwd), static_cast<long long>(mx));
  }
}

// the capped graph into the context: edge count, max forward degree; stats + error to pinned memory
__global__ void k_cap_commit(const int* __restrict__ koff, const int* __restrict__ kflag, long long ne,
                             unsigned long long* __restrict__ counters, int* __restrict__ errw,
                             long long* __restrict__ stats, const int* __restrict__ err, long long* __restrict__ host) {
  if (threadIdx.x != 0) return;
  const long long kept = ne ? static_cast<long long>(koff[ne - 1]) + kflag[ne - 1] : 0;
  stats[kStKept] = kept;
  counters[kEdgeCount] = static_cast<unsigned long long>(kept);
  errw[3] = static_cast<int>(stats[kStMaxFwd]);
  for (int k = 0; k < kStWords; ++k) host[kHStat + k] = stats[k];
  host[kHErr] = *err;
}

__global__ void k_cap_total(const int* __restrict__ off, long long i, long long* __restrict__ host, int slot) {
  if (threadIdx.x == 0) host[slot] = off[i];
}

// multi-GPU: install a gathered E* list {a, b, iu, -} (rows with a < 0 are padding), stable
__global__ void k_cap_flag_rows(const int4* __restrict__ rows, long long n, int* __restrict__ f) {
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < n;
       k += static_cast<long long>(gridDim.x) * blockDim.x)
    f[k] = rows[k].x >= 0;
}

__global__ void k_cap_install(const int4* __restrict__ rows, long long n, const int* __restrict__ f,
                              const int* __restrict__ off, int2* __restrict__ edges, unsigned short* __restrict__ iu,
                              long long cap, int* __restrict__ fwd) {
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < n;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    if (!f[k]) continue;
    const int4 r = rows[k];
    const long long o = off[k];
    if (o < cap) {
      edges[o] = make_int2(r.x, r.y);
      iu[o] = static_cast<unsigned short>(r.z);
    }
    atomicAdd(fwd + r.x, 1);
  }
}

__global__ void k_cap_install_commit(const int* __restrict__ off, const int* __restrict__ f, long long n,
                                     const int* __restrict__ fwd, int nr, unsigned long long* __restrict__ counters,
                                     int* __restrict__ errw) {
  int mx = 0;
  for (int i = threadIdx.x; i < nr; i += blockDim.x) mx = max(mx, fwd[i]);
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
  __shared__ int wm[16];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < static_cast<int>(blockDim.x >> 6); ++w) mx = max(mx, wm[w]);
    counters[kEdgeCount] = n ? static_cast<unsigned long long>(off[n - 1] + f[n - 1]) : 0ull;
    errw[0] = 0;
    errw[3] = max(mx, wm[0]);
    errw[kErrOverflow] = 0;
  }
}

__global__ void k_copy_edges_iu(const int2* __restrict__ edges, const unsigned short* __restrict__ iu,
                                const unsigned long long* __restrict__ count, long long cap, int4* __restrict__ out,
                                long long n_pad) {
  const long long ne = min(min(static_cast<long long>(*count), cap), n_pad);
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < n_pad;
       k += static_cast<long long>(gridDim.x) * blockDim.x)
    out[k] = k < ne ? make_int4(edges[k].x, edges[k].y, iu[k], 0) : make_int4(-1, -1, 0, 0);
}

// The query's ZeroDivisionError pairs (kernels.hpp kErrZdCount) against the candidates T: a pair with a
// read outside T is visited by that read's loop, which never breaks (or earlier by the other read's), so
// the reference raises (cluster.py:205-209, 179-181); pairs of two T reads are left to the replay, which
// raises where a replayed loop reaches one.  host[0]: 1 raise, 2 the list overflowed (undecidable), 0.
__global__ __launch_bounds__(256) void k_cap_zd_outside(const int* __restrict__ errw, const int* __restrict__ t_of,
                                                         long long* __restrict__ host) {
  const int cnt = errw[kErrZdCount], cap = errw[kErrZdCap];
  const int m = min(cnt, cap);
  const int2* L = reinterpret_cast<const int2*>(errw + kErrZdList);
  bool out = false;
  for (int k = threadIdx.x; k < m; k += blockDim.x) {
    const int2 p = L[k];
    out = out || t_of[p.x] < 0 || t_of[p.y] < 0;
  }
  out = __syncthreads_or(out);
  if (threadIdx.x == 0) host[0] = out ? 1 : (cnt > cap ? 2 : 0);
}

// fslr_long_pairs: each unordered pair once (the slot of its lower-rank read), its edge (a, b, I, U)
// appended to the long-edge list and to the context's edges; a pair that raises ZeroDivisionError is
// listed in the error words (the caller decides once the edge cap's binding is known)
__global__ void k_cap_pairs_out(const unsigned long long* __restrict__ ukey, int ns, const int* __restrict__ T,
                                const int2* __restrict__ flags, int4* __restrict__ out4, long long cap4,
                                int2* __restrict__ edges, unsigned short* __restrict__ edge_iu, long long edge_cap,
                                unsigned long long* __restrict__ cnt, int* __restrict__ fwd, int* __restrict__ errw) {
  for (int sl = blockIdx.x * blockDim.x + threadIdx.x; sl < ns; sl += gridDim.x * blockDim.x) {
    const unsigned long long key = ukey[sl];
    const int x = T[key >> 25], y = static_cast<int>(key & kKeyMask);
    if (y < x) continue;
    const int2 f = flags[sl];
    raise_zd(errw, f.x & 1, x, y);
    if (!(f.x & 4)) continue;
    const int I = f.y & 0xffff, U = f.y >> 16;
    const unsigned long long k = atomicAdd(cnt, 1ull);
    if (static_cast<long long>(k) < cap4) out4[k] = make_int4(x, y, I, U);
    if (static_cast<long long>(k) < edge_cap) {
      edges[k] = make_int2(x, y);
      edge_iu[k] = static_cast<unsigned short>(min(I, 255) | (min(U, 255) << 8));
    }
    atomicMax(errw + 3, atomicAdd(fwd + x, 1) + 1);     // the forward-degree maximum (cap binding)
  }
}

// ---- 6. the replay sharded over ranks (multi-GPU) -------------------------------
// A loop of T depends on another T read's loop only when one's intervals hit the other's
// (k_cap_mirror's pairs), so the components of the T-T hit graph replay independently: each rank
// replays the components assigned to it and reports only the E* rows its loops do not form in the
// lower read's loop.  Every rank holds the gathered E* (a, b) rows (row w * m + i = rank w's i-th
// edge, a < 0 = padding) and computes the closure T itself.

// the gathered rows' forward degrees
__global__ void k_cap_gfwd(const int2* __restrict__ rows, long long n, int* __restrict__ fwd) {
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < n;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int a = rows[k].x;
    if (a >= 0) atomicAdd(fwd + a, 1);
  }
}

// Every rank sorts its edges by (a, b) before the gather (fslr_sort_edges), so each read's forward edges
// are one run of the gathered rows (in its owner's block): the closure walks those runs instead of an
// adjacency built with per-edge atomics.  [gstart[a], gend[a]) = the run of a; flag: a block not sorted.
__global__ void k_cap_runs(const int2* __restrict__ rows, long long n, long long m, int* __restrict__ gstart,
                           int* __restrict__ gend, int* __restrict__ flag, unsigned long long* __restrict__ valid) {
  unsigned long long cnt = 0;
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < n;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int a = rows[k].x;
    if (a < 0) continue;
    ++cnt;
    const long long kb = k % m;
    const int prev = kb ? rows[k - 1].x : -1;
    if (prev > a || (kb && prev < 0)) atomicOr(flag, 1);          // unsorted, or a row after the padding
    if (prev != a) gstart[a] = static_cast<int>(k);
    const int next = kb + 1 < m && k + 1 < n ? rows[k + 1].x : -1;
    if (next != a) gend[a] = static_cast<int>(k + 1);
  }
  cnt = block_reduce256(cnt, [](unsigned long long x, unsigned long long y) { return x + y; });
  if (threadIdx.x == 0 && cnt) atomicAdd(valid, cnt);
}

// forward degrees from the runs and their total (equal to the valid rows when every read has one run)
__global__ void k_cap_runfwd(const int* __restrict__ gstart, const int* __restrict__ gend, int n, int* __restrict__ fwd,
                             unsigned long long* __restrict__ tot) {
  unsigned long long s = 0;
  for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < n; x += gridDim.x * blockDim.x) {
    const int f = gend[x] - gstart[x];
    fwd[x] = f;
    s += static_cast<unsigned long long>(f);
  }
  s = block_reduce256(s, [](unsigned long long x, unsigned long long y) { return x + y; });
  if (threadIdx.x == 0 && s) atomicAdd(tot, s);
}

// this context's edges by lower read (stable): keys and their positions, then the permutation
__global__ void k_edge_keys(const int2* __restrict__ e, long long n, unsigned* __restrict__ key,
                            int* __restrict__ val) {
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < n;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    key[k] = static_cast<unsigned>(e[k].x);
    val[k] = static_cast<int>(k);
  }
}

__global__ void k_edge_permute(const int2* __restrict__ e, const unsigned short* __restrict__ iu,
                               const int* __restrict__ idx, long long n, int2* __restrict__ oe,
                               unsigned short* __restrict__ oiu) {
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < n;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int i = idx[k];
    oe[k] = e[i];
    oiu[k] = iu[i];
  }
}

// the T-T pairs of this rank's visit lists, one per list element ((-1, -1): a partner outside T), and
// each T read's local hit count.  One wavefront per T-interval.
__global__ __launch_bounds__(256) void k_cap_tdeps(const int* __restrict__ seq, const int* __restrict__ ioff,
                                                   const int* __restrict__ tread, const int* __restrict__ t_of, int nti,
                                                   int2* __restrict__ pairs, int* __restrict__ thits) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int ti = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); ti < nti; ti += nw) {
    const int t = tread[ti];
    const int b0 = ioff[ti], b1 = ioff[ti + 1];
    for (int k = b0 + lane; k < b1; k += 64) {
      const int ty = t_of[seq[k]];
      pairs[k] = ty >= 0 ? make_int2(t, ty) : make_int2(-1, -1);
    }
    if (lane == 0 && b1 > b0) atomicAdd(thits + t, b1 - b0);
  }
}

// per T read: its hits summed over the ranks' gathered counts (the cost of its loop)
__global__ void k_cap_tcost(const int* __restrict__ gath, int world, int nt, int* __restrict__ cost) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += gridDim.x * blockDim.x) {
    int s = 0;
    for (int w = 0; w < world; ++w) s += gath[static_cast<long long>(w) * 2 * nt + nt + t];
    cost[t] = s;
  }
}

// per component (its root = smallest t): its cost (the hits of its reads, plus one per read), and the
// roots order them and the ranks are assigned on the device (k_cap_assign_head / _tail)
__global__ void k_cap_ccost(const int* __restrict__ comp, const int* __restrict__ cost, int nt,
                            unsigned long long* __restrict__ ccost) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += gridDim.x * blockDim.x)
    atomicAdd(ccost + comp[t], static_cast<unsigned long long>(cost[t]) + 1ull);
}

// every T slot as a sort key of 31 + tb bits (tb = bits of nt, so the sort skips the empty high digits): a
// root's (cost descending, then root ascending), all ones for the others (sorted last)
__device__ __forceinline__ unsigned long long cap_key_none(int tb) { return (1ull << (31 + tb)) - 1; }
__global__ void k_cap_rootkeys(const int* __restrict__ comp, const unsigned long long* __restrict__ ccost, int nt,
                               int tb, unsigned long long* __restrict__ keys) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += gridDim.x * blockDim.x)
    keys[t] = comp[t] == t ? ((0x7fffffffull - min(ccost[t], 0x7fffffffull)) << tb) | static_cast<unsigned>(t)
                           : cap_key_none(tb);
}

// the components onto ranks, the same on every rank: the kCapHead largest one by one onto the
// least-loaded rank (ties: the lower rank), by one lane; the rest (sorted by cost, descending) dealt
// in snake order, rank 0 .. W-1 then W-1 .. 0, whose sums differ by at most the largest of them
constexpr int kCapHead = 256;
__global__ void k_cap_assign_head(const unsigned long long* __restrict__ sorted, int nt, int world, int tb,
                                  int* __restrict__ dmap) {
  // One wavefront walks the components (the greedy is sequential) with every value wave-uniform, so
  // the loop runs on the scalar unit: the keys arrive by scalar loads, up to 8 ranks' loads stay in
  // scalar registers (every index static after unrolling); more ranks keep them in LDS.  (One thread
  // with a per-thread array indexed by the rank — scratch memory — took 183 us for 256 components at
  // W = 8, profiles/r06/r6i; a wave-wide min-reduction per component 105 us, r6v; one lane's vector
  // loop 78 us, r6w.)
  __shared__ long long lds_load[kMaxDest];
  const int lane = threadIdx.x & 63;
  const int nh = min(nt, kCapHead);
  const unsigned long long none = cap_key_none(tb), tmask = (1ull << tb) - 1;
  if (world <= 8) {
    // loads as 32-bit (load << 3 | rank) words: the least-loaded rank (ties: the lower) is a tree of
    // seven scalar mins.  Costs are scaled down when 256 of the largest could overflow 29 bits.
    const unsigned long long c0 = nh > 0 && sorted[0] != none ? 0x7fffffffull - (sorted[0] >> tb) : 0ull;
    int shift = 0;
    while ((c0 >> shift) > (1ull << 21)) ++shift;   // 256 x 2^21 = 2^29
    unsigned L[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    for (int k0 = 0; k0 < nh; k0 += 8) {
      unsigned long long kk[8];                    // uniform addresses: 8 scalar loads, one wait
#pragma unroll
      for (int u = 0; u < 8; ++u) kk[u] = k0 + u < nh ? sorted[k0 + u] : none;
      bool done = false;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const unsigned long long key = kk[u];
        if (key == none) {
          done = true;
          break;
        }
        unsigned w8[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) w8[q] = q < world ? (L[q] << 3) | static_cast<unsigned>(q) : 0xFFFFFFFFu;
        const unsigned m01 = min(w8[0], w8[1]), m23 = min(w8[2], w8[3]), m45 = min(w8[4], w8[5]),
                       m67 = min(w8[6], w8[7]);
        const int d = static_cast<int>(min(min(m01, m23), min(m45, m67)) & 7u);
        const unsigned cost = static_cast<unsigned>((0x7fffffffull - (key >> tb)) >> shift);
#pragma unroll
        for (int q = 0; q < 8; ++q) L[q] += q == d ? cost : 0u;
        if (lane == 0) dmap[static_cast<int>(key & tmask)] = d;
      }
      if (done) break;
    }
    return;
  }
  for (int q = lane; q < kMaxDest; q += kWave) lds_load[q] = 0;
  __syncthreads();
  for (int k = 0; k < nh; ++k) {
    const unsigned long long key = sorted[k];
    if (key == none) break;
    int d = 0;
    long long best = lds_load[0];
    for (int q = 1; q < world; ++q) {
      const long long v = lds_load[q];
      if (v < best) {
        best = v;
        d = q;
      }
    }
    __syncthreads();
    if (lane == 0) {
      lds_load[d] = best + static_cast<long long>(0x7fffffffull - (key >> tb));
      dmap[static_cast<int>(key & tmask)] = d;
    }
    __syncthreads();
  }
}

__global__ void k_cap_assign_tail(const unsigned long long* __restrict__ sorted, int nt, int world, int tb,
                                  int* __restrict__ dmap) {
  for (int k = kCapHead + blockIdx.x * blockDim.x + threadIdx.x; k < nt; k += gridDim.x * blockDim.x) {
    const unsigned long long key = sorted[k];
    if (key == cap_key_none(tb)) continue;
    const int j = k - kCapHead, r = j % world;
    dmap[static_cast<int>(key & ((1ull << tb) - 1))] = (j / world) & 1 ? world - 1 - r : r;
  }
}

// every T read's rank: its component root's (dmap holds the roots' ranks)
__global__ void k_cap_tdest(const int* __restrict__ comp, const int* __restrict__ dmap, int nt, int* __restrict__ tdest) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += gridDim.x * blockDim.x) tdest[t] = dmap[comp[t]];
}


// per T-interval: the rank replaying its read's component (sort key), and its index
__global__ void k_cap_tikey(const int* __restrict__ tread, const int* __restrict__ tdest, int nti,
                            unsigned* __restrict__ key, int* __restrict__ val) {
  for (int ti = blockIdx.x * blockDim.x + threadIdx.x; ti < nti; ti += gridDim.x * blockDim.x) {
    key[ti] = static_cast<unsigned>(tdest[tread[ti]]);
    val[ti] = ti;
  }
}

// the local counts in destination order, and per destination its T-intervals and hits (block
// histograms in LDS, then one atomic per bin and block)
__global__ __launch_bounds__(256) void k_cap_sendcnt(const int* __restrict__ tsorted, const unsigned* __restrict__ skey,
                                                     const int* __restrict__ icnt, int nti, int* __restrict__ scnt,
                                                     long long* __restrict__ totals) {
  __shared__ long long h[2 * kMaxDest];
  for (int i = threadIdx.x; i < 2 * kMaxDest; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nti; i += gridDim.x * blockDim.x) {
    const int d = static_cast<int>(skey[i]);
    const int cnt = icnt[tsorted[i]];
    scnt[i] = cnt;
    atomicAdd(reinterpret_cast<unsigned long long*>(h + d), 1ull);
    atomicAdd(reinterpret_cast<unsigned long long*>(h + kMaxDest + d), static_cast<unsigned long long>(cnt));
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * kMaxDest; i += blockDim.x)
    if (h[i]) atomicAdd(reinterpret_cast<unsigned long long*>(totals + i), static_cast<unsigned long long>(h[i]));
}

// the local hit lists in destination order; one wavefront per T-interval
__global__ __launch_bounds__(256) void k_cap_pack(const int* __restrict__ tsorted, const int* __restrict__ scnt,
                                                  const int* __restrict__ shoff, const int* __restrict__ seq,
                                                  const int* __restrict__ ioff, int nti, int* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < nti; i += nw) {
    const int cnt = scnt[i];
    if (!cnt) continue;
    const int* src = seq + ioff[tsorted[i]];
    int* dst = out + shoff[i];
    for (int k = lane; k < cnt; k += 64) dst[k] = src[k];
  }
}

// receiving rank: its T-intervals' counts summed over the W sources (an interval's hits come from the
// one rank indexing its chromosome), at the interval's place in T order (others stay 0)
__global__ void k_cap_recv_sum(const int* __restrict__ rcnt, int world, int nmine, const int* __restrict__ mine,
                               int* __restrict__ icnt) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nmine; i += gridDim.x * blockDim.x) {
    int s = 0;
    for (int w = 0; w < world; ++w) s += rcnt[static_cast<long long>(w) * nmine + i];
    icnt[mine[i]] = s;
  }
}

// the received lists into the visit sequence; roff = exclusive scan of rcnt (source-major, the
// layout of the received hits).  One wavefront per received T-interval.
__global__ __launch_bounds__(256) void k_cap_recv_assemble(const int* __restrict__ rcnt, const int* __restrict__ roff,
                                                           const int* __restrict__ rhits, int world, int nmine,
                                                           const int* __restrict__ mine, const int* __restrict__ ioff,
                                                           int* __restrict__ seq) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < nmine; i += nw) {
    int dst = ioff[mine[i]];
    for (int w = 0; w < world; ++w) {
      const long long j = static_cast<long long>(w) * nmine + i;
      const int cnt = rcnt[j];
      if (!cnt) continue;
      const int* src = rhits + roff[j];
      for (int k = lane; k < cnt; k += 64) seq[dst + k] = src[k];
      dst += cnt;
    }
  }
}

// the gathered rows this rank decides (a T endpoint in one of its components): who = 0 when a's loop
// forms the edge, 1 when b's does, 2 when neither; changes k << 2 | who for who != 0
__global__ void k_cap_classify_shard(const int2* __restrict__ rows, long long n, const int* __restrict__ t_of,
                                     const int* __restrict__ tdest, const int* __restrict__ comp, int rank,
                                     const int* __restrict__ pbrk, const unsigned long long* __restrict__ ukey, const int* __restrict__ tsb,
                                     const int* __restrict__ fpos, const unsigned char* __restrict__ vis2,
                                     int* __restrict__ chg, unsigned* __restrict__ nchg, int* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  for (long long k0 = (blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x) & ~63ll; k0 < n;
       k0 += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long k = k0 + lane;
    int w = 0;
    if (k < n) {
      const int2 e = rows[k];
      const int ta = e.x >= 0 ? t_of[e.x] : -1, tb = e.x >= 0 ? t_of[e.y] : -1;
      const int t = ta >= 0 ? ta : tb;
      if (t >= 0 && tdest[t] == rank) {
        if (ta >= 0 && tb >= 0 && comp[ta] != comp[tb]) {
          atomicOr(err, kCapErrState);                // E* partners hit each other: one component
        } else if (!loop_reaches(e.x, e.y, t_of, pbrk, ukey, tsb, fpos, vis2, err)) {
          w = loop_reaches(e.y, e.x, t_of, pbrk, ukey, tsb, fpos, vis2, err) ? 1 : 2;
        }
      }
    }
    const unsigned long long m = __ballot(w != 0);
    if (!m) continue;
    unsigned base = 0;
    if (lane == 0) base = atomicAdd(nchg, static_cast<unsigned>(__popcll(m)));
    base = static_cast<unsigned>(__shfl(static_cast<int>(base), 0));
    if (w) chg[base + mbcnt(m)] = static_cast<int>((k << 2) | w);
  }
}

// T reads (of this rank's components) whose loop reached the cap
__global__ void k_cap_count_capped(const int* __restrict__ pbrk, int nt, long long* __restrict__ stats) {
  int capped = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nt; i += gridDim.x * blockDim.x) capped += pbrk[i] != kInf;
  for (int o = 32; o > 0; o >>= 1) capped += __shfl_xor(capped, o);
  if ((threadIdx.x & 63) == 0 && capped)
    atomicAdd(reinterpret_cast<unsigned long long*>(stats + kStCapped), static_cast<unsigned long long>(capped));
}

// every rank's changes (-1 = padding): who per gathered row, edges formed per loop
__global__ void k_cap_apply(const int* __restrict__ chg, long long n, const int2* __restrict__ rows,
                            unsigned char* __restrict__ who, int* __restrict__ formed, long long* __restrict__ stats) {
  long long drop = 0, bwd = 0;
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < n;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int v = chg[k];
    if (v < 0) continue;
    const int r = v >> 2, w = v & 3;
    const int2 e = rows[r];
    who[r] = static_cast<unsigned char>(w);
    atomicSub(formed + e.x, 1);
    if (w == 1) atomicAdd(formed + e.y, 1);
    drop += w == 2;
    bwd += w == 1;
  }
  for (int o = 32; o > 0; o >>= 1) {
    drop += __shfl_xor(drop, o);
    bwd += __shfl_xor(bwd, o);
  }
  if ((threadIdx.x & 63) == 0) {
    if (drop) atomicAdd(reinterpret_cast<unsigned long long*>(stats + kStDropped), static_cast<unsigned long long>(drop));
    if (bwd) atomicAdd(reinterpret_cast<unsigned long long*>(stats + kStBackward), static_cast<unsigned long long>(bwd));
  }
}

// this rank's block of rows (its own edges, in its edge order): kept flags
__global__ void k_cap_local_flags(const int2* __restrict__ rows, const unsigned char* __restrict__ who, long long m,
                                  int* __restrict__ kflag) {
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < m;
       i += static_cast<long long>(gridDim.x) * blockDim.x)
    kflag[i] = rows[i].x >= 0 && who[i] != 2;
}

// its kept edges compacted, as (the read whose loop forms it, partner), and edges per former read
__global__ void k_cap_local_compact(const int2* __restrict__ edges, const unsigned short* __restrict__ iu, long long m,
                                    const int* __restrict__ kflag, const int* __restrict__ koff,
                                    const unsigned char* __restrict__ who, int2* __restrict__ oe,
                                    unsigned short* __restrict__ oiu, int* __restrict__ lfwd) {
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < m;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    if (!kflag[i]) continue;
    const int2 e = edges[i];
    const bool fl = who[i] == 1;
    oe[koff[i]] = fl ? make_int2(e.y, e.x) : e;
    oiu[koff[i]] = iu[i];
    atomicAdd(lfwd + (fl ? e.y : e.x), 1);
  }
}

// each loop this rank replayed formed exactly the edges the changes give it; the largest count
__global__ void k_cap_check_shard(const int* __restrict__ T, int nt, const int* __restrict__ tdest, int rank,
                                  const int* __restrict__ own, const int* __restrict__ formed, int n,
                                  long long* __restrict__ stats, int* __restrict__ err) {
  int mx = 0;
  const int m = max(n, nt);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
    if (i < nt && tdest[i] == rank && formed[T[i]] != own[i]) atomicOr(err, kCapErrState);
    if (i < n) mx = max(mx, formed[i]);
  }
  mx = block_reduce256(mx, [](int x, int y) { return max(x, y); });
  if (threadIdx.x == 0) atomicMax(reinterpret_cast<long long*>(stats + kStMaxFwd), static_cast<long long>(mx));
}

__global__ void k_cap_commit_shard(const int* __restrict__ koff, const int* __restrict__ kflag, long long m,
                                   unsigned long long* __restrict__ counters, int* __restrict__ errw,
                                   long long* __restrict__ stats, const int* __restrict__ err,
                                   long long* __restrict__ host) {
  if (threadIdx.x != 0) return;
  const long long kept = m ? static_cast<long long>(koff[m - 1]) + kflag[m - 1] : 0;
  stats[kStKept] = kept;
  counters[kEdgeCount] = static_cast<unsigned long long>(kept);
  errw[0] = 0;
  errw[3] = static_cast<int>(stats[kStMaxFwd]);
  errw[kErrOverflow] = 0;
  for (int k = 0; k < kStWords; ++k) host[kHStat + k] = stats[k];
  host[kHErr] = *err;
}

// ---- the restricted gather -----------------------------------------------------------------------
// A read x joins the closure T only when fwd(x) + back(x) >= thr with back(x) <= bwd(x) over E*, and
// only rows whose lower read is in T are walked by the closure, break a loop or change: the rows
// of S = {x : fwd(x) + bwd(x) >= thr} suffice (3% of E* at cfg5).  Each rank holds every forward row
// of the reads it owns (the partition routes a pair to its lower read's owner: fwd, the context's
// forward degrees, is the whole of it); bwd is a sum over ranks of counts clipped at thr (the test
// fwd + sum >= thr is unchanged by the clip).
__global__ void k_cap_bwdc(const int2* __restrict__ e, long long ne, int* __restrict__ bwd) {
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < ne;
       i += static_cast<long long>(gridDim.x) * blockDim.x)
    atomicAdd(bwd + e[i].y, 1);
}

__global__ void k_cap_clip8(const int* __restrict__ cnt, int n, int thr, unsigned char* __restrict__ out) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    out[i] = static_cast<unsigned char>(min(cnt[i], thr));
}

__global__ void k_cap_rflags(const int2* __restrict__ e, long long ne, const int* __restrict__ fwd,
                             const void* __restrict__ bwd, int eb, int thr, int* __restrict__ flag) {
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < ne;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int a = e[i].x;
    const int b = eb == 1 ? static_cast<int>(static_cast<const unsigned char*>(bwd)[a]) : static_cast<const int*>(bwd)[a];
    flag[i] = fwd[a] + b >= thr;
  }
}

__global__ void k_cap_rcompact(const int2* __restrict__ e, long long ne, const int* __restrict__ flag,
                               const int* __restrict__ off, int2* __restrict__ rows, int* __restrict__ rmap) {
  for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < ne;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    if (!flag[i]) continue;
    rows[off[i]] = e[i];
    rmap[off[i]] = static_cast<int>(i);
  }
}

// the restricted rows by lower read (stable): a sorted (row, local edge) pair list
__global__ void k_cap_rpermute(const int2* __restrict__ rows, const int* __restrict__ rmap, const int* __restrict__ idx,
                               long long n, int2* __restrict__ orows, int* __restrict__ ormap) {
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < n;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int i = idx[k];
    orows[k] = rows[i];
    ormap[k] = rmap[i];
  }
}

// this rank's block of the restricted rows, applied in place on its edges: formers' counts moved,
// re-oriented rows flipped, dropped rows marked (a = -1) and listed for the hole fill
__global__ void k_cap_rapply(const unsigned char* __restrict__ gwho, const int* __restrict__ rmap, long long nr,
                             int2* __restrict__ edges, int* __restrict__ fwd, int* __restrict__ drops,
                             unsigned* __restrict__ ndrop) {
  const int lane = threadIdx.x & 63;
  for (long long j0 = (blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x) & ~63ll; j0 < nr;
       j0 += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long j = j0 + lane;
    const int w = j < nr ? gwho[j] : 0;
    int k = 0;
    if (w) {
      k = rmap[j];
      const int2 e = edges[k];
      atomicSub(fwd + e.x, 1);
      if (w == 1) {
        edges[k] = make_int2(e.y, e.x);
        atomicAdd(fwd + e.y, 1);
      } else {
        edges[k].x = -1;
      }
    }
    const unsigned long long dm = __ballot(w == 2);
    if (!dm) continue;
    unsigned base = 0;
    if (lane == 0) base = atomicAdd(ndrop, static_cast<unsigned>(__popcll(dm)));
    base = static_cast<unsigned>(__shfl(static_cast<int>(base), 0));
    if (w == 2) drops[base + mbcnt(dm)] = k;
  }
}

// reads with no gathered forward row (outside S, or none at all): their own forward edges, held here
__global__ void k_cap_addfwd(int* __restrict__ formed, const int* __restrict__ gfwd, const int* __restrict__ rfwd,
                             int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    if (gfwd[i] == 0) formed[i] += rfwd[i];
}

__global__ void k_fill(int* __restrict__ p, int n, int v) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = v;
}

int bits_for(long long v) {
  int b = 1;
  while ((1ll << b) <= v) ++b;
  return b;
}

int wave_grid(long long items) {
  return static_cast<int>(std::max<long long>(1, std::min<long long>(8192, (items + 3) / 4)));
}

}  // namespace
}  // namespace fslr

using namespace fslr;

// ---- host side: buffers -----------------------------------------------------------------------
// Grow-only device arenas, one per phase (their sizes are known at the phase's start).
struct CapArena {
  char* base = nullptr;
  size_t cap = 0;
};

struct CapWork {
  CapArena ar[11];                     // 0: per read / per edge, 1: per T read / T-interval, 2: per hit (scratch),
                                      // 3: multi-GPU offsets, 4: the visit sequence; the sharded replay:
                                      // 5: gathered rows, 6: plan (per T read / T-interval), 7: T-T pairs,
                                      // 8: received offsets and changes, 9: edge sort scratch,
                                      // 10: the restricted gather (per local edge / read)
  void* temp = nullptr;
  size_t temp_bytes = 0;
  long long* host = nullptr;          // pinned, device-mapped
  long long* host_dev = nullptr;
  int thr = 0;
  int all_shard = 0, all_n_shards = 1;  // cap_local(all_reads): the query shard whose reads form T
  int64_t n = 0, ne = 0, nt = 0, nti = 0, nloc = 0, nseq = 0, ns = 0;
  // the read space of the replay: the uploaded reads, or with reads of more than FSLR_MAX_L
  // intervals (fslr_set_long_reads) the real reads behind the virtual ones
  const int *vreal = nullptr, *vbase = nullptr, *rlen = nullptr, *off2 = nullptr, *umax = nullptr;
  int n_umax = FSLR_MAX_L;
  // phase 0
  int *state = nullptr, *back = nullptr, *t_of = nullptr, *T = nullptr, *toff = nullptr, *formed = nullptr;
  int *aoff = nullptr, *acur = nullptr, *adj = nullptr, *fl0 = nullptr, *fl1 = nullptr;   // frontier closure
  int* tl = nullptr;                  // the frontier closure's members of T (joining order; fcnt[32] of them)
  unsigned* fcnt = nullptr;
  unsigned long long *tv = nullptr, *tvs = nullptr;
  int *chg = nullptr, *err = nullptr, *kflag = nullptr, *koff = nullptr;
  long long* stats = nullptr;
  unsigned char* who = nullptr;
  int2* oedges = nullptr;
  unsigned short* oiu = nullptr;
  // phase 1
  int *tread = nullptr, *tq = nullptr, *icnt = nullptr, *ioff = nullptr, *pbrk = nullptr, *own = nullptr,
      *tpar = nullptr;
  int* tsb = nullptr;                 // each read of T's first slot (tsb[nt] = the slot count)
  int *sbeg = nullptr, *send = nullptr, *indeg = nullptr, *ready = nullptr;   // the loops' dependency DAG
  unsigned* queue = nullptr;
  unsigned long long *ck = nullptr, *ck2 = nullptr;
  // phase 2 (local lists: seqp, seq; then the sequence)
  int *seqp = nullptr, *seq = nullptr, *sval = nullptr, *sval2 = nullptr, *head = nullptr, *hs = nullptr,
      *slot_of = nullptr, *fpos = nullptr, *mslot = nullptr;
  int2* flags = nullptr;
  unsigned long long *skey = nullptr, *skey2 = nullptr, *ukey = nullptr;
  int2* upairs = nullptr;
  unsigned char* vis2 = nullptr;
  int4* rec = nullptr;
  // multi-GPU assembly
  int *gsum = nullptr, *loff = nullptr;
  bool prepared = false;              // fslr_cap_local ran on the current edges
  // the sharded replay (fslr_cap_install_pairs ... fslr_cap_apply_changes)
  bool gmode = false;                 // the closure runs over the gathered rows
  const int2* grows = nullptr;        // gathered E* (a, b) rows, a < 0 = padding (the caller's buffer)
  int *gstart = nullptr, *gend = nullptr;   // each read's run of forward rows (sorted blocks)
  int* gflag = nullptr;
  unsigned long long* gtot = nullptr;       // [2]: valid rows, the runs' total
  bool g_sorted = false;
  int* gfwd = nullptr;                // their forward degrees
  unsigned char* gwho = nullptr;      // per row: 0 formed in a's loop, 1 in b's, 2 dropped
  int64_t g_rows = 0, g_m = 0;
  int g_world = 1, g_rank = 0;
  int *comp = nullptr, *tcost = nullptr, *tdest = nullptr, *tival = nullptr, *tsorted = nullptr, *scnt = nullptr,
      *shoff = nullptr;
  unsigned *tikey = nullptr, *tikey2 = nullptr;
  long long* totals = nullptr;        // [2 kMaxDest]: T-intervals and hits per destination
  unsigned long long* ccost = nullptr;
  int2* roots = nullptr;
  int* dmap = nullptr;
  int64_t nmine = 0, mine_off = 0, planned = 0;
  int2* tdeps = nullptr;
  int *roff = nullptr, *chgl = nullptr;
  unsigned* nchg = nullptr;
  int64_t n_chg = 0;
  bool replayed = false;              // fslr_cap_replay_shard ran (changes ready)
  bool runs1 = false;                 // one GPU: the edge list is grouped by lower read (gstart / gend)
  // the restricted gather (fslr_cap_bwd_counts, fslr_cap_restrict, fslr_cap_install_restricted):
  // local forward counts, the local backward counts (before the sum over ranks), kept flags and
  // offsets of the local edges, the kept rows and their local edge index, local who
  int *rcnt = nullptr, *rflag = nullptr, *rkoff = nullptr, *rmap = nullptr;
  int2* rrows = nullptr;
  int64_t r_ne = 0, r_n = 0;
  int r_thr = 0;
  bool r_counted = false, r_ready = false, g_restricted = false;
};

void fslr_cap_free(fslr_ctx* c) {
  CapWork* w = c->capw;
  if (!w) return;
  for (auto& a : w->ar)
    if (a.base) (void)hipFree(a.base);
  if (w->temp) (void)hipFree(w->temp);
  if (w->host) (void)hipHostFree(w->host);
  delete w;
  c->capw = nullptr;
}


namespace {

// carve typed sub-arrays out of one arena (256-B aligned); grow it first if needed
struct Carve {
  struct Req {
    void** p;
    size_t bytes;
  };
  Req reqs[32];
  int nreq = 0;
  template <typename T>
  void add(T** p, int64_t count) {
    reqs[nreq++] = {reinterpret_cast<void**>(p), static_cast<size_t>(std::max<int64_t>(count, 1)) * sizeof(T)};
  }
  int commit(fslr_ctx* c, CapArena& a) {
    size_t total = 0;
    for (int i = 0; i < nreq; ++i) total += (reqs[i].bytes + 255) & ~size_t(255);
    if (total > a.cap) {
      if (a.base) (void)hipFree(a.base);
      a.base = nullptr;
      a.cap = 0;
      const size_t want = total + total / 8;
      hipError_t e = hipMalloc(reinterpret_cast<void**>(&a.base), want);
      if (e != hipSuccess) return fail(c, FSLR_ERR_NOMEM, std::string("cap replay hipMalloc: ") + hipGetErrorString(e));
      a.cap = want;
    }
    size_t off = 0;
    for (int i = 0; i < nreq; ++i) {
      *reqs[i].p = a.base + off;
      off += (reqs[i].bytes + 255) & ~size_t(255);
    }
    return FSLR_OK;
  }
};

int ensure_temp(fslr_ctx* c, CapWork* w, size_t need) {
  if (need <= w->temp_bytes) return FSLR_OK;
  if (w->temp) (void)hipFree(w->temp);
  w->temp = nullptr;
  w->temp_bytes = 0;
  HIP_TRY(c, hipMalloc(&w->temp, need + need / 8 + 4096));
  w->temp_bytes = need + need / 8 + 4096;
  return FSLR_OK;
}

int cap_work(fslr_ctx* c, CapWork** out) {
  c->hooked = false;                 // every cap path may rewrite the edges
  if (!c->capw) {
    c->capw = new CapWork();
    HIP_TRY(c, hipHostMalloc(reinterpret_cast<void**>(&c->capw->host), kHWords * sizeof(long long), hipHostMallocMapped));
    HIP_TRY(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&c->capw->host_dev), c->capw->host, 0));
  }
  *out = c->capw;
  return FSLR_OK;
}

long long host_word(CapWork* w, int k) {
  return static_cast<const volatile long long*>(w->host)[k];
}

void set_space(fslr_ctx* c, CapWork* w) {
  if (c->lg_set) {
    w->n = c->lg_n_real;
    w->vreal = c->lg_vreal;
    w->vbase = c->lg_vbase;
    w->rlen = c->lg_rlen;
    w->off2 = c->lg_off2;
    w->umax = c->lg_umax;
    w->n_umax = c->lg_n_umax;
  } else {
    w->n = c->n;
    w->vreal = w->vbase = w->rlen = w->off2 = nullptr;
    w->umax = c->umax;
    w->n_umax = FSLR_MAX_L;
  }
}

// The closure over an edge list: rounds over every edge and read (default), or FSLR_CAP_CLOSURE=frontier,
// rounds over the joined reads' forward edges only, through an adjacency built with per-edge atomics.
// Measured at cfg5 (profiles/r04/r4e/): the whole replay 5.15 ms with rounds, 5.9 ms with the frontier
// (its adjacency build, 1.2 ms, costs more than the rounds it saves).  Gathered rows sorted by lower
// read (the sharded replay) have their adjacency for free and always take the frontier.
bool cap_rounds_closure() {
  static const bool v = [] {
    const char* e = std::getenv("FSLR_CAP_CLOSURE");
    return !(e && std::strcmp(e, "frontier") == 0);
  }();
  return v;
}

// The loops' replay: one wavefront per dependency component (default), or FSLR_CAP_REPLAY=dag, a ready
// queue over the loops' DAG (k_cap_replay_dag).  Measured at cfg5 (profiles/r04/cap/): the DAG
// replay's cross-wave hand-offs (agent-scope release / acquire through memory, a few microseconds
// each along the longest dependency chain) made it 7.2 ms against 2.5 ms per component.
// one GPU: the closure over the edge list's runs and the classification of T's runs only, when every
// read's forward edges are one run of the list (default; FSLR_CAP_RUNS=0: always the full-list path)
bool cap_runs_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("FSLR_CAP_RUNS");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return v;
}

// the slots' sort: the segmented radix sort per read of T (hipcub, default), FSLR_CAP_SLOTSORT=lds a
// bitonic sort per read in LDS (a segment of more than 8192 hits: the segmented sort; measured slower:
// 3.32 vs 3.17 ms for the cfg5 replay), =global one radix sort of (read, partner) keys over the whole
// sequence (3.57 ms)
int cap_slot_sort() {
  static const int v = [] {
    const char* e = std::getenv("FSLR_CAP_SLOTSORT");
    if (e && std::strcmp(e, "global") == 0) return 0;
    if (e && std::strcmp(e, "lds") == 0) return 2;
    return 1;
  }();
  return v;
}

// workgroups of a frontier round (grid-stride over the frontier): FSLR_CAP_FGRID, default 1024 (256 and
// 128 measured the same on the cfg5 replay, profiles/r04/r4r/)
int cap_frontier_grid() {
  static const int v = [] {
    const char* e = std::getenv("FSLR_CAP_FGRID");
    const int g = e ? std::atoi(e) : 1024;
    return g >= 1 && g <= 65536 ? g : 1024;
  }();
  return v;
}

bool cap_dag_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("FSLR_CAP_REPLAY");
    return e && std::strcmp(e, "dag") == 0;
  }();
  return v;
}

// FSLR_DEBUG_CAP=1: the dependency components' sizes and per-stage times on stderr (diagnostics; the
// stage times synchronize the stream)
bool cap_debug() {
  static const bool v = std::getenv("FSLR_DEBUG_CAP") != nullptr;
  return v;
}

struct CapTimer {
  bool on;
  hipStream_t s;
  std::chrono::steady_clock::time_point t;
  explicit CapTimer(hipStream_t st) : on(cap_debug()), s(st), t(std::chrono::steady_clock::now()) {
    if (on) (void)hipStreamSynchronize(s);
    t = std::chrono::steady_clock::now();
  }
  void lap(const char* what) {
    if (!on) return;
    (void)hipStreamSynchronize(s);
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "fslr: cap stage %-14s %8.3f ms\n", what,
                 std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
};

// Phase A: the closure T over E* = E[0 .. ne) with forward degrees F (all_reads: every read,
// fslr_long_pairs), the T-intervals and their
// local hit counts; the local visit lists (partner reads, search order) at w->seq[0 .. nloc),
// segments at w->ioff (local counts).
int cap_local(fslr_ctx* c, int thr, CapWork* w, const int2* E, const int* F, int64_t ne, bool all_reads = false,
              const int* rstart = nullptr, const int* rend = nullptr) {
  hipStream_t s = c->stream;
  CapTimer tm(s);
  set_space(c, w);
  const int64_t n = w->n;
  w->thr = thr;
  w->ne = ne;
  w->prepared = false;
  {
    Carve cv;
    cv.add(&w->state, n);
    cv.add(&w->back, n);
    cv.add(&w->t_of, n);
    cv.add(&w->T, n);
    cv.add(&w->toff, n + 1);
    cv.add(&w->formed, n);
    cv.add(&w->tv, n);
    cv.add(&w->tvs, n);
    cv.add(&w->chg, 16);
    cv.add(&w->err, 4);
    cv.add(&w->stats, kStWords);
    cv.add(&w->kflag, ne);
    cv.add(&w->koff, ne);
    cv.add(&w->who, ne);
    cv.add(&w->oedges, ne);
    cv.add(&w->oiu, ne);
    cv.add(&w->aoff, n + 1);
    cv.add(&w->acur, n);
    cv.add(&w->adj, ne);
    cv.add(&w->fl0, n);
    cv.add(&w->fl1, n);
    cv.add(&w->tl, n);
    cv.add(&w->fcnt, 64);
    if (int rc = cv.commit(c, w->ar[0])) return rc;
  }
  HIP_TRY(c, hipMemsetAsync(w->err, 0, 4 * sizeof(int), s));
  HIP_TRY(c, hipMemsetAsync(w->stats, 0, kStWords * sizeof(long long), s));
  // 1. closure.  Frontier rounds (batches of 16, one sync per batch), or FSLR_CAP_CLOSURE=rounds:
  // rounds over every edge and read in batches of 8 (chg[0] = 1 starts each batch)
  const bool frontier = !all_reads && (rstart || !cap_rounds_closure());
  if (all_reads) k_cap_all<<<grid_for(n), 256, 0, s>>>(w->state, static_cast<int>(n), w->all_shard, w->all_n_shards);
  else if (!frontier) k_cap_init<<<grid_for(n), 256, 0, s>>>(F, static_cast<int>(n), thr, w->state, w->back);
  HIP_TRY(c, hipGetLastError());
  if (frontier) {
    HIP_TRY(c, hipMemsetAsync(w->fcnt, 0, 64 * sizeof(unsigned), s));
  }
  if (frontier && !rstart) {
    // the adjacency of E grouped by its lower read (rows sorted by lower read come with their runs)
    HIP_TRY(c, hipMemsetAsync(w->acur, 0, static_cast<size_t>(n) * sizeof(int), s));
    if (ne > 0) k_cap_adj_count<<<grid_for(ne), 256, 0, s>>>(E, ne, w->acur);
    // aoff[0] = 0, aoff[1 .. n] = the inclusive scan of the counts
    size_t tb = 0;
    HIP_TRY(c, hipcub::DeviceScan::InclusiveSum(nullptr, tb, w->acur, w->aoff + 1, static_cast<int>(n), s));
    if (int rc = ensure_temp(c, w, tb)) return rc;
    tb = w->temp_bytes;
    HIP_TRY(c, hipcub::DeviceScan::InclusiveSum(w->temp, tb, w->acur, w->aoff + 1, static_cast<int>(n), s));
    HIP_TRY(c, hipMemsetAsync(w->aoff, 0, sizeof(int), s));
    HIP_TRY(c, hipMemsetAsync(w->acur, 0, static_cast<size_t>(n) * sizeof(int), s));
    if (ne > 0) k_cap_adj_fill<<<grid_for(ne), 256, 0, s>>>(E, ne, w->aoff, w->acur, w->adj);
  }
  unsigned ntl = 0;                    // the frontier closure: |T|
  if (frontier) {
    k_cap_seed<<<grid_for(n), 256, 0, s>>>(F, static_cast<int>(n), thr, w->state, w->back, w->fl0, w->fcnt, w->tl,
                                           w->fcnt + 32);
    HIP_TRY(c, hipGetLastError());
    int* fl[2] = {w->fl0, w->fl1};
    for (int batch = 0;; ++batch) {
      // rounds r = 0 .. 15 of the batch: frontier fl[r & 1] (count fcnt[r]) -> fl[(r + 1) & 1] (fcnt[r + 1])
      const int fg = cap_frontier_grid();
      for (int r = 0; r < 16; ++r) {
        if (rstart)
          k_cap_frontier_w<true><<<fg, 256, 0, s>>>(rstart, rend, E, nullptr, F, thr, w->back, fl[r & 1], w->fcnt + r,
                                                     fl[(r + 1) & 1], w->fcnt + r + 1, w->tl, w->fcnt + 32,
                                                     static_cast<int>(n), ne);
        else
          k_cap_frontier_w<false><<<fg, 256, 0, s>>>(w->aoff, nullptr, nullptr, w->adj, F, thr, w->back, fl[r & 1],
                                                      w->fcnt + r, fl[(r + 1) & 1], w->fcnt + r + 1, w->tl, w->fcnt + 32,
                                                      static_cast<int>(n), ne);
      }
      HIP_TRY(c, hipGetLastError());
      unsigned last = 0;
      HIP_TRY(c, hipMemcpyAsync(&last, w->fcnt + 16, sizeof(unsigned), hipMemcpyDeviceToHost, s));
      HIP_TRY(c, hipMemcpyAsync(&ntl, w->fcnt + 32, sizeof(unsigned), hipMemcpyDeviceToHost, s));
      HIP_TRY(c, hipStreamSynchronize(s));
      if (!last) break;
      if (batch > (n >> 4) + 2) return fail(c, FSLR_ERR_STATE, "edge cap closure does not converge");
      // the next batch starts from frontier fl[0] (16 rounds: an even count) with fcnt[0] = fcnt[16]
      k_cap_fcnt_roll<<<1, 64, 0, s>>>(w->fcnt);
      HIP_TRY(c, hipGetLastError());
    }
  }
  for (int batch = 0; !all_reads && !frontier; ++batch) {
    HIP_TRY(c, hipMemsetAsync(w->chg, 0, 16 * sizeof(int), s));
    HIP_TRY(c, hipMemsetAsync(w->chg, 0xff, sizeof(int), s));
    for (int r = 1; r <= 8; ++r) {
      k_cap_back<<<grid_for(ne), 256, 0, s>>>(E, ne, w->state, w->back, w->chg + r - 1);
      k_cap_join<<<grid_for(n), 256, 0, s>>>(F, static_cast<int>(n), thr, w->state, w->back, w->chg + r - 1,
                                             w->chg + r);
    }
    HIP_TRY(c, hipGetLastError());
    int last = 0;
    HIP_TRY(c, hipMemcpyAsync(&last, w->chg + 8, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    if (!last) break;
    if (batch > (n >> 3) + 2) return fail(c, FSLR_ERR_STATE, "edge cap closure does not converge");
  }
  tm.lap("closure");
  // T in rank order, T-intervals.  The frontier closure listed T's members: sorted, their interval
  // counts scanned (no pass over every read but t_of's reset); the rounds closure: a scan of all reads
  size_t tb = 0;
  if (frontier) {
    const int ntt = static_cast<int>(ntl);
    int* tlen = reinterpret_cast<int*>(w->tv);
    if (ntt > 1) {
      HIP_TRY(c, hipcub::DeviceRadixSort::SortKeys(nullptr, tb, w->tl, w->T, ntt, 0, bits_for(n), s));
      if (int rc = ensure_temp(c, w, tb)) return rc;
      tb = w->temp_bytes;
      HIP_TRY(c, hipcub::DeviceRadixSort::SortKeys(w->temp, tb, w->tl, w->T, ntt, 0, bits_for(n), s));
    } else if (ntt == 1) {
      HIP_TRY(c, hipMemcpyAsync(w->T, w->tl, sizeof(int), hipMemcpyDeviceToDevice, s));
    }
    HIP_TRY(c, hipMemsetAsync(w->t_of, 0xff, static_cast<size_t>(n) * sizeof(int), s));
    k_cap_tfin<<<grid_for(ntt + 1), 256, 0, s>>>(w->T, ntt, c->rmeta, w->rlen, w->t_of, tlen);
    tb = 0;
    HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, tlen, w->toff, ntt + 1, s));
    if (int rc = ensure_temp(c, w, tb)) return rc;
    tb = w->temp_bytes;
    HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(w->temp, tb, tlen, w->toff, ntt + 1, s));
    k_cap_total<<<1, 64, 0, s>>>(w->toff, ntt, w->host_dev, kHNti);
    w->host[kHNt] = ntt;
  } else {
    k_cap_tpack<<<grid_for(n), 256, 0, s>>>(w->state, c->rmeta, w->rlen, static_cast<int>(n), w->tv);
    HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, w->tv, w->tvs, static_cast<int>(n), s));
    if (int rc = ensure_temp(c, w, tb)) return rc;
    tb = w->temp_bytes;
    HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(w->temp, tb, w->tv, w->tvs, static_cast<int>(n), s));
    k_cap_tlist<<<grid_for(n), 256, 0, s>>>(w->state, w->tv, w->tvs, static_cast<int>(n), w->T, w->toff, w->t_of,
                                            w->host_dev);
  }
  if (!all_reads && c->zd_lost)
    return fail(c, FSLR_ERR_STATE, "the ZeroDivisionError pair list overflowed (grown since); rerun the query");
  if (!all_reads) k_cap_zd_outside<<<1, 256, 0, s>>>(c->errw, w->t_of, w->host_dev + kHZd);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipStreamSynchronize(s));
  w->nt = host_word(w, kHNt);
  w->nti = host_word(w, kHNti);
  if (!all_reads && host_word(w, kHZd) == 1) return fail(c, FSLR_ERR_ZERO_DIVISION, "division by zero");
  if (!all_reads && host_word(w, kHZd) == 2)
    return fail(c, FSLR_ERR_STATE, "too many ZeroDivisionError pairs to replay the edge cap; rerun the query");
  const int nt = static_cast<int>(w->nt), nti = static_cast<int>(w->nti);
  {
    Carve cv;
    cv.add(&w->tread, nti);
    cv.add(&w->tq, nti);
    cv.add(&w->icnt, nti + 1);
    cv.add(&w->ioff, nti + 1);
    cv.add(&w->gsum, nti + 1);
    cv.add(&w->pbrk, nt);
    cv.add(&w->own, nt);
    cv.add(&w->tsb, nt + 1);
    cv.add(&w->tpar, nt);
    cv.add(&w->ck, nt);
    cv.add(&w->ck2, nt);
    cv.add(&w->sbeg, nt);
    cv.add(&w->send, nt);
    cv.add(&w->indeg, nt);
    cv.add(&w->ready, nt);
    cv.add(&w->queue, 4);
    if (int rc = cv.commit(c, w->ar[1])) return rc;
  }
  if (nt > 0) {
    k_cap_tread<<<grid_for(nt), 256, 0, s>>>(w->toff, nt, w->tread);
    HIP_TRY(c, hipMemsetAsync(w->tq, 0xff, static_cast<size_t>(nti) * sizeof(int), s));
    if (!c->lg_set && !w->vreal)
      k_cap_tq_bs<<<grid_for(nti), 256, 0, s>>>(w->tread, w->T, w->toff, nti, c->rmeta, c->iv,
                                                c->filter_active ? c->fmap : nullptr,
                                                c->filter_active ? c->crange_f : c->crange, c->s_start, c->idx4,
                                                w->tq, w->err);
    else
      k_cap_tq<<<grid_for(c->ni_idx), 256, 0, s>>>(c->idx4, static_cast<int>(c->ni_idx), w->t_of, w->toff, w->vreal,
                                                   w->vbase, w->tq);
    // 2. hits of the T-intervals this index holds: count, scan, emit top-down, ties, partner reads
    k_cap_hits<false><<<wave_grid(nti), 256, 0, s>>>(w->tq, w->tread, w->T, c->idx4, c->rng_s, w->vreal, nti,
                                                      w->icnt, nullptr, nullptr);
    HIP_TRY(c, hipGetLastError());
  }
  HIP_TRY(c, hipMemsetAsync(w->icnt + nti, 0, sizeof(int), s));
  tb = 0;
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, w->icnt, w->ioff, nti + 1, s));
  if (int rc = ensure_temp(c, w, tb)) return rc;
  tb = w->temp_bytes;
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(w->temp, tb, w->icnt, w->ioff, nti + 1, s));
  k_cap_total<<<1, 64, 0, s>>>(w->ioff, nti, w->host_dev, kHNloc);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipStreamSynchronize(s));
  w->nloc = host_word(w, kHNloc);
  tm.lap("T, hit counts");
  if (w->nloc >= (int64_t(1) << 31)) return fail(c, FSLR_ERR_NOMEM, "edge cap replay: more than 2^31 hits");
  {
    Carve c2, c4;
    c2.add(&w->seqp, w->nloc);
    c4.add(&w->seq, w->nloc);
    if (int rc = c2.commit(c, w->ar[2])) return rc;
    if (int rc = c4.commit(c, w->ar[4])) return rc;
  }
  if (nti > 0 && w->nloc > 0) {
    k_cap_hits<true><<<wave_grid(nti), 256, 0, s>>>(w->tq, w->tread, w->T, c->idx4, c->rng_s, w->vreal, nti, nullptr,
                                                     w->ioff, w->seqp);
    k_cap_seq<<<wave_grid(nti), 256, 0, s>>>(w->seqp, c->idx4, w->ioff, w->vreal, nti, w->seq);
    HIP_TRY(c, hipGetLastError());
  }
  tm.lap("hit lists");
  w->prepared = true;
  return FSLR_OK;
}

// Phase B: the sequence (w->seq, segments w->ioff, w->nseq elements) -> slots, predicates, loops,
// the capped graph written back into the context.
// 3. slots: the distinct partners of each read of T — a stable radix sort of (t, partner) keys by
// sequence position, unique — and each slot's pair predicate.  Returns the slot count in w->ns.
int cap_slots(fslr_ctx* c, CapWork* w) {
  hipStream_t s = c->stream;
  const int nt = static_cast<int>(w->nt), nti = static_cast<int>(w->nti);
  const int m = static_cast<int>(w->nseq);
  {
    Carve cv;                          // the sequence itself lives in arena 4
    cv.add(&w->sval, m);
    cv.add(&w->sval2, m);
    cv.add(&w->head, m);
    cv.add(&w->hs, m);
    cv.add(&w->slot_of, m);
    cv.add(&w->fpos, m);
    cv.add(&w->flags, m);
    cv.add(&w->mslot, m);
    cv.add(&w->skey, m);
    cv.add(&w->skey2, m);
    cv.add(&w->ukey, m);
    cv.add(&w->upairs, m);
    cv.add(&w->vis2, m);
    cv.add(&w->rec, m);
    if (int rc = cv.commit(c, w->ar[2])) return rc;
  }
  w->ns = 0;
  if (m == 0) {
    HIP_TRY(c, hipMemsetAsync(w->tsb, 0, static_cast<size_t>(nt + 1) * sizeof(int), s));
    return FSLR_OK;
  }
  CapTimer tm(s);
  size_t b1 = 0, b2 = 0, b3 = 0;
  const int kbits = 25 + bits_for(nt);
  int mode = cap_slot_sort();                                      // 0 global, 1 segmented radix, 2 LDS
  unsigned* pkey = reinterpret_cast<unsigned*>(w->skey);           // segmented: 32-bit partners
  unsigned* pkey2 = pkey + m;
  int* segb = reinterpret_cast<int*>(w->ck);                       // nt + 1 segment offsets (ck: 2 nt ints)
  const int pbits = bits_for(std::max<int64_t>(w->n, 1));
  unsigned* segmax = reinterpret_cast<unsigned*>(w->chg) + 8;
  HIP_TRY(c, hipMemsetAsync(segmax, 0, sizeof(unsigned), s));
  k_cap_segb<<<grid_for(nt + 1), 256, 0, s>>>(w->ioff, w->toff, nt, segb, segmax);
  if (mode == 2) {
    unsigned smax = 0;
    HIP_TRY(c, hipMemcpyAsync(&smax, segmax, sizeof(smax), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    if (smax > static_cast<unsigned>(kSegBig)) mode = 1;          // a segment beyond the LDS sort
  }
  const bool seg = mode != 0;
  if (mode == 2) {
    k_cap_segsort<kSegSmall><<<std::min(nt, 8192), 256, 0, s>>>(w->seq, segb, nt, 0, pkey2, w->sval2);
    k_cap_segsort<kSegBig><<<std::min(nt, 512), 256, 0, s>>>(w->seq, segb, nt, kSegSmall, pkey2, w->sval2);
    HIP_TRY(c, hipGetLastError());
  } else if (seg) {
    k_cap_pkeys<<<grid_for(m), 256, 0, s>>>(w->seq, m, pkey, w->sval);
    HIP_TRY(c, hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, b1, pkey, pkey2, w->sval, w->sval2, m, nt, segb,
                                                           segb + 1, 0, pbits, s));
  } else {
    k_cap_keys<<<wave_grid(nti), 256, 0, s>>>(w->seq, w->ioff, w->tread, nti, w->skey, w->sval);
    HIP_TRY(c, hipcub::DeviceRadixSort::SortPairs(nullptr, b1, w->skey, w->skey2, w->sval, w->sval2, m, 0, kbits, s));
  }
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, b2, w->head, w->hs, m, s));
  HIP_TRY(c, hipcub::DeviceRadixSort::SortKeys(nullptr, b3, w->ck, w->ck2, std::max(nt, 1), 0, 50, s));
  if (int rc = ensure_temp(c, w, std::max({b1, b2, b3}))) return rc;
  size_t tb = w->temp_bytes;
  if (seg) {
    if (mode == 1)
      HIP_TRY(c, hipcub::DeviceSegmentedRadixSort::SortPairs(w->temp, tb, pkey, pkey2, w->sval, w->sval2, m, nt, segb,
                                                             segb + 1, 0, pbits, s));
    k_cap_rekey<<<wave_grid(nt), 256, 0, s>>>(pkey2, segb, nt, w->skey2);
  } else {
    HIP_TRY(c, hipcub::DeviceRadixSort::SortPairs(w->temp, tb, w->skey, w->skey2, w->sval, w->sval2, m, 0, kbits, s));
  }
  k_cap_heads<<<grid_for(m), 256, 0, s>>>(w->skey2, m, w->head);
  tb = w->temp_bytes;
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(w->temp, tb, w->head, w->hs, m, s));
  k_cap_slots<<<grid_for(m), 256, 0, s>>>(w->skey2, w->sval2, w->head, w->hs, m, w->slot_of, w->ukey, w->fpos,
                                          w->host_dev);
  k_cap_tsb<<<grid_for(nt + 1), 256, 0, s>>>(w->hs, w->head, segb, nt, m, w->tsb);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipStreamSynchronize(s));
  const int ns = static_cast<int>(host_word(w, kHNslots));
  w->ns = ns;
  tm.lap("slots: sort");
  k_cap_eval<<<wave_grid((ns + 63) / 64), 256, 0, s>>>(w->ukey, ns, w->T, c->rmeta, c->iv, w->rlen, w->off2, c->last_qcut,
                                           c->last_ncut, w->umax, w->n_umax, w->flags);
  HIP_TRY(c, hipGetLastError());
  tm.lap("slots: eval");
  return FSLR_OK;
}

// 3 + 4: slots, predicates and every read of T's loop (pbrk, own, visit marks)
int cap_loops(fslr_ctx* c, CapWork* w) {
  hipStream_t s = c->stream;
  const int thr = w->thr;
  const int nt = static_cast<int>(w->nt);
  const int m = static_cast<int>(w->nseq);
  if (int rc = cap_slots(c, w)) return rc;
  CapTimer tm(s);
  const int ns = static_cast<int>(w->ns);
  if (m > 0) {
    // mirror slots; each read's earlier T partners (its in-degree in the loops' dependency DAG)
    // (one pair per slot, (-1, -1) for none: compacting the T-T pairs through one counter cost 0.9 ms)
    k_cap_mirror<<<grid_for(ns), 256, 0, s>>>(w->ukey, ns, w->tsb, w->T, w->t_of, w->mslot, w->upairs, w->err);
    k_cap_recs<<<grid_for(m), 256, 0, s>>>(w->slot_of, w->ukey, w->fpos, w->flags, w->mslot, w->T, w->t_of, m, w->rec);
    HIP_TRY(c, hipMemsetAsync(w->vis2, 0, static_cast<size_t>(ns), s));
    tm.lap("loops: mirror");
    bool dag_ok = false;
    if (cap_dag_enabled()) {
      HIP_TRY(c, hipMemsetAsync(w->sbeg, 0, static_cast<size_t>(nt) * sizeof(int), s));
      HIP_TRY(c, hipMemsetAsync(w->send, 0, static_cast<size_t>(nt) * sizeof(int), s));
      HIP_TRY(c, hipMemsetAsync(w->indeg, 0, static_cast<size_t>(nt) * sizeof(int), s));
      HIP_TRY(c, hipMemsetAsync(w->ready, 0xff, static_cast<size_t>(nt) * sizeof(int), s));
      HIP_TRY(c, hipMemsetAsync(w->queue, 0, 4 * sizeof(unsigned), s));
      k_cap_dag_bounds<<<grid_for(ns), 256, 0, s>>>(w->ukey, ns, w->sbeg, w->send);
      k_cap_dag_indeg<<<grid_for(ns), 256, 0, s>>>(w->upairs, ns, w->indeg);
      k_cap_dag_seed<<<grid_for(nt), 256, 0, s>>>(w->indeg, nt, w->ready, w->queue + 1);
      // 4. the loops, each as soon as its earlier T partners' loops are done
      k_cap_replay_dag<<<std::min(wave_grid(nt), 2048), 256, 0, s>>>(nt, thr, w->T, w->t_of, w->toff, w->ioff, w->rec,
                                                                    w->fpos, w->ukey, w->sbeg, w->send, w->indeg,
                                                                    w->ready, w->queue, w->vis2, w->pbrk, w->own,
                                                                    w->err);
      HIP_TRY(c, hipGetLastError());
      int derr[2] = {0, 0};
      HIP_TRY(c, hipMemcpyAsync(derr, w->err, sizeof(derr), hipMemcpyDeviceToHost, s));
      HIP_TRY(c, hipStreamSynchronize(s));
      dag_ok = derr[1] == 0;
      if (!dag_ok) {                     // a loop never became ready (cannot happen): replay per component
        std::fprintf(stderr, "fslr: edge-cap DAG replay stalled; replaying per component\n");
        HIP_TRY(c, hipMemsetAsync(w->err + 1, 0, sizeof(int), s));
        HIP_TRY(c, hipMemsetAsync(w->vis2, 0, static_cast<size_t>(ns), s));
      }
    }
    if (!dag_ok) {
      // the dependency components, one wavefront per component, its reads in rank order
      HIP_TRY(c, launch_uf_init(w->tpar, nt, s));
      HIP_TRY(c, launch_uf_pair_list(w->tpar, w->upairs, ns, s));
      HIP_TRY(c, launch_uf_finalize(w->tpar, nt, s));
      k_cap_ckeys<<<grid_for(nt), 256, 0, s>>>(w->tpar, nt, w->ck);
      size_t tb = w->temp_bytes;
      HIP_TRY(c, hipcub::DeviceRadixSort::SortKeys(w->temp, tb, w->ck, w->ck2, nt, 0, 25 + bits_for(nt), s));
      tm.lap("loops: comps");
      if (cap_debug()) {
        std::vector<int> par(nt), toff(nt + 1), ioff(static_cast<size_t>(w->nti) + 1);
        HIP_TRY(c, hipMemcpyAsync(par.data(), w->tpar, nt * sizeof(int), hipMemcpyDeviceToHost, s));
        HIP_TRY(c, hipMemcpyAsync(toff.data(), w->toff, (nt + 1) * sizeof(int), hipMemcpyDeviceToHost, s));
        HIP_TRY(c, hipMemcpyAsync(ioff.data(), w->ioff, ioff.size() * sizeof(int), hipMemcpyDeviceToHost, s));
        HIP_TRY(c, hipStreamSynchronize(s));
        std::vector<long long> sz(nt, 0), hits(nt, 0);
        for (int t = 0; t < nt; ++t) {
          ++sz[par[t]];
          hits[par[t]] += ioff[toff[t + 1]] - ioff[toff[t]];
        }
        long long ncomp = 0, big = 0, bighits = 0, maxhits = 0;
        for (int t = 0; t < nt; ++t) {
          ncomp += sz[t] > 0;
          if (sz[t] > big) { big = sz[t]; bighits = hits[t]; }
          maxhits = std::max(maxhits, hits[t]);
        }
        std::fprintf(stderr, "fslr: cap replay %d loops in %lld components; largest %lld loops (%lld hits); most hits %lld; %lld hits\n",
                     nt, ncomp, big, bighits, maxhits, static_cast<long long>(w->nseq));
      }
      k_cap_replay<<<wave_grid(nt), 256, 0, s>>>(w->ck2, nt, thr, w->toff, w->ioff, w->rec, w->fpos, w->vis2,
                                                 w->pbrk, w->own, w->err);
      HIP_TRY(c, hipGetLastError());
    }
  } else if (nt > 0) {
    // no T read has a hit: no loop breaks
    k_fill<<<grid_for(nt), 256, 0, s>>>(w->pbrk, nt, kInf);
    k_fill<<<grid_for(nt), 256, 0, s>>>(w->own, nt, 0);
    HIP_TRY(c, hipGetLastError());
  }
  w->ns = ns;
  tm.lap("loops: replay");
  return FSLR_OK;
}

int cap_core(fslr_ctx* c, CapWork* w, fslr_cap_stats* cs) {
  hipStream_t s = c->stream;
  const int64_t n = w->n, ne = w->ne;
  const int nt = static_cast<int>(w->nt);
  if (int rc = cap_loops(c, w)) return rc;
  const int ns = static_cast<int>(w->ns);
  CapTimer tm(s);
  // 5. the capped graph
  // edges formed per loop, from the E* forward degrees (fwd[x] = E* edges (x, .), as the query or the
  // install left them)
  if (!w->runs1)
    HIP_TRY(c, hipMemcpyAsync(w->formed, c->fwd, static_cast<size_t>(n) * sizeof(int), hipMemcpyDeviceToDevice, s));
  if (w->runs1) {
    // the forward degrees become the edges formed per loop in place (the changes move a few)
    // only T's runs can change: classified in place, then the dropped rows' holes filled
    unsigned* cnt = reinterpret_cast<unsigned*>(w->chg);          // [0] dropped, [1] holes, [2] survivors
    HIP_TRY(c, hipMemsetAsync(cnt, 0, 4 * sizeof(unsigned), s));
    if (nt > 0)
      k_cap_classify_runs<<<std::min(wave_grid(nt), 4096), 256, 0, s>>>(
          c->edges, w->gstart, w->gend, w->T, nt, w->t_of, w->pbrk, w->ukey, w->tsb, w->fpos, w->vis2, c->fwd,
          w->kflag, cnt, w->stats, w->err);
    k_cap_holes<<<256, 256, 0, s>>>(w->kflag, cnt, ne, w->koff, cnt + 1);
    k_cap_survivors<<<256, 256, 0, s>>>(c->edges, cnt, ne, w->adj, cnt + 2);
    k_cap_fill<<<256, 256, 0, s>>>(c->edges, c->edge_iu, w->koff, w->adj, cnt + 1, w->err);
    k_cap_check<<<grid_for(std::max<int64_t>(n, nt)), 256, 0, s>>>(w->T, nt, w->own, w->pbrk, c->fwd,
                                                                   static_cast<int>(n), w->stats, w->err);
    k_cap_commit_runs<<<1, 64, 0, s>>>(cnt, ne, c->counters, c->errw, w->stats, w->err, w->host_dev, false);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipStreamSynchronize(s));
  } else if (ne > 0) {
    k_cap_classify<<<grid_for(ne), 256, 0, s>>>(c->edges, ne, w->t_of, w->pbrk, w->ukey, w->tsb, w->fpos, w->vis2,
                                                w->kflag, w->who, w->formed, w->stats, w->err);
    size_t tb = 0;
    HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, w->kflag, w->koff, static_cast<int>(ne), s));
    if (int rc = ensure_temp(c, w, tb)) return rc;
    tb = w->temp_bytes;
    HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(w->temp, tb, w->kflag, w->koff, static_cast<int>(ne), s));
    k_cap_compact<<<grid_for(ne), 256, 0, s>>>(c->edges, c->edge_iu, ne, w->who, w->koff, w->oedges, w->oiu);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipMemcpyAsync(c->edges, w->oedges, static_cast<size_t>(ne) * sizeof(int2), hipMemcpyDeviceToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(c->edge_iu, w->oiu, static_cast<size_t>(ne) * sizeof(unsigned short),
                              hipMemcpyDeviceToDevice, s));
  }
  if (!w->runs1) {
    k_cap_check<<<grid_for(std::max<int64_t>(n, nt)), 256, 0, s>>>(w->T, nt, w->own, w->pbrk, w->formed,
                                                                   static_cast<int>(n), w->stats, w->err);
    HIP_TRY(c, hipMemcpyAsync(c->fwd, w->formed, static_cast<size_t>(n) * sizeof(int), hipMemcpyDeviceToDevice, s));
    k_cap_commit<<<1, 64, 0, s>>>(w->koff, w->kflag, ne, c->counters, c->errw, w->stats, w->err, w->host_dev);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  w->runs1 = false;
  tm.lap("classify");
  const long long err = host_word(w, kHErr);
  if (err & kCapErrZd) return fail(c, FSLR_ERR_ZERO_DIVISION, "division by zero");
  if (err & kCapErrState) return fail(c, FSLR_ERR_STATE, "edge cap replay: inconsistent loop replay");
  cs->applied = 1;
  cs->max_fwd = static_cast<int32_t>(host_word(w, kHStat + kStMaxFwd));
  cs->candidates = w->nt;
  cs->capped = host_word(w, kHStat + kStCapped);
  cs->hits = w->nseq;
  cs->pairs = ns;
  cs->dropped = host_word(w, kHStat + kStDropped);
  cs->backward = host_word(w, kHStat + kStBackward);
  w->prepared = false;
  return FSLR_OK;
}

// edge count, max forward degree; FSLR_OK and *binds = false when E* is the reference's graph
int cap_peek(fslr_ctx* c, int thr, int64_t* ne, bool* binds) {
  long long pk[4] = {0, 0, 0, 0};
  if (c->counters) {
    if (int rc = peek_counts(c, pk)) return rc;
  } else {
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  if (pk[1] == FSLR_ERR_ZERO_DIVISION) return fail(c, FSLR_ERR_ZERO_DIVISION, "division by zero");
  *ne = pk[0];
  // a listed ZeroDivisionError pair raises when every loop runs to its end (the cap does not bind);
  // otherwise only where a loop reaches it (cap_local: a pair with a read outside T; the replay)
  if (pk[3] > 0 && !c->cap_stats.applied && pk[2] <= thr) return fail(c, FSLR_ERR_ZERO_DIVISION, "division by zero");
  if (*ne > c->edge_cap) return fail(c, FSLR_ERR_STATE, "edge buffer overflowed; reserve and rerun the query");
  *binds = !c->cap_stats.applied && pk[2] > thr;
  if (!*binds && !c->cap_stats.applied) {
    std::memset(&c->cap_stats, 0, sizeof(c->cap_stats));
    c->cap_stats.max_fwd = static_cast<int32_t>(pk[2]);
  }
  return FSLR_OK;
}

}  // namespace

extern "C" int fslr_apply_edge_cap(fslr_ctx* c, int32_t thr, fslr_cap_stats* out) {
  if (!c) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  int64_t ne = 0;
  bool binds = false;
  if (int rc = cap_peek(c, thr, &ne, &binds)) return rc;
  if (!binds) {
    if (out) *out = c->cap_stats;
    return FSLR_OK;
  }
  if (!c->last_full && !c->edges_global)
    return fail(c, FSLR_ERR_STATE, "the edge cap binds: its replay needs the last query to cover every read on "
                                   "one context (fslr_query over [0, n_reads)) or fslr_cap_install_edges");
  if (c->filter_active)
    return fail(c, FSLR_ERR_STATE, "the index covers a chromosome subset: use fslr_cap_local / fslr_cap_replay");
  if (int rc = ensure_bwd_ranges(c)) return rc;
  CapWork* w = nullptr;
  if (int rc = cap_work(c, &w)) return rc;
  // each read's forward edges one run of the list (the sweep engine's order)?  Then the closure walks
  // the runs and only T's runs are classified (FSLR_CAP_RUNS=0: the full-list path)
  w->runs1 = false;
  if (!c->lg_set && ne > 0 && cap_runs_enabled()) {
    const int n = static_cast<int>(c->n);
    {
      Carve cv;
      cv.add(&w->gstart, n);
      cv.add(&w->gend, n);
      cv.add(&w->gflag, 4);
      if (int rc = cv.commit(c, w->ar[5])) return rc;
    }
    hipStream_t s = c->stream;
    HIP_TRY(c, hipMemsetAsync(w->gstart, 0, static_cast<size_t>(n) * sizeof(int), s));
    HIP_TRY(c, hipMemsetAsync(w->gend, 0, static_cast<size_t>(n) * sizeof(int), s));
    HIP_TRY(c, hipMemsetAsync(w->gflag, 0, 4 * sizeof(int), s));
    k_cap_runs1<<<grid_for(ne), 256, 0, s>>>(c->edges, ne, w->gstart, w->gend, w->gflag);
    HIP_TRY(c, hipGetLastError());
    int flag = 0;
    HIP_TRY(c, hipMemcpyAsync(&flag, w->gflag, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    w->runs1 = flag == 0;
    if (cap_debug()) std::fprintf(stderr, "fslr: cap edge list grouped by lower read: %d\n", w->runs1);
  }
  if (int rc = cap_local(c, thr, w, c->edges, c->fwd, ne, false, w->runs1 ? w->gstart : nullptr,
                         w->runs1 ? w->gend : nullptr))
    return rc;
  w->nseq = w->nloc;
  fslr_cap_stats cs;
  std::memset(&cs, 0, sizeof(cs));
  if (int rc = cap_core(c, w, &cs)) return rc;
  c->cap_stats = cs;
  if (out) *out = cs;
  return FSLR_OK;
}

extern "C" int fslr_copy_edges_iu_device(fslr_ctx* c, int32_t* dst, int64_t n_pad) {
  if (!c || (!dst && n_pad) || n_pad < 0) return FSLR_ERR_INVALID;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  HIP_TRY(c, hipSetDevice(c->device));
  if (n_pad == 0) return FSLR_OK;
  if (!c->edge_cap) return fail(c, FSLR_ERR_STATE, "no query has run");
  k_copy_edges_iu<<<grid_for(n_pad), 256, 0, c->stream>>>(c->edges, c->edge_iu, c->counters + kEdgeCount, c->edge_cap,
                                                          reinterpret_cast<int4*>(dst), n_pad);
  HIP_TRY(c, hipGetLastError());
  return FSLR_OK;
}

extern "C" int fslr_cap_install_edges(fslr_ctx* c, const int32_t* rows, int64_t n_rows) {
  if (!c || (!rows && n_rows) || n_rows < 0 || n_rows >= (int64_t(1) << 31)) return FSLR_ERR_INVALID;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  if (c->edge_cap < n_rows) {
    if (int rc = fslr_reserve_edges(c, n_rows)) return rc;
  }
  if (!c->counters) return fail(c, FSLR_ERR_STATE, "no query has run");
  CapWork* w = nullptr;
  if (int rc = cap_work(c, &w)) return rc;
  int *f = nullptr, *off = nullptr;
  Carve cv;
  cv.add(&f, n_rows);
  cv.add(&off, n_rows);
  if (int rc = cv.commit(c, w->ar[3])) return rc;
  const int4* r4 = reinterpret_cast<const int4*>(rows);
  HIP_TRY(c, hipMemsetAsync(c->fwd, 0, static_cast<size_t>(c->n) * sizeof(int), s));
  if (n_rows > 0) {
    k_cap_flag_rows<<<grid_for(n_rows), 256, 0, s>>>(r4, n_rows, f);
    size_t tb = 0;
    HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, f, off, static_cast<int>(n_rows), s));
    if (int rc = ensure_temp(c, w, tb)) return rc;
    tb = w->temp_bytes;
    HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(w->temp, tb, f, off, static_cast<int>(n_rows), s));
    k_cap_install<<<grid_for(n_rows), 256, 0, s>>>(r4, n_rows, f, off, c->edges, c->edge_iu, c->edge_cap, c->fwd);
  }
  k_cap_install_commit<<<1, 1024, 0, s>>>(off, f, n_rows, c->fwd, static_cast<int>(c->n), c->counters, c->errw);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipStreamSynchronize(s));
  c->edges_global = true;
  c->cap_gmode = false;
  std::memset(&c->cap_stats, 0, sizeof(c->cap_stats));
  return FSLR_OK;
}

extern "C" int fslr_cap_local(fslr_ctx* c, int32_t thr, int64_t* n_ti, int64_t* n_hits) {
  if (!c || !n_ti || !n_hits) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  *n_ti = *n_hits = 0;
  if (c->cap_gmode) {                  // the sharded replay: the closure over the gathered rows
    CapWork* w = c->capw;
    if (int rc = ensure_bwd_ranges(c)) return rc;
    if (int rc = cap_local(c, thr, w, w->grows, w->gfwd, w->g_rows, false, w->g_sorted ? w->gstart : nullptr,
                           w->g_sorted ? w->gend : nullptr))
      return rc;
    w->planned = 0;
    w->replayed = false;
    *n_ti = w->nti;
    *n_hits = w->nloc;
    return FSLR_OK;
  }
  if (!c->edges_global && !c->last_full)
    return fail(c, FSLR_ERR_STATE, "fslr_cap_local needs every E* edge on this context (fslr_cap_install_edges)");
  int64_t ne = 0;
  bool binds = false;
  if (int rc = cap_peek(c, thr, &ne, &binds)) return rc;
  if (!binds) return fail(c, FSLR_ERR_STATE, "the edge cap does not bind");
  if (int rc = ensure_bwd_ranges(c)) return rc;
  CapWork* w = nullptr;
  if (int rc = cap_work(c, &w)) return rc;
  if (int rc = cap_local(c, thr, w, c->edges, c->fwd, ne)) return rc;
  *n_ti = w->nti;
  *n_hits = w->nloc;
  return FSLR_OK;
}

extern "C" int fslr_cap_copy_local(fslr_ctx* c, int32_t* counts, int32_t* hits) {
  if (!c || !c->capw || !c->capw->prepared) return c ? fail(c, FSLR_ERR_STATE, "fslr_cap_local first") : FSLR_ERR_INVALID;
  CapWork* w = c->capw;
  if ((!counts && w->nti) || (!hits && w->nloc)) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  if (w->nti)
    HIP_TRY(c, hipMemcpyAsync(counts, w->icnt, static_cast<size_t>(w->nti) * sizeof(int), hipMemcpyDeviceToDevice,
                              c->stream));
  if (w->nloc)
    HIP_TRY(c, hipMemcpyAsync(hits, w->seq, static_cast<size_t>(w->nloc) * sizeof(int), hipMemcpyDeviceToDevice,
                              c->stream));
  return FSLR_OK;
}

extern "C" int fslr_cap_replay(fslr_ctx* c, const int32_t* counts, const int32_t* lists, int64_t pad, int32_t world,
                               fslr_cap_stats* out) {
  if (!c || world < 1 || pad < 0) return FSLR_ERR_INVALID;
  if (!c->capw || !c->capw->prepared) return fail(c, FSLR_ERR_STATE, "fslr_cap_local first");
  CapWork* w = c->capw;
  if ((!counts && w->nti) || (!lists && pad)) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const int nti = static_cast<int>(w->nti);
  const int64_t nall = static_cast<int64_t>(world) * nti;
  if (nall >= (int64_t(1) << 31)) return fail(c, FSLR_ERR_INVALID, "too many T-intervals");
  {
    Carve cv;
    cv.add(&w->loff, nall + 1);
    if (int rc = cv.commit(c, w->ar[3])) return rc;
  }
  // global counts and offsets, then each rank's segments into the sequence
  k_cap_sum_counts<<<grid_for(nti + 1), 256, 0, s>>>(counts, world, nti, w->gsum);
  size_t b1 = 0, b2 = 0;
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, b1, w->gsum, w->ioff, nti + 1, s));
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, b2, counts, w->loff, static_cast<int>(std::max<int64_t>(nall, 1)), s));
  if (int rc = ensure_temp(c, w, std::max(b1, b2))) return rc;
  size_t tb = w->temp_bytes;
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(w->temp, tb, w->gsum, w->ioff, nti + 1, s));
  if (nall > 0) {
    tb = w->temp_bytes;
    HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(w->temp, tb, counts, w->loff, static_cast<int>(nall), s));
  }
  k_cap_total<<<1, 64, 0, s>>>(w->ioff, nti, w->host_dev, kHNseq);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipStreamSynchronize(s));
  w->nseq = host_word(w, kHNseq);
  if (w->nseq >= (int64_t(1) << 31)) return fail(c, FSLR_ERR_NOMEM, "edge cap replay: more than 2^31 hits");
  {
    Carve cv;                          // the local list was copied out (fslr_cap_copy_local)
    cv.add(&w->seq, w->nseq);
    if (int rc = cv.commit(c, w->ar[4])) return rc;
  }
  if (nti > 0 && w->nseq > 0)
    k_cap_assemble<<<wave_grid(nti), 256, 0, s>>>(counts, w->loff, lists, pad, world, nti, w->ioff, w->seq);
  HIP_TRY(c, hipGetLastError());
  fslr_cap_stats cs;
  std::memset(&cs, 0, sizeof(cs));
  w->runs1 = false;                 // the full-list classification
  if (int rc = cap_core(c, w, &cs)) return rc;
  c->cap_stats = cs;
  if (out) *out = cs;
  return FSLR_OK;
}

extern "C" int fslr_long_pairs(fslr_ctx* c, const fslr_params* p, int64_t* n_edges) {
  return fslr_long_pairs_shard(c, p, 0, 1, n_edges);
}

extern "C" int fslr_long_pairs_shard(fslr_ctx* c, const fslr_params* p, int32_t shard, int32_t n_shards,
                                     int64_t* n_edges) {
  if (!c || !p || !n_edges || n_shards < 1 || shard < 0 || shard >= n_shards) return FSLR_ERR_INVALID;
  *n_edges = 0;
  if (!c->lg_set) return fail(c, FSLR_ERR_STATE, "fslr_set_long_reads first");
  if (!c->index_built || c->filter_active) return fail(c, FSLR_ERR_STATE, "fslr_build_index (every chromosome) first");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  if (int rc = ensure_bwd_ranges(c)) return rc;
  c->last_qcut = p->qlen_cut;
  c->last_ncut = p->nal_cut;
  c->last_full = false;
  c->edges_global = false;
  std::memset(&c->cap_stats, 0, sizeof(c->cap_stats));
  CapWork* w = nullptr;
  if (int rc = cap_work(c, &w)) return rc;
  // the shard's reads' hits (every read: n_shards 1), any thresholds; each pair from its lower read's slot
  w->all_shard = shard;
  w->all_n_shards = n_shards;
  const int rc_local = cap_local(c, 0, w, c->edges, c->fwd, 0, true);
  w->all_shard = 0;
  w->all_n_shards = 1;
  if (rc_local) return rc_local;
  w->nseq = w->nloc;
  if (int rc = cap_slots(c, w)) return rc;
  const int ns = static_cast<int>(w->ns);
  // every pair is in both reads' slots: at most ns / 2 edges (a shard's slots: a pair's other read may
  // lie outside it, at most ns)
  const int64_t need = std::max<int64_t>((n_shards > 1 ? ns : ns / 2) + 1, 1024);
  if (need > c->lg_edge_cap) {
    if (dalloc(c, &c->lg_edges, need)) return FSLR_ERR_NOMEM;
    c->lg_edge_cap = need;
  }
  if (need > c->edge_cap)
    if (int rc = fslr_reserve_edges(c, need)) return rc;
  if (!c->lg_cnt && dalloc(c, &c->lg_cnt, 4)) return FSLR_ERR_NOMEM;
  HIP_TRY(c, hipMemsetAsync(c->lg_cnt, 0, 4 * sizeof(unsigned long long), s));
  HIP_TRY(c, hipMemsetAsync(c->fwd, 0, static_cast<size_t>(c->n) * sizeof(int), s));
  HIP_TRY(c, hipMemsetAsync(c->errw, 0, kErrSticky * sizeof(int), s));   // ZeroDivisionError pairs included
  c->q_thr = p->edge_threshold;
  c->zd_host = true;
  c->zd_lost = false;
  if (ns > 0)
    k_cap_pairs_out<<<grid_for(ns), 256, 0, s>>>(w->ukey, ns, w->T, w->flags, c->lg_edges, c->lg_edge_cap, c->edges,
                                                  c->edge_iu, c->edge_cap, c->lg_cnt, c->fwd, c->errw);
  HIP_TRY(c, hipGetLastError());
  unsigned long long cnt = 0;
  HIP_TRY(c, hipMemcpyAsync(&cnt, c->lg_cnt, sizeof(cnt), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipMemcpyAsync(c->counters + kEdgeCount, &cnt, sizeof(cnt), hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  w->prepared = false;
  if (static_cast<int64_t>(cnt) > c->lg_edge_cap || static_cast<int64_t>(cnt) > c->edge_cap)
    return fail(c, FSLR_ERR_STATE, "long-pair edge list overflowed");
  c->lg_n_edges = static_cast<int64_t>(cnt);
  c->last_engine = FSLR_ENGINE_WALK;
  *n_edges = c->lg_n_edges;
  return FSLR_OK;
}

extern "C" int fslr_cap_replay_pairs(fslr_ctx* c, int32_t thr, const int32_t* a, const int32_t* b, int64_t ne,
                                     uint8_t* who, int32_t* fwd, fslr_cap_stats* out) {
  if (!c || ne < 0 || ((!a || !b || !who) && ne) || ne >= (int64_t(1) << 31)) return FSLR_ERR_INVALID;
  if (!c->reads_set || !c->index_built || c->filter_active)
    return fail(c, FSLR_ERR_STATE, "fslr_build_index (every chromosome) first");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const int64_t n = c->lg_set ? c->lg_n_real : c->n;
  // the edge list (read ranks of the replay's read space, a < b) becomes this context's E*
  std::vector<int2> ab(static_cast<size_t>(ne));
  std::vector<int> deg(static_cast<size_t>(n), 0);
  int max_fwd = 0;
  for (int64_t k = 0; k < ne; ++k) {
    if (a[k] < 0 || a[k] >= b[k] || b[k] >= n) return fail(c, FSLR_ERR_INVALID, "edges must be (a < b) read ranks");
    ab[k] = make_int2(a[k], b[k]);
    max_fwd = std::max(max_fwd, ++deg[a[k]]);
  }
  if (ne > c->edge_cap)
    if (int rc = fslr_reserve_edges(c, ne)) return rc;
  if (!c->counters) return fail(c, FSLR_ERR_STATE, "no query has run");
  if (ne) HIP_TRY(c, hipMemcpyAsync(c->edges, ab.data(), ab.size() * sizeof(int2), hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemsetAsync(c->edge_iu, 0, std::max<int64_t>(ne, 1) * sizeof(unsigned short), s));
  HIP_TRY(c, hipMemcpyAsync(c->fwd, deg.data(), deg.size() * sizeof(int), hipMemcpyHostToDevice, s));
  const unsigned long long ne_u = static_cast<unsigned long long>(ne);
  HIP_TRY(c, hipMemcpyAsync(c->counters + kEdgeCount, &ne_u, sizeof(ne_u), hipMemcpyHostToDevice, s));
  int ew[kErrZdCount] = {};                 // the query's ZeroDivisionError pairs stay listed (cap_local)
  ew[3] = max_fwd;
  HIP_TRY(c, hipMemcpyAsync(c->errw, ew, sizeof(ew), hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  c->edges_global = true;
  std::memset(&c->cap_stats, 0, sizeof(c->cap_stats));
  fslr_cap_stats cs;
  std::memset(&cs, 0, sizeof(cs));
  cs.max_fwd = max_fwd;
  if (max_fwd > thr) {
    if (int rc = ensure_bwd_ranges(c)) return rc;
    CapWork* w = nullptr;
    if (int rc = cap_work(c, &w)) return rc;
    if (int rc = cap_local(c, thr, w, c->edges, c->fwd, ne)) return rc;
    w->nseq = w->nloc;
    w->runs1 = false;                 // the full-list classification
    if (int rc = cap_core(c, w, &cs)) return rc;
    if (ne) HIP_TRY(c, hipMemcpyAsync(who, w->who, static_cast<size_t>(ne), hipMemcpyDeviceToHost, s));
    if (fwd) HIP_TRY(c, hipMemcpyAsync(fwd, c->fwd, static_cast<size_t>(n) * sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
  } else {
    if (ne) std::memset(who, 0, static_cast<size_t>(ne));
    if (fwd) std::copy(deg.begin(), deg.end(), fwd);
  }
  c->cap_stats = cs;
  if (out) *out = cs;
  return FSLR_OK;
}

// ---- the sharded replay (multi-GPU): host side ---------------------------------------------------
namespace {
int cap_install(fslr_ctx* c, const int32_t* pairs, int64_t n_rows, int32_t world, int32_t rank, bool restricted) {
  if (!c || (!pairs && n_rows) || n_rows < 0 || world < 1 || world > kMaxDest || rank < 0 || rank >= world ||
      n_rows % world)
    return FSLR_ERR_INVALID;
  if (n_rows >= (int64_t(1) << 29)) return fail(c, FSLR_ERR_INVALID, "sharded edge cap: at most 2^29 gathered rows");
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  if (c->lg_set) return fail(c, FSLR_ERR_STATE, "the sharded edge cap takes reads of at most FSLR_MAX_L intervals");
  if (!c->counters) return fail(c, FSLR_ERR_STATE, "no query has run");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  CapWork* w = nullptr;
  if (int rc = cap_work(c, &w)) return rc;
  {
    Carve cv;
    cv.add(&w->gfwd, c->n);
    cv.add(&w->gstart, c->n);
    cv.add(&w->gend, c->n);
    cv.add(&w->gwho, n_rows);
    cv.add(&w->gflag, 4);
    cv.add(&w->gtot, 2);
    if (int rc = cv.commit(c, w->ar[5])) return rc;
  }
  w->grows = reinterpret_cast<const int2*>(pairs);
  const size_t nb = static_cast<size_t>(std::max<int64_t>(c->n, 1)) * sizeof(int);
  HIP_TRY(c, hipMemsetAsync(w->gstart, 0, nb, s));
  HIP_TRY(c, hipMemsetAsync(w->gend, 0, nb, s));
  HIP_TRY(c, hipMemsetAsync(w->gflag, 0, 4 * sizeof(int), s));
  HIP_TRY(c, hipMemsetAsync(w->gtot, 0, 2 * sizeof(unsigned long long), s));
  // each read's run of forward rows (every block sorted by a: fslr_sort_edges before the gather)
  const int64_t m = n_rows / world;
  if (n_rows) k_cap_runs<<<grid_for(n_rows), 256, 0, s>>>(w->grows, n_rows, m, w->gstart, w->gend, w->gflag, w->gtot);
  k_cap_runfwd<<<grid_for(c->n), 256, 0, s>>>(w->gstart, w->gend, static_cast<int>(c->n), w->gfwd, w->gtot + 1);
  HIP_TRY(c, hipGetLastError());
  unsigned long long tot[2] = {0, 0};
  int flag = 0;
  HIP_TRY(c, hipMemcpyAsync(tot, w->gtot, sizeof(tot), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipMemcpyAsync(&flag, w->gflag, sizeof(flag), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  w->g_sorted = !flag && tot[0] == tot[1];
  if (cap_debug()) std::fprintf(stderr, "fslr: cap install %lld rows, sorted %d\n", static_cast<long long>(n_rows), w->g_sorted);
  if (!w->g_sorted) {                 // unsorted blocks: forward degrees by atomics, the closure by adjacency
    HIP_TRY(c, hipMemsetAsync(w->gfwd, 0, nb, s));
    if (n_rows) k_cap_gfwd<<<grid_for(n_rows), 256, 0, s>>>(w->grows, n_rows, w->gfwd);
    HIP_TRY(c, hipGetLastError());
  }
  w->g_rows = n_rows;
  w->g_m = n_rows / world;
  w->g_world = world;
  w->g_rank = rank;
  w->prepared = false;
  w->planned = 0;
  w->replayed = false;
  w->g_restricted = restricted;
  c->cap_gmode = true;
  c->edges_global = false;
  std::memset(&c->cap_stats, 0, sizeof(c->cap_stats));
  return FSLR_OK;
}
}  // namespace

extern "C" int fslr_cap_install_pairs(fslr_ctx* c, const int32_t* pairs, int64_t n_rows, int32_t world, int32_t rank) {
  if (c && c->capw) c->capw->r_ready = c->capw->r_counted = false;
  return cap_install(c, pairs, n_rows, world, rank, false);
}

extern "C" int fslr_cap_bwd_counts(fslr_ctx* c, int32_t thr, void* out, int32_t elem_bytes) {
  if (!c || !out || (elem_bytes != 1 && elem_bytes != 4) || thr < 1 || (elem_bytes == 1 && thr > 255))
    return FSLR_ERR_INVALID;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  if (c->lg_set) return fail(c, FSLR_ERR_STATE, "the sharded edge cap takes reads of at most FSLR_MAX_L intervals");
  if (!c->counters) return fail(c, FSLR_ERR_STATE, "no query has run");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  long long pk[4] = {0, 0, 0, 0};
  if (int rc = peek_counts(c, pk)) return rc;
  const int64_t ne = std::min<int64_t>(pk[0], c->edge_cap), n = c->n;
  if (ne >= (int64_t(1) << 31)) return fail(c, FSLR_ERR_INVALID, "too many edges for the restricted gather");
  CapWork* w = nullptr;
  if (int rc = cap_work(c, &w)) return rc;
  {
    Carve cv;
    cv.add(&w->rcnt, n);
    cv.add(&w->rflag, ne);
    cv.add(&w->rkoff, ne);
    cv.add(&w->rmap, ne);
    cv.add(&w->rrows, ne);
    if (int rc = cv.commit(c, w->ar[10])) return rc;
  }
  int* bcnt = elem_bytes == 4 ? static_cast<int*>(out) : w->rcnt;
  HIP_TRY(c, hipMemsetAsync(bcnt, 0, static_cast<size_t>(std::max<int64_t>(n, 1)) * sizeof(int), s));
  if (ne > 0) k_cap_bwdc<<<grid_for(ne), 256, 0, s>>>(c->edges, ne, bcnt);
  if (elem_bytes == 1 && n > 0)
    k_cap_clip8<<<grid_for(n), 256, 0, s>>>(w->rcnt, static_cast<int>(n), thr, static_cast<unsigned char*>(out));
  HIP_TRY(c, hipGetLastError());
  w->r_ne = ne;
  w->r_thr = thr;
  w->r_counted = true;
  w->r_ready = false;
  return FSLR_OK;
}

extern "C" int fslr_cap_restrict(fslr_ctx* c, const void* bwd, int32_t elem_bytes, int64_t* n_rows) {
  if (!c || !bwd || !n_rows || (elem_bytes != 1 && elem_bytes != 4)) return FSLR_ERR_INVALID;
  *n_rows = 0;
  CapWork* w = c->capw;
  if (!w || !w->r_counted) return fail(c, FSLR_ERR_STATE, "fslr_cap_bwd_counts first");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const int64_t ne = w->r_ne;
  int64_t kept = 0;
  if (ne > 0) {
    k_cap_rflags<<<grid_for(ne), 256, 0, s>>>(c->edges, ne, c->fwd, bwd, elem_bytes, w->r_thr, w->rflag);
    size_t tb = 0;
    HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, w->rflag, w->rkoff, static_cast<int>(ne), s));
    if (int rc = ensure_temp(c, w, tb)) return rc;
    tb = w->temp_bytes;
    HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(w->temp, tb, w->rflag, w->rkoff, static_cast<int>(ne), s));
    k_cap_rcompact<<<grid_for(ne), 256, 0, s>>>(c->edges, ne, w->rflag, w->rkoff, w->rrows, w->rmap);
    HIP_TRY(c, hipGetLastError());
    int last[2] = {0, 0};
    HIP_TRY(c, hipMemcpyAsync(last, w->rkoff + ne - 1, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(last + 1, w->rflag + ne - 1, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    kept = static_cast<int64_t>(last[0]) + last[1];
  }
  if (kept > 1) {
    // sorted by lower read (each read's rows one run of the gathered blocks); only these rows need it
    unsigned *k1 = nullptr, *k2 = nullptr;
    int *v1 = nullptr, *v2 = nullptr, *ormap = nullptr;
    int2* orows = nullptr;
    {
      Carve cv;
      cv.add(&k1, kept);
      cv.add(&k2, kept);
      cv.add(&v1, kept);
      cv.add(&v2, kept);
      cv.add(&orows, kept);
      cv.add(&ormap, kept);
      if (int rc = cv.commit(c, w->ar[9])) return rc;
    }
    const int nk = static_cast<int>(kept);
    k_edge_keys<<<grid_for(kept), 256, 0, s>>>(w->rrows, kept, k1, v1);
    size_t tb = 0;
    HIP_TRY(c, hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k1, k2, v1, v2, nk, 0, bits_for(c->n), s));
    if (int rc = ensure_temp(c, w, tb)) return rc;
    tb = w->temp_bytes;
    HIP_TRY(c, hipcub::DeviceRadixSort::SortPairs(w->temp, tb, k1, k2, v1, v2, nk, 0, bits_for(c->n), s));
    k_cap_rpermute<<<grid_for(kept), 256, 0, s>>>(w->rrows, w->rmap, v2, kept, orows, ormap);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipMemcpyAsync(w->rrows, orows, static_cast<size_t>(kept) * sizeof(int2), hipMemcpyDeviceToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(w->rmap, ormap, static_cast<size_t>(kept) * sizeof(int), hipMemcpyDeviceToDevice, s));
  }
  w->r_n = kept;
  w->r_ready = true;
  *n_rows = kept;
  return FSLR_OK;
}

extern "C" int fslr_cap_copy_restricted(fslr_ctx* c, int32_t* dst, int64_t n_pad) {
  if (!c || n_pad < 0 || (!dst && n_pad)) return FSLR_ERR_INVALID;
  CapWork* w = c->capw;
  if (!w || !w->r_ready) return fail(c, FSLR_ERR_STATE, "fslr_cap_restrict first");
  if (n_pad < w->r_n) return fail(c, FSLR_ERR_INVALID, "n_pad below this rank's restricted row count");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  if (w->r_n)
    HIP_TRY(c, hipMemcpyAsync(dst, w->rrows, static_cast<size_t>(w->r_n) * sizeof(int2), hipMemcpyDeviceToDevice, s));
  if (n_pad > w->r_n) {
    k_fill<<<grid_for(2 * (n_pad - w->r_n)), 256, 0, s>>>(dst + 2 * w->r_n, static_cast<int>(2 * (n_pad - w->r_n)), -1);
    HIP_TRY(c, hipGetLastError());
  }
  return FSLR_OK;
}

extern "C" int fslr_cap_install_restricted(fslr_ctx* c, const int32_t* pairs, int64_t n_rows, int32_t world,
                                           int32_t rank) {
  if (!c || world < 1 || n_rows < 0 || n_rows % world) return FSLR_ERR_INVALID;
  CapWork* w = c->capw;
  if (!w || !w->r_ready) return fail(c, FSLR_ERR_STATE, "fslr_cap_restrict first");
  if (n_rows / world < w->r_n) return fail(c, FSLR_ERR_INVALID, "the blocks are smaller than this rank's restricted rows");
  return cap_install(c, pairs, n_rows, world, rank, true);
}

extern "C" int fslr_cap_sizes(fslr_ctx* c, int64_t* n_t, int64_t* n_ti, int64_t* n_hits) {
  if (!c || !n_t || !n_ti || !n_hits) return FSLR_ERR_INVALID;
  if (!c->capw || !c->capw->prepared) return fail(c, FSLR_ERR_STATE, "fslr_cap_local first");
  *n_t = c->capw->nt;
  *n_ti = c->capw->nti;
  *n_hits = c->capw->nloc;
  return FSLR_OK;
}

extern "C" int fslr_cap_dep_local(fslr_ctx* c, int32_t* out) {
  if (!c) return FSLR_ERR_INVALID;
  CapWork* w = c->capw;
  if (!c->cap_gmode || !w || !w->prepared) return fail(c, FSLR_ERR_STATE, "fslr_cap_install_pairs, fslr_cap_local first");
  const int nt = static_cast<int>(w->nt), nti = static_cast<int>(w->nti);
  if (!out && nt) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  if (nt == 0) return FSLR_OK;
  {
    Carve cv;
    cv.add(&w->tdeps, w->nloc);
    if (int rc = cv.commit(c, w->ar[7])) return rc;
  }
  int* par = out;
  int* thits = out + nt;
  HIP_TRY(c, hipMemsetAsync(thits, 0, static_cast<size_t>(nt) * sizeof(int), s));
  HIP_TRY(c, launch_uf_init(par, nt, s));
  if (w->nloc > 0) {
    k_cap_tdeps<<<wave_grid(nti), 256, 0, s>>>(w->seq, w->ioff, w->tread, w->t_of, nti, w->tdeps, thits);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, launch_uf_pair_list(par, w->tdeps, w->nloc, s));
  }
  HIP_TRY(c, launch_uf_finalize(par, nt, s));
  return FSLR_OK;
}

extern "C" int fslr_cap_shard_plan(fslr_ctx* c, const int32_t* gathered, int32_t world, int32_t rank, int64_t* sizes) {
  if (!c || !sizes) return FSLR_ERR_INVALID;
  CapWork* w = c->capw;
  if (!c->cap_gmode || !w || !w->prepared) return fail(c, FSLR_ERR_STATE, "fslr_cap_install_pairs, fslr_cap_local first");
  if (world != w->g_world || rank != w->g_rank) return fail(c, FSLR_ERR_INVALID, "world / rank differ from fslr_cap_install_pairs");
  const int nt = static_cast<int>(w->nt), nti = static_cast<int>(w->nti);
  if (!gathered && nt) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  {
    Carve cv;
    cv.add(&w->comp, nt);
    cv.add(&w->tcost, nt);
    cv.add(&w->tdest, nt);
    cv.add(&w->tikey, nti);
    cv.add(&w->tikey2, nti);
    cv.add(&w->tival, nti);
    cv.add(&w->tsorted, nti);
    cv.add(&w->scnt, nti + 1);
    cv.add(&w->shoff, nti + 1);
    cv.add(&w->totals, 2 * kMaxDest);
    cv.add(&w->ccost, nt);
    cv.add(&w->roots, nt);
    cv.add(&w->dmap, nt);
    if (int rc = cv.commit(c, w->ar[6])) return rc;
  }
  CapTimer tm(s);
  // the components of the T-T hit graph: the union of the ranks' local forests; each component's cost
  // and the list of roots, on the device
  unsigned long long* rkeys = reinterpret_cast<unsigned long long*>(w->roots);   // then sorted into ccost
  if (nt > 0) {
    HIP_TRY(c, launch_uf_init(w->comp, nt, s));
    HIP_TRY(c, launch_uf_strided(w->comp, gathered, world, nt, 2ll * nt, s));
    HIP_TRY(c, launch_uf_finalize(w->comp, nt, s));
    k_cap_tcost<<<grid_for(nt), 256, 0, s>>>(gathered, world, nt, w->tcost);
    HIP_TRY(c, hipMemsetAsync(w->ccost, 0, static_cast<size_t>(nt) * sizeof(unsigned long long), s));
    k_cap_ccost<<<grid_for(nt), 256, 0, s>>>(w->comp, w->tcost, nt, w->ccost);
    const int kbits = bits_for(nt);
    k_cap_rootkeys<<<grid_for(nt), 256, 0, s>>>(w->comp, w->ccost, nt, kbits, rkeys);
    // largest first (ties: the smaller root), the other slots last; then the ranks, on the device
    size_t tb = 0;
    HIP_TRY(c, hipcub::DeviceRadixSort::SortKeys(nullptr, tb, rkeys, w->ccost, nt, 0, 31 + kbits, s));
    if (int rc = ensure_temp(c, w, tb)) return rc;
    tb = w->temp_bytes;
    HIP_TRY(c, hipcub::DeviceRadixSort::SortKeys(w->temp, tb, rkeys, w->ccost, nt, 0, 31 + kbits, s));
    k_cap_assign_head<<<1, kWave, 0, s>>>(w->ccost, nt, world, kbits, w->dmap);
    if (nt > kCapHead)
      k_cap_assign_tail<<<grid_for(nt - kCapHead), 256, 0, s>>>(w->ccost, nt, world, kbits, w->dmap);
    k_cap_tdest<<<grid_for(nt), 256, 0, s>>>(w->comp, w->dmap, nt, w->tdest);
    HIP_TRY(c, hipGetLastError());
  }
  tm.lap("plan: unions + assign");
  // the T-intervals grouped by destination (stable: T order inside a group), their counts and hits
  HIP_TRY(c, hipMemsetAsync(w->totals, 0, 2 * kMaxDest * sizeof(long long), s));
  HIP_TRY(c, hipMemsetAsync(w->scnt + nti, 0, sizeof(int), s));
  if (nti > 0) {
    k_cap_tikey<<<grid_for(nti), 256, 0, s>>>(w->tread, w->tdest, nti, w->tikey, w->tival);
    size_t tb = 0;
    const int kb = bits_for(world);
    HIP_TRY(c, hipcub::DeviceRadixSort::SortPairs(nullptr, tb, w->tikey, w->tikey2, w->tival, w->tsorted, nti, 0, kb, s));
    if (int rc = ensure_temp(c, w, tb)) return rc;
    tb = w->temp_bytes;
    HIP_TRY(c, hipcub::DeviceRadixSort::SortPairs(w->temp, tb, w->tikey, w->tikey2, w->tival, w->tsorted, nti, 0, kb, s));
    k_cap_sendcnt<<<std::min(grid_for(nti), 1024), 256, 0, s>>>(w->tsorted, w->tikey2, w->icnt, nti, w->scnt, w->totals);
    HIP_TRY(c, hipGetLastError());
  }
  size_t tb = 0;
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, w->scnt, w->shoff, nti + 1, s));
  if (int rc = ensure_temp(c, w, tb)) return rc;
  tb = w->temp_bytes;
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(w->temp, tb, w->scnt, w->shoff, nti + 1, s));
  long long tot[2 * kMaxDest];
  HIP_TRY(c, hipMemcpyAsync(tot, w->totals, sizeof(tot), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  int64_t off = 0, hits = 0;
  for (int d = 0; d < world; ++d) {
    sizes[d] = tot[d];
    sizes[world + d] = tot[kMaxDest + d];
    if (d < rank) off += tot[d];
    hits += tot[kMaxDest + d];
  }
  tm.lap("plan: group");
  if (hits != w->nloc) return fail(c, FSLR_ERR_STATE, "sharded edge cap: hit totals differ from the local lists");
  w->nmine = tot[rank];
  w->mine_off = off;
  w->planned = 1;
  return FSLR_OK;
}

extern "C" int fslr_cap_shard_pack(fslr_ctx* c, int32_t* counts, int32_t* hits) {
  if (!c) return FSLR_ERR_INVALID;
  CapWork* w = c->capw;
  if (!c->cap_gmode || !w || !w->planned) return fail(c, FSLR_ERR_STATE, "fslr_cap_shard_plan first");
  if ((!counts && w->nti) || (!hits && w->nloc)) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const int nti = static_cast<int>(w->nti);
  if (nti) HIP_TRY(c, hipMemcpyAsync(counts, w->scnt, static_cast<size_t>(nti) * sizeof(int), hipMemcpyDeviceToDevice, s));
  if (nti && w->nloc) {
    k_cap_pack<<<wave_grid(nti), 256, 0, s>>>(w->tsorted, w->scnt, w->shoff, w->seq, w->ioff, nti, hits);
    HIP_TRY(c, hipGetLastError());
  }
  return FSLR_OK;
}

extern "C" int fslr_cap_replay_shard(fslr_ctx* c, const int32_t* rcounts, const int32_t* rhits, int64_t* n_changes,
                                     fslr_cap_stats* part) {
  if (!c || !n_changes) return FSLR_ERR_INVALID;
  *n_changes = 0;
  CapWork* w = c->capw;
  if (!c->cap_gmode || !w || !w->planned) return fail(c, FSLR_ERR_STATE, "fslr_cap_shard_plan first");
  const int world = w->g_world, nti = static_cast<int>(w->nti), nt = static_cast<int>(w->nt);
  const int nmine = static_cast<int>(w->nmine);
  const int64_t nrc = static_cast<int64_t>(world) * nmine;
  if (!rcounts && nrc) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  {
    Carve cv;
    cv.add(&w->roff, nrc + 1);
    cv.add(&w->chgl, w->g_rows);
    cv.add(&w->nchg, 4);
    if (int rc = cv.commit(c, w->ar[8])) return rc;
  }
  HIP_TRY(c, hipMemsetAsync(w->err, 0, 4 * sizeof(int), s));
  HIP_TRY(c, hipMemsetAsync(w->stats, 0, kStWords * sizeof(long long), s));
  HIP_TRY(c, hipMemsetAsync(w->nchg, 0, 4 * sizeof(unsigned), s));
  // this rank's T-intervals get the received counts, every other one none; the sequence offsets
  HIP_TRY(c, hipMemsetAsync(w->icnt, 0, static_cast<size_t>(nti + 1) * sizeof(int), s));
  const int* mine = w->tsorted + w->mine_off;
  if (nmine > 0) {
    k_cap_recv_sum<<<grid_for(nmine), 256, 0, s>>>(rcounts, world, nmine, mine, w->icnt);
    HIP_TRY(c, hipGetLastError());
  }
  size_t b1 = 0, b2 = 0;
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, b1, w->icnt, w->ioff, nti + 1, s));
  if (nrc > 0) HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, b2, rcounts, w->roff, static_cast<int>(nrc), s));
  if (int rc = ensure_temp(c, w, std::max(b1, b2))) return rc;
  size_t tb = w->temp_bytes;
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(w->temp, tb, w->icnt, w->ioff, nti + 1, s));
  if (nrc > 0) {
    tb = w->temp_bytes;
    HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(w->temp, tb, rcounts, w->roff, static_cast<int>(nrc), s));
  }
  k_cap_total<<<1, 64, 0, s>>>(w->ioff, nti, w->host_dev, kHNseq);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipStreamSynchronize(s));
  w->nseq = host_word(w, kHNseq);
  if (w->nseq >= (int64_t(1) << 31)) return fail(c, FSLR_ERR_NOMEM, "edge cap replay: more than 2^31 hits");
  if (w->nseq && !rhits) return FSLR_ERR_INVALID;
  {
    Carve cv;
    cv.add(&w->seq, w->nseq);
    if (int rc = cv.commit(c, w->ar[4])) return rc;
  }
  if (nmine > 0 && w->nseq > 0) {
    k_cap_recv_assemble<<<wave_grid(nmine), 256, 0, s>>>(rcounts, w->roff, rhits, world, nmine, mine, w->ioff, w->seq);
    HIP_TRY(c, hipGetLastError());
  }
  // slots, predicates and loops of this rank's components (every other T read has no hit: no break)
  if (int rc = cap_loops(c, w)) return rc;
  CapTimer tm(s);
  const int ns = static_cast<int>(w->ns);
  if (w->g_rows > 0) {
    k_cap_classify_shard<<<grid_for(w->g_rows), 256, 0, s>>>(w->grows, w->g_rows, w->t_of, w->tdest, w->comp, w->g_rank,
                                                             w->pbrk, w->ukey, w->tsb, w->fpos, w->vis2, w->chgl, w->nchg,
                                                             w->err);
    HIP_TRY(c, hipGetLastError());
  }
  if (nt > 0) {
    k_cap_count_capped<<<grid_for(nt), 256, 0, s>>>(w->pbrk, nt, w->stats);
    HIP_TRY(c, hipGetLastError());
  }
  tm.lap("classify");
  unsigned nch = 0;
  int err = 0;
  long long capped = 0;
  HIP_TRY(c, hipMemcpyAsync(&nch, w->nchg, sizeof(nch), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipMemcpyAsync(&err, w->err, sizeof(err), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipMemcpyAsync(&capped, w->stats + kStCapped, sizeof(capped), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  if (err & kCapErrZd) return fail(c, FSLR_ERR_ZERO_DIVISION, "division by zero");
  if (err & kCapErrState) return fail(c, FSLR_ERR_STATE, "sharded edge cap: inconsistent loop replay");
  w->n_chg = nch;
  w->replayed = true;
  *n_changes = nch;
  if (part) {
    std::memset(part, 0, sizeof(*part));
    part->applied = 1;
    part->candidates = w->nt;
    part->capped = capped;
    part->hits = w->nseq;
    part->pairs = ns;
  }
  return FSLR_OK;
}

extern "C" int fslr_cap_copy_changes(fslr_ctx* c, int32_t* dst, int64_t n_pad) {
  if (!c || n_pad < 0 || (!dst && n_pad)) return FSLR_ERR_INVALID;
  CapWork* w = c->capw;
  if (!c->cap_gmode || !w || !w->replayed) return fail(c, FSLR_ERR_STATE, "fslr_cap_replay_shard first");
  if (n_pad < w->n_chg) return fail(c, FSLR_ERR_INVALID, "n_pad below this rank's change count");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  if (w->n_chg) HIP_TRY(c, hipMemcpyAsync(dst, w->chgl, static_cast<size_t>(w->n_chg) * sizeof(int), hipMemcpyDeviceToDevice, s));
  if (n_pad > w->n_chg) {
    k_fill<<<grid_for(n_pad - w->n_chg), 256, 0, s>>>(dst + w->n_chg, static_cast<int>(n_pad - w->n_chg), -1);
    HIP_TRY(c, hipGetLastError());
  }
  return FSLR_OK;
}

extern "C" int fslr_cap_apply_changes(fslr_ctx* c, const int32_t* changes, int64_t n, fslr_cap_stats* out) {
  if (!c || n < 0 || (!changes && n)) return FSLR_ERR_INVALID;
  CapWork* w = c->capw;
  if (!c->cap_gmode || !w || !w->replayed) return fail(c, FSLR_ERR_STATE, "fslr_cap_replay_shard first");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const int64_t nr = c->n, rows = w->g_rows, m = w->g_m;
  const int nt = static_cast<int>(w->nt);
  const int64_t mloc = std::min(m, c->edge_cap);
  CapTimer tm(s);
  HIP_TRY(c, hipMemsetAsync(w->err, 0, 4 * sizeof(int), s));
  HIP_TRY(c, hipMemsetAsync(w->stats, 0, kStWords * sizeof(long long), s));
  if (rows) HIP_TRY(c, hipMemsetAsync(w->gwho, 0, static_cast<size_t>(rows), s));
  HIP_TRY(c, hipMemcpyAsync(w->formed, w->gfwd, static_cast<size_t>(nr) * sizeof(int), hipMemcpyDeviceToDevice, s));
  if (n > 0) {
    k_cap_apply<<<grid_for(n), 256, 0, s>>>(changes, n, w->grows, w->gwho, w->formed, w->stats);
    HIP_TRY(c, hipGetLastError());
  }
  tm.lap("apply: changes");
  // this rank's own edges (block g_rank of the rows): kept ones compacted and re-oriented, their formers;
  // with the restricted gather its rows of S are applied in place through their local edge index and
  // the dropped rows' holes filled from the tail
  const bool rs = w->g_restricted;
  unsigned* rcnt3 = reinterpret_cast<unsigned*>(w->chg);          // [0] dropped, [1] holes, [2] survivors
  if (rs) {
    // the maximum then covers S and this rank's reads outside S (the caller's MAX over ranks)
    if (nr) k_cap_addfwd<<<grid_for(nr), 256, 0, s>>>(w->formed, w->gfwd, c->fwd, static_cast<int>(nr));
    HIP_TRY(c, hipMemsetAsync(rcnt3, 0, 4 * sizeof(unsigned), s));
    if (w->r_n)
      k_cap_rapply<<<grid_for(w->r_n), 256, 0, s>>>(w->gwho + w->g_rank * m, w->rmap, w->r_n, c->edges, c->fwd,
                                                    w->rflag, rcnt3);
    k_cap_holes<<<256, 256, 0, s>>>(w->rflag, rcnt3, w->r_ne, w->rkoff, rcnt3 + 1);
    k_cap_survivors<<<256, 256, 0, s>>>(c->edges, rcnt3, w->r_ne, w->rmap, rcnt3 + 2);
    k_cap_fill<<<256, 256, 0, s>>>(c->edges, c->edge_iu, w->rkoff, w->rmap, rcnt3 + 1, w->err);
    HIP_TRY(c, hipGetLastError());
  } else {
    const int2* blk = w->grows + w->g_rank * m;
    const unsigned char* wblk = w->gwho + w->g_rank * m;
    HIP_TRY(c, hipMemsetAsync(c->fwd, 0, static_cast<size_t>(nr) * sizeof(int), s));
    if (mloc > 0) {
      k_cap_local_flags<<<grid_for(mloc), 256, 0, s>>>(blk, wblk, mloc, w->kflag);
      size_t tb = 0;
      HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, w->kflag, w->koff, static_cast<int>(mloc), s));
      if (int rc = ensure_temp(c, w, tb)) return rc;
      tb = w->temp_bytes;
      HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(w->temp, tb, w->kflag, w->koff, static_cast<int>(mloc), s));
      k_cap_local_compact<<<grid_for(mloc), 256, 0, s>>>(c->edges, c->edge_iu, mloc, w->kflag, w->koff, wblk,
                                                         w->oedges, w->oiu, c->fwd);
      HIP_TRY(c, hipGetLastError());
      HIP_TRY(c, hipMemcpyAsync(c->edges, w->oedges, static_cast<size_t>(mloc) * sizeof(int2), hipMemcpyDeviceToDevice,
                                s));
      HIP_TRY(c, hipMemcpyAsync(c->edge_iu, w->oiu, static_cast<size_t>(mloc) * sizeof(unsigned short),
                                hipMemcpyDeviceToDevice, s));
    }
  }
  tm.lap("apply: local");
  k_cap_check_shard<<<grid_for(std::max<int64_t>(nr, nt)), 256, 0, s>>>(w->T, nt, w->tdest, w->g_rank, w->own, w->formed,
                                                                       static_cast<int>(nr), w->stats, w->err);
  HIP_TRY(c, hipGetLastError());
  if (rs)
    k_cap_commit_runs<<<1, 64, 0, s>>>(rcnt3, w->r_ne, c->counters, c->errw, w->stats, w->err, w->host_dev, true);
  else
    k_cap_commit_shard<<<1, 64, 0, s>>>(w->koff, w->kflag, mloc, c->counters, c->errw, w->stats, w->err, w->host_dev);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipStreamSynchronize(s));
  const long long err = host_word(w, kHErr);
  w->prepared = false;
  w->planned = 0;
  w->replayed = false;
  w->g_restricted = w->r_ready = w->r_counted = false;
  c->cap_gmode = false;
  if (err & kCapErrState) return fail(c, FSLR_ERR_STATE, "sharded edge cap: a replayed loop's edge count differs");
  fslr_cap_stats cs;
  std::memset(&cs, 0, sizeof(cs));
  cs.applied = 1;
  cs.max_fwd = static_cast<int32_t>(host_word(w, kHStat + kStMaxFwd));
  cs.candidates = w->nt;
  cs.dropped = host_word(w, kHStat + kStDropped);
  cs.backward = host_word(w, kHStat + kStBackward);
  c->cap_stats = cs;
  if (out) *out = cs;
  return FSLR_OK;
}

extern "C" int fslr_sort_edges(fslr_ctx* c) {
  if (!c) return FSLR_ERR_INVALID;
  c->hooked = false;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  HIP_TRY(c, hipSetDevice(c->device));
  if (!c->counters || !c->edge_cap) return FSLR_OK;
  hipStream_t s = c->stream;
  long long pk[4] = {0, 0, 0, 0};
  if (int rc = peek_counts(c, pk)) return rc;
  const int64_t ne = std::min<int64_t>(pk[0], c->edge_cap);
  if (ne < 2) return FSLR_OK;
  if (ne >= (int64_t(1) << 31)) return fail(c, FSLR_ERR_INVALID, "too many edges to sort");
  CapWork* w = nullptr;
  if (int rc = cap_work(c, &w)) return rc;
  unsigned *k1 = nullptr, *k2 = nullptr;
  int *v1 = nullptr, *v2 = nullptr;
  int2* oe = nullptr;
  unsigned short* oiu = nullptr;
  {
    Carve cv;
    cv.add(&k1, ne);
    cv.add(&k2, ne);
    cv.add(&v1, ne);
    cv.add(&v2, ne);
    cv.add(&oe, ne);
    cv.add(&oiu, ne);
    if (int rc = cv.commit(c, w->ar[9])) return rc;
  }
  const int n = static_cast<int>(ne);
  k_edge_keys<<<grid_for(ne), 256, 0, s>>>(c->edges, ne, k1, v1);
  size_t tb = 0;
  HIP_TRY(c, hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k1, k2, v1, v2, n, 0, bits_for(c->n), s));
  if (int rc = ensure_temp(c, w, tb)) return rc;
  tb = w->temp_bytes;
  HIP_TRY(c, hipcub::DeviceRadixSort::SortPairs(w->temp, tb, k1, k2, v1, v2, n, 0, bits_for(c->n), s));
  k_edge_permute<<<grid_for(ne), 256, 0, s>>>(c->edges, c->edge_iu, v2, ne, oe, oiu);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipMemcpyAsync(c->edges, oe, static_cast<size_t>(ne) * sizeof(int2), hipMemcpyDeviceToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(c->edge_iu, oiu, static_cast<size_t>(ne) * sizeof(unsigned short), hipMemcpyDeviceToDevice, s));
  return FSLR_OK;
}
