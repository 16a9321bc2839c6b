// components.hip — connected components (replaces get_subgraphs, cluster.py:230-234, i.e.
// networkx.connected_components over the graph built at cluster.py:221).
//
// Lock-free union-find: roots are hooked larger-under-smaller with a CAS, so the root of a
// component is its minimum read rank — the order networkx yields components in (first inserted
// node = minimum rank when every edge is added in its lower-rank read's loop).
// Every parent pointer goes to an ancestor with a smaller rank, and a node's ancestors stay its
// ancestors, so any value a node's parent ever held is still a valid step towards its root.  The
// find walk therefore uses ordinary (cached, possibly stale) loads: a stale value is just an
// older ancestor.  Only the hook is a coherent agent-scope CAS; when it fails, its returned value
// (the fresh parent of the would-be root) continues the walk, so every retry moves strictly up
// the tree and the loop ends.  Kernel boundaries make the final forest visible to finalize.
#include <algorithm>

#include "kernels.hpp"

namespace fslr {
namespace {

// plain (cached) single-copy-atomic accesses: wavefront scope adds no coherence bits
__device__ __forceinline__ int ld_rlx(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
__device__ __forceinline__ void st_rlx(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

__device__ int uf_find(int* p, int x) {
  while (true) {
    const int px = ld_rlx(p + x);
    if (px == x) return x;
    const int ppx = ld_rlx(p + px);
    if (ppx != px) st_rlx(p + x, ppx);   // path halving; ppx is still an ancestor of x
    x = ppx;
  }
}

__device__ void uf_union(int* p, int a, int b) {
  while (true) {
    a = uf_find(p, a);
    b = uf_find(p, b);
    if (a == b) return;
    if (a > b) { const int t = a; a = b; b = t; }
    const int old = atomicCAS(p + b, b, a);   // hook the larger root under the smaller (coherent)
    if (old == b) return;
    b = old;                                  // fresh parent of b: continue strictly upwards
  }
}

__global__ void k_uf_init(int* p, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = i;
}

__global__ void k_uf_edges(int* p, const int2* __restrict__ edges, const unsigned long long* __restrict__ count,
                           long long cap, int* err) {
  const long long cnt = static_cast<long long>(*count);
  if (cnt > cap && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err + kErrOverflow, 2);
  const long long ne = min(cnt, cap);
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < ne;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int2 e = edges[k];
    uf_union(p, e.x, e.y);
  }
}

// from the identity: every read points to its smallest neighbour below it (one atomicMin per edge, no
// finds; pointers only go down, so it is a forest of partial unions of the same components); the unions
// over every edge then find short paths: 0.049 vs 0.070 ms for the components at cfg3 (profiles/r05/r5u/)
__global__ void k_uf_hook_min(int* p, const int2* __restrict__ edges, const unsigned long long* __restrict__ count,
                              long long cap) {
  const long long ne = min(static_cast<long long>(*count), cap);
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < ne;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int2 e = edges[k];
    const int lo = min(e.x, e.y), hi = max(e.x, e.y);
    if (lo != hi) atomicMin(p + hi, lo);
  }
}

__global__ void k_uf_pairs(int* p, const int* __restrict__ src, const int* __restrict__ dst, long long n,
                           int period) {
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < n;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int s = src ? src[k] : static_cast<int>(k % period);
    uf_union(p, s, dst[k]);
  }
}

// the same pre-hook over a pair list ((a, b), a < 0 or b < 0 = padding)
__global__ void k_uf_hook_min_pairs(int* p, const int2* __restrict__ pairs, long long n) {
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < n;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int2 e = pairs[k];
    if (e.x < 0 || e.y < 0) continue;
    const int lo = min(e.x, e.y), hi = max(e.x, e.y);
    if (lo != hi) atomicMin(p + hi, lo);
  }
}

// a gathered edge list (the multi-GPU merge): (a, b) pairs, a < 0 = padding
__global__ void k_uf_pair_list(int* p, const int2* __restrict__ pairs, long long n) {
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < n;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int2 e = pairs[k];
    if (e.x >= 0) uf_union(p, e.x, e.y);
  }
}

// the same pre-hook over W label blocks (k_uf_strided's pairs (k, vals[w * stride + k]))
__global__ void k_uf_hook_min_strided(int* p, const int* __restrict__ vals, long long blocks, int n, long long stride) {
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < blocks * n;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long w = k / n;
    const int i = static_cast<int>(k - w * n);
    const int v = vals[w * stride + i];
    const int lo = min(i, v), hi = max(i, v);
    if (lo != hi) atomicMin(p + hi, lo);
  }
}

// W label blocks of n values at vals + w * stride (the multi-GPU cap's gathered forests): union of
// k and vals[w * stride + k] for every block w
__global__ void k_uf_strided(int* p, const int* __restrict__ vals, long long blocks, int n, long long stride) {
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < blocks * n;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long w = k / n;
    const int i = static_cast<int>(k - w * n);
    uf_union(p, i, vals[w * stride + i]);
  }
}

// this context's edges as (a, b) pairs, padded with (-1, -1) to n_pad (count read on the device)
__global__ void k_copy_edges(const int2* __restrict__ edges, const unsigned long long* __restrict__ count,
                             long long cap, int2* __restrict__ out, long long n_pad) {
  const long long ne = min(min(static_cast<long long>(*count), cap), n_pad);
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < n_pad;
       k += static_cast<long long>(gridDim.x) * blockDim.x)
    out[k] = k < ne ? edges[k] : make_int2(-1, -1);
}

// find without path halving: the finalize pass's only store is each node's own root.  (With
// halving here, another thread's late halving store into p[x] — an ancestor that is not the root —
// could land after x's own root store and leave x labelled with a non-root.)
__device__ int uf_root(int* p, int x) {
  while (true) {
    const int px = ld_rlx(p + x);
    if (px == x) return x;
    x = px;
  }
}

// A finalized forest's (read, root) pairs of the reads that are not their own root, in read order (the
// multi-GPU merge exchanges these instead of the raw edges: unions of the same partition).  A stream
// compaction without contended atomics: each block counts its contiguous range, one block scans the
// counts, each block writes its range at its offset.
constexpr int kForestBlocks = 1024;

// (finalize fused: each read's root is found and stored here, so k_forest_write reads final parents)
__global__ __launch_bounds__(256) void k_forest_count(int* __restrict__ p, int n, int chunk, int* __restrict__ bcnt) {
  __shared__ int ws[4];
  const int b0 = blockIdx.x * chunk, b1 = min(n, b0 + chunk);
  int c = 0;
  for (int x = b0 + static_cast<int>(threadIdx.x); x < b1; x += blockDim.x) {
    const int r = uf_root(p, x);
    st_rlx(p + x, r);
    c += r != x;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) bcnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// exclusive scan of the block counts in place (nb <= kForestBlocks), the total into *cnt
__global__ __launch_bounds__(kForestBlocks) void k_forest_scan(int* __restrict__ bcnt, int nb,
                                                               unsigned long long* __restrict__ cnt) {
  __shared__ int v[kForestBlocks];
  const int t = threadIdx.x;
  v[t] = t < nb ? bcnt[t] : 0;
  __syncthreads();
  for (int o = 1; o < kForestBlocks; o <<= 1) {
    const int add = t >= o ? v[t - o] : 0;
    __syncthreads();
    v[t] += add;
    __syncthreads();
  }
  if (t < nb) bcnt[t] = t ? v[t - 1] : 0;
  if (t == kForestBlocks - 1) *cnt = static_cast<unsigned long long>(v[t]);
}

__global__ __launch_bounds__(256) void k_forest_write(const int* __restrict__ p, int n, int chunk,
                                                      const int* __restrict__ bcnt, int2* __restrict__ out) {
  __shared__ int ws[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b0 = blockIdx.x * chunk, b1 = min(n, b0 + chunk);
  int base = bcnt[blockIdx.x];
  for (int x0 = b0; x0 < b1; x0 += blockDim.x) {
    const int x = x0 + static_cast<int>(threadIdx.x);
    const int r = x < b1 ? p[x] : x;
    const bool t = r != x;
    const unsigned long long m = __ballot(t);
    if (lane == 0) ws[w] = __popcll(m);
    __syncthreads();
    int before = 0, total = 0;
    for (int k = 0; k < 4; ++k) {
      before += k < w ? ws[k] : 0;
      total += ws[k];
    }
    if (t) out[base + before + __popcll(m & ((1ull << lane) - 1ull))] = make_int2(x, r);
    base += total;
    __syncthreads();
  }
}

__global__ void k_uf_finalize(int* p, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    st_rlx(p + i, uf_root(p, i));
}

}  // namespace

// one launch instead of four fills per query: counters, error words and forward degrees to 0, and the
// union-find parents to the identity (the sweep's pair kernel hooks them as it forms edges, so the
// components after it skip k_uf_init and k_uf_hook_min)
__global__ void k_query_reset(unsigned long long* __restrict__ counters, int nc, int* __restrict__ err, int ne,
                              int* __restrict__ fwd, int* __restrict__ parent, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nc) counters[i] = 0ull;
  if (i < ne) err[i] = 0;
  for (int k = i; k < n; k += gridDim.x * blockDim.x) {
    fwd[k] = 0;
    if (parent) parent[k] = k;
  }
}

hipError_t launch_query_reset(unsigned long long* counters, int nc, int* err, int ne, int* fwd, int* parent, int n,
                              hipStream_t s) {
  const long long work = std::max<long long>(std::max(nc, ne), n);
  k_query_reset<<<grid_for(work), 256, 0, s>>>(counters, nc, err, ne, fwd, parent, n);
  return hipGetLastError();
}

hipError_t launch_uf_init(int* parent, int n, hipStream_t s) {
  if (n > 0) k_uf_init<<<grid_for(n), 256, 0, s>>>(parent, n);
  return hipGetLastError();
}

// parent: the identity (launch_uf_init) — the min pre-hook overwrites links, which every edge's union then restores
hipError_t launch_uf_edges(int* parent, const int2* edges, const unsigned long long* count, long long cap, int* err,
                           hipStream_t s) {
  if (cap > 0) k_uf_hook_min<<<grid_for(cap), 256, 0, s>>>(parent, edges, count, cap);
  if (cap > 0) k_uf_edges<<<grid_for(cap), 256, 0, s>>>(parent, edges, count, cap, err);
  return hipGetLastError();
}

// parent already hooked by the edges' atomicMin (the sweep's pair kernel, SweepArgs::parent): the unions only
hipError_t launch_uf_unions(int* parent, const int2* edges, const unsigned long long* count, long long cap, int* err,
                            hipStream_t s) {
  if (cap > 0) k_uf_edges<<<grid_for(cap), 256, 0, s>>>(parent, edges, count, cap, err);
  return hipGetLastError();
}

hipError_t launch_uf_pairs(int* parent, const int* src, const int* dst, long long n, int period, hipStream_t s) {
  if (n > 0 && period > 0) k_uf_pairs<<<grid_for(n), 256, 0, s>>>(parent, src, dst, n, period);
  return hipGetLastError();
}

// parent: the identity (launch_uf_init), as for launch_uf_edges
hipError_t launch_uf_pair_list(int* parent, const int2* pairs, long long n, hipStream_t s) {
  if (n > 0) k_uf_hook_min_pairs<<<grid_for(n), 256, 0, s>>>(parent, pairs, n);
  if (n > 0) k_uf_pair_list<<<grid_for(n), 256, 0, s>>>(parent, pairs, n);
  return hipGetLastError();
}

// parent: the identity (launch_uf_init), as for launch_uf_edges
hipError_t launch_uf_strided(int* parent, const int* vals, long long blocks, int n, long long stride, hipStream_t s) {
  if (blocks > 0 && n > 0) k_uf_hook_min_strided<<<grid_for(blocks * n), 256, 0, s>>>(parent, vals, blocks, n, stride);
  if (blocks > 0 && n > 0) k_uf_strided<<<grid_for(blocks * n), 256, 0, s>>>(parent, vals, blocks, n, stride);
  return hipGetLastError();
}

hipError_t launch_copy_edges(const int2* edges, const unsigned long long* count, long long cap, int2* out,
                             long long n_pad, hipStream_t s) {
  if (n_pad > 0) k_copy_edges<<<grid_for(n_pad), 256, 0, s>>>(edges, count, cap, out, n_pad);
  return hipGetLastError();
}

hipError_t launch_forest_pairs(int* parent, int n, int2* out, unsigned long long* cnt, int* bcnt, hipStream_t s) {
  const int chunk = std::max(256, (n + kForestBlocks - 1) / kForestBlocks);
  const int nb = std::max(1, (n + chunk - 1) / chunk);
  k_forest_count<<<nb, 256, 0, s>>>(parent, n, chunk, bcnt);
  k_forest_scan<<<1, kForestBlocks, 0, s>>>(bcnt, nb, cnt);
  k_forest_write<<<nb, 256, 0, s>>>(parent, n, chunk, bcnt, out);
  return hipGetLastError();
}

hipError_t launch_uf_finalize(int* parent, int n, hipStream_t s) {
  if (n > 0) k_uf_finalize<<<grid_for(n), 256, 0, s>>>(parent, n);
  return hipGetLastError();
}

}  // namespace fslr
