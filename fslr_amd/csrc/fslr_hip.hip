// fslr_hip.hip — MI355X (gfx950 / CDNA4) kernels for fslr's clustering hot path.
//
// Replaces, on the GPU, the per-query-read driver of the reference
// (/root/reference/fslr/cluster.py:187-227) together with the interval index it
// queries (cluster.py:124-130 + superintervals) and the connected components
// (cluster.py:230-234).  C ABI: include/fslr_hip.h.  Design: DESIGN.md.
//
// Device data (HBM, structure-of-records, 16 B per record):
//   rmeta[N]   int4 {iv offset, len | flags<<16, qlen2, n_alignments}   (rank order)
//   iv[NI]     int4 {chrom, start, end, thr}                             (CSR, data order)
//   idx[NI]    int4 {start, end, pmax_end, read<<6 | j}   intervals sorted by (chrom,start)
//   iv_pos[NI] int  position of CSR interval k in idx
//
// Kernels:
//   index_*      radix sort of (chrom<<32 | start), scatter, max-scan of (chrom<<32 | end)
//   query_kernel one wavefront per query read A (grid-stride over ranks):
//                (1) candidate scan: for every interval of A, 64 lanes walk the sorted
//                    index forward (start <= end_A) and backward (prefix-max end >= start_A)
//                    with coalesced 1 KiB loads; hits with rank(B) > A go to an LDS queue
//                (2) evaluation: one candidate (A, B, i, j) per lane; lane walks B's
//                    intervals j (its own gather), A's intervals i come from registers by
//                    v_readlane (wave-uniform).  Per row j it forms the 64-bit overlap mask
//                    O_j and match mask M_j over A and runs the first-fit greedy on them;
//                    the pair is evaluated by exactly one candidate: the one whose (j, i)
//                    is the first overlapping interval pair in B-major order (witness rule).
//   uf_*         lock-free union-find (hook larger root under smaller) → label = min rank.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "fslr_hip.h"

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kQueueCap = 2 * kWave;
constexpr int kPassStride = 2 * FSLR_MAX_L;
constexpr int kMaxCoord = 1 << 30;

enum Counter { kEdgeCount = 0, kEval = 1, kJacc = 2, kCand = 3, kAlgoBytes = 4, kNumCounters = 5 };

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

// cluster.py:178-183 different_lengths_or_alignments → returns "pair passes" (not different);
// *zd = the reference would raise ZeroDivisionError (max == 0).
__device__ __forceinline__ bool lengths_pass(int q1, int q2, int n1, int n2, double qcut, double ncut,
                                             bool* zd) {
  int mn = min(q1, q2), mx = max(q1, q2);
  if (mx == 0) { *zd = true; return false; }
  if (static_cast<double>(mn) / static_cast<double>(mx) >= qcut) return true;
  mn = min(n1, n2); mx = max(n1, n2);
  if (mx == 0) { *zd = true; return false; }
  return static_cast<double>(mn) / static_cast<double>(mx) >= ncut;
}

// ---------------------------------------------------------------- index build
__global__ void k_fill_iv_read(const int4* __restrict__ rmeta, int n, int* __restrict__ iv_read) {
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
    const int4 m = rmeta[r];
    const int len = m.y & 0xffff;
    for (int k = 0; k < len; ++k) iv_read[m.x + k] = r;
  }
}

__global__ void k_make_keys(const int4* __restrict__ iv, int ni, unsigned long long* __restrict__ keys,
                            int* __restrict__ vals) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ni; k += gridDim.x * blockDim.x) {
    const int4 r = iv[k];
    keys[k] = (static_cast<unsigned long long>(r.x) << 32) | static_cast<unsigned>(r.y);
    vals[k] = k;
  }
}

__global__ void k_scatter_index(const unsigned long long* __restrict__ skeys, const int* __restrict__ svals,
                                const int4* __restrict__ iv, const int* __restrict__ iv_read,
                                const int4* __restrict__ rmeta, int ni, int4* __restrict__ idx,
                                int* __restrict__ iv_pos, unsigned long long* __restrict__ endkey,
                                int2* __restrict__ crange) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < ni; q += gridDim.x * blockDim.x) {
    const int k = svals[q];
    const int r = iv_read[k];
    const int j = k - rmeta[r].x;
    const int4 rec = iv[k];
    idx[q] = make_int4(rec.y, rec.z, 0, (r << 6) | j);
    iv_pos[k] = q;
    endkey[q] = (static_cast<unsigned long long>(rec.x) << 32) | static_cast<unsigned>(rec.z);
    const int c = rec.x;
    if (q == 0 || static_cast<int>(skeys[q - 1] >> 32) != c) crange[c].x = q;
    if (q == ni - 1 || static_cast<int>(skeys[q + 1] >> 32) != c) crange[c].y = q + 1;
  }
}

__global__ void k_set_thr(const int* __restrict__ thr, int4* __restrict__ iv, int ni) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ni; k += gridDim.x * blockDim.x) iv[k].w = thr[k];
}

__global__ void k_set_pmax(const unsigned long long* __restrict__ pmaxkey, int4* __restrict__ idx, int ni) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < ni; q += gridDim.x * blockDim.x)
    idx[q].z = static_cast<int>(static_cast<unsigned>(pmaxkey[q]));
}

struct MaxU64 {
  __device__ __forceinline__ unsigned long long operator()(unsigned long long a, unsigned long long b) const {
    return a > b ? a : b;
  }
};

// ---------------------------------------------------------------- pair kernel
struct QueryArgs {
  const int4* rmeta;
  const int4* iv;
  const int* iv_pos;
  const int4* idx;
  const int2* crange;
  const unsigned char* pass;
  double qlen_cut, nal_cut;
  int a_begin, a_end;
  int2* edges;
  unsigned short* edge_iu;
  long long edge_cap;
  int* fwd;
  unsigned long long* counters;
  int* err;       // [0] code, [1] a, [2] b
  int* max_fwd;
};

template <bool kGeneralThr>
__global__ __launch_bounds__(kBlock) void query_kernel(QueryArgs g) {
  __shared__ unsigned long long queue[kWavesPerBlock][kQueueCap];
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  unsigned long long* Q = queue[wv];
  const int nwaves = gridDim.x * kWavesPerBlock;
  unsigned long long w_eval = 0, w_jacc = 0, w_cand = 0;
  unsigned long long l_bytes = 0;   // per lane: algorithmic bytes of the pairs it evaluated
  int w_maxfwd = 0;

  for (int a = g.a_begin + blockIdx.x * kWavesPerBlock + wv; a < g.a_end; a += nwaves) {
    const int4 am = g.rmeta[a];
    const int offA = __builtin_amdgcn_readfirstlane(am.x);
    const int LA = __builtin_amdgcn_readfirstlane(am.y & 0xffff);
    const bool hazA = (__builtin_amdgcn_readfirstlane(am.y) >> 16) & 1;
    const int q1 = __builtin_amdgcn_readfirstlane(am.z), n1 = __builtin_amdgcn_readfirstlane(am.w);
    // A's intervals live in lanes 0..LA-1; wave-uniform reads via v_readlane.
    int4 my = make_int4(-1, 0, 0, 0);
    int mypos = 0;
    if (lane < LA) {
      my = g.iv[offA + lane];
      mypos = g.iv_pos[offA + lane];
    }
    const unsigned long long fullA = LA == 64 ? ~0ull : ((1ull << LA) - 1ull);
    int qn = 0;
    int fwdA = 0;

    // evaluate the first nb queue entries (one per lane), then compact the queue
    auto process = [&](int nb) {
      wave_lds_sync();
      const bool act = lane < nb;
      const unsigned long long e = act ? Q[lane] : 0ull;
      const int rem = qn - nb;
      const unsigned long long mv = lane < rem ? Q[nb + lane] : 0ull;
      wave_lds_sync();
      if (lane < rem) Q[lane] = mv;
      qn = rem;

      const int B = static_cast<int>(e >> 12);
      const int ic = static_cast<int>((e >> 6) & 63);
      const int jc = static_cast<int>(e & 63);
      int4 bm = make_int4(0, 0, 0, 0);
      if (act) bm = g.rmeta[B];
      const int offB = bm.x;
      const int LB = act ? (bm.y & 0xffff) : 0;
      const bool haz = hazA || ((bm.y >> 16) & 1);
      bool zd = false;
      const bool lenok = act && lengths_pass(q1, bm.z, n1, bm.w, g.qlen_cut, g.nal_cut, &zd);
      const bool full = lenok && !haz;
      unsigned long long freeA = fullA;
      int I = 0;
      int state = act ? 0 : 2;          // 0: witness unknown, 1: canonical, 2: duplicate / idle
      for (int j = 0; j < LB; ++j) {
        const int4 b = g.iv[offB + j];
        unsigned long long O = 0ull, M = 0ull;
        for (int i = 0; i < LA; ++i) {
          const int ci = rdl(my.x, i), si = rdl(my.y, i), ei = rdl(my.z, i), ti = rdl(my.w, i);
          const bool same = b.x == ci;
          const int lo = max(b.y, si), hi = min(b.z, ei);
          const int o = max(hi - lo, 0);
          bool mt;
          if (kGeneralThr) mt = same && thr_ok(o, ti) && thr_ok(o, b.w);
          else mt = same && o >= max(ti, b.w);
          O |= static_cast<unsigned long long>(same && hi >= lo) << i;
          M |= static_cast<unsigned long long>(mt) << i;
        }
        if (state == 0 && O != 0ull) state = (j == jc && __builtin_ctzll(O) == ic) ? 1 : 2;
        if (state == 2 || (state == 1 && !full)) break;
        const unsigned long long m = M & freeA;
        if (m) { freeA ^= m & (~m + 1ull); ++I; }
      }
      const bool canon = state == 1;
      // SURVEY §8d unit cost: both reads' interval records + both read records, no reuse
      if (canon) l_bytes += 16ull * static_cast<unsigned long long>(LA + LB) + 32ull;
      bool edge = false;
      int U = 0;
      if (canon && lenok && haz) {
        // exact replay of cluster.py:152-161 (i-major, used-skip, break) for pairs holding an
        // aln_size == 0 interval: ZeroDivisionError exactly when the reference divides by it
        unsigned long long used = 0ull;
        I = 0;
        for (int i = 0; i < LA && !zd; ++i) {
          const int4 ai = g.iv[offA + i];
          for (int j = 0; j < LB; ++j) {
            if ((used >> j) & 1ull) continue;
            const int4 b = g.iv[offB + j];
            if (b.x != ai.x) continue;
            if (ai.w == FSLR_THR_ZERO_ALN || b.w == FSLR_THR_ZERO_ALN) { zd = true; break; }
            const int o = max(min(ai.z, b.z) - max(ai.y, b.y), 0);
            if (thr_ok(o, ai.w) && thr_ok(o, b.w)) { used |= 1ull << j; ++I; break; }
          }
        }
      }
      if (canon && zd) {
        if (atomicCAS(g.err, 0, FSLR_ERR_ZERO_DIVISION) == 0) { g.err[1] = a; g.err[2] = B; }
      } else if (canon && lenok && I > 0) {
        U = LA + LB - I;
        edge = g.pass[(I - 1) * kPassStride + (U - 1)] != 0;
      }
      const unsigned long long cm = __ballot(canon);
      const unsigned long long jm = __ballot(canon && lenok);
      w_eval += __popcll(cm);
      w_jacc += __popcll(jm);
      const unsigned long long em = __ballot(edge);
      const int ne = __popcll(em);
      if (ne) {
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(&g.counters[kEdgeCount], static_cast<unsigned long long>(ne));
        base = __shfl(base, 0);
        if (edge) {
          const long long k = static_cast<long long>(base) + mbcnt(em);
          if (k < g.edge_cap) {
            g.edges[k] = make_int2(a, B);
            g.edge_iu[k] = static_cast<unsigned short>(I | (U << 8));
          }
        }
        fwdA += ne;
      }
    };

    auto push = [&](bool cand, unsigned long long entry) {
      const unsigned long long m = __ballot(cand);
      if (cand) Q[qn + mbcnt(m)] = entry;
      qn += __popcll(m);
      if (qn >= kWave) process(kWave);
    };

    for (int i = 0; i < LA; ++i) {
      const int ci = rdl(my.x, i), si = rdl(my.y, i), ei = rdl(my.z, i), pi = rdl(mypos, i);
      const int2 cr = g.crange[ci];
      // forward: sorted positions after pi with start <= end_i (all overlap, end >= start >= start_i)
      for (int base = pi + 1; base < cr.y; base += kWave) {
        const int q = base + lane;
        bool ok = false;
        int rj = 0;
        if (q < cr.y) {
          const int4 r = g.idx[q];
          ok = r.x <= ei;
          rj = r.w;
        }
        const unsigned long long okm = __ballot(ok);
        w_cand += __popcll(okm);
        push(ok && (rj >> 6) > a, (static_cast<unsigned long long>(rj >> 6) << 12) |
                                      (static_cast<unsigned long long>(i) << 6) | (rj & 63));
        if (okm != ~0ull) break;
      }
      // backward: positions before pi while prefix-max end >= start_i; hit iff end >= start_i
      for (int base = pi - 1; base >= cr.x; base -= kWave) {
        const int q = base - lane;
        bool cont = false, ok = false;
        int rj = 0;
        if (q >= cr.x) {
          const int4 r = g.idx[q];
          cont = r.z >= si;
          ok = cont && r.y >= si;
          rj = r.w;
        }
        const unsigned long long cm = __ballot(cont);
        w_cand += __popcll(__ballot(ok));
        push(ok && (rj >> 6) > a, (static_cast<unsigned long long>(rj >> 6) << 12) |
                                      (static_cast<unsigned long long>(i) << 6) | (rj & 63));
        if (cm != ~0ull) break;
      }
    }
    while (qn > 0) process(min(qn, kWave));
    if (lane == 0) g.fwd[a] = fwdA;
    w_maxfwd = max(w_maxfwd, fwdA);
  }
  for (int o = 32; o > 0; o >>= 1) l_bytes += __shfl_xor(l_bytes, o);
  if (lane == 0) {
    if (l_bytes) atomicAdd(&g.counters[kAlgoBytes], l_bytes);
    if (w_eval) atomicAdd(&g.counters[kEval], w_eval);
    if (w_jacc) atomicAdd(&g.counters[kJacc], w_jacc);
    if (w_cand) atomicAdd(&g.counters[kCand], w_cand);
    if (w_maxfwd) atomicMax(g.max_fwd, w_maxfwd);
  }
}

// ---------------------------------------------------------------- union-find
__device__ __forceinline__ int ld_rlx(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rlx(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    const int old = atomicCAS(p + b, b, a);   // hook the larger root under the smaller
    if (old == b) return;
    b = old;
  }
}

__global__ void k_uf_init(int* p, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = i;
}

__global__ void k_uf_edges(int* p, const int2* __restrict__ edges, const unsigned long long* __restrict__ count,
                           long long cap) {
  const long long ne = min(static_cast<long long>(*count), cap);
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < ne;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int2 e = edges[k];
    uf_union(p, e.x, e.y);
  }
}

__global__ void k_uf_pairs(int* p, const int* __restrict__ src, const int* __restrict__ dst, long long n) {
  for (long long k = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; k < n;
       k += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int s = src ? src[k] : static_cast<int>(k);
    uf_union(p, s, dst[k]);
  }
}

__global__ void k_uf_finalize(int* p, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    st_rlx(p + i, uf_find(p, i));
}

int grid_for(long long n, int block = 256, int cap = 256 * 16) {
  long long g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<int>(g);
}

}  // namespace

// ==================================================================== host side
struct fslr_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::string err;
  int64_t n = 0, ni = 0;
  int n_chroms = 0;
  bool general_thr = false;
  bool reads_set = false, index_built = false;
  // device buffers
  int4* rmeta = nullptr;
  int4* iv = nullptr;
  int* iv_pos = nullptr;
  int* iv_read = nullptr;
  int4* idx = nullptr;
  int2* crange = nullptr;
  unsigned long long* keys = nullptr;
  unsigned long long* keys2 = nullptr;
  int* vals = nullptr;
  int* vals2 = nullptr;
  unsigned long long* endkey = nullptr;
  unsigned long long* pmaxkey = nullptr;
  void* temp = nullptr;
  size_t temp_bytes = 0;
  unsigned char* pass = nullptr;
  int2* edges = nullptr;
  unsigned short* edge_iu = nullptr;
  int64_t edge_cap = 0;
  int* fwd = nullptr;
  int* parent = nullptr;
  unsigned long long* counters = nullptr;
  int* errw = nullptr;     // [0..2] error, [3] max_fwd
  int64_t cap_n = 0, cap_ni = 0, cap_chroms = 0;
  std::vector<unsigned char> pass_host;
  std::vector<unsigned char> aln_zero_host;   // per CSR interval: thr == FSLR_THR_ZERO_ALN at set_reads
  // profiling
  bool profiling = false;
  hipEvent_t ev[8] = {};
  bool ev_ok = false;
  float t_index = 0, t_query = 0, t_comp = 0, t_total = 0;
  bool t_index_rec = false, t_query_rec = false, t_comp_rec = false;
};

namespace {

int fail(fslr_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIP_TRY(ctx, expr)                                                                       \
  do {                                                                                           \
    hipError_t e_ = (expr);                                                                      \
    if (e_ != hipSuccess)                                                                        \
      return fail((ctx), FSLR_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));       \
  } while (0)

template <typename T>
int dalloc(fslr_ctx* c, T** p, size_t count) {
  if (*p) { (void)hipFree(*p); *p = nullptr; }
  if (count == 0) count = 1;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
  if (e != hipSuccess) return fail(c, FSLR_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  return FSLR_OK;
}

int ensure_capacity(fslr_ctx* c, int64_t n, int64_t ni, int n_chroms) {
  int rc;
  if (n > c->cap_n) {
    if ((rc = dalloc(c, &c->rmeta, n)) || (rc = dalloc(c, &c->fwd, n)) || (rc = dalloc(c, &c->parent, n)))
      return rc;
    c->cap_n = n;
  }
  if (ni > c->cap_ni) {
    if ((rc = dalloc(c, &c->iv, ni)) || (rc = dalloc(c, &c->iv_pos, ni)) || (rc = dalloc(c, &c->iv_read, ni)) ||
        (rc = dalloc(c, &c->idx, ni)) || (rc = dalloc(c, &c->keys, ni)) || (rc = dalloc(c, &c->keys2, ni)) ||
        (rc = dalloc(c, &c->vals, ni)) || (rc = dalloc(c, &c->vals2, ni)) || (rc = dalloc(c, &c->endkey, ni)) ||
        (rc = dalloc(c, &c->pmaxkey, ni)))
      return rc;
    c->cap_ni = ni;
    // temp storage for the radix sort and the max-scan
    size_t b1 = 0, b2 = 0;
    HIP_TRY(c, hipcub::DeviceRadixSort::SortPairs(nullptr, b1, c->keys, c->keys2, c->vals, c->vals2,
                                                  static_cast<int>(ni), 0, 64, c->stream));
    HIP_TRY(c, hipcub::DeviceScan::InclusiveScan(nullptr, b2, c->endkey, c->pmaxkey, MaxU64(),
                                                 static_cast<int>(ni), c->stream));
    const size_t need = std::max(b1, b2);
    if (need > c->temp_bytes) {
      if (c->temp) (void)hipFree(c->temp);
      c->temp = nullptr;
      HIP_TRY(c, hipMalloc(&c->temp, need));
      c->temp_bytes = need;
    }
  }
  if (n_chroms > c->cap_chroms) {
    if ((rc = dalloc(c, &c->crange, n_chroms))) return rc;
    c->cap_chroms = n_chroms;
  }
  if (!c->pass) {
    if ((rc = dalloc(c, &c->pass, FSLR_MAX_L * kPassStride))) return rc;
    if ((rc = dalloc(c, &c->counters, kNumCounters))) return rc;
    if ((rc = dalloc(c, &c->errw, 4))) return rc;
  }
  return FSLR_OK;
}

int bits_for(int v) {
  int b = 1;
  while ((1 << b) <= v) ++b;
  return b;
}

}  // namespace

extern "C" {

int fslr_abi_version(void) { return FSLR_ABI_VERSION; }

const char* fslr_last_error(const fslr_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int fslr_ctx_create(int device, void* stream, fslr_ctx** out) {
  if (!out) return FSLR_ERR_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return FSLR_ERR_HIP;
  if (device < 0 || device >= ndev) return FSLR_ERR_INVALID;
  if (hipSetDevice(device) != hipSuccess) return FSLR_ERR_HIP;
  fslr_ctx* c = new fslr_ctx();
  c->device = device;
  if (stream) {
    c->stream = static_cast<hipStream_t>(stream);
  } else {
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) { delete c; return FSLR_ERR_HIP; }
    c->own_stream = true;
  }
  *out = c;
  return FSLR_OK;
}

void fslr_ctx_destroy(fslr_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  void* bufs[] = {c->rmeta, c->iv, c->iv_pos, c->iv_read, c->idx, c->crange, c->keys, c->keys2, c->vals,
                  c->vals2, c->endkey, c->pmaxkey, c->temp, c->pass, c->edges, c->edge_iu, c->fwd, c->parent,
                  c->counters, c->errw};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (c->ev_ok)
    for (auto& e : c->ev) (void)hipEventDestroy(e);
  if (c->own_stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int fslr_set_profiling(fslr_ctx* c, int enable) {
  if (!c) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  if (enable && !c->ev_ok) {
    for (auto& e : c->ev) HIP_TRY(c, hipEventCreate(&e));
    c->ev_ok = true;
  }
  c->profiling = enable != 0;
  return FSLR_OK;
}

int fslr_set_reads(fslr_ctx* c, const fslr_reads* r) {
  if (!c || !r) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  const int64_t n = r->n_reads, ni = r->n_intervals;
  if (n < 0 || ni < 0 || n >= FSLR_MAX_READS || ni >= (int64_t(1) << 31) - 1)
    return fail(c, FSLR_ERR_INVALID, "read / interval count out of range");
  if (r->n_chroms < 1 || r->n_chroms >= (1 << 24)) return fail(c, FSLR_ERR_INVALID, "n_chroms out of range");
  if (!r->read_off || !r->read_qlen2 || !r->read_nal || !r->iv_chrom || !r->iv_start || !r->iv_end || !r->iv_thr)
    return fail(c, FSLR_ERR_INVALID, "null array");
  if (r->read_off[0] != 0 || r->read_off[n] != ni) return fail(c, FSLR_ERR_INVALID, "read_off does not span intervals");
  std::vector<int4> rm(static_cast<size_t>(n));
  std::vector<int4> iv(static_cast<size_t>(ni));
  c->aln_zero_host.assign(static_cast<size_t>(ni), 0);
  bool general = false;
  for (int64_t k = 0; k < ni; ++k) {
    const int ch = r->iv_chrom[k], s = r->iv_start[k], e = r->iv_end[k], t = r->iv_thr[k];
    if (ch < 0 || ch >= r->n_chroms) return fail(c, FSLR_ERR_INVALID, "chrom id out of range");
    if (s < 0 || e < s || e >= kMaxCoord) return fail(c, FSLR_ERR_INVALID, "interval coordinates out of [0, 2^30)");
    if (t < 0 && t != FSLR_THR_ZERO_ALN) general = true;
    if (t == FSLR_THR_ZERO_ALN) c->aln_zero_host[k] = 1;
    iv[k] = make_int4(ch, s, e, t);
  }
  for (int64_t i = 0; i < n; ++i) {
    const int o = r->read_off[i], len = r->read_off[i + 1] - o;
    if (len < 1 || len > FSLR_MAX_L)
      return fail(c, FSLR_ERR_INVALID, "every read needs 1.." + std::to_string(FSLR_MAX_L) + " intervals");
    int flags = 0;
    for (int k = o; k < o + len; ++k)
      if (iv[k].w == FSLR_THR_ZERO_ALN) flags |= 1;
    rm[i] = make_int4(o, len | (flags << 16), r->read_qlen2[i], r->read_nal[i]);
  }
  int rc = ensure_capacity(c, n, ni, r->n_chroms);
  if (rc) return rc;
  c->n = n;
  c->ni = ni;
  c->n_chroms = r->n_chroms;
  c->general_thr = general;
  if (n) HIP_TRY(c, hipMemcpyAsync(c->rmeta, rm.data(), n * sizeof(int4), hipMemcpyHostToDevice, c->stream));
  if (ni) HIP_TRY(c, hipMemcpyAsync(c->iv, iv.data(), ni * sizeof(int4), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->reads_set = true;
  c->index_built = false;
  return FSLR_OK;
}

int fslr_set_thresholds(fslr_ctx* c, const int32_t* thr) {
  if (!c || (!thr && c->ni)) return FSLR_ERR_INVALID;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  HIP_TRY(c, hipSetDevice(c->device));
  bool general = false;
  for (int64_t k = 0; k < c->ni; ++k)
    if (thr[k] < 0 && thr[k] != FSLR_THR_ZERO_ALN) general = true;
  if ((c->aln_zero_host.size() != static_cast<size_t>(c->ni)))
    return fail(c, FSLR_ERR_STATE, "internal: zero-aln map missing");
  for (int64_t k = 0; k < c->ni; ++k)
    if ((thr[k] == FSLR_THR_ZERO_ALN) != (c->aln_zero_host[k] != 0))
      return fail(c, FSLR_ERR_INVALID, "FSLR_THR_ZERO_ALN must mark the same intervals as in fslr_set_reads");
  if (c->ni) {
    int* tmp = nullptr;
    HIP_TRY(c, hipMallocAsync(reinterpret_cast<void**>(&tmp), c->ni * sizeof(int), c->stream));
    HIP_TRY(c, hipMemcpyAsync(tmp, thr, c->ni * sizeof(int), hipMemcpyHostToDevice, c->stream));
    k_set_thr<<<grid_for(c->ni), 256, 0, c->stream>>>(tmp, c->iv, static_cast<int>(c->ni));
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipFreeAsync(tmp, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  c->general_thr = general;
  return FSLR_OK;
}

int fslr_reserve_edges(fslr_ctx* c, int64_t capacity) {
  if (!c || capacity < 0) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  if (capacity <= c->edge_cap) return FSLR_OK;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  int rc;
  if ((rc = dalloc(c, &c->edges, capacity)) || (rc = dalloc(c, &c->edge_iu, capacity))) return rc;
  c->edge_cap = capacity;
  return FSLR_OK;
}

int fslr_build_index(fslr_ctx* c) {
  if (!c) return FSLR_ERR_INVALID;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->profiling) HIP_TRY(c, hipEventRecord(c->ev[0], c->stream));
  const int ni = static_cast<int>(c->ni), n = static_cast<int>(c->n);
  if (ni > 0) {
    HIP_TRY(c, hipMemsetAsync(c->crange, 0, c->n_chroms * sizeof(int2), c->stream));
    k_fill_iv_read<<<grid_for(n), 256, 0, c->stream>>>(c->rmeta, n, c->iv_read);
    k_make_keys<<<grid_for(ni), 256, 0, c->stream>>>(c->iv, ni, c->keys, c->vals);
    size_t tb = c->temp_bytes;
    HIP_TRY(c, hipcub::DeviceRadixSort::SortPairs(c->temp, tb, c->keys, c->keys2, c->vals, c->vals2, ni, 0,
                                                  32 + bits_for(c->n_chroms), c->stream));
    k_scatter_index<<<grid_for(ni), 256, 0, c->stream>>>(c->keys2, c->vals2, c->iv, c->iv_read, c->rmeta, ni,
                                                         c->idx, c->iv_pos, c->endkey, c->crange);
    tb = c->temp_bytes;
    HIP_TRY(c, hipcub::DeviceScan::InclusiveScan(c->temp, tb, c->endkey, c->pmaxkey, MaxU64(), ni, c->stream));
    k_set_pmax<<<grid_for(ni), 256, 0, c->stream>>>(c->pmaxkey, c->idx, ni);
    HIP_TRY(c, hipGetLastError());
  }
  if (c->profiling) HIP_TRY(c, hipEventRecord(c->ev[1], c->stream));
  c->t_index_rec = c->profiling;
  c->index_built = true;
  return FSLR_OK;
}

int fslr_query(fslr_ctx* c, const fslr_params* p, int64_t a_begin, int64_t a_end) {
  if (!c || !p || !p->pass_table) return FSLR_ERR_INVALID;
  if (!c->index_built) return fail(c, FSLR_ERR_STATE, "fslr_build_index first");
  if (a_begin < 0 || a_end > c->n || a_begin > a_end) return fail(c, FSLR_ERR_INVALID, "bad read range");
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->edge_cap == 0) {
    int rc = fslr_reserve_edges(c, std::max<int64_t>(1 << 16, 12 * c->n));
    if (rc) return rc;
  }
  c->pass_host.assign(p->pass_table, p->pass_table + FSLR_MAX_L * kPassStride);
  HIP_TRY(c, hipMemcpyAsync(c->pass, c->pass_host.data(), c->pass_host.size(), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipMemsetAsync(c->counters, 0, kNumCounters * sizeof(unsigned long long), c->stream));
  HIP_TRY(c, hipMemsetAsync(c->errw, 0, 4 * sizeof(int), c->stream));
  if (c->n) HIP_TRY(c, hipMemsetAsync(c->fwd, 0, c->n * sizeof(int), c->stream));
  QueryArgs g;
  g.rmeta = c->rmeta;
  g.iv = c->iv;
  g.iv_pos = c->iv_pos;
  g.idx = c->idx;
  g.crange = c->crange;
  g.pass = c->pass;
  g.qlen_cut = p->qlen_cut;
  g.nal_cut = p->nal_cut;
  g.a_begin = static_cast<int>(a_begin);
  g.a_end = static_cast<int>(a_end);
  g.edges = c->edges;
  g.edge_iu = c->edge_iu;
  g.edge_cap = c->edge_cap;
  g.fwd = c->fwd;
  g.counters = c->counters;
  g.err = c->errw;
  g.max_fwd = c->errw + 3;
  const int64_t nq = a_end - a_begin;
  if (c->profiling) HIP_TRY(c, hipEventRecord(c->ev[2], c->stream));
  if (nq > 0) {
    const int blocks = static_cast<int>(std::min<int64_t>((nq + kWavesPerBlock - 1) / kWavesPerBlock, 256 * 8));
    if (c->general_thr)
      query_kernel<true><<<blocks, kBlock, 0, c->stream>>>(g);
    else
      query_kernel<false><<<blocks, kBlock, 0, c->stream>>>(g);
    HIP_TRY(c, hipGetLastError());
  }
  if (c->profiling) HIP_TRY(c, hipEventRecord(c->ev[3], c->stream));
  c->t_query_rec = c->profiling;
  return FSLR_OK;
}

int fslr_components(fslr_ctx* c) {
  if (!c) return FSLR_ERR_INVALID;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->profiling) HIP_TRY(c, hipEventRecord(c->ev[4], c->stream));
  const int n = static_cast<int>(c->n);
  if (n) {
    k_uf_init<<<grid_for(n), 256, 0, c->stream>>>(c->parent, n);
    if (c->edge_cap) k_uf_edges<<<grid_for(c->edge_cap), 256, 0, c->stream>>>(c->parent, c->edges, c->counters,
                                                                             c->edge_cap);
    k_uf_finalize<<<grid_for(n), 256, 0, c->stream>>>(c->parent, n);
    HIP_TRY(c, hipGetLastError());
  }
  if (c->profiling) HIP_TRY(c, hipEventRecord(c->ev[5], c->stream));
  c->t_comp_rec = c->profiling;
  return FSLR_OK;
}

int fslr_run(fslr_ctx* c, const fslr_params* p) {
  int rc = fslr_build_index(c);
  if (rc) return rc;
  if ((rc = fslr_query(c, p, 0, c->n))) return rc;
  return fslr_components(c);
}

int fslr_sync(fslr_ctx* c) {
  if (!c) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FSLR_OK;
}

int fslr_read_stats(fslr_ctx* c, fslr_query_stats* out) {
  if (!c || !out) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  unsigned long long cnt[kNumCounters] = {};
  int ew[4] = {};
  if (c->counters) {
    HIP_TRY(c, hipMemcpyAsync(cnt, c->counters, sizeof(cnt), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipMemcpyAsync(ew, c->errw, sizeof(ew), hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  out->n_edges = static_cast<int64_t>(cnt[kEdgeCount]);
  out->evaluated_pairs = static_cast<int64_t>(cnt[kEval]);
  out->jaccard_evals = static_cast<int64_t>(cnt[kJacc]);
  out->candidates = static_cast<int64_t>(cnt[kCand]);
  out->error = ew[0];
  out->err_a = ew[1];
  out->err_b = ew[2];
  out->max_fwd = ew[3];
  out->algo_bytes = static_cast<int64_t>(cnt[kAlgoBytes]);
  if (ew[0] == FSLR_ERR_ZERO_DIVISION) {
    c->err = "division by zero";
    return FSLR_ERR_ZERO_DIVISION;
  }
  return FSLR_OK;
}

int fslr_get_timings(fslr_ctx* c, fslr_timings* out) {
  if (!c || !out) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  std::memset(out, 0, sizeof(*out));
  if (!c->ev_ok) return FSLR_OK;
  if (c->t_index_rec) HIP_TRY(c, hipEventElapsedTime(&out->index_ms, c->ev[0], c->ev[1]));
  if (c->t_query_rec) HIP_TRY(c, hipEventElapsedTime(&out->query_ms, c->ev[2], c->ev[3]));
  if (c->t_comp_rec) HIP_TRY(c, hipEventElapsedTime(&out->components_ms, c->ev[4], c->ev[5]));
  if (c->t_index_rec && c->t_comp_rec) HIP_TRY(c, hipEventElapsedTime(&out->total_ms, c->ev[0], c->ev[5]));
  return FSLR_OK;
}

int fslr_get_labels(fslr_ctx* c, int32_t* labels) {
  if (!c || (!labels && c->n)) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->n) HIP_TRY(c, hipMemcpyAsync(labels, c->parent, c->n * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FSLR_OK;
}

int fslr_get_fwd_degree(fslr_ctx* c, int32_t* fwd) {
  if (!c || (!fwd && c->n)) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->n) HIP_TRY(c, hipMemcpyAsync(fwd, c->fwd, c->n * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FSLR_OK;
}

int fslr_get_edges(fslr_ctx* c, int32_t* a, int32_t* b, uint16_t* iu, int64_t capacity) {
  if (!c) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  unsigned long long cnt = 0;
  if (c->counters)
    HIP_TRY(c, hipMemcpyAsync(&cnt, c->counters + kEdgeCount, sizeof(cnt), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  const int64_t ne = static_cast<int64_t>(cnt);
  if (ne > c->edge_cap) return fail(c, FSLR_ERR_STATE, "edge buffer overflowed; reserve and rerun");
  if (ne > capacity) return fail(c, FSLR_ERR_INVALID, "output capacity too small");
  if (ne == 0) return FSLR_OK;
  std::vector<int2> tmp(static_cast<size_t>(ne));
  HIP_TRY(c, hipMemcpyAsync(tmp.data(), c->edges, ne * sizeof(int2), hipMemcpyDeviceToHost, c->stream));
  if (iu) HIP_TRY(c, hipMemcpyAsync(iu, c->edge_iu, ne * sizeof(uint16_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  for (int64_t k = 0; k < ne; ++k) {
    if (a) a[k] = tmp[k].x;
    if (b) b[k] = tmp[k].y;
  }
  return FSLR_OK;
}

int fslr_labels_device_ptr(fslr_ctx* c, void** dptr) {
  if (!c || !dptr) return FSLR_ERR_INVALID;
  *dptr = c->parent;
  return FSLR_OK;
}

int fslr_copy_labels_device(fslr_ctx* c, int32_t* dst) {
  if (!c || (!dst && c->n)) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->n) HIP_TRY(c, hipMemcpyAsync(dst, c->parent, c->n * sizeof(int), hipMemcpyDeviceToDevice, c->stream));
  return FSLR_OK;
}

int fslr_copy_fwd_device(fslr_ctx* c, int32_t* dst) {
  if (!c || (!dst && c->n)) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->n) HIP_TRY(c, hipMemcpyAsync(dst, c->fwd, c->n * sizeof(int), hipMemcpyDeviceToDevice, c->stream));
  return FSLR_OK;
}

int fslr_union_pairs(fslr_ctx* c, const int32_t* src, const int32_t* dst, int64_t n, int on_device) {
  if (!c || !dst || n < 0) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  if (n == 0) return FSLR_OK;
  const int* ds = src;
  const int* dd = dst;
  int* tmp = nullptr;
  if (!on_device) {
    HIP_TRY(c, hipMallocAsync(reinterpret_cast<void**>(&tmp), (src ? 2 : 1) * n * sizeof(int), c->stream));
    HIP_TRY(c, hipMemcpyAsync(tmp, dst, n * sizeof(int), hipMemcpyHostToDevice, c->stream));
    dd = tmp;
    if (src) {
      HIP_TRY(c, hipMemcpyAsync(tmp + n, src, n * sizeof(int), hipMemcpyHostToDevice, c->stream));
      ds = tmp + n;
    }
  }
  k_uf_pairs<<<grid_for(n), 256, 0, c->stream>>>(c->parent, ds, dd, n);
  HIP_TRY(c, hipGetLastError());
  if (tmp) {
    HIP_TRY(c, hipFreeAsync(tmp, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  return FSLR_OK;
}

int fslr_finalize_labels(fslr_ctx* c) {
  if (!c) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  const int n = static_cast<int>(c->n);
  if (n) k_uf_finalize<<<grid_for(n), 256, 0, c->stream>>>(c->parent, n);
  HIP_TRY(c, hipGetLastError());
  return FSLR_OK;
}

}  // extern "C"
