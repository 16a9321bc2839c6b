// long.hip — read pairs with a read of more than FSLR_MAX_L intervals.
//
// The reference has no per-read interval limit: overall_jaccard_similarity (cluster.py:140-170)
// walks any two lists (its l2_comparisons scratch holds 100000 columns, :195).  The pair engines
// give an interval one lane or one bit of a 64-bit row / column mask, so a longer read is uploaded
// as several *virtual* reads of <= 64 intervals: virtual rank r < n_real is real read r (its first
// 64 intervals), ranks >= n_real are the further chunks of the long reads.  The sweep (sweep.hip)
// then meets every overlapping interval pair of the virtual reads once and writes its match entries
// (pair gate different_lengths_or_alignments :178-183 and calculate_overlap >= overlap :133-136
// applied — both depend only on the two reads' qlen2 / n_alignments and the two intervals, so a
// chunk inherits its real read's values).  Here:
//   1. k_long_split: an entry of two short real reads is passed on unchanged (fslr_sweep_evaluate
//      decides those pairs); an entry that touches a long read is mapped to real reads and interval
//      indices (ra < rb, ia in ra's list, jb in rb's list — calculate_overlap is symmetric, so the
//      orientation only picks list1 = the lower-rank read, whose loop meets the pair first without
//      the cap, cluster.py:197-208); entries within one real read (its chunks) are dropped
//      (:203-204).
//   2. the mapped entries are sorted by (ra, rb, ia, jb) (two stable radix passes) and split into
//      runs, one per read pair.
//   3. k_long_greedy, one thread per pair: first-fit in the reference's order — rows ascending, the
//      lowest unused matching column (:152-161) — with the used-column set as a bitmap of rb's
//      length in global scratch.  I = matches, U = L_a + L_b - I (:165), edge iff I > 0 and
//      U <= umax[I - 1] (the cutoff lookup :216-219 folded on the host like pass_table).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <string>
#include <vector>

#include "ctx.hpp"
#include "kernels.hpp"

namespace fslr {
namespace {

constexpr int kLongBlock = 256;
constexpr int kLongPerThread = 8;
constexpr unsigned kRank25 = (1u << 25) - 1;

__global__ void __launch_bounds__(kLongBlock)
k_long_split(const unsigned long long* __restrict__ ent, long long n, const int* __restrict__ vreal,
             const int* __restrict__ vbase, const int* __restrict__ rlen,
             unsigned long long* __restrict__ short_out, unsigned long long* __restrict__ pk_out,
             unsigned long long* __restrict__ ij_out, long long long_cap, unsigned long long* __restrict__ cnt) {
  __shared__ unsigned s_short, s_long;
  __shared__ unsigned long long b_short, b_long;
  if (threadIdx.x == 0) s_short = s_long = 0;
  __syncthreads();
  const long long base = static_cast<long long>(blockIdx.x) * (kLongBlock * kLongPerThread);
  unsigned long long e[kLongPerThread];
  unsigned long long pk[kLongPerThread], ij[kLongPerThread];
  unsigned char cls[kLongPerThread];
  unsigned ns = 0, nl = 0;
#pragma unroll
  for (int u = 0; u < kLongPerThread; ++u) {
    const long long k = base + u * kLongBlock + threadIdx.x;       // coalesced within each u
    cls[u] = 0;
    if (k >= n) continue;
    const unsigned long long v = ent[k];
    e[u] = v;
    const int A = static_cast<int>(v >> 39);
    const int B = static_cast<int>((v >> 14) & kRank25);
    const int i = static_cast<int>((v >> 7) & 127), j = static_cast<int>(v & 127);
    int ra = vreal[A], rb = vreal[B];
    if (ra == rb) continue;                                       // chunks of one read: its own hits
    if (rlen[ra] <= FSLR_MAX_L && rlen[rb] <= FSLR_MAX_L) {
      cls[u] = 1;
      ++ns;
      continue;
    }
    long long ia = vbase[A] + i, jb = vbase[B] + j;
    if (ra > rb) {
      const int t = ra; ra = rb; rb = t;
      const long long tt = ia; ia = jb; jb = tt;
    }
    pk[u] = (static_cast<unsigned long long>(ra) << 25) | static_cast<unsigned>(rb);
    ij[u] = (static_cast<unsigned long long>(ia) << 32) | static_cast<unsigned long long>(jb);
    cls[u] = 2;
    ++nl;
  }
  const unsigned os = ns ? atomicAdd(&s_short, ns) : 0u;     // LDS atomics: block-local offsets
  const unsigned ol = nl ? atomicAdd(&s_long, nl) : 0u;
  __syncthreads();
  if (threadIdx.x == 0) {                                        // one global atomic per class and block
    b_short = s_short ? atomicAdd(&cnt[0], static_cast<unsigned long long>(s_short)) : 0ull;
    b_long = s_long ? atomicAdd(&cnt[1], static_cast<unsigned long long>(s_long)) : 0ull;
  }
  __syncthreads();
  unsigned long long ps = b_short + os, pl = b_long + ol;
#pragma unroll
  for (int u = 0; u < kLongPerThread; ++u) {
    if (cls[u] == 1) short_out[ps++] = e[u];
    if (cls[u] == 2) {
      if (static_cast<long long>(pl) < long_cap) {
        pk_out[pl] = pk[u];
        ij_out[pl] = ij[u];
      }
      ++pl;
    }
  }
}

// bitmap words of each pair's partner list (rb = low 25 bits of the pair key)
__global__ void k_long_words(const unsigned long long* __restrict__ uniq, const int* __restrict__ nruns,
                             const int* __restrict__ rlen, long long* __restrict__ words) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= *nruns) return;
  const int rb = static_cast<int>(uniq[r] & kRank25);
  words[r] = (rlen[rb] + 31) >> 5;
}

__global__ void __launch_bounds__(kLongBlock)
k_long_greedy(const unsigned long long* __restrict__ uniq, const int* __restrict__ run_len,
              const int* __restrict__ run_off, const int* __restrict__ nruns,
              const unsigned long long* __restrict__ ij, const long long* __restrict__ words,
              const long long* __restrict__ woff, unsigned* __restrict__ bits, const int* __restrict__ rlen,
              const int* __restrict__ umax, int n_umax, int4* __restrict__ edges, long long edge_cap,
              unsigned long long* __restrict__ cnt) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= *nruns) return;
  const int ra = static_cast<int>(uniq[r] >> 25), rb = static_cast<int>(uniq[r] & kRank25);
  unsigned* used = bits + woff[r];
  for (long long w = 0; w < words[r]; ++w) used[w] = 0u;
  const int o = run_off[r], m = run_len[r];
  int I = 0;
  long long row_done = -1;                 // a row stops at its first free matching column (:158-161)
  for (int t = o; t < o + m; ++t) {
    const unsigned long long v = ij[t];
    const long long ia = static_cast<long long>(v >> 32);
    const unsigned jb = static_cast<unsigned>(v & 0xFFFFFFFFu);
    if (ia == row_done) continue;
    const unsigned bit = 1u << (jb & 31);
    if (used[jb >> 5] & bit) continue;
    used[jb >> 5] |= bit;
    ++I;
    row_done = ia;
  }
  const int U = rlen[ra] + rlen[rb] - I;
  if (I > 0 && I <= n_umax && U <= umax[I - 1]) {
    const unsigned long long k = atomicAdd(&cnt[2], 1ull);
    if (static_cast<long long>(k) < edge_cap) edges[k] = make_int4(ra, rb, I, U);
  }
}

constexpr int kMaxRealL = 4096;           // the cap replay's general pair evaluator (cap.hip kMaxLongL)

// the CSR offset of each long real read's second chunk: its intervals beyond FSLR_MAX_L are the
// consecutive chunks from there (prep.split_long_reads lays a read's chunks out in order)
__global__ void k_long_off2(const int4* __restrict__ rmeta, const int* __restrict__ vreal,
                            const int* __restrict__ vbase, int n_real, int nv, int* __restrict__ off2) {
  for (int v = n_real + blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += gridDim.x * blockDim.x)
    if (vbase[v] == FSLR_MAX_L) off2[vreal[v]] = rmeta[v].x;
}

template <typename T>
int grow(fslr_ctx* c, T** p, int64_t* cap, int64_t need) {
  if (need <= *cap) return FSLR_OK;
  const int64_t nc = need + (need >> 2) + 1024;
  if (int rc = dalloc(c, p, static_cast<size_t>(nc))) return rc;
  *cap = nc;
  return FSLR_OK;
}

}  // namespace
}  // namespace fslr

using namespace fslr;

void fslr_long_free(fslr_ctx* c) {
  void* bufs[] = {c->lg_vreal, c->lg_vbase, c->lg_rlen, c->lg_umax, c->lg_off2, c->lg_pk, c->lg_ij, c->lg_pk2, c->lg_ij2,
                  c->lg_edges, c->lg_cnt,   c->lg_uniq, c->lg_rlen_run, c->lg_roff, c->lg_words, c->lg_woff,
                  c->lg_bits,  c->lg_temp, c->lg_ent, c->lg_short};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
}

// The virtual CSR of a real one (the layout fslr_set_long_reads describes): virtual
// read r < n is real read r with its first FSLR_MAX_L intervals, the further FSLR_MAX_L-interval
// chunks of the long reads follow as reads n, n + 1, ... in real-rank, then chunk order; a chunk
// keeps its real read's qlen2 and n_alignments (the pair gate, cluster.py:178-183, and
// calculate_overlap, :133-136, see only those and the two intervals).  Uploaded with
// fslr_set_reads, the maps with fslr_set_long_reads (umax later: fslr_set_long_cutoffs).
extern "C" int fslr_set_reads_any(fslr_ctx* c, const fslr_reads* r) {
  if (c) c->hooked = false;
  if (!c || !r || r->n_reads < 0 || r->n_intervals < 0 || !r->read_off) return FSLR_ERR_INVALID;
  const int64_t n = r->n_reads, ni = r->n_intervals;
  if (r->read_off[0] != 0 || r->read_off[n] != ni) return fail(c, FSLR_ERR_INVALID, "read_off does not span intervals");
  std::vector<int> extra(static_cast<size_t>(n)), rlen(static_cast<size_t>(n));
  int64_t n_extra = 0;
  bool any_long = false;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t L = static_cast<int64_t>(r->read_off[i + 1]) - r->read_off[i];
    if (L < 1 || L > kMaxRealL)
      return fail(c, FSLR_ERR_INVALID, "every read needs 1.." + std::to_string(kMaxRealL) + " intervals");
    rlen[i] = static_cast<int>(L);
    extra[i] = static_cast<int>((L + FSLR_MAX_L - 1) / FSLR_MAX_L - 1);
    n_extra += extra[i];
    any_long |= L > FSLR_MAX_L;
  }
  if (!any_long) return fslr_set_reads(c, r);
  const int64_t nv = n + n_extra;
  if (nv >= FSLR_MAX_READS) return fail(c, FSLR_ERR_INVALID, "too many reads after the split into chunks");
  std::vector<int32_t> voff(static_cast<size_t>(nv) + 1), vreal(static_cast<size_t>(nv)), vbase(static_cast<size_t>(nv));
  std::vector<int32_t> vq(static_cast<size_t>(nv)), vn(static_cast<size_t>(nv));
  std::vector<int> perm(static_cast<size_t>(ni));
  // virtual read lengths: first chunks (ranks 0 .. n-1), then the further chunks in order
  int64_t v = n;
  for (int64_t i = 0; i < n; ++i) {
    vreal[i] = static_cast<int32_t>(i);
    vbase[i] = 0;
    voff[i + 1] = std::min(rlen[i], FSLR_MAX_L);
    for (int k = 1; k <= extra[i]; ++k, ++v) {
      vreal[v] = static_cast<int32_t>(i);
      vbase[v] = k * FSLR_MAX_L;
      voff[v + 1] = std::min(rlen[i] - k * FSLR_MAX_L, FSLR_MAX_L);
    }
  }
  voff[0] = 0;
  for (int64_t u = 0; u < nv; ++u) voff[u + 1] += voff[u];
  for (int64_t u = 0; u < nv; ++u) {
    const int64_t src = static_cast<int64_t>(r->read_off[vreal[u]]) + vbase[u];
    for (int64_t k = voff[u]; k < voff[u + 1]; ++k) perm[k] = static_cast<int>(src + (k - voff[u]));
    vq[u] = r->read_qlen2 ? r->read_qlen2[vreal[u]] : 0;
    vn[u] = r->read_nal ? r->read_nal[vreal[u]] : 0;
  }
  auto take = [&](const int32_t* a) {
    std::vector<int32_t> out;
    if (!a) return out;
    out.resize(static_cast<size_t>(ni));
    for (int64_t k = 0; k < ni; ++k) out[k] = a[perm[k]];
    return out;
  };
  const std::vector<int32_t> ch = take(r->iv_chrom), st = take(r->iv_start), en = take(r->iv_end),
                             th = take(r->iv_thr), dp = take(r->iv_data_pos);
  fslr_reads vr = *r;
  vr.n_reads = nv;
  vr.read_off = voff.data();
  vr.read_qlen2 = r->read_qlen2 ? vq.data() : nullptr;
  vr.read_nal = r->read_nal ? vn.data() : nullptr;
  vr.iv_chrom = r->iv_chrom ? ch.data() : nullptr;
  vr.iv_start = r->iv_start ? st.data() : nullptr;
  vr.iv_end = r->iv_end ? en.data() : nullptr;
  vr.iv_thr = r->iv_thr ? th.data() : nullptr;
  vr.iv_data_pos = r->iv_data_pos ? dp.data() : nullptr;
  if (int rc = fslr_set_reads(c, &vr)) return rc;
  // the cutoff table comes per query (fslr_set_long_cutoffs); a placeholder covers the longest read
  int maxl = 0;
  for (int L : rlen) maxl = std::max(maxl, L);
  std::vector<int32_t> um(static_cast<size_t>(maxl), 0);
  if (int rc = fslr_set_long_reads(c, n, vreal.data(), vbase.data(), rlen.data(), um.data(), maxl)) return rc;
  c->lg_perm.swap(perm);
  return FSLR_OK;
}

extern "C" int fslr_set_long_cutoffs(fslr_ctx* c, const int32_t* umax, int32_t n_umax) {
  if (!c || n_umax < 0 || (!umax && n_umax)) return FSLR_ERR_INVALID;
  if (!c->lg_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads_any (reads of more than FSLR_MAX_L intervals) first");
  HIP_TRY(c, hipSetDevice(c->device));
  int maxl = 0;
  std::vector<int> rl(static_cast<size_t>(c->lg_n_real));
  if (c->lg_n_real) HIP_TRY(c, hipMemcpy(rl.data(), c->lg_rlen, rl.size() * sizeof(int), hipMemcpyDeviceToHost));
  for (int L : rl) maxl = std::max(maxl, L);
  if (n_umax < maxl) return fail(c, FSLR_ERR_INVALID, "umax must cover I up to the longest read");
  if (n_umax > c->lg_n_umax && dalloc(c, &c->lg_umax, n_umax)) return FSLR_ERR_NOMEM;
  if (n_umax) HIP_TRY(c, hipMemcpyAsync(c->lg_umax, umax, n_umax * sizeof(int), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->lg_n_umax = n_umax;
  return FSLR_OK;
}

extern "C" int fslr_set_long_reads(fslr_ctx* c, int64_t n_real, const int32_t* vreal, const int32_t* vbase,
                                   const int32_t* rlen, const int32_t* umax, int32_t n_umax) {
  if (c) c->hooked = false;
  if (!c || n_real < 0 || !vreal || !vbase || (!rlen && n_real) || (!umax && n_umax) || n_umax < 0)
    return FSLR_ERR_INVALID;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first (the virtual CSR)");
  HIP_TRY(c, hipSetDevice(c->device));
  const int64_t nv = c->n;
  if (n_real > nv) return fail(c, FSLR_ERR_INVALID, "n_real exceeds the uploaded (virtual) reads");
  // the virtual CSR: rank r < n_real is real read r; each virtual read lies inside its real read
  std::vector<int> lens(static_cast<size_t>(n_real));
  int maxl = 0;
  for (int64_t r = 0; r < n_real; ++r) {
    if (rlen[r] < 1) return fail(c, FSLR_ERR_INVALID, "real read without intervals");
    lens[r] = rlen[r];
    maxl = std::max(maxl, rlen[r]);
  }
  for (int64_t v = 0; v < nv; ++v) {
    const int r = vreal[v];
    if (r < 0 || r >= n_real || (v < n_real && r != v) || vbase[v] < 0 || vbase[v] >= lens[r])
      return fail(c, FSLR_ERR_INVALID, "virtual read map out of range");
  }
  if (n_umax < maxl) return fail(c, FSLR_ERR_INVALID, "umax must cover I up to the longest read");
  if (maxl > kMaxRealL) return fail(c, FSLR_ERR_INVALID, "reads of more than 4096 intervals are not supported");
  if (dalloc(c, &c->lg_vreal, nv) || dalloc(c, &c->lg_vbase, nv) || dalloc(c, &c->lg_rlen, n_real) ||
      dalloc(c, &c->lg_umax, n_umax) || dalloc(c, &c->lg_off2, std::max<int64_t>(n_real, 1)) ||
      (!c->lg_cnt && dalloc(c, &c->lg_cnt, 4)))
    return FSLR_ERR_NOMEM;
  HIP_TRY(c, hipMemcpyAsync(c->lg_vreal, vreal, nv * sizeof(int), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->lg_vbase, vbase, nv * sizeof(int), hipMemcpyHostToDevice, c->stream));
  if (n_real) HIP_TRY(c, hipMemcpyAsync(c->lg_rlen, rlen, n_real * sizeof(int), hipMemcpyHostToDevice, c->stream));
  if (n_umax) HIP_TRY(c, hipMemcpyAsync(c->lg_umax, umax, n_umax * sizeof(int), hipMemcpyHostToDevice, c->stream));
  if (nv > n_real)
    k_long_off2<<<grid_for(nv - n_real), 256, 0, c->stream>>>(c->rmeta, c->lg_vreal, c->lg_vbase, n_real, nv, c->lg_off2);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->lg_n_real = n_real;
  c->lg_n_umax = n_umax;
  c->lg_set = true;
  c->lg_n_edges = 0;
  return FSLR_OK;
}

// the split + long-pair stage over n entries at `entries` (device); short entries to short_dst
static int long_evaluate(fslr_ctx* c, const void* entries, int64_t n, void* short_dst, int64_t* n_short,
                         int64_t* n_long_edges) {
  HIP_TRY(c, hipSetDevice(c->device));
  const hipStream_t s = c->stream;
  unsigned long long h[4] = {};
  HIP_TRY(c, hipMemsetAsync(c->lg_cnt, 0, 4 * sizeof(unsigned long long), s));
  // 1. split (the long-entry buffers grow and the split reruns when they were too small)
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (n) {
      const long long per = kLongBlock * kLongPerThread;
      const unsigned grid = static_cast<unsigned>((n + per - 1) / per);
      HIP_TRY(c, hipMemsetAsync(c->lg_cnt, 0, 4 * sizeof(unsigned long long), s));
      k_long_split<<<grid, kLongBlock, 0, s>>>(static_cast<const unsigned long long*>(entries), n, c->lg_vreal,
                                               c->lg_vbase, c->lg_rlen, static_cast<unsigned long long*>(short_dst),
                                               c->lg_pk, c->lg_ij, c->lg_cap, c->lg_cnt);
      HIP_TRY(c, hipGetLastError());
    }
    HIP_TRY(c, hipMemcpyAsync(h, c->lg_cnt, sizeof(h), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    if (static_cast<int64_t>(h[1]) <= c->lg_cap) break;
    const int64_t need = static_cast<int64_t>(h[1]);
    int64_t cap = c->lg_cap, cap2 = c->lg_cap, cap3 = c->lg_cap, cap4 = c->lg_cap;
    if (grow(c, &c->lg_pk, &cap, need) || grow(c, &c->lg_ij, &cap2, need) || grow(c, &c->lg_pk2, &cap3, need) ||
        grow(c, &c->lg_ij2, &cap4, need))
      return FSLR_ERR_NOMEM;
    c->lg_cap = cap;
  }
  *n_short = static_cast<int64_t>(h[0]);
  const int64_t nl = static_cast<int64_t>(h[1]);
  c->lg_n_edges = 0;
  *n_long_edges = 0;
  if (nl == 0) return FSLR_OK;
  if (nl >= (int64_t(1) << 31)) return fail(c, FSLR_ERR_INVALID, "too many long-read match entries");
  // 2. sort by (ra, rb, ia, jb): ij first, then the pair key (stable), then runs
  const int m = static_cast<int>(nl);
  if (nl + 1 > c->lg_run_cap) {
    const int64_t rc = nl + (nl >> 2) + 1024;
    if (dalloc(c, &c->lg_uniq, rc) || dalloc(c, &c->lg_rlen_run, rc) || dalloc(c, &c->lg_roff, rc) ||
        dalloc(c, &c->lg_words, rc) || dalloc(c, &c->lg_woff, rc))
      return FSLR_ERR_NOMEM;
    c->lg_run_cap = rc;
  }
  size_t t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0;
  int* d_nruns = reinterpret_cast<int*>(c->lg_cnt + 3);
  HIP_TRY(c, hipcub::DeviceRadixSort::SortPairs(nullptr, t1, c->lg_ij, c->lg_ij2, c->lg_pk, c->lg_pk2, m, 0, 64, s));
  HIP_TRY(c, hipcub::DeviceRadixSort::SortPairs(nullptr, t2, c->lg_pk2, c->lg_pk, c->lg_ij2, c->lg_ij, m, 0, 50, s));
  HIP_TRY(c, hipcub::DeviceRunLengthEncode::Encode(nullptr, t3, c->lg_pk, c->lg_uniq, c->lg_rlen_run, d_nruns, m, s));
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, t4, c->lg_rlen_run, c->lg_roff, m, s));
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, t5, c->lg_words, c->lg_woff, m, s));
  const size_t tb = std::max({t1, t2, t3, t4, t5});
  if (tb > c->lg_temp_bytes) {
    if (dalloc(c, &c->lg_temp, tb)) return FSLR_ERR_NOMEM;
    c->lg_temp_bytes = tb;
  }
  size_t tt = c->lg_temp_bytes;
  HIP_TRY(c, hipcub::DeviceRadixSort::SortPairs(c->lg_temp, tt, c->lg_ij, c->lg_ij2, c->lg_pk, c->lg_pk2, m, 0, 64, s));
  tt = c->lg_temp_bytes;
  HIP_TRY(c, hipcub::DeviceRadixSort::SortPairs(c->lg_temp, tt, c->lg_pk2, c->lg_pk, c->lg_ij2, c->lg_ij, m, 0, 50, s));
  tt = c->lg_temp_bytes;
  HIP_TRY(c, hipcub::DeviceRunLengthEncode::Encode(c->lg_temp, tt, c->lg_pk, c->lg_uniq, c->lg_rlen_run, d_nruns, m, s));
  tt = c->lg_temp_bytes;
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(c->lg_temp, tt, c->lg_rlen_run, c->lg_roff, m, s));
  const unsigned g = static_cast<unsigned>((m + kLongBlock - 1) / kLongBlock);
  HIP_TRY(c, hipMemsetAsync(c->lg_words, 0, static_cast<size_t>(m) * sizeof(long long), s));
  k_long_words<<<g, kLongBlock, 0, s>>>(c->lg_uniq, d_nruns, c->lg_rlen, c->lg_words);
  HIP_TRY(c, hipGetLastError());
  tt = c->lg_temp_bytes;
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(c->lg_temp, tt, c->lg_words, c->lg_woff, m, s));
  // bitmap size: the last run's offset + words (runs beyond nruns have 0 words)
  long long wtot[2] = {};
  HIP_TRY(c, hipMemcpyAsync(&wtot[0], c->lg_woff + (m - 1), sizeof(long long), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipMemcpyAsync(&wtot[1], c->lg_words + (m - 1), sizeof(long long), hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  const int64_t nwords = wtot[0] + wtot[1];
  if (grow(c, &c->lg_bits, &c->lg_bits_cap, nwords)) return FSLR_ERR_NOMEM;
  // 3. first-fit per pair; edges (ra, rb, I, U), grown and rerun on overflow
  for (int attempt = 0; attempt < 2; ++attempt) {
    HIP_TRY(c, hipMemsetAsync(c->lg_cnt + 2, 0, sizeof(unsigned long long), s));
    k_long_greedy<<<g, kLongBlock, 0, s>>>(c->lg_uniq, c->lg_rlen_run, c->lg_roff, d_nruns, c->lg_ij, c->lg_words,
                                           c->lg_woff, c->lg_bits, c->lg_rlen, c->lg_umax, c->lg_n_umax, c->lg_edges,
                                           c->lg_edge_cap, c->lg_cnt);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipMemcpyAsync(h, c->lg_cnt, sizeof(h), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    if (static_cast<int64_t>(h[2]) <= c->lg_edge_cap) break;
    if (grow(c, &c->lg_edges, &c->lg_edge_cap, static_cast<int64_t>(h[2]))) return FSLR_ERR_NOMEM;
  }
  c->lg_n_edges = static_cast<int64_t>(h[2]);
  *n_long_edges = c->lg_n_edges;
  return FSLR_OK;
}

extern "C" int fslr_long_query(fslr_ctx* c, const fslr_params* p, int64_t* n_long_edges) {
  if (!c || !p || !n_long_edges) return FSLR_ERR_INVALID;
  if (!c->lg_set) return fail(c, FSLR_ERR_STATE, "fslr_set_long_reads first");
  HIP_TRY(c, hipSetDevice(c->device));
  // 1. every match entry of the virtual index (one destination), into a context-owned buffer
  int64_t cnt = 0;
  int rc = fslr_sweep_partition(c, p, 1, 6, c->lg_ent, c->lg_ent_cap, &cnt);
  if (rc == FSLR_ERR_STATE && cnt > c->lg_ent_cap) {
    if (grow(c, &c->lg_ent, &c->lg_ent_cap, cnt)) return FSLR_ERR_NOMEM;
    rc = fslr_sweep_partition(c, p, 1, 6, c->lg_ent, c->lg_ent_cap, &cnt);
  }
  if (rc) return rc;
  // 2. split; pairs with a long read decided here
  if (grow(c, &c->lg_short, &c->lg_short_cap, std::max<int64_t>(cnt, 1))) return FSLR_ERR_NOMEM;
  int64_t n_short = 0;
  if ((rc = long_evaluate(c, c->lg_ent, cnt, c->lg_short, &n_short, n_long_edges))) return rc;
  // 3. pairs of two short reads: the sweep's pair stage
  return fslr_sweep_evaluate(c, p, c->lg_short, n_short);
}

extern "C" int fslr_get_long_edges(fslr_ctx* c, int32_t* a, int32_t* b, int32_t* I, int32_t* U, int64_t capacity) {
  if (!c || capacity < 0) return FSLR_ERR_INVALID;
  if (c->lg_n_edges > capacity) return fail(c, FSLR_ERR_INVALID, "output capacity too small");
  if (c->lg_n_edges == 0) return FSLR_OK;
  HIP_TRY(c, hipSetDevice(c->device));
  std::vector<int4> tmp(static_cast<size_t>(c->lg_n_edges));
  HIP_TRY(c, hipMemcpyAsync(tmp.data(), c->lg_edges, tmp.size() * sizeof(int4), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  for (size_t k = 0; k < tmp.size(); ++k) {
    if (a) a[k] = tmp[k].x;
    if (b) b[k] = tmp[k].y;
    if (I) I[k] = tmp[k].z;
    if (U) U[k] = tmp[k].w;
  }
  return FSLR_OK;
}
