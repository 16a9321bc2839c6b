// kernels.hpp — internal interface between the C API (capi.hip) and the gfx950 kernels.
//
// Device layout (all in HBM, see DESIGN.md "Data layout"):
//   rmeta[N]    int4 {iv offset, len | flags<<16, qlen2, n_alignments}       rank order
//   iv[NI]      int4 {chrom, start, end, thr}                                 CSR (rank, data order)
//   qpos[NI]    int  q = position of CSR interval k in the (chrom,start)-sorted index
//   rng_s[NI]   int2 {n_fwd, bwd_begin} per sorted position q: positions q+1 .. q+n_fwd all
//               overlap it (start <= end_q); bwd_begin .. q-1 are the earlier positions whose
//               prefix-max end reaches start_q (hit iff end >= start_q)
//   idx4[NI]    int4 {start, end, thr, read << 6 | j} of the interval at sorted position
//   idx_gate[NI] int2 {qlen2, nal | LB << 24 | haz << 31} of the read at sorted position
//               (the pair gate's inputs, read beside the hit; nal < 2^24 is validated)
#pragma once
#include <hip/hip_runtime.h>

#include <cassert>
#include <cstddef>
#include <cstdint>

// The bounds-checked build (make -C fslr_amd/csrc bounds -> libfslr_hip_bounds.so): a device assert on
// the global indices of the paths only dense inputs reach (k_sweep<2>'s deep tiles, k_sweep_pairs' long
// runs and windows, the cap replay's frontier).  A failing index aborts the launch with its file:line
// instead of reading another allocation.  Compiled out of the product build.
#ifdef FSLR_DEBUG_BOUNDS
#define FSLR_BOUND(i, n) assert(static_cast<long long>(i) >= 0 && static_cast<long long>(i) < static_cast<long long>(n))
#else
#define FSLR_BOUND(i, n) ((void)0)
#endif

namespace fslr {

constexpr int kWave = 64;
constexpr int kPassStride = 128;      // 2 * FSLR_MAX_L
constexpr int kMaxCoord = 1 << 30;
constexpr int kShardShift = 6;
// error words (QueryArgs::err): [0] code, [1] a, [2] b, [3] max forward degree, [4] overflow flags
// (1: deferred list, 2: edge buffer) — a query that lost pairs; its labels are refused
constexpr int kErrWords = 8;
constexpr int kErrOverflow = 4;
// [6]: pairs whose evaluation raises ZeroDivisionError (cluster.py:135, 179, 181), listed as int2
// (a, b) from word kErrZdList (capacity at word kErrZdCap).  The engines only list them: whether the
// reference raises depends on whether a loop reaches the pair, which the edge cap decides
// (fslr_read_stats, fslr_apply_edge_cap).  A repeated partition and its evaluation keep the count.
constexpr int kErrZdCount = 6;
// [7]: sticky flags of repeated multi-GPU partitions (32: totals differed), kept across queries and
// cleared by the next synchronous fslr_sweep_partition / fslr_query
constexpr int kErrSticky = 7;
constexpr int kErrKeep = 6;           // a repeat's reset clears [0, kErrKeep); a query's all kErrWords
constexpr int kErrZdCap = 8;          // never reset: the list's capacity in pairs
constexpr int kErrZdList = 16;
constexpr int kZdListInit = 1 << 16;
// query shards own blocks of 64 consecutive ranks, round robin

__host__ __device__ inline bool shard_owns(int read, int shard, int n_shards) {
  return n_shards == 1 || ((read >> kShardShift) % n_shards) == shard;
}

// Device counters.  The two hot atomics (edge / deferred appends) sit on cache lines of their own;
// the pair kernel's per-wave statistics are plain stores into per-wave slots (`wstat`) summed by a
// small reduction kernel, so no wave ever retires through a contended global atomic.
enum Counter { kEdgeCount = 0,          // atomic (own 128-B line)
               kDeferCount = 16,        // atomic (own 128-B line)
               kEval = 32, kJacc = 33, kCand = 34, kAlgoBytes = 35, kOverflow = 36, kGather = 37,
               kMatchEntries = 38, kMatchedPairs = 39, kMaxFwd = 40, kWalked = 41,
               kSecBase = 48,           // FSLR_SECTION_PROF builds: per-section cycle sums of the pair kernel
               kHeavyCount = 64,        // atomic (own 128-B line): reads handed to the partitioned launch
               kQueueBase = 80,         // pair kernel work queues: 8 counters, one 128-B line each
               kQueueStride = 16,
               kQueueBase2 = kQueueBase + 8 * kQueueStride,   // the partitioned launch's queues
               kSwTests = kQueueBase2 + 8 * kQueueStride,     // sweep: interval pairs tested
               kSwNdev = kSwTests + 8,                        // sweep: entry count for the kernels (sync-free query)
               kNumCounters = kSwTests + 16 };
// per-wave statistics of query_kernel: fields 0..8 (sum, except kWsMaxFwd: max; kWsWalked: index
// records walked, every pass counted), then (section-
// timing builds) 8 section sums, slowest read cycles (max), its rank, wave cycles max / min,
// wave count, cycle sums of reads 0, 1 and >= 2 of the wave
enum WaveStat { kWsEval = 0, kWsJacc, kWsCand, kWsAlgoBytes, kWsOverflow, kWsMatchEntries, kWsMatchedPairs,
                kWsMaxFwd, kWsWalked, kWsBase = 9, kWsProf = kWsBase + 16, kWStride = 32 };

// ---- pair predicates shared by the pair kernels (query.hip) and the cap replay (cap.hip) ----
// interval accepts overlap o (fslr_hip.h: thr >= 0 ? o >= thr : o <= ~thr)
__device__ __forceinline__ bool thr_ok(int o, int t) { return t >= 0 ? o >= t : o <= ~t; }

// calculate_overlap(i1, i2) >= overlap (cluster.py:133-136), same chromosome already checked
__device__ __forceinline__ bool iv_match_general(int sa, int ea, int ta, int sb, int eb, int tb) {
  const int o = max(min(ea, eb) - max(sa, sb), 0);
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

// ---- index build (index.hip) -------------------------------------------------------------
struct IndexBufs {
  int shard, n_shards;                // A-side outputs (qpos, rng_s) only for reads of this query shard
  const int4* rmeta;
  const int4* iv;
  const unsigned* dchrom;             // [NI] or nullptr: chromosome per data position (start-sorted
  const int4* drec;                   //      order given) and {start, end, thr, tag} per data position
  const int2* dgate;                  // [NI] data order: the owning read's gate word (idx_gate)
  const int* data_pos;                // [NI] CSR index -> data position
  int* chist;                         // scratch [64 x (NI / 1024 + 1)] chromosome counts per sub-tile
  unsigned long long* keys;           // scratch [NI] x2 (double buffer for the sort)
  unsigned long long* keys2;
  int* vals;
  int* vals2;
  int* s_start;                       // scratch [NI] starts in sorted order
  unsigned long long* endkey;         // scratch [NI]
  unsigned long long* pmaxkey;        // scratch [NI]
  void* temp;
  size_t temp_bytes;
  const int2* crange;                 // [n_chroms] {begin, end} in sorted order (host counts)
  int* qpos;                          // out [NI] CSR order
  int2* rng_s;                        // out [NI] sorted order
  int* swin;                          // out [NI] the sweep's forward window (k_ranges: swin)
  long long* tile_tests;              // out [NI / 64 + 1] or nullptr: per 64-position tile, the sum of swin
                                      // (the lean build; the sweep's plan then skips k_tile_tests)
  int4* idx4;                         // out [NI]
  int2* idx_gate;                     // out [NI]
};
// bytes of hipcub temp storage the index build needs for ni intervals
hipError_t index_temp_bytes(int ni, size_t* bytes, hipStream_t s);
// full = false: only what the sweep engine reads (records, gate words, forward counts); applies to
// the data-order path with <= 64 chromosomes (the other paths always build everything)
hipError_t launch_build_index(const IndexBufs& b, int n_reads, int ni, int n_chroms, bool full, hipStream_t s);
// a lean (sweep-only) index's full scatter again: the (chrom, end) keys and the data -> sorted map the
// walk parts and the backward ranges read (same records, same order)
hipError_t launch_index_rescatter(const IndexBufs& b, int ni, int n_chroms, hipStream_t s);
// a lean index's (chrom, end) keys alone (its end column stays in b.vals): what the backward ranges read
// the sweep windows again from the index's thresholds (after fslr_set_thresholds patched them)
hipError_t launch_index_swin(const IndexBufs& b, int ni, hipStream_t s);
hipError_t launch_index_endkeys(const IndexBufs& b, int ni, int n_chroms, hipStream_t s);
// the walk engine's parts of a sweep-only index (qpos, tile prefix, backward ranges)
hipError_t launch_index_walk_parts(const IndexBufs& b, int n_reads, int ni, hipStream_t s);
// the backward scan ranges alone (tile prefix of end + k_ranges<true>): no CSR map, so it also
// serves a chromosome-filtered index
hipError_t launch_index_bwd_ranges(const IndexBufs& b, int ni, hipStream_t s);
// thresholds into iv[k].w and (when the index exists) idx4[qpos[k]].z
hipError_t launch_set_thr(const int* thr, int4* iv, const int* qpos, int4* idx4, const int* data_pos,
                          int4* drec, int ni, hipStream_t s);

// ---- pair kernel (query.hip) -------------------------------------------------------------
struct QueryArgs {
  const int4* rmeta;
  const int4* iv;
  const int* qpos;
  const int2* rng_s;
  const int4* idx4;
  const int2* idx_gate;
  const int* umax;                    // [64]: pair with I matches is an edge iff U <= umax[I-1]
  int4* lb;                           // [N] scratch: per query read {qlo, qhi, nlo, nhi} (length gate)
  double qlen_cut, nal_cut;
  int a_begin, a_end;
  int shard, n_shards;                // query reads: blocks of 64 ranks of [a_begin, a_end) dealt round robin
  int nv;                             // (launch_query) number of this shard's query reads
  int k_static;                       // (launch_query) grid-stride sweeps before the work queues
  int pass_records;                   // (launch_query) forward records per partner partition (0: one pass)
  int* heavy;                         // [a_end] reads for the partitioned launch (query_kernel<., true>)
  int2* edges;
  unsigned short* edge_iu;
  long long edge_cap;
  int* fwd;
  unsigned long long* defer;          // deferred pairs (query_kernel → deferred_kernel)
  long long defer_cap;
  unsigned long long* counters;
  int* err;                           // [0] code, [1] a, [2] b, [3] max forward degree
  int mode;                           // profiling ablation (FSLR_ABLATE): 0 full, 1 scan only, 2 no greedy
  unsigned long long* wstat;          // [wstat_waves x kWStride] per-wave statistics (plain stores)
  int wstat_waves;
  unsigned long long* diag;           // FSLR_SECTION_PROF: [N] per read (start cycle in its wave) << 32 | cycles
  hipEvent_t ev_k0, ev_k1;            // (profiling) recorded around the main pair-kernel launch, or null
};
// thr_mode: 0 = every non-sentinel threshold >= 1 (fast match), 1 = general encoding
hipError_t launch_query(const QueryArgs& a, int thr_mode, hipStream_t s);
// per read a in [a0, a1): lb[a] = the length gate as integer ranges {qlo, qhi, nlo, nhi}
hipError_t launch_len_bounds(const int4* rmeta, int a0, int a1, double qcut, double ncut, int4* lb, hipStream_t s);
// waves of the largest query_kernel grid (the size of QueryArgs::wstat)
int query_max_waves();

// ---- position sweep (sweep.hip) ------------------------------------------------------------
struct SweepArgs {
  const int4* rmeta;
  const unsigned char* rlen8;         // [n_reads] interval count of each read (1 B: stays in L2)
  const int4* idx4;
  const int2* idx_gate;
  const int2* rng_s;
  const int* swin;                    // [NI] the sweep's forward window of each position (k_ranges)
  const int* umax;
  int ni, n_reads;
  int nq;                             // query positions [0, nq) of the index (the rest: a forward halo)
  int a_begin, a_end;                 // reads whose pairs (as the lower rank A) are evaluated
  double qlen_cut, nal_cut;
  int4* lb;                           // [n_reads] length-gate ranges (launch_len_bounds)
  long long* tile_cnt;                // [ceil(ni / 64)] match entries of each 64-position tile
  long long* tile_off;                // its exclusive scan: the tile's place in `ent`
  long long* tile_tests;              // [tiles] pair tests of the tile (its forward-range total)
  bool tests_ready;                   // tile_tests already hold the sums (the lean index build's)
  long long* tile_ub;                 // their exclusive scan: the tile's upper-bound slot in ent_ub
  unsigned long long* ent_ub;         // (one pass) entries at their tiles' upper-bound slots
  long long ub_cap;
  unsigned long long* ent;            // [n_ent] match entries A << 39 | B << 14 | i << 7 | j, tile order
  unsigned long long* ent_sorted;     // [n_ent] grouped by A
  unsigned long long* ent_mid;        // (mode 3) [n_ent] grouping scratch
  unsigned long long* pair_scr;       // [n_ent] free during k_sweep_pairs (the grouping's other buffer):
                                      // long runs are bucketed there at their own positions
  int* grp;                           // [grp_ints()] grouping-sort bucket counts / offsets (null: radix sort)
  int* hist_mat;                      // (mode 2, one GPU) k_sweep<2> writes [bucket][block] counts of the
                                      // coarse A buckets A >> hist_lo here (null: the grouping counts them)
  int hist_lo, hist_h;                // coarse bucket shift and count (<= sweep_hist_max())
  int hist_mod;                       // 1: bucket = (A >> hist_lo) % hist_h (a partition's destinations)
  long long* dest_totals;             // (partition) per destination entry totals, filled by k_sweep_total when small
  long long n_ent;                    // (emit / pairs) entries of the count pass (host; with n_dev: an estimate)
  const long long* n_dev;             // null, or the device word holding the count (sync-free repeat query)
  long long ent_cap;                  // capacity of ent / ent_sorted (grouping-sort scatter bound)
  void* temp;                         // hipcub scratch (tile scan, grouping sort)
  size_t temp_bytes;
  int2* edges;
  unsigned short* edge_iu;
  long long edge_cap;
  int* fwd;
  int* parent;                        // non-null: each edge (A, B) also takes parent[B] down to A (the union-find's
                                      // min pre-hook, components.hip); the query reset made it the identity
  unsigned long long* counters;
  int* err;
  unsigned long long* wstat;          // per-wave statistics slots [waves x 4] (no contended atomics)
  int wstat_waves;
  int* wlo;                           // (one-pass sweep) [waves + 1]: wave w sweeps tiles [wlo[w], wlo[w + 1])

  hipEvent_t ev[5];                   // (profiling) count | scan | emit | sort | pairs boundaries, or null
  hipEvent_t k0, k1;                  // (profiling) around the sweep kernel launch alone, or null
  hipEvent_t p0, p1;                  // (profiling) around the pair-stage kernel (k_sweep_pairs) alone, or null
};
size_t sweep_temp_bytes(long long ent_cap, long long ni, hipStream_t s);
int sweep_max_waves();
// per tile: pair tests and their scan (the one-pass upper-bound slots)
hipError_t launch_sweep_plan(const SweepArgs& a, hipStream_t s);
// mode 2: the one-pass sweep (entries to ent_ub); mode 0: the count pass of the two-pass fallback.
// Then the tile scan; total_dev[0..2] = entries, upper-bound total, overflow flags (read after a sync)
hipError_t launch_sweep_count(const SweepArgs& a, int mode, long long* total_dev, hipStream_t s,
                              long long* n_dev = nullptr, long long cap = -1);
// packs (mode 2) or writes (mode 0: emit pass) the entries to `ent` (mode 3: they are there), groups
// them by A, evaluates the pairs
hipError_t launch_sweep_pairs(const SweepArgs& a, int mode, hipStream_t s);
// only the packing / emit step of launch_sweep_pairs: dense entries in a.ent
hipError_t launch_sweep_dense(const SweepArgs& a, int mode, hipStream_t s);
int grp_ints();
// the one-GPU sweep counts its entries per coarse A bucket while it writes them (no grouping count
// pass): sets a.hist_mat / hist_lo / hist_h for the input's read count
void sweep_coarse_hist(SweepArgs& a);
// the partition's variant: the sweep counts its entries per destination (A >> shift) % n_dest
void sweep_dest_hist(SweepArgs& a, int n_dest, int shift);
// multi-GPU: the sweep's entries (mode 2: in the tile slots; 0: dense in a.ent) grouped by destination
// (A >> shift) % n_dest into dst (entries beyond dst_cap dropped); totals[k] (device) per destination
hipError_t launch_sweep_partition(const SweepArgs& a, int mode, int shift, int n_dest, unsigned long long* dst,
                                  long long dst_cap, long long* totals, hipStream_t s);

// ---- multi-GPU sweep (shard.hip) -------------------------------------------------------------
constexpr int kMaxDest = 64;          // destination ranks of one partition
// the data-order records of the owned chromosomes (lmap[c] >= 0: its local number), compacted in
// data order (stable), their chromosome renumbered lmap[c]
// the position split (shard.hip): per 64-position tile its pair tests and forward-window end; the
// data positions of a sorted-position range and their records in data order
hipError_t launch_tile_costs(const int* swin, int ni, long long* tests, long long* reach, hipStream_t s);
hipError_t launch_pos_select(const int* qd, int ni, int lo, int end, int* flags, int* offs, int* sel,
                             void* temp, size_t temp_bytes, hipStream_t s);
hipError_t launch_pos_gather(const int* sel, int m, const unsigned* dchrom, const int4* drec, const int2* dgate,
                             const int* lmap, unsigned* fdchrom, int4* fdrec, int2* fdgate, hipStream_t s);
hipError_t launch_chrom_filter(const unsigned* dchrom, const int4* drec, const int2* dgate, const int* lmap, int ni,
                               unsigned* fdchrom, int4* fdrec, int2* fdgate, int* flags, int* offs, void* temp,
                               size_t temp_bytes, hipStream_t s);


// ---- upload (upload.hip): fslr_set_reads' validation and packing on the device ----------------
enum UploadErr { kUpErrChrom = 1, kUpErrCoord = 2, kUpErrDataPos = 6 };
constexpr int kUpHistLds = 4096;      // chromosomes counted in LDS (more: global atomics)
struct UploadArgs {
  // the caller's columns, copied as they are
  const int *off, *qlen2, *nal, *chrom, *start, *end, *thr, *dp;   // dp null: no data order
  int n, ni, n_chroms;
  bool reads_ok;                      // read_off passed the host checks (k_up_reads / k_up_data may run)
  // outputs
  int4* iv;
  int4* rmeta;
  unsigned char* rlen8;
  unsigned* dch;
  int4* drc;
  int2* dgt;
  int* inv;                           // [ni] scratch
  unsigned long long* chrom_cnt;      // [n_chroms], zeroed by the caller
  unsigned long long* err;            // [2] first failure (index << 3 | code): columns, data order; ~0 by the caller
};
hipError_t launch_upload_pack(const UploadArgs& a, hipStream_t s);

// ---- rows -> the clustering input (rows.hip): fslr_set_reads_rows ------------------------------
enum RowsErr { kRowsErrOrder = 1, kRowsErrCode = 2, kRowsErrChrom = 4, kRowsErrCoord = 8, kRowsErrNal = 16,
               kRowsErrQlen = 32 };
struct RowsWork {
  // the uploaded fillings' columns [n_rows] (file order)
  const long long *chrom, *start, *end, *aln, *qcode, *nal, *qlen2;
  // the data list and the ranks
  int* ord32;                          // [n_rows] order as int32
  unsigned char* flag;                 // [n_rows] keep flag of each data position
  int* sel;                            // [n_rows] the data list: rows in data order
  int* nsel;                           // [1] its length
  int* first;                          // [n_codes] first data position of each qname code
  int* f;                              // [m] 1 at a qname's first position
  int* fscan;                          // [m] their exclusive scan: the read rank
  int *key, *val, *key_s, *perm;       // [m] the grouping sort (rank, data position)
  long long* code_of_rank;             // [m] qname code of each rank
  // the CSR columns
  int* off;                            // [m + 1] read offsets
  int *ch_raw, *st32, *en32, *dp;      // [m] chromosome number, start, end, data position
  long long* aln_k;                    // [m] aln_size (threshold folds)
  int *q2, *nal32;                     // [m] per read
  int* present;                        // [n_cids] chromosomes present
  int* stat;                           // [4] max read length, n_alignments varies, general thresholds, aln 0
  int* err;                            // [1] RowsErr bits
  void* temp;
  size_t temp_bytes;
};
hipError_t rows_rank(const RowsWork& w, long long n_rows, long long n_codes, const long long* order,
                     const unsigned char* keep, long long out[2], hipStream_t s);
size_t rows_temp_bytes(long long n, hipStream_t s);
hipError_t rows_csr(const RowsWork& w, int m, int n_reads, long long n_cids, hipStream_t s);
hipError_t rows_fold(const long long* aln_k, int ni, double p, const int* ch_raw, const int* dmap, int* thr, int* ch,
                     int* stat, hipStream_t s);
hipError_t rows_zero_flags(const int* thr, int ni, unsigned char* z, hipStream_t s);

// ---- components (components.hip) ---------------------------------------------------------
hipError_t launch_uf_init(int* parent, int n, hipStream_t s);
// counters[0, nc), err[0, ne) and fwd[0, n) to zero in one launch (start of a query)
hipError_t launch_query_reset(unsigned long long* counters, int nc, int* err, int ne, int* fwd, int* parent, int n,
                              hipStream_t s);
// count > cap (edges were lost) sets err[kErrOverflow]
hipError_t launch_uf_edges(int* parent, const int2* edges, const unsigned long long* count, long long cap, int* err,
                           hipStream_t s);
hipError_t launch_uf_unions(int* parent, const int2* edges, const unsigned long long* count, long long cap, int* err,
                            hipStream_t s);
// src == nullptr: src[k] = k mod period
hipError_t launch_uf_pairs(int* parent, const int* src, const int* dst, long long n, int period, hipStream_t s);
hipError_t launch_uf_finalize(int* parent, int n, hipStream_t s);
hipError_t launch_uf_pair_list(int* parent, const int2* pairs, long long n, hipStream_t s);
// (x, parent[x]) for every x of a finalized forest with parent[x] != x, in x order; *cnt = their count;
// bcnt: [1024] scratch
// the finalized forest's (read, root) pairs in read order (finalizes parent on the way); *cnt = their count
hipError_t launch_forest_pairs(int* parent, int n, int2* out, unsigned long long* cnt, int* bcnt, hipStream_t s);
// union of k and vals[w * stride + k] for k < n, w < blocks
hipError_t launch_uf_strided(int* parent, const int* vals, long long blocks, int n, long long stride, hipStream_t s);
hipError_t launch_copy_edges(const int2* edges, const unsigned long long* count, long long cap, int2* out,
                             long long n_pad, hipStream_t s);

inline int grid_for(long long n, int block = 256, int cap = 256 * 16) {
  long long g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<int>(g);
}

}  // namespace fslr
