// ctx.hpp — the context behind the C ABI's opaque fslr_ctx (internal to libfslr_hip.so):
// HBM buffers, stream, the last query's parameters, error text.  Shared by capi.hip and cap.hip.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "fslr_hip.h"
#include "kernels.hpp"

struct fslr_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::string err;
  int64_t n = 0, ni = 0;
  int n_chroms = 0;
  int thr_mode = 0;
  bool reads_set = false, index_built = false, have_data_pos = false;
  // parent is the identity taken down by the last sweep query's edges (SweepArgs::parent): the next
  // fslr_components / fslr_local_forest runs only the unions; anything else that writes the edges or the
  // parents clears it
  bool hooked = false;
  bool index_full = false;                 // the walk engine's index parts exist (qpos, backward ranges)
  bool bwd_ranges = false;                 // backward scan ranges exist (the cap replay's hits; no qpos)
  bool index_lean = false;                 // lean scatter (no data -> sorted map; `vals` holds the ends)
  bool lean_keys = false;                  // a lean index's (chrom, end) keys were made (k_endkey)
  int built_n_chroms = 0;                  // chromosomes of the built index (filtered: the owned ones)
  // multi-GPU sweep: the index covers the chromosomes of a filter (fslr_set_chrom_filter)
  bool filter_active = false;
  int n_chroms_f = 0;                       // chromosomes the filter keeps (numbered 0 .. n_chroms_f - 1)
  int* fmap = nullptr;                      // [n_chroms] its local number, -1 = another rank's
  int fmap_cap = 0;
  int64_t ni_idx = 0;                       // positions of the index (ni, or the filtered count)
  std::vector<int64_t> chrom_counts;        // intervals per chromosome (set_reads)
  unsigned* fdchrom = nullptr;              // the filtered data-order arrays
  int4* fdrec = nullptr;
  int2* fdgate = nullptr;
  int64_t f_cap = 0;
  int2* crange_f = nullptr;                 // [n_chroms_f] chromosome ranges of the filtered index
  int64_t crange_f_cap = 0;
  // the position split (fslr_set_position_filter): the index holds the sorted positions [pf_lo, pf_end)
  // of the full index (pf_on), the sweep queries [pf_lo, pf_hi); the selection is kept (pf_set) so
  // fslr_use_position_filter re-activates it after a chromosome filter
  bool pf_set = false, pf_on = false;
  int64_t pf_lo = 0, pf_hi = 0, pf_end = 0;
  uint64_t pf_gen = 0;                      // reads_gen of the selection
  uint64_t pf_thr_gen = 0;                  // thr_gen of the plan (its halo covers those thresholds' windows)
  uint64_t thr_gen = 0;                     // bumped whenever the thresholds change in place
  int* pf_sel = nullptr;                    // [pf_end - pf_lo] their data positions, ascending
  int64_t pf_sel_cap = 0;
  int* pf_lmap = nullptr;                   // [n_chroms] chromosome -> the range's own numbering, -1
  int64_t pf_lmap_cap = 0;
  std::vector<int2> pf_cr;                  // the range's chromosome ranges (local positions)
  long long* pf_cost = nullptr;             // [2 x tiles] fslr_position_costs scratch
  int64_t pf_cost_cap = 0;
  uint64_t reads_gen = 0;                   // bumped by every set_reads
  int* grp = nullptr;                       // [grp_ints()] grouping sort: bucket counts / offsets
  long long* part_cnt = nullptr;            // partition scratch: per (destination, block) counts + offsets
  // the last synchronous fslr_sweep_partition (fslr_sweep_partition_repeat replays it without a readback)
  uint64_t pt_gen = 0;
  double pt_q = 0, pt_nc = 0;
  std::vector<int> pt_umax;
  int pt_ndest = 0, pt_shift = 0;
  int64_t pt_sum = 0;
  std::vector<long long> pt_counts;
  int shard = 0, n_shards = 1;             // fslr_set_shard: A-side index data for this shard only
  int built_shard = 0, built_n_shards = 1;
  // device buffers
  int4* rmeta = nullptr;
  unsigned char* rlen8 = nullptr;  // [N] interval count per read (the pair stage's L lookups)
  int4* iv = nullptr;
  int* qpos = nullptr;       // [NI] CSR interval -> its position in the sorted index
  int2* rng_s = nullptr;     // [NI] sorted position -> {n_fwd, bwd_begin}
  int* swin = nullptr;       // [NI] sorted position -> the sweep's forward window (<= n_fwd)
  int4* idx4 = nullptr;
  int2* idx_gate = nullptr;
  unsigned long long* defer = nullptr;
  int64_t defer_cap = 0;
  int* data_pos = nullptr;
  unsigned* dchrom = nullptr;    // data order (start-sorted `data` list): chromosome
  int4* drec = nullptr;          // data order: {start, end, thr, read << 6 | j}
  int2* dgate = nullptr;         // data order: the owning read's gate word {qlen2, nal | L << 24 | haz << 31}
  int* chist = nullptr;          // index build scratch: per-chromosome counts per 1024-position sub-tile
  int* s_start = nullptr;
  int2* crange = nullptr;
  unsigned long long* keys = nullptr;
  unsigned long long* keys2 = nullptr;
  int* vals = nullptr;
  int* vals2 = nullptr;
  unsigned long long* endkey = nullptr;
  unsigned long long* pmaxkey = nullptr;   // per 256-position tile: max (chrom, end) key, then its scan
  void* temp = nullptr;
  size_t temp_bytes = 0;
  int* umax = nullptr;     // [FSLR_MAX_L] derived from the pass table
  int4* lbounds = nullptr; // [N] per query read: exact integer ranges of the length gate
  int64_t lb_gen = -1;     // lbounds hold every read's ranges for this input generation and cuts
  double lb_q = 0.0, lb_n = 0.0;
  int2* edges = nullptr;
  unsigned short* edge_iu = nullptr;
  int64_t edge_cap = 0;
  int* fwd = nullptr;
  int* heavy = nullptr;      // [N] reads handed to the partitioned pair-kernel launch
  int* parent = nullptr;
  int* upl = nullptr;                        // fslr_set_reads: the caller's columns as copied (upload.hip)
  int64_t upl_cap = 0;
  unsigned long long* upl64 = nullptr;       // [n_chroms + 2]: intervals per chromosome, first failures
  int64_t upl64_cap = 0;
  int2* forest = nullptr;                    // [n] the local forest's (read, root) pairs (fslr_local_forest)
  unsigned long long* forest_cnt = nullptr;  // [1] their count (device)
  int* forest_blk = nullptr;                 // [1024] compaction scratch
  unsigned long long* counters = nullptr;
  unsigned long long* wstat = nullptr;       // [wstat_waves x kWStride] per-wave statistics of the pair kernel
  int wstat_waves = 0;
  unsigned long long* diag = nullptr;        // FSLR_SECTION_PROF builds: per-read timing of the pair kernel
  int* errw = nullptr;     // [0..2] error, [3] max_fwd, ... then the ZeroDivisionError pair list (kernels.hpp)
  // fslr_rows_upload / fslr_set_reads_rows (rows.hip): the uploaded rows and the CSR the device made
  long long* rows_col = nullptr;    // [7 x rows_cap] chrom, start, end, aln, qcode, nal, qlen2
  int64_t rows_cap = 0, rows_n = 0, rows_codes = 0, rows_cids = 0;
  long long* rows_ord = nullptr;    // [rows_cap] the start order
  unsigned char* rows_keep = nullptr;
  int* rows_int = nullptr;          // [16 x rows_cap + ...] the build's int scratch and CSR columns
  int64_t rows_int_cap = 0;
  long long* rows_l = nullptr;      // [2 x rows_cap] aln in CSR order, qname code of each rank
  void* rows_temp = nullptr;
  size_t rows_temp_bytes = 0;
  bool rows_set = false;            // the reads came from fslr_set_reads_rows (fslr_get_csr, fold)
  std::vector<int> rows_dmap;       // chromosome number -> dense id, and its inverse
  std::vector<int64_t> rows_cid;
  int zd_cap = 0;          // capacity of that list (pairs)
  bool zd_lost = false;    // this series' ZeroDivisionError list overflowed (a zd_host query; grown since)
  bool zd_host = false;    // the last query's ZeroDivisionError pairs are decided by the caller (a partition,
                           // an evaluation or a long-read query: the edge cap's binding is known there)
  int q_thr = 0;           // the last query's edge_threshold (fslr_read_stats: does the cap bind?)
  // position-sweep engine (sweep.hip)
  long long* sw_tile = nullptr;             // [4 x tiles]: entries, their scan, pair tests, their scan
  long long* sw_total = nullptr;            // [4] pinned host memory, device-mapped: entries, bound, flags
  long long* sw_total_dev = nullptr;        // its device address
  unsigned long long* ent_ub = nullptr;     // one-pass sweep output at upper-bound tile slots
  int64_t ent_ub_cap = 0;
  int64_t sw_tiles = 0;
  unsigned long long* sw_wstat = nullptr;   // per-wave statistics slots of the sweep kernels
  int* sw_wlo = nullptr;                    // [waves + 1] the one-pass sweep's first tile per wave
  int sw_wstat_waves = 0;
  hipEvent_t sw_ev[5] = {};                 // (profiling) count | scan | emit | sort | pairs
  bool sw_ev_rec = false;
  unsigned long long* ent = nullptr;        // match entries, tile order
  unsigned long long* ent_sorted = nullptr; // grouped by read A
  int64_t ent_cap = 0;
  void* sweep_temp = nullptr;
  size_t sweep_temp_bytes = 0;
  bool any_zero_aln = false;                // an aln_size == 0 interval: the walk engine replays it
  // sync-free repeat query: a full one-pass sweep query on unchanged input (same reads, thresholds,
  // filter, parameters) has the previous query's entry count, so the host need not read it back
  long long* idx_tt = nullptr;              // the lean index build's per-tile window sums (SweepArgs::tile_tests)
  int64_t idx_tt_cap = 0;
  bool idx_tt_valid = false;
  bool reuse = true;                        // fslr_set_query_reuse: repeat queries keep what they can
  uint64_t input_gen = 1;                   // bumped by set_reads / set_thresholds / set_chrom_filter / set_shard
  uint64_t sw_prev_gen = 0;                 // input_gen of the last synchronous sweep query (0: none)
  double sw_prev_q = 0, sw_prev_nc = 0;
  std::vector<int> sw_prev_umax;
  int64_t sw_prev_a0 = -1, sw_prev_a1 = -1, sw_prev_n = 0;
  bool sw_fast_used = false;                // the last query ran sync-free
  int last_engine = FSLR_ENGINE_WALK;
  int* thr_tmp = nullptr;
  int64_t cap_n = 0, cap_ni = 0, cap_chroms = 0;
  std::vector<int> umax_host, umax_dev_copy;   // dev copy: what c->umax holds
  std::vector<unsigned char> aln_zero_host;   // per CSR interval: FSLR_THR_ZERO_ALN at set_reads
  int ablate = 0;
  // the last query (fslr_query / fslr_query_shard): what fslr_apply_edge_cap replays
  bool last_full = false;                // covered every read [0, n) with one shard
  double last_qcut = 0.0, last_ncut = 0.0;
  fslr_cap_stats cap_stats = {};
  bool edges_global = false;             // every E* edge is on this context (fslr_cap_install_edges)
  bool cap_gmode = false;                // gathered E* rows installed for the sharded replay (fslr_cap_install_pairs)
  struct CapWork* capw = nullptr;        // the device cap replay's buffers (cap.hip)
  // reads of more than FSLR_MAX_L intervals (long.hip): the virtual-read map and the long-pair stage
  bool lg_set = false;
  // fslr_set_reads_any: virtual interval k is real interval lg_perm[k] (thresholds arrive in the real
  // CSR's order and are permuted); empty when the reads were uploaded as they are
  std::vector<int> lg_perm;
  int64_t lg_n_real = 0, lg_n_edges = 0;
  int lg_n_umax = 0;
  int* lg_vreal = nullptr;                  // [virtual reads] real read
  int* lg_vbase = nullptr;                  // [virtual reads] index of its first interval in the real read
  int* lg_rlen = nullptr;                   // [real reads] interval count
  int* lg_umax = nullptr;                   // [n_umax] largest passing U per I (cluster.py:216-219)
  int* lg_off2 = nullptr;                   // [real reads] CSR offset of a long read's intervals beyond FSLR_MAX_L
  unsigned long long *lg_pk = nullptr, *lg_ij = nullptr, *lg_pk2 = nullptr, *lg_ij2 = nullptr;
  int64_t lg_cap = 0;
  unsigned long long* lg_cnt = nullptr;     // [4] short entries, long entries, long edges, run count
  unsigned long long* lg_uniq = nullptr;    // per pair run: (ra << 25 | rb)
  int *lg_rlen_run = nullptr, *lg_roff = nullptr;
  long long *lg_words = nullptr, *lg_woff = nullptr;
  int64_t lg_run_cap = 0;
  unsigned* lg_bits = nullptr;              // used-column bitmaps of the first-fit
  int64_t lg_bits_cap = 0;
  int4* lg_edges = nullptr;                 // (ra, rb, I, U)
  int64_t lg_edge_cap = 0;
  unsigned char* lg_temp = nullptr;
  unsigned long long *lg_ent = nullptr, *lg_short = nullptr;   // the sweep's entries; the short-pair ones
  int64_t lg_ent_cap = 0, lg_short_cap = 0;
  size_t lg_temp_bytes = 0;
  // profiling
  bool profiling = false;                  // the pair-kernel event ring (fslr_set_profiling 1 or 2)
  bool prof_phases = false;                // per-phase events too (fslr_set_profiling 1)
  hipEvent_t ev[8] = {};
  // (profiling) a ring of event pairs around the main pair-kernel launch of the last kKernRing queries
  static constexpr int kKernRing = 256;
  std::vector<hipEvent_t> kev;
  int64_t n_kern = 0;
  std::vector<hipEvent_t> kev2;            // the same ring around the sweep's pair-stage kernel
  int64_t n_kern2 = 0;
  bool ev_ok = false;
  bool t_index_rec = false, t_query_rec = false, t_comp_rec = false, t_kernel_rec = false;
};

// frees the long-read stage's buffers (long.hip)
void fslr_long_free(fslr_ctx* c);
// frees the cap replay's buffers (cap.hip)
void fslr_cap_free(fslr_ctx* c);

namespace fslr {

// builds the walk engine's index parts of a sweep-only index (capi.hip); no-op when present
int ensure_walk_index(fslr_ctx* c);
// {edge count, error code, max forward degree} of the last query through pinned memory; syncs
int peek_counts(fslr_ctx* c, long long out[4]);   // edges, err code, max_fwd, ZeroDivisionError pairs
// the backward scan ranges of the (possibly chromosome-filtered) index, without the CSR map (capi.hip)
int ensure_bwd_ranges(fslr_ctx* c);


inline int fail(fslr_ctx* c, int code, const std::string& msg) {
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
  if (*p) {
    (void)hipFree(*p);
    *p = nullptr;
  }
  if (count == 0) count = 1;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
  if (e != hipSuccess) return fail(c, FSLR_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  return FSLR_OK;
}

}  // namespace fslr
