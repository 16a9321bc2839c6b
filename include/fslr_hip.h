/*
 * fslr_hip.h — C ABI of the MI355X (gfx950) clustering hot path of fslr.
 *
 * The reference (kcleal/fslr, pure Python) has no native FFI for this path; its
 * hot path is the Python driver in fslr/cluster.py calling the third-party
 * native interval index `superintervals`.  Each entry point below replaces one
 * reference interface (file:line into /root/reference/fslr/):
 *
 *   fslr_set_reads        cluster.py:189-191  the per-read interval lists
 *                         (`query_intervals`) handed to the driver, packed CSR
 *   fslr_build_index      cluster.py:124-130  build_interval_trees (per-chrom
 *                         superintervals.IntervalMap add/build)
 *   fslr_query            cluster.py:187-227  query_interval_trees: candidate
 *                         search (:201), seen-set (:205-208),
 *                         different_lengths_or_alignments (:178-183),
 *                         overall_jaccard_similarity (:140-170),
 *                         calculate_overlap (:133-136), cutoff lookup (:218-219)
 *   fslr_query_shard      the same over one multi-GPU shard of the query reads
 *   fslr_components       cluster.py:230-234  get_subgraphs (networkx
 *                         connected_components)
 *   fslr_set_chrom_filter,
 *   fslr_sweep_partition,
 *   fslr_sweep_evaluate   cluster.py:187-227 split over ranks by chromosome (the sweep engine's
 *                         multi-GPU path)
 *   fslr_union_pairs      (multi-GPU merge of per-shard component labels; no
 *                         reference counterpart — the reference is single-process)
 *   fslr_copy_edges_device, fslr_components_from_pairs, fslr_local_forest,
 *   fslr_copy_forest_pairs
 *                         (multi-GPU merge of the ranks' gathered local forests: get_subgraphs,
 *                         cluster.py:230-234, over the union of the ranks' edges)
 *   fslr_copy_edges_iu_device,
 *   fslr_cap_install_edges,
 *   fslr_cap_local,
 *   fslr_cap_copy_local,
 *   fslr_cap_replay      cluster.py:197-224 the edge cap (:223-224) replayed on a rank that holds every
 *                         E* edge but indexes only its chromosomes (multi-GPU)
 *   fslr_cap_install_pairs, fslr_cap_sizes, fslr_cap_dep_local, fslr_cap_shard_plan,
 *   fslr_cap_shard_pack, fslr_cap_replay_shard, fslr_cap_copy_changes,
 *   fslr_cap_apply_changes, fslr_cap_bwd_counts, fslr_cap_restrict, fslr_cap_copy_restricted,
 *   fslr_cap_install_restricted
 *                         cluster.py:197-224 the same loops sharded over the ranks by the components of
 *                         the candidates' hit graph (multi-GPU)
 *   fslr_set_long_reads,
 *   fslr_long_query,
 *   fslr_get_long_edges   cluster.py:140-170 overall_jaccard_similarity for reads of more than
 *                         FSLR_MAX_L intervals (the reference has no limit; its l2_comparisons
 *                         scratch holds 100000 columns, :195)
 *
 * Conventions: plain C types, caller-owned host arrays, library-owned device
 * memory behind an opaque context.  Every function returns FSLR_OK (0) or an
 * error code; fslr_last_error() gives the message.  Calls on one context are
 * not re-entrant; different contexts are independent.
 *
 * Semantics the caller folds in on the host (so the device does integer work
 * only, bit-exact to the reference's IEEE-double comparisons):
 *   iv_thr[k]   overlap threshold of interval k for `calculate_overlap >= overlap`
 *               (cluster.py:133-136): with o = max(0, min(e1,e2) - max(s1,s2)),
 *               interval k accepts o iff  thr >= 0 ? o >= thr : o <= ~thr.
 *               FSLR_THR_ZERO_ALN marks aln_size == 0 (the reference raises
 *               ZeroDivisionError when such an interval is compared).
 *   pass_table  [FSLR_MAX_L][2*FSLR_MAX_L] bytes: pass_table[(I-1)*2*FSLR_MAX_L + (U-1)]
 *               = (I/U >= cutoff(I)) evaluated in Python floats (cluster.py:218-219).
 *   qlen_cut, nal_cut = 1 - qlen_diff, 1 - n_alignment_diff (Python floats);
 *               the device evaluates fl(min/max) >= cut in IEEE double, as Python does,
 *               once per query read to get the exact integer range of partner values that
 *               pass (the ratio test is monotone on each side of the read's own value).
 */
#ifndef FSLR_HIP_H
#define FSLR_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FSLR_ABI_VERSION 21
#define FSLR_MAX_L 64                /* max intervals per read (bitmask width) */
#define FSLR_MAX_READS (1 << 25)     /* read rank packs into bits 6..30 of the index record */
#define FSLR_THR_ZERO_ALN INT32_MIN

enum {
    FSLR_OK = 0,
    FSLR_ERR_ZERO_DIVISION = 1,   /* the reference would raise ZeroDivisionError */
    FSLR_ERR_INVALID = 2,         /* bad arguments / unsupported input */
    FSLR_ERR_HIP = 3,             /* HIP runtime failure */
    FSLR_ERR_NOMEM = 4,
    FSLR_ERR_STATE = 5            /* call order violated (e.g. query before index) */
};

typedef struct fslr_ctx fslr_ctx;

/* Rank-ordered CSR of the prepared intervals.  Reads are in first-appearance
 * order of the start-sorted `data` list; a read's intervals are in `data` order
 * (cluster.py:189-191).  All coordinates must lie in [0, 2^30). */
typedef struct {
    int64_t n_reads;
    int64_t n_intervals;
    int32_t n_chroms;              /* iv_chrom values lie in [0, n_chroms) */
    const int32_t *read_off;       /* [n_reads+1] */
    const int32_t *read_qlen2;     /* [n_reads]  keep_fillings qlen2 (cluster.py:26-29) */
    const int32_t *read_nal;       /* [n_reads]  n_alignments, in [0, 2^24) */
    const int32_t *iv_chrom;       /* [n_intervals] */
    const int32_t *iv_start;       /* min(rstart, rend)  (cluster.py:111) */
    const int32_t *iv_end;         /* max(rstart, rend)  (cluster.py:112) */
    const int32_t *iv_thr;         /* folded overlap threshold, see above */
    const int32_t *iv_data_pos;    /* optional (NULL): position of each interval in the start-sorted
                                      `data` list (cluster.py:114).  With it the index build is one
                                      stable pass on chromosome instead of a (chrom, start) sort. */
} fslr_reads;

/* fslr_params.flags & 3: the pair engine of fslr_query.  Both compute the same edge set E*,
 * forward degrees and ZeroDivisionError; they differ in what they count (fslr_query_stats).
 *   WALK   one wavefront per query read walks its intervals' hits and dedupes its partners
 *          (the reference's seen-set): counts evaluated_pairs and jaccard_evals.  Any input.
 *   SWEEP  one forward sweep over the sorted index meets every overlapping interval pair once;
 *          match entries are grouped per read and the greedy runs per pair (sweep.hip).  Needs
 *          overlap thresholds >= 1 (overlap > 0) and no aln_size == 0 interval; does not count
 *          evaluated_pairs / jaccard_evals (reported as -1).
 *   AUTO   SWEEP when the input allows it and the query covers all reads, else WALK. */
#define FSLR_ENGINE_AUTO 0
#define FSLR_ENGINE_WALK 1
#define FSLR_ENGINE_SWEEP 2

typedef struct {
    double qlen_cut;               /* 1 - qlen_diff */
    double nal_cut;                /* 1 - n_alignment_diff */
    const uint8_t *pass_table;     /* host pointer, FSLR_MAX_L * 2*FSLR_MAX_L bytes */
    int32_t edge_threshold;        /* main.py:221 (10); reported against, see max_fwd */
    int32_t flags;                 /* FSLR_ENGINE_* in bits 0..1; other bits reserved, 0 */
} fslr_params;

typedef struct {
    int64_t evaluated_pairs;       /* unique candidate read pairs (the reference's seen-set size) */
    int64_t jaccard_evals;         /* pairs that passed different_lengths_or_alignments */
    int64_t candidates;            /* WALK: interval-level index hits (before pair dedupe); SWEEP: overlapping
                                      interval pairs of two different reads */
    int64_t n_edges;               /* edges of E* (may exceed edge capacity, see fslr_reserve_edges) */
    int32_t max_fwd;               /* max over reads of forward (higher-rank) edges */
    int32_t error;                 /* FSLR_OK or FSLR_ERR_ZERO_DIVISION */
    int32_t err_a, err_b;          /* read ranks of the pair that raised */
    int64_t algo_bytes;            /* sum over evaluated pairs of 16*(L_A+L_B)+32 */
    int64_t overflow_candidates;   /* candidates of reads past the per-wave partner-set limit (witness path) */
    int64_t gather_pairs;          /* pairs evaluated by gathering B's intervals (general thresholds,
                                      aln_size==0 replay, match-list overflow) */
    int64_t match_entries;         /* matching interval pairs recorded in the per-read match lists (SWEEP:
                                      of read pairs that pass different_lengths_or_alignments) */
    int64_t matched_pairs;         /* read pairs with at least one matching interval pair (SWEEP: gate-passing) */
    int64_t deferred;              /* entries on the deferred (gather-evaluated) list */
    int64_t deferred_capacity;     /* its capacity; deferred > capacity ⇒ FSLR_ERR_STATE, reserve + rerun */
    int64_t edge_capacity;         /* edge buffer capacity; n_edges > capacity ⇒ reserve + rerun */
    int64_t walked_records;        /* index records the pair kernels walked (every partner-partition pass) */
    int32_t engine;                /* FSLR_ENGINE_WALK or FSLR_ENGINE_SWEEP: the engine that ran */
    int32_t overflow_flags;        /* 1 deferred list, 2 edge buffer, 4 sweep partner table (rerun with WALK),
                                      8 | 16 sweep entry buffers (rerun) */
    int64_t pair_tests;            /* SWEEP: overlapping interval pairs tested (each pair once) */
    int64_t entry_capacity;        /* SWEEP: match-entry buffer (grown automatically) */
    int64_t zd_pairs;              /* read pairs whose evaluation raises ZeroDivisionError (both qlen2 or both
                                      n_alignments 0 at the length gate, cluster.py:178-183; an aln_size == 0
                                      interval met by first-fit, :133-136).  The reference raises only if a loop
                                      reaches one: always when the edge cap does not bind (max_fwd <=
                                      edge_threshold: fslr_read_stats returns FSLR_ERR_ZERO_DIVISION after
                                      fslr_query), otherwise fslr_apply_edge_cap decides.  After
                                      fslr_sweep_partition / fslr_sweep_evaluate / fslr_long_query /
                                      fslr_long_pairs the caller decides (the binding may be known only over
                                      every rank); overflow_flags 64: the list grew, rerun the query */
} fslr_query_stats;

typedef struct {
    float index_ms;                /* fslr_build_index device time */
    float query_ms;                /* fslr_query: pair kernel device time (events around the launch) */
    float components_ms;           /* union-find device time */
    float total_ms;                /* first to last event of the last fslr_run/individual calls */
    float pair_kernel_ms;          /* the main pair-kernel launch alone (WALK: query_kernel; SWEEP: the count pass) */
    float sweep_count_ms;          /* SWEEP phases of the last query: count pass (+ statistics), */
    float sweep_emit_ms;           /*   emit pass, */
    float sweep_sort_ms;           /*   grouping sort, */
    float sweep_pairs_ms;          /*   per-read pair evaluation */
} fslr_timings;

/* The reference's per-query-read edge cap (cluster.py:223-224), see fslr_apply_edge_cap. */
typedef struct {
    int32_t applied;               /* 1: the cap bound (max forward degree > edge_threshold) and was replayed */
    int32_t max_fwd;               /* max over reads of the edges formed in the read's own loop */
    int64_t candidates;            /* reads whose loop could reach the cap (replayed) */
    int64_t capped;                /* reads whose loop reached it (left hits unvisited) */
    int64_t hits;                  /* index hits of the replayed loops */
    int64_t pairs;                 /* distinct pairs of those hits, evaluated on the device */
    int64_t dropped;               /* E* edges that no loop reached (absent from the reference graph) */
    int64_t backward;              /* edges formed in the higher-rank read's loop */
} fslr_cap_stats;

int  fslr_abi_version(void);
/* first 16 hex digits of the sha256 of the kernel sources the library was built from (the sorted
 * .hip and .hpp files of fslr_amd/csrc, then this header): a binding can refuse a stale build */
const char *fslr_source_hash(void);
const char *fslr_last_error(const fslr_ctx *ctx);

/* device: HIP ordinal; stream: hipStream_t to launch on (NULL = the library creates one). */
int  fslr_ctx_create(int device, void *stream, fslr_ctx **out);
void fslr_ctx_destroy(fslr_ctx *ctx);
int  fslr_set_profiling(fslr_ctx *ctx, int enable);     /* 1: hipEvents per phase + around the pair kernel;
                                                           2: around the pair kernel only (fewer stream
                                                           markers in a timed loop); 0: off */
/* enable (the default) = a sweep query on unchanged input (reads, thresholds, filter, range, cuts) repeats
 * the last synchronous one: it keeps the length-gate ranges and its entry count stays on the device (no
 * mid-query readback).  0 = every query does the full work, as a single query on new input does. */
int  fslr_set_query_reuse(fslr_ctx *ctx, int enable);

/* Copy the CSR (host pointers) into context-owned HBM buffers (H2D). */
int  fslr_set_reads(fslr_ctx *ctx, const fslr_reads *reads);
/* The clustering input from rows (the columnar CLI path).  fslr_rows_upload copies
 * keep_fillings' rows (cluster.py:14-31), file order, as int64 columns (syncs; a caller may run it while
 * it sorts the starts).  fslr_set_reads_rows takes prepare_data's start order of those rows (the
 * argsort of `start`, cluster.py:114) and, optionally, mask_sequences2's keep flag per row
 * (cluster.py:89-106); on the device it forms the `data` list, ranks the reads by first appearance in
 * it and groups each read's intervals in data order (cluster.py:189-191), numbers the chromosomes
 * present densely in ascending order, folds the overlap thresholds for `overlap` (fslr_reads iv_thr)
 * and sets the reads as fslr_set_reads with iv_data_pos would.  A read of more than FSLR_MAX_L
 * intervals sets nothing: FSLR_ERR_INVALID with info->max_len > FSLR_MAX_L (use fslr_set_reads_any).
 * fslr_get_read_codes: the qname code of each read rank.  fslr_get_csr: the CSR the device made (as
 * fslr_reads with its folded thresholds, plus aln_size per interval, the data position of each interval and the chromosome
 * number of each dense id; NULL outputs are skipped).  fslr_fold_thresholds: the thresholds of another
 * overlap, folded on the device (as fslr_set_thresholds). */
typedef struct {
    int64_t n_rows;                /* fillings */
    int64_t n_codes;               /* qcode values lie in [0, n_codes) */
    int64_t n_chrom_ids;           /* chrom values lie in [0, n_chrom_ids) */
    const int64_t *chrom;          /* rename_chromosomes' number (cluster.py:34-43) */
    const int64_t *start, *end;    /* min / max of rstart, rend (cluster.py:111-112) */
    const int64_t *aln;            /* aln_size */
    const int64_t *qcode;          /* the row's qname code */
    const int64_t *nal;            /* n_alignments */
    const int64_t *qlen2;          /* the row's read's keep_fillings qlen2 */
} fslr_rows;
typedef struct {
    int64_t n_reads, n_intervals;
    int32_t n_chroms;              /* chromosomes present (dense ids) */
    int32_t max_len;               /* longest read */
    int32_t nal_varies;            /* n_alignments differs between intervals of a read */
    int32_t general_thresholds;    /* a threshold below 1 (overlap <= 0): the sweep does not apply */
    int32_t any_zero_aln;          /* an aln_size == 0 interval */
    int32_t pad;
} fslr_rows_info;
int  fslr_rows_upload(fslr_ctx *ctx, const fslr_rows *rows);
int  fslr_set_reads_rows(fslr_ctx *ctx, const int64_t *order, const uint8_t *keep, double overlap,
                         fslr_rows_info *info);
int  fslr_get_read_codes(fslr_ctx *ctx, int64_t *codes);
int  fslr_get_csr(fslr_ctx *ctx, int32_t *read_off, int32_t *read_qlen2, int32_t *read_nal, int32_t *iv_chrom,
                  int32_t *iv_start, int32_t *iv_end, int64_t *iv_aln, int32_t *iv_thr, int64_t *data_pos,
                  int64_t *chrom_ids);
int  fslr_fold_thresholds(fslr_ctx *ctx, double overlap);
/* Replace the folded overlap thresholds (iv_thr, CSR order) without re-uploading
 * or re-indexing: the index does not depend on them (calculate_overlap's
 * `percentage`, cluster.py:157, is a query-time parameter). */
int  fslr_set_thresholds(fslr_ctx *ctx, const int32_t *iv_thr);
/* Edge buffer capacity (edges of E*); grows only. */
int  fslr_reserve_edges(fslr_ctx *ctx, int64_t capacity);
/* Deferred-pair list capacity (pairs evaluated by gathering intervals); grows only. */
int  fslr_reserve_deferred(fslr_ctx *ctx, int64_t capacity);

/* Multi-GPU: build the query-side index data (positions, scan ranges) only for the reads of
 * query shard `shard` of `n_shards` (see fslr_query_shard); the walked index stays complete.
 * Takes effect at the next fslr_build_index; fslr_query then needs n_shards == 1. */
int  fslr_set_shard(fslr_ctx *ctx, int32_t shard, int32_t n_shards);
/* cluster.py:124-130 — sort intervals by (chrom, start), prefix-max of end. Async. */
int  fslr_build_index(fslr_ctx *ctx);
/* cluster.py:187-227 — all candidate pairs of query reads with rank in
 * [a_begin, a_end) against every read of higher rank.  Async; stats are read
 * with fslr_read_stats. */
int  fslr_query(fslr_ctx *ctx, const fslr_params *params, int64_t a_begin, int64_t a_end);
/* Multi-GPU query shard: the reads of rank blocks [64 k, 64 k + 64) with k % n_shards == shard
 * (balanced: low ranks have more higher-rank partners).  The shards of 0..n_shards-1 together
 * evaluate exactly the pairs of fslr_query(ctx, params, 0, n_reads).  Async. */
int  fslr_query_shard(fslr_ctx *ctx, const fslr_params *params, int32_t shard, int32_t n_shards);
/* cluster.py:197-224 — the edge cap.  The query computes E* (every candidate pair); when a read
 * has more than edge_threshold forward edges, the reference's graph depends on the order its loops
 * visit pairs.  This replays those loops exactly (search order of the superintervals stand-in the
 * golden fixtures were made with: descending (start, -end, data position)) for the reads that can
 * reach the cap, drops the E* edges no loop reaches, re-orients edges as (read whose loop formed
 * it, partner) and sets forward degrees to the edges formed per loop.  No-op (no sync beyond one
 * counter read) when the cap does not bind.  Needs the last query to be fslr_query over all reads
 * (or fslr_cap_install_edges on an unfiltered index).  The replay runs on the device: loops of
 * different components of the candidates' partner graph are independent.
 * Call between fslr_query and fslr_components.  Syncs; out may be NULL. */
int  fslr_apply_edge_cap(fslr_ctx *ctx, int32_t edge_threshold, fslr_cap_stats *out);
/* The same check without a host round trip, for a repeated query on unchanged input: the device ORs
 * (max forward degree > edge_threshold) | (a listed ZeroDivisionError pair) << 1 into a sticky word (async);
 * fslr_edge_cap_deferred_read syncs, returns the word and clears it.  A nonzero word means a step needed
 * fslr_apply_edge_cap (or raised): its results are to be recomputed synchronously. */
int  fslr_edge_cap_deferred(fslr_ctx *ctx, int32_t edge_threshold);
int  fslr_edge_cap_deferred_read(fslr_ctx *ctx, int32_t *flags);
/* cluster.py:230-234 — union-find over the edges: label = min rank in component.  Async.  Every query
 * resets the parents to the identity; a sweep-engine query (fslr_query, fslr_sweep_evaluate) also
 * pre-hooks them as its pair kernel forms the edges, and the next fslr_components / fslr_local_forest
 * then runs only the unions (any call that rewrites the edges or the parents in between — the edge cap,
 * fslr_sort_edges, fslr_reserve_edges, an upload, fslr_union_pairs — makes it start from the identity
 * again).  Labels (fslr_get_labels) are those of the last fslr_components / fslr_local_forest /
 * fslr_components_from_pairs until the next query. */
int  fslr_components(fslr_ctx *ctx);
/* Multi-GPU sweep.  A rank indexes only the chromosomes it owns, sweeps them and
 * routes the match entries to the rank owning each pair's first read, which evaluates the pairs.
 * An interval only meets intervals of its own chromosome (cluster.py:159-160), so the first-fit
 * matching of a pair is the union of its per-chromosome matchings and the split is exact.
 *
 * fslr_set_chrom_filter: owned[n_chroms] != 0 marks the chromosomes the next fslr_build_index
 * indexes (NULL: all).  Needs iv_data_pos and n_chroms <= 64.  The filtered index serves only
 * fslr_sweep_partition (fslr_query refuses it).  Syncs.
 * fslr_sweep_partition: sweep the filtered index (every query read, the pair gates applied) and
 * write its match entries (8 bytes each, layout internal to the library) to the device buffer dst
 * grouped by destination k = (a >> block_shift) % n_dest, a = the pair's first (lower-rank) read:
 * rank blocks dealt round robin, n_dest <= 64; counts[k] = entries for k.  Syncs; FSLR_ERR_STATE if
 * sum(counts) > dst_cap (counts are still filled: grow dst and call again).  Pairs that raise
 * ZeroDivisionError are listed, not raised (fslr_query_stats zd_pairs; fslr_cap_local raises for those
 * the capped loops reach).
 * fslr_sweep_evaluate: evaluate the pairs of the n entries (a device buffer: every rank's segment
 * for this rank, concatenated in any order) into this context's edges and forward degrees.  Every
 * entry of a pair must be present, so each pair's first read belongs to one destination.  Needs only
 * fslr_set_reads.  Async; fslr_read_stats / fslr_components / fslr_get_edges follow as after
 * fslr_query. */
int  fslr_set_chrom_filter(fslr_ctx *ctx, const uint8_t *owned);
/* The position split: a rank sweeps a contiguous range of the (chrom, start)-sorted
 * positions, cut where the pair tests balance, whatever the chromosomes.
 * fslr_position_costs: after fslr_build_index over every chromosome, per tile of 64 sorted positions
 *   its pair tests (the sum of its forward counts) and the end of its forward window (max q + n_fwd(q)
 *   + 1); n_tiles = ceil(n_intervals / 64).  Syncs.
 * fslr_set_position_filter: the next fslr_build_index indexes the sorted positions [lo, end) only and
 *   fslr_sweep_partition sweeps the pairs whose lower position lies in [lo, hi); end must cover the
 *   forward windows of [lo, hi) (fslr_position_costs).  Every pair of overlapping intervals is met by
 *   the rank holding its lower position.  Needs iv_data_pos and <= 64 chromosomes.  Syncs.
 * fslr_position_entries: after fslr_build_index over every chromosome, the match entries of each
 *   tile under the query parameters p (the one-pass sweep over the full index, as fslr_query's):
 *   the per-entry work (partition, exchange, evaluation) is most of a rank's cost where pair tests
 *   rarely match.  Syncs.
 * fslr_use_position_filter: make the last position filter of these reads active again (after
 *   fslr_set_chrom_filter, which the edge cap's sharded replay lists its hits with). */
int  fslr_position_costs(fslr_ctx *ctx, int64_t *tile_tests, int64_t *tile_reach, int64_t n_tiles);
int  fslr_position_entries(fslr_ctx *ctx, const fslr_params *p, int64_t *tile_entries, int64_t n_tiles);
int  fslr_set_position_filter(fslr_ctx *ctx, int64_t lo, int64_t hi, int64_t end);
int  fslr_use_position_filter(fslr_ctx *ctx);
/* Multi-GPU edge cap (cluster.py:197-224).  The replayed loops need every E* edge
 * and every hit of the reads that can reach the cap; a rank's index holds its chromosomes' hits.
 * fslr_copy_edges_iu_device: this context's edges as int32 rows {a, b, I | U << 8, 0} into a device
 *   buffer of n_pad rows, padded with a = -1 (async).  The ranks all-gather them.
 * fslr_cap_install_edges: the n_rows gathered rows (device; a < 0 = padding) become this context's
 *   edge list and forward degrees (as after a full query).  Syncs.
 * fslr_cap_local: the replay's candidates, their intervals (*n_ti, the same on every rank) and the
 *   search-ordered hits of the intervals this rank's index holds (*n_hits).  Syncs.
 * fslr_cap_copy_local: counts[n_ti] (int32, 0 for other ranks' intervals) and hits[n_hits] (the
 *   partner reads, interval after interval) into device buffers (async).  The ranks all-gather both:
 *   counts as world x n_ti, hits padded to `pad` per rank.
 * fslr_cap_replay: replay the loops from the gathered lists and write the capped graph into this
 *   context as fslr_apply_edge_cap does (every rank gets the same graph).  Syncs; out may be NULL. */
int  fslr_copy_edges_iu_device(fslr_ctx *ctx, int32_t *dst, int64_t n_pad);
int  fslr_cap_install_edges(fslr_ctx *ctx, const int32_t *rows, int64_t n_rows);
int  fslr_cap_local(fslr_ctx *ctx, int32_t edge_threshold, int64_t *n_ti, int64_t *n_hits);
int  fslr_cap_copy_local(fslr_ctx *ctx, int32_t *counts, int32_t *hits);
int  fslr_cap_replay(fslr_ctx *ctx, const int32_t *counts, const int32_t *hits, int64_t pad, int32_t world,
                     fslr_cap_stats *out);
/* The multi-GPU edge cap sharded over the ranks (cluster.py:197-224).  Two loops of the
 * replay depend on each other only when an interval of one read hits an interval of the other, so the
 * components of that graph over the candidates T replay independently, each on one rank.
 * fslr_cap_install_pairs: n_rows gathered E* rows as int32 (a, b) pairs (device; a < 0 = padding;
 *   rank w's block is rows [w m, (w + 1) m), m = n_rows / world, in its fslr_copy_edges_device order,
 *   after fslr_sort_edges).  The rows are read in place: keep them unchanged until
 *   fslr_cap_apply_changes.
 *   This context's own edges stay its edge list; fslr_cap_local then computes the closure T over the
 *   gathered rows and lists the hits of T's intervals on this rank's chromosomes (async + syncs).
 * fslr_cap_sizes: |T|, its intervals, the local hits (after fslr_cap_local).
 * fslr_cap_dep_local: out[2 |T|] (device): out[t] = the root (smallest index) of T read t in the forest
 *   of the T-T hits on this rank's chromosomes, out[|T| + t] = its local hit count (async).
 * fslr_cap_shard_plan: gathered = the ranks' out arrays (world x 2 |T|).  Unions the forests, assigns the
 *   components to ranks by cost (hits; largest first onto the least-loaded rank: the same on every
 *   rank) and groups the local lists by destination.  sizes[d] = T-intervals sent to rank d (the same on
 *   every rank), sizes[world + d] = local hits sent to rank d.  Syncs.
 * fslr_cap_shard_pack: counts (sum sizes[0 .. world) int32) and hits (sum sizes[world ..)) for one
 *   all_to_all each, destination-major (async).  The rank receives world x sizes[rank] counts.
 * fslr_cap_replay_shard: replays the loops of this rank's components from the received counts and hits
 *   (source-major) and lists the gathered rows it decides that the lower read's loop does not form:
 *   *n_changes of them; part (may be NULL): its candidates, capped loops, hits and slots.  Syncs.
 * fslr_cap_copy_changes: the changes (int32 row << 2 | who, who 1 = formed in b's loop, 2 = dropped)
 *   padded with -1 to n_pad (device, async).  The ranks all-gather them.
 * fslr_cap_apply_changes: every rank's changes: this context keeps its own capped edges (re-oriented as
 *   (former, partner)) and their formers' counts (fwd), errw max_fwd = the largest edges-per-loop;
 *   the components of the capped graph then come from the ranks' local forests (fslr_local_forest).
 *   Syncs; out: applied, max_fwd, candidates, dropped, backward (capped / hits / pairs: the sum of the
 *   ranks' parts).
 * The restricted gather: only rows whose lower read x has fwd(x) + bwd(x) >= edge_threshold over E* can
 * take part (the closure's join test, cluster.py:210-213 via DESIGN.md §11), about 3% of E* at cfg5.
 * fslr_cap_bwd_counts: this rank's counts of its edges per upper read b into out
 *   (device, n_reads elements of elem_bytes: 1 = uint8 clipped at edge_threshold <= 255, 4 = int32;
 *   async); the caller sums them over the ranks (all_reduce; uint8 needs world x threshold <= 255).
 * fslr_cap_restrict: from the summed counts, this rank's rows of S (its edges whose lower read has
 *   fwd + bwd >= threshold, sorted by lower read: no fslr_sort_edges of the whole list is needed);
 *   *n_rows = their count (syncs).
 * fslr_cap_copy_restricted: those rows as int32 (a, b) pairs padded with -1 to n_pad (device, async).
 * fslr_cap_install_restricted: the ranks' gathered restricted rows, as fslr_cap_install_pairs (the rest
 *   of the sequence is unchanged); fslr_cap_apply_changes then maps this rank's block back onto its
 *   edges and its max_fwd covers S and this rank's reads outside S: the MAX over ranks is the capped
 *   graph's. */
/* The multi-GPU merge by local forests (get_subgraphs, cluster.py:230-234, over the union of the ranks'
 * edges).  fslr_local_forest: union-find over this context's edges; the (read, root) pairs of the
 * reads that are not their own root are kept (the same partition as the edges, in fewer pairs);
 * *n_pairs (may be NULL: no sync) gets their count.  fslr_copy_forest_pairs: those pairs as int32
 * (read, root) into a device buffer of n_pad pairs, padded with -1 (async).  The ranks all-gather
 * them and fslr_components_from_pairs takes the union. */
int  fslr_local_forest(fslr_ctx *ctx, int64_t *n_pairs);
int  fslr_copy_forest_pairs(fslr_ctx *ctx, int32_t *dst, int64_t n_pad);
/* fslr_sort_edges: this context's edge list (with I, U) grouped by a, stably, in place (syncs once for
 * the count).  The sharded cap's ranks sort before the gather, so each read's forward edges are one run of
 * the gathered rows (the closure walks the runs; unsorted blocks still work, through an adjacency). */
int  fslr_sort_edges(fslr_ctx *ctx);
int  fslr_cap_install_pairs(fslr_ctx *ctx, const int32_t *pairs, int64_t n_rows, int32_t world, int32_t rank);
int  fslr_cap_sizes(fslr_ctx *ctx, int64_t *n_t, int64_t *n_ti, int64_t *n_hits);
int  fslr_cap_dep_local(fslr_ctx *ctx, int32_t *out);
int  fslr_cap_shard_plan(fslr_ctx *ctx, const int32_t *gathered, int32_t world, int32_t rank, int64_t *sizes);
int  fslr_cap_shard_pack(fslr_ctx *ctx, int32_t *counts, int32_t *hits);
int  fslr_cap_replay_shard(fslr_ctx *ctx, const int32_t *counts, const int32_t *hits, int64_t *n_changes,
                           fslr_cap_stats *part);
int  fslr_cap_copy_changes(fslr_ctx *ctx, int32_t *dst, int64_t n_pad);
int  fslr_cap_apply_changes(fslr_ctx *ctx, const int32_t *changes, int64_t n, fslr_cap_stats *out);
int  fslr_cap_bwd_counts(fslr_ctx *ctx, int32_t edge_threshold, void *out, int32_t elem_bytes);
int  fslr_cap_restrict(fslr_ctx *ctx, const void *bwd, int32_t elem_bytes, int64_t *n_rows);
int  fslr_cap_copy_restricted(fslr_ctx *ctx, int32_t *dst, int64_t n_pad);
int  fslr_cap_install_restricted(fslr_ctx *ctx, const int32_t *pairs, int64_t n_rows, int32_t world, int32_t rank);
int  fslr_sweep_partition(fslr_ctx *ctx, const fslr_params *params, int32_t n_dest, int32_t block_shift,
                          void *dst, int64_t dst_cap, int64_t *counts);
int  fslr_sweep_evaluate(fslr_ctx *ctx, const fslr_params *params, const void *entries, int64_t n);
/* fslr_sweep_partition_repeat: fslr_sweep_partition again on unchanged input (no fslr_set_* since),
 * parameters and split, without the readback: the entries land where the last synchronous call put
 * them (its counts), and a device check flags any difference (fslr_read_stats then returns
 * FSLR_ERR_STATE with overflow_flags & 32: rerun synchronously).  Async.  FSLR_ERR_STATE when the last
 * synchronous call was for another input, parameters or split.  The repeated steps of a benchmark
 * or of a service querying one resident input use it. */
int  fslr_sweep_partition_repeat(fslr_ctx *ctx, const fslr_params *params, int32_t n_dest, int32_t block_shift,
                                 void *dst, int64_t dst_cap);

/* Reads of more than FSLR_MAX_L intervals.  The caller uploads a *virtual* CSR with
 * fslr_set_reads: virtual read v < n_real is real read v (its first <= FSLR_MAX_L intervals), reads
 * v >= n_real are the further <= FSLR_MAX_L-interval chunks of the long reads; vreal[v] = its real
 * read, vbase[v] = the index of its first interval in the real read's list, rlen[r] = the real
 * read's interval count, umax[I-1] = the largest U with I/U >= cutoff(I) (cluster.py:216-219, Python
 * floats), for I = 1 .. n_umax >= max(rlen).  Syncs.
 * fslr_long_query (after fslr_build_index): sweep the virtual index (every match entry), decide the
 * pairs with a long read with the reference's first-fit over their real interval lists (list1 = the
 * lower-rank read) into a list of (a, b, I, U) edges (*n_long_edges), and the pairs of two short
 * reads with the sweep's pair stage into the context's edges and forward degrees (as fslr_query:
 * fslr_read_stats, reserve and rerun on overflow; then fslr_components).  Syncs.
 * fslr_get_long_edges: D2H of the long-pair edges (sync); union them into the labels with
 * fslr_union_pairs + fslr_finalize_labels after fslr_components. */
int  fslr_set_long_reads(fslr_ctx *ctx, int64_t n_real, const int32_t *vreal, const int32_t *vbase,
                         const int32_t *rlen, const int32_t *umax, int32_t n_umax);
/* The same without a caller-made split: fslr_set_reads_any takes the REAL CSR (reads of 1..4096
 * intervals), makes the virtual CSR and maps above and uploads them (as fslr_set_reads when no read
 * exceeds FSLR_MAX_L).  Later fslr_set_thresholds calls take iv_thr in the real CSR's interval order
 * too.  fslr_set_long_cutoffs sets umax (as above) before fslr_long_query / fslr_long_pairs /
 * fslr_cap_replay_pairs.  Replaces the host-side split a binding would otherwise re-implement
 * (reference: overall_jaccard_similarity takes lists of any length, cluster.py:140-170). */
int  fslr_set_reads_any(fslr_ctx *ctx, const fslr_reads *reads);
int  fslr_set_long_cutoffs(fslr_ctx *ctx, const int32_t *umax, int32_t n_umax);
int  fslr_long_query(fslr_ctx *ctx, const fslr_params *params, int64_t *n_long_edges);
int  fslr_get_long_edges(fslr_ctx *ctx, int32_t *a, int32_t *b, int32_t *I, int32_t *U, int64_t capacity);
/* The general pair path (any overlap, aln_size == 0 intervals, qlen2 / n_alignments
 * 0, reads of up to 4096 intervals), replacing cluster.py:197-222 where the sweep's gates do not
 * apply.  fslr_long_pairs (after fslr_set_reads [+ fslr_set_long_reads] and fslr_build_index):
 * every read's search-ordered hits, each distinct pair decided once by the reference's first-fit
 * (list1 = the lower-rank read) into the long-edge list (fslr_get_long_edges, I and U unclamped) and
 * the context's edges and forward degrees (then fslr_components); FSLR_ERR_ZERO_DIVISION when a pair
 * raises.  Syncs.
 * fslr_cap_replay_pairs: the edge cap (cluster.py:223-224) replayed over the given E* — ne pairs of
 * real read ranks a < b, host arrays — in the read space of the last fslr_set_reads (+
 * fslr_set_long_reads).  who[k] = 0 when edge k is formed in a's loop, 1 in b's, 2 when the capped
 * graph drops it; fwd[n_reads] (may be NULL) = edges formed in each read's own loop.  The capped
 * graph also becomes the context's edges (fslr_components).  Syncs; out may be NULL. */
int  fslr_long_pairs(fslr_ctx *ctx, const fslr_params *params, int64_t *n_edges);
/* fslr_long_pairs for the pairs whose lower-rank read lies in query shard `shard` of `n_shards` (read
 * blocks of 64 dealt round robin, as fslr_query_shard): the shards together give fslr_long_pairs'
 * edges, each pair once (the multi-GPU split of the inputs the sweep does not take). */
int  fslr_long_pairs_shard(fslr_ctx *ctx, const fslr_params *params, int32_t shard, int32_t n_shards,
                           int64_t *n_edges);
int  fslr_cap_replay_pairs(fslr_ctx *ctx, int32_t edge_threshold, const int32_t *a, const int32_t *b, int64_t ne,
                           uint8_t *who, int32_t *fwd, fslr_cap_stats *out);

/* build_index + query(all reads) + components, enqueued back to back.  Async. */
int  fslr_run(fslr_ctx *ctx, const fslr_params *params);

int  fslr_sync(fslr_ctx *ctx);
/* syncs; returns stats.error, or FSLR_ERR_STATE when the edge or deferred buffer overflowed
 * (reserve and rerun the query: components and labels of an overflowed query are refused) */
int  fslr_read_stats(fslr_ctx *ctx, fslr_query_stats *out);
int  fslr_get_timings(fslr_ctx *ctx, fslr_timings *out);        /* syncs */
/* Profiling: durations (ms) of the main pair-kernel launch of the last min(n, 256) queries since
 * profiling was enabled, oldest first (hipEvents recorded on the context's stream around that one
 * launch).  Syncs; returns the count or -error. */
int  fslr_get_pair_kernel_times(fslr_ctx *ctx, float *ms, int32_t n);
/* The same for one stage kernel: stage 0 = the main pair kernel (as above), 1 = the sweep engine's
 * pair-stage kernel (the evaluation of the grouped match entries).  Syncs; count or -error. */
int  fslr_get_stage_kernel_times(fslr_ctx *ctx, int32_t stage, float *ms, int32_t n);
/* Raw device counters of the last query (diagnostics; layout is internal, kernels.hpp:
 * Counter).  Copies min(n, 32) words, syncs, returns the count or -error. */
int  fslr_read_counters(fslr_ctx *ctx, uint64_t *out, int n);

/* D2H copies (sync). */
int  fslr_get_labels(fslr_ctx *ctx, int32_t *labels);          /* [n_reads] min-rank root; FSLR_ERR_STATE
                                                                   after an overflowed query */
int  fslr_get_fwd_degree(fslr_ctx *ctx, int32_t *fwd);         /* [n_reads] */
int  fslr_get_edges(fslr_ctx *ctx, int32_t *a, int32_t *b, uint16_t *iu, int64_t capacity);
                                                                /* iu = I | (U << 8); returns count via stats */

/* Device-side views for collectives (e.g. RCCL all_gather of labels). */
int  fslr_labels_device_ptr(fslr_ctx *ctx, void **dptr);
/* Copy the [n_reads] labels into a caller-owned device buffer on this device (async, ctx stream). */
int  fslr_copy_labels_device(fslr_ctx *ctx, int32_t *dst);
/* Copy the [n_reads] forward degrees into a caller-owned device buffer (async, ctx stream). */
int  fslr_copy_fwd_device(fslr_ctx *ctx, int32_t *dst);
/* Union (src[k], dst[k]) into the context's forest; pointers are device pointers
 * on this context's device when on_device != 0, else host.  src == NULL means
 * src[k] = k mod n_reads, so W concatenated label vectors merge in one call.
 * Follow with fslr_finalize_labels.  Async. */
int  fslr_union_pairs(fslr_ctx *ctx, const int32_t *src, const int32_t *dst, int64_t n, int on_device);
int  fslr_finalize_labels(fslr_ctx *ctx);
/* Copy this context's edges as int32 (a, b) pairs into a caller-owned device buffer of n_pad pairs,
 * padded with (-1, -1); the edge count is read on the device, so n_pad only has to be at least it
 * (the multi-GPU merge pads every rank to the largest count).  Async, ctx stream. */
int  fslr_copy_edges_device(fslr_ctx *ctx, int32_t *dst, int64_t n_pad);
/* Labels = connected components (min-rank roots) of the n int32 (a, b) device pairs at `pairs`
 * (pairs with a < 0 are skipped): the union of W ranks' gathered edge lists.  Async. */
int  fslr_components_from_pairs(fslr_ctx *ctx, const int32_t *pairs, int64_t n);

#ifdef __cplusplus
}
#endif
#endif /* FSLR_HIP_H */
