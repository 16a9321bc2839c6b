/*
 * fslr_oracle.c — CPU restatement of fslr's clustering hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker for the HIP product path:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it.  The product (fslr_amd/) never links or calls it.
 *
 * It restates, in plain C with IEEE double arithmetic (== CPython float), the
 * reference functions (all citations into /root/reference/fslr/):
 *
 *   oracle_query()          cluster.py:187-227  query_interval_trees (driver,
 *                           seen-set, per-query-read edge cap)
 *     search()              cluster.py:124-130,201 build_interval_trees +
 *                           superintervals IntervalMap.search_values, end-inclusive;
 *                           hit order = descending position in (start asc,
 *                           end desc, insertion asc) — the library's order is
 *                           undocumented, it only matters when
 *                           the edge cap binds
 *     lengths_differ()      cluster.py:178-183  different_lengths_or_alignments
 *     jaccard()             cluster.py:140-170  overall_jaccard_similarity
 *     overlap_ok()          cluster.py:133-136  calculate_overlap (>= percentage)
 *     cutoff lookup         cluster.py:216-219
 *   components              cluster.py:230-234 + networkx connected_components:
 *                           components numbered in order of their first node's
 *                           insertion into the graph (G.add_edge(query, other)).
 *
 * ZeroDivisionError of the reference (aln_size == 0 in calculate_overlap,
 * max(qlen2)==0 / max(n_alignments)==0 in different_lengths_or_alignments) is
 * returned as ORACLE_ZERO_DIVISION at the exact point the reference would raise.
 *
 * Inputs are the rank-ordered CSR the reference builds implicitly at
 * cluster.py:189-191 (query_intervals: reads in first-appearance order of the
 * start-sorted `data` list, each read's intervals in `data` order), with
 * per-interval fields exactly as in IntervalItem (cluster.py:10-11).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_OK 0
#define ORACLE_ZERO_DIVISION 1
#define ORACLE_EDGE_CAPACITY 2
#define ORACLE_NOMEM 3
#define ORACLE_BAD_INPUT 4

typedef struct {
    int64_t n_reads;
    const int64_t *read_off;   /* [n_reads+1] CSR offsets (rank order) */
    const int64_t *chrom;      /* per interval */
    const int64_t *start;
    const int64_t *end;
    const int64_t *aln;        /* aln_size (query length of the alignment) */
    const int64_t *qlen2;      /* per interval, as carried by IntervalItem */
    const int64_t *nal;        /* n_alignments, per interval */
    const int64_t *data_pos;   /* position in the start-sorted `data` list (tree insertion order) */
} oracle_input;

typedef struct {
    double overlap;            /* --overlap (percentage) */
    const double *cutoffs;     /* --jaccard-cutoffs */
    int64_t n_cutoffs;
    double qlen_diff;
    double nal_diff;
    int64_t edge_threshold;    /* main.py:221 hard-codes 10 */
    int64_t use_cap;           /* 1 = reference behaviour; 0 = E* (no cap) */
    int64_t query_end;         /* evaluate query reads [0, query_end) only (-1 = all): bounded CPU samples */
} oracle_params;

typedef struct {
    int64_t evaluated_pairs;   /* pairs that passed the seen-set (cluster.py:205-208) */
    int64_t jaccard_evals;     /* pairs that reached overall_jaccard_similarity */
    int64_t interval_hits;     /* search_values hits visited */
    int64_t n_edges;
    int64_t max_fwd;           /* max over reads of edges added in the read's own loop */
    int64_t n_components;
    int64_t err_a, err_b;      /* pair (ranks) that raised, if any */
} oracle_stats;

/* ---------------- seen-pair hash set ---------------- */
typedef struct { uint64_t *slot; uint64_t mask; uint64_t count; } pairset;

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}

static int ps_init(pairset *s, uint64_t cap) {
    uint64_t n = 1024;
    while (n < cap * 2) n <<= 1;
    s->slot = (uint64_t *)malloc(n * sizeof(uint64_t));
    if (!s->slot) return -1;
    memset(s->slot, 0xff, n * sizeof(uint64_t));
    s->mask = n - 1; s->count = 0;
    return 0;
}

static int ps_grow(pairset *s) {
    pairset t;
    if (ps_init(&t, (s->mask + 1)) != 0) return -1;
    for (uint64_t i = 0; i <= s->mask; i++) {
        uint64_t k = s->slot[i];
        if (k == UINT64_MAX) continue;
        uint64_t h = mix64(k) & t.mask;
        while (t.slot[h] != UINT64_MAX) h = (h + 1) & t.mask;
        t.slot[h] = k; t.count++;
    }
    free(s->slot);
    *s = t;
    return 0;
}

/* returns 1 if inserted (was absent), 0 if present, -1 on OOM */
static int ps_insert(pairset *s, uint64_t k) {
    if ((s->count + 1) * 2 > s->mask + 1) { if (ps_grow(s) != 0) return -1; }
    uint64_t h = mix64(k) & s->mask;
    while (s->slot[h] != UINT64_MAX) {
        if (s->slot[h] == k) return 0;
        h = (h + 1) & s->mask;
    }
    s->slot[h] = k; s->count++;
    return 1;
}

/* ---------------- per-chromosome interval index (superintervals stand-in) ---------------- */
typedef struct {
    int64_t n;
    int64_t *iv;      /* interval ids in (start asc, end desc, insertion asc) order */
    int64_t *st;      /* starts in that order */
    int64_t *pmax;    /* prefix max of end */
} chrom_index;

static const oracle_input *g_in;   /* for qsort comparator */

static int cmp_iv(const void *pa, const void *pb) {
    int64_t a = *(const int64_t *)pa, b = *(const int64_t *)pb;
    if (g_in->start[a] != g_in->start[b]) return g_in->start[a] < g_in->start[b] ? -1 : 1;
    if (g_in->end[a] != g_in->end[b]) return g_in->end[a] > g_in->end[b] ? -1 : 1;
    if (g_in->data_pos[a] != g_in->data_pos[b]) return g_in->data_pos[a] < g_in->data_pos[b] ? -1 : 1;
    return 0;
}

/* ---------------- predicates ---------------- */

/* cluster.py:133-136 calculate_overlap(i1, i2) >= percentage; sets *zd on ZeroDivisionError */
static int overlap_ok(const oracle_input *in, int64_t a, int64_t b, double pct, int *zd) {
    int64_t lo = in->start[a] > in->start[b] ? in->start[a] : in->start[b];
    int64_t hi = in->end[a] < in->end[b] ? in->end[a] : in->end[b];
    int64_t o = hi - lo;
    if (o < 0) o = 0;
    if (in->aln[a] == 0 || in->aln[b] == 0) { *zd = 1; return 0; }
    double r1 = (double)o / (double)in->aln[a];
    double r2 = (double)o / (double)in->aln[b];
    double r = r1 < r2 ? r1 : r2;     /* Python min(): first of equals; value identical */
    return r >= pct;
}

/* cluster.py:178-183; returns 1 = "different" (skip pair) */
static int lengths_differ(int64_t q1, int64_t q2, int64_t n1, int64_t n2, double qd, double nd, int *zd) {
    int64_t mn = q1 < q2 ? q1 : q2, mx = q1 < q2 ? q2 : q1;
    if (mx == 0) { *zd = 1; return 0; }
    if ((double)mn / (double)mx >= 1.0 - qd) return 0;
    mn = n1 < n2 ? n1 : n2; mx = n1 < n2 ? n2 : n1;
    if (mx == 0) { *zd = 1; return 0; }
    if ((double)mn / (double)mx >= 1.0 - nd) return 0;
    return 1;
}

/* cluster.py:140-170: first-fit greedy; returns intersection count, *U = union */
static int64_t jaccard(const oracle_input *in, int64_t a0, int64_t la, int64_t b0, int64_t lb,
                       double pct, unsigned char *used, int64_t *U, int *zd) {
    memset(used, 0, (size_t)lb);
    int64_t inter = 0;
    for (int64_t i = 0; i < la; i++) {
        for (int64_t j = 0; j < lb; j++) {
            if (used[j]) continue;
            if (in->chrom[a0 + i] == in->chrom[b0 + j]) {
                int ok = overlap_ok(in, a0 + i, b0 + j, pct, zd);
                if (*zd) return 0;
                if (ok) { used[j] = 1; inter++; break; }
            }
        }
    }
    *U = la + lb - inter;   /* union = intersection + zeros, zeros = la+lb-2*inter */
    return inter;
}

/* ---------------- driver ---------------- */

/* per-chromosome indexes over all intervals (build_interval_trees, cluster.py:124-130) */
typedef struct {
    int64_t *read_of;     /* interval -> read rank */
    chrom_index *ci;
    int64_t nc;
    int64_t *cnt, *all;
    int64_t maxlen;
} oracle_index;

static void index_free(oracle_index *ix) {
    free(ix->read_of); free(ix->ci); free(ix->cnt); free(ix->all);
    memset(ix, 0, sizeof(*ix));
}

static int index_build(const oracle_input *in, oracle_index *ix) {
    memset(ix, 0, sizeof(*ix));
    const int64_t N = in->n_reads;
    if (N < 0 || !in->read_off) return ORACLE_BAD_INPUT;
    const int64_t NI = in->read_off[N];
    ix->read_of = (int64_t *)malloc((size_t)(NI > 0 ? NI : 1) * sizeof(int64_t));
    if (!ix->read_of) return ORACLE_NOMEM;
    int64_t maxlen = 1, cmax = -1, cmin = 0;
    for (int64_t r = 0; r < N; r++) {
        for (int64_t k = in->read_off[r]; k < in->read_off[r + 1]; k++) ix->read_of[k] = r;
        if (in->read_off[r + 1] - in->read_off[r] > maxlen) maxlen = in->read_off[r + 1] - in->read_off[r];
    }
    for (int64_t k = 0; k < NI; k++) {
        if (in->chrom[k] > cmax) cmax = in->chrom[k];
        if (in->chrom[k] < cmin) cmin = in->chrom[k];
    }
    if (cmin < 0 || cmax > (1 << 24)) { index_free(ix); return ORACLE_BAD_INPUT; }
    const int64_t nc = cmax + 1;
    ix->nc = nc;
    ix->maxlen = maxlen;
    ix->ci = (chrom_index *)calloc((size_t)(nc > 0 ? nc : 1), sizeof(chrom_index));
    ix->cnt = (int64_t *)calloc((size_t)(nc > 0 ? nc : 1), sizeof(int64_t));
    ix->all = (int64_t *)malloc((size_t)(NI > 0 ? NI : 1) * 3 * sizeof(int64_t));
    if (!ix->ci || !ix->cnt || !ix->all) { index_free(ix); return ORACLE_NOMEM; }
    chrom_index *ci = ix->ci;
    for (int64_t k = 0; k < NI; k++) ix->cnt[in->chrom[k]]++;
    int64_t off = 0;
    for (int64_t c = 0; c < nc; c++) {
        ci[c].n = 0; ci[c].iv = ix->all + off; ci[c].st = ix->all + NI + off; ci[c].pmax = ix->all + 2 * NI + off;
        off += ix->cnt[c];
    }
    for (int64_t k = 0; k < NI; k++) { chrom_index *x = &ci[in->chrom[k]]; x->iv[x->n++] = k; }
    g_in = in;
    for (int64_t c = 0; c < nc; c++) {
        chrom_index *x = &ci[c];
        if (x->n > 1) qsort(x->iv, (size_t)x->n, sizeof(int64_t), cmp_iv);
        int64_t m = INT64_MIN;
        for (int64_t t = 0; t < x->n; t++) {
            x->st[t] = in->start[x->iv[t]];
            if (in->end[x->iv[t]] > m) m = in->end[x->iv[t]];
            x->pmax[t] = m;
        }
    }
    return ORACLE_OK;
}

/* Reached lists for the lean seen-set (oracle_query_lean): the partners > r that read r's own
 * query inserted into `seen` before its first edge-cap break, for reads whose query broke. */
typedef struct { int64_t *off; int32_t *pool; int64_t n, cap; unsigned char *broke; } reached_lists;

static int rl_push(reached_lists *rl, int32_t v) {
    if (rl->n == rl->cap) {
        int64_t nc = rl->cap ? rl->cap * 2 : (1 << 20);
        int32_t *np = (int32_t *)realloc(rl->pool, (size_t)nc * sizeof(int32_t));
        if (!np) return -1;
        rl->pool = np; rl->cap = nc;
    }
    rl->pool[rl->n++] = v;
    return 0;
}

static int cmp_i32(const void *x, const void *y) {
    int32_t a = *(const int32_t *)x, b = *(const int32_t *)y;
    return (a > b) - (a < b);
}

static int query_impl(const oracle_input *in, const oracle_params *p,
                      int64_t *edge_a, int64_t *edge_b, int32_t *edge_I, int32_t *edge_U, int64_t edge_capacity,
                      int32_t *fwd_count, int32_t *comp, oracle_stats *st, int lean);

int oracle_query(const oracle_input *in, const oracle_params *p,
                 int64_t *edge_a, int64_t *edge_b, int32_t *edge_I, int32_t *edge_U, int64_t edge_capacity,
                 int32_t *fwd_count, int32_t *comp, oracle_stats *st) {
    return query_impl(in, p, edge_a, edge_b, edge_I, edge_U, edge_capacity, fwd_count, comp, st, 0);
}

/* oracle_query with the seen-set (cluster.py:205-207) held per read instead of as one set of
 * pairs — the same answer in O(reads + reached pairs of broken reads) memory, for full-size runs
 * (config 5: ~1e10 distinct pairs would not fit a pair hash set).  Why it is the same set: when
 * read a meets partner b,
 *   - b > a: {a, b} can only have been inserted earlier in a's own query -> a per-query stamp;
 *   - b < a: {a, b} was inserted in b's query iff b's query visited a before it stopped.  A query
 *     that never met the edge-cap break visited every hit partner, and hits are symmetric (a's
 *     interval overlaps b's), so it visited a; a query that broke visited exactly the partners it
 *     recorded in its reached list (partners > b only: the others are never queried again).
 * tests/test_oracle.py checks both forms equal on every capped fixture. */
int oracle_query_lean(const oracle_input *in, const oracle_params *p,
                      int64_t *edge_a, int64_t *edge_b, int32_t *edge_I, int32_t *edge_U, int64_t edge_capacity,
                      int32_t *fwd_count, int32_t *comp, oracle_stats *st) {
    return query_impl(in, p, edge_a, edge_b, edge_I, edge_U, edge_capacity, fwd_count, comp, st, 1);
}

static int query_impl(const oracle_input *in, const oracle_params *p,
                      int64_t *edge_a, int64_t *edge_b, int32_t *edge_I, int32_t *edge_U, int64_t edge_capacity,
                      int32_t *fwd_count, int32_t *comp, oracle_stats *st, int lean) {
    memset(st, 0, sizeof(*st));
    st->err_a = st->err_b = -1;
    const int64_t N = in->n_reads;
    oracle_index ix;
    int brc = index_build(in, &ix);
    if (brc != ORACLE_OK) return brc;
    int64_t *read_of = ix.read_of;
    chrom_index *ci = ix.ci;
    unsigned char *used = (unsigned char *)malloc((size_t)ix.maxlen);
    if (!used) { index_free(&ix); return ORACLE_NOMEM; }

    pairset seen;
    if (ps_init(&seen, 1 << 16) != 0) { index_free(&ix); free(used); return ORACLE_NOMEM; }
    reached_lists rl;
    memset(&rl, 0, sizeof(rl));
    int64_t *stamp = NULL;                         /* lean: last query read that met each read */
    int rc = ORACLE_OK;
    int64_t ne = 0;
    /* graph node insertion order (networkx dict order) */
    int64_t *ins_order = (int64_t *)malloc((size_t)(N > 0 ? N : 1) * sizeof(int64_t));
    int64_t n_ins = 0;
    int64_t *ins_pos = (int64_t *)malloc((size_t)(N > 0 ? N : 1) * sizeof(int64_t));
    int64_t *uf = (int64_t *)malloc((size_t)(N > 0 ? N : 1) * sizeof(int64_t));
    if (!ins_order || !ins_pos || !uf) { rc = ORACLE_NOMEM; goto done; }
    if (lean) {
        rl.off = (int64_t *)malloc((size_t)(N + 1) * sizeof(int64_t));
        rl.broke = (unsigned char *)calloc((size_t)(N > 0 ? N : 1), 1);
        stamp = (int64_t *)malloc((size_t)(N > 0 ? N : 1) * sizeof(int64_t));
        if (!rl.off || !rl.broke || !stamp) { rc = ORACLE_NOMEM; goto done; }
        for (int64_t r = 0; r < N; r++) stamp[r] = -1;
        rl.off[0] = 0;
    }
    for (int64_t r = 0; r < N; r++) { ins_pos[r] = -1; uf[r] = r; fwd_count[r] = 0; }

    const int64_t qend = (p->query_end >= 0 && p->query_end < N) ? p->query_end : N;
    for (int64_t a = 0; a < qend && rc == ORACLE_OK; a++) {
        int64_t edges = 0;
        const int64_t rl_begin = rl.n;
        const int64_t a0 = in->read_off[a], la = in->read_off[a + 1] - a0;
        for (int64_t i = 0; i < la && rc == ORACLE_OK; i++) {
            const int64_t itv = a0 + i;
            chrom_index *x = &ci[in->chrom[itv]];
            const int64_t qs = in->start[itv], qe = in->end[itv];
            /* upper bound: first position with start > qe */
            int64_t lo = 0, hi = x->n;
            while (lo < hi) { int64_t mid = (lo + hi) >> 1; if (x->st[mid] <= qe) lo = mid + 1; else hi = mid; }
            for (int64_t t = lo - 1; t >= 0 && x->pmax[t] >= qs; t--) {
                const int64_t o = x->iv[t];
                if (in->end[o] < qs) continue;           /* not a hit */
                st->interval_hits++;
                const int64_t b = read_of[o];
                if (b == a) continue;                     /* cluster.py:203-204 */
                int ins;
                if (!lean) {
                    const uint64_t lo_r = (uint64_t)(a < b ? a : b), hi_r = (uint64_t)(a < b ? b : a);
                    ins = ps_insert(&seen, lo_r * (uint64_t)N + hi_r);
                } else if (stamp[b] == a) {
                    ins = 0;                              /* met earlier in this query */
                } else {
                    stamp[b] = a;
                    if (b > a) {
                        ins = 1;
                        if (rl_push(&rl, (int32_t)b) != 0) ins = -1;
                    } else if (!rl.broke[b]) {
                        ins = 0;                          /* b's unbroken query visited a */
                    } else {
                        const int32_t key = (int32_t)a;
                        ins = bsearch(&key, rl.pool + rl.off[b], (size_t)(rl.off[b + 1] - rl.off[b]),
                                      sizeof(int32_t), cmp_i32) ? 0 : 1;
                    }
                }
                if (ins < 0) { rc = ORACLE_NOMEM; break; }
                if (ins == 0) continue;                   /* cluster.py:205-207 */
                st->evaluated_pairs++;
                int zd = 0;
                int diff = lengths_differ(in->qlen2[itv], in->qlen2[o], in->nal[itv], in->nal[o],
                                          p->qlen_diff, p->nal_diff, &zd);
                if (zd) { rc = ORACLE_ZERO_DIVISION; st->err_a = a; st->err_b = b; break; }
                if (diff) continue;                       /* cluster.py:209-210 */
                st->jaccard_evals++;
                const int64_t b0 = in->read_off[b], lb = in->read_off[b + 1] - b0;
                int64_t U = 0;
                int64_t I = jaccard(in, a0, la, b0, lb, p->overlap, used, &U, &zd);
                if (zd) { rc = ORACLE_ZERO_DIVISION; st->err_a = a; st->err_b = b; break; }
                if (I == 0) continue;                     /* cluster.py:216-217 */
                double target = (I - 1 < p->n_cutoffs) ? p->cutoffs[I - 1] : p->cutoffs[p->n_cutoffs - 1];
                double j = (double)I / (double)U;
                if (j >= target) {
                    if (ne >= edge_capacity) { rc = ORACLE_EDGE_CAPACITY; break; }
                    edge_a[ne] = a; edge_b[ne] = b; edge_I[ne] = (int32_t)I; edge_U[ne] = (int32_t)U;
                    ne++;
                    if (ins_pos[a] < 0) { ins_pos[a] = n_ins; ins_order[n_ins++] = a; }
                    if (ins_pos[b] < 0) { ins_pos[b] = n_ins; ins_order[n_ins++] = b; }
                    /* union-find on ranks (root = min insertion position handled below) */
                    int64_t ra = a, rb = b;
                    while (uf[ra] != ra) { uf[ra] = uf[uf[ra]]; ra = uf[ra]; }
                    while (uf[rb] != rb) { uf[rb] = uf[uf[rb]]; rb = uf[rb]; }
                    if (ra != rb) { if (ra < rb) uf[rb] = ra; else uf[ra] = rb; }
                    edges++;
                    fwd_count[a]++;
                }
                if (p->use_cap && edges >= p->edge_threshold) {         /* cluster.py:223-224 */
                    if (lean) rl.broke[a] = 1;
                    break;
                }
            }
        }
        if (lean) {
            /* keep the reached list only for a broken query; sorted for the lookups above */
            if (!rl.broke[a]) rl.n = rl_begin;
            else qsort(rl.pool + rl_begin, (size_t)(rl.n - rl_begin), sizeof(int32_t), cmp_i32);
            rl.off[a + 1] = rl.n;
        }
        if (fwd_count[a] > st->max_fwd) st->max_fwd = fwd_count[a];
    }
    st->n_edges = ne;
    if (rc == ORACLE_OK) {
        /* components in order of first-inserted node (networkx iterates G in insertion order) */
        int64_t *root_comp = (int64_t *)malloc((size_t)(N > 0 ? N : 1) * sizeof(int64_t));
        if (!root_comp) { rc = ORACLE_NOMEM; goto done; }
        for (int64_t r = 0; r < N; r++) { root_comp[r] = -1; comp[r] = -1; }
        int64_t nc2 = 0;
        for (int64_t t = 0; t < n_ins; t++) {
            int64_t v = ins_order[t], rv = v;
            while (uf[rv] != rv) rv = uf[rv];
            if (root_comp[rv] < 0) root_comp[rv] = nc2++;
            comp[v] = (int32_t)root_comp[rv];
        }
        st->n_components = nc2;
        free(root_comp);
    }
done:
    free(rl.off); free(rl.pool); free(rl.broke); free(stamp);
    free(seen.slot); index_free(&ix); free(used);
    free(ins_order); free(ins_pos); free(uf);
    return rc;
}

/* KAT entry points: single predicate evaluations on explicit interval lists. */
int oracle_jaccard_lists(int64_t la, const int64_t *ca, const int64_t *sa, const int64_t *ea, const int64_t *aa,
                         int64_t lb, const int64_t *cb, const int64_t *sb, const int64_t *eb, const int64_t *ab,
                         double pct, int64_t *I_out, int64_t *U_out) {
    /* pack both lists into one oracle_input so the same code path is exercised */
    int64_t n = la + lb;
    int64_t *buf = (int64_t *)malloc((size_t)(n > 0 ? n : 1) * 4 * sizeof(int64_t));
    unsigned char *used = (unsigned char *)malloc((size_t)(lb > 0 ? lb : 1));
    if (!buf || !used) { free(buf); free(used); return ORACLE_NOMEM; }
    int64_t *c = buf, *s = buf + n, *e = buf + 2 * n, *al = buf + 3 * n;
    for (int64_t k = 0; k < la; k++) { c[k] = ca[k]; s[k] = sa[k]; e[k] = ea[k]; al[k] = aa[k]; }
    for (int64_t k = 0; k < lb; k++) { c[la + k] = cb[k]; s[la + k] = sb[k]; e[la + k] = eb[k]; al[la + k] = ab[k]; }
    oracle_input in;
    memset(&in, 0, sizeof(in));
    in.chrom = c; in.start = s; in.end = e; in.aln = al;
    int zd = 0;
    int64_t U = 0;
    int64_t I = (la && lb) ? jaccard(&in, 0, la, la, lb, pct, used, &U, &zd) : 0;
    free(buf); free(used);
    if (zd) return ORACLE_ZERO_DIVISION;
    if (!(la && lb)) U = 0;    /* cluster.py:142-143 returns (0, 0) */
    *I_out = I; *U_out = U;
    return ORACLE_OK;
}

int oracle_lengths_differ(int64_t q1, int64_t q2, int64_t n1, int64_t n2, double qd, double nd, int32_t *out) {
    int zd = 0;
    int r = lengths_differ(q1, q2, n1, n2, qd, nd, &zd);
    if (zd) return ORACLE_ZERO_DIVISION;
    *out = r;
    return ORACLE_OK;
}

/* ---------------- CPU baseline (bench.py's cpu_baseline leg only) ----------------
 * The uncapped graph E* (every candidate pair evaluated once, in its lower-rank read's loop: the
 * reference's result whenever the edge cap does not bind) over the query reads whose 64-rank block
 * k has k % stride == 0, spread over nthreads POSIX threads sharing one index (blocks dealt round
 * robin, as the GPU shards deal them).  Counts only; no graph. */
#include <pthread.h>

typedef struct {
    const oracle_input *in;
    const oracle_params *p;
    const oracle_index *ix;
    int64_t tid, nthreads, stride;
    oracle_stats st;
    int rc;
} count_job;

static void *count_worker(void *arg) {
    count_job *j = (count_job *)arg;
    const oracle_input *in = j->in;
    const oracle_params *p = j->p;
    const int64_t N = in->n_reads;
    int64_t *stamp = (int64_t *)malloc((size_t)(N > 0 ? N : 1) * sizeof(int64_t));
    unsigned char *used = (unsigned char *)malloc((size_t)j->ix->maxlen);
    if (!stamp || !used) { free(stamp); free(used); j->rc = ORACLE_NOMEM; return NULL; }
    for (int64_t r = 0; r < N; r++) stamp[r] = -1;
    const int64_t nblk = (N + 63) / 64;
    int64_t k_own = 0;
    for (int64_t blk = 0; blk < nblk && j->rc == ORACLE_OK; blk += j->stride) {
        if ((k_own++ % j->nthreads) != j->tid) continue;
        const int64_t a_hi = (blk + 1) * 64 < N ? (blk + 1) * 64 : N;
        for (int64_t a = blk * 64; a < a_hi && j->rc == ORACLE_OK; a++) {
            const int64_t a0 = in->read_off[a], la = in->read_off[a + 1] - a0;
            for (int64_t i = 0; i < la; i++) {
                const int64_t itv = a0 + i;
                const chrom_index *x = &j->ix->ci[in->chrom[itv]];
                const int64_t qs = in->start[itv], qe = in->end[itv];
                int64_t lo = 0, hi = x->n;
                while (lo < hi) { int64_t mid = (lo + hi) >> 1; if (x->st[mid] <= qe) lo = mid + 1; else hi = mid; }
                for (int64_t t = lo - 1; t >= 0 && x->pmax[t] >= qs; t--) {
                    const int64_t o = x->iv[t];
                    if (in->end[o] < qs) continue;
                    j->st.interval_hits++;
                    const int64_t b = j->ix->read_of[o];
                    if (b <= a || stamp[b] == a) continue;   /* own read, lower rank (its loop), seen */
                    stamp[b] = a;
                    j->st.evaluated_pairs++;
                    int zd = 0;
                    if (lengths_differ(in->qlen2[itv], in->qlen2[o], in->nal[itv], in->nal[o], p->qlen_diff,
                                       p->nal_diff, &zd) || zd) {
                        if (zd) j->rc = ORACLE_ZERO_DIVISION;
                        continue;
                    }
                    j->st.jaccard_evals++;
                    const int64_t b0 = in->read_off[b], lb = in->read_off[b + 1] - b0;
                    int64_t U = 0;
                    const int64_t I = jaccard(in, a0, la, b0, lb, p->overlap, used, &U, &zd);
                    if (zd) { j->rc = ORACLE_ZERO_DIVISION; continue; }
                    if (I == 0) continue;
                    const double target = (I - 1 < p->n_cutoffs) ? p->cutoffs[I - 1] : p->cutoffs[p->n_cutoffs - 1];
                    if ((double)I / (double)U >= target) j->st.n_edges++;
                }
            }
        }
    }
    free(stamp); free(used);
    return NULL;
}

int oracle_count_threads(const oracle_input *in, const oracle_params *p, int64_t nthreads, int64_t stride,
                         oracle_stats *st) {
    memset(st, 0, sizeof(*st));
    if (nthreads < 1 || nthreads > 1024 || stride < 1) return ORACLE_BAD_INPUT;
    oracle_index ix;
    int rc = index_build(in, &ix);
    if (rc != ORACLE_OK) return rc;
    count_job *jobs = (count_job *)calloc((size_t)nthreads, sizeof(count_job));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!jobs || !th) { free(jobs); free(th); index_free(&ix); return ORACLE_NOMEM; }
    for (int64_t t = 0; t < nthreads; t++) {
        jobs[t].in = in; jobs[t].p = p; jobs[t].ix = &ix;
        jobs[t].tid = t; jobs[t].nthreads = nthreads; jobs[t].stride = stride; jobs[t].rc = ORACLE_OK;
        if (pthread_create(&th[t], NULL, count_worker, &jobs[t]) != 0) { jobs[t].rc = ORACLE_NOMEM; th[t] = 0; }
    }
    for (int64_t t = 0; t < nthreads; t++) {
        if (th[t]) pthread_join(th[t], NULL);
        st->interval_hits += jobs[t].st.interval_hits;
        st->evaluated_pairs += jobs[t].st.evaluated_pairs;
        st->jaccard_evals += jobs[t].st.jaccard_evals;
        st->n_edges += jobs[t].st.n_edges;
        if (jobs[t].rc != ORACLE_OK) rc = jobs[t].rc;
    }
    free(jobs); free(th); index_free(&ix);
    return rc;
}
