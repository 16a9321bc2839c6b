/*
 * fslr_ingest.h — host-side C ABI for reading `{name}.mappings.bed`.
 *
 * Replaces the reference's `pd.read_csv(f'{basename}.mappings.bed', sep='\t')`
 * (fslr/main.py:209 in /root/reference) for the columns the clustering path reads
 * (cluster.py:14 keep_fillings, cluster.py:109 prepare_data: chrom, rstart, rend, qname,
 * n_alignments, aln_size, qstart, qend), and `pd.factorize(col, sort=False)` on
 * the string columns.  It never guesses: a column is handed back as int64 only
 * when every field is a canonical decimal integer (pandas infers int64 for it and
 * writes it back unchanged); a string column is factorized only when no field is
 * empty or one of pandas' default NA spellings and the column is not all-integer.
 * Otherwise the call returns FSLR_INGEST_DECLINE and the caller reads the file
 * with pandas.  Quoted fields (any '"') make fslr_tsv_open decline.
 *
 * Plain C types, caller-owned output arrays, library-owned parse state behind an
 * opaque handle.  Lines are split over std::thread workers (memory-bound scan).
 */
#ifndef FSLR_INGEST_H
#define FSLR_INGEST_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define FSLR_INGEST_OK 0
#define FSLR_INGEST_ERROR 1
#define FSLR_INGEST_DECLINE 2   /* valid file, but pandas would not type it the way this fast path does */

typedef struct FslrTsv FslrTsv;

/* Read the whole file, split lines and the header. n_threads <= 0: $OMP_NUM_THREADS, else
 * min(hardware concurrency, 16). */
int fslr_tsv_open(const char *path, int n_threads, FslrTsv **out, char *err, size_t errlen);
void fslr_tsv_close(FslrTsv *t);
int64_t fslr_tsv_rows(const FslrTsv *t);
int fslr_tsv_cols(const FslrTsv *t);
/* Header name of column `col` (NUL-terminated, owned by the handle). */
const char *fslr_tsv_colname(const FslrTsv *t, int col);
/* Column index of `name`, or -1. */
int fslr_tsv_find(const FslrTsv *t, const char *name);

/* out[rows]: the column as int64 if every field is a canonical integer, else DECLINE. */
int fslr_tsv_int_column(const FslrTsv *t, int col, int64_t *out);
/* fslr_tsv_int_column for n columns in one pass over the rows (cols distinct): outs[k][rows]. */
int fslr_tsv_int_columns(const FslrTsv *t, int n, const int32_t *cols, int64_t *const *outs);

/* codes[rows] (int32, first-appearance order like pd.factorize(sort=False)).
 * Returns the number of unique values in *n_uniq and their total byte length in
 * *uniq_bytes; fetch them with fslr_tsv_uniques. */
int fslr_tsv_factorize(FslrTsv *t, int col, int32_t *codes, int64_t *n_uniq, int64_t *uniq_bytes);
/* After fslr_tsv_factorize on `col`: concatenated unique values (buf[uniq_bytes])
 * and their end offsets (ends[n_uniq]). */
int fslr_tsv_uniques(const FslrTsv *t, int col, char *buf, int64_t *ends);

/* Writer for the outputs (reference main.py:349 `.mappings.cluster.bed`, main.py:352
 * `.mappings.representative.bed`, both `to_csv(sep='\t', index=False)`): the input's own bytes
 * per kept row plus a suffix.  fslr_tsv_verbatim is OK only when pandas would write every input
 * column back byte-identically (canonical int64 columns, or text columns with no numeric,
 * bool or NA spelling besides empty); otherwise DECLINE and the caller writes with pandas. */
int fslr_tsv_verbatim(const FslrTsv *t);
/* fslr_tsv_verbatim and the canonical-int columns int_cols (outs[k][rows]) in the same pass over
 * the rows: OK only when both hold (DECLINE otherwise: the pandas path reads the file). */
int fslr_tsv_scan(const FslrTsv *t, int n_int, const int32_t *int_cols, int64_t *const *outs);
/* fslr_tsv_scan that also factorizes the string columns str_cols in the same pass (codes
 * str_codes[k][rows] as fslr_tsv_factorize; str_counts[2k] = uniques, str_counts[2k+1] = their
 * bytes, fetched with fslr_tsv_uniques); DECLINE as fslr_tsv_scan, or when a string column holds an
 * NA field or only canonical ints. */
int fslr_tsv_scan_all(FslrTsv *t, int n_int, const int32_t *int_cols, int64_t *const *outs, int n_str,
                      const int32_t *str_cols, int32_t *const *str_codes, int64_t *str_counts);
/* Header = input header + header_suffix.  Row k of the output = input row rows_out[k] (LF line
 * end) + suffix suffix_id[k], where suffix u is suffix_buf[suffix_ends[u-1] .. suffix_ends[u]). */
int fslr_tsv_write(const FslrTsv *t, const char *path, const char *header_suffix, const int64_t *rows_out,
                   int64_t n_out, const int32_t *suffix_id, const char *suffix_buf, const int64_t *suffix_ends,
                   char *err, size_t errlen);

/* Suffix text DataFrame.to_csv writes for n_keys rows of n_cols numeric columns: per key,
 * "\t" + value for each column, concatenated into out (cap bytes), ends[k] = end of key k.
 * kinds[c]: 0 = int64 (decimal), 1 = float64 (numpy str(): Python's shortest round-trip repr).
 * DECLINE on a NaN / inf value (pandas writes its na_rep / own text). */
int fslr_format_suffix(int n_cols, const int32_t *kinds, const void *const *cols, int64_t n_keys, char *out,
                       int64_t cap, int64_t *ends);

/* Reads of the prepared interval list (prepare_data order, cluster.py:109-121) grouped by rank =
 * order of first appearance of their code (cluster.py:189-191): read_code[r] (capacity n), off[r]
 * (capacity n + 1) and perm = the list positions in CSR order (by rank, list order inside a read).
 * codes must lie in [0, n_codes). */
int fslr_group_by_first_appearance(const int64_t *codes, int64_t n, int64_t n_codes, int64_t *read_code,
                                   int64_t *n_reads, int64_t *off, int64_t *perm);

/* dst[a][k] = src[a][idx[k]] for k < n and each of the n_arrays int64 columns (n_threads <= 0: all
 * cores).  prepare_data's start sort + mask as one threaded pass. */
/* keep_fillings (cluster.py:14-31) and prepare_data's per-row columns (cluster.py:109-121) over the
 * rows with row_keep[i] != 0 (NULL: all): each qname's first and last row dropped, the fillings'
 * start = min(rstart, rend), end = max(...), aln_size, qname code, n_alignments, qlen2 = max(qend) -
 * min(qstart) over the qname's fillings, chrom = chrom_lut[ccode]; outputs hold n_rows elements,
 * *n_out of them written, in file order. */
int fslr_fillings(int64_t n_rows, const int32_t *qcode, int64_t n_q, const uint8_t *row_keep, const int64_t *rstart,
                  const int64_t *rend, const int64_t *aln, const int64_t *qstart, const int64_t *qend,
                  const int64_t *nal, const int32_t *ccode, const int64_t *chrom_lut, int64_t *n_out, int64_t *frow,
                  int64_t *start, int64_t *end, int64_t *aln_o, int64_t *qc_o, int64_t *nal_o, int64_t *qlen2_o,
                  int64_t *chrom_o, int n_threads);
int fslr_gather_i64(int n_arrays, const int64_t *const *src, int64_t *const *dst, const int64_t *idx, int64_t n,
                    int n_threads);
/* prepare_data's start order (cluster.py:114, df.sort_values('start')) when no two keys tie: a
 * stable radix argsort into order[n].  Returns 1 (every key distinct: the order any sort gives,
 * pandas' quicksort included), 0 (a tie: order undefined, sort with numpy's quicksort for pandas'
 * tie order), -1 (max - min >= 2^32 or n >= 2^32: not sorted), -2 bad arguments. */
int fslr_argsort_distinct(const int64_t *keys, int64_t n, int64_t *order, int n_threads);

#ifdef __cplusplus
}
#endif
#endif
