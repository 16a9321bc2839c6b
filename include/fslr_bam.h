/*
 * fslr_bam.h — host-side C ABI for decoding the aligned reads of `{name}.bwa_dodi.bam` into the
 * columns `collect_mapping_info.mapping_info` needs (the producer of the
 * `.mappings.bed` input of the clustering path).
 *
 * Replaces the reference's pysam calls in fslr/collect_mapping_info.py (in /root/reference):
 *   af.fetch(until_eof=True)                   :23   every record, file order
 *   a.flag, a.qname, a.mapq, a.rname           :24,26-27,76,98
 *   r.cigartuples[0] / [-1] (S or H clips)     :13-16
 *   r.infer_read_length()                      :11   M I S = X H lengths (hard clips included)
 *   a.reference_start + 1, a.reference_end     :77-78  pos + 1, pos + M D N = X lengths
 *   a.get_tag('AS')                            :40,99  integer tag types only
 *   pri_read.get_forward_sequence()            :51   SEQ, reverse-complemented when flag & 16
 *   af.get_reference_name(tid)                 :76
 *
 * BGZF blocks are inflated in parallel (std::thread, zlib raw inflate), then the SAMv1 §4.2
 * records are indexed in one pass.  Plain C types, caller-owned output arrays, library-owned
 * decoded stream behind an opaque handle.
 */
#ifndef FSLR_BAM_H
#define FSLR_BAM_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define FSLR_BAM_OK 0
#define FSLR_BAM_ERROR 1

typedef struct FslrBam FslrBam;

/* Read and decode the whole file (n_threads <= 0: all cores). */
int fslr_bam_open(const char *path, int n_threads, FslrBam **out, char *err, size_t errlen);
void fslr_bam_close(FslrBam *b);

int64_t fslr_bam_n_records(const FslrBam *b);
int fslr_bam_n_refs(const FslrBam *b);
/* Reference name (NUL-terminated, library-owned) and length of target tid. */
const char *fslr_bam_ref_name(const FslrBam *b, int tid);
int64_t fslr_bam_ref_len(const FslrBam *b, int tid);
/* Total bytes of all read names (without NULs), for fslr_bam_columns' qname_buf. */
int64_t fslr_bam_qname_bytes(const FslrBam *b);

/* Per record (file order), every array of length fslr_bam_n_records():
 *   flag, tid, pos (0-based reference_start), mapq,
 *   ref_span   = sum of M D N = X lengths (reference_end - reference_start),
 *   read_len   = infer_read_length(): sum of M I S = X H lengths,
 *   clip_first / clip_last = length of the first / last CIGAR op if it is S or H, else 0,
 *   n_cigar    = number of CIGAR ops,
 *   as_tag     = the AS tag's integer value; as_kind = 1 integer AS, 0 no AS tag, 2 non-integer AS,
 *   l_seq      = SEQ length (0 for '*'),
 *   qname_end  = cumulative end offset of each name in qname_buf (names concatenated). */
int fslr_bam_columns(const FslrBam *b, int32_t *flag, int32_t *tid, int64_t *pos, int32_t *mapq, int64_t *ref_span,
                     int64_t *read_len, int64_t *clip_first, int64_t *clip_last, int32_t *n_cigar, int64_t *as_tag,
                     int8_t *as_kind, int64_t *l_seq, int64_t *qname_end, char *qname_buf);

/* get_forward_sequence() of record rec into out (l_seq bytes, no NUL): the SEQ letters
 * ("=ACMGRSVTWYHKDBN"), reverse-complemented when flag & 16 (A<->T, C<->G, other letters kept
 * as pysam's complement table maps them). */
int fslr_bam_forward_seq(const FslrBam *b, int64_t rec, char *out);

#ifdef __cplusplus
}
#endif
#endif
