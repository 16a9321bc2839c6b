"""``fslr`` command line, clustering entry (``fslr --skip-alignment``).

Mirrors the reference click command (/root/reference/fslr/main.py:19-41): same
options, defaults, messages and output files for the clustering block
(main.py:190-352).  The read-filtering / primer-labelling / bwa+dodi alignment
stages (main.py:76-188) are outside this build: without ``--skip-alignment`` the
command stops with an error instead of running them.

Output assembly (main.py:247-352) is vectorised: cluster ids come straight from
the device union-find labels instead of a DataFrame of Python sets, with the
same values and dtypes the reference writes.
"""
from __future__ import annotations

import os
import sys
import time
import warnings

import click
import numpy as np
from ._lazy import pandas as pd

from . import __version__, cluster, fastcli, ingest

# primer names of the reference's primers.csv (fslr/primers.csv:2-7); main.py:59-67 validates
# --primers against them even under --skip-alignment
PRIMER_NAMES = ('21q1', '17p6', 'XpYpM', '16p1', 'M613', 'M615')
# primer_seq column of the reference's primers.csv: collect_mapping_info's 'missing bread' rows take
# their query span from the primer length (collect_mapping_info.py:130,148)
PRIMER_SEQS = {'21q1': 'CTACCTCTCTCGACACCAAG', '17p6': 'GGCTGAACTATAGCCTCTGC', 'XpYpM': 'AACACACTGGAAAACCTGGT',
               '16p1': 'CTGCCCTAGAAGTGAGAAGTCCA', 'M613': 'GGAGGAAAGCATGTTTCTGAG', 'M615': 'TAGTGGACAAACACGAGAGGC'}


def assign_clusters(bed_file: pd.DataFrame, G: cluster.ClusterGraph):
    """main.py:251-342: add ``cluster`` / ``n_reads`` columns to ``bed_file`` (in place).

    Clustered reads get their component index (components ordered by min read
    rank = networkx order, cluster.py:230-234) and the component size; every
    other qname of ``bed_file`` gets the next ids in first-appearance order with
    n_reads 1.  Both columns are float when any such singleton exists (the
    reference's left merge introduces NaN before fillna), int otherwise.
    """
    codes, uniq = ingest.factorize_qname(bed_file)
    rank_names = G.qnames_by_rank
    node = G.node_mask
    cid_by_name = pd.Series(G.component_id[node], index=pd.Index(rank_names[node], dtype=object))
    size_by_name = pd.Series(G.comp_size[node], index=cid_by_name.index)
    u = pd.Index(uniq, dtype=object)
    ucid = cid_by_name.reindex(u).to_numpy()
    usize = size_by_name.reindex(u).to_numpy()
    n_cluster = int(G.roots.size)
    single = np.isnan(ucid.astype(np.float64))
    k = int(single.sum())
    ucid = ucid.astype(np.float64)
    usize = usize.astype(np.float64)
    ucid[single] = np.arange(n_cluster, n_cluster + k, dtype=np.float64)   # uniq is first-appearance order
    usize[single] = 1.0
    if codes.size and (codes < 0).any():
        raise ValueError('missing qname values are not supported')
    if k:
        bed_file['cluster'] = ucid[codes]
        bed_file['n_reads'] = usize[codes]
    else:
        bed_file['cluster'] = ucid[codes].astype(np.int64)
        bed_file['n_reads'] = usize[codes].astype(np.int64)
    return bed_file


@click.command()
@click.option('--name', required=True, help='Sample name')
@click.option('--out', required=True, help='Output folder')
@click.option('--ref', required=True, help='Reference genome')
@click.option('--primers', required=True, help='Comma-separated list of primer names. Make sure these are listed in primers.csv')
@click.option('--basecalled', required=False, help='Folder of basecalled reads in fastq format to analyse')
@click.option('--trim-threshold', required=False, help='Threshold in range 0-1. Fraction of maximum primer alignment score; primer sites with lower scores are labelled False', default=0.4, type=float, show_default=True)
@click.option('--keep-temp', required=False, is_flag=True, flag_value=True, help='Keep temp files')
@click.option('--regions', required=False, type=click.Path(exists=True), help='Target regions in bed form to perform biased mapping')
@click.option('--bias', required=False, default=1.05, show_default=True, type=float, help='Multiply alignment score by bias if alignment falls within target regions')
@click.option('--procs', required=False, default=1, show_default=True, help='Number of processors to use')
@click.option('--reference-mask', required=False, type=click.Path(exists=True), help='A bed file containing target regions for creating a masked reference. Reads are first aligned to the masked reference, prior to using the main reference')
@click.option('--skip-alignment', required=False, is_flag=True, help='Skip alignment step')
@click.option('--skip-clustering', required=False, is_flag=True, help='Skip clustering step')
@click.option('--jaccard-cutoffs', required=False, default='1,1,0.66,0.66,0.66,0.5', show_default=True, help="Comma-separated list of Jaccard similarity thresholds for N-1 intersections e.g. where index=0 corresponds to one the threshold for 1 intersection.")
@click.option('--overlap', required=False, default=0.8, show_default=True, help="A number between 0 and 1. Zero means two reads don't overlap at all, while 1 means the start and end of the reads is identical.")
@click.option('--n-alignment-diff', default=0.25, required=False, show_default=True, help='How much the number of alignments in one cluster can differ. Fraction in the range 0-1.')
@click.option('--qlen-diff', default=0.04, required=False, show_default=True, help="Max difference in query length. Fraction in the range 0-1.")
@click.option('--cluster-mask', default='subtelomere', required=False, show_default=True, help="Comma separated list of chromosome names to be excluded from the clustering. Use 'subtelomere' to exclude alignments within 500kb of telomere end")
@click.option('--filter-high-coverage', required=False, is_flag=True, help='Filter regions with high coverage')
@click.option('--filter-false', required=False, is_flag=True, help='Use reads with both primers labeled')
@click.option('--device', required=False, default=None, type=int, help='HIP device ordinal for the clustering kernels (default: $LOCAL_RANK or 0)')
@click.option('--gpus', required=False, default=1, show_default=True, type=click.IntRange(1, 64),
              help='GPUs for the clustering query: one process per GPU, chromosome-split sweep with RCCL '
                   'exchange (ranks share devices over gloo when fewer are visible)')
@click.option('--timings', required=False, is_flag=True, help='Print per-stage wall times to stderr')
@click.option('--native-io/--pandas-io', default=True, show_default=True,
              help='Read .mappings.bed and write the outputs with the native threaded reader/writer '
                   '(fslr_ingest.h); inputs it cannot type exactly like pandas fall back to pandas')
@click.version_option(__version__)
def pipeline(**args):
    # the reference ignores all warnings (main.py:13): FutureWarning, and pandas' SettingWithCopyWarning by
    # its message (its class would import pandas, which the columnar path never needs)
    warnings.filterwarnings('ignore', category=FutureWarning)
    warnings.filterwarnings('ignore', message=r'\s*A value is trying to be set on a copy')
    basename = f'{args["out"]}/{args["name"]}'
    print('Basename: ', basename, file=sys.stderr)
    primers = args['primers'].split(',')
    known = set(PRIMER_NAMES)
    for p in primers:
        if p not in known:
            raise ValueError('Input primer name not in primers.csv', p, known)
    if not os.path.exists(args['out']):
        os.mkdir(args['out'])
    if not args['skip_alignment']:
        raise click.UsageError('the read filtering / primer labelling / bwa+dodi alignment stages are not part of '
                               'this build; run with --skip-alignment on an existing {name}.mappings.bed')
    if not args['skip_clustering']:
        if not run_clustering(args, basename):
            return                               # main.py:247-249 returns before 'fslr finished'
    print('fslr finished')


def run_clustering(args, basename):
    """main.py:190-352."""
    t = {}
    t0 = time.perf_counter()
    print('Making clusters')
    if (args.get('gpus') or 1) > 1:
        # the other ranks start now: their interpreter, torch import and process-group rendezvous run
        # while this process reads and prepares the input (fslr_amd.multi.RankPool)
        from . import multi
        multi.pool(args['gpus'], first_device=args.get('device') or 0)
    path = f'{basename}.mappings.bed'
    tsv = _open_tsv(path) if args.get('native_io', True) else None
    t['read.open'] = time.perf_counter() - t0
    try:
        if tsv is not None and not args['filter_high_coverage']:
            # the columnar path (fastcli): codes and int columns, no frame of rows; the scan checks
            # that every column round-trips through pandas (verbatim) while parsing the int columns
            try:
                cols = tsv.scan_all(fastcli.INT_COLS, fastcli.STR_COLS)
            except KeyError:
                cols = None
            if cols is not None:
                t['read_csv'] = time.perf_counter() - t0
                try:
                    return fastcli.run(args, basename, tsv, cols[0], cols[1], t)
                except fastcli.Fallback:
                    pass
        if tsv is not None and not tsv.verbatim():
            tsv.close()
            tsv = None
        bed_file = None
        if tsv is not None:
            bed_file = ingest.frame_from(tsv, int_columns=ingest.INT_COLUMNS + ('alignment_score',))
            if bed_file is None:
                tsv.close()
                tsv = None
        if bed_file is None:
            bed_file = pd.read_csv(path, sep='\t')
        t['read_csv'] = time.perf_counter() - t0
        return _cluster_and_write(args, basename, bed_file, tsv, t)
    finally:
        if tsv is not None:
            tsv.close()


def _open_tsv(path):
    """The native reader's TsvFile, or None when it declines the file (pandas reads it)."""
    try:
        tsv = ingest.TsvFile(path)
    except (FileNotFoundError, OSError):
        return None
    if tsv.declined:
        tsv.close()
        return None
    return tsv


def _native_tsv(path):
    """The native reader's TsvFile when every input column would round-trip through pandas unchanged,
    so that writing the input's own row bytes equals ``to_csv`` of the pandas frame (reference
    main.py:349,352); else None (pandas reads the file)."""
    tsv = _open_tsv(path)
    if tsv is not None and not tsv.verbatim():
        tsv.close()
        return None
    return tsv


def _native_open(path):
    """(TsvFile, frame of the columns clustering and the writers read) or (None, None)."""
    tsv = _native_tsv(path)
    if tsv is None:
        return None, None
    bed = ingest.frame_from(tsv, int_columns=ingest.INT_COLUMNS + ('alignment_score',))
    if bed is None:
        tsv.close()
        return None, None
    return tsv, bed


def _cluster_and_write(args, basename, bed_file, tsv, t):
    chromosome_mask = set()
    if args['cluster_mask']:
        allowed = set(bed_file['chrom'])
        for item in args['cluster_mask'].split(','):
            if item in allowed or item == 'subtelomere':
                chromosome_mask.add(item)
    jaccard_cutoffs = [float(i) for i in args['jaccard_cutoffs'].split(',')]
    overlap = args['overlap']
    edge_threshold = 10
    qlen_diff = args['qlen_diff']
    n_alignments_diff = args['n_alignment_diff']
    chr_lengths = cluster.get_chromosome_lengths(f'{basename}.bwa_dodi.bam')
    bed_file, chr_lengths, chromosome_mask, chrom_to_num_map = cluster.rename_chromosomes(
        bed_file, chr_lengths, chromosome_mask)
    if args['filter_false']:
        bed_file = cluster.delete_false(bed_file)
    t1 = time.perf_counter()
    fillings = cluster.keep_fillings(bed_file)
    if args['filter_high_coverage']:
        fillings = cluster.filter_high_coverage(fillings, bed_file, chr_lengths, threshold=10000)
    data = cluster.prepare_data(fillings, chromosome_mask, chr_lengths, threshold=500_000)
    t['prepare'] = time.perf_counter() - t1
    t1 = time.perf_counter()
    data.csr()                                   # the device layout (host; cached on data)
    t['csr'] = time.perf_counter() - t1
    t2 = time.perf_counter()
    interval_tree = cluster.build_interval_trees(data, device=args.get('device'), n_gpus=args.get('gpus') or 1)
    t['upload'] = time.perf_counter() - t2       # context, CSR H2D, index build
    t2 = time.perf_counter()
    match_data, network = cluster.query_interval_trees(interval_tree, data, overlap, jaccard_cutoffs,
                                                       edge_threshold, qlen_diff, n_alignments_diff)
    t['query'] = time.perf_counter() - t2        # pair engine, cap, components, D2H, match_df
    if network.number_of_edges() == 0:          # main.py:247: #components == #nodes only for an empty graph
        print('No clusters were found.')
        return False
    t3 = time.perf_counter()
    assign_clusters(bed_file, network)
    if tsv is None:                              # the native writer copies the input's own chrom text
        bed_file = cluster.chrom_to_str(bed_file, chrom_to_num_map)
    if tsv is not None:
        added = [c for c in bed_file.columns if c not in set(tsv.columns)]
        tsv.write_rows(f'{basename}.mappings.cluster.bed', bed_file.index.to_numpy(), bed_file[added],
                       ingest.factorize_qname(bed_file))
    else:
        bed_file.to_csv(f'{basename}.mappings.cluster.bed', index=False, sep='\t')
    bed_representative = cluster.choose_alignment(bed_file)
    if tsv is not None:
        added = [c for c in bed_representative.columns if c not in set(tsv.columns)]
        tsv.write_rows(f'{basename}.mappings.representative.bed', bed_representative.index.to_numpy(),
                       bed_representative[added], ingest.factorize_qname(bed_representative))
    else:
        bed_representative.to_csv(f'{basename}.mappings.representative.bed', index=False, sep='\t')
    t['write'] = time.perf_counter() - t3
    if args.get('timings'):
        st = network.stats
        print('timings_s ' + ' '.join(f'{k}={v:.3f}' for k, v in t.items()) +
              f' evaluated_pairs={st["evaluated_pairs"]} edges={st["n_edges"]} max_fwd={st["max_fwd"]}',
              file=sys.stderr)
    return True


def main():  # console entry
    pipeline()


if __name__ == '__main__':
    main()
