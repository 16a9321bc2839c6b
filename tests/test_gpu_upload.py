"""fslr_set_reads on the device (upload.hip): the caller's columns are validated and packed on the GPU.

Each invalid input raises FslrError with the message of its first failure (interval columns first,
then the reads, then the data order), and a failed upload leaves the context refusing queries until a
valid one; a valid upload after it gives the oracle's graph.
"""
import numpy as np
import pytest

from fslr_amd import _lib, synth
from fslr_amd.prep import fold_overlap_threshold, pass_table
from oracle import oracle as O

pytestmark = pytest.mark.gpu
CUTS = [1, 1, 0.66, 0.66, 0.66, 0.5]


def _csr():
    return synth.generate(2000, 8, 5).interval_data().csr()


def _upload(ctx, csr, thr, **over):
    cols = dict(read_off=csr.read_off, read_qlen2=csr.read_qlen2, read_nal=csr.read_nal, iv_chrom=csr.iv_chrom,
                iv_start=csr.iv_start, iv_end=csr.iv_end, iv_thr=thr, n_chroms=csr.n_chroms,
                iv_data_pos=csr.data_pos)
    cols.update(over)
    ctx.set_reads(**cols)


def _copy(a):
    return np.array(a, dtype=np.int64, copy=True)


@pytest.mark.parametrize('case', ['chrom', 'coord', 'chrom_before_coord', 'read_len', 'nal', 'qlen2',
                                  'dp_range', 'dp_dup', 'dp_unsorted', 'coord_before_read'])
def test_invalid_upload_raises_first_failure(case):
    csr = _csr()
    thr = fold_overlap_threshold(csr.iv_aln, 0.8)
    ctx = _lib.Context(0)
    over, want = {}, None
    ch, st, en = _copy(csr.iv_chrom), _copy(csr.iv_start), _copy(csr.iv_end)
    if case == 'chrom':
        ch[777] = csr.n_chroms
        over, want = dict(iv_chrom=ch), 'chrom id out of range'
    elif case == 'coord':
        en[500] = st[500] - 1
        over, want = dict(iv_end=en), 'interval coordinates'
    elif case == 'chrom_before_coord':
        en[900] = -5
        ch[901] = -1
        over, want = dict(iv_end=en, iv_chrom=ch), 'interval coordinates'   # the lower index fails first
    elif case == 'read_len':
        off = _copy(csr.read_off)
        off[10] = off[9]                          # read 9 has no interval
        over, want = dict(read_off=off), 'every read needs'
    elif case == 'nal':
        nal = _copy(csr.read_nal)
        nal[3] = 1 << 24
        over, want = dict(read_nal=nal), 'n_alignments outside'
    elif case == 'qlen2':
        q = _copy(csr.read_qlen2)
        q[5] = -1
        over, want = dict(read_qlen2=q), 'qlen2 < 0'
    elif case == 'dp_range':
        dp = _copy(csr.data_pos)
        dp[100] = csr.n_intervals
        over, want = dict(iv_data_pos=dp), 'start-sorted permutation'
    elif case == 'dp_dup':
        dp = _copy(csr.data_pos)
        dp[100] = dp[101]
        over, want = dict(iv_data_pos=dp), 'start-sorted permutation'
    elif case == 'dp_unsorted':
        dp = _copy(csr.data_pos)
        inv = np.argsort(dp)
        a, b = inv[10], inv[2000]                 # swap two data positions of different starts
        assert csr.iv_start[a] != csr.iv_start[b]
        dp[a], dp[b] = dp[b], dp[a]
        over, want = dict(iv_data_pos=dp), 'start-sorted permutation'
    elif case == 'coord_before_read':
        q = _copy(csr.read_qlen2)
        q[0] = -1
        st[5000] = -3
        over, want = dict(read_qlen2=q, iv_start=st), 'interval coordinates'   # columns before reads
    with pytest.raises(_lib.FslrError, match=want):
        _upload(ctx, csr, thr, **over)
    with pytest.raises(_lib.FslrError):
        ctx.build_index()                         # the failed upload left no reads behind
    # a valid upload on the same context: the oracle's graph
    _upload(ctx, csr, thr)
    ctx.reserve_edges(12 * csr.n_reads)
    ctx.build_index()
    st_ = ctx.run_query(1 - 0.04, 1 - 0.25, pass_table(CUTS))
    cnt = np.diff(csr.read_off)
    o = O.run_core(O.OracleCSR(csr.read_off, csr.iv_chrom, csr.iv_start, csr.iv_end, csr.iv_aln,
                               np.repeat(csr.read_qlen2, cnt), np.repeat(csr.read_nal, cnt), csr.data_pos),
                   use_cap=False)
    a, b, I, U = ctx.edges(st_['n_edges'])
    assert sorted(zip(a.tolist(), b.tolist(), I.tolist(), U.tolist())) == \
        sorted(zip(o['edge_a'].tolist(), o['edge_b'].tolist(), o['edge_I'].tolist(), o['edge_U'].tolist()))
    ctx.close()
