"""The CLI's host stages on the CPU: both clustering blocks of ``fslr --skip-alignment`` — the
columnar one (fslr_amd.fastcli, native reader/writer) and the pandas one — against the
reference's own output files for every fixture, with the CPU oracle standing in for the device
query (the GPU CLI tests, tests/test_gpu_parity.py, run the same fixtures through the device).

The oracle is test infrastructure: it replaces ``cluster.build_interval_trees`` /
``cluster.query_graph`` here only, so the host code around the query is what is checked.
"""
import os
import shutil
import tempfile

import numpy as np
import pytest

import fixtures as fx
from fslr_amd import cluster
from oracle import oracle as O


def _oracle_graph(trees, data, overlap, cuts, thr, qlen_diff, diff):
    csr = data.csr()
    cnt = np.diff(csr.read_off)
    oc = O.OracleCSR(csr.read_off, csr.iv_chrom, csr.iv_start, csr.iv_end, csr.iv_aln,
                     np.repeat(csr.read_qlen2, cnt), np.repeat(csr.read_nal, cnt), csr.data_pos)
    o = O.run_core(oc, overlap, cuts, qlen_diff, diff, thr, use_cap=True)
    n = csr.n_reads
    comp = o['comp']
    lab = np.arange(n, dtype=np.int32)
    has = comp >= 0
    if has.any():
        first = np.full(int(comp.max()) + 1, n, np.int64)
        idx = np.flatnonzero(has)
        np.minimum.at(first, comp[idx], idx)
        lab[idx] = first[comp[idx]]
    return cluster.RawGraph(data, csr, lab, o['edge_a'].astype(np.int32), o['edge_b'].astype(np.int32),
                            o['edge_I'].astype(np.int32), o['edge_U'].astype(np.int32), o['fwd'],
                            dict(o['stats'], engine='oracle'))


@pytest.fixture
def oracle_query(monkeypatch):
    monkeypatch.setattr(cluster, 'build_interval_trees', lambda data, device=None, n_gpus=1, ctx=None: None)
    monkeypatch.setattr(cluster, '_open_context', lambda device=None: None)
    monkeypatch.setattr(cluster, 'query_graph', _oracle_graph)


def _run(name, tmp, io_flag):
    from click.testing import CliRunner
    from fslr_amd.main import pipeline
    with open(os.path.join(tmp, 'fx.mappings.bed'), 'w') as fh:
        fh.write(fx.input_bed_text(name))
    shutil.copy(fx.input_bam(name), os.path.join(tmp, 'fx.bwa_dodi.bam'))
    args = ['--name', 'fx', '--out', tmp, '--ref', 'unused.fa', '--primers', '21q1', '--skip-alignment',
            '--timings'] + fx.meta(name)['args'] + [io_flag]
    return CliRunner().invoke(pipeline, args, catch_exceptions=True)


@pytest.mark.parametrize('io_flag', ['--native-io', '--pandas-io'])
@pytest.mark.parametrize('name', fx.FIXTURES)
def test_cli_host_stages_match_reference_outputs(name, io_flag, oracle_query):
    meta = fx.meta(name)
    with tempfile.TemporaryDirectory() as tmp:
        res = _run(name, tmp, io_flag)
        if meta['exception']:
            assert isinstance(res.exception, ZeroDivisionError), res.output
            return
        assert res.exit_code == 0, (res.output, res.exception)
        # the native flag takes the columnar block (fastcli) on every fixture input
        if fx.expected_text(name, 'cluster') is not None:
            assert ('path=columns' in res.output) == (io_flag == '--native-io')
        for which in ('cluster', 'representative'):
            want = fx.expected_text(name, which)
            path = os.path.join(tmp, f'fx.mappings.{which}.bed')
            if want is None:
                assert not os.path.exists(path)
                assert 'No clusters were found.' in res.output
            else:
                assert open(path).read() == want, f'{name}: {which} output differs'
