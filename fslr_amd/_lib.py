"""ctypes binding of ``libfslr_hip.so`` (C ABI: include/fslr_hip.h).

The HIP library is the only compute path: there is no CPU fallback.  If the
shared object is missing or no HIP device is present, every entry point raises
``HipUnavailable`` — loudly, never silently.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

LIB_PATH = os.environ.get('FSLR_LIB') or os.path.join(os.path.dirname(os.path.abspath(__file__)), 'libfslr_hip.so')

ABI_VERSION = 21         # include/fslr_hip.h FSLR_ABI_VERSION this binding is written against
FSLR_OK, FSLR_ERR_ZERO_DIVISION, FSLR_ERR_INVALID, FSLR_ERR_HIP, FSLR_ERR_NOMEM, FSLR_ERR_STATE = range(6)
FSLR_MAX_L = 64
FSLR_MAX_READS = 1 << 25
FSLR_THR_ZERO_ALN = -(1 << 31)
PASS_STRIDE = 2 * FSLR_MAX_L
# pair engines (fslr_params.flags & 3, include/fslr_hip.h)
ENGINES = {'auto': 0, 'walk': 1, 'sweep': 2}
ENGINE_NAMES = {1: 'walk', 2: 'sweep'}

# every symbol include/fslr_hip.h declares (checked by tests/test_abi.py)
EXPORTED = ['fslr_abi_version', 'fslr_last_error', 'fslr_ctx_create', 'fslr_ctx_destroy', 'fslr_set_profiling',
            'fslr_set_reads', 'fslr_set_thresholds', 'fslr_reserve_edges', 'fslr_reserve_deferred',
            'fslr_set_shard', 'fslr_build_index', 'fslr_query', 'fslr_query_shard',
            'fslr_components', 'fslr_run', 'fslr_sync', 'fslr_read_stats', 'fslr_get_timings', 'fslr_read_counters',
            'fslr_get_labels',
            'fslr_get_fwd_degree', 'fslr_get_edges', 'fslr_labels_device_ptr', 'fslr_copy_labels_device',
            'fslr_copy_fwd_device', 'fslr_union_pairs', 'fslr_finalize_labels', 'fslr_apply_edge_cap',
            'fslr_get_pair_kernel_times', 'fslr_set_chrom_filter', 'fslr_sweep_partition', 'fslr_sweep_evaluate',
            'fslr_sweep_partition_repeat',
            'fslr_copy_edges_device', 'fslr_components_from_pairs', 'fslr_set_long_reads', 'fslr_long_query',
            'fslr_get_long_edges', 'fslr_copy_edges_iu_device', 'fslr_cap_install_edges', 'fslr_cap_local',
            'fslr_cap_copy_local', 'fslr_cap_replay', 'fslr_get_stage_kernel_times', 'fslr_long_pairs',
            'fslr_cap_replay_pairs', 'fslr_source_hash', 'fslr_set_reads_any', 'fslr_set_long_cutoffs',
            'fslr_cap_install_pairs', 'fslr_cap_sizes', 'fslr_cap_dep_local', 'fslr_cap_shard_plan',
            'fslr_cap_shard_pack', 'fslr_cap_replay_shard', 'fslr_cap_copy_changes', 'fslr_cap_apply_changes',
            'fslr_local_forest', 'fslr_copy_forest_pairs', 'fslr_sort_edges', 'fslr_cap_bwd_counts',
            'fslr_cap_restrict', 'fslr_cap_copy_restricted', 'fslr_cap_install_restricted', 'fslr_rows_upload',
            'fslr_set_reads_rows', 'fslr_get_read_codes', 'fslr_get_csr', 'fslr_fold_thresholds',
            'fslr_position_costs', 'fslr_position_entries', 'fslr_set_position_filter', 'fslr_use_position_filter', 'fslr_long_pairs_shard',
            'fslr_edge_cap_deferred', 'fslr_edge_cap_deferred_read', 'fslr_set_query_reuse']


class HipUnavailable(RuntimeError):
    pass


class FslrError(RuntimeError):
    pass


class Reads(ctypes.Structure):
    _fields_ = [('n_reads', ctypes.c_int64), ('n_intervals', ctypes.c_int64), ('n_chroms', ctypes.c_int32)] + [
        (f, ctypes.c_void_p) for f in ('read_off', 'read_qlen2', 'read_nal', 'iv_chrom', 'iv_start', 'iv_end',
                                       'iv_thr', 'iv_data_pos')]


class Rows(ctypes.Structure):
    _fields_ = [('n_rows', ctypes.c_int64), ('n_codes', ctypes.c_int64), ('n_chrom_ids', ctypes.c_int64)] + [
        (f, ctypes.c_void_p) for f in ('chrom', 'start', 'end', 'aln', 'qcode', 'nal', 'qlen2')]


class RowsInfo(ctypes.Structure):
    _fields_ = [('n_reads', ctypes.c_int64), ('n_intervals', ctypes.c_int64)] + [
        (f, ctypes.c_int32) for f in ('n_chroms', 'max_len', 'nal_varies', 'general_thresholds', 'any_zero_aln',
                                      'pad')]

    def as_dict(self):
        return {f: int(getattr(self, f)) for f, _ in self._fields_ if f != 'pad'}


class Params(ctypes.Structure):
    _fields_ = [('qlen_cut', ctypes.c_double), ('nal_cut', ctypes.c_double), ('pass_table', ctypes.c_void_p),
                ('edge_threshold', ctypes.c_int32), ('flags', ctypes.c_int32)]


class QueryStats(ctypes.Structure):
    _fields_ = [('evaluated_pairs', ctypes.c_int64), ('jaccard_evals', ctypes.c_int64),
                ('candidates', ctypes.c_int64), ('n_edges', ctypes.c_int64), ('max_fwd', ctypes.c_int32),
                ('error', ctypes.c_int32), ('err_a', ctypes.c_int32), ('err_b', ctypes.c_int32),
                ('algo_bytes', ctypes.c_int64), ('overflow_candidates', ctypes.c_int64),
                ('gather_pairs', ctypes.c_int64), ('match_entries', ctypes.c_int64),
                ('matched_pairs', ctypes.c_int64), ('deferred', ctypes.c_int64),
                ('deferred_capacity', ctypes.c_int64), ('edge_capacity', ctypes.c_int64),
                ('walked_records', ctypes.c_int64), ('engine', ctypes.c_int32), ('overflow_flags', ctypes.c_int32),
                ('pair_tests', ctypes.c_int64), ('entry_capacity', ctypes.c_int64), ('zd_pairs', ctypes.c_int64)]

    def as_dict(self):
        d = {f: getattr(self, f) for f, _ in self._fields_}
        d['engine'] = ENGINE_NAMES.get(d['engine'], d['engine'])
        return d


class CapStats(ctypes.Structure):
    _fields_ = [('applied', ctypes.c_int32), ('max_fwd', ctypes.c_int32)] + [
        (f, ctypes.c_int64) for f in ('candidates', 'capped', 'hits', 'pairs', 'dropped', 'backward')]

    def as_dict(self):
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


class Timings(ctypes.Structure):
    _fields_ = [('index_ms', ctypes.c_float), ('query_ms', ctypes.c_float), ('components_ms', ctypes.c_float),
                ('total_ms', ctypes.c_float), ('pair_kernel_ms', ctypes.c_float), ('sweep_count_ms', ctypes.c_float),
                ('sweep_emit_ms', ctypes.c_float), ('sweep_sort_ms', ctypes.c_float), ('sweep_pairs_ms', ctypes.c_float)]

    def as_dict(self):
        return {f: float(getattr(self, f)) for f, _ in self._fields_}


_lib = None


def load(path: str = LIB_PATH):
    """Load the shared library (no device access)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise HipUnavailable(f'{path} is not built: run `python -c "import __graft_entry__ as g; g.build()"` '
                             '(or `make -C fslr_amd/csrc`).  There is no CPU fallback.')
    L = ctypes.CDLL(path)
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
    sig = {
        'fslr_abi_version': (ctypes.c_int, []),
        'fslr_last_error': (ctypes.c_char_p, [vp]),
        'fslr_ctx_create': (ctypes.c_int, [ctypes.c_int, vp, ctypes.POINTER(vp)]),
        'fslr_ctx_destroy': (None, [vp]),
        'fslr_set_profiling': (ctypes.c_int, [vp, ctypes.c_int]),
        'fslr_set_query_reuse': (ctypes.c_int, [vp, ctypes.c_int]),
        'fslr_set_reads': (ctypes.c_int, [vp, ctypes.POINTER(Reads)]),
        'fslr_set_thresholds': (ctypes.c_int, [vp, vp]),
        'fslr_reserve_edges': (ctypes.c_int, [vp, i64]),
        'fslr_reserve_deferred': (ctypes.c_int, [vp, i64]),
        'fslr_set_shard': (ctypes.c_int, [vp, i32, i32]),
        'fslr_build_index': (ctypes.c_int, [vp]),
        'fslr_query': (ctypes.c_int, [vp, ctypes.POINTER(Params), i64, i64]),
        'fslr_query_shard': (ctypes.c_int, [vp, ctypes.POINTER(Params), i32, i32]),
        'fslr_components': (ctypes.c_int, [vp]),
        'fslr_run': (ctypes.c_int, [vp, ctypes.POINTER(Params)]),
        'fslr_sync': (ctypes.c_int, [vp]),
        'fslr_read_stats': (ctypes.c_int, [vp, ctypes.POINTER(QueryStats)]),
        'fslr_get_timings': (ctypes.c_int, [vp, ctypes.POINTER(Timings)]),
        'fslr_read_counters': (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
        'fslr_get_labels': (ctypes.c_int, [vp, vp]),
        'fslr_get_fwd_degree': (ctypes.c_int, [vp, vp]),
        'fslr_get_edges': (ctypes.c_int, [vp, vp, vp, vp, i64]),
        'fslr_labels_device_ptr': (ctypes.c_int, [vp, ctypes.POINTER(vp)]),
        'fslr_copy_labels_device': (ctypes.c_int, [vp, vp]),
        'fslr_copy_fwd_device': (ctypes.c_int, [vp, vp]),
        'fslr_union_pairs': (ctypes.c_int, [vp, vp, vp, i64, ctypes.c_int]),
        'fslr_finalize_labels': (ctypes.c_int, [vp]),
        'fslr_apply_edge_cap': (ctypes.c_int, [vp, i32, ctypes.POINTER(CapStats)]),
        'fslr_get_pair_kernel_times': (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_float), i32]),
        'fslr_get_stage_kernel_times': (ctypes.c_int, [vp, i32, ctypes.POINTER(ctypes.c_float), i32]),
        'fslr_set_chrom_filter': (ctypes.c_int, [vp, vp]),
        'fslr_sweep_partition': (ctypes.c_int, [vp, ctypes.POINTER(Params), i32, i32, vp, i64,
                                                ctypes.POINTER(ctypes.c_int64)]),
        'fslr_sweep_partition_repeat': (ctypes.c_int, [vp, ctypes.POINTER(Params), i32, i32, vp, i64]),
        'fslr_sweep_evaluate': (ctypes.c_int, [vp, ctypes.POINTER(Params), vp, i64]),
        'fslr_copy_edges_device': (ctypes.c_int, [vp, vp, i64]),
        'fslr_components_from_pairs': (ctypes.c_int, [vp, vp, i64]),
        'fslr_set_long_reads': (ctypes.c_int, [vp, i64, vp, vp, vp, vp, i32]),
        'fslr_set_reads_any': (ctypes.c_int, [vp, ctypes.POINTER(Reads)]),
        'fslr_set_long_cutoffs': (ctypes.c_int, [vp, vp, i32]),
        'fslr_long_query': (ctypes.c_int, [vp, ctypes.POINTER(Params), ctypes.POINTER(ctypes.c_int64)]),
        'fslr_get_long_edges': (ctypes.c_int, [vp, vp, vp, vp, vp, i64]),
        'fslr_long_pairs': (ctypes.c_int, [vp, ctypes.POINTER(Params), ctypes.POINTER(ctypes.c_int64)]),
        'fslr_cap_replay_pairs': (ctypes.c_int, [vp, i32, vp, vp, i64, vp, vp, ctypes.POINTER(CapStats)]),
        'fslr_copy_edges_iu_device': (ctypes.c_int, [vp, vp, i64]),
        'fslr_cap_install_edges': (ctypes.c_int, [vp, vp, i64]),
        'fslr_cap_local': (ctypes.c_int, [vp, i32, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
        'fslr_cap_copy_local': (ctypes.c_int, [vp, vp, vp]),
        'fslr_cap_replay': (ctypes.c_int, [vp, vp, vp, i64, i32, ctypes.POINTER(CapStats)]),
        'fslr_cap_install_pairs': (ctypes.c_int, [vp, vp, i64, i32, i32]),
        'fslr_local_forest': (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int64)]),
        'fslr_sort_edges': (ctypes.c_int, [vp]),
        'fslr_copy_forest_pairs': (ctypes.c_int, [vp, vp, i64]),
        'fslr_cap_sizes': (ctypes.c_int, [vp] + [ctypes.POINTER(ctypes.c_int64)] * 3),
        'fslr_cap_dep_local': (ctypes.c_int, [vp, vp]),
        'fslr_cap_shard_plan': (ctypes.c_int, [vp, vp, i32, i32, vp]),
        'fslr_cap_shard_pack': (ctypes.c_int, [vp, vp, vp]),
        'fslr_cap_replay_shard': (ctypes.c_int, [vp, vp, vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(CapStats)]),
        'fslr_cap_copy_changes': (ctypes.c_int, [vp, vp, i64]),
        'fslr_cap_apply_changes': (ctypes.c_int, [vp, vp, i64, ctypes.POINTER(CapStats)]),
        'fslr_cap_bwd_counts': (ctypes.c_int, [vp, i32, vp, i32]),
        'fslr_cap_restrict': (ctypes.c_int, [vp, vp, i32, ctypes.POINTER(ctypes.c_int64)]),
        'fslr_cap_copy_restricted': (ctypes.c_int, [vp, vp, i64]),
        'fslr_cap_install_restricted': (ctypes.c_int, [vp, vp, i64, i32, i32]),
        'fslr_rows_upload': (ctypes.c_int, [vp, ctypes.POINTER(Rows)]),
        'fslr_set_reads_rows': (ctypes.c_int, [vp, vp, vp, ctypes.c_double, ctypes.POINTER(RowsInfo)]),
        'fslr_get_read_codes': (ctypes.c_int, [vp, vp]),
        'fslr_get_csr': (ctypes.c_int, [vp] + [vp] * 10),
        'fslr_fold_thresholds': (ctypes.c_int, [vp, ctypes.c_double]),
        'fslr_position_costs': (ctypes.c_int, [vp, vp, vp, i64]),
        'fslr_position_entries': (ctypes.c_int, [vp, vp, vp, i64]),
        'fslr_set_position_filter': (ctypes.c_int, [vp, i64, i64, i64]),
        'fslr_use_position_filter': (ctypes.c_int, [vp]),
        'fslr_long_pairs_shard': (ctypes.c_int, [vp, ctypes.POINTER(Params), i32, i32, ctypes.POINTER(ctypes.c_int64)]),
        'fslr_edge_cap_deferred': (ctypes.c_int, [vp, i32]),
        'fslr_edge_cap_deferred_read': (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int32)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.fslr_abi_version() != ABI_VERSION:
        raise HipUnavailable(f'{path} has ABI {L.fslr_abi_version()}, this binding needs {ABI_VERSION}: rebuild it')
    want = source_hash()
    if want is not None and os.environ.get('FSLR_ALLOW_STALE') != '1':
        if not hasattr(L, 'fslr_source_hash'):
            raise HipUnavailable(f'{path} carries no source hash (fslr_source_hash): rebuild it (make -C fslr_amd/csrc), '
                                 f'or set FSLR_ALLOW_STALE=1 to load it anyway')
        L.fslr_source_hash.restype = ctypes.c_char_p
        L.fslr_source_hash.argtypes = []
        got = L.fslr_source_hash().decode()
        if got != want:
            raise HipUnavailable(f'{path} was built from other sources (hash {got}, the sources beside it hash to '
                                 f'{want}): rebuild it (make -C fslr_amd/csrc)')
    _lib = L
    return L


def source_hash():
    """The hash the Makefile embeds (fslr_source_hash): sha256 of the sorted csrc/*.hip and *.hpp, then
    include/fslr_hip.h, first 16 hex digits; None when the sources are not beside the package."""
    import glob
    import hashlib
    here = os.path.dirname(os.path.abspath(__file__))
    csrc = os.path.join(here, 'csrc')
    hdr = os.path.join(os.path.dirname(here), 'include', 'fslr_hip.h')
    files = sorted(os.path.basename(p) for p in glob.glob(os.path.join(csrc, '*.hip')) + glob.glob(os.path.join(csrc, '*.hpp')))
    if not files or not os.path.exists(hdr):
        return None
    h = hashlib.sha256()
    for f in files:
        with open(os.path.join(csrc, f), 'rb') as fh:
            h.update(fh.read())
    with open(hdr, 'rb') as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


_contexts_created = False


def contexts_created() -> bool:
    """True once this process created a Context (the library's HIP runtime is initialised)."""
    return _contexts_created


class Context:
    """One HIP device context (library-owned HBM buffers + a stream)."""

    def __init__(self, device: int = 0, stream: int | None = None, profiling: bool = False):
        """``stream``: a hipStream_t handle (e.g. ``torch.cuda.Stream().cuda_stream``); None or 0
        (the null stream cannot be shared) = the library creates its own stream."""
        self._L = load()
        h = ctypes.c_void_p()
        rc = self._L.fslr_ctx_create(int(device), ctypes.c_void_p(stream) if stream else None, ctypes.byref(h))
        if rc != FSLR_OK:
            raise HipUnavailable(f'fslr_ctx_create(device={device}) failed (rc={rc}): no usable HIP device')
        self._h = h
        global _contexts_created
        _contexts_created = True
        self.device = device
        self.n_reads = 0
        self.edge_capacity = 0
        self._keep = ()
        if profiling:
            self._check(self._L.fslr_set_profiling(self._h, 1))

    def set_query_reuse(self, enable: bool):
        """False: every query does the full work (length-gate ranges, entry-count readback), as a single
        query on new input does; True (default): a repeat on unchanged input keeps them."""
        self._check(self._L.fslr_set_query_reuse(self._h, 1 if enable else 0))

    def set_profiling(self, level: int):
        """1: per-phase events and the pair-kernel events; 2: the pair-kernel events only; 0: off."""
        self._check(self._L.fslr_set_profiling(self._h, int(level)))

    def close(self):
        if getattr(self, '_h', None):
            self._L.fslr_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc == FSLR_OK:
            return
        msg = (self._L.fslr_last_error(self._h) or b'').decode()
        if rc == FSLR_ERR_ZERO_DIVISION:
            raise ZeroDivisionError('division by zero')
        raise FslrError(f'fslr error {rc}: {msg}')

    # -- data -------------------------------------------------------------------------
    def set_reads(self, read_off, read_qlen2, read_nal, iv_chrom, iv_start, iv_end, iv_thr, n_chroms,
                  iv_data_pos=None):
        arrs = [np.ascontiguousarray(x, dtype=np.int32) for x in
                (read_off, read_qlen2, read_nal, iv_chrom, iv_start, iv_end, iv_thr)]
        dp = None if iv_data_pos is None else np.ascontiguousarray(iv_data_pos, dtype=np.int32)
        r = Reads(len(arrs[1]), len(arrs[3]), int(n_chroms), *(_ptr(a) for a in arrs),
                  _ptr(dp) if dp is not None else None)
        self._check(self._L.fslr_set_reads(self._h, ctypes.byref(r)))
        self._data_order = dp is not None
        if arrs[2].size and (arrs[2].min() < 0 or arrs[2].max() >= (1 << 24)):
            raise ValueError('n_alignments must lie in [0, 2**24) for the device path')
        self.n_reads = len(arrs[1])
        self.n_intervals = len(arrs[3])

    def load_csr_any(self, csr, iv_thr):
        """Upload a CSR whose reads may have more than FSLR_MAX_L intervals (fslr_set_reads_any: the
        library splits them into chunks); thresholds here and in set_thresholds are in
        the CSR's own interval order.  Labels and forward degrees then cover the virtual reads (the
        real reads first)."""
        arrs = [np.ascontiguousarray(x, dtype=np.int32) for x in
                (csr.read_off, csr.read_qlen2, csr.read_nal, csr.iv_chrom, csr.iv_start, csr.iv_end, iv_thr)]
        dp = np.ascontiguousarray(csr.data_pos, dtype=np.int32) if getattr(csr, 'start_sorted', True) else None
        r = Reads(len(arrs[1]), len(arrs[3]), int(csr.n_chroms), *(_ptr(a) for a in arrs),
                  _ptr(dp) if dp is not None else None)
        self._check(self._L.fslr_set_reads_any(self._h, ctypes.byref(r)))
        self._data_order = dp is not None
        L = np.diff(arrs[0].astype(np.int64))
        self.n_reads = int(len(arrs[1]) + np.maximum((L + FSLR_MAX_L - 1) // FSLR_MAX_L - 1, 0).sum())
        self.n_intervals = len(arrs[3])

    def rows_upload(self, cols, n_codes, n_chrom_ids):
        """fslr_rows_upload: keep_fillings' rows (``cols``: int64 columns chrom, start, end, aln, qcode,
        nal, qlen2 in file order).  Releases the GIL while it copies (a caller sorts beside it)."""
        names = ('chrom', 'start', 'end', 'aln', 'qcode', 'nal', 'qlen2')
        arrs = [np.ascontiguousarray(cols[k], dtype=np.int64) for k in names]
        self._rows_keep = arrs
        r = Rows(int(arrs[0].size), int(n_codes), int(n_chrom_ids), *(_ptr(a) for a in arrs))
        self._check(self._L.fslr_rows_upload(self._h, ctypes.byref(r)))

    def set_reads_rows(self, order, keep, overlap) -> dict:
        """fslr_set_reads_rows: the reads from the uploaded rows, their start order and mask keep flags
        (None: all); thresholds folded for ``overlap``.  Returns the info dict; raises FslrError (with
        ``info``) when the rows do not fit (a read of more than FSLR_MAX_L intervals)."""
        o = np.ascontiguousarray(order, dtype=np.int64)
        k = None if keep is None else np.ascontiguousarray(keep).view(np.uint8)
        info = RowsInfo()
        rc = self._L.fslr_set_reads_rows(self._h, _ptr(o), _ptr(k) if k is not None else None, float(overlap),
                                         ctypes.byref(info))
        self._rows_keep = None
        d = info.as_dict()
        if rc != FSLR_OK:
            try:
                self._check(rc)
            except FslrError as e:
                e.info = d
                raise
        self.n_reads = d['n_reads']
        self.n_intervals = d['n_intervals']
        self._data_order = True
        return d

    def has_data_order(self) -> bool:
        """The reads came with prepare_data's start-sorted data order (the data-order index build, which
        the chromosome filter and the position split need)."""
        return bool(getattr(self, '_data_order', False))

    def read_codes(self) -> np.ndarray:
        out = np.empty(self.n_reads, np.int64)
        self._check(self._L.fslr_get_read_codes(self._h, _ptr(out)))
        return out

    def device_csr(self, n_intervals: int, n_chroms: int):
        """The CSR a fslr_set_reads_rows context holds, as host arrays (fslr_get_csr)."""
        n, ni = self.n_reads, int(n_intervals)
        out = dict(read_off=np.empty(n + 1, np.int32), read_qlen2=np.empty(n, np.int32), read_nal=np.empty(n, np.int32),
                   iv_chrom=np.empty(ni, np.int32), iv_start=np.empty(ni, np.int32), iv_end=np.empty(ni, np.int32),
                   iv_aln=np.empty(ni, np.int64), iv_thr=np.empty(ni, np.int32), data_pos=np.empty(ni, np.int64))
        out['chrom_ids'] = np.empty(max(1, int(n_chroms)), np.int64)
        self._check(self._L.fslr_get_csr(self._h, *(_ptr(out[k]) for k in ('read_off', 'read_qlen2', 'read_nal',
                                                                        'iv_chrom', 'iv_start', 'iv_end', 'iv_aln',
                                                                        'iv_thr', 'data_pos', 'chrom_ids'))))
        return out

    def fold_thresholds(self, overlap):
        self.thr_gen = getattr(self, 'thr_gen', 0) + 1
        self._check(self._L.fslr_fold_thresholds(self._h, float(overlap)))

    def set_long_cutoffs(self, umax):
        u = np.ascontiguousarray(umax, dtype=np.int32)
        self._check(self._L.fslr_set_long_cutoffs(self._h, _ptr(u), int(u.size)))

    def load_csr(self, csr, iv_thr):
        """Upload a ``fslr_amd.prep.CSR`` (with its start-sorted data order) and thresholds."""
        # the data-order index build needs the list in start order (prepare_data's sort); any other
        # order (a caller-built list) takes the full (chrom, start) sort
        self.set_reads(csr.read_off, csr.read_qlen2, csr.read_nal, csr.iv_chrom, csr.iv_start, csr.iv_end, iv_thr,
                       csr.n_chroms, iv_data_pos=csr.data_pos if getattr(csr, 'start_sorted', True) else None)

    def set_thresholds(self, iv_thr):
        t = np.ascontiguousarray(iv_thr, dtype=np.int32)
        self.thr_gen = getattr(self, 'thr_gen', 0) + 1     # a position plan is cut for the old windows
        self._check(self._L.fslr_set_thresholds(self._h, _ptr(t)))

    def reserve_edges(self, cap):
        self._check(self._L.fslr_reserve_edges(self._h, int(cap)))
        self.edge_capacity = max(self.edge_capacity, int(cap))

    # -- compute (async) ------------------------------------------------------------------
    def _params(self, qlen_cut, nal_cut, pass_table, edge_threshold, engine='auto'):
        pt = np.ascontiguousarray(pass_table, dtype=np.uint8)
        assert pt.size == FSLR_MAX_L * PASS_STRIDE
        self._keep = (pt,)
        return Params(float(qlen_cut), float(nal_cut), _ptr(pt), int(edge_threshold), ENGINES[engine])

    def build_index(self):
        self._check(self._L.fslr_build_index(self._h))

    def query(self, qlen_cut, nal_cut, pass_table, edge_threshold=10, a_begin=0, a_end=None, engine='auto'):
        """``engine``: 'auto' (the sweep when the input allows it and the query covers every read),
        'walk' (counts evaluated_pairs / jaccard_evals) or 'sweep' (fslr_hip.h FSLR_ENGINE_*)."""
        p = self._params(qlen_cut, nal_cut, pass_table, edge_threshold, engine)
        a_end = self.n_reads if a_end is None else a_end
        self._check(self._L.fslr_query(self._h, ctypes.byref(p), int(a_begin), int(a_end)))

    def set_shard(self, shard: int, n_shards: int):
        """Build the query-side index data only for shard `shard` of `n_shards` (fslr_set_shard)."""
        self._check(self._L.fslr_set_shard(self._h, int(shard), int(n_shards)))

    def query_shard(self, qlen_cut, nal_cut, pass_table, shard, n_shards, edge_threshold=10):
        """Query shard `shard` of `n_shards` (rank blocks of 64 dealt round robin; fslr_query_shard)."""
        p = self._params(qlen_cut, nal_cut, pass_table, edge_threshold)
        self._check(self._L.fslr_query_shard(self._h, ctypes.byref(p), int(shard), int(n_shards)))

    # -- multi-GPU sweep (fslr_hip.h fslr_set_chrom_filter / fslr_sweep_partition / _evaluate) ----
    def set_chrom_filter(self, owned):
        """Index only the chromosomes with ``owned[c]`` true at the next build_index (None: all)."""
        if owned is None:
            self._check(self._L.fslr_set_chrom_filter(self._h, None))
            return
        o = np.ascontiguousarray(np.asarray(owned, dtype=bool).astype(np.uint8))
        self._check(self._L.fslr_set_chrom_filter(self._h, _ptr(o)))

    def position_costs(self):
        """(pair tests, forward-window end) per 64-position tile of the full index (fslr_position_costs)."""
        nt = (self.n_intervals + 63) // 64
        tests, reach = np.zeros(nt, np.int64), np.zeros(nt, np.int64)
        self._check(self._L.fslr_position_costs(self._h, _ptr(tests), _ptr(reach), nt))
        return tests, reach

    def position_entries(self, qlen_cut, nal_cut, pass_table, edge_threshold=10):
        """Match entries per 64-position tile of the full index under these parameters
        (fslr_position_entries: a counting sweep)."""
        nt = (self.n_intervals + 63) // 64
        ent = np.zeros(nt, np.int64)
        p = self._params(qlen_cut, nal_cut, pass_table, edge_threshold)
        self._check(self._L.fslr_position_entries(self._h, ctypes.byref(p), _ptr(ent), nt))
        return ent

    def set_position_filter(self, lo, hi, end):
        self._check(self._L.fslr_set_position_filter(self._h, int(lo), int(hi), int(end)))

    def use_position_filter(self):
        self._check(self._L.fslr_use_position_filter(self._h))

    def sweep_partition(self, qlen_cut, nal_cut, pass_table, n_dest, block_shift, dst, edge_threshold=10):
        """Sweep the (filtered) index and write the match entries grouped by destination
        (a >> block_shift) % n_dest into ``dst`` (an int64 device tensor on this context's device).
        Returns (ok, counts[n_dest]); ok False means ``dst`` was too small and nothing usable was
        written: grow it to counts.sum() and call again."""
        p = self._params(qlen_cut, nal_cut, pass_table, edge_threshold)
        counts = np.zeros(int(n_dest), np.int64)
        cap = int(dst.numel())
        rc = self._L.fslr_sweep_partition(self._h, ctypes.byref(p), int(n_dest), int(block_shift),
                                          ctypes.c_void_p(dst.data_ptr()) if cap else None, cap,
                                          counts.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
        if rc == FSLR_ERR_STATE and counts.sum() > cap:
            return False, counts
        self._check(rc)
        return True, counts

    def sweep_partition_repeat(self, qlen_cut, nal_cut, pass_table, n_dest, block_shift, dst, edge_threshold=10):
        """sweep_partition again on unchanged input, parameters and split, without the readback: the
        entries land where the last synchronous call put them (async).  A difference is flagged on
        the device and raised by the next stats() (fslr_sweep_partition_repeat)."""
        p = self._params(qlen_cut, nal_cut, pass_table, edge_threshold)
        self._check(self._L.fslr_sweep_partition_repeat(self._h, ctypes.byref(p), int(n_dest), int(block_shift),
                                                        ctypes.c_void_p(dst.data_ptr()), int(dst.numel())))

    def sweep_evaluate(self, qlen_cut, nal_cut, pass_table, entries, n, edge_threshold=10):
        """Evaluate the pairs of the first ``n`` entries of the int64 device tensor ``entries`` (async)."""
        p = self._params(qlen_cut, nal_cut, pass_table, edge_threshold)
        self._check(self._L.fslr_sweep_evaluate(self._h, ctypes.byref(p),
                                                ctypes.c_void_p(entries.data_ptr()) if n else None, int(n)))

    def labels_into(self, t):
        """Copy the [n_reads] labels into the int32 device tensor ``t`` (async, context stream)."""
        self._check(self._L.fslr_copy_labels_device(self._h, ctypes.c_void_p(t.data_ptr())))

    def edges_into(self, t, n_pad: int):
        """Copy this context's edges as (a, b) int32 pairs into the device tensor ``t`` (at least
        2 * n_pad int32), padded with (-1, -1) to n_pad pairs (async, context stream)."""
        assert t.numel() * t.element_size() >= 8 * n_pad
        self._check(self._L.fslr_copy_edges_device(self._h, ctypes.c_void_p(t.data_ptr()), int(n_pad)))

    def sort_edges(self):
        """This context's edges (with I, U) grouped by lower read, stably, in place."""
        self._check(self._L.fslr_sort_edges(self._h))

    def local_forest(self, count: bool = True):
        """Union-find over this context's edges, keeping the (read, root) pairs of non-root reads; their
        count (one sync) or None (async)."""
        if not count:
            self._check(self._L.fslr_local_forest(self._h, None))
            return None
        k = ctypes.c_int64()
        self._check(self._L.fslr_local_forest(self._h, ctypes.byref(k)))
        return int(k.value)

    def forest_pairs_into(self, t, n_pad: int):
        """The local forest's (read, root) int32 pairs into device tensor ``t`` (int64 view), padded."""
        self._check(self._L.fslr_copy_forest_pairs(self._h, ctypes.c_void_p(t.data_ptr()) if n_pad else None,
                                                   int(n_pad)))

    def components_from_pairs(self, t, n_pairs: int):
        """Labels = components of the n_pairs (a, b) int32 pairs in the device tensor ``t``
        (a < 0 = padding): the union of the ranks' gathered edge lists (async)."""
        self._check(self._L.fslr_components_from_pairs(self._h, ctypes.c_void_p(t.data_ptr()), int(n_pairs)))

    def union_label_vectors(self, t):
        """Union (k mod n_reads, t[k]) for the int32 device tensor ``t`` of W label vectors, then
        finalise the labels (async)."""
        self._check(self._L.fslr_union_pairs(self._h, None, ctypes.c_void_p(t.data_ptr()), int(t.numel()), 1))
        self._check(self._L.fslr_finalize_labels(self._h))

    def apply_edge_cap(self, edge_threshold=10) -> dict:
        """Replay the reference's per-read edge cap (cluster.py:223-224) on the last full query."""
        cs = CapStats()
        self._check(self._L.fslr_apply_edge_cap(self._h, int(edge_threshold), ctypes.byref(cs)))
        return cs.as_dict()

    def edge_cap_deferred(self, edge_threshold=10):
        """The edge-cap check of a repeated query without a host round trip (fslr_edge_cap_deferred)."""
        self._check(self._L.fslr_edge_cap_deferred(self._h, int(edge_threshold)))

    def edge_cap_deferred_read(self) -> int:
        """Sync; the deferred checks' sticky word (1: the cap bound, 2: a ZeroDivisionError pair), cleared."""
        f = ctypes.c_int32()
        self._check(self._L.fslr_edge_cap_deferred_read(self._h, ctypes.byref(f)))
        return int(f.value)

    # -- multi-GPU edge cap (fslr_hip.h fslr_cap_*) ------------------------------------------------
    def edges_iu_into(self, t, n_pad: int):
        """This context's edges as int32 rows {a, b, I | U << 8, 0} into the device tensor ``t`` (at least
        4 * n_pad int32), padded with a = -1 (async)."""
        assert t.numel() * t.element_size() >= 16 * n_pad
        self._check(self._L.fslr_copy_edges_iu_device(self._h, ctypes.c_void_p(t.data_ptr()), int(n_pad)))

    def cap_install_edges(self, t, n_rows: int):
        """The gathered E* rows (device tensor, a < 0 = padding) become this context's edges."""
        self._check(self._L.fslr_cap_install_edges(self._h, ctypes.c_void_p(t.data_ptr()) if n_rows else None,
                                                   int(n_rows)))

    def cap_local(self, edge_threshold=10):
        """Candidates and the search-ordered hits of the candidate intervals this index holds:
        returns (n_ti, n_hits)."""
        nti, nh = ctypes.c_int64(0), ctypes.c_int64(0)
        self._check(self._L.fslr_cap_local(self._h, int(edge_threshold), ctypes.byref(nti), ctypes.byref(nh)))
        return int(nti.value), int(nh.value)

    def cap_copy_local(self, counts, hits):
        self._check(self._L.fslr_cap_copy_local(self._h, ctypes.c_void_p(counts.data_ptr()),
                                                ctypes.c_void_p(hits.data_ptr())))

    def cap_replay(self, counts, hits, pad: int, world: int) -> dict:
        cs = CapStats()
        self._check(self._L.fslr_cap_replay(self._h, ctypes.c_void_p(counts.data_ptr()),
                                            ctypes.c_void_p(hits.data_ptr()), int(pad), int(world),
                                            ctypes.byref(cs)))
        return cs.as_dict()

    # -- multi-GPU edge cap sharded by the candidates' hit components (fslr_hip.h) ----------------
    @staticmethod
    def _dp(t, n):
        return ctypes.c_void_p(t.data_ptr()) if n else None

    def cap_install_pairs(self, t, n_rows: int, world: int, rank: int):
        """The gathered E* (a, b) int32 rows (device tensor; a < 0 = padding), rank w's block at w m."""
        self._check(self._L.fslr_cap_install_pairs(self._h, self._dp(t, n_rows), int(n_rows), int(world), int(rank)))

    def cap_bwd_counts(self, edge_threshold: int, t):
        """This rank's edge counts per upper read into device tensor ``t`` (uint8: clipped at the
        threshold, or int32), for the sum over ranks."""
        eb = t.element_size()
        self._check(self._L.fslr_cap_bwd_counts(self._h, int(edge_threshold), ctypes.c_void_p(t.data_ptr()), eb))

    def cap_restrict(self, t) -> int:
        """The rows of S from the summed counts ``t``; their count (one sync)."""
        k = ctypes.c_int64()
        self._check(self._L.fslr_cap_restrict(self._h, ctypes.c_void_p(t.data_ptr()), t.element_size(),
                                              ctypes.byref(k)))
        return int(k.value)

    def cap_copy_restricted(self, t, n_pad: int):
        self._check(self._L.fslr_cap_copy_restricted(self._h, self._dp(t, n_pad), int(n_pad)))

    def cap_install_restricted(self, t, n_rows: int, world: int, rank: int):
        self._check(self._L.fslr_cap_install_restricted(self._h, self._dp(t, n_rows), int(n_rows), int(world),
                                                        int(rank)))

    def cap_sizes(self):
        """(|T|, T-intervals, local hits) after cap_local."""
        v = [ctypes.c_int64() for _ in range(3)]
        self._check(self._L.fslr_cap_sizes(self._h, *[ctypes.byref(x) for x in v]))
        return tuple(int(x.value) for x in v)

    def cap_dep_local(self, t):
        """t[0 .. 2|T|) (int32 device): local forest roots of T reads, then their local hit counts."""
        self._check(self._L.fslr_cap_dep_local(self._h, ctypes.c_void_p(t.data_ptr())))

    def cap_shard_plan(self, gathered, world: int, rank: int):
        """The components' ranks; returns (T-intervals per destination, local hits per destination)."""
        sizes = np.zeros(2 * world, np.int64)
        self._check(self._L.fslr_cap_shard_plan(self._h, ctypes.c_void_p(gathered.data_ptr()), int(world), int(rank),
                                                _ptr(sizes)))
        return sizes[:world].copy(), sizes[world:].copy()

    def cap_shard_pack(self, counts, hits):
        self._check(self._L.fslr_cap_shard_pack(self._h, ctypes.c_void_p(counts.data_ptr()),
                                                ctypes.c_void_p(hits.data_ptr())))

    def cap_replay_shard(self, counts, hits):
        """Replay this rank's components from the received lists; returns (changes, partial cap stats)."""
        nch = ctypes.c_int64()
        cs = CapStats()
        self._check(self._L.fslr_cap_replay_shard(self._h, ctypes.c_void_p(counts.data_ptr()),
                                                  ctypes.c_void_p(hits.data_ptr()), ctypes.byref(nch), ctypes.byref(cs)))
        return int(nch.value), cs.as_dict()

    def cap_copy_changes(self, t, n_pad: int):
        self._check(self._L.fslr_cap_copy_changes(self._h, self._dp(t, n_pad), int(n_pad)))

    def cap_apply_changes(self, t, n: int) -> dict:
        cs = CapStats()
        self._check(self._L.fslr_cap_apply_changes(self._h, self._dp(t, n), int(n), ctypes.byref(cs)))
        return cs.as_dict()

    def components(self):
        self._check(self._L.fslr_components(self._h))

    def run(self, qlen_cut, nal_cut, pass_table, edge_threshold=10, engine='auto'):
        p = self._params(qlen_cut, nal_cut, pass_table, edge_threshold, engine)
        self._check(self._L.fslr_run(self._h, ctypes.byref(p)))

    def sync(self):
        self._check(self._L.fslr_sync(self._h))

    # -- results ------------------------------------------------------------------------
    def reserve_deferred(self, cap):
        self._check(self._L.fslr_reserve_deferred(self._h, int(cap)))

    def stats(self, check: bool = True) -> dict:
        """Counters of the last query.  With ``check`` a buffer overflow raises FslrError;
        ``run_query`` grows the buffers and reruns instead."""
        s = QueryStats()
        rc = self._L.fslr_read_stats(self._h, ctypes.byref(s))
        if rc == FSLR_ERR_STATE and not check:
            return s.as_dict()
        self._check(rc)
        return s.as_dict()

    def run_query(self, qlen_cut, nal_cut, pass_table, edge_threshold=10, a_begin=0, a_end=None,
                  engine='auto') -> dict:
        """query + stats, growing the edge / deferred buffers and rerunning on overflow (and with the
        walk engine if the sweep's per-read partner table overflowed)."""
        while True:
            self.query(qlen_cut, nal_cut, pass_table, edge_threshold, a_begin, a_end, engine)
            st = self.stats(check=False)
            grow = False
            if st['overflow_flags'] & 4:
                engine = 'walk'
                grow = True
            if st['overflow_flags'] & 24:         # sweep entry buffers (a sync-free repeat query): rerun
                grow = True
            if st['overflow_flags'] & 64:         # the ZeroDivisionError pair list (the cap binds): rerun
                grow = True
            if st['n_edges'] > st['edge_capacity']:
                self.reserve_edges(int(st['n_edges'] * 1.25) + 4096)
                grow = True
            if st['deferred'] > st['deferred_capacity']:
                self.reserve_deferred(int(st['deferred'] * 1.25) + 4096)
                grow = True
            if not grow:
                self.stats()          # raises on a device-side error (ZeroDivisionError)
                return st

    def timings(self) -> dict:
        t = Timings()
        self._check(self._L.fslr_get_timings(self._h, ctypes.byref(t)))
        return t.as_dict()

    def pair_kernel_times(self, n: int = 256) -> np.ndarray:
        """Durations (ms) of the main pair-kernel launch of the last ``n`` queries (profiling contexts)."""
        out = np.zeros(n, np.float32)
        got = self._L.fslr_get_pair_kernel_times(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n)
        if got < 0:
            self._check(-got)
        return out[:got]

    def stage_kernel_times(self, stage: int, n: int = 256) -> np.ndarray:
        """Durations (ms) of one stage kernel of the last ``n`` queries: 0 the main pair kernel, 1 the sweep
        engine's pair-stage kernel (profiling contexts)."""
        out = np.zeros(n, np.float32)
        got = self._L.fslr_get_stage_kernel_times(self._h, int(stage),
                                                  out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n)
        if got < 0:
            self._check(-got)
        return out[:got]

    def counters(self, n: int = 80) -> np.ndarray:
        """Raw device counters of the last query (kernels.hpp Counter; diagnostics)."""
        out = np.zeros(n, np.uint64)
        got = self._L.fslr_read_counters(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n)
        if got < 0:
            self._check(-got)
        return out[:got]

    def labels(self) -> np.ndarray:
        out = np.empty(self.n_reads, np.int32)
        self._check(self._L.fslr_get_labels(self._h, _ptr(out)))
        return out

    def fwd_degree(self) -> np.ndarray:
        out = np.empty(self.n_reads, np.int32)
        self._check(self._L.fslr_get_fwd_degree(self._h, _ptr(out)))
        return out

    def edges(self, n_edges: int):
        a = np.empty(n_edges, np.int32)
        b = np.empty(n_edges, np.int32)
        iu = np.empty(n_edges, np.uint16)
        self._check(self._L.fslr_get_edges(self._h, _ptr(a), _ptr(b), _ptr(iu), int(n_edges)))
        return a, b, (iu & 0xff).astype(np.int32), (iu >> 8).astype(np.int32)

    def labels_device_ptr(self) -> int:
        p = ctypes.c_void_p()
        self._check(self._L.fslr_labels_device_ptr(self._h, ctypes.byref(p)))
        return p.value

    def copy_labels_device(self, dptr: int):
        self._check(self._L.fslr_copy_labels_device(self._h, ctypes.c_void_p(dptr)))

    def copy_fwd_device(self, dptr: int):
        self._check(self._L.fslr_copy_fwd_device(self._h, ctypes.c_void_p(dptr)))

    def union_pairs(self, src, dst, n, on_device: bool):
        """Union (src[k], dst[k]); ``src`` None means src[k] = k mod n_reads.  Pointers are ints when on_device."""
        if on_device:
            self._check(self._L.fslr_union_pairs(self._h, ctypes.c_void_p(src) if src else None,
                                                 ctypes.c_void_p(dst), int(n), 1))
        else:
            s = None if src is None else np.ascontiguousarray(src, np.int32)
            d = np.ascontiguousarray(dst, np.int32)
            self._check(self._L.fslr_union_pairs(self._h, _ptr(s) if s is not None else None, _ptr(d), int(n), 0))

    # -- reads of more than FSLR_MAX_L intervals (fslr_hip.h fslr_set_long_reads / fslr_long_query) --
    def set_long_reads(self, n_real, vreal, vbase, rlen, umax):
        arrs = [np.ascontiguousarray(x, dtype=np.int32) for x in (vreal, vbase, rlen, umax)]
        self._check(self._L.fslr_set_long_reads(self._h, int(n_real), *(_ptr(a) for a in arrs), int(arrs[3].size)))

    def long_query(self, qlen_cut, nal_cut, pass_table, edge_threshold=10) -> int:
        """Sweep the virtual index and decide every pair (fslr_long_query); returns the long-pair edge count."""
        p = self._params(qlen_cut, nal_cut, pass_table, edge_threshold)
        ne = ctypes.c_int64(0)
        self._check(self._L.fslr_long_query(self._h, ctypes.byref(p), ctypes.byref(ne)))
        return int(ne.value)

    def long_pairs(self, qlen_cut, nal_cut, pass_table, edge_threshold=10) -> int:
        """Decide every distinct pair with the general evaluator (fslr_long_pairs); returns the edge count."""
        p = self._params(qlen_cut, nal_cut, pass_table, edge_threshold)
        ne = ctypes.c_int64(0)
        self._check(self._L.fslr_long_pairs(self._h, ctypes.byref(p), ctypes.byref(ne)))
        return int(ne.value)

    def long_pairs_shard(self, qlen_cut, nal_cut, pass_table, shard, n_shards, edge_threshold=10) -> int:
        """fslr_long_pairs for the pairs whose lower read lies in query shard ``shard`` of ``n_shards``."""
        p = self._params(qlen_cut, nal_cut, pass_table, edge_threshold)
        ne = ctypes.c_int64(0)
        self._check(self._L.fslr_long_pairs_shard(self._h, ctypes.byref(p), int(shard), int(n_shards),
                                                  ctypes.byref(ne)))
        return int(ne.value)

    def cap_replay_pairs(self, edge_threshold, a, b, n_reads: int):
        """The edge cap over the E* pairs (a < b): returns (who, fwd, cap stats) — fslr_cap_replay_pairs."""
        a = np.ascontiguousarray(a, np.int32)
        b = np.ascontiguousarray(b, np.int32)
        who = np.empty(a.shape[0], np.uint8)
        fwd = np.empty(int(n_reads), np.int32)
        cs = CapStats()
        self._check(self._L.fslr_cap_replay_pairs(self._h, int(edge_threshold), _ptr(a), _ptr(b), int(a.shape[0]),
                                                  _ptr(who), _ptr(fwd), ctypes.byref(cs)))
        return who, fwd, cs.as_dict()

    def long_edges(self, n_edges: int):
        out = [np.empty(n_edges, np.int32) for _ in range(4)]
        self._check(self._L.fslr_get_long_edges(self._h, *(_ptr(a) for a in out), int(n_edges)))
        return tuple(out)

    def finalize_labels(self):
        self._check(self._L.fslr_finalize_labels(self._h))
