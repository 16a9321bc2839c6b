"""The C-ABI library loads and exports every symbol include/fslr_hip.h declares (no device calls)."""
import ctypes
import os
import re
import shutil
import subprocess

import pytest

from fslr_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, 'include', 'fslr_hip.h')


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r'^\s*(?:int|void|const char)\s+\*?\s*(fslr_\w+)\s*\(', text, re.M)))


@pytest.fixture(scope='module')
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(['make', '-s', '-C', os.path.join(REPO, 'fslr_amd', 'csrc')], check=True)
    return _lib.load()


def test_header_matches_binding_list():
    assert declared_symbols() == sorted(_lib.EXPORTED)


def test_library_exports_all_symbols(lib):
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_abi_version(lib):
    assert lib.fslr_abi_version() == _lib.ABI_VERSION == 21


def test_gfx950_code_object_present(tmp_path):
    # --offloading extracts the bundled code objects next to its input: run it on a copy
    lib_copy = tmp_path / 'libfslr_hip.so'
    shutil.copy(_lib.LIB_PATH, lib_copy)
    out = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-objdump', '--offloading', str(lib_copy)], capture_output=True,
                         text=True)
    if out.returncode != 0:  # older objdump: fall back to a byte search of the embedded bundle
        assert b'gfx950' in open(_lib.LIB_PATH, 'rb').read()
    else:
        assert 'gfx950' in out.stdout + out.stderr or b'gfx950' in open(_lib.LIB_PATH, 'rb').read()


def test_null_context_is_rejected(lib):
    lib.fslr_set_reads.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    assert lib.fslr_set_reads(None, None) == _lib.FSLR_ERR_INVALID
    _lib._lib = None     # restore full signatures for later tests
