"""The C-ABI library loads and exports every entry point include/sparkey_gpu.h declares; host-side
logic that needs no GPU (index sizing, header validation) matches the oracle.  CPU only.
"""
import ctypes
import os
import re

import pytest

import oracle
from helpers import key_value_puts, make_log

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "sparkey_gpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sparkey_\w+)\s*\(", src)))


def test_exports_every_declared_symbol(native):
    lib = ctypes.CDLL(native.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 12
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(native.EXPORTED) == names


def test_version(native):
    assert "gfx950" in native.version()


@pytest.mark.parametrize("n,hs,sp", [(0, 0, 0.0), (1000, 0, 0.0), (1000, 8, 2.5), (9000, 4, 1.3), (3, 0, 1.0)])
def test_index_size_matches_oracle(native, oracle_mod, n, hs, sp):
    log = make_log(key_value_puts(n))
    opts = native.make_opts(hash_size=hs, hash_seed=1, sparsity=sp)
    assert native.index_size(log[:84], opts) == oracle.index_size(log, hs, sp)


def test_index_size_header_errors(native):
    opts = native.make_opts(hash_seed=1)
    log = bytearray(make_log(key_value_puts(5)))
    with pytest.raises(OSError):
        native.index_size(b"\0" * 84, opts)
    log[8] = 1  # minor version > 0
    with pytest.raises(OSError):
        native.index_size(bytes(log), opts)
    with pytest.raises(ValueError):
        native.index_size(make_log(key_value_puts(5))[:84], native.make_opts(hash_size=5))


def test_package_imports_without_fallback(native):
    import sparkey
    assert sparkey.Sparkey.getIndexFile("/tmp/x") == "/tmp/x.spi"
    assert sparkey.Sparkey.getLogFile("/tmp/x.spi") == "/tmp/x.spl"
    assert sparkey.Sparkey.setEnding("/tmp/x.", ".spl") == "/tmp/x.spl"
