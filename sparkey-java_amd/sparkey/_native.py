"""ctypes binding of libsparkey_gpu.so (include/sparkey_gpu.h).

The hash-file build has no CPU fallback: if the HIP library is missing this module raises at
import time, and every build call goes through the GPU.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SPARKEY_GPU_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libsparkey_gpu.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(f"libsparkey_gpu.so not built ({LIB_PATH}); run python sparkey-java_amd/build.py")

_lib = ctypes.CDLL(LIB_PATH)

OK = 0
E_NOT_LOG = -1
E_VERSION = -2
E_CORRUPT_LOG = -3
E_NO_FREE_SLOTS = -4
E_CORRUPT_DATA = -5
E_VLQ = -6
E_HEADER = -7
E_UNSUPPORTED = -8
E_IO = -9
E_GPU = -10
E_ARG = -11
E_BUFFER = -12

METHOD_AUTO = 0
METHOD_IN_MEMORY = 1
METHOD_SORTING = 2


class BuildOpts(ctypes.Structure):
    _fields_ = [("hash_size", ctypes.c_int32), ("hash_seed", ctypes.c_int32), ("sparsity", ctypes.c_double),
                ("max_memory", ctypes.c_int64), ("method", ctypes.c_int32), ("device", ctypes.c_int32)]


class BuildStats(ctypes.Structure):
    _fields_ = [("num_records", ctypes.c_int64), ("num_puts", ctypes.c_int64), ("num_deletes", ctypes.c_int64),
                ("num_entries", ctypes.c_int64), ("capacity", ctypes.c_int64), ("garbage_size", ctypes.c_int64),
                ("max_displacement", ctypes.c_int64), ("hash_collisions", ctypes.c_int64),
                ("total_displacement", ctypes.c_int64), ("hash_size", ctypes.c_int32),
                ("address_size", ctypes.c_int32), ("placement_path", ctypes.c_int32),
                ("framing_path", ctypes.c_int32), ("device_ms", ctypes.c_double)]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}


_vp = ctypes.c_void_p
_lib.sparkey_build_index_file.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(BuildOpts), ctypes.c_int32,
                                          ctypes.POINTER(BuildStats), ctypes.c_char_p, ctypes.c_size_t]
_lib.sparkey_build_index_file.restype = ctypes.c_int
_lib.sparkey_build_index_mem.argtypes = [_vp, ctypes.c_uint64, _vp, ctypes.c_uint64, ctypes.POINTER(BuildOpts),
                                         ctypes.POINTER(BuildStats), ctypes.c_char_p, ctypes.c_size_t]
_lib.sparkey_build_index_mem.restype = ctypes.c_int
_lib.sparkey_index_size.argtypes = [_vp, ctypes.c_uint64, ctypes.POINTER(BuildOpts)]
_lib.sparkey_index_size.restype = ctypes.c_int64
_lib.sparkey_plan_create.argtypes = [ctypes.POINTER(_vp), ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint64,
                                     ctypes.c_char_p, ctypes.c_size_t]
_lib.sparkey_plan_create.restype = ctypes.c_int
_lib.sparkey_plan_build_device.argtypes = [_vp, _vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64,
                                           ctypes.POINTER(BuildOpts), _vp, ctypes.POINTER(BuildStats),
                                           ctypes.c_char_p, ctypes.c_size_t]
_lib.sparkey_plan_build_device.restype = ctypes.c_int
_lib.sparkey_plan_set_profiling.argtypes = [_vp, ctypes.c_int32]
_lib.sparkey_plan_set_profiling.restype = None
_lib.sparkey_plan_stage_count.argtypes = [_vp]
_lib.sparkey_plan_stage_count.restype = ctypes.c_int32
_lib.sparkey_plan_stage_name.argtypes = [_vp, ctypes.c_int32]
_lib.sparkey_plan_stage_name.restype = ctypes.c_char_p
_lib.sparkey_plan_stage_ms.argtypes = [_vp, ctypes.c_int32]
_lib.sparkey_plan_stage_ms.restype = ctypes.c_double
_lib.sparkey_plan_destroy.argtypes = [_vp]
_lib.sparkey_plan_destroy.restype = None
_lib.sparkey_gpu_version.argtypes = []
_lib.sparkey_gpu_version.restype = ctypes.c_char_p
_lib.sparkey_strerror.argtypes = [ctypes.c_int]
_lib.sparkey_strerror.restype = ctypes.c_char_p

EXPORTED = ["sparkey_build_index_file", "sparkey_build_index_mem", "sparkey_index_size", "sparkey_plan_create",
            "sparkey_plan_build_device", "sparkey_plan_set_profiling", "sparkey_plan_stage_count",
            "sparkey_plan_stage_name", "sparkey_plan_stage_ms", "sparkey_plan_destroy", "sparkey_gpu_version",
            "sparkey_strerror"]


class SparkeyIOError(OSError):
    """The reference throws java.io.IOException for these codes."""


class SparkeyRuntimeError(RuntimeError):
    """The reference throws RuntimeException for these codes."""


class SparkeyGpuError(RuntimeError):
    """HIP runtime failure (no reference counterpart)."""


_IO_CODES = {E_NOT_LOG, E_VERSION, E_CORRUPT_LOG, E_NO_FREE_SLOTS, E_HEADER, E_IO, E_UNSUPPORTED}
_RUNTIME_CODES = {E_CORRUPT_DATA, E_VLQ}


def raise_for(code: int, msg: str):
    text = f"{msg} [code {code}]"
    if code in _IO_CODES:
        err = SparkeyIOError(text)
    elif code in _RUNTIME_CODES:
        err = SparkeyRuntimeError(text)
    elif code == E_ARG:
        err = ValueError(text)
    elif code == E_BUFFER:
        err = ValueError(text)
    else:
        err = SparkeyGpuError(text)
    err.code = code
    raise err


def make_opts(hash_size=0, hash_seed=0, sparsity=0.0, max_memory=1 << 62, method=METHOD_IN_MEMORY, device=0):
    return BuildOpts(hash_size, ctypes.c_int32(hash_seed).value, float(sparsity), int(max_memory), int(method),
                     int(device))


def index_size(log_header: bytes, opts: BuildOpts) -> int:
    n = _lib.sparkey_index_size(log_header, len(log_header), ctypes.byref(opts))
    if n < 0:
        raise_for(int(n), _lib.sparkey_strerror(int(n)).decode())
    return int(n)


def build_index_file(log_path: str, index_path: str, opts: BuildOpts, fsync: bool = False) -> BuildStats:
    stats = BuildStats()
    err = ctypes.create_string_buffer(512)
    rc = _lib.sparkey_build_index_file(os.fsencode(log_path), os.fsencode(index_path), ctypes.byref(opts),
                                       1 if fsync else 0, ctypes.byref(stats), err, 512)
    if rc != OK:
        raise_for(rc, err.value.decode(errors="replace"))
    return stats


def build_index_mem(log: bytes, opts: BuildOpts):
    """Host bytes in, (.spi bytes, BuildStats) out."""
    n = index_size(log[:84], opts) if len(log) >= 84 else 112
    out = ctypes.create_string_buffer(max(n, 1))
    stats = BuildStats()
    err = ctypes.create_string_buffer(512)
    rc = _lib.sparkey_build_index_mem(log, len(log), out, n, ctypes.byref(opts), ctypes.byref(stats), err, 512)
    if rc != OK:
        raise_for(rc, err.value.decode(errors="replace"))
    return out.raw[:n], stats


def version() -> str:
    return _lib.sparkey_gpu_version().decode()


class Plan:
    """Device-resident builds: workspace kept across calls (bench / embedding)."""

    def __init__(self, device: int = 0, max_log_bytes: int = 0, max_records: int = 0):
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(512)
        rc = _lib.sparkey_plan_create(ctypes.byref(h), device, max_log_bytes, max_records, err, 512)
        if rc != OK:
            raise_for(rc, err.value.decode(errors="replace"))
        self._h = h

    def build(self, log_header: bytes, d_log: int, log_len: int, d_out: int, out_cap: int, opts: BuildOpts,
              stream: int = 0) -> BuildStats:
        stats = BuildStats()
        err = ctypes.create_string_buffer(512)
        rc = _lib.sparkey_plan_build_device(self._h, log_header, ctypes.c_void_p(d_log), log_len,
                                            ctypes.c_void_p(d_out), out_cap, ctypes.byref(opts),
                                            ctypes.c_void_p(stream), ctypes.byref(stats), err, 512)
        if rc != OK:
            raise_for(rc, err.value.decode(errors="replace"))
        return stats

    def set_profiling(self, enabled: bool) -> None:
        _lib.sparkey_plan_set_profiling(self._h, 1 if enabled else 0)

    def stage_times(self):
        n = _lib.sparkey_plan_stage_count(self._h)
        return [(_lib.sparkey_plan_stage_name(self._h, i).decode(), _lib.sparkey_plan_stage_ms(self._h, i))
                for i in range(n)]

    def close(self) -> None:
        if self._h:
            _lib.sparkey_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
