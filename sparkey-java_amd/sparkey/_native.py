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



def _preload_torch_hip() -> None:
    """One HIP runtime per process: when PyTorch is installed, load the libamdhip64 it bundles
    before ours, so libsparkey_gpu.so binds to it (same SONAME) whichever of the two is imported
    first.  Two runtimes in one process do not see the same devices."""
    if os.environ.get("SPARKEY_GPU_SYSTEM_HIP"):
        return
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    path = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(path):
        ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


_preload_torch_hip()
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
E_CORRUPT_RECORD = -13  # RuntimeException from the log iterator (SparkeyLogIterator.java:117-136)

METHOD_AUTO = 0
METHOD_IN_MEMORY = 1
METHOD_SORTING = 2


class BuildOpts(ctypes.Structure):
    _fields_ = [("hash_size", ctypes.c_int32), ("hash_seed", ctypes.c_int32), ("sparsity", ctypes.c_double),
                ("max_memory", ctypes.c_int64), ("method", ctypes.c_int32), ("device", ctypes.c_int32),
                ("num_gpus", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class BuildStats(ctypes.Structure):
    _fields_ = [("num_records", ctypes.c_int64), ("num_puts", ctypes.c_int64), ("num_deletes", ctypes.c_int64),
                ("num_entries", ctypes.c_int64), ("capacity", ctypes.c_int64), ("garbage_size", ctypes.c_int64),
                ("max_displacement", ctypes.c_int64), ("hash_collisions", ctypes.c_int64),
                ("total_displacement", ctypes.c_int64), ("hash_size", ctypes.c_int32),
                ("address_size", ctypes.c_int32), ("placement_path", ctypes.c_int32),
                ("framing_path", ctypes.c_int32), ("partition_passes", ctypes.c_int32),
                ("sharded", ctypes.c_int32), ("device_ms", ctypes.c_double), ("entry_bytes", ctypes.c_int32),
                ("reserved0", ctypes.c_int32)]

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
_lib.sparkey_release_cached_resources.argtypes = []
_lib.sparkey_release_cached_resources.restype = None
_lib.sparkey_shard_comm_unique_id.argtypes = [_vp, ctypes.c_char_p, ctypes.c_size_t]
_lib.sparkey_shard_comm_unique_id.restype = ctypes.c_int
_lib.sparkey_shard_comm_create.argtypes = [ctypes.POINTER(_vp), _vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_char_p, ctypes.c_size_t]
_lib.sparkey_shard_comm_create.restype = ctypes.c_int
_AG_FN = ctypes.CFUNCTYPE(ctypes.c_int, _vp, _vp, _vp, ctypes.c_uint64)
_A2A_FN = ctypes.CFUNCTYPE(ctypes.c_int, _vp, _vp, ctypes.POINTER(ctypes.c_uint64), _vp, ctypes.POINTER(ctypes.c_uint64))


class ShardTransport(ctypes.Structure):
    _fields_ = [("ctx", _vp), ("all_gather", _AG_FN), ("all_to_all", _A2A_FN)]


_lib.sparkey_shard_comm_create_host.argtypes = [ctypes.POINTER(_vp), ctypes.POINTER(ShardTransport), ctypes.c_int32,
                                                ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p, ctypes.c_size_t]
_lib.sparkey_shard_comm_create_host.restype = ctypes.c_int
_lib.sparkey_build_index_sharded_device.argtypes = [_vp, ctypes.c_uint64, ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                                                    ctypes.POINTER(BuildOpts), ctypes.POINTER(BuildStats),
                                                    ctypes.c_char_p, ctypes.c_size_t]
_lib.sparkey_build_index_sharded_device.restype = ctypes.c_int
_lib.sparkey_shard_comm_destroy.argtypes = [_vp]
_lib.sparkey_shard_comm_destroy.restype = None
_lib.sparkey_shard_geometry.argtypes = [_vp, ctypes.c_uint64, ctypes.POINTER(BuildOpts), ctypes.c_int32, ctypes.c_int32,
                                        ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                        ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                        ctypes.c_char_p, ctypes.c_size_t]
_lib.sparkey_shard_geometry.restype = ctypes.c_int
_lib.sparkey_shard_build.argtypes = [_vp, _vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64, ctypes.c_uint64,
                                     ctypes.POINTER(BuildOpts), _vp, ctypes.c_uint64, _vp, ctypes.POINTER(BuildStats),
                                     ctypes.c_char_p, ctypes.c_size_t]
_lib.sparkey_shard_build.restype = ctypes.c_int
_lib.sparkey_shard_phase_count.argtypes = [_vp]
_lib.sparkey_shard_phase_count.restype = ctypes.c_int32
_lib.sparkey_shard_phase_name.argtypes = [_vp, ctypes.c_int32]
_lib.sparkey_shard_phase_name.restype = ctypes.c_char_p
_lib.sparkey_shard_phase_ms.argtypes = [_vp, ctypes.c_int32]
_lib.sparkey_shard_phase_ms.restype = ctypes.c_double
_lib.sparkey_multi_phase_count.argtypes = [ctypes.c_int32]
_lib.sparkey_multi_phase_count.restype = ctypes.c_int32
_lib.sparkey_multi_phase_name.argtypes = [ctypes.c_int32, ctypes.c_int32]
_lib.sparkey_multi_phase_name.restype = ctypes.c_char_p
_lib.sparkey_multi_phase_ms.argtypes = [ctypes.c_int32, ctypes.c_int32]
_lib.sparkey_multi_phase_ms.restype = ctypes.c_double


_lib.sparkey_file_last_phases.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int32]
_lib.sparkey_file_last_phases.restype = ctypes.c_int32
_lib.sparkey_debug_set.argtypes = [ctypes.c_char_p, ctypes.c_int64]
_lib.sparkey_debug_set.restype = ctypes.c_int
_lib.sparkey_debug_get.argtypes = [ctypes.c_char_p]
_lib.sparkey_debug_get.restype = ctypes.c_int64


def debug_set(name: str, value) -> None:
    """Sets a test / diagnostic switch (csrc/knobs.hpp; None or a negative value unsets it).  No switch
    changes a build's bytes: each forces a device path or geometry the default choice would not take."""
    v = -1 if value is None or value is False else (1 if value is True else int(value))
    if _lib.sparkey_debug_set(name.encode(), v) != OK:
        raise ValueError(f"unknown switch {name!r}")


def debug_get(name: str) -> int:
    v = int(_lib.sparkey_debug_get(name.encode()))
    if v == E_ARG:
        raise ValueError(f"unknown switch {name!r}")
    return v


class debug:
    """with debug(no_uniform=1, serial_framing=1): ... -- switches set for the block, restored after."""

    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.old = {k: debug_get(k) for k in self.kv}
        for k, v in self.kv.items():
            debug_set(k, v)
        return self

    def __exit__(self, *a):
        for k, v in self.old.items():
            debug_set(k, v)


def file_last_phases() -> dict:
    """Phases (ms) of this thread's last single-GPU build_index_file."""
    v = (ctypes.c_double * 5)()
    _lib.sparkey_file_last_phases(v, 5)
    return dict(zip(("open_header", "read_h2d", "build", "d2h_write", "fsync_close"), [float(x) for x in v]))


def multi_last_phases(rank: int) -> list:
    """[(phase, ms)] of rank `rank` of this process's last num_gpus > 1 build."""
    return [(_lib.sparkey_multi_phase_name(rank, i).decode(), _lib.sparkey_multi_phase_ms(rank, i))
            for i in range(_lib.sparkey_multi_phase_count(rank))]


def shard_unique_id() -> bytes:
    """An RCCL unique id (128 bytes) for sparkey_shard_comm_create; made on one rank, sent to all."""
    buf = ctypes.create_string_buffer(128)
    err = ctypes.create_string_buffer(512)
    rc = _lib.sparkey_shard_comm_unique_id(buf, err, 512)
    if rc != OK:
        raise_for(rc, err.value.decode(errors="replace"))
    return buf.raw


def _torch_transport(group=None) -> ShardTransport:
    """sparkey_shard_transport over torch.distributed (the default group, or `group`) on host buffers."""
    import numpy as np
    import torch
    import torch.distributed as dist

    def view(ptr, n):
        if n == 0:
            return torch.empty(0, dtype=torch.uint8)
        return torch.from_numpy(np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(ptr)))

    def all_gather(ctx, send, recv, nbytes):
        try:
            w = dist.get_world_size(group)
            if nbytes:
                dist.all_gather_into_tensor(view(recv, nbytes * w), view(send, nbytes).clone(), group=group)
            return 0
        except Exception:  # noqa: BLE001  (reported to the library as a failed collective)
            return 1

    def all_to_all(ctx, send, send_bytes, recv, recv_bytes):
        try:
            w = dist.get_world_size(group)
            sb = [int(send_bytes[r]) for r in range(w)]
            rb = [int(recv_bytes[r]) for r in range(w)]
            inp = view(send, sum(sb)).clone()
            out = torch.empty(sum(rb), dtype=torch.uint8)
            dist.all_to_all_single(out, inp, rb, sb, group=group)
            if sum(rb):
                view(recv, sum(rb)).copy_(out)
            return 0
        except Exception:  # noqa: BLE001
            return 1

    t = ShardTransport(None, _AG_FN(all_gather), _A2A_FN(all_to_all))
    t._keep = (all_gather, all_to_all)
    return t


def build_index_sharded_device(log_header: bytes, file_len: int, d_bufs, d_outs, opts: BuildOpts) -> BuildStats:
    """The multi-GPU build over device-resident log ranges (sparkey_build_index_sharded_device):
    d_bufs[r] / d_outs[r] are device addresses of rank r's log range and .spi part
    (shard_geometry(..., r, opts.num_gpus))."""
    n = len(d_bufs)
    if n != len(d_outs) or n != max(1, int(opts.num_gpus)):
        # (the library reads d_bufs[rank] / d_outs[rank] for every rank < num_gpus)
        raise ValueError(f"build_index_sharded_device: {len(d_bufs)} log ranges and {len(d_outs)} outputs "
                         f"for num_gpus = {int(opts.num_gpus)}")
    bufs = (_vp * n)(*[ctypes.c_void_p(int(x)) for x in d_bufs])
    outs = (_vp * n)(*[ctypes.c_void_p(int(x)) for x in d_outs])
    stats = BuildStats()
    err = ctypes.create_string_buffer(512)
    rc = _lib.sparkey_build_index_sharded_device(log_header, file_len, bufs, outs, ctypes.byref(opts),
                                                 ctypes.byref(stats), err, 512)
    if rc != OK:
        raise_for(rc, err.value.decode(errors="replace"))
    return stats


def shard_geometry(log_header: bytes, file_len: int, opts, rank: int, world: int):
    """(buf_lo, buf_hi, out_off, out_len): the log bytes rank `rank` holds and the .spi bytes it makes."""
    v = [ctypes.c_uint64() for _ in range(4)]
    err = ctypes.create_string_buffer(512)
    rc = _lib.sparkey_shard_geometry(log_header, file_len, ctypes.byref(opts), rank, world,
                                     *[ctypes.byref(x) for x in v], err, 512)
    if rc != OK:
        raise_for(rc, err.value.decode(errors="replace"))
    return tuple(int(x.value) for x in v)


class ShardComm:
    """Communicator of one rank of the sharded build: RCCL (sparkey_shard_comm_create), or, with
    `group`, the collectives of a torch.distributed process group on host buffers
    (sparkey_shard_comm_create_host: e.g. gloo, to rehearse several ranks on one GPU)."""

    def __init__(self, unique_id: bytes, rank: int, world: int, device: int, group=None):
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(512)
        self._transport = None
        if group is not None or unique_id is None:
            self._transport = _torch_transport(group)
            rc = _lib.sparkey_shard_comm_create_host(ctypes.byref(h), ctypes.byref(self._transport), rank, world, device,
                                                     err, 512)
        else:
            rc = _lib.sparkey_shard_comm_create(ctypes.byref(h), unique_id, rank, world, device, err, 512)
        if rc != OK:
            raise_for(rc, err.value.decode(errors="replace"))
        self._h = h

    def build(self, plan, log_header: bytes, file_len: int, d_buf: int, buf_lo: int, buf_hi: int, opts,
              d_out: int, out_cap: int, stream: int = 0) -> BuildStats:
        """One rank's whole sharded build (sparkey_shard_build)."""
        stats = BuildStats()
        err = ctypes.create_string_buffer(512)
        rc = _lib.sparkey_shard_build(plan._h, self._h, log_header, file_len, ctypes.c_void_p(d_buf), buf_lo, buf_hi,
                                      ctypes.byref(opts), ctypes.c_void_p(d_out), out_cap, ctypes.c_void_p(stream),
                                      ctypes.byref(stats), err, 512)
        if rc != OK:
            raise_for(rc, err.value.decode(errors="replace"))
        return stats

    def phases(self):
        n = _lib.sparkey_shard_phase_count(self._h)
        return [(_lib.sparkey_shard_phase_name(self._h, i).decode(), _lib.sparkey_shard_phase_ms(self._h, i))
                for i in range(n)]

    def close(self) -> None:
        if self._h:
            _lib.sparkey_shard_comm_destroy(self._h)
            self._h = None



class ShardFrameResult(ctypes.Structure):
    _fields_ = [("exit", ctypes.c_int64), ("num_records", ctypes.c_int64), ("num_deletes", ctypes.c_int64),
                ("err_pos", ctypes.c_int64), ("rc", ctypes.c_int32), ("framing_path", ctypes.c_int32)]


class ShardExactResult(ctypes.Structure):
    _fields_ = [("num_entries", ctypes.c_int64), ("garbage_size", ctypes.c_int64), ("err_pos", ctypes.c_int64),
                ("rc", ctypes.c_int32), ("reserved", ctypes.c_int32)]


_u64p = ctypes.POINTER(ctypes.c_uint64)
_i64p = ctypes.POINTER(ctypes.c_int64)
_E = [ctypes.c_char_p, ctypes.c_size_t]
_SIGS = {
    "sparkey_shard_begin": ([_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(BuildOpts),
                             ctypes.c_int32, ctypes.c_int32] + _E, ctypes.c_int),
    "sparkey_shard_slot_range": ([_vp, ctypes.c_int32, _u64p, _u64p], ctypes.c_int),
    "sparkey_shard_max_record_len": ([_vp], ctypes.c_int64),
    "sparkey_shard_find_entry": ([_vp, ctypes.c_uint64, ctypes.c_uint64, _vp, _i64p] + _E, ctypes.c_int),
    "sparkey_shard_frame": ([_vp, ctypes.c_int64, ctypes.c_int64, _vp, ctypes.POINTER(ShardFrameResult)] + _E,
                            ctypes.c_int),
    "sparkey_shard_frame_capacity": ([_vp, ctypes.c_int64, ctypes.c_int64], ctypes.c_int64),
    "sparkey_shard_frame_bin_async": ([_vp, ctypes.c_int64, ctypes.c_int64, _vp, ctypes.c_uint64, _vp, _vp] + _E,
                                      ctypes.c_int),
    "sparkey_shard_bin_row": ([_vp, _vp, ctypes.c_uint64, ctypes.c_uint64, _i64p, _vp, _vp] + _E, ctypes.c_int),
    "sparkey_shard_summarize_dev": ([_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_int32, ctypes.c_int32, _vp, _vp] + _E,
                                    ctypes.c_int),
    "sparkey_shard_place_dev": ([_vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, ctypes.c_int32, _vp] + _E, ctypes.c_int),
    "sparkey_shard_finish_dev": ([_vp, _vp, ctypes.c_int32, ctypes.c_int32, _vp, _vp] + _E, ctypes.c_int),
    "sparkey_shard_header_dev": ([_vp, _vp, ctypes.c_int32, ctypes.c_int64, _vp, _vp] + _E, ctypes.c_int),
    "sparkey_shard_pairs": ([_vp, _u64p, ctypes.c_uint64] + _E, ctypes.c_int),
    "sparkey_shard_key_record_size": ([_vp], ctypes.c_int32),
    "sparkey_shard_fetch_keys": ([_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp] + _E, ctypes.c_int),
    "sparkey_shard_compare_keys": ([_vp, _vp, ctypes.c_uint64, ctypes.c_uint32, _vp, ctypes.POINTER(ctypes.c_int32)]
                                   + _E, ctypes.c_int),
    "sparkey_shard_apply_spill": ([_vp, _vp, ctypes.c_uint64, _vp] + _E, ctypes.c_int),
    "sparkey_shard_boundary": ([_vp, _vp, _u64p] + _E, ctypes.c_int),
    "sparkey_shard_stats": ([_vp, ctypes.c_uint64, ctypes.c_int32, _vp, _i64p] + _E, ctypes.c_int),
    "sparkey_shard_first_empty": ([_vp, _vp, _i64p] + _E, ctypes.c_int),
    "sparkey_shard_exact_record_size": ([_vp], ctypes.c_int32),
    "sparkey_shard_exact_frame": ([_vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _i64p, _vp, _u64p] + _E,
                                  ctypes.c_int),
    "sparkey_shard_exact_pack": ([_vp, _vp, ctypes.c_uint64, _vp] + _E, ctypes.c_int),
    "sparkey_shard_exact_build": ([_vp, _vp, ctypes.c_uint64, _vp, ctypes.POINTER(ShardExactResult)] + _E, ctypes.c_int),
    "sparkey_shard_exact_extract": ([_vp, ctypes.c_uint64, ctypes.c_uint64, _vp, _vp] + _E, ctypes.c_int),
    "sparkey_index_header": ([_vp, ctypes.POINTER(BuildOpts), ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                              ctypes.c_int64, ctypes.c_int64, _vp] + _E, ctypes.c_int),
    "sparkey_log_append": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64, _u64p, _vp]
                           + _E, ctypes.c_int),
    "sparkey_get_batch": ([_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint64, _vp, _vp, _vp]
                          + _E, ctypes.c_int),
    "sparkey_hash_batch": ([_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64, _vp, _vp,
                            _vp] + _E, ctypes.c_int),
    "sparkey_wanted_slot_batch": ([_vp, _vp, ctypes.c_uint64, ctypes.c_uint64, _vp, _vp] + _E, ctypes.c_int),
}
for _name, (_args, _res) in _SIGS.items():
    _f = getattr(_lib, _name)
    _f.argtypes = _args
    _f.restype = _res

EXPORTED = list(_SIGS) + ["sparkey_build_index_file", "sparkey_build_index_mem", "sparkey_index_size", "sparkey_plan_create",
            "sparkey_plan_build_device", "sparkey_plan_set_profiling", "sparkey_plan_stage_count",
            "sparkey_plan_stage_name", "sparkey_plan_stage_ms", "sparkey_plan_destroy", "sparkey_gpu_version",
            "sparkey_strerror", "sparkey_release_cached_resources", "sparkey_shard_comm_unique_id",
            "sparkey_shard_comm_create", "sparkey_shard_comm_destroy", "sparkey_shard_geometry", "sparkey_shard_build",
            "sparkey_shard_phase_count", "sparkey_shard_phase_name", "sparkey_shard_phase_ms",
            "sparkey_multi_phase_count", "sparkey_multi_phase_name", "sparkey_multi_phase_ms",
            "sparkey_file_last_phases", "sparkey_debug_set", "sparkey_debug_get", "sparkey_shard_comm_create_host",
            "sparkey_build_index_sharded_device"]


class SparkeyIOError(OSError):
    """The reference throws java.io.IOException for these codes."""


class SparkeyRuntimeError(RuntimeError):
    """The reference throws RuntimeException for these codes."""


class SparkeyGpuError(RuntimeError):
    """HIP runtime failure (no reference counterpart)."""


_IO_CODES = {E_NOT_LOG, E_VERSION, E_CORRUPT_LOG, E_NO_FREE_SLOTS, E_HEADER, E_IO, E_UNSUPPORTED}
_RUNTIME_CODES = {E_CORRUPT_DATA, E_VLQ, E_CORRUPT_RECORD}


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


def make_opts(hash_size=0, hash_seed=0, sparsity=0.0, max_memory=1 << 62, method=METHOD_IN_MEMORY, device=0,
              num_gpus=0):
    """num_gpus > 1: sparkey_build_index_file / _mem shard the log over devices device .. device + num_gpus - 1
    (the shard_transport switch = 2: every rank on `device`, for tests on one GPU)."""
    return BuildOpts(hash_size, ctypes.c_int32(hash_seed).value, float(sparsity), int(max_memory), int(method),
                     int(device), int(num_gpus), 0)


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


def release_cached_resources() -> None:
    """Frees the per-device contexts the file / host-memory entry points keep across calls."""
    _lib.sparkey_release_cached_resources()


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


def index_header(log_header: bytes, opts: BuildOpts, num_entries: int, garbage_size: int, max_displacement: int,
                 hash_collisions: int, total_displacement: int) -> bytes:
    """The 112-byte .spi header for the given totals (IndexHeader.java:125-155)."""
    out = ctypes.create_string_buffer(112)
    err = ctypes.create_string_buffer(512)
    rc = _lib.sparkey_index_header(log_header, ctypes.byref(opts), num_entries, garbage_size, max_displacement,
                                   hash_collisions, total_displacement, out, err, 512)
    if rc != OK:
        raise_for(rc, err.value.decode(errors="replace"))
    return out.raw


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

    def log_append(self, header84: bytearray, d_kind: int, d_keys: int, d_key_off: int, d_values: int,
                   d_val_off: int, n: int, d_out: int, out_cap: int, stream: int = 0) -> int:
        """Batched LogWriter.put / delete on device buffers (sparkey_log_append); header84 is updated in
        place; returns the bytes written."""
        hb = (ctypes.c_uint8 * 84).from_buffer(header84)
        written = ctypes.c_uint64()
        err = ctypes.create_string_buffer(512)
        rc = _lib.sparkey_log_append(self._h, hb, ctypes.c_void_p(d_kind), ctypes.c_void_p(d_keys),
                                     ctypes.c_void_p(d_key_off), ctypes.c_void_p(d_values), ctypes.c_void_p(d_val_off),
                                     n, ctypes.c_void_p(d_out), out_cap, ctypes.byref(written),
                                     ctypes.c_void_p(stream), err, 512)
        if rc != OK:
            raise_for(rc, err.value.decode(errors="replace"))
        return int(written.value)

    def get_batch(self, d_log: int, log_len: int, d_index: int, index_len: int, d_keys: int, d_key_off: int, n: int,
                  d_value_pos: int, d_value_len: int, stream: int = 0) -> None:
        """Batched IndexHash.get on device buffers (sparkey_get_batch)."""
        err = ctypes.create_string_buffer(512)
        rc = _lib.sparkey_get_batch(self._h, ctypes.c_void_p(d_log), log_len, ctypes.c_void_p(d_index), index_len,
                                    ctypes.c_void_p(d_keys), ctypes.c_void_p(d_key_off), n,
                                    ctypes.c_void_p(d_value_pos), ctypes.c_void_p(d_value_len),
                                    ctypes.c_void_p(stream), err, 512)
        if rc != OK:
            raise_for(rc, err.value.decode(errors="replace"))

    def hash_batch(self, d_keys: int, d_key_off: int, n: int, hash_size: int, seed: int, capacity: int, d_hash: int,
                   d_slot: int = 0, stream: int = 0) -> None:
        """Batched HashType.hash (+ getWantedSlot when capacity > 0) on device keys (sparkey_hash_batch)."""
        err = ctypes.create_string_buffer(512)
        rc = _lib.sparkey_hash_batch(self._h, ctypes.c_void_p(d_keys), ctypes.c_void_p(d_key_off), n, hash_size,
                                     ctypes.c_int32(seed).value, capacity, ctypes.c_void_p(d_hash),
                                     ctypes.c_void_p(d_slot or None), ctypes.c_void_p(stream), err, 512)
        if rc != OK:
            raise_for(rc, err.value.decode(errors="replace"))

    def wanted_slot_batch(self, d_hash: int, n: int, capacity: int, d_slot: int, stream: int = 0) -> None:
        """Long.remainderUnsigned(hash, capacity) per hash on the device (sparkey_wanted_slot_batch)."""
        err = ctypes.create_string_buffer(512)
        rc = _lib.sparkey_wanted_slot_batch(self._h, ctypes.c_void_p(d_hash), n, capacity, ctypes.c_void_p(d_slot),
                                            ctypes.c_void_p(stream), err, 512)
        if rc != OK:
            raise_for(rc, err.value.decode(errors="replace"))

    def set_profiling(self, enabled: bool) -> None:
        _lib.sparkey_plan_set_profiling(self._h, 1 if enabled else 0)

    # ---- sharded build steps (include/sparkey_gpu.h "sharded build"; orchestrated by sharded.py) ----
    def _call(self, name, *args):
        err = ctypes.create_string_buffer(512)
        rc = getattr(_lib, name)(self._h, *args, err, 512)
        if rc != OK:
            raise_for(rc, err.value.decode(errors="replace"))

    def shard_begin(self, log_header: bytes, file_len: int, d_buf: int, buf_lo: int, buf_hi: int, opts: BuildOpts,
                    rank: int, world: int) -> None:
        self._call("sparkey_shard_begin", log_header, file_len, ctypes.c_void_p(d_buf), buf_lo, buf_hi,
                   ctypes.byref(opts), rank, world)

    def shard_slot_range(self, rank: int):
        lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
        if _lib.sparkey_shard_slot_range(self._h, rank, ctypes.byref(lo), ctypes.byref(hi)) != OK:
            raise ValueError("bad rank")
        return lo.value, hi.value

    def shard_max_record_len(self) -> int:
        return int(_lib.sparkey_shard_max_record_len(self._h))

    def shard_find_entry(self, lo: int, window: int, stream: int = 0) -> int:
        v = ctypes.c_int64()
        self._call("sparkey_shard_find_entry", lo, window, ctypes.c_void_p(stream), ctypes.byref(v))
        return v.value

    def shard_frame(self, entry: int, frame_end: int, stream: int = 0) -> ShardFrameResult:
        r = ShardFrameResult()
        self._call("sparkey_shard_frame", entry, frame_end, ctypes.c_void_p(stream), ctypes.byref(r))
        return r

    def shard_frame_capacity(self, entry: int, frame_end: int) -> int:
        v = int(_lib.sparkey_shard_frame_capacity(self._h, entry, frame_end))
        if v < 0:
            raise ValueError("bad shard frame range")
        return v

    def shard_frame_bin_async(self, entry: int, frame_end: int, d_send: int, send_cap: int, d_row: int,
                              stream: int = 0) -> None:
        self._call("sparkey_shard_frame_bin_async", entry, frame_end, ctypes.c_void_p(d_send or None), send_cap,
                   ctypes.c_void_p(d_row), ctypes.c_void_p(stream))

    # the *_dev steps and shard_bin_row only enqueue work on `stream` (results stay on the device)
    def shard_bin_row(self, d_send: int, send_cap: int, n: int, scalars, d_row: int, stream: int = 0) -> None:
        sc = (ctypes.c_int64 * 8)(*[int(v) for v in scalars])
        self._call("sparkey_shard_bin_row", ctypes.c_void_p(d_send or None), send_cap, n, sc, ctypes.c_void_p(d_row),
                   ctypes.c_void_p(stream))

    def shard_summarize_dev(self, d_recv: int, n_recv: int, d_digits: int, stride: int, fixed_regions: bool,
                            d_fun: int, stream: int = 0) -> None:
        self._call("sparkey_shard_summarize_dev", ctypes.c_void_p(d_recv or None), n_recv, ctypes.c_void_p(d_digits or None),
                   stride, 1 if fixed_regions else 0, ctypes.c_void_p(d_fun), ctypes.c_void_p(stream))

    def shard_place_dev(self, d_funs: int, d_slots: int, d_spill: int, spill_cap: int, d_flags: int, inline_cap: int,
                        stream: int = 0) -> None:
        self._call("sparkey_shard_place_dev", ctypes.c_void_p(d_funs), ctypes.c_void_p(d_slots),
                   ctypes.c_void_p(d_spill), spill_cap, ctypes.c_void_p(d_flags), inline_cap, ctypes.c_void_p(stream))

    def shard_finish_dev(self, d_rows: int, stride: int, inline_cap: int, d_out: int, stream: int = 0) -> None:
        self._call("sparkey_shard_finish_dev", ctypes.c_void_p(d_rows), stride, inline_cap, ctypes.c_void_p(d_out),
                   ctypes.c_void_p(stream))

    def shard_header_dev(self, d_fin: int, stride: int, num_entries: int, d_header: int, stream: int = 0) -> None:
        self._call("sparkey_shard_header_dev", ctypes.c_void_p(d_fin), stride, num_entries, ctypes.c_void_p(d_header),
                   ctypes.c_void_p(stream))

    def shard_pairs(self, n_pairs: int):
        out = (ctypes.c_uint64 * max(1, 2 * n_pairs))()
        self._call("sparkey_shard_pairs", out, n_pairs)
        return [int(out[i]) for i in range(2 * n_pairs)]

    def shard_key_record_size(self) -> int:
        return int(_lib.sparkey_shard_key_record_size(self._h))

    def shard_fetch_keys(self, d_addrs: int, n: int, d_records: int, rec_size: int, stream: int = 0) -> None:
        self._call("sparkey_shard_fetch_keys", ctypes.c_void_p(d_addrs), n, ctypes.c_void_p(d_records), rec_size,
                   ctypes.c_void_p(stream))

    def shard_compare_keys(self, d_records: int, n_pairs: int, rec_size: int, stream: int = 0) -> int:
        dup = ctypes.c_int32()
        self._call("sparkey_shard_compare_keys", ctypes.c_void_p(d_records), n_pairs, rec_size,
                   ctypes.c_void_p(stream), ctypes.byref(dup))
        return dup.value

    def shard_apply_spill(self, d_spill: int, n: int, stream: int = 0) -> None:
        self._call("sparkey_shard_apply_spill", ctypes.c_void_p(d_spill), n, ctypes.c_void_p(stream))

    def shard_boundary(self, stream: int = 0):
        out = (ctypes.c_uint64 * 4)()
        self._call("sparkey_shard_boundary", ctypes.c_void_p(stream), out)
        return [int(x) for x in out]

    def shard_stats(self, prev_hash: int, prev_occ: int, stream: int = 0):
        out = (ctypes.c_int64 * 3)()
        self._call("sparkey_shard_stats", prev_hash, prev_occ, ctypes.c_void_p(stream), out)
        return int(out[0]), int(out[1]), int(out[2])

    # ---- sharded exact path (logs with DELETEs or duplicate keys) ----
    def shard_first_empty(self, stream: int = 0) -> int:
        v = ctypes.c_int64()
        self._call("sparkey_shard_first_empty", ctypes.c_void_p(stream), ctypes.byref(v))
        return v.value

    def shard_exact_record_size(self) -> int:
        return int(_lib.sparkey_shard_exact_record_size(self._h))

    def shard_exact_frame(self, entry: int, frame_end: int, n_records: int, starts, stream: int = 0):
        world = len(starts)
        st = (ctypes.c_int64 * world)(*[int(v) for v in starts])
        counts = (ctypes.c_uint64 * world)()
        self._call("sparkey_shard_exact_frame", entry, frame_end, n_records, st, ctypes.c_void_p(stream), counts)
        return [int(x) for x in counts]

    def shard_exact_pack(self, d_send: int, send_bytes: int, stream: int = 0) -> None:
        self._call("sparkey_shard_exact_pack", ctypes.c_void_p(d_send or None), send_bytes, ctypes.c_void_p(stream))

    def shard_exact_build(self, d_recv: int, n: int, stream: int = 0) -> ShardExactResult:
        r = ShardExactResult()
        self._call("sparkey_shard_exact_build", ctypes.c_void_p(d_recv or None), n, ctypes.c_void_p(stream),
                   ctypes.byref(r))
        return r

    def shard_exact_extract(self, a: int, b: int, d_dst: int = 0, stream: int = 0) -> None:
        self._call("sparkey_shard_exact_extract", a, b, ctypes.c_void_p(d_dst or None), ctypes.c_void_p(stream))

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
