"""Sharded .spi build: one process per GPU, the log's byte range split across the ranks.

REFERENCE ORCHESTRATOR, test and rehearsal use only.  The product orchestrator is the C++ one behind
the C-ABI (csrc/shard_host.cpp: sparkey_shard_build, and sparkey_build_index_file / _mem with
num_gpus > 1), which also shards SNAPPY / ZSTD logs by their block chain; this module
gathers those on every rank.  It stays as an independent restatement of the same steps over
torch.distributed, so that the CPU tests (gloo, tests/shard_sim.py) check the orchestration logic
against the oracle, and `bench.py --orchestrator python` can compare the two.

The reference build is single-threaded (Sparkey.java:36, IndexHash.createNew IndexHash.java:131-167);
this module splits the same computation at the points where ranks must exchange data and runs the
device steps of include/sparkey_gpu.h ("sharded build") in between:

  1. entries    rank g > 0 finds a record start c_g near the head of its byte range
                (sparkey_shard_find_entry); the c_g are all-gathered; rank g frames the records
                starting in [c_g, c_{g+1}) (sparkey_shard_frame) and reports its exact exit x_g.
                x_g == c_{g+1} proves c_{g+1} is on the true record chain (by induction from
                c_0 = 84); otherwise rank g+1 re-frames from x_g and the check repeats.
  2. exchange   every (hash, address) entry goes to the rank that owns its slot range: one
                all_to_all of 16-byte entries.
  3. placement  each rank computes the carry function of its slot range; the all-gathered
                functions give every rank's carry-in (the ring's wrap-around fixed point
                included); entries placed past a range end are all-gathered to their owner.
                Equal-hash pairs are checked against the keys, fetched from the ranks holding
                those records (IndexHash.java:606-636).
  4. stats      calculateMaxDisplacement (IndexHash.java:195-245) per range with the boundary slots
                exchanged; the totals are reduced and rank 0 writes the 112-byte header.

Logs the canonical layout does not cover (DELETEs, duplicate keys) take the sharded exact path
(_exact): the canonical placement of the PUT records splits the ring at empty slots
into exact ranges, every record goes to the owner of its range with its header and key, and each
owner replays IndexHash.put / delete (IndexHash.java:454-665) on its range.  SNAPPY / ZSTD logs, keys
over 4 KiB and tables the PUT records fill are gathered on every rank and built with the single-GPU
path (correct, not scaled).

Collectives go through torch.distributed: backend "nccl" (RCCL over xGMI) moves device tensors;
"gloo" (CPU tests, several ranks on one GPU) stages them through host memory.
"""
from __future__ import annotations

import contextlib
import struct
import time
from dataclasses import dataclass, field

import numpy as np
import torch

LOG_HEADER_SIZE = 84
INDEX_HEADER_SIZE = 112
ENTRY_BYTES = 16
SPILL_BYTES = 32
SPILL_INLINE = 64  # spilled slots per rank that travel with the placement flags
_HDR = struct.Struct("<IIIiqqqqqqiiqi")


def _vlq_size(v: int) -> int:  # Util.java:102-128
    n = 1
    while n < 9 and v >= (1 << (7 * n)):
        n += 1
    return n


def max_record_len(max_key_len: int, max_value_len: int) -> int:
    """Longest record a log with these header maxima can hold (PUT or DELETE)."""
    put = _vlq_size(max_key_len + 1) + _vlq_size(max_value_len) + max_key_len + max_value_len
    dele = 1 + _vlq_size(max_key_len) + max_key_len
    return max(1, put, dele)


def entry_window(max_rec: int) -> int:
    """How far past its candidate window a rank walks the candidates to find its entry."""
    return max(4096, 8 * max_rec)


@dataclass
class ShardLayout:
    """Byte ranges of the log per rank and the bytes each rank must hold."""
    data_end: int
    file_len: int
    world: int
    max_rec: int
    window: int
    lo: list
    hi: list
    small: bool  # too small to split: rank 0 frames the whole log

    def buffer_range(self, rank: int):
        """[buf_lo, buf_hi) of global log bytes rank `rank` loads onto its GPU (buf_lo 4 KiB aligned)."""
        if self.small:
            return (0, self.file_len) if rank == 0 else (0, 0)
        lo = 0 if rank == 0 else (self.lo[rank] // 4096) * 4096
        hi = self.file_len if rank == self.world - 1 else min(self.file_len, self.hi[rank] + self.overlap)
        return lo, hi

    @property
    def overlap(self) -> int:
        return 2 * self.max_rec + self.window + 64


def parse_log_header(header: bytes) -> dict:
    f = _HDR.unpack(header[:LOG_HEADER_SIZE])
    keys = ("magic", "major", "minor", "file_id", "num_puts", "num_deletes", "data_end", "max_key_len",
            "max_value_len", "delete_size", "compression_type", "block_size", "put_size", "max_entries_per_block")
    return dict(zip(keys, f))


def _switch(name: str) -> bool:
    """The library's test switch `name` (sparkey_debug_get), False where the library is not loaded
    (the CPU simulation of the device steps)."""
    try:
        from . import _native
    except (ImportError, OSError):  # (OSError: the library is there but cannot load, e.g. no libamdhip64)
        return False
    return _native.debug_get(name) > 0


def uniform_record_size(h: dict) -> int:
    """R when the header proves every record is a PUT of exactly R bytes (no DELETE, one-byte VLQs,
    putSize == numPuts * R == dataEnd - 84); else 0.  Mirrors uniform_record_size in sparkey_gpu.cpp:
    the shard entries are then arithmetic (each rank's framing still checks every record header)."""
    k, v = int(h["max_key_len"]), int(h["max_value_len"])
    r = _vlq_size(k + 1) + _vlq_size(v) + k + v
    ok = (h["num_deletes"] == 0 and h["num_puts"] > 0 and k + 1 < 128 and v < 128 and r <= 256 and
          h["put_size"] == h["num_puts"] * r and h["data_end"] - LOG_HEADER_SIZE == h["put_size"] and
          not _switch("no_uniform"))
    return r if ok else 0


def shard_layout(header: bytes, file_len: int, world: int) -> ShardLayout:
    h = parse_log_header(header)
    data_end = max(int(h["data_end"]), LOG_HEADER_SIZE)
    mrec = max_record_len(max(0, h["max_key_len"]), max(0, h["max_value_len"]))
    win = entry_window(mrec)
    span = data_end - LOG_HEADER_SIZE
    lo = [LOG_HEADER_SIZE + (g * span) // world for g in range(world)]
    hi = lo[1:] + [data_end]
    small = world > 1 and span // world < 2 * (mrec + win) + 64
    return ShardLayout(data_end, file_len, world, mrec, win, lo, hi, small)


# ------------------------------------------------------------------------------------------------
# collectives
# ------------------------------------------------------------------------------------------------
class Comm:
    """torch.distributed collectives on device tensors (nccl/RCCL) or staged through host (gloo)."""

    def __init__(self, group=None, device=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device_native = dist.get_backend(group) == "nccl"
        self.tdev = device if self.device_native else torch.device("cpu")

    def _to(self, t: torch.Tensor) -> torch.Tensor:
        return t if t.device == self.tdev else t.to(self.tdev)

    def allgather_i64(self, vals) -> np.ndarray:
        t = torch.tensor([int(v) for v in vals], dtype=torch.int64, device=self.tdev)
        out = torch.empty(self.world * t.numel(), dtype=torch.int64, device=self.tdev)
        self.dist.all_gather_into_tensor(out, t, group=self.group)
        return out.cpu().numpy().reshape(self.world, -1)

    def all_to_all(self, send: torch.Tensor, in_splits, out_splits, out_device) -> torch.Tensor:
        """1-D tensors; splits in elements of send's dtype."""
        recv = torch.empty(int(sum(out_splits)), dtype=send.dtype, device=self.tdev)
        self.dist.all_to_all_single(recv, self._to(send), [int(x) for x in out_splits], [int(x) for x in in_splits],
                                    group=self.group)
        return recv if recv.device == out_device else recv.to(out_device)

    def allgather_var(self, t: torch.Tensor, n: int, out_device):
        """Every rank's first n[rank] elements of a 1-D tensor -> list of tensors (padded exchange)."""
        counts = self.allgather_i64([n])[:, 0]
        m = max(1, int(counts.max()))
        pad = torch.zeros(m, dtype=t.dtype, device=self.tdev)
        if n:
            pad[:n] = self._to(t[:n])
        out = torch.empty(self.world * m, dtype=t.dtype, device=self.tdev)
        self.dist.all_gather_into_tensor(out, pad, group=self.group)
        res = []
        for r in range(self.world):
            piece = out[r * m: r * m + int(counts[r])]
            res.append(piece if piece.device == out_device else piece.to(out_device))
        return res

    def allgather_fixed(self, t: torch.Tensor) -> torch.Tensor:
        """Every rank's 1-D tensor of the same length -> (world, len), on the collective's device."""
        t = self._to(t)
        out = torch.empty(self.world * t.numel(), dtype=t.dtype, device=self.tdev)
        self.dist.all_gather_into_tensor(out, t, group=self.group)
        return out.view(self.world, -1)

    def barrier(self):
        self.dist.barrier(group=self.group)


# ------------------------------------------------------------------------------------------------
# device steps (the C-ABI); tests substitute a CPU simulation with the same methods
# ------------------------------------------------------------------------------------------------
class GpuShardSteps:
    """The sparkey_shard_* steps of one rank on its GPU (through a sparkey_plan)."""

    def __init__(self, device: torch.device, plan=None):
        from . import _native
        self.n = _native
        self.device = device
        self.plan = plan if plan is not None else _native.Plan(device.index or 0)
        # every torch op and every C-ABI step of the build runs in order on this one stream (its own:
        # the C-ABI reads a NULL stream as the plan's stream, so the default stream cannot be shared)
        self.tstream = torch.cuda.Stream(device)
        self.stream = self.tstream.cuda_stream
        self.header = None
        self._fun = self._fin = None  # device results kept across builds (each build ends synchronised)

    def stream_ctx(self):
        return torch.cuda.stream(self.tstream)

    def alloc(self, nbytes: int) -> torch.Tensor:
        return torch.empty(max(16, (nbytes + 15) // 16 * 16), dtype=torch.uint8, device=self.device)

    def begin(self, header, file_len, buf, buf_lo, buf_hi, opts, rank, world):
        self.header = header
        self.plan.shard_begin(header, file_len, buf.data_ptr(), buf_lo, buf_hi, opts, rank, world)

    def slot_range(self, r):
        return self.plan.shard_slot_range(r)

    def max_record_len(self):
        return self.plan.shard_max_record_len()

    def find_entry(self, lo, window):
        return self.plan.shard_find_entry(lo, window, self.stream)

    def frame(self, entry, frame_end):
        r = self.plan.shard_frame(entry, frame_end, self.stream)
        return {"exit": r.exit, "n": r.num_records, "ndel": r.num_deletes, "rc": r.rc, "err_pos": r.err_pos,
                "framing_path": r.framing_path}

    def frame_capacity(self, entry: int, frame_end: int) -> int:
        return self.plan.shard_frame_capacity(entry, frame_end)

    # the next five only enqueue device work on the build stream: their results are device tensors
    def frame_bin_async(self, entry: int, frame_end: int, send, cap: int, row: torch.Tensor) -> None:
        self.plan.shard_frame_bin_async(entry, frame_end, 0 if send is None else send.data_ptr(), cap, row.data_ptr(),
                                        self.stream)

    def bin_row(self, send, n: int, scalars, row: torch.Tensor) -> None:
        """send None (one rank): the entries stay on the device where the framing left them."""
        self.plan.shard_bin_row(0 if send is None else send.data_ptr(), 0 if send is None else send.numel() // ENTRY_BYTES,
                                n, scalars, row.data_ptr(), self.stream)

    def summarize(self, recv, n: int, rows: torch.Tensor, digit_col: int, fixed: bool) -> torch.Tensor:
        """recv None: the entries bin_row kept (one rank)."""
        if self._fun is None:
            self._fun = torch.empty(2, dtype=torch.int64, device=self.device)
        fun = self._fun
        rows = rows if rows.device == self.device else rows.to(self.device)
        self._keep = rows
        self.plan.shard_summarize_dev(0 if recv is None else recv.data_ptr(), n, rows.data_ptr() + 8 * digit_col,
                                      rows.shape[1], fixed, fun.data_ptr(), self.stream)
        return fun

    def write_header(self, fin: torch.Tensor, num_entries: int, out: torch.Tensor) -> None:
        fin = fin if fin.device == self.device else fin.to(self.device)
        self._keep_fin = fin
        self.plan.shard_header_dev(fin.data_ptr(), fin.shape[1], num_entries, out.data_ptr(), self.stream)

    def place(self, funs: torch.Tensor, out: torch.Tensor, out_off: int, spill: torch.Tensor, spill_cap: int,
              flags: torch.Tensor, inline_cap: int) -> None:
        funs = funs if funs.device == self.device else funs.to(self.device)
        self._keep_funs = funs
        self.plan.shard_place_dev(funs.data_ptr(), out.data_ptr() + out_off, spill.data_ptr(), spill_cap,
                                  flags.data_ptr(), inline_cap, self.stream)

    def finish(self, rows: torch.Tensor, inline_cap: int) -> torch.Tensor:
        if self._fin is None:
            self._fin = torch.empty(12, dtype=torch.int64, device=self.device)
        out = self._fin
        rows = rows if rows.device == self.device else rows.to(self.device)
        self._keep_rows = rows
        self.plan.shard_finish_dev(rows.data_ptr(), rows.shape[1], inline_cap, out.data_ptr(), self.stream)
        return out

    def pairs(self, n):
        return np.array(self.plan.shard_pairs(n), dtype=np.uint64)

    def key_record_size(self):
        return self.plan.shard_key_record_size()

    def fetch_keys(self, addrs: torch.Tensor, n: int, rec: torch.Tensor, rec_size: int):
        self.plan.shard_fetch_keys(addrs.data_ptr(), n, rec.data_ptr(), rec_size, self.stream)

    def compare_keys(self, rec: torch.Tensor, npairs: int, rec_size: int) -> int:
        return self.plan.shard_compare_keys(rec.data_ptr(), npairs, rec_size, self.stream)

    def apply_spill(self, spill: torch.Tensor, n: int):
        self.plan.shard_apply_spill(spill.data_ptr(), n, self.stream)

    def boundary(self):
        return self.plan.shard_boundary(self.stream)

    def stats(self, prev_hash, prev_occ):
        return self.plan.shard_stats(prev_hash, prev_occ, self.stream)

    def index_header(self, opts, num_entries, garbage, max_disp, collisions, total_disp) -> bytes:
        return self.n.index_header(self.header, opts, num_entries, garbage, max_disp, collisions, total_disp)

    # exact path (DELETEs, duplicate keys): include/sparkey_gpu.h "sharded exact path"
    def first_empty(self) -> int:
        return self.plan.shard_first_empty(self.stream)

    def exact_record_size(self) -> int:
        return self.plan.shard_exact_record_size()

    def exact_frame(self, entry: int, frame_end: int, n_records: int, starts) -> list:
        return self.plan.shard_exact_frame(entry, frame_end, n_records, starts, self.stream)

    def exact_pack(self, send: torch.Tensor) -> None:
        self.plan.shard_exact_pack(send.data_ptr(), send.numel(), self.stream)

    def exact_build(self, recv: torch.Tensor, n: int) -> dict:
        self._keep_recv = recv  # the replay's log: read again by exact_extract
        r = self.plan.shard_exact_build(recv.data_ptr() if n else 0, n, self.stream)
        return {"rc": r.rc, "err_pos": r.err_pos, "num_entries": r.num_entries, "garbage": r.garbage_size}

    def exact_extract(self, a: int, b: int, dst: torch.Tensor = None, dst_off: int = 0) -> None:
        self.plan.shard_exact_extract(a, b, 0 if dst is None else dst.data_ptr() + dst_off, self.stream)

    def full_build(self, log: torch.Tensor, file_len: int, out: torch.Tensor, opts):
        st = self.plan.build(self.header, log.data_ptr(), file_len, out.data_ptr(), out.numel(), opts, self.stream)
        return {"num_entries": st.num_entries, "garbage_size": st.garbage_size, "max_displacement": st.max_displacement,
                "hash_collisions": st.hash_collisions, "total_displacement": st.total_displacement,
                "placement_path": st.placement_path}

    def to_host_bytes(self, t: torch.Tensor) -> bytes:
        return t.cpu().numpy().tobytes()

    def from_host(self, b, dtype=torch.uint8) -> torch.Tensor:
        return torch.frombuffer(bytearray(b), dtype=dtype).to(self.device)


# ------------------------------------------------------------------------------------------------
# the orchestration
# ------------------------------------------------------------------------------------------------
@dataclass
class ShardResult:
    out: torch.Tensor        # this rank's part of the .spi: [header (rank 0)] + slots [slot_lo, slot_hi)
    slot_lo: int
    slot_hi: int
    out_offset: int          # byte offset of `out` in the .spi file
    stats: dict = field(default_factory=dict)
    path: str = "sharded"    # "sharded" or "gathered" (exact single-GPU build of the whole log)
    rounds: int = 0          # entry-verification rounds
    n_pairs: int = 0         # equal-hash pairs checked against their keys (all ranks)
    n_spill: int = 0         # slots placed past a range end (all ranks)
    phase_ms: dict = field(default_factory=dict)  # host wall time per phase on this rank


def _compose(fs):
    """Compose carry functions f(x) = max(c, x + a) left to right (apply fs[0] first)."""
    c, a = 0, 0
    first = True
    for fc, fa in fs:
        if first:
            c, a, first = fc, fa, False
        else:
            c, a = max(fc, c + fa), a + fa
    return c, a


def _apply(f, x):
    return max(f[0], x + f[1])


class ShardedBuilder:
    """One rank's side of a sharded .spi build (call build() on every rank of the group)."""

    def __init__(self, steps, comm: Comm):
        self.s = steps
        self.c = comm
        self._ebb = 0
        self._geo = {}
        self._bufs = {}

    def _buf(self, name: str, n: int, dtype=torch.int64) -> torch.Tensor:
        """A scratch tensor kept across builds (each build ends synchronised on the host)."""
        t = self._bufs.get(name)
        if t is None or t.numel() != n or t.dtype != dtype:
            t = torch.empty(n, dtype=dtype, device=self.s.device)
            self._bufs[name] = t
        return t

    def build(self, header: bytes, file_len: int, buf: torch.Tensor, buf_lo: int, buf_hi: int, opts) -> ShardResult:
        ctx = self.s.stream_ctx() if hasattr(self.s, "stream_ctx") else contextlib.nullcontext()
        with ctx:
            return self._build(header, file_len, buf, buf_lo, buf_hi, opts)

    def _build(self, header, file_len, buf, buf_lo, buf_hi, opts) -> ShardResult:
        s, c = self.s, self.c
        clock = [time.perf_counter()]
        phase = {}

        def mark(name):
            t = time.perf_counter()
            phase[name] = (t - clock[0]) * 1e3
            clock[0] = t

        g, G = c.rank, c.world
        key = (bytes(header[:LOG_HEADER_SIZE]), file_len, G)
        geo = self._geo.get(key)
        if geo is None:  # the host-side geometry of this log, kept for the next build of it
            lay = shard_layout(header, file_len, G)
            h = parse_log_header(header)
            self._geo = {key: (lay, h, uniform_record_size(h))}
            geo = self._geo[key]
        lay, h, uni = geo
        data_end = lay.data_end
        s.begin(header, file_len, buf, buf_lo, buf_hi, opts, g, G)
        if h["compression_type"] != 0:  # SNAPPY / ZSTD: the whole log on every rank, the single-GPU build
            slot_lo, slot_hi = s.slot_range(g)
            slot_size = _slot_size(h, opts, data_end)
            out_off = 0 if g == 0 else INDEX_HEADER_SIZE + slot_lo * slot_size
            out_len = (INDEX_HEADER_SIZE if g == 0 else 0) + (slot_hi - slot_lo) * slot_size
            res = ShardResult(out=None, slot_lo=slot_lo, slot_hi=slot_hi, out_offset=out_off, rounds=0,
                              phase_ms=phase)
            return self._gathered(res, header, file_len, buf, buf_lo, buf_hi, lay, opts, slot_size, out_len)

        # ---- 1 entries: speculate, frame, verify by induction from c_0 = 84 ----
        if g == 0:
            c_g = LOG_HEADER_SIZE
        elif lay.small:
            c_g = data_end
        elif uni:  # uniform records: the first record start at or after lo
            c_g = min(data_end, LOG_HEADER_SIZE + -(-(lay.lo[g] - LOG_HEADER_SIZE) // uni) * uni)
        else:
            c_g = s.find_entry(lay.lo[g], lay.window)
        mark("find_entry")
        if lay.small or uni:  # every rank's entry follows from the header: no gather
            cs = [LOG_HEADER_SIZE if r == 0 else (data_end if lay.small else
                  min(data_end, LOG_HEADER_SIZE + -(-(lay.lo[r] - LOG_HEADER_SIZE) // uni) * uni)) for r in range(G)]
        else:
            cs = [int(v) for v in c.allgather_i64([c_g])[:, 0]]
        mark("gather_entries")
        entries = []
        for r, v in enumerate(cs):
            ok = v >= 0 and (r == 0 or (lay.small and v == data_end) or lay.lo[r] <= v <= data_end)
            if ok and entries and entries[-1] is not None and v < entries[-1]:
                ok = False
            entries.append(v if ok else None)

        def frame_end(r):
            if r == G - 1:
                return data_end
            return entries[r + 1] if entries[r + 1] is not None else lay.hi[r]

        todo = {r for r in range(G) if entries[r] is not None}
        framed = set()  # entries this rank framed speculatively (sparkey_shard_frame_bin_async)
        rounds = 0
        send = None
        L = 8 + G + 256  # the verification row: frame scalars, entries per destination, per coarse digit
        row = self._buf("row", L)
        if g not in todo:  # (re-framed from the previous rank's exit in a later round)
            row.zero_()
            row[:7] = -1
        while True:
            rounds += 1
            if g in todo:
                fe = frame_end(g)
                if entries[g] not in framed:
                    # framing, bin and row enqueued without waiting; the row says if it held
                    framed.add(entries[g])
                    # (one rank: the entries stay in place, bounded by the plan's own workspace)
                    cap = (1 << 62) if G == 1 else s.frame_capacity(entries[g], fe)
                    if _switch("shard_sync_frame"):  # (tests: every attempt is retried)
                        cap = 0
                    send = None if G == 1 else s.alloc(max(1, cap) * ENTRY_BYTES)
                    s.frame_bin_async(entries[g], fe, send, cap, row)
                else:  # the speculative attempt did not hold: frame with every retry, then bin
                    mine = s.frame(entries[g], fe)  # owns nothing when entries[g] >= fe
                    n_mine = int(mine["n"]) if not mine["rc"] else 0
                    send = None if G == 1 else s.alloc(max(1, n_mine) * ENTRY_BYTES)
                    s.bin_row(send, n_mine, [entries[g], fe, mine["exit"], mine["n"], mine["ndel"], mine["rc"],
                                             mine["err_pos"], 0], row)
            mark("frame_launch")
            rows = c.allgather_fixed(row)
            mark("rows_gather")
            R = rows.cpu().numpy()
            mark("rows_wait")
            todo = {r for r in range(G) if R[r][7]}  # speculative attempts to redo, the entries unchanged
            if todo:
                continue
            done = True
            for r in range(G):
                ent, fe, ex, n, nd, rc, epos = (int(x) for x in R[r][:7])
                if rc:
                    from ._native import raise_for
                    raise_for(rc, f"{_code_text(rc)} (log offset {epos})")
                if r == G - 1:
                    break
                nxt = min(ex, data_end)
                if int(R[r + 1][0]) == nxt and entries[r + 1] == nxt:
                    continue
                entries[r + 1] = nxt  # rank r + 1 re-frames from the verified exit
                todo = {r + 1}
                done = False
                break
            if done:
                break
        totals = R[:, 3].astype(np.int64)
        n_total = int(totals.sum())
        n_deletes = int(R[:, 4].sum())
        slot_lo, slot_hi = s.slot_range(g)
        self._ebb = _entry_block_bits(h)
        slot_size = _slot_size(h, opts, data_end)
        out_off = 0 if g == 0 else INDEX_HEADER_SIZE + slot_lo * slot_size
        out_len = (INDEX_HEADER_SIZE if g == 0 else 0) + (slot_hi - slot_lo) * slot_size
        res = ShardResult(out=None, slot_lo=slot_lo, slot_hi=slot_hi, out_offset=out_off, rounds=rounds,
                          phase_ms=phase)
        mark("frame+verify")

        if n_total - n_deletes >= _capacity(h, opts):  # the PUT records may fill the table: one lane's replay
            return self._gathered(res, header, file_len, buf, buf_lo, buf_hi, lay, opts, slot_size, out_len)

        # ---- 2 exchange: every PUT entry to the owner of its slot range (binned while framing; the bins
        #      leave DELETE records out: they only matter to the exact path) ----
        if send is None and G > 1:
            send = s.alloc(16)
        M = R[:, 8:8 + G]                                  # M[src][dst]
        n_mine = int(M[g].sum())
        out_splits = [int(M[r][g]) * 2 for r in range(G)]  # int64 elements (2 per entry)
        n_recv = sum(out_splits) // 2
        if G == 1:  # nothing to exchange: the entries stay where the framing left them
            recv = None
        else:
            in_splits = [int(x) * 2 for x in M[g]]
            recv = c.all_to_all(send.view(torch.int64)[: 2 * n_mine], in_splits, out_splits, buf.device)
        mark("all_to_all")

        # ---- 3 placement and stats on the device; the host sees one row per rank at the end ----
        out = s.alloc(out_len)
        hdr_off = INDEX_HEADER_SIZE if g == 0 else 0
        spill_cap = 4096
        spill = self._buf("spill", spill_cap * SPILL_BYTES, torch.uint8)
        flags = self._buf("flags", 4 + 4 * SPILL_INLINE)
        fixed = True
        while True:
            # the runs arrive grouped by coarse digit: no first partition pass
            fun = s.summarize(recv, n_recv, rows, 8 + G, fixed)
            mark("summarize")
            funs = c.allgather_fixed(fun)                   # every rank's carry function
            mark("funs_gather")
            s.place(funs, out, hdr_off, spill, spill_cap, flags, SPILL_INLINE)
            mark("place_launch")
            frows = c.allgather_fixed(flags)                # flags + inline spilled slots of every rank
            mark("flags_gather")
            fin = s.finish(frows, SPILL_INLINE)             # spill applied; flags, boundary slots, range stats
            mark("finish_launch")
            fins = c.allgather_fixed(fin)
            mark("fins_gather")
            if g == 0:  # the header from the same rows (rewritten below if a slow path runs)
                s.write_header(fins, n_total, out)
            host = fins.cpu().numpy()
            F, bnd = host[:, :4], host[:, 4:]
            if F[:, 3].any() and fixed:  # a bucket outgrew its fixed region on some rank: dense runs
                fixed = False
                continue
            if F[:, 3].any():
                raise RuntimeError("sharded placement aborted")
            break
        mark("place")
        res.n_spill, res.n_pairs = int(F[:, 0].sum()), int(F[:, 1].sum())
        # DELETE records, or equal-hash pairs this step cannot prove distinct: the exact path
        exact = n_deletes > 0 or bool(F[:, 2].any())
        if not exact and F[:, 1].sum() > 0:
            exact = self._pairs_share_a_key(int(F[g, 1]), entries, data_end, buf.device)
        host_header = exact
        if int(F[:, 0].max()) > SPILL_INLINE:  # more spilled slots than the rows carry: exchange them all
            host_header = True
            n_spill = int(F[g, 0])
            if n_spill > spill_cap:
                spill_cap = n_spill
                spill = s.alloc(spill_cap * SPILL_BYTES)
                s.place(funs, out, hdr_off, spill, spill_cap, flags, SPILL_INLINE)
            pieces = c.allgather_var(spill.view(torch.int64), 4 * n_spill, buf.device)
            allsp = torch.cat([p for p in pieces if p.numel()])
            s.apply_spill(allsp, allsp.numel() // 4)
            if not exact:
                bnd = self._range_stats(slot_lo, slot_hi)
        mark("spill")
        if exact:  # the ring splits at the slots the PUT placement left empty (now complete on every rank)
            done = self._exact(res, out, hdr_off, entries, frame_end, int(R[g][3]), opts, h, slot_lo, slot_hi,
                               slot_size, buf.device)
            if done is not None:
                mark("exact")
                return done
            return self._gathered(res, header, file_len, buf, buf_lo, buf_hi, lay, opts, slot_size, out_len)

        # ---- 4 stats: per-range sums (the first slot is not compared with its predecessor) and the
        #      boundary slots of every rank; the cross-range comparisons are added here ----
        max_disp, collisions, total_disp = _combine_stats(bnd)
        stats = {"num_entries": n_total, "garbage_size": 0, "max_displacement": max_disp,
                 "hash_collisions": collisions, "total_displacement": total_disp, "placement_path": 0}
        if g == 0 and host_header:
            hdr = s.index_header(opts, n_total, 0, max_disp, collisions, total_disp)
            out[:INDEX_HEADER_SIZE].copy_(s.from_host(hdr))
        res.out = out[:out_len]  # (the allocation is rounded up)
        res.stats = stats
        mark("stats")
        return res

    def _range_stats(self, slot_lo, slot_hi) -> np.ndarray:
        """Every rank's {boundary slots, non-empty, max displacement, collisions, total displacement}."""
        s, c = self.s, self.c
        nonempty = int(slot_hi > slot_lo)
        bslots = s.boundary()
        mx, col, tot = s.stats(0, 0) if nonempty else (0, 0, 0)
        return c.allgather_i64([_signed(v) for v in bslots] + [nonempty, mx, col, tot])

    # ---- the sharded exact path ----
    def _exact(self, res, out, hdr_off, entries, frame_end, n_records, opts, h, slot_lo, slot_hi, slot_size, device):
        """IndexHash.put / delete (IndexHash.java:454-665) replayed on exact ranges: the ring splits at the
        slots the canonical placement of all PUT records leaves empty (no probe or backward shift crosses
        one), rank r's range running from the first such slot of its slot range to the next rank's.
        Returns None when the log needs the gathered path (no empty slot, keys over 4 KiB)."""
        s, c = self.s, self.c
        g, G = c.rank, c.world
        cap = _capacity(h, opts)
        E = [int(v) for v in c.allgather_i64([s.first_empty()])[:, 0]]
        have = [r for r in range(G) if E[r] >= 0]
        rs = s.exact_record_size()
        if not have or rs <= 0:
            return None
        ranges = {}
        for i, r in enumerate(have):
            a, b = E[r], E[have[(i + 1) % len(have)]]
            ranges[r] = (a, b + cap if b <= a else b)
        # every record (PUT and DELETE) with its header and key to the owner of its wanted slot's range
        counts = s.exact_frame(entries[g], frame_end(g), n_records, E)
        n_send = sum(counts)
        send = s.alloc(max(1, n_send) * rs)
        s.exact_pack(send)
        M = c.allgather_i64(counts)  # M[src][dst]
        n_recv = int(sum(M[r][g] for r in range(G)))
        if G == 1:
            recv = send
        else:
            recv = c.all_to_all(send[: n_send * rs], [x * rs for x in counts], [int(M[r][g]) * rs for r in range(G)],
                                device)
        rep = s.exact_build(recv, n_recv)
        rows = c.allgather_i64([rep["rc"], rep["err_pos"], rep["num_entries"], rep["garbage"]])
        bad = sorted((int(x[1]), int(x[0])) for x in rows if x[0])
        if bad:
            from ._native import raise_for
            raise_for(bad[0][1], f"{_code_text(bad[0][1])} (log offset {bad[0][0]})")
        # the replayed slots to the ranks whose slices hold them (mostly a rank's own slice; the run
        # before the first empty slot of a slice was replayed by the previous range's owner)
        slices = [s.slot_range(r) for r in range(G)]

        def pieces(r):
            if r not in ranges:
                return []
            a, b = ranges[r]
            segs = [(a, min(b, cap))] + ([(0, b - cap)] if b > cap else [])
            got = []
            for q in range(G):
                lo, hi = slices[q]
                for x, y in segs:
                    u, v = max(x, lo), min(y, hi)
                    if u < v:
                        got.append((q, u, v))
            return got

        mine = pieces(g)
        for q, u, v in mine:
            if q == g:
                s.exact_extract(u, v, out, hdr_off + (u - slot_lo) * slot_size)
        if G > 1:
            to = [0] * G
            for q, u, v in mine:
                if q != g:
                    to[q] += (v - u) * slot_size
            send2 = s.alloc(max(1, sum(to)))
            at = [sum(to[:q]) for q in range(G)]
            for q, u, v in mine:
                if q != g:
                    s.exact_extract(u, v, send2, at[q])
                    at[q] += (v - u) * slot_size
            frm = [sum((v - u) * slot_size for q, u, v in pieces(r) if q == g) if r != g else 0 for r in range(G)]
            recv2 = c.all_to_all(send2[: sum(to)], to, frm, device)
            at2 = 0
            for r in range(G):
                if r == g:
                    continue
                for q, u, v in pieces(r):
                    if q == g:
                        nb = (v - u) * slot_size
                        o = hdr_off + (u - slot_lo) * slot_size
                        out[o: o + nb].copy_(recv2[at2: at2 + nb])
                        at2 += nb
        bnd = self._range_stats(slot_lo, slot_hi)
        max_disp, collisions, total_disp = _combine_stats(bnd)
        n_entries, garbage = int(rows[:, 2].sum()), int(rows[:, 3].sum())
        if g == 0:
            hdr = s.index_header(opts, n_entries, garbage, max_disp, collisions, total_disp)
            out[:INDEX_HEADER_SIZE].copy_(s.from_host(hdr))
        res.out = out[:hdr_off + (slot_hi - slot_lo) * slot_size]  # (the allocation is rounded up)
        res.stats = {"num_entries": n_entries, "garbage_size": garbage, "max_displacement": max_disp,
                     "hash_collisions": collisions, "total_displacement": total_disp, "placement_path": 2}
        res.path = "exact"
        return res

    # equal-hash pairs: fetch both keys from the ranks that hold the records, compare on device
    def _pairs_share_a_key(self, n_pairs, entries, data_end, device) -> bool:
        s, c = self.s, self.c
        G = c.world
        addrs = s.pairs(n_pairs) if n_pairs else np.zeros(0, dtype=np.uint64)
        starts = np.array([e if e is not None else data_end for e in entries], dtype=np.int64)
        pos = (addrs & np.uint64(~(1 << 63) & 0xFFFFFFFFFFFFFFFF)).astype(np.int64)
        owner = np.searchsorted(starts, pos >> self._ebb, side="right") - 1
        owner = np.clip(owner, 0, G - 1)
        order = np.argsort(owner, kind="stable")
        req = addrs[order].astype(np.int64)
        counts = np.bincount(owner, minlength=G).astype(np.int64)
        M = c.allgather_i64(counts.tolist())
        rs = s.key_record_size()
        send = torch.from_numpy(req.copy()).to(device) if req.size else torch.zeros(1, dtype=torch.int64, device=device)
        got = c.all_to_all(send[: req.size], counts.tolist(), [int(M[r][c.rank]) for r in range(G)], device)
        n_req = got.numel()
        rec = s.alloc(max(1, n_req) * rs)
        if n_req:
            s.fetch_keys(got, n_req, rec, rs)
        back = c.all_to_all(rec[: n_req * rs], [int(M[r][c.rank]) * rs for r in range(G)],
                            (counts * rs).tolist(), device)
        # back holds the records in request order; put them back in pair order
        inv = np.empty_like(order)
        inv[order] = np.arange(order.size)
        dup = 0
        if n_pairs:
            idx = torch.from_numpy(inv.astype(np.int64)).to(device)
            recs = back.view(-1, rs)[idx].reshape(-1).contiguous()
            dup = s.compare_keys(recs, n_pairs, rs)
        return bool(c.allgather_i64([int(dup != 0)])[:, 0].any())

    # exact path for non-canonical logs: every rank gathers the whole log and builds it
    def _gathered(self, res, header, file_len, buf, buf_lo, buf_hi, lay, opts, slot_size, out_len):
        s, c = self.s, self.c
        g, G = c.rank, c.world
        if lay.small:
            own_lo, own_hi = (0, file_len) if g == 0 else (0, 0)
        else:
            own_lo = 0 if g == 0 else lay.lo[g]
            own_hi = file_len if g == G - 1 else lay.lo[g + 1]
        piece = buf[own_lo - buf_lo: own_hi - buf_lo] if own_hi > own_lo else buf[:0]
        pieces = c.allgather_var(piece, piece.numel(), buf.device)
        log = s.alloc(file_len + 16)
        at = 0
        for p in pieces:
            log[at: at + p.numel()].copy_(p)
            at += p.numel()
        full = s.alloc(INDEX_HEADER_SIZE + _capacity(parse_log_header(header), opts) * slot_size)
        stats = s.full_build(log, file_len, full, opts)
        lo = 0 if g == 0 else INDEX_HEADER_SIZE + res.slot_lo * slot_size
        out = s.alloc(out_len)
        out[:out_len].copy_(full[lo: lo + out_len])
        res.out = out[:out_len]
        res.stats = stats
        res.path = "gathered"
        return res


def _combine_stats(bnd):
    """calculateMaxDisplacement (IndexHash.java:195-245) from every rank's range row: the per-range sums
    plus the comparisons across range boundaries and the wrap quirk."""
    max_disp, collisions, total_disp = int(bnd[:, 5].max()), int(bnd[:, 6].sum()), int(bnd[:, 7].sum())
    prev = None  # (hash, occupied) of the last slot of the previous non-empty range
    for r in range(bnd.shape[0]):
        if not bnd[r][4]:
            continue
        if prev is not None and prev[1] and prev[0] == int(bnd[r][0]) & 0xFFFFFFFFFFFFFFFF:
            collisions += 1  # calculateMaxDisplacement compares every slot with the one before
        prev = (int(bnd[r][2]) & 0xFFFFFFFFFFFFFFFF, int(bnd[r][3] != 0))
    # wrap quirk (IndexHash.java:239-241): slot 0 and slot cap-1 occupied with equal hashes
    last = max(r for r in range(bnd.shape[0]) if bnd[r][4])
    if bnd[0][1] != 0 and bnd[last][3] != 0 and bnd[0][0] == bnd[last][2]:
        collisions += 1
    return max_disp, collisions, total_disp


_CODE_TEXT = {-1: "File is not a Sparkey log file", -2: "Incompatible version", -3: "Corrupt log file",
              -4: "No free slots in the hash", -5: "Corrupt data", -6: "Too long VLQ value",
              -7: "Too large max key len"}


def _code_text(rc: int) -> str:
    return _CODE_TEXT.get(rc, "error")


def _capacity(h: dict, opts) -> int:
    """IndexHash.java:135-145: capacity = 1 | (long)(numPuts * max(sparsity, 1.3))."""
    sp = max(float(opts.sparsity), 1.3)
    v = float(h["num_puts"]) * sp
    return 1 | (int(v) if v == v else 0)


def _signed(v: int) -> int:
    v = int(v) & 0xFFFFFFFFFFFFFFFF
    return v - (1 << 64) if v >= (1 << 63) else v


def _entry_block_bits(h: dict) -> int:  # IndexHash.java:123-129
    ebb = 0
    while (1 << ebb) < h["max_entries_per_block"]:
        ebb += 1
    return ebb


def _slot_size(h: dict, opts, data_end: int) -> int:
    ebb = _entry_block_bits(h)
    addr = 4 if h["data_end"] <= (1 << (30 - ebb)) else 8
    hs = opts.hash_size or (4 if h["num_puts"] < (1 << 23) else 8)
    return hs + addr
