"""Bulk log writes on the GPU: the step before the build.

LogWriter.put / delete for a batch of records at a time (LogWriter.java:96-115,
UncompressedBlockOutput.java:34-45, LogHeader.java:161-172), NONE compression: the records are
VLQ-encoded and laid out in HBM by sparkey_log_append, and the 84-byte log header is updated the way
the reference's writer updates it.  A log built on the device can go straight into the device build
(Plan.build) without a host round trip.  No CPU fallback.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native
from .log_writer import LOG_HEADER_SIZE, LogHeader

PUT, DELETE = 1, 0


def _pack(parts: Sequence[bytes]):
    off = np.zeros(len(parts) + 1, dtype=np.int64)
    if parts:
        np.cumsum([len(p) for p in parts], out=off[1:])
    data = np.frombuffer(b"".join(parts), dtype=np.uint8) if parts else np.zeros(0, dtype=np.uint8)
    return (data if data.size else np.zeros(1, dtype=np.uint8)), off


def new_log_header(file_identifier: int, compression_block_size: int = 0) -> bytearray:
    """The header LogWriter.createNew writes for an empty NONE log (LogWriter.java:34-43)."""
    return bytearray(LogHeader(0, compression_block_size, file_identifier).to_bytes())


class GpuLogAppender:
    """Appends batches of PUT / DELETE records to a log on one GPU."""

    def __init__(self, device: int = 0):
        self.device = torch.device("cuda", device)
        self.plan = _native.Plan(device)

    def close(self) -> None:
        self.plan.close()

    def append_device(self, header: bytearray, d_kind, d_keys, d_key_off, d_values, d_val_off, n: int,
                      d_out, out_cap: int, stream: int = 0) -> int:
        """Device buffers in; records written at d_out; header updated in place; bytes written out."""
        return self.plan.log_append(header, d_kind.data_ptr(), d_keys.data_ptr(), d_key_off.data_ptr(),
                                    d_values.data_ptr(), d_val_off.data_ptr(), n, d_out.data_ptr(), out_cap, stream)

    def append(self, header: bytearray, ops: Sequence[Tuple[int, bytes, Optional[bytes]]]) -> bytes:
        """ops = [(PUT, key, value) | (DELETE, key, None)]; returns the appended record bytes."""
        kind = np.array([k for k, _, _ in ops], dtype=np.uint8) if ops else np.zeros(1, dtype=np.uint8)
        keys, koff = _pack([k for _, k, _ in ops])
        vals, voff = _pack([v if v is not None else b"" for _, _, v in ops])
        dev = self.device
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        cap = int(koff[-1] + voff[-1]) + 20 * len(ops) + 16
        out = torch.empty(cap, dtype=torch.uint8, device=dev)
        n = self.append_device(header, t(kind), t(keys), t(koff), t(vals), t(voff), len(ops), out, cap)
        return out[:n].cpu().numpy().tobytes()
