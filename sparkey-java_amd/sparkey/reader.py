"""Batched lookups on the GPU over a built hash file: the step after writeHash.

Mirrors the reference reader's lookup (SparkeyReader.getAsByteArray -> IndexHash.get,
IndexHash.java:398-452) for a batch of keys at a time: the log and the index are kept resident in
HBM, keys go in as one packed buffer, and each result is the value's (offset, length) in the log.
There is no CPU fallback: the lookups run in libsparkey_gpu.so (sparkey_get_batch).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _native


def pack_keys(keys: Sequence[bytes]):
    """Keys -> (uint8 bytes, uint64 offsets of n + 1 entries)."""
    off = np.zeros(len(keys) + 1, dtype=np.uint64)
    if keys:
        np.cumsum([len(k) for k in keys], out=off[1:])
    data = np.frombuffer(b"".join(keys), dtype=np.uint8) if keys else np.zeros(0, dtype=np.uint8)
    return data, off


class GpuHashReader:
    """A log (.spl) and its hash file (.spi), resident on one GPU, answering batches of gets."""

    def __init__(self, log: bytes, index: bytes, device: int = 0):
        self.device = torch.device("cuda", device)
        self.log_host = log
        self.d_log = torch.frombuffer(bytearray(log), dtype=torch.uint8).to(self.device)
        self.d_index = torch.frombuffer(bytearray(index), dtype=torch.uint8).to(self.device)
        self.plan = _native.Plan(device)

    def close(self) -> None:
        self.plan.close()

    def locate_batch(self, d_keys: torch.Tensor, d_key_off: torch.Tensor, n: int, stream: int = 0):
        """Device keys in, device (value_pos, value_len) out (int64, -1 = absent)."""
        pos = torch.empty(max(1, n), dtype=torch.int64, device=self.device)
        ln = torch.empty(max(1, n), dtype=torch.int64, device=self.device)
        self.plan.get_batch(self.d_log.data_ptr(), self.d_log.numel(), self.d_index.data_ptr(), self.d_index.numel(),
                            d_keys.data_ptr(), d_key_off.data_ptr(), n, pos.data_ptr(), ln.data_ptr(), stream)
        return pos[:n], ln[:n]

    def get_batch(self, keys: Sequence[bytes]) -> List[Optional[bytes]]:
        """IndexHash.get for every key: its value, or None."""
        data, off = pack_keys(keys)
        d_keys = torch.from_numpy(data.copy() if data.size else np.zeros(1, dtype=np.uint8)).to(self.device)
        d_off = torch.from_numpy(off.view(np.int64).copy()).to(self.device)
        pos, ln = self.locate_batch(d_keys, d_off, len(keys))
        pos, ln = pos.cpu().numpy(), ln.cpu().numpy()
        return [None if p < 0 else self.log_host[p: p + l] for p, l in zip(pos.tolist(), ln.tolist())]

    def get(self, key: bytes) -> Optional[bytes]:
        return self.get_batch([key])[0]
