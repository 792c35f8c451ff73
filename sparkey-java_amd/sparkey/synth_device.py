"""The C2 / C4 synthetic logs (synth.fixed_log_range) generated with torch on the device, byte for byte
the same as the numpy generator: every byte of the fixed-record log is a function of its record index
(key = LE64(i) || LE64(splitmix64(i ^ seed)), value = splitmix64 words of (i, j)), so a rank of a
sharded build -- or a single 118 GB C4 log -- is made in HBM without a host copy.  Test and benchmark
data only; the build never calls this.  torch int64 arithmetic wraps like uint64, and logical right
shifts are arithmetic shifts with the sign bits masked off."""
from __future__ import annotations

import torch

from .log_writer import LOG_HEADER_SIZE
from .synth import _header

_M64 = (1 << 64) - 1


def _s64(v: int) -> int:
    """A uint64 constant as the int64 with the same bits."""
    v &= _M64
    return v - (1 << 64) if v >= 1 << 63 else v


def _shr(x: torch.Tensor, k: int) -> torch.Tensor:
    return (x >> k) & ((1 << (64 - k)) - 1)


def splitmix64(x: torch.Tensor) -> torch.Tensor:
    """synth.splitmix64 on int64 tensors (the same bits as the uint64 version)."""
    z = x + _s64(0x9E3779B97F4A7C15)
    z = (z ^ _shr(z, 30)) * _s64(0xBF58476D1CE4E5B9)
    z = (z ^ _shr(z, 27)) * _s64(0x94D049BB133111EB)
    return z ^ _shr(z, 31)


def _records(i0: int, i1: int, key_len: int, value_len: int, seed: int, device) -> torch.Tensor:
    """Records i0 .. i1-1 of fixed_log as a flat uint8 tensor ((i1 - i0) * (2 + key_len + value_len) bytes)."""
    m = i1 - i0
    rec = 2 + key_len + value_len
    extra = (key_len - 16) + value_len
    words = (extra + 7) // 8
    i = torch.arange(i0, i1, dtype=torch.int64, device=device)
    w = torch.empty((m, 2 + words), dtype=torch.int64, device=device)
    w[:, 0] = i
    w[:, 1] = splitmix64(i ^ _s64(seed))
    base = i * 64 + _s64(seed * 0x9E3779B97F4A7C15)
    w[:, 2:] = splitmix64(base[:, None] + torch.arange(words, dtype=torch.int64, device=device)[None, :])
    out = torch.empty((m, rec), dtype=torch.uint8, device=device)
    out[:, 0] = key_len + 1
    out[:, 1] = value_len
    out[:, 2:] = w.view(torch.uint8).view(m, (2 + words) * 8)[:, :rec - 2]
    return out.view(-1)


def fixed_log_range(n: int, lo: int, hi: int, key_len: int = 16, value_len: int = 100, seed: int = 1,
                    file_id: int = 0x5EED5EED, block_size: int = 0, device="cuda", out: torch.Tensor = None,
                    chunk: int = 1 << 22):
    """Bytes [lo, hi) of synth.fixed_log(n, ...) as a uint8 tensor on `device` (or written into `out`,
    which must hold hi - lo bytes).  Returns (84-byte header, tensor)."""
    assert key_len >= 16 and key_len + 1 < 128 and value_len < 128
    rec = 2 + key_len + value_len
    total = LOG_HEADER_SIZE + n * rec
    hi = min(hi, total)
    lo = min(lo, hi)
    header = _header(n, key_len, value_len, n * rec, total, file_id, block_size)
    buf = out if out is not None else torch.empty(hi - lo, dtype=torch.uint8, device=device)
    assert buf.numel() >= hi - lo
    if lo < LOG_HEADER_SIZE:
        k = min(hi, LOG_HEADER_SIZE) - lo
        buf[:k] = torch.frombuffer(bytearray(header[lo:lo + k]), dtype=torch.uint8).to(buf.device)
    i0 = max(0, (lo - LOG_HEADER_SIZE) // rec)
    i1 = min(n, max(0, (hi - LOG_HEADER_SIZE + rec - 1) // rec))
    for a in range(i0, i1, chunk):
        b = min(i1, a + chunk)
        body = _records(a, b, key_len, value_len, seed, buf.device)
        start = LOG_HEADER_SIZE + a * rec  # file offset of body[0]
        s0, s1 = max(lo, start), min(hi, start + body.numel())
        if s1 > s0:
            buf[s0 - lo: s1 - lo] = body[s0 - start: s1 - start]
        del body
    return header, buf


def fixed_log(n: int, key_len: int = 16, value_len: int = 100, seed: int = 1, file_id: int = 0x5EED5EED,
              block_size: int = 0, device="cuda", out: torch.Tensor = None) -> torch.Tensor:
    """The whole fixed_log(n, ...) .spl on the device."""
    rec = 2 + key_len + value_len
    return fixed_log_range(n, 0, LOG_HEADER_SIZE + n * rec, key_len, value_len, seed, file_id, block_size, device,
                           out)[1]


def fixed_keys(idx: torch.Tensor, key_len: int = 16, value_len: int = 100, seed: int = 1) -> torch.Tensor:
    """The keys of records `idx` (int64, on any device) as a (len(idx), key_len) uint8 tensor."""
    assert key_len == 16
    w = torch.stack([idx, splitmix64(idx ^ _s64(seed))], dim=1)
    return w.contiguous().view(torch.uint8).view(idx.numel(), 16)
