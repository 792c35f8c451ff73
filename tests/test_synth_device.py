"""The torch generator of the fixed-record logs (sparkey/synth_device.py, used for the C4-sized logs
made in HBM) writes exactly synth.fixed_log_range's bytes: every range, chunk boundary and the keys.
CPU (torch on the host); the GPU tests then use it on cuda:0."""
import numpy as np
import pytest
import torch

from sparkey import synth, synth_device


@pytest.mark.parametrize("lo,hi", [(0, 84 + 118 * 3000), (0, 50), (37, 1234), (84 + 118 * 5 + 3, 84 + 118 * 2999 - 7),
                                   (84 + 118 * 3000 - 5, 84 + 118 * 3000 + 100)])
@pytest.mark.parametrize("chunk", [777, 1 << 22])
def test_matches_numpy_generator(lo, hi, chunk):
    h1, a = synth.fixed_log_range(3000, lo, hi, seed=7, file_id=9)
    h2, b = synth_device.fixed_log_range(3000, lo, hi, seed=7, file_id=9, device="cpu", chunk=chunk)
    assert h1 == h2 and np.array_equal(a, b.numpy())


def test_other_shapes_and_keys():
    for klen, vlen in ((16, 0), (24, 127), (126, 1)):
        a = synth.fixed_log(500, klen, vlen, seed=3)
        b = synth_device.fixed_log(500, klen, vlen, seed=3, device="cpu")
        assert np.array_equal(a, b.numpy())
    full = synth.fixed_log(3000, seed=7)
    idx = torch.tensor([0, 1, 1234, 2999], dtype=torch.int64)
    keys = synth_device.fixed_keys(idx, seed=7).numpy()
    for j, i in enumerate(idx.tolist()):
        assert keys[j].tobytes() == full[84 + 118 * i + 2: 84 + 118 * i + 18].tobytes()
