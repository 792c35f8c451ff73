"""The host-supplied collectives of the C++ orchestrator (sparkey_shard_transport,
sparkey_shard_comm_create_host) as the Python binding implements them over torch.distributed: the
all-gather and the all-to-all the sharded build issues, in world-size 2 and 3 gloo groups on the CPU.
On a GPU the same transport carries sparkey_shard_build between processes that share one device
(bench.py --gpus N --backend gloo, tests/test_multi_gpu_abi.py)."""
import ctypes
import os
import sys

import pytest
import torch.multiprocessing as mp

from sharded_harness import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, os.path.join(ROOT, "sparkey-java_amd"))
    import torch.distributed as dist
    from sparkey import _native
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = _native._torch_transport()
        send = (ctypes.c_uint8 * 5)(*[rank * 10 + i for i in range(5)])
        recv = (ctypes.c_uint8 * (5 * world))()
        rc1 = t.all_gather(None, ctypes.addressof(send), ctypes.addressof(recv), 5)
        sb = (ctypes.c_uint64 * world)(*[rank + 1 + d for d in range(world)])   # bytes to rank d
        rb = (ctypes.c_uint64 * world)(*[s + 1 + rank for s in range(world)])   # bytes from rank s
        src = (ctypes.c_uint8 * sum(sb))(*[(rank * 50 + i) % 256 for i in range(sum(sb))])
        dst = (ctypes.c_uint8 * sum(rb))()
        rc2 = t.all_to_all(None, ctypes.addressof(src), sb, ctypes.addressof(dst), rb)
        empty = t.all_gather(None, ctypes.addressof(send), ctypes.addressof(recv), 0)
        q.put((rank, rc1, list(recv), rc2, list(dst), empty))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_torch_transport_collectives(native, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, rc1, recv, rc2, dst, empty = q.get(timeout=120)
        res[r] = (rc1, recv, rc2, dst, empty)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    gathered = [s * 10 + i for s in range(world) for i in range(5)]
    for r in range(world):
        rc1, recv, rc2, dst, empty = res[r]
        assert rc1 == 0 and rc2 == 0 and empty == 0 and recv == gathered
        want = []
        for s in range(world):  # rank s's run for rank r: after its runs for ranks 0 .. r-1
            off = sum(s + 1 + d for d in range(r))
            want += [(s * 50 + off + i) % 256 for i in range(s + 1 + r)]
        assert dst == want, (r, dst, want)
