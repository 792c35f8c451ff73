"""Ranks fail together when a collective of the host-supplied transport fails on one rank
(sparkey_shard_comm_create_host, csrc/shard_host.cpp HostColl).  Two processes share cuda:0 over a
gloo group (as `bench.py --gpus N --backend gloo` rehearses); the `shard_coll_fail` switch, set in rank
1's process only, makes that rank's k-th collective fail its device-to-host copy.  The rank still takes
part with an all-ones row (or, from the exchange on, joins every collective up to the finish rows), so
for every k both ranks return an error -- none waits in a collective its peer never enters -- or, for k
past the build's last collective, both succeed with the single-GPU bytes.  The group stays usable:
the next k runs in the same processes.  Every collective of the build is covered: the canonical steps'
rows and exchanges, and the equal-hash key check's (200K keys: 32-bit hashes with collisions).
"""
import datetime
import os
import sys

import pytest
import torch.multiprocessing as mp

from sharded_harness import free_port

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KS = list(range(1, 14))
# progress lines (a GPU box kills a run that writes nothing for 3 minutes): gpurun_out/ on the box
PROGRESS = os.path.join(ROOT, "gpurun_out", "host_coll_failure.log")


def _progress(msg):
    try:
        os.makedirs(os.path.dirname(PROGRESS), exist_ok=True)
        with open(PROGRESS, "a") as f:
            f.write(msg + "\n")
    except OSError:
        pass


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, os.path.join(ROOT, "sparkey-java_amd"))
    import torch
    import torch.distributed as dist
    from sparkey import _native, synth
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=30))
    _progress(f"rank {rank}: group up")
    plan = None
    try:
        dev = torch.device("cuda", 0)
        log = synth.fixed_log(200_000, 16, 100, seed=3, file_id=0x77)
        header = log[:84].tobytes()
        opts = _native.make_opts(hash_seed=19, device=0)
        lo, hi, off, ln = _native.shard_geometry(header, int(log.size), opts, rank, world)
        buf = torch.from_numpy(log[lo:hi]).to(dev)
        d_out = torch.empty(max(16, ln), dtype=torch.uint8, device=dev)
        plan = _native.Plan(0)
        _native.debug_set("frame_ticket", 1)  # (ranks share the device)
        res = []
        for k in KS + [None]:
            comm = _native.ShardComm(None, rank, world, 0)
            if rank == 1:
                _native.debug_set("shard_coll_fail", k)
            try:
                st = comm.build(plan, header, int(log.size), buf.data_ptr(), lo, hi, opts, d_out.data_ptr(), ln)
                torch.cuda.synchronize(dev)
                res.append((k, "ok", st.sharded, bytes(d_out[:ln].cpu().numpy())))
            except Exception as e:  # noqa: BLE001
                res.append((k, "err", type(e).__name__, str(e)[:200]))
            finally:
                _native.debug_set("shard_coll_fail", None)
                comm.close()
            _progress(f"rank {rank}: k={k} {res[-1][1]} {res[-1][2]} {res[-1][3] if res[-1][1] == 'err' else ''}")
            dist.barrier()
        q.put((rank, off, res))
    except Exception as e:  # noqa: BLE001  (reported to the parent at once instead of a silent exit)
        import traceback
        _progress(f"rank {rank}: fatal {e!r}")
        q.put((rank, None, traceback.format_exc()))
    finally:
        if plan is not None:
            plan.close()
        dist.destroy_process_group()


def test_one_rank_collective_failure_fails_every_rank(native):
    import oracle
    from sparkey import synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    _progress("start")
    try:
        for _ in range(2):
            r, off, res = q.get(timeout=150)
            assert off is not None, f"rank {r} failed: {res}"
            out[r] = (off, res)
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    log = synth.fixed_log(200_000, 16, 100, seed=3, file_id=0x77)
    want = oracle.build_index(log.tobytes(), 19)
    failed = 0
    for i, k in enumerate(KS + [None]):
        a, b = out[0][1][i], out[1][1][i]
        assert a[0] == b[0] == k
        assert a[1] == b[1], (k, a[1:3], b[1:3])  # both fail, or both succeed
        if a[1] == "err":
            failed += 1
            assert a[2] == b[2] == "SparkeyGpuError", (k, a, b)
        else:
            for off, piece in ((out[0][0], a[3]), (out[1][0], b[3])):
                assert piece == want[off:off + len(piece)], k
    # the build's collectives: entries checkpoint, frame rows, buffers checkpoint, entry exchange, carry,
    # flag and finish rows, then (32-bit hashes: equal-hash pairs) the pair counts, address and key
    # exchanges and the verdict -- a failure in any of them fails both ranks
    assert failed >= 11, failed
    assert out[0][1][-2][1] == "ok"  # (k past the last collective: the build)
    assert out[0][1][-1][1] == "ok"  # (no switch: the build)
