"""Multi-process sharded build on ONE GPU: every rank of a torchrun/gloo group runs its steps on
cuda:0 (collectives staged through host memory) and rank 0 checks the assembled .spi against the
single-GPU build of the same log.  Run on the GPU box:

    python -m torch.distributed.run --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29533 \\
        tools/shard_gloo_check.py [--records 200000]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sparkey-java_amd"), ROOT]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=200000)
    args = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    from sparkey import _native, synth
    from sparkey.sharded import Comm, GpuShardSteps, ShardedBuilder, shard_layout
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    log = synth.mixed_log(args.records, 8, 64, 100, seed=21)
    header = log[:84].tobytes()
    lay = shard_layout(header, log.size, world)
    lo, hi = lay.buffer_range(rank)
    buf = torch.from_numpy(log[lo:hi].copy()).to(dev)
    opts = _native.make_opts(hash_seed=4321)
    res = ShardedBuilder(GpuShardSteps(dev), Comm(device=dev)).build(header, log.size, buf, lo, hi, opts)
    part = res.out.cpu()
    sizes = [None] * world
    dist.all_gather_object(sizes, (res.out_offset, res.slot_lo, res.slot_hi, res.path))
    parts = [torch.empty(0, dtype=torch.uint8)] * world
    gathered = [None] * world
    dist.all_gather_object(gathered, part.numpy().tobytes())
    if rank == 0:
        single, _ = _native.build_index_mem(log.tobytes(), opts)
        spi = bytearray(len(single))
        slot = (len(single) - 112) // max(1, (sizes[-1][2]))
        for r in range(world):
            off, s_lo, s_hi, path = sizes[r]
            n = (112 if r == 0 else 0) + (s_hi - s_lo) * slot
            spi[off: off + n] = gathered[r][:n]
        ok = bytes(spi) == single
        print(f"shard_gloo_check world={world} records={args.records} path={[s[3] for s in sizes]} identical={ok}")
        if not ok:
            sys.exit(1)
    del parts
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
