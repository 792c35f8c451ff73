"""Sharded exact-path rehearsal on ONE GPU: the churn log (overwrites + DELETEs) built
by sparkey_build_index_mem with opts.num_gpus = N ranks as threads of this process on cuda:0
(the shard_transport switch = 2), against the single-GPU device build of the same log.
Prints per-rank phase times (host wall, sparkey_multi_phase_*) and checks the .spi is identical.

    python tools/shard_rehearsal.py --entries 10000000 --ranks 1,2,4 [--reps 3]

Under rocprofv3 --kernel-trace the kernels' own durations separate GPU work from waiting: ranks
sharing one GPU run their kernels concurrently, so a rank's wall phase can hold other ranks' work."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparkey-java_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--entries", type=int, default=10_000_000)
    ap.add_argument("--ranks", default="1,2,4")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--full-table", action="store_true", help="the old full-capacity local table (A/B)")
    args = ap.parse_args()
    import torch
    from sparkey import _native, synth

    _native.debug_set("shard_transport", 2)
    if args.full_table:
        _native.debug_set("exact_full_table", 1)
    n = args.entries
    t0 = time.time()
    log = synth.churn_log(n, int(n * 0.8), 0.1, seed=9)
    raw = log.tobytes()
    print(f"log: {n} records, {len(raw)} bytes ({time.time() - t0:.1f} s)", flush=True)
    dev = torch.device("cuda", 0)
    opts = _native.make_opts(hash_seed=5, device=0)
    size = _native.index_size(raw[:84], opts)
    d_log = torch.from_numpy(log).to(dev)
    d_spi = torch.empty(size, dtype=torch.uint8, device=dev)
    plan = _native.Plan(0, len(raw), n)
    ms = []
    for _ in range(args.reps + 1):
        torch.cuda.synchronize()
        t = time.perf_counter()
        st = plan.build(raw[:84], d_log.data_ptr(), len(raw), d_spi.data_ptr(), size, opts)
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t) * 1e3)
    single = d_spi.cpu().numpy().tobytes()
    plan.close()
    del d_log, d_spi
    res = {"entries": n, "single_gpu_device_build_ms": min(ms[1:]), "single_placement_path": st.placement_path}
    print(json.dumps(res), flush=True)
    for w in [int(x) for x in args.ranks.split(",")]:
        if w < 2:
            continue
        o = _native.make_opts(hash_seed=5, device=0, num_gpus=w)
        walls, per_rank = [], None
        for i in range(args.reps + 1):
            t = time.perf_counter()
            got, st = _native.build_index_mem(raw, o)
            walls.append((time.perf_counter() - t) * 1e3)
            if i == args.reps:
                per_rank = [_native.multi_last_phases(r) for r in range(w)]
        line = {"ranks": w, "sharded": st.sharded, "identical_to_single_gpu": got == single,
                "wall_ms_mem_to_mem": min(walls[1:]),
                "phase_ms": {f"rank{r}": {k: round(v, 3) for k, v in ph} for r, ph in enumerate(per_rank)}}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
