"""Benchmark: device-resident Sparkey hash-file (.spi) builds on MI355X.

One step = one full IndexHash.createNew-equivalent build of the BASELINE.json config C2 log
(10M PUTs, 16-byte keys, 100-byte values, NONE) already resident in HBM, into a device-resident
.spi image (header + table): framing, MurmurHash3, placement, stats.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--entries 10000000] [--no-cpu-baseline]

With N > 1 (torch.distributed.run, one rank per GPU) every rank builds its own independent log of
the same shape (weak scaling, no data-path collective; see DESIGN.md "multi-GPU").
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "sparkey-java_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def stage_bytes(stage, n, data_end, slot, cap):
    """Algorithmic bytes per launch of each stage (DESIGN.md "rooflines")."""
    log = data_end - 84
    table = 112 + slot * cap
    return {
        "speculate": log,                     # every log byte read once
        "walk": 0,
        "count": 0,
        "scan_chunks": 0,
        "emit": log + 16 * n,                 # log read once, 16-byte (hash, address) entries written
        "scan_buckets": 0,
        "scatter": 32 * n,                    # entries read + written once
        "summary": 16 * n,                    # entries read once
        "carry": 0,
        "place": 16 * n + slot * cap,         # entries read once, every slot written once
        "verify": 0,
        "stats": slot * cap,                  # table read once
    }.get(stage, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--entries", type=int, default=10_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=1)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    import sparkey
    from sparkey import _native, synth

    n = args.entries
    t0 = time.time()
    log_np = synth.fixed_log(n, 16, 100, seed=args.seed + rank, file_id=0x5EED0000 + rank)
    gen_s = time.time() - t0
    header = log_np[:84].tobytes()
    log_len = log_np.size
    d_log = torch.from_numpy(log_np).to(dev)
    seed = 0x2545F491
    opts = _native.make_opts(hash_size=0, hash_seed=seed, sparsity=0.0, method=_native.METHOD_IN_MEMORY,
                             device=local_rank)
    out_len = _native.index_size(header, opts)
    d_out = torch.empty(out_len, dtype=torch.uint8, device=dev)
    plan = _native.Plan(local_rank, log_len, n)
    stream = torch.cuda.current_stream(dev)
    s_handle = stream.cuda_stream

    def one_build():
        return plan.build(header, d_log.data_ptr(), log_len, d_out.data_ptr(), out_len, opts, s_handle)

    for _ in range(args.warmup):
        stats = one_build()

    # timed region: K builds; per-stage HIP events recorded on the build stream
    plan.set_profiling(True)
    stage_acc = {}
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        stats = one_build()
        for name, ms in plan.stage_times():
            stage_acc[name] = stage_acc.get(name, 0.0) + ms
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    plan.set_profiling(False)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_per_step = elapsed * 1000.0 / args.steps
    total_keys = n * world * args.steps
    value = total_keys / elapsed
    slot = stats.hash_size + stats.address_size
    cap = stats.capacity
    data_end = log_len
    stage_ms = {k: v / args.steps for k, v in stage_acc.items()}
    dom = max(stage_ms, key=lambda k: stage_ms[k]) if stage_ms else None
    dom_bytes = stage_bytes(dom, n, data_end, slot, cap) if dom else 0
    achieved = dom_bytes / (stage_ms[dom] * 1e-3) / 1e9 if dom and stage_ms[dom] > 0 else 0.0
    b_alg = (data_end - 84) + 112 + slot * cap
    build_gbs = b_alg / (ms_per_step * 1e-3) / 1e9

    # sanity of the device result + host-to-host rate (H2D log, build, D2H .spi)
    spi_head = d_out[:112].cpu().numpy().tobytes()
    num_entries = int.from_bytes(spi_head[60:68], "little")
    assert num_entries == n and stats.placement_path == 0, stats.as_dict()
    h2h = None
    if rank == 0:
        pinned = torch.from_numpy(log_np).pin_memory()
        host_out = torch.empty(out_len, dtype=torch.uint8).pin_memory()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            d_log.copy_(pinned, non_blocking=True)
            one_build()
            host_out.copy_(d_out, non_blocking=True)
            torch.cuda.synchronize(dev)
        h2h = n * reps / (time.perf_counter() - t1)

    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if dom and os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            traffic = pmc.get("per_launch_hbm_bytes", {}).get(dom)
        except Exception:
            traffic = None

    cpu = None
    parity = None
    if rank == 0 and not args.no_cpu_baseline:
        import oracle
        oracle.build()
        log_bytes = log_np.tobytes()
        t2 = time.perf_counter()
        want = oracle.build_index(log_bytes, seed, method=oracle.IN_MEMORY)
        cpu_s = time.perf_counter() - t2
        got = d_out.cpu().numpy().tobytes()
        parity = got == want
        cpu = {"value": n / cpu_s, "unit": "keys/s", "cores": 1, "kind": "port",
               "sample": f"full C2 log ({n} entries), oracle IN_MEMORY sequential restatement, 1 thread, "
                         f"{cpu_s:.1f} s", "bit_identical_to_gpu": parity}

    if rank == 0:
        line = {
            "metric": "keys/s device-resident hash-file build, 10M entries; HBM GB/s vs peak",
            "value": value,
            "unit": "keys/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic",
            "config": {"workload": "C2: 10M PUTs x (16 B key, 100 B value), CompressionType.NONE, IN_MEMORY",
                       "entries_per_gpu": n, "log_bytes": int(log_len), "hash_bytes": stats.hash_size,
                       "address_bytes": stats.address_size, "capacity": int(cap), "spi_bytes": int(out_len),
                       "parallelism": f"independent shards x{world}" if world > 1 else "single"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "algorithmic_bytes_per_launch": dom_bytes,
                         "avg_launch_ms": stage_ms.get(dom) if dom else None},
            "build_hbm_gbs": build_gbs,
            "build_algorithmic_bytes": b_alg,
            "stage_ms": stage_ms,
            "host_to_host_keys_per_s": h2h,
            "cpu_baseline": cpu,
            "gen_s": gen_s,
            "version": sparkey.version(),
        }
        print(json.dumps(line))
    plan.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
