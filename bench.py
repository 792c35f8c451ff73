"""Benchmark: device-resident Sparkey hash-file (.spi) builds on MI355X.

One step = one full IndexHash.createNew-equivalent build (framing, MurmurHash3, placement, stats,
header) of a C2-shaped log (16-byte keys, 100-byte values, NONE) already resident in HBM, into a
device-resident .spi image.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--entries N] [--no-cpu-baseline]
                    [--workload c2|c3|c4|c5|churn|snappy|zstd|get|append]

N = 1: the C2 log (10M records) built on one GPU; the line carries the per-stage roofline and the
CPU baseline (the oracle's sequential IN_MEMORY restatement on the host, timed on the same log).
--workload c4: BASELINE's configs[3] size, 1B records, on one GPU.
N > 1 (torch.distributed.run, one rank per GPU, RCCL): ONE index over a log of N x 125M C2-shaped
records (C4 -- 1B records -- at N = 8) whose byte range is split across the ranks, each
rank generating its range in HBM -- weak scaling, 125M records per GPU; afterwards every rank's slice
is checked against one single-GPU build of the whole log.  Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import platform
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "sparkey-java_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "keys/s device-resident hash-file build, 10M entries; HBM GB/s vs peak"
PMC_SUMMARIES = [os.path.join(ROOT, "profiles", f) for f in ("r06_pmc_summary.json", "r05_pmc_summary.json", "r04_pmc_summary.json", "r03_pmc_summary.json",
                                                               "r02_pmc_summary.json", "r01_pmc_summary.json")]
HASH_SEED = 0x2545F491


def stage_bytes(stage, n, data_end, slot, cap, passes=2, comp_end=None, eb=16):
    """Algorithmic bytes per launch of each stage.  passes: partition passes left to
    the partition stage (1 when the uniform framing wrote the digit regions itself); eb: bytes an
    entry takes between the framing and the placement (stats.entry_bytes: 12 on uniform logs)."""
    log = data_end - 84
    return {
        "frame": log + eb * n,                # log read once, (hash, address) entries written
        "emit": log + 16 * n,                 # serial path: 16-byte entries
        "partition": passes * 2 * eb * n,     # radix passes, entries read + written once each
        "summary": eb * n,                    # entries read once
        "place": eb * n + slot * cap,         # entries read once, every slot written once
        "stats": slot * cap,                  # table read once
        "exact": 3 * 16 * n + 2 * slot * cap,  # entries read, grouped, replayed; segment slots cleared + written
        # SNAPPY (data_end = the virtual log's end): blocks read once, decompressed bytes written once
        "snappy_decode": (comp_end or data_end) - 84 + log,
        "snappy_rewrite": 2 * slot * cap,      # internal table read, final table written
        "zstd_decode": (comp_end or data_end) - 84 + log,   # (as SNAPPY)
        "zstd_rewrite": 2 * slot * cap,
    }.get(stage, 0)


def pmc_traffic(workload, stage):
    """HBM bytes per launch of `stage` on `workload` from the committed rocprofv3 PMC summary
    (tools/pmc_summary.py), or None when that workload's kernel was not counted."""
    for path in PMC_SUMMARIES:
        try:
            with open(path) as f:
                pmc = json.load(f)
        except (OSError, ValueError):
            continue
        per = pmc.get("per_launch_hbm_bytes_by_workload", {}).get(workload)
        if per is None and workload == "c2":
            per = pmc.get("per_launch_hbm_bytes")
        if per and stage in per:
            return per[stage]
    return None


def host_info():
    """The CPU the baseline ran on: model, logical CPUs of the machine and of this process."""
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count()
    return {"cpu_model": model, "nproc": os.cpu_count(), "usable_cpus": usable}


WORKLOADS = {
    "c2": {"name": "C2: 10M PUTs x (16 B key, 100 B value), CompressionType.NONE, IN_MEMORY", "sorting": False,
           "path": 0},
    "c3": {"name": "C3: PUTs x (8-64 B key, 100 B value), CompressionType.NONE, IN_MEMORY", "sorting": False,
           "path": 0},
    "c1x": {"name": "WriteHashBenchmark's data at its 10M parameter: put(\"key_\" + i, \"value_\" + i), block size "
                    "1024, CompressionType.NONE, IN_MEMORY (WriteHashBenchmark.java:43-76)", "sorting": False, "path": 0},
    "c5": {"name": "C5: C3 log, SORTING constructionMethod", "sorting": True, "path": 0},
    "churn": {"name": "C2 shape with overwrites and DELETEs: keys from a pool of 0.8 n, 10% DELETE records, "
                      "IN_MEMORY (exact replay over slot segments)", "sorting": False, "path": 2},
    "snappy": {"name": "C2 records (10M PUTs x (16 B key, 100 B value)), CompressionType.SNAPPY, 64 KiB blocks, "
                       "IN_MEMORY", "sorting": False, "path": 0},
    "zstd": {"name": "C2 records (10M PUTs x (16 B key, 100 B value)), CompressionType.ZSTD (level 3), 64 KiB "
                     "blocks, IN_MEMORY", "sorting": False, "path": 0},
    "append": {"name": "GPU log producer (batched LogWriter.put)", "sorting": False, "path": 0},
    "c4": {"name": "C4: 1B PUTs x (16 B key, 100 B value), CompressionType.NONE, IN_MEMORY, one GPU (118 GB log "
                   "in HBM)", "sorting": False, "path": 0},
    "get": {"name": "batched IndexHash.get of every key of the C2 index (log and index resident in HBM)",
            "sorting": False, "path": 0},
}


def appends(args, dev):
    """--workload append: one step = LogWriter.put of n C2 records in one batch (sparkey_log_append),
    keys and values already in HBM; the result is checked byte for byte against the C2 log."""
    import numpy as np
    import sparkey
    from sparkey import synth
    from sparkey.gpu_log import GpuLogAppender, new_log_header
    n = args.entries
    log_np = synth.fixed_log(n, 16, 100, seed=args.seed, file_id=0x5EED0000)
    recs = log_np[84:].reshape(n, 118)
    keys = torch.from_numpy(np.ascontiguousarray(recs[:, 2:18]).reshape(-1)).to(dev)
    vals = torch.from_numpy(np.ascontiguousarray(recs[:, 18:]).reshape(-1)).to(dev)
    koff = torch.arange(0, 16 * (n + 1), 16, dtype=torch.int64, device=dev)
    voff = torch.arange(0, 100 * (n + 1), 100, dtype=torch.int64, device=dev)
    kind = torch.ones(n, dtype=torch.uint8, device=dev)
    out = torch.empty(118 * n, dtype=torch.uint8, device=dev)
    app = GpuLogAppender(dev.index)
    stream = torch.cuda.Stream(dev)

    def step():
        hdr = new_log_header(0x5EED0000)
        app.append_device(hdr, kind, keys, koff, vals, voff, n, out, out.numel(), stream.cuda_stream)
        return hdr

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        hdr = step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    assert bytes(hdr) == log_np[:84].tobytes(), "header differs from the C2 log's"
    assert torch.equal(out, torch.from_numpy(log_np[84:]).to(dev)), "records differ from the C2 log"
    app.close()
    ms = el * 1000.0 / args.steps
    return {"metric": "records/s, batched LogWriter.put of the C2 records (extra measurement, not the headline)",
            "value": n * args.steps / el, "ms_per_step": ms, "unit": "records/s",
            "config": {"workload": "GPU log producer: 10M PUTs (16 B key, 100 B value) -> the C2 log bytes",
                       "entries": n, "log_bytes": int(log_np.size), "parallelism": "single"},
            "hbm_gbs": (116 * n + 118 * n) / (ms * 1e-3) / 1e9,
            "roofline": None, "cpu_baseline": None, "version": sparkey.version()}


def lookups(args, dev):
    """--workload get: one step = IndexHash.get of all n C2 keys in one batch (sparkey_get_batch)."""
    import numpy as np
    import sparkey
    from sparkey import _native, synth
    n = args.entries
    log_np = synth.fixed_log(n, 16, 100, seed=args.seed, file_id=0x5EED0000)
    header = log_np[:84].tobytes()
    d_log = torch.from_numpy(log_np).to(dev)
    opts = _native.make_opts(hash_size=0, hash_seed=HASH_SEED, device=dev.index)
    out_len = _native.index_size(header, opts)
    d_index = torch.empty(out_len, dtype=torch.uint8, device=dev)
    plan = _native.Plan(dev.index, log_np.size, n)
    plan.build(header, d_log.data_ptr(), log_np.size, d_index.data_ptr(), out_len, opts)
    keys = torch.from_numpy(np.ascontiguousarray(log_np[84:].reshape(n, 118)[:, 2:18]).reshape(-1)).to(dev)
    key_off = torch.arange(0, 16 * (n + 1), 16, dtype=torch.int64, device=dev)
    pos = torch.empty(n, dtype=torch.int64, device=dev)
    ln = torch.empty(n, dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(dev)

    def step():
        plan.get_batch(d_log.data_ptr(), log_np.size, d_index.data_ptr(), out_len, keys.data_ptr(),
                       key_off.data_ptr(), n, pos.data_ptr(), ln.data_ptr(), stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    want = torch.arange(n, dtype=torch.int64, device=dev) * 118 + 84 + 18
    assert bool((pos == want).all()) and bool((ln == 100).all()), "lookup results differ from the log layout"
    plan.close()
    return {"metric": "lookups/s, batched IndexHash.get over the C2 index (extra measurement, not the headline)",
            "value": n * args.steps / el, "ms_per_step": el * 1000.0 / args.steps, "unit": "lookups/s",
            "config": {"workload": WORKLOADS["get"]["name"], "entries": n, "log_bytes": int(log_np.size),
                       "spi_bytes": int(out_len), "parallelism": "single"},
            "roofline": None, "cpu_baseline": None, "version": sparkey.version()}


def single_gpu(args, dev):
    import sparkey
    from sparkey import _native, synth

    n = args.entries
    wl = WORKLOADS[args.workload]
    method = _native.METHOD_SORTING if wl["sorting"] else _native.METHOD_IN_MEMORY
    t0 = time.time()
    if args.workload == "c2":
        log_np = synth.fixed_log(n, 16, 100, seed=args.seed, file_id=0x5EED0000)
    elif args.workload in ("c3", "c5"):
        log_np = synth.mixed_log(n, 8, 64, 100, seed=args.seed + 2)
    elif args.workload == "c1x":
        log_np = synth.key_value_log_np(n)
    elif args.workload in ("snappy", "zstd"):
        log_np = synth.snappy_log(synth.fixed_log(n, 16, 100, seed=args.seed, file_id=0x5EED0000), 118, 65536,
                                  codec=args.workload)
    else:
        log_np = synth.churn_log(n, int(n * 0.8), 0.1, seed=args.seed + 4)
    gen_s = time.time() - t0
    header = log_np[:84].tobytes()
    log_len = log_np.size
    d_log = torch.from_numpy(log_np).to(dev)
    opts = _native.make_opts(hash_size=0, hash_seed=HASH_SEED, sparsity=0.0, method=method, device=dev.index)
    out_len = _native.index_size(header, opts)
    d_out = torch.empty(out_len, dtype=torch.uint8, device=dev)
    plan = _native.Plan(dev.index, log_len, n)
    stream = torch.cuda.Stream(dev)
    s_handle = stream.cuda_stream

    def one_build():
        return plan.build(header, d_log.data_ptr(), log_len, d_out.data_ptr(), out_len, opts, s_handle)

    torch.cuda.synchronize(dev)
    for _ in range(args.warmup):
        stats = one_build()
    # timed region: K builds
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        stats = one_build()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    headline_spi = d_out.cpu().numpy().tobytes()  # the headline path's own output (checked below)
    # stage times: the same builds again with HIP events recorded at the stage boundaries on the
    # build's stream (each event adds a few microseconds between kernels, so they stay out of the
    # timed region)
    plan.set_profiling(True)
    stage_acc = {}
    n_prof = max(1, min(args.steps, 10))
    for _ in range(n_prof):
        one_build()
        for name, ms in plan.stage_times():
            stage_acc[name] = stage_acc.get(name, 0.0) + ms
    torch.cuda.synchronize(dev)
    plan.set_profiling(False)

    ms_per_step = elapsed * 1000.0 / args.steps
    slot = stats.hash_size + stats.address_size
    cap = stats.capacity
    stage_ms = {k: v / n_prof for k, v in stage_acc.items()}
    dom = max(stage_ms, key=lambda k: stage_ms[k]) if stage_ms else None
    passes = stats.partition_passes
    # SNAPPY: the inner build's stages run over the virtual log (84 + 118 n bytes for C2 records)
    frame_end = 84 + 118 * n if args.workload in ("snappy", "zstd") else log_len
    eb = stats.entry_bytes or 16
    dom_bytes = stage_bytes(dom, n, frame_end, slot, cap, passes, comp_end=log_len, eb=eb) if dom else 0
    achieved = dom_bytes / (stage_ms[dom] * 1e-3) / 1e9 if dom and stage_ms[dom] > 0 else 0.0
    b_alg = (log_len - 84) + 112 + slot * cap
    assert stats.placement_path == wl["path"] and stats.framing_path in (0, 2, 4), stats.as_dict()
    assert wl["path"] != 0 or stats.num_entries == n, stats.as_dict()

    if args.quick:  # (profiling runs: the timed builds only)
        plan.close()
        return {"value": n * args.steps / elapsed, "ms_per_step": ms_per_step,
                "config": {"workload": wl["name"], "entries": n, "log_bytes": int(log_len), "parallelism": "single"},
                "stage_ms": stage_ms, "roofline": None, "cpu_baseline": None, "version": sparkey.version()}
    # host-to-host rate (north_star): H2D of the log from pinned memory, the build, D2H of the .spi
    pinned = torch.from_numpy(log_np).pin_memory()
    host_out = torch.empty(out_len, dtype=torch.uint8).pin_memory()
    torch.cuda.synchronize(dev)
    reps = 3
    t1 = time.perf_counter()
    with torch.cuda.stream(stream):
        for _ in range(reps):
            d_log.copy_(pinned, non_blocking=True)
            one_build()
            host_out.copy_(d_out, non_blocking=True)
            stream.synchronize()
    h2h = n * reps / (time.perf_counter() - t1)

    # the same workload through the general speculative framing (k_frame), when the log's records are
    # uniform and the default build took k_frame_uniform
    general = general_spi = None
    if stats.framing_path == 2:
        _native.debug_set("no_uniform", 1)
        try:
            one_build()
            torch.cuda.synchronize(dev)
            plan.set_profiling(True)
            g_acc, g_steps = {}, max(3, args.steps // 2)
            t_g = time.perf_counter()
            for _ in range(g_steps):
                g_stats = one_build()
                for name, ms in plan.stage_times():
                    g_acc[name] = g_acc.get(name, 0.0) + ms
            torch.cuda.synchronize(dev)
            g_el = time.perf_counter() - t_g
            plan.set_profiling(False)
            assert g_stats.framing_path in (0, 4), g_stats.as_dict()
            general_spi = d_out.cpu().numpy().tobytes()  # (compared with the headline build below)
            g_stage = {k: v / g_steps for k, v in g_acc.items()}
            general = {"ms_per_step": g_el * 1000.0 / g_steps, "keys_per_s": n * g_steps / g_el,
                       "stage_ms": g_stage,
                       "frame_achieved_gbs": stage_bytes("frame", n, frame_end, slot, cap) / (g_stage["frame"] * 1e-3) / 1e9}
        finally:
            _native.debug_set("no_uniform", None)

    # file -> file (north_star: "log file in, hash file out"): sparkey_build_index_file, the entry
    # point the JNI shim calls, on the same log written to a file; page-cache warm, fsync off (the
    # writer's default), its per-device context kept across calls
    file_rate = file_spi = None
    file_phases = None
    tmpdir = tempfile.mkdtemp(prefix="sparkey_bench_")
    log_path, spi_path = os.path.join(tmpdir, "bench.spl"), os.path.join(tmpdir, "bench.spi")
    try:
        log_np.tofile(log_path)
        if args.workload in ("c1x", "c2", "c3", "c5", "churn", "snappy", "zstd"):
            # as SparkeyWriter.writeHash does it: a fresh "-tmp" file, then renamed over the .spi
            # (each timed call writes a new file; replacing the old .spi -- an unlink of ~200 MB of
            # page cache, ~20 ms on the box -- happens after the clock stops)
            _native.build_index_file(log_path, spi_path, opts)
            reps_f = 3
            file_phases = {}
            t_calls = 0.0
            for i in range(reps_f):
                tmp = f"{spi_path}-tmp{i}"
                t_f = time.perf_counter()
                _native.build_index_file(log_path, tmp, opts)
                t_calls += time.perf_counter() - t_f
                for k, v in _native.file_last_phases().items():
                    file_phases[k] = file_phases.get(k, 0.0) + v / reps_f
            for i in range(reps_f):
                os.replace(f"{spi_path}-tmp{i}", spi_path)
            file_rate = n * reps_f / t_calls
            with open(spi_path, "rb") as f:
                file_spi = f.read()
            _native.release_cached_resources()

        cpu = None
        if not args.no_cpu_baseline:
            import oracle
            oracle.build()
            mname = "SORTING" if wl["sorting"] else "IN_MEMORY"
            method_o = oracle.SORTING if wl["sorting"] else oracle.IN_MEMORY
            t2 = time.perf_counter()
            want = oracle.build_index(log_np, HASH_SEED, method=method_o)
            cpu_s = time.perf_counter() - t2
            # the same restatement file -> file: read the log file, build, write the .spi file
            t3 = time.perf_counter()
            with open(log_path, "rb") as f:
                log_file_bytes = f.read()
            want_f = oracle.build_index(log_file_bytes, HASH_SEED, method=method_o)
            with open(spi_path + ".cpu", "wb") as f:
                f.write(want_f)
            cpu_file_s = time.perf_counter() - t3
            del log_file_bytes
            cpu = {"value": n / cpu_s, "unit": "keys/s", "cores": 1, "kind": "port",
                   "sample": f"full {args.workload.upper()} log ({n} records), oracle {mname} sequential "
                             f"restatement (oracle/), 1 thread, {cpu_s:.2f} s", "host": host_info(),
                   "file_to_file_keys_per_s": n / cpu_file_s,
                   "bit_identical_to_gpu": headline_spi == want,
                   "file_bit_identical_to_gpu": None if file_spi is None else file_spi == want_f}
    finally:
        shutil.rmtree(tmpdir, ignore_errors=True)
    plan.close()
    parity = None
    if args.workload == "c2" and not args.no_parity:
        del d_log, d_out
        torch.cuda.empty_cache()
        parity = parity_checks(args, dev, headline_spi, general_spi)
        if cpu is not None:
            parity["c2_device_bit_identical_to_oracle"] = cpu["bit_identical_to_gpu"]
            parity["c2_file_to_file_bit_identical_to_oracle"] = cpu["file_bit_identical_to_gpu"]
    if general is not None:
        general["bit_identical_to_headline"] = general_spi == headline_spi
    return {
        "value": n * args.steps / elapsed, "ms_per_step": ms_per_step,
        "config": {"workload": wl["name"],
                   "entries": n, "log_bytes": int(log_len), "hash_bytes": stats.hash_size,
                   "address_bytes": stats.address_size, "capacity": int(cap), "spi_bytes": int(out_len),
                   "parallelism": "single"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     # (counters are keyed by workload and size: "c3" is the 10M run, "c3_100000000" 100M)
                     "traffic": pmc_traffic(args.workload if n == 10_000_000 else f"{args.workload}_{n}",
                                            {("frame", 2): "frame_uniform",
                                                            ("partition", 1): "partition_regions"}.get(
                         (dom, stats.framing_path if dom == "frame" else passes), dom)),
                     "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_ms": stage_ms.get(dom) if dom else None},
        "build_hbm_gbs": b_alg / (ms_per_step * 1e-3) / 1e9,
        "stage_gbs": {k: stage_bytes(k, n, frame_end, slot, cap, passes, comp_end=log_len, eb=eb) / (v * 1e-3) / 1e9
                      for k, v in stage_ms.items() if v > 0 and stage_bytes(k, n, frame_end, slot, cap, passes)},
        "build_algorithmic_bytes": b_alg,
        "stage_ms": stage_ms,
        "framing": {0: "k_frame (speculative)", 1: "serial walk", 2: "k_frame_uniform (uniform records)",
                    4: "k_frame3 (short/long walks, one-byte VLQs)"}[stats.framing_path],
        "general_framing": general,
        "host_to_host_keys_per_s": h2h,
        "file_to_file_keys_per_s": file_rate,
        "file_to_file_phase_ms": file_phases,
        "cpu_baseline": cpu,
        "parity": parity,
        "gen_s": gen_s,
        "version": sparkey.version(),
    }


def single_gpu_c4(args, dev):
    """--workload c4: BASELINE.json configs[3]'s 1B records (16 B key, 100 B value) on ONE GPU -- a
    118 GB log generated in HBM (sparkey/synth_device.py), a 20.8 GB .spi.  Timed like the C2 line;
    checked by the header's numEntries and IndexHash.get of every 1000th key (sparkey_get_batch), and
    the CPU baseline's bit-identity on a bounded C2-shaped sample of the same records."""
    import sparkey
    from sparkey import _native, synth_device
    n = args.entries
    t0 = time.time()
    d_log = synth_device.fixed_log(n, 16, 100, seed=args.seed, file_id=0x5EED0000, device=dev)
    torch.cuda.synchronize(dev)
    gen_s = time.time() - t0
    header = d_log[:84].cpu().numpy().tobytes()
    log_len = d_log.numel()
    opts = _native.make_opts(hash_size=0, hash_seed=HASH_SEED, sparsity=0.0, method=_native.METHOD_IN_MEMORY,
                             device=dev.index)
    out_len = _native.index_size(header, opts)
    d_out = torch.empty(out_len, dtype=torch.uint8, device=dev)
    plan = _native.Plan(dev.index)
    stream = torch.cuda.Stream(dev)

    def one_build():
        return plan.build(header, d_log.data_ptr(), log_len, d_out.data_ptr(), out_len, opts, stream.cuda_stream)

    for _ in range(args.warmup):
        stats = one_build()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        stats = one_build()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    plan.set_profiling(True)
    stage_acc, n_prof = {}, max(1, min(args.steps, 5))
    for _ in range(n_prof):
        one_build()
        for name, ms in plan.stage_times():
            stage_acc[name] = stage_acc.get(name, 0.0) + ms
    plan.set_profiling(False)
    stage_ms = {k: v / n_prof for k, v in stage_acc.items()}
    slot = stats.hash_size + stats.address_size
    cap = stats.capacity
    passes = stats.partition_passes
    dom = max(stage_ms, key=lambda k: stage_ms[k])
    dom_bytes = stage_bytes(dom, n, log_len, slot, cap, passes, eb=stats.entry_bytes or 16)
    achieved = dom_bytes / (stage_ms[dom] * 1e-3) / 1e9
    b_alg = (log_len - 84) + 112 + slot * cap
    ms_per_step = elapsed * 1000.0 / args.steps
    assert stats.num_entries == n and stats.placement_path == 0, stats.as_dict()
    # IndexHash.get of every 1000th key: the value of record i sits at 84 + 118 i + 18, 100 bytes
    idx = torch.arange(0, n, 1000, dtype=torch.int64, device=dev)
    keys = synth_device.fixed_keys(idx, seed=args.seed).reshape(-1)
    key_off = torch.arange(0, 16 * (idx.numel() + 1), 16, dtype=torch.int64, device=dev)
    pos = torch.empty(idx.numel(), dtype=torch.int64, device=dev)
    vlen = torch.empty(idx.numel(), dtype=torch.int64, device=dev)
    plan.get_batch(d_log.data_ptr(), log_len, d_out.data_ptr(), out_len, keys.data_ptr(), key_off.data_ptr(),
                   idx.numel(), pos.data_ptr(), vlen.data_ptr())
    gets_ok = bool((pos == idx * 118 + 84 + 18).all()) and bool((vlen == 100).all())
    hdr = d_out[:112].cpu().numpy().tobytes()
    plan.close()
    del d_log, d_out, keys, key_off, pos, vlen
    torch.cuda.empty_cache()
    cpu = None
    if not args.no_cpu_baseline:  # a bounded sample: the first 50M of the same records as their own log
        import oracle
        oracle.build()
        m = 50_000_000
        d_s = synth_device.fixed_log(m, 16, 100, seed=args.seed, file_id=0x5EED0000, device=dev)
        s_hdr = d_s[:84].cpu().numpy().tobytes()
        s_len = _native.index_size(s_hdr, opts)
        d_so = torch.empty(s_len, dtype=torch.uint8, device=dev)
        p2 = _native.Plan(dev.index)
        p2.build(s_hdr, d_s.data_ptr(), d_s.numel(), d_so.data_ptr(), s_len, opts)
        p2.close()
        gpu_sample = d_so.cpu().numpy()
        host = d_s.cpu().numpy()
        del d_s, d_so
        t2 = time.perf_counter()
        want = oracle.build_index(host, HASH_SEED)
        cpu_s = time.perf_counter() - t2
        cpu = {"value": m / cpu_s, "unit": "keys/s", "cores": 1, "kind": "port",
               "sample": f"the first {m} of the C4 records as their own log, oracle IN_MEMORY sequential "
                         f"restatement (oracle/), 1 thread, {cpu_s:.2f} s", "host": host_info(),
               "bit_identical_to_gpu_on_sample": bool(np_equal(gpu_sample, want))}
    return {
        "value": n * args.steps / elapsed, "ms_per_step": ms_per_step,
        "config": {"workload": WORKLOADS["c4"]["name"], "entries": n, "log_bytes": int(log_len),
                   "hash_bytes": stats.hash_size, "address_bytes": stats.address_size, "capacity": int(cap),
                   "spi_bytes": int(out_len), "parallelism": "single"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": pmc_traffic(f"c4_{n}", {("frame", 2): "frame_uniform", ("partition", 1):
                                                        "partition_regions"}.get(
                         (dom, stats.framing_path if dom == "frame" else passes), dom)),
                     "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_ms": stage_ms[dom]},
        "build_hbm_gbs": b_alg / (ms_per_step * 1e-3) / 1e9,
        "build_algorithmic_bytes": b_alg,
        "stage_ms": stage_ms,
        "checks": {"num_entries": int.from_bytes(hdr[60:68], "little"), "gets_every_1000th_key_ok": gets_ok},
        "cpu_baseline": cpu, "gen_s": gen_s, "version": sparkey.version(),
    }


def np_equal(a, b_bytes):
    import numpy as np
    return a.size == len(b_bytes) and np.array_equal(a, np.frombuffer(b_bytes, dtype=np.uint8))


def parity_checks(args, dev, headline_spi, general_spi):
    """Outside every timed region (N = 1, default workload): the device paths the headline does not
    take, each checked byte for byte -- the general framing of the C2 log against the headline build,
    and the C3-shaped (k_frame3), C5 (SORTING), exact-path, SNAPPY and ZSTD builds against the oracle.
    Returns {check: bool} plus the sizes used."""
    import oracle
    from sparkey import _native, synth
    oracle.build()
    out = {"c2_general_framing_equals_headline": None if general_spi is None else general_spi == headline_spi}
    n3 = args.parity_c3_entries

    def gpu_vs_oracle(log_np, seed, method, want_path=None):
        header = log_np[:84].tobytes()
        opts = _native.make_opts(hash_size=0, hash_seed=seed, method=method, device=dev.index)
        size = _native.index_size(header, opts)
        d_log = torch.from_numpy(log_np).to(dev)
        d_out = torch.empty(size, dtype=torch.uint8, device=dev)
        plan = _native.Plan(dev.index, log_np.size, 0)
        try:
            st = plan.build(header, d_log.data_ptr(), log_np.size, d_out.data_ptr(), size, opts)
            got = d_out.cpu().numpy().tobytes()
        finally:
            plan.close()
        del d_log, d_out
        want = oracle.build_index(log_np, seed, method=method)
        return got == want and (want_path is None or st.framing_path == want_path), st

    t0 = time.time()
    c3 = synth.mixed_log(n3, 8, 64, 100, seed=args.seed + 2)
    ok, st = gpu_vs_oracle(c3, HASH_SEED, _native.METHOD_IN_MEMORY)
    out[f"c3_{n3}_in_memory"] = ok
    out["c3_framing_path"] = st.framing_path
    ok, _ = gpu_vs_oracle(c3, HASH_SEED, _native.METHOD_SORTING)
    out[f"c5_{n3}_sorting"] = ok
    del c3
    churn = synth.churn_log(1_000_000, 800_000, 0.1, seed=args.seed + 4)
    for name, method in (("in_memory", _native.METHOD_IN_MEMORY), ("sorting", _native.METHOD_SORTING)):
        ok, st = gpu_vs_oracle(churn, HASH_SEED, method)
        out[f"churn_1000000_exact_{name}"] = ok and st.placement_path == 2
    del churn
    for codec in ("snappy", "zstd"):
        clog = synth.snappy_log(synth.fixed_log(1_000_000, 16, 100, seed=args.seed, file_id=0x5EED0000), 118, 65536,
                                codec=codec)
        ok, _ = gpu_vs_oracle(clog, HASH_SEED, _native.METHOD_IN_MEMORY)
        out[f"{codec}_1000000"] = ok
    out["seconds"] = round(time.time() - t0, 1)
    return out


def block_sums(t, block=1 << 28):
    """Per 256 MiB block of a device byte tensor: (sum of its int64 words, sum of word * (2 * position
    + 1)), wrapping mod 2^64, plus the bytes after the last whole word -- a checksum of checksums that
    compares two .spi images without moving them to the host."""
    n8 = t.numel() // 8
    words = t[: n8 * 8].view(torch.int64)
    out = []
    for a in range(0, n8, block // 8):
        w = words[a: a + block // 8]
        pos = torch.arange(a, a + w.numel(), dtype=torch.int64, device=t.device) * 2 + 1
        out.append((int(w.sum()), int((w * pos).sum())))
    return out, t[n8 * 8:].cpu().numpy().tobytes()


def sharded(args, dev, world, rank):
    """N > 1 (one process per GPU): ONE index over a log of N x entries C2-shaped records (C4 at N = 8 with
    the default 125M per GPU: 1B records) whose byte range is split across the ranks; each rank generates
    its range in HBM.  Each rank runs sparkey_shard_build -- the C++ orchestrator behind the C-ABI
    (csrc/shard_host.cpp) -- over its own RCCL communicator (unique id from rank 0 via
    torch.distributed, whose gloo group only carries the control messages: id, barrier, timing max).
    --backend gloo: the same C++ orchestrator with its collectives over gloo on host buffers
    (sparkey_shard_comm_create_host), every rank on one GPU (a rehearsal).  --orchestrator python runs
    sparkey/sharded.py's ShardedBuilder over torch.distributed instead.  After the timed region
    (--check, on by default): rank 0 builds the whole log on one GPU and compares every rank's slice
    of the .spi with it, by per-block checksums."""
    import torch.distributed as dist
    import sparkey
    from sparkey import _native, synth, synth_device

    n_total = args.entries * world
    churn = args.workload == "churn"  # overwrites + DELETEs: the sharded exact path
    compressed = args.workload in ("snappy", "zstd")  # each rank decodes its own blocks
    full_log = None
    t0 = time.time()
    opts = _native.make_opts(hash_size=0, hash_seed=HASH_SEED, method=_native.METHOD_IN_MEMORY, device=dev.index)
    if churn:  # (every rank makes the whole log, then keeps its byte range)
        full_log = synth.churn_log(n_total, int(n_total * 0.8), 0.1, seed=args.seed + 4)
        file_len = int(full_log.size)
        header = full_log[:84].tobytes()
    elif compressed:  # (every rank makes the whole compressed log, then keeps its byte range)
        full_log = synth.snappy_log(synth.fixed_log(n_total, 16, 100, seed=args.seed, file_id=0x5EED0000), 118, 65536,
                                    codec=args.workload)
        file_len = int(full_log.size)
        header = full_log[:84].tobytes()
    else:
        file_len = 84 + n_total * 118
        header, _ = synth.fixed_log_range(n_total, 0, 84, 16, 100, seed=args.seed, file_id=0x5EED0000)
    lo, hi, out_off, out_len = _native.shard_geometry(header, file_len, opts, rank, world)
    if churn or compressed:
        buf = torch.from_numpy(full_log[lo:hi]).to(dev)
    else:  # the rank's byte range, generated in HBM
        _, buf = synth_device.fixed_log_range(n_total, lo, hi, 16, 100, seed=args.seed, file_id=0x5EED0000,
                                              device=dev)
    torch.cuda.synchronize(dev)
    gen_s = time.time() - t0
    # (the plan's workspace for twice the rank's records, so that no timed build grows it; the one-GPU
    #  rehearsal of N ranks reserves for the records alone -- N ranks of C4's 125M fit 288 GB only so)
    # (the one-GPU rehearsal reserves no per-byte framing workspace either: the uniform framing writes
    #  digit regions, and the warm-up build grows what a rank needs)
    plan_bytes = (118 * args.entries + 65536 * 4) if compressed else hi - lo
    plan = _native.Plan(dev.index, 0 if args.backend == "gloo" else plan_bytes,
                        (1 if args.backend == "gloo" else 2) * args.entries)
    stream = torch.cuda.Stream(dev)
    phases = {}
    shared_gpu = args.backend == "gloo"  # (the rehearsal: every rank on one GPU)
    if shared_gpu:
        _native.debug_set("frame_ticket", 1)  # builds share the device: framing regions by ticket
    if args.orchestrator == "python":
        from sparkey.sharded import Comm, GpuShardSteps, ShardedBuilder
        builder = ShardedBuilder(GpuShardSteps(dev, plan), Comm(device=dev))

        def one_build():
            r = builder.build(header, file_len, buf, lo, hi, opts)
            for k, v in r.phase_ms.items():
                phases[k] = phases.get(k, 0.0) + v
            return r.out, {"sharded": {"sharded": 1, "exact": 2, "gathered": 3}[r.path],
                           "num_entries": r.stats["num_entries"], "out_offset": r.out_offset}
    else:
        if shared_gpu:  # gloo on host buffers between the processes (sparkey_shard_comm_create_host)
            comm = _native.ShardComm(None, rank, world, dev.index)
        else:
            uid = [_native.shard_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            comm = _native.ShardComm(uid[0], rank, world, dev.index)
        d_out = torch.empty(max(16, out_len), dtype=torch.uint8, device=dev)

        def one_build():
            st = comm.build(plan, header, file_len, buf.data_ptr(), lo, hi, opts, d_out.data_ptr(), out_len,
                            stream.cuda_stream)
            for k, v in comm.phases():
                phases[k] = phases.get(k, 0.0) + v
            return d_out[:out_len], {"sharded": st.sharded, "num_entries": st.num_entries}

    for _ in range(args.warmup):
        out, info = one_build()
    phases.clear()
    dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        out, info = one_build()
    torch.cuda.synchronize(dev)
    dist.barrier()
    elapsed = time.perf_counter() - t_start
    free_b, total_b = torch.cuda.mem_get_info(dev)  # (device-wide: every rank of a one-GPU rehearsal)
    t = torch.tensor([elapsed, float(total_b - free_b)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t[0].item())
    device_used_gb = round(float(t[1].item()) / 1e9, 1)
    if churn:
        assert info["sharded"] == 2, info
    else:
        assert info["sharded"] == 1 and info["num_entries"] == n_total, info
    identical = None
    check_s = None
    one_gpu_ms = None
    if not args.no_check:  # every rank's slice against ONE single-GPU build of the whole log (rank 0)
        t_c = time.time()
        mine = (info.get("out_offset", out_off), int(out.numel()), block_sums(out))
        del out
        pieces = [None] * world
        dist.all_gather_object(pieces, mine)
        plan.close()
        if args.orchestrator == "cpp":  # (every rank's buffers go before rank 0's whole-log build)
            comm.close()
            del d_out
        torch.cuda.empty_cache()
        if shared_gpu or rank == 0:
            del buf
            torch.cuda.empty_cache()
        if rank == 0:
            if full_log is not None:
                d_full = torch.from_numpy(full_log).to(dev)
            else:
                d_full = synth_device.fixed_log(n_total, 16, 100, seed=args.seed, file_id=0x5EED0000, device=dev)
            size = _native.index_size(header, opts)
            d_spi = torch.empty(size, dtype=torch.uint8, device=dev)
            p1 = _native.Plan(dev.index)
            p1.build(header, d_full.data_ptr(), d_full.numel(), d_spi.data_ptr(), size, opts)  # (also the warm-up)
            # the same whole log built on ONE GPU, timed as the sharded builds are (host clock around
            # finished builds): the denominator of the N-GPU speed-up (IndexHash.java:131-167: one call,
            # one index)
            k1 = max(1, min(args.steps, 5))
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            for _ in range(k1):
                p1.build(header, d_full.data_ptr(), d_full.numel(), d_spi.data_ptr(), size, opts)
            torch.cuda.synchronize(dev)
            one_gpu_ms = (time.perf_counter() - t1) * 1000.0 / k1
            p1.close()
            del d_full
            bad = [r for r, (off, ln, sums) in enumerate(pieces) if block_sums(d_spi[off:off + ln]) != sums]
            covered = sorted((off, ln) for off, ln, _ in pieces)
            contiguous = covered[0][0] == 0 and all(a + la == b for (a, la), (b, _) in zip(covered, covered[1:])) \
                and covered[-1][0] + covered[-1][1] == size
            identical = not bad and contiguous
            if not identical:
                identical = {"identical": False, "ranks_differing": bad, "slices_cover_the_file": contiguous}
            del d_spi
            torch.cuda.empty_cache()
        check_s = round(time.time() - t_c, 1)
        dist.barrier()
    else:
        plan.close()
    if shared_gpu:
        _native.debug_set("frame_ticket", None)
    slot = 16
    from sparkey.sharded import parse_log_header
    cap = 1 | int(parse_log_header(header)["num_puts"] * 1.3)
    ms_per_step = elapsed * 1000.0 / args.steps
    b_alg_per_gpu = ((file_len - 84) + 112 + slot * cap) / world
    if compressed:  # + the decoded records written and read back by the framing
        b_alg_per_gpu += 2 * 118 * n_total / world
    achieved = b_alg_per_gpu / (ms_per_step * 1e-3) / 1e9
    c4 = n_total == 1_000_000_000 and not churn
    return {
        "value": n_total * args.steps / elapsed, "ms_per_step": ms_per_step,
        "config": {"workload": (f"churn: {args.entries} records per GPU x {world} GPUs = {n_total} (keys from a pool "
                                f"of 0.8 n, 10% DELETEs) in ONE index, sharded exact path" if churn else
                                ("C4: " if c4 else "") +
                                f"C2 shape, {args.entries} PUTs per GPU x {world} GPUs = {n_total} in ONE index "
                                f"(16 B key, 100 B value, {args.workload.upper() + ' 64 KiB blocks' if compressed else 'NONE'}"
                                ", IN_MEMORY)"),
                   "entries": n_total, "entries_per_gpu": args.entries, "log_bytes": file_len, "capacity": cap,
                   "spi_bytes": 112 + slot * cap,
                   "parallelism": f"log byte-range sharded x{world}, " +
                   ("gloo on host buffers, every rank on one GPU (rehearsal)" if shared_gpu else
                    "RCCL all_to_all of (hash, address) entries"),
                   "orchestrator": "C++ sparkey_shard_build (C-ABI)" if args.orchestrator == "cpp"
                   else "Python ShardedBuilder"},
        "roofline": {"bound": "hbm", "kernel": "whole sharded build per GPU", "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": pmc_traffic(f"sharded_rank_{args.entries}", "build"),
                     "algorithmic_bytes_per_launch": b_alg_per_gpu, "avg_launch_ms": ms_per_step},
        "phase_ms_rank0": {k: v / args.steps for k, v in phases.items()},
        "bit_identical_to_single_gpu": identical,
        # the same N x entries log built whole on one GPU (rank 0, after the timed region): what N GPUs
        # buy over one for ONE index (a strong-scaling reference; the driver's own scaling figure is
        # the weak-scaling curve of `value` over N)
        "one_gpu_same_log": None if one_gpu_ms is None else {
            "ms": one_gpu_ms, "keys_per_s": n_total / (one_gpu_ms * 1e-3),
            "speedup_n_gpus_over_one": one_gpu_ms / ms_per_step,
            "speedup_per_gpu": one_gpu_ms / ms_per_step / world,
            "note": ("ranks share one GPU (gloo rehearsal): the sharded time is not an N-GPU time"
                     if shared_gpu else "one GPU of this node, same log, same plan options")},
        "check_s": check_s,
        "device_used_gb_after_timed_builds": device_used_gb,
        "cpu_baseline": None,
        "gen_s": gen_s,
        "version": sparkey.version(),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--entries", type=int, default=None,
                    help="records (per GPU at N > 1); default 10M at N = 1 (C2), 125M per GPU at N > 1 (C4 at N = 8), "
                         "1B for --workload c4")
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS),
                    help="c2 (the headline metric); c3 / c5 / churn are extra single-GPU measurements")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--quick", action="store_true", help="timed device builds only (profiling runs)")
    ap.add_argument("--no-parity", action="store_true", help="skip the N = 1 parity leg (other device paths)")
    ap.add_argument("--parity-c3-entries", type=int, default=10_000_000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--backend", default="nccl", help="nccl (RCCL); gloo only to rehearse N > 1 ranks on one GPU")
    ap.add_argument("--sharded", action="store_true", help="the sharded build even at N = 1 (rehearsal)")
    ap.add_argument("--no-check", action="store_true",
                    help="sharded: skip comparing the .spi with a single-GPU build (done after the timed region)")
    ap.add_argument("--orchestrator", default="cpp", choices=["cpp", "python"],
                    help="sharded: the C-ABI's sparkey_shard_build (C++, the product) or sparkey/sharded.py over "
                         "torch.distributed (the test-only reference orchestrator; it gathers compressed logs)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.entries is None:
        args.entries = 1_000_000_000 if args.workload == "c4" else (125_000_000 if world > 1 else 10_000_000)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.backend == "gloo":
        local_rank = 0  # rehearsal: every rank on the one GPU
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1 or args.sharded:
        import torch.distributed as dist
        if args.backend == "nccl" and args.orchestrator == "python":
            dist.init_process_group("nccl", device_id=dev)
        elif world == 1 and "RANK" not in os.environ:  # (--sharded at N = 1 without a launcher: a local store,
            dist.init_process_group("gloo", store=dist.HashStore(), rank=0, world_size=1)  # so rocprofv3 can run it)
        else:  # (the C++ orchestrator moves the data over its own RCCL communicator)
            dist.init_process_group("gloo")
        r = sharded(args, dev, world, rank)
        dist.destroy_process_group()
    elif args.workload == "get":
        r = lookups(args, dev)
    elif args.workload == "append":
        r = appends(args, dev)
    elif args.workload == "c4":
        r = single_gpu_c4(args, dev)
    else:
        r = single_gpu(args, dev)
    if rank == 0:
        metric = r.pop("metric", METRIC)
        line = {"metric": metric, "value": r.pop("value"), "unit": r.pop("unit", "keys/s"), "n_gpus": world,
                "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": r.pop("ms_per_step"), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic"}
        line.update(r)
        print(json.dumps(line))


if __name__ == "__main__":
    main()
