"""Sharded C2-shape builds at growing sizes against the single-GPU build, on one GPU: the C++
orchestrator (sparkey_build_index_mem, num_gpus = N as threads, threads-one-device transport) and the
Python orchestrator (tests/sharded_harness.run_threads).  Prints the first differing slot on a
mismatch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("sparkey-java_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))


def first_diff(a, b):
    n = min(len(a), len(b))
    for i in range(0, n, 1 << 16):
        if a[i:i + (1 << 16)] != b[i:i + (1 << 16)]:
            for j in range(i, min(n, i + (1 << 16))):
                if a[j] != b[j]:
                    return j
    return -1 if len(a) == len(b) else n


def main():
    from sparkey import _native, synth
    import sharded_harness
    os.environ["SPARKEY_SHARD_TRANSPORT"] = "threads-one-device"
    for n in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "300000,3000000,6000000").split(",")]:
        log = synth.fixed_log(n, 16, 100, seed=1, file_id=0x5EED0000).tobytes()
        seed = 0x2545F491
        single, _ = _native.build_index_mem(log, _native.make_opts(hash_seed=seed, device=0))
        for world in (2, 4):
            got, st = _native.build_index_mem(log, _native.make_opts(hash_seed=seed, device=0, num_gpus=world))
            d = first_diff(got, single)
            print(f"n={n} cpp world={world}: {'identical' if d < 0 else f'DIFFERS at byte {d} (slot {(d - 112) // 16})'}",
                  flush=True)
            spi, metas = sharded_harness.run_threads(log, world, dict(hash_seed=seed, device=0))
            d = first_diff(spi, single)
            print(f"n={n} python world={world}: {'identical' if d < 0 else f'DIFFERS at byte {d} (slot {(d - 112) // 16})'}"
                  f" {[m['path'] for m in metas]}", flush=True)


if __name__ == "__main__":
    main()
