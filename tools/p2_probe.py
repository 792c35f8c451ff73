"""One C2 build (10M records) through the device plan, for cost attribution with the debug knobs
(SPARKEY_PART2_DEBUG, SPARKEY_PLACE_DEBUG): prints the stage times of the last of three builds."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparkey-java_amd"))


def main():
    import torch
    from sparkey import _native, synth
    n = 10_000_000
    log = synth.fixed_log(n, 16, 100, seed=1, file_id=0x5EED0000)
    dev = torch.device("cuda", 0)
    d_log = torch.from_numpy(log).to(dev)
    opts = _native.make_opts(hash_seed=0x2545F491, device=0)
    size = _native.index_size(log[:84].tobytes(), opts)
    d_out = torch.empty(size, dtype=torch.uint8, device=dev)
    plan = _native.Plan(0, log.size, n)
    plan.set_profiling(True)
    for _ in range(3):
        plan.build(log[:84].tobytes(), d_log.data_ptr(), log.size, d_out.data_ptr(), size, opts)
    print("stages", {k: round(v, 4) for k, v in plan.stage_times()}, flush=True)
    plan.close()


if __name__ == "__main__":
    main()
