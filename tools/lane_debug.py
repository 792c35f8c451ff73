"""k_frame_lane diagnostics on the GPU: the lane-geometry test's logs with small regions, per-pass
counts of unflagged regions (SPARKEY_LANE_DEBUG) and the framing path taken."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("sparkey-java_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
from helpers import make_log, random_puts  # noqa: E402
from sparkey import _native  # noqa: E402
import oracle  # noqa: E402

os.environ["SPARKEY_LANE_DEBUG"] = "1"
os.environ["SPARKEY_FRAME_DEBUG"] = "1"
for region in sys.argv[1:] or ["256", "512"]:
    os.environ["SPARKEY_LANE_REGION"] = region
    for seed, (kmin, kmax, vmin, vmax), hs in [(81, (8, 64, 100, 100), 8), (83, (1, 40, 20, 60), 4),
                                               (87, (10, 100, 0, 60), 8), (89, (0, 126, 0, 127), 8)]:
        log = make_log(random_puts(20000, seed=seed, kmin=kmin, kmax=kmax, vmin=vmin, vmax=vmax))
        print(f"== region {region} seed {seed}", file=sys.stderr, flush=True)
        got, st = _native.build_index_mem(log, _native.make_opts(hash_size=hs, hash_seed=seed))
        ok = got == oracle.build_index(log, seed, hash_size=hs)
        print(f"region {region} seed {seed}: framing {st.framing_path} oracle {'ok' if ok else 'DIFF'}",
              file=sys.stderr, flush=True)
