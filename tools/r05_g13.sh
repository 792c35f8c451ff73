set -o pipefail
O=gpurun_out/r05g13; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_compressed.py tests/test_gpu_zstd.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
ROUNDS=2 bash tools/r05_ab.sh r05g13/c3 "--workload c3 --entries 10000000 --steps 5 --warmup 1" new7 new8
ROUNDS=2 bash tools/r05_ab.sh r05g13/c2 "--workload c2 --steps 10 --warmup 2" new7 new8 new7:no_uniform new8:no_uniform
ROUNDS=1 bash tools/r05_ab.sh r05g13/c1x "--workload c1x --steps 10 --warmup 2" new7 new8
