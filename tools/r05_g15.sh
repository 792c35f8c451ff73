set -o pipefail
O=gpurun_out/r05g15; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_sharded_gpu.py tests/test_multi_gpu_abi.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
ROUNDS=2 bash tools/r05_ab.sh r05g15/c1x "--workload c1x --steps 10 --warmup 2" new8 new9
ROUNDS=1 bash tools/r05_ab.sh r05g15/c3k "--workload c3 --entries 10000000 --steps 5 --warmup 1" new8:no_frame3 new9:no_frame3
