set -o pipefail
O=gpurun_out/r05g10; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/pytest_parity.log 2>&1 || { tail -40 $O/pytest_parity.log; exit 1; }
tail -2 $O/pytest_parity.log
ROUNDS=2 bash tools/r05_ab.sh r05g10/c3 "--workload c3 --entries 10000000 --steps 5 --warmup 1" new1 new6 new6:frame3_c=2048
ROUNDS=2 bash tools/r05_ab.sh r05g10/c2g "--workload c2 --steps 5 --warmup 1" new6:no_uniform new6:no_uniform,frame3_c=1024 new6:no_uniform,frame3_c=2048
