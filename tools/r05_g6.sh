set -o pipefail
O=gpurun_out/r05g6; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/pytest_parity.log 2>&1 || { tail -40 $O/pytest_parity.log; exit 1; }
tail -2 $O/pytest_parity.log
ABDEBUG=frame_debug ROUNDS=2 bash tools/r05_ab.sh r05g6/ab "--workload c3 --entries 10000000 --steps 5 --warmup 1" r04 new1 new3 new3:frame3_persist=0
ROUNDS=1 bash tools/r05_ab.sh r05g6/ab100 "--workload c3 --entries 100000000 --steps 5 --warmup 1" r04 new3 new3:frame3_persist=0
