set -o pipefail
O=gpurun_out/r05g18; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_compressed.py tests/test_gpu_zstd.py tests/test_file_build.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
ROUNDS=3 bash tools/r05_ab.sh r05g18/c2 "--workload c2 --steps 20 --warmup 3" new10 new11
