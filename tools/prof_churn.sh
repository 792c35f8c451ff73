set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/pc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 -k "exact or deletes or overwrite or interleaved or smoke" > gpurun_out/pc/t.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pc/trace -o run -- python3 bench.py --workload churn --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pc/trace.log 2>&1
