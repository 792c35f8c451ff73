set -o pipefail
O=gpurun_out/r05g16; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 bench.py --steps 20 --warmup 3 --quick --no-parity --no-cpu-baseline > $O/c2.log 2>&1 || exit 1
python3 tools/gap_trace.py $(find $O/c2 -name '*kernel_trace.csv' | head -1) k_build_init
ROUNDS=1 bash tools/r05_ab.sh r05g16/c1x "--workload c1x --steps 10 --warmup 2" new8 new10
