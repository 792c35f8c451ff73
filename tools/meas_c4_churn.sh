O=gpurun_out/r06f2; mkdir -p $O; export TMPDIR=/tmp
( while sleep 50; do echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4.jsonl 2> $O/c4.err \
 && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4trace -o run -- python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $O/c4trace.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/churntrace -o run -- python3 bench.py --workload churn --steps 5 --warmup 1 --no-cpu-baseline > $O/churntrace.log 2>&1 \
 && timeout -k 10 300 python -u bench.py --workload churn --steps 10 --warmup 2 --no-cpu-baseline > $O/churn.jsonl 2> $O/churn.err && echo all done
