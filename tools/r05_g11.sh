set -o pipefail
O=gpurun_out/r05g11; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_large.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u bench.py --workload c3 --entries 100000000 --steps 10 --warmup 2 --no-cpu-baseline > $O/c3_100m.jsonl 2> $O/c3_100m.err || { tail -5 $O/c3_100m.err; exit 1; }
tail -1 $O/c3_100m.jsonl | cut -c1-600
timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 > $O/c2.jsonl 2> $O/c2.err || { tail -5 $O/c2.err; exit 1; }
tail -1 $O/c2.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('stage_ms'), d.get('general_framing'))"
