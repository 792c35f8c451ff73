#!/bin/bash
# k_frame3's throughput cost by phase: rocprofv3 kernel trace of C3 10M with the kernel stopped after
# phase k (frame3_stop=k; the host then reframes with k_frame, whose time is not counted here).
# usage: r05_stops.sh TAG "extra switches" stops...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1; X=$2; shift 2
O=gpurun_out/$T; mkdir -p $O
for k in "$@"; do
  sw="frame3_stop=$k"; [ "$k" = "-" ] && sw=""
  [ -n "$X" ] && sw="${sw:+$sw,}$X"
  SPARKEY_DEBUG=$sw timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s$k -o run -- \
    python3 bench.py --workload c3 --entries 10000000 --steps 5 --warmup 1 --quick --no-parity --no-cpu-baseline \
    > $O/s$k.log 2>&1 || exit 1
  f=$(find $O/s$k -name '*kernel_stats.csv' | head -1)
  python3 -c "import csv,sys; r=[x for x in csv.DictReader(open(sys.argv[1])) if 'k_frame3' in x['Name']]; print('stop=' + sys.argv[2], sys.argv[3], [(x['Calls'], round(float(x['AverageNs'])/1e3, 1)) for x in r])" $f "$k" "[$X]" >> $O/stops.txt || exit 1
done
cat $O/stops.txt
