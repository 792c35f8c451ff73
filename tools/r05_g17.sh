ROUNDS=2 bash tools/r05_ab.sh r05g17/c3 "--workload c3 --entries 10000000 --steps 5 --warmup 1" new10 new10:frame3_cover=1 new10:frame3_cover=1,frame3_short=2 new10:frame3_short=2
