ROUNDS=2 bash tools/r05_ab.sh r05g14/c3 "--workload c3 --entries 10000000 --steps 5 --warmup 1" new8 new8:frame_look=16 new8:frame_look=64 new8:frame_region=6144 new8:frame_region=10240
