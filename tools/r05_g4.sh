bash tools/r05_sq.sh r05g4/new1 k_frame3 "--workload c3 --entries 10000000" && bash tools/r05_sq.sh r05g4/r04 k_frame3 "--workload c3 --entries 10000000" r04
