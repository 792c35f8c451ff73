bash tools/r05_stops.sh r05g7/np "frame3_persist=0" - 0 1 2 3 4 5 && bash tools/r05_stops.sh r05g7/nb "frame3_persist=0,no_buckets" - 5
