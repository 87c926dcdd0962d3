#!/bin/bash
# A/B: straddle routing (ab_var/librrt_straddle.so) vs the in-tree build on the 8-way cfg3 split
set -u
mkdir -p gpurun_out
for p in 1 2; do
  timeout -k 10 300 python3 tools/ab_workload.py --workload cfg3 --world 8 --rounds 3 0 > gpurun_out/st_base_$p.log 2>&1 || exit $?
  echo "base $p $(tail -1 gpurun_out/st_base_$p.log)"
  RRT_LIB=ab_var/librrt_straddle.so timeout -k 10 300 python3 tools/ab_workload.py --workload cfg3 --world 8 --rounds 3 0 > gpurun_out/st_var_$p.log 2>&1 || exit $?
  echo "straddle $p $(tail -1 gpurun_out/st_var_$p.log)"
done
