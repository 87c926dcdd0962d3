#!/bin/bash
# A/B of the batch kernel's tail-priority threshold (RRT_AB_PRIO_TICKS, wall-clock ticks at 100 MHz)
# on cfg3: the 8-way split (slowest rank) and the whole frame.  Each run under its own time limit.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for t in ${PRIO_LIST:-50000 12500 5000 1000}; do
  echo "=== prio $t" | tee -a gpurun_out/ab_prio.log
  RRT_AB_PRIO_TICKS=$t timeout -k 10 200 python3 tools/ab_workload.py --workload cfg3 --world 8 --rounds 3 0 >> gpurun_out/ab_prio.log 2>&1 || exit $?
  RRT_AB_PRIO_TICKS=$t timeout -k 10 200 python3 tools/ab_workload.py --workload cfg3 --rounds 3 0 >> gpurun_out/ab_prio.log 2>&1 || exit $?
done
