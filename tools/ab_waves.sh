#!/bin/bash
# A/B of the register budget (waves per SIMD, the variant byte) of each workload's main kernel.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/ab_workload.py --workload cfg5 --rounds 2 2 3 4 > gpurun_out/ab_waves_cfg5.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/ab_workload.py --workload cfg4 --rounds 3 0 4 5 6 > gpurun_out/ab_waves_cfg4.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/ab_workload.py --workload cfg2 --rounds 3 0 3 4 5 > gpurun_out/ab_waves_cfg2.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/ab_workload.py --workload cfg3 --rounds 3 0 3 4 5 > gpurun_out/ab_waves_cfg3.log 2>&1 || exit $?
