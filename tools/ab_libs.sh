#!/bin/bash
# A/B of librrt builds (tools/build_variant.sh) on a bench workload: one process per build and
# pass, interleaved; stops at the first fault / timeout.  Usage: tools/ab_libs.sh WORKLOAD PASSES NAME...
# (NAME "base" = the in-tree build)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
WL=$1; PASSES=$2; shift 2
for p in $(seq 1 "$PASSES"); do
  for name in "$@"; do
    lib=relativistic-ray-tracer_amd/librrt.so
    [ "$name" != base ] && lib=ab_var/librrt_$name.so
    RRT_LIB=$lib timeout -k 10 300 python3 tools/ab_workload.py --workload "$WL" --rounds 3 0 > gpurun_out/ab_${WL}_${name}_$p.log 2>&1
    rc=$?
    echo "$WL $name pass $p rc=$rc $(tail -1 gpurun_out/ab_${WL}_${name}_$p.log)" | tee -a gpurun_out/ab_libs.log
    if [ $rc -ge 124 ]; then exit $rc; fi
  done
done
