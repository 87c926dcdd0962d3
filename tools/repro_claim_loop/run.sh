#!/bin/bash
# Compile the claim-loop reproducer (never run it) in three forms and check each listing:
# inlined body + __shfl broadcast (splits), out-of-line body, readfirstlane broadcast.
set -u
cd "$(dirname "$0")"
out=${1:-/tmp/repro_claim_loop}
mkdir -p "$out"
for v in "inline_shfl:" "noinline_shfl:-DBODY_ATTR=__noinline__" "inline_readfirstlane:-DBROADCAST(k)=__builtin_amdgcn_readfirstlane(k)"; do
  name=${v%%:*}; flags=${v#*:}
  (cd "$out" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 $flags -c "$OLDPWD/claim_loop.hip" \
     -o $name.o --save-temps > /dev/null 2>&1 && mv claim_loop-hip-amdgcn-amd-amdhsa-gfx950.s $name.s)
  printf '%-22s ' "$name"; python3 check_isa.py "$out/$name.s" | sed 's/^_Z10claim_loopPjjPKfPfj: //'
done
