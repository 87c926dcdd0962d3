#!/bin/bash
# round-5 final call: the straddle A/B, then the PMC passes and the kernel profiles / bench lines
set -u
bash tools/_gpu_cmd_st.sh || exit $?
RTAG=r05 tools/gpu_session.sh pmcall || exit $?
cp gpurun_out/r05_*_pmc.json profiles/ && tools/gpu_session.sh profall benchall
