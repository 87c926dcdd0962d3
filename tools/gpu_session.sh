#!/bin/bash
# One gpurun session: every GPU step under its own time limit; stop at the first fault /
# abort / timeout (exit codes 124, 134, 137, 139 or > 128).  Ordinary test failures (exit 1)
# do not stop the session.  Usage: tools/gpu_session.sh STEP...   (steps: test smoke bench prof pmc)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/session.log
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 )) s)" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $name: stopping" | tee -a gpurun_out/session.log; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    test)  run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python3 bench.py --steps 5 --warmup 2 ;;
    bench4) run bench4 600 python3 bench.py --workload cfg4 --steps 2 --warmup 1 ;;
    bench5) run bench5 900 python3 bench.py --workload cfg5 --steps 1 --warmup 1 ;;
    bench2) run bench2 600 python3 bench.py --workload cfg2 --steps 5 --warmup 2 ;;
    benchm3) run benchm3 900 python3 bench.py --workload m3 --steps 2 --warmup 1 ;;
    prof2) run prof2 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python3 bench.py --workload cfg2 --steps 5 --warmup 2 --no-cpu-baseline ;;
    profm3) run profm3 900 rocprofv3 --kernel-trace --stats -d gpurun_out/profm3 -o run --output-format csv -- python3 bench.py --workload m3 --steps 2 --warmup 1 --no-cpu-baseline ;;
    traffic) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 tools/ab_kernels.py --rounds 1 def:0:0
           run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python3 tools/ab_kernels.py --rounds 1 def:0:0
           run traffic 60 python3 tools/pmc_traffic.py ;;
    traffic_all)  # PMC FETCH/WRITE per launch of the default kernels on cfg3 / cfg4 / cfg5 -> profiles/r02_traffic*.json
           run pmc3_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc3_fetch -o run --output-format csv -- python3 tools/ab_kernels.py --rounds 1 def:0:0
           run pmc3_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc3_write -o run --output-format csv -- python3 tools/ab_kernels.py --rounds 1 def:0:0
           run traffic3 60 python3 tools/pmc_traffic.py --workload cfg3 --fetch gpurun_out/pmc3_fetch --write gpurun_out/pmc3_write --out gpurun_out/r02_traffic.json
           run pmc4_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc4_fetch -o run --output-format csv -- python3 tools/ab_workload.py --workload cfg4 --rounds 1 0
           run pmc4_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc4_write -o run --output-format csv -- python3 tools/ab_workload.py --workload cfg4 --rounds 1 0
           run traffic4 60 python3 tools/pmc_traffic.py --workload cfg4 --fetch gpurun_out/pmc4_fetch --write gpurun_out/pmc4_write --out gpurun_out/r02_traffic_cfg4.json
           run pmc5_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc5_fetch -o run --output-format csv -- python3 tools/ab_workload.py --workload cfg5 --rounds 1 0
           run pmc5_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc5_write -o run --output-format csv -- python3 tools/ab_workload.py --workload cfg5 --rounds 1 0
           run traffic5 60 python3 tools/pmc_traffic.py --workload cfg5 --fetch gpurun_out/pmc5_fetch --write gpurun_out/pmc5_write --out gpurun_out/r02_traffic_cfg5.json ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    pmc)   run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 tools/ab_kernels.py --rounds 1 ${AB_VARIANTS:-lean2:0:2 mega2:4:2}
           run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python3 tools/ab_kernels.py --rounds 1 ${AB_VARIANTS:-lean2:0:2 mega2:4:2}
           run pmc_valu 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_valu -o run --output-format csv -- python3 tools/ab_kernels.py --rounds 1 ${AB_VARIANTS:-lean2:0:2 mega2:4:2}
           run pmc_wait 600 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_wait -o run --output-format csv -- python3 tools/ab_kernels.py --rounds 1 ${AB_VARIANTS:-lean2:0:2 mega2:4:2}
           run pmc_mix 600 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 --kernel-trace -d gpurun_out/pmc_mix -o run --output-format csv -- python3 tools/ab_kernels.py --rounds 1 ${AB_VARIANTS:-lean2:0:2 mega2:4:2}
           run pmc_mix2 600 rocprofv3 --pmc SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 --kernel-trace -d gpurun_out/pmc_mix2 -o run --output-format csv -- python3 tools/ab_kernels.py --rounds 1 ${AB_VARIANTS:-lean2:0:2 mega2:4:2} ;;
    cache) run pmc_lat 600 rocprofv3 --pmc TCP_TCP_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace -d gpurun_out/pmc_lat -o run --output-format csv -- python3 tools/ab_kernels.py --rounds 1 ${AB_VARIANTS:-def:0:0}
           run pmc_l2 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/pmc_l2 -o run --output-format csv -- python3 tools/ab_kernels.py --rounds 1 ${AB_VARIANTS:-def:0:0}
           run pmc_wait 600 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS --kernel-trace -d gpurun_out/pmc_wait -o run --output-format csv -- python3 tools/ab_kernels.py --rounds 1 ${AB_VARIANTS:-def:0:0} ;;
    hang)  # diagnostic build with the watchdog (RRT_WATCHDOG_MS): the round-3 profile-build hang case
           run hang_b1 180 env RRT_LIB=tools/librrt_prof.so RRT_WATCHDOG_MS=20000 python3 tools/phase_profile.py --case bunny_B1_160x120_s16 --flags 2097152
           run hang_cfg3 180 env RRT_LIB=tools/librrt_prof.so RRT_WATCHDOG_MS=20000 python3 tools/phase_profile.py --case cfg3_bunny_1080p_s64 --flags 0 --region 0 0 1920 540 ;;
    hang_nowd)  # the same diagnostic build without the watchdog (round 3's exact command shape)
           run hang_b1_nowd 60 env RRT_LIB=tools/librrt_prof.so python3 tools/phase_profile.py --case bunny_B1_160x120_s16 --flags 2097152
           run hang_cfg3_nowd 60 env RRT_LIB=tools/librrt_prof.so python3 tools/phase_profile.py --case cfg3_bunny_1080p_s64 --flags 0 --region 0 0 1920 540
           run hang_cfg3_full 60 env RRT_LIB=tools/librrt_prof.so python3 tools/phase_profile.py --case cfg3_bunny_1080p_s64 --flags 2097152 ;;
    phase8all) # per-pixel time maps (gpurun_out/px_*.npz) of every rank's tile set of the 8-way cfg3 split
           for k in 0 1 2 3 4 5 6 7; do
             RRT_LIB=tools/librrt_prof.so run ph8_r$k 300 python3 tools/phase_profile.py --flags 0 --rank $k 8 || exit $?; done ;;
    abq)   # A/B of two builds (in-tree vs ab_var/librrt_$ABQ_VAR.so): cfg3 bit-exact + frame time, then the 8-way split
           run abq_exact 300 python3 tools/ab_kernels.py --rounds 3 def:0:0 &&
           run abq_exact_var 300 env RRT_LIB=ab_var/librrt_${ABQ_VAR}.so python3 tools/ab_kernels.py --rounds 3 def:0:0 &&
           bash tools/ab_libs.sh cfg3 2 base ${ABQ_VAR} &&
           run abq_w8 300 python3 tools/ab_workload.py --workload cfg3 --world 8 --rounds 3 0 &&
           run abq_w8_var 300 env RRT_LIB=ab_var/librrt_${ABQ_VAR}.so python3 tools/ab_workload.py --workload cfg3 --world 8 --rounds 3 0 ;;
    prof8) # kernel trace of every rank's tile set of the 8-way cfg3 split (batch vs heavy kernel per launch)
           run prof8 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o run --output-format csv -- python3 tools/ab_workload.py --workload cfg3 --world 8 --rounds 3 0 ;;
    kerr)  run pytest_kerr 600 python3 -u -m pytest tests/test_gpu_kerr.py -x -q -s --timeout 300 --timeout-method thread ;;
    cli)   run pytest_cli 600 python3 -u -m pytest tests/test_gpu_cli.py -x -q -s --timeout 300 --timeout-method thread ;;
    phase8) # phase profiles of the slowest and the fastest rank's tile sets of the 8-way cfg3 split
           RRT_LIB=tools/librrt_prof.so run ph8_r4 300 python3 tools/phase_profile.py --flags 0 --rank 4 8 &&
           RRT_LIB=tools/librrt_prof.so run ph8_r0 300 python3 tools/phase_profile.py --flags 0 --rank 0 8 ;;
    path)  # the path pool kernel (depth >= 2): its own parity tests, then every depth >= 2 golden in every variant
           run pytest_path 300 python3 -u -m pytest tests/test_gpu_path.py -x -v -s --timeout 120 --timeout-method thread &&
           run pytest_deep 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "m2 or m3 or m4" ;;
    pathprof) RRT_LIB=tools/librrt_prof.so run pathprof 300 python3 tools/path_profile.py --workload m3 ;;
    ab8)   run ab8 900 python3 tools/ab_workload.py --workload cfg3 --world 8 --rounds ${AB_ROUNDS:-3} ${AB_WVARIANTS:-0 4096} ;;
    abw)   run abw 900 python3 tools/ab_workload.py --workload ${AB_WORKLOAD:-cfg5} --rounds ${AB_ROUNDS:-2} ${AB_WVARIANTS:-0 0:2048} ;;
    prof5) run prof5 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python3 bench.py --workload cfg5 --steps 1 --warmup 1 --no-cpu-baseline ;;
    diag)  run diag 600 python3 tools/diag_clear.py --res 64 128 192 256 ;;
    ab)    run ab 900 python3 tools/ab_kernels.py --rounds ${AB_ROUNDS:-3} ${AB_VARIANTS:-lean1:0:1 lean2:0:2 lean3:0:3 lean4:0:4 mega2:4:2} ;;
    avail) run avail 120 rocprofv3 --list-avail ;;
    ubench) run ubench_f64 300 ./tools/ubench_f64 ;;
    cropfloor)  # the cfg3 lit streak alone on an idle GPU: the per-pixel latency floor of the frame's tail
           run crop_streak 300 python3 tools/crop_probe.py --region 960 600 24 16 --no-counters --flags 0 &&
           run crop_tiles 300 python3 tools/crop_probe.py --region 960 576 32 64 --no-counters --flags 0 ;;
    valu)  # PMC passes over the bench's launches (-> tools/pmc_valu.py): FP64 VALU mix, lane utilisation,
           # clock; HBM fetch / write.  One rocprofv3 run per pass.
           W=${PMC_WORKLOAD:-cfg3}; K=${PMC_KERNEL:-rrt_batch_kernel<1, 4>}
           run pmc_valu_$W 600 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmcv_$W -o run --output-format csv -- python3 bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline
           run pmc_fetch_$W 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf_$W -o run --output-format csv -- python3 bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline
           run pmc_write_$W 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw_$W -o run --output-format csv -- python3 bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline
           run pmc_json_$W 60 python3 tools/pmc_valu.py gpurun_out/pmcv_$W gpurun_out/pmcf_$W gpurun_out/pmcw_$W --workload $W --kernel "$K" --out gpurun_out/${RTAG:-r04}_${W}_pmc.json ;;
    cropw) # the streak crop at 2..5 waves/SIMD (register budget vs spills) and its phase profile
           run cropw 300 python3 tools/crop_probe.py --region 960 600 24 16 --no-counters --flags 0:2 0:3 0:4 0:5 &&
           RRT_LIB=tools/librrt_prof.so run crop_phase 300 python3 tools/phase_profile.py --region 960 600 24 16 --flags 0 ;;
    cropd) # the streak crop without walks (diagnostic flags; results are not the reference's) and its counters
           run cropd 300 python3 tools/crop_probe.py --region 960 600 24 16 --flags 0 1073741824 268435456 536870912 65536 ;;
    crop)  run crop 300 python3 tools/crop_probe.py --region 960 600 24 16 --no-counters --flags 0 262144 ;;
    parity) run pytest_parity 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kerr.py tests/test_gpu_cli.py -x -q --timeout 300 --timeout-method thread ;;
    abtree) run abtree3 600 python3 tools/ab_workload.py --workload cfg3 --rounds 3 0 0:262144 &&
            run abtree4 600 python3 tools/ab_workload.py --workload cfg4 --rounds 2 0 0:262144 &&
            run abtree5 900 python3 tools/ab_workload.py --workload cfg5 --rounds 1 0 0:262144 ;;
    heavy) # heavy-pixel slot path: parity (BASELINE frames + small cases), A/B on cfg3, per-pixel phase profile
           run pytest_heavy 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "baseline or noheavy or bunny_B or spheres_B" &&
           run abheavy 600 python3 tools/ab_workload.py --workload cfg3 --rounds 3 0 0:1048576 65536 196608 &&
           run profheavy 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profheavy -o run --output-format csv -- python3 tools/ab_workload.py --workload cfg3 --rounds 2 0 0:1048576 &&
           RRT_LIB=tools/librrt_prof.so run phase3h 300 python3 tools/phase_profile.py --flags 0 ;;
    profheavy) # per-kernel durations with and without the heavy path (cfg3)
           run profheavy 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profheavy -o run --output-format csv -- python3 tools/ab_workload.py --workload cfg3 --rounds 2 0 0:1048576 ;;
    phaseall) # phase profiles of cfg3 (frame + streak crop), cfg4 and cfg5 on the -DRRT_PROFILE=1 build (make prof)
           RRT_LIB=tools/librrt_prof.so run phase3 300 python3 tools/phase_profile.py --flags 0 &&
           RRT_LIB=tools/librrt_prof.so run phase_crop 300 python3 tools/phase_profile.py --region 960 600 24 16 --flags 0 &&
           RRT_LIB=tools/librrt_prof.so run phase4 300 python3 tools/phase_profile.py --workload cfg4 --flags 0 &&
           RRT_LIB=tools/librrt_prof.so run phase5 600 python3 tools/phase_profile.py --workload cfg5 --flags 0 ;;
    phase) RRT_LIB=tools/librrt_prof.so run phase3 300 python3 tools/phase_profile.py --flags 0 &&
           RRT_LIB=tools/librrt_prof.so run phase_crop 300 python3 tools/phase_profile.py --region 960 600 24 16 --flags 0 ;;
    abdeep) run abdeep 900 python3 tools/ab_workload.py --workload m3 --rounds 2 0 2 4 0:16 0:131072 ;;
    deeptests) run pytest_deep 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "m2 or m3 or m4" ;;
    pmcall) # PMC of every workload's main kernel on this build, copied into profiles/ for the bench lines
           for wk in "cfg3:rrt_batch_kernel<1, 4>" "cfg4:rrt_batch_kernel<2, 5>" "cfg2:rrt_batch_kernel<1, 4>" "m3:rrt_render_kernel<true, false, 0, ...>" "cfg5:rrt_batch_kernel<3, 3>"; do
             PMC_WORKLOAD=${wk%%:*} PMC_KERNEL=${wk#*:} bash tools/gpu_session.sh valu || exit $?
             cp gpurun_out/${RTAG:-r04}_${wk%%:*}_pmc.json profiles/ ; done ;;
    profall) run prof3 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline &&
             run prof4 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run --output-format csv -- python3 bench.py --workload cfg4 --steps 3 --warmup 1 --no-cpu-baseline &&
             run prof5 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python3 bench.py --workload cfg5 --steps 1 --warmup 1 --no-cpu-baseline &&
             run prof2 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python3 bench.py --workload cfg2 --steps 5 --warmup 2 --no-cpu-baseline &&
             run profm3 900 rocprofv3 --kernel-trace --stats -d gpurun_out/profm3 -o run --output-format csv -- python3 bench.py --workload m3 --steps 2 --warmup 1 --no-cpu-baseline ;;
    benchall) run bench 600 python3 bench.py --steps 5 --warmup 2 && run bench2 600 python3 bench.py --workload cfg2 --steps 5 --warmup 2 &&
              run bench4 600 python3 bench.py --workload cfg4 --steps 2 --warmup 1 && run bench5 900 python3 bench.py --workload cfg5 --steps 1 --warmup 1 &&
              run benchm3 900 python3 bench.py --workload m3 --steps 2 --warmup 1 ;;
    abfresh) # fresh-pixel continuations for the launch's last claims (cfg3 8-way), rounds 3
           run abfresh 600 python3 tools/ab_workload.py --workload cfg3 --world 8 --rounds 3 0 0:0:RRT_AB_CONT_FRESH=2048 0:0:RRT_AB_CONT_FRESH=8192 0:0:RRT_AB_CONT_FRESH=32768 ;;
    abdeal) # tile deals of the 8-way split: serpentine (lib), serpentine + row offset S (serS), lattice (latS)
           for wl in cfg5 cfg3 cfg4; do for sp in lib ser1 ser3 lat3; do
             run abdeal_${wl}_$sp 600 python3 tools/ab_workload.py --workload $wl --world 8 --rounds 2 --split $sp 0 || exit $?; done; done ;;
    abdeal2) # lattice deals (rank = (tx + S ty) % 8) against the serpentine, ranks in rotated order; cfg4 heavy blocks of 8 waves
           run abnw8 600 python3 tools/ab_workload.py --workload cfg4 --world 8 --rounds 3 --rotate --split lat3 0 0:0:RRT_AB_HEAVY_NW=8 0:0:RRT_AB_HEAVY_NW=2 || exit $?
           for wl in cfg4 cfg3 cfg5; do for sp in lib lat1 lat3 lat5; do
             [ $wl = cfg5 ] && [ $sp = lat1 ] && continue
             run abdeal2_${wl}_$sp 600 python3 tools/ab_workload.py --workload $wl --world 8 --rounds 3 --rotate --split $sp 0 || exit $?; done; done ;;
    phase5r) # cfg5 rank 0 (slowest) and rank 3 of the 8-way split on the profile build: slowest pixels, per-pixel times
           RRT_LIB=tools/librrt_prof.so run ph5_r0 300 python3 tools/phase_profile.py --workload cfg5 --flags 0 --rank 0 8 &&
           RRT_LIB=tools/librrt_prof.so run ph5_r3 300 python3 tools/phase_profile.py --workload cfg5 --flags 0 --rank 3 8 ;;
    kcont) # Kerr continuations: parity on cfg5's framing, then the 8-way split with / without them and 16-px tiles
           run pytest_kcont 900 python3 -u -m pytest tests/test_gpu_kerr.py -x -q -s --timeout 600 --timeout-method thread -k cfg5_framing &&
           run abk8 600 python3 tools/ab_workload.py --workload cfg5 --world 8 --rounds 2 --rotate 0 0:0:RRT_AB_CONT=0 &&
           run abk8t16 600 python3 tools/ab_workload.py --workload cfg5 --world 8 --rounds 2 --rotate --tile 16 0 0:0:RRT_AB_CONT=0 &&
           run ab38 600 python3 tools/ab_workload.py --workload cfg3 --world 8 --rounds 3 --rotate 0 &&
           run ab48 600 python3 tools/ab_workload.py --workload cfg4 --world 8 --rounds 3 --rotate 0 ;;
    phase4r) # cfg4 ranks 6 and 3 of the 8-way (lattice) split on the profile build
           RRT_LIB=tools/librrt_prof.so run ph4_r6 300 python3 tools/phase_profile.py --workload cfg4 --flags 0 --rank 6 8 &&
           RRT_LIB=tools/librrt_prof.so run ph4_r3 300 python3 tools/phase_profile.py --workload cfg4 --flags 0 --rank 3 8 ;;
    ab3)   # claim order (back part first), tail-priority threshold, 16 / 8-px tiles: 8-way splits and whole frames
           run ab3_c3 600 python3 tools/ab_workload.py --workload cfg3 --world 8 --rounds 3 --rotate 0 0:0:RRT_AB_BACK_FIRST=1 0:0:RRT_AB_PRIO_TICKS=10000 0:0:RRT_AB_PRIO_TICKS=25000 &&
           run ab3_c3t16 600 python3 tools/ab_workload.py --workload cfg3 --world 8 --rounds 3 --rotate --tile 16 0 0:0:RRT_AB_BACK_FIRST=1 &&
           run ab3_c4 600 python3 tools/ab_workload.py --workload cfg4 --world 8 --rounds 3 --rotate 0 0:0:RRT_AB_PRIO_TICKS=10000 0:0:RRT_AB_PRIO_TICKS=25000 &&
           run ab3_c4t16 600 python3 tools/ab_workload.py --workload cfg4 --world 8 --rounds 3 --rotate --tile 16 0 &&
           run ab3_c5t16 600 python3 tools/ab_workload.py --workload cfg5 --world 8 --rounds 2 --rotate --tile 16 0:0:RRT_AB_CONT=0 &&
           run ab3_c5t8 600 python3 tools/ab_workload.py --workload cfg5 --world 8 --rounds 2 --rotate --tile 8 0:0:RRT_AB_CONT=0 &&
           run ab3_w3 600 python3 tools/ab_workload.py --workload cfg3 --rounds 5 0 0:0:RRT_AB_PRIO_TICKS=25000 &&
           run ab3_w3t16 600 python3 tools/ab_workload.py --workload cfg3 --rounds 5 --tile 16 0 &&
           run ab3_w4 600 python3 tools/ab_workload.py --workload cfg4 --rounds 3 0 &&
           run ab3_w4t16 600 python3 tools/ab_workload.py --workload cfg4 --rounds 3 --tile 16 0 &&
           run ab3_w5 900 python3 tools/ab_workload.py --workload cfg5 --rounds 1 0 &&
           run ab3_w5t16 900 python3 tools/ab_workload.py --workload cfg5 --rounds 1 --tile 16 0 ;;
    w8all) # 8-way projections of the BASELINE configs on this build (every rank's tiles on one GPU, rotated order)
           run w8_cfg3 600 python3 tools/ab_workload.py --workload cfg3 --world 8 --rounds 3 --rotate 0 &&
           run w8_cfg4 600 python3 tools/ab_workload.py --workload cfg4 --world 8 --rounds 3 --rotate 0 &&
           run w8_cfg5 600 python3 tools/ab_workload.py --workload cfg5 --world 8 --rounds 2 --rotate 0 ;;
    abflags) # scheduler flag variants of the whole library (tools/build_variant.sh) against the in-tree build
           bash tools/ab_libs.sh cfg3 3 base sink sinktrk && bash tools/ab_libs.sh cfg4 2 base sink sinktrk &&
           bash tools/ab_libs.sh cfg5 1 base sink sinktrk && bash tools/ab_libs.sh m3 1 base sink sinktrk &&
           bash tools/ab_libs.sh cfg2 2 base sink sinktrk ;;
    final) # the round's final evidence: GPU suite, smoke, every bench line, kernel stats, PMC, 8-way projections
           RTAG=${RTAG:-r06} bash tools/gpu_session.sh test smoke benchall w8all profall || exit $? ;;
    abwaves6) # waves/SIMD budgets of the batch kernels on the sink build (variant = waves), whole frames
           run abw6_c3 600 python3 tools/ab_workload.py --workload cfg3 --rounds 4 0 3 5 &&
           run abw6_c4 600 python3 tools/ab_workload.py --workload cfg4 --rounds 3 0 4 &&
           run abw6_c2 600 python3 tools/ab_workload.py --workload cfg2 --rounds 3 0 3 5 &&
           run abw6_c5 900 python3 tools/ab_workload.py --workload cfg5 --rounds 1 0 2 4 ;;
    abflags2) # more build flags on top of the sink build: no loop unrolling, size-mode live-range splitting
           bash tools/ab_libs.sh cfg3 3 base nounroll ssize && bash tools/ab_libs.sh cfg4 2 base nounroll ssize &&
           bash tools/ab_libs.sh cfg2 2 base nounroll ssize && bash tools/ab_libs.sh cfg5 1 base nounroll ssize &&
           bash tools/ab_libs.sh m3 1 base nounroll ssize ;;
    w24all) # 2- and 4-way projections of the BASELINE configs (every rank's tiles on one GPU, rotated order)
           for n in 2 4; do
             run w${n}_cfg3 600 python3 tools/ab_workload.py --workload cfg3 --world $n --rounds 3 --rotate 0 || exit $?
             run w${n}_cfg4 600 python3 tools/ab_workload.py --workload cfg4 --world $n --rounds 3 --rotate 0 || exit $?
             run w${n}_cfg5 900 python3 tools/ab_workload.py --workload cfg5 --world $n --rounds 1 --rotate 0 || exit $?; done ;;
    abknobs4) # the continuation / heavy-kernel run-time knobs on the lattice deal (cfg4 8-way): room, samples left,
           # heavy waves 3x CU (variant bits 28..31), heavy kernel at 5 waves/SIMD (bits 24..27)
           run abknobs4 600 python3 tools/ab_workload.py --workload cfg4 --world 8 --rounds 3 --rotate 0 0:0:RRT_AB_CONT_ROOM=64 0:0:RRT_AB_CONT_MIN=32 805306368 83886080 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
