#!/usr/bin/env python3
"""FP64 VALU roofline inputs per launch of the render's main kernel from rocprofv3 PMC passes
(tools/gpu_session.sh `valu`): FP64 instruction mix, VALU lane utilisation, VALU busy share and
the effective clock, plus HBM FETCH/WRITE and the scratch split when those passes are given.
Writes the JSON bench.py reads (profiles/r03_<workload>_pmc.json, profiles/r03_traffic_<wl>.json).

Counter meanings (rocprofv3, gfx950): SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F64 count wave-level
instructions; SQ_ACTIVE_INST_VALU counts quad-cycles a wave spends issuing VALU work and
SQ_THREAD_CYCLES_VALU the same weighted by active lanes, so their ratio / 64 is the lane
utilisation; SQ_BUSY_CYCLES and GRBM_GUI_ACTIVE are summed over the 8 XCDs (effective clock =
GRBM_GUI_ACTIVE / 8 / kernel time, MI355X_MICROARCH.md 'DVFS give-back')."""
import argparse
import csv
import sys
import glob
import json
import os


def per_dispatch(dirs, match):
    """{counter: mean over dispatches of the kernels whose name contains `match`} + durations.
    A name librrt abbreviates ("rrt_render_kernel<true, false, 0, ...>") matches by its prefix."""
    if match.endswith("...>"):
        match = match[:-4]
    vals, durs = {}, {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if match not in k:
                    continue
                did = (f, int(r["Dispatch_Id"]))
                vals.setdefault(r["Counter_Name"], {}).setdefault(did, 0.0)
                vals[r["Counter_Name"]][did] += float(r["Counter_Value"])
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if match in r["Kernel_Name"]:
                    durs[(f, int(r["Dispatch_Id"]))] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    mean = {c: sum(v.values()) / len(v) for c, v in vals.items()}
    n = {c: len(v) for c, v in vals.items()}
    dur = sum(durs.values()) / len(durs) if durs else None
    return mean, n, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+", help="rocprofv3 -d output directories (one per PMC pass)")
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--kernel", required=True, help="main kernel name as librrt reports it, e.g. 'rrt_batch_kernel<1, 5>'")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    m, n, dur = per_dispatch(a.dirs, a.kernel)
    if not m:
        raise SystemExit(f"no dispatch of {a.kernel} in {a.dirs}")
    g = m.get
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "relativistic-ray-tracer_amd"))
    import rrt
    out = {"workload": a.workload, "main_kernel": a.kernel, "kernel": a.kernel, "build_id": rrt.build_id(), "counters": m,
           "dispatches": n, "kernel_s_under_profiler": dur}
    if g("SQ_INSTS_VALU_FMA_F64") is not None:
        fma, add, mul = g("SQ_INSTS_VALU_FMA_F64", 0.0), g("SQ_INSTS_VALU_ADD_F64", 0.0), g("SQ_INSTS_VALU_MUL_F64", 0.0)
        trans = g("SQ_INSTS_VALU_TRANS_F64", 0.0)
        util = g("SQ_THREAD_CYCLES_VALU") / (64.0 * g("SQ_ACTIVE_INST_VALU")) if g("SQ_ACTIVE_INST_VALU") else None
        insts = fma + add + mul + trans
        out.update({
            "fp64_wave_insts_per_launch": insts,
            "valu_lane_util": util,
            # lane-level FP64 flops: an FMA is 2, add / mul / transcendental 1, over the active lanes
            "fp64_flops_per_launch": (2.0 * fma + add + mul + trans) * 64.0 * (util or 1.0),
            "fp64_share_of_valu": insts / g("SQ_INSTS_VALU") if g("SQ_INSTS_VALU") else None,
        })
    if g("GRBM_GUI_ACTIVE") and dur:
        out["clock_hz"] = g("GRBM_GUI_ACTIVE") / 8.0 / dur
    if g("SQ_ACTIVE_INST_VALU") and g("GRBM_GUI_ACTIVE") and dur:
        # VALU issue quad-cycles over every SIMD's cycles (1024 SIMDs), a share of issue capacity
        out["valu_busy_frac"] = 4.0 * g("SQ_ACTIVE_INST_VALU") / (1024.0 * g("GRBM_GUI_ACTIVE") / 8.0)
    if g("FETCH_SIZE") is not None or g("WRITE_SIZE") is not None:
        fetch = 2.0 * g("FETCH_SIZE", 0.0) * 1024  # gfx950: FETCH_SIZE reports half of wide reads
        write = g("WRITE_SIZE", 0.0) * 1024
        out["hbm_bytes"] = fetch + write
        out["fetch_bytes"], out["write_bytes"] = fetch, write
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "counters"}))


if __name__ == "__main__":
    main()
