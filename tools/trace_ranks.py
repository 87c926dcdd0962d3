#!/usr/bin/env python3
"""Per-launch timeline from a rocprofv3 kernel trace of tools/ab_workload.py --world N: for each
render launch (rrt_pixel_proof_kernel, then rrt_heavy_kernel on the side stream beside
rrt_batch_kernel), the pass, batch and heavy kernels' durations and which one ends the launch.
Usage: python3 tools/trace_ranks.py gpurun_out/prof8/run_kernel_trace.csv [--world 8]"""
import argparse
import csv
import json

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--world", type=int, default=8)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    ks.sort()
    launches, cur = [], None
    for s, e, n in ks:
        if "rrt_pixel_proof_kernel" in n:
            cur = {"pass": (s, e)}
            launches.append(cur)
        elif cur is not None and "rrt_heavy_kernel" in n:
            cur["heavy"] = (s, e)
        elif cur is not None and "rrt_batch_kernel" in n:
            cur["batch"] = (s, e)
    out = []
    for i, L in enumerate(launches):
        if "batch" not in L:
            continue
        p0 = L["pass"][0]
        end = max(L["batch"][1], L.get("heavy", (0, 0))[1])
        rec = {"launch": i, "rank": i % a.world, "span_ms": (end - p0) / 1e6,
               "pass_ms": (L["pass"][1] - L["pass"][0]) / 1e6,
               "batch_start_ms": (L["batch"][0] - p0) / 1e6, "batch_ms": (L["batch"][1] - L["batch"][0]) / 1e6}
        if "heavy" in L:
            rec.update(heavy_start_ms=(L["heavy"][0] - p0) / 1e6, heavy_ms=(L["heavy"][1] - L["heavy"][0]) / 1e6,
                       ended_by="heavy" if L["heavy"][1] > L["batch"][1] else "batch")
        out.append(rec)
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in rec.items()}))
    if out:
        spans = np.array([r["span_ms"] for r in out])
        print(json.dumps({"launches": len(out), "span_ms_median": float(np.median(spans)),
                          "ended_by_heavy": sum(r.get("ended_by") == "heavy" for r in out)}))


if __name__ == "__main__":
    main()
