#!/usr/bin/env python3
"""HBM traffic per launch of the render kernel from rocprofv3 PMC passes (gpu_session.sh `pmc`):
FETCH_SIZE and WRITE_SIZE (kilobytes) of the matching dispatches, with the gfx950 correction of
MI355X_MICROARCH.md (FETCH_SIZE reports half the bytes of wide reads: doubled; WRITE_SIZE as is).
Writes the JSON bench.py --traffic reads."""
import argparse
import csv
import json
import os


def kernel_values(d, counter):
    f = os.path.join(d, "run_counter_collection.csv")
    vals = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if k.startswith("void "):
            k = k[len("void "):]
        if r["Counter_Name"] != counter or not k.startswith("rrt_"):
            continue
        if not any(s in k for s in ("batch", "first", "pixel_proof", "sample", "render_kernel", "mega")):
            continue
        name = k.split("(")[0]
        did = int(r["Dispatch_Id"])
        vals.setdefault(name, {}).setdefault(did, 0.0)
        vals[name][did] += float(r["Counter_Value"])
    return {n: sum(v.values()) / len(v) for n, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", default="gpurun_out/pmc_fetch")
    ap.add_argument("--write", default="gpurun_out/pmc_write")
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--out", default="gpurun_out/traffic.json")
    a = ap.parse_args()
    fetch, write = kernel_values(a.fetch, "FETCH_SIZE"), kernel_values(a.write, "WRITE_SIZE")
    if not fetch:
        raise SystemExit("no render-kernel dispatch in the PMC output")
    # one render launch = the pre-pass (pixel miss proof or sample 0, if any) + the main kernel
    names = sorted(fetch, key=lambda n: (0 if n.startswith(("rrt_first", "rrt_pixel_proof")) else 1, n))
    fkb = sum(fetch[n] for n in names)
    wkb = sum(write.get(n, 0.0) for n in names)
    out = {"workload": a.workload, "kernel": " + ".join(names), "fetch_size_kb": fkb, "write_size_kb": wkb,
           "per_kernel": {n: {"fetch_size_kb": fetch[n], "write_size_kb": write.get(n, 0.0)} for n in names},
           "hbm_bytes_per_launch": 2.0 * fkb * 1024 + wkb * 1024,
           "note": "FETCH_SIZE x 2 (gfx950 wide-read correction) + WRITE_SIZE, KB -> bytes, mean over dispatches"}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
