#!/usr/bin/env python3
"""TEST INFRASTRUCTURE: the C restatement's speed relative to the compiled reference renderer on
the same cores and the same sample (SURVEY 8(d) CPU-baseline plan).  Runs in the build container
only (needs oracle/_ref/ref_render, built from /root/reference by oracle/ref/Makefile); writes
profiles/r03_cpu_ratio.json, which bench.py attaches to its cpu_baseline on the GPU box (where the
reference does not travel).

Sample per workload: a band of full-width rows through the frame centre (-p cell mode of the
reference, y in sampleBuffer coordinates), rendered by
  * the reference: `ref_render -t N ... -p 0 y0 W rows` minus its own scene-load time (-Q run);
  * the restatement: oracle_lib.render over the same region, N pthreads.
Both use the keyed RNG, so they do the same work; their outputs are compared bit for bit.
Usage: python3 tools/cpu_ratio.py [--threads 8] [--workloads cfg3 cfg2 cfg4]"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "relativistic-ray-tracer_amd"))
import oracle_lib as O  # noqa: E402
import rrt_scenes  # noqa: E402

BIN = os.path.join(ROOT, "oracle", "_ref", "ref_render")
DAE = "/root/reference/pathtracer/dae/sky"
# workload -> (dae, frame w, h, spp, -B args or None, rows in the band)
WL = {
    "cfg3": ("CBbunny.dae", 1920, 1080, 64, None, 48),
    "cfg2": ("CBspheres_lambertian.dae", 1920, 1080, 64, ["0", "1", "0", "0", "0.1"], 24),
    "cfg4": ("@cfg4", 3840, 2160, 256, None, 8),
}


def ref_time(cmd, cwd):
    t0 = time.perf_counter()
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, cwd=cwd)
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--workloads", nargs="*", default=list(WL))
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_cpu_ratio.json"))
    a = ap.parse_args()
    out = json.load(open(a.out)) if os.path.exists(a.out) else {}
    for name in a.workloads:
        dae, W, H, spp, bh, rows = WL[name]
        with tempfile.TemporaryDirectory() as td:
            if dae.startswith("@"):
                path = os.path.join(td, "scene.dae")
                rrt_scenes.write_cfg4_dae(path)
            else:
                path = os.path.join(DAE, dae)
            y0 = H // 2 - rows // 2
            base = [BIN, "-t", str(a.threads), "-S", "0", "-O", os.path.join(td, "ref"), "-s", str(spp),
                    "-r", str(W), str(H)] + (["-B"] + bh if bh else [])
            t_load = min(ref_time(base + ["-Q", path], td) for _ in range(2))
            t_ref = ref_time(base + ["-f", os.path.join(td, "o.png"), "-p", "0", str(y0), str(W), str(rows), path], td)
            rrgb = np.load(os.path.join(td, "ref_px_rgb.npy"))
            rcnt = np.load(os.path.join(td, "ref_px_count.npy"))
            s = O.Scene(os.path.join(td, "ref.rrts"))
            cam = O.load_camera(os.path.join(td, "ref.rrtc"))
            c = (0.0, 1.0, 0.0, 0.1, 0.1) if not bh else tuple(float(v) for v in bh)
            p = O.make_params(W, H, ns_aa=spp, bh=c)
            t0 = time.perf_counter()
            rgb, cnt, _, _ = O.render(s, cam, p, 0, y0, W, rows, threads=a.threads)
            t_res = time.perf_counter() - t0
            same = bool(np.array_equal(rgb.view(np.uint32), rrgb.view(np.uint32)) and np.array_equal(cnt, rcnt))
        samples = int(cnt.astype(np.int64).sum())
        t_render = t_ref - t_load
        out[name] = {"speed_ratio": t_render / t_res, "reference_s": t_render, "reference_load_s": t_load,
                     "restatement_s": t_res, "samples": samples, "threads": a.threads, "bit_identical": same,
                     "reference_msamples_per_s": samples / t_render / 1e6,
                     "restatement_msamples_per_s": samples / t_res / 1e6,
                     "sample": f"rows {y0}..{y0 + rows - 1} (sampleBuffer y) of the {W}x{H} frame, {spp} spp",
                     "where": f"build container, {a.threads} threads, {O_cpu()}"}
        print(name, json.dumps(out[name]), flush=True)
        assert same, f"{name}: restatement differs from the reference on the sample"
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


def O_cpu():
    with open("/proc/cpuinfo") as f:
        for line in f:
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    return "?"


if __name__ == "__main__":
    main()
