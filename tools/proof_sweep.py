#!/usr/bin/env python3
"""Soundness sweep of the camera / pixel / shadow proofs over random black holes, cameras and
resolutions (tests/proof_sweep.py) -> profiles/r03_proof_sweep.json.  Two sweeps: inside the
envelope the library enables the proofs in (include/rrt.h RRT_PROOF_*: delta_theta in
[0.04, 0.6], r_s <= 0.5 x the room's largest extent) and beyond it (delta_theta in [0.005, 1.2],
r_s up to 1.5 x the room's extent), reporting per proof the share proven, the smallest headroom
(margin / deviation of the recurrence from the reference's march) and violations (a proven ray or
pixel the reference's march contradicts).  TEST INFRASTRUCTURE (CPU, oracle restatement)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "relativistic-ray-tracer_amd"))
import proof_sweep as P  # noqa: E402


def summary(res):
    out = {}
    for k in ("camera", "pixel", "shadow"):
        rows = [r[k] for r in res]
        out[k] = {"configs": len(rows), "violations": sum(r["violations"] for r in rows),
                  "mean_proven": sum(r["proven"] for r in rows) / max(len(rows), 1)}
        if k != "pixel":
            w = max((r["worst_dev_over_margin"] for r in rows), default=0.0)
            out[k]["worst_dev_over_margin"] = w
            out[k]["min_headroom"] = (1.0 / w) if w > 0 else None
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", type=int, default=240)
    ap.add_argument("--beyond", type=int, default=120)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_proof_sweep.json"))
    a = ap.parse_args()
    t0 = time.time()

    def log(i, r):
        print(i, r["scene"], [round(v, 3) for v in r["bh"]], r["frame"],
              {k: {kk: (round(vv, 6) if isinstance(vv, float) else vv) for kk, vv in r[k].items()}
               for k in ("camera", "pixel", "shadow")}, flush=True)

    inside = P.sweep(a.configs, 2024, n_cam=600, n_pix=120, n_shadow=600, log=log)
    beyond = P.sweep(a.beyond, 4048, n_cam=400, n_pix=60, n_shadow=400, log=log, dt_range=(0.005, 1.2), rs_max=1.5)
    out = {"envelope": {"delta_theta": list(P.DT_RANGE), "rs_over_box_max": P.RS_OVER_BOX_MAX},
           "inside": summary(inside), "beyond": summary(beyond), "seconds": time.time() - t0,
           "configs_inside": inside, "configs_beyond": beyond}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("envelope", "inside", "beyond", "seconds")}, indent=1))


if __name__ == "__main__":
    main()
