#!/usr/bin/env python3
"""What ends a launch: the pixels that stop last (tools/phase_profile.py's per-pixel maps from the
profile build: elapsed time, speculation rounds and stop time of every batch-kernel pixel).

Usage: tail_analysis.py gpurun_out/px_<case>_0.npz gpurun_out/pp_<case>.json ..."""
import json
import sys

import numpy as np


def report(npz, pp):
    d = np.load(npz)
    t, e, rd = d["ms"], d["end"], d["rounds"]
    j = json.load(open(pp))["results"]["0"]
    K = j["kernel_ms"]
    m = e >= 0
    print(f"{npz}: kernel {K:.2f} ms (profile build), claims exhausted at {j['exhausted_at']:.2f} of it, "
          f"{int(m.sum())} pixels")
    for thr in (0.7, 0.8, 0.9):
        s = m & (e > thr)
        if not s.any():
            continue
        start = e[s] - t[s] / K
        print(f"  stopping after {thr:.1f}: {int(s.sum())} pixels, {t[s].mean():.2f} ms each on average, "
              f"rounds {np.bincount(rd[s], minlength=8)[1:8].tolist()} (1..7), claimed at "
              f"{np.quantile(start, 0.5):.2f} (median) / {start.max():.2f} (last) of the launch")


if __name__ == "__main__":
    a = sys.argv[1:]
    for i in range(0, len(a), 2):
        report(a[i], a[i + 1])
