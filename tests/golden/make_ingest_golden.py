#!/usr/bin/env python3
"""Golden fixtures for the native COLLADA ingest (include/rrt.h rrt_collada_load).

TEST INFRASTRUCTURE ONLY (build container; needs /root/reference and oracle/_ref/ref_render,
built by `make -C oracle/ref`).  For every scene asset the reference ships, runs the reference's
own loader through the oracle harness in dump-only mode (`ref_render -Q -r W H`: Collada parser
-> Application::load -> get_static_scene, Camera::configure/place/set_screen_size) and records
the SHA-256 of the flattened scene (.rrts) and camera record (.rrtc) it writes.  Small assets are
also copied (as input data) into tests/golden/dae/ so the ingest tests run without the reference.

Output: tests/golden/ingest.json = {scene: {"src": relative path under dae/, "w": W, "h": H,
"rrts_sha256": ..., "rrtc_sha256": ..., "bytes": n, "committed": bool}}
"""
import hashlib
import json
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
GOLD = os.path.join(ROOT, "tests", "golden")
DAE = "/root/reference/pathtracer/dae"
BIN = os.path.join(ROOT, "oracle", "_ref", "ref_render")
W, H = 64, 48
COMMIT_LIMIT = 2_000_000  # bytes: inputs up to this size are copied into tests/golden/dae/
SKIP = {"CBbunny_microfacet_cu", "bunny_microfacet_cu", "bunny_microfacet_cu_unlit", "bunny_unlit", "bunny",
        "CBspheres_tex"}  # duplicates of committed meshes (kept reference-only)


def main():
    out = {}
    tmp = tempfile.mkdtemp()
    for sub in sorted(os.listdir(DAE)):
        for f in sorted(os.listdir(os.path.join(DAE, sub))):
            if not f.endswith(".dae"):
                continue
            name = f[:-4]
            src = os.path.join(DAE, sub, f)
            pre = os.path.join(tmp, name)
            subprocess.run([BIN, "-Q", "-r", str(W), str(H), "-O", pre, src], check=True,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            size = os.path.getsize(src)
            commit = size <= COMMIT_LIMIT and name not in SKIP
            if commit:
                shutil.copy(src, os.path.join(GOLD, "dae", f))
            out[name] = {"src": f"{sub}/{f}", "w": W, "h": H, "bytes": size, "committed": commit,
                         "rrts_sha256": hashlib.sha256(open(pre + ".rrts", "rb").read()).hexdigest(),
                         "rrtc_sha256": hashlib.sha256(open(pre + ".rrtc", "rb").read()).hexdigest()}
            print(name, size, "committed" if commit else "reference-only")
    with open(os.path.join(GOLD, "ingest.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    shutil.rmtree(tmp)


if __name__ == "__main__":
    main()
