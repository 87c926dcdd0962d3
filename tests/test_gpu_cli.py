"""GPU: the reference's command line, end to end (rrt_render = main.cpp's windowless path over
rrt::PathTracer, the native COLLADA ingest and librrt's HIP kernels).  The PNG and the sampling-
rate PNG it writes must equal, pixel for pixel, the files the reference itself wrote for the same
flags (tests/golden/<case>/ref.png, ref_rate.png; make_golden.py KEEP_PNG)."""
import json
import os
import subprocess

import numpy as np
import pytest

from golden_cases import GOLD
from png_util import read_png

pytestmark = pytest.mark.gpu
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
CLI = os.path.join(ROOT, "relativistic-ray-tracer_amd", "rrt_render")


@pytest.mark.parametrize("case", ["spheres_96x72_s8_l4", "cfg1_spheres_480x360_s8", "bunny_1080p_s64_crop"])
def test_cli_png_matches_reference(case, tmp_path):
    info = json.load(open(os.path.join(GOLD, case, "case.json")))
    out = str(tmp_path / "out.png")
    cmd = [CLI] + info["args"] + ["-f", out, os.path.join(GOLD, "dae", info["dae"])]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    print(r.stdout[-400:], r.stderr[-400:])
    assert r.returncode == 0
    assert np.array_equal(read_png(out), read_png(os.path.join(GOLD, case, "ref.png")))
    assert np.array_equal(read_png(str(tmp_path / "out_rate.png")), read_png(os.path.join(GOLD, case, "ref_rate.png")))


@pytest.mark.parametrize("case", ["cfg1_spheres_480x360_s8", "bunny_1080p_s64_crop"])
@pytest.mark.parametrize("devices", ["0,0", "0,0,0"])
def test_cli_device_group_matches_reference(case, devices, tmp_path):
    """--devices: rrt::PathTracer over a device group (rrt_group: one context per listed GPU,
    block-cyclic tiles, gather to member 0 and unpack).  On one GPU the members share the device,
    so the gather takes device copies (RCCL needs distinct devices); the partition, the packed
    buffers and the unpack are the multi-GPU plan's, and the PNGs must still equal the reference's."""
    info = json.load(open(os.path.join(GOLD, case, "case.json")))
    out = str(tmp_path / "out.png")
    cmd = [CLI] + info["args"] + ["--devices", devices, "-f", out, os.path.join(GOLD, "dae", info["dae"])]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    print(r.stdout[-400:], r.stderr[-400:])
    assert r.returncode == 0 and "device(s)" in r.stdout
    assert np.array_equal(read_png(out), read_png(os.path.join(GOLD, case, "ref.png")))
    assert np.array_equal(read_png(str(tmp_path / "out_rate.png")), read_png(os.path.join(GOLD, case, "ref_rate.png")))


def test_cli_usage_and_errors(tmp_path):
    assert subprocess.run([CLI], capture_output=True).returncode == 1
    r = subprocess.run([CLI, "-f", str(tmp_path / "x.png"), "/nonexistent.dae"], capture_output=True, text=True)
    assert r.returncode == 2 and "cannot open" in r.stderr


def test_cli_kerr_matches_restatement(tmp_path):
    """--kerr A: the CLI renders the Kerr spacetime; its PNG is the tonemapped
    restatement render of the same flags (parity against the reference: unpinned, no Kerr there)."""
    import oracle_lib as ol
    from golden_cases import Case
    from test_image_io import tonemap
    case = "spheres_96x72_s8_l4"
    c = Case(case)
    out = str(tmp_path / "kerr.png")
    cmd = [CLI] + c.info["args"] + ["--kerr", "0.9", "0", "1", "0", "-f", out, os.path.join(GOLD, "dae", c.info["dae"])]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    print(r.stdout[-400:], r.stderr[-400:])
    assert r.returncode == 0
    g = c.cfg
    p = ol.make_params(c.frame_w, c.frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                       ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                       max_tolerance=g["max_tolerance"], bh=g["bh"], kerr=(0.9, (0.0, 1.0, 0.0)))
    rgb, _, _, _ = ol.render(ol.Scene(c.scene_path), ol.load_camera(c.camera_path), p, 0, 0, c.frame_w, c.frame_h)
    want = tonemap(rgb)[::-1].copy().view(np.uint8).reshape(c.frame_h, c.frame_w, 4)
    got = read_png(out)
    assert np.array_equal(got, want)
    assert not np.array_equal(got, read_png(os.path.join(GOLD, case, "ref.png")))
