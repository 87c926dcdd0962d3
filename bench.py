#!/usr/bin/env python3
"""bench.py -- Msamples/s of the relativistic path tracer's hot path on MI355X.

Workload (BASELINE.json configs[2], the config the metric is quoted on): CBbunny.dae at
1920x1080, 64 spp (adaptive: batch 32, tol 0.05), Schwarzschild black hole (centre (0,1,0),
r_s 0.1, dtheta 0.1), max_ray_depth 1 -- the reference defaults.  The scene is the reference's
own asset (a copy under tests/golden/dae/), read by the native COLLADA ingest
(rrt_collada_load: byte-identical to the reference loader's scene and placed camera); scene and
camera are HBM-resident before timing.  --workload cfg4 runs BASELINE configs[3] on the
generated 100k-triangle torus-knot scene (rrt_scenes.py; CBdragon.dae is missing upstream) at
3840x2160, 256 spp; --workload cfg5 runs configs[4]: the Kerr integrator (a/M 0.9)
with the generated HDR sky environment map, CBbunny at 3840x2160, 1024 spp.

One step = one full frame.  With N GPUs (one process per GPU, torchrun) the frame's tiles
(32x32; 16x16 for cfg5) are dealt over the ranks as a lattice (rrt_partition_tiles: tile (tx, ty)
to rank (tx + S ty) % N); every rank renders its tiles into a
packed buffer and rank 0 gathers them over RCCL and unpacks them into the frame (the only
exchange step).  Total work is fixed, so scaling is "strong".

value = actual camera samples in the frame (sum of the per-pixel sampleCountBuffer, i.e.
adaptive-aware) x steps / max-over-ranks wall time.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "relativistic-ray-tracer_amd"))
# importing rrt does not load librrt.so (rrt.lib() does, on first use): the parent of a
# multi-rank run loads no HIP library and touches no GPU before its ranks start
import rrt  # noqa: E402
import rrt_frame  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
WORKLOADS = {
    "cfg3": dict(dae="CBbunny.dae", w=1920, h=1080, spp=64, bh=((0.0, 1.0, 0.0), 0.1, 0.1), row_stride=8,
                 desc="cfg3: CBbunny.dae 1920x1080 64spp, Schwarzschild geodesic (r_s 0.1, dtheta 0.1), depth 1"),
    "cfg2": dict(dae="CBspheres_lambertian.dae", w=1920, h=1080, spp=64, bh=((0.0, 1.0, 0.0), 0.0, 0.1),
                 row_stride=8, desc="cfg2: CBspheres_lambertian.dae 1920x1080 64spp, flat limit (r_s 0), depth 1"),
    "cfg1": dict(dae="CBspheres_lambertian.dae", w=480, h=360, spp=8, bh=((0.0, 1.0, 0.0), 0.1, 0.1), row_stride=2,
                 desc="cfg1: CBspheres_lambertian.dae 480x360 8spp, Schwarzschild"),
    "cfg4": dict(dae="@cfg4", w=3840, h=2160, spp=256, bh=((0.0, 1.0, 0.0), 0.1, 0.1), row_stride=32,
                 desc="cfg4: torus knot (100k tris, CBdragon substitute) in CBempty, 3840x2160 256spp, "
                      "Schwarzschild, depth 1"),
    "m3": dict(dae="CBspheres_lambertian.dae", w=1920, h=1080, spp=64, bh=((0.0, 1.0, 0.0), 0.1, 0.1), row_stride=24,
               depth=3, desc="m3: CBspheres_lambertian.dae 1920x1080 64spp, Schwarzschild, max_ray_depth 3 "
                             "(at_least_one_bounce_radiance, part1_code.cpp:69-101)"),
    "cfg5": dict(dae="CBbunny.dae", w=3840, h=2160, spp=1024, bh=((0.0, 1.0, 0.0), 0.1, 0.1), row_stride=24,
                 kerr=(0.9, (0.0, 1.0, 0.0)), env="@sky", tile=16,
                 desc="cfg5: CBbunny.dae 3840x2160 1024spp, Kerr a/M 0.9 (axis +y, r_s 0.1, dtheta 0.1) + "
                      "1024x512 HDR sky envmap, depth 1"),
}


# reference-rendered goldens (tests/golden/, made by the compiled reference under the keyed RNG)
# that cover each workload's frame: bench.py checks the frame it timed against them bit for bit
VERIFY = {"cfg1": ["cfg1_spheres_480x360_s8"], "cfg2": ["cfg2_spheres_1080p_s64_flat"],
          "cfg3": ["cfg3_bunny_1080p_s64"],
          "cfg4": ["cfg4_knot_4k_s256_crop", "cfg4_knot_4k_s256_crop2", "cfg4_knot_4k_s256_crop3"],
          "m3": ["m3_spheres_1080p_s64_crop", "m3_spheres_1080p_s64_crop2"]}


def verify_frame(workload, rgb, cnt):
    """Compare the timed frame (rgb [H][W][3] f32, cnt [H][W] i32, sampleBuffer layout) with the
    workload's reference goldens, bit for bit -> (verified: bool | None, note)."""
    names = VERIFY.get(workload)
    if not names:
        why = {"cfg5": "Kerr has no reference (parity unpinned); tests/test_gpu_kerr.py pins crops of this "
                       "framing against the restatement",
               }
        return None, why.get(workload, "no reference golden for this workload")
    notes = []
    for n in names:
        d = os.path.join(GOLD, n)
        with open(os.path.join(d, "case.json")) as f:
            reg = json.load(f)["region"]
        px = np.load(os.path.join(d, "px.npz"))
        ys, xs = slice(reg["y0"], reg["y0"] + reg["h"]), slice(reg["x0"], reg["x0"] + reg["w"])
        got_rgb, got_cnt = rgb[ys, xs], cnt[ys, xs]
        bad = (got_rgb.view(np.uint32) != px["rgb"].view(np.uint32)).any(-1) | (got_cnt != px["count"])
        if bad.any():
            return False, f"{n}: {int(bad.sum())} of {bad.size} pixels differ from the reference golden"
        notes.append(f"{n} ({reg['w']}x{reg['h']} at {reg['x0']},{reg['y0']})")
    return True, "bit-exact (RGB and sample counts) vs reference goldens: " + ", ".join(notes)


def load_workload_env(wl, workdir):
    """The workload's environment map texels (generated sky EXR read by the native loader), or None."""
    if not wl.get("env"):
        return None
    import rrt_scenes
    path = os.path.join(workdir, "sky.exr")
    rrt_scenes.write_cfg5_envmap(path)
    return rrt.load_exr(path)


def load_workload_scene(wl, workdir):
    """Native COLLADA ingest of the workload's scene -> (SceneFile, CameraState, .rrts, .rrtc)
    (the .rrts/.rrtc copies feed the CPU baseline's restatement)."""
    if wl["dae"].startswith("@"):
        import rrt_scenes
        path = os.path.join(workdir, wl["dae"][1:] + ".dae")
        rrt_scenes.write_cfg4_dae(path)
    else:
        path = os.path.join(GOLD, "dae", wl["dae"])
    scene, cam = rrt.load_collada(path, wl["w"], wl["h"])
    spath, cpath = os.path.join(workdir, "scene.rrts"), os.path.join(workdir, "camera.rrtc")
    scene.save(spath)
    rc = rrt.lib().rrt_camera_state_file_save(cpath.encode(), cam)
    assert rc == 0
    return scene, cam, spath, cpath
TILE = 32  # the split's tile side; cfg5 deals 16-px tiles (WORKLOADS "tile"): its cost sits in the lensed
           # ring around the hole, and finer tiles spread it over the ranks (8-way slowest rank 243 -> 217 ms,
           # profiles/r06_deal_w8.txt); cfg3 / cfg4 are faster at 32 (3.15 vs 3.23 ms, 3.03 vs 3.23 ms)
AUDIT_EVERY_LOG2 = 10  # proof audit: every 1024th proven ray / pixel of the executed-work pass
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
BYTES_AABB, BYTES_PRIM, BYTES_PIXEL = 48, 72, 16  # SURVEY 8(d) algorithmic bytes
BYTES_PLANE = 32  # plane-cull record (DPlane) read per plane test


# MI355X FP64 vector peak (spec, AMD MI355X datasheet: 78.6 TFLOP/s FP64 vector = 256 CUs x
# 128 flop/clk x 2.4 GHz, i.e. a wave64 FP64 FMA every 4 cycles per SIMD; tools/ubench_f64.hip
# measures that issue rate on the box, profiles/r03_ubench_f64.log)
FP64_PEAK_TFLOPS = 78.6
FP64_CYCLES_PER_WAVE_INST = 4.0
N_SIMD = 1024


PROFILE_ROUNDS = ("r06", "r05", "r04", "r03")  # profiles/ files searched, newest first (each must match the build)


def find_profile(explicit, names, workload, kernel):
    """The first profiles/ JSON (or the explicit path) recorded for this workload, kernel and
    librrt.so build (rrt.build_id) -- numbers from another build are never attached to this line."""
    paths = [explicit] if explicit else [os.path.join(ROOT, "profiles", n) for n in names]
    bid = rrt.build_id()
    for path in paths:
        if path and os.path.exists(path):
            with open(path) as f:
                d = json.load(f)
            if (d.get("workload") == workload and kernel in (d.get("kernel"), d.get("main_kernel")) and
                    d.get("build_id") == bid):
                d["_path"] = os.path.relpath(path, ROOT)
                return d
    return None


def rooflines(loc_bytes, ref_bytes, main_ms, kernel_name, main_kernel, traffic, pmc, out_bytes=0.0):
    """The dominant kernel against its real bound, FP64 VALU issue (PMC, profiles/r03_*_pmc.json),
    and against HBM on the survey's algorithmic bytes, both per launch of that
    kernel over its HIP-event time in this run.  The algorithmic bytes are reads of a scene that
    stays L2/MALL-resident, so the HBM line's `traffic` (PMC FETCH/WRITE of the same kernel,
    split into register-spill scratch and the rest) is what HBM actually moved."""
    t = main_ms * 1e-3
    hbm_ach = loc_bytes / t / 1e9
    src = pmc if (pmc and pmc.get("hbm_bytes") is not None) else traffic
    hbm = {"bound": "hbm", "achieved": hbm_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm_ach / HBM_PEAK_GBS,
           "traffic": src.get("hbm_bytes", src.get("hbm_bytes_per_launch")) if src else None,
           # WRITE_SIZE beyond the kernel's outputs is register-spill scratch (the kernel writes nothing
           # else); FETCH_SIZE mixes scratch reloads with scene reads that miss L2
           "traffic_scratch_writes": max(src["write_bytes"] - out_bytes, 0.0) if src and "write_bytes" in src else None,
           "traffic_fetch": src.get("fetch_bytes") if src else None,
           "output_bytes": out_bytes,
           "traffic_source": src["_path"] if src else None,
           "kernel": main_kernel, "kernel_ms": main_ms, "launch": kernel_name,
           "algorithmic_bytes_per_launch": float(loc_bytes),
           "reference_algorithm_bytes_per_launch": float(ref_bytes),
           "reference_equivalent_GBps": ref_bytes / t / 1e9}
    out = {"roofline_hbm": hbm}
    if pmc:
        flops = pmc["fp64_flops_per_launch"]
        ach = flops / t / 1e12
        insts = pmc["fp64_wave_insts_per_launch"]
        clk = pmc.get("clock_hz") or 2.4e9
        out["roofline"] = {
            "bound": "fp64_valu", "achieved": ach, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": ach / FP64_PEAK_TFLOPS, "traffic": hbm["traffic"], "kernel": main_kernel, "kernel_ms": main_ms,
            "fp64_flops_per_launch": flops, "fp64_wave_insts_per_launch": insts,
            "valu_lane_util": pmc["valu_lane_util"],
            # share of the chip's FP64 issue slots (a wave64 FP64 op per 4 cycles per SIMD) used
            "fp64_issue_frac": insts * FP64_CYCLES_PER_WAVE_INST / (N_SIMD * clk * t),
            "valu_busy_frac": pmc.get("valu_busy_frac"),
            "source": pmc["_path"]}
    else:
        out["roofline"] = dict(hbm, note="no PMC profile of this kernel build: HBM line only")
    return out


def host_cores():
    """Host cores this process may use: the affinity mask, capped by a cgroup CPU quota (the GPU
    box's share of its host)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(wl, threads, row_stride, scene_path, camera_path, env=None):
    """The oracle restatement (oracle/restate, bit-exact with the reference) on the host cores,
    over every `row_stride`-th row of the same frame (a representative bounded sample)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    s = O.Scene(scene_path)
    if env is not None:
        s.set_envmap(env)
    cam = O.load_camera(camera_path)
    c, r_s, dt = wl["bh"]
    p = O.make_params(wl["w"], wl["h"], ns_aa=wl["spp"], max_ray_depth=wl.get("depth", 1), bh=(c[0], c[1], c[2], r_s, dt),
                      kerr=wl.get("kerr"))
    rows = list(range(row_stride // 2, wl["h"], row_stride))
    samples = 0
    t0 = time.perf_counter()
    for y in rows:
        _, cnt, _, _ = O.render(s, cam, p, 0, y, wl["w"], 1, threads=threads)
        samples += int(cnt.sum())
    dt_s = time.perf_counter() - t0
    out = {"value": samples / dt_s / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
           "cpu_model": cpu_model(), "host_cores_visible": os.cpu_count(),
           "sample": f"rows {rows[0]}::{row_stride} of the {wl['w']}x{wl['h']} frame ({len(rows)} rows, "
                     f"{samples} samples, {dt_s:.1f} s); oracle/restate (C, bit-exact with the reference "
                     f"under the keyed RNG), pthreads over 32-px tiles"}
    # the restatement's speed relative to the compiled reference on the same cores and sample,
    # measured in the build container (tools/cpu_ratio.py; the reference does not travel here)
    ratio_path = os.path.join(ROOT, "profiles", "r03_cpu_ratio.json")
    if os.path.exists(ratio_path):
        with open(ratio_path) as f:
            rr = json.load(f).get(wl_name(wl))
        if rr:
            out["restatement_over_reference_speed"] = rr["speed_ratio"]
            out["reference_equivalent_value"] = out["value"] / rr["speed_ratio"]
            out["ratio_measured"] = rr["where"]
    return out


def wl_name(wl):
    return next(k for k, v in WORKLOADS.items() if v is wl)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_launch_cmd(argv, n, port):
    """The torchrun command that runs this script as n ranks on one node (the driver's own form)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def check_world(gpus, env=None):
    """How this process takes part in a --gpus N run: "launch" (no WORLD_SIZE and N > 1: start the
    N ranks), "rank" (one of WORLD_SIZE == N ranks) or "single".  A WORLD_SIZE that disagrees
    with --gpus is an error, never a relabelled run."""
    env = os.environ if env is None else env
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus {gpus} < 1")
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "launch" if gpus > 1 else "single"
    if int(ws) != gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={ws} but --gpus {gpus}")
    return "rank" if gpus > 1 else "single"


def launch_ranks(gpus, argv):
    """Parent of a multi-GPU run (pathtracer.cpp:279-281 starts one worker per thread; here one
    process per GPU): checks the GPU count WITHOUT initialising HIP (torch.cuda.device_count()
    does not, on this image), starts the ranks with torchrun and returns its exit code.  Rank 0
    prints the JSON line straight to this process's stdout."""
    import torch
    n = torch.cuda.device_count()
    if n < gpus:
        raise SystemExit(f"bench.py --gpus {gpus}: only {n} GPU(s) visible")
    return subprocess.run(rank_launch_cmd(argv, gpus, _free_port())).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="cfg3", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--variant", type=int, default=0, help="rrt_render_params.variant (A/B: waves per SIMD)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-row-stride", type=int, default=0, help="0 = the workload's default")
    ap.add_argument("--traffic", default=None,
                    help="PMC-measured HBM bytes per launch (tools/pmc_traffic.py) for roofline.traffic; "
                         "default profiles/r0N_traffic_<workload>.json, newest round first")
    ap.add_argument("--pmc", default=None,
                    help="PMC FP64 VALU counters per launch (tools/pmc_valu.py) for the fp64_valu roofline; "
                         "default profiles/r0N_<workload>_pmc.json, newest round first")
    a = ap.parse_args()

    mode = check_world(a.gpus)
    if mode == "launch":
        sys.exit(launch_ranks(a.gpus, sys.argv[1:]))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        if torch.cuda.device_count() <= local:
            raise SystemExit(f"bench.py rank {rank}: no GPU for local rank {local}")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        world = dist.get_world_size()
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    wl = WORKLOADS[a.workload]
    W, H = wl["w"], wl["h"]

    import tempfile
    workdir = tempfile.mkdtemp(prefix="rrt_bench_")
    r = rrt.Renderer(device=torch.cuda.current_device())
    scene, cam_state, scene_path, camera_path = load_workload_scene(wl, workdir)
    r.set_scene(scene)
    r.set_camera(rrt.camera_desc(cam_state))
    env = load_workload_env(wl, workdir)
    r.set_envmap(env)
    kerr = wl.get("kerr")
    r.set_black_hole(*wl["bh"], **({"spin": kerr[0], "axis": kerr[1]} if kerr else {}))
    depth = wl.get("depth", 1)
    params = rrt.render_params(W, H, ns_aa=wl["spp"], max_ray_depth=depth, variant=a.variant)

    tile = wl.get("tile", TILE)
    plan = rrt_frame.FramePlan(W, H, world, tile)
    tiles = plan.tiles(rank)
    tpix = plan.tpix
    # packed per-rank result (rrt_frame.py layout): f32 rgb then i32 counts
    packed = torch.zeros(plan.words, dtype=torch.int32, device=dev)
    p_rgb = packed.data_ptr()
    p_cnt = packed.data_ptr() + plan.count_offset * 4
    stream = torch.cuda.current_stream()
    s_handle = stream.cuda_stream
    if rank == 0:
        frame_rgb = torch.zeros(H * W * 3, dtype=torch.float32, device=dev)
        frame_cnt = torch.zeros(H * W, dtype=torch.int32, device=dev)

    kern_ms = []

    def step(timed):
        # poison every output buffer in-stream first (NaN radiance, count -1): the frame verified
        # after the timed steps can only come from the last of them (~33 MB per 1080p frame, ~10 us)
        packed.fill_(-1)
        if rank == 0:
            frame_rgb.view(torch.int32).fill_(-1)
            frame_cnt.fill_(-1)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        r.render_tiles_device(params, tiles, tile, p_rgb, p_cnt, stream=s_handle)
        e1.record(stream)
        bufs = rrt_frame.gather(dist, packed, rank, world)  # RCCL over xGMI; the only exchange
        if rank == 0:
            for q in range(world):
                base = bufs[q].data_ptr()
                r.unpack_tiles_device(plan.tiles(q), tile, W, H, base, base + plan.count_offset * 4,
                                      frame_rgb.data_ptr(), frame_cnt.data_ptr(), stream=s_handle)
        if timed:
            kern_ms.append((e0, e1))

    for _ in range(a.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    k_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in kern_ms]))
    # the timed launches' own HIP events (recorded by librrt on this stream around each launch and
    # before its main kernel): the dominant kernel's average duration, for the roofline
    tot_ms, main_ms = r.launch_times(min(a.steps, 32))
    main_ms = float(np.mean(main_ms))

    kernel_name = r.stats().kernel.decode()

    # work of this rank's launch, counted by the counting kernel outside the timed region: the
    # work the renderer executes (roofline) and the reference algorithm's work
    n_loc = len(tiles)
    pix_local = sum(min(tile, W - int(x)) * min(tile, H - int(y)) for x, y in tiles)

    def count_pass(flags):
        ctr = torch.zeros(max(n_loc, 1) * tpix * 4, dtype=torch.int32, device=dev)
        tmp = torch.zeros(max(n_loc, 1) * tpix * 4, dtype=torch.int32, device=dev)
        cparams = rrt.render_params(W, H, ns_aa=wl["spp"], max_ray_depth=depth, flags=rrt.RRT_RENDER_COUNTERS | flags)
        r.render_tiles_device(cparams, tiles, tile, tmp.data_ptr(), tmp.data_ptr() + n_loc * tpix * 3 * 4,
                              d_counters=ctr.data_ptr(), stream=s_handle)
        torch.cuda.synchronize()
        c4 = ctr.view(-1, 4).to(torch.int64).sum(0).cpu().numpy()
        cnt = float(tmp[n_loc * tpix * 3:n_loc * tpix * 4].to(torch.int64).sum().item())
        t = torch.tensor([cnt] + [float(v) for v in c4] + [float(pix_local)], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t)
        return [float(v) for v in t.cpu().numpy()], c4

    (samples, bbox, micro, prim, queries, pixels), _ = count_pass(0)
    # the executed-work pass runs the proofs: audit every 1024th proven ray (and pixel) exactly
    r.set_proof_audit(AUDIT_EVERY_LOG2)
    (_, x_bbox, x_micro, x_prim, x_plane, _), xc4 = count_pass(rrt.RRT_RENDER_COUNT_EXECUTED)
    r.set_proof_audit(-1)
    audit = r.proof_audit()
    if world > 1:
        at = torch.tensor([[v["checked"], v["violations"]] for v in audit.values()], dtype=torch.float64, device=dev)
        dist.all_reduce(at)
        audit = {k: {"checked": int(at[i, 0]), "violations": int(at[i, 1])} for i, k in enumerate(audit)}
    audit_violations = sum(v["violations"] for v in audit.values())
    loc_bytes = BYTES_AABB * xc4[0] + BYTES_PRIM * xc4[2] + BYTES_PLANE * xc4[3] + BYTES_PIXEL * pix_local
    ref_bytes = BYTES_AABB * bbox + BYTES_PRIM * prim + BYTES_PIXEL * pixels
    main_kernel = kernel_name.split(" + ")[-1]
    traffic = find_profile(a.traffic, [f"{r}_traffic_{a.workload}.json" for r in PROFILE_ROUNDS], a.workload, kernel_name)
    pmc = find_profile(a.pmc, [f"{r}_{a.workload}_pmc.json" for r in PROFILE_ROUNDS], a.workload, main_kernel)

    verified = None
    if rank == 0:
        # sanity: the gathered frame holds every pixel's sample count
        frame_samples = int(frame_cnt.to(torch.int64).sum().item())
        assert frame_samples == int(samples), (frame_samples, samples)
        # the frame the timed steps produced (every step rewrites all of it), against the reference
        verified, verify_note = verify_frame(a.workload, frame_rgb.view(H, W, 3).cpu().numpy(),
                                             frame_cnt.view(H, W).cpu().numpy())
        value = samples * a.steps / elapsed / 1e6
        work = {"aabb_tests": bbox / samples, "micro_steps": micro / samples, "prim_tests": prim / samples,
                "queries": queries / samples}
        xwork = {"aabb_tests": x_bbox / samples, "micro_steps": x_micro / samples, "prim_tests": x_prim / samples,
                 "plane_tests": x_plane / samples}
        out = {
            "metric": "Msamples/sec (whole node), 1080p 64spp CBbunny + Schwarzschild geodesic"
            if a.workload == "cfg3" else f"Msamples/sec (whole node), {wl['desc']}",
            "value": value,
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("generated torus-knot scene (rrt_scenes.py)" if wl["dae"].startswith("@") else
                     "reference scene asset") + " via the native COLLADA ingest" +
                    (", generated HDR sky envmap (rrt_scenes.py)" if env is not None else "") + ", keyed RNG seed 0",
            "config": {"workload": wl["desc"], "frame": [W, H], "spp": wl["spp"], "tile": tile,
                       "partition": (f"lattice deal of {tile}x{tile} tiles over {world} GPUs, RCCL gather to rank 0"
                                     if world > 1 else "whole frame on 1 GPU, no gather")},
            "verified": verified,
            "verify": verify_note,
            "samples_per_frame": int(samples),
            "nominal_msamples_per_s": W * H * wl["spp"] * a.steps / elapsed / 1e6,
            "kernel_ms_rank0": k_ms,
            "main_kernel_ms_rank0": main_ms,
            "work_per_sample_reference": work,
            "work_per_sample_executed": xwork,
            # run-time audit of the proofs (skipped marches): every 2^AUDIT_EVERY_LOG2-th proven ray
            # of the untimed executed-work pass re-marched exactly (rrt_set_proof_audit)
            "proof_violations": audit_violations,
            "proof_audit": dict(audit, every=1 << AUDIT_EVERY_LOG2),
        }
        out.update(rooflines(loc_bytes, ref_bytes, main_ms, kernel_name, main_kernel, traffic, pmc,
                             out_bytes=float(BYTES_PIXEL * pix_local)))
        if world == 1 and not a.no_cpu_baseline:
            threads = a.cpu_threads or host_cores()
            out["cpu_baseline"] = cpu_baseline(wl, threads, a.cpu_row_stride or wl["row_stride"], scene_path,
                                               camera_path, env)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if rank == 0 and verified is False:
        sys.exit("bench.py: the timed frame differs from the reference: " + verify_note)
    if rank == 0 and audit_violations:
        sys.exit(f"bench.py: the proof audit found {audit_violations} proven rays the exact march contradicts")


if __name__ == "__main__":
    main()
