"""bench.py's multi-GPU launch contract (CPU): `--gpus N` without torchrun's WORLD_SIZE starts N
ranks itself (pathtracer.cpp:279-281 starts one worker per thread; here one process per GPU), a
WORLD_SIZE that disagrees with --gpus is an error, and a request for more GPUs than are visible
fails loudly instead of printing a one-GPU line labelled N."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_check_world_modes():
    assert bench.check_world(1, {}) == "single"
    assert bench.check_world(4, {}) == "launch"
    assert bench.check_world(4, {"WORLD_SIZE": "4"}) == "rank"
    assert bench.check_world(1, {"WORLD_SIZE": "1"}) == "single"
    with pytest.raises(SystemExit):
        bench.check_world(2, {"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        bench.check_world(1, {"WORLD_SIZE": "8"})
    with pytest.raises(SystemExit):
        bench.check_world(0, {})


def test_launch_command_is_the_drivers_torchrun_form():
    cmd = bench.rank_launch_cmd(["--gpus", "8", "--steps", "3"], 8, 29500)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]
    assert os.path.samefile(cmd[cmd.index("--master-port=29500") + 1], os.path.join(ROOT, "bench.py"))


def test_too_many_gpus_fails_loudly():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["HIP_VISIBLE_DEVICES"] = env["CUDA_VISIBLE_DEVICES"] = ""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode != 0
    assert "GPU(s) visible" in p.stderr
    assert '"n_gpus"' not in p.stdout


def test_world_size_mismatch_fails_loudly():
    env = dict(os.environ, WORLD_SIZE="1")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in p.stderr
