"""bench.py --gpus N runs N ranks by itself (torch.distributed.run on 127.0.0.1) when no launcher
set WORLD_SIZE, and refuses to report N GPUs it does not have."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_self_launch_runs_n_ranks():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line == {"launch_check": True, "world_size": 2, "all_reduce": 2.0, "requested": 2}


def test_more_gpus_than_visible_fails():
    env = _env()
    env["HIP_VISIBLE_DEVICES"] = ""  # none visible (also true on this CPU-only host)
    env["CUDA_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "8"], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 2
    assert "GPU(s) visible" in r.stderr
