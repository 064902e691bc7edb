"""bench.py's N-rank pipeline (SURVEY §8 row e; camera.h:276-294 is the reference's row-parallel
loop) on one GPU: two ranks launched by torch.distributed.run share the device and gather over gloo
(RCCL refuses two ranks on one device). Each rank renders its 4-row blocks packed into its tile
(CRT_TILING_PACKED), the tiles are all-gathered on the side stream while the next frame renders,
and every rank's last assembled frame must equal the one-rank frame bit for bit."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
ARGS = ["--width", "160", "--height", "98", "--spp", "8", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["CRT_BENCH_BACKEND"] = "gloo"
    return env


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ranks_run(ranks, extra, env):
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
                        "--master-addr=127.0.0.1", f"--master-port={_port()}", str(ROOT / "bench.py"),
                        "--gpus", str(ranks), *ARGS, *extra],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("ranks", [2, 3])
def test_bench_ranks_assemble_the_one_rank_frame(tmp_path, ranks):
    """... and the bench line's frame_check says so by itself: the N-rank digest equals the N=1
    digest and every rank holds the same frame."""
    one = tmp_path / "one"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *ARGS, "--dump-frame", str(one)],
                       capture_output=True, text=True, timeout=600, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    line1 = json.loads(r.stdout.strip().splitlines()[-1])
    many = tmp_path / "many"
    line = _ranks_run(ranks, ["--dump-frame", str(many)], _env())
    want = np.load(f"{one}.rank0.npy")
    assert want.shape == (98, 160, 3) and np.isfinite(want).all()
    for k in range(ranks):
        assert np.array_equal(np.load(f"{many}.rank{k}.npy"), want), f"rank {k}"
    fc1, fc = line1["frame_check"], line["frame_check"]
    assert fc1["ranks_agree"] is True
    assert fc["ranks_agree"] is True and fc["frame_digest"] == fc1["frame_digest"]
    assert fc["rank_digests"] == [fc1["frame_digest"]] * ranks


def test_bench_frame_check_flags_a_rank_that_differs():
    env = _env()
    env["CRT_BENCH_CORRUPT_RANK"] = "1"
    fc = _ranks_run(2, [], env)["frame_check"]
    assert fc["ranks_agree"] is False
    assert fc["rank_digests"][0] != fc["rank_digests"][1]
