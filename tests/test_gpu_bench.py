"""bench.py's multi-rank run on the GPU box: `bench.py --gpus 2` started directly (no
launcher) must run two ranks, report n_gpus == 2, time ms/step with the gather and unpack
inside the timed region, and assemble a frame equal to a single-context render of the same
accumID sequence (--verify, rank 0).  Both ranks share the box's one GPU, so the collectives
are gloo's (host-staged); the RCCL form of the same loop is
tests/test_gpu_distributed.py::test_rccl_process_group_frame_pipeline.  The seeds depend only
on (accumID, W, H, x, y) (deviceCode.cu:288-289), so the split cannot change a pixel."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, timeout=300):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [l for l in r.stdout.splitlines() if l.strip().startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


@pytest.mark.parametrize("mode", ["progressive", "frame"])
def test_bench_gpus2_spawns_two_ranks(mode):
    r, out = _bench(["--gpus", "2", "--dist-backend", "gloo", "--config", "c2", "--steps", "3",
                     "--warmup", "1", "--mode", mode, "--verify", "--no-cpu-baseline"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert out is not None, r.stderr[-3000:]
    assert out["n_gpus"] == 2
    assert out["verify"]["mismatches"] == 0
    assert out["verify"]["pixels"] == 512 * 512
    assert out["ms_per_step"] > 0 and out["value"] > 0
    assert out["config"]["chain_timeouts"] == 0
    assert "gather" in out["config"]["parallelism"]
    # the whole job's rays: 2 ranks x batch 8 frames per step (progressive), 8 split (frame)
    frames = 16 if mode == "progressive" else 8
    assert out["frames_per_launch"] == frames
    assert abs(out["value"] - 512 * 512 * frames / (out["ms_per_step"] / 1e3) / 1e6) < 0.01 * out["value"]
    # exactly one JSON line on stdout (the launcher relays rank 0's)
    assert len([l for l in r.stdout.splitlines() if l.strip()]) == 1


@pytest.mark.parametrize("n", [4, 8])
def test_bench_more_ranks_progressive(n):
    """The driver's scaling run at N = 4 and 8 rehearsed on the one GPU (gloo): the deal of the
    frame's 64x64 tiles over N ranks, the launcher, and rank 0's assembled frame against a
    single-context render (--verify)."""
    r, out = _bench(["--gpus", str(n), "--dist-backend", "gloo", "--config", "c2", "--steps", "2",
                     "--warmup", "1", "--verify", "--no-cpu-baseline"], timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    assert out is not None and out["n_gpus"] == n, r.stderr[-3000:]
    assert out["verify"]["mismatches"] == 0 and out["config"]["chain_timeouts"] == 0
    assert out["frames_per_launch"] == 8 * n


def test_bench_secondary_block():
    """The primary line carries the secondary configs' measurements (C2 primary, C3t second)."""
    r, out = _bench(["--config", "c2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                     "--no-single-compare", "--secondary", "c3t", "--secondary-steps", "2"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert out["n_gpus"] == 1 and out["config"]["name"] == "c2"
    s = out["secondary"]["c3t"]
    assert "error" not in s, s
    assert s["value"] > 0 and s["ms_per_frame"] > 0 and s["roofline"]["frac"] > 0
    assert s["chain_timeouts"] == 0
