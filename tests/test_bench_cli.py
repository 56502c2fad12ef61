"""bench.py's rank handling (no GPU): `--gpus N` must mean N ranks.

Under a launcher (WORLD_SIZE set) --gpus has to agree with it; started directly with
--gpus N > 1, bench.py launches N ranks itself through torch.distributed.run (a child
process, never an exec) -- here, with no GPU, every RCCL rank refuses to start and the
launcher's failure is bench.py's exit status.  The GPU form of this test, which renders with
two ranks and checks the assembled frame, is tests/test_gpu_bench.py."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "2"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr


def test_gpus_spawns_ranks():
    r = _run(["--gpus", "2", "--config", "c2", "--steps", "1", "--warmup", "0",
              "--dist-backend", "nccl", "--no-cpu-baseline"])
    # the launcher started two ranks, and each refused: 2 RCCL ranks on a machine without GPUs
    assert "[launcher] 2 ranks" in r.stderr
    assert "--nproc-per-node=2" in r.stderr
    assert "2 RCCL ranks need 2 GPUs" in r.stderr
    assert r.returncode != 0
    assert r.stdout.strip() == ""
