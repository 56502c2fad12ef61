"""The C++ multi-GPU drop-in (include/icon_rt_hip_multi.h, libicon_rt_multi.so): one process,
one context per device, the frame's 64x64 tiles dealt by cost, packed tiles sent to device 0
over an RCCL communicator from ncclCommInitAll and unpacked there.  On the one-GPU box the
communicator has one rank (device 0 sends to itself): the frames -- single and progressive
(the accum tiles stay sharded on their device across frames) -- must equal the plain
irt_render path of the same app bit for bit (that path is pinned to the oracle by
tests/test_app.py).  The integrator's call sequence is INTEGRATION.md section 6."""
import os
import subprocess

import numpy as np
import pytest

import irt
from helpers import FRAMING

pytestmark = pytest.mark.gpu
APP = os.path.join(os.path.dirname(irt.LIB_PATH), "icon_rt")


def _run(tmp_path, name, extra, size=200, limit=1):
    vp, vi, vu, fovy = FRAMING
    out = str(tmp_path / name)
    cmd = [APP, "--synth", "2", "3", "47", "--size", str(size), str(size), "--camera",
           *[str(v) for v in (*vp, *vi, *vu)], "-fovy", str(fovy), "--true-size",
           "--sample-limit", str(limit), "--dump-fb", out] + extra
    r = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    return np.fromfile(out, np.uint32).reshape(size, size), r


@pytest.mark.parametrize("limit", [1, 5])
def test_multi_one_device_equals_irt_render(tmp_path, limit):
    ref, _ = _run(tmp_path, "ref.bin", [], limit=limit)
    got, r = _run(tmp_path, "multi.bin", ["--gpus", "1"], limit=limit)
    assert "RCCL gather" in r.stderr
    assert (ref != 0).mean() > 0.3
    assert np.array_equal(got, ref), int((got != ref).sum())


def test_multi_bench_progressive_batches(tmp_path):
    """--bench through irt_multi_render with 4 chained frames per call: the last frame equals
    the single-device app's after the same frames."""
    ref, _ = _run(tmp_path, "ref.bin", ["--bench", "12", "--frames-per-launch", "4"])
    got, r = _run(tmp_path, "multi.bin", ["--gpus", "1", "--bench", "12", "--frames-per-launch", "4"])
    assert "1 device(s)" in r.stdout
    # --dump-fb is written after the bench loop: the last of the 12 benched frames
    assert np.array_equal(got, ref)
