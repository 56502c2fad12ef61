"""End to end: the C++ icon_rt app (host/icon_rt_main.cpp, the mirror of hostCode.cu
main()) renders a `.ic` file through the C ABI and writes icon_rt.png; its pixels must be
the oracle's frame (PNG rows flipped vertically, pipeline.cu:735-737)."""
import os
import struct
import subprocess
import zlib

import numpy as np
import pytest

import irt
from helpers import FRAMING

pytestmark = pytest.mark.gpu
APP = os.path.join(os.path.dirname(irt.LIB_PATH), "icon_rt")


def read_png_rgba(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat = 8, b""
    w = h = None
    while pos < len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        if typ == b"IHDR":
            w, h = struct.unpack(">II", body[:8])
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    rows = np.frombuffer(raw, np.uint8).reshape(h, 1 + 4 * w)
    assert (rows[:, 0] == 0).all()
    return rows[:, 1:].copy().view(np.uint32).reshape(h, w)


@pytest.mark.parametrize("size,true_size", [(64, True), (512, False)])
def test_icon_rt_app_png_matches_oracle(tmp_path, size, true_size):
    cells = irt.synth_grid(2, 1, 31)
    ic = str(tmp_path / "grid.ic")
    irt.save_ic(ic, cells)
    vp, vi, vu, fovy = FRAMING
    cmd = [APP, ic, "--size", str(size), str(size), "--camera",
           *[str(v) for v in (*vp, *vi, *vu)], "-fovy", str(fovy)]
    if true_size:
        cmd.append("--true-size")
    out = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert "Output: icon_rt.png" in out.stdout
    png = read_png_rgba(str(tmp_path / "icon_rt.png"))[::-1]
    # the reference divides dir_du/dir_dv by 512 whatever --size says (hostCode.cu:944-945)
    import oracle as O
    S = O.OracleScene(cells)
    lut, vr = S.default_lut()
    S.set_transfunc(lut, vr)
    div = (size, size) if true_size else (512, 512)
    p = S.params(S.camera(size, size, FRAMING, camera_div=div))
    _, fb, _ = S.render(p, size, size)
    assert np.array_equal(png, fb)
    assert (fb != 0).mean() > 0.3
