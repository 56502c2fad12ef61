"""The oracle's analysis hooks (oracle_trace_pixels, oracle_trace_misses; test and profiling
infrastructure only, used by profiles/sample_pattern.py and profiles/void_bounds.py) agree with
the oracle's own statistics for the same rays: every counted sampleVolume call is one traced
letter ('m' outside every cell, 'l' located and rejected, 'A' accepted), and every 'm' one
dumped point, which no record's sample() accepts."""
import ctypes as C

import numpy as np

import irt
import oracle as O
from helpers import FRAMING


def test_trace_hooks_match_the_oracle_counts():
    cells = irt.synth_grid(2, 3, 47, terrain=4000.0)  # convert_icon terrain: voids under land
    W = 96
    S = O.OracleScene(cells)
    lut, vr = S.default_lut()
    S.set_transfunc(lut, vr)
    params = S.params(S.camera(W, W, FRAMING), accum_id=3, raygen=0)
    ys, xs = np.mgrid[0:W:3, 0:W:3]
    xy = np.ascontiguousarray(np.stack([xs.ravel(), ys.ravel()], 1).astype(np.int32))
    _, _, st = S.render_pixels(params, W, W, xy, fast=2)
    lib = O.olib()
    lib.oracle_trace_pixels.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_int, C.c_int,
                                        C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int]
    stride = 4096
    out = np.zeros(xy.shape[0] * stride, np.uint8)
    assert lib.oracle_trace_pixels(cells.ctypes.data, cells.size, C.byref(params), W, W,
                                   xy.ctypes.data, xy.shape[0], out.ctypes.data, stride, 0) == 0
    text = b"".join(bytes(r[:np.argmin(r)]) for r in out.reshape(-1, stride)).decode()
    nm, nl, na = text.count("m"), text.count("l"), text.count("A")
    assert nm + nl + na == st.locate_calls and nl + na == st.samples_found
    assert nm > 0 and na > 0
    lib.oracle_trace_misses.restype = C.c_long
    lib.oracle_trace_misses.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_int, C.c_int,
                                        C.c_void_p, C.c_int, C.c_void_p, C.c_long, C.c_int]
    pts = np.zeros(3 * nm, np.float32)
    n = lib.oracle_trace_misses(cells.ctypes.data, cells.size, C.byref(params), W, W,
                                xy.ctypes.data, xy.shape[0], pts.ctypes.data, nm, 0)
    assert n == nm
    # none of the points lies in a cell (the brute-force first-hit scan, deviceCode.cu:116-123)
    for p in pts.reshape(-1, 3)[:: max(1, nm // 50)]:
        for i in range(0, cells.size, max(1, cells.size // 400)):
            v = C.c_float()
            assert O.olib().oracle_sample(cells.ctypes.data + i * cells.itemsize, O.v3(p), C.byref(v)) == 0
