"""Loading helpers for tests/golden/*.npz (made by tests/golden/make_golden.py)."""
import glob
import os

import numpy as np

import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FRAME_FIXTURES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "f*.npz")))


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["cells"] = np.ascontiguousarray(d["cells"]).view(O.CELL_DTYPE).ravel()
    return d


def oracle_scene(d):
    """An OracleScene configured exactly like the fixture (its own LUT and value range)."""
    S = O.OracleScene(d["cells"])
    S.set_transfunc(d["lut"], tuple(d["value_range"]), float(d["opacity_scale"]))
    return S


def params(S, d, accum_id):
    c = d["camera12"]
    return S.params((c[0:3], c[3:6], c[6:9], c[9:12]), accum_id=int(accum_id),
                    raygen=int(d["raygen"]), unit_distance=float(d["unit_distance"]),
                    accel_mode=int(d.get("accel_mode", 0)), mode=int(d.get("mode", 0)))
