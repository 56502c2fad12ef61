"""The scene build on the GPU (csrc/irt_build.hip) against its host restatement
(host/irt_scene.cpp), byte for byte: cell headers with radial bins and sub-cell masks, fat
candidate entries, height/value blocks, the sphere table.  Both build from the same
irt_build.h functions; this pins that the device compiles them to the same arithmetic.

Also: streamed creation (irt_create_begin / _append / _end, irt_create_synth,
irt_create_from_file) builds the same scene as one irt_create call.
"""
import numpy as np
import pytest

import irt
from helpers import terrain_cells

pytestmark = pytest.mark.gpu


def _scenes():
    out = {
        "r1b00_l4": irt.synth_grid(1, 0, 4),           # cone-mode triangles (> 15 degrees)
        "ico12": irt.synth_grid(1, 0, 4)[:12],          # --num-cells 12
        "r2b02_l90": irt.synth_grid(2, 2, 90),
        "r2b03_l47_noise": irt.synth_grid(2, 3, 47, noise=0.2),
        "terrain": terrain_cells(11),                   # spheres, unsorted, inverted records
        "filtered": irt.filter_cells(irt.synth_grid(2, 2, 20), (-30, 60), (-90, 45)),
        "empty": irt.synth_grid(1, 0, 4)[:0],
    }
    # every record in one column (a cell with more entries than the device edge search
    # keeps in registers: the host computes that cell's edges)
    deep = irt.synth_grid(2, 4, 31)
    deep = np.repeat(deep[:1], 300)
    for k in range(300):
        deep["height"][k] += np.float32(1000.0 * k)
    out["one_deep_column"] = deep
    return out


SCENES = _scenes()


def _compare(ctx, scene, label):
    for name in irt.SCENE_ARRAYS:
        a, b = ctx.array(name), scene.array(name)
        assert a.size == b.size, f"{label} {name}: {a.size} vs {b.size} bytes"
        if not np.array_equal(a, b):
            w = np.nonzero(a.view(np.uint8) != b.view(np.uint8))[0]
            raise AssertionError(f"{label} {name}: {w.size} bytes differ, first at {w[0]}")
    assert ctx.info.locatorFaceRes == scene.info.locatorFaceRes
    assert ctx.info.locatorEntries == scene.info.locatorEntries


@pytest.mark.parametrize("name", sorted(SCENES))
def test_device_build_matches_host_restatement(name):
    cells = SCENES[name]
    ctx = irt.Context(cells, 0)
    scene = irt.DebugScene(cells)
    _compare(ctx, scene, name)
    # the volume facts come from the host fold either way
    for f in ("bounds", "sphericalBounds", "dataRange"):
        assert bytes(getattr(ctx.info, f)) == bytes(getattr(scene.info, f)), f
    ctx.close()
    scene.close()


def test_streamed_creation_builds_the_same_scene(tmp_path):
    cells = irt.synth_grid(2, 3, 90)
    whole = irt.Context(cells, 0)
    # uneven chunks, one of them splitting a column
    cuts = [0, 7, 1000, 1001, 5000, cells.size]
    parts = (cells[a:b] for a, b in zip(cuts[:-1], cuts[1:]))
    streamed = irt.Context.streamed(parts, cells.size, 0)
    synth = irt.Context.synth(2, 3, 90, 0)
    irt.save_ic(str(tmp_path / "g.ic"), cells)
    loaded = irt.Context.from_file(str(tmp_path / "g.ic"), -1, 0)
    truncated = irt.Context.from_file(str(tmp_path / "g.ic"), 2000, 0)
    ref = irt.Context(cells[:2000], 0)
    for name in irt.SCENE_ARRAYS:
        a = whole.array(name)
        for other in (streamed, synth, loaded):
            assert np.array_equal(a, other.array(name)), name
        assert np.array_equal(ref.array(name), truncated.array(name)), name
    for other in (streamed, synth, loaded):
        assert bytes(other.info) [:-8] == bytes(whole.info)[:-8]  # all but deviceBytes
    for c in (whole, streamed, synth, loaded, truncated, ref):
        c.close()


def test_streamed_creation_rejects_bad_input():
    cells = irt.synth_grid(2, 0, 31)
    with pytest.raises(irt.IrtError):
        irt.Context.streamed([cells[:5]], cells.size, 0)  # fewer than announced
    bad = cells.copy()
    bad["numLayers"][3] = 40
    with pytest.raises(irt.IrtError):
        irt.Context.streamed([bad], bad.size, 0)
