"""The slot table's invariant, on the host build (CPU; irt_common.h kSlot4, the restatement in
helpers.restate_slots): a scene gets a table when its cells' radial edges are, all together, at
most three values U0 < U1 < U2.  Then every cell's edges are some of the U, so for any radius r
of table bin b = (U_{b-1}, U_b] the cell's own bin is the same, and slot (cell, s, b) must
give exactly what the cell header gives the wave-wide scan (Tracer::locate_wave) for every such
r: the admitted-candidate count, the list start, the sub-cell mask, the first admitted
candidate's fat entry, and whether r sits on the cell's own bin edge (the second pass).

Checked here, slot by slot, against the header path at the table bin's ends and middle, on flat
grids and on a lat/lon-filtered grid whose border cells hold fewer records and fewer edges.
The GPU tests check the device-built table against the same restatement and the frames
through it (tests/test_gpu_slots.py).
"""
import numpy as np
import pytest

import irt
from helpers import restate_slots, slot_unit_sub

INF = np.float32(np.inf)


def header_path(H, F, s, r):
    """Tracer::locate_wave's first step from the cell header H (32 u32) for a sample at radius r
    in sub-cell s: (c, list start, m8, first admitted entry or None, on the cell's bin edge)."""
    e = H[:3].astype(np.uint32).view(np.float32)
    b = int((e < r).sum())  # bin_of
    beg = int(H[4 + b - 1]) if b else 0
    n = int(H[4 + b]) - beg
    m8 = (int(H[8 + s]) >> (8 * b)) & 0xFF & ((1 << n) - 1 if n < 8 else 0xFF)
    c = bin(m8).count("1") + max(n - 8, 0)
    first = None
    if c:
        j = (m8 & -m8).bit_length() - 1 if m8 else 8
        first = F[int(H[3]) + beg + j]
    edge = b < 3 and r == e[b]
    return c, int(H[3]) + beg, m8, first, bool(edge)


@pytest.mark.parametrize("subs", [4, 2, 1])
@pytest.mark.parametrize("scene", ["r2b02_l90", "r2b03_l20", "r2b02_l47_noise", "filtered"])
def test_slots_equal_the_header_path(scene, subs):
    cells = {"r2b02_l90": lambda: irt.synth_grid(2, 2, 90),
             "r2b03_l20": lambda: irt.synth_grid(2, 3, 20),
             "r2b02_l47_noise": lambda: irt.synth_grid(2, 2, 47, noise=0.2),
             "filtered": lambda: irt.filter_cells(irt.synth_grid(2, 3, 40), (-30, 60), (-90, 45))}[scene]()
    D = irt.DebugScene(cells)
    hdr, fat = D.array("bin_hdr"), D.array("fat")
    slots = restate_slots(hdr, fat, subs)
    assert slots is not None
    H = hdr.view(np.uint32).reshape(-1, 32)
    F = fat.view(np.uint32).reshape(-1, 16)
    E = H[:, :3]
    U = np.unique(E[E != 0x7F800000].view(np.float32))
    nb = U.size + 1
    S = slots.reshape(H.shape[0], 16 // subs, nb, 32)
    rng = np.random.default_rng(5)
    cellsWith = np.nonzero(H[:, 7])[0]
    pick = np.concatenate([cellsWith[:40], rng.choice(cellsWith, min(200, cellsWith.size), replace=False)])
    checked = edges = copies = 0
    for cell in pick:
        for b in range(nb):
            lo = U[b - 1] if b else np.float32(6.0e6)
            hi = U[b] if b < U.size else np.float32(6.5e6)
            radii = [np.nextafter(lo, INF), np.float32((np.float64(lo) + hi) / 2)]
            if b < U.size:
                radii.append(hi)  # the table bin's upper edge belongs to it (bin_of: e < r)
            for s in (0, 5, 10, 15, 3, 12):
                u, i = slot_unit_sub(s, subs)
                slot = S[cell, u, b]
                for r in radii:
                    c, start, m8, first, edge = header_path(H[cell], F, s, np.float32(r))
                    # the kernel's reading of the slot (Tracer::locate_wave, OPT_SLOT)
                    sm8 = (int(slot[18]) >> (8 * i)) & 0xFF
                    j = (sm8 & -sm8).bit_length() - 1 if sm8 else 8
                    sc = bin(sm8).count("1") + (int(slot[16]) & 0xFFFFFF)
                    assert sc == c and slot[17] == start and sm8 == m8, (cell, s, b, r)
                    if c:
                        got = slot[:16] if j == int(slot[16]) >> 24 else F[int(slot[17]) + j]
                        assert np.array_equal(got, first), (cell, s, b, r)
                        copies += j == int(slot[16]) >> 24
                    own = slot[19] != 0x7F800000 and np.float32(r) == slot[19:20].view(np.float32)[0]
                    assert own == edge, (cell, s, b, r)
                    edges += edge
                    checked += 1
    assert checked > 1000
    assert copies > checked // 3  # the slot's copy serves most samples
    if scene != "r2b03_l20":  # one level band per record there: no cell edges
        assert edges > 0  # samples exactly on a cell's own edge were among them
    D.close()
