"""Shared scene/frame helpers for the test-suite (oracle on the CPU, product on the GPU)."""
import numpy as np

import irt
import oracle as O

FRAMING = irt.FRAMING_CAMERA


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def oracle_frame(cells, W, H, camera=None, accum_ids=(0,), raygen=0, lut=None, value_range=None,
                 opacity_scale=1.0, unit_distance=None, threads=0, rect=None, accel_mode=0,
                 mode=0):
    """Oracle frames with the reference's main()-style setup; returns (accum, fb, stats, scene)."""
    S = O.OracleScene(cells)
    if lut is None:
        lut, vr = S.default_lut()
        value_range = vr if value_range is None else value_range
    S.set_transfunc(lut, value_range, opacity_scale)
    cam = S.camera(W, H, camera)
    accum = np.zeros((H, W, 4), np.float32)
    fb = np.zeros((H, W), np.uint32)
    stats = []
    for aid in accum_ids:
        p = S.params(cam, accum_id=aid, raygen=raygen, unit_distance=unit_distance,
                     accel_mode=accel_mode, mode=mode)
        _, _, st = S.render(p, W, H, rect=rect, accum=accum, fb=fb, threads=threads)
        stats.append(st)
    return accum, fb, stats, S


class GpuFrame:
    """Device framebuffer (torch tensors as HBM allocations) for one context."""

    def __init__(self, ctx, W, H):
        import torch
        self.torch = torch
        self.ctx, self.W, self.H = ctx, W, H
        self.fb = torch.zeros(W * H, dtype=torch.int32, device=f"cuda:{ctx.device}")
        self.accum = torch.zeros(W * H * 4, dtype=torch.float32, device=f"cuda:{ctx.device}")

    def render(self, lp):
        s = self.torch.cuda.current_stream(self.ctx.device).cuda_stream
        self.ctx.render(lp, self.W, self.H, self.fb.data_ptr(), self.accum.data_ptr(), s)
        self.torch.cuda.synchronize(self.ctx.device)
        return self.ctx.stats()

    def host(self):
        a = self.accum.cpu().numpy().reshape(self.H, self.W, 4)
        f = self.fb.cpu().numpy().view(np.uint32).reshape(self.H, self.W)
        return a, f


def gpu_frame(cells, W, H, camera=None, accum_ids=(0,), raygen=0, lut=None, value_range=None,
              opacity_scale=1.0, device=0, unit_distance=None, accel_mode=0, mode=0):
    setup = irt.setup_frame(cells, W, H, camera=camera, raygen=raygen)
    if lut is None:
        lut, value_range = setup.lut, setup.value_range
    ctx = irt.Context(cells, device)
    ctx.set_transfunc(lut, value_range, opacity_scale)
    if mode != irt.MODE_USER_GEOM:
        ctx.build_wedge_accel(cells)
    fr = GpuFrame(ctx, W, H)
    stats = []
    lp = setup.lp
    lp.accelMode = accel_mode
    lp.mode = mode
    if unit_distance is not None:
        lp.unitDistance = unit_distance
    for aid in accum_ids:
        lp.accumID = aid
        stats.append(fr.render(lp))
    a, f = fr.host()
    return a, f, stats, ctx


def terrain_cells(seed=11, bisections=1, levels=70):
    """A synthetic scene with terrain-following record boundaries (per-column offsets, like
    ICON's HHL), a few unsorted-height records, zero-thickness records (numLayers 0, as
    convert_icon writes for numLayers % 32 == 1) and inverted records."""
    cells = irt.synth_grid(2, bisections, levels)
    rng = np.random.default_rng(seed)
    ncol = cells.size // 3
    for c in range(ncol):  # per-column terrain offset, shrinking with height
        off = np.float32(rng.uniform(0, 3000))
        for k in range(3):
            i = 3 * c + k
            nl = int(cells["numLayers"][i])
            h = cells["height"][i].astype(np.float64)
            h[:nl + 1] += off * (1.0 - (h[:nl + 1] - 6.371229e6) / 75e3)
            cells["height"][i][:nl + 1] = h[:nl + 1].astype(np.float32)
        for k in (1, 2):  # keep the stack contiguous (record k starts where k-1 ends)
            i = 3 * c + k
            cells["height"][i][0] = cells["height"][i - 1][cells["numLayers"][i - 1]]
    for i in rng.choice(cells.size, 40, replace=False):
        nl = int(cells["numLayers"][i])
        if i % 4 == 0 and nl >= 3:
            h = cells["height"][i]
            h[1], h[2] = h[2], h[1]
        elif i % 4 == 1:
            cells["numLayers"][i] = 0  # zero-thickness record
        elif i % 4 == 2:
            cells["height"][i][nl] = cells["height"][i][0] - 1.0  # inverted: never hit
    return cells


def on_radius(v, r):
    """A float32 point in direction v whose float32 |p| (sqrtf(x*x+y*y+z*z), as
    toSpherical computes it) equals r exactly, when one is found nearby."""
    v = np.asarray(v, np.float64)
    v = v / np.linalg.norm(v)
    r = np.float32(r)
    s = np.float64(r)
    p = (v * s).astype(np.float32)
    for _ in range(64):
        q = np.sqrt(np.float32(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]))
        if q == r:
            break
        s *= 1 + (float(r) - float(q)) / float(r) * 0.999 + (1e-8 if q < r else -1e-8)
        p = (v * s).astype(np.float32)
    return p


def locator_points(cells, seed, n_random=400, n_cols=80):
    """Points for point-location checks: random ones in the shell, and per sampled column
    points exactly on (and one float either side of) every record boundary -- where the
    per-cell radial bin edges sit -- at the cell centre, on edge midpoints and at a corner
    (shared triangle edges: the lower record index must win)."""
    rng = np.random.default_rng(seed)
    top = cells["height"][np.arange(cells.size), cells["numLayers"]]
    sbl, sbu = float(cells["height"][:, 0].min()), float(top.max())
    d = rng.normal(size=(n_random, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    pts = list((d * rng.uniform(sbl - 50, sbu + 50, (n_random, 1))).astype(np.float32))
    for i in rng.choice(cells.size, min(n_cols, cells.size), replace=False):
        c = cells[i]
        lat, lon = c["lat"].astype(np.float64), c["lon"].astype(np.float64)
        cd = np.stack([np.cos(lat) * np.cos(lon), np.cos(lat) * np.sin(lon), np.sin(lat)], 1)
        nl = int(c["numLayers"])
        for hh in (c["height"][0], c["height"][nl], c["height"][nl // 2]):
            for rr in (hh, np.nextafter(hh, np.float32(np.inf)), np.nextafter(hh, np.float32(0))):
                for v in (cd.mean(0), cd[0] + cd[1], cd[0]):
                    pts.append(on_radius(v, rr))
    return np.array(pts, np.float32)


# ---- the slot table (irt_common.h kSlot4), restated from a scene's header and entry bytes
_POP = np.array([bin(k).count("1") for k in range(256)], np.uint32)
_CTZ = np.array([8] + [(k & -k).bit_length() - 1 for k in range(1, 256)], np.uint32)


def slot_member(u, i, subs):
    """irt_common.h slot_member: sub-cell i of slot unit u (4 x 4 sub-cells)."""
    if subs == 4:
        return (2 * (u // 2) + (i >> 1)) * 4 + 2 * (u % 2) + (i & 1)
    return 2 * u + i if subs == 2 else u


def slot_unit_sub(s, subs):
    """irt_common.h slot_unit, slot_sub: sub-cell s's unit and its index in the unit."""
    if subs == 4:
        return (s // 8) * 2 + (s % 4) // 2, (((s // 4) & 1) << 1) | (s & 1)
    return (s >> 1, s & 1) if subs == 2 else (s, 0)


def restate_slots(hdr: np.ndarray, fat: np.ndarray, subs: int = 4) -> np.ndarray:
    """irt_common.h slot_fill over every (cell, slot unit of `subs` sub-cells, table bin), from
    the scene's header and fat-entry bytes (kBinHdrWords = 32 with 4 x 4 sub-cells, 16 words per
    entry); None when the cells' edges are more than three distinct values."""
    INF = 0x7F800000
    H = hdr.view(np.uint32).reshape(-1, 32).astype(np.int64)
    F = fat.view(np.uint32).reshape(-1, 16)
    E = H[:, :3]
    U = np.unique(E[E != INF].astype(np.uint32).view(np.float32))
    if U.size > 3:
        return None
    ne, nb, units = U.size, U.size + 1, 16 // subs
    Ef = E.astype(np.uint32).view(np.float32)
    out = np.zeros((H.shape[0], units, nb, 32), np.uint32)
    rows = np.arange(H.shape[0])
    for b in range(nb):
        k = (Ef <= U[b - 1]).sum(1) if b else np.zeros(H.shape[0], np.int64)
        up = np.float32(U[b]) if b < ne else np.float32(np.inf)
        own = (b < ne) & (k < 3) & (Ef[rows, np.minimum(k, 2)] == up)
        beg = np.where(k > 0, H[rows, 3 + k], 0)  # word 4 + k - 1
        n = H[rows, 4 + k] - beg
        lenmask = np.where(n < 8, (1 << np.clip(n, 0, 8)) - 1, 0xFF)
        nx = np.where(n > 8, n - 8, 0)
        for u in range(units):
            masks = np.zeros(H.shape[0], np.int64)
            firsts = []
            for i in range(subs):
                m8 = (H[:, 8 + slot_member(u, i, subs)] >> (8 * k)) & 0xFF & lenmask
                masks |= m8 << (8 * i)
                firsts.append(np.where(m8 > 0, _CTZ[m8], np.where(nx > 0, 8, 15)))
            # the position that is the most sub-cells' first admitted candidate (lowest on a tie)
            jU = np.full(H.shape[0], 15, np.int64)
            most = np.zeros(H.shape[0], np.int64)
            for j in range(9):
                cnt = sum((f == j).astype(np.int64) for f in firsts)
                upd = cnt > most
                jU = np.where(upd, j, jU)
                most = np.where(upd, cnt, most)
            has = jU != 15
            first = H[:, 3] + beg + jU
            out[has, u, b, :16] = F[first[has]]
            out[:, u, b, 16] = np.minimum(nx, 0xFFFFFF) | (jU << 24)
            out[:, u, b, 17] = H[:, 3] + beg
            out[:, u, b, 18] = masks
            out[:, u, b, 19] = np.where(own, np.float32(up).view(np.uint32), INF)
    return out.reshape(-1)
