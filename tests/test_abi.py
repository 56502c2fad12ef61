"""The C-ABI library loads and exports every symbol include/*.h declares (no GPU calls)."""
import ctypes as C
import glob
import os
import re

import irt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(irt_[a-z0-9_]+)\s*\(", src):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 30
    lib = C.CDLL(irt.LIB_PATH)
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing


def test_cell_record_layout():
    assert irt.CELL_DTYPE.itemsize == 284  # icon_rt::ICONCell (ICONGrid.h:59-76)
    assert irt.CELL_DTYPE.fields["numLayers"][1] == 24
    assert irt.CELL_DTYPE.fields["height"][1] == 28
    assert irt.CELL_DTYPE.fields["value"][1] == 156


def test_errors_are_reported_not_raised():
    L = irt.lib()
    n = C.c_size_t()
    rc = L.irt_load_ic(b"/nonexistent/file.ic", -1, None, 0, C.byref(n))
    assert rc == -4 and b"cannot open" in L.irt_last_error()
    cells = irt.synth_grid(1, 0, 4)
    cells["numLayers"][3] = 40
    info = irt.VolumeInfo()
    rc = L.irt_compute_volume_info(cells.ctypes.data, cells.size, C.byref(info))
    assert rc == -3 and b"numLayers" in L.irt_last_error()


def test_context_calls_reject_a_null_context():
    """Context entry points check their handle before touching a device (no GPU needed)."""
    L = irt.lib()
    assert L.irt_set_timing_interval(None, 8) == -1
    assert b"irt_set_timing_interval" in L.irt_last_error()
    assert L.irt_reset_render_stats_total(None) == -1
    st = irt.RenderStats()
    assert L.irt_get_render_stats(None, C.byref(st)) == -1
