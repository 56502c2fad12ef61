"""The C-ABI library loads and exports every symbol include/*.h declares (no GPU calls)."""
import ctypes as C
import glob
import os
import re

import irt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# header -> the library that exports it (icon_rt_hip_multi.h: the RCCL multi-GPU layer,
# a library of its own so that the product library never links a second RCCL into torch)
LIBS = {"icon_rt_hip_multi.h": "libicon_rt_multi.so"}


def declared_functions(header=None):
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        if header is not None and os.path.basename(h) != header:
            continue
        if header is None and os.path.basename(h) in LIBS:
            continue
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


def test_multi_library_exports_every_declared_symbol():
    """libicon_rt_multi.so (one process, N devices, RCCL) loads without a GPU and exports
    include/icon_rt_hip_multi.h; it rejects a null handle before touching a device."""
    for header, so in LIBS.items():
        names = declared_functions(header)
        assert len(names) >= 8
        lib = C.CDLL(os.path.join(os.path.dirname(irt.LIB_PATH), so))
        missing = [n for n in sorted(names) if not hasattr(lib, n)]
        assert not missing, missing
    lib.irt_multi_last_error.restype = C.c_char_p
    assert lib.irt_multi_set_transfunc(None, None, 0, irt.box1(0, 1), C.c_float(1.0)) == -1
    assert b"null handle" in lib.irt_multi_last_error()
    assert lib.irt_multi_num_devices(None) == 0


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
