import sys, time, faulthandler
sys.path.insert(0, "icon-ray-tracing_amd/python"); sys.path.insert(0, "tests")
faulthandler.dump_traceback_later(100, exit=True)
import numpy as np, irt
for name, args in [("r1b00", (1, 0, 4)), ("r2b00", (2, 0, 4)), ("r2b01", (2, 1, 4))]:
    cells = irt.synth_grid(*args)
    print(name, cells.size, flush=True)
    t = time.time()
    S = irt.DebugScene(cells); print("  host", time.time() - t, S.info.locatorFaceRes, S.info.locatorEntries, flush=True)
    t = time.time()
    c = irt.Context(cells, 0); print("  device", time.time() - t, flush=True)
    for k in irt.SCENE_ARRAYS:
        print("  ", k, np.array_equal(c.array(k), S.array(k)), flush=True)
