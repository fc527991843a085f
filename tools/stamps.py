"""Per-phase cycle breakdown of the long-segment PC block (diagnostic build with -DRSP_STAMPS).
Run: RSP_LIB=.../librsp_stamps.so python tools/stamps.py"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "radar-signal-process_amd"))
import torch  # noqa: E402
from rsp import _capi, presets, synth  # noqa: E402
from rsp.engine import Engine  # noqa: E402

spec = presets.v2(128, 4096)
eng = Engine(spec)
B = int(os.environ.get("CPIS", "16"))
echo = synth.echo_torch(spec, B, seed=7)
out = torch.empty((B, 128, 4096), dtype=torch.complex64, device="cuda")
for it in range(3):
    eng.pc_dev(echo, out)
torch.cuda.synchronize()
lib = _capi.load_library()
nb = B * 128
buf = (C.c_ulonglong * (8 * 8192))()
lib.rsp_debug_stamps.argtypes = [C.c_void_p, C.c_int]
assert lib.rsp_debug_stamps(buf, 8192) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 8)[:nb, :6].astype(np.int64)
names = ["load", "fft1", "H", "fft2", "store"]
d = np.diff(st, axis=1)
tot = st[:, 5] - st[:, 0]
print("blocks", nb, "total cycles median %d p10 %d p90 %d" % tuple(np.percentile(tot, [50, 10, 90])))
for i, n in enumerate(names):
    print("  %-6s median %7d  p10 %7d  p90 %7d  share %.2f" % ((n,) + tuple(np.percentile(d[:, i], [50, 10, 90])) + (np.median(d[:, i]) / np.median(tot),)))
