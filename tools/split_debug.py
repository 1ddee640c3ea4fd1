"""Development: decode the damaged variants of the 1080p RI fixture one at a time with the lean
split launch; print the MCU rows that differ from the oracle and those intervals' pieces."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("RJ_DEBUG_K1_PIECES", "1")
import numpy as np  # noqa: E402
import rocjpeg_amd as R  # noqa: E402
from tests import oracle_lib as O, gpu_util as G  # noqa: E402
from tests.test_decode_gpu import _variants, run_both  # noqa: E402

ent = [e for e in O.manifest() if e["name"] == "p420_q90_ri_1920x1080"][0]
G.torch()
dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
for name, data in _variants(O.fixture_bytes(ent)).items():
    print("=== variant", name, flush=True)
    st, ost, got, want = run_both(dec, data, R.OutputFormat.RGB)
    g, w = got[0], want[0]
    rows = sorted({int(r) // 16 for r in np.nonzero((g != w).any(axis=1))[0]})
    print("status", st, ost, "bad MCU rows", rows, flush=True)
    for mr in rows[:3]:
        cols = np.nonzero((g[mr * 16:mr * 16 + 16] != w[mr * 16:mr * 16 + 16]).any(axis=0))[0]
        print(f"  row {mr}: bad MCU cols {sorted({int(c) // 48 for c in cols})[:20]}", flush=True)
    for mr in rows[:1]:
        for mc in [38, 39, 40, 41, 49, 50, 51]:
            y, x = mr * 16, mc * 48
            print(f"  ({mr},{mc}) got {g[y, x:x + 12].tolist()} / {g[y + 8, x + 24:x + 36].tolist()}  want {w[y, x:x + 12].tolist()} / {w[y + 8, x + 24:x + 36].tolist()}", flush=True)
