"""The drop-in boundary exercised from plain C (tests/c/jpegdecode_c.c: gcc, include/rocjpeg.h,
librocjpeg_amd.so and the HIP runtime only -- no Python, no torch), following the reference
samples' call sequence (samples/jpegDecode/jpegdecode.cpp:72-163 for one file,
samples/jpegDecodeBatched/jpegdecodebatched.cpp:82-194 for several).  Output bytes must equal
the oracle's for every channel."""
import os
import subprocess

import numpy as np
import pytest

import rocjpeg_amd as R
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

EXE = os.path.join(O.ROOT, "tests", "c", "jpegdecode_c")
NAMES = ["p420_q90_ri_256x128", "mug_422", "pp420_opt_200x150", "cp444_prog_ri_136x72", "cp422_prog_97x67"]
FORMATS = list(R.OutputFormat)


def _expected(data, fmt):
    from tests import gpu_util as G
    s = R.JpegStream(data)
    info = s.info()
    shapes = G.channel_shapes(fmt, info["subsampling"], info["widths"], info["heights"])
    st, want = O.oracle_decode(data, int(fmt), shapes)
    assert st == 0
    return b"".join(np.ascontiguousarray(w).tobytes() for w in want)


@pytest.mark.parametrize("fmt", FORMATS, ids=[f.name for f in FORMATS])
def test_c_caller_single_and_batched(tmp_path, fmt):
    if not os.access(EXE, os.X_OK):
        pytest.fail(f"{EXE} not built (make -C tests/c; __graft_entry__.build() does it)")
    by = {f["name"]: f for f in O.manifest()}
    files, want = [], []
    for n in NAMES:
        d = O.fixture_bytes(by[n])
        p = tmp_path / f"{n}.jpg"
        p.write_bytes(d)
        files.append(str(p))
        want.append(_expected(d, fmt))
    # one file (rocJpegDecode), then all of them (rocJpegDecodeBatched)
    for sel in ([files[0]], files):
        out = tmp_path / "out.raw"
        r = subprocess.run([EXE, str(int(fmt)), str(out)] + sel, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        exp = b"".join(want[:len(sel)])
        assert out.read_bytes() == exp
