"""The reference's own test suite, run against the drop-in library: the 13 CTest command lines of
/root/reference/samples/CMakeLists.txt:25-179 (5 output formats, the perf and batched samples, 6
crop variants with -crop 960,540,2880,1620), each on a directory holding the reference's three
4K fixtures (tests/golden/img/mug_{420,422,400}.jpg, data/images/ in the reference).  The
samples are this repository's restatement (tests/c/rj_samples.cpp: their command line, their
destination sizing and their -o dump), linked with -lrocjpeg so they load librocjpeg.so.0 by its
SONAME.  Pass criterion as in the reference: exit code 0.  On top of it, every jpegdecode line
and the batched crop line run again with -o, and each dumped file must equal the oracle's
output put through the same dump rule (samples/rocjpeg_samples_utils.h:479-628)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

BIN = os.path.join(O.ROOT, "tests", "c")
CROP = "960,540,2880,1620"
# (name, sample, extra args) -- samples/CMakeLists.txt:25-179, in file order
CTESTS = [
    ("jpeg-decode-fmt-native", "jpegdecode", []),
    ("jpeg-decode-fmt-yuv-planar", "jpegdecode", ["-fmt", "yuv_planar"]),
    ("jpeg-decode-fmt-y", "jpegdecode", ["-fmt", "y"]),
    ("jpeg-decode-fmt-rgb", "jpegdecode", ["-fmt", "rgb"]),
    ("jpeg-decode-fmt-rgb-planar", "jpegdecode", ["-fmt", "rgb_planar"]),
    ("jpeg-decode-perf-fmt-native", "jpegdecodeperf", []),
    ("jpeg-decode-batch-fmt-native", "jpegdecodebatched", []),
    ("jpeg-decode-crop-fmt-native", "jpegdecode", ["-crop", CROP]),
    ("jpeg-decode-crop-fmt-yuv-planar", "jpegdecode", ["-fmt", "yuv_planar", "-crop", CROP]),
    ("jpeg-decode-crop-fmt-y", "jpegdecode", ["-fmt", "y", "-crop", CROP]),
    ("jpeg-decode-crop-fmt-rgb", "jpegdecode", ["-fmt", "rgb", "-crop", CROP]),
    ("jpeg-decode-crop-fmt-rgb-planar", "jpegdecode", ["-fmt", "rgb_planar", "-crop", CROP]),
    ("jpeg-decode-crop-batch-fmt-native", "jpegdecodebatched", ["-crop", CROP]),
]
FMT = {"native": 0, "yuv_planar": 1, "y": 2, "rgb": 3, "rgb_planar": 4}
CSS = {0: "444", 1: "440", 2: "422", 3: "420", 5: "400"}  # RocJpegChromaSubsampling (api/rocjpeg.h:86-94)


@pytest.fixture(scope="module")
def images(tmp_path_factory):
    d = tmp_path_factory.mktemp("data_images")
    for n in ("mug_420.jpg", "mug_422.jpg", "mug_400.jpg"):
        shutil.copy(os.path.join(O.GOLD, "img", n), d / n)
    return d


def run(sample, args, timeout=120):
    exe = os.path.join(BIN, sample + "_rj")
    if not os.access(exe, os.X_OK):
        pytest.fail(f"{exe} not built (make -C tests/c; __graft_entry__.build() does it)")
    return subprocess.run([exe] + args, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("name,sample,extra", CTESTS, ids=[c[0] for c in CTESTS])
def test_reference_ctest_line(images, name, sample, extra):
    r = run(sample, ["-i", str(images)] + extra)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])


def dest(fmt, css, W, H, crop):
    """(visible w, h, [(pitch, alloc rows, dump bytes, dump rows)] per channel): the samples'
    sizing (rocjpeg_samples_utils.h:318-399) and dump (:479-628), restated."""
    l, t, r, b = crop
    rw, rh = r - l, b - t
    roi = rw > 0 and rh > 0 and rw <= W[0] and rh <= H[0]
    w, h = (rw, rh) if roi else (W[0], H[0])
    if fmt == 0:
        ch = {"444": [(w, h, w, h)] * 3, "440": [(w, h, w, h)] + [(w, h >> 1, w, h >> 1)] * 2,
              "422": [(2 * w, h, 2 * w, h)], "420": [(w, h, w, h), (w, h >> 1, w, h >> 1)],
              "400": [(w, h, w, h)]}[css]
    elif fmt == 1:
        if css == "400":
            ch = [(w, h, w, h)]
        else:
            hs, vs = css in ("422", "420"), css in ("440", "420")
            ch = [(w if roi else W[c], h if roi else H[c], w if c == 0 or not hs else w >> 1,
                   h if c == 0 or not vs else h >> 1) for c in range(3)]
    elif fmt == 2:
        ch = [(w, h, w, h)]
    elif fmt == 3:
        ch = [(3 * w, h, 3 * w, h)]
    else:
        ch = [(w, h, w, h)] * 3
    return w, h, ch


def expected_dump(data, fmt, crop):
    from rocjpeg_amd import JpegStream
    info = JpegStream(data).info()
    css = CSS[int(info["subsampling"])]
    w, h, ch = dest(fmt, css, info["widths"], info["heights"], crop)
    st, bufs = O.oracle_decode(data, fmt, [(rows, pitch) for pitch, rows, _, _ in ch], crop)
    assert st == 0
    out = b"".join(np.ascontiguousarray(buf[:dr, :dw]).tobytes() for buf, (_, _, dw, dr) in zip(bufs, ch))
    return w, h, css, out


def out_name(path, fmt, css, w, h):
    base = os.path.splitext(os.path.basename(path))[0]
    desc, ext = {0: ({"444": "444", "440": "440", "422": "422_yuyv", "420": "nv12", "400": "400"}[css], "yuv"),
                 1: ("planar", "yuv"), 2: ("400", "yuv"), 3: ("packed", "rgb"), 4: ("planar", "rgb")}[fmt]
    return f"{base}_{w}x{h}_{desc}.{ext}"


DUMPS = [c for c in CTESTS if c[1] != "jpegdecodeperf"]


@pytest.mark.parametrize("name,sample,extra", DUMPS, ids=[c[0] for c in DUMPS])
def test_reference_ctest_line_output_matches_oracle(images, tmp_path, name, sample, extra):
    """The same command line with -o <dir>: every dumped image equals the oracle's bytes."""
    r = run(sample, ["-i", str(images), "-o", str(tmp_path)] + extra)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    fmt = FMT[extra[extra.index("-fmt") + 1]] if "-fmt" in extra else 0
    crop = tuple(int(x) for x in extra[extra.index("-crop") + 1].split(",")) if "-crop" in extra else (0, 0, 0, 0)
    for img in sorted(os.listdir(images)):
        p = os.path.join(images, img)
        with open(p, "rb") as f:
            data = f.read()
        w, h, css, want = expected_dump(data, fmt, crop)
        got_path = tmp_path / out_name(p, fmt, css, w, h)
        assert got_path.exists(), (got_path, sorted(os.listdir(tmp_path)))
        got = got_path.read_bytes()
        assert len(got) == len(want), (img, len(got), len(want))
        if got != want:
            a, b = np.frombuffer(got, np.uint8), np.frombuffer(want, np.uint8)
            k = int(np.flatnonzero(a != b)[0])
            pytest.fail(f"{img}: first differing byte {k} of {len(want)}: {a[k]} vs {b[k]}")


def test_samples_load_the_reference_soname():
    """The restated samples are linked like a rocJPEG application: DT_NEEDED librocjpeg.so.0,
    resolved to this repository's library (the reference's SONAME, CMakeLists.txt:148,155)."""
    exe = os.path.join(BIN, "jpegdecode_rj")
    r = subprocess.run(["readelf", "-d", exe], capture_output=True, text=True)
    assert "librocjpeg.so.0" in r.stdout
    r = subprocess.run(["ldd", exe], capture_output=True, text=True)
    line = next(x for x in r.stdout.splitlines() if "librocjpeg.so.0" in x)
    assert os.path.join("rocjpeg_amd", "librocjpeg.so.0") in line, line
