#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (run in the build container).

Inputs : synthetic JPEGs made here with Pillow (bundled libjpeg-turbo) and IJG cjpeg 9.4
         (/opt/conda/bin/cjpeg, for sampling layouts Pillow cannot emit), plus copies of the
         reference's own test images (reference data/images/mug_{420,422,400}.jpg).
Goldens: per fixture, SHA-256 of (a) libjpeg 9.4 quantised coefficients and (b) libjpeg 9.4
         ISLOW native planes (oracle/libjpeg_golden.c), and (c) the reference parser's
         output (src/rocjpeg_parser.cpp built into oracle/_ref/librefparser.so).
The generated manifest is data (inputs + expected outputs); no reference source is stored.
"""
import ctypes
import hashlib
import io
import json
import os
import shutil
import struct
import subprocess
import sys
import tempfile

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
REF_IMAGES = "/root/reference/data/images"
GOLDEN_TOOL = os.path.join(ROOT, "oracle", "build", "libjpeg_golden")
CJPEG = "/opt/conda/bin/cjpeg"


def source_rgb(seed, w, h):
    """Seeded crop of the reference mug image plus N(0, 2) noise (BASELINE.md generator)."""
    base = Image.open(os.path.join(REF_IMAGES, "mug_420.jpg")).convert("RGB")
    rng = np.random.default_rng(seed)
    x0 = int(rng.integers(0, base.width - w + 1))
    y0 = int(rng.integers(0, base.height - h + 1))
    a = np.asarray(base.crop((x0, y0, x0 + w, y0 + h)), dtype=np.float32)
    a = a + rng.normal(0.0, 2.0, a.shape)
    return np.clip(a, 0, 255).astype(np.uint8)


def pillow_jpeg(rgb, **kw):
    b = io.BytesIO()
    Image.fromarray(rgb).save(b, "JPEG", **kw)
    return b.getvalue()


def cjpeg_jpeg(rgb, args, gray=False, scans=None):
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "in.pgm" if gray else "in.ppm")
        im = Image.fromarray(rgb)
        (im.convert("L") if gray else im).save(src)
        if scans is not None:  # a custom progressive scan script (cjpeg -scans)
            sp = os.path.join(td, "scans.txt")
            with open(sp, "w") as f:
                f.write(scans)
            args = args + ["-scans", sp]
        out = subprocess.run([CJPEG] + args + [src], check=True, capture_output=True).stdout
    return out


# Y's first scans in three bands, then two successive-approximation refinements of the whole
# band (the first has three producer scans -- the pipelined launch's limit)
SCANS_3BANDS = """0,1,2: 0-0, 0, 1;
0: 1-5, 0, 2;
0: 6-20, 0, 2;
0: 21-63, 0, 2;
1: 1-63, 0, 1;
2: 1-63, 0, 1;
0: 1-63, 2, 1;
0: 1-63, 1, 0;
0,1,2: 0-0, 1, 0;
1: 1-63, 1, 0;
2: 1-63, 1, 0;
"""
# non-interleaved DC scans, Y's first scans in five bands and refinements of band unions (four
# producers: the decoder falls back to level-by-level refinement)
SCANS_5BANDS = """0: 0-0, 0, 0;
1: 0-0, 0, 0;
2: 0-0, 0, 0;
0: 1-2, 0, 1;
0: 3-5, 0, 1;
0: 6-14, 0, 1;
0: 15-30, 0, 1;
0: 31-63, 0, 1;
1: 1-63, 0, 0;
2: 1-63, 0, 0;
0: 1-30, 1, 0;
0: 31-63, 1, 0;
"""


def read_coef(path):
    b = open(path, "rb").read()
    assert b[:4] == b"JCOF"
    nc = struct.unpack_from("i", b, 4)[0]
    off, h = 8, hashlib.sha256()
    dims = []
    for _ in range(nc):
        hs, vs, wb, hb = struct.unpack_from("4i", b, off)
        off += 16
        h.update(b[off:off + wb * hb * 128])
        off += wb * hb * 128
        dims.append([wb, hb])
    return h.hexdigest(), dims


def read_planes(path):
    b = open(path, "rb").read()
    assert b[:4] == b"JPLN"
    nc = struct.unpack_from("i", b, 4)[0]
    off, h = 8, hashlib.sha256()
    for _ in range(nc):
        hs, vs, pw, ph, rw, rh = struct.unpack_from("6i", b, off)
        off += 24
        a = np.frombuffer(b, np.uint8, pw * ph, off).reshape(ph, pw)
        off += pw * ph
        h.update(np.ascontiguousarray(a[:rh, :rw]).tobytes())
    return h.hexdigest()


class RefParseOut(ctypes.Structure):
    _fields_ = [
        ("ok", ctypes.c_int), ("width", ctypes.c_uint16), ("height", ctypes.c_uint16),
        ("ncomp", ctypes.c_uint8), ("scan_ncomp", ctypes.c_uint8),
        ("comp_id", ctypes.c_uint8 * 4), ("comp_h", ctypes.c_uint8 * 4), ("comp_v", ctypes.c_uint8 * 4),
        ("comp_tq", ctypes.c_uint8 * 4), ("qt_loaded", ctypes.c_uint8 * 4), ("qt", ctypes.c_uint8 * 256),
        ("ht_loaded", ctypes.c_uint8 * 2), ("dc_bits", ctypes.c_uint8 * 32), ("dc_vals", ctypes.c_uint8 * 24),
        ("ac_bits", ctypes.c_uint8 * 32), ("ac_vals", ctypes.c_uint8 * 324),
        ("scan_cs", ctypes.c_uint8 * 4), ("scan_td", ctypes.c_uint8 * 4), ("scan_ta", ctypes.c_uint8 * 4),
        ("restart_interval", ctypes.c_uint16), ("num_mcus", ctypes.c_uint32), ("slice_data_size", ctypes.c_uint32),
        ("slice_data_offset", ctypes.c_int64), ("css", ctypes.c_int),
    ]


def ref_parse(lib, data):
    o = RefParseOut()
    lib.ref_parse(data, ctypes.c_size_t(len(data)), ctypes.byref(o))
    return {
        "ok": o.ok, "width": o.width, "height": o.height, "ncomp": o.ncomp, "scan_ncomp": o.scan_ncomp,
        "restart_interval": o.restart_interval, "num_mcus": o.num_mcus, "css": o.css,
        "slice_data_size": o.slice_data_size, "slice_data_offset": o.slice_data_offset,
        "comp_hv": [[o.comp_h[i], o.comp_v[i]] for i in range(4)],
    }


def fixtures():
    """(name, bytes, note) -- sizes >= 64x64 (the reference's minimum, rocjpeg_vaapi_decoder.cpp:290)."""
    out = []
    s = 1234
    def add(name, data, note):
        out.append((name, data, note))
    add("p420_q90_ri_256x128", pillow_jpeg(source_rgb(s + 0, 256, 128), quality=90, subsampling=2, restart_marker_rows=1), "4:2:0 q90, RI = 1 MCU row")
    add("p420_q75_nori_200x150", pillow_jpeg(source_rgb(s + 1, 200, 150), quality=75, subsampling=2), "4:2:0 no DRI, ragged edges")
    add("p420_q90_odd_97x65", pillow_jpeg(source_rgb(s + 2, 97, 65), quality=90, subsampling=2, restart_marker_rows=1), "odd W and H")
    add("p422_q90_ri_192x96", pillow_jpeg(source_rgb(s + 3, 192, 96), quality=90, subsampling=1, restart_marker_rows=1), "4:2:2 (h2v1)")
    add("p422_q80_odd_65x99", pillow_jpeg(source_rgb(s + 4, 65, 99), quality=80, subsampling=1), "4:2:2 odd")
    add("p444_q95_ri_128x128", pillow_jpeg(source_rgb(s + 5, 128, 128), quality=95, subsampling=0, restart_marker_rows=1), "4:4:4")
    add("p444_q85_odd_71x67", pillow_jpeg(source_rgb(s + 6, 71, 67), quality=85, subsampling=0), "4:4:4 odd")
    add("p420_q100_ri_128x64", pillow_jpeg(source_rgb(s + 7, 128, 64), quality=100, subsampling=2, restart_marker_blocks=3), "q100, RI = 3 MCUs (not a row multiple)")
    add("p420_q10_160x96", pillow_jpeg(source_rgb(s + 8, 160, 96), quality=10, subsampling=2), "q10, sparse blocks")
    add("p420_opt_ri_176x144", pillow_jpeg(source_rgb(s + 9, 176, 144), quality=92, subsampling=2, optimize=True, restart_marker_rows=2), "optimised (non-standard) Huffman tables, RI = 2 rows")
    add("p400_q85_ri_96x72", pillow_jpeg(np.ascontiguousarray(source_rgb(s + 10, 96, 72)[:, :, 0]), quality=85, restart_marker_blocks=7), "grayscale, RI = 7 blocks")
    add("c440_q90_160x120", cjpeg_jpeg(source_rgb(s + 11, 160, 120), ["-quality", "90", "-sample", "1x2,1x1,1x1", "-restart", "1"]), "4:4:0 (h1v2) via cjpeg")
    add("c422v_q90_128x96", cjpeg_jpeg(source_rgb(s + 12, 128, 96), ["-quality", "90", "-sample", "2x2,1x2,1x2"]), "Y 2x2 / C 1x2 (mug_422 layout)")
    add("c420_q88_ri5b_144x80", cjpeg_jpeg(source_rgb(s + 13, 144, 80), ["-quality", "88", "-sample", "2x2,1x1,1x1", "-restart", "5B"]), "cjpeg 4:2:0, RI = 5 MCUs")
    add("c411_q90_128x64", cjpeg_jpeg(source_rgb(s + 14, 128, 64), ["-quality", "90", "-sample", "4x1,1x1,1x1"]), "4:1:1: reference returns JPEG_NOT_SUPPORTED")
    add("p420_prog_128x96", pillow_jpeg(source_rgb(s + 15, 128, 96), quality=90, subsampling=2, progressive=True), "progressive (SOF2): reference parser ignores SOF2")
    add("p420_q90_ri_1920x1080", pillow_jpeg(source_rgb(s + 16, 1920, 1080), quality=90, subsampling=2, restart_marker_blocks=120), "bench workload sample (C2)")
    add("p420_q90_nori_1920x1080", pillow_jpeg(source_rgb(s + 17, 1920, 1080), quality=90, subsampling=2), "1080p without DRI")
    full = pillow_jpeg(source_rgb(s + 18, 192, 128), quality=90, subsampling=2, restart_marker_rows=1)
    add("p420_trunc_192x128", full[: len(full) * 3 // 5], "truncated stream (no EOI): libjpeg zero-fill semantics")
    # progressive (SOF2), SURVEY 8f rank 2 / config C5: decoded here (the reference rejects it)
    add("pp420_q90_1920x1080", pillow_jpeg(source_rgb(s + 19, 1920, 1080), quality=90, subsampling=2, progressive=True), "progressive 4:2:0 q90 1080p (C5 sample)")
    add("pp420_opt_200x150", pillow_jpeg(source_rgb(s + 20, 200, 150), quality=85, subsampling=2, progressive=True, optimize=True), "progressive, optimised per-scan tables, ragged edges")
    add("cp444_prog_ri_136x72", cjpeg_jpeg(source_rgb(s + 21, 136, 72), ["-quality", "90", "-sample", "1x1,1x1,1x1", "-progressive", "-restart", "1"]), "progressive 4:4:4, DRI = 1 MCU row in every scan")
    add("cp422_prog_97x67", cjpeg_jpeg(source_rgb(s + 22, 97, 67), ["-quality", "80", "-sample", "2x1,1x1,1x1", "-progressive"]), "progressive 4:2:2, odd size")
    add("cp420_prog_ri3_160x112", cjpeg_jpeg(source_rgb(s + 23, 160, 112), ["-quality", "95", "-sample", "2x2,1x1,1x1", "-progressive", "-restart", "3B"]), "progressive 4:2:0, DRI = 3 MCUs")
    add("cp400_prog_120x80", cjpeg_jpeg(source_rgb(s + 24, 120, 80), ["-quality", "90", "-progressive"], gray=True), "progressive grayscale")
    add("cp440_prog_96x80", cjpeg_jpeg(source_rgb(s + 25, 96, 80), ["-quality", "90", "-sample", "1x2,1x1,1x1", "-progressive"]), "progressive 4:4:0")
    add("cp420_scans3_128x96", cjpeg_jpeg(source_rgb(s + 27, 128, 96), ["-quality", "92", "-sample", "2x2,1x1,1x1"], scans=SCANS_3BANDS), "progressive, custom script: Y first scans in 3 bands, Al 2 -> 1 -> 0")
    add("cp420_scans5_112x80", cjpeg_jpeg(source_rgb(s + 28, 112, 80), ["-quality", "90", "-sample", "2x2,1x1,1x1", "-restart", "2B"], scans=SCANS_5BANDS), "progressive, custom script: non-interleaved DC, 5 Y bands, refinements over band unions, DRI 2 MCUs")
    fullp = pillow_jpeg(source_rgb(s + 26, 192, 128), quality=90, subsampling=2, progressive=True)
    add("pp420_prog_trunc_192x128", fullp[: len(fullp) * 11 // 20], "truncated progressive stream: later scans missing, insufficient-data semantics")
    return out


def main():
    if not os.path.isfile(GOLDEN_TOOL):
        sys.exit("build oracle/ first (make -C oracle)")
    reflib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "librefparser.so"))
    os.makedirs(os.path.join(GOLD, "img"), exist_ok=True)
    manifest = {"generator": "tools/make_golden.py", "fixtures": []}
    items = fixtures()
    for m in ("420", "422", "400"):
        dst = os.path.join(GOLD, "img", f"mug_{m}.jpg")
        shutil.copyfile(os.path.join(REF_IMAGES, f"mug_{m}.jpg"), dst)
        items.append((f"mug_{m}", open(dst, "rb").read(), "reference fixture data/images/mug_%s.jpg" % m))
    with tempfile.TemporaryDirectory() as td:
        for name, data, note in items:
            path = os.path.join(GOLD, "img", name + ".jpg")
            if not name.startswith("mug_"):
                with open(path, "wb") as f:
                    f.write(data)
            ent = {"name": name, "file": f"img/{name}.jpg", "bytes": len(data), "note": note,
                   "sha256": hashlib.sha256(data).hexdigest(), "ref_parse": ref_parse(reflib, data)}
            cpath, ppath = os.path.join(td, "c.bin"), os.path.join(td, "p.bin")
            rc1 = subprocess.run([GOLDEN_TOOL, "coef", path, cpath], capture_output=True)
            rc2 = subprocess.run([GOLDEN_TOOL, "planes", path, ppath], capture_output=True)
            if rc1.returncode == 0 and rc2.returncode == 0:
                ent["libjpeg_coef_sha256"], ent["coef_dims"] = read_coef(cpath)
                ent["libjpeg_planes_sha256"] = read_planes(ppath)
            manifest["fixtures"].append(ent)
            print(name, len(data), ent["ref_parse"]["ok"], ent.get("coef_dims"))
    with open(os.path.join(GOLD, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
