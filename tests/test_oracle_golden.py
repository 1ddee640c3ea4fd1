"""The oracle is pinned before it is trusted (CPU, no GPU):
 * coefficients and ISLOW planes vs IJG libjpeg 9.4 dumps (hashes in tests/golden/manifest.json,
   produced by tools/make_golden.py + oracle/libjpeg_golden.c);
 * parser fields vs the reference's own parser (src/rocjpeg_parser.cpp) as recorded in the
   manifest, and -- when oracle/_ref is built -- live against librefparser.so.
"""
import ctypes
import hashlib
import os

import numpy as np
import pytest

from tests import oracle_lib as O

FIX = O.manifest()
DECODABLE = [f for f in FIX if "libjpeg_coef_sha256" in f]


@pytest.mark.parametrize("ent", DECODABLE, ids=[f["name"] for f in DECODABLE])
def test_coefficients_match_libjpeg(ent):
    data = O.fixture_bytes(ent)
    assert hashlib.sha256(data).hexdigest() == ent["sha256"]
    st, coefs, dims = O.decode_coefs(data)
    assert st == 0
    assert [list(d) for d in dims] == ent["coef_dims"]
    assert O.sha(coefs) == ent["libjpeg_coef_sha256"]


@pytest.mark.parametrize("ent", DECODABLE, ids=[f["name"] for f in DECODABLE])
def test_planes_match_libjpeg(ent):
    data = O.fixture_bytes(ent)
    st, planes, dims = O.decode_planes(data)
    assert st == 0
    h = hashlib.sha256()
    # libjpeg IDCTs only the blocks inside width/height_in_blocks; compare that region
    pr = ent["ref_parse"] if ent["ref_parse"]["ok"] else O.frame_info(data)
    hmax = max(hv[0] for hv in pr["comp_hv"][: pr["ncomp"]])
    vmax = max(hv[1] for hv in pr["comp_hv"][: pr["ncomp"]])
    for c, p in enumerate(planes):
        hc, vc = pr["comp_hv"][c]
        if pr["ncomp"] == 1:
            hc = vc = hmax = vmax = 1
        cw = -(-pr["width"] * hc // hmax)
        ch = -(-pr["height"] * vc // vmax)
        rw, rh = -(-cw // 8) * 8, -(-ch // 8) * 8
        h.update(np.ascontiguousarray(p[:rh, :rw]).tobytes())
    assert h.hexdigest() == ent["libjpeg_planes_sha256"]


class OjParams(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint16), ("height", ctypes.c_uint16), ("precision", ctypes.c_uint8),
                ("ncomp", ctypes.c_uint8), ("comp", ctypes.c_uint8 * 16), ("qt_loaded", ctypes.c_uint8 * 4),
                ("qt_zz", ctypes.c_uint8 * 256), ("ht_loaded", ctypes.c_uint8 * 2), ("ht", ctypes.c_uint8 * 412),
                ("scan_ncomp", ctypes.c_uint8), ("scomp", ctypes.c_uint8 * 12), ("restart_interval", ctypes.c_uint16),
                ("num_mcus", ctypes.c_uint32), ("ecs_offset", ctypes.c_uint32), ("ecs_size", ctypes.c_uint32),
                ("css", ctypes.c_int), ("sof_seen", ctypes.c_uint8)]


@pytest.mark.parametrize("ent", FIX, ids=[f["name"] for f in FIX])
def test_oracle_parser_matches_reference_parser(ent):
    data = O.fixture_bytes(ent)
    p = OjParams()
    ok = O.oracle().oj_parse(data, ctypes.c_size_t(len(data)), ctypes.byref(p))
    r = ent["ref_parse"]
    assert ok == r["ok"]
    if not ok:
        return
    assert (p.width, p.height, p.ncomp, p.scan_ncomp) == (r["width"], r["height"], r["ncomp"], r["scan_ncomp"])
    assert (p.restart_interval, p.num_mcus, p.css) == (r["restart_interval"], r["num_mcus"], r["css"])
    assert (p.ecs_offset, p.ecs_size) == (r["slice_data_offset"], r["slice_data_size"]) or (
        # truncated stream: the reference's FFD9 scan runs one byte past the buffer (rocjpeg_parser.cpp:407)
        "trunc" in ent["name"] and p.ecs_size + 1 == r["slice_data_size"])


def test_cvt_u8_semantics():
    f = O.oracle().oj_cvt_u8
    assert [f(x) for x in (0.5, 1.5, 2.5, -0.3, 255.6, 254.5, -1e9, 1e9)] == [0, 2, 2, 0, 255, 254, 0, 255]
    assert f(float("nan")) == 0


def test_csc_gray_is_identity_within_rounding():
    rgb = (ctypes.c_uint8 * 3)()
    for y in (0, 17, 128, 255):
        O.oracle().oj_csc_pixel(y, 128, 128, rgb)
        assert list(rgb) == [y, y, y]


def test_crafted_refine_overshoot_matches_libjpeg_turbo():
    """The Se = 63 refinement overshoot of tests/jpeg_craft.py: the oracle's coefficients put the
    new coefficient at natural index 63 (libjpeg jdphuff.c natural_order[64] == 63), and its
    grayscale ISLOW plane equals Pillow's libjpeg-turbo decode of the same bytes (grayscale: no
    upsampling or colour conversion in between)."""
    import io

    PIL = pytest.importorskip("PIL.Image")
    from tests import jpeg_craft as C

    data = C.prog_gray_refine_overshoot(64, 64)
    st, coefs, dims = O.decode_coefs(data)
    assert st == 0 and dims == [(8, 8)]
    blocks = coefs.reshape(-1, 64)
    for b, blk in enumerate(blocks):
        assert set(np.nonzero(blk)[0]) == {1, 19, 63}
        assert blk[63] == (1 if (b >> 2) & 1 else -1)
        assert blk[19] == (1 if b & 1 else -1)
    st, planes, _ = O.decode_planes(data)
    assert st == 0
    assert np.array_equal(np.asarray(PIL.open(io.BytesIO(data))), planes[0])


def test_remapped_pair_codes_the_same_coefficients():
    """The crafted streams of test_decode_gpu.test_same_tables_other_component_map: equal
    tables, other component-to-table map, same coefficients (checked by the oracle)."""
    from tests.test_decode_gpu import remapped_pair
    A, B = remapped_pair()
    sa, ca, _ = O.decode_coefs(A)
    sb, cb, _ = O.decode_coefs(B)
    assert sa == sb == 0 and np.array_equal(ca, cb)
    ia, ib = A.index(b"\xff\xda"), B.index(b"\xff\xda")
    assert A[:ia] == B[:ib]  # identical headers up to the SOS (DQT, SOF, DHT)
