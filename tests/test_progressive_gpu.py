"""Parity of the progressive (SOF2) decode path -- K0 destuff of every scan's intervals, K1p
(rj_prog.hip) into dense coefficients, K2 over them -- with the CPU oracle, byte for byte
(oracle/jpeg_oracle.c decode_progressive, pinned against libjpeg 9.4's coefficients and planes
for every fixture used here, tests/test_oracle_golden.py).

The reference cannot decode these streams at all (its parser handles SOF0 only,
src/rocjpeg_parser.cpp:74-104); SURVEY.md 8f rank 2 / BASELINE config C5."""
import numpy as np
import pytest

import rocjpeg_amd as R
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu


def is_progressive(data):
    pos = 2
    while pos + 4 <= len(data):
        while data[pos] == 0xFF:
            pos += 1
        m = data[pos]
        if m == 0xC2:
            return True
        if m in (0xC0, 0xC1, 0xDA):
            return False
        pos += 1 + ((data[pos + 1] << 8) | data[pos + 2])
    return False


FIX = O.manifest()
PROG = [f for f in FIX if "libjpeg_coef_sha256" in f and is_progressive(O.fixture_bytes(f))]
SMALL = [f for f in PROG if f["bytes"] < 100_000]
# fixtures whose scan script keeps every refinement scan within three producer scans (a batch
# holding any other stream falls back to level-by-level refinement: rj_decoder.cpp prog_pipe)
PIPELINED = [f for f in SMALL if f["name"] != "cp420_scans5_112x80"]
BASE = [f for f in FIX if "libjpeg_coef_sha256" in f and f["ref_parse"]["ok"] and f["ref_parse"]["css"] in (0, 1, 2, 3, 5)
        and f["bytes"] < 100_000]
FORMATS = list(R.OutputFormat)


@pytest.fixture(scope="module", params=[0, 1], ids=["auto_path", "general_path"])
def dec(request):
    from tests import gpu_util as G
    G.torch()
    d = R.JpegDecoder(R.Backend.HARDWARE, 0)
    d.set_path_policy(request.param)
    yield d
    d.close()


def run_both(dec, data, fmt, crop=(0, 0, 0, 0)):
    from tests import gpu_util as G
    s = R.JpegStream(data)
    nc, css, w, h = dec.image_info(s)
    shapes = G.channel_shapes(fmt, css, w, h, roi=crop)
    bufs, img = G.gpu_buffers(shapes)
    st = dec.decode(s, R.decode_params(fmt, crop), img)
    got = G.to_host(bufs)
    ost, want = O.oracle_decode(data, int(fmt), shapes, crop)
    return st, ost, got, want


def test_fixture_set():
    names = {f["name"] for f in PROG}
    # 4:2:0 / 4:2:2 / 4:4:4 / 4:4:0 / gray, DRI, optimised tables, truncation, the C5 1080p sample
    for n in ("pp420_q90_1920x1080", "cp444_prog_ri_136x72", "cp420_prog_ri3_160x112", "cp400_prog_120x80",
              "cp440_prog_96x80", "cp422_prog_97x67", "pp420_opt_200x150", "pp420_prog_trunc_192x128",
              "cp420_scans3_128x96", "cp420_scans5_112x80"):
        assert n in names, n


@pytest.mark.parametrize("fmt", FORMATS, ids=[f.name for f in FORMATS])
@pytest.mark.parametrize("ent", PROG, ids=[f["name"] for f in PROG])
def test_progressive_matches_oracle(dec, ent, fmt):
    from tests import gpu_util as G
    st, ost, got, want = run_both(dec, O.fixture_bytes(ent), fmt)
    assert st == ost == 0
    for c, (g, w) in enumerate(zip(got, want)):
        assert G.first_mismatch(g, w) is None, (c, G.first_mismatch(g, w))


CROPS = [(8, 8, 72, 56), (3, 5, 60, 61), (0, 0, 64, 32)]


@pytest.mark.parametrize("crop", CROPS, ids=[str(c) for c in CROPS])
@pytest.mark.parametrize("fmt", [R.OutputFormat.RGB, R.OutputFormat.NATIVE, R.OutputFormat.YUV_PLANAR])
@pytest.mark.parametrize("ent", SMALL[:4], ids=[f["name"] for f in SMALL[:4]])
def test_progressive_roi(dec, ent, fmt, crop):
    from tests import gpu_util as G
    st, ost, got, want = run_both(dec, O.fixture_bytes(ent), fmt, crop)
    assert st == ost == 0
    for c, (g, w) in enumerate(zip(got, want)):
        assert G.first_mismatch(g, w) is None, (c, G.first_mismatch(g, w))


def _truncations(data):
    """Cut inside each third of the stream: later scans missing, a scan ending mid-interval
    (libjpeg's insufficient-data rule: zero bits, then the rest of the interval skipped)."""
    out = {}
    for frac in (0.3, 0.55, 0.8, 0.97):
        cut = int(len(data) * frac)
        if data[cut - 1] == 0xFF:
            cut -= 1
        out[f"cut{int(frac * 100)}"] = data[:cut]
    return out


@pytest.mark.parametrize("ent", [f for f in PROG if f["name"] in ("pp420_opt_200x150", "cp420_prog_ri3_160x112",
                                                                   "cp444_prog_ri_136x72")],
                         ids=lambda f: f["name"])
def test_progressive_truncated(dec, ent):
    from tests import gpu_util as G
    for name, data in _truncations(O.fixture_bytes(ent)).items():
        st, ost, got, want = run_both(dec, data, R.OutputFormat.RGB)
        assert st == ost, (name, st, ost)
        if st == 0:
            assert G.first_mismatch(got[0], want[0]) is None, (name, G.first_mismatch(got[0], want[0]))


@pytest.mark.parametrize("fmt", [R.OutputFormat.RGB, R.OutputFormat.Y])
def test_ac_refine_zero_run_overshoot_at_se63(dec, fmt):
    """A Se = 63 AC refinement whose new coefficient's zero run passes position 63 (corrupt
    data no encoder writes): libjpeg stores it at natural index 63 (jdphuff.c, natural_order[64]
    == 63).  The crafted stream (tests/jpeg_craft.py) hits it in every block; the oracle's
    result on it equals libjpeg-turbo's (tests/test_oracle_golden.py).  k_prog_wave must store
    it there too (the clamp to 63 had been lost)."""
    from tests import gpu_util as G
    from tests import jpeg_craft as C
    data = C.prog_gray_refine_overshoot(64, 64)
    st, ost, got, want = run_both(dec, data, fmt)
    assert st == ost == 0
    for c, (g, w) in enumerate(zip(got, want)):
        assert G.first_mismatch(g, w) is None, (c, G.first_mismatch(g, w))


@pytest.mark.parametrize("resident", [False, True], ids=["staged", "resident"])
@pytest.mark.parametrize("fmt", [R.OutputFormat.RGB, R.OutputFormat.YUV_PLANAR, R.OutputFormat.NATIVE])
def test_batch_mixed_progressive_and_baseline(dec, fmt, resident):
    """Progressive and baseline streams in one rocJpegDecodeBatched call (both pipelines share
    K0 and the output stage), streams staged per call or resident in HBM."""
    from tests import gpu_util as G
    datas = [O.fixture_bytes(e) for e in PROG if e in PIPELINED or e["bytes"] >= 100_000]
    datas += [O.fixture_bytes(e) for e in BASE[:6]]
    datas += [O.fixture_bytes(e) for e in PIPELINED]  # the same streams twice in one batch
    streams = [R.JpegStream(d) for d in datas]
    if resident:
        dec.streams_to_device(streams)
    shapes_all, bufs_all, imgs = [], [], []
    for s in streams:
        nc, css, w, h = dec.image_info(s)
        shapes = G.channel_shapes(fmt, css, w, h)
        bufs, img = G.gpu_buffers(shapes)
        shapes_all.append(shapes)
        bufs_all.append(bufs)
        imgs.append(img)
    assert dec.decode_batched(streams, R.decode_params(fmt), imgs) == 0
    for k, (d, shapes, bufs) in enumerate(zip(datas, shapes_all, bufs_all)):
        ost, want = O.oracle_decode(d, int(fmt), shapes)
        assert ost == 0
        for c, (g, w) in enumerate(zip(G.to_host(bufs), want)):
            assert G.first_mismatch(g, w) is None, (k, c, G.first_mismatch(g, w))


def test_batch_after_reparse_swaps_stream_kinds(dec):
    """Stream handles re-parsed with the other kind of data (baseline -> progressive and
    progressive -> baseline, rocJpegStreamParse on a used handle) decode like fresh ones in one
    batch: nothing cached by the earlier parse (interval tables, the lane sort's length buckets,
    resident copies) survives into the new plan."""
    from tests import gpu_util as G
    fmt = R.OutputFormat.RGB
    prog = [O.fixture_bytes(e) for e in PIPELINED][:3]
    base = [O.fixture_bytes(e) for e in BASE[:3]]
    streams = [R.JpegStream(d) for d in base + prog]
    dec.streams_to_device(streams)
    datas = prog + base  # every handle now holds the other kind
    for s, d in zip(streams, datas):
        s.parse(d)
    shapes_all, bufs_all, imgs = [], [], []
    for s in streams:
        nc, css, w, h = dec.image_info(s)
        shapes = G.channel_shapes(fmt, css, w, h)
        bufs, img = G.gpu_buffers(shapes)
        shapes_all.append(shapes)
        bufs_all.append(bufs)
        imgs.append(img)
    assert dec.decode_batched(streams, R.decode_params(fmt), imgs) == 0
    for k, (d, shapes, bufs) in enumerate(zip(datas, shapes_all, bufs_all)):
        ost, want = O.oracle_decode(d, int(fmt), shapes)
        assert ost == 0
        for c, (g, w) in enumerate(zip(G.to_host(bufs), want)):
            assert G.first_mismatch(g, w) is None, (k, c, G.first_mismatch(g, w))


def test_progressive_timings(dec):
    from tests import gpu_util as G
    data = O.fixture_bytes(next(f for f in PROG if f["name"] == "pp420_q90_1920x1080"))
    s = R.JpegStream(data)
    nc, css, w, h = dec.image_info(s)
    bufs, img = G.gpu_buffers(G.channel_shapes(R.OutputFormat.RGB, css, w, h))
    dec.set_profiling(True)
    try:
        assert dec.decode(s, R.decode_params(R.OutputFormat.RGB), img) == 0
        t = dec.last_timings()
    finally:
        dec.set_profiling(False)
    assert t["prog_images"] == 1 and t["prog_levels"] >= 2 and t["prog_intervals"] == 10
    assert t["prog_entropy_ms"] > 0 and t["prog_rows_ms"] > 0
    assert t["prog_coef_bytes"] == 1920 * 1088 * 3 // 2 * 2  # 4:2:0, MCU-padded, int16
    # per-kernel launches: first-scan lanes (+ DC refinement lanes), AC refinement waves, fold
    assert t["prog_kernel_launches"][1] >= 1 and t["prog_kernel_launches"][2] >= 1
    assert all(t["prog_kernel_ms"][j] > 0 and t["prog_kernel_bytes"][j] > 0 for j in (1, 2))
    assert sum(t["prog_kernel_ms"][1:]) <= t["prog_entropy_ms"] * 1.01


LAYOUTS = {
    # the refinement scans level by level (the path taken when a scan has more than three
    # producer scans)
    "level_by_level": {"RJ_PROG_PIPE": "0"},
    # pipelined, the AC first scans in a wave grid ahead of the refinement grid (large batches)
    "two_grids": {"RJ_PROG_WAVE_ALL": "0"},
    # pipelined, every scan in one wave grid (small batches)
    "one_grid": {"RJ_PROG_WAVE_ALL": "1"},
}


@pytest.mark.parametrize("layout", list(LAYOUTS))
def test_progressive_layouts_match_oracle(layout):
    """Each launch layout of the progressive path (rj_decoder.cpp, prog_pipe / prog_wave_all),
    forced through its environment switch -- same bytes as the oracle for every fixture."""
    import os
    from tests import gpu_util as G
    G.torch()
    env = LAYOUTS[layout]
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        d = R.JpegDecoder(R.Backend.HARDWARE, 0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    try:
        datas = [O.fixture_bytes(e) for e in PROG]
        streams = [R.JpegStream(x) for x in datas]
        bufs_all, imgs, shapes_all = [], [], []
        for s in streams:
            nc, css, w, h = d.image_info(s)
            shapes = G.channel_shapes(R.OutputFormat.RGB, css, w, h)
            bufs, img = G.gpu_buffers(shapes)
            bufs_all.append(bufs)
            imgs.append(img)
            shapes_all.append(shapes)
        assert d.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs) == 0
        for x, shapes, bufs in zip(datas, shapes_all, bufs_all):
            ost, want = O.oracle_decode(x, int(R.OutputFormat.RGB), shapes)
            assert ost == 0
            assert G.first_mismatch(G.to_host(bufs)[0], want[0]) is None
    finally:
        d.close()


@pytest.mark.parametrize("layout", ["one_grid", "two_grids"])
def test_progressive_many_images_one_call(layout):
    """Hundreds of progressive images in one call (each small fixture many times over, DRI and
    no-DRI scripts mixed): every refinement wave follows its producers through the progress
    counters under load, in both pipelined layouts -- every image equals the oracle."""
    import os
    from tests import gpu_util as G
    G.torch()
    env = LAYOUTS[layout]
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        d = R.JpegDecoder(R.Backend.HARDWARE, 0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    try:
        base = [O.fixture_bytes(e) for e in PIPELINED]
        want = {}
        datas = [base[i % len(base)] for i in range(320)]
        streams = [R.JpegStream(x) for x in datas]
        dec_bufs, imgs, shapes_all = [], [], []
        for s in streams:
            nc, css, w, h = d.image_info(s)
            shapes = G.channel_shapes(R.OutputFormat.RGB, css, w, h)
            bufs, img = G.gpu_buffers(shapes)
            dec_bufs.append(bufs)
            imgs.append(img)
            shapes_all.append(shapes)
        assert d.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs) == 0
        for k, (x, shapes, bufs) in enumerate(zip(datas, shapes_all, dec_bufs)):
            key = k % len(base)
            if key not in want:
                ost, ref = O.oracle_decode(x, int(R.OutputFormat.RGB), shapes)
                assert ost == 0
                want[key] = ref[0]
            assert G.first_mismatch(G.to_host(bufs)[0], want[key]) is None, k
    finally:
        d.close()


def test_progressive_1080p_batch_one_call(dec):
    """The C5 sample (1080p 4:2:0, ten scans, no DRI) 96 times in one call: every image equals
    the oracle's decode (compared on the device), at the scale where the refinement waves of
    many images share the chip."""
    from tests import gpu_util as G
    t = G.torch()
    ent = next(f for f in PROG if f["name"] == "pp420_q90_1920x1080")
    data = O.fixture_bytes(ent)
    streams = [R.JpegStream(data) for _ in range(96)]
    nc, css, w, h = dec.image_info(streams[0])
    shapes = G.channel_shapes(R.OutputFormat.RGB, css, w, h)
    bufs_all, imgs = [], []
    for _ in streams:
        bufs, img = G.gpu_buffers(shapes)
        bufs_all.append(bufs)
        imgs.append(img)
    assert dec.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs) == 0
    ost, want = O.oracle_decode(data, int(R.OutputFormat.RGB), shapes)
    assert ost == 0
    ref = t.from_numpy(want[0]).to("cuda")
    bad = [k for k, bufs in enumerate(bufs_all) if not t.equal(bufs[0], ref)]
    assert not bad, bad[:8]


def test_progressive_producer_wait_give_up_is_clean():
    """A refinement wave whose producers never report progress gives up after its bounded wait
    and the call returns ROCJPEG_STATUS_EXECUTION_FAILED -- no hang, no fault.  Forced with the
    test hook RJ_TEST_PROG_GIVEUP (k_prog_wave waits for a count no producer reaches, with a
    short poll budget).  The same handle still decodes baseline streams exactly afterwards, and a
    handle without the hook decodes the progressive streams exactly."""
    import os
    from tests import gpu_util as G
    G.torch()
    env = {"RJ_TEST_PROG_GIVEUP": "1", "RJ_PROG_WAVE_ALL": "1"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        d = R.JpegDecoder(R.Backend.HARDWARE, 0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    good = R.JpegDecoder(R.Backend.HARDWARE, 0)
    try:
        def batch(dec, datas):
            streams = [R.JpegStream(x) for x in datas]
            bufs_all, imgs, shapes_all = [], [], []
            for s in streams:
                nc, css, w, h = dec.image_info(s)
                shapes = G.channel_shapes(R.OutputFormat.RGB, css, w, h)
                bufs, img = G.gpu_buffers(shapes)
                bufs_all.append(bufs)
                imgs.append(img)
                shapes_all.append(shapes)
            st = dec.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs)
            return st, shapes_all, bufs_all

        prog = [O.fixture_bytes(e) for e in PIPELINED]
        st, _, _ = batch(d, prog)
        assert st == R.Status.EXECUTION_FAILED, R.error_name(st)
        base = [O.fixture_bytes(e) for e in BASE[:4]]
        for dec, datas in ((d, base), (good, prog)):
            st, shapes_all, bufs_all = batch(dec, datas)
            assert st == 0, R.error_name(st)
            for x, shapes, bufs in zip(datas, shapes_all, bufs_all):
                ost, want = O.oracle_decode(x, int(R.OutputFormat.RGB), shapes)
                assert ost == 0
                assert G.first_mismatch(G.to_host(bufs)[0], want[0]) is None
    finally:
        d.close()
        good.close()
