"""Parity of the HIP decode path (through the C ABI) with the CPU oracle, byte for byte, over
every committed fixture, every output format, batches, ROI crops and the error paths."""
import numpy as np
import pytest

import rocjpeg_amd as R
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

FIX = O.manifest()
# baseline fixtures (the reference parser accepts them); progressive ones: test_progressive_gpu.py
DECODABLE = [f for f in FIX if "libjpeg_coef_sha256" in f and f["ref_parse"]["ok"] and f["ref_parse"]["css"] in (0, 1, 2, 3, 5)]
SMALL = [f for f in DECODABLE if f["bytes"] < 100_000]
FORMATS = list(R.OutputFormat)


@pytest.fixture(scope="module", params=[0, 1], ids=["auto_path", "general_path"])
def dec(request):
    """policy 0: fused K2 wherever the output window allows it; 1: always the general path."""
    from tests import gpu_util as G
    G.torch()
    d = R.JpegDecoder(R.Backend.HARDWARE, 0)
    d.set_path_policy(request.param)
    yield d
    d.close()


def run_both(dec, data, fmt, crop=(0, 0, 0, 0), pad=0):
    from tests import gpu_util as G
    s = R.JpegStream(data)
    nc, css, w, h = dec.image_info(s)
    shapes = G.channel_shapes(fmt, css, w, h, roi=crop, rgb_pitch_pad=pad)
    bufs, img = G.gpu_buffers(shapes)
    st = dec.decode(s, R.decode_params(fmt, crop), img)
    got = G.to_host(bufs)
    ost, want = O.oracle_decode(data, int(fmt), shapes, crop)
    return st, ost, got, want


@pytest.mark.parametrize("fmt", FORMATS, ids=[f.name for f in FORMATS])
@pytest.mark.parametrize("ent", DECODABLE, ids=[f["name"] for f in DECODABLE])
def test_decode_matches_oracle(dec, ent, fmt):
    from tests import gpu_util as G
    data = O.fixture_bytes(ent)
    st, ost, got, want = run_both(dec, data, fmt)
    assert st == ost == 0
    for c, (g, w) in enumerate(zip(got, want)):
        assert G.first_mismatch(g, w) is None, (c, G.first_mismatch(g, w))


@pytest.mark.parametrize("ent", SMALL, ids=[f["name"] for f in SMALL])
def test_rgb_padded_pitch(dec, ent):
    st, ost, got, want = run_both(dec, O.fixture_bytes(ent), R.OutputFormat.RGB, pad=13)
    assert st == ost == 0
    assert np.array_equal(got[0], want[0])


CROPS = [(8, 8, 72, 56), (16, 0, 64, 64), (3, 5, 60, 61), (1, 1, 64, 64), (0, 0, 64, 32)]


@pytest.mark.parametrize("crop", CROPS, ids=[str(c) for c in CROPS])
@pytest.mark.parametrize("fmt", FORMATS, ids=[f.name for f in FORMATS])
@pytest.mark.parametrize("ent", SMALL, ids=[f["name"] for f in SMALL])
def test_roi_matches_oracle(dec, ent, fmt, crop):
    from tests import gpu_util as G
    st, ost, got, want = run_both(dec, O.fixture_bytes(ent), fmt, crop)
    assert st == ost == 0
    for c, (g, w) in enumerate(zip(got, want)):
        assert G.first_mismatch(g, w) is None, (c, G.first_mismatch(g, w))


@pytest.mark.parametrize("fmt", [R.OutputFormat.RGB, R.OutputFormat.YUV_PLANAR, R.OutputFormat.NATIVE])
def test_batched_mixed_matches_oracle(dec, fmt):
    from tests import gpu_util as G
    ents = [e for e in DECODABLE if e["bytes"] < 400_000]
    streams, all_bufs, imgs, wants = [], [], [], []
    for e in ents:
        data = O.fixture_bytes(e)
        s = R.JpegStream(data)
        nc, css, w, h = dec.image_info(s)
        shapes = G.channel_shapes(fmt, css, w, h)
        bufs, img = G.gpu_buffers(shapes)
        streams.append(s)
        all_bufs.append(bufs)
        imgs.append(img)
        wants.append(O.oracle_decode(data, int(fmt), shapes)[1])
    assert dec.decode_batched(streams, R.decode_params(fmt), imgs) == 0
    for e, bufs, want in zip(ents, all_bufs, wants):
        for c, (g, w) in enumerate(zip(G.to_host(bufs), want)):
            assert G.first_mismatch(g, w) is None, (e["name"], c, G.first_mismatch(g, w))


def test_resident_streams_same_output(dec):
    from tests import gpu_util as G
    ents = [e for e in DECODABLE if e["ref_parse"]["css"] == 3][:6]
    streams = [R.JpegStream(O.fixture_bytes(e)) for e in ents]
    dec.streams_to_device(streams)
    imgs, all_bufs = [], []
    for s in streams:
        nc, css, w, h = dec.image_info(s)
        bufs, img = G.gpu_buffers(G.channel_shapes(R.OutputFormat.RGB, css, w, h))
        imgs.append(img)
        all_bufs.append(bufs)
    assert dec.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs) == 0
    for e, bufs in zip(ents, all_bufs):
        data = O.fixture_bytes(e)
        want = O.oracle_decode(data, int(R.OutputFormat.RGB), [tuple(bufs[0].shape)])[1]
        assert np.array_equal(G.to_host(bufs)[0], want[0]), e["name"]


def test_error_statuses(dec):
    from tests import gpu_util as G
    by = {f["name"]: f for f in FIX}
    # 4:1:1: VCN path rejects it (rocjpeg_vaapi_decoder.cpp:633-636)
    s = R.JpegStream(O.fixture_bytes(by["c411_q90_128x64"]))
    bufs, img = G.gpu_buffers([(64, 3 * 128)])
    assert dec.decode(s, R.decode_params(R.OutputFormat.RGB), img) == R.Status.JPEG_NOT_SUPPORTED
    # progressive: the reference parser fails on the SOF2 stream (comp id mismatch at SOS);
    # this decoder parses and decodes it (tests/test_progressive_gpu.py)
    assert R.JpegStream().try_parse(O.fixture_bytes(by["p420_prog_128x96"])) == R.Status.SUCCESS
    # NULL destination channel for a kernel-written format
    s = R.JpegStream(O.fixture_bytes(by["p420_q90_ri_256x128"]))
    img = R.make_image([0, 0, 0, 0], [768, 0, 0, 0])
    assert dec.decode(s, R.decode_params(R.OutputFormat.RGB), img) == R.Status.INVALID_PARAMETER
    # image smaller than 64x64 (rocjpeg_vaapi_decoder.cpp:586-592)
    from PIL import Image
    import io
    b = io.BytesIO()
    Image.new("RGB", (48, 48), (10, 200, 30)).save(b, "JPEG", quality=90)
    s = R.JpegStream(b.getvalue())
    bufs, img = G.gpu_buffers([(48, 144)])
    assert dec.decode(s, R.decode_params(R.OutputFormat.RGB), img) == R.Status.JPEG_NOT_SUPPORTED
    # empty batch succeeds
    assert dec.decode_batched([], R.decode_params(R.OutputFormat.RGB), []) in (0, R.Status.INVALID_PARAMETER)


# ---- chunked (self-synchronising) entropy decode of long intervals ----
BIG_NORI = [f for f in DECODABLE if f["ref_parse"]["restart_interval"] == 0 and f["bytes"] > 200_000]


def _ecs_span(data):
    """(start, end) of the entropy-coded segment after the (only) SOS."""
    i = data.index(b"\xff\xda")
    start = i + 2 + int.from_bytes(data[i + 2:i + 4], "big")
    end = data.rindex(b"\xff\xd9")
    return start, end


def _variants(data):
    """Damaged copies of a long no-restart stream: truncated (libjpeg's insufficient-data path,
    which the chunked decode hands to the serial re-decode) and with flipped bits mid-stream
    (the chunks must still agree with the true decode wherever they synchronise)."""
    s, e = _ecs_span(data)
    out = {}
    for frac in (0.37, 0.81):
        cut = s + int((e - s) * frac)
        if data[cut - 1] == 0xFF:
            cut -= 1
        out[f"trunc{int(frac * 100)}"] = data[:cut] + b"\xff\xd9"
    buf = bytearray(data)
    rng = np.random.default_rng(7)
    for pos in rng.integers(s + 1000, e - 1000, 24):
        if buf[pos] != 0xFF and buf[pos - 1] != 0xFF and buf[pos + 1] != 0x00:
            nb = buf[pos] ^ (1 << int(rng.integers(0, 8)))
            if nb != 0xFF:
                buf[pos] = nb
    out["bitflips"] = bytes(buf)
    return out


@pytest.mark.parametrize("ent", BIG_NORI, ids=[f["name"] for f in BIG_NORI])
def test_long_interval_damaged_streams(dec, ent):
    """Parity on damaged long no-restart streams, where the chunked K1 meets truncation and
    corrupt codes (the oracle restates libjpeg's semantics for both)."""
    from tests import gpu_util as G
    for name, data in _variants(O.fixture_bytes(ent)).items():
        st, ost, got, want = run_both(dec, data, R.OutputFormat.RGB)
        assert st == ost, name
        if st == 0:
            assert G.first_mismatch(got[0], want[0]) is None, (name, G.first_mismatch(got[0], want[0]))


def test_long_interval_batch_mixed(dec):
    """A batch mixing long no-restart streams (chunked), restart-interval streams (one lane per
    interval) and their damaged variants, decoded in one call."""
    from tests import gpu_util as G
    datas = []
    for ent in BIG_NORI + SMALL[:4]:
        d = O.fixture_bytes(ent)
        datas.append(d)
        if ent in BIG_NORI:
            datas.extend(_variants(d).values())
    streams = [R.JpegStream(d) for d in datas]
    shapes_all, bufs_all, imgs = [], [], []
    for s in streams:
        nc, css, w, h = dec.image_info(s)
        shapes = G.channel_shapes(R.OutputFormat.RGB, css, w, h)
        bufs, img = G.gpu_buffers(shapes)
        shapes_all.append(shapes)
        bufs_all.append(bufs)
        imgs.append(img)
    st = dec.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs)
    assert st == 0
    for d, shapes, bufs in zip(datas, shapes_all, bufs_all):
        ost, want = O.oracle_decode(d, int(R.OutputFormat.RGB), shapes)
        assert ost == 0
        assert G.first_mismatch(G.to_host(bufs)[0], want[0]) is None


@pytest.fixture(scope="module",
                params=[(0, 4, {}), (1, 4, {}), (0, 1, {}), (1, 1, {}), (0, 1, {"RJ_LPT": "0", "RJ_K1_SOLO": "0"}),
                        (0, 1, {"RJ_SPLIT_OUTLIERS": "1", "RJ_SPLIT_OUTLIER_FRAC": "1"}),
                        (1, 1, {"RJ_SPLIT_OUTLIERS": "1", "RJ_SPLIT_OUTLIER_FRAC": "1"})],
                ids=["g4", "general_g4", "g1", "general_g1", "g1_short_first", "split_outliers_g1",
                     "split_outliers_general_g1"])
def pdec(request):
    """A decoder that sorts the K1 lanes of every call with no split interval by length
    (RJ_PIPE_MIN=1) and, with 4 groups, pipelines it: interval length classes on separate
    streams, each class's K2 rows after the K1 lanes of its class and all earlier ones.  A batch
    of row-interval images takes the lean K1 (rj_huff.hip), a batch with any other image the
    exact K1 (rj_entropy.hip); the lean outlier split (head + tail lanes per long interval) is
    forced on every long interval here (RJ_SPLIT_OUTLIER_FRAC=1)."""
    import os
    from tests import gpu_util as G
    G.torch()
    policy, groups, extra = request.param
    # (RJ_CHUNK_MIN: no call-time interval split, so that these small calls keep the layouts)
    env = {"RJ_PIPE_MIN": "1", "RJ_PIPE_GROUPS": str(groups), "RJ_CHUNK_MIN": str(1 << 30), **extra}
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
    d.set_path_policy(policy)
    d.groups = groups
    d.extra = extra
    d.set_profiling(True)
    yield d
    d.close()


@pytest.mark.parametrize("fmt", [R.OutputFormat.RGB, R.OutputFormat.YUV_PLANAR, R.OutputFormat.NATIVE])
def test_pipelined_batch_matches_oracle(pdec, fmt):
    """Pipelined launch over a batch of restart-interval and short streams (no interval split):
    rows of every length class, damaged variants included, byte-identical to the oracle."""
    from tests import gpu_util as G
    big = [e for e in DECODABLE if e["name"] == "p420_q90_ri_1920x1080"]
    datas = [O.fixture_bytes(e) for e in SMALL for _ in range(3)]
    for e in big:
        d = O.fixture_bytes(e)
        datas.append(d)
        datas.extend(_variants(d).values())
    streams = [R.JpegStream(d) for d in datas]
    shapes_all, bufs_all, imgs = [], [], []
    for s in streams:
        nc, css, w, h = pdec.image_info(s)
        shapes = G.channel_shapes(fmt, css, w, h)
        bufs, img = G.gpu_buffers(shapes)
        shapes_all.append(shapes)
        bufs_all.append(bufs)
        imgs.append(img)
    assert pdec.decode_batched(streams, R.decode_params(fmt), imgs) == 0
    t = pdec.last_timings()
    assert t["split_intervals"] == 0 and t["pipe_groups"] == pdec.groups, (t["split_intervals"], t["pipe_groups"])
    for k, (d, shapes, bufs) in enumerate(zip(datas, shapes_all, bufs_all)):
        ost, want = O.oracle_decode(d, int(fmt), shapes)
        assert ost == 0
        for c, (g, w) in enumerate(zip(G.to_host(bufs), want)):
            assert G.first_mismatch(g, w) is None, (k, c, G.first_mismatch(g, w))


@pytest.mark.parametrize("fmt", [R.OutputFormat.RGB, R.OutputFormat.YUV_PLANAR])
def test_pipelined_row_aligned_batch(pdec, fmt):
    """Every interval exactly one MCU row (DRI = MCUs per row): the pipelined K2 takes its rows
    straight from the sorted K1 lane order.  Damaged variants included."""
    from tests import gpu_util as G
    datas = []
    for e in DECODABLE:
        if e["name"] in ("p420_q90_ri_1920x1080", "p420_trunc_192x128"):
            d = O.fixture_bytes(e)
            datas += [d, d]
            if e["name"] == "p420_q90_ri_1920x1080":
                datas.extend(_variants(d).values())
    streams = [R.JpegStream(d) for d in datas]
    shapes_all, bufs_all, imgs = [], [], []
    for s in streams:
        nc, css, w, h = pdec.image_info(s)
        shapes = G.channel_shapes(fmt, css, w, h)
        bufs, img = G.gpu_buffers(shapes)
        shapes_all.append(shapes)
        bufs_all.append(bufs)
        imgs.append(img)
    assert pdec.decode_batched(streams, R.decode_params(fmt), imgs) == 0
    t = pdec.last_timings()
    assert t["pipe_groups"] == pdec.groups
    if pdec.groups > 1:
        assert t["pipe_lane_rows"] == 1
    assert t["lean_k1"] == 1
    if pdec.extra.get("RJ_SPLIT_OUTLIERS") == "1":
        # the 1080p intervals (and the damaged ones) near the longest are split
        assert t["lean_split"] > 0
    for k, (d, shapes, bufs) in enumerate(zip(datas, shapes_all, bufs_all)):
        ost, want = O.oracle_decode(d, int(fmt), shapes)
        assert ost == 0
        for c, (g, w) in enumerate(zip(G.to_host(bufs), want)):
            assert G.first_mismatch(g, w) is None, (k, c, G.first_mismatch(g, w))


# ---- the reference's size limits (rocjpeg_vaapi_decoder.cpp:586-592: 64 .. 16384 per side) ----
def _noise_jpeg(w, h, sub, rst_rows=1, seed=3):
    import io
    from PIL import Image
    rng = np.random.default_rng(seed)
    a = np.clip(128 + 60 * np.sin(np.arange(w, dtype=np.float32)[None, :, None] / 11.0) +
                rng.normal(0, 20, (h, w, 3)).astype(np.float32), 0, 255)
    b = io.BytesIO()
    mcu_w = 16 if sub in (1, 2) else 8
    kw = dict(quality=85, subsampling=sub)
    if rst_rows:
        kw["restart_marker_blocks"] = rst_rows * ((w + mcu_w - 1) // mcu_w)
    Image.fromarray(a.astype(np.uint8)).save(b, "JPEG", **kw)
    return b.getvalue()


@pytest.mark.parametrize("w,h,sub,rst", [(16384, 64, 2, 1), (64, 16384, 2, 1), (16384, 80, 0, 0), (64, 64, 2, 1),
                                         (16384, 2048, 2, 1)],
                         ids=["16384x64_420_ri", "64x16384_420_ri", "16384x80_444_nori", "64x64_420", "16384x2048_420"])
@pytest.mark.parametrize("fmt", [R.OutputFormat.RGB, R.OutputFormat.YUV_PLANAR], ids=["RGB", "YUV_PLANAR"])
def test_largest_and_smallest_accepted_sizes(dec, w, h, sub, rst, fmt):
    """The edges of the accepted size range decode like the oracle: 16384-wide rows (256-KB
    RGB rows, 1024 MCUs per row: the longest interval a row image can have), 16384-tall
    columns, a 16384-wide restart-less 4:4:4 strip (chunk lanes), the 64x64 minimum, and a
    16384 x 2048 4:2:0 picture (100 MB RGB)."""
    data = _noise_jpeg(w, h, sub, rst)
    st, ost, got, want = run_both(dec, data, fmt)
    assert st == 0 and ost == 0
    for g, x in zip(got, want):
        assert np.array_equal(g, x)


@pytest.mark.parametrize("color", [(128, 128, 128), (200, 30, 90)], ids=["gray128", "color"])
@pytest.mark.parametrize("rst", [1, 0], ids=["ri_row", "nori"])
def test_flat_images_with_two_bit_blocks(dec, color, rst):
    """A flat 1080p picture with optimised tables: every block is a 1-bit DC code and a 1-bit EOB
    (one two-symbol K1 step), so a lane's first phases use less than one 32-bit word of its bit
    ring and the decoder's consumed-word count starts below zero -- it must not read as the
    lane's end to the mover that feeds the ring (rj_huff.hip RJ_HL_FIN).  Lean K1 (row
    intervals) and the chunk lanes (no restart markers)."""
    import io
    from PIL import Image
    b = io.BytesIO()
    kw = dict(quality=90, subsampling=2, optimize=True)
    if rst:
        kw["restart_marker_blocks"] = 1920 // 16
    Image.new("RGB", (1920, 1080), color).save(b, "JPEG", **kw)
    st, ost, got, want = run_both(dec, b.getvalue(), R.OutputFormat.RGB)
    assert st == 0 and ost == 0
    for g, x in zip(got, want):
        assert np.array_equal(g, x)


@pytest.mark.parametrize("w,h", [(16385, 64), (64, 16385), (63, 64), (64, 63)])
def test_sizes_outside_the_range_are_refused(dec, w, h):
    """One pixel outside either edge: JPEG_NOT_SUPPORTED, as the reference's SubmitDecode
    returns (rocjpeg_vaapi_decoder.cpp:586-592); the parse itself succeeds."""
    from tests import gpu_util as G
    data = _noise_jpeg(w, h, 2, 0)
    s = R.JpegStream(data)
    bufs, img = G.gpu_buffers([(h, 3 * w)])
    assert dec.decode(s, R.decode_params(R.OutputFormat.RGB), img) == R.Status.JPEG_NOT_SUPPORTED


# ---- table de-duplication across streams (the DC table's two-symbol entries) ----
def remapped_pair(w=128, h=64):
    """Two baseline 4:2:0 streams with identical DHT and DQT bytes that code the same
    coefficients with the component-to-table map the other way round: stream A reads Y with
    (DC 0, AC 0) and chroma with (DC 1, AC 1), stream B Y with (DC 0, AC 1) and chroma with
    (DC 1, AC 0).  The DC tables' codes are short enough that DC + AC pairs fit one K1 table
    entry, and the two AC tables assign different codes, so a DC pair read with the other
    stream's AC table decodes garbage (tests/jpeg_craft.py baseline_420)."""
    import io
    from PIL import Image
    from tests import jpeg_craft as J
    rng = np.random.default_rng(11)
    yy, xx = np.mgrid[0:h, 0:w]
    a = np.stack([96 + 0.6 * xx, 80 + 0.9 * yy, 140 - 0.3 * xx], -1) + rng.normal(0, 9, (h, w, 3))
    b = io.BytesIO()
    Image.fromarray(np.clip(a, 0, 255).astype(np.uint8)).save(b, "JPEG", quality=92, subsampling=2)
    st, coefs, dims = O.decode_coefs(b.getvalue())
    assert st == 0
    blocks = [coefs[i:i + 64].astype(int) for i in range(0, coefs.size, 64)]
    _, acs = J.baseline_symbols(blocks)
    acs = sorted(acs | {0x00, 0xF0})
    dc_len = {0: 2, 1: 2, 2: 3, 3: 3, 4: 4, 5: 5, 6: 6, 7: 7, 8: 8, 9: 9, 10: 10, 11: 11}
    ac0 = {s: 8 for s in acs}
    ac1 = {s: (7 if k == 0 else 8) for k, s in enumerate(acs)}
    qz = [[2] * 64, [3] * 64]
    A = J.baseline_420(w, h, coefs, dims, qz, [dc_len, dc_len], [ac0, ac1], [(0, 0), (1, 1), (1, 1)])
    B = J.baseline_420(w, h, coefs, dims, qz, [dc_len, dc_len], [ac0, ac1], [(0, 1), (1, 0), (1, 0)])
    return A, B


@pytest.mark.parametrize("order", ["AB", "BA", "ABBA"])
def test_same_tables_other_component_map(dec, order):
    """Streams whose DHT / DQT bytes are equal but whose components map to the tables
    differently get table sets of their own in one batch (the K1 table image of a DC table
    carries second symbols read with one AC table)."""
    from tests import gpu_util as G
    A, B = remapped_pair()
    datas = [A if c == "A" else B for c in order]
    for d in datas:  # the oracle decodes both to the same coefficients
        assert O.oracle_decode(d, int(R.OutputFormat.RGB), [(64, 384)])[0] == 0
    streams = [R.JpegStream(d) for d in datas]
    bufs_all, imgs = [], []
    for s in streams:
        bufs, img = G.gpu_buffers([(64, 384)])
        bufs_all.append(bufs)
        imgs.append(img)
    assert dec.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs) == 0
    for k, (d, bufs) in enumerate(zip(datas, bufs_all)):
        want = O.oracle_decode(d, int(R.OutputFormat.RGB), [(64, 384)])[1]
        assert G.first_mismatch(G.to_host(bufs)[0], want[0]) is None, (order, k)
