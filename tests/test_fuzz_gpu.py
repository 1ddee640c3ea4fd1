"""Robustness of the GPU path on corrupt input: random byte damage inside the entropy-coded data
of baseline and progressive streams, decoded in batches.  Every call must return (no fault, no
hang) and be deterministic; baseline streams must still match the oracle byte for byte (its
corrupt-data semantics are libjpeg's: bad codes read as 17 bits / symbol 0, zeros past the data),
progressive ones are checked for determinism and status only -- corrupt codes that place a
coefficient outside the scan's band are outside the progressive exactness domain."""
import numpy as np
import pytest

import rocjpeg_amd as R
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

FIX = O.manifest()


def _is_prog(d):
    pos = 2
    while pos + 4 <= len(d):
        while d[pos] == 0xFF:
            pos += 1
        if d[pos] == 0xC2:
            return True
        if d[pos] in (0xC0, 0xC1, 0xDA):
            return False
        pos += 1 + ((d[pos + 1] << 8) | d[pos + 2])
    return False


def _first_sos_end(d):
    i = d.index(b"\xff\xda")
    return i + 2 + int.from_bytes(d[i + 2:i + 4], "big")


def scan_ranges(d):
    """[start, end) of every scan's entropy-coded data (up to the next marker other than RSTn)."""
    out, i = [], 0
    while True:
        i = d.find(b"\xff\xda", i)
        if i < 0:
            return out
        s = i + 2 + int.from_bytes(d[i + 2:i + 4], "big")
        e = s
        while e + 1 < len(d) and not (d[e] == 0xFF and d[e + 1] not in (0x00, 0xFF) and not 0xD0 <= d[e + 1] <= 0xD7):
            e += 1
        out.append((s, e))
        i = e


def damage(d, seed, nhits=12):
    """Flip bits / overwrite bytes inside the scans' entropy-coded data, never creating FF (no new
    markers) and never touching FF or the byte after one (marker structure and headers intact)."""
    rng = np.random.default_rng(seed)
    buf = bytearray(d)
    ranges = [(a, b) for a, b in scan_ranges(d) if b - a > 24]
    pos_all = []
    for _ in range(nhits):
        a, b = ranges[int(rng.integers(0, len(ranges)))]
        pos_all.append(int(rng.integers(a + 4, b - 4)))
    for pos in pos_all:
        if buf[pos] == 0xFF or buf[pos - 1] == 0xFF or buf[pos + 1] == 0x00:
            continue
        v = buf[pos] ^ (1 << int(rng.integers(0, 8))) if rng.random() < 0.7 else int(rng.integers(0, 255))
        if v != 0xFF:
            buf[pos] = v
    return bytes(buf)


BASE = [f for f in FIX if "libjpeg_coef_sha256" in f and f["ref_parse"]["ok"] and f["ref_parse"]["css"] in (0, 1, 2, 3, 5)
        and f["bytes"] < 100_000]
PROG = [f for f in FIX if "libjpeg_coef_sha256" in f and _is_prog(O.fixture_bytes(f)) and f["bytes"] < 100_000]


def _decode_batch(dec, datas):
    from tests import gpu_util as G
    streams, bufs_all, imgs, shapes_all = [], [], [], []
    for d in datas:
        s = R.JpegStream(d)
        nc, css, w, h = dec.image_info(s)
        shapes = G.channel_shapes(R.OutputFormat.RGB, css, w, h)
        bufs, img = G.gpu_buffers(shapes)
        streams.append(s)
        bufs_all.append(bufs)
        imgs.append(img)
        shapes_all.append(shapes)
    st = dec.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs)
    return st, [G.to_host(b)[0] for b in bufs_all], shapes_all


@pytest.fixture(scope="module")
def dec():
    from tests import gpu_util as G
    G.torch()
    d = R.JpegDecoder(R.Backend.HARDWARE, 0)
    yield d
    d.close()


@pytest.mark.parametrize("seed", range(4))
def test_fuzz_baseline_matches_oracle(dec, seed):
    datas = [damage(O.fixture_bytes(e), seed * 100 + k) for k, e in enumerate(BASE)]
    st, outs, shapes = _decode_batch(dec, datas)
    assert st == 0
    for d, o, shp in zip(datas, outs, shapes):
        ost, want = O.oracle_decode(d, int(R.OutputFormat.RGB), shp)
        assert ost == 0
        assert np.array_equal(o, want[0])


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_progressive_runs_and_is_deterministic(dec, seed):
    datas = [damage(O.fixture_bytes(e), seed * 100 + k, nhits=30) for k, e in enumerate(PROG)]
    st1, outs1, _ = _decode_batch(dec, datas)
    st2, outs2, _ = _decode_batch(dec, datas)
    assert st1 == st2 == 0
    for a, b in zip(outs1, outs2):
        assert np.array_equal(a, b)


def _coarse_quant_jpegs():
    """Streams whose quantisers are all 255 (DQT maximum for 8-bit tables): once damaged, decoded
    coefficients x quantiser leave the int32 IDCT's exact domain (|x| < 2^14, rj_math.h), which
    K2 detects per strip and hands to the 64-bit restatement of jidctint.c.  Restart interval one
    MCU row (the lean K1 with raw DC differences) and none (the chunked K1), four subsamplings."""
    import io
    from PIL import Image
    rng = np.random.default_rng(7)
    out = []
    for (w, h), sub, rst in [((256, 128), 2, True), ((200, 72), 0, True), ((160, 96), 1, True),
                             ((256, 128), 2, False), ((97, 65), 2, False)]:
        a = np.clip(128 + 90 * np.sin(np.arange(w)[None, :, None] / 7.0) + rng.normal(0, 40, (h, w, 3)), 0, 255)
        b = io.BytesIO()
        kw = dict(qtables=[[255] * 64, [255] * 64], subsampling=sub)
        if rst:
            kw["restart_marker_blocks"] = (w + 15) // 16
        Image.fromarray(a.astype(np.uint8)).save(b, "JPEG", **kw)
        out.append(b.getvalue())
    g = io.BytesIO()
    Image.fromarray(rng.integers(0, 255, (64, 96), dtype=np.uint8)).save(g, "JPEG", qtables=[[255] * 64],
                                                                          restart_marker_blocks=12)
    out.append(g.getvalue())
    return out


def test_coarse_quant_clean_streams_stay_in_int32_domain(dec):
    base = _coarse_quant_jpegs()
    dec.set_profiling(True)
    st, outs, shapes = _decode_batch(dec, base)
    tm = dec.last_timings()
    dec.set_profiling(False)
    assert st == 0 and tm["wide_rows"] == 0
    for d, o, shp in zip(base, outs, shapes):
        ost, want = O.oracle_decode(d, int(R.OutputFormat.RGB), shp)
        assert ost == 0 and np.array_equal(o, want[0])


@pytest.mark.parametrize("seed", range(3))
def test_fuzz_coarse_quant_outside_int32_domain(dec, seed):
    base = _coarse_quant_jpegs()
    datas = base + [damage(d, seed * 100 + k, nhits=40) for k, d in enumerate(base)]
    dec.set_profiling(True)
    st, outs, shapes = _decode_batch(dec, datas)
    tm = dec.last_timings()
    dec.set_profiling(False)
    assert st == 0
    assert tm["wide_rows"] > 0  # the fix-up path ran (the undamaged streams stay in the int32 domain)
    for d, o, shp in zip(datas, outs, shapes):
        ost, want = O.oracle_decode(d, int(R.OutputFormat.RGB), shp)
        assert ost == 0
        assert np.array_equal(o, want[0])


def _patch_dqt(d, value):
    """Every quantiser of every 8-bit DQT table set to `value` (the entropy-coded data unchanged:
    the same coefficients, dequantised to value / original times as much)."""
    buf = bytearray(d)
    i = 2
    while i + 4 <= len(buf):
        assert buf[i] == 0xFF
        m, ln = buf[i + 1], (buf[i + 2] << 8) | buf[i + 3]
        if m == 0xDA:
            break
        if m == 0xDB:
            j = i + 4
            while j < i + 2 + ln:
                assert buf[j] >> 4 == 0  # 8-bit tables only
                buf[j + 1:j + 65] = bytes([value]) * 64
                j += 65
        i += 2 + ln
    return bytes(buf)


def test_dot2_domain_band_goes_to_the_fixup_launch(dec):
    """Clean streams whose dequantised coefficients lie between the dot2 IDCT's exact domain
    (|DC| <= 1151, |AC| <= 1023, rj_math.h) and the int32 IDCT's (|x| < 2^14): noise encoded with
    quantisers 40, then every quantiser raised to 255 (coefficients up to ~+-40 dequantise to
    ~+-10,000).  K2 flags those strips and the fix-up launch decodes their rows again -- oracle
    bit-exact, baseline and every restart layout of _coarse_quant_jpegs."""
    import io
    from PIL import Image
    rng = np.random.default_rng(11)
    datas = []
    for (w, h), sub, rst in [((256, 128), 2, True), ((160, 96), 0, True), ((200, 72), 2, False)]:
        a = rng.integers(0, 255, (h, w, 3), dtype=np.uint8)
        b = io.BytesIO()
        kw = dict(qtables=[[40] * 64, [40] * 64], subsampling=sub)
        if rst:
            kw["restart_marker_blocks"] = (w + 15) // 16
        Image.fromarray(a).save(b, "JPEG", **kw)
        datas.append(_patch_dqt(b.getvalue(), 255))
    dec.set_profiling(True)
    st, outs, shapes = _decode_batch(dec, datas)
    tm = dec.last_timings()
    dec.set_profiling(False)
    assert st == 0 and tm["wide_rows"] > 0
    for d, o, shp in zip(datas, outs, shapes):
        ost, want = O.oracle_decode(d, int(R.OutputFormat.RGB), shp)
        assert ost == 0 and np.array_equal(o, want[0])
