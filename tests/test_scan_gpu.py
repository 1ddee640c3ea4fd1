"""GPU marker scan (rocJpegAmdStreamParseDevice, rj_scan.hip) == the host parser, table for
table: the entropy-coded segment end (the reference's ParseEOI, src/rocjpeg_parser.cpp:400-416),
the restart-interval table and the destuffing work units -- on every fixture and on damaged
streams that exercise each marker rule (fill bytes, missing / extra / foreign markers,
truncation, no EOI, garbage after EOI).  Device-parsed streams then decode byte-identically to
the oracle."""
import numpy as np
import pytest

import rocjpeg_amd as R
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

FIX = O.manifest()
ALL = [f for f in FIX if f["ref_parse"]["ok"]]
DECODABLE = [f for f in ALL if "libjpeg_coef_sha256" in f and f["ref_parse"]["css"] in (0, 1, 2, 3, 5)]


@pytest.fixture(scope="module")
def dec():
    from tests import gpu_util as G
    G.torch()
    d = R.JpegDecoder(R.Backend.HARDWARE, 0)
    yield d
    d.close()


def _sos_end(data):
    i = data.index(b"\xff\xda")
    return i + 2 + int.from_bytes(data[i + 2:i + 4], "big")


def variants(data):
    """Damaged copies; each keeps the header intact."""
    s = _sos_end(data)
    e = data.rfind(b"\xff\xd9")
    e = e if e > s else len(data)
    body = data[s:e]
    out = {"orig": data}
    rng = np.random.default_rng(11)
    out["trunc"] = data[:s + len(body) // 2]
    out["no_eoi"] = data[:e]
    out["garbage_after_eoi"] = data + bytes(rng.integers(0, 256, 300, dtype=np.uint8)) + b"\xff\xd9\xff\xd0"
    rst = [k for k in range(len(body) - 1) if body[k] == 0xFF and 0xD0 <= body[k + 1] <= 0xD7]
    if rst:
        k = rst[len(rst) // 2]
        out["rst_missing"] = data[:s + k] + data[s + k + 2:]
        out["rst_extra"] = data[:s + k] + b"\xff\xd3" + data[s + k:]
        out["rst_fill"] = data[:s + k] + b"\xff\xff\xff" + data[s + k:]
        k2 = rst[-1]
        out["rst_tail_removed"] = data[:s + rst[0]] + data[s + rst[0] + 2:s + k2] + data[s + k2 + 2:]
    mid = s + len(body) // 3
    while data[mid - 1] == 0xFF or data[mid] == 0xFF:
        mid += 1
    out["foreign_marker"] = data[:mid] + b"\xff\xe1" + data[mid:]
    out["fill_run"] = data[:mid] + b"\xff\xff\xff\xff\x00" + data[mid:]
    out["ff_at_end"] = data[:e] + b"\xff"
    # a fill byte and the EOI across the scan's 1-KB step boundary (ECS bytes 1023 | 1024, 1025 =
    # FF | FF D9): the fill byte is not a drop (an FF counts only below the end)
    for cut in (1023, 2047):
        if len(body) > cut + 64:
            b = bytearray(body[:cut])
            if b[-1] == 0xFF:
                b[-1] = 0x12
            out[f"fill_eoi_step_{cut + 1}"] = data[:s] + bytes(b) + b"\xff\xff\xd9"
    return out


def _tables(s):
    return s.info(), s.intervals(), s.destuff_blocks()


@pytest.mark.parametrize("ent", ALL, ids=[f["name"] for f in ALL])
def test_device_scan_equals_host_parse(dec, ent):
    datas = variants(O.fixture_bytes(ent))
    st, dev = dec.parse_device(list(datas.values()))
    t = dec.last_timings()
    assert t["scan_host_fallbacks"] == 0
    if st == R.Status.SUCCESS and ent["ref_parse"]["css"] in (0, 1, 2, 3, 5):
        assert t["scan_device_streams"] > 0  # the tables below came from the GPU
    for (name, d), sd in zip(datas.items(), dev):
        h = R.JpegStream()
        hst = h.try_parse(d)
        if hst != R.Status.SUCCESS:
            continue  # the batch call reports the first failure; compared below
        assert _tables(sd) == _tables(h), name
    hosts = [R.JpegStream().try_parse(d) for d in datas.values()]
    first_bad = next((x for x in hosts if x != R.Status.SUCCESS), R.Status.SUCCESS)
    assert st == first_bad


def test_device_scan_batch_all_fixtures_and_decode(dec):
    """All fixtures (baseline and progressive) in one device-parse call, then one batched decode
    of the decodable ones, byte-identical to the oracle."""
    from tests import gpu_util as G
    ents = [f for f in FIX if "libjpeg_coef_sha256" in f and f["bytes"] < 600_000]
    datas = [O.fixture_bytes(e) for e in ents]
    st, streams = dec.parse_device(datas)
    assert st == R.Status.SUCCESS
    t = dec.last_timings()
    assert t["scan_device_streams"] >= len([e for e in ents if e["ref_parse"]["ok"]]) - 4
    assert t["scan_host_fallbacks"] == 0
    keep, bufs_all, imgs, shapes_all = [], [], [], []
    for d, s in zip(datas, streams):
        nc, css, w, h = dec.image_info(s)
        if css not in (0, 1, 2, 3, 5) or w[0] < 64 or h[0] < 64:
            continue
        shapes = G.channel_shapes(R.OutputFormat.RGB, css, w, h)
        bufs, img = G.gpu_buffers(shapes)
        keep.append((d, s))
        bufs_all.append(bufs)
        imgs.append(img)
        shapes_all.append(shapes)
    assert dec.decode_batched([s for _, s in keep], R.decode_params(R.OutputFormat.RGB), imgs) == 0
    for (d, _), shapes, bufs in zip(keep, shapes_all, bufs_all):
        ost, want = O.oracle_decode(d, int(R.OutputFormat.RGB), shapes)
        assert ost == 0
        assert G.first_mismatch(G.to_host(bufs)[0], want[0]) is None


@pytest.mark.parametrize("ent", [f for f in DECODABLE if f["ref_parse"]["restart_interval"]][:4],
                         ids=lambda f: f["name"])
def test_device_parsed_damaged_decode(dec, ent):
    """Damaged restart-interval streams parsed on the device decode like the oracle."""
    from tests import gpu_util as G
    for name, d in variants(O.fixture_bytes(ent)).items():
        st, (s,) = dec.parse_device([d])
        if st != R.Status.SUCCESS:
            continue
        nc, css, w, h = dec.image_info(s)
        shapes = G.channel_shapes(R.OutputFormat.RGB, css, w, h)
        bufs, img = G.gpu_buffers(shapes)
        dst = dec.decode(s, R.decode_params(R.OutputFormat.RGB), img)
        ost, want = O.oracle_decode(d, int(R.OutputFormat.RGB), shapes)
        assert dst == ost, name
        if ost == 0:
            assert G.first_mismatch(G.to_host(bufs)[0], want[0]) is None, name
