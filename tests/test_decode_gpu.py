"""Parity of the HIP decode path (through the C ABI) with the CPU oracle, byte for byte, over
every committed fixture, every output format, batches, ROI crops and the error paths."""
import numpy as np
import pytest

import rocjpeg_amd as R
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

FIX = O.manifest()
DECODABLE = [f for f in FIX if "libjpeg_coef_sha256" in f and f["ref_parse"]["css"] in (0, 1, 2, 3, 5)]
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
    # progressive: the reference parser fails on the SOF2 stream (comp id mismatch at SOS)
    assert R.JpegStream().try_parse(O.fixture_bytes(by["p420_prog_128x96"])) == R.Status.BAD_JPEG
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
