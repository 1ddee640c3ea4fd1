"""Per-call chunk geometry (rj_decoder.cpp, rj_device.h rj_chunks_cb): a call
whose intervals cannot fill the chip cuts them into chunks of the call's length (the call's
bytes over one round of decoder lanes, at least the handle's floor, 384 B by default), decoded
by the self-synchronising chunk lanes (rj_huff.hip k_huff_chunk) with rj_entropy.hip's
resolution and serial fallback.  Small calls of row-interval images -- the reference's
rocJpegDecode shape -- therefore run the chunk path on intervals of a few KB, with damaged
variants that reach the fallback; a handle whose floor exceeds every interval keeps the lean
K1.  Both must equal the oracle byte for byte.  Reference path: src/rocjpeg_decoder.cpp:104-185
(one image) and 196-292 (batched)."""
import os

import numpy as np
import pytest

import rocjpeg_amd as R
from tests import gpu_util as G
from tests import oracle_lib as O
from tests.test_decode_gpu import _variants

pytestmark = pytest.mark.gpu

RI_1080 = next(f for f in O.manifest() if f["name"] == "p420_q90_ri_1920x1080")


def _handle(env):
    G.torch()
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return R.JpegDecoder(R.Backend.HARDWARE, 0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def dec():
    d = _handle({})
    d.set_profiling(True)
    yield d
    d.close()


@pytest.fixture(scope="module")
def lean_dec():
    d = _handle({"RJ_CHUNK_MIN": str(1 << 30)})
    d.set_profiling(True)
    yield d
    d.close()


def _decode_batch(d, datas, fmt=R.OutputFormat.RGB):
    streams = [R.JpegStream(x) for x in datas]
    bufs_all, imgs, shapes_all = [], [], []
    for s in streams:
        nc, css, w, h = d.image_info(s)
        shapes = G.channel_shapes(fmt, css, w, h)
        bufs, img = G.gpu_buffers(shapes)
        shapes_all.append(shapes)
        bufs_all.append(bufs)
        imgs.append(img)
    st = d.decode_batched(streams, R.decode_params(fmt), imgs)
    return st, d.last_timings(), bufs_all, shapes_all


def _check(datas, bufs_all, shapes_all, fmt=R.OutputFormat.RGB):
    for k, (x, bufs, shapes) in enumerate(zip(datas, bufs_all, shapes_all)):
        ost, want = O.oracle_decode(x, int(fmt), shapes)
        assert ost == 0
        for c, (g, w) in enumerate(zip(G.to_host(bufs), want)):
            assert G.first_mismatch(g, w) is None, (k, c, G.first_mismatch(g, w))


@pytest.mark.parametrize("fmt", [R.OutputFormat.RGB, R.OutputFormat.YUV_PLANAR], ids=["RGB", "YUV_PLANAR"])
def test_one_row_image_is_split_at_the_floor(dec, fmt):
    """One 1080p image with one MCU row per interval (68 intervals of ~4 KB): the call cuts
    every interval into chunks, decodes each speculative chunk under its MCU's 6 phase
    hypotheses, which fit the chip down to the 192-B hypothesis floor (rj_decoder.cpp; without
    hypotheses the floor is 384 B, rj_device.h RJ_CHUNK_MIN_BYTES), and decodes it like the
    oracle."""
    data = O.fixture_bytes(RI_1080)
    st, tm, bufs, shapes = _decode_batch(dec, [data], fmt)
    assert st == 0
    assert tm["chunk_bytes"] == 192 and tm["lean_k1"] == 0 and tm["chunk_k1"] == 1 and tm["chunk_hyp"] == 6
    assert tm["split_intervals"] > 0 and tm["chunks"] > tm["intervals"]
    _check([data], bufs, shapes, fmt)


def test_small_batch_with_damaged_rows(dec):
    """Sixteen row-interval images, their truncated and bit-flipped variants among them: the
    truncated ones end inside a chunked interval (resolution hands it to the serial re-decode,
    libjpeg's insufficient-data rule), the flipped ones must resynchronise where the true
    decode does."""
    data = O.fixture_bytes(RI_1080)
    datas = [data] * 12 + list(_variants(data).values()) + [data]
    st, tm, bufs, shapes = _decode_batch(dec, datas)
    assert st == 0 and tm["split_intervals"] > 0
    _check(datas, bufs, shapes)


def test_floor_above_every_interval_keeps_the_lean_k1(dec, lean_dec):
    """RJ_CHUNK_MIN above every interval: the same call stays one lane per interval (lean K1),
    and both handles write identical bytes."""
    data = O.fixture_bytes(RI_1080)
    st, tm, bufs_l, shapes = _decode_batch(lean_dec, [data, data])
    assert st == 0 and tm["lean_k1"] == 1 and tm["split_intervals"] == 0
    st, tm2, bufs_c, _ = _decode_batch(dec, [data, data])
    assert st == 0 and tm2["lean_k1"] == 0
    for a, b in zip(bufs_l, bufs_c):
        for x, y in zip(G.to_host(a), G.to_host(b)):
            assert np.array_equal(x, y)
    _check([data, data], bufs_c, shapes)


@pytest.fixture(scope="module")
def hyp_decs():
    out = {}
    for h in (1, 2):
        out[h] = _handle({"RJ_K1_HYP": str(h)})
        out[h].set_profiling(True)
    yield out
    for d in out.values():
        d.close()


def test_without_hypotheses_the_floor_is_384(hyp_decs):
    """RJ_K1_HYP=1: the same image at the handle's floor, one lane per chunk."""
    data = O.fixture_bytes(RI_1080)
    st, tm, bufs, shapes = _decode_batch(hyp_decs[1], [data])
    assert st == 0 and tm["chunk_bytes"] == 384 and tm["chunk_hyp"] == 1
    _check([data], bufs, shapes)


def test_phase_hypotheses_match_the_oracle(dec, hyp_decs):
    """Small calls decode every speculative chunk under several MCU-phase hypotheses
    (rj_device.h rj_chunk_lanes): up to the call's largest MCU's 6 blocks (4:2:0), as many as
    fit one round of lanes; a 2-hypothesis handle leaves the phases 2..5 void, and 1 is the
    round-4 layout.  4:2:0, 4:2:2 and gray images with intervals of several chunks, in one call (the
    gray image's MCU has one block: its extra hypothesis lanes stay empty), must equal the oracle
    under each, with the same bytes."""
    by = {f["name"]: f for f in O.manifest()}
    datas = [O.fixture_bytes(by[n]) for n in ("mug_420", "mug_422", "mug_400")] + [O.fixture_bytes(RI_1080)]
    st, tm, bufs, shapes = _decode_batch(dec, datas)
    # (three 4K restart-less images cut at the 384-B floor: as many hypotheses as fit one round)
    assert st == 0 and tm["chunk_k1"] == 1 and 2 <= tm["chunk_hyp"] <= 6, tm
    _check(datas, bufs, shapes)
    for h, d in hyp_decs.items():
        st, tm_h, bufs_h, _ = _decode_batch(d, datas)
        assert st == 0 and tm_h["chunk_hyp"] == h, (h, tm_h["chunk_hyp"])
        for a, b in zip(bufs, bufs_h):
            for x, y in zip(G.to_host(a), G.to_host(b)):
                assert np.array_equal(x, y), h


def test_phase_hypotheses_on_damaged_rows(dec):
    """Truncated and bit-flipped variants under 6 hypotheses: a speculative lane of any phase
    that meets damaged data must still hand the interval to the resolution or the serial
    fallback exactly as the single-hypothesis layout does (the oracle decides)."""
    data = O.fixture_bytes(RI_1080)
    datas = [data] + list(_variants(data).values())
    st, tm, bufs, shapes = _decode_batch(dec, datas)
    assert st == 0 and tm["chunk_hyp"] == 6
    _check(datas, bufs, shapes)
