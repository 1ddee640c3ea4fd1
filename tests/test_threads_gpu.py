"""Several host threads decoding at once, as the reference's jpegdecodeperf does (one
rocJpegCreate per thread, samples/jpegDecodePerf/jpegdecodeperf.cpp:228-257), and several threads
sharing one handle (the handle serialises its calls: rj_decoder.cpp's per-handle mutex and the
sorted per-stream locks).  Every output is compared with the oracle byte for byte."""
import threading

import numpy as np
import pytest

import rocjpeg_amd as R
from tests import gpu_util as G
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

NAMES = ["p420_q90_ri_256x128", "mug_422", "p444_q95_ri_128x128", "cp420_prog_ri3_160x112", "p422_q90_ri_192x96",
         "p420_q75_nori_200x150", "pp420_opt_200x150", "c440_q90_160x120", "p420_opt_ri_176x144", "mug_400",
         "cp444_prog_ri_136x72", "p420_q90_odd_97x65"]


def _fixtures():
    by = {f["name"]: f for f in O.manifest()}
    return [O.fixture_bytes(by[n]) for n in NAMES]


def _want(datas, fmt):
    out = []
    for d in datas:
        info = R.JpegStream(d).info()
        shapes = G.channel_shapes(fmt, info["subsampling"], info["widths"], info["heights"])
        st, want = O.oracle_decode(d, int(fmt), shapes)
        assert st == 0
        out.append((shapes, want))
    return out


def _run_threads(nthreads, work):
    errs = []
    barrier = threading.Barrier(nthreads)

    def wrap(t):
        try:
            barrier.wait()
            work(t)
        except Exception as e:  # collected: a failing thread fails the test
            errs.append(f"thread {t}: {e!r}")

    th = [threading.Thread(target=wrap, args=(t,)) for t in range(nthreads)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not any(x.is_alive() for x in th), "a decode thread hung"
    assert not errs, errs


@pytest.mark.parametrize("fmt", [R.OutputFormat.RGB, R.OutputFormat.YUV_PLANAR])
def test_threads_own_handles_concurrent(fmt):
    """4 threads, one handle each, different images, single-image and batched calls, 3 rounds."""
    G.torch()
    import torch
    datas = _fixtures()
    wants = _want(datas, fmt)

    def work(t):
        dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
        try:
            mine = list(range(t, len(datas), 4))
            for rnd in range(3):
                streams = [R.JpegStream(datas[k]) for k in mine]
                bufs, imgs = [], []
                for k in mine:
                    shapes = wants[k][0]
                    b = [torch.full(s, 0xA5, dtype=torch.uint8, device="cuda:0") for s in shapes]
                    bufs.append(b)
                    imgs.append(R.make_image([x.data_ptr() for x in b], [s[1] for s in shapes]))
                # the fills run on torch's stream, the decode on the handle's: wait for them
                torch.cuda.synchronize()
                if rnd == 1:  # one batched call over the thread's images
                    st = dec.decode_batched(streams, R.decode_params(fmt), imgs)
                    assert st == 0, R.error_name(st)
                else:  # rocJpegDecode per image (samples/jpegDecode/jpegdecode.cpp:163)
                    for s, img in zip(streams, imgs):
                        st = dec.decode(s, R.decode_params(fmt), img)
                        assert st == 0, R.error_name(st)
                torch.cuda.synchronize()
                for k, b in zip(mine, bufs):
                    for c, (g, w) in enumerate(zip(b, wants[k][1])):
                        assert np.array_equal(g.cpu().numpy(), w), (NAMES[k], rnd, c)
                for s in streams:
                    s.close()
        finally:
            dec.close()

    _run_threads(4, work)


def test_threads_share_one_handle():
    """4 threads on ONE handle: calls serialise on the handle, every result still exact."""
    G.torch()
    import torch
    fmt = R.OutputFormat.RGB
    datas = _fixtures()
    wants = _want(datas, fmt)
    dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
    try:
        def work(t):
            for rnd in range(2):
                for k in range(t, len(datas), 4):
                    s = R.JpegStream(datas[k])
                    shapes = wants[k][0]
                    b = [torch.full(x, 0xA5, dtype=torch.uint8, device="cuda:0") for x in shapes]
                    torch.cuda.synchronize()  # the fill (torch's stream) before the decode (the handle's)
                    st = dec.decode(s, R.decode_params(fmt), R.make_image([x.data_ptr() for x in b], [x[1] for x in shapes]))
                    assert st == 0, R.error_name(st)
                    torch.cuda.synchronize()
                    for c, (g, w) in enumerate(zip(b, wants[k][1])):
                        assert np.array_equal(g.cpu().numpy(), w), (NAMES[k], rnd, c)
                    s.close()

        _run_threads(4, work)
    finally:
        dec.close()


def test_eight_handles_batch1_coalesced():
    """jpegdecodeperf's default shape: 8 threads, a handle each, one image per call
    (jpegdecodeperf.cpp:201-202,228-257).  Concurrent small calls on one device are decoded
    together (rj_coalesce.h); every caller still gets its own images and its own status: threads
    use three output formats (calls with other parameters are not combined), and one thread's
    every third call is an unsupported 4:1:1 stream, which must fail alone while the calls
    combined with it succeed."""
    G.torch()
    import torch
    fmts = [R.OutputFormat.RGB, R.OutputFormat.YUV_PLANAR, R.OutputFormat.NATIVE]
    datas = _fixtures()
    wants = {f: _want(datas, f) for f in fmts}
    by = {f["name"]: f for f in O.manifest()}
    bad = O.fixture_bytes(by["c411_q90_128x64"])
    c0 = R.coalesce_stats()

    def work(t):
        fmt = fmts[t % 3]
        dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
        try:
            for rnd in range(12):
                k = (t + rnd) % len(datas)
                if t == 7 and rnd % 3 == 0:
                    s = R.JpegStream(bad)
                    b = torch.full((64, 384), 0xA5, dtype=torch.uint8, device="cuda:0")
                    torch.cuda.synchronize()
                    st = dec.decode(s, R.decode_params(fmt), R.make_image([b.data_ptr()], [384]))
                    assert st == R.Status.JPEG_NOT_SUPPORTED, R.error_name(st)
                    s.close()
                    continue
                s = R.JpegStream(datas[k])
                shapes = wants[fmt][k][0]
                b = [torch.full(x, 0xA5, dtype=torch.uint8, device="cuda:0") for x in shapes]
                torch.cuda.synchronize()
                st = dec.decode(s, R.decode_params(fmt), R.make_image([x.data_ptr() for x in b], [x[1] for x in shapes]))
                assert st == 0, R.error_name(st)
                for c, (g, w) in enumerate(zip(b, wants[fmt][k][1])):
                    assert np.array_equal(g.cpu().numpy(), w), (NAMES[k], fmt.name, rnd, c)
                s.close()
        finally:
            dec.close()

    _run_threads(8, work)
    c1 = R.coalesce_stats()
    assert c1[0] - c0[0] == 8 * 12  # every call took part
