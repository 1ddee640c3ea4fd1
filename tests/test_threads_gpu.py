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


def _c2_images(count, seed0=1234):
    import os
    import sys
    sys.path.insert(0, O.ROOT)
    import bench
    bench._init_gen()
    return [bench._make_jpeg((s, bench.WORKLOADS["c2"]["gen"])) for s in range(seed0, seed0 + count)]


def test_eight_handles_batch1_one_bad_caller_latency():
    """jpegdecodeperf's shape with one misbehaving caller: 8 threads, a handle each, one 1080p
    image per call, rounds in lockstep; in the second run thread 7's every call is an unsupported
    stream.  The coalescer checks each member before the combined call (Decoder::Check), so the
    bad call fails alone and the healthy ones are decoded once, together: their outputs stay
    oracle-exact and their p90 call latency stays within 1.5x of the clean run's (+0.3 ms of
    timer slack).  Reference: rocjpeg_decoder.h:174 (per-handle serialisation)."""
    G.torch()
    import time

    import torch
    fmt = R.OutputFormat.RGB
    datas = _c2_images(8, seed0=5150)
    want = [O.oracle_decode(d, int(fmt), [(1080, 5760)])[1][0] for d in datas]
    by = {f["name"]: f for f in O.manifest()}
    bad = O.fixture_bytes(by["c411_q90_128x64"])
    rounds = 40

    def run(with_bad):
        lat = [[] for _ in range(8)]
        outs = [torch.full((1080, 5760), 0xA5, dtype=torch.uint8, device="cuda:0") for _ in range(8)]
        torch.cuda.synchronize()

        def work(t):
            dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
            try:
                good = R.JpegStream(datas[t])
                bs = R.JpegStream(bad)
                bbuf = torch.full((64, 384), 0xA5, dtype=torch.uint8, device="cuda:0")
                torch.cuda.synchronize()
                img = R.make_image([outs[t].data_ptr()], [5760])
                bimg = R.make_image([bbuf.data_ptr()], [384])
                for rnd in range(rounds):
                    barrier.wait()
                    if with_bad and t == 7:
                        st = dec.decode(bs, R.decode_params(fmt), bimg)
                        assert st == R.Status.JPEG_NOT_SUPPORTED, R.error_name(st)
                        continue
                    t0 = time.perf_counter()
                    st = dec.decode(good, R.decode_params(fmt), img)
                    lat[t].append(time.perf_counter() - t0)
                    assert st == 0, R.error_name(st)
                good.close()
                bs.close()
            finally:
                dec.close()

        import threading
        barrier = threading.Barrier(8)
        _run_threads(8, work)
        for t in range(8 if not with_bad else 7):
            assert np.array_equal(outs[t].cpu().numpy(), want[t]), t
        healthy = np.concatenate([np.array(lat[t][5:]) for t in range(7)])  # (the first rounds warm up)
        return float(np.percentile(healthy, 90))

    clean = run(False)
    with_bad = run(True)
    assert with_bad <= 1.5 * clean + 0.3e-3, (clean, with_bad)
