"""Batch-level behaviour on the GPU:
  * a full C2-size call (1024 x 1080p 4:2:0, DRI one MCU row) under the default layout (lean
    K1, longest intervals first), every image compared with the oracle on the device;
  * rocJpegAmdStreamParseDevice with a corrupt header in the batch: no stream is
    left half-parsed, the good streams decode exactly;
  * destinations that are not on the handle's device (pinned and pageable host memory) are
    routed through staging and land byte-identical (SURVEY.md 8e destination routing)."""
import io
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import rocjpeg_amd as R
from tests import oracle_lib as O
from tests.gpu_util import channel_shapes, torch

pytestmark = pytest.mark.gpu

ROOT = O.ROOT


@pytest.fixture(scope="module")
def dec():
    torch()
    d = R.JpegDecoder(R.Backend.HARDWARE, 0)
    yield d
    d.close()


def _c2_images(count, seed0=1234, workload="c2"):
    """The bench's generator (seeded crops of the mug image + N(0,2) noise, Pillow q90, restart
    interval = one MCU row; C2: 1080p 4:2:0, C4: 640x480..3840x2160 by seed), threaded."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    bench._init_gen()
    gen = bench.WORKLOADS[workload]["gen"]
    with ThreadPoolExecutor(16) as ex:
        return list(ex.map(bench._make_jpeg, [(s, gen) for s in range(seed0, seed0 + count)]))


@pytest.fixture(scope="module", params=[{"RJ_SPLIT_OUTLIERS": "1", "RJ_SPLIT_OUTLIER_FRAC": "1"}],
                ids=["split_outliers"])
def split_dec(request):
    """A handle whose lean outlier split has no cap on the share of split intervals (read at
    handle creation): every interval longer than 9/16 of the longest gets a head and a tail
    lane (512-thread workgroups, two per CU), which C2's near-uniform rows never trigger by
    default."""
    torch()
    env = request.param
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
    yield d
    d.close()


def test_c2_1024_split_launch(split_dec):
    """The C2 call with the lean outlier split forced: the intervals near the longest decoded by
    head + tail lanes, every image equal to the oracle."""
    t = torch()
    distinct, copies = 64, 16
    datas = _c2_images(distinct, seed0=4321)
    with ThreadPoolExecutor(16) as ex:
        want = list(ex.map(lambda d: O.oracle_decode(d, int(R.OutputFormat.RGB), [(1080, 5760)]), datas))
    streams = [R.JpegStream(datas[i % distinct]) for i in range(distinct * copies)]
    out = t.full((len(streams), 1080, 5760), 0xA5, dtype=t.uint8, device="cuda")
    imgs = [R.make_image([out[i].data_ptr()], [5760]) for i in range(len(streams))]
    split_dec.set_profiling(True)
    st = split_dec.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs)
    tm = split_dec.last_timings()
    split_dec.set_profiling(False)
    assert st == 0, R.error_name(st)
    assert tm["lean_k1"] == 1 and tm["lean_split"] > 0
    ref = t.from_numpy(np.stack([w[0] for _, w in want])).to("cuda")
    bad = [i for i in range(len(streams)) if not t.equal(out[i], ref[i % distinct])]
    assert not bad, f"{len(bad)} images differ, first {bad[:8]}"


@pytest.fixture(scope="module")
def two_round_dec():
    """A handle with the five-wave lean layout off (RJ_K1_FIVE=0, read at handle creation): the
    intervals past one round of lanes run as a second round."""
    torch()
    old = os.environ.get("RJ_K1_FIVE")
    os.environ["RJ_K1_FIVE"] = "0"
    try:
        d = R.JpegDecoder(R.Backend.HARDWARE, 0)
    finally:
        if old is None:
            del os.environ["RJ_K1_FIVE"]
        else:
            os.environ["RJ_K1_FIVE"] = old
    yield d
    d.close()


def test_c2_1024_two_round_layout(two_round_dec):
    """The C2 call with the overflow intervals as a second round of lean lanes (the layout
    before the fifth waves, still the one for batches past five waves per CU): every image
    equal to the oracle."""
    t = torch()
    distinct, copies = 64, 16
    datas = _c2_images(distinct, seed0=777)
    with ThreadPoolExecutor(16) as ex:
        want = list(ex.map(lambda d: O.oracle_decode(d, int(R.OutputFormat.RGB), [(1080, 5760)]), datas))
    streams = [R.JpegStream(datas[i % distinct]) for i in range(distinct * copies)]
    out = t.full((len(streams), 1080, 5760), 0xA5, dtype=t.uint8, device="cuda")
    imgs = [R.make_image([out[i].data_ptr()], [5760]) for i in range(len(streams))]
    two_round_dec.set_profiling(True)
    st = two_round_dec.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs)
    tm = two_round_dec.last_timings()
    two_round_dec.set_profiling(False)
    assert st == 0, R.error_name(st)
    assert tm["lean_k1"] == 1 and tm["lean_five"] == 0 and tm["lean_split"] == 0
    ref = t.from_numpy(np.stack([w[0] for _, w in want])).to("cuda")
    bad = [i for i in range(len(streams)) if not t.equal(out[i], ref[i % distinct])]
    assert not bad, f"{len(bad)} images differ, first {bad[:8]}"


@pytest.fixture(scope="module")
def split5_dec():
    """A handle whose five-wave lean calls split as many of their longest intervals as the five
    waves per CU hold (RJ_K1_SPLIT5_T near 0, read at handle creation)."""
    torch()
    old = os.environ.get("RJ_K1_SPLIT5_T")
    os.environ["RJ_K1_SPLIT5_T"] = "0.05"
    try:
        d = R.JpegDecoder(R.Backend.HARDWARE, 0)
    finally:
        if old is None:
            del os.environ["RJ_K1_SPLIT5_T"]
        else:
            os.environ["RJ_K1_SPLIT5_T"] = old
    yield d
    d.close()


def _damaged(data, seed):
    """A C2 stream with bytes flipped inside its entropy-coded data (corrupt codes, desynchronised
    intervals), or truncated mid-scan (libjpeg's insufficient-data path)."""
    s = data.index(b"\xff\xda")
    s += 2 + int.from_bytes(data[s + 2:s + 4], "big")
    e = len(data) - 2
    rng = np.random.default_rng(seed)
    if seed % 2:
        cut = s + int((e - s) * (0.3 + 0.6 * rng.random()))
        if data[cut - 1] == 0xFF:
            cut -= 1
        return data[:cut] + b"\xff\xd9"
    buf = bytearray(data)
    for pos in rng.integers(s + 64, e - 64, 40):
        if buf[pos] != 0xFF and buf[pos - 1] != 0xFF and buf[pos + 1] != 0x00:
            nb = buf[pos] ^ (1 << int(rng.integers(0, 8)))
            if nb != 0xFF:
                buf[pos] = nb
    return bytes(buf)


def test_c2_1024_split5_damaged(split5_dec):
    """The five-wave lean launch with its longest intervals split (head + tail lanes in the same
    launch) over a C2 batch with damaged streams: a tail that runs out of data short of its piece
    writes libjpeg's zero blocks itself; every image equal to the oracle."""
    t = torch()
    distinct, copies = 64, 16
    datas = _c2_images(48, seed0=2024)
    datas += [_damaged(datas[k], k) for k in range(16)]
    with ThreadPoolExecutor(16) as ex:
        want = list(ex.map(lambda d: O.oracle_decode(d, int(R.OutputFormat.RGB), [(1080, 5760)]), datas))
    assert all(st == 0 for st, _ in want)
    streams = [R.JpegStream(datas[i % distinct]) for i in range(distinct * copies)]
    out = t.full((len(streams), 1080, 5760), 0xA5, dtype=t.uint8, device="cuda")
    imgs = [R.make_image([out[i].data_ptr()], [5760]) for i in range(len(streams))]
    split5_dec.set_profiling(True)
    st = split5_dec.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs)
    tm = split5_dec.last_timings()
    split5_dec.set_profiling(False)
    assert st == 0, R.error_name(st)
    cu = t.cuda.get_device_properties(0).multi_processor_count
    if 256 * cu < tm["intervals"] <= 320 * cu:
        assert tm["lean_five"] == 1 and tm["lean_split"] > 0
    ref = t.from_numpy(np.stack([w[0] for _, w in want])).to("cuda")
    bad = [i for i in range(len(streams)) if not t.equal(out[i], ref[i % distinct])]
    assert not bad, f"{len(bad)} images differ, first {bad[:8]}"


@pytest.fixture(scope="module", params=["1", "2"], ids=["live", "live_giveup"])
def live_dec(request):
    """A handle with K2 beside K1 (live rows, rj_device.h RjLive; RJ_K2_LIVE read at handle
    creation): "1" the live launch as measured; "2" a test knob under which the live launch never
    sees K1 resident, so every live workgroup leaves without a ticket and the stream-ordered K2
    after K1 takes every published row -- the path a K2 dispatched ahead of K1 falls back to."""
    torch()
    old = os.environ.get("RJ_K2_LIVE")
    os.environ["RJ_K2_LIVE"] = request.param
    try:
        d = R.JpegDecoder(R.Backend.HARDWARE, 0)
    finally:
        if old is None:
            del os.environ["RJ_K2_LIVE"]
        else:
            os.environ["RJ_K2_LIVE"] = old
    yield request.param, d
    d.close()


def test_c2_1024_live_rows_damaged(live_dec):
    """Live rows over a C2 batch with damaged streams (K1 lanes finishing out of order, split
    heads that never meet their tails): the rows published while K1 runs decoded beside it, the
    rest after it, the synced split rows by the split-aware instance -- every row exactly once
    (ticket accounting below) and every image equal to the oracle."""
    mode, dec = live_dec
    t = torch()
    distinct, copies = 64, 16
    datas = _c2_images(48, seed0=3033)
    datas += [_damaged(datas[k], k + 7) for k in range(16)]
    with ThreadPoolExecutor(16) as ex:
        want = list(ex.map(lambda d: O.oracle_decode(d, int(R.OutputFormat.RGB), [(1080, 5760)]), datas))
    assert all(st == 0 for st, _ in want)
    streams = [R.JpegStream(datas[i % distinct]) for i in range(distinct * copies)]
    out = t.full((len(streams), 1080, 5760), 0xA5, dtype=t.uint8, device="cuda")
    imgs = [R.make_image([out[i].data_ptr()], [5760]) for i in range(len(streams))]
    dec.set_profiling(True)
    st = dec.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs)
    tm = dec.last_timings()
    dec.set_profiling(False)
    assert st == 0, R.error_name(st)
    cu = t.cuda.get_device_properties(0).multi_processor_count
    if 256 * cu < tm["intervals"] <= 320 * cu:
        assert tm["live"] == 1 and tm["lean_five"] == 1
        rows = tm["live_rows"] + tm["rest_rows"]
        assert 0 < rows <= 1024 * 68 and rows >= 1024 * 68 - tm["lean_split"]
        if mode == "2":
            assert tm["live_pad"] == 1 and tm["live_rows"] == 0
    ref = t.from_numpy(np.stack([w[0] for _, w in want])).to("cuda")
    bad = [i for i in range(len(streams)) if not t.equal(out[i], ref[i % distinct])]
    assert not bad, f"{len(bad)} images differ, first {bad[:8]}"


@pytest.mark.parametrize("parts", ["2", "3", "4"])
def test_c2_1024_host_streams_split_handles(parts, monkeypatch):
    """The drop-in input path: 1024 C2 streams in host memory (each call stages them over PCIe), on
    a handle with profiling off -- the call is cut into `parts` parts (RJ_SPLIT_PARTS), each decoded
    on its own handle and host thread (rj_decoder.h DecodeSplit), the uploads in order, so a part's
    upload overlaps the earlier parts' kernels.  Every image equal to the oracle; a bad stream in a
    later part fails the call with its status."""
    t = torch()
    monkeypatch.setenv("RJ_SPLIT_PARTS", parts)
    dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
    distinct, copies = 64, 16
    datas = _c2_images(distinct, seed0=6060)
    with ThreadPoolExecutor(16) as ex:
        want = list(ex.map(lambda d: O.oracle_decode(d, int(R.OutputFormat.RGB), [(1080, 5760)]), datas))
    streams = [R.JpegStream(datas[i % distinct]) for i in range(distinct * copies)]
    out = t.full((len(streams), 1080, 5760), 0xA5, dtype=t.uint8, device="cuda")
    imgs = [R.make_image([out[i].data_ptr()], [5760]) for i in range(len(streams))]
    st = dec.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs)
    assert st == 0, R.error_name(st)
    ref = t.from_numpy(np.stack([w[0] for _, w in want])).to("cuda")
    bad = [i for i in range(len(streams)) if not t.equal(out[i], ref[i % distinct])]
    assert not bad, f"{len(bad)} images differ, first {bad[:8]}"
    by = {f["name"]: f for f in O.manifest()}
    s411 = R.JpegStream(O.fixture_bytes(by["c411_q90_128x64"]))
    st = dec.decode_batched(streams[:900] + [s411] + streams[901:], R.decode_params(R.OutputFormat.RGB), imgs)
    assert st == R.Status.JPEG_NOT_SUPPORTED, R.error_name(st)
    st = dec.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs)  # and the handle goes on
    assert st == 0, R.error_name(st)
    dec.close()


def test_c2_1024_default_pipelined_layout(dec):
    t = torch()
    distinct, copies = 256, 4
    datas = _c2_images(distinct)
    with ThreadPoolExecutor(16) as ex:  # the oracle call releases the GIL
        want = list(ex.map(lambda d: O.oracle_decode(d, int(R.OutputFormat.RGB), [(1080, 5760)]), datas))
    assert all(st == 0 for st, _ in want)
    streams = [R.JpegStream(datas[i % distinct]) for i in range(distinct * copies)]
    dec.streams_to_device(streams)
    out = t.full((len(streams), 1080, 5760), 0xA5, dtype=t.uint8, device="cuda")
    imgs = [R.make_image([out[i].data_ptr()], [5760]) for i in range(len(streams))]
    dec.set_profiling(True)
    st = dec.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs)
    tm = dec.last_timings()
    dec.set_profiling(False)
    assert st == 0, R.error_name(st)
    assert tm["images"] == 1024 and tm["intervals"] == 1024 * 68
    # the layout the bench runs: lean K1, one launch, longest intervals first; the 4,096 intervals
    # past one round of four decoder waves per CU run as fifth waves (rj_huff.hip k_huff<RJ_HL_DEC5>)
    assert tm["lean_k1"] == 1 and tm["pipe_groups"] == 1 and tm["split_intervals"] == 0
    cu = t.cuda.get_device_properties(0).multi_processor_count
    five = 256 * cu < 1024 * 68 <= 320 * cu
    assert tm["lean_five"] == int(five)
    # ... with the longest intervals as head + tail lanes in the same launch (RJ_K1_SPLIT5_T)
    assert (tm["lean_split"] > 0) == five
    ref = t.from_numpy(np.stack([w[0] for _, w in want])).to("cuda")
    bad = [i for i in range(len(streams)) if not t.equal(out[i], ref[i % distinct])]
    assert not bad, f"{len(bad)} images differ, first {bad[:8]}"


@pytest.mark.parametrize("tune", ["1", "0"])
def test_c2_1024_entry_placement_search(tune, monkeypatch):
    """The entry-buffer placement search (rj_decoder.h PlaceStep): a fresh handle's first large
    resident calls time K1 + K2 with three entry buffers and keep the fastest; every call's output
    (each with another entry buffer) equals the oracle, the timings report the search, and
    RJ_PLACE_TUNE=0 leaves it off.  Reference path: src/rocjpeg_decoder.cpp:196-292."""
    t = torch()
    monkeypatch.setenv("RJ_PLACE_TUNE", tune)
    dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
    distinct, copies = 64, 16
    datas = _c2_images(distinct, seed0=4242)
    with ThreadPoolExecutor(16) as ex:
        want = list(ex.map(lambda d: O.oracle_decode(d, int(R.OutputFormat.RGB), [(1080, 5760)]), datas))
    streams = [R.JpegStream(datas[i % distinct]) for i in range(distinct * copies)]
    dec.streams_to_device(streams)
    out = t.empty((len(streams), 1080, 5760), dtype=t.uint8, device="cuda")
    imgs = [R.make_image([out[i].data_ptr()], [5760]) for i in range(len(streams))]
    ref = t.from_numpy(np.stack([w[0] for _, w in want])).to("cuda")
    tms = []
    for call in range(6):  # 2 warm calls, 3 measured candidates, then the kept one
        out.fill_(0xA5)
        st = dec.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs)
        assert st == 0, R.error_name(st)
        tms.append(dec.last_timings())
        bad = [i for i in range(len(streams)) if not t.equal(out[i], ref[i % distinct])]
        assert not bad, f"call {call}: {len(bad)} images differ, first {bad[:8]}"
    if tune == "1":
        assert [tm["place_tried"] for tm in tms] == [0, 0, 1, 2, 3, 3]
        assert [tm["place_pick"] for tm in tms[:4]] == [-1] * 4 and 0 <= tms[-1]["place_pick"] <= 2
        assert all(x > 0 for x in tms[-1]["place_ms"][:3]) and tms[-1]["place_ms"][3] == 0
    else:
        assert all(tm["place_tried"] == 0 and tm["place_pick"] == -1 for tm in tms)
    dec.close()


def test_c4_1024_default_outlier_split(dec):
    """BASELINE config C4 on one GPU (the per-rank shard of the 8-GPU config): 1024 mixed-resolution
    4:2:0 images (640x480 ... 3840x2160, RI = one MCU row; 256 distinct x 4) in one
    rocJpegDecodeBatched call under the DEFAULT handle settings.  This is the one config whose
    default layout splits outlier intervals (the 3840-wide rows: head + tail lanes, rj_huff.hip);
    every image is compared with the oracle on the device.  Reference path:
    src/rocjpeg_decoder.cpp:196-292 (DecodeBatched)."""
    t = torch()
    distinct, copies = 256, 4
    datas = _c2_images(distinct, seed0=1234, workload="c4")
    with ThreadPoolExecutor(16) as ex:
        want = list(ex.map(lambda d: O.oracle_decode(d, int(R.OutputFormat.RGB), [_rgb_shape(d)]), datas))
    assert all(st == 0 for st, _ in want)
    sizes = {(w_[0].shape[1] // 3, w_[0].shape[0]) for _, w_ in want}
    assert sizes == {(640, 480), (1280, 720), (1920, 1080), (2560, 1440), (3840, 2160)}
    streams = [R.JpegStream(datas[i % distinct]) for i in range(distinct * copies)]
    dec.streams_to_device(streams)
    nbytes = [want[i % distinct][1][0].size for i in range(len(streams))]
    out = t.full((sum(nbytes),), 0xA5, dtype=t.uint8, device="cuda")
    views, imgs, off = [], [], 0
    for i, nb in enumerate(nbytes):
        h, p = want[i % distinct][1][0].shape
        views.append(out[off:off + nb].view(h, p))
        imgs.append(R.make_image([views[-1].data_ptr()], [p]))
        off += nb
    dec.set_profiling(True)
    st = dec.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs)
    tm = dec.last_timings()
    dec.set_profiling(False)
    assert st == 0, R.error_name(st)
    assert tm["images"] == 1024 and tm["lean_k1"] == 1
    assert tm["lean_split"] > 0, "the default C4 layout splits its outlier intervals"
    bad = []
    for j in range(distinct):
        ref = t.from_numpy(want[j][1][0]).to("cuda")
        bad += [i for i in range(j, len(streams), distinct) if not t.equal(views[i], ref)]
    assert not bad, f"{len(bad)} images differ, first {sorted(bad)[:8]}"


def _planar_shapes(data, fmt):
    info = R.JpegStream(data).info()
    return channel_shapes(fmt, info["subsampling"], info["widths"], info["heights"])


@pytest.mark.parametrize("workload,fmt", [("c3", R.OutputFormat.YUV_PLANAR), ("c2nori", R.OutputFormat.RGB),
                                          ("c5", R.OutputFormat.RGB)],
                         ids=["c3_444_422_yuv_planar", "c2nori_restartless", "c5_progressive_distinct"])
def test_full_batch_other_configs(dec, workload, fmt):
    """BASELINE config C5 (progressive 1080p 4:2:0, 256 distinct images x 4), C3 (1024 x 1080p, 4:4:4 and 4:2:2 alternating, RI one MCU row ->
    YUV_PLANAR: the lean K1 with two sampling geometries in one call) and the C2 no-DRI twin
    (every interval a whole 1080p image: the self-synchronising chunk lanes), each as the bench
    runs it -- 1024 resident images (256 distinct x 4) in one rocJpegDecodeBatched call under the
    default handle settings -- every channel of every image compared with the oracle on the
    device.  Reference path: src/rocjpeg_decoder.cpp:196-292."""
    t = torch()
    distinct, copies = 256, 4
    datas = _c2_images(distinct, seed0=1234, workload=workload)
    shapes = [_planar_shapes(d, fmt) for d in datas]
    with ThreadPoolExecutor(16) as ex:
        want = list(ex.map(lambda k: O.oracle_decode(datas[k], int(fmt), shapes[k]), range(distinct)))
    assert all(st == 0 for st, _ in want)
    streams = [R.JpegStream(datas[i % distinct]) for i in range(distinct * copies)]
    dec.streams_to_device(streams)
    outs, imgs = [], []
    for i in range(len(streams)):
        ts = [t.full(sh, 0xA5, dtype=t.uint8, device="cuda") for sh in shapes[i % distinct]]
        outs.append(ts)
        imgs.append(R.make_image([x.data_ptr() for x in ts], [sh[1] for sh in shapes[i % distinct]]))
    dec.set_profiling(True)
    st = dec.decode_batched(streams, R.decode_params(fmt), imgs)
    tm = dec.last_timings()
    dec.set_profiling(False)
    assert st == 0, R.error_name(st)
    assert tm["images"] == 1024
    if workload == "c3":
        assert tm["lean_k1"] == 1 and {i["subsampling"] for i in (R.JpegStream(d).info() for d in datas[:2])} == {0, 2}
    elif workload == "c5":
        # 256 DISTINCT progressive images (x 4) in one call, the bench's one-grid pipelined
        # layout: every image's ten scans run side by side with producer / consumer waits whose
        # timing now differs from image to image (the 96-copy test had one chain)
        assert tm["prog_images"] == 1024 and len(set(datas)) == distinct
    else:
        assert tm["lean_k1"] == 0 and tm["split_intervals"] == 1024  # one interval per image, chunked
    bad = []
    for j in range(distinct):
        refs = [t.from_numpy(np.ascontiguousarray(w)).to("cuda") for w in want[j][1]]
        bad += [i for i in range(j, len(streams), distinct)
                if not all(t.equal(o, r) for o, r in zip(outs[i], refs))]
    assert not bad, f"{len(bad)} images differ, first {sorted(bad)[:8]}"


def _rgb_shape(data):
    """(rows, pitch) of the RGB destination, from the SOF0 header."""
    i = data.index(b"\xff\xc0")
    h = (data[i + 5] << 8) | data[i + 6]
    w = (data[i + 7] << 8) | data[i + 8]
    return (h, 3 * w)


def _fixture(name):
    ent = next(f for f in O.manifest() if f["name"] == name)
    return O.fixture_bytes(ent)


def test_parse_device_corrupt_header_leaves_no_pending_stream(dec):
    t = torch()
    good = [_fixture("p420_q90_ri_256x128"), _fixture("p444_q95_ri_128x128")]
    bad = bytearray(good[0])
    i = bad.index(b"\xff\xc0")
    bad[i + 2:i + 4] = b"\x00\x01"  # SOF0 segment length 1: the header walk fails
    st, streams = dec.parse_device(good + [bytes(bad)])
    assert st == R.Status.BAD_JPEG
    for s, d in zip(streams[:2], good):
        nc, css, w, h = dec.image_info(s)
        shapes = channel_shapes(R.OutputFormat.RGB, css, w, h)
        buf = t.zeros(shapes[0], dtype=t.uint8, device="cuda")
        assert dec.decode(s, R.decode_params(R.OutputFormat.RGB), R.make_image([buf.data_ptr()], [shapes[0][1]])) == 0
        ost, want = O.oracle_decode(d, int(R.OutputFormat.RGB), shapes)
        assert ost == 0 and np.array_equal(buf.cpu().numpy(), want[0])
    # the stream whose header failed is not decodable
    buf = t.zeros((128, 768), dtype=t.uint8, device="cuda")
    assert dec.decode(streams[2], R.decode_params(R.OutputFormat.RGB), R.make_image([buf.data_ptr()], [768])) != 0


@pytest.mark.parametrize("fmt", [R.OutputFormat.RGB, R.OutputFormat.YUV_PLANAR, R.OutputFormat.NATIVE])
@pytest.mark.parametrize("where", ["pinned", "pageable", "mixed"])
def test_host_destinations_are_routed(dec, fmt, where):
    t = torch()
    names = ["p420_q90_ri_256x128", "p422_q90_ri_192x96", "p444_q95_ri_128x128", "p420_q90_odd_97x65",
             "p420_prog_128x96"]
    datas = [_fixture(n) for n in names]
    streams = [R.JpegStream(d) for d in datas]
    bufs, imgs, shapes = [], [], []
    for k, s in enumerate(streams):
        nc, css, w, h = dec.image_info(s)
        shp = channel_shapes(fmt, css, w, h, rgb_pitch_pad=16 if fmt == R.OutputFormat.RGB else 0)
        shapes.append(shp)
        host = where == "pinned" or (where == "mixed" and k % 2 == 0)
        if where == "pageable" or (where == "mixed" and k % 2 == 1 and k != 3):
            bb = [np.full(sh, 0xA5, np.uint8) for sh in shp]
            ptrs = [b.ctypes.data for b in bb]
        elif host:
            bb = [t.full(sh, 0xA5, dtype=t.uint8).pin_memory() for sh in shp]
            ptrs = [b.data_ptr() for b in bb]
        else:  # device (k == 3 in the mixed batch)
            bb = [t.full(sh, 0xA5, dtype=t.uint8, device="cuda") for sh in shp]
            ptrs = [b.data_ptr() for b in bb]
        bufs.append(bb)
        imgs.append(R.make_image(ptrs, [sh[1] for sh in shp]))
    dec.set_profiling(True)
    st = dec.decode_batched(streams, R.decode_params(fmt), imgs)
    tm = dec.last_timings()
    dec.set_profiling(False)
    assert st == 0, R.error_name(st)
    assert tm["routed_images"] == (4 if where == "mixed" else 5)
    for d, bb, shp in zip(datas, bufs, shapes):
        ost, want = O.oracle_decode(d, int(fmt), shp)
        assert ost == 0
        for b, w_ in zip(bb, want):
            got = b if isinstance(b, np.ndarray) else b.cpu().numpy()
            assert np.array_equal(got, w_)
