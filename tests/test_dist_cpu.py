"""Multi-GPU batched decode on CPU (gloo, world_size 2 and 4): the work table rank 0 builds from the
JPEG headers (rocJpegAmdBuildWorkTable), the LPT shards (rocJpegAmdAssignShards) and the one
broadcast (rocjpeg_amd/shard.py) -- SURVEY.md 8e.  No GPU: decode calls are not made here."""
import io
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from rocjpeg_amd import shard as S  # noqa: E402

C4_SIZES = [(640, 480), (1280, 720), (1920, 1080), (2560, 1440), (3840, 2160)]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _c4_blob(count, distinct_per_size=3):
    """A C4-like batch: `count` images uniform over the five C4 sizes by seed (bench.py's
    generator), each a reference to one of 3 real q90 4:2:0 encodes per size (crops of the
    reference mug image + noise, restart interval one MCU row)."""
    from PIL import Image
    base = np.asarray(Image.open(os.path.join(ROOT, "tests", "golden", "img", "mug_420.jpg")).convert("RGB"))
    enc = {}
    for si, (w, h) in enumerate(C4_SIZES):
        for k in range(distinct_per_size):
            rng = np.random.default_rng(100 * si + k)
            y0 = int(rng.integers(0, base.shape[0] - h + 1))
            x0 = int(rng.integers(0, base.shape[1] - w + 1))
            a = base[y0:y0 + h, x0:x0 + w].astype(np.float32) + rng.normal(0.0, 2.0, (h, w, 3))
            b = io.BytesIO()
            Image.fromarray(np.clip(a, 0, 255).astype(np.uint8)).save(
                b, "JPEG", quality=90, subsampling=2, restart_marker_blocks=(w + 15) // 16)
            enc[(si, k)] = b.getvalue()
    keys = sorted(enc)
    parts, offs = [], {}
    pos = 0
    for key in keys:
        offs[key] = pos
        parts.append(enc[key])
        pos += len(enc[key])
    blob = np.frombuffer(b"".join(parts), dtype=np.uint8)
    pick = [((i % 5), (i // 5) % distinct_per_size) for i in range(count)]
    return blob, np.array([offs[p] for p in pick], np.uint64), np.array([len(enc[p]) for p in pick], np.uint32), pick


def test_work_table_fields_and_lpt_balance():
    blob, offs, sizes, pick = _c4_blob(8192)
    t = S.build_work_table(blob, offs, sizes)
    assert len(t) == 8192 and t.dtype.itemsize == 64
    for rec, (si, _) in zip(t[:10], pick[:10]):
        w, h = C4_SIZES[si]
        assert (rec["width"], rec["height"], rec["subsampling"]) == (w, h, 3)
        assert rec["restart_intervals"] == (h + 15) // 16  # one MCU row each
        assert rec["flags"] == 0 and rec["cost"] > 0
        assert 0 < rec["ecs_bytes"] < rec["stream_bytes"]
    for world in (2, 4, 8):
        tt = t.copy()
        cost = S.assign_shards(tt, world)
        # every image exactly once, on a valid shard, dest_device = shard
        assert set(np.unique(tt["shard"])) == set(range(world))
        assert np.array_equal(tt["dest_device"], tt["shard"])
        assert sum(int((tt["shard"] == r).sum()) for r in range(world)) == 8192
        # the shard costs are what the records say, and LPT keeps them within 5 %
        for r in range(world):
            assert int(tt["cost"][tt["shard"] == r].sum()) == int(cost[r])
        assert S.imbalance(cost) <= 0.05, (world, cost)


def test_work_table_flags_bad_and_unsupported():
    good = open(os.path.join(ROOT, "tests", "golden", "img", "p420_q90_ri_256x128.jpg"), "rb").read()
    c411 = open(os.path.join(ROOT, "tests", "golden", "img", "c411_q90_128x64.jpg"), "rb").read()
    prog = open(os.path.join(ROOT, "tests", "golden", "img", "p420_prog_128x96.jpg"), "rb").read()
    junk = b"\x00\x01garbage" * 10
    parts = [good, c411, prog, junk]
    blob = np.frombuffer(b"".join(parts), dtype=np.uint8)
    sizes = np.array([len(p) for p in parts], np.uint32)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    t = S.build_work_table(blob, offs, sizes, base_offset=1000)
    assert list(t["flags"]) == [0, S.WORK_UNSUPPORTED, S.WORK_PROGRESSIVE, S.WORK_BAD]
    assert list(t["stream_offset"]) == [int(o) + 1000 for o in offs]
    assert t["cost"][1] == 0 and t["cost"][3] == 0 and t["cost"][2] > 0
    S.assign_shards(t, 3, shard_devices=[5, 6, 7])
    assert set(t["dest_device"]) <= {5, 6, 7}
    assert (t["shard"] >= 0).all()


def test_work_table_refuses_streams_outside_the_blob():
    """An index whose offset + size runs past the blob is refused before any byte is read, by the
    Python wrapper and by the C entry point itself (its blob_bytes bound)."""
    import ctypes

    from rocjpeg_amd import lib
    good = open(os.path.join(ROOT, "tests", "golden", "img", "p420_q90_ri_256x128.jpg"), "rb").read()
    blob = np.frombuffer(good, dtype=np.uint8)
    offs = np.array([0, 16], np.uint64)
    sizes = np.array([len(good), len(good)], np.uint32)
    with pytest.raises(ValueError):
        S.build_work_table(blob, offs, sizes)
    items = np.zeros(2, dtype=S.WORK_ITEM_DTYPE)
    st = lib().rocJpegAmdBuildWorkTable(ctypes.c_void_p(blob.ctypes.data), len(good),
                                        offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                        sizes.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), 2,
                                        ctypes.c_void_p(items.ctypes.data))
    assert st == -2  # ROCJPEG_STATUS_INVALID_PARAMETER
    huge = np.array([np.uint64(2**63)], np.uint64)
    st = lib().rocJpegAmdBuildWorkTable(ctypes.c_void_p(blob.ctypes.data), len(good),
                                        huge.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                        sizes.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), 1,
                                        ctypes.c_void_p(items.ctypes.data))
    assert st == -2


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from rocjpeg_amd import shard as S_
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    blob, offs, sizes, _ = _c4_blob(2000)
    table = None
    if rank == 0:
        table = S_.build_work_table(blob, offs, sizes)
        S_.assign_shards(table, world)
    got = S_.broadcast_table(table, src=0, device=torch.device("cpu"))
    mine = S_.shard_of(got, rank)
    # each rank reads its images from the shared blob by offset: the bytes are real JPEGs
    first = bytes(blob[int(mine["stream_offset"][0]):int(mine["stream_offset"][0]) + int(mine["stream_bytes"][0])])
    q.put((rank, got.tobytes(), [int(i) for i in mine["index"]], first[:2] == b"\xff\xd8"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_table_broadcast_and_shards_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, tbytes, idx, jpeg_ok = q.get(timeout=180)
        got[r] = (tbytes, idx, jpeg_ok)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the table round-trips bit for bit
    assert all(got[r][0] == got[0][0] for r in range(world))
    table = np.frombuffer(got[0][0], dtype=S.WORK_ITEM_DTYPE)
    assert len(table) == 2000 and np.array_equal(table["index"], np.arange(2000))
    # every image on exactly one rank
    allidx = [i for r in range(world) for i in got[r][1]]
    assert sorted(allidx) == list(range(2000))
    assert all(got[r][2] for r in range(world))
    cost = [int(table["cost"][table["shard"] == r].sum()) for r in range(world)]
    assert S.imbalance(cost) <= 0.05
