"""Multi-GPU batched decode through the C ABI (include/rocjpeg_amd.h, csrc/rj_comm.cpp): the
library's own RCCL communicator, the work-table broadcast and rocJpegAmdDecodeBatchedSharded
(the reference's batched call is src/rocjpeg_decoder.cpp:196-292).  The GPU box
has one MI355X, and RCCL refuses two ranks on one device, so these run the communicator at one
rank: the whole sharded call (table build, LPT, broadcast, parse, decode) from Python and from a
plain C program (tests/c/jpegdecode_sharded_c.c, one forked process per rank), every image
compared with the oracle.  The multi-rank protocol (chunked table exchange with rank 0's status,
error paths, the resident shard entry points) runs with 3 ranks sharing the GPU through the
library's shared-memory test transport (RJ_COMM_TEST_SHM).  The table logic over gloo at 2 and 4
ranks is tests/test_dist_cpu.py."""
import ctypes
import os
import struct
import subprocess

import numpy as np
import pytest

import rocjpeg_amd as R
from rocjpeg_amd import shard as S
from tests import gpu_util as G
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

NAMES = ["p420_q90_ri_256x128", "mug_422", "mug_420", "pp420_opt_200x150", "cp444_prog_ri_136x72",
         "cp422_prog_97x67", "mug_400"]
EXE = os.path.join(O.ROOT, "tests", "c", "jpegdecode_sharded_c")


def _batch():
    by = {f["name"]: f for f in O.manifest()}
    datas = [O.fixture_bytes(by[n]) for n in NAMES]
    sizes = np.array([len(d) for d in datas], np.uint32)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    return datas, np.frombuffer(b"".join(datas), np.uint8), offs, sizes


def test_comm_one_rank_sharded_decode_matches_oracle():
    G.torch()
    import torch
    datas, blob, offs, sizes = _batch()
    comm = S.Comm(0, 1, 0, S.comm_unique_id())
    r, n, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    assert R.lib().rocJpegAmdCommInfo(comm.handle, ctypes.byref(r), ctypes.byref(n), ctypes.byref(d)) == 0
    assert (r.value, n.value, d.value) == (0, 1, 0)
    dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
    try:
        for fmt in (R.OutputFormat.RGB, R.OutputFormat.YUV_PLANAR):
            outs, imgs = [], []
            for data in datas:
                info = R.JpegStream(data).info()
                shapes = G.channel_shapes(fmt, info["subsampling"], info["widths"], info["heights"])
                ts = [torch.full(s, 0xA5, dtype=torch.uint8, device="cuda:0") for s in shapes]
                outs.append((ts, shapes))
                imgs.append(R.make_image([t.data_ptr() for t in ts], [s[1] for s in shapes]))
            arr = (R.RocJpegImage * len(imgs))(*imgs)
            torch.cuda.synchronize()  # the fills before the decode (another stream)
            st, table = comm.decode_batched_sharded(dec.handle, blob, offs, sizes, R.decode_params(fmt), arr)
            assert st == 0, R.error_name(st)
            torch.cuda.synchronize()
            assert (table["shard"] == 0).all() and list(table["index"]) == list(range(len(datas)))
            assert list(table["flags"][[3, 4, 5]]) == [S.WORK_PROGRESSIVE] * 3 and (table["flags"][[0, 1, 2, 6]] == 0).all()
            for data, (ts, shapes) in zip(datas, outs):
                ost, want = O.oracle_decode(data, int(fmt), shapes)
                assert ost == 0
                for t, w in zip(ts, want):
                    assert np.array_equal(t.cpu().numpy(), w)
        # the broadcast alone at one rank is the identity
        t = np.zeros(3, dtype=S.WORK_ITEM_DTYPE)
        t["index"] = [7, 8, 9]
        assert np.array_equal(comm.broadcast_table(t, 3), t)
    finally:
        dec.close()
        comm.close()


def test_sharded_decode_refuses_bad_arguments():
    G.torch()
    datas, blob, offs, sizes = _batch()
    comm = S.Comm(0, 1, 0, S.comm_unique_id())
    dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
    try:
        arr = (R.RocJpegImage * len(datas))()
        bad = sizes.copy()
        bad[-1] += 1  # runs past the blob
        st, _ = comm.decode_batched_sharded(dec.handle, blob, offs, bad, R.decode_params(R.OutputFormat.RGB), arr)
        assert st == int(R.Status.INVALID_PARAMETER)
        L = R.lib()
        assert L.rocJpegAmdDecodeBatchedSharded(dec.handle, None, None, 0, None, None, 0, None, None, None) == \
            int(R.Status.INVALID_PARAMETER)
        assert L.rocJpegAmdCommInitRank(0, 2, None, 0, ctypes.byref(ctypes.c_void_p())) == int(R.Status.INVALID_PARAMETER)
    finally:
        dec.close()
        comm.close()


def test_plain_c_caller_sharded(tmp_path):
    """tests/c/jpegdecode_sharded_c.c: gcc, include/rocjpeg*.h, librocjpeg_amd.so and the HIP
    runtime -- no Python in the decode process; one rank here (one GPU)."""
    if not os.access(EXE, os.X_OK):
        pytest.fail(f"{EXE} not built (make -C tests/c; __graft_entry__.build() does it)")
    datas, _, _, _ = _batch()
    files = []
    for k, d in enumerate(datas):
        p = tmp_path / f"{k}.jpg"
        p.write_bytes(d)
        files.append(str(p))
    fmt = R.OutputFormat.RGB
    prefix = str(tmp_path / "out")
    r = subprocess.run([EXE, "1", str(int(fmt)), prefix] + files, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = open(prefix + ".0", "rb").read()
    got, pos = {}, 0
    while pos < len(raw):
        idx, nbytes = struct.unpack_from("<II", raw, pos)
        got[idx] = raw[pos + 8:pos + 8 + nbytes]
        pos += 8 + nbytes
    assert sorted(got) == list(range(len(datas)))
    for k, data in enumerate(datas):
        info = R.JpegStream(data).info()
        shapes = G.channel_shapes(fmt, info["subsampling"], info["widths"], info["heights"])
        ost, want = O.oracle_decode(data, int(fmt), shapes)
        assert ost == 0 and got[k] == b"".join(np.ascontiguousarray(w).tobytes() for w in want)


def test_multi_rank_protocol_shared_gpu(tmp_path):
    """3 processes, one GPU, the library's communicator over its shared-memory test transport
    (csrc/rj_comm.cpp ShmBus; RCCL refuses two ranks on one device): the same chunks, header and
    checks as the RCCL broadcast.  tests/comm_rank_worker.py runs, on every rank in step:
    the resident shard (rocJpegAmdShardCreate / Decode twice, own images oracle-exact, the rest
    untouched), a 9,000-record table (three chunks), a rank with no destinations, a failed plan
    on rank 0, a rank with a different count, and one more exchange to show the ranks stayed in
    step (no error path may leave a rank waiting in the collective)."""
    import json
    import sys
    world = 3
    shm = f"/dev/shm/rj_comm_test_{os.getpid()}"
    if os.path.exists(shm):
        os.unlink(shm)
    # the test build of the library: the product library has no test transport
    env = dict(os.environ, RJ_COMM_TEST_SHM=shm,
               RJ_LIB_PATH=os.path.join(O.ROOT, "rocjpeg_amd", "librocjpeg_amd_testcomm.so"))
    outs = [str(tmp_path / f"r{r}.json") for r in range(world)]
    procs = [subprocess.Popen([sys.executable, "-m", "tests.comm_rank_worker", str(r), str(world), outs[r]],
                              cwd=O.ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world)]
    try:
        logs = [p.communicate(timeout=240)[0] for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        if os.path.exists(shm):
            os.unlink(shm)
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    res = [json.load(open(o)) for o in outs]
    n = len(res[0]["table_shard"])
    assert all(r["create"] == 0 and r["decode"] == [0, 0] for r in res)
    assert all(r["table_shard"] == res[0]["table_shard"] for r in res)
    assert sorted(i for r in res for i in r["images"]) == list(range(n))
    assert all(len(r["images"]) > 0 for r in res)
    assert all(r["oracle_exact"] and r["others_untouched"] for r in res)
    assert all(r["big_table"][0] == 0 and r["big_table"][1] == res[0]["big_table"][1] for r in res)
    inv = int(R.Status.INVALID_PARAMETER)
    assert res[1]["bad_rank1"][0] == inv
    assert all(res[r]["bad_rank1"] == [0, True] for r in (0, 2))
    assert all(r["plan_fail"] == inv for r in res)
    assert [r["count_mismatch"] for r in res] == [0, 0, inv]
    assert all(r["after"] == [0, [5, 6, 7]] for r in res)
