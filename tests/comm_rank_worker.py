"""One rank of the multi-rank communicator test (tests/test_comm_gpu.py): several of these
processes share the one GPU and talk through the library's shared-memory test transport
(RJ_COMM_TEST_SHM, csrc/rj_comm.cpp), so the multi-rank protocol of the work-table exchange --
chunks, status header, checks, error paths -- and the resident sharded decode run with real
device buffers.  Writes one JSON result per rank.  TEST INFRASTRUCTURE.

    python -m tests.comm_rank_worker RANK NRANKS OUT_JSON
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["p420_q90_ri_256x128", "mug_422", "mug_420", "pp420_opt_200x150", "cp444_prog_ri_136x72",
         "cp422_prog_97x67", "mug_400", "p444_q95_ri_128x128", "p422_q90_ri_192x96", "p420_q75_nori_200x150",
         "c440_q90_160x120", "p420_opt_ri_176x144"]


def batch():
    from tests import oracle_lib as O
    by = {f["name"]: f for f in O.manifest()}
    datas = [O.fixture_bytes(by[n]) for n in NAMES]
    sizes = np.array([len(d) for d in datas], np.uint32)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    return datas, np.frombuffer(b"".join(datas), np.uint8), offs, sizes


def main():
    rank, nranks, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    import torch
    import rocjpeg_amd as R
    from rocjpeg_amd import shard as S
    from tests import gpu_util as G
    from tests import oracle_lib as O

    torch.cuda.set_device(0)
    res = {"rank": rank}
    comm = S.Comm(0, nranks, rank, b"\0" * 128)
    dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
    datas, blob, offs, sizes = batch()
    fmt = R.OutputFormat.RGB

    def dests():
        outs, imgs = [], []
        for data in datas:
            info = R.JpegStream(data).info()
            shapes = G.channel_shapes(fmt, info["subsampling"], info["widths"], info["heights"])
            ts = [torch.full(s, 0xA5, dtype=torch.uint8, device="cuda:0") for s in shapes]
            outs.append((ts, shapes))
            imgs.append(R.make_image([t.data_ptr() for t in ts], [s[1] for s in shapes]))
        torch.cuda.synchronize()  # the fills (torch's stream) before the decodes (the handle's)
        return outs, (R.RocJpegImage * len(imgs))(*imgs)

    def check(outs, idx):
        ok = True
        for k in idx:
            ts, shapes = outs[k]
            ost, want = O.oracle_decode(datas[k], int(fmt), shapes)
            ok = ok and ost == 0 and all(np.array_equal(t.cpu().numpy(), w) for t, w in zip(ts, want))
        return ok

    # 1. the resident shard: create (collective), decode twice, every own image oracle-exact
    sh = S.Shard(comm, dec.handle, blob, offs, sizes)
    res["create"] = sh.status
    mine = sh.images() if sh.status == 0 else []
    outs, arr = dests()
    st1 = sh.decode(R.decode_params(fmt), arr)
    st2 = sh.decode(R.decode_params(fmt), arr)
    torch.cuda.synchronize()
    res["decode"] = [st1, st2]
    res["images"] = mine
    res["table_shard"] = [int(x) for x in sh.table["shard"]]
    res["oracle_exact"] = check(outs, mine)
    untouched = [k for k in range(len(datas)) if k not in mine]
    res["others_untouched"] = all(bool((t == 0xA5).all().item()) for k in untouched for t in outs[k][0])
    sh.close()

    # 2. a table larger than one chunk (4096 records): 9,000 records, bit for bit on every rank
    n = 9000
    t = np.zeros(n, dtype=S.WORK_ITEM_DTYPE)
    if rank == 0:
        rng = np.random.default_rng(7)
        t.view(np.uint8)[:] = rng.integers(0, 256, t.nbytes, dtype=np.uint8)
    got = t.copy()
    st = R.lib().rocJpegAmdBroadcastWorkTable(comm.handle, ctypes.c_void_p(got.ctypes.data), n)
    res["big_table"] = [st, O.sha(got.view(np.uint8))]

    # 3. rank 1 passes no destinations: it alone reports INVALID_PARAMETER, after the collective
    outs, arr = dests()
    table = np.zeros(len(datas), dtype=S.WORK_ITEM_DTYPE)
    ptr = ctypes.c_void_p(blob.ctypes.data)
    L = R.lib()
    st = L.rocJpegAmdDecodeBatchedSharded(dec.handle, comm.handle, ptr, blob.nbytes,
                                          offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                          sizes.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), len(datas),
                                          ctypes.byref(R.decode_params(fmt)), None if rank == 1 else arr,
                                          ctypes.c_void_p(table.ctypes.data))
    torch.cuda.synchronize()
    own = [int(i) for i in table["index"][table["shard"] == rank]]
    res["bad_rank1"] = [st, check(outs, own) if st == 0 else None]

    # 4. rank 0's plan fails (a stream outside its blob): every rank returns that status
    bad = sizes.copy()
    if rank == 0:
        bad[-1] += 1
    st = L.rocJpegAmdDecodeBatchedSharded(dec.handle, comm.handle, ptr, blob.nbytes,
                                          offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                          bad.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), len(datas),
                                          ctypes.byref(R.decode_params(fmt)), arr, None)
    res["plan_fail"] = st

    # 5. a rank whose count differs from rank 0's: INVALID_PARAMETER there, the others go on
    cnt = n - 1 if rank == nranks - 1 else n
    got = np.zeros(n, dtype=S.WORK_ITEM_DTYPE)
    st = L.rocJpegAmdBroadcastWorkTable(comm.handle, ctypes.c_void_p(got.ctypes.data), cnt)
    res["count_mismatch"] = st

    # 6. still in step afterwards: one more small exchange
    t3 = np.zeros(3, dtype=S.WORK_ITEM_DTYPE)
    if rank == 0:
        t3["index"] = [5, 6, 7]
    st = L.rocJpegAmdBroadcastWorkTable(comm.handle, ctypes.c_void_p(t3.ctypes.data), 3)
    res["after"] = [st, [int(x) for x in t3["index"]]]

    dec.close()
    comm.close()
    with open(out, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
