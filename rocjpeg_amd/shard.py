"""Multi-GPU batched decode: the per-image work table, LPT shards, one broadcast.

The reference decodes on one device per handle (src/rocjpeg_api.cpp:107-120); its batched call
(src/rocjpeg_decoder.cpp:196-292) is what every rank runs here, on its own shard.  The flow, one
process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI):

  rank 0   build_work_table()   header walk of every image (C-ABI rocJpegAmdBuildWorkTable)
           assign_shards()      greedy LPT on the decode-cost estimate (rocJpegAmdAssignShards)
  all      broadcast_table()    ONE broadcast of the 64-byte records (the only collective)
  rank r   shard_of(table, r)   its images; it parses them from the shared bitstream blob and
                                calls rocJpegDecodeBatched on them

No bitstream, pixel or pointer crosses ranks: `stream_offset` is an offset into a blob every
rank can read (a dataset file on the node), and each rank's output lands on its own GPU
(`dest_device`).  The records are the ctypes/numpy mirror of RocJpegAmdWorkItem
(include/rocjpeg_amd.h).
"""
import ctypes

import numpy as np

from . import Status, lib

WORK_ITEM_DTYPE = np.dtype([
    ("stream_offset", "<u8"), ("stream_bytes", "<u4"), ("ecs_bytes", "<u4"),
    ("width", "<u4"), ("height", "<u4"), ("subsampling", "<i4"), ("restart_intervals", "<u4"),
    ("flags", "<u4"), ("shard", "<i4"), ("dest_device", "<i4"), ("index", "<u4"),
    ("cost", "<u8"), ("reserved", "<u8"),
])
assert WORK_ITEM_DTYPE.itemsize == 64

WORK_PROGRESSIVE = 1
WORK_BAD = 2
WORK_UNSUPPORTED = 4


def _u8_pointer(blob):
    """(ctypes pointer, keep-alive) for a bytes-like or uint8 ndarray blob (no copy for arrays)."""
    if isinstance(blob, np.ndarray):
        if blob.dtype != np.uint8 or not blob.flags["C_CONTIGUOUS"]:
            raise ValueError("blob must be a contiguous uint8 array")
        return ctypes.c_void_p(blob.ctypes.data), blob
    buf = np.frombuffer(blob, dtype=np.uint8)
    return ctypes.c_void_p(buf.ctypes.data), buf


def build_work_table(blob, offsets, sizes, base_offset=0):
    """One record per image of `blob` (images at `offsets`, `sizes` bytes).  `base_offset` is
    added to every stream_offset (the blob is one part of a larger logical blob)."""
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    sizes = np.ascontiguousarray(sizes, dtype=np.uint32)
    n = len(offsets)
    if len(sizes) != n:
        raise ValueError("offsets and sizes differ in length")
    table = np.zeros(n, dtype=WORK_ITEM_DTYPE)
    if n == 0:
        return table
    ptr, keep = _u8_pointer(blob)
    if np.any(offsets.astype(np.uint64) + sizes.astype(np.uint64) > np.uint64(keep.nbytes)):
        raise ValueError("a stream lies outside the blob")
    st = lib().rocJpegAmdBuildWorkTable(ptr, keep.nbytes, offsets.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                        sizes.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n,
                                        ctypes.c_void_p(table.ctypes.data))
    del keep
    if st != 0:
        raise RuntimeError(f"rocJpegAmdBuildWorkTable: {Status(st)!r}")
    if base_offset:
        table["stream_offset"] += np.uint64(base_offset)
    return table


def concat_tables(tables):
    """Join per-part tables into one batch table (index = position in the batch)."""
    t = np.concatenate(tables) if tables else np.zeros(0, dtype=WORK_ITEM_DTYPE)
    t["index"] = np.arange(len(t), dtype=np.uint32)
    return t


def assign_shards(table, num_shards, shard_devices=None):
    """Greedy LPT in place (shard, dest_device); returns each shard's summed cost."""
    n = len(table)
    cost = np.zeros(num_shards, dtype=np.uint64)
    devs = None
    if shard_devices is not None:
        devs = (ctypes.c_int * num_shards)(*[int(d) for d in shard_devices])
    st = lib().rocJpegAmdAssignShards(ctypes.c_void_p(table.ctypes.data) if n else None, n, int(num_shards), devs,
                                      cost.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    if st != 0:
        raise RuntimeError(f"rocJpegAmdAssignShards: {Status(st)!r}")
    return cost


def imbalance(shard_cost):
    """max / mean - 1 of the shards' assigned cost."""
    c = np.asarray(shard_cost, dtype=np.float64)
    return float(c.max() / c.mean() - 1.0) if len(c) and c.mean() > 0 else 0.0


def broadcast_table(table, src=0, device=None):
    """The one collective of the path: rank `src` sends its table (a length, then the records as
    bytes), every rank returns the same table.  `device`: where the tensors live for the backend
    (a CUDA device for nccl/RCCL, cpu for gloo)."""
    import torch
    import torch.distributed as dist
    dev = device if device is not None else torch.device("cpu")
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return table
    rank = dist.get_rank()
    n = torch.tensor([len(table) if rank == src else 0], dtype=torch.int64, device=dev)
    dist.broadcast(n, src=src)
    nbytes = int(n.item()) * WORK_ITEM_DTYPE.itemsize
    if rank == src:
        payload = torch.from_numpy(np.ascontiguousarray(table).view(np.uint8).copy()).to(dev)
    else:
        payload = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    if nbytes:
        dist.broadcast(payload, src=src)
    return payload.cpu().numpy().view(WORK_ITEM_DTYPE).copy()


def shard_of(table, rank):
    """This rank's records, in batch order."""
    return table[table["shard"] == rank]


class Blob:
    """A logical bitstream blob made of parts (e.g. one dataset file per generator rank, each
    memory-mapped): global offset -> bytes."""

    def __init__(self, parts):
        self.parts = list(parts)
        self.bases = np.cumsum([0] + [len(p) for p in self.parts])[:-1].astype(np.uint64)

    def part_base(self, k):
        return int(self.bases[k])

    def get(self, offset, size):
        k = int(np.searchsorted(self.bases, np.uint64(offset), side="right")) - 1
        o = int(offset) - int(self.bases[k])
        return bytes(self.parts[k][o:o + int(size)])


class CommId(ctypes.Structure):
    """RocJpegAmdCommId (= ncclUniqueId): 128 opaque bytes one rank creates and sends to the others."""
    _fields_ = [("internal", ctypes.c_char * 128)]


def comm_unique_id():
    """rocJpegAmdCommGetUniqueId: the id as 128 bytes (one rank calls it; the caller distributes it)."""
    cid = CommId()
    st = lib().rocJpegAmdCommGetUniqueId(ctypes.byref(cid))
    if st != 0:
        raise RuntimeError(f"rocJpegAmdCommGetUniqueId: {Status(st)!r}")
    return ctypes.string_at(ctypes.addressof(cid), 128)  # all 128 bytes (the c_char field would stop at a NUL)


class Comm:
    """The library's own RCCL communicator (include/rocjpeg_amd.h "Multi-GPU batched decode through
    the C ABI"): the work-table broadcast and the sharded batched decode run in C++ against it, so
    a C caller and this binding take the same path."""

    def __init__(self, device_id, nranks, rank, uid):
        cid = CommId()
        ctypes.memmove(ctypes.addressof(cid), bytes(uid), 128)
        self.handle = ctypes.c_void_p()
        st = lib().rocJpegAmdCommInitRank(int(device_id), int(nranks), ctypes.byref(cid), int(rank),
                                           ctypes.byref(self.handle))
        if st != 0:
            raise RuntimeError(f"rocJpegAmdCommInitRank: {Status(st)!r}")
        self.rank, self.nranks, self.device = int(rank), int(nranks), int(device_id)

    def broadcast_table(self, table, count):
        """rank 0's `count` records -> every rank (rocJpegAmdBroadcastWorkTable); returns the table."""
        t = np.ascontiguousarray(table) if table is not None else np.zeros(count, dtype=WORK_ITEM_DTYPE)
        if len(t) != count:
            raise ValueError("table length differs from count")
        st = lib().rocJpegAmdBroadcastWorkTable(self.handle, ctypes.c_void_p(t.ctypes.data) if count else None, count)
        if st != 0:
            raise RuntimeError(f"rocJpegAmdBroadcastWorkTable: {Status(st)!r}")
        return t

    def decode_batched_sharded(self, dec_handle, blob, offsets, sizes, params, destinations):
        """rocJpegAmdDecodeBatchedSharded over the whole batch (`destinations`: a ctypes array of
        RocJpegImage, one per image; this rank writes its own).  Returns (status, table)."""
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        sizes = np.ascontiguousarray(sizes, dtype=np.uint32)
        n = len(offsets)
        table = np.zeros(n, dtype=WORK_ITEM_DTYPE)
        ptr, keep = _u8_pointer(blob)
        st = lib().rocJpegAmdDecodeBatchedSharded(dec_handle, self.handle, ptr, keep.nbytes,
                                                  offsets.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                                  sizes.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n,
                                                  ctypes.byref(params), destinations,
                                                  ctypes.c_void_p(table.ctypes.data))
        del keep
        return st, table

    def close(self):
        if self.handle:
            lib().rocJpegAmdCommDestroy(self.handle)
            self.handle = ctypes.c_void_p()


class Shard:
    """This rank's share of a sharded batch, resident on the handle's GPU (rocJpegAmdShardCreate:
    plan on rank 0 + broadcast + GPU marker-scan parse of this rank's images).  decode() is
    rocJpegAmdShardDecode: rocJpegDecodeBatched over the resident images, image i of the batch
    into destinations[i].  Collective at create: every rank of the communicator calls it."""

    def __init__(self, comm, dec_handle, blob, offsets, sizes):
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        sizes = np.ascontiguousarray(sizes, dtype=np.uint32)
        n = len(offsets)
        self.table = np.zeros(n, dtype=WORK_ITEM_DTYPE)
        self.count = n
        ptr, keep = _u8_pointer(blob)
        self.handle = ctypes.c_void_p()
        self.status = lib().rocJpegAmdShardCreate(dec_handle, comm.handle, ptr, keep.nbytes,
                                                  offsets.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                                  sizes.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n,
                                                  ctypes.c_void_p(self.table.ctypes.data) if n else None,
                                                  ctypes.byref(self.handle))
        del keep

    def images(self):
        """This rank's batch indices."""
        cnt = ctypes.c_int()
        st = lib().rocJpegAmdShardGetImages(self.handle, ctypes.byref(cnt), None, 0)
        if st != 0:
            raise RuntimeError(f"rocJpegAmdShardGetImages: {Status(st)!r}")
        idx = (ctypes.c_int * max(1, cnt.value))()
        lib().rocJpegAmdShardGetImages(self.handle, ctypes.byref(cnt), idx, cnt.value)
        return [idx[k] for k in range(cnt.value)]

    def decode(self, params, destinations):
        """destinations: a ctypes array of RocJpegImage, one per image of the batch."""
        return lib().rocJpegAmdShardDecode(self.handle, ctypes.byref(params), destinations)

    def close(self):
        if self.handle:
            lib().rocJpegAmdShardDestroy(self.handle)
            self.handle = ctypes.c_void_p()
