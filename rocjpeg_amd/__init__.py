"""rocjpeg_amd -- MI355X-native drop-in for rocJPEG's decode path.

The product is the C-ABI library ``librocjpeg_amd.so`` (include/rocjpeg.h); this module is a
thin ctypes mirror of that API for Python callers, tests and bench.py.  It never falls back to
a CPU decoder: without the built library (or without a gfx950 GPU for decode calls) it raises.
"""
import ctypes
import enum
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# RJ_LIB_PATH: an experimental build variant of the same library (development A/B runs)
LIB_PATH = os.environ.get("RJ_LIB_PATH") or os.path.join(_HERE, "librocjpeg_amd.so")

# exported symbols declared by include/rocjpeg.h and include/rocjpeg_amd.h
API_SYMBOLS = (
    "rocJpegStreamCreate", "rocJpegStreamParse", "rocJpegStreamDestroy", "rocJpegCreate", "rocJpegDestroy",
    "rocJpegGetImageInfo", "rocJpegDecode", "rocJpegDecodeBatched", "rocJpegGetErrorName",
)
EXT_SYMBOLS = (
    "rocJpegAmdGetCoalesceStats", "rocJpegAmdGetLastParseTimings", "rocJpegAmdStreamGetInfo", "rocJpegAmdStreamsToDevice", "rocJpegAmdSetProfiling", "rocJpegAmdGetLastTimings",
    "rocJpegAmdSetPathPolicy", "rocJpegAmdGetStream", "rocJpegAmdStreamParseDevice", "rocJpegAmdStreamGetIntervals",
    "rocJpegAmdStreamGetDestuffBlocks", "rocJpegAmdBuildWorkTable", "rocJpegAmdAssignShards",
    "rocJpegAmdCommGetUniqueId", "rocJpegAmdCommInitRank", "rocJpegAmdCommDestroy", "rocJpegAmdCommInfo",
    "rocJpegAmdBroadcastWorkTable", "rocJpegAmdShardPlan", "rocJpegAmdDecodeBatchedSharded",
    "rocJpegAmdShardCreate", "rocJpegAmdShardDecode", "rocJpegAmdShardGetImages", "rocJpegAmdShardDestroy",
    "rocJpegAmdGetAbiVersion", "rocJpegAmdStreamGetLeanTables",
)
ABI_VERSION = 8  # include/rocjpeg_amd.h ROCJPEG_AMD_ABI_VERSION


class Status(enum.IntEnum):  # api/rocjpeg.h:53-67
    SUCCESS = 0
    NOT_INITIALIZED = -1
    INVALID_PARAMETER = -2
    BAD_JPEG = -3
    JPEG_NOT_SUPPORTED = -4
    OUTOF_MEMORY = -5
    EXECUTION_FAILED = -6
    ARCH_MISMATCH = -7
    INTERNAL_ERROR = -8
    IMPLEMENTATION_NOT_SUPPORTED = -9
    HW_JPEG_DECODER_NOT_SUPPORTED = -10
    RUNTIME_ERROR = -11
    NOT_IMPLEMENTED = -12


class Css(enum.IntEnum):  # api/rocjpeg.h:86-94
    CSS_444 = 0
    CSS_440 = 1
    CSS_422 = 2
    CSS_420 = 3
    CSS_411 = 4
    CSS_400 = 5
    UNKNOWN = -1


class OutputFormat(enum.IntEnum):  # api/rocjpeg.h:124-141
    NATIVE = 0
    YUV_PLANAR = 1
    Y = 2
    RGB = 3
    RGB_PLANAR = 4


class Backend(enum.IntEnum):  # api/rocjpeg.h:176-179
    HARDWARE = 0
    HYBRID = 1


class RocJpegImage(ctypes.Structure):
    _fields_ = [("channel", ctypes.c_void_p * 4), ("pitch", ctypes.c_uint32 * 4)]


class _Crop(ctypes.Structure):
    _fields_ = [("left", ctypes.c_int16), ("top", ctypes.c_int16), ("right", ctypes.c_int16),
                ("bottom", ctypes.c_int16)]


class _Target(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32)]


class RocJpegDecodeParams(ctypes.Structure):
    _fields_ = [("output_format", ctypes.c_int), ("crop_rectangle", _Crop), ("target_dimension", _Target)]


class RocJpegAmdTimings(ctypes.Structure):
    _fields_ = [("h2d_ms", ctypes.c_float), ("destuff_ms", ctypes.c_float), ("huffman_ms", ctypes.c_float),
                ("idct_ms", ctypes.c_float), ("output_ms", ctypes.c_float), ("total_ms", ctypes.c_float),
                ("ecs_bytes", ctypes.c_uint64), ("coef_bytes", ctypes.c_uint64), ("output_bytes", ctypes.c_uint64),
                ("images", ctypes.c_uint32), ("intervals", ctypes.c_uint32), ("fused_images", ctypes.c_uint32),
                ("host_ms", ctypes.c_float), ("entropy_chunks_ms", ctypes.c_float),
                ("entropy_resolve_ms", ctypes.c_float), ("entropy_serial_ms", ctypes.c_float),
                ("chunks", ctypes.c_uint32), ("split_intervals", ctypes.c_uint32),
                ("serial_fallbacks", ctypes.c_uint32), ("pipe_groups", ctypes.c_uint32),
                ("pipe_lane_rows", ctypes.c_uint32),
                ("k1_launch_ms_sum", ctypes.c_float), ("k2_launch_ms_sum", ctypes.c_float),
                ("k1_launches", ctypes.c_uint32), ("k2_launches", ctypes.c_uint32),
                ("entry_bytes", ctypes.c_uint64),
                ("prog_entropy_ms", ctypes.c_float), ("prog_rows_ms", ctypes.c_float),
                ("prog_images", ctypes.c_uint32), ("prog_intervals", ctypes.c_uint32),
                ("prog_levels", ctypes.c_uint32), ("prog_pad", ctypes.c_uint32),
                ("prog_coef_bytes", ctypes.c_uint64),
                ("scan_device_streams", ctypes.c_uint32), ("scan_host_fallbacks", ctypes.c_uint32),
                ("prog_kernel_ms", ctypes.c_float * 3), ("prog_kernel_launches", ctypes.c_uint32 * 3),
                ("prog_kernel_bytes", ctypes.c_uint64 * 3),
                ("routed_images", ctypes.c_uint32), ("lean_k1", ctypes.c_uint32),
                ("wide_rows", ctypes.c_uint32), ("lean_split", ctypes.c_uint32),
                ("chunk_k1", ctypes.c_uint32), ("chunk_bytes", ctypes.c_uint32),
                ("chunk_hyp", ctypes.c_uint32), ("lean_five", ctypes.c_uint32),
                ("live", ctypes.c_uint32), ("live_rows", ctypes.c_uint32), ("rest_rows", ctypes.c_uint32),
                ("live_pad", ctypes.c_uint32), ("live_ms", ctypes.c_float), ("rest_ms", ctypes.c_float),
                ("place_ms", ctypes.c_float * 4), ("place_tried", ctypes.c_uint32), ("place_pick", ctypes.c_int32)]


class RocJpegAmdInterval(ctypes.Structure):  # include/rocjpeg_amd.h
    _fields_ = [(k, ctypes.c_uint32) for k in ("src_off", "src_len", "dst_off", "dst_len", "mcu_first", "mcu_count",
                                               "flags", "ent_off", "chunk0", "reserved")]


class RocJpegError(RuntimeError):
    def __init__(self, status, what=""):
        self.status = Status(status) if status in Status._value2member_map_ else status
        super().__init__(f"{what}: {self.status!r}")


_lib = None


def lib():
    """Load librocjpeg_amd.so (raises if it has not been built -- there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.isfile(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run __graft_entry__.build() (make -C rocjpeg_amd)")
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.rocJpegStreamCreate.argtypes = [ctypes.POINTER(vp)]
        L.rocJpegStreamParse.argtypes = [ctypes.c_char_p, sz, vp]
        L.rocJpegStreamDestroy.argtypes = [vp]
        L.rocJpegCreate.argtypes = [i32, i32, ctypes.POINTER(vp)]
        L.rocJpegDestroy.argtypes = [vp]
        L.rocJpegGetImageInfo.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(i32),
                                          ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
        L.rocJpegDecode.argtypes = [vp, vp, ctypes.POINTER(RocJpegDecodeParams), ctypes.POINTER(RocJpegImage)]
        L.rocJpegDecodeBatched.argtypes = [vp, ctypes.POINTER(vp), i32, ctypes.POINTER(RocJpegDecodeParams),
                                           ctypes.POINTER(RocJpegImage)]
        L.rocJpegGetErrorName.argtypes = [i32]
        L.rocJpegGetErrorName.restype = ctypes.c_char_p
        L.rocJpegAmdStreamGetInfo.argtypes = [vp, ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(i32),
                                              ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                              ctypes.POINTER(ctypes.c_uint32)]
        L.rocJpegAmdStreamsToDevice.argtypes = [vp, ctypes.POINTER(vp), i32]
        L.rocJpegAmdSetProfiling.argtypes = [vp, i32]
        L.rocJpegAmdGetLastTimings.argtypes = [vp, ctypes.POINTER(RocJpegAmdTimings)]
        L.rocJpegAmdSetPathPolicy.argtypes = [vp, i32]
        L.rocJpegAmdGetStream.argtypes = [vp, ctypes.POINTER(vp)]
        L.rocJpegAmdStreamParseDevice.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(sz), i32,
                                                  ctypes.POINTER(vp)]
        L.rocJpegAmdStreamGetIntervals.argtypes = [vp, ctypes.POINTER(RocJpegAmdInterval), ctypes.c_uint32,
                                                   ctypes.POINTER(ctypes.c_uint32)]
        L.rocJpegAmdStreamGetDestuffBlocks.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32,
                                                       ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
        L.rocJpegAmdBuildWorkTable.argtypes = [vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                               ctypes.POINTER(ctypes.c_uint32), i32, vp]
        L.rocJpegAmdAssignShards.argtypes = [vp, i32, i32, ctypes.POINTER(i32), ctypes.POINTER(ctypes.c_uint64)]
        L.rocJpegAmdCommGetUniqueId.argtypes = [vp]
        L.rocJpegAmdCommInitRank.argtypes = [i32, i32, vp, i32, ctypes.POINTER(vp)]
        L.rocJpegAmdCommDestroy.argtypes = [vp]
        L.rocJpegAmdCommInfo.argtypes = [vp, ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(i32)]
        L.rocJpegAmdBroadcastWorkTable.argtypes = [vp, vp, i32]
        L.rocJpegAmdShardPlan.argtypes = [vp, vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                          ctypes.POINTER(ctypes.c_uint32), i32, vp]
        L.rocJpegAmdDecodeBatchedSharded.argtypes = [vp, vp, vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                                     ctypes.POINTER(ctypes.c_uint32), i32, vp, vp, vp]
        L.rocJpegAmdShardCreate.argtypes = [vp, vp, vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                            ctypes.POINTER(ctypes.c_uint32), i32, vp, ctypes.POINTER(vp)]
        L.rocJpegAmdShardDecode.argtypes = [vp, vp, vp]
        L.rocJpegAmdShardGetImages.argtypes = [vp, ctypes.POINTER(i32), vp, i32]
        L.rocJpegAmdShardDestroy.argtypes = [vp]
        L.rocJpegAmdGetAbiVersion.argtypes = [ctypes.POINTER(i32)]
        if hasattr(L, "rocJpegAmdStreamGetLeanTables"):  # (absent from same-ABI A/B builds of older commits)
            L.rocJpegAmdStreamGetLeanTables.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
        if hasattr(L, "rocJpegAmdGetLastParseTimings"):
            L.rocJpegAmdGetLastParseTimings.argtypes = [vp, ctypes.POINTER(ctypes.c_double), i32]
        if hasattr(L, "rocJpegAmdGetCoalesceStats"):
            u64p = ctypes.POINTER(ctypes.c_uint64)
            L.rocJpegAmdGetCoalesceStats.argtypes = [u64p, u64p, u64p]
        for name in API_SYMBOLS + EXT_SYMBOLS:
            if name != "rocJpegGetErrorName" and (name in API_SYMBOLS or hasattr(L, name)):
                getattr(L, name).restype = i32
        v = ctypes.c_int()
        if L.rocJpegAmdGetAbiVersion(ctypes.byref(v)) != 0 or v.value != ABI_VERSION:
            raise ImportError(f"{LIB_PATH}: extension ABI {v.value}, this binding needs {ABI_VERSION} (rebuild)")
        _lib = L
    return _lib


def _check(st, what):
    if st != 0:
        raise RocJpegError(st, what)


def error_name(status):
    return lib().rocJpegGetErrorName(int(status)).decode()


class JpegStream:
    """RocJpegStreamHandle (rocJpegStreamCreate / Parse / Destroy).  Keeps the bytes alive: the
    parsed stream borrows them (reference src/rocjpeg_parser.cpp:413)."""

    def __init__(self, data=None):
        self.handle = ctypes.c_void_p()
        _check(lib().rocJpegStreamCreate(ctypes.byref(self.handle)), "rocJpegStreamCreate")
        self._data = None
        if data is not None:
            self.parse(data)

    def parse(self, data):
        self._data = bytes(data)
        st = lib().rocJpegStreamParse(self._data, len(self._data), self.handle)
        _check(st, "rocJpegStreamParse")

    def try_parse(self, data):
        self._data = bytes(data)
        return Status(lib().rocJpegStreamParse(self._data, len(self._data), self.handle))

    def info(self):
        nc, css = ctypes.c_uint8(), ctypes.c_int()
        w, h, nri = (ctypes.c_uint32 * 4)(), (ctypes.c_uint32 * 4)(), ctypes.c_uint32()
        _check(lib().rocJpegAmdStreamGetInfo(self.handle, ctypes.byref(nc), ctypes.byref(css), w, h, ctypes.byref(nri)),
               "rocJpegAmdStreamGetInfo")
        return {"num_components": nc.value, "subsampling": css.value, "widths": list(w), "heights": list(h),
                "restart_intervals": nri.value}

    def intervals(self):
        """The restart-interval table the parse built (rocJpegAmdStreamGetIntervals)."""
        n = ctypes.c_uint32()
        _check(lib().rocJpegAmdStreamGetIntervals(self.handle, None, 0, ctypes.byref(n)), "rocJpegAmdStreamGetIntervals")
        arr = (RocJpegAmdInterval * max(1, n.value))()
        _check(lib().rocJpegAmdStreamGetIntervals(self.handle, arr, n.value, ctypes.byref(n)), "rocJpegAmdStreamGetIntervals")
        return [tuple(getattr(arr[i], k) for k, _ in RocJpegAmdInterval._fields_) for i in range(n.value)]

    def destuff_blocks(self):
        """(ecs_size, [(src_off, len|first<<31, dst_off, zero_end), ...])."""
        n, e = ctypes.c_uint32(), ctypes.c_uint32()
        _check(lib().rocJpegAmdStreamGetDestuffBlocks(self.handle, None, 0, ctypes.byref(n), ctypes.byref(e)),
               "rocJpegAmdStreamGetDestuffBlocks")
        arr = (ctypes.c_uint32 * (4 * max(1, n.value)))()
        _check(lib().rocJpegAmdStreamGetDestuffBlocks(self.handle, arr, n.value, ctypes.byref(n), ctypes.byref(e)),
               "rocJpegAmdStreamGetDestuffBlocks")
        return e.value, [tuple(arr[4 * i:4 * i + 4]) for i in range(n.value)]

    def close(self):
        if self.handle:
            lib().rocJpegStreamDestroy(self.handle)
            self.handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def coalesce_stats():
    """(calls, combined calls, member calls) of the library's coalescing of concurrent small calls
    (include/rocjpeg_amd.h rocJpegAmdGetCoalesceStats)."""
    c, k, m = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().rocJpegAmdGetCoalesceStats(ctypes.byref(c), ctypes.byref(k), ctypes.byref(m)), "coalesce stats")
    return c.value, k.value, m.value


def decode_params(fmt=OutputFormat.RGB, crop=(0, 0, 0, 0)):
    p = RocJpegDecodeParams()
    p.output_format = int(fmt)
    p.crop_rectangle.left, p.crop_rectangle.top, p.crop_rectangle.right, p.crop_rectangle.bottom = crop
    return p


def make_image(ptrs, pitches):
    img = RocJpegImage()
    for i, (p, s) in enumerate(zip(ptrs, pitches)):
        img.channel[i] = p
        img.pitch[i] = s
    return img


class JpegDecoder:
    """RocJpegHandle (rocJpegCreate / Decode / DecodeBatched / Destroy)."""

    def __init__(self, backend=Backend.HARDWARE, device_id=0):
        self.handle = ctypes.c_void_p()
        st = lib().rocJpegCreate(int(backend), int(device_id), ctypes.byref(self.handle))
        if st != 0:
            if self.handle:
                lib().rocJpegDestroy(self.handle)
            self.handle = ctypes.c_void_p()
            raise RocJpegError(st, "rocJpegCreate")

    def image_info(self, stream):
        nc, css = ctypes.c_uint8(), ctypes.c_int()
        w, h = (ctypes.c_uint32 * 4)(), (ctypes.c_uint32 * 4)()
        _check(lib().rocJpegGetImageInfo(self.handle, stream.handle, ctypes.byref(nc), ctypes.byref(css), w, h),
               "rocJpegGetImageInfo")
        return nc.value, css.value, list(w), list(h)

    def decode(self, stream, params, image):
        return Status(lib().rocJpegDecode(self.handle, stream.handle, ctypes.byref(params), ctypes.byref(image)))

    def decode_batched(self, streams, params, images):
        n = len(streams)
        hs = (ctypes.c_void_p * n)(*[s.handle for s in streams])
        arr = (RocJpegImage * n)(*images)
        return Status(lib().rocJpegDecodeBatched(self.handle, hs, n, ctypes.byref(params), arr))

    def parse_device(self, datas):
        """rocJpegAmdStreamParseDevice: parse `datas` (bytes) with the marker scan on this GPU;
        returns (status, [JpegStream])."""
        streams = [JpegStream() for _ in datas]
        for s, d in zip(streams, datas):
            s._data = bytes(d)
        n = len(datas)
        ptrs = (ctypes.c_char_p * n)(*[s._data for s in streams])
        lens = (ctypes.c_size_t * n)(*[len(s._data) for s in streams])
        hs = (ctypes.c_void_p * n)(*[s.handle for s in streams])
        st = Status(lib().rocJpegAmdStreamParseDevice(self.handle, ptrs, lens, n, hs))
        return st, streams

    def last_parse_timings(self):
        """Stage times (ms) of this handle's last parse_device call (rocJpegAmdGetLastParseTimings)."""
        ms = (ctypes.c_double * 6)()
        _check(lib().rocJpegAmdGetLastParseTimings(self.handle, ms, 6), "parse timings")
        keys = ("headers", "resident_alloc", "copy_upload", "kernel_readback", "adopt", "total")
        return {k: round(ms[i], 3) for i, k in enumerate(keys)}

    def streams_to_device(self, streams):
        n = len(streams)
        hs = (ctypes.c_void_p * n)(*[s.handle for s in streams])
        _check(lib().rocJpegAmdStreamsToDevice(self.handle, hs, n), "rocJpegAmdStreamsToDevice")

    def set_profiling(self, on=True):
        _check(lib().rocJpegAmdSetProfiling(self.handle, int(on)), "rocJpegAmdSetProfiling")

    def set_path_policy(self, policy):
        _check(lib().rocJpegAmdSetPathPolicy(self.handle, int(policy)), "rocJpegAmdSetPathPolicy")

    def last_timings(self):
        t = RocJpegAmdTimings()
        _check(lib().rocJpegAmdGetLastTimings(self.handle, ctypes.byref(t)), "rocJpegAmdGetLastTimings")
        out = {}
        for k, _ in RocJpegAmdTimings._fields_:
            v = getattr(t, k)
            out[k] = list(v) if isinstance(v, ctypes.Array) else v
        return out

    def hip_stream(self):
        s = ctypes.c_void_p()
        _check(lib().rocJpegAmdGetStream(self.handle, ctypes.byref(s)), "rocJpegAmdGetStream")
        return s.value

    def close(self):
        if self.handle:
            lib().rocJpegDestroy(self.handle)
            self.handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
