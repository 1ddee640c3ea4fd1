"""ctypes access to the CPU oracle (oracle/build/liboracle.so) and the reference builds in
oracle/_ref/.  TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use this module."""
import ctypes
import hashlib
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "liboracle.so")
REF_PARSER_SO = os.path.join(ROOT, "oracle", "_ref", "librefparser.so")
REF_CSC_SO = os.path.join(ROOT, "oracle", "_ref", "librefcsc.so")

_lib = None


def oracle():
    global _lib
    if _lib is None:
        if not os.path.isfile(ORACLE_SO):
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "build/liboracle.so"], check=True)
        _lib = ctypes.CDLL(ORACLE_SO)
        _lib.oj_coef_dims.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
        _lib.oj_decode_coefs.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
        _lib.oj_decode_planes.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
        _lib.oj_decode.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int16, ctypes.c_int16,
                                   ctypes.c_int16, ctypes.c_int16, ctypes.c_void_p, ctypes.c_void_p]
        _lib.oj_cvt_u8.argtypes = [ctypes.c_float]
        _lib.oj_cvt_u8.restype = ctypes.c_uint8
        _lib.oj_csc_pixel.argtypes = [ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_void_p]
    return _lib


def manifest():
    with open(os.path.join(GOLD, "manifest.json")) as f:
        return json.load(f)["fixtures"]


def fixture_bytes(ent):
    with open(os.path.join(GOLD, ent["file"]), "rb") as f:
        return f.read()


def coef_dims(data):
    dims = (ctypes.c_int32 * 8)()
    st = oracle().oj_coef_dims(data, len(data), dims)
    return st, [(dims[2 * c], dims[2 * c + 1]) for c in range(4) if dims[2 * c]]


def decode_coefs(data):
    st, dims = coef_dims(data)
    if st != 0:
        return st, None, dims
    out = np.zeros(sum(w * h * 64 for w, h in dims), np.int16)
    st = oracle().oj_decode_coefs(data, len(data), out.ctypes.data)
    return st, out, dims


def decode_planes(data):
    st, dims = coef_dims(data)
    if st != 0:
        return st, None, dims
    out = np.zeros(sum(w * h * 64 for w, h in dims), np.uint8)
    st = oracle().oj_decode_planes(data, len(data), out.ctypes.data)
    planes, off = [], 0
    for w, h in dims:
        planes.append(out[off:off + w * h * 64].reshape(h * 8, w * 8))
        off += w * h * 64
    return st, planes, dims


def oracle_decode(data, fmt, channel_shapes, crop=(0, 0, 0, 0), fill=0xA5):
    """channel_shapes: list of (rows, pitch) per channel (None = NULL channel)."""
    bufs, ptrs, pitches = [], (ctypes.c_void_p * 4)(), (ctypes.c_uint32 * 4)()
    for i, shp in enumerate(channel_shapes):
        if shp is None:
            bufs.append(None)
            continue
        rows, pitch = shp
        b = np.full((rows, pitch), fill, np.uint8)
        bufs.append(b)
        ptrs[i] = b.ctypes.data
        pitches[i] = pitch
    st = oracle().oj_decode(data, len(data), fmt, crop[0], crop[1], crop[2], crop[3], ptrs, pitches)
    return st, bufs


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def frame_info(data):
    """Frame header fields (SOF0/1/2) in the manifest's ref_parse shape -- for the progressive
    fixtures, which the reference parser rejects (it records zeros for them)."""
    pos = 2
    while pos + 4 <= len(data):
        while data[pos] == 0xFF:
            pos += 1
        m = data[pos]
        ln = (data[pos + 1] << 8) | data[pos + 2]
        if m in (0xC0, 0xC1, 0xC2):
            seg = pos + 1
            h = (data[seg + 3] << 8) | data[seg + 4]
            w = (data[seg + 5] << 8) | data[seg + 6]
            nc = data[seg + 7]
            hv = [[data[seg + 9 + 3 * i] >> 4, data[seg + 9 + 3 * i] & 15] for i in range(nc)]
            hv += [[0, 0]] * (4 - nc)
            return {"ok": 1, "width": w, "height": h, "ncomp": nc, "comp_hv": hv}
        pos += 1 + ln
    raise ValueError("no frame header")
