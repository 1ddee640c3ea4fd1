"""Pins the oracle's per-pixel colour conversion against the reference's OWN HIP kernels
(src/rocjpeg_hip_kernels.cpp compiled unmodified for gfx950 into oracle/_ref/librefcsc.so):
every (Y, U, V) triple, i.e. all 16.7 M inputs, through ColorConvertYUV444ToRGB, and the NV12
kernel's nearest chroma on random planes.  The whole output stage (all 13 kernels a gfx950
device reaches, every format, CSS and ROI rule) is pinned in tests/test_output_stage_ref_gpu.py."""
import ctypes
import os

import numpy as np
import pytest

from tests import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ref():
    if not os.path.isfile(O.REF_CSC_SO):
        pytest.skip("oracle/_ref/librefcsc.so not built (needs /root/reference at build time)")
    from tests import gpu_util as G
    G.torch()
    return ctypes.CDLL(O.REF_CSC_SO)


def oracle_csc(y, u, v):
    n = y.size
    out = np.zeros((n, 3), np.uint8)
    f = O.oracle().oj_csc_bulk
    f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_size_t, ctypes.c_void_p]
    y, u, v = (np.ascontiguousarray(a.reshape(-1)) for a in (y, u, v))
    f(y.ctypes.data, u.ctypes.data, v.ctypes.data, n, out.ctypes.data)
    return out


def test_all_yuv_triples_444(ref):
    from tests import gpu_util as G
    t = G.torch()
    p = np.arange(1 << 24, dtype=np.uint32).reshape(4096, 4096)
    planes = np.stack([(p >> 16) & 255, (p >> 8) & 255, p & 255]).astype(np.uint8)
    src = t.from_numpy(planes.copy()).cuda()
    dst = t.zeros((4096, 4096 * 3), dtype=t.uint8, device="cuda")
    f = ref.ref_yuv444_to_rgb
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                  ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
    f(None, 4096, 4096, dst.data_ptr(), 4096 * 3, src.data_ptr(), 4096, 4096 * 4096, 2 * 4096 * 4096)
    t.cuda.synchronize()
    got = dst.cpu().numpy().reshape(-1, 3)
    want = oracle_csc(planes[0], planes[1], planes[2])
    bad = np.argwhere((got != want).any(1))
    assert len(bad) == 0, (len(bad), got[bad[0][0]], want[bad[0][0]], planes[:, bad[0][0] // 4096, bad[0][0] % 4096])


def test_nv12_kernel_nearest_chroma(ref):
    from tests import gpu_util as G
    t = G.torch()
    rng = np.random.default_rng(7)
    W, H = 256, 64
    Y = rng.integers(0, 256, (H, W), dtype=np.uint8)
    U = rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8)
    V = rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8)
    uv = np.stack([U, V], -1).reshape(H // 2, W)
    dy, duv = t.from_numpy(Y).cuda(), t.from_numpy(uv.copy()).cuda()
    dst = t.zeros((H, 3 * W), dtype=t.uint8, device="cuda")
    f = ref.ref_nv12_to_rgb
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                  ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
    f(None, W, H, dst.data_ptr(), 3 * W, dy.data_ptr(), W, duv.data_ptr(), W)
    t.cuda.synchronize()
    up_u = np.repeat(np.repeat(U, 2, 0), 2, 1)
    up_v = np.repeat(np.repeat(V, 2, 0), 2, 1)
    want = oracle_csc(Y, up_u, up_v).reshape(H, 3 * W)
    assert np.array_equal(dst.cpu().numpy(), want)
