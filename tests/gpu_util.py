"""GPU-side helpers for the parity tests: destination buffers in HBM (torch is only the
allocator here) and the reference's destination sizing (samples/rocjpeg_samples_utils.h:318-399)."""
import numpy as np

import rocjpeg_amd as R

_torch = None


def torch():
    global _torch
    if _torch is None:
        import torch as t
        if not t.cuda.is_available():
            raise RuntimeError("GPU tests need a GPU")
        _torch = t
    return _torch


def channel_shapes(fmt, css, info_w, info_h, roi=None, rgb_pitch_pad=0):
    """(rows, pitch) per channel as the reference samples allocate them."""
    W, H = info_w[0], info_h[0]
    if roi is not None:
        rw, rh = roi[2] - roi[0], roi[3] - roi[1]
        if 0 < rw <= W and 0 < rh <= H:
            W, H = rw, rh
            info_w = [W, W, W, 0]
            info_h = [H, H, H, 0]
    if fmt == R.OutputFormat.NATIVE:
        return {0: [(H, W)] * 3, 1: [(H, W), (H >> 1, W), (H >> 1, W)], 2: [(H, 2 * W)],
                3: [(H, W), (H >> 1, W)], 5: [(H, W)]}[css]
    if fmt == R.OutputFormat.YUV_PLANAR:
        if css == 5:
            return [(H, W)]
        return [(H, W), (info_h[1] or 1, info_w[1] or 1), (info_h[2] or 1, info_w[2] or 1)]
    if fmt == R.OutputFormat.Y:
        return [(H, W)]
    if fmt == R.OutputFormat.RGB:
        return [(H, 3 * W + rgb_pitch_pad)]
    return [(H, W)] * 3


def gpu_buffers(shapes, fill=0xA5):
    t = torch()
    bufs = [t.full((r, p), fill, dtype=t.uint8, device="cuda") for r, p in shapes]
    img = R.make_image([b.data_ptr() for b in bufs], [b.shape[1] for b in bufs])
    return bufs, img


def to_host(bufs):
    torch().cuda.synchronize()
    return [b.cpu().numpy() for b in bufs]


def first_mismatch(a, b):
    d = np.argwhere(a != b)
    return None if len(d) == 0 else (tuple(d[0]), int(a[tuple(d[0])]), int(b[tuple(d[0])]), len(d))
