"""Pins the oracle's output stage (oracle/jpeg_oracle.c oj_output_stage: every output format,
chroma replication rule and ROI quirk) against the reference's OWN HIP kernels, run on random
component planes.

`RefOutputStage` replays RocJpegDecoder's output dispatch (src/rocjpeg_decoder.cpp:143-180) and
its helpers -- CopyChannel (:372-399), GetChromaHeight (:413-434), ColorConvertToRGB (:450-494),
ColorConvertToRGBPlanar (:511-557), GetPlanarYUVOutputFormat (:576-605), GetYOutputFormat
(:620-636) -- over a VA surface laid out as the VCN decoder leaves it (fourcc per
src/rocjpeg_vaapi_decoder.cpp:612-632: 444P, 422V for 4:4:0, packed YUYV for 4:2:2, NV12,
Y800), calling the 13 kernels of src/rocjpeg_hip_kernels.cpp that a gfx950 device can reach
(compiled unmodified into oracle/_ref/librefcsc.so, oracle/ref_shims/ref_csc_shim.cpp).
Plane copies (hipMemcpy2DAsync in CopyChannel) are replayed with torch copies.

The product path is pinned to the oracle elsewhere (tests/test_decode_gpu.py); this closes the
chain oracle == reference kernels for 4:4:4, 4:4:0, 4:2:2 (YUYV), 4:2:0 (NV12) and 4:0:0, with
and without ROI (even and odd crop edges)."""
import ctypes
import os
import zlib

import numpy as np
import pytest

import rocjpeg_amd as R
from tests import oracle_lib as O
from tests.gpu_util import channel_shapes

pytestmark = pytest.mark.gpu

CSS = {"444": 0, "440": 1, "422": 2, "420": 3, "400": 5}
FMTS = [R.OutputFormat.NATIVE, R.OutputFormat.YUV_PLANAR, R.OutputFormat.Y, R.OutputFormat.RGB,
        R.OutputFormat.RGB_PLANAR]
W, H = 256, 128          # picture size
PW, PH = 448, 200        # decoded (padded) luma plane: every ROI read stays inside it
ROIS = {"full": None, "even": (32, 16, W - 32, H - 16), "odd": (17, 9, 17 + 101, 9 + 61)}


@pytest.fixture(scope="module")
def ref():
    if not os.path.isfile(O.REF_CSC_SO):
        pytest.skip("oracle/_ref/librefcsc.so not built (needs /root/reference at build time)")
    from tests import gpu_util as G
    G.torch()
    lib = ctypes.CDLL(O.REF_CSC_SO)
    u32, vp = ctypes.c_uint32, ctypes.c_void_p
    sig = {
        "ref_yuv444_to_rgb": [vp, u32, u32, vp, u32, vp, u32, u32, u32],
        "ref_yuv440_to_rgb": [vp, u32, u32, vp, u32, vp, u32, u32, u32],
        "ref_yuyv_to_rgb": [vp, u32, u32, vp, u32, vp, u32],
        "ref_nv12_to_rgb": [vp, u32, u32, vp, u32, vp, u32, vp, u32],
        "ref_yuv400_to_rgb": [vp, u32, u32, vp, u32, vp, u32],
        "ref_yuv444_to_rgb_planar": [vp, u32, u32, vp, vp, vp, u32, vp, u32, u32, u32],
        "ref_yuv440_to_rgb_planar": [vp, u32, u32, vp, vp, vp, u32, vp, u32, u32, u32],
        "ref_yuyv_to_rgb_planar": [vp, u32, u32, vp, vp, vp, u32, vp, u32],
        "ref_nv12_to_rgb_planar": [vp, u32, u32, vp, vp, vp, u32, vp, u32, vp, u32],
        "ref_yuv400_to_rgb_planar": [vp, u32, u32, vp, vp, vp, u32, vp, u32],
        "ref_yuyv_extract_y": [vp, u32, u32, vp, u32, vp, u32],
        "ref_uv_to_planar": [vp, u32, u32, vp, vp, u32, vp, u32],
        "ref_yuyv_to_planar": [vp, u32, u32, vp, vp, vp, u32, u32, vp, u32],
    }
    for name, args in sig.items():
        getattr(lib, name).argtypes = args
    return lib


def make_planes(css, seed):
    """Random decoded component planes (luma PW x PH; chroma per the sampling)."""
    rng = np.random.default_rng(seed)
    cw, ch = {0: (PW, PH), 1: (PW, PH // 2), 2: (PW // 2, PH), 3: (PW // 2, PH // 2), 5: (0, 0)}[css]
    planes = [rng.integers(0, 256, (PH, PW), dtype=np.uint8)]
    if cw:
        planes += [rng.integers(0, 256, (ch, cw), dtype=np.uint8) for _ in range(2)]
    return planes


def make_surface(css, planes):
    """The VA surface (one linear buffer) + offsets/pitches, as rocjpeg_vaapi_decoder.cpp maps it
    into HIP (HipInteropDeviceMem: offset[3], pitch[3])."""
    Y = planes[0]
    if css == 2:  # packed YUYV: Y0 U0 Y1 V0
        s = np.empty((PH, 2 * PW), np.uint8)
        s[:, 0::4], s[:, 2::4] = Y[:, 0::2], Y[:, 1::2]
        s[:, 1::4], s[:, 3::4] = planes[1], planes[2]
        return s.reshape(-1), [0, 0, 0], [2 * PW, 0, 0]
    if css == 3:  # NV12: Y, then interleaved UV rows
        uv = np.stack([planes[1], planes[2]], -1).reshape(PH // 2, PW)
        return np.concatenate([Y.reshape(-1), uv.reshape(-1)]), [0, PW * PH, 0], [PW, PW, 0]
    if css == 5:
        return Y.reshape(-1), [0, 0, 0], [PW, 0, 0]
    u, v = planes[1].reshape(-1), planes[2].reshape(-1)
    return np.concatenate([Y.reshape(-1), u, v]), [0, Y.size, Y.size + u.size], [PW, PW, PW]


class RefOutputStage:
    """rocjpeg_decoder.cpp:124-180 and helpers, over a device surface, with the reference kernels."""

    def __init__(self, lib, t, css, surface, offsets, pitches):
        self.lib, self.t, self.css = lib, t, css
        pad = 1 << 16  # the kernels read whole 8/16-byte groups past the last pixel
        self.surf = t.zeros(surface.size + pad, dtype=t.uint8, device="cuda")
        self.surf[:surface.size].copy_(t.from_numpy(surface))
        self.base = self.surf.data_ptr()
        self.off, self.pitch = offsets, pitches

    def copy_channel(self, rows, c, dst, dpitch, roi):  # CopyChannel :372-399 (hipMemcpy2DAsync)
        if self.pitch[c] == 0 or dpitch[c] == 0 or dst[c] is None:
            return
        ro = 0
        if roi:
            left, top = roi[0], roi[1]
            if self.css in (3, 1) and c in (1, 2):
                top >>= 1
            if self.css == 2:
                left *= 2
            ro = top * self.pitch[c] + left
        start = self.off[c] + ro
        src = self.surf.as_strided((rows, dpitch[c]), (self.pitch[c], 1), start)
        dst[c][:rows, :dpitch[c]].copy_(src)

    def run(self, fmt, roi, dst, dpitch):
        css, L = self.css, self.lib
        valid = roi is not None and 0 < roi[2] - roi[0] <= W and 0 < roi[3] - roi[1] <= H
        roi = roi if valid else None
        pw, ph = (roi[2] - roi[0], roi[3] - roi[1]) if roi else (W, H)
        chroma_h = {3: ph >> 1, 0: ph, 5: 0, 2: ph, 1: ph >> 1}[css]  # GetChromaHeight :413-434
        ptr = [d.data_ptr() if d is not None else None for d in dst]
        if fmt == R.OutputFormat.NATIVE:
            self.copy_channel(ph, 0, dst, dpitch, roi)
            if css == 3:
                self.copy_channel(chroma_h, 1, dst, dpitch, roi)
            elif css in (0, 1):
                self.copy_channel(chroma_h, 1, dst, dpitch, roi)
                self.copy_channel(chroma_h, 2, dst, dpitch, roi)
        elif fmt == R.OutputFormat.YUV_PLANAR:  # GetPlanarYUVOutputFormat :576-605
            ro = 0
            if roi and css == 3:
                ro = (roi[1] >> 1) * self.pitch[1] + roi[0]
            elif roi and css == 2:
                ro = roi[1] * self.pitch[0] + roi[0] * 2
            if css == 2:
                L.ref_yuyv_to_planar(None, pw, ph, ptr[0], ptr[1], ptr[2], dpitch[0], dpitch[1], self.base + ro,
                                     self.pitch[0])
            else:
                self.copy_channel(ph, 0, dst, dpitch, roi)
                if css == 3:
                    L.ref_uv_to_planar(None, pw >> 1, ph >> 1, ptr[1], ptr[2], dpitch[1],
                                       self.base + self.off[1] + ro, self.pitch[1])
                elif css in (0, 1):
                    self.copy_channel(chroma_h, 1, dst, dpitch, roi)
                    self.copy_channel(chroma_h, 2, dst, dpitch, roi)
        elif fmt == R.OutputFormat.Y:  # GetYOutputFormat :620-636
            if css == 2:
                ro = roi[1] * self.pitch[0] + roi[0] * 2 if roi else 0
                L.ref_yuyv_extract_y(None, pw, ph, ptr[0], dpitch[0], self.base + ro, self.pitch[0])
            else:
                self.copy_channel(ph, 0, dst, dpitch, roi)
        else:  # ColorConvertToRGB :450-494 / ColorConvertToRGBPlanar :511-557
            ro = ruv = 0
            if roi:
                top, left = roi[1], roi[0]
                if css in (1, 3):
                    ruv = (top >> 1) * self.pitch[1] + left
                elif css == 2:
                    left *= 2
                ro = top * self.pitch[0] + left
            b, p0 = self.base + ro, self.pitch[0]
            if fmt == R.OutputFormat.RGB:
                d = (ptr[0], dpitch[0])
                if css == 0:
                    L.ref_yuv444_to_rgb(None, pw, ph, *d, b, p0, self.off[1] + ro, self.off[2] + ro)
                elif css == 1:  # the reference leaves `+ roi_uv_offset` commented out (:468-471)
                    L.ref_yuv440_to_rgb(None, pw, ph, *d, b, p0, self.off[1], self.off[2])
                elif css == 2:
                    L.ref_yuyv_to_rgb(None, pw, ph, *d, b, p0)
                elif css == 3:
                    L.ref_nv12_to_rgb(None, pw, ph, *d, b, p0, self.base + self.off[1] + ruv, self.pitch[1])
                else:
                    L.ref_yuv400_to_rgb(None, pw, ph, *d, b, p0)
            else:
                d = (ptr[0], ptr[1], ptr[2], dpitch[0])
                if css == 0:
                    L.ref_yuv444_to_rgb_planar(None, pw, ph, *d, b, p0, self.off[1] + ro, self.off[2] + ro)
                elif css == 1:
                    L.ref_yuv440_to_rgb_planar(None, pw, ph, *d, b, p0, self.off[1], self.off[2])
                elif css == 2:
                    L.ref_yuyv_to_rgb_planar(None, pw, ph, *d, b, p0)
                elif css == 3:
                    L.ref_nv12_to_rgb_planar(None, pw, ph, *d, b, p0, self.base + self.off[1] + ruv, self.pitch[1])
                else:
                    L.ref_yuv400_to_rgb_planar(None, pw, ph, *d, b, p0)
        self.t.cuda.synchronize()


def oracle_output(css, planes, fmt, roi, shapes, fill):
    """oj_output_stage on the same planes into host buffers pre-filled with `fill`."""
    lib = O.oracle()
    f = lib.oj_output_stage
    f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 4 + [ctypes.c_int16] * 4 + [ctypes.c_void_p] * 2
    keep = [np.ascontiguousarray(p) for p in planes] + [np.zeros((1, 1), np.uint8)] * (3 - len(planes))
    pl = (ctypes.c_void_p * 3)(*[k.ctypes.data for k in keep[:3]])
    pw = (ctypes.c_int32 * 3)(*[k.shape[1] if k.size > 1 else 0 for k in keep[:3]])
    ph = (ctypes.c_int32 * 3)(*[k.shape[0] if k.size > 1 else 0 for k in keep[:3]])
    bufs = [np.full(s, fill, np.uint8) for s in shapes]
    chp = (ctypes.c_void_p * 4)(*([b.ctypes.data for b in bufs] + [None] * (4 - len(bufs))))
    pit = (ctypes.c_uint32 * 4)(*([s[1] for s in shapes] + [0] * (4 - len(shapes))))
    cl, ct, cr, cb = roi if roi else (0, 0, 0, 0)
    st = f(pl, pw, ph, css, W, H, int(fmt), cl, ct, cr, cb, chp, pit)
    return st, bufs


def dest_shapes(fmt, css, roi):
    """Reference sample sizing (samples/rocjpeg_samples_utils.h:318-399), with room for the
    reference kernels' whole-group writes past the last pixel (they write up to 7 px / 1 row
    beyond the picture, rocjpeg_hip_kernels.cpp:1573-1574); only the picture is compared."""
    iw = [W, {0: W, 1: W, 2: W >> 1, 3: W >> 1, 5: 0}[css]] * 2
    ih = [H, {0: H, 1: H >> 1, 2: H, 3: H >> 1, 5: 0}[css]] * 2
    iw = [iw[0], iw[1], iw[1], 0]
    ih = [ih[0], ih[1], ih[1], 0]
    shp = channel_shapes(fmt, css, iw, ih, roi=roi)
    if fmt in (R.OutputFormat.RGB, R.OutputFormat.RGB_PLANAR) or \
            (fmt in (R.OutputFormat.YUV_PLANAR, R.OutputFormat.Y) and css in (2, 3)):
        pad = 48 if fmt == R.OutputFormat.RGB else 16
        # planar RGB: every plane uses pitch[0] (rocjpeg_decoder.cpp:525-544)
        shp = [(r + 2, p + pad if (fmt != R.OutputFormat.RGB_PLANAR) else shp[0][1] + pad) for r, p in shp]
    return shp


@pytest.mark.parametrize("roi_name", list(ROIS))
@pytest.mark.parametrize("fmt", FMTS, ids=[f.name for f in FMTS])
@pytest.mark.parametrize("css_name", list(CSS))
def test_output_stage_matches_reference_kernels(ref, css_name, fmt, roi_name):
    from tests import gpu_util as G
    t = G.torch()
    css, roi = CSS[css_name], ROIS[roi_name]
    planes = make_planes(css, seed=zlib.crc32(f"{css_name}/{fmt.name}/{roi_name}".encode()))
    surface, offs, pitches = make_surface(css, planes)
    shapes = dest_shapes(fmt, css, roi)
    # bytes the oracle writes: those that differ between two runs with different fills
    st0, o0 = oracle_output(css, planes, fmt, roi, shapes, 0x00)
    st1, o1 = oracle_output(css, planes, fmt, roi, shapes, 0xFF)
    assert st0 == 0 and st1 == 0
    written = [a == b for a, b in zip(o0, o1)]
    assert any(m.any() for m in written)
    dst = [t.full(s, 0x5A, dtype=t.uint8, device="cuda") for s in shapes] + [None] * (4 - len(shapes))
    stage = RefOutputStage(ref, t, css, surface, offs, pitches)
    stage.run(fmt, roi, dst, [s[1] for s in shapes] + [0] * (4 - len(shapes)))
    for k, (want, m) in enumerate(zip(o0, written)):
        got = dst[k].cpu().numpy()
        # where the oracle wrote, the reference wrote the same byte
        want_w = np.where(m, want, 0)
        got_w = np.where(m, got, 0)
        bad = np.argwhere(want_w != got_w)
        assert len(bad) == 0, (k, len(bad), tuple(bad[0]), int(got[tuple(bad[0])]), int(want[tuple(bad[0])]))
