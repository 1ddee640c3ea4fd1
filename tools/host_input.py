#!/usr/bin/env python3
"""Drop-in (non-resident) decode rate of the C2 batch by host staging thread count, plus a
pinned-memory copy / DMA probe.  Development aid (gpurun): python tools/host_input.py"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    from multiprocessing import get_context
    pool = get_context("fork").Pool(16, initializer=bench._init_gen)
    path, offs, sizes = bench.dataset_part("c2", 0, 1024, pool)
    pool.close()
    raw = open(path, "rb").read()
    datas = [raw[int(o):int(o) + int(s)] for o, s in zip(offs, sizes)]
    import torch
    import rocjpeg_amd as R
    from tests.gpu_util import channel_shapes
    torch.cuda.set_device(0)
    streams = [R.JpegStream(d) for d in datas]
    out = torch.empty(1024 * 1080 * 5760, dtype=torch.uint8, device="cuda")
    imgs = [R.make_image([out[i * 1080 * 5760:].data_ptr()], [5760]) for i in range(1024)]
    arr = (R.RocJpegImage * 1024)(*imgs)
    hs = (ctypes.c_void_p * 1024)(*[s.handle for s in streams])
    params = R.decode_params(R.OutputFormat.RGB)
    for nt in (1, 4, 8, 16, 32):
        os.environ["RJ_HOST_THREADS"] = str(nt)
        dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
        L = R.lib()
        assert L.rocJpegDecodeBatched(dec.handle, hs, 1024, ctypes.byref(params), arr) == 0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            assert L.rocJpegDecodeBatched(dec.handle, hs, 1024, ctypes.byref(params), arr) == 0
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        dec.set_profiling(True)
        L.rocJpegDecodeBatched(dec.handle, hs, 1024, ctypes.byref(params), arr)
        t = dec.last_timings()
        dec.set_profiling(False)
        print(f"threads {nt:2d}: {1024 / dt:9.1f} images/s, {dt * 1e3:.2f} ms/call; profiled: host {t['host_ms']:.2f} "
              f"h2d+stage {t['h2d_ms']:.2f} K0 {t['destuff_ms']:.2f} K1 {t['huffman_ms']:.2f} K2 {t['idct_ms']:.2f} "
              f"total {t['total_ms']:.2f} ms", flush=True)
        dec.close()
    # raw probes: pinned->device DMA of 285 MB in one copy, and a 16-thread memcpy into pinned memory
    nb = int(sum(len(d) for d in datas))
    pin = torch.empty(nb, dtype=torch.uint8).pin_memory()
    dst = torch.empty(nb, dtype=torch.uint8, device="cuda")
    dst.copy_(pin, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        dst.copy_(pin, non_blocking=True)
    torch.cuda.synchronize()
    print(f"H2D pinned {nb / 1e6:.0f} MB: {5 * nb / (time.perf_counter() - t0) / 1e9:.1f} GB/s", flush=True)
    src = np.frombuffer(raw, np.uint8)[:nb]
    pv = pin.numpy()
    from concurrent.futures import ThreadPoolExecutor
    for nt in (1, 8, 16, 32):
        parts = [(nb * k // nt, nb * (k + 1) // nt) for k in range(nt)]
        with ThreadPoolExecutor(nt) as ex:
            t0 = time.perf_counter()
            for _ in range(3):
                list(ex.map(lambda p: np.copyto(pv[p[0]:p[1]], src[p[0]:p[1]]), parts))
            print(f"memcpy into pinned, {nt} threads: {3 * nb / (time.perf_counter() - t0) / 1e9:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
