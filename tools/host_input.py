#!/usr/bin/env python3
"""Drop-in (non-resident) decode rate of the C2 batch by host staging thread count
(RJ_HOST_THREADS), configurations alternating over rounds (HI_ROUNDS x HI_CALLS calls; HI_PROFILE=1
adds a call with the handle's stage events), plus a pinned-memory copy / DMA probe (HI_PROBE=0
skips it).  Development aid (gpurun):  python tools/host_input.py [[env]/threads ...]  e.g. 0/8 0/12
The part before '/' was RJ_HOST_SPLIT, the host-input split measured in round 3 and not kept
(profiles/r3_experiments/host_input_split_ab.txt)."""
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
    configs = sys.argv[1:] or ["0/8", "0.5,0.5/8"]
    L = R.lib()
    decs = {}
    for c in configs:
        split, _, nt = c.partition("/")
        os.environ["RJ_HOST_SPLIT"] = split
        os.environ["RJ_HOST_THREADS"] = nt or "8"
        decs[c] = R.JpegDecoder(R.Backend.HARDWARE, 0)
        assert L.rocJpegDecodeBatched(decs[c].handle, hs, 1024, ctypes.byref(params), arr) == 0
    torch.cuda.synchronize()
    rates = {c: [] for c in configs}
    for rnd in range(int(os.environ.get("HI_ROUNDS", "3"))):
        for c in configs:
            t0 = time.perf_counter()
            for _ in range(int(os.environ.get("HI_CALLS", "8"))):
                assert L.rocJpegDecodeBatched(decs[c].handle, hs, 1024, ctypes.byref(params), arr) == 0
            torch.cuda.synchronize()
            rates[c].append(int(os.environ.get("HI_CALLS", "8")) * 1024 / (time.perf_counter() - t0))
            if os.environ.get("HI_PROFILE"):  # one more call with the handle's stage events
                decs[c].set_profiling(True)
                L.rocJpegDecodeBatched(decs[c].handle, hs, 1024, ctypes.byref(params), arr)
                t = decs[c].last_timings()
                decs[c].set_profiling(False)
                print(f"  profiled ({'last part' if c.split('/')[0] not in ('0', '1') else 'whole call'}): "
                      f"host {t['host_ms']:.2f} h2d+stage {t['h2d_ms']:.2f} K0 {t['destuff_ms']:.2f} "
                      f"K1 {t['huffman_ms']:.2f} K2 {t['idct_ms']:.2f} total {t['total_ms']:.2f} ms", flush=True)
            print(f"round {rnd} {c:16s} {rates[c][-1]:9.1f} images/s", flush=True)
    for c in configs:
        print(f"{c:16s} median {sorted(rates[c])[len(rates[c]) // 2]:9.1f} images/s  ({', '.join(f'{r:.0f}' for r in rates[c])})")
        decs[c].close()
    if os.environ.get("HI_PROBE", "1") == "0":
        return
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
