"""K2's time against where its buffers live, in ONE process (development probe).

Three handles (each with its own entry buffer) and three output arenas (one 6.4-GB torch
allocation each): every (handle, arena) pair decodes the C2 batch; prints K1 / K2 ms per pair
(profiled calls, HIP events).  If K2 follows the arena, the output's placement decides its
mode; if it follows the handle, the entry buffer's.
    python3 tools/k2_placement_probe.py [handles] [arenas] [calls]
    python3 tools/k2_placement_probe.py shift KB,KB,...   (one arena; a fresh handle per entry-stream
        shift RJ_ENT_SHIFT_KB, destroyed before the next; RJ_DEBUG_HOST prints the addresses)
"""
import ctypes
import os
import sys
from multiprocessing import get_context

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import rocjpeg_amd as R

    if len(sys.argv) > 2 and sys.argv[1] == "shift":
        return shift_probe([int(x) for x in sys.argv[2].split(",")])
    nh = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    na = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    calls = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    with get_context("fork").Pool(16, initializer=bench._init_gen) as pool:
        path, offs, sizes = bench.dataset_part("c2", 0, 1024, pool)
    with open(path, "rb") as f:
        raw = f.read()
    datas = [raw[int(o):int(o) + int(s)] for o, s in zip(offs, sizes)]
    fmt = R.OutputFormat.RGB
    decs = [R.JpegDecoder(R.Backend.HARDWARE, 0) for _ in range(max(nh, na))]
    runs = [bench.BatchRun(decs[k], datas, fmt, "cuda:0") for k in range(na)]
    L = R.lib()
    base = runs[0]
    print("arenas:", " ".join(hex(r.out.data_ptr()) for r in runs), flush=True)
    for rep in range(2):
        for h in range(nh):
            d = decs[h]
            for a in range(na):
                arr = runs[a].arr
                for _ in range(2):
                    assert L.rocJpegDecodeBatched(d.handle, base.hs, base.n, ctypes.byref(base.params), arr) == 0
                d.set_profiling(True)
                k1, k2 = [], []
                for _ in range(calls):
                    assert L.rocJpegDecodeBatched(d.handle, base.hs, base.n, ctypes.byref(base.params), arr) == 0
                    t = d.last_timings()
                    k1.append(t["huffman_ms"])
                    k2.append(t["idct_ms"])
                d.set_profiling(False)
                torch.cuda.synchronize()
                print(f"rep {rep} handle {h} arena {a}: K1 {np.median(k1):.3f} K2 {np.median(k2):.3f} ms", flush=True)


def load_c2():
    import bench
    with get_context("fork").Pool(16, initializer=bench._init_gen) as pool:
        path, offs, sizes = bench.dataset_part("c2", 0, 1024, pool)
    with open(path, "rb") as f:
        raw = f.read()
    return [raw[int(o):int(o) + int(s)] for o, s in zip(offs, sizes)]


def shift_probe(shifts, calls=4):
    import torch

    import bench
    import rocjpeg_amd as R
    datas = load_c2()
    fmt = R.OutputFormat.RGB
    d0 = R.JpegDecoder(R.Backend.HARDWARE, 0)
    run = bench.BatchRun(d0, datas, fmt, "cuda:0")
    L = R.lib()
    print("arena:", hex(run.out.data_ptr()), flush=True)
    for rep in range(2):
        for sh in shifts:
            os.environ["RJ_ENT_SHIFT_KB"] = str(sh)
            d = R.JpegDecoder(R.Backend.HARDWARE, 0)
            for _ in range(2):
                assert L.rocJpegDecodeBatched(d.handle, run.hs, run.n, ctypes.byref(run.params), run.arr) == 0
            d.set_profiling(True)
            k1, k2 = [], []
            for _ in range(calls):
                assert L.rocJpegDecodeBatched(d.handle, run.hs, run.n, ctypes.byref(run.params), run.arr) == 0
                t = d.last_timings()
                k1.append(t["huffman_ms"])
                k2.append(t["idct_ms"])
            d.set_profiling(False)
            torch.cuda.synchronize()
            print(f"rep {rep} shift {sh} KB: K1 {np.median(k1):.3f} K2 {np.median(k2):.3f} ms", flush=True)
            d.close()
            del d


if __name__ == "__main__":
    main()
