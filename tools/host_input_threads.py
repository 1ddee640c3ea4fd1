"""The drop-in input path (bitstreams in host memory, staged by every rocJpegDecodeBatched call)
with T caller threads, each with its own handle and 1024 / T of the C2 images, as the reference's
jpegdecodeperf runs its threads (samples/jpegDecodePerf/jpegdecodeperf.cpp:228-257): does one
caller's H2D staging overlap another's decode?  Prints aggregate images/s per T.
Development aid / evidence: python tools/host_input_threads.py [calls] [T,T,...]"""
import ctypes
import os
import sys
import threading
import time
from multiprocessing import get_context

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import rocjpeg_amd as R  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    tlist = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 4]
    n = 1024
    with get_context("spawn").Pool(16, initializer=bench._init_gen) as pool:
        path, offs, sizes = bench.dataset_part("c2", 0, n, pool)
    blob = open(path, "rb").read()
    datas = [blob[int(o):int(o) + int(s)] for o, s in zip(offs, sizes)]
    out = torch.empty((n, 1080, 5760), dtype=torch.uint8, device="cuda")
    L = R.lib()
    for T in tlist:
        per = n // T
        rates, errs = [0.0] * T, []
        barrier = threading.Barrier(T + 1)

        def worker(t):
            try:
                d = R.JpegDecoder(R.Backend.HARDWARE, 0)
                mine = list(range(t * per, (t + 1) * per))
                streams = [R.JpegStream(datas[i]) for i in mine]
                hs = (ctypes.c_void_p * per)(*[s.handle for s in streams])
                imgs = (R.RocJpegImage * per)(*[R.make_image([out[i].data_ptr()], [5760]) for i in mine])
                par = R.decode_params(R.OutputFormat.RGB)
                st = L.rocJpegDecodeBatched(d.handle, hs, per, ctypes.byref(par), imgs)  # warm
                barrier.wait()
                for _ in range(calls):
                    st |= L.rocJpegDecodeBatched(d.handle, hs, per, ctypes.byref(par), imgs)
                if st != 0:
                    raise RuntimeError(R.error_name(st))
                barrier.wait()
                for s in streams:
                    s.close()
                d.close()
            except Exception as e:
                errs.append(repr(e))
                barrier.abort()

        th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        for x in th:
            x.start()
        barrier.wait()
        t0 = time.perf_counter()
        barrier.wait()
        dt = time.perf_counter() - t0
        for x in th:
            x.join()
        if errs:
            print(f"T={T}: error {errs[0]}", flush=True)
            continue
        print(f"T={T}: {n * calls / dt:9.0f} images/s aggregate ({dt / calls * 1e3:.2f} ms per 1024 images)", flush=True)


if __name__ == "__main__":
    main()
