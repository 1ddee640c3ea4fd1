"""Parse-rate probe on the C2 batch: rocJpegAmdStreamParseDevice (with its stage split) against
host rocJpegStreamParse on one thread.  Usage: python tools/scan_timing.py [batch]"""
import os
import sys
import time
from multiprocessing import get_context

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    pool = get_context("fork").Pool(16, initializer=bench._init_gen)
    path, offs, sizes = bench.dataset_part("c2", 0, n, pool)
    pool.close()
    raw = open(path, "rb").read()
    datas = [raw[int(o):int(o) + int(s)] for o, s in zip(offs, sizes)]
    import rocjpeg_amd as R
    dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
    dec.parse_device(datas[:8])
    for rep in range(4):
        t = time.perf_counter()
        st, ss = dec.parse_device(datas)
        dt = time.perf_counter() - t
        print(f"device parse: status {st}, {dt * 1e3:.2f} ms, {n / dt:.0f} images/s, stages {dec.last_parse_timings()}",
              flush=True)
        for s in ss:
            s.close()
    t = time.perf_counter()
    ss = [R.JpegStream(b) for b in datas]
    dt = time.perf_counter() - t
    print(f"host parse, 1 thread: {dt * 1e3:.2f} ms, {n / dt:.0f} images/s")


if __name__ == "__main__":
    main()
