"""jpegdecodeperf's shape alone (8 threads, a handle each, one C2 image per rocJpegDecodeBatched,
resident streams), for A/B of the coalescing settings, which the library reads once per process:
run one process per setting, e.g. RJ_COALESCE_WAIT_US=0 python tools/threads_probe.py.
Prints the summed rate, the per-thread spread and the coalescing counters.  Development aid."""
import ctypes
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import rocjpeg_amd as R  # noqa: E402
from tests import gpu_util as G  # noqa: E402


def main(threads=8, per=16, budget_s=1.5):
    t = G.torch()
    bench._init_gen()
    gen = bench.WORKLOADS["c2"]["gen"]
    datas = [bench._make_jpeg((s, gen)) for s in range(4321, 4321 + threads * per)]
    L = R.lib()
    rates = [0.0] * threads
    barrier = threading.Barrier(threads)
    c0 = R.coalesce_stats()

    def worker(k):
        d = R.JpegDecoder(R.Backend.HARDWARE, 0)
        st, streams = d.parse_device(datas[k * per:(k + 1) * per])
        assert st == 0
        out = t.empty((1080, 5760), dtype=t.uint8, device="cuda")
        img = R.make_image([out.data_ptr()], [5760])
        par = R.decode_params(R.OutputFormat.RGB)
        hs = (ctypes.c_void_p * len(streams))(*[s.handle for s in streams])
        for j in range(3):
            L.rocJpegDecodeBatched(d.handle, bench._sub(hs, ctypes.c_void_p, j, 1), 1, ctypes.byref(par),
                                   ctypes.byref(img))
        barrier.wait()
        tot, cnt, t_end = 0.0, 0, time.perf_counter() + budget_s
        while time.perf_counter() < t_end:
            t0 = time.perf_counter()
            r = L.rocJpegDecodeBatched(d.handle, bench._sub(hs, ctypes.c_void_p, cnt % per, 1), 1,
                                       ctypes.byref(par), ctypes.byref(img))
            tot += time.perf_counter() - t0
            assert r == 0
            cnt += 1
        rates[k] = cnt / tot
        for s in streams:
            s.close()
        d.close()

    th = [threading.Thread(target=worker, args=(k,)) for k in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    c1 = R.coalesce_stats()
    calls, comb, memb = (c1[i] - c0[i] for i in range(3))
    env = {k: v for k, v in os.environ.items() if k.startswith("RJ_COALESCE")}
    print(f"{env} threads {threads}: summed {sum(rates):8.1f} img/s, spread {max(rates) / min(rates):.3f}, "
          f"calls {calls}, combined {comb}, members/combined {memb / max(1, comb):.2f}", flush=True)


if __name__ == "__main__":
    main()
