"""H2D upload rates from pinned host memory on the GPU box: one copy, 8-MB pieces on one stream,
and pieces spread over 2 / 4 streams (whether several DMA engines raise the rate), for the marker
scan's upload (rj_decoder.cpp ParseOnDeviceImpl).  Development aid.  Usage: python tools/h2d_probe.py"""
import time

import torch


def rate(fn, nbytes, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return nbytes / best / 1e9, best * 1e3


def main():
    n = 285 << 20
    piece = 8 << 20
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h.fill_(7)
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(4)]

    def one():
        d.copy_(h, non_blocking=True)

    def pieces(k):
        def f():
            for i, o in enumerate(range(0, n, piece)):
                with torch.cuda.stream(streams[i % k]):
                    d[o:o + piece].copy_(h[o:o + piece], non_blocking=True)
        return f

    print(f"one copy      : {rate(one, n)[0]:6.1f} GB/s", flush=True)
    for k in (1, 2, 4):
        g, ms = rate(pieces(k), n)
        print(f"pieces x{k} str: {g:6.1f} GB/s ({ms:.2f} ms for {n >> 20} MB)", flush=True)


if __name__ == "__main__":
    main()
