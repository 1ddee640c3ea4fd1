"""Development: decode fixtures through one K1 and report the first mismatch with the oracle per
plane (block row / column), with the call's K1 counters.  Usage: python tools/debug_k1.py NAME...
(names from tests/golden/manifest.json, or c2nori:SEED for a bench C2 no-DRI image)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rocjpeg_amd as R  # noqa: E402
from tests import gpu_util as G  # noqa: E402
from tests import oracle_lib as O  # noqa: E402


def data_of(name):
    if name.startswith("c2nori:"):
        import bench
        bench._init_gen()
        return bench._make_jpeg((int(name.split(":")[1]), bench.WORKLOADS["c2nori"]["gen"]))
    return O.fixture_bytes(next(f for f in O.manifest() if f["name"] == name))


def main():
    G.torch()
    dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
    fmt = R.OutputFormat.YUV_PLANAR
    for name in sys.argv[1:]:
        data = data_of(name)
        s = R.JpegStream(data)
        nc, css, w, h = dec.image_info(s)
        shapes = G.channel_shapes(fmt, css, w, h)
        bufs, img = G.gpu_buffers(shapes)
        dec.set_profiling(True)
        st = dec.decode(s, R.decode_params(fmt), img)
        tm = dec.last_timings()
        dec.set_profiling(False)
        got = G.to_host(bufs)
        ost, want = O.oracle_decode(data, int(fmt), shapes)
        keys = ("intervals", "chunks", "split_intervals", "serial_fallbacks", "lean_k1", "chunk_k1")
        print(name, f"{w}x{h}", "status", st, ost, {k: tm[k] for k in keys}, flush=True)
        for c, (g, x) in enumerate(zip(got, want)):
            d = np.argwhere(g != x)
            if len(d) == 0:
                print(f"  plane {c}: exact")
                continue
            r0, c0 = d[0]
            blocks = {(int(a) // 8, int(b) // 8) for a, b in d}
            print(f"  plane {c}: {len(d)} px differ in {len(blocks)} blocks, first at ({r0},{c0}) block "
                  f"({r0 // 8},{c0 // 8}) got {g[r0, c0]} want {x[r0, c0]}; last block {max(blocks)}")
    dec.close()


if __name__ == "__main__":
    main()
