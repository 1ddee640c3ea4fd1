"""Development: stage times of small calls (batch 1 / 16 / 128 of C2 images, resident) under the
handle's chunk floor (env RJ_CHUNK_MIN, read at handle creation).  Usage:
python tools/shape_profile.py [--nori] MIN...  (one handle per floor; prints one line per shape)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import rocjpeg_amd as R  # noqa: E402
from tests import gpu_util as G  # noqa: E402


def main():
    args = sys.argv[1:]
    nori = "--nori" in args
    mins = [a for a in args if a != "--nori"] or ["1024"]
    t = G.torch()
    bench._init_gen()
    gen = bench.WORKLOADS["c2nori" if nori else "c2"]["gen"]
    shapes = [int(x) for x in os.environ.get("SHAPES", "1,4,8,16,128").split(",")]
    datas = [bench._make_jpeg((s, gen)) for s in range(1234, 1234 + max(shapes))]
    for m in mins:
        os.environ["RJ_CHUNK_MIN"] = m
        dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
        for bs in shapes:
            streams = [R.JpegStream(d) for d in datas[:bs]]
            dec.streams_to_device(streams)
            outs = [t.empty((1080, 5760), dtype=t.uint8, device="cuda") for _ in range(bs)]
            imgs = [R.make_image([o.data_ptr()], [o.shape[1]]) for o in outs]
            params = R.decode_params(R.OutputFormat.RGB)
            for _ in range(3):
                assert dec.decode_batched(streams, params, imgs) == 0
            t.cuda.synchronize()
            n = 20
            t0 = time.perf_counter()
            for _ in range(n):
                dec.decode_batched(streams, params, imgs)
            wall = (time.perf_counter() - t0) / n * 1e3
            dec.set_profiling(True)
            dec.decode_batched(streams, params, imgs)
            tm = dec.last_timings()
            dec.set_profiling(False)
            keys = ("host_ms", "h2d_ms", "destuff_ms", "huffman_ms", "idct_ms", "output_ms", "total_ms")
            print(f"min {m:>10} batch {bs:4d} wall {wall:.3f} ms | " +
                  " ".join(f"{k[:-3]} {tm[k]:.3f}" for k in keys) +
                  f" | chunk_bytes {tm['chunk_bytes']} chunks {tm['chunks']} split {tm['split_intervals']}"
                  f" lean {tm['lean_k1']} fb {tm['serial_fallbacks']}", flush=True)
        dec.close()


if __name__ == "__main__":
    main()
