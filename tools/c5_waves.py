"""Development: per-scan wave timing of C5 images (RJ_DEBUG_WAVES=1 output on stderr) for one
image and for batches (sizes as arguments, default 1 64; 64 distinct images repeated), to
separate the refinement chain from the batch's contention."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import rocjpeg_amd as R  # noqa: E402
from tests import gpu_util as G  # noqa: E402


def main():
    t = G.torch()
    bench._init_gen()
    gen = bench.WORKLOADS["c5"]["gen"]
    datas = [bench._make_jpeg((s, gen)) for s in range(1234, 1234 + 64)]
    dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
    for bs in [int(a) for a in sys.argv[1:]] or [1, 64]:
        streams = [R.JpegStream(datas[k % len(datas)]) for k in range(bs)]
        dec.streams_to_device(streams)
        outs = [t.empty((1080, 5760), dtype=t.uint8, device="cuda") for _ in range(bs)]
        imgs = [R.make_image([o.data_ptr()], [o.shape[1]]) for o in outs]
        params = R.decode_params(R.OutputFormat.RGB)
        for _ in range(2):
            assert dec.decode_batched(streams, params, imgs) == 0
        t.cuda.synchronize()
        print(f"---- batch {bs}", file=sys.stderr, flush=True)
        assert dec.decode_batched(streams, params, imgs) == 0
        t.cuda.synchronize()
    dec.close()


if __name__ == "__main__":
    main()
