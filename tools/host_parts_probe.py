"""The drop-in input path by DecodeSplit part count (development probe): the C2 batch from host
memory (fresh stream objects, so every call stages the bitstreams), one handle per part count
(RJ_SPLIT_PARTS set before the handle is created), 2 warm + 5 timed calls each.
    python3 tools/host_parts_probe.py [parts,parts,...]
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from multiprocessing import get_context

    import bench
    base = bench.part_base("c2", 0, 1024)
    if os.path.exists(base + ".bin") and os.path.exists(base + ".idx.npy"):  # (no fork under a profiler)
        path, offs, sizes = bench.dataset_part("c2", 0, 1024, None)
    else:
        with get_context("fork").Pool(16, initializer=bench._init_gen) as pool:
            path, offs, sizes = bench.dataset_part("c2", 0, 1024, pool)
    raw = open(path, "rb").read()
    datas = [raw[int(o):int(o) + int(s)] for o, s in zip(offs, sizes)]
    import torch

    import rocjpeg_amd as R
    assert torch.cuda.is_available()
    out = torch.empty(1024 * 1080 * 5760, dtype=torch.uint8, device="cuda")
    imgs = [R.make_image([out[i * 1080 * 5760:].data_ptr()], [5760]) for i in range(1024)]
    arr = (R.RocJpegImage * 1024)(*imgs)
    params = R.decode_params(R.OutputFormat.RGB)
    L = R.lib()
    for parts in (sys.argv[1] if len(sys.argv) > 1 else "2,3").split(","):
        os.environ["RJ_SPLIT_PARTS"] = parts
        dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
        streams = [R.JpegStream(d) for d in datas]
        hs = (ctypes.c_void_p * 1024)(*[s.handle for s in streams])
        for _ in range(2):
            assert L.rocJpegDecodeBatched(dec.handle, hs, 1024, ctypes.byref(params), arr) == 0
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            assert L.rocJpegDecodeBatched(dec.handle, hs, 1024, ctypes.byref(params), arr) == 0
            ts.append(time.perf_counter() - t0)
        print(f"parts {parts}: per call ms " + " ".join(f"{t * 1e3:.2f}" for t in ts) +
              f"  -> {1024 * 5 / sum(ts):.0f} images/s", flush=True)
        for s in streams:
            s.close()
        dec.close()


if __name__ == "__main__":
    main()
