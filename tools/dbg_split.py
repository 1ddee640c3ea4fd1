"""Development: one C2 image through the forced lean outlier split; first mismatching rows vs the
oracle (RJ_DEBUG_K1_PIECES prints the pieces)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("RJ_SPLIT_OUTLIERS", "1")
os.environ.setdefault("RJ_SPLIT_OUTLIER_FRAC", "1")
import numpy as np
import torch
import rocjpeg_amd as R
from tests import oracle_lib as O
import tests.test_batch_gpu as T
distinct = int(sys.argv[1]) if len(sys.argv) > 1 else 1
copies = int(sys.argv[2]) if len(sys.argv) > 2 else 1
datas = T._c2_images(distinct, seed0=4321)
dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
streams = [R.JpegStream(datas[i % distinct]) for i in range(distinct * copies)]
out = torch.full((len(streams), 1080, 5760), 0xA5, dtype=torch.uint8, device="cuda")
imgs = [R.make_image([out[i].data_ptr()], [5760]) for i in range(len(streams))]
dec.set_profiling(True)
st = dec.decode_batched(streams, R.decode_params(R.OutputFormat.RGB), imgs)
tm = dec.last_timings()
print("status", st, "lean_split", tm["lean_split"], "lean_five", tm["lean_five"])
for i, d in enumerate(datas[:4]):
    ost, want = O.oracle_decode(d, int(R.OutputFormat.RGB), [(1080, 5760)])
    for c in range(copies):
        g = out[i + c * distinct].cpu().numpy()
        rows = np.nonzero((g != want[0]).any(axis=1))[0]
        print("image", i, "copy", c, "mismatching pixel rows", len(rows), rows[:12] // 16)
        if c >= 1:
            break
