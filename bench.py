#!/usr/bin/env python3
"""bench.py -- images/s of rocJpegDecodeBatched on MI355X (BASELINE.json `metric`).

Workload (BASELINE.json configs[1], "C2"): per GPU a batch of 1024 synthetic 1920x1080 4:2:0
baseline JPEGs (q90, DRI = 120 MCUs = one MCU row), ROCJPEG_OUTPUT_RGB.  A step = one
rocJpegDecodeBatched call per rank over that rank's shard, bitstreams already resident in HBM,
RGB written to HBM.

Multi-GPU (rocjpeg_amd/shard.py): one process per GPU.  Every rank generates one
part of the dataset into a file on the node (before any GPU call); rank 0 reads the headers of
all parts, builds the 64-byte-per-image work table, assigns images to ranks by LPT and
broadcasts the table (RCCL) -- the only collective; each rank parses its own images from the
shared files and decodes them on its own GPU.  `--gpus N` with no WORLD_SIZE in the
environment launches the N ranks itself (torch.distributed.run, before touching the GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--workload c2|c2nori|c3|c4|c5]

At N = 1 the line also carries `extra_workloads`: the other BASELINE configs measured in the
same run with the same contract -- c2nori (the no-DRI twin set), C3 (4:4:4 +
4:2:2 -> YUV_PLANAR), C4 (mixed resolution, per GPU) and C5 (progressive).
"""
import argparse
import ctypes
import io
import json
import os
import re
import socket
import subprocess
import sys
import time
from multiprocessing import get_context

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MUG = os.path.join(ROOT, "tests", "golden", "img", "mug_420.jpg")
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
TABLE_BYTES = 1828          # JpegStreamParameters per image: the 8(d) basis
PROG_KERNELS = ("k_prog", "k_prog_wave", "k_prog_fold")  # RocJpegAmdTimings.prog_kernel_*
C4_SIZES = [(640, 480), (1280, 720), (1920, 1080), (2560, 1440), (3840, 2160)]
SEED0 = 1234
GEN_VERSION = 1  # bump when the generator changes (dataset files are cached per node)

# generator arguments: (w, h, subsampling, restart = one MCU row, progressive); w == 0: C4 sizes
# by seed; sub == -1: 4:4:4 / 4:2:2 alternating by seed (C3)
WORKLOADS = {
    "c2": {"gen": (1920, 1080, 2, True, False), "fmt": "RGB",
           "data": "synthetic: seeded 1920x1080 crops of the reference mug_420.jpg + N(0,2) noise, Pillow q90 4:2:0 DRI=120",
           "workload": "C2: batch of {batch} x 1920x1080 4:2:0 baseline JPEG q90, RI=120 MCUs per GPU, ROCJPEG_OUTPUT_RGB, bitstreams resident in HBM"},
    "c2nori": {"gen": (1920, 1080, 2, False, False), "fmt": "RGB",
               "data": "synthetic: the C2 seeds encoded without DRI (SURVEY.md 8d no-DRI twin set)",
               "workload": "C2 no-DRI twin: batch of {batch} x 1920x1080 4:2:0 baseline q90, no restart markers, ROCJPEG_OUTPUT_RGB, resident"},
    "c3": {"gen": (1920, 1080, -1, True, False), "fmt": "YUV_PLANAR",
           "data": "synthetic: seeded 1920x1080 crops of mug_420.jpg + N(0,2) noise, Pillow q90, 4:4:4 / 4:2:2 alternating, DRI = 1 MCU row",
           "workload": "C3: batch of {batch} x 1920x1080 baseline q90, 4:4:4 and 4:2:2 alternating, ROCJPEG_OUTPUT_YUV_PLANAR, resident"},
    "c4": {"gen": (0, 0, 2, True, False), "fmt": "RGB",
           "data": "synthetic: seeded crops of mug_420.jpg + N(0,2) noise, sizes 640x480..3840x2160 uniform by seed, Pillow q90 4:2:0, DRI = 1 MCU row",
           "workload": "C4: batch of {batch} mixed-resolution 4:2:0 baseline JPEGs per GPU (640x480..3840x2160), LPT-sharded, ROCJPEG_OUTPUT_RGB, resident"},
    "c5": {"gen": (1920, 1080, 2, False, True), "fmt": "RGB",
           "data": "synthetic: seeded 1920x1080 crops of mug_420.jpg + N(0,2) noise, Pillow q90 4:2:0 progressive=True (no DRI)",
           "workload": "C5: batch of {batch} x 1920x1080 4:2:0 progressive JPEG q90 (10 scans, no DRI), ROCJPEG_OUTPUT_RGB, resident"},
}


def host_cores():
    """CPU cores this job may use: the affinity mask, capped by a cgroup CPU quota and by
    OMP_NUM_THREADS (the GPU box sets it to the job's CPU share; nproc there shows the whole
    machine).  Returns (cores, nproc, rule)."""
    nproc = os.cpu_count() or 1
    cores, rule = nproc, "nproc"
    try:
        aff = len(os.sched_getaffinity(0))
        if aff < cores:
            cores, rule = aff, "sched_getaffinity"
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            c = max(1, int(int(q) // int(p)))
            if c < cores:
                cores, rule = c, "cgroup cpu.max"
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and 0 < int(omp) < cores:
        cores, rule = int(omp), "OMP_NUM_THREADS (the job's CPU share)"
    return cores, nproc, rule


# ------------------------------------------------------------------ dataset (host only)
_BASE = None


def _init_gen():
    global _BASE
    from PIL import Image
    _BASE = np.asarray(Image.open(MUG).convert("RGB"))


def _make_jpeg(job):
    """Seeded crop of the reference mug image + N(0,2) noise, Pillow/libjpeg-turbo q90
    (BASELINE.md generator)."""
    seed, (w, h, sub, rst, prog) = job
    if w == 0:
        w, h = C4_SIZES[seed % len(C4_SIZES)]
    if sub == -1:
        sub = 0 if seed % 2 == 0 else 1
    from PIL import Image
    rng = np.random.default_rng(seed)
    y0 = int(rng.integers(0, _BASE.shape[0] - h + 1))
    x0 = int(rng.integers(0, _BASE.shape[1] - w + 1))
    a = _BASE[y0:y0 + h, x0:x0 + w].astype(np.float32) + rng.normal(0.0, 2.0, (h, w, 3))
    kw = dict(quality=90, subsampling=sub)
    if rst:
        kw["restart_marker_blocks"] = (w + 7) // 8 if sub == 0 else (w + 15) // 16  # one MCU row
    if prog:
        kw["progressive"] = True
    b = io.BytesIO()
    Image.fromarray(np.clip(a, 0, 255).astype(np.uint8)).save(b, "JPEG", **kw)
    return b.getvalue()


def data_dir():
    d = os.environ.get("RJ_BENCH_DATA") or os.path.join("/tmp", f"rocjpeg_amd_bench_{os.getuid()}")
    os.makedirs(d, exist_ok=True)
    return d


def part_base(name, part, count):
    return os.path.join(data_dir(), f"{name}_v{GEN_VERSION}_p{part}_n{count}")


def dataset_part(name, part, count, pool):
    """Part `part` of workload `name` (seeds SEED0 + part * count ...): one file of concatenated
    JPEGs plus an index, generated once per node and shared by the ranks.  Returns
    (path, offsets, sizes)."""
    base = part_base(name, part, count)
    if not (os.path.exists(base + ".bin") and os.path.exists(base + ".idx.npy")):
        seeds = range(SEED0 + part * count, SEED0 + (part + 1) * count)
        blobs = pool.map(_make_jpeg, [(s, WORKLOADS[name]["gen"]) for s in seeds], chunksize=4)
        sizes = np.array([len(b) for b in blobs], dtype=np.uint64)
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
        tmp = f"{base}.{os.getpid()}"
        with open(tmp + ".bin", "wb") as f:
            for b in blobs:
                f.write(b)
        np.save(tmp + ".idx.npy", np.stack([offs, sizes]))
        os.replace(tmp + ".bin", base + ".bin")
        os.replace(tmp + ".idx.npy", base + ".idx.npy")
    idx = np.load(base + ".idx.npy")
    return base + ".bin", idx[0], idx[1]


# ------------------------------------------------------------------ CPU baselines
def _turbo_proc(go, q, path, items, budget_s):
    """One host core: libjpeg-turbo (Pillow) decodes of this worker's images to RGB, timed
    around the decode loop only (samples/jpegDecodePerf/jpegdecodeperf.cpp:153-186)."""
    from PIL import Image
    with open(path, "rb") as f:
        data = [None] * len(items)
        for j, (o, s) in enumerate(items):
            f.seek(int(o))
            data[j] = f.read(int(s))
    go.wait()
    n, t0 = 0, time.perf_counter()
    while True:
        for b in data:
            Image.open(io.BytesIO(b)).convert("RGB").load()
            n += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    q.put((n, time.perf_counter() - t0))


class TurboBaseline:
    """libjpeg-turbo on the job's host cores, one process per core, each decoding its shard of
    the same files (BASELINE.md "CPU baseline plan").  The processes are forked before any GPU
    call and wait on an event; they exit by returning (no SIGTERM)."""

    def __init__(self, path, offs, sizes, cores, budget_s=1.5, per_core=24):
        ctx = get_context("fork")
        self.go, self.q = ctx.Event(), ctx.Queue()
        n = len(offs)
        self.procs = []
        for c in range(cores):
            sel = [(offs[(c * per_core + j) % n], sizes[(c * per_core + j) % n]) for j in range(per_core)]
            p = ctx.Process(target=_turbo_proc, args=(self.go, self.q, path, sel, budget_s), daemon=True)
            p.start()
            self.procs.append(p)
        self.cores = cores

    def run(self):
        self.go.set()
        res = [self.q.get(timeout=600) for _ in self.procs]
        for p in self.procs:
            p.join(timeout=60)
        rate = sum(n / t for n, t in res)  # the reference sums per-thread rates (jpegdecodeperf.cpp:281-300)
        return rate, sum(n for n, _ in res), max(t for _, t in res)


def cpu_oracle(datas, shapes, fmt, budget_s=5.0):
    """The C restatement (oracle/jpeg_oracle.c), one thread, on a bounded sample: context."""
    from tests import oracle_lib as O
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s and n < len(datas):
        st, _ = O.oracle_decode(datas[n], fmt, shapes[n])
        assert st == 0
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 3), "unit": "images/s", "cores": 1, "kind": "port",
            "sample": f"{n} images of the batch, oracle/jpeg_oracle.c, 1 thread, {dt:.1f} s"}


def pmc_traffic(kernel, batch, launches, workload="c2"):
    """HBM bytes per launch of `kernel` from the committed PMC profile of this workload
    (tools/gpu_pmc.sh + tools/pmc_traffic.py: 2 x FETCH_SIZE + WRITE_SIZE per decode call, the
    gfx950 correction of MI355X_MICROARCH.md), scaled to this batch.  (bytes, source) or None."""
    name = "pmc_traffic.json" if workload == "c2" else f"pmc_traffic_{workload}.json"
    path = os.path.join(ROOT, "profiles", name)
    try:
        with open(path) as f:
            prof = json.load(f)
        ks = prof["kernels"]
        per_image = ks[kernel]["hbm_bytes_per_image"]
        if kernel == "k_rows":  # a lean split call's K2: the plain and split-aware launches together
            per_image += ks.get("k_rows_split", {}).get("hbm_bytes_per_image", 0.0)
        return int(per_image * batch / max(1, launches)), f"profiles/{name} ({prof.get('commit', '?')})"
    except (OSError, KeyError, ValueError):
        return None


# ------------------------------------------------------------------ one batch on the GPU
def parity_sample(n, k=16):
    """k image indices spread over a batch of n (first and last included)."""
    return sorted({int(round(i * (n - 1) / max(1, k - 1))) for i in range(k)}) if n else []


class BatchRun:
    """A rank's batch: streams parsed on the GPU (rocJpegAmdStreamParseDevice, resident), the
    destinations in one HBM arena sized as the reference samples size them
    (samples/rocjpeg_samples_utils.h:318-399, tests/gpu_util.py channel_shapes)."""

    def __init__(self, dec, datas, fmt, dev):
        import torch
        import rocjpeg_amd as R
        from tests.gpu_util import channel_shapes
        self.R, self.dec, self.datas, self.fmt = R, dec, datas, fmt
        t0 = time.perf_counter()
        st, self.streams = dec.parse_device(datas)
        if st != 0:
            raise RuntimeError(f"rocJpegAmdStreamParseDevice: {R.error_name(st)}")
        # the first call on a handle also allocates its pinned staging and scan buffers; the rate
        # reported is the median of 3 further calls on the same images (their streams closed)
        self.parse_first_s = time.perf_counter() - t0
        warm = []
        for _ in range(3):
            t0 = time.perf_counter()
            st, extra = dec.parse_device(datas)
            warm.append(time.perf_counter() - t0)
            self.parse_stages_ms = dec.last_parse_timings()
            for x in extra:
                x.close()
            if st != 0:
                raise RuntimeError(f"rocJpegAmdStreamParseDevice: {R.error_name(st)}")
        self.parse_s = float(np.median(warm))
        dec.streams_to_device(self.streams)  # progressive streams are host-parsed: make them resident too
        self.shapes = []
        for s in self.streams:
            nc, css, w, h = dec.image_info(s)
            self.shapes.append(channel_shapes(fmt, css, w, h))
        total = sum(r * p for shp in self.shapes for r, p in shp)
        self.out = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
        imgs, self.views, off = [], [], 0
        for shp in self.shapes:
            ptrs, pitches, vv = [], [], []
            for r, p in shp:
                ptrs.append(self.out[off:].data_ptr())
                pitches.append(p)
                vv.append(self.out[off:off + r * p].view(r, p))
                off += r * p
            imgs.append(R.make_image(ptrs, pitches))
            self.views.append(vv)
        self.params = R.decode_params(fmt)
        self.n = len(self.streams)
        self.hs = (ctypes.c_void_p * self.n)(*[s.handle for s in self.streams])
        self.arr = (R.RocJpegImage * self.n)(*imgs)

    def step(self):
        st = self.R.lib().rocJpegDecodeBatched(self.dec.handle, self.hs, self.n, ctypes.byref(self.params), self.arr)
        if st != 0:
            raise RuntimeError(self.R.error_name(st))

    def timed(self, steps, warmup, world=1, dev=None):  # dev: where the collective's tensors live
        """W untimed steps, then K steps bracketed by barrier + synchronize; max over ranks."""
        import torch
        import torch.distributed as dist
        for _ in range(warmup):
            self.step()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            self.step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed

    def profiled(self, steps):
        """Per-stage / per-kernel device times (HIP events on each launch's stream) over a
        separate pass -- never the timed one."""
        self.dec.set_profiling(True)
        acc, last = {}, None
        for _ in range(steps):
            self.step()
            last = self.dec.last_timings()
            for k, v in last.items():
                if isinstance(v, float):
                    acc[k] = acc.get(k, 0.0) + v
                elif isinstance(v, list) and v and isinstance(v[0], float):
                    acc[k] = [a + b for a, b in zip(acc.get(k, [0.0] * len(v)), v)]
        self.dec.set_profiling(False)
        for k, v in acc.items():
            last[k] = [x / steps for x in v] if isinstance(v, list) else v / steps
        return last

    def parity(self, idx):
        """Images `idx` of the current outputs (the last timed step's) vs the CPU oracle (the
        oracle calls release the GIL: 16 threads)."""
        from concurrent.futures import ThreadPoolExecutor
        from tests import oracle_lib as O
        with ThreadPoolExecutor(16) as ex:
            wants = list(ex.map(lambda q: O.oracle_decode(self.datas[q], int(self.fmt), self.shapes[q]), idx))
        ok = True
        for q, (ost, want) in zip(idx, wants):
            ok = ok and ost == 0 and all(np.array_equal(v.cpu().numpy(), w_) for v, w_ in zip(self.views[q], want))
        return bool(ok)


    def close(self):
        import torch
        del self.views, self.out, self.arr
        for s in self.streams:
            s.close()
        torch.cuda.empty_cache()


def _sub(arr, ctype, start, k):
    """k entries of a ctypes array from `start` (no copy)."""
    return (ctype * k).from_address(ctypes.addressof(arr) + start * ctypes.sizeof(ctype))


def _shape_loop(call, n, k, budget_s=0.6, min_calls=8):
    """Synchronous calls of k images each, cycling over n images, for ~budget_s: (images/s,
    per-call latency mean / p50 / p90 in ms).  The timing brackets each call only, as
    jpegdecodeperf.cpp:153-157 does."""
    lat, start = [], 0
    call(0, k)  # warm (first use of this shape)
    t_end = time.perf_counter() + budget_s
    while len(lat) < min_calls or time.perf_counter() < t_end:
        if start + k > n:
            start = 0
        t0 = time.perf_counter()
        call(start, k)
        lat.append(time.perf_counter() - t0)
        start += k
    a = np.array(lat) * 1e3
    return {"images_per_s": round(k * len(a) / (a.sum() * 1e-3), 1), "calls": len(a),
            "latency_ms": {"mean": round(float(a.mean()), 4), "p50": round(float(np.median(a)), 4),
                           "p90": round(float(np.percentile(a, 90)), 4)}}


def call_shapes(dec, datas, fmt, dev, threads=8):
    """The reference's default call shapes, on the same C2 images:
      - rocJpegDecode, one image per call (samples/jpegDecode/jpegdecode.cpp:163);
      - rocJpegDecodeBatched at 16 and 128 images per call;
      - jpegdecodeperf's default: batch 1 per rocJpegDecodeBatched, `threads` host threads with
        one handle each (jpegdecodeperf.cpp:201-202, 228-257), per-thread rates summed
        (:268-271, 281-300); once with streams from rocJpegStreamParse (host memory, as the
        sample does) and once resident.
    Resident streams unless stated.  Returns a dict for the JSON line."""
    import threading
    import torch
    import rocjpeg_amd as R
    L = R.lib()
    res = {}
    b = BatchRun(dec, datas[:256], fmt, dev)
    n = b.n
    p = ctypes.byref(b.params)

    def one(start, k):
        st = L.rocJpegDecode(dec.handle, b.hs[start], p, ctypes.byref(b.arr[start]))
        if st != 0:
            raise RuntimeError(R.error_name(st))

    def batched(start, k):
        st = L.rocJpegDecodeBatched(dec.handle, _sub(b.hs, ctypes.c_void_p, start, k), k, p,
                                    _sub(b.arr, R.RocJpegImage, start, k))
        if st != 0:
            raise RuntimeError(R.error_name(st))

    res["decode_batch1"] = _shape_loop(one, n, 1)
    res["batched_16"] = _shape_loop(batched, n, 16)
    res["batched_128"] = _shape_loop(batched, n, 128)
    shapes = b.shapes
    b.close()

    def perf_threads(resident, budget_s=1.0, bad_caller=False):
        """jpegdecodeperf: each thread its own handle, its own images, batch 1.  bad_caller: the
        last thread's every call is an unsupported (4:1:1) stream, which must fail alone; the rates
        and latencies are the healthy threads'."""
        per = max(1, min(len(datas), 256) // threads)
        rates, errs = [0.0] * threads, []
        lats = [[] for _ in range(threads)]
        barrier = threading.Barrier(threads)
        bad_bytes = open(os.path.join(ROOT, "tests", "golden", "img", "c411_q90_128x64.jpg"), "rb").read()

        def worker(t):
            try:
                d = R.JpegDecoder(R.Backend.HARDWARE, dev.index or 0)
                if bad_caller and t == threads - 1:
                    bs = R.JpegStream(bad_bytes)
                    bout = torch.empty(64 * 384, dtype=torch.uint8, device=dev)
                    bimg = R.make_image([bout.data_ptr()], [384])
                    bpar = R.decode_params(fmt)
                    hb = (ctypes.c_void_p * 1)(bs.handle)
                    barrier.wait()
                    t_end = time.perf_counter() + budget_s
                    while time.perf_counter() < t_end:
                        st_ = L.rocJpegDecodeBatched(d.handle, hb, 1, ctypes.byref(bpar), ctypes.byref(bimg))
                        if st_ != int(R.Status.JPEG_NOT_SUPPORTED):
                            raise RuntimeError("the bad caller got " + R.error_name(st_))
                    bs.close()
                    d.close()
                    return
                mine = datas[t * per:(t + 1) * per]
                if resident:
                    st_, streams = d.parse_device(mine)
                    if st_ != 0:
                        raise RuntimeError(R.error_name(st_))
                else:
                    streams = [R.JpegStream(x) for x in mine]
                hs = (ctypes.c_void_p * len(streams))(*[s.handle for s in streams])
                shp = shapes[0]
                outs = [torch.empty(r * q, dtype=torch.uint8, device=dev) for r, q in shp]
                img = R.make_image([o.data_ptr() for o in outs], [q for _, q in shp])
                par = R.decode_params(fmt)
                for j in range(2):  # warm
                    L.rocJpegDecodeBatched(d.handle, _sub(hs, ctypes.c_void_p, j % len(streams), 1), 1,
                                           ctypes.byref(par), ctypes.byref(img))
                barrier.wait()
                tot, cnt, t_end = 0.0, 0, time.perf_counter() + budget_s
                while time.perf_counter() < t_end:
                    j = cnt % len(streams)
                    t0 = time.perf_counter()
                    st_ = L.rocJpegDecodeBatched(d.handle, _sub(hs, ctypes.c_void_p, j, 1), 1, ctypes.byref(par),
                                                 ctypes.byref(img))
                    tot += time.perf_counter() - t0
                    lats[t].append(time.perf_counter() - t0)
                    if st_ != 0:
                        raise RuntimeError(R.error_name(st_))
                    cnt += 1
                rates[t] = cnt / tot if tot > 0 else 0.0
                for s_ in streams:
                    s_.close()
                d.close()
            except Exception as e:  # reported, never silent
                errs.append(repr(e))
                try:
                    barrier.abort()
                except Exception:
                    pass

        th = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        if errs:
            return {"error": errs[0]}
        healthy = [r for t, r in enumerate(rates) if not (bad_caller and t == threads - 1)]
        lat = np.concatenate([np.array(x) for x in lats if x]) * 1e3
        return {"images_per_s_summed": round(sum(healthy), 1), "threads": threads,
                "per_thread_images_per_s": [round(r, 1) for r in healthy],
                "spread_max_over_min": round(max(healthy) / min(healthy), 3) if min(healthy) > 0 else None,
                "latency_ms": {"p50": round(float(np.median(lat)), 4), "p90": round(float(np.percentile(lat, 90)), 4)},
                **({"bad_caller": "thread %d: an unsupported stream per call, failing alone" % (threads - 1)}
                   if bad_caller else {})}

    def perf_sample(passes=12, count=256):
        """The same shape from C, without the Python interpreter lock between the threads: the
        restated jpegdecodeperf (tests/c/rj_samples.cpp, linked -lrocjpeg) over `count` of the
        images written to a directory, -t threads -b 1 -fmt rgb, `passes` passes per thread."""
        import shutil
        import tempfile
        exe = os.path.join(ROOT, "tests", "c", "jpegdecodeperf_rj")
        if not os.access(exe, os.X_OK):
            return {"error": f"{exe} not built"}
        d = tempfile.mkdtemp(prefix="rj_perf_")
        try:
            for k, x in enumerate(datas[:count]):
                with open(os.path.join(d, f"img{k:04d}.jpg"), "wb") as f:
                    f.write(x)
            r = subprocess.run([exe, "-i", d, "-t", str(threads), "-b", "1", "-fmt", "rgb", "-n", str(passes)],
                               capture_output=True, text=True, timeout=300)
        finally:
            shutil.rmtree(d, ignore_errors=True)
        m = re.search(r"images/s summed ([0-9.]+)", r.stdout)
        if r.returncode != 0 or not m:
            return {"error": (r.stdout + r.stderr)[-500:]}
        return {"images_per_s_summed": float(m.group(1)), "threads": threads, "images": min(count, len(datas)),
                "passes": passes, "command": f"jpegdecodeperf_rj -t {threads} -b 1 -fmt rgb -n {passes}"}

    res[f"perf_threads{threads}_batch1_c_sample"] = perf_sample()
    res[f"perf_threads{threads}_batch1_host_streams"] = perf_threads(False)
    res[f"perf_threads{threads}_batch1_resident"] = perf_threads(True)
    # the coalescer with one misbehaving caller: healthy callers' p90 latency
    res[f"perf_threads{threads}_batch1_resident_one_bad_caller"] = perf_threads(True, bad_caller=True)
    c0 = R.coalesce_stats()
    res["coalescing"] = {"calls": c0[0], "combined_calls": c0[1], "combined_members": c0[2],
                         "note": "process totals of rocJpegAmdGetCoalesceStats: concurrent small calls "
                                 "on one device decoded together (rj_coalesce.h)"}
    res["note"] = ("1080p 4:2:0 C2 images -> RGB; latency = host wall time of one synchronous call; "
                   "jpegdecodeperf-style rates are per-thread images/s summed (jpegdecodeperf.cpp:268-271)")
    return res


def combined_blob(name, world, count, rank):
    """The whole batch as one file on the node: the ranks' dataset parts concatenated (rank 0
    writes it once; every rank memory-maps it).  Returns (path, offsets, sizes) of all
    world x count images, offsets into that file."""
    import torch.distributed as dist
    base = os.path.join(data_dir(), f"{name}_v{GEN_VERSION}_all_w{world}_n{count}")
    if rank == 0 and not (os.path.exists(base + ".bin") and os.path.exists(base + ".idx.npy")):
        offs, sizes, pos = [], [], 0
        tmp = f"{base}.{os.getpid()}"
        with open(tmp + ".bin", "wb") as f:
            for r in range(world):
                pb = part_base(name, r, count)
                idx = np.load(pb + ".idx.npy")
                offs.append(idx[0].astype(np.uint64) + np.uint64(pos))
                sizes.append(idx[1])
                with open(pb + ".bin", "rb") as g:
                    while True:
                        chunk = g.read(64 << 20)
                        if not chunk:
                            break
                        f.write(chunk)
                        pos += len(chunk)
        np.save(tmp + ".idx.npy", np.stack([np.concatenate(offs), np.concatenate(sizes)]))
        os.replace(tmp + ".bin", base + ".bin")
        os.replace(tmp + ".idx.npy", base + ".idx.npy")
    dist.barrier()
    idx = np.load(base + ".idx.npy")
    return base + ".bin", idx[0], idx[1]


class ShardRun(BatchRun):
    """A rank's share of a sharded batch through the C ABI: rocJpegAmdShardCreate (collective:
    plan + broadcast + GPU parse of this rank's images, resident), then each step is
    rocJpegAmdShardDecode with destinations for the whole batch (only this rank's are real)."""

    def __init__(self, dec, comm, blob, offs, sizes, fmt, dev):
        import torch
        import rocjpeg_amd as R
        from rocjpeg_amd import shard as S
        from tests.gpu_util import channel_shapes
        self.R, self.dec, self.fmt, self.comm = R, dec, fmt, comm
        t0 = time.perf_counter()
        self.shard = S.Shard(comm, dec.handle, blob, offs, sizes)
        if self.shard.status != 0:
            raise RuntimeError(f"rocJpegAmdShardCreate: {R.error_name(self.shard.status)}")
        self.parse_s = time.perf_counter() - t0
        self.mine = self.shard.images()
        self.datas = [bytes(blob[int(offs[i]):int(offs[i]) + int(sizes[i])]) for i in self.mine]
        self.streams = [R.JpegStream(d) for d in self.datas]  # host-parsed twins: shapes, host-input rate
        self.shapes = []
        for st in self.streams:
            nc, css, w, h = dec.image_info(st)
            self.shapes.append(channel_shapes(fmt, css, w, h))
        total = sum(r * p for shp in self.shapes for r, p in shp)
        self.out = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
        imgs, self.views, off = [], [], 0
        for shp in self.shapes:
            ptrs, pitches, vv = [], [], []
            for r, p in shp:
                ptrs.append(self.out[off:].data_ptr())
                pitches.append(p)
                vv.append(self.out[off:off + r * p].view(r, p))
                off += r * p
            imgs.append(R.make_image(ptrs, pitches))
            self.views.append(vv)
        self.params = R.decode_params(fmt)
        self.n = len(self.mine)
        self.arr = (R.RocJpegImage * max(1, self.n))(*imgs)
        self.arr_all = (R.RocJpegImage * len(offs))()
        for k, i in enumerate(self.mine):
            self.arr_all[i] = imgs[k]

    def step(self):
        st = self.shard.decode(self.params, self.arr_all)
        if st != 0:
            raise RuntimeError(self.R.error_name(st))

    def close(self):
        self.shard.close()
        self.comm.close()
        super().close()


def kernel_table(t, n):
    """(summed launch ms per call, launches per call, units (images) per launch) per kernel of
    a profiled pass; the pipelined K1/K2 launches each take an equal share of the intervals."""
    kern = {}
    if t["k1_launches"]:  # lean K1 (row images) is k_huff, the chunk-lane K1 k_huff_chunk (k_entropy: RJ_K1_CHUNK=0)
        k1 = "k_huff" if t["lean_k1"] else ("k_huff_chunk" if t["chunk_k1"] else "k_entropy")
        kern[k1] = (t["k1_launch_ms_sum"], t["k1_launches"], n / t["k1_launches"])
    if t["k2_launches"]:
        kern["k_rows"] = (t["k2_launch_ms_sum"], t["k2_launches"], n / t["k2_launches"])
    kern["k_destuff"] = (t["destuff_ms"], 1, n)
    if t["prog_images"]:
        for j, name in enumerate(PROG_KERNELS):
            if t["prog_kernel_launches"][j]:
                kern[name] = (t["prog_kernel_ms"][j], t["prog_kernel_launches"][j], n / t["prog_kernel_launches"][j])
        kern["k_rows_dense"] = (t["prog_rows_ms"], 1, n)
    return kern


def roofline(t, n, workload, per_image_bytes):
    """achieved = algorithmic bytes per image (ECS + 1,828 B tables + output)
    x the images one launch of the dominant kernel processes / its average launch time."""
    kern = kernel_table(t, n)
    dom = max(kern, key=lambda k: kern[k][0])
    ms_sum, launches, units = kern[dom]
    avg_ms = ms_sum / launches
    ach = units * per_image_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    r = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None,
         "basis": "SURVEY.md 8(d): (ECS + 1,828 B tables + output bytes) per image x images per launch / avg launch time",
         "algorithmic_bytes_per_image": int(per_image_bytes), "images_per_launch": round(units, 2),
         "avg_launch_ms": round(avg_ms, 4), "launches_per_step": launches,
         "per_kernel_launch_ms_sum": {k: round(v[0], 4) for k, v in kern.items()}}
    tr = pmc_traffic(dom, n, launches, workload)
    if tr:
        r["traffic"], r["traffic_source"] = tr
    # intermediate-inclusive figures (what the kernels actually move through HBM by design)
    entb = t["entry_bytes"]
    if dom in ("k_entropy", "k_huff", "k_huff_chunk") and t["k1_launches"]:
        b = (t["ecs_bytes"] + entb) / t["k1_launches"]
        r["achieved_incl_intermediates"] = round(b / (avg_ms * 1e-3) / 1e9, 2)
    if "k_rows" in kern:
        ms, la, _ = kern["k_rows"]
        b = (entb + t["output_bytes"]) / la
        r["stage2_k_rows"] = {"bytes_per_launch": int(b), "avg_launch_ms": round(ms / la, 4),
                              "achieved": round(b / (ms / la * 1e-3) / 1e9, 2),
                              "frac": round(b / (ms / la * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                              "basis": "sparse entries read + output written (BASELINE.md stage-2 efficiency)"}
    return r


def run_extra(name, dec, pool_path, steps, warmup, dev):
    """One more BASELINE config on this GPU with the same contract (N = 1 only)."""
    import rocjpeg_amd as R
    path, offs, sizes = pool_path
    with open(path, "rb") as f:
        raw = f.read()
    datas = [raw[int(o):int(o) + int(s)] for o, s in zip(offs, sizes)]
    del raw
    fmt = getattr(R.OutputFormat, WORKLOADS[name]["fmt"])
    b = BatchRun(dec, datas, fmt, dev)
    el = b.timed(steps, warmup)
    t = b.profiled(2)
    per_img = (t["ecs_bytes"] + TABLE_BYTES * b.n + t["output_bytes"]) / b.n
    rf = roofline(t, b.n, name, per_img)
    res = {"value": round(b.n * steps / el, 2), "unit": "images/s", "ms_per_step": round(el / steps * 1e3, 3),
           "steps": steps, "warmup": warmup, "workload": WORKLOADS[name]["workload"].format(batch=b.n),
           "output_format": WORKLOADS[name]["fmt"], "parity_sample": b.parity(parity_sample(b.n)),
           "parity_sample_images": len(parity_sample(b.n)),
           "roofline": {k: rf[k] for k in ("kernel", "achieved", "frac", "avg_launch_ms", "launches_per_step")},
           "per_kernel_launch_ms_sum": rf["per_kernel_launch_ms_sum"], "host_ms": round(t["host_ms"], 3),
           "split_intervals": t["split_intervals"], "serial_fallbacks": t["serial_fallbacks"]}
    if name == "c5":
        # a lone progressive image per rocJpegDecode (jpegdecode.cpp:163): its latency is set by
        # the longest scan's serial chain, not by the batch
        import rocjpeg_amd as R_
        L = R_.lib()
        p = ctypes.byref(b.params)

        def one(start, k):
            st = L.rocJpegDecode(dec.handle, b.hs[start], p, ctypes.byref(b.arr[start]))
            if st != 0:
                raise RuntimeError(R_.error_name(st))

        res["decode_batch1"] = _shape_loop(one, min(b.n, 64), 1, budget_s=1.0, min_calls=8)
    b.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--runs", type=int, default=5, help="timed runs of K steps; value = the median run (SURVEY 8d)")
    ap.add_argument("--batch", type=int, default=1024, help="images per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the other BASELINE configs at N=1")
    ap.add_argument("--path", type=int, default=0, help="0 auto (fused where legal), 1 general two-stage path")
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU, launched before this process touches the GPU; exit with its code
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    wl = WORKLOADS[args.workload]
    extras = [] if (world > 1 or args.no_extras) else [w for w in ("c2nori", "c3", "c4", "c5") if w != args.workload]

    # ---- host only (no GPU call yet): this rank's dataset part, the extra configs' data,
    # the CPU baseline's processes ----
    cores, nproc, core_rule = host_cores()
    t_gen = time.perf_counter()
    gen_pool = get_context("fork").Pool(max(1, min(cores, 32)), initializer=_init_gen)
    mine = dataset_part(args.workload, rank, args.batch, gen_pool)
    extra_data = {w: dataset_part(w, 0, args.batch, gen_pool) for w in extras} if rank == 0 else {}
    gen_pool.close()
    gen_pool.join()
    t_gen = time.perf_counter() - t_gen
    turbo = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # the CPU comparator: N = 1 only
        turbo = TurboBaseline(mine[0], mine[1], mine[2], cores)

    import torch
    import torch.distributed as dist
    # RJ_BENCH_SHARE_GPU=1 (rehearsal of the N > 1 path on a box with fewer GPUs than ranks):
    # ranks share the visible GPUs round-robin and talk over gloo on the host; the reported
    # numbers are then not a scaling measurement
    share = os.environ.get("RJ_BENCH_SHARE_GPU") == "1"
    gpu = local_rank % max(1, torch.cuda.device_count()) if share else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    cdev = torch.device("cpu") if share else dev  # the collectives' tensors
    if world > 1:
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        dist.barrier()  # every part is on disk

    if share and world > 1:  # the test build of the library carries the shared-memory test transport
        os.environ["RJ_LIB_PATH"] = os.path.join(ROOT, "rocjpeg_amd", "librocjpeg_amd_testcomm.so")
    import rocjpeg_amd as R
    from rocjpeg_amd import shard as S
    dec = R.JpegDecoder(R.Backend.HARDWARE, gpu)
    dec.set_path_policy(args.path)
    fmt = getattr(R.OutputFormat, wl["fmt"])
    t_tab = time.perf_counter()
    shard_cost, bcast_via = None, "none (one rank)"
    if world == 1:
        # N = 1: the drop-in call itself, rocJpegDecodeBatched over resident streams
        raw = np.memmap(mine[0], dtype=np.uint8, mode="r")
        datas = [bytes(raw[int(o):int(o) + int(z)]) for o, z in zip(mine[1], mine[2])]
        table = S.build_work_table(raw, mine[1], mine[2])
        del raw
        shard_cost = S.assign_shards(table, 1)
        t_build = t_tab = time.perf_counter() - t_tab
        run = BatchRun(dec, datas, fmt, dev)
    else:
        # N > 1: the C-ABI sharded entry a C caller uses (include/rocjpeg_amd.h): the batch is one
        # blob on the node (the ranks' parts concatenated), rocJpegAmdShardCreate plans on rank 0,
        # broadcasts the 64-B work table over the library's own communicator (RCCL; ranks that
        # share a GPU in the RJ_BENCH_SHARE_GPU rehearsal use its shared-memory test transport)
        # and keeps this rank's images resident; each step is rocJpegAmdShardDecode.
        path, offs, sizes = combined_blob(args.workload, world, args.batch, rank)
        blob = np.memmap(path, dtype=np.uint8, mode="r")
        if share:
            os.environ["RJ_COMM_TEST_SHM"] = f"/dev/shm/rj_bench_comm_{os.environ.get('MASTER_PORT', '0')}"
            if rank == 0 and os.path.exists(os.environ["RJ_COMM_TEST_SHM"]):
                os.unlink(os.environ["RJ_COMM_TEST_SHM"])
            dist.barrier()
        uid = torch.zeros(128, dtype=torch.uint8, device=cdev)
        if rank == 0 and not share:
            uid.copy_(torch.frombuffer(bytearray(S.comm_unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, src=0)
        comm = S.Comm(gpu, world, rank, bytes(uid.cpu().numpy()))
        t_tab = time.perf_counter()
        run = ShardRun(dec, comm, blob, offs, sizes, fmt, dev)
        t_tab = t_build = time.perf_counter() - t_tab
        table = run.shard.table
        shard_cost = [int(table["cost"][table["shard"] == r].sum()) for r in range(world)]
        bcast_via = ("rocJpegAmdShardCreate / rocJpegAmdShardDecode (librocjpeg_amd.so): work table over "
                     + ("the shared-memory test transport (RJ_BENCH_SHARE_GPU rehearsal)" if share else "RCCL"))
    datas = run.datas
    n = run.n

    # the median of >= 5 timed runs, each exactly K steps bracketed by barrier +
    # synchronize (max over ranks); the warm-up steps precede the first run only
    runs = [run.timed(args.steps, args.warmup if r == 0 else 0, world, cdev) for r in range(max(1, args.runs))]
    elapsed = float(np.median(runs))
    # parity of the timed run's own output (the last step's), before anything else writes it
    parity = run.parity(parity_sample(n))
    imgs = torch.tensor([n], dtype=torch.int64, device=cdev)
    if world > 1:
        dist.all_reduce(imgs)
    imgs_total = int(imgs.item()) * args.steps

    t = run.profiled(max(2, min(args.steps, 5)))
    per_img = (t["ecs_bytes"] + TABLE_BYTES * n + t["output_bytes"]) / n
    rf = roofline(t, n, args.workload, per_img)

    # PCIe-inclusive rate: the same images from host memory in every call (fresh
    # stream objects: each call stages the bitstreams through pinned memory + H2D)
    host_streams = [R.JpegStream(b) for b in datas]
    hs2 = (ctypes.c_void_p * n)(*[s.handle for s in host_streams])
    L = R.lib()
    st = L.rocJpegDecodeBatched(dec.handle, hs2, n, ctypes.byref(run.params), run.arr)
    torch.cuda.synchronize()
    t_h = time.perf_counter()
    for _ in range(5):
        st |= L.rocJpegDecodeBatched(dec.handle, hs2, n, ctypes.byref(run.params), run.arr)
    torch.cuda.synchronize()
    host_rate = 5 * n / (time.perf_counter() - t_h) if st == 0 else None
    t_p = time.perf_counter()
    for s in host_streams:
        s.parse(s._data)
    parse_host_rate = n / (time.perf_counter() - t_p)
    del host_streams

    shapes_res = None
    if rank == 0 and world == 1 and not args.no_extras:
        try:
            shapes_res = call_shapes(dec, datas, fmt, dev)
        except Exception as e:  # reported in the line, never silent
            shapes_res = {"error": repr(e)}

    res = None
    if rank == 0:
        K = args.steps
        res = {
            "metric": "images/s (1080p 4:2:0 batch) at 1/2/4/8 MI355X + achieved HBM GB/s",
            "value": round(imgs_total / elapsed, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / K * 1e3, 4),
            "runs": {"count": len(runs), "statistic": "median",
                     "ms_per_step": [round(x / K * 1e3, 4) for x in runs],
                     "spread": round((max(runs) - min(runs)) / elapsed, 5)},
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": wl["data"],
            "config": {"workload": wl["workload"].format(batch=args.batch), "batch_per_gpu": args.batch,
                       "output_format": wl["fmt"],
                       "parallelism": f"images sharded over {world} rank(s) by LPT on a broadcast work table",
                       "ecs_bytes_per_image": round(t["ecs_bytes"] / n)},
            **({"rehearsal": "RJ_BENCH_SHARE_GPU: ranks share the visible GPUs over gloo, not a scaling measurement"}
               if share and world > 1 else {}),
            "roofline": rf,
            "stages_ms_per_step": {k: round(t[k], 4) for k in ("host_ms", "h2d_ms", "destuff_ms", "huffman_ms",
                                                                "idct_ms", "output_ms", "total_ms")},
            "huffman_detail": {"intervals": t["intervals"], "chunks": t["chunks"],
                               "split_intervals": t["split_intervals"], "serial_fallbacks": t["serial_fallbacks"],
                               "entry_bytes_per_image": round(t["entry_bytes"] / n), "lean_k1": t["lean_k1"],
                               "lean_split": t["lean_split"], "lean_five": t.get("lean_five", 0), "chunk_k1": t["chunk_k1"]},
            "live_rows": {"live": t["live"], "rows_beside_k1": t["live_rows"], "rows_after_k1": t["rest_rows"],
                          "gave_up": t["live_pad"], "live_span_ms": round(t["live_ms"], 4),
                          "after_k1_span_ms": round(t["rest_ms"], 4)},
            # rj_decoder.h: the entry buffers the handle's first large calls tried (K1 + K2 ms each), the one kept
            "entry_placement": {"k1_k2_ms": [round(x, 4) for x in t["place_ms"][:t["place_tried"]]],
                                "picked": t["place_pick"]},
            "end_to_end_algorithmic_GBps": round(imgs_total * per_img / elapsed / 1e9, 2),
            "host_input_images_per_s_per_gpu": round(host_rate, 1) if host_rate else None,
            "parse_images_per_s": {"host_1_thread": round(parse_host_rate, 1),
                                   "gpu_marker_scan": round(n / run.parse_s, 1),
                                   "gpu_marker_scan_first_call": round(n / getattr(run, "parse_first_s", run.parse_s), 1),
                                   "gpu_marker_scan_stages_ms": getattr(run, "parse_stages_ms", None)},
            "parity_timed_output": parity,
            "parity_timed_output_images": len(parity_sample(n)),
            "work_table": {"images": int(len(table)), "bytes": int(table.nbytes),
                           "build_ms" if world == 1 else "create_ms": round(t_build * 1e3, 2),
                           "broadcast": bcast_via,
                           "lpt_imbalance": round(S.imbalance(shard_cost), 5),
                           "images_per_rank": [int((table["shard"] == r).sum()) for r in range(world)]},
            "dataset_gen_s": round(t_gen, 1),
        }
        if shapes_res is not None:
            res["call_shapes"] = shapes_res
        if t["prog_images"]:
            res["progressive_detail"] = {"images": t["prog_images"], "intervals": t["prog_intervals"],
                                         "levels": t["prog_levels"], "k1p_ms": round(t["prog_entropy_ms"], 4),
                                         "k2_dense_ms": round(t["prog_rows_ms"], 4)}
    run.close()
    if rank == 0 and extras:
        res["extra_workloads"] = {w: run_extra(w, dec, extra_data[w], max(3, args.steps // 2), 1, dev) for w in extras}
    if rank == 0:
        if turbo is not None:
            rate, nimg, wall = turbo.run()
            res["cpu_baseline"] = {
                "value": round(rate, 1), "unit": "images/s", "cores": cores, "kind": "reference",
                "lib": "libjpeg-turbo 3.1 (Pillow bundle): the reference's host decode path of BASELINE config C1; "
                       "BT.601 + fancy upsampling, a throughput comparator, not a parity oracle",
                "sample": f"{nimg} decodes of this run's images, {cores} processes (one per core; {core_rule}; "
                          f"nproc={nproc}), ~{wall:.1f} s each, per-process rates summed as jpegdecodeperf.cpp does"}
            res["cpu_oracle_1core"] = cpu_oracle(datas, run.shapes, int(fmt))
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
