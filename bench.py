#!/usr/bin/env python3
"""bench.py -- images/s of rocJpegDecodeBatched on MI355X (BASELINE.json `metric`).

Workload (BASELINE.json configs[1], "C2"): a batch of 1024 synthetic 1920x1080 4:2:0 baseline
JPEGs (q90, DRI = 120 MCUs = one MCU row), ROCJPEG_OUTPUT_RGB.  A step = one
rocJpegDecodeBatched call over the whole batch with the bitstreams already resident in HBM
(rocJpegAmdStreamsToDevice, outside the timed region) and RGB written to HBM.  N GPUs = N
ranks, each decoding its own batch (weak scaling; whole images are independent).  Rank 0
builds the work table (one seed per image) and broadcasts it (RCCL); nothing crosses GPUs
in the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--workload c2|c3|c4|c5]

The other BASELINE.json configs are available as --workload (never the driver's default line):
  c3  1024 x 1080p, 4:4:4 and 4:2:2 alternating, ROCJPEG_OUTPUT_YUV_PLANAR
  c4  mixed resolution 4:2:0 (640x480 .. 3840x2160, uniform by seed), RGB, DRI = one MCU row
  c5  progressive 4:2:0 1080p q90 (Pillow progressive=True, no DRI), RGB
"""
import argparse
import ctypes
import io
import json
import os
import sys
import time
from multiprocessing import get_context

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MUG = os.path.join(ROOT, "tests", "golden", "img", "mug_420.jpg")
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
PROG_KERNELS = ("k_prog", "k_prog_wave", "k_prog_fold")  # RocJpegAmdTimings.prog_kernel_*

_BASE = None


def _init_worker():
    global _BASE
    from PIL import Image
    _BASE = np.asarray(Image.open(MUG).convert("RGB"))


C4_SIZES = [(640, 480), (1280, 720), (1920, 1080), (2560, 1440), (3840, 2160)]


def _make_jpeg(args):
    """Seeded crop of the reference mug image + N(0,2) noise, encoded q90 with DRI = one MCU
    row (BASELINE.md generator).  w == 0: size drawn from C4_SIZES by the seed."""
    seed, w, h, quality, sub, rst_blocks, progressive = args
    if w == 0:
        w, h = C4_SIZES[seed % len(C4_SIZES)]
        rst_blocks = (w + 15) // 16 if rst_blocks else 0  # MCUs per row
    if sub == -1:  # C3: 4:4:4 and 4:2:2 alternating
        sub = 0 if seed % 2 == 0 else 1
        rst_blocks = (w + 7) // 8 if sub == 0 else (w + 15) // 16  # one MCU row
    from PIL import Image
    rng = np.random.default_rng(seed)
    y0 = int(rng.integers(0, _BASE.shape[0] - h + 1))
    x0 = int(rng.integers(0, _BASE.shape[1] - w + 1))
    a = _BASE[y0:y0 + h, x0:x0 + w].astype(np.float32) + rng.normal(0.0, 2.0, (h, w, 3))
    b = io.BytesIO()
    kw = dict(quality=quality, subsampling=sub)
    if rst_blocks:
        kw["restart_marker_blocks"] = rst_blocks
    if progressive:
        kw["progressive"] = True
    Image.fromarray(np.clip(a, 0, 255).astype(np.uint8)).save(b, "JPEG", **kw)
    return b.getvalue()


def make_dataset(seeds, w=1920, h=1080, quality=90, sub=2, rst_blocks=120, procs=16, progressive=False):
    jobs = [(int(s), w, h, quality, sub, rst_blocks, progressive) for s in seeds]
    with get_context("fork").Pool(procs, initializer=_init_worker) as pool:
        return pool.map(_make_jpeg, jobs, chunksize=8)


def cpu_baseline(data_list, shapes, fmt, what, budget_s=12.0):
    """The CPU oracle (oracle/jpeg_oracle.c, a plain single-threaded restatement of the same
    decode: Huffman, ISLOW IDCT, reference CSC) on a bounded sample of the same images."""
    from tests import oracle_lib as O
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s and n < len(data_list):
        st, _ = O.oracle_decode(data_list[n], fmt, shapes[n])
        assert st == 0
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 3), "unit": "images/s", "cores": 1, "kind": "port",
            "sample": f"{n} of the batch's {what}, oracle/jpeg_oracle.c, 1 thread, {dt:.1f} s"}


def _turbo_worker(blobs):
    from PIL import Image
    t0 = time.perf_counter()
    for b in blobs:
        Image.open(io.BytesIO(b)).convert("RGB").load()
    return len(blobs), time.perf_counter() - t0


def turbo_baseline(data_list, procs):
    """Context only (not the cpu_baseline): Pillow's libjpeg-turbo on `procs` host cores."""
    per = max(1, min(len(data_list) // procs, 48))
    shards = [data_list[(i * per) % len(data_list):][:per] for i in range(procs)]
    t0 = time.perf_counter()
    with get_context("fork").Pool(procs) as pool:
        res = pool.map(_turbo_worker, shards)
    wall = time.perf_counter() - t0
    n = sum(r[0] for r in res)
    return {"value": round(n / max(wall, 1e-9), 1), "unit": "images/s", "cores": procs,
            "lib": "Pillow bundled libjpeg-turbo (BT.601 + fancy upsampling: throughput context only)"}


def pmc_traffic(kernel, batch, launches, workload="c2"):
    """HBM bytes per launch of `kernel` from the committed PMC profile (tools/gpu_pmc.sh +
    tools/pmc_traffic.py on this workload; profiles/pmc_traffic.json for C2,
    pmc_traffic_<workload>.json for the others): FETCH_SIZE x 2 (gfx950 correction,
    MI355X_MICROARCH.md HBM section) + WRITE_SIZE summed over a decode call, per image, scaled to
    this call's batch and divided over its launches of the kernel.  None if absent."""
    name = "pmc_traffic.json" if workload == "c2" else f"pmc_traffic_{workload}.json"
    path = os.path.join(ROOT, "profiles", name)
    try:
        with open(path) as f:
            prof = json.load(f)
        k = prof["kernels"][kernel]
        return int(k["hbm_bytes_per_image"] * batch / max(1, launches))
    except (OSError, KeyError, ValueError):
        return None


def work_table(rank, world, batch, device):
    """Rank 0 builds the work table (one image seed per slot, `batch` images per rank) and one
    broadcast (RCCL on GPUs, gloo in the CPU tests) hands every rank the whole table; each rank
    keeps its own row.  Returns this rank's seeds."""
    import torch
    import torch.distributed as dist
    table = torch.empty((world, batch), dtype=torch.int64, device=device)
    if rank == 0:
        table.copy_(torch.arange(world * batch, dtype=torch.int64).view(world, batch) + 1234)
    if world > 1:
        dist.broadcast(table, src=0)
    return table[rank].cpu().tolist()


def _workloads():
    import rocjpeg_amd as R
    return {
        "c2": {"gen": {}, "fmt": R.OutputFormat.RGB,
               "data": "synthetic: seeded 1920x1080 crops of the reference mug_420.jpg + N(0,2) noise, Pillow q90 4:2:0 DRI=120",
               "workload": "C2: batch of {batch} x 1920x1080 4:2:0 baseline JPEG q90, RI=120 MCUs, ROCJPEG_OUTPUT_RGB, bitstreams resident in HBM",
               "sample": "1920x1080 4:2:0 q90 RI=120 images -> RGB"},
        "c3": {"gen": {"sub": -1}, "fmt": R.OutputFormat.YUV_PLANAR,
               "data": "synthetic: seeded 1920x1080 crops of mug_420.jpg + N(0,2) noise, Pillow q90, 4:4:4 / 4:2:2 alternating, DRI = 1 MCU row",
               "workload": "C3: batch of {batch} x 1920x1080 baseline q90, 4:4:4 and 4:2:2 alternating, ROCJPEG_OUTPUT_YUV_PLANAR, resident",
               "sample": "1920x1080 4:4:4 / 4:2:2 images -> YUV_PLANAR"},
        "c4": {"gen": {"w": 0, "h": 0}, "fmt": R.OutputFormat.RGB,
               "data": "synthetic: seeded crops of mug_420.jpg + N(0,2) noise, sizes 640x480..3840x2160 uniform by seed, Pillow q90 4:2:0, DRI = 1 MCU row",
               "workload": "C4: batch of {batch} mixed-resolution 4:2:0 baseline JPEGs per GPU (640x480..3840x2160), ROCJPEG_OUTPUT_RGB, resident",
               "sample": "mixed-resolution 4:2:0 images -> RGB"},
        "c5": {"gen": {"rst_blocks": 0, "progressive": True}, "fmt": R.OutputFormat.RGB,
               "data": "synthetic: seeded 1920x1080 crops of mug_420.jpg + N(0,2) noise, Pillow q90 4:2:0 progressive=True (no DRI)",
               "workload": "C5: batch of {batch} x 1920x1080 4:2:0 progressive JPEG q90 (10 scans, no DRI), ROCJPEG_OUTPUT_RGB, resident",
               "sample": "1920x1080 4:2:0 q90 progressive images -> RGB"},
    }


def main():
    global WORKLOADS
    WORKLOADS = _workloads()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--path", type=int, default=0, help="0 auto (fused where legal), 1 general two-stage path")
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c4", "c5"])
    args = ap.parse_args()
    wl = WORKLOADS[args.workload]

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    seeds = work_table(rank, world, args.batch, dev)
    procs = max(1, min(16, (os.cpu_count() or 16)))
    t_gen = time.perf_counter()
    data = make_dataset(seeds, procs=procs, **wl["gen"])
    t_gen = time.perf_counter() - t_gen

    import rocjpeg_amd as R
    dec = R.JpegDecoder(R.Backend.HARDWARE, local_rank)
    dec.set_path_policy(args.path)
    streams = [R.JpegStream(b) for b in data]
    dec.streams_to_device(streams)
    # destinations: one HBM arena, every channel sized as the reference samples size them
    # (samples/rocjpeg_samples_utils.h:318-399, tests/gpu_util.py channel_shapes)
    from tests.gpu_util import channel_shapes
    fmt = wl["fmt"]
    shapes = []
    for s in streams:
        nc, css, w, h = dec.image_info(s)
        shapes.append(channel_shapes(fmt, css, w, h))
    total = sum(r * p for shp in shapes for r, p in shp)
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    imgs, views, off = [], [], 0
    for shp in shapes:
        ptrs, pitches, vv = [], [], []
        for r, p in shp:
            ptrs.append(out[off:].data_ptr())
            pitches.append(p)
            vv.append(out[off:off + r * p].view(r, p))
            off += r * p
        imgs.append(R.make_image(ptrs, pitches))
        views.append(vv)
    params = R.decode_params(fmt)
    n = len(streams)
    hs = (ctypes.c_void_p * n)(*[s.handle for s in streams])
    arr = (R.RocJpegImage * n)(*imgs)
    L = R.lib()

    def step():
        st = L.rocJpegDecodeBatched(dec.handle, hs, n, ctypes.byref(params), arr)
        if st != 0:
            raise RuntimeError(R.error_name(st))

    for _ in range(args.warmup):
        step()
    dec.set_profiling(True)
    k1 = {}
    stage = {"host_ms": 0.0, "h2d_ms": 0.0, "destuff_ms": 0.0, "huffman_ms": 0.0, "idct_ms": 0.0, "output_ms": 0.0}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = None
    for _ in range(args.steps):
        step()
        last = dec.last_timings()
        for k in stage:
            stage[k] += last[k]
        for k in ("entropy_chunks_ms", "entropy_resolve_ms", "entropy_serial_ms", "k1_launch_ms_sum",
                  "k2_launch_ms_sum", "prog_entropy_ms", "prog_rows_ms"):
            k1[k] = k1.get(k, 0.0) + last[k]
        for j, name in enumerate(PROG_KERNELS):
            k1[name] = k1.get(name, 0.0) + last["prog_kernel_ms"][j]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    dec.set_profiling(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # PCIe-inclusive rate: the same batch from host memory (fresh stream objects, so
    # every call stages the bitstreams through pinned memory + H2D); reported, never `value`
    host_streams = [R.JpegStream(b) for b in data]
    hs2 = (ctypes.c_void_p * n)(*[s.handle for s in host_streams])
    st = L.rocJpegDecodeBatched(dec.handle, hs2, n, ctypes.byref(params), arr)  # warm-up
    torch.cuda.synchronize()
    t_h = time.perf_counter()
    host_steps = 3
    for _ in range(host_steps):
        st |= L.rocJpegDecodeBatched(dec.handle, hs2, n, ctypes.byref(params), arr)
    torch.cuda.synchronize()
    host_rate = host_steps * n / (time.perf_counter() - t_h) if st == 0 else None
    del host_streams

    # parse rates (outside the timed region): host parser (rocJpegStreamParse, one thread) and
    # the GPU marker scan (rocJpegAmdStreamParseDevice: headers on the host, O(bytes) on the GPU,
    # streams left resident -- includes their HBM allocations)
    t_p = time.perf_counter()
    tmp = [R.JpegStream(b) for b in data]
    parse_host_rate = n / (time.perf_counter() - t_p)
    del tmp
    dec.parse_device(data[:8])  # warm-up (first launch, buffers)
    t_p = time.perf_counter()
    pst, tmp = dec.parse_device(data)
    parse_dev_rate = n / (time.perf_counter() - t_p) if pst == 0 else None
    del tmp

    # parity spot-check of this run's output (first images vs the CPU oracle), outside timing
    from tests import oracle_lib as O
    parity_ok = True
    for q in range(min(2, n)):
        ost, want = O.oracle_decode(data[q], int(fmt), shapes[q])
        parity_ok = parity_ok and ost == 0 and all(np.array_equal(v.cpu().numpy(), w_) for v, w_ in zip(views[q], want))
    parity_ok = bool(parity_ok)

    if rank == 0:
        K = args.steps
        imgs_total = world * args.batch * K
        value = imgs_total / elapsed
        per = {k: v / K for k, v in stage.items()}
        ecs = last["ecs_bytes"]
        coef = last["coef_bytes"]
        outb = last["output_bytes"]
        # per-kernel launch durations (HIP events on each launch's own stream, summed over the
        # call's launches -- with the pipelined launch K1 and K2 run as two launches each) and
        # the algorithmic bytes those launches move (DESIGN.md "Roofline"):
        #   K0 k_destuff: ECS bytes read + written; K1 k_entropy: destuffed ECS read + sparse
        #   entries written; K2 k_rows: entries read + output written
        entb = last["entry_bytes"]
        kern = {
            "k_destuff": (stage["destuff_ms"] / K, 1, 2 * ecs),
            "k_entropy": (k1["k1_launch_ms_sum"] / K, max(1, last["k1_launches"]), ecs + entb),
            "k_rows": (k1["k2_launch_ms_sum"] / K, max(1, last["k2_launches"]), entb + outb),
        }
        if last["prog_images"]:
            # progressive: k_prog lanes read their destuffed scans and write the
            # coefficient band / DC-refinement bits; k_prog_wave reads its scans and writes a
            # first scan's band + masks, or reads the nonzero masks and writes one 32-B record per
            # refined block; k_prog_fold reads the records and reads +
            # writes each touched dense block; K2 (dense) reads the coefficients, writes the output
            pc = last["prog_coef_bytes"]
            for j, name in enumerate(PROG_KERNELS):
                if last["prog_kernel_launches"][j]:
                    kern[name] = (k1[name] / K, last["prog_kernel_launches"][j], last["prog_kernel_bytes"][j])
            kern["k_rows_dense"] = (k1["prog_rows_ms"] / K, 1, pc + outb)
        dom = max(kern, key=lambda k: kern[k][0])
        t_sum, launches, algo_bytes = kern[dom]
        ach = algo_bytes / (t_sum * 1e-3) / 1e9 if t_sum > 0 else 0.0
        traffic = pmc_traffic(dom, args.batch, launches, args.workload)
        res = {
            "metric": "images/s (1080p 4:2:0 batch) at 1/2/4/8 MI355X + achieved HBM GB/s",
            "value": round(value, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": wl["data"],
            "config": {"workload": wl["workload"].format(batch=args.batch),
                       "batch_per_gpu": args.batch, "output_format": fmt.name, "parallelism": f"images sharded, {world} rank(s)",
                       "ecs_bytes_per_image": round(ecs / args.batch)},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "algorithmic_bytes_per_launch": int(algo_bytes / launches),
                         "avg_launch_ms": round(t_sum / launches, 4), "launches_per_step": launches,
                         "per_kernel_launch_ms_sum": {k: round(v[0], 4) for k, v in kern.items()}},
            "stages_ms_per_step": {k: round(v, 4) for k, v in per.items()},
            "huffman_detail": dict({k: round(v / K, 4) for k, v in k1.items()}, chunks=last["chunks"],
                                   intervals=last["intervals"], split_intervals=last["split_intervals"],
                                   serial_fallbacks=last["serial_fallbacks"]),
            "end_to_end_algorithmic_GBps": round((ecs + outb) / (elapsed / K) / 1e9, 2),
            "host_input_images_per_s_per_gpu": round(host_rate, 1) if host_rate else None,
            "parse_images_per_s": {"host_1_thread": round(parse_host_rate, 1),
                                   "gpu_marker_scan": round(parse_dev_rate, 1) if parse_dev_rate else None},
            "parity_first_image": parity_ok,
            "dataset_gen_s": round(t_gen, 1),
        }
        if last["prog_images"]:
            res["progressive_detail"] = {"images": last["prog_images"], "intervals": last["prog_intervals"],
                                         "levels": last["prog_levels"],
                                         "k1p_ms": round(k1["prog_entropy_ms"] / K, 4),
                                         "k1p_launches": {n: last["prog_kernel_launches"][j]
                                                          for j, n in enumerate(PROG_KERNELS)},
                                         "k2_dense_ms": round(k1["prog_rows_ms"] / K, 4)}
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(data, shapes, int(fmt), wl["sample"])
            res["cpu_libjpeg_turbo"] = turbo_baseline(data, procs)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
