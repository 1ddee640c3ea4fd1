#!/usr/bin/env python3
"""bench.py -- images/s of rocJpegDecodeBatched on MI355X (BASELINE.json `metric`).

Workload (BASELINE.json configs[1], "C2"): a batch of 1024 synthetic 1920x1080 4:2:0 baseline
JPEGs (q90, DRI = 120 MCUs = one MCU row), ROCJPEG_OUTPUT_RGB.  A step = one
rocJpegDecodeBatched call over the whole batch with the bitstreams already resident in HBM
(rocJpegAmdStreamsToDevice, outside the timed region) and RGB written to HBM.  N GPUs = N
ranks, each decoding its own batch (weak scaling; whole images are independent).  Rank 0
builds the work table (one seed per image) and broadcasts it (RCCL); nothing crosses GPUs
in the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
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

_BASE = None


def _init_worker():
    global _BASE
    from PIL import Image
    _BASE = np.asarray(Image.open(MUG).convert("RGB"))


def _make_jpeg(args):
    """Seeded 1080p crop of the reference mug image + N(0,2) noise, encoded 4:2:0 q90 with
    DRI = one MCU row (BASELINE.md generator)."""
    seed, w, h, quality, sub, rst_blocks = args
    from PIL import Image
    rng = np.random.default_rng(seed)
    y0 = int(rng.integers(0, _BASE.shape[0] - h + 1))
    x0 = int(rng.integers(0, _BASE.shape[1] - w + 1))
    a = _BASE[y0:y0 + h, x0:x0 + w].astype(np.float32) + rng.normal(0.0, 2.0, (h, w, 3))
    b = io.BytesIO()
    kw = dict(quality=quality, subsampling=sub)
    if rst_blocks:
        kw["restart_marker_blocks"] = rst_blocks
    Image.fromarray(np.clip(a, 0, 255).astype(np.uint8)).save(b, "JPEG", **kw)
    return b.getvalue()


def make_dataset(seeds, w=1920, h=1080, quality=90, sub=2, rst_blocks=120, procs=16):
    jobs = [(int(s), w, h, quality, sub, rst_blocks) for s in seeds]
    with get_context("fork").Pool(procs, initializer=_init_worker) as pool:
        return pool.map(_make_jpeg, jobs, chunksize=8)


def cpu_baseline(data_list, budget_s=12.0):
    """The CPU oracle (oracle/jpeg_oracle.c, a plain single-threaded restatement of the same
    decode: Huffman, ISLOW IDCT, reference CSC) on a bounded sample of the same images."""
    from tests import oracle_lib as O
    lib = O.oracle()
    w3, h = 1920 * 3, 1080
    out = np.zeros((h, w3), np.uint8)
    ptrs = (ctypes.c_void_p * 4)(out.ctypes.data, None, None, None)
    pitches = (ctypes.c_uint32 * 4)(w3, 0, 0, 0)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s and n < len(data_list):
        d = data_list[n]
        st = lib.oj_decode(d, len(d), 3, 0, 0, 0, 0, ptrs, pitches)
        assert st == 0
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 3), "unit": "images/s", "cores": 1, "kind": "port",
            "sample": f"{n} of the batch's 1920x1080 4:2:0 q90 RI=120 images -> RGB, oracle/jpeg_oracle.c, 1 thread, {dt:.1f} s"}


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


def pmc_traffic(kernel, batch, launches):
    """HBM bytes per launch of `kernel` from the committed PMC profile (tools/gpu_pmc.sh +
    tools/pmc_traffic.py on this workload): FETCH_SIZE x 2 (gfx950 correction, MI355X_MICROARCH.md
    HBM section) + WRITE_SIZE summed over a decode call, per image, scaled to this call's batch
    and divided over its launches of the kernel.  None if absent."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--path", type=int, default=0, help="0 auto (fused where legal), 1 general two-stage path")
    args = ap.parse_args()

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
    data = make_dataset(seeds, procs=procs)
    t_gen = time.perf_counter() - t_gen

    import rocjpeg_amd as R
    dec = R.JpegDecoder(R.Backend.HARDWARE, local_rank)
    dec.set_path_policy(args.path)
    streams = [R.JpegStream(b) for b in data]
    dec.streams_to_device(streams)
    nc, css, w, h = dec.image_info(streams[0])
    W, H = w[0], h[0]
    out = torch.empty((args.batch, H, 3 * W), dtype=torch.uint8, device=dev)
    imgs = [R.make_image([out[i].data_ptr()], [3 * W]) for i in range(args.batch)]
    params = R.decode_params(R.OutputFormat.RGB)
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
                  "k2_launch_ms_sum"):
            k1[k] = k1.get(k, 0.0) + last[k]
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

    # parity spot-check of this run's output (first image vs the CPU oracle), outside timing
    from tests import oracle_lib as O
    ost, want = O.oracle_decode(data[0], 3, [(H, 3 * W)])
    parity_ok = bool(ost == 0 and np.array_equal(out[0].cpu().numpy(), want[0]))

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
        dom = max(kern, key=lambda k: kern[k][0])
        t_sum, launches, algo_bytes = kern[dom]
        ach = algo_bytes / (t_sum * 1e-3) / 1e9 if t_sum > 0 else 0.0
        traffic = pmc_traffic(dom, args.batch, launches)
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
            "data": "synthetic: seeded 1920x1080 crops of the reference mug_420.jpg + N(0,2) noise, Pillow q90 4:2:0 DRI=120",
            "config": {"workload": "C2: batch of 1024 x 1920x1080 4:2:0 baseline JPEG q90, RI=120 MCUs, ROCJPEG_OUTPUT_RGB, bitstreams resident in HBM",
                       "batch_per_gpu": args.batch, "output_format": "RGB", "parallelism": f"images sharded, {world} rank(s)",
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
            "parity_first_image": parity_ok,
            "dataset_gen_s": round(t_gen, 1),
        }
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(data)
            res["cpu_libjpeg_turbo"] = turbo_baseline(data, procs)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
