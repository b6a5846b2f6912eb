#!/usr/bin/env python3
"""bench.py -- device-resident fp32 -> ZFP encode throughput (BASELINE.json metric), 1..N MI355X.

Workload (BASELINE configs[1] = C2): a 256 Mi-float contiguous fp32 gradient bucket per GPU (1-D, 4-value blocks),
fixed rate 16 (the caller's default, hw/models/train_imagenet.py:155), inputs resident in HBM before timing.
A step = one encode of the whole bucket (one gfx950 kernel launch). N > 1: one process per GPU, each encodes its
own 256 Mi shard of an N x 1 GiB bucket (weak scaling, the C4 sharding); the RCCL all-gather of the compressed
shards is timed separately and reported under "allgather" (it is the exchange step, not the encode metric).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from gcow_amd import codec  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table); 6.29 TB/s measured float4 copy
N_VALUES = 256 * 1024 * 1024


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--rate", type=float, default=16.0)
    ap.add_argument("--values", type=int, default=N_VALUES)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-allgather", action="store_true")
    ap.add_argument("--no-host-e2e", action="store_true")
    return ap.parse_args()


def cpu_baseline(x: torch.Tensor, rate: float):
    """The reference sw/ encoder (compiled in place from /root/reference into oracle/_ref) on this host's cores.
    sw/ only has a 2-D layout (sw/src/zfp.c:12-24), so the same bucket bytes are viewed as 16384 x 16384 and coded
    with the same expert params sw/ would get for rate 16 in 2-D (minbits = maxbits = 256). Falls back to the 1-D
    restatement (oracle port) when oracle/_ref is absent."""
    import ctypes as C

    import numpy as np

    from oracle import oracle as O

    a = x.detach().cpu().numpy()
    R = O.ref()
    if R is not None:
        side = int(round(a.size ** 0.5))
        rows = a.size // side
        a2 = a[: rows * side].reshape(rows, side)
        p = O.rate(rate, 2)
        out = np.zeros(O.max_words(a2.shape, p) + 4, np.uint64)
        t0 = time.perf_counter()
        R.gcow_ref_compress_2d(a2.ctypes.data_as(C.POINTER(C.c_float)), side, rows, *p.tuple(),
                               out.ctypes.data_as(C.POINTER(C.c_uint64)), out.nbytes)
        dt = time.perf_counter() - t0
        kind, sample = "reference", "sw/ zfp_compress (g++ -O2) on the full bucket viewed as %dx%d fp32, fixed rate %g " \
                                    "(minbits=maxbits=%d), 1 thread" % (rows, side, rate, p.maxbits)
        cores = 1
    else:
        p = O.rate(rate, 1)
        t0 = time.perf_counter()
        O.compress(a, p)
        dt = time.perf_counter() - t0
        kind, sample = "port", "oracle C restatement, full bucket 1-D fixed rate %g, 1 thread" % rate
        cores = 1
    return {"value": round(a.nbytes / dt / 2 ** 30, 4), "unit": "GiB/s", "cores": cores, "kind": kind,
            "sample": sample, "seconds": round(dt, 3), "cpu": platform.processor() or platform.machine()}


def load_pmc_traffic(kernel_substr: str, workload: str):
    """HBM bytes per launch from a committed rocprofv3 --pmc pass (profiles/*pmc_traffic.json), or None."""
    prof = os.path.join(ROOT, "profiles")
    if not os.path.isdir(prof):
        return None
    for f in sorted(os.listdir(prof), reverse=True):
        if f.endswith("pmc_traffic.json"):
            try:
                d = json.load(open(os.path.join(prof, f)))
            except Exception:
                continue
            if d.get("workload") == workload and kernel_substr in d.get("kernel", ""):
                return d.get("hbm_bytes_per_launch")
    return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    n = args.values
    x = torch.empty(n, dtype=torch.float32, device=dev)
    codec.fill_normal(x, 1e-3, seed=0x67636F77 + rank, inject=True)
    p = codec.rate(args.rate, 1)
    enc = codec.Encoder((n,), torch.float32, p, dev)
    stream = torch.cuda.current_stream(dev)

    for _ in range(args.warmup):
        enc(x, stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        enc(x, stream)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps  # one kernel per step on this stream: HIP-event kernel time
    step_ms = wall * 1e3 / args.steps
    if world > 1:
        t = torch.tensor([step_ms, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        step_ms, kern_ms = t.tolist()

    in_bytes = n * 4
    out_bytes = n * args.rate / 8
    value = world * in_bytes / (step_ms / 1e3) / 2 ** 30
    workload = "c2_1d_fp32_fixed_rate%g_%dMi_per_gpu" % (args.rate, n // (1 << 20))
    achieved = (in_bytes + out_bytes) / (kern_ms / 1e3) / 1e9

    extra = {}
    # RCCL all-gather of the compressed shards (C4 exchange step), timed on its own
    if world > 1 and not args.no_allgather:
        from gcow_amd import dist as gdist
        nb = n // 4
        e = enc(x, stream)
        for _ in range(2):
            full = gdist.allgather_fixed(e.words, nb, p.maxbits)
        torch.cuda.synchronize()
        dist.barrier()
        ta = time.perf_counter()
        reps = max(3, args.steps // 4)
        for _ in range(reps):
            e = enc(x, stream)
            full = gdist.allgather_fixed(e.words, nb, p.maxbits)
        torch.cuda.synchronize()
        dist.barrier()
        ag_ms = (time.perf_counter() - ta) * 1e3 / reps
        t = torch.tensor([ag_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ag_ms = t.item()
        # parity of the gathered single stream: rank 0 re-encodes every rank's shard locally and compares
        ok = True
        if rank == 0:
            y = torch.empty_like(x)
            shard_words = nb * p.maxbits // 64
            for r in range(world):
                codec.fill_normal(y, 1e-3, seed=0x67636F77 + r, inject=True)
                er = codec.encode(y, p)
                ok = ok and bool(torch.equal(er.words[:shard_words], full[r * shard_words:(r + 1) * shard_words]))
            del y
        extra["encode_allgather"] = {"ms_per_step": round(ag_ms, 4),
                                     "GiBps_input": round(world * in_bytes / (ag_ms / 1e3) / 2 ** 30, 2),
                                     "gathered_bytes_per_rank": int(full.numel() * 8),
                                     "gathered_stream_equals_single_gpu_encode": ok}
        del full

    if rank == 0 and world == 1 and not args.no_host_e2e:
        # path that starts and ends in host memory: pinned H2D of the bucket + encode + D2H of the stream
        h_in = x.cpu().pin_memory()
        h_out = torch.empty(int(out_bytes // 8), dtype=torch.int64, pin_memory=True)
        for _ in range(2):
            x.copy_(h_in, non_blocking=True)
            e = enc(x, stream)
            h_out.copy_(e.words[: h_out.numel()], non_blocking=True)
        torch.cuda.synchronize()
        th = time.perf_counter()
        reps = 5
        for _ in range(reps):
            x.copy_(h_in, non_blocking=True)
            e = enc(x, stream)
            h_out.copy_(e.words[: h_out.numel()], non_blocking=True)
        torch.cuda.synchronize()
        h_ms = (time.perf_counter() - th) * 1e3 / reps
        henc = codec.HostEncoder(n, torch.float32, p, chunks=8, device=dev)
        for _ in range(2):
            henc(h_in, h_out)
        th = time.perf_counter()
        for _ in range(reps):
            henc(h_in, h_out)
        o_ms = (time.perf_counter() - th) * 1e3 / reps
        extra["host_e2e"] = {"ms_per_step": round(h_ms, 3), "GiBps_input": round(in_bytes / (h_ms / 1e3) / 2 ** 30, 2),
                             "overlapped_ms_per_step": round(o_ms, 3),
                             "overlapped_GiBps_input": round(in_bytes / (o_ms / 1e3) / 2 ** 30, 2),
                             "note": "pinned hipMemcpyAsync H2D + encode + D2H, PCIe-inclusive (not `value`); "
                                     "overlapped = 8 chunks, H2D / encode / D2H on three streams (codec.HostEncoder)"}
        del h_in, h_out

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(x, args.rate)
        except Exception as ex:  # the GPU measurement stands on its own
            cpu = {"error": repr(ex)}

    if rank == 0:
        kname = "k_encode_fixed1d_np"
        traffic = load_pmc_traffic(kname, workload)
        line = {
            "metric": "GiB/s device-resident fp32->ZFP encode, 256Mi-float bucket, 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_ms, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: N(0,1e-3) fp32 with 1/64 zero, 1/4096 tiny (INT_MIN path), 1/4096 subnormal blocks",
            "config": {"workload": workload, "values_per_gpu": n, "layout": "1-D contiguous, 4-value blocks",
                       "mode": "fixed-rate", "rate_bits_per_value": args.rate, "minbits": p.minbits,
                       "maxbits": p.maxbits, "bucket_bytes_total": world * in_bytes},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic,
                         "kernel": kname, "kernel_ms": round(kern_ms, 5),
                         "algorithmic_bytes_per_launch": int(in_bytes + out_bytes)},
            "cpu_baseline": cpu,
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
