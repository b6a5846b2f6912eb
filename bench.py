#!/usr/bin/env python3
"""bench.py -- device-resident fp32 -> ZFP encode throughput (BASELINE.json metric) on 1..N MI355X.

Workload (BASELINE configs[1] = C2): a 256 Mi-float contiguous fp32 gradient bucket per GPU (1-D, 4-value blocks),
fixed rate 16 (the caller's default, hw/models/train_imagenet.py:155), inputs resident in HBM before timing. A step is
one encode of the whole bucket (one gfx950 kernel launch). `value` = all ranks' input bytes / the max-over-ranks time
of exactly --steps steps after --warmup untimed ones (weak scaling: every rank encodes its own 256 Mi shard of an
N x 1 GiB bucket, the C4 sharding; no collective on the encode path).

`python bench.py --gpus N` with N > 1 and no torchrun environment launches N worker processes itself (torchrun on
127.0.0.1, before this process touches the GPU); under torchrun (the driver's launch) it is one of the ranks.

Extra objects on the same JSON line (they never change `value`):
  roofline          the encode kernel's HIP-event time vs the HBM roofline (read-only bytes per BASELINE.md, and
                    read + write), traffic = rocprofv3 PMC bytes per launch from profiles/ (traffic_source names it)
  per_launch_ms     first / median / max kernel time over the timed steps (the clock ramps under a burst of launches)
  steady_state      the same kernel after >= 0.25 s of back-to-back launches
  N > 1:  encode_allgather (C4 exchange: encode + RCCL all-gather of the compressed shards, gathered stream checked
          against the oracle on sampled ranges of every shard), subgroups (1/2/4/.. ranks over dist.new_group),
          strong (8 GiB split k ways), c5_sharded (bf16 accuracy 1e-6: encode + length exchange + padded all-gather
          + one-launch stitch, checked against the oracle at every shard start), hook_exchange (the DDP hook's whole
          exchange: all-gather + decode-mean of every stream vs the sharded receive, both checked)
  N = 1:  host_e2e (pinned H2D + encode + D2H; PCIe-inclusive), configs (C2 rate 8 encode and rate 16 decode, C3 512^3
          rate 8 / accuracy 1e-3 encode + decode, C5 bf16 accuracy 1e-6 / 1e-3 device and host path), cpu_baseline
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import statistics
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table); 6.29 TB/s measured float4 copy
N_VALUES = 256 * 1024 * 1024
SEED = 0x67636F77
METRIC = "GiB/s device-resident fp32->ZFP encode, 256Mi-float bucket, 1/2/4/8 GPU"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rate", type=float, default=16.0)
    ap.add_argument("--values", type=int, default=N_VALUES)
    ap.add_argument("--strong-gib", type=float, default=8.0, help="C4 strong-scaling bucket (GiB of fp32)")
    ap.add_argument("--c5-values", type=int, default=N_VALUES, help="bf16 values per rank in the c5_sharded leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="only the headline measurement")
    ap.add_argument("--stub", action="store_true",
                    help="harness self-test on CPU: gloo, a trivial step instead of the encode (tests only)")
    ap.add_argument("--stub-mismatch", action="store_true",
                    help="stub mode: report a failed oracle check (tests that the run then exits non-zero)")
    ap.add_argument("--multi-legs", action="store_true",
                    help="run the N > 1 legs (exchange, subgroups, strong, c5_sharded) even at N = 1, over a one-rank "
                         "RCCL group (tests: exercises the multi-GPU code on a one-GPU box)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------------------------------ launcher
def launcher_cmd(nproc: int, argv) -> list:
    """torchrun's single-node standalone rendezvous on 127.0.0.1: its c10d store binds port 0 itself and the workers
    are handed the port it got (no port picked here and released before torchrun binds it: VERDICT r5's race)."""
    return [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr=127.0.0.1",
            "--nproc-per-node=%d" % nproc, os.path.abspath(__file__)] + list(argv)


def launch(args, argv) -> int:
    """N > 1 without a torchrun environment: start N ranks (one process per GPU) through torchrun on 127.0.0.1, each
    with the argument list this process was given (`argv`), and return its exit code. Called before anything
    initialises HIP in this process."""
    cmd = launcher_cmd(args.gpus, argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["GCOW_BENCH_LAUNCHER"] = "self"
    return subprocess.call(cmd, env=env)


# ------------------------------------------------------------------------------------------------------ timing
class Ctx:
    def __init__(self, args):
        self.args = args
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.stub = args.stub
        self.group = self.world > 1 or (args.multi_legs and not args.stub)
        # one rank (--multi-legs at N = 1): an in-process store, no port to race other jobs on the box for
        solo = {"store": dist.HashStore(), "rank": 0, "world_size": 1} if self.world == 1 and self.group else {}
        if self.group:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if self.stub:
                dist.init_process_group("gloo", **solo)
            else:
                torch.cuda.set_device(self.local)
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local), **solo)
        self.dev = torch.device("cpu") if self.stub else torch.device("cuda", self.local)
        if not self.stub:
            torch.cuda.set_device(self.dev)

    def sync(self):
        if not self.stub:
            torch.cuda.synchronize(self.dev)

    def barrier(self, group=None):
        if self.world > 1:
            dist.barrier(group=group)

    def max_over_ranks(self, vals, group=None):
        if self.world == 1:
            return list(vals)
        t = torch.tensor(list(vals), dtype=torch.float64, device=self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        return t.tolist()


def timed(ctx: Ctx, step, warmup: int, steps: int, group=None, stream=None, walls=None):
    """W untimed steps, then exactly K steps bracketed by barrier + synchronize on both sides. Returns (wall ms per
    step, per-step kernel ms from HIP events on `stream` -- [] in stub mode). `walls` (a list) receives the host wall
    ms of every call, warmup included (meaningful for steps that synchronise themselves, e.g. HostEncoder)."""
    def call():
        t = time.perf_counter()
        step()
        if walls is not None:
            walls.append(round((time.perf_counter() - t) * 1e3, 3))
    for _ in range(warmup):
        call()
    ctx.sync()
    ctx.barrier(group)
    ctx.sync()
    evs = []
    if not ctx.stub:
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t0 = time.perf_counter()
    if evs:
        evs[0].record(stream)
    for i in range(steps):
        call()
        if evs:
            evs[i + 1].record(stream)
    ctx.sync()
    ctx.barrier(group)
    ctx.sync()
    wall = (time.perf_counter() - t0) * 1e3 / steps
    per = [evs[i].elapsed_time(evs[i + 1]) for i in range(steps)] if evs else []
    return wall, per


def steady_ms(ctx: Ctx, step, stream, settle_s: float = 0.25, steps: int = 50) -> float:
    """The same step's HIP-event time once the clock has settled under load (settle_s of back-to-back steps first):
    the sustained figure beside the driver-protocol one (5 + 20 launches, inside the DVFS dip)."""
    t_end = time.perf_counter() + settle_s
    while time.perf_counter() < t_end:
        for _ in range(10):
            step()
        ctx.sync()
    _, per = timed(ctx, step, 0, steps, stream=stream)
    return round(sum(per) / len(per), 4)


def gib(nbytes: float, ms: float) -> float:
    return nbytes / (ms / 1e3) / 2 ** 30


def roof(read_bytes: float, write_bytes: float, ms: float, kernel: str, basis: str = "read") -> dict:
    """Roofline of one kernel (or pass sequence). `achieved` counts the uncompressed side only (BASELINE.md:63): the
    values read for an encoder (basis "read"), the values written for a decoder (basis "write");
    `achieved_read_write` adds the compressed bytes."""
    a = (read_bytes if basis == "read" else write_bytes) / (ms / 1e3) / 1e9
    arw = (read_bytes + write_bytes) / (ms / 1e3) / 1e9
    return {"bound": "hbm", "achieved": round(a, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(a / HBM_PEAK_GBPS, 4), "basis": "uncompressed bytes %s" % basis,
            "achieved_read_write": round(arw, 1),
            "frac_read_write": round(arw / HBM_PEAK_GBPS, 4), "kernel": kernel, "kernel_ms": round(ms, 5),
            "algorithmic_read_bytes": int(read_bytes), "algorithmic_write_bytes": int(write_bytes)}


def load_pmc_traffic(kernel_substr: str, workload: str):
    """HBM bytes per launch (read + write) from a committed rocprofv3 --pmc pass: (bytes, file) or (None, None)."""
    prof = os.path.join(ROOT, "profiles")
    if not os.path.isdir(prof):
        return None, None
    for f in sorted(os.listdir(prof), reverse=True):
        if f.endswith("pmc_traffic.json"):
            try:
                d = json.load(open(os.path.join(prof, f)))
            except Exception:
                continue
            if d.get("workload") == workload and kernel_substr in d.get("kernel", ""):
                return d.get("hbm_bytes_per_launch"), "profiles/" + f
    return None, None


# ------------------------------------------------------------------------------------------------------ oracle checks
def _u64(t: torch.Tensor):
    import numpy as np
    return t.contiguous().cpu().numpy().view(np.uint64)


def bits_at(words, off: int, nbits: int):
    """nbits bits of a uint64 word array starting at bit off, as ceil(nbits / 64) words (LSB-first)."""
    import numpy as np
    nw = (nbits + 63) // 64
    w = np.concatenate([words, np.zeros(2, np.uint64)])
    i, sh = off // 64, off % 64
    out = w[i:i + nw + 1].copy()
    if sh:
        out = (out[:nw] >> np.uint64(sh)) | (out[1:nw + 1] << np.uint64(64 - sh))
    else:
        out = out[:nw]
    if nbits % 64:
        out[-1] &= np.uint64((1 << (nbits % 64)) - 1)
    return out


def check_fixed_gathered(full: torch.Tensor, world: int, n: int, p, samples: int = 1 << 16) -> bool:
    """Rank 0: for every shard r, regenerate r's input, oracle-encode a sampled range (the shard's start and a
    16-block-aligned interior offset) and compare it with the gathered stream's words at that block."""
    import numpy as np

    from gcow_amd import codec
    from oracle import oracle as O
    op = O.expert(*p.tuple())
    y = torch.empty(n, dtype=torch.float32, device=full.device)
    rng = np.random.default_rng(7)
    ok = True
    nb = n // 4
    for r in range(world):
        codec.fill_normal(y, 1e-3, seed=SEED + r, inject=True)
        for off in (0, int(rng.integers(0, (n - samples) // 64)) * 64):
            a = y[off:off + samples].cpu().numpy()
            w, bits = O.compress(a, op)
            b0 = r * nb + off // 4
            got = bits_at(_u64(full[(b0 * p.maxbits) // 64:(b0 * p.maxbits + bits) // 64 + 2]),
                          (b0 * p.maxbits) % 64, bits)
            ok = ok and got.tobytes() == w.tobytes()
    return ok


# ------------------------------------------------------------------------------------------------------ legs
def leg_c4_exchange(ctx, enc, x, p, n, out_bytes):
    from gcow_amd import dist as gdist
    nb = n // 4
    res = {}

    def step():
        e = enc(x)
        res["full"] = gdist.allgather_fixed(e.words, nb, p.maxbits)

    reps = max(3, ctx.args.steps // 4)
    ms, _ = timed(ctx, step, 2, reps)
    ms = ctx.max_over_ranks([ms])[0]
    full = res.pop("full")
    ok = check_fixed_gathered(full, ctx.world, n, p) if ctx.rank == 0 else None
    d = {"ms_per_step": round(ms, 4), "GiBps_input": round(gib(ctx.world * n * 4, ms), 2),
         "gathered_bytes_per_rank": int(full.numel() * 8),
         "allgather_GBps_per_rank_ingress": round((ctx.world - 1) * out_bytes / (ms / 1e3) / 1e9, 1),
         "gathered_stream_matches_oracle": ok,
         "oracle_check": "every shard: its first 64 Ki values and a random interior 64 Ki-value range re-encoded by "
                         "the oracle, compared with the gathered stream at that block"}
    del full
    return d


def leg_subgroups(ctx, p, n):
    """The 1/2/4/.. curve inside the N-rank job: k-rank sub-communicators over the first k ranks (dist.new_group),
    members encode their own 256 Mi shard then all-gather the compressed shards within the subgroup."""
    from gcow_amd import codec
    from gcow_amd import dist as gdist
    ks = [k for k in (1, 2, 4, 8, 16, 32) if k < ctx.world] + [ctx.world]
    groups = {k: (dist.new_group(list(range(k))) if k < ctx.world else None) for k in ks}
    x = torch.empty(n, dtype=torch.float32, device=ctx.dev)
    codec.fill_normal(x, 1e-3, seed=SEED + ctx.rank, inject=True)
    enc = codec.Encoder((n,), torch.float32, p, ctx.dev)
    nb = n // 4
    curve = []
    for k in ks:
        member = ctx.rank < k
        e_ms = a_ms = 0.0
        if member:
            g = groups[k]
            e_ms, _ = timed(ctx, lambda: enc(x), 3, 10, group=g)
            res = {}

            def step():
                e = enc(x)
                res["f"] = gdist.allgather_fixed(e.words, nb, p.maxbits, group=g)

            a_ms, _ = timed(ctx, step, 1, 4, group=g)
            res.clear()
        ctx.barrier()
        e_ms, a_ms = ctx.max_over_ranks([e_ms, a_ms])
        curve.append({"k": k, "encode_ms": round(e_ms, 4), "encode_GiBps": round(gib(k * n * 4, e_ms), 2),
                      "encode_allgather_ms": round(a_ms, 4)})
    del x, enc
    return curve


def leg_strong(ctx, p, total_values):
    """C4 strong scaling: one total_values bucket split over k = 1, 2, 4, .. ranks (each member encodes
    total/k values; all-gather of the compressed shards within the k-rank subgroup)."""
    from gcow_amd import codec
    from gcow_amd import dist as gdist
    ks = [k for k in (1, 2, 4, 8, 16, 32) if k < ctx.world] + [ctx.world]
    out = []
    for k in ks:
        g = dist.new_group(list(range(k))) if k < ctx.world else None
        member = ctx.rank < k
        e_ms = a_ms = 0.0
        if member:
            m = total_values // k // 64 * 64
            x = torch.empty(m, dtype=torch.float32, device=ctx.dev)
            codec.fill_normal(x, 1e-3, seed=SEED + 1000 + ctx.rank, inject=True)
            enc = codec.Encoder((m,), torch.float32, p, ctx.dev)
            e_ms, _ = timed(ctx, lambda: enc(x), 3, 10, group=g)
            res = {}

            def step():
                e = enc(x)
                res["f"] = gdist.allgather_fixed(e.words, m // 4, p.maxbits, group=g)

            a_ms, _ = timed(ctx, step, 1, 3, group=g)
            res.clear()
            del x, enc
            torch.cuda.empty_cache()
        ctx.barrier()
        e_ms, a_ms = ctx.max_over_ranks([e_ms, a_ms])
        out.append({"k": k, "values_per_rank": total_values // k, "encode_ms": round(e_ms, 4),
                    "encode_GiBps": round(gib(total_values * 4, e_ms), 2), "encode_allgather_ms": round(a_ms, 4)})
    return {"bucket_bytes": total_values * 4, "curve": out}


def leg_c5_sharded(ctx, n):
    """C5 at N ranks: each rank encodes its own 256 Mi bf16 shard at accuracy 1e-6, then the variable-rate exchange
    (length all-gather, padded stream all-gather, one-launch stitch). Rank 0 checks every shard's first 64 Ki values
    against the oracle at the shard's stitched bit offset, and the total bit count against the per-shard sum."""
    import numpy as np

    from gcow_amd import codec
    from gcow_amd import dist as gdist
    p = codec.accuracy(1e-6)
    x32 = torch.empty(n, dtype=torch.float32, device=ctx.dev)
    codec.fill_normal(x32, 1e-3, seed=SEED + ctx.rank, inject=True)
    xb = x32.to(torch.bfloat16)
    del x32
    enc = codec.Encoder((n,), torch.bfloat16, p, ctx.dev)
    e_ms, _ = timed(ctx, lambda: enc(xb), 3, 10)
    res = {}

    def step():
        e = enc(xb)
        res["o"] = gdist.allgather_variable(e.words, e.bits_dev)

    a_ms, _ = timed(ctx, step, 1, 4)
    e_ms, a_ms = ctx.max_over_ranks([e_ms, a_ms])
    words, total = res.pop("o")
    lens = gdist.gather_lengths(enc.bits_dev, ctx.dev)[1]
    ok = None
    if ctx.rank == 0:
        from oracle import oracle as O
        op = O.expert(*p.tuple())
        ok = total == sum(lens)
        y = torch.empty(n, dtype=torch.float32, device=ctx.dev)
        off = 0
        for r in range(ctx.world):
            codec.fill_normal(y, 1e-3, seed=SEED + r, inject=True)
            a = y[: 1 << 16].to(torch.bfloat16).cpu().view(torch.int16).numpy().view(np.uint16)
            w, b = O.compress(a, op)
            got = bits_at(_u64(words[off // 64:(off + b) // 64 + 2]), off % 64, b)
            ok = ok and got.tobytes() == w.tobytes()
            off += lens[r]
        del y
    del xb, enc, words
    return {"values_per_rank": n, "dtype": "bf16", "mode": "accuracy 1e-6",
            "encode_ms": round(e_ms, 4), "encode_GiBps_input": round(gib(ctx.world * n * 2, e_ms), 2),
            "encode_exchange_ms": round(a_ms, 4), "compressed_bits_total": int(total),
            "stitched_stream_matches_oracle": ok}


def leg_hook_exchange(ctx, n):
    """The DDP hook's whole exchange at N ranks on one 256 Mi-value fp32 bucket per rank (rate 16 and accuracy 1e-6,
    the caller's defaults): `allgather` = encode, all-gather of the streams (lengths first for variable rate), one
    decode-mean of all W streams (ddp.compressed_allgather_hook); `sharded` = encode, cut positions, all-to-all of
    the shard pieces, one decode-mean of this rank's shard, all-gather of the mean shards
    (ddp.compressed_sharded_hook). Both give the same bucket bit for bit (checked); rank 0 also checks the first
    64 Ki values of the sharded result against the oracle's mean of every rank's decode."""
    import numpy as np

    from gcow_amd import codec, ddp
    from gcow_amd import dist as gdist
    W = ctx.world
    x = torch.empty(n, dtype=torch.float32, device=ctx.dev)
    codec.fill_normal(x, 1e-3, seed=SEED + 77 + ctx.rank, inject=True)
    out = {}
    for name, p, stride in (("rate16", codec.rate(16, 1), 0), ("acc1e-6", codec.accuracy(1e-6), 16)):
        # both hooks encode with the 8-block index (ddp.SHARDED_INDEX_STRIDE); the all-gather hook sends it packed
        sstride = ddp.SHARDED_INDEX_STRIDE if stride else 0
        enc = senc = codec.Encoder((n,), torch.float32, p, ctx.dev, index_stride=sstride)
        ag = torch.empty(n, dtype=torch.float32, device=ctx.dev)
        sh = torch.empty(n, dtype=torch.float32, device=ctx.dev)

        def allgather_path():
            e = enc(x)
            if stride:
                _, lens_h = gdist.gather_lengths(e.bits_dev, ctx.dev)
                sw = max(1, max((b + 63) // 64 for b in lens_h))
                g = gdist.allgather_padded(e.words, (lens_h[ctx.rank] + 63) // 64, sw, pad=2)
                pk = codec.pack_index16(e.index, n, p)
                ni = pk.numel()
                idx = torch.empty(W * ni, dtype=torch.int64, device=ctx.dev)
                gdist.allgather_into(idx, pk)
                codec.decode_mean(g, sw, W, n, p, idx, ni, codec.INDEX_PACKED16, out=ag)
            else:
                nw = ((n + 3) // 4 * p.maxbits + 63) // 64
                g = torch.zeros(W * nw + 2, dtype=torch.int64, device=ctx.dev)
                gdist.allgather_into(g[: W * nw], e.words[:nw].contiguous())
                codec.decode_mean(g, nw, W, n, p, out=ag)

        def sharded_path():
            e = senc(x)
            if stride:
                pieces, pw, pidx, iw, lo, hi = gdist.shard_pieces_variable(e.words, e.bits_dev, e.index, n, sstride)
            else:
                pieces, pw, lo, hi = gdist.shard_pieces_fixed(e.words, n, p.maxbits)
                pidx, iw = None, 0
            shard = sh[lo:hi]
            if hi > lo:
                codec.decode_mean(pieces, pw, W, hi - lo, p, pidx, iw, sstride, out=shard)
            gdist.allgather_shards(sh, shard, n)

        a_ms, _ = timed(ctx, allgather_path, 1, 4)
        s_ms, _ = timed(ctx, sharded_path, 1, 4)
        a_ms, s_ms = ctx.max_over_ranks([a_ms, s_ms])
        same = bool(torch.equal(ag.view(torch.int32), sh.view(torch.int32)))
        same = bool(ctx.max_over_ranks([0.0 if same else 1.0])[0] == 0.0)
        ok = None
        if ctx.rank == 0:
            from oracle import oracle as O
            op = O.expert(*p.tuple())
            m = 1 << 16
            y = torch.empty(n, dtype=torch.float32, device=ctx.dev)
            acc = np.zeros(m, np.float32)
            for r in range(W):
                codec.fill_normal(y, 1e-3, seed=SEED + 77 + r, inject=True)
                a = y[:m].cpu().numpy()
                acc = acc + O.decompress(O.compress(a, op)[0], (m,), op)
            want = acc / np.float32(W)
            ok = bool(np.array_equal(sh[:m].cpu().numpy().view(np.uint32), want.view(np.uint32))) and same
            del y
        out[name] = {"allgather_exchange_ms": round(a_ms, 4), "sharded_exchange_ms": round(s_ms, 4),
                     "sharded_equals_allgather": same, "sharded_mean_matches_oracle": ok}
        del enc, senc, ag, sh
        torch.cuda.empty_cache()
    del x
    return out


def leg_host_e2e(ctx, enc, x, p, n, in_bytes, out_bytes):
    from gcow_amd import codec
    h_in = x.cpu().pin_memory()
    h_out = torch.empty(int(out_bytes // 8) + 2, dtype=torch.int64, pin_memory=True)
    nwo = int(out_bytes // 8)

    def seq():
        x.copy_(h_in, non_blocking=True)
        e = enc(x)
        h_out[:nwo].copy_(e.words[:nwo], non_blocking=True)

    settle_host(lambda: (seq(), ctx.sync()))
    h_ms, _ = timed(ctx, seq, 0, 5)
    henc = codec.HostEncoder(n, torch.float32, p, chunks=16, device=ctx.dev)
    settle_host(lambda: henc(h_in, h_out), 0.25)
    o_ms, _ = timed(ctx, lambda: henc(h_in, h_out), 0, 5)
    ok = host_stream_check(henc, h_in, h_out, p)
    return {"ms_per_step": round(h_ms, 3), "GiBps_input": round(gib(in_bytes, h_ms), 2),
            "overlapped_ms_per_step": round(o_ms, 3), "overlapped_GiBps_input": round(gib(in_bytes, o_ms), 2),
            "host_stream_matches_oracle": ok,
            "note": "pinned H2D + encode + D2H, PCIe-inclusive (not `value`); overlapped: 16 chunks on 3 streams"}


def settle_host(step, seconds: float = 1.0) -> list:
    """Untimed calls of a host-resident step (it synchronises itself) for `seconds` of wall time, at least two; returns
    their wall ms. After a long GPU-only phase the first ~0.55 s of PCIe traffic runs its D2H copies at about half
    rate whatever the copy issue order or buffers (profiles/r06_host_path_transient.log: 19.3 ms per call, then 11.8
    from one call to the next, ~0.55 s in), so a count of warmup calls is not a warm state."""
    walls = []
    t_end = time.perf_counter() + seconds
    while len(walls) < 2 or time.perf_counter() < t_end:
        t = time.perf_counter()
        step()
        walls.append(round((time.perf_counter() - t) * 1e3, 3))
    return walls


def oracle_threads() -> int:
    """Threads for the oracle checks and the multi-thread CPU legs: the CPUs this process may actually use, i.e.
    min(sched_getaffinity, the cgroup's CPU quota) -- not the host's CPU count."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    q = _cpu_quota()
    return max(1, min(aff, int(q)) if q else aff)


def host_stream_check(henc, h_in: torch.Tensor, h_out: torch.Tensor, p) -> bool:
    """One more HostEncoder call (the timed object, 16 chunks) into a zeroed pinned buffer; the WHOLE host-resident
    stream is compared with the threaded oracle's encode of the same host bucket (every chunk seam included)."""
    import numpy as np

    from oracle import oracle as O
    h_out.zero_()
    bits = henc(h_in, h_out)
    a = h_in.numpy() if h_in.dtype == torch.float32 else h_in.view(torch.int16).numpy().view(np.uint16)
    w, b = O.compress(a, O.expert(*p.tuple()), threads=oracle_threads())
    nw = (b + 63) // 64
    return bool(bits == b and np.array_equal(h_out[:nw].numpy().view(np.uint64), w[:nw]))


def leg_configs(ctx):
    """C3 and C5 at N = 1, each with its own roofline fraction (read-only bytes = the input; read + write adds the
    compressed bytes)."""
    from gcow_amd import codec
    out = {}
    # C2 at rate 8 (rates 16 and 8) and the rate-16 decode (8(f) rank 1), same bucket as the headline
    n = N_VALUES
    x = torch.empty(n, dtype=torch.float32, device=ctx.dev)
    codec.fill_normal(x, 1e-3, seed=SEED, inject=True)
    st = torch.cuda.current_stream(ctx.dev)
    enc8 = codec.Encoder((n,), torch.float32, codec.rate(8, 1), ctx.dev)
    w8, per = timed(ctx, lambda: enc8(x, st), 5, 20, stream=st)
    k8 = sum(per) / len(per)
    out["c2_rate8"] = {"ms_per_step": round(w8, 4), "GiBps_input": round(gib(n * 4, w8), 2), "kernel_ms": round(k8, 4),
                       "steady_ms": steady_ms(ctx, lambda: enc8(x, st), st),
                       "encode_roofline": roof(n * 4, n, k8, "k_encode_fixed1d_np<F32, 32>")}
    del enc8
    enc16 = codec.Encoder((n,), torch.float32, codec.rate(16, 1), ctx.dev)
    e16 = enc16(x, st)
    back = torch.empty_like(x)
    wd, dper = timed(ctx, lambda: codec.decode(e16, out=back, stream=st), 5, 20, stream=st)
    dk = sum(dper) / len(dper)
    out["c2_rate16_decode"] = {"ms_per_step": round(wd, 4), "GiBps_output": round(gib(n * 4, wd), 2),
                               "kernel_ms": round(dk, 4), "max_abs_err": float((back - x).abs().max()),
                               "steady_ms": steady_ms(ctx, lambda: codec.decode(e16, out=back, stream=st), st),
                               "decode_roofline": roof(n * 2, n * 4, dk, "k_decode_fixed1d_np<64, 16>", basis="write")}
    del enc16, e16, back, x
    torch.cuda.empty_cache()
    f = codec.c3_field(ctx.dev)  # the field tests/test_gpu_parity.py::test_c3_full_size_roundtrip checks
    nbytes = f.numel() * 4
    for name, p, stride in (("c3_512cube_rate8", codec.rate(8, 3), 0),
                            ("c3_512cube_acc1e-3", codec.accuracy(1e-3), 1)):
        enc = codec.Encoder(tuple(f.shape), torch.float32, p, ctx.dev, index_stride=stride)
        st = torch.cuda.current_stream(ctx.dev)
        e_ms, per = timed(ctx, lambda: enc(f, st), 5, 20, stream=st)
        k_ms = sum(per) / len(per)
        e = enc(f, st)
        cbits = e.bits
        back = torch.empty_like(f)
        d_ms, dper = timed(ctx, lambda: codec.decode(e, out=back, stream=st), 5, 20, stream=st)
        dk = sum(dper) / len(dper)
        err = float((back - f).abs().max())
        es = steady_ms(ctx, lambda: enc(f, st), st)
        ds = steady_ms(ctx, lambda: codec.decode(e, out=back, stream=st), st)
        kn = "k_encode3d_fixed" if stride == 0 else "k_count3d + k_scan_ranges + k_encode3d_var"
        out[name] = {"encode_ms": round(k_ms, 4), "encode_GiBps_input": round(gib(nbytes, k_ms), 2),
                     "decode_ms": round(dk, 4), "decode_GiBps_output": round(gib(nbytes, dk), 2),
                     "encode_steady_ms": es, "decode_steady_ms": ds,
                     "bits_per_value": round(cbits / f.numel(), 3), "max_abs_err": err,
                     "encode_roofline": roof(nbytes, cbits / 8, k_ms, kn),
                     "decode_roofline": roof(cbits / 8, nbytes, dk, "k_decode3d_fixed" if stride == 0 else
                                             "k_decode_staged<3>", basis="write")}
        del enc, back, e
    del f
    torch.cuda.empty_cache()
    n = N_VALUES
    x32 = torch.empty(n, dtype=torch.float32, device=ctx.dev)
    codec.fill_normal(x32, 1e-3, seed=SEED, inject=True)
    xb = x32.to(torch.bfloat16)
    del x32
    host_legs = []
    for name, tol in (("c5_bf16_acc1e-6", 1e-6), ("c5_bf16_acc1e-3", 1e-3)):
        p = codec.accuracy(tol)
        enc = codec.Encoder((n,), torch.bfloat16, p, ctx.dev, index_stride=16)
        st = torch.cuda.current_stream(ctx.dev)
        _, per = timed(ctx, lambda: enc(xb, st), 5, 20, stream=st)
        k_ms = sum(per) / len(per)
        cbits = enc(xb, st).bits
        er = roof(n * 2, cbits / 8, k_ms,
                  "k_count1d_var_tile + k_scan_ranges_mw + k_encode1d_var_tile (+ k_encode1d_var_tile_big)")
        # HBM bytes of one encode (all four kernels) from a committed PMC pass (tools/c5_traffic.py); the input is read
        # twice (count + coder) and the byte lengths written and read once
        er["traffic"], src = load_pmc_traffic("k_count1d_var_tile", name + "_256Mi")
        er["traffic_source"] = src
        # the receive side (the caller's codec cost is compress + decompress, hw/models/train_imagenet.py:458-467):
        # the 1-D variable-rate decode of this stream (block index every 16 blocks) into fp32, given the stream as a
        # receiver holds it (its own length, not the encoder's capacity-sized buffer)
        e = exact_stream(enc(xb, st))
        back = torch.empty(n, dtype=torch.float32, device=ctx.dev)
        _, dper = timed(ctx, lambda: codec.decode(e, out=back, stream=st), 5, 20, stream=st)
        dk = sum(dper) / len(dper)
        dr = roof(cbits / 8, n * 4, dk, "k_decode1d_var_lean<128>", basis="write")
        # the same decode into a bf16 tensor (the bf16 bucket's own dtype: rounded to nearest even in the store)
        back_b = torch.empty(n, dtype=torch.bfloat16, device=ctx.dev)
        _, bper = timed(ctx, lambda: codec.decode(e, out=back_b, stream=st), 5, 20, stream=st)
        bk = sum(bper) / len(bper)
        es = steady_ms(ctx, lambda: enc(xb, st), st)
        ds = steady_ms(ctx, lambda: codec.decode(e, out=back, stream=st), st)
        del back_b
        out[name] = {"encode_ms": round(k_ms, 4), "encode_GiBps_input": round(gib(n * 2, k_ms), 2),
                     "encode_steady_ms": es, "decode_steady_ms": ds,
                     "bits_per_value": round(cbits / n, 3), "encode_roofline": er,
                     "decode_ms": round(dk, 4), "decode_GiBps_output": round(gib(n * 4, dk), 2),
                     "decode_roofline": dr,
                     "decode_bf16_out_ms": round(bk, 4), "decode_bf16_out_GiBps_output": round(gib(n * 2, bk), 2)}
        host_legs.append((name, p))
        del enc, e, back
    del xb
    torch.cuda.empty_cache()
    # the same bucket in fp32 at the caller's default tolerance: encode and the receive-side decode
    x32 = torch.empty(n, dtype=torch.float32, device=ctx.dev)
    codec.fill_normal(x32, 1e-3, seed=SEED, inject=True)
    p = codec.accuracy(1e-6)
    enc = codec.Encoder((n,), torch.float32, p, ctx.dev, index_stride=16)
    st = torch.cuda.current_stream(ctx.dev)
    _, per = timed(ctx, lambda: enc(x32, st), 5, 20, stream=st)
    k_ms = sum(per) / len(per)
    e = exact_stream(enc(x32, st))
    cbits = e.bits
    back = torch.empty_like(x32)
    _, dper = timed(ctx, lambda: codec.decode(e, out=back, stream=st), 5, 20, stream=st)
    dk = sum(dper) / len(dper)
    out["var1d_f32_acc1e-6"] = {
        "encode_ms": round(k_ms, 4), "encode_GiBps_input": round(gib(n * 4, k_ms), 2),
        "bits_per_value": round(cbits / n, 3),
        "encode_roofline": roof(n * 4, cbits / 8, k_ms, "k_count1d_var_tile + k_scan_ranges_mw + k_encode1d_var_tile"),
        "decode_ms": round(dk, 4), "decode_GiBps_output": round(gib(n * 4, dk), 2),
        "decode_roofline": roof(cbits / 8, n * 4, dk, "k_decode1d_var_lean<128>", basis="write")}
    del x32, enc, e, back
    torch.cuda.empty_cache()
    out["decode_mean_w8"] = leg_decode_mean(ctx)
    # the C5 host paths last: their PCIe-bound, mostly idle GPU phases lower the clocks a cold device leg right after
    # them would start from
    x32 = torch.empty(n, dtype=torch.float32, device=ctx.dev)
    codec.fill_normal(x32, 1e-3, seed=SEED, inject=True)
    xb = x32.to(torch.bfloat16)
    del x32
    h_in = xb.cpu().pin_memory()
    del xb
    for name, p in host_legs:
        h_out = torch.empty(codec.max_output_bytes((n,), p, torch.bfloat16) // 8 + 2, dtype=torch.int64,
                            pin_memory=True)
        henc = codec.HostEncoder(n, torch.bfloat16, p, chunks=16, device=ctx.dev)
        sw = settle_host(lambda: henc(h_in, h_out))
        hw = []
        h_ms, _ = timed(ctx, lambda: henc(h_in, h_out), 0, 5, walls=hw)
        h_ok = host_stream_check(henc, h_in, h_out, p)
        out[name].update({"host_path_ms": round(h_ms, 3), "host_path_GiBps_input": round(gib(n * 2, h_ms), 2),
                          "host_path_calls_ms": hw, "host_path_settle_calls_ms": sw[:12],
                          "host_path_stream_matches_oracle": h_ok,
                          "host_path_note": "pinned bf16 H2D + encode + D2H, 16 overlapped chunks (PCIe-bound)"})
        del h_out, henc
    del h_in
    return out


def exact_stream(e):
    """The Encoded `e` with its words cut to the stream's own length (the buffer a receiver holds): the variable-rate
    decoder sizes its stage by the buffer's average bits per block (gcow_kernels.hip launch_decode1d_var)."""
    from gcow_amd import codec
    return codec.Encoded(e.stream(), e.bits_dev, e.shape, e.params, e.index, e.index_stride)


def leg_decode_mean(ctx, W: int = 8, names=("rate16", "acc1e-6")):
    """The receive side of gcow_amd.ddp.compressed_allgather_hook on one GPU: W = 8 ranks' streams of 256 Mi fp32
    values (W different buckets of the bench distribution) decoded and averaged in one launch (codec.decode_mean), at
    rate 16 (the caller's default rate, hw/models/train_imagenet.py:155) and accuracy 1e-6 (the caller's default
    tolerance, :154). Roofline basis: the fp32 mean written; read + write adds the W compressed streams."""
    from gcow_amd import codec, ddp
    n = N_VALUES
    x = torch.empty(n, dtype=torch.float32, device=ctx.dev)
    mean = torch.empty_like(x)
    st = torch.cuda.current_stream(ctx.dev)
    res = {}
    for name, p, stride in (("rate16", codec.rate(16, 1), 0), ("acc1e-6", codec.accuracy(1e-6), 16)):
        if name not in names:
            continue
        # variable rate: encoded with the sharded hook's index (every 8 blocks); the all-gather hook's index (every 16
        # blocks) is every other entry of it -- the stream words do not depend on the spacing
        sstride = ddp.SHARDED_INDEX_STRIDE if stride else 0
        enc = codec.Encoder((n,), torch.float32, p, ctx.dev, index_stride=sstride)
        parts, idx, bits = [], [], 0
        for r in range(W):
            codec.fill_normal(x, 1e-3, seed=SEED + r, inject=True)
            e = enc(x, st)
            parts.append(e.stream().clone())
            if stride:
                idx.append(e.index.clone())
            bits += e.bits
        sw = max(t.numel() for t in parts)
        buf = torch.zeros(W * sw + 2, dtype=torch.int64, device=ctx.dev)
        for r, t in enumerate(parts):
            buf[r * sw:r * sw + t.numel()] = t
        ix8 = torch.cat(idx) if stride else None
        ni8 = idx[0].numel() if stride else 0
        # the all-gather hook's index (ddp.compressed_allgather_hook): every 8 blocks, packed into 16-block entries
        ixp = torch.cat([codec.pack_index16(t, n, p) for t in idx]) if stride else None
        nip = ixp.numel() // W if stride else 0
        del parts, idx, enc
        kp = codec.INDEX_PACKED16 if stride else 0
        forms = {"packed": lambda: codec.decode_mean(buf, sw, W, n, p, ixp, nip, kp, out=mean, stream=st)}
        ix16 = None
        if stride:  # the same decode with the plain 8-block index, and with a plain 16-block index (16-block chunks)
            ix16 = ix8.view(W, ni8)[:, ::stride // sstride].contiguous().view(-1)
            forms["8"] = lambda: codec.decode_mean(buf, sw, W, n, p, ix8, ni8, sstride, out=mean, stream=st)
            forms["16"] = lambda: codec.decode_mean(buf, sw, W, n, p, ix16, ix16.numel() // W, stride, out=mean,
                                                    stream=st)
        kt = {f: [] for f in forms}
        for _ in range(2):  # the forms interleaved (two rounds), so no form always meets the clock state of one slot
            for f, fn in forms.items():
                kt[f] += timed(ctx, fn, 3, 10, stream=st)[1]
        k = sum(kt["packed"]) / len(kt["packed"])
        k8 = round(sum(kt["8"]) / len(kt["8"]), 4) if stride else None
        k16 = round(sum(kt["16"]) / len(kt["16"]), 4) if stride else None
        del ix16
        kname = "k_decode_mean_fixed1d_np<64>" if stride == 0 else "k_decode_mean1d_var_lean<128, 64, 8, packed16>"
        # the sharded receive (ddp.compressed_sharded_hook): one rank's decode-mean of its 1/W shard from the W pieces
        # the all-to-all delivers (cut here from the same streams; the exchange itself is an N > 1 leg)
        pieces, pw, pidx, iw, lo, hi = shard0_pieces(buf, sw, W, n, p, ix8, ni8, sstride or 16)
        shard = mean[lo:hi]
        _, sper = timed(ctx, lambda: codec.decode_mean(pieces, pw, W, hi - lo, p, pidx, iw, sstride, out=shard,
                                                       stream=st), 3, 10, stream=st)
        ks = sum(sper) / len(sper)
        res[name] = {"streams": W, "values": n, "kernel_ms": round(k, 4), "bits_per_value": round(bits / W / n, 3),
                     "roofline": roof(bits / 8, n * 4, k, kname, basis="write"),
                     "index": "packed16 (8-block chunks)" if stride else None,
                     "kernel_ms_index_stride8": k8, "kernel_ms_index_stride16": k16,
                     "sharded_receive_kernel_ms": round(ks, 4), "sharded_receive_values": hi - lo,
                     "sharded_index_stride": sstride}
        del buf, ixp, ix8, pieces, pidx
        torch.cuda.empty_cache()
    del x, mean
    return res


def shard0_pieces(buf, sw, W, n, p, ix, ni, index_stride=16):
    """What rank 0 of a W-rank ddp.compressed_sharded_hook holds after its all-to-all, built locally from W streams
    laid out sw words apart (with their block indexes, ni entries apart, for variable rate): every stream cut at rank
    0's shard (gcow_amd.dist.shard_plan) -- fixed rate at b * maxbits, variable rate at the index, the index slice
    rebased to the piece's first word. -> (pieces, piece_words, index or None, index_words, lo, hi)."""
    from gcow_amd import codec
    from gcow_amd import dist as gdist
    bounds, per = gdist.shard_plan(n, W)
    lo, hi = bounds[0]
    nb = (n + 3) // 4
    b1 = min((hi + 3) // 4, nb)
    dev = buf.device
    if codec.is_fixed(p):
        pw = (b1 * p.maxbits + 63) // 64
        pieces = torch.zeros(W * pw + 2, dtype=torch.int64, device=dev)
        for s in range(W):
            pieces[s * pw:(s + 1) * pw] = buf[s * sw:s * sw + pw]
        return pieces, pw, None, 0, lo, hi
    nc = (b1 + index_stride - 1) // index_stride
    ends = ix.view(W, ni)[:, nc].tolist() if nc < ni else None
    pw = 1
    for s in range(W):
        end_bit = ends[s] if ends is not None else 64 * sw
        pw = max(pw, (end_bit + 63) // 64)
    pieces = torch.zeros(W * pw + 2, dtype=torch.int64, device=dev)
    pidx = torch.empty(W * nc, dtype=torch.int64, device=dev)
    for s in range(W):  # rank 0's shard starts at bit 0 of every stream
        pieces[s * pw:(s + 1) * pw] = buf[s * sw:s * sw + pw]
        pidx[s * nc:(s + 1) * nc] = ix[s * ni:s * ni + nc]
    return pieces, pw, pidx, nc, lo, hi


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def _cpu_quota():
    """CPUs' worth of time the cgroup grants this process (cpu.max), or None when unlimited / unknown."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(x: torch.Tensor, rate: float, dev) -> dict:
    """The reference's CPU path on this host's cores, best of N, encode only, host-resident:
      reference        sw/ zfp_compress compiled from /root/reference/sw/src (oracle/_ref, g++ -O3), one thread (sw/
                       has no threads), 2-D (its only layout: sw/src/zfp.c:12-24) on the WHOLE 256 Mi bucket viewed as
                       16384 x 16384, fixed rate `rate` (2-D minbits = maxbits = 16 rate);
      port_1t          the oracle restatement (gcc -O3 -march=native, built here) on the C2 config (1-D rate `rate`),
                       1 thread, the bucket's first 32 Mi values;
      port_mt          the same on the whole bucket with T = min(sched_getaffinity, cgroup CPU quota) threads (the
                       CPUs this process can use; `cores` = T) over block-aligned shards + a serial bit stitch;
      c3_*, c5_*       the restatement on the C3 field (512^3, 3-D rate 8 / accuracy 1e-3; the sw/ reference has no
                       3-D) and the C5 bucket (256 Mi bf16, accuracy 1e-6; no bf16 in sw/): T threads on the whole
                       input, 1 thread on a bounded slice.
    The headline is `reference`; without oracle/_ref it is port_1t and `reference_missing` says why. Every leg is also
    reported as flat `<leg>_GiBps` / `<leg>_cores` scalars (the driver's record keeps scalars, not nested objects);
    the long descriptions go to the top-level `cpu_baseline_legs`."""
    import ctypes as C

    import numpy as np

    from gcow_amd import codec
    from oracle import oracle as O
    a = x.detach().cpu().numpy()
    legs = {}

    def best(fn, reps):
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return min(ts)

    def leg(name, nbytes, dt, cores, sample, reps):
        legs[name] = {"value": round(nbytes / dt / 2 ** 30, 4), "unit": "GiB/s of uncompressed input", "cores": cores,
                      "seconds_best": round(dt, 4), "best_of": reps, "sample": sample}

    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    T = oracle_threads()
    R = O.ref()
    missing = None
    if R is not None:
        side = 16384
        a2 = a[: side * side].reshape(side, side)
        assert a2.flags.c_contiguous
        p = O.rate(rate, 2)
        out = np.zeros(O.max_words(a2.shape, p) + 4, np.uint64)
        dt = best(lambda: R.gcow_ref_compress_2d(a2.ctypes.data_as(C.POINTER(C.c_float)), side, side, *p.tuple(),
                                                   out.ctypes.data_as(C.POINTER(C.c_uint64)), out.nbytes), 3)
        leg("reference", a2.nbytes, dt, 1, "sw/ zfp_compress, whole bucket as 16384^2 fp32 (2-D), rate %g, 1 thread"
            % rate, 3)
        del out
    else:
        missing = "oracle/_ref/libgcow_ref.so absent (built from /root/reference/sw/src by oracle/Makefile)"
        print("bench.py: WARNING: " + missing, file=sys.stderr)
    L, flags = O.native_lib()
    p1 = O.rate(rate, 1)
    s1 = np.ascontiguousarray(a[: 32 << 20])
    leg("port_1t", s1.nbytes, best(lambda: O.compress(s1, p1, L=L), 5), 1,
        "oracle restatement (%s), 1-D rate %g, first 32 Mi values, 1 thread" % (flags, rate), 5)
    leg("port_mt", a.nbytes, best(lambda: O.compress(a, p1, threads=T, L=L), 5), T,
        "oracle restatement, 1-D rate %g, whole 256 Mi bucket, %d threads (= usable CPUs)" % (rate, T), 5)
    del s1
    # C3: the 512^3 field the GPU configs leg times
    f = codec.c3_field(dev).cpu().numpy()
    slab = np.ascontiguousarray(f[:64])
    for name, op in (("c3_rate8", O.rate(8, 3)), ("c3_acc1e-3", O.accuracy(1e-3))):
        leg(name + "_port_mt", f.nbytes, best(lambda: O.compress(f, op, threads=T, L=L), 3), T,
            "oracle restatement, 3-D %s, whole 512^3 C3 field, %d threads" % (name[3:], T), 3)
        leg(name + "_port_1t", slab.nbytes, best(lambda: O.compress(slab, op, L=L), 3), 1,
            "oracle restatement, 3-D %s, 512 x 512 x 64 of the C3 field, 1 thread" % name[3:], 3)
    del f, slab
    # C5: the bf16 bucket (exact widening, accuracy 1e-6)
    hb = x.to(torch.bfloat16).cpu().view(torch.int16).numpy().view(np.uint16)
    op = O.accuracy(1e-6)
    leg("c5_bf16_acc1e-6_port_mt", hb.nbytes, best(lambda: O.compress(hb, op, threads=T, L=L), 3), T,
        "oracle restatement, 1-D bf16 accuracy 1e-6, whole 256 Mi C5 bucket, %d threads" % T, 3)
    h1 = np.ascontiguousarray(hb[: 32 << 20])
    leg("c5_bf16_acc1e-6_port_1t", h1.nbytes, best(lambda: O.compress(h1, op, L=L), 3), 1,
        "oracle restatement, 1-D bf16 accuracy 1e-6, first 32 Mi values, 1 thread", 3)
    head = legs.get("reference") or legs["port_1t"]
    d = {"value": head["value"], "unit": "GiB/s", "cores": head["cores"],
         "kind": "reference" if "reference" in legs else "port", "sample": head["sample"],
         "cpu": _cpu_model()[:60], "host_cpus": os.cpu_count(), "affinity_cpus": aff,
         "cgroup_cpu_quota": _cpu_quota(), "usable_cpus": T}
    for k, v in legs.items():
        d[k + "_GiBps"] = v["value"]
        d[k + "_cores"] = v["cores"]
    if missing:
        d["reference_missing"] = missing
    return d, legs


# ------------------------------------------------------------------------------------------------------ main
def parity_failures(obj, path="") -> list:
    """Paths of every `*_matches_oracle` flag in the bench line that is False (None = not checked on this rank)."""
    bad = []
    if isinstance(obj, dict):
        for k, v in obj.items():
            if k.endswith("_matches_oracle") and v is False:
                bad.append(path + k)
            else:
                bad += parity_failures(v, path + k + ".")
    elif isinstance(obj, list):
        for i, v in enumerate(obj):
            bad += parity_failures(v, "%s%d." % (path, i))
    return bad


def finish(ctx: Ctx, line) -> int:
    """Print the JSON line (rank 0), tear down the group, and return the exit code: 3 when an oracle check in the
    line failed, so a stitch / shard-offset bug on the driver's N-rank run is an rc != 0, not a `false` in a tail."""
    bad = []
    if line is not None:
        print(json.dumps(line), flush=True)
        bad = parity_failures(line)
        if bad:
            print("bench.py: ORACLE CHECK FAILED: %s" % ", ".join(bad), file=sys.stderr, flush=True)
    if ctx.group:
        dist.destroy_process_group()
    return 3 if bad else 0


def stub_worker(ctx: Ctx):
    """Harness self-test (tests/test_bench_launcher.py): the same timing / max-over-ranks / JSON path with a trivial
    CPU step."""
    t = torch.ones(1 << 12)
    wall, _ = timed(ctx, lambda: t.sum(), ctx.args.warmup, ctx.args.steps)
    wall = ctx.max_over_ranks([wall])[0]
    me = [ctx.rank, ctx.local, ctx.world, os.environ.get("GCOW_BENCH_LAUNCHER", "torchrun"),
          os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT")]
    ranks = [None] * ctx.world
    if ctx.world > 1:
        dist.all_gather_object(ranks, me)
    else:
        ranks = [me]
    line = None
    if ctx.rank == 0:
        line = {"metric": METRIC, "value": round(gib(ctx.world * ctx.args.values * 4, wall), 3),
                "unit": "GiB/s", "n_gpus": ctx.world, "steps": ctx.args.steps, "warmup": ctx.args.warmup,
                "ms_per_step": round(wall, 5), "data": "stub", "ranks": ranks,
                "stub_check": {"stream_matches_oracle": not ctx.args.stub_mismatch}}
    return finish(ctx, line)


def worker(args):
    ctx = Ctx(args)
    if ctx.stub:
        return stub_worker(ctx)
    from gcow_amd import codec  # after the device is set: libgcow.so shares torch's HIP runtime

    n = args.values
    world, rank = ctx.world, ctx.rank
    x = torch.empty(n, dtype=torch.float32, device=ctx.dev)
    codec.fill_normal(x, 1e-3, seed=SEED + rank, inject=True)
    p = codec.rate(args.rate, 1)
    enc = codec.Encoder((n,), torch.float32, p, ctx.dev)
    stream = torch.cuda.current_stream(ctx.dev)
    step_ms, per = timed(ctx, lambda: enc(x, stream), args.warmup, args.steps, stream=stream)
    kern_ms = sum(per) / len(per)
    step_ms, kern_ms = ctx.max_over_ranks([step_ms, kern_ms])

    in_bytes = n * 4
    out_bytes = n * args.rate / 8
    value = world * gib(in_bytes, step_ms)
    workload = "c2_1d_fp32_fixed_rate%g_%dMi_per_gpu" % (args.rate, n // (1 << 20))
    kname = "k_encode_fixed1d_np"
    roofline = roof(in_bytes, out_bytes, kern_ms, kname)
    traffic, src = load_pmc_traffic(kname, workload)
    roofline["traffic"] = traffic
    # committed rocprofv3 --pmc pass (FETCH_SIZE + WRITE_SIZE per launch of this kernel and workload); not this run
    roofline["traffic_source"] = src
    if p.maxbits in (32, 64):
        # measured device-copy ceiling of the encoder's own access pattern (BASELINE.md:59): the same grid, loads and
        # stores without the coding (k_copy_pattern1d), same protocol, right after the headline
        cp_out = torch.empty(n // 4 * p.maxbits // 64 + 1, dtype=torch.int64, device=ctx.dev)
        _, cper = timed(ctx, lambda: codec.copy_pattern(x, cp_out, p.maxbits, stream), args.warmup, args.steps,
                        stream=stream)
        ck = ctx.max_over_ranks([sum(cper) / len(cper)])[0]
        # flat scalars (the driver's record keeps scalar fields of `roofline`, not nested objects)
        roofline["copy_ceiling_kernel"] = "k_copy_pattern1d"
        roofline["copy_ceiling_ms"] = round(ck, 5)
        roofline["copy_ceiling_frac"] = round(in_bytes / (ck / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)
        roofline["copy_ceiling_frac_read_write"] = round((in_bytes + out_bytes) / (ck / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)
        roofline["kernel_over_copy_ceiling"] = round(kern_ms / ck, 4)
        del cp_out
    extra = {"per_launch_ms": {"first": round(per[0], 4), "median": round(statistics.median(per), 4),
                               "min": round(min(per), 4), "max": round(max(per), 4)}}
    # the same kernel once the clock has settled under load (>= 0.25 s of back-to-back launches)
    t_end = time.perf_counter() + 0.25
    while time.perf_counter() < t_end:
        for _ in range(50):
            enc(x, stream)
        ctx.sync()
    s_ms, sper = timed(ctx, lambda: enc(x, stream), 0, 200, stream=stream)
    sk = sum(sper) / len(sper)
    s_ms, sk = ctx.max_over_ranks([s_ms, sk])
    extra["steady_state"] = {"ms_per_step": round(s_ms, 5), "GiBps": round(world * gib(in_bytes, s_ms), 2),
                             "kernel_ms": round(sk, 5), "frac": round(in_bytes / (sk / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                             "frac_read_write": round((in_bytes + out_bytes) / (sk / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)}

    if not args.no_extras:
        if world > 1 or ctx.group:
            extra["encode_allgather"] = leg_c4_exchange(ctx, lambda t: enc(t, stream), x, p, n, out_bytes)
            torch.cuda.empty_cache()
            extra["subgroups"] = leg_subgroups(ctx, p, n)
            torch.cuda.empty_cache()
            del x, enc
            torch.cuda.empty_cache()
            extra["strong"] = leg_strong(ctx, p, int(args.strong_gib * (1 << 30)) // 4)
            extra["c5_sharded"] = leg_c5_sharded(ctx, args.c5_values)
            torch.cuda.empty_cache()
            extra["hook_exchange"] = leg_hook_exchange(ctx, args.c5_values)
        else:
            # the device legs first: the host paths' PCIe-bound phases leave the GPU idle and its clocks low for
            # whatever cold leg follows them
            extra["configs"] = leg_configs(ctx)
            extra["host_e2e"] = leg_host_e2e(ctx, lambda t: enc(t, stream), x, p, n, in_bytes, out_bytes)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            if "x" not in locals():
                x = torch.empty(n, dtype=torch.float32, device=ctx.dev)
                codec.fill_normal(x, 1e-3, seed=SEED, inject=True)
            cpu, extra["cpu_baseline_legs"] = cpu_baseline(x, args.rate, ctx.dev)
        except Exception as ex:  # the GPU measurement stands on its own
            cpu = {"error": repr(ex)}
            print("bench.py: cpu_baseline failed: %r" % (ex,), file=sys.stderr)

    line = None
    if rank == 0:
        line = {
            "metric": METRIC,
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
                       "maxbits": p.maxbits, "bucket_bytes_total": world * in_bytes,
                       "launcher": os.environ.get("GCOW_BENCH_LAUNCHER", "torchrun" if world > 1 else "none")},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        line.update(extra)
    return finish(ctx, line)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args, argv))
    sys.exit(worker(args))


if __name__ == "__main__":
    main()
