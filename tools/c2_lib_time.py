#!/usr/bin/env python3
"""C2 encode (256 Mi fp32 1-D, rate 16) with one libgcow.so build: the bench's driver protocol (5 untimed + 20
timed launches, mean HIP-event time) and steady state (after 0.25 s of back-to-back launches, 100 launches), plus
a stream digest so A/B builds can be compared. usage: c2_lib_time.py [--lib abv/libgcow_X.so] [--rate 16]
Run builds alternately in separate processes (tools/build_variant.sh makes them)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if "--lib" in sys.argv:
    from gcow_amd import _ffi  # noqa: E402
    _ffi.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
from gcow_amd import codec  # noqa: E402

rate = float(sys.argv[sys.argv.index("--rate") + 1]) if "--rate" in sys.argv else 16.0
n = 256 << 20
x = torch.empty(n, dtype=torch.float32, device="cuda")
codec.fill_normal(x, 1e-3, seed=0x67636F77, inject=True)
enc = codec.Encoder((n,), torch.float32, codec.rate(rate, 1))
st = torch.cuda.current_stream()


def timed(warm, steps):
    for _ in range(warm):
        enc(x, st)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    ev[0].record(st)
    for i in range(steps):
        enc(x, st)
        ev[i + 1].record(st)
    torch.cuda.synchronize()
    per = [ev[i].elapsed_time(ev[i + 1]) for i in range(steps)]
    return sum(per) / len(per), per


cold, per = timed(5, 20)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.25:
    for _ in range(50):
        enc(x, st)
    torch.cuda.synchronize()
steady, _ = timed(0, 100)
e = enc(x, st)
digest = int(e.words[: e.nwords].view(torch.int64).sum().item())
print(json.dumps({"lib": os.path.basename(sys.argv[sys.argv.index("--lib") + 1]) if "--lib" in sys.argv else "product",
                  "rate": rate, "cold_ms": round(cold, 4), "first_ms": round(per[0], 4),
                  "median_ms": round(sorted(per)[len(per) // 2], 4), "steady_ms": round(steady, 4),
                  "digest": digest}), flush=True)
