#!/usr/bin/env python3
"""Time the 1-D variable-rate encoder of one libgcow.so build on the C5 bucket (256 Mi bf16, accuracy 1e-6 and
1e-3): driver protocol (5 + 20 launches) and steady state. usage: var1d_time.py [--lib path/to/libgcow.so]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
if "--lib" in sys.argv:
    from gcow_amd import _ffi  # noqa: E402
    _ffi.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
from gcow_amd import codec  # noqa: E402

FORM = "single_pass" if "--sp" in sys.argv else "tile"  # --sp: the look-back form (else the default tile form)


def timed(fn, warm, steps):
    st = torch.cuda.current_stream()
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(steps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


n = 256 << 20
x32 = torch.empty(n, dtype=torch.float32, device="cuda")
codec.fill_normal(x32, 1e-3, seed=0x67636F77, inject=True)
xb = x32.to(torch.bfloat16)
del x32
out = {"lib": os.path.basename(sys.argv[sys.argv.index("--lib") + 1]) if "--lib" in sys.argv else "product"}
for tol in (1e-6, 1e-3):
    enc = codec.Encoder((n,), torch.bfloat16, codec.accuracy(tol), "cuda", index_stride=16)
    with codec.var1d_variant(FORM):
        cold = timed(lambda: enc(xb), 5, 20)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.25:
            for _ in range(20):
                enc(xb)
            torch.cuda.synchronize()
        d = {"cold_ms": round(cold, 4), "steady_ms": round(timed(lambda: enc(xb), 0, 100), 4)}
    if "--sp" in sys.argv:
        with codec.var1d_variant(FORM, stats=True):  # look-back polls / fallbacks / windows of one launch
            enc(xb)
            torch.cuda.synchronize()
        nt = (n // 4 + 1023) // 1024
        d["lookback_polls_fallbacks_windows_polling_max_first2048"] = enc.ws[2 * nt:2 * nt + 6].tolist()
    out["acc%g" % tol] = d
    del enc
print(json.dumps(out), flush=True)
