#!/usr/bin/env python3
"""C5 (256 Mi bf16 1-D, accuracy 1e-6 / 1e-3) and 1-D fp32 variable-rate encode: the 1-D variable-rate encoder forms
(FORMS below), interleaved in one process. Per form: the driver protocol
(5 untimed + 20 timed launches, mean of the HIP-event times) and steady state (after 0.25 s of back-to-back
launches, 100 launches). Streams of both forms are compared with each other (the GPU parity tests compare them with
the oracle). One JSON line per case."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gcow_amd import codec  # noqa: E402


def timed(fn, warm, steps):
    st = torch.cuda.current_stream()
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    ev[0].record(st)
    for i in range(steps):
        fn()
        ev[i + 1].record(st)
    torch.cuda.synchronize()
    per = [ev[i].elapsed_time(ev[i + 1]) for i in range(steps)]
    return sum(per) / len(per), per


def steady(fn):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.25:
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
    return timed(fn, 0, 100)[0]


FORMS = ("tile", "range", "single_pass")  # default (tile count + scan + placed tile coder), k_encode1d_var, look-back


def main():
    n = 256 << 20
    x32 = torch.empty(n, dtype=torch.float32, device="cuda")
    codec.fill_normal(x32, 1e-3, seed=0x67636F77, inject=True)
    xb = x32.to(torch.bfloat16)
    cases = [("c5_bf16_acc1e-6", xb, 1e-6), ("c5_bf16_acc1e-3", xb, 1e-3)]
    if "--f32" in sys.argv:
        cases += [("var_f32_acc1e-6", x32, 1e-6)]
    for name, x, tol in cases:
        p = codec.accuracy(tol)
        enc = codec.Encoder((n,), x.dtype, p, "cuda", index_stride=16)
        res = {"case": name}
        streams = {}
        for rnd in range(2):
            for form in FORMS:
                with codec.var1d_variant(form):
                    cold, per = timed(lambda: enc(x), 5, 20)
                    st = steady(lambda: enc(x))
                    e = enc(x)
                    bits = e.bits
                if form == "single_pass" and rnd == 0:  # look-back behaviour of one launch
                    with codec.var1d_variant(form, stats=True):
                        enc(x)
                        torch.cuda.synchronize()
                    nt = (n // 4 + 1023) // 1024
                    st_ = enc.ws[2 * nt:2 * nt + 6].tolist()
                    res["lookback"] = {"tiles": nt, "polls": st_[0], "fallbacks": st_[1], "windows": st_[2],
                                       "polling_tiles": st_[3], "max_polls": st_[4], "polls_first_2048": st_[5]}
                if rnd == 0:
                    streams[form] = (bits, e.stream().clone())
                res.setdefault(form, []).append({"cold_ms": round(cold, 4), "first_ms": round(per[0], 4),
                                                 "steady_ms": round(st, 4)})
        s0 = streams[FORMS[0]]
        res["bits_per_value"] = round(s0[0] / n, 3)
        res["streams_equal"] = all(s0[0] == streams[f][0] and torch.equal(s0[1], streams[f][1]) for f in FORMS[1:])
        print(json.dumps(res), flush=True)
        del enc, streams
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
