#!/usr/bin/env python3
"""C2 (256 Mi fp32 1-D, fixed rate 16 and 8) encode: A/B of coder variants selected by an environment variable read
at each launch (default GCOW_FIXED1D_LEAN: 6 = lean-6, 7 = the variant under test), interleaved in one process over
several rounds in ABBA order with 2 s pauses (a variant run right after another's burst starts in a deeper DVFS dip).
Per variant and round: the driver protocol (5 untimed + 20 timed launches, mean of the HIP-event times, the bench's
`value`) and steady state (after 0.25 s of back-to-back launches, 100 launches). The variants' streams are compared
with each other (the GPU parity tests compare them with the oracle). One JSON line per case.
usage: c2_ab.py [--var NAME] [--vals 6,7] [--rounds 3]"""
import argparse
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--var", default="GCOW_FIXED1D_LEAN")
    ap.add_argument("--vals", default="6,7")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--rates", default="16,8")
    a = ap.parse_args()
    vals = a.vals.split(",")
    n = 256 << 20
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    codec.fill_normal(x, 1e-3, seed=0x67636F77, inject=True)
    for rate in [int(r) for r in a.rates.split(",")]:
        enc = codec.Encoder((n,), torch.float32, codec.rate(rate, 1), "cuda")
        res = {"case": "c2_rate%d" % rate, "var": a.var}
        streams = {}
        for rnd in range(a.rounds):
            for v in (vals if rnd % 2 == 0 else vals[::-1]):  # ABBA: the DVFS state after a burst favours neither
                os.environ[a.var] = v
                time.sleep(2.0)  # let the clock settle between variants
                cold, per = timed(lambda: enc(x), 5, 20)
                st = steady(lambda: enc(x))
                if rnd == 0:
                    streams[v] = enc(x).stream().clone()
                res.setdefault(v, []).append({"cold_ms": round(cold, 4), "first_ms": round(per[0], 4),
                                              "steady_ms": round(st, 4)})
        os.environ.pop(a.var, None)
        for v in vals:
            res[v + "_mean"] = {k: round(sum(r[k] for r in res[v]) / len(res[v]), 4) for k in ("cold_ms", "steady_ms")}
        res["streams_equal"] = all(torch.equal(streams[vals[0]], streams[v]) for v in vals[1:])
        print(json.dumps(res), flush=True)
        del enc, streams
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
