#!/usr/bin/env python3
"""Short, fixed-count runs of the C3 / C5 encoders for rocprofv3 kernel traces and PMC passes (few dispatches, so
a counter pass stays within seconds).  usage: prof_cases.py [c2] [c3] [c5] [--reps N]"""
import argparse
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if "--lib" in sys.argv:  # A/B: profile another build of libgcow.so
    from gcow_amd import _ffi  # noqa: E402
    _ffi.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
from gcow_amd import codec  # noqa: E402


def c2(reps):
    n = 256 << 20
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    codec.fill_normal(x)
    enc = codec.Encoder((n,), torch.float32, codec.rate(16, 1))
    for _ in range(reps):
        enc(x)
    torch.cuda.synchronize()


def c3(reps):
    n = 512
    g = torch.arange(n, device="cuda", dtype=torch.float64) / n
    x = (torch.sin(6 * math.pi * g)[None, None, :] * torch.cos(4 * math.pi * g)[None, :, None] *
         torch.sin(2 * math.pi * g)[:, None, None]).float()
    noise = torch.empty(n ** 3, dtype=torch.float32, device="cuda")
    codec.fill_normal(noise, 1e-3, inject=False)
    x += noise.view(n, n, n)
    del noise
    for p, stride in ((codec.rate(8, 3), 0), (codec.accuracy(1e-3), 1)):
        enc = codec.Encoder(x.shape, torch.float32, p, index_stride=stride)
        out = torch.empty_like(x)
        for _ in range(reps):
            e = enc(x)
            codec.decode(e, out=out)
        torch.cuda.synchronize()


def c3dec(reps):
    """The C3 rate-8 and accuracy-1e-3 decoders alone (streams encoded once, untimed), on the bench's C3 field."""
    x = codec.c3_field("cuda")
    for p, stride in ((codec.rate(8, 3), 0), (codec.accuracy(1e-3), 1)):
        e = codec.Encoder(x.shape, torch.float32, p, index_stride=stride)(x)
        out = torch.empty_like(x)
        for _ in range(reps):
            codec.decode(e, out=out)
        torch.cuda.synchronize()


def c5(reps):
    n = 256 << 20
    xf = torch.empty(n, dtype=torch.float32, device="cuda")
    codec.fill_normal(xf)
    xb = xf.to(torch.bfloat16)
    del xf
    for tol in (1e-6, 1e-3):
        enc = codec.Encoder((n,), torch.bfloat16, codec.accuracy(tol))
        for _ in range(reps):
            enc(xb)
        torch.cuda.synchronize()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cases", nargs="*", default=["c3", "c5"])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--lib", default=None, help="libgcow.so to load instead of the in-tree build")
    a = ap.parse_args()
    for c in a.cases:
        globals()[c](a.reps)
    print("prof_cases done", flush=True)
