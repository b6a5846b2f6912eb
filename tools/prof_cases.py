#!/usr/bin/env python3
"""Short, fixed-count runs of the C3 / C5 encoders for rocprofv3 kernel traces and PMC passes (few dispatches, so
a counter pass stays within seconds).  usage: prof_cases.py [c2] [c3] [c5] [--reps N]"""
import argparse
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
    """The C3 rate-8 and accuracy-1e-3 encode + decode pairs on the bench's C3 field (codec.c3_field)."""
    x = codec.c3_field("cuda")
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


def vdec(reps):
    """1-D variable-rate decode (block index every 16 blocks) of the fp32 and the bf16 C5 bucket at accuracy 1e-6, and
    of the bf16 one at 1e-3, each stream in a buffer of its own length (the stage is sized by its average)."""
    n = 256 << 20
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    codec.fill_normal(x)
    out = torch.empty_like(x)
    for src, tol in ((x, 1e-6), (x.to(torch.bfloat16), 1e-6), (x.to(torch.bfloat16), 1e-3)):
        e = codec.encode(src, codec.accuracy(tol), index_stride=16)
        e = codec.Encoded(e.stream(), e.bits_dev, e.shape, e.params, e.index, e.index_stride)
        for _ in range(reps):
            codec.decode(e, out=out)
        torch.cuda.synchronize()


def dmean(reps, W=8):
    """decode_mean over W streams of 256 Mi values: rate 16, then accuracy 1e-6 with the block index every 16 and
    every 8 blocks (the sharded hook's spacing), and every 8 blocks sent packed into 16-block entries (the all-gather
    hook's form, codec.pack_index16)."""
    n = 256 << 20
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    out = torch.empty_like(x)
    for p, stride in ((codec.rate(16, 1), 0), (codec.accuracy(1e-6), 16), (codec.accuracy(1e-6), 8),
                      (codec.accuracy(1e-6), codec.INDEX_PACKED16)):
        enc = codec.Encoder((n,), torch.float32, p, index_stride=8 if stride == codec.INDEX_PACKED16 else stride)
        ss, ix = [], []
        for r in range(W):
            codec.fill_normal(x, 1e-3, seed=0x67636F77 + r)
            e = enc(x)
            ss.append(e.stream().clone())
            if stride == codec.INDEX_PACKED16:
                ix.append(codec.pack_index16(e.index, n, p).clone())
            else:
                ix.append(e.index.clone() if stride else None)
        sw = max(s.numel() for s in ss)
        buf = torch.zeros(W * sw + 2, dtype=torch.int64, device="cuda")
        for r, s in enumerate(ss):
            buf[r * sw:r * sw + s.numel()] = s
        idx = torch.cat(ix) if stride else None
        ni = ix[0].numel() if stride else 0
        for _ in range(reps):
            codec.decode_mean(buf, sw, W, n, p, idx, ni, stride, out=out)
        torch.cuda.synchronize()
        del buf, ss, ix, enc


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cases", nargs="*", default=["c3", "c5"])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--lib", default=None, help="libgcow.so to load instead of the in-tree build")
    ap.add_argument("--var1d-form", default="tile", choices=sorted(codec.VAR1D_FORMS),
                    help="1-D variable-rate encoder form (test-only variant setter)")
    a = ap.parse_args()
    with codec.var1d_variant(a.var1d_form):
        for c in a.cases:
            globals()[c](a.reps)
    print("prof_cases done", flush=True)
