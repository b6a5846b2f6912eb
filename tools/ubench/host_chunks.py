#!/usr/bin/env python3
"""HostEncoder (pinned host bucket -> H2D -> encode -> D2H, overlapped on three streams) at several chunk counts:
C2 (256 Mi fp32, rate 16) and C5 (256 Mi bf16, accuracy 1e-6 / 1e-3); checks each result against one device encode.
usage: host_chunks.py [chunks ...]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gcow_amd import codec  # noqa: E402


def timeit(fn, reps=4):
    fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    return 1e3 * sorted(t)[len(t) // 2]


def main():
    ks = [int(a) for a in sys.argv[1:]] or [8, 16, 32, 64]
    n = 256 << 20
    xf = torch.empty(n, dtype=torch.float32, device="cuda")
    codec.fill_normal(xf)
    cases = [("c2_f32_rate16", xf, codec.rate(16, 1)), ("c5_bf16_acc1e-6", None, codec.accuracy(1e-6)),
             ("c5_bf16_acc1e-3", None, codec.accuracy(1e-3))]
    for name, x, p in cases:
        if x is None:
            x = xf.to(torch.bfloat16)
        e = codec.Encoder((n,), x.dtype, p)(x)
        bits = e.bits
        ref = e.words[:(bits + 63) // 64].cpu()
        h_in = x.cpu().pin_memory()
        h_out = torch.empty(codec.max_output_bytes((n,), p, x.dtype) // 8 + 2, dtype=torch.int64, pin_memory=True)
        nbytes = n * x.element_size()
        for k in ks:
            henc = codec.HostEncoder(n, x.dtype, p, chunks=k)
            assert henc(h_in, h_out) == bits and torch.equal(h_out[:ref.numel()], ref), (name, k)
            ms = timeit(lambda: henc(h_in, h_out))
            print({"case": name, "chunks": len(henc.bounds), "ms": round(ms, 3),
                   "GiBps_input": round(nbytes / (ms / 1e3) / 2 ** 30, 2)}, flush=True)
            del henc
        del h_in, h_out


if __name__ == "__main__":
    main()
