#!/usr/bin/env python3
"""A short, fixed workload for rocprofv3 --pmc passes of the 1-D variable-rate decoders (one libgcow.so build, --lib):
the C5 bucket (256 Mi bf16, accuracy 1e-6 and 1e-3) encoded once and decoded 3 times into fp32 (k_decode1d_var_lean),
then decode_mean over W = 8 streams of 64 Mi fp32 values (accuracy 1e-6, index every 8 blocks) 3 times."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if "--lib" in sys.argv:
    from gcow_amd import _ffi  # noqa: E402
    _ffi.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
from gcow_amd import codec  # noqa: E402

n = 256 << 20
x32 = torch.empty(n, dtype=torch.float32, device="cuda")
codec.fill_normal(x32, 1e-3, seed=0x67636F77, inject=True)
xb = x32.to(torch.bfloat16)
out = torch.empty(n, dtype=torch.float32, device="cuda")
for tol in (1e-6, 1e-3):
    e = codec.encode(xb, codec.accuracy(tol), index_stride=16)
    e = codec.Encoded(e.stream(), e.bits_dev, e.shape, e.params, e.index, e.index_stride)
    for _ in range(3):
        codec.decode(e, out=out)
del xb, e
m, W = 64 << 20, 8
p = codec.accuracy(1e-6)
enc = codec.Encoder((m,), torch.float32, p, index_stride=8)
parts, idx = [], []
for r in range(W):
    codec.fill_normal(x32[:m], 1e-3, seed=0x67636F77 + r, inject=True)
    e = enc(x32[:m])
    parts.append(e.stream().clone())
    idx.append(e.index.clone())
sw = max(t.numel() for t in parts)
buf = torch.zeros(W * sw + 2, dtype=torch.int64, device="cuda")
for r, t in enumerate(parts):
    buf[r * sw:r * sw + t.numel()] = t
ix = torch.cat(idx)
for _ in range(3):
    codec.decode_mean(buf, sw, W, m, p, ix, idx[0].numel(), 8, out=out[:m])
torch.cuda.synchronize()
print("ok")
