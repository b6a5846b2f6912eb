#!/usr/bin/env python3
"""1-D variable-rate decode time across accuracies (256 Mi fp32, index every 16 blocks): where the lean decoder's
64-bit-per-block stage stops holding a workgroup's span, the general path takes over."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
if len(sys.argv) > 1:  # A/B: another build of libgcow.so
    from gcow_amd import _ffi  # noqa: E402
    _ffi.LIB_PATH = os.path.abspath(sys.argv[1])
from gcow_amd import codec  # noqa: E402

n = 256 << 20
x = torch.empty(n, dtype=torch.float32, device="cuda")
codec.fill_normal(x)
out = torch.empty_like(x)
for tol in (1e-3, 1e-5, 1e-6, 2e-7, 1e-7, 1e-8):
    e = codec.encode(x, codec.accuracy(tol), index_stride=16)
    for _ in range(3):
        codec.decode(e, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        codec.decode(e, out=out)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 10 * 1e3
    print({"lib": os.path.basename(sys.argv[1]) if len(sys.argv) > 1 else "libgcow.so", "tol": tol, "bits_per_block": round(e.bits / (n / 4), 1), "ms": round(ms, 3)}, flush=True)
