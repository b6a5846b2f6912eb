#!/usr/bin/env python3
"""C5 (256 Mi bf16 1-D, accuracy 1e-6 / 1e-3, block index every 16 blocks) encode and decode for one libgcow.so build
(--lib, default the in-tree build): the driver protocol (5 untimed + 20 timed launches) and steady state (after
0.25 s of back-to-back launches), plus a digest of the stream. Run it once per build, alternating builds, for an A/B
on one box (tools/c3_time.py is the C3 twin)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gcow_amd import _ffi  # noqa: E402

LIB = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1]) if "--lib" in sys.argv else None
if LIB:
    _ffi.LIB_PATH = LIB
from gcow_amd import codec  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools"))
from c5_ab import steady, timed  # noqa: E402

n = 256 << 20
x32 = torch.empty(n, dtype=torch.float32, device="cuda")
codec.fill_normal(x32, 1e-3, seed=0x67636F77, inject=True)
x = x32.to(torch.bfloat16)
del x32
out = torch.empty(n, dtype=torch.float32, device="cuda")
res = {"lib": os.path.basename(LIB) if LIB else "in-tree"}
for name, tol in (("acc1e-6", 1e-6), ("acc1e-3", 1e-3)):
    enc = codec.Encoder((n,), torch.bfloat16, codec.accuracy(tol), "cuda", index_stride=16)
    e = enc(x)
    cold_e, _ = timed(lambda: enc(x), 5, 20)
    st_e = steady(lambda: enc(x))
    if "--capacity" not in sys.argv:  # the stream in a buffer of its own length (what a receiver holds)
        e = codec.Encoded(e.stream(), e.bits_dev, e.shape, e.params, e.index, e.index_stride)
    cold_d, _ = timed(lambda: codec.decode(e, out=out), 5, 20)
    st_d = steady(lambda: codec.decode(e, out=out))
    torch.cuda.synchronize()
    w = e.stream().view(torch.int64)
    res[name] = {"enc_cold": round(cold_e, 4), "enc_steady": round(st_e, 4), "dec_cold": round(cold_d, 4),
                 "dec_steady": round(st_d, 4), "bits": int(e.bits),
                 "digest": int((w * torch.arange(1, w.numel() + 1, device=w.device)).sum().item())}
    del enc, e
    torch.cuda.empty_cache()
print(json.dumps(res), flush=True)
