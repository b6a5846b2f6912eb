#!/usr/bin/env python3
"""1-D decoders for one libgcow.so build (--lib, default the in-tree build): the C2 decode (256 Mi fp32,
rate 16), decode_mean over W = 8 rate-16 streams and over W = 8 accuracy-1e-6 streams (the all-gather hook's
receive side), each as the driver protocol
(5 untimed + 20 timed launches) and steady state (after 0.25 s of back-to-back launches), plus a digest of the
outputs. Run it once per build, alternating builds, for an A/B on one box (tools/c5_ab_summary.py reads the logs)."""
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


def digest(t):
    w = t.view(torch.int32).to(torch.int64)
    return int((w * torch.arange(1, w.numel() + 1, device=w.device)).sum().item())


n = 256 << 20
W = 8
p = codec.rate(16, 1)
x = torch.empty(n, dtype=torch.float32, device="cuda")
out = torch.empty_like(x)
enc = codec.Encoder((n,), torch.float32, p)
res = {"lib": os.path.basename(LIB) if LIB else "in-tree"}
codec.fill_normal(x, 1e-3, seed=0x67636F77, inject=True)
e = enc(x)
cold, _ = timed(lambda: codec.decode(e, out=out), 5, 20)
st = steady(lambda: codec.decode(e, out=out))
torch.cuda.synchronize()
res["c2_decode"] = {"enc_cold": 0.0, "enc_steady": 0.0, "dec_cold": round(cold, 4), "dec_steady": round(st, 4),
                    "digest": digest(out)}
sw = e.stream().numel()
buf = torch.zeros(W * sw + 2, dtype=torch.int64, device="cuda")
for r in range(W):
    codec.fill_normal(x, 1e-3, seed=0x67636F77 + r, inject=True)
    buf[r * sw:(r + 1) * sw] = enc(x).stream()
cold, _ = timed(lambda: codec.decode_mean(buf, sw, W, n, p, out=out), 5, 20)
st = steady(lambda: codec.decode_mean(buf, sw, W, n, p, out=out))
torch.cuda.synchronize()
res["decode_mean_w8"] = {"enc_cold": 0.0, "enc_steady": 0.0, "dec_cold": round(cold, 4), "dec_steady": round(st, 4),
                         "digest": digest(out)}
# decode_mean over W = 8 variable-rate streams (accuracy 1e-6, block index every 16 blocks): the lean var decoder
pa = codec.accuracy(1e-6)
enc = codec.Encoder((n,), torch.float32, pa, index_stride=16)
streams, idx = [], []
for r in range(W):
    codec.fill_normal(x, 1e-3, seed=0x67636F77 + r, inject=True)
    e = enc(x)
    streams.append(e.stream().clone())
    idx.append(e.index.clone())
sw = max(t.numel() for t in streams)
del buf
buf = torch.zeros(W * sw + 2, dtype=torch.int64, device="cuda")
for r, t in enumerate(streams):
    buf[r * sw:r * sw + t.numel()] = t
ix, ni = torch.cat(idx), idx[0].numel()
cold, _ = timed(lambda: codec.decode_mean(buf, sw, W, n, pa, ix, ni, 16, out=out), 5, 20)
st = steady(lambda: codec.decode_mean(buf, sw, W, n, pa, ix, ni, 16, out=out))
torch.cuda.synchronize()
res["decode_mean_acc1e-6_w8"] = {"enc_cold": 0.0, "enc_steady": 0.0, "dec_cold": round(cold, 4),
                                 "dec_steady": round(st, 4), "digest": digest(out)}
print(json.dumps(res), flush=True)
