#!/usr/bin/env python3
"""C3 (512^3 fp32, the bench's field) encode and decode, rate 8 and accuracy 1e-3, for one libgcow.so build
(--lib, default the in-tree build): the driver protocol (5 untimed + 20 timed launches) and steady state (after
0.25 s of back-to-back launches). Run it once per build, alternating builds, for an A/B on one box."""
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

x = codec.c3_field("cuda")
out = torch.empty_like(x)
res = {"lib": os.path.basename(LIB) if LIB else "in-tree"}
for name, p, stride in (("rate8", codec.rate(8, 3), 0), ("acc1e-3", codec.accuracy(1e-3), 1)):
    enc = codec.Encoder(x.shape, torch.float32, p, index_stride=stride)
    e = enc(x)
    cold_e, _ = timed(lambda: enc(x), 5, 20)
    st_e = steady(lambda: enc(x))
    cold_d, _ = timed(lambda: codec.decode(e, out=out), 5, 20)
    st_d = steady(lambda: codec.decode(e, out=out))
    torch.cuda.synchronize()
    res[name] = {"enc_cold": round(cold_e, 4), "enc_steady": round(st_e, 4), "dec_cold": round(cold_d, 4),
                 "dec_steady": round(st_d, 4), "bits": int(e.bits),
                 "stream_sum": int(e.stream().view(torch.int64).sum().item()),
                 "decode_sum": float(out.double().sum().item())}
print(json.dumps(res), flush=True)
