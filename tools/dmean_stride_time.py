#!/usr/bin/env python3
"""decode_mean over W = 8 variable-rate streams (256 Mi fp32 values each, accuracy 1e-6) with the block index every
8 or every 16 blocks (--stride), and the sharded-receive size (1/8 of the values): the driver protocol (5 + 20) and
steady state, plus an output digest. One JSON line."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if "--lib" in sys.argv:
    from gcow_amd import _ffi  # noqa: E402
    _ffi.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
from gcow_amd import codec  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools"))
from c5_ab import steady, timed  # noqa: E402

sarg = sys.argv[sys.argv.index("--stride") + 1] if "--stride" in sys.argv else "16"
packed = sarg == "packed"  # the all-gather hook's form: 8-block index packed to the 16-block size
stride = 8 if packed else int(sarg)
same = "--same" in sys.argv  # every rank's stream the same (ablation builds that stage one stream for all)
W = 8
res = {"stride": sarg, "lib": os.path.basename(sys.argv[sys.argv.index("--lib") + 1]) if "--lib" in sys.argv else "in-tree"}
for n in (256 << 20, 32 << 20):
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    out = torch.empty_like(x)
    pa = codec.accuracy(1e-6)
    enc = codec.Encoder((n,), torch.float32, pa, index_stride=stride)
    streams, idx = [], []
    for r in range(W):
        codec.fill_normal(x, 1e-3, seed=0x67636F77 + (0 if same else r), inject=True)
        e = enc(x)
        streams.append(e.stream().clone())
        idx.append(codec.pack_index16(e.index, n, pa) if packed else e.index.clone())
    sw = max(t.numel() for t in streams)
    sw += sw & 1 if same else 0  # --same: every stream at the same 16-byte phase of the buffer
    buf = torch.zeros(W * sw + 2, dtype=torch.int64, device="cuda")
    for r, t in enumerate(streams):
        buf[r * sw:r * sw + t.numel()] = t
    ix, ni = torch.cat(idx), idx[0].numel()
    ist = codec.INDEX_PACKED16 if packed else stride
    cold, _ = timed(lambda: codec.decode_mean(buf, sw, W, n, pa, ix, ni, ist, out=out), 5, 20)
    st = steady(lambda: codec.decode_mean(buf, sw, W, n, pa, ix, ni, ist, out=out))
    torch.cuda.synchronize()
    w = out.view(torch.int32).to(torch.int64)
    res["n%dMi" % (n >> 20)] = {"cold_ms": round(cold, 4), "steady_ms": round(st, 4),
                                "digest": int((w * torch.arange(1, w.numel() + 1, device=w.device)).sum().item())}
    del buf, streams, idx, enc, x, out
    torch.cuda.empty_cache()
print(json.dumps(res), flush=True)
