#!/usr/bin/env python3
"""How many k_decode1d_var_lean workgroups (128 index chunks of 16 blocks) have a stream span larger than the LDS
stage (CAPB bits per block on average) and take the general path: the bench's 1-D buckets at accuracy 1e-6 / 1e-3."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gcow_amd import codec  # noqa: E402

n = 256 << 20
x = torch.empty(n, dtype=torch.float32, device="cuda")
codec.fill_normal(x)
for name, src in (("f32", x), ("bf16", x.to(torch.bfloat16))):
    for tol in (1e-6, 1e-3):
        e = codec.encode(src, codec.accuracy(tol), index_stride=16)
        idx = e.index.cpu().long()
        nch = idx.numel()
        lanes = 128
        ng = nch // lanes
        starts = (idx[0:ng * lanes:lanes] >> 6) & ~1
        ends = torch.cat([idx[lanes::lanes][: ng - 1], torch.tensor([e.bits])])
        ends = (ends + 63) >> 6
        span = ends - starts  # 64-bit words
        for capb in (56, 64, 72, 80):
            cap = lanes * 16 * capb // 64
            over = int((span > cap).sum())
            print({"src": name, "tol": tol, "bits_per_block": round(e.bits / (n / 4), 2), "capb": capb,
                   "workgroups": ng, "over_capacity": over, "frac": round(over / ng, 5)}, flush=True)
