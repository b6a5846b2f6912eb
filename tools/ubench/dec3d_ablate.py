"""Interleaved timing of the 3-D decoder ablation modes (tools/ubench/dec3d_ablate.hip) on the C3 field, rate 8.
usage: python tools/ubench/dec3d_ablate.py [MODES]   (build: see the .hip header; libdec3d.so next to this file)"""
import ctypes as C
import math
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from gcow_amd import codec  # noqa: E402

L = C.CDLL(os.path.join(HERE, "libdec3d.so"))
L.dec3_run.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
n = 512
g = torch.arange(n, device="cuda", dtype=torch.float64) / n
x = (torch.sin(6 * math.pi * g)[None, None, :] * torch.cos(4 * math.pi * g)[None, :, None] *
     torch.sin(2 * math.pi * g)[:, None, None]).float()
noise = torch.empty(n ** 3, dtype=torch.float32, device="cuda")
codec.fill_normal(noise, 1e-3, inject=False)
x += noise.view(n, n, n)
del noise
e = codec.encode(x, codec.rate(8, 3))
ref = codec.decode(e)
out = torch.empty_like(x)
sink = torch.empty(128 ** 3, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream()
modes = [int(m) for m in (sys.argv[1].split(",") if len(sys.argv) > 1 else "0,1,2,3,4".split(","))]
res = {m: [] for m in modes}
for rnd in range(6):
    for m in modes:
        for _ in range(3):
            L.dec3_run(m, e.words.data_ptr(), out.data_ptr(), sink.data_ptr(), st.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10):
            L.dec3_run(m, e.words.data_ptr(), out.data_ptr(), sink.data_ptr(), st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        res[m].append(e0.elapsed_time(e1) / 10)
for m in modes:
    out.zero_()
    L.dec3_run(m, e.words.data_ptr(), out.data_ptr(), sink.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    v = sorted(res[m])
    print("mode %d: median %.4f ms  min %.4f ms  equal-to-product-decode: %s" % (
        m, v[len(v) // 2], v[0], bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))), flush=True)
