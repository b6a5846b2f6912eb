"""Interleaved A/B timing of the ablation kernels (one process, rounds interleaved; cdna guide 5.4 rule 24)."""
import ctypes as C
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from gcow_amd import codec  # noqa: E402

L = C.CDLL(os.path.join(HERE, "libablate.so"))
L.ablate_run.argtypes = [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_int, C.c_void_p]
n = 256 * 1024 * 1024
x = torch.empty(n, dtype=torch.float32, device="cuda")
codec.fill_normal(x)
out = torch.empty(n // 4, dtype=torch.int64, device="cuda")
st = torch.cuda.current_stream()
wgs = int(sys.argv[2]) if len(sys.argv) > 2 else 16
# each spec is MODE or MODE:WGS (per-mode grid, all timed in one process, rounds interleaved)
specs = [m for m in (sys.argv[1].split(",") if len(sys.argv) > 1 else "0,1,2,3,4".split(","))]
modes = specs
wgs_of = {m: (int(m.split(":")[1]) if ":" in m else wgs) for m in modes}
mode_of = {m: int(m.split(":")[0]) for m in modes}
res = {m: [] for m in modes}
for rnd in range(6):
    for m in modes:
        for _ in range(2):
            L.ablate_run(mode_of[m], x.data_ptr(), n // 4, out.data_ptr(), wgs_of[m], st.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10):
            L.ablate_run(mode_of[m], x.data_ptr(), n // 4, out.data_ptr(), wgs_of[m], st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        res[m].append(e0.elapsed_time(e1) / 10)
ref = torch.empty_like(out)
L.ablate_run(12, x.data_ptr(), n // 4, ref.data_ptr(), wgs, st.cuda_stream)
torch.cuda.synchronize()
same = {}
for m in modes:
    out.zero_()
    L.ablate_run(mode_of[m], x.data_ptr(), n // 4, out.data_ptr(), wgs_of[m], st.cuda_stream)
    torch.cuda.synchronize()
    same[m] = bool(torch.equal(out, ref))
for m in modes:
    v = sorted(res[m])
    print("mode %s wgs %d: median %.4f ms  min %.4f ms  (%.0f GB/s algorithmic)  equal-to-mode-12: %s" % (m, wgs_of[m], v[len(v) // 2], v[0], 1.5 * 2**30 / (v[len(v)//2] / 1e3) / 1e9, same[m]))
