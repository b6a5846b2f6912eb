"""Cold-start launch pattern (the driver's bench: 5 warmups, sync, 20 timed launches) for several kernels, each after
an idle gap: per-launch HIP-event durations. Shows whether the clock dip that follows a burst of launches slows a
kernel (compute-bound at the lowered clock) or not (memory-bound).
usage: python tools/ubench/cold.py MODE[,MODE...]   (MODE: 'enc' = product encoder, or an ablate.hip mode number)"""
import ctypes as C
import os
import statistics
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from gcow_amd import codec  # noqa: E402

L = C.CDLL(os.path.join(HERE, "libablate.so"))
L.ablate_run.argtypes = [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_int, C.c_void_p]
L.ablate_stamp_copy.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
n = 256 * 1024 * 1024
x = torch.empty(n, dtype=torch.float32, device="cuda")
codec.fill_normal(x)
out = torch.empty(n // 4, dtype=torch.int64, device="cuda")
st = torch.cuda.current_stream()
enc = codec.Encoder((n,), torch.float32, codec.rate(16, 1))
wgs = 16


slot = [0]


def run(m):
    if m == "stamp":
        L.ablate_run(90, x.data_ptr(), n // 4, out.data_ptr(), slot[0] % 32, st.cuda_stream)
        slot[0] += 1
    elif m == "enc":
        enc(x, st)
    else:
        L.ablate_run(int(m), x.data_ptr(), n // 4, out.data_ptr(), wgs, st.cuda_stream)


modes = sys.argv[1].split(",") if len(sys.argv) > 1 else ["enc", "9", "55"]
for rnd in range(3):
    for m in modes:
        torch.cuda.synchronize()
        time.sleep(0.5)
        for _ in range(5):
            run(m)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
        ev[0].record(st)
        for i in range(20):
            run(m)
            ev[i + 1].record(st)
        torch.cuda.synchronize()
        d = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(20)]
        if m == "stamp":  # in-kernel clock of the 20 timed launches (slots 5..24 of this burst)
            import numpy as np
            clk = []
            for i in range(5, 25):
                a = np.zeros(4 * 32768, np.uint64)
                L.ablate_stamp_copy(a.ctypes.data, (slot[0] - 25 + i) % 32, 32768)
                a = a.reshape(-1, 4).astype(np.float64)
                c = (a[:, 1] - a[:, 0]) / np.maximum(a[:, 3] - a[:, 2], 1) * 100.0
                clk.append(float(np.median(c)))
            print("   in-kernel clock MHz per launch:", " ".join("%.0f" % c for c in clk), flush=True)
        # then steady: 0.3 s of launches, 50 timed
        t_end = time.perf_counter() + 0.3
        while time.perf_counter() < t_end:
            for _ in range(20):
                run(m)
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(50):
            run(m)
        e1.record(st)
        torch.cuda.synchronize()
        print("round %d mode %-4s cold mean %.1f us median %.1f max %.1f | steady %.1f us | %s" % (
            rnd, m, sum(d) / 20, statistics.median(d), max(d), e0.elapsed_time(e1) * 1e3 / 50,
            " ".join("%.0f" % v for v in d)), flush=True)
