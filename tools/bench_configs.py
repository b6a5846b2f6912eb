#!/usr/bin/env python3
"""Secondary measurements for BASELINE configs 3 and 5 and the decoder (one JSON line per case, 1 GPU).

  c2_decode   256 Mi fp32 1-D rate 16: decode throughput
  c2_rate8    256 Mi fp32 1-D rate 8 encode
  c3          512^3 fp32 3-D: encode + decode, fixed rate 8 and accuracy 1e-3 (with block index)
  c5          256 Mi bf16 1-D variable rate (accuracy 1e-6 / 1e-3): device encode, and the host-resident
              path (pinned H2D of the bf16 bucket + encode + D2H of the stream), sequential and overlapped in
              chunks (codec.HostEncoder)
  var_f32     256 Mi fp32 1-D accuracy 1e-6 / 1e-3 encode
  var_decode  256 Mi fp32 1-D accuracy 1e-6 / 1e-3 decode (block index every 16 blocks)
Timing: HIP events on the launching stream, median of interleaved rounds.
"""
import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if "--lib" in sys.argv:  # A/B: time another build of libgcow.so (e.g. ab/variant.so)
    from gcow_amd import _ffi  # noqa: E402
    _ffi.LIB_PATH = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
from gcow_amd import codec  # noqa: E402


def timeit(fn, reps=20, rounds=5, settle_s=0.2):
    """Median per-call time; the first `settle_s` seconds of back-to-back calls are untimed (MI355X clocks dip for
    ~5-10 ms after a burst starts and recover over ~50 ms)."""
    st = torch.cuda.current_stream()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < settle_s:
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    ts.sort()
    return ts[len(ts) // 2]


def emit(**kw):
    print(json.dumps(kw), flush=True)


def c2_decode():
    n = 256 << 20
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    codec.fill_normal(x)
    p = codec.rate(16, 1)
    e = codec.encode(x, p)
    out = torch.empty_like(x)
    ms = timeit(lambda: codec.decode(e, out=out))
    emit(case="c2_decode_rate16", ms=round(ms, 4), GiBps_output=round(n * 4 / (ms / 1e3) / 2 ** 30, 1),
         GBps_traffic=round((n * 4 + n * 2) / (ms / 1e3) / 1e9, 1))
    p8 = codec.rate(8, 1)
    enc8 = codec.Encoder((n,), torch.float32, p8)
    ms = timeit(lambda: enc8(x))
    emit(case="c2_encode_rate8", ms=round(ms, 4), GiBps_input=round(n * 4 / (ms / 1e3) / 2 ** 30, 1))


def c3():
    x = codec.c3_field("cuda")  # the field bench.py times and tests/test_gpu_parity.py checks
    for name, p, stride in (("rate8", codec.rate(8, 3), 0), ("acc1e-3", codec.accuracy(1e-3), 1)):
        enc = codec.Encoder(x.shape, torch.float32, p, index_stride=stride)
        ms_e = timeit(lambda: enc(x), reps=5)
        e = enc(x)
        bits = e.bits
        out = torch.empty_like(x)
        ms_d = timeit(lambda: codec.decode(e, out=out), reps=5)
        err = float((out - x).abs().max())
        emit(case="c3_%s" % name, encode_ms=round(ms_e, 3), decode_ms=round(ms_d, 3),
             encode_GiBps=round(x.numel() * 4 / (ms_e / 1e3) / 2 ** 30, 1),
             decode_GiBps=round(x.numel() * 4 / (ms_d / 1e3) / 2 ** 30, 1),
             roundtrip_GiBps=round(x.numel() * 4 / ((ms_e + ms_d) / 1e3) / 2 ** 30, 1),
             bits_per_value=round(bits / x.numel(), 3), max_abs_err=err)


def var_f32():
    n = 256 << 20
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    codec.fill_normal(x)
    for tol in (1e-6, 1e-3):
        enc = codec.Encoder((n,), torch.float32, codec.accuracy(tol))
        ms = timeit(lambda: enc(x), reps=5)
        e = enc(x)
        emit(case="var_f32_acc%g" % tol, ms=round(ms, 3), GiBps_input=round(n * 4 / (ms / 1e3) / 2 ** 30, 1),
             bits_per_value=round(e.bits / n, 3))


def var_decode():
    """1-D variable-rate decode (the receiving side of the compressed all-gather DDP hook): 256 Mi fp32, accuracy
    1e-6 / 1e-3, block index every 16 blocks."""
    n = 256 << 20
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    codec.fill_normal(x)
    out = torch.empty_like(x)
    for tol in (1e-6, 1e-3):
        e = codec.encode(x, codec.accuracy(tol), index_stride=16)
        ms = timeit(lambda: codec.decode(e, out=out), reps=3)
        emit(case="var_decode_f32_acc%g" % tol, ms=round(ms, 3), GiBps_output=round(n * 4 / (ms / 1e3) / 2 ** 30, 1),
             bits_per_value=round(e.bits / n, 3))
    xb = x.to(torch.bfloat16)
    e = codec.encode(xb, codec.accuracy(1e-6), index_stride=16)
    ms = timeit(lambda: codec.decode(e, out=out), reps=3)
    emit(case="var_decode_bf16src_acc1e-06", ms=round(ms, 3), GiBps_output=round(n * 4 / (ms / 1e3) / 2 ** 30, 1),
         bits_per_value=round(e.bits / n, 3))


def decode_mean(W=8):
    """The receive side of the compressed all-gather hook on one GPU: W streams of 256 Mi fp32 values (W different
    buckets) decoded and averaged in one launch (codec.decode_mean), rate 16 and accuracy 1e-6."""
    n = 256 << 20
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    out = torch.empty_like(x)
    for name, p, stride in (("rate16", codec.rate(16, 1), 0), ("acc1e-6", codec.accuracy(1e-6), 16)):
        enc = codec.Encoder((n,), torch.float32, p, index_stride=stride)
        streams, idx, lens = [], [], []
        for r in range(W):
            codec.fill_normal(x, 1e-3, seed=0x67636F77 + r)
            e = enc(x)
            streams.append(e.stream().clone())
            idx.append(e.index.clone() if e.index is not None else None)
            lens.append(e.bits)
        sw = max(s.numel() for s in streams)
        buf = torch.zeros(W * sw + 2, dtype=torch.int64, device="cuda")
        for r, s in enumerate(streams):
            buf[r * sw:r * sw + s.numel()] = s
        ix = torch.cat(idx) if stride else None
        ni = idx[0].numel() if stride else 0
        ms = timeit(lambda: codec.decode_mean(buf, sw, W, n, p, ix, ni, stride, out=out), reps=3)
        cbytes = sum(lens) / 8
        emit(case="decode_mean_%s_W%d" % (name, W), ms=round(ms, 3),
             GBps_write=round(n * 4 / (ms / 1e3) / 1e9, 1),
             GBps_read_write=round((n * 4 + cbytes) / (ms / 1e3) / 1e9, 1),
             bits_per_value=round(sum(lens) / W / n, 3))
        # a bf16 bucket: written in the kernel (rounded to nearest even) vs an fp32 temporary + cast + copy
        ob = torch.empty(n, dtype=torch.bfloat16, device="cuda")
        ms_b = timeit(lambda: codec.decode_mean(buf, sw, W, n, p, ix, ni, stride, out=ob), reps=3)
        ms_c = timeit(lambda: ob.copy_(codec.decode_mean(buf, sw, W, n, p, ix, ni, stride, out=out).to(torch.bfloat16)),
                      reps=3)
        emit(case="decode_mean_%s_W%d_bf16_out" % (name, W), ms=round(ms_b, 3), ms_fp32_then_cast=round(ms_c, 3))
        del buf, streams, idx, enc, ob


def c5():
    n = 256 << 20
    xf = torch.empty(n, dtype=torch.float32, device="cuda")
    codec.fill_normal(xf)
    xb = xf.to(torch.bfloat16)
    del xf
    for tol in (1e-6, 1e-3):
        p = codec.accuracy(tol)
        enc = codec.Encoder((n,), torch.bfloat16, p)
        ms = timeit(lambda: enc(xb), reps=5)
        e = enc(xb)
        bits = e.bits
        nw = (bits + 63) // 64
        h_in = xb.cpu().pin_memory()
        h_out = torch.empty(nw, dtype=torch.int64, pin_memory=True)
        d_in = torch.empty_like(xb)

        def host_path():
            d_in.copy_(h_in, non_blocking=True)
            ee = enc(d_in)
            h_out.copy_(ee.words[:nw], non_blocking=True)

        ms_h = timeit(host_path, reps=3)
        # overlapped host path: chunked H2D / encode / D2H on three streams (codec.HostEncoder)
        h_out2 = torch.empty(codec.max_output_bytes((n,), p, torch.bfloat16) // 8 + 2, dtype=torch.int64,
                             pin_memory=True)
        henc = codec.HostEncoder(n, torch.bfloat16, p, chunks=16)
        assert henc(h_in, h_out2) == bits
        ms_p = timeit(lambda: henc(h_in, h_out2), reps=3)
        emit(case="c5_bf16_acc%g" % tol, encode_ms=round(ms, 3),
             encode_GiBps_input=round(n * 2 / (ms / 1e3) / 2 ** 30, 1), bits_per_value=round(bits / n, 3),
             host_path_ms=round(ms_h, 3), host_path_GiBps_input=round(n * 2 / (ms_h / 1e3) / 2 ** 30, 2),
             host_overlapped_ms=round(ms_p, 3), host_overlapped_GiBps_input=round(n * 2 / (ms_p / 1e3) / 2 ** 30, 2),
             host_overlapped_chunks=len(henc.bounds))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cases", nargs="*", default=["c2_decode", "c3", "var_f32", "c5"])
    ap.add_argument("--lib", default=None, help="libgcow.so to load instead of the in-tree build")
    a = ap.parse_args()
    if a.lib:
        print("lib", a.lib, flush=True)
    for c in a.cases:
        globals()[c]()
