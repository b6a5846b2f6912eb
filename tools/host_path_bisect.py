"""Bisect which earlier bench leg makes the C5 accuracy-1e-6 host path serialise its H2D and D2H copies (19.3 ms
instead of 11.7 ms). Modes:
  full      bench.leg_configs as the bench runs it
  no_dm     the same with leg_decode_mean skipped
  dm_only   leg_decode_mean, then the C5 host legs exactly as leg_configs runs them
Prints the host legs' per-call ms."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

mode = sys.argv[1]
args = bench.parse(["--no-cpu-baseline"])
ctx = bench.Ctx(args)
from gcow_amd import codec  # noqa: E402

if mode == "no_dm":
    bench.leg_decode_mean = lambda ctx: {}
if mode in ("full", "no_dm"):
    out = bench.leg_configs(ctx)
else:
    if mode in ("dm_only", "dm_ab"):
        bench.leg_decode_mean(ctx)
    elif mode == "dm_w2":
        bench.leg_decode_mean(ctx, W=2)
    elif mode in ("dm_rate16", "dm_acc1e-6"):
        bench.leg_decode_mean(ctx, names=(mode[3:],))
    elif mode == "alloc":
        ts = [torch.empty(1 << 29, dtype=torch.uint8, device=ctx.dev) for _ in range(10)]
        for t in ts:
            t.zero_()
        torch.cuda.synchronize()
        del ts
        torch.cuda.empty_cache()
    n = bench.N_VALUES
    x32 = torch.empty(n, dtype=torch.float32, device=ctx.dev)
    codec.fill_normal(x32, 1e-3, seed=bench.SEED, inject=True)
    xb = x32.to(torch.bfloat16)
    del x32
    h_in = xb.cpu().pin_memory()
    del xb
    out = {}
    if mode == "force":
        # give each new HostEncoder's H2D and D2H streams their first copies while the device is idle (so both pick the
        # first free copy engine), then time the encoder: does the pair stay serialised?
        import time
        p = codec.accuracy(1e-6)
        h_out = torch.empty(codec.max_output_bytes((n,), p, torch.bfloat16) // 8 + 2, dtype=torch.int64,
                            pin_memory=True)
        for ahead in (False, True, False, True):
            for forced in (False, True):
                henc = codec.HostEncoder(n, torch.bfloat16, p, chunks=16, device=ctx.dev, issue_ahead=ahead)  # the issue-ahead variant was measured and removed (round 6)
                if forced:
                    torch.cuda.synchronize()
                    with torch.cuda.stream(henc.s_d2h):
                        h_out[:1024].copy_(henc.words[:1024], non_blocking=True)
                    torch.cuda.synchronize()
                    with torch.cuda.stream(henc.s_h2d):
                        henc.bufs[0][:1024].copy_(h_in[:1024], non_blocking=True)
                    torch.cuda.synchronize()
                hw = []
                bench.timed(ctx, lambda: henc(h_in, h_out), 2, 5, walls=hw)
                print("issue_ahead=%s forced=%s" % (ahead, forced), hw, flush=True)
                del henc
        sys.exit(0)
    if mode == "dm_ab":
        import time
        p = codec.accuracy(1e-6)
        h_out = torch.empty(codec.max_output_bytes((n,), p, torch.bfloat16) // 8 + 2, dtype=torch.int64,
                            pin_memory=True)
        for ahead in (False, True, False, True):
            henc = codec.HostEncoder(n, torch.bfloat16, p, chunks=16, device=ctx.dev, issue_ahead=ahead)  # the issue-ahead variant was measured and removed (round 6)
            hw = []
            bench.timed(ctx, lambda: henc(h_in, h_out), 2, 5, walls=hw)
            print("issue_ahead=%s" % ahead, hw, flush=True)
            del henc
        dsrc = torch.empty(n, dtype=torch.bfloat16, device=ctx.dev)
        ddst = torch.empty(n // 4, dtype=torch.int64, device=ctx.dev)
        sa, sb = torch.cuda.Stream(ctx.dev), torch.cuda.Stream(ctx.dev)
        for both in (False, True, False, True):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with torch.cuda.stream(sa):
                dsrc.copy_(h_in, non_blocking=True)
            if both:
                with torch.cuda.stream(sb):
                    h_out[: n // 4].copy_(ddst, non_blocking=True)
            torch.cuda.synchronize()
            print("bare h2d%s %.3f ms" % (" + d2h" if both else "", (time.perf_counter() - t0) * 1e3), flush=True)
        sys.exit(0)
    for name, tol in (("c5_bf16_acc1e-6", 1e-6), ("c5_bf16_acc1e-3", 1e-3)):
        p = codec.accuracy(tol)
        h_out = torch.empty(codec.max_output_bytes((n,), p, torch.bfloat16) // 8 + 2, dtype=torch.int64,
                            pin_memory=True)
        henc = codec.HostEncoder(n, torch.bfloat16, p, chunks=16, device=ctx.dev)
        hw = []
        bench.timed(ctx, lambda: henc(h_in, h_out), 2, 5, walls=hw)
        out[name] = {"host_path_calls_ms": hw}
        del h_out, henc
for k in ("c5_bf16_acc1e-6", "c5_bf16_acc1e-3"):
    print(mode, k, out[k]["host_path_calls_ms"], flush=True)
