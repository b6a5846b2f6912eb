import sys, os, numpy as np, torch
sys.path.insert(0, os.getcwd())
if len(sys.argv) > 1:
    from gcow_amd import _ffi; _ffi.LIB_PATH = os.path.abspath(sys.argv[1])
from gcow_amd import codec
from oracle import oracle as O
n = 409600
for mode in ("rate8", "rate16"):
    p = codec.rate(8 if mode == "rate8" else 16, 1)
    op = O.expert(*p.tuple())
    bad = 0
    for trial in range(3):
        xs = [torch.randn(n, device="cuda") * 1e-3 for _ in range(3)]
        streams = [torch.cuda.Stream() for _ in range(3)]
        outs = []
        for x, st in zip(xs, streams):
            with torch.cuda.stream(st):
                e = codec.encode(x, p)
                nw = e.nwords
                g = torch.zeros(nw + 2, dtype=torch.int64, device="cuda")
                g[:nw] = e.words[:nw]
                outs.append(codec.decode_mean(g, nw, 1, n, p))
        torch.cuda.synchronize()
        for x, o in zip(xs, outs):
            a = x.cpu().numpy()
            want = np.zeros(n, np.float32) + O.decompress(O.compress(a, op)[0], (n,), op)
            want = want / np.float32(1)
            if not np.array_equal(o.cpu().numpy().view(np.uint32), want.view(np.uint32)):
                d = np.nonzero(o.cpu().numpy().view(np.uint32) != want.view(np.uint32))[0]
                bad += 1
                print(mode, "mismatch", d.size, d[:5])
    print(mode, "bad", bad)
