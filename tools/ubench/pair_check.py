import numpy as np, sys, os, torch
sys.path.insert(0, os.getcwd())
if len(sys.argv) > 1:
    from gcow_amd import _ffi; _ffi.LIB_PATH = os.path.abspath(sys.argv[1])
from gcow_amd import codec
from oracle import oracle as O
torch.manual_seed(0)
layers = torch.nn.Sequential(*[torch.nn.Linear(640, 640, bias=False) for _ in range(3)]).cuda()
x = torch.randn(32, 640, device="cuda")
layers(x).square().mean().backward()
op = O.rate(16, 1)
for l in layers:
    g = l.weight.grad.reshape(-1).contiguous()
    e = codec.encode(g, codec.rate(16, 1))
    d = codec.decode(e).cpu().numpy()
    gh = g.cpu().numpy()
    w, bits = O.compress(gh, op)
    assert e.to_bytes() == w.tobytes()
    ref = O.decompress(w, gh.shape, op)
    bad = np.nonzero(d.view(np.uint32) != ref.view(np.uint32))[0]
    print("mismatches", bad.size, bad[:8])
    for i in bad[:3]:
        b = i // 4
        print(" block", b, hex(int(w[b])), d[4*b:4*b+4], ref[4*b:4*b+4])
