import os, sys, json, numpy as np, torch
sys.path.insert(0, os.getcwd())
from gcow_amd import codec as gc
fx = json.load(open('tests/golden/libzfp_fixtures.json'))
z = np.load('tests/golden/libzfp_fixtures.npz')
for name in ('1d_n64__rate_8.0', '1d_n64__rate_16.0', '1d_n1000__rate_8.0', '1d_n1000__rate_16.0'):
    c = [c for c in fx['cases'] if c['name'] == name][0]
    words = z[name + '__stream']; dref = z[name + '__decoded']
    n = dref.size
    t = torch.from_numpy(np.concatenate([words, np.zeros(2, np.uint64)]).view(np.int64)).cuda()
    d = gc.decode(t, (n,), gc.expert(*c['params'])).cpu().numpy()
    bad = np.nonzero(d.view(np.uint32) != dref.view(np.uint32))[0]
    print(name, 'mismatches', len(bad), 'first blocks', sorted(set((bad // 4).tolist()))[:10])
    for i in sorted(set((bad // 4).tolist()))[:3]:
        print('  block', i, d[4*i:4*i+4], dref[4*i:4*i+4])
from oracle import oracle as O
for r in (8, 16):
    for n in (262147, 262144, 4097):
        a = O.gen_normal(n, 1e-3, 0x1234 + n, True)
        op = O.rate(r, 1)
        w_ref, bits = O.compress(a, op)
        ref = O.decompress(w_ref, a.shape, op)
        p = gc.expert(*op.tuple())
        e = gc.encode(torch.from_numpy(a).cuda(), p)
        d = gc.decode(e).cpu().numpy()
        bad = np.nonzero(d.view(np.uint32) != ref.view(np.uint32))[0]
        print("r", r, "n", n, "mismatch", len(bad), bad[:8], d[bad[:4]] if len(bad) else "", ref[bad[:4]] if len(bad) else "")
