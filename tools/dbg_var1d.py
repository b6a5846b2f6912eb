#!/usr/bin/env python3
"""Debug helper: encode one of the variable-rate parity inputs with each 1-D variable-rate form and report where the
stream first differs from the oracle's (word index, tile)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gcow_amd import codec  # noqa: E402
from oracle import oracle as O  # noqa: E402


def subnormal_case(tol):
    rng = np.random.default_rng(int(-np.log10(tol) * 10))
    nb = 3000
    sub = rng.integers(-(2 ** 23) + 1, 2 ** 23, (nb, 4)).astype(np.float64) * 2.0 ** -149
    small = rng.integers(-(2 ** 8), 2 ** 8, (nb, 4)).astype(np.float64) * 2.0 ** -149
    norm = rng.standard_normal((nb, 4)) * 2.0 ** rng.integers(-126, -100, (nb, 1))
    kind = rng.integers(0, 4, nb)
    a = np.where(kind[:, None] == 0, sub, np.where(kind[:, None] == 1, small, np.where(kind[:, None] == 2, norm, 0.0)))
    return a.astype(np.float32).reshape(-1)[:-1], O.accuracy(tol)


a, op = subnormal_case(1e-40)
w_ref, bits_ref = O.compress(a, op)
ref = w_ref.view(np.uint64)
x = torch.from_numpy(a).cuda()
for name, env in (("pipe", {}), ("tile", {"GCOW_VAR1D_PIPE": "0"}), ("range", {"GCOW_VAR1D_FORM": "range"})):
    for k in ("GCOW_VAR1D_PIPE", "GCOW_VAR1D_FORM"):
        os.environ.pop(k, None)
    os.environ.update(env)
    e = codec.encode(x, codec.expert(*op.tuple()), index_stride=16)
    torch.cuda.synchronize()
    got = np.frombuffer(e.to_bytes(), dtype=np.uint64)
    d = np.nonzero(got[:ref.size] != ref)[0]
    print(name, "bits", e.bits, bits_ref, "ndiff", d.size, "first", d[:8].tolist(),
          "bit->tile", [(int(i) * 64) for i in d[:3]])
    if d.size:
        i = int(d[0])
        print("  got", hex(int(got[i])), "ref", hex(int(ref[i])))
