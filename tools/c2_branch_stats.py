#!/usr/bin/env python3
"""Branch statistics of the C2 lean coder (k_encode_fixed1d_np) on the bench distribution, from the oracle's N(0, 1e-3)
generator (CPU, numpy): the distribution of sh = 31 - M0 (empty planes above the block maximum), of the group-phase
length jg (window nibbles before 3 coefficients are significant), and how many extra wave-uniform pair steps
(pairs 2+, 12 VALU each) a wave of 64 consecutive blocks runs. usage: python tools/c2_branch_stats.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O
n = 4*64*4096*4
a = O.gen_normal(n, 1e-3, 0x67636F77, True).reshape(-1,4)
m = np.abs(a).max(axis=1)
mb = m.view(np.uint32)
E = (mb >> 23).astype(np.int64)
s = ((283 - E) << 23).astype(np.uint32).view(np.float32)
with np.errstate(all='ignore'):
    q = (a * s[:,None])
q = np.where(np.isfinite(q) & (np.abs(q) < 2**31), q, -2.0**31).astype(np.int64).astype(np.int32).astype(np.int64)
# lift int32 wrap
def w32(x): return ((x + 2**31) % 2**32) - 2**31
x,y,z,w = q[:,0],q[:,1],q[:,2],q[:,3]
x = w32(x+w) >> 1; w = w32(w-x)
z = w32(z+y) >> 1; y = w32(y-z)
x = w32(x+z) >> 1; z = w32(z-x)
w = w32(w+y) >> 1; y = w32(y-w)
w = w32(w + (y>>1)); y = w32(y - (w>>1))
NB = 0xaaaaaaaa
u = [((v + NB) % 2**32) ^ NB for v in (x,y,z,w)]
u = [np.asarray(v, dtype=np.uint64) for v in u]
def clz(v):
    v = v.astype(np.uint64); r = np.full(v.shape, 32)
    nz = v != 0
    r[nz] = 31 - np.floor(np.log2(v[nz].astype(np.float64))).astype(np.int64)
    return r
sh = clz(u[0]|u[1]|u[2]|u[3]|1)
o23 = u[2]|u[3]
jg = np.minimum(clz(o23), 31) - sh
tiny = (mb >= 1) & (mb < (29 << 23))
valid = ~tiny & (m > 0)
print("blocks", len(sh), "sh dist", np.bincount(sh[valid])[:6]/valid.sum())
print("jg dist", np.bincount(np.clip(jg[valid],0,20))[:12]/valid.sum())
# waves: 64 consecutive blocks per wave-step (lane l: block b0 + 256k + l -> a wave holds 64 consecutive blocks)
W = jg.reshape(-1,64)
mx = W.max(axis=1)
# loop: pair1 if any jg>=2; pairs jj=4.. while any(jj <= jg)
pairs_extra = np.maximum(0, (mx - 4)//2 + 1)
print("P(any jg>=2)", (mx>=2).mean(), "mean extra pair iterations (pairs 2+)", pairs_extra.mean(), np.bincount(pairs_extra)[:8]/len(mx))
