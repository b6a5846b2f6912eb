"""Loop-trip model of the 3-D rate-8 decoder's group phase on a C3-like field (64^3 of the C3 generator with N(0,1e-3)
noise, oracle-encoded): per wave of 64 consecutive blocks, the sum over planes of the slowest lane's trips for the
per-one-bit ctz loop and for 8-bit chunks (profiles/r03_c3_decode_group_table_negative.log). CPU only."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import oracle as O
n=64
g=np.arange(n)/512.0
x=(np.sin(6*np.pi*g)[None,None,:]*np.cos(4*np.pi*g)[None,:,None]*np.sin(2*np.pi*g)[:,None,None]).astype(np.float32)
rng=np.random.default_rng(1)
x=(x+rng.standard_normal(x.shape).astype(np.float32)*np.float32(1e-3)).astype(np.float32)
p=O.rate(8,3)
w,bits=O.compress(x,p)
print('bits',bits, 'blocks', bits//512)
words=np.concatenate([w,np.zeros(4,np.uint64)])
bitsarr=np.unpackbits(words.view(np.uint8),bitorder='little')
def dec_block(pos0):
    pos=pos0; maxbits=512
    if not bitsarr[pos]: return None
    pos+=9; bits=maxbits-9
    # prec for rate: maxprec 64 -> kmin 0; budget = bits
    n_=0; stats=[]
    for k in range(31,-1,-1):
        if not bits: break
        m=min(n_,bits); bits-=m; pos+=m
        ones=0; gbits=0; start=pos
        if n_<64 and bits:
            # serial group
            while n_<64 and bits:
                bits-=1; b=bitsarr[pos]; pos+=1
                if not b: break
                while n_<63 and bits:
                    bits-=1; b=bitsarr[pos]; pos+=1
                    if b: break
                    n_+=1
                ones+=1; n_+=1
            gbits=pos-start
        stats.append((k,m,ones,gbits,n_))
    return stats
blocks=[dec_block(512*b) for b in range(bits//512)]
# waves of 64 consecutive blocks
tot_serial=0; tot_chunks=0; tot_planes=0; lanes_serial=0
for wv in range(len(blocks)//64):
    B=blocks[64*wv:64*wv+64]
    for K in range(31,-1,-1):
        s=[0]; c=[0]; present=False
        for st in B:
            d={k:(m,o,gb,nn) for k,m,o,gb,nn in st}
            if K in d:
                present=True
                m,o,gb,nn=d[K]
                s.append(o+1); c.append((gb+7)//8); lanes_serial+=o+1
        if present:
            tot_planes+=1; tot_serial+=max(s); tot_chunks+=max(c)
nw=len(blocks)//64
print('per wave: planes',tot_planes/nw,'serial iters (max over lanes)',tot_serial/nw,'chunk iters',tot_chunks/nw,'avg lane serial iters',lanes_serial/len(blocks))
b=blocks[100]
print(b)
