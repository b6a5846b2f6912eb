"""TEST INFRASTRUCTURE ONLY -- an oracle-backed stand-in for gcow_amd.dist.DeviceCodec on CPU tensors.

The multi-rank exchange code (gcow_amd.dist.encode_allgather / allgather_variable, both gcow_amd.ddp hooks) takes its
codec calls by injection; with this object the product protocol functions run unchanged over gloo process groups on
the CPU, while every byte of codec work is the oracle's (oracle/zfp_oracle.c, pinned by the reference goldens and
libzfp fixtures). `records` keeps what each call saw, so tests can check the exchange end to end.
"""
from __future__ import annotations

import numpy as np
import torch

from oracle import oracle as O


def _params(p) -> O.Params:
    return O.expert(*p.tuple())


def _np_values(x: torch.Tensor) -> np.ndarray:
    x = x.reshape(-1).contiguous()
    if x.dtype == torch.bfloat16:
        return x.view(torch.int16).numpy().view(np.uint16).copy()
    return x.float().numpy().copy() if x.dtype != torch.float32 else x.numpy().copy()


def _u64(t: torch.Tensor) -> np.ndarray:
    return t.contiguous().numpy().view(np.uint64)


class OracleCodec:
    def __init__(self):
        self.records = []

    def encode(self, x: torch.Tensor, params, index_stride: int = 0, slot=None):
        a = _np_values(x)
        p = _params(params)
        w, bits = O.compress(a, p)
        words = torch.from_numpy(np.concatenate([w, np.zeros(2, np.uint64)]).view(np.int64).copy())
        index = None
        if index_stride:
            lens = O.block_bits(a, p).astype(np.uint64)
            off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
            index = torch.from_numpy(off[::index_stride].view(np.int64).copy())
        self.records.append(("encode", a, bits))
        return words, torch.tensor([bits], dtype=torch.int64), index

    def stitch_shards(self, dst: torch.Tensor, src: torch.Tensor, shard_words: int, lens: torch.Tensor, nshards: int):
        d = np.zeros(dst.numel() + 1, np.uint64)
        s = _u64(src)
        off = 0
        for r in range(nshards):
            b = int(lens[r])
            if b:
                seg = np.concatenate([s[r * shard_words:(r + 1) * shard_words], np.zeros(1, np.uint64)])
                O.lib().orc_stitch(O._p(d, O.C.c_uint64), off, O._p(seg, O.C.c_uint64), b)
            off += b
        dst.copy_(torch.from_numpy(d[: dst.numel()].view(np.int64).copy()))
        self.records.append(("stitch", [int(v) for v in lens[:nshards]]))
        return dst

    def decode(self, words: torch.Tensor, n: int, params, index=None, index_stride: int = 0, out=None):
        v = O.decompress(_u64(words), (n,), _params(params))
        t = torch.from_numpy(v)
        if out is not None:
            out.copy_(t)
            return out
        return t

    def pack_index16(self, index8: torch.Tensor, n: int, params) -> torch.Tensor:
        """include/gcow.h GCOW_INDEX_PACKED16, restated in numpy: entry c = idx8[2c] | (idx8[2c+1] - idx8[2c]) << 48."""
        i8 = index8.numpy().view(np.uint64)[: (n + 31) // 32]
        a = i8[0::2]
        b = np.zeros_like(a)
        b[: len(i8[1::2])] = i8[1::2] - a[: len(i8[1::2])]
        assert b.max(initial=0) < 1 << 16 and a.max(initial=0) < 1 << 48
        self.records.append(("pack_index16", n))
        return torch.from_numpy((a | (b << np.uint64(48))).view(np.int64).copy())

    def decode_mean(self, streams: torch.Tensor, stream_words: int, nstreams: int, n: int, params, index=None,
                    index_words: int = 0, index_stride: int = 0, out=None):
        if index is not None and index_stride == 0x1010:  # packed16: unpack to the 8-block chunk starts
            pk = index.numpy().view(np.uint64).reshape(nstreams, index_words)
            lo = pk & np.uint64((1 << 48) - 1)
            un = np.stack([lo, lo + (pk >> np.uint64(48))], axis=2).reshape(nstreams, 2 * index_words)
            index, index_words, index_stride = torch.from_numpy(un.view(np.int64).copy().reshape(-1)), \
                2 * index_words, 8
        s = _u64(streams)
        p = _params(params)
        acc = np.zeros(n, np.float32)
        for r in range(nstreams):
            seg = s[r * stream_words:(r + 1) * stream_words]
            if index is None:
                dec = O.decompress(seg, (n,), p)  # fixed rate: block b at b * maxbits of the segment
            else:  # decoded chunk by chunk from the gathered index (its first block need not start at bit 0)
                dec = np.zeros(n, np.float32)
                ix = index.numpy()[r * index_words:(r + 1) * index_words].view(np.uint64)
                w = np.concatenate([seg, np.zeros(2, np.uint64)])
                for k, off in enumerate(ix[: (n + 4 * index_stride - 1) // (4 * index_stride)]):
                    m = min(4 * index_stride, n - 4 * index_stride * k)
                    chunk = np.zeros(m, np.float32)
                    dims, nn = O._shape((m,))
                    O.lib().orc_decompress_at(O._p(chunk, O.C.c_float), dims, nn, None, O.C.byref(p),
                                              O._p(w, O.C.c_uint64), len(w), int(off))
                    lo = 4 * index_stride * k
                    dec[lo:lo + m] = chunk
                if int(ix[0]) == 0:  # a whole stream: the index agrees with its sequential decode
                    assert np.array_equal(O.decompress(seg, (n,), p).view(np.uint32), dec.view(np.uint32)), r
            acc = acc + dec
        acc = acc / np.float32(nstreams)
        self.records.append(("decode_mean", nstreams, acc.copy()))
        t = torch.from_numpy(acc)
        if out is not None:
            out.copy_(t)
            return out
        return t
