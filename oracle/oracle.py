"""TEST INFRASTRUCTURE ONLY -- ctypes loader for the CPU oracle (oracle/liboracle.so) and, when built,
the reference sw/ encoder compiled in place (oracle/_ref/libgcow_ref.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module; the product
package gcow_amd/ never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
F32, BF16 = 3, 5


class Params(C.Structure):
    _fields_ = [("minbits", C.c_uint), ("maxbits", C.c_uint), ("maxprec", C.c_uint), ("minexp", C.c_int)]

    def tuple(self):
        return (self.minbits, self.maxbits, self.maxprec, self.minexp)

    def __repr__(self):
        return "Params(%d, %d, %d, %d)" % self.tuple()


_lib = None
_ref = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        _lib = _bind(C.CDLL(path))
    return _lib


_native = None


def native_lib():
    """The restatement compiled for the host it runs on (gcc -O3 -march=native, into a temp dir): the CPU-baseline
    build. Returns (lib, flags); falls back to the prebuilt liboracle.so (-march=x86-64-v2)
    when no compiler is available."""
    global _native
    if _native is None:
        import shutil
        import tempfile
        flags = ["-O3", "-march=native"]
        cc = shutil.which("gcc")
        if cc:
            d = tempfile.mkdtemp(prefix="gcow_oracle_native_")
            so = os.path.join(d, "liboracle_native.so")
            r = subprocess.run([cc, *flags, "-fPIC", "-shared", "-pthread", "-o", so, os.path.join(HERE, "zfp_oracle.c"),
                                "-lm"], capture_output=True)
            if r.returncode == 0:
                _native = (_bind(C.CDLL(so)), " ".join(flags))
        if _native is None:
            _native = (lib(), "-O3 -march=x86-64-v2 (prebuilt; no compiler)")
    return _native


def _bind(L):
    if True:
        P = C.POINTER
        L.orc_block_exponent.restype = C.c_int
        L.orc_block_exponent.argtypes = [P(C.c_float), C.c_uint]
        L.orc_fwd_cast.argtypes = [P(C.c_int32), P(C.c_float), C.c_uint, C.c_int]
        L.orc_fwd_xform.argtypes = [P(C.c_int32), C.c_uint]
        L.orc_inv_xform.argtypes = [P(C.c_int32), C.c_uint]
        L.orc_fwd_reorder.argtypes = [P(C.c_uint32), P(C.c_int32), C.c_uint]
        L.orc_perm.restype = P(C.c_ubyte)
        L.orc_perm.argtypes = [C.c_uint]
        L.orc_encode_ints.restype = C.c_uint
        L.orc_encode_ints.argtypes = [P(C.c_uint64), P(C.c_uint64), P(C.c_uint32), C.c_uint, C.c_uint, C.c_uint]
        L.orc_encode_iblock.restype = C.c_uint
        L.orc_encode_iblock.argtypes = [P(C.c_uint64), P(C.c_uint64), C.c_uint, C.c_uint, C.c_uint, P(C.c_int32),
                                        C.c_uint]
        L.orc_encode_fblock.restype = C.c_uint
        L.orc_encode_fblock.argtypes = [P(C.c_uint64), P(C.c_uint64), P(Params), P(C.c_float), C.c_uint]
        L.orc_gather_block.argtypes = [P(C.c_float), C.c_void_p, C.c_int, C.c_uint, P(C.c_size_t),
                                       P(C.c_ssize_t), P(C.c_size_t)]
        L.orc_precision.restype = C.c_uint
        L.orc_precision.argtypes = [C.c_int, C.c_uint, C.c_int, C.c_uint]
        L.orc_num_blocks.restype = C.c_size_t
        L.orc_num_blocks.argtypes = [C.c_uint, P(C.c_size_t)]
        L.orc_compress.restype = C.c_uint64
        L.orc_compress.argtypes = [C.c_void_p, C.c_int, C.c_uint, P(C.c_size_t), P(C.c_ssize_t), P(Params),
                                   P(C.c_uint64), C.c_size_t]
        L.orc_compress_mt.restype = C.c_uint64
        L.orc_compress_mt.argtypes = L.orc_compress.argtypes + [C.c_int]
        L.orc_compress_mt_off.restype = C.c_uint64
        L.orc_compress_mt_off.argtypes = L.orc_compress.argtypes + [C.c_int, P(C.c_uint64)]
        L.orc_block_bits.argtypes = [C.c_void_p, C.c_int, C.c_uint, P(C.c_size_t), P(C.c_ssize_t), P(Params),
                                     P(C.c_uint32)]
        L.orc_decompress.restype = C.c_uint64
        L.orc_decompress.argtypes = [P(C.c_float), C.c_uint, P(C.c_size_t), P(C.c_ssize_t), P(Params),
                                     P(C.c_uint64), C.c_size_t]
        for f in ("orc_set_accuracy",):
            getattr(L, f).argtypes = [P(Params), C.c_double]
        L.orc_set_rate.argtypes = [P(Params), C.c_double, C.c_uint]
        L.orc_set_precision.argtypes = [P(Params), C.c_uint]
        L.orc_gen_bump2d.argtypes = [P(C.c_float), C.c_size_t, C.c_int]
        L.orc_gen_normal.argtypes = [P(C.c_float), C.c_size_t, C.c_double, C.c_uint64, C.c_int]
        L.orc_decompress_at.restype = C.c_uint64
        L.orc_decompress_at.argtypes = L.orc_decompress.argtypes + [C.c_uint64]
        L.orc_decompress_mt.restype = C.c_uint64
        L.orc_decompress_mt.argtypes = L.orc_decompress.argtypes + [C.c_int, P(C.c_uint64)]
        L.orc_stitch.argtypes = [P(C.c_uint64), C.c_uint64, P(C.c_uint64), C.c_uint64]
        L.orc_header_bits.restype = C.c_uint
        L.orc_header_bits.argtypes = [P(Params)]
        L.orc_write_header.restype = C.c_uint
        L.orc_write_header.argtypes = [P(C.c_uint64), C.c_uint, P(C.c_size_t), C.c_uint, P(Params)]
        L.orc_read_header.restype = C.c_uint
        L.orc_read_header.argtypes = [P(C.c_uint64), P(C.c_uint), P(C.c_size_t), P(C.c_uint), P(Params)]
    return L


def ref():
    """Reference sw/ encoder (2-D only) compiled from /root/reference sources, or None if not built."""
    global _ref
    if _ref is None:
        path = os.path.join(HERE, "_ref", "libgcow_ref.so")
        if not os.path.exists(path):
            return None
        L = C.CDLL(path)
        P = C.POINTER
        L.gcow_ref_compress_2d.restype = C.c_size_t
        L.gcow_ref_compress_2d.argtypes = [P(C.c_float), C.c_size_t, C.c_size_t, C.c_uint, C.c_uint, C.c_uint,
                                           C.c_int, P(C.c_uint64), C.c_size_t]
        L.gcow_ref_set_accuracy.restype = C.c_double
        L.gcow_ref_set_accuracy.argtypes = [C.c_double, P(C.c_uint), P(C.c_uint), P(C.c_uint), P(C.c_int)]
        L.gcow_ref_block_exponent.restype = C.c_int
        L.gcow_ref_block_exponent.argtypes = [P(C.c_float), C.c_uint]
        L.gcow_ref_fwd_cast.argtypes = [P(C.c_int32), P(C.c_float), C.c_uint, C.c_int]
        L.gcow_ref_fwd_decorrelate_2d.argtypes = [P(C.c_int32)]
        L.gcow_ref_fwd_reorder_2d.argtypes = [P(C.c_uint32), P(C.c_int32)]
        L.gcow_ref_encode_iblock.restype = C.c_uint
        L.gcow_ref_encode_iblock.argtypes = [P(C.c_uint64), C.c_size_t, C.c_uint, C.c_uint, C.c_uint, C.c_uint,
                                             P(C.c_int32), P(C.c_uint64)]
        _ref = L
    return _ref


def _p(a, ct):
    return a.ctypes.data_as(C.POINTER(ct))


# ------------------------------------------------------------------ parameter helpers
def accuracy(tol: float) -> Params:
    p = Params()
    lib().orc_set_accuracy(C.byref(p), tol)
    return p


def rate(r: float, dims: int) -> Params:
    p = Params()
    lib().orc_set_rate(C.byref(p), r, dims)
    return p


def precision(prec: int) -> Params:
    p = Params()
    lib().orc_set_precision(C.byref(p), prec)
    return p


def expert(minbits, maxbits, maxprec, minexp) -> Params:
    return Params(minbits, maxbits, maxprec, minexp)


# ------------------------------------------------------------------ array API
def _shape(shape):
    """shape given numpy-style (slowest first); oracle wants (nx, ny, nz) fastest first."""
    dims = len(shape)
    n = (C.c_size_t * 4)(*(list(reversed(shape)) + [0] * (4 - dims)))
    return dims, n


def max_words(shape, p: Params) -> int:
    dims = len(shape)
    nb = 1
    for s in shape:
        nb *= (s + 3) // 4
    size = 4 ** dims
    mb = 9 + size - 1 + size * min(p.maxprec, 32)
    if p.maxbits >= 9:
        mb = min(mb, p.maxbits)
    mb = max(mb, p.minbits)
    return (nb * mb + 63) // 64 + 2


def compress(arr: np.ndarray, p: Params, threads: int = 0, L=None, offsets: bool = False):
    """Encode a C-contiguous float32 (or bf16-as-uint16) array. Returns (words[uint64], total_bits), plus (offsets)
    the threaded encode's shard start bits (uint64[T + 1]) that `decompress(..., threads=T, offsets=...)` resumes at."""
    arr = np.ascontiguousarray(arr)
    dtype = BF16 if arr.dtype == np.uint16 else F32
    if dtype == F32:
        assert arr.dtype == np.float32
    dims, n = _shape(arr.shape)
    nw = max_words(arr.shape, p)
    out = np.zeros(nw, dtype=np.uint64)
    L = L or lib()
    offs = None
    if offsets:
        T = max(1, threads or 1)
        offs = np.zeros(T + 1, np.uint64)
        bits = L.orc_compress_mt_off(arr.ctypes.data, dtype, dims, n, None, C.byref(p), _p(out, C.c_uint64), nw, T,
                                     _p(offs, C.c_uint64))
        nb = lib().orc_num_blocks(dims, n)
        offs = offs[: min(T, max(nb, 1)) + 1].copy()
    elif threads and threads > 1:
        bits = L.orc_compress_mt(arr.ctypes.data, dtype, dims, n, None, C.byref(p), _p(out, C.c_uint64), nw,
                                 threads)
    else:
        bits = L.orc_compress(arr.ctypes.data, dtype, dims, n, None, C.byref(p), _p(out, C.c_uint64), nw)
    w = out[: (bits + 63) // 64].copy()
    return (w, int(bits), offs) if offsets else (w, int(bits))


def block_bits(arr: np.ndarray, p: Params) -> np.ndarray:
    arr = np.ascontiguousarray(arr)
    dtype = BF16 if arr.dtype == np.uint16 else F32
    dims, n = _shape(arr.shape)
    nb = lib().orc_num_blocks(dims, n)
    out = np.zeros(nb, dtype=np.uint32)
    lib().orc_block_bits(arr.ctypes.data, dtype, dims, n, None, C.byref(p), _p(out, C.c_uint32))
    return out


def decompress(words: np.ndarray, shape, p: Params, threads: int = 0, offsets=None) -> np.ndarray:
    """Decode into a float32 array of `shape`. threads > 1 splits the blocks as the threaded encode does: each shard
    starts at offsets[t] (from compress(..., offsets=True) with the same thread count), or at t * per * maxbits for a
    fixed-rate stream when offsets is None."""
    dims, n = _shape(shape)
    out = np.zeros(shape, dtype=np.float32)
    w = np.ascontiguousarray(words, dtype=np.uint64)
    w = np.concatenate([w, np.zeros(2, np.uint64)])
    if threads and threads > 1 and (offsets is not None or p.minbits == p.maxbits):
        T = len(offsets) - 1 if offsets is not None else threads
        offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
        lib().orc_decompress_mt(_p(out, C.c_float), dims, n, None, C.byref(p), _p(w, C.c_uint64), len(w), T,
                                None if offs is None else _p(offs, C.c_uint64))
    else:
        lib().orc_decompress(_p(out, C.c_float), dims, n, None, C.byref(p), _p(w, C.c_uint64), len(w))
    return out


def gen_bump2d(n: int, f32sum: bool = False) -> np.ndarray:
    out = np.empty((n, n), dtype=np.float32)
    lib().orc_gen_bump2d(_p(out, C.c_float), n, int(f32sum))
    return out


def gen_normal(count: int, sigma: float = 1e-3, seed: int = 0x67636F77, inject: bool = True) -> np.ndarray:
    out = np.empty(count, dtype=np.float32)
    lib().orc_gen_normal(_p(out, C.c_float), count, sigma, seed, int(inject))
    return out


# ------------------------------------------------------------------ stage API (known-answer tests)
def block_exponent(block: np.ndarray) -> int:
    b = np.ascontiguousarray(block, dtype=np.float32)
    return lib().orc_block_exponent(_p(b, C.c_float), b.size)


def fwd_cast(fblock: np.ndarray, emax: int) -> np.ndarray:
    f = np.ascontiguousarray(fblock, dtype=np.float32)
    q = np.zeros(f.size, dtype=np.int32)
    lib().orc_fwd_cast(_p(q, C.c_int32), _p(f, C.c_float), f.size, emax)
    return q


def fwd_xform(iblock: np.ndarray, dims: int) -> np.ndarray:
    q = np.array(iblock, dtype=np.int32)
    lib().orc_fwd_xform(_p(q, C.c_int32), dims)
    return q


def inv_xform(iblock: np.ndarray, dims: int) -> np.ndarray:
    q = np.array(iblock, dtype=np.int32)
    lib().orc_inv_xform(_p(q, C.c_int32), dims)
    return q


def fwd_reorder(iblock: np.ndarray, dims: int) -> np.ndarray:
    q = np.ascontiguousarray(iblock, dtype=np.int32)
    u = np.zeros(q.size, dtype=np.uint32)
    lib().orc_fwd_reorder(_p(u, C.c_uint32), _p(q, C.c_int32), dims)
    return u


def perm(dims: int) -> list:
    P = lib().orc_perm(dims)
    return [P[i] for i in range(4 ** dims)]


def encode_ints(ublock: np.ndarray, maxbits: int, maxprec: int, pos0: int = 0, words: np.ndarray | None = None):
    u = np.ascontiguousarray(ublock, dtype=np.uint32)
    if words is None:
        words = np.zeros(64, dtype=np.uint64)
    pos = C.c_uint64(pos0)
    bits = lib().orc_encode_ints(_p(words, C.c_uint64), C.byref(pos), _p(u, C.c_uint32), maxbits, maxprec, u.size)
    return words, int(pos.value), int(bits)


def encode_iblock(iblock: np.ndarray, minbits, maxbits, maxprec, dims, pos0=0, words=None):
    q = np.array(iblock, dtype=np.int32)
    if words is None:
        words = np.zeros(512, dtype=np.uint64)
    pos = C.c_uint64(pos0)
    bits = lib().orc_encode_iblock(_p(words, C.c_uint64), C.byref(pos), minbits, maxbits, maxprec,
                                   _p(q, C.c_int32), dims)
    return words, int(pos.value), int(bits)


def put_bits_header(words: np.ndarray, value: int, nbits: int, pos0: int = 0) -> int:
    """Write a header field via the oracle's coder path (used by known-answer tests)."""
    # encode the header as verbatim bits: set bits directly (LSB-first)
    for i in range(nbits):
        if (value >> i) & 1:
            p = pos0 + i
            words[p >> 6] |= np.uint64(1) << np.uint64(p & 63)
    return pos0 + nbits


# ------------------------------------------------------------------ zfp 0.5.5 header (zfpy byte streams)
def write_header(shape, p: Params, zfp_type: int = 3):
    """Header words (3 x uint64) and bit count, as zfp_write_header(ZFP_HEADER_FULL)."""
    dims, n = _shape(shape)
    w = np.zeros(3, np.uint64)
    bits = lib().orc_write_header(_p(w, C.c_uint64), dims, n, zfp_type, C.byref(p))
    return w, int(bits)


def read_header(words):
    """-> (shape numpy-style, zfp_type, Params, header bits); header bits 0 when the magic does not match."""
    w = np.zeros(3, np.uint64)
    src = np.ascontiguousarray(words, dtype=np.uint64)[:3]
    w[: len(src)] = src
    dims, n, t, p = C.c_uint(), (C.c_size_t * 4)(), C.c_uint(), Params()
    bits = lib().orc_read_header(_p(w, C.c_uint64), C.byref(dims), n, C.byref(t), C.byref(p))
    shape = tuple(reversed([n[i] for i in range(dims.value)])) if bits else ()
    return shape, t.value, p, int(bits)


def compress_zfp(arr: np.ndarray, p: Params):
    """zfpy.compress_numpy-style stream: header, then the blocks at the following bit, flushed to 64 bits."""
    h, hb = write_header(arr.shape, p)
    w, bits = compress(arr, p)
    out = np.zeros((hb + bits + 63) // 64 + 1, np.uint64)
    out[:3] |= h[:len(out[:3])]
    lib().orc_stitch(_p(out, C.c_uint64), hb, _p(w, C.c_uint64), bits)
    return out[: (hb + bits + 63) // 64].copy(), hb + bits


def decompress_zfp(words: np.ndarray) -> np.ndarray:
    shape, t, p, hb = read_header(words)
    assert hb and t == 3, "not a float zfp stream"
    dims, n = _shape(shape)
    out = np.zeros(shape, dtype=np.float32)
    w = np.concatenate([np.ascontiguousarray(words, dtype=np.uint64), np.zeros(2, np.uint64)])
    lib().orc_decompress_at(_p(out, C.c_float), dims, n, None, C.byref(p), _p(w, C.c_uint64), len(w), hb)
    return out
