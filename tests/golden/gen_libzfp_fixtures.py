"""Generate libzfp 0.5.5 golden vectors (run in the build container only; never at test time).

LLNL zfp 0.5.5 (conda package zfp-0.5.5-h2531618_6, /opt/conda/lib/libzfp.so.0.5.5) is the third-party library gcow's
sw/ encoder is byte-identical to on 2-D; it pins the 1-D, 3-D, fixed-rate, precision,
expert and decode behaviour that the reference's own goldens (2-D, accuracy 1e-3) do not cover.
Streams are headerless (zfp_compress without zfp_write_header), as sw/ writes them.

Output: tests/golden/libzfp_fixtures.npz (inputs, streams, decoded arrays) + libzfp_fixtures.json (index).
"""
import ctypes as C
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402  (input generator only)

Z = C.CDLL("/opt/conda/lib/libzfp.so.0.5.5")
Z.stream_open.restype = C.c_void_p
Z.stream_open.argtypes = [C.c_void_p, C.c_size_t]
Z.stream_close.argtypes = [C.c_void_p]
Z.zfp_stream_open.restype = C.c_void_p
Z.zfp_stream_open.argtypes = [C.c_void_p]
Z.zfp_stream_close.argtypes = [C.c_void_p]
Z.zfp_stream_set_params.restype = C.c_int
Z.zfp_stream_set_params.argtypes = [C.c_void_p, C.c_uint, C.c_uint, C.c_uint, C.c_int]
Z.zfp_stream_params.argtypes = [C.c_void_p] + [C.POINTER(C.c_uint)] * 3 + [C.POINTER(C.c_int)]
Z.zfp_stream_set_rate.restype = C.c_double
Z.zfp_stream_set_rate.argtypes = [C.c_void_p, C.c_double, C.c_int, C.c_uint, C.c_int]
Z.zfp_stream_set_accuracy.restype = C.c_double
Z.zfp_stream_set_accuracy.argtypes = [C.c_void_p, C.c_double]
Z.zfp_stream_set_precision.restype = C.c_uint
Z.zfp_stream_set_precision.argtypes = [C.c_void_p, C.c_uint]
Z.zfp_stream_rewind.argtypes = [C.c_void_p]
for f in ("zfp_field_1d", "zfp_field_2d", "zfp_field_3d"):
    getattr(Z, f).restype = C.c_void_p
Z.zfp_field_1d.argtypes = [C.c_void_p, C.c_int, C.c_uint]
Z.zfp_field_2d.argtypes = [C.c_void_p, C.c_int, C.c_uint, C.c_uint]
Z.zfp_field_3d.argtypes = [C.c_void_p, C.c_int, C.c_uint, C.c_uint, C.c_uint]
Z.zfp_field_free.argtypes = [C.c_void_p]
Z.zfp_compress.restype = C.c_size_t
Z.zfp_compress.argtypes = [C.c_void_p, C.c_void_p]
Z.zfp_decompress.restype = C.c_size_t
Z.zfp_decompress.argtypes = [C.c_void_p, C.c_void_p]
ZFP_FLOAT = 3


def field(arr):
    s = arr.shape
    if len(s) == 1:
        return Z.zfp_field_1d(arr.ctypes.data, ZFP_FLOAT, s[0])
    if len(s) == 2:
        return Z.zfp_field_2d(arr.ctypes.data, ZFP_FLOAT, s[1], s[0])
    return Z.zfp_field_3d(arr.ctypes.data, ZFP_FLOAT, s[2], s[1], s[0])


def zstream(mode, dims):
    zs = Z.zfp_stream_open(None)
    kind, val = mode
    if kind == "rate":
        Z.zfp_stream_set_rate(zs, val, ZFP_FLOAT, dims, 0)
    elif kind == "acc":
        Z.zfp_stream_set_accuracy(zs, val)
    elif kind == "prec":
        Z.zfp_stream_set_precision(zs, val)
    else:
        assert Z.zfp_stream_set_params(zs, *val)
    a, b, c, d = C.c_uint(), C.c_uint(), C.c_uint(), C.c_int()
    Z.zfp_stream_params(zs, C.byref(a), C.byref(b), C.byref(c), C.byref(d))
    return zs, (a.value, b.value, c.value, d.value)


def zcompress(arr, mode):
    arr = np.ascontiguousarray(arr, dtype=np.float32)
    zs, params = zstream(mode, arr.ndim)
    cap = arr.size * 16 + 4096
    buf = np.zeros(cap // 8, dtype=np.uint64)
    bs = Z.stream_open(buf.ctypes.data, buf.nbytes)
    Z.zfp_stream_set_bit_stream.argtypes = [C.c_void_p, C.c_void_p]
    Z.zfp_stream_set_bit_stream(zs, bs)
    Z.zfp_stream_rewind(zs)
    fld = field(arr)
    nbytes = Z.zfp_compress(zs, fld)
    assert nbytes > 0
    Z.zfp_field_free(fld)
    # decode
    out = np.zeros_like(arr)
    Z.zfp_stream_rewind(zs)
    fld = field(out)
    Z.zfp_decompress(zs, fld)
    Z.zfp_field_free(fld)
    Z.zfp_stream_close(zs)
    Z.stream_close(bs)
    return buf[: nbytes // 8].copy(), out, params


def f32(bits):
    return np.array([bits], dtype=np.uint32).view(np.float32)[0]


def special_1d():
    """Blocks that exercise every bit-exactness corner of SURVEY 0.5 / Appendix A."""
    blocks = [
        [0.0, 0.0, 0.0, 0.0],
        [-0.0, 0.0, -0.0, 0.0],
        [1e-35, -2e-35, 3e-36, 0.0],  # emax <= -98: scale overflows -> INT_MIN path
        [1e-40, -1e-41, 1.4e-45, 0.0],  # subnormals
        [f32(0x7FC00000), 1.0, -0.5, 0.25],  # NaN skipped by max, cast -> INT_MIN
        [np.inf, 1.0, -1.0, 0.0],  # Inf -> emax 0 (glibc frexp)
        [-np.inf, 3e9, 1.0, 2.0],  # Inf + out-of-range cast
        [1e30, 1e-30, -1e30, 5.0],
        [3.4028235e38, -3.4028235e38, 1.0, 0.0],
        [1.0, 2.0, 4.0, 8.0],
        [-1.0, -1.0, -1.0, -1.0],
        [0.5, -0.5, 0.5, -0.5],
        [1.1754944e-38, -1.1754944e-38, 1e-38, 0.0],  # smallest normal boundary
        [1e10, -1e10, 12345.678, -0.001],
        [f32(0x7F800001), f32(0xFFC00000), f32(0x7FC00000), f32(0x7FFFFFFF)],  # all NaN
        [123.0, 123.0, 123.0, 123.0],
        [2.0**-98, 2.0**-99, 0.0, 0.0],
        [2.0**-97, -(2.0**-97), 0.0, 0.0],
        [1.0, 0.0, 0.0, 0.0],
        [0.0, 0.0, 0.0, -1.0],
    ]
    return np.array(blocks, dtype=np.float32).reshape(-1)


def main():
    cases = []
    arrays = {}
    inputs = {}

    def add_input(name, arr):
        inputs[name] = np.ascontiguousarray(arr, dtype=np.float32)

    for n in (1, 2, 3, 4, 5, 6, 7, 8, 13, 64, 257, 1000, 4099):
        add_input("1d_n%d" % n, O.gen_normal(n, 1e-3, 0x67636F77 + n, True))
    add_input("1d_inject", O.gen_normal(1 << 14, 1e-3, 0x67636F77, True))
    add_input("1d_special", special_1d())
    add_input("1d_special_tail", special_1d()[:-1])
    add_input("2d_9x10", O.gen_normal(90, 1.0, 7, False).reshape(10, 9))
    add_input("2d_16x16", O.gen_normal(256, 1.0, 8, False).reshape(16, 16))
    add_input("2d_bump37", O.gen_bump2d(37))
    add_input("2d_special", np.concatenate([special_1d(), special_1d()[:48]]).reshape(8, 16))
    add_input("3d_16x16x16", O.gen_normal(4096, 1e-3, 9, True).reshape(16, 16, 16))
    add_input("3d_9x10x7", O.gen_normal(630, 1.0, 10, False).reshape(7, 10, 9))
    add_input("3d_special", np.tile(special_1d(), 7)[:4 * 4 * 8].reshape(8, 4, 4))
    x = np.arange(12, dtype=np.float64) / 12
    g = (np.sin(6 * np.pi * x)[None, None, :] * np.cos(4 * np.pi * x)[None, :, None] * np.sin(2 * np.pi * x)[:, None, None])
    add_input("3d_wave12", (g + 1e-3 * O.gen_normal(12 ** 3, 1.0, 11, False).reshape(12, 12, 12)).astype(np.float32))

    modes = [("rate", 4.0), ("rate", 8.0), ("rate", 16.0), ("rate", 32.0), ("rate", 2.5),
             ("acc", 1e-1), ("acc", 1e-3), ("acc", 1e-6), ("prec", 8), ("prec", 20), ("prec", 33),
             ("expert", (24, 60, 18, -20)), ("expert", (40, 400, 64, -1074)), ("expert", (1, 16658, 64, -1074))]
    for iname, arr in inputs.items():
        for mode in modes:
            words, dec, params = zcompress(arr, mode)
            cname = "%s__%s_%s" % (iname, mode[0], "_".join(str(v) for v in np.atleast_1d(mode[1])))
            arrays[cname + "__stream"] = words
            if dec.size <= 4096:
                arrays[cname + "__decoded"] = dec
            cases.append(dict(name=cname, input=iname, shape=list(arr.shape), mode=mode[0],
                              value=mode[1] if mode[0] != "expert" else list(mode[1]), params=list(params),
                              bytes=int(words.nbytes),
                              stream_sha256=hashlib.sha256(words.tobytes()).hexdigest(),
                              decoded_sha256=hashlib.sha256(dec.tobytes()).hexdigest()))
    for k, v in inputs.items():
        arrays["input__" + k] = v
    np.savez_compressed(os.path.join(HERE, "libzfp_fixtures.npz"), **arrays)
    with open(os.path.join(HERE, "libzfp_fixtures.json"), "w") as f:
        json.dump(dict(generator="libzfp 0.5.5 (/opt/conda/lib/libzfp.so.0.5.5), headerless streams",
                       script="tests/golden/gen_libzfp_fixtures.py", cases=cases), f, indent=1)
    print("cases:", len(cases))


if __name__ == "__main__":
    main()
