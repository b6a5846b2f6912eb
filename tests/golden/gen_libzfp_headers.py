"""Generate libzfp 0.5.5 golden vectors for the zfp stream header (run in the build container only).

The reference caller compresses with zfpy.compress_numpy (hw/models/train_imagenet.py:459-465), which writes a
ZFP_HEADER_FULL header (magic 'zfp' + codec version, 52-bit field metadata, 12- or 64-bit mode) before the blocks;
sw/ declares the header constants (sw/include/common.h:16-21) but never writes them. These fixtures pin the header
bits for every mode class (rate / precision / accuracy short forms, their range limits, expert and default long
forms) and whole header+stream byte strings as zfpy produces them (zfp_write_header, then zfp_compress at the
following bit), plus libzfp's decode of those streams via zfp_read_header.

Output: tests/golden/libzfp_headers.json + libzfp_headers.npz.
"""
import ctypes as C
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import gen_libzfp_fixtures_4d  # noqa: E402,F401  (adds zfp_field_4d to gen_libzfp_fixtures.field)
import gen_libzfp_fixtures as G  # noqa: E402
from gen_libzfp_fixtures import Z, ZFP_FLOAT, zstream  # noqa: E402
from oracle import oracle as O  # noqa: E402  (input generator only)

Z.zfp_write_header.restype = C.c_size_t
Z.zfp_write_header.argtypes = [C.c_void_p, C.c_void_p, C.c_uint]
Z.zfp_read_header.restype = C.c_size_t
Z.zfp_read_header.argtypes = [C.c_void_p, C.c_void_p, C.c_uint]
Z.zfp_stream_flush.restype = C.c_size_t
Z.zfp_stream_flush.argtypes = [C.c_void_p]
Z.zfp_stream_set_bit_stream.argtypes = [C.c_void_p, C.c_void_p]
Z.zfp_field_alloc.restype = C.c_void_p
Z.zfp_field_set_pointer.argtypes = [C.c_void_p, C.c_void_p]
Z.zfp_field_size.restype = C.c_size_t
Z.zfp_field_size.argtypes = [C.c_void_p, C.POINTER(C.c_uint)]
Z.zfp_field_dimensionality.restype = C.c_uint
Z.zfp_field_dimensionality.argtypes = [C.c_void_p]
Z.zfp_field_type.restype = C.c_int
Z.zfp_field_type.argtypes = [C.c_void_p]
Z.zfp_stream_params.argtypes = [C.c_void_p] + [C.POINTER(C.c_uint)] * 3 + [C.POINTER(C.c_int)]
HEADER_FULL = 7


def params_of(zs):
    a, b, c, d = C.c_uint(), C.c_uint(), C.c_uint(), C.c_int()
    Z.zfp_stream_params(zs, C.byref(a), C.byref(b), C.byref(c), C.byref(d))
    return [a.value, b.value, c.value, d.value]


def with_header(arr, mode, compress=True):
    arr = np.ascontiguousarray(arr, dtype=np.float32)
    if mode[0] == "expert":
        zs = Z.zfp_stream_open(None)
        if not Z.zfp_stream_set_params(zs, *mode[1]):
            Z.zfp_stream_close(zs)
            return None  # libzfp rejects these parameters
        params = params_of(zs)
    else:
        zs, params = zstream(mode, arr.ndim)
    buf = np.zeros((arr.size * 16 + 4096) // 8, dtype=np.uint64)
    bs = Z.stream_open(buf.ctypes.data, buf.nbytes)
    Z.zfp_stream_set_bit_stream(zs, bs)
    Z.zfp_stream_rewind(zs)
    fld = G.field(arr)
    hbits = Z.zfp_write_header(zs, fld, HEADER_FULL)
    if compress:
        nbytes = Z.zfp_compress(zs, fld)
    else:
        nbytes = Z.zfp_stream_flush(zs) and 0
        nbytes = (hbits + 63) // 64 * 8
    Z.zfp_field_free(fld)
    words = buf[: nbytes // 8].copy()
    # read back with libzfp (what zfpy.decompress_numpy does)
    Z.zfp_stream_rewind(zs)
    rf = Z.zfp_field_alloc()
    rbits = Z.zfp_read_header(zs, rf, HEADER_FULL)
    assert rbits == hbits, (rbits, hbits)
    dims = Z.zfp_field_dimensionality(rf)
    sz = (C.c_uint * 4)()
    Z.zfp_field_size(rf, sz)
    rparams = params_of(zs)
    dec = None
    if compress:
        dec = np.zeros(arr.shape, dtype=np.float32)
        Z.zfp_field_set_pointer(rf, dec.ctypes.data)
        Z.zfp_decompress(zs, rf)
    Z.zfp_field_free(rf)
    Z.zfp_stream_close(zs)
    Z.stream_close(bs)
    return dict(header_bits=int(hbits), params=list(params), read_params=rparams, read_dims=int(dims),
                read_shape=[int(sz[i]) for i in range(dims)], 
                words=words, decoded=dec)


def main():
    cases, arrays = [], {}
    # header-only cases over every mode class and limit (no data needed: the header depends on shape + params)
    shapes = [(1000,), (1,), (7, 100), (7, 6, 5), (1 << 20,), (3, 4, 5, 6), (4096, 1, 2, 4096)]
    modes = [("rate", 16.0), ("rate", 8.0), ("rate", 2.5), ("rate", 128.0), ("rate", 129.0),
             ("acc", 1e-3), ("acc", 1e-6), ("acc", 0.5),
             ("prec", 1), ("prec", 20), ("prec", 64),
             ("expert", (10, 200, 30, -50)), ("expert", (1, 16657, 64, -1074)), ("expert", (1, 16658, 64, -10)),
             ("expert", (1, 16657, 64, 843)), ("expert", (1, 16657, 64, 844)), ("expert", (64, 64, 63, -1074)),
             ("expert", (2048, 2048, 64, -1074)), ("expert", (2049, 2049, 64, -1074)), ("expert", (1, 20000, 64, -1074)),
             ("expert", (5, 16657, 64, -10)), ("expert", (1, 16657, 128, -1074))]
    for shp in shapes:
        for mode in modes:
            if mode[0] == "rate" and len(shp) in (1, 4) and mode[1] > 100:
                continue
            arr = np.zeros(shp, np.float32)
            r = with_header(arr, mode, compress=False)
            if r is None:
                print("libzfp rejects", mode)
                continue
            name = "hdr_%s__%s_%s" % ("x".join(map(str, shp)), mode[0], "_".join(str(v) for v in np.atleast_1d(mode[1])))
            cases.append(dict(name=name, kind="header", shape=list(shp), mode=mode[0],
                              value=mode[1] if mode[0] != "expert" else list(mode[1]), params=r["params"],
                              header_bits=r["header_bits"], header_words=[int(w) for w in r["words"]],
                              read_params=r["read_params"], read_dims=r["read_dims"], read_shape=r["read_shape"]))
    # whole zfpy-style streams: header then blocks at the following bit
    inputs = {
        "1d_n1000": O.gen_normal(1000, 1e-3, 0x67636F77 + 1000, True),
        "1d_n4099": O.gen_normal(4099, 1e-3, 0x67636F77 + 4099, True),
        "2d_10x9": O.gen_normal(90, 1.0, 7, False).reshape(10, 9),
        "2d_bump37": O.gen_bump2d(37),
        "3d_7x10x9": O.gen_normal(630, 1.0, 10, False).reshape(7, 10, 9),
        "4d_3x6x5x7": O.gen_normal(630, 1.0, 11, False).reshape(3, 6, 5, 7),
    }
    smodes = [("rate", 16.0), ("rate", 8.0), ("acc", 1e-3), ("acc", 1e-6), ("prec", 20), ("expert", (10, 200, 30, -50))]
    for iname, arr in inputs.items():
        arrays["input__" + iname] = arr
        for mode in smodes:
            r = with_header(arr, mode)
            name = "zfpy_%s__%s_%s" % (iname, mode[0], "_".join(str(v) for v in np.atleast_1d(mode[1])))
            arrays[name + "__stream"] = r["words"]
            arrays[name + "__decoded"] = r["decoded"]
            cases.append(dict(name=name, kind="stream", input=iname, shape=list(arr.shape), mode=mode[0],
                              value=mode[1] if mode[0] != "expert" else list(mode[1]), params=r["params"],
                              header_bits=r["header_bits"], read_params=r["read_params"],
                              bytes=int(r["words"].nbytes),
                              stream_sha256=hashlib.sha256(r["words"].tobytes()).hexdigest(),
                              decoded_sha256=hashlib.sha256(r["decoded"].tobytes()).hexdigest()))
    np.savez_compressed(os.path.join(HERE, "libzfp_headers.npz"), **arrays)
    with open(os.path.join(HERE, "libzfp_headers.json"), "w") as f:
        json.dump(dict(generator="libzfp 0.5.5 (/opt/conda/lib/libzfp.so.0.5.5) zfp_write_header(ZFP_HEADER_FULL) "
                                 "+ zfp_compress; zfp_read_header + zfp_decompress",
                       script="tests/golden/gen_libzfp_headers.py", cases=cases), f, indent=1)
    print("cases:", len(cases))


if __name__ == "__main__":
    main()
