"""Generate libzfp 0.5.5 4-D golden vectors (run in the build container only; never at test time).

The 4-D path is SURVEY.md 8(f) rank 4 (sw/ declares gather_partial_4d_block, sw/src/encode.c:90-126, and reserves
nw / sw in zfp_input, sw/include/types.h:51-56, but zfp_compress never reaches it). libzfp 0.5.5 (zfp_field_4d)
pins it: streams and decoded arrays for rate, accuracy, precision and expert modes, partial blocks on every axis and
special values. Output: tests/golden/libzfp_fixtures_4d.npz + libzfp_fixtures_4d.json (same layout as the 1-3-D set).
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
import gen_libzfp_fixtures as G  # noqa: E402  (libzfp bindings and the stream helpers)
from oracle import oracle as O  # noqa: E402  (input generator only)

G.Z.zfp_field_4d.restype = C.c_void_p
G.Z.zfp_field_4d.argtypes = [C.c_void_p, C.c_int, C.c_uint, C.c_uint, C.c_uint, C.c_uint]
_field_1to3 = G.field


def _field(arr):
    if arr.ndim == 4:
        s = arr.shape
        return G.Z.zfp_field_4d(arr.ctypes.data, G.ZFP_FLOAT, s[3], s[2], s[1], s[0])
    return _field_1to3(arr)


G.field = _field


def main():
    inputs = {}
    rng = np.random.default_rng(4)
    inputs["4d_5x6x7x9"] = (rng.standard_normal((5, 6, 7, 9)) * 1e-2).astype(np.float32)
    x = np.arange(8, dtype=np.float64) / 8
    g = (np.sin(2 * np.pi * x)[None, None, None, :] * np.cos(2 * np.pi * x)[None, None, :, None] *
         np.sin(4 * np.pi * x)[None, :, None, None] * np.cos(np.pi * x)[:, None, None, None])
    inputs["4d_wave8"] = (g + 1e-3 * O.gen_normal(8 ** 4, 1.0, 12, False).reshape(8, 8, 8, 8)).astype(np.float32)
    sp = np.tile(G.special_1d(), 13)[:4 * 4 * 4 * 5].reshape(5, 4, 4, 4)
    inputs["4d_special"] = sp.astype(np.float32)
    inputs["4d_1x2x3x5"] = O.gen_normal(30, 1.0, 13, False).reshape(1, 2, 3, 5)
    modes = [("rate", 2.0), ("rate", 8.0), ("rate", 2.5), ("acc", 1e-3), ("acc", 1e-6), ("prec", 12),
             ("expert", (1, 16658, 64, -1074)), ("expert", (300, 900, 20, -30))]
    cases, arrays = [], {}
    for iname, arr in inputs.items():
        for mode in modes:
            words, dec, params = G.zcompress(arr, mode)
            cname = "%s__%s_%s" % (iname, mode[0], "_".join(str(v) for v in np.atleast_1d(mode[1])))
            arrays[cname + "__stream"] = words
            arrays[cname + "__decoded"] = dec
            cases.append(dict(name=cname, input=iname, shape=list(arr.shape), mode=mode[0],
                              value=mode[1] if mode[0] != "expert" else list(mode[1]), params=list(params),
                              bytes=int(words.nbytes), stream_sha256=hashlib.sha256(words.tobytes()).hexdigest(),
                              decoded_sha256=hashlib.sha256(dec.tobytes()).hexdigest()))
    for k, v in inputs.items():
        arrays["input__" + k] = v
    np.savez_compressed(os.path.join(HERE, "libzfp_fixtures_4d.npz"), **arrays)
    with open(os.path.join(HERE, "libzfp_fixtures_4d.json"), "w") as f:
        json.dump(dict(generator="libzfp 0.5.5 (/opt/conda/lib/libzfp.so.0.5.5) zfp_field_4d, headerless streams",
                       script="tests/golden/gen_libzfp_fixtures_4d.py", cases=cases), f, indent=1)
    print("cases:", len(cases))


if __name__ == "__main__":
    main()
