"""zfp 0.5.5 stream header (zfpy byte streams): the oracle restatement against libzfp-generated fixtures.

Fixtures: tests/golden/libzfp_headers.{json,npz} from tests/golden/gen_libzfp_headers.py (libzfp 0.5.5
zfp_write_header(ZFP_HEADER_FULL) + zfp_compress, zfp_read_header + zfp_decompress).
"""
import hashlib
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
META = json.load(open(os.path.join(GOLD, "libzfp_headers.json")))
HDR = [c for c in META["cases"] if c["kind"] == "header"]
STREAMS = [c for c in META["cases"] if c["kind"] == "stream"]


@pytest.fixture(scope="module")
def npz():
    return np.load(os.path.join(GOLD, "libzfp_headers.npz"))


@pytest.mark.parametrize("c", HDR, ids=lambda c: c["name"])
def test_header_bits_match_libzfp(orc, c):
    w, bits = orc.write_header(tuple(c["shape"]), orc.expert(*c["params"]))
    assert bits == c["header_bits"]
    nw = (bits + 63) // 64
    assert [int(x) for x in w[:nw]] == c["header_words"]
    shape, t, p, rbits = orc.read_header(np.array(c["header_words"], np.uint64))
    assert rbits == bits and t == 3
    assert list(reversed(shape)) == c["read_shape"] and len(shape) == c["read_dims"]
    assert list(p.tuple()) == c["read_params"]


@pytest.mark.parametrize("c", STREAMS, ids=lambda c: c["name"])
def test_zfpy_stream_matches_libzfp(orc, npz, c):
    a = npz["input__" + c["input"]]
    w, bits = orc.compress_zfp(a, orc.expert(*c["params"]))
    assert w.nbytes == c["bytes"]
    assert hashlib.sha256(w.tobytes()).hexdigest() == c["stream_sha256"]
    d = orc.decompress_zfp(npz[c["name"] + "__stream"])
    assert hashlib.sha256(d.tobytes()).hexdigest() == c["decoded_sha256"]


def test_bad_magic_rejected(orc):
    w, _ = orc.write_header((10,), orc.rate(16, 1))
    w[0] ^= 1
    assert orc.read_header(w)[3] == 0
