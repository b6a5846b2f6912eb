"""zfp 0.5.5 header streams (zfpy.compress_numpy byte format) through libgcow.so.

CPU: the host header writer/reader against libzfp fixtures (tests/golden/libzfp_headers.json).
GPU: device encode-with-header byte-identical to libzfp's zfp_write_header + zfp_compress, and device decode of
libzfp's header streams equal to libzfp's zfp_read_header + zfp_decompress; a large 1-D case against the oracle.
"""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
META = json.load(open(os.path.join(GOLD, "libzfp_headers.json")))
HDR = [c for c in META["cases"] if c["kind"] == "header"]
STREAMS = [c for c in META["cases"] if c["kind"] == "stream"]


@pytest.fixture(scope="module")
def codec():
    from gcow_amd import codec as c
    return c


@pytest.fixture(scope="module")
def npz():
    return np.load(os.path.join(GOLD, "libzfp_headers.npz"))


@pytest.mark.parametrize("c", HDR, ids=lambda c: c["name"])
def test_host_header_matches_libzfp(codec, c):
    w, bits = codec.write_header(tuple(c["shape"]), codec.expert(*c["params"]))
    assert bits == c["header_bits"]
    assert w[: (bits + 63) // 64] == c["header_words"]
    shape, p, rb = codec.read_header(c["header_words"])
    assert rb == bits and list(p.tuple()) == c["read_params"] and list(reversed(shape)) == c["read_shape"]


def test_header_rejects(codec):
    from gcow_amd._ffi import GcowError
    w, _ = codec.write_header((5, 6), codec.rate(8, 2))
    with pytest.raises(GcowError):
        codec.read_header([w[0] ^ 0xFF] + w[1:])
    with pytest.raises(GcowError):
        codec.read_header([(w[0] & ~(3 << 32)) | (1 << 32), w[1], w[2]])  # zfp type int64 -> not float


@pytest.mark.gpu
@pytest.mark.parametrize("c", STREAMS, ids=lambda c: c["name"])
def test_device_zfpy_stream(codec, npz, c):
    a = npz["input__" + c["input"]]
    x = torch.from_numpy(a).cuda()
    w = codec.compress_zfp(x, codec.expert(*c["params"]))
    b = w.cpu().numpy().tobytes()
    assert len(b) == c["bytes"]
    assert hashlib.sha256(b).hexdigest() == c["stream_sha256"]
    s = torch.from_numpy(npz[c["name"] + "__stream"].view(np.int64)).cuda()
    d = codec.decompress_numpy(s)
    assert tuple(d.shape) == tuple(c["shape"])
    assert hashlib.sha256(d.cpu().numpy().tobytes()).hexdigest() == c["decoded_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["rate16", "rate8", "acc1e-6", "prec20"])
def test_device_zfpy_large_1d(codec, orc, mode):
    n = (1 << 22) + 3  # partial last block
    a = orc.gen_normal(n, 1e-3, 4242, True)
    p = {"rate16": codec.rate(16, 1), "rate8": codec.rate(8, 1), "acc1e-6": codec.accuracy(1e-6),
         "prec20": codec.precision(20)}[mode]
    w = codec.compress_zfp(torch.from_numpy(a).cuda(), p)
    ref, bits = orc.compress_zfp(a, orc.expert(*p.tuple()))
    assert np.array_equal(w.cpu().numpy().view(np.uint64), ref)
    d = codec.decompress_numpy(w)
    assert np.array_equal(d.cpu().numpy(), orc.decompress_zfp(ref))
