"""The oracle is pinned before it is trusted: reference goldens (SHA-256 manifest), the reference's known-answer
vectors, libzfp 0.5.5 fixtures (1-D/2-D/3-D, all modes, decode) and the reference sw/ compiled in place."""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _sha(b):
    return hashlib.sha256(b).hexdigest()


def load_json(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


@pytest.mark.parametrize("g", load_json("reference_goldens.json")["goldens"], ids=lambda g: g["file"])
def test_reference_goldens(orc, g):
    """sw/tests/test_zfp.cpp:61-107: 2-D bump, tolerance 1e-3, byte-compare against compressed_2d_<n>.zfp."""
    a = orc.gen_bump2d(g["n"], g["recipe"] == "bump_f32sum")
    w, bits = orc.compress(a, orc.accuracy(g["tolerance"]))
    assert w.nbytes == g["bytes"]
    assert [int(x) for x in w[:3]] == g["first_words"]
    assert _sha(w.tobytes()) == g["sha256"]


KA = load_json("reference_known_answers.json")


def test_accuracy_params(orc):
    # common.c:6-21 on tolerance 1e-3 -> (1, 16658, 64, -10)
    assert orc.accuracy(1e-3).tuple() == (1, 16658, 64, -10)
    assert orc.accuracy(1e-6).minexp == -20
    assert orc.rate(16, 1).tuple() == (64, 64, 64, -1074)
    assert orc.rate(8, 3).tuple() == (512, 512, 64, -1074)


def test_known_gather(orc):
    k = KA["gather_2d"]
    nx, ny = k["nx"], k["ny"]
    raw = (np.arange(nx * ny, dtype=np.float32) + 1).reshape(ny, nx)
    blocks = []
    for by in range(2):
        for bx in range(2):
            f = np.zeros(16, np.float32)
            n = (C.c_size_t * 3)(nx, ny, 0)
            b = (C.c_size_t * 3)(bx, by, 0)
            orc.lib().orc_gather_block(f.ctypes.data_as(C.POINTER(C.c_float)), raw.ctypes.data, orc.F32, 2, n, None, b)
            blocks.append(f.astype(int).tolist())
    assert blocks == k["expected_blocks"]


def _gather_partial_3x3(orc, raw3x3):
    f = np.zeros(16, np.float32)
    n = (C.c_size_t * 3)(3, 3, 0)
    b = (C.c_size_t * 3)(0, 0, 0)
    orc.lib().orc_gather_block(f.ctypes.data_as(C.POINTER(C.c_float)), raw3x3.ctypes.data, orc.F32, 2, n, None, b)
    return f


def test_known_emax_cast_decorrelate_reorder(orc):
    ramp = np.array([[i + 4 * j + 1 for i in range(3)] for j in range(3)], np.float32)
    assert orc.block_exponent(_gather_partial_3x3(orc, ramp)) == KA["emax"]["ramp_3x3"]["expected"]
    bump = orc.gen_bump2d(3)
    fb = _gather_partial_3x3(orc, bump)
    assert orc.block_exponent(fb) == KA["emax"]["bump_3x3"]["expected"]
    assert orc.fwd_cast(fb, KA["cast"]["emax"]).tolist() == KA["cast"]["expected"]
    assert orc.fwd_xform(np.array(KA["decorrelate"]["input"]), 2).tolist() == KA["decorrelate"]["expected"]
    assert orc.fwd_reorder(np.array(KA["reorder"]["input"]), 2).tolist() == KA["reorder"]["expected"]


def test_known_encode_all_bitplanes(orc):
    k = KA["encode_all_bitplanes"]
    p = orc.accuracy(k["tolerance"])
    maxprec = orc.lib().orc_precision(k["emax"], p.maxprec, p.minexp, 2)
    assert maxprec == k["expected_maxprec"]
    words = np.zeros(16, np.uint64)
    pos = 0
    for _ in range(k["repeat"]):
        pos = orc.put_bits_header(words, 2 * (k["emax"] + 127) + 1, 9, pos)
        words, pos, _ = orc.encode_ints(np.array(k["ublock"]), 0xFFFFFFFF, maxprec, pos, words)
    assert pos // 64 == len(k["expected_words"]) - 1  # 8 full words before the flush
    assert [int(x) for x in words[:9]] == [int(x) for x in k["expected_words"]]


def test_known_encode_iblock(orc):
    k = KA["encode_iblock"]
    p = orc.accuracy(k["tolerance"])
    maxprec = orc.lib().orc_precision(k["e"], p.maxprec, p.minexp, 2)
    assert maxprec == k["expected_maxprec"]
    words = np.zeros(8, np.uint64)
    pos = orc.put_bits_header(words, 2 * k["e"] + 1, 9, 0)
    words, pos, bits = orc.encode_iblock(np.array(k["iblock"]), p.minbits, p.maxbits, maxprec, 2, pos, words)
    assert bits == k["expected_iblock_bits"] and pos == 9 + bits
    assert [int(x) for x in words[:2]] == [int(x) for x in k["expected_words"]]


@pytest.mark.parametrize("key", ["integration_3x3", "single_block_4x4"])
def test_known_streams(orc, key):
    k = KA[key]
    w, _ = orc.compress(orc.gen_bump2d(k["n"]), orc.accuracy(1e-3))
    assert [int(x) for x in w] == [int(x) for x in k["expected_words"]]


FX = load_json("libzfp_fixtures.json")


@pytest.fixture(scope="module")
def fxa():
    return np.load(os.path.join(GOLD, "libzfp_fixtures.npz"))


@pytest.mark.parametrize("c", FX["cases"], ids=lambda c: c["name"])
def test_libzfp_fixture(orc, fxa, c):
    a = fxa["input__" + c["input"]]
    p = orc.Params(*c["params"])
    w, bits = orc.compress(a, p)
    assert w.nbytes == c["bytes"]
    assert _sha(w.tobytes()) == c["stream_sha256"]
    d = orc.decompress(fxa[c["name"] + "__stream"], a.shape, p)
    assert _sha(d.tobytes()) == c["decoded_sha256"]


FX4 = load_json("libzfp_fixtures_4d.json")


@pytest.fixture(scope="module")
def fxa4():
    return np.load(os.path.join(GOLD, "libzfp_fixtures_4d.npz"))


@pytest.mark.parametrize("c", FX4["cases"], ids=lambda c: c["name"])
def test_libzfp_fixture_4d(orc, fxa4, c):
    """4-D blocks (perm_4, the w-axis lift, 256-bit planes) against libzfp 0.5.5."""
    a = fxa4["input__" + c["input"]]
    p = orc.Params(*c["params"])
    w, bits = orc.compress(a, p)
    assert w.nbytes == c["bytes"]
    assert _sha(w.tobytes()) == c["stream_sha256"]
    d = orc.decompress(fxa4[c["name"] + "__stream"], a.shape, p)
    assert _sha(d.tobytes()) == c["decoded_sha256"]


def test_reference_sw_build_agrees(orc):
    """oracle/_ref: the reference sw/ compiled in place; 2-D expert-param sweep against the restatement."""
    R = orc.ref()
    if R is None:
        pytest.skip("oracle/_ref not built (reference tree absent)")
    rng = np.random.default_rng(1)
    for shape in [(9, 13), (16, 16), (33, 7)]:
        a = (rng.standard_normal(shape) * 1e-3).astype(np.float32)
        a[0, :3] = [1e-35, np.nan, np.inf]
        for p in [orc.accuracy(1e-3), orc.accuracy(1e-6), orc.rate(8, 2), orc.rate(16, 2), orc.precision(12),
                  orc.expert(20, 90, 20, -30)]:
            w, _ = orc.compress(a, p)
            out = np.zeros(orc.max_words(shape, p) + 4, np.uint64)
            nb = R.gcow_ref_compress_2d(a.ctypes.data_as(C.POINTER(C.c_float)), shape[1], shape[0], *p.tuple(),
                                        out.ctypes.data_as(C.POINTER(C.c_uint64)), out.nbytes)
            assert out.tobytes()[:nb] == w.tobytes(), (shape, p)


def test_threaded_equals_serial(orc):
    a = orc.gen_normal(1 << 15, inject=True)
    for p in [orc.rate(16, 1), orc.accuracy(1e-6), orc.accuracy(1e-3)]:
        w1, b1 = orc.compress(a, p)
        w2, b2 = orc.compress(a, p, threads=5)
        assert b1 == b2 and np.array_equal(w1, w2)


@pytest.mark.parametrize("shape,mode", [((1 << 16) + 3, "acc1e-6"), ((1 << 16) + 3, "rate16"), ((37, 41, 45), "acc1e-3"),
                                        ((37, 41, 45), "rate8"), ((100, 99), "prec20"), ((5,), "acc1e-6")])
def test_threaded_decode_equals_serial(orc, shape, mode):
    """The threaded oracle decode (the full-size GPU decode checks use it) equals the serial decode: variable rate
    from the threaded encode's shard offsets, fixed rate from block positions; more threads than blocks too."""
    shape = shape if isinstance(shape, tuple) else (shape,)
    dims = len(shape)
    p = {"acc1e-6": orc.accuracy(1e-6), "acc1e-3": orc.accuracy(1e-3), "rate16": orc.rate(16, dims),
         "rate8": orc.rate(8, dims), "prec20": orc.precision(20)}[mode]
    a = orc.gen_normal(int(np.prod(shape)), 1e-3, 5, True).reshape(shape)
    w, b = orc.compress(a, p)
    w2, b2, offs = orc.compress(a, p, threads=7, offsets=True)
    assert b2 == b and np.array_equal(w2, w) and int(offs[-1]) == b and int(offs[0]) == 0
    ref = orc.decompress(w, shape, p).view(np.uint32)
    assert np.array_equal(orc.decompress(w, shape, p, threads=7, offsets=offs).view(np.uint32), ref)
    if p.minbits == p.maxbits:
        assert np.array_equal(orc.decompress(w, shape, p, threads=5).view(np.uint32), ref)


def test_block_bits_sum(orc):
    a = orc.gen_normal(4099, inject=True)
    p = orc.accuracy(1e-6)
    bb = orc.block_bits(a, p)
    _, bits = orc.compress(a, p)
    assert int(bb.sum()) == bits


def test_accuracy_bound(orc):
    a = orc.gen_normal(4096, sigma=1.0, inject=False)
    for tol in (1e-1, 1e-3, 1e-6):
        p = orc.accuracy(tol)
        w, _ = orc.compress(a, p)
        d = orc.decompress(w, a.shape, p)
        assert np.max(np.abs(d - a)) <= tol
