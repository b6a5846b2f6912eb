"""The closed-form block length the variable-rate count passes use (`encode_ints_length` and
`count_block1d_var` in gcow_amd/csrc) restated in Python and checked against the oracle's embedded coder
(encode.c:279-339 restated in oracle/zfp_oracle.c) on random negabinary blocks of 4, 16, 64 and 256 coefficients.
The device code itself is covered by every variable-rate GPU parity test (a wrong length shifts all later blocks)."""
import numpy as np
import pytest


def _lead(v):
    return int(v).bit_length() - 1  # -1 for 0


def length_formula(u, prec):
    """Same backward pass as encode_ints_length<B> (codec_device.h): suffix ORs S_j, z_j = leading zeros of S_j
    (all ones for 0), K = 31 - kmin."""
    B = len(u)
    kmin = 32 - prec if prec < 32 else 0
    if kmin >= 32:
        return 0
    K = 31 - kmin

    def ffbh(v):
        return 0xFFFFFFFF if v == 0 else 32 - int(v).bit_length()

    S = int(u[B - 1])
    on = ffbh(S) <= K
    n = 1 + B * K + (1 if on else 0)
    c = 1 if on else 0
    for j in range(B - 2, -1, -1):
        uj = int(u[j])
        S |= uj
        z = ffbh(S)
        on = z <= K
        n -= min(z, K)
        n += 1 if (on and (uj ^ S) < uj) else 0
        c += 1 if on else 0
    return n + (B - 2 if c == B else c)


def length_b4_integer(u, prec):
    """The 4-coefficient form var1d.hip's v1_prep evaluates without compare-to-mask selects:
    4 + 4 K - sum_{j<3} c_j + sum_{j<3} e_j with c_j = min(z_j, K + 1) and e_j = [c_j <= K] * bit 31 of u_j << c_j
    (the hardware shift takes the count's low 5 bits)."""
    kmin = 32 - prec if prec < 32 else 0
    K = 31 - kmin

    def ffbh(v):
        return 0xFFFFFFFF if v == 0 else 32 - int(v).bit_length()

    S2 = int(u[2]) | int(u[3])
    S1 = int(u[1]) | S2
    S0 = int(u[0]) | S1
    n = 4 + 4 * K
    for uj, S in ((int(u[0]), S0), (int(u[1]), S1), (int(u[2]), S2)):
        c = min(ffbh(S), K + 1)
        n += ((((uj << (c & 31)) & 0xFFFFFFFF) >> 31) & min(K + 1 - c, 1)) - c
    return n


def length_leading_planes(u, prec):
    """The earlier form of the same pass (leading planes L_j and their suffix maxima R_j), kept as a cross-check."""
    B = len(u)
    kmin = 32 - prec if prec < 32 else 0
    last = _lead(u[B - 1])
    n = 32 - max(kmin, last) - B * kmin + max(last, kmin) + (1 if last >= kmin else 0)
    c = 1 if last >= kmin else 0
    rn = last
    for j in range(B - 2, -1, -1):
        lj = _lead(u[j])
        rj = max(lj, rn)
        on = rj >= kmin
        n += max(rj, kmin)
        n += 1 if (on and lj == rj) else 0
        c += 1 if on else 0
        rn = rj
    return n + (B - 2 if c == B else c)


def length_per_plane(u, prec):
    """The unsimplified sum over planes: n_{k+1} verbatim bits plus the group part of plane k."""
    B = len(u)
    kmin = 32 - prec if prec < 32 else 0
    lead = [_lead(v) for v in u]
    total, n = 0, 0
    for k in range(31, kmin - 1, -1):
        nk = max([j + 1 for j in range(B) if lead[j] >= k], default=0)
        total += n
        if n < B:
            if nk == n:
                total += 1
            else:
                m = sum(1 for j in range(n, B) if lead[j] == k)
                q = nk - 1
                total += m + (B - 1 if q == B - 1 else q + 2) - n
        n = nk
    return total


def _blocks(rng, size, count):
    for _ in range(count):
        decay = rng.random() * 1.5  # magnitude falling with coefficient index, as after the decorrelating lift
        sh = np.minimum(32, (rng.integers(0, 8, size) + decay * np.arange(size)).astype(int))
        u = np.array([(int(rng.integers(0, 2 ** 32)) >> int(s)) if s < 32 else 0 for s in sh], dtype=np.uint32)
        if rng.random() < 0.3:
            rng.shuffle(u)
        if rng.random() < 0.1:
            u[:] = 0
        yield u, int(rng.integers(1, 33))


@pytest.mark.parametrize("size", [4, 16, 64, 256])
def test_length_formula_matches_coder(orc, size):
    rng = np.random.default_rng(0x67636F77 + size)
    words = np.zeros(256 * 33 // 64 + 64, dtype=np.uint64)  # room for the longest untruncated 256-value block
    for u, prec in _blocks(rng, size, 1500 if size <= 64 else 300):
        words[:] = 0
        _, _, bits = orc.encode_ints(u, 1 << 30, prec, words=words)
        assert length_formula(u, prec) == bits, (u.tolist(), prec)
        assert length_per_plane(u, prec) == bits, (u.tolist(), prec)
        assert length_leading_planes(u, prec) == bits, (u.tolist(), prec)
        if size == 4:
            assert length_b4_integer(u, prec) == bits, (u.tolist(), prec)


def test_length_formula_extremes(orc):
    words = np.zeros(256, dtype=np.uint64)
    for size in (4, 16, 64):
        for u in (np.zeros(size, np.uint32), np.full(size, 0xFFFFFFFF, np.uint32),
                  np.eye(1, size, size - 1, dtype=np.uint32)[0] * 0x80000000,
                  np.eye(1, size, 0, dtype=np.uint32)[0]):
            for prec in (1, 2, 16, 31, 32):
                words[:] = 0
                _, _, bits = orc.encode_ints(u, 1 << 30, prec, words=words)
                assert length_formula(u, prec) == bits
                if size == 4:
                    assert length_b4_integer(u, prec) == bits
