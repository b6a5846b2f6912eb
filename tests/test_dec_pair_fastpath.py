"""Host emulation of the fixed-rate 1-D two-plane decoder's fast path (gcow_kernels.hip decode_block1d_pair, 64-bit
blocks), both step forms (GCOW_DEC_PAIR2 = 1: select-free steps; 0: the budget- and window-guarded steps), against
the oracle's decode of the same blocks (oracle/zfp_oracle.c, libzfp decode_ints semantics, sw/src/decode.c:141-183
with the block-size fix). The claim checked: every block the fast path does not flag special decodes bit-exactly, on
encoder output (the C2 distribution, wide-range and sparse blocks) and on arbitrary 64-bit words (nonzero padding,
long group phases, plane codes crossing the budget)."""
import numpy as np
import pytest

M64 = (1 << 64) - 1
NB = 0xAAAAAAAA


def dec_plane_cx(t):  # gcow_kernels.hip dec_plane_cx: (n, budget bits - 1, 7 stream bits) -> nibble | len << 4 | n' << 8
    n0, r, b = t >> 10, (t >> 7) & 7, t & 127
    n, bits = n0, r + 1
    if n >= 4:
        m = min(bits, 4)
        return (b & ((1 << m) - 1)) | (m << 4) | (4 << 8)
    m = min(n, bits)
    x, pos = b & ((1 << m) - 1), m
    bits -= m
    while n < 4 and bits:
        bits -= 1
        g = (b >> pos) & 1
        pos += 1
        if not g:
            break
        while n < 3 and bits:
            bits -= 1
            one = (b >> pos) & 1
            pos += 1
            if one:
                break
            n += 1
        x += 1 << n
        n += 1
    return x | (pos << 4) | (n << 8)


def dec_pair_cx(t):  # gcow_kernels.hip dec_pair_cx
    n, b = t >> 10, t & 1023
    e1 = dec_plane_cx((((n << 3) | 7) << 7) | (b & 127))
    x1, l1, n1 = e1 & 15, (e1 >> 4) & 15, e1 >> 8
    e2 = dec_plane_cx((((n1 << 3) | 7) << 7) | ((b >> l1) & 127))
    x2, l2, n2 = e2 & 15, (e2 >> 4) & 15, e2 >> 8
    r1, r2 = min(n1, 3), min(n2, 3)
    if l1 + l2 <= 10:
        return x1 | (x2 << 4) | (l1 << 8) | ((l1 + l2) << 12) | (r1 << 16) | (r2 << 18) | (1 << 20)
    return x1 | (l1 << 8) | (l1 << 12) | (r1 << 16) | (r1 << 18)


TAB = [dec_pair_cx(t) for t in range(3 * 1024)]


def bitrev32(v):
    return int("{:032b}".format(v)[::-1], 2)


def window_to_coeffs(Y, top, u):
    for i in range(4):
        field = 0
        for j in range(16):
            field |= ((Y >> (4 * j + i)) & 1) << j
        u[i] |= bitrev32(field) >> (31 - top)


def gather_tab():  # gcow_kernels.hip make_gather_tab
    T = [0] * 1024
    for s in range(4):
        for b in range(256):
            r = 0
            for i in range(4):
                r |= ((b >> i) & 1) << (8 * i + 7 - 2 * s)
                r |= ((b >> (4 + i)) & 1) << (8 * i + 6 - 2 * s)
            T[256 * s + b] = r
    return T


GT = gather_tab()


def perm_b32(s0, s1, sel):  # v_perm_b32 for selector bytes 0..7 and 0x0c (zero)
    src = [(s1 >> (8 * k)) & 255 for k in range(4)] + [(s0 >> (8 * k)) & 255 for k in range(4)]
    out = 0
    for k in range(4):
        c = (sel >> (8 * k)) & 255
        out |= (src[c] if c < 8 else 0) << (8 * k)
    return out


def window_to_coeffs_lds(Y, top, u):  # gcow_kernels.hip window_to_coeffs_lds
    lo, hi = Y & 0xFFFFFFFF, Y >> 32
    A = GT[lo & 255] | GT[256 + ((lo >> 8) & 255)] | GT[512 + ((lo >> 16) & 255)] | GT[768 + (lo >> 24)]
    B = GT[hi & 255] | GT[256 + ((hi >> 8) & 255)] | GT[512 + ((hi >> 16) & 255)] | GT[768 + (hi >> 24)]
    for i in range(4):
        u[i] |= perm_b32(A, B, ((4 + i) << 24) | (i << 16) | 0x0C0C) >> (31 - top)


def test_gather_window_matches_transpose():
    rng = np.random.default_rng(9)
    for _ in range(3000):
        Y = int(rng.integers(0, 2 ** 63)) * 2 + int(rng.integers(0, 2))
        top = int(rng.integers(0, 32))
        a, b = [0] * 4, [0] * 4
        window_to_coeffs(Y, top, a)
        window_to_coeffs_lds(Y, top, b)
        assert a == b, (hex(Y), top, a, b)


def i32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >> 31 else v


def inv_lift(x, y, z, w):  # codec_device.h inv_lift (int32 wraparound)
    y = i32(y + (w >> 1)); w = i32(w - (y >> 1))
    y = i32(y + w); w = i32(w << 1); w = i32(w - y)
    z = i32(z + x); x = i32(x << 1); x = i32(x - z)
    y = i32(y + z); z = i32(z << 1); z = i32(z - y)
    w = i32(w + x); x = i32(x << 1); x = i32(x - w)
    return x, y, z, w


def dequant_scale(emax):
    e = emax - 30
    if e >= -126:
        return np.uint32((e + 127) << 23).view(np.float32)
    if e >= -149:
        return np.uint32(1 << (e + 149)).view(np.float32)
    return np.float32(0.0)


def fast_pair(w, new):
    """decode_block1d_pair's fast path for one 64-bit block: (special, 4 float32 bit patterns)."""
    nonzero = w & 1
    emax = ((w >> 1) & 255) - 127
    r = (w >> 9) if (nonzero or not new) else 0  # pair2: a zero header bit is a block of empty planes
    z = (r & -r).bit_length() - 1 if r else 64
    M0 = 31 - z
    pos, Y, n, j = 9 + z, 0, 0, 0
    if new:
        jm = min(M0, 15)
        for it in range(16):
            if not ((M0 >= 0) if it == 0 else (n < 3 and pos < 64 and j <= jm)):
                break
            e = TAB[(n << 10) | ((w >> pos) & 1023)]
            Y = (Y | ((e & 255) << (4 * j))) & M64
            pos += (e >> 12) & 15
            n = (e >> 18) & 3
            j += 1 + ((e >> 20) & 1)
        special = M0 >= 0 and (pos > 64 or j >= 16)
    else:
        cross = False
        for _ in range(16):
            rem = 64 - min(pos, 64)
            if not (n < 3 and rem and j <= M0 and j < 16 and not cross):
                break
            e = TAB[(n << 10) | ((w >> pos) & 1023)]
            l1, l2 = (e >> 8) & 15, (e >> 12) & 15
            cross = l1 > rem
            two = bool((e >> 20) & 1) and l2 <= rem and j < M0 and j < 15
            if not cross:
                Y = (Y | (((e & 255) if two else (e & 15)) << (4 * j))) & M64
                pos += l2 if two else l1
                n = (e >> (18 if two else 16)) & 3
                j += 2 if two else 1
        special = cross or (n < 3 and pos < 64 and j <= M0)
    if new:  # unconditional: 0 at pos = 64; lanes with pos > 64 or j >= 16 are special
        Y = (Y | ((((w >> (pos - 1)) >> 1) << (4 * (j & 15))) & M64)) & M64 if j < 16 else Y
    elif j < 16 and pos < 64:
        Y = (Y | ((w >> pos) << (4 * j))) & M64
    u = [0, 0, 0, 0]
    if M0 >= 0:
        window_to_coeffs(Y, M0, u)
        p2 = pos + 4 * (16 - min(j, 16))
        if p2 < 64 and M0 >= 16:
            window_to_coeffs(w >> p2, M0 - 16, u)
    q = [i32((v ^ NB) - NB) for v in u]
    q = inv_lift(*q)
    sc = dequant_scale(emax)
    if new:  # q = 0 for a zero header bit; one ldexp per value, exponents under -149 as -256 (a signed zero)
        e = emax - 30 if emax - 30 >= -149 else -256
        f = np.array([np.ldexp(np.float32(v), e) for v in q], np.float32)
    else:
        f = np.array([sc * np.float32(v) if nonzero else np.float32(0.0) for v in q], np.float32)
    return special, f.view(np.uint32)


def _blocks(orc):
    rng = np.random.default_rng(5)
    vals = [orc.gen_normal(4 * 6000, seed=11)]                              # the C2 distribution (zeros, tiny, subnormal)
    wide = rng.standard_normal(4 * 3000).astype(np.float32)
    wide *= np.float32(2.0) ** rng.integers(-40, 40, wide.size).astype(np.float32)  # long group phases
    vals.append(wide)
    sparse = np.zeros(4 * 2000, np.float32)
    sparse[rng.integers(0, sparse.size, 1500)] = rng.standard_normal(1500).astype(np.float32)
    vals.append(sparse)
    small = rng.standard_normal(4 * 1500).astype(np.float32)
    small *= np.float32(2.0) ** rng.integers(-128, -100, small.size).astype(np.float32)  # scales 2^-158 .. 2^-130
    vals.append(small)
    a = np.concatenate(vals)
    words, _ = orc.compress(a, orc.rate(16, 1))
    arb = rng.integers(0, 2 ** 63, 4000, dtype=np.int64).astype(np.uint64) * np.uint64(2) + \
        rng.integers(0, 2, 4000, dtype=np.int64).astype(np.uint64)      # arbitrary words: nonzero padding, any codes
    # adversarial words: a header, z empty planes, then sparse bits (long zero runs: group phases that run past the
    # 16-plane window or across the 64-bit budget, steps from nibble 15, blocks with M0 < 16)
    adv = []
    for _ in range(6000):
        z = int(rng.integers(0, 55))
        hdr = int(rng.integers(0, 512)) | 1
        tail = 0
        for k in range(9 + z + 1, 64):
            if rng.random() < 0.12:
                tail |= 1 << k
        adv.append(hdr | (1 << (9 + z)) | tail)
    return np.concatenate([words[: a.size // 4], arb, np.array(adv, np.uint64)])


@pytest.mark.parametrize("new", [True, False], ids=["pair2", "pair"])
def test_fast_path_matches_oracle(orc, new):
    words = _blocks(orc)
    ref = orc.decompress(np.concatenate([words, np.zeros(2, np.uint64)]), (4 * words.size,), orc.rate(16, 1))
    ref = ref.view(np.uint32).reshape(-1, 4)
    nspecial = 0
    for b, w in enumerate(words.tolist()):
        special, f = fast_pair(int(w), new)
        if special:
            nspecial += 1
            continue
        assert np.array_equal(f, ref[b]), (b, hex(int(w)), f, ref[b])
    assert 0 < nspecial < words.size // 4  # the fast path takes most blocks; the adversarial words reach the special cases
