"""Host emulation of the variable-rate lean block decoder's group phase (gcow_kernels.hip dec_block1d_lean): the
plane-table form (one (n, 7 bits) lookup per plane) and the pair-table form (PAIR: 16-bit DecTabLP entries, up to two
planes per (n, 10 bits) lookup, the plane table for a step that may take one plane only), each against a plain
plane-by-plane decode of the same bits (libzfp decode_ints semantics without a budget, sw/src/decode.c:141-183). The
claims checked: both forms send the same blocks to the general decoder, and on every other block they give the same
nibble of every coded plane and the same block length."""
import random

import pytest

from test_dec_pair_fastpath import dec_pair_cx, dec_plane_cx

M64 = (1 << 64) - 1


def lean_pair_tab():  # gcow_kernels.hip make_dec_lean_pair
    t16 = []
    for t in range(3 * 1024):
        e = dec_pair_cx(t)
        t16.append((e & 255) | (((e >> 12) & 15) << 8) | (((e >> 18) & 3) << 12) | (((e >> 20) & 1) << 14))
    t7 = [dec_plane_cx(((((t >> 7) << 3) | 7) << 7) | (t & 127)) for t in range(5 * 128)]
    return t16 + t7


LP = lean_pair_tab()


def plane_by_plane(bits, nbelow):
    """Every coded plane through the no-budget plane table: -> (nibbles, length in bits)."""
    pos, n, nib = 0, 0, []
    for _ in range(nbelow):
        e = dec_plane_cx((((min(n, 4) << 3) | 7) << 7) | ((bits >> pos) & 127))
        nib.append(e & 15)
        pos += (e >> 4) & 15
        n = e >> 8
    return nib, pos


def lean(bits, nbelow, pair):
    """dec_block1d_lean's group phase + verbatim run over `bits` (the stream from the first coded plane on); the
    window is re-read as the kernel does. -> (nibbles, length) or None (left to the general decoder)."""
    wbase, off, n, G, j = 0, 0, 0, 0, 0
    gw = bits & M64
    if pair:
        lim = min(nbelow, 8)
        while n < 3 and j < lim:
            if off > 54:
                wbase += off
                gw = (bits >> wbase) & M64
                off = 0
            b = (gw >> off) & 1023
            e = LP[(n << 10) | b]
            nib, ln, nn, two = e & 255, (e >> 8) & 15, (e >> 12) & 3, e >> 14
            if two and j + 1 >= lim:
                e7 = LP[3 * 1024 + ((n << 7) | (b & 127))]
                nib, ln, nn, two = e7 & 15, (e7 >> 4) & 15, e7 >> 8, 0
            G |= nib << (4 * j)
            off += ln
            n = nn
            j += 1 + two
    else:
        while n < 3 and j < nbelow and j < 8:
            if off > 57:
                wbase += off
                gw = (bits >> wbase) & M64
                off = 0
            e = LP[3 * 1024 + ((n << 7) | ((gw >> off) & 127))]
            G |= (e & 15) << (4 * j)
            off += (e >> 4) & 15
            n = e >> 8
            j += 1
    if n < 3 and j < nbelow:
        return None
    assert G < 1 << 32 and j <= 8
    vpos = wbase + off
    t = nbelow - j
    nib = [(G >> (4 * k)) & 15 for k in range(j)] + [(bits >> (vpos + 4 * k)) & 15 for k in range(t)]
    return nib, vpos + 4 * t


def _streams(seed, count):
    rng = random.Random(seed)
    for _ in range(count):
        p1 = rng.choice([0.05, 0.2, 0.5, 0.8, 0.95])
        bits = 0
        for k in range(200):
            bits |= int(rng.random() < p1) << k
        yield bits, rng.randint(1, 32)


@pytest.mark.parametrize("seed", range(4))
def test_lean_pair_matches_plane_by_plane(seed):
    general = 0
    for bits, nbelow in _streams(seed, 3000):
        want = plane_by_plane(bits, nbelow)
        one = lean(bits, nbelow, False)
        two = lean(bits, nbelow, True)
        assert (one is None) == (two is None), (hex(bits), nbelow)
        if one is None:
            general += 1
            continue
        assert one == want, (hex(bits), nbelow)
        assert two == want, (hex(bits), nbelow)
    assert general < 3000


def test_lean_pair_exhaustive_short_blocks():
    # every 12-bit prefix (then ones or zeros) with 1..10 coded planes: all steps that may take one plane only
    for fill in (0, (1 << 200) - 1):
        for pre in range(1 << 12):
            bits = pre | ((fill >> 12) << 12)
            for nbelow in range(1, 11):
                want = plane_by_plane(bits, nbelow)
                got = lean(bits, nbelow, True)
                assert (got is None) == (lean(bits, nbelow, False) is None)
                if got is not None:
                    assert got == want, (hex(bits), nbelow)
