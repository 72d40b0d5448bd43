"""Exhaustive / property tests of the oracle's fixed-point primitives.

Each primitive of oracle/polar_oracle.c (a bit-width-exact restatement of the SystemC
source) is checked against an independent closed-form restatement of the same
reference text, over the whole input range that the hot path uses.
Reference citations are in polar_oracle.c.
"""
import itertools

import numpy as np
import pytest

import util


def sm(v, q=6):
    """int -> Q-bit SM pattern; v may be '-0' encoded as ('-', 0)."""
    if isinstance(v, tuple):
        return (1 << (q - 1)) | v[1]
    return ((1 << (q - 1)) if v < 0 else 0) | abs(v)


def all_sm(q=6):
    return list(range(1 << q))   # every Q-bit pattern incl. -0


def dec(p, q):
    return (p >> (q - 1)) & 1, p & ((1 << (q - 1)) - 1)


def test_qconv_format_all_6bit(oracle_mod):
    L = oracle_mod.lib()
    for c in range(-32, 32):
        p = c & 63
        got = L.orc_qconv_format(6, p)
        if c == -32:
            exp = 0                      # -32 -> +0 (no 6-bit SM encoding of 32)
        elif c < 0:
            exp = 32 | (-c)
        else:
            exp = c
        assert got == exp, (c, got, exp)


def test_F_exhaustive(oracle_mod):
    L = oracle_mod.lib()
    for a, b in itertools.product(all_sm(), repeat=2):
        sa, ma = dec(a, 6)
        sb, mb = dec(b, 6)
        assert L.orc_F_sm(6, a, b) == (((sa ^ sb) << 5) | min(ma, mb))


@pytest.mark.parametrize("q", [6, 7, 8])
def test_Gext_exhaustive(oracle_mod, q):
    L = oracle_mod.lib()
    for a, b in itertools.product(all_sm(q), repeat=2):
        sa, ma = dec(a, q)
        sb, mb = dec(b, q)
        for u in (0, 1):
            sa2 = sa ^ u
            m = ma + mb if sa2 == sb else abs(ma - mb)
            s = sb if ma < mb else sa2
            assert L.orc_Gext_sm(q, a, b, u) == ((s << q) | m), (q, a, b, u)


def test_G_saturates_at_15(oracle_mod):
    L = oracle_mod.lib()
    for a, b in itertools.product(all_sm(), repeat=2):
        sa, ma = dec(a, 6)
        sb, mb = dec(b, 6)
        for u in (0, 1):
            sa2 = sa ^ u
            m = ma + mb if sa2 == sb else abs(ma - mb)
            s = sb if ma < mb else sa2
            assert L.orc_G_sm(6, a, b, u) == ((s << 5) | min(m, 15))


def test_signed_zero_decides_one():
    # hard(-0) = 1 : a tie |a| == |b| with opposite signs yields magnitude 0 and sign(a')
    s, m = util.G((np.array([1]), np.array([5])), (np.array([0]), np.array([5])), 0)
    assert (int(s[0]), int(m[0])) == (1, 0)


def test_full_adder_sat_clamps_511(oracle_mod):
    L = oracle_mod.lib()
    q = 11
    for ma in (0, 1, 255, 496, 511):
        for mb in (0, 15, 255, 511):
            for sa, sb in itertools.product((0, 1), repeat=2):
                a, b = (sa << 10) | ma, (sb << 10) | mb
                m = ma + mb if sa == sb else abs(ma - mb)
                s = sb if ma < mb else sa
                assert L.orc_full_adder_sat_sm(q, a, b) == ((s << 10) | min(m, 511))


def _np_leaf(vals, fb):
    s = np.array([[(v >> 5) & 1 for v in vals]])
    m = np.array([[v & 31 for v in vals]])
    x = util.leaf((s, m), fb)[0]
    return sum(int(b) << i for i, b in enumerate(x))


def test_leaf16_matches_recursive_restatement(oracle_mod):
    rng = np.random.default_rng(16)
    for t in range(3000):
        if t % 3 == 0:
            vals = rng.integers(0, 64, 16)
        elif t % 3 == 1:
            vals = rng.choice([0, 1, 32, 33, 31, 63], 16)      # zero-heavy / -0 / saturated
        else:
            vals = rng.integers(0, 4, 16) | (rng.integers(0, 2, 16) << 5)
        fb = int(rng.integers(0, 1 << 16)) if t % 5 else int(rng.choice([0, 0xFFFF, 0x8000, 0xFFFE, 0xFF00, 0x00FF]))
        assert oracle_mod.leaf16(vals, fb) == _np_leaf(vals, fb), (list(vals), hex(fb))


def test_leaf16_noiseless_is_codeword(oracle_mod):
    rng = np.random.default_rng(3)
    for _ in range(500):
        fb = int(rng.integers(0, 1 << 16))
        u = rng.integers(0, 2, 16) & np.array([(fb >> k) & 1 for k in range(16)])
        x = util.encode_np(u[None, :])[0]
        vals = [sm(-31) if b else sm(31) for b in x]
        assert oracle_mod.leaf16(vals, fb) == sum(int(b) << i for i, b in enumerate(x))


def test_rep_add_tree_pairing_and_order(oracle_mod):
    rng = np.random.default_rng(4)
    for _ in range(2000):
        vals = rng.integers(0, 64, 16)
        old = int(rng.integers(0, 1 << 11))
        s = np.array([[(v >> 5) & 1 for v in vals]])
        m = np.array([[v & 31 for v in vals]])
        ts, tm = util.rep_tree((s, m))
        acc = util.G((ts, tm), (np.array([(old >> 10) & 1]), np.array([old & 1023])), 0, 511)
        exp = (int(acc[0][0]) << 10) | int(acc[1][0])
        assert oracle_mod.rep_add_tree16(vals, old) == exp


def test_min_mask_tie_rule_is_bitrev(oracle_mod):
    bitrev = [int("{:04b}".format(i)[::-1], 2) for i in range(16)]
    rng = np.random.default_rng(5)
    for _ in range(3000):
        mags = rng.integers(0, 4, 16)          # many ties
        r = oracle_mod.min_mask16(mags.astype(np.uint32))
        mn, mask = r >> 16, r & 0xFFFF
        assert mn == mags.min()
        cands = [l for l in range(16) if mags[l] == mn]
        win = min(cands, key=lambda l: bitrev[l])
        assert mask == 1 << win, (list(mags), hex(mask), win)


def test_group_classification(oracle_mod):
    L = oracle_mod.lib()
    assert L.orc_classify_group(0) == 0x00
    assert L.orc_classify_group(0xFFFF) == 0x0F
    assert L.orc_classify_group(0x8000) == 0x02
    assert L.orc_classify_group(0xFFFE) == 0x04
    for fb in (0x0001, 0x7FFF, 0xC000, 0xFFFC, 0x1234):
        assert L.orc_classify_group(fb) == 0x08


def _sm8_of_byte(b):
    """Mirror of polar::sm8_of_byte (csrc/polar_sc_device.h): the per-mask kernels' LDS table."""
    t = b & 63
    m = min(t, 64 - t) & 31
    return (0x80 if t >= 33 else 0) | m


def _sm8_pair(lo, hi):
    """Mirror of polar::sm8_pair: v_perm duplicates each byte into its half, then & 0x801F801F."""
    x = (lo & 0xFF) | ((lo & 0xFF) << 8) | ((hi & 0xFF) << 16) | ((hi & 0xFF) << 24)
    return x & 0x801F801F


def _conv_pair(raw):
    """Mirror of polar::conv_pair (schedule interpreter, Ctx::chan)."""
    out = 0
    for h in (0, 16):
        t = (raw >> h) & 0x3F
        m = min(t, (0x40 - t) & 0xFFFF) & 0x1F
        s = (t + 0x7FDF) & 0x8000
        out |= (m | s) << h
    return out


def test_device_channel_conversions_match_qconv_all_bytes(oracle_mod):
    """Every int8 channel byte (the reference keeps the low 6 bits, sc_bigint<6>) converts to
    the SM value of qconv_format (scalar.h:229-239) under both device formulas."""
    L = oracle_mod.lib()
    for b in range(256):
        q = L.orc_qconv_format(6, b & 63)          # 6-bit SM: bit 5 sign, bits 0..4 magnitude
        exp16 = ((q >> 5) << 15) | (q & 31)
        got = _sm8_pair(_sm8_of_byte(b), _sm8_of_byte(255 - b))
        assert got & 0xFFFF == exp16, b
        q2 = L.orc_qconv_format(6, (255 - b) & 63)
        assert got >> 16 == ((q2 >> 5) << 15) | (q2 & 31), b
        assert _conv_pair(b | ((255 - b) << 16)) == got, b
