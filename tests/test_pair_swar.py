"""CPU check of the byte-parallel (SWAR) stage arithmetic of the pair kernels' upper levels
(polar_sc_pair.h: F4, G4, conv4, ubits4, prow, ppack) and the quad byte transpose of the
channel reads (polar_sc_device.h QuadSel / quad_transpose), restated line for line on numpy uint32
and compared exhaustively with the per-value SM16 definitions the register code uses
(polar_sc_device.h F_sm / G_sm<GSAT> / conv_pair, in turn pinned to the oracle): every pair of
SM8 values and flip flag in every byte position, the other three bytes random, for Q = 6 and 7
(Q = 8 takes the 16-bit path: two magnitudes no longer fit 7 bits)."""
import numpy as np
import pytest

U = np.uint64   # 32-bit arithmetic in uint64 with explicit masking (no wrap warnings)
M32 = 0xFFFFFFFF
B_SGN, B_MAG, B_ONE = 0x80808080, 0x7F7F7F7F, 0x01010101


def consts(Q):
    QMAG = (1 << (Q - 1)) - 1
    GSAT = (1 << (Q - 2)) - 1
    return QMAG, GSAT


# ---- transcription of polar_sc_pair.h ---------------------------------------------------
def sub32(a, b):
    return (a - b) & M32 if np.isscalar(a) else (a.astype(np.int64) - np.asarray(b, np.int64)).astype(U) & U(M32)


def bmask7(t):
    g = t & U(B_SGN)
    return sub32(g, g >> U(7))


def bsel7(m, a, b):
    return (m & a) | (~m & U(M32) & b)


def F4(a, b):
    ma, mb = a & U(B_MAG), b & U(B_MAG)
    ge = bmask7(sub32(ma | U(B_SGN), mb))
    return ((a ^ b) & U(B_SGN)) | bsel7(ge, mb, ma)


def G4(a, b, u, Q):
    _, GSAT = consts(Q)
    SATV = U(GSAT * B_ONE)
    ma, mb, x = a & U(B_MAG), b & U(B_MAG), a ^ b ^ u
    t1, t2 = sub32(ma | U(B_SGN), mb), sub32(mb | U(B_SGN), ma)
    ad = bsel7(bmask7(t1), t1, t2)
    m = bsel7(bmask7(x), ad, (ma + mb) & U(M32))
    m = bsel7(bmask7(sub32(m | U(B_SGN), SATV)), SATV, m)
    return ((b ^ (x & t1)) & U(B_SGN)) | m


def conv4(raw, Q):
    QMAG, _ = consts(Q)
    QM, QP = (1 << Q) - 1, 1 << Q
    t = raw & U(QM * B_ONE)
    v = sub32(U(QP * B_ONE), t)
    mn = bsel7(bmask7(sub32(t | U(B_SGN), v)), v, t)
    return (((t + U((127 - QP // 2) * B_ONE)) & U(M32)) & U(B_SGN)) | (mn & U(QMAG * B_ONE))


def perm(s0, s1, sel):
    """__builtin_amdgcn_perm for selectors 0..7 (bytes of s0:s1) and 12 (zero)."""
    both = (np.asarray(s0, U) << U(32)) | np.asarray(s1, U)
    out = np.zeros_like(both)
    for i in range(4):
        k = (sel >> (8 * i)) & 0xFF
        if k == 12:
            continue
        assert k < 8
        out |= ((both >> U(8 * k)) & U(0xFF)) << U(8 * i)
    return out


def prow(d, odd, Q):
    QMAG, _ = consts(Q)
    return perm(d, d, 0x03030101 if odd else 0x02020000) & U((0x8000 | QMAG) * 0x00010001)


def ppack(v0, v1, Q):
    QMAG, _ = consts(Q)
    t0 = (v0 & U(QMAG * 0x00010001)) | ((v0 >> U(8)) & U(0x00800080))
    t1 = (v1 & U(QMAG * 0x00010001)) | ((v1 >> U(8)) & U(0x00800080))
    return perm(t1, t0, 0x06020400)


def ubits16(d0, d1, q):
    o = U(q & 15)
    lo = (((d0 & U(0xFFFF)) | (d1 << U(16))) & U(M32)) >> o
    hi = ((d0 >> U(16)) | (d1 & U(0xFFFF0000))) >> o
    return (lo & U(0xFFFF)) | ((hi << U(16)) & U(M32))


def ubits4s(d16, k):
    y = ((d16 << U(7 - k)) if k <= 7 else (d16 >> U(k - 7))) & U(0x01800180)
    return (y | (y << U(7))) & U(M32)


def ubits4(d, q):
    y = ((d >> U(q & 15)) & U(0x00030003)) << U(7)
    return (y | (y << U(7))) & U(M32)


# ---- per-value references (one SM8 value, SM16 arithmetic of polar_sc_device.h) -----------
def sm16(b8):
    return ((b8 & 0x80) << 8) | (b8 & 0x7F)


def sm8(v16, QMAG):
    return (v16 & QMAG) | ((v16 >> 8) & 0x80)


def ref_F(a, b, Q):
    QMAG, _ = consts(Q)
    A, B = sm16(a), sm16(b)
    return sm8(np.minimum(A & 0x7FFF, B & 0x7FFF) | ((A ^ B) & 0x8000), QMAG)


def ref_G(a, b, u, Q):
    """G_sm<GSAT> on one 16-bit half (u: flip flag 0 / 1)."""
    QMAG, GSAT = consts(Q)
    A, B = sm16(a).astype(np.int64), sm16(b).astype(np.int64)
    ma, mb = A & 0x7FFF, B & 0x7FFF
    d = (ma - mb) & 0xFFFF
    x = A ^ (u << 15) ^ B
    m = np.where(x & 0x8000, np.abs(ma - mb), ma + mb)
    m = np.minimum(m, GSAT)
    return sm8(((B ^ (x & ~d)) & 0x8000) | m, QMAG)


def ref_conv(raw, Q):
    QMAG, _ = consts(Q)
    QM, QP = (1 << Q) - 1, 1 << Q
    t = raw & QM
    m = np.minimum(t, QP - t) & QMAG
    return np.where(t >= QP // 2 + 1, 0x80, 0) | m


def sm8_values(Q):
    QMAG, _ = consts(Q)
    mags = np.arange(QMAG + 1)
    return np.concatenate([mags, mags | 0x80]).astype(np.int64)


def spread(rng, vals, pos):
    """dwords with `vals` in byte `pos` and random values of the same set elsewhere"""
    out = np.zeros(vals.size, U)
    for k in range(4):
        v = vals if k == pos else rng.permutation(vals)
        out |= v.astype(U) << U(8 * k)
    return out


def byte(d, k):
    return ((d >> U(8 * k)) & U(0xFF)).astype(np.int64)


@pytest.mark.parametrize("Q", [6, 7])
def test_swar_f_g_exhaustive(Q):
    rng = np.random.default_rng(Q)
    v = sm8_values(Q)
    A, B = np.meshgrid(v, v, indexing="ij")
    A, B = A.ravel(), B.ravel()
    for pos in range(4):
        a, b = spread(rng, A, pos), spread(rng, B, pos)
        assert (byte(F4(a, b), pos) == ref_F(A, B, Q)).all(), "F4 byte %d" % pos
        for uflag in (0, 1):
            u = U(0x80 << (8 * pos)) if uflag else U(0)
            # don't-care bits in u (ubits4 leaves some) must not matter
            u = u | U(0x01004000)
            got = byte(G4(a, b, u, Q), pos)
            assert (got == ref_G(A, B, uflag, Q)).all(), "G4 byte %d u %d" % (pos, uflag)


@pytest.mark.parametrize("Q", [6, 7])
def test_swar_conv_exhaustive(Q):
    rng = np.random.default_rng(10 + Q)
    raw = np.arange(256, dtype=np.int64)
    for pos in range(4):
        d = spread(rng, raw, pos)
        assert (byte(conv4(d, Q), pos) == ref_conv(raw, Q)).all(), "conv4 byte %d" % pos


def lane_pos(pl):
    return pl ^ (3 if pl & 4 else 0)   # POLAR_LANE_REMAP


def test_quad_transpose():
    """QuadSel / quad_transpose on a 16-lane row: lane k of a quad holds the four position
    bytes of combination k; afterwards byte c of lane l is combination c at lane_pos(l)."""
    rng = np.random.default_rng(4)
    comb = rng.integers(0, 256, size=(4, 16))          # comb[c][position]
    x = np.zeros(16, np.int64)
    for pl in range(16):
        q, k = pl >> 2, pl & 3
        for b in range(4):
            x[pl] |= int(comb[k][4 * q + b]) << (8 * b)
    def dpp_quad(v, pat):   # quad_perm: lane i of a quad reads lane pat[i]
        return np.array([v[(l & ~3) + pat[l & 3]] for l in range(16)])
    def vperm(s0, s1, sel):
        return np.array([int(perm(U(int(s0[l])), U(int(s1[l])), int(sel[l]))) for l in range(16)])
    s1 = np.zeros(16, np.int64)
    s2 = np.zeros(16, np.int64)
    for pl in range(16):
        k, m = pl & 3, lane_pos(pl) & 3
        s1[pl] = m | ((4 + m) << 8) | ((m ^ 2) << 16) | ((4 + (m ^ 2)) << 24)
        s2[pl] = (0 << (8 * k)) | (1 << (8 * (k ^ 1))) | (6 << (8 * (k ^ 2))) | (7 << (8 * (k ^ 3)))
    t1 = dpp_quad(x, (1, 0, 3, 2))
    y = vperm(t1, x, s1)
    t2 = dpp_quad(y, (2, 3, 0, 1))
    out = vperm(t2, y, s2)
    for pl in range(16):
        for c in range(4):
            assert (out[pl] >> (8 * c)) & 0xFF == comb[c][lane_pos(pl)], (pl, c)


@pytest.mark.parametrize("Q", [6, 7, 8])
def test_slot_row_pack_roundtrip(Q):
    rng = np.random.default_rng(20 + Q)
    v = sm8_values(Q)
    d = np.zeros(4096, U)
    for k in range(4):
        d |= rng.choice(v, 4096).astype(U) << U(8 * k)
    r0, r1 = prow(d, False, Q), prow(d, True, Q)
    # row 2i: bytes 0 (lo frame) and 2 (hi frame); row 2i + 1: bytes 1 and 3 (SM16 halves)
    for r, (bl, bh) in ((r0, (0, 2)), (r1, (1, 3))):
        assert ((r & U(0xFFFF)).astype(np.int64) == sm16(byte(d, bl))).all()
        assert ((r >> U(16)).astype(np.int64) == sm16(byte(d, bh))).all()
    assert (ppack(r0, r1, Q) == d).all()


def test_ubits4():
    rng = np.random.default_rng(3)
    d = rng.integers(0, 1 << 32, 2048, dtype=np.uint64)
    for q in range(0, 16, 2):
        u = ubits4(d, q)
        for bit, src in ((7, q), (15, q + 1), (23, 16 + q), (31, 17 + q)):
            assert (((u >> U(bit)) & U(1)) == ((d >> U(src)) & U(1))).all(), (q, bit)


def test_ubits16_ubits4s():
    """the per-batch partial-sum dword (words q .. q + 15 from two bit dwords) and the flags of
    row pair k of it equal the flags of words q + k, q + k + 1 read directly"""
    rng = np.random.default_rng(4)
    d0 = rng.integers(0, 1 << 32, 512, dtype=np.uint64)
    d1 = rng.integers(0, 1 << 32, 512, dtype=np.uint64)
    for q in range(0, 16, 2):
        d16 = ubits16(d0, d1, q)
        for k in range(0, 16, 2):
            w = q + k   # local word within (d0, d1)
            got = ubits4s(d16, k)
            for bit, word, half in ((7, w, 0), (15, w + 1, 0), (23, w, 16), (31, w + 1, 16)):
                srcd = d0 if word < 16 else d1
                exp = (srcd >> U(half + (word & 15))) & U(1)
                assert (((got >> U(bit)) & U(1)) == exp).all(), (q, k, bit)
