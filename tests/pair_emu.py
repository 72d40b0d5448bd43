"""CPU emulation of the pair kernels (test infrastructure).

The generated subtree decoders of a pair plan (polar_sc_pairgen.cpp, Decoder.kernel_source())
are transpiled to Python and run on 64-lane numpy vectors with the same cross-lane semantics
as the device (DPP row exchanges with POLAR_LANE_REMAP, v_permlane16/32_swap); the upper-level
ops of the plan (polar_sc_pair.h pop_*) are restated on the same layout. The emulated decode
must equal the oracle bit for bit, which pins the generator and the frame-pair layout without
a GPU; tests/test_pair.py then checks the device against the oracle.

Values: every u32 register is a uint32 array of 64 lanes; lane = 16 row + pl."""
import re

import numpy as np

U32 = np.uint32
LANE = np.arange(64, dtype=np.int64)
SGN, MAG = 0x80008000, 0x7FFF7FFF
# the datapath format of the emulated source (configure): LLR_BITS, CA2, EXTENDED, log2 PAR
# (PAR 16; PAR 4 / 8 in SIGMAG: the PAR words as lane groups of a device word)
QB, CA2, EXT, WIDE, LPAR = 6, False, True, False, 4
QMAG = GSAT = REPSAT = GSAT2 = VMAG = 0
PARW, PPW = 16, 1


def configure(q=6, ca2=False, ext=True, lpar=4):
    """polar_sc_device.h's format constants for LLR_BITS q, CA2 / SIGMAG, EXTENDED, PAR 2^lpar"""
    global QB, CA2, EXT, WIDE, QMAG, GSAT, REPSAT, GSAT2, VMAG, LPAR, PARW, PPW
    QB, CA2, EXT, LPAR = q, bool(ca2), bool(ext), lpar
    if LPAR < 4 and CA2:
        raise NotImplementedError("pair_emu: CA2 at PAR 4 / 8 (the two's complement word trees) is GPU-tested only")
    PARW, PPW = (1 << LPAR if LPAR < 4 else 16), (16 >> LPAR if LPAR < 4 else 1)
    WIDE = QB > 8 or (CA2 and QB > 7)   # 16-bit slot rows (polar_sc_pair.h POLAR_PAIR_S16)
    QMAG = (1 << (QB - 1)) - 1
    GSAT = (1 << (QB - 1)) - 1 if CA2 else (1 << (QB - 2)) - 1
    REPSAT = (1 << (QB + LPAR)) - 1 if CA2 else (1 << (QB + LPAR - 1)) - 1
    GSAT2 = GSAT * 0x00010001
    VMAG = (1 << QB) - 1 if CA2 else QMAG


def configure_from(src):
    """configure() from the #defines of a generated source"""
    m = re.search(r"#define POLAR_Q (\d+)", src)
    lp = re.search(r"#define POLAR_LPAR (\d+)", src)
    lpar = int(lp.group(1)) if lp else 4
    if lpar > 4:
        raise NotImplementedError("pair_emu: PAR 32 / 64 (the PAR words across rows) is GPU-tested only")
    configure(int(m.group(1)) if m else 6, "#define POLAR_CA2 1" in src, "#define POLAR_EXT 0" not in src, lpar)


configure()


def V(x):
    a = np.asarray(x)
    if a.dtype == np.bool_:
        return a
    if a.ndim == 0:
        return np.full(64, int(a) & 0xFFFFFFFF, dtype=U32)
    return a.astype(np.int64).astype(U32) if a.dtype != U32 else a


def lo(x):
    return V(x).astype(np.int64) & 0xFFFF


def hi(x):
    return V(x).astype(np.int64) >> 16


def pk(l, h):
    return ((np.asarray(l, np.int64) & 0xFFFF) | ((np.asarray(h, np.int64) & 0xFFFF) << 16)).astype(U32)


def s16(x):
    x = np.asarray(x, np.int64) & 0xFFFF
    return np.where(x >= 0x8000, x - 0x10000, x)


def pk_min(a, b):
    return pk(np.minimum(lo(a), lo(b)), np.minimum(hi(a), hi(b)))


def pk_max_u16(a, b):
    return pk(np.maximum(lo(a), lo(b)), np.maximum(hi(a), hi(b)))


def pk_add(a, b):
    return pk(lo(a) + lo(b), hi(a) + hi(b))


def pk_sub(a, b):
    return pk(lo(a) - lo(b), hi(a) - hi(b))


def pk_mad_u16(a, b, c):
    return pk(lo(a) * lo(b) + lo(c), hi(a) * hi(b) + hi(c))


def pk_mul_lo(a, b):
    return pk(lo(a) * lo(b), hi(a) * hi(b))


def pk_sra(a, s):
    return pk(s16(lo(a)) >> s, s16(hi(a)) >> s)


def pk_shl(a, s):
    return pk(lo(a) << s, hi(a) << s)


def pk_abs_i16(a):
    return pk(np.maximum(s16(lo(a)), s16(-s16(lo(a)))), np.maximum(s16(hi(a)), s16(-s16(hi(a)))))


def bsel(m, a, b):
    m, a, b = V(m), V(a), V(b)
    return (a & m) | (b & ~m)


def opaque(x):
    return V(x)


def sel(c, a, b):
    return np.where(np.asarray(c, bool), V(a), V(b)).astype(U32)


def land(a, b):
    return np.logical_and(np.asarray(a) != 0, np.asarray(b) != 0)


def row_even(row):
    return sel((V(row) & 1) == 0, 0xFFFFFFFF, 0)


def row_lo2(row):
    return sel(V(row) < 2, 0xFFFFFFFF, 0)


def F_sm(a, b):
    a, b = V(a), V(b)
    return pk_min(a & MAG, b & MAG) | ((a ^ b) & SGN)


def G_sm(SAT, a, b, u):
    a, b, u = V(a), V(b), V(u)
    ma, mb = a & MAG, b & MAG
    d = pk_sub(ma, mb)
    x = a ^ u ^ b
    m = bsel(pk_sra(x, 15), pk_abs_i16(d), pk_add(ma, mb))
    if SAT:
        m = pk_min(m, SAT * 0x00010001)
    return ((b ^ (x & ~d)) & SGN) | m


# ---- lanes ----------------------------------------------------------------------------
def lane_pos(pl):
    pl = np.asarray(pl, np.int64)
    return pl ^ np.where(pl & 4, 3, 0)


def xorlane_phys(H, v):
    return V(v)[LANE ^ H]


def xorlane(H, v):
    if H == 4:
        return V(v)[LANE ^ 7]        # row_half_mirror (the remapped lane order)
    return xorlane_phys(H, v)


class Lanes:
    def __init__(self):
        self.pl = (LANE & 15).astype(U32)
        self.pos = lane_pos(LANE & 15).astype(U32)
        p = self.pos.astype(np.int64)
        self.br = (((p & 1) << 3) | ((p & 2) << 1) | ((p & 4) >> 1) | ((p & 8) >> 3)).astype(U32)
        self.a = {h: np.where(p & h, 0, 0xFFFFFFFF).astype(U32) for h in (1, 2, 4, 8)}


def plane_mask(I, p):
    return pk_sra(pk_shl(p, 15 - I), 15)


def plane_put(I, acc, v):
    return ((V(v) >> (15 - I)) & (0x00010001 << I)) | V(acc)


def F_root(I, a, b, S):
    return pk_min(V(a) & MAG, V(b) & MAG), plane_put(I, S, V(a) ^ V(b))


def G_root(I, a, b, u, S):
    a, b, u = V(a), V(b), V(u)
    ma, mb = a & MAG, b & MAG
    d = pk_sub(ma, mb)
    x = a ^ u ^ b
    S = plane_put(I, S, b ^ (x & ~d))
    return pk_min(bsel(pk_sra(x, 15), pk_abs_i16(d), pk_add(ma, mb)), GSAT2), S


def G_split(I, ma, mb, X, LT):
    xm = plane_mask(I, X)
    d = pk_sub(ma, mb)
    LT = plane_put(I, LT, d)
    return pk_min(bsel(xm, pk_abs_i16(d), pk_add(ma, mb)), GSAT2), LT


# ---- CA2 on split words (polar_sc_device.h): a zero's sign is don't-care, MIN of width w is
# magnitude 2^(w-1) with the sign set; F ops that can meet it take the key min
def ca2_nzs(M, S):
    return pk_mul_lo(pk_min(M, 0x00010001), S)


def ca2_nz(m):
    return pk_sub(0, V(m) & MAG)


def pk_min_key(MW, a, b):
    K2 = (1 << (MW - 1)) * 0x00010001
    return V(pk_min(V(a) ^ K2, V(b) ^ K2)) ^ K2


def ca2_minbit(MW, m):
    return pk_add(m, (0x8000 - (1 << (MW - 1))) * 0x00010001)


def F_ca2(MW, a, b):
    a, b = V(a), V(b)
    m = pk_min_key(MW, a & MAG, b & MAG)
    return m | (((a ^ b) | ca2_minbit(MW, m)) & SGN)


def F_root_min(I, MW, a, b, S):
    a, b = V(a), V(b)
    m = pk_min_key(MW, a & MAG, b & MAG)
    return m, plane_put(I, S, (a ^ b) | ca2_minbit(MW, m))


def F_split_min(I, MW, ma, mb, MP):
    m = pk_min_key(MW, ma, mb)
    return m, plane_put(I, MP, ca2_minbit(MW, m))


def F_split_biased_min(I, MW, ma, mb, FS):
    m = pk_min_key(MW, ma, mb)
    s = V(plane_mask(I, FS)) | pk_sra(ca2_minbit(MW, m), 15)
    return pk_add(pk_sub(m ^ s, s), 0x02000200)


def chan_sm16(raw):
    """channel pair -> SM16 (conv_pair, or CA2 magnitude + sign)"""
    if not CA2:
        return conv_pair(raw)
    QM, QP = (1 << QB) - 1, 1 << QB
    t = V(raw) & (QM * 0x00010001)
    sg = (t << (16 - QB)) & SGN
    return sg | bsel(pk_sra(sg, 15), pk_sub(QP * 0x00010001, t), t)


def F_pair(a, b):
    return F_ca2(QB, a, b) if CA2 else F_sm(a, b)


def hard_pair(v):
    return (V(v) & ca2_nz(v) & SGN) if CA2 else (V(v) & SGN)


def G_split_x(I, ma, mb, X, LT):
    """G_split without the clamp (PAR 64 G_extended)"""
    xm = plane_mask(I, X)
    d = pk_sub(ma, mb)
    return bsel(xm, pk_abs_i16(d), pk_add(ma, mb)), plane_put(I, LT, d)


def spc_sub(row, ln):
    """SPC key bits below the word index: (row, the lane key)"""
    return (V(row) << 4) | spc_lk(ln)


def rep_acc_rows(acc, t0, t1, t2, t3):
    return rep_acc(rep_acc(rep_acc(rep_acc(acc, t0), t1), t2), t3)


def rep_sm_rows(acc, v, ln):
    t = rows4(row_add_tree(v, ln))
    for tt in (t.t0, t.t1, t.t2, t.t3):
        acc = G_sm(REPSAT, tt, acc, 0)
    return acc


def spc_lk(ln):
    """polar_sc_pair.h spc_lk: bitrev4(position), or (PAR 4 / 8) (group, bitrev_LPAR(position in
    the group)), polar_sc_device.h spc_lane_key"""
    return spc_lane_key(ln) if LPAR < 4 else ln.br


def spc_sub2(row, ln):
    """two-word nodes: (row & 1, the lane key)"""
    return ((V(row) & 1) << 4) | spc_lk(ln)


def rep2_acc(t):
    q = swap16(t)
    return rep_acc(rep_acc(V(0), q.a), q.b)


def rep2_sm(v, ln):
    r = swap16(row_add_tree(v, ln))
    return G_sm(REPSAT, r.b, G_sm(REPSAT, r.a, 0, 0), 0)


def F_split_biased(I, ma, mb, FS):
    m, s = pk_min(ma, mb), plane_mask(I, FS)
    return pk_add(pk_sub(m ^ s, s), 0x02000200)


def F_split_sm(I, ma, mb, FS):
    return pk_min(ma, mb) | (plane_mask(I, FS) & SGN)


def row_sum_biased(v):
    v = V(v).astype(np.int64)
    rows = v.reshape(4, 16).sum(axis=1)
    return (np.repeat(rows, 16) & 0xFFFFFFFF).astype(U32)


def rep_acc(acc, t):
    x = pk_add(acc, t)
    x = pk_sub(x, 0x20002000)
    l = np.clip(s16(lo(x)), -REPSAT, REPSAT)
    h = np.clip(s16(hi(x)), -REPSAT, REPSAT)
    return pk(l, h)


def rep_any_zero(acc):
    return bool(((lo(acc) == 0) | (hi(acc) == 0)).any())


def row_add_tree(v, ln):
    v = V(v)
    for H in (8, 4, 2, 1):
        p = xorlane(H, v)
        v = G_sm(0, bsel(ln.a[H], v, p), bsel(ln.a[H], p, v), 0)
    return v


def row_min_u32(v):
    v = V(v)
    for H in (8, 4, 2, 1):
        v = np.minimum(v, xorlane(H, v))
    return v


def row_xor(v):
    v = V(v)
    for H in (8, 4, 2, 1):
        v = v ^ xorlane(H, v)
    return v


class X2:
    def __init__(self, a, b):
        self.a, self.b = a, b


class X4:
    def __init__(self, t0, t1, t2, t3):
        self.t0, self.t1, self.t2, self.t3 = t0, t1, t2, t3


def swap16(x):
    x = V(x)
    return X2(x[LANE & ~16], x[LANE | 16])


def swap32(x):
    x = V(x)
    return X2(x[LANE & ~32], x[LANE | 32])


def hswap(x):
    x = V(x).astype(np.int64)
    return (((x >> 16) | (x << 16)) & 0xFFFFFFFF).astype(U32)


def bcast_lo(x):
    x = V(x).astype(np.int64) & 0xFFFF
    return (x | (x << 16)).astype(U32)


def bcast_hi(x):
    x = V(x).astype(np.int64) >> 16
    return (x | (x << 16)).astype(U32)


def rep_acc_solo(acc, t0, t1, t2, t3):
    for t in (t0, t1, t2, t3):
        acc = rep_acc(acc, t)
    for t in (t0, t1, t2, t3):
        acc = rep_acc(acc, V(t) >> 16)
    return acc


def rep_sm_solo(acc, v, ln):
    t = rows4(row_add_tree(v, ln))
    for tt in (t.t0, t.t1, t.t2, t.t3):
        acc = G_sm(REPSAT, tt, acc, 0)
    for tt in (t.t0, t.t1, t.t2, t.t3):
        acc = G_sm(REPSAT, V(tt) >> 16, acc, 0)
    return acc


def rep_any_zero_lo(acc):
    return bool((lo(acc) == 0).any())


def rows4(x):
    p = swap16(x)
    q0, q1 = swap32(p.a), swap32(p.b)
    return X4(q0.a, q1.a, q0.b, q1.b)


def popcount(x):
    x = V(x).astype(np.int64)
    return np.array([bin(int(v)).count("1") for v in x], dtype=U32)


def leaf_ms(FB, B, W, M, S, ln):
    bm = ((1 << W) - 1) << B
    sub = FB & bm
    if sub == 0:
        return V(0)
    if sub == bm:
        return V(S)
    if W == 2:
        if (sub >> B) == 1:
            return (V(S) ^ xorlane(1, S)) & ln.a[1]
        PM, PS = xorlane(1, M), xorlane(1, S)
        lt = pk_sra(pk_sub(PM, M), 15)
        u1 = bsel(lt, S, PS)
        return bsel(ln.a[1], xorlane(1, u1), u1)
    H = W // 2
    PM, PS = xorlane(H, M), xorlane(H, S)
    SF = V(S) ^ PS
    Mf = pk_min(M, PM)
    xa = leaf_ms(FB, B, H, Mf, SF, ln)
    x = SF ^ xorlane(H, xa)
    lt = pk_sra(pk_sub(PM, M), 15)
    Mb = pk_mad_u16(Mf, x | 0x00010001, pk_max_u16(M, PM))
    if not EXT:
        Mb = pk_min(Mb, GSAT2)
    xb = leaf_ms(FB, B + H, H, Mb, V(S) ^ (x & ~lt), ln)
    return bsel(ln.a[H], xa ^ xorlane(H, xb), xb)


def ca2_allinfo(W, S, Z, ln):
    """polar_sc_device.h ca2_allinfo: an all-information CA2 block on (sign, zero) masks"""
    S, Z = V(S), V(Z)
    if W == 2:
        return S & ~Z
    H = W // 2
    PS, PZ = xorlane(H, S), xorlane(H, Z)
    xa = ca2_allinfo(H, S ^ PS, Z | PZ, ln)
    u = xorlane(H, xa)
    xb = ca2_allinfo(H, bsel(Z, PS ^ u, S), Z & PZ, ln)
    return bsel(ln.a[H], xa ^ xorlane(H, xb), xb)


def leaf_ca2(FB, B, W, MW, M, S, ln):
    """polar_sc_device.h leaf_ca2"""
    bm = ((1 << W) - 1) << B
    sub = FB & bm
    if sub == 0:
        return V(0)
    if sub == bm and W >= 4 and MW == 0:
        return ca2_allinfo(W, S, pk_sra(pk_sub(M, 0x00010001), 15), ln)
    if W == 2:
        if sub == bm:
            return ca2_nzs(M, S)
        if (sub >> B) == 1:
            T = ca2_nzs(M, S)
            return (T ^ xorlane(1, T)) & ln.a[1]
        v = pk_sub(V(M) ^ V(S), S)
        return pk_sra(pk_add(v, xorlane(1, v)), 15)
    H = W // 2
    PM, PS = xorlane(H, M), xorlane(H, S)
    SX = V(S) ^ PS
    if MW:
        Mf = pk_min_key(MW, M, PM)
        SF = SX | pk_sra(ca2_minbit(MW, Mf), 15)
    else:
        Mf, SF = pk_min(M, PM), SX
    xa = leaf_ca2(FB, B, H, MW, Mf, SF, ln)
    x = SX ^ xorlane(H, xa)
    lt = pk_sra(pk_sub(PM, M), 15)
    Mb = pk_mad_u16(pk_min(M, PM) if MW else Mf, x | 0x00010001, pk_max_u16(M, PM))
    if not EXT:
        Mb = pk_min(Mb, GSAT2)
    xb = leaf_ca2(FB, B + H, H, MW + 1 if (MW and EXT) else 0, Mb, V(S) ^ (x & ~lt), ln)
    return bsel(ln.a[H], xa ^ xorlane(H, xb), xb)


def leaf_gen_ca2(FB, MW, M, S, ln):
    return leaf_ca2(FB & 0xFFFF, 0, 16, MW, M, S, ln)


def leaf_gen(FB, M, S, ln):
    """polar_sc_device.h leaf_gen: the plain leaf (PRUNING_LEVEL 1 decoders are not emulated)."""
    if (FB >> 16) & 7:
        raise NotImplementedError("PRUNING_LEVEL 1 leaf decoders")
    return leaf_ms(FB & 0xFFFF, 0, 16, M, S, ln)


# ---- PAR 4 / 8 (polar_sc_device.h word_gen, polar_sc_pair.h rep_groups_*), SIGMAG ----------
def bitrev_n(v, bits):
    v = np.asarray(v, np.int64)
    r = np.zeros_like(v)
    for i in range(bits):
        r |= ((v >> i) & 1) << (bits - 1 - i)
    return r


def spc_lane_key(ln):
    p = ln.pos.astype(np.int64)
    m = (1 << LPAR) - 1
    return ((p & ~m) | bitrev_n(p & m, LPAR)).astype(U32)


def tree_step(D, v, ln):
    p = xorlane(D, v)
    a = ln.a[D]
    return G_sm(0, bsel(a, v, p), bsel(a, p, v), 0)


def add_tree_w(W, DMIN, v, ln):
    v = V(v)
    while W // 2 >= DMIN:
        v = tree_step(W // 2, v, ln)
        W //= 2
    return v


def xor_tree_w(W, DMIN, v):
    v = V(v)
    while W // 2 >= DMIN:
        v = v ^ xorlane(W // 2, v)
        W //= 2
    return v


def min_tree_w(W, DMIN, v):
    v = V(v)
    while W // 2 >= DMIN:
        v = np.minimum(v, xorlane(W // 2, v))
        W //= 2
    return v


def rep_sat_add(acc, t):
    return G_sm(REPSAT, t, acc, 0)


def group_totals(t):
    """per lane the totals of groups gr ^ 0 .. gr ^ (PPW - 1)"""
    if PPW == 2:
        return [V(t), xorlane(PARW, t)]
    v = [V(t), xorlane(PARW, t), xorlane(2 * PARW, t)]
    v.append(xorlane(PARW, v[2]))
    return v


def group_chain(CNT, acc, t, gr):
    gr = np.asarray(gr, np.int64)
    if CNT == 1:
        return rep_sat_add(acc, t)
    v = [V(t), xorlane(PARW, t)] if CNT == 2 else group_totals(t)
    for j in range(CNT):
        acc = rep_sat_add(acc, np.choose((gr & (CNT - 1)) ^ j, v).astype(U32))
    return acc


def group_order(t, gr):
    gr = np.asarray(gr, np.int64)
    v = group_totals(t)
    return [np.choose((gr & (PPW - 1)) ^ k, v).astype(U32) for k in range(PPW)]


def rep_groups_rows(acc, lam, ln):
    o = group_order(add_tree_w(PARW, 1, lam, ln), ln.pos.astype(np.int64) >> LPAR)
    r = [rows4(x) for x in o]
    for row in ("t0", "t1", "t2", "t3"):
        for k in range(PPW):
            acc = rep_sat_add(acc, getattr(r[k], row))
    return acc


def rep_groups_2(lam, ln):
    o = group_order(add_tree_w(PARW, 1, lam, ln), ln.pos.astype(np.int64) >> LPAR)
    q = [swap16(x) for x in o]
    acc = V(0)
    for k in range(PPW):
        acc = rep_sat_add(acc, q[k].a)
    for k in range(PPW):
        acc = rep_sat_add(acc, q[k].b)
    return acc


def rep_groups_1(lam, ln):
    return group_chain(PPW, V(0), add_tree_w(PARW, 1, lam, ln), ln.pos.astype(np.int64) >> LPAR)


def F_split_rep(I, MW, ma, mb, FS):
    return F_split_sm(I, ma, mb, FS)


def leaf_dp(B, W, L, fb, fbm, ln):
    """Spec_P{W} on lanes [B, B + W) (polar_sc_device.h leaf_dp, SIGMAG)"""
    bm = ((1 << W) - 1) << B
    sub = fb & bm
    L = V(L)
    if sub == 0:
        return V(0)
    if sub == bm:
        return L & SGN
    if W == 2:
        P = xorlane(1, L)
        u0 = (L ^ P) & fbm
        u0p = xorlane(1, u0)
        d = pk_sub(P & MAG, L & MAG)
        u1 = bsel(d, L, P ^ u0p) & fbm
        return bsel(ln.a[1], u0 ^ xorlane(1, u1), u1)
    H = W // 2
    P = xorlane(H, L)
    xa = leaf_dp(B, H, F_sm(L, P), fb, fbm, ln)
    Lb = G_sm(0 if EXT else GSAT, P, L, xorlane(H, xa))
    xb = leaf_dp(B + H, H, Lb, fb, fbm, ln)
    return bsel(ln.a[H], xa ^ xorlane(H, xb), xb)


def leaf_kind_w(W, L, kind, ln):
    L = V(L)
    if kind == 5:
        return L & SGN
    if kind in (1, 3):
        return add_tree_w(W, 1 if kind == 1 else 2, L, ln) & SGN
    dm = 2 if kind == 4 else 1
    h = L & SGN
    par = xor_tree_w(W, dm, h)
    mg = (L & 0x7FFF7FFF).astype(np.int64)
    br = bitrev_n(ln.pos.astype(np.int64) & (W - 1), LPAR)
    mlo, mhi = V(((mg & 0xFFFF) << 4) | br), V(((mg >> 16) << 4) | br)
    klo, khi = min_tree_w(W, dm, mlo), min_tree_w(W, dm, mhi)
    flo = np.where(klo == mlo, par & 0x8000, 0).astype(U32)
    fhi = np.where(khi == mhi, par & 0x80000000, 0).astype(U32)
    return h ^ flo ^ fhi


def word_spc(W, L, ln):
    L = V(L)
    h = L & SGN
    par = xor_tree_w(W, 1, h)
    mg = L & MAG
    lk = spc_lane_key(ln)
    klo = min_tree_w(W, 1, ((mg & 0xFF) << 24) | lk)
    khi = min_tree_w(W, 1, (((mg >> 16) & 0xFF) << 24) | lk)
    flo = np.where(((par & 0x8000) != 0) & ((klo & 15) == lk), 0x8000, 0).astype(U32)
    fhi = np.where(((par & 0x80000000) != 0) & ((khi & 15) == lk), 0x80000000, 0).astype(U32)
    return h ^ flo ^ fhi


WN_R0, WN_R1, WN_REP, WN_SPC, WN_RN = 0x00, 0x0F, 0x02, 0x04, 0x08


def wn_class(info, g0, cnt):
    ty = [(info >> (7 * (g0 + t))) & 15 for t in range(cnt)]
    r0, r1 = 0, 0x0F
    for T in ty:
        r0 |= T
        r1 &= T
    if r0 == WN_R0:
        return WN_R0
    if r1 == WN_R1:
        return WN_R1
    if all(T == WN_R0 for T in ty[:-1]) and ty[-1] == WN_REP:
        return WN_REP
    if all(T == WN_R1 for T in ty[1:]) and ty[0] == WN_SPC:
        return WN_SPC
    return WN_RN


def word_leaf_gen(B, FB, INFO, L, ln):
    kind = (INFO >> (7 * (B >> LPAR) + 4)) & 7
    if kind:
        return leaf_kind_w(PARW, L, kind, ln)
    fbm = np.where((FB >> ln.pos.astype(np.int64)) & 1, SGN, 0).astype(U32)
    return leaf_dp(B, PARW, L, FB, fbm, ln)


def word_gen(B, W, FB, INFO, L, ln):
    """polar_sc_device.h word_gen: the word tree of a PAR 4 / 8 leaf record"""
    H, h, g0 = W // 2, (W >> LPAR) // 2, B >> LPAR
    prune = (INFO >> 28) & 1
    tl = wn_class(INFO, g0, h) if prune else WN_RN
    tr = wn_class(INFO, g0 + h, h) if prune else WN_RN
    lz = tl == WN_R0
    L = V(L)
    P = xorlane(H, L)
    xa = V(0)
    if not lz:
        La = F_sm(L, P)
        if tl == WN_REP:
            xa = group_chain(h, V(0), add_tree_w(PARW, 1, La, ln), (ln.pos.astype(np.int64) >> LPAR) - g0) & SGN
        elif h == 1:
            xa = word_leaf_gen(B, FB, INFO, La, ln)
        else:
            xa = word_gen(B, H, FB, INFO, La, ln)
    Lb = G_sm(GSAT, P, L, V(0) if lz else xorlane(H, xa))
    if tr == WN_R1:
        xb = Lb & SGN
    elif tr == WN_SPC:
        xb = word_spc(H, Lb, ln)
    elif h == 1:
        xb = word_leaf_gen(B + H, FB, INFO, Lb, ln)
    else:
        xb = word_gen(B + H, H, FB, INFO, Lb, ln)
    xbp = xorlane(H, xb)
    return bsel(ln.a[H], xbp if lz else xa ^ xbp, xb)


def leaf_word_gen(FB, INFO, M, S, ln):
    return pk_sra(word_gen(0, 16, FB, INFO, V(M) | (V(S) & SGN), ln), 15)


def sm8_pair(l, h):
    l, h = V(l).astype(np.int64), V(h).astype(np.int64)
    b0, b1 = l & 0xFF, h & 0xFF
    r = b0 | (b0 << 8) | (b1 << 16) | (b1 << 24)
    return (r & ((0x8000 | VMAG) * 0x00010001)).astype(U32)


def slot_unpack(h):
    if WIDE:   # 16-bit slots hold the SM16 pair itself
        return V(h)
    return sm8_pair(h, V(h) >> 8)


def slot_pack(v):
    if WIDE:
        return V(v)
    v = V(v).astype(np.int64)
    t = (v & (VMAG * 0x00010001)) | ((v >> 8) & 0x00800080)
    return ((t & 0xFF) | (((t >> 16) & 0xFF) << 8)).astype(U32)


def conv_pair(raw):
    QM, QP = (1 << QB) - 1, 1 << QB
    SB = 0x8000 - (QP // 2 + 1)
    t = V(raw) & (QM * 0x00010001)
    m = pk_min(t, pk_sub(QP * 0x00010001, t)) & (QMAG * 0x00010001)
    return m | (pk_add(t, SB * 0x00010001) & SGN)


# ---- transpiler of a generated subtree decoder ------------------------------------------
_REF_FNS = ("F_root", "G_root", "G_split", "G_split_x", "F_root_min", "F_split_min")


def _split_top(s, sep=","):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([":
            depth += 1
        elif ch in ")]":
            depth -= 1
        if ch == sep and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    out.append(cur)
    return [x.strip() for x in out]


def _expr(e):
    e = re.sub(r"\b(0x[0-9a-fA-F]+|\d+)u\b", r"\1", e)
    e = e.replace("__builtin_elementwise_min", "np.minimum").replace("__builtin_popcount", "popcount")
    e = e.replace("(u32)", "")
    e = e.replace("true", "True").replace("ln.a1", "ln.a[1]").replace("ln.a2", "ln.a[2]")
    # template calls f<a, b>(x) -> f(a, b, x)
    e = re.sub(r"\b(\w+)<([^<>()]*)>\(", lambda m: "%s(%s, " % (m.group(1), m.group(2)), e)
    return e


_NOWRAP = set()   # variables of type X2 / X4 / bool (not wrapped into u32 lane vectors)


def _stmt(st):
    """one C statement of the generated code -> list of Python statements"""
    st = st.strip()
    if not st or st.startswith("asm volatile") or st.startswith("__builtin_amdgcn_sched_barrier"):
        return []
    m = re.match(r"^(const\s+)?(u32|X2|X4|bool)\s+(.*)$", st)
    if m:
        out = []
        for d in _split_top(m.group(3)):
            mm = re.match(r"^(\w+)(\[(\d+)\])?(\s*=\s*(.*))?$", d, re.S)
            name, cnt, init = mm.group(1), mm.group(3), mm.group(5)
            if m.group(2) != "u32":
                _NOWRAP.add(name)
            if init is not None and re.search(r"\b%s\b" % re.escape(name), init):
                raise ValueError("pair_emu: %r is read in its own initializer (C++ shadowing)" % name)
            if cnt is not None:
                out.append("%s = [V(0) for _ in range(%s)]" % (name, cnt))
            elif init is None:
                out.append("%s = V(0)" % name)
            else:
                out += _assign(name, "=", init)
        return out
    m = re.match(r"^([\w\[\]\.]+)\s*(\^=|\|=|&=|=)\s*(.*)$", st, re.S)
    if m:
        return _assign(m.group(1), m.group(2), m.group(3))
    m = re.match(r"^(BST|BSTM)\((.*)\)$", st)
    if m:
        return ["%s(%s)" % (m.group(1), _expr(m.group(2)))]
    raise ValueError("pair_emu: cannot transpile %r" % st)


def _assign(lhs, op, rhs):
    rhs = rhs.strip()
    m = re.match(r"^(%s)<([\d, ]+)>\((.*)\)$" % "|".join(_REF_FNS), rhs, re.S)
    if m:
        args = _split_top(m.group(3))
        ref = args[-1]
        return ["%s, %s = %s(%s, %s)" % (lhs, ref, m.group(1), m.group(2), ", ".join(_expr(a) for a in args))]
    if op == "=" and lhs in _NOWRAP:
        return ["%s = %s" % (lhs, _expr(rhs))]
    if op == "=":
        return ["%s = V(%s)" % (lhs, _expr(rhs))]
    return ["%s = V(%s %s (%s))" % (lhs, lhs, op[0], _expr(rhs))]


def transpile_sub(src, sid, left=False):
    """Python source of subtree decoder `sid` of a generated pair source: a function
    sub_<sid>(CH, BST, BSTM, ln, c). left: its _L variant (CA2, the subtree at word 0)."""
    # (fused plans have only the variants that read the root as F / G of the parent, _F / _G;
    # their bodies are the same code on CH(j), which the emulation supplies)
    sfx = "_L" if left else ""
    for name in ("void polar_psub_%d%s(" % (sid, sfx), "void polar_psub_%d_F%s(" % (sid, sfx),
                 "void polar_psub_%d_G%s(" % (sid, sfx)):
        if name in src:
            start = src.index(name)
            break
    else:
        raise ValueError("pair_emu: no decoder %d%s in the source" % (sid, sfx))
    body_start = src.index("{", start) + 1
    depth, i = 1, body_start
    while depth:
        if src[i] == "{":
            depth += 1
        elif src[i] == "}":
            depth -= 1
        i += 1
    body = src[body_start:i - 1]
    body = re.sub(r"//[^\n]*", "", body)
    body = re.sub(r"const u32 lane_[^;]*;", "", body)
    body = re.sub(r"Lanes ln;\s*ln\.init\([^;]*\);", "", body)
    body = re.sub(r"struct \{ u32 row; \} c; c\.row = [^;]*;", "", body)
    body = re.sub(r"asm volatile\([^;]*\);", "", body)
    body = body.replace("= {}", "= V(0)")
    lines = ["def sub_%d(CH, BST, BSTM, ln, c):" % sid]
    indent = 1
    stack = []
    toks = re.split(r"([{};])", body)
    cur = ""
    for t in toks:
        if t == ";":
            for p in _stmt(cur):
                lines.append("    " * indent + p)
            cur = ""
        elif t == "{":
            c2 = cur.strip()
            mm = re.match(r"^if\s*\((.*)\)$", c2, re.S)
            if mm:
                lines.append("    " * indent + "if %s:" % _expr(mm.group(1)))
                indent += 1
                lines.append("    " * indent + "pass")
                stack.append(True)
            else:
                assert not c2, c2
                stack.append(False)
            cur = ""
        elif t == "}":
            assert not cur.strip(), cur
            if stack.pop():
                indent -= 1
            cur = ""
        else:
            cur += t
    return "\n".join(lines)


class Sub:
    """Compiled Python subtree decoders of one generated pair source."""

    def __init__(self, src, nsubs):
        configure_from(src)
        self.fns = {}
        g = dict(globals())
        for sid in range(nsubs):
            code = transpile_sub(src, sid)
            exec(compile(code, "<psub_%d>" % sid, "exec"), g)
            self.fns[sid] = g["sub_%d" % sid]
        for m in re.finditer(r"void polar_psub_(\d+)(?:_[FG])?_L\(", src):   # CA2 leftmost variants
            sid = int(m.group(1))
            code = transpile_sub(src, sid, left=True).replace("def sub_%d(" % sid, "def sub_%d_L(" % sid)
            exec(compile(code, "<psub_%d_L>" % sid, "exec"), g)
            self.fns[(sid, "L")] = g["sub_%d_L" % sid]


class Ctx:
    def __init__(self):
        self.row = (LANE >> 4).astype(U32)


# ---- the whole decode ----------------------------------------------------------------
def is_solo(src):
    """the generated source is of the solo layout (polar_sc_pair.h POLAR_SOLO)"""
    return "#define POLAR_SOLO 1" in src


def decode(dec, llr):
    """Emulated decode of int8 frames [B, N] with pair plan `dec`: x^ [B, N] uint8."""
    src = dec.kernel_source()
    st = dec.stats
    S = st["sub_words"]
    subs = Sub(src, st["n_sub_kinds"])   # (configures the format of the source)
    upper = _upper_ops(src)
    N = dec.N
    G = N // 16
    B = llr.shape[0]
    out = np.zeros((B, N), np.uint8)
    ln, c = Lanes(), Ctx()
    if is_solo(src):
        # one frame per wave: the halves are the frame's words 8 j + 4 h + r ("virtual frames")
        for f in range(B):
            bits = _decode_pair(llr[f].astype(np.int64), None, G // 2, S, upper, subs, ln, c, solo=True)
            out[f] = _bits_to_frames(bits, G, ln, solo=True)
        return out
    for p in range(0, B, 2):
        f0, f1 = p, min(p + 1, B - 1)
        bits = _decode_pair(llr[f0].astype(np.int64), llr[f1].astype(np.int64), G, S, upper, subs, ln, c)
        x0, x1 = _bits_to_frames(bits, G, ln)
        out[p] = x0
        if p + 1 < B:
            out[p + 1] = x1
    return out


def _upper_ops(src):
    """the upper-level calls of polar_sc_pair_kernel (seg 0) as tuples"""
    k0 = src.index("polar_sc_pair_kernel(")
    body = src[k0:src.index("pair_out(", k0)]
    ops = []
    for m in re.finditer(r"(pop_fg_split<(\w+)>|pop_rep|pop_r1spc<(\w+)>|pop_h<(\w+)>|polar_psub_(\d+)(?:_([FG]))?(_L)?|"
                         r"pop_chain<(\d+), (\w+), (\w+)>)\(([^;]*)\);", body):
        args = [a.strip() for a in _split_top(m.group(11))]
        if m.group(1).startswith("pop_chain"):
            # a fused descent: record 0 (F, or G with partial sums at ub), then F / zero-u G
            d, isg0 = int(m.group(8)), m.group(10) == "true"
            k, n4, ub, gm = int(args[1]), int(args[2]), int(args[3]), int(args[4].rstrip("u"))
            ops.append(("G" if isg0 else "F", k, n4, ub))
            for i in range(1, d):
                ops.append(("G" if (gm >> i) & 1 else "F", k + i, n4 >> i, -1))
        elif m.group(1).startswith("pop_fg_split"):
            ops.append(("G" if m.group(2) == "true" else "F", int(args[1]), int(args[2]), int(args[3])))
        elif m.group(1) == "pop_rep":
            ops.append(("REP", int(args[1]), int(args[2]), int(args[3])))
        elif m.group(1).startswith("pop_r1spc"):
            ops.append(("SPC" if m.group(3) == "true" else "R1", int(args[1]), int(args[2]), int(args[3]), int(args[4])))
        elif m.group(1).startswith("pop_h"):
            ops.append(("H0" if m.group(4) == "true" else "H", int(args[1]), int(args[2])))
        else:
            lvl = int(re.search(r"lvl_row\((\d+)\)", args[0]).group(1))
            if m.group(6):
                # the subtree root as F / G of its parent's slot rows (pair_fused): that
                # record, restated, then the decoder on the root level
                isg = m.group(6) == "G"
                nq = None   # (the decoder's root rows: half the parent's, filled in _decode_pair)
                ops.append(("FG_ROOT", isg, lvl, int(args[3]) if isg else -1))
                ops.append(("SUB", int(m.group(5)), lvl + 1, int(args[2]), bool(m.group(7))))
            else:
                ops.append(("SUB", int(m.group(5)), lvl, int(args[2]), bool(m.group(7))))
    return ops


def _decode_pair(c0, c1, G, S, upper, subs, ln, c, solo=False):
    """solo: c0 is the frame, G its virtual words per half (N / 32)"""
    pos = lane_pos(LANE & 15)
    row = LANE >> 4
    # slots: level k (node of G >> k words) -> list of G >> k >> 2 rows (u16 SM8 pairs)
    slots = {}
    nbd = G // 64
    bits = [V(0) for _ in range(max(nbd, 1))]

    def chan(j):
        if solo:   # row j: words 8 j + 4 h + r
            off = 16 * (8 * j + row) + pos
            return chan_sm16((c0[off] & 0xFFFF) | ((c0[off + 64] & 0xFFFF) << 16))
        off = 16 * (4 * j + row) + pos
        return chan_sm16((c0[off] & 0xFFFF) | ((c1[off] & 0xFFFF) << 16))

    def src(k, j):
        return chan(j) if k == 0 else slot_unpack(slots[k][j])

    def ubit(l):
        return (V(bits[l >> 4]) << (15 - (l & 15))) & SGN

    def bput(l0, cnt, acc):
        if cnt >= 16:
            bits[l0 >> 4] = V(acc)
        else:
            m = ((1 << cnt) - 1) << (l0 & 15)
            mm = m | (m << 16)
            bits[l0 >> 4] = (bits[l0 >> 4] & ~V(mm)) | (V(acc) & mm)

    for op in upper:
        kind = op[0]
        if kind == "FG_ROOT":
            # the parent level's slot holds 2 nq rows; the root level gets F / G of its halves
            _, isg, k, ub = op
            nq = len(slots[k]) // 2
            op = ("G" if isg else "F", k, nq, ub)
            kind = op[0]
        if kind in ("F", "G"):
            _, k, n4, ub = op
            outk = []
            for j in range(n4):
                a, b = src(k, j), src(k, n4 + j)
                if kind == "F":
                    r = F_pair(a, b)
                else:
                    r = G_sm(GSAT, a, b, ubit(ub + j) if ub >= 0 else 0)
                outk.append(slot_pack(r))
            slots[k + 1] = outk
        elif kind == "REP":
            _, k, n4, l0 = op
            acc = V(0)
            lams = [F_pair(src(k, j), src(k, n4 + j)) for j in range(n4)]
            for lam in lams:
                if LPAR < 4:   # PAR 4 / 8: the exact chain over the groups (prep_body)
                    acc = rep_groups_rows(acc, lam, ln)
                    continue
                sg = pk_sra(lam, 15)
                t = rows4(row_sum_biased(pk_add(pk_sub((lam & MAG) ^ sg, sg), 0x02000200)))
                if solo:
                    acc = rep_acc_solo(acc, t.t0, t.t1, t.t2, t.t3)
                else:
                    acc = rep_acc(rep_acc(rep_acc(rep_acc(acc, t.t0), t.t1), t.t2), t.t3)
            if not CA2 and LPAR >= 4 and (rep_any_zero_lo if solo else rep_any_zero)(acc):
                acc = V(0)
                for lam in lams:
                    if solo:
                        acc = rep_sm_solo(acc, lam, ln)
                        continue
                    t = rows4(row_add_tree(lam, ln))
                    for tt in (t.t0, t.t1, t.t2, t.t3):
                        acc = G_sm(REPSAT, tt, acc, 0)
            full = pk_sra(bcast_lo(acc) if solo else acc, 15)
            for l in range(0, n4, 16):
                bput(l0 + l, min(16, n4 - l), full)
        elif kind in ("R1", "SPC"):
            _, k, n4, ub, l0 = op
            acc = V(0)
            par = V(0)
            klo = V(0xFFFFFFFF)
            khi = V(0xFFFFFFFF)
            for j in range(n4):
                lam = G_sm(GSAT, src(k, j), src(k, n4 + j), ubit(ub + j) if ub >= 0 else 0)
                h = hard_pair(lam)
                q = (l0 + j) & 15
                acc = acc | (h >> (15 - q))
                if q == 15 or j + 1 == n4:
                    first = max((l0 + j) & ~15, l0)
                    bput(first, l0 + j + 1 - first, acc)
                    acc = V(0)
                if kind == "SPC" and solo:
                    # key (|lambda|, word 8 j + 4 h + r, bitrev4(position))
                    par = par ^ h
                    wk = ((j << 7) | (row << 4)).astype(U32)
                    klo = np.minimum(klo, ((lam & 0xFF) << 24) | wk)
                    khi = np.minimum(khi, (((lam >> 16) & 0xFF) << 24) | wk | 64)
                elif kind == "SPC":
                    par = par ^ h
                    wk = ((4 * j + row) << 4).astype(U32)
                    klo = np.minimum(klo, ((lam & 0xFF) << 24) | wk)
                    khi = np.minimum(khi, (((lam >> 16) & 0xFF) << 24) | wk)
            if kind == "SPC" and solo:
                parity = (int(np.bitwise_xor.reduce(V(par).astype(np.int64))) >> 15) & 1
                parity ^= (int(np.bitwise_xor.reduce(V(par).astype(np.int64))) >> 31) & 1
                k = np.minimum(klo | ln.br, khi | ln.br).min()
                if parity:
                    l = l0 + int((k >> 7) & 0x1FFFF)
                    hb = 16 if (k & 64) else 0
                    for L in range(64):
                        if (int(k) & 63) == ((int(row[L]) << 4) | int(ln.br[L])):
                            bits[l >> 4][L] ^= U32(1 << ((l & 15) + hb))
            elif kind == "SPC":
                lk = spc_lk(ln)
                par = row_xor(par)
                klo = row_min_u32(klo | lk)
                khi = row_min_u32(khi | lk)
                p = swap16(par)
                par = p.a ^ p.b
                p = swap32(par)
                par = p.a ^ p.b
                for _ in (16, 32):
                    a = swap16(klo) if _ == 16 else swap32(klo)
                    b = swap16(khi) if _ == 16 else swap32(khi)
                    klo, khi = np.minimum(a.a, a.b), np.minimum(b.a, b.b)
                flo = land(land(par & 0x8000, (klo & 15) == lk), ((klo >> 4) & 3) == row)
                fhi = land(land(par & 0x80000000, (khi & 15) == lk), ((khi >> 4) & 3) == row)
                for L in range(64):
                    if flo[L]:
                        l = l0 + int((klo[L] >> 6) & 0x3FFFF)
                        bits[l >> 4][L] ^= U32(1 << (l & 15))
                    if fhi[L]:
                        l = l0 + int((khi[L] >> 6) & 0x3FFFF)
                        bits[l >> 4][L] ^= U32(0x10000 << (l & 15))
        elif kind in ("H", "H0"):
            _, l0, n4 = op
            if n4 >= 16:
                for e in range(n4 >> 4):
                    bb = bits[((l0 + n4) >> 4) + e]
                    bits[(l0 >> 4) + e] = bb.copy() if kind == "H0" else bits[(l0 >> 4) + e] ^ bb
            else:
                m = ((1 << n4) - 1) << (l0 & 15)
                mm = V(m | (m << 16))
                d = bits[l0 >> 4]
                sh = (d >> n4) & mm
                bits[l0 >> 4] = ((d & ~mm) | sh) if kind == "H0" else (d ^ sh)
        elif kind == "SUB":
            _, sid, k, l0, left = op
            rows = slots[k]

            def CH(j, rows=rows):
                return slot_unpack(rows[j])

            def BST(d, v, l0=l0):
                bits[(l0 >> 4) + d] = V(v)

            def BSTM(m, v, l0=l0):
                mm = V(m) << (l0 & 15)
                bits[l0 >> 4] = (bits[l0 >> 4] & ~mm) | ((V(v) << (l0 & 15)) & mm)

            subs.fns[(sid, "L") if left else sid](CH, BST, BSTM, ln, c)
    return bits


def _bits_to_frames(bits, G, ln, solo=False):
    """partial sums (local words per lane) -> x^ of both frames (solo: of the one frame)"""
    pos = lane_pos(LANE & 15)
    row = LANE >> 4
    if solo:
        x = np.zeros(G * 16, np.uint8)
        for d, v in enumerate(bits):
            v = v.astype(np.int64)
            for j in range(16):
                for h in range(2):
                    w = 8 * (16 * d + j) + 4 * h + row
                    ok = w < G
                    x[(16 * w + pos)[ok]] = ((v >> (j + 16 * h)) & 1)[ok]
        return x
    x = np.zeros((2, G * 16), np.uint8)
    for d, v in enumerate(bits):
        v = v.astype(np.int64)
        for j in range(16):
            l = 16 * d + j
            w = 4 * l + row
            ok = w < G
            x[0, (16 * w + pos)[ok]] = ((v >> j) & 1)[ok]
            x[1, (16 * w + pos)[ok]] = ((v >> (16 + j)) & 1)[ok]
    return x[0], x[1]


def run_sub(dec, sid, rows, subs=None):
    """Emulated subtree decoder `sid` of pair plan `dec` on root slot rows (uint16 [S/4, 64]):
    its partial-sum dwords uint32 [max(1, S/64), 64] (polar_sc_debug_subtree on the device)."""
    if subs is None:
        subs = Sub(dec.kernel_source(), dec.stats["n_sub_kinds"])
    S = dec.stats["sub_words"]
    wpr = 8 if is_solo(dec.kernel_source()) else 4
    bits = [V(0) for _ in range(max(1, S // (16 * wpr)))]

    def CH(j):
        return slot_unpack(V(rows[j]))

    def BST(d, v):
        bits[d] = V(v)

    def BSTM(m, v):
        mm = V(m)
        bits[0] = (bits[0] & ~mm) | (V(v) & mm)

    subs.fns[sid](CH, BST, BSTM, Lanes(), Ctx())
    return np.stack(bits)


def random_rows(rng, S):
    """random root slot rows of a subtree: SM8 pairs with magnitude <= 31 (zeros included)"""
    mag = rng.integers(0, 32, size=(S // 4, 64, 2))
    mag[rng.random(mag.shape) < 0.1] = 0
    sgn = rng.integers(0, 2, size=(S // 4, 64, 2))
    b = (sgn << 7) | mag
    return (b[..., 0] | (b[..., 1] << 8)).astype(np.uint16)
