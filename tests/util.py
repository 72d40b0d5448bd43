"""Shared test helpers: fixtures, synthetic frames, and a numpy interpreter of the compiled
decode schedule (used to validate the host schedule compiler on CPU, independently of the
GPU kernel and of the C oracle)."""
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MASKS_JSON = os.path.join(ROOT, "data", "frozen_masks.json")
KAT_JSON = os.path.join(ROOT, "tests", "golden", "kat_codewords.json")

_masks = None


def masks():
    global _masks
    if _masks is None:
        with open(MASKS_JSON) as f:
            _masks = json.load(f)["masks"]
    return _masks


def mask(name):
    m = masks()[name]
    b = np.frombuffer(bytes.fromhex(m["hex"]), dtype=np.uint8)
    return np.unpackbits(b, bitorder="little")[: m["N"]].astype(np.uint8)


def kat():
    with open(KAT_JSON) as f:
        return json.load(f)["codewords"]


def encode_np(u):
    """x = u F^{(x)n} (natural order), vectorised over rows."""
    x = np.array(u, dtype=np.uint8, copy=True)
    B, N = x.shape
    h = 1
    while h < N:
        v = x.reshape(B, N // (2 * h), 2, h)
        v[:, :, 0, :] ^= v[:, :, 1, :]
        h *= 2
    return x


def synth_frames(info_mask, batch, ebn0_db=2.5, seed=0xF0, rate=None):
    """The reference C-sim chain: random info bits, x = uF, BPSK
    (bit1 -> -1, sc_bpsk.h:53), AWGN sigma = 1/sqrt(2 R 10^(EbN0/10)) (main.cpp:91-98),
    llr = clamp(trunc(4 y), -31, 31) (sc_quantizer.h:77-79). Returns (llr int8, x uint8)."""
    rng = np.random.default_rng(seed)
    N = info_mask.size
    R = rate if rate is not None else max(int(info_mask.sum()), 1) / N
    u = (rng.integers(0, 2, size=(batch, N), dtype=np.uint8) & info_mask[None, :].astype(np.uint8))
    x = encode_np(u)
    sigma = 1.0 / np.sqrt(2.0 * R * 10.0 ** (ebn0_db / 10.0))
    y = np.where(x == 1, -1.0, 1.0).astype(np.float32) + sigma * rng.standard_normal((batch, N), dtype=np.float32)
    q = np.trunc(4.0 * y)
    llr = np.clip(q, -31, 31).astype(np.int8)
    return llr, x


# ----------------------------------------------------------------------------------------
# numpy SM primitives: values are (s, m) int arrays
# ----------------------------------------------------------------------------------------
def sm_from_llr(llr, q=6):
    h = 1 << (q - 1)
    t = ((llr.astype(np.int32) & (2 * h - 1)) ^ h) - h   # sign-extend q bits
    m = np.abs(t) & (h - 1)
    s = ((t < 0) & (m != 0)).astype(np.int32)
    return s, m


def F(a, b):
    return a[0] ^ b[0], np.minimum(a[1], b[1])


def G(a, b, u, sat=None):
    sa2 = a[0] ^ u
    same = sa2 == b[0]
    m = np.where(same, a[1] + b[1], np.abs(a[1] - b[1]))
    s = np.where(a[1] < b[1], b[0], sa2)
    if sat is not None:
        m = np.minimum(m, sat)
    return s, m


def leaf(lam, fb):
    """Spec_P16_ext on lam = (s, m) arrays [B, n]; returns x [B, n] (exact)."""
    s, m = lam
    n = s.shape[1]
    if n == 2:
        f0, f1 = fb & 1, (fb >> 1) & 1
        u0 = (s[:, 0] ^ s[:, 1]) & f0
        sg = np.where(m[:, 0] < m[:, 1], s[:, 1], s[:, 0] ^ u0) & f1
        return np.stack([u0 ^ sg, sg], axis=1)
    h = n // 2
    a = (s[:, :h], m[:, :h])
    b = (s[:, h:], m[:, h:])
    xa = leaf(F(a, b), fb & ((1 << h) - 1))
    xb = leaf(G(a, b, xa), fb >> h)
    return np.concatenate([xa ^ xb, xb], axis=1)


def leaf_kind(lam, kind):
    """PRUNING_LEVEL 1 leaf decoders (POLAR_LEAF_REP/SPC/REP2/SPC2) on lam = (s, m) [B, P]."""
    s, m = lam
    B, P = s.shape
    L = P.bit_length() - 1
    if kind == 5:                           # Spec_Node_R1
        return s.copy()
    if kind in (1, 3):                      # REP_REP2_P_SM: folds P/2 .. 2 (exact), then REP_2
        ts, tm = s, m
        n = P
        while n > 2:
            h = n // 2
            ts, tm = G((ts[:, :h], tm[:, :h]), (ts[:, h:n], tm[:, h:n]), 0)
            n = h
        if kind == 1:
            sig = np.where(tm[:, 0] < tm[:, 1], ts[:, 1], ts[:, 0])
            return np.repeat(sig[:, None], P, axis=1)
        return np.tile(ts[:, :2], (1, P // 2))
    # SPC / SPC2: flip the tournament minimum (ties -> smallest bitrev_L) of the whole word or
    # of each class of even / odd positions when its sign parity is odd
    br = np.array([int(format(l, "0%db" % L)[::-1], 2) for l in range(P)])
    key = (m << L) | br[None, :]
    x = s.copy()
    classes = [np.arange(P)] if kind == 2 else [np.arange(0, P, 2), np.arange(1, P, 2)]
    for c in classes:
        par = s[:, c].sum(axis=1) & 1
        j = c[key[:, c].argmin(axis=1)]
        x[np.arange(B), j] ^= par
    return x


def rep_tree(lam):
    s, m = lam
    n = s.shape[1]
    while n > 1:
        h = n // 2
        s, m = G((s[:, :h], m[:, :h]), (s[:, h:n], m[:, h:n]), 0)
        n = h
    return s[:, 0], m[:, 0]


def run_schedule(ops, N, llr, par=16, q=6):
    """Interpret a compiled schedule (list of dicts from Decoder.schedule(), SIGMAG) on a
    batch. Records count 16-LLR words; PAR > 16 groups are par / 16 consecutive words."""
    B = llr.shape[0]
    Gw = N // 16
    P16 = par // 16
    L = par.bit_length() - 1
    gsat, repsat = (1 << (q - 2)) - 1, (1 << (q + L - 1)) - 1
    s, m = sm_from_llr(llr, q)
    chan = (s.reshape(B, Gw, 16), m.reshape(B, Gw, 16))
    buf = {0: chan}
    bits = np.zeros((B, Gw, 16), dtype=np.int32)
    brp = np.array([int(format(l, "0%db" % L)[::-1], 2) for l in range(par)])

    def words(k, lo, hi):
        return buf[k][0][:, lo:hi], buf[k][1][:, lo:hi]

    def ubits(upos, n):
        if upos < 0:
            return 0
        return bits[:, upos:upos + n]

    def flat(x, i):   # PAR word i of a [B, n, 16] array as [B, par] positions
        return x[:, i * P16:(i + 1) * P16].reshape(x.shape[0], par)

    for op in ops:
        code, k, n, pos, upos, fb = op["op"], op["level"], op["n"], op["pos"], op["upos"], op["fb"]
        exact = bool(fb & (1 << 19))
        if code == "END":
            break
        if code in ("F", "G", "FLEAF", "GLEAF", "REP", "R1", "SPC"):
            a, b = words(k, 0, n), words(k, n, 2 * n)
        if code == "F":
            buf[k + 1] = F(a, b)
        elif code == "G":
            buf[k + 1] = G(a, b, ubits(upos, n), None if exact else gsat)
        elif code in ("FLEAF", "GLEAF"):
            lam = F(a, b) if code == "FLEAF" else G(a, b, ubits(upos, 1), None if exact else gsat)
            w = (lam[0][:, 0], lam[1][:, 0])
            kind = (fb >> 16) & 7
            bits[:, pos] = leaf(w, fb & 0xFFFF) if kind == 0 else leaf_kind(w, kind)
        elif code == "PLEAF":
            w = (buf[k][0][:, 0:n].reshape(B, par), buf[k][1][:, 0:n].reshape(B, par))
            bits[:, pos:pos + n] = leaf_kind(w, (fb >> 16) & 7).reshape(B, n, 16)
        elif code == "REP":
            lam = F(a, b)
            acc = (np.zeros(B, np.int32), np.zeros(B, np.int32))
            for i in range(n // P16):
                t = rep_tree((flat(lam[0], i), flat(lam[1], i)))
                acc = G(t, acc, 0, repsat)
            bits[:, pos:pos + n] = acc[0][:, None, None]
        elif code in ("R1", "SPC"):
            lam = G(a, b, ubits(upos, n), gsat)
            h = lam[0].copy()
            if code == "SPC":
                par_ = h.reshape(B, -1).sum(axis=1) & 1
                wi = np.arange(n)
                # key: (|l|, PAR word, bitrev_L(position in the PAR word))
                posp = (wi % P16)[:, None] * 16 + np.arange(16)[None, :]
                key = (lam[1].astype(np.int64) << 32) | ((wi // P16)[None, :, None] << L) | brp[posp][None, :, :]
                idx = key.reshape(B, -1).argmin(axis=1)
                fl = np.zeros(B * n * 16, dtype=np.int32)
                fl[np.arange(B) * n * 16 + idx] = par_
                h ^= fl.reshape(B, n, 16)
            bits[:, pos:pos + n] = h
        elif code == "H":
            bits[:, pos:pos + n] ^= bits[:, pos + n:pos + 2 * n]
        elif code == "H0":
            bits[:, pos:pos + n] = bits[:, pos + n:pos + 2 * n]
        else:
            raise ValueError(code)
    return bits.reshape(B, N).astype(np.uint8)


def decode_vectors():
    """tests/golden/decode_vectors.npz (tools/make_decode_vectors.py): {case: (mask name,
    llr [B, N] int8, x^ [B, N] uint8)}."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "decode_vectors.npz")
    z = np.load(path, allow_pickle=False)
    out = {}
    for key in sorted({k.split("__")[0] for k in z.files}):
        llr = z[key + "__llr"]
        x = np.unpackbits(z[key + "__xhat"], axis=1, bitorder="little")[:, : llr.shape[1]]
        out[key] = (str(z[key + "__mask"]), llr, x)
    return out
