"""The restatement across the reference's swept datapath (oracle/polar_oracle.c
orc_set_format): PAR 2..64 (polar_parameters.h:8; script_tests.sh:11 runs 16 and 64, the RTL
sweeps 4..64), CA2 vs SIGMAG (config.h:11; script/parser.sh:15,43), EXTENDED 0/1
(config.h:14) and LLR_BITS up to 9 (parser_comp.sh:12; 9-bit LLRs need the int16 channel).

* the literal FSM and the recursive restatement agree on random masks (including groups of
  every pruned class at the given PAR) and random LLRs over the whole input range, under
  every pruning-sweep configuration;
* noiseless frames decode to the sent codeword in every format;
* the CA2 primitives follow scalar.h / functions.h:48-118 bit for bit (hand-computed cases).
"""
import itertools

import numpy as np
import pytest

import util


def _mask(rng, N, par, kind):
    if kind == 0:
        return rng.integers(0, 2, N).astype(np.uint8)
    if kind == 1:   # groups of every class do_prunning distinguishes at this PAR
        all1 = (1 << par) - 1
        pats = [0, all1, 1 << (par - 1), all1 & ~1, 3 << (par - 2), all1 & ~3, int(rng.integers(0, 1 << min(par, 62)))]
        return np.concatenate([[(int(p) >> k) & 1 for k in range(par)] for p in rng.choice(pats, N // par)]).astype(np.uint8)
    return (rng.random(N) < np.linspace(0, 1, N) ** 0.5).astype(np.uint8)


FORMATS = [dict(par=p, sigmag=s, extended=e, llr_bits=q)
           for p, s, e, q in itertools.product([2, 4, 8, 16, 32, 64], [1, 0], [1, 0], [6, 8])]


@pytest.mark.parametrize("fmt", FORMATS, ids=lambda f: "p%d_%s_e%d_q%d" % (f["par"], "sm" if f["sigmag"] else "ca2",
                                                                          f["extended"], f["llr_bits"]))
def test_fsm_equals_recursive_formats(oracle_mod, fmt):
    rng = np.random.default_rng(fmt["par"] * 131 + fmt["sigmag"] * 7 + fmt["extended"] * 3 + fmt["llr_bits"])
    par = fmt["par"]
    for trial in range(10):
        N = int(2 ** rng.integers(max(5, int(np.log2(par)) + 1), 11))
        mask = _mask(rng, N, par, trial % 3)
        llr = rng.integers(-128, 128, size=(3, N)).astype(np.int8)
        llr[:, rng.integers(0, N, 8)] = -(1 << (fmt["llr_bits"] - 1))     # the -2^(Q-1) corner
        for c7 in (None,) + oracle_mod.SWEEP_CONFIGS[trial % 11: trial % 11 + 1]:
            a = oracle_mod.decode_fsm(mask, llr, config=c7, **fmt)
            b = oracle_mod.decode_rec(mask, llr, config=c7, **fmt)
            np.testing.assert_array_equal(a, b, err_msg="trial %d cfg %s" % (trial, c7))


@pytest.mark.parametrize("par", [2, 4, 8, 16, 32, 64])
@pytest.mark.parametrize("sigmag", [1, 0])
def test_noiseless_roundtrip_formats(oracle_mod, par, sigmag):
    rng = np.random.default_rng(par + 100 * sigmag)
    for q in (5, 6, 8, 9):
        N = max(128, 4 * par)
        mask = _mask(rng, N, par, 2)
        u = rng.integers(0, 2, size=(4, N)).astype(np.uint8) & mask
        x = util.encode_np(u)
        amp = (1 << (q - 1)) - 1
        llr = np.where(x == 1, -amp, amp).astype(np.int16)
        for ext in (1, 0):
            got = oracle_mod.decode_fsm(mask, llr, llr_bits=q, par=par, sigmag=sigmag, extended=ext)
            np.testing.assert_array_equal(got, x, err_msg="q %d ext %d" % (q, ext))


def test_llr_bits_9_int16_channel(oracle_mod):
    """9-bit LLRs (QUANT 9) only fit an int16 channel; the low 9 bits are the LLR."""
    rng = np.random.default_rng(9)
    mask = util.mask("FB_N1024_K512")
    llr = rng.integers(-256, 256, size=(4, 1024)).astype(np.int16)
    a = oracle_mod.decode_fsm(mask, llr, llr_bits=9)
    np.testing.assert_array_equal(a, oracle_mod.decode_rec(mask, llr, llr_bits=9))
    # the same values through bits above bit 8 are ignored (sc_bigint<9>)
    np.testing.assert_array_equal(a, oracle_mod.decode_fsm(mask, (llr.astype(np.int32) + 512).astype(np.int16),
                                                           llr_bits=9))


def test_ca2_primitives(oracle_mod):
    """functions.h:48-118 / scalar.h on hand-computed 6-bit cases."""
    L = oracle_mod.lib()
    p = lambda v: v & 63                   # 6-bit pattern of a signed value
    # F_function_C2: min of qabs, sign xor; qabs(-32) = -32 is the (signed) minimum
    assert L.orc_F_ca2(6, p(-5), p(9)) == p(-5)
    assert L.orc_F_ca2(6, p(-5), p(-9)) == p(5)
    assert L.orc_F_ca2(6, p(0), p(-9)) == p(0)          # no negative zero in CA2
    assert L.orc_F_ca2(6, p(-32), p(3)) == p(-32)       # -(-32) wraps to -32
    assert L.orc_F_ca2(6, p(-32), p(-3)) == p(-32)
    # G_function_C2: sa ? lb - la : lb + la, saturated to +-31
    assert L.orc_G_ca2(6, p(20), p(20), 0) == p(31)
    assert L.orc_G_ca2(6, p(20), p(-20), 1) == p(-31)
    assert L.orc_G_ca2(6, p(7), p(7), 1) == p(0)
    assert L.orc_G_ca2(6, p(-32), p(3), 0) == p(-29)
    # G_extended_C2: exact, 7-bit result
    assert L.orc_Gext_ca2(6, p(-32), p(-32), 0) == (-64) & 127
    assert L.orc_Gext_ca2(6, p(31), p(31), 0) == 62


def test_formats_change_results(oracle_mod):
    """PAR, CA2 and EXTENDED are real datapath switches: on AWGN frames at low SNR each of
    them changes some decisions relative to the shipped configuration."""
    mask = util.mask("FB_N1024_K512")
    llr, _ = util.synth_frames(mask, 256, ebn0_db=0.0, seed=3)
    base = oracle_mod.decode_fsm(mask, llr)
    for kw in (dict(par=64), dict(par=4), dict(sigmag=0), dict(extended=0)):
        assert (oracle_mod.decode_fsm(mask, llr, **kw) != base).any(), kw
