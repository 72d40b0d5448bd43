"""Oracle pinning: known-answer vectors of the reference (the 9 codewords hard-coded in
src/testbench/sc_encoder/sc_encoder.h:74-88) and the cross-check of the two independent
restatements (literal FSM of my_module.h vs the recursive Appendix-A formulation)."""
import numpy as np
import pytest

import util


@pytest.mark.parametrize("mask_name,key", [("FB_N8_K4", "cw8x4"), ("FB_N512_K256", "cw512x256"),
                                           ("FB_N1024_K512", "cw1024x512")])
def test_kat_codewords_are_valid(oracle_mod, mask_name, key):
    """x = u F^(x)n with u zero on frozen positions (natural order, bit 1 = info)."""
    mask = util.mask(mask_name)
    x = np.array(util.kat()[key], dtype=np.uint8)
    u = oracle_mod.encode(x)          # F^(x)n is an involution over GF(2)
    assert not (u & (1 - mask)[None, :]).any()
    np.testing.assert_array_equal(oracle_mod.encode(u), x)


def test_kat_cw1024_not_valid_for_generated_mask():
    mask = util.mask("frozen_n_1024_k_512")
    x = np.array(util.kat()["cw1024x512"], dtype=np.uint8)
    u = util.encode_np(x)
    assert (u & (1 - mask)[None, :]).any()


@pytest.mark.parametrize("mask_name,key", [("FB_N512_K256", "cw512x256"), ("FB_N1024_K512", "cw1024x512")])
@pytest.mark.parametrize("amp", [31, 1, 7])
def test_kat_noiseless_decode(oracle_mod, mask_name, key, amp):
    mask = util.mask(mask_name)
    x = np.array(util.kat()[key], dtype=np.uint8)
    llr = np.where(x == 1, -amp, amp).astype(np.int8)
    np.testing.assert_array_equal(oracle_mod.decode_fsm(mask, llr), x)
    np.testing.assert_array_equal(oracle_mod.decode_rec(mask, llr), x)


def test_fsm_state_census_c2(oracle_mod):
    """State visits per frame for FB_N1024_K512 (C2): 20 leaves (R_STATE), 7 REP, 4 R1,
    6 SPC; every F has a matching G."""
    mask = util.mask("FB_N1024_K512")
    llr, _ = util.synth_frames(mask, 2, seed=1)
    _, cnt = oracle_mod.decode_fsm(mask, llr, return_counts=True)
    per = {k: v // 2 for k, v in cnt.items()}
    assert per["R"] == 20 and per["F_REP"] == 7 and per["G_R1"] == 4 and per["G_SPC"] == 6
    assert per["F"] == per["G"] == 29 and per["H"] + per["H0"] == 39


def _random_mask(rng, N, kind):
    if kind == 0:
        m = rng.integers(0, 2, N)
    elif kind == 1:
        pats = [0, 0xFFFF, 0x8000, 0xFFFE, int(rng.integers(0, 65536))]
        m = np.concatenate([[(p >> k) & 1 for k in range(16)] for p in rng.choice(pats, N // 16)])
    elif kind == 2:
        m = (rng.random(N) < np.linspace(0, 1, N) ** 0.5).astype(int)
    else:
        m = np.full(N, int(rng.integers(0, 2)))
    return m.astype(np.uint8)


def test_fsm_equals_recursive_restatement(oracle_mod):
    rng = np.random.default_rng(11)
    for trial in range(240):
        N = int(2 ** rng.integers(5, 12))
        mask = _random_mask(rng, N, trial % 4)
        llr = rng.integers(-32, 32, size=(6, N)).astype(np.int8)
        if trial % 7 == 0:
            llr = rng.integers(-1, 2, size=(6, N)).astype(np.int8)
        if trial % 11 == 0:
            llr = rng.integers(-128, 128, size=(6, N)).astype(np.int8)
        np.testing.assert_array_equal(oracle_mod.decode_fsm(mask, llr), oracle_mod.decode_rec(mask, llr),
                                      err_msg="trial %d N=%d" % (trial, N))


@pytest.mark.parametrize("name", ["FB_N128_K64", "FB_N1024_K512", "frozen_n_2048_k_1024", "FB_N2048_K1024"])
def test_noiseless_property(oracle_mod, name):
    """Noiseless channel (all |llr| = 31): the decoder returns the sent codeword."""
    mask = util.mask(name)
    rng = np.random.default_rng(8)
    u = rng.integers(0, 2, size=(16, mask.size), dtype=np.uint8) & mask[None, :]
    x = util.encode_np(u)
    llr = np.where(x == 1, -31, 31).astype(np.int8)
    np.testing.assert_array_equal(oracle_mod.decode_fsm(mask, llr), x)


def test_stale_node_stack_is_harmless(oracle_mod):
    """Node_type_stack is not reset by INIT (my_module.h:328); decoding frames one by one
    or as a batch (stale entries carried over) gives identical results."""
    mask = util.mask("frozen_n_1024_k_512")
    llr, _ = util.synth_frames(mask, 5, ebn0_db=0.5, seed=9)
    batch = oracle_mod.decode_fsm(mask, llr)
    single = np.concatenate([oracle_mod.decode_fsm(mask, llr[i:i + 1]) for i in range(5)])
    np.testing.assert_array_equal(batch, single)


@pytest.mark.parametrize("case", ["c1", "c2_snr", "c2_edge", "c3"])
def test_restatement_reproduces_committed_vectors(oracle_mod, case):
    """The oracle still decodes the committed regression vectors to the committed x^."""
    name, llr, x = util.decode_vectors()[case]
    np.testing.assert_array_equal(oracle_mod.decode_fsm(util.mask(name), llr), x, err_msg=case)


@pytest.mark.parametrize("q", [5, 7, 8])
def test_fsm_equals_recursive_other_llr_bits(oracle_mod, q):
    """LLR_BITS 5..8 (config.h:2; the reference's pruning sweep runs at QUANT = 8,
    script/script_tests.sh:9,25): both restatements agree on the whole int8 range (the low
    q bits are the LLR), noiseless frames decode, and q = 6 through the switch is the default."""
    rng = np.random.default_rng(70 + q)
    for trial in range(60):
        N = int(2 ** rng.integers(5, 11))
        mask = _random_mask(rng, N, trial % 4)
        llr = rng.integers(-128, 128, size=(5, N)).astype(np.int8)
        np.testing.assert_array_equal(oracle_mod.decode_fsm(mask, llr, llr_bits=q),
                                      oracle_mod.decode_rec(mask, llr, llr_bits=q), err_msg="trial %d" % trial)
    mask = util.mask("FB_N1024_K512")
    x = np.array(util.kat()["cw1024x512"], dtype=np.uint8)
    amp = (1 << (q - 1)) - 1
    np.testing.assert_array_equal(oracle_mod.decode_fsm(mask, np.where(x == 1, -amp, amp).astype(np.int8),
                                                        llr_bits=q), x)
    llr, _ = util.synth_frames(mask, 6, ebn0_db=1.0, seed=5)
    np.testing.assert_array_equal(oracle_mod.decode_fsm(mask, llr, llr_bits=6), oracle_mod.decode_fsm(mask, llr))
    with pytest.raises(ValueError):
        oracle_mod.decode_fsm(mask, llr, llr_bits=10)
