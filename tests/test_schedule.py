"""Host schedule compiler (libpolar_sc.so, host-only entry points; no GPU needed).

The compiled op list must reproduce the literal FSM of my_module::do_action: interpreted
by the numpy executor in tests/util.py it must be bit-exact with the oracle, and its op
census must match the FSM's state census."""
import numpy as np
import pytest

import util


@pytest.mark.parametrize("name", ["FB_N128_K64", "FB_N512_K256", "FB_N1024_K512", "frozen_n_1024_k_512",
                                  "frozen_n_1024_k_768", "FB_N2048_K1024", "frozen_n_2048_k_1024",
                                  "frozen_n_4096_k_2048"])
def test_schedule_equals_fsm(pkg, oracle_mod, name):
    mask = util.mask(name)
    dec = pkg.Decoder(mask)
    llr, _ = util.synth_frames(mask, 24, ebn0_db=1.0, seed=17)
    np.testing.assert_array_equal(util.run_schedule(dec.schedule(), mask.size, llr),
                                  oracle_mod.decode_fsm(mask, llr))


def test_schedule_random_masks(pkg, oracle_mod):
    rng = np.random.default_rng(21)
    for trial in range(120):
        N = int(2 ** rng.integers(5, 11))
        if trial % 3 == 0:
            mask = rng.integers(0, 2, N)
        elif trial % 3 == 1:
            pats = [0, 0xFFFF, 0x8000, 0xFFFE, int(rng.integers(0, 65536))]
            mask = np.concatenate([[(p >> k) & 1 for k in range(16)] for p in rng.choice(pats, N // 16)])
        else:
            mask = (rng.random(N) < np.linspace(0, 1, N)).astype(int)
        mask = mask.astype(np.uint8)
        llr = rng.integers(-32, 32, size=(4, N)).astype(np.int8)
        dec = pkg.Decoder(mask)
        np.testing.assert_array_equal(util.run_schedule(dec.schedule(), N, llr), oracle_mod.decode_fsm(mask, llr),
                                      err_msg="trial %d" % trial)


@pytest.mark.parametrize("name", ["FB_N1024_K512", "frozen_n_2048_k_1024", "frozen_n_65536_k_32768"])
def test_op_census_matches_fsm_states(pkg, oracle_mod, name):
    mask = util.mask(name)
    dec = pkg.Decoder(mask)
    oc = dec.stats["op_count"]
    llr = np.zeros((1, mask.size), dtype=np.int8)
    _, st = oracle_mod.decode_fsm(mask, llr, return_counts=True)
    assert oc.get("FLEAF", 0) + oc.get("GLEAF", 0) == st["R"]
    assert oc.get("REP", 0) == st["F_REP"]
    assert oc.get("R1", 0) == st["G_R1"]
    assert oc.get("SPC", 0) == st["G_SPC"]
    assert oc.get("H", 0) == st["H"] and oc.get("H0", 0) == st["H0"]
    assert oc.get("F", 0) + oc.get("FLEAF", 0) == st["F"]
    assert oc.get("G", 0) + oc.get("GLEAF", 0) == st["G"]


def test_group_census_c3(pkg):
    """frozen_n_65536_k_32768 group types."""
    s = pkg.Decoder(util.mask("frozen_n_65536_k_32768")).stats
    assert (s["n_r0"], s["n_r1"], s["n_rep"], s["n_spc"], s["n_rn"]) == (1667, 1535, 142, 273, 479)
    s = pkg.Decoder(util.mask("FB_N1024_K512")).stats
    assert (s["n_r0"], s["n_r1"], s["n_rep"], s["n_spc"], s["n_rn"]) == (15, 16, 7, 6, 20)


def test_schedule_shapes(pkg):
    dec = pkg.Decoder(util.mask("FB_N1024_K512"))
    ops = dec.schedule()
    assert ops[-1]["op"] == "END"
    assert ops[0]["op"] == "F" and ops[0]["level"] == 0 and ops[0]["n"] == 32   # root is never pruned
    for o in ops[:-1]:
        assert o["n"] >= 1 and (o["n"] & (o["n"] - 1)) == 0
        if o["op"] in ("H", "H0"):
            assert o["pos"] % (2 * o["n"]) == 0
        if o["op"] in ("G", "GLEAF", "R1", "SPC") and o["upos"] >= 0:
            assert o["pos"] - o["upos"] == o["n"]
