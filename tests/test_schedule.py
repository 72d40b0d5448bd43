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


# ---- the reference's pruning sweep (script/script_tests.sh:103-122) -------------------------
def _config(pkg, c7):
    c = pkg.default_config()
    (c.pruning_level, c.elag_r1, c.elag_rep, c.elag_spc, c.elag_rep2, c.elag_spc2, c.elag_h0) = c7
    return c


def _special_mask(rng, N):
    """random mask with planted R0 / R1 / REP / SPC / REP2 / SPC2 groups"""
    pats = [0, 0xFFFF, 0x8000, 0xFFFE, 0xC000, 0xFFFC]
    mask = (rng.random(N) < rng.choice([0.2, 0.5, 0.8])).astype(np.uint8)
    for g in range(N // 16):
        if rng.random() < 0.6:
            p = int(rng.choice(pats))
            mask[16 * g:16 * g + 16] = [(p >> k) & 1 for k in range(16)]
    return mask


SWEEP_EXTRA = ((2, 1, 1, 1, 0, 0, 0), (2, 1, 1, 1, 1, 1, 1), (1, 0, 1, 0, 1, 0, 0), (1, 0, 0, 1, 0, 1, 0))


def test_sweep_configs_fsm_equals_recursive(oracle_mod):
    rng = np.random.default_rng(5)
    for trial in range(40):
        N = int(2 ** rng.integers(5, 12))
        mask = _special_mask(rng, N)
        llr = rng.integers(-32, 32, size=(6, N)).astype(np.int8)
        for c7 in oracle_mod.SWEEP_CONFIGS + SWEEP_EXTRA:
            np.testing.assert_array_equal(oracle_mod.decode_fsm(mask, llr, config=c7),
                                          oracle_mod.decode_rec(mask, llr, config=c7), err_msg=str((trial, c7)))


def test_sweep_configs_schedule_equals_fsm(pkg, oracle_mod):
    rng = np.random.default_rng(6)
    for trial in range(24):
        N = int(2 ** rng.integers(5, 12))
        mask = _special_mask(rng, N)
        llr = rng.integers(-32, 32, size=(4, N)).astype(np.int8)
        for c7 in oracle_mod.SWEEP_CONFIGS + SWEEP_EXTRA:
            dec = pkg.Decoder(mask, config=_config(pkg, c7))
            np.testing.assert_array_equal(util.run_schedule(dec.schedule(), N, llr),
                                          oracle_mod.decode_fsm(mask, llr, config=c7), err_msg=str((trial, c7)))


@pytest.mark.parametrize("c7", [(0, 0, 0, 0, 0, 0, 0), (1, 1, 1, 1, 1, 1, 0), (2, 1, 0, 0, 0, 0, 1),
                                (2, 1, 1, 1, 0, 0, 0)])
def test_sweep_op_census_matches_fsm_states(pkg, oracle_mod, c7):
    mask = util.mask("frozen_n_2048_k_1024")
    dec = pkg.Decoder(mask, config=_config(pkg, c7))
    oc = dec.stats["op_count"]
    _, st = oracle_mod.decode_fsm(mask, np.zeros((1, mask.size), np.int8), return_counts=True, config=c7)
    assert oc.get("FLEAF", 0) + oc.get("GLEAF", 0) == st["R"]
    assert oc.get("REP", 0) == st["F_REP"] and oc.get("R1", 0) == st["G_R1"] and oc.get("SPC", 0) == st["G_SPC"]
    assert oc.get("G", 0) + oc.get("GLEAF", 0) == st["G"]
    if c7[0] == 2 and not c7[6]:
        # ELAG_H0 = 0: F_R0 states instead of the H0 route; the schedule keeps the
        # equivalent H0 ops (H over zeros == H0)
        assert oc.get("H", 0) + oc.get("H0", 0) == st["H"] and st["H0"] == 0
        assert oc.get("H0", 0) == st["F_R0"]
    else:
        assert oc.get("H", 0) == st["H"] and oc.get("H0", 0) == st["H0"]
    if c7[0] < 2:
        assert st["F_REP"] == st["G_R1"] == st["G_SPC"] == st["H0"] == 0


def test_sweep_configs_change_results(pkg, oracle_mod):
    """the sweep points are different decoders (pruned decoders differ from plain SC on noisy
    frames); every config still decodes noiseless codewords"""
    mask = util.mask("FB_N1024_K512")
    llr, x = util.synth_frames(mask, 200, ebn0_db=1.0, seed=3)
    outs = {c7: oracle_mod.decode_fsm(mask, llr, config=c7) for c7 in oracle_mod.SWEEP_CONFIGS}
    assert len({o.tobytes() for o in outs.values()}) >= 3
    clean = np.where(x == 1, -20, 20).astype(np.int8)
    for c7 in oracle_mod.SWEEP_CONFIGS:
        np.testing.assert_array_equal(oracle_mod.decode_fsm(mask, clean[:8], config=c7), x[:8])


def test_unsupported_configs(pkg):
    mask = util.mask("FB_N128_K64")
    for field, val in (("elag_rare", 1), ("llr_bits", 10), ("llr_bits", 4), ("par", 2), ("par", 128), ("par", 48),
                       ("sigmag", 2), ("extended", 2), ("pruning_level", 3)):
        c = pkg.default_config()
        setattr(c, field, val)
        with pytest.raises(pkg.PolarError):
            pkg.Decoder(mask, config=c)
    # N must hold two PAR words (INIT, my_module.h:294-309)
    c = pkg.default_config()
    c.par = 64
    with pytest.raises(pkg.PolarError):
        pkg.Decoder(np.ones(64, np.uint8), config=c)
    for field, val in (("llr_bits", 9), ("par", 64), ("par", 32), ("par", 8), ("par", 4), ("sigmag", 0)):
        c = pkg.default_config()
        setattr(c, field, val)
        dec = pkg.Decoder(mask, config=c)
        assert dec.stats["kernel"] == 2   # the interpreter compiled for the format
    c = pkg.default_config()
    c.extended = 0                        # EXTENDED 0: the per-mask kernel with saturating leaves
    assert pkg.Decoder(mask, config=c).stats["kernel"] == 1


@pytest.mark.parametrize("par", [32, 64])
def test_schedule_par_words_equals_fsm(pkg, oracle_mod, par):
    """PAR 32 / 64 (polar_parameters.h:8; script_tests.sh:11 sweeps 16 and 64): the schedule of
    16-LLR device words -- PAR-word leaves expanded into exact F / G / leaf records, PR1 leaf
    decoders as PLEAF records, REP / SPC per PAR word -- interpreted in numpy equals the
    literal FSM at that PAR under every pruning-sweep configuration."""
    rng = np.random.default_rng(par)
    for c7 in oracle_mod.SWEEP_CONFIGS + (None,):
        for name in ("FB_N1024_K512", "frozen_n_2048_k_1024", "frozen_n_4096_k_2048"):
            mask = util.mask(name)
            cfg = pkg.default_config()
            cfg.par = par
            if c7 is not None:
                (cfg.pruning_level, cfg.elag_r1, cfg.elag_rep, cfg.elag_spc, cfg.elag_rep2, cfg.elag_spc2,
                 cfg.elag_h0) = c7
            dec = pkg.Decoder(mask, cfg)
            llr, _ = util.synth_frames(mask, 12, ebn0_db=1.0, seed=par)
            llr[:, :40] = rng.integers(-32, 32, size=(12, 40))
            got = util.run_schedule(dec.schedule(), mask.size, llr, par=par)
            np.testing.assert_array_equal(got, oracle_mod.decode_fsm(mask, llr, config=c7, par=par),
                                          err_msg="%s %s" % (name, c7))
