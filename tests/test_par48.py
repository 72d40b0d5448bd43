"""PAR 4 / 8 (script_RTL_sim.sh:97-330; polar_parameters.h:8) on the generated pair kernel: the
PAR words are aligned lane groups of a device word (polar_sc_device.h PAR 4 / 8 section). The
host compiles the tree down to one-word nodes (polar_sc_host.cpp compile_node, ppw > 1); each
one-word leaf record decodes its whole word tree with its frozen bits and group classes
(word_info: R0 / R1 / REP / SPC / RN and the PRUNING_LEVEL 1 leaf kinds) as template
constants (word_gen), REP nodes run the exact per-group trees chained in order
(polar_sc_pair.h rep_groups_*), and SPC keys order the lanes by (word, group,
bitrev_{PAR}(position)) (spc_lane_key).

CPU: plan selection and the generated source. GPU: bit-exact with the literal FSM at PAR 4 / 8
on reference, planted (every pruned group class) and structured masks, AWGN and edge LLRs,
PRUNING_LEVEL 0 / 1 / 2, EXTENDED 0 / 1, LLR_BITS 5 .. 9, SIGMAG and CA2 (the word trees on
two's complement values converted from the split form; MIN on the leftmost path reaches the leaf
of word 0 through the key-min F of the _L decoder)."""
import numpy as np
import pytest

import util
from test_gpu_parity import _assert_same
from sc_polar_decoder_hls_amd._plansets import c7_fields, par48_gpu_items


def cfg(pkg, **kw):
    c = pkg.default_config()
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def test_par48_plans_take_the_pair_kernel(pkg):
    m = util.mask("frozen_n_16384_k_8192")
    for par in (4, 8):
        for q in (5, 6, 8, 9):
            for ext in (0, 1):
                for pl in (0, 1, 2):
                    d = pkg.Decoder(m, config=cfg(pkg, par=par, llr_bits=q, extended=ext, pruning_level=pl))
                    assert d.stats["kernel"] == 3, (par, q, ext, pl, d.stats["kernel"])
            # CA2: the word trees on two's complement values, every pruning level
            for pl in (0, 1, 2):
                d = pkg.Decoder(m, config=cfg(pkg, par=par, llr_bits=q, sigmag=0, pruning_level=pl))
                assert d.stats["kernel"] == 3, (par, q, "ca2", pl, d.stats["kernel"])
        src = pkg.Decoder(m, config=cfg(pkg, par=par, sigmag=0)).kernel_source()
        assert "#define POLAR_CA2 1" in src and "polar_psub_0_L(" in src and "F_split_rep<" in src
        src = pkg.Decoder(m, config=cfg(pkg, par=par)).kernel_source()
        assert "#define POLAR_LPAR %d" % (2 if par == 4 else 3) in src
        assert "leaf_word_gen<" in src and "leaf_gen<" not in src
    # a forced solo layout is refused (the solo half ops are PAR 16 only)
    with pytest.raises(Exception):
        pkg.Decoder(m, config=cfg(pkg, par=4), tuning={"layout": 2, "kernel": 3})


def test_par48_subtrees_cut_in_device_words(pkg):
    """compile_node's subtree cut counts device words (a PAR 4 group is a quarter word): the
    subtree records cover sub_words words each and tile the codeword."""
    m = util.mask("frozen_n_16384_k_8192")
    for par in (4, 8):
        for S in (32, 64, 256):
            d = pkg.Decoder(m, config=cfg(pkg, par=par, pruning_level=0), tuning={"kernel": 3, "sub_words": S})
            assert d.stats["sub_words"] == S
            assert d.stats["n_sub_calls"] == m.size // 16 // S, (par, S, d.stats)


def test_par48_leaf_records_carry_the_word_classes(pkg):
    """Every one-word leaf record of a PAR 4 / 8 plan names its word's frozen bits and group
    classes (FB, INFO template arguments) -- equal words share one instantiation."""
    m = util.mask("frozen_n_4096_k_2048")
    d = pkg.Decoder(m, config=cfg(pkg, par=4))
    src = d.kernel_source()
    import re
    calls = re.findall(r"leaf_word_gen<0x([0-9a-f]+)u, 0x([0-9a-f]+)u>", src)
    assert calls
    for fb, info in calls:
        fb, info = int(fb, 16), int(info, 16)
        assert (info >> 28) & 1 == 1 and fb < (1 << 16)   # PRUNING_LEVEL 2 (shipped)


@pytest.mark.parametrize("par", [8, 4])
def test_par48_generated_code_emulated(pkg, oracle_mod, par):
    """CPU: the generated PAR 4 / 8 code (leaf_word_gen word trees, rep_groups_* REP chains,
    group-ordered SPC keys, the upper loops' REP) emulated on 64-lane waves (tests/pair_emu.py)
    equals the FSM at PRUNING_LEVEL 0 / 1 / 2 on a reference mask, a planted mask with every
    group class and the N = 1024 K = 922 code of script_RTL_sim.sh's PAR loop."""
    import pair_emu
    from sc_polar_decoder_hls_amd._plansets import planted_mask
    rng = np.random.default_rng(par)
    masks = [util.mask("frozen_n_2048_k_1024"), planted_mask(rng, 2048, par), util.mask("frozen_n_1024_k_922")]
    try:
        for i, m in enumerate(masks):
            for c7 in ((2, 1, 1, 1, 0, 0, 1), (1, 1, 1, 1, 1, 1, 0), (0, 0, 0, 0, 0, 0, 0)):
                c = cfg(pkg, par=par, **c7_fields(c7))
                dec = pkg.Decoder(m, config=c, tuning={"kernel": 3, "sub_words": 32})
                llr, _ = util.synth_frames(m, 3, ebn0_db=1.0, seed=par + i)
                llr = np.clip(llr, -31, 31).astype(np.int8)
                _assert_same(pair_emu.decode(dec, llr), oracle_mod.decode_fsm(m, llr, config=c7, par=par),
                             "emulated PAR %d mask %d %s" % (par, i, c7))
    finally:
        pair_emu.configure()


def test_par48_group_order_is_needed(pkg, oracle_mod, monkeypatch):
    """A mutation of the emulation (the groups of a word chained in reverse order) differs from
    the FSM: the REP chains' group order is exercised, not vacuous."""
    import pair_emu
    orig = pair_emu.group_order
    monkeypatch.setattr(pair_emu, "group_order", lambda t, gr: orig(t, gr)[::-1])
    orig_chain = pair_emu.group_chain
    monkeypatch.setattr(pair_emu, "group_chain", lambda CNT, acc, t, gr: orig_chain(CNT, acc, t, np.asarray(gr) ^ (CNT - 1)))
    m = util.mask("frozen_n_2048_k_1024")
    dec = pkg.Decoder(m, config=cfg(pkg, par=4), tuning={"kernel": 3, "sub_words": 32})
    llr, _ = util.synth_frames(m, 8, ebn0_db=0.0, seed=9)
    llr = np.clip(llr, -31, 31).astype(np.int8)
    try:
        assert (pair_emu.decode(dec, llr) != oracle_mod.decode_fsm(m, llr, par=4)).any()
    finally:
        pair_emu.configure()


def frames(mask, q, n_awgn, n_edge, seed):
    rng = np.random.default_rng(seed)
    amp = (1 << (q - 1)) - 1
    awgn, _ = util.synth_frames(mask, n_awgn, ebn0_db=1.0, seed=seed)
    awgn = np.clip(awgn.astype(np.int32) * (1 << q) // 64, -amp, amp)
    e = rng.integers(-(amp + 1), amp + 1, size=(n_edge, mask.size))
    e[:, rng.integers(0, mask.size, mask.size // 8)] = -(amp + 1)
    e[:, rng.integers(0, mask.size, mask.size // 8)] = 0
    e[0, :64] = -(amp + 1)                        # (CA2: MIN on the leftmost path)
    llr = np.concatenate([awgn, e])
    return llr.astype(np.int16 if q > 8 else np.int8)


@pytest.mark.gpu
@pytest.mark.parametrize("item", par48_gpu_items(), ids=lambda it: it[0])
def test_par48_pair_kernel_gpu(pkg, cuda, oracle_mod, item):
    name, mask, fields, tun = item
    c = cfg(pkg, **fields)
    dec = pkg.Decoder(mask, config=c, tuning=tun)
    assert dec.stats["kernel"] == 3, (name, dec.stats["kernel"])
    q = fields.get("llr_bits", 6)
    llr = frames(mask, q, 5, 4, seed=mask.size + q + c.par)
    out = dec.decode(cuda.from_numpy(llr).cuda())
    cuda.cuda.synchronize()
    c7 = (c.pruning_level, c.elag_r1, c.elag_rep, c.elag_spc, c.elag_rep2, c.elag_spc2, c.elag_h0)
    ref = oracle_mod.decode_fsm(mask, llr, config=c7, llr_bits=q, par=c.par, sigmag=c.sigmag, extended=c.extended)
    _assert_same(pkg.unpack_bits(out.cpu().numpy(), mask.size), ref, "PAR %d %s" % (c.par, name))


@pytest.mark.gpu
@pytest.mark.parametrize("par", [4, 8])
def test_par48_pair_kernel_full_batch(pkg, cuda, oracle_mod, par):
    """The format_speed shape (N = 16384, 4096 frames): sampled against the FSM, the batch
    consistent, and noiseless codewords decode exactly."""
    mask = util.mask("frozen_n_16384_k_8192")
    dec = pkg.Decoder(mask, config=cfg(pkg, par=par))
    llr = np.concatenate([frames(mask, 6, 2, 2, seed=par)] * 1024)
    out = dec.decode(cuda.from_numpy(llr).cuda())
    cuda.cuda.synchronize()
    got = pkg.unpack_bits(out[:4].cpu().numpy(), mask.size)
    _assert_same(got, oracle_mod.decode_fsm(mask, llr[:4], par=par), "full PAR %d" % par)
    assert (out.view(1024, 4, -1) == out[:4].unsqueeze(0)).all()
    rng = np.random.default_rng(par)
    u = rng.integers(0, 2, size=(4096, mask.size), dtype=np.uint8) & mask[None, :]
    x = util.encode_np(u)
    out = dec.decode(cuda.from_numpy(np.where(x == 1, -17, 17).astype(np.int8)).cuda())
    cuda.cuda.synchronize()
    assert (pkg.unpack_bits(out.cpu().numpy(), mask.size) == x).all(), par
