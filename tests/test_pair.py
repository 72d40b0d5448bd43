"""Pair plans (polar_sc_pair.h, polar_sc_pairgen.cpp): one frame pair per wave, four words per
register, generated subtree decoders of up to 256 words, upper levels as loops over stage-slot
rows (LDS or HBM), optional grid tier.

CPU tests: plan statistics, hipRTC compilation of the generated source.
GPU tests: bit-exact against the oracle (literal my_module FSM) on reference masks and on
structured masks that put R0 / R1 / REP / SPC nodes at every size (the cross-row steps of the
nodes of 1, 2 and 4 words), for every waves-per-pair count, subtree size, LDS / HBM slot
placement and with the grid tier."""
import numpy as np
import pytest

import util
from test_gpu_parity import _assert_same


def pair(pkg, mask, **tuning):
    """a pair plan in the frame-pair layout (the automatic layout would decode small batches
    with its solo alternate, tests/test_solo.py)"""
    return pkg.Decoder(mask, tuning=dict(dict(layout=1), **tuning, kernel=3))


# the plan lists live in the package's build tooling (build() compiles them ahead)
from sc_polar_decoder_hls_amd._plansets import (PAR64_MASKS, PAIR_PARS, PARITY_MASKS, gpu_par64_plans, gpu_plans,  # noqa: F401
                                                struct_masks, struct_sub_words, structured_mask, wave_mask)


def run(pkg, torch, dec, llr):
    out = dec.decode(torch.from_numpy(np.ascontiguousarray(llr)).cuda())
    torch.cuda.synchronize()
    return pkg.unpack_bits(out.cpu().numpy(), dec.N)


def test_pair_plan_stats(pkg):
    s = pair(pkg, util.mask("frozen_n_65536_k_32768")).stats
    assert (s["kernel"], s["sub_words"], s["storage"]) == (3, 256, 1)
    assert s["n_sub_calls"] >= s["n_sub_kinds"] > 0 and s["tier_steps"] == 0
    # per pair: (G - 2 S) / 4 slot rows of 128 B (subtree roots read as F / G of their parents)
    # + G / 64 bit rows of 256 B; with the roots in a slot level of their own, (G - S) / 4
    assert s["scratch_bytes_per_wave"] == (4096 - 512) // 4 * 128 + 4096 // 64 * 256
    s1 = pair(pkg, util.mask("frozen_n_65536_k_32768"), sub_root=1).stats
    assert s1["scratch_bytes_per_wave"] == (4096 - 256) // 4 * 128 + 4096 // 64 * 256
    assert "_F(c.slot_ptr" in pair(pkg, util.mask("frozen_n_65536_k_32768")).kernel_source()
    assert "_F(c.slot_ptr" not in pair(pkg, util.mask("frozen_n_65536_k_32768"), sub_root=1).kernel_source()
    # automatic: fused from 16 subtrees per frame on (N = 16384, G = 4 S: slot roots)
    assert "_F(c.slot_ptr" not in pair(pkg, util.mask("frozen_n_16384_k_8192")).kernel_source()
    assert "_F(c.slot_ptr" in pair(pkg, util.mask("frozen_n_16384_k_8192"), sub_root=2).kernel_source()
    # waves per pair: more while the batch leaves SIMDs without 2 waves, never past one dispatch
    # round (1536 pairs x 2 waves of 248 registers would be two rounds at 2 waves per SIMD)
    c3 = pair(pkg, util.mask("frozen_n_65536_k_32768"))
    assert [c3.launch_info(b, cus=256)["waves_per_block"] for b in (4096, 3072, 2048, 512)] == [1, 1, 2, 8]
    s = pair(pkg, util.mask("frozen_n_2048_k_1024")).stats
    assert s["sub_words"] == 64
    s = pair(pkg, util.mask("frozen_n_262144_k_131072"), tier_words=1024).stats
    assert s["tier_words"] == 1024 and s["tier_steps"] > 20
    with pytest.raises(pkg.PolarError):
        pair(pkg, util.mask("frozen_n_4096_k_2048"), sub_words=256)   # > G / 2
    with pytest.raises(pkg.PolarError):
        pair(pkg, util.mask("frozen_n_4096_k_2048"), sub_words=16)    # < 32: 8-row slot groups


@pytest.mark.parametrize("N", [2048, 8192])
def test_pair_generated_code_emulated(pkg, oracle_mod, N):
    """CPU: the generated subtree decoders transpiled and run on emulated 64-lane waves
    (tests/pair_emu.py: DPP rows, permlane swaps) with the upper levels restated on the same
    layout decode bit-exactly like the oracle -- structured masks, every subtree size."""
    import pair_emu
    for i, mask in enumerate(struct_masks(N)):
        llr, _ = util.synth_frames(mask, 2, ebn0_db=0.5, seed=i)
        ref = oracle_mod.decode_fsm(mask, llr)
        for sw in struct_sub_words(N):
            dec = pair(pkg, mask, sub_words=sw)
            _assert_same(pair_emu.decode(dec, llr), ref, "emulated N=%d mask %d S=%d" % (N, i, sw))
    mask = util.mask("frozen_n_2048_k_1024")
    rng = np.random.default_rng(2)
    u = rng.integers(0, 2, size=(4, mask.size), dtype=np.uint8) & mask[None, :]
    x = util.encode_np(u)
    llr = np.where(x == 1, -9, 9).astype(np.int8)
    for sw in (32, 64):
        assert (pair_emu.decode(pair(pkg, mask, sub_words=sw), llr) == x).all()


@pytest.mark.gpu
def test_pair_subtrees_equal_emulation(pkg, cuda):
    """Every generated subtree decoder on the device (polar_sc_debug_subtree) equals its CPU
    emulation on random root LLRs."""
    import pair_emu
    rng = np.random.default_rng(5)
    for name, sw in (("frozen_n_2048_k_1024", 64), ("frozen_n_2048_k_1024", 32), ("frozen_n_8192_k_4096", 256)):
        dec = pair(pkg, util.mask(name), sub_words=sw)
        subs = pair_emu.Sub(dec.kernel_source(), dec.stats["n_sub_kinds"])
        for sid in range(dec.stats["n_sub_kinds"]):
            rows = pair_emu.random_rows(rng, sw)
            got = dec.debug_subtree(sid, rows)
            ref = pair_emu.run_sub(dec, sid, rows, subs)
            assert (got == ref).all(), "%s S=%d subtree %d" % (name, sw, sid)


@pytest.mark.parametrize("sub_words", [32, 128])
def test_pair_source_compiles(pkg, sub_words):
    """hipRTC build of a generated pair source (host only)."""
    dec = pair(pkg, util.mask("frozen_n_8192_k_4096"), sub_words=sub_words)
    assert dec.compile()


@pytest.mark.gpu
@pytest.mark.parametrize("name,batch", PARITY_MASKS)
def test_pair_parity_masks(pkg, cuda, oracle_mod, name, batch):
    mask = util.mask(name)
    llr, _ = util.synth_frames(mask, batch, ebn0_db=1.0, seed=batch)
    _assert_same(run(pkg, cuda, pair(pkg, mask), llr), oracle_mod.decode_fsm(mask, llr), name)


@pytest.mark.gpu
@pytest.mark.parametrize("N", [2048, 8192, 32768])
def test_pair_parity_structured(pkg, cuda, oracle_mod, N):
    """R0 / R1 / REP / SPC nodes of every size, AWGN and edge LLRs (zeros, -32, saturated)."""
    rng = np.random.default_rng(N + 1)
    for rep, mask in enumerate(struct_masks(N)):
        llr, _ = util.synth_frames(mask, 6, ebn0_db=0.5, seed=rep)
        edge = rng.choice(np.array([0, 0, 1, -1, 31, -31, -32, 5], np.int8), size=(3, N))
        llr = np.concatenate([llr, edge])
        for sw in struct_sub_words(N):
            dec = pair(pkg, mask, sub_words=sw)
            _assert_same(run(pkg, cuda, dec, llr), oracle_mod.decode_fsm(mask, llr), "N=%d rep %d S=%d" % (N, rep, sw))


@pytest.mark.gpu
@pytest.mark.parametrize("wpg", [1, 2, 4, 8])
def test_pair_waves_per_pair(pkg, cuda, oracle_mod, wpg):
    """W waves per frame pair split the upper F / G / R1 / SPC / H ops (the SPC partials meet
    in LDS); subtrees and REP run on the lead wave."""
    for name in ("frozen_n_16384_k_8192", None):
        mask = util.mask(name) if name else wave_mask()
        llr, _ = util.synth_frames(mask, 7, ebn0_db=1.0, seed=wpg)
        dec = pair(pkg, mask, waves_per_group=wpg, sub_words=64)
        _assert_same(run(pkg, cuda, dec, llr), oracle_mod.decode_fsm(mask, llr), "%s W=%d" % (name, wpg))


@pytest.mark.gpu
@pytest.mark.parametrize("lds_slots,batch", [(256, 300), (1024, 4096)])
def test_pair_forced_lds_levels(pkg, cuda, oracle_mod, lds_slots, batch):
    """polar_sc_tuning.lds_slots on a pair plan: the slot levels of nodes up to that many
    words sit in LDS whatever the batch -- fewer than the default at 300 frames (W = 8, where
    every level fits), more at 4096 (W = 1, 8 pairs per CU: the default keeps one level)."""
    mask = util.mask("frozen_n_65536_k_32768")
    llr, _ = util.synth_frames(mask, batch, ebn0_db=1.0, seed=lds_slots)
    dec = pair(pkg, mask, lds_slots=lds_slots)
    info, dflt = dec.launch_info(batch), pair(pkg, mask).launch_info(batch)
    assert info["lds_row0"] != dflt["lds_row0"], (info, dflt)
    got = run(pkg, cuda, dec, llr)
    _assert_same(got, run(pkg, cuda, pair(pkg, mask), llr), "lds_slots %d vs default" % lds_slots)
    idx = np.r_[0:3, batch - 3:batch]
    _assert_same(got[idx], oracle_mod.decode_fsm(mask, llr[idx]), "lds_slots %d vs oracle" % lds_slots)


@pytest.mark.gpu
def test_pair_all_hbm_slots_large_batch(pkg, cuda, oracle_mod):
    """A batch large enough that no slot level fits the LDS share of a pair (every level in
    HBM): equal to the hybrid kernel on every frame and to the oracle on a sample."""
    mask = util.mask("frozen_n_2048_k_1024")
    B = 40001
    llr, _ = util.synth_frames(mask, B, ebn0_db=1.5, seed=3)
    got = run(pkg, cuda, pair(pkg, mask), llr)
    ref = run(pkg, cuda, pkg.Decoder(mask, tuning={"kernel": 2}), llr)
    _assert_same(got, ref, "pair vs hybrid")
    idx = np.r_[0:40, B - 40:B]
    _assert_same(got[idx], oracle_mod.decode_fsm(mask, llr[idx]), "pair vs oracle")


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 4, 9])
def test_pair_grid_tier(pkg, cuda, oracle_mod, batch):
    """Grid tier forced at 512 words on N = 32768 (ragged batches): grid launches of the upper
    F / G over all pairs, the segments in between."""
    mask = util.mask("frozen_n_32768_k_29492")
    llr, _ = util.synth_frames(mask, batch, ebn0_db=3.0, seed=batch)
    dec = pair(pkg, mask, tier_words=512, sub_words=128)
    assert dec.stats["tier_steps"] > 0
    _assert_same(run(pkg, cuda, dec, llr), oracle_mod.decode_fsm(mask, llr), "tier batch %d" % batch)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", [1, 2])
def test_subtree_root_slot_vs_fused(pkg, cuda, oracle_mod, layout):
    """Subtree roots from a slot level of their own (sub_root 1) and as F / G of the parent's
    slot rows (the default): equal on every frame of a C3-sized sample, equal to the oracle."""
    mask = util.mask("frozen_n_65536_k_32768")
    llr, _ = util.synth_frames(mask, 6, ebn0_db=1.0, seed=31)
    a = run(pkg, cuda, pair(pkg, mask, layout=layout, sub_root=2), llr)
    b = run(pkg, cuda, pair(pkg, mask, layout=layout, sub_root=1), llr)
    _assert_same(a, b, "fused vs slot roots, layout %d" % layout)
    _assert_same(a, oracle_mod.decode_fsm(mask, llr), "fused roots vs oracle, layout %d" % layout)


@pytest.mark.gpu
def test_pair_c5_sample(pkg, cuda, oracle_mod):
    mask = util.mask("frozen_n_262144_k_131072")
    llr, _ = util.synth_frames(mask, 3, ebn0_db=1.0, seed=5)
    ref = oracle_mod.decode_fsm(mask, llr)
    _assert_same(run(pkg, cuda, pair(pkg, mask), llr), ref, "C5 pair")
    _assert_same(run(pkg, cuda, pair(pkg, mask, tier_words=1024), llr), ref, "C5 pair tier")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["frozen_n_16384_k_8192", "frozen_n_65536_k_32768"])
def test_pair_misaligned_channel(pkg, cuda, oracle_mod, name):
    """Channel rows at an odd device address: the root chains take the byte-load path instead
    of the dword loads + quad transpose (chan8b vs chan8a), with the same bits."""
    mask = util.mask(name)
    llr, _ = util.synth_frames(mask, 3, ebn0_db=1.0, seed=11)
    flat = cuda.zeros(llr.size + 16, dtype=cuda.int8, device="cuda")
    view = flat[1:1 + llr.size].view(llr.shape)
    view.copy_(cuda.from_numpy(llr))
    dec = pair(pkg, mask)
    out = dec.decode(view)
    cuda.cuda.synchronize()
    _assert_same(pkg.unpack_bits(out.cpu().numpy(), mask.size), oracle_mod.decode_fsm(mask, llr), "misaligned " + name)


def test_pair_register_budget(pkg):
    """The launch guard (polar_sc_jit.cpp kernel_regs / fit_waves, polar_sc_plan_launch_info):
    the registers of a generated kernel come from its kernel descriptor (granulated VGPR +
    AGPR count, equal to the ELF metadata's unified .vgpr_count rounded to 8), and a launch
    never puts more waves of a block on a SIMD than its 512 registers per lane hold. Checked on
    C5 and on the chain_max = 4 plans of the structured N = 32768 mask -- the configuration of
    the round-3 dispatch abort -- which hipRTC compiles to exactly 256 registers (the
    512-thread launch bound), so the full 8-wave block still fits."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import check_rtc_registers as cr
    cache = os.path.join(os.path.dirname(pkg._build.LIB), "rtc_cache")
    plans = [(util.mask("frozen_n_262144_k_131072"), {}),
             (struct_masks(32768)[0], {"sub_words": 64, "chain_max": 4, "sub_root": 1}),
             (struct_masks(32768)[0], {"sub_words": 256, "chain_max": 4, "sub_root": 1})]
    for m, tun in plans:
        dec = pair(pkg, m, **tun)
        for batch in (9, 64, 4096, 40001):
            info = dec.launch_info(batch)
            W, regs = info["waves_per_block"], info["regs"]
            assert 0 < regs <= 512 and W >= 1, info
            assert -(-W // 4) * regs <= 512, info
        co = cr.find_code(cache, info["code_key"])   # (also checks the key's Python restatement)
        assert co, info["code_key"]
        meta = {name: (vgpr, wg) for name, vgpr, _, wg in cr.kernels(co)}
        vgpr, wg = meta["polar_sc_pair_kernel"]
        assert regs == -(-vgpr // 8) * 8, (regs, vgpr)
        assert not cr.over_budget(vgpr, 0, wg)[0]
    # an automatic 8-wave launch (small batch) of the chain_max = 4 kernel: 2 waves of 256
    # registers per SIMD
    info = pair(pkg, struct_masks(32768)[0], sub_words=64, chain_max=4, sub_root=1).launch_info(9)
    assert (info["regs"], info["waves_per_block"]) == (256, 8), info


def test_forced_kernel_errors(pkg):
    """A forced kernel / subtree size the plan cannot use is an error, not a silent fallback."""
    with pytest.raises(pkg.PolarError):
        pkg.Decoder(util.mask("FB_N1024_K512"), tuning={"kernel": 3})     # N < 2048: no pair kernel
    with pytest.raises(pkg.PolarError):
        pkg.Decoder(util.mask("frozen_n_8192_k_4096"), tuning={"kernel": 2, "sub_words": 256})   # hybrid <= 128
    assert pkg.Decoder(util.mask("frozen_n_8192_k_4096"), tuning={"kernel": 2, "sub_words": 128}).stats["kernel"] == 2


def par64_config(pkg, q=6, par=64):
    c = pkg.default_config()
    c.par, c.llr_bits = par, q
    return c


def test_pair_par64_plan(pkg):
    """PAR 64 (script_tests.sh:11, 124) takes the pair kernel: subtrees cut at PAR-word
    multiples, the PAR word's exact leaf expanded into F / G_extended / 16-LLR leaf records."""
    d = pkg.Decoder(util.mask("frozen_n_65536_k_32768"), config=par64_config(pkg))
    s = d.stats
    assert (s["kernel"], s["sub_words"]) == (3, 256) and s["n_sub_calls"] > 0
    src = d.kernel_source()
    assert "#define POLAR_LPAR 6" in src and "G_split_x" in src
    d = pkg.Decoder(util.mask("frozen_n_65536_k_32768"), config=par64_config(pkg, par=32))
    assert d.stats["kernel"] == 3 and "#define POLAR_LPAR 5" in d.kernel_source()


@pytest.mark.gpu
@pytest.mark.parametrize("par", PAIR_PARS)
@pytest.mark.parametrize("name,batch", PAR64_MASKS)
def test_pair_par64_parity(pkg, cuda, oracle_mod, name, batch, par):
    """PAR 32 / 64 on the pair kernel against the oracle's literal FSM at that PAR: REP over the
    PAR word's exact ADD_TREE (PAR 64: words (0, 2), (1, 3), halves, positions; PAR 32: words
    (0, 1), positions) with the 2^(Q+LPAR-1)-1 clamp, SPC ties by (PAR word, bitrev_LPAR
    (position)), G_extended inside the PAR word."""
    mask = util.mask(name)
    llr, _ = util.synth_frames(mask, batch, ebn0_db=1.0, seed=batch)
    edge = np.random.default_rng(batch).choice(np.array([0, 0, 1, -1, 31, -31, -32, 5], np.int8), size=(2, mask.size))
    llr = np.concatenate([llr, edge])
    dec = pkg.Decoder(mask, config=par64_config(pkg, par=par))
    assert dec.stats["kernel"] == 3
    _assert_same(run(pkg, cuda, dec, llr), oracle_mod.decode_fsm(mask, llr, par=par), "PAR %d %s" % (par, name))


@pytest.mark.gpu
@pytest.mark.parametrize("par", PAIR_PARS)
@pytest.mark.parametrize("N", [8192, 32768])
def test_pair_par64_structured(pkg, cuda, oracle_mod, N, par):
    """PAR 32 / 64 on structured masks (R0 / R1 / REP / SPC nodes of every size), subtrees of
    64 and 256 words, AWGN and edge LLRs."""
    rng = np.random.default_rng(N + 64)
    for rep, mask in enumerate(struct_masks(N)[:2]):
        llr, _ = util.synth_frames(mask, 4, ebn0_db=0.5, seed=rep)
        edge = rng.choice(np.array([0, 0, 1, -1, 31, -31, -32, 5], np.int8), size=(3, N))
        llr = np.concatenate([llr, edge])
        ref = oracle_mod.decode_fsm(mask, llr, par=par)
        for sw in (64, 256):
            dec = pkg.Decoder(mask, config=par64_config(pkg, par=par), tuning={"kernel": 3, "sub_words": sw})
            _assert_same(run(pkg, cuda, dec, llr), ref, "PAR %d N=%d rep %d S=%d" % (par, N, rep, sw))


def test_launch_info_and_compile_from_two_threads(pkg):
    """polar_sc_plan_launch_info compiles under the plan lock: launch_info and
    compile on the same uncompiled plan from two threads agree, and the plan is compiled once
    (every launch_info reports the same machine code)."""
    import threading
    dec = pair(pkg, util.mask("frozen_n_2048_k_1024"), sub_words=32)
    infos, errs = [], []

    def info():
        try:
            infos.append(dec.launch_info(64))
        except Exception as e:   # pragma: no cover - reported below
            errs.append(e)

    def comp():
        try:
            dec.compile()
        except Exception as e:   # pragma: no cover
            errs.append(e)

    ts = [threading.Thread(target=f) for f in (info, comp, info, comp)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    assert len({i["code_key"] for i in infos}) == 1 and infos[0]["regs"] > 0, infos
