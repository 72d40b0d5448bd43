"""Solo layout of the pair plans (polar_sc_pair.h POLAR_SOLO, polar_sc_tuning.layout = 2): one
frame per wave, the two 16-bit halves carry the frame's words 8 j + 4 h + r, so an op on a
node of >= 16 words is n / 8 instructions instead of n / 4; nodes of 8 words are split across
the halves (the generated "half ops"), nodes of 4 words and below are the pair code's.

CPU: the generated solo code emulated (tests/pair_emu.py) equals the oracle; plan statistics
and argument checks. GPU: bit-exact against the oracle on reference masks, structured masks
with R0 / R1 / REP / SPC nodes of every size (AWGN and edge LLRs), every waves-per-frame count,
subtrees of 64 .. 512 words, the grid tier, C5; every subtree decoder equals its emulation."""
import numpy as np
import pytest

import util
from test_gpu_parity import _assert_same
from sc_polar_decoder_hls_amd._plansets import PARITY_MASKS, solo_sub_words, struct_masks, wave_mask


def solo(pkg, mask, **tuning):
    return pkg.Decoder(mask, tuning=dict(tuning, kernel=3, layout=2))


def run(pkg, torch, dec, llr):
    out = dec.decode(torch.from_numpy(np.ascontiguousarray(llr)).cuda())
    torch.cuda.synchronize()
    return pkg.unpack_bits(out.cpu().numpy(), dec.N)


def edge_llr(rng, n, N):
    return rng.choice(np.array([0, 0, 1, -1, 31, -31, -32, 5], np.int8), size=(n, N))


def test_solo_plan_stats(pkg):
    m = util.mask("frozen_n_65536_k_32768")
    d = solo(pkg, m)
    s = d.stats
    # default subtree size of a solo plan: min(512, N / 32) words, forced or automatic
    assert (s["kernel"], s["sub_words"], s["storage"]) == (3, 512, 1)
    # per frame: (G - S) / 8 slot rows of 128 B + G / 128 bit rows of 256 B (solo plans keep the
    # subtree roots in a slot level of their own; sub_root 2 reads them as F / G of the parents)
    assert s["scratch_bytes_per_wave"] == (4096 - 512) // 8 * 128 + 4096 // 128 * 256
    assert s["lds_bytes_per_wave"] == 512 // 8 * 128
    s2 = solo(pkg, m, sub_root=2).stats
    assert s2["scratch_bytes_per_wave"] == (4096 - 1024) // 8 * 128 + 4096 // 128 * 256
    s3 = solo(pkg, m, sub_words=256).stats
    assert s3["scratch_bytes_per_wave"] == (4096 - 256) // 8 * 128 + 4096 // 128 * 256
    assert "#define POLAR_SOLO 1" in d.kernel_source()
    assert "POLAR_SOLO" not in pkg.Decoder(m).kernel_source()
    info = d.launch_info(64, cus=256)
    assert info["blocks"] == 64 and info["waves_per_block"] == 8, info   # one block per frame
    assert info["alt_layout"] == 0 and info["alt_max_batch"] == 0   # a forced layout has no alternate
    # the automatic layout: the solo alternate takes batches of <= 2 frames per SIMD, with the
    # solo defaults whatever the pair plan's tuning
    for tun in (None, {"sub_words": 64, "waves_per_group": 2}):
        a = pkg.Decoder(m, tuning=tun)
        for cus, b in ((256, 2048), (64, 512)):
            i1, i2 = a.launch_info(b, cus=cus), a.launch_info(b + 1, cus=cus)
            assert (i1["alt_layout"], i1["alt_max_batch"]) == (2, b), (tun, i1)
            assert (i1["layout"], i1["sub_words"], i2["layout"]) == (2, 512, 1), (tun, i1, i2)
    assert pkg.Decoder(m, tuning={"layout": 1}).launch_info(64, cus=256)["alt_layout"] == 0
    assert solo(pkg, m, sub_words=512).stats["sub_words"] == 512
    with pytest.raises(pkg.PolarError):
        solo(pkg, util.mask("frozen_n_4096_k_2048"), sub_words=32)    # < 64: 8-row slot groups
    with pytest.raises(pkg.PolarError):
        pair_dec = pkg.Decoder(m, tuning={"kernel": 3, "sub_words": 512})   # pair: <= 256
        del pair_dec


@pytest.mark.parametrize("N", [2048, 8192])
def test_solo_generated_code_emulated(pkg, oracle_mod, N):
    """CPU: solo subtree decoders transpiled and run on emulated 64-lane waves, the upper
    levels restated on the solo layout: bit-exact with the oracle, structured masks, every
    subtree size, AWGN and edge LLRs."""
    import pair_emu
    rng = np.random.default_rng(N + 2)
    for i, mask in enumerate(struct_masks(N)):
        llr, _ = util.synth_frames(mask, 2, ebn0_db=0.5, seed=i)
        llr = np.concatenate([llr, edge_llr(rng, 1, N)])
        ref = oracle_mod.decode_fsm(mask, llr)
        for sw in solo_sub_words(N):
            _assert_same(pair_emu.decode(solo(pkg, mask, sub_words=sw), llr), ref, "emulated N=%d mask %d S=%d" % (N, i, sw))
            if sw < N // 32:   # roots as F / G of their parents
                _assert_same(pair_emu.decode(solo(pkg, mask, sub_words=sw, sub_root=2), llr), ref,
                             "emulated N=%d mask %d S=%d fused roots" % (N, i, sw))


@pytest.mark.gpu
def test_solo_subtrees_equal_emulation(pkg, cuda):
    """Every generated solo subtree decoder on the device (polar_sc_debug_subtree) equals its
    CPU emulation on random root LLRs."""
    import pair_emu
    rng = np.random.default_rng(6)
    for name, sw in (("frozen_n_2048_k_1024", 64), ("frozen_n_8192_k_4096", 256), ("frozen_n_16384_k_8192", 512)):
        dec = solo(pkg, util.mask(name), sub_words=sw)
        subs = pair_emu.Sub(dec.kernel_source(), dec.stats["n_sub_kinds"])
        for sid in range(dec.stats["n_sub_kinds"]):
            rows = pair_emu.random_rows(rng, sw // 2)
            got = dec.debug_subtree(sid, rows)
            ref = pair_emu.run_sub(dec, sid, rows, subs)
            assert (got == ref).all(), "%s S=%d subtree %d" % (name, sw, sid)


@pytest.mark.gpu
@pytest.mark.parametrize("name,batch", PARITY_MASKS)
def test_solo_parity_masks(pkg, cuda, oracle_mod, name, batch):
    mask = util.mask(name)
    llr, _ = util.synth_frames(mask, batch, ebn0_db=1.0, seed=batch + 100)
    _assert_same(run(pkg, cuda, solo(pkg, mask), llr), oracle_mod.decode_fsm(mask, llr), "solo " + name)


@pytest.mark.gpu
@pytest.mark.parametrize("N", [2048, 8192, 32768])
def test_solo_parity_structured(pkg, cuda, oracle_mod, N):
    """R0 / R1 / REP / SPC nodes of every size (the half ops of 8-word nodes, the cross-half
    REP order and SPC ties), AWGN and edge LLRs (zeros, -32, saturated)."""
    rng = np.random.default_rng(N + 3)
    for rep, mask in enumerate(struct_masks(N)):
        llr, _ = util.synth_frames(mask, 5, ebn0_db=0.5, seed=rep + 40)
        llr = np.concatenate([llr, edge_llr(rng, 3, N)])
        ref = oracle_mod.decode_fsm(mask, llr)
        for sw in solo_sub_words(N):
            _assert_same(run(pkg, cuda, solo(pkg, mask, sub_words=sw), llr), ref, "solo N=%d rep %d S=%d" % (N, rep, sw))


@pytest.mark.gpu
@pytest.mark.parametrize("wpg", [1, 2, 4, 8])
def test_solo_waves_per_frame(pkg, cuda, oracle_mod, wpg):
    """W waves per frame split the upper F / G / R1 / SPC / H ops (the SPC partials of both
    halves meet in LDS)."""
    for name in ("frozen_n_16384_k_8192", None):
        mask = util.mask(name) if name else wave_mask()
        llr, _ = util.synth_frames(mask, 5, ebn0_db=1.0, seed=wpg + 20)
        dec = solo(pkg, mask, waves_per_group=wpg, sub_words=64)
        _assert_same(run(pkg, cuda, dec, llr), oracle_mod.decode_fsm(mask, llr), "solo %s W=%d" % (name, wpg))


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 3])
def test_solo_grid_tier(pkg, cuda, oracle_mod, batch):
    mask = util.mask("frozen_n_32768_k_29492")
    llr, _ = util.synth_frames(mask, batch, ebn0_db=3.0, seed=batch + 7)
    dec = solo(pkg, mask, tier_words=512, sub_words=128)
    assert dec.stats["tier_steps"] > 0
    _assert_same(run(pkg, cuda, dec, llr), oracle_mod.decode_fsm(mask, llr), "solo tier batch %d" % batch)


@pytest.mark.gpu
def test_solo_c5_sample(pkg, cuda, oracle_mod):
    mask = util.mask("frozen_n_262144_k_131072")
    llr, _ = util.synth_frames(mask, 3, ebn0_db=1.0, seed=15)
    ref = oracle_mod.decode_fsm(mask, llr)
    for sw in (256, 512):
        _assert_same(run(pkg, cuda, solo(pkg, mask, sub_words=sw), llr), ref, "C5 solo S=%d" % sw)


@pytest.mark.gpu
def test_solo_misaligned_channel(pkg, cuda, oracle_mod):
    mask = util.mask("frozen_n_16384_k_8192")
    llr, _ = util.synth_frames(mask, 3, ebn0_db=1.0, seed=12)
    flat = cuda.zeros(llr.size + 16, dtype=cuda.int8, device="cuda")
    view = flat[1:1 + llr.size].view(llr.shape)
    view.copy_(cuda.from_numpy(llr))
    out = solo(pkg, mask).decode(view)
    cuda.cuda.synchronize()
    _assert_same(pkg.unpack_bits(out.cpu().numpy(), mask.size), oracle_mod.decode_fsm(mask, llr), "solo misaligned")


# ---- 9-bit LLRs (LLR_BITS 9, parser_comp.sh:12): 16-bit slot rows, the int16 channel ------------
def q9_frames(mask, n_awgn, n_edge, seed):
    rng = np.random.default_rng(seed)
    awgn, _ = util.synth_frames(mask, n_awgn, ebn0_db=1.0, seed=seed)
    awgn = np.clip(awgn.astype(np.int32) * 8, -255, 255)
    edge = rng.integers(-256, 256, size=(n_edge, mask.size))
    edge[:, rng.integers(0, mask.size, 64)] = -256
    edge[:, rng.integers(0, mask.size, 64)] = 0
    return np.concatenate([awgn, edge]).astype(np.int16)


def q9cfg(pkg, ext=1):
    c = pkg.default_config()
    c.llr_bits, c.extended = 9, ext
    return c


def test_solo_q9_plans(pkg):
    """9-bit plans take the solo layout (forced, and as the automatic alternate of small
    batches); CA2 plans do not (the half ops of 8-word nodes have no CA2 form)."""
    m = util.mask("frozen_n_16384_k_8192")
    d = pkg.Decoder(m, config=q9cfg(pkg), tuning={"kernel": 3, "layout": 2})
    assert "#define POLAR_SOLO 1" in d.kernel_source() and "#define POLAR_Q 9" in d.kernel_source()
    a = pkg.Decoder(m, config=q9cfg(pkg))
    i1, i2 = a.launch_info(64, cus=256), a.launch_info(4096, cus=256)
    assert (i1["layout"], i1["alt_layout"], i2["layout"]) == (2, 2, 1), (i1, i2)
    c = pkg.default_config()
    c.sigmag = 0
    with pytest.raises(pkg.PolarError):
        pkg.Decoder(m, config=c, tuning={"kernel": 3, "layout": 2})
    assert pkg.Decoder(m, config=c).launch_info(64, cus=256)["alt_layout"] == 0


@pytest.mark.parametrize("N", [2048, 8192])
def test_solo_q9_emulated(pkg, oracle_mod, N):
    """CPU: the solo code at LLR_BITS 9 (16-bit slot rows) emulated equals the FSM."""
    import pair_emu
    for i, mask in enumerate([util.mask("frozen_n_%d_k_%d" % (N, N // 2))] + list(struct_masks(N))[:2]):
        llr = q9_frames(mask, 1, 2, seed=N + i)
        for ext in (1, 0):
            ref = oracle_mod.decode_fsm(mask, llr, llr_bits=9, extended=ext)
            dec = pkg.Decoder(mask, config=q9cfg(pkg, ext), tuning={"kernel": 3, "layout": 2, "sub_words": 64})
            _assert_same(pair_emu.decode(dec, llr), ref, "emulated solo q9 N=%d mask %d ext %d" % (N, i, ext))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["frozen_n_2048_k_1024", "frozen_n_16384_k_8192", "frozen_n_65536_k_32768", "struct"])
def test_solo_q9_parity(pkg, cuda, oracle_mod, name):
    """LLR_BITS 9 in the solo layout: the automatic plan decodes these small batches solo; the
    whole 9-bit range incl. -256, both EXTENDED switches, int16 and int8 entry points."""
    mask = struct_masks(8192)[1] if name == "struct" else util.mask(name)
    llr = q9_frames(mask, 4, 3, seed=mask.size + 90)
    small = np.clip(llr, -128, 127).astype(np.int8)
    for ext in (1, 0):
        dec = pkg.Decoder(mask, config=q9cfg(pkg, ext))
        assert dec.launch_info(llr.shape[0])["layout"] == 2
        out = dec.decode(cuda.from_numpy(llr).cuda())
        out8 = dec.decode(cuda.from_numpy(small).cuda())
        cuda.cuda.synchronize()
        _assert_same(pkg.unpack_bits(out.cpu().numpy(), mask.size),
                     oracle_mod.decode_fsm(mask, llr, llr_bits=9, extended=ext), "solo q9 %s ext %d" % (name, ext))
        _assert_same(pkg.unpack_bits(out8.cpu().numpy(), mask.size),
                     oracle_mod.decode_fsm(mask, small, llr_bits=9, extended=ext), "solo q9 i8 %s ext %d" % (name, ext))


@pytest.mark.gpu
def test_solo_q9_c5_share(pkg, cuda, oracle_mod):
    """The C5 8-GPU share shape (64 frames of N = 262144) at LLR_BITS 9: solo, sampled against the
    FSM, the rest of the batch equal to the sampled frames' repeats."""
    mask = util.mask("frozen_n_262144_k_131072")
    base = q9_frames(mask, 1, 1, seed=262)
    llr = np.concatenate([base] * 32)
    dec = pkg.Decoder(mask, config=q9cfg(pkg))
    assert dec.launch_info(64)["layout"] == 2
    out = dec.decode(cuda.from_numpy(llr).cuda())
    cuda.cuda.synchronize()
    _assert_same(pkg.unpack_bits(out[:2].cpu().numpy(), mask.size), oracle_mod.decode_fsm(mask, base, llr_bits=9),
                 "C5 share q9")
    assert (out.view(32, 2, -1) == out[:2].unsqueeze(0)).all()
