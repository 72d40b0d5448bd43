"""Hybrid plans (N > 1024): the schedule interpreter for the upper tree levels plus generated
straight-line decoders for every mixed subtree of polar_sc_tuning.sub_words words
(polar_sc_interp.h OP_SUB, polar_sc_jit.cpp hybrid_source).

CPU tests: plan statistics and hipRTC compilation of the generated source (no GPU needed).
GPU tests: bit-exact against the oracle for every subtree size, including subtrees whose root
children are REP / R1 / SPC nodes (the root-split path of the generator), and against the
plain interpreter on a full C3 batch."""
import numpy as np
import pytest

import util


def make(pkg, mask, jit="1", sub_words=None, tier_words=None):
    """Plan with explicit kernel selection (polar_sc_tuning): jit "0" = the schedule
    interpreter; sub_words / tier_words as given (tier_words 0 = no grid tier)."""
    t = {"kernel": 2 if jit == "1" else 1}   # the hybrid kernel explicitly (the default for N >= 2048 is the pair kernel)
    if sub_words is not None:
        t["sub_words"] = sub_words
    if tier_words is not None:
        t["tier_words"] = tier_words if tier_words else -1
    return pkg.Decoder(mask, tuning=t)


def structured_mask(rng, N):
    """16-bit groups drawn from the pruned node patterns (R0, R1, REP, SPC) and random ones,
    so subtree roots get REP / R1 / SPC children."""
    pats = [0, 0xFFFF, 0x8000, 0xFFFE, int(rng.integers(0, 65536))]
    groups = rng.choice(pats, N // 16)
    return np.concatenate([[(int(p) >> k) & 1 for k in range(16)] for p in groups]).astype(np.uint8)


def test_hybrid_plan_stats(pkg):
    s = make(pkg, util.mask("frozen_n_65536_k_32768")).stats
    # N >= 32768: 128-word (2048-LLR) subtrees
    assert (s["kernel"], s["sub_words"], s["n_sub_kinds"], s["n_sub_calls"]) == (2, 128, 27, 27)
    s = make(pkg, util.mask("frozen_n_65536_k_32768"), sub_words=64).stats
    assert (s["kernel"], s["sub_words"], s["n_sub_kinds"], s["n_sub_calls"]) == (2, 64, 43, 47)
    assert s["storage"] == 1
    s = make(pkg, util.mask("FB_N1024_K512")).stats
    assert s["kernel"] == 1 and s["sub_words"] == 0
    s = make(pkg, util.mask("frozen_n_65536_k_32768"), jit="0").stats
    assert s["kernel"] == 0 and s["n_sub_calls"] == 0
    s = make(pkg, util.mask("frozen_n_8192_k_4096"), sub_words=8).stats
    assert s["kernel"] == 2 and s["sub_words"] == 8 and s["n_sub_calls"] >= s["n_sub_kinds"] > 0


def test_grid_tier_plan(pkg):
    """Grid tier: C3 / C5 plans cut their schedule at the F / G records of >= 1024 words (2 / 4
    upper levels); polar_sc_tuning.tier_words moves the cut (-1 = single kernel); plans too small for
    an HBM level above the LDS region have none."""
    s = make(pkg, util.mask("frozen_n_65536_k_32768")).stats
    assert (s["tier_words"], s["tier_steps"]) == (1024, 10)
    s = make(pkg, util.mask("frozen_n_262144_k_131072")).stats
    assert s["tier_words"] == 1024 and s["tier_steps"] > 30
    assert make(pkg, util.mask("frozen_n_65536_k_32768"), tier_words=0).stats["tier_steps"] == 0
    assert make(pkg, util.mask("frozen_n_65536_k_32768"), tier_words=2048).stats["tier_steps"] == 4
    # (batches with a frame group per CU take the root-only cut at launch: polar_sc_jit.cpp
    # launch_tier; test_hybrid_equals_interpreter_full_c3 runs it at 512 groups)
    assert make(pkg, util.mask("frozen_n_32768_k_29492")).stats["tier_steps"] == 0
    assert make(pkg, util.mask("frozen_n_32768_k_29492"), tier_words=512).stats["tier_steps"] > 0
    assert make(pkg, util.mask("frozen_n_65536_k_32768"), jit="0").stats["tier_steps"] == 0


def test_plan_n524288(pkg):
    """The largest reference mask (N = 2^19): HBM-scratch storage with the 1024-slot LDS
    region, grid tier at 1024 words, and scratch sized for the upper levels of one group."""
    s = make(pkg, util.mask("frozen_n_524288_k_262144")).stats
    assert (s["N"], s["K"], s["groups"]) == (524288, 262144, 32768)
    assert (s["n_r0"], s["n_r1"], s["n_rep"], s["n_spc"], s["n_rn"]) == (14575, 13875, 662, 1341, 2315)
    assert s["storage"] == 1 and s["kernel"] == 2 and s["tier_words"] == 1024 and s["tier_steps"] > 40
    # LDS: 1023 slots of 8-bit pairs + the 64-dword partial-sum window + the SPC exchange area
    assert s["lds_bytes_per_wave"] == (1023 * 64 * 2) + (64 + 24) * 256
    # HBM: slots [0, G - 1024) as 128-byte rows + 2048 bit dwords of 256 bytes
    assert s["scratch_bytes_per_wave"] == (32768 - 1024) * 128 + 2048 * 256


def test_hybrid_schedule_export_unchanged(pkg):
    """The exported schedule stays the plain op list (no device-internal records)."""
    mask = util.mask("frozen_n_8192_k_4096")
    a = make(pkg, mask).schedule()
    b = make(pkg, mask, jit="0").schedule()
    assert a == b and all(o["op"] in ("F", "G", "FLEAF", "GLEAF", "REP", "R1", "SPC", "H", "H0", "END") for o in a)


@pytest.mark.parametrize("sub_words", [2, 8, 64])
def test_hybrid_source_compiles(pkg, sub_words):
    rng = np.random.default_rng(sub_words)
    dec = make(pkg, structured_mask(rng, 4096), sub_words=sub_words)
    src = dec.kernel_source()
    assert "polar_sc_hybrid_kernel" in src and "polar_sub_0(" in src
    dec.compile()   # hipRTC for gfx950 on the host


@pytest.mark.parametrize("q", [5, 8])
def test_llr_bits_kernels_compile(pkg, q):
    """LLR_BITS 5..8 plans are specialised through POLAR_Q in the hipRTC kernels: the per-mask
    kernel (N <= 1024) and the pair kernel (N >= 2048), PRUNING_LEVEL 1 leaf decoders included,
    the pair kernel for the other formats from N = 1024 (PAR 64 PRUNING_LEVEL 1: PAR-word leaf
    decoders, round 6), and below that the interpreter compiled by hipRTC."""
    for name, pr, par, kernel in (("FB_N1024_K512", 2, 16, 1), ("frozen_n_4096_k_2048", 2, 16, 3),
                                  ("FB_N1024_K512", 1, 16, 1), ("frozen_n_4096_k_2048", 1, 16, 3),
                                  ("FB_N1024_K512", 1, 64, 3), ("FB_N512_K256", 1, 64, 2)):
        c = pkg.default_config()
        c.llr_bits, c.pruning_level, c.par = q, pr, par
        dec = pkg.Decoder(util.mask(name), config=c)
        assert dec.stats["kernel"] == kernel, (name, pr)
        assert "#define POLAR_Q %d" % q in dec.kernel_source()
        dec.compile()


def test_clang_flags_knob(pkg, monkeypatch):
    """POLAR_SC_CLANG_FLAGS (compiler A/Bs) reaches the clang driver and keys the code-object
    cache: a valid flag builds a code object of its own, an invalid one fails the compile
    instead of falling back to hipRTC (which would ignore it)."""
    mask = util.mask("FB_N128_K64")
    base = pkg.Decoder(mask).launch_info(1)["code_key"]
    monkeypatch.setenv("POLAR_SC_CLANG_FLAGS", "-mllvm --amdgpu-schedule-metric-bias=0")
    dec = pkg.Decoder(mask)
    assert dec.compile() and dec.launch_info(1)["code_key"] == base   # same code, own cache entry
    monkeypatch.setenv("POLAR_SC_CLANG_FLAGS", "-fno-such-clang-flag")
    with pytest.raises(pkg.PolarError):
        pkg.Decoder(mask).compile()



@pytest.mark.gpu
@pytest.mark.parametrize("sub_words", [2, 4, 8, 16, 32, 64])
def test_hybrid_parity_sub_sizes(pkg, cuda, oracle_mod, sub_words):
    rng = np.random.default_rng(100 + sub_words)
    cases = [structured_mask(rng, 2048), structured_mask(rng, 4096), util.mask("frozen_n_4096_k_2048"),
             (rng.random(2048) < np.linspace(0, 1, 2048) ** 0.5).astype(np.uint8)]
    for ci, mask in enumerate(cases):
        dec = make(pkg, mask, sub_words=sub_words)
        assert dec.stats["kernel"] == 2
        llr = rng.integers(-32, 32, size=(11, mask.size)).astype(np.int8)
        out = dec.decode(cuda.from_numpy(llr).cuda())
        cuda.cuda.synchronize()
        got = pkg.unpack_bits(out.cpu().numpy(), mask.size)
        ref = oracle_mod.decode_fsm(mask, llr)
        bad = np.nonzero((got != ref).any(axis=1))[0]
        assert bad.size == 0, "sub_words %d case %d: frames %s differ" % (sub_words, ci, bad[:8])


@pytest.mark.gpu
def test_hybrid_hbm_scratch_sub_sizes(pkg, cuda, oracle_mod):
    """HBM-scratch plans (N = 8192): subtrees inside and across the LDS partial-sum window."""
    mask = util.mask("frozen_n_8192_k_4096")
    llr, _ = util.synth_frames(mask, 9, ebn0_db=1.0, seed=8192)
    ref = oracle_mod.decode_fsm(mask, llr)
    for sw in (4, 32, 64):
        dec = make(pkg, mask, sub_words=sw)
        assert dec.stats["storage"] == 1 and dec.stats["kernel"] == 2
        out = dec.decode(cuda.from_numpy(llr).cuda())
        cuda.cuda.synchronize()
        np.testing.assert_array_equal(pkg.unpack_bits(out.cpu().numpy(), mask.size), ref, err_msg="sub %d" % sw)


@pytest.mark.gpu
def test_hybrid_equals_interpreter_full_c3(pkg, cuda):
    """Full BASELINE C3 batch (4096 frames of N = 65536): hybrid == plain interpreter."""
    import bench
    mask = util.mask("frozen_n_65536_k_32768")
    llr, _ = bench.gen_frames_torch(cuda, mask, 4096, 2.0, 3, cuda.device("cuda"))
    outs = [make(pkg, mask, jit=j).decode(llr) for j in ("1", "0")]
    cuda.cuda.synchronize()
    assert cuda.equal(outs[0], outs[1])


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [13, 64])
def test_grid_tier_parity_forced(pkg, cuda, oracle_mod, batch):
    """A grid tier forced onto N = 32768 (F / G of >= 512 words grid-wide, the rest in
    segments): bit-exact against the oracle, ragged batch included, and equal to the single
    kernel decode of the same plan shape."""
    mask = util.mask("frozen_n_32768_k_29492")
    awgn, _ = util.synth_frames(mask, batch, ebn0_db=3.0, seed=batch)
    llr = np.clip(awgn.astype(np.int32), -31, 31).astype(np.int8)
    dec = make(pkg, mask, tier_words=512)
    assert dec.stats["tier_steps"] > 0
    t = cuda.from_numpy(llr).cuda()
    out = dec.decode(t)
    one = make(pkg, mask, tier_words=0).decode(t)
    cuda.cuda.synchronize()
    assert cuda.equal(out, one)
    np.testing.assert_array_equal(pkg.unpack_bits(out.cpu().numpy(), mask.size), oracle_mod.decode_fsm(mask, llr))


@pytest.mark.gpu
def test_grid_tier_equals_single_kernel_c5(pkg, cuda):
    """C5 (N = 262144) at its 8-GPU share of 64 frames: the grid-tier decode equals the single
    hybrid kernel bit for bit (both are checked against the oracle on sampled frames by
    test_gpu_parity.py::test_parity_c5_mask_sample)."""
    import bench
    mask = util.mask("frozen_n_262144_k_131072")
    llr, _ = bench.gen_frames_torch(cuda, mask, 64, 2.0, 5, cuda.device("cuda"))
    a = make(pkg, mask)
    assert a.stats["tier_steps"] > 0
    outs = [a.decode(llr), make(pkg, mask, tier_words=0).decode(llr)]
    cuda.cuda.synchronize()
    assert cuda.equal(outs[0], outs[1])
