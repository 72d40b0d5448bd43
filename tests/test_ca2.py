"""CA2 (two's complement datapath, config.h:11; functions.h:48-118) on the generated pair kernel
(polar_sc_pair.h / polar_sc_device.h POLAR_CA2; polar_sc_pairgen.cpp PairGen::ca2): the split
code on magnitude + sign with a zero's sign don't-care, hard decisions masking zeros, REP without
the exact-SM fallback, and MIN (-2^(w-1), absorbing under F_function_C2's qabs wrap) on the
leftmost path and in the first PAR word (the _L variant of the first subtree decoder).

CPU: the generated CA2 code emulated (tests/pair_emu.py) equals the oracle, and a mutation that
makes MIN non-absorbing is caught. GPU: bit-exact with the literal FSM at CA2 on reference,
structured and first-word-information masks, AWGN and edge LLRs (MIN in every frame), LLR_BITS
5 .. 9 (8-bit LLRs: 16-bit slot rows; 9-bit: the int16 channel), PAR 16 / 32 / 64, EXTENDED 0 / 1,
PRUNING_LEVEL 0 / 2, waves per pair 1 .. 8, subtree sizes 32 .. 256."""
import numpy as np
import pytest

import util
from test_gpu_parity import _assert_same
from sc_polar_decoder_hls_amd._plansets import ca2_first_mask, ca2_gpu_items, struct_masks


def cfg(pkg, **kw):
    c = pkg.default_config()
    c.sigmag = 0
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def edge_llr(rng, n, N, q=6):
    amp = (1 << (q - 1)) - 1
    e = rng.integers(-(amp + 1), amp + 1, size=(n, N))
    e[:, rng.integers(0, N, N // 8)] = -(amp + 1)                              # MIN
    e[:, rng.integers(0, N, N // 8)] = 0
    e[0, :64] = -(amp + 1)                                                     # MIN on the leftmost path
    return e


def frames(mask, q, n_awgn, n_edge, seed):
    rng = np.random.default_rng(seed)
    amp = (1 << (q - 1)) - 1
    awgn, _ = util.synth_frames(mask, n_awgn, ebn0_db=1.0, seed=seed)
    awgn = np.clip(awgn.astype(np.int32) * (1 << q) // 64, -amp, amp)
    llr = np.concatenate([awgn, edge_llr(rng, n_edge, mask.size, q)])
    return llr.astype(np.int16 if q > 8 else np.int8)


def test_ca2_plans_take_the_pair_kernel(pkg):
    m = util.mask("frozen_n_16384_k_8192")
    for par in (16, 32, 64):
        for q in (5, 6, 7, 8, 9):
            for ext in (0, 1):
                for pl in (0, 2):
                    d = pkg.Decoder(m, config=cfg(pkg, par=par, llr_bits=q, extended=ext, pruning_level=pl))
                    assert d.stats["kernel"] == 3, (par, q, ext, pl, d.stats["kernel"])
    # PRUNING_LEVEL 1: the leaf decoders (REP / SPC / REP2 / SPC2 / R1) on the pair kernel, at
    # PAR 32 / 64 those of the whole PAR word (OP_PLEAF, pleaf_pair)
    d1 = pkg.Decoder(m, config=cfg(pkg, pruning_level=1, elag_r1=1, elag_rep=1, elag_spc=1, elag_rep2=1, elag_spc2=1))
    assert d1.stats["kernel"] == 3
    kinds = {(o["fb"] >> 16) & 7 for o in d1.schedule() if o["op"] in ("FLEAF", "GLEAF")}
    assert kinds == {0, 1, 2, 3, 4, 5}, kinds   # every decoder, the CA2 R1 leaf (5) included
    for par in (32, 64):
        dp = pkg.Decoder(m, config=cfg(pkg, par=par, pruning_level=1, elag_r1=1, elag_rep=1, elag_spc=1, elag_rep2=1,
                                       elag_spc2=1))
        assert dp.stats["kernel"] == 3 and "pleaf_pair<5>" in dp.kernel_source(), par
    # (N = 1024: the pair kernel too since round 6; below it the interpreter)
    assert pkg.Decoder(util.mask("FB_N1024_K512"), config=cfg(pkg)).stats["kernel"] == 3
    assert pkg.Decoder(util.mask("FB_N512_K256"), config=cfg(pkg)).stats["kernel"] != 3
    src = pkg.Decoder(m, config=cfg(pkg)).kernel_source()
    assert "#define POLAR_CA2 1" in src and "polar_psub_0_L(" in src and "leaf_gen_ca2<" in src
    assert "POLAR_CA2" not in pkg.Decoder(m).kernel_source()
    # 8-bit CA2 LLRs: 16-bit slot rows (|MIN| = 128 does not fit an SM8 byte)
    s8 = pkg.Decoder(m, config=cfg(pkg, llr_bits=8)).stats
    s7 = pkg.Decoder(m, config=cfg(pkg, llr_bits=7)).stats
    assert s8["scratch_bytes_per_wave"] > s7["scratch_bytes_per_wave"]


@pytest.mark.parametrize("N", [1024, 2048, 8192])
def test_ca2_generated_code_emulated(pkg, oracle_mod, N):
    """CPU: the CA2 subtree decoders and upper levels emulated on 64-lane waves equal the FSM
    (structured masks, the first word informative so that leaf 0 meets MIN, edge LLRs)."""
    import pair_emu
    masks = [util.mask("frozen_n_%d_k_%d" % (N, N // 2)), ca2_first_mask(N)] + list(struct_masks(N))
    for i, mask in enumerate(masks):
        llr = frames(mask, 6, 1, 2, seed=N + i)
        for ext in (1, 0):
            ref = oracle_mod.decode_fsm(mask, llr, sigmag=0, extended=ext)
            dec = pkg.Decoder(mask, config=cfg(pkg, extended=ext), tuning={"kernel": 3, "sub_words": 32})
            _assert_same(pair_emu.decode(dec, llr), ref, "emulated CA2 N=%d mask %d ext %d" % (N, i, ext))


def test_ca2_min_absorbing_is_needed(pkg, oracle_mod, monkeypatch):
    """A mutation of the emulation (F_function_C2 without the qabs wrap: MIN not absorbing)
    differs from the FSM on MIN inputs -- the MIN path is exercised, not vacuous."""
    import pair_emu
    monkeypatch.setattr(pair_emu, "pk_min_key", lambda MW, a, b: pair_emu.pk_min(a, b))
    mask = ca2_first_mask(2048)
    llr = frames(mask, 6, 0, 3, seed=5)
    dec = pkg.Decoder(mask, config=cfg(pkg), tuning={"kernel": 3, "sub_words": 32})
    assert (pair_emu.decode(dec, llr) != oracle_mod.decode_fsm(mask, llr, sigmag=0)).any()


@pytest.mark.gpu
@pytest.mark.parametrize("item", ca2_gpu_items(), ids=lambda it: it[0])
def test_ca2_pair_kernel_gpu(pkg, cuda, oracle_mod, item):
    name, mask, fields, tun = item
    c = cfg(pkg, **fields)
    dec = pkg.Decoder(mask, config=c, tuning=tun)
    assert dec.stats["kernel"] == 3, (name, dec.stats["kernel"])
    q = fields.get("llr_bits", 6)
    llr = frames(mask, q, 5, 4, seed=mask.size + q)
    out = dec.decode(cuda.from_numpy(llr).cuda())
    cuda.cuda.synchronize()
    c7 = (c.pruning_level, c.elag_r1, c.elag_rep, c.elag_spc, c.elag_rep2, c.elag_spc2, c.elag_h0)
    ref = oracle_mod.decode_fsm(mask, llr, config=c7, llr_bits=q, par=c.par, sigmag=0, extended=c.extended)
    _assert_same(pkg.unpack_bits(out.cpu().numpy(), mask.size), ref, "CA2 " + name)


@pytest.mark.gpu
def test_ca2_pair_kernel_full_batch(pkg, cuda, oracle_mod):
    """The format_speed shape (N = 16384, 4096 frames, 1 wave per pair): sampled against the FSM,
    and noiseless codewords decode exactly over the whole batch."""
    mask = util.mask("frozen_n_16384_k_8192")
    for par in (16, 64):
        dec = pkg.Decoder(mask, config=cfg(pkg, par=par))
        llr = np.concatenate([frames(mask, 6, 2, 2, seed=par)] * 1024)
        out = dec.decode(cuda.from_numpy(llr).cuda())
        cuda.cuda.synchronize()
        got = pkg.unpack_bits(out[:4].cpu().numpy(), mask.size)
        _assert_same(got, oracle_mod.decode_fsm(mask, llr[:4], par=par, sigmag=0), "CA2 full PAR %d" % par)
        assert (out.view(1024, 4, -1) == out[:4].unsqueeze(0)).all()
        rng = np.random.default_rng(par)
        u = rng.integers(0, 2, size=(4096, mask.size), dtype=np.uint8) & mask[None, :]
        x = util.encode_np(u)
        out = dec.decode(cuda.from_numpy(np.where(x == 1, -17, 17).astype(np.int8)).cuda())
        cuda.cuda.synchronize()
        assert (pkg.unpack_bits(out.cpu().numpy(), mask.size) == x).all(), par


def test_ca2_leaf_vs_oracle(pkg, oracle_mod):
    """CPU: the CA2 leaf of the generated code (leaf_ca2, incl. the all-information blocks on
    sign / zero masks, ca2_allinfo) emulated on 64 lanes equals the oracle's Spec_P16_ext in CA2
    (oracle/polar_oracle.c spec_pn) on words with dense zeros, for every pattern class."""
    import pair_emu
    pair_emu.configure(6, ca2=True, ext=True)
    try:
        ln = pair_emu.Lanes()
        rng = np.random.default_rng(16)
        pats = [0xFFFF, 0xFFFE, 0xFF00, 0xF0F0, 0xFEE8, 0xE800, 0x8000, 0xFFF0, 0xCCCC, 0xFF0F] + \
            [int(x) for x in rng.integers(0, 1 << 16, 20)]
        pos = pair_emu.lane_pos(pair_emu.LANE & 15)
        row = pair_emu.LANE >> 4
        for fb in pats:
            for trial in range(6):
                p0 = (0.1, 0.3, 0.6)[trial % 3]
                v = rng.integers(-31, 32, size=(2, 4, 16))
                v[rng.random(v.shape) < p0] = 0
                val = v[:, row, pos]                       # [frame, lane]
                M = pair_emu.pk(np.abs(val[0]), np.abs(val[1]))
                # (odd trials: zeros carry a set sign bit, which the split code must ignore)
                neg = (val < 0) | ((val == 0) & (trial % 2 == 1) & (rng.random(val.shape) < 0.5))
                S = pair_emu.pk(np.where(neg[0], 0xFFFF, 0), np.where(neg[1], 0xFFFF, 0))
                x = pair_emu.V(pair_emu.leaf_gen_ca2(fb, 0, M, S, ln)).astype(np.int64)
                with oracle_mod._format(6, 16, 0, 1):
                    for f in range(2):
                        for r in range(4):
                            want = oracle_mod.leaf16(v[f, r] & 63, fb)
                            got = 0
                            for L in range(16 * r, 16 * r + 16):
                                got |= ((x[L] >> (15 + 16 * f)) & 1) << int(pos[L])
                            assert got == want, (hex(fb), trial, f, r, v[f, r].tolist(), hex(got), hex(want))
    finally:
        pair_emu.configure()
