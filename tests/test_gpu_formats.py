"""GPU parity across the reference's swept datapath formats: PAR 4 / 8 / 16 / 32 / 64
(polar_parameters.h:8; script_tests.sh:11,124 sweeps 16 and 64), CA2 vs SIGMAG (config.h:11;
script/parser.sh:15,43), EXTENDED 0/1 (config.h:14) and LLR_BITS up to 9 (parser_comp.sh:12;
int16 channel). Formats without a generated kernel run the schedule interpreter compiled by
hipRTC with their POLAR_* switches; every format must equal the literal FSM at the same format bit for bit, on AWGN
frames, on the whole input range (incl. the -2^(Q-1) wrap of CA2) and under PRUNING_LEVEL 0 /
1 / 2 configurations. Masks cover the LDS (N <= 4096) and HBM-scratch (N = 16384) storage."""
import numpy as np
import pytest

import util
# FORMATS: (par, sigmag, extended, llr_bits); build() prewarms every plan decoded here
from sc_polar_decoder_hls_amd._plansets import FORMATS, FORMAT_C7 as CONFIGS, format_seed, planted_mask, \
    PRUNING_SWEEP, high_rate_items
from test_gpu_parity import _assert_same

pytestmark = pytest.mark.gpu


def _decoder(pkg, mask, fmt, c7):
    par, sigmag, ext, q = fmt
    c = pkg.default_config()
    (c.pruning_level, c.elag_r1, c.elag_rep, c.elag_spc, c.elag_rep2, c.elag_spc2, c.elag_h0) = c7
    c.par, c.sigmag, c.extended, c.llr_bits = par, sigmag, ext, q
    return pkg.Decoder(mask, config=c)


@pytest.mark.parametrize("fmt", FORMATS, ids=lambda f: "p%d_%s_e%d_q%d" % (f[0], "sm" if f[1] else "ca2", f[2], f[3]))
def test_formats_vs_oracle(pkg, cuda, oracle_mod, fmt):
    par, sigmag, ext, q = fmt
    rng = np.random.default_rng(format_seed(fmt))
    amp = (1 << (q - 1)) - 1
    masks = [("FB_N1024_K512", util.mask("FB_N1024_K512")), ("planted_4096", planted_mask(rng, 4096, par)),
             ("frozen_n_16384_k_8192", util.mask("frozen_n_16384_k_8192"))]
    for name, mask in masks:
        B = 24 if mask.size <= 4096 else 9
        awgn, _ = util.synth_frames(mask, B // 2, ebn0_db=1.0, seed=q)
        awgn = np.clip(awgn.astype(np.int32) * (1 << q) // 64, -amp, amp)
        edge = rng.integers(-(amp + 1), amp + 1, size=(B - B // 2, mask.size))
        edge[:, rng.integers(0, mask.size, 64)] = -(amp + 1)          # the -2^(Q-1) corner
        llr = np.concatenate([awgn, edge]).astype(np.int16 if q > 8 else np.int8)
        for c7 in CONFIGS:
            dec = _decoder(pkg, mask, fmt, c7)
            out = dec.decode(cuda.from_numpy(llr).cuda())
            cuda.cuda.synchronize()
            got = pkg.unpack_bits(out.cpu().numpy(), mask.size)
            ref = oracle_mod.decode_fsm(mask, llr, config=c7, llr_bits=q, par=par, sigmag=sigmag, extended=ext)
            _assert_same(got, ref, "%s fmt %s cfg %s storage %d" % (name, fmt, c7, dec.stats["storage"]))
            if par == 16 and sigmag == 1 and q <= 8:   # EXTENDED 0: the generated kernels
                assert dec.stats["kernel"] in (1, 3), (name, fmt, c7, dec.stats["kernel"])
            if par in (32, 64) and sigmag == 1 and mask.size >= 1024:
                assert dec.stats["kernel"] == 3, (name, fmt, c7, dec.stats["kernel"])   # the pair kernel
            if par == 16 and sigmag == 1 and q == 9 and mask.size >= 1024:   # 16-bit slots
                assert dec.stats["kernel"] == 3, (name, fmt, c7, dec.stats["kernel"])
            if par in (4, 8) and mask.size >= 1024:   # PAR words as lane groups (SIGMAG, CA2)
                assert dec.stats["kernel"] == 3, (name, fmt, c7, dec.stats["kernel"])
            if sigmag == 0 and par >= 16 and mask.size >= 1024:
                assert dec.stats["kernel"] == 3, (name, fmt, c7, dec.stats["kernel"])   # CA2 on the pair kernel


@pytest.mark.parametrize("q", [6, 9])
def test_int16_channel_matches_int8(pkg, cuda, oracle_mod, q):
    """polar_sc_decode_i16: int16 frames decode like the same values as int8 (where they fit),
    for the shipped format too (whose int8 path is the per-mask kernel)."""
    mask = util.mask("FB_N1024_K512")
    llr, _ = util.synth_frames(mask, 32, ebn0_db=2.0, seed=16)
    c = pkg.default_config()
    c.llr_bits = q
    dec = pkg.Decoder(mask, config=c)
    a = dec.decode(cuda.from_numpy(llr).cuda())
    b = dec.decode(cuda.from_numpy(llr.astype(np.int16)).cuda())
    cuda.cuda.synchronize()
    assert (a.cpu().numpy() == b.cpu().numpy()).all()
    _assert_same(pkg.unpack_bits(b.cpu().numpy(), mask.size), oracle_mod.decode_fsm(mask, llr, llr_bits=q), "i16")


@pytest.mark.parametrize("name", ["frozen_n_2048_k_1024", "frozen_n_16384_k_8192", "frozen_n_65536_k_32768"])
def test_int16_channel_hybrid_plans(pkg, cuda, oracle_mod, name):
    """polar_sc_decode_i16 on plans whose int8 path runs generated subtree decoders (the pair
    kernel): the int16 interpreter runs the plan's schedule without subtree records and must
    give the int8 path's bits (it skipped the subtrees)."""
    mask = util.mask(name)
    llr, _ = util.synth_frames(mask, 11, ebn0_db=1.5, seed=1616)
    dec = pkg.Decoder(mask)
    assert dec.stats["kernel"] in (2, 3) and dec.stats["n_sub_calls"] > 0
    a = dec.decode(cuda.from_numpy(llr).cuda())
    b = dec.decode(cuda.from_numpy(llr.astype(np.int16)).cuda())
    cuda.cuda.synchronize()
    assert (a.cpu().numpy() == b.cpu().numpy()).all()
    _assert_same(pkg.unpack_bits(b.cpu().numpy(), mask.size), oracle_mod.decode_fsm(mask, llr), "i16 " + name)


@pytest.mark.parametrize("name", ["frozen_n_2048_k_1024", "frozen_n_16384_k_8192", "frozen_n_65536_k_32768", "struct"])
def test_llr9_pair_kernel(pkg, cuda, oracle_mod, name):
    """LLR_BITS 9 on the pair kernel (polar_sc_pair.h SLOT16: SM16 stage slots, the int16
    channel): the whole 9-bit input range incl. -256 and +-255, both EXTENDED switches, the
    int16 entry point and the int8 one (widened on the device), equal to the FSM at LLR_BITS 9."""
    from sc_polar_decoder_hls_amd._plansets import struct_masks
    mask = struct_masks(8192)[1] if name == "struct" else util.mask(name)
    rng = np.random.default_rng(mask.size + 9)
    awgn, _ = util.synth_frames(mask, 6, ebn0_db=1.0, seed=9)
    awgn = np.clip(awgn.astype(np.int32) * 8, -255, 255)
    edge = rng.integers(-256, 256, size=(3, mask.size))
    edge[0, rng.integers(0, mask.size, 64)] = -256
    llr = np.concatenate([awgn, edge]).astype(np.int16)
    small = np.clip(llr, -128, 127).astype(np.int8)
    for ext in (1, 0):
        c = pkg.default_config()
        c.llr_bits, c.extended = 9, ext
        dec = pkg.Decoder(mask, config=c)
        assert dec.stats["kernel"] == 3, dec.stats["kernel"]
        out = dec.decode(cuda.from_numpy(llr).cuda())
        out8 = dec.decode(cuda.from_numpy(small).cuda())
        cuda.cuda.synchronize()
        _assert_same(pkg.unpack_bits(out.cpu().numpy(), mask.size),
                     oracle_mod.decode_fsm(mask, llr, llr_bits=9, extended=ext), "%s i16 ext %d" % (name, ext))
        _assert_same(pkg.unpack_bits(out8.cpu().numpy(), mask.size),
                     oracle_mod.decode_fsm(mask, small, llr_bits=9, extended=ext), "%s i8 ext %d" % (name, ext))


def test_formats_noiseless_full_size(pkg, cuda):
    """PAR 64 and CA2 at a full C2 batch (65536 frames): noiseless codewords decode exactly
    (size-independent property)."""
    mask = util.mask("FB_N1024_K512")
    rng = np.random.default_rng(64)
    u = rng.integers(0, 2, size=(65536, mask.size), dtype=np.uint8) & mask[None, :]
    x = util.encode_np(u)
    llr = np.where(x == 1, -17, 17).astype(np.int8)
    t = cuda.from_numpy(llr).cuda()
    for fmt in ((64, 1, 1, 6), (16, 0, 1, 6), (64, 0, 0, 8)):
        dec = _decoder(pkg, mask, fmt, (2, 1, 1, 1, 0, 0, 1))
        out = dec.decode(t)
        cuda.cuda.synchronize()
        assert (pkg.unpack_bits(out.cpu().numpy(), mask.size) == x).all(), fmt


def _sweep_cfg(pkg, c7, par):
    c = pkg.default_config()
    (c.pruning_level, c.elag_r1, c.elag_rep, c.elag_spc, c.elag_rep2, c.elag_spc2, c.elag_h0) = c7
    c.par, c.llr_bits = par, 8
    return c


@pytest.mark.parametrize("par", [16, 64, 8, 4])
def test_script_tests_pruning_sweep(pkg, cuda, oracle_mod, par):
    """script/script_tests.sh:103-213 as the reference runs it: the 11 pruning configurations
    on frozen_n_32768_k_29492 (its lines 105-106) at QUANT 8, for PAR 16 and 64 (line 124),
    and the same sweep at PAR 8 and 4 (the PAR values of script_RTL_sim.sh).
    PAR 16 plans run on the schedule interpreter here (tuning kernel = 1, one code object for
    the format); the generated-subtree kernels are swept in test_gpu_configs.py."""
    mask = util.mask("frozen_n_32768_k_29492")
    awgn, _ = util.synth_frames(mask, 8, ebn0_db=3.5, seed=par)
    llr = np.clip(awgn.astype(np.int32) * 4, -127, 127).astype(np.int8)
    t = cuda.from_numpy(llr).cuda()
    for c7 in oracle_mod.SWEEP_CONFIGS:
        dec = pkg.Decoder(mask, config=_sweep_cfg(pkg, c7, par), tuning={"kernel": 1})
        out = dec.decode(t)
        cuda.cuda.synchronize()
        got = pkg.unpack_bits(out.cpu().numpy(), mask.size)
        _assert_same(got, oracle_mod.decode_fsm(mask, llr, config=c7, llr_bits=8, par=par), "PAR %d %s" % (par, c7))


@pytest.mark.parametrize("par", [16, 64, 32, 8, 4])
def test_script_tests_pruning_sweep_pair_kernel(pkg, cuda, oracle_mod, par):
    """The same loop on the kernel the plans select by default: the generated pair kernel for
    every configuration, PRUNING_LEVEL 1's REP / SPC / REP2 / SPC2 leaves included (PAR 64 / 32:
    the decoders of the whole PAR word, polar_sc_pair.h pleaf_pair; PAR 8 / 4: the word trees
    of the leaf records with their group classes as template constants, polar_sc_device.h
    word_gen)."""
    mask = util.mask("frozen_n_32768_k_29492")
    awgn, _ = util.synth_frames(mask, 8, ebn0_db=3.5, seed=16)
    llr = np.clip(awgn.astype(np.int32) * 4, -127, 127).astype(np.int8)
    t = cuda.from_numpy(llr).cuda()
    for c7 in PRUNING_SWEEP:
        dec = pkg.Decoder(mask, config=_sweep_cfg(pkg, c7, par))
        assert dec.stats["kernel"] == 3, c7
        out = dec.decode(t)
        cuda.cuda.synchronize()
        got = pkg.unpack_bits(out.cpu().numpy(), mask.size)
        _assert_same(got, oracle_mod.decode_fsm(mask, llr, config=c7, llr_bits=8, par=par), "pair PAR %d %s" % (par, c7))


@pytest.mark.parametrize("par", [16, 64])
@pytest.mark.parametrize("name", ["frozen_n_2048_k_1844", "frozen_n_4096_k_3686", "frozen_n_8192_k_7372",
                                  "frozen_n_16384_k_14746"])
def test_script_tests_rate09_codes(pkg, cuda, oracle_mod, par, name):
    """script/script_tests.sh:7-58: the rate-0.9 codes N = 2048 .. 16384 at QUANT 8, PAR 16 and
    64, shipped pruning configuration (PAR 16: the per-mask / hybrid kernels)."""
    mask = util.mask(name)
    awgn, _ = util.synth_frames(mask, 16, ebn0_db=4.0, seed=par)
    llr = np.clip(awgn.astype(np.int32) * 4, -127, 127).astype(np.int8)
    dec = pkg.Decoder(mask, config=_sweep_cfg(pkg, oracle_mod.DEFAULT_CONFIG, par))
    out = dec.decode(cuda.from_numpy(llr).cuda())
    cuda.cuda.synchronize()
    got = pkg.unpack_bits(out.cpu().numpy(), mask.size)
    _assert_same(got, oracle_mod.decode_fsm(mask, llr, llr_bits=8, par=par), "%s PAR %d" % (name, par))


@pytest.mark.parametrize("item", high_rate_items(), ids=lambda it: it[0])
def test_high_rate_codes_formats(pkg, cuda, oracle_mod, item):
    """The rate-0.9 codes of script_tests.sh:7-9 and the N = 1024 K = 922 code of
    script_RTL_sim.sh:87-97 (its PAR 4..64 loop) across PAR, SIGMAG / CA2 and LLR_BITS 6 / 8:
    high-rate codes make the R1 / SPC nodes and the all-information leaves dominate. Every
    format runs a generated kernel (N = 1024 non-shipped formats: the pair kernel, round 6)."""
    name, mask, fields, _ = item
    c = pkg.default_config()
    for k, v in fields.items():
        setattr(c, k, v)
    dec = pkg.Decoder(mask, config=c)
    assert dec.stats["kernel"] in (1, 3), (name, dec.stats["kernel"])
    q = fields["llr_bits"]
    amp = (1 << (q - 1)) - 1
    rng = np.random.default_rng(mask.size + q)
    awgn, _ = util.synth_frames(mask, 8, ebn0_db=4.0, seed=q)
    awgn = np.clip(awgn.astype(np.int32) * (1 << q) // 64, -amp, amp)
    edge = rng.integers(-(amp + 1), amp + 1, size=(4, mask.size))
    edge[0, :64] = -(amp + 1)
    llr = np.concatenate([awgn, edge]).astype(np.int16 if q > 8 else np.int8)
    out = dec.decode(cuda.from_numpy(llr).cuda())
    cuda.cuda.synchronize()
    ref = oracle_mod.decode_fsm(mask, llr, llr_bits=q, par=c.par, sigmag=c.sigmag, extended=c.extended)
    _assert_same(pkg.unpack_bits(out.cpu().numpy(), mask.size), ref, name)
