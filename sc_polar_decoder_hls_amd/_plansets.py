"""The plans the benchmark and the GPU test suite decode with, compiled ahead into
lib/rtc_cache/ by __graft_entry__.build() (host only, hipRTC), so that a GPU box loads their
code objects instead of compiling them (C5's pair kernel alone takes ~2 minutes).

Build tooling, not a decode path: the lists here are data (masks of data/frozen_masks.json,
structured masks from a seeded generator, datapath formats of the reference's sweep scripts);
tests/test_pair.py and tests/test_gpu_formats.py parametrise over the same lists.
"""
import functools
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MASKS_JSON = os.path.join(ROOT, "data", "frozen_masks.json")


@functools.lru_cache(maxsize=None)
def _masks():
    with open(MASKS_JSON) as f:
        return json.load(f)["masks"]


def mask_names():
    return list(_masks())


def mask(name):
    """Information mask (uint8, 1 = info) of a frozen-table fixture (data/frozen_masks.json)."""
    m = _masks()[name]
    b = np.frombuffer(bytes.fromhex(m["hex"]), dtype=np.uint8)
    return np.unpackbits(b, bitorder="little")[: m["N"]].astype(np.uint8)


# ---- pair plans (tests/test_pair.py) ---------------------------------------------------------
def structured_mask(rng, N, p_special=0.7):
    """Nodes of random size whose frozen pattern is R0 / R1 / REP / SPC (or random), so that the
    pruned node ops appear at every level (1 .. N/64 words)."""
    m = (rng.random(N) < 0.5).astype(np.uint8)
    pos = 0
    while pos < N:
        size = 16 << int(rng.integers(0, 6))
        size = min(size, N - pos)
        if rng.random() < p_special:
            kind = int(rng.integers(0, 4))
            blk = np.zeros(size, np.uint8)
            if kind == 1:
                blk[:] = 1                  # R1
            elif kind == 2:
                blk[-1] = 1                 # REP
            elif kind == 3:
                blk[:] = 1
                blk[0] = 0                  # SPC
            m[pos:pos + size] = blk
        pos += size
    return m


@functools.lru_cache(maxsize=None)
def struct_masks(N):
    rng = np.random.default_rng(N)
    return tuple(structured_mask(rng, N) for _ in range(3))


@functools.lru_cache(maxsize=None)
def wave_mask():
    return structured_mask(np.random.default_rng(4242), 16384, 0.9)


PARITY_MASKS = [("frozen_n_2048_k_1024", 23), ("FB_N2048_K1024", 8), ("frozen_n_4096_k_2048", 17),
                ("frozen_n_8192_k_4096", 9), ("frozen_n_16384_k_8192", 7), ("frozen_n_32768_k_29492", 5),
                ("frozen_n_2048_k_1844", 12), ("frozen_n_16384_k_14746", 6), ("frozen_n_65536_k_32768", 5)]
STRUCT_SUB_WORDS = (32, 64, 256)
PAR64_MASKS = [("frozen_n_2048_k_1024", 9), ("frozen_n_16384_k_8192", 5), ("frozen_n_16384_k_14746", 5),
               ("frozen_n_65536_k_32768", 3)]


def struct_sub_words(N):
    return [sw for sw in STRUCT_SUB_WORDS if sw <= N // 32]   # subtrees of at most half the code


def gpu_plans():
    """(name, mask, tuning) of every pair plan the GPU tests decode with."""
    p = {"kernel": 3, "layout": 1}   # (tests/test_pair.py pair(): the frame-pair layout)
    out = [(n, mask(n), dict(p)) for n, _ in PARITY_MASKS]
    for N in (2048, 8192, 32768):
        for i, m in enumerate(struct_masks(N)):
            out += [("struct%d_%d" % (N, i), m, dict(p, sub_words=sw)) for sw in struct_sub_words(N)]
    out += [("frozen_n_2048_k_1024", mask("frozen_n_2048_k_1024"), dict(p, sub_words=sw)) for sw in (32, 64)]
    out += [("frozen_n_8192_k_4096", mask("frozen_n_8192_k_4096"), dict(p, sub_words=256)),
            ("frozen_n_16384_k_8192", mask("frozen_n_16384_k_8192"), dict(p, sub_words=64)),
            ("wave_mask", wave_mask(), dict(p, sub_words=64)),
            ("frozen_n_32768_k_29492", mask("frozen_n_32768_k_29492"), dict(p, tier_words=512, sub_words=128)),
            ("frozen_n_262144_k_131072", mask("frozen_n_262144_k_131072"), dict(p)),
            ("frozen_n_262144_k_131072", mask("frozen_n_262144_k_131072"), dict(p, tier_words=1024)),
            ("frozen_n_65536_k_32768", mask("frozen_n_65536_k_32768"), dict(p, lds_slots=256)),
            ("frozen_n_65536_k_32768", mask("frozen_n_65536_k_32768"), dict(p, lds_slots=1024)),
            ("frozen_n_65536_k_32768", mask("frozen_n_65536_k_32768"), dict(p, sub_root=1)),
            ("frozen_n_65536_k_32768", mask("frozen_n_65536_k_32768"), dict(p, sub_root=2)),
            ("frozen_n_65536_k_32768", mask("frozen_n_65536_k_32768"), {"kernel": 3, "layout": 2, "sub_root": 1}),
            ("frozen_n_65536_k_32768", mask("frozen_n_65536_k_32768"), {"kernel": 3, "layout": 2, "sub_root": 2})]
    for wpg in (1, 2, 4, 8):
        out += [("frozen_n_16384_k_8192", mask("frozen_n_16384_k_8192"), dict(p, waves_per_group=wpg, sub_words=64)),
                ("wave_mask", wave_mask(), dict(p, waves_per_group=wpg, sub_words=64))]
    return out


SOLO_SUB_WORDS = (64, 256, 512)


def solo_sub_words(N):
    """solo plans: subtrees of 64 .. 512 words, at most half the code"""
    return [sw for sw in SOLO_SUB_WORDS if sw <= N // 32]


def solo_plans():
    """(name, mask, tuning) of the solo-layout GPU tests (tests/test_solo.py) and the bench."""
    t = {"kernel": 3, "layout": 2}
    out = [(n, mask(n), dict(t)) for n, _ in PARITY_MASKS]
    for N in (2048, 8192, 32768):
        for i, m in enumerate(struct_masks(N)):
            out += [("struct%d_%d" % (N, i), m, dict(t, sub_words=sw)) for sw in solo_sub_words(N)]
    out += [("frozen_n_2048_k_1024", mask("frozen_n_2048_k_1024"), dict(t, sub_words=64)),
            ("frozen_n_8192_k_4096", mask("frozen_n_8192_k_4096"), dict(t, sub_words=256)),
            ("frozen_n_16384_k_8192", mask("frozen_n_16384_k_8192"), dict(t, sub_words=512)),
            ("frozen_n_16384_k_8192", mask("frozen_n_16384_k_8192"), dict(t, sub_words=64)),
            ("wave_mask", wave_mask(), dict(t, sub_words=64)),
            ("frozen_n_32768_k_29492", mask("frozen_n_32768_k_29492"), dict(t, tier_words=512, sub_words=128)),
            ("frozen_n_262144_k_131072", mask("frozen_n_262144_k_131072"), dict(t, sub_words=256)),
            ("frozen_n_262144_k_131072", mask("frozen_n_262144_k_131072"), dict(t, sub_words=512)),
            ("frozen_n_65536_k_32768", mask("frozen_n_65536_k_32768"), dict(t, sub_words=512))]
    for wpg in (1, 2, 4, 8):
        out += [("frozen_n_16384_k_8192", mask("frozen_n_16384_k_8192"), dict(t, waves_per_group=wpg, sub_words=64)),
                ("wave_mask", wave_mask(), dict(t, waves_per_group=wpg, sub_words=64))]
    return out


PAIR_PARS = (32, 64)   # PAR > 16 on the pair kernel (script_tests.sh:11,124 sweeps 64)


def gpu_par64_plans():
    """(name, mask, config fields, tuning) of the PAR 32 / 64 pair-kernel GPU tests and bench
    entries."""
    out = []
    for par in PAIR_PARS:
        out += [(n, mask(n), {"par": par}, {"kernel": 3}) for n, _ in PAR64_MASKS]
        for N in (8192, 32768):
            for i, m in enumerate(struct_masks(N)[:2]):
                out += [("struct%d_%d" % (N, i), m, {"par": par}, {"kernel": 3, "sub_words": sw}) for sw in (64, 256)]
    return out


def cpu_test_plans():
    """(name, mask, tuning) of the plans the CPU register-budget test compiles (the round-3
    dispatch abort's configuration: chain_max = 4 on the structured N = 32768 mask)."""
    return [("struct32768_0", struct_masks(32768)[0], {"kernel": 3, "layout": 1, "sub_words": sw, "chain_max": 4,
                                                       "sub_root": 1}) for sw in (64, 256)] + \
        [("struct16384_0", struct_masks(16384)[0], {"kernel": 3, "layout": 1, "sub_words": 64, "chain_max": 4,
                                                    "sub_root": 1}),
         # tests/test_solo.py::test_solo_plan_stats: a pair-tuned automatic plan and its solo alternate
         ("frozen_n_65536_k_32768", mask("frozen_n_65536_k_32768"), {"sub_words": 64, "waves_per_group": 2})]


# ---- CA2 on the pair kernel (tests/test_ca2.py) -------------------------------------------------
def ca2_first_mask(N):
    """the rate-1/2 reference mask of N with information bits in its first 16-LLR word, so that
    leaf 0 is decoded and meets MIN (-2^(Q-1)) on the leftmost path"""
    m = mask("frozen_n_%d_k_%d" % (N, N // 2)).copy()
    m[:16] = np.random.default_rng(N).integers(0, 2, 16)
    m[[3, 5, 11, 15]] = 1
    return m


def ca2_gpu_items():
    """(id, mask, CA2 config fields, tuning) of the CA2 pair-kernel GPU tests"""
    out = []
    for n in ("frozen_n_2048_k_1024", "frozen_n_16384_k_8192", "frozen_n_65536_k_32768"):
        out.append((n, mask(n), {}, None))
    for N in (2048, 16384):
        out.append(("first%d" % N, ca2_first_mask(N), {}, None))
    for i, m in enumerate(struct_masks(8192)):
        out += [("struct8192_%d_s%d" % (i, sw), m, {}, {"kernel": 3, "layout": 1, "sub_words": sw}) for sw in (32, 256)]
    fm = ca2_first_mask(16384)
    for par in (16, 32, 64):
        for q in (5, 6, 7, 8, 9):
            for ext in (1, 0):
                out.append(("first16384_p%d_q%d_e%d" % (par, q, ext), fm, {"par": par, "llr_bits": q, "extended": ext}, None))
    out.append(("first16384_pl0", fm, {"pruning_level": 0}, None))
    # PRUNING_LEVEL 1 at PAR 16: the leaf records' REP / SPC / REP2 / SPC2 / R1 decoders
    for c7 in PRUNING_SWEEP:
        if c7[0] == 1:
            out.append(("first16384_pl1_%s" % "".join(map(str, c7[1:])), fm, c7_fields(c7), None))
    out.append(("first2048_pl1_q8_e0", ca2_first_mask(2048), dict(c7_fields((1, 1, 1, 1, 1, 1, 0)), llr_bits=8,
                                                                   extended=0), None))
    # ... and at PAR 32 / 64: the decoders of the whole PAR word (OP_PLEAF)
    for par in (32, 64):
        for c7 in ((1, 1, 0, 0, 0, 0, 0), (1, 1, 1, 1, 0, 0, 0), (1, 1, 1, 1, 1, 1, 0)):
            out.append(("first16384_p%d_pl1_%s" % (par, "".join(map(str, c7[1:]))), fm, dict(c7_fields(c7), par=par), None))
        out.append(("first16384_p%d_pl1_q8_e0" % par, fm, dict(c7_fields((1, 1, 1, 1, 1, 1, 0)), par=par, llr_bits=8,
                                                             extended=0), None))
    out.append(("first2048_p64_pl0", ca2_first_mask(2048), {"par": 64, "pruning_level": 0}, None))
    for wpg in (1, 2, 4, 8):
        out.append(("wave_mask_w%d" % wpg, wave_mask(), {}, {"kernel": 3, "layout": 1, "waves_per_group": wpg, "sub_words": 64}))
    out.append(("first16384_fused", fm, {}, {"kernel": 3, "layout": 1, "sub_root": 2}))
    out.append(("tier32768", mask("frozen_n_32768_k_29492"), {}, {"kernel": 3, "layout": 1, "tier_words": 512,
                                                                   "sub_words": 128}))
    return out


# ---- PAR 4 / 8 on the pair kernel (tests/test_par48.py) ---------------------------------
def par48_gpu_items():
    """(id, mask, config fields, tuning) of the PAR 4 / 8 pair-kernel GPU tests"""
    out = []
    for par in (4, 8):
        P = {"par": par}
        for n in ("frozen_n_2048_k_1024", "frozen_n_16384_k_8192", "frozen_n_65536_k_32768"):
            out.append(("%s_p%d" % (n, par), mask(n), P, None))
        rng = np.random.default_rng(480 + par)
        pm = planted_mask(rng, 16384, par)
        for c7 in (SHIPPED_C7, (1, 1, 1, 1, 1, 1, 0), (0, 0, 0, 0, 0, 0, 0), (2, 1, 1, 1, 1, 1, 1)):
            out.append(("planted16384_p%d_pl%d_%d" % (par, c7[0], sum(c7)), pm, dict(c7_fields(c7), **P), None))
        for q in (5, 8, 9):
            for ext in (1, 0):
                out.append(("planted16384_p%d_q%d_e%d" % (par, q, ext), pm, dict(P, llr_bits=q, extended=ext), None))
        for i, m in enumerate(struct_masks(8192)):
            out += [("struct8192_%d_p%d_s%d" % (i, par, sw), m, P, {"kernel": 3, "layout": 1, "sub_words": sw})
                    for sw in (32, 256)]
        for wpg in (1, 8):
            out.append(("wave_mask_p%d_w%d" % (par, wpg), wave_mask(), P,
                        {"kernel": 3, "layout": 1, "waves_per_group": wpg, "sub_words": 64}))
        out.append(("planted16384_p%d_fused" % par, pm, P, {"kernel": 3, "layout": 1, "sub_root": 2}))
        out.append(("tier32768_p%d" % par, mask("frozen_n_32768_k_29492"), P,
                    {"kernel": 3, "layout": 1, "tier_words": 512, "sub_words": 128}))
        # CA2: the first word informative (MIN reaches the leaf of word 0), every pruning level
        C = dict(P, sigmag=0)
        fm = ca2_first_mask(16384)
        for n in ("frozen_n_2048_k_1024", "frozen_n_65536_k_32768"):
            out.append(("%s_p%d_ca2" % (n, par), mask(n), C, None))
        for c7 in (SHIPPED_C7, (1, 1, 1, 1, 1, 1, 0), (0, 0, 0, 0, 0, 0, 0)):
            out.append(("first16384_p%d_ca2_pl%d" % (par, c7[0]), fm, dict(c7_fields(c7), **C), None))
            out.append(("planted16384_p%d_ca2_pl%d" % (par, c7[0]), pm, dict(c7_fields(c7), **C), None))
        for q in (5, 8, 9):
            for ext in (1, 0):
                out.append(("first16384_p%d_ca2_q%d_e%d" % (par, q, ext), fm, dict(C, llr_bits=q, extended=ext), None))
        out.append(("first2048_p%d_ca2_s32" % par, ca2_first_mask(2048), C, {"kernel": 3, "layout": 1, "sub_words": 32}))
        out.append(("first16384_p%d_ca2_fused" % par, fm, C, {"kernel": 3, "layout": 1, "sub_root": 2}))
    return out


# ---- LLR_BITS 9 (tests/test_gpu_formats.py test_llr9_pair_kernel, tests/test_solo.py q9 tests):
# automatic plans, which hold the solo alternate for small batches ----------------------------
Q9_MASKS = ("frozen_n_2048_k_1024", "frozen_n_16384_k_8192", "frozen_n_65536_k_32768", "frozen_n_262144_k_131072")


def q9_items():
    out = []
    for ext in (1, 0):
        out += [(n, mask(n), {"llr_bits": 9, "extended": ext}, None) for n in Q9_MASKS]
        out.append(("struct8192_1", struct_masks(8192)[1], {"llr_bits": 9, "extended": ext}, None))
    return out


def ca2_items():
    """ca2_gpu_items as prewarm items (CA2 config fields)"""
    return [(n, m, dict(f, sigmag=0), t) for n, m, f, t in ca2_gpu_items()]


# ---- datapath formats (tests/test_gpu_formats.py): (PAR, SIGMAG, EXTENDED, LLR_BITS) ---------
FORMATS = [
    (16, 0, 1, 6), (16, 0, 1, 8), (16, 0, 0, 6), (16, 1, 0, 6), (16, 1, 1, 9), (16, 0, 1, 9),
    (32, 1, 1, 6), (32, 0, 1, 6), (32, 1, 0, 8), (64, 1, 1, 6), (64, 1, 1, 8), (64, 0, 1, 6), (64, 1, 0, 6), (64, 0, 0, 8),
    (64, 1, 1, 9),
    # PAR 4 / 8 (script_RTL_sim.sh:97-330): PAR words as lane groups of a device word
    (8, 1, 1, 6), (8, 0, 1, 6), (8, 1, 0, 8), (8, 1, 1, 8), (4, 1, 1, 6), (4, 0, 0, 8), (4, 1, 1, 8),
    (4, 1, 1, 9),
]

# the rate-0.9 codes of script_tests.sh:7-9 (QUANT 8)
RATE09_MASKS = ("frozen_n_2048_k_1844", "frozen_n_4096_k_3686", "frozen_n_8192_k_7372", "frozen_n_16384_k_14746")

# ---- pruning / ELAG sweep (tests/test_gpu_configs.py, test_gpu_formats.py) -------------------
# (pruning_level, elag_r1, elag_rep, elag_spc, elag_rep2, elag_spc2, elag_h0): the loop of
# script/script_tests.sh:103-122, then REP2 / SPC2 / H0 switched at PRUNING_LEVEL 2
PRUNING_SWEEP = (
    (0, 0, 0, 0, 0, 0, 0), (1, 0, 0, 0, 0, 0, 0), (1, 1, 0, 0, 0, 0, 0), (1, 1, 1, 0, 0, 0, 0),
    (1, 1, 1, 1, 0, 0, 0), (1, 1, 1, 1, 1, 0, 0), (1, 1, 1, 1, 1, 1, 0), (2, 0, 0, 0, 0, 0, 1),
    (2, 1, 0, 0, 0, 0, 1), (2, 1, 1, 0, 0, 0, 1), (2, 1, 1, 1, 0, 0, 1),
    (2, 1, 1, 1, 0, 0, 0), (2, 1, 1, 1, 1, 1, 1),
)
SHIPPED_C7 = (2, 1, 1, 1, 0, 0, 1)   # config.h
SWEEP_MASKS = ("FB_N128_K64", "FB_N1024_K512", "frozen_n_2048_k_1024", "frozen_n_8192_k_4096")
PLANTED_N = (32, 256, 1024, 4096)
FORMAT_C7 = ((2, 1, 1, 1, 0, 0, 1), (1, 1, 1, 1, 1, 1, 0), (0, 0, 0, 0, 0, 0, 0), (2, 1, 1, 1, 1, 1, 0))
QBITS_MASKS = ("FB_N128_K64", "FB_N1024_K512", "frozen_n_4096_k_2048")


def planted_mask(rng, N, par=16):
    """Random mask with PAR groups of every pruned class (R0 / R1 / REP / SPC / REP2 / SPC2)."""
    all1 = (1 << par) - 1
    pats = [0, all1, 1 << (par - 1), all1 & ~1, 3 << (par - 2), all1 & ~3]
    m = (rng.random(N) < 0.5).astype(np.uint8)
    for g in range(N // par):
        if rng.random() < 0.6:
            p = int(rng.choice(pats))
            m[par * g:par * g + par] = [(p >> k) & 1 for k in range(par)]
    return m


def sweep_planted_mask(N):
    return planted_mask(np.random.default_rng(800 + N), N)


def format_seed(fmt):
    par, sigmag, ext, q = fmt
    return par * 7 + sigmag * 3 + ext + q * 11


def format_masks(fmt):
    """(name, mask) of the format test: LDS (N <= 4096) and HBM-scratch (N = 16384) storage."""
    par = fmt[0]
    return [("FB_N1024_K512", mask("FB_N1024_K512")),
            ("planted_4096", planted_mask(np.random.default_rng(format_seed(fmt)), 4096, par)),
            ("frozen_n_16384_k_8192", mask("frozen_n_16384_k_8192"))]


def c7_fields(c7):
    keys = ("pruning_level", "elag_r1", "elag_rep", "elag_spc", "elag_rep2", "elag_spc2", "elag_h0")
    return dict(zip(keys, c7))


def sweep_items():
    """(name, mask, config fields, tuning) of every plan the pruning / format sweeps decode."""
    out = []
    for c7 in PRUNING_SWEEP:
        out += [(n, mask(n), c7_fields(c7), None) for n in SWEEP_MASKS]
        out += [("planted%d" % N, sweep_planted_mask(N), c7_fields(c7), None) for N in PLANTED_N]
    # script_tests.sh:105-106's loop at PAR 16, QUANT 8 on the default (pair) kernel
    out += [("frozen_n_32768_k_29492", mask("frozen_n_32768_k_29492"), dict(c7_fields(c7), llr_bits=8, par=par), None)
            for c7 in PRUNING_SWEEP for par in (16, 64, 32, 8, 4)]
    for q in (5, 7, 8):
        for c7 in (SHIPPED_C7, (1, 1, 1, 1, 1, 1, 0)):
            out += [(n, mask(n), dict(c7_fields(c7), llr_bits=q), None) for n in QBITS_MASKS]
    for fmt in FORMATS:
        par, sigmag, ext, q = fmt
        for n, m in format_masks(fmt):
            out += [(n, m, dict(c7_fields(c7), par=par, sigmag=sigmag, extended=ext, llr_bits=q), None)
                    for c7 in FORMAT_C7]
    return out


def prewarm_all(verbose=False):
    """Compile every plan above (and the reference-config plan of every mask fixture) into
    lib/rtc_cache/."""
    import sc_polar_decoder_hls_amd as pkg
    from sc_polar_decoder_hls_amd import _build
    _build.prewarm({n: mask(n) for n in mask_names() if mask(n).size >= 32}, verbose=verbose)
    # the schedule interpreter of every datapath format the GPU tests exercise (LDS and
    # HBM-scratch storage): its source depends on the format, not on the mask
    cfgs = []
    for par, sigmag, ext, q in FORMATS:
        c = pkg.default_config()
        c.par, c.sigmag, c.extended, c.llr_bits = par, sigmag, ext, q
        cfgs.append(c)
    _build.prewarm({n: mask(n) for n in ("FB_N1024_K512", "frozen_n_16384_k_8192")}, configs=cfgs, verbose=verbose)
    q8 = pkg.default_config()
    q8.llr_bits = 8
    _build.prewarm({n: mask(n) for n in RATE09_MASKS}, configs=[q8], verbose=verbose)
    _build.prewarm_plans(gpu_plans() + solo_plans() + cpu_test_plans(), verbose=verbose)
    _build.prewarm_items(gpu_par64_plans(), verbose=verbose)
    # the pruning / ELAG / format sweeps: PRUNING_LEVEL 1 leaf decoders and EXTENDED 0 run the
    # generated kernels (one code object per mask and configuration); the interpreter formats
    # share one per format
    _build.prewarm_items(sweep_items(), verbose=verbose)
    _build.prewarm_items(ca2_items(), verbose=verbose)
    _build.prewarm_items(q9_items(), verbose=verbose)
    _build.prewarm_items(par48_gpu_items(), verbose=verbose)
    _build.prewarm_items(high_rate_items(), verbose=verbose)


# ---- high-rate codes across the formats (tests/test_gpu_formats.py
# test_high_rate_codes_formats): the rate-0.9 codes of script_tests.sh:7-9 and the N = 1024
# K = 922 code of script_RTL_sim.sh:87-97 (PAR 4..64 at QUANT 8; N = 1024 on the pair kernel
# since round 6), at LLR_BITS 6 and 8, SIGMAG and CA2 ------------------------------------------
HIGH_RATE_MASKS = ("frozen_n_1024_k_922", "frozen_n_2048_k_1844", "frozen_n_4096_k_3686")
HIGH_RATE_FORMATS = [(p, s, e, q) for q in (6, 8) for p, s, e in
                     ((64, 1, 1), (32, 1, 1), (16, 1, 1), (8, 1, 1), (4, 1, 1), (64, 0, 0), (16, 0, 1), (4, 0, 1))] + \
    [(64, 0, 1, 9), (64, 0, 0, 9)]   # (CA2 at LLR_BITS 9, PAR 64: the saturating REP accumulate)


def high_rate_items():
    out = []
    for n in HIGH_RATE_MASKS:
        for p, s, e, q in HIGH_RATE_FORMATS:
            out.append(("%s_p%d_%s_e%d_q%d" % (n, p, "sm" if s else "ca2", e, q), mask(n),
                        {"par": p, "sigmag": s, "extended": e, "llr_bits": q}, None))
    return out
