"""The plan lists build() prewarms (sc_polar_decoder_hls_amd/_plansets.py) are the ones the GPU
tests decode: the pruning sweep equals the oracle's (script_tests.sh:103-122) plus the two
level-2 variants, the planted masks are reproducible, and every sweep item makes a plan."""
import numpy as np

from sc_polar_decoder_hls_amd import _plansets as ps


def test_sweep_lists_match_oracle(oracle_mod):
    assert ps.PRUNING_SWEEP[:len(oracle_mod.SWEEP_CONFIGS)] == oracle_mod.SWEEP_CONFIGS
    assert ps.SHIPPED_C7 == oracle_mod.DEFAULT_CONFIG
    assert len(set(ps.PRUNING_SWEEP)) == len(ps.PRUNING_SWEEP)


def test_planted_masks_reproducible():
    for N in ps.PLANTED_N:
        a, b = ps.sweep_planted_mask(N), ps.sweep_planted_mask(N)
        assert a.dtype == np.uint8 and a.size == N and (a == b).all()
    fmt = ps.FORMATS[0]
    rng = np.random.default_rng(ps.format_seed(fmt))
    assert (ps.planted_mask(rng, 4096, fmt[0]) == ps.format_masks(fmt)[1][1]).all()


def test_sweep_items_make_plans(pkg):
    """Every sweep item is a valid plan; the shipped datapath (SIGMAG, PAR 16, LLR_BITS <= 8)
    takes a generated kernel whatever its pruning level or EXTENDED switch."""
    seen = set()
    for name, mask, fields, _ in ps.sweep_items():
        key = (name, tuple(sorted(fields.items())))
        if key in seen or mask.size > 8192:
            continue
        seen.add(key)
        c = pkg.default_config()
        for k, v in fields.items():
            setattr(c, k, v)
        st = pkg.Decoder(mask, c).stats
        if c.sigmag == 1 and c.par == 16 and c.llr_bits <= 8 and mask.size >= 64:
            assert st["kernel"] in (1, 3), (name, fields, st["kernel"])
