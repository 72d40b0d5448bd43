"""GPU parity over the reference's pruning sweep (script/script_tests.sh:103-122): every
config decodes on the device bit-exact with the config-aware literal FSM oracle. Every config
runs the generated kernels of the shipped datapath (per-mask for N <= 1024, pair above),
PRUNING_LEVEL 1's REP / SPC / REP2 / SPC2 leaf decoders included (leaf_gen)."""
import numpy as np
import pytest

import util
from sc_polar_decoder_hls_amd._plansets import PRUNING_SWEEP, QBITS_MASKS, SHIPPED_C7, SWEEP_MASKS, \
    PLANTED_N, sweep_planted_mask
from test_gpu_parity import _assert_same

pytestmark = pytest.mark.gpu

GENERATED = (1, 3)   # stats["kernel"]: per-mask, pair


def _cfg(pkg, c7):
    c = pkg.default_config()
    (c.pruning_level, c.elag_r1, c.elag_rep, c.elag_spc, c.elag_rep2, c.elag_spc2, c.elag_h0) = c7
    return c


def _run(pkg, torch, mask, llr, c7):
    dec = pkg.Decoder(mask, config=_cfg(pkg, c7))
    out = dec.decode(torch.from_numpy(np.ascontiguousarray(llr)).cuda())
    torch.cuda.synchronize()
    return pkg.unpack_bits(out.cpu().numpy(), mask.size), dec.stats["kernel"]


@pytest.mark.parametrize("name", SWEEP_MASKS)
def test_sweep_configs_awgn(pkg, cuda, oracle_mod, name):
    mask = util.mask(name)
    batch = 41 if mask.size <= 1024 else 11
    llr, _ = util.synth_frames(mask, batch, ebn0_db=1.0, seed=99)
    for c7 in PRUNING_SWEEP:
        got, kernel = _run(pkg, cuda, mask, llr, c7)
        _assert_same(got, oracle_mod.decode_fsm(mask, llr, config=c7), "%s %s kernel %d" % (name, c7, kernel))
        assert mask.size < 32 or kernel in GENERATED, (name, c7, kernel)


def test_sweep_configs_planted_groups(pkg, cuda, oracle_mod):
    """Masks planted with PAR groups of every pruned class, so that each PRUNING_LEVEL 1 leaf
    decoder (REP / SPC / REP2 / SPC2) and each level-2 node class occurs."""
    rng = np.random.default_rng(8)
    for N in PLANTED_N:
        mask = sweep_planted_mask(N)
        llr = rng.integers(-32, 32, size=(19, N)).astype(np.int8)
        for c7 in PRUNING_SWEEP:
            got, kernel = _run(pkg, cuda, mask, llr, c7)
            _assert_same(got, oracle_mod.decode_fsm(mask, llr, config=c7), "N=%d %s kernel %d" % (N, c7, kernel))
            assert N < 64 or kernel in GENERATED, (N, c7, kernel)


@pytest.mark.parametrize("q", [5, 7, 8])
def test_llr_bits_configs(pkg, cuda, oracle_mod, q):
    """LLR_BITS other than the shipped 6 (config.h:2; the reference's pruning sweep runs at
    QUANT = 8, script/script_tests.sh:9,25): the per-mask and pair kernels (PRUNING_LEVEL 2 and
    PRUNING_LEVEL 1 with its leaf decoders) against the oracle at the same LLR_BITS, on AWGN
    frames at that quantisation and on the whole int8 range."""
    rng = np.random.default_rng(50 + q)
    amp = (1 << (q - 1)) - 1
    for name in QBITS_MASKS:
        mask = util.mask(name)
        awgn, _ = util.synth_frames(mask, 12, ebn0_db=1.5, seed=q)
        awgn = np.clip(awgn.astype(np.int32) * (1 << q) // 64, -amp, amp)
        llr = np.concatenate([awgn, rng.integers(-128, 128, size=(7, mask.size))]).astype(np.int8)
        for c7 in (SHIPPED_C7, (1, 1, 1, 1, 1, 1, 0)):
            c = _cfg(pkg, c7)
            c.llr_bits = q
            dec = pkg.Decoder(mask, config=c)
            out = dec.decode(cuda.from_numpy(llr).cuda())
            cuda.cuda.synchronize()
            got = pkg.unpack_bits(out.cpu().numpy(), mask.size)
            _assert_same(got, oracle_mod.decode_fsm(mask, llr, config=c7, llr_bits=q),
                         "%s q=%d %s kernel %d" % (name, q, c7, dec.stats["kernel"]))
