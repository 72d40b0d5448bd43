"""The launch shapes bench.py times, decoded whole.

The pair kernel's launch depends on the batch: waves per frame pair W, which stage-slot levels
sit in LDS and whether F-descent chains run (W = 1 only). The other GPU tests decode a few
frames, i.e. W = 8 with several LDS levels; these decode the full timed batches through the
default plan -- C3: 4096 frames of frozen_n_65536_k_32768 (W = 1, 8 pairs per CU, only the
subtree-root level in LDS, chains of 3); C5: 512 and 64 frames of frozen_n_262144_k_131072
(W = 8) -- and check every frame: a noiseless round trip (random information bits, LLR
magnitudes 1..31 with the codeword's signs: SC recovers x exactly) on all frames but 8, and
equality with the oracle's literal FSM on 8 AWGN frames placed across the same launch (first,
middle and last pairs, both halves)."""
import numpy as np
import pytest

import util
from test_gpu_parity import _assert_same

# (mask, frames per GPU, layout, waves per block of the launch): C3 decodes in the frame-pair
# layout (one block per pair), C5 in the solo layout (one block per frame, subtrees of 512
# words) -- the automatic layout's choice for those batches on a 256-CU MI355X
# (+ the automatic layout's crossover, DESIGN.md 3.2.2 "The switch point, measured": 2048 frames
# of N = 65536 are the last batch in the solo layout, 3072 the first back in the pair layout, at
# one wave per pair so that the 1536 pairs stay one dispatch round)
SHAPES = [("frozen_n_65536_k_32768", 4096, 1, 1), ("frozen_n_262144_k_131072", 512, 2, 4),
          ("frozen_n_262144_k_131072", 64, 2, 8), ("frozen_n_65536_k_32768", 2048, 2, 1),
          ("frozen_n_65536_k_32768", 3072, 1, 1)]


def noiseless_batch(torch, mask, batch, seed):
    """[batch, N] int8 LLRs on the GPU: x = u F^{(x)n} for random information bits u, LLR sign
    from x (bit 1 -> negative), magnitude uniform in 1..31; and x as [batch, N] uint8."""
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    N = mask.size
    m = torch.from_numpy(mask.astype(np.uint8)).cuda()
    x = torch.randint(0, 2, (batch, N), generator=g, device="cuda", dtype=torch.uint8) & m
    h = 1
    while h < N:
        v = x.view(batch, N // (2 * h), 2, h)
        v[:, :, 0, :] ^= v[:, :, 1, :]
        h *= 2
    mag = torch.randint(1, 32, (batch, N), generator=g, device="cuda", dtype=torch.int16)
    llr = torch.where(x.bool(), -mag, mag).to(torch.int8)
    return llr, x


def awgn_rows(batch):
    """8 frame indices spread over the launch: the first, middle and last pairs (both frames)
    plus one odd-pair high frame."""
    mid = (batch // 4) * 2
    return np.array(sorted({0, 1, mid, mid + 1, batch - 2, batch - 1, 5, batch // 3 * 2 + 1}))


@pytest.mark.gpu
@pytest.mark.parametrize("name,batch,layout,W", SHAPES)
def test_timed_shape_full_batch(pkg, cuda, oracle_mod, name, batch, layout, W):
    torch = cuda
    mask = util.mask(name)
    N = mask.size
    dec = pkg.Decoder(mask)
    info = dec.launch_info(batch)
    # the shape bench.py times: one block per pair (solo: per frame), W waves
    blocks = batch // 2 if layout == 1 else batch
    assert (info["kernel"], info["layout"], info["waves_per_block"], info["blocks"]) == (3, layout, W, blocks), info
    if layout == 2:
        assert info["sub_words"] == 512, info
    # the code object build() prewarmed (the ROCm clang driver's), not a hipRTC rebuild on this
    # machine (a cache-key mismatch once made every timed kernel hipRTC code)
    assert info["compiler"] == 1, info
    if W == 1 and layout == 1:
        # C3: the subtrees' parent level in LDS (the roots are read as F / G of it), F-descent
        # chains in the generated kernel
        S = dec.stats["sub_words"]
        assert info["lds_bytes"] == 2 * S // 4 * 128 + 3 * 256, info
        assert "pop_chain<3" in dec.kernel_source()
    llr, x = noiseless_batch(torch, mask, batch, seed=batch)
    rows = awgn_rows(batch)
    noisy, _ = util.synth_frames(mask, rows.size, ebn0_db=1.0, seed=batch + 7)
    llr[torch.from_numpy(rows).cuda()] = torch.from_numpy(noisy).cuda()
    out = dec.decode(llr)
    torch.cuda.synchronize()
    got = pkg.unpack_bits(out.cpu().numpy(), N)
    keep = np.ones(batch, bool)
    keep[rows] = False
    _assert_same(got[keep], x.cpu().numpy()[keep], "%s x %d: noiseless round trip" % (name, batch))
    _assert_same(got[rows], oracle_mod.decode_fsm(mask, noisy), "%s x %d: AWGN frames vs oracle" % (name, batch))
