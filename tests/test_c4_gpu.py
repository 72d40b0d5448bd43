"""C4 on the GPU (BASELINE.json configs[3]: N=1024 K=512, 2^20 frames sharded over the GPUs
by scatter / gather). It replaces the reference's single-stream frame loop
(src/testbench/sc_top_module.h:141-155) by per-rank shards.

* Two ranks share the one MI355X of the test box (gloo collectives on CPU tensors, the same
  helpers bench.py drives over RCCL): rank 0 holds the batch, scatter_shards hands each rank
  its LLR shard, each rank decodes it with the HIP path, gather_to_root reassembles x^ on
  rank 0. The result must equal a single-process HIP decode of the whole batch and the CPU
  oracle on sampled frames.
* One rank's C4 shard at 8 GPUs (2^20 / 8 = 131072 frames) is decoded in one launch and
  checked by the size-independent noiseless encode -> decode round trip.

The parent process never initialises the GPU before spawning the ranks.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _c4_rank(rank, world, port, total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import util
        import sc_polar_decoder_hls_amd as pkg
        from sc_polar_decoder_hls_amd import sharding
        torch.cuda.set_device(0)
        cpu = torch.device("cpu")
        mask = util.mask("FB_N1024_K512")
        N = mask.size
        dec = pkg.Decoder(mask)
        full = llr = None
        if rank == 0:
            llr, _ = util.synth_frames(mask, total, ebn0_db=2.5, seed=4242)
            full = torch.from_numpy(llr)
        shard = sharding.scatter_shards(full, total, (N,), torch.int8, dist, cpu)
        start, count = sharding.shard_bounds(total, world, rank)
        out = dec.decode(shard.cuda()) if count else torch.zeros((0, dec.words), dtype=torch.int64)
        torch.cuda.synchronize()
        got = sharding.gather_to_root(out.cpu(), total, dist, cpu)
        if rank == 0:
            single = dec.decode(full.cuda()).cpu()
            same = bool(torch.equal(got, single))
            from oracle import oracle
            idx = np.random.default_rng(1).choice(total, size=96, replace=False)
            bits = pkg.unpack_bits(got.numpy()[idx], N)
            ref = oracle.decode_fsm(mask, llr[idx])
            q.put(("ok", same, bool((bits == ref).all()), [sharding.shard_bounds(total, world, r) for r in range(world)]))
    except Exception as e:   # surface worker failures to the test
        q.put(("err", repr(e), None, None))
        raise
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("total", [4099, 16384])
def test_c4_scatter_decode_gather_two_ranks(pkg, total):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c4_rank, args=(r, 2, port, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        status, same, oracle_ok, spans = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert status == "ok", same
    assert same, "scatter -> HIP decode -> gather differs from a single-process HIP decode"
    assert oracle_ok, "reassembled batch differs from the oracle on sampled frames"
    assert sum(c for _, c in spans) == total and all(c > 0 for _, c in spans)
    assert all(p.exitcode == 0 for p in procs)


@pytest.mark.gpu
def test_c4_shard_noiseless_roundtrip(pkg, cuda):
    """One 8-GPU C4 shard (131072 frames of N=1024 K=512) in one decode launch: noiseless
    LLRs of random codewords decode to the sent codeword (size-independent property)."""
    import util
    from sc_polar_decoder_hls_amd import sharding
    mask = util.mask("FB_N1024_K512")
    B = sharding.shard_bounds(1 << 20, 8, 3)[1]
    assert B == 131072
    dev = cuda.device("cuda")
    g = cuda.Generator(device=dev)
    g.manual_seed(31)
    m = cuda.from_numpy(mask.astype(np.uint8)).to(dev)
    x = cuda.randint(0, 2, (B, mask.size), generator=g, device=dev, dtype=cuda.uint8) & m
    h = 1
    while h < mask.size:                     # x = u F^(x)n (in place)
        v = x.view(B, mask.size // (2 * h), 2, h)
        v[:, :, 0, :] ^= v[:, :, 1, :]
        h *= 2
    amp = cuda.randint(1, 32, (B, 1), generator=g, device=dev, dtype=cuda.int16)
    llr = ((1 - 2 * x.to(cuda.int16)) * amp).to(cuda.int8).contiguous()
    dec = pkg.Decoder(mask)
    out = dec.decode(llr)
    cuda.cuda.synchronize()
    got = pkg.unpack_bits(out.cpu().numpy(), mask.size)
    np.testing.assert_array_equal(got, x.cpu().numpy())
