"""GPU parity: the HIP decoder (through the C ABI) must be bit-exact with the CPU oracle
(literal restatement of my_module::do_action) on the same LLR frames."""
import numpy as np
import pytest

import util

pytestmark = pytest.mark.gpu


def make_decoder(pkg, mask, jit=True, **tuning):
    """jit=True: default plan (per-mask register kernel for N <= 1024); False: schedule
    interpreter (polar_sc_tuning.kernel = 1)."""
    return pkg.Decoder(mask, tuning=dict(tuning, kernel=0 if jit else 1))


def _decode(pkg, torch, mask, llr, jit=True):
    dec = make_decoder(pkg, mask, jit)
    out = dec.decode(torch.from_numpy(np.ascontiguousarray(llr)).cuda())
    torch.cuda.synchronize()
    return pkg.unpack_bits(out.cpu().numpy(), mask.size)


def _assert_same(got, ref, what):
    bad = np.nonzero((got != ref).any(axis=1))[0]
    assert bad.size == 0, "%s: %d/%d frames differ (first %s)" % (what, bad.size, len(ref), bad[:8])


def test_dpp_row_exchange(pkg, cuda):
    t = pkg.selftest_lanes()
    lanes = np.arange(64)
    for h in range(4):
        np.testing.assert_array_equal(t[h], lanes ^ (1 << h), err_msg="xorlane<%d>" % (1 << h))
    # frame-pair layout (polar_sc_pair.h swap16 / swap32): rows (x0 x1 x2 x3) ->
    # (x0 x0 x2 x2), (x1 x1 x3 x3) and (x0 x1 x0 x1), (x2 x3 x2 x3)
    np.testing.assert_array_equal(t[4], lanes & ~16, err_msg="permlane16_swap a")
    np.testing.assert_array_equal(t[5], lanes | 16, err_msg="permlane16_swap b")
    np.testing.assert_array_equal(t[6], lanes & ~32, err_msg="permlane32_swap a")
    np.testing.assert_array_equal(t[7], lanes | 32, err_msg="permlane32_swap b")


@pytest.mark.parametrize("name", ["FB_N128_K64", "FB_N256_K128", "FB_N512_K256", "FB_N1024_K512",
                                  "frozen_n_1024_k_512", "frozen_n_1024_k_768", "FB_N2048_K1024",
                                  "frozen_n_2048_k_1024", "frozen_n_4096_k_2048"])
@pytest.mark.parametrize("ebn0", [0.0, 2.5])
@pytest.mark.parametrize("jit", [True, False], ids=["maskkernel", "interp"])
def test_parity_awgn(pkg, cuda, oracle_mod, name, ebn0, jit):
    mask = util.mask(name)
    batch = 67 if mask.size <= 1024 else 19
    llr, _ = util.synth_frames(mask, batch, ebn0_db=ebn0, seed=1234 + int(ebn0 * 10))
    _assert_same(_decode(pkg, cuda, mask, llr, jit), oracle_mod.decode_fsm(mask, llr), name)


@pytest.mark.parametrize("kind", ["uniform6", "int8_wrap", "zero", "sat", "minus32", "tiny"])
@pytest.mark.parametrize("jit", [True, False], ids=["maskkernel", "interp"])
def test_parity_llr_edge_cases(pkg, cuda, oracle_mod, kind, jit):
    mask = util.mask("FB_N1024_K512")
    rng = np.random.default_rng(99)
    shape = (40, mask.size)
    llr = {
        "uniform6": lambda: rng.integers(-31, 32, shape),
        "int8_wrap": lambda: rng.integers(-128, 128, shape),
        "zero": lambda: np.zeros(shape, int),
        "sat": lambda: rng.choice([-31, 31], shape),
        "minus32": lambda: rng.choice([-32, -1, 0, 1], shape),
        "tiny": lambda: rng.integers(-1, 2, shape),
    }[kind]().astype(np.int8)
    _assert_same(_decode(pkg, cuda, mask, llr, jit), oracle_mod.decode_fsm(mask, llr), kind)


@pytest.mark.parametrize("batch", [1, 3, 8, 9, 15, 16, 33])
def test_parity_ragged_batches(pkg, cuda, oracle_mod, batch):
    mask = util.mask("FB_N1024_K512")
    llr, _ = util.synth_frames(mask, batch, ebn0_db=1.0, seed=batch)
    _assert_same(_decode(pkg, cuda, mask, llr), oracle_mod.decode_fsm(mask, llr), "batch %d" % batch)


def test_parity_random_masks(pkg, cuda, oracle_mod):
    rng = np.random.default_rng(2024)
    for trial in range(40):
        N = int(2 ** rng.integers(5, 12))
        kind = trial % 4
        if kind == 0:
            mask = rng.integers(0, 2, N)
        elif kind == 1:
            pats = [0, 0xFFFF, 0x8000, 0xFFFE, int(rng.integers(0, 65536))]
            mask = np.concatenate([[(p >> k) & 1 for k in range(16)] for p in rng.choice(pats, N // 16)])
        elif kind == 2:
            mask = (rng.random(N) < np.linspace(0, 1, N) ** 0.5).astype(int)
        else:
            mask = np.full(N, trial & 1)
        mask = mask.astype(np.uint8)
        llr = rng.integers(-32, 32, size=(13, N)).astype(np.int8)
        _assert_same(_decode(pkg, cuda, mask, llr, jit=(trial % 2 == 0)), oracle_mod.decode_fsm(mask, llr),
                     "random mask trial %d N=%d" % (trial, N))


def test_kat_codewords_noiseless(pkg, cuda):
    cws = util.kat()
    for name, key in (("FB_N512_K256", "cw512x256"), ("FB_N1024_K512", "cw1024x512")):
        mask = util.mask(name)
        x = np.array(cws[key], dtype=np.uint8)
        llr = np.where(x == 1, -31, 31).astype(np.int8)
        np.testing.assert_array_equal(_decode(pkg, cuda, mask, llr), x, err_msg=key)


def test_u16_and_host_entry_points(pkg, cuda, oracle_mod):
    mask = util.mask("frozen_n_1024_k_512")
    llr, _ = util.synth_frames(mask, 21, ebn0_db=1.5, seed=5)
    ref = oracle_mod.decode_fsm(mask, llr)
    dec = pkg.Decoder(mask)
    assert dec.stats["storage"] == 2
    w16 = dec.decode_u16(cuda.from_numpy(llr).cuda())
    cuda.cuda.synchronize()
    bits16 = np.unpackbits(w16.cpu().numpy().view(np.uint8), axis=1, bitorder="little")
    _assert_same(bits16, ref, "decode_u16")
    host = dec.decode_host(llr)
    _assert_same(pkg.unpack_bits(host, mask.size), ref, "decode_host")


@pytest.mark.parametrize("jit", [True, False], ids=["maskkernel", "interp"])
def test_n32_output_padding(pkg, cuda, oracle_mod, jit):
    rng = np.random.default_rng(32)
    mask = rng.integers(0, 2, 32).astype(np.uint8)
    llr = rng.integers(-31, 32, size=(11, 32)).astype(np.int8)
    dec = make_decoder(pkg, mask, jit)
    out = dec.decode(cuda.from_numpy(llr).cuda())
    cuda.cuda.synchronize()
    words = out.cpu().numpy().view(np.uint64)
    assert words.shape == (11, 1) and not (words >> np.uint64(32)).any()
    _assert_same(pkg.unpack_bits(words, 32), oracle_mod.decode_fsm(mask, llr), "N=32")


@pytest.mark.parametrize("name,batch", [("frozen_n_8192_k_4096", 17), ("frozen_n_16384_k_8192", 9)])
def test_parity_hbm_scratch_path(pkg, cuda, oracle_mod, name, batch):
    mask = util.mask(name)
    dec = pkg.Decoder(mask)
    assert dec.stats["storage"] == 1
    llr, _ = util.synth_frames(mask, batch, ebn0_db=1.0, seed=77)
    _assert_same(_decode(pkg, cuda, mask, llr), oracle_mod.decode_fsm(mask, llr), name)


def test_parity_c3_mask_sample(pkg, cuda, oracle_mod):
    """BASELINE config C3 mask (N=65536) on a sample the oracle finishes in seconds."""
    mask = util.mask("frozen_n_65536_k_32768")
    llr, _ = util.synth_frames(mask, 9, ebn0_db=1.0, seed=65536)
    _assert_same(_decode(pkg, cuda, mask, llr), oracle_mod.decode_fsm(mask, llr), "C3 sample")


def test_parity_c5_mask_sample(pkg, cuda, oracle_mod):
    """BASELINE config C5 mask (N=262144): 3 frames vs the oracle."""
    mask = util.mask("frozen_n_262144_k_131072")
    llr, _ = util.synth_frames(mask, 3, ebn0_db=1.0, seed=262144)
    _assert_same(_decode(pkg, cuda, mask, llr), oracle_mod.decode_fsm(mask, llr), "C5 sample")


def test_parity_n524288_mask_sample(pkg, cuda, oracle_mod):
    """The largest reference mask (Generated_Frozen_Bit/frozen_n_524288_k_262144.txt,
    SURVEY.md 5): 2 frames vs the oracle (grid tier + HBM scratch at N = 2^19)."""
    mask = util.mask("frozen_n_524288_k_262144")
    llr, _ = util.synth_frames(mask, 2, ebn0_db=1.0, seed=524288)
    _assert_same(_decode(pkg, cuda, mask, llr), oracle_mod.decode_fsm(mask, llr), "N=524288 sample")


def test_full_size_c2_noiseless_roundtrip(pkg, cuda):
    """At BASELINE C2 size (65536 frames): noiseless LLRs must decode to the sent codeword
    (size-independent encode -> decode round trip)."""
    mask = util.mask("FB_N1024_K512")
    rng = np.random.default_rng(7)
    B = 65536
    u = rng.integers(0, 2, size=(B, mask.size), dtype=np.uint8) & mask[None, :]
    x = util.encode_np(u)
    llr = np.where(x == 1, -31, 31).astype(np.int8)
    for jit in (True, False):
        got = _decode(pkg, cuda, mask, llr, jit)
        assert (got == x).all()
    dec = pkg.Decoder(mask)
    info = dec.codeword_to_info(pkg.pack_bits(got[:64]))
    np.testing.assert_array_equal(info, u[:64][:, mask.astype(bool)])


def test_mask_kernel_equals_interpreter_full_c2(pkg, cuda):
    """The two kernel families agree bit-for-bit on a full C2 batch of AWGN frames."""
    import bench
    mask = util.mask("FB_N1024_K512")
    llr, _ = bench.gen_frames_torch(cuda, mask, 65536, 2.0, 99, cuda.device("cuda"))
    outs = []
    for jit in (True, False):
        dec = make_decoder(pkg, mask, jit)
        outs.append(dec.decode(llr).cpu().numpy())
    cuda.cuda.synchronize()
    assert (outs[0] == outs[1]).all()


@pytest.mark.parametrize("name", ["FB_N1024_K512", "FB_N128_K64"])
def test_misaligned_input_pointer(pkg, cuda, oracle_mod, name):
    """LLR rows handed over at an odd device address (the mask kernel's byte-copy staging)."""
    mask = util.mask(name)
    llr, _ = util.synth_frames(mask, 19, ebn0_db=1.0, seed=4)
    flat = cuda.zeros(llr.size + 16, dtype=cuda.int8, device="cuda")
    view = flat[3:3 + llr.size].view(llr.shape)
    view.copy_(cuda.from_numpy(llr))
    assert view.data_ptr() % 16 == 3
    dec = make_decoder(pkg, mask, True)
    got = pkg.unpack_bits(dec.decode(view).cpu().numpy(), mask.size)
    _assert_same(got, oracle_mod.decode_fsm(mask, llr), "misaligned " + name)


def test_c_cli_decode_file(pkg, cuda, oracle_mod, tmp_path):
    """The plain-C example caller decodes an LLR file through polar_sc_decode_host."""
    import subprocess
    from sc_polar_decoder_hls_amd import _build
    mask = util.mask("frozen_n_1024_k_768")
    tab = tmp_path / "mask.txt"
    tab.write_text(" ".join(str(int(b)) for b in mask))
    llr, _ = util.synth_frames(mask, 29, ebn0_db=2.0, seed=29)
    (tmp_path / "llr.bin").write_bytes(llr.tobytes())
    r = subprocess.run([_build.build_cli(), str(tab), "0", str(tmp_path / "llr.bin"), str(tmp_path / "x.bin")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    words = np.frombuffer((tmp_path / "x.bin").read_bytes(), dtype=np.uint64).reshape(29, -1)
    _assert_same(pkg.unpack_bits(words, mask.size), oracle_mod.decode_fsm(mask, llr), "C CLI")


@pytest.mark.parametrize("wpg", [1, 2, 4, 16])
@pytest.mark.parametrize("name,batch", [("frozen_n_2048_k_1024", 21), ("frozen_n_4096_k_2048", 13),
                                        ("frozen_n_16384_k_8192", 9)])
def test_interpreter_waves_per_group(pkg, cuda, oracle_mod, name, batch, wpg):
    """Schedule interpreter with 1..16 cooperating waves per 8-frame group (split F/G/H/R1
    ops, leaves/REP/SPC on wave 0, barriers between differently split ops)."""
    mask = util.mask(name)
    llr, _ = util.synth_frames(mask, batch, ebn0_db=1.5, seed=wpg)
    dec = make_decoder(pkg, mask, False, waves_per_group=wpg)
    out = dec.decode(cuda.from_numpy(np.ascontiguousarray(llr)).cuda())
    cuda.cuda.synchronize()
    got = pkg.unpack_bits(out.cpu().numpy(), mask.size)
    _assert_same(got, oracle_mod.decode_fsm(mask, llr), "%s wpg=%d" % (name, wpg))


@pytest.mark.parametrize("case", ["c1", "c2_snr", "c2_edge", "c3"])
@pytest.mark.parametrize("jit", [True, False], ids=["maskkernel", "interp"])
def test_gpu_matches_committed_vectors(pkg, cuda, case, jit):
    """GPU decode of the committed regression vectors (tests/golden/decode_vectors.npz)."""
    name, llr, x = util.decode_vectors()[case]
    _assert_same(_decode(pkg, cuda, util.mask(name), llr, jit), x, case)

@pytest.mark.parametrize("name,batch", [("FB_N1024_K512", 40003), ("FB_N256_K128", 60001)])
def test_mask_kernel_large_ragged_batch(pkg, cuda, oracle_mod, name, batch):
    """The per-mask kernel on a batch of several dispatch rounds with a ragged tail: equal to
    the schedule interpreter on every frame, and to the oracle on a sample."""
    mask = util.mask(name)
    llr, _ = util.synth_frames(mask, batch, ebn0_db=1.5, seed=77)
    dev = cuda.from_numpy(llr).cuda()
    ref = make_decoder(pkg, mask, False).decode(dev)
    got = make_decoder(pkg, mask, True).decode(dev)
    cuda.cuda.synchronize()
    g = pkg.unpack_bits(got.cpu().numpy(), mask.size)
    _assert_same(g, pkg.unpack_bits(ref.cpu().numpy(), mask.size), "per-mask vs interpreter " + name)
    idx = np.r_[0:48, batch - 40:batch]
    _assert_same(g[idx], oracle_mod.decode_fsm(mask, llr[idx]), "per-mask vs oracle " + name)
