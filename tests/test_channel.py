"""Frame source and error accounting of the reference testbench:
the C-sim chain (encoder -> BPSK -> xorshift128 x2 -> Box-Muller -> adder -> quantizer) and
sc_error_counter, as a CPU restatement (oracle/polar_channel_oracle.c) and on the GPU
(csrc/polar_sc_channel.hip).

GPU vs CPU tolerance: the chain is float; the GPU uses the device math library for logf /
sinf / cosf, the restatement glibc (as the reference's x86 C-sim). Both follow the same
operation order without contraction, so a quantized LLR may differ only where the
unquantized value lies within an ulp of a quantizer step: the test requires >= 99.99 % of
LLRs identical and every difference to be exactly +-1. Sent codewords and the xorshift
stream states (GF(2) jump-ahead vs sequential stepping) must match exactly."""
import os

import numpy as np
import pytest

import util

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KAT_N = {8: "cw8x4", 512: "cw512x256", 1024: "cw1024x512"}


def kat_rows(N):
    return np.array(util.kat()[KAT_N[N]], dtype=np.uint8)


@pytest.mark.parametrize("N,frame0", [(1024, 0), (1024, 7), (64, 1000), (65536, 3), (32, 123456)])
def test_jump_ahead_states_match_sequential_streams(pkg, oracle_mod, N, frame0):
    st = pkg.csim_states(N, 0xF0, frame0, 3)
    for i in range(3):
        np.testing.assert_array_equal(st[i], oracle_mod.csim_states(N, 0xF0, frame0 + i), err_msg="frame %d" % i)


def test_seed_word_replication(pkg, oracle_mod):
    """xMk = (mask, mask, mask, mask) of the 8-bit seed (sc_xorshift128.h:60-61)."""
    s = oracle_mod.csim_states(32, 0xF0, 0)
    m = 0xF0F0F0F0
    assert list(s) == [0x12311178 & m, 0x65498732 | m, 0xFEDCAA01 ^ m, (0xF489A179 + m) & 0xFFFFFFFF,
                       0x98765432 & m, 0x12345678 | m, 0xFCBADEFF ^ m, (0x12121212 + m) & 0xFFFFFFFF]


def test_restatement_frame_offsets_consistent(oracle_mod):
    sig = 0.75
    llr_all, x_all = oracle_mod.csim_frames(1024, 0xF0, 0, 6, sig, codewords=kat_rows(1024))
    llr_tail, x_tail = oracle_mod.csim_frames(1024, 0xF0, 3, 3, sig, codewords=kat_rows(1024))
    np.testing.assert_array_equal(llr_all[3:], llr_tail)
    np.testing.assert_array_equal(x_all[3:], x_tail)


def test_encoder_cycles_kat_codewords(oracle_mod):
    """sc_encoder.h:91-122: frame f sends cw1024x512[f % 3]; BPSK maps 1 -> -1."""
    cw = kat_rows(1024)
    llr, x = oracle_mod.csim_frames(1024, 0xF0, 0, 5, 0.0, codewords=cw)
    for f in range(5):
        np.testing.assert_array_equal(x[f], cw[f % 3])
        np.testing.assert_array_equal(llr[f], np.where(cw[f % 3] == 1, -4, 4))   # sigma 0: +-1 * beta


def test_quantizer_saturation_and_sigma(pkg, oracle_mod):
    llr, _ = oracle_mod.csim_frames(1024, 0xF0, 0, 4, 20.0)
    assert llr.min() == -31 and llr.max() == 31
    # main.cpp:91-98 prints Sigma = 0.7499 for snr 2.5, R 0.5
    assert abs(pkg.csim_sigma(2.5, 0.5) - 0.7499) < 5e-5


def test_error_counter_semantics(oracle_mod):
    """sc_error_counter.h:68-99: per-frame errors in an sc_uint<10> (mod 1024)."""
    N = 2048
    ref = np.zeros((3, N), dtype=np.uint8)
    hat = ref.copy()
    hat[0, :5] = 1          # 5 errors
    hat[1, :1024] = 1       # 1024 errors: wraps to 0 -> no frame error, 0 bit errors counted
    c = oracle_mod.count_errors(hat, ref)
    assert list(c) == [5, 1, 1029]


def test_glibc_restatement_exhaustive(tmp_path):
    """polar_sc_glibcf.h (the device's logf / sinf / cosf) equals the host glibc bit for bit on
    every float of the frame chain's domain: logf on [0, 1], sinf / cosf on [0, 8]
    (tools/glibcf_check.cpp, about 3.2e9 inputs)."""
    import subprocess
    exe = str(tmp_path / "glibcf_check")
    subprocess.check_call(["g++", "-O2", "-mfma", "-ffp-contract=off", "-std=c++17",
                           os.path.join(ROOT, "tools", "glibcf_check.cpp"), "-o", exe, "-lm"])
    r = subprocess.run([exe, "1"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(" 0 mismatches") == 3, r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("frame0,ebn0", [(0, 2.5), (1000, 2.5), (77777, 0.0), (123, 6.0)])
def test_gpu_chain_matches_restatement(pkg, cuda, oracle_mod, frame0, ebn0):
    """The device frame chain equals the C restatement (glibc logf / sinf / cosf) exactly:
    every LLR and every sent bit."""
    N, B = 1024, 512
    sigma = pkg.csim_sigma(ebn0, 0.5)
    llr, xref = pkg.csim_frames(N, B, sigma, seed=0xF0, frame0=frame0, codewords=kat_rows(N))
    ref_llr, ref_x = oracle_mod.csim_frames(N, 0xF0, frame0, B, sigma, codewords=kat_rows(N))
    np.testing.assert_array_equal(llr.cpu().numpy(), ref_llr)
    np.testing.assert_array_equal(pkg.unpack_bits(xref.cpu().numpy(), N), ref_x)


@pytest.mark.gpu
def test_gpu_chain_frames_decode_and_count(pkg, cuda, oracle_mod):
    """Decoder on the reference chain's own frames (bit-exact vs the oracle on the same LLRs)
    and the device error counter vs the restatement."""
    N, B = 1024, 256
    mask = util.mask("FB_N1024_K512")
    llr, xref = pkg.csim_frames(N, B, pkg.csim_sigma(1.0, 0.5), codewords=kat_rows(N))
    dec = pkg.Decoder(mask)
    xhat = dec.decode(llr)
    counts = pkg.count_errors(xhat, xref, N)
    cuda.cuda.synchronize()
    llr_np = llr.cpu().numpy()
    ref_hat = oracle_mod.decode_fsm(mask, llr_np)
    np.testing.assert_array_equal(pkg.unpack_bits(xhat.cpu().numpy(), N), ref_hat)
    ref_counts = oracle_mod.count_errors(ref_hat, pkg.unpack_bits(xref.cpu().numpy(), N))
    np.testing.assert_array_equal(counts.cpu().numpy().astype(np.uint64), ref_counts)
