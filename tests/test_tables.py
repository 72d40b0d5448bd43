"""Frozen-table tooling against the reference's Frozen_Bit_Generator.

* Golden fixtures (tests/golden/tables/, made by tools/make_table_fixtures.py from the
  reference generator's own output): fbgen.generate_fb_file reproduces polar_parameters.h and
  the FB_N*_K*.txt "affect" file byte for byte.
* Live reference (oracle/_ref/fb_generator, built from Frozen_Bit_Generator/main.cpp when the
  reference sources are present; skipped otherwise): a sweep of N, K, PAR, En on random
  orders and masks.
* Round trips: load_parameters_h(parameters_h_text(mask)) == mask, and a plan built from the
  parsed header has the same schedule as one built from the mask.
"""
import json
import os
import subprocess
import tempfile

import numpy as np
import pytest

import sc_polar_decoder_hls_amd as pkg
from sc_polar_decoder_hls_amd import fbgen

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "tables")
ROOT = os.path.dirname(HERE)
FBGEN_REF = os.path.join(ROOT, "oracle", "_ref", "fb_generator")
CASES = sorted(os.listdir(GOLD))


def run_ours(N, K, P, En, ifile, inp):
    with tempfile.TemporaryDirectory() as t:
        aff = os.path.join(t, "affect.txt")
        out = os.path.join(t, "polar_parameters.h")
        assert fbgen.generate_fb_file(ifile, N, out, K, aff, P, En, inp)
        hdr = open(out, "rb").read()
        affect = open(aff, "rb").read() if os.path.exists(aff) else None
    return hdr, affect


def run_ref(N, K, P, En, ifile, inp):
    with tempfile.TemporaryDirectory() as t:
        cwd = os.path.join(t, "a", "b")
        os.makedirs(cwd)
        os.makedirs(os.path.join(t, "Frozen_Bit_Tab"))
        opath = os.path.join(t, "out") + os.sep
        os.makedirs(opath)
        subprocess.run([FBGEN_REF, str(N), str(K), str(P), str(En), ifile, str(inp), opath], cwd=cwd,
                       check=True, stdout=subprocess.DEVNULL)
        hdr = open(opath + "polar_parameters.h", "rb").read()
        aff = os.path.join(t, "Frozen_Bit_Tab", "FB_N%d_K%d.txt" % (N, K))
        affect = open(aff, "rb").read() if os.path.exists(aff) else None
    return hdr, affect


@pytest.mark.parametrize("case", CASES)
def test_golden_generator_output(case):
    d = os.path.join(GOLD, case)
    c = json.load(open(os.path.join(d, "cmd.json")))
    hdr, affect = run_ours(c["N"], c["K"], c["PAR"], c["En"], os.path.join(d, "input.txt"), c["Input"])
    assert hdr == open(os.path.join(d, "polar_parameters.h"), "rb").read()
    if c["Input"] == 0:
        assert affect == open(os.path.join(d, "affect.txt"), "rb").read()
    else:
        assert affect is None


@pytest.mark.parametrize("case", CASES)
def test_golden_header_parses_back(case):
    d = os.path.join(GOLD, case)
    c = json.load(open(os.path.join(d, "cmd.json")))
    mask, par = pkg.load_parameters_h(os.path.join(d, "polar_parameters.h"))
    assert par == c["PAR"] and mask.size == c["N"] and int(mask.sum()) == c["K"]
    if c["Input"] == 1:
        want = np.array(open(os.path.join(d, "input.txt")).read().split()[: c["N"]], dtype=np.uint8)
        assert np.array_equal(mask, want)
    else:
        order = np.array(open(os.path.join(d, "input.txt")).read().split("\n")[3].split(), dtype=np.uint32)
        assert np.array_equal(mask, pkg.mask_from_order(order, c["N"], c["K"]))


def _write_order(path, order, n_header):
    with open(path, "w", newline="") as f:
        f.write("%d\r\n0\r\n0\r\n" % n_header + "    ".join(str(int(v)) for v in order) + "    ")


@pytest.mark.skipif(not os.path.exists(FBGEN_REF), reason="reference generator not built (oracle/_ref)")
@pytest.mark.parametrize("N", [16, 64, 512, 4096, 32768])
def test_live_reference_sweep(N, tmp_path):
    rng = np.random.default_rng(N)
    big = 2 * N if N < 32768 else N        # orders longer than N exercise the < N filter
    order = rng.permutation(big).astype(np.uint32)
    ofile = str(tmp_path / "order.txt")
    _write_order(ofile, order, big)
    mfile = str(tmp_path / "mask.txt")
    mask = (rng.random(N) < 0.5).astype(np.uint8)
    with open(mfile, "w") as f:
        f.write(" ".join(str(int(v)) for v in mask))
    for P in (4, 16, 64):
        if P > N:
            continue
        for En in (0, 1):
            K = int(rng.integers(0, N + 1))
            assert run_ours(N, K, P, En, ofile, 0) == run_ref(N, K, P, En, ofile, 0), (N, K, P, En)
            assert run_ours(N, int(mask.sum()), P, En, mfile, 1) == run_ref(N, int(mask.sum()), P, En, mfile, 1)


@pytest.mark.parametrize("N,P", [(32, 4), (128, 16), (1024, 16), (1024, 64), (65536, 16)])
def test_parameters_h_round_trip(N, P, tmp_path):
    rng = np.random.default_rng(N + P)
    mask = (rng.random(N) < 0.5).astype(np.uint8)
    for concat in (False, True):
        p = tmp_path / ("p%d.h" % concat)
        p.write_text(pkg.parameters_h_text(mask, par=P, concat=concat))
        got, par = pkg.load_parameters_h(str(p))
        assert par == P and np.array_equal(got, mask)


def test_plan_from_parameters_h(tmp_path):
    d = os.path.join(GOLD, "n1024_k512_p16_en1_order")
    mask, _ = pkg.load_parameters_h(os.path.join(d, "polar_parameters.h"))
    ref = pkg.load_frozen_tab(os.path.join(d, "input.txt"), 512)
    assert np.array_equal(mask, ref)
    a, b = pkg.Decoder(mask), pkg.Decoder(ref)
    assert a.schedule() == b.schedule()


def test_table_errors(tmp_path):
    with pytest.raises(pkg.PolarError):
        pkg.mask_from_order(np.arange(10, dtype=np.uint32), 16, 8)          # too few entries < N
    with pytest.raises(pkg.PolarError):
        pkg.mask_from_order(np.array([0, 1, 1, 2], dtype=np.uint32), 4, 2)  # duplicate
    with pytest.raises(pkg.PolarError):
        pkg.parameters_h_text(np.ones(24, dtype=np.uint8))                  # N not a power of two
    bad = tmp_path / "bad.h"
    bad.write_text("#define _NBITS 64\n#define PAR 16\n")
    with pytest.raises(pkg.PolarError):
        pkg.load_parameters_h(str(bad))
    assert not fbgen.generate_fb_file(str(tmp_path / "missing.txt"), 16, str(tmp_path / "o.h"), 8,
                                      str(tmp_path / "a.txt"), 16, 0, 0)
