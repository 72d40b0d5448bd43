"""C ABI boundary (include/polar_sc.h) without a GPU: the library loads, exports every
declared symbol, validates its arguments, and reads the reference's table formats."""
import ctypes
import os
import re

import numpy as np
import pytest

import util

HEADER = os.path.join(util.ROOT, "include", "polar_sc.h")


def declared_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|const char \*)\s*(polar_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_declared_symbol(pkg):
    lib = pkg.lib()
    decl = declared_functions()
    assert len(decl) >= 15
    missing = [f for f in decl if not hasattr(lib, f)]
    assert not missing, missing
    assert set(decl) == set(pkg.EXPORTS)
    assert lib.polar_sc_abi_version() == 5


def test_no_oracle_in_product():
    """The product library and package never reference the oracle (test infrastructure)."""
    pkgdir = os.path.join(util.ROOT, "sc_polar_decoder_hls_amd")
    for root, _, files in os.walk(pkgdir):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                assert "oracle" not in open(os.path.join(root, f)).read().lower(), f


def test_tuning_validation_and_no_environment(pkg, monkeypatch):
    """polar_sc_tuning: out-of-range fields -> -EINVAL; the plan (and its generated kernel
    source) depends on the mask, config and tuning only, never on the environment."""
    m = util.mask("FB_N1024_K512")
    for bad in ({"kernel": 4}, {"waves_per_group": 3}, {"waves_per_group": 32}, {"sub_words": 1024},
                {"tier_words": -2}, {"tier_words": 1000}, {"lds_slots": 300}, {"hybrid_waves": 16},
                {"chain_max": 5}, {"chain_max": -1}, {"sub_inline": 3}, {"sub_inline": -1}, {"layout": 3},
                {"layout": -1}, {"sub_root": 3}, {"sub_root": -1}):
        with pytest.raises(pkg.PolarError) as e:
            pkg.Decoder(m, tuning=bad)
        assert e.value.rc == -22, bad
    # a layout only pair plans have (N >= 2048), and solo only at PAR 16: -ENOTSUP
    with pytest.raises(pkg.PolarError) as e:
        pkg.Decoder(m, tuning={"layout": 2})
    assert e.value.rc == -95
    c64 = pkg.default_config()
    c64.par = 64
    with pytest.raises(pkg.PolarError) as e:
        pkg.Decoder(util.mask("frozen_n_16384_k_8192"), config=c64, tuning={"layout": 2})
    assert e.value.rc == -95
    # 9-bit LLRs: the pair kernel with 16-bit stage slots (both layouts since round 6)
    c9 = pkg.default_config()
    c9.llr_bits = 9
    d9 = pkg.Decoder(util.mask("frozen_n_16384_k_8192"), config=c9)
    assert d9.stats["kernel"] == 3 and "#define POLAR_Q 9" in d9.kernel_source()
    assert d9.stats["scratch_bytes_per_wave"] == (1024 - 256) // 4 * 256 + 1024 // 64 * 256   # 256 B slot rows
    assert pkg.Decoder(util.mask("FB_N1024_K512"), config=c9).stats["kernel"] != 1   # (per-mask: LLR_BITS <= 8)
    assert pkg.Decoder(util.mask("frozen_n_16384_k_8192"), config=c9, tuning={"layout": 2}).stats["kernel"] == 3
    # CA2: no solo layout (the half ops of 8-word nodes have no CA2 form)
    ca2 = pkg.default_config()
    ca2.sigmag = 0
    with pytest.raises(pkg.PolarError) as e:
        pkg.Decoder(util.mask("frozen_n_16384_k_8192"), config=ca2, tuning={"layout": 2})
    assert e.value.rc == -95
    with pytest.raises(KeyError):
        pkg.make_tuning({"wpg": 1})
    src = pkg.Decoder(m).kernel_source()
    big = util.mask("frozen_n_65536_k_32768")
    st = pkg.Decoder(big).stats
    for k in ("POLAR_SC_JIT", "POLAR_SC_MASK_PERSIST", "POLAR_SC_MASK_DUAL", "POLAR_SC_MASK_WPB",
              "POLAR_SC_MASK_MIN_WAVES", "POLAR_SC_ROOT_RESPLIT", "POLAR_SC_ROOT_PACK", "POLAR_SC_SUB_WORDS",
              "POLAR_SC_TIER_WORDS", "POLAR_SC_LDS_SLOTS", "POLAR_SC_HYBRID_WAVES", "POLAR_SC_WAVES_PER_GROUP",
              "POLAR_SC_RTC_EXTRA"):
        monkeypatch.setenv(k, "0" if k in ("POLAR_SC_JIT", "POLAR_SC_ROOT_PACK") else "1")
    assert pkg.Decoder(m).kernel_source() == src
    assert pkg.Decoder(big).stats == st
    assert pkg.Decoder(m, tuning={"kernel": "interp"}).stats["kernel"] == 0
    txt = open(os.path.join(util.ROOT, "sc_polar_decoder_hls_amd", "csrc", "polar_sc_host.cpp")).read()
    assert re.findall(r'getenv\("(\w+)"\)', txt) == ["POLAR_SC_VERBOSE"]   # error detail on stderr only
    txt = open(os.path.join(util.ROOT, "sc_polar_decoder_hls_amd", "csrc", "polar_sc_jit.cpp")).read()
    # the cache directory, extra clang flags for compiler A/Bs (part of the cache key, so the
    # machine code -- and polar_sc_plan_launch_info's code_key -- says which flags built it), and
    # the time a child compile may take before hipRTC builds the kernel instead
    assert sorted(re.findall(r'getenv\("(\w+)"\)', txt)) == ["POLAR_SC_CLANG_FLAGS", "POLAR_SC_CLANG_TIMEOUT",
                                                              "POLAR_SC_RTC_CACHE"]


def test_default_config_is_reference(pkg):
    c = pkg.default_config()
    assert (c.llr_bits, c.par, c.sigmag, c.extended, c.pruning_level) == (6, 16, 1, 1, 2)
    assert (c.elag_r1, c.elag_rep, c.elag_spc, c.elag_rep2, c.elag_spc2, c.elag_rare, c.elag_h0) == (1, 1, 1, 0, 0, 0, 1)


def test_plan_argument_validation(pkg):
    for N in (0, 16, 48, 1000, 3 << 20):
        with pytest.raises(pkg.PolarError) as e:
            pkg.Decoder(np.ones(N, np.uint8))
        assert e.value.rc == -22
    c = pkg.default_config()
    c.llr_bits = 10
    with pytest.raises(pkg.PolarError) as e:
        pkg.Decoder(np.ones(64, np.uint8), c)
    assert e.value.rc == -95
    lib = pkg.lib()
    assert lib.polar_sc_plan_create(None, 64, None, None) == -22
    assert lib.polar_sc_decode(None, None, None, 1, None) == -22
    assert lib.polar_sc_plan_destroy(None) == -22


def test_plan_stats_and_storage(pkg):
    s = pkg.Decoder(util.mask("FB_N1024_K512")).stats
    assert (s["N"], s["K"], s["groups"]) == (1024, 512, 64)
    assert s["op_count"]["END"] == 1 and s["n_ops"] == sum(s["op_count"].values())
    big = pkg.Decoder(util.mask("frozen_n_65536_k_32768")).stats
    assert big["storage"] == 1 and big["scratch_bytes_per_wave"] > 0


def test_load_mask_file_roundtrip(pkg, tmp_path):
    for name in ("frozen_n_1024_k_512", "frozen_n_4096_k_2048"):
        mask = util.mask(name)
        p = tmp_path / (name + ".txt")
        p.write_text(" ".join(str(int(b)) for b in mask))     # Generated_Frozen_Bit format
        np.testing.assert_array_equal(pkg.load_mask_file(str(p)), mask)


def test_load_frozen_tab_semantics(pkg, tmp_path):
    rng = np.random.default_rng(1)
    order = rng.permutation(256)
    p = tmp_path / "FB_N256_K100.txt"
    p.write_text("256\r\n0\r\n0\r\n" + "    ".join(str(v) for v in order) + "    ")
    mask = pkg.load_frozen_tab(str(p), K=100)
    exp = np.zeros(256, np.uint8)
    exp[order[:100]] = 1
    np.testing.assert_array_equal(mask, exp)
    # a larger table used for a smaller N keeps only indices < N (Writer.h:61-69)
    m128 = pkg.load_frozen_tab(str(p), K=40, N=128)
    sub = [v for v in order if v < 128][:40]
    exp = np.zeros(128, np.uint8)
    exp[sub] = 1
    np.testing.assert_array_equal(m128, exp)


def test_loader_errors(pkg, tmp_path):
    with pytest.raises(pkg.PolarError) as e:
        pkg.load_mask_file(str(tmp_path / "missing.txt"))
    assert e.value.rc == -2
    bad = tmp_path / "bad.txt"
    bad.write_text("0 1 2 1")
    with pytest.raises(pkg.PolarError):
        pkg.load_mask_file(str(bad))


@pytest.mark.skipif(not os.path.isdir("/root/reference/Frozen_Bit_Tab"), reason="reference tree absent")
def test_loaders_on_reference_tables(pkg):
    masks = util.masks()
    for name, m in masks.items():
        path = os.path.join("/root/reference", m["source"])
        got = pkg.load_frozen_tab(path, K=m["K"], N=m["N"]) if m["format"] == "tab" else pkg.load_mask_file(path)
        np.testing.assert_array_equal(got, util.mask(name), err_msg=name)


def test_codeword_to_info_host(pkg):
    mask = util.mask("FB_N1024_K512")
    rng = np.random.default_rng(2)
    u = rng.integers(0, 2, size=(5, 1024), dtype=np.uint8) & mask[None, :]
    x = util.encode_np(u)
    dec = pkg.Decoder(mask)
    np.testing.assert_array_equal(dec.codeword_to_info(pkg.pack_bits(x)), u[:, mask.astype(bool)])


def test_pack_unpack_bits(pkg):
    rng = np.random.default_rng(3)
    for N in (32, 64, 1024, 100):
        b = rng.integers(0, 2, size=(3, N)).astype(np.uint8)
        np.testing.assert_array_equal(pkg.unpack_bits(pkg.pack_bits(b), N), b)


def _cli(pkg):
    from sc_polar_decoder_hls_amd import _build
    pkg.build()
    return _build.build_cli()


def test_c_cli_stats_generated_mask_format(pkg, tmp_path):
    """examples/polar_decode_cli.c: plain C through include/polar_sc.h, Generated_Frozen_Bit
    format (space-separated 0/1 tokens), plan census matches the Python binding."""
    import subprocess
    import util
    mask = util.mask("frozen_n_1024_k_512")
    p = tmp_path / "frozen_n_1024_k_512.txt"
    p.write_text(" ".join(str(int(b)) for b in mask))
    r = subprocess.run([_cli(pkg), str(p), "0", "--stats"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    st = pkg.Decoder(mask).stats
    assert ("N=1024 K=512 groups=64 R0=%d R1=%d REP=%d SPC=%d RN=%d" %
            (st["n_r0"], st["n_r1"], st["n_rep"], st["n_spc"], st["n_rn"])) in r.stdout


def test_decode_entry_points_reject_bad_tensors(pkg):
    """decode / decode_u16 / trace validate device, dtype, shape and contiguity before any
    pointer reaches the C ABI (a CPU tensor or a short row would fault the GPU)."""
    import torch
    import util
    dec = pkg.Decoder(util.mask("FB_N128_K64"))
    cpu = torch.zeros((4, 128), dtype=torch.int8)
    for fn in (dec.decode, dec.decode_u16, dec.trace):
        with pytest.raises(TypeError):
            fn(cpu)                                   # host tensor
        with pytest.raises(TypeError):
            fn(np.zeros((4, 128), np.int8))           # not a tensor at all
    with pytest.raises(TypeError):
        dec.decode(torch.zeros((4, 128), dtype=torch.int16))
    assert dec._check_out is not None
    # out-tensor checks (device-independent part)
    with pytest.raises(ValueError):
        pkg.Decoder._check_out(torch.zeros((4, 3), dtype=torch.int64), cpu, (4, 2), torch.int64)
    with pytest.raises(ValueError):
        pkg.Decoder._check_out(torch.zeros((4, 8), dtype=torch.int64), cpu, (4, 8), torch.int16)
    with pytest.raises(ValueError):
        pkg.Decoder._check_out(torch.zeros((8, 4), dtype=torch.int16).t(), cpu, (4, 8), torch.int16)
