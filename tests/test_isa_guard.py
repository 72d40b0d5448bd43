"""The launch guard and the round-3 dispatch abort.

Round 3 saw `HSA_STATUS_ERROR_INVALID_ISA` (the queue's register-invalid dispatch error) on a
pair plan with F-descent chains of 4 records built by torch's hipRTC, dispatched as 8-wave
blocks. Established since (tools/rtc_isa_check.py on the committed round-3 source,
tools/isa_dispatch_probe.cpp on an MI355X, profiles/r05_ab/isa_r3_probe.log):
  * torch's hipRTC builds that kernel with 128 VGPRs + 128 AGPRs (accum_offset 128) and 760 B
    of scratch, the ROCm clang driver with 256 VGPRs and 548 B: both are 256 unified
    registers, and both dispatch as 8-wave blocks -- so do the clang object with its scratch
    padded to the aborted dispatch's 812 B and the hipRTC object at 4 waves;
  * neither the AGPR split nor the scratch size decides a dispatch; what an 8-wave block needs
    is ceil(8 / 4) x the unified register allocation (the descriptor's granulated count,
    AGPRs included) <= 512 -- the condition the aborted object broke and the one the launch
    guard (polar_sc_jit.cpp kernel_regs / fit_waves) enforces before every launch.
This CPU test builds a chain-4 plan with both compilers and checks that the descriptor's count
is the unified one (AGPRs included, equal to the metadata's .vgpr_count in granules of 8) and
that the guard's waves-per-block decision equals that condition for every block size."""
import pytest

import util  # noqa: F401  (tests/ on the path)


def _ric():
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import rtc_isa_check
    return rtc_isa_check


def _fits(regs, W):
    return -(-W // 4) * regs <= 512


def test_guard_matches_register_condition_both_compilers(pkg):
    ric = _ric()
    from sc_polar_decoder_hls_amd._plansets import struct_masks
    dec = pkg.Decoder(struct_masks(16384)[0], tuning={"kernel": 3, "layout": 1, "sub_words": 64, "chain_max": 4,
                                                      "sub_root": 1})   # (round 3: roots in a slot level)
    src = dec.kernel_source()
    assert "pop_chain<4" in src
    objs = {"clang": ric.clang_compile(src), "torch_hiprtc": ric.hiprtc_compile(ric.torch_hiprtc(), src)[0]}
    seen_agpr = False
    for comp, co in objs.items():
        kd = ric.kernel_descriptors(co)["polar_sc_pair_kernel"]
        meta = ric.metadata(co)["polar_sc_pair_kernel"]
        regs = kd["regs_unified"]
        # the descriptor's count is the unified VGPR + AGPR allocation
        assert regs == -(-meta["vgpr_count"] // 8) * 8, (comp, kd, meta)
        if meta["agpr_count"]:
            seen_agpr = True
            assert kd["rsrc3_accum_offset"] + meta["agpr_count"] <= regs, (comp, kd, meta)
        for W in (1, 2, 4, 8, 16):
            kept = ric.guard(regs, 64 * W)
            assert _fits(regs, kept) and (kept == W) == _fits(regs, W), (comp, W, regs, kept)
    # the library's guard on its own object of the plan agrees with the same condition
    info = dec.launch_info(9)
    assert _fits(info["regs"], info["waves_per_block"]) and info["compiler"] in (1, 2), info
    assert seen_agpr or pytest.skip("this hipRTC allocated no AGPRs for the plan")
