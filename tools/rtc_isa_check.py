#!/usr/bin/env python3
"""Kernel descriptors of one plan's generated code, built by each compiler the library can use
(CPU only): torch's bundled hipRTC (what a process that imported torch first resolves), the
ROCm hipRTC, and the ROCm clang driver (the library's default when no GPU is open).

This is the investigation of the round-3 dispatch abort: `HSA_STATUS_ERROR_INVALID_ISA` on
tests/test_pair.py::test_pair_parity_structured[32768], whose dispatch was
grid [2560], workgroup [512] (8 waves), private_seg_size 812, group_seg_size 69632 -- the
structured N = 32768 mask with subtrees of 64 words and F-descent chains of up to 4 records,
compiled by torch's hipRTC (the round-3 default). For every kernel of every build it prints
the AMDHSA kernel descriptor (group / private segment size, compute_pgm_rsrc1/2/3 fields,
kernel_code_properties) and the code-object metadata, and the decision of the library's
launch guard (polar_sc_jit.cpp kernel_regs / fit_waves) next to the hardware condition
checked here: the block's waves per SIMD x the unified register allocation <= 512.

    python tools/rtc_isa_check.py [--sub-words 64] [--chain-max 4] [--json out.json]
"""
import argparse
import ctypes
import json
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
CSRC = os.path.join(ROOT, "sc_polar_decoder_hls_amd", "csrc")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
HEADERS = ("polar_sc_device.h", "polar_sc_interp.h", "polar_sc_pair.h")
RTC_OPTS = ("--gpu-architecture=gfx950", "-O3", "-std=c++17")   # polar_sc_jit.cpp kRtcOpts


def torch_hiprtc():
    import importlib.util
    spec = importlib.util.find_spec("torch")
    return os.path.join(os.path.dirname(spec.origin), "lib", "libhiprtc.so")


def hiprtc_compile(lib_path, src, csrc=CSRC):
    """code object of `src` built by the hipRTC library at lib_path (options and embedded
    headers as polar_sc_jit.cpp rtc_compile)"""
    lib = ctypes.CDLL(lib_path)
    prog = ctypes.c_void_p()
    hdr_txt = [open(os.path.join(csrc, h), "rb").read() for h in HEADERS]
    hdrs = (ctypes.c_char_p * 3)(*hdr_txt)
    names = (ctypes.c_char_p * 3)(*[h.encode() for h in HEADERS])
    rc = lib.hiprtcCreateProgram(ctypes.byref(prog), src.encode(), b"polar_sc_mask.hip", 3, hdrs, names)
    assert rc == 0, rc
    opts = (ctypes.c_char_p * len(RTC_OPTS))(*[o.encode() for o in RTC_OPTS])
    rc = lib.hiprtcCompileProgram(prog, len(RTC_OPTS), opts)
    n = ctypes.c_size_t()
    lib.hiprtcGetProgramLogSize(prog, ctypes.byref(n))
    log = ctypes.create_string_buffer(n.value + 1)
    lib.hiprtcGetProgramLog(prog, log)
    if rc != 0:
        raise RuntimeError("hipRTC %s failed (%d): %s" % (lib_path, rc, log.value.decode(errors="replace")[-2000:]))
    lib.hiprtcGetCodeSize(prog, ctypes.byref(n))
    code = ctypes.create_string_buffer(n.value)
    lib.hiprtcGetCode(prog, code)
    ver = (ctypes.c_int(), ctypes.c_int())
    lib.hiprtcVersion(ctypes.byref(ver[0]), ctypes.byref(ver[1]))
    return code.raw, "%d.%d" % (ver[0].value, ver[1].value)


def clang_compile(src, csrc=CSRC):
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "k.hip")
        with open(p, "w") as f:
            f.write("#include <hip/hip_runtime.h>\n" + src)
        co = os.path.join(d, "k.co")
        subprocess.run([CLANG, "-x", "hip", "--offload-arch=gfx950", "--cuda-device-only", "--no-gpu-bundle-output",
                        "-O3", "-std=c++17", "-w", "-I" + csrc, "-c", "-o", co, p], check=True)
        return open(co, "rb").read()


def elf_sections(data):
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
    return secs, shstrndx


def kernel_descriptors(data):
    """{kernel name: descriptor fields} from the <name>.kd symbols (AMDHSA code object v5)"""
    secs, _ = elf_sections(data)
    out = {}
    for s in secs:
        if s[1] != 2:   # SHT_SYMTAB
            continue
        strs = secs[s[6]]
        for o in range(0, s[5], 24):
            name_off, info, other, shndx, value, size = struct.unpack_from("<IBBHQQ", data, s[4] + o)
            nm = data[strs[4] + name_off:].split(b"\0", 1)[0].decode()
            if not nm.endswith(".kd"):
                continue
            sec = secs[shndx]
            off = sec[4] + (value - sec[3])
            kd = data[off:off + 64]
            gseg, pseg, karg = struct.unpack_from("<III", kd, 0)
            rsrc3, rsrc1, rsrc2 = struct.unpack_from("<III", kd, 44)
            props, = struct.unpack_from("<H", kd, 56)
            out[nm[:-3]] = {
                "group_segment_fixed_size": gseg, "private_segment_fixed_size": pseg, "kernarg_size": karg,
                "rsrc1_vgpr_granules": rsrc1 & 63, "regs_unified": ((rsrc1 & 63) + 1) * 8,
                "rsrc1_sgpr_granules": (rsrc1 >> 6) & 15,
                "rsrc2_scratch_en": rsrc2 & 1, "rsrc2_user_sgprs": (rsrc2 >> 1) & 31,
                "rsrc3_accum_offset": ((rsrc3 & 63) + 1) * 4, "rsrc3_tg_split": (rsrc3 >> 16) & 1,
                "props_private_segment_buffer": props & 1, "props_flat_scratch_init": (props >> 5) & 1,
                "props_private_segment_size": (props >> 6) & 1, "props_uses_dynamic_stack": (props >> 11) & 1,
                "rsrc1": "0x%08x" % rsrc1, "rsrc2": "0x%08x" % rsrc2, "rsrc3": "0x%08x" % rsrc3,
            }
    return out


def metadata(data):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(data)
        f.flush()
        notes = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True).stdout
    out = {}
    for blk in re.split(r"\n\s+- \.agpr_count:", notes)[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        get = lambda k: int(re.search(r"\.%s:\s+(\d+)" % k, blk).group(1)) if re.search(r"\.%s:\s+(\d+)" % k, blk) else None
        out[name] = {"agpr_count": int(blk.split()[0]), "vgpr_count": get("vgpr_count"), "sgpr_count": get("sgpr_count"),
                     "private_segment_fixed_size": get("private_segment_fixed_size"),
                     "max_flat_workgroup_size": get("max_flat_workgroup_size"),
                     "uses_dynamic_stack": "uses_dynamic_stack:  true" in blk or ".uses_dynamic_stack: true" in blk}
    return out


def patch_private_size(data, name, new):
    """copy of a code object whose kernel `name` declares `new` bytes of private segment per
    lane (kernel descriptor and metadata note): a larger scratch allocation than the code
    uses, harmless, to test whether the private segment size alone decides a dispatch"""
    kds = kernel_descriptors(data)
    old = kds[name]["private_segment_fixed_size"]
    b = bytearray(data)
    secs, _ = elf_sections(data)
    for s in secs:
        if s[1] != 2:
            continue
        strs = secs[s[6]]
        for o in range(0, s[5], 24):
            name_off, _, _, shndx, value, _ = struct.unpack_from("<IBBHQQ", data, s[4] + o)
            if data[strs[4] + name_off:].split(b"\0", 1)[0].decode() == name + ".kd":
                sec = secs[shndx]
                struct.pack_into("<I", b, sec[4] + (value - sec[3]) + 4, new)
    key = b"\xbb.private_segment_fixed_size"
    i = data.find(key)
    while i >= 0:
        j = i + len(key)
        if data[j] == 0xcd and struct.unpack_from(">H", data, j + 1)[0] == old:
            struct.pack_into(">H", b, j + 1, new)
        i = data.find(key, i + 1)
    return bytes(b)


def guard(regs, wg):
    """polar_sc_jit.cpp fit_waves restated: waves per block the launch keeps (of wg / 64)"""
    W = wg // 64
    if regs > 512:
        return 0
    while W > 1 and ((W + 3) // 4) * regs > 512:
        W //= 2
    return W


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sub-words", type=int, default=64)
    ap.add_argument("--chain-max", type=int, default=4)
    ap.add_argument("--compilers", default="torch_hiprtc,rocm_hiprtc,clang")
    ap.add_argument("--json")
    ap.add_argument("--source", help="a generated source file instead of this tree's plan (e.g. of an older commit)")
    ap.add_argument("--csrc", default=CSRC, help="the device headers that source includes")
    ap.add_argument("--save-co", help="directory: write <compiler>.co (and clang_p<size>.co for --pad-private)")
    ap.add_argument("--pad-private", type=int, default=0, help="also save the clang object declaring this private size")
    args = ap.parse_args()
    if args.source:
        src = open(args.source).read()
        res = {"plan": {"source": args.source, "csrc": args.csrc}}
    else:
        import sc_polar_decoder_hls_amd as pkg
        from sc_polar_decoder_hls_amd._plansets import struct_masks
        dec = pkg.Decoder(struct_masks(32768)[0], tuning={"kernel": 3, "layout": 1, "sub_words": args.sub_words, "sub_root": 1,
                                                          "chain_max": args.chain_max})
        src = dec.kernel_source()
        res = {"plan": {"mask": "struct32768_0", "sub_words": args.sub_words, "chain_max": args.chain_max}}
    for comp in args.compilers.split(","):
        if comp == "clang":
            code, ver = clang_compile(src, args.csrc), "ROCm clang"
        else:
            path = torch_hiprtc() if comp == "torch_hiprtc" else "/opt/rocm/lib/libhiprtc.so"
            code, ver = hiprtc_compile(path, src, args.csrc)
        if args.save_co:
            os.makedirs(args.save_co, exist_ok=True)
            open(os.path.join(args.save_co, comp + ".co"), "wb").write(code)
            if comp == "clang" and args.pad_private:
                padded = patch_private_size(code, "polar_sc_pair_kernel", args.pad_private)
                assert kernel_descriptors(padded)["polar_sc_pair_kernel"]["private_segment_fixed_size"] == args.pad_private
                assert metadata(padded)["polar_sc_pair_kernel"]["private_segment_fixed_size"] == args.pad_private
                open(os.path.join(args.save_co, "clang_p%d.co" % args.pad_private), "wb").write(padded)
        kds, meta = kernel_descriptors(code), metadata(code)
        ks = {}
        for name, kd in kds.items():
            m = meta.get(name, {})
            wg = m.get("max_flat_workgroup_size") or 64
            ks[name] = dict(kd, **{"meta_" + k: v for k, v in m.items()},
                            launch_guard_waves=guard(kd["regs_unified"], wg), block_waves=wg // 64)
        res[comp] = {"version": ver, "kernels": ks}
        k = ks.get("polar_sc_pair_kernel", {})
        print("%-13s %-10s pair kernel: regs %s (accum_offset %s, agpr %s, vgpr_count %s), private %s B, "
              "scratch_en %s, dynamic stack %s, guard W %s of %s" %
              (comp, ver, k.get("regs_unified"), k.get("rsrc3_accum_offset"), k.get("meta_agpr_count"),
               k.get("meta_vgpr_count"), k.get("private_segment_fixed_size"), k.get("rsrc2_scratch_en"),
               k.get("props_uses_dynamic_stack"), k.get("launch_guard_waves"), k.get("block_waves")))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
