#!/usr/bin/env python3
"""Generate the committed fixtures from the reference tree (run in the build container only).

The reference (ydelomier/SC_Polar_decoder_HLS) cannot be built or run here, so the only
known-answer data it holds are:
  * the 9 hard-coded codewords of src/testbench/sc_encoder/sc_encoder.h:74-88
    (cw8x4, cw512x256, cw1024x512) -> tests/golden/kat_codewords.json
  * its frozen-bit tables (Frozen_Bit_Tab/FB_N*_K*.txt reliability orders and
    Generated_Frozen_Bit/frozen_n_*_k_*.txt 0/1 masks) -> data/frozen_masks.json,
    stored as derived information-bit masks (bit i of the mask = frozen-table bit i,
    1 = information, packed LSB-first and hex-encoded), with the rule that derived them
    (Frozen_Bit_Generator/src/Writer.h:35-105).

Nothing here is executed at test/bench time; /root/reference does not exist on the GPU box.
"""
import json
import os
import re
import sys

REF = os.environ.get("POLAR_REF", "/root/reference")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse_kat():
    path = os.path.join(REF, "src/testbench/sc_encoder/sc_encoder.h")
    txt = open(path).read()
    out = {}
    for name in ("cw8x4", "cw512x256", "cw1024x512"):
        m = re.search(r"const bool\s+%s\[3\]\[(\d+)\]\s*=\s*\{(.*?)\};" % name, txt, re.S)
        n = int(m.group(1))
        rows = re.findall(r"\{([^{}]*)\}", m.group(2))
        cws = [[int(t) for t in re.findall(r"[01]", r)] for r in rows]
        assert len(cws) == 3 and all(len(c) == n for c in cws), name
        out[name] = cws
    return out


def load_frozen_tab(path, N, K):
    """Writer.h:35-93 (Input=0): line 1 = N, lines 2-3 skipped, line 4 = reliability
    order (most reliable first); keep indices < N; the first K are information bits."""
    lines = open(path).read().splitlines()
    order = [int(t) for t in lines[3].split()]
    order = [v for v in order if v < N]
    mask = [0] * N
    for v in order[:K]:
        mask[v] = 1
    return mask


def load_mask_file(path):
    """Writer.h:95-105 (Input=1): one line of N tokens 0/1, 1 = information bit."""
    return [int(t) for t in open(path).read().split()]


def pack_hex(mask):
    b = bytearray((len(mask) + 7) // 8)
    for i, v in enumerate(mask):
        if v:
            b[i >> 3] |= 1 << (i & 7)
    return b.hex()


TABLES = [
    # (name, kind, relative path, N, K)
    ("FB_N128_K64", "tab", "Frozen_Bit_Tab/FB_N128_K64.txt", 128, 64),
    ("FB_N256_K128", "tab", "Frozen_Bit_Tab/FB_N256_K128.txt", 256, 128),
    ("FB_N512_K256", "tab", "Frozen_Bit_Tab/FB_N512_K256.txt", 512, 256),
    ("FB_N1024_K512", "tab", "Frozen_Bit_Tab/FB_N1024_K512.txt", 1024, 512),
    ("FB_N2048_K1024", "tab", "Frozen_Bit_Tab/FB_N2048_K1024.txt", 2048, 1024),
    ("FB_N8_K4", "tab", "Frozen_Bit_Tab/FB_N8_K4.txt", 8, 4),
    ("frozen_n_1024_k_512", "mask", "Generated_Frozen_Bit/frozen_n_1024_k_512.txt", 1024, 512),
    ("frozen_n_1024_k_768", "mask", "Generated_Frozen_Bit/frozen_n_1024_k_768.txt", 1024, 768),
    # (the N = 1024 code of script_RTL_sim.sh:87-97's PAR 4..64 loop)
    ("frozen_n_1024_k_922", "mask", "Generated_Frozen_Bit/frozen_n_1024_k_922.txt", 1024, 922),
    ("frozen_n_2048_k_1024", "mask", "Generated_Frozen_Bit/frozen_n_2048_k_1024.txt", 2048, 1024),
    ("frozen_n_4096_k_2048", "mask", "Generated_Frozen_Bit/frozen_n_4096_k_2048.txt", 4096, 2048),
    ("frozen_n_8192_k_4096", "mask", "Generated_Frozen_Bit/frozen_n_8192_k_4096.txt", 8192, 4096),
    ("frozen_n_16384_k_8192", "mask", "Generated_Frozen_Bit/frozen_n_16384_k_8192.txt", 16384, 8192),
    ("frozen_n_32768_k_29492", "mask", "Generated_Frozen_Bit/frozen_n_32768_k_29492.txt", 32768, 29492),
    # the rate-0.9 codes of script/script_tests.sh:7-8 (PAR 16 / 64 sweep at QUANT 8)
    ("frozen_n_2048_k_1844", "mask", "Generated_Frozen_Bit/frozen_n_2048_k_1844.txt", 2048, 1844),
    ("frozen_n_4096_k_3686", "mask", "Generated_Frozen_Bit/frozen_n_4096_k_3686.txt", 4096, 3686),
    ("frozen_n_8192_k_7372", "mask", "Generated_Frozen_Bit/frozen_n_8192_k_7372.txt", 8192, 7372),
    ("frozen_n_16384_k_14746", "mask", "Generated_Frozen_Bit/frozen_n_16384_k_14746.txt", 16384, 14746),
    ("frozen_n_65536_k_32768", "mask", "Generated_Frozen_Bit/frozen_n_65536_k_32768.txt", 65536, 32768),
    ("frozen_n_262144_k_131072", "mask", "Generated_Frozen_Bit/frozen_n_262144_k_131072.txt", 262144, 131072),
    # the largest reference masks (N up to 524288)
    ("frozen_n_524288_k_262144", "mask", "Generated_Frozen_Bit/frozen_n_524288_k_262144.txt", 524288, 262144),
]


def main():
    if not os.path.isdir(REF):
        sys.exit("reference tree not found at %s" % REF)
    kat = parse_kat()
    kat_doc = {
        "source": "src/testbench/sc_encoder/sc_encoder.h:74-88 (ydelomier/SC_Polar_decoder_HLS)",
        "note": "codewords x in natural order; cw512x256 is valid for FB_N512_K256, "
                "cw1024x512 for FB_N1024_K512, cw8x4 for FB_N8_K4",
        "codewords": kat,
    }
    os.makedirs(os.path.join(ROOT, "tests/golden"), exist_ok=True)
    with open(os.path.join(ROOT, "tests/golden/kat_codewords.json"), "w") as f:
        json.dump(kat_doc, f)

    masks = {}
    for name, kind, rel, N, K in TABLES:
        p = os.path.join(REF, rel)
        mask = load_frozen_tab(p, N, K) if kind == "tab" else load_mask_file(p)
        assert len(mask) == N and sum(mask) == K, (name, len(mask), sum(mask))
        masks[name] = {"N": N, "K": K, "source": rel, "format": kind, "hex": pack_hex(mask)}
    os.makedirs(os.path.join(ROOT, "data"), exist_ok=True)
    with open(os.path.join(ROOT, "data/frozen_masks.json"), "w") as f:
        json.dump({
            "note": "information-bit masks derived from the reference's frozen tables "
                    "(Frozen_Bit_Generator/src/Writer.h:35-105): bit i (LSB-first hex) = "
                    "frozen-table bit i, 1 = information bit",
            "masks": masks,
        }, f, indent=1)
    print("wrote kat_codewords.json and frozen_masks.json (%d masks)" % len(masks))


if __name__ == "__main__":
    main()
