#!/usr/bin/env python3
"""Golden fixtures for the frozen-table tooling: run the reference's own Frozen_Bit_Generator
(built from its sources by `make -C oracle ref` into oracle/_ref/fb_generator) on reference
tables and store inputs + outputs under tests/golden/tables/ (data only, no reference source).

Each case directory holds: `cmd.json` (arguments), `input.txt` (the IFile, a reference data
file), `polar_parameters.h` and, for Input = 0, `affect.txt` (the FB_N*_K*.txt it writes).
Run in the build container (needs /root/reference):  python tools/make_table_fixtures.py
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden", "tables")

# (name, N, K, PAR, En, reference input file, Input)
CASES = [
    ("n128_k64_p16_en0_order", 128, 64, 16, 0, "Frozen_Bit_Tab/FB_N1024_K512.txt", 0),
    ("n1024_k512_p16_en1_order", 1024, 512, 16, 1, "Frozen_Bit_Tab/FB_N1024_K512.txt", 0),
    ("n32_k16_p4_en1_order", 32, 16, 4, 1, "Frozen_Bit_Tab/FB_N32_K16.txt", 0),
    ("n256_k100_p64_en0_order", 256, 100, 64, 0, "Frozen_Bit_Tab/FB_N256_K128.txt", 0),
    ("n1024_k768_p64_en0_mask", 1024, 768, 64, 0, "Generated_Frozen_Bit/frozen_n_1024_k_768.txt", 1),
    ("n2048_k1024_p16_en1_mask", 2048, 1024, 16, 1, "Generated_Frozen_Bit/frozen_n_2048_k_1024.txt", 1),
]


def run_reference(fbgen, N, K, P, En, ifile, inp):
    """Run the reference generator in a scratch tree; returns (parameters_h, affect or None)."""
    with tempfile.TemporaryDirectory() as t:
        cwd = os.path.join(t, "a", "b")
        os.makedirs(cwd)
        os.makedirs(os.path.join(t, "Frozen_Bit_Tab"))
        opath = os.path.join(t, "out") + os.sep
        os.makedirs(opath)
        subprocess.run([fbgen, str(N), str(K), str(P), str(En), ifile, str(inp), opath], cwd=cwd, check=True,
                       stdout=subprocess.DEVNULL)
        with open(opath + "polar_parameters.h", "rb") as f:
            hdr = f.read()
        aff = os.path.join(t, "Frozen_Bit_Tab", "FB_N%d_K%d.txt" % (N, K))
        affect = open(aff, "rb").read() if os.path.exists(aff) else None
    return hdr, affect


def main():
    sys.path.insert(0, ROOT)
    from oracle import oracle
    fbgen = oracle.build_ref()
    if not fbgen:
        sys.exit("reference sources not available")
    for name, N, K, P, En, rel, inp in CASES:
        d = os.path.join(OUT, name)
        os.makedirs(d, exist_ok=True)
        src = os.path.join(REF, rel)
        shutil.copyfile(src, os.path.join(d, "input.txt"))
        hdr, affect = run_reference(fbgen, N, K, P, En, src, inp)
        with open(os.path.join(d, "polar_parameters.h"), "wb") as f:
            f.write(hdr)
        if affect is not None:
            with open(os.path.join(d, "affect.txt"), "wb") as f:
                f.write(affect)
        with open(os.path.join(d, "cmd.json"), "w") as f:
            json.dump({"N": N, "K": K, "PAR": P, "En": En, "Input": inp, "source": rel}, f)
        print(name, len(hdr), None if affect is None else len(affect))


if __name__ == "__main__":
    main()
