"""Frozen_Bit_Generator's command line over the C ABI table writers.

    python -m sc_polar_decoder_hls_amd.fbgen N K P En IFile Input OPath

Same arguments, outputs and quirks as the reference tool (Frozen_Bit_Generator/main.cpp:12-52,
src/Writer.h:21-167):
  * Input = 0: IFile is a reliability order in the Frozen_Bit_Tab format. Entries >= N are
    dropped, the first K remaining are information bits, and the subset order is written to
    ../../Frozen_Bit_Tab/FB_N{N}_K{K}.txt relative to the working directory (the "affect" file).
  * Input = 1: IFile holds N 0/1 tokens on its first line (1 = information bit).
  * Both write OPath + "polar_parameters.h" (OPath is concatenated as given, so it normally
    ends with a path separator). En = 1 writes PAR-wide strings, 0 one sc_bv<1> per bit.
  * A missing IFile prints the reference's error line and exits with status 0.
The plan API consumes the result with Decoder(load_parameters_h(path)[0]).
"""
import os
import sys

import numpy as np

from . import frozen_tab_text, mask_from_order, parameters_h_text


def generate_fb_file(i_filename, nbit, o_filename, kbit, affect_file, par, en, i_file_case):
    """Writer::Generate_FB_File (Writer.h:21-167). Returns False if IFile is missing."""
    if not os.path.exists(i_filename):
        print("!!! ERROR file does not exist : %s !!!" % i_filename)
        return False
    with open(i_filename, "rb") as f:
        lines = f.read().decode("ascii", "replace").split("\n")
    if int(i_file_case) == 0:
        order = np.array([int(t) for t in lines[3].split()], dtype=np.uint32)   # line 4
        with open(affect_file, "w", newline="") as f:
            f.write(frozen_tab_text(order, nbit))
        mask = mask_from_order(order, nbit, kbit)
    else:
        mask = np.array([int(t) for t in lines[0].split()][:nbit], dtype=np.uint8)
        if mask.size != nbit:
            raise ValueError("%s: %d bits, expected %d" % (i_filename, mask.size, nbit))
    with open(o_filename, "w", newline="") as f:
        f.write(parameters_h_text(mask, par=par, concat=bool(int(en))))
    print("fin")
    return True


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    print("(II) USER GUIDE : command N K P En IFile Input OPath")
    if len(argv) < 7:
        return 255   # the reference returns -1
    nbit, kbit, par, en = int(argv[0]), int(argv[1]), int(argv[2]), int(argv[3])
    i_filename, i_case, o_path = argv[4], int(argv[5]), argv[6]
    o_filename = o_path + "polar_parameters.h"
    affect = "../../Frozen_Bit_Tab/FB_N%d_K%d.txt" % (nbit, kbit)
    generate_fb_file(i_filename, nbit, o_filename, kbit, affect, par, en, i_case)
    return 0


if __name__ == "__main__":
    sys.exit(main())
