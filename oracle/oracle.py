"""ctypes binding of the CPU oracle (oracle/polar_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker / timed CPU baseline. The product package
(sc_polar_decoder_hls_amd) never imports this module.
"""
import contextlib
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

# FSM state indices of orc_decode_fsm's state_counts (polar_oracle.c)
STATES = ("INIT", "F", "R", "G", "H", "H0", "F_REP", "G_R1", "G_SPC", "END", "F_R0")

NODE_R0, NODE_R1, NODE_REP, NODE_SPC, NODE_RN = 0x00, 0x0F, 0x02, 0x04, 0x08


def build(force=False):
    """Compile the oracle with its Makefile (gcc); returns the .so path."""
    srcs = [os.path.join(_HERE, f) for f in ("polar_oracle.c", "polar_channel_oracle.c", "Makefile")]
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < max(map(os.path.getmtime, srcs)):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


REF_SRC = "/root/reference"
FBGEN = os.path.join(_HERE, "_ref", "fb_generator")


def build_ref():
    """Compile the reference's Frozen_Bit_Generator into oracle/_ref/ (only where the reference
    sources exist, i.e. in the build container); returns the binary path or None."""
    if os.path.exists(os.path.join(REF_SRC, "Frozen_Bit_Generator", "main.cpp")):
        subprocess.check_call(["make", "-s", "-C", _HERE, "ref", "REF=" + REF_SRC])
    return FBGEN if os.path.exists(FBGEN) else None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        u32, i32, p = ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p
        for name, args in (("orc_qconv_format", (i32, u32)), ("orc_F_sm", (i32, u32, u32)),
                           ("orc_G_sm", (i32, u32, u32, u32)), ("orc_Gext_sm", (i32, u32, u32, u32)),
                           ("orc_full_adder_sm", (i32, u32, u32)), ("orc_full_adder_sat_sm", (i32, u32, u32)),
                           ("orc_leaf16", (p, u32)), ("orc_rep_add_tree16", (p, u32)),
                           ("orc_min_mask16", (p,)), ("orc_classify_group", (u32,))):
            f = getattr(L, name)
            f.argtypes = list(args)
            f.restype = u32 if name != "orc_classify_group" else i32
        L.orc_decode_fsm.argtypes = [i32, p, p, p, i32, p]
        L.orc_decode_fsm.restype = i32
        L.orc_decode_rec.argtypes = [i32, p, p, p, i32]
        L.orc_decode_rec.restype = i32
        L.orc_decode_fsm_cfg.argtypes = [i32, p, p, p, i32, p, p]
        L.orc_decode_fsm_cfg.restype = i32
        L.orc_decode_rec_cfg.argtypes = [i32, p, p, p, i32, p]
        L.orc_decode_rec_cfg.restype = i32
        for name in ("orc_leaf_rep16", "orc_leaf_spc16"):
            getattr(L, name).argtypes = [p, i32]
            getattr(L, name).restype = u32
        L.orc_encode.argtypes = [i32, p, p, i32]
        L.orc_encode.restype = None
        L.orc_set_llr_bits.argtypes = [i32]
        L.orc_set_llr_bits.restype = i32
        L.orc_set_format.argtypes = [i32, i32, i32, i32]
        L.orc_set_format.restype = i32
        L.orc_decode_fsm16.argtypes = [i32, p, p, p, i32, p, p]
        L.orc_decode_fsm16.restype = i32
        L.orc_decode_rec16.argtypes = [i32, p, p, p, i32, p]
        L.orc_decode_rec16.restype = i32
        for name in ("orc_F_ca2", "orc_G_ca2", "orc_Gext_ca2"):
            getattr(L, name).argtypes = [i32, u32, u32] + ([u32] if name != "orc_F_ca2" else [])
            getattr(L, name).restype = u32
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# The reference's pruning sweep (script/script_tests.sh:103-122), in its order:
# (PRUNING_LEVEL, ELAG_R1, ELAG_REP, ELAG_SPC, ELAG_REP2, ELAG_SPC2, ELAG_H0)
SWEEP_CONFIGS = (
    (0, 0, 0, 0, 0, 0, 0), (1, 0, 0, 0, 0, 0, 0), (1, 1, 0, 0, 0, 0, 0), (1, 1, 1, 0, 0, 0, 0),
    (1, 1, 1, 1, 0, 0, 0), (1, 1, 1, 1, 1, 0, 0), (1, 1, 1, 1, 1, 1, 0), (2, 0, 0, 0, 0, 0, 1),
    (2, 1, 0, 0, 0, 0, 1), (2, 1, 1, 0, 0, 0, 1), (2, 1, 1, 1, 0, 0, 1),
)
DEFAULT_CONFIG = (2, 1, 1, 1, 0, 0, 1)


def _cfg(config):
    if config is None:
        return None
    c = np.ascontiguousarray(config, dtype=np.int32)
    assert c.shape == (7,)
    return c


@contextlib.contextmanager
def _format(llr_bits=6, par=16, sigmag=1, extended=1):
    """Datapath of the restatement for the calling thread: LLR_BITS (config.h:2), PAR
    (polar_parameters.h:8), SIGMAG / CA2 (config.h:11) and EXTENDED (config.h:14); the
    defaults are the shipped configuration."""
    if lib().orc_set_format(int(llr_bits), int(par), 0 if sigmag else 1, 1 if extended else 0) != 0:
        raise ValueError("bad format: llr_bits %r (5..9), par %r (2..64, power of two)" % (llr_bits, par))
    try:
        yield
    finally:
        lib().orc_set_format(6, 16, 0, 1)


def _llr_bits(q):
    return _format(q)


def _llr_array(llr, llr_bits):
    """int8 frames (llr_bits <= 8) or int16 frames (any llr_bits; the only form for 9)."""
    a = np.atleast_2d(np.asarray(llr))
    if a.dtype == np.int16 or llr_bits > 8:
        return np.ascontiguousarray(a, dtype=np.int16), True
    return np.ascontiguousarray(a, dtype=np.int8), False


def decode_fsm(mask, llr, return_counts=False, config=None, llr_bits=6, par=16, sigmag=1, extended=1):
    """Literal FSM decode. mask: (N,) 0/1; llr: (B, N) int8 (or int16). Returns xhat (B, N)
    uint8. config: 7-tuple (see SWEEP_CONFIGS) or None for the shipped config.h; llr_bits:
    LLR_BITS (5..9, the low llr_bits of each input are the LLR); par / sigmag / extended: the
    datapath (see _format)."""
    mask = np.ascontiguousarray(mask, dtype=np.uint8)
    llr, wide = _llr_array(llr, llr_bits)
    B, N = llr.shape
    out = np.zeros((B, N), dtype=np.uint8)
    counts = np.zeros(len(STATES), dtype=np.int64)
    c = _cfg(config)
    fn = lib().orc_decode_fsm16 if wide else lib().orc_decode_fsm_cfg
    with _format(llr_bits, par, sigmag, extended):
        rc = fn(N, _ptr(mask), _ptr(llr), _ptr(out), B, _ptr(counts), None if c is None else _ptr(c))
    if rc != 0:
        raise RuntimeError("orc_decode_fsm failed: %d" % rc)
    if return_counts:
        return out, dict(zip(STATES, counts.tolist()))
    return out


def decode_rec(mask, llr, config=None, llr_bits=6, par=16, sigmag=1, extended=1):
    """Recursive-restatement decode (same I/O as decode_fsm)."""
    mask = np.ascontiguousarray(mask, dtype=np.uint8)
    llr, wide = _llr_array(llr, llr_bits)
    B, N = llr.shape
    out = np.zeros((B, N), dtype=np.uint8)
    c = _cfg(config)
    fn = lib().orc_decode_rec16 if wide else lib().orc_decode_rec_cfg
    with _format(llr_bits, par, sigmag, extended):
        rc = fn(N, _ptr(mask), _ptr(llr), _ptr(out), B, None if c is None else _ptr(c))
    if rc != 0:
        raise RuntimeError("orc_decode_rec failed: %d" % rc)
    return out


def leaf_rep16(word, sel=0):
    """REP_REP2_16_SM on 16 six-bit SM patterns -> 16-bit x."""
    w = np.ascontiguousarray(word, dtype=np.uint32)
    return int(lib().orc_leaf_rep16(_ptr(w), sel))


def leaf_spc16(word, sel=0):
    """SPC_SPC2_Node_16 (SM) on 16 six-bit SM patterns -> 16-bit x."""
    w = np.ascontiguousarray(word, dtype=np.uint32)
    return int(lib().orc_leaf_spc16(_ptr(w), sel))


def encode(u):
    """x = u F^{(x)n}, natural order. u: (B, N) 0/1."""
    u = np.ascontiguousarray(np.atleast_2d(u), dtype=np.uint8)
    B, N = u.shape
    x = np.zeros_like(u)
    lib().orc_encode(N, _ptr(u), _ptr(x), B)
    return x


def leaf16(llr_sm, fb):
    a = np.ascontiguousarray(llr_sm, dtype=np.uint32)
    return lib().orc_leaf16(_ptr(a), fb)


def rep_add_tree16(llr_sm, old):
    a = np.ascontiguousarray(llr_sm, dtype=np.uint32)
    return lib().orc_rep_add_tree16(_ptr(a), old)


def min_mask16(llr_sm):
    a = np.ascontiguousarray(llr_sm, dtype=np.uint32)
    return lib().orc_min_mask16(_ptr(a))


def csim_states(N, seed, frame0):
    """xorshift128 states (2 streams x 4 words) at the start of frame `frame0`."""
    out = np.zeros(8, dtype=np.uint32)
    lib().orc_csim_states(ctypes.c_uint32(N), ctypes.c_uint32(seed), ctypes.c_uint64(frame0), _ptr(out))
    return out


def csim_frames(N, seed, frame0, nframes, sigma, codewords=None, beta=4, vsatn=-31, vsatp=31):
    """Reference C-sim chain frames (polar_channel_oracle.c): (llr int8 [n, N], x uint8 [n, N])."""
    llr = np.zeros((nframes, N), dtype=np.int8)
    x = np.zeros((nframes, N), dtype=np.uint8)
    cw = None if codewords is None else np.ascontiguousarray(codewords, dtype=np.uint8)
    lib().orc_csim_frames(ctypes.c_uint32(N), ctypes.c_uint32(seed), ctypes.c_uint64(frame0), ctypes.c_int(nframes),
                          ctypes.c_float(sigma), ctypes.c_int(beta), ctypes.c_int(vsatn), ctypes.c_int(vsatp),
                          None if cw is None else _ptr(cw), ctypes.c_int(0 if cw is None else cw.shape[0]),
                          _ptr(llr), _ptr(x))
    return llr, x


def count_errors(xhat, xref):
    """sc_error_counter semantics: [sum of per-frame errors mod 1024, frame errors, exact bit errors]."""
    xhat = np.ascontiguousarray(xhat, dtype=np.uint8)
    xref = np.ascontiguousarray(xref, dtype=np.uint8)
    counts = np.zeros(3, dtype=np.uint64)
    lib().orc_count_errors(ctypes.c_uint32(xhat.shape[1]), ctypes.c_int(xhat.shape[0]), _ptr(xhat), _ptr(xref),
                           _ptr(counts))
    return counts
