"""sc_polar_decoder_hls_amd -- MI355X-native batched SC polar decoder.

Host-side mirror of the reference decoder's interface (ydelomier/SC_Polar_decoder_HLS,
SC_MODULE my_module, src/module/my_module.h:15-36, fed by wrapper_in/wrapper_out):

  * the frozen-bit table goes in once (the `FB` port, read by do_prunning,
    my_module.h:61-166)           -> Decoder(info_mask) / Decoder.load_frozen_bits()
  * frames of 6-bit two's-complement LLRs go in (`e` port via wrapper_in.h:26-44) and the
    estimated codeword x^ comes out (`s` port via wrapper_out.h:26-36)
                                  -> Decoder.decode(llr) -> hard bits

Everything above is a thin ctypes layer over the C ABI of libpolar_sc.so
(include/polar_sc.h); the decode itself runs only as HIP kernels on gfx950. There is no CPU
fallback: if the library is missing or no GPU is visible, decode raises.
"""
import ctypes
import os

import numpy as np

from . import _build

__all__ = [
    "Decoder", "PolarError", "load_frozen_tab", "load_mask_file", "unpack_bits", "pack_bits",
    "default_config", "make_tuning", "lib", "selftest_lanes", "OPS", "build", "csim_sigma", "csim_states", "csim_frames",
    "count_errors",
]

build = _build.build

OPS = {1: "F", 2: "G", 3: "FLEAF", 4: "GLEAF", 5: "REP", 6: "R1", 7: "SPC", 8: "H", 9: "H0", 10: "END", 14: "PLEAF"}
# device-only records of polar_sc_trace (include/polar_sc.h)
TRACE_OPS = {**OPS, 11: "WOPEN", 12: "WFLUSH", 13: "SUB"}

_ERRNO = {22: "EINVAL", 12: "ENOMEM", 95: "ENOTSUP", 2: "ENOENT", 5: "EIO"}


class PolarError(RuntimeError):
    def __init__(self, fn, rc):
        msg = "%s failed: %d (%s)" % (fn, rc, _ERRNO.get(-rc, "?"))
        try:
            msg += " - " + lib().polar_sc_strerror(rc).decode()
        except Exception:
            pass
        super().__init__(msg)
        self.rc = rc


class polar_sc_config(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "llr_bits", "par", "sigmag", "extended", "pruning_level", "elag_r1", "elag_rep",
        "elag_spc", "elag_rep2", "elag_spc2", "elag_rare", "elag_h0", "strict_llr")]


class polar_sc_tuning(ctypes.Structure):
    """Kernel selection / launch shape of a plan (include/polar_sc.h); all 0 = automatic."""
    _fields_ = [(n, ctypes.c_int32) for n in (
        "kernel", "waves_per_group", "sub_words", "tier_words", "lds_slots", "hybrid_waves", "chain_max",
        "sub_inline", "layout", "sub_root")]


def make_tuning(tuning):
    """dict (field -> int; kernel may be "auto" / "interp") or polar_sc_tuning or None."""
    if tuning is None or isinstance(tuning, polar_sc_tuning):
        return tuning
    t = polar_sc_tuning()
    for k, v in dict(tuning).items():
        if k == "kernel" and isinstance(v, str):
            v = {"auto": 0, "interp": 1}[v]
        if k not in [f for f, _ in polar_sc_tuning._fields_]:
            raise KeyError("unknown tuning field %r" % k)
        setattr(t, k, int(v))
    return t


class polar_sc_op(ctypes.Structure):
    _fields_ = [("code", ctypes.c_int32), ("level", ctypes.c_int32), ("n", ctypes.c_int32),
                ("pos", ctypes.c_int32), ("upos", ctypes.c_int32), ("fb", ctypes.c_uint32),
                ("reserved", ctypes.c_int32 * 2)]


class polar_sc_trace_rec(ctypes.Structure):
    _fields_ = [("code", ctypes.c_int32), ("level", ctypes.c_int32), ("n", ctypes.c_int32),
                ("pos", ctypes.c_int32), ("cycles", ctypes.c_uint64)]


class polar_sc_plan_stats(ctypes.Structure):
    _fields_ = [("N", ctypes.c_uint32), ("K", ctypes.c_uint32), ("groups", ctypes.c_uint32),
                ("n_r0", ctypes.c_uint32), ("n_r1", ctypes.c_uint32), ("n_rep", ctypes.c_uint32),
                ("n_spc", ctypes.c_uint32), ("n_rn", ctypes.c_uint32), ("n_ops", ctypes.c_uint32),
                ("op_count", ctypes.c_uint32 * 16), ("word_ops", ctypes.c_uint64),
                ("storage", ctypes.c_uint32), ("lds_bytes_per_wave", ctypes.c_uint32),
                ("scratch_bytes_per_wave", ctypes.c_uint64), ("kernel", ctypes.c_uint32),
                ("sub_words", ctypes.c_uint32), ("n_sub_kinds", ctypes.c_uint32), ("n_sub_calls", ctypes.c_uint32),
                ("tier_steps", ctypes.c_uint32), ("tier_words", ctypes.c_uint32)]


class polar_sc_launch_info(ctypes.Structure):
    _fields_ = [("kernel", ctypes.c_uint32), ("regs", ctypes.c_uint32), ("regs_seg", ctypes.c_uint32),
                ("waves_per_block", ctypes.c_uint32), ("blocks", ctypes.c_uint64), ("lds_bytes", ctypes.c_uint32),
                ("lds_row0", ctypes.c_uint32), ("code_key", ctypes.c_uint64), ("layout", ctypes.c_uint32),
                ("sub_words", ctypes.c_uint32), ("compiler", ctypes.c_uint32), ("alt_layout", ctypes.c_uint32),
                ("alt_max_batch", ctypes.c_uint64)]


# exported symbols of include/polar_sc.h (tests check that the library exports all of them)
EXPORTS = (
    "polar_sc_default_config", "polar_sc_plan_create", "polar_sc_plan_create_tuned", "polar_sc_plan_destroy",
    "polar_sc_decode",
    "polar_sc_decode_u16", "polar_sc_plan_prepare", "polar_sc_decode_host", "polar_load_frozen_tab",
    "polar_load_mask_file", "polar_codeword_to_info", "polar_sc_plan_get_stats",
    "polar_sc_plan_get_schedule", "polar_sc_selftest_lanes", "polar_sc_strerror",
    "polar_sc_abi_version", "polar_sc_plan_compile", "polar_sc_plan_kernel_source",
    "polar_csim_frames", "polar_csim_states", "polar_count_errors",
    "polar_mask_from_order", "polar_write_frozen_tab", "polar_write_parameters_h", "polar_parse_parameters_h",
    "polar_sc_trace", "polar_sc_decode_i16", "polar_sc_debug_subtree", "polar_sc_plan_launch_info",
)

_lib = None


def lib():
    """Load libpolar_sc.so (built in-tree by build()). Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_build.LIB):
        raise RuntimeError("libpolar_sc.so is not built (%s); run sc_polar_decoder_hls_amd.build() "
                           "or __graft_entry__.build()" % _build.LIB)
    # torch first: its bundled HIP runtime is then the one the library binds to (loaded the
    # other way round, the process would hold two HIP runtimes and the library would see no
    # device once torch initialises its own)
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(_build.LIB)
    p, sz, u32, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int
    sig = {
        "polar_sc_default_config": [p],
        "polar_sc_plan_create": [ctypes.POINTER(p), u32, p, p],
        "polar_sc_plan_create_tuned": [ctypes.POINTER(p), u32, p, p, p],
        "polar_sc_plan_destroy": [p],
        "polar_sc_decode": [p, p, p, sz, p],
        "polar_sc_decode_u16": [p, p, p, sz, p],
        "polar_sc_decode_i16": [p, p, p, sz, p],
        "polar_sc_plan_prepare": [p, sz],
        "polar_sc_decode_host": [p, p, p, sz],
        "polar_load_frozen_tab": [ctypes.c_char_p, u32, u32, p, u32, ctypes.POINTER(u32)],
        "polar_load_mask_file": [ctypes.c_char_p, p, u32, ctypes.POINTER(u32)],
        "polar_codeword_to_info": [p, p, p, sz],
        "polar_sc_plan_get_stats": [p, p],
        "polar_sc_plan_get_schedule": [p, p, u32, ctypes.POINTER(u32)],
        "polar_sc_selftest_lanes": [p],
        "polar_sc_debug_subtree": [p, u32, p, p],
        "polar_sc_plan_compile": [p],
        "polar_sc_plan_launch_info": [p, sz, u32, p],
        "polar_sc_plan_kernel_source": [p, ctypes.c_char_p, sz, ctypes.POINTER(sz)],
        "polar_sc_strerror": [i32],
        "polar_sc_abi_version": [],
        "polar_csim_frames": [u32, u32, ctypes.c_uint64, sz, ctypes.c_float, i32, i32, i32, p, u32, p, p, p],
        "polar_csim_states": [u32, u32, ctypes.c_uint64, sz, p],
        "polar_count_errors": [p, p, u32, sz, p, p],
        "polar_mask_from_order": [p, u32, u32, u32, p, u32],
        "polar_sc_trace": [p, p, p, sz, p, u32, ctypes.POINTER(u32), ctypes.POINTER(ctypes.c_double),
                           ctypes.POINTER(ctypes.c_uint64)],
        "polar_write_frozen_tab": [p, u32, u32, ctypes.c_char_p, sz, ctypes.POINTER(sz)],
        "polar_write_parameters_h": [p, u32, u32, i32, ctypes.c_char_p, sz, ctypes.POINTER(sz)],
        "polar_parse_parameters_h": [ctypes.c_char_p, p, u32, ctypes.POINTER(u32), ctypes.POINTER(u32)],
    }
    for name, args in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = ctypes.c_char_p if name == "polar_sc_strerror" else i32
    _lib = L
    return L


def _check(fn, rc):
    if rc != 0:
        raise PolarError(fn, rc)


def default_config():
    c = polar_sc_config()
    _check("polar_sc_default_config", lib().polar_sc_default_config(ctypes.byref(c)))
    return c


def _np_ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def load_frozen_tab(path, K, N=0):
    """Frozen_Bit_Tab/FB_N*_K*.txt -> information mask (uint8, 1 = info). Writer.h:35-93."""
    cap = 1 << 21
    buf = np.zeros(cap, dtype=np.uint8)
    n = ctypes.c_uint32(0)
    _check("polar_load_frozen_tab",
           lib().polar_load_frozen_tab(os.fsencode(path), N, K, _np_ptr(buf), cap, ctypes.byref(n)))
    return buf[:n.value].copy()


def load_mask_file(path):
    """Generated_Frozen_Bit/frozen_n_*_k_*.txt -> information mask. Writer.h:95-105."""
    cap = 1 << 21
    buf = np.zeros(cap, dtype=np.uint8)
    n = ctypes.c_uint32(0)
    _check("polar_load_mask_file",
           lib().polar_load_mask_file(os.fsencode(path), _np_ptr(buf), cap, ctypes.byref(n)))
    return buf[:n.value].copy()


def _text_call(name, *args):
    n = ctypes.c_size_t(0)
    _check(name, getattr(lib(), name)(*args, None, 0, ctypes.byref(n)))
    buf = ctypes.create_string_buffer(n.value + 1)
    _check(name, getattr(lib(), name)(*args, buf, n.value + 1, ctypes.byref(n)))
    return buf.raw[:n.value].decode("ascii")


def mask_from_order(order, N, K):
    """Reliability order (most reliable first) -> information mask of N bits, K info bits.
    Entries >= N are dropped first (Writer.h:61-93)."""
    o = np.ascontiguousarray(order, dtype=np.uint32)
    out = np.zeros(N, dtype=np.uint8)
    _check("polar_mask_from_order", lib().polar_mask_from_order(_np_ptr(o), o.size, N, K, _np_ptr(out), N))
    return out


def frozen_tab_text(order, N):
    """FB_N{N}_K{K}.txt text of the order's subset < N (Writer.h:71-79)."""
    o = np.ascontiguousarray(order, dtype=np.uint32)
    return _text_call("polar_write_frozen_tab", _np_ptr(o), o.size, N)


def parameters_h_text(info_mask, par=16, concat=False):
    """polar_parameters.h for an information mask, as Frozen_Bit_Generator writes it
    (Writer.h:110-162); concat = the generator's En flag."""
    m = np.ascontiguousarray(np.asarray(info_mask) != 0, dtype=np.uint8)
    return _text_call("polar_write_parameters_h", _np_ptr(m), m.size, par, 1 if concat else 0)


def load_parameters_h(path):
    """polar_parameters.h -> (information mask, PAR)."""
    cap = 1 << 21
    buf = np.zeros(cap, dtype=np.uint8)
    n, par = ctypes.c_uint32(0), ctypes.c_uint32(0)
    _check("polar_parse_parameters_h", lib().polar_parse_parameters_h(os.fsencode(path), _np_ptr(buf), cap,
                                                                       ctypes.byref(n), ctypes.byref(par)))
    return buf[:n.value].copy(), par.value


def unpack_bits(words, N):
    """[B, ceil(N/64)] uint64/int64 (bit i of word j = x[64j+i]) -> [B, N] uint8."""
    w = np.ascontiguousarray(np.asarray(words)).view(np.uint8)
    w = w.reshape(w.shape[0], -1) if w.ndim > 1 else w.reshape(1, -1)
    return np.unpackbits(w, axis=1, bitorder="little")[:, :N]


def pack_bits(bits):
    """[B, N] 0/1 -> [B, ceil(N/64)] uint64 (inverse of unpack_bits)."""
    b = np.atleast_2d(np.asarray(bits, dtype=np.uint8))
    B, N = b.shape
    W = (N + 63) // 64
    pad = np.zeros((B, W * 64), dtype=np.uint8)
    pad[:, :N] = b
    return np.packbits(pad, axis=1, bitorder="little").view(np.uint64).reshape(B, W)


def _torch():
    import torch  # plumbing only: device memory and streams
    return torch


def _device_cus():
    """compute units of torch's current GPU once torch has initialised it, else 0. Never
    opens the GPU itself: a process with the GPU open compiles generated kernels with hipRTC
    instead of the clang driver (polar_sc_jit.cpp)."""
    try:
        import torch
        if torch.cuda.is_initialized():
            return int(torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count)
    except Exception:
        pass
    return 0


class Decoder:
    """A compiled decode plan for one frozen-bit table (== my_module after do_prunning).

    info_mask: (N,) array, nonzero = information bit (frozen-table bit 1).
    config:    polar_sc_config or None (reference config.h); other configs -> ENOTSUP.
    tuning:    polar_sc_tuning, a dict of its fields, or None (automatic kernel selection).
    """

    def __init__(self, info_mask=None, config=None, tuning=None):
        self._plan = ctypes.c_void_p(None)
        self.N = 0
        if info_mask is not None:
            self.load_frozen_bits(info_mask, config, tuning)

    # -- FB port ---------------------------------------------------------------------------
    def load_frozen_bits(self, info_mask, config=None, tuning=None):
        mask = np.ascontiguousarray(np.asarray(info_mask).astype(np.uint8) != 0, dtype=np.uint8)
        if mask.ndim != 1:
            raise ValueError("info_mask must be 1-D")
        self.close()
        plan = ctypes.c_void_p(None)
        cfg = ctypes.byref(config) if config is not None else None
        tun = make_tuning(tuning)
        _check("polar_sc_plan_create_tuned",
               lib().polar_sc_plan_create_tuned(ctypes.byref(plan), int(mask.size), _np_ptr(mask), cfg,
                                                ctypes.byref(tun) if tun is not None else None))
        self._plan = plan
        self.mask = mask
        self.N = int(mask.size)
        self.K = int(mask.sum())
        self.words = (self.N + 63) // 64
        return self

    def close(self):
        if getattr(self, "_plan", None) is not None and self._plan.value:
            lib().polar_sc_plan_destroy(self._plan)
        self._plan = ctypes.c_void_p(None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- introspection ----------------------------------------------------------------------
    @property
    def stats(self):
        s = polar_sc_plan_stats()
        _check("polar_sc_plan_get_stats", lib().polar_sc_plan_get_stats(self._plan, ctypes.byref(s)))
        d = {f: getattr(s, f) for f, _ in polar_sc_plan_stats._fields_ if f != "op_count"}
        d["op_count"] = {OPS[c]: int(s.op_count[c]) for c in OPS if s.op_count[c]}
        return d

    def schedule(self):
        """The compiled op list as a list of dicts (code name, level, n, pos, upos, fb)."""
        n = ctypes.c_uint32(0)
        _check("polar_sc_plan_get_schedule", lib().polar_sc_plan_get_schedule(self._plan, None, 0, ctypes.byref(n)))
        arr = (polar_sc_op * n.value)()
        _check("polar_sc_plan_get_schedule", lib().polar_sc_plan_get_schedule(self._plan, arr, n.value, ctypes.byref(n)))
        return [dict(op=OPS.get(o.code, o.code), level=o.level, n=o.n, pos=o.pos, upos=o.upos, fb=o.fb)
                for o in arr]

    def compile(self):
        """Build the plan's generated kernel now (host only); False if the plan uses the
        schedule interpreter instead."""
        rc = lib().polar_sc_plan_compile(self._plan)
        if rc == -95:
            return False
        _check("polar_sc_plan_compile", rc)
        return True

    def launch_info(self, batch, cus=None):
        """Launch shape of a decode of `batch` frames (polar_sc_plan_launch_info, host only:
        compiles the generated kernel if needed) as a dict; code_key as 16 hex digits.
        cus=None: the compute units of the current GPU when torch sees one (the count the
        decode itself uses to pick the layout), else 0 (= 256, MI355X)."""
        if cus is None:
            cus = _device_cus()
        r = polar_sc_launch_info()
        _check("polar_sc_plan_launch_info", lib().polar_sc_plan_launch_info(self._plan, int(batch), int(cus),
                                                                            ctypes.byref(r)))
        d = {f: getattr(r, f) for f, _ in polar_sc_launch_info._fields_}
        d["code_key"] = "%016x" % r.code_key
        return d

    def kernel_source(self):
        n = ctypes.c_size_t(0)
        rc = lib().polar_sc_plan_kernel_source(self._plan, None, 0, ctypes.byref(n))
        if rc == -95:
            return None
        _check("polar_sc_plan_kernel_source", rc)
        buf = ctypes.create_string_buffer(n.value + 1)
        _check("polar_sc_plan_kernel_source",
               lib().polar_sc_plan_kernel_source(self._plan, buf, n.value + 1, ctypes.byref(n)))
        return buf.value.decode()

    def prepare(self, max_batch):
        _check("polar_sc_plan_prepare", lib().polar_sc_plan_prepare(self._plan, int(max_batch)))

    # -- e -> s ports -----------------------------------------------------------------------
    def _check_llr(self, llr, allow16=False):
        torch = _torch()
        dtypes = (torch.int8, torch.int16) if allow16 else (torch.int8,)
        if not (isinstance(llr, torch.Tensor) and llr.is_cuda and llr.dtype in dtypes):
            raise TypeError("llr must be a CUDA %s tensor" % ("int8 or int16" if allow16 else "int8"))
        if llr.dim() != 2 or llr.shape[1] != self.N or not llr.is_contiguous():
            raise ValueError("llr must be contiguous [B, %d]" % self.N)
        return torch

    @staticmethod
    def _check_out(out, llr, shape, dtype):
        torch = _torch()
        if not isinstance(out, torch.Tensor) or tuple(out.shape) != tuple(shape) or out.dtype != dtype \
                or not out.is_contiguous():
            raise ValueError("out must be a contiguous %s tensor %s" % (dtype, list(shape)))
        if out.device != llr.device:
            raise ValueError("out must be on the device of llr (%s), not %s" % (llr.device, out.device))

    def decode(self, llr, out=None, stream=None):
        """Decode frames resident on the GPU.

        llr: torch.int8 CUDA tensor [B, N] (contiguous). Returns (or fills `out`) a torch.int64
        CUDA tensor [B, ceil(N/64)] whose bits are x^ (bit i of word j = x^[64j+i]).
        Asynchronous on `stream` (default: torch's current stream of llr's device). An int16
        tensor goes through polar_sc_decode_i16 (the channel for 9-bit LLRs).
        """
        torch = self._check_llr(llr, allow16=True)
        B = llr.shape[0]
        if out is None:
            out = torch.empty((B, self.words), dtype=torch.int64, device=llr.device)
        else:
            self._check_out(out, llr, (B, self.words), torch.int64)
        # the C side picks the code objects / scratch of the current HIP device
        fn = "polar_sc_decode_i16" if llr.dtype == torch.int16 else "polar_sc_decode"
        with torch.cuda.device(llr.device):
            s = stream if stream is not None else torch.cuda.current_stream(llr.device)
            _check(fn, getattr(lib(), fn)(
                self._plan, ctypes.c_void_p(llr.data_ptr()), ctypes.c_void_p(out.data_ptr()), B,
                ctypes.c_void_p(s.cuda_stream)))
        return out

    def trace(self, llr, out=None):
        """Per-op monitor: decode `llr` (as decode(), synchronously) with the instrumented
        kernel and return (records, info). records: one dict per device op (op, level, n, pos,
        nodeN = LLRs of the source node, cycles); info: clock_ghz, total_cycles, us."""
        torch = self._check_llr(llr)
        B = llr.shape[0]
        if out is None:
            out = torch.empty((B, self.words), dtype=torch.int64, device=llr.device)
        else:
            self._check_out(out, llr, (B, self.words), torch.int64)
        with torch.cuda.device(llr.device):
            torch.cuda.synchronize(llr.device)
            n = ctypes.c_uint32(0)
            _check("polar_sc_trace", lib().polar_sc_trace(self._plan, ctypes.c_void_p(llr.data_ptr()),
                                                          ctypes.c_void_p(out.data_ptr()), B, None, 0,
                                                          ctypes.byref(n), None, None))
            recs = (polar_sc_trace_rec * n.value)()
            ghz, tot = ctypes.c_double(0), ctypes.c_uint64(0)
            _check("polar_sc_trace", lib().polar_sc_trace(self._plan, ctypes.c_void_p(llr.data_ptr()),
                                                          ctypes.c_void_p(out.data_ptr()), B, recs, n.value,
                                                          ctypes.byref(n), ctypes.byref(ghz), ctypes.byref(tot)))
        rows = [dict(op=TRACE_OPS.get(r.code, r.code), level=r.level, n=r.n, pos=r.pos, nodeN=self.N >> r.level,
                     cycles=int(r.cycles)) for r in recs]
        info = dict(clock_ghz=ghz.value, total_cycles=int(tot.value),
                    us=(tot.value / ghz.value / 1e3) if ghz.value > 0 else None, frames=B, out=out)
        return rows, info

    def decode_u16(self, llr, out=None, stream=None):
        """As decode(), output int16 [B, N/16]: the TYPE_BITS tokens of my_module's `s` port."""
        torch = self._check_llr(llr)
        B = llr.shape[0]
        if out is None:
            out = torch.empty((B, self.N // 16), dtype=torch.int16, device=llr.device)
        else:
            self._check_out(out, llr, (B, self.N // 16), torch.int16)
        with torch.cuda.device(llr.device):
            s = stream if stream is not None else torch.cuda.current_stream(llr.device)
            _check("polar_sc_decode_u16", lib().polar_sc_decode_u16(
                self._plan, ctypes.c_void_p(llr.data_ptr()), ctypes.c_void_p(out.data_ptr()), B,
                ctypes.c_void_p(s.cuda_stream)))
        return out

    def debug_subtree(self, sid, rows):
        """Test hook of pair plans: generated subtree decoder `sid` on root slot rows (uint16
        [S/4, 64], SM8 pairs; solo layout: [S/8, 64]); returns its partial-sum dwords uint32
        [max(1, S/64), 64] (solo: [max(1, S/128), 64])."""
        torch = _torch()
        S = self.stats["sub_words"]
        nbits = max(1, S // (128 if "#define POLAR_SOLO 1" in self.kernel_source() else 64))
        inp = torch.from_numpy(np.ascontiguousarray(rows, dtype=np.uint16).view(np.int16)).cuda()
        out = torch.zeros((max(1, S // 64), 64), dtype=torch.int32, device="cuda")
        _check("polar_sc_debug_subtree", lib().polar_sc_debug_subtree(self._plan, int(sid), ctypes.c_void_p(inp.data_ptr()),
                                                                       ctypes.c_void_p(out.data_ptr())))
        return out.cpu().numpy().view(np.uint32)[:nbits]

    def decode_host(self, llr):
        """Host arrays in/out (synchronous): int8 [B, N] -> uint64 [B, ceil(N/64)]."""
        a = np.ascontiguousarray(np.atleast_2d(llr), dtype=np.int8)
        if a.shape[1] != self.N:
            raise ValueError("llr must be [B, %d]" % self.N)
        out = np.zeros((a.shape[0], self.words), dtype=np.uint64)
        _check("polar_sc_decode_host", lib().polar_sc_decode_host(self._plan, _np_ptr(a), _np_ptr(out), a.shape[0]))
        return out

    def codeword_to_info(self, xhat):
        """x^ words [B, ceil(N/64)] (host) -> information bits [B, K] (u^ = x^ F^(x)n)."""
        x = np.ascontiguousarray(np.atleast_2d(np.asarray(xhat)).view(np.uint64))
        out = np.zeros((x.shape[0], self.K), dtype=np.uint8)
        _check("polar_codeword_to_info", lib().polar_codeword_to_info(self._plan, _np_ptr(x), _np_ptr(out), x.shape[0]))
        return out


def selftest_lanes():
    """Run the cross-lane exchange self-test on the current GPU; returns [8, 64] source lanes
    (DPP distances 1, 2, 4, 8; permlane16_swap results 0 / 1; permlane32_swap results 0 / 1)."""
    torch = _torch()
    buf = torch.zeros(8 * 64, dtype=torch.int32, device="cuda")
    _check("polar_sc_selftest_lanes", lib().polar_sc_selftest_lanes(ctypes.c_void_p(buf.data_ptr())))
    return buf.view(8, 64).cpu().numpy()


# ---------------------------------------------------------------------------------------
# Frame source and error accounting of the reference testbench (include/polar_sc.h)
# ---------------------------------------------------------------------------------------
def csim_sigma(ebn0_db, rate):
    """sigma of the testbench (src/testbench/main.cpp:91-98), in float32 like the reference."""
    f32 = np.float32
    return float(f32(1.0) / np.sqrt(f32(2.0) * f32(rate) * np.power(f32(10.0), f32(ebn0_db) / f32(10.0), dtype=f32),
                                     dtype=f32))


def csim_states(N, seed, frame0, batch):
    """Host: xorshift128 states at the start of frames frame0.. ([batch, 8] uint32)."""
    out = np.zeros((batch, 8), dtype=np.uint32)
    _check("polar_csim_states", lib().polar_csim_states(ctypes.c_uint32(N), ctypes.c_uint32(seed), ctypes.c_uint64(frame0),
                                   ctypes.c_size_t(batch), out.ctypes.data_as(ctypes.c_void_p)))
    return out


def csim_frames(N, batch, sigma, seed=0xF0, frame0=0, codewords=None, beta=4, vsatn=-31, vsatp=31,
                device=None, stream=None):
    """The reference's C-sim frame chain on the GPU: (llr int8 [batch, N], x^ref int64
    [batch, ceil(N/64)]) torch tensors on `device`."""
    import torch
    dev = torch.device("cuda") if device is None else device
    llr = torch.empty((batch, N), dtype=torch.int8, device=dev)
    xref = torch.empty((batch, (N + 63) // 64), dtype=torch.int64, device=dev)
    cw = None if codewords is None else np.ascontiguousarray(codewords, dtype=np.uint8)
    ncw = 0 if cw is None else cw.shape[0]
    st = torch.cuda.current_stream(dev) if stream is None else stream
    _check("polar_csim_frames", lib().polar_csim_frames(ctypes.c_uint32(N), ctypes.c_uint32(seed), ctypes.c_uint64(frame0),
                                   ctypes.c_size_t(batch), ctypes.c_float(sigma), ctypes.c_int(beta),
                                   ctypes.c_int(vsatn), ctypes.c_int(vsatp),
                                   None if cw is None else cw.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(ncw),
                                   ctypes.c_void_p(llr.data_ptr()), ctypes.c_void_p(xref.data_ptr()),
                                   ctypes.c_void_p(st.cuda_stream)))
    return llr, xref


def count_errors(xhat, xref, N, counts=None, stream=None):
    """sc_error_counter on the GPU: adds [bit errors mod 1024 per frame, frame errors, exact bit
    errors] into `counts` (int64 tensor [3], created when None) and returns it."""
    import torch
    if counts is None:
        counts = torch.zeros(3, dtype=torch.int64, device=xhat.device)
    st = torch.cuda.current_stream(xhat.device) if stream is None else stream
    _check("polar_count_errors", lib().polar_count_errors(ctypes.c_void_p(xhat.data_ptr()), ctypes.c_void_p(xref.data_ptr()),
                                    ctypes.c_uint32(N), ctypes.c_size_t(xhat.shape[0]),
                                    ctypes.c_void_p(counts.data_ptr()), ctypes.c_void_p(st.cuda_stream)))
    return counts
