// polar_sc_interp.h -- the schedule interpreter of the batched SC polar decoder (CDNA4,
// gfx950): per-group storage, the op implementations and the decode loop. Included by
// polar_sc_kernels.hip (hipcc: the generic interpreter kernels) and by the generated
// source of hybrid plans (polar_sc_jit.cpp, hipRTC: the same loop with OP_SUB records that
// call generated subtree decoders). No standard headers: hipRTC-clean.
//
// Execution model:
//   * One wave64 decodes 8 frames. The wave is 4 DPP rows of 16 lanes; the lane holding
//     word position p (lane_pos, polar_sc_device.h) of row r owns LLR 16w+p of every word w
//     of frames f0+r (low 16-bit half of every register) and f0+4+r (high half). PAR = 16
//     of the reference (my_module.h works on one 16-LLR word per cycle) == one DPP row
//     here, so the F/G/H word loops of my_module::do_action are lane-private and the only
//     cross-lane traffic is the leaf (Spec_PolarDec_16), the REP adder tree, the SPC
//     min/parity trees and output packing, all done with DPP row ops.
//   * LLRs are sign-magnitude in packed 16-bit halves (bit 15 = sign, bits 0..14 =
//     magnitude): "SM16". All arithmetic is v_pk_* on two frames at once.
//   * The control flow of the reference FSM does not depend on LLR values, so the host
//     compiles it once per frozen mask into a flat op list (polar_sc_host.cpp); the kernel
//     interprets it with wave-uniform (scalar) control.
//   * Per wave, stage LLRs of the current tree path live in LDS (slot s, lane L at dword
//     s*64+L: conflict-free ds_read_b32) or, for large N, in an HBM scratch area with the
//     same layout (one 256-byte coalesced access per wave per slot). Partial sums
//     (bit_mem_1 of the reference) are per lane: dword d holds words 16d..16d+15, low 16
//     bits = low-half frame, high 16 bits = high-half frame.
#pragma once

#include "polar_sc_device.h"

#ifndef POLAR_SC_SUBS
#define POLAR_SC_SUBS 0
#endif

namespace polar {

typedef unsigned int uint32_t;
typedef int int32_t;
typedef unsigned short uint16_t;
typedef signed char int8_t;
typedef unsigned char uint8_t;
typedef __SIZE_TYPE__ size_t;


enum : int {
    OP_F = 1, OP_G = 2, OP_FLEAF = 3, OP_GLEAF = 4, OP_REP = 5, OP_R1 = 6, OP_SPC = 7,
    OP_H = 8, OP_H0 = 9, OP_END = 10,
    OP_WOPEN = 11, OP_WFLUSH = 12,  // HBM-scratch plans: partial-sum window of a 128-word subtree
    OP_SUB = 13                     // hybrid plans: generated subtree decoder `fb` at node (level, pos)
};
constexpr int WIN_DWORDS = 16;      // 256 words of partial sums (polar_sc_host.cpp LDS_LOW_SLOTS / 16)

struct Op {            // == polar_sc_op (include/polar_sc.h)
    int32_t code, level, n, pos, upos;
    uint32_t fb;
    int32_t r0, r1;
};

// ---------------------------------------------------------------------------------------
// Per-group storage. GMEM = false (small N): every stage slot and the bit dwords in LDS.
// GMEM = true (large N): the slots of the upper tree levels [0, lds0) and the bit dwords in
// HBM scratch, the slots of the lower levels [lds0, nslot) in LDS -- every level moves the
// same volume per frame, and the lower levels run the narrow, latency-bound ops. HBM slots
// hold SM8 pairs (stage values above the leaves never exceed magnitude 31), half the bytes. Slot s,
// lane L lives at dword s*64+L of its space (one 256-byte row per wave access). Base
// pointers include the lane offset; slot / bit-dword indices are wave-uniform.
// ---------------------------------------------------------------------------------------
template <bool GMEM>
struct Ctx;
template <class C> struct GMEM_OF;
template <bool GMEM> struct GMEM_OF<Ctx<GMEM>> { static constexpr bool value = GMEM; };

template <bool GMEM>
struct Ctx {
    uint16_t *hs;          // HBM scratch (GMEM): slots [0, lds0) as SM8 pairs (128 B rows)
    uint32_t *hbit;        // HBM scratch (GMEM): bit dwords (256 B rows)
    uint32_t *lb;          // LDS: slots [lds0, nslot) (GMEM) / slots + bit dwords (!GMEM)
    int lds0;              // first slot held in LDS (0 when !GMEM)
    int wd0;               // GMEM: first bit dword of the open partial-sum window, -1 = none
    uint32_t nslot;        // G - 1
    int G;
    const int8_t *llr_lo, *llr_hi;   // frame rows (lane offset included)
    Lanes ln;
    __device__ __forceinline__ bool in_lds(int slot) const { return !GMEM || slot >= lds0; }
    __device__ __forceinline__ uint32_t ldl(int slot) const { return lb[(slot - lds0) * 64]; }
    __device__ __forceinline__ uint32_t ldh(int slot) const
    {
        const uint32_t h = hs[slot * 64];
        return sm8_pair(h, h >> 8);
    }
    __device__ __forceinline__ void stl(int slot, uint32_t v) const { lb[(slot - lds0) * 64] = v; }
    __device__ __forceinline__ void sth(int slot, uint32_t v) const { hs[slot * 64] = (uint16_t)sm16_to_sm8x2(v); }
    __device__ __forceinline__ uint32_t ld(int slot) const { return in_lds(slot) ? ldl(slot) : ldh(slot); }
    // storage known at compile time (callers branch once per op on in_lds)
    template <bool L> __device__ __forceinline__ uint32_t ldx(int slot) const { return L ? ldl(slot) : ldh(slot); }
    __device__ __forceinline__ void st(int slot, uint32_t v) const
    {
        if (in_lds(slot)) stl(slot, v);
        else sth(slot, v);
    }
    // bit dword d: LDS window (ops inside a windowed subtree), HBM bits, or LDS (!GMEM)
    __device__ __forceinline__ uint32_t *wl(int d) const { return lb + ((int)nslot - lds0 + d - wd0) * 64; }
    __device__ __forceinline__ uint32_t bld(int d) const
    {
        if constexpr (GMEM) return wd0 >= 0 ? *wl(d) : hbit[d * 64];
        else return lb[(nslot + d) * 64];
    }
    // bit dword of an op that is never windowed (its node is wider than the window): a plain
    // load, not a flat one through a selected pointer (which would also wait for the LDS)
    __device__ __forceinline__ uint32_t bld_nowin(int d) const
    {
        if constexpr (GMEM) return hbit[d * 64];
        else return lb[(nslot + d) * 64];
    }
    __device__ __forceinline__ void bst(int d, uint32_t v) const
    {
        if constexpr (GMEM) {
            if (wd0 >= 0) *wl(d) = v;
            else hbit[d * 64] = v;
        } else {
            lb[(nslot + d) * 64] = v;
        }
    }
    __device__ __forceinline__ int lvl_off(int k) const { return G - (G >> (k - 1)); }  // k >= 1
    __device__ __forceinline__ uint32_t chan(int w) const
    {
        return conv_pair((uint32_t)(uint8_t)llr_lo[16 * w] | ((uint32_t)(uint8_t)llr_hi[16 * w] << 16));
    }
    // source word i of a level-k node (k = 0: channel)
    __device__ __forceinline__ uint32_t src(int k, int i) const
    {
        return (k == 0) ? chan(i) : ld(lvl_off(k) + i);
    }
};

#if POLAR_SC_SUBS
// defined by the generated source of a hybrid plan: subtree decoder `id` reads its root
// words from LDS dword `ldo` (+ 64 per word) and writes its partial sums at word `pos`
template <bool GMEM>
__device__ void polar_sub_call(const Ctx<GMEM> &c, int id, int ldo, int pos);
#endif

// partial-sum flags (bits 15/31) of bit_mem word q
__device__ __forceinline__ uint32_t ubit(uint32_t dword, int q) { return (dword << (15 - (q & 15))) & SGN; }

// write n (< 16, aligned) words of hard-decision flags packed in `acc` (bit j = word pos+j)
template <class C>
__device__ __forceinline__ void bits_put_small(const C &c, int pos, int n, uint32_t acc)
{
    uint32_t mlo = ((1u << n) - 1u) << (pos & 15);
    uint32_t m = mlo | (mlo << 16);
    uint32_t d = c.bld(pos >> 4);
    c.bst(pos >> 4, (d & ~m) | (acc & m));
}

// ---------------------------------------------------------------------------------------
// Ops
// ---------------------------------------------------------------------------------------
// SL / DL: source / destination slots in LDS (else HBM scratch)
template <bool ISG, bool ROOT, bool SL, bool DL, class C>
__device__ __forceinline__ void fg_words(const C &c, int k, int n, int upos, int i0, int i1)
{
    const int dst = c.lvl_off(k + 1);
    const int s0 = ROOT ? 0 : c.lvl_off(k);
    auto src = [&](int w) -> uint32_t {
        if constexpr (ROOT) return c.chan(w);
        else if constexpr (SL) return c.ldl(s0 + w);
        else return c.ldh(s0 + w);
    };
    auto put = [&](int w, uint32_t v) {
        if constexpr (DL) c.stl(dst + w, v);
        else c.sth(dst + w, v);
    };
    int i = i0;
    // CH words per iteration: 2 CH independent source loads in flight (16 for HBM sources:
    // the upper levels are latency-bound on the few waves of a group)
    constexpr int CH = (SL || ROOT) ? 8 : 16;
    for (; i + CH <= i1; i += CH) {
        uint32_t a[CH], b[CH], r[CH];
#pragma unroll
        for (int j = 0; j < CH; j++) {
            a[j] = src(i + j);
            b[j] = src(n + i + j);
        }
        if constexpr (ISG) {
            // partial sums of words upos+i .. upos+i+CH-1 (at most two bit dwords)
            uint32_t u0 = 0, u1 = 0;
            if (upos >= 0) {
                // ops wider than the partial-sum window (2n > 16 * WIN_DWORDS words) are never
                // windowed (polar_sc_host.cpp window_schedule)
                if (GMEM_OF<C>::value && n > 8 * WIN_DWORDS) {
                    u0 = c.bld_nowin((upos + i) >> 4);
                    u1 = c.bld_nowin((upos + i + CH - 1) >> 4);
                } else {
                    u0 = c.bld((upos + i) >> 4);
                    u1 = c.bld((upos + i + CH - 1) >> 4);
                }
            }
#pragma unroll
            for (int j = 0; j < CH; j++) {
                const int q = upos + i + j;
                const uint32_t u = (upos >= 0) ? ubit(((q >> 4) == ((upos + i) >> 4)) ? u0 : u1, q) : 0u;
                r[j] = G_sm<GSAT>(a[j], b[j], u);
            }
        } else {
#pragma unroll
            for (int j = 0; j < CH; j++) r[j] = F_sm(a[j], b[j]);
        }
#pragma unroll
        for (int j = 0; j < CH; j++) put(i + j, r[j]);
    }
    for (; i < i1; i++) {
        const uint32_t a = src(i), b = src(n + i);
        uint32_t r;
        if constexpr (ISG) {
            const uint32_t u = (upos >= 0) ? ubit(c.bld((upos + i) >> 4), upos + i) : 0u;
            r = G_sm<GSAT>(a, b, u);
        } else {
            r = F_sm(a, b);
        }
        put(i, r);
    }
}

// F_STATE / G_STATE word loops (my_module.h:373-445, 704-781) for n >= 2 output words:
// dst[i] = F(src[i], src[n+i]) or G(src[i], src[n+i], bit_mem[upos+i]), i in [i0, i1)
// (the words of this wave when the op is split across the waves of a group).
template <bool ISG, class C>
__device__ __forceinline__ void op_fg(const C &c, int k, int n, int upos, int i0, int i1)
{
    const bool dl = c.in_lds(c.lvl_off(k + 1));
    if (k == 0) {
        if (dl) fg_words<ISG, true, false, true>(c, k, n, upos, i0, i1);
        else fg_words<ISG, true, false, false>(c, k, n, upos, i0, i1);
    } else if (c.in_lds(c.lvl_off(k))) {
        fg_words<ISG, false, true, true>(c, k, n, upos, i0, i1);
    } else if (dl) {
        fg_words<ISG, false, false, true>(c, k, n, upos, i0, i1);
    } else {
        fg_words<ISG, false, false, false>(c, k, n, upos, i0, i1);
    }
}

// F/G with NB_ITER = 1 followed by R_STATE: Spec_Polar_Decoder on reg_result
// (my_module.h:544-612)
template <bool ISG, class C>
__device__ __forceinline__ void op_leaf(const C &c, int k, int pos, int upos, uint32_t fb)
{
    uint32_t a = c.src(k, 0), b = c.src(k, 1);
    uint32_t L;
    if constexpr (ISG) {
        uint32_t u = (upos >= 0) ? ubit(c.bld(upos >> 4), upos) : 0u;
        L = G_sm<GSAT>(a, b, u);
    } else {
        L = F_sm(a, b);
    }
    // fb bits 16..18: PRUNING_LEVEL 1 leaf decoder (POLAR_LEAF_*, include/polar_sc.h)
    uint32_t x;
    switch (fb >> 16) {
    case 1: x = leaf_rep(L, c.ln); break;
    case 2: x = leaf_spc<false>(L, c.ln); break;
    case 3: x = leaf_rep2(L, c.ln); break;
    case 4: x = leaf_spc<true>(L, c.ln); break;
    default: x = leaf16(L, fb & 0xFFFFu, c.ln); break;
    }
    int b4 = pos & 15;
    uint32_t m = 0x10001u << b4;
    uint32_t d = c.bld(pos >> 4);
    c.bst(pos >> 4, (d & ~m) | (x >> (15 - b4)));
}

// F_REP_STATE (my_module.h:1292-1390): lambda = F(parent); per word the 16-lane exact SM
// adder tree, accumulated over words in order by the 11-bit saturating SM adder
// (ADDER_TREE_16, functions.h:3190-3205); x = all sign(acc).
template <bool L, class C>
__device__ __forceinline__ void rep_body(const C &c, int s0, int n, int pos)
{
    // value chain in two's complement (exact sums and 511 clamps, polar_sc_device.h); the
    // exact SM chain only when some frame ends on a zero total (sign-of-zero rule). Source
    // words are loaded 8 at a time (one round trip per 8 words for HBM slots).
    uint32_t acc = 0;
    auto word = [&](uint32_t lam) {
        const uint32_t sg = pk_sra(lam, 15);
        acc = rep_acc(acc, row_sum_biased(pk_add(pk_sub((lam & MAG) ^ sg, sg), 0x02000200u)));
    };
    int i = 0;
    for (; i + 8 <= n; i += 8) {
        uint32_t a[8], b[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            a[j] = c.template ldx<L>(s0 + i + j);
            b[j] = c.template ldx<L>(s0 + n + i + j);
        }
#pragma unroll
        for (int j = 0; j < 8; j++) word(F_sm(a[j], b[j]));
    }
    for (; i < n; i++) word(F_sm(c.template ldx<L>(s0 + i), c.template ldx<L>(s0 + n + i)));
    if (rep_any_zero(acc)) {
        acc = 0;
        for (i = 0; i < n; i++) {
            uint32_t lam = F_sm(c.template ldx<L>(s0 + i), c.template ldx<L>(s0 + n + i));
            uint32_t t = row_add_tree(lam, c.ln);
            acc = G_sm<REPSAT>(t, acc, 0u);
        }
    }
    // two's complement or SM16: the decision is bit 15 / 31 either way
    const uint32_t full = pk_sra(acc, 15);
    if (n >= 16) {
        for (int j = 0; j < n / 16; j++) c.bst((pos >> 4) + j, full);
    } else {
        bits_put_small(c, pos, n, full);
    }
}

template <class C>
__device__ __forceinline__ void op_rep(const C &c, int k, int n, int pos)
{
    const int s0 = c.lvl_off(k);
    if (c.in_lds(s0)) rep_body<true>(c, s0, n, pos);
    else rep_body<false>(c, s0, n, pos);
}

// G_R1_STATE (my_module.h:1571-1642) and G_SPC_STATE (my_module.h:1737-1842):
// lambda = G(parent, bits[upos..]); x = sign(lambda); SPC additionally flips the first
// minimum-|lambda| position (lexicographic (|l|, word, bitrev4(lane)) == Min_Mask_16_SM
// tournament + strict '<' across words) when the parity of x is odd.
// [i0, i1): the words of this wave (R1 split in whole 16-word chunks; SPC is never split).
template <bool SPC, bool L, class C>
__device__ __forceinline__ void r1spc_body(const C &c, int s0, int n, int upos, int pos, int i0, int i1)
{
    uint32_t ud = 0, acc = 0, par = 0;
    uint32_t key_lo = 0xFFFFFFFFu, key_hi = 0xFFFFFFFFu;
    auto word = [&](int i, uint32_t a, uint32_t b) {
        uint32_t u = 0;
        if (upos >= 0) {
            if (((upos + i) & 15) == 0 || i == i0) ud = c.bld((upos + i) >> 4);
            u = ubit(ud, upos + i);
        }
        uint32_t lam = G_sm<GSAT>(a, b, u);
        uint32_t h = lam & SGN;
        int q = (pos + i) & 15;
        acc |= h >> (15 - q);
        if (n >= 16 && q == 15) { c.bst((pos + i) >> 4, acc); acc = 0; }
        if constexpr (SPC) {
            par ^= h;
            uint32_t klo = ((lam & QMAG) << 24) | ((uint32_t)i << 4);
            uint32_t khi = (((lam >> 16) & QMAG) << 24) | ((uint32_t)i << 4);
            key_lo = __builtin_elementwise_min(key_lo, klo);
            key_hi = __builtin_elementwise_min(key_hi, khi);
        }
    };
    // source words 8 at a time (one round trip per 8 words for HBM slots), used in order
    int i = i0;
    for (; i + 8 <= i1; i += 8) {
        uint32_t a[8], b[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            a[j] = c.template ldx<L>(s0 + i + j);
            b[j] = c.template ldx<L>(s0 + n + i + j);
        }
#pragma unroll
        for (int j = 0; j < 8; j++) word(i + j, a[j], b[j]);
    }
    for (; i < i1; i++) word(i, c.template ldx<L>(s0 + i), c.template ldx<L>(s0 + n + i));
    if (n < 16) bits_put_small(c, pos, n, acc);
    if constexpr (SPC) {
        par = row_xor(par);
        key_lo = row_min_u32(key_lo | c.ln.br);
        key_hi = row_min_u32(key_hi | c.ln.br);
        uint32_t flip_lo = ((par & 0x8000u) && (key_lo & 15u) == c.ln.br) ? 1u : 0u;
        uint32_t flip_hi = ((par & 0x80000000u) && (key_hi & 15u) == c.ln.br) ? 1u : 0u;
        if (flip_lo) {
            int w = pos + (int)((key_lo >> 4) & 0xFFFFFu);
            c.bst(w >> 4, c.bld(w >> 4) ^ (1u << (w & 15)));
        }
        if (flip_hi) {
            int w = pos + (int)((key_hi >> 4) & 0xFFFFFu);
            c.bst(w >> 4, c.bld(w >> 4) ^ (0x10000u << (w & 15)));
        }
    }
}

// G_R1_STATE (my_module.h:1571-1642) and G_SPC_STATE (my_module.h:1737-1842):
// lambda = G(parent, bits[upos..]); x = sign(lambda); SPC additionally flips the first
// minimum-|lambda| position (lexicographic (|l|, word, bitrev4(lane)) == Min_Mask_16_SM
// tournament + strict '<' across words) when the parity of x is odd.
// [i0, i1): the words of this wave (R1 split in whole 16-word chunks; SPC is never split).
template <bool SPC, class C>
__device__ __forceinline__ void op_r1spc(const C &c, int k, int n, int upos, int pos, int i0, int i1)
{
    const int s0 = c.lvl_off(k);
    if (c.in_lds(s0)) r1spc_body<SPC, true>(c, s0, n, upos, pos, i0, i1);
    else r1spc_body<SPC, false>(c, s0, n, upos, pos, i0, i1);
}

// H_STATE / H0_STATE (my_module.h:903-932, 1020-1042):
// bits[pos..pos+n) = bits[pos..pos+n) ^ bits[pos+n..pos+2n)   (H)
//                  = bits[pos+n..pos+2n)                      (H0)
// [j0, j1): the bit dwords of this wave when n >= 16 (split across the waves of a group)
template <bool H0, class C>
__device__ __forceinline__ void op_h(const C &c, int pos, int n, int j0, int j1)
{
    if (n >= 16) {
        const int da = pos >> 4, db = (pos + n) >> 4;
        int j = j0;
        for (; j + 8 <= j1; j += 8) {   // 8 dwords per round trip
            uint32_t a[8], b[8];
#pragma unroll
            for (int t = 0; t < 8; t++) {
                b[t] = c.bld(db + j + t);
                a[t] = H0 ? 0u : c.bld(da + j + t);
            }
#pragma unroll
            for (int t = 0; t < 8; t++) c.bst(da + j + t, a[t] ^ b[t]);
        }
        for (; j < j1; j++) {
            uint32_t b = c.bld(db + j);
            c.bst(da + j, H0 ? b : (c.bld(da + j) ^ b));
        }
    } else {
        uint32_t mlo = ((1u << n) - 1u) << (pos & 15);
        uint32_t m = mlo | (mlo << 16);
        uint32_t d = c.bld(pos >> 4);
        uint32_t sh = (d >> n) & m;
        c.bst(pos >> 4, H0 ? ((d & ~m) | sh) : (d ^ sh));
    }
}

// ---------------------------------------------------------------------------------------
// The decode kernel. A "group" of `wpg` waves decodes 8 frames together; a block holds
// `gpb` groups (gpb > 1 only when wpg == 1). With wpg > 1 the waves share the group's stage
// storage and split every op that is wide enough (F/G: n >= wpg words; H/H0/R1: n >= 16 wpg
// words, in whole bit dwords); leaves, REP and SPC run on wave 0. A block barrier precedes
// an op whenever it or the op before it was split, so every read sees the writes of the
// waves that produced it. The schedule is data independent, so all groups of a block pass
// the same barriers.
//   llr:  [batch][N] int8;   out: [batch][out_stride] uint16 (bit_mem_1 words, END order)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ bool op_split(int code, int n, int wpg)
{
    if (wpg <= 1) return false;
    switch (code) {
    case OP_F:
    case OP_G: return n >= wpg;
    case OP_H:
    case OP_H0:
    case OP_R1: return n >= 16 * wpg;
    default: return false;
    }
}

// TRACE (the per-op monitor, polar_sc_trace): the lead wave of group 0 stamps the shader
// clock (s_memtime) when each op starts, after its barrier: trace[2 + i] for device op i, the
// END record's slot holding the finish time; trace[0] / trace[1] = s_memrealtime (100 MHz)
// at start and finish, to calibrate the clock.
template <bool GMEM, bool TRACE = false>
__device__ __forceinline__ void decode_body(
    const int8_t *__restrict__ llr, uint16_t *__restrict__ out, const Op *__restrict__ ops,
    uint32_t *__restrict__ scratch, int N, int batch, int out_stride, int wpg, int gpb,
    int group_dwords, int lds_dwords, int lds0, unsigned long long *__restrict__ trace = nullptr)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int lane = threadIdx.x & 63;
    const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: scalar loop control
    const int wi = wib % wpg;                       // wave index in its group
    // the wave that runs the unsplit ops: rotated over the groups so that the lead waves of
    // the groups sharing a CU do not all sit on the same SIMD
    const int lead = wpg > 1 ? (int)(blockIdx.x % (unsigned)wpg) : 0;
    const int gib = wib / wpg;                      // group index in the block
    const long group = (long)blockIdx.x * gpb + gib;
    const int G = N >> 4;
    const int row = lane >> 4;
    const int pl = lane & 15;

    Ctx<GMEM> c;
    c.G = G;
    c.nslot = (uint32_t)(G - 1);
    c.lds0 = GMEM ? lds0 : 0;
    c.wd0 = -1;
    c.lb = smem + (size_t)gib * (size_t)lds_dwords + lane;
    // HBM part of the group: lds0 slots of 64 u16 (SM8 pairs), then the bit dwords
    uint32_t *const gbase = GMEM ? scratch + (size_t)group * (size_t)group_dwords : nullptr;
    c.hs = GMEM ? (uint16_t *)gbase + lane : nullptr;
    c.hbit = GMEM ? gbase + (size_t)lds0 * 32 + lane : nullptr;
    long f_lo = group * 8 + row, f_hi = group * 8 + 4 + row;
    const long f_lo_c = f_lo < batch ? f_lo : (long)batch - 1;
    const long f_hi_c = f_hi < batch ? f_hi : (long)batch - 1;
    c.ln.init((uint32_t)pl);
    c.llr_lo = llr + (size_t)f_lo_c * (size_t)N + c.ln.pos;   // the word position of this lane
    c.llr_hi = llr + (size_t)f_hi_c * (size_t)N + c.ln.pos;

    // an idle group is a whole block when wpg > 1 (gpb == 1), so no barrier is stranded
    if (group * 8 >= batch) return;

    // clear partial-sum memory (H0 may read words the H0 route never wrote)
    const int nbd = (G + 15) >> 4;
    if (wi == lead)
        for (int d = 0; d < nbd; d++) c.bst(d, 0u);

    const bool tracer = TRACE && group == 0 && wi == lead && lane == 0;
    if (tracer) trace[0] = __builtin_amdgcn_s_memrealtime();
    bool prev_split = true;
    int win_d0 = -1;   // GMEM: first bit dword of the open partial-sum window
    // the record of the next op is loaded while the current one runs (the schedule of a
    // large N outgrows the scalar cache; the device copy ends with a spare END record)
    Op cur = ops[0];
    for (int oi = 0;; oi++) {
        const int code = __builtin_amdgcn_readfirstlane(cur.code);
        if (code == OP_END) {
            if (tracer) {
                trace[2 + oi] = __builtin_readcyclecounter();
                trace[1] = __builtin_amdgcn_s_memrealtime();
            }
            break;
        }
        const Op nxt = ops[oi + 1];
        const int k = __builtin_amdgcn_readfirstlane(cur.level);
        const int n = __builtin_amdgcn_readfirstlane(cur.n);
        const int pos = __builtin_amdgcn_readfirstlane(cur.pos);
        const int upos = __builtin_amdgcn_readfirstlane(cur.upos);
        const uint32_t fb = (uint32_t)__builtin_amdgcn_readfirstlane((int)cur.fb);
        const int flag = __builtin_amdgcn_readfirstlane(cur.r0);
        cur = nxt;
        const bool split = op_split(code, n, wpg);
        if (wpg > 1 && (split || prev_split)) __syncthreads();
        if (tracer) trace[2 + oi] = __builtin_readcyclecounter();
        prev_split = split;
        if constexpr (GMEM) {
            if (code == OP_WOPEN || code == OP_WFLUSH) {
                // open: clear the window (bits start at 0); flush: copy it to the HBM bits
                if (wi == lead) {
                    c.wd0 = pos >> 4;
                    for (int j = 0; j < WIN_DWORDS; j++) {
                        if (code == OP_WOPEN) *c.wl(c.wd0 + j) = 0u;
                        else c.hbit[(c.wd0 + j) * 64] = *c.wl(c.wd0 + j);
                    }
                }
                win_d0 = code == OP_WOPEN ? (pos >> 4) : -1;
                continue;
            }
            c.wd0 = flag ? win_d0 : -1;
        }
        if (!split && wi != lead) continue;
        // this wave's share of a split op (whole op otherwise)
        const int i0 = split ? (int)(((long)n * wi) / wpg) : 0;
        const int i1 = split ? (int)(((long)n * (wi + 1)) / wpg) : n;
        switch (code) {
        case OP_F: op_fg<false>(c, k, n, -1, i0, i1); break;
        case OP_G: op_fg<true>(c, k, n, upos, i0, i1); break;
        case OP_FLEAF: op_leaf<false>(c, k, pos, -1, fb); break;
        case OP_GLEAF: op_leaf<true>(c, k, pos, upos, fb); break;
        case OP_REP: op_rep(c, k, n, pos); break;
        case OP_R1: op_r1spc<false>(c, k, n, upos, pos, i0, i1); break;
        case OP_SPC: op_r1spc<true>(c, k, n, upos, pos, 0, n); break;
        case OP_H: op_h<false>(c, pos, n, i0 >> 4, i1 >> 4); break;
        case OP_H0: op_h<true>(c, pos, n, i0 >> 4, i1 >> 4); break;
#if POLAR_SC_SUBS
        case OP_SUB:
            // a whole subtree as generated straight-line code (hybrid plans, polar_sc_jit.cpp):
            // its root words are in the level-k stage slot in LDS, its bits go to `pos`
            polar_sub_call(c, (int)fb, (int)(c.lb - smem) + (c.lvl_off(k) - c.lds0) * 64, pos);
            break;
#endif
        default: break;
        }
    }
    if constexpr (GMEM) c.wd0 = -1;
    if (wpg > 1) __syncthreads();
    if (wi != lead) return;

    // END (my_module.h:1848-1869) + wrapper_out: emit bit_mem words in natural order.
    const bool st_lo = f_lo < batch, st_hi = f_hi < batch;
    uint16_t *o_lo = out + (size_t)f_lo * (size_t)out_stride;
    uint16_t *o_hi = out + (size_t)f_hi * (size_t)out_stride;
    for (int d = 0; d < nbd; d++) {
        uint32_t t = row_transpose16(to_position_order(c.bld(d), c.ln), c.ln);   // lane pl: word 16d+pl
        int w = 16 * d + pl;
        if (w < G) {
            if (st_lo) o_lo[w] = (uint16_t)(t & 0xFFFFu);
            if (st_hi) o_hi[w] = (uint16_t)(t >> 16);
        }
    }
    for (int w = G + pl; w < out_stride; w += 16) {   // pad words (N = 32 with u64 output)
        if (st_lo) o_lo[w] = 0;
        if (st_hi) o_hi[w] = 0;
    }
}

}  // namespace polar
