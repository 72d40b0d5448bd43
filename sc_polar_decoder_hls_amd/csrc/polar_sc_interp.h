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
//     magnitude): "SM16", or (POLAR_CA2) two's complement i16 halves. All arithmetic is
//     v_pk_* on two frames at once (the dp_* datapath of polar_sc_device.h).
//   * PAR > 16 (POLAR_LPAR): a PAR word is P16 consecutive 16-LLR device words. The host
//     expands every PAR-word leaf into device ops (exact G flagged in the op), PR1 leaf
//     decoders of whole PAR words are OP_PLEAF records, REP / SPC work per PAR word.
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
// LDS words through address-space-3 pointers: ds_read / ds_write, never flat accesses (which
// also count against vmcnt and wait behind outstanding HBM stores)
typedef __attribute__((address_space(3))) uint32_t lds_u32;


enum : int {
    OP_F = 1, OP_G = 2, OP_FLEAF = 3, OP_GLEAF = 4, OP_REP = 5, OP_R1 = 6, OP_SPC = 7,
    OP_H = 8, OP_H0 = 9, OP_END = 10,
    OP_WOPEN = 11, OP_WFLUSH = 12,  // HBM-scratch plans: partial-sum window of a 128-word subtree
    OP_SUB = 13,                    // hybrid plans: generated subtree decoder `fb` at node (level, pos)
    OP_PLEAF = 14,                  // PAR > 16: PRUNING_LEVEL 1 leaf decoder (fb kind) of the PAR word at (level, pos)
    // grid-tier plans (polar_sc_host.cpp tier_schedule): the schedule runs as segments between
    // grid-wide F / G launches; a segment ends with OP_SEGEND (no output) or OP_END (the last)
    // and every segment but the first starts with OP_SEGCONT (the partial sums persist)
    OP_SEGEND = 15, OP_SEGCONT = 16
};
// op.fb fields besides the leaf frozen pattern (bits 0..15) and PR1 leaf kind (16..18)
constexpr uint32_t FB_EXACT = 1u << 19;   // G / GLEAF inside a PAR-word leaf: G_extended (no clamp)
__device__ __forceinline__ int fb_width(uint32_t fb) { return QB + (int)((fb >> 20) & 15u); }   // operand width
// HBM-scratch plans keep the levels of the nodes of at most W words (W = G - lds0, the plan's
// LDS region, polar_sc_host.cpp lds_slots) in LDS, and the partial sums of the current W-word
// subtree in an LDS window of W / 16 dwords
constexpr int SPC_XWAVES = 8;       // HBM-scratch plans: an SPC op splits over at most this many waves
                                    // (their parity / min-key partials meet in an LDS exchange area
                                    // of 3 x 64 dwords per wave after the window)

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

// HBM slot element: two 8-bit values, or a whole register when LLRs need 9 bits
template <bool B> struct SlotT { typedef uint16_t T; };
template <> struct SlotT<true> { typedef uint32_t T; };
typedef SlotT<SLOT16>::T slot_t;
// LDS stage slots of HBM-scratch plans: the HBM element (8-bit pairs) when the values fit it,
// i.e. not inside PAR-word leaves (PAR > 16, whose exact G widens the operands)
constexpr bool LDS8 = !SLOT16 && P16 == 1;
typedef SlotT<!LDS8>::T lslot_t;
typedef __attribute__((address_space(3))) lslot_t lds_slot;
#if POLAR_CHAN16
typedef short chan_t;          // int16 channel stream (polar_sc_decode_i16)
#else
typedef int8_t chan_t;
#endif

template <bool GMEM>
struct Ctx {
    slot_t *hs;            // HBM scratch (GMEM): slots [0, lds0), 8-bit pairs (128 B rows)
    uint32_t *hbit;        // HBM scratch (GMEM): bit dwords (256 B rows)
    lds_u32 *lb;           // !GMEM: LDS slots + bit dwords (u32 per lane)
    lds_slot *ls;          // GMEM: LDS slots [lds0, nslot) (lslot_t per lane)
    lds_u32 *lw;           // GMEM: the partial-sum window (win dwords), then the SPC exchange area
    int win;               // GMEM: window dwords (W / 16)
    int lds0;              // first slot held in LDS (0 when !GMEM)
    int wd0;               // GMEM: first bit dword of the open partial-sum window, -1 = none
    uint32_t nslot;        // G - 1
    int G;
    const chan_t *llr_lo, *llr_hi;   // frame rows (lane offset included)
    Lanes ln;
    __device__ __forceinline__ bool in_lds(int slot) const { return !GMEM || slot >= lds0; }
    __device__ __forceinline__ uint32_t ldl(int slot) const
    {
        if constexpr (GMEM && LDS8) return slot_unpack(ls[(slot - lds0) * 64]);
        else if constexpr (GMEM) return ls[(slot - lds0) * 64];
        else return lb[slot * 64];
    }
    __device__ __forceinline__ uint32_t ldh(int slot) const
    {
        if constexpr (SLOT16) return hs[slot * 64];
        else return slot_unpack(hs[slot * 64]);
    }
    __device__ __forceinline__ void stl(int slot, uint32_t v) const
    {
        if constexpr (GMEM && LDS8) ls[(slot - lds0) * 64] = (lslot_t)slot_pack(v);
        else if constexpr (GMEM) ls[(slot - lds0) * 64] = v;
        else lb[slot * 64] = v;
    }
    __device__ __forceinline__ void sth(int slot, uint32_t v) const
    {
        if constexpr (SLOT16) hs[slot * 64] = v;
        else hs[slot * 64] = (uint16_t)slot_pack(v);
    }
    __device__ __forceinline__ uint32_t ld(int slot) const { return in_lds(slot) ? ldl(slot) : ldh(slot); }
    // storage known at compile time (callers branch once per op on in_lds)
    template <bool L> __device__ __forceinline__ uint32_t ldx(int slot) const { return L ? ldl(slot) : ldh(slot); }
    __device__ __forceinline__ void st(int slot, uint32_t v) const
    {
        if (in_lds(slot)) stl(slot, v);
        else sth(slot, v);
    }
    // bit dword d: LDS window (ops inside a windowed subtree), HBM bits, or LDS (!GMEM)
    __device__ __forceinline__ lds_u32 *wl(int d) const { return lw + (d - wd0) * 64; }
    // GMEM: the SPC exchange area after the window (SPC_XWAVES x 3 dwords per lane)
    __device__ __forceinline__ lds_u32 *xs() const { return lw + win * 64; }
    __device__ __forceinline__ uint32_t bld(int d) const
    {
        if constexpr (GMEM) {
            if (wd0 >= 0) return *wl(d);   // wave-uniform branch: a ds_read or a global load
            return hbit[d * 64];
        } else {
            return lb[(nslot + d) * 64];
        }
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
        return dp_chan((uint32_t)(uint16_t)(short)llr_lo[16 * w] | ((uint32_t)(uint16_t)(short)llr_hi[16 * w] << 16));
    }
    // source word i of a level-k node (k = 0: channel)
    __device__ __forceinline__ uint32_t src(int k, int i) const
    {
        return (k == 0) ? chan(i) : ld(lvl_off(k) + i);
    }
};

// a root word of a generated subtree decoder from its LDS stage slot (8-bit pairs or SM16)
__device__ __forceinline__ uint32_t ch_load(uint32_t v) { return v; }
__device__ __forceinline__ uint32_t ch_load(uint16_t v) { return slot_unpack(v); }

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
// SL / DL: source / destination slots in LDS (else HBM scratch). X: exact G (G_extended
// inside a PAR-word leaf, no clamp); w: operand width (CA2 F wrap point).
template <bool ISG, bool ROOT, bool SL, bool DL, bool X, class C>
__device__ __forceinline__ void fg_words(const C &c, int k, int n, int upos, int i0, int i1, int w)
{
    const int dst = c.lvl_off(k + 1);
    const int s0 = ROOT ? 0 : c.lvl_off(k);
    auto src = [&](int w_) -> uint32_t {
        if constexpr (ROOT) return c.chan(w_);
        else if constexpr (SL) return c.ldl(s0 + w_);
        else return c.ldh(s0 + w_);
    };
    auto put = [&](int w_, uint32_t v) {
        if constexpr (DL) c.stl(dst + w_, v);
        else c.sth(dst + w_, v);
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
                if (GMEM_OF<C>::value && n > 8 * c.win) {
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
                r[j] = dp_G<!X>(a[j], b[j], u);
            }
        } else {
#pragma unroll
            for (int j = 0; j < CH; j++) r[j] = dp_F(a[j], b[j], w);
        }
#pragma unroll
        for (int j = 0; j < CH; j++) put(i + j, r[j]);
    }
    for (; i < i1; i++) {
        const uint32_t a = src(i), b = src(n + i);
        uint32_t r;
        if constexpr (ISG) {
            const uint32_t u = (upos >= 0) ? ubit(c.bld((upos + i) >> 4), upos + i) : 0u;
            r = dp_G<!X>(a, b, u);
        } else {
            r = dp_F(a, b, w);
        }
        put(i, r);
    }
}

// F_STATE / G_STATE word loops (my_module.h:373-445, 704-781) for n >= 2 output words:
// dst[i] = F(src[i], src[n+i]) or G(src[i], src[n+i], bit_mem[upos+i]), i in [i0, i1)
// (the words of this wave when the op is split across the waves of a group).
template <bool ISG, bool X, class C>
__device__ __forceinline__ void op_fg_x(const C &c, int k, int n, int upos, int i0, int i1, int w)
{
    const bool dl = c.in_lds(c.lvl_off(k + 1));
    if (k == 0) {
        if (dl) fg_words<ISG, true, false, true, X>(c, k, n, upos, i0, i1, w);
        else fg_words<ISG, true, false, false, X>(c, k, n, upos, i0, i1, w);
    } else if (c.in_lds(c.lvl_off(k))) {
        fg_words<ISG, false, true, true, X>(c, k, n, upos, i0, i1, w);
    } else if (dl) {
        fg_words<ISG, false, false, true, X>(c, k, n, upos, i0, i1, w);
    } else {
        fg_words<ISG, false, false, false, X>(c, k, n, upos, i0, i1, w);
    }
}
template <bool ISG, class C>
__device__ __forceinline__ void op_fg(const C &c, int k, int n, int upos, int i0, int i1, uint32_t fb)
{
    // exact G only occurs inside PAR-word leaves (PAR > 16), always on LDS levels
    if constexpr (ISG && P16 > 1) {
        if (fb & FB_EXACT) {
            fg_words<ISG, false, true, true, true>(c, k, n, upos, i0, i1, fb_width(fb));
            return;
        }
    }
    op_fg_x<ISG, false>(c, k, n, upos, i0, i1, fb_width(fb));
}

// PRUNING_LEVEL 1 leaf decoders of one 16-LLR word (R_STATE, my_module.h:566-593) in the
// configured format: REP / REP2 (sel 1) / SPC / SPC2 (sel 1); w: operand width
__device__ __forceinline__ uint32_t leaf_kind_dp(uint32_t L, uint32_t kind, const Lanes &ln, int w)
{
    if (kind == 5) return L & SGN;   // Spec_Node_R1: VECTOR_SIGN
    if constexpr (!CA2) {
        switch (kind) {
        case 1: return leaf_rep(L, ln);
        case 2: return leaf_spc<false>(L, ln);
        case 3: return leaf_rep2(L, ln);
        default: return leaf_spc<true>(L, ln);
        }
    } else {
        // REP_{16}_CA2 / REP_REP2 (functions.h:870-1260): sign of the exact sum (of each
        // position class for REP2); exact i16 sums, pairs at distance 8, 4, 2 (, 1)
        if (kind == 1 || kind == 3) {
            uint32_t v = L;
            v = pk_add(v, xorlane<8>(v));
            v = pk_add(v, xorlane<4>(v));
            v = pk_add(v, xorlane<2>(v));
            if (kind == 1) v = pk_add(v, xorlane<1>(v));
            return v & SGN;
        }
        // SPC_{16} / SPC_SPC2 CA2 (functions.h:2024-2250, 2700-2930): sign ^ (parity & mask),
        // the tournament on qabs (signed: the wrapped qabs(-2^(w-1)) is the minimum)
        const bool spc2 = kind == 4;
        const uint32_t h = L & SGN;
        uint32_t par = h;
        par ^= xorlane<8>(par);
        par ^= xorlane<4>(par);
        par ^= xorlane<2>(par);
        if (!spc2) par ^= xorlane<1>(par);
        const uint32_t qa = pk_add(ca2_qabs(L, w), (1u << (w - 1)) * 0x00010001u);   // order-preserving, >= 0
        uint32_t klo = ((qa & 0xFFFFu) << 4) | ln.br, khi = ((qa >> 16) << 4) | ln.br;
        const uint32_t mlo0 = klo, mhi0 = khi;
        klo = __builtin_elementwise_min(klo, xorlane<8>(klo));
        khi = __builtin_elementwise_min(khi, xorlane<8>(khi));
        klo = __builtin_elementwise_min(klo, xorlane<4>(klo));
        khi = __builtin_elementwise_min(khi, xorlane<4>(khi));
        klo = __builtin_elementwise_min(klo, xorlane<2>(klo));
        khi = __builtin_elementwise_min(khi, xorlane<2>(khi));
        if (!spc2) {
            klo = __builtin_elementwise_min(klo, xorlane<1>(klo));
            khi = __builtin_elementwise_min(khi, xorlane<1>(khi));
        }
        const uint32_t flo = (klo == mlo0) ? (par & 0x8000u) : 0u;
        const uint32_t fhi = (khi == mhi0) ? (par & 0x80000000u) : 0u;
        return h ^ flo ^ fhi;
    }
}

// (the PAR-word helpers -- bitrev_n .. word_node, spc keys, PARW -- live in polar_sc_device.h:
// the generated pair kernels of PAR 4 / 8 decode their device words with them too)

// F/G with NB_ITER = 1 followed by R_STATE: Spec_Polar_Decoder on reg_result
// (my_module.h:544-612). Inside a PAR-word leaf (PAR > 16) G may be exact (FB_EXACT) and
// the operands wider than LLR_BITS.
template <bool ISG, class C>
__device__ __forceinline__ void op_leaf(const C &c, int k, int pos, int upos, uint32_t fb, uint32_t info = 0)
{
    uint32_t a = c.src(k, 0), b = c.src(k, 1);
    uint32_t L;
    int w = fb_width(fb);
    if constexpr (ISG) {
        uint32_t u = (upos >= 0) ? ubit(c.bld(upos >> 4), upos) : 0u;
        if (P16 > 1 && (fb & FB_EXACT)) {
            L = dp_G<false>(a, b, u);
            w += 1;
        } else {
            L = dp_G<true>(a, b, u);
        }
    } else {
        L = dp_F(a, b, w);
    }
    uint32_t x;
    if constexpr (LPAR < 4) {
        // PAR 4 / 8: the whole 16-LLR node below the F / G -- its PAR words, their pruning and
        // leaves (info: the group classes, polar_sc_host.cpp word_info)
        x = word_node<0, 16>(L, fb & 0xFFFFu, info, c.ln);
    } else {
        // fb bits 16..18: PRUNING_LEVEL 1 leaf decoder (POLAR_LEAF_*, include/polar_sc.h)
        const uint32_t kind = (fb >> 16) & 7u;
        x = kind ? leaf_kind_dp(L, kind, c.ln, w) : leaf16_dp(L, fb & 0xFFFFu, c.ln, w);
    }
    int b4 = pos & 15;
    uint32_t m = 0x10001u << b4;
    uint32_t d = c.bld(pos >> 4);
    c.bst(pos >> 4, (d & ~m) | (x >> (15 - b4)));
}

// The shipped datapath (SIGMAG, PAR 16, LLR_BITS <= 8): the packed fast paths below. Any
// other format takes the generic 32-bit REP value path and PAR-word SPC keys.


// bits [pos, pos + n) of the partial sums = per-half decision flags `full` (0xFFFF / 0)
template <class C>
__device__ __forceinline__ void bits_fill(const C &c, int pos, int n, uint32_t full)
{
    if (n >= 16) {
        for (int j = 0; j < n / 16; j++) c.bst((pos >> 4) + j, full);
    } else {
        bits_put_small(c, pos, n, full);
    }
}

// F_REP_STATE (my_module.h:1292-1390): lambda = F(parent); per PAR word the exact pair tree
// of its PAR LLRs (ADD_TREE_{PAR}), accumulated over the PAR words in order by the saturating
// adder of ADDER_TREE_{PAR} (functions.h:3163-3320); x = all sign(acc).
template <bool L, class C>
__device__ __forceinline__ void rep_body(const C &c, int s0, int n, int pos)
{
    if constexpr (DEFAULT_FMT) {
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
        bits_fill(c, pos, n, pk_sra(acc, 15));
    } else if constexpr (LPAR < 4) {
        // PAR 4 / 8: the PAR words of each device word are its lane groups -- the exact pair
        // tree of every group, then the saturating chain over the groups in order (words in
        // order, groups in lane order); SM or CA2 arithmetic throughout
        uint32_t acc = 0;
        const uint32_t gr = c.ln.pos >> LPAR;
        for (int i = 0; i < n; i++) {
            const uint32_t lam = dp_F(c.template ldx<L>(s0 + i), c.template ldx<L>(s0 + n + i), QB);
            acc = group_chain<PPW>(acc, add_tree_w<PARW, 1>(lam, c.ln), gr);
        }
        bits_fill(c, pos, n, pk_sra(acc, 15));
    } else {
        // every format: the exact PAR-word totals as 32-bit values per frame, the saturating
        // chain in 32 bits (CA2: qadd, the decision is the sign; SIGMAG: the same value chain,
        // with the exact SM chain when a frame ends on zero)
        int alo = 0, ahi = 0;
        const int sat = (int)REPSAT;
        for (int i = 0; i < n; i += P16) {
            int tlo = 0, thi = 0;
            for (int j = 0; j < P16; j++) {
                const uint32_t lam = dp_F(c.template ldx<L>(s0 + i + j), c.template ldx<L>(s0 + n + i + j), QB);
                tlo += val_lo(lam);
                thi += val_hi(lam);
            }
            tlo = (int)row_sum32((uint32_t)tlo);
            thi = (int)row_sum32((uint32_t)thi);
            alo = __builtin_elementwise_min(__builtin_elementwise_max(alo + tlo, -sat), sat);
            ahi = __builtin_elementwise_min(__builtin_elementwise_max(ahi + thi, -sat), sat);
        }
        uint32_t full = (alo < 0 ? 0xFFFFu : 0u) | (ahi < 0 ? 0xFFFF0000u : 0u);
        if constexpr (!CA2) {
            if (__builtin_amdgcn_ballot_w64(alo == 0 || ahi == 0) != 0ull) {
                // ADD_TREE_{PAR}_SM pair tree (words at distance P16/2 .. 1, then the row) and
                // qfull_adder_sat_sm over the PAR words: the sign of a zero total
                uint32_t acc = 0;
                for (int i = 0; i < n; i += P16) {
                    uint32_t v[P16];
#pragma unroll
                    for (int j = 0; j < P16; j++)
                        v[j] = F_sm(c.template ldx<L>(s0 + i + j), c.template ldx<L>(s0 + n + i + j));
#pragma unroll
                    for (int m = P16; m > 1; m /= 2)
#pragma unroll
                        for (int j = 0; j < m / 2; j++) v[j] = G_sm<0>(v[j], v[j + m / 2], 0u);
                    acc = G_sm<REPSAT>(row_add_tree(v[0], c.ln), acc, 0u);
                }
                full = pk_sra(acc, 15);
            }
        }
        bits_fill(c, pos, n, full);
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
// minimum-|lambda| position (lexicographic (|l|, PAR word, bitrev(position)) == Min_Mask
// tournament + strict '<' across PAR words) when the parity of x is odd.
// [i0, i1): the words of this wave (R1 split in whole 16-word chunks; SPC is never split).
// xw > 1 (SPC split over xw waves of an HBM-scratch group, wave index xi): every wave
// reduces its words' parity and min keys, the partials meet in the LDS exchange area, and wave
// 0 of the split applies the flip (after the barrier, so every wave's decisions are stored).
template <bool SPC, bool L, class C>
__device__ __forceinline__ void r1spc_body(const C &c, int s0, int n, int upos, int pos, int i0, int i1, int xw = 1,
                                           int xi = 0)
{
    uint32_t ud = 0, acc = 0, par = 0;
    uint32_t key_lo = 0xFFFFFFFFu, key_hi = 0xFFFFFFFFu;
    auto word = [&](int i, uint32_t a, uint32_t b) {
        uint32_t u = 0;
        if (upos >= 0) {
            if (((upos + i) & 15) == 0 || i == i0) ud = c.bld((upos + i) >> 4);
            u = ubit(ud, upos + i);
        }
        uint32_t lam = dp_G<true>(a, b, u);
        uint32_t h = lam & SGN;
        int q = (pos + i) & 15;
        acc |= h >> (15 - q);
        if (n >= 16 && q == 15) { c.bst((pos + i) >> 4, acc); acc = 0; }
        if constexpr (SPC) {
            par ^= h;
            const uint32_t mg = spc_mag(lam), wk = spc_word_key(i);
            uint32_t klo = ((mg & 0xFFu) << 24) | wk;
            uint32_t khi = (((mg >> 16) & 0xFFu) << 24) | wk;
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
        const uint32_t lk = spc_lane_key(c.ln);
        key_lo = row_min_u32(key_lo | lk);
        key_hi = row_min_u32(key_hi | lk);
        if constexpr (GMEM_OF<C>::value) {
            if (xw > 1) {
                lds_u32 *const x = c.xs();
                x[(3 * xi) * 64] = par;
                x[(3 * xi + 1) * 64] = key_lo;
                x[(3 * xi + 2) * 64] = key_hi;
                __syncthreads();
                if (xi != 0) return;
                for (int w = 1; w < xw; w++) {
                    par ^= x[(3 * w) * 64];
                    key_lo = __builtin_elementwise_min(key_lo, (uint32_t)x[(3 * w + 1) * 64]);
                    key_hi = __builtin_elementwise_min(key_hi, (uint32_t)x[(3 * w + 2) * 64]);
                }
            }
        }
        const uint32_t bm = SPC_LANE_BITS;
        uint32_t flip_lo = ((par & 0x8000u) && (key_lo & bm) == lk) ? 1u : 0u;
        uint32_t flip_hi = ((par & 0x80000000u) && (key_hi & bm) == lk) ? 1u : 0u;
        if (flip_lo) {
            int w = pos + spc_key_word(key_lo);
            c.bst(w >> 4, c.bld(w >> 4) ^ (1u << (w & 15)));
        }
        if (flip_hi) {
            int w = pos + spc_key_word(key_hi);
            c.bst(w >> 4, c.bld(w >> 4) ^ (0x10000u << (w & 15)));
        }
    }
}

template <bool SPC, class C>
__device__ __forceinline__ void op_r1spc(const C &c, int k, int n, int upos, int pos, int i0, int i1, int xw = 1,
                                         int xi = 0)
{
    const int s0 = c.lvl_off(k);
    if (c.in_lds(s0)) r1spc_body<SPC, true>(c, s0, n, upos, pos, i0, i1, xw, xi);
    else r1spc_body<SPC, false>(c, s0, n, upos, pos, i0, i1, xw, xi);
}

// PAR > 16: the PRUNING_LEVEL 1 leaf decoders (R_STATE, my_module.h:566-593; library.h:
// 187-280) of the PAR word whose P16 device words are the level-k node at `pos` (the LLRs
// F / G wrote there): REP (kind 1) / SPC (2) / REP2 (3, sel 1) / SPC2 (4, sel 1), the pair
// trees and tournaments over PAR positions (words at distance P16/2 .. 1 first, then the row).
template <class C>
__device__ __forceinline__ void op_pleaf(const C &c, int k, int pos, uint32_t kind)
{
    if constexpr (P16 > 1) {
        const int s0 = c.lvl_off(k);   // a node of <= 4 words: always an LDS level
        uint32_t v[P16];
#pragma unroll
        for (int j = 0; j < P16; j++) v[j] = c.ldl(s0 + j);
        uint32_t x[P16];
        if (kind == 5) {   // Spec_Node_R1: VECTOR_SIGN
#pragma unroll
            for (int j = 0; j < P16; j++) x[j] = v[j] & SGN;
        } else if (kind == 1 || kind == 3) {
            uint32_t t[P16];
#pragma unroll
            for (int j = 0; j < P16; j++) t[j] = v[j];
#pragma unroll
            for (int m = P16; m > 1; m /= 2)
#pragma unroll
                for (int j = 0; j < m / 2; j++) t[j] = CA2 ? pk_add(t[j], t[j + m / 2]) : G_sm<0>(t[j], t[j + m / 2], 0u);
            uint32_t r;
            if constexpr (CA2) {
                r = t[0];
                r = pk_add(r, xorlane<8>(r));
                r = pk_add(r, xorlane<4>(r));
                r = pk_add(r, xorlane<2>(r));
                if (kind == 1) r = pk_add(r, xorlane<1>(r));
                r &= SGN;
            } else {
                r = kind == 1 ? leaf_rep(t[0], c.ln) : leaf_rep2(t[0], c.ln);
            }
#pragma unroll
            for (int j = 0; j < P16; j++) x[j] = r;
        } else {
            const bool spc2 = kind == 4;
            uint32_t par = 0;
#pragma unroll
            for (int j = 0; j < P16; j++) par ^= v[j] & SGN;
            par ^= xorlane<8>(par);
            par ^= xorlane<4>(par);
            par ^= xorlane<2>(par);
            if (!spc2) par ^= xorlane<1>(par);
            // keys: (magnitude, bitrev_LPAR(16 j + pos)); SIGMAG: the Q-1-bit |l|; CA2: qabs at
            // QB bits (the wrapped -2^(QB-1) is the minimum), biased to stay non-negative
            const uint32_t lk = c.ln.br << (LPAR - 4);
            uint32_t klo = 0xFFFFFFFFu, khi = 0xFFFFFFFFu, mlo[P16], mhi[P16];
#pragma unroll
            for (int j = 0; j < P16; j++) {
                const uint32_t mg = CA2 ? pk_add(ca2_qabs(v[j], QB), (1u << (QB - 1)) * 0x00010001u) : (v[j] & MAG);
                const uint32_t wk = lk | bitrev_n((uint32_t)j, LPAR - 4);
                mlo[j] = ((mg & 0xFFFFu) << 8) | wk;
                mhi[j] = ((mg >> 16) << 8) | wk;
                klo = __builtin_elementwise_min(klo, mlo[j]);
                khi = __builtin_elementwise_min(khi, mhi[j]);
            }
            klo = __builtin_elementwise_min(klo, xorlane<8>(klo));
            khi = __builtin_elementwise_min(khi, xorlane<8>(khi));
            klo = __builtin_elementwise_min(klo, xorlane<4>(klo));
            khi = __builtin_elementwise_min(khi, xorlane<4>(khi));
            klo = __builtin_elementwise_min(klo, xorlane<2>(klo));
            khi = __builtin_elementwise_min(khi, xorlane<2>(khi));
            if (!spc2) {
                klo = __builtin_elementwise_min(klo, xorlane<1>(klo));
                khi = __builtin_elementwise_min(khi, xorlane<1>(khi));
            }
#pragma unroll
            for (int j = 0; j < P16; j++) {
                const uint32_t flo = (klo == mlo[j]) ? (par & 0x8000u) : 0u;
                const uint32_t fhi = (khi == mhi[j]) ? (par & 0x80000000u) : 0u;
                x[j] = (v[j] & SGN) ^ flo ^ fhi;
            }
        }
        // x (sign-position flags per lane, word pos + j) into the partial sums
#pragma unroll
        for (int j = 0; j < P16; j++) {
            const int wd = pos + j, b4 = wd & 15;
            const uint32_t m = 0x10001u << b4;
            const uint32_t d = c.bld(wd >> 4);
            c.bst(wd >> 4, (d & ~m) | (x[j] >> (15 - b4)));
        }
    }
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
__device__ __forceinline__ bool op_split(int code, int n, int wpg, bool gmem)
{
    if (wpg <= 1) return false;
    switch (code) {
    case OP_F:
    case OP_G: return n >= wpg;
    case OP_H:
    case OP_H0:
    case OP_R1: return n >= 16 * wpg;
    case OP_SPC: return gmem && n >= 16 * (wpg < SPC_XWAVES ? wpg : SPC_XWAVES);   // whole dwords per wave
    default: return false;
    }
}

// TRACE (the per-op monitor, polar_sc_trace): the lead wave of group 0 stamps the shader
// clock (s_memtime) when each op starts, after its barrier: trace[2 + i] for device op i, the
// END record's slot holding the finish time; trace[0] / trace[1] = s_memrealtime (100 MHz)
// at start and finish, to calibrate the clock.
template <bool GMEM, bool TRACE = false>
__device__ __forceinline__ void decode_body(
    const chan_t *__restrict__ llr, uint16_t *__restrict__ out, const Op *__restrict__ ops,
    uint32_t *__restrict__ scratch, int N, int batch, int out_stride, int wpg, int gpb,
    int group_dwords, int lds_dwords, int lds0, unsigned long long *__restrict__ trace = nullptr)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int lane = threadIdx.x & 63;
    const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: scalar loop control
    const int lw = __builtin_ctz((unsigned)wpg);    // wpg is a power of two
    const int wi = wib & (wpg - 1);                 // wave index in its group
    // the wave that runs the unsplit ops: rotated over the groups so that the lead waves of
    // the groups sharing a CU do not all sit on the same SIMD
    const int lead = wpg > 1 ? (int)(blockIdx.x & (unsigned)(wpg - 1)) : 0;
    const int gib = wib >> lw;                      // group index in the block
    const long group = (long)blockIdx.x * gpb + gib;
    const int G = N >> 4;
    const int row = lane >> 4;
    const int pl = lane & 15;

    Ctx<GMEM> c;
    c.G = G;
    c.nslot = (uint32_t)(G - 1);
    c.lds0 = GMEM ? lds0 : 0;
    c.wd0 = -1;
    lds_u32 *const gl = (lds_u32 *)smem + (size_t)gib * (size_t)lds_dwords;
    c.lb = gl + lane;
    // GMEM: W - 1 slots of lslot_t per lane, then the window and the SPC exchange area (dwords)
    c.win = (G - c.lds0) >> 4;
    c.ls = (lds_slot *)gl + lane;
    c.lw = gl + (size_t)(G - 1 - c.lds0) * (size_t)(64 * sizeof(lslot_t) / 4) + lane;
    // HBM part of the group: lds0 slots of 64 u16 (SM8 pairs), then the bit dwords
    uint32_t *const gbase = GMEM ? scratch + (size_t)group * (size_t)group_dwords : nullptr;
    c.hs = GMEM ? (slot_t *)gbase + lane : nullptr;
    c.hbit = GMEM ? gbase + (size_t)lds0 * (SLOT16 ? 64 : 32) + lane : nullptr;
    long f_lo = group * 8 + row, f_hi = group * 8 + 4 + row;
    const long f_lo_c = f_lo < batch ? f_lo : (long)batch - 1;
    const long f_hi_c = f_hi < batch ? f_hi : (long)batch - 1;
    c.ln.init((uint32_t)pl);
    c.llr_lo = llr + (size_t)f_lo_c * (size_t)N + c.ln.pos;   // the word position of this lane
    c.llr_hi = llr + (size_t)f_hi_c * (size_t)N + c.ln.pos;

    // an idle group is a whole block when wpg > 1 (gpb == 1), so no barrier is stranded
    if (group * 8 >= batch) return;

    // clear partial-sum memory (H0 may read words the H0 route never wrote), unless this is a
    // continuation segment of a grid-tier plan
    const int nbd = (G + 15) >> 4;
    const bool fresh = __builtin_amdgcn_readfirstlane(ops[0].code) != OP_SEGCONT;
    if (wi == lead && fresh)
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
        if (code == OP_SEGEND) return;   // grid-tier segment: the next launch continues
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
        const uint32_t info = (uint32_t)__builtin_amdgcn_readfirstlane(cur.r1);   // PAR < 16 leaves
        cur = nxt;
        const bool split = op_split(code, n, wpg, GMEM);
        if (wpg > 1 && (split || prev_split)) __syncthreads();
        if (tracer) trace[2 + oi] = __builtin_readcyclecounter();
        prev_split = split;
        if constexpr (GMEM) {
            if (code == OP_WOPEN || code == OP_WFLUSH) {
                // open: clear the window (bits start at 0); flush: copy it to the HBM bits
                if (wi == lead) {
                    c.wd0 = pos >> 4;
                    lds_u32 *const w = c.wl(c.wd0);
                    if (code == OP_WOPEN) {
#pragma unroll
                        for (int j = 0; j < c.win; j++) w[j * 64] = 0u;
                    } else {
                        for (int j0 = 0; j0 < c.win; j0 += 16) {
                            uint32_t t[16];   // 16 LDS reads in flight, then the HBM stores
#pragma unroll
                            for (int j = 0; j < 16; j++) t[j] = w[(j0 + j) * 64];
#pragma unroll
                            for (int j = 0; j < 16; j++) c.hbit[(c.wd0 + j0 + j) * 64] = t[j];
                        }
                    }
                }
                win_d0 = code == OP_WOPEN ? (pos >> 4) : -1;
                continue;
            }
            c.wd0 = flag ? win_d0 : -1;
        }
        if (!split && wi != lead) continue;
        // this wave's share of a split op (whole op otherwise)
        const int i0 = split ? (n * wi) >> lw : 0;
        const int i1 = split ? (n * (wi + 1)) >> lw : n;
        switch (code) {
        case OP_F: op_fg<false>(c, k, n, -1, i0, i1, fb); break;
        case OP_G: op_fg<true>(c, k, n, upos, i0, i1, fb); break;
        case OP_FLEAF: op_leaf<false>(c, k, pos, -1, fb, info); break;
        case OP_GLEAF: op_leaf<true>(c, k, pos, upos, fb, info); break;
        case OP_REP: op_rep(c, k, n, pos); break;
        case OP_R1: op_r1spc<false>(c, k, n, upos, pos, i0, i1); break;
        case OP_SPC:
            if (split) {
                // at most SPC_XWAVES waves (0 .. xw-1 counted from the lead) take n / xw words each
                const int xw = wpg < SPC_XWAVES ? wpg : SPC_XWAVES;
                const int xi = (wi - lead) & (wpg - 1);
                if (xi < xw) op_r1spc<true>(c, k, n, upos, pos, (n / xw) * xi, (n / xw) * (xi + 1), xw, xi);
                else __syncthreads();   // the exchange barrier of the split
            } else {
                op_r1spc<true>(c, k, n, upos, pos, 0, n);
            }
            break;
        case OP_H: op_h<false>(c, pos, n, i0 >> 4, i1 >> 4); break;
        case OP_H0: op_h<true>(c, pos, n, i0 >> 4, i1 >> 4); break;
        case OP_PLEAF: op_pleaf(c, k, pos, (fb >> 16) & 7u); break;
#if POLAR_SC_SUBS
        case OP_SUB:
            // a whole subtree as generated straight-line code (hybrid plans, polar_sc_jit.cpp):
            // its root words are in the level-k stage slot in LDS, its bits go to `pos`
            // (in lslot_t units for GMEM plans, dwords otherwise)
            if constexpr (GMEM)
                polar_sub_call(c, (int)fb, (int)(c.ls - (lds_slot *)smem) + (c.lvl_off(k) - c.lds0) * 64, pos);
            else
                polar_sub_call(c, (int)fb, (int)(c.lb - (lds_u32 *)smem) + c.lvl_off(k) * 64, pos);
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

// ---------------------------------------------------------------------------------------
// Grid tier (large N, hybrid plans): one F or G record of an upper-level node for every frame
// group at once. Wave w of the grid takes words [cw*j, cw*j + cw) of group w / chunks (j =
// w % chunks), so one group's wide op spans many CUs instead of the 8 waves of its block; the
// segments of the schedule between these launches run in the hybrid kernel (OP_SEGEND /
// OP_SEGCONT). Sources and destinations are HBM levels (nodes wider than the LDS region).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void tier_body(const chan_t *__restrict__ llr, uint32_t *__restrict__ scratch, int N,
                                          int batch, int group_dwords, int lds0, int code, int k, int n, int upos,
                                          uint32_t fb, int cw)
{
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
    const int chunks = (n + cw - 1) / cw;
    const long group = wave / chunks;
    const int j = wave - (int)group * chunks;
    if (group * 8 >= batch) return;
    const int G = N >> 4;
    const int row = lane >> 4;
    Ctx<true> c;
    c.G = G;
    c.nslot = (uint32_t)(G - 1);
    c.lds0 = lds0;
    c.wd0 = -1;
    c.lb = nullptr;
    c.ls = nullptr;
    c.lw = nullptr;
    c.win = (G - lds0) >> 4;
    uint32_t *const gbase = scratch + (size_t)group * (size_t)group_dwords;
    c.hs = (slot_t *)gbase + lane;
    c.hbit = gbase + (size_t)lds0 * (SLOT16 ? 64 : 32) + lane;
    const long f_lo = group * 8 + row, f_hi = group * 8 + 4 + row;
    const long f_lo_c = f_lo < batch ? f_lo : (long)batch - 1;
    const long f_hi_c = f_hi < batch ? f_hi : (long)batch - 1;
    c.ln.init((uint32_t)(lane & 15));
    c.llr_lo = llr + (size_t)f_lo_c * (size_t)N + c.ln.pos;
    c.llr_hi = llr + (size_t)f_hi_c * (size_t)N + c.ln.pos;
    const int i0 = j * cw, i1 = i0 + cw < n ? i0 + cw : n;
    const int w = fb_width(fb);
    if (code == OP_G) {
        if (k == 0) fg_words<true, true, false, false, false>(c, k, n, upos, i0, i1, w);
        else fg_words<true, false, false, false, false>(c, k, n, upos, i0, i1, w);
    } else {
        if (k == 0) fg_words<false, true, false, false, false>(c, k, n, -1, i0, i1, w);
        else fg_words<false, false, false, false, false>(c, k, n, -1, i0, i1, w);
    }
}

}  // namespace polar
