// polar_sc_pair.h -- the frame-pair layout of the large-N decode kernels (CDNA4, gfx950).
// Included by the generated source of pair plans (polar_sc_pairgen.cpp, hipRTC). No standard
// headers: hipRTC-clean.
//
// Why a second layout. The per-mask kernel (polar_sc_jit.cpp) puts 8 frames in a wave: the
// four 16-lane DPP rows hold four frame pairs, every register one 16-LLR word of each. That
// maximises work per instruction, which is what a 65536-frame batch of N = 1024 needs. For long
// codes (N = 65536 .. 524288, hundreds to a few thousand frames per GPU) the decode is
// latency-bound instead: the successive-cancellation schedule is a serial chain per frame and
// one wave issues a VALU instruction about every 5 cycles. Here one wave holds
// ONE frame pair (the 16-bit halves) and its four rows hold four consecutive words of the same
// node: register j of a node of w >= 4 words has word 4 j + r in row r. A stage op on n words
// is n / 4 instructions instead of n, the serial chain of a frame pair is ~4x shorter, and a
// batch gives 4x more independent waves.
//
//   * lane (row r, pl) holds position lane_pos(pl) (POLAR_LANE_REMAP, polar_sc_device.h) of
//     word 4 j + r of frames 2 p (low 16-bit half) and 2 p + 1 (high half);
//   * nodes of 2 words keep word (r & 1) in row r, nodes of 1 word are replicated in all rows
//     (the children of a 4-word node come out of one v_permlane32_swap, those of a 2-word
//     node out of one v_permlane16_swap: both operands of the F / G at once, no select);
//   * partial sums (bit_mem): per lane, "local word" l = w / 4 of row r; dword d holds local
//     words 16 d .. 16 d + 15 (bit j low frame, bit 16 + j high frame);
//   * upper levels (nodes wider than the register-resident subtree of S words): one stage
//     slot per level, a slot row = 64 lanes x u16 (SM8 pairs: low / high frame byte) = 4 words
//     of the pair; levels of nodes <= lds_words words sit in LDS, wider ones in HBM scratch.
#pragma once

#include "polar_sc_device.h"

namespace polar {

typedef unsigned short u16;
typedef __attribute__((address_space(3))) u16 lds_u16;
typedef __attribute__((address_space(3))) u32 lds_w32;

// ---------------------------------------------------------------------------------------
// cross-row exchange (gfx950 v_permlane16_swap_b32 / v_permlane32_swap_b32 with both
// operands the same register)
// ---------------------------------------------------------------------------------------
struct X2 {
    u32 a, b;
};
// rows (x0, x1, x2, x3) -> a = (x0, x0, x2, x2), b = (x1, x1, x3, x3)
__device__ __forceinline__ X2 swap16(u32 x)
{
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return X2{(u32)r[0], (u32)r[1]};
}
// rows (x0, x1, x2, x3) -> a = (x0, x1, x0, x1), b = (x2, x3, x2, x3)
__device__ __forceinline__ X2 swap32(u32 x)
{
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return X2{(u32)r[0], (u32)r[1]};
}
// the four row values of a register in every lane: t[r] = x of row r
struct X4 {
    u32 t0, t1, t2, t3;
};
__device__ __forceinline__ X4 rows4(u32 x)
{
    const X2 p = swap16(x);           // (x0 x0 x2 x2), (x1 x1 x3 x3)
    const X2 q0 = swap32(p.a), q1 = swap32(p.b);
    return X4{q0.a, q1.a, q0.b, q1.b};
}

// per-lane selection helpers of the generated code (one spelling that the CPU emulation of
// the generated source, tests/pair_emu.py, reads too)
__device__ __forceinline__ u32 sel(bool c, u32 a, u32 b) { return c ? a : b; }
__device__ __forceinline__ bool land(bool a, bool b) { return a && b; }
__device__ __forceinline__ u32 row_even(u32 row) { return (row & 1u) ? 0u : 0xFFFFFFFFu; }   // rows 0, 2
__device__ __forceinline__ u32 row_lo2(u32 row) { return row < 2u ? 0xFFFFFFFFu : 0u; }       // rows 0, 1

// ---------------------------------------------------------------------------------------
// per-pair context
// ---------------------------------------------------------------------------------------
constexpr int PAIR_MAX_WAVES = 8;   // launch bound 512 threads: <= 256 VGPRs per wave

struct PairCtx {
    const unsigned char *chl, *chh;   // channel bytes at this lane's position, frames lo / hi
    u16 *hs;                          // HBM stage slots of the pair (lane offset included)
    lds_u16 *ls;                      // LDS stage slots [lds_row0, ..) (lane offset included)
    u32 *hb;                          // HBM partial-sum dwords of the pair (lane offset included)
    lds_w32 *lx;                      // LDS exchange area: 3 dwords x waves (lane offset included)
    int G;                            // 16-LLR words per frame
    int lds_row0;                     // first slot row held in LDS
    int wi, W;                        // wave index in the pair's workgroup, waves
    int row;                          // DPP row 0..3
    bool lead;                        // the wave that runs the serial ops
    Lanes ln;
    // first slot row of level k (a node of G >> k words), k >= 1
    __device__ __forceinline__ int lvl_row(int k) const { return (G - (G >> (k - 1))) >> 2; }
    __device__ __forceinline__ bool in_lds(int r) const { return r >= lds_row0; }
    template <bool L>
    __device__ __forceinline__ u32 ld(int r) const
    {
        if constexpr (L) return slot_unpack((u32)ls[(r - lds_row0) * 64]);
        else return slot_unpack((u32)hs[r * 64]);
    }
    template <bool L>
    __device__ __forceinline__ void st(int r, u32 v) const
    {
        if constexpr (L) ls[(r - lds_row0) * 64] = (u16)slot_pack(v);
        else hs[r * 64] = (u16)slot_pack(v);
    }
    // raw slot row r (SM8 pair) through a generic pointer (subtree roots)
    __device__ __forceinline__ const u16 *slot_ptr(int r) const
    {
        return in_lds(r) ? (const u16 *)(ls + (r - lds_row0) * 64) : hs + r * 64;
    }
    // channel register j of the root: words 4 j + row of both frames (wrapper_in + qconv_format)
    __device__ __forceinline__ u32 chan(int j) const
    {
        return conv_pair((u32)chl[64 * j] | ((u32)chh[64 * j] << 16));
    }
    __device__ __forceinline__ u32 bld(int d) const { return hb[d * 64]; }
    __device__ __forceinline__ void bst(int d, u32 v) const { hb[d * 64] = v; }
    __device__ __forceinline__ void sync() const
    {
        if (W > 1) __syncthreads();
    }
};

// bits of local words [l0, l0 + cnt) (cnt <= 16, inside one dword) := acc (bit j = word l0 + j
// at bit position (l0 + j) % 16, both halves)
__device__ __forceinline__ void pbits_put(const PairCtx &c, int l0, int cnt, u32 acc)
{
    if (cnt >= 16) {
        c.bst(l0 >> 4, acc);
    } else {
        const u32 m = ((1u << cnt) - 1u) << (l0 & 15), mm = m | (m << 16);
        c.bst(l0 >> 4, (c.bld(l0 >> 4) & ~mm) | (acc & mm));
    }
}

// partial-sum flag (bits 15 / 31) of local word q from its dword
__device__ __forceinline__ u32 ubit_p(u32 dword, int q) { return (dword << (15 - (q & 15))) & SGN; }

// ---------------------------------------------------------------------------------------
// upper-level ops (nodes wider than the register-resident subtrees): loops over slot rows,
// split over the W waves of the pair in contiguous row ranges
// ---------------------------------------------------------------------------------------
// F_STATE / G_STATE word loops (my_module.h:373-445, 704-781): dst[j] = F(src[j], src[n4 + j])
// or G(src[j], src[n4 + j], bit_mem[local word ub + j]) for rows j in [j0, j1)
template <bool ISG, bool ROOT, bool SL, bool DL>
__device__ __forceinline__ void pfg_rows(const PairCtx &c, int s0, int d0, int n4, int ub, int j0, int j1)
{
    auto src = [&](int j) -> u32 {
        if constexpr (ROOT) return c.chan(j);
        else return c.template ld<SL>(s0 + j);
    };
    // rows per batch: HBM sources keep 2 x 32 row loads in flight (a lone wave per SIMD pair
    // hides the HBM latency only with many loads outstanding), LDS sources 2 x 8
    constexpr int CH = (ROOT || !SL) ? 32 : 8;
    int j = j0;
    for (; j + CH <= j1; j += CH) {
        u32 a[CH], b[CH], r[CH];
#pragma unroll
        for (int t = 0; t < CH; t++) {
            a[t] = src(j + t);
            b[t] = src(n4 + j + t);
        }
        if constexpr (ISG) {
            u32 u0 = 0, u1 = 0;
            if (ub >= 0) {
                u0 = c.bld((ub + j) >> 4);
                u1 = c.bld((ub + j + CH - 1) >> 4);
            }
#pragma unroll
            for (int t = 0; t < CH; t++) {
                const int q = ub + j + t;
                const u32 u = ub >= 0 ? ubit_p((((q >> 4) == ((ub + j) >> 4)) ? u0 : u1), q) : 0u;
                r[t] = G_sm<GSAT>(a[t], b[t], u);
            }
        } else {
#pragma unroll
            for (int t = 0; t < CH; t++) r[t] = F_sm(a[t], b[t]);
        }
#pragma unroll
        for (int t = 0; t < CH; t++) c.template st<DL>(d0 + j + t, r[t]);
    }
    for (; j < j1; j++) {
        const u32 a = src(j), b = src(n4 + j);
        u32 r;
        if constexpr (ISG) r = G_sm<GSAT>(a, b, ub >= 0 ? ubit_p(c.bld((ub + j) >> 4), ub + j) : 0u);
        else r = F_sm(a, b);
        c.template st<DL>(d0 + j, r);
    }
}

// F / G of the node at level k (its words in slot level k, the channel for k = 0) into the
// slot of level k + 1: n4 = output rows (n / 4), ub = local word of the partial sums or -1
template <bool ISG>
__device__ __forceinline__ void pop_fg(const PairCtx &c, int k, int n4, int ub, int j0, int j1)
{
    const int d0 = c.lvl_row(k + 1);
    const bool dl = c.in_lds(d0);
    if (k == 0) {
        if (dl) pfg_rows<ISG, true, false, true>(c, 0, d0, n4, ub, j0, j1);
        else pfg_rows<ISG, true, false, false>(c, 0, d0, n4, ub, j0, j1);
    } else {
        const int s0 = c.lvl_row(k);
        if (c.in_lds(s0)) pfg_rows<ISG, false, true, true>(c, s0, d0, n4, ub, j0, j1);
        else if (dl) pfg_rows<ISG, false, false, true>(c, s0, d0, n4, ub, j0, j1);
        else pfg_rows<ISG, false, false, false>(c, s0, d0, n4, ub, j0, j1);
    }
}
template <bool ISG>
__device__ __noinline__ void pop_fg_split(const PairCtx &c, int k, int n4, int ub)
{
    pop_fg<ISG>(c, k, n4, ub, (n4 * c.wi) / c.W, (n4 * (c.wi + 1)) / c.W);
}

// source word pair of a pruned-node op (REP / R1 / SPC): row j of the parent's two halves
template <bool ROOT, bool SL>
__device__ __forceinline__ void psrc2(const PairCtx &c, int s0, int n4, int j, u32 &a, u32 &b)
{
    if constexpr (ROOT) {
        a = c.chan(j);
        b = c.chan(n4 + j);
    } else {
        a = c.template ld<SL>(s0 + j);
        b = c.template ld<SL>(s0 + n4 + j);
    }
}

// F_REP_STATE (my_module.h:1292-1390) over n4 rows = n words: the exact pair tree of every
// word (ADD_TREE_16), accumulated over the words IN ORDER (word 4 j + r) by the saturating
// adder (511); x = all sign(acc). Two's-complement value chain, the exact SM chain only when
// some frame ends on a zero total (polar_sc_device.h rep_acc). One wave (the chain is serial).
template <bool ROOT, bool SL>
__device__ __forceinline__ void prep_body(const PairCtx &c, int s0, int n4, int l0)
{
    u32 acc = 0;
    for (int j = 0; j < n4; j++) {
        u32 a, b;
        psrc2<ROOT, SL>(c, s0, n4, j, a, b);
        const u32 lam = F_sm(a, b), sg = pk_sra(lam, 15);
        const X4 t = rows4(row_sum_biased(pk_add(pk_sub((lam & MAG) ^ sg, sg), 0x02000200u)));
        acc = rep_acc(rep_acc(rep_acc(rep_acc(acc, t.t0), t.t1), t.t2), t.t3);
    }
    if (rep_any_zero(acc)) {
        acc = 0;
        for (int j = 0; j < n4; j++) {
            u32 a, b;
            psrc2<ROOT, SL>(c, s0, n4, j, a, b);
            const X4 t = rows4(row_add_tree(F_sm(a, b), c.ln));
            acc = G_sm<REPSAT>(t.t0, acc, 0u);
            acc = G_sm<REPSAT>(t.t1, acc, 0u);
            acc = G_sm<REPSAT>(t.t2, acc, 0u);
            acc = G_sm<REPSAT>(t.t3, acc, 0u);
        }
    }
    const u32 full = pk_sra(acc, 15);   // two's complement or SM16: the decision is bit 15 / 31
    for (int l = 0; l < n4; l += 16) pbits_put(c, l0 + l, n4 - l < 16 ? n4 - l : 16, full);
}
__device__ __noinline__ void pop_rep(const PairCtx &c, int k, int n4, int l0)
{
    if (k == 0) prep_body<true, false>(c, 0, n4, l0);
    else if (c.in_lds(c.lvl_row(k))) prep_body<false, true>(c, c.lvl_row(k), n4, l0);
    else prep_body<false, false>(c, c.lvl_row(k), n4, l0);
}

// G_R1_STATE (my_module.h:1571-1642) / G_SPC_STATE (my_module.h:1737-1842) over rows [j0, j1)
// (whole partial-sum dwords per wave): lambda = G(parent, bits), x = sign(lambda); SPC: the
// parity of x over the node and the first minimum (|lambda|, word, bitrev4(position)) -- the
// Min_Mask tournament plus the strict '<' across words -- flipped when the parity is odd.
// The waves' partials meet in the LDS exchange area; the lead wave flips.
template <bool SPC, bool ROOT, bool SL>
__device__ __forceinline__ void pr1spc_body(const PairCtx &c, int s0, int n4, int ub, int l0, int j0, int j1,
                                            bool part)
{
    u32 acc = 0, par = 0, klo = 0xFFFFFFFFu, khi = 0xFFFFFFFFu, ud = 0;
    for (int j = j0; j < j1; j++) {
        u32 a, b;
        psrc2<ROOT, SL>(c, s0, n4, j, a, b);
        u32 u = 0;
        if (ub >= 0) {
            if (j == j0 || ((ub + j) & 15) == 0) ud = c.bld((ub + j) >> 4);
            u = ubit_p(ud, ub + j);
        }
        const u32 lam = G_sm<GSAT>(a, b, u), h = lam & SGN;
        const int q = (l0 + j) & 15;
        acc |= h >> (15 - q);
        if (q == 15 || j + 1 == j1) {
            const int first = ((l0 + j) & ~15) > l0 + j0 ? ((l0 + j) & ~15) : l0 + j0;
            pbits_put(c, first, l0 + j + 1 - first, acc);
            acc = 0;
        }
        if constexpr (SPC) {
            par ^= h;
            const u32 wk = (u32)(4 * j + c.row) << 4;   // word index in the node
            klo = __builtin_elementwise_min(klo, ((lam & 0xFFu) << 24) | wk);
            khi = __builtin_elementwise_min(khi, (((lam >> 16) & 0xFFu) << 24) | wk);
        }
    }
    if constexpr (SPC) {
        par = row_xor(par);
        klo = row_min_u32(klo | c.ln.br);
        khi = row_min_u32(khi | c.ln.br);
        {   // across the four rows
            X2 p = swap16(par);
            par = p.a ^ p.b;
            p = swap32(par);
            par = p.a ^ p.b;
            X2 a = swap16(klo), b = swap16(khi);
            klo = __builtin_elementwise_min(a.a, a.b);
            khi = __builtin_elementwise_min(b.a, b.b);
            a = swap32(klo);
            b = swap32(khi);
            klo = __builtin_elementwise_min(a.a, a.b);
            khi = __builtin_elementwise_min(b.a, b.b);
        }
        if (c.W > 1) {   // across the waves of the pair
            lds_w32 *const x = c.lx;
            x[(3 * c.wi) * 64] = part ? par : 0u;
            x[(3 * c.wi + 1) * 64] = part ? klo : 0xFFFFFFFFu;
            x[(3 * c.wi + 2) * 64] = part ? khi : 0xFFFFFFFFu;
            __syncthreads();
            if (!c.lead) return;
            par = 0;
            klo = khi = 0xFFFFFFFFu;
            for (int w = 0; w < c.W; w++) {
                par ^= x[(3 * w) * 64];
                klo = __builtin_elementwise_min(klo, (u32)x[(3 * w + 1) * 64]);
                khi = __builtin_elementwise_min(khi, (u32)x[(3 * w + 2) * 64]);
            }
        }
        // the flipped word: 4 (key >> 6) + ((key >> 4) & 3), position bitrev4^-1(key & 15)
        const bool flo = (par & 0x8000u) && (klo & 15u) == c.ln.br && (int)((klo >> 4) & 3u) == c.row;
        const bool fhi = (par & 0x80000000u) && (khi & 15u) == c.ln.br && (int)((khi >> 4) & 3u) == c.row;
        if (flo) {
            const int l = l0 + (int)((klo >> 6) & 0x3FFFFu);
            c.bst(l >> 4, c.bld(l >> 4) ^ (1u << (l & 15)));
        }
        if (fhi) {
            const int l = l0 + (int)((khi >> 6) & 0x3FFFFu);
            c.bst(l >> 4, c.bld(l >> 4) ^ (0x10000u << (l & 15)));
        }
    }
}
template <bool SPC>
__device__ __noinline__ void pop_r1spc(const PairCtx &c, int k, int n4, int ub, int l0)
{
    // whole dwords per wave (n4 is a multiple of 16 above the subtrees of >= 64 words)
    const int nd = (n4 + 15) >> 4;
    const int d0 = (nd * c.wi) / c.W, d1 = (nd * (c.wi + 1)) / c.W;
    const int j0 = 16 * d0 < n4 ? 16 * d0 : n4, j1 = 16 * d1 < n4 ? 16 * d1 : n4;
    const bool part = j1 > j0;
    if (!SPC && !part) return;
    if (k == 0) pr1spc_body<SPC, true, false>(c, 0, n4, ub, l0, j0, j1, part);
    else if (c.in_lds(c.lvl_row(k))) pr1spc_body<SPC, false, true>(c, c.lvl_row(k), n4, ub, l0, j0, j1, part);
    else pr1spc_body<SPC, false, false>(c, c.lvl_row(k), n4, ub, l0, j0, j1, part);
}

// H_STATE / H0_STATE (my_module.h:903-932, 1020-1042) on local words [l0, l0 + n4) and
// [l0 + n4, l0 + 2 n4): whole dwords split over the waves
template <bool H0>
__device__ __noinline__ void pop_h(const PairCtx &c, int l0, int n4)
{
    if (n4 >= 16) {
        const int nd = n4 >> 4, da = l0 >> 4, db = (l0 + n4) >> 4;
        const int e0 = (nd * c.wi) / c.W, e1 = (nd * (c.wi + 1)) / c.W;
        int e = e0;
        for (; e + 8 <= e1; e += 8) {
            u32 a[8], b[8];
#pragma unroll
            for (int t = 0; t < 8; t++) {
                b[t] = c.bld(db + e + t);
                a[t] = H0 ? 0u : c.bld(da + e + t);
            }
#pragma unroll
            for (int t = 0; t < 8; t++) c.bst(da + e + t, a[t] ^ b[t]);
        }
        for (; e < e1; e++) c.bst(da + e, (H0 ? 0u : c.bld(da + e)) ^ c.bld(db + e));
    } else if (c.lead) {
        const u32 m = ((1u << n4) - 1u) << (l0 & 15), mm = m | (m << 16);
        const u32 d = c.bld(l0 >> 4), sh = (d >> n4) & mm;
        c.bst(l0 >> 4, H0 ? ((d & ~mm) | sh) : (d ^ sh));
    }
}

// END (my_module.h:1848-1869) + wrapper_out: the partial sums of every local word, transposed
// inside each row (lane j of row r: the 16 position bits of local word 16 d + j = word
// 4 (16 d + j) + r), stored as u16 words in natural order
__device__ __noinline__ void pair_out(const PairCtx &c, unsigned short *o_lo, unsigned short *o_hi, bool st_lo,
                                         bool st_hi, int out_stride)
{
    const int nd = c.G >> 6;   // dwords per lane (G / 4 local words)
    const int e0 = (nd * c.wi) / c.W, e1 = (nd * (c.wi + 1)) / c.W;
    for (int d = e0; d < e1; d++) {
        const u32 t = row_transpose16(to_position_order(c.bld(d), c.ln), c.ln);
        const int w = 4 * (16 * d + (int)c.ln.pl) + c.row;
        if (st_lo) o_lo[w] = (unsigned short)(t & 0xFFFFu);
        if (st_hi) o_hi[w] = (unsigned short)(t >> 16);
    }
    if (c.lead)
        for (int w = c.G + (int)c.ln.pl + 16 * c.row; w < out_stride; w += 64) {   // pad words
            if (st_lo) o_lo[w] = 0;
            if (st_hi) o_hi[w] = 0;
        }
}

// the pair's storage: HBM scratch of `pair_dwords` per pair = slot rows (128 B each) then
// the partial-sum dwords (256 B rows); LDS: slot rows [lds_row0, total) then the SPC exchange
__device__ __forceinline__ bool pair_init(PairCtx &c, const signed char *llr, unsigned int *scratch, int N, int batch,
                                          long pair, int pair_dwords, int slot_rows, int lds_row0, int wi, int W,
                                          lds_u16 *lbase)
{
    const int lane = threadIdx.x & 63;
    c.G = N >> 4;
    c.row = lane >> 4;
    c.ln.init((u32)(lane & 15));
    c.wi = wi;
    c.W = W;
    c.lead = wi == 0;
    c.lds_row0 = lds_row0;
    const long f_lo = 2 * pair, f_hi = 2 * pair + 1;
    const long fl = f_lo < batch ? f_lo : (long)batch - 1, fh = f_hi < batch ? f_hi : (long)batch - 1;
    const int off = 16 * c.row + (int)c.ln.pos;
    c.chl = (const unsigned char *)llr + fl * (long)N + off;
    c.chh = (const unsigned char *)llr + fh * (long)N + off;
    unsigned int *base = scratch + pair * (long)pair_dwords;
    c.hs = (u16 *)base + lane;
    c.hb = base + (slot_rows >> 1) * 64 + lane;   // slot_rows x 128 B = slot_rows / 2 dword rows
    c.ls = lbase + lane;
    c.lx = (lds_w32 *)(lbase + (slot_rows > lds_row0 ? slot_rows - lds_row0 : 0) * 64) + lane;
    return f_lo < batch;
}

// Grid tier of pair plans: one F / G record of an upper-level node for every frame pair at
// once (HBM levels only); wave w takes rows [cw j, cw j + cw) of pair w / chunks
__device__ __forceinline__ void pair_tier_body(const signed char *llr, unsigned int *scratch, int N, int batch,
                                               int pair_dwords, int slot_rows, int code_g, int k, int n4, int ub,
                                               int cw)
{
    const int wave = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
    const int chunks = (n4 + cw - 1) / cw;
    const long pair = wave / chunks;
    const int j = wave - (int)pair * chunks;
    if (2 * pair >= batch) return;
    PairCtx c;
    pair_init(c, llr, scratch, N, batch, pair, pair_dwords, slot_rows, slot_rows, 0, 1, nullptr);
    const int j0 = j * cw, j1 = j0 + cw < n4 ? j0 + cw : n4;
    if (code_g) pop_fg<true>(c, k, n4, ub, j0, j1);
    else pop_fg<false>(c, k, n4, ub, j0, j1);
}

}  // namespace polar
