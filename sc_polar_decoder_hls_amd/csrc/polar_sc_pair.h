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
//     slot per level; a slot row = 4 words of the pair, stored by row pairs: the slot dword of
//     rows 2 i, 2 i + 1 of a lane holds the SM8 bytes (row 2 i frame lo, row 2 i + 1 lo, row 2 i
//     hi, row 2 i + 1 hi), and the four dwords of row pairs 4 g .. 4 g + 3 of a lane are
//     contiguous (16 B per lane, 1 KB per group of 8 rows: one dwordx4 / b128 access per lane);
//     levels of nodes <= lds_words words sit in LDS, wider ones in HBM scratch. The upper F / G run on those four bytes at once (SWAR
//     below) while two magnitudes fit 7 bits (Q <= 7).
//
// Solo layout (POLAR_SOLO 1, polar_sc_tuning.layout = 2): ONE frame per wave. The two 16-bit
// halves carry the two interleaved halves of the frame's nodes instead of two frames: register
// j of a node of w >= 8 words has word 8 j + 4 h + r in row r, half h. For nodes of >= 16 words
// F / G / H / R1 pair word 8 j + 4 h + r with 8 (j + w / 16) + 4 h + r -- same row, same half --
// so every loop below runs unchanged on "virtual frames" h of half the words (G = N / 32
// virtual words per half); an op on a node of n words is n / 8 instructions instead of n / 4.
// Only REP and SPC combine the halves (word order / tie order across h), and the channel rows
// (real words 8 j + 4 h + r: 128-byte row stride, half h at + 64) and the output differ.
// Nodes of 8 words and below are handled in the generated subtree code (polar_sc_pairgen.cpp).
//
// CA2 plans (POLAR_CA2, config.h:11): the same layout and code on magnitude + sign with the
// conventions of polar_sc_device.h (a zero's sign is don't-care; MIN = magnitude 2^(Q-1) with
// the sign set): slot values keep Q magnitude bits, the upper F takes the key min (MIN
// absorbing, F4 / F_pair), hard decisions mask zeros, REP needs no exact-SM fallback (a zero
// total decides 0). 8-bit LLRs keep 16-bit slot rows (|MIN| = 128 does not fit an SM8 byte).
#pragma once

#include "polar_sc_device.h"

#ifndef POLAR_SOLO
#define POLAR_SOLO 0
#endif

namespace polar {

constexpr bool PAIR_SOLO = POLAR_SOLO != 0;
// bytes between channel rows j and j + 1 of one (virtual) frame
constexpr unsigned ROWB = PAIR_SOLO ? 128u : 64u;

// rotate the 16-bit halves (solo: the other half of the frame's node, lane-local)
__device__ __forceinline__ u32 hswap(u32 x) { return __builtin_amdgcn_alignbit(x, x, 16); }
// the low / high half in both halves
__device__ __forceinline__ u32 bcast_lo(u32 x) { return __builtin_amdgcn_perm(x, x, 0x01000100u); }
__device__ __forceinline__ u32 bcast_hi(u32 x) { return __builtin_amdgcn_perm(x, x, 0x03020302u); }

typedef unsigned short u16;
typedef __attribute__((address_space(3))) u16 lds_u16;
typedef __attribute__((address_space(3))) u32 lds_w32;
typedef __attribute__((address_space(1))) u32 g_u32;
typedef __attribute__((address_space(1))) unsigned char g_u8;
typedef __attribute__((address_space(1))) unsigned short g_u16;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(1))) u32x4 g_u32x4;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;

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

// G_extended on split words (inside a PAR 64 word, functions.h Spec_P64_ext): G_split without
// the clamp -- magnitudes grow by at most one bit per level, far below the 15 of an SM16 half
template <int I>
__device__ __forceinline__ u32 G_split_x(u32 ma, u32 mb, u32 X, u32 &LT)
{
    const u32 xm = opaque(plane_mask<I>(X));
    const u32 d = pk_sub(ma, mb);
    LT = plane_put<I>(LT, d);
    return bsel(xm, pk_abs_i16(d), pk_add(ma, mb));
}

// PAR 64 (POLAR_LPAR 6): a PAR word is four device words = the four rows of one register of a
// node (and one slot row); PAR 32 (5): two device words = rows (0, 1) / (2, 3) of a register;
// PAR 16: one device word = one row
constexpr bool PAIR_P64 = LPAR == 6, PAIR_P32 = LPAR == 5;
static_assert(LPAR >= 2 && LPAR <= 6, "pair plans: PAR 4 .. 64");
__device__ __forceinline__ u32 bitrev2(u32 r) { return ((r & 1u) << 1) | (r >> 1); }
// SPC key bits below the register index (bits 0..5): the tie order of equal magnitudes inside a
// register -- PAR 16: (word = row, then bitrev4(position)); PAR 32: (PAR word row / 2, then
// bitrev5(position in it) = (bitrev4(position), row & 1)); PAR 64: bitrev6(position in the PAR
// word) = (bitrev4(position), then bitrev2(row)) (polar_sc_interp.h spc_word_key / spc_lane_key)
__device__ __forceinline__ u32 spc_sub(u32 row, const Lanes &ln)
{
    // PAR 4 / 8: (word = row, group, bitrev_{LPAR}(position in the group)), polar_sc_device.h
    // spc_lane_key
    if constexpr (LPAR < 4) return (row << 4) | spc_lane_key(ln);
    if constexpr (PAIR_P64) return (ln.br << 2) | bitrev2(row);
    else if constexpr (PAIR_P32) return ((row >> 1) << 5) | (ln.br << 1) | (row & 1u);
    else return (row << 4) | ln.br;
}
// the key bits of a lane inside one device word: bitrev4(position) (PAR >= 16), or (group,
// bitrev_{LPAR}(position in the group)) for PAR 4 / 8
__device__ __forceinline__ u32 spc_lk(const Lanes &ln)
{
    if constexpr (LPAR < 4) return spc_lane_key(ln);
    else return ln.br;
}
// the same for a node of two words (row r holds word r & 1): PAR 16 two PAR words, PAR 32 one
__device__ __forceinline__ u32 spc_sub2(u32 row, const Lanes &ln)
{
    return PAIR_P32 ? (ln.br << 1) | (row & 1u) : ((row & 1u) << 4) | spc_lk(ln);
}
// REP accumulation of one register's four row totals (row_sum_biased values, +8192 per half):
// PAR 16 -- four PAR words in order (word 4 i + row); PAR 32 -- two PAR words, the exact totals
// of rows (0, 1) and (2, 3); PAR 64 -- one PAR word, its exact total
__device__ __forceinline__ u32 rep_acc_rows(u32 acc, u32 t0, u32 t1, u32 t2, u32 t3)
{
    if constexpr (PAIR_P64) {
        const u32 t = pk_sub(pk_add(pk_add(t0, t1), pk_add(t2, t3)), 0x60006000u);   // 4 x 8192 -> 8192
        return rep_acc(acc, t);
    } else if constexpr (PAIR_P32) {
        acc = rep_acc(acc, pk_sub(pk_add(t0, t1), 0x20002000u));                      // 2 x 8192 -> 8192
        return rep_acc(acc, pk_sub(pk_add(t2, t3), 0x20002000u));
    } else {
        return rep_acc(rep_acc(rep_acc(rep_acc(acc, t0), t1), t2), t3);
    }
}
// PAR 4 / 8 (LPAR < 4): the PAR words of a device word are its lane groups. REP accumulates the
// exact pair tree of every group (ADD_TREE_{PAR}), groups in lane order within a word, words in
// order, in exact SM arithmetic with the REP clamp (the interpreter's rep_body, polar_sc_device.h
// group_chain). group_order: per lane the totals of groups 0 .. PPW - 1 of its own row's word.
// (templates on the group width PW = PARW, so that PAR >= 16 plans never instantiate them)
template <int PW>
__device__ __forceinline__ void group_order(u32 t, u32 gr, u32 *o)
{
    if constexpr (16 / PW == 2) {
        const u32 p = xorlane<PW>(t);
        o[0] = (gr & 1u) ? p : t;
        o[1] = (gr & 1u) ? t : p;
    } else {
        const u32 v1 = xorlane<PW>(t), v2 = xorlane<2 * PW>(t), v3 = xorlane<PW>(v2);
#pragma unroll
        for (u32 k = 0; k < 4; k++) {
            const u32 j = (gr & 3u) ^ k;
            o[k] = j == 0 ? t : j == 1 ? v1 : j == 2 ? v2 : v3;
        }
    }
}
// PAR 32 / 64 at PRUNING_LEVEL 1 (OP_PLEAF): the leaf decoder of the PAR word held by one
// register (PAR 64: row r = word r) or by a two-word node (PAR 32: row r = word r & 1) --
// R1 (5) / REP (1) / SPC (2) / REP2 (3) / SPC2 (4), R_STATE (my_module.h:566-593;
// library.h:187-280) as the interpreter's op_pleaf computes it: the word pair trees first
// (PAR 64: words (0, 2), (1, 3), then the halves; exact SM or CA2 sums), then the lane tree;
// SPC keys (|lambda|, bitrev_{LPAR}(16 j + position)). v: the SM16 / two's complement word
// per lane; returns sign-position flags.
template <int KIND>
__device__ __forceinline__ u32 pleaf_pair(u32 v, const Lanes &ln, u32 row)
{
    if constexpr (KIND == 5) {
        return v & SGN;
    } else if constexpr (KIND == 1 || KIND == 3) {
        u32 t = v;
        if constexpr (PAIR_P64) {
            const X2 q = swap32(t);
            t = CA2 ? pk_add(q.a, q.b) : G_sm<0>(q.a, q.b, 0u);
        }
        {
            const X2 q = swap16(t);
            t = CA2 ? pk_add(q.a, q.b) : G_sm<0>(q.a, q.b, 0u);
        }
        if constexpr (CA2) {
            t = pk_add(t, xorlane<8>(t));
            t = pk_add(t, xorlane<4>(t));
            t = pk_add(t, xorlane<2>(t));
            if constexpr (KIND == 1) t = pk_add(t, xorlane<1>(t));
            return t & SGN;
        } else if constexpr (KIND == 1) {
            return leaf_rep(t, ln);
        } else {
            return leaf_rep2(t, ln);
        }
    } else {
        constexpr bool spc2 = KIND == 4;
        u32 par = v & SGN;
        if constexpr (PAIR_P64) {
            const X2 q = swap32(par);
            par = q.a ^ q.b;
        }
        {
            const X2 q = swap16(par);
            par = q.a ^ q.b;
        }
        par ^= xorlane<8>(par);
        par ^= xorlane<4>(par);
        par ^= xorlane<2>(par);
        if constexpr (!spc2) par ^= xorlane<1>(par);
        const u32 mg = CA2 ? pk_add(ca2_qabs(v, QB), (1u << (QB - 1)) * 0x00010001u) : (v & MAG);
        const u32 wk = (ln.br << (LPAR - 4)) | bitrev_n(PAIR_P64 ? row : (row & 1u), LPAR - 4);
        const u32 mlo = ((mg & 0xFFFFu) << 8) | wk, mhi = ((mg >> 16) << 8) | wk;
        u32 klo = mlo, khi = mhi;
        if constexpr (PAIR_P64) {
            const X2 a = swap32(klo), b = swap32(khi);
            klo = __builtin_elementwise_min(a.a, a.b);
            khi = __builtin_elementwise_min(b.a, b.b);
        }
        {
            const X2 a = swap16(klo), b = swap16(khi);
            klo = __builtin_elementwise_min(a.a, a.b);
            khi = __builtin_elementwise_min(b.a, b.b);
        }
        klo = __builtin_elementwise_min(klo, xorlane<8>(klo));
        khi = __builtin_elementwise_min(khi, xorlane<8>(khi));
        klo = __builtin_elementwise_min(klo, xorlane<4>(klo));
        khi = __builtin_elementwise_min(khi, xorlane<4>(khi));
        klo = __builtin_elementwise_min(klo, xorlane<2>(klo));
        khi = __builtin_elementwise_min(khi, xorlane<2>(khi));
        if constexpr (!spc2) {
            klo = __builtin_elementwise_min(klo, xorlane<1>(klo));
            khi = __builtin_elementwise_min(khi, xorlane<1>(khi));
        }
        const u32 flo = klo == mlo ? (par & 0x8000u) : 0u;
        const u32 fhi = khi == mhi ? (par & 0x80000000u) : 0u;
        return (v & SGN) ^ flo ^ fhi;
    }
}

// the REP input of one register: F of the split operands as the word trees take it -- SM16, or
// (CA2) two's complement, with the key min and the MIN sign (MW > 0) on the leftmost path
template <int I, int MW>
__device__ __forceinline__ u32 F_split_rep(u32 ma, u32 mb, u32 FS)
{
    if constexpr (CA2) {
        if constexpr (MW > 0) {
            const u32 m = pk_min_key<MW>(ma, mb), sg = plane_mask<I>(FS) | pk_sra(ca2_minbit<MW>(m), 15);
            return pk_sub(m ^ sg, sg);
        } else {
            const u32 m = pk_min(ma, mb), sg = plane_mask<I>(FS);
            return pk_sub(m ^ sg, sg);
        }
    } else {
        return F_split_sm<I>(ma, mb, FS);
    }
}
// one register of a node (row r = word 4 i + r), acc the same in every lane
template <int PW = PARW>
__device__ __forceinline__ u32 rep_groups_rows(u32 acc, u32 lam, const Lanes &ln)
{
    u32 o[PPW > 1 ? PPW : 1];
    group_order<PW>(add_tree_w<PW, 1>(lam, ln), ln.pos >> LPAR, o);
    X4 r[PPW > 1 ? PPW : 1];
#pragma unroll
    for (int k = 0; k < PPW; k++) r[k] = rows4(o[k]);
#pragma unroll
    for (int k = 0; k < PPW; k++) acc = rep_sat_add(acc, r[k].t0);
#pragma unroll
    for (int k = 0; k < PPW; k++) acc = rep_sat_add(acc, r[k].t1);
#pragma unroll
    for (int k = 0; k < PPW; k++) acc = rep_sat_add(acc, r[k].t2);
#pragma unroll
    for (int k = 0; k < PPW; k++) acc = rep_sat_add(acc, r[k].t3);
    return acc;
}
// a node of two words (row r holds word r & 1) / of one word (replicated in the rows)
template <int PW = PARW>
__device__ __forceinline__ u32 rep_groups_2(u32 lam, const Lanes &ln)
{
    u32 o[PPW > 1 ? PPW : 1];
    group_order<PW>(add_tree_w<PW, 1>(lam, ln), ln.pos >> LPAR, o);
    X2 q[PPW > 1 ? PPW : 1];
#pragma unroll
    for (int k = 0; k < PPW; k++) q[k] = swap16(o[k]);
    u32 acc = 0u;
#pragma unroll
    for (int k = 0; k < PPW; k++) acc = rep_sat_add(acc, q[k].a);
#pragma unroll
    for (int k = 0; k < PPW; k++) acc = rep_sat_add(acc, q[k].b);
    return acc;
}
template <int PW = PARW>
__device__ __forceinline__ u32 rep_groups_1(u32 lam, const Lanes &ln)
{
    return group_chain<16 / PW>(0u, add_tree_w<PW, 1>(lam, ln), ln.pos >> LPAR);
}

// the exact SM chain (rep_any_zero fallback) over one register: SM16 per lane v (row r = word
// 4 i + r) -> the ADD_TREE of each PAR word (PAR 64: words (0, 2), (1, 3), then the halves,
// then the positions; PAR 32: words (0, 1), then the positions -- rep_add_tree's order),
// accumulated with the REP clamp
__device__ __forceinline__ u32 rep_sm_rows(u32 acc, u32 v, const Lanes &ln)
{
    if constexpr (PAIR_P64) {
        const X2 q = swap32(v);
        const u32 v1 = G_sm<0>(q.a, q.b, 0u);
        const X2 r = swap16(v1);
        return G_sm<REPSAT>(row_add_tree(G_sm<0>(r.a, r.b, 0u), ln), acc, 0u);
    } else if constexpr (PAIR_P32) {
        const X2 q = swap16(v);
        const X4 t = rows4(row_add_tree(G_sm<0>(q.a, q.b, 0u), ln));
        acc = G_sm<REPSAT>(t.t0, acc, 0u);
        return G_sm<REPSAT>(t.t2, acc, 0u);
    } else {
        const X4 t = rows4(row_add_tree(v, ln));
        acc = G_sm<REPSAT>(t.t0, acc, 0u);
        acc = G_sm<REPSAT>(t.t1, acc, 0u);
        acc = G_sm<REPSAT>(t.t2, acc, 0u);
        return G_sm<REPSAT>(t.t3, acc, 0u);
    }
}

// Solo layout: the REP chain of one register's words in order -- half 0 (words 8 j + r), then
// half 1 (8 j + 4 + r); the accumulator is the low half (the high half is don't-care)
__device__ __forceinline__ u32 rep_acc_solo(u32 acc, u32 t0, u32 t1, u32 t2, u32 t3)
{
    acc = rep_acc(rep_acc(rep_acc(rep_acc(acc, t0), t1), t2), t3);
    return rep_acc(rep_acc(rep_acc(rep_acc(acc, t0 >> 16), t1 >> 16), t2 >> 16), t3 >> 16);
}
__device__ __forceinline__ u32 rep_sm_solo(u32 acc, u32 v, const Lanes &ln)
{
    const X4 t = rows4(row_add_tree(v, ln));
    acc = G_sm<REPSAT>(t.t0, acc, 0u);
    acc = G_sm<REPSAT>(t.t1, acc, 0u);
    acc = G_sm<REPSAT>(t.t2, acc, 0u);
    acc = G_sm<REPSAT>(t.t3, acc, 0u);
    acc = G_sm<REPSAT>(t.t0 >> 16, acc, 0u);
    acc = G_sm<REPSAT>(t.t1 >> 16, acc, 0u);
    acc = G_sm<REPSAT>(t.t2 >> 16, acc, 0u);
    return G_sm<REPSAT>(t.t3 >> 16, acc, 0u);
}
// true if the (low-half) accumulator of some lane is zero
__device__ __forceinline__ bool rep_any_zero_lo(u32 acc)
{
    return __builtin_amdgcn_ballot_w64((acc & 0xFFFFu) == 0u) != 0ull;
}

// REP of a node of two words (row r holds word r & 1): the biased row sums t -> accumulator
// (PAR 16: two PAR words in order; PAR 32: one PAR word, its exact total)
__device__ __forceinline__ u32 rep2_acc(u32 t)
{
    const X2 q = swap16(t);
    if constexpr (PAIR_P32) return rep_acc(0u, pk_sub(pk_add(q.a, q.b), 0x20002000u));
    else return rep_acc(rep_acc(0u, q.a), q.b);
}
// its exact SM chain from the SM16 word per lane
__device__ __forceinline__ u32 rep2_sm(u32 v, const Lanes &ln)
{
    if constexpr (PAIR_P32) {
        const X2 r = swap16(v);
        return G_sm<REPSAT>(row_add_tree(G_sm<0>(r.a, r.b, 0u), ln), 0u, 0u);
    } else {
        const X2 r = swap16(row_add_tree(v, ln));
        return G_sm<REPSAT>(r.b, G_sm<REPSAT>(r.a, 0u, 0u), 0u);
    }
}

constexpr int PAIR_MAX_WAVES = 8;   // launch bound 512 threads: <= 256 VGPRs per wave

// ---------------------------------------------------------------------------------------
// slot dwords (row pairs, SM8 bytes lo_even, lo_odd, hi_even, hi_odd)
// ---------------------------------------------------------------------------------------
// row (odd ? 2 i + 1 : 2 i) of a slot dword as the SM16 pair of the register code
__device__ __forceinline__ u32 prow8(u32 d, bool odd)
{
    return __builtin_amdgcn_perm(d, d, odd ? 0x03030101u : 0x02020000u) & ((0x8000u | VMAG) * 0x00010001u);
}
// two SM16 pairs (rows 2 i, 2 i + 1) -> slot dword
__device__ __forceinline__ u32 ppack8(u32 v0, u32 v1)
{
    const u32 t0 = (v0 & (VMAG * 0x00010001u)) | ((v0 >> 8) & 0x00800080u);   // SM8 in bytes 0, 2
    const u32 t1 = (v1 & (VMAG * 0x00010001u)) | ((v1 >> 8) & 0x00800080u);
    return __builtin_amdgcn_perm(t1, t0, 0x06020400u);
}
// the partial sums of local words q .. q + 15 as one dword (bit i = word q + i of the low
// frame, bit 16 + i of the high frame) from the dwords d0 (words 16 (q / 16) ..) and d1 (the
// next 16)
__device__ __forceinline__ u32 ubits16(u32 d0, u32 d1, int q)
{
    const int o = q & 15;
    const u32 lo = ((d0 & 0xFFFFu) | (d1 << 16)) >> o, hi = ((d0 >> 16) | (d1 & 0xFFFF0000u)) >> o;
    return (lo & 0xFFFFu) | (hi << 16);
}
// partial-sum flags of local words q + k, q + k + 1 (k even) from ubits16(.., q) at the sign
// bits of the slot bytes (bits 7, 15, 23, 31; the other bits are don't-care: only sign bits
// are read)
// (k a constant after unrolling)
__device__ __forceinline__ u32 ubits4s(u32 d16, int k)
{
    const u32 y = (k <= 7 ? d16 << (7 - k) : d16 >> (k - 7)) & 0x01800180u;   // bits 7, 8, 23, 24
    return y | (y << 7);
}
// the same from a partial-sum dword and a run-time even q (bits q & 15, + 1 of it)
__device__ __forceinline__ u32 ubits4(u32 dword, int q)
{
    const u32 y = ((dword >> (q & 15)) & 0x00030003u) << 7;
    return y | (y << 7);
}

// SWAR on four SM8 bytes (sign bit 7, magnitude bits 0..6): exact while two magnitudes sum
// below 128 (CA2: |MIN| = 2^(Q-1) included, LLR_BITS <= 6)
constexpr bool PAIR_SWAR = 2u * (CA2 ? QMAG + 1u : QMAG) < 128u;
constexpr u32 B_SGN = 0x80808080u, B_MAG = 0x7F7F7F7Fu, B_ONE = 0x01010101u;
// 0x7F in the bytes whose bit 7 is set, 0 elsewhere
__device__ __forceinline__ u32 bmask7(u32 t)
{
    const u32 g = t & B_SGN;
    return g - (g >> 7);
}
__device__ __forceinline__ u32 bsel7(u32 m, u32 a, u32 b) { return (m & a) | (~m & b); }   // v_bfi
// F_sm on four bytes: min of the magnitudes, xor of the signs. CA2: F_function_C2 -- the min
// of the keys m ^ 2^(Q-1) (MIN -> key 0 wins), the sign set for MIN
__device__ __forceinline__ u32 F4(u32 a, u32 b)
{
    if constexpr (CA2) {
        constexpr u32 KB = (1u << (QB - 1)) * B_ONE;
        const u32 ka = (a & B_MAG) ^ KB, kb = (b & B_MAG) ^ KB;    // keys <= 2^Q - 1 < 128
        const u32 k = bsel7(bmask7((ka | B_SGN) - kb), kb, ka);   // min key
        return (((a ^ b) | ~(k + 0x7F7F7F7Fu)) & B_SGN) | (k ^ KB);   // bit 7 of k + 127: k != 0
    } else {
        const u32 ma = a & B_MAG, mb = b & B_MAG;
        const u32 ge = bmask7((ma | B_SGN) - mb);   // |a| >= |b|
        return ((a ^ b) & B_SGN) | bsel7(ge, mb, ma);
    }
}
// G_sm<GSAT> on four bytes; u: flip flags at the sign bits
__device__ __forceinline__ u32 G4(u32 a, u32 b, u32 u)
{
    constexpr u32 SATV = GSAT * B_ONE;
    const u32 ma = a & B_MAG, mb = b & B_MAG, x = a ^ b ^ u;   // x bit 7: sign(a') != sign(b)
    const u32 t1 = (ma | B_SGN) - mb, t2 = (mb | B_SGN) - ma;   // bit 7: |a| >= |b|, |b| >= |a|
    const u32 ad = bsel7(bmask7(t1), t1, t2);                  // | |a| - |b| | in bits 0..6
    u32 m = bsel7(bmask7(x), ad, ma + mb);                      // bit 7 clear
    m = bsel7(bmask7((m | B_SGN) - SATV), SATV, m);             // min(m, GSAT)
    return ((b ^ (x & t1)) & B_SGN) | m;                        // |a| < |b| ? sign(b) : sign(a')
}
// channel bytes (two's complement, low Q bits) -> SM8: conv_pair on four bytes; CA2: the
// value as magnitude + sign (MIN -> magnitude 2^(Q-1))
__device__ __forceinline__ u32 conv4(u32 raw)
{
    constexpr u32 QM = (1u << QB) - 1u, QP = 1u << QB;
    const u32 t = raw & (QM * B_ONE), v = QP * B_ONE - t;       // QP - t in [1, QP] per byte
    if constexpr (CA2) {
        const u32 sg = (t << (8 - QB)) & B_SGN;                   // bit Q-1 -> bit 7
        return sg | bsel7(bmask7(sg), v, t);
    } else {
        const u32 mn = bsel7(bmask7((t | B_SGN) - v), v, t);        // min(t, QP - t)
        return ((t + (127u - QP / 2u) * B_ONE) & B_SGN) | (mn & (QMAG * B_ONE));   // sign: t > QP / 2
    }
}
// F of two SM16 pairs of the stage width: F_sm, or F_function_C2 with MIN absorbing
__device__ __forceinline__ u32 F_pair(u32 a, u32 b)
{
    if constexpr (CA2) return F_ca2<QB>(a, b);
    else return F_sm(a, b);
}
// hard decisions (bits 15 / 31) of an SM16 pair: the signs; CA2: of the nonzero values
__device__ __forceinline__ u32 hard_pair(u32 v)
{
    if constexpr (CA2) return v & ca2_nz(v) & SGN;
    else return v & SGN;
}
// F / G of a slot dword pair (either arithmetic)
template <bool ISG>
__device__ __forceinline__ u32 fg4_8(u32 a, u32 b, u32 u)
{
    if constexpr (PAIR_SWAR) {
        if constexpr (ISG) return G4(a, b, u);
        else return F4(a, b);
    } else if constexpr (ISG) {
        return ppack8(G_sm<GSAT>(prow8(a, false), prow8(b, false), (u << 8) & SGN),
                      G_sm<GSAT>(prow8(a, true), prow8(b, true), u & SGN));
    } else {
        return ppack8(F_pair(prow8(a, false), prow8(b, false)), F_pair(prow8(a, true), prow8(b, true)));
    }
}

// ---------------------------------------------------------------------------------------
// slot formats. SM8 (LLR_BITS <= 8): a row pair (slot rows 2 i, 2 i + 1) is one dword of SM8
// bytes, an 8-row group 16 B per lane. SLOT16 (LLR_BITS 9, where the F magnitudes of the
// channel reach 255 and do not fit an SM8 byte): every slot row is the register format itself,
// one SM16 pair; a row pair is two dwords, an 8-row group 32 B per lane. The loops below see a
// row pair as su_t and an 8-row group as sg_t; u flags of a row pair keep the SM8 positions
// (bits 7 / 23 row 2 i, 15 / 31 row 2 i + 1, ubits4).
// ---------------------------------------------------------------------------------------
#if POLAR_Q > 8 || (POLAR_CA2 && POLAR_Q > 7)
#define POLAR_PAIR_S16 1
#else
#define POLAR_PAIR_S16 0
#endif
constexpr bool PAIR_S16 = POLAR_PAIR_S16 != 0;   // (9-bit LLRs; CA2 8-bit LLRs: |MIN| = 128)
constexpr int GD = PAIR_S16 ? 8 : 4;   // dwords per lane of an 8-row group
#if POLAR_Q > 8
typedef short chan_el;                 // int16 channel (polar_sc_decode_i16)
#else
typedef unsigned char chan_el;
#endif
#if POLAR_PAIR_S16
typedef u32x2 su_t;
typedef u32x8 sg_t;
__device__ __forceinline__ u32 prow(su_t d, bool odd) { return odd ? d.y : d.x; }
__device__ __forceinline__ su_t ppack(u32 v0, u32 v1) { return su_t{v0, v1}; }
__device__ __forceinline__ su_t sget(const sg_t &g, int t) { return su_t{g[2 * t], g[2 * t + 1]}; }
__device__ __forceinline__ void sset(sg_t &g, int t, su_t v)
{
    g[2 * t] = v.x;
    g[2 * t + 1] = v.y;
}
template <bool ISG>
__device__ __forceinline__ su_t fg4(su_t a, su_t b, u32 u)
{
    if constexpr (ISG) return su_t{G_sm<GSAT>(a.x, b.x, (u << 8) & SGN), G_sm<GSAT>(a.y, b.y, u & SGN)};
    else return su_t{F_pair(a.x, b.x), F_pair(a.y, b.y)};
}
#else
typedef u32 su_t;
typedef u32x4 sg_t;
__device__ __forceinline__ u32 prow(su_t d, bool odd) { return prow8(d, odd); }
__device__ __forceinline__ su_t ppack(u32 v0, u32 v1) { return ppack8(v0, v1); }
__device__ __forceinline__ su_t sget(const sg_t &g, int t) { return g[t]; }
__device__ __forceinline__ void sset(sg_t &g, int t, su_t v) { g[t] = v; }
template <bool ISG>
__device__ __forceinline__ su_t fg4(su_t a, su_t b, u32 u) { return fg4_8<ISG>(a, b, u); }
#endif
typedef __attribute__((address_space(1))) su_t g_su;
typedef __attribute__((address_space(3))) su_t lds_su;
typedef __attribute__((address_space(1))) sg_t g_sg;
typedef __attribute__((address_space(3))) sg_t lds_sg;
typedef __attribute__((address_space(1))) chan_el g_chan;

// ---------------------------------------------------------------------------------------
// per-pair context
// ---------------------------------------------------------------------------------------
// 14 registers: passed by value to the noinline upper-level functions (in registers; a
// reference would put it on the private stack). Global pointers carry address space 1 so that
// the loads and stores through them are global_*, not flat_*.
struct PairCtx {
    const g_chan *chl, *chh;          // channel LLRs at this lane's position, frames lo / hi
    g_u32 *hs;                        // HBM stage slots of the pair (lane offset 4 lane included)
    g_u32 *hb;                        // HBM partial-sum dwords of the pair (lane offset included)
    lds_w32 *ls;                      // LDS stage slots [lds_row0, ..) (lane offset 4 lane included)
    int lxo;                          // LDS exchange area (3 dwords x waves, dword per lane) offset
    int G;                            // 16-LLR words per frame
    int lds_row0;                     // first slot row held in LDS (even)
    int wi, W;                        // wave index in the pair's workgroup, waves
    __device__ __forceinline__ u32 row() const { return (threadIdx.x & 63u) >> 4; }   // DPP row
    __device__ __forceinline__ bool lead() const { return wi == 0; }   // runs the serial ops
    __device__ __forceinline__ Lanes lanes() const
    {
        Lanes ln;
        ln.init(threadIdx.x & 15u);
        return ln;
    }
    __device__ __forceinline__ lds_w32 *lx() const { return ls + lxo - 3 * (int)(threadIdx.x & 63u); }
    // first slot row of level k (a node of G >> k words), k >= 1 (even)
    __device__ __forceinline__ int lvl_row(int k) const { return (G - (G >> (k - 1))) >> 2; }
    __device__ __forceinline__ bool in_lds(int r) const { return r >= lds_row0; }
    // dword offset of slot row pair r / 2 (r even) from the lane's base
    static __device__ __forceinline__ int sofs(int r) { return (r >> 3) * 64 * GD + ((r >> 1) & 3) * (GD / 4); }
    // slot rows r, r + 1 (r even)
    template <bool L>
    __device__ __forceinline__ su_t ld2(int r) const
    {
        if constexpr (L) return *(const lds_su *)(ls + sofs(r - lds_row0));
        else return *(const g_su *)(hs + sofs(r));
    }
    // slot rows r .. r + 7 (r a multiple of 8)
    template <bool L>
    __device__ __forceinline__ sg_t ld8(int r) const
    {
        if constexpr (L) return *(const lds_sg *)(ls + ((r - lds_row0) >> 3) * 64 * GD);
        else return *(const g_sg *)(hs + (r >> 3) * 64 * GD);
    }
    template <bool L>
    __device__ __forceinline__ void st8(int r, sg_t v) const
    {
        if constexpr (L) *(lds_sg *)(ls + ((r - lds_row0) >> 3) * 64 * GD) = v;
        else *(g_sg *)(hs + (r >> 3) * 64 * GD) = v;
    }
    // the slot from row r on (r a multiple of 8) through a generic pointer (subtree roots)
    __device__ __forceinline__ const u32 *slot_ptr(int r) const
    {
        return in_lds(r) ? (const u32 *)(ls + ((r - lds_row0) >> 3) * 64 * GD) : (const u32 *)(hs + (r >> 3) * 64 * GD);
    }
    // channel rows j, j + 1 (j even) as a slot row pair (wrapper_in + qconv_format)
    __device__ __forceinline__ su_t chan2(int j) const
    {
#if POLAR_Q > 8
        const u32 r0 = (u32)(unsigned short)chl[ROWB * j] | ((u32)(unsigned short)chh[ROWB * j] << 16);
        const u32 r1 = (u32)(unsigned short)chl[ROWB * j + ROWB] | ((u32)(unsigned short)chh[ROWB * j + ROWB] << 16);
        return ppack(chan_sm16(r0), chan_sm16(r1));
#else
        const u32 lo = (u32)chl[ROWB * j] | ((u32)chl[ROWB * j + ROWB] << 8);
        const u32 hi = (u32)chh[ROWB * j] | ((u32)chh[ROWB * j + ROWB] << 8);
        const u32 raw = lo | (hi << 16);
        if constexpr (PAIR_SWAR) return conv4(raw);
        else return ppack(chan_sm16(raw & 0x00FF00FFu), chan_sm16((raw >> 8) & 0x00FF00FFu));
#endif
    }
    // channel rows j .. j + 7 (j a multiple of 8) as an 8-row group, element loads (chan2)
    __device__ __forceinline__ sg_t chan8b(int j) const
    {
        sg_t g;
        sset(g, 0, chan2(j));
        sset(g, 1, chan2(j + 2));
        sset(g, 2, chan2(j + 4));
        sset(g, 3, chan2(j + 6));
        return g;
    }
    __device__ __forceinline__ u32 bld(int d) const { return hb[d * 64]; }
    __device__ __forceinline__ void bst(int d, u32 v) const { hb[d * 64] = v; }
    __device__ __forceinline__ void sync() const
    {
        if (W > 1) __syncthreads();
    }
};

// ---------------------------------------------------------------------------------------
// channel reads by dwords (wrapper_in): the four lanes of a quad hold the positions 4 q ..
// 4 q + 3 of a word (lane_pos keeps quads whole). Lane k of the quad loads the dword of those
// positions of combination k = (frame lo / hi = k >> 1, row 2 i + (k & 1)) and a 4 x 4 byte
// transpose inside the quad (two quad DPP moves, two v_perm with per-lane selectors) gives
// every lane its position of all four: the slot dword. One 4-byte load per lane and slot
// dword instead of four byte loads.
// ---------------------------------------------------------------------------------------
// wave-uniform copy of a pointer (SGPRs): loads through (uniform base + 32-bit lane offset)
// take the saddr form, one VGPR per address instead of a 64-bit pair per load
template <class T>
__device__ __forceinline__ T *uniform_ptr(T *p)
{
    const unsigned long v = (unsigned long)p;
    const u32 lo = __builtin_amdgcn_readfirstlane((u32)v), hi = __builtin_amdgcn_readfirstlane((u32)(v >> 32));
    return (T *)(((unsigned long)hi << 32) | lo);
}
struct ChanQ {
    const g_u8 *base;   // frame lo, byte 0 (wave-uniform)
    u32 off;            // this lane's combination at row 0, positions 4 q .. (bytes from base)
    QuadSel sel;        // v_perm selectors of the two transpose rounds (polar_sc_device.h)
    bool al;            // frames 4-byte aligned (else the byte-load path)
};
__device__ __forceinline__ ChanQ chan_quad(const PairCtx &c)
{
    const u32 lane = threadIdx.x & 63u, pl = lane & 15u, k = pl & 3u;
    ChanQ q;
    // chl = frame lo + 16 row + pos; chh - chl = (hi frame - lo frame) N (uniform)
    q.base = uniform_ptr((const g_u8 *)c.chl - (16u * (lane >> 4) + lane_pos(pl)));
    const u32 dhi = __builtin_amdgcn_readfirstlane((u32)((const g_u8 *)c.chh - (const g_u8 *)c.chl));
    q.off = 16u * (lane >> 4) + (pl & ~3u) + ROWB * (k & 1u) + ((k & 2u) ? dhi : 0u);
    q.sel.init(pl);
    q.al = ((u32)(unsigned long)q.base & 3u) == 0u;
    return q;
}
__device__ __forceinline__ u32 quad_transpose(u32 x, const ChanQ &q) { return quad_transpose(x, q.sel); }
__device__ __forceinline__ u32 chan_conv(u32 raw)
{
    if constexpr (PAIR_SWAR) return conv4(raw);
    else return ppack8(chan_sm16(raw & 0x00FF00FFu), chan_sm16((raw >> 8) & 0x00FF00FFu));
}
// channel rows j .. j + 7 (j a multiple of 8) as four slot dwords, aligned frames
__device__ __forceinline__ u32x4 chan8a(const ChanQ &q, int j)
{
    u32 raw[4];
#pragma unroll
    for (int t = 0; t < 4; t++)   // rows j + 2 t, + 1: words 4 (j + 2 t) + r (+ 4)
        raw[t] = *(const g_u32 *)(q.base + (ROWB * (u32)(j + 2 * t) + q.off));
    u32x4 r;
#pragma unroll
    for (int t = 0; t < 4; t++) r[t] = chan_conv(quad_transpose(raw[t], q));
    return r;
}
__device__ __forceinline__ sg_t chan8(const PairCtx &c, const ChanQ &q, int j)
{
#if POLAR_PAIR_S16
    (void)q;   // int16 channel / 16-bit slots: element loads
    return c.chan8b(j);
#else
    if (!q.al) return c.chan8b(j);
    return chan8a(q, j);
#endif
}

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
// or G(src[j], src[n4 + j], bit_mem[local word ub + j]) for rows j in [j0, j1) (even bounds),
// one slot dword (two rows, both frames) per step
template <bool ISG, bool ROOT, bool SL, bool DL>
__device__ __forceinline__ void pfg_rows(const PairCtx &c, int s0, int d0, int n4, int ub, int j0, int j1)
{
    // groups of 8 rows (4 row pairs, one dwordx4 per lane) per batch; two batches in flight
    // (ping-pong: the loads of the next batch are issued before the arithmetic of this one).
    // HBM: 2 x 4 dwordx4 loads (+ 3 partial-sum dwords) per batch; the channel 8 x 4 byte
    // loads; LDS 2 x 2 b128.
    constexpr int NG = (ROOT ? 2 : (SL ? 2 : 4)) / (PAIR_S16 ? 2 : 1);   // (16-bit slots: the same registers)
    ChanQ cq;
    if constexpr (ROOT && !PAIR_S16) cq = chan_quad(c);
    constexpr int RB = 8 * NG;   // rows per batch
    auto src = [&](int j) -> sg_t {
        if constexpr (ROOT) return chan8(c, cq, j);
        else return c.template ld8<SL>(s0 + j);
    };
    struct Batch {
        sg_t a[NG], b[NG];
        u32 u0, u1, u2;   // (scalars: a selected array element would go to scratch)
    };
    auto load = [&](Batch &x, int j) {
#pragma unroll
        for (int g = 0; g < NG; g++) {
            x.a[g] = src(j + 8 * g);
            x.b[g] = src(n4 + j + 8 * g);
        }
        if constexpr (ISG) {
            // the partial sums of local words ub + j .. ub + j + RB - 1: at most 3 dwords
            const int dlast = (ub + n4 - 1) >> 4, q0 = (ub + j) >> 4;
            x.u0 = ub >= 0 ? c.bld(q0) : 0u;
            x.u1 = ub >= 0 ? c.bld(q0 + 1 < dlast ? q0 + 1 : dlast) : 0u;
            x.u2 = ub >= 0 ? c.bld(q0 + 2 < dlast ? q0 + 2 : dlast) : 0u;
        }
    };
    auto work = [&](const Batch &x, int j) {
        u32 uq[(RB + 15) / 16];   // partial sums of words ub + j + 16 h .. (RB <= 32: from u0 .. u2)
        if constexpr (ISG) {
            uq[0] = ubits16(x.u0, x.u1, ub + j);
            if constexpr (RB > 16) uq[1] = ubits16(x.u1, x.u2, ub + j);
        }
#pragma unroll
        for (int g = 0; g < NG; g++) {
            sg_t r;
#pragma unroll
            for (int t = 0; t < 4; t++) {
                if constexpr (ISG) {
                    const int k = 8 * g + 2 * t;   // row in the batch
                    const u32 u = ub >= 0 ? ubits4s(uq[k >> 4], k & 15) : 0u;
                    sset(r, t, fg4<true>(sget(x.a[g], t), sget(x.b[g], t), u));
                } else {
                    sset(r, t, fg4<false>(sget(x.a[g], t), sget(x.b[g], t), 0u));
                }
            }
            c.template st8<DL>(d0 + j + 8 * g, r);
        }
    };
    // row counts are multiples of 8 (subtrees of >= 32 words)
    const int nb = (j1 - j0) / RB, jlast = j0 + (nb - 1) * RB;
    int j = j0;
    if (nb > 0) {
        Batch x, y;
        load(x, j);
        for (;;) {
            load(y, j + RB < jlast ? j + RB : jlast);   // (the last batch re-loads itself: unused)
            work(x, j);
            j += RB;
            if (j > jlast) break;
            load(x, j + RB < jlast ? j + RB : jlast);
            work(y, j);
            j += RB;
            if (j > jlast) break;
        }
    }
    for (; j < j1; j += 8) {   // remaining groups
        Batch x;
        const sg_t a = src(j), b = src(n4 + j);
        sg_t r;
        const u32 ud = ub >= 0 ? c.bld((ub + j) >> 4) : 0u;
#pragma unroll
        for (int t = 0; t < 4; t++) {
            if constexpr (ISG) sset(r, t, fg4<true>(sget(a, t), sget(b, t), ub >= 0 ? ubits4(ud, ub + j + 2 * t) : 0u));
            else sset(r, t, fg4<false>(sget(a, t), sget(b, t), 0u));
        }
        (void)x;
        c.template st8<DL>(d0 + j, r);
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
__device__ __noinline__ void pop_fg_split(PairCtx c, int k, int n4, int ub)
{
    const int ng = n4 >> 3;   // groups of 8 rows
    pop_fg<ISG>(c, k, n4, ub, 8 * ((ng * c.wi) / c.W), 8 * ((ng * (c.wi + 1)) / c.W));
}

// A chain of D F / G records, each consuming the node the previous one wrote (the F_STATE
// descent of my_module.h:373-445 from a node to its leftmost subtree, or G_STATE then that
// descent): record 0 at level k over n4 output rows (ISG0: G with the partial sums at local
// word ub, else F), records i = 1 .. D - 1 at level k + i: F, or G with zero partial sums
// (the H0 route, bit i of gm). Every level is still written (its G reads it later), but the
// chain's own reads of levels k + 1 .. k + D - 1 come from registers: per column of 8 output
// rows of the last record, the 2^(D-1) row groups of record 0 at rows j0 + m nl are computed
// and folded pairwise. Columns split over the W waves, two in flight.
// AL: the channel frames are 4-byte aligned (dword reads, chan8), else byte reads (chan8b).
// PP: two columns in flight (ping-pong), except for root chains of D >= 4 (64 channel dwords
// per column; the generator emits D <= 3).
template <int D, bool ROOT, bool ISG0, bool AL>
__device__ __noinline__ void pchain(PairCtx c, int k, int n4, int ub, u32 gm)
{
    constexpr int M = 1 << (D - 1);
    constexpr bool PP = !ROOT || D <= 3;   // (D <= 3 from the generator)
    const int nl = n4 >> (D - 1);   // rows of the last record's output (a multiple of 8)
    const int ng = nl >> 3;
    const int g0 = (ng * c.wi) / c.W, g1 = (ng * (c.wi + 1)) / c.W;
    if (g1 <= g0) return;
    const int s0 = ROOT ? 0 : c.lvl_row(k);
    const bool sl = !ROOT && c.in_lds(s0);
    ChanQ cq;
    if constexpr (ROOT && !PAIR_S16) cq = chan_quad(c);
    // HBM slots and partial sums through a wave-uniform base + one 32-bit lane offset
    const u32 lane = threadIdx.x & 63u;
    const g_u8 *const hsb = (const g_u8 *)uniform_ptr(c.hs - (u32)GD * lane);
    const g_u8 *const hbb = (const g_u8 *)uniform_ptr(c.hb - lane);
    auto ldh = [&](int r) -> sg_t { return *(const g_sg *)(hsb + ((u32)(r >> 3) * (256u * GD) + (4u * GD) * lane)); };
    auto sth = [&](int r, sg_t v) { *(g_sg *)(hsb + ((u32)(r >> 3) * (256u * GD) + (4u * GD) * lane)) = v; };
    auto st = [&](int r, sg_t v) {
        if (c.in_lds(r)) c.template st8<true>(r, v);
        else sth(r, v);
    };
    struct Col {
        sg_t a[M], b[M];
        u32 u[M];
    };
    auto load = [&](Col &x, int g) {
#pragma unroll
        for (int m = 0; m < M; m++) {
            const int j = 8 * g + m * nl;
            if constexpr (ROOT && AL && !PAIR_S16) {
                x.a[m] = chan8a(cq, j);
                x.b[m] = chan8a(cq, n4 + j);
            } else if constexpr (ROOT) {
                x.a[m] = c.chan8b(j);
                x.b[m] = c.chan8b(n4 + j);
            } else if (sl) {
                x.a[m] = c.template ld8<true>(s0 + j);
                x.b[m] = c.template ld8<true>(s0 + n4 + j);
            } else {
                x.a[m] = ldh(s0 + j);
                x.b[m] = ldh(s0 + n4 + j);
            }
            if constexpr (ISG0) x.u[m] = ub >= 0 ? *(const g_u32 *)(hbb + ((u32)((ub + j) >> 4) * 256u + 4u * lane)) : 0u;
        }
    };
    auto work = [&](Col &x, int g) {
        const int j0 = 8 * g;
        const int d1 = c.lvl_row(k + 1);
#pragma unroll
        for (int m = 0; m < M; m++) {
            const int j = j0 + m * nl;
#pragma unroll
            for (int t = 0; t < 4; t++) {
                if constexpr (ISG0) sset(x.a[m], t, fg4<true>(sget(x.a[m], t), sget(x.b[m], t), ub >= 0 ? ubits4(x.u[m], ub + j + 2 * t) : 0u));
                else sset(x.a[m], t, fg4<false>(sget(x.a[m], t), sget(x.b[m], t), 0u));
            }
            st(d1 + j, x.a[m]);
        }
#pragma unroll
        for (int i = 1; i < D; i++) {
            const int h = M >> i;
            const int di = c.lvl_row(k + 1 + i);
            if ((gm >> i) & 1u) {
#pragma unroll
                for (int m = 0; m < h; m++) {
#pragma unroll
                    for (int t = 0; t < 4; t++) sset(x.a[m], t, fg4<true>(sget(x.a[m], t), sget(x.a[m + h], t), 0u));
                    st(di + j0 + m * nl, x.a[m]);
                }
            } else {
#pragma unroll
                for (int m = 0; m < h; m++) {
#pragma unroll
                    for (int t = 0; t < 4; t++) sset(x.a[m], t, fg4<false>(sget(x.a[m], t), sget(x.a[m + h], t), 0u));
                    st(di + j0 + m * nl, x.a[m]);
                }
            }
        }
    };
    if constexpr (!PP) {
        for (int g = g0; g < g1; g++) {
            Col x;
            load(x, g);
            work(x, g);
        }
    } else {
        Col x, y;
        int g = g0;
        load(x, g);
        for (;;) {
            if (g + 1 < g1) load(y, g + 1);
            work(x, g);
            if (++g >= g1) break;
            if (g + 1 < g1) load(x, g + 1);
            work(y, g);
            if (++g >= g1) break;
        }
    }
}
template <int D, bool ROOT, bool ISG0>
__device__ __forceinline__ void pop_chain(const PairCtx &c, int k, int n4, int ub, u32 gm)
{
    if (c.W > 1) {
        // several waves per pair (small batches): the records one by one, each split over all
        // the waves by row groups -- same-box A/B at C5 (W = 8): 1.51 ms this way vs 1.63 ms
        // chained (profiles/r03_ab/chain_c5_ab.txt); the chains pay at W = 1 (C3 -15 %)
        pop_fg_split<ISG0>(c, k, n4, ub);
#pragma unroll
        for (int i = 1; i < D; i++) {
            c.sync();
            if ((gm >> i) & 1u) pop_fg_split<true>(c, k + i, n4 >> i, -1);
            else pop_fg_split<false>(c, k + i, n4 >> i, -1);
        }
        return;
    }
    if constexpr (PAIR_S16) pchain<D, ROOT, ISG0, false>(c, k, n4, ub, gm);   // (int16 channel: element loads)
    else if (ROOT && !chan_quad(c).al) pchain<D, ROOT, ISG0, false>(c, k, n4, ub, gm);
    else pchain<D, ROOT, ISG0, true>(c, k, n4, ub, gm);
}

// source dwords of a pruned-node op (REP / R1 / SPC): rows j, j + 1 (j even) of the parent's
// two halves, slot format
template <bool ROOT, bool SL>
__device__ __forceinline__ void psrc2(const PairCtx &c, int s0, int n4, int j, su_t &a, su_t &b)
{
    if constexpr (ROOT) {
        a = c.chan2(j);
        b = c.chan2(n4 + j);
    } else {
        a = c.template ld2<SL>(s0 + j);
        b = c.template ld2<SL>(s0 + n4 + j);
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
    for (int j = 0; j < n4; j += 2) {
        su_t a, b;
        psrc2<ROOT, SL>(c, s0, n4, j, a, b);
#pragma unroll
        for (int o = 0; o < 2; o++) {
            const u32 lam = F_pair(prow(a, o), prow(b, o)), sg = pk_sra(lam, 15);
            if constexpr (LPAR < 4) {   // PAR 4 / 8: the exact chain over the groups (SM / CA2)
                acc = rep_groups_rows(acc, CA2 ? pk_sub((lam & MAG) ^ sg, sg) : lam, c.lanes());
                continue;
            }
            const X4 t = rows4(row_sum_biased(pk_add(pk_sub((lam & MAG) ^ sg, sg), 0x02000200u)));
            if constexpr (PAIR_SOLO) acc = rep_acc_solo(acc, t.t0, t.t1, t.t2, t.t3);
            else acc = rep_acc_rows(acc, t.t0, t.t1, t.t2, t.t3);
        }
    }
    // (CA2: the exact sums of ADD_TREE_{n}_CA2 / VECTOR_ADD are this chain, and a zero total
    // decides 0: no fallback)
    if (!CA2 && LPAR >= 4 && (PAIR_SOLO ? rep_any_zero_lo(acc) : rep_any_zero(acc))) {
        const Lanes ln = c.lanes();
        acc = 0;
        for (int j = 0; j < n4; j += 2) {
            su_t a, b;
            psrc2<ROOT, SL>(c, s0, n4, j, a, b);
#pragma unroll
            for (int o = 0; o < 2; o++) {
                if constexpr (PAIR_SOLO) acc = rep_sm_solo(acc, F_sm(prow(a, o), prow(b, o)), ln);
                else acc = rep_sm_rows(acc, F_sm(prow(a, o), prow(b, o)), ln);
            }
        }
    }
    if constexpr (PAIR_SOLO) acc = bcast_lo(acc);   // one frame: both halves of the node
    const u32 full = pk_sra(acc, 15);   // two's complement or SM16: the decision is bit 15 / 31
    for (int l = 0; l < n4; l += 16) pbits_put(c, l0 + l, n4 - l < 16 ? n4 - l : 16, full);
}
__device__ __noinline__ void pop_rep(PairCtx c, int k, int n4, int l0)
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
    su_t da{}, db{};
    const int row = (int)c.row();
    const u32 ksub = SPC ? spc_sub((u32)row, c.lanes()) : 0u;
    for (int j = j0; j < j1; j++) {
        if (((j - j0) & 1) == 0) psrc2<ROOT, SL>(c, s0, n4, j, da, db);
        const u32 a = prow(da, j & 1), b = prow(db, j & 1);
        u32 u = 0;
        if (ub >= 0) {
            if (j == j0 || ((ub + j) & 15) == 0) ud = c.bld((ub + j) >> 4);
            u = ubit_p(ud, ub + j);
        }
        const u32 lam = G_sm<GSAT>(a, b, u), h = hard_pair(lam);
        const int q = (l0 + j) & 15;
        acc |= h >> (15 - q);
        if (q == 15 || j + 1 == j1) {
            const int first = ((l0 + j) & ~15) > l0 + j0 ? ((l0 + j) & ~15) : l0 + j0;
            pbits_put(c, first, l0 + j + 1 - first, acc);
            acc = 0;
        }
        if constexpr (SPC && PAIR_SOLO) {
            // (word 8 j + 4 h + r, position) order: half 1 keys carry bit 6
            par ^= h;
            const u32 wk = ((u32)j << 7) | ksub;
            klo = __builtin_elementwise_min(klo, ((lam & 0xFFu) << 24) | wk);
            khi = __builtin_elementwise_min(khi, (((lam >> 16) & 0xFFu) << 24) | wk | 64u);
        } else if constexpr (SPC) {
            par ^= h;
            const u32 wk = ((u32)j << 6) | ksub;   // (word, position) order
            klo = __builtin_elementwise_min(klo, ((lam & 0xFFu) << 24) | wk);
            khi = __builtin_elementwise_min(khi, (((lam >> 16) & 0xFFu) << 24) | wk);
        }
    }
    if constexpr (SPC) {
        const Lanes ln = c.lanes();
        par = row_xor(par);
        klo = row_min_u32(klo);
        khi = row_min_u32(khi);
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
            lds_w32 *const x = c.lx();
            x[(3 * c.wi) * 64] = part ? par : 0u;
            x[(3 * c.wi + 1) * 64] = part ? klo : 0xFFFFFFFFu;
            x[(3 * c.wi + 2) * 64] = part ? khi : 0xFFFFFFFFu;
            __syncthreads();
            if (!c.lead()) return;
            par = 0;
            klo = khi = 0xFFFFFFFFu;
            for (int w = 0; w < c.W; w++) {
                par ^= x[(3 * w) * 64];
                klo = __builtin_elementwise_min(klo, (u32)x[(3 * w + 1) * 64]);
                khi = __builtin_elementwise_min(khi, (u32)x[(3 * w + 2) * 64]);
            }
        }
        if constexpr (PAIR_SOLO) {
            // one frame: the parity of both halves, the first minimum of both
            const u32 k = __builtin_elementwise_min(klo, khi);
            if (((par ^ (par << 16)) & 0x80000000u) && (k & 63u) == ksub) {
                const int l = l0 + (int)((k >> 7) & 0x1FFFFu);
                c.bst(l >> 4, c.bld(l >> 4) ^ (((k & 64u) ? 0x10000u : 1u) << (l & 15)));
            }
            return;
        }
        // the flipped word: 4 (key >> 6) + ((key >> 4) & 3), position bitrev4^-1(key & 15)
        const bool flo = (par & 0x8000u) && (klo & 63u) == ksub;
        const bool fhi = (par & 0x80000000u) && (khi & 63u) == ksub;
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
__device__ __noinline__ void pop_r1spc(PairCtx c, int k, int n4, int ub, int l0)
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
__device__ __noinline__ void pop_h(PairCtx c, int l0, int n4)
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
    } else if (c.lead()) {
        const u32 m = ((1u << n4) - 1u) << (l0 & 15), mm = m | (m << 16);
        const u32 d = c.bld(l0 >> 4), sh = (d >> n4) & mm;
        c.bst(l0 >> 4, H0 ? ((d & ~mm) | sh) : (d ^ sh));
    }
}

// END (my_module.h:1848-1869) + wrapper_out: the partial sums of every local word, transposed
// inside each row (lane j of row r: the 16 position bits of local word 16 d + j = word
// 4 (16 d + j) + r), stored as u16 words in natural order
__device__ __noinline__ void pair_out(PairCtx c, g_u16 *o_lo, g_u16 *o_hi, bool st_lo, bool st_hi, int out_stride)
{
    const Lanes ln = c.lanes();
    const int row = (int)c.row();
    const int nd = c.G >> 6;   // dwords per lane (G / 4 local words)
    const int e0 = (nd * c.wi) / c.W, e1 = (nd * (c.wi + 1)) / c.W;
    for (int d = e0; d < e1; d++) {
        const u32 t = row_transpose16(to_position_order(c.bld(d), ln), ln);
        if constexpr (PAIR_SOLO) {   // half h of local word l, row r: word 8 l + 4 h + r
            const int w = 8 * (16 * d + (int)ln.pl) + row;
            if (st_lo) {
                o_lo[w] = (unsigned short)(t & 0xFFFFu);
                o_lo[w + 4] = (unsigned short)(t >> 16);
            }
        } else {
            const int w = 4 * (16 * d + (int)ln.pl) + row;
            if (st_lo) o_lo[w] = (unsigned short)(t & 0xFFFFu);
            if (st_hi) o_hi[w] = (unsigned short)(t >> 16);
        }
    }
    if (c.lead())
        for (int w = (PAIR_SOLO ? 2 : 1) * c.G + (int)ln.pl + 16 * row; w < out_stride; w += 64) {   // pad words
            if (st_lo) o_lo[w] = 0;
            if (st_hi) o_hi[w] = 0;
        }
}

// the pair's storage: HBM scratch of `pair_dwords` per pair = slot rows (128 B each) then
// the partial-sum dwords (256 B rows); LDS: slot rows [lds_row0, total) then the SPC exchange
__device__ __forceinline__ bool pair_init(PairCtx &c, const signed char *llr, unsigned int *scratch, int N, int batch,
                                          long pair, int pair_dwords, int slot_rows, int lds_row0, int wi, int W,
                                          lds_w32 *lbase)
{
    const int lane = threadIdx.x & 63;
    c.G = PAIR_SOLO ? N >> 5 : N >> 4;   // (solo: virtual words per half)
    c.wi = wi;
    c.W = W;
    c.lds_row0 = lds_row0;
    const long f_lo = PAIR_SOLO ? pair : 2 * pair, f_hi = 2 * pair + 1;
    const long fl = f_lo < batch ? f_lo : (long)batch - 1, fh = f_hi < batch ? f_hi : (long)batch - 1;
    const int off = 16 * (int)c.row() + (int)c.lanes().pos;
    c.chl = (const g_chan *)llr + fl * (long)N + off;
    c.chh = PAIR_SOLO ? c.chl + 64 : (const g_chan *)llr + fh * (long)N + off;   // (solo: words 8 j + 4 + r)
    g_u32 *base = (g_u32 *)scratch + pair * (long)pair_dwords;
    c.hs = base + GD * lane;
    c.hb = base + slot_rows * 8 * GD + lane;   // slot_rows x 128 B (16-bit slots: 256 B)
    c.ls = lbase + GD * lane;
    c.lxo = (slot_rows > lds_row0 ? slot_rows - lds_row0 : 0) * 8 * GD;
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
    if ((PAIR_SOLO ? pair : 2 * pair) >= batch) return;
    PairCtx c;
    pair_init(c, llr, scratch, N, batch, pair, pair_dwords, slot_rows, slot_rows, 0, 1, nullptr);
    const int j0 = j * cw, j1 = j0 + cw < n4 ? j0 + cw : n4;
    if (code_g) pop_fg<true>(c, k, n4, ub, j0, j1);
    else pop_fg<false>(c, k, n4, ub, j0, j1);
}

}  // namespace polar
