// polar_sc_device.h -- CDNA4 device primitives of the SC polar decoder, shared by the
// schedule-interpreter kernels (polar_sc_kernels.hip, hipcc) and the per-mask kernels
// generated at plan time (polar_sc_jit.cpp, hipRTC). No standard headers: hipRTC-clean.
//
// Representation "SM16": two frames per 32-bit register, one per 16-bit half; each half is
// sign-magnitude (bit 15 = sign, bits 0..14 = magnitude), the number format of the
// reference (SIGMAG, src/module/config.h:11) with room for the leaf's width growth.
#pragma once

namespace polar {

typedef unsigned int u32;
typedef unsigned long long u64;
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));

constexpr u32 SGN = 0x80008000u;   // sign flags of both halves
constexpr u32 MAG = 0x7FFF7FFFu;   // magnitudes of both halves

// The datapath format (the reference's compile-time switches). The hipcc-built schedule
// interpreter is the shipped configuration; generated (hipRTC) kernels of other plans define
// these first:
//   POLAR_Q     LLR_BITS (config.h:2), 5..9; 9-bit LLRs keep 16-bit HBM stage slots
//   POLAR_CA2   1: two's complement datapath (config.h:11 CA2, functions.h:48-118), values
//               are i16 per half; 0: SIGMAG (SM16: bit 15 sign, bits 0..14 magnitude)
//   POLAR_EXT   EXTENDED (config.h:14): exact leaves (1) or saturating G inside leaves (0)
//   POLAR_LPAR  log2 PAR (polar_parameters.h:8), 2..6 on the device: a PAR word is P16
//               consecutive 16-LLR device words (PAR >= 16), or PPW PAR words share one
//               device word (PAR 4 / 8: a sub-row of 4 / 8 lanes)
//   POLAR_CHAN16  channel stream of int16 LLRs instead of int8
#ifndef POLAR_Q
#define POLAR_Q 6
#endif
#ifndef POLAR_CA2
#define POLAR_CA2 0
#endif
#ifndef POLAR_EXT
#define POLAR_EXT 1
#endif
#ifndef POLAR_LPAR
#define POLAR_LPAR 4
#endif
#ifndef POLAR_CHAN16
#define POLAR_CHAN16 0
#endif
static_assert(POLAR_Q >= 5 && POLAR_Q <= 9, "LLR_BITS 5..9");
static_assert(POLAR_LPAR >= 2 && POLAR_LPAR <= 6, "PAR 4..64 on the device");
constexpr int QB = POLAR_Q;
constexpr bool CA2 = POLAR_CA2 != 0;
constexpr bool EXT = POLAR_EXT != 0;
constexpr int LPAR = POLAR_LPAR;
constexpr int P16 = LPAR >= 4 ? 1 << (LPAR - 4) : 1;   // device words per PAR word
constexpr int PPW = LPAR < 4 ? 16 >> LPAR : 1;          // PAR words per device word
constexpr bool SLOT16 = QB > 8;                 // HBM stage slots hold 16-bit values
constexpr u32 QMAG = (1u << (QB - 1)) - 1u;     // channel / F magnitude bound (31 at 6 bits)
// G clamp: SIGMAG qsat_sm<Q-1> (15 at Q 6, functions.h:186-194), CA2 qsat<Q> (31, :63-75)
constexpr u32 GSAT = CA2 ? (1u << (QB - 1)) - 1u : (1u << (QB - 2)) - 1u;
// REP accumulator clamp (ADDER_TREE_{PAR}, functions.h:3163-3320): SIGMAG
// qfull_adder_sat_sm<Q+L+1> -> 2^(Q+L-1)-1 (511 at Q 6, PAR 16); CA2 qadd<Q+L+1> -> 2^(Q+L)-1
constexpr u32 REPSAT = CA2 ? (1u << (QB + LPAR)) - 1u : (1u << (QB + LPAR - 1)) - 1u;
constexpr u32 GSAT2 = GSAT * 0x00010001u;
// magnitude field of a stage value in the split / slot forms of the generated kernels: SIGMAG
// magnitudes stay <= QMAG; CA2 keeps |MIN| = 2^(Q-1), the absorbing value of F_function_C2's
// qabs wrap (functions.h:48-61, scalar.h:42-49), as magnitude 2^(Q-1) with the sign set
constexpr u32 VMAG = CA2 ? (1u << QB) - 1u : QMAG;

// ---------------------------------------------------------------------------------------
// packed 16-bit helpers (v_pk_* on gfx950)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ u32 U(u16x2 v) { return __builtin_bit_cast(u32, v); }
__device__ __forceinline__ u16x2 V(u32 v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ u32 pk_min(u32 a, u32 b) { return U(__builtin_elementwise_min(V(a), V(b))); }
__device__ __forceinline__ u32 pk_add(u32 a, u32 b) { return U(V(a) + V(b)); }
__device__ __forceinline__ u32 pk_max_u16(u32 a, u32 b) { return U(__builtin_elementwise_max(V(a), V(b))); }
// a * b + c per 16-bit half, modulo 2^16 (v_pk_mad_u16)
__device__ __forceinline__ u32 pk_mad_u16(u32 a, u32 b, u32 c) { return U(V(a) * V(b) + V(c)); }
__device__ __forceinline__ u32 pk_sub(u32 a, u32 b) { return U(V(a) - V(b)); }
__device__ __forceinline__ u32 pk_mul_lo(u32 a, u32 b) { return U(V(a) * V(b)); }
__device__ __forceinline__ u32 pk_sra(u32 a, short s)
{
    i16x2 x = __builtin_bit_cast(i16x2, a);
    x = x >> s;
    return __builtin_bit_cast(u32, x);
}
__device__ __forceinline__ u32 pk_shl(u32 a, unsigned short s) { return U(V(a) << s); }
__device__ __forceinline__ u32 pk_abs_i16(u32 a)
{
    i16x2 x = __builtin_bit_cast(i16x2, a);
    i16x2 y = -x;
    return __builtin_bit_cast(u32, __builtin_elementwise_max(x, y));
}
// bitwise select: m ? a : b
__device__ __forceinline__ u32 bsel(u32 m, u32 a, u32 b) { return (a & m) | (b & ~m); }
// the same with the mask hidden from the optimiser: a mask known to be 0 / 0xFFFF per half
// is otherwise rewritten into v_cmp + v_cndmask per half + v_perm (8 instructions for 1)
__device__ __forceinline__ u32 opaque(u32 m)
{
    asm("" : "+v"(m));
    return m;
}
__device__ __forceinline__ u32 bselo(u32 m, u32 a, u32 b) { return bsel(opaque(m), a, b); }

// F_function_SM (shared/src/functions.h:124-145): sign xor, magnitude min, no saturation.
__device__ __forceinline__ u32 F_sm(u32 a, u32 b)
{
    return pk_min(a & MAG, b & MAG) | ((a ^ b) & SGN);
}

// qfull_add_sub_sm (shared/src/scalar.h:196-225) on SM16, followed by an optional clamp:
//   a' = a with sign ^ u; same signs -> |a|+|b|, else ||a|-|b||;
//   sign = |a| < |b| ? sign(b) : sign(a')      (ties -> sign(a'), may produce -0)
// SAT = 15 : G_function_SM, VECTOR_SAT_SM<P,Q-1> clamp (functions.h:186-194, scalar.h:94-99)
// SAT = 511: qfull_adder_sat_sm<11> of the REP accumulator (scalar.h:164-194)
// SAT = 0  : G_extended_SM / qfull_adder_sm (exact; leaves and the REP pair tree)
// u holds sign-flip flags at bit positions 15/31 only.
template <int SAT>
__device__ __forceinline__ u32 G_sm(u32 a, u32 b, u32 u)
{
    const u32 ma = a & MAG, mb = b & MAG;
    const u32 d = pk_sub(ma, mb);             // bit 15 set iff |a| < |b|
    const u32 x = a ^ u ^ b;                  // bit 15 set iff sign(a') != sign(b)
    u32 m = bsel(pk_sra(x, 15), pk_abs_i16(d), pk_add(ma, mb));
    if constexpr (SAT != 0) m = pk_min(m, (u32)SAT * 0x00010001u);
    // |a| < |b| -> sign(b); otherwise sign(a') = sign(b) ^ x
    return ((b ^ (x & ~d)) & SGN) | m;
}

// ---------------------------------------------------------------------------------------
// cross-lane exchange inside a 16-lane DPP row
// ---------------------------------------------------------------------------------------
// Lane order. POLAR_LANE_REMAP = 0: lane l of a row holds word position l. With 1 (the
// per-mask kernels), positions 4..7 and 12..15 sit mirrored in their quad
// (lane = p ^ (p & 4 ? 3 : 0), an involution). Partners at position distance 8 / 4 / 2 / 1
// are then lanes l^8 (row_ror:8), l^7 (row_half_mirror), l^2, l^1 (quad_perm): one DPP
// each, where the identity order needs two for distance 4.
#ifndef POLAR_LANE_REMAP
#define POLAR_LANE_REMAP 0
#endif
__device__ __forceinline__ u32 lane_pos(u32 lane)
{
    return POLAR_LANE_REMAP ? (lane ^ ((lane & 4u) ? 3u : 0u)) : lane;
}

// value of physical lane (l ^ H)
template <int H>
__device__ __forceinline__ u32 xorlane_phys(u32 v)
{
    if constexpr (H == 1) {
        return __builtin_amdgcn_update_dpp(0u, v, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
    } else if constexpr (H == 2) {
        return __builtin_amdgcn_update_dpp(0u, v, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
    } else if constexpr (H == 4) {
        u32 t = __builtin_amdgcn_update_dpp(0u, v, 0x141, 0xF, 0xF, true);  // row_half_mirror: l^7
        return __builtin_amdgcn_update_dpp(0u, t, 0x1B, 0xF, 0xF, true);   // quad_perm [3,2,1,0]: ^3
    } else {
        static_assert(H == 8, "row partner distance");
        return __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xF, 0xF, true);  // row_ror:8
    }
}
// value at word-position distance H (the partner of the leaf / pair-tree recursions)
template <int H>
__device__ __forceinline__ u32 xorlane(u32 v)
{
    if constexpr (POLAR_LANE_REMAP && H == 4)
        return __builtin_amdgcn_update_dpp(0u, v, 0x141, 0xF, 0xF, true);   // row_half_mirror: l^7
    else
        return xorlane_phys<H>(v);
}

// per-lane constants: all-ones where the lane is the lower ("a") member of its pair at
// word-position distance H
struct Lanes {
    u32 a1, a2, a4, a8;   // lane masks
    u32 pl;               // physical lane in the row, 0..15
    u32 pos;              // word position held by this lane (lane_pos(pl))
    u32 br;               // bitrev4(pos)
    template <int H> __device__ __forceinline__ u32 amask() const
    {
        if constexpr (H == 1) return a1;
        else if constexpr (H == 2) return a2;
        else if constexpr (H == 4) return a4;
        else return a8;
    }
    __device__ __forceinline__ void init(u32 p)
    {
        pl = p;
        pos = lane_pos(p);
        br = ((pos & 1u) << 3) | ((pos & 2u) << 1) | ((pos & 4u) >> 1) | ((pos & 8u) >> 3);
        a1 = (pos & 1u) ? 0u : 0xFFFFFFFFu;
        a2 = (pos & 2u) ? 0u : 0xFFFFFFFFu;
        a4 = (pos & 4u) ? 0u : 0xFFFFFFFFu;
        a8 = (pos & 8u) ? 0u : 0xFFFFFFFFu;
    }
};

// per-lane data back to identity lane order (lane p receives position p's value)
__device__ __forceinline__ u32 to_position_order(u32 v, const Lanes &ln)
{
    if constexpr (POLAR_LANE_REMAP)
        return bselo(ln.a4, v, __builtin_amdgcn_update_dpp(0u, v, 0x1B, 0xF, 0xF, true));  // quad mirror
    else
        return v;
}

// ---------------------------------------------------------------------------------------
// Leaf: Spec_PolarDec_16 -> Spec_P16_ext<6> (functions.h:521-546, 413-492, 366-384):
// exact SC over the 16 LLRs of one word, F (min) + G_extended (exact, width grows).
// Executed by all 16 lanes of each row (4 rows x 2 halves = 8 frames at once).
// Returns x (the 16 encoded bits) as sign-position flags per lane.
// Blocks whose frozen pattern is all-frozen return 0; all-information blocks return the
// hard decisions of their LLRs, which is what the recursion computes for them
// (induction on G with u = x_a: sign(a') = sign(b)).
// ---------------------------------------------------------------------------------------
// (a) frozen pattern known only at run time (schedule interpreter)
template <int B, int W>
__device__ __forceinline__ u32 leaf_rec(u32 L, u32 fb, u32 fbm, const Lanes &ln)
{
    constexpr u32 bm = ((1u << W) - 1u) << B;
    const u32 sub = fb & bm;
    if (sub == 0u) return 0u;
    if (sub == bm) return L & SGN;
    if constexpr (W == 2) {
        // Spec_P2 (functions.h:366-384): lane B = a, lane B+1 = b
        u32 P = xorlane<1>(L);
        u32 u0 = (L ^ P) & fbm;                   // F_simplified & fb[B]   (valid on a)
        u32 u0p = xorlane<1>(u0);
        u32 d = pk_sub(P & MAG, L & MAG);         // |a| < |b|              (on b)
        u32 u1 = bsel(d, L, P ^ u0p) & fbm;       // G_simplified & fb[B+1] (valid on b)
        u32 u1p = xorlane<1>(u1);
        return bsel(ln.a1, u0 ^ u1p, u1);
    } else {
        constexpr int H = W / 2;
        u32 P = xorlane<H>(L);
        u32 La = F_sm(L, P);                             // valid on a-lanes
        u32 xa = leaf_rec<B, H>(La, fb, fbm, ln);
        u32 Lb = G_sm<0>(P, L, xorlane<H>(xa));          // valid on b-lanes
        u32 xb = leaf_rec<B + H, H>(Lb, fb, fbm, ln);
        return bsel(ln.template amask<H>(), xa ^ xorlane<H>(xb), xb);
    }
}

__device__ __forceinline__ u32 leaf16(u32 L, u32 fb, const Lanes &ln)
{
    u32 fbm = ((fb >> ln.pos) & 1u) ? SGN : 0u;   // the frozen bit of this lane's word position
    return leaf_rec<0, 16>(L, fb, fbm, ln);
}

// ---------------------------------------------------------------------------------------
// Row reductions
// ---------------------------------------------------------------------------------------
// ADD_TREE_16_SM (functions.h:3036-3083): pair (j, j+8), then (j, j+4) ... with the lower
// lane as operand a. Butterfly form: both partners compute combine(lower, upper), so every
// lane ends with the row total (same pairing and operand order as the reference tree).
__device__ __forceinline__ u32 row_add_tree(u32 v, const Lanes &ln)
{
    u32 p;
    p = xorlane<8>(v); v = G_sm<0>(bsel(ln.a8, v, p), bsel(ln.a8, p, v), 0u);
    p = xorlane<4>(v); v = G_sm<0>(bsel(ln.a4, v, p), bsel(ln.a4, p, v), 0u);
    p = xorlane<2>(v); v = G_sm<0>(bsel(ln.a2, v, p), bsel(ln.a2, p, v), 0u);
    p = xorlane<1>(v); v = G_sm<0>(bsel(ln.a1, v, p), bsel(ln.a1, p, v), 0u);
    return v;
}

__device__ __forceinline__ u32 row_min_u32(u32 v)
{
    v = __builtin_elementwise_min(v, xorlane<8>(v));
    v = __builtin_elementwise_min(v, xorlane<4>(v));
    v = __builtin_elementwise_min(v, xorlane<2>(v));
    v = __builtin_elementwise_min(v, xorlane<1>(v));
    return v;
}

__device__ __forceinline__ u32 row_xor(u32 v)
{
    v ^= xorlane<8>(v);
    v ^= xorlane<4>(v);
    v ^= xorlane<2>(v);
    v ^= xorlane<1>(v);
    return v;
}

// 16x16 bit transpose inside a row on both 16-bit halves: lane l bit j <- lane j bit l.
__device__ __forceinline__ u32 row_transpose16(u32 v, const Lanes &ln)
{
    u32 p;
    p = xorlane_phys<8>(v); v = bsel((((ln.pl & 8u) != 0u) ? 0u : 0xFFFFFFFFu), (v & 0x00FF00FFu) | ((p & 0x00FF00FFu) << 8), ((p >> 8) & 0x00FF00FFu) | (v & 0xFF00FF00u));
    p = xorlane_phys<4>(v); v = bsel((((ln.pl & 4u) != 0u) ? 0u : 0xFFFFFFFFu), (v & 0x0F0F0F0Fu) | ((p & 0x0F0F0F0Fu) << 4), ((p >> 4) & 0x0F0F0F0Fu) | (v & 0xF0F0F0F0u));
    p = xorlane_phys<2>(v); v = bsel((((ln.pl & 2u) != 0u) ? 0u : 0xFFFFFFFFu), (v & 0x33333333u) | ((p & 0x33333333u) << 2), ((p >> 2) & 0x33333333u) | (v & 0xCCCCCCCCu));
    p = xorlane_phys<1>(v); v = bsel((((ln.pl & 1u) != 0u) ? 0u : 0xFFFFFFFFu), (v & 0x55555555u) | ((p & 0x55555555u) << 1), ((p >> 1) & 0x55555555u) | (v & 0xAAAAAAAAu));
    return v;
}

// ---------------------------------------------------------------------------------------
// PRUNING_LEVEL 1 leaf decoders (R_STATE, my_module.h:566-593). SM16 word in, sign-position
// flags per lane out (like leaf16).
// ---------------------------------------------------------------------------------------
// Spec_REP_Node -> REP_16_SM (functions.h:1049-1060, 996-1016): exact SM pair sums at
// distance 8, 4, 2, then the sign rule of REP_2_SM (|a| < |b| ? sign b : sign a) -- the sign
// of the full pair-tree total; x = 16 copies.
__device__ __forceinline__ u32 leaf_rep(u32 L, const Lanes &ln) { return row_add_tree(L, ln) & SGN; }

// Spec_REP_REP2_Node with sel = 1 -> REP_REP2_16_SM (functions.h:1353-1420): the same folds
// at distance 8, 4, 2 leave the exact totals of the even and the odd positions; x[i] = the
// SM sign of its class total (res2 = (sigb, siga), repeated).
__device__ __forceinline__ u32 leaf_rep2(u32 v, const Lanes &ln)
{
    u32 p;
    p = xorlane<8>(v); v = G_sm<0>(bsel(ln.a8, v, p), bsel(ln.a8, p, v), 0u);
    p = xorlane<4>(v); v = G_sm<0>(bsel(ln.a4, v, p), bsel(ln.a4, p, v), 0u);
    p = xorlane<2>(v); v = G_sm<0>(bsel(ln.a2, v, p), bsel(ln.a2, p, v), 0u);
    return v & SGN;
}

// Spec_SPC_Node -> SPC_Node_16 (functions.h:2111-2136; SPC_Parity_16 :1633-1644,
// SPC_Min_Mask_16_SM :1919-1937): h = signs; flip h at the minimum |lambda| (tournament at
// distance 8, 4, 2, 1, the upper lane winning only when strictly smaller: ties -> smallest
// bitrev4(position)) when the parity of h is odd. SPC2 (SPC_SPC2_Node_16 with sel = 1,
// :2786-2811, :2254-2300, :2534-2580): parity and minimum per class of even / odd positions
// (folds at distance 8, 4, 2 only), both class minima may flip.
template <bool SPC2>
__device__ __forceinline__ u32 leaf_spc(u32 L, const Lanes &ln)
{
    const u32 h = L & SGN;
    u32 par = h;
    par ^= xorlane<8>(par);
    par ^= xorlane<4>(par);
    par ^= xorlane<2>(par);
    if constexpr (!SPC2) par ^= xorlane<1>(par);
    u32 klo = ((L & 0x7FFFu) << 4) | ln.br, khi = (((L >> 16) & 0x7FFFu) << 4) | ln.br;
    const u32 mlo0 = klo, mhi0 = khi;
    klo = __builtin_elementwise_min(klo, xorlane<8>(klo));
    khi = __builtin_elementwise_min(khi, xorlane<8>(khi));
    klo = __builtin_elementwise_min(klo, xorlane<4>(klo));
    khi = __builtin_elementwise_min(khi, xorlane<4>(khi));
    klo = __builtin_elementwise_min(klo, xorlane<2>(klo));
    khi = __builtin_elementwise_min(khi, xorlane<2>(khi));
    if constexpr (!SPC2) {
        klo = __builtin_elementwise_min(klo, xorlane<1>(klo));
        khi = __builtin_elementwise_min(khi, xorlane<1>(khi));
    }
    const u32 flo = (klo == mlo0) ? (par & 0x8000u) : 0u;
    const u32 fhi = (khi == mhi0) ? (par & 0x80000000u) : 0u;
    return h ^ flo ^ fhi;
}

// ---------------------------------------------------------------------------------------
// Channel LLR -> SM16: wrapper_in + Adapt_format/qconv_format (wrapper_in.h:34,
// library.h:18-28, scalar.h:229-239). The LLR is the low 6 bits (sc_bigint<6>); -32 -> +0.
// ---------------------------------------------------------------------------------------
// raw = b_lo | b_hi << 16 (two int8 LLRs, any bits above bit 5 ignored) -> SM16 pair.
// With t = raw & 63: |LLR| = min(t, 64 - t) & 31 (t = 32, i.e. -32, -> 0) and the sign is
// set iff t >= 33 (t + 0x7FDF reaches bit 15).
__device__ __forceinline__ u32 conv_pair(u32 raw)
{
    constexpr u32 QM = (1u << QB) - 1u, QP = 1u << QB;
    constexpr u32 SB = 0x8000u - (QP / 2u + 1u);   // t + SB reaches bit 15 iff t > 2^(Q-1)
    u32 t = raw & (QM * 0x00010001u);
    u32 m = pk_min(t, pk_sub(QP * 0x00010001u, t)) & (QMAG * 0x00010001u);
    return m | (pk_add(t, SB * 0x00010001u) & SGN);
}

// Channel byte -> SM8 (bit 7 sign, bits 0..4 magnitude): the per-mask kernels keep a
// 256-entry copy of this map in LDS and convert a word with two lookups + 2 VALU.
__device__ __forceinline__ u32 sm8_of_byte(u32 b)
{
    constexpr u32 QP = 1u << QB;
    const u32 t = b & (QP - 1u);
    const u32 m = (t < QP - t ? t : QP - t) & QMAG;
    return (t >= QP / 2u + 1u ? 0x80u : 0u) | m;
}
// Byte transpose inside a quad of lanes (the four lanes of positions 4q .. 4q + 3 of a word,
// which lane_pos keeps together): lane k of the quad holds the dword of those positions of
// "combination" k (frame, word, ...); afterwards byte c of every lane is combination c's byte
// at the lane's own position. Two quad-perm DPP moves and two v_perm with per-lane selectors.
struct QuadSel {
    u32 s1, s2;
    __device__ __forceinline__ void init(u32 pl)
    {
        const u32 k = pl & 3u, m = lane_pos(pl) & 3u;
        // round 1: [x_k[m], x_k^1[m], x_k[m ^ 2], x_k^1[m ^ 2]] from (own = bytes 0..3, partner = 4..7)
        s1 = m | ((4u + m) << 8) | ((m ^ 2u) << 16) | ((4u + (m ^ 2u)) << 24);
        // round 2: byte k <- y[0], k ^ 1 <- y[1], k ^ 2 <- partner y[2] (6), k ^ 3 <- partner y[3] (7)
        s2 = (0u << (8 * k)) | (1u << (8 * (k ^ 1u))) | (6u << (8 * (k ^ 2u))) | (7u << (8 * (k ^ 3u)));
    }
};
__device__ __forceinline__ u32 quad_transpose(u32 x, const QuadSel &q)
{
    const u32 t1 = __builtin_amdgcn_update_dpp(0u, x, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
    const u32 y = __builtin_amdgcn_perm(t1, x, q.s1);
    const u32 t2 = __builtin_amdgcn_update_dpp(0u, y, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
    return __builtin_amdgcn_perm(t2, y, q.s2);
}

// two SM8 bytes (low byte of lo, low byte of hi) -> SM16 pair: duplicate each byte into both
// bytes of its half, keep bit 15 and bits 0..4
__device__ __forceinline__ u32 sm8_pair(u32 lo, u32 hi)
{
    return __builtin_amdgcn_perm(hi, lo, 0x04040000u) & ((0x8000u | QMAG) * 0x00010001u);
}

// ---------------------------------------------------------------------------------------
// Leaf in split form (per-mask kernels): M = magnitudes (u16 pair), S = sign masks (0xFFFF
// in a negative half), frozen pattern FB known at compile time. Same recursion and results
// as leaf_rec with every frozen-pattern decision resolved statically:
//   F : M = min(M, M'), S = S ^ S'
//   G : x = S_F ^ U (signs of a' and b differ; S_F = S ^ S' is the F sign, U the partner's
//       partial sums as masks), |a| < |b| from M' - M, magnitude = x ? |M' - M| : M' + M,
//       sign = S ^ (x & ~lt)   (same signs -> sign(b); differ -> lt ? sign(b) : sign(a'))
// Returns x as 16-bit masks (0xFFFF = bit 1).
// ---------------------------------------------------------------------------------------
template <u32 FB, int B, int W>
__device__ __forceinline__ u32 leaf_ms(u32 M, u32 S, const Lanes &ln)
{
    constexpr u32 bm = ((1u << W) - 1u) << B;
    constexpr u32 sub = FB & bm;
    if constexpr (sub == 0u) {
        return 0u;
    } else if constexpr (sub == bm) {
        return S;
    } else if constexpr (W == 2) {
        if constexpr ((sub >> B) == 1u) {
            return (S ^ xorlane<1>(S)) & ln.a1;                 // (1, 0): x = [sa ^ sb, 0]
        } else {
            const u32 PM = xorlane<1>(M), PS = xorlane<1>(S);    // (0, 1): x = [u1, u1]
            const u32 lt = pk_sra(pk_sub(PM, M), 15);
            const u32 u1 = bselo(lt, S, PS);                     // valid on the b lane
            return bselo(ln.a1, xorlane<1>(u1), u1);
        }
    } else {
        constexpr int H = W / 2;
        const u32 PM = xorlane<H>(M), PS = xorlane<H>(S);
        const u32 SF = S ^ PS;
        const u32 Mf = pk_min(M, PM);
        const u32 xa = leaf_ms<FB, B, H>(Mf, SF, ln);
        const u32 x = opaque(SF ^ xorlane<H>(xa));
        const u32 lt = opaque(pk_sra(pk_sub(PM, M), 15));
        // magnitude: signs differ -> max - min, else max + min  (min = the F magnitude)
        // (EXTENDED = 0: Function_G's clamp inside the leaf too, as leaf_dp)
        u32 Mb = pk_mad_u16(Mf, x | 0x00010001u, pk_max_u16(M, PM));
        if constexpr (!EXT) Mb = pk_min(Mb, GSAT2);
        const u32 xb = leaf_ms<FB, B + H, H>(Mb, S ^ (x & ~lt), ln);
        return bselo(ln.template amask<H>(), xa ^ xorlane<H>(xb), xb);
    }
}

// A generated leaf record (polar_sc_op.fb: frozen pattern in bits 0..15, PRUNING_LEVEL 1
// decoder in bits 16..18): the plain leaf, or the REP / SPC / REP2 / SPC2 row decoders of the
// interpreter (leaf_kind_dp, SIGMAG) on the SM16 word of the split operands. Same output
// convention as leaf_ms (16-bit masks).
template <u32 FB>
__device__ __forceinline__ u32 leaf_gen(u32 M, u32 S, const Lanes &ln)
{
    constexpr u32 KIND = (FB >> 16) & 7u;
    static_assert(KIND <= 4, "POLAR_LEAF_R1 is a CA2 decoder");
    if constexpr (KIND == 0) {
        return leaf_ms<FB & 0xFFFFu, 0, 16>(M, S, ln);
    } else {
        const u32 L = M | (S & SGN);
        u32 x;
        if constexpr (KIND == 1) x = leaf_rep(L, ln);
        else if constexpr (KIND == 2) x = leaf_spc<false>(L, ln);
        else if constexpr (KIND == 3) x = leaf_rep2(L, ln);
        else x = leaf_spc<true>(L, ln);
        return pk_sra(x, 15);
    }
}

// packed root magnitudes of the per-mask kernels: the low / high byte of each 16-bit half
__device__ __forceinline__ u32 rlo(u32 p) { return p & 0x00FF00FFu; }
__device__ __forceinline__ u32 rhi(u32 p) { return __builtin_amdgcn_perm(p, p, 0x0C030C01u); }

// SM16 pair with magnitudes <= 31 -> two SM8 bytes (low frame in bits 0..7, high frame in
// bits 8..15); inverse of sm8_pair
__device__ __forceinline__ u32 sm16_to_sm8x2(u32 v)
{
    const u32 t = (v & (QMAG * 0x00010001u)) | ((v >> 8) & 0x00800080u);   // SM8 in bytes 0 and 2
    return __builtin_amdgcn_perm(t, t, 0x0C0C0200u);              // bytes [0, 2] -> [0, 1]
}

// ---------------------------------------------------------------------------------------
// Split stage words (per-mask kernels): magnitudes as u16 pairs (M) and the signs of 16
// words packed in one "plane" dword (bit i = low frame of word i, bit 16 + i = high frame),
// the same layout as the partial sums. F is then one v_pk_min per word plus one XOR per
// 16 words; G needs the sign plane only as a mask per word (2 ops) and emits the
// |a| < |b| flags back into a plane.
// ---------------------------------------------------------------------------------------
// bit I of each half of plane p -> 0xFFFF / 0 per half
template <int I>
__device__ __forceinline__ u32 plane_mask(u32 p)
{
    return pk_sra(pk_shl(p, (unsigned short)(15 - I)), 15);
}
// bits 15 / 31 of v -> bits I / 16 + I of the plane
template <int I>
__device__ __forceinline__ u32 plane_put(u32 acc, u32 v)
{
    return ((v >> (15 - I)) & (0x00010001u << I)) | acc;
}
// F on the channel (SM16 in, split out)
template <int I>
__device__ __forceinline__ u32 F_root(u32 a, u32 b, u32 &S)
{
    S = plane_put<I>(S, a ^ b);
    return pk_min(a & MAG, b & MAG);
}
// G on the channel (SM16 in, split out): G_sm<15> with the sign emitted into a plane
template <int I>
__device__ __forceinline__ u32 G_root(u32 a, u32 b, u32 u, u32 &S)
{
    const u32 ma = a & MAG, mb = b & MAG;
    const u32 d = pk_sub(ma, mb);
    const u32 x = a ^ u ^ b;
    S = plane_put<I>(S, b ^ (x & ~d));
    return pk_min(bsel(opaque(pk_sra(x, 15)), pk_abs_i16(d), pk_add(ma, mb)), GSAT2);
}
// G on split words: X = plane of sign(a') ^ sign(b); returns the clamped magnitude and puts
// |a| < |b| into LT. The output sign plane is then sign(b) ^ (X & ~LT) per 16 words.
template <int I>
__device__ __forceinline__ u32 G_split(u32 ma, u32 mb, u32 X, u32 &LT)
{
    const u32 xm = opaque(plane_mask<I>(X));
    const u32 d = pk_sub(ma, mb);
    LT = plane_put<I>(LT, d);
    return pk_min(bsel(xm, pk_abs_i16(d), pk_add(ma, mb)), GSAT2);
}
// REP word from split parent words: F value + 512 per half, and its SM16 form
template <int I>
__device__ __forceinline__ u32 F_split_biased(u32 ma, u32 mb, u32 FS)
{
    const u32 m = pk_min(ma, mb), s = plane_mask<I>(FS);
    return pk_add(pk_sub(m ^ s, s), 0x02000200u);
}
template <int I>
__device__ __forceinline__ u32 F_split_sm(u32 ma, u32 mb, u32 FS)
{
    return pk_min(ma, mb) | (plane_mask<I>(FS) & SGN);
}

// ---------------------------------------------------------------------------------------
// CA2 (config.h:11) on the split / SM16 forms of the generated pair kernels (POLAR_CA2). The
// two's complement values are kept as magnitude + sign, with two conventions
// (functions.h:48-118; F_function_C2, G_function_C2, G_simplified_C2):
//   * a zero magnitude is the value 0 whatever its sign bit: F_function_C2 / G_function_C2
//     never make a -0, the ops below read such a sign as don't-care, and hard decisions mask
//     it (ca2_nzs);
//   * MIN of width w, -2^(w-1) -- the pattern qabs leaves negative (scalar.h:42-49) -- is
//     magnitude 2^(w-1) with the sign set. F_function_C2 returns it whenever an operand is MIN
//     (the signed min takes the negative qabs, and its negation wraps to itself). Only the
//     leftmost path can hold MIN (the channel, then F of F ...: G_function_C2 saturates to
//     +-(2^(Q-1) - 1)) and the first PAR word, where G_extended_C2 of two MINs is the MIN one
//     bit wider; the generators give those F ops the key min below (MIN -> key 0).
// G_function_C2 / G_extended_C2 are the SIGMAG split code with the CA2 clamp (GSAT): b + a'
// has magnitude |mb +- ma|, and the SM sign rule gives its sign whenever it is not 0.
// ---------------------------------------------------------------------------------------
// sign masks S (0xFFFF per negative half) of the values (M, S) with the zeros made positive
// (the 1 hidden from the optimiser: it rewrites min(M, 1) as M != 0, v_cmp + v_cndmask per half
// + v_perm, 6 instructions for 1)
__device__ __forceinline__ u32 ca2_nzs(u32 M, u32 S) { return pk_mul_lo(pk_min(M, opaque(0x00010001u)), S); }
// bit 15 / 31 set where the magnitude is not 0 (hard decision mask of an SM16 pair)
__device__ __forceinline__ u32 ca2_nz(u32 m) { return pk_sub(0u, m & MAG); }
// F_function_C2 magnitude at width MW: min over m ^ 2^(MW-1) (MIN -> 0, m < 2^(MW-1) -> m + 2^(MW-1))
template <int MW>
__device__ __forceinline__ u32 pk_min_key(u32 a, u32 b)
{
    constexpr u32 K2 = (1u << (MW - 1)) * 0x00010001u;
    return pk_min(a ^ K2, b ^ K2) ^ K2;
}
// bit 15 / 31 set where an F_function_C2 magnitude of width MW is MIN (magnitudes <= 2^(MW-1))
template <int MW>
__device__ __forceinline__ u32 ca2_minbit(u32 m) { return pk_add(m, (0x8000u - (1u << (MW - 1))) * 0x00010001u); }
// F_function_C2 on SM16 pairs of width MW (the result's sign: MIN, else the xor; 0 don't-care)
template <int MW>
__device__ __forceinline__ u32 F_ca2(u32 a, u32 b)
{
    const u32 m = pk_min_key<MW>(a & MAG, b & MAG);
    return m | (((a ^ b) | ca2_minbit<MW>(m)) & SGN);
}
// F_root / F on split words / the REP value with MIN absorbing (the leftmost path)
template <int I, int MW>
__device__ __forceinline__ u32 F_root_min(u32 a, u32 b, u32 &S)
{
    const u32 m = pk_min_key<MW>(a & MAG, b & MAG);
    S = plane_put<I>(S, (a ^ b) | ca2_minbit<MW>(m));
    return m;
}
template <int I, int MW>
__device__ __forceinline__ u32 F_split_min(u32 ma, u32 mb, u32 &MP)
{
    const u32 m = pk_min_key<MW>(ma, mb);
    MP = plane_put<I>(MP, ca2_minbit<MW>(m));
    return m;
}
template <int I, int MW>
__device__ __forceinline__ u32 F_split_biased_min(u32 ma, u32 mb, u32 FS)
{
    const u32 m = pk_min_key<MW>(ma, mb), s = plane_mask<I>(FS) | pk_sra(ca2_minbit<MW>(m), 15);
    return pk_add(pk_sub(m ^ s, s), 0x02000200u);
}
// channel pair (16-bit halves, low Q bits two's complement) -> SM16: qconv_format (SIGMAG,
// conv_pair) or, CA2, the value itself as magnitude + sign (Adapt_format leaves it, library.h:18-28)
__device__ __forceinline__ u32 chan_sm16(u32 raw)
{
    if constexpr (CA2) {
        constexpr u32 QM = (1u << QB) - 1u, QP = 1u << QB;
        const u32 t = raw & (QM * 0x00010001u), s = (t << (16 - QB)) & SGN;
        return s | bsel(pk_sra(s, 15), pk_sub(QP * 0x00010001u, t), t);
    } else {
        return conv_pair(raw);
    }
}

// An all-information block of a CA2 leaf without MIN: its SC decisions depend on the signs and
// zeros of its LLRs only. With u = the left decisions, G never cancels (a nonzero F value decides
// its sign xor, so a' takes the sign of b; with a zero F value one operand is 0): the G value is
// 0 iff both operands are, else it has b's sign, or a' = sign(a) ^ u when b is 0. So the
// recursion runs on (sign, zero) masks: F = (sa ^ sb, za | zb), G = (zb ? sa ^ u : sb, za & zb),
// a 2-LLR block decides its true signs. Checked exhaustively against the SC recursion for 4 LLRs
// in [-3, 3] and 8 LLRs in [-2, 2], and on the device against the FSM (tests/test_ca2.py).
// S: sign masks (don't-care on zeros), Z: 0xFFFF where the magnitude is 0.
template <int W>
__device__ __forceinline__ u32 ca2_allinfo(u32 S, u32 Z, const Lanes &ln)
{
    if constexpr (W == 2) {
        return S & ~Z;
    } else {
        constexpr int H = W / 2;
        const u32 PS = xorlane<H>(S), PZ = xorlane<H>(Z);
        const u32 xa = ca2_allinfo<H>(S ^ PS, Z | PZ, ln);               // valid on a-lanes
        const u32 u = xorlane<H>(xa);                                     // (b-lanes: S = sb, PS = sa)
        const u32 xb = ca2_allinfo<H>(bselo(Z, PS ^ u, S), Z & PZ, ln);  // valid on b-lanes
        return bselo(ln.template amask<H>(), xa ^ xorlane<H>(xb), xb);
    }
}

// Leaf Spec_P16_ext / Spec_P16 in CA2 (functions.h:366-546 with F_function_C2, G_extended_C2
// or G_function_C2, F_simplified_C2 / G_simplified_C2, :89-118) on split words with the
// conventions above (the recursion of functions.h:413-492). MW != 0: the leaf can hold
// MIN of width MW (the first PAR word), its F ops take the key min and its exact G children
// MIN one bit wider. Unlike SIGMAG an all-information block of 4+ LLRs is not its hard
// decisions (a zero F value decides 0, not the sign xor): without MIN it takes ca2_allinfo.
template <u32 FB, int B, int W, int MW>
__device__ __forceinline__ u32 leaf_ca2(u32 M, u32 S, const Lanes &ln)
{
    constexpr u32 bm = ((1u << W) - 1u) << B;
    constexpr u32 sub = FB & bm;
    if constexpr (sub == 0u) {
        return 0u;
    } else if constexpr (sub == bm && W >= 4 && MW == 0) {
        return ca2_allinfo<W>(S, opaque(pk_sra(pk_sub(M, 0x00010001u), 15)), ln);   // (zero masks: M - 1 < 0)
    } else if constexpr (W == 2) {
        if constexpr (sub == bm) {
            return ca2_nzs(M, S);                                  // x = (sign a, sign b)
        } else if constexpr ((sub >> B) == 1u) {
            const u32 T = ca2_nzs(M, S);                           // (1, 0): x = [sa ^ sb, 0]
            return (T ^ xorlane<1>(T)) & ln.a1;
        } else {
            const u32 v = pk_sub(M ^ S, S);                        // (0, 1): x = [u1, u1], u1 = a + b < 0
            return pk_sra(pk_add(v, xorlane<1>(v)), 15);
        }
    } else {
        constexpr int H = W / 2;
        const u32 PM = xorlane<H>(M), PS = xorlane<H>(S);
        const u32 SX = S ^ PS;
        u32 Mf, SF;
        if constexpr (MW != 0) {
            Mf = pk_min_key<MW>(M, PM);
            SF = SX | pk_sra(ca2_minbit<MW>(Mf), 15);
        } else {
            Mf = pk_min(M, PM);
            SF = SX;
        }
        const u32 xa = leaf_ca2<FB, B, H, MW>(Mf, SF, ln);
        const u32 x = opaque(SX ^ xorlane<H>(xa));                 // sign(a') ^ sign(b)
        const u32 lt = opaque(pk_sra(pk_sub(PM, M), 15));
        u32 Mb = pk_mad_u16(MW != 0 ? pk_min(M, PM) : Mf, x | 0x00010001u, pk_max_u16(M, PM));
        if constexpr (!EXT) Mb = pk_min(Mb, GSAT2);
        const u32 xb = leaf_ca2<FB, B + H, H, (MW != 0 && EXT) ? MW + 1 : 0>(Mb, S ^ (x & ~lt), ln);
        return bselo(ln.template amask<H>(), xa ^ xorlane<H>(xb), xb);
    }
}

// ---------------------------------------------------------------------------------------
// REP nodes (Spec_REP, functions.h:3086-3107) -- value path. The reference decision is the
// sign of acc = sat511(... sat511(T_1 + sat511(T_0 + 0)) ...) where T_w is the exact
// pair-tree sum of word w. Every step is an exact sum or a clamp, so the two's-complement
// chain below carries the same value; only a zero total needs the SM sign-of-zero rule,
// which the caller resolves with the exact SM path (rep_exact_*).
// ---------------------------------------------------------------------------------------
// row total in every lane (rotation butterfly; 32-bit adds take the DPP operand directly)
__device__ __forceinline__ u32 row_sum_biased(u32 v)
{
    v += __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xF, 0xF, true);   // row_ror:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x124, 0xF, 0xF, true);   // row_ror:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x122, 0xF, 0xF, true);   // row_ror:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x121, 0xF, 0xF, true);   // row_ror:1
    return v;
}
// acc = clamp(acc + T, -511, 511) with T = row total - 16 * 512 (two's complement halves)
__device__ __forceinline__ u32 rep_acc(u32 acc, u32 total_biased)
{
    if constexpr (CA2 && REPSAT >= 0x4000u) {
        // CA2 with LLR_BITS 9 at PAR 64: |acc| <= 2^15 - 1 plus a PAR word's total overflows
        // the 16-bit half; the saturating packed add (v_pk_add_i16 clamp) then the symmetric
        // bound is the clamp of the exact sum (qadd, functions.h:63-75)
        const i16x2 t = __builtin_bit_cast(i16x2, pk_sub(total_biased, 0x20002000u));
        i16x2 v = __builtin_elementwise_add_sat(__builtin_bit_cast(i16x2, acc), t);
        v = __builtin_elementwise_max(v, (i16x2){(short)-(int)REPSAT, (short)-(int)REPSAT});
        return __builtin_bit_cast(u32, v);
    }
    u32 t = pk_sub(pk_add(acc, total_biased), 0x20002000u);
    i16x2 v = __builtin_bit_cast(i16x2, t);
    v = __builtin_elementwise_min(v, (i16x2){(short)REPSAT, (short)REPSAT});
    v = __builtin_elementwise_max(v, (i16x2){(short)-(int)REPSAT, (short)-(int)REPSAT});
    return __builtin_bit_cast(u32, v);
}
// true if some frame of the wave ended with a zero accumulator
__device__ __forceinline__ bool rep_any_zero(u32 acc)
{
    const bool z = ((acc & 0xFFFFu) == 0u) || ((acc >> 16) == 0u);
    return __builtin_amdgcn_ballot_w64(z) != 0ull;
}

// ---------------------------------------------------------------------------------------
// Format-generic datapath of the schedule interpreter (polar_sc_interp.h): SIGMAG on SM16
// halves, or CA2 on i16 halves (config.h:11). The per-mask / generated-subtree kernels keep
// the SIGMAG-only split-word code above; plans of any other format run the interpreter
// compiled by hipRTC with their POLAR_* switches.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ u32 pk_min_i16(u32 a, u32 b)
{
    return __builtin_bit_cast(u32, __builtin_elementwise_min(__builtin_bit_cast(i16x2, a), __builtin_bit_cast(i16x2, b)));
}
__device__ __forceinline__ u32 pk_max_i16(u32 a, u32 b)
{
    return __builtin_bit_cast(u32, __builtin_elementwise_max(__builtin_bit_cast(i16x2, a), __builtin_bit_cast(i16x2, b)));
}
// both halves sign-extended from their low w bits (w-bit two's complement wrap)
__device__ __forceinline__ u32 sext_w(u32 v, int w)
{
    const short s = (short)(16 - w);
    return pk_sra(pk_shl(v, (unsigned short)s), s);
}
// qabs<w> (scalar.h:42-49): -v in w bits, so qabs(-2^(w-1)) = -2^(w-1)
__device__ __forceinline__ u32 ca2_qabs(u32 v, int w) { return sext_w(pk_abs_i16(v), w); }
// F_function_C2 (functions.h:48-61) at width w: signed min of the qabs values, negated in w
// bits when the signs differ
__device__ __forceinline__ u32 ca2_F(u32 a, u32 b, int w)
{
    const u32 mn = pk_min_i16(ca2_qabs(a, w), ca2_qabs(b, w));
    const u32 m = pk_sra(a ^ b, 15);
    return sext_w(pk_sub(mn ^ m, m), w);
}
// G_function_C2 / G_extended_C2 (functions.h:63-87): u flags (bits 15 / 31): b - a, else
// b + a; SAT != 0: qsat to +-SAT
template <u32 SAT>
__device__ __forceinline__ u32 ca2_G(u32 a, u32 b, u32 u)
{
    const u32 m = pk_sra(u & SGN, 15);
    u32 d = pk_add(b, pk_sub(a ^ m, m));
    if constexpr (SAT != 0) d = pk_min_i16(pk_max_i16(d, (0x10000u - SAT) * 0x00010001u), SAT * 0x00010001u);
    return d;
}

// Function_F / Function_G of the configured format (functions.h:287-308). w: width of the
// operands (CA2 only: the qabs wrap point); stage values are QB bits wide, exact leaf
// levels one bit wider per G_extended above them.
__device__ __forceinline__ u32 dp_F(u32 a, u32 b, int w)
{
    if constexpr (CA2) return ca2_F(a, b, w);
    else return F_sm(a, b);
}
template <bool SAT>
__device__ __forceinline__ u32 dp_G(u32 a, u32 b, u32 u)
{
    if constexpr (CA2) return ca2_G<SAT ? GSAT : 0u>(a, b, u);
    else return G_sm<SAT ? GSAT : 0>(a, b, u);
}
// channel word: raw = two LLRs (16-bit halves, sign-extended from the input type) ->
// wrapper_in + Adapt_format (library.h:18-28): qconv_format (SIGMAG) or unchanged (CA2)
__device__ __forceinline__ u32 dp_chan(u32 raw)
{
    if constexpr (CA2) return sext_w(raw, QB);
    else return conv_pair(raw);
}
// HBM stage slots: two 8-bit values per lane (SM8 pairs / int8 pairs), or (9-bit LLRs) the
// 32-bit register as is
__device__ __forceinline__ u32 slot_unpack(u32 h)
{
    if constexpr (CA2) return pk_sra(__builtin_amdgcn_perm(h, h, 0x010C000Cu), 8);   // bytes 0,1 -> 1,3
    else return sm8_pair(h, h >> 8);
}
__device__ __forceinline__ u32 slot_pack(u32 v)
{
    if constexpr (CA2) return __builtin_amdgcn_perm(v, v, 0x0C0C0200u);             // bytes 0,2 -> 0,1
    else return sm16_to_sm8x2(v);
}

// Spec_Polar_Decoder on one 16-LLR word with run-time frozen pattern, both formats, exact
// (EXTENDED = 1: G_extended, widths grow) or saturating (EXTENDED = 0: Function_G at Q)
// (functions.h:354-760). w: width of the leaf's input values. An all-frozen block decodes to
// 0; an all-information block to its hard decisions only in SIGMAG (CA2 F has no -0).
template <int B, int W>
__device__ __forceinline__ u32 leaf_dp(u32 L, u32 fb, u32 fbm, const Lanes &ln, int w)
{
    constexpr u32 bm = ((1u << W) - 1u) << B;
    const u32 sub = fb & bm;
    if (sub == 0u) return 0u;
    if (!CA2 && sub == bm) return L & SGN;
    if constexpr (W == 2) {
        // Spec_P2 (functions.h:366-384): lane B = a, lane B+1 = b
        u32 P = xorlane<1>(L);
        u32 u0 = (L ^ P) & fbm;                   // F_simplified & fb[B]   (valid on a)
        u32 u0p = xorlane<1>(u0);
        u32 u1;
        if constexpr (CA2) {
            u1 = ca2_G<0>(P, L, u0p) & fbm;       // sign of b -+ a         (on b)
        } else {
            u32 d = pk_sub(P & MAG, L & MAG);     // |a| < |b|              (on b)
            u1 = bsel(d, L, P ^ u0p) & fbm;       // G_simplified & fb[B+1] (valid on b)
        }
        u32 u1p = xorlane<1>(u1);
        return bsel(ln.a1, u0 ^ u1p, u1);
    } else {
        constexpr int H = W / 2;
        u32 P = xorlane<H>(L);
        u32 La = dp_F(L, P, w);                              // valid on a-lanes
        u32 xa = leaf_dp<B, H>(La, fb, fbm, ln, w);
        u32 Lb = dp_G<!EXT>(P, L, xorlane<H>(xa));            // valid on b-lanes
        u32 xb = leaf_dp<B + H, H>(Lb, fb, fbm, ln, EXT ? w + 1 : w);
        return bsel(ln.template amask<H>(), xa ^ xorlane<H>(xb), xb);
    }
}

__device__ __forceinline__ u32 leaf16_dp(u32 L, u32 fb, const Lanes &ln, int w)
{
    u32 fbm = ((fb >> ln.pos) & 1u) ? SGN : 0u;   // the frozen bit of this lane's word position
    return leaf_dp<0, 16>(L, fb, fbm, ln, w);
}

// 32-bit row sum (every lane gets the total of its 16-lane row)
__device__ __forceinline__ u32 row_sum32(u32 v)
{
    v += __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xF, 0xF, true);   // row_ror:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x124, 0xF, 0xF, true);   // row_ror:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x122, 0xF, 0xF, true);   // row_ror:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x121, 0xF, 0xF, true);   // row_ror:1
    return v;
}
// the two halves as signed 32-bit values (two's complement value; SIGMAG converted)
__device__ __forceinline__ int val_lo(u32 v)
{
    if constexpr (CA2) return (int)(short)(v & 0xFFFFu);
    else return (v & 0x8000u) ? -(int)(v & 0x7FFFu) : (int)(v & 0x7FFFu);
}
__device__ __forceinline__ int val_hi(u32 v) { return val_lo(v >> 16); }
// ---------------------------------------------------------------------------------------
// PAR words, SPC keys and the PAR 4 / 8 device-word decoder (schedule interpreter and
// generated pair kernels)
// ---------------------------------------------------------------------------------------
// bit reversal of the low `bits` bits
__device__ __forceinline__ u32 bitrev_n(u32 v, int bits)
{
    return bits ? (__builtin_bitreverse32(v) >> (32 - bits)) : 0u;
}
// SPC search key of device word i (the lane's bitrev4 position is ORed in later, shifted by
// LPAR - 4): PAR word index, then bitrev_{LPAR}(position in the PAR word) -- the order of the
// Min_Mask_{PAR} tournament within a PAR word plus the strict '<' across PAR words
// PAR < 16: the PAR words of device word i are its lane groups: key i << 4, the lane part
// (spc_lane_key) carries the group and bitrev_{LPAR}(position in the group)
__device__ __forceinline__ u32 spc_word_key(int i)
{
    if constexpr (LPAR < 4) return (u32)i << 4;
    else return ((u32)(i / P16) << LPAR) | bitrev_n((u32)(i % P16), LPAR - 4);
}
// device word of a min key
__device__ __forceinline__ int spc_key_word(u32 key)
{
    const u32 k = key & 0xFFFFFFu;
    if constexpr (LPAR < 4) return (int)(k >> 4);
    else return (int)((k >> LPAR) * P16 + bitrev_n(k & (u32)(P16 - 1), LPAR - 4));
}
// the lane's part of an SPC key and the mask that isolates it
__device__ __forceinline__ u32 spc_lane_key(const Lanes &ln)
{
    if constexpr (LPAR < 4)
        return (ln.pos & ~(u32)((1 << LPAR) - 1)) | bitrev_n(ln.pos & (u32)((1 << LPAR) - 1), LPAR);
    else
        return ln.br << (LPAR - 4);
}
constexpr u32 SPC_LANE_BITS = LPAR < 4 ? 15u : (15u << (LPAR - 4));
// |lambda| of a (saturated) G output as the SPC trees compare it (VECTOR_ABS_SM / qabs)
__device__ __forceinline__ u32 spc_mag(u32 lam)
{
    if constexpr (CA2) return pk_abs_i16(lam);
    else return lam & MAG;
}

constexpr bool DEFAULT_FMT = !CA2 && LPAR == 4 && QB <= 8;
constexpr int PARW = 1 << LPAR;   // PAR in lanes (PAR < 16: a lane group of a device word)

// ---------------------------------------------------------------------------------------
// PAR 4 / 8 (LPAR < 4): PPW PAR words share a device word as aligned lane groups
// ---------------------------------------------------------------------------------------
// one level of the exact pair tree ADD_TREE_{PAR} (functions.h:3036-3083): partners at position
// distance D, the lower lane as operand a; butterfly, so both partners hold the pair total
template <int D>
__device__ __forceinline__ u32 tree_step(u32 v, const Lanes &ln)
{
    const u32 p = xorlane<D>(v);
    if constexpr (CA2) return pk_add(v, p);
    else return G_sm<0>(bsel(ln.template amask<D>(), v, p), bsel(ln.template amask<D>(), p, v), 0u);
}
// pair-tree levels at distances W/2 .. DMIN (DMIN 2: REP2, the even / odd classes)
template <int W, int DMIN>
__device__ __forceinline__ u32 add_tree_w(u32 v, const Lanes &ln)
{
    if constexpr (W / 2 >= DMIN) return add_tree_w<W / 2, DMIN>(tree_step<W / 2>(v, ln), ln);
    else return v;
}
template <int W, int DMIN>
__device__ __forceinline__ u32 xor_tree_w(u32 v)
{
    if constexpr (W / 2 >= DMIN) return xor_tree_w<W / 2, DMIN>(v ^ xorlane<W / 2>(v));
    else return v;
}
template <int W, int DMIN>
__device__ __forceinline__ u32 min_tree_w(u32 v)
{
    if constexpr (W / 2 >= DMIN) return min_tree_w<W / 2, DMIN>(__builtin_elementwise_min(v, xorlane<W / 2>(v)));
    else return v;
}
// REP accumulator step (ADDER_TREE_{PAR} accumulate, functions.h:3163-3320): acc + T,
// saturated at REPSAT (SIGMAG: qfull_adder_sat_sm; CA2: qadd)
__device__ __forceinline__ u32 rep_sat_add(u32 acc, u32 t)
{
    if constexpr (CA2) {
        const u32 d = pk_add(acc, t);
        return pk_min_i16(pk_max_i16(d, (0x10000u - REPSAT) * 0x00010001u), REPSAT * 0x00010001u);
    } else {
        return G_sm<REPSAT>(t, acc, 0u);
    }
}
// the saturating chain over CNT consecutive lane groups (PARW lanes each) in group order;
// t = each lane's group total, gr = the lane's group index relative to the first one
template <int CNT>
__device__ __forceinline__ u32 group_chain(u32 acc, u32 t, u32 gr)
{
    if constexpr (CNT == 1) {
        return rep_sat_add(acc, t);
    } else if constexpr (CNT == 2) {
        const u32 o = xorlane<PARW>(t);
        acc = rep_sat_add(acc, (gr & 1u) ? o : t);
        return rep_sat_add(acc, (gr & 1u) ? t : o);
    } else {   // CNT == 4 (PAR 4, a whole word): the totals of groups gr ^ 1, ^ 2, ^ 3
        u32 v[4];
        v[0] = t;
        v[1] = xorlane<PARW>(t);
        v[2] = xorlane<2 * PARW>(t);
        v[3] = xorlane<PARW>(v[2]);
#pragma unroll
        for (u32 j = 0; j < 4; j++) {
            const u32 k = (gr & 3u) ^ j;
            acc = rep_sat_add(acc, k == 0 ? v[0] : k == 1 ? v[1] : k == 2 ? v[2] : v[3]);
        }
        return acc;
    }
}
// PRUNING_LEVEL 1 leaf decoders of one PAR word of W (= PAR) lanes (library.h:187-280):
// REP / REP2 / SPC / SPC2 / R1, as leaf_kind_dp over a lane group
template <int W>
__device__ __forceinline__ u32 leaf_kind_w(u32 L, u32 kind, const Lanes &ln, int w)
{
    if (kind == 5) return L & SGN;   // Spec_Node_R1: VECTOR_SIGN
    if (kind == 1) return add_tree_w<W, 1>(L, ln) & SGN;
    if (kind == 3) return add_tree_w<W, 2>(L, ln) & SGN;
    const bool spc2 = kind == 4;
    const u32 h = L & SGN;
    const u32 par = spc2 ? xor_tree_w<W, 2>(h) : xor_tree_w<W, 1>(h);
    u32 mg;
    if constexpr (CA2) mg = pk_add(ca2_qabs(L, w), (1u << (w - 1)) * 0x00010001u);   // order-preserving, >= 0
    else mg = L & 0x7FFF7FFFu;
    const u32 br = bitrev_n(ln.pos & (u32)(W - 1), LPAR);
    u32 klo = ((mg & 0xFFFFu) << 4) | br, khi = ((mg >> 16) << 4) | br;
    const u32 mlo0 = klo, mhi0 = khi;
    klo = spc2 ? min_tree_w<W, 2>(klo) : min_tree_w<W, 1>(klo);
    khi = spc2 ? min_tree_w<W, 2>(khi) : min_tree_w<W, 1>(khi);
    const u32 flo = (klo == mlo0) ? (par & 0x8000u) : 0u;
    const u32 fhi = (khi == mhi0) ? (par & 0x80000000u) : 0u;
    return h ^ flo ^ fhi;
}
// group classes of a word (the host's do_prunning result, polar_sc_host.cpp word_info):
// per group g, bits 7g..7g+3 = class (NODE_* codes), 7g+4..7g+6 = PR1 leaf kind; bit 28 =
// PRUNING_LEVEL 2
constexpr u32 WN_R0 = 0x00, WN_R1 = 0x0F, WN_REP = 0x02, WN_SPC = 0x04, WN_RN = 0x08;
__device__ __forceinline__ u32 wgroup_type(u32 info, int g) { return (info >> (7 * g)) & 15u; }
__device__ __forceinline__ u32 wgroup_kind(u32 info, int g) { return (info >> (7 * g + 4)) & 7u; }
// node class of groups [g0, g0 + cnt) as the F / G loops aggregate it (my_module.h:403-471,
// 739-806; polar_sc_host.cpp node_class)
__device__ __forceinline__ u32 wnode_class(u32 info, int g0, int cnt)
{
    u32 r0 = 0, r1 = 0x0F;
    bool r0_but_last = true, r1_but_first = true;
    for (int t = 0; t < cnt; t++) {
        const u32 T = wgroup_type(info, g0 + t);
        r0 |= T;
        r1 &= T;
        if (t + 1 < cnt && T != WN_R0) r0_but_last = false;
        if (t > 0 && T != WN_R1) r1_but_first = false;
    }
    if (r0 == WN_R0) return WN_R0;
    if (r1 == WN_R1) return WN_R1;
    if (r0_but_last && wgroup_type(info, g0 + cnt - 1) == WN_REP) return WN_REP;
    if (r1_but_first && wgroup_type(info, g0) == WN_SPC) return WN_SPC;
    return WN_RN;
}
// G_SPC_STATE on the W lanes of a node inside a word (my_module.h:1737-1842): hard decisions,
// parity over the node, flip at the minimum (|lambda|, group, bitrev_{LPAR}(position))
template <int W>
__device__ __forceinline__ u32 word_spc(u32 L, const Lanes &ln)
{
    const u32 h = L & SGN;
    const u32 par = xor_tree_w<W, 1>(h);
    const u32 mg = spc_mag(L), lk = spc_lane_key(ln);
    u32 klo = ((mg & 0xFFu) << 24) | lk, khi = (((mg >> 16) & 0xFFu) << 24) | lk;
    klo = min_tree_w<W, 1>(klo);
    khi = min_tree_w<W, 1>(khi);
    const u32 flo = ((par & 0x8000u) && (klo & 15u) == lk) ? 0x8000u : 0u;
    const u32 fhi = ((par & 0x80000000u) && (khi & 15u) == lk) ? 0x80000000u : 0u;
    return h ^ flo ^ fhi;
}
// the PAR-word leaf of group g at lanes [B, B + PAR): its PR1 decoder or Spec_P{PAR} exact
template <int B>
__device__ __forceinline__ u32 word_leaf(u32 L, u32 fb, u32 info, int g, const Lanes &ln)
{
    const u32 kind = wgroup_kind(info, g);
    if (kind) return leaf_kind_w<PARW>(L, kind, ln, QB);
    const u32 fbm = ((fb >> ln.pos) & 1u) ? SGN : 0u;
    return leaf_dp<B, PARW>(L, fb, fbm, ln, QB);
}
// compile_node (polar_sc_host.cpp) inside one device word: the node of W LLRs at lanes
// [B, B + W) (W / PAR >= 2 groups), its LLRs L valid on those lanes; returns x (sign-position
// flags) on the same lanes. F / G at these levels are the stage functions (G saturated), the
// PAR-word leaves exact; children pruned at PRUNING_LEVEL 2 as the FSM prunes them.
template <int B, int W>
__device__ u32 word_node(u32 L, u32 fb, u32 info, const Lanes &ln)
{
    constexpr int H = W / 2;               // child LLRs
    constexpr int h = (W >> LPAR) / 2;     // groups per child
    const int g0 = B >> LPAR;
    const bool prune = (info >> 28) & 1u;
    const u32 tl = prune ? wnode_class(info, g0, h) : WN_RN;
    const u32 tr = prune ? wnode_class(info, g0 + h, h) : WN_RN;
    const u32 P = xorlane<H>(L);      // the partner: on a-lanes b, on b-lanes a
    const u32 gr = (ln.pos >> LPAR) - (u32)g0;   // group of the lane relative to g0
    u32 xa = 0;
    const bool lz = tl == WN_R0;           // H0 route: no F, G with u = 0, then H0
    if (!lz) {
        const u32 La = dp_F(L, P, QB);   // valid on [B, B + H)
        if (tl == WN_REP) {
            xa = group_chain<h>(0u, add_tree_w<PARW, 1>(La, ln), gr) & SGN;   // F_REP_STATE
        } else {
            if constexpr (h == 1) xa = word_leaf<B>(La, fb, info, g0, ln);
            else xa = word_node<B, H>(La, fb, info, ln);
        }
    }
    const u32 Lb = dp_G<true>(P, L, lz ? 0u : xorlane<H>(xa));   // valid on [B + H, B + W)
    u32 xb;
    if (tr == WN_R1) {
        xb = Lb & SGN;                         // G_R1_STATE
    } else if (tr == WN_SPC) {
        xb = word_spc<H>(Lb, ln);              // G_SPC_STATE
    } else {
        if constexpr (h == 1) xb = word_leaf<B + H>(Lb, fb, info, g0 + 1, ln);
        else xb = word_node<B + H, H>(Lb, fb, info, ln);
    }
    const u32 xbp = xorlane<H>(xb);
    return bsel(ln.template amask<H>(), lz ? xbp : (xa ^ xbp), xb);
}


// The same decoder with the word's frozen bits and group classes known at compile time: the
// generated pair kernels of PAR 4 / 8 call it on every leaf record (FB = the word's frozen bits,
// INFO = polar_sc_host.cpp word_info), and every pruning decision above folds away.
constexpr u32 wg_type(u32 info, int g) { return (info >> (7 * g)) & 15u; }
constexpr u32 wg_kind(u32 info, int g) { return (info >> (7 * g + 4)) & 7u; }
constexpr u32 wn_class_ct(u32 info, int g0, int cnt)
{
    u32 r0 = 0, r1 = 0x0F;
    bool r0_but_last = true, r1_but_first = true;
    for (int t = 0; t < cnt; t++) {
        const u32 T = wg_type(info, g0 + t);
        r0 |= T;
        r1 &= T;
        if (t + 1 < cnt && T != WN_R0) r0_but_last = false;
        if (t > 0 && T != WN_R1) r1_but_first = false;
    }
    if (r0 == WN_R0) return WN_R0;
    if (r1 == WN_R1) return WN_R1;
    if (r0_but_last && wg_type(info, g0 + cnt - 1) == WN_REP) return WN_REP;
    if (r1_but_first && wg_type(info, g0) == WN_SPC) return WN_SPC;
    return WN_RN;
}
template <int B, u32 FB, u32 INFO>
__device__ __forceinline__ u32 word_leaf_gen(u32 L, const Lanes &ln)
{
    constexpr u32 kind = wg_kind(INFO, B >> LPAR);
    if constexpr (kind != 0u) return leaf_kind_w<PARW>(L, kind, ln, QB);
    else return leaf_dp<B, PARW>(L, FB, ((FB >> ln.pos) & 1u) ? SGN : 0u, ln, QB);
}
template <int B, int W, u32 FB, u32 INFO>
__device__ __forceinline__ u32 word_gen(u32 L, const Lanes &ln)
{
    constexpr int H = W / 2;               // child LLRs
    constexpr int h = (W >> LPAR) / 2;     // groups per child
    constexpr int g0 = B >> LPAR;
    constexpr bool prune = ((INFO >> 28) & 1u) != 0u;
    constexpr u32 tl = prune ? wn_class_ct(INFO, g0, h) : WN_RN;
    constexpr u32 tr = prune ? wn_class_ct(INFO, g0 + h, h) : WN_RN;
    constexpr bool lz = tl == WN_R0;       // H0 route
    const u32 P = xorlane<H>(L);
    u32 xa = 0;
    if constexpr (!lz) {
        const u32 La = dp_F(L, P, QB);
        if constexpr (tl == WN_REP) xa = group_chain<h>(0u, add_tree_w<PARW, 1>(La, ln), (ln.pos >> LPAR) - (u32)g0) & SGN;
        else if constexpr (h == 1) xa = word_leaf_gen<B, FB, INFO>(La, ln);
        else xa = word_gen<B, H, FB, INFO>(La, ln);
    }
    const u32 Lb = dp_G<true>(P, L, lz ? 0u : xorlane<H>(xa));
    u32 xb;
    if constexpr (tr == WN_R1) xb = Lb & SGN;
    else if constexpr (tr == WN_SPC) xb = word_spc<H>(Lb, ln);
    else if constexpr (h == 1) xb = word_leaf_gen<B + H, FB, INFO>(Lb, ln);
    else xb = word_gen<B + H, H, FB, INFO>(Lb, ln);
    const u32 xbp = xorlane<H>(xb);
    return bsel(ln.template amask<H>(), lz ? xbp : (xa ^ xbp), xb);
}
// a PAR 4 / 8 leaf record of the generated kernels on split operands (S: 16-bit sign masks):
// 16-bit masks like leaf_ms. CA2: the word tree runs on the two's complement values, which the
// split form gives back exactly (a zero's sign is don't-care: (0 ^ S) - S = 0; MIN = magnitude
// 2^(w-1) with the sign set -> -2^(w-1))
template <u32 FB, u32 INFO>
__device__ __forceinline__ u32 leaf_word_gen(u32 M, u32 S, const Lanes &ln)
{
    if constexpr (CA2) return pk_sra(word_gen<0, 16, FB, INFO>(pk_sub(M ^ S, S), ln), 15);
    else return pk_sra(word_gen<0, 16, FB, INFO>(M | (S & SGN), ln), 15);
}
// A CA2 leaf record of the generated kernels: leaf_ca2, or its PRUNING_LEVEL 1 decoder (fb bits
// 16..18: REP / SPC / REP2 / SPC2 / R1, the interpreter's leaf_kind_w on the two's complement
// word; the split form gives it back exactly, MIN included)
template <u32 FB, int MW>
__device__ __forceinline__ u32 leaf_gen_ca2(u32 M, u32 S, const Lanes &ln)
{
    constexpr u32 KIND = (FB >> 16) & 7u;
    if constexpr (KIND == 0) return leaf_ca2<FB & 0xFFFFu, 0, 16, MW>(M, S, ln);
    else return pk_sra(leaf_kind_w<16>(pk_sub(M ^ S, S), KIND, ln, QB), 15);
}
}  // namespace polar
