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

// ---------------------------------------------------------------------------------------
// packed 16-bit helpers (v_pk_* on gfx950)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ u32 U(u16x2 v) { return __builtin_bit_cast(u32, v); }
__device__ __forceinline__ u16x2 V(u32 v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ u32 pk_min(u32 a, u32 b) { return U(__builtin_elementwise_min(V(a), V(b))); }
__device__ __forceinline__ u32 pk_add(u32 a, u32 b) { return U(V(a) + V(b)); }
__device__ __forceinline__ u32 pk_sub(u32 a, u32 b) { return U(V(a) - V(b)); }
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
    u32 a2 = a ^ u;
    u32 ma = a & MAG, mb = b & MAG;
    u32 d = pk_sub(ma, mb);                   // bit 15 set iff |a| < |b|
    u32 sum = pk_add(ma, mb);
    u32 dif = pk_abs_i16(d);
    u32 dm = pk_sra(a2 ^ b, 15);              // 0xFFFF where signs differ
    u32 m = bsel(dm, dif, sum);
    if constexpr (SAT != 0) m = pk_min(m, (u32)SAT * 0x00010001u);
    u32 s = bsel(d, b, a2) & SGN;             // only bits 15/31 of the selector matter
    return s | m;
}

// ---------------------------------------------------------------------------------------
// cross-lane exchange inside a 16-lane DPP row: value of lane (l ^ H)
// ---------------------------------------------------------------------------------------
template <int H>
__device__ __forceinline__ u32 xorlane(u32 v)
{
    if constexpr (H == 1) {
        return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    } else if constexpr (H == 2) {
        return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    } else if constexpr (H == 4) {
        u32 t = __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, false);  // row_half_mirror: l^7
        return __builtin_amdgcn_mov_dpp(t, 0x1B, 0xF, 0xF, false);   // quad_perm [3,2,1,0]: ^3
    } else {
        static_assert(H == 8, "row partner distance");
        return __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false);  // row_ror:8
    }
}

// per-lane constants: all-ones where the lane is the lower ("a") member of its pair at
// distance H
struct Lanes {
    u32 a1, a2, a4, a8;   // lane masks
    u32 pl;               // PAR lane 0..15
    u32 br;               // bitrev4(pl)
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
        br = ((p & 1u) << 3) | ((p & 2u) << 1) | ((p & 4u) >> 1) | ((p & 8u) >> 3);
        a1 = (p & 1u) ? 0u : 0xFFFFFFFFu;
        a2 = (p & 2u) ? 0u : 0xFFFFFFFFu;
        a4 = (p & 4u) ? 0u : 0xFFFFFFFFu;
        a8 = (p & 8u) ? 0u : 0xFFFFFFFFu;
    }
};

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
    u32 fbm = ((fb >> ln.pl) & 1u) ? SGN : 0u;
    return leaf_rec<0, 16>(L, fb, fbm, ln);
}

// (b) frozen pattern FB known at compile time (per-mask kernels): the same recursion with
// every frozen-pattern decision resolved statically. Mixed 2-blocks are (1,0) -> x=[u0,0]
// and (0,1) -> x=[u1,u1] (F_simplified / G_simplified with the frozen lane's bit = 0).
template <u32 FB, int B, int W>
__device__ __forceinline__ u32 leaf_ct(u32 L, const Lanes &ln)
{
    constexpr u32 bm = ((1u << W) - 1u) << B;
    constexpr u32 sub = FB & bm;
    if constexpr (sub == 0u) {
        return 0u;
    } else if constexpr (sub == bm) {
        return L & SGN;
    } else if constexpr (W == 2) {
        u32 P = xorlane<1>(L);
        if constexpr ((sub >> B) == 1u) {
            // fb = (1, 0): u0 = sign(a) ^ sign(b), u1 = 0 -> x = [u0, 0]
            return ((L ^ P) & SGN) & ln.a1;
        } else {
            // fb = (0, 1): u0 = 0, u1 = |a| < |b| ? sign(b) : sign(a) -> x = [u1, u1]
            u32 d = pk_sub(P & MAG, L & MAG);
            u32 u1 = bsel(d, L, P) & SGN;        // valid on the b lane
            return bsel(ln.a1, xorlane<1>(u1), u1);
        }
    } else {
        constexpr int H = W / 2;
        u32 P = xorlane<H>(L);
        u32 xa = leaf_ct<FB, B, H>(F_sm(L, P), ln);
        u32 Lb = G_sm<0>(P, L, xorlane<H>(xa));
        u32 xb = leaf_ct<FB, B + H, H>(Lb, ln);
        return bsel(ln.template amask<H>(), xa ^ xorlane<H>(xb), xb);
    }
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
    p = xorlane<8>(v); v = bsel(ln.a8, (v & 0x00FF00FFu) | ((p & 0x00FF00FFu) << 8), ((p >> 8) & 0x00FF00FFu) | (v & 0xFF00FF00u));
    p = xorlane<4>(v); v = bsel(ln.a4, (v & 0x0F0F0F0Fu) | ((p & 0x0F0F0F0Fu) << 4), ((p >> 4) & 0x0F0F0F0Fu) | (v & 0xF0F0F0F0u));
    p = xorlane<2>(v); v = bsel(ln.a2, (v & 0x33333333u) | ((p & 0x33333333u) << 2), ((p >> 2) & 0x33333333u) | (v & 0xCCCCCCCCu));
    p = xorlane<1>(v); v = bsel(ln.a1, (v & 0x55555555u) | ((p & 0x55555555u) << 1), ((p >> 1) & 0x55555555u) | (v & 0xAAAAAAAAu));
    return v;
}

// ---------------------------------------------------------------------------------------
// Channel LLR -> SM16: wrapper_in + Adapt_format/qconv_format (wrapper_in.h:34,
// library.h:18-28, scalar.h:229-239). The LLR is the low 6 bits (sc_bigint<6>); -32 -> +0.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ u32 conv_half(int c)
{
    int t = (int)((u32)c << 26) >> 26;      // sign-extend 6 bits
    u32 m = (u32)(t < 0 ? -t : t) & 31u;
    u32 s = (t < 0 && m != 0u) ? 0x8000u : 0u;
    return m | s;
}

// raw = b_lo | b_hi << 16 (two int8 LLRs) -> SM16 pair
__device__ __forceinline__ u32 conv_pair(u32 raw)
{
    u32 t = pk_sra(pk_shl(raw, 10), 10);                     // sign-extend 6 bits per half
    u32 m = pk_abs_i16(t) & 0x001F001Fu;                     // |t|, -32 -> 0
    // sign iff t in [-31, -1]  <=>  x = t+31 in [0, 30]  <=>  x >= 0 && x - 31 < 0
    u32 x = pk_add(t, 0x001F001Fu);
    u32 w = pk_sub(x, 0x001F001Fu);
    return m | ((~x & w) & SGN);
}

}  // namespace polar
