// polar_sc_jit.cpp -- per-frozen-mask decode kernels, generated at plan time and compiled
// with hipRTC for gfx950.
//
// The reference is specialised per code the same way: Frozen_Bit_Generator writes the mask
// into polar_parameters.h and the HLS design is re-synthesised for it
// (Frozen_Bit_Generator/src/Writer.h:110-162, script/script_tests.sh:17-58). Here the
// compiled schedule (polar_sc_op list) is unrolled into straight-line HIP: every stage
// buffer is a register array with compile-time indices, every partial-sum position and
// every leaf frozen pattern is a constant, and there is no interpreter loop at all.
// Used for N <= 1024 (all stage buffers fit in VGPRs). Larger N use hybrid kernels: the
// schedule interpreter (polar_sc_interp.h) for the upper tree levels, with every mixed
// subtree of sub_words words (1024 LLRs by default) decoded by generated straight-line code
// of the same kind.
#include "polar_sc_plan.hpp"

#include <hip/hiprtc.h>

#include <dirent.h>
#include <dlfcn.h>
#include <elf.h>
#include <fcntl.h>
#include <signal.h>
#include <spawn.h>
#include <sys/stat.h>
#include <sys/wait.h>
extern char **environ;   // (POSIX: the environment handed to the spawned compiler)
#include <utime.h>
#include <zlib.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace {
// per-mask kernels: waves per block and the launch bound's minimum waves per SIMD. The
// register allocator targets 4 waves per SIMD (123 VGPRs at C2). Measured alternatives, all
// slower on the same box and removed: a persistent batch loop (78.9 vs 72.8 us), two batches
// per wave in straight-line code (80.9 vs 73.6 us), 1 / 2 waves per block (74.2 / 74.7 vs
// 73.7 us), re-splitting the root from LDS for the root G (77 vs 72 us) -- DESIGN.md 3.1.
constexpr int MASK_WPB = polar_host::MASK_WAVES_PER_BLOCK;
constexpr int MASK_MIN_WAVES = 4;
}  // namespace

namespace {
#include "polar_sc_device_src.inc"   // kPolarDeviceSrc: polar_sc_device.h as a string
#include "polar_sc_interp_src.inc"   // kPolarInterpSrc: polar_sc_interp.h as a string
#include "polar_sc_pair_src.inc"     // kPolarPairSrc: polar_sc_pair.h as a string
}

namespace polar_host {

bool jit_supported(uint32_t N) { return N >= 32 && N <= 1024; }

namespace {

struct Gen {
    const std::vector<polar_sc_op> &ops;   // schedule of the code (or subtree) of 16 * 2^LG LLRs
    std::ostringstream o;
    int LG;
    // per-mask kernels: the channel words are split once (root_presplit) into m<LG> / s<LG>,
    // so the root ops run on split words like every other level
    bool presplit = false;
    // per-mask kernels: the root magnitudes packed two words per register (bytes of word j
    // and j + G/2 in each 16-bit half): half the root registers for 2 VALU more per root
    // F / G word. C2: 158 -> 126 VGPRs, 3 -> 4 waves per SIMD, 76.7 -> 72.7 / 75.5 us on one
    // box
    bool pack = false;
    Gen(const std::vector<polar_sc_op> &ops_, int lg) : ops(ops_), LG(lg) {}

    // Partial sums: u32 bw[max(1, G / 16)], dword j = groups 16 j .. 16 j + 15, low frame in
    // bits 0..15 and high frame in bits 16..31 (the layout every consumer wants, so H ops
    // are one or two instructions and the G ops take their u flags without repacking).
    // 16 partial-sum words starting at q (only the low n bits of each half are used)
    static std::string get16(int q)
    {
        std::ostringstream s;
        if (q % 16 == 0) s << "bw[" << q / 16 << "]";
        else s << "(bw[" << q / 16 << "] >> " << q % 16 << ")";
        return s.str();
    }
    static std::string hexmask(int pos, int n)   // bits [pos % 16, +n) of both halves
    {
        std::ostringstream s;
        const unsigned m = ((1u << n) - 1u) << (pos % 16);
        s << "0x" << std::hex << (m | (m << 16)) << std::dec << "u";
        return s.str();
    }
    // write n <= 16 partial-sum words at pos from acc (low frame bits 0..n-1, high 16..)
    void put(int pos, int n, const std::string &acc)
    {
        if (n >= 16) {
            o << "    bw[" << pos / 16 << "] = " << acc << ";\n";
        } else {
            o << "    bw[" << pos / 16 << "] = bsel(" << hexmask(pos, n) << ", (" << acc << ") << " << pos % 16 << ", bw["
              << pos / 16 << "]);\n";
        }
    }
    // the same from a full mask per half (0xFFFF / 0: every bit of a half equal, as the leaf
    // and REP decisions are): the bits land in place without a shift or an AND
    void put_mask(int pos, int n, const std::string &m)
    {
        if (n >= 16) o << "    bw[" << pos / 16 << "] = " << m << ";\n";
        else o << "    bw[" << pos / 16 << "] = bsel(" << hexmask(pos, n) << ", " << m << ", bw[" << pos / 16 << "]);\n";
    }
    // G-type ops: loop over n words with partial sums from upos (or zero)
    void ucache(int upos, int i)
    {
        if ((i & 15) == 0) {
            if (upos >= 0) o << "    c_ = " << get16(upos + i) << ";\n";
            else o << "    c_ = 0u;\n";
        }
    }
    static std::string uflag(int i)
    {
        std::ostringstream s;
        s << "(c_ << " << (15 - (i & 15)) << ")";   // G_sm / G_root read only bits 15 and 31 of u
        return s.str();
    }

    // Stage words below the root are split (polar_sc_device.h): m<d>[i] magnitudes and
    // s<d>[k] sign planes of words 16k..16k+15. The root reads SM16 channel words CH(i).
    static int planes(int words) { return words >= 16 ? words / 16 : 1; }
    std::string M(int sd, int i) const
    {
        std::ostringstream s;
        if (pack && sd == LG) {
            // packed root: pr[j] holds words j (low bytes) and j + G/2 (high bytes)
            const int h = 1 << (LG - 1);
            // (opaque: the compiler would otherwise rebuild the unpacked words from the
            // presplit and keep all of them live, 180 VGPRs instead of 126)
            if (i < h) s << "rlo(opaque(pr[" << i << "]))";
            else s << "rhi(opaque(pr[" << i - h << "]))";
        } else {
            s << "m" << sd << "[" << i << "]";
        }
        return s.str();
    }
    // sign plane of depth sd shifted so that word i is at bit 0 (bits past the op's words are
    // don't-care: every consumer reads only the bits of its own words)
    std::string P(int sd, int i) const
    {
        std::ostringstream s;
        if (i % 16 == 0) s << "s" << sd << "[" << i / 16 << "]";
        else s << "(s" << sd << "[" << i / 16 << "] >> " << i % 16 << ")";
        return s.str();
    }
    static std::string U(int upos, int k)
    {
        return upos >= 0 ? get16(upos + 16 * k) : std::string("0u");
    }

    // After an F-type op (F, FLEAF, REP) the parent words stay live until the matching G.
    // An empty asm that redefines them in place (no instruction) stops the optimiser from
    // carrying the F op's intermediates over to the G op, which would multiply the
    // registers held across the whole left subtree.
    void clobber_parent(int sd, int n)
    {
        if (sd == LG && !presplit) return;   // root: channel words are re-read from LDS
        if (pack && sd == LG) {
            for (int i = 0; i < n; i++) o << "  asm volatile(\"\" : \"+v\"(pr[" << i << "]));\n";
        } else {
            for (int i = 0; i < 2 * n; i++) o << "  asm volatile(\"\" : \"+v\"(" << M(sd, i) << "));\n";
        }
        for (int k = 0; k < planes(2 * n); k++) o << "  asm volatile(\"\" : \"+v\"(s" << sd << "[" << k << "]));\n";
    }

    // scheduling fence: keeps the straight-line code from hoisting every load of a long
    // op (e.g. the 64 channel words of the root F) and inflating the register footprint
    void fence() { o << "  __builtin_amdgcn_sched_barrier(0);\n"; }
    void chunk_fence(int i, int n)
    {
        if ((i & 7) == 7 && i + 1 < n) fence();
    }
    // X_[k] = sign(a') ^ sign(b) planes of a G-type op on split words
    void xplanes(int sd, int n, int upos)
    {
        const int np = planes(n);
        o << "    u32 X_[" << np << "], LT_[" << np << "] = {};\n";
        for (int k = 0; k < np; k++)
            o << "    X_[" << k << "] = " << P(sd, 16 * k) << " ^ " << P(sd, n + 16 * k) << " ^ " << U(upos, k) << ";\n";
    }

    // A subtree decoder's root children can be REP / R1 / SPC (the root of a whole code's
    // never are): those ops read split words, so the root words are split into m<LG> / s<LG>
    // from CH() first.
    bool root_split_needed() const
    {
        for (const polar_sc_op &op : ops)
            if (op.level == 0 && (op.code == POLAR_OP_REP || op.code == POLAR_OP_R1 || op.code == POLAR_OP_SPC))
                return true;
        return false;
    }
    void root_split(int words)
    {
        for (int k = 0; k < planes(words); k++) o << "    s" << LG << "[" << k << "] = 0u;\n";
        for (int i = 0; i < words; i++) {
            o << "    { const u32 v_ = CH(" << i << "); " << M(LG, i) << " = v_ & MAG; s" << LG << "[" << i / 16
              << "] = plane_put<" << i % 16 << ">(s" << LG << "[" << i / 16 << "], v_); }\n";
            chunk_fence(i, words);
        }
    }

    // Per-mask kernels: wrapper_in + qconv_format (wrapper_in.h:26-44, scalar.h:229-239) once
    // per frame. (Tried in round 4 and reverted: one ds_read_b32 per root register + quad byte
    // transpose + SWAR conversion instead of the 12 byte / table reads: 236 more VALU per wave,
    // 84.0 vs 83.4 us on one box, profiles/r04_ab/c2_presplit_ab.txt -- the presplit is not
    // LDS-bound.) Every channel word becomes a magnitude pair m<LG>[w] and a bit of the sign
    // plane s<LG>[w / 16] (two LDS tables give |LLR| and the sign of a channel byte), so the
    // root F / G are the split-word ops of every other level (F: 1 VALU per word instead of
    // 10, G: 10 instead of 18) for a conversion of about 3 VALU per word.
    void root_presplit(int words)
    {
        for (int k = 0; k < planes(words); k++) o << "  s" << LG << "[" << k << "] = 0u;\n";
        if (pack) {
            // one SM8 lookup per channel byte (sign bit 7, magnitude below): the four bytes of
            // a packed root register (a0 = word i lo, b0 = word j lo, a1 = word i hi, b1 = word
            // j hi) give its magnitudes by one mask and the sign-plane bits of words i and j by
            // one shift + and-or each (bits 7 / 23 and 15 / 31 land on bits i % 16 / 16 + i % 16)
            const int h = words / 2;
            for (int i = 0; i < h; i++) {
                const int j = i + h, si = 7 - i % 16, sj = 15 - j % 16;
                const std::string shi = si >= 0 ? "(r_ >> " + std::to_string(si) + ")" : "(r_ << " + std::to_string(-si) + ")";
                o << "#ifndef POLAR_PRESPLIT_TABS\n"
                  // (byte packing by two v_perm_b32 + OR; -DPOLAR_PRESPLIT_SHIFT: by shifts, the compiler's
                  // shift / OR3 forms)
                  << "#ifndef POLAR_PRESPLIT_SHIFT\n"
                  << "  { const u32 r_ = __builtin_amdgcn_perm((u32)tab8_[chl[" << 16 * j << "]], (u32)tab8_[chl[" << 16 * i
                  << "]], 0x0C0C0400u) | __builtin_amdgcn_perm((u32)tab8_[chh[" << 16 * j << "]], (u32)tab8_[chh[" << 16 * i
                  << "]], 0x04000C0Cu);\n"
                  << "#else\n"
                  << "  { const u32 r_ = (u32)tab8_[chl[" << 16 * i << "]] | ((u32)tab8_[chl[" << 16 * j << "]] << 8) | ((u32)tab8_[chh["
                  << 16 * i << "]] << 16) | ((u32)tab8_[chh[" << 16 * j << "]] << 24);\n"
                  << "#endif\n"
                  << "    pr[" << i << "] = r_ & (QMAG * 0x01010101u);\n"
                  << "    s" << LG << "[" << i / 16 << "] |= " << shi << " & " << (0x00010001u << (i % 16)) << "u;\n"
                  << "    s" << LG << "[" << j / 16 << "] |= (r_ >> " << sj << ") & " << (0x00010001u << (j % 16)) << "u; }\n"
                  // (A/B: -DPOLAR_PRESPLIT_TABS, the separate magnitude and sign tables of round 2)
                  << "#else\n"
                  << "  { const u32 a0_ = chl[" << 16 * i << "], a1_ = chh[" << 16 * i << "], b0_ = chl[" << 16 * j
                  << "], b1_ = chh[" << 16 * j << "];\n"
                  << "    pr[" << i << "] = (u32)tabm_[a0_] | ((u32)tabm_[b0_] << 8) | ((u32)tabm_[a1_] << 16) | ((u32)tabm_[b1_] << 24);\n"
                  << "    s" << LG << "[" << i / 16 << "] |= ((u32)tabs_[a0_] | ((u32)tabs_[a1_] << 16)) << " << i % 16 << ";\n"
                  << "    s" << LG << "[" << j / 16 << "] |= ((u32)tabs_[b0_] | ((u32)tabs_[b1_] << 16)) << " << j % 16
                  << "; }\n#endif\n";
                chunk_fence(i, h);
            }
            return;
        }
        for (int i = 0; i < words; i++) {
            o << "  { const u32 bl_ = chl[" << 16 * i << "], bh_ = chh[" << 16 * i << "];\n"
              << "    " << M(LG, i) << " = (u32)tabm_[bl_] | ((u32)tabm_[bh_] << 16);\n"
              << "    s" << LG << "[" << i / 16 << "] |= ((u32)tabs_[bl_] | ((u32)tabs_[bh_] << 16)) << " << i % 16
              << "; }\n";
            chunk_fence(i, words);
        }
    }

    void op(const polar_sc_op &op)
    {
        const int sd = LG - op.level, cd = sd - 1, n = op.n, np = planes(n);
        const bool root = sd == LG && !presplit;
        fence();
        if (root && (op.code == POLAR_OP_REP || op.code == POLAR_OP_R1 || op.code == POLAR_OP_SPC)) root_split(2 * n);
        switch (op.code) {
        case POLAR_OP_F:
            o << "  { // F level " << op.level << " n " << n << "\n";
            if (root) {
                o << "    u32 P_[" << np << "] = {};\n";
                for (int i = 0; i < n; i++) {
                    o << "    " << M(cd, i) << " = F_root<" << i % 16 << ">(CH(" << i << "), CH(" << n + i << "), P_["
                      << i / 16 << "]);\n";
                    chunk_fence(i, n);
                }
                for (int k = 0; k < np; k++) o << "    s" << cd << "[" << k << "] = P_[" << k << "];\n";
            } else {
                for (int i = 0; i < n; i++) {
                    o << "    " << M(cd, i) << " = pk_min(" << M(sd, i) << ", " << M(sd, n + i) << ");\n";
                    chunk_fence(i, n);
                }
                for (int k = 0; k < np; k++)
                    o << "    s" << cd << "[" << k << "] = " << P(sd, 16 * k) << " ^ " << P(sd, n + 16 * k) << ";\n";
            }
            o << "  }\n";
            clobber_parent(sd, n);
            break;
        case POLAR_OP_G:
            o << "  { // G level " << op.level << " n " << n << " upos " << op.upos << "\n";
            if (root) {
                o << "    u32 c_, P_[" << np << "] = {};\n";
                for (int i = 0; i < n; i++) {
                    ucache(op.upos, i);
                    o << "    " << M(cd, i) << " = G_root<" << i % 16 << ">(CH(" << i << "), CH(" << n + i << "), "
                      << uflag(i) << ", P_[" << i / 16 << "]);\n";
                    chunk_fence(i, n);
                }
                for (int k = 0; k < np; k++) o << "    s" << cd << "[" << k << "] = P_[" << k << "];\n";
            } else {
                xplanes(sd, n, op.upos);
                for (int i = 0; i < n; i++) {
                    o << "    " << M(cd, i) << " = G_split<" << i % 16 << ">(" << M(sd, i) << ", " << M(sd, n + i) << ", X_["
                      << i / 16 << "], LT_[" << i / 16 << "]);\n";
                    chunk_fence(i, n);
                }
                for (int k = 0; k < np; k++)
                    o << "    s" << cd << "[" << k << "] = " << P(sd, n + 16 * k) << " ^ (X_[" << k << "] & ~LT_[" << k
                      << "]);\n";
            }
            o << "  }\n";
            break;
        case POLAR_OP_FLEAF:
        case POLAR_OP_GLEAF: {
            const bool f = op.code == POLAR_OP_FLEAF;
            o << "  { // " << (f ? "F" : "G") << "+leaf pos " << op.pos << " fb 0x" << std::hex << op.fb << std::dec << "\n";
            if (root) {
                if (f) {
                    o << "    const u32 a_ = CH(0), b_ = CH(1);\n"
                      << "    const u32 M_ = pk_min(a_ & MAG, b_ & MAG), S_ = pk_sra(a_ ^ b_, 15);\n";
                } else {
                    o << "    u32 c_; ";
                    ucache(op.upos, 0);
                    o << "    const u32 L_ = G_sm<GSAT>(CH(0), CH(1), " << uflag(0) << ");\n"
                      << "    const u32 M_ = L_ & MAG, S_ = pk_sra(L_, 15);\n";
                }
            } else if (f) {
                o << "    const u32 M_ = pk_min(" << M(sd, 0) << ", " << M(sd, 1) << ");\n"
                  << "    const u32 S_ = plane_mask<0>(" << P(sd, 0) << " ^ " << P(sd, 1) << ");\n";
            } else {
                o << "    const u32 xm_ = opaque(plane_mask<0>(" << P(sd, 0) << " ^ " << P(sd, 1) << " ^ " << U(op.upos, 0)
                  << "));\n"
                  << "    const u32 d_ = pk_sub(" << M(sd, 0) << ", " << M(sd, 1) << ");\n"
                  << "    const u32 M_ = pk_min(bsel(xm_, pk_abs_i16(d_), pk_add(" << M(sd, 0) << ", " << M(sd, 1)
                  << ")), GSAT2);\n"
                  << "    const u32 S_ = plane_mask<0>(" << P(sd, 1) << ") ^ (xm_ & ~pk_sra(d_, 15));\n";
            }
            o << "    const u32 x_ = leaf_gen<0x" << std::hex << (op.fb & 0x7FFFFu) << std::dec << "u>(M_, S_, ln);\n";
            put_mask(op.pos, 1, "x_");
            o << "  }\n";
            if (f) clobber_parent(sd, 1);
            break;
        }
        case POLAR_OP_REP: {
            // value chain in two's complement; the exact SM chain only when a total is 0
            o << "#ifndef REP_FSB\n#ifndef POLAR_REP_FSB\n"
                 "#define REP_FSB(I, a, b, fs) pk_mad_u16(pk_min(a, b), plane_mask<I>(fs) | 0x00010001u, 0x02000200u)\n"
                 "#else\n#define REP_FSB(I, a, b, fs) F_split_biased<I>(a, b, fs)\n#endif\n#endif\n";
            o << "  { // REP n " << n << " pos " << op.pos << "\n    u32 acc_ = 0u, full_, FS_[" << np << "];\n";
            for (int k = 0; k < np; k++)
                o << "    FS_[" << k << "] = " << P(sd, 16 * k) << " ^ " << P(sd, n + 16 * k) << ";\n";
            for (int i = 0; i < n; i++) {
                // the F value + 512 per half as one multiply-add: |F| x (+1 / -1) + 512 (the sign
                // plane's mask OR 1 is -1 / +1 per half; F_split_biased with -DPOLAR_REP_FSB)
                const std::string t = "row_sum_biased(REP_FSB(" + std::to_string(i % 16) + ", " + M(sd, i) + ", " +
                                      M(sd, n + i) + ", FS_[" + std::to_string(i / 16) + "]))";
                if (i + 1 < n) {
                    o << "    acc_ = rep_acc(acc_, " << t << ");\n";
                } else {
                    // the last step without the clamp: a clamp keeps the sign and zero, and the
                    // unclamped sum (|acc| <= 511 plus one word, <= 1007) fits the 16-bit half
                    // (-DPOLAR_REP_CLAMP_LAST: clamped, for A/Bs)
                    o << "#ifndef POLAR_REP_CLAMP_LAST\n    acc_ = pk_sub(pk_add(acc_, " << t << "), 0x20002000u);\n#else\n"
                      << "    acc_ = rep_acc(acc_, " << t << ");\n#endif\n";
                }
                chunk_fence(i, n);
            }
            o << "    if (rep_any_zero(acc_)) {\n      acc_ = 0u;\n";
            for (int i = 0; i < n; i++)
                o << "      acc_ = G_sm<REPSAT>(row_add_tree(F_split_sm<" << i % 16 << ">(" << M(sd, i) << ", " << M(sd, n + i)
                  << ", FS_[" << i / 16 << "]), ln), acc_, 0u);\n";
            // two's complement or SM16: the hard decision is bit 15 / 31 either way
            o << "    }\n    full_ = pk_sra(acc_, 15);\n";
            for (int j = 0; j < n; j += 16) put_mask(op.pos + j, n < 16 ? n : 16, "full_");
            o << "  }\n";
            clobber_parent(sd, n);
            break;
        }
        case POLAR_OP_R1:
        case POLAR_OP_SPC: {
            const bool spc = op.code == POLAR_OP_SPC;
            o << "  { // " << (spc ? "SPC" : "R1") << " n " << n << " pos " << op.pos << " upos " << op.upos << "\n";
            xplanes(sd, n, op.upos);
            // SPC keys (|lambda|, word, bitrev4(position)): for nodes of <= 64 words both frames'
            // keys fit the 16-bit halves of one register (|lambda| <= GSAT <= 63 in 6 bits, the
            // word in 6, the position added after the loop), one packed min per word
            // (-DPOLAR_SPC_KEY32: a 32-bit key per frame, for A/Bs)
            const bool k16 = n <= 64;
            if (spc) o << "    u32 klo_ = 0xFFFFFFFFu, khi_ = 0xFFFFFFFFu, par_ = 0u, kk_ = 0xFFFFFFFFu;\n";
            for (int i = 0; i < n; i++) {
                if (spc) {
                    o << "    { const u32 l_ = G_split<" << i % 16 << ">(" << M(sd, i) << ", " << M(sd, n + i) << ", X_["
                      << i / 16 << "], LT_[" << i / 16 << "]);\n";
                    if (k16)
                        o << "#ifndef POLAR_SPC_KEY32\n      kk_ = pk_min(kk_, pk_shl(l_, 10) | " << ((i << 4) * 0x00010001u)
                          << "u);\n#else\n";
                    o << "      klo_ = __builtin_elementwise_min(klo_, (l_ << 24) | " << (i << 4) << "u);\n"
                      << "      khi_ = __builtin_elementwise_min(khi_, ((l_ >> 16) << 24) | " << (i << 4) << "u);\n"
                      << (k16 ? "#endif\n" : "") << "    }\n";
                } else
                    o << "    LT_[" << i / 16 << "] = plane_put<" << i % 16 << ">(LT_[" << i / 16 << "], pk_sub(" << M(sd, i)
                      << ", " << M(sd, n + i) << "));\n";
                chunk_fence(i, n);
            }
            // hard decisions: sign(b) ^ (X & ~LT), already in partial-sum layout
            for (int k = 0; k < np; k++) {
                o << "    { const u32 h_ = " << P(sd, n + 16 * k) << " ^ (X_[" << k << "] & ~LT_[" << k << "]);\n";
                put(op.pos + 16 * k, n < 16 ? n : 16, "h_");
                if (spc) o << "      par_ ^= h_; }\n";
                else o << "    }\n";
            }
            if (spc) {
                // parity of each frame's hard decisions; flip the partial sum at the least
                // reliable position when it is odd
                if (n < 16) {
                    const unsigned m = (1u << n) - 1u;
                    o << "    par_ &= 0x" << std::hex << (m | (m << 16)) << std::dec << "u;\n";
                }
                if (k16) o << "#ifndef POLAR_SPC_KEY32\n    klo_ = kk_ & 0xFFFFu; khi_ = kk_ >> 16;\n#endif\n";
                o << "    par_ = ((__builtin_popcount(par_ & 0xFFFFu) & 1u) << 15) | ((__builtin_popcount(par_ >> 16) & 1u) << 31);\n"
                     "    par_ = row_xor(par_);\n"
                     "    klo_ = row_min_u32(klo_ | ln.br); khi_ = row_min_u32(khi_ | ln.br);\n";
                // the word index: bits 4.. of the key (16-bit keys: bits 4..9, |lambda| above)
                if (k16) o << "#ifndef POLAR_SPC_KEY32\n    const u32 ilo_ = (klo_ >> 4) & 63u, ihi_ = (khi_ >> 4) & 63u;\n#else\n";
                o << "    const u32 ilo_ = (klo_ >> 4) & 0xFFFFFu, ihi_ = (khi_ >> 4) & 0xFFFFFu;\n";
                if (k16) o << "#endif\n";
                o <<
                     "    const bool flo_ = (par_ & 0x8000u) && (klo_ & 15u) == ln.br;\n"
                     "    const bool fhi_ = (par_ & 0x80000000u) && (khi_ & 15u) == ln.br;\n";
                if (n <= 16) {
                    o << "    bw[" << op.pos / 16 << "] ^= (flo_ ? 1u << (" << op.pos % 16 << " + ilo_) : 0u) | (fhi_ ? 0x10000u << ("
                      << op.pos % 16 << " + ihi_) : 0u);\n";
                } else {
                    for (int k = 0; k < n / 16; k++)
                        o << "    bw[" << op.pos / 16 + k << "] ^= (flo_ && (ilo_ >> 4) == " << k
                          << "u ? 1u << (ilo_ & 15u) : 0u) | (fhi_ && (ihi_ >> 4) == " << k
                          << "u ? 0x10000u << (ihi_ & 15u) : 0u);\n";
                }
            }
            o << "  }\n";
            break;
        }
        case POLAR_OP_H:
        case POLAR_OP_H0: {
            const bool h = op.code == POLAR_OP_H;
            o << "  { // " << (h ? "H" : "H0") << " pos " << op.pos << " n " << n << "\n";
            if (n >= 16) {
                for (int k = 0; k < n / 16; k++)
                    o << "    bw[" << op.pos / 16 + k << "] " << (h ? "^=" : "=") << " bw[" << (op.pos + n) / 16 + k << "];\n";
            } else {
                const int j = op.pos / 16;
                if (h)
                    o << "    bw[" << j << "] ^= (bw[" << j << "] >> " << n << ") & " << hexmask(op.pos, n) << ";\n";
                else
                    o << "    bw[" << j << "] = bsel(" << hexmask(op.pos, n) << ", bw[" << j << "] >> " << n << ", bw[" << j
                      << "]);\n";
            }
            o << "  }\n";
            break;
        }
        default:
            break;
        }
    }

    void stage_arrays(bool with_root)
    {
        for (int d = 1; d < LG; d++)
            o << "  u32 m" << d << "[" << (1 << d) << "], s" << d << "[" << planes(1 << d) << "];\n";
        if (with_root && pack) o << "  u32 pr[" << (1 << (LG - 1)) << "], s" << LG << "[" << planes(1 << LG) << "];\n";
        else if (with_root) o << "  u32 m" << LG << "[" << (1 << LG) << "], s" << LG << "[" << planes(1 << LG) << "];\n";
    }
    void all_ops()
    {
        for (const polar_sc_op &op : ops) {
            if (op.code == POLAR_OP_END) break;
            this->op(op);
        }
    }

    // Subtree decoder `id` of a hybrid plan (polar_sc_interp.h, OP_SUB): the root words come
    // from the interpreter's LDS stage slot (SM16), the partial sums go back to its bit
    // storage at word `pos`.
    void sub_function(int id, bool gmem)
    {
        const int words = 1 << LG;
        const char *ctx = gmem ? "Ctx<true>" : "Ctx<false>";
        o << "__device__ __noinline__ void polar_sub_" << id << "(const " << ctx << " &c, int ldo, int pos)\n{\n"
          << "  extern __shared__ __attribute__((aligned(16))) u32 smem[];\n"
          << (gmem ? "  const lds_slot *cin_ = (const lds_slot *)smem + ldo;\n"
                   : "  const lds_u32 *cin_ = (const lds_u32 *)smem + ldo;\n")
          << "  const Lanes ln = c.ln;\n"
          << "  u32 bw[" << (words >= 16 ? words / 16 : 1) << "] = {};\n";
        stage_arrays(root_split_needed());
        all_ops();
        if (words >= 16) {
            for (int j = 0; j < words / 16; j++) o << "  c.bst((pos >> 4) + " << j << ", bw[" << j << "]);\n";
        } else {
            const unsigned m = (1u << words) - 1u;
            o << "  { const u32 m_ = 0x" << std::hex << (m | (m << 16)) << std::dec << "u << (pos & 15);\n"
              << "    const u32 d_ = c.bld(pos >> 4);\n"
              << "    c.bst(pos >> 4, (d_ & ~m_) | ((bw[0] << (pos & 15)) & m_)); }\n";
        }
        o << "}\n\n";
    }

    std::string run_mask(const polar_sc_plan &p)
    {
        const int N = (int)p.N, G = (int)p.G;
        // Channel staging: each wave copies its 8 frames (8 x N bytes, contiguous rows of the
        // [batch][N] input) HBM -> LDS with global_load_lds_dwordx4, then reads the bytes of
        // its lane (position 16 w + pl of frames row / row + 4) from there once, into the split
        // root words (root_presplit). Frame stride N + 16 bytes keeps the four rows of a read
        // in different banks. One 8-frame batch per wave; the launch is one wave per batch.
        const int FS = N + 16, LPF = N / 16;   // LDS frame stride, 16-byte chunks (lanes) per frame
        const int wpb = MASK_WPB;
        presplit = true;
        pack = G >= 2;
        o << "#define POLAR_LANE_REMAP 1\n#define POLAR_Q " << p.cfg.llr_bits << "\n"
          << (p.cfg.extended ? "" : "#define POLAR_EXT 0\n")   // EXTENDED = 0: saturating leaves
          << "#include \"polar_sc_device.h\"\nusing namespace polar;\n"
          << "typedef const __attribute__((address_space(1))) void *gas_t;\n"
          << "typedef __attribute__((address_space(3))) void *las_t;\n"
          << "extern \"C\" __global__ void __launch_bounds__(" << 64 * wpb << ", " << MASK_MIN_WAVES
          << ") polar_sc_mask_kernel(\n"
          << "    const unsigned char *__restrict__ llr, unsigned short *__restrict__ out, int batch, int out_stride)\n{\n"
          << "  __shared__ uint4 stage_[" << wpb << " * 8 * " << FS / 16 << "];\n"
          // channel byte -> SM8 (qconv_format; bit 7 sign), and -> |LLR|, sign for the unpacked root
          << "  __shared__ unsigned char tab8_[256], tabm_[256], tabs_[256];\n"
          << "  for (u32 t_ = threadIdx.x; t_ < 256u; t_ += " << 64 * wpb << "u) { const u32 v_ = sm8_of_byte(t_);\n"
          << "    tab8_[t_] = (unsigned char)v_; tabm_[t_] = (unsigned char)(v_ & QMAG); tabs_[t_] = (unsigned char)(v_ >> 7); }\n"
          << "  __syncthreads();\n"
          << "  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: SGPR batch indices\n"
          << "  const long nw_ = ((long)batch + 7) / 8;\n"
          << "  long wave = (long)blockIdx.x * " << wpb << " + wib;\n"
          << "  if (wave >= nw_) return;\n"
          << "  unsigned char *st_ = (unsigned char *)stage_ + wib * " << 8 * FS << ";\n"
          << "  const bool al_ = (((unsigned long)llr) & 15u) == 0u;\n"
          << "  const unsigned char *lla_ = (const unsigned char *)((unsigned long)llr & ~15ul);   // 16-byte aligned\n"
          // async HBM -> LDS copy of the 8 frames of batch w, frames past the batch clamped to
          // the last one. Uniform frame base (SGPR) + lane offset: one VGPR for all eight
          // loads, and branch-free -- a branch in the middle of the straight-line decode costs
          // the register allocator ~100 VGPRs. lla_: the input rounded down to 16 bytes (an
          // unaligned input is byte-copied instead and the async rows are overwritten).
          << "  auto fetch_ = [&](long w, int lane) {\n"
          << "    const long f0_ = w * 8;\n";
        for (int f = 0; f < 8; f++)
            for (int c = 0; c < (LPF + 63) / 64; c++) {
                // the LDS row of lane i is base + 16 i whatever its global address, so a frame
                // of fewer than 64 chunks (N < 1024) loads with the other lanes masked off
                // the frame index clamped to the batch is wave-uniform: readfirstlane keeps it
                // (and the frame address) in SGPRs -- computed per lane it cost ~150 VALU and
                // 16 v_cndmask per wave
                const std::string ch = "(" + std::to_string(c * 64) + " + lane)";
                o << "    { const int fr_ = __builtin_amdgcn_readfirstlane((int)(f0_ + " << f << " < batch ? f0_ + " << f
                  << " : (long)batch - 1));\n"
                  << "      if (" << (LPF - c * 64 >= 64 ? std::string("true") : "lane < " + std::to_string(LPF - c * 64))
                  << ") __builtin_amdgcn_global_load_lds((gas_t)(lla_ + (long)fr_ * " << N << " + " << ch
                  << " * 16), (las_t)(st_ + " << f * FS + c * 1024 << "), 16, 0, 0); }\n";
            }
        // Lane-derived values are recomputed after the fetch (the empty asm makes the lane
        // index opaque): kept from the top they would stay live across the whole decode
        // (~30 VGPRs, 4 -> 3 waves per SIMD).
        o << "  };\n"
          << "  {\n"
          << "  int lane = threadIdx.x & 63;\n"
          << "  asm volatile(\"\" : \"+v\"(lane));\n"
          << "  const int row = lane >> 4, pl = lane & 15;\n"
          << "  Lanes ln; ln.init((u32)pl);\n"
          << "  const unsigned char *chl = st_ + row * " << FS << " + ln.pos, *chh = st_ + (row + 4) * " << FS
          << " + ln.pos;\n"
          << "  fetch_(wave, lane);\n"
          << "  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this batch's channel is in LDS\n"
          << "  if (!al_) {   // input not 16-byte aligned: byte copy\n"
          << "    for (int q = lane; q < " << 8 * N << "; q += 64) {\n"
          << "      const int f = q / " << N << ", off = q % " << N << ";\n"
          << "      const long fr = wave * 8 + f < batch ? wave * 8 + f : (long)batch - 1;\n"
          << "      st_[f * " << FS << " + off] = llr[fr * " << N << " + off];\n"
          << "    }\n"
          << "  }\n"
          << "  __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"wavefront\");\n"
          << "  __builtin_amdgcn_wave_barrier();\n"
          << "  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"wavefront\");\n"
          << "  u32 bw[" << (G >= 16 ? G / 16 : 1) << "] = {};\n";
        stage_arrays(true);
        root_presplit(G);
        all_ops();
        // END (my_module.h:1848-1869) + wrapper_out: x^ words in natural order
        o << "  const long f_lo = wave * 8 + (lane >> 4), f_hi = f_lo + 4;\n"
          << "  const bool st_lo = f_lo < batch, st_hi = f_hi < batch;\n"
          << "  unsigned short *o_lo = out + (size_t)f_lo * out_stride, *o_hi = out + (size_t)f_hi * out_stride;\n";
        for (int c = 0; c < (G + 15) / 16; c++) {
            o << "  { const u32 t_ = row_transpose16(to_position_order(" << get16(16 * c) << ", ln), ln); const int w_ = " << 16 * c << " + pl;\n"
              << "    if (w_ < " << G << ") { if (st_lo) o_lo[w_] = (unsigned short)(t_ & 0xFFFFu); "
              << "if (st_hi) o_hi[w_] = (unsigned short)(t_ >> 16); } }\n";
        }
        o << "  for (int w_ = " << G << " + pl; w_ < out_stride; w_ += 16) { if (st_lo) o_lo[w_] = 0; if (st_hi) o_hi[w_] = 0; }\n"
          << "  }\n";
        o << "}\n";
        return o.str();
    }
};

}  // namespace

// Hybrid plan: the schedule interpreter (polar_sc_interp.h, with OP_SUB) plus one generated
// subtree decoder per distinct mixed subtree of p.sub_words words. with_subs = false: the
// plain interpreter alone, specialised on the plan's POLAR_Q (the per-op monitor of per-mask
// plans whose LLR_BITS is not the hipcc-built 6).
std::string hybrid_source(const polar_sc_plan &p, bool with_subs = true, bool chan16 = false)
{
    std::ostringstream o;
    const bool gm = p.gmem != 0;
    const int waves = with_subs ? p.hybrid_waves : HYBRID_MAX_WAVES;
    int lpar = 0;   // log2 PAR
    while ((1 << lpar) < p.cfg.par) lpar++;
    o << "#define POLAR_LANE_REMAP 1\n#define POLAR_SC_SUBS " << (with_subs ? 1 : 0) << "\n#define POLAR_Q "
      << p.cfg.llr_bits << "\n#define POLAR_CA2 " << (p.cfg.sigmag ? 0 : 1) << "\n#define POLAR_EXT "
      << (p.cfg.extended ? 1 : 0) << "\n#define POLAR_LPAR " << lpar << "\n#define POLAR_CHAN16 " << (chan16 ? 1 : 0)
      << "\n#include \"polar_sc_interp.h\"\n";
    if (with_subs) {
        o << "namespace polar {\n#define CH(w) ch_load(cin_[(w) * 64])\n";
        int lg = 0;
        while ((1 << lg) < p.sub_words) lg++;
        for (size_t id = 0; id < p.subs.size(); id++) {
            Gen g(p.subs[id], lg);
            g.sub_function((int)id, gm);
            o << g.o.str();
        }
        const char *ctx = gm ? "Ctx<true>" : "Ctx<false>";
        o << "#undef CH\ntemplate <>\n__device__ void polar_sub_call<" << (gm ? "true" : "false") << ">(const " << ctx
          << " &c, int id, int ldo, int pos)\n{\n  switch (id) {\n";
        for (size_t id = 0; id < p.subs.size(); id++)
            o << "  case " << id << ": polar_sub_" << id << "(c, ldo, pos); return;\n";
        o << "  default: return;\n  }\n}\n}  // namespace polar\n";
    }
    o << "extern \"C\" __global__ void __launch_bounds__(" << waves * 64 << ") polar_sc_hybrid_kernel(\n"
      << "    const polar::chan_t *__restrict__ llr, unsigned short *__restrict__ out, const polar::Op *__restrict__ ops,\n"
      << "    unsigned int *__restrict__ scratch, int N, int batch, int out_stride, int wpg, int gpb, int group_dwords,\n"
      << "    int lds_dwords, int lds0)\n{\n"
      << "  polar::decode_body<" << (gm ? "true" : "false")
      << ">(llr, out, ops, scratch, N, batch, out_stride, wpg, gpb, group_dwords, lds_dwords, lds0);\n}\n"
      // the per-op monitor variant (polar_sc_trace)
      << "extern \"C\" __global__ void __launch_bounds__(" << waves * 64 << ") polar_sc_hybrid_trace_kernel(\n"
      << "    const polar::chan_t *__restrict__ llr, unsigned short *__restrict__ out, const polar::Op *__restrict__ ops,\n"
      << "    unsigned int *__restrict__ scratch, int N, int batch, int out_stride, int wpg, int gpb, int group_dwords,\n"
      << "    int lds_dwords, int lds0, unsigned long long *__restrict__ trace)\n{\n"
      << "  polar::decode_body<" << (gm ? "true" : "false")
      << ", true>(llr, out, ops, scratch, N, batch, out_stride, wpg, gpb, group_dwords, lds_dwords, lds0, trace);\n}\n";
    if (gm && with_subs)   // grid tier: upper-level F / G over all frame groups (polar_sc_interp.h tier_body)
        o << "extern \"C\" __global__ void __launch_bounds__(256) polar_sc_tier_kernel(\n"
          << "    const polar::chan_t *__restrict__ llr, unsigned int *__restrict__ scratch, int N, int batch,\n"
          << "    int group_dwords, int lds0, int code, int k, int n, int upos, unsigned int fb, int cw)\n{\n"
          << "  polar::tier_body(llr, scratch, N, batch, group_dwords, lds0, code, k, n, upos, fb, cw);\n}\n";
    return o.str();
}

std::string jit_source(const polar_sc_plan &p)
{
    if (p.pair) return pair_source(p);
    if (p.hybrid) return hybrid_source(p);
    return Gen(p.ops, p.lg).run_mask(p);
}

namespace {
// Code-object cache: hipRTC output keyed by a hash of the generated source, the embedded
// device headers and the options, kept next to the library (lib/rtc_cache/, or
// $POLAR_SC_RTC_CACHE). The hybrid kernels of the large-N configurations take minutes to
// compile (C5: ~120 subtree decoders); __graft_entry__.build() compiles the benchmark plans
// once on the build host and the cache travels with the in-tree library.
const char *const kRtcOpts[] = {"--gpu-architecture=gfx950", "-O3", "-std=c++17"};

uint64_t fnv1a(uint64_t h, const char *s, size_t n)
{
    for (size_t i = 0; i < n; i++) {
        h ^= (unsigned char)s[i];
        h *= 1099511628211ull;
    }
    return h;
}

std::string cache_dir()
{
    if (const char *e = std::getenv("POLAR_SC_RTC_CACHE")) return e;   // "" disables the cache
    Dl_info info;
    if (!dladdr((const void *)&cache_dir, &info) || !info.dli_fname) return "";
    std::string so = info.dli_fname;
    const size_t slash = so.rfind('/');
    return (slash == std::string::npos ? std::string(".") : so.substr(0, slash)) + "/rtc_cache";
}

// the cache key: the source, the embedded headers it includes, the options, the hipRTC version
// (rtc = false: objects of the offline clang driver, whose identity is part of `src` instead)
uint64_t source_key(const std::string &src, bool rtc = true)
{
    uint64_t h = 1469598103934665603ull;
    h = fnv1a(h, src.data(), src.size());
    // the embedded headers the source includes (interp.h and pair.h include device.h only)
    h = fnv1a(h, kPolarDeviceSrc, sizeof kPolarDeviceSrc);
    if (src.find("\"polar_sc_interp.h\"") != std::string::npos) h = fnv1a(h, kPolarInterpSrc, sizeof kPolarInterpSrc);
    if (src.find("\"polar_sc_pair.h\"") != std::string::npos) h = fnv1a(h, kPolarPairSrc, sizeof kPolarPairSrc);
    for (const char *o : kRtcOpts) h = fnv1a(h, o, std::strlen(o) + 1);
    if (!rtc) return h;
    int ver_major = 0, ver_minor = 0;
    hiprtcVersion(&ver_major, &ver_minor);
    h = fnv1a(h, (const char *)&ver_major, sizeof ver_major);
    h = fnv1a(h, (const char *)&ver_minor, sizeof ver_minor);
    return h;
}

}  // namespace

// Identity of the machine code a plan runs: FNV-1a over the executable sections and .rodata
// (the kernel descriptors) of its compiled code object. Two code objects with equal
// instructions and descriptors get the same key whatever the source text they came from
// (hipRTC names a module-unique symbol after the source, so the whole file differs);
// profiles record it and bench.py reuses their counters only for the same machine code.
uint64_t code_key(const polar_sc_plan &p)
{
    const std::vector<char> &code = p.jit_code;
    if ((!p.jit && !p.hybrid && !p.pair) || code.size() < sizeof(Elf64_Ehdr) ||
        std::memcmp(code.data(), ELFMAG, SELFMAG) != 0)
        return 0;
    Elf64_Ehdr eh;
    std::memcpy(&eh, code.data(), sizeof eh);
    if (eh.e_ident[EI_CLASS] != ELFCLASS64 || eh.e_shentsize != sizeof(Elf64_Shdr) || eh.e_shstrndx >= eh.e_shnum ||
        eh.e_shoff + (uint64_t)eh.e_shnum * sizeof(Elf64_Shdr) > code.size())
        return 0;
    std::vector<Elf64_Shdr> sh(eh.e_shnum);
    std::memcpy(sh.data(), code.data() + eh.e_shoff, sh.size() * sizeof(Elf64_Shdr));
    const Elf64_Shdr &names = sh[eh.e_shstrndx];
    uint64_t h = 1469598103934665603ull;
    for (const Elf64_Shdr &s : sh) {
        if (s.sh_type != SHT_PROGBITS || s.sh_offset + s.sh_size > code.size() || s.sh_name >= names.sh_size ||
            names.sh_offset + names.sh_size > code.size())
            continue;
        const char *nm = code.data() + names.sh_offset + s.sh_name;
        if ((s.sh_flags & SHF_EXECINSTR) || std::strncmp(nm, ".rodata", names.sh_size - s.sh_name) == 0)
            h = fnv1a(h, code.data() + s.sh_offset, s.sh_size);
    }
    return h;
}

namespace {
// cache entries: <key>.cox = "PSCX" + the object's size (u64, little endian) + the object as
// an xz stream (the generated code is 8-bit instruction encodings that LZMA packs ~5x against
// zlib's ~2x: the prewarmed set that travels with the library to every GPU box is ~70 MB
// instead of ~175). liblzma comes from the image (liblzma.so.5, no header there): its two
// stable buffer functions through dlopen. Without it entries are stored as <key>.coz = "PSCZ"
// + size + zlib deflate; both, and a plain <key>.co, still load.
std::string cache_path(const std::string &src, bool rtc = true)
{
    const std::string dir = cache_dir();
    if (dir.empty()) return "";
    char name[40];
    std::snprintf(name, sizeof name, "/%016llx.cox", (unsigned long long)source_key(src, rtc));
    return dir + name;
}

struct Lzma {
    // lzma_easy_buffer_encode / lzma_stream_buffer_decode (lzma/container.h); lzma_ret 0 = LZMA_OK
    typedef int (*enc_t)(uint32_t preset, int check, const void *allocator, const uint8_t *in, size_t in_size,
                         uint8_t *out, size_t *out_pos, size_t out_size);
    typedef int (*dec_t)(uint64_t *memlimit, uint32_t flags, const void *allocator, const uint8_t *in, size_t *in_pos,
                         size_t in_size, uint8_t *out, size_t *out_pos, size_t out_size);
    enc_t enc = nullptr;
    dec_t dec = nullptr;
    Lzma()
    {
        if (void *h = dlopen("liblzma.so.5", RTLD_NOW | RTLD_LOCAL)) {
            enc = (enc_t)dlsym(h, "lzma_easy_buffer_encode");
            dec = (dec_t)dlsym(h, "lzma_stream_buffer_decode");
        }
    }
};
const Lzma &lzma_lib()
{
    static const Lzma l;
    return l;
}

bool read_all(const std::string &path, std::vector<char> &buf)
{
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    buf.assign((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    return true;
}

bool cache_load(const std::string &path, std::vector<char> &code)
{
    if (path.empty()) return false;
    std::vector<char> buf;
    std::string used = path;   // <key>.cox
    bool ok = false;
    if (read_all(path, buf) && buf.size() > 12 && std::memcmp(buf.data(), "PSCX", 4) == 0 && lzma_lib().dec) {
        uint64_t n = 0, memlimit = ~0ull;
        std::memcpy(&n, buf.data() + 4, 8);
        if (n < 4 || n > (1ull << 32)) return false;
        std::vector<char> out(n);
        size_t in_pos = 0, out_pos = 0;
        if (lzma_lib().dec(&memlimit, 0u, nullptr, (const uint8_t *)buf.data() + 12, &in_pos, buf.size() - 12,
                           (uint8_t *)out.data(), &out_pos, (size_t)n) != 0 ||
            out_pos != n)
            return false;
        buf.swap(out);
        ok = true;
    }
    if (!ok) {
        used = path.substr(0, path.size() - 1) + "z";   // <key>.coz
        if (read_all(used, buf) && buf.size() > 12 && std::memcmp(buf.data(), "PSCZ", 4) == 0) {
            uint64_t n = 0;
            std::memcpy(&n, buf.data() + 4, 8);
            if (n < 4 || n > (1ull << 32)) return false;
            std::vector<char> out(n);
            uLongf len = (uLongf)n;
            if (uncompress((Bytef *)out.data(), &len, (const Bytef *)buf.data() + 12, (uLong)(buf.size() - 12)) != Z_OK ||
                len != n)
                return false;
            buf.swap(out);
        } else {
            used = path.substr(0, path.size() - 1);   // <key>.co: an uncompressed entry
            if (!read_all(used, buf)) return false;
        }
    }
    if (buf.size() < 4 || std::memcmp(buf.data(), "\x7f" "ELF", 4) != 0) return false;
    code.swap(buf);
    (void)utime(used.c_str(), nullptr);   // mark as in use (stale entries can be pruned by age)
    return true;
}

void cache_store(const std::string &path, const std::vector<char> &obj)
{
    if (path.empty()) return;
    std::vector<char> code;
    std::string dst = path;
    const uint64_t n = obj.size();
    if (lzma_lib().enc) {
        // xz, preset 6, CRC64 check (LZMA_CHECK_CRC64 = 4)
        code.resize(12 + obj.size() + obj.size() / 2 + 65536);
        size_t pos = 0;
        if (lzma_lib().enc(6u, 4, nullptr, (const uint8_t *)obj.data(), obj.size(), (uint8_t *)code.data() + 12, &pos,
                           code.size() - 12) != 0)
            return;
        code.resize(12 + pos);
        std::memcpy(code.data(), "PSCX", 4);
    } else {
        uLongf clen = compressBound((uLong)obj.size());
        code.resize(12 + clen);
        if (compress2((Bytef *)code.data() + 12, &clen, (const Bytef *)obj.data(), (uLong)obj.size(), 6) != Z_OK) return;
        code.resize(12 + clen);
        std::memcpy(code.data(), "PSCZ", 4);
        dst = path.substr(0, path.size() - 1) + "z";
    }
    std::memcpy(code.data() + 4, &n, 8);
    const size_t slash = dst.rfind('/');
    (void)mkdir(dst.substr(0, slash).c_str(), 0755);
    // unique per process and call: prewarm compiles from several threads, and two of them may
    // store the same key
    static std::atomic<unsigned> seq{0};
    const std::string tmp = dst + ".tmp." + std::to_string((long)getpid()) + "." + std::to_string(seq++);
    {
        std::ofstream f(tmp, std::ios::binary);
        if (!f) return;
        f.write(code.data(), (std::streamsize)code.size());
        if (!f) {
            std::remove(tmp.c_str());
            return;
        }
    }
    if (std::rename(tmp.c_str(), dst.c_str()) != 0) std::remove(tmp.c_str());
}

// ---- generated kernels compiled by the ROCm toolchain's clang driver ----------------------
// hipRTC is resolved by soname, and a process that imported torch first (the Python package
// does, to share torch's HIP runtime) gets torch's bundled hipRTC / comgr, an older LLVM than
// the system ROCm's. Its code is worse for these kernels: the pair kernel's noinline subtree
// decoders and slot loops get a 128-VGPR budget plus AGPR spill slots (86 AGPRs, ~3000
// accvgpr moves at C5; the system ROCm 7.2 compiler: 248 VGPRs, no AGPRs), and the per-mask
// kernel 0.75 % fewer VALU but slower code. Same sources, same box, cache files swapped
// (profiles/r04_ab/compiler_ab.txt): C2 70.75 / 70.76 vs 71.99 / 71.93 us, C3 0.876 / 0.867 vs
// 0.902 / 0.907 ms, the C5 64-frame share 1.326 / 1.328 vs 1.362 / 1.360 ms. So every generated
// kernel is compiled by the clang driver of the toolchain the library was built with (a child
// process, its own cache key), when it exists and this process has no GPU open (a compile after
// the GPU runtime started is left to hipRTC; prewarmed plans never compile at decode time).
bool gpu_open()
{
    DIR *d = opendir("/proc/self/fd");
    if (!d) return true;
    bool open = false;
    char path[64], target[64];
    while (dirent *e = readdir(d)) {
        std::snprintf(path, sizeof path, "/proc/self/fd/%s", e->d_name);
        const ssize_t n = readlink(path, target, sizeof target - 1);
        if (n <= 0) continue;
        target[n] = 0;
        if (std::strcmp(target, "/dev/kfd") == 0) open = true;
    }
    closedir(d);
    return open;
}

// the ROCm clang driver of the toolchain this library was built with (_build.py defines the
// path); "" when it is not installed here
std::string rocm_clang()
{
#ifdef POLAR_ROCM_CLANG
    if (access(POLAR_ROCM_CLANG, X_OK) == 0) return POLAR_ROCM_CLANG;
#endif
    return "";
}

bool write_file(const std::string &path, const char *data, size_t n)
{
    std::ofstream f(path, std::ios::binary);
    f.write(data, (std::streamsize)n);
    return (bool)f;
}

// POLAR_SC_CLANG_FLAGS: extra clang driver arguments (whitespace separated) for compiler A/Bs;
// part of the cache key, and never satisfied by hipRTC
std::vector<std::string> extra_clang_flags()
{
    std::vector<std::string> out;
    const char *e = getenv("POLAR_SC_CLANG_FLAGS");
    std::istringstream in(e ? e : "");
    for (std::string w; in >> w;) out.push_back(w);
    return out;
}

// identity of the clang driver for the cache key of its objects (the hipRTC
// version says nothing about the compiler that built them): the driver's path and version text
// as the library build found them (_build.py). Not the binary's size or mtime: the cache travels
// with the library to GPU boxes of the same image, whose files need not carry the same mtimes
// -- a key that differed there made every decode fall back to hipRTC code (round 5, r05_v1).
std::string clang_identity()
{
#if defined(POLAR_ROCM_CLANG) && defined(POLAR_ROCM_CLANG_VERSION)
    return std::string(POLAR_ROCM_CLANG) + " " + POLAR_ROCM_CLANG_VERSION;
#else
    return "no clang";
#endif
}

// seconds a child compile may take before it is killed and hipRTC builds the kernel instead
// (POLAR_SC_CLANG_TIMEOUT; the inlined C5 subtree variant, the longest, takes ~250 s)
int clang_timeout_s()
{
    const char *e = getenv("POLAR_SC_CLANG_TIMEOUT");
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? v : 900;
}

int offline_compile(const std::string &src, std::vector<char> &code, std::string &log,
                    const std::vector<std::string> &extra)
{
    const std::string clang = rocm_clang();
    if (clang.empty() || gpu_open()) return -ENOENT;
    char tmpl[] = "/tmp/polar_sc_rtc_XXXXXX";
    if (!mkdtemp(tmpl)) return -EIO;
    const std::string dir = tmpl, in = dir + "/k.hip", out = dir + "/k.co", lg = dir + "/log";
    const std::string text = "#include <hip/hip_runtime.h>\n" + src;
    bool ok = write_file(in, text.data(), text.size()) &&
              write_file(dir + "/polar_sc_device.h", kPolarDeviceSrc, sizeof kPolarDeviceSrc - 1) &&
              write_file(dir + "/polar_sc_pair.h", kPolarPairSrc, sizeof kPolarPairSrc - 1) &&
              write_file(dir + "/polar_sc_interp.h", kPolarInterpSrc, sizeof kPolarInterpSrc - 1);
    int rc = -EIO;
    if (ok) {
        const std::string inc = "-I" + dir;
        std::vector<const char *> argv = {clang.c_str(), "-x", "hip", "--offload-arch=gfx950", "--cuda-device-only",
                                          "--no-gpu-bundle-output", "-O3", "-std=c++17", "-w", inc.c_str()};
        for (const std::string &w : extra) argv.push_back(w.c_str());
        for (const char *w : {"-c", "-o", out.c_str(), in.c_str()}) argv.push_back(w);
        argv.push_back(nullptr);
        posix_spawn_file_actions_t fa;
        posix_spawn_file_actions_init(&fa);
        posix_spawn_file_actions_addopen(&fa, 1, lg.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
        posix_spawn_file_actions_adddup2(&fa, 1, 2);
        // the driver in a process group of its own, so that a timeout kills the tools it spawned
        // (lld, the offload bundler, a non-integrated cc1) with it
        posix_spawnattr_t sa;
        posix_spawnattr_init(&sa);
        posix_spawnattr_setflags(&sa, POSIX_SPAWN_SETPGROUP);
        posix_spawnattr_setpgroup(&sa, 0);
        // the driver's own temporaries (offload objects, bundles) go to the scratch directory too,
        // so that a killed compile leaves nothing behind
        const std::string tmpenv = "TMPDIR=" + dir;
        std::vector<const char *> envp;
        for (char **e = environ; *e; ++e)
            if (std::strncmp(*e, "TMPDIR=", 7) != 0) envp.push_back(*e);
        envp.push_back(tmpenv.c_str());
        envp.push_back(nullptr);
        pid_t pid;
        if (posix_spawn(&pid, clang.c_str(), &fa, &sa, (char *const *)argv.data(), (char *const *)envp.data()) == 0) {
            int status = 0;
            pid_t w = 0;
            // bounded wait: a hung compiler must not hang the decode (it is killed, and the
            // caller falls back to hipRTC)
            for (long waited_ms = 0; (w = waitpid(pid, &status, WNOHANG)) == 0; waited_ms += 20) {
                if (waited_ms >= 1000l * clang_timeout_s()) {
                    kill(-pid, SIGKILL);   // the whole group (pgid == the driver's pid)
                    w = waitpid(pid, &status, 0);
                    log += "clang driver killed after " + std::to_string(clang_timeout_s()) + " s\n";
                    status = -1;
                    break;
                }
                usleep(20000);
            }
            if (w == pid && status != -1 && WIFEXITED(status) && WEXITSTATUS(status) == 0) {
                std::ifstream f(out, std::ios::binary);
                std::vector<char> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
                if (buf.size() >= 4 && std::memcmp(buf.data(), "\x7f" "ELF", 4) == 0) {
                    code.swap(buf);
                    rc = 0;
                }
            }
        }
        posix_spawn_file_actions_destroy(&fa);
        posix_spawnattr_destroy(&sa);
        std::ifstream lf(lg);
        log.assign((std::istreambuf_iterator<char>(lf)), std::istreambuf_iterator<char>());
    }
    if (DIR *d = opendir(dir.c_str())) {   // every file the compile left (a flat directory)
        while (dirent *e = readdir(d))
            if (std::strcmp(e->d_name, ".") != 0 && std::strcmp(e->d_name, "..") != 0)
                std::remove((dir + "/" + e->d_name).c_str());
        closedir(d);
    }
    rmdir(dir.c_str());
    return rc;
}

// whole: a generated kernel source (compiled by the clang driver when available, under its own
// cache key); otherwise, and for the interpreter sources, hipRTC
// *compiler (optional): which compiler built the returned object, POLAR_SC_COMPILER_*
int rtc_compile(const std::string &src, std::vector<char> &code, std::string &log, bool whole = false,
                uint32_t *compiler = nullptr)
{
    if (compiler) *compiler = POLAR_SC_COMPILER_HIPRTC;
    if (whole) {
        const std::vector<std::string> extra = extra_clang_flags();
        std::string key = src + "\n// offline clang driver: " + clang_identity() + "\n";
        for (const std::string &w : extra) key += "// " + w + "\n";
        const std::string opath = cache_path(key, false);
        if (cache_load(opath, code)) {
            if (compiler) *compiler = POLAR_SC_COMPILER_CLANG;
            return 0;
        }
        if (offline_compile(src, code, log, extra) == 0) {   // (a hit is not stored again: ADVICE r05)
            if (compiler) *compiler = POLAR_SC_COMPILER_CLANG;
            cache_store(opath, code);
            return 0;
        }
        if (!extra.empty()) {
            log += "POLAR_SC_CLANG_FLAGS set: no cached object and no clang driver to build one\n";
            return -EIO;
        }
    }
    const std::string cpath = cache_path(src);
    if (cache_load(cpath, code)) return 0;
    hiprtcProgram prog;
    const char *hdrs[] = {kPolarDeviceSrc, kPolarInterpSrc, kPolarPairSrc};
    const char *names[] = {"polar_sc_device.h", "polar_sc_interp.h", "polar_sc_pair.h"};
    if (hiprtcCreateProgram(&prog, src.c_str(), "polar_sc_mask.hip", 3, hdrs, names) != HIPRTC_SUCCESS) return -EIO;
    hiprtcResult rc = hiprtcCompileProgram(prog, (int)(sizeof kRtcOpts / sizeof kRtcOpts[0]), (const char **)kRtcOpts);
    size_t log_size = 0;
    hiprtcGetProgramLogSize(prog, &log_size);
    if (log_size > 1) {
        log.resize(log_size);
        hiprtcGetProgramLog(prog, &log[0]);
    }
    if (rc != HIPRTC_SUCCESS) {
        hiprtcDestroyProgram(&prog);
        return -EIO;
    }
    size_t code_size = 0;
    hiprtcGetCodeSize(prog, &code_size);
    code.resize(code_size);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    cache_store(cpath, code);
    return 0;
}
}  // namespace

// int16 channel (polar_sc_decode_i16): the interpreter of the plan's format on int16 LLRs
int jit_load16(const polar_sc_plan &p, DevState &st)
{
    if (st.fn16) return 0;
    if (p.code16.empty()) {
        int rc = rtc_compile(hybrid_source(p, false, true), p.code16, p.jit_log);
        if (rc) return rc;
    }
    if (hipModuleLoadData(&st.module16, p.code16.data()) != hipSuccess) return -EIO;
    if (hipModuleGetFunction(&st.fn16, st.module16, "polar_sc_hybrid_kernel") != hipSuccess) return -EIO;
    return 0;
}

int jit_compile(const polar_sc_plan &p)
{
    if (!p.jit_code.empty()) return 0;
    std::string src;
    try {   // (the generators throw on a schedule they do not support: an error, not an abort)
        src = jit_source(p);
    } catch (const std::exception &e) {
        p.jit_log = e.what();
        return -ENOTSUP;
    }
    return rtc_compile(src, p.jit_code, p.jit_log, true, &p.jit_compiler);
}

// Per-mask plans whose LLR_BITS is not the hipcc-built 6: the per-op monitor runs the schedule
// interpreter compiled by hipRTC with the plan's POLAR_Q (DevState::ifn_trace).
int jit_load_interp(const polar_sc_plan &p, DevState &st)
{
    if (st.ifn_trace) return 0;
    if (p.interp_code.empty()) {
        int rc = rtc_compile(hybrid_source(p, false), p.interp_code, p.jit_log);
        if (rc) return rc;
    }
    if (hipModuleLoadData(&st.imodule, p.interp_code.data()) != hipSuccess) return -EIO;
    if (hipModuleGetFunction(&st.ifn_trace, st.imodule, "polar_sc_hybrid_trace_kernel") != hipSuccess) return -EIO;
    return 0;
}

// Registers per lane of kernel `name` in a gfx950 code object, from its kernel descriptor
// (symbol "<name>.kd", AMDHSA code object v5): compute_pgm_rsrc1 bits 0..5 hold
// GRANULATED_WORKITEM_VGPR_COUNT, which on gfx90a and later counts the unified VGPR + AGPR
// allocation in granules of 8. hipRTC can add AGPRs to a 256-VGPR call graph; the hardware
// then rejects a dispatch whose waves do not fit (HSA_STATUS_ERROR_INVALID_ISA), so the launch
// shape is checked against this before every launch. -1: no such kernel.
int kernel_regs(const std::vector<char> &code, const char *name)
{
    if (code.size() < sizeof(Elf64_Ehdr) || std::memcmp(code.data(), ELFMAG, SELFMAG) != 0) return -1;
    Elf64_Ehdr eh;
    std::memcpy(&eh, code.data(), sizeof eh);
    if (eh.e_ident[EI_CLASS] != ELFCLASS64 || eh.e_shentsize != sizeof(Elf64_Shdr) ||
        eh.e_shoff + (uint64_t)eh.e_shnum * sizeof(Elf64_Shdr) > code.size())
        return -1;
    std::vector<Elf64_Shdr> sh(eh.e_shnum);
    std::memcpy(sh.data(), code.data() + eh.e_shoff, sh.size() * sizeof(Elf64_Shdr));
    const std::string want = std::string(name) + ".kd";
    for (const Elf64_Shdr &s : sh) {
        if (s.sh_type != SHT_SYMTAB || s.sh_link >= sh.size() || s.sh_entsize != sizeof(Elf64_Sym)) continue;
        const Elf64_Shdr &strs = sh[s.sh_link];
        if (s.sh_offset + s.sh_size > code.size() || strs.sh_offset + strs.sh_size > code.size()) continue;
        for (uint64_t o = 0; o + sizeof(Elf64_Sym) <= s.sh_size; o += sizeof(Elf64_Sym)) {
            Elf64_Sym sym;
            std::memcpy(&sym, code.data() + s.sh_offset + o, sizeof sym);
            if (sym.st_name >= strs.sh_size) continue;
            const char *nm = code.data() + strs.sh_offset + sym.st_name;
            if (std::strncmp(nm, want.c_str(), strs.sh_size - sym.st_name) != 0) continue;
            if (sym.st_shndx >= sh.size()) return -1;
            const Elf64_Shdr &sec = sh[sym.st_shndx];   // the descriptor's section (.rodata)
            const uint64_t off = sec.sh_offset + (sym.st_value - sec.sh_addr);
            if (sym.st_value < sec.sh_addr || off + 64 > code.size()) return -1;
            uint32_t rsrc1;
            std::memcpy(&rsrc1, code.data() + off + 48, 4);   // compute_pgm_rsrc1
            return (int)((rsrc1 & 63u) + 1u) * 8;
        }
    }
    return -1;
}

// registers of the plan's decode kernel and (pair plans with a grid tier) its segment kernel,
// from the compiled code object (jit_compile first)
void code_regs(const polar_sc_plan &p, int &regs, int &regs_seg)
{
    const char *main = p.pair ? "polar_sc_pair_kernel" : (p.hybrid ? "polar_sc_hybrid_kernel" : "polar_sc_mask_kernel");
    regs = kernel_regs(p.jit_code, main);
    // hybrid plans launch their traced variant with the same shape
    if (p.hybrid && regs > 0) regs = std::max(regs, kernel_regs(p.jit_code, "polar_sc_hybrid_trace_kernel"));
    regs_seg = p.pair && !p.pair_tier.steps.empty() ? kernel_regs(p.jit_code, "polar_sc_pair_seg_kernel") : 0;
}

// the largest waves-per-block count <= W (halving) whose waves fit the 512 registers per lane
// of a SIMD (a block's waves are spread over the CU's 4 SIMDs); 0 when not even one wave fits
int fit_waves(int regs, int W)
{
    if (regs <= 0) return W;   // (the hipcc-built interpreter: fixed launch bounds)
    if (regs > SIMD_REGS) return 0;
    while (W > 1 && ((W + 3) / 4) * regs > SIMD_REGS) W /= 2;
    return W;
}

int jit_load(const polar_sc_plan &p, DevState &st)
{
    if (st.fn) return 0;
    int rc = jit_compile(p);
    if (rc) {
        std::fprintf(stderr, "polar_sc: hipRTC build failed (%d)%s%s\n", rc, p.jit_log.empty() ? "" : ":\n",
                     p.jit_log.c_str());
        return rc;
    }
    // register budget of the decode kernels (before anything is loaded on the device)
    {
        code_regs(p, st.regs, st.regs_seg);
        if (st.regs > SIMD_REGS || st.regs_seg > SIMD_REGS) {
            std::fprintf(stderr, "polar_sc: generated kernel needs %d registers per lane (> %d): not launchable\n",
                         std::max(st.regs, st.regs_seg), SIMD_REGS);
            return -ENOTSUP;
        }
    }
    if (hipError_t e = hipModuleLoadData(&st.module, p.jit_code.data()); e != hipSuccess) {
        std::fprintf(stderr, "polar_sc: hipModuleLoadData: %s\n", hipGetErrorString(e));
        return -EIO;
    }
    if (p.pair) {
        if (hipModuleGetFunction(&st.fn, st.module, "polar_sc_pair_kernel") != hipSuccess ||
            hipModuleGetFunction(&st.fn_subtest, st.module, "polar_sc_pair_subtest_kernel") != hipSuccess) {
            std::fprintf(stderr, "polar_sc: pair kernels missing from the code object\n");
            return -EIO;
        }
        if (!p.pair_tier.steps.empty() &&
            (hipModuleGetFunction(&st.fn_seg, st.module, "polar_sc_pair_seg_kernel") != hipSuccess ||
             hipModuleGetFunction(&st.fn_tier, st.module, "polar_sc_pair_tier_kernel") != hipSuccess))
            return -EIO;
        return 0;
    }
    if (hipModuleGetFunction(&st.fn, st.module, p.hybrid ? "polar_sc_hybrid_kernel" : "polar_sc_mask_kernel") !=
        hipSuccess)
        return -EIO;
    if (p.hybrid && hipModuleGetFunction(&st.fn_trace, st.module, "polar_sc_hybrid_trace_kernel") != hipSuccess)
        return -EIO;
    if (!p.tiers.empty() && hipModuleGetFunction(&st.fn_tier, st.module, "polar_sc_tier_kernel") != hipSuccess)
        return -EIO;
    return 0;
}

int jit_launch(const polar_sc_plan &p, const DevState &st, const int8_t *llr, uint16_t *out, long batch,
               int out_stride, void *stream)
{
    (void)p;
    if (fit_waves(st.regs, MASK_WPB) != MASK_WPB) return -ENOTSUP;   // (123 registers at C2)
    const long waves = (batch + 7) / 8;   // one 8-frame batch per wave (run_mask)
    const unsigned blocks = (unsigned)((waves + MASK_WPB - 1) / MASK_WPB);
    int b = (int)batch;
    void *args[] = {(void *)&llr, (void *)&out, (void *)&b, (void *)&out_stride};
    hipError_t e = hipModuleLaunchKernel(st.fn, blocks, 1, 1, 64 * MASK_WPB, 1, 1, 0, (hipStream_t)stream, args,
                                         nullptr);
    return e == hipSuccess ? 0 : -EIO;
}

// hybrid kernel: the interpreter's launch shape (polar_sc_kernels.hip, polar_sc_launch_decode)
int launch_interp_fn(hipFunction_t fn, const polar_sc_plan &p, const DevState &st, const int8_t *llr, uint16_t *out,
                     long batch, int out_stride, int wpg, void *stream, unsigned long long *trace, const void *ops)
{
    const long groups = (batch + 7) / 8;
    const unsigned lds = (unsigned)p.lds_group_dwords * 4u;
    if (!ops) ops = st.ops;
    void *scratch = st.scratch;
    int N = (int)p.N, b = (int)batch, gpb = 1, gd = p.hbm_group_dwords, ld = p.lds_group_dwords, l0 = p.lds0;
    void *args[] = {(void *)&llr, (void *)&out, (void *)&ops, (void *)&scratch, (void *)&N, (void *)&b,
                    (void *)&out_stride, (void *)&wpg, (void *)&gpb, (void *)&gd, (void *)&ld, (void *)&l0,
                    (void *)&trace};
    hipError_t e = hipModuleLaunchKernel(fn, (unsigned)groups, 1, 1, (unsigned)(64 * wpg), 1, 1, lds,
                                         (hipStream_t)stream, args, nullptr);
    return e == hipSuccess ? 0 : -EIO;
}

// Grid-tier plans: one launch per tier step, in schedule order on the caller's stream. Grid
// steps run the F / G record over all frame groups, TIER_CW words per wave (256-thread
// blocks); segment steps run the hybrid kernel on the segment's records.
constexpr int TIER_CW = 64;

int launch_tier(const polar_sc_plan &p, const DevState &st, const int8_t *llr, uint16_t *out, long batch,
                int out_stride, int wpg, void *stream)
{
    const long groups = (batch + 7) / 8;
    const unsigned lds = (unsigned)p.lds_group_dwords * 4u;
    void *scratch = st.scratch;
    int N = (int)p.N, b = (int)batch, gpb = 1, gd = p.hbm_group_dwords, ld = p.lds_group_dwords, l0 = p.lds0;
    int cw = TIER_CW;
    unsigned long long *no_trace = nullptr;
    // batches with at least one frame group per CU keep every CU busy inside the hybrid
    // kernel: they take the root-only cut (tiers[1]) when the plan has one
    const long cus = st.simds > 0 ? st.simds / 4 : 256;
    const size_t ti = (p.tiers.size() > 1 && groups >= cus) ? 1 : 0;
    const TierPlan &tp = p.tiers[ti];
    for (const TierStep &t : tp.steps) {
        hipError_t e;
        if (t.grid) {
            int code = t.op.code, k = t.op.level, n = t.op.n, upos = t.op.upos;
            unsigned fb = t.op.fb;
            const long waves = groups * (long)((n + cw - 1) / cw);
            void *args[] = {(void *)&llr, (void *)&scratch, (void *)&N, (void *)&b, (void *)&gd, (void *)&l0,
                            (void *)&code, (void *)&k, (void *)&n, (void *)&upos, (void *)&fb, (void *)&cw};
            e = hipModuleLaunchKernel(st.fn_tier, (unsigned)((waves + 3) / 4), 1, 1, 256, 1, 1, 0,
                                      (hipStream_t)stream, args, nullptr);
        } else {
            const void *ops = (const polar_sc_op *)st.seg_ops[ti] + t.off;
            void *args[] = {(void *)&llr, (void *)&out, (void *)&ops, (void *)&scratch, (void *)&N, (void *)&b,
                            (void *)&out_stride, (void *)&wpg, (void *)&gpb, (void *)&gd, (void *)&ld, (void *)&l0,
                            (void *)&no_trace};
            e = hipModuleLaunchKernel(st.fn, (unsigned)groups, 1, 1, (unsigned)(64 * wpg), 1, 1, lds,
                                      (hipStream_t)stream, args, nullptr);
        }
        if (e != hipSuccess) return -EIO;
    }
    return 0;
}

// Pair plans (polar_sc_pair.h): one block of W waves per frame pair. W grows while the pairs
// cannot give every SIMD two waves (C3's 2048 pairs: 1; C5's 256 or 32: 8), then is capped so
// that the block's waves fit the register file (kernel_regs). The stage slots of the smallest
// levels go to LDS while they fit the share of a CU's 160 KB that one resident pair gets
// (all-HBM otherwise); with a grid tier they stay below the tier's cut.
PairShape pair_shape(const polar_sc_plan &p, long batch, int simds, int regs, int regs_seg)
{
    PairShape sh;
    sh.pairs = p.solo ? batch : (batch + 1) / 2;   // blocks: frame pairs, or frames (solo)
    const long cus = simds > 0 ? simds / 4 : 256;
    int W = p.tune.waves_per_group;
    if (W == 0) {
        // more waves per pair while the batch leaves SIMDs without 2 waves, but never past one
        // dispatch round: the blocks must all be resident at once (512 / regs waves per SIMD).
        // Same box (profiles/r06_v3 layout_ab): 1536 pairs at W = 2 (3072 waves of 248 registers,
        // two rounds) 1.27 ms, where 2048 pairs at W = 1 take 0.83 ms
        const long sm = simds > 0 ? simds : 1024;
        const long wps = regs > 0 ? std::max(1, 512 / regs) : 2;
        W = 1;
        while (W < PAIR_WAVES_MAX && sh.pairs * W < 2 * sm && sh.pairs * 2 * W <= sm * wps) W *= 2;
    }
    if (W > PAIR_WAVES_MAX) W = PAIR_WAVES_MAX;
    const bool tier = !p.pair_tier.steps.empty();
    W = fit_waves(regs, W);
    if (tier) W = std::min(W, fit_waves(regs_seg, W));
    sh.W = W;
    if (W == 0) return sh;
    const long per_cu = (sh.pairs + cus - 1) / cus;
    // LDS: levels of nodes S .. L words ((2 L - S) / wpr slot rows of 128 B) + the SPC exchange
    // (3 W rows of 256 B)
    const long budget = CU_LDS_BYTES / (per_cu > 0 ? per_cu : 1) - 3l * W * 256l;
    // (S: the smallest slot level -- the subtree roots, or their parents when the roots are
    // read as F / G of them, pair_fused)
    const int S = p.pair_fused ? 2 * p.sub_words : p.sub_words, G = (int)p.G, wpr = p.wpr();
    const long bpw = p.slot_row_bytes() / wpr;   // slot bytes per word
    int L = 0;
    for (int w = S; w <= G / 2; w *= 2) {
        if (tier && w >= p.pair_tier.tw) break;
        if (bpw * (2l * w - S) <= budget) L = w;
    }
    // polar_sc_tuning.lds_slots: the levels of nodes up to this many words in LDS whatever
    // the batch (fewer pairs then fit a CU: the A/B of keeping more levels on chip)
    if (const int want = p.tune.lds_slots) {
        L = 0;
        for (int w = S; w <= G / 2 && w <= want; w *= 2)
            if (!(tier && w >= p.pair_tier.tw) && bpw * (2l * w - S) + 3l * W * 256l <= CU_LDS_BYTES) L = w;
    }
    const int lds_rows = L ? (2 * L - S) / wpr : 0;
    sh.lds_row0 = p.pair_slot_rows - lds_rows;
    sh.lds = (unsigned)(lds_rows * p.slot_row_bytes() + 3 * W * 256);
    return sh;
}

int jit_launch_pair(const polar_sc_plan &p, const DevState &st, const int8_t *llr, uint16_t *out, long batch,
                    int out_stride, void *stream)
{
    const PairShape sh = pair_shape(p, batch, st.simds, st.regs, st.regs_seg);
    if (sh.W == 0) return -ENOTSUP;
    const bool tier = !p.pair_tier.steps.empty();
    int N = (int)p.N, b = (int)batch, pd = p.pair_dwords, sr = p.pair_slot_rows, lds_row0 = sh.lds_row0;
    const long pairs = sh.pairs;
    void *scratch = st.scratch;
    auto segment = [&](hipFunction_t fn, int seg) {
        void *args[] = {(void *)&llr, (void *)&out, (void *)&scratch, (void *)&N, (void *)&b, (void *)&out_stride,
                        (void *)&pd, (void *)&sr, (void *)&lds_row0, (void *)&seg};
        return hipModuleLaunchKernel(fn, (unsigned)pairs, 1, 1, (unsigned)(64 * sh.W), 1, 1, sh.lds,
                                     (hipStream_t)stream, args, nullptr);
    };
    if (!tier) return segment(st.fn, 0) == hipSuccess ? 0 : -EIO;
    int cw = TIER_CW;
    for (const TierStep &t : p.pair_tier.steps) {
        hipError_t e;
        if (t.grid) {
            int g = t.op.code == POLAR_OP_G ? 1 : 0, k = t.op.level, n4 = t.op.n / p.wpr();
            int ub = t.op.upos >= 0 ? t.op.upos / p.wpr() : -1;
            const long waves = pairs * (long)((n4 + cw - 1) / cw);
            void *args[] = {(void *)&llr, (void *)&scratch, (void *)&N, (void *)&b, (void *)&pd, (void *)&sr,
                            (void *)&g, (void *)&k, (void *)&n4, (void *)&ub, (void *)&cw};
            e = hipModuleLaunchKernel(st.fn_tier, (unsigned)((waves + 3) / 4), 1, 1, 256, 1, 1, 0, (hipStream_t)stream,
                                      args, nullptr);
        } else {
            e = segment(st.fn_seg, t.off);
        }
        if (e != hipSuccess) return -EIO;
    }
    return 0;
}

int jit_launch_hybrid(const polar_sc_plan &p, const DevState &st, const int8_t *llr, uint16_t *out, long batch,
                      int out_stride, int wpg, void *stream, unsigned long long *trace)
{
    wpg = fit_waves(st.regs, wpg);   // the block's waves must fit the register file
    if (wpg == 0) return -ENOTSUP;
    if (!trace && !p.tiers.empty()) return launch_tier(p, st, llr, out, batch, out_stride, wpg, stream);
    return launch_interp_fn(trace ? st.fn_trace : st.fn, p, st, llr, out, batch, out_stride, wpg, stream, trace);
}

}  // namespace polar_host
