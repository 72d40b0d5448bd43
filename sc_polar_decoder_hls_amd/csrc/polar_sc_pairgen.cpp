// polar_sc_pairgen.cpp -- generated decode kernels of pair plans (N >= 2048 in the shipped
// datapath): the frame-pair layout of polar_sc_pair.h.
//
// A pair plan's device schedule (polar_sc_host.cpp compile_node with subtrees of S words) has
// two parts:
//   * the upper levels (nodes wider than S words): F / G / REP / R1 / SPC / H records over
//     slot rows, emitted here as calls of the loop functions of polar_sc_pair.h, split over
//     the W waves of the pair where that is legal;
//   * every mixed node of S words: one OP_SUB record, whose own schedule becomes straight-line
//     register code (PairGen::sub_function) -- the per-mask kernel's split-word code
//     (polar_sc_jit.cpp Gen) rewritten for four words per register and the cross-row steps of
//     the nodes of 2 and 4 words.
// The reference is specialised per code the same way (Frozen_Bit_Generator writes the mask into
// polar_parameters.h and the HLS design is re-synthesised for it, Writer.h:110-162).
#include "polar_sc_plan.hpp"

#include <map>
#include <set>
#include <stdexcept>
#include <sstream>
#include <string>
#include <tuple>
#include <vector>

namespace polar_host {

namespace {

struct PairGen {
    const std::vector<polar_sc_op> &ops;   // subtree schedule, levels / positions relative to its root
    std::ostringstream o;
    int LG;                                // the subtree root has 2^LG words
    // solo layout (polar_sc_pair.h POLAR_SOLO): one frame per wave, a register of a node of
    // >= 8 words holds words 8 j + 4 h + r (half h, row r); nodes of 4 words and below are
    // replicated in both halves, so their ops are the pair code's
    bool solo;
    int wpr;                               // words per register of the lane-private nodes: 4 / 8
    std::map<int, std::string> small1;     // result masks of 1-word nodes, by word position
    std::map<int, std::string> small2;     // result masks of 2-word nodes (row r: word r & 1)
    int nvar = 0;
    // CA2 plans (POLAR_CA2; polar_sc_device.h): hard decisions mask zeros, REP has no exact-SM
    // fallback, and in the decoder of the leftmost subtree (`left`, the _L variant) the F-type
    // ops that can meet MIN take the key min: those of the first PAR word (pos < p16 words),
    // which include the leftmost path
    bool ca2 = false, left = false;
    int q = 6, p16 = 1;
    // PAR 4 / 8 (pw): the PAR words are lane groups of a device word; one-word leaf records
    // decode the whole word tree (leaf_word_gen: frozen bits + group classes from reserved[1]),
    // REP runs the exact group chains (polar_sc_pair.h rep_groups_*), SPC keys take the group
    bool pw = false;

    PairGen(const std::vector<polar_sc_op> &ops_, int lg, bool solo_ = false)
        : ops(ops_), LG(lg), solo(solo_), wpr(solo_ ? 8 : 4) {}

    // MIN width of an F-type op's operands (0: they cannot hold MIN); fb bits 20..23 = operand
    // width above LLR_BITS (PAR > 16 leaf expansion), GLEAF: + 1 behind an exact G
    int min_width(const polar_sc_op &op, bool gleaf = false) const
    {
        if (!ca2 || !left || op.pos >= p16) return 0;
        return q + (int)((op.fb >> 20) & 15u) + (gleaf && (op.fb & FB_EXACT) ? 1 : 0);
    }
    // hard decision masks of a G result (sign plane / masks h, magnitude l) in CA2: zeros decide 0
    std::string hard_plane(const std::string &h, const std::string &nzp) const { return ca2 ? "(" + h + ") & " + nzp : h; }

    // registers of a node of 2^sd words
    int regs(int sd) const { return solo ? (sd >= 3 ? 1 << (sd - 3) : 1) : (sd >= 2 ? 1 << (sd - 2) : 1); }
    static int planes(int r) { return r >= 16 ? r / 16 : 1; }
    static std::string M(int sd, int i) { return "m" + std::to_string(sd) + "[" + std::to_string(i) + "]"; }
    // sign plane of register i of a node of 2^sd words, shifted so that register i is at bit 0
    static std::string P(int sd, int i)
    {
        std::ostringstream s;
        if (i % 16 == 0) s << "s" << sd << "[" << i / 16 << "]";
        else s << "(s" << sd << "[" << i / 16 << "] >> " << i % 16 << ")";
        return s.str();
    }
    // partial sums of local words l .. l + 15 (local word l at bit 0)
    static std::string get16(int l)
    {
        std::ostringstream s;
        if (l % 16 == 0) s << "bw[" << l / 16 << "]";
        else s << "(bw[" << l / 16 << "] >> " << l % 16 << ")";
        return s.str();
    }
    static std::string U(int ub, int k) { return ub >= 0 ? get16(ub + 16 * k) : std::string("0u"); }
    static std::string hexmask(int l, int cnt)
    {
        std::ostringstream s;
        const unsigned m = ((1u << cnt) - 1u) << (l % 16);
        s << "0x" << std::hex << (m | (m << 16)) << std::dec << "u";
        return s.str();
    }
    // local words [l, l + cnt) (cnt <= 16, one dword) := acc (bit j = local word l + j)
    void put(int l, int cnt, const std::string &acc)
    {
        if (cnt >= 16) o << "    bw[" << l / 16 << "] = " << acc << ";\n";
        else
            o << "    bw[" << l / 16 << "] = bsel(" << hexmask(l, cnt) << ", (" << acc << ") << " << l % 16 << ", bw["
              << l / 16 << "]);\n";
    }
    // the same from a full mask per half (leaf / REP decisions): no shift, no AND
    void put_mask(int l, int cnt, const std::string &m)
    {
        if (cnt >= 16) o << "    bw[" << l / 16 << "] = " << m << ";\n";
        else o << "    bw[" << l / 16 << "] = bsel(" << hexmask(l, cnt) << ", " << m << ", bw[" << l / 16 << "]);\n";
    }
    std::string var(const char *p) { return std::string(p) + std::to_string(nvar++) + "_"; }
    // No scheduling fences in the subtree decoders (the per-mask kernel keeps them for its
    // register budget): the machine scheduler may then overlap an op's independent prefix
    // with the previous op's dependent tail. Same box, two rounds (tools/pair_stamps.py
    // --variant nofence, profiles/r04_ab/subtree_fence_ab_stamps.txt): C5 64-frame share
    // 1326 / 1335 vs 1345 / 1350 us (subtrees -1.5 %), C3 unchanged (980 / 979 vs 989 / 975).
    void fence() {}
    void chunk_fence(int, int) {}
    // after an F-type op the parent words stay live until the matching G: an empty asm that
    // redefines them keeps the F op's intermediates from being carried across the left subtree
    void clobber_parent(int sd, int n4)
    {
        if (sd == LG) return;   // root words are re-read from the slot
        for (int i = 0; i < 2 * n4; i++) o << "  asm volatile(\"\" : \"+v\"(" << M(sd, i) << "));\n";
        for (int k = 0; k < planes(2 * n4); k++) o << "  asm volatile(\"\" : \"+v\"(s" << sd << "[" << k << "]));\n";
    }
    static const char *swp(int pd) { return pd == 2 ? "swap32" : "swap16"; }
    // split root words (for REP / R1 / SPC children of the subtree root)
    void root_split(int words)
    {
        for (int k = 0; k < planes(words); k++) o << "  s" << LG << "[" << k << "] = 0u;\n";
        for (int i = 0; i < words; i++) {
            o << "  { const u32 v_ = CH(" << i << "); " << M(LG, i) << " = v_ & MAG; s" << LG << "[" << i / 16
              << "] = plane_put<" << i % 16 << ">(s" << LG << "[" << i / 16 << "], v_); }\n";
            chunk_fence(i, words);
        }
    }
    // u flags of a small G-type op (bit 0 / 16 planes) from the left sibling's result mask
    std::string small_u(int n, int upos)
    {
        if (upos < 0) return "0u";
        const std::map<int, std::string> &m = n == 1 ? small1 : small2;
        auto it = m.find(upos);
        if (it == m.end()) throw std::runtime_error("pairgen: missing small result");
        return "(" + it->second + " & 0x00010001u)";
    }

    // ---- ops on nodes of >= 4 output words: lane-private, four words per register ----------
    void big_op(const polar_sc_op &op, int pd, int cd, int n4)
    {
        const int np = planes(n4), l0 = op.pos / wpr, ub = op.upos >= 0 ? op.upos / wpr : -1;
        const bool root = pd == LG;   // the subtree root: SM16 words re-read from its stage slot
        if (root && (op.code == POLAR_OP_REP || op.code == POLAR_OP_R1 || op.code == POLAR_OP_SPC)) root_split(2 * n4);
        if (root && op.code == POLAR_OP_F) {
            const int mw = min_width(op);
            o << "  { // F n " << op.n << " (root)\n    u32 P_[" << np << "] = {};\n";
            for (int i = 0; i < n4; i++) {
                o << "    " << M(cd, i) << " = " << (mw ? "F_root_min<" : "F_root<") << i % 16
                  << (mw ? ", " + std::to_string(mw) : std::string()) << ">(CH(" << i << "), CH(" << n4 + i << "), P_["
                  << i / 16 << "]);\n";
                chunk_fence(i, n4);
            }
            for (int k = 0; k < np; k++) o << "    s" << cd << "[" << k << "] = P_[" << k << "];\n";
            o << "  }\n";
            return;
        }
        if (root && op.code == POLAR_OP_G) {
            o << "  { // G n " << op.n << " upos " << op.upos << " (root)\n    u32 c_, P_[" << np << "] = {};\n";
            for (int i = 0; i < n4; i++) {
                if ((i & 15) == 0) o << "    c_ = " << (ub >= 0 ? get16(ub + i) : std::string("0u")) << ";\n";
                o << "    " << M(cd, i) << " = G_root<" << i % 16 << ">(CH(" << i << "), CH(" << n4 + i << "), (c_ << "
                  << 15 - (i & 15) << "), P_[" << i / 16 << "]);\n";
                chunk_fence(i, n4);
            }
            for (int k = 0; k < np; k++) o << "    s" << cd << "[" << k << "] = P_[" << k << "];\n";
            o << "  }\n";
            return;
        }
        switch (op.code) {
        case POLAR_OP_F: {
            const int mw = min_width(op);
            o << "  { // F n " << op.n << "\n";
            if (mw) o << "    u32 MP_[" << np << "] = {};\n";
            for (int i = 0; i < n4; i++) {
                if (mw)
                    o << "    " << M(cd, i) << " = F_split_min<" << i % 16 << ", " << mw << ">(" << M(pd, i) << ", "
                      << M(pd, n4 + i) << ", MP_[" << i / 16 << "]);\n";
                else
                    o << "    " << M(cd, i) << " = pk_min(" << M(pd, i) << ", " << M(pd, n4 + i) << ");\n";
                chunk_fence(i, n4);
            }
            for (int k = 0; k < np; k++)
                o << "    s" << cd << "[" << k << "] = " << P(pd, 16 * k) << " ^ " << P(pd, n4 + 16 * k)
                  << (mw ? " | MP_[" + std::to_string(k) + "]" : std::string()) << ";\n";
            o << "  }\n";
            clobber_parent(pd, n4);
            break;
        }
        case POLAR_OP_G:
            o << "  { // G n " << op.n << " upos " << op.upos << "\n    u32 X_[" << np << "], LT_[" << np << "] = {};\n";
            for (int k = 0; k < np; k++)
                o << "    X_[" << k << "] = " << P(pd, 16 * k) << " ^ " << P(pd, n4 + 16 * k) << " ^ " << U(ub, k) << ";\n";
            for (int i = 0; i < n4; i++) {
                o << "    " << M(cd, i) << " = G_split<" << i % 16 << ">(" << M(pd, i) << ", " << M(pd, n4 + i) << ", X_["
                  << i / 16 << "], LT_[" << i / 16 << "]);\n";
                chunk_fence(i, n4);
            }
            for (int k = 0; k < np; k++)
                o << "    s" << cd << "[" << k << "] = " << P(pd, n4 + 16 * k) << " ^ (X_[" << k << "] & ~LT_[" << k
                  << "]);\n";
            o << "  }\n";
            break;
        case POLAR_OP_REP: {
            // value chain in two's complement over the words in order (4 i + row), the exact
            // SM chain only when a total is 0
            o << "  { // REP n " << op.n << "\n    u32 acc_ = 0u, FS_[" << np << "];\n";
            for (int k = 0; k < np; k++)
                o << "    FS_[" << k << "] = " << P(pd, 16 * k) << " ^ " << P(pd, n4 + 16 * k) << ";\n";
            // (solo: the words of a register in order 8 i + r, then 8 i + 4 + r, into the low half)
            const int mw = min_width(op);
            if (pw) {
                for (int i = 0; i < n4; i++)
                    o << "    acc_ = rep_groups_rows(acc_, F_split_rep<" << i % 16 << ", " << mw << ">(" << M(pd, i) << ", "
                      << M(pd, n4 + i) << ", FS_[" << i / 16 << "]), ln);\n";
            }
            for (int i = 0; i < n4 && !pw; i++) {
                o << "    { const X4 t_ = rows4(row_sum_biased(" << (mw ? "F_split_biased_min<" : "F_split_biased<") << i % 16
                  << (mw ? ", " + std::to_string(mw) : std::string()) << ">(" << M(pd, i) << ", " << M(pd, n4 + i)
                  << ", FS_[" << i / 16 << "])));\n"
                  << "      acc_ = " << (solo ? "rep_acc_solo" : "rep_acc_rows") << "(acc_, t_.t0, t_.t1, t_.t2, t_.t3); }\n";
                chunk_fence(i, n4);
            }
            if (!ca2 && !pw) {   // (CA2: the two's complement chain is exact and a zero total decides 0)
                o << "    if (" << (solo ? "rep_any_zero_lo" : "rep_any_zero") << "(acc_)) {\n      acc_ = 0u;\n";
                for (int i = 0; i < n4; i++)
                    o << "      acc_ = " << (solo ? "rep_sm_solo" : "rep_sm_rows") << "(acc_, F_split_sm<" << i % 16 << ">("
                      << M(pd, i) << ", " << M(pd, n4 + i) << ", FS_[" << i / 16 << "]), ln);\n";
                o << "    }\n";
            }
            o << "    const u32 full_ = pk_sra(" << (solo ? "bcast_lo(acc_)" : "acc_") << ", 15);\n";
            for (int j = 0; j < n4; j += 16) put_mask(l0 + j, n4 < 16 ? n4 : 16, "full_");
            o << "  }\n";
            clobber_parent(pd, n4);
            break;
        }
        case POLAR_OP_R1:
        case POLAR_OP_SPC: {
            const bool spc = op.code == POLAR_OP_SPC;
            o << "  { // " << (spc ? "SPC" : "R1") << " n " << op.n << " upos " << op.upos << "\n    u32 X_[" << np
              << "], LT_[" << np << "] = {};\n";
            if (ca2) o << "    u32 NZ_[" << np << "] = {};\n";
            for (int k = 0; k < np; k++)
                o << "    X_[" << k << "] = " << P(pd, 16 * k) << " ^ " << P(pd, n4 + 16 * k) << " ^ " << U(ub, k) << ";\n";
            if (spc) o << "    u32 klo_ = 0xFFFFFFFFu, khi_ = 0xFFFFFFFFu, par_ = 0u;\n    const u32 rw_ = spc_sub(c.row, ln);\n";
            for (int i = 0; i < n4; i++) {
                // key: (|lambda|, word, bitrev4(position)); solo: word 8 i + 4 h + r (bit 6 = h)
                // (CA2: the nonzero plane of the G magnitudes)
                const std::string nzput = ca2 ? "      NZ_[" + std::to_string(i / 16) + "] = plane_put<" +
                                                    std::to_string(i % 16) + ">(NZ_[" + std::to_string(i / 16) +
                                                    "], pk_sub(0u, l_));\n"
                                              : std::string();
                if (spc)
                    o << "    { const u32 l_ = G_split<" << i % 16 << ">(" << M(pd, i) << ", " << M(pd, n4 + i) << ", X_["
                      << i / 16 << "], LT_[" << i / 16 << "]);\n" << nzput
                      << "      klo_ = __builtin_elementwise_min(klo_, (l_ << 24) | rw_ | " << (solo ? i << 7 : i << 6)
                      << "u);\n"
                      << "      khi_ = __builtin_elementwise_min(khi_, ((l_ >> 16) << 24) | rw_ | "
                      << (solo ? (i << 7) | 64 : i << 6) << "u); }\n";
                else if (ca2)
                    o << "    { const u32 l_ = G_split<" << i % 16 << ">(" << M(pd, i) << ", " << M(pd, n4 + i) << ", X_["
                      << i / 16 << "], LT_[" << i / 16 << "]);\n" << nzput << "    }\n";
                else
                    o << "    LT_[" << i / 16 << "] = plane_put<" << i % 16 << ">(LT_[" << i / 16 << "], pk_sub(" << M(pd, i)
                      << ", " << M(pd, n4 + i) << "));\n";
                chunk_fence(i, n4);
            }
            for (int k = 0; k < np; k++) {
                o << "    { const u32 h_ = "
                  << hard_plane(P(pd, n4 + 16 * k) + " ^ (X_[" + std::to_string(k) + "] & ~LT_[" + std::to_string(k) + "])",
                                "NZ_[" + std::to_string(k) + "]")
                  << ";\n";
                put(l0 + 16 * k, n4 < 16 ? n4 : 16, "h_");
                if (spc) o << "      par_ ^= h_; }\n";
                else o << "    }\n";
            }
            if (spc) {
                if (n4 < 16) {
                    const unsigned m = (1u << n4) - 1u;
                    o << "    par_ &= 0x" << std::hex << (m | (m << 16)) << std::dec << "u;\n";
                }
                if (solo) {
                    // one frame: parity of both halves, the first minimum of both
                    o << "    par_ = (__builtin_popcount(par_) & 1u) << 15;\n"
                         "    par_ = row_xor(par_);\n"
                         "    klo_ = row_min_u32(__builtin_elementwise_min(klo_, khi_));\n"
                         "    { X2 p_ = swap16(par_); par_ = p_.a ^ p_.b; p_ = swap32(par_); par_ = p_.a ^ p_.b;\n"
                         "      X2 a_ = swap16(klo_); klo_ = __builtin_elementwise_min(a_.a, a_.b);\n"
                         "      a_ = swap32(klo_); klo_ = __builtin_elementwise_min(a_.a, a_.b); }\n"
                         "    const u32 ilo_ = (klo_ >> 7) & 0x1FFFFu, hs_ = (klo_ >> 2) & 16u;\n"
                         "    const bool flo_ = land(par_ & 0x8000u, (klo_ & 63u) == rw_);\n";
                    if (n4 <= 16)
                        o << "    bw[" << l0 / 16 << "] ^= sel(flo_, 1u << (" << l0 % 16 << " + ilo_ + hs_), 0u);\n";
                    else
                        for (int k = 0; k < n4 / 16; k++)
                            o << "    bw[" << l0 / 16 + k << "] ^= sel(land(flo_, (ilo_ >> 4) == " << k
                              << "u), 1u << ((ilo_ & 15u) + hs_), 0u);\n";
                    o << "  }\n";
                    break;
                }
                o << "    par_ = ((__builtin_popcount(par_ & 0xFFFFu) & 1u) << 15) | ((__builtin_popcount(par_ >> 16) & 1u) << 31);\n"
                     "    par_ = row_xor(par_);\n"
                     "    klo_ = row_min_u32(klo_); khi_ = row_min_u32(khi_);\n"
                     "    { X2 p_ = swap16(par_); par_ = p_.a ^ p_.b; p_ = swap32(par_); par_ = p_.a ^ p_.b;\n"
                     "      X2 a_ = swap16(klo_), b_ = swap16(khi_);\n"
                     "      klo_ = __builtin_elementwise_min(a_.a, a_.b); khi_ = __builtin_elementwise_min(b_.a, b_.b);\n"
                     "      a_ = swap32(klo_); b_ = swap32(khi_);\n"
                     "      klo_ = __builtin_elementwise_min(a_.a, a_.b); khi_ = __builtin_elementwise_min(b_.a, b_.b); }\n"
                     "    const u32 ilo_ = (klo_ >> 6) & 0x3FFFFu, ihi_ = (khi_ >> 6) & 0x3FFFFu;\n"
                     "    const bool flo_ = land(par_ & 0x8000u, (klo_ & 63u) == rw_);\n"
                     "    const bool fhi_ = land(par_ & 0x80000000u, (khi_ & 63u) == rw_);\n";
                if (n4 <= 16) {
                    o << "    bw[" << l0 / 16 << "] ^= sel(flo_, 1u << (" << l0 % 16 << " + ilo_), 0u) | sel(fhi_, 0x10000u << ("
                      << l0 % 16 << " + ihi_), 0u);\n";
                } else {
                    for (int k = 0; k < n4 / 16; k++)
                        o << "    bw[" << l0 / 16 + k << "] ^= sel(land(flo_, (ilo_ >> 4) == " << k
                          << "u), 1u << (ilo_ & 15u), 0u) | sel(land(fhi_, (ihi_ >> 4) == " << k
                          << "u), 0x10000u << (ihi_ & 15u), 0u);\n";
                }
            }
            o << "  }\n";
            break;
        }
        case POLAR_OP_H:
        case POLAR_OP_H0: {
            const bool h = op.code == POLAR_OP_H;
            o << "  { // " << (h ? "H" : "H0") << " n " << op.n << "\n";
            if (n4 >= 16) {
                for (int k = 0; k < n4 / 16; k++)
                    o << "    bw[" << l0 / 16 + k << "] " << (h ? "^=" : "=") << " bw[" << (l0 + n4) / 16 + k << "];\n";
            } else {
                const int j = l0 / 16;
                if (h)
                    o << "    bw[" << j << "] ^= (bw[" << j << "] >> " << n4 << ") & " << hexmask(l0, n4) << ";\n";
                else
                    o << "    bw[" << j << "] = bsel(" << hexmask(l0, n4) << ", bw[" << j << "] >> " << n4 << ", bw[" << j
                      << "]);\n";
            }
            o << "  }\n";
            break;
        }
        default:
            throw std::runtime_error("pairgen: unexpected op");
        }
    }

    // ---- solo layout: ops with 4 output words (a parent of 8 words = one register, word
    // 4 h + r in half h, row r) ------------------------------------------------------------
    // the children of an 8-word node sit in the two halves of one register: F / REP use the
    // half rotated into place (symmetric ops: both halves get the result); G / R1 / SPC are
    // computed in the low half (a = word r, b = word r + 4) and broadcast. Decisions of a
    // 4-word node go to local word pos / 8, half (pos / 4) & 1, all rows.
    static std::string bitmask(int l, int hd)
    {
        std::ostringstream s;
        s << "0x" << std::hex << (1u << (l % 16 + 16 * hd)) << std::dec << "u";
        return s.str();
    }
    // the sign(a') ^ sign(b) plane bit 0 of a half op: sign planes of both halves + u of the left
    // sibling (half 0 of local word ub)
    std::string half_x(int pd, int ub)
    {
        std::ostringstream s;
        s << "s" << pd << "[0] ^ hswap(s" << pd << "[0])";
        if (ub >= 0) s << " ^ (bw[" << ub / 16 << "] >> " << ub % 16 << ")";
        return s.str();
    }
    void half_op(const polar_sc_op &op, int pd, int cd)
    {
        const int l = op.pos / 8, hd = (op.pos / 4) & 1, ub = op.upos >= 0 ? op.upos / 8 : -1;
        const std::string mp = M(pd, 0), sp = "s" + std::to_string(pd) + "[0]";
        switch (op.code) {
        case POLAR_OP_F:
            o << "  { // F n 4 (halves)\n    " << M(cd, 0) << " = pk_min(" << mp << ", hswap(" << mp << "));\n    s" << cd
              << "[0] = " << sp << " ^ hswap(" << sp << ");\n  }\n";
            break;
        case POLAR_OP_G:
            o << "  { // G n 4 upos " << op.upos << " (halves)\n    u32 LT_ = 0u; const u32 X_ = " << half_x(pd, ub)
              << ";\n    const u32 m_ = G_split<0>(" << mp << ", hswap(" << mp << "), X_, LT_);\n    " << M(cd, 0)
              << " = bcast_lo(m_);\n    s" << cd << "[0] = bcast_lo(hswap(" << sp << ") ^ (X_ & ~LT_));\n  }\n";
            break;
        case POLAR_OP_REP:
            o << "  { // REP n 4 (halves)\n    u32 acc_ = 0u; const u32 FS_ = " << sp << " ^ hswap(" << sp
              << "), mb_ = hswap(" << mp << ");\n"
              << "    { const X4 t_ = rows4(row_sum_biased(F_split_biased<0>(" << mp << ", mb_, FS_)));\n"
              << "      acc_ = rep_acc_rows(acc_, t_.t0, t_.t1, t_.t2, t_.t3); }\n"
              << "    if (rep_any_zero(acc_)) {\n      acc_ = rep_sm_rows(0u, F_split_sm<0>(" << mp << ", mb_, FS_), ln);\n    }\n"
              << "    bw[" << l / 16 << "] = bsel(" << bitmask(l, hd) << ", pk_sra(acc_, 15), bw[" << l / 16 << "]);\n  }\n";
            break;
        case POLAR_OP_R1:
            o << "  { // R1 n 4 upos " << op.upos << " (halves)\n    const u32 X_ = " << half_x(pd, ub)
              << ";\n    const u32 LT_ = plane_put<0>(0u, pk_sub(" << mp << ", hswap(" << mp << ")));\n"
              << "    const u32 h_ = hswap(" << sp << ") ^ (X_ & ~LT_);\n"
              << "    bw[" << l / 16 << "] = bsel(" << bitmask(l, hd) << ", h_ << " << l % 16 + 16 * hd << ", bw[" << l / 16
              << "]);\n  }\n";
            break;
        case POLAR_OP_SPC:
            o << "  { // SPC n 4 upos " << op.upos << " (halves)\n    u32 LT_ = 0u; const u32 X_ = " << half_x(pd, ub)
              << ";\n    const u32 l_ = G_split<0>(" << mp << ", hswap(" << mp << "), X_, LT_);\n"
              << "    const u32 h_ = hswap(" << sp << ") ^ (X_ & ~LT_);\n"
              << "    u32 par_ = row_xor((h_ & 1u) << 15);\n"
              << "    const u32 rw_ = spc_sub(c.row, ln);\n"
              << "    u32 klo_ = row_min_u32(((l_ & 0xFFu) << 24) | rw_);\n"
              << "    { X2 p_ = swap16(par_); par_ = p_.a ^ p_.b; p_ = swap32(par_); par_ = p_.a ^ p_.b;\n"
              << "      X2 a_ = swap16(klo_); klo_ = __builtin_elementwise_min(a_.a, a_.b);\n"
              << "      a_ = swap32(klo_); klo_ = __builtin_elementwise_min(a_.a, a_.b); }\n"
              << "    const bool flo_ = land(par_ & 0x8000u, (klo_ & 63u) == rw_);\n"
              << "    bw[" << l / 16 << "] = bsel(" << bitmask(l, hd) << ", (h_ ^ sel(flo_, 1u, 0u)) << " << l % 16 + 16 * hd
              << ", bw[" << l / 16 << "]);\n  }\n";
            break;
        case POLAR_OP_H:
        case POLAR_OP_H0: {
            // node of 8 words at pos: children in halves 0 / 1 of local word pos / 8
            const bool h = op.code == POLAR_OP_H;
            const int j = l / 16, b = l % 16;
            o << "  { // " << (h ? "H" : "H0") << " n 4 (halves)\n";
            if (h) o << "    bw[" << j << "] ^= (bw[" << j << "] >> 16) & " << (1u << b) << "u;\n";
            else o << "    bw[" << j << "] = bsel(" << (1u << b) << "u, bw[" << j << "] >> 16, bw[" << j << "]);\n";
            o << "  }\n";
            break;
        }
        default:
            throw std::runtime_error("pairgen: unexpected half op");
        }
    }

    // ---- ops with 1 or 2 output words: the cross-row steps --------------------------------
    void small_op(const polar_sc_op &op, int pd, int cd)
    {
        const int n = op.n;
        const char *sw = swp(pd);
        switch (op.code) {
        case POLAR_OP_F: {
            const int mw = min_width(op);
            o << "  { // F n " << n << "\n    const X2 m_ = " << sw << "(" << M(pd, 0) << "), s_ = " << sw << "(s" << pd
              << "[0]);\n    " << M(cd, 0);
            if (mw)
                o << " = pk_min_key<" << mw << ">(m_.a, m_.b); s" << cd << "[0] = (s_.a ^ s_.b) | plane_put<0>(0u, ca2_minbit<"
                  << mw << ">(" << M(cd, 0) << "));\n  }\n";
            else
                o << " = pk_min(m_.a, m_.b); s" << cd << "[0] = s_.a ^ s_.b;\n  }\n";
            break;
        }
        case POLAR_OP_G:
            // (G_extended inside a PAR 64 word, fb bit 19: no clamp)
            o << "  { // G n " << n << " upos " << op.upos << ((op.fb & FB_EXACT) ? " exact" : "") << "\n    const X2 m_ = "
              << sw << "(" << M(pd, 0) << "), s_ = " << sw << "(s" << pd << "[0]);\n    u32 LT_ = 0u; const u32 X_ = s_.a ^ s_.b ^ "
              << small_u(n, op.upos) << ";\n    " << M(cd, 0) << " = " << ((op.fb & FB_EXACT) ? "G_split_x" : "G_split")
              << "<0>(m_.a, m_.b, X_, LT_);\n    s" << cd << "[0] = s_.b ^ (X_ & ~LT_);\n  }\n";
            break;
        case POLAR_OP_FLEAF:
        case POLAR_OP_GLEAF: {
            const bool f = op.code == POLAR_OP_FLEAF;
            const std::string x = var("x");
            o << "  u32 " << x << ";\n  { // " << (f ? "F" : "G") << "+leaf pos " << op.pos << " fb 0x" << std::hex << op.fb
              << std::dec << "\n    const X2 m_ = swap16(" << M(pd, 0) << "), s_ = swap16(s" << pd << "[0]);\n";
            const int mw = min_width(op, !f);
            if (f && mw) {
                o << "    const u32 M_ = pk_min_key<" << mw << ">(m_.a, m_.b), S_ = plane_mask<0>(s_.a ^ s_.b) | pk_sra(ca2_minbit<"
                  << mw << ">(M_), 15);\n";
            } else if (f) {
                o << "    const u32 M_ = pk_min(m_.a, m_.b), S_ = plane_mask<0>(s_.a ^ s_.b);\n";
            } else {
                o << "    const u32 xm_ = opaque(plane_mask<0>(s_.a ^ s_.b ^ " << small_u(1, op.upos) << "));\n"
                  << "    const u32 d_ = pk_sub(m_.a, m_.b);\n"
                  << ((op.fb & FB_EXACT) ? "    const u32 M_ = bsel(xm_, pk_abs_i16(d_), pk_add(m_.a, m_.b));\n"
                                         : "    const u32 M_ = pk_min(bsel(xm_, pk_abs_i16(d_), pk_add(m_.a, m_.b)), GSAT2);\n")
                  << "    const u32 S_ = plane_mask<0>(s_.b) ^ (xm_ & ~pk_sra(d_, 15));\n";
            }
            if (pw)
                o << "    " << x << " = leaf_word_gen<0x" << std::hex << (op.fb & 0xFFFFu) << "u, 0x" << (uint32_t)op.reserved[1]
                  << std::dec << "u>(M_, S_, ln);\n  }\n";
            else if (ca2)
                o << "    " << x << " = leaf_gen_ca2<0x" << std::hex << (op.fb & 0x7FFFFu) << std::dec << "u, " << mw
                  << ">(M_, S_, ln);\n  }\n";
            else
                o << "    " << x << " = leaf_gen<0x" << std::hex << (op.fb & 0x7FFFFu) << std::dec << "u>(M_, S_, ln);\n  }\n";
            small1[op.pos] = x;
            break;
        }
        case POLAR_OP_REP: {
            const std::string x = var("x");
            const int mw = min_width(op);
            o << "  u32 " << x << ";\n  { // REP n " << n << "\n    const X2 m_ = " << sw << "(" << M(pd, 0)
              << "), s_ = " << sw << "(s" << pd << "[0]);\n    const u32 FS_ = s_.a ^ s_.b;\n";
            if (pw) {
                o << "    const u32 acc_ = " << (n == 1 ? "rep_groups_1" : "rep_groups_2") << "(F_split_rep<0, " << mw
                  << ">(m_.a, m_.b, FS_), ln);\n"
                  << "    " << x << " = pk_sra(acc_, 15);\n  }\n";
                (n == 1 ? small1 : small2)[op.pos] = x;
                break;
            }
            o << "    const u32 t_ = row_sum_biased("
              << (mw ? "F_split_biased_min<0, " + std::to_string(mw) + ">" : std::string("F_split_biased<0>"))
              << "(m_.a, m_.b, FS_));\n";
            // (2 words: two PAR 16 words in order, or one PAR 32 word -- rep2_acc / rep2_sm)
            if (n == 1) o << "    u32 acc_ = rep_acc(0u, t_);\n";
            else o << "    u32 acc_ = rep2_acc(t_);\n";
            if (!ca2) {
                o << "    if (rep_any_zero(acc_)) {\n";
                if (n == 1) o << "      acc_ = G_sm<REPSAT>(row_add_tree(F_split_sm<0>(m_.a, m_.b, FS_), ln), 0u, 0u);\n";
                else o << "      acc_ = rep2_sm(F_split_sm<0>(m_.a, m_.b, FS_), ln);\n";
                o << "    }\n";
            }
            o << "    " << x << " = pk_sra(acc_, 15);\n  }\n";
            (n == 1 ? small1 : small2)[op.pos] = x;
            break;
        }
        case POLAR_OP_R1:
        case POLAR_OP_SPC: {
            const bool spc = op.code == POLAR_OP_SPC;
            const std::string x = var("x");
            o << "  u32 " << x << ";\n  { // " << (spc ? "SPC" : "R1") << " n " << n << "\n    const X2 m_ = " << sw << "("
              << M(pd, 0) << "), s_ = " << sw << "(s" << pd << "[0]);\n    u32 LT_ = 0u; const u32 X_ = s_.a ^ s_.b ^ "
              << small_u(n, op.upos) << ";\n";
            if (!spc && ca2) {
                o << "    const u32 l_ = G_split<0>(m_.a, m_.b, X_, LT_);\n"
                  << "    " << x << " = ca2_nzs(l_, plane_mask<0>(s_.b ^ (X_ & ~LT_)));\n  }\n";
            } else if (!spc) {
                o << "    LT_ = plane_put<0>(0u, pk_sub(m_.a, m_.b));\n"
                  << "    " << x << " = plane_mask<0>(s_.b ^ (X_ & ~LT_));\n  }\n";
            } else {
                o << "    const u32 l_ = G_split<0>(m_.a, m_.b, X_, LT_);\n"
                  << "    const u32 h_ = " << (ca2 ? "ca2_nzs(l_, plane_mask<0>(s_.b ^ (X_ & ~LT_)))" : "plane_mask<0>(s_.b ^ (X_ & ~LT_))")
                  << ";\n"
                  << "    u32 par_ = row_xor(h_);\n";
                // key bits below the magnitude: bitrev4(position), and for 2 words the word
                // (PAR 16: above it; PAR 32: below it, spc_sub2)
                const std::string wk = n == 1 ? "spc_lk(ln)" : "spc_sub2(c.row, ln)";
                o << "    u32 klo_ = row_min_u32(((l_ & 0xFFu) << 24) | " << wk << ");\n"
                  << "    u32 khi_ = row_min_u32((((l_ >> 16) & 0xFFu) << 24) | " << wk << ");\n";
                if (n == 2)
                    o << "    { const X2 p_ = swap16(par_); par_ = p_.a ^ p_.b;\n"
                         "      const X2 a_ = swap16(klo_), b_ = swap16(khi_);\n"
                         "      klo_ = __builtin_elementwise_min(a_.a, a_.b); khi_ = __builtin_elementwise_min(b_.a, b_.b); }\n";
                const std::string kb = n == 1 ? "15u" : "31u";
                o << "    const bool flo_ = land(par_ & 0x8000u, (klo_ & " << kb << ") == " << wk << ");\n"
                  << "    const bool fhi_ = land(par_ & 0x80000000u, (khi_ & " << kb << ") == " << wk << ");\n"
                  << "    " << x << " = h_ ^ sel(flo_, 0xFFFFu, 0u) ^ sel(fhi_, 0xFFFF0000u, 0u);\n  }\n";
            }
            (n == 1 ? small1 : small2)[op.pos] = x;
            break;
        }
        case POLAR_OP_H:
        case POLAR_OP_H0: {
            const bool h = op.code == POLAR_OP_H;
            if (n == 1) {
                // node of 2 words at pos: row r holds word r & 1 = [xL ^ xR, xR]
                const std::string x = var("x"), R = small1.at(op.pos + 1);
                o << "  const u32 " << x << " = " << R;
                if (h) o << " ^ (" << small1.at(op.pos) << " & row_even(c.row))";
                o << ";   // " << (h ? "H" : "H0") << " n 1\n";
                small2[op.pos] = x;
            } else {
                // node of 4 words at pos: row r holds word r, into the partial sums at local pos / 4
                const std::string R = small2.at(op.pos + 2);
                // (block-local names never end in a digit + '_': the small results are x<k>_)
                o << "  { // " << (h ? "H" : "H0") << " n 2\n    const u32 w_ = " << R;
                if (h) o << " ^ (" << small2.at(op.pos) << " & row_lo2(c.row))";
                o << ";\n";
                if (solo) {   // local word pos / 8, half (pos / 4) & 1
                    const int l = op.pos / 8;
                    o << "    bw[" << l / 16 << "] = bsel(" << bitmask(l, (op.pos / 4) & 1) << ", w_, bw[" << l / 16 << "]);\n";
                } else {
                    put_mask(op.pos / 4, 1, "w_");
                }
                o << "  }\n";
            }
            break;
        }
        default:
            throw std::runtime_error("pairgen: unexpected small op");
        }
    }

    // PAR 32 / 64, PRUNING_LEVEL 1: the leaf decoder of the PAR word the previous F / G wrote
    // (this record's own node, 2 / 4 words: polar_sc_pair.h pleaf_pair)
    void pleaf_op(const polar_sc_op &op, int pd)
    {
        const unsigned kind = (op.fb >> 16) & 7u;
        const std::string x = var("x"), mp = M(pd, 0);
        o << "  u32 " << x << ";\n  { // PLEAF n " << op.n << " kind " << kind << "\n    const u32 sm_ = plane_mask<0>(s" << pd
          << "[0]);\n    " << x << " = pk_sra(pleaf_pair<" << kind << ">("
          << (ca2 ? "pk_sub(" + mp + " ^ sm_, sm_)" : mp + " | (sm_ & SGN)") << ", ln, c.row), 15);\n  }\n";
        if (op.n == 2) small2[op.pos] = x;
        else if (op.n == wpr) put_mask(op.pos / wpr, 1, x);
        else throw std::runtime_error("pairgen: PLEAF of an unexpected size");
    }

    void op(const polar_sc_op &op)
    {
        const int pd = LG - op.level, cd = pd - 1;
        fence();
        if (op.code == POLAR_OP_PLEAF) {
            pleaf_op(op, pd);
            return;
        }
        if (op.code == POLAR_OP_H || op.code == POLAR_OP_H0) {
            // H of a node of 2n words: small when the node is 2 or 4 words
            if (op.n <= 2) small_op(op, pd, cd);
            else if (op.n < wpr) half_op(op, pd, cd);
            else big_op(op, pd, cd, op.n / wpr);
            return;
        }
        if (op.n >= wpr) big_op(op, pd, cd, op.n / wpr);
        else if (op.n == 4 && solo) half_op(op, pd, cd);
        else small_op(op, pd, cd);
    }

    // subtree decoder `id`: root words from the slot dwords at src_ (rows j, j + 1: CH), partial sums to
    // the pair's bit dwords from local word l0
    // inl: inlined at its call sites (polar_sc_tuning.sub_inline = 2) instead of a call
    // kind: where the root words come from (CH(j), defined before the function): 0 = the
    // root's stage slot at src_; 1 / 2 = F / G of the parent's slot rows at src_ (G: the partial
    // sums of the left sibling from local word ub_, -1 = zero)
    void sub_function(int id, bool inl, int kind = 0)
    {
        const int words = 1 << LG, R = regs(LG), lw = words / wpr, nbw = lw >= 16 ? lw / 16 : 1;   // lw: local words
        const int nq = words / wpr;   // rows of the root node (the parent has 2 nq)
        o << "#undef CH\n";
        if (kind == 0) o << "#define CH(j) prow(SLOT(j), ((j) & 1) != 0)\n";
        else if (kind == 1) o << "#define CH(j) prow(fg4<false>(SLOT(j), SLOT((j) + " << nq << "), 0u), ((j) & 1) != 0)\n";
        else
            o << "#define CH(j) prow(fg4<true>(SLOT(j), SLOT((j) + " << nq << "), ub_ >= 0 ? ubits4(hb_[((ub_ + ((j) & ~1)) >> 4) * 64], "
              << "ub_ + ((j) & ~1)) : 0u), ((j) & 1) != 0)\n";
        // (plain arguments: a PairCtx passed by reference would live on the private stack)
        o << "__device__ " << (inl ? "__forceinline__" : "__noinline__") << " void polar_psub_" << id
          << (kind == 1 ? "_F" : kind == 2 ? "_G" : "") << (left ? "_L" : "") << "(const u32 *src_, g_u32 *hb_, int l0"
          << (kind == 2 ? ", int ub_" : "") << ")\n{\n"
          << "  const u32 lane_ = threadIdx.x & 63u;\n  Lanes ln; ln.init(lane_ & 15u);\n"
          << "  struct { u32 row; } c; c.row = lane_ >> 4;\n  u32 bw[" << nbw << "] = {};\n";
        bool split_root = false;   // REP / R1 / SPC children of the root read split root words
        for (const polar_sc_op &op : ops)
            if (op.level == 0 && (op.code == POLAR_OP_REP || op.code == POLAR_OP_R1 || op.code == POLAR_OP_SPC))
                split_root = true;
        for (int d = 0; d <= LG; d++)
            if (d < LG || split_root)
                o << "  u32 m" << d << "[" << regs(d) << "], s" << d << "[" << planes(regs(d)) << "];\n";
        (void)R;
        for (const polar_sc_op &op : ops) {
            if (op.code == POLAR_OP_END) break;
            this->op(op);
        }
        if (lw >= 16) {
            for (int j = 0; j < nbw; j++) o << "  BST(" << j << ", bw[" << j << "]);\n";
        } else {
            const unsigned m = (1u << lw) - 1u;
            o << "  BSTM(0x" << std::hex << (m | (m << 16)) << std::dec << "u, bw[0]);\n";
        }
        o << "}\n\n";
    }
};
// a root word of a subtree decoder: row j of its stage slot (row-pair dwords, SM8) -> SM16
// partial-sum dword d of the subtree to the pair's bits (masked: subtrees of < 64 words)
// SLOT(j): the slot dword of rows j & ~1, (j & ~1) + 1 (row pairs, 8-row groups); CH(j): a root
// row of a subtree decoder (defined per decoder variant, PairGen::sub_function)
const char *const kPairCH = "#define SLOT(j) src_[((j) >> 3) * 256 + (((j) >> 1) & 3)]\n"
                            "#define BST(d, v) (hb_[((l0 >> 4) + (d)) * 64] = (v))\n"
                            "#define BSTM(m, v) (hb_[(l0 >> 4) * 64] = (hb_[(l0 >> 4) * 64] & ~((m) << (l0 & 15))) | \\\n"
                            "    (((v) << (l0 & 15)) & ((m) << (l0 & 15))))\n";

// upper-level record -> call of a polar_sc_pair.h loop function
// (wpr: words per slot row of one (virtual) frame -- 4 pair, 8 solo)
// ca2: the SUB at word 0 calls the _L variant of its decoder (PairGen::left)
void upper_call(std::ostringstream &o, const polar_sc_op &op, int wpr, bool ca2)
{
    const char *lv = ca2 && op.pos == 0 ? "_L" : "";
    const int n4 = op.n / wpr, l0 = op.pos / wpr, ub = op.upos >= 0 ? op.upos / wpr : -1;
    o << "    c.sync(); ";
    switch (op.code) {
    case POLAR_OP_F: o << "pop_fg_split<false>(c, " << op.level << ", " << n4 << ", -1);"; break;
    case POLAR_OP_G: o << "pop_fg_split<true>(c, " << op.level << ", " << n4 << ", " << ub << ");"; break;
    case POLAR_OP_REP: o << "if (c.lead()) pop_rep(c, " << op.level << ", " << n4 << ", " << l0 << ");"; break;
    case POLAR_OP_R1: o << "pop_r1spc<false>(c, " << op.level << ", " << n4 << ", " << ub << ", " << l0 << ");"; break;
    case POLAR_OP_SPC: o << "pop_r1spc<true>(c, " << op.level << ", " << n4 << ", " << ub << ", " << l0 << ");"; break;
    case POLAR_OP_H: o << "pop_h<false>(c, " << l0 << ", " << n4 << ");"; break;
    case POLAR_OP_H0: o << "pop_h<true>(c, " << l0 << ", " << n4 << ");"; break;
    case POLAR_OP_SUB:
        if (op.reserved[1] == 0)
            o << "if (c.lead()) polar_psub_" << op.fb << lv << "(c.slot_ptr(c.lvl_row(" << op.level << ")), c.hb, " << l0 << ");";
        else   // the root as F / G of the parent's slot rows (pair_fused)
            o << "if (c.lead()) polar_psub_" << op.fb << (op.reserved[1] == 1 ? "_F" : "_G") << lv << "(c.slot_ptr(c.lvl_row("
              << op.level - 1 << ")), c.hb, " << l0 << (op.reserved[1] == 2 ? ", " + std::to_string(ub) : std::string())
              << ");";
        break;
    default: throw std::runtime_error("pairgen: unexpected upper op");
    }
    o << "   // " << op.code << " level " << op.level << " n " << op.n << " pos " << op.pos << "\n";
}

// F / G records that fuse into one pop_chain call (polar_sc_pair.h): record i + 1 is F, or G
// with zero partial sums (the H0 route), on the node record i wrote -- one level down, half the
// words. At most PAIR_CHAIN_MAX records (2^(D-1) row groups of each operand per column): a
// noinline chain of 4 records takes the kernel to the full 256 registers of an 8-wave block
// (torch's hipRTC: 128 VGPRs + 128 AGPRs and 760 B of scratch; the ROCm clang driver: 256
// VGPRs, 548 B), 3 records stay well below. The round-3 dispatch abort of a chain-4 plan
// (HSA_STATUS_ERROR_INVALID_ISA) does not recur with either object of the committed source:
// both dispatch at 8 waves, also with the scratch padded to the aborted dispatch's 812 B
// (tools/rtc_isa_check.py, tools/isa_dispatch_probe.cpp, profiles/r05_ab/isa_r3_probe.log);
// what an 8-wave block needs is ceil(8 / 4) x the descriptor's unified register count <= 512,
// which the launch guard enforces (polar_sc_jit.cpp kernel_regs / fit_waves).
constexpr int PAIR_CHAIN_MAX = 3;
int chain_len(const std::vector<polar_sc_op> &ops, size_t i, int cmax)
{
    const polar_sc_op &o0 = ops[i];
    if (o0.code != POLAR_OP_F && o0.code != POLAR_OP_G) return 1;
    int d = 1;
    while (d < cmax && i + d < ops.size()) {
        const polar_sc_op &p = ops[i + d - 1], &q = ops[i + d];
        const bool fg = q.code == POLAR_OP_F || (q.code == POLAR_OP_G && q.upos < 0);
        if (!fg || q.level != p.level + 1 || 2 * q.n != p.n) break;
        d++;
    }
    return d;
}
void chain_call(std::ostringstream &o, const std::vector<polar_sc_op> &ops, size_t i, int d, int wpr)
{
    const polar_sc_op &o0 = ops[i];
    unsigned gm = 0;
    for (int k = 1; k < d; k++)
        if (ops[i + k].code == POLAR_OP_G) gm |= 1u << k;
    const bool g0 = o0.code == POLAR_OP_G;
    o << "    c.sync(); pop_chain<" << d << ", " << (o0.level == 0 ? "true" : "false") << ", " << (g0 ? "true" : "false")
      << ">(c, " << o0.level << ", " << o0.n / wpr << ", " << (g0 && o0.upos >= 0 ? o0.upos / wpr : -1) << ", " << gm
      << "u);   // chain";
    for (int k = 0; k < d; k++) {
        const polar_sc_op &q = ops[i + k];
        o << (k ? " |" : "") << " " << q.code << " level " << q.level << " n " << q.n << " pos " << q.pos;
    }
    o << "\n";
}

// one decode kernel: a block of W waves per frame pair; `seg` selects the schedule segment
// (the cases between POLAR_OP_SEGEND records; 0 when the plan has no grid tier)
void pair_kernel(std::ostringstream &o, const char *name, const std::vector<polar_sc_op> &ops, int cmax, bool solo,
                 bool ca2)
{
    const int wpr = solo ? 8 : 4;
    o << "extern \"C\" __global__ void __launch_bounds__(" << 64 * PAIR_WAVES_MAX << ") " << name << "(\n"
      << "    const signed char *__restrict__ llr, unsigned short *__restrict__ out, unsigned int *__restrict__ scratch,\n"
      << "    int N, int batch, int out_stride, int pair_dwords, int slot_rows, int lds_row0, int seg)\n{\n"
      << "  extern __shared__ __attribute__((aligned(16))) unsigned int smem_[];\n"
      << "  PairCtx c;\n"
      << "  const int W = blockDim.x >> 6, wi = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n"
      << "  const long pair = blockIdx.x;   // (solo: the frame)\n"
      << "  if (" << (solo ? "pair" : "2 * pair") << " >= batch) return;\n"
      << "  pair_init(c, llr, scratch, N, batch, pair, pair_dwords, slot_rows, lds_row0, wi, W, (lds_w32 *)smem_);\n"
      << "  switch (seg) {\n  case 0:\n";
    int seg = 0;
    for (size_t i = 0; i < ops.size(); i++) {
        const polar_sc_op &op = ops[i];
        if (op.code == POLAR_OP_END) break;
        if (op.code == POLAR_OP_SEGEND) {
            o << "    return;\n  case " << ++seg << ":\n";
            continue;
        }
        const int d = chain_len(ops, i, cmax);
        if (d >= 2) {
            chain_call(o, ops, i, d, wpr);
            i += (size_t)d - 1;
            continue;
        }
        upper_call(o, op, wpr, ca2);
    }
    o << "    c.sync();\n";
    if (solo)
        o << "    pair_out(c, (g_u16 *)out + pair * (long)out_stride, (g_u16 *)out + pair * (long)out_stride, true, false,\n"
          << "             out_stride);\n";
    else
        o << "    pair_out(c, (g_u16 *)out + (2 * pair) * (long)out_stride, (g_u16 *)out + (2 * pair + 1) * (long)out_stride,\n"
          << "             2 * pair < batch,\n"
          << "             2 * pair + 1 < batch, out_stride);\n";
    o << "    return;\n  default: return;\n  }\n}\n";
}

}  // namespace

// The whole generated source of a pair plan: subtree decoders, the decode kernel (one case
// per schedule segment of the grid tier, or one), the tier kernel.
std::string pair_source(const polar_sc_plan &p)
{
    std::ostringstream o;
    const bool solo = p.solo != 0;
    const bool ca2 = p.cfg.sigmag == 0;
    const bool s16 = p.wide_slots();   // 16-bit slot rows (polar_sc_pair.h POLAR_PAIR_S16)
    const int wpr = solo ? 8 : 4;
    o << "#define POLAR_LANE_REMAP 1\n" << (solo ? "#define POLAR_SOLO 1\n" : "") << (ca2 ? "#define POLAR_CA2 1\n" : "")
      << "#define POLAR_Q " << p.cfg.llr_bits
      << "\n#define POLAR_LPAR "
      << (p.cfg.par == 64 ? 6 : p.cfg.par == 32 ? 5 : p.cfg.par == 16 ? 4 : p.cfg.par == 8 ? 3 : 2)
      << "\n" << (p.cfg.extended ? "" : "#define POLAR_EXT 0\n")   // EXTENDED = 0: saturating leaves
      << "#include \"polar_sc_pair.h\"\n"
      << "namespace polar {\n"
      // (16-bit slots, LLR_BITS 9: a row pair is two SM16 dwords, 8-row groups of 8 dwords per lane)
      << (s16 ? "#define SLOT(j) (*(const su_t *)(src_ + ((j) >> 3) * 512 + (((j) >> 1) & 3) * 2))\n" : "")
      << (s16 ? kPairCH + std::string(kPairCH).find('\n') + 1 : kPairCH);
    int lg = 0;
    while ((1 << lg) < p.sub_words) lg++;
    // the decoder variants the kernels call (SUB records: reserved[1] = root kind), and the
    // subtest kernel's (kind 1 of a fused plan: its root rows fed through F with +QMAG)
    // (CA2: the decoder of the subtree at word 0 also as its _L variant, PairGen::left)
    std::set<std::tuple<int, int, bool>> need;
    for (const std::vector<polar_sc_op> *ops : {&p.pair_ops, &p.pair_tier.seg_ops})
        for (const polar_sc_op &op : *ops)
            if (op.code == POLAR_OP_SUB) need.insert({(int)op.fb, op.reserved[1], ca2 && op.pos == 0});
    for (size_t id = 0; id < p.subs.size(); id++) need.insert({(int)id, p.pair_fused ? 1 : 0, false});
    for (const auto &v : need) {
        PairGen g(p.subs[std::get<0>(v)], lg, solo);
        g.ca2 = ca2;
        g.left = std::get<2>(v);
        g.q = p.cfg.llr_bits;
        g.p16 = (int)p.p16;
        g.pw = p.ppw > 1;
        g.sub_function(std::get<0>(v), p.tune.sub_inline == 2, std::get<1>(v));
        o << g.o.str();
    }
    o << "}  // namespace polar\nusing namespace polar;\n";
    // the decode kernel over the whole schedule, and (grid-tier plans) the segment kernel
    const int cmax = p.tune.chain_max ? p.tune.chain_max : PAIR_CHAIN_MAX;
    pair_kernel(o, "polar_sc_pair_kernel", p.pair_ops, cmax, solo, ca2);
    // test hook (polar_sc_debug_subtree): subtree decoder `id` on 64 lanes of root slot rows
    // in[64 j + lane] (u16 SM8 pairs, repacked into row-pair dwords in LDS), its partial-sum
    // dwords to out[64 d + lane]
    // (fused plans: the decoder reads its root as F of parent rows = [the root rows; +QMAG],
    // which gives back the root rows exactly, -0 included)
    const int rp = p.sub_words / wpr / 2;   // row-pair dwords of the root slot
    const int tot = p.pair_fused ? 2 * rp : rp;
    const int gd = s16 ? 8 : 4;             // dwords per lane of an 8-row group
    o << "extern \"C\" __global__ void __launch_bounds__(64) polar_sc_pair_subtest_kernel(\n"
      << "    const unsigned short *__restrict__ in, unsigned int *__restrict__ out, int id)\n{\n"
      << "  __shared__ unsigned int rows_[" << (tot < 4 ? 4 : tot) * gd / 4 << " * 64];\n"
      << "  const int lane = threadIdx.x & 63;\n";
    if (!s16) {
        if (p.pair_fused)
            o << "  for (int i = " << rp << "; i < " << tot << "; i++) rows_[(i >> 2) * 256 + 4 * lane + (i & 3)] = QMAG * 0x01010101u;\n";
        o << "  for (int i = 0; i < " << rp << "; i++) {\n"
          << "    const unsigned int r0 = in[128 * i + lane], r1 = in[128 * i + 64 + lane];\n"
          << "    rows_[(i >> 2) * 256 + 4 * lane + (i & 3)] = (r0 & 0xFFu) | ((r1 & 0xFFu) << 8) | ((r0 >> 8) << 16) |\n"
          << "                                                ((r1 >> 8) << 24);\n"
          << "  }\n";
    } else {   // the SM8 test rows as SM16 pairs, two dwords per row pair
        if (p.pair_fused)
            o << "  for (int i = " << 2 * rp << "; i < " << 2 * tot << "; i++) rows_[(i >> 3) * 512 + 8 * lane + (i & 7)] = QMAG * 0x00010001u;\n";
        o << "  for (int i = 0; i < " << 2 * rp << "; i++) {\n"
          << "    const unsigned int v = in[64 * i + lane];\n"
          << "    rows_[(i >> 3) * 512 + 8 * lane + (i & 7)] = (v & 0x7Fu) | ((v & 0x80u) << 8) | (((v >> 8) & 0x7Fu) << 16) |\n"
          << "                                                ((v & 0x8000u) << 16);\n"
          << "  }\n";
    }
    o << "  const unsigned int *src = rows_ + " << gd << " * lane;\n"
      << "  switch (id) {\n";
    for (size_t id = 0; id < p.subs.size(); id++)
        o << "  case " << id << ": polar_psub_" << id << (p.pair_fused ? "_F" : "") << "(src, (g_u32 *)out + lane, 0); return;\n";
    o << "  default: return;\n  }\n}\n";
    if (!p.pair_tier.steps.empty()) {
        pair_kernel(o, "polar_sc_pair_seg_kernel", p.pair_tier.seg_ops, cmax, solo, ca2);
        o << "extern \"C\" __global__ void __launch_bounds__(256) polar_sc_pair_tier_kernel(\n"
          << "    const signed char *__restrict__ llr, unsigned int *__restrict__ scratch, int N, int batch, int pair_dwords,\n"
          << "    int slot_rows, int code_g, int k, int n4, int ub, int cw)\n{\n"
          << "  pair_tier_body(llr, scratch, N, batch, pair_dwords, slot_rows, code_g, k, n4, ub, cw);\n}\n";
    }
    return o.str();
}

}  // namespace polar_host
