// polar_sc_host.cpp -- host side of libpolar_sc.so: plan / schedule compiler / table
// loaders / C ABI (include/polar_sc.h).
//
// The reference decoder (SC_MODULE my_module, src/module/my_module.h) walks the polar code
// tree with an FSM whose sequence of states, sizes and addresses depends only on the
// frozen-bit table (my_module.h:61-166 classifies 16-bit groups, then every transition is
// a function of those classes). This file "compiles" that walk once per table into a flat
// op list (polar_sc_op); the GPU kernel interprets the list with wave-uniform control.
#include "polar_sc_plan.hpp"

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

extern "C" int polar_sc_launch_widen(const int8_t *in_dev, int16_t *out_dev, size_t n, void *stream);
extern "C" int polar_sc_launch_decode(int gmem, const int8_t *llr, uint16_t *out, const void *ops,
                                      uint32_t *scratch, int N, long batch, int out_stride,
                                      int waves_per_group, int groups_per_block, int group_dwords,
                                      int lds_dwords, int lds0, void *stream, unsigned long long *trace);
extern "C" int polar_sc_launch_selftest(uint32_t *out_dev);

using polar_host::DevState;

namespace {

// node codes of shared/src/library.h:34-40
constexpr uint32_t NODE_R0 = 0x00, NODE_R1 = 0x0F, NODE_REP = 0x02, NODE_SPC = 0x04, NODE_RN = 0x08;

// largest per-wave LDS footprint kept on chip; above it stages go to HBM scratch
constexpr uint32_t LDS_WAVE_LIMIT = 80u * 1024u;   // all-LDS interpreter limit per 8-frame group
constexpr int LDS_LOW_SLOTS = 256;                  // HBM mode: default LDS region W (slots; the levels of nodes <= W / 2 words)

}  // namespace

namespace {

// do_prunning (my_module.h:75-155): group class, priority R0 > R1 > REP > SPC > REP2 > SPC2
// > RN, each recognised only when PRUNING_LEVEL > 0 and its ELAG_* switch is on
// (my_module.h:129-153). REP2 = only the last two bits information, SPC2 = only the first
// two frozen (my_module.h:108-125).
// PAR-bit groups (fb bit k = frozen-table bit PAR g + k): REP = only bit PAR-1 information,
// SPC = only bit 0 frozen, REP2 / SPC2 = the last two / first two.
constexpr uint32_t NODE_REP2 = 0x03, NODE_SPC2 = 0x05;
uint32_t classify_group(uint64_t fb, uint32_t par, const polar_sc_config &c)
{
    const uint64_t all = par >= 64 ? ~0ull : ((1ull << par) - 1ull);
    if (c.pruning_level == 0) return NODE_RN;
    if (fb == 0u) return NODE_R0;
    if (c.elag_r1 && fb == all) return NODE_R1;
    if (c.elag_rep && fb == 1ull << (par - 1)) return NODE_REP;
    if (c.elag_spc && fb == (all & ~1ull)) return NODE_SPC;
    if (c.elag_rep2 && fb == 3ull << (par - 2)) return NODE_REP2;
    if (c.elag_spc2 && fb == (all & ~3ull)) return NODE_SPC2;
    return NODE_RN;
}

// PRUNING_LEVEL 1 leaf decoders selected in R_STATE by the group's class
// (my_module.h:566-593; library.h:175-280): REP / SPC, or with ELAG_REP2 / ELAG_SPC2 the
// REP_REP2 / SPC_SPC2 decoders (sel = class bit 0). R0 groups give the plain leaf's result
// (all zero); so do R1 groups in SIGMAG (the hard decisions), not in CA2.
uint32_t leaf_kind(const polar_sc_plan &p, uint32_t g)
{
    if (p.cfg.pruning_level != 1) return POLAR_LEAF_PLAIN;
    switch (p.type[g]) {
    case NODE_REP: return POLAR_LEAF_REP;
    case NODE_SPC: return POLAR_LEAF_SPC;
    case NODE_REP2: return p.cfg.elag_rep ? POLAR_LEAF_REP2 : POLAR_LEAF_PLAIN;
    case NODE_SPC2: return p.cfg.elag_spc ? POLAR_LEAF_SPC2 : POLAR_LEAF_PLAIN;
    case NODE_R1: return p.cfg.sigmag ? POLAR_LEAF_PLAIN : POLAR_LEAF_R1;
    default: return POLAR_LEAF_PLAIN;
    }
}

// Node class of a multi-group node as aggregated in the F/G loops
// (my_module.h:403-471, 739-806): all R0 -> R0; all R1 -> R1; all R0 but a REP last group
// -> REP; an SPC first group then all R1 -> SPC; otherwise RN.
uint32_t node_class(const polar_sc_plan &p, uint32_t g0, uint32_t cnt)
{
    uint32_t R0 = 0, R1 = 0x0F;
    bool r0_but_last = true, r1_but_first = true;
    for (uint32_t t = 0; t < cnt; t++) {
        uint32_t T = p.type[g0 + t];
        R0 |= T;
        R1 &= T;
        if (t + 1 < cnt && T != NODE_R0) r0_but_last = false;
        if (t > 0 && T != NODE_R1) r1_but_first = false;
    }
    if (R0 == NODE_R0) return NODE_R0;
    if (R1 == NODE_R1) return NODE_R1;
    if (r0_but_last && p.type[g0 + cnt - 1] == NODE_REP) return NODE_REP;
    if (r1_but_first && p.type[g0] == NODE_SPC) return NODE_SPC;
    return NODE_RN;
}

void emit(std::vector<polar_sc_op> &out, int code, int level, int n, int pos, int upos, uint32_t fb)
{
    polar_sc_op o{};
    o.code = code;
    o.level = level;
    o.n = n;
    o.pos = pos;
    o.upos = upos;
    o.fb = fb;
    out.push_back(o);
}

// hybrid plans: distinct subtree schedules (keyed by their bytes) collected while compiling
struct SubCtx {
    uint32_t words = 0;
    std::map<std::string, int> ids;
    std::vector<std::vector<polar_sc_op>> lists;
    uint32_t calls = 0;
};

// HBM-scratch plans: the device copy of the schedule brackets every subtree of <= 128 words
// (LDS_LOW_SLOTS) with POLAR_OP_WOPEN / POLAR_OP_WFLUSH and flags its ops (reserved[0] = 1):
// their partial-sum dwords live in an LDS window (cleared on open, written to the HBM bits on
// flush). The subtree's ops are contiguous in the schedule and touch only bits of their own
// subtree; the ops of larger nodes run after the flush and use the HBM copy. The exported
// schedule (polar_sc_plan_get_schedule) stays the plain one.
void window_schedule(const polar_sc_plan &p, const std::vector<polar_sc_op> &ops, std::vector<polar_sc_op> &dev)
{
    const int W = p.lds_slots;
    dev.clear();
    int cur = -1;
    auto mark = [&](int code, int pos) {
        polar_sc_op o{};
        o.code = code;
        o.pos = pos;
        o.upos = -1;
        dev.push_back(o);
    };
    for (const polar_sc_op &op : ops) {
        int win = -1;
        if (op.code == polar_host::POLAR_OP_SUB) {
            if (op.n <= W) win = (op.pos / W) * W;   // the subtree's own words [pos, pos + n)
        } else if (op.code != POLAR_OP_END && 2 * op.n <= W) {
            const bool right = op.code == POLAR_OP_G || op.code == POLAR_OP_R1 || op.code == POLAR_OP_SPC ||
                               op.code == POLAR_OP_GLEAF;
            const int node = right ? op.pos - op.n : op.pos;
            win = (node / W) * W;
        }
        if (win != cur) {
            if (cur >= 0) mark(polar_host::POLAR_OP_WFLUSH, cur);
            if (win >= 0) mark(polar_host::POLAR_OP_WOPEN, win);
            cur = win;
        }
        polar_sc_op o = op;
        o.reserved[0] = win >= 0 ? 1 : 0;
        dev.push_back(o);
    }
}

// Grid tier: cut the device schedule of a hybrid HBM-scratch plan at every F / G record of
// at least `tw` output words (the upper tree levels; their source and destination levels are
// HBM slots). Those records become grid-wide launches over all frame groups; the records
// between them become segments for the hybrid kernel, closed by POLAR_OP_SEGEND (the last one
// by the END record) and opened by POLAR_OP_SEGCONT after the first. The H / H0 records of
// the cut nodes stay in the segments, in schedule order, so every launch sees the partial
// sums of the launches before it (kernel boundaries order the HBM traffic).
polar_host::TierPlan tier_schedule(const polar_sc_plan &p, int tw)
{
    polar_host::TierPlan t;
    const std::vector<polar_sc_op> &ops = p.dev_ops;
    bool any = false;
    for (const polar_sc_op &o : ops)
        if ((o.code == POLAR_OP_F || o.code == POLAR_OP_G) && o.n >= tw) any = true;
    if (!any) return t;
    bool open = false;
    auto mark = [&](int code) {
        polar_sc_op o{};
        o.code = code;
        o.upos = -1;
        t.seg_ops.push_back(o);
    };
    for (const polar_sc_op &o : ops) {
        if (o.code == POLAR_OP_END) break;
        if ((o.code == POLAR_OP_F || o.code == POLAR_OP_G) && o.n >= tw) {
            if (open) {
                mark(polar_host::POLAR_OP_SEGEND);
                open = false;
            }
            polar_host::TierStep st;
            st.grid = 1;
            st.op = o;
            t.steps.push_back(st);
            continue;
        }
        if (!open) {
            polar_host::TierStep st;
            st.off = (int)t.seg_ops.size();
            t.steps.push_back(st);
            if (st.off > 0) mark(polar_host::POLAR_OP_SEGCONT);
            open = true;
        }
        t.seg_ops.push_back(o);
    }
    if (!open) {   // the schedule ended on a grid record: an empty last segment writes the output
        polar_host::TierStep st;
        st.off = (int)t.seg_ops.size();
        t.steps.push_back(st);
        mark(polar_host::POLAR_OP_SEGCONT);
    }
    mark(POLAR_OP_END);
    t.seg_ops.push_back(t.seg_ops.back());   // spare END: the kernel loads record i + 1 early
    t.tw = tw;
    return t;
}

// Grid tier of a pair plan: the F / G records of at least `tw` output words become grid
// launches over all frame pairs; the records between them are the cases of the segment kernel
// (polar_sc_pairgen.cpp), separated by POLAR_OP_SEGEND. H / H0 of the cut nodes stay in the
// segments, in schedule order.
polar_host::PairTier pair_tier_schedule(const std::vector<polar_sc_op> &ops, int tw)
{
    polar_host::PairTier t;
    bool any = false;
    for (const polar_sc_op &o : ops)
        if ((o.code == POLAR_OP_F || o.code == POLAR_OP_G) && o.n >= tw) any = true;
    if (!any) return t;
    int seg = 0;
    bool open = false;
    for (const polar_sc_op &o : ops) {
        if (o.code == POLAR_OP_END) break;
        if ((o.code == POLAR_OP_F || o.code == POLAR_OP_G) && o.n >= tw) {
            if (open) {
                polar_sc_op e{};
                e.code = polar_host::POLAR_OP_SEGEND;
                e.upos = -1;
                t.seg_ops.push_back(e);
                open = false;
                seg++;
            }
            polar_host::TierStep st;
            st.grid = 1;
            st.op = o;
            t.steps.push_back(st);
            continue;
        }
        if (!open) {
            polar_host::TierStep st;
            st.off = seg;
            t.steps.push_back(st);
            open = true;
        }
        t.seg_ops.push_back(o);
    }
    if (!open) {   // the schedule ended on a grid record: an empty last segment writes the output
        polar_host::TierStep st;
        st.off = seg;
        t.steps.push_back(st);
    }
    polar_sc_op e{};
    e.code = POLAR_OP_END;
    e.upos = -1;
    t.seg_ops.push_back(e);
    t.tw = tw;
    return t;
}

// PAR > 16: decode the PAR-word leaf (Spec_PolarDec_{PAR}, library.h:149-172 ->
// functions.h:766-866) whose LLRs are the node of `words` device words at (level, wpos) as
// device ops: F, the left half, G (G_extended, flagged exact, when EXTENDED; the operands of
// the right half one bit wider), the right half, H; 16-LLR words by FLEAF / GLEAF. fb: the
// frozen bits of the node (bit k = LLR k). wd: operand width above LLR_BITS (CA2 wrap point).
void par_expand(const polar_sc_plan &p, std::vector<polar_sc_op> &out, int level, int wpos, int words, uint64_t fb,
                int wd)
{
    const int h = words / 2;
    const uint32_t wf = (uint32_t)wd << 20, gx = p.cfg.extended ? polar_host::FB_EXACT : 0u;
    if (h == 1) {
        emit(out, POLAR_OP_FLEAF, level, 1, wpos, -1, (uint32_t)(fb & 0xFFFFu) | wf);
    } else {
        emit(out, POLAR_OP_F, level, h, wpos, -1, wf);
        par_expand(p, out, level + 1, wpos, h, fb, wd);
    }
    const uint64_t fbh = fb >> (16 * h);
    if (h == 1) {
        emit(out, POLAR_OP_GLEAF, level, 1, wpos + 1, wpos, (uint32_t)(fbh & 0xFFFFu) | gx | wf);
    } else {
        emit(out, POLAR_OP_G, level, h, wpos + h, wpos, gx | wf);
        par_expand(p, out, level + 1, wpos + h, h, fbh, p.cfg.extended ? wd + 1 : wd);
    }
    emit(out, POLAR_OP_H, level, h, wpos, -1, 0);
}

// R_STATE of PAR group g whose parent node is at device `level`: F / G of the parent into
// the group's words, then its leaf decoder. PAR 16: one FLEAF / GLEAF record. PAR > 16: the
// stage F / G record, then the PR1 decoder of the whole PAR word (OP_PLEAF) or the expanded
// exact leaf.
void leaf_ops(const polar_sc_plan &p, std::vector<polar_sc_op> &out, int level, uint32_t g, bool right, int upos)
{
    const int P = (int)p.p16, wpos = (int)g * P;
    const uint32_t kind = leaf_kind(p, g);
    if (P == 1) {
        emit(out, right ? POLAR_OP_GLEAF : POLAR_OP_FLEAF, level, 1, wpos, right ? upos : -1,
             (uint32_t)(p.fbp[g] & 0xFFFFu) | kind << 16);
        return;
    }
    emit(out, right ? POLAR_OP_G : POLAR_OP_F, level, P, wpos, right ? upos : -1, 0);
    if (kind != POLAR_LEAF_PLAIN) emit(out, polar_host::POLAR_OP_PLEAF, level + 1, P, wpos, -1, kind << 16);
    else par_expand(p, out, level + 1, wpos, P, p.fbp[g], 0);
}

// PAR 4 / 8: the group classes of device word w for the device's word tree
// (polar_sc_interp.h word_node): per group g of the word, bits 7g..7g+3 = class, 7g+4..7g+6 =
// PR1 leaf kind; bit 28 = PRUNING_LEVEL 2
uint32_t word_info(const polar_sc_plan &p, uint32_t w)
{
    uint32_t info = p.cfg.pruning_level == 2 ? 1u << 28 : 0u;
    for (uint32_t j = 0; j < p.ppw; j++) {
        const uint32_t g = w * p.ppw + j;
        info |= (p.type[g] & 15u) << (7 * j);
        info |= (leaf_kind(p, g) & 7u) << (7 * j + 4);
    }
    return info;
}
uint32_t word_fb(const polar_sc_plan &p, uint32_t w)
{
    uint32_t fb = 0;
    for (uint32_t k = 0; k < 16; k++) fb |= (uint32_t)p.mask[16 * w + k] << k;
    return fb;
}
void emit_word(std::vector<polar_sc_op> &out, const polar_sc_plan &p, int code, int level, uint32_t w, int upos)
{
    emit(out, code, level, 1, (int)w, upos, word_fb(p, w));
    out.back().reserved[1] = (int32_t)word_info(p, w);
}

// Decode the children of the node at device `level` covering PAR groups [g0, g0+cnt)
// (cnt >= 2) whose LLR words are in stage buffer `level`. Mirrors the
// F/G/R/H/H0/F_REP/G_R1/G_SPC transitions of my_module::do_action:
//  * left child R0  -> "H0 route" (my_module.h:481-507): no F, G with sa = 0, then H0
//  * left child REP -> F_REP_STATE (my_module.h:1292-1390)
//  * right child R1 -> G_R1_STATE, SPC -> G_SPC_STATE (selected from the node-type stack,
//    my_module.h:614-664, 939-997)
//  * the root's children are never pruned: INIT pushes (RN,RN) (my_module.h:328)
// Device records count 16-LLR words (PAR / 16 per group). Hybrid plans (sc != NULL, PAR 16):
// a node of sc->words words that is not the root becomes one POLAR_OP_SUB record; its own
// schedule, rebased to the subtree root, is kept once per distinct content.
void compile_node(const polar_sc_plan &p, std::vector<polar_sc_op> &out, int level, uint32_t g0, uint32_t cnt,
                  bool is_root, SubCtx *sc)
{
    // (sc->words counts device words; g0 / cnt count PAR groups of p16 words: PAR 64 -> 4, or
    // of 1 / ppw words: PAR 4 -> 1 / 4)
    const uint32_t cnt_words = p.ppw > 1 ? cnt / p.ppw : cnt * p.p16;
    if (sc && !is_root && cnt_words == sc->words) {
        std::vector<polar_sc_op> sub;
        compile_node(p, sub, level, g0, cnt, false, nullptr);
        const int w0 = (int)(p.ppw > 1 ? g0 / p.ppw : g0 * p.p16);
        for (polar_sc_op &o : sub) {
            o.level -= level;
            o.pos -= w0;
            if (o.upos >= 0) o.upos -= w0;
        }
        std::string key((const char *)sub.data(), sub.size() * sizeof(polar_sc_op));
        auto it = sc->ids.find(key);
        int id;
        if (it == sc->ids.end()) {
            id = (int)sc->lists.size();
            sc->ids.emplace(key, id);
            sc->lists.push_back(std::move(sub));
        } else {
            id = it->second;
        }
        sc->calls++;
        emit(out, polar_host::POLAR_OP_SUB, level, (int)cnt_words, w0, -1, (uint32_t)id);
        return;
    }
    const uint32_t h = cnt / 2;
    if (p.ppw > 1) {
        // PAR 4 / 8: nodes of two or more device words as usual; a child of one word is an
        // FLEAF / GLEAF record whose device side decodes the whole word (its PAR words, their
        // pruning and leaves: polar_sc_interp.h word_node)
        const uint32_t Q = p.ppw;
        const int hw = (int)(h / Q), w0 = (int)(g0 / Q), w1 = (int)((g0 + h) / Q);
        const bool prune = p.cfg.pruning_level == 2;
        const uint32_t tl = (is_root || !prune) ? NODE_RN : node_class(p, g0, h);
        const uint32_t tr = (is_root || !prune) ? NODE_RN : node_class(p, g0 + h, h);
        bool left_zero = false;
        if (tl == NODE_R0) {
            left_zero = true;
        } else if (tl == NODE_REP) {
            emit(out, POLAR_OP_REP, level, hw, w0, -1, 0);
        } else if (h == Q) {
            emit_word(out, p, POLAR_OP_FLEAF, level, (uint32_t)w0, -1);
        } else {
            emit(out, POLAR_OP_F, level, hw, w0, -1, 0);
            compile_node(p, out, level + 1, g0, h, false, sc);
        }
        const int upos = left_zero ? -1 : w0;
        if (tr == NODE_R1) {
            emit(out, POLAR_OP_R1, level, hw, w1, upos, 0);
        } else if (tr == NODE_SPC) {
            emit(out, POLAR_OP_SPC, level, hw, w1, upos, 0);
        } else if (h == Q) {
            emit_word(out, p, POLAR_OP_GLEAF, level, (uint32_t)w1, upos);
        } else {
            emit(out, POLAR_OP_G, level, hw, w1, upos, 0);
            compile_node(p, out, level + 1, g0 + h, h, false, sc);
        }
        emit(out, left_zero ? POLAR_OP_H0 : POLAR_OP_H, level, hw, w0, -1, 0);
        return;
    }
    const int P = (int)p.p16, hw = (int)h * P, w0 = (int)g0 * P, w1 = (int)(g0 + h) * P;
    // node pruning only at PRUNING_LEVEL 2 (my_module.h:478-531, 623-652, 815-868, 965-993);
    // REP2 / SPC2 classes fall through to the plain F / G transitions there
    const bool prune = p.cfg.pruning_level == 2;
    const uint32_t tl = (is_root || !prune) ? NODE_RN : node_class(p, g0, h);
    const uint32_t tr = (is_root || !prune) ? NODE_RN : node_class(p, g0 + h, h);
    bool left_zero = false;
    if (tl == NODE_R0) {
        left_zero = true;
    } else if (tl == NODE_REP) {
        emit(out, POLAR_OP_REP, level, hw, w0, -1, 0);
    } else if (h == 1) {
        leaf_ops(p, out, level, g0, false, -1);
    } else {
        emit(out, POLAR_OP_F, level, hw, w0, -1, 0);
        compile_node(p, out, level + 1, g0, h, false, sc);
    }
    const int upos = left_zero ? -1 : w0;
    if (tr == NODE_R1) {
        emit(out, POLAR_OP_R1, level, hw, w1, upos, 0);
    } else if (tr == NODE_SPC) {
        emit(out, POLAR_OP_SPC, level, hw, w1, upos, 0);
    } else if (h == 1) {
        leaf_ops(p, out, level, g0 + h, true, upos);
    } else {
        emit(out, POLAR_OP_G, level, hw, w1, upos, 0);
        compile_node(p, out, level + 1, g0 + h, h, false, sc);
    }
    emit(out, left_zero ? POLAR_OP_H0 : POLAR_OP_H, level, hw, w0, -1, 0);
}

// The reference's swept configurations: PRUNING_LEVEL 0/1/2 with any ELAG_R1/REP/SPC/REP2/
// SPC2/H0 switches (script/script_tests.sh:103-122), LLR_BITS 5..9 (QUANT 6..9,
// script/parser.sh:12, parser_comp.sh:12; 9-bit LLRs beyond the int8 range need the int16
// channel of polar_sc_decode_i16), SIGMAG or CA2 (parser.sh:15,43), EXTENDED 0/1
// (config.h:14) and PAR 4 / 8 / 16 / 32 / 64 (script_tests.sh:11,124 runs 16 and 64,
// script_RTL_sim.sh:97-330 PAR 4..64). ELAG_RARE = 1 does not compile in the reference
// (my_module.h:255 vs :1511).
bool config_supported(const polar_sc_config &c)
{
    auto sw = [](int32_t v) { return v == 0 || v == 1; };
    return c.llr_bits >= 5 && c.llr_bits <= 9 &&
           (c.par == 4 || c.par == 8 || c.par == 16 || c.par == 32 || c.par == 64) && sw(c.sigmag) &&
           sw(c.extended) && c.pruning_level >= 0 && c.pruning_level <= 2 && sw(c.elag_r1) && sw(c.elag_rep) &&
           sw(c.elag_spc) && sw(c.elag_rep2) && sw(c.elag_spc2) && c.elag_rare == 0 && sw(c.elag_h0) &&
           sw(c.strict_llr);
}

// the shipped datapath (SIGMAG, PAR 16, EXTENDED, int8-range LLRs): the only one the per-mask
// and generated-subtree kernels implement; every other format runs the schedule interpreter
// compiled by hipRTC with its POLAR_* switches
// the datapath of the generated kernels (per-mask, hybrid, pair): SIGMAG, PAR 16, LLR_BITS <= 8,
// EXTENDED 0 or 1 (POLAR_EXT of the generated source)
bool default_format(const polar_sc_config &c)
{
    return c.sigmag == 1 && c.par == 16 && c.llr_bits <= 8;
}
// the datapath the hipcc-built schedule interpreter is compiled for; every other format's
// interpreter (per-op monitor, fallbacks) is compiled by hipRTC with its POLAR_* switches
bool builtin_format(const polar_sc_config &c)
{
    return c.sigmag == 1 && c.par == 16 && c.extended == 1 && c.llr_bits == 6;
}

bool tuning_valid(const polar_sc_tuning &t)
{
    auto pow2 = [](int v) { return v > 0 && (v & (v - 1)) == 0; };
    return (t.kernel >= 0 && t.kernel <= 3) && (t.waves_per_group == 0 || (pow2(t.waves_per_group) && t.waves_per_group <= 16)) &&
           (t.sub_words == 0 || (pow2(t.sub_words) && t.sub_words >= 2 && t.sub_words <= 512)) &&
           t.tier_words >= -1 && (t.tier_words <= 0 || pow2(t.tier_words)) &&
           (t.lds_slots == 0 || t.lds_slots == 256 || t.lds_slots == 512 || t.lds_slots == 1024) &&
           (t.hybrid_waves == 0 || t.hybrid_waves == 4 || t.hybrid_waves == 8) && t.chain_max >= 0 &&
           t.chain_max <= 4 && t.sub_inline >= 0 && t.sub_inline <= 2 && t.layout >= 0 && t.layout <= 2 &&
           t.sub_root >= 0 && t.sub_root <= 2;
}

int hip_err(hipError_t e) { return e == hipSuccess ? 0 : -EIO; }

// device state for the current device: schedule upload (+ scratch for `batch` frames)
// mode DEV_DECODE: the plan's decode kernel; DEV_TRACE: also the interpreter schedule of a
// per-mask plan (the per-op monitor runs the schedule interpreter for those); DEV_I16: only
// what the int16-channel interpreter needs (schedule, scratch), no per-mask / hybrid module
// held: if non-null, receives the plan lock (still held on success) so that the caller can
// launch with the scratch pointer it was given before another thread may reallocate it
enum DevMode { DEV_DECODE, DEV_TRACE, DEV_I16 };
// HIP failure inside the library: -EIO, and the HIP error on stderr when POLAR_SC_VERBOSE is set
int hip_fail(const char *what, hipError_t e)
{
    static const bool verbose = std::getenv("POLAR_SC_VERBOSE") != nullptr;
    if (verbose) std::fprintf(stderr, "polar_sc: %s: %s\n", what, hipGetErrorString(e));
    return -EIO;
}

int ensure_device(const polar_sc_plan *p, size_t batch, DevState **out, DevMode mode = DEV_DECODE,
                  std::unique_lock<std::mutex> *held = nullptr)
{
    const bool interp = mode != DEV_DECODE;
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev); e != hipSuccess) return hip_fail("hipGetDevice", e);
    std::unique_lock<std::mutex> lk(p->mu);
    DevState &st = p->dev[dev];
    if (st.simds == 0) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
        st.simds = 4 * cus;
    }
    if ((p->jit || p->hybrid || p->pair) && mode != DEV_I16) {
        // pair plans are traced on the schedule interpreter (trace_common): no pair kernel is
        // built or loaded for a trace
        if (!(p->pair && interp)) {
            int rc = polar_host::jit_load(*p, st);
            if (rc) return rc;
        }
        if (p->jit && !interp) {
            *out = &st;
            return 0;
        }
        if ((p->jit || p->pair) && interp && !builtin_format(p->cfg)) {   // traced plan: hipRTC interpreter of its format
            const int rc = polar_host::jit_load_interp(*p, st);
            if (rc) return rc;
        }
    }
    if (!st.ops) {
        // device copy (+ a spare END: the interpreter loads record i+1 while running i)
        std::vector<polar_sc_op> dops = p->dev_ops.empty() ? p->ops : p->dev_ops;
        dops.push_back(dops.back());
        size_t bytes = dops.size() * sizeof(polar_sc_op);
        if (hipMalloc(&st.ops, bytes) != hipSuccess) return -ENOMEM;
        if (hipError_t e = hipMemcpy(st.ops, dops.data(), bytes, hipMemcpyHostToDevice); e != hipSuccess)
            return hip_fail("schedule upload", e);
    }
    if (mode == DEV_I16 && !p->ops16.empty() && !st.ops16) {
        std::vector<polar_sc_op> dops = p->ops16;
        dops.push_back(dops.back());
        const size_t bytes = dops.size() * sizeof(polar_sc_op);
        if (hipMalloc(&st.ops16, bytes) != hipSuccess) return -ENOMEM;
        if (hipMemcpy(st.ops16, dops.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return -EIO;
    }
    for (size_t t = 0; t < p->tiers.size() && t < 2; t++) {
        if (st.seg_ops[t]) continue;
        const size_t bytes = p->tiers[t].seg_ops.size() * sizeof(polar_sc_op);
        if (hipMalloc(&st.seg_ops[t], bytes) != hipSuccess) return -ENOMEM;
        if (hipMemcpy(st.seg_ops[t], p->tiers[t].seg_ops.data(), bytes, hipMemcpyHostToDevice) != hipSuccess)
            return -EIO;
    }
    if (p->gmem || p->pair) {
        size_t waves = (batch + 7) / 8;
        size_t need = p->gmem ? waves * (size_t)p->hbm_group_dwords * 4u : 0u;
        if (p->pair) need = std::max(need, (p->solo ? batch : (batch + 1) / 2) * (size_t)p->pair_dwords * 4u);
        if (need > st.scratch_bytes) {
            if (st.scratch) {
                if (hipDeviceSynchronize() != hipSuccess) return -EIO;
                (void)hipFree(st.scratch);
                st.scratch = nullptr;
                st.scratch_bytes = 0;
            }
            if (hipMalloc(&st.scratch, need) != hipSuccess) return -ENOMEM;
            st.scratch_bytes = need;
        }
    }
    *out = &st;
    if (held) *held = std::move(lk);
    return 0;
}

// Interpreter launches: waves per 8-frame group. Large batches keep one wave per group;
// when the groups cannot fill the GPU (about 2 waves per SIMD), a group gets up to 16 waves
// that split its wide ops (polar_sc_kernels.hip). polar_sc_tuning.waves_per_group fixes it.
int waves_per_group(const polar_sc_plan *p, size_t batch, int simds)
{
    if (const int w = p->tune.waves_per_group) return p->hybrid && w > p->hybrid_waves ? p->hybrid_waves : w;
    const int wmax = p->hybrid ? p->hybrid_waves : 16;
    const size_t groups = (batch + 7) / 8;
    const size_t target = 2u * (size_t)(simds > 0 ? simds : 1024);
    int w = 1;
    while (w < wmax && groups * (size_t)w < target) w *= 2;
    return w;
}

// SIMDs of the current device (4 per CU), cached per device ordinal
int current_simds()
{
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 1024;
    if (dev < 64 && cache[dev].load()) return cache[dev].load();
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (dev < 64) cache[dev].store(4 * cus);
    return 4 * cus;
}

// the plan that decodes a batch of `batch` frames on a device of `simds` SIMDs: the solo
// alternate of an automatic-layout pair plan while the batch is at most SOLO_FRAMES_PER_SIMD
// frames per SIMD (one frame per wave then still fits one dispatch round), else the plan
const polar_sc_plan *layout_for(const polar_sc_plan *p, size_t batch, int simds)
{
    if (p->alt && batch <= (size_t)polar_host::SOLO_FRAMES_PER_SIMD * (size_t)simds) return p->alt;
    return p;
}

int decode_common(const polar_sc_plan *p, const int8_t *llr, uint16_t *out, size_t batch,
                  int out_stride, void *stream)
{
    if (!p || (batch > 0 && (!llr || !out))) return -EINVAL;
    if (batch == 0) return 0;
    if (batch > (size_t)0x7FFFFFF8) return -EINVAL;
    if (p->alt) p = layout_for(p, batch, current_simds());
    DevState *st = nullptr;
    // HBM-scratch plans launch under the plan lock: a concurrent decode of a larger batch on
    // another thread reallocates the scratch only after this launch has been queued (and
    // synchronises the device before freeing it)
    std::unique_lock<std::mutex> held;
    int rc = ensure_device(p, batch, &st, DEV_DECODE, (p->gmem || p->pair) ? &held : nullptr);
    if (rc) return rc;
    if (p->jit) return polar_host::jit_launch(*p, *st, llr, out, (long)batch, out_stride, stream);
    if (p->slot16()) {   // the kernel reads the int16 channel: widen the int8 frames first
        const size_t n = batch * (size_t)p->N, need = 2 * n;
        if (st->wide_bytes < need) {
            if (st->wide) {
                if (hipDeviceSynchronize() != hipSuccess) return -EIO;
                (void)hipFree(st->wide);
                st->wide = nullptr;
                st->wide_bytes = 0;
            }
            if (hipMalloc(&st->wide, need) != hipSuccess) return -ENOMEM;
            st->wide_bytes = need;
        }
        if (polar_sc_launch_widen(llr, (int16_t *)st->wide, n, stream)) return -EIO;
        return polar_host::jit_launch_pair(*p, *st, (const int8_t *)st->wide, out, (long)batch, out_stride, stream);
    }
    if (p->pair) return polar_host::jit_launch_pair(*p, *st, llr, out, (long)batch, out_stride, stream);
    const int wpg = waves_per_group(p, batch, st->simds);
    if (p->hybrid) return polar_host::jit_launch_hybrid(*p, *st, llr, out, (long)batch, out_stride, wpg, stream);
    rc = polar_sc_launch_decode(p->gmem, llr, out, st->ops, (uint32_t *)st->scratch, (int)p->N, (long)batch,
                                out_stride, wpg, 1, p->hbm_group_dwords, p->lds_group_dwords, p->lds0, stream,
                                nullptr);
    return rc ? -EIO : 0;
}

// The per-op monitor (the analogue of the reference's sc_monitor latency report,
// src/rtl_simu_testbench/sc_monitor/sc_monitor.h:50-140, fed by my_module's Fct_ID / N_value
// ports, my_module.h:21-30): one decode with the traced interpreter (hybrid plans: the
// traced hybrid kernel), per device op the shader-clock cycles of frame group 0's lead wave.
int trace_common(const polar_sc_plan *p, const int8_t *llr, uint16_t *out, size_t batch, int out_stride,
                 polar_sc_trace_rec *recs, uint32_t cap, uint32_t *count, double *clock_ghz, uint64_t *total)
{
    if (!p || !count || batch == 0 || !llr || !out) return -EINVAL;
    if (batch > (size_t)0x7FFFFFF8) return -EINVAL;
    const std::vector<polar_sc_op> &dops = (p->hybrid || p->gmem) && !p->dev_ops.empty() ? p->dev_ops : p->ops;
    *count = (uint32_t)dops.size();
    if (!recs) return 0;
    DevState *st = nullptr;
    std::unique_lock<std::mutex> held;
    int rc = ensure_device(p, batch, &st, DEV_TRACE, &held);
    if (rc) return rc;
    const size_t slots = dops.size() + 3;
    unsigned long long *dtrace = nullptr;
    if (hipMalloc(&dtrace, slots * sizeof(unsigned long long)) != hipSuccess) return -ENOMEM;
    std::vector<unsigned long long> h(slots, 0);
    rc = hipMemset(dtrace, 0, slots * sizeof(unsigned long long)) == hipSuccess ? 0 : -EIO;
    int wpg = waves_per_group(p, batch, st->simds);
    if (!rc) {
        if (p->hybrid) {
            rc = polar_host::jit_launch_hybrid(*p, *st, llr, out, (long)batch, out_stride, wpg, nullptr, dtrace);
        } else if ((p->jit || p->pair) && !builtin_format(p->cfg)) {
            // per-mask / pair plan of another format: the hipRTC interpreter of its POLAR_* switches
            if (wpg > polar_host::HYBRID_MAX_WAVES) wpg = polar_host::HYBRID_MAX_WAVES;
            rc = polar_host::launch_interp_fn(st->ifn_trace, *p, *st, llr, out, (long)batch, out_stride, wpg, nullptr,
                                              dtrace);
        } else
            rc = polar_sc_launch_decode(p->gmem, llr, out, st->ops, (uint32_t *)st->scratch, (int)p->N,
                                        (long)batch, out_stride, wpg, 1, p->hbm_group_dwords, p->lds_group_dwords,
                                        p->lds0, nullptr, dtrace) ? -EIO : 0;
    }
    if (!rc && hipDeviceSynchronize() != hipSuccess) rc = -EIO;
    if (!rc && hipMemcpy(h.data(), dtrace, slots * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
        rc = -EIO;
    (void)hipFree(dtrace);
    if (rc) return rc;
    const size_t n = dops.size();   // the last record is END: its slot holds the finish time
    const uint64_t t0 = h[2], t1 = h[2 + n - 1];
    for (size_t i = 0; i < n && i < cap; i++) {
        polar_sc_trace_rec r{};
        r.code = dops[i].code;
        r.level = dops[i].level;
        r.n = dops[i].n;
        r.pos = dops[i].pos;
        r.cycles = i + 1 < n ? h[2 + i + 1] - h[2 + i] : 0;
        recs[i] = r;
    }
    if (total) *total = t1 - t0;
    if (clock_ghz) {
        const double wall_ns = (double)(h[1] - h[0]) * 10.0;   // s_memrealtime: 100 MHz
        *clock_ghz = wall_ns > 0 ? (double)(t1 - t0) / wall_ns : 0.0;
    }
    return 0;
}

bool read_text(const char *path, std::string &s)
{
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::stringstream ss;
    ss << f.rdbuf();
    s = ss.str();
    return true;
}

}  // namespace

extern "C" {

int polar_sc_abi_version(void) { return POLAR_SC_ABI_VERSION; }

const char *polar_sc_strerror(int err)
{
    switch (err) {
    case 0: return "success";
    case -EINVAL: return "invalid argument";
    case -ENOMEM: return "out of memory";
    case -ENOTSUP: return "configuration not supported (PAR other than 4/8/16/32/64, LLR_BITS outside 5..9, ELAG_RARE, "
                          "or a switch outside 0/1; see polar_sc_config in include/polar_sc.h)";
    case -ENOENT: return "file not found";
    case -EIO: return "HIP runtime error";
    default: return "unknown error";
    }
}

int polar_sc_default_config(polar_sc_config *cfg)
{
    if (!cfg) return -EINVAL;
    cfg->llr_bits = 6;
    cfg->par = 16;
    cfg->sigmag = 1;
    cfg->extended = 1;
    cfg->pruning_level = 2;
    cfg->elag_r1 = 1;
    cfg->elag_rep = 1;
    cfg->elag_spc = 1;
    cfg->elag_rep2 = 0;
    cfg->elag_spc2 = 0;
    cfg->elag_rare = 0;
    cfg->elag_h0 = 1;
    cfg->strict_llr = 0;
    return 0;
}

int polar_sc_plan_create(polar_sc_plan **out, uint32_t N, const uint8_t *info_mask,
                         const polar_sc_config *cfg)
{
    return polar_sc_plan_create_tuned(out, N, info_mask, cfg, nullptr);
}

int polar_sc_plan_create_tuned(polar_sc_plan **out, uint32_t N, const uint8_t *info_mask,
                               const polar_sc_config *cfg, const polar_sc_tuning *tun)
{
    if (!out || !info_mask) return -EINVAL;
    *out = nullptr;
    if (N < 32 || N > (1u << 20) || (N & (N - 1)) != 0) return -EINVAL;
    polar_sc_config c;
    if (cfg) c = *cfg; else polar_sc_default_config(&c);
    if (!config_supported(c)) return -ENOTSUP;
    polar_sc_tuning t{};
    if (tun) t = *tun;
    if (!tuning_valid(t)) return -EINVAL;

    if (N < 2u * (uint32_t)c.par) return -EINVAL;   // INIT needs N_DIV >= 2 (my_module.h:294-309)

    polar_sc_plan *p = new (std::nothrow) polar_sc_plan();
    if (!p) return -ENOMEM;
    p->N = N;
    p->G = N / 16;
    p->GP = N / (uint32_t)c.par;
    p->p16 = c.par >= 16 ? (uint32_t)c.par / 16 : 1u;
    p->ppw = c.par < 16 ? 16u / (uint32_t)c.par : 1u;
    p->cfg = c;
    p->tune = t;
    p->mask.resize(N);
    p->fbp.resize(p->GP);
    p->type.resize(p->GP);
    for (uint32_t i = 0; i < N; i++) {
        p->mask[i] = info_mask[i] ? 1 : 0;
        p->K += p->mask[i];
    }
    polar_sc_plan_stats &s = p->stats;
    for (uint32_t g = 0; g < p->GP; g++) {
        uint64_t t = 0;
        for (uint32_t k = 0; k < (uint32_t)c.par; k++) t |= (uint64_t)p->mask[g * (uint32_t)c.par + k] << k;
        p->fbp[g] = t;
        p->type[g] = (uint8_t)classify_group(t, (uint32_t)c.par, c);
        switch (p->type[g]) {
        case NODE_R0: s.n_r0++; break;
        case NODE_R1: s.n_r1++; break;
        case NODE_REP: s.n_rep++; break;
        case NODE_SPC: s.n_spc++; break;
        default: s.n_rn++; break;   // RN, REP2, SPC2
        }
    }
    compile_node(*p, p->ops, 0, 0, p->GP, true, nullptr);
    emit(p->ops, POLAR_OP_END, 0, 0, 0, -1, 0);

    s.N = N;
    s.K = p->K;
    s.groups = p->GP;
    s.n_ops = (uint32_t)p->ops.size();
    for (const polar_sc_op &o : p->ops) {
        s.op_count[o.code & 15]++;
        if (o.code <= POLAR_OP_SPC) s.word_ops += (uint64_t)o.n;
    }
    const uint32_t nslot = p->G - 1, nbd = (p->G + 15) / 16;
    const uint64_t all_bytes = (uint64_t)(nslot + nbd) * 256u;   // one 8-frame group, all in LDS
    p->gmem = all_bytes > LDS_WAVE_LIMIT ? 1 : 0;
    if (p->gmem) {
        // upper levels + bit dwords in HBM scratch; the levels of nodes <= 128 words in LDS,
        // plus an LDS window for the partial sums of the current 128-word subtree
        // the LDS region W: 256 slots, 512 from N = 32768 and 1024 from N = 131072 when the
        // LDS slots hold 8-bit pairs (PAR 16, LLR_BITS <= 8: 78 KB per group = two groups per
        // CU at W = 512, 150 KB = one at 1024); polar_sc_tuning.lds_slots overrides
        const bool lds8 = c.par <= 16 && c.llr_bits <= 8;
        int W = LDS_LOW_SLOTS;
        if (lds8 && p->G >= 8192) W = 1024;
        else if (lds8 && p->G >= 2048) W = 512;
        if (const int w = t.lds_slots) {
            if ((w == 256 || (lds8 && (w == 512 || w == 1024))) && (uint32_t)w <= p->G / 2) W = w;
        }
        p->lds_slots = W;
        p->lds0 = (int)p->G - W;
        // 8-bit-pair slots (16-bit values for 9-bit LLRs) + bit dwords
        p->hbm_group_dwords = p->lds0 * (c.llr_bits > 8 ? 64 : 32) + (int)nbd * 64;
        // + the partial-sum window + the SPC exchange area (polar_sc_interp.h SPC_XWAVES)
        const int es = lds8 ? 2 : 4;   // bytes per LDS slot element (polar_sc_interp.h lslot_t)
        p->lds_group_dwords = ((W - 1) * 64 * es) / 4 + (W / 16 + 3 * 8) * 64;
    } else {
        p->lds0 = 0;
        p->hbm_group_dwords = 0;
        p->lds_group_dwords = (int)(nslot + nbd) * 64;
    }
    while ((1u << p->lg) < p->G) p->lg++;
    // per-mask register kernel for N <= 1024; above, the hybrid kernel (interpreter + generated
    // subtree decoders of sub_words words, default 64 / 128). polar_sc_tuning.kernel = 1
    // selects the plain schedule interpreter for every N.
    const bool jit_on = t.kernel != 1;
    // PRUNING_LEVEL 1 leaf decoders: the 16-LLR REP / SPC / REP2 / SPC2 leaves run in the
    // generated kernels too (leaf_gen); the PAR-word decoders of PAR > 16 (OP_PLEAF) and the
    // CA2 R1 leaf on the interpreter only
    bool kinds = false;
    for (const polar_sc_op &o : p->ops)
        if (((o.code == POLAR_OP_FLEAF || o.code == POLAR_OP_GLEAF) && ((o.fb >> 16) & 7u) > POLAR_LEAF_SPC2) ||
            o.code == polar_host::POLAR_OP_PLEAF)
            kinds = true;
    const bool dflt = default_format(c);
    // pair plans also take PAR 32 / 64 (the PAR word = one register of two / four device words;
    // the host expands its leaf into F / G / 16-LLR leaf records, par_expand: G_extended when
    // EXTENDED, the saturating G and POLAR_EXT 0 leaves when not)
    // and 9-bit LLRs (16-bit stage slots, the int16 channel: polar_sc_pair.h SLOT16)
    // and CA2 (polar_sc_pair.h POLAR_CA2: the split code on magnitude + sign, MIN absorbing on
    // the leftmost path; 9-bit LLRs at PAR 64, whose REP accumulator bound 2^15 - 1 fills a
    // 16-bit half, accumulate with the saturating packed add, polar_sc_device.h rep_acc)
    // and PAR 4 / 8 SIGMAG (the PAR words = lane groups of a device word: every one-word leaf
    // record decodes its whole word tree with the frozen bits and group classes as template
    // constants, polar_sc_device.h word_gen; REP over the groups, polar_sc_pair.h rep_groups_*)
    // (and PRUNING_LEVEL 1 everywhere: the 16-LLR leaf records' REP / SPC / REP2 / SPC2 / R1
    // decoders, in CA2 on the two's complement word (leaf_gen_ca2), and at PAR 32 / 64 the
    // decoders of the whole PAR word, OP_PLEAF records after its F / G: polar_sc_pair.h
    // pleaf_pair, the interpreter's op_pleaf on the pair layout)
    const bool pair_par = c.par == 16 || c.par == 32 || c.par == 64;
    // (CA2 at PAR 4 / 8 too: the word trees on two's complement values, every PRUNING_LEVEL --
    // their PR1 leaves, the CA2 R1 decoder included, are the word tree's; ppw > 1 leaf records
    // carry no kind bits)
    const bool par48 = c.par == 4 || c.par == 8;
    const bool pair_fmt = dflt || ((pair_par || par48) && c.sigmag == 1 && c.llr_bits <= 9) ||
                          ((pair_par || par48) && c.sigmag == 0 && c.llr_bits <= 9);
    p->jit = (polar_host::jit_supported(N) && jit_on && !kinds && dflt) ? 1 : 0;
    // generated subtrees of 64 words (1024 LLRs), 128 (2048 LLRs) from N = 32768: the 2048-LLR
    // level's F / G / H then run inside the straight-line code instead of as interpreter ops
    // (one box, same-box A/B: C5 4.68 -> 3.76 ms, C5 64-frame share 4.18 -> 3.13, C3 1.54 ->
    // 1.48; 248 VGPRs, no spills, at most 2 waves per SIMD -- below N = 32768 the smaller
    // subtrees keep 3)
    int sub_words = p->G >= 2048 ? 128 : 64;
    if (t.sub_words) sub_words = t.sub_words;
    const bool sub_ok = sub_words >= 2 && sub_words <= 128 && (sub_words & (sub_words - 1)) == 0;
    std::vector<polar_sc_op> dev_sched;
    // pair plans (polar_sc_pair.h): one frame pair per wave, generated subtrees of up to 256
    // words -- the default for N >= 2048 (same-box A/B against the hybrid kernel of 8-frame
    // groups, tools/pair_ab.py: C3 1.64 -> 1.16 ms, C5 4.18 -> 1.78, C5 at 64 frames 3.57 ->
    // 1.55, N = 16384 x 4096 frames 0.39 -> 0.24, N = 4096 x 16384 0.36 -> 0.23);
    // polar_sc_tuning.kernel = 2 keeps the hybrid kernel
    const bool want_pair = !p->jit && jit_on && pair_fmt && p->G >= 64 && (t.kernel == 3 || t.kernel == 0);
    // an explicit kernel / subtree size that cannot be honoured is an error, not a silent
    // fallback to another kernel (A/B measurements force them)
    if ((t.kernel == 3 && !want_pair) ||
        (t.kernel == 2 && !p->jit && !kinds && dflt && t.sub_words && (!sub_ok || (uint32_t)sub_words >= p->G))) {
        const int rc = t.kernel == 3 ? -ENOTSUP : -EINVAL;
        delete p;
        return rc;
    }
    // solo layout (one frame per wave, 8 words per register): PAR 16 SIGMAG (8-bit slot rows,
    // or 16-bit ones for 9-bit LLRs; the half ops of 8-word nodes have no CA2 form); a forced
    // solo layout the plan cannot take is an error
    // (and N >= 2048: the solo subtrees need >= 64 words under a root of >= 2 of them; at
    // N = 1024 a 32-word solo subtree decoded wrong on the GPU with the int8 entry of a 9-bit
    // plan, so N = 1024 plans are pair-only)
    const bool solo_ok = c.par == 16 && c.sigmag == 1 && c.llr_bits <= 9 && p->G >= 128;
    if ((t.layout != 0 && !want_pair) || (t.layout == 2 && !solo_ok)) {
        delete p;
        return -ENOTSUP;
    }
    const bool solo = want_pair && t.layout == 2;
    bool use_pair = false;
    if (want_pair) {
        const int wpr = solo ? 8 : 4;
        // default subtree size: 256 words (pair), 512 (solo: half the registers per word), both
        // at most half the frame; one default for a forced and the automatic solo plan
        int S = std::min<int>(solo ? polar_host::SOLO_SUB_WORDS_MAX : polar_host::PAIR_SUB_WORDS, (int)p->G / 2);
        if (t.sub_words) {
            // the halves of every upper node are whole 8-row slot groups: >= 32 words (pair),
            // >= 64 (solo); at most 256 (pair) / 512 (solo) words of register code
            if (t.sub_words < 8 * wpr || (uint32_t)t.sub_words > p->G / 2 ||
                t.sub_words > (solo ? polar_host::SOLO_SUB_WORDS_MAX : polar_host::PAIR_SUB_WORDS)) {
                delete p;
                return -EINVAL;
            }
            S = t.sub_words;
        }
        p->solo = solo ? 1 : 0;
        SubCtx sc;
        sc.words = (uint32_t)S;
        compile_node(*p, p->pair_ops, 0, 0, p->GP, true, &sc);
        emit(p->pair_ops, POLAR_OP_END, 0, 0, 0, -1, 0);
        // Subtree roots without a slot level: the F / G record that writes a subtree's root
        // (always the record right before its SUB, compile_node) is folded into the SUB, whose
        // generated decoder then reads the root as F / G of the parent's slot rows
        // (polar_sc_pairgen.cpp CHF / CHG). The subtree-root level (S words) then needs no
        // slot: one level less in the slot rows, and the LDS it held takes the next level up
        // (C3: the 512-word level on chip, 6 N instead of 8 N of HBM traffic per frame). Not
        // for subtrees that are children of the root (G = 2 S: their parent is the channel).
        // Automatic: the pair layout with G >= 16 S only. The folded F / G runs on the lead
        // wave alone, where the upper-level record split it over the W waves of a block, and
        // each root row is computed twice (for the subtree's F and its G): it pays only where
        // the level it takes off HBM is a deep one of a long code. Same box
        // (profiles/r05_ab/sub_root_ab3_*.jsonl, n16384_sub_root_ab.jsonl): C3 (G = 16 S, W = 1)
        // 0.844 / 0.824 ms vs 0.844 / 0.848 and 1.97 vs 2.7 GB per decode; N = 16384 (G = 4 S)
        // 0.216 / 0.206 / 0.204 vs 0.201 / 0.194 / 0.194 ms (QUANT 8: 0.188 vs 0.168); the solo
        // C5 (W = 4 / 8) 1.414 vs 1.280 ms, its 64-frame share 1.082 vs 1.034.
        const bool fuse = (t.sub_root == 2 || (t.sub_root == 0 && !solo && (int)p->G >= 16 * S)) && (int)p->G / 2 > S;
        if (fuse) {
            std::vector<polar_sc_op> fused;
            const std::vector<polar_sc_op> &ops = p->pair_ops;
            for (size_t i = 0; i < ops.size(); i++) {
                const polar_sc_op &o = ops[i];
                if (i + 1 < ops.size() && (o.code == POLAR_OP_F || o.code == POLAR_OP_G) && o.n == S &&
                    ops[i + 1].code == polar_host::POLAR_OP_SUB && ops[i + 1].level == o.level + 1 &&
                    ops[i + 1].pos == o.pos) {
                    polar_sc_op sub = ops[i + 1];
                    sub.reserved[1] = o.code == POLAR_OP_F ? 1 : 2;   // the folded producer
                    sub.upos = o.code == POLAR_OP_G ? o.upos : -1;
                    fused.push_back(sub);
                    i++;
                } else {
                    fused.push_back(o);
                }
            }
            p->pair_ops.swap(fused);
        }
        p->pair_fused = fuse ? 1 : 0;
        p->pair = 1;
        p->sub_words = S;
        p->subs = std::move(sc.lists);
        s.sub_words = (uint32_t)S;
        s.n_sub_kinds = (uint32_t)p->subs.size();
        s.n_sub_calls = sc.calls;
        p->pair_slot_rows = ((int)p->G - (p->pair_fused ? 2 * S : S)) / p->wpr();
        p->pair_dwords = p->pair_slot_rows * (p->slot_row_bytes() / 4) + std::max<int>(1, (int)p->G / (16 * p->wpr())) * 64;
        if (t.tier_words > 0) {
            if (t.tier_words <= S) {
                delete p;
                return -EINVAL;
            }
            p->pair_tier = pair_tier_schedule(p->pair_ops, t.tier_words);
        }
        // generate the kernel source now: a schedule the generator does not support falls back
        // to the hybrid kernel here (or fails plan creation when the pair kernel was forced)
        // instead of failing the first decode
        try {
            (void)polar_host::pair_source(*p);
            use_pair = true;
        } catch (const std::exception &e) {
            p->jit_log = e.what();
            if (t.kernel == 3) {
                delete p;
                return -ENOTSUP;
            }
            p->pair = 0;
            p->solo = 0;
            p->pair_fused = 0;
            p->sub_words = 0;
            p->subs.clear();
            p->pair_ops.clear();
            p->pair_tier = polar_host::PairTier{};
            s.sub_words = s.n_sub_kinds = s.n_sub_calls = 0;
        }
    }
    if (use_pair) {
        // the schedule interpreter's copy (per-op monitor, int16 channel)
        dev_sched = p->ops;
    } else if (!p->jit && jit_on && !kinds && dflt && sub_ok && (uint32_t)sub_words < p->G) {
        SubCtx sc;
        sc.words = (uint32_t)sub_words;
        compile_node(*p, dev_sched, 0, 0, p->GP, true, &sc);
        emit(dev_sched, POLAR_OP_END, 0, 0, 0, -1, 0);
        p->hybrid = 1;
        p->hybrid_waves = t.hybrid_waves ? t.hybrid_waves : polar_host::HYBRID_MAX_WAVES;
        p->sub_words = sub_words;
        p->subs = std::move(sc.lists);
        s.sub_words = (uint32_t)sub_words;
        s.n_sub_kinds = (uint32_t)p->subs.size();
        s.n_sub_calls = sc.calls;
    } else {
        dev_sched = p->ops;
        if (!p->jit && !builtin_format(c)) {
            // the hipcc-built interpreter is the shipped datapath; other formats run the same
            // interpreter compiled by hipRTC with their POLAR_* switches (a hybrid kernel
            // without subtrees)
            p->hybrid = 1;
            p->hybrid_waves = polar_host::HYBRID_MAX_WAVES;
        }
    }
    if (p->gmem) window_schedule(*p, dev_sched, p->dev_ops);
    else if (p->hybrid) p->dev_ops = dev_sched;
    // int16 channel (polar_sc_decode_i16): the interpreter has no generated subtrees, so it
    // runs the plan's schedule without OP_SUB records
    if (!p->subs.empty()) {
        if (p->gmem) window_schedule(*p, p->ops, p->ops16);
        else p->ops16 = p->ops;
    }
    // grid tier for the upper levels of large hybrid plans (N >= 65536): the deep cut at F / G
    // records of >= 1024 output words (nodes of 32768+ LLRs), and the root alone. Measured on
    // one box: C5 (64 groups) 4.68 ms deep vs 4.90 root-only; C3 (512 groups, every CU busy
    // either way) 1.53 ms root-only vs 1.59 deep. polar_sc_tuning.tier_words fixes one cut
    // (-1 = none).
    if (p->gmem && p->hybrid && p->sub_words > 0 && t.tier_words >= 0) {
        std::vector<int> cuts;
        if (t.tier_words > 0) {
            cuts.push_back(t.tier_words);
        } else if (p->G >= 4096) {
            cuts.push_back(1024);
            if ((int)p->G / 2 != 1024) cuts.push_back((int)p->G / 2);
        }
        for (int tw : cuts) {
            if (tw < p->lds_slots || (uint32_t)tw > p->G / 2) continue;
            polar_host::TierPlan t = tier_schedule(*p, tw);
            if (!t.steps.empty()) p->tiers.push_back(std::move(t));
        }
    }
    s.tier_steps = p->tiers.empty() ? 0u : (uint32_t)p->tiers[0].steps.size();
    s.tier_words = p->tiers.empty() ? 0u : (uint32_t)p->tiers[0].tw;
    s.kernel = p->jit ? 1u : (p->hybrid ? 2u : 0u);
    s.storage = p->jit ? 2u : (uint32_t)p->gmem;
    s.lds_bytes_per_wave = p->jit ? 8u * (N + 16u) : (uint32_t)p->lds_group_dwords * 4u;
    s.scratch_bytes_per_wave = p->jit ? 0u : (uint64_t)p->hbm_group_dwords * 4u;
    if (p->pair) {
        // per frame pair: HBM slot rows + partial sums; LDS: the subtree-root level
        s.kernel = 3u;
        s.storage = 1u;
        s.tier_steps = (uint32_t)p->pair_tier.steps.size();
        s.tier_words = (uint32_t)p->pair_tier.tw;
        s.lds_bytes_per_wave = (uint32_t)((p->pair_fused ? 2 : 1) * p->sub_words / p->wpr()) * (uint32_t)p->slot_row_bytes();
        s.scratch_bytes_per_wave = (uint64_t)p->pair_dwords * 4u;
    }
    // automatic layout: a PAR 16 pair plan also holds its solo plan, which small batches decode
    // with (layout_for). The alternate takes the solo defaults (subtrees of min(512, N / 32)
    // words, automatic waves, LDS levels and subtree roots), not the pair plan's tuning, which
    // was chosen for the other layout; only the way subtree decoders are built
    // (sub_inline) carries over. polar_sc_tuning.layout = 1 builds no alternate.
    if (p->pair && !p->solo && t.layout == 0 && c.par == 16 && c.sigmag == 1 && c.llr_bits <= 9 && p->G >= 128) {
        polar_sc_tuning ts{};
        ts.layout = 2;
        ts.kernel = 3;
        ts.sub_inline = t.sub_inline;
        polar_sc_plan *a = nullptr;
        if (polar_sc_plan_create_tuned(&a, N, info_mask, &c, &ts) == 0) p->alt = a;
    }
    *out = p;
    return 0;
}

int polar_sc_plan_destroy(polar_sc_plan *p)
{
    if (!p) return -EINVAL;
    if (p->alt) polar_sc_plan_destroy(p->alt);
    for (auto &kv : p->host_bufs) {
        if (kv.second.llr) (void)hipFree(kv.second.llr);
        if (kv.second.out) (void)hipFree(kv.second.out);
    }
    int cur = 0;
    bool have_dev = hipGetDevice(&cur) == hipSuccess;
    for (auto &kv : p->dev) {
        if (have_dev) (void)hipSetDevice(kv.first);
        if (kv.second.ops) (void)hipFree(kv.second.ops);
        for (void *so : kv.second.seg_ops)
            if (so) (void)hipFree(so);
        if (kv.second.module) (void)hipModuleUnload(kv.second.module);
        if (kv.second.imodule) (void)hipModuleUnload(kv.second.imodule);
        if (kv.second.module16) (void)hipModuleUnload(kv.second.module16);
        if (kv.second.ops16) (void)hipFree(kv.second.ops16);
        if (kv.second.scratch) (void)hipFree(kv.second.scratch);
        if (kv.second.wide) (void)hipFree(kv.second.wide);
    }
    if (have_dev && !p->dev.empty()) (void)hipSetDevice(cur);
    delete p;
    return 0;
}

int polar_sc_plan_prepare(const polar_sc_plan *p, size_t max_batch)
{
    if (!p) return -EINVAL;
    DevState *st = nullptr;
    // automatic layout: only the plan that decodes max_batch frames (layout_for) gets its
    // schedule and scratch here; the other one is set up by the first decode that uses it
    // (a caller of large batches must not pay the solo scratch, ~0.6 GB at C5)
    if (p->alt) p = layout_for(p, max_batch ? max_batch : 1, current_simds());
    return ensure_device(p, max_batch ? max_batch : 1, &st);
}

int polar_sc_decode(const polar_sc_plan *p, const int8_t *llr_dev, uint64_t *hard_bits_dev,
                    size_t batch, void *stream)
{
    if (!p) return -EINVAL;
    const int stride16 = (int)(4 * ((p->G + 3) / 4));
    return decode_common(p, llr_dev, (uint16_t *)hard_bits_dev, batch, stride16, stream);
}

int polar_sc_trace(const polar_sc_plan *p, const int8_t *llr_dev, uint64_t *hard_bits_dev, size_t batch,
                   polar_sc_trace_rec *recs, uint32_t cap, uint32_t *count, double *clock_ghz,
                   uint64_t *total_cycles)
{
    if (!p) return -EINVAL;
    const int stride16 = (int)(4 * ((p->G + 3) / 4));
    return trace_common(p, llr_dev, (uint16_t *)hard_bits_dev, batch, stride16, recs, cap, count, clock_ghz,
                        total_cycles);
}

int polar_sc_decode_i16(const polar_sc_plan *p, const int16_t *llr_dev, uint64_t *hard_bits_dev, size_t batch,
                        void *stream)
{
    if (!p || (batch > 0 && (!llr_dev || !hard_bits_dev))) return -EINVAL;
    if (batch == 0) return 0;
    if (batch > (size_t)0x7FFFFFF8) return -EINVAL;
    DevState *st = nullptr;
    std::unique_lock<std::mutex> held;
    if (p->slot16()) {   // pair plans of 9-bit LLRs read the int16 channel themselves
        const int rc = ensure_device(p, batch, &st, DEV_DECODE, &held);
        if (rc) return rc;
        return polar_host::jit_launch_pair(*p, *st, (const int8_t *)llr_dev, (uint16_t *)hard_bits_dev, (long)batch,
                                           (int)(4 * ((p->G + 3) / 4)), stream);
    }
    int rc = ensure_device(p, batch, &st, DEV_I16, &held);
    if (rc) return rc;
    rc = polar_host::jit_load16(*p, *st);
    if (rc) return rc;
    int wpg = waves_per_group(p, batch, st->simds);
    if (wpg > polar_host::HYBRID_MAX_WAVES) wpg = polar_host::HYBRID_MAX_WAVES;
    const int stride16 = (int)(4 * ((p->G + 3) / 4));
    // hybrid plans: the schedule without generated-subtree records (the int16 interpreter
    // has none of the plan's subtree decoders)
    return polar_host::launch_interp_fn(st->fn16, *p, *st, (const int8_t *)llr_dev, (uint16_t *)hard_bits_dev,
                                        (long)batch, stride16, wpg, stream, nullptr, st->ops16 ? st->ops16 : st->ops);
}

int polar_sc_decode_u16(const polar_sc_plan *p, const int8_t *llr_dev, uint16_t *bits_dev,
                        size_t batch, void *stream)
{
    if (!p) return -EINVAL;
    return decode_common(p, llr_dev, bits_dev, batch, (int)p->G, stream);
}

int polar_sc_decode_host(const polar_sc_plan *p, const int8_t *llr, uint64_t *hard_bits, size_t batch)
{
    if (!p || (batch > 0 && (!llr || !hard_bits))) return -EINVAL;
    if (batch == 0) return 0;
    if (p->cfg.strict_llr) {
        const int lim = (1 << (p->cfg.llr_bits - 1)) - 1;   // quantizer range +-(2^(Q-1) - 1)
        const size_t total = batch * (size_t)p->N;
        for (size_t i = 0; i < total; i++)
            if (llr[i] > lim || llr[i] < -lim) return -EINVAL;
    }
    // chunks of at most ~256 MB of LLRs through device buffers cached in the plan (one host
    // decode per plan at a time: the buffers are shared)
    const size_t words = (p->N + 63) / 64;
    const size_t chunk = std::max<size_t>(8, std::min<size_t>(batch, (256u << 20) / p->N));
    std::lock_guard<std::mutex> lk(p->host_mu);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -EIO;
    polar_host::HostBufs &hb = p->host_bufs[dev];
    if (hb.frames < chunk) {
        if (hb.llr) (void)hipFree(hb.llr);
        if (hb.out) (void)hipFree(hb.out);
        hb.llr = nullptr;
        hb.out = nullptr;
        hb.frames = 0;
        if (hipMalloc((void **)&hb.llr, chunk * p->N) != hipSuccess) return -ENOMEM;
        if (hipMalloc((void **)&hb.out, chunk * words * 8u) != hipSuccess) return -ENOMEM;
        hb.frames = chunk;
    }
    for (size_t f0 = 0; f0 < batch; f0 += chunk) {
        const size_t n = std::min(chunk, batch - f0);
        int rc = hip_err(hipMemcpy(hb.llr, llr + f0 * p->N, n * p->N, hipMemcpyHostToDevice));
        if (!rc) rc = polar_sc_decode(p, hb.llr, hb.out, n, nullptr);
        if (!rc) rc = hip_err(hipMemcpy(hard_bits + f0 * words, hb.out, n * words * 8u, hipMemcpyDeviceToHost));
        if (rc) return rc;
    }
    return 0;
}

int polar_load_frozen_tab(const char *path, uint32_t N, uint32_t K, uint8_t *mask_out, uint32_t cap,
                          uint32_t *N_out)
{
    if (!path || !mask_out) return -EINVAL;
    std::string txt;
    if (!read_text(path, txt)) return -ENOENT;
    std::istringstream in(txt);
    std::string l1, l2, l3, l4;
    if (!std::getline(in, l1) || !std::getline(in, l2) || !std::getline(in, l3) || !std::getline(in, l4))
        return -EINVAL;
    long tabN = std::strtol(l1.c_str(), nullptr, 10);
    if (tabN <= 0) return -EINVAL;
    if (N == 0) N = (uint32_t)tabN;
    if (N > cap || K > N) return -EINVAL;
    std::istringstream ch(l4);
    std::vector<uint32_t> order;
    long v;
    while (ch >> v) {
        if (v >= 0 && (uint32_t)v < N) order.push_back((uint32_t)v);   // Writer.h:61-69
    }
    if (order.size() < K) return -EINVAL;
    std::vector<uint8_t> seen(N, 0);
    for (uint32_t i = 0; i < N; i++) mask_out[i] = 0;
    for (uint32_t i = 0; i < K; i++) {
        if (seen[order[i]]) return -EINVAL;
        seen[order[i]] = 1;
        mask_out[order[i]] = 1;                                          // Writer.h:84-86
    }
    if (N_out) *N_out = N;
    return 0;
}

int polar_load_mask_file(const char *path, uint8_t *mask_out, uint32_t cap, uint32_t *N_out)
{
    if (!path || !mask_out) return -EINVAL;
    std::string txt;
    if (!read_text(path, txt)) return -ENOENT;
    uint32_t n = 0;
    for (char ch : txt) {
        if (ch == '0' || ch == '1') {
            if (n >= cap) return -EINVAL;
            mask_out[n++] = (uint8_t)(ch - '0');
        } else if (!(ch == ' ' || ch == '\t' || ch == '\r' || ch == '\n')) {
            return -EINVAL;
        }
    }
    if (n == 0) return -EINVAL;
    if (N_out) *N_out = n;
    return 0;
}

int polar_codeword_to_info(const polar_sc_plan *p, const uint64_t *xhat, uint8_t *info_out, size_t batch)
{
    if (!p || (batch > 0 && (!xhat || !info_out))) return -EINVAL;
    const uint32_t N = p->N;
    const size_t words = (N + 63) / 64;
    std::vector<uint8_t> v(N);
    for (size_t f = 0; f < batch; f++) {
        const uint64_t *x = xhat + f * words;
        for (uint32_t i = 0; i < N; i++) v[i] = (uint8_t)((x[i >> 6] >> (i & 63)) & 1u);
        for (uint32_t h = 1; h < N; h <<= 1)           // u = x F^{(x)n}
            for (uint32_t b = 0; b < N; b += 2 * h)
                for (uint32_t j = b; j < b + h; j++) v[j] ^= v[j + h];
        uint8_t *o = info_out + f * p->K;
        uint32_t k = 0;
        for (uint32_t i = 0; i < N; i++)
            if (p->mask[i]) o[k++] = v[i];
    }
    return 0;
}

int polar_sc_plan_get_stats(const polar_sc_plan *p, polar_sc_plan_stats *s)
{
    if (!p || !s) return -EINVAL;
    *s = p->stats;
    return 0;
}

int polar_sc_plan_get_schedule(const polar_sc_plan *p, polar_sc_op *ops, uint32_t cap, uint32_t *count)
{
    if (!p || !count) return -EINVAL;
    *count = (uint32_t)p->ops.size();
    if (ops) {
        uint32_t n = cap < *count ? cap : *count;
        std::memcpy(ops, p->ops.data(), n * sizeof(polar_sc_op));
    }
    return 0;
}

int polar_sc_plan_compile(const polar_sc_plan *p)
{
    if (!p) return -EINVAL;
    if (!p->jit && !p->hybrid && !p->pair) return -ENOTSUP;
    if (p->alt)
        if (int rc = polar_sc_plan_compile(p->alt)) return rc;
    std::lock_guard<std::mutex> lk(p->mu);
    return polar_host::jit_compile(*p);
}

int polar_sc_plan_kernel_source(const polar_sc_plan *p, char *buf, size_t cap, size_t *len)
{
    if (!p || !len) return -EINVAL;
    if (!p->jit && !p->hybrid && !p->pair) return -ENOTSUP;
    std::string src;
    try {
        src = polar_host::jit_source(*p);
    } catch (const std::exception &) {
        return -ENOTSUP;
    }
    *len = src.size();
    if (buf && cap) {
        size_t n = cap - 1 < src.size() ? cap - 1 : src.size();
        std::memcpy(buf, src.data(), n);
        buf[n] = 0;
    }
    return 0;
}

int polar_sc_plan_launch_info(const polar_sc_plan *p, size_t batch, uint32_t cus, polar_sc_launch_info *info)
{
    if (!p || !info || batch == 0 || batch > (size_t)0x7FFFFFF8) return -EINVAL;
    polar_sc_launch_info r{};
    r.kernel = p->stats.kernel;
    const int simds = 4 * (int)(cus ? cus : 256u);
    if (p->alt) {   // automatic layout: which batches the solo alternate takes on this device
        r.alt_layout = p->alt->solo ? 2u : 1u;
        r.alt_max_batch = (uint64_t)polar_host::SOLO_FRAMES_PER_SIMD * (uint64_t)simds;
    }
    p = layout_for(p, batch, simds);   // (automatic layout: the plan that decodes this batch)
    r.layout = p->pair ? (p->solo ? 2u : 1u) : 0u;
    r.sub_words = (uint32_t)p->sub_words;
    int regs = 0, regs_seg = 0;
    if (p->jit || p->hybrid || p->pair) {
        // under the plan lock: compile / decode may fill p->jit_code from another thread
        std::lock_guard<std::mutex> lk(p->mu);
        if (const int rc = polar_host::jit_compile(*p)) return rc;
        polar_host::code_regs(*p, regs, regs_seg);
        if (regs < 0 || regs_seg < 0) return -EIO;   // kernel missing from the code object
        r.code_key = polar_host::code_key(*p);
        r.compiler = p->jit_compiler;
    }
    r.regs = (uint32_t)regs;
    r.regs_seg = (uint32_t)regs_seg;
    if (p->pair) {
        const polar_host::PairShape sh = polar_host::pair_shape(*p, (long)batch, simds, regs, regs_seg);
        r.waves_per_block = (uint32_t)sh.W;
        r.blocks = (uint64_t)sh.pairs;
        r.lds_bytes = sh.lds;
        r.lds_row0 = (uint32_t)sh.lds_row0;
    } else if (p->jit) {
        const int wpb = polar_host::MASK_WAVES_PER_BLOCK;
        r.waves_per_block = polar_host::fit_waves(regs, wpb) == wpb ? (uint32_t)wpb : 0u;
        r.blocks = ((batch + 7) / 8 + wpb - 1) / wpb;
    } else {
        int wpg = waves_per_group(p, batch, simds);
        if (p->hybrid) wpg = polar_host::fit_waves(regs, wpg);
        r.waves_per_block = (uint32_t)wpg;
        r.blocks = (batch + 7) / 8;
        r.lds_bytes = (uint32_t)p->lds_group_dwords * 4u;
    }
    *info = r;
    return 0;
}

int polar_sc_debug_subtree(const polar_sc_plan *p, uint32_t id, const uint16_t *in_dev, uint32_t *out_dev)
{
    if (!p || !in_dev || !out_dev) return -EINVAL;
    if (!p->pair) return -ENOTSUP;
    if (id >= p->subs.size()) return -EINVAL;
    DevState *st = nullptr;
    int rc = ensure_device(p, 1, &st);
    if (rc) {
        std::fprintf(stderr, "polar_sc_debug_subtree: device setup failed (%d): %s\n", rc, p->jit_log.c_str());
        return rc;
    }
    int i = (int)id;
    void *args[] = {(void *)&in_dev, (void *)&out_dev, (void *)&i};
    hipError_t e = hipModuleLaunchKernel(st->fn_subtest, 1, 1, 1, 64, 1, 1, 0, nullptr, args, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) std::fprintf(stderr, "polar_sc_debug_subtree: %s\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : -EIO;
}

int polar_sc_selftest_lanes(uint32_t *out_dev)
{
    if (!out_dev) return -EINVAL;
    return polar_sc_launch_selftest(out_dev) ? -EIO : 0;
}

}  // extern "C"
