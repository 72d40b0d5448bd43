// polar_sc_plan.hpp -- private definition of polar_sc_plan (include/polar_sc.h), shared by
// the host plan/schedule code (polar_sc_host.cpp) and the per-mask kernel generator
// (polar_sc_jit.cpp).
#pragma once

#include "../../include/polar_sc.h"

#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace polar_host {

struct DevState {
    void *ops = nullptr;          // schedule (interpreter kernels)
    void *scratch = nullptr;      // HBM stage scratch (interpreter, large N)
    size_t scratch_bytes = 0;
    void *wide = nullptr;         // int16 copy of an int8 batch (pair plans of 9-bit LLRs)
    size_t wide_bytes = 0;
    hipModule_t module = nullptr; // per-mask kernel
    hipFunction_t fn = nullptr;
    hipFunction_t fn_trace = nullptr;   // hybrid plans: the per-op monitor variant
    hipFunction_t fn_tier = nullptr;    // grid-tier plans: upper-level F / G over all groups
    hipFunction_t fn_seg = nullptr;     // pair plans with a grid tier: the segment kernel
    hipFunction_t fn_subtest = nullptr; // pair plans: one generated subtree decoder (test hook)
    void *seg_ops[2] = {nullptr, nullptr};   // grid-tier plans: the segment schedules per tier plan
    hipModule_t imodule = nullptr;      // per-mask plans with llr_bits != 6: hipRTC interpreter
    hipFunction_t ifn_trace = nullptr;  //   (per-op monitor only)
    hipModule_t module16 = nullptr;     // interpreter on the int16 channel (polar_sc_decode_i16)
    hipFunction_t fn16 = nullptr;
    void *ops16 = nullptr;              //   and its schedule when it differs from `ops`
    int simds = 0;                // SIMDs of the device (4 per CU), for launch sizing
    // registers per lane (VGPR + AGPR allocation, kernel descriptor) of the generated decode
    // kernel and of the pair segment kernel: the launch shape is capped so that a block's
    // waves fit (kernel_regs, fit_waves); 0 = not a generated kernel
    int regs = 0, regs_seg = 0;
};

enum JitMode { JIT_OFF = 0, JIT_AUTO = 1 };

// device staging buffers of polar_sc_decode_host
struct HostBufs {
    int8_t *llr = nullptr;
    uint64_t *out = nullptr;
    size_t frames = 0;
};

// device-internal schedule records (never exported): the partial-sum window of HBM-scratch
// plans, and the generated-subtree call of hybrid plans
enum { POLAR_OP_WOPEN = 11, POLAR_OP_WFLUSH = 12, POLAR_OP_SUB = 13, POLAR_OP_PLEAF = 14,
       POLAR_OP_SEGEND = 15, POLAR_OP_SEGCONT = 16 };

// grid tier of a hybrid HBM-scratch plan: the decode as a sequence of launches -- F / G
// records of the upper-level nodes over all frame groups at once (grid), and the schedule
// segments between them (the hybrid kernel, one block per group)
struct TierStep {
    int grid = 0;          // 1: grid F / G launch of record `op`; 0: segment at seg_ops[off]
    polar_sc_op op{};
    int off = 0;
};
struct TierPlan {
    int tw = 0;                        // F / G records of >= tw output words run grid-wide
    std::vector<TierStep> steps;
    std::vector<polar_sc_op> seg_ops;  // the segment schedules, concatenated
};
// polar_sc_op.fb of G / GLEAF records inside a PAR-word leaf (PAR > 16): G_extended (no
// clamp); bits 20..23: operand width above LLR_BITS (polar_sc_interp.h)
constexpr uint32_t FB_EXACT = 1u << 19;

// hybrid kernels: by default at most 8 waves per 8-frame group (one 512-thread block, the
// kernel's launch bound); polar_sc_tuning.hybrid_waves (4 or 8) changes it.
// Measured (tools/wpg_sweep.py): C5 (512 frames) 6.50 -> 5.99 ms from 4 to 8 waves, C3
// (4096 frames, which keeps 4 waves per group) unchanged; 16 waves (1024-thread blocks with
// spilled subtree code) failed to launch (HSA_STATUS_ERROR_INVALID_ISA).
constexpr int HYBRID_MAX_WAVES = 8;

// pair plans (polar_sc_pair.h): at most this many waves per frame pair (512-thread blocks,
// <= 256 VGPRs per wave), subtrees of at most PAIR_SUB_WORDS words in registers
constexpr int PAIR_WAVES_MAX = 8;
constexpr int PAIR_SUB_WORDS = 256;
constexpr int SOLO_SUB_WORDS_MAX = 512;   // solo plans: half the registers per word
// automatic layout: solo while the batch is at most this many frames per SIMD (the solo
// kernels take ~248 registers, so two waves per SIMD keep one dispatch round; beyond that the
// pair layout's two frames per wave win -- tools/layout_ab.py, profiles/r05_ab/)
constexpr int SOLO_FRAMES_PER_SIMD = 2;
// unified register file per SIMD lane (VGPRs + AGPRs) shared by the waves on the SIMD
constexpr int SIMD_REGS = 512;
// one CU's LDS (gfx950)
constexpr long CU_LDS_BYTES = 160l * 1024l;

// launch shape of a pair plan for one batch (jit_launch_pair, polar_sc_plan_launch_info)
struct PairShape {
    int W = 0;            // waves per frame pair (0: the kernel does not fit, -ENOTSUP)
    long pairs = 0;       // blocks (frame pairs; solo plans: frames)
    int lds_row0 = 0;     // first stage-slot row held in LDS
    unsigned lds = 0;     // dynamic LDS bytes per block
};

// grid tier of a pair plan: `seg_ops` is the upper schedule with POLAR_OP_SEGEND where the grid
// launches of `steps` (grid records) run; steps alternate with the segment kernel's cases
struct PairTier {
    int tw = 0;
    std::vector<TierStep> steps;       // grid: op; segment: off = segment index (the kernel's `seg`)
    std::vector<polar_sc_op> seg_ops;
};

}  // namespace polar_host

struct polar_sc_plan {
    uint32_t N = 0, G = 0, K = 0;    // G: 16-LLR device words (N / 16)
    uint32_t GP = 0, p16 = 1;        // PAR groups (N / PAR), device words per group (PAR >= 16)
    uint32_t ppw = 1;                // PAR groups per device word (PAR 4 / 8: 4 / 2)
    int lg = 0;                      // log2(N/16)
    polar_sc_config cfg{};
    polar_sc_tuning tune{};          // kernel selection / launch shape (all 0 = automatic)
    std::vector<uint8_t> mask;       // N, 1 = information
    std::vector<uint64_t> fbp;       // GP, Bit_Frozen (bit k = mask[PAR g + k])
    std::vector<uint8_t> type;       // GP, Node_Type
    std::vector<polar_sc_op> ops;
    std::vector<polar_sc_op> dev_ops;   // device copy when it differs (HBM-scratch plans)
    // the schedule interpreter's copy for the int16 channel (polar_sc_decode_i16): the plan's
    // schedule without generated-subtree records (windowed for HBM-scratch plans); empty when
    // it equals dev_ops (or ops)
    std::vector<polar_sc_op> ops16;
    polar_sc_plan_stats stats{};
    int gmem = 0;
    // interpreter storage of one 8-frame group (dwords): HBM scratch part, LDS part, and the
    // first stage slot held in LDS (polar_sc_kernels.hip, Ctx)
    int hbm_group_dwords = 0, lds_group_dwords = 0, lds0 = 0;
    int lds_slots = 256;             // HBM-scratch plans: LDS region W (slots [G - W, G - 1))
    int jit = 0;                     // 1: decode with the per-mask kernel
    // hybrid plans (N > 1024): the device schedule stops at every mixed node of sub_words
    // words with a POLAR_OP_SUB record; subs[id] is that subtree's own schedule (levels and
    // positions relative to the subtree root), compiled to straight-line code
    int hybrid = 0;
    int hybrid_waves = 8;            // waves per group cap = launch bound / 64 of the hybrid kernel
    int sub_words = 0;
    std::vector<std::vector<polar_sc_op>> subs;
    // grid tier (hybrid HBM plans, polar_sc_host.cpp tier_schedule): F / G records of at
    // least tw output words run as grid-wide launches. tiers[0]: the deep cut; tiers[1]
    // (when it differs): the root only, taken by batches with a frame group per CU or more
    // (polar_sc_jit.cpp launch_tier). Empty: single-kernel decode.
    std::vector<polar_host::TierPlan> tiers;
    // pair plans (N >= 2048, shipped datapath; polar_sc_pairgen.cpp): one frame pair per wave,
    // subtrees of sub_words words as generated register code (subs), the upper levels as
    // loops over stage-slot rows (pair_ops); optional grid tier (pair_tier.steps non-empty)
    int pair = 0;
    // solo layout of a pair plan (polar_sc_pair.h POLAR_SOLO): one frame per block, a slot row /
    // register = 8 words of the frame (pair: 4 words of two frames)
    int solo = 0;
    // automatic layout (polar_sc_tuning.layout = 0) of a PAR 16 pair plan: the solo plan of the
    // same mask, used by decodes whose batch leaves SIMDs idle in the pair layout
    // (polar_sc_host.cpp layout_for); owned, destroyed with this plan
    polar_sc_plan *alt = nullptr;
    std::vector<polar_sc_op> pair_ops;
    polar_host::PairTier pair_tier;
    // subtree roots read as F / G of their parent's slot rows (SUB records carry the folded
    // producer in reserved[1]: 1 = F, 2 = G with upos); the subtree-root level has no slot
    int pair_fused = 0;
    int pair_slot_rows = 0;          // stage-slot rows per pair / solo frame (levels of nodes G/2 .. sub_words, or 2 sub_words when fused)
    int pair_dwords = 0;             // HBM scratch per pair / frame: slot rows (128 B) + bit dwords (256 B)
    int wpr() const { return solo ? 8 : 4; }   // words of one (virtual) frame per slot row
    // bytes of a slot row (64 lanes): SM8 pairs, or SM16 pairs for 9-bit LLRs (polar_sc_pair.h SLOT16)
    // 16-bit slot rows: 9-bit LLRs, and CA2 8-bit LLRs (|MIN| = 128 does not fit an SM8 byte)
    bool wide_slots() const { return cfg.llr_bits > 8 || (cfg.sigmag == 0 && cfg.llr_bits > 7); }
    int slot_row_bytes() const { return wide_slots() ? 256 : 128; }
    bool slot16() const { return pair && cfg.llr_bits > 8; }   // (the kernel reads the int16 channel)
    mutable std::mutex mu;
    mutable std::map<int, polar_host::DevState> dev;
    mutable std::mutex host_mu;                             // polar_sc_decode_host staging
    mutable std::map<int, polar_host::HostBufs> host_bufs;
    mutable std::vector<char> jit_code;   // compiled code object (lazily built)
    mutable uint32_t jit_compiler = 0;    // POLAR_SC_COMPILER_* of jit_code
    mutable std::vector<char> interp_code;   // per-mask plans, llr_bits != 6: traced interpreter
    mutable std::vector<char> code16;        // interpreter on the int16 channel (polar_sc_decode_i16)
    mutable std::string jit_log;
};

namespace polar_host {
// per-mask kernel: generate source, compile with hipRTC for gfx950 (host only), load it on
// the current device, launch it
std::string jit_source(const polar_sc_plan &p);
std::string pair_source(const polar_sc_plan &p);
int jit_launch_pair(const polar_sc_plan &p, const DevState &st, const int8_t *llr, uint16_t *out, long batch,
                    int out_stride, void *stream);
int jit_compile(const polar_sc_plan &p);                 // fills p.jit_code (idempotent)
int jit_load(const polar_sc_plan &p, DevState &st);      // module + function on this device
int jit_launch(const polar_sc_plan &p, const DevState &st, const int8_t *llr, uint16_t *out,
               long batch, int out_stride, void *stream);
int jit_launch_hybrid(const polar_sc_plan &p, const DevState &st, const int8_t *llr, uint16_t *out, long batch,
                      int out_stride, int wpg, void *stream, unsigned long long *trace = nullptr);
int jit_load_interp(const polar_sc_plan &p, DevState &st);
int jit_load16(const polar_sc_plan &p, DevState &st);
int launch_interp_fn(hipFunction_t fn, const polar_sc_plan &p, const DevState &st, const int8_t *llr, uint16_t *out,
                     long batch, int out_stride, int wpg, void *stream, unsigned long long *trace,
                     const void *ops = nullptr);   // schedule: nullptr = st.ops
bool jit_supported(uint32_t N);
int kernel_regs(const std::vector<char> &code, const char *name);   // -1: no such kernel
int fit_waves(int regs, int W);
void code_regs(const polar_sc_plan &p, int &regs, int &regs_seg);
constexpr int MASK_WAVES_PER_BLOCK = 4;   // per-mask kernel launch (polar_sc_jit.cpp MASK_WPB)
PairShape pair_shape(const polar_sc_plan &p, long batch, int simds, int regs, int regs_seg);
uint64_t code_key(const polar_sc_plan &p);   // hash of the compiled kernels' instructions + descriptors (0: none)
}  // namespace polar_host
