/*
 * polar_sc.h -- C ABI of the MI355X-native batched SC polar decoder (libpolar_sc.so).
 *
 * Drop-in boundary for the hot path of ydelomier/SC_Polar_decoder_HLS: the decoder core
 * SC_MODULE(my_module) (src/module/my_module.h:15-36) plus its stream adapters
 * wrapper_in (src/module/wrapper_in.h:26-44) and wrapper_out (src/module/wrapper_out.h:26-36),
 * i.e. the testbench-level contract
 *
 *     decode(llr_in, frozen_bits) -> hard_bits
 *
 * where llr_in is the quantizer's stream of 6-bit two's-complement LLRs
 * (src/testbench/sc_quantizer/sc_quantizer.h:69-81), frozen_bits is the frozen-bit table
 * (FB port, my_module.h:33; bit = 1 -> information bit) and hard_bits is the estimated
 * codeword x^ (bit_mem_1 streamed out by END, my_module.h:1859-1866), natural order.
 *
 * Plain pointers and sizes only; no HIP, torch or C++ types cross this boundary. Every
 * function returns 0 on success or a negative errno value (-EINVAL, -ENOMEM, -ENOTSUP,
 * -ENOENT, -EIO for a HIP runtime failure); polar_sc_strerror() names it.
 */
#ifndef POLAR_SC_H
#define POLAR_SC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define POLAR_SC_ABI_VERSION 5
#define POLAR_SC_PAR 16

/*
 * Decoder configuration. Mirrors the compile-time switches of the reference's
 * src/module/config.h:2-30 (+ PAR from polar_parameters.h:8). The default
 * (polar_sc_default_config) is the configuration the reference ships. Also accepted, the
 * design space the reference's scripts sweep:
 *   * pruning_level 0/1/2 with any combination of elag_r1 / elag_rep / elag_spc / elag_rep2 /
 *     elag_spc2 / elag_h0 (script/script_tests.sh:103-122);
 *   * llr_bits 5..9 (QUANT, script/parser.sh:12, parser_comp.sh:12): the LLR is the low
 *     llr_bits of each channel value (int8 frames, or int16 frames via polar_sc_decode_i16);
 *   * sigmag 1 (SIGMAG) or 0 (CA2, the two's complement datapath of functions.h:48-118)
 *     (script/parser.sh:15,43);
 *   * extended 1/0 (config.h:14: exact or saturating leaves);
 *   * par 4, 8, 16, 32 or 64 (script_tests.sh:11 runs 16 and 64, script_RTL_sim.sh 4..64).
 * The shipped datapath (sigmag 1, par 16, llr_bits <= 8; either extended, every pruning level
 * and elag combination) runs the generated kernels; for N >= 1024 so does every other format
 * (the pair kernel: par 4 .. 64, sigmag 0 / 1, llr_bits 5..9, every pruning level); smaller
 * codes outside the shipped datapath run the schedule interpreter compiled for it. elag_rare = 1
 * (does not compile in the reference, my_module.h:255 vs :1511) is rejected with -ENOTSUP.
 */
typedef struct polar_sc_config {
    int32_t llr_bits;       /* LLR_BITS            (config.h:2)      default 6  */
    int32_t par;            /* PAR                 (polar_parameters.h:8) 16    */
    int32_t sigmag;         /* SIGMAG=1 / CA2=0    (config.h:11)     default 1  */
    int32_t extended;       /* EXTENDED            (config.h:14)     default 1  */
    int32_t pruning_level;  /* PRUNING_LEVEL       (config.h:16)     default 2  */
    int32_t elag_r1;        /* ELAG_R1             (config.h:19)     default 1  */
    int32_t elag_rep;       /* ELAG_REP            (config.h:20)     default 1  */
    int32_t elag_spc;       /* ELAG_SPC            (config.h:21)     default 1  */
    int32_t elag_rep2;      /* ELAG_REP2           (config.h:22)     default 0  */
    int32_t elag_spc2;      /* ELAG_SPC2           (config.h:23)     default 0  */
    int32_t elag_rare;      /* ELAG_RARE           (config.h:26)     default 0  */
    int32_t elag_h0;        /* ELAG_H0             (config.h:28)     default 1  */
    int32_t strict_llr;     /* 0: LLRs are taken modulo 2^llr_bits like the reference's
                               sc_bigint<LLR_BITS> LLR (config.h:6); 1: polar_sc_decode_host
                               rejects |llr| > 2^(llr_bits-1) - 1 with -EINVAL (the device
                               entry point never validates).               default 0 */
} polar_sc_config;

/* Kernel selection and launch shape of a plan (all zero = automatic, what
 * polar_sc_plan_create uses). The decode result never depends on these; they exist for tests
 * and measurements. The generated kernels depend only on the mask, the config and this
 * struct (never on the environment). Out-of-range values -> -EINVAL. */
typedef struct polar_sc_tuning {
    int32_t kernel;           /* 0 = automatic; 1 = the schedule interpreter for every N
                                 (no per-mask / generated-subtree code); 2 = the hybrid
                                 kernel (8-frame groups) for N > 1024; 3 = the pair kernel
                                 (one frame pair per wave) for N >= 2048, and N = 1024
                                 outside the shipped datapath. A forced kernel or sub_words the plan
                                 cannot use is an error (-ENOTSUP / -EINVAL), never a
                                 silent fallback */
    int32_t waves_per_group;  /* interpreter / hybrid launches: waves per 8-frame group, 0 =
                                 automatic (more when the batch cannot fill the GPU), else 1,
                                 2, 4, 8 or 16 (capped at the hybrid kernel's bound) */
    int32_t sub_words;        /* hybrid / pair plans: generated subtree size in 16-LLR words,
                                 0 = automatic (hybrid: 64, 128 from N = 32768; pair:
                                 min(256, N / 32)), else a power of two 2..128 (hybrid) or
                                 32..256 and <= N / 32 (pair) */
    int32_t tier_words;       /* hybrid HBM-scratch plans: F / G records of >= this many words
                                 run as grid launches; 0 = automatic, -1 = no grid tier */
    int32_t lds_slots;        /* HBM-scratch plans: stage slots held in LDS, 0 = automatic,
                                 else 256, 512 or 1024; pair plans: the levels of nodes of
                                 up to this many words sit in LDS whatever the batch (the
                                 default fits them to the LDS share of the resident pairs) */
    int32_t hybrid_waves;     /* hybrid plans: waves per group of the kernel's launch bound,
                                 0 = automatic (8), else 4 or 8 */
    int32_t chain_max;        /* pair plans: F / G records fused into one descent chain
                                 (pop_chain), 0 = automatic (3), 1 = no fusion, 2, 3 or 4
                                 (4 can exceed the register budget of an 8-wave block: the
                                 launch then runs fewer waves per pair, see
                                 polar_sc_plan_launch_info) */
    int32_t sub_inline;       /* pair plans: how the kernel runs its generated subtree
                                 decoders. 0 = automatic, 1 = as calls (one __noinline__
                                 function per distinct subtree), 2 = inlined into the kernel
                                 at every call site (no call frame: no callee-saved register
                                 stores; longer hipRTC compile) */
    int32_t layout;           /* pair plans: 0 = automatic, 1 = frame pairs (two frames per
                                 wave in the 16-bit halves, four words per register), 2 = solo
                                 (one frame per wave, the halves carry words 8 j + 4 h + r:
                                 eight words per register, half the instructions per frame on
                                 nodes of >= 16 words; PAR 16 SIGMAG only, LLR_BITS <= 9) */
    int32_t sub_root;         /* pair plans: where a generated subtree decoder reads its root.
                                 0 = automatic (2 in the frame-pair layout when the frame
                                 has at least 16 subtrees, 1 otherwise),
                                 1 = from a stage slot written by the
                                 upper-level F / G, 2 = as F / G of its parent's slot rows
                                 (the subtree-root level then needs no slot) */
} polar_sc_tuning;

/* Immutable decode plan: N, config, frozen mask, compiled decode schedule and its device
 * copy. Safe to share between threads. Decode calls on different streams may overlap for
 * plans whose stats.storage is 0 or 2 (state in LDS / registers); a storage == 1 plan
 * (large N, stage LLRs in an HBM scratch owned by the plan) must be used by one stream at a
 * time on a device -- create one plan per stream to overlap those. */
typedef struct polar_sc_plan polar_sc_plan;

/* One step of the compiled, data-independent decode schedule (introspection only; the
 * device consumes the same records). Replaces the FSM walk of my_module::do_action. */
typedef struct polar_sc_op {
    int32_t code;   /* POLAR_OP_* */
    int32_t level;  /* source stage level (0 = channel LLRs, k = node of N/16 >> k words) */
    int32_t n;      /* words (16 LLRs / 16 bits) per operand half */
    int32_t pos;    /* first bit_mem word written (or combined, for H/H0) */
    int32_t upos;   /* first bit_mem word of partial sums for G-type ops, -1 = zero (H0 route) */
    uint32_t fb;    /* leaf ops: bits 0..15 frozen pattern of the 16-LLR word, bits 16..18 the
                       leaf decoder (POLAR_LEAF_*; non-plain only at pruning_level 1).
                       PAR > 16 leaves (expanded into F / G / FLEAF / GLEAF / H records):
                       bit 19 = G_extended (no clamp), bits 20..23 = operand width above
                       llr_bits. PAR 4 / 8: FLEAF / GLEAF decode the whole 16-LLR word
                       (its PAR words); bits 0..15 its frozen pattern */
    int32_t reserved[2];   /* [1], PAR 4 / 8 leaf records: per PAR word g of the word, bits
                              7g..7g+3 its do_prunning class, 7g+4..7g+6 its PR1 leaf
                              decoder; bit 28 = PRUNING_LEVEL 2 */
} polar_sc_op;

enum {
    POLAR_OP_F = 1,      /* f_loop of F_STATE        (my_module.h:373-445)  */
    POLAR_OP_G = 2,      /* g_loop of G_STATE        (my_module.h:704-781)  */
    POLAR_OP_FLEAF = 3,  /* F with NB_ITER=1 + R_STATE leaf (my_module.h:595) */
    POLAR_OP_GLEAF = 4,  /* G with NB_ITER=1 + R_STATE leaf                  */
    POLAR_OP_REP = 5,    /* F_REP_STATE              (my_module.h:1292-1390) */
    POLAR_OP_R1 = 6,     /* G_R1_STATE               (my_module.h:1571-1642) */
    POLAR_OP_SPC = 7,    /* G_SPC_STATE              (my_module.h:1737-1842) */
    POLAR_OP_H = 8,      /* H_STATE                  (my_module.h:881-998)   */
    POLAR_OP_H0 = 9,     /* H0_STATE                 (my_module.h:1002-1104) */
    POLAR_OP_END = 10,   /* END                      (my_module.h:1848-1869) */
    POLAR_OP_PLEAF = 14  /* PAR > 16: R_STATE PRUNING_LEVEL 1 decoder (fb bits 16..18) of the
                            PAR word whose n words are the level-`level` node at pos */
};

/* leaf decoders of R_STATE at PRUNING_LEVEL 1 (my_module.h:566-593) */
enum {
    POLAR_LEAF_PLAIN = 0,   /* Spec_Polar_Decoder (library.h:149-172); also R0 / R1 groups   */
    POLAR_LEAF_REP = 1,     /* Spec_REP_Node (library.h:189-210, functions.h:1167-1176)     */
    POLAR_LEAF_SPC = 2,     /* Spec_SPC_Node (library.h:235-256, functions.h:2111-2136)     */
    POLAR_LEAF_REP2 = 3,    /* Spec_REP_REP2_Node, sel 1 (library.h:212-233, functions.h:1353-1420) */
    POLAR_LEAF_SPC2 = 4,    /* Spec_SPC_SPC2_Node, sel 1 (library.h:258-280, functions.h:2786-2811) */
    POLAR_LEAF_R1 = 5       /* Spec_Node_R1 (library.h:180-185): the hard decisions. SIGMAG plans
                               decode R1 groups with the plain leaf, which gives the same bits;
                               in CA2 it does not (F has no -0) */
};

typedef struct polar_sc_plan_stats {
    uint32_t N, K, groups;            /* N, information bits, N/PAR (do_prunning groups) */
    uint32_t n_r0, n_r1, n_rep, n_spc, n_rn;   /* do_prunning group census          */
    uint32_t n_ops;                   /* schedule length (incl. END)                   */
    uint32_t op_count[16];            /* per POLAR_OP_* code                           */
    uint64_t word_ops;                /* sum over ops of processed words (F/G-type)    */
    uint32_t storage;                 /* stage LLR storage of the decode kernel:
                                         0 = LDS (schedule interpreter), 1 = HBM scratch
                                         (interpreter, large N), 2 = VGPRs (per-mask kernel,
                                         N <= 1024)                                      */
    uint32_t lds_bytes_per_wave;      /* LDS footprint of one 8-frame group: storage 2:
                                         the staged channel frames; 0: all stage slots and
                                         partial sums; 1: the lower tree levels. Pair plans
                                         (kernel 3): per frame pair, the subtree-root slot
                                         level only -- the launch puts more levels in LDS
                                         when the batch leaves room (up to ~129 KB per
                                         pair; polar_sc_plan_launch_info.lds_bytes)      */
    uint64_t scratch_bytes_per_wave;  /* HBM scratch of one 8-frame group (storage 1:
                                         upper tree levels + partial sums), else 0. Pair
                                         plans: per frame pair (slot rows + partial sums) */
    uint32_t kernel;                  /* decode kernel: 0 = schedule interpreter,
                                         1 = per-mask kernel (N <= 1024), 2 = hybrid
                                         (interpreter for the upper tree levels, generated
                                         code for every mixed subtree of sub_words),
                                         3 = pair kernel (one frame pair per wave, generated
                                         subtree decoders, upper levels over stage-slot
                                         rows; the default for N >= 2048, and for
                                         N = 1024 outside the shipped datapath)          */
    uint32_t sub_words;               /* hybrid / pair: subtree size in 16-LLR words      */
    uint32_t n_sub_kinds;             /* hybrid / pair: distinct generated subtree decoders */
    uint32_t n_sub_calls;             /* hybrid / pair: subtree decoder calls per frame
                                         group / pair                                    */
    uint32_t tier_steps;              /* hybrid, large N: launches per decode of the grid
                                         tier (upper-level F / G over all frame groups +
                                         the schedule segments between them), else 0     */
    uint32_t tier_words;              /* grid tier: F / G records of >= this many output
                                         words run grid-wide, else 0                     */
} polar_sc_plan_stats;

/* Fill *cfg with the reference configuration (config.h as shipped). */
int polar_sc_default_config(polar_sc_config *cfg);

/* Compile a plan. N: power of two, 32 <= N <= 2^20 (INIT needs N/16 >= 2 words,
 * my_module.h:294-309). info_mask: N bytes, nonzero = information bit (frozen table
 * bit = 1, Frozen_Bit_Generator/src/Writer.h:86-93). cfg: NULL -> reference default.
 * Replaces do_prunning (my_module.h:61-166) + the FB FIFO load. Host-only: it does not
 * touch the GPU (the schedule is uploaded on the first device decode). */
int polar_sc_plan_create(polar_sc_plan **out, uint32_t N, const uint8_t *info_mask,
                         const polar_sc_config *cfg);
/* Same with explicit kernel selection (tun == NULL: automatic, as polar_sc_plan_create). */
int polar_sc_plan_create_tuned(polar_sc_plan **out, uint32_t N, const uint8_t *info_mask,
                               const polar_sc_config *cfg, const polar_sc_tuning *tun);
int polar_sc_plan_destroy(polar_sc_plan *plan);

/* Decode `batch` frames already resident on the current HIP device.
 *   llr_dev:       [batch][N] int8 two's-complement LLRs (wrapper_in input stream order)
 *   hard_bits_dev: [batch][ceil(N/64)] uint64, bit i of word j = x^[64 j + i]
 *                  (for N = 32 the high half of each frame's single word is zero)
 *   stream:        hipStream_t (NULL = default stream); the call is asynchronous.
 * Replaces one INIT..END pass of my_module::do_action per frame (my_module.h:174-1877).
 * The first call on a device uploads the schedule (synchronously); for graph capture,
 * call polar_sc_plan_prepare first. */
int polar_sc_decode(const polar_sc_plan *plan, const int8_t *llr_dev, uint64_t *hard_bits_dev,
                    size_t batch, void *stream);

/* Same, with the output as [batch][N/16] uint16 words (bit i of word j = x^[16 j + i]),
 * which is exactly the sequence of TYPE_BITS tokens my_module writes to its `s` port. */
int polar_sc_decode_u16(const polar_sc_plan *plan, const int8_t *llr_dev, uint16_t *bits_dev,
                        size_t batch, void *stream);

/* Same as polar_sc_decode with int16 channel values ([batch][N] int16, the low llr_bits of
 * each are the LLR): the channel for 9-bit LLRs beyond the int8 range (LLR_BITS 9,
 * script/parser_comp.sh:12). Pair plans of 9-bit LLRs (N >= 1024) read the int16 frames
 * directly; other plans run the schedule interpreter of the plan's format. */
int polar_sc_decode_i16(const polar_sc_plan *plan, const int16_t *llr_dev, uint64_t *hard_bits_dev,
                        size_t batch, void *stream);

/* Upload the schedule and reserve device scratch for up to max_batch frames on the
 * current device, so that later polar_sc_decode calls allocate nothing. An automatic-layout
 * pair plan (polar_sc_launch_info.alt_layout != 0) decodes batches of at most alt_max_batch
 * frames with its solo alternate: prepare sets up the plan that decodes max_batch frames,
 * and the other one is set up by the first decode that needs it (call prepare once per batch
 * class before graph capture; polar_sc_tuning.layout = 1 builds no alternate at all).
 * polar_sc_plan_compile builds both kernels of such a plan. */
int polar_sc_plan_prepare(const polar_sc_plan *plan, size_t max_batch);

/* Host-pointer convenience: copies in, decodes, copies out, synchronises.
 * hard_bits: [batch][ceil(N/64)] uint64 as for polar_sc_decode. */
int polar_sc_decode_host(const polar_sc_plan *plan, const int8_t *llr, uint64_t *hard_bits,
                         size_t batch);

/* Frozen_Bit_Tab/FB_N{N}_K{K}.txt reader (Writer.h:35-93, Input=0): line 1 = table size,
 * lines 2-3 ignored, line 4 = reliability order (most reliable first). Indices >= N are
 * dropped, the first K remaining are information bits. N = 0 -> the table's own size.
 * mask_out: capacity `cap` bytes; *N_out receives N. */
int polar_load_frozen_tab(const char *path, uint32_t N, uint32_t K, uint8_t *mask_out,
                          uint32_t cap, uint32_t *N_out);

/* Generated_Frozen_Bit/frozen_n_{N}_k_{K}.txt reader (Writer.h:95-105, Input=1):
 * whitespace-separated 0/1 tokens, 1 = information bit. */
int polar_load_mask_file(const char *path, uint8_t *mask_out, uint32_t cap, uint32_t *N_out);

/* u^ = x^ . F^{(x)n} (F = [[1,0],[1,1]], self-inverse), keep the information positions.
 * xhat: [batch][ceil(N/64)] uint64 host array; info_out: [batch][K] bytes (0/1). Host-side. */
int polar_codeword_to_info(const polar_sc_plan *plan, const uint64_t *xhat, uint8_t *info_out,
                           size_t batch);

int polar_sc_plan_get_stats(const polar_sc_plan *plan, polar_sc_plan_stats *stats);

/* Copy the compiled schedule (at most cap ops) and its length. */
int polar_sc_plan_get_schedule(const polar_sc_plan *plan, polar_sc_op *ops, uint32_t cap,
                               uint32_t *count);

/* Per-mask kernel (plans with stats.storage == 2, N <= 1024): generate its HIP source and
 * compile it for gfx950 now (host only, no GPU needed: the ROCm clang driver, or hipRTC when
 * the driver is absent or the process has a GPU open); otherwise it is built
 * on the first decode. -ENOTSUP for plans that use the hipcc-built schedule interpreter
 * (polar_sc_tuning.kernel = 1). */
int polar_sc_plan_compile(const polar_sc_plan *plan);

/* The generated per-mask kernel source (NUL-terminated, truncated to cap); *len = full size. */
int polar_sc_plan_kernel_source(const polar_sc_plan *plan, char *buf, size_t cap, size_t *len);

/* Launch shape a polar_sc_decode of `batch` frames would use on a device with `cus` compute
 * units (0 = 256, MI355X), computed on the host (compiles the generated kernel if
 * needed; no GPU). The waves of a block must fit the 512 registers per SIMD lane that they
 * share (VGPRs + AGPRs, from the code object's kernel descriptor); the decode lowers its
 * waves per frame group / pair until they do, and returns -ENOTSUP when not even one wave
 * fits (waves_per_block = 0 here). */
typedef struct polar_sc_launch_info {
    uint32_t kernel;            /* stats.kernel */
    uint32_t regs;              /* registers per lane of the decode kernel (allocation
                                   granule), 0 for the hipcc-built interpreter */
    uint32_t regs_seg;          /* pair plans with a grid tier: the segment kernel's */
    uint32_t waves_per_block;   /* waves per frame group / pair; 0: not launchable */
    uint64_t blocks;            /* workgroups of the decode launch */
    uint32_t lds_bytes;         /* dynamic LDS per block */
    uint32_t lds_row0;          /* pair plans: first stage-slot row held in LDS */
    uint64_t code_key;          /* identity of the machine code: hash of the instructions
                                   and kernel descriptors of the plan's compiled code
                                   object (equal code -> equal key whatever the source
                                   text), 0 = none */
    uint32_t layout;            /* pair plans: 1 = frame pairs, 2 = solo (one frame per
                                   wave); an automatic-layout plan decodes batches of at
                                   most 2 frames per SIMD solo; 0 = not a pair plan */
    uint32_t sub_words;         /* hybrid / pair plans: subtree size of the decoding plan */
    uint32_t compiler;          /* which compiler built the generated kernel:
                                   POLAR_SC_COMPILER_CLANG (the ROCm clang driver the library
                                   was built with: the default when no GPU is open in the
                                   process, or a code object it cached) or
                                   POLAR_SC_COMPILER_HIPRTC (hipRTC: no clang driver, or a GPU
                                   already open and no cached clang object); 0 = none */
    uint32_t alt_layout;        /* automatic-layout pair plans: the layout of the alternate
                                   plan that decodes small batches (2 = solo), 0 = the plan
                                   has none (forced layout, PAR != 16, LLR_BITS 9, or a
                                   frame the solo code cannot take) */
    uint64_t alt_max_batch;     /* batches of at most this many frames (2 per SIMD of `cus`
                                   compute units) decode with the alternate; 0 = none */
} polar_sc_launch_info;

enum { POLAR_SC_COMPILER_CLANG = 1, POLAR_SC_COMPILER_HIPRTC = 2 };

int polar_sc_plan_launch_info(const polar_sc_plan *plan, size_t batch, uint32_t cus, polar_sc_launch_info *info);

/* ---- Frame source and error accounting of the reference testbench ---- */

/* The reference's C-sim frame chain for frames frame0 .. frame0+batch-1, generated on the
 * current device (src/testbench/sc_top_module.h:101-160): encoder (frame f sends row
 * f % ncw of `codewords`, [ncw][N] host bytes 0/1; ncw = 0 -> all-zero codewords, as the
 * reference does for N not in {8, 512, 1024}, sc_encoder.h:91-122), BPSK (bit 1 -> -1),
 * two xorshift128 streams seeded from the 8-bit `seed8` (sc_xorshift128.h:56-125),
 * Box-Muller (sc_awgn.h:60-89), v = bpsk + noise * sigma (sc_adder.h:135-154), and
 * (short)(v * beta) clamped to [vsatn, vsatp] (sc_quantizer.h:69-81; the testbench uses
 * beta 4, -31, 31, sigma = 1/sqrt(2 R 10^(EbN0/10))).
 *   llr_dev:  [batch][N] int8, the decoder input (16-byte aligned)
 *   xref_dev: [batch][ceil(N/64)] uint64 sent codewords (bit i of word j = x[64j+i]), or NULL
 * Synchronous. Frames are independent (per-frame stream states by GF(2) jump-ahead). */
int polar_csim_frames(uint32_t N, uint32_t seed8, uint64_t frame0, size_t batch, float sigma,
                      int beta, int vsatn, int vsatp, const uint8_t *codewords, uint32_t ncw,
                      int8_t *llr_dev, uint64_t *xref_dev, void *stream);

/* Host: the two xorshift128 stream states at the start of each frame, states[f][0..3] =
 * stream 1 (x, y, z, w), states[f][4..7] = stream 2. */
int polar_csim_states(uint32_t N, uint32_t seed8, uint64_t frame0, size_t batch, uint32_t *states);

/* sc_error_counter (sc_error_counter.h:50-126) on the device: adds to counts_dev[3]
 * (unsigned 64-bit): [0] per-frame bit errors taken modulo 1024 (the reference's
 * sc_uint<10>), [1] frames whose wrapped count is non-zero, [2] exact bit errors.
 * xhat_dev / xref_dev: [batch][ceil(N/64)] uint64 as polar_sc_decode writes. Asynchronous. */
int polar_count_errors(const uint64_t *xhat_dev, const uint64_t *xref_dev, uint32_t N, size_t batch,
                       unsigned long long *counts_dev, void *stream);

/* ---- Per-op monitor ----
 * The analogue of the reference's latency monitor (sc_monitor.h:50-140 over my_module's
 * Fct_ID / N_value ports, my_module.h:21-30): one synchronous decode of `batch` resident
 * frames (hard_bits_dev receives the same x^ as polar_sc_decode) with the schedule
 * interpreter instrumented (hybrid plans: the hybrid kernel; per-mask and pair plans are
 * profiled on the interpreter, which runs the same schedule, and the pair kernel is not
 * compiled for it; tools/pair_stamps.py stamps the pair kernel itself). For every device op, the shader-clock
 * cycles from its start to the next op's start, measured on the lead wave of frame group 0
 * while the rest of the batch runs. recs == NULL: only *count (the number of device ops,
 * END included) is returned. Device ops are the schedule of polar_sc_plan_get_schedule plus,
 * for HBM-scratch plans, partial-sum window records (code 11 open / 12 flush) and, for hybrid
 * plans, generated-subtree calls (code 13) in place of the subtree's ops. */
typedef struct polar_sc_trace_rec {
    int32_t code;       /* POLAR_OP_* (or 11 / 12 / 13, see above) */
    int32_t level;      /* source stage level (node of N >> level LLRs) */
    int32_t n;          /* words per operand half */
    int32_t pos;
    uint64_t cycles;    /* shader clock cycles of this op (0 for END) */
} polar_sc_trace_rec;

int polar_sc_trace(const polar_sc_plan *plan, const int8_t *llr_dev, uint64_t *hard_bits_dev, size_t batch,
                   polar_sc_trace_rec *recs, uint32_t cap, uint32_t *count, double *clock_ghz,
                   uint64_t *total_cycles);

/* ---- Frozen-table tooling: Frozen_Bit_Generator (main.cpp:12-52, src/Writer.h:21-167) ---- */

/* Writer.h:61-93: keep the entries of a reliability order (most reliable first) that are
 * < N; the first K of them are information bits. mask_out: N bytes (cap >= N), 1 = info.
 * -EINVAL unless exactly N distinct entries remain. */
int polar_mask_from_order(const uint32_t *order, uint32_t count, uint32_t N, uint32_t K, uint8_t *mask_out,
                          uint32_t cap);

/* Writer.h:71-79: the FB_N{N}_K{K}.txt ("affect") text of that subset order. Text goes to
 * buf (NUL-terminated, truncated to cap); *len = full length. */
int polar_write_frozen_tab(const uint32_t *order, uint32_t count, uint32_t N, char *buf, size_t cap,
                           size_t *len);

/* Writer.h:110-162: polar_parameters.h for an information mask, byte for byte as the
 * reference generator writes it. par: PAR (power of two <= N); concat: the generator's En
 * (1 = PAR-wide strings, 0 = one sc_bv<1> per bit). Output as for polar_write_frozen_tab. */
int polar_write_parameters_h(const uint8_t *info_mask, uint32_t N, uint32_t par, int32_t concat, char *buf,
                             size_t cap, size_t *len);

/* Read a polar_parameters.h (either form) back: mask_out (cap >= N bytes, 1 = info),
 * *N_out = _NBITS, *par_out = PAR. */
int polar_parse_parameters_h(const char *path, uint8_t *mask_out, uint32_t cap, uint32_t *N_out,
                             uint32_t *par_out);

/* GPU self-test of the cross-lane exchange patterns the kernels rely on.
 * out_dev: 8*64 uint32 on the device; entry [h][lane] (h = 0..3) = source lane seen by `lane`
 * for DPP partner distance 1<<h; [4], [5] = the two results of v_permlane16_swap and [6], [7]
 * those of v_permlane32_swap of the lane id with itself. Synchronous. */
int polar_sc_selftest_lanes(uint32_t *out_dev);

/* Test hook of pair plans (stats.kernel == 3): run generated subtree decoder `id` on one
 * wave (one frame pair): in_dev = its root as stage-slot rows, [S/4 rows][64 lanes] uint16
 * (SM8 pairs: low byte = frame 0, high byte = frame 1, lane 16 r + l = word 4 j + r, position
 * of lane l of polar_sc_pair.h); out_dev = its partial sums, [max(1, S/64) dwords][64 lanes].
 * Synchronous. -ENOTSUP for other plans. */
int polar_sc_debug_subtree(const polar_sc_plan *plan, uint32_t id, const uint16_t *in_dev, uint32_t *out_dev);

const char *polar_sc_strerror(int err);
int polar_sc_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* POLAR_SC_H */
