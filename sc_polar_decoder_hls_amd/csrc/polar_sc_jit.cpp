// polar_sc_jit.cpp -- per-frozen-mask decode kernels, generated at plan time and compiled
// with hipRTC for gfx950.
//
// The reference is specialised per code the same way: Frozen_Bit_Generator writes the mask
// into polar_parameters.h and the HLS design is re-synthesised for it
// (Frozen_Bit_Generator/src/Writer.h:110-162, script/script_tests.sh:17-58). Here the
// compiled schedule (polar_sc_op list) is unrolled into straight-line HIP: every stage
// buffer is a register array with compile-time indices, every partial-sum position and
// every leaf frozen pattern is a constant, and there is no interpreter loop at all.
// Used for N <= 1024 (all stage buffers fit in VGPRs); larger N use the schedule
// interpreter in polar_sc_kernels.hip.
#include "polar_sc_plan.hpp"

#include <hip/hiprtc.h>

#include <cerrno>
#include <cstdio>
#include <cstring>
#include <sstream>

namespace {
#include "polar_sc_device_src.inc"   // kPolarDeviceSrc: polar_sc_device.h as a string
}

namespace polar_host {

bool jit_supported(uint32_t N) { return N >= 32 && N <= 1024; }

namespace {

struct Gen {
    const polar_sc_plan &p;
    std::ostringstream o;
    int LG;
    explicit Gen(const polar_sc_plan &pp) : p(pp), LG(pp.lg) {}

    // word i of the node of depth sd (2^sd words)
    std::string S(int sd, int i) const
    {
        std::ostringstream s;
        if (sd == LG) s << "CH(" << i << ")";
        else s << "b" << sd << "[" << i << "]";
        return s.str();
    }
    // 16 partial-sum words starting at q: low frame bits 0..15, high frame bits 16..31
    static std::string get16(int q)
    {
        std::ostringstream s;
        s << "(((u32)(bl >> " << q << ") & 0xFFFFu) | ((u32)(bh >> " << q << ") << 16))";
        return s.str();
    }
    void put(int pos, int n, const std::string &acc)
    {
        unsigned long long m = ((n >= 64) ? ~0ull : ((1ull << n) - 1ull)) << pos;
        o << "    { const u32 a_ = " << acc << "; const u64 m_ = 0x" << std::hex << m << std::dec
          << "ull; bl = (bl & ~m_) | (((u64)(a_ & 0xFFFFu) << " << pos << ") & m_); bh = (bh & ~m_) | (((u64)(a_ >> 16) << "
          << pos << ") & m_); }\n";
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
        s << "((c_ << " << (15 - (i & 15)) << ") & SGN)";
        return s.str();
    }

    // scheduling fence: keeps the straight-line code from hoisting every load of a long
    // op (e.g. the 64 channel words of the root F) and inflating the register footprint
    void fence() { o << "  __builtin_amdgcn_sched_barrier(0);\n"; }
    void chunk_fence(int i, int n)
    {
        if ((i & 7) == 7 && i + 1 < n) fence();
    }

    void op(const polar_sc_op &op)
    {
        const int sd = LG - op.level, cd = sd - 1, n = op.n;
        fence();
        switch (op.code) {
        case POLAR_OP_F:
            o << "  // F level " << op.level << " n " << n << "\n";
            for (int i = 0; i < n; i++) {
                o << "  b" << cd << "[" << i << "] = F_sm(" << S(sd, i) << ", " << S(sd, n + i) << ");\n";
                chunk_fence(i, n);
            }
            break;
        case POLAR_OP_G:
            o << "  { // G level " << op.level << " n " << n << " upos " << op.upos << "\n    u32 c_;\n";
            for (int i = 0; i < n; i++) {
                ucache(op.upos, i);
                o << "    b" << cd << "[" << i << "] = G_sm<15>(" << S(sd, i) << ", " << S(sd, n + i) << ", "
                  << uflag(i) << ");\n";
                chunk_fence(i, n);
            }
            o << "  }\n";
            break;
        case POLAR_OP_FLEAF:
        case POLAR_OP_GLEAF: {
            o << "  { // " << (op.code == POLAR_OP_FLEAF ? "F" : "G") << "+leaf pos " << op.pos << " fb 0x" << std::hex
              << op.fb << std::dec << "\n";
            if (op.code == POLAR_OP_FLEAF) {
                o << "    const u32 L_ = F_sm(" << S(sd, 0) << ", " << S(sd, 1) << ");\n";
            } else {
                o << "    u32 c_; ";
                ucache(op.upos, 0);
                o << "    const u32 L_ = G_sm<15>(" << S(sd, 0) << ", " << S(sd, 1) << ", " << uflag(0) << ");\n";
            }
            o << "    const u32 x_ = leaf_ct<0x" << std::hex << op.fb << std::dec << "u, 0, 16>(L_, ln);\n";
            put(op.pos, 1, "((x_ >> 15) & 1u) | ((x_ >> 15) & 0x10000u)");
            o << "  }\n";
            break;
        }
        case POLAR_OP_REP:
            o << "  { // REP n " << n << " pos " << op.pos << "\n    u32 acc_ = 0u;\n";
            for (int i = 0; i < n; i++) {
                o << "    acc_ = G_sm<511>(row_add_tree(F_sm(" << S(sd, i) << ", " << S(sd, n + i) << "), ln), acc_, 0u);\n";
                chunk_fence(i, n);
            }
            o << "    const u32 full_ = ((acc_ & 0x8000u) ? 0x0000FFFFu : 0u) | ((acc_ & 0x80000000u) ? 0xFFFF0000u : 0u);\n";
            for (int j = 0; j < n; j += 16) put(op.pos + j, n < 16 ? n : 16, "full_");
            o << "  }\n";
            break;
        case POLAR_OP_R1:
        case POLAR_OP_SPC: {
            const bool spc = op.code == POLAR_OP_SPC;
            o << "  { // " << (spc ? "SPC" : "R1") << " n " << n << " pos " << op.pos << " upos " << op.upos
              << "\n    u32 c_, acc_ = 0u, par_ = 0u, klo_ = 0xFFFFFFFFu, khi_ = 0xFFFFFFFFu;\n";
            for (int i = 0; i < n; i++) {
                ucache(op.upos, i);
                o << "    { const u32 l_ = G_sm<15>(" << S(sd, i) << ", " << S(sd, n + i) << ", " << uflag(i)
                  << "); const u32 h_ = l_ & SGN; acc_ |= h_ >> " << (15 - (i & 15)) << ";";
                if (spc)
                    o << " par_ ^= h_; klo_ = __builtin_elementwise_min(klo_, ((l_ & 0x1Fu) << 24) | " << (i << 4)
                      << "u); khi_ = __builtin_elementwise_min(khi_, (((l_ >> 16) & 0x1Fu) << 24) | " << (i << 4)
                      << "u);";
                o << " }\n";
                chunk_fence(i, n);
                if ((i & 15) == 15 || i == n - 1) {
                    put(op.pos + (i & ~15), n < 16 ? n : 16, "acc_");
                    o << "    acc_ = 0u;\n";
                }
            }
            if (spc) {
                o << "    par_ = row_xor(par_);\n"
                     "    klo_ = row_min_u32(klo_ | ln.br); khi_ = row_min_u32(khi_ | ln.br);\n"
                     "    if ((par_ & 0x8000u) && (klo_ & 15u) == ln.br) bl ^= 1ull << ("
                  << op.pos << " + ((klo_ >> 4) & 0xFFFFFu));\n"
                     "    if ((par_ & 0x80000000u) && (khi_ & 15u) == ln.br) bh ^= 1ull << ("
                  << op.pos << " + ((khi_ >> 4) & 0xFFFFFu));\n";
            }
            o << "  }\n";
            break;
        }
        case POLAR_OP_H:
        case POLAR_OP_H0: {
            unsigned long long m = ((n >= 64) ? ~0ull : ((1ull << n) - 1ull)) << op.pos;
            o << "  { const u64 m_ = 0x" << std::hex << m << std::dec << "ull; // " << (op.code == POLAR_OP_H ? "H" : "H0")
              << " pos " << op.pos << " n " << n << "\n";
            if (op.code == POLAR_OP_H)
                o << "    bl ^= (bl >> " << n << ") & m_; bh ^= (bh >> " << n << ") & m_; }\n";
            else
                o << "    bl = (bl & ~m_) | ((bl >> " << n << ") & m_); bh = (bh & ~m_) | ((bh >> " << n << ") & m_); }\n";
            break;
        }
        default:
            break;
        }
    }

    std::string run()
    {
        const int N = (int)p.N, G = (int)p.G;
        o << "#include \"polar_sc_device.h\"\nusing namespace polar;\n"
          << "#define CH(w) conv_pair((u32)chl[16 * (w)] | ((u32)chh[16 * (w)] << 16))\n"
          << "extern \"C\" __global__ void __launch_bounds__(256) polar_sc_mask_kernel(\n"
          << "    const unsigned char *__restrict__ llr, unsigned short *__restrict__ out, int batch, int out_stride)\n{\n"
          << "  const int lane = threadIdx.x & 63, row = lane >> 4, pl = lane & 15;\n"
          << "  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);\n"
          << "  if (wave * 8 >= batch) return;\n"
          << "  const long f_lo = wave * 8 + row, f_hi = wave * 8 + 4 + row;\n"
          << "  const long fl = f_lo < batch ? f_lo : (long)batch - 1, fh = f_hi < batch ? f_hi : (long)batch - 1;\n"
          << "  const unsigned char *__restrict__ chl = llr + fl * " << N << " + pl;\n"
          << "  const unsigned char *__restrict__ chh = llr + fh * " << N << " + pl;\n"
          << "  Lanes ln; ln.init((u32)pl);\n"
          << "  u64 bl = 0, bh = 0;\n";
        for (int d = 1; d < LG; d++) o << "  u32 b" << d << "[" << (1 << d) << "];\n";
        for (const polar_sc_op &op : p.ops) {
            if (op.code == POLAR_OP_END) break;
            this->op(op);
        }
        // END (my_module.h:1848-1869) + wrapper_out: x^ words in natural order
        o << "  const bool st_lo = f_lo < batch, st_hi = f_hi < batch;\n"
          << "  unsigned short *o_lo = out + (size_t)f_lo * out_stride, *o_hi = out + (size_t)f_hi * out_stride;\n";
        for (int c = 0; c < (G + 15) / 16; c++) {
            o << "  { const u32 t_ = row_transpose16(" << get16(16 * c) << ", ln); const int w_ = " << 16 * c << " + pl;\n"
              << "    if (w_ < " << G << ") { if (st_lo) o_lo[w_] = (unsigned short)(t_ & 0xFFFFu); "
              << "if (st_hi) o_hi[w_] = (unsigned short)(t_ >> 16); } }\n";
        }
        o << "  for (int w_ = " << G << " + pl; w_ < out_stride; w_ += 16) { if (st_lo) o_lo[w_] = 0; if (st_hi) o_hi[w_] = 0; }\n"
          << "}\n";
        return o.str();
    }
};

}  // namespace

std::string jit_source(const polar_sc_plan &p) { return Gen(p).run(); }

int jit_compile(const polar_sc_plan &p)
{
    if (!p.jit_code.empty()) return 0;
    const std::string src = jit_source(p);
    hiprtcProgram prog;
    const char *hdrs[] = {kPolarDeviceSrc};
    const char *names[] = {"polar_sc_device.h"};
    if (hiprtcCreateProgram(&prog, src.c_str(), "polar_sc_mask.hip", 1, hdrs, names) != HIPRTC_SUCCESS) return -EIO;
    const char *opts[] = {"--gpu-architecture=gfx950", "-O3", "-std=c++17"};
    hiprtcResult rc = hiprtcCompileProgram(prog, 3, opts);
    size_t log_size = 0;
    hiprtcGetProgramLogSize(prog, &log_size);
    if (log_size > 1) {
        p.jit_log.resize(log_size);
        hiprtcGetProgramLog(prog, &p.jit_log[0]);
    }
    if (rc != HIPRTC_SUCCESS) {
        hiprtcDestroyProgram(&prog);
        return -EIO;
    }
    size_t code_size = 0;
    hiprtcGetCodeSize(prog, &code_size);
    p.jit_code.resize(code_size);
    hiprtcGetCode(prog, p.jit_code.data());
    hiprtcDestroyProgram(&prog);
    return 0;
}

int jit_load(const polar_sc_plan &p, DevState &st)
{
    if (st.fn) return 0;
    int rc = jit_compile(p);
    if (rc) return rc;
    if (hipModuleLoadData(&st.module, p.jit_code.data()) != hipSuccess) return -EIO;
    if (hipModuleGetFunction(&st.fn, st.module, "polar_sc_mask_kernel") != hipSuccess) return -EIO;
    return 0;
}

int jit_launch(const polar_sc_plan &p, const DevState &st, const int8_t *llr, uint16_t *out, long batch,
               int out_stride, void *stream)
{
    (void)p;
    const long waves = (batch + 7) / 8;
    const unsigned blocks = (unsigned)((waves + 3) / 4);
    int b = (int)batch;
    void *args[] = {(void *)&llr, (void *)&out, (void *)&b, (void *)&out_stride};
    hipError_t e = hipModuleLaunchKernel(st.fn, blocks, 1, 1, 256, 1, 1, 0, (hipStream_t)stream, args, nullptr);
    return e == hipSuccess ? 0 : -EIO;
}

}  // namespace polar_host
