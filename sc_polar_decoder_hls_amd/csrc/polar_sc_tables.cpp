// polar_sc_tables.cpp -- frozen-table tooling of the C ABI (host only, no HIP).
//
// The reference specialises its decoder per code with Frozen_Bit_Generator
// (Frozen_Bit_Generator/main.cpp:12-52 -> src/Writer.h:21-167): it reads either a
// reliability order (Frozen_Bit_Tab format, Input = 0) or a 0/1 mask (Generated_Frozen_Bit
// format, Input = 1), writes the subset order back as FB_N{N}_K{K}.txt (the "affect" file,
// Input = 0 only) and emits polar_parameters.h, the header my_module.h compiles against.
// These functions produce the same bytes from in-memory tables, and read a
// polar_parameters.h back into an information mask, so that a plan can be created from the
// exact header a reference build used.
#include "polar_sc.h"

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

namespace {

bool pow2(uint64_t v) { return v && !(v & (v - 1)); }

// ostream text of a double the way `o_file << (log2(x))` prints it (default precision 6)
std::string dbl(double v)
{
    std::ostringstream s;
    s << v;
    return s.str();
}

// An output "file" that supports the reference's seekp(-k, cur) followed by overwriting
// writes (Writer.h:141 and :156 rewind over the trailing separator).
struct SeekBuf {
    std::string s;
    size_t pos = 0;
    void put(const std::string &t)
    {
        for (char c : t) {
            if (pos < s.size()) s[pos] = c;
            else s.push_back(c);
            pos++;
        }
    }
    void seek_back(size_t k) { pos = pos >= k ? pos - k : 0; }
};

int copy_out(const std::string &txt, char *buf, size_t cap, size_t *len)
{
    if (!len) return -EINVAL;
    *len = txt.size();
    if (buf && cap) {
        const size_t n = cap - 1 < txt.size() ? cap - 1 : txt.size();
        std::memcpy(buf, txt.data(), n);
        buf[n] = 0;
    }
    return 0;
}

bool read_file(const char *path, std::string &out)
{
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::ostringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

}  // namespace

extern "C" {

// Writer.h:61-69 (keep the order entries < N) and :84-93 (the first K are information bits)
int polar_mask_from_order(const uint32_t *order, uint32_t count, uint32_t N, uint32_t K, uint8_t *mask_out,
                          uint32_t cap)
{
    if (!order || !mask_out || N == 0 || N > cap || K > N) return -EINVAL;
    std::vector<uint32_t> sub;
    sub.reserve(N);
    for (uint32_t i = 0; i < count; i++)
        if (order[i] < N) sub.push_back(order[i]);
    if (sub.size() != N) return -EINVAL;   // the reference reads N entries of the subset
    std::vector<uint8_t> seen(N, 0);
    for (uint32_t i = 0; i < N; i++) {
        if (seen[sub[i]]) return -EINVAL;
        seen[sub[i]] = 1;
        mask_out[sub[i]] = i < K ? 1 : 0;
    }
    return 0;
}

// The "affect" file of Writer.h:71-79: "N\n0\n0\n" then the order entries < N, each
// followed by four spaces, no final newline (the Frozen_Bit_Tab/FB_N*_K*.txt format, with
// '\n' line ends where the shipped tables carry CRLF).
int polar_write_frozen_tab(const uint32_t *order, uint32_t count, uint32_t N, char *buf, size_t cap, size_t *len)
{
    if (!order || N == 0) return -EINVAL;
    std::string t = std::to_string(N) + "\n0\n0\n";
    uint32_t k = 0;
    for (uint32_t i = 0; i < count && k < N; i++) {
        if (order[i] >= N) continue;
        t += std::to_string(order[i]) + "    ";
        k++;
    }
    if (k != N) return -EINVAL;
    return copy_out(t, buf, cap, len);
}

// polar_parameters.h exactly as Writer.h:110-162 writes it. info_mask[i] is Frozen_Bit[i]
// (1 = information). concat = En: 1 -> `const sc_bv<PAR> Frozen_Bits[N_DIVIDED]` with one
// PAR-character string per group, MSB (= the group's last bit) first; 0 -> `sc_bv<1>
// Frozen_Bits[_NBITS]` with the strings in a comment.
int polar_write_parameters_h(const uint8_t *info_mask, uint32_t N, uint32_t par, int32_t concat, char *buf,
                             size_t cap, size_t *len)
{
    if (!info_mask || !pow2(N) || !pow2(par) || par > N) return -EINVAL;
    const long NB = (long)N, P = (long)par;
    auto fb = [&](long i) { return std::string(info_mask[i] ? "1" : "0"); };
    SeekBuf o;
    o.put("#ifndef POLAR_HEADER_H\n#define POLAR_HEADER_H\n\n");
    o.put("#define _NBITS       " + std::to_string(NB) + "\n");
    o.put("#define _LOG2N       " + dbl(std::log2((double)NB)) + "\n");
    o.put("#define _DEPTH       " + dbl(std::log2((double)NB) + 1) + "\n\n");
    o.put("#define PAR          " + std::to_string(P) + "\n");
    o.put("#define LOG2_PAR     " + dbl(std::log2((double)P)) + "\n");
    o.put("#define N_DIVIDED    (_NBITS / PAR) \n");
    o.put("#define DEPTH_DIV    " + dbl(std::log2((double)(NB / P)) + 1) + "\n\n");
    o.put("#define COUNTER      sc_uint<_DEPTH>\n\n");
    if (concat) {
        o.put("const sc_bv<PAR> Frozen_Bits[N_DIVIDED] = {\n   //");
        for (long i = 0; i < NB; i++) o.put(fb(i) + ", ");
        o.put("\n     \"");
        for (long i = 0; i < NB / P; i++) {
            for (long j = 0; j < P; j++) o.put(fb((i + 1) * P - 1 - j));
            o.put("\", \"");
        }
        o.seek_back(3);
        o.put("\n};\n\n");
    } else {
        o.put("const sc_bv<1> Frozen_Bits[_NBITS] = {\n   // \"");
        for (long i = 0; i < NB / P; i++) {
            for (long j = 0; j < P; j++) o.put(fb((i + 1) * P - 1 - j));
            o.put("\", \"");
        }
        o.put("\n     ");
        for (long i = 0; i < NB; i++) o.put(fb(i) + ", ");
        o.seek_back(2);
        o.put("\n};\n\n");
    }
    o.put("\n#endif // POLAR_HEADER_H\n");
    return copy_out(o.s, buf, cap, len);
}

// Read a polar_parameters.h (either form) back: _NBITS, PAR and the frozen bits.
int polar_parse_parameters_h(const char *path, uint8_t *mask_out, uint32_t cap, uint32_t *N_out, uint32_t *par_out)
{
    if (!path || !mask_out) return -EINVAL;
    std::string txt;
    if (!read_file(path, txt)) return -ENOENT;
    auto define = [&](const char *name, long &v) {
        const std::string key = std::string("#define ") + name;
        size_t p = txt.find(key);
        if (p == std::string::npos) return false;
        p += key.size();
        if (p >= txt.size() || (txt[p] != ' ' && txt[p] != '\t')) return false;
        char *end = nullptr;
        v = std::strtol(txt.c_str() + p, &end, 10);
        return end != txt.c_str() + p;
    };
    long N = 0, P = 0;
    if (!define("_NBITS", N) || !define("PAR", P)) return -EINVAL;
    if (N <= 0 || P <= 0 || !pow2((uint64_t)N) || !pow2((uint64_t)P) || P > N || (uint64_t)N > cap) return -EINVAL;
    const size_t arr = txt.find("Frozen_Bits[");
    if (arr == std::string::npos) return -EINVAL;
    const size_t open = txt.find('{', arr), close = txt.find("};", arr);
    if (open == std::string::npos || close == std::string::npos || close < open) return -EINVAL;
    const size_t decl = txt.rfind('\n', arr);
    const std::string head = txt.substr(decl == std::string::npos ? 0 : decl, arr - (decl == std::string::npos ? 0 : decl));
    const bool concat = head.find("sc_bv<1>") == std::string::npos;   // sc_bv<PAR> form
    // the body has one commented line (starting with //) and one code line; read the code
    std::string body = txt.substr(open + 1, close - open - 1);
    std::string code;
    std::istringstream lines(body);
    for (std::string l; std::getline(lines, l);) {
        size_t q = l.find_first_not_of(" \t\r");
        if (q == std::string::npos || l.compare(q, 2, "//") == 0) continue;
        code += l;
    }
    std::vector<uint8_t> bits;
    if (concat) {
        // "b(P-1) .. b0", one string per group, MSB first
        size_t q = 0;
        while ((q = code.find('"', q)) != std::string::npos) {
            const size_t e = code.find('"', q + 1);
            if (e == std::string::npos) return -EINVAL;
            const std::string g = code.substr(q + 1, e - q - 1);
            if ((long)g.size() != P) return -EINVAL;
            for (long j = P - 1; j >= 0; j--) {
                if (g[j] != '0' && g[j] != '1') return -EINVAL;
                bits.push_back((uint8_t)(g[j] - '0'));
            }
            q = e + 1;
        }
    } else {
        for (char c : code) {
            if (c == '0' || c == '1') bits.push_back((uint8_t)(c - '0'));
            else if (!(c == ',' || c == ' ' || c == '\t' || c == '\r')) return -EINVAL;
        }
    }
    if ((long)bits.size() != N) return -EINVAL;
    std::memcpy(mask_out, bits.data(), bits.size());
    if (N_out) *N_out = (uint32_t)N;
    if (par_out) *par_out = (uint32_t)P;
    return 0;
}

}  // extern "C"
