// trace.cpp -- evaluator operation trace (see trace.h).
#include "trace.h"

#include "seal/seal.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <set>
#include <sstream>

namespace seal
{
namespace trace
{
namespace
{
std::mutex g_mu;
std::set<std::string> g_written;
thread_local int t_depth = 0;

const char *dir()
{
    static const char *d = std::getenv("MHE_EVAL_TRACE");
    return (d && d[0]) ? d : nullptr;
}

std::uint64_t fnv(const void *p, std::size_t bytes, std::uint64_t h = 0xcbf29ce484222325ull)
{
    const unsigned char *b = static_cast<const unsigned char *>(p);
    for (std::size_t i = 0; i < bytes; i++)
    {
        h ^= b[i];
        h *= 0x100000001b3ull;
    }
    return h;
}

std::string hex(std::uint64_t v)
{
    char buf[20];
    std::snprintf(buf, sizeof buf, "%016llx", (unsigned long long)v);
    return buf;
}

// <kind>_<id>.bin: header of u64 words then the payload
void put(const std::string &name, const std::uint64_t *hdr, std::size_t hwords, const void *payload,
         std::size_t bytes)
{
    std::lock_guard<std::mutex> g(g_mu);
    if (!g_written.insert(name).second) return;
    std::ofstream f(std::string(dir()) + "/" + name + ".bin", std::ios::binary);
    f.write(reinterpret_cast<const char *>(hdr), (std::streamsize)(hwords * 8));
    f.write(static_cast<const char *>(payload), (std::streamsize)bytes);
}
} // namespace

bool enabled()
{
    return dir() != nullptr;
}

Scope::Scope() : top_(enabled() && t_depth == 0)
{
    t_depth++;
}

Scope::~Scope()
{
    t_depth--;
}

std::string num(double v)
{
    char buf[40];
    std::snprintf(buf, sizeof buf, "%.17g", v);
    return buf;
}

std::string ct(const Ciphertext &c)
{
    // header: size, limbs, n, scale bits, ntt flag
    const std::uint64_t *w = c.data();
    const std::size_t words = c.size() * c.coeff_modulus_size() * c.poly_modulus_degree();
    double sc = c.scale();
    std::uint64_t sb;
    std::memcpy(&sb, &sc, 8);
    const std::uint64_t hdr[5] = { c.size(), c.coeff_modulus_size(), c.poly_modulus_degree(), sb,
                                   c.is_ntt_form() ? 1u : 0u };
    const std::string id = "c" + hex(fnv(w, words * 8, fnv(hdr, sizeof hdr)));
    put(id, hdr, 5, w, words * 8);
    return id;
}

std::string pt(const Plaintext &p)
{
    // header: limbs, words, scale bits
    const std::uint64_t *w = p.data();
    double sc = p.scale();
    std::uint64_t sb;
    std::memcpy(&sb, &sc, 8);
    const std::uint64_t hdr[3] = { p.limbs(), p.coeff_count(), sb };
    const std::string id = "p" + hex(fnv(w, p.coeff_count() * 8, fnv(hdr, sizeof hdr)));
    put(id, hdr, 3, w, p.coeff_count() * 8);
    return id;
}

std::string vec(const double *re, const double *im, std::size_t n)
{
    // header: count, complex flag; payload re[n] then im[n]
    std::vector<double> v(re, re + n);
    if (im) v.insert(v.end(), im, im + n);
    const std::uint64_t hdr[2] = { n, im ? 1u : 0u };
    const std::string id = "v" + hex(fnv(v.data(), v.size() * 8, fnv(hdr, sizeof hdr)));
    put(id, hdr, 2, v.data(), v.size() * 8);
    return id;
}

void record(const char *op, const std::vector<std::string> &in, const std::string &out, const std::string &extra)
{
    std::ostringstream s;
    s << "{\"op\": \"" << op << "\", \"in\": [";
    bool first = true;
    for (const auto &i : in)
    {
        s << (first ? "" : ", ") << '"' << i << '"';
        first = false;
    }
    s << "], \"out\": \"" << out << '"';
    if (!extra.empty()) s << ", " << extra;
    s << "}\n";
    std::lock_guard<std::mutex> g(g_mu);
    std::ofstream f(std::string(dir()) + "/trace.jsonl", std::ios::app);
    f << s.str();
}
} // namespace trace
} // namespace seal
