// trace.h -- evaluator operation trace (internal to libmhe_seal.so).
//
// With MHE_EVAL_TRACE=<dir> set, every top-level seal::Evaluator / CKKSEncoder / Encryptor
// operation appends one JSON line to <dir>/trace.jsonl naming the operation, its arguments and
// the content ids of the ciphertexts / plaintexts / vectors it read and wrote; every object is
// written once to <dir>/<kind>_<id>.bin (content-addressed).  Operations called from inside a
// traced operation are not recorded (a thread-local depth), so a reduced-error add is one record.
// The checker (tests/trace_replay.py, test infrastructure) replays the records through the CPU
// oracle and compares every output word and scale.  Off (a single branch per operation) unless set.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace seal
{
class Ciphertext;
class Plaintext;

namespace trace
{
bool enabled();

// depth guard: top() is true for the outermost traced operation of this thread
class Scope
{
public:
    Scope();
    ~Scope();
    bool top() const { return top_; }

private:
    bool top_;
};

std::string ct(const Ciphertext &c);                                  // "c<id>"
std::string pt(const Plaintext &p);                                   // "p<id>"
std::string vec(const double *re, const double *im, std::size_t n);   // "v<id>"
std::string num(double v);                                            // exact decimal

// one record: op name, "in" ids, "out" id (may be empty), extra JSON members ("\"k\": v, ...")
void record(const char *op, const std::vector<std::string> &in, const std::string &out, const std::string &extra = "");
} // namespace trace
} // namespace seal
