// The cross-stream ordering rule of PolyStore (seal.cpp), kept free of HIP so the CPU tests can
// check it (tests/cpp/stream_order_test.cpp).
//
// A device buffer has a last writer stream (nullptr: none; writer_done: known complete on the
// host) and the set of streams that read it since that write.  Before an access on stream s,
// s waits (device-side: event record + stream wait) on
//   read:            the writer, unless it is s or done;
//   write / release: the writer as above and every reader other than s.
// release = the buffer goes back to the engine's allocator on s: the allocator orders reuse after
// s (same stream) or after an event recorded on s (other streams), so every other stream that
// touched the buffer must be ordered before s first.  Before this rule the free waited only on s,
// and a block still read by another thread's stream could be handed out again on s.
#pragma once
#include <algorithm>
#include <vector>

namespace seal
{
namespace detail
{
enum class Access
{
    read,
    write,
    release
};

template <class S>
std::vector<S> order_before(S s, S writer, bool writer_done, const std::vector<S> &readers, Access a)
{
    std::vector<S> w;
    if (writer && writer != s && !writer_done) w.push_back(writer);
    if (a != Access::read)
        for (S r : readers)
            if (r && r != s && std::find(w.begin(), w.end(), r) == w.end()) w.push_back(r);
    return w;
}
} // namespace detail
} // namespace seal
