// CPU unit test of PolyStore's cross-stream ordering rule (fhe-gpt-2_amd/seal/stream_order.h): a
// small model of streams, buffers and the engine's caching allocator runs access sequences and
// checks that no block is handed out again while a stream that touched it may still be running.
#include <cassert>
#include <cstdio>
#include <map>
#include <set>
#include <vector>

#include "../../fhe-gpt-2_amd/seal/stream_order.h"

using seal::detail::Access;
using seal::detail::order_before;

static int fails = 0;
#define CHECK(c)                                                                                  \
    do                                                                                            \
    {                                                                                             \
        if (!(c))                                                                                 \
        {                                                                                         \
            std::printf("FAIL line %d: %s\n", __LINE__, #c);                                     \
            fails++;                                                                              \
        }                                                                                         \
    } while (0)

// Model: every stream runs its queue in order; "covers(a, b)" = all work enqueued on b so far is
// ordered before the next work on a (a waited on b, transitively).
struct Model
{
    std::map<int, std::set<int>> after; // stream -> streams it has waited on (transitively)
    void wait(int a, int b)
    {
        if (a == b) return;
        after[a].insert(b);
        for (int x : after[b]) after[a].insert(x);
    }
    bool covers(int a, int b) { return a == b || after[a].count(b); }
};

int main()
{
    // the rule itself
    {
        auto w = order_before<int>(1, 0, true, {}, Access::read);
        CHECK(w.empty());
        w = order_before<int>(1, 2, false, {}, Access::read);
        CHECK(w == std::vector<int>({ 2 }));
        w = order_before<int>(2, 2, false, { 3, 4 }, Access::read);
        CHECK(w.empty());
        w = order_before<int>(1, 2, false, { 3, 1, 4 }, Access::write);
        CHECK(w == std::vector<int>({ 2, 3, 4 }));
        w = order_before<int>(2, 2, false, { 3, 4, 3 }, Access::release);
        CHECK(w == std::vector<int>({ 3, 4 }));
        w = order_before<int>(1, 2, true, { 2, 5 }, Access::release);
        CHECK(w == std::vector<int>({ 2, 5 }));
    }
    // a buffer written on stream 1, read on streams 2 and 3, freed on its writer's stream, then
    // reused by an allocation on stream 1 (no wait: same stream) and on stream 4 (waits on the
    // free's event): in both cases the readers must be covered.
    for (int reuse_on : { 1, 4 })
    {
        Model m;
        const int writer = 1;
        std::vector<int> readers;
        for (int r : { 2, 3 })
        {
            for (int x : order_before<int>(r, writer, false, {}, Access::read)) m.wait(r, x);
            readers.push_back(r);
        }
        CHECK(m.covers(2, 1) && m.covers(3, 1)); // readers saw the write
        const int s = writer;                    // release() frees on the writer's stream
        for (int x : order_before<int>(s, writer, false, readers, Access::release)) m.wait(s, x);
        // allocator: same stream -> stream order; other stream -> waits on an event recorded on s
        if (reuse_on != s) m.wait(reuse_on, s);
        CHECK(m.covers(reuse_on, 2) && m.covers(reuse_on, 3));
        // without the rule (free ordered on s alone) the readers would not be covered
        Model bare;
        if (reuse_on != s) bare.wait(reuse_on, s);
        CHECK(!bare.covers(reuse_on, 2));
    }
    // a write on stream 5 after reads on 2 and 3 and a write on 1 waits for all of them
    {
        Model m;
        for (int x : order_before<int>(5, 1, false, { 2, 3 }, Access::write)) m.wait(5, x);
        CHECK(m.covers(5, 1) && m.covers(5, 2) && m.covers(5, 3));
    }
    std::printf(fails ? "FAILED %d\n" : "ALL PASSED\n", fails);
    return fails ? 1 : 0;
}
