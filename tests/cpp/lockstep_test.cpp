// CPU unit test of seal::Lockstep's round logic (fhe-gpt-2_amd/seal/lockstep_core.h) with stubbed
// launches, built plain and under -fsanitize=thread and -fsanitize=address (tests/test_stream_order.py).
// Member threads submit sequences of stub operations; the merged "launch" records which members'
// requests ran together.  Checks: every request runs exactly once, in its member's program order,
// in a round with the same-numbered request of every member still active; members that leave early
// (shorter sequences) never stall the others; rounds and merged counts add up.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "../../fhe-gpt-2_amd/seal/lockstep_core.h"

struct Req
{
    int member, seq;
    int ran_in_round = -1;
    int round_size = 0;
};

static int fails = 0;
#define CHECK(c)                                                 \
    do                                                           \
    {                                                            \
        if (!(c))                                                \
        {                                                        \
            std::printf("FAIL line %d: %s\n", __LINE__, #c);    \
            fails++;                                             \
        }                                                        \
    } while (0)

static void run(int members, const std::vector<int> &lengths, int spin)
{
    seal::detail::LockstepCore<Req> core((std::size_t)members);
    std::vector<std::vector<Req>> reqs(members);
    for (int m = 0; m < members; m++)
        for (int k = 0; k < lengths[m]; k++) reqs[m].push_back(Req{ m, k });
    std::atomic<int> round_no{ 0 };
    std::mutex log_mu;
    std::vector<std::vector<std::pair<int, int>>> rounds; // (member, seq) per executed round
    auto exec = [&](std::vector<Req *> &batch) {
        const int r = round_no.fetch_add(1);
        std::vector<std::pair<int, int>> got;
        for (Req *q : batch)
        {
            q->ran_in_round = r; // written by the executing thread, read by the owner after submit returns
            q->round_size = (int)batch.size();
            got.push_back({ q->member, q->seq });
        }
        volatile int x = 0;
        for (int i = 0; i < spin; i++) x = x + i; // a stub launch that takes a while
        std::lock_guard<std::mutex> g(log_mu);
        rounds.push_back(got);
    };
    std::vector<std::thread> th;
    std::vector<int> seen_order_ok(members, 1);
    for (int m = 0; m < members; m++)
        th.emplace_back([&, m] {
            int last_round = -1;
            for (Req &q : reqs[m])
            {
                core.submit(&q, exec);
                // the request ran before submit returned, after the member's previous request
                if (q.ran_in_round <= last_round) seen_order_ok[m] = 0;
                last_round = q.ran_in_round;
            }
            core.leave(exec);
        });
    for (auto &t : th) t.join();
    for (int m = 0; m < members; m++)
    {
        CHECK(seen_order_ok[m]);
        for (const Req &q : reqs[m]) CHECK(q.ran_in_round >= 0);
    }
    // every round holds the k-th request of each member whose sequence is longer than k
    std::map<int, int> per_seq;
    int total = 0;
    for (const auto &r : rounds)
    {
        if (r.empty()) continue;
        const int k = r[0].second;
        int expect = 0;
        for (int m = 0; m < members; m++) expect += lengths[m] > k;
        CHECK((int)r.size() == expect);
        for (const auto &p : r) CHECK(p.second == k);
        per_seq[k]++;
        total += (int)r.size();
    }
    int want_total = 0;
    for (int l : lengths) want_total += l;
    CHECK(total == want_total);
    CHECK(core.rounds() == rounds.size());
    for (const auto &kv : per_seq) CHECK(kv.second == 1);
}

int main()
{
    run(4, { 50, 50, 50, 50 }, 0);
    run(4, { 50, 20, 50, 5 }, 100);   // members leave early
    run(8, { 7, 1, 30, 30, 0, 12, 30, 2 }, 10);
    run(1, { 20 }, 0);
    for (int rep = 0; rep < 20; rep++) run(3, { 10 + rep, 10, 3 + rep % 4 }, rep);
    std::printf(fails ? "FAILED (%d)\n" : "ALL PASSED\n", fails);
    return fails ? 1 : 0;
}
