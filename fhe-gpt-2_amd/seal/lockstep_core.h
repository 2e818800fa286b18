// The round logic of seal::Lockstep (seal.cpp), kept free of HIP and of the evaluator so the CPU
// tests can drive it from many threads under ThreadSanitizer / AddressSanitizer
// (tests/cpp/lockstep_test.cpp, tests/test_stream_order.py).
//
// `active` member threads each submit one request per round; the last one to arrive takes the
// round's requests and runs them (outside the lock) as one merged call, then bumps the round and
// wakes the others, which return only after their request ran.  A member that leaves lowers
// `active`; if everyone still active has already arrived, the leaver runs the round for them.
#pragma once
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <vector>

namespace seal
{
namespace detail
{
template <class Req>
class LockstepCore
{
public:
    explicit LockstepCore(std::size_t members) : active_(members) {}

    // Submit `r` for the current round and return once the round that holds it has run.
    // exec(std::vector<Req *> &batch) runs on whichever thread completes the round.
    template <class Exec>
    void submit(Req *r, Exec &&exec)
    {
        std::unique_lock<std::mutex> lk(mu_);
        const std::uint64_t my_round = round_;
        reqs_.push_back(r);
        if (++arrived_ >= active_)
            run_round(lk, exec);
        else
            cv_.wait(lk, [&] { return round_ != my_round; });
    }

    // The calling member stops taking part; a round everyone else already joined runs now.
    template <class Exec>
    void leave(Exec &&exec)
    {
        std::unique_lock<std::mutex> lk(mu_);
        if (active_) active_--;
        if (arrived_ > 0 && arrived_ >= active_) run_round(lk, exec);
    }

    std::size_t rounds() const
    {
        std::lock_guard<std::mutex> g(mu_);
        return rounds_run_;
    }
    std::size_t merged() const
    {
        std::lock_guard<std::mutex> g(mu_);
        return merged_;
    }

private:
    template <class Exec>
    void run_round(std::unique_lock<std::mutex> &lk, Exec &exec)
    {
        std::vector<Req *> batch;
        batch.swap(reqs_);
        // late submitters of the next round block on mu_ until the round number moves on
        lk.unlock();
        exec(batch);
        lk.lock();
        arrived_ = 0;
        round_++;
        rounds_run_++;
        if (batch.size() > 1) merged_ += batch.size();
        cv_.notify_all();
    }

    mutable std::mutex mu_;
    std::condition_variable cv_;
    std::size_t active_;
    std::size_t arrived_ = 0;
    std::uint64_t round_ = 0;
    std::size_t rounds_run_ = 0, merged_ = 0;
    std::vector<Req *> reqs_;
};
} // namespace detail
} // namespace seal
