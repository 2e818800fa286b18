// The batched (not SEAL API) evaluator entry points against their one-by-one counterparts, word for
// word and scale for scale: rotate_vectors (keyed steps, NAF-composed steps, step 0, mixed levels),
// rescale_to_next_inplace_many, relinearize_inplace_many and multiply_reduced_error_many (equal
// levels, and unequal levels where the reduced-error adjustment runs).  N = 2^13 and 2^16.
//   seal_batch_test <log N>
#include "seal/seal.h"
#include "../../include/mhe.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>

using namespace seal;

static int g_fail = 0;
static bool same(const Ciphertext &a, const Ciphertext &b)
{
    if (a.size() != b.size() || a.coeff_modulus_size() != b.coeff_modulus_size() || a.scale() != b.scale() ||
        a.parms_id() != b.parms_id())
        return false;
    const PolyStore &x = a.store(), &y = b.store();
    return x.words() == y.words() && std::memcmp(x.host(), y.host(), x.words() * 8) == 0;
}
static void check(const std::string &what, bool ok)
{
    std::printf("[%s] %s\n", ok ? "PASS" : "FAIL", what.c_str());
    if (!ok) g_fail++;
}

int main(int argc, char **argv)
{
    const int logN = argc > 1 ? std::atoi(argv[1]) : 13;
    const std::size_t N = (std::size_t)1 << logN;
    std::vector<int> bits{ 51 };
    for (int i = 0; i < 6; i++) bits.push_back(46);
    bits.push_back(51);
    EncryptionParameters parms(scheme_type::ckks);
    parms.set_poly_modulus_degree(N);
    parms.set_coeff_modulus(CoeffModulus::Create(N, bits));
    parms.set_random_generator(
        std::make_shared<Blake2xbPRNGFactory>(std::array<std::uint64_t, 8>{ 3, 1, 4, 1, 5, 9, 2, 6 }));
    SEALContext ctx(parms, true, sec_level_type::none);
    KeyGenerator keygen(ctx);
    PublicKey pk;
    keygen.create_public_key(pk);
    RelinKeys rlk;
    keygen.create_relin_keys(rlk);
    const int slots = (int)N / 2;
    // +-2^i for i < 5: steps 3, 5 and -7 below have no key of their own (SEAL's NAF path)
    std::vector<int> steps;
    for (int i = 0; i < 5; i++)
    {
        steps.push_back(1 << i);
        steps.push_back(slots - (1 << i));
    }
    GaloisKeys glk;
    keygen.create_galois_keys(steps, glk);
    CKKSEncoder encoder(ctx);
    Encryptor encryptor(ctx, pk);
    Evaluator ev(ctx, encoder);
    const double scale = std::pow(2.0, 46);
    std::mt19937_64 g(11);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    auto fresh = [&](int drop) {
        std::vector<double> v(slots);
        for (auto &x : v) x = U(g);
        Plaintext p;
        Ciphertext c;
        encoder.encode(v, scale, p);
        encryptor.encrypt(p, c);
        for (int i = 0; i < drop; i++) ev.mod_switch_to_next_inplace(c);
        return c;
    };
    try
    {
        // rotate_vectors: 11 entries over two levels, keyed, NAF (3, 5, -7) and zero steps
        std::vector<Ciphertext> in;
        std::vector<int> st{ 1, 3, 0, 16, slots - 1, 5, 2, -7, 4, 8, 1 };
        for (std::size_t i = 0; i < st.size(); i++) in.push_back(fresh(i % 3 == 2 ? 1 : 0));
        std::vector<Ciphertext> out(st.size()), want(st.size());
        std::vector<const Ciphertext *> pin;
        std::vector<Ciphertext *> pout;
        for (std::size_t i = 0; i < st.size(); i++)
        {
            pin.push_back(&in[i % 4 == 3 ? 0 : i]); // some entries share an input
            pout.push_back(&out[i]);
        }
        ev.rotate_vectors(pin, st, glk, pout);
        bool ok = true;
        for (std::size_t i = 0; i < st.size(); i++)
        {
            ev.rotate_vector(*pin[i], st[i], glk, want[i]);
            ok = ok && same(out[i], want[i]);
        }
        check("rotate_vectors == rotate_vector (11 entries, 2 levels, keyed / NAF / zero steps)", ok);

        // rescale_to_next_inplace_many on products (size 3 and relinearized size 2), two levels
        std::vector<Ciphertext> r1, r2;
        for (int i = 0; i < 10; i++)
        {
            Ciphertext a = fresh(i % 2), b = fresh(i % 2), m;
            ev.multiply(a, b, m);
            if (i % 3) ev.relinearize_inplace(m, rlk);
            r1.push_back(m);
        }
        r2 = r1;
        std::vector<Ciphertext *> pr;
        for (auto &c : r1) pr.push_back(&c);
        ev.rescale_to_next_inplace_many(pr);
        ok = true;
        for (std::size_t i = 0; i < r2.size(); i++)
        {
            ev.rescale_to_next_inplace(r2[i]);
            ok = ok && same(r1[i], r2[i]);
        }
        check("rescale_to_next_inplace_many == rescale_to_next_inplace (10 entries, sizes 2 / 3, 2 levels)", ok);

        // relinearize_inplace_many: 9 size-3 entries over three levels and one size-2 entry
        std::vector<Ciphertext> l1, l2;
        for (int i = 0; i < 10; i++)
        {
            Ciphertext a = fresh(i % 3), b = fresh(i % 3), m;
            ev.multiply(a, b, m);
            if (i == 9) ev.relinearize_inplace(m, rlk);
            l1.push_back(m);
        }
        l2 = l1;
        std::vector<Ciphertext *> pl;
        for (auto &c : l1) pl.push_back(&c);
        ev.relinearize_inplace_many(pl, rlk);
        ok = true;
        for (std::size_t i = 0; i < l2.size(); i++)
        {
            ev.relinearize_inplace(l2[i], rlk);
            ok = ok && same(l1[i], l2[i]);
        }
        check("relinearize_inplace_many == relinearize_inplace (10 entries, 3 levels, one already size 2)", ok);

        // multiply_reduced_error_many: equal levels and both unequal orders
        std::vector<Ciphertext> A, B, M(12), W(12);
        for (int i = 0; i < 12; i++)
        {
            A.push_back(fresh(i % 4 == 1 ? 1 : 0));
            B.push_back(fresh(i % 4 == 2 ? 2 : 0));
        }
        std::vector<const Ciphertext *> pa, pb;
        std::vector<Ciphertext *> pm;
        for (int i = 0; i < 12; i++)
        {
            pa.push_back(&A[i]);
            pb.push_back(&B[i % 5 == 4 ? 0 : i]);
            pm.push_back(&M[i]);
        }
        ev.multiply_reduced_error_many(pa, pb, rlk, pm);
        ok = true;
        for (int i = 0; i < 12; i++)
        {
            ev.multiply_reduced_error(*pa[i], *pb[i], rlk, W[i]);
            ok = ok && same(M[i], W[i]);
        }
        check("multiply_reduced_error_many == multiply_reduced_error (12 entries, equal and unequal levels)", ok);

        // Lockstep group: 4 threads run one operation sequence on their own inputs; the group
        // merges their rotations, relinearizations, reduced-error products and rescales into
        // batched launches.  Every result equals the sequence run alone, including a member with
        // an extra operation (misaligned rounds) and one that leaves after half the sequence.
        {
            constexpr int M = 4;
            std::vector<Ciphertext> x0, y0;
            for (int m = 0; m < M; m++)
            {
                x0.push_back(fresh(0));
                y0.push_back(fresh(0));
            }
            auto sequence = [&](int m, std::vector<Ciphertext> &res) {
                Ciphertext x = x0[m], y = y0[m], r1, r2, t;
                ev.rotate_vector(x, 1, glk, r1);                 // keyed
                ev.rotate_vector_inplace(y, 3, glk);             // NAF-composed
                std::vector<Ciphertext> rr(2);
                ev.rotate_vectors({ &x, &y }, { 2, slots - 1 }, glk, { &rr[0], &rr[1] });
                ev.multiply_reduced_error(r1, rr[0], rlk, t);    // product + relinearization
                ev.rescale_to_next_inplace(t);
                if (m == 1) ev.rotate_vector_inplace(t, 4, glk); // misaligns this member's rounds
                ev.multiply_inplace_reduced_error(y, rr[1], rlk);
                ev.rescale_to_next_inplace(y);
                res = { r1, y, rr[0], rr[1], t };
                if (m == 3) return;                              // leaves early
                Ciphertext sq;
                ev.square(t, sq);
                ev.relinearize_inplace(sq, rlk);
                ev.rescale_to_next_inplace(sq);
                ev.rotate_vector_inplace(sq, slots - 16, glk);
                res.push_back(sq);
            };
            std::vector<std::vector<Ciphertext>> alone(M), grouped(M);
            for (int m = 0; m < M; m++) sequence(m, alone[m]);
            Lockstep group(M);
            {
                std::vector<std::thread> th;
                for (int m = 0; m < M; m++)
                    th.emplace_back([&, m] {
                        Lockstep::Member member(group);
                        sequence(m, grouped[m]);
                    });
                for (auto &t : th) t.join();
            }
            bool ok = true;
            for (int m = 0; m < M; m++)
            {
                ok = ok && alone[m].size() == grouped[m].size();
                for (std::size_t i = 0; ok && i < alone[m].size(); i++) ok = same(alone[m][i], grouped[m][i]);
            }
            std::printf("lockstep: %zu rounds, %zu member calls merged\n", group.rounds(), group.merged_calls());
            check("Lockstep group (4 threads; rotations, relinearizations, products, rescales merged) == each alone",
                  ok && group.merged_calls() > 0);

            // the same members as a FiberBatch on this thread (one stream, no thread wake-ups),
            // including a fiber that throws half way: the others finish with the same words and the
            // error comes back from run()
            std::vector<std::vector<Ciphertext>> fibered(M);
            FiberBatch::run(M, [&](std::size_t m) { sequence((int)m, fibered[m]); });
            ok = true;
            for (int m = 0; m < M; m++)
            {
                ok = ok && alone[m].size() == fibered[m].size();
                for (std::size_t i = 0; ok && i < alone[m].size(); i++) ok = same(alone[m][i], fibered[m][i]);
            }
            std::printf("fibers: %zu rounds, %zu member calls merged\n", FiberBatch::last_rounds(),
                        FiberBatch::last_merged());
            check("FiberBatch (4 fibers on one thread; the same merges) == each alone", ok && FiberBatch::last_merged() > 0);
            std::vector<std::vector<Ciphertext>> part(M);
            bool fb_threw = false;
            try
            {
                FiberBatch::run(M, [&](std::size_t m) {
                    if (m == 2)
                    {
                        Ciphertext x = x0[m], r;
                        ev.rotate_vector(x, 1, glk, r);
                        throw std::runtime_error("fiber 2 fails");
                    }
                    sequence((int)m, part[m]);
                });
            }
            catch (const std::runtime_error &e)
            {
                fb_threw = std::string(e.what()) == "fiber 2 fails";
            }
            ok = fb_threw;
            for (int m = 0; m < M; m++)
                if (m != 2)
                    for (std::size_t i = 0; ok && i < alone[m].size(); i++) ok = same(alone[m][i], part[m][i]);
            check("FiberBatch: a fiber's exception comes back from run(), the other fibers' words unchanged", ok);
        }

        // An allocation that fails part way through a batched rescale (injected: the engine's nth
        // next device allocation reports out of memory).  Alone, the call must throw with every entry
        // unchanged; merged in a FiberBatch round, lockstep_execute re-runs each member's call on its
        // own, so every member must end up rescaled exactly once -- a group committed before the
        // failure and rescaled again by the retry is a silently wrong ciphertext (two levels down).
        {
            auto two_groups = [&](std::vector<Ciphertext> &v) {
                v.clear();
                for (int i = 0; i < 6; i++)
                {
                    Ciphertext a = fresh(i < 3 ? 1 : 0), b = fresh(i < 3 ? 1 : 0), m;
                    ev.multiply(a, b, m);
                    ev.relinearize_inplace(m, rlk);
                    v.push_back(m);
                }
            };
            std::vector<Ciphertext> base, want;
            two_groups(base);
            want = base;
            for (auto &c : want) ev.rescale_to_next_inplace(c);
            bool ok_alone = true, ok_fiber = true;
            int threw_alone = 0, retried = 0;
            // the fallbacks and failed allocations must be counted, not silent
            const std::uint64_t fb0 = merged_call_fallbacks();
            std::uint64_t ar0 = 0, af0 = 0;
            mhe_alloc_stats(&ar0, &af0, 0);
            for (int nth = 1; nth <= 10; nth++)
            {
                std::vector<Ciphertext> v = base;
                std::vector<Ciphertext *> pv;
                for (auto &c : v) pv.push_back(&c);
                mhe_debug_fail_alloc(ctx.engine(), nth);
                bool thrown = false;
                try
                {
                    ev.rescale_to_next_inplace_many(pv);
                }
                catch (const std::runtime_error &)
                {
                    thrown = true;
                }
                mhe_debug_fail_alloc(ctx.engine(), 0);
                threw_alone += thrown ? 1 : 0;
                for (std::size_t i = 0; i < v.size(); i++) ok_alone = ok_alone && same(v[i], thrown ? base[i] : want[i]);
                // two fibers rescaling one entry per round (rescale_to_next_inplace is a merge point):
                // fiber 0 the lower-level f[0..2], fiber 1 the top-level f[3..5], so every merged call
                // holds two (level, size) groups and a failure in the second finds the first done
                std::vector<Ciphertext> f = base;
                mhe_debug_fail_alloc(ctx.engine(), nth);
                try
                {
                    FiberBatch::run(2, [&](std::size_t m) {
                        for (int r = 0; r < 3; r++) ev.rescale_to_next_inplace(f[3 * m + r]);
                    });
                }
                catch (const std::exception &e)
                {
                    std::printf("  nth %d: FiberBatch threw: %s\n", nth, e.what());
                    ok_fiber = false;
                }
                const bool fired = nth <= 6; // 6 allocations: one per entry, two per merged round
                mhe_debug_fail_alloc(ctx.engine(), 0);
                retried += fired ? 1 : 0;
                for (std::size_t i = 0; i < f.size(); i++) ok_fiber = ok_fiber && same(f[i], want[i]);
            }
            check("rescale_to_next_inplace_many: an allocation failure part way leaves every entry unchanged (" +
                      std::to_string(threw_alone) + " of 10 injection points threw)",
                  ok_alone && threw_alone > 0);
            check("FiberBatch: a merged rescale that fails part way is re-run per member, each entry rescaled once (" +
                      std::to_string(retried) + " failing merged calls)",
                  ok_fiber && retried > 0);
            std::uint64_t ar1 = 0, af1 = 0;
            mhe_alloc_stats(&ar1, &af1, 0);
            const std::uint64_t fb = merged_call_fallbacks() - fb0, af = af1 - af0;
            check("the merged-call fallbacks (" + std::to_string(fb) + ") and failed allocations (" + std::to_string(af) +
                      ") are counted: at least one per failing merged call / injected failure",
                  fb >= (std::uint64_t)retried && af >= (std::uint64_t)(retried + threw_alone));
        }

        // A merged relinearization of more than 8 entries (10 fibers, one relinearize_inplace each)
        // runs as two engine chunks of in-place key switches.  When the second chunk fails
        // (injected), lockstep_execute re-runs each member alone: the first chunk's entries are
        // already relinearized (size 2) and must not be switched a second time.
        {
            const int F = 10;
            std::vector<Ciphertext> base(F), want(F);
            for (int i = 0; i < F; i++)
            {
                Ciphertext a = fresh(1), b = fresh(1);
                ev.multiply(a, b, base[i]);
                want[i] = base[i];
                ev.relinearize_inplace(want[i], rlk);
            }
            const std::uint64_t fb0 = merged_call_fallbacks();
            std::vector<Ciphertext> f = base;
            mhe_debug_fail_switch(ctx.engine(), 2);
            bool ok = true;
            try
            {
                FiberBatch::run(F, [&](std::size_t m) { ev.relinearize_inplace(f[m], rlk); });
            }
            catch (const std::exception &e)
            {
                std::printf("  FiberBatch threw: %s\n", e.what());
                ok = false;
            }
            mhe_debug_fail_switch(ctx.engine(), 0);
            for (int i = 0; i < F; i++) ok = ok && same(f[i], want[i]);
            const std::uint64_t fb = merged_call_fallbacks() - fb0;
            check("FiberBatch: a 10-entry merged relinearization whose second chunk fails is re-run per member, "
                  "each entry switched once (" + std::to_string(fb) + " fallback)",
                  ok && fb == 1);
        }

        bool threw = false;
        try
        {
            std::vector<Ciphertext *> bad{ &M[0], &M[0] };
            ev.multiply_reduced_error_many({ &A[0], &A[1] }, { &B[0], &B[1] }, rlk, bad);
        }
        catch (const std::invalid_argument &)
        {
            threw = true;
        }
        check("multiply_reduced_error_many rejects repeated destinations", threw);
    }
    catch (const std::exception &e)
    {
        std::printf("exception: %s\nFAILED\n", e.what());
        return 1;
    }
    std::printf(g_fail ? "FAILED (%d)\n" : "ALL PASSED\n", g_fail);
    return g_fail ? 1 : 0;
}
