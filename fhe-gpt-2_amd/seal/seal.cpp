// seal.cpp -- the SEAL-3.6-compatible C++ surface (include/seal/seal.h) over the C ABI of
// include/mhe.h.  Host code only: every polynomial operation is one or a few libmhe calls on
// the calling thread's HIP stream; this file owns the bookkeeping SEAL keeps around them
// (parms_id chain, scales, sizes, argument checks and their exception messages).
//
// Reference behaviour followed (modified SEAL 3.6.6 under
// gpt2_ckks/gpt2-ckks/single-key/seal-modified-3.6.6/native/src/seal/):
//   context.cpp (modulus switching chain), ciphertext.h, plaintext.h, keygenerator.cpp,
//   encryptor.cpp:88-166, decryptor.cpp (ckks_decrypt), ckks.h/ckks.cpp (CKKSEncoder),
//   evaluator.cpp (all Evaluator entry points; line numbers cited per method).
#include "lockstep_core.h"
#include "stream_order.h"
#include "seal/seal.h"

#include "../../include/mhe.h"
#include "random_internal.h"
#include "trace.h"

#include <algorithm>
#include <cmath>
#include <atomic>
#include <condition_variable>
#include <exception>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <thread>
#include <unordered_map>

#include <csignal>
#include <sys/mman.h>
#include <ucontext.h>
#include <unistd.h>

namespace seal
{
namespace
{
// One traced operation (trace.h): the input ids are taken at entry, the output id at a normal exit;
// nested operations (depth > 0) and operations that throw leave no record.
template <class F>
class TraceOp
{
public:
    TraceOp(const char *op, F out) : op_(op), out_(out), unc_(std::uncaught_exceptions()) {}
    bool top() const { return sc_.top(); }
    void in(std::initializer_list<std::string> v) { in_.assign(v.begin(), v.end()); }
    std::string extra;
    ~TraceOp()
    {
        if (!sc_.top() || std::uncaught_exceptions() != unc_) return;
        try
        {
            trace::record(op_, in_, out_(), extra);
        }
        catch (...)
        {
        }
    }

private:
    trace::Scope sc_;
    const char *op_;
    F out_;
    std::vector<std::string> in_;
    int unc_;
};
} // namespace
#define TRACE_OP(NAME, OUT, ...)                                                   \
    TraceOp trace_op_(NAME, [&]() -> std::string { return OUT; });             \
    if (trace_op_.top()) trace_op_.in({ __VA_ARGS__ })
#define TRACE_EXTRA(S) \
    if (trace_op_.top()) trace_op_.extra = (S)

const parms_id_type parms_id_zero = { 0, 0, 0, 0 };

struct LsOp
{
    enum Kind
    {
        ROT,
        RESC,
        RELIN,
        MULRE
    } kind = ROT;
    std::vector<const Ciphertext *> in, in2;
    std::vector<int> steps;
    std::vector<Ciphertext *> out;
    const GaloisKeys *gk = nullptr;
    const RelinKeys *rk = nullptr;
    const Evaluator *ev = nullptr;
    std::exception_ptr err;
};

namespace
{
thread_local Lockstep::Impl *tl_ls = nullptr;        // the calling thread's group, while merging
thread_local Lockstep::Impl *tl_ls_member = nullptr; // the group the thread is a member of
thread_local int tl_ls_direct = 0;            // > 0 inside a round's execution: calls run directly
thread_local FiberBatch::Impl *tl_fb = nullptr; // the FiberBatch running on this thread
bool fiber_merging(); // inside a FiberBatch fiber (defined with FiberBatch::Impl)
struct LsDirect
{
    LsDirect() { ++tl_ls_direct; }
    ~LsDirect() { --tl_ls_direct; }
};
} // namespace



namespace
{
[[noreturn]] void raise(int rc)
{
    const std::string msg = mhe_last_error();
    switch (rc)
    {
    case MHE_ERR_ARG: throw std::invalid_argument(msg);
    case MHE_ERR_RANGE:
        if (msg.find("out of range") != std::string::npos) throw std::out_of_range(msg);
        throw std::invalid_argument(msg);
    default: throw std::runtime_error(msg);
    }
}

inline void chk(int rc)
{
    if (rc != MHE_OK) raise(rc);
}

// util::are_close (util/common.h): |a-b| < eps * max(|a|, |b|, 1)
bool are_close(double a, double b)
{
    const double scale = std::max({ std::fabs(a), std::fabs(b), 1.0 });
    return std::fabs(a - b) < std::numeric_limits<double>::epsilon() * scale;
}

int product_bits(const std::vector<Modulus> &cm, std::size_t count)
{
    std::vector<std::uint64_t> prod(count + 1, 0);
    prod[0] = 1;
    std::size_t words = 1;
    for (std::size_t j = 0; j < count; j++)
    {
        std::uint64_t carry = 0;
        for (std::size_t w = 0; w < words; w++)
        {
            const unsigned __int128 t = (unsigned __int128)prod[w] * cm[j].value() + carry;
            prod[w] = (std::uint64_t)t;
            carry = (std::uint64_t)(t >> 64);
        }
        if (carry) prod[words++] = carry;
    }
    return (int)(64 * (words - 1)) + (64 - __builtin_clzll(prod[words - 1]));
}

// the factory key generation and encryption draw their PRNGs from (SEAL: the context installs
// DefaultFactory when the parameters carry none, context.cpp:464-467)
std::shared_ptr<UniformRandomGeneratorFactory> factory_of(const SEALContext &ctx)
{
    return ctx.key_context_data()->parms().random_generator_or_default();
}

std::vector<std::uint64_t> moduli_of(const SEALContext &ctx)
{
    std::vector<std::uint64_t> q;
    for (auto &m : ctx.key_context_data()->parms().coeff_modulus()) q.push_back(m.value());
    return q;
}
} // namespace

// ------------------------------------------------------------------------------ Modulus
int Modulus::bit_count() const noexcept
{
    return value_ ? 64 - __builtin_clzll(value_) : 0;
}

std::vector<Modulus> CoeffModulus::Create(std::size_t poly_modulus_degree, std::vector<int> bit_sizes)
{
    std::vector<std::uint64_t> out(bit_sizes.size());
    chk(mhe_coeff_modulus_create(poly_modulus_degree, bit_sizes.data(), (int)bit_sizes.size(), out.data()));
    return std::vector<Modulus>(out.begin(), out.end());
}

parms_id_type blake2b_parms_id(const std::uint64_t *words, std::size_t count); // serialize.cpp

parms_id_type EncryptionParameters::parms_id() const
{
    // SEAL's parms_id (encryptionparams.cpp:124-158): BLAKE2b-256 of [scheme, n, coeff moduli...,
    // plain modulus] as u64 words; the CKKS plain modulus is the zero Modulus (one word)
    std::vector<std::uint64_t> w{ (std::uint64_t)scheme_, (std::uint64_t)n_ };
    for (auto &m : coeff_modulus_) w.push_back(m.value());
    w.push_back(0);
    return blake2b_parms_id(w.data(), w.size());
}

// ------------------------------------------------------------------------------ SEALContext
struct SEALContext::Impl : std::enable_shared_from_this<SEALContext::Impl>
{
    EncryptionParameters parms;
    std::vector<std::shared_ptr<ContextData>> levels; // by number of primes - 1
    std::map<parms_id_type, std::shared_ptr<const ContextData>> by_id;
    std::shared_ptr<const ContextData> key, first, last;
    mhe_ctx *eng = nullptr;
    std::size_t K = 0;
    sec_level_type sec_level = sec_level_type::tc128;
    bool insecure = false;
    std::mutex mu;
    std::unordered_map<std::thread::id, void *> streams;
    // streams of threads that have exited: the next new thread takes one instead of creating a
    // stream (and with it a scratch workspace) of its own.  A stream is never destroyed while the
    // context lives -- objects written on it keep it as their writer -- so without the pool a
    // process that starts threads per batch (the reference's OpenMP team, ResNetRunner::infer_batch)
    // would grow one workspace per thread it ever ran.
    std::vector<void *> idle;

    // the calling thread's leases: on thread exit each still-living context gets the stream back
    struct Leases
    {
        std::vector<std::weak_ptr<Impl>> ctx;
        ~Leases()
        {
            const auto id = std::this_thread::get_id();
            for (auto &w : ctx)
                if (auto p = w.lock()) p->release(id);
        }
    };

    void release(std::thread::id id)
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = streams.find(id);
        if (it == streams.end()) return;
        idle.push_back(it->second);
        streams.erase(it);
    }

    void *stream()
    {
        static thread_local Leases leases;
        std::lock_guard<std::mutex> g(mu);
        auto it = streams.find(std::this_thread::get_id());
        if (it != streams.end()) return it->second;
        void *s = nullptr;
        if (!idle.empty())
        {
            s = idle.back(); // ordered after its previous thread's work: same stream
            idle.pop_back();
        }
        else
            chk(mhe_stream_create(eng, &s));
        streams.emplace(std::this_thread::get_id(), s);
        leases.ctx.push_back(weak_from_this());
        return s;
    }

    ~Impl()
    {
        for (auto &kv : streams) idle.push_back(kv.second);
        for (void *s : idle)
        {
            (void)mhe_stream_sync(eng, s);
            (void)mhe_stream_destroy(eng, s);
        }
        if (eng) (void)mhe_ctx_destroy(eng);
    }
};

namespace
{
// CoeffModulus::MaxBitCount (modulus.cpp:112-116, util/hestdparms.h: HomomorphicEncryption.org
// classical tables; the modified SEAL adds 65536 -> 1792 for tc128)
int max_bit_count(std::size_t n, sec_level_type sec)
{
    static const std::map<std::size_t, int> tc128{ { 1024, 27 },   { 2048, 54 },   { 4096, 109 },  { 8192, 218 },
                                                   { 16384, 438 }, { 32768, 881 }, { 65536, 1792 } };
    static const std::map<std::size_t, int> tc192{ { 1024, 19 }, { 2048, 37 }, { 4096, 75 },
                                                   { 8192, 152 }, { 16384, 305 }, { 32768, 611 } };
    static const std::map<std::size_t, int> tc256{ { 1024, 14 }, { 2048, 29 }, { 4096, 58 },
                                                   { 8192, 118 }, { 16384, 237 }, { 32768, 476 } };
    const std::map<std::size_t, int> *t = sec == sec_level_type::tc128   ? &tc128
                                          : sec == sec_level_type::tc192 ? &tc192
                                          : sec == sec_level_type::tc256 ? &tc256
                                                                         : nullptr;
    if (!t) return std::numeric_limits<int>::max();
    auto it = t->find(n);
    return it == t->end() ? 0 : it->second;
}
} // namespace

int CoeffModulus::MaxBitCount(std::size_t poly_modulus_degree, sec_level_type sec_level) noexcept
{
    const int m = max_bit_count(poly_modulus_degree, sec_level);
    return m == std::numeric_limits<int>::max() ? 0 : m;
}

SEALContext::SEALContext(const EncryptionParameters &parms, bool expand_mod_chain, sec_level_type sec_level)
{
    if (parms.scheme() != scheme_type::ckks) throw std::invalid_argument("unsupported scheme");
    const auto &cm = parms.coeff_modulus();
    const std::size_t n = parms.poly_modulus_degree();
    if (cm.empty()) throw std::invalid_argument("coeff_modulus is not set");
    if (!n || (n & (n - 1))) throw std::invalid_argument("poly_modulus_degree is not a power of two");
    int log_n = 0;
    while ((std::size_t(1) << log_n) < n) log_n++;

    auto impl = std::make_shared<Impl>();
    impl->parms = parms;
    impl->K = cm.size();
    // context.cpp:207-220: parameters above the HomomorphicEncryption.org bound for the requested
    // security level are kept but flagged; key generators, encryptors, ... then refuse them
    impl->sec_level = sec_level;
    if (product_bits(cm, cm.size()) > max_bit_count(n, sec_level)) impl->insecure = true;
    std::vector<std::uint64_t> q;
    for (auto &m : cm) q.push_back(m.value());
    int device = 0;
    if (const char *d = std::getenv("MHE_DEVICE")) device = std::atoi(d);
    chk(mhe_ctx_create(&impl->eng, log_n, q.data(), (int)q.size(), device));

    // context.cpp: key level (all primes) -> first (drop the special prime) -> ... -> one prime
    const std::size_t K = impl->K;
    impl->levels.resize(K);
    auto make_level = [&](std::size_t count) {
        auto cd = std::make_shared<ContextData>();
        cd->parms_ = parms;
        cd->parms_.set_coeff_modulus(std::vector<Modulus>(cm.begin(), cm.begin() + count));
        cd->parms_id_ = cd->parms_.parms_id();
        cd->total_bits_ = product_bits(cm, count);
        impl->levels[count - 1] = cd;
        impl->by_id[cd->parms_id_] = cd;
        return cd;
    };
    auto key = make_level(K);
    impl->key = key;
    if (K == 1)
    {
        key->chain_index_ = 0;
        impl->first = impl->last = key;
    }
    else
    {
        key->chain_index_ = K - 1;
        std::shared_ptr<ContextData> prev = key;
        const std::size_t lowest = expand_mod_chain ? 1 : K - 1;
        for (std::size_t c = K - 1; c >= lowest; c--)
        {
            auto cd = make_level(c);
            cd->chain_index_ = c - 1;
            cd->prev_ = prev;
            prev->next_ = cd;
            if (c == K - 1) impl->first = cd;
            impl->last = cd;
            prev = cd;
            if (c == 1) break;
        }
    }
    impl_ = impl;
}

std::shared_ptr<const SEALContext::ContextData> SEALContext::get_context_data(const parms_id_type &id) const
{
    auto it = impl_->by_id.find(id);
    return it == impl_->by_id.end() ? nullptr : it->second;
}
std::shared_ptr<const SEALContext::ContextData> SEALContext::key_context_data() const { return impl_->key; }
std::shared_ptr<const SEALContext::ContextData> SEALContext::first_context_data() const { return impl_->first; }
std::shared_ptr<const SEALContext::ContextData> SEALContext::last_context_data() const { return impl_->last; }
const parms_id_type &SEALContext::key_parms_id() const { return impl_->key->parms_id(); }
const parms_id_type &SEALContext::first_parms_id() const { return impl_->first->parms_id(); }
const parms_id_type &SEALContext::last_parms_id() const { return impl_->last->parms_id(); }
bool SEALContext::parameters_set() const noexcept { return impl_ && impl_->eng && !impl_->insecure; }
sec_level_type SEALContext::sec_level() const noexcept
{
    return impl_ && !impl_->insecure ? impl_->sec_level : sec_level_type::none;
}

namespace
{
void require_set(const SEALContext &ctx)
{
    if (!ctx.parameters_set()) throw std::invalid_argument("encryption parameters are not set correctly");
}
} // namespace
bool SEALContext::using_keyswitching() const noexcept { return impl_ && impl_->K > 1; }
mhe_ctx *SEALContext::engine() const { return impl_->eng; }
void *SEALContext::stream() const { return impl_->stream(); }
std::size_t SEALContext::key_size() const { return impl_->K; }
std::shared_ptr<void> SEALContext::handle() const { return impl_; }
void *SEALContext::stream_of(void *handle) { return static_cast<Impl *>(handle)->stream(); }

// ------------------------------------------------------------------------------ PolyStore
void PolyStore::bind(const SEALContext &ctx)
{
    if (eng_ == ctx.engine()) return;
    release();
    hold_ = ctx.handle();
    eng_ = ctx.engine();
}

void *PolyStore::thread_stream() const
{
    if (!hold_) throw std::logic_error("polynomial storage is not bound to a context");
    return SEALContext::stream_of(hold_.get());
}

// Cross-stream ordering (stream_order.h): device-side waits, no host blocking.
void PolyStore::wait_writer(void *s) const
{
    for (void *w : detail::order_before<void *>(s, writer_, writer_done_, {}, detail::Access::read))
        chk(mhe_stream_wait(eng_, s, w));
}

void PolyStore::wait_all(void *s) const
{
    for (void *w : detail::order_before<void *>(s, writer_, writer_done_, readers_, detail::Access::write))
        chk(mhe_stream_wait(eng_, s, w));
    readers_.clear();
}

void PolyStore::release()
{
    if (dev_)
    {
        std::lock_guard<std::mutex> g(*mu_);
        void *s = writer_ ? writer_ : thread_stream();
        for (void *w : detail::order_before<void *>(s, writer_, writer_done_, readers_, detail::Access::release))
            (void)mhe_stream_wait(eng_, s, w);
        (void)mhe_free_async(eng_, dev_, s);
    }
    dev_ = nullptr;
    cap_ = 0;
    readers_.clear();
    writer_ = nullptr;
    writer_done_ = true;
}

PolyStore::~PolyStore()
{
    release();
}

void PolyStore::resize_words(std::size_t words, bool preserve)
{
    if (!eng_) throw std::logic_error("polynomial storage is not bound to a context");
    if (words <= cap_ || (!dev_valid_ && host_valid_))
    {
        words_ = words;
        if (host_valid_ && host_.size() < words) host_.resize(words, 0);
        if (!dev_valid_ && host_valid_ && words > cap_ && dev_)
        {
            // host is the authority: the device copy is reallocated on the next upload
            std::lock_guard<std::mutex> g(*mu_);
            void *s = thread_stream();
            wait_all(s);
            (void)mhe_free_async(eng_, dev_, s);
            dev_ = nullptr;
            cap_ = 0;
        }
        return;
    }
    void *s = thread_stream();
    std::lock_guard<std::mutex> g(*mu_);
    wait_all(s);
    void *p = nullptr;
    chk(mhe_malloc_async(eng_, &p, words * sizeof(std::uint64_t), s));
    if (preserve && dev_ && words_) chk(mhe_memcpy_d2d(eng_, p, dev_, std::min(words_, words) * 8, s));
    if (dev_) (void)mhe_free_async(eng_, dev_, s);
    dev_ = static_cast<std::uint64_t *>(p);
    cap_ = words;
    words_ = words;
    writer_ = s;
    writer_done_ = false;
    dev_valid_ = true;
    // the device copy is authoritative from here on; a host mirror is only kept when it already
    // held data (a fresh store would otherwise zero-fill a host vector of the full size)
    if (preserve && host_valid_ && !host_.empty())
        host_.resize(words, 0);
    else
    {
        host_valid_ = false;
        host_.clear();
    }
}

const std::uint64_t *PolyStore::dev_read(void *s) const
{
    if (!eng_) throw std::logic_error("polynomial storage is not bound to a context");
    std::lock_guard<std::mutex> g(*mu_);
    if (!dev_valid_)
    {
        auto *self = const_cast<PolyStore *>(this);
        if (!dev_ || cap_ < words_)
        {
            wait_all(s);
            if (dev_) (void)mhe_free_async(eng_, dev_, s);
            void *p = nullptr;
            chk(mhe_malloc_async(eng_, &p, words_ * sizeof(std::uint64_t), s));
            self->dev_ = static_cast<std::uint64_t *>(p);
            self->cap_ = words_;
        }
        wait_all(s);
        chk(mhe_memcpy_h2d(eng_, dev_, host_.data(), words_ * 8, s));
        chk(mhe_stream_sync(eng_, s));
        dev_valid_ = true;
        writer_ = s;
        writer_done_ = true;
    }
    if (writer_ != s && std::find(readers_.begin(), readers_.end(), s) == readers_.end())
    {
        wait_writer(s); // once per (write, reading stream): the stream is then ordered after it
        readers_.push_back(s);
    }
    return dev_;
}

std::uint64_t *PolyStore::dev_write(void *s, bool overwrite)
{
    if (!eng_) throw std::logic_error("polynomial storage is not bound to a context");
    if (!dev_valid_)
    {
        if (overwrite)
        {
            std::lock_guard<std::mutex> g(*mu_);
            if (!dev_ || cap_ < words_)
            {
                wait_all(s);
                if (dev_) (void)mhe_free_async(eng_, dev_, s);
                void *p = nullptr;
                chk(mhe_malloc_async(eng_, &p, words_ * sizeof(std::uint64_t), s));
                dev_ = static_cast<std::uint64_t *>(p);
                cap_ = words_;
            }
            dev_valid_ = true;
        }
        else
            (void)dev_read(s);
    }
    std::lock_guard<std::mutex> g(*mu_);
    wait_all(s);
    writer_ = s;
    writer_done_ = false;
    host_valid_ = false;
    return dev_;
}

const std::uint64_t *PolyStore::host() const
{
    if (!host_valid_)
    {
        std::lock_guard<std::mutex> g(*mu_);
        void *s = writer_ ? writer_ : thread_stream();
        host_.resize(words_);
        if (words_)
        {
            chk(mhe_memcpy_d2h(eng_, host_.data(), dev_, words_ * 8, s));
            chk(mhe_stream_sync(eng_, s));
        }
        writer_done_ = true;
        host_valid_ = true;
    }
    return host_.data();
}

std::uint64_t *PolyStore::host()
{
    const PolyStore *c = this;
    c->host();
    if (eng_)
    {
        std::lock_guard<std::mutex> g(*mu_);
        for (void *r : readers_) chk(mhe_stream_sync(eng_, r));
        readers_.clear();
        dev_valid_ = false;
    }
    return host_.data();
}

void PolyStore::copy_from(const PolyStore &o)
{
    hold_ = o.hold_;
    eng_ = o.eng_;
    words_ = o.words_;
    if (!eng_ || (!o.dev_valid_ && o.host_valid_))
    {
        host_ = o.host_;
        host_valid_ = true;
        dev_valid_ = !eng_;
        return;
    }
    void *s = thread_stream();
    const std::uint64_t *src = o.dev_read(s);
    void *p = nullptr;
    chk(mhe_malloc_async(eng_, &p, std::max<std::size_t>(words_, 1) * 8, s));
    if (words_) chk(mhe_memcpy_d2d(eng_, p, src, words_ * 8, s));
    dev_ = static_cast<std::uint64_t *>(p);
    cap_ = words_;
    writer_ = s;
    writer_done_ = false;
    dev_valid_ = true;
    host_valid_ = false;
}

PolyStore::PolyStore(const PolyStore &o)
{
    copy_from(o);
}

PolyStore &PolyStore::operator=(const PolyStore &o)
{
    if (this == &o) return *this;
    if (eng_ && eng_ == o.eng_ && dev_ && cap_ >= o.words_ && (o.dev_valid_ || !o.host_valid_))
    {
        // same engine, enough room: copy in place on this thread's stream
        void *s = thread_stream();
        const std::uint64_t *src = o.dev_read(s);
        std::uint64_t *dst = dev_write(s, true);
        words_ = o.words_;
        if (words_) chk(mhe_memcpy_d2d(eng_, dst, src, words_ * 8, s));
        return *this;
    }
    release();
    copy_from(o);
    return *this;
}

PolyStore::PolyStore(PolyStore &&o) noexcept
{
    *this = std::move(o);
}

PolyStore &PolyStore::operator=(PolyStore &&o) noexcept
{
    if (this == &o) return *this;
    std::swap(hold_, o.hold_);
    std::swap(eng_, o.eng_);
    std::swap(dev_, o.dev_);
    std::swap(words_, o.words_);
    std::swap(cap_, o.cap_);
    std::swap(host_, o.host_);
    std::swap(host_valid_, o.host_valid_);
    std::swap(dev_valid_, o.dev_valid_);
    std::swap(mu_, o.mu_);
    std::swap(writer_, o.writer_);
    std::swap(writer_done_, o.writer_done_);
    std::swap(readers_, o.readers_);
    return *this;
}

// ------------------------------------------------------------------------------ Ciphertext
Ciphertext::Ciphertext(const SEALContext &context, MemoryPoolHandle) : Ciphertext(context, context.first_parms_id())
{}

Ciphertext::Ciphertext(const SEALContext &context, parms_id_type parms_id, MemoryPoolHandle)
{
    auto cd = context.get_context_data(parms_id);
    if (!cd) throw std::invalid_argument("parms_id is not valid for encryption parameters");
    store_.bind(context);
    parms_id_ = parms_id;
    coeff_modulus_size_ = cd->parms().coeff_modulus().size();
    poly_modulus_degree_ = cd->parms().poly_modulus_degree();
}

void Ciphertext::resize(const SEALContext &context, parms_id_type parms_id, std::size_t size)
{
    auto cd = context.get_context_data(parms_id);
    if (!cd) throw std::invalid_argument("parms_id is not valid for encryption parameters");
    if (size < 2 && size != 0) throw std::invalid_argument("invalid size");
    store_.bind(context);
    parms_id_ = parms_id;
    coeff_modulus_size_ = cd->parms().coeff_modulus().size();
    poly_modulus_degree_ = cd->parms().poly_modulus_degree();
    size_ = size;
    store_.resize_words(size * coeff_modulus_size_ * poly_modulus_degree_);
}

void Ciphertext::resize(const SEALContext &context, std::size_t size)
{
    resize(context, parms_id_ == parms_id_zero ? context.first_parms_id() : parms_id_, size);
}

void Ciphertext::resize(std::size_t size)
{
    if (size < 2 && size != 0) throw std::invalid_argument("invalid size");
    size_ = size;
    store_.resize_words(size * coeff_modulus_size_ * poly_modulus_degree_);
}

bool Ciphertext::is_transparent() const
{
    if (!store_.words() || size_ < 2) return false;
    const std::uint64_t *p = data(1);
    const std::size_t cnt = (size_ - 1) * coeff_modulus_size_ * poly_modulus_degree_;
    return std::all_of(p, p + cnt, [](std::uint64_t x) { return x == 0; });
}

void Plaintext::set_level(const SEALContext &ctx, const parms_id_type &id, std::size_t limbs)
{
    store_.bind(ctx);
    store_.resize_words(limbs * ctx.key_context_data()->parms().poly_modulus_degree(), false);
    parms_id_ = id;
    limbs_ = limbs;
}

// ------------------------------------------------------------------------------ KeyGenerator
// keygenerator.cpp: secret key (sparse ternary with the modified hamming weight, else ternary)
// in NTT form at the key level; public key and key-switching keys are symmetric encryptions of
// zero at the key level (rlwe.cpp encrypt_zero_symmetric), the latter with
// (P mod q_i) * s'_i added to digit i's limb i (keygenerator.cpp:384-414).
namespace
{
struct Poly
{
    std::vector<std::uint64_t> h;
};

// temporary device buffer on stream s
struct DevBuf
{
    mhe_ctx *eng;
    void *s;
    std::uint64_t *p = nullptr;
    DevBuf(mhe_ctx *e, void *st, std::size_t words) : eng(e), s(st)
    {
        void *q = nullptr;
        chk(mhe_malloc_async(eng, &q, std::max<std::size_t>(words, 1) * 8, s));
        p = static_cast<std::uint64_t *>(q);
    }
    ~DevBuf() { (void)mhe_free_async(eng, p, s); }
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
};

void upload(mhe_ctx *eng, void *s, std::uint64_t *dst, const std::vector<std::uint64_t> &h)
{
    chk(mhe_memcpy_h2d(eng, dst, h.data(), h.size() * 8, s));
    chk(mhe_stream_sync(eng, s)); // the host vector is temporary
}

// encrypt_zero_symmetric (rlwe.cpp:289-373) at a level of `limbs` primes, NTT form, no seed
// saved: bootstrap PRNG <- `seed`; its first 64 bytes seed the PRNG of a = c1 (sample_poly_uniform,
// NTT form directly); e = sample_poly_cbd from the bootstrap PRNG's next bytes; c0 = -(a*s + e).
void sym_encrypt_zero(const SEALContext &ctx, const prng_seed_type &seed, const std::uint64_t *sk,
                            std::size_t limbs, std::uint64_t *c0, std::uint64_t *c1, void *s)
{
    mhe_ctx *eng = ctx.engine();
    const std::size_t n = ctx.key_context_data()->parms().poly_modulus_degree();
    rnd::sample_uniform_dev(eng, rnd::stream_prefix_seed(seed), moduli_of(ctx), limbs, n, c1, s);
    rnd::sample_cbd_dev(eng, seed, prng_seed_byte_count, limbs, c0, s);
    chk(mhe_ntt_forward(eng, c0, 1, (int)limbs, 0, s));
    DevBuf t(eng, s, limbs * n);
    chk(mhe_multiply_plain(eng, sk, c1, t.p, 1, (int)limbs, s));
    chk(mhe_add(eng, t.p, c0, c0, 1, (int)limbs, s));
    chk(mhe_negate(eng, c0, c0, 1, (int)limbs, s));
}

// generate_one_kswitch_key (keygenerator.cpp:384-414) truncated to `digits` digits: digit j is an
// encryption of zero over the key level (its own bootstrap seed, next_seed()) with
// (P mod q_j) * new_key added to limb j of c0; the stored key keeps primes q_0..q_{digits-1} and
// P ([digits][2][digits+1][n]).  digits = K-1 is SEAL's full key; a truncated key is SEAL's key
// restricted to those digits and primes (the whole digit is drawn, then the kept limbs copied).
void make_kswitch_key(const SEALContext &ctx, const std::function<prng_seed_type()> &next_seed,
                      const std::uint64_t *sk, const std::uint64_t *new_key, std::size_t digits, PolyStore &dest)
{
    const std::size_t K = ctx.key_size(), n = ctx.key_context_data()->parms().poly_modulus_degree();
    const auto &cm = ctx.key_context_data()->parms().coeff_modulus();
    if (K < 2) throw std::logic_error("keyswitching is not supported by the context");
    if (digits < 1 || digits > K - 1) throw std::invalid_argument("key digits out of range");
    mhe_ctx *eng = ctx.engine();
    void *s = ctx.stream();
    const std::size_t KL = digits + 1; // stored limbs
    dest.bind(ctx);
    dest.resize_words(digits * 2 * KL * n, false);
    std::uint64_t *d = dest.dev_write(s, true);
    DevBuf t(eng, s, K * n);
    const bool full = KL == K;
    DevBuf tmp(eng, s, full ? 1 : 2 * K * n);
    const std::uint64_t P = cm[K - 1].value();
    for (std::size_t j = 0; j < digits; j++)
    {
        std::uint64_t *c0 = full ? d + j * 2 * K * n : tmp.p, *c1 = c0 + K * n;
        sym_encrypt_zero(ctx, next_seed(), sk, K, c0, c1, s);
        std::vector<std::uint64_t> f(K, 0);
        f[j] = P % cm[j].value();
        chk(mhe_multiply_scalar(eng, new_key, f.data(), t.p, 1, (int)K, s));
        chk(mhe_add(eng, c0, t.p, c0, 1, (int)K, s));
        if (!full)
            for (int c = 0; c < 2; c++)
            {
                const std::uint64_t *src = tmp.p + c * K * n;
                std::uint64_t *dst = d + (j * 2 + c) * KL * n;
                chk(mhe_memcpy_d2d(eng, dst, src, digits * n * 8, s));
                chk(mhe_memcpy_d2d(eng, dst + digits * n, src + (K - 1) * n, n * 8, s));
            }
    }
}
} // namespace

// Deferred Galois keys (see seal.h, KeyGenerator::create_deferred_galois_keys): a client-side key
// provider holding the secret key and, per key index, its Galois element and a 512-bit seed.
// Digit j of a materialised key draws its bootstrap seed from bytes [64j, 64j+64) of that seed's
// stream, so a key re-materialised larger keeps its smaller prefix.
struct KeyMaker
{
    std::mutex mu;
    SEALContext ctx;
    PolyStore sk; // NTT form over the key level
    std::map<std::size_t, std::pair<std::uint32_t, prng_seed_type>> elts;
    explicit KeyMaker(const SEALContext &c) : ctx(c) {}
};

std::size_t KSwitchKeys::size() const
{
    if (!maker_) return keys_.size();
    std::lock_guard<std::mutex> lk(maker_->mu);
    std::size_t c = maker_->elts.size();
    for (const auto &kv : keys_)
        if (!maker_->elts.count(kv.first)) c++;
    return c;
}

bool KSwitchKeys::has_index(std::size_t i) const
{
    if (maker_)
    {
        std::lock_guard<std::mutex> lk(maker_->mu);
        if (maker_->elts.count(i)) return true;
    }
    return keys_.count(i) != 0;
}

const PolyStore &KSwitchKeys::key(std::size_t i) const
{
    auto it = keys_.find(i);
    if (it == keys_.end()) throw std::out_of_range("kswitch_keys_index");
    return it->second;
}

std::size_t KSwitchKeys::limbs_of(std::size_t i) const
{
    auto it = limbs_of_.find(i);
    return it == limbs_of_.end() ? key_limbs_ : it->second;
}

const std::uint64_t *KSwitchKeys::key_for(std::size_t i, std::size_t L, void *stream, std::size_t &key_limbs) const
{
    if (maker_)
    {
        std::lock_guard<std::mutex> lk(maker_->mu);
        auto e = maker_->elts.find(i);
        if (e != maker_->elts.end())
        {
            auto lt = limbs_of_.find(i);
            if (lt == limbs_of_.end() || lt->second < L + 1)
            {
                // materialise (or grow) the level-truncated key on the maker's context stream
                const SEALContext &ctx = maker_->ctx;
                const std::size_t K = ctx.key_size();
                const std::size_t digits = std::min(K - 1, std::max<std::size_t>(L, 1));
                void *s = ctx.stream();
                const std::size_t n = ctx.key_context_data()->parms().poly_modulus_degree();
                DevBuf rot(ctx.engine(), s, K * n);
                const std::uint64_t *sk = maker_->sk.dev_read(s);
                chk(mhe_permute_galois(ctx.engine(), sk, e->second.first, rot.p, 1, (int)K, s));
                Blake2xbPRNG seeds(e->second.second);
                PolyStore fresh;
                make_kswitch_key(
                    ctx,
                    [&] {
                        prng_seed_type d;
                        seeds.generate(prng_seed_byte_count, reinterpret_cast<seal_byte *>(d.data()));
                        return d;
                    },
                    sk, rot.p, digits, fresh);
                auto kt = keys_.find(i);
                if (kt != keys_.end()) retired_.push_back(std::move(kt->second));
                keys_[i] = std::move(fresh);
                limbs_of_[i] = digits + 1;
            }
            key_limbs = limbs_of_[i];
            return keys_.find(i)->second.dev_read(stream);
        }
    }
    key_limbs = limbs_of(i);
    if (key_limbs < L + 1)
        throw std::invalid_argument("key-switching key is truncated below the ciphertext level");
    return key(i).dev_read(stream);
}

std::map<std::size_t, std::size_t> KSwitchKeys::usage() const
{
    std::map<std::size_t, std::size_t> u;
    for (const auto &kv : keys_) u[kv.first] = limbs_of(kv.first);
    return u;
}

std::size_t KSwitchKeys::device_bytes() const
{
    std::size_t b = 0;
    for (const auto &kv : keys_) b += kv.second.words() * 8;
    for (const auto &r : retired_) b += r.words() * 8;
    return b;
}

void KSwitchKeys::insert(std::size_t index, PolyStore &&key, std::size_t limbs)
{
    keys_[index] = std::move(key);
    limbs_of_[index] = limbs;
}

KeyGenerator::KeyGenerator(const SEALContext &context) : ctx_(context)
{
    require_set(context);
    // keygenerator.cpp:62-84: the secret key from a fresh PRNG of the parameters' factory,
    // sparse ternary with the modified Hamming weight (or ternary for weight 0), NTT form
    const auto &parms = context.key_context_data()->parms();
    rng_ = factory_of(context);
    const std::size_t K = context.key_size(), n = parms.poly_modulus_degree();
    const std::size_t hw = parms.secret_key_hamming_weight();
    const auto q = moduli_of(context);
    std::vector<std::uint64_t> h(K * n);
    {
        auto prng = rng_->create();
        if (hw)
            rnd::sample_sparse_ternary_host(*prng, q, n, hw, h.data());
        else
            rnd::sample_ternary_host(*prng, q, K, n, h.data());
    }
    void *s = context.stream();
    sk_.data().set_level(context, context.key_parms_id(), K);
    std::uint64_t *d = sk_.data().store().dev_write(s, true);
    upload(context.engine(), s, d, h);
    std::fill(h.begin(), h.end(), 0);
    chk(mhe_ntt_forward(context.engine(), d, 1, (int)K, 0, s));
}

KeyGenerator::KeyGenerator(const SEALContext &context, const SecretKey &secret_key) : ctx_(context), sk_(secret_key)
{
    require_set(context);
    if (secret_key.parms_id() != context.key_parms_id())
        throw std::invalid_argument("secret key is not valid for encryption parameters");
    rng_ = factory_of(context);
}

namespace
{
// generate_pk (keygenerator.cpp:87-112): encrypt_zero_symmetric at the key level
prng_seed_type make_public_key(const SEALContext &ctx, UniformRandomGeneratorFactory &rng, const SecretKey &sk,
                               PublicKey &destination)
{
    const std::size_t K = ctx.key_size(), n = ctx.key_context_data()->parms().poly_modulus_degree();
    void *s = ctx.stream();
    Ciphertext &pk = destination.data();
    pk.resize(ctx, ctx.key_parms_id(), 2);
    pk.is_ntt_form() = true;
    pk.scale() = 1.0;
    std::uint64_t *d = pk.store().dev_write(s, true);
    const prng_seed_type seed = rng.next_seed();
    sym_encrypt_zero(ctx, seed, sk.data().store().dev_read(s), K, d, d + K * n, s);
    return rnd::stream_prefix_seed(seed);
}
} // namespace

void KeyGenerator::create_public_key(PublicKey &destination) { make_public_key(ctx_, *rng_, sk_, destination); }

Serializable<PublicKey> KeyGenerator::create_public_key()
{
    PublicKey pk;
    const prng_seed_type seed = make_public_key(ctx_, *rng_, sk_, pk);
    return Serializable<PublicKey>(std::move(pk), SeedMap{ { 0, { seed } } });
}

void KeyGenerator::kswitch_key(const std::uint64_t *new_key, PolyStore &dest, std::size_t digits,
                               std::vector<prng_seed_type> *seeds)
{
    make_kswitch_key(
        ctx_,
        [&] {
            const prng_seed_type sd = rng_->next_seed();
            if (seeds) seeds->push_back(rnd::stream_prefix_seed(sd));
            return sd;
        },
        sk_.data().store().dev_read(ctx_.stream()), new_key, digits, dest);
}

void KeyGenerator::create_relin_keys(RelinKeys &destination) { relin_keys_into(destination, nullptr); }

Serializable<RelinKeys> KeyGenerator::create_relin_keys()
{
    RelinKeys rk;
    SeedMap seeds;
    relin_keys_into(rk, &seeds);
    return Serializable<RelinKeys>(std::move(rk), std::move(seeds));
}

void KeyGenerator::relin_keys_into(RelinKeys &destination, SeedMap *seeds)
{
    // create_relin_keys (keygenerator.cpp:115-149): key-switching key of s^2
    const std::size_t K = ctx_.key_size(), n = ctx_.key_context_data()->parms().poly_modulus_degree();
    void *s = ctx_.stream();
    DevBuf s2(ctx_.engine(), s, K * n);
    const std::uint64_t *sk = sk_.data().store().dev_read(s);
    chk(mhe_multiply_plain(ctx_.engine(), sk, sk, s2.p, 1, (int)K, s));
    PolyStore key;
    kswitch_key(s2.p, key, K - 1, seeds ? &(*seeds)[RelinKeys::get_index(2)] : nullptr);
    destination.insert(RelinKeys::get_index(2), std::move(key), K);
    destination.parms_id() = ctx_.key_parms_id();
    destination.set_key_limbs(K);
}

void KeyGenerator::create_galois_keys(const std::vector<std::pair<std::uint32_t, std::size_t>> &elt_limbs,
                                      GaloisKeys &destination)
{
    // create_galois_keys (keygenerator.cpp:152-190): per element, the key-switching key of
    // s(X^elt) (apply_galois_ntt on the NTT-form secret key); here truncated per element to the
    // level it is used at (limbs = ciphertext limbs; >= K-1 keeps SEAL's full key)
    const std::size_t K = ctx_.key_size(), n = ctx_.key_context_data()->parms().poly_modulus_degree();
    if (K < 2) throw std::logic_error("keyswitching is not supported by the context");
    void *s = ctx_.stream();
    DevBuf rot(ctx_.engine(), s, K * n);
    for (const auto &el : elt_limbs)
    {
        const std::uint32_t elt = el.first;
        if (!(elt & 1) || elt >= 2 * n) throw std::invalid_argument("Galois element is not valid");
        if (destination.has_key(elt)) continue;
        const std::size_t digits = std::min(K - 1, std::max<std::size_t>(el.second, 1));
        const std::uint64_t *sk = sk_.data().store().dev_read(s);
        chk(mhe_permute_galois(ctx_.engine(), sk, elt, rot.p, 1, (int)K, s));
        PolyStore key;
        kswitch_key(rot.p, key, digits);
        destination.insert(GaloisKeys::get_index(elt), std::move(key), digits + 1);
    }
    destination.parms_id() = ctx_.key_parms_id();
    destination.set_key_limbs(K);
}

void KeyGenerator::create_galois_keys_from_elts(const std::vector<std::uint32_t> &elts, GaloisKeys &destination)
{
    galois_keys_into(elts, destination, nullptr);
}

void KeyGenerator::galois_keys_into(const std::vector<std::uint32_t> &elts, GaloisKeys &destination, SeedMap *seeds)
{
    // create_galois_keys (keygenerator.cpp:152-190) with SEAL's full keys; seeds receives every
    // digit's public seed per key index
    const std::size_t K = ctx_.key_size(), n = ctx_.key_context_data()->parms().poly_modulus_degree();
    if (K < 2) throw std::logic_error("keyswitching is not supported by the context");
    void *s = ctx_.stream();
    DevBuf rot(ctx_.engine(), s, K * n);
    for (std::uint32_t elt : elts)
    {
        if (!(elt & 1) || elt >= 2 * n) throw std::invalid_argument("Galois element is not valid");
        if (destination.has_key(elt)) continue;
        const std::uint64_t *sk = sk_.data().store().dev_read(s);
        chk(mhe_permute_galois(ctx_.engine(), sk, elt, rot.p, 1, (int)K, s));
        PolyStore key;
        kswitch_key(rot.p, key, K - 1, seeds ? &(*seeds)[GaloisKeys::get_index(elt)] : nullptr);
        destination.insert(GaloisKeys::get_index(elt), std::move(key), K);
    }
    destination.parms_id() = ctx_.key_parms_id();
    destination.set_key_limbs(K);
}

void KeyGenerator::create_deferred_galois_keys_from_elts(const std::vector<std::uint32_t> &elts, GaloisKeys &destination)
{
    const std::size_t K = ctx_.key_size(), n = ctx_.key_context_data()->parms().poly_modulus_degree();
    if (K < 2) throw std::logic_error("keyswitching is not supported by the context");
    auto maker = destination.maker();
    if (!maker)
    {
        maker = std::make_shared<KeyMaker>(ctx_);
        maker->sk = sk_.data().store();
        destination.set_maker(maker);
    }
    std::lock_guard<std::mutex> lk(maker->mu);
    for (std::uint32_t elt : elts)
    {
        if (!(elt & 1) || elt >= 2 * n) throw std::invalid_argument("Galois element is not valid");
        const std::size_t idx = GaloisKeys::get_index(elt);
        if (!maker->elts.count(idx)) maker->elts[idx] = { elt, rng_->next_seed() };
    }
    destination.parms_id() = ctx_.key_parms_id();
    destination.set_key_limbs(K);
}

namespace
{
std::vector<std::uint32_t> elts_from_steps(const SEALContext &ctx, const std::vector<int> &steps)
{
    // GaloisTool::get_elts_from_steps (util/galois.cpp:96-104)
    const int log_n = __builtin_ctzll(ctx.key_context_data()->parms().poly_modulus_degree());
    std::vector<std::uint32_t> elts;
    for (int st : steps)
    {
        const std::uint32_t e = mhe_galois_elt_from_step(log_n, st);
        if (!e) throw std::invalid_argument("step count too large");
        elts.push_back(e);
    }
    return elts;
}

std::vector<std::uint32_t> elts_all(const SEALContext &ctx)
{
    // GaloisTool::get_elts_all (util/galois.cpp:106-131), generator 5
    const std::size_t n = ctx.key_context_data()->parms().poly_modulus_degree();
    const std::uint64_t m = 2 * n;
    const int log_n = __builtin_ctzll(n);
    std::vector<std::uint32_t> elts{ (std::uint32_t)(m - 1) };
    std::uint64_t pos = 5, neg = 1;
    // inverse of 5 mod m (m a power of two): 5^(m/4 - 1)
    for (std::uint64_t k = 0; k < m / 4 - 1; k++) neg = (neg * 5) & (m - 1);
    for (int i = 0; i < log_n - 1; i++)
    {
        elts.push_back((std::uint32_t)pos);
        pos = (pos * pos) & (m - 1);
        elts.push_back((std::uint32_t)neg);
        neg = (neg * neg) & (m - 1);
    }
    return elts;
}
} // namespace

void KeyGenerator::create_galois_keys(const std::vector<int> &steps, GaloisKeys &destination)
{
    create_galois_keys_from_elts(elts_from_steps(ctx_, steps), destination);
}

void KeyGenerator::create_galois_keys(GaloisKeys &destination)
{
    create_galois_keys_from_elts(elts_all(ctx_), destination);
}

Serializable<GaloisKeys> KeyGenerator::create_galois_keys(const std::vector<int> &steps)
{
    GaloisKeys gk;
    SeedMap seeds;
    galois_keys_into(elts_from_steps(ctx_, steps), gk, &seeds);
    return Serializable<GaloisKeys>(std::move(gk), std::move(seeds));
}

Serializable<GaloisKeys> KeyGenerator::create_galois_keys()
{
    GaloisKeys gk;
    SeedMap seeds;
    galois_keys_into(elts_all(ctx_), gk, &seeds);
    return Serializable<GaloisKeys>(std::move(gk), std::move(seeds));
}

void KeyGenerator::create_deferred_galois_keys(const std::vector<int> &steps, GaloisKeys &destination)
{
    create_deferred_galois_keys_from_elts(elts_from_steps(ctx_, steps), destination);
}

void KeyGenerator::create_deferred_galois_keys(GaloisKeys &destination)
{
    create_deferred_galois_keys_from_elts(elts_all(ctx_), destination);
}

const GaloisKeys &KeyGenerator::power_of_two_keys()
{
    std::lock_guard<std::mutex> lk(*pow2_mu_);
    if (!pow2_)
    {
        const int log_n = __builtin_ctzll(ctx_.key_context_data()->parms().poly_modulus_degree());
        std::vector<int> steps;
        for (int i = 0; i < log_n - 1; i++)
        {
            steps.push_back(1 << i);
            steps.push_back(-(1 << i));
        }
        pow2_ = std::make_shared<GaloisKeys>();
        create_deferred_galois_keys(steps, *pow2_);
    }
    return *pow2_;
}

// ------------------------------------------------------------------------------ CKKSEncoder
CKKSEncoder::CKKSEncoder(const SEALContext &context) : ctx_(context)
{
    require_set(context);
    const auto &parms = context.first_context_data()->parms();
    const std::size_t n = parms.poly_modulus_degree();
    slots_ = n >> 1;
    sparse_slots_ = parms.sparse_slots() ? parms.sparse_slots() : slots_;
    chk(mhe_encoder_create(&enc_, __builtin_ctzll(n)));
}

CKKSEncoder::~CKKSEncoder()
{
    if (enc_) (void)mhe_encoder_destroy(enc_);
}

void CKKSEncoder::encode_internal(const double *re, const double *im, std::size_t count, parms_id_type parms_id,
                                  double scale, Plaintext &destination)
{
    auto cd = ctx_.get_context_data(parms_id);
    if (!cd) throw std::invalid_argument("parms_id is not valid for encryption parameters");
    const std::size_t L = cd->parms().coeff_modulus().size();
    if (count > slots_) throw std::invalid_argument("values_size is too large");
    void *s = ctx_.stream();
    destination.set_level(ctx_, parms_id, L);
    destination.scale() = scale;
    chk(mhe_ckks_encode(ctx_.engine(), enc_, re, im, count, scale, (int)L, destination.store().dev_write(s, true),
                        s));
}

void CKKSEncoder::encode(const std::vector<double> &values, parms_id_type parms_id, double scale,
                         Plaintext &destination, MemoryPoolHandle)
{
    TRACE_OP("encode", trace::pt(destination), trace::vec(values.data(), nullptr, values.size()));
    TRACE_EXTRA("\"scale\": " + trace::num(scale));
    encode_internal(values.data(), nullptr, values.size(), parms_id, scale, destination);
}

void CKKSEncoder::encode(const std::vector<std::complex<double>> &values, parms_id_type parms_id, double scale,
                         Plaintext &destination, MemoryPoolHandle)
{
    std::vector<double> re(values.size()), im(values.size());
    for (std::size_t i = 0; i < values.size(); i++)
    {
        re[i] = values[i].real();
        im[i] = values[i].imag();
    }
    TRACE_OP("encode", trace::pt(destination), trace::vec(re.data(), im.data(), re.size()));
    TRACE_EXTRA("\"scale\": " + trace::num(scale));
    encode_internal(re.data(), im.data(), values.size(), parms_id, scale, destination);
}

void CKKSEncoder::encode(const std::vector<double> &values, double scale, Plaintext &destination, MemoryPoolHandle)
{
    encode(values, ctx_.first_parms_id(), scale, destination);
}

void CKKSEncoder::encode(const std::vector<std::complex<double>> &values, double scale, Plaintext &destination,
                         MemoryPoolHandle)
{
    encode(values, ctx_.first_parms_id(), scale, destination);
}

void CKKSEncoder::encode(double value, parms_id_type parms_id, double scale, Plaintext &destination, MemoryPoolHandle)
{
    TRACE_OP("encode_const", trace::pt(destination));
    TRACE_EXTRA("\"value\": " + trace::num(value) + ", \"scale\": " + trace::num(scale) + ", \"limbs\": " +
                std::to_string(ctx_.get_context_data(parms_id) ? ctx_.get_context_data(parms_id)->parms().coeff_modulus().size() : 0));
    auto cd = ctx_.get_context_data(parms_id);
    if (!cd) throw std::invalid_argument("parms_id is not valid for encryption parameters");
    const std::size_t L = cd->parms().coeff_modulus().size();
    std::vector<std::uint64_t> r(L);
    chk(mhe_ckks_encode_scalar(ctx_.engine(), value, scale, (int)L, r.data()));
    void *s = ctx_.stream();
    destination.set_level(ctx_, parms_id, L);
    destination.scale() = scale;
    chk(mhe_set_scalar(ctx_.engine(), r.data(), destination.store().dev_write(s, true), 1, (int)L, s));
}

void CKKSEncoder::encode(double value, double scale, Plaintext &destination, MemoryPoolHandle)
{
    encode(value, ctx_.first_parms_id(), scale, destination);
}

void CKKSEncoder::decode_internal(const Plaintext &plain, std::vector<std::complex<double>> &out)
{
    if (!plain.is_ntt_form()) throw std::invalid_argument("plain is not in NTT form");
    auto cd = ctx_.get_context_data(plain.parms_id());
    if (!cd) throw std::invalid_argument("plain is not valid for encryption parameters");
    const std::size_t L = cd->parms().coeff_modulus().size();
    std::vector<double> re(sparse_slots_), im(sparse_slots_);
    void *s = ctx_.stream();
    chk(mhe_ckks_decode(ctx_.engine(), enc_, plain.store().dev_read(s), (int)L, plain.scale(),
                        sparse_slots_ == slots_ ? 0 : sparse_slots_, re.data(), im.data(), s));
    out.resize(sparse_slots_);
    for (std::size_t i = 0; i < sparse_slots_; i++) out[i] = { re[i], im[i] };
}

void CKKSEncoder::decode(const Plaintext &plain, std::vector<std::complex<double>> &destination, MemoryPoolHandle)
{
    decode_internal(plain, destination);
}

void CKKSEncoder::decode(const Plaintext &plain, std::vector<double> &destination, MemoryPoolHandle)
{
    std::vector<std::complex<double>> z;
    decode_internal(plain, z);
    destination.resize(z.size());
    for (std::size_t i = 0; i < z.size(); i++) destination[i] = z[i].real();
}

// ------------------------------------------------------------------------------ Encryptor
Encryptor::Encryptor(const SEALContext &context, const PublicKey &public_key)
    : ctx_(context), pk_(public_key), asymmetric_(true)
{
    require_set(context);
    if (public_key.parms_id() != context.key_parms_id())
        throw std::invalid_argument("public key is not valid for encryption parameters");
    rng_ = factory_of(context);
}

Encryptor::Encryptor(const SEALContext &context, const SecretKey &secret_key)
    : ctx_(context), sk_(secret_key), asymmetric_(false), has_sk_(true)
{
    require_set(context);
    if (secret_key.parms_id() != context.key_parms_id())
        throw std::invalid_argument("secret key is not valid for encryption parameters");
    rng_ = factory_of(context);
}

Encryptor::Encryptor(const SEALContext &context, const PublicKey &public_key, const SecretKey &secret_key)
    : Encryptor(context, public_key)
{
    set_secret_key(secret_key);
}

void Encryptor::set_public_key(const PublicKey &public_key)
{
    if (public_key.parms_id() != ctx_.key_parms_id())
        throw std::invalid_argument("public key is not valid for encryption parameters");
    pk_ = public_key;
    asymmetric_ = true;
}

void Encryptor::set_secret_key(const SecretKey &secret_key)
{
    if (secret_key.parms_id() != ctx_.key_parms_id())
        throw std::invalid_argument("secret key is not valid for encryption parameters");
    sk_ = secret_key;
    has_sk_ = true;
}

void Encryptor::encrypt_zero_at(std::size_t L, Ciphertext &dest, bool symmetric, prng_seed_type *public_seed) const
{
    // encryptor.cpp:88-166 (encrypt_zero_internal): public-key encryption runs one level up
    // (the key level for the first data level) and is divided and rounded down by the dropped
    // prime; secret-key encryption runs at the level itself.
    const std::size_t K = ctx_.key_size(), n = ctx_.key_context_data()->parms().poly_modulus_degree();
    mhe_ctx *eng = ctx_.engine();
    void *s = ctx_.stream();
    std::uint64_t *d = dest.store().dev_write(s, true);
    const prng_seed_type seed = rng_->next_seed();
    if (symmetric)
    {
        if (!has_sk_) throw std::logic_error("secret key is not set");
        sym_encrypt_zero(ctx_, seed, sk_.data().store().dev_read(s), L, d, d + L * n, s);
        if (public_seed) *public_seed = rnd::stream_prefix_seed(seed);
        return;
    }
    if (!asymmetric_) throw std::logic_error("public key is not set");
    // encrypt_zero_asymmetric (rlwe.cpp:220-286): one PRNG; u ternary, then e_0, e_1 (CBD)
    const std::size_t m = L < K ? L + 1 : L;
    const std::uint64_t *pk = pk_.data().store().dev_read(s);
    DevBuf u(eng, s, m * n), c(eng, s, 2 * m * n), e(eng, s, 2 * m * n), state(eng, s, 1);
    auto *st = reinterpret_cast<std::uint32_t *>(state.p);
    chk(mhe_prng_small(eng, seed.data(), 0, MHE_SAMPLE_TERNARY, (int)m, u.p, st, s));
    chk(mhe_prng_small(eng, seed.data(), 4 * n, MHE_SAMPLE_CBD, (int)m, e.p, st, s));
    chk(mhe_prng_small(eng, seed.data(), 10 * n, MHE_SAMPLE_CBD, (int)m, e.p + m * n, st, s));
    chk(mhe_ntt_forward(eng, u.p, 1, (int)m, 0, s));
    chk(mhe_ntt_forward(eng, e.p, 2, (int)m, 0, s));
    for (int j = 0; j < 2; j++)
    {
        // pk_j restricted to the first m primes: limbs 0..m-1 of poly j ([2][K][n] layout)
        chk(mhe_multiply_plain(eng, u.p, pk + j * K * n, c.p + j * m * n, 1, (int)m, s));
        chk(mhe_add(eng, e.p + j * m * n, c.p + j * m * n, c.p + j * m * n, 1, (int)m, s));
    }
    if (m == L)
        chk(mhe_memcpy_d2d(eng, d, c.p, 2 * L * n * 8, s));
    else
        chk(mhe_rescale_to_next(eng, c.p, d, 2, (int)m, s));
}

void Encryptor::zero_at(parms_id_type parms_id, Ciphertext &destination, bool symmetric,
                        prng_seed_type *public_seed) const
{
    auto cd = ctx_.get_context_data(parms_id);
    if (!cd) throw std::invalid_argument("parms_id is not valid for encryption parameters");
    destination.resize(ctx_, parms_id, 2);
    destination.is_ntt_form() = true;
    destination.scale() = 1.0;
    encrypt_zero_at(cd->parms().coeff_modulus().size(), destination, symmetric, public_seed);
}

void Encryptor::encrypt_zero(parms_id_type parms_id, Ciphertext &destination, MemoryPoolHandle) const
{
    // SEAL's encrypt_zero / encrypt are public-key encryptions (encryptor.h:158-164, encryptor.cpp:
    // 177-181): without a public key they throw, even when a secret key is set
    zero_at(parms_id, destination, false, nullptr);
}

void Encryptor::encrypt_zero(Ciphertext &destination, MemoryPoolHandle pool) const
{
    encrypt_zero(ctx_.first_parms_id(), destination, pool);
}

void Encryptor::encrypt_zero_symmetric(parms_id_type parms_id, Ciphertext &destination, MemoryPoolHandle) const
{
    zero_at(parms_id, destination, true, nullptr);
}

void Encryptor::encrypt_zero_symmetric(Ciphertext &destination, MemoryPoolHandle pool) const
{
    encrypt_zero_symmetric(ctx_.first_parms_id(), destination, pool);
}

Serializable<Ciphertext> Encryptor::encrypt_zero_symmetric(parms_id_type parms_id, MemoryPoolHandle) const
{
    Ciphertext c;
    prng_seed_type seed{};
    zero_at(parms_id, c, true, &seed);
    return Serializable<Ciphertext>(std::move(c), SeedMap{ { 0, { seed } } });
}

Serializable<Ciphertext> Encryptor::encrypt_zero_symmetric(MemoryPoolHandle pool) const
{
    return encrypt_zero_symmetric(ctx_.first_parms_id(), pool);
}

void Encryptor::encrypt(const Plaintext &plain, Ciphertext &destination, MemoryPoolHandle) const
{
    encrypt_plain(plain, destination, false, nullptr);
}

Serializable<Ciphertext> Encryptor::encrypt(const Plaintext &plain, MemoryPoolHandle) const
{
    // a public-key encryption has no seed to save (encrypt_symmetric is the seeded form)
    Ciphertext c;
    encrypt_plain(plain, c, false, nullptr);
    return Serializable<Ciphertext>(std::move(c), SeedMap{});
}

void Encryptor::encrypt_symmetric(const Plaintext &plain, Ciphertext &destination, MemoryPoolHandle) const
{
    encrypt_plain(plain, destination, true, nullptr);
}

Serializable<Ciphertext> Encryptor::encrypt_symmetric(const Plaintext &plain, MemoryPoolHandle) const
{
    Ciphertext c;
    prng_seed_type seed{};
    encrypt_plain(plain, c, true, &seed);
    return Serializable<Ciphertext>(std::move(c), SeedMap{ { 0, { seed } } });
}

void Encryptor::encrypt_plain(const Plaintext &plain, Ciphertext &destination, bool symmetric,
                              prng_seed_type *public_seed) const
{
    TRACE_OP("encrypt", trace::ct(destination), trace::pt(plain));
    // encrypt_internal (encryptor.cpp:168-239), CKKS branch: the plaintext is added to c0 only, so a
    // symmetric encryption keeps c1 = the seeded uniform polynomial
    if (!plain.is_ntt_form()) throw std::invalid_argument("plain must be in NTT form");
    auto cd = ctx_.get_context_data(plain.parms_id());
    if (!cd) throw std::invalid_argument("plain is not valid for encryption parameters");
    const std::size_t L = cd->parms().coeff_modulus().size();
    zero_at(plain.parms_id(), destination, symmetric, public_seed);
    void *s = ctx_.stream();
    std::uint64_t *d = destination.store().dev_write(s);
    chk(mhe_add(ctx_.engine(), d, plain.store().dev_read(s), d, 1, (int)L, s));
    destination.scale() = plain.scale();
}

// ------------------------------------------------------------------------------ Decryptor
Decryptor::Decryptor(const SEALContext &context, const SecretKey &secret_key) : ctx_(context), sk_(secret_key)
{
    require_set(context);
    if (secret_key.parms_id() != context.key_parms_id())
        throw std::invalid_argument("secret key is not valid for encryption parameters");
}

void Decryptor::decrypt(const Ciphertext &encrypted, Plaintext &destination)
{
    // decryptor.cpp ckks_decrypt: <(c0, c1, c2, ...), (1, s, s^2, ...)> in NTT form
    auto cd = ctx_.get_context_data(encrypted.parms_id());
    if (!cd || encrypted.size() < 2) throw std::invalid_argument("encrypted is not valid for encryption parameters");
    if (!encrypted.is_ntt_form()) throw std::invalid_argument("encrypted must be in NTT form");
    const std::size_t L = cd->parms().coeff_modulus().size(), n = cd->parms().poly_modulus_degree();
    mhe_ctx *eng = ctx_.engine();
    void *s = ctx_.stream();
    const std::uint64_t *c = encrypted.store().dev_read(s);
    const std::uint64_t *sk = sk_.data().store().dev_read(s);
    Plaintext out;
    out.set_level(ctx_, encrypted.parms_id(), L);
    std::uint64_t *d = out.store().dev_write(s, true);
    chk(mhe_memcpy_d2d(eng, d, c, L * n * 8, s));
    DevBuf t(eng, s, L * n), sp(eng, s, L * n);
    chk(mhe_memcpy_d2d(eng, sp.p, sk, L * n * 8, s)); // s restricted to the level (first L limbs)
    for (std::size_t k = 1; k < encrypted.size(); k++)
    {
        if (k > 1) chk(mhe_multiply_plain(eng, sp.p, sk, sp.p, 1, (int)L, s));
        chk(mhe_multiply_plain(eng, c + k * L * n, sp.p, t.p, 1, (int)L, s));
        chk(mhe_add(eng, d, t.p, d, 1, (int)L, s));
    }
    out.scale() = encrypted.scale();
    destination = std::move(out);
}

// ------------------------------------------------------------------------------ Evaluator
namespace
{
struct Level
{
    std::size_t L, n;
    double total_bits;
    std::shared_ptr<const SEALContext::ContextData> cd;
};

Level level_of(const SEALContext &ctx, const parms_id_type &id, const char *what)
{
    auto cd = ctx.get_context_data(id);
    if (!cd) throw std::invalid_argument(std::string(what) + " is not valid for encryption parameters");
    return { cd->parms().coeff_modulus().size(), cd->parms().poly_modulus_degree(),
             (double)cd->total_coeff_modulus_bit_count(), cd };
}

Level check_ct(const SEALContext &ctx, const Ciphertext &ct, const char *what)
{
    Level lv = level_of(ctx, ct.parms_id(), what);
    if (ct.size() < 2 || ct.coeff_modulus_size() != lv.L || ct.store().words() != ct.size() * lv.L * lv.n ||
        ct.store().engine() != ctx.engine())
        throw std::invalid_argument(std::string(what) + " is not valid for encryption parameters");
    return lv;
}

// is_scale_within_bounds (evaluator.cpp): 0 < scale and log2(scale) < total bits of the level
void check_scale(double scale, const Level &lv)
{
    if (scale <= 0 || static_cast<int>(std::log2(scale)) >= (int)lv.total_bits)
        throw std::invalid_argument("scale out of bounds (2^" + std::to_string(std::log2(scale)) + " at " +
                                    std::to_string(lv.L) + " limbs, " + std::to_string(lv.total_bits) + " bits)");
}
} // namespace

struct Evaluator::VecCache
{
    struct Key
    {
        std::uint64_t hi, lo;
        std::size_t limbs;
        std::uint64_t scale_bits;
        bool operator<(const Key &o) const
        {
            if (hi != o.hi) return hi < o.hi;
            if (lo != o.lo) return lo < o.lo;
            if (limbs != o.limbs) return limbs < o.limbs;
            return scale_bits < o.scale_bits;
        }
    };
    std::mutex mu;
    std::map<Key, Plaintext> entries;
    std::size_t bytes = 0;
    std::size_t cap = [] {
        const char *e = std::getenv("MHE_VEC_CACHE_GB");
        const double gb = e ? std::atof(e) : 48.0;
        return gb > 0 ? (std::size_t)(gb * 1e9) : (std::size_t)0;
    }();
};

Evaluator::Evaluator(const SEALContext &context, CKKSEncoder &encoder)
    : context_(context), encoder_(encoder), vcache_(std::make_shared<VecCache>())
{
    if (!context.parameters_set()) throw std::invalid_argument("encryption parameters are not set correctly");
}

const Plaintext &Evaluator::cached_vector_plain(const Ciphertext &encrypted, std::uint64_t id_hi, std::uint64_t id_lo,
                                                const std::function<std::vector<double>()> &make,
                                                Plaintext &scratch) const
{
    const Level lv = check_ct(context_, encrypted, "encrypted");
    std::uint64_t sb;
    const double sc = encrypted.scale();
    std::memcpy(&sb, &sc, sizeof sb);
    const VecCache::Key key{ id_hi, id_lo, lv.L, sb };
    VecCache &vc = *vcache_;
    const std::size_t sz = lv.L * lv.n * sizeof(std::uint64_t);
    bool fits;
    {
        std::lock_guard<std::mutex> g(vc.mu);
        auto it = vc.entries.find(key);
        if (it != vc.entries.end()) return it->second;
        fits = vc.cap > 0 && vc.bytes + sz <= vc.cap;
    }
    if (!fits)
    {
        encode_vector_for(encrypted, make(), scratch);
        return scratch;
    }
    Plaintext pt;
    encode_vector_for(encrypted, make(), pt);
    std::lock_guard<std::mutex> g(vc.mu);
    auto r = vc.entries.emplace(key, std::move(pt)); // another thread may have made the same entry
    if (r.second) vc.bytes += sz;
    return r.first->second;
}

std::size_t Evaluator::vector_cache_entries() const
{
    std::lock_guard<std::mutex> g(vcache_->mu);
    return vcache_->entries.size();
}

std::size_t Evaluator::vector_cache_bytes() const
{
    std::lock_guard<std::mutex> g(vcache_->mu);
    return vcache_->bytes;
}

std::size_t Evaluator::limbs_of(const parms_id_type &id) const
{
    return level_of(context_, id, "parms_id").L;
}

namespace
{
// destination takes src's level, size, scale and form; its previous contents are not kept (no copy)
void fresh_dest(const SEALContext &ctx, const Ciphertext &src, Ciphertext &dst, std::size_t size)
{
    dst.resize(ctx, src.parms_id(), 0);
    dst.resize(size);
    dst.scale() = src.scale();
    dst.is_ntt_form() = src.is_ntt_form();
}
} // namespace

void Evaluator::negate_inplace(Ciphertext &encrypted) const
{
    TRACE_OP("negate", trace::ct(encrypted), trace::ct(encrypted));
    // evaluator.cpp:78-101
    Level lv = check_ct(context_, encrypted, "encrypted");
    void *s = context_.stream();
    std::uint64_t *p = encrypted.store().dev_write(s);
    chk(mhe_negate(context_.engine(), p, p, (int)encrypted.size(), (int)lv.L, s));
}

void Evaluator::negate(const Ciphertext &encrypted, Ciphertext &destination) const
{
    TRACE_OP("negate", trace::ct(destination), trace::ct(encrypted));
    if (&encrypted == &destination) return negate_inplace(destination);
    Level lv = check_ct(context_, encrypted, "encrypted");
    void *s = context_.stream();
    fresh_dest(context_, encrypted, destination, encrypted.size());
    chk(mhe_negate(context_.engine(), encrypted.store().dev_read(s), destination.store().dev_write(s, true),
                   (int)encrypted.size(), (int)lv.L, s));
}

namespace
{
void check_pair(const SEALContext &ctx, const Ciphertext &a, const Ciphertext &b, bool scales)
{
    check_ct(ctx, a, "encrypted1");
    check_ct(ctx, b, "encrypted2");
    if (a.parms_id() != b.parms_id()) throw std::invalid_argument("encrypted1 and encrypted2 parameter mismatch");
    if (a.is_ntt_form() != b.is_ntt_form()) throw std::invalid_argument("NTT form mismatch");
    if (scales && !are_close(a.scale(), b.scale())) throw std::invalid_argument("scale mismatch");
}
} // namespace

void Evaluator::add_inplace(Ciphertext &encrypted1, const Ciphertext &encrypted2) const
{
    TRACE_OP("add", trace::ct(encrypted1), trace::ct(encrypted1), trace::ct(encrypted2));
    // evaluator.cpp:103-164
    check_pair(context_, encrypted1, encrypted2, true);
    const std::size_t L = encrypted1.coeff_modulus_size(), n = encrypted1.poly_modulus_degree();
    const std::size_t s1 = encrypted1.size(), s2 = encrypted2.size(), mn = std::min(s1, s2);
    void *s = context_.stream();
    if (s1 < s2) encrypted1.resize(context_, encrypted1.parms_id(), s2);
    const std::uint64_t *b = encrypted2.store().dev_read(s);
    std::uint64_t *a = encrypted1.store().dev_write(s);
    chk(mhe_add(context_.engine(), a, b, a, (int)mn, (int)L, s));
    if (s1 < s2) chk(mhe_memcpy_d2d(context_.engine(), a + mn * L * n, b + mn * L * n, (s2 - mn) * L * n * 8, s));
}

void Evaluator::add(const Ciphertext &encrypted1, const Ciphertext &encrypted2, Ciphertext &destination) const
{
    TRACE_OP("add", trace::ct(destination), trace::ct(encrypted1), trace::ct(encrypted2));
    if (&encrypted2 == &destination)
        add_inplace(destination, encrypted1);
    else if (&encrypted1 != &destination && encrypted1.size() == encrypted2.size())
    {
        // SEAL copies encrypted1 then adds; writing the sum directly saves a pass over HBM
        check_pair(context_, encrypted1, encrypted2, true);
        void *s = context_.stream();
        destination.resize(context_, encrypted1.parms_id(), encrypted1.size());
        const std::uint64_t *a = encrypted1.store().dev_read(s), *b = encrypted2.store().dev_read(s);
        chk(mhe_add(context_.engine(), a, b, destination.store().dev_write(s, true), (int)encrypted1.size(),
                    (int)encrypted1.coeff_modulus_size(), s));
        destination.scale() = encrypted1.scale();
        destination.is_ntt_form() = encrypted1.is_ntt_form();
    }
    else
    {
        destination = encrypted1;
        add_inplace(destination, encrypted2);
    }
}

void Evaluator::add_many(const std::vector<Ciphertext> &encrypteds, Ciphertext &destination) const
{
    // evaluator.cpp:166-185
    if (encrypteds.empty()) throw std::invalid_argument("encrypteds cannot be empty");
    for (auto &e : encrypteds)
        if (&e == &destination) throw std::invalid_argument("encrypteds must be different from destination");
    destination = encrypteds[0];
    for (std::size_t i = 1; i < encrypteds.size(); i++) add_inplace(destination, encrypteds[i]);
}

void Evaluator::sub_inplace(Ciphertext &encrypted1, const Ciphertext &encrypted2) const
{
    TRACE_OP("sub", trace::ct(encrypted1), trace::ct(encrypted1), trace::ct(encrypted2));
    // evaluator.cpp:187-246
    check_pair(context_, encrypted1, encrypted2, true);
    const std::size_t L = encrypted1.coeff_modulus_size(), n = encrypted1.poly_modulus_degree();
    const std::size_t s1 = encrypted1.size(), s2 = encrypted2.size(), mn = std::min(s1, s2);
    void *s = context_.stream();
    if (s1 < s2) encrypted1.resize(context_, encrypted1.parms_id(), s2);
    const std::uint64_t *b = encrypted2.store().dev_read(s);
    std::uint64_t *a = encrypted1.store().dev_write(s);
    chk(mhe_sub(context_.engine(), a, b, a, (int)mn, (int)L, s));
    if (s1 < s2)
        chk(mhe_negate(context_.engine(), b + mn * L * n, a + mn * L * n, (int)(s2 - mn), (int)L, s));
}

void Evaluator::sub(const Ciphertext &encrypted1, const Ciphertext &encrypted2, Ciphertext &destination) const
{
    TRACE_OP("sub", trace::ct(destination), trace::ct(encrypted1), trace::ct(encrypted2));
    if (&encrypted2 == &destination)
    {
        sub_inplace(destination, encrypted1);
        negate_inplace(destination);
    }
    else
    {
        destination = encrypted1;
        sub_inplace(destination, encrypted2);
    }
}

void Evaluator::multiply_inplace(Ciphertext &encrypted1, const Ciphertext &encrypted2, MemoryPoolHandle) const
{
    TRACE_OP("multiply", trace::ct(encrypted1), trace::ct(encrypted1), trace::ct(encrypted2));
    // evaluator.cpp:248-285, ckks_multiply :673-773 (size 2 x size 2 -> 3)
    check_ct(context_, encrypted1, "encrypted1");
    check_ct(context_, encrypted2, "encrypted2");
    if (encrypted1.parms_id() != encrypted2.parms_id())
        throw std::invalid_argument("encrypted1 and encrypted2 parameter mismatch");
    if (!encrypted1.is_ntt_form() || !encrypted2.is_ntt_form())
        throw std::invalid_argument("encrypted1 or encrypted2 must be in NTT form");
    if (encrypted1.size() != 2 || encrypted2.size() != 2)
        throw std::logic_error("only size-2 ciphertexts are multiplied (relinearize first)");
    Level lv = level_of(context_, encrypted1.parms_id(), "encrypted1");
    const double new_scale = encrypted1.scale() * encrypted2.scale();
    check_scale(new_scale, lv);
    void *s = context_.stream();
    PolyStore out;
    out.bind(context_);
    out.resize_words(3 * lv.L * lv.n, false);
    const std::uint64_t *a = encrypted1.store().dev_read(s), *b = encrypted2.store().dev_read(s);
    chk(mhe_ct_multiply(context_.engine(), a, b, out.dev_write(s, true), (int)lv.L, s));
    encrypted1.store() = std::move(out);
    encrypted1.resize(3);
    encrypted1.scale() = new_scale;
}

void Evaluator::multiply(const Ciphertext &encrypted1, const Ciphertext &encrypted2, Ciphertext &destination,
                         MemoryPoolHandle) const
{
    TRACE_OP("multiply", trace::ct(destination), trace::ct(encrypted1), trace::ct(encrypted2));
    if (&encrypted1 != &destination && &encrypted2 != &destination && encrypted1.size() == 2 &&
        encrypted2.size() == 2)
    {
        // ckks_multiply into a fresh destination (SEAL copies encrypted1 first)
        check_ct(context_, encrypted1, "encrypted1");
        check_ct(context_, encrypted2, "encrypted2");
        if (encrypted1.parms_id() != encrypted2.parms_id())
            throw std::invalid_argument("encrypted1 and encrypted2 parameter mismatch");
        if (!encrypted1.is_ntt_form() || !encrypted2.is_ntt_form())
            throw std::invalid_argument("encrypted1 or encrypted2 must be in NTT form");
        Level lv = level_of(context_, encrypted1.parms_id(), "encrypted1");
        const double new_scale = encrypted1.scale() * encrypted2.scale();
        check_scale(new_scale, lv);
        void *s = context_.stream();
        fresh_dest(context_, encrypted1, destination, 3);
        const std::uint64_t *a = encrypted1.store().dev_read(s), *b = encrypted2.store().dev_read(s);
        chk(mhe_ct_multiply(context_.engine(), a, b, destination.store().dev_write(s, true), (int)lv.L, s));
        destination.scale() = new_scale;
        return;
    }
    if (&encrypted2 == &destination)
        multiply_inplace(destination, encrypted1);
    else
    {
        destination = encrypted1;
        multiply_inplace(destination, encrypted2);
    }
}

void Evaluator::multiply_many(const std::vector<Ciphertext> &encrypteds, const RelinKeys &, Ciphertext &destination,
                              MemoryPoolHandle) const
{
    // evaluator.cpp:1468-1543: BFV only in SEAL 3.6
    if (encrypteds.empty()) throw std::invalid_argument("encrypteds vector must not be empty");
    for (auto &e : encrypteds)
        if (&e == &destination) throw std::invalid_argument("encrypteds must be different from destination");
    level_of(context_, encrypteds[0].parms_id(), "encrypteds");
    throw std::logic_error("unsupported scheme");
}

void Evaluator::exponentiate_inplace(Ciphertext &encrypted, std::uint64_t exponent, const RelinKeys &relin_keys,
                                     MemoryPoolHandle) const
{
    // evaluator.cpp:1545-1576 (delegates to multiply_many: BFV only)
    level_of(context_, encrypted.parms_id(), "encrypted");
    if (!context_.get_context_data(relin_keys.parms_id()))
        throw std::invalid_argument("relin_keys is not valid for encryption parameters");
    if (exponent == 0) throw std::invalid_argument("exponent cannot be 0");
    if (exponent == 1) return;
    throw std::logic_error("unsupported scheme");
}

void Evaluator::square_inplace(Ciphertext &encrypted, MemoryPoolHandle) const
{
    TRACE_OP("square", trace::ct(encrypted), trace::ct(encrypted));
    // evaluator.cpp:816-845, ckks_square :1000-1059
    Level lv = check_ct(context_, encrypted, "encrypted");
    if (!encrypted.is_ntt_form()) throw std::invalid_argument("encrypted must be in NTT form");
    if (encrypted.size() != 2) throw std::logic_error("only size-2 ciphertexts are squared (relinearize first)");
    const double new_scale = encrypted.scale() * encrypted.scale();
    check_scale(new_scale, lv);
    void *s = context_.stream();
    PolyStore out;
    out.bind(context_);
    out.resize_words(3 * lv.L * lv.n, false);
    chk(mhe_ct_square(context_.engine(), encrypted.store().dev_read(s), out.dev_write(s, true), (int)lv.L, s));
    encrypted.store() = std::move(out);
    encrypted.resize(3);
    encrypted.scale() = new_scale;
}

void Evaluator::square(const Ciphertext &encrypted, Ciphertext &destination, MemoryPoolHandle) const
{
    TRACE_OP("square", trace::ct(destination), trace::ct(encrypted));
    if (&encrypted == &destination) return square_inplace(destination);
    Level lv = check_ct(context_, encrypted, "encrypted");
    if (!encrypted.is_ntt_form()) throw std::invalid_argument("encrypted must be in NTT form");
    if (encrypted.size() != 2) throw std::logic_error("only size-2 ciphertexts are squared (relinearize first)");
    const double new_scale = encrypted.scale() * encrypted.scale();
    check_scale(new_scale, lv);
    void *s = context_.stream();
    fresh_dest(context_, encrypted, destination, 3);
    chk(mhe_ct_square(context_.engine(), encrypted.store().dev_read(s), destination.store().dev_write(s, true),
                      (int)lv.L, s));
    destination.scale() = new_scale;
}

void Evaluator::switch_key(Ciphertext &encrypted, const std::uint64_t *target, const KSwitchKeys &keys,
                           std::size_t index) const
{
    // switch_key_inplace (evaluator.cpp:2281-2525): ct[0..1] += KS(target)
    const std::size_t L = encrypted.coeff_modulus_size();
    void *s = context_.stream();
    std::size_t kl = 0;
    const std::uint64_t *key = keys.key_for(index, L, s, kl);
    std::uint64_t *ct = encrypted.store().dev_write(s);
    chk(mhe_switch_key(context_.engine(), ct, target, key, (int)kl, (int)L, s));
}

void Evaluator::relinearize_inplace(Ciphertext &encrypted, const RelinKeys &relin_keys, MemoryPoolHandle) const
{
    if (tl_ls || fiber_merging())
    {
        LsOp op;
        op.kind = LsOp::RELIN;
        op.out = { &encrypted };
        op.rk = &relin_keys;
        if (lockstep_submit(op)) return;
    }
    TRACE_OP("relinearize", trace::ct(encrypted), trace::ct(encrypted));
    // relinearize_internal (evaluator.cpp:1061-1116)
    Level lv = check_ct(context_, encrypted, "encrypted");
    if (relin_keys.parms_id() != context_.key_parms_id())
        throw std::invalid_argument("relin_keys is not valid for encryption parameters");
    if (!encrypted.is_ntt_form()) throw std::invalid_argument("encrypted must be in NTT form");
    void *s = context_.stream();
    std::size_t size = encrypted.size();
    if (size == 3)
    {
        std::size_t kl = 0;
        const std::uint64_t *key = relin_keys.key_for(RelinKeys::get_index(2), lv.L, s, kl);
        std::uint64_t *ct = encrypted.store().dev_write(s);
        chk(mhe_relinearize(context_.engine(), ct, key, (int)kl, (int)lv.L, s));
        size = 2;
    }
    while (size > 2)
    {
        // fold the last component with the key for s^(size-1)
        std::uint64_t *ct = encrypted.store().dev_write(s);
        switch_key(encrypted, ct + (size - 1) * lv.L * lv.n, relin_keys, RelinKeys::get_index(size - 1));
        size--;
    }
    encrypted.resize(size);
}

void Evaluator::relinearize(const Ciphertext &encrypted, const RelinKeys &relin_keys, Ciphertext &destination,
                            MemoryPoolHandle) const
{
    TRACE_OP("relinearize", trace::ct(destination), trace::ct(encrypted));
    destination = encrypted;
    relinearize_inplace(destination, relin_keys);
}

void Evaluator::mod_switch_to_next_inplace(Ciphertext &encrypted, MemoryPoolHandle) const
{
    TRACE_OP("mod_switch", trace::ct(encrypted), trace::ct(encrypted));
    // mod_switch_drop_to_next (evaluator.cpp:1183-1246) -- CKKS mod_switch_to_next
    Level lv = check_ct(context_, encrypted, "encrypted");
    if (!encrypted.is_ntt_form()) throw std::invalid_argument("CKKS encrypted must be in NTT form");
    auto next = lv.cd->next_context_data();
    if (!next) throw std::invalid_argument("end of modulus switching chain reached");
    void *s = context_.stream();
    const std::size_t size = encrypted.size();
    PolyStore out;
    out.bind(context_);
    out.resize_words(size * (lv.L - 1) * lv.n, false);
    chk(mhe_mod_switch_drop(context_.engine(), encrypted.store().dev_read(s), out.dev_write(s, true), (int)size,
                            (int)lv.L, s));
    const double scale = encrypted.scale();
    encrypted.store() = std::move(out);
    encrypted.resize(context_, next->parms_id(), size);
    encrypted.scale() = scale;
}

void Evaluator::mod_switch_to_next(const Ciphertext &encrypted, Ciphertext &destination, MemoryPoolHandle) const
{
    TRACE_OP("mod_switch", trace::ct(destination), trace::ct(encrypted));
    destination = encrypted;
    mod_switch_to_next_inplace(destination);
}

void Evaluator::mod_switch_to_next_inplace(Plaintext &plain) const
{
    TRACE_OP("pt_mod_switch", trace::pt(plain), trace::pt(plain));
    // mod_switch_drop_to_next(Plaintext) (evaluator.cpp:1248-1281)
    if (!plain.is_ntt_form()) throw std::invalid_argument("plain is not in NTT form");
    Level lv = level_of(context_, plain.parms_id(), "plain");
    auto next = lv.cd->next_context_data();
    if (!next) throw std::invalid_argument("end of modulus switching chain reached");
    const double scale = plain.scale();
    plain.set_level(context_, next->parms_id(), lv.L - 1); // shrinking keeps the first L-1 limbs
    plain.scale() = scale;
}

void Evaluator::mod_switch_to_inplace(Ciphertext &encrypted, parms_id_type parms_id, MemoryPoolHandle) const
{
    TRACE_OP("mod_switch", trace::ct(encrypted), trace::ct(encrypted));
    // evaluator.cpp:1326-1348
    Level cur = check_ct(context_, encrypted, "encrypted");
    auto target = context_.get_context_data(parms_id);
    if (!target) throw std::invalid_argument("parms_id is not valid for encryption parameters");
    if (cur.cd->chain_index() < target->chain_index())
        throw std::invalid_argument("cannot switch to higher level modulus");
    if (encrypted.parms_id() == parms_id) return;
    if (!encrypted.is_ntt_form()) throw std::invalid_argument("CKKS encrypted must be in NTT form");
    // all dropped limbs at once: copy the kept prefix of every component
    const std::size_t L2 = target->parms().coeff_modulus().size(), n = cur.n, size = encrypted.size();
    void *s = context_.stream();
    PolyStore out;
    out.bind(context_);
    out.resize_words(size * L2 * n, false);
    std::uint64_t *d = out.dev_write(s, true);
    const std::uint64_t *p = encrypted.store().dev_read(s);
    for (std::size_t k = 0; k < size; k++)
        chk(mhe_memcpy_d2d(context_.engine(), d + k * L2 * n, p + k * cur.L * n, L2 * n * 8, s));
    const double scale = encrypted.scale();
    encrypted.store() = std::move(out);
    encrypted.resize(context_, parms_id, size);
    encrypted.scale() = scale;
}

void Evaluator::mod_switch_to(const Ciphertext &encrypted, parms_id_type parms_id, Ciphertext &destination,
                              MemoryPoolHandle) const
{
    TRACE_OP("mod_switch", trace::ct(destination), trace::ct(encrypted));
    destination = encrypted;
    mod_switch_to_inplace(destination, parms_id);
}

void Evaluator::mod_switch_to_inplace(Plaintext &plain, parms_id_type parms_id) const
{
    TRACE_OP("pt_mod_switch", trace::pt(plain), trace::pt(plain));
    // evaluator.cpp:1350-1376
    auto cur = context_.get_context_data(plain.parms_id());
    auto target = context_.get_context_data(parms_id);
    if (!cur) throw std::invalid_argument("plain is not valid for encryption parameters");
    if (!target) throw std::invalid_argument("parms_id is not valid for encryption parameters");
    if (!plain.is_ntt_form()) throw std::invalid_argument("plain is not in NTT form");
    if (cur->chain_index() < target->chain_index())
        throw std::invalid_argument("cannot switch to higher level modulus");
    if (plain.parms_id() == parms_id) return;
    const std::size_t L2 = target->parms().coeff_modulus().size();
    const double scale = plain.scale();
    plain.set_level(context_, parms_id, L2); // shrinking keeps the prefix limbs
    plain.scale() = scale;
}

void Evaluator::rescale_to_next(const Ciphertext &encrypted, Ciphertext &destination, MemoryPoolHandle) const
{
    TRACE_OP("rescale", trace::ct(destination), trace::ct(encrypted));
    // evaluator.cpp:1378-1414, mod_switch_scale_to_next :1118-1181
    Level lv = check_ct(context_, encrypted, "encrypted");
    if (context_.last_parms_id() == encrypted.parms_id())
        throw std::invalid_argument("end of modulus switching chain reached");
    if (!encrypted.is_ntt_form()) throw std::invalid_argument("CKKS encrypted must be in NTT form");
    auto next = lv.cd->next_context_data();
    const double q_last = (double)lv.cd->parms().coeff_modulus().back().value();
    const double new_scale = encrypted.scale() / q_last;
    Level nl = level_of(context_, next->parms_id(), "parms_id");
    check_scale(new_scale, nl);
    void *s = context_.stream();
    const std::size_t size = encrypted.size();
    PolyStore out;
    out.bind(context_);
    out.resize_words(size * (lv.L - 1) * lv.n, false);
    chk(mhe_rescale_to_next(context_.engine(), encrypted.store().dev_read(s), out.dev_write(s, true), (int)size,
                            (int)lv.L, s));
    const bool ntt = encrypted.is_ntt_form();
    destination.store() = std::move(out);
    destination.resize(context_, next->parms_id(), size);
    destination.scale() = new_scale;
    destination.is_ntt_form() = ntt;
}

void Evaluator::rescale_to_next_inplace(Ciphertext &encrypted, MemoryPoolHandle) const
{
    if (tl_ls || fiber_merging())
    {
        LsOp op;
        op.kind = LsOp::RESC;
        op.out = { &encrypted };
        if (lockstep_submit(op)) return;
    }
    rescale_to_next(encrypted, encrypted);
}

void Evaluator::rescale_to_inplace(Ciphertext &encrypted, parms_id_type parms_id, MemoryPoolHandle) const
{
    TRACE_OP("rescale", trace::ct(encrypted), trace::ct(encrypted));
    // evaluator.cpp:1416-1466
    Level cur = check_ct(context_, encrypted, "encrypted");
    auto target = context_.get_context_data(parms_id);
    if (!target) throw std::invalid_argument("parms_id is not valid for encryption parameters");
    if (cur.cd->chain_index() < target->chain_index())
        throw std::invalid_argument("cannot switch to higher level modulus");
    while (encrypted.parms_id() != parms_id) rescale_to_next(encrypted, encrypted);
}

void Evaluator::multiply_plain_inplace(Ciphertext &encrypted, const Plaintext &plain, MemoryPoolHandle) const
{
    multiply_plain(encrypted, plain, encrypted);
}

void Evaluator::multiply_plain(const Ciphertext &encrypted, const Plaintext &plain, Ciphertext &destination,
                               MemoryPoolHandle) const
{
    TRACE_OP("multiply_plain", trace::ct(destination), trace::ct(encrypted), trace::pt(plain));
    // evaluator.cpp:1726-1761, multiply_plain_ntt :1891-1930 (out of place: no copy of encrypted)
    Level lv = check_ct(context_, encrypted, "encrypted");
    if (plain.is_ntt_form()) level_of(context_, plain.parms_id(), "plain");
    if (encrypted.is_ntt_form() != plain.is_ntt_form()) throw std::invalid_argument("NTT form mismatch");
    if (!encrypted.is_ntt_form()) throw std::invalid_argument("encrypted must be in NTT form");
    if (encrypted.parms_id() != plain.parms_id())
        throw std::invalid_argument("encrypted_ntt and plain_ntt parameter mismatch");
    const double new_scale = encrypted.scale() * plain.scale();
    check_scale(new_scale, lv);
    void *s = context_.stream();
    const std::uint64_t *b = plain.store().dev_read(s);
    if (&encrypted == &destination)
    {
        std::uint64_t *a = destination.store().dev_write(s);
        chk(mhe_multiply_plain(context_.engine(), a, b, a, (int)destination.size(), (int)lv.L, s));
    }
    else
    {
        fresh_dest(context_, encrypted, destination, encrypted.size());
        const std::uint64_t *a = encrypted.store().dev_read(s);
        chk(mhe_multiply_plain(context_.engine(), a, b, destination.store().dev_write(s, true),
                               (int)encrypted.size(), (int)lv.L, s));
    }
    destination.scale() = new_scale;
}

namespace
{
void add_sub_plain(const SEALContext &ctx, Ciphertext &encrypted, const Plaintext &plain, bool sub)
{
    // evaluator.cpp:1578-1724 (CKKS branch): component 0 +-= plain
    Level lv = check_ct(ctx, encrypted, "encrypted");
    if (encrypted.is_ntt_form() != plain.is_ntt_form()) throw std::invalid_argument("NTT form mismatch");
    if (encrypted.parms_id() != plain.parms_id())
        throw std::invalid_argument("encrypted and plain parameter mismatch");
    if (!are_close(encrypted.scale(), plain.scale())) throw std::invalid_argument("scale mismatch");
    void *s = ctx.stream();
    const std::uint64_t *b = plain.store().dev_read(s);
    std::uint64_t *a = encrypted.store().dev_write(s);
    if (sub)
        chk(mhe_sub(ctx.engine(), a, b, a, 1, (int)lv.L, s));
    else
        chk(mhe_add(ctx.engine(), a, b, a, 1, (int)lv.L, s));
}
} // namespace

void Evaluator::add_plain_inplace(Ciphertext &encrypted, const Plaintext &plain) const
{
    TRACE_OP("add_plain", trace::ct(encrypted), trace::ct(encrypted), trace::pt(plain));
    add_sub_plain(context_, encrypted, plain, false);
}

void Evaluator::add_plain(const Ciphertext &encrypted, const Plaintext &plain, Ciphertext &destination) const
{
    TRACE_OP("add_plain", trace::ct(destination), trace::ct(encrypted), trace::pt(plain));
    destination = encrypted;
    add_plain_inplace(destination, plain);
}

void Evaluator::sub_plain_inplace(Ciphertext &encrypted, const Plaintext &plain) const
{
    TRACE_OP("sub_plain", trace::ct(encrypted), trace::ct(encrypted), trace::pt(plain));
    add_sub_plain(context_, encrypted, plain, true);
}

void Evaluator::sub_plain(const Ciphertext &encrypted, const Plaintext &plain, Ciphertext &destination) const
{
    TRACE_OP("sub_plain", trace::ct(destination), trace::ct(encrypted), trace::pt(plain));
    destination = encrypted;
    sub_plain_inplace(destination, plain);
}

void Evaluator::transform_to_ntt_inplace(Ciphertext &encrypted) const
{
    TRACE_OP("ntt_fwd", trace::ct(encrypted), trace::ct(encrypted));
    // evaluator.cpp:2025-2071
    Level lv = check_ct(context_, encrypted, "encrypted");
    if (encrypted.is_ntt_form()) throw std::invalid_argument("encrypted is already in NTT form");
    void *s = context_.stream();
    chk(mhe_ntt_forward(context_.engine(), encrypted.store().dev_write(s), (int)encrypted.size(), (int)lv.L, 0, s));
    encrypted.is_ntt_form() = true;
}

void Evaluator::transform_from_ntt_inplace(Ciphertext &encrypted) const
{
    TRACE_OP("ntt_inv", trace::ct(encrypted), trace::ct(encrypted));
    // evaluator.cpp:2073-2118
    Level lv = check_ct(context_, encrypted, "encrypted");
    if (!encrypted.is_ntt_form()) throw std::invalid_argument("encrypted is not in NTT form");
    void *s = context_.stream();
    chk(mhe_ntt_inverse(context_.engine(), encrypted.store().dev_write(s), (int)encrypted.size(), (int)lv.L, 0, s));
    encrypted.is_ntt_form() = false;
}

void Evaluator::apply_galois_inplace(Ciphertext &encrypted, std::uint32_t galois_elt, const GaloisKeys &galois_keys,
                                     MemoryPoolHandle) const
{
    TRACE_OP("galois", trace::ct(encrypted), trace::ct(encrypted));
    TRACE_EXTRA("\"elt\": " + std::to_string(galois_elt));
    // evaluator.cpp:2120-2222
    Level lv = check_ct(context_, encrypted, "encrypted");
    if (galois_keys.parms_id() != context_.key_parms_id())
        throw std::invalid_argument("galois_keys is not valid for encryption parameters");
    if (!(galois_elt & 1) || galois_elt >= 2 * lv.n) throw std::invalid_argument("Galois element is not valid");
    if (encrypted.size() > 2) throw std::invalid_argument("encrypted size must be 2");
    if (!encrypted.is_ntt_form()) throw std::invalid_argument("encrypted must be in NTT form");
    if (!galois_keys.has_key(galois_elt)) throw std::invalid_argument("Galois key not present");
    void *s = context_.stream();
    std::size_t kl = 0;
    const std::uint64_t *key = galois_keys.key_for(GaloisKeys::get_index(galois_elt), lv.L, s, kl);
    chk(mhe_apply_galois(context_.engine(), encrypted.store().dev_write(s), galois_elt, key, (int)kl, (int)lv.L, s));
}

void Evaluator::rotate_internal(Ciphertext &encrypted, int steps, const GaloisKeys &galois_keys) const
{
    // evaluator.cpp:2224-2279
    Level lv = level_of(context_, encrypted.parms_id(), "encrypted");
    if (galois_keys.parms_id() != context_.key_parms_id())
        throw std::invalid_argument("galois_keys is not valid for encryption parameters");
    if (steps == 0) return;
    const int log_n = __builtin_ctzll(lv.n);
    const std::uint32_t elt = mhe_galois_elt_from_step(log_n, steps);
    if (!elt) throw std::invalid_argument("step count too large");
    if (galois_keys.has_key(elt))
    {
        apply_galois_inplace(encrypted, elt, galois_keys);
        return;
    }
    // NAF decomposition (util/numth.h:22-42)
    std::vector<int> naf;
    {
        const bool sign = steps < 0;
        int v = std::abs(steps);
        for (int i = 0; v; i++)
        {
            const int zi = (v & 1) ? 2 - (v & 3) : 0;
            v = (v - zi) >> 1;
            if (zi) naf.push_back((sign ? -zi : zi) * (1 << i));
        }
    }
    if (naf.size() == 1) throw std::invalid_argument("Galois key not present");
    for (int st : naf)
        if ((std::size_t)std::abs(st) != (lv.n >> 1)) rotate_internal(encrypted, st, galois_keys);
}

void Evaluator::rotate_vector_inplace(Ciphertext &encrypted, int steps, const GaloisKeys &galois_keys,
                                      MemoryPoolHandle) const
{
    if (tl_ls || fiber_merging())
    {
        LsOp op;
        op.kind = LsOp::ROT;
        op.in = { &encrypted };
        op.steps = { steps };
        op.out = { &encrypted };
        op.gk = &galois_keys;
        if (lockstep_submit(op)) return;
    }
    TRACE_OP("rotate", trace::ct(encrypted), trace::ct(encrypted));
    TRACE_EXTRA("\"step\": " + std::to_string(steps));
    rotate_internal(encrypted, steps, galois_keys);
}

void Evaluator::apply_galois_to(const Ciphertext &encrypted, std::uint32_t galois_elt, const GaloisKeys &galois_keys,
                                Ciphertext &destination) const
{
    TRACE_OP("galois", trace::ct(destination), trace::ct(encrypted));
    TRACE_EXTRA("\"elt\": " + std::to_string(galois_elt));
    // apply_galois_inplace (evaluator.cpp:2120-2222) reading encrypted and writing destination
    Level lv = check_ct(context_, encrypted, "encrypted");
    if (galois_keys.parms_id() != context_.key_parms_id())
        throw std::invalid_argument("galois_keys is not valid for encryption parameters");
    if (!(galois_elt & 1) || galois_elt >= 2 * lv.n) throw std::invalid_argument("Galois element is not valid");
    if (encrypted.size() > 2) throw std::invalid_argument("encrypted size must be 2");
    if (!encrypted.is_ntt_form()) throw std::invalid_argument("encrypted must be in NTT form");
    if (!galois_keys.has_key(galois_elt)) throw std::invalid_argument("Galois key not present");
    void *s = context_.stream();
    std::size_t kl = 0;
    const std::uint64_t *key = galois_keys.key_for(GaloisKeys::get_index(galois_elt), lv.L, s, kl);
    fresh_dest(context_, encrypted, destination, 2);
    chk(mhe_apply_galois_to(context_.engine(), encrypted.store().dev_read(s), destination.store().dev_write(s, true),
                            galois_elt, key, (int)kl, (int)lv.L, s));
}

void Evaluator::rotate_vector(const Ciphertext &encrypted, int steps, const GaloisKeys &galois_keys,
                              Ciphertext &destination, MemoryPoolHandle) const
{
    if (tl_ls || fiber_merging())
    {
        LsOp op;
        op.kind = LsOp::ROT;
        op.in = { &encrypted };
        op.steps = { steps };
        op.out = { &destination };
        op.gk = &galois_keys;
        if (lockstep_submit(op)) return;
    }
    TRACE_OP("rotate", trace::ct(destination), trace::ct(encrypted));
    TRACE_EXTRA("\"step\": " + std::to_string(steps));
    if (&encrypted != &destination && steps != 0)
    {
        Level lv = level_of(context_, encrypted.parms_id(), "encrypted");
        if (galois_keys.parms_id() != context_.key_parms_id())
            throw std::invalid_argument("galois_keys is not valid for encryption parameters");
        const std::uint32_t elt = mhe_galois_elt_from_step(__builtin_ctzll(lv.n), steps);
        if (!elt) throw std::invalid_argument("step count too large");
        if (galois_keys.has_key(elt)) return apply_galois_to(encrypted, elt, galois_keys, destination);
    }
    destination = encrypted;
    rotate_vector_inplace(destination, steps, galois_keys);
}

// ------------------------------------------------------------------------------ batching switch
namespace
{
std::atomic<bool> g_batched{ true };
}
void set_batched_launches(bool on)
{
    g_batched.store(on);
}
bool batched_launches()
{
    return g_batched.load();
}

// ------------------------------------------------------------------------------ Lockstep
struct Lockstep::Impl
{
    detail::LockstepCore<LsOp> core;
    explicit Impl(std::size_t m) : core(m) {}
    // a round's merged call, run by the member that completes the round (lockstep_core.h)
    static void execute(std::vector<LsOp *> &batch)
    {
        LsDirect d;
        batch[0]->ev->lockstep_execute(batch);
    }
};

// ------------------------------------------------------------------------------ FiberBatch
// Guard pages of the live fiber stacks, lock-free so a signal handler may read them.
static constexpr int kGuardSlots = 4096;
static std::atomic<std::uintptr_t> g_guards[kGuardSlots];
static void guard_list(void *page, bool add)
{
    const std::uintptr_t a = reinterpret_cast<std::uintptr_t>(page);
    for (auto &slot : g_guards)
    {
        std::uintptr_t want = add ? 0 : a;
        if (slot.compare_exchange_strong(want, add ? a : 0)) return;
    }
}

bool fiber_stack_guard(const void *addr)
{
    const std::uintptr_t x = reinterpret_cast<std::uintptr_t>(addr), page = (std::uintptr_t)sysconf(_SC_PAGESIZE);
    for (const auto &slot : g_guards)
    {
        const std::uintptr_t g = slot.load(std::memory_order_relaxed);
        if (g && x >= g && x < g + page) return true;
    }
    return false;
}

struct FiberBatch::Impl
{
    // A fiber's stack: mmap'ed, with a PROT_NONE guard page below it (stacks grow down), so an
    // overflow faults at a known address instead of silently corrupting a neighbouring heap block.
    // Live guard pages are listed in g_guards for fiber_stack_guard (a fault handler's question).
    struct Stack
    {
        void *base = nullptr; // guard page + usable bytes
        std::size_t bytes = 0;
        Stack() = default;
        Stack(const Stack &) = delete;
        Stack &operator=(const Stack &) = delete;
        Stack(Stack &&o) noexcept : base(o.base), bytes(o.bytes) { o.base = nullptr; }
        ~Stack()
        {
            if (!base) return;
            guard_list(base, false);
            munmap(base, bytes);
        }
        void alloc(std::size_t usable)
        {
            const std::size_t page = (std::size_t)sysconf(_SC_PAGESIZE);
            usable = (usable + page - 1) / page * page;
            bytes = usable + page;
            base = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_STACK, -1, 0);
            if (base == MAP_FAILED)
            {
                base = nullptr;
                throw std::runtime_error("FiberBatch: stack allocation failed");
            }
            if (mprotect(base, page, PROT_NONE) != 0) throw std::runtime_error("FiberBatch: guard page failed");
            guard_list(base, true);
        }
        char *sp() const { return static_cast<char *>(base) + (bytes - usable()); }
        std::size_t usable() const { return bytes - (std::size_t)sysconf(_SC_PAGESIZE); }
    };
    struct Fiber
    {
        ucontext_t ctx{};
        Stack stack;
        std::size_t idx = 0;
        bool done = false, blocked = false;
        std::exception_ptr err;
    };
    ucontext_t sched{};
    std::vector<Fiber> fibers;
    Fiber *current = nullptr;
    std::vector<LsOp *> pending;
    // elementwise engine launches parked by the fibers (mhe_set_launch_hook): one per fiber per round
    std::vector<std::pair<mhe_ctx *, mhe_launch *>> launches;
    std::size_t launch_rounds = 0, launches_merged = 0;
    const std::function<void(std::size_t)> *work = nullptr;
    std::size_t rounds = 0, merged = 0;

    // makecontext passes int arguments: the group pointer in two halves
    static void entry(unsigned lo, unsigned hi)
    {
        Impl *g = reinterpret_cast<Impl *>(((std::uintptr_t)hi << 32) | (std::uintptr_t)lo);
        Fiber *f = g->current;
        try
        {
            (*g->work)(f->idx);
        }
        catch (...)
        {
            f->err = std::current_exception();
        }
        f->done = true; // returns to uc_link = the scheduler
    }
    // fiber i's context: its own stack, entry(), back to the scheduler at the end
    __attribute__((noinline)) void init(std::size_t i, std::size_t stack_bytes)
    {
        Fiber &f = fibers[i];
        f.idx = i;
        f.stack.alloc(stack_bytes);
        if (getcontext(&f.ctx) != 0) throw std::runtime_error("FiberBatch: getcontext failed");
        f.ctx.uc_stack.ss_sp = f.stack.sp();
        f.ctx.uc_stack.ss_size = f.stack.usable();
        f.ctx.uc_link = &sched;
        const std::uintptr_t self = reinterpret_cast<std::uintptr_t>(this);
        makecontext(&f.ctx, reinterpret_cast<void (*)()>(&Impl::entry), 2, (unsigned)(self & 0xFFFFFFFFu),
                    (unsigned)(self >> 32));
    }
    // the calling fiber's merge point: park `op` for the round and yield to the scheduler
    void submit(LsOp &op)
    {
        Fiber *f = current;
        pending.push_back(&op);
        f->blocked = true;
        swapcontext(&f->ctx, &sched);
    }
    // the engine's launch hook: inside a fiber the launch is parked for the round (the same-numbered
    // elementwise launches of the fibers run as one batched launch); elsewhere it runs now
    static void launch_hook(mhe_ctx *ctx, mhe_launch *l, void *user)
    {
        Impl *g = static_cast<Impl *>(user);
        if (!g->current || tl_ls_direct > 0)
        {
            mhe_launch *one[1] = { l };
            mhe_launch_run(ctx, one, 1);
            return;
        }
        Fiber *f = g->current;
        g->launches.push_back({ ctx, l });
        f->blocked = true;
        swapcontext(&f->ctx, &g->sched);
    }
    // one round's parked launches, grouped by context (mhe_launch_run batches equal shapes)
    void run_launches()
    {
        while (!launches.empty())
        {
            mhe_ctx *ctx = launches.front().first;
            std::vector<mhe_launch *> ls;
            std::vector<std::pair<mhe_ctx *, mhe_launch *>> rest;
            for (auto &p : launches) (p.first == ctx ? (void)ls.push_back(p.second) : rest.push_back(p));
            mhe_launch_run(ctx, ls.data(), (int)ls.size());
            launch_rounds++;
            if (ls.size() > 1) launches_merged += ls.size();
            launches.swap(rest);
        }
    }
};

namespace
{
thread_local std::size_t tl_fb_rounds = 0, tl_fb_merged = 0;
bool fiber_merging()
{
    return tl_fb && tl_fb->current;
}
} // namespace

void FiberBatch::run(std::size_t count, const std::function<void(std::size_t)> &work, std::size_t stack_bytes)
{
    if (tl_fb) throw std::logic_error("FiberBatch::run: already inside a fiber batch");
    Impl g;
    g.work = &work;
    g.fibers.resize(count);
    for (std::size_t i = 0; i < count; i++) g.init(i, stack_bytes);
    // an alternate signal stack for this thread (if it has none), so a handler installed with
    // SA_ONSTACK can still run -- and report -- when a fiber overflows into its guard page
    struct AltStack
    {
        std::vector<char> mem;
        bool set = false;
        AltStack()
        {
            stack_t cur{};
            if (sigaltstack(nullptr, &cur) == 0 && (cur.ss_flags & SS_DISABLE))
            {
                mem.resize(64 * 1024);
                stack_t st{};
                st.ss_sp = mem.data();
                st.ss_size = mem.size();
                set = sigaltstack(&st, nullptr) == 0;
            }
        }
        ~AltStack()
        {
            if (!set) return;
            stack_t st{};
            st.ss_flags = SS_DISABLE;
            (void)sigaltstack(&st, nullptr);
        }
    } alt;
    tl_fb = &g;
    mhe_set_launch_hook(&Impl::launch_hook, &g);
    struct Reset
    {
        ~Reset()
        {
            mhe_set_launch_hook(nullptr, nullptr);
            tl_fb = nullptr;
        }
    } reset;
    for (;;)
    {
        // every runnable fiber runs to its next merge point (or its end)
        bool ran = false;
        for (auto &f : g.fibers)
            if (!f.done && !f.blocked)
            {
                ran = true;
                g.current = &f;
                swapcontext(&g.sched, &f.ctx);
                g.current = nullptr;
            }
        if (!g.pending.empty() || !g.launches.empty())
        {
            // one round: the parked elementwise launches as batched launches, the parked evaluator
            // calls as one merged call (lockstep_execute), then every parked fiber resumes with its
            // result or its own error (the fibers' data are independent, so the order is free)
            g.run_launches();
            if (!g.pending.empty())
            {
                std::vector<LsOp *> batch;
                batch.swap(g.pending);
                {
                    LsDirect d;
                    batch[0]->ev->lockstep_execute(batch);
                }
                g.rounds++;
                if (batch.size() > 1) g.merged += batch.size();
            }
            for (auto &f : g.fibers) f.blocked = false;
            continue;
        }
        if (!ran) break; // every fiber finished
    }
    tl_fb_rounds = g.rounds + g.launch_rounds;
    tl_fb_merged = g.merged + g.launches_merged;
    for (auto &f : g.fibers)
        if (f.err) std::rethrow_exception(f.err);
}

long FiberBatch::current()
{
    return (tl_fb && tl_fb->current) ? (long)tl_fb->current->idx : -1;
}

std::size_t FiberBatch::last_rounds()
{
    return tl_fb_rounds;
}

std::size_t FiberBatch::last_merged()
{
    return tl_fb_merged;
}

Lockstep::Lockstep(std::size_t members) : impl_(std::make_unique<Impl>(members)) {}
Lockstep::~Lockstep() = default;
std::size_t Lockstep::rounds() const
{
    return impl_->core.rounds();
}
std::size_t Lockstep::merged_calls() const
{
    return impl_->core.merged();
}

Lockstep::Member::Member(Lockstep &group, bool active) : g_(group)
{
    tl_ls_member = group.impl_.get();
    tl_ls = active ? tl_ls_member : nullptr;
}

Lockstep::Active::Active() : saved_(tl_ls) { tl_ls = tl_ls_member; }
Lockstep::Active::~Active() { tl_ls = saved_; }

Lockstep::Member::~Member()
{
    tl_ls = nullptr;
    tl_ls_member = nullptr;
    g_.impl_->core.leave(Impl::execute);
}

bool Evaluator::lockstep_submit(LsOp &op) const
{
    if (tl_ls_direct > 0 || trace::enabled()) return false;
    if (fiber_merging())
    {
        op.ev = this;
        tl_fb->submit(op);
        if (op.err) std::rethrow_exception(op.err);
        return true;
    }
    Lockstep::Impl *g = tl_ls;
    if (!g) return false;
    op.ev = this;
    g->core.submit(&op, Lockstep::Impl::execute);
    if (op.err) std::rethrow_exception(op.err);
    return true;
}

static std::atomic<std::uint64_t> g_merged_fallbacks{ 0 };

std::uint64_t merged_call_fallbacks(bool reset)
{
    return reset ? g_merged_fallbacks.exchange(0) : g_merged_fallbacks.load();
}

void Evaluator::lockstep_execute(std::vector<LsOp *> &ops) const
{
    // one member's call as it would have run alone
    auto run_one = [&](LsOp &o) {
        try
        {
            switch (o.kind)
            {
            case LsOp::ROT:
                if (o.in.size() == 1 && o.out[0] == o.in[0])
                    rotate_vector_inplace(*o.out[0], o.steps[0], *o.gk);
                else if (o.in.size() == 1)
                    rotate_vector(*o.in[0], o.steps[0], *o.gk, *o.out[0]);
                else
                    rotate_vectors(o.in, o.steps, *o.gk, o.out);
                break;
            case LsOp::RESC: rescale_to_next_inplace_many(o.out); break;
            case LsOp::RELIN: relinearize_inplace_many(o.out, *o.rk); break;
            case LsOp::MULRE:
                if (o.out[0] == o.in[0])
                    multiply_inplace_reduced_error(*o.out[0], *o.in2[0], *o.rk);
                else
                    multiply_reduced_error(*o.in[0], *o.in2[0], *o.rk, *o.out[0]);
                break;
            }
        }
        catch (...)
        {
            o.err = std::current_exception();
        }
    };
    bool same = ops.size() > 1;
    for (LsOp *o : ops) same = same && o->kind == ops[0]->kind && o->gk == ops[0]->gk && o->rk == ops[0]->rk;
    if (!same)
    {
        for (LsOp *o : ops) run_one(*o);
        return;
    }
    try
    {
        // the members' entries as one batch; an output that is also an input (in place) or repeated
        // goes through a temporary
        std::vector<const Ciphertext *> in, in2;
        std::vector<int> steps;
        std::vector<Ciphertext *> out, dst;
        for (LsOp *o : ops)
        {
            in.insert(in.end(), o->in.begin(), o->in.end());
            in2.insert(in2.end(), o->in2.begin(), o->in2.end());
            steps.insert(steps.end(), o->steps.begin(), o->steps.end());
            dst.insert(dst.end(), o->out.begin(), o->out.end());
        }
        const LsOp::Kind kind = ops[0]->kind;
        if (kind == LsOp::RESC)
        {
            rescale_to_next_inplace_many(dst);
            return;
        }
        if (kind == LsOp::RELIN)
        {
            relinearize_inplace_many(dst, *ops[0]->rk);
            return;
        }
        std::vector<Ciphertext> tmp(dst.size());
        out = dst;
        for (std::size_t i = 0; i < dst.size(); i++)
        {
            bool alias = false;
            for (std::size_t j = 0; j < dst.size() && !alias; j++)
                alias = dst[i] == in[j] || (kind == LsOp::MULRE && dst[i] == in2[j]) || (j != i && dst[i] == dst[j]);
            if (alias) out[i] = &tmp[i];
        }
        if (kind == LsOp::ROT)
            rotate_vectors(in, steps, *ops[0]->gk, out);
        else
            multiply_reduced_error_many(in, in2, *ops[0]->rk, out);
        for (std::size_t i = 0; i < dst.size(); i++)
            if (out[i] != dst[i]) *dst[i] = std::move(tmp[i]);
    }
    catch (...)
    {
        // The merged call validates every entry before its first launch (rescale / relinearize), or
        // wrote only outputs that are not inputs (rotations, products through temporaries), so the
        // members' operands are unchanged here: each member's call runs again on its own and gets
        // its own result or its own error, as without the group.  Counted (merged_call_fallbacks):
        // a fallback means a merged launch failed, which a healthy run never sees.
        g_merged_fallbacks.fetch_add(1);
        for (LsOp *o : ops) run_one(*o);
    }
}

void Evaluator::rotate_vectors(const std::vector<const Ciphertext *> &encrypted, const std::vector<int> &steps,
                               const GaloisKeys &galois_keys, const std::vector<Ciphertext *> &destinations) const
{
    if (tl_ls || fiber_merging())
    {
        LsOp op;
        op.kind = LsOp::ROT;
        op.in = encrypted;
        op.steps = steps;
        op.out = destinations;
        op.gk = &galois_keys;
        if (lockstep_submit(op)) return;
    }
    if (encrypted.size() != steps.size() || encrypted.size() != destinations.size())
        throw std::invalid_argument("encrypted, steps and destinations must have the same size");
    if (!batched_launches())
    {
        for (std::size_t i = 0; i < destinations.size(); i++) rotate_vector(*encrypted[i], steps[i], galois_keys, *destinations[i]);
        return;
    }
    for (std::size_t i = 0; i < destinations.size(); i++)
    {
        if (!encrypted[i] || !destinations[i]) throw std::invalid_argument("null ciphertext");
        for (std::size_t j = 0; j < destinations.size(); j++)
            if ((j != i && destinations[i] == destinations[j]) || destinations[i] == encrypted[j])
                throw std::invalid_argument("destinations must be distinct and must not be inputs");
    }
    if (galois_keys.parms_id() != context_.key_parms_id())
        throw std::invalid_argument("galois_keys is not valid for encryption parameters");
    // traced as one "rotate" record per entry (the fallbacks below are nested)
    trace::Scope tsc;
    std::vector<std::string> tin;
    if (tsc.top())
        for (const Ciphertext *c : encrypted) tin.push_back(trace::ct(*c));
    // entries that run batched, grouped by level (chain index)
    std::map<std::size_t, std::vector<std::size_t>> groups;
    std::vector<std::uint32_t> elt(encrypted.size(), 0);
    for (std::size_t i = 0; i < encrypted.size(); i++)
    {
        Level lv = level_of(context_, encrypted[i]->parms_id(), "encrypted");
        if (steps[i] == 0) continue;
        const std::uint32_t e = mhe_galois_elt_from_step(__builtin_ctzll(lv.n), steps[i]);
        if (!e) throw std::invalid_argument("step count too large");
        if (!galois_keys.has_key(e)) continue;
        elt[i] = e;
        groups[lv.L].push_back(i);
    }
    void *s = context_.stream();
    std::vector<bool> done(encrypted.size(), false);
    auto launch = [&](const std::vector<std::size_t> &idx, std::size_t L) {
        std::vector<const std::uint64_t *> in, keys;
        std::vector<std::uint64_t *> out;
        std::vector<std::uint32_t> elts;
        std::vector<int> kls;
        for (std::size_t i : idx)
        {
            const Ciphertext &c = *encrypted[i];
            check_ct(context_, c, "encrypted");
            if (c.size() > 2) throw std::invalid_argument("encrypted size must be 2");
            if (!c.is_ntt_form()) throw std::invalid_argument("encrypted must be in NTT form");
            std::size_t kl = 0;
            keys.push_back(galois_keys.key_for(GaloisKeys::get_index(elt[i]), L, s, kl));
            kls.push_back((int)kl);
            elts.push_back(elt[i]);
        }
        // inputs are read, then destinations re-sized and written (no destination is an input)
        for (std::size_t i : idx) in.push_back(encrypted[i]->store().dev_read(s));
        for (std::size_t i : idx)
        {
            fresh_dest(context_, *encrypted[i], *destinations[i], 2);
            out.push_back(destinations[i]->store().dev_write(s, true));
        }
        chk(mhe_apply_galois_batch(context_.engine(), (int)idx.size(), in.data(), out.data(), elts.data(), keys.data(),
                                   kls.data(), (int)L, s));
        for (std::size_t i : idx) done[i] = true;
    };
    for (auto &g : groups)
    {
        std::vector<std::size_t> idx = g.second;
        if (idx.size() < 2) continue;
        // one call for the level: the engine runs the rotations of an input that appears more than
        // once off one shared ModUp (csrc/hoist.h) and puts the entries of one key side by side in
        // its launches, so they share the key stream (k_ks_row_mac / k_ks_hoist_mac)
        std::stable_sort(idx.begin(), idx.end(), [&](std::size_t a, std::size_t b) { return elt[a] < elt[b]; });
        launch(idx, g.first);
    }
    for (std::size_t i = 0; i < encrypted.size(); i++)
        if (!done[i]) rotate_vector(*encrypted[i], steps[i], galois_keys, *destinations[i]);
    if (tsc.top())
        for (std::size_t i = 0; i < encrypted.size(); i++)
            trace::record("rotate", { tin[i] }, trace::ct(*destinations[i]), "\"step\": " + std::to_string(steps[i]));
}

void Evaluator::relinearize_inplace_many(const std::vector<Ciphertext *> &encrypted, const RelinKeys &relin_keys) const
{
    if (!batched_launches())
    {
        for (Ciphertext *c : encrypted)
            if (c && c->size() > 2) relinearize_inplace(*c, relin_keys);
        return;
    }
    // relinearize_inplace of every entry; size-3 entries of one level share one batched key switch
    trace::Scope tsc; // traced as one "relinearize" record per entry
    std::vector<std::string> tin;
    if (tsc.top())
        for (const Ciphertext *c : encrypted) tin.push_back(c ? trace::ct(*c) : std::string());
    if (relin_keys.parms_id() != context_.key_parms_id())
        throw std::invalid_argument("relin_keys is not valid for encryption parameters");
    std::map<std::size_t, std::vector<Ciphertext *>> groups;
    for (std::size_t i = 0; i < encrypted.size(); i++)
    {
        Ciphertext *c = encrypted[i];
        if (!c) throw std::invalid_argument("null ciphertext");
        for (std::size_t j = 0; j < i; j++)
            if (encrypted[j] == c) throw std::invalid_argument("entries must be distinct");
        Level lv = check_ct(context_, *c, "encrypted");
        if (!c->is_ntt_form()) throw std::invalid_argument("encrypted must be in NTT form");
        if (c->size() == 3) groups[lv.L].push_back(c);
    }
    void *s = context_.stream();
    // every group's key first (a missing or truncated key throws before any entry is changed: the
    // switches below work in place, and a merged Lockstep / FiberBatch call that throws re-runs its
    // members one by one, lockstep_execute)
    std::map<std::size_t, std::pair<const std::uint64_t *, int>> gkey;
    for (auto &g : groups)
    {
        std::size_t kl = 0;
        const std::uint64_t *k = relin_keys.key_for(RelinKeys::get_index(2), g.first, s, kl);
        gkey[g.first] = { k, (int)kl };
    }
    for (auto &g : groups)
    {
        std::vector<Ciphertext *> &v = g.second;
        if (v.size() < 2) continue; // relinearized one by one below
        const std::size_t L = g.first;
        std::vector<std::uint64_t *> ct;
        std::vector<const std::uint64_t *> target, keys;
        std::vector<int> kls;
        for (Ciphertext *c : v)
        {
            keys.push_back(gkey[L].first);
            kls.push_back(gkey[L].second);
            std::uint64_t *d = c->store().dev_write(s);
            ct.push_back(d);
            target.push_back(d + 2 * L * c->poly_modulus_degree());
        }
        // one engine launch sequence (at most 8 entries, MHE_MAXB) per chunk, and each chunk's entries
        // marked relinearized (size 2) as soon as it is done: the switches work in place, so if a later
        // chunk fails, a member re-run by lockstep_execute finds the finished entries at size 2 and
        // skips them instead of switching them a second time
        constexpr std::size_t kChunk = 8;
        for (std::size_t i0 = 0; i0 < v.size(); i0 += kChunk)
        {
            const int B = (int)std::min(kChunk, v.size() - i0);
            chk(mhe_switch_key_batch(context_.engine(), B, ct.data() + i0, target.data() + i0, keys.data() + i0,
                                     kls.data() + i0, (int)L, s));
            for (int e = 0; e < B; e++) v[i0 + e]->resize(2);
        }
    }
    for (Ciphertext *c : encrypted)
        if (c->size() > 2) relinearize_inplace(*c, relin_keys);
    if (tsc.top())
        for (std::size_t i = 0; i < encrypted.size(); i++) trace::record("relinearize", { tin[i] }, trace::ct(*encrypted[i]));
}

void Evaluator::multiply_reduced_error_many(const std::vector<const Ciphertext *> &encrypted1,
                                            const std::vector<const Ciphertext *> &encrypted2,
                                            const RelinKeys &relin_keys,
                                            const std::vector<Ciphertext *> &destinations) const
{
    if (encrypted1.size() != encrypted2.size() || encrypted1.size() != destinations.size())
        throw std::invalid_argument("encrypted1, encrypted2 and destinations must have the same size");
    if (!batched_launches())
    {
        for (std::size_t i = 0; i < destinations.size(); i++)
            multiply_reduced_error(*encrypted1[i], *encrypted2[i], relin_keys, *destinations[i]);
        return;
    }
    for (std::size_t i = 0; i < destinations.size(); i++)
    {
        if (!encrypted1[i] || !encrypted2[i] || !destinations[i]) throw std::invalid_argument("null ciphertext");
        for (std::size_t j = 0; j < destinations.size(); j++)
            if ((j != i && destinations[i] == destinations[j]) || destinations[i] == encrypted1[j] ||
                destinations[i] == encrypted2[j])
                throw std::invalid_argument("destinations must be distinct and must not be inputs");
    }
    trace::Scope tsc; // traced as one "mul_re" record per entry
    std::vector<std::string> t1, t2;
    if (tsc.top())
        for (std::size_t i = 0; i < encrypted1.size(); i++)
        {
            t1.push_back(trace::ct(*encrypted1[i]));
            t2.push_back(trace::ct(*encrypted2[i]));
        }
    // the products as multiply_reduced_error makes them (size 3), then one batched relinearization
    void *s = context_.stream();
    for (std::size_t i = 0; i < destinations.size(); i++)
    {
        const Ciphertext &a = *encrypted1[i], &b = *encrypted2[i];
        Ciphertext &d = *destinations[i];
        const bool same = a.coeff_modulus_size() == b.coeff_modulus_size() && a.parms_id() == b.parms_id() &&
                          a.size() == 2 && b.size() == 2;
        if (!same)
        {
            d = a;
            reduced_error_op(d, b, Rmode::mul);
            continue;
        }
        check_pair(context_, a, b, false);
        const Level lv = level_of(context_, a.parms_id(), "encrypted1");
        const double new_scale = b.scale() * b.scale();
        check_scale(new_scale, lv);
        const std::uint64_t *pa = a.store().dev_read(s), *pb = b.store().dev_read(s);
        fresh_dest(context_, a, d, 3);
        chk(mhe_ct_multiply(context_.engine(), pa, pb, d.store().dev_write(s, true), (int)lv.L, s));
        d.scale() = new_scale;
    }
    relinearize_inplace_many(destinations, relin_keys);
    if (tsc.top())
        for (std::size_t i = 0; i < destinations.size(); i++)
            trace::record("mul_re", { t1[i], t2[i] }, trace::ct(*destinations[i]));
}

void Evaluator::rescale_to_next_inplace_many(const std::vector<Ciphertext *> &encrypted) const
{
    if (!batched_launches())
    {
        for (Ciphertext *c : encrypted) rescale_to_next_inplace(*c);
        return;
    }
    // rescale_to_next of every entry; entries of one level and size run as one batched launch
    trace::Scope tsc; // traced as one "rescale" record per entry
    std::vector<std::string> tin;
    if (tsc.top())
        for (const Ciphertext *c : encrypted) tin.push_back(c ? trace::ct(*c) : std::string());
    std::map<std::pair<std::size_t, std::size_t>, std::vector<Ciphertext *>> groups;
    // every entry is validated before the first group launches, so a bad entry throws with every
    // ciphertext unchanged (as the first failing one-by-one call would leave the rest)
    for (Ciphertext *c : encrypted)
    {
        if (!c) throw std::invalid_argument("null ciphertext");
        Level lv = check_ct(context_, *c, "encrypted");
        if (context_.last_parms_id() == c->parms_id()) throw std::invalid_argument("end of modulus switching chain reached");
        if (!c->is_ntt_form()) throw std::invalid_argument("CKKS encrypted must be in NTT form");
        auto next = lv.cd->next_context_data();
        check_scale(c->scale() / (double)lv.cd->parms().coeff_modulus().back().value(),
                    level_of(context_, next->parms_id(), "parms_id"));
        groups[{ lv.L, c->size() }].push_back(c);
    }
    // every group's results go to fresh buffers first and are committed after the last launch, so
    // a failing group leaves every entry unchanged (a merged Lockstep / FiberBatch call that throws
    // re-runs its members one by one, lockstep_execute)
    void *s = context_.stream();
    struct Staged
    {
        Ciphertext *c;
        PolyStore out;
        parms_id_type next;
        double scale;
        std::size_t size;
    };
    std::vector<Staged> staged;
    staged.reserve(encrypted.size());
    for (auto &g : groups)
    {
        std::vector<Ciphertext *> &v = g.second;
        const std::size_t size = g.first.second;
        std::vector<const std::uint64_t *> in;
        std::vector<std::uint64_t *> out;
        for (Ciphertext *cp : v)
        {
            Ciphertext &c = *cp;
            Level lv = check_ct(context_, c, "encrypted");
            auto next = lv.cd->next_context_data();
            staged.push_back({ cp, PolyStore(), next->parms_id(),
                               c.scale() / (double)lv.cd->parms().coeff_modulus().back().value(), size });
            PolyStore &o = staged.back().out;
            o.bind(context_);
            o.resize_words(size * (lv.L - 1) * lv.n, false);
            in.push_back(c.store().dev_read(s));
            out.push_back(o.dev_write(s, true));
        }
        chk(mhe_rescale_batch(context_.engine(), (int)v.size(), in.data(), out.data(), (int)size, (int)g.first.first, s));
    }
    for (Staged &e : staged)
    {
        const bool ntt = e.c->is_ntt_form();
        e.c->store() = std::move(e.out);
        e.c->resize(context_, e.next, e.size);
        e.c->scale() = e.scale;
        e.c->is_ntt_form() = ntt;
    }
    if (tsc.top())
        for (std::size_t i = 0; i < encrypted.size(); i++) trace::record("rescale", { tin[i] }, trace::ct(*encrypted[i]));
}

void Evaluator::complex_conjugate_inplace(Ciphertext &encrypted, const GaloisKeys &galois_keys, MemoryPoolHandle) const
{
    TRACE_OP("galois", trace::ct(encrypted), trace::ct(encrypted));
    TRACE_EXTRA("\"elt\": " + std::to_string(2 * encrypted.poly_modulus_degree() - 1));
    const std::size_t n = level_of(context_, encrypted.parms_id(), "encrypted").n;
    apply_galois_inplace(encrypted, (std::uint32_t)(2 * n - 1), galois_keys);
}

void Evaluator::complex_conjugate(const Ciphertext &encrypted, const GaloisKeys &galois_keys, Ciphertext &destination,
                                  MemoryPoolHandle) const
{
    TRACE_OP("galois", trace::ct(destination), trace::ct(encrypted));
    TRACE_EXTRA("\"elt\": " + std::to_string(2 * encrypted.poly_modulus_degree() - 1));
    if (&encrypted == &destination) return complex_conjugate_inplace(destination, galois_keys);
    const std::size_t n = level_of(context_, encrypted.parms_id(), "encrypted").n;
    apply_galois_to(encrypted, (std::uint32_t)(2 * n - 1), galois_keys, destination);
}

// ---- modified SEAL entry points (evaluator.cpp:287-486) ------------------------------------
// add_const / multiply_const encode the constant at the first level and mod-switch it to the
// ciphertext's level; the engine produces exactly those residues (its size checks against the
// first level) and applies them per limb without materialising the constant polynomial.
void Evaluator::add_const_inplace(Ciphertext &encrypted, double value) const
{
    TRACE_OP("add_const", trace::ct(encrypted), trace::ct(encrypted));
    TRACE_EXTRA("\"value\": " + trace::num(value));
    Level lv = check_ct(context_, encrypted, "encrypted");
    const std::size_t L1 = context_.first_context_data()->parms().coeff_modulus().size();
    std::vector<std::uint64_t> r(lv.L);
    chk(mhe_ckks_encode_scalar_at(context_.engine(), value, encrypted.scale(), (int)L1, (int)lv.L, r.data()));
    if (!encrypted.is_ntt_form()) throw std::invalid_argument("NTT form mismatch");
    void *s = context_.stream();
    std::uint64_t *a = encrypted.store().dev_write(s);
    chk(mhe_add_scalar(context_.engine(), a, r.data(), a, 1, (int)lv.L, s));
}

void Evaluator::add_const(const Ciphertext &encrypted, double value, Ciphertext &destination) const
{
    TRACE_OP("add_const", trace::ct(destination), trace::ct(encrypted));
    TRACE_EXTRA("\"value\": " + trace::num(value));
    if (&encrypted == &destination) return add_const_inplace(destination, value);
    Level lv = check_ct(context_, encrypted, "encrypted");
    const std::size_t L1 = context_.first_context_data()->parms().coeff_modulus().size();
    std::vector<std::uint64_t> r(lv.L);
    chk(mhe_ckks_encode_scalar_at(context_.engine(), value, encrypted.scale(), (int)L1, (int)lv.L, r.data()));
    if (!encrypted.is_ntt_form()) throw std::invalid_argument("NTT form mismatch");
    void *s = context_.stream();
    const std::size_t pw = lv.L * lv.n;
    fresh_dest(context_, encrypted, destination, encrypted.size());
    const std::uint64_t *a = encrypted.store().dev_read(s);
    std::uint64_t *d = destination.store().dev_write(s, true);
    chk(mhe_add_scalar(context_.engine(), a, r.data(), d, 1, (int)lv.L, s));
    if (encrypted.size() > 1)
        chk(mhe_memcpy_d2d(context_.engine(), d + pw, a + pw, (encrypted.size() - 1) * pw * 8, s));
}

void Evaluator::multiply_const_inplace(Ciphertext &encrypted, double value) const
{
    TRACE_OP("multiply_const", trace::ct(encrypted), trace::ct(encrypted));
    TRACE_EXTRA("\"value\": " + trace::num(value));
    Level lv = check_ct(context_, encrypted, "encrypted");
    const std::size_t L1 = context_.first_context_data()->parms().coeff_modulus().size();
    std::vector<std::uint64_t> r(lv.L);
    chk(mhe_ckks_encode_scalar_at(context_.engine(), value, encrypted.scale(), (int)L1, (int)lv.L, r.data()));
    if (!encrypted.is_ntt_form()) throw std::invalid_argument("NTT form mismatch");
    const double new_scale = encrypted.scale() * encrypted.scale();
    check_scale(new_scale, lv);
    void *s = context_.stream();
    std::uint64_t *a = encrypted.store().dev_write(s);
    chk(mhe_multiply_scalar(context_.engine(), a, r.data(), a, (int)encrypted.size(), (int)lv.L, s));
    encrypted.scale() = new_scale;
}

void Evaluator::multiply_const(const Ciphertext &encrypted, double value, Ciphertext &destination) const
{
    TRACE_OP("multiply_const", trace::ct(destination), trace::ct(encrypted));
    TRACE_EXTRA("\"value\": " + trace::num(value));
    if (&encrypted == &destination) return multiply_const_inplace(destination, value);
    Level lv = check_ct(context_, encrypted, "encrypted");
    const std::size_t L1 = context_.first_context_data()->parms().coeff_modulus().size();
    std::vector<std::uint64_t> r(lv.L);
    chk(mhe_ckks_encode_scalar_at(context_.engine(), value, encrypted.scale(), (int)L1, (int)lv.L, r.data()));
    if (!encrypted.is_ntt_form()) throw std::invalid_argument("NTT form mismatch");
    const double new_scale = encrypted.scale() * encrypted.scale();
    check_scale(new_scale, lv);
    void *s = context_.stream();
    fresh_dest(context_, encrypted, destination, encrypted.size());
    chk(mhe_multiply_scalar(context_.engine(), encrypted.store().dev_read(s), r.data(),
                            destination.store().dev_write(s, true), (int)encrypted.size(), (int)lv.L, s));
    destination.scale() = new_scale;
}

void Evaluator::multiply_plain_add_reduced_error(Ciphertext &acc, const Ciphertext &encrypted,
                                                 const Plaintext &plain) const
{
    TRACE_OP("multiply_plain_add", trace::ct(acc), trace::ct(acc), trace::ct(encrypted), trace::pt(plain));
    // multiply_plain(encrypted, plain, tmp) + add_inplace_reduced_error(acc, tmp) at equal levels,
    // one kernel (bit-identical): acc takes the product's scale, as the reduced-error add assigns it
    Level lv = check_ct(context_, encrypted, "encrypted");
    Level la = check_ct(context_, acc, "encrypted1");
    if (la.L != lv.L || acc.size() != encrypted.size())
        throw std::invalid_argument("multiply_plain_add: acc and encrypted must share level and size");
    if (!encrypted.is_ntt_form() || !plain.is_ntt_form() || !acc.is_ntt_form())
        throw std::invalid_argument("NTT form mismatch");
    if (encrypted.parms_id() != plain.parms_id())
        throw std::invalid_argument("encrypted_ntt and plain_ntt parameter mismatch");
    const double new_scale = encrypted.scale() * plain.scale();
    check_scale(new_scale, lv);
    void *s = context_.stream();
    const std::uint64_t *b = plain.store().dev_read(s);
    const std::uint64_t *a = encrypted.store().dev_read(s);
    chk(mhe_multiply_plain_add(context_.engine(), a, b, acc.store().dev_write(s), (int)encrypted.size(), (int)lv.L, s));
    acc.scale() = new_scale;
}

void Evaluator::multiply_plain_sum(const std::vector<const Ciphertext *> &encrypted,
                                   const std::vector<const Plaintext *> &plain, Ciphertext &destination) const
{
    if (encrypted.empty() || encrypted.size() != plain.size())
        throw std::invalid_argument("encrypted and plain must be non-empty and of the same size");
    for (std::size_t k = 0; k < encrypted.size(); k++)
        if (!encrypted[k] || !plain[k] || encrypted[k] == &destination)
            throw std::invalid_argument("multiply_plain_sum: null operand or destination among the inputs");
    // term by term under the evaluator trace (one record per operation) or with batching off
    if (trace::enabled() || !batched_launches())
    {
        multiply_plain(*encrypted[0], *plain[0], destination);
        for (std::size_t k = 1; k < encrypted.size(); k++)
            multiply_plain_add_reduced_error(destination, *encrypted[k], *plain[k]);
        return;
    }
    const Ciphertext &e0 = *encrypted[0];
    Level lv = check_ct(context_, e0, "encrypted");
    double new_scale = 0;
    for (std::size_t k = 0; k < encrypted.size(); k++)
    {
        const Ciphertext &e = *encrypted[k];
        const Plaintext &p = *plain[k];
        Level lk = check_ct(context_, e, "encrypted");
        if (lk.L != lv.L || e.size() != e0.size())
            throw std::invalid_argument("multiply_plain_add: acc and encrypted must share level and size");
        if (!e.is_ntt_form() || !p.is_ntt_form()) throw std::invalid_argument("NTT form mismatch");
        if (e.parms_id() != p.parms_id()) throw std::invalid_argument("encrypted_ntt and plain_ntt parameter mismatch");
        new_scale = e.scale() * p.scale();
        check_scale(new_scale, lv);
    }
    void *s = context_.stream();
    std::vector<const std::uint64_t *> a, b;
    for (std::size_t k = 0; k < encrypted.size(); k++)
    {
        a.push_back(encrypted[k]->store().dev_read(s));
        b.push_back(plain[k]->store().dev_read(s));
    }
    fresh_dest(context_, e0, destination, e0.size());
    chk(mhe_multiply_plain_sum(context_.engine(), (int)a.size(), a.data(), b.data(), destination.store().dev_write(s, true),
                               0, (int)e0.size(), (int)lv.L, s));
    destination.scale() = new_scale; // the last term's product scale, as the reduced-error adds leave it
}

namespace
{
template <typename T>
void split(const std::vector<T> &v, std::vector<double> &re, std::vector<double> &im);
template <>
void split<double>(const std::vector<double> &v, std::vector<double> &re, std::vector<double> &im)
{
    re = v;
    im.clear();
}
template <>
void split<std::complex<double>>(const std::vector<std::complex<double>> &v, std::vector<double> &re,
                                 std::vector<double> &im)
{
    re.resize(v.size());
    im.resize(v.size());
    for (std::size_t i = 0; i < v.size(); i++)
    {
        re[i] = v[i].real();
        im[i] = v[i].imag();
    }
}
} // namespace

template <typename T>
void Evaluator::multiply_vector_inplace(Ciphertext &encrypted, const std::vector<T> &value) const
{
    // evaluator.cpp:303-310: encode at the first level, mod_switch_to, multiply_plain
    Plaintext plain;
    encode_vector_for(encrypted, value, plain);
    multiply_plain_inplace(encrypted, plain);
}

template <typename T>
void Evaluator::encode_vector_for(const Ciphertext &encrypted, const std::vector<T> &value, Plaintext &plain) const
{
    // CKKSEncoder::encode(value, encrypted.scale()) at the first level, then mod_switch_to the
    // ciphertext's level: only the kept limbs are produced (SEAL's bounds are checked at the
    // first level)
    Level lv = check_ct(context_, encrypted, "encrypted");
    const std::size_t L1 = context_.first_context_data()->parms().coeff_modulus().size();
    if (value.size() > lv.n / 2) throw std::invalid_argument("values_size is too large");
    std::vector<double> re, im;
    split<T>(value, re, im);
    TRACE_OP("encode_for", trace::pt(plain), trace::vec(re.data(), im.empty() ? nullptr : im.data(), re.size()));
    TRACE_EXTRA("\"scale\": " + trace::num(encrypted.scale()) + ", \"limbs\": " + std::to_string(lv.L));
    void *s = context_.stream();
    plain.set_level(context_, encrypted.parms_id(), lv.L);
    plain.scale() = encrypted.scale();
    chk(mhe_ckks_encode_at(context_.engine(), encoder_.handle(), re.data(), im.empty() ? nullptr : im.data(),
                           re.size(), encrypted.scale(), (int)L1, (int)lv.L, plain.store().dev_write(s, true), s));
}

template void Evaluator::encode_vector_for<double>(const Ciphertext &, const std::vector<double> &, Plaintext &) const;
template void Evaluator::encode_vector_for<std::complex<double>>(const Ciphertext &,
                                                                 const std::vector<std::complex<double>> &,
                                                                 Plaintext &) const;

template void Evaluator::multiply_vector_inplace<double>(Ciphertext &, const std::vector<double> &) const;
template void Evaluator::multiply_vector_inplace<std::complex<double>>(
    Ciphertext &, const std::vector<std::complex<double>> &) const;

// evaluator.cpp:312-486 (Kim et al., CT-RSA 2022): when the levels differ, the operand at the
// higher level is multiplied by s_other * q_last / s^2 (multiply_const), its scale forced to
// s_other * q_last, rescaled and mod-switched down to the other operand's level; equal levels
// only copy the scale across.  Same operation order and scale assignments as the reference.
void Evaluator::reduced_error_op(Ciphertext &encrypted1, const Ciphertext &encrypted2, Rmode mode) const
{
    auto op_inplace = [&](Ciphertext &a, const Ciphertext &b) {
        if (mode == Rmode::add)
            add_inplace(a, b);
        else if (mode == Rmode::sub)
            sub_inplace(a, b);
        else
            multiply_inplace(a, b);
    };
    auto op_out = [&](const Ciphertext &a, const Ciphertext &b, Ciphertext &d) {
        if (mode == Rmode::add)
            add(a, b, d);
        else if (mode == Rmode::sub)
            sub(a, b, d);
        else
            multiply(a, b, d);
    };
    const std::size_t l1 = encrypted1.coeff_modulus_size(), l2 = encrypted2.coeff_modulus_size();
    if (l1 == l2)
    {
        encrypted1.scale() = encrypted2.scale();
        op_inplace(encrypted1, encrypted2);
    }
    else if (l1 < l2)
    {
        const double q = static_cast<double>(level_of(context_, encrypted2.parms_id(), "encrypted2")
                                                 .cd->parms()
                                                 .coeff_modulus()[l2 - 1]
                                                 .value());
        Ciphertext adj;
        const double scale_adjust = encrypted1.scale() * q / (encrypted2.scale() * encrypted2.scale());
        multiply_const(encrypted2, scale_adjust, adj);
        adj.scale() = encrypted1.scale() * q;
        rescale_to_next_inplace(adj);
        mod_switch_to_inplace(adj, encrypted1.parms_id());
        encrypted1.scale() = adj.scale();
        op_inplace(encrypted1, adj);
    }
    else
    {
        const double q = static_cast<double>(level_of(context_, encrypted1.parms_id(), "encrypted1")
                                                 .cd->parms()
                                                 .coeff_modulus()[l1 - 1]
                                                 .value());
        Ciphertext adj;
        const double scale_adjust = encrypted2.scale() * q / (encrypted1.scale() * encrypted1.scale());
        multiply_const(encrypted1, scale_adjust, adj);
        adj.scale() = encrypted2.scale() * q;
        rescale_to_next_inplace(adj);
        mod_switch_to_inplace(adj, encrypted2.parms_id());
        adj.scale() = encrypted2.scale();
        op_out(adj, encrypted2, encrypted1);
    }
}

void Evaluator::reduced_error_out(const Ciphertext &encrypted1, const Ciphertext &encrypted2, Ciphertext &destination,
                                  Rmode mode, const RelinKeys *relin_keys) const
{
    if (tl_ls && mode == Rmode::mul)
    {
        LsOp op;
        op.kind = LsOp::MULRE;
        op.in = { &encrypted1 };
        op.in2 = { &encrypted2 };
        op.out = { &destination };
        op.rk = relin_keys;
        if (lockstep_submit(op)) return;
    }
    TRACE_OP(mode == Rmode::add ? "add_re" : mode == Rmode::sub ? "sub_re" : "mul_re", trace::ct(destination),
             trace::ct(encrypted1), trace::ct(encrypted2));
    // equal levels: encrypted1 takes encrypted2's scale, then the op (reduced_error_op); written
    // out of place so encrypted1 is not copied first
    const bool same = encrypted1.coeff_modulus_size() == encrypted2.coeff_modulus_size() &&
                      encrypted1.parms_id() == encrypted2.parms_id() && encrypted1.size() == encrypted2.size() &&
                      encrypted1.size() == 2 && &encrypted1 != &destination && &encrypted2 != &destination;
    if (!same)
    {
        destination = encrypted1;
        reduced_error_op(destination, encrypted2, mode);
        if (mode == Rmode::mul) relinearize_inplace(destination, *relin_keys);
        return;
    }
    check_pair(context_, encrypted1, encrypted2, false);
    void *s = context_.stream();
    const Level lv = level_of(context_, encrypted1.parms_id(), "encrypted1");
    const std::uint64_t *a = encrypted1.store().dev_read(s), *b = encrypted2.store().dev_read(s);
    if (mode == Rmode::mul)
    {
        const double new_scale = encrypted2.scale() * encrypted2.scale();
        check_scale(new_scale, lv);
        fresh_dest(context_, encrypted1, destination, 3);
        chk(mhe_ct_multiply(context_.engine(), a, b, destination.store().dev_write(s, true), (int)lv.L, s));
        destination.scale() = new_scale;
        relinearize_inplace(destination, *relin_keys);
        return;
    }
    fresh_dest(context_, encrypted1, destination, 2);
    std::uint64_t *d = destination.store().dev_write(s, true);
    if (mode == Rmode::add)
        chk(mhe_add(context_.engine(), a, b, d, 2, (int)lv.L, s));
    else
        chk(mhe_sub(context_.engine(), a, b, d, 2, (int)lv.L, s));
    destination.scale() = encrypted2.scale();
}

void Evaluator::add_inplace_reduced_error(Ciphertext &encrypted1, const Ciphertext &encrypted2) const
{
    TRACE_OP("add_re", trace::ct(encrypted1), trace::ct(encrypted1), trace::ct(encrypted2));
    reduced_error_op(encrypted1, encrypted2, Rmode::add);
}

void Evaluator::sub_inplace_reduced_error(Ciphertext &encrypted1, const Ciphertext &encrypted2) const
{
    TRACE_OP("sub_re", trace::ct(encrypted1), trace::ct(encrypted1), trace::ct(encrypted2));
    reduced_error_op(encrypted1, encrypted2, Rmode::sub);
}

void Evaluator::multiply_inplace_reduced_error(Ciphertext &encrypted1, const Ciphertext &encrypted2,
                                               const RelinKeys &relin_keys) const
{
    if (tl_ls || fiber_merging())
    {
        LsOp op;
        op.kind = LsOp::MULRE;
        op.in = { &encrypted1 };
        op.in2 = { &encrypted2 };
        op.out = { &encrypted1 };
        op.rk = &relin_keys;
        if (lockstep_submit(op)) return;
    }
    TRACE_OP("mul_re", trace::ct(encrypted1), trace::ct(encrypted1), trace::ct(encrypted2));
    reduced_error_op(encrypted1, encrypted2, Rmode::mul);
    relinearize_inplace(encrypted1, relin_keys);
}
} // namespace seal
