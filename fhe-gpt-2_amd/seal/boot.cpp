// boot.cpp -- CKKS bootstrapping over the seal:: surface (include/mhe_boot.h).
//
// Ciphertext-operation sequences follow cnn_ckks/cpu-ckks/single-key/ckks_bootstrapping/
// Bootstrapper.cpp and ModularReducer.cpp and cnn_ckks/common/Polynomial.cpp (cited per
// function); the host-side coefficient generation restates the reference's (see the header).
#include "mhe_boot.h"

#include <quadmath.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <functional>
#include <map>
#include <mutex>
#include <thread>
#include <stdexcept>

#include "../../include/mhe.h"
#include "trace.h"

using namespace seal;
using cd = std::complex<double>;

// ============================================================================ common/func.cpp
void oddbabycount(long &mink, long &minm, long deg)
{
    // common/func.cpp:90-115: the (k, m) minimising the odd baby-step cost estimate among
    // shapes of minimal depth ceil(log2 k) + m = ceil(log2 deg)
    long m, mind = 0;
    double mineval = 100000;
    for (long k = 2; k <= deg; k += 2)
    {
        m = 1;
        while ((1L << m) * k < deg) m++;
        if (std::ceil(std::log(k) / std::log(2)) + m == std::ceil(std::log(deg) / std::log(2)))
        {
            const double eval = std::ceil((deg + 0.0) / (k + 0.0)) + k / 2 - 5 + m + std::ceil(std::log(k)) +
                                std::max(3.0 - m, std::ceil((deg + 0.0) / (1.5 * (1L << (m - 1)) * k)));
            if (mineval > eval)
            {
                mineval = eval;
                mink = k;
                minm = m;
                mind = (long)(std::ceil(std::log(k) / std::log(2)) + m);
            }
            else if (mineval == eval && mind > std::ceil(std::log(k) / std::log(2)) + m)
            {
                mink = k;
                minm = m;
                mind = (long)(std::ceil(std::log(k) / std::log(2)) + m);
            }
        }
    }
}

void babycount(long &mink, long &minm, long deg)
{
    // common/func.cpp:117-140: minimise log2(d/k) + k + d/k - 3 non-scalar products
    mink = 2;
    double d_over_k = static_cast<double>(deg) / mink;
    int log2_d_over_k = (int)std::ceil(std::log2(d_over_k));
    int ceil_d_over_k = (int)std::ceil(d_over_k);
    int min_mul = log2_d_over_k + (int)mink + ceil_d_over_k - 3;
    minm = log2_d_over_k;
    for (int i = 3; i < 2 * std::sqrt((double)deg); i++)
    {
        d_over_k = static_cast<double>(deg) / i;
        log2_d_over_k = (int)std::ceil(std::log2(d_over_k));
        ceil_d_over_k = (int)std::ceil(d_over_k);
        const int curr_mul = log2_d_over_k + i + ceil_d_over_k - 3;
        if (min_mul > curr_mul)
        {
            mink = i;
            min_mul = curr_mul;
            minm = log2_d_over_k;
        }
    }
}

int giantstep(int M)
{
    // common/func.cpp:203-213: k minimising ceil(M/k) + k - 1
    int minval = M, mink = 1;
    for (int k = 1; k <= 3 * std::sqrt((double)M); k++)
    {
        const int currval = (int)std::ceil((M + 0.0) / (k + 0.0)) + k - 1;
        if (currval < minval)
        {
            minval = currval;
            mink = k;
        }
    }
    return mink;
}

void rotation(int logslot, int Nh, int shiftcount, const std::vector<cd> &vec, std::vector<cd> &rtnvec)
{
    // common/func.cpp:215-224
    const int slotlen = 1 << logslot, repeatcount = Nh / slotlen;
    rtnvec.clear();
    rtnvec.reserve(Nh);
    for (int j = 0; j < repeatcount; j++)
        for (int i = 0; i < slotlen; i++) rtnvec.push_back(vec[((slotlen + i + shiftcount) % slotlen + slotlen) % slotlen]);
}

// ======================================================================== boot::Polynomial
namespace boot
{
Polynomial::Polynomial(long d) : coeff(d + 1, 0.0), chebcoeff(d + 1, 0.0), deg(d) {}

void Polynomial::set_zero_polynomial(long d)
{
    deg = d;
    coeff.assign(d + 1, 0.0);
    chebcoeff.assign(d + 1, 0.0);
}

void Polynomial::set_chebyshev(const std::vector<double> &cheb)
{
    deg = (long)cheb.size() - 1;
    chebcoeff = cheb;
    cheb_to_power();
}

void Polynomial::cheb_to_power()
{
    // Polynomial.cpp:110-123 (T_i by the three-term recurrence, summed in the power basis); only
    // meaningful in double precision for small degrees, which is where `coeff` is read
    coeff.assign(deg + 1, 0.0);
    std::vector<double> t0(deg + 1, 0.0), t1(deg + 1, 0.0), t2(deg + 1, 0.0);
    t0[0] = 1.0;
    if (deg >= 1) t1[1] = 1.0;
    for (long i = 0; i <= deg; i++)
    {
        const std::vector<double> &ti = i == 0 ? t0 : t1;
        for (long j = 0; j <= i; j++) coeff[j] += chebcoeff[i] * ti[j];
        if (i >= 1 && i < deg)
        {
            std::fill(t2.begin(), t2.end(), 0.0);
            for (long j = 0; j <= i; j++) t2[j + 1] += 2 * t1[j];
            for (long j = 0; j <= i - 1; j++) t2[j] -= t0[j];
            t0.swap(t1);
            t1.swap(t2);
        }
    }
}

void Polynomial::constmul(double c)
{
    for (auto &v : coeff) v *= c;
    for (auto &v : chebcoeff) v *= c;
}

double Polynomial::evaluate(double x) const
{
    // Clenshaw
    double b1 = 0, b2 = 0;
    for (long j = deg; j >= 1; j--)
    {
        const double b0 = 2 * x * b1 - b2 + chebcoeff[j];
        b2 = b1;
        b1 = b0;
    }
    return x * b1 - b2 + chebcoeff[0];
}

void divide_poly(Polynomial &quotient, Polynomial &remainder, const Polynomial &target, long m)
{
    // p = q T_m + r, deg r < m, using T_j = 2 T_{j-m} T_m - T_{|j-2m|} (j > m) and T_m = T_0 T_m.
    // Same polynomials as the reference's power-basis long division (Polynomial.cpp:890-916).
    if (target.deg < m)
    {
        quotient.set_zero_polynomial(0);
        remainder = target;
        return;
    }
    std::vector<double> r = target.chebcoeff, q(target.deg - m + 1, 0.0);
    for (long j = target.deg; j >= m; j--)
    {
        const double a = r[j];
        r[j] = 0;
        if (j == m)
            q[0] += a;
        else
        {
            q[j - m] += 2 * a;
            r[std::labs(j - 2 * m)] -= a;
        }
    }
    r.resize(m);
    quotient.set_chebyshev(q);
    remainder.set_chebyshev(r);
}

void Polynomial::generate_poly_heap_manual(long k, long m)
{
    // Polynomial.cpp:169-206: node j splits into quotient 2(j+1)-1 and remainder 2(j+1) by
    // T_{k 2^(m-1-level)}; a node below that degree passes on as the remainder only
    heap_k = k;
    heap_m = m;
    heaplen = (1L << (heap_m + 1)) - 1;
    poly_heap.assign(heaplen, nullptr);
    poly_heap[0] = std::make_shared<Polynomial>(*this);
    poly_heap[0]->poly_heap.clear();
    long chebdeg = heap_k << heap_m;
    for (long i = 0; i < heap_m; i++)
    {
        chebdeg >>= 1;
        const long first = (1L << i) - 1, last = (1L << (i + 1)) - 1;
        for (long j = first; j < last; j++)
        {
            if (!poly_heap[j]) continue;
            if (poly_heap[j]->deg < chebdeg)
                poly_heap[2 * (j + 1)] = std::make_shared<Polynomial>(*poly_heap[j]);
            else
            {
                auto qn = std::make_shared<Polynomial>(), rn = std::make_shared<Polynomial>();
                divide_poly(*qn, *rn, *poly_heap[j], chebdeg);
                poly_heap[2 * (j + 1) - 1] = qn;
                poly_heap[2 * (j + 1)] = rn;
            }
        }
    }
}

void Polynomial::generate_poly_heap_odd()
{
    oddbabycount(heap_k, heap_m, deg);
    generate_poly_heap_manual(heap_k, heap_m);
}

void Polynomial::generate_poly_heap()
{
    babycount(heap_k, heap_m, deg);
    generate_poly_heap_manual(heap_k, heap_m);
}

void Polynomial::write_heap_to_file(std::ostream &out) const
{
    // Polynomial.cpp:217-230 layout: heaplen, then "index deg" and deg+1 Chebyshev coefficients
    out.precision(17);
    out << heaplen << "\n";
    for (long index = 0; index < heaplen; index++)
        if (poly_heap[index])
        {
            out << index << " " << poly_heap[index]->deg << "\n";
            for (long i = 0; i <= poly_heap[index]->deg; i++) out << poly_heap[index]->chebcoeff[i] << "\n";
            out << "\n";
        }
}

void Polynomial::read_heap_from_file(std::istream &in)
{
    // Polynomial.cpp:232-253
    long index = 0, in_deg = 0;
    in >> heaplen;
    poly_heap.assign(heaplen, nullptr);
    while (index < heaplen - 1 && (in >> index >> in_deg))
    {
        std::vector<double> c(in_deg + 1);
        for (auto &v : c) in >> v;
        poly_heap[index] = std::make_shared<Polynomial>();
        poly_heap[index]->set_chebyshev(c);
    }
    heap_m = 0;
    while ((1L << (heap_m + 1)) - 1 < heaplen) heap_m++;
    if (poly_heap[0])
    {
        set_chebyshev(poly_heap[0]->chebcoeff);
        // heap_k from the top split degree: deg < k 2^m
        heap_k = 1;
        while ((heap_k << heap_m) <= deg) heap_k++;
    }
}

void Polynomial::homomorphic_poly_evaluation(SEALContext &, CKKSEncoder &, Encryptor &, Evaluator &evaluator,
                                             RelinKeys &relin_keys, Ciphertext &rtn, Ciphertext &cipher, Decryptor &)
{
    // Polynomial.cpp:256-560
    const double zero = 1. / cipher.scale();
    if (deg == 1)
    {
        evaluator.multiply_const(cipher, coeff[1], rtn);
        evaluator.rescale_to_next_inplace(rtn);
        evaluator.add_const(rtn, coeff[0], rtn);
        return;
    }
    if (deg == 2)
    {
        Ciphertext squared;
        evaluator.square(cipher, squared);
        evaluator.relinearize_inplace(squared, relin_keys);
        evaluator.rescale_to_next_inplace(squared);
        evaluator.multiply_const_inplace(squared, coeff[2]);
        evaluator.rescale_to_next_inplace(squared);
        if (std::abs(coeff[1]) >= zero)
        {
            evaluator.multiply_const(cipher, coeff[1], rtn);
            evaluator.rescale_to_next_inplace(rtn);
            evaluator.add_reduced_error(rtn, squared, rtn);
        }
        else
            rtn = squared;
        evaluator.add_const_inplace(rtn, coeff[0]);
        return;
    }
    if (deg == 3)
    {
        Ciphertext squared, cubic;
        evaluator.square(cipher, squared);
        evaluator.relinearize_inplace(squared, relin_keys);
        evaluator.rescale_to_next_inplace(squared);
        evaluator.multiply_const(cipher, coeff[3], cubic);
        evaluator.rescale_to_next_inplace(cubic);
        evaluator.multiply_inplace_reduced_error(cubic, squared, relin_keys);
        evaluator.rescale_to_next_inplace(cubic);
        if (std::abs(coeff[1]) >= zero)
        {
            evaluator.multiply_const(cipher, coeff[1], rtn);
            evaluator.rescale_to_next_inplace(rtn);
            evaluator.add_reduced_error(rtn, cubic, rtn);
        }
        else
            rtn = cubic;
        if (std::abs(coeff[2]) >= zero)
        {
            evaluator.multiply_const_inplace(squared, coeff[2]);
            evaluator.rescale_to_next_inplace(squared);
            evaluator.add_reduced_error(rtn, squared, rtn);
        }
        evaluator.add_const_inplace(rtn, coeff[0]);
        return;
    }
    if (poly_heap.empty()) throw std::logic_error("polynomial heap is not generated");

    // baby steps T_1 .. T_{k-1}: T_2i = 2 T_i^2 - 1, T_i = 2 T_{2^a} T_{i-2^a} - T_{|2^(a+1) - i|}
    std::vector<Ciphertext> baby(heap_k);
    std::vector<bool> babybool(heap_k, false);
    baby[1] = cipher;
    babybool[1] = true;
    for (long i = 2; i < heap_k; i *= 2)
    {
        evaluator.square(baby[i / 2], baby[i]);
        evaluator.relinearize_inplace(baby[i], relin_keys);
        evaluator.rescale_to_next_inplace(baby[i]);
        evaluator.double_inplace(baby[i]);
        evaluator.add_const(baby[i], -1.0, baby[i]);
        babybool[i] = true;
    }
    // T_i for 2^a < i < 2^(a+1) needs only T's below 2^a (res, diff < 2^a): each band's products
    // and rescales run as one batch (each T_i's operations are the reference's, in its order)
    for (long lo = 2; lo < heap_k; lo *= 2)
    {
        std::vector<long> band;
        for (long i = lo + 1; i < std::min(2 * lo, heap_k); i++)
            if (!babybool[i]) band.push_back(i);
        if (band.empty()) continue;
        std::vector<const Ciphertext *> m1, m2;
        std::vector<Ciphertext *> mo;
        for (long i : band)
        {
            const long lpow2 = 1L << (int)std::floor(std::log(i) / std::log(2));
            m1.push_back(&baby[lpow2]);
            m2.push_back(&baby[i - lpow2]);
            mo.push_back(&baby[i]);
        }
        evaluator.multiply_reduced_error_many(m1, m2, relin_keys, mo);
        evaluator.rescale_to_next_inplace_many(mo);
        for (long i : band)
        {
            const long lpow2 = 1L << (int)std::floor(std::log(i) / std::log(2));
            const long res = i - lpow2, diff = std::labs(lpow2 - res);
            evaluator.double_inplace(baby[i]);
            evaluator.sub_reduced_error(baby[i], baby[diff], baby[i]);
            babybool[i] = true;
        }
    }
    for (long i = 1; i < heap_k; i++)
    {
        if (babybool[i]) continue; // (every i is covered by a band above)
        const long lpow2 = 1L << (int)std::floor(std::log(i) / std::log(2));
        const long res = i - lpow2, diff = std::labs(lpow2 - res);
        evaluator.multiply_reduced_error(baby[lpow2], baby[res], relin_keys, baby[i]);
        evaluator.rescale_to_next_inplace(baby[i]);
        evaluator.double_inplace(baby[i]);
        evaluator.sub_reduced_error(baby[i], baby[diff], baby[i]);
        babybool[i] = true;
    }

    // giant steps T_k, T_2k, T_4k, ...
    std::vector<Ciphertext> giant(heap_m);
    {
        const long lpow2 = 1L << ((int)std::ceil(std::log(heap_k) / std::log(2)) - 1);
        const long res = heap_k - lpow2, diff = std::labs(lpow2 - res);
        if (res == 0)
            giant[0] = baby[lpow2];
        else if (diff == 0)
        {
            evaluator.square(baby[lpow2], giant[0]);
            evaluator.relinearize_inplace(giant[0], relin_keys);
            evaluator.rescale_to_next_inplace(giant[0]);
            evaluator.double_inplace(giant[0]);
            evaluator.add_const(giant[0], -1.0, giant[0]);
        }
        else
        {
            evaluator.multiply_reduced_error(baby[lpow2], baby[res], relin_keys, giant[0]);
            evaluator.rescale_to_next_inplace(giant[0]);
            evaluator.double_inplace(giant[0]);
            evaluator.sub_reduced_error(giant[0], baby[diff], giant[0]);
        }
    }
    for (long i = 1; i < heap_m; i++)
    {
        evaluator.square(giant[i - 1], giant[i]);
        evaluator.relinearize_inplace(giant[i], relin_keys);
        evaluator.rescale_to_next_inplace(giant[i]);
        evaluator.double_inplace(giant[i]);
        evaluator.add_const_inplace(giant[i], -1.0);
    }

    // leaves: sum_j c_j T_j by multiply_const + rescale.  Every term of every leaf is made first
    // and all of them are rescaled as one batch; each leaf is then summed in the reference's order.
    std::vector<Ciphertext> cipherheap(heaplen);
    std::vector<bool> cipherheapbool(heaplen, false);
    long heapfirst = (1L << heap_m) - 1, heaplast = (1L << (heap_m + 1)) - 1;
    {
        std::vector<std::vector<Ciphertext>> terms(heaplen);
        std::vector<Ciphertext *> resc;
        for (long i = heapfirst; i < heaplast; i++)
        {
            if (!poly_heap[i]) continue;
            const Polynomial &p = *poly_heap[i];
            cipherheapbool[i] = true;
            evaluator.multiply_const(baby[1], p.chebcoeff[1], cipherheap[i]);
            resc.push_back(&cipherheap[i]);
            long cnt = 0;
            for (long j = 2; j <= p.deg; j++)
                if (!(std::abs(p.chebcoeff[j]) <= zero)) cnt++;
            terms[i].resize(cnt);
            long t = 0;
            for (long j = 2; j <= p.deg; j++)
            {
                if (std::abs(p.chebcoeff[j]) <= zero) continue;
                evaluator.multiply_const(j < heap_k ? baby[j] : giant[0], p.chebcoeff[j], terms[i][t]);
                resc.push_back(&terms[i][t++]);
            }
        }
        evaluator.rescale_to_next_inplace_many(resc);
        for (long i = heapfirst; i < heaplast; i++)
        {
            if (!poly_heap[i]) continue;
            const Polynomial &p = *poly_heap[i];
            if (!(std::abs(p.chebcoeff[1]) <= zero)) evaluator.add_const_inplace(cipherheap[i], p.chebcoeff[0]);
            for (Ciphertext &tm : terms[i]) evaluator.add_reduced_error(cipherheap[i], tm, cipherheap[i]);
        }
    }
    // combine: node = quotient * T_{k 2^g} + remainder; the nodes of one depth as one batch
    long depth = heap_m, gindex = 0;
    while (depth != 0)
    {
        depth--;
        heapfirst = (1L << depth) - 1;
        heaplast = (1L << (depth + 1)) - 1;
        std::vector<long> prod;
        std::vector<const Ciphertext *> m1, m2;
        std::vector<Ciphertext *> mo;
        for (long i = heapfirst; i < heaplast; i++)
        {
            if (!poly_heap[i]) continue;
            cipherheapbool[i] = true;
            if (!cipherheapbool[2 * (i + 1) - 1])
                cipherheap[i] = std::move(cipherheap[2 * (i + 1)]); // the child is not read again
            else
            {
                prod.push_back(i);
                m1.push_back(&cipherheap[2 * (i + 1) - 1]);
                m2.push_back(&giant[gindex]);
                mo.push_back(&cipherheap[i]);
            }
        }
        evaluator.multiply_reduced_error_many(m1, m2, relin_keys, mo);
        evaluator.rescale_to_next_inplace_many(mo);
        for (long i : prod) evaluator.add_reduced_error(cipherheap[i], cipherheap[2 * (i + 1)], cipherheap[i]);
        gindex++;
    }
    rtn = std::move(cipherheap[0]);
}
} // namespace boot

// ===================================================================== coefficient generation
// The multi-interval Remez exchange of cnn_ckks/common/Remez.cpp (boot::Remez, used through
// ckks_bootstrapping/RemezCos.h and RemezArcsin.h), restated in binary128 (__float128): the
// reference runs it in NTL RR at 1000 bits.  Same initial reference set (better_initialize), the
// same linear solve with an alternating-sign error column (getcoeffwitherr), the same scan for
// the error's extrema with its ternary refinement (getextreme_local), the same selection of an
// alternating set (choosemaxs), iterated until the alternation levels agree.  The binary128 stop
// is 2^-85 relative spread (the reference's 2^-120 is below binary128's resolution of the error);
// the resulting polynomial is the same minimax polynomial to far more digits than the doubles the
// homomorphic evaluation uses.
namespace
{
using f128 = __float128;
const f128 kPi = acosq(-1);

struct RemezPt
{
    f128 x = 0, y = 0;
    long locmm = 0;
};

// RemezParam.h defaults
struct RemezParams
{
    double log_scan_step_diff = 9.5;
    long binary_prec = 10;
    long log_round_prec = 100;
    double stop_log2 = -85; // binary128 stand-in for log_approx_degree = 120
    int max_iter = 60;
};

f128 chebeval(long deg, const std::vector<f128> &c, f128 u)
{
    // common/func.cpp:46-58: the three-term recurrence, summed in order
    f128 t0 = 1, t1 = u, r = c[0] * t0 + (deg >= 1 ? c[1] * t1 : 0);
    for (long i = 2; i <= deg; i++)
    {
        const f128 t2 = 2 * u * t1 - t0;
        t0 = t1;
        t1 = t2;
        r += c[i] * t2;
    }
    return r;
}

f128 fracpart(f128 x)
{
    return x - roundq(x); // common/func.cpp:3-5
}

class RemezExchange
{
public:
    RemezExchange(long K, double log_width, long deg, std::function<f128(f128)> f, RemezParams prm = {})
        : K_(K), deg_(deg), f_(std::move(f)), prm_(prm), sample_(deg + 2), coeff_(deg + 1)
    {
        width_ = powq(2, -(f128)log_width);
        sc_ = width_ / powq(2, (f128)prm.log_scan_step_diff);
        log_width_ = log_width;
    }

    // generate_optimal_poly (Remez.cpp:558-582): coefficients of T_j(x / K)
    std::vector<f128> run()
    {
        better_initialize();
        iterations = 0;
        const f128 stop = powq(2, (f128)prm_.stop_log2);
        f128 prev = -1;
        while (iterations < prm_.max_iter)
        {
            getcoeffwitherr();
            getextreme();
            choosemaxs();
            iterations++;
            const f128 spread = (max_err - min_err) / min_err;
            if (spread <= stop) break;
            if (prev >= 0 && spread >= prev && spread < powq(2, -60)) break; // at binary128's floor
            prev = spread;
        }
        getcoeffwitherr(); // the polynomial of the final reference set
        return coeff_;
    }

    f128 max_err = 1000, min_err = 1;
    int iterations = 0;
    std::vector<RemezPt> extremes() const { return extreme_; }

private:
    void better_initialize()
    {
        // Remez.cpp:27-93: nodes per interval from the interpolation-error bound of each, then
        // Chebyshev nodes of every interval
        const long deg_bdd = deg_ + 2;
        std::vector<int> nodecount(K_, 1);
        long tot_deg = 2 * K_ - 1;
        const double err = std::pow(2.0, -log_width_);
        std::vector<double> bdd(K_);
        double temp = 0;
        for (long i = 1; i <= 2 * K_ - 1; i++) temp -= std::log2((double)i);
        temp += (2 * K_ - 1) * std::log2(2 * M_PI);
        temp += std::log2(err);
        for (long i = 0; i < K_; i++)
        {
            bdd[i] = temp;
            for (long j = 1; j <= K_ - 1 - i; j++) bdd[i] += std::log2((double)j + err);
            for (long j = 1; j <= K_ - 1 + i; j++) bdd[i] += std::log2((double)j + err);
        }
        for (int iter = 0; iter < 200; iter++)
        {
            if (tot_deg >= deg_bdd) break;
            const int maxi = (int)(std::max_element(bdd.begin(), bdd.end()) - bdd.begin());
            if (maxi != 0)
            {
                if (tot_deg + 2 > deg_bdd) break;
                for (long i = 0; i < K_; i++)
                {
                    bdd[i] -= std::log2((double)(tot_deg + 1));
                    bdd[i] -= std::log2((double)(tot_deg + 2));
                    bdd[i] += 2.0 * std::log2(2.0 * M_PI);
                    if (i != maxi)
                    {
                        bdd[i] += std::log2(std::abs((double)(i - maxi)) + err);
                        bdd[i] += std::log2((double)(i + maxi) + err);
                    }
                    else
                    {
                        bdd[i] += std::log2(err) - 1.0;
                        bdd[i] += std::log2(2.0 * (double)i + err);
                    }
                }
                tot_deg += 2;
            }
            else
            {
                bdd[0] -= std::log2((double)(tot_deg + 1));
                bdd[0] += std::log2(err) - 1.0;
                bdd[0] += std::log2(2.0 * M_PI);
                for (long i = 1; i < K_; i++)
                {
                    bdd[i] -= std::log2((double)(tot_deg + 1));
                    bdd[i] += std::log2(2.0 * M_PI);
                    bdd[i] += std::log2((double)i + err);
                }
                tot_deg += 1;
            }
            nodecount[maxi] += 1;
        }
        if (tot_deg == deg_bdd - 1)
        {
            nodecount[0]++;
            tot_deg++;
        }
        int cnt = 0;
        if (nodecount[0] % 2 != 0) sample_[cnt++].x = 0;
        for (long i = K_ - 1; i > 0; i--)
            for (int j = 1; j <= nodecount[i]; j++)
            {
                const f128 t = (f128)(2 * j - 1) * kPi / (f128)(2 * nodecount[i]);
                sample_[cnt++].x = (f128)i + width_ * cosq(t);
                sample_[cnt++].x = (f128)(-i) - width_ * cosq(t);
            }
        for (int j = 1; j <= nodecount[0] / 2; j++)
        {
            const f128 t = (f128)(2 * j - 1) * kPi / (f128)(2 * nodecount[0]);
            sample_[cnt++].x = width_ * cosq(t);
            sample_[cnt++].x = -width_ * cosq(t);
        }
        if (cnt != deg_ + 2) throw std::logic_error("Remez: initial reference set has the wrong size");
        std::sort(sample_.begin(), sample_.end(), [](const RemezPt &a, const RemezPt &b) { return a.x < b.x; });
        for (auto &p : sample_) p.y = f_(p.x);
    }

    void getcoeffwitherr()
    {
        // Remez.cpp:178-214: sum_j c_j T_j(x_i / K) + (-1)^(i+1) E = f(x_i), i < deg + 2, by
        // Gaussian elimination with partial pivoting
        const long n = deg_ + 2;
        std::vector<f128> m(n * n), v(n);
        for (long i = 0; i < n; i++)
        {
            const f128 u = sample_[i].x / K_;
            f128 *row = &m[i * n];
            row[0] = 1;
            if (deg_ >= 1) row[1] = u;
            for (long j = 2; j < deg_ + 1; j++) row[j] = 2 * u * row[j - 1] - row[j - 2];
            row[deg_ + 1] = 2 * (i % 2) - 1;
            v[i] = sample_[i].y;
        }
        for (long k = 0; k < n; k++)
        {
            long piv = k;
            for (long i = k + 1; i < n; i++)
                if (fabsq(m[i * n + k]) > fabsq(m[piv * n + k])) piv = i;
            if (piv != k)
            {
                for (long j = 0; j < n; j++) std::swap(m[k * n + j], m[piv * n + j]);
                std::swap(v[k], v[piv]);
            }
            const f128 d = m[k * n + k];
            if (d == 0) throw std::runtime_error("Remez: singular reference set");
            for (long i = k + 1; i < n; i++)
            {
                const f128 r = m[i * n + k] / d;
                if (r == 0) continue;
                for (long j = k; j < n; j++) m[i * n + j] -= r * m[k * n + j];
                v[i] -= r * v[k];
            }
        }
        for (long k = n; k-- > 0;)
        {
            f128 t = v[k];
            for (long j = k + 1; j < n; j++) t -= m[k * n + j] * v[j];
            v[k] = t / m[k * n + k];
        }
        for (long i = 0; i <= deg_; i++) coeff_[i] = v[i];
        const f128 sc = powq(2, (f128)prm_.log_round_prec);
        current_err_ = floorq(sc * fabsq(v[deg_ + 1])) / sc;
    }

    f128 errf(f128 x) const { return chebeval(deg_, coeff_, x / K_) - f_(x); }

    void getextreme_local(std::vector<RemezPt> &out, long k) const
    {
        // Remez.cpp:216-386: scan [k - w, k + w] in steps sc; at every change of the error's
        // direction (and at the interval ends) refine the extremum by binary_prec ternary steps;
        // keep it when |error| reaches the current level
        long inc_1 = 0, inc_2 = 0, tmpinc;
        f128 scan_1, scan_2 = (f128)k - width_;
        f128 scan_y1, scan_y2 = errf(scan_2);
        f128 detail[3], prec_sc, prec_ext = 0, prec_x, tmp;
        long prec_iter, prec_ind, tmp_inc;
        bool prec_end;
        out.clear();
        while (scan_2 < (f128)k + width_ + sc_)
        {
            scan_1 = scan_2;
            scan_2 = scan_1 + sc_;
            if (fracpart(scan_2) > width_ + sc_ / 2)
            {
                // past the right end: the last point's side of the interval end
                scan_1 = roundq(scan_1) + width_;
                scan_2 = roundq(scan_2) + 1 - width_;
                scan_y1 = errf(scan_1);
                scan_y2 = errf(scan_2);
                prec_end = false;
                prec_x = scan_1 - sc_;
                while (!prec_end)
                {
                    prec_sc = (scan_1 - prec_x) / 2;
                    prec_end = true;
                    for (int j = 0; j < 3; j++) detail[j] = scan_1 - 2 * prec_sc + prec_sc * j;
                    prec_iter = 0;
                    while (prec_iter < prm_.binary_prec)
                    {
                        prec_ext = errf(detail[0]);
                        prec_ind = 0;
                        for (int j = 1; j < 3; j++)
                        {
                            tmp = errf(detail[j]);
                            if ((inc_2 == 1 && prec_ext < tmp) || (inc_2 == -1 && prec_ext > tmp))
                            {
                                prec_ext = tmp;
                                prec_ind = j;
                            }
                        }
                        if (prec_ind != 2) prec_end = false;
                        prec_x = detail[prec_ind];
                        prec_sc = prec_sc / 2;
                        for (int j = 0; j < 3; j++)
                            detail[j] = (prec_x + prec_sc < scan_1 ? prec_x + prec_sc : scan_1) - 2 * prec_sc + prec_sc * j;
                        prec_iter++;
                    }
                    tmpinc = inc_2 == 1 ? 1 : -1;
                    if (tmpinc * prec_ext >= current_err_)
                    {
                        RemezPt p;
                        p.x = prec_x;
                        p.y = prec_ext;
                        p.locmm = inc_2 == 1 ? 1 : -1;
                        out.push_back(p);
                    }
                    if (!prec_end) inc_2 = -inc_2;
                }
                inc_2 = 0;
            }
            else
            {
                inc_1 = inc_2;
                scan_y1 = scan_y2;
                scan_y2 = errf(scan_2);
                if (scan_y1 < scan_y2)
                    inc_2 = 1;
                else if (scan_y1 > scan_y2)
                    inc_2 = -1;
                else
                    inc_2 = 0;
                if ((inc_1 == 1 && inc_2 != 1) || (inc_1 == -1 && inc_2 != -1) || inc_1 == 0)
                {
                    prec_end = false;
                    tmp_inc = inc_2;
                    prec_x = scan_2;
                    while (!prec_end)
                    {
                        prec_sc = (prec_x - scan_1) / 2;
                        prec_end = true;
                        for (int j = 0; j < 3; j++)
                            detail[j] = inc_1 != 0 ? scan_1 - prec_sc + prec_sc * j : scan_1 + prec_sc * j;
                        prec_iter = 0;
                        while (prec_iter < prm_.binary_prec)
                        {
                            prec_ext = errf(detail[0]);
                            prec_ind = 0;
                            for (int j = 1; j < 3; j++)
                            {
                                tmp = errf(detail[j]);
                                if ((inc_1 == 1 && prec_ext < tmp) || (inc_1 == -1 && prec_ext > tmp))
                                {
                                    prec_ext = tmp;
                                    prec_ind = j;
                                }
                                else if (inc_1 == 0)
                                {
                                    if ((inc_2 == 1 && prec_ext > tmp) || (inc_2 == -1 && prec_ext < tmp))
                                    {
                                        prec_ext = tmp;
                                        prec_ind = j;
                                    }
                                }
                            }
                            if (inc_1 == 0 && prec_ind != 0) prec_end = false;
                            prec_x = detail[prec_ind];
                            prec_sc = prec_sc / 2;
                            for (int j = 0; j < 3; j++)
                            {
                                if (inc_1 == 0)
                                    detail[j] = (prec_x - prec_sc > scan_1 ? prec_x - prec_sc : scan_1) + prec_sc * j;
                                else
                                    detail[j] = prec_x - prec_sc + prec_sc * j;
                            }
                            prec_iter++;
                        }
                        tmpinc = inc_2 == 1 ? -1 : 1;
                        if (tmpinc * prec_ext >= current_err_)
                        {
                            RemezPt p;
                            p.x = prec_x;
                            p.y = prec_ext;
                            p.locmm = inc_2 == 1 ? -1 : 1;
                            out.push_back(p);
                        }
                        if (!prec_end) inc_2 = -inc_2;
                    }
                    inc_2 = tmp_inc;
                }
            }
        }
    }

    void getextreme()
    {
        // Remez.cpp:388-430: every interval scanned on its own thread, then merged in x order
        const long nint = 2 * K_ - 1;
        std::vector<std::vector<RemezPt>> local(nint);
        std::vector<std::thread> thr;
        const long nt = std::max(1L, std::min<long>(nint, (long)std::thread::hardware_concurrency()));
        for (long t = 0; t < nt; t++)
            thr.emplace_back([&, t] {
                for (long i = t; i < nint; i += nt) getextreme_local(local[i], i - K_ + 1);
            });
        for (auto &t : thr) t.join();
        extreme_.clear();
        for (auto &v : local) extreme_.insert(extreme_.end(), v.begin(), v.end());
        max_err = 0;
        for (auto &p : extreme_)
            if (max_err < fabsq(p.y)) max_err = fabsq(p.y);
        std::sort(extreme_.begin(), extreme_.end(), [](const RemezPt &a, const RemezPt &b) { return a.x < b.x; });
    }

    void choosemaxs()
    {
        // Remez.cpp:432-556: one point (the largest |error|) per run of equal sign, then drop
        // the smallest neighbouring pairs (or an end point) until deg + 2 alternating points remain
        const long ec = (long)extreme_.size();
        if (ec < deg_ + 2) throw std::runtime_error("Remez: too few extrema");
        std::vector<RemezPt> extract;
        max_err = 0;
        min_err = 1000;
        std::vector<long> run;
        auto flush = [&] {
            f128 best = 0;
            long bi = run[0];
            for (long i : run)
                if (best < fabsq(extreme_[i].y))
                {
                    best = fabsq(extreme_[i].y);
                    bi = i;
                }
            extract.push_back(extreme_[bi]);
            run.clear();
        };
        long ind = 0;
        while (ind < ec)
        {
            if (run.empty() || extreme_[ind].locmm * extreme_[ind - 1].locmm == 1)
                run.push_back(ind++);
            else
                flush();
        }
        flush();
        long count = (long)extract.size();
        auto erase_at = [&](long i, long k) {
            extract.erase(extract.begin() + i, extract.begin() + i + k);
            count -= k;
        };
        while (count > deg_ + 2)
        {
            f128 minsum = 100000;
            long minindex = 0;
            if (count == deg_ + 3)
            {
                if (fabsq(extract[0].y) > fabsq(extract[count - 1].y))
                    erase_at(count - 1, 1);
                else
                    erase_at(0, 1);
            }
            else if (count == deg_ + 4)
            {
                for (long i = 0; i < count; i++)
                {
                    const f128 s2 = fabsq(extract[i].y) + fabsq(extract[(i + 1) % count].y);
                    if (minsum > s2)
                    {
                        minsum = s2;
                        minindex = i;
                    }
                }
                if (minindex == count - 1)
                {
                    // the pair (last, first): drop the first and the last
                    extract.erase(extract.begin());
                    extract.pop_back();
                    count -= 2;
                }
                else
                    erase_at(minindex, 2);
            }
            else
            {
                for (long i = 0; i < count - 1; i++)
                {
                    const f128 s2 = fabsq(extract[i].y) + fabsq(extract[i + 1].y);
                    if (minsum > s2)
                    {
                        minsum = s2;
                        minindex = i;
                    }
                }
                if (minindex == 0)
                    erase_at(0, 1);
                else if (minindex == count - 2)
                    erase_at(count - 1, 1);
                else
                    erase_at(minindex, 2);
            }
        }
        for (long i = 0; i < deg_ + 2; i++)
        {
            sample_[i].x = extract[i].x;
            sample_[i].y = f_(sample_[i].x);
            if (max_err < fabsq(extract[i].y)) max_err = fabsq(extract[i].y);
            if (min_err > fabsq(extract[i].y)) min_err = fabsq(extract[i].y);
        }
    }

    long K_, deg_;
    std::function<f128(f128)> f_;
    RemezParams prm_;
    f128 width_, sc_, current_err_ = 0;
    double log_width_;
    std::vector<RemezPt> sample_, extreme_;
    std::vector<f128> coeff_;
};

// arcsin by Newton on sin (common/func.cpp:19-26), to binary128 precision
f128 arcsin_newton(f128 x)
{
    f128 r = x;
    for (int i = 0; i < 200 && fabsq(sinq(r) - x) > powq(2, -110); i++) r = r - (sinq(r) - x) / cosq(r);
    return r;
}

// one generated polynomial per parameter set (three bootstrappers share the ResNet's)
std::mutex g_remez_mu;
std::map<std::string, std::vector<double>> g_remez_cache;

std::vector<double> remez_cached(const std::string &key, const std::function<std::vector<double>()> &make)
{
    std::lock_guard<std::mutex> g(g_remez_mu);
    auto it = g_remez_cache.find(key);
    if (it != g_remez_cache.end()) return it->second;
    auto v = make();
    g_remez_cache[key] = v;
    return v;
}
} // namespace

std::vector<double> remez_chebyshev(long K, double log_width, long deg, const std::function<f128(f128)> &f,
                                    double log_scan_step_diff, int *iterations, double *spread)
{
    RemezParams prm;
    prm.log_scan_step_diff = log_scan_step_diff;
    RemezExchange r(K, log_width, deg, f, prm);
    auto cq = r.run();
    if (iterations) *iterations = r.iterations;
    if (spread) *spread = (double)((r.max_err - r.min_err) / r.min_err);
    std::vector<double> out(cq.size());
    for (std::size_t j = 0; j < cq.size(); j++) out[j] = (double)cq[j];
    return out;
}

RemezCos::RemezCos(long K, double lw, long d, long sf) : boundary_K(K), deg(d), scale_factor(sf), log_width(lw) {}

static f128 cos_target(f128 x, long scale_factor)
{
    // RemezCos.h:11-14
    if (scale_factor % 2 == 0) return cosq(2 * kPi * (x - (f128)0.25) / scale_factor);
    return sinq(2 * kPi * x / scale_factor);
}

std::vector<double> RemezCos::chebyshev_coefficients(int *iterations, double *spread) const
{
    // Remez(boundary_K, log_width, deg) with RemezCos::function_value (RemezCos.h)
    const std::string key = "cos " + std::to_string(boundary_K) + " " + std::to_string(log_width) + " " +
                            std::to_string(deg) + " " + std::to_string(scale_factor);
    int it = 0;
    double sp = 0;
    auto c = remez_cached(key, [&] {
        const long sf = scale_factor;
        return remez_chebyshev(boundary_K, log_width, deg, [sf](f128 x) { return cos_target(x, sf); }, 9.5, &it, &sp);
    });
    if (iterations) *iterations = it;
    if (spread) *spread = sp;
    return c;
}

void RemezCos::generate_optimal_poly(boot::Polynomial &poly) const
{
    poly.set_chebyshev(chebyshev_coefficients());
}

double RemezCos::max_error(const boot::Polynomial &poly) const
{
    const double w = std::pow(2.0, -log_width);
    double err = 0;
    for (long i = -(boundary_K - 1); i <= boundary_K - 1; i++)
        for (int j = 0; j <= 64; j++)
        {
            const double x = i - w + 2 * w * j / 64.0;
            err = std::max(err, std::abs(poly.evaluate(x / boundary_K) - (double)cos_target(x, scale_factor)));
        }
    return err;
}

RemezArcsin::RemezArcsin(double lw, long d) : log_width(lw), deg(d) {}

void RemezArcsin::generate_optimal_poly(boot::Polynomial &poly) const
{
    // Remez(1, log_width, deg) with RemezArcsin::function_value = arcsin(x) / (2 pi)
    // (RemezArcsin.h; ModularReducer.cpp:12-17 sets log_scan_step_diff 12 for it)
    const std::string key = "asin " + std::to_string(log_width) + " " + std::to_string(deg);
    auto c = remez_cached(key, [&] {
        return remez_chebyshev(1, log_width, deg, [](f128 x) { return arcsin_newton(x) / (2 * kPi); }, 12);
    });
    poly.set_chebyshev(c);
}

// =========================================================================== ModularReducer
ModularReducer::ModularReducer(long K, double lw, long d, long ndf, long ideg, SEALContext &ctx, CKKSEncoder &enc,
                               Encryptor &encr, Evaluator &ev, RelinKeys &rk, Decryptor &dec)
    : boundary_K(K), log_width(lw), deg(d), num_double_formula(ndf),
      inverse_log_width(-std::log2(std::sin(2 * M_PI * std::pow(2.0, -lw)))), inverse_deg(ideg), context(ctx),
      encoder(enc), encryptor(encr), evaluator(ev), relin_keys(rk), decryptor(dec),
      poly_generator(K, lw, d, 1L << ndf), inverse_poly_generator(inverse_log_width, ideg)
{
    // ModularReducer.cpp:3-20
}

void ModularReducer::double_angle_formula(Ciphertext &cipher)
{
    // ModularReducer.cpp:22-28: cos 2t = 2 cos^2 t - 1
    evaluator.square_inplace(cipher);
    evaluator.relinearize_inplace(cipher, relin_keys);
    evaluator.rescale_to_next_inplace(cipher);
    evaluator.double_inplace(cipher);
    evaluator.add_const(cipher, -1.0, cipher);
}

void ModularReducer::double_angle_formula_scaled(Ciphertext &cipher, double scale_coeff)
{
    // ModularReducer.cpp:30-36
    evaluator.square_inplace(cipher);
    evaluator.relinearize_inplace(cipher, relin_keys);
    evaluator.rescale_to_next_inplace(cipher);
    evaluator.double_inplace(cipher);
    evaluator.add_const(cipher, -scale_coeff, cipher);
}

void ModularReducer::generate_sin_cos_polynomial()
{
    poly_generator.generate_optimal_poly(sin_cos_polynomial);
    sin_cos_polynomial.generate_poly_heap();
}

void ModularReducer::generate_inverse_sine_polynomial()
{
    // ModularReducer.cpp:43-53
    inverse_poly_generator.generate_optimal_poly(inverse_sin_polynomial);
    if (inverse_deg > 3) inverse_sin_polynomial.generate_poly_heap_odd();
    if (inverse_deg == 1)
    {
        scale_inverse_coeff = inverse_sin_polynomial.coeff[1];
        for (int i = 0; i < num_double_formula; i++) scale_inverse_coeff = std::sqrt(scale_inverse_coeff);
        sin_cos_polynomial.constmul(scale_inverse_coeff);
        sin_cos_polynomial.generate_poly_heap();
    }
}

void ModularReducer::write_polynomials()
{
    std::ofstream sin_cos_out("cosine.txt"), inverse_out("inverse_sine.txt");
    sin_cos_polynomial.write_heap_to_file(sin_cos_out);
    inverse_sin_polynomial.write_heap_to_file(inverse_out);
}

void ModularReducer::modular_reduction(Ciphertext &rtn, Ciphertext &cipher)
{
    // ModularReducer.cpp:62-80
    Ciphertext tmp1, tmp2;
    tmp1 = cipher;
    sin_cos_polynomial.homomorphic_poly_evaluation(context, encoder, encryptor, evaluator, relin_keys, tmp2, tmp1,
                                                   decryptor);
    if (inverse_deg == 1)
    {
        double curr_scale = scale_inverse_coeff;
        for (int i = 0; i < num_double_formula; i++)
        {
            curr_scale = curr_scale * curr_scale;
            double_angle_formula_scaled(tmp2, curr_scale);
        }
        rtn = tmp2;
    }
    else
    {
        for (int i = 0; i < num_double_formula; i++) double_angle_formula(tmp2);
        inverse_sin_polynomial.homomorphic_poly_evaluation(context, encoder, encryptor, evaluator, relin_keys, rtn,
                                                           tmp2, decryptor);
    }
}

// ============================================================================= Bootstrapper
Bootstrapper::Bootstrapper(long _loge, long _logn, long _logNh, long _L, double _final_scale, long _boundary_K,
                           long _sin_cos_deg, long _scale_factor, long _inverse_deg, SEALContext &_context,
                           KeyGenerator &_keygen, CKKSEncoder &_encoder, Encryptor &_encryptor, Decryptor &_decryptor,
                           Evaluator &_evaluator, RelinKeys &_relin_keys, GaloisKeys &_gal_keys)
    : loge(_loge), logn(_logn), n(1L << _logn), logNh(_logNh), Nh(1L << _logNh), L(_L), final_scale(_final_scale),
      boundary_K(_boundary_K), sin_cos_deg(_sin_cos_deg), scale_factor(_scale_factor), inverse_deg(_inverse_deg),
      context(_context), keygen(_keygen), encoder(_encoder), encryptor(_encryptor), decryptor(_decryptor),
      evaluator(_evaluator), relin_keys(_relin_keys), gal_keys(_gal_keys)
{
    // Bootstrapper.cpp:3-17
    mod_reducer = std::make_unique<ModularReducer>(boundary_K, (double)loge, sin_cos_deg, scale_factor, inverse_deg,
                                                   context, encoder, encryptor, evaluator, relin_keys, decryptor);
}

void Bootstrapper::addLeftRotKeys_Linear_to_vector_3(std::vector<int> &gal_steps_vector)
{
    // Bootstrapper.cpp:82-176: the baby and giant steps of the three CoeffToSlot BSGS levels
    const int div_part1 = (int)std::floor(logn / 3.0);
    const int div_part2 = (int)std::floor((logn - div_part1) / 2.0);
    const int div_part3 = (int)logn - div_part1 - div_part2;
    const int totlen1 = (1 << div_part1) - 1, totlen2 = (1 << div_part2) - 1, totlen3 = (1 << div_part3) - 1;
    const int basicstep1 = 1 << (logn - div_part1), basicstep2 = 1 << (logn - div_part1 - div_part2),
              basicstep3 = 1;
    const int gs1 = giantstep(totlen1 + 1);
    const int gs1_e = logn != logNh ? giantstep(2 * totlen1 + 1) : 0;
    const int gs2 = giantstep(2 * totlen2 + 1), gs3 = giantstep(2 * totlen3 + 1);
    const int basicstart1 = -totlen1 + gs1 * (int)std::floor((totlen1 + 0.0) / (gs1 + 0.0));
    const int giantfirst1 = -(int)std::floor((totlen1 + 0.0) / (gs1 + 0.0));
    const int giantlast1 = (int)std::floor((2 * totlen1 + 0.0) / (gs1 + 0.0)) + giantfirst1;
    const int giantlast1_e = logn != logNh ? (int)std::floor((totlen1 + 0.0) / (gs1 + 0.0)) : 0;
    const int basicstart2 = -totlen2 + gs2 * (int)std::floor((totlen2 + 0.0) / (gs2 + 0.0));
    const int giantfirst2 = -(int)std::floor((totlen2 + 0.0) / (gs2 + 0.0));
    const int giantlast2 = (int)std::floor((2 * totlen2 + 0.0) / (gs2 + 0.0)) + giantfirst2;
    const int basicstart3 = -totlen3 + gs3 * (int)std::floor((totlen3 + 0.0) / (gs3 + 0.0));
    const int giantfirst3 = -(int)std::floor((totlen3 + 0.0) / (gs3 + 0.0));
    const int giantlast3 = (int)std::floor((2 * totlen3 + 0.0) / (gs3 + 0.0)) + giantfirst3;
    const int nh = (int)Nh;
    auto add = [&](int st) {
        if (std::find(gal_steps_vector.begin(), gal_steps_vector.end(), st) == gal_steps_vector.end())
            gal_steps_vector.push_back(st);
    };
    for (int i = basicstart1; i < basicstart1 + gs1; i++)
        if (i != 0) add((nh + i * basicstep1) % nh);
    for (int i = 1; i < gs1_e; i++) add(i * basicstep1);
    for (int i = basicstart2; i < basicstart2 + gs2; i++)
        if (i != 0) add((nh + i * basicstep2) % nh);
    for (int i = basicstart3; i < basicstart3 + gs3; i++)
        if (i != 0) add((nh + i * basicstep3) % nh);
    for (int i = giantfirst1; i <= giantlast1; i++)
        if (i != 0) add((nh + i * gs1 * basicstep1) % nh);
    for (int i = 1; i <= giantlast1_e; i++) add(i * gs1_e * basicstep1);
    for (int i = giantfirst2; i <= giantlast2; i++)
        if (i != 0) add((nh + i * gs2 * basicstep2) % nh);
    for (int i = giantfirst3; i <= giantlast3; i++)
        if (i != 0) add((nh + i * gs3 * basicstep3) % nh);
}

void Bootstrapper::addBootKeys_3(GaloisKeys &keys)
{
    // Bootstrapper.cpp:367-385
    std::vector<int> gal_steps_vector{ 0 };
    for (int i = 0; i < logNh; i++) gal_steps_vector.push_back(1 << i);
    addLeftRotKeys_Linear_to_vector_3(gal_steps_vector);
    keygen.create_galois_keys(gal_steps_vector, keys);
    slot_vec.push_back(logn);
    change_logn(logn);
}

void Bootstrapper::change_logn(long new_logn)
{
    // Bootstrapper.cpp:499-510
    logn = new_logn;
    n = 1L << logn;
    slot_index = -1;
    for (std::size_t i = 0; i < slot_vec.size(); i++)
        if (slot_vec[i] == logn)
        {
            slot_index = (long)i;
            break;
        }
    if (slot_index == -1) throw std::logic_error("LT coefficients were not generated for this logn");
}

namespace
{
// A linear map on n-slot vectors as diagonals: out[x] = sum_d D_d[x] * v[(x + d) mod n].
using Diags = std::map<int, std::vector<cd>>;

// Butterfly stage i of the special FFT without bit reversal (the decoding direction; the
// stages orig_coeffvec of Bootstrapper.cpp:512-553): blocks of 2^(i+1), twiddle
// zeta_j = exp(i pi 5^j / 2^(i+2)) for j < 2^i: (a, b) -> (a + zeta b, a - zeta b).
Diags fft_stage(int logn, int i)
{
    const int n = 1 << logn, b = 1 << (i + 1), h = b / 2;
    Diags D;
    for (int d : { -h, 0, h }) D[d].assign(n, 0.0);
    const double theta = M_PI / (2 * n) * (1 << (logn - 1 - i));
    long power = 1;
    for (int j = 0; j < h; j++)
    {
        const cd zeta = std::polar(1.0, theta * power);
        for (int k = 0; k < n / b; k++)
        {
            const int x = k * b + j;
            D[0][x] = 1.0;
            D[h][x] = zeta;
            D[-h][x + h] = 1.0;
            D[0][x + h] = -zeta;
        }
        power = (5 * power) % (1L << (i + 3));
    }
    return D;
}

// Inverse butterfly stage i (orig_invcoeffvec, Bootstrapper.cpp:555-590): blocks of n / 2^i,
// (x, y) -> ((x + y) / 2, zeta^-1 (x - y) / 2) -- the inverse of fft_stage(logn - 1 - i).
Diags ifft_stage(int logn, int i)
{
    const int n = 1 << logn, b = n >> i, h = b / 2;
    Diags D;
    for (int d : { -h, 0, h }) D[d].assign(n, 0.0);
    const double theta = -M_PI / (2 * n) * (1 << i);
    long power = 1;
    for (int j = 0; j < h; j++)
    {
        const cd zeta = std::polar(1.0, theta * power);
        for (int k = 0; k < n / b; k++)
        {
            const int x = k * b + j;
            D[0][x] = 0.5;
            D[h][x] = 0.5;
            D[-h][x + h] = 0.5 * zeta;
            D[0][x + h] = -0.5 * zeta;
        }
        power = (5 * power) % (1L << ((logn - 1 - i) + 3));
    }
    return D;
}

// A o B (B applied first): (A B)_{a+b}[x] = A_a[x] B_b[x + a]
Diags compose(const Diags &A, const Diags &B, int n)
{
    Diags R;
    for (const auto &a : A)
        for (const auto &bb : B)
        {
            auto &r = R[a.first + bb.first];
            if (r.empty()) r.assign(n, 0.0);
            for (int x = 0; x < n; x++) r[x] += a.second[x] * bb.second[((x + a.first) % n + n) % n];
        }
    return R;
}

Diags merge_stages(bool inverse, int logn, int first, int last)
{
    const int n = 1 << logn;
    Diags M = inverse ? ifft_stage(logn, first) : fft_stage(logn, first);
    for (int s = first + 1; s < last; s++) M = compose(inverse ? ifft_stage(logn, s) : fft_stage(logn, s), M, n);
    return M;
}

// BSGS layout: index offset/step + totlen (bsgs_linear_transform), or offset/step mod (totlen+1)
// (rotated_bsgs_linear_transform, for a level whose offsets wrap around the n-slot period)
std::vector<std::vector<cd>> layout(const Diags &M, int n, int step, int totlen, bool cyclic)
{
    std::vector<std::vector<cd>> out(cyclic ? totlen + 1 : 2 * totlen + 1, std::vector<cd>(n, 0.0));
    for (const auto &d : M)
    {
        if (d.first % step) throw std::logic_error("LT diagonal off the BSGS grid");
        const int k = d.first / step;
        const int idx = cyclic ? ((k % (totlen + 1)) + (totlen + 1)) % (totlen + 1) : k + totlen;
        if (idx < 0 || idx >= (int)out.size()) throw std::logic_error("LT diagonal outside the BSGS range");
        for (int x = 0; x < n; x++) out[idx][x] += d.second[x];
    }
    return out;
}
} // namespace

namespace boot
{
void lt_coefficients_3_merged(int ln, long logNh, long boundary_K, LTDiags &f1, LTDiags &f2, LTDiags &f3,
                              LTDiags &i1, LTDiags &i2, LTDiags &i3)
{
    // The same diagonals derived independently: each group of butterfly stages as a product of
    // sparse diagonal matrices (compose / layout above), with the reference's scalings and 2n-slot
    // extensions.  Equal to lt_coefficients_3 up to rounding (a few ULPs, boot_host_test); kept as
    // the check of the reference-order restatement below.
    const int cn = 1 << ln;
    if (ln > logNh) throw std::logic_error("slot count above N/2");
    const cd I(0, 1);
    if (ln == logNh)
    {
        // full slots (genfftcoeff_3 / geninvfftcoeff_3, curr_logn == logNh branches,
        // Bootstrapper.cpp:1131-1249, 1531-1650): no 2n-slot extensions; the last SlotToCoeff
        // group and the first CoeffToSlot group wrap around the slot period (rotated BSGS); the
        // CoeffToSlot input is scaled by 1/K and its last group by 1/2 (the real/imaginary split of
        // coefftoslot_full_3 doubles it back).
        {
            const int d3 = (int)std::floor(ln / 3.0), d2 = (int)std::floor((ln - d3) / 2.0), d1 = ln - d3 - d2;
            const int t1 = (1 << d1) - 1, t2 = (1 << d2) - 1, t3 = (1 << d3) - 1;
            f1 = layout(merge_stages(false, ln, 0, d1), cn, 1, t1, false);
            f2 = layout(merge_stages(false, ln, d1, d1 + d2), cn, 1 << d1, t2, false);
            f3 = layout(merge_stages(false, ln, d1 + d2, ln), cn, 1 << (d1 + d2), t3, true);
        }
        {
            const int d1 = (int)std::floor(ln / 3.0), d2 = (int)std::floor((ln - d1) / 2.0), d3 = ln - d1 - d2;
            const int t1 = (1 << d1) - 1, t2 = (1 << d2) - 1, t3 = (1 << d3) - 1;
            i1 = layout(merge_stages(true, ln, 0, d1), cn, 1 << (ln - d1), t1, true);
            i2 = layout(merge_stages(true, ln, d1, d1 + d2), cn, 1 << (ln - d1 - d2), t2, false);
            i3 = layout(merge_stages(true, ln, d1 + d2, ln), cn, 1, t3, false);
            for (auto &v : i1)
                for (auto &x : v) x *= 1.0 / (double)boundary_K;
            for (auto &v : i3)
                for (auto &x : v) x *= 0.5;
        }
        return;
    }
    {
        // SlotToCoeff: stages 0.. in groups of div1 (step 1), div2 (step 2^div1), div3
        const int d3 = (int)std::floor(ln / 3.0), d2 = (int)std::floor((ln - d3) / 2.0), d1 = ln - d3 - d2;
        const int t1 = (1 << d1) - 1, t2 = (1 << d2) - 1, t3 = (1 << d3) - 1;
        f1 = layout(merge_stages(false, ln, 0, d1), cn, 1, t1, false);
        f2 = layout(merge_stages(false, ln, d1, d1 + d2), cn, 1 << d1, t2, false);
        f3 = layout(merge_stages(false, ln, d1 + d2, ln), cn, 1 << (d1 + d2), t3, false);
        for (auto *g : { &f1, &f2 })
            for (auto &v : *g)
            {
                v.resize(2 * cn);
                for (int j = 0; j < cn; j++) v[j + cn] = v[j];
            }
        for (auto &v : f3)
        {
            v.resize(2 * cn);
            for (int j = 0; j < cn; j++) v[j + cn] = I * v[j];
        }
    }
    {
        // CoeffToSlot: inverse stages in groups of div1 (step 2^(logn-div1), cyclic), div2, div3 (step 1)
        const int d1 = (int)std::floor(ln / 3.0), d2 = (int)std::floor((ln - d1) / 2.0), d3 = ln - d1 - d2;
        const int t1 = (1 << d1) - 1, t2 = (1 << d2) - 1, t3 = (1 << d3) - 1;
        i1 = layout(merge_stages(true, ln, 0, d1), cn, 1 << (ln - d1), t1, true);
        i2 = layout(merge_stages(true, ln, d1, d1 + d2), cn, 1 << (ln - d1 - d2), t2, false);
        i3 = layout(merge_stages(true, ln, d1 + d2, ln), cn, 1, t3, false);
        const double s1 = 1.0 / ((double)boundary_K * (double)(1L << (logNh - ln)));
        for (auto &v : i1)
            for (auto &x : v) x *= s1;
        for (auto &v : i3)
        {
            v.resize(2 * cn);
            for (int j = 0; j < cn; j++)
            {
                v[j] *= 0.5;
                v[j + cn] = -I * v[j];
            }
        }
    }
}
} // namespace boot

// ------------------------------------------------------------------ reference operation order
// genorigcoeff + genfftcoeff_3 + geninvfftcoeff_3 (Bootstrapper.cpp:512-592, 1116-1383, 1516-1776)
// restated with the reference's loops, so every double is produced by the same operations in the
// same order: the butterfly stages (orig_coeffvec / orig_invcoeffvec) from std::polar, each merged
// diagonal as the running product of 3^div stage entries, summed into its BSGS slot case by case.
// The reference's CNN target is built at -O0 (cnn_ckks/CMakeLists.txt), so std::polar's cos() and
// sin() are two libm calls (never merged into sincos(), whose last bit differs for some angles), and
// a complex product is (ac - bd) + (ad + bc) i without FMA contraction.
namespace
{
// one butterfly stage: entries [3][n] (index 0, 1, 2 = offsets -w, 0, +w of the reference's tmpcount)
using StageCoeff = std::array<std::vector<cd>, 3>;

__attribute__((noinline)) cd polar_o0(double theta)
{
    double t = theta;
    const double c = std::cos(t);
    asm volatile("" : "+x"(t)); // a separate sin() call, as at -O0
    const double sn = std::sin(t);
    return cd(1.0 * c, 1.0 * sn);
}

// (a + bi)(c + di) = (ac - bd) + (ad + bc) i, each product rounded, no FMA (libgcc __muldc3 / GCC's
// inline expansion for finite operands)
__attribute__((optimize("fp-contract=off"))) inline cd cmul(const cd &x, const cd &y)
{
    const double a = x.real(), b = x.imag(), c = y.real(), d = y.imag();
    const double ac = a * c, bd = b * d, ad = a * d, bc = b * c;
    return cd(ac - bd, ad + bc);
}

__attribute__((optimize("fp-contract=off"))) void genorigcoeff_one(int ln, std::vector<StageCoeff> &fwd,
                                                                      std::vector<StageCoeff> &inv)
{
    // Bootstrapper.cpp:512-592 for one slot count (u fixed)
    const int n = 1 << ln;
    fwd.assign(ln, StageCoeff{});
    inv.assign(ln, StageCoeff{});
    for (auto &st : fwd)
        for (auto &v : st) v.assign(n, cd(0.0, 0.0));
    for (auto &st : inv)
        for (auto &v : st) v.assign(n, cd(0.0, 0.0));
    double theta_0 = M_PI / (double)(2L * n);
    int blocklen = 1, blockcount = n;
    for (int i = 0; i < ln; i++)
    {
        blocklen <<= 1;
        blockcount >>= 1;
        const double theta = theta_0 * (double)(1 << (ln - 1 - i));
        int power = 1;
        cd zeta = polar_o0(theta * (double)power);
        for (int j = 0; j < blocklen / 2; j++)
        {
            for (int k = 0; k < blockcount; k++)
            {
                const int a = k * blocklen + j, b = a + blocklen / 2;
                fwd[i][1][a] = 1.0;
                fwd[i][1][b] = -zeta;
                fwd[i][0][a] = 0.0;
                fwd[i][0][b] = 1.0;
                fwd[i][2][a] = zeta;
                fwd[i][2][b] = 0.0;
            }
            power = (5 * power) % (1 << (i + 3));
            zeta = polar_o0(theta * (double)power);
        }
    }
    theta_0 = -M_PI / (double)(2L * n);
    blocklen = n;
    blockcount = 1;
    for (int i = 0; i < ln; i++)
    {
        const double theta = theta_0 * (double)(1 << i);
        int power = 1;
        cd zeta = polar_o0(theta * (double)power);
        for (int j = 0; j < blocklen / 2; j++)
        {
            for (int k = 0; k < blockcount; k++)
            {
                const int a = k * blocklen + j, b = a + blocklen / 2;
                inv[i][1][a] = 0.5;
                inv[i][1][b] = cd(-0.5 * zeta.real(), -0.5 * zeta.imag());
                inv[i][0][a] = 0.0;
                inv[i][0][b] = cd(0.5 * zeta.real(), 0.5 * zeta.imag());
                inv[i][2][a] = 0.5;
                inv[i][2][b] = 0.0;
            }
            power = (5 * power) % (1 << ((ln - 1 - i) + 3));
            zeta = polar_o0(theta * (double)power);
        }
        blocklen >>= 1;
        blockcount <<= 1;
    }
}

// One merged group: the reference's loop over the 3^div stage-entry choices (genfftcoeff_3's j loop).
// Case j picks entry tmpcount[p] of stage p0 + p; its offset weight is 2^p (forward, `rev` false) or
// 2^(div-1-p) (inverse); the running product is read at (k + step (n + current_pos)) mod n and added
// into out[slot(pos)][k] for k < n.
template <class Slot>
__attribute__((optimize("fp-contract=off"))) void merge_group(const std::vector<StageCoeff> &orig, int p0, int div,
                                                              bool rev, int step, int n, Slot slot, boot::LTDiags &out)
{
    std::vector<int> tmpcount(div);
    std::vector<cd> tmpvec(n);
    const int all_case_count = (int)std::pow(3, div);
    auto wt = [&](int p) { return rev ? 1 << (div - 1 - p) : 1 << p; };
    for (int j = 0; j < all_case_count; j++)
    {
        int ind = j, pos = 0;
        for (int p = 0; p < div; p++)
        {
            const int ind_res = ind % 3;
            pos += (ind_res - 1) * wt(p);
            tmpcount[p] = ind_res;
            ind = (ind - ind_res) / 3;
        }
        int current_pos = pos;
        for (int k = 0; k < n; k++) tmpvec[k] = cd(1.0, 0.0);
        for (int p = 0; p < div; p++)
        {
            current_pos = current_pos - (tmpcount[p] - 1) * wt(p);
            const std::vector<cd> &st = orig[p0 + p][tmpcount[p]];
            for (int k = 0; k < n; k++) tmpvec[k] = cmul(tmpvec[k], st[(k + step * (n + current_pos)) % n]);
        }
        std::vector<cd> &dst = out[slot(pos)];
        for (int k = 0; k < n; k++) dst[k] += tmpvec[k];
    }
}
} // namespace

namespace boot
{
__attribute__((optimize("fp-contract=off"))) void lt_coefficients_3(int ln, long logNh, long boundary_K, LTDiags &f1,
                                                                       LTDiags &f2, LTDiags &f3, LTDiags &i1,
                                                                       LTDiags &i2, LTDiags &i3)
{
    if (ln > logNh) throw std::logic_error("slot count above N/2");
    const int n = 1 << ln;
    const bool full = ln == logNh;
    std::vector<StageCoeff> of, oi;
    genorigcoeff_one(ln, of, oi);
    const int ext = full ? 1 : 2; // the sparse branch's diagonals are 2n long (second half filled below)
    auto sized = [&](LTDiags &g, int count, int len) { g.assign(count, std::vector<cd>(len, cd(0.0, 0.0))); };
    {
        // genfftcoeff_3 (Bootstrapper.cpp:1116-1383)
        const int d3 = (int)std::floor(ln / 3.0), d2 = (int)std::floor((ln - d3) / 2.0), d1 = ln - d3 - d2;
        const int t1 = (1 << d1) - 1, t2 = (1 << d2) - 1, t3 = (1 << d3) - 1;
        const int s1 = 1, s2 = 1 << d1, s3 = 1 << (d1 + d2);
        sized(f1, 2 * t1 + 1, ext * n);
        sized(f2, 2 * t2 + 1, ext * n);
        sized(f3, full ? t3 + 1 : 2 * t3 + 1, ext * n);
        merge_group(of, 0, d1, false, s1, n, [&](int pos) { return pos + t1; }, f1);
        merge_group(of, d1, d2, false, s2, n, [&](int pos) { return pos + t2; }, f2);
        if (full)
            merge_group(of, d1 + d2, d3, false, s3, n, [&](int pos) { return (pos + t3 + 1) % (t3 + 1); }, f3);
        else
            merge_group(of, d1 + d2, d3, false, s3, n, [&](int pos) { return pos + t3; }, f3);
        if (!full)
        {
            for (auto *g : { &f1, &f2 })
                for (auto &v : *g)
                    for (int j = 0; j < n; j++) v[j + n] = v[j];
            for (auto &v : f3)
                for (int j = 0; j < n; j++) v[j + n] = cmul(cd(0.0, 1.0), v[j]);
        }
    }
    {
        // geninvfftcoeff_3 (Bootstrapper.cpp:1516-1776)
        const int d1 = (int)std::floor(ln / 3.0), d2 = (int)std::floor((ln - d1) / 2.0), d3 = ln - d1 - d2;
        const int t1 = (1 << d1) - 1, t2 = (1 << d2) - 1, t3 = (1 << d3) - 1;
        const int s1 = 1 << (ln - d1), s2 = 1 << (ln - d1 - d2), s3 = 1;
        sized(i1, t1 + 1, n);
        sized(i2, 2 * t2 + 1, n);
        sized(i3, 2 * t3 + 1, full ? n : 2 * n);
        merge_group(oi, 0, d1, true, s1, n, [&](int pos) { return (pos + t1 + 1) % (t1 + 1); }, i1);
        merge_group(oi, d1, d2, true, s2, n, [&](int pos) { return pos + t2; }, i2);
        merge_group(oi, d1 + d2, d3, true, s3, n, [&](int pos) { return pos + t3; }, i3);
        // complex<double> *= double scales both parts by the same double
        const double sc1 = full ? 1.0 / (double)boundary_K : 1.0 / (double)(boundary_K * (1L << (logNh - ln)));
        for (auto &v : i1)
            for (int j = 0; j < n; j++) v[j] = cd(v[j].real() * sc1, v[j].imag() * sc1);
        for (auto &v : i3)
            for (int j = 0; j < n; j++)
            {
                v[j] = cd(v[j].real() * 0.5, v[j].imag() * 0.5);
                if (!full) v[j + n] = cmul(cd(0.0, -1.0), v[j]);
            }
    }
}
} // namespace boot

void Bootstrapper::generate_LT_coefficient_3()
{
    const std::size_t U = slot_vec.size();
    fftcoeff1.assign(U, {});
    fftcoeff2.assign(U, {});
    fftcoeff3.assign(U, {});
    invfftcoeff1.assign(U, {});
    invfftcoeff2.assign(U, {});
    invfftcoeff3.assign(U, {});
    for (std::size_t u = 0; u < U; u++)
        boot::lt_coefficients_3((int)slot_vec[u], logNh, boundary_K, fftcoeff1[u], fftcoeff2[u], fftcoeff3[u],
                                invfftcoeff1[u], invfftcoeff2[u], invfftcoeff3[u]);
}

void Bootstrapper::prepare_mod_polynomial()
{
    mod_reducer->generate_sin_cos_polynomial();
    mod_reducer->generate_inverse_sine_polynomial();
}

bool Bootstrapper::PtKey::operator<(const PtKey &o) const
{
    if (diag != o.diag) return diag < o.diag;
    if (shift != o.shift) return shift < o.shift;
    if (limbs != o.limbs) return limbs < o.limbs;
    if (scale != o.scale) return scale < o.scale;
    if (coeff_logn != o.coeff_logn) return coeff_logn < o.coeff_logn;
    return coeff_scale < o.coeff_scale;
}

namespace
{
std::mutex g_pt_mu;
// the input scale of the bootstrap running on this thread -- and fiber: the fibers of a
// seal::FiberBatch interleave on one thread at every merge point (Bootstrapper objects are shared by
// the threads of an image batch, like the reference's OpenMP team shares bootstrapper_1..3)
thread_local std::vector<double> tl_initial_scales;
double &initial_scale_slot()
{
    const std::size_t i = (std::size_t)(seal::FiberBatch::current() + 1);
    if (tl_initial_scales.size() <= i) tl_initial_scales.resize(i + 1, 0.0);
    return tl_initial_scales[i];
}
bool pt_cache_on()
{
    const char *e = std::getenv("MHE_BOOT_PT_CACHE");
    return !(e && e[0] == '0');
}
} // namespace

void Bootstrapper::multiply_diag(Ciphertext &ct, const std::vector<cd> &diag, int coeff_logn, int shift,
                                 Ciphertext &dest, double coeff_scale, bool accumulate)
{
    Plaintext local;
    const Plaintext &pt = diag_plain(ct, diag, coeff_logn, shift, coeff_scale, local);
    // accumulate: dest += ct * pt (the loop's add_inplace_reduced_error fused into the product)
    if (accumulate)
        evaluator.multiply_plain_add_reduced_error(dest, ct, pt);
    else
        evaluator.multiply_plain(ct, pt, dest);
}

void Bootstrapper::diag_sum(const std::vector<Ciphertext *> &cts, const std::vector<const std::vector<cd> *> &diags,
                            int coeff_logn, int shift, double coeff_scale, Ciphertext &dest)
{
    // multiply_diag(cts[0], ..., dest) then multiply_diag(cts[j], ..., dest, accumulate) for j > 0:
    // the products and their sum in one pass (Evaluator::multiply_plain_sum), the same words
    std::vector<Plaintext> locals(cts.size());
    std::vector<const Ciphertext *> cs;
    std::vector<const Plaintext *> ps;
    for (std::size_t j = 0; j < cts.size(); j++)
    {
        ps.push_back(&diag_plain(*cts[j], *diags[j], coeff_logn, shift, coeff_scale, locals[j]));
        cs.push_back(cts[j]);
    }
    evaluator.multiply_plain_sum(cs, ps, dest);
}

const Plaintext &Bootstrapper::diag_plain(Ciphertext &ct, const std::vector<cd> &diag, int coeff_logn, int shift,
                                          double coeff_scale, Plaintext &local)
{
    // rotation(coeff_logn, Nh, shift, diag) + multiply_vector_reduced_error (Bootstrapper.cpp:1983-1984):
    // the diagonal is encoded at ct.scale() on the first level and kept at ct's level
    const PtKey key{ &diag, shift, ct.coeff_modulus_size(), ct.scale(), coeff_scale, coeff_logn };
    const Plaintext *pt = nullptr;
    if (pt_cache_on())
    {
        std::lock_guard<std::mutex> lk(g_pt_mu);
        auto it = pt_cache_.find(key);
        if (it != pt_cache_.end()) pt = &it->second;
    }
    if (!pt)
    {
        std::vector<cd> rc;
        rotation(coeff_logn, (int)Nh, shift, diag, rc);
        if (coeff_scale != 1.0)
            for (auto &x : rc) x *= coeff_scale;
        evaluator.encode_vector_for(ct, rc, local);
        if (pt_cache_on())
        {
            std::lock_guard<std::mutex> lk(g_pt_mu);
            pt = &pt_cache_.emplace(key, std::move(local)).first->second;
        }
        else
            pt = &local;
    }
    return *pt;
}

std::size_t Bootstrapper::verify_cache()
{
    // re-encode every cached diagonal and compare (debugging aid; synchronises)
    std::lock_guard<std::mutex> lk(g_pt_mu);
    std::size_t bad_entries = 0;
    for (const auto &kv : pt_cache_)
    {
        const PtKey &k = kv.first;
        auto cdp = context.first_context_data();
        while (cdp && cdp->parms().coeff_modulus().size() != k.limbs) cdp = cdp->next_context_data();
        if (!cdp) continue;
        Ciphertext dummy(context, cdp->parms_id());
        dummy.resize(context, cdp->parms_id(), 2);
        dummy.scale() = k.scale;
        std::vector<cd> rc;
        rotation(k.coeff_logn, (int)Nh, k.shift, *static_cast<const std::vector<cd> *>(k.diag), rc);
        if (k.coeff_scale != 1.0)
            for (auto &x : rc) x *= k.coeff_scale;
        Plaintext fresh;
        evaluator.encode_vector_for(dummy, rc, fresh);
        const std::uint64_t *a = fresh.store().host(), *b = kv.second.store().host();
        std::size_t bad = 0;
        for (std::size_t i = 0; i < fresh.store().words(); i++) bad += a[i] != b[i];
        if (bad)
        {
            bad_entries++;
            std::fprintf(stderr, "pt cache entry corrupt: diag %p shift %d limbs %zu scale 2^%.3f logn %d: %zu words\n",
                         k.diag, k.shift, k.limbs, std::log2(k.scale), k.coeff_logn, bad);
        }
    }
    std::fprintf(stderr, "pt cache check: %zu entries, %zu corrupt\n", pt_cache_.size(), bad_entries);
    return bad_entries;
}

void Bootstrapper::bsgs_linear_transform(Ciphertext &rtncipher, Ciphertext &cipher, int totlen, int basicstep,
                                         int coeff_logn, const std::vector<std::vector<cd>> &fftcoeff,
                                         double coeff_scale)
{
    // Bootstrapper.cpp:1952-2016 (coeff_scale: sfl_half_3's fftcoeff3_scale factor)
    const int gs1 = giantstep(2 * totlen + 1);
    const int basicstart1 = -totlen + gs1 * (int)std::floor((totlen + 0.0) / (gs1 + 0.0));
    const int giantfirst1 = -(int)std::floor((totlen + 0.0) / (gs1 + 0.0));
    const int giantlast1 = (int)std::floor((2 * totlen + 0.0) / (gs1 + 0.0)) + giantfirst1;
    const int nh = (int)Nh;
    std::vector<Ciphertext> babyct(gs1);
    // the baby-step rotations of one input are independent: batched launches
    {
        std::vector<const Ciphertext *> in;
        std::vector<int> st;
        std::vector<Ciphertext *> out;
        for (int i = basicstart1; i < basicstart1 + gs1; i++)
        {
            if (i == 0)
                babyct[i - basicstart1] = cipher;
            else
            {
                in.push_back(&cipher);
                st.push_back((nh + i * basicstep) % nh);
                out.push_back(&babyct[i - basicstart1]);
            }
        }
        evaluator.rotate_vectors(in, st, gal_keys, out);
    }
    // every giant step's inner sum first, then their rotations (independent) in batched launches,
    // then the outer sum in the reference's order: the same operations on the same words
    const int ng = giantlast1 - giantfirst1 + 1;
    std::vector<Ciphertext> giantct(ng), rotct(ng);
    for (int i = giantfirst1; i <= giantlast1; i++)
    {
        const int jlast = i != giantlast1 ? basicstart1 + gs1 - 1 : totlen - i * gs1;
        std::vector<Ciphertext *> cts;
        std::vector<const std::vector<cd> *> diags;
        for (int j = basicstart1; j <= jlast; j++)
        {
            cts.push_back(&babyct[j - basicstart1]);
            diags.push_back(&fftcoeff[(i * gs1 + j) + totlen]);
        }
        if (!cts.empty()) diag_sum(cts, diags, coeff_logn, (-i) * gs1 * basicstep, coeff_scale, giantct[i - giantfirst1]);
    }
    giant_rotate_sum(giantct, rotct, giantfirst1, gs1, basicstep, rtncipher);
}

void Bootstrapper::giant_rotate_sum(std::vector<Ciphertext> &giantct, std::vector<Ciphertext> &rotct, int first,
                                    int gs, int basicstep, Ciphertext &rtncipher)
{
    // giant step i = first + k: rotate its inner sum by i * gs * basicstep (i != 0), then
    // tmpct = sum over k in order (Bootstrapper.cpp:1990-2015 / 2059-2084)
    const int nh = (int)Nh;
    std::vector<const Ciphertext *> in;
    std::vector<int> st;
    std::vector<Ciphertext *> out;
    for (std::size_t k = 0; k < giantct.size(); k++)
    {
        const int i = first + (int)k;
        if (i == 0) continue;
        in.push_back(&giantct[k]);
        st.push_back((nh + i * gs * basicstep) % nh);
        out.push_back(&rotct[k]);
    }
    evaluator.rotate_vectors(in, st, gal_keys, out);
    Ciphertext tmpct;
    for (std::size_t k = 0; k < giantct.size(); k++)
    {
        Ciphertext &term = (first + (int)k != 0) ? rotct[k] : giantct[k];
        if (k == 0)
            tmpct = std::move(term); // the terms are dead after the sum: no device copies
        else
            evaluator.add_inplace_reduced_error(tmpct, term);
    }
    rtncipher = std::move(tmpct);
}

void Bootstrapper::rotated_bsgs_linear_transform(Ciphertext &rtncipher, Ciphertext &cipher, int totlen,
                                                 int basicstep, int coeff_logn,
                                                 const std::vector<std::vector<cd>> &fftcoeff, double coeff_scale)
{
    // Bootstrapper.cpp:2018-2085
    const int gs2 = giantstep(totlen + 1);
    const int giantlast2 = (int)std::floor((totlen + 0.0) / (gs2 + 0.0));
    const int nh = (int)Nh;
    std::vector<Ciphertext> babyct(gs2);
    {
        std::vector<const Ciphertext *> in;
        std::vector<int> st;
        std::vector<Ciphertext *> out;
        for (int i = 0; i < gs2; i++)
        {
            if (i == 0)
                babyct[i] = cipher;
            else
            {
                in.push_back(&cipher);
                st.push_back((nh + i * basicstep) % nh);
                out.push_back(&babyct[i]);
            }
        }
        evaluator.rotate_vectors(in, st, gal_keys, out);
    }
    std::vector<Ciphertext> giantct(giantlast2 + 1), rotct(giantlast2 + 1);
    for (int i = 0; i <= giantlast2; i++)
    {
        const int jlast = i != giantlast2 ? gs2 - 1 : totlen - i * gs2;
        std::vector<Ciphertext *> cts;
        std::vector<const std::vector<cd> *> diags;
        for (int j = 0; j <= jlast; j++)
        {
            cts.push_back(&babyct[j]);
            diags.push_back(&fftcoeff[i * gs2 + j]);
        }
        if (!cts.empty()) diag_sum(cts, diags, coeff_logn, (-i) * gs2 * basicstep, coeff_scale, giantct[i]);
    }
    giant_rotate_sum(giantct, rotct, 0, gs2, basicstep, rtncipher);
}

void Bootstrapper::sfl_half_3(Ciphertext &rtncipher, Ciphertext &cipher)
{
    // Bootstrapper.cpp:2453-2490
    const int div_part3 = (int)std::floor(logn / 3.0);
    const int div_part2 = (int)std::floor((logn - div_part3) / 2.0);
    const int div_part1 = (int)logn - div_part3 - div_part2;
    const int totlen1 = (1 << div_part1) - 1, totlen2 = (1 << div_part2) - 1, totlen3 = (1 << div_part3) - 1;
    const int basicstep1 = 1, basicstep2 = 1 << div_part1, basicstep3 = 1 << (div_part1 + div_part2);

    Ciphertext tmpct;
    bsgs_linear_transform(tmpct, cipher, totlen1, basicstep1, (int)logn + 1, fftcoeff1[slot_index]);
    evaluator.rescale_to_next_inplace(tmpct);
    Ciphertext tmpct2;
    bsgs_linear_transform(tmpct2, tmpct, totlen2, basicstep2, (int)logn + 1, fftcoeff2[slot_index]);
    evaluator.rescale_to_next_inplace(tmpct2);

    const auto &modulus = context.first_context_data()->parms().coeff_modulus();
    const auto curr_level = context.get_context_data(tmpct2.parms_id())->chain_index();
    const double mod_zero = (double)modulus[0].value();
    const double curr_mod = (double)modulus[curr_level].value();
    // fftcoeff3_scale = fftcoeff3 * curr_mod * q0 * final_scale / (2 s^2 initial_scale)
    const double init = initial_scale_slot() != 0 ? initial_scale_slot() : initial_scale;
    const double coeff_scale = curr_mod * mod_zero * final_scale / (2 * tmpct2.scale() * tmpct2.scale() * init);
    bsgs_linear_transform(rtncipher, tmpct2, totlen3, basicstep3, (int)logn + 1, fftcoeff3[slot_index],
                          coeff_scale);
    evaluator.rescale_to_next_inplace(rtncipher);
}

void Bootstrapper::sflinv_3(Ciphertext &rtncipher, Ciphertext &cipher)
{
    // Bootstrapper.cpp:2531-2552
    const int div_part1 = (int)std::floor(logn / 3.0);
    const int div_part2 = (int)std::floor((logn - div_part1) / 2.0);
    const int div_part3 = (int)logn - div_part1 - div_part2;
    const int totlen1 = (1 << div_part1) - 1, totlen2 = (1 << div_part2) - 1, totlen3 = (1 << div_part3) - 1;
    const int basicstep1 = 1 << (logn - div_part1), basicstep2 = 1 << (logn - div_part1 - div_part2),
              basicstep3 = 1;

    Ciphertext tmpct;
    rotated_bsgs_linear_transform(tmpct, cipher, totlen1, basicstep1, (int)logn, invfftcoeff1[slot_index]);
    evaluator.rescale_to_next_inplace(tmpct);
    Ciphertext tmpct2;
    bsgs_linear_transform(tmpct2, tmpct, totlen2, basicstep2, (int)logn, invfftcoeff2[slot_index]);
    evaluator.rescale_to_next_inplace(tmpct2);
    bsgs_linear_transform(rtncipher, tmpct2, totlen3, basicstep3, (int)logn + 1, invfftcoeff3[slot_index]);
    evaluator.rescale_to_next_inplace(rtncipher);
}

void Bootstrapper::sfl_full_half_3(Ciphertext &rtncipher, Ciphertext &cipher)
{
    sfl_full_common(rtncipher, cipher, true);
}

void Bootstrapper::sfl_full_3(Ciphertext &rtncipher, Ciphertext &cipher)
{
    sfl_full_common(rtncipher, cipher, false);
}

void Bootstrapper::sfl_full_common(Ciphertext &rtncipher, Ciphertext &cipher, bool half)
{
    // Bootstrapper.cpp:2422-2458 (sfl_full_3) / 2499-2536 (sfl_full_half_3, the extra 1/2): full
    // slots, the last group rotated (cyclic) and scaled as in sfl_half_3
    const int div_part3 = (int)std::floor(logn / 3.0);
    const int div_part2 = (int)std::floor((logn - div_part3) / 2.0);
    const int div_part1 = (int)logn - div_part3 - div_part2;
    const int totlen1 = (1 << div_part1) - 1, totlen2 = (1 << div_part2) - 1, totlen3 = (1 << div_part3) - 1;
    const int basicstep1 = 1, basicstep2 = 1 << div_part1, basicstep3 = 1 << (div_part1 + div_part2);

    Ciphertext tmpct;
    bsgs_linear_transform(tmpct, cipher, totlen1, basicstep1, (int)logn, fftcoeff1[slot_index]);
    evaluator.rescale_to_next_inplace(tmpct);
    Ciphertext tmpct2;
    bsgs_linear_transform(tmpct2, tmpct, totlen2, basicstep2, (int)logn, fftcoeff2[slot_index]);
    evaluator.rescale_to_next_inplace(tmpct2);

    const auto &modulus = context.first_context_data()->parms().coeff_modulus();
    const auto curr_level = context.get_context_data(tmpct2.parms_id())->chain_index();
    const double mod_zero = (double)modulus[0].value();
    const double curr_mod = (double)modulus[curr_level].value();
    const double init = initial_scale_slot() != 0 ? initial_scale_slot() : initial_scale;
    const double coeff_scale =
        curr_mod * mod_zero * final_scale / ((half ? 2 : 1) * tmpct2.scale() * tmpct2.scale() * init);
    rotated_bsgs_linear_transform(rtncipher, tmpct2, totlen3, basicstep3, (int)logn, fftcoeff3[slot_index],
                                  coeff_scale);
    evaluator.rescale_to_next_inplace(rtncipher);
}

void Bootstrapper::sflinv_full_3(Ciphertext &rtncipher, Ciphertext &cipher)
{
    // Bootstrapper.cpp:2561-2584
    const int div_part1 = (int)std::floor(logn / 3.0);
    const int div_part2 = (int)std::floor((logn - div_part1) / 2.0);
    const int div_part3 = (int)logn - div_part1 - div_part2;
    const int totlen1 = (1 << div_part1) - 1, totlen2 = (1 << div_part2) - 1, totlen3 = (1 << div_part3) - 1;
    const int basicstep1 = 1 << (logn - div_part1), basicstep2 = 1 << (logn - div_part1 - div_part2),
              basicstep3 = 1;

    Ciphertext tmpct;
    rotated_bsgs_linear_transform(tmpct, cipher, totlen1, basicstep1, (int)logn, invfftcoeff1[slot_index]);
    evaluator.rescale_to_next_inplace(tmpct);
    Ciphertext tmpct2;
    bsgs_linear_transform(tmpct2, tmpct, totlen2, basicstep2, (int)logn, invfftcoeff2[slot_index]);
    evaluator.rescale_to_next_inplace(tmpct2);
    bsgs_linear_transform(rtncipher, tmpct2, totlen3, basicstep3, (int)logn, invfftcoeff3[slot_index]);
    evaluator.rescale_to_next_inplace(rtncipher);
}

void Bootstrapper::coefftoslot_full_3(Ciphertext &rtncipher1, Ciphertext &rtncipher2, Ciphertext &cipher)
{
    // Bootstrapper.cpp:2705-2724: the slots of the real and the imaginary part of the coefficients
    // (t + conj t, and (-i t) + conj(-i t)); -i is a scale-1 plaintext, so no rescale
    Ciphertext tmpct1, tmpct2, tmpct3, tmpct4;
    sflinv_full_3(tmpct1, cipher);
    Plaintext minus_i;
    encoder.encode(std::vector<cd>((std::size_t)Nh, cd(0.0, -1.0)), 1.0, minus_i);
    evaluator.mod_switch_to_inplace(minus_i, tmpct1.parms_id());
    evaluator.multiply_plain(tmpct1, minus_i, tmpct2);
    evaluator.complex_conjugate(tmpct2, gal_keys, tmpct3);
    evaluator.complex_conjugate(tmpct1, gal_keys, tmpct4);
    evaluator.add_reduced_error(tmpct1, tmpct4, rtncipher1);
    evaluator.add_reduced_error(tmpct2, tmpct3, rtncipher2);
}

void Bootstrapper::slottocoeff_full_half_3(Ciphertext &rtncipher, Ciphertext &cipher1, Ciphertext &cipher2)
{
    // Bootstrapper.cpp:2744-2760: recombine real + i * imaginary, then SlotToCoeff
    Ciphertext tmpct1, tmpct3;
    Plaintext plus_i;
    encoder.encode(std::vector<cd>((std::size_t)Nh, cd(0.0, 1.0)), 1.0, plus_i);
    evaluator.mod_switch_to_inplace(plus_i, cipher2.parms_id());
    evaluator.multiply_plain(cipher2, plus_i, tmpct1);
    evaluator.add_reduced_error(cipher1, tmpct1, tmpct3);
    sfl_full_half_3(rtncipher, tmpct3);
}

void Bootstrapper::slottocoeff_full_3(Ciphertext &rtncipher, Ciphertext &cipher1, Ciphertext &cipher2)
{
    // Bootstrapper.cpp:2726-2742
    Ciphertext tmpct1, tmpct3;
    Plaintext plus_i;
    encoder.encode(std::vector<cd>((std::size_t)Nh, cd(0.0, 1.0)), 1.0, plus_i);
    evaluator.mod_switch_to_inplace(plus_i, cipher2.parms_id());
    evaluator.multiply_plain(cipher2, plus_i, tmpct1);
    evaluator.add_reduced_error(cipher1, tmpct1, tmpct3);
    sfl_full_3(rtncipher, tmpct3);
}

void Bootstrapper::bootstrap_full_3(Ciphertext &rtncipher, Ciphertext &cipher)
{
    // Bootstrapper.cpp:3155-3176: complex slots
    modraise_inplace(cipher);
    const auto &modulus = context.first_context_data()->parms().coeff_modulus();
    cipher.scale() = (double)modulus[0].value();
    Ciphertext rtn1, rtn2;
    coefftoslot_full_3(rtn1, rtn2, cipher);
    Ciphertext modrtn1, modrtn2;
    mod_reducer->modular_reduction(modrtn1, rtn1);
    mod_reducer->modular_reduction(modrtn2, rtn2);
    slottocoeff_full_3(rtncipher, modrtn1, modrtn2);
    rtncipher.scale() = final_scale;
}

void Bootstrapper::bootstrap_3(Ciphertext &rtncipher, Ciphertext &cipher)
{
    // Bootstrapper.cpp:3421-3425
    initial_scale_slot() = cipher.scale();
    if (logn != logNh) throw std::logic_error("complex sparse-slot bootstrapping is not provided: use bootstrap_real_3");
    bootstrap_full_3(rtncipher, cipher);
}

void Bootstrapper::bootstrap_inplace_3(Ciphertext &cipher)
{
    Ciphertext rtncipher;
    bootstrap_3(rtncipher, cipher);
    cipher = rtncipher;
}

void Bootstrapper::bootstrap_full_real_3(Ciphertext &rtncipher, Ciphertext &cipher)
{
    // Bootstrapper.cpp:3250-3274
    modraise_inplace(cipher);
    const auto &modulus = context.first_context_data()->parms().coeff_modulus();
    cipher.scale() = (double)modulus[0].value();
    Ciphertext rtn1, rtn2;
    coefftoslot_full_3(rtn1, rtn2, cipher);
    Ciphertext modrtn1, modrtn2;
    mod_reducer->modular_reduction(modrtn1, rtn1);
    mod_reducer->modular_reduction(modrtn2, rtn2);
    slottocoeff_full_half_3(rtncipher, modrtn1, modrtn2);
    rtncipher.scale() = final_scale;
    Ciphertext conjct;
    evaluator.complex_conjugate(rtncipher, gal_keys, conjct);
    evaluator.add_inplace_reduced_error(rtncipher, conjct);
}

void Bootstrapper::coefftoslot_3(Ciphertext &rtncipher, Ciphertext &cipher)
{
    // Bootstrapper.cpp:2675-2680
    Ciphertext tmpct1, tmpct2;
    sflinv_3(tmpct1, cipher);
    evaluator.complex_conjugate(tmpct1, gal_keys, tmpct2);
    evaluator.add_reduced_error(tmpct1, tmpct2, rtncipher);
}

void Bootstrapper::slottocoeff_half_3(Ciphertext &rtncipher, Ciphertext &cipher)
{
    // Bootstrapper.cpp:2689-2694
    Ciphertext tmpct1, tmpct2;
    sfl_half_3(tmpct1, cipher);
    evaluator.rotate_vector(tmpct1, (int)n, gal_keys, tmpct2);
    evaluator.add_reduced_error(tmpct1, tmpct2, rtncipher);
}

void Bootstrapper::modraise_inplace(Ciphertext &cipher)
{
    // Bootstrapper.cpp:2894-2948; the centered lift runs on the GPU (mhe_modraise)
    if (cipher.size() != 2) throw std::invalid_argument("Ciphertexts of size 2 are supported only!");
    if (cipher.coeff_modulus_size() != 1)
        throw std::invalid_argument("Ciphertexts in the lowest level are supported only!");
    if (cipher.is_ntt_form()) evaluator.transform_from_ntt_inplace(cipher);
    Ciphertext encrypted_copy(cipher);
    cipher.resize(context, context.first_parms_id(), 2);
    const std::size_t limbs = cipher.coeff_modulus_size();
    void *s = context.stream();
    {
        // the lift is one record of the evaluator trace (tests/trace_replay.py "modraise"), between
        // the traced transform_from_ntt / transform_to_ntt
        seal::trace::Scope tsc;
        const std::string tin = tsc.top() ? seal::trace::ct(encrypted_copy) : std::string();
        const std::uint64_t *src = encrypted_copy.store().dev_read(s);
        std::uint64_t *dst = cipher.store().dev_write(s, true);
        if (mhe_modraise(context.engine(), src, dst, 2, (int)limbs, s) != MHE_OK) throw std::runtime_error(mhe_last_error());
        cipher.is_ntt_form() = false;
        if (tsc.top()) seal::trace::record("modraise", { tin }, seal::trace::ct(cipher));
    }
    evaluator.transform_to_ntt_inplace(cipher);
}

void Bootstrapper::bootstrap_sparse_real_3(Ciphertext &rtncipher, Ciphertext &cipher)
{
    // Bootstrapper.cpp:3166-3236
    modraise_inplace(cipher);
    const auto &modulus = context.first_context_data()->parms().coeff_modulus();
    cipher.scale() = (double)modulus[0].value();

    Ciphertext rot;
    for (long i = logn; i < logNh; ++i)
    {
        evaluator.rotate_vector(cipher, (int)(1L << i), gal_keys, rot);
        evaluator.add_inplace(cipher, rot);
    }

    Ciphertext rtn;
    if (logn == 0)
    {
        std::vector<cd> cts_vec(Nh, 0.0);
        for (long i = 0; i < Nh; i++)
            cts_vec[i] = i % 2 == 0 ? cd(1.0 / (2.0 * boundary_K * (1L << logNh)))
                                    : -cd(0, 1.0) / (2.0 * boundary_K * (1L << logNh));
        evaluator.multiply_vector_reduced_error(cipher, cts_vec, rtn);
        evaluator.rescale_to_next_inplace(rtn);
        Ciphertext conjrtn;
        evaluator.complex_conjugate(rtn, gal_keys, conjrtn);
        evaluator.add_inplace_reduced_error(rtn, conjrtn);
    }
    else
        coefftoslot_3(rtn, cipher);

    Ciphertext modrtn;
    mod_reducer->modular_reduction(modrtn, rtn);

    if (logn == 0)
    {
        const auto curr_level = context.get_context_data(modrtn.parms_id())->chain_index();
        const double mod_zero = (double)modulus[0].value(), curr_mod = (double)modulus[curr_level].value();
        const double init = initial_scale_slot() != 0 ? initial_scale_slot() : initial_scale;
        const double scale_adj = curr_mod * mod_zero * final_scale / (modrtn.scale() * modrtn.scale() * init);
        std::vector<cd> stc_vec(Nh, 0.0);
        for (long i = 0; i < Nh; i++) stc_vec[i] = i % 2 == 0 ? cd(scale_adj) : cd(0, 1.0) * scale_adj;
        evaluator.multiply_vector_reduced_error(modrtn, stc_vec, rtncipher);
        evaluator.rescale_to_next_inplace(rtncipher);
        Ciphertext rotrtncipher;
        evaluator.rotate_vector(rtncipher, 1, gal_keys, rotrtncipher);
        evaluator.add_inplace_reduced_error(rtncipher, rotrtncipher);
    }
    else
        slottocoeff_half_3(rtncipher, modrtn);

    if (const char *v = std::getenv("MHE_BOOT_PT_CHECK"); v && v[0] == '1') verify_cache();
    rtncipher.scale() = final_scale;
    Ciphertext conjct;
    evaluator.complex_conjugate(rtncipher, gal_keys, conjct);
    evaluator.add_inplace_reduced_error(rtncipher, conjct);
}

void Bootstrapper::bootstrap_real_3(Ciphertext &rtncipher, Ciphertext &cipher)
{
    // Bootstrapper.cpp:3421-3425 (initial_scale kept per thread)
    initial_scale_slot() = cipher.scale();
    if (logn == logNh)
        bootstrap_full_real_3(rtncipher, cipher);
    else
        bootstrap_sparse_real_3(rtncipher, cipher);
}

void Bootstrapper::bootstrap_inplace_real_3(Ciphertext &cipher)
{
    Ciphertext rtncipher;
    bootstrap_real_3(rtncipher, cipher);
    cipher = rtncipher;
}
