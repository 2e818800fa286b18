// comp.cpp -- approximate sign / ReLU by minimax composite polynomials (include/mhe_comp.h)
// over the seal:: surface: evaluation-tree search (comp/program.cpp), Chebyshev-basis
// polynomial evaluation (comp/SEALfunc.cpp:33-313) and the ReLU wrapper (comp/SEALcomp.cpp).
// Every ciphertext operation is the reference's, in the reference's order; the host-side
// arithmetic (tree shapes, index bookkeeping) keeps the reference's floating-point expressions
// (e.g. log(i)/log(2)) so the same trees and coefficient slots come out.
#include "mhe_comp.h"

#include <cmath>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <memory>
#include <stdexcept>

#include "mhe_cnn.h" // pow2, log2 helpers

namespace
{
long ceil_to_int(double x)
{
    return static_cast<long>(std::ceil(x) + 0.5); // common/MinicompFunc.cpp:28-31
}

// 2^floor(log2 i) exactly as the reference computes it (PolyUpdate.cpp:43,48,132,137)
int msb_pow(int i)
{
    return static_cast<int>(pow2(static_cast<int>(std::log(static_cast<double>(i)) / std::log(2.0))));
}
} // namespace

namespace minicomp
{
void Tree::clear()
{
    depth = 0;
    type = evaltype::none;
    tree.assign({ -1, 0 });
}

void Tree::merge(const Tree &a, const Tree &b, int g)
{
    // PolyUpdate.cpp:119-140: root g, a's nodes under child 2, b's under child 3.  a and b are
    // copied first because the result may alias one of them.
    if (a.type != b.type) throw std::invalid_argument("the types of two trees are not the same");
    const Tree A = a, B = b;
    clear();
    type = A.type;
    depth = std::max(A.depth, B.depth) + 1;
    tree.assign(static_cast<size_t>(pow2(depth + 1)), -1);
    tree[1] = g;
    for (int i = 1; i <= pow2(A.depth + 1) - 1; i++) tree[i + msb_pow(i)] = A.tree[i];
    for (int i = 1; i <= pow2(B.depth + 1) - 1; i++) tree[i + 2 * msb_pow(i)] = B.tree[i];
}

void Tree::print() const
{
    std::cout << "depth of tree: " << depth << std::endl;
    for (int i = 0; i <= depth; i++)
    {
        for (int j = (int)pow2(i); j < pow2(i + 1); j++) std::cout << tree[j] << " ";
        std::cout << std::endl;
    }
    std::cout << "m: " << m << "\nl: " << l << "\nb: " << b << std::endl;
}

long num_one(long n)
{
    long c = 0;
    for (; n > 0; n >>= 1) c += n & 1;
    return c;
}

// per node: degree of the (sub)polynomial it evaluates (SEALfunc.cpp:76-86, 326-335)
static std::vector<long> node_degrees(long deg, const Tree &tree)
{
    std::vector<long> d(static_cast<size_t>(pow2(tree.depth + 1)), -1);
    d[1] = deg;
    for (int i = 1; i <= tree.depth; i++)
        for (int j = (int)pow2(i); j < pow2(i + 1); j++)
            d[j] = (j % 2 == 0) ? tree.tree[j / 2] - 1 : d[j / 2] - tree.tree[j / 2];
    return d;
}

long coeff_number(long deg, Tree &tree)
{
    // SEALfunc.cpp:320-346: leaves hold decomp_deg+1 coefficients each
    const std::vector<long> d = node_degrees(deg, tree);
    long num = 0;
    for (size_t i = 0; i < d.size(); i++)
        if (tree.tree[i] == 0) num += d[i] + 1;
    return num;
}
} // namespace minicomp

// ------------------------------------------------------------------------ tree search
void upgrade_oddbaby(long n, Tree &tree)
{
    // comp/program.cpp:3-56.  f[i][j]: non-scalar multiplications to evaluate an odd degree-i
    // polynomial at depth j given T_1..T_{2^l-1} and T_{2^k}, k < m; split at g = 2^k.
    const long d = ceil_to_int(std::log(static_cast<double>(n)) / std::log(2.0));
    long total_min = 10000, min_m = 0, min_l = 0;
    Tree best;
    for (long l = 1; pow2(l) - 1 <= n; l++)
        for (long m = 1; pow2(m - 1) < n; m++)
        {
            std::vector<std::vector<int>> f(n + 1, std::vector<int>(d + 1, 0));
            std::vector<std::vector<Tree>> G(n + 1, std::vector<Tree>(d + 1, Tree(evaltype::oddbaby)));
            f[1][1] = 0;
            for (long i = 3; i <= n; i += 2) f[i][1] = 10000;
            for (long j = 2; j <= d; j++)
                for (long i = 1; i <= n; i += 2)
                {
                    if (i <= pow2(l) - 1 && i <= pow2(j - 1))
                    {
                        f[i][j] = 0;
                        continue;
                    }
                    int best_f = 10000;
                    Tree t;
                    for (long k = 1; k <= m - 1 && pow2(k) < i && k < j; k++)
                    {
                        const long g = pow2(k);
                        const int cand = f[i - g][j - 1] + f[g - 1][j] + 1;
                        if (cand < best_f)
                        {
                            best_f = cand;
                            t.merge(G[g - 1][j], G[i - g][j - 1], (int)g);
                        }
                    }
                    f[i][j] = best_f;
                    G[i][j] = t;
                }
            if (f[n][d] + pow2(l - 1) + m - 2 < total_min)
            {
                total_min = f[n][d] + pow2(l - 1) + m - 2;
                best = G[n][d];
                min_m = m;
                min_l = l;
            }
        }
    tree = best;
    tree.m = (int)min_m;
    tree.l = (int)min_l;
}

void upgrade_baby(long n, Tree &tree)
{
    // comp/program.cpp:57-157: baby-step giant-step with T_2..T_b and T_{2^k b}
    const long d = ceil_to_int(std::log(static_cast<double>(n + 1)) / std::log(2.0));
    long total_min = 10000, min_m = 0, min_b = 0;
    Tree best;
    const evaltype type = evaltype::baby;
    if (n == 1)
    {
        total_min = 0;
        best = Tree(type);
        min_m = 1;
        min_b = 1;
    }
    for (long b = 1; b <= n; b++)
        for (long m = 1; pow2(m - 1) * b <= n; m++)
        {
            std::vector<std::vector<int>> f(n + 1, std::vector<int>(d + 1, 0));
            std::vector<std::vector<Tree>> G(n + 1, std::vector<Tree>(d + 1, Tree(type)));
            for (long j = 1; j <= d; j++)
                for (long i = 1; i <= n; i++)
                {
                    if (i + 1 > pow2(j))
                    {
                        f[i][j] = 10000;
                        G[i][j] = Tree(type);
                        continue;
                    }
                    if ((b == 1 && m >= 2 && i <= 2 && i <= pow2(j - 1)) || (i <= b && i <= pow2(j - 1)))
                    {
                        f[i][j] = 0;
                        G[i][j] = Tree(type);
                        continue;
                    }
                    int best_f = 10000;
                    Tree t;
                    auto consider = [&](long g) {
                        if (g <= pow2(j - 1) && 2 <= g && g < i && f[i - g][j - 1] + f[g - 1][j] + 1 < best_f)
                        {
                            best_f = f[i - g][j - 1] + f[g - 1][j] + 1;
                            t.merge(G[g - 1][j], G[i - g][j - 1], (int)g);
                        }
                    };
                    for (long k = 2; k <= b; k++) consider(k);
                    for (long k = 0; k <= m - 1; k++) consider(pow2(k) * b);
                    f[i][j] = best_f;
                    G[i][j] = t;
                }
            if (f[n][d] + m + b - 2 < total_min)
            {
                total_min = f[n][d] + m + b - 2;
                best = G[n][d];
                min_m = m;
                min_b = b;
            }
        }
    tree = best;
    tree.m = (int)min_m;
    tree.b = (int)min_b;
}

// ------------------------------------------------------------------------ evaluation
namespace seal
{
namespace
{
// T_{m+n} = 2 T_m T_n - T_{|m-n|} (SEALfunc.cpp:52-59)
void evalT(Evaluator &evaluator, RelinKeys &relin_keys, Ciphertext &Tmplusn, const Ciphertext &Tm,
           const Ciphertext &Tn, const Ciphertext &Tmminusn)
{
    Ciphertext temp;
    evaluator.multiply_reduced_error(Tm, Tn, relin_keys, temp);
    evaluator.add_inplace_reduced_error(temp, temp);
    evaluator.rescale_to_next_inplace(temp);
    evaluator.sub_reduced_error(temp, Tmminusn, Tmplusn);
}
} // namespace

void eval_polynomial_integrate(Encryptor &encryptor, Evaluator &evaluator, Decryptor &, CKKSEncoder &encoder,
                               PublicKey &, SecretKey &, RelinKeys &relin_keys, Ciphertext &res, Ciphertext &cipher,
                               long deg, const std::vector<double> &decomp_coeff, Tree &tree)
{
    // SEALfunc.cpp:60-313
    const double scale = cipher.scale();
    const long n = static_cast<long>(cipher.poly_modulus_degree() / 2);
    const long total_depth = ceil_to_int(std::log(static_cast<double>(deg + 1)) / std::log(2.0));
    const long nodes = pow2(tree.depth + 1);
    const std::vector<long> ddeg = minicomp::node_degrees(deg, tree);
    std::vector<long> start_index(static_cast<size_t>(nodes), -1);
    std::vector<std::unique_ptr<Ciphertext>> T(100), pt(100);
    Ciphertext temp1, ctxt_zero;

    // Enc(0) at scale^2 (lazy scaling) for the baby variant
    {
        Plaintext plain_zero;
        encoder.encode(std::vector<double>(n, 0.0), scale * scale, plain_zero);
        encryptor.encrypt(plain_zero, ctxt_zero);
    }
    long temp_index = tree.type == evaltype::oddbaby ? 1 : 0;
    for (long i = 1; i < nodes; i++)
        if (tree.tree[i] == 0)
        {
            start_index[i] = temp_index;
            temp_index += ddeg[i] + 1;
        }

    // T0 = Enc(1) at the input scale, T1 = x (SEALfunc.cpp:33-50)
    T[0] = std::make_unique<Ciphertext>();
    T[1] = std::make_unique<Ciphertext>(cipher);
    {
        Plaintext plain_1;
        encoder.encode(std::vector<double>(n, 1.0), scale, plain_1);
        encryptor.encrypt(plain_1, *T[0]);
    }
    auto need = [](const std::unique_ptr<Ciphertext> &p, const char *what) -> Ciphertext & {
        if (!p) throw std::runtime_error(std::string(what) + " is not set");
        return *p;
    };

    if (tree.type == evaltype::oddbaby)
    {
        // The reference's operation sequence per node, with the independent work of one depth
        // issued together: the leaves' rescales as one batch, and every product of the depth (the
        // internal nodes' spines, the giant step and the odd baby steps, all relinearized with one
        // key) as one multiply_reduced_error_many, then their rescales as one batch.  Each
        // ciphertext sees the same operations in the same order as in SEALfunc.cpp:60-313, so the
        // words are the same; only the launches are shared.
        for (long i = 1; i <= total_depth; i++)
        {
            // leaves finishing at depth i: odd polynomials in T_1, T_3, ...
            std::vector<Ciphertext *> resc;
            for (long j = 1; j < nodes; j++)
            {
                if (tree.tree[j] != 0 || total_depth + 1 - minicomp::num_one(j) != i) continue;
                long idx = start_index[j];
                pt[j] = std::make_unique<Ciphertext>();
                evaluator.multiply_const(need(T[1], "T[1]"), decomp_coeff[idx], *pt[j]);
                idx += 2;
                for (long k = 3; k <= ddeg[j]; k += 2)
                {
                    evaluator.multiply_const(need(T[k], "T[k]"), decomp_coeff[idx], temp1);
                    evaluator.add_inplace_reduced_error(*pt[j], temp1);
                    idx += 2;
                }
                resc.push_back(pt[j].get());
            }
            evaluator.rescale_to_next_inplace_many(resc);

            // every product of this depth
            std::vector<const Ciphertext *> m1, m2;
            std::vector<Ciphertext *> mo;
            std::vector<std::unique_ptr<Ciphertext>> extra; // spine products after a node's first
            struct Spine
            {
                long j, kend;
                std::vector<Ciphertext *> terms;
            };
            std::vector<Spine> spines;
            // internal nodes finishing at depth i (odd index: the start of a right spine)
            for (long j = 1; j < nodes; j++)
            {
                if (tree.tree[j] <= 0 || total_depth + 1 - minicomp::num_one(j) != i || j % 2 != 1) continue;
                Spine sp{ j, j, {} };
                long k = j;
                pt[j] = std::make_unique<Ciphertext>();
                m1.push_back(&need(T[tree.tree[k]], "T[tree.tree[k]]"));
                m2.push_back(&need(pt[2 * k + 1], "pt"));
                mo.push_back(pt[j].get());
                k *= 2;
                while (tree.tree[k] != 0)
                {
                    extra.push_back(std::make_unique<Ciphertext>());
                    m1.push_back(&need(T[tree.tree[k]], "T[tree.tree[k]]"));
                    m2.push_back(&need(pt[2 * k + 1], "pt"));
                    mo.push_back(extra.back().get());
                    sp.terms.push_back(extra.back().get());
                    k *= 2;
                }
                sp.kend = k;
                spines.push_back(std::move(sp));
            }
            // giant step T_{2^i} and odd baby steps T_j, 2^{i-1} < j < 2^i (evalT: T_{m+n} =
            // 2 T_m T_n - T_{|m-n|})
            struct Step
            {
                long g;
                const Ciphertext *minus;
                std::unique_ptr<Ciphertext> prod;
            };
            std::vector<Step> steps;
            auto add_step = [&](long g, long m, long nn, long mn) {
                Step st{ g, &need(T[mn], "T"), std::make_unique<Ciphertext>() };
                m1.push_back(&need(T[m], "T"));
                m2.push_back(&need(T[nn], "T"));
                mo.push_back(st.prod.get());
                steps.push_back(std::move(st));
            };
            if (i <= tree.m - 1) add_step(pow2(i), pow2(i - 1), pow2(i - 1), 0);
            if (i <= tree.l)
                for (long j = pow2(i - 1) + 1; j <= pow2(i) - 1; j += 2) add_step(j, pow2(i - 1), j - pow2(i - 1), pow2(i) - j);
            evaluator.multiply_reduced_error_many(m1, m2, relin_keys, mo);

            resc.clear();
            for (Spine &sp : spines)
            {
                for (Ciphertext *t : sp.terms) evaluator.add_inplace_reduced_error(*pt[sp.j], *t);
                resc.push_back(pt[sp.j].get());
            }
            for (Step &st : steps)
            {
                evaluator.add_inplace_reduced_error(*st.prod, *st.prod);
                resc.push_back(st.prod.get());
            }
            evaluator.rescale_to_next_inplace_many(resc);
            for (Spine &sp : spines) evaluator.add_inplace_reduced_error(*pt[sp.j], need(pt[sp.kend], "pt[k]"));
            for (Step &st : steps)
            {
                T[st.g] = std::make_unique<Ciphertext>();
                evaluator.sub_reduced_error(*st.prod, *st.minus, *T[st.g]);
            }
        }
        res = std::move(need(pt[1], "pt[1]"));
        return;
    }

    if (tree.type != evaltype::baby) throw std::invalid_argument("unsupported evaluation type");
    for (long i = 1; i <= total_depth; i++)
    {
        for (long j = 1; j < nodes; j++)
        {
            if (tree.tree[j] != 0 || total_depth + 1 - minicomp::num_one(j) != i) continue;
            long idx = start_index[j];
            pt[j] = std::make_unique<Ciphertext>(ctxt_zero);
            for (long k = 0; k <= ddeg[j]; k++, idx++)
            {
                if (std::fabs(decomp_coeff[idx]) <= 1.0 / scale) continue; // avoid transparent ciphertexts
                evaluator.multiply_const(need(T[k], "T[k]"), decomp_coeff[idx], temp1);
                evaluator.add_inplace(*pt[j], temp1);
            }
            evaluator.rescale_to_next_inplace(*pt[j]);
        }
        std::vector<long> inter;
        for (long j = 1; j < nodes; j++)
        {
            if (tree.tree[j] <= 0 || total_depth + 1 - minicomp::num_one(j) != i) continue;
            // skip nodes on the left spine of an internal node already evaluated this stage
            bool covered = false;
            for (long s : inter)
            {
                long tmp = j;
                while (true)
                {
                    if (tmp == s)
                    {
                        covered = true;
                        break;
                    }
                    if (tmp % 2 == 0)
                        tmp /= 2;
                    else
                        break;
                }
            }
            if (covered) continue;
            inter.push_back(j);
            long k = j;
            pt[j] = std::make_unique<Ciphertext>();
            evaluator.multiply_reduced_error(need(T[tree.tree[k]], "T[tree.tree[k]]"), need(pt[2 * k + 1], "pt"),
                                             relin_keys, *pt[j]);
            k *= 2;
            while (tree.tree[k] != 0)
            {
                evaluator.multiply_reduced_error(need(T[tree.tree[k]], "T[tree.tree[k]]"), need(pt[2 * k + 1], "pt"),
                                                 relin_keys, temp1);
                evaluator.add_inplace(*pt[j], temp1);
                k *= 2;
            }
            evaluator.rescale_to_next_inplace(*pt[j]);
            evaluator.add_inplace_reduced_error(*pt[j], need(pt[k], "pt[k]"));
        }
        auto make_T = [&](long g) {
            T[g] = std::make_unique<Ciphertext>();
            if (g % 2 == 0)
                evalT(evaluator, relin_keys, *T[g], need(T[g / 2], "T[g/2]"), need(T[g / 2], "T[g/2]"),
                      need(T[0], "T[0]"));
            else
                evalT(evaluator, relin_keys, *T[g], need(T[g / 2], "T[g/2]"), need(T[(g + 1) / 2], "T[(g+1)/2]"),
                      need(T[1], "T[1]"));
        };
        for (long j = 2; j <= tree.b; j++)
            if (pow2(i - 1) < j && j <= pow2(i)) make_T(j);
        for (long j = 1; j <= tree.m - 1; j++)
        {
            const long g = pow2(j) * tree.b;
            if (pow2(i - 1) < g && g <= pow2(i)) make_T(g);
        }
    }
    res = need(pt[1], "pt[1]");
}
} // namespace seal

// ------------------------------------------------------------------------ ReLU
void minimax_ReLU_seal(long comp_no, std::vector<int> deg, long alpha, std::vector<Tree> &tree, double scaled_val,
                       long, seal::Encryptor &encryptor, seal::Evaluator &evaluator, seal::Decryptor &decryptor,
                       seal::CKKSEncoder &encoder, seal::PublicKey &public_key, seal::SecretKey &secret_key,
                       seal::RelinKeys &relin_keys, seal::Ciphertext &cipher_in, seal::Ciphertext &cipher_res)
{
    // SEALcomp.cpp:3-60: sgn(x)/2 by the composite polynomial, then x (1 + sgn x)/2
    using namespace seal;
    const char *dir = std::getenv("MHE_COMP_DIR");
    const std::string path = std::string(dir ? dir : "../result") + "/d" + std::to_string(alpha) + ".txt";
    std::ifstream in(path);
    if (!in) throw std::runtime_error("cannot open " + path);
    std::vector<std::vector<double>> coeff(comp_no);
    for (long i = 0; i < comp_no; i++)
        for (long j = 0; j < minicomp::coeff_number(deg[i], tree[i]); j++)
        {
            double c;
            if (!(in >> c)) throw std::runtime_error("too few coefficients in " + path);
            coeff[i].push_back(c);
        }
    // component i feeds component i+1 at scale 1/scale_val[i+1]; the last one yields sgn/2
    std::vector<double> scale_val(comp_no, 2.0);
    scale_val[0] = 1.0;
    scale_val[comp_no - 1] = scaled_val;
    for (long i = 0; i + 1 < comp_no; i++)
        for (double &c : coeff[i]) c /= scale_val[i + 1];
    for (double &c : coeff[comp_no - 1]) c *= 0.5;

    Ciphertext cipher_x = cipher_in, cipher_half, cipher_temp;
    for (long i = 0; i < comp_no; i++)
        eval_polynomial_integrate(encryptor, evaluator, decryptor, encoder, public_key, secret_key, relin_keys,
                                  cipher_x, cipher_x, deg[i], coeff[i], tree[i]);
    const long n = static_cast<long>(cipher_in.poly_modulus_degree() / 2);
    Plaintext plain_half;
    encoder.encode(std::vector<double>(n, 0.5), cipher_x.scale(), plain_half);
    encryptor.encrypt(plain_half, cipher_half);
    evaluator.add_reduced_error(cipher_x, cipher_half, cipher_temp);
    evaluator.multiply_reduced_error(cipher_temp, cipher_in, relin_keys, cipher_res);
    evaluator.rescale_to_next_inplace(cipher_res);
}

// ------------------------------------------------------------------------ plain restatement
// minimax_ReLU_seal on plain doubles, for checking decrypted results: the same d<alpha>.txt
// coefficients, the same scalings between the components and the same odd baby-step giant-step
// trees, evaluated as eval_polynomial_integrate's oddbaby branch does (SEALfunc.cpp:60-313) -- the
// leaves in T_1, T_3, ..., the right spines, T_{2^i} = 2 T_{2^(i-1)}^2 - T_0 and the odd baby steps
// T_j = 2 T_{2^(i-1)} T_{j-2^(i-1)} - T_{2^i-j} -- on one value.  So a decrypted network and its
// plain twin differ by the encryption's error (noise, rescaling, bootstrapping) only, not by the
// polynomial's distance from the exact ReLU.
MinimaxReluPlain::MinimaxReluPlain(long comp_no, std::vector<int> deg, long alpha, std::vector<Tree> tree,
                                   double scaled_val)
    : comp_no_(comp_no), deg_(std::move(deg)), tree_(std::move(tree))
{
    const char *dir = std::getenv("MHE_COMP_DIR");
    const std::string path = std::string(dir ? dir : "../result") + "/d" + std::to_string(alpha) + ".txt";
    std::ifstream in(path);
    if (!in) throw std::runtime_error("cannot open " + path);
    coeff_.assign(comp_no, {});
    for (long i = 0; i < comp_no; i++)
    {
        if (tree_[i].type != evaltype::oddbaby) throw std::invalid_argument("MinimaxReluPlain: oddbaby trees only");
        for (long j = 0; j < minicomp::coeff_number(deg_[i], tree_[i]); j++)
        {
            double c;
            if (!(in >> c)) throw std::runtime_error("too few coefficients in " + path);
            coeff_[i].push_back(c);
        }
    }
    // the scalings of minimax_ReLU_seal
    std::vector<double> scale_val(comp_no, 2.0);
    scale_val[0] = 1.0;
    scale_val[comp_no - 1] = scaled_val;
    for (long i = 0; i + 1 < comp_no; i++)
        for (double &c : coeff_[i]) c /= scale_val[i + 1];
    for (double &c : coeff_[comp_no - 1]) c *= 0.5;
}

double MinimaxReluPlain::eval_component(long c, double x) const
{
    const Tree &tree = tree_[c];
    const long deg = deg_[c];
    const std::vector<double> &dc = coeff_[c];
    const long total_depth = ceil_to_int(std::log(static_cast<double>(deg + 1)) / std::log(2.0));
    const long nodes = pow2(tree.depth + 1);
    const std::vector<long> ddeg = minicomp::node_degrees(deg, tree);
    std::vector<long> start_index(static_cast<size_t>(nodes), -1);
    long temp_index = 1;
    for (long i = 1; i < nodes; i++)
        if (tree.tree[i] == 0)
        {
            start_index[i] = temp_index;
            temp_index += ddeg[i] + 1;
        }
    std::vector<double> T(1024, std::nan("")), pt(static_cast<size_t>(nodes), std::nan(""));
    T[0] = 1.0;
    T[1] = x;
    for (long i = 1; i <= total_depth; i++)
    {
        for (long j = 1; j < nodes; j++)
        {
            if (tree.tree[j] != 0 || total_depth + 1 - minicomp::num_one(j) != i) continue;
            long idx = start_index[j];
            double v = T[1] * dc[idx];
            idx += 2;
            for (long k = 3; k <= ddeg[j]; k += 2, idx += 2) v += T[k] * dc[idx];
            pt[j] = v;
        }
        std::vector<std::pair<long, double>> next_T;
        for (long j = 1; j < nodes; j++)
        {
            if (tree.tree[j] <= 0 || total_depth + 1 - minicomp::num_one(j) != i || j % 2 != 1) continue;
            long k = j;
            double v = T[tree.tree[k]] * pt[2 * k + 1];
            k *= 2;
            while (tree.tree[k] != 0)
            {
                v += T[tree.tree[k]] * pt[2 * k + 1];
                k *= 2;
            }
            pt[j] = v + pt[k];
        }
        if (i <= tree.m - 1) next_T.push_back({ pow2(i), 2.0 * T[pow2(i - 1)] * T[pow2(i - 1)] - T[0] });
        if (i <= tree.l)
            for (long j = pow2(i - 1) + 1; j <= pow2(i) - 1; j += 2)
                next_T.push_back({ j, 2.0 * T[pow2(i - 1)] * T[j - pow2(i - 1)] - T[pow2(i) - j] });
        for (auto &g : next_T) T[g.first] = g.second;
    }
    if (std::isnan(pt[1])) throw std::runtime_error("MinimaxReluPlain: tree left the root unset");
    return pt[1];
}

double MinimaxReluPlain::operator()(double u) const
{
    double x = u;
    for (long i = 0; i < comp_no_; i++) x = eval_component(i, x);
    return (x + 0.5) * u; // x is sgn(u)/2
}
