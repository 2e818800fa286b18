// Hoisted rotations: several rotations of one ciphertext share one ModUp, bit-exact with SEAL's
// one-at-a-time switch_key_inplace (evaluator.cpp:2193-2214 + 2345-2525).
//
// A rotation by Galois element g permutes the NTT slots of c0 and c1 (out[k] = in[pi(k)],
// util/galois.cpp:18-51) and key-switches the permuted c1.  In coefficient form the permuted digit
// J is a signed permutation of the unrotated digit a_J: coefficient a_k moves to position
// t = k g mod 2N, negated (q_J - a_k) when t >= N.  SEAL lifts that canonical residue to every
// output prime I and NTTs it.  Lifting first and permuting after gives the same slots except at the
// negated positions, where (q_J - a_k) mod p_I differs from -(a_k mod p_I) by (q_J mod p_I):
//     D^g_{I,J}[k] = D_{I,J}[pi(k)] + (q_J mod p_I) * M^g_I[k]      (every a_k != 0, k >= 1)
// with D_{I,J} = NTT_{p_I}(a_J mod p_I) the ModUp of the UNROTATED c1 (computed once for all the
// rotations) and M^g_I = NTT_{p_I}(negation mask of g), a table per Galois element and prime.
// Digit I of output prime I is the permuted input limb itself (q_I mod p_I = 0), as in SEAL.
// The identity fails only where a_k = 0 at a negated position (SEAL keeps 0, not q_J): a scan of
// the digits flags such inputs on the device, and their rotations take the classic path in the
// same launch sequence (kernels that return at once when their flag says so), so no host sync.
#pragma once

// A hoisted key-MAC launch: item z = blockIdx.z is one input (its D, c1 and flag) with up to
// MHE_HOIST_R of its rotations (key, Galois element, mask table, output key products each).
#define MHE_HOIST_R 8
struct HoistPtrs
{
    const u64 *D[MHE_MAXB];    // [L+1][L][n] ModUp of the unrotated c1, canonical, NTT form, brev8 blocks ((I, I) unused)
    const u64 *c1[MHE_MAXB];   // [L][n] the unrotated c1, NTT form
    const int *flag[MHE_MAXB]; // != 0: the input has a zero coefficient, the classic path runs its rotations
    int R[MHE_MAXB];           // rotations of the item
    const u64 *key[MHE_MAXB][MHE_HOIST_R];  // [digits][2][key_limbs][n] (SEAL layout or prepared, ntt.h load_key)
    const u64 *mask[MHE_MAXB][MHE_HOIST_R]; // [K][n] M^g: NTT of the rotation's negation mask, canonical, by prime index
    u64 *acc[MHE_MAXB][MHE_HOIST_R];        // [2][L+1][n] key inner products
    u32 einv[MHE_MAXB][MHE_HOIST_R];        // g^-1 mod 2N: slot k of the rotation reads D at m iff k = pi_{g^-1}(m)
    int key_limbs[MHE_MAXB][MHE_HOIST_R];
};

// D keeps the 256 slots of each 256-aligned block in bit-reversed order: slot m at position
// (m & ~255) | brev8(m & 255).  In that order the Galois permutation inside a block is affine,
// u -> (g u + H) mod 256 (H fixed per block), so lanes reading consecutive positions of one block
// hit LDS / memory positions an odd stride apart -- no bank conflicts (hoisted MACs below).
__device__ __forceinline__ u32 brev8(u32 x)
{
    return __builtin_bitreverse32(x) >> 24;
}

// Slot read by output slot k of a rotation by g in NTT form (util/galois.cpp:18-51).
__device__ __forceinline__ u32 galois_src(u32 k, u32 elt, int log_n)
{
    const u32 n = 1u << log_n;
    const u32 reversed = __builtin_bitreverse32(n + k) >> (31 - log_n); // rev over log_n + 1 bits
    const u32 idx = (u32)(((u64)elt * reversed) >> 1) & (n - 1);
    return __builtin_bitreverse32(idx) >> (32 - log_n);
}

// acc_r[k][I] = sum_J D^g_{I,J}[k] * key_r[J][k][I] for output prime I = blockIdx.y and every
// rotation r of item z = blockIdx.z, over a tile of 256 * HE slots m of D (HE per lane, lanes
// consecutive).  Each D word is read once (coalesced) for all the item's rotations: rotation r
// uses it at its output slot k = pi_{g_r^-1}(m) (pi_g^-1 = pi_{g^-1}), and that slot's key words,
// mask word and key products are read / written there -- inside one 256-slot row, since pi maps
// rows to rows.  FP64 arithmetic (every prime below 2^51); cm[J * K + pi] = (q_J mod p, (q_J mod p) / p).
// R (the item's rotation count) is a template parameter so the digit loop is straight-line code: all
// 2R key words and the D word of digit J + 1 are in flight while digit J's products run.  Used when
// the items of a launch rotate by different keys; k_ks_hoist_mac_sh below when they share them.
template <int R>
__global__ __launch_bounds__(256, (R <= 4) ? 4 : 2) void k_ks_hoist_mac(HoistPtrs P, const PrimeDev *__restrict__ primes,
                                                         const TwF *__restrict__ cm, int L, int K, int log_n)
{
    const u32 bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    if (*P.flag[bz]) return; // uniform: the classic path computes this item's rotations
    const size_t n = (size_t)1 << log_n;
    const int I = (int)by;
    const int pi = (I == L) ? K - 1 : I;
    const PrimeDev p = primes[pi];
    const double q = (double)p.q, qinv = 1.0 / q;
    const u64 *__restrict__ D = P.D[bz] + (size_t)I * L * n;
    const u64 *__restrict__ c1 = P.c1[bz];
    const u32 u = threadIdx.x, m = bx * 256u + brev8(u); // D position bx 256 + u holds slot m
    u32 k[R];
    double mk[R], a0[R], a1[R];
    // key limb slot of rotation r for this output prime (uniform; recomputed from the kernel
    // arguments where used, so no VGPRs hold the key pointers)
    auto kslot = [&](int r) {
        const int kl = P.key_limbs[bz][r];
        return P.key[bz][r] + (size_t)((I == L) ? kl - 1 : I) * n;
    };
    // bit r: rotation r's key slot for this prime holds doubles (kdm) / 48-bit planes (k48)
    u32 kdm = 0, k48 = 0;
#pragma unroll
    for (int r = 0; r < R; r++)
    {
        const int f = key_slot_format(kslot(r)[n - 1]);
        kdm |= (f == 1 ? 1u : 0u) << r;
        k48 |= (f == 2 ? 1u : 0u) << r;
        k[r] = galois_src(m, P.einv[bz][r], log_n);
        mk[r] = fp_from_u52(P.mask[bz][r][(size_t)pi * n + k[r]]);
        a0[r] = a1[r] = 0.0;
    }
    // the same load instructions every digit (KP: every key's slot SEAL's layout 0 / doubles 1 /
    // 48-bit planes 2, or -1 per key), so the compiler counts the waits of the one-digit-ahead
    // prefetch instead of draining it
    auto load = [&](int J, u64 &dv, u64 (&w0)[R], u64 (&w1)[R], auto kp_tag) {
        constexpr int KP = decltype(kp_tag)::value;
        dv = (J == I) ? c1[(size_t)J * n + m] : D[(size_t)J * n + bx * 256u + u];
#pragma unroll
        for (int r = 0; r < R; r++)
        {
            const size_t ks = (size_t)P.key_limbs[bz][r] * n;
            const u64 *k0 = kslot(r) + (size_t)(2 * J) * ks;
            const u64 *k1 = k0 + ks;
            if (KP == 2 || (KP == -1 && ((k48 >> r) & 1)))
            {
                const u32 *l0 = reinterpret_cast<const u32 *>(k0), *l1 = reinterpret_cast<const u32 *>(k1);
                w0[r] = (u64)l0[k[r]] | ((u64)reinterpret_cast<const unsigned short *>(l0 + n)[k[r]] << 32);
                w1[r] = (u64)l1[k[r]] | ((u64)reinterpret_cast<const unsigned short *>(l1 + n)[k[r]] << 32);
            }
            else
            {
                w0[r] = k0[k[r]];
                w1[r] = k1[k[r]];
            }
        }
    };
    // a key word as a double
    auto kw = [&](u64 w, int r, auto kp_tag) {
        constexpr int KP = decltype(kp_tag)::value;
        if (KP == 1 || (KP == -1 && ((kdm >> r) & 1))) return key_word_f(w);
        return fp_from_u52(w);
    };
    // lazy sums while L products (|.| < 1.25p each) add up exactly, else a reduction every second digit
    const bool lz = p.q < (1ull << 47) && (double)L * 1.25 * q < 9007199254740992.0;
    auto run = [&](auto kp_tag) {
    u64 dv, w0[R], w1[R];
    load(0, dv, w0, w1, kp_tag);
    for (int J = 0; J < L; J++)
    {
        u64 ndv = 0, nw0[R], nw1[R];
        load(J + 1 < L ? J + 1 : J, ndv, nw0, nw1, kp_tag); // the last digit again at the end
        const double dd = fp_from_u52(dv);
        const TwF c = cm[(size_t)J * K + pi]; // (q_J mod p, / p); (0, 0) for J == I
#pragma unroll
        for (int r = 0; r < R; r++)
        {
            // canonical D (< p) + c M (|.| < 1.5p): |.| < 2.5p < 2^53, centred by one reduction
            const double d = fp_reduce(dd + fp_mulmod(mk[r], c.x, c.y, q), q, qinv);
            a0[r] += fp_mulmod_gen(d, kw(w0[r], r, kp_tag), q, qinv);
            a1[r] += fp_mulmod_gen(d, kw(w1[r], r, kp_tag), q, qinv);
            if (!lz && (J & 1))
            {
                a0[r] = fp_reduce(a0[r], q, qinv);
                a1[r] = fp_reduce(a1[r], q, qinv);
            }
        }
        dv = ndv;
#pragma unroll
        for (int r = 0; r < R; r++)
        {
            w0[r] = nw0[r];
            w1[r] = nw1[r];
        }
    }
    };
    const u32 all = (1u << R) - 1;
    if (kdm == all)
        run(std::integral_constant<int, 1>{});
    else if (k48 == all)
        run(std::integral_constant<int, 2>{});
    else if ((kdm | k48) == 0)
        run(std::integral_constant<int, 0>{});
    else
        run(std::integral_constant<int, -1>{});
#pragma unroll
    for (int r = 0; r < R; r++)
    {
        u64 *o0 = P.acc[bz][r] + (size_t)I * n;
        u64 *o1 = o0 + (size_t)(L + 1) * n;
        o0[k[r]] = fp_canon(a0[r], q, qinv);
        o1[k[r]] = fp_canon(a1[r], q, qinv);
    }
}

// The items of a launch all rotate by the same R keys (the images of a FiberBatch at one BSGS step).
// One 1024-lane workgroup per (256-slot row of D, output prime I) computes every item's rotations:
// per digit J the 2R key rows the row's slots map to (rotation r: row rho_r^-1, the same for every
// slot of the row) are read once, coalesced, into LDS as doubles, and every item's lanes gather
// them there -- the key words cross HBM / L2 once for all the items, not once per item, and no
// lane issues scattered global loads (the per-item kernel spent 9.2 ms at 8 x 7 rotations, 31 limbs,
// 67% of its wave cycles waiting on them).  The mask term is folded out of the digit loop:
//     sum_J (D_J[pi(k)] + c_J M[k]) key_J[k] = sum_J D_J[pi(k)] key_J[k] + M[k] sum_J c_J key_J[k]
// with KC[k] = sum_J c_J key_J[k] accumulated by the lanes that stage the key words.  Lane group
// g = tid / 256 holds IPL items (2 for R <= 4, else 1: the accumulators of 2 x 8 rotations spill at
// 128 VGPRs); blockIdx.z picks the block of 4 IPL items.
struct HoistShared
{
    const u64 *D[MHE_MAXB];
    const u64 *c1[MHE_MAXB];
    const int *flag[MHE_MAXB];
    u64 *acc[MHE_MAXB][MHE_HOIST_R];
    const u64 *key[MHE_HOIST_R];
    const u64 *mask[MHE_HOIST_R];
    u32 einv[MHE_HOIST_R];
    int key_limbs[MHE_HOIST_R];
    int Z; // items (<= MHE_MAXB)
};
#ifndef MHE_HOIST_PF
#define MHE_HOIST_PF 2 // digits of key / D words in flight ahead of the one being staged
#endif
template <int R>
__global__ __launch_bounds__(1024) void k_ks_hoist_mac_sh(HoistShared P, const PrimeDev *__restrict__ primes,
                                                          const TwF *__restrict__ cm, int L, int K, int log_n)
{
    constexpr int NV = 2 * R * 256;          // staged key words per digit: [kk][r][column]
    constexpr int S = (NV + 1023) / 1024;    // per lane
    constexpr int IPL = R <= 4 ? 2 : 1;      // items per lane
    constexpr int PF = MHE_HOIST_PF;
    __shared__ double kb[2][NV];
    const size_t n = (size_t)1 << log_n;
    // grp, and the key row a lane stages, are uniform per wave: readfirstlane makes that visible, so
    // the kernel-argument arrays they index are read with scalar loads (per-lane indices made the
    // compiler read them with vector loads and wait vmcnt(0) for each -- draining the prefetches)
    const int tid = threadIdx.x, grp = __builtin_amdgcn_readfirstlane(tid >> 8);
    const u32 u = (u32)(tid & 255), m = blockIdx.x * 256u + brev8(u); // D position blockIdx.x 256 + u holds slot m
    const int I = (int)blockIdx.y;
    const int pi = (I == L) ? K - 1 : I;
    const PrimeDev p = primes[pi];
    const double q = (double)p.q, qinv = 1.0 / q;
    // this lane's items (uniform per 256-lane group): present and not flagged
    const int i0 = (int)blockIdx.z * 4 * IPL + grp * IPL, i1 = i0 + 1;
    const bool v0 = i0 < P.Z && !*P.flag[i0], v1 = IPL > 1 && i1 < P.Z && !*P.flag[i1];
    // rotation r's output slot for this lane's D slot as a bit-reversed column, 8 bits each (its
    // block is rho_r^-1 of this block for every slot of it; consecutive lanes read kb an odd stride
    // apart); the full slot is recomputed for the epilogue
    u32 kcol[(R + 3) / 4];
#pragma unroll
    for (int w = 0; w < (R + 3) / 4; w++) kcol[w] = 0;
#pragma unroll
    for (int r = 0; r < R; r++) kcol[r / 4] |= brev8(galois_src(m, P.einv[r], log_n) & 255u) << (8 * (r % 4));
    double a0[IPL][R], a1[IPL][R];
    u32 kdm = 0, k48 = 0; // bit r: rotation r's key slot holds doubles / 48-bit planes, read once
#pragma unroll
    for (int r = 0; r < R; r++)
    {
#pragma unroll
        for (int it = 0; it < IPL; it++) a0[it][r] = a1[it][r] = 0.0;
        const int kl = P.key_limbs[r];
        const int f = key_slot_format(P.key[r][(size_t)((I == L) ? kl - 1 : I) * n + n - 1]);
        kdm |= (f == 1 ? 1u : 0u) << r;
        k48 |= (f == 2 ? 1u : 0u) << r;
    }
    // staging: word v = tid + 1024 s is bit-reversed column v & 255 of key row (kk, r) =
    // (v / (256 R), (v / 256) % R), read from the key at its natural column and written to kb at v.
    // Every load below is issued unconditionally (lanes past NV and digits past L re-read valid
    // words, discarded), so the loads in flight have fixed counts and the compiler waits for the
    // oldest ones only (vmcnt(N)) instead of draining all of them at each digit.
    auto stage_load = [&](int J, u64 (&sv)[S], auto kp_tag) {
        constexpr int KP = decltype(kp_tag)::value; // as in k_ks_hoist_mac
#pragma unroll
        for (int s = 0; s < S; s++)
        {
            const int v = min(tid + 1024 * s, NV - 1);
            const int vw = __builtin_amdgcn_readfirstlane(v >> 8); // the wave's 64 lanes share one key row
            const int kk = vw / R, r = vw % R, c = v & 255;
            const int kl = P.key_limbs[r];
            const u64 *slot = P.key[r] + ((size_t)(2 * J + kk) * kl + (size_t)((I == L) ? kl - 1 : I)) * n;
            const u32 x = (galois_src(blockIdx.x * 256u, P.einv[r], log_n) & ~255u) + brev8((u32)c); // block rho_r^-1
            if (KP == 2 || (KP == -1 && ((k48 >> r) & 1)))
            {
                const u32 *lo = reinterpret_cast<const u32 *>(slot);
                sv[s] = (u64)lo[x] | ((u64)reinterpret_cast<const unsigned short *>(lo + n)[x] << 32);
            }
            else
                sv[s] = slot[x];
        }
    };
    // the items' D words (unflagged lanes of absent items read item 0's)
    const u64 *D0 = P.D[v0 ? i0 : 0] + (size_t)I * L * n, *C0 = P.c1[v0 ? i0 : 0];
    const u64 *D1 = P.D[(IPL > 1 && v1) ? i1 : 0] + (size_t)I * L * n, *C1 = P.c1[(IPL > 1 && v1) ? i1 : 0];
    auto d_load = [&](int J, u64 (&d)[IPL]) {
        const size_t off = (size_t)J * n + m, pos = (size_t)J * n + blockIdx.x * 256u + u;
        d[0] = (J == I) ? C0[off] : D0[pos];
        if constexpr (IPL > 1) d[IPL - 1] = (J == I) ? C1[off] : D1[pos];
    };
    const bool lz = p.q < (1ull << 47) && (double)L * 1.25 * q < 9007199254740992.0;
    double kc[S];
#pragma unroll
    for (int s = 0; s < S; s++) kc[s] = 0.0;
    auto run = [&](auto kp_tag) {
        // ring of PF digits in flight
        u64 sv[PF][S], dv[PF][IPL];
#pragma unroll
        for (int u = 0; u < PF; u++)
        {
            const int Ju = u < L ? u : L - 1;
            stage_load(Ju, sv[u], kp_tag);
            d_load(Ju, dv[u]);
        }
        for (int J0 = 0; J0 < L; J0 += PF)
        {
#pragma unroll
            for (int u = 0; u < PF; u++)
            {
                const int J = J0 + u;
                if (J >= L) break; // uniform
                const int buf = J & 1;
                const TwF c = cm[(size_t)J * K + pi]; // (q_J mod p, / p); (0, 0) for J == I
#pragma unroll
                for (int s = 0; s < S; s++)
                {
                    const int v = tid + 1024 * s;
                    // the staged word as a double
                    constexpr int KP = decltype(kp_tag)::value;
                    const int kr = __builtin_amdgcn_readfirstlane((min(v, NV - 1) >> 8) % R);
                    const double w = (KP == 1 || (KP == -1 && ((kdm >> kr) & 1))) ? key_word_f(sv[u][s])
                                                                                  : fp_from_u52(sv[u][s]);
                    if (v < NV) kb[buf][v] = w;
                    kc[s] += fp_mulmod(w, c.x, c.y, q); // |term| < 1.5p; reduced every second digit
                    if (J & 1) kc[s] = fp_reduce(kc[s], q, qinv);
                }
                double dd[IPL];
#pragma unroll
                for (int it = 0; it < IPL; it++) dd[it] = fp_from_u52(dv[u][it]);
                // the ring slot is free again: digit J + PF (the last digit again past the end)
                const int Jn = J + PF < L ? J + PF : L - 1;
                stage_load(Jn, sv[u], kp_tag);
                d_load(Jn, dv[u]);
                lds_barrier(); // kb[buf] visible (its previous contents, digit J - 2, read before the last barrier)
#pragma unroll
                for (int r = 0; r < R; r++)
                {
                    const u32 x = (kcol[r / 4] >> (8 * (r % 4))) & 255u;
                    const double w0 = kb[buf][r * 256 + x], w1 = kb[buf][(R + r) * 256 + x];
                    a0[0][r] += fp_mulmod_gen(dd[0], w0, q, qinv);
                    a1[0][r] += fp_mulmod_gen(dd[0], w1, q, qinv);
                    if constexpr (IPL > 1)
                    {
                        a0[IPL - 1][r] += fp_mulmod_gen(dd[IPL - 1], w0, q, qinv);
                        a1[IPL - 1][r] += fp_mulmod_gen(dd[IPL - 1], w1, q, qinv);
                    }
                    if (!lz && (J & 1))
                    {
#pragma unroll
                        for (int it = 0; it < IPL; it++)
                        {
                            a0[it][r] = fp_reduce(a0[it][r], q, qinv);
                            a1[it][r] = fp_reduce(a1[it][r], q, qinv);
                        }
                    }
                }
            }
        }
    };
    const u32 all = (1u << R) - 1;
    if (kdm == all)
        run(std::integral_constant<int, 1>{});
    else if (k48 == all)
        run(std::integral_constant<int, 2>{});
    else if ((kdm | k48) == 0)
        run(std::integral_constant<int, 0>{});
    else
        run(std::integral_constant<int, -1>{});
    // KC through LDS: every lane's staged words' sums, then each item's M[k] KC[k]
    lds_barrier();
#pragma unroll
    for (int s = 0; s < S; s++)
    {
        const int v = tid + 1024 * s;
        if (v < NV) kb[0][v] = fp_reduce(kc[s], q, qinv);
    }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < R; r++)
    {
        const u32 k = galois_src(m, P.einv[r], log_n), x = brev8(k & 255u);
        const double mk = fp_from_u52(P.mask[r][(size_t)pi * n + k]);
        const double c0 = fp_mulmod_gen(mk, kb[0][r * 256 + x], q, qinv);
        const double c1v = fp_mulmod_gen(mk, kb[0][(R + r) * 256 + x], q, qinv);
#pragma unroll
        for (int it = 0; it < IPL; it++)
        {
            if (!(it ? v1 : v0)) continue;
            u64 *o0 = P.acc[it ? i1 : i0][r] + (size_t)I * n;
            u64 *o1 = o0 + (size_t)(L + 1) * n;
            // |acc| < 2^53 (lazy: L 1.25p sums; else reduced every second digit)
            o0[k] = fp_canon(fp_reduce(a0[it][r], q, qinv) + c0, q, qinv);
            o1[k] = fp_canon(fp_reduce(a1[it][r], q, qinv) + c1v, q, qinv);
        }
    }
}

// flag = 1 when a digit of the coefficient-form input has a zero at a slot k >= 1 (slot 0 is
// never negated): then the hoisting identity may not hold and the classic path runs.
__global__ void k_zero_scan(const u64 *__restrict__ coeff, int log_n, size_t total, int *flag)
{
    const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= total) return;
    const size_t k = g & (((size_t)1 << log_n) - 1);
    if (k != 0 && coeff[g] == 0) flag[0] = 1;
}

// The negation mask of Galois element g in coefficient form, replicated over K limbs: slot
// t mod N of X^(k g) is 1 when k g mod 2N >= N (the coefficient moved there is negated).
__global__ void k_negmask(u64 *out, u32 elt, int K, int log_n)
{
    const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t n = (size_t)1 << log_n;
    if (g >= (size_t)K * n) return;
    const size_t limb = g >> log_n;
    const u32 k = (u32)(g & (n - 1));
    const u32 t = (u32)(((u64)k * elt) & (2 * n - 1));
    out[limb * n + (t & (n - 1))] = t >= n ? 1 : 0;
}
