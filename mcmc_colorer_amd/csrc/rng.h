// mcmc_colorer_amd/csrc/rng.h -- random streams of the reference's --mcmccpu path, as
// counter-addressable functions usable from host and device code.
//
//  * minstd_rand0 (std::default_random_engine in libstdc++), the engine of ColoringMCMC_CPU
//    (graph_coloring/coloringMCMC_CPU.cpp:53). Skip-ahead x_{k+j} = x_k * 16807^j mod (2^31-1)
//    lets every vertex compute its own draw of a sweep: vertex v of sweep t uses engine draw
//    K0 + t*n + v + 1 (the bulk draw at coloringMCMC_CPU.cpp:139 is in vertex order).
//  * generate_canonical<float,24> (libstdc++ random.tcc:3348-3380): one engine call per float.
//  * uniform_int_distribution<uint32_t>(0, nCol-1) over minstd (libstdc++ uniform_int_dist.h,
//    "fallback (2 divisions)"), used for the initial coloring (coloringMCMC_CPU.cpp:61).
//  * glibc rand() TYPE_3 (stdlib/random_r.c): r[i] = r[i-3] + r[i-31] mod 2^32, output r >> 1.
//    Linear over Z/2^32, so it jumps ahead with x^k mod (x^31 - x^28 - 1). The reference draws
//    from it in setupRnd2 (graphCPU.cpp:308) and on CDF overflow (coloringMCMC_CPU.cpp:518).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define MCMC_HD __host__ __device__ __forceinline__
#else
#define MCMC_HD inline
#endif

namespace mcmc {

constexpr uint32_t kMinstdM = 2147483647u;
constexpr uint32_t kMinstdA = 16807u;

// (a * b) mod (2^31 - 1) for a, b < 2^31, by Mersenne folding (no 64-bit division).
MCMC_HD uint32_t minstd_mulmod(uint32_t a, uint32_t b) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    uint64_t r = (p & kMinstdM) + (p >> 31);
    r = (r & kMinstdM) + (r >> 31);
    if (r >= kMinstdM) r -= kMinstdM;
    return (uint32_t)r;
}

MCMC_HD uint32_t minstd_pow(uint32_t a, uint64_t e) {
    uint32_t r = 1;
    while (e) {
        if (e & 1) r = minstd_mulmod(r, a);
        a = minstd_mulmod(a, a);
        e >>= 1;
    }
    return r;
}

// Discrete logarithm base 16807 modulo 2^31 - 1: the L in [0, N), N = 2^31 - 2, with 16807^L = x.
// 16807 is a primitive root of the prime 2^31 - 1 (the reason minstd uses it: Park & Miller), so
// every state x in [1, 2^31 - 2] has exactly one. N = 2 * 3^2 * 7 * 11 * 31 * 151 * 331 is smooth:
// Pohlig-Hellman -- per prime power q^e, L mod q^e is the d < q^e with (16807^(N/q^e))^d =
// x^(N/q^e), found by stepping; the Chinese remainder theorem assembles L. About 900 mulmods.
// Returns 0xFFFFFFFF for x outside the group (0 or >= 2^31 - 1).
// Use: engine draw j after state x_t is x_t 16807^j = 16807^(L(x_t) + j), so the vertices whose
// draw lands in a given set of states follow from the states' logarithms (dense_sparse.h).
constexpr uint32_t kMinstdN = kMinstdM - 1u;   // the multiplicative group's order
MCMC_HD uint32_t minstd_dlog(uint32_t x) {
    if (x == 0u || x >= kMinstdM) return 0xFFFFFFFFu;
    const uint32_t qe[7] = {2u, 9u, 7u, 11u, 31u, 151u, 331u};
    uint64_t L = 0;
    for (int i = 0; i < 7; i++) {
        const uint32_t q = qe[i], m = kMinstdN / q;
        const uint32_t g = minstd_pow(kMinstdA, m), h = minstd_pow(x, m);
        uint32_t y = 1u, d = 0u;
        while (y != h && d < q) {
            y = minstd_mulmod(y, g);
            d++;
        }
        if (d == q) return 0xFFFFFFFFu;
        // CRT coefficient: m (m^-1 mod q), so it is 1 mod q and 0 mod the other prime powers
        const uint32_t mr = m % q;
        uint32_t inv = 1u;
        while ((uint64_t)mr * inv % q != 1u) inv++;
        L = (L + (uint64_t)d * ((uint64_t)m * inv % kMinstdN)) % kMinstdN;
    }
    return (uint32_t)L;
}

// linear_congruential_engine::seed(s): x0 = s mod m, or 1 when that is 0.
MCMC_HD uint32_t minstd_seed_state(uint32_t seed) {
    uint32_t s = seed % kMinstdM;
    return s == 0 ? 1u : s;
}

// generate_canonical<float,24>(minstd): float(x - 1) / 2^31, clamped to nextafter(1, 0).
// float(uint32) rounds to nearest-even on host (cvtsi2ss) and device (v_cvt_f32_u32) alike;
// the scale by 2^-31 is exact.
MCMC_HD float minstd_canonical(uint32_t x) {
    float r = (float)(x - 1u) * 0x1p-31f;
    return r >= 1.0f ? 0x1.fffffep-1f : r;
}

// uniform_int_distribution<uint32_t>(0, nCol-1) constants for the minstd range [1, 2^31-2].
struct UniformIntConst {
    uint32_t scaling;
    uint32_t past;
};
MCMC_HD UniformIntConst uniform_int_const(uint32_t nCol) {
    const uint32_t urngrange = 2147483645u;
    UniformIntConst k;
    k.scaling = urngrange / nCol;
    k.past = nCol * k.scaling;
    return k;
}

// ------------------------------------------------------------------------------------------------
// glibc TYPE_3 rand(). State = the 31 most recent words r[i-31..i-1] (oldest first); the next
// output is (r[i-31] + r[i-3]) >> 1. After srand(s) the window is r[313..343] (310 discards).
struct GlibcWindow {
    uint32_t r[31];
};

MCMC_HD GlibcWindow glibc_srand(uint32_t seed) {
    uint32_t s[344];
    if (seed == 0) seed = 1;
    s[0] = seed;
    int32_t word = (int32_t)seed;
    for (int i = 1; i < 31; i++) {
        int32_t hi = word / 127773, lo = word % 127773;   // C truncating division, as glibc
        word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        s[i] = (uint32_t)word;
    }
    for (int i = 31; i < 34; i++) s[i] = s[i - 31];
    for (int i = 34; i < 344; i++) s[i] = s[i - 31] + s[i - 3];
    GlibcWindow w;
    for (int i = 0; i < 31; i++) w.r[i] = s[313 + i];
    return w;
}

// Sequential draw on a window held as a ring: head = index of the oldest word r[i-31].
MCMC_HD uint32_t glibc_next(uint32_t* ring, uint32_t& head) {
    uint32_t v = ring[head] + ring[(head + 28) % 31];
    ring[head] = v;
    head = (head + 1) % 31;
    return v >> 1;
}

// Polynomials over Z/2^32 modulo P(x) = x^31 - x^28 - 1, i.e. x^31 == x^28 + 1.
struct GlibcPoly {
    uint32_t c[31];
};

MCMC_HD GlibcPoly glibc_poly_mul(const GlibcPoly& a, const GlibcPoly& b) {
    uint32_t t[61];
    for (int i = 0; i < 61; i++) t[i] = 0;
    for (int i = 0; i < 31; i++)
        for (int j = 0; j < 31; j++) t[i + j] += a.c[i] * b.c[j];
    for (int d = 60; d >= 31; d--) {   // x^d = x^(d-3) + x^(d-31)
        t[d - 3] += t[d];
        t[d - 31] += t[d];
    }
    GlibcPoly r;
    for (int i = 0; i < 31; i++) r.c[i] = t[i];
    return r;
}

MCMC_HD GlibcPoly glibc_poly_mulx(const GlibcPoly& a) {
    GlibcPoly r;
    uint32_t top = a.c[30];
    for (int i = 30; i > 0; i--) r.c[i] = a.c[i - 1];
    r.c[0] = top;        // x^31 -> 1 + x^28
    r.c[28] += top;
    return r;
}

MCMC_HD GlibcPoly glibc_poly_xpow(uint64_t k) {
    GlibcPoly r, b;
    for (int i = 0; i < 31; i++) { r.c[i] = 0; b.c[i] = 0; }
    r.c[0] = 1;
    b.c[1] = 1;
    while (k) {
        if (k & 1) r = glibc_poly_mul(r, b);
        b = glibc_poly_mul(b, b);
        k >>= 1;
    }
    return r;
}

// Advance a window by k draws: r[n+k+j] = sum_i [x^(k+j) mod P]_i * r[n+i].
MCMC_HD GlibcWindow glibc_jump(const GlibcWindow& w, uint64_t k) {
    GlibcPoly q = glibc_poly_xpow(k);
    GlibcWindow out;
    for (int j = 0; j < 31; j++) {
        uint32_t acc = 0;
        for (int i = 0; i < 31; i++) acc += q.c[i] * w.r[i];
        out.r[j] = acc;
        q = glibc_poly_mulx(q);
    }
    return out;
}

}  // namespace mcmc
