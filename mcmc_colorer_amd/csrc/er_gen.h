// mcmc_colorer_amd/csrc/er_gen.h -- the build's counter-based G(n, p) generator, shared verbatim by
// the device (graph_er.hip) and the CPU restatement (oracle/), so both enumerate the same graph.
//
// the reference's setupRnd2 (5e13 sequential glibc draws at n = 1e7) is
// infeasible, so configs 3-4 use this documented generator ("counter-based Philox + geometric
// skips, fixed seed"); parity there is GPU vs restatement on the same graph. Definition:
//
//   T = 2^16 columns per block. For every row i in [0, n) and every column block Y with
//   Y >= i / T, stream (i, Y) walks the columns j of block Y with j > i:
//     j = max(Y*T, i + 1) - 1;  repeat { j += skip(next u); if j >= min(n, (Y+1)*T) stop; edge {i, j} }
//   skip(u) = 1 + floor(ln(u) * inv_l1p), inv_l1p = 1 / log1p(-p) (computed once on the host in
//   double from p = (double)(float)prob, like setupRnd2's comparison, graphCPU.cpp:308);
//   u = (x + 1) * 2^-32 for the stream's successive Philox4x32-10 outputs x (4 per counter),
//   counter = {k, i, Y, 0x45524721}, k = 0, 1, ..., key = {seed & 0xffffffff, seed >> 32}.
//   Every edge is emitted exactly once (i < j), both arcs are stored. p >= 1: complete graph;
//   p <= 0: empty.
//
// Each edge is present independently with probability p: the gaps between successive present
// columns of a stream are i.i.d. geometric(p) (inversion of the geometric CDF). ln() is computed
// by det_log from +, -, *, / only, so a host build and a gfx950 build (both -ffp-contract=off)
// produce bit-identical skips.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define ER_HD __host__ __device__ __forceinline__
#else
#define ER_HD inline
#endif

namespace er {

constexpr uint32_t kBlockLog2 = 16;
constexpr uint32_t kTag = 0x45524721u;

struct Philox4 {
    uint32_t v[4];
};

ER_HD void mulhilo(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
    const uint64_t p = (uint64_t)a * b;
    hi = (uint32_t)(p >> 32);
    lo = (uint32_t)p;
}

// Philox4x32-10 (Salmon, Moraes, Dror, Shaw: "Parallel random numbers: as easy as 1, 2, 3", SC'11).
ER_HD Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; r++) {
        uint32_t hi0, lo0, hi1, lo1;
        mulhilo(0xD2511F53u, c0, hi0, lo0);
        mulhilo(0xCD9E8D57u, c2, hi1, lo1);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return Philox4{{c0, c1, c2, c3}};
}

// Natural log of u in (0, 1], from +, -, *, / only (identical on host and device): u = m * 2^e with
// m in [sqrt(1/2), sqrt(2)), ln m = 2 atanh(s), s = (m-1)/(m+1), |s| < 0.1716, series to s^25.
ER_HD double det_log(double u) {
    union { double d; uint64_t b; } x;
    x.d = u;
    int e = (int)((x.b >> 52) & 0x7FF) - 1023;
    x.b = (x.b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull;   // m in [1, 2)
    double m = x.d;
    if (m > 1.4142135623730951) { m = m * 0.5; e += 1; }
    const double s = (m - 1.0) / (m + 1.0);
    const double s2 = s * s;
    double poly = 1.0 / 25.0;
    poly = poly * s2 + 1.0 / 23.0;
    poly = poly * s2 + 1.0 / 21.0;
    poly = poly * s2 + 1.0 / 19.0;
    poly = poly * s2 + 1.0 / 17.0;
    poly = poly * s2 + 1.0 / 15.0;
    poly = poly * s2 + 1.0 / 13.0;
    poly = poly * s2 + 1.0 / 11.0;
    poly = poly * s2 + 1.0 / 9.0;
    poly = poly * s2 + 1.0 / 7.0;
    poly = poly * s2 + 1.0 / 5.0;
    poly = poly * s2 + 1.0 / 3.0;
    poly = poly * s2 + 1.0;
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    return ((double)e * ln2_hi + 2.0 * s * poly) + (double)e * ln2_lo;
}

// Skip to the next present column: 1 + floor(ln(u) * inv_l1p), capped (a cap beyond any block ends
// the stream just as well).
ER_HD uint32_t geo_skip(uint32_t x, double inv_l1p) {
    const double u = ((double)x + 1.0) * 2.3283064365386963e-10;   // (x + 1) / 2^32, exact
    const double t = det_log(u) * inv_l1p;                            // >= 0
    if (!(t < 2147483647.0)) return 0x7FFFFFFFu;
    return 1u + (uint32_t)t;
}

// Walks stream (i, Y); calls emit(j) for every present column. Returns the number of edges.
// p_mode: 0 regular, 1 complete (p >= 1), 2 empty (p <= 0).
template <class Emit>
ER_HD uint32_t walk_stream(uint64_t seed, double inv_l1p, int p_mode, uint32_t n, uint32_t i, uint32_t Y,
                           Emit&& emit) {
    const uint64_t lo64 = (uint64_t)Y << kBlockLog2;
    const uint64_t hi64 = ((uint64_t)(Y + 1) << kBlockLog2) < n ? ((uint64_t)(Y + 1) << kBlockLog2) : n;
    uint64_t j = (lo64 > (uint64_t)i + 1 ? lo64 : (uint64_t)i + 1);
    if (j >= hi64 || p_mode == 2) return 0;
    uint32_t cnt = 0;
    if (p_mode == 1) {
        for (; j < hi64; j++, cnt++) emit((uint32_t)j);
        return cnt;
    }
    j -= 1;
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    for (uint32_t k = 0;; k++) {
        const Philox4 r = philox4x32_10(k, i, Y, kTag, k0, k1);
        for (int q = 0; q < 4; q++) {
            j += geo_skip(r.v[q], inv_l1p);
            if (j >= hi64) return cnt;
            emit((uint32_t)j);
            cnt++;
        }
    }
}

// ---- R-MAT (Kronecker) stand-in for configs[4] ------------------------------
// SNAP LiveJournal / Reddit are not available here, so C5 runs on a synthetic power-law graph of
// similar size and skew. Definition (mcmc_graph_rmat):
//   n = 2^scale vertices, E = edge_factor * n edge draws e = 0 .. E-1. Draw e picks one quadrant
//   per level l = 0 .. scale-1, most significant bit first, from x = word (l % 4) of
//   Philox4x32-10(counter {e_lo, e_hi, l / 4, 0x524D4154}, key {seed_lo, seed_hi}):
//   x < tA -> (0,0), x < tAB -> (0,1), x < tABC -> (1,0), else (1,1), with the uint32 thresholds
//   tA = floor(a 2^32), tAB = floor((a+b) 2^32), tABC = floor((a+b+c) 2^32) (double, clamped).
//   Both endpoints go through rmat_scramble (a fixed bijection of [0, 2^scale), so the hubs are
//   not the low ids). Self-loops are dropped, both arcs of every other draw kept, duplicates
//   merged; neighbour lists ascending.
constexpr uint32_t kRmatTag = 0x524D4154u;

struct RmatConst {
    uint32_t scale, mask, tA, tAB, tABC, k0, k1;
};

ER_HD uint32_t rmat_scramble(uint32_t x, const RmatConst& k) {
    const uint32_t h = (k.scale + 1u) / 2u;
    x = (x * 0x9E3779B1u) & k.mask;   // odd multiplier: a bijection mod 2^scale
    x ^= x >> h;
    x = (x * 0x85EBCA6Bu) & k.mask;
    x ^= x >> h;
    return (x ^ (k.k0 * 0xC2B2AE35u)) & k.mask;
}

ER_HD void rmat_edge(uint64_t e, const RmatConst& k, uint32_t& i, uint32_t& j) {
    i = 0;
    j = 0;
    for (uint32_t l = 0; l < k.scale; l += 4) {
        const Philox4 r = philox4x32_10((uint32_t)e, (uint32_t)(e >> 32), l >> 2, kRmatTag, k.k0, k.k1);
        for (uint32_t q = 0; q < 4 && l + q < k.scale; q++) {
            const uint32_t x = r.v[q];
            const uint32_t ib = x >= k.tAB ? 1u : 0u;
            const uint32_t jb = ((x >= k.tA && x < k.tAB) || x >= k.tABC) ? 1u : 0u;
            i = (i << 1) | ib;
            j = (j << 1) | jb;
        }
    }
    i = rmat_scramble(i, k);
    j = rmat_scramble(j, k);
}

}  // namespace er
