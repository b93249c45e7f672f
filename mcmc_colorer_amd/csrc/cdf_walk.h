// mcmc_colorer_amd/csrc/cdf_walk.h -- exact fp32 CDF walk of extract_new_color over runs of
// equal probabilities (graph_coloring/coloringMCMC_CPU.cpp:505-520), for large nCol.
//
// The reference walks every colour: `cdf += p[c]; if (cdf > u) break;` in fp32 with
// round-to-nearest-even. p takes only two values per vertex (fill_p, :393-481: eps / pf, or
// eps / hi), so the walk is a sequence of RUNS of identical addends. Inside one binade
// [2^e, 2^(e+1)) of cdf every sum rounds to a multiple of U = ulp(cdf), so adding x moves the
// mantissa integer k by round(x / U) -- a constant, except when x / U has fraction exactly 1/2
// (a tie): then RNE picks the even neighbour, so every tie result is even and, from the second
// step of the run inside the binade on, the increment is constant again. cdf_run therefore takes
// explicit fp32 steps until two consecutive steps of the run stayed in one binade, then jumps
// with integer arithmetic on the mantissa to the first step that exceeds u or leaves the binade.
// Bit-identical to the step-by-step walk (pinned by tests/test_wide.py against a numpy float32
// walk and by GPU parity with the oracle); O(runs + binades) instead of O(nCol).
#pragma once
#include <stdint.h>

#include "rng.h"   // MCMC_HD

namespace mcmc {

MCMC_HD uint32_t f32_bits(float x) {
    union { float f; uint32_t u; } c;
    c.f = x;
    return c.u;
}
MCMC_HD float f32_from(uint32_t b) {
    union { float f; uint32_t u; } c;
    c.u = b;
    return c.f;
}

// cdf += x, r times, in fp32 (no contraction). Returns the 1-based step whose result first
// exceeds u (cdf then holds that result), or 0 when no step did (cdf after all r steps).
// Requires x > 0, cdf >= 0 and finite values below 2^127.
MCMC_HD bool pos_normal(float x) { return x >= 1.17549435e-38f && x < 3.0e38f; }

MCMC_HD uint32_t cdf_run(float& cdf, float x, uint32_t r, float u) {
    uint32_t j = 0;
    if (!pos_normal(x)) {   // the jumps assume a positive normal addend (pf < 0 needs eps * Zv > 1)
        for (; j < r;) {
            cdf += x;
            j++;
            if (cdf > u) return j;
        }
        return 0;
    }
    int inb = 0;   // consecutive steps of this run that stayed inside one binade
    while (j < r) {
        const float prev = cdf;
        const float nx = prev + x;
        j++;
        cdf = nx;
        if (nx > u) return j;
        const uint32_t bp = f32_bits(prev), bn = f32_bits(nx);
        const bool same = prev > 0.0f && (bp >> 23) == (bn >> 23) && (bn >> 23) != 0u;
        inb = same ? inb + 1 : 0;
        if (inb < 2 || j == r) continue;
        // constant increment kD (mantissa units) for every further step inside this binade
        const uint32_t kD = bn - bp;
        if (kD == 0) return 0;   // x vanishes below half an ulp: cdf stays <= u to the end
        const uint32_t E = bn >> 23;
        const uint32_t kk = (bn & 0x7FFFFFu) | 0x800000u;
        const uint32_t rem = r - j;
        const uint32_t ibin = (0xFFFFFFu - kk) / kD;   // steps that stay below 2^(e+1)
        const uint32_t lim = ibin < rem ? ibin : rem;
        // u >= cdf, so u's exponent is >= E; a stop inside this binade needs u in it
        const uint32_t bu = f32_bits(u);
        if ((bu >> 23) == E) {
            const uint32_t T = (bu & 0x7FFFFFu) | 0x800000u;   // u = T * U exactly
            const uint32_t istop = (T - kk) / kD + 1u;          // first i with kk + i kD > T
            if (istop <= lim) {
                cdf = f32_from(bn + istop * kD);
                return j + istop;
            }
        }
        cdf = f32_from(bn + lim * kD);
        j += lim;
        inb = 0;   // the next step leaves the binade (or the run is over)
    }
    return 0;
}

// extract_new_color for the "own colour" distribution of fill_p's cases (i) and (iii)
// (:402-412, :471-479): p[c] = hi for c == cv, eps otherwise. Returns the colour, or nCol for
// a CDF overflow (the glibc fallback, :517-520).
MCMC_HD uint32_t walk_own(uint32_t nCol, uint32_t cv, float eps, float hi, float u) {
    float cdf = 0.0f;
    uint32_t s = cdf_run(cdf, eps, cv, u);
    if (s) return s - 1u;
    if (cdf_run(cdf, hi, 1u, u)) return cv;
    s = cdf_run(cdf, eps, nCol - cv - 1u, u);
    return s ? cv + s : nCol;
}

// Increment of the mantissa integer k (units of U = ulp of binade E: cdf = k U, k in [2^23, 2^24))
// when x is added inside the binade: round(x / U) to nearest. Returns false on a tie (x / U has
// fraction exactly 1/2: the rounding then depends on k's parity) or when x / U >= 2^8 (the sum
// leaves the binade anyway). x must be a positive normal float.
MCMC_HD bool binade_inc(float x, uint32_t E, uint32_t& d) {
    const uint32_t bx = f32_bits(x);
    const uint32_t ex = bx >> 23, mx = (bx & 0x7FFFFFu) | 0x800000u;   // x = mx 2^(ex - 150)
    if (ex >= E) {
        if (ex - E > 7u) return false;
        d = mx << (ex - E);
        return true;
    }
    const uint32_t sh = E - ex;
    if (sh > 25u) { d = 0; return true; }   // x / U < 2^-2
    const uint32_t rem = mx & ((1u << sh) - 1u), half = 1u << (sh - 1u);
    if (rem == half) return false;
    d = (mx >> sh) + (rem > half ? 1u : 0u);
    return true;
}

// Case (ii) (:414-420): p[c] = eps where colour c is occupied (bit set in `mask`, nCol bits,
// 32 per word), pf where it is free. Per 32-colour word: inside one binade the sum is order-free
// (k += popc * dE + (32 - popc) * dP) as long as neither addend ties, the word's end stays in the
// binade and does not pass u -- then the word costs O(1); runs of empty words jump with cdf_run;
// any other word is walked colour by colour.
template <typename MaskT>
MCMC_HD uint32_t walk_mask(const MaskT* mask, uint32_t nCol, float eps, float pf, float u) {
    float cdf = 0.0f;
    const uint32_t bu = f32_bits(u);
    if (!pos_normal(eps) || !pos_normal(pf)) {   // the word arithmetic needs positive normal addends
        for (uint32_t c = 0; c < nCol; c++) {
            cdf += (((uint32_t)mask[c >> 5] >> (c & 31u)) & 1u) ? eps : pf;
            if (cdf > u) return c;
        }
        return nCol;
    }
    for (uint32_t c = 0; c < nCol;) {
        const uint32_t w = c >> 5;
        const uint32_t nb = nCol - c < 32u ? nCol - c : 32u;
        const uint32_t word = (uint32_t)mask[w] & (nb == 32u ? ~0u : ((1u << nb) - 1u));
        if (word == 0u && nb == 32u) {   // a run of all-free words
            uint32_t z = 1;
            while (c + 32u * (z + 1u) <= nCol && mask[w + z] == 0u) z++;
            const uint32_t s = cdf_run(cdf, pf, 32u * z, u);
            if (s) return c + s - 1u;
            c += 32u * z;
            continue;
        }
        const uint32_t bc = f32_bits(cdf);
        const uint32_t E = bc >> 23;
        uint32_t dE = 0, dP = 0;
        if (E != 0u && binade_inc(eps, E, dE) && binade_inc(pf, E, dP)) {
            const uint32_t ne = (uint32_t)__builtin_popcount(word);
            const uint64_t kend = (uint64_t)((bc & 0x7FFFFFu) | 0x800000u) + (uint64_t)ne * dE + (uint64_t)(nb - ne) * dP;
            // no stop inside the word: cdf is monotone, so its end must stay <= u
            const bool below_u = (bu >> 23) > E || kend <= (uint64_t)((bu & 0x7FFFFFu) | 0x800000u);
            if (kend <= 0xFFFFFFu && below_u) {
                cdf = f32_from((E << 23) | ((uint32_t)kend & 0x7FFFFFu));
                c += nb;
                continue;
            }
        }
        for (uint32_t b = 0; b < nb; b++) {
            cdf += ((word >> b) & 1u) ? eps : pf;
            if (cdf > u) return c + b;
        }
        c += nb;
    }
    return nCol;
}

// walk_own with the table E[k] = fl(...fl(eps + eps)... + eps) (k terms, E[0] = 0): the cdf before
// colour cv is E[cv], so a stop before cv is a binary search and the rest is two steps.
MCMC_HD uint32_t walk_own_tab(const float* E, uint32_t nCol, uint32_t cv, float eps, float hi, float u) {
    if (!(eps > 0.0f)) return walk_own(nCol, cv, eps, hi, u);   // E is monotone only for eps > 0
    const float ecv = E[cv];
    if (ecv > u) {   // the first k in [1, cv] with E[k] > u stops at colour k - 1
        uint32_t lo = 1, up = cv;
        while (lo < up) {
            const uint32_t mid = (lo + up) >> 1;
            if (E[mid] > u) up = mid; else lo = mid + 1u;
        }
        return lo - 1u;
    }
    float cdf = ecv + hi;
    if (cdf > u) return cv;
    const uint32_t s = cdf_run(cdf, eps, nCol - cv - 1u, u);
    return s ? cv + s : nCol;
}

// The table of walk_own_tab, host side (nCol + 1 entries).
inline void eps_table(float eps, uint32_t nCol, float* E) {
    E[0] = 0.0f;
    for (uint32_t k = 1; k <= nCol; k++) E[k] = E[k - 1] + eps;
}

}  // namespace mcmc
