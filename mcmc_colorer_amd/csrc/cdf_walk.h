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
MCMC_HD uint32_t cdf_run(float& cdf, float x, uint32_t r, float u) {
    uint32_t j = 0;
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

// Case (ii) (:414-420): p[c] = eps where colour c is occupied (bit set in `mask`, nCol bits,
// 32 per word), pf where it is free. Runs are read off the mask with count-trailing-zeros.
template <typename MaskT>
MCMC_HD uint32_t walk_mask(const MaskT* mask, uint32_t nCol, float eps, float pf, float u) {
    float cdf = 0.0f;
    uint32_t c = 0;
    while (c < nCol) {
        const uint32_t occ = (mask[c >> 5] >> (c & 31u)) & 1u;
        // length of the run of equal bits starting at c
        uint32_t len = 0, cc = c;
        while (cc < nCol) {
            const uint32_t b = cc & 31u;
            uint32_t w = mask[cc >> 5] >> b;
            if (!occ) w = ~w;
            // w: bit i set while the run continues; (32 - b) bits of this word remain
            const uint32_t stop = ~w;
            const uint32_t avail = 32u - b;
            const uint32_t t = stop ? (uint32_t)__builtin_ctz(stop) : 32u;
            const uint32_t take = t < avail ? t : avail;
            len += take;
            cc += take;
            if (take < avail) break;
        }
        if (cc > nCol) len -= cc - nCol;
        const uint32_t s = cdf_run(cdf, occ ? eps : pf, len, u);
        if (s) return c + s - 1u;
        c += len;
    }
    return nCol;
}

}  // namespace mcmc
