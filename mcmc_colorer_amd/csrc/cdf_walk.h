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

// binade_inc with ties kept: x / U = d + tie / 2 (tie: the fraction is exactly 1/2, and the sum
// k + x / U rounds to the even neighbour). False only when x / U >= 2^8.
MCMC_HD bool binade_inc_t(float x, uint32_t E, uint32_t& d, uint32_t& tie) {
    const uint32_t bx = f32_bits(x);
    const uint32_t ex = bx >> 23, mx = (bx & 0x7FFFFFu) | 0x800000u;
    tie = 0;
    if (ex >= E) {
        if (ex - E > 7u) return false;
        d = mx << (ex - E);
        return true;
    }
    const uint32_t sh = E - ex;
    if (sh > 25u) { d = 0; return true; }
    const uint32_t rem = mx & ((1u << sh) - 1u), half = 1u << (sh - 1u);
    tie = rem == half ? 1u : 0u;
    d = (mx >> sh) + (rem > half ? 1u : 0u);
    return true;
}

// One 32-colour word of a binade with a tying addend, as a function of the parity of the mantissa
// integer k on entry: a step adds d, plus 1 when the addend ties and k + d is odd (round half to
// even), so the word's total increment and k's parity on exit depend on the entry parity only.
// Colours [b0, nb) of `word`; a[p], q[p]: increment and exit parity for entry parity p.
MCMC_HD void tie_word(uint32_t word, uint32_t b0, uint32_t nb, uint32_t dE, uint32_t tE, uint32_t dP, uint32_t tP,
                      uint32_t (&a)[2], uint32_t (&q)[2]) {
    uint32_t a0 = 0, a1 = 0, p0 = 0, p1 = 1;
    for (uint32_t b = b0; b < nb; b++) {
        const bool occ = (word >> b) & 1u;
        const uint32_t d = occ ? dE : dP, t = occ ? tE : tP;
        const uint32_t i0 = d + (t & ((p0 + d) & 1u)), i1 = d + (t & ((p1 + d) & 1u));
        a0 += i0;
        a1 += i1;
        p0 = (p0 + i0) & 1u;
        p1 = (p1 + i1) & 1u;
    }
    a[0] = a0;
    a[1] = a1;
    q[0] = p0;
    q[1] = p1;
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

// First of 64 candidates (0..63) whose predicate holds, -1 if none. On the device every lane of
// the wave evaluates its own candidate and a ballot picks the first (all 64 lanes must be active
// and call it together); the host build loops.
template <typename Pred>
MCMC_HD int first_of_64(Pred pred) {
#ifdef __HIP_DEVICE_COMPILE__
    const unsigned long long b = __ballot(pred((int)__lane_id()));
    return b ? __ffsll(b) - 1 : -1;
#else
    for (int l = 0; l < 64; l++)
        if (pred(l)) return l;
    return -1;
#endif
}

// Length of the run of colours of one kind (`bit`: 1 occupied, 0 free) from colour c, across words,
// capped at nCol.
MCMC_HD uint32_t mask_run_len(const uint32_t* mask, uint32_t nCol, uint32_t c, uint32_t bit) {
    uint32_t r = 0, x = c;
    while (x < nCol) {
        const uint32_t wv = bit ? ~mask[x >> 5] : mask[x >> 5];   // set bits: the other kind
        const uint32_t rest = wv >> (x & 31u);
        const uint32_t len = rest ? (uint32_t)__builtin_ctz(rest) : 32u - (x & 31u);
        r += len;
        x += len;
        if (rest) break;
    }
    return r < nCol - c ? r : nCol - c;
}

// walk_mask with word prefix counts pre[w] = occupied colours in words < w (NWW + 1 entries),
// for a whole wave. Inside a binade with non-tying increments dE, dP the mantissa integer after
// colour x is k0 + occ(c..x) dE + free(c..x) dP: monotone, so the first colour whose sum passes
// T (u's mantissa when u is in this binade, else the binade's top) is found by testing 64 word
// ends at once, then the 32 colours of the hit word at once. At T = u that colour is the stop;
// at the binade's top it takes one explicit fp32 step (the rounding changes there) and the walk
// continues in the next binade. Binades whose increments tie (or cdf = 0) step one colour at a
// time. Cost: O(binades + nCol / 2048) wave steps instead of O(nCol / 32) serial ones.
MCMC_HD uint32_t walk_mask_pre(const uint32_t* mask, const uint32_t* pre, uint32_t nCol, float eps, float pf,
                               float u, bool tie_scan = true) {
    if (!pos_normal(eps) || !pos_normal(pf)) return walk_mask(mask, nCol, eps, pf, u);
    const uint32_t NWW = (nCol + 31u) >> 5;
    const uint32_t bu = f32_bits(u);
    float cdf = 0.0f;
    uint32_t c = 0;
    while (c < nCol) {
        const uint32_t bc = f32_bits(cdf);
        const uint32_t E = bc >> 23;
        uint32_t dE = 0, dP = 0, tE = 0, tP = 0;
        // (increments below 2^20: 64 words x 32 colours of them, ties included, stay below 2^32 in the
        // uint32 word functions and their scan; a larger increment leaves the binade within 16
        // steps, so the run-by-run path below is as short)
        if (tie_scan && E != 0u && binade_inc_t(eps, E, dE, tE) && binade_inc_t(pf, E, dP, tP) && (tE | tP) != 0u &&
            (dE | dP) < (1u << 20)) {
            // a tie binade with mixed words: each word is a function of k's parity on entry
            // (tie_word); 64 words at a time, the functions composed by a wave scan, the first word
            // whose end passes T found by a ballot, then that word colour by colour (a violator's
            // mask with runs of a few colours crossed such a binade run by run: ~250 us per walk)
            const uint32_t k0 = (bc & 0x7FFFFFu) | 0x800000u;
            const uint32_t T = ((bu >> 23) == E) ? ((bu & 0x7FFFFFu) | 0x800000u) : 0xFFFFFFu;
            const uint32_t w0 = c >> 5;
            uint32_t k = k0, wf = NWW, ks = 0;
            for (uint32_t wb = w0; wb < NWW && wf == NWW; wb += 64u) {
#ifdef __HIP_DEVICE_COMPILE__
                const uint32_t lane = __lane_id(), w = wb + lane;
                uint32_t fa[2] = {0u, 0u}, fq[2] = {0u, 1u};   // identity past the last word
                if (w < NWW)
                    tie_word(mask[w], w == w0 ? (c & 31u) : 0u, nCol - 32u * w < 32u ? nCol - 32u * w : 32u, dE, tE,
                             dP, tP, fa, fq);
                for (int o = 1; o < 64; o <<= 1) {   // inclusive scan: the words before, then this one
                    const uint32_t pa0 = __shfl_up(fa[0], o, 64), pa1 = __shfl_up(fa[1], o, 64);
                    const uint32_t pq0 = __shfl_up(fq[0], o, 64), pq1 = __shfl_up(fq[1], o, 64);
                    if (lane >= (uint32_t)o) {
                        const uint32_t na0 = pa0 + fa[pq0], na1 = pa1 + fa[pq1];
                        const uint32_t nq0 = fq[pq0], nq1 = fq[pq1];
                        fa[0] = na0;
                        fa[1] = na1;
                        fq[0] = nq0;
                        fq[1] = nq1;
                    }
                }
                const uint32_t kend = k + fa[k & 1u];
                const unsigned long long hb = __ballot(w < NWW && kend > T);
                const uint32_t kprev = __shfl_up(kend, 1, 64);
                if (hb) {
                    const uint32_t f = (uint32_t)(__ffsll(hb) - 1);
                    wf = wb + f;
                    ks = f == 0u ? k : __shfl(kprev, f, 64);
                } else {
                    k = __shfl(kend, 63, 64);
                }
#else
                for (uint32_t w = wb; w < wb + 64u && w < NWW; w++) {
                    uint32_t fa[2], fq[2];
                    tie_word(mask[w], w == w0 ? (c & 31u) : 0u, nCol - 32u * w < 32u ? nCol - 32u * w : 32u, dE, tE, dP,
                             tP, fa, fq);
                    const uint32_t kend = k + fa[k & 1u];
                    if (kend > T) {
                        wf = w;
                        ks = k;
                        break;
                    }
                    k = kend;
                }
#endif
            }
            if (wf == NWW) return nCol;   // the rest of the walk stays in the binade at or below u
            const uint32_t word = mask[wf];
            const uint32_t nb = nCol - 32u * wf < 32u ? nCol - 32u * wf : 32u;
            uint32_t kk = ks, y = nCol, kb = ks;
            bool occ = false;
            for (uint32_t b = wf == w0 ? (c & 31u) : 0u; b < nb; b++) {
                occ = (word >> b) & 1u;
                const uint32_t d = occ ? dE : dP, t = occ ? tE : tP;
                kb = kk;
                kk += d + (t & ((kk + d) & 1u));
                if (kk > T) {
                    y = 32u * wf + b;
                    break;
                }
            }
            if (T < 0xFFFFFFu) return y;   // u is in this binade: the sum passes it at y
            cdf = f32_from((E << 23) | (kb & 0x7FFFFFu));   // the sum leaves the binade at y: one fp32 step
            cdf += occ ? eps : pf;
            if (cdf > u) return y;
            c = y + 1u;
            continue;
        }
        if (E == 0u || !binade_inc(eps, E, dE) || !binade_inc(pf, E, dP)) {
            // cdf = 0 or a tying increment: the run of equal addends from c (colours of one kind,
            // across words) by cdf_run, exact step by step where the rounding depends on the sum's
            // parity (a violator with few free colours crosses a tie binade over thousands of
            // occupied ones: colour-by-colour steps cost ~90 us there)
            const uint32_t bit = (mask[c >> 5] >> (c & 31u)) & 1u;
            const uint32_t r = mask_run_len(mask, nCol, c, bit);
            const uint32_t s = cdf_run(cdf, bit ? eps : pf, r, u);
            if (s) return c + s - 1u;
            c += r;
            continue;
        }
        if (dE == 0u && dP == 0u) return nCol;   // every further sum rounds back to cdf (<= u)
        const uint64_t k0 = (bc & 0x7FFFFFu) | 0x800000u;
        const uint64_t T = ((bu >> 23) == E) ? (uint64_t)((bu & 0x7FFFFFu) | 0x800000u) : 0xFFFFFFull;
        const uint32_t w0 = c >> 5;
        const uint32_t occ0 = pre[w0] + (uint32_t)__builtin_popcount(mask[w0] & ((1u << (c & 31u)) - 1u));
        // the mantissa integer after the last colour of word w >= w0 (colours [c, min(32(w+1), nCol)))
        auto kend = [&](uint32_t w) -> uint64_t {
            const uint32_t x = 32u * (w + 1u) < nCol ? 32u * (w + 1u) : nCol;
            const uint32_t occ = pre[w + 1u] - occ0;
            return k0 + (uint64_t)occ * dE + (uint64_t)(x - c - occ) * dP;
        };
        uint32_t wf = NWW;   // the word holding the first colour whose sum passes T
        for (uint32_t wb = w0; wb < NWW; wb += 64u) {
            const int f = first_of_64([&](int l) {
                const uint32_t w = wb + (uint32_t)l;
                return w < NWW && kend(w) > T;
            });
            if (f >= 0) {
                wf = wb + (uint32_t)f;
                break;
            }
        }
        if (wf == NWW) return nCol;   // the rest of the walk stays in the binade at or below u
        const uint32_t b0 = wf == w0 ? (c & 31u) : 0u;
        const uint64_t ks = wf == w0 ? k0 : kend(wf - 1u);   // before colour 32 wf + b0
        const uint32_t word = mask[wf] >> b0;
        const uint32_t nb = (nCol - 32u * wf < 32u ? nCol - 32u * wf : 32u) - b0;
        auto kat = [&](uint32_t i) -> uint64_t {   // after the first i colours from b0
            const uint32_t occ = (uint32_t)__builtin_popcount(i >= 32u ? word : word & ((1u << i) - 1u));
            return ks + (uint64_t)occ * dE + (uint64_t)(i - occ) * dP;
        };
        const int fb = first_of_64([&](int l) { return (uint32_t)l < nb && kat((uint32_t)l + 1u) > T; });
        const uint32_t i = (uint32_t)fb;   // kend(wf) > T, so fb >= 0
        const uint32_t y = 32u * wf + b0 + i;
        if (T < 0xFFFFFFu) return y;   // u is in this binade: the sum passes it at y (in or above the binade)
        const uint64_t kb = kat(i);     // the sum leaves the binade at y: one exact fp32 step
        cdf = f32_from((E << 23) | ((uint32_t)kb & 0x7FFFFFu));
        cdf += ((word >> i) & 1u) ? eps : pf;
        if (cdf > u) return y;
        c = y + 1u;
    }
    return nCol;
}

// walk_own with the table E[k] = fl(...fl(eps + eps)... + eps) (k terms, E[0] = 0): the cdf before
// colour cv is E[cv], so a stop before cv is a binary search and the rest is two steps.
// ecv = E[cv], loaded by the caller (the evaluation issues it with its other loads).
MCMC_HD uint32_t walk_own_tab_e(const float* E, float ecv, uint32_t nCol, uint32_t cv, float eps, float hi, float u) {
    if (!(eps > 0.0f)) return walk_own(nCol, cv, eps, hi, u);   // E is monotone only for eps > 0
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

MCMC_HD uint32_t walk_own_tab(const float* E, uint32_t nCol, uint32_t cv, float eps, float hi, float u) {
    return walk_own_tab_e(E, eps > 0.0f ? E[cv] : 0.0f, nCol, cv, eps, hi, u);
}

// The table of walk_own_tab, host side (nCol + 1 entries).
inline void eps_table(float eps, uint32_t nCol, float* E) {
    E[0] = 0.0f;
    for (uint32_t k = 1; k <= nCol; k++) E[k] = E[k - 1] + eps;
}

}  // namespace mcmc
