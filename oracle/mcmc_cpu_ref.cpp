// oracle/mcmc_cpu_ref.cpp -- TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline).
// See mcmc_cpu_ref.h for scope and the rule that the product never links this file.
//
// Every function cites the reference lines (paths relative to /root/reference/src) it restates.
// Compile with -O2 -ffp-contract=off: the reference host code is plain x86-64 SSE float
// arithmetic with no FMA contraction, and parity is bit-exact.
#include "mcmc_cpu_ref.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <numeric>
#include <random>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

// ---------------------------------------------------------------------------------------------
// Minimal CSR view. The reference GraphStruct (graph/graph.h:37-79) uses uint32 cumulDegs; the
// oracle widens offsets to uint64 so the same code runs on graphs with more than 2^32 arcs.
struct CSR {
    uint32_t        nNodes;
    const uint64_t* cumulDegs;
    const uint32_t* neighs;
};

// minstd_rand0 skip-ahead, used only by the OpenMP variant to split the per-sweep bulk draw
// (coloringMCMC_CPU.cpp:139) across threads. Pinned against std::minstd_rand0 by tests.
constexpr uint64_t kM = 2147483647ull;
constexpr uint64_t kA = 16807ull;
inline uint64_t mulmod(uint64_t a, uint64_t b) { return (a * b) % kM; }
inline uint64_t powmod(uint64_t a, uint64_t e) {
    uint64_t r = 1;
    while (e) { if (e & 1) r = mulmod(r, a); a = mulmod(a, a); e >>= 1; }
    return r;
}
// generate_canonical<float,24> over minstd (libstdc++ random.tcc:3348-3380): one engine call,
// float(x - 1) / float(2147483646.0L) == float(x - 1) / 2^31, clamped to nextafter(1, 0).
inline float canonical_from_state(uint64_t x) {
    float r = static_cast<float>(x - 1) / 2147483648.0f;
    if (r >= 1.0f) r = std::nextafter(1.0f, 0.0f);
    return r;
}

// ---------------------------------------------------------------------------------------------
// Restatement of ColoringMCMC_CPU (graph_coloring/coloringMCMC_CPU.h:12-108).
class ColoringMCMC_CPU {
public:
    ColoringMCMC_CPU(const CSR& g, const oracle_params& params, uint32_t seed)
        // ctor: coloringMCMC_CPU.cpp:7-98
        : str(g), nNodes(g.nNodes), seed(seed), nCol(params.nCol), epsilon(params.epsilon),
          tabooIteration(params.tabooIteration), iter(0), maxiter(params.maxRip), maxIterReached(false) {
        C = std::vector<uint32_t>(nNodes);
        Cstar = std::vector<uint32_t>(nNodes);
        q = std::vector<float>(nNodes);
        qstar = std::vector<float>(nNodes);
        p = std::vector<float>(nCol);
        nodeProbab = std::vector<float>(nNodes);
        freeColors = std::vector<bool>(nCol);
        Cviols = std::vector<bool>(nNodes);
        Cstarviols = std::vector<bool>(nNodes);
        colorIdx = std::vector<size_t>(nCol);
        taboo = std::vector<uint32_t>(nNodes, 0);
        // :53-55  engine + distributions
        gen = std::default_random_engine(seed);
        unifInitColors = std::uniform_int_distribution<uint32_t>(0, nCol - 1);
        unifDistr = std::uniform_real_distribution<float>(0, 1);
        // :61  baseline random coloration, one uniform_int draw per node in node order
        countingDraws = 0;
        for (auto& val : C) val = unifInitColors(gen);
        // :89-97 tail cutting threshold
        if (params.tailcut) z = (50 > nNodes / 2000) ? 50 : (nNodes / 2000);
        else z = 0;
    }

    // violation_count (coloringMCMC_CPU.cpp:328-351): vertices with >= 1 same-colored neighbour.
    size_t violation_count(const std::vector<uint32_t>& currentColoring, std::vector<bool>& violations) {
        size_t viol = 0;
        for (size_t i = 0; i < nNodes; i++) {
            violations[i] = 0;
            const uint32_t nodeColor = currentColoring[i];
            const uint32_t* b = str.neighs + str.cumulDegs[i];
            const uint32_t* e = str.neighs + str.cumulDegs[i + 1];
            size_t nodeViolations = std::count_if(b, e, [&](uint32_t w) { return nodeColor == currentColoring[w]; });
            if (nodeViolations > 0) { violations[i] = 1; viol++; }
        }
        return viol;
    }

    // count_free_colors (coloringMCMC_CPU.cpp:361-383)
    size_t count_free_colors(size_t currentNode, const std::vector<uint32_t>& currentColoring,
                             std::vector<bool>& fc) const {
        std::fill(fc.begin(), fc.end(), 1);
        const uint32_t* b = str.neighs + str.cumulDegs[currentNode];
        const uint32_t* e = str.neighs + str.cumulDegs[currentNode + 1];
        for (const uint32_t* it = b; it != e; ++it) fc[currentColoring[*it]] = 0;
        return std::count(fc.begin(), fc.end(), 1);
    }

    // fill_p (coloringMCMC_CPU.cpp:392-481), "Baseline" variant; colorIdx is the identity (:131-132).
    void fill_p(size_t currentNode, size_t Zv, const std::vector<bool>& fc, std::vector<float>& pv) const {
        size_t idx = 0;
        const size_t Zvcomp = nCol - Zv;
        const uint32_t currentColor = C[currentNode];
        if (Cviols[currentNode] == 1) {
            auto nFreeColors = std::accumulate(fc.begin(), fc.end(), 0);
            if (nFreeColors == 0) {
                for (auto& val : pv) { val = (idx == currentColor) ? 1.0f - (nCol - 1) * epsilon : epsilon; idx++; }
                return;
            }
            for (auto& val : pv) { val = fc[idx] ? (1.0f - epsilon * Zv) / (float)Zvcomp : epsilon; idx++; }
        } else {
            for (auto& val : pv) { val = (colorIdx[idx] == currentColor) ? 1.0f - (nCol - 1) * epsilon : epsilon; idx++; }
        }
    }

    // extract_new_color (coloringMCMC_CPU.cpp:492-528). Returns true when the CDF never exceeded
    // the threshold (the "fix for overflowing" branch, :516-520). In the single-thread variant the
    // glibc draw is taken right here, in vertex order, exactly like the reference.
    bool extract_new_color(size_t currentNode, const std::vector<float>& pVect, bool drawNow) {
        if (taboo[currentNode] > 0) {                                // :496-501
            taboo[currentNode]--;
            Cstar[currentNode] = C[currentNode];
            q[currentNode] = (1.0f - (nCol - 1) * epsilon);
            return false;
        }
        float experimentThrsh = nodeProbab[currentNode];
        float cdf = 0;
        size_t idx;
        for (idx = 0; idx < pVect.size(); idx++) {                   // :510-514 (strict >)
            cdf += pVect[idx];
            if (cdf > experimentThrsh) break;
        }
        bool overflow = false;
        if (idx >= nCol) {                                           // :517-520
            overflow = true;
            if (!drawNow) return true;                               // OpenMP variant: replay later
            idx = rand() % (nCol - 1);
            glibcDraws++;
        }
        q[currentNode] = pVect[idx];
        Cstar[currentNode] = idx;
        taboo[currentNode] = (Cstar[currentNode] == C[currentNode]) * tabooIteration;   // :526
        return overflow;
    }

    // fill_qstar (coloringMCMC_CPU.cpp:531-551): output-dead in the reference, kept for its cost.
    void fill_qstar(size_t currentNode, size_t Zv, const std::vector<bool>& fc) {
        const size_t Zvcomp = nCol - Zv;
        const uint32_t currentColor = Cstar[currentNode];
        if (Cstarviols[currentNode] == 1) {
            qstar[currentNode] = fc[currentColor] ? (1.0f - epsilon * Zv) / (float)Zvcomp : epsilon;
        } else {
            qstar[currentNode] = (Cstar[currentNode] == C[currentNode]) ? 1.0f - (nCol - 1) * epsilon : epsilon;
        }
    }

    // run() (coloringMCMC_CPU.cpp:115-321). The per-sweep debugger hook (:244, two
    // system("stty") fork/execs) is excluded from the loop, as SURVEY.md §8d prescribes.
    void run(std::vector<uint64_t>& traj, uint32_t sweepLimit, int nthreads, int tailcutRepair) {
        Cviol = violation_count(C, Cviols);                          // :127
        size_t ii = 0;
        for (auto& v : colorIdx) v = ii++;                           // :131-132
        auto t0 = std::chrono::steady_clock::now();
        while (Cviol > z) {                                          // :136
            if (sweepLimit && sweepsRun >= sweepLimit) break;
            if (nthreads <= 1) sweep_serial(traj);
            else sweep_parallel(traj, nthreads);
            sweepsRun++;
            std::swap(C, Cstar);                                     // :259-260
            std::swap(Cviol, Cstarviol);
            iter++;                                                  // :264-269
            if (iter > maxiter) { maxIterReached = true; break; }
        }
        auto t1 = std::chrono::steady_clock::now();
        loopSeconds = std::chrono::duration<double>(t1 - t0).count();
        traj.push_back(Cviol);
        if (tailcutRepair) tail_cut();
    }

    void sweep_serial(std::vector<uint64_t>& traj) {
        for (auto& val : nodeProbab) val = unifDistr(gen);           // :139
        Cviol = violation_count(C, Cviols);                          // :152
        traj.push_back(Cviol);
        for (size_t i = 0; i < nNodes; i++) {                        // :183-204
            size_t Zvcomp = count_free_colors(i, C, freeColors);
            size_t Zv = nCol - Zvcomp;
            fill_p(i, Zv, freeColors, p);
            extract_new_color(i, p, true);
        }
        Cstarviol = violation_count(Cstar, Cstarviols);              // :211
        for (size_t i = 0; i < nNodes; i++) {                        // :218-230
            size_t Zvcomp = count_free_colors(i, Cstar, freeColors);
            fill_qstar(i, nCol - Zvcomp, freeColors);
        }
    }

    // OpenMP variant: the same Jacobi sweep split over threads. Bit-identical because every vertex
    // reads only C, its own u and its own taboo; overflow events are replayed afterwards in
    // ascending vertex order (the order loop 1 would have drawn them in).
    void sweep_parallel(std::vector<uint64_t>& traj, int nthreads) {
#ifdef _OPENMP
        // Bulk draw of n floats (:139) split by minstd skip-ahead from the current engine state.
        const uint64_t x0 = gen();                                   // draw #1 of this sweep
        const uint64_t n = nNodes;
        #pragma omp parallel for num_threads(nthreads) schedule(static)
        for (int64_t t = 0; t < nthreads; t++) {
            uint64_t a = n * t / nthreads, b = n * (t + 1) / nthreads;
            if (a >= b) continue;
            uint64_t x = mulmod(x0, powmod(kA, a));
            for (uint64_t v = a; v < b; v++) { nodeProbab[v] = canonical_from_state(x); x = mulmod(x, kA); }
        }
        gen.seed(mulmod(x0, powmod(kA, n - 1)));                     // engine now n draws further
        size_t viol = 0;
        #pragma omp parallel for num_threads(nthreads) schedule(static) reduction(+ : viol)
        for (int64_t i = 0; i < (int64_t)nNodes; i++) {
            const uint32_t c = C[i];
            bool v = false;
            for (uint64_t k = str.cumulDegs[i]; k < str.cumulDegs[i + 1]; k++)
                if (C[str.neighs[k]] == c) { v = true; break; }
            viol += v;
            violflag[i] = v;
        }
        for (size_t i = 0; i < nNodes; i++) Cviols[i] = violflag[i];
        Cviol = viol;
        traj.push_back(Cviol);
        std::vector<std::vector<uint32_t>> ev(nthreads);
        #pragma omp parallel num_threads(nthreads)
        {
            int tid = omp_get_thread_num();
            std::vector<bool> fc(nCol);
            std::vector<float> pv(nCol);
            #pragma omp for schedule(static)
            for (int64_t i = 0; i < (int64_t)nNodes; i++) {
                size_t Zvcomp = count_free_colors(i, C, fc);
                fill_p(i, nCol - Zvcomp, fc, pv);
                if (extract_new_color(i, pv, false)) ev[tid].push_back((uint32_t)i);
            }
        }
        for (auto& list : ev)                                        // ascending: static schedule
            for (uint32_t i : list) {
                uint32_t idx = rand() % (nCol - 1);
                glibcDraws++;
                Cstar[i] = idx;
                taboo[i] = (Cstar[i] == C[i]) * tabooIteration;
            }
        size_t sviol = 0;
        #pragma omp parallel for num_threads(nthreads) schedule(static) reduction(+ : sviol)
        for (int64_t i = 0; i < (int64_t)nNodes; i++) {
            const uint32_t c = Cstar[i];
            bool v = false;
            for (uint64_t k = str.cumulDegs[i]; k < str.cumulDegs[i + 1]; k++)
                if (Cstar[str.neighs[k]] == c) { v = true; break; }
            sviol += v;
            violflag[i] = v;
        }
        for (size_t i = 0; i < nNodes; i++) Cstarviols[i] = violflag[i];
        Cstarviol = sviol;
        // loop 2 (fill_qstar) is output-dead; the OpenMP baseline skips it (documented).
#else
        (void)nthreads;
        sweep_serial(traj);
#endif
    }

    // Tail cutting (coloringMCMC_CPU.cpp:272-311) with the k++ fix and a pass bound.
    void tail_cut() {
        std::vector<size_t> histBins(nCol);
        if (z > 0) {                                                 // :272-278
            std::fill(histBins.begin(), histBins.end(), 0);
            size_t ii = 0;
            for (auto& v : colorIdx) v = ii++;
            for (uint32_t val : C) histBins[val]++;
            std::sort(colorIdx.begin(), colorIdx.end(), [&](int i, int j) { return histBins[i] < histBins[j]; });
        }
        while (Cviol > 0 && tailcutPasses < 1000) {                 // :281-311
            for (size_t i = 0; i < nNodes; i++) {
                if (Cviols[i]) {
                    std::fill(freeColors.begin(), freeColors.end(), 1);
                    for (uint64_t k = str.cumulDegs[i]; k < str.cumulDegs[i + 1]; k++)
                        freeColors[C[str.neighs[k]]] = 0;
                    for (size_t j = 0; j < nCol; j++)
                        if (freeColors[colorIdx[j]]) { C[i] = colorIdx[j]; break; }
                }
            }
            Cviol = violation_count(C, Cviols);
            tailcutPasses++;
        }
    }

    CSR str;
    size_t nNodes;
    uint32_t seed;
    uint32_t nCol;
    float epsilon;
    uint32_t tabooIteration;
    uint32_t z = 0;
    size_t iter;
    size_t maxiter;
    bool maxIterReached;
    size_t Cviol = 0, Cstarviol = 0;
    std::vector<uint32_t> C, Cstar, taboo;
    std::vector<float> p, q, qstar, nodeProbab;
    std::vector<bool> freeColors, Cviols, Cstarviols;
    std::vector<uint8_t> violflag;
    std::vector<size_t> colorIdx;
    std::default_random_engine gen;
    std::uniform_int_distribution<uint32_t> unifInitColors;
    std::uniform_real_distribution<float> unifDistr;
    uint64_t countingDraws = 0;
    uint64_t glibcDraws = 0;
    double loopSeconds = 0;
    uint32_t sweepsRun = 0;
    uint32_t tailcutPasses = 0;
};

// Counts the engine draws the uniform_int initial coloring consumed, by replaying it on a copy.
uint64_t count_init_draws(uint32_t seed, uint32_t nCol, uint64_t n) {
    std::default_random_engine g(seed);
    const uint64_t urange = 2147483645ull, uerange = (uint64_t)(nCol - 1) + 1;
    const uint64_t scaling = urange / uerange, past = uerange * scaling;
    uint64_t draws = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t r;
        do { r = g() - 1; draws++; } while (r >= past);
    }
    return draws;
}

}  // namespace

extern "C" {

void oracle_srand(uint32_t seed) { srand(seed); }
int32_t oracle_rand(void) { return rand(); }
void oracle_rand_skip(uint64_t k) { for (uint64_t i = 0; i < k; i++) (void)rand(); }
void oracle_free(void* p) { free(p); }

// glibc stdlib/random.c + random_r.c: initstate(seed, buf, 128) selects TYPE_3, keeps buf as the
// live state (state = buf + 1) and leaves fptr = &state[3], rptr = &state[0] after its 310
// discards (310 = 10 * 31). The next output is (state[3] + state[0]) >> 1 stored at state[3]:
// oldest word at state[3], ring order state[3..30], state[0..2].
static int32_t g_glibc_buf[32];
void oracle_set_glibc_window(const uint32_t window[31]) {
    initstate(1, (char*)g_glibc_buf, sizeof(g_glibc_buf));
    int32_t* state = g_glibc_buf + 1;
    for (int k = 0; k < 28; k++) state[3 + k] = (int32_t)window[k];
    for (int k = 0; k < 3; k++) state[k] = (int32_t)window[28 + k];
}

void oracle_minstd_seq(uint32_t seed, uint64_t count, uint32_t* out) {
    std::minstd_rand0 g(seed);
    for (uint64_t i = 0; i < count; i++) out[i] = (uint32_t)g();
}

void oracle_canonical_seq(uint32_t seed, uint64_t skip, uint64_t count, float* out) {
    std::default_random_engine g(seed);
    g.discard(skip);
    std::uniform_real_distribution<float> d(0, 1);
    for (uint64_t i = 0; i < count; i++) out[i] = d(g);
}

uint64_t oracle_uniform_int_seq(uint32_t seed, uint32_t nCol, uint64_t count, uint32_t* out) {
    std::default_random_engine g(seed);
    std::uniform_int_distribution<uint32_t> d(0, nCol - 1);
    for (uint64_t i = 0; i < count; i++) out[i] = d(g);
    return count_init_draws(seed, nCol, count);
}

// Graph::setupRnd2 (graph/graphCPU.cpp:291-404). Upper triangle including the diagonal, row-major,
// bit k set iff (double)rand()/RAND_MAX < prob (float prob promoted to double, :441); diagonal
// cleared in the degree pass (:333-335); neighbour lists come out ascending.
int oracle_setup_rnd2(uint32_t n, float prob, uint64_t** row_off, uint32_t** col_idx, uint64_t* m) {
    const size_t nn = n;
    const size_t vecSize = nn * (nn + 1) / 2;
    std::vector<bool> boolGraph(vecSize);
    for (size_t i = 0; i < vecSize; i++) boolGraph[i] = ((double)rand() / (RAND_MAX)) >= prob ? 0 : 1;
    uint64_t* cumulDegs = (uint64_t*)calloc(nn + 1, sizeof(uint64_t));
    if (!cumulDegs) return -1;
    uint64_t nEdges = 0;
    size_t i = 0, j = 0;
    for (size_t k = 0; k < vecSize; k++) {
        if (j == i) boolGraph[k] = 0;
        if (boolGraph[k]) { cumulDegs[i + 1]++; cumulDegs[j + 1]++; nEdges += 2; }
        i++;
        if (i == nn) { j++; i = j; }
    }
    for (size_t v = 1; v < nn + 1; v++) cumulDegs[v] += cumulDegs[v - 1];
    uint32_t* neighs = (uint32_t*)malloc(std::max<uint64_t>(nEdges, 1) * sizeof(uint32_t));
    if (!neighs) { free(cumulDegs); return -1; }
    std::vector<uint64_t> tempDegs(nn, 0);
    i = j = 0;
    for (size_t k = 0; k < vecSize; k++) {
        if (boolGraph[k]) {
            neighs[cumulDegs[j] + tempDegs[j]++] = (uint32_t)i;
            neighs[cumulDegs[i] + tempDegs[i]++] = (uint32_t)j;
        }
        i++;
        if (i == nn) { j++; i = j; }
    }
    *row_off = cumulDegs;
    *col_idx = neighs;
    *m = nEdges;
    return 0;
}

// ---- the build's counter-based G(n, p) (er_gen.h definition, restated) ----------------------------
namespace {

void philox10(uint32_t ctr[4], uint32_t key0, uint32_t key1) {
    const uint32_t M[2] = {0xD2511F53u, 0xCD9E8D57u};
    uint32_t k[2] = {key0, key1};
    for (int round = 0; round < 10; round++) {
        const uint64_t p0 = (uint64_t)M[0] * ctr[0];
        const uint64_t p1 = (uint64_t)M[1] * ctr[2];
        const uint32_t out[4] = {(uint32_t)(p1 >> 32) ^ ctr[1] ^ k[0], (uint32_t)p1,
                                 (uint32_t)(p0 >> 32) ^ ctr[3] ^ k[1], (uint32_t)p0};
        for (int q = 0; q < 4; q++) ctr[q] = out[q];
        k[0] += 0x9E3779B9u;
        k[1] += 0xBB67AE85u;
    }
}

// ln(u), u in (0, 1]: u = m 2^e, m in [sqrt(1/2), sqrt(2)), ln m = 2 s (1 + s^2/3 + ... + s^24/25).
double series_log(double u) {
    uint64_t bits;
    std::memcpy(&bits, &u, 8);
    int e = (int)((bits >> 52) & 0x7FF) - 1023;
    bits = (bits & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull;
    double m;
    std::memcpy(&m, &bits, 8);
    if (m > 1.4142135623730951) { m = m * 0.5; e += 1; }
    const double s = (m - 1.0) / (m + 1.0), s2 = s * s;
    double poly = 1.0 / 25.0;
    for (int k = 11; k >= 0; k--) poly = poly * s2 + 1.0 / (double)(2 * k + 1);
    return ((double)e * 6.93147180369123816490e-01 + 2.0 * s * poly) + (double)e * 1.90821492927058770002e-10;
}

}  // namespace

// Stream (i, Y) of the definition: calls emit(j) for every present column j of block Y, j > i.
}  // extern "C"
namespace {
template <class Emit>
void er_walk_stream(uint32_t n, int mode, double inv, uint64_t seed, uint32_t i, uint32_t Y, Emit&& emit) {
    const uint32_t T = 65536;
    const uint64_t end = std::min<uint64_t>(n, (uint64_t)(Y + 1) * T);
    uint64_t j = std::max<uint64_t>((uint64_t)Y * T, (uint64_t)i + 1);
    if (j >= end || mode == 2) return;
    if (mode == 1) {
        for (; j < end; j++) emit((uint32_t)j);
        return;
    }
    j -= 1;
    for (uint32_t k = 0;; k++) {
        uint32_t c[4] = {k, i, Y, 0x45524721u};
        philox10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
        for (int q = 0; q < 4; q++) {
            const double t = series_log(((double)c[q] + 1.0) * 2.3283064365386963e-10) * inv;
            const uint64_t skip = (t < 2147483647.0) ? 1u + (uint32_t)t : 0x7FFFFFFFu;
            j += skip;
            if (j >= end) return;
            emit((uint32_t)j);
        }
    }
}

struct ErConst {
    int mode;
    double inv;
};
ErConst er_const(double prob) {
    const double p = (double)(float)prob;
    const int mode = p >= 1.0 ? 1 : (p <= 0.0 ? 2 : 0);
    return ErConst{mode, mode == 0 ? 1.0 / std::log1p(-p) : 0.0};
}
}  // namespace
extern "C" {

int oracle_er_fast(uint32_t n, double prob, uint64_t seed, uint64_t** row_off, uint32_t** col_idx, uint64_t* m) {
    const ErConst ec = er_const(prob);
    const uint32_t T = 65536, nb = (uint32_t)(((uint64_t)n + T - 1) / T);
    std::vector<std::pair<uint32_t, uint32_t>> edges;
    for (uint32_t i = 0; i < n && ec.mode != 2; i++)
        for (uint32_t Y = i / T; Y < nb; Y++)
            er_walk_stream(n, ec.mode, ec.inv, seed, i, Y, [&](uint32_t j) { edges.emplace_back(i, j); });
    uint64_t* off = (uint64_t*)calloc((size_t)n + 1, sizeof(uint64_t));
    if (!off) return -1;
    for (auto& e : edges) { off[e.first + 1]++; off[e.second + 1]++; }
    for (uint32_t v = 0; v < n; v++) off[v + 1] += off[v];
    uint32_t* idx = (uint32_t*)malloc(std::max<uint64_t>(off[n], 1) * sizeof(uint32_t));
    if (!idx) { free(off); return -1; }
    std::vector<uint64_t> cur(off, off + n);
    for (auto& e : edges) { idx[cur[e.first]++] = e.second; idx[cur[e.second]++] = e.first; }
    for (uint32_t v = 0; v < n; v++) std::sort(idx + off[v], idx + off[v + 1]);
    *row_off = off;
    *col_idx = idx;
    *m = off[n];
    return 0;
}

// Neighbour lists of selected rows of the same G(n, p), without enumerating the whole graph (the
// C3 graph has 1e11 arcs): row v's arcs are its own streams (v, Y), Y >= v's block (j > v), plus
// every i < v whose stream (i, block(v)) emits v -- all streams (i, X) into the sampled rows' blocks
// X are walked once (OpenMP over i). *row_off[k + 1], *col_idx: rows in the given order, each
// ascending. Allocates like oracle_er_fast.
int oracle_er_rows(uint32_t n, double prob, uint64_t seed, const uint32_t* rows, uint32_t k, int nthreads,
                   uint64_t** row_off, uint32_t** col_idx) {
    const ErConst ec = er_const(prob);
    const uint32_t T = 65536, nb = (uint32_t)(((uint64_t)n + T - 1) / T);
    std::vector<std::vector<uint32_t>> adj(k);
    for (uint32_t s = 0; s < k; s++) {
        if (rows[s] >= n) return -1;
        for (uint32_t Y = rows[s] / T; Y < nb; Y++)
            er_walk_stream(n, ec.mode, ec.inv, seed, rows[s], Y, [&](uint32_t j) { adj[s].push_back(j); });
    }
    std::vector<uint32_t> blocks;
    for (uint32_t s = 0; s < k; s++) blocks.push_back(rows[s] / T);
    std::sort(blocks.begin(), blocks.end());
    blocks.erase(std::unique(blocks.begin(), blocks.end()), blocks.end());
    for (uint32_t X : blocks) {
        std::vector<int32_t> slot(T, -1);   // block-local column -> sampled row
        for (uint32_t s = 0; s < k; s++)
            if (rows[s] / T == X) slot[rows[s] - X * T] = (int32_t)s;
        const uint32_t iend = (uint32_t)std::min<uint64_t>(n, (uint64_t)(X + 1) * T);
        std::vector<std::vector<std::pair<uint32_t, uint32_t>>> found(std::max(nthreads, 1));
#ifdef _OPENMP
        #pragma omp parallel for num_threads(std::max(nthreads, 1)) schedule(dynamic, 4096)
#endif
        for (int64_t ii = 0; ii < (int64_t)iend; ii++) {
            int tid = 0;
#ifdef _OPENMP
            tid = omp_get_thread_num();
#endif
            const uint32_t i = (uint32_t)ii;
            er_walk_stream(n, ec.mode, ec.inv, seed, i, X, [&](uint32_t j) {
                const int32_t s = slot[j - X * T];
                if (s >= 0) found[tid].emplace_back((uint32_t)s, i);
            });
        }
        for (auto& f : found)
            for (auto& e : f) adj[e.first].push_back(e.second);
    }
    uint64_t* off = (uint64_t*)calloc((size_t)k + 1, sizeof(uint64_t));
    if (!off) return -1;
    for (uint32_t s = 0; s < k; s++) off[s + 1] = off[s] + adj[s].size();
    uint32_t* idx = (uint32_t*)malloc(std::max<uint64_t>(off[k], 1) * sizeof(uint32_t));
    if (!idx) { free(off); return -1; }
    for (uint32_t s = 0; s < k; s++) {
        std::sort(adj[s].begin(), adj[s].end());
        std::copy(adj[s].begin(), adj[s].end(), idx + off[s]);
    }
    *row_off = off;
    *col_idx = idx;
    return 0;
}

// u of engine draw number pos[i] (1-based) of std::default_random_engine(seed): the bulk draw of
// coloringMCMC_CPU.cpp:139 gives vertex v of sweep t draw K0 + t n + v + 1. minstd skip-ahead
// x_pos = x_0 16807^pos mod (2^31 - 1), then generate_canonical (canonical_from_state); pinned
// against g.discard() by tests/test_oracle.py.
void oracle_canonical_at(uint32_t seed, const uint64_t* pos, uint64_t k, float* out) {
    uint64_t x0 = (uint64_t)seed % kM;
    if (x0 == 0) x0 = 1;
    for (uint64_t i = 0; i < k; i++) out[i] = canonical_from_state(mulmod(x0, powmod(kA, pos[i])));
}

// u of the k consecutive engine draws start, start + 1, ... of default_random_engine(seed): the bulk
// draw of one sweep (coloringMCMC_CPU.cpp:139), one skip-ahead then sequential minstd steps.
void oracle_canonical_from(uint32_t seed, uint64_t start, uint64_t k, float* out) {
    uint64_t x0 = (uint64_t)seed % kM;
    if (x0 == 0) x0 = 1;
    uint64_t x = k ? mulmod(x0, powmod(kA, start)) : 0;
    for (uint64_t i = 0; i < k; i++) {
        out[i] = canonical_from_state(x);
        x = mulmod(x, kA);
    }
}

// One vertex of loop 1 (coloringMCMC_CPU.cpp:183-204) from its neighbours' colours: violation flag
// (violation_count :329-351: own colour used by a neighbour), count_free_colors (:361-383), fill_p
// (:392-481, colorIdx the identity) and extract_new_color (:492-528, taboo 0). Returns 1 for a CDF
// overflow (the colour then comes from rand(), :516-520; *color untouched), else 0.
int oracle_vertex_update(uint32_t nCol, float epsilon, uint32_t cv, const uint32_t* nbr_colors, uint64_t deg,
                         float u, uint32_t* color, int* viol) {
    std::vector<bool> fc(nCol, true);
    bool v = false;
    for (uint64_t i = 0; i < deg; i++) {
        fc[nbr_colors[i]] = false;
        v = v || nbr_colors[i] == cv;
    }
    *viol = v ? 1 : 0;
    const size_t Zvcomp = std::count(fc.begin(), fc.end(), true);
    const size_t Zv = nCol - Zvcomp;
    std::vector<float> p(nCol);
    for (uint32_t c = 0; c < nCol; c++) {
        if (v) {
            if (Zvcomp == 0) p[c] = (c == cv) ? 1.0f - (nCol - 1) * epsilon : epsilon;
            else p[c] = fc[c] ? (1.0f - epsilon * Zv) / (float)Zvcomp : epsilon;
        } else {
            p[c] = (c == cv) ? 1.0f - (nCol - 1) * epsilon : epsilon;
        }
    }
    float cdf = 0;
    for (uint32_t c = 0; c < nCol; c++) {
        cdf += p[c];
        if (cdf > u) { *color = c; return 0; }
    }
    return 1;
}

// Graph::doStats (graphCPU.cpp:433-450) -> maxDeg, the default nCol (main.cu:162).
uint32_t oracle_max_deg(uint32_t n, const uint64_t* row_off) {
    uint32_t maxDeg = 0;
    for (uint32_t v = 0; v < n; v++) maxDeg = std::max<uint32_t>(maxDeg, (uint32_t)(row_off[v + 1] - row_off[v]));
    return maxDeg;
}

int oracle_mcmc_run(uint32_t n, const uint64_t* row_off, const uint32_t* col_idx, const oracle_params* prm,
                    uint32_t seed, uint32_t* out_init, uint32_t* out_colors, uint64_t* traj, uint64_t traj_cap,
                    uint32_t sweep_limit, int nthreads, oracle_result* res) {
    if (!prm || prm->nCol == 0 || !out_colors || !res) return -1;
    CSR g{n, row_off, col_idx};
    ColoringMCMC_CPU mc(g, *prm, seed);
    mc.violflag.resize(n);
    if (out_init) std::copy(mc.C.begin(), mc.C.end(), out_init);
    std::vector<uint64_t> tr;
    tr.reserve(prm->maxRip + 2);
    mc.run(tr, sweep_limit, nthreads, prm->tailcutRepair);
    std::copy(mc.C.begin(), mc.C.end(), out_colors);
    if (traj) for (uint64_t k = 0; k < std::min<uint64_t>(traj_cap, tr.size()); k++) traj[k] = tr[k];
    res->iter = (uint32_t)mc.iter;
    res->maxIterReached = mc.maxIterReached;
    res->finalViol = mc.Cviol;
    res->trajLen = tr.size();
    res->glibcDraws = mc.glibcDraws;
    res->initDraws = count_init_draws(seed, prm->nCol, n);
    res->loopSeconds = mc.loopSeconds;
    res->sweepsRun = mc.sweepsRun;
    res->tailcutPasses = mc.tailcutPasses;
    return 0;
}

// saveStats / saveColor (graph_coloring/coloringMCMC_CPUutils.cpp:70-109).
int oracle_save_outputs(const char* log_path, const char* colors_path, uint32_t n, uint64_t nEdges, uint32_t maxDeg,
                        uint32_t minDeg, float meanDeg, float prob, uint32_t seed, uint32_t repetition, float duration,
                        const oracle_params* prm, const oracle_result* res, const uint32_t* colors) {
    std::ofstream outFile(log_path);
    if (!outFile) return -1;
    const uint32_t nCol = prm->nCol;
    outFile << "MCMC Colorer - CPU version - Report" << std::endl;
    outFile << "-------------------------------------------" << std::endl;
    outFile << "GRAPH INFO" << std::endl;
    outFile << "Nodes: " << n << " - Edges: " << nEdges << std::endl;
    outFile << "Max deg: " << maxDeg << " - Min deg: " << minDeg << " - Avg deg: " << meanDeg << std::endl;
    outFile << "Edge probability (for randomly generated graphs): " << prob << std::endl;
    outFile << "Seed: " << seed << std::endl;
    outFile << "-------------------------------------------" << std::endl;
    outFile << "EXECUTION INFO" << std::endl;
    outFile << "Repetition: " << repetition << std::endl;
    outFile << "Execution time: " << duration << std::endl;
    outFile << "Iteration performed: " << res->iter << std::endl;
    outFile << "Max iteration reached: " << (res->maxIterReached ? "yes" : "no") << std::endl;
    outFile << "-------------------------------------------" << std::endl;
    outFile << "Color histogram:" << std::endl;
    std::vector<size_t> histBins(nCol, 0);
    for (uint32_t v = 0; v < n; v++) histBins[colors[v]]++;
    size_t usedCols = 0;
    for (size_t idx = 0; idx < nCol; idx++) { outFile << idx << ": " << histBins[idx] << std::endl; if (histBins[idx]) usedCols++; }
    outFile << "Number of colors: " << nCol << " - Used colors: " << usedCols << std::endl;
    outFile << "Color ratio: " << prm->numColorRatio << std::endl;
    float mean = std::accumulate(histBins.begin(), histBins.end(), 0) / (float)nCol;
    float variance = 0;
    for (size_t val : histBins) variance += ((val - mean) * (val - mean));
    variance /= (float)nCol;
    float sd = sqrtf(variance);
    outFile << "Average number of nodes for each color: " << mean << std::endl;
    outFile << "Variance: " << variance << std::endl;
    outFile << "StD: " << sd << std::endl;
    std::ofstream cf(colors_path);
    if (!cf) return -1;
    for (uint32_t v = 0; v < n; v++) cf << v << " " << colors[v] << std::endl;
    return 0;
}

}  // extern "C"
