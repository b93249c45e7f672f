// oracle/mcmc_gpu_ref.cpp -- TEST INFRASTRUCTURE ONLY (parity oracle).
//
// Sequential restatement of the reference's GPU colorer as compiled by default -- ColoringMCMC with
// COLOR_BALANCE_DYNAMIC_DISTR, STANDARD_INIT and TABOO (graph_coloring/coloringMCMC.h:22-41) --
// the build's "reference-GPU-semantics mode" (SURVEY.md §8f row 2). Written from the source text:
//   coloringMCMC_main.cu:101-298       run(): init, the do/while loop, the tail cut
//   coloringMCMC_balance.cu:79-143     selectStarColoringBalanceDynamic (one thread per vertex)
//   coloringMCMC_utils.cu:24-33        initColoring;  :64-70 genDynamicDistribution
//   coloringMCMC_utils.cu:73-119       tailCutting (one thread) and conflictCounter (edge counts)
//   coloringMCMC_utils.cu:184-198      calcConflicts (sum of the per-vertex edge counts)
//   GPUutils/GPURandomizer.cu:8-13     curand_init(seed, tid, 0) per vertex
// Every thread of the reference kernels touches only its own vertex's outputs and state, so a
// loop over the vertices in any order is the same computation.
//
// Literal details kept: the star buffer of a taboo'd vertex is NOT written (it keeps the value of
// two sweeps before, the reference's pointer swap); Zp == 0 draws nothing; the proposal walk stops
// at threshold >= u (do/while with `threshold < randnum`); 1 - (nCol-1)*eps is fused
// (nvcc contracts a - b*c by default); the host's conflictCounter after the loop is the count of
// the colouring BEFORE the last sweep when the loop ran out of iterations (:163, :229, :279).
// Deviation (documented): a colour equal to nCol (initColoring when u == 1.0f, p ~ 3e-8)
// makes the reference write colorsChecker one slot past the vertex's row, into the next vertex's
// row -- a data race in the parallel sweep; here a colour >= nCol occupies nothing.
//
// XORWOW (cuRAND): salts and the uniform map from cuRAND's published header, the transition and
// the 2^67 subsequence jump from Marsaglia/cuRAND; this file's jump is written independently of
// the product's (row-major GF(2) matrices here, column-major there), and tests pin both against
// rocRAND's engine (same transition and jump, other salts).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#include "mcmc_cpu_ref.h"

namespace {

struct Xw {
    uint32_t v[5];
    uint32_t d;
};

inline uint32_t xw_next(Xw& s) {
    const uint32_t t = s.v[0] ^ (s.v[0] >> 2);
    for (int i = 0; i < 4; i++) s.v[i] = s.v[i + 1];
    s.v[4] = (s.v[4] ^ (s.v[4] << 4)) ^ (t ^ (t << 1));
    s.d += 362437u;
    return s.v[4] + s.d;
}

inline float xw_uniform(uint32_t x) {
    // CURAND_2POW32_INV = 2^-32; x * 2^-32 + 2^-33 (the product is exact)
    const float a = (float)x * 2.3283064365386963e-10f;
    return a + 1.16415321826934814453125e-10f;
}

// 160 x 160 GF(2) matrices, row-major: row r = 5 words, bit c set when output bit r depends on
// input bit c. Bit b of word w is state bit 32w + b.
struct Mat {
    uint32_t r[160][5];
};

void mat_mul(const Mat& A, const Mat& B, Mat& out) {   // out = A * B
    Mat t;
    for (int i = 0; i < 160; i++) {
        uint32_t acc[5] = {0, 0, 0, 0, 0};
        for (int k = 0; k < 160; k++)
            if ((A.r[i][k >> 5] >> (k & 31)) & 1u)
                for (int w = 0; w < 5; w++) acc[w] ^= B.r[k][w];
        std::memcpy(t.r[i], acc, sizeof(acc));
    }
    out = t;
}

void mat_apply(const Mat& A, uint32_t v[5]) {
    uint32_t out[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < 160; i++) {
        uint32_t par = 0;
        for (int w = 0; w < 5; w++) par ^= A.r[i][w] & v[w];
        if (__builtin_popcount(par) & 1) out[i >> 5] |= 1u << (i & 31);
    }
    std::memcpy(v, out, sizeof(out));
}

// P[k] = A^(2^(67+k)), k = 0..31.
const std::vector<Mat>& seq_jumps() {
    static std::vector<Mat> P;
    static std::once_flag once;
    std::call_once(once, [] {
        Mat A;
        std::memset(&A, 0, sizeof(A));
        // one step as rows: out v0..v3 = in v1..v4; out v4 = v4 ^ v4<<4 ^ t ^ t<<1, t = v0 ^ v0>>2
        for (int i = 0; i < 128; i++) A.r[i][(i + 32) >> 5] |= 1u << ((i + 32) & 31);
        for (int b = 0; b < 32; b++) {
            uint32_t* row = A.r[128 + b];
            auto set = [&](int bit) { row[bit >> 5] ^= 1u << (bit & 31); };
            set(128 + b);                       // v4
            if (b >= 4) set(128 + b - 4);       // v4 << 4
            // t bit j = v0[j] ^ v0[j+2];  out gets t[b] ^ t[b-1]
            set(b);
            if (b + 2 < 32) set(b + 2);
            if (b >= 1) {
                set(b - 1);
                if (b + 1 < 32) set(b + 1);
            }
        }
        Mat J = A;
        for (int s = 0; s < 67; s++) mat_mul(J, J, J);
        P.resize(32);
        P[0] = J;
        for (int k = 1; k < 32; k++) mat_mul(P[k - 1], P[k - 1], P[k]);
    });
    return P;
}

Xw xw_init(uint64_t seed, uint64_t sub, int flavor) {
    uint32_t t0, t1;
    if (flavor == 0) {   // cuRAND
        t0 = 1099087573u * ((uint32_t)seed ^ 0xaad26b49u);
        t1 = 2591861531u * ((uint32_t)(seed >> 32) ^ 0xf7dcefddu);
    } else {             // rocRAND (rocrand_xorwow.h:113-122)
        t0 = 1228688033u * ((uint32_t)seed ^ 0x2c7f967fu);
        t1 = 2073658381u * ((uint32_t)(seed >> 32) ^ 0xa03697cbu);
    }
    Xw s;
    s.d = 6615241u + t1 + t0;
    s.v[0] = 123456789u + t0;
    s.v[1] = 362436069u ^ t0;
    s.v[2] = 521288629u + t1;
    s.v[3] = 88675123u ^ t1;
    s.v[4] = 5783321u + t0;
    const auto& P = seq_jumps();
    for (int k = 0; sub && k < 32; k++, sub >>= 1)
        if (sub & 1u) mat_apply(P[k], s.v);
    return s;
}

// conflictCounter kernel (coloringMCMC_utils.cu:103-119): same-colour neighbours with a larger id.
uint32_t edge_conflicts(uint32_t v, const uint64_t* off, const uint32_t* idx, const uint32_t* C) {
    uint32_t c = 0;
    for (uint64_t k = off[v]; k < off[v + 1]; k++) c += (C[idx[k]] == C[v]) && (v < idx[k]);
    return c;
}

uint64_t count_conflicts(uint32_t n, const uint64_t* off, const uint32_t* idx, const uint32_t* C) {
    uint64_t s = 0;
    for (uint32_t v = 0; v < n; v++) s += edge_conflicts(v, off, idx, C);
    return s;
}

}  // namespace

extern "C" {

void oracle_xorwow_init(uint64_t seed, uint64_t subsequence, int flavor, uint32_t out[6]) {
    const Xw s = xw_init(seed, subsequence, flavor);
    std::memcpy(out, s.v, 5 * sizeof(uint32_t));
    out[5] = s.d;
}

void oracle_xorwow_next(uint32_t st[6], uint32_t count, uint32_t* out) {
    Xw s;
    std::memcpy(s.v, st, 5 * sizeof(uint32_t));
    s.d = st[5];
    for (uint32_t i = 0; i < count; i++) out[i] = xw_next(s);
    std::memcpy(st, s.v, 5 * sizeof(uint32_t));
    st[5] = s.d;
}

void oracle_gpurand_init(uint32_t n, uint32_t seed, uint32_t* states) {
    // GPURand(n, seed): initCurand(states, (uint32_t)seed, n) -> curand_init(seed, tid, 0)
    for (uint32_t v = 0; v < n; v++) oracle_xorwow_init(seed, v, 0, states + 6ull * v);
}

int oracle_mcmc_gpu_run(uint32_t n, const uint64_t* off, const uint32_t* idx, const oracle_params* prm,
                        uint32_t* states, uint32_t* out_colors, uint64_t* traj,
                        uint64_t traj_cap, uint32_t tail_max_passes, uint64_t* tail_traj,
                        oracle_gpu_result* res) {
    if (!prm || !states || !out_colors || !res) return -1;
    const uint32_t nCol = prm->nCol;
    const float eps = prm->epsilon;
    if (nCol < 2) return -1;
    std::vector<Xw> S(n);
    for (uint32_t v = 0; v < n; v++) {
        std::memcpy(S[v].v, states + 6ull * v, 5 * sizeof(uint32_t));
        S[v].d = states[6ull * v + 5];
    }
    // coloring_d memset (:107), taboo_d (:110). starColoring_d's initial content is never read: a
    // vertex is first taboo'd at sweep 1, when that buffer holds the initial colouring.
    std::vector<uint32_t> A(n, 0), B(n, 0), taboo(n, 0);
    uint32_t* C = A.data();
    uint32_t* Cs = B.data();
    std::vector<uint32_t> ordered(nCol);
    for (uint32_t i = 0; i < nCol; i++) ordered[i] = i;  // :130-131
    for (uint32_t v = 0; v < n; v++)                      // initColoring (utils.cu:24-33)
        C[v] = (uint32_t)(int)(xw_uniform(xw_next(S[v])) * (float)nCol);
    const uint32_t z = prm->tailcut ? std::max<uint32_t>(50u, n / 2000u) : 0u;   // :150-157
    const float hi = std::fma(-(float)(nCol - 1), eps, 1.0f);
    std::vector<float> p(nCol);
    std::vector<uint32_t> hist(nCol + 1);
    std::vector<uint8_t> chk(nCol);
    uint64_t tl = 0;
    auto push = [&](uint64_t c) { if (traj && tl < traj_cap) traj[tl] = c; tl++; };
    uint32_t rip = 0, sweeps = 0;
    uint64_t conflictCounter = 0;
    bool broke = false;
    do {                                                  // :160-269
        rip++;
        conflictCounter = count_conflicts(n, off, idx, C);
        push(conflictCounter);
        if (conflictCounter <= z) { broke = true; break; }
        std::fill(hist.begin(), hist.end(), 0u);
        for (uint32_t v = 0; v < n; v++) hist[std::min(C[v], nCol)]++;   // :211-214
        for (uint32_t c = 0; c < nCol; c++)                                // genDynamicDistribution
            p[c] = (1 - ((float)hist[c] / (float)n)) / (float)(nCol - 1);
        for (uint32_t v = 0; v < n; v++) {                 // selectStarColoringBalanceDynamic
            if (taboo[v] > 0) { taboo[v]--; continue; }    // star not written
            const uint32_t nodeCol = C[v];
            std::fill(chk.begin(), chk.end(), 0);
            for (uint64_t k = off[v]; k < off[v + 1]; k++)
                if (C[idx[k]] < nCol) chk[C[idx[k]]] = 1;
            float reminder = 0;
            uint32_t Zn = 0;
            for (uint32_t i = 0; i < nCol; i++) {
                Zn += chk[i];
                reminder += (float)chk[i] * (p[ordered[i]] - eps);
            }
            const uint32_t Zp = nCol - Zn;
            if (!Zp) { Cs[v] = nodeCol; continue; }
            const float u = xw_uniform(xw_next(S[v]));
            uint32_t i = 0;
            float thr = 0, q;
            if (nodeCol < nCol && chk[nodeCol]) {
                const float r = reminder / (float)Zp;
                do {
                    q = chk[i] ? eps : (p[ordered[i]] + r);
                    thr += q;
                    i++;
                } while (thr < u && i < nCol);
            } else {
                do {
                    q = (nodeCol == i) ? hi : eps;
                    thr += q;
                    i++;
                } while (thr < u && i < nCol);
            }
            Cs[v] = i - 1;
            taboo[v] = (Cs[v] == nodeCol) * prm->tabooIteration;
        }
        sweeps++;
        std::swap(C, Cs);                                   // :263-265
    } while (rip < prm->maxRip);
    if (!broke) push(count_conflicts(n, off, idx, C));     // the last sweep's "nuovi conflitti"
    res->rip = rip;
    res->maxIterReached = rip == prm->maxRip;               // :294-295
    res->sweeps = sweeps;
    res->conflictCounter = conflictCounter;
    res->trajLen = tl;
    uint32_t passes = 0;
    if (prm->tailcut) {                                     // :271-290
        std::vector<uint32_t> stats(std::max(n, nCol) + 1, 0);
        for (uint32_t v = 0; v < n; v++) stats[C[v]]++;
        for (uint32_t i = 0; i < nCol; i++) ordered[i] = i;
        std::sort(&ordered[0], &ordered[0] + nCol, [&](int i, int j) { return stats[i] < stats[j]; });
        std::vector<uint32_t> cnt(n);
        while (conflictCounter > 0 && passes < tail_max_passes) {
            for (uint32_t v = 0; v < n; v++) cnt[v] = edge_conflicts(v, off, idx, C);
            uint64_t resolved = 0;                          // tailCutting <<<1,1>>>
            for (uint32_t v = 0; v < n && resolved < conflictCounter; v++) {
                if (!cnt[v]) continue;
                resolved++;
                std::fill(chk.begin(), chk.end(), 0);
                for (uint64_t k = off[v]; k < off[v + 1]; k++)
                    if (C[idx[k]] < nCol) chk[C[idx[k]]] = 1;
                uint32_t nodeCol = C[v];
                uint32_t j = 0;
                while (nodeCol < nCol && chk[nodeCol] && j < nCol) { nodeCol = ordered[j]; j++; }
                C[v] = nodeCol;
            }
            conflictCounter = count_conflicts(n, off, idx, C);
            if (tail_traj) tail_traj[passes] = conflictCounter;
            passes++;
        }
    }
    res->tailcutPasses = passes;
    res->finalConflicts = count_conflicts(n, off, idx, C);
    std::memcpy(out_colors, C, sizeof(uint32_t) * n);
    for (uint32_t v = 0; v < n; v++) {
        std::memcpy(states + 6ull * v, S[v].v, 5 * sizeof(uint32_t));
        states[6ull * v + 5] = S[v].d;
    }
    return 0;
}

}  // extern "C"
