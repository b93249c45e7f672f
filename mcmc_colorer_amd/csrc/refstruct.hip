// mcmc_colorer_amd/csrc/refstruct.hip -- "refstruct": the reference CUDA path's per-sweep STRUCTURE
// re-expressed in HIP, as the timing baseline of SURVEY.md §8d ("Reference CUDA path rate for the
// 10x target"; CUDA cannot run on MI355X and no numbers are published). Written from the survey's
// table (rows g1-g5), not hipified, and NOT part of the colouring path: its semantics are the
// reference GPU colorer's (XORWOW draws, edge conflict count, dynamic balance distribution), which
// differ from --mcmccpu by design, so it is timed, never parity-checked.
//
// One sweep, as ColoringMCMC::run with COLOR_BALANCE_DYNAMIC_DISTR (coloringMCMC_main.cu:168-262):
//   calcConflicts(C)      conflictCounter kernel (thread per vertex, serial row walk, 64-thread
//                         blocks) + block sum + D2H of the partials + host sum   (utils.cu:103-198)
//   memset(checker)       n * nCol bytes                                          (main.cu:181)
//   D2H C (4n B), host histogram, H2D of nCol counts                              (main.cu:228-231)
//   genDynamicDistribution (nCol threads)                                         (utils.cu:64-70)
//   selectStarColoringBalanceDynamic: checker scatter per neighbour, nCol scan, one uniform draw,
//                         CDF walk, Cstar/taboo write                             (balance.cu:79-143)
//   calcConflicts(Cstar)  as above                                                (main.cu:246)
//   swap
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <chrono>
#include <vector>

#include "mcmc_common.h"

namespace mcmc {
namespace {

constexpr uint32_t kRefThreads = 64;   // threadsPerBlock of the reference (64-thread blocks)

// curandState-sized per-vertex generator state (48 B: XORWOW words + Box-Muller fields).
struct XorwowState {
    uint32_t d, v[5];
    uint32_t boxmuller_flag, boxmuller_flag_double;
    float boxmuller_extra;
    uint32_t pad;
    double boxmuller_extra_double;
};

__device__ __forceinline__ float xorwow_uniform(XorwowState& s) {
    uint32_t t = s.v[0] ^ (s.v[0] >> 2);
    s.v[0] = s.v[1];
    s.v[1] = s.v[2];
    s.v[2] = s.v[3];
    s.v[3] = s.v[4];
    s.v[4] = (s.v[4] ^ (s.v[4] << 4)) ^ (t ^ (t << 1));
    s.d += 362437u;
    return (float)(s.v[4] + s.d) * 2.3283064e-10f + 1.1641532e-10f;   // (0, 1]
}

__global__ void ref_init_kernel(uint32_t n, uint32_t nCol, uint32_t seed, uint32_t* C, XorwowState* states) {
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    XorwowState s{};
    uint64_t z = ((uint64_t)seed << 32) ^ (0x9E3779B97F4A7C15ull * (v + 1));
    for (int i = 0; i < 5; i++) {
        z ^= z >> 31; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 27;
        s.v[i] = (uint32_t)(z >> 17) | 1u;
    }
    s.d = 6615241u + v;
    states[v] = s;
    C[v] = min((uint32_t)(xorwow_uniform(states[v]) * nCol), nCol - 1);
}

// Monochromatic edges counted once (idx < neighbour), thread per vertex, serial row walk.
__global__ void ref_conflict_kernel(uint32_t n, uint32_t* out, const uint32_t* C, const uint64_t* row_off,
                                    const uint32_t* col_idx) {
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const uint64_t b = row_off[v], e = row_off[v + 1];
    const uint32_t cv = C[v];
    uint32_t k = 0;
    for (uint64_t i = b; i < e; i++) {
        const uint32_t w = col_idx[i];
        k += (C[w] == cv) && (v < w);
    }
    out[v] = k;
}

// Two-per-thread block sum (sumReduction's shape), partials back to the host.
__global__ void ref_sum_kernel(uint32_t n, const uint32_t* in, uint32_t* partial) {
    __shared__ uint32_t s[2 * kRefThreads];
    const uint32_t i = blockIdx.x * 2 * blockDim.x + threadIdx.x;
    uint32_t x = (i < n ? in[i] : 0u) + (i + blockDim.x < n ? in[i + blockDim.x] : 0u);
    s[threadIdx.x] = x;
    __syncthreads();
    for (uint32_t k = blockDim.x / 2; k > 0; k >>= 1) {
        if (threadIdx.x < k) s[threadIdx.x] += s[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = s[0];
}

__global__ void ref_dyn_distribution_kernel(float* p, uint32_t nCol, uint32_t n, const uint32_t* stats) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nCol) return;
    p[c] = (1.0f - (float)stats[c] / (float)n) / (float)(nCol - 1);
}

__global__ void ref_select_kernel(uint32_t n, uint32_t* Cs, float* qs, uint32_t nCol, const uint32_t* C,
                                  const uint64_t* row_off, const uint32_t* col_idx, uint8_t* checker,
                                  uint32_t* taboo, uint32_t tabooIteration, const float* pdyn, XorwowState* states,
                                  float eps) {
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    if (taboo[v] > 0) {
        taboo[v]--;
        qs[v] = 1.0f - (nCol - 1) * eps;
        return;
    }
    const uint64_t b = row_off[v], e = row_off[v + 1];
    const uint32_t cv = C[v];
    uint8_t* chk = checker + (size_t)v * nCol;
    for (uint64_t i = b; i < e; i++) chk[C[col_idx[i]]] = 1;
    float rem = 0.0f;
    uint32_t zn = 0;
    for (uint32_t c = 0; c < nCol; c++) {
        zn += chk[c];
        rem += chk[c] * (pdyn[c] - eps);
    }
    const uint32_t zp = nCol - zn;
    if (!zp) {
        Cs[v] = cv;
        qs[v] = 1.0f;
        return;
    }
    XorwowState s = states[v];
    const float u = xorwow_uniform(s);
    states[v] = s;
    uint32_t c = 0;
    float thr = 0.0f, q = 0.0f;
    if (chk[cv]) {
        const float r = rem / (float)zp;
        do {
            q = chk[c] ? eps : pdyn[c] + r;
            thr += q;
            c++;
        } while (thr < u && c < nCol);
    } else {
        do {
            q = (c == cv) ? 1.0f - (nCol - 1) * eps : eps;
            thr += q;
            c++;
        } while (thr < u && c < nCol);
    }
    qs[v] = q;
    Cs[v] = c - 1;
    taboo[v] = (c - 1 == cv) * tabooIteration;
}

struct RefBuffers {
    uint32_t *C = nullptr, *Cs = nullptr, *taboo = nullptr, *conf = nullptr, *partial = nullptr, *stats = nullptr;
    float *qs = nullptr, *pdyn = nullptr;
    uint8_t* checker = nullptr;
    XorwowState* states = nullptr;
    ~RefBuffers() {
        (void)hipFree(C); (void)hipFree(Cs); (void)hipFree(taboo); (void)hipFree(conf); (void)hipFree(partial);
        (void)hipFree(stats); (void)hipFree(qs); (void)hipFree(pdyn); (void)hipFree(checker); (void)hipFree(states);
    }
};

}  // namespace
}  // namespace mcmc

using namespace mcmc;

extern "C" int mcmc_refstruct_bench(const mcmc_graph* g, uint32_t nCol, uint32_t sweeps, uint32_t seed,
                                    double* ms_per_sweep, uint64_t* conflicts_out) {
    if (!g || !ms_per_sweep) return fail(MCMC_E_ARG, "NULL argument");
    if (nCol < 2 || sweeps == 0) return fail(MCMC_E_ARG, "nCol >= 2 and sweeps >= 1 required");
    const GraphDev& gd = g->g;
    const uint32_t n = gd.n;
    MCMC_HIP_TRY(hipSetDevice(gd.device));
    RefBuffers B;
    const uint32_t blocks = (n + kRefThreads - 1) / kRefThreads;
    const uint32_t half = (n + 2 * kRefThreads - 1) / (2 * kRefThreads);
    MCMC_HIP_TRY(hipMalloc(&B.C, 4ull * n));
    MCMC_HIP_TRY(hipMalloc(&B.Cs, 4ull * n));
    MCMC_HIP_TRY(hipMalloc(&B.taboo, 4ull * n));
    MCMC_HIP_TRY(hipMalloc(&B.conf, 4ull * n));
    MCMC_HIP_TRY(hipMalloc(&B.partial, 4ull * half));
    MCMC_HIP_TRY(hipMalloc(&B.stats, 4ull * nCol));
    MCMC_HIP_TRY(hipMalloc(&B.qs, 4ull * n));
    MCMC_HIP_TRY(hipMalloc(&B.pdyn, 4ull * nCol));
    MCMC_HIP_TRY(hipMalloc(&B.checker, (size_t)n * nCol));
    MCMC_HIP_TRY(hipMalloc(&B.states, sizeof(XorwowState) * n));
    MCMC_HIP_TRY(hipMemset(B.taboo, 0, 4ull * n));
    ref_init_kernel<<<blocks, kRefThreads>>>(n, nCol, seed, B.C, B.states);
    MCMC_HIP_TRY(hipDeviceSynchronize());
    std::vector<uint32_t> hC(n), hpart(half), hstats(nCol);
    uint64_t conflicts = 0;
    auto calc_conflicts = [&](const uint32_t* col) -> int {
        ref_conflict_kernel<<<blocks, kRefThreads>>>(n, B.conf, col, gd.row_off, gd.col_idx);
        MCMC_HIP_TRY(hipDeviceSynchronize());
        ref_sum_kernel<<<half, kRefThreads>>>(n, B.conf, B.partial);
        MCMC_HIP_TRY(hipDeviceSynchronize());
        MCMC_HIP_TRY(hipMemcpy(hpart.data(), B.partial, 4ull * half, hipMemcpyDeviceToHost));
        conflicts = 0;
        for (uint32_t i = 0; i < half; i++) conflicts += hpart[i];
        return MCMC_OK;
    };
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t s = 0; s < sweeps; s++) {
        int rc = calc_conflicts(B.C);
        if (rc) return rc;
        MCMC_HIP_TRY(hipMemset(B.checker, 0, (size_t)n * nCol));
        MCMC_HIP_TRY(hipMemcpy(hC.data(), B.C, 4ull * n, hipMemcpyDeviceToHost));
        std::fill(hstats.begin(), hstats.end(), 0u);
        for (uint32_t v = 0; v < n; v++) hstats[hC[v] < nCol ? hC[v] : nCol - 1]++;
        MCMC_HIP_TRY(hipMemcpy(B.stats, hstats.data(), 4ull * nCol, hipMemcpyHostToDevice));
        ref_dyn_distribution_kernel<<<(nCol + kRefThreads - 1) / kRefThreads, kRefThreads>>>(B.pdyn, nCol, n, B.stats);
        ref_select_kernel<<<blocks, kRefThreads>>>(n, B.Cs, B.qs, nCol, B.C, gd.row_off, gd.col_idx, B.checker,
                                                   B.taboo, 0u, B.pdyn, B.states, 1e-8f);
        MCMC_HIP_TRY(hipDeviceSynchronize());
        rc = calc_conflicts(B.Cs);
        if (rc) return rc;
        std::swap(B.C, B.Cs);
    }
    const auto t1 = std::chrono::steady_clock::now();
    *ms_per_sweep = std::chrono::duration<double, std::milli>(t1 - t0).count() / sweeps;
    if (conflicts_out) *conflicts_out = conflicts;
    return MCMC_OK;
}
