// mcmc_colorer_amd/csrc/luby.hip -- the reference's Luby colorer (ColoringLuby::run_fast,
// graph_coloring/coloringLubyFast.cu:21-174, `--lubygpu`) on the CSR.
//
// One colour per outer round: the uncoloured nodes are the candidates (prune_eligible_clear_is,
// :112-118); inner rounds until no candidate is left: every node draws curand_uniform from its
// own XORWOW state (set_initial_distr_k, coloringLuby.cu:232-243 -- ALL nodes draw, candidates or
// not) and a candidate with u < 0.5 is selected; a selected node is dropped when a selected
// neighbour has a degree >= its own (check_conflicts_fast_k, :121-148); the survivors join the
// colour's independent set and they and their neighbours stop being candidates
// (update_eligible_fast_k, :150-168); then the set takes colour k (add_color_and_check_uncolored_k,
// coloringLuby.cu:328-341).
//
// The reference's conflict kernel reads and clears the selection flags in place, so its outcome
// depends on thread timing. This build fixes the schedule where every read precedes every write:
// the flags are read from the draw's snapshot and the survivors written to a second array. It is
// one of the reference's possible executions, deterministic, and always an independent set.
// The reference's fast_colorer_k drives the rounds with device-side launches (dynamic
// parallelism); here every kernel of a round reads a device control block (LubyCtl) and returns
// once the loop is over, so the host enqueues rounds in batches and reads the block once per batch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "mcmc_common.h"
#include "xorwow.h"

namespace mcmc {
namespace {

constexpr int kLubyThreads = 256;
constexpr uint32_t kLubyBatch = 32;   // rounds enqueued per host check

// The round loop's state, on the device: every kernel of a round returns at once when `finished`,
// so rounds are enqueued in batches and the host reads this block once per batch.
struct LubyCtl {
    uint32_t finished;   // no node left uncoloured (or an error)
    uint32_t left;       // this round: a candidate is left (check_finished_k)
    uint32_t grew;       // this round: the independent set gained a node
    uint32_t k;          // colours given so far
    uint32_t r;          // inner rounds run
    uint32_t stale;      // consecutive inner rounds without a survivor
    uint32_t unc;        // after a colour: a node is still uncoloured
    uint32_t err;        // no progress
};

// set_initial_distr_k: every node advances its state once; sel = u < 0.5 && cand. Opens the
// round in the control block (round count, cleared left / grew flags).
__global__ __launch_bounds__(kLubyThreads) void luby_draw_kernel(uint32_t n, uint32_t* __restrict__ st,
                                                                 const uint8_t* __restrict__ cand,
                                                                 uint8_t* __restrict__ sel, LubyCtl* ctl) {
    if (ctl->finished) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ctl->r++;
        ctl->left = 0;
        ctl->grew = 0;
    }
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        xw::State s;
#pragma unroll
        for (int k = 0; k < 5; k++) s.v[k] = st[(size_t)k * n + v];
        s.d = st[(size_t)5 * n + v];
        const float u = xw::uniform(xw::next(s));
#pragma unroll
        for (int k = 0; k < 5; k++) st[(size_t)k * n + v] = s.v[k];
        st[(size_t)5 * n + v] = s.d;
        sel[v] = (u < 0.5f && cand[v]) ? 1 : 0;
    }
}

// check_conflicts_fast_k on the snapshot: v survives iff no selected neighbour has degree >= deg v.
// One wave per selected node, lanes over its row.
__global__ __launch_bounds__(kLubyThreads) void luby_conflict_kernel(const uint64_t* __restrict__ ro,
                                                                     const uint32_t* __restrict__ col, uint32_t n,
                                                                     const uint8_t* __restrict__ sel,
                                                                     uint8_t* __restrict__ keep, const LubyCtl* ctl) {
    if (ctl->finished) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t v = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; v < n; v += nw) {
        if (!sel[v]) {
            if (lane == 0) keep[v] = 0;
            continue;
        }
        const uint64_t rb = ro[v], re = ro[v + 1], dv = re - rb;
        bool drop = false;
        for (uint64_t k = rb + lane; k < re && !drop; k += 64) {
            const uint32_t w = col[k];
            if (sel[w] && dv <= ro[w + 1] - ro[w]) drop = true;
        }
        drop = __ballot(drop) != 0ull;
        if (lane == 0) keep[v] = drop ? 0 : 1;
    }
}

// update_eligible_fast_k: is |= keep; a kept node and its neighbours stop being candidates (stores
// of 0 only: their order does not matter).
__global__ __launch_bounds__(kLubyThreads) void luby_update_kernel(const uint64_t* __restrict__ ro,
                                                                   const uint32_t* __restrict__ col, uint32_t n,
                                                                   const uint8_t* __restrict__ keep,
                                                                   uint8_t* __restrict__ cand, uint8_t* __restrict__ is,
                                                                   const LubyCtl* ctl) {
    if (ctl->finished) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t v = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; v < n; v += nw) {
        if (!keep[v]) continue;
        if (lane == 0) {
            is[v] = 1;
            cand[v] = 0;
        }
        for (uint64_t k = ro[v] + lane; k < ro[v + 1]; k += 64) cand[col[k]] = 0;
    }
}

// check_finished_k: *left = 1 if a candidate is left; *grew = 1 if the set gained a node this round.
__global__ __launch_bounds__(kLubyThreads) void luby_check_kernel(uint32_t n, const uint8_t* __restrict__ cand,
                                                                  const uint8_t* __restrict__ keep, LubyCtl* ctl) {
    if (ctl->finished) return;
    bool c = false, g = false;
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        c |= cand[v] != 0;
        g |= keep[v] != 0;
    }
    if (__ballot(c) && (threadIdx.x & 63u) == 0) ctl->left = 1;
    if (__ballot(g) && (threadIdx.x & 63u) == 0) ctl->grew = 1;
}

// When the round left no candidate: add_color_and_check_uncolored_k then prune_eligible_clear_is
// for the next colour: coloring[is] = k + 1; cand = uncoloured; is = 0; unc = 1 if a node is
// uncoloured.
__global__ __launch_bounds__(kLubyThreads) void luby_color_kernel(uint32_t n, uint32_t* __restrict__ coloring,
                                                                  uint8_t* __restrict__ is, uint8_t* __restrict__ cand,
                                                                  LubyCtl* ctl) {
    if (ctl->finished || ctl->left) return;
    const uint32_t k = ctl->k + 1u;   // ctl->k moves in luby_tick_kernel, after every block has read it
    bool u = false;
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        uint32_t c = coloring[v];
        if (is[v]) coloring[v] = c = k;
        is[v] = 0;
        cand[v] = c == 0 ? 1 : 0;
        u |= c == 0;
    }
    if (__ballot(u) && (threadIdx.x & 63u) == 0) ctl->unc = 1;
}

// The loop control of the round (fast_colorer_k's while / do-while): one thread.
__global__ void luby_tick_kernel(LubyCtl* ctl) {
    if (ctl->finished) return;
    if (ctl->left) {   // the inner loop goes on
        ctl->stale = ctl->grew ? 0u : ctl->stale + 1u;
        if (ctl->stale > 100000u) {   // a self-loop node can never survive its own check: the reference spins
            ctl->err = 1;
            ctl->finished = 1;
        }
        return;
    }
    ctl->k++;
    ctl->stale = 0;
    if (!ctl->unc) ctl->finished = 1;
    ctl->unc = 0;
}

}  // namespace
}  // namespace mcmc

using namespace mcmc;

extern "C" int mcmc_luby_run(const mcmc_graph* g, mcmc_gpurand* rand, uint32_t* colors, uint32_t* num_colors,
                             uint32_t* rounds) {
    if (!g || !rand || !colors) return fail(MCMC_E_ARG, "NULL argument");
    const GraphDev& gd = g->g;
    if (!gd.row_off) return fail(MCMC_E_ARG, "Luby needs a CSR graph (mcmc_graph_upload / _simulate)");
    const uint32_t n = gd.n;
    if (num_colors) *num_colors = 0;
    if (rounds) *rounds = 0;
    if (n == 0) return MCMC_OK;
    if (rand->n != n || rand->device != gd.device)
        return fail(MCMC_E_ARG, "Luby: the RNG states must be the graph's (same node count and device)");
    MCMC_HIP_TRY(hipSetDevice(gd.device));
    uint32_t* C = nullptr;
    uint8_t* b = nullptr;   // cand | sel | keep | is, n bytes each
    LubyCtl* ctl = nullptr;
    auto cleanup = [&]() { (void)hipFree(C); (void)hipFree(b); (void)hipFree(ctl); };
#define LTRY(expr)                                                                                  \
    do {                                                                                            \
        hipError_t _e = (expr);                                                                     \
        if (_e != hipSuccess) {                                                                     \
            cleanup();                                                                              \
            return fail(MCMC_E_HIP, std::string("Luby: " #expr ": ") + hipGetErrorString(_e));      \
        }                                                                                           \
    } while (0)
    LTRY(hipMalloc(&C, sizeof(uint32_t) * n));
    LTRY(hipMalloc(&b, 4ull * n));
    LTRY(hipMalloc(&ctl, sizeof(LubyCtl)));
    LTRY(hipMemset(ctl, 0, sizeof(LubyCtl)));
    uint8_t *cand = b, *sel = b + n, *keep = b + 2ull * n, *is = b + 3ull * n;
    LTRY(hipMemset(C, 0, sizeof(uint32_t) * n));   // run_fast :30-33
    LTRY(hipMemset(is, 0, n));
    LTRY(hipMemset(cand, 1, n));
    uint32_t* st = rand->states[rand->cur];
    const uint32_t tblocks = std::max<uint32_t>(1u, std::min<uint32_t>((n + kLubyThreads - 1) / kLubyThreads, 8192u));
    const uint32_t wblocks = std::max<uint32_t>(1u, std::min<uint32_t>((n + 3u) / 4u, 65535u));
    LubyCtl h{};
    for (;;) {   // kLubyBatch rounds per host check; rounds past the end are no-ops
        for (uint32_t q = 0; q < kLubyBatch; q++) {
            luby_draw_kernel<<<tblocks, kLubyThreads, 0, 0>>>(n, st, cand, sel, ctl);
            luby_conflict_kernel<<<wblocks, kLubyThreads, 0, 0>>>(gd.row_off, gd.col_idx, n, sel, keep, ctl);
            luby_update_kernel<<<wblocks, kLubyThreads, 0, 0>>>(gd.row_off, gd.col_idx, n, keep, cand, is, ctl);
            luby_check_kernel<<<tblocks, kLubyThreads, 0, 0>>>(n, cand, keep, ctl);
            luby_color_kernel<<<tblocks, kLubyThreads, 0, 0>>>(n, C, is, cand, ctl);
            luby_tick_kernel<<<1, 1, 0, 0>>>(ctl);
        }
        LTRY(hipGetLastError());
        LTRY(hipMemcpy(&h, ctl, sizeof(LubyCtl), hipMemcpyDeviceToHost));
        if (h.finished) break;
    }
    if (h.err) {
        cleanup();
        return fail(MCMC_E_DEVICE, "Luby: no progress (a candidate can never be selected: self loop?)");
    }
    const uint32_t k = h.k, r = h.r;
    LTRY(hipMemcpy(colors, C, sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
#undef LTRY
    cleanup();
    if (num_colors) *num_colors = k;
    if (rounds) *rounds = r;
    return MCMC_OK;
}
