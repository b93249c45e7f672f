// mcmc_colorer_amd/csrc/sweep_wide.h -- the wide sweep: nCol > 256 (uint16 colour replicas).
// Included by mcmc_sweep.hip inside namespace mcmc, after SweepArgs / DevState / the commit.
//
// The reference's default colour count is maxDeg (main.cu:53,162), so any power-law --graph input
//  runs with thousands of colours: occupancy masks of nCol bits no longer fit a
// lane's registers and the step-by-step CDF walk is O(nCol) per vertex. The CPU semantics are
// unchanged (coloringMCMC_CPU.cpp:115-270); what changes is how a sweep finds them:
//   * most vertices are NOT violating, and then fill_p is the "own colour" distribution (cases
//     (i)/(iii), :402-412, :471-479) whose walk needs only C[v] and u_v -- no occupancy set;
//   * only violating vertices need the occupancy set and pf (case (ii), :414-420).
// So a sweep is two launches plus the commit (commit_kernel<uint16_t>):
//   wide_tscan_kernel  (default) violation flags (violation_count, :329-351) from the slab edge
//                      layout with LDS colour-fingerprint tiles (see the kernel); every violator
//                      found is flagged once (word atomic) and, untaboo'd, listed for a walk.
//   wide_xscan_kernel  (MCMC_WIDE_SCAN=l2) the same from the XCD-slab edge layout (get_xslab
//                      below). The column space is cut into 8 slabs of S vertices;
//                      slab s's entries are read only by workgroups b with b % 8 == s, which share
//                      one XCD under round-robin dispatch, so the slab's colours (2 S bytes: 1 MiB at
//                      C5) stay in that XCD's 4 MiB L2 while the entries stream past (placement only
//                      changes speed). Every local edge is stored ONCE (in the slab of one end,
//                      picked by the parity of i + j) and a monochromatic edge flags both ends; an
//                      arc to another rank's row is kept and flags its own row. Entries are 32-bit:
//                      row delta from the 256-entry chunk's base row | slab-local column, stored
//                      lane-transposed (lane l: entries l, l + 64, l + 128, l + 192).
//   wide_scan_kernel   fallback (MCMC_WIDE_SCAN=csr, or no layout): arc-parallel pass over the CSR
//                      in 256-arc chunks, the row of an arc found by binary search.
//   wide_eval_kernel   lane per vertex, 8 vertices per lane with every load issued up front: viol ->
//                      Cviol; otherwise u_v, the own-colour walk (a range test, the F(u) table, else
//                      walk_own_tab; cdf_walk.h), Cstar / taboo / overflow event into the
//                      workgroup's ordered event list. Beside it, in the same launch, kWalkBlocks
//                      walk workgroups take the violators (walk_tasks): occupancy mask of nCol bits
//                      in LDS (ds_or), word prefix counts, then one wave walks it (walk_mask_pre:
//                      the first colour passing u found 64 words / 32 colours at a time); a hub's
//                      gathers are split over several workgroups through a global mask.
// All are grid-stride or one-shot and exit at once when the loop is done.

constexpr uint32_t kWideChunk = 256;      // entries (arcs) per wave chunk: 64 lanes x 4
constexpr uint32_t kWideMaskWords = 2048; // nCol <= 65536
constexpr uint32_t kWideMaxCol = 65535;
constexpr int kWideWalkThreads = 256;
#ifndef MCMC_WIDE_EVAL_PER
#define MCMC_WIDE_EVAL_PER 8
#endif
constexpr int kWideEvalPer = MCMC_WIDE_EVAL_PER;   // vertices per evaluation lane
constexpr uint32_t kSplitArcs = 2048;     // arcs per task of a split walk (SweepArgs::split_arcs)
#ifndef MCMC_WALK_BLOCKS
#define MCMC_WALK_BLOCKS 1024   // 4 per CU: the violator-heavy C5 sweep 0.44 -> 0.32 ms (256 / 512 / 1024 measured), none idle when converged
#endif
constexpr uint32_t kWalkBlocks = MCMC_WALK_BLOCKS;   // walk workgroups beside the evaluation
static_assert(kWalkBlocks == kIncWalkSlots, "one incremental-count slot per walk workgroup");
constexpr uint32_t kSplitMax = 64;        // violators with a global occupancy mask (split walks)
constexpr uint32_t kWalkLight = 512;      // light walks: one wave each (SweepArgs::walk_light)
constexpr uint32_t kWalkLdsWords = 4096;  // walk workgroup LDS budget for the light walks' mask sets (16 KiB)
// MCMC_PHASE_DUMP buffer: 8 words per workgroup (4096), then 2 per walk task (walk_task_stamp)
constexpr uint32_t kPhaseTaskBase = 8u * 4096u, kPhaseTaskMax = 32768u;
constexpr size_t kPhaseWords = kPhaseTaskBase + 2u * kPhaseTaskMax;
constexpr uint32_t kXsPad = 0xFFFFFFFFu;  // padding entry of the slab layout (never a valid entry)

// Violators. The scans flag vertex l (byte wflag[l]; one atomic per flag decides the first) and
// list it for a walk unless it is taboo'd (the evaluation keeps those). The walks (fill_p cases
// (i)/(ii)) run as extra workgroups of the evaluation launch, beside the evaluation proper. A light
// violator (at most walk_light arcs) goes to the front of wlist (wcount[0]) and is walked by ONE
// wave; a heavy one to the back (wcount[1]: index nloc - 1 - k) and is walked by a whole workgroup:
// heavy task k < wcount[1] walks heavy violator k (from chunk 0 of its arcs); a violator above
// split_arcs arcs, while kSplitMax global masks last, takes a slot and nt - 1 more tasks
// (wcount[1] + xbase[slot] ...), its arcs dealt out split_arcs per task. wcount: [0] light, [1]
// heavy violators, [2..3] one 64-bit word (extra tasks, slots taken) -- zeroed by the commit (the
// sweep's last kernel) for the next sweep.
__device__ __forceinline__ bool walk_heavy(const SweepArgs& a, uint64_t deg) {
    return deg > a.walk_light || deg > a.split_arcs;
}
__device__ __forceinline__ void push_violator_at(const SweepArgs& a, uint32_t l, uint32_t idx, uint64_t deg) {
    const uint32_t nloc = a.v_end - a.v_begin;
    uint32_t slot = 0xFFFFFFFFu;
    if (deg > a.split_arcs) {
        const uint32_t nx = (uint32_t)((deg + a.split_arcs - 1) / a.split_arcs) - 1u;
        const unsigned long long r =
            atomicAdd(reinterpret_cast<unsigned long long*>(a.wcount + 2), (1ull << 32) | (unsigned long long)nx);
        const uint32_t s = (uint32_t)(r >> 32);
        if (s < kSplitMax) {   // past kSplitMax: its extra tasks lie beyond every live slot's and do nothing
            slot = s;
            a.gdone[kSplitMax + s] = idx;            // sidx
            a.gdone[2 * kSplitMax + s] = (uint32_t)r; // xbase
        }
    }
    a.wlist[idx] = a.v_begin + l;
    a.wlist[nloc + idx] = slot;
}
__device__ __forceinline__ void push_violator(const SweepArgs& a, uint32_t l) {
    const uint64_t deg = a.row_off[l + 1] - a.row_off[l];
    if (walk_heavy(a, deg)) push_violator_at(a, l, a.v_end - a.v_begin - 1u - atomicAdd(&a.wcount[1], 1u), deg);
    else push_violator_at(a, l, atomicAdd(&a.wcount[0], 1u), deg);
}
__device__ __forceinline__ void flag_violator(const SweepArgs& a, uint32_t l, uint32_t) {
    if (a.wflag[l]) return;
    const uint32_t bit = 1u << (8u * (l & 3u));
    if (atomicOr(reinterpret_cast<uint32_t*>(a.wflag) + (l >> 2), bit) & bit) return;
    if (a.taboo != nullptr && a.taboo[l] > 0) return;
    push_violator(a, l);
}
// flag_violator for up to two rows per lane of a wave (l0 where want0, l1 where want1; all lanes
// call it): the flag atomics and the rows' offsets are issued side by side, and the walk list's slots
// are taken by ONE counter atomic per wave -- a device-scope atomic on one word serialises at ~90 per
// us, and a chain of dependent round trips per flagged row made a sweep with 11 000 violators' scan
// ~60 us slower than a converged one.
__device__ __forceinline__ void flag_violators_wave(const SweepArgs& a, uint32_t l0, bool want0, uint32_t l1 = 0,
                                                    bool want1 = false) {
    if (!__ballot(want0 || want1)) return;
    bool first0 = false, first1 = false;
    uint64_t d0 = 0, d1 = 0;
    if (want0) {
        const uint32_t bit = 1u << (8u * (l0 & 3u));
        first0 = (atomicOr(reinterpret_cast<uint32_t*>(a.wflag) + (l0 >> 2), bit) & bit) == 0u;
        d0 = a.row_off[l0 + 1] - a.row_off[l0];
    }
    if (want1) {
        const uint32_t bit = 1u << (8u * (l1 & 3u));
        first1 = (atomicOr(reinterpret_cast<uint32_t*>(a.wflag) + (l1 >> 2), bit) & bit) == 0u;
        d1 = a.row_off[l1 + 1] - a.row_off[l1];
    }
    const bool push0 = first0 && !(a.taboo != nullptr && a.taboo[l0] > 0);
    const bool push1 = first1 && !(a.taboo != nullptr && a.taboo[l1] > 0);
    const bool h0 = push0 && walk_heavy(a, d0), h1 = push1 && walk_heavy(a, d1);
    const uint64_t m0 = __ballot(push0 && !h0), m1 = __ballot(push1 && !h1);   // light
    const uint64_t g0 = __ballot(h0), g1 = __ballot(h1);                       // heavy
    if ((m0 | m1 | g0 | g1) == 0) return;
    const int lane = (int)(threadIdx.x & 63u);
    uint32_t base = 0, hbase = 0;
    if (m0 | m1) {
        const int lead = __ffsll((long long)(m0 | m1)) - 1;
        if (lane == lead) base = atomicAdd(&a.wcount[0], (uint32_t)(__popcll(m0) + __popcll(m1)));
        base = __shfl(base, lead, 64);
    }
    if (g0 | g1) {
        const int lead = __ffsll((long long)(g0 | g1)) - 1;
        if (lane == lead) hbase = atomicAdd(&a.wcount[1], (uint32_t)(__popcll(g0) + __popcll(g1)));
        hbase = __shfl(hbase, lead, 64);
    }
    const uint32_t top = a.v_end - a.v_begin - 1u;   // heavy violator k sits at top - k
    const uint64_t below = (1ull << lane) - 1ull;
    if (push0)
        push_violator_at(a, l0, h0 ? top - (hbase + (uint32_t)__popcll(g0 & below)) : base + (uint32_t)__popcll(m0 & below),
                         d0);
    if (push1)
        push_violator_at(a, l1,
                         h1 ? top - (hbase + (uint32_t)__popcll(g0) + (uint32_t)__popcll(g1 & below))
                            : base + (uint32_t)__popcll(m0) + (uint32_t)__popcll(m1 & below),
                         d1);
}
// One end of a monochromatic kept edge in a full scan: its row's same-colour count (incremental
// contexts) and its flag.
__device__ __forceinline__ void mono_end(const SweepArgs& a, uint32_t l, uint32_t t) {
    if (a.inc_vcnt != nullptr) atomicAdd(&a.inc_vcnt[l], 1u);
    flag_violator(a, l, t);
}

// ---- incremental violation counts (single context, symmetric CSR without repeated arcs) ---------
// Most vertices keep their colour once a power-law graph with nCol = maxDeg is nearly proper (C5:
// ~1200 of 4.2M change per sweep, mostly CDF overflows), so the violation flags of C_t follow from
// those of C_t-1 and the rows that changed: every row keeps vcnt = its arcs to same-coloured
// neighbours (violation_count, coloringMCMC_CPU.cpp:329-351, is vcnt > 0). Per sweep t:
//   wide_inc_delta_kernel  each row v that changed (C_t-1 -> C_t; the writers' slots of sweep t-1,
//                          gathered into one dense list by its commit)
//                          moves both ends of each arc (v, w) by [C_t[v] == C_t[w]] -
//                          [C_t-1[v] == C_t-1[w]] (an arc whose w changed too only from the smaller
//                          end; self-arcs never move); a count leaving 0 is listed (touched). Hubs
//                          (rows above inc_hub_arcs arcs) take a workgroup each, other rows a wave.
//   wide_tscan_kernel      (its launch, in an incremental sweep) the violators of C_t: those of C_t-1
//                          (the evaluation's slots) and the touched rows, where vcnt > 0
//                          (flag_violator dedupes); and C_t+1's replica (and fingerprints) start as
//                          C_t on the changed rows, so the writers store changes only.
// A full sweep (the first, after a slot overflowed, or when the changed rows carry more than
// inc_thresh arcs) zeroes the counts here and the tile scan counts every monochromatic edge at both
// ends (mono_end). Exact, not approximate (tests/test_wide.py::test_wide_incremental_counts).
__device__ __forceinline__ void inc_touch(const SweepArgs& a, uint32_t l, uint32_t t) {
    const uint32_t p = t & 1u, nloc = a.v_end - a.v_begin;
    const uint32_t idx = atomicAdd(&a.inc[kIncTch + p], 1u);
    if (idx < nloc) a.inc_tch[(size_t)p * nloc + idx] = l;
    else a.inc[kIncTchOvf + p] = 1u;
}
// Arcs k, k + step, ... < k1 of changed row v (colour cov in C_t-1, cnv in C_t): the other ends'
// counts move; returns this thread's part of v's own move.
__device__ __forceinline__ int inc_arcs(const SweepArgs& a, const uint16_t* __restrict__ Cp,
                                        const uint16_t* __restrict__ Cn, uint32_t v, uint32_t cov, uint32_t cnv,
                                        uint64_t k, uint64_t k1, uint32_t step, uint32_t t) {
    int dv = 0;
    for (; k < k1; k += 4ull * step) {
        uint32_t w[4], ow[4], nw[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint64_t kk = k + (uint64_t)j * step;
            w[j] = kk < k1 ? a.col_idx[kk] : v;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            ow[j] = Cp[w[j]];
            nw[j] = Cn[w[j]];
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (w[j] == v) continue;                      // a self-arc (or past the row): never moves
            if (ow[j] != nw[j] && w[j] < v) continue;    // both ends changed: counted from row w
            const int d = (int)(nw[j] == cnv) - (int)(ow[j] == cov);
            if (d != 0) {
                dv += d;
                const uint32_t lw = w[j] - a.v_begin;   // counts of this context's rows only
                if (lw < a.v_end - a.v_begin) {
                    const uint32_t old = atomicAdd(&a.inc_vcnt[lw], (uint32_t)d);
                    if (d > 0 && old == 0u) inc_touch(a, lw, t);
                }
            }
        }
    }
    return dv;
}
__device__ __forceinline__ void inc_own(const SweepArgs& a, uint32_t v, int dv, uint32_t t) {
    const uint32_t l = v - a.v_begin;
    if (dv == 0 || l >= a.v_end - a.v_begin) return;   // another rank's row: its counts live there
    const uint32_t old = atomicAdd(&a.inc_vcnt[l], (uint32_t)dv);
    if (dv > 0 && old == 0u) inc_touch(a, l, t);
}
constexpr uint32_t kIncHubLds = 1024;   // hubs whose tasks a workgroup scans in LDS (more: a workgroup each)
constexpr uint32_t kIncHubTask = 4096;  // arcs per hub task (4 per thread of a 1024-thread workgroup)
__global__ __launch_bounds__(1024) void wide_inc_delta_kernel(SweepArgs a) {
    DevState* st = a.st;
    if (a.check_done && st->done) return;
    const uint32_t t = st->t, nloc = a.v_end - a.v_begin, p = t & 1u;
    uint32_t* ctl = a.inc;
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // lists sweep t appends to (their last reader: sweep t - 1)
        const uint32_t q = p ^ 1u;
        ctl[kIncOvf + q] = 0;
        ctl[kIncTch + q] = 0;
        ctl[kIncTchOvf + q] = 0;
        ctl[kIncHubN + q] = 0;
    }
    const uint16_t* __restrict__ Cn = reinterpret_cast<const uint16_t*>(p ? a.colors1 : a.colors0);   // C_t
    const uint16_t* __restrict__ Cp = reinterpret_cast<const uint16_t*>(p ? a.colors0 : a.colors1);   // C_t-1
    if (ctl[kIncMode]) {   // full sweep: the tile scan recounts
        for (uint32_t l = blockIdx.x * blockDim.x + threadIdx.x; l < nloc; l += gridDim.x * blockDim.x)
            a.inc_vcnt[l] = 0;
        // other ranks' vertices that changed into C_t (a delta-mode commit wrote them into C_t's buffer
        // only): C_t+1's buffer takes them before this sweep's commit adds the next changes
        uint16_t* __restrict__ Cs = const_cast<uint16_t*>(Cp);
        const uint32_t nd = ctl[kIncDenseN + p], nh = ctl[kIncHubN + p];
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nd + nh; i += gridDim.x * blockDim.x) {
            const uint32_t v = i < nd ? a.inc_dense[(size_t)p * a.inc_lcap + i] : a.inc_hub[(size_t)p * a.inc_lcap + (i - nd)];
            if (v - a.v_begin >= nloc) Cs[v] = Cn[v];
        }
        return;
    }
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t nh = ctl[kIncHubN + p];
    if (nh > 0 && nh <= kIncHubLds) {
        // hubs cut into tasks of kIncHubTask arcs over the grid (one hub of C5's 29 438 arcs is 8
        // tasks, not one workgroup's 29 dependent steps): every workgroup scans the hubs' task counts
        __shared__ uint32_t s_pre[kIncHubLds], s_v[kIncHubLds], s_w[16];
        uint32_t nt = 0, hv = 0;
        if (threadIdx.x < nh) {
            hv = a.inc_hub[(size_t)p * a.inc_lcap + threadIdx.x];
            nt = (uint32_t)((a.row_off_g[hv + 1] - a.row_off_g[hv] + kIncHubTask - 1) / kIncHubTask);
        }
        uint32_t in = nt;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(in, o, 64);
            if (lane >= (uint32_t)o) in += y;
        }
        if (lane == 63u) s_w[wave] = in;
        __syncthreads();
        uint32_t tot = 0;
        for (uint32_t k = 0; k < blockDim.x / 64u; k++) {
            if (k < wave) in += s_w[k];
            tot += s_w[k];
        }
        if (threadIdx.x < nh) {
            s_pre[threadIdx.x] = in;   // inclusive: tasks of hubs 0..threadIdx.x
            s_v[threadIdx.x] = hv;
        }
        __syncthreads();
        for (uint32_t task = blockIdx.x; task < tot; task += gridDim.x) {
            uint32_t lo = 0, hi = nh - 1u;   // the first hub whose inclusive count passes task
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_pre[mid] > task) hi = mid; else lo = mid + 1u;
            }
            const uint32_t v = s_v[lo], c = task - (lo ? s_pre[lo - 1u] : 0u);
            const uint64_t rb = a.row_off_g[v] + (uint64_t)c * kIncHubTask;
            const uint64_t re = min<uint64_t>(a.row_off_g[v + 1], rb + kIncHubTask);
            int dv = inc_arcs(a, Cp, Cn, v, Cp[v], Cn[v], rb + threadIdx.x, re, blockDim.x, t);
            for (int o = 32; o > 0; o >>= 1) dv += __shfl_xor(dv, o, 64);
            if (lane == 0) inc_own(a, v, dv, t);
        }
    } else {
        for (uint32_t h = blockIdx.x; h < nh; h += gridDim.x) {   // many hubs: a workgroup each
            const uint32_t v = a.inc_hub[(size_t)p * a.inc_lcap + h];
            int dv = inc_arcs(a, Cp, Cn, v, Cp[v], Cn[v], a.row_off_g[v] + threadIdx.x, a.row_off_g[v + 1], blockDim.x, t);
            for (int o = 32; o > 0; o >>= 1) dv += __shfl_xor(dv, o, 64);
            if (lane == 0) inc_own(a, v, dv, t);
        }
    }
    // other rows (the commit gathered them into one dense list): a wave each
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6, nd = ctl[kIncDenseN + p];
    const uint32_t* dn = a.inc_dense + (size_t)p * a.inc_lcap;
    for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < nd; i += nw) {
        const uint32_t v = dn[i];
        int dv = inc_arcs(a, Cp, Cn, v, Cp[v], Cn[v], a.row_off_g[v] + lane, a.row_off_g[v + 1], 64u, t);
        for (int o = 32; o > 0; o >>= 1) dv += __shfl_xor(dv, o, 64);
        if (lane == 0) inc_own(a, v, dv, t);
    }
}

// An incremental sweep's flag pass (the tile scan's launch, all its threads).
__device__ void wide_inc_flags(const SweepArgs& a, uint32_t t) {
    const uint32_t nloc = a.v_end - a.v_begin, p = t & 1u;
    const uint32_t* ctl = a.inc;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, nthr = gridDim.x * blockDim.x;
    {   // C_t+1's buffer (and fingerprints) = C_t on the rows that changed into C_t
        const uint16_t* __restrict__ C = reinterpret_cast<const uint16_t*>(p ? a.colors1 : a.colors0);
        uint16_t* __restrict__ Cs = reinterpret_cast<uint16_t*>(p ? a.colors0 : a.colors1);
        const uint8_t* fp = p ? a.wfp1 : a.wfp0;
        uint8_t* fpn = p ? a.wfp0 : a.wfp1;
        const uint32_t nh = ctl[kIncHubN + p], nd = ctl[kIncDenseN + p];
        for (uint32_t i = tid; i < nd + nh; i += nthr) {
            const uint32_t v = i < nd ? a.inc_dense[(size_t)p * a.inc_lcap + i] : a.inc_hub[(size_t)p * a.inc_lcap + (i - nd)];
            Cs[v] = C[v];
            if (a.fp_live) fpn[v] = fp[v];
        }
    }
    const uint32_t lane = threadIdx.x & 63u, tw = tid & ~63u;   // wave-uniform loops (flag_violators_wave)
    if (ctl[kIncTchOvf + p]) {
        for (uint32_t l0 = tw; l0 < nloc; l0 += nthr) {
            const uint32_t l = l0 + lane;
            flag_violators_wave(a, l < nloc ? l : 0u, l < nloc && (int32_t)a.inc_vcnt[l] > 0);
        }
        return;
    }
    // candidates: the violators of C_t-1 (the evaluation's slots of sweep t-1) and the touched rows
    const uint32_t vs = 2u + a.inc_slot, nv = a.evnblk * a.inc_slot, ntc = ctl[kIncTch + p];
    for (uint32_t i0 = tw; i0 < nv + ntc; i0 += nthr) {
        const uint32_t i = i0 + lane;
        uint32_t l = 0;
        bool cand = false;
        if (i < nv) {
            const uint32_t* sl = a.inc_vslot + ((size_t)(p ^ 1u) * a.evnblk + i / a.inc_slot) * vs;
            const uint32_t k = i % a.inc_slot;
            if (k < min(sl[0], a.inc_slot)) {
                l = sl[2 + k];
                cand = true;
            }
        } else if (i < nv + ntc) {
            l = a.inc_tch[(size_t)p * nloc + (i - nv)];
            cand = true;
        }
        flag_violators_wave(a, l, cand && (int32_t)a.inc_vcnt[l] > 0);
    }
}

__global__ __launch_bounds__(256) void wide_xscan_kernel(SweepArgs a) {
    DevState* st = a.st;
    if (a.check_done && st->done) return;
    const uint32_t t = st->t;
    const uint16_t* __restrict__ C = reinterpret_cast<const uint16_t*>((t & 1) ? a.colors1 : a.colors0);
    const uint32_t s = blockIdx.x & (kXSlabs - 1u);   // blocks b, b + 8, ... share an XCD: one slab
    const uint32_t wpb = blockDim.x >> 6;
    const uint32_t stride = (gridDim.x / kXSlabs) * wpb;
    const uint32_t c1 = a.xs_chunk0[s + 1];
    uint32_t ch = a.xs_chunk0[s] + (blockIdx.x / kXSlabs) * wpb + (threadIdx.x >> 6);
    if (ch >= c1) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t cb = a.xs_cbits, cmask = (1u << cb) - 1u, colbase = s * a.xs_S;
    const uint32_t vb = a.v_begin, nloc = a.v_end - a.v_begin;
    const uint32_t* __restrict__ ent = a.xs_ent + 4u * lane;
    uint4 q = *reinterpret_cast<const uint4*>(ent + (size_t)ch * kWideChunk);
    uint32_t base = a.xs_base[ch];
    for (;;) {
        const uint32_t nx = ch + stride;
        const bool more = nx < c1;
        uint4 qn = make_uint4(kXsPad, kXsPad, kXsPad, kXsPad);
        uint32_t bn = 0;
        if (more) {   // the next chunk's entries are in flight while this one's colours are gathered
            qn = *reinterpret_cast<const uint4*>(ent + (size_t)nx * kWideChunk);
            bn = a.xs_base[nx];
        }
        const uint32_t e[4] = {q.x, q.y, q.z, q.w};
        uint32_t r[4], j[4], cr[4], cc[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            r[i] = base + (e[i] >> cb);
            j[i] = colbase + (e[i] & cmask);
            cr[i] = 0;
            cc[i] = 1;
            if (e[i] != kXsPad) {
                cr[i] = C[(vb + r[i])];
                cc[i] = C[j[i]];
            }
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
            if (e[i] != kXsPad && cr[i] == cc[i]) {   // rare: a monochromatic edge
                flag_violator(a, r[i], t);
                if (a.xs_sym && j[i] - vb < nloc) flag_violator(a, j[i] - vb, t);
            }
        }
        if (!more) break;
        ch = nx;
        q = qn;
        base = bn;
    }
}

// LDS mode (default). The colours gathered per arc are replaced by 8-bit fingerprints (the
// colour's low byte): equal colours have equal fingerprints, so an arc whose fingerprints differ
// is not monochromatic, and the rare match is settled on the full colours. wide_fp_kernel writes
// the fingerprints of C_t (n bytes); one 1024-thread workgroup per CU then, for each piece dealt to
// it (slab s, chunks [c0, c1)), stages the fingerprints of vertices [s 2^17, (s+1) 2^17) in LDS
// (128 KiB) and streams the piece's chunks, every wave with the next chunk in flight: the column
// fingerprint is a random LDS read, the row fingerprint a byte gather from the fingerprint array
// (rows ascend through a chunk), so a sweep moves the entries, one fingerprint pass per slab and
// no per-arc L2 request.
constexpr uint32_t kTsLog = 17;                                  // 2^17 vertices per LDS tile
constexpr int kTscanThreads = 1024;
constexpr uint32_t kTsUnroll = 3;                               // chunks per wave step
#ifndef MCMC_TS_DEPTH
#define MCMC_TS_DEPTH 2
#endif
constexpr uint32_t kTsDepth = MCMC_TS_DEPTH;                     // chunk sets in flight per wave (2 or 3)
constexpr uint32_t kTsCand = 1024;                              // LDS candidate list (8 KiB)
constexpr uint32_t kTsWin = 1024;                               // row-fingerprint window per wave (bytes)
constexpr size_t kTscanLds = (size_t)1 << kTsLog;                // 128 KiB of fingerprints

__global__ __launch_bounds__(256) void wide_fp_kernel(SweepArgs a) {
    DevState* st = a.st;
    if (a.check_done && st->done) return;
    const uint32_t t = st->t;
    const uint16_t* __restrict__ C = reinterpret_cast<const uint16_t*>((t & 1) ? a.colors1 : a.colors0);
    const uint32_t n = a.n;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; 8u * k < n; k += gridDim.x * blockDim.x) {
        const uint32_t v = 8u * k;
        uint32_t w[2] = {0, 0};
        if (v + 8u <= n) {
            const uint4 q = *reinterpret_cast<const uint4*>(C + v);
            const uint32_t c[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int i = 0; i < 4; i++) w[i >> 1] |= ((c[i] & 0xFFu) | ((c[i] >> 8) & 0xFF00u)) << (16u * (i & 1));
        } else {
            for (uint32_t i = 0; v + i < n; i++) w[i >> 2] |= ((uint32_t)C[(v + i)] & 0xFFu) << (8u * (i & 3u));
        }
        *reinterpret_cast<uint2*>(((t & 1) ? a.wfp1 : a.wfp0) + v) = make_uint2(w[0], w[1]);
    }
}

// one workgroup per CU (its LDS): 4 waves per SIMD, so up to 128 VGPRs without spilling
__global__ __launch_bounds__(kTscanThreads, 4) void wide_tscan_kernel(SweepArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lfp[];
    __shared__ uint2 cand[kTsCand];   // fingerprint matches (local row, column) of the piece
    __shared__ uint32_t ncand;
    __shared__ __attribute__((aligned(16))) uint8_t wins[kTscanThreads / 64][kTsWin];   // row windows, one per wave
    DevState* st = a.st;
    if (a.check_done && st->done) return;
    if (a.inc != nullptr && a.inc[kIncMode] == 0) {   // incremental sweep: the flags from the moved counts
        wide_inc_flags(a, st->t);
        return;
    }
    if (threadIdx.x == 0) ncand = 0;
    const uint32_t t = st->t;
    const uint16_t* __restrict__ C = reinterpret_cast<const uint16_t*>((t & 1) ? a.colors1 : a.colors0);
    const uint8_t* __restrict__ fp = (t & 1) ? a.wfp1 : a.wfp0;   // fingerprints of C_t
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nwave = blockDim.x >> 6;
    const uint32_t vb = a.v_begin, nloc = a.v_end - a.v_begin, n = a.n;
    const uint32_t p1 = a.xs_wgp[blockIdx.x + 1];
    uint8_t* win = wins[wave];
    const uint32_t* __restrict__ ent = a.xs_ent + 4u * lane;
    constexpr uint32_t cmask = (1u << kTsLog) - 1u;
    for (uint32_t p = a.xs_wgp[blockIdx.x]; p < p1; p++) {
        const uint32_t s = a.xs_pieces[3 * p], c0 = a.xs_pieces[3 * p + 1], c1 = a.xs_pieces[3 * p + 2];
        const uint32_t v0 = s << kTsLog;
        const uint32_t nv = min(1u << kTsLog, n - v0);
        __syncthreads();   // the previous piece's reads are done with the tile
        {   // stage the tile: all of a thread's 16-byte loads in flight, then the LDS stores
            const uint32_t nk = (nv + 15u) / 16u;   // fp has 16 bytes of slack past n
            const uint32_t bd = blockDim.x;
            const uint4 z4 = make_uint4(0, 0, 0, 0);
            for (uint32_t k0 = threadIdx.x; k0 < nk; k0 += 8u * bd) {
                // eight named registers (an array here was placed in scratch)
#define MCMC_TS_LD(u) const uint4 t##u = (k0 + (u) * bd < nk) ? *reinterpret_cast<const uint4*>(fp + v0 + 16u * (k0 + (u) * bd)) : z4;
#define MCMC_TS_ST(u) if (k0 + (u) * bd < nk) *reinterpret_cast<uint4*>(lfp + 16u * (k0 + (u) * bd)) = t##u;
                MCMC_TS_LD(0) MCMC_TS_LD(1) MCMC_TS_LD(2) MCMC_TS_LD(3)
                MCMC_TS_LD(4) MCMC_TS_LD(5) MCMC_TS_LD(6) MCMC_TS_LD(7)
                MCMC_TS_ST(0) MCMC_TS_ST(1) MCMC_TS_ST(2) MCMC_TS_ST(3)
                MCMC_TS_ST(4) MCMC_TS_ST(5) MCMC_TS_ST(6) MCMC_TS_ST(7)
#undef MCMC_TS_LD
#undef MCMC_TS_ST
            }
        }
        __syncthreads();
        // a wave takes kTsUnroll chunks at a time (ch, ch + nwave, ...). Vector loads complete in
        // order, so each step issues its fingerprint gathers BEFORE the next set's entries and
        // waits only for the gathers; fingerprint matches go to an LDS candidate list settled once
        // per piece (their colour loads would otherwise wait for the prefetch every step).
        uint32_t ch = c0 + wave;
        if (ch < c1) {
            const uint4 pad4 = make_uint4(kXsPad, kXsPad, kXsPad, kXsPad);
            const uint32_t S = kTsUnroll * nwave;   // chunks from one set of this wave to its next
            // set `cs` (chunks cs, cs + nwave, ...) into (Y, BY); chunks past the piece are padding
            auto load_set = [&](uint4 (&Y)[kTsUnroll], uint32_t (&BY)[kTsUnroll], uint32_t cs) {
#pragma unroll
                for (uint32_t u = 0; u < kTsUnroll; u++) {
                    const uint32_t c = cs + u * nwave;
                    Y[u] = pad4;
                    BY[u] = 0;
                    if (c < c1) {
                        Y[u] = *reinterpret_cast<const uint4*>(ent + (size_t)c * kWideChunk);
                        BY[u] = a.xs_base[c];
                    }
                }
            };
            // one step: set `ch` from (X, BX); the set MCMC_TS_DEPTH - 1 ahead is loaded into (Y, BY)
            // behind this step's fingerprint gathers. Returns false once the piece is done.
            auto step = [&](uint4 (&X)[kTsUnroll], uint32_t (&BX)[kTsUnroll], uint4 (&Y)[kTsUnroll],
                            uint32_t (&BY)[kTsUnroll]) -> bool {
                if (ch >= c1) return false;
                uint32_t e[4 * kTsUnroll], r[4 * kTsUnroll], fr[4 * kTsUnroll], fc[4 * kTsUnroll];
#pragma unroll
                for (uint32_t u = 0; u < kTsUnroll; u++) {
                    e[4 * u] = X[u].x;
                    e[4 * u + 1] = X[u].y;
                    e[4 * u + 2] = X[u].z;
                    e[4 * u + 3] = X[u].w;
                }
                // row fingerprints: each chunk's rows ascend from its base, so one 16-byte load per
                // lane fetches a 1 KiB window of them (from base rounded down to 16); entries past
                // the window (rare) gather their byte
                uint4 wv[kTsUnroll];
                uint32_t w0[kTsUnroll];
#pragma unroll
                for (uint32_t u = 0; u < kTsUnroll; u++) {
                    w0[u] = (vb + BX[u]) & ~15u;
                    wv[u] = *reinterpret_cast<const uint4*>(fp + w0[u] + 16u * lane);   // fp has 2 KiB of slack
                }
#pragma unroll
                for (uint32_t i = 0; i < 4 * kTsUnroll; i++) {
                    r[i] = BX[i / 4] + (e[i] >> kTsLog);
                    fc[i] = e[i] != kXsPad ? (uint32_t)lfp[e[i] & cmask] : 1u;
                }
                load_set(Y, BY, ch + (kTsDepth - 1u) * S);   // behind the gathers
#pragma unroll
                for (uint32_t u = 0; u < kTsUnroll; u++) {   // the wave's window slot: its own LDS ops stay in order
                    *reinterpret_cast<uint4*>(win + 16u * lane) = wv[u];
#pragma unroll
                    for (uint32_t k = 0; k < 4; k++) {
                        const uint32_t i = 4 * u + k;
                        const uint32_t d = vb + r[i] - w0[u];
                        fr[i] = e[i] == kXsPad ? 0u : d < kTsWin ? (uint32_t)win[d] : (uint32_t)fp[vb + r[i]];
                    }
                }
#pragma unroll
                for (uint32_t i = 0; i < 4 * kTsUnroll; i++) {
                    if (e[i] != kXsPad && fr[i] == fc[i]) {   // fingerprints match (1 in 256 at random)
                        const uint32_t k = atomicAdd(&ncand, 1u);
                        if (k < kTsCand) {
                            cand[k] = make_uint2(r[i], v0 + (e[i] & cmask));
                        } else {   // list full: settle it here
                            const uint32_t j = v0 + (e[i] & cmask);
                            if (C[(vb + r[i])] == C[j]) {
                                mono_end(a, r[i], t);
                                if (a.xs_sym && j - vb < nloc) mono_end(a, j - vb, t);
                            }
                        }
                    }
                }
                ch += S;
                return true;
            };
            // register sets rotate by expansion, never by copy (a copy would wait for its loads)
            uint4 qa[kTsUnroll], qb[kTsUnroll];
            uint32_t ba[kTsUnroll], bb[kTsUnroll];
            load_set(qa, ba, ch);
#if MCMC_TS_DEPTH == 3
            uint4 qc[kTsUnroll];
            uint32_t bc[kTsUnroll];
            load_set(qb, bb, ch + S);
            for (;;) {
                if (!step(qa, ba, qc, bc)) break;
                if (!step(qb, bb, qa, ba)) break;
                if (!step(qc, bc, qb, bb)) break;
            }
#else
            for (;;) {
                if (!step(qa, ba, qb, bb)) break;
                if (!step(qb, bb, qa, ba)) break;
            }
#endif
        }
        __syncthreads();
        const uint32_t nc = min(ncand, kTsCand);
        for (uint32_t k0 = threadIdx.x & ~63u; k0 < nc; k0 += blockDim.x) {   // the candidates: compare colours
            const uint32_t k = k0 + lane;
            uint2 rc = make_uint2(0u, 0u);
            bool mono = false;
            if (k < nc) {
                rc = cand[k];
                mono = C[(vb + rc.x)] == C[rc.y];
            }
            const bool other = mono && a.xs_sym && rc.y - vb < nloc;
            if (a.inc_vcnt != nullptr) {
                if (mono) atomicAdd(&a.inc_vcnt[rc.x], 1u);
                if (other) atomicAdd(&a.inc_vcnt[rc.y - vb], 1u);
            }
            flag_violators_wave(a, rc.x, mono, other ? rc.y - vb : 0u, other);
        }
        __syncthreads();
        if (threadIdx.x == 0) ncand = 0;
    }
}

__global__ __launch_bounds__(256) void wide_scan_kernel(SweepArgs a) {
    DevState* st = a.st;
    if (a.check_done && st->done) return;
    const uint32_t t = st->t;
    const uint16_t* __restrict__ C = reinterpret_cast<const uint16_t*>((t & 1) ? a.colors1 : a.colors0);
    const uint64_t* __restrict__ ro = a.row_off;
    const uint64_t a0 = a.arc_begin, m = a.arc_count;
    const int lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t ch = wave; ch < a.nchunks; ch += nwaves) {
        const uint64_t k0 = (uint64_t)ch * kWideChunk + 4u * (uint32_t)lane;   // local arc index
        if (k0 >= m) continue;
        const uint4 q = *reinterpret_cast<const uint4*>(a.col_idx + a0 + k0);   // a0 % 4 == 0
        uint32_t id[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int i = 1; i < 4; i++)
            if (k0 + i >= m) id[i] = 0u;   // slack past m: gather a valid address, ignore below
        uint32_t nc[4];
#pragma unroll
        for (int i = 0; i < 4; i++) nc[i] = C[id[i]];
        // row of arc k0: the largest r in [lo, hi] with ro[r] - a0 <= k0
        uint32_t lo = a.chunk_row[ch], hi = a.chunk_row[ch + 1];
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1u) >> 1;
            if (ro[mid] - a0 <= k0) lo = mid; else hi = mid - 1u;
        }
        uint32_t r = lo;
        uint64_t rend = ro[r + 1] - a0;
        uint32_t own = C[(a.v_begin + r)];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint64_t k = k0 + i;
            if (k >= m) break;
            if (rend <= k) {
                do { r++; rend = ro[r + 1] - a0; } while (rend <= k);
                own = C[(a.v_begin + r)];
            }
            if (nc[i] == own) flag_violator(a, r, t);
        }
    }
}

// Occupancy of arcs [k0, k1) of N(v) (count_free_colors, coloringMCMC_CPU.cpp:362-383) OR-ed into
// the LDS mask, 8 independent gathers per thread in flight.
__device__ __forceinline__ void walk_gather(const SweepArgs& a, const uint16_t* __restrict__ C, uint32_t* mask,
                                            uint64_t k0, uint64_t k1) {
    for (uint64_t k = k0 + threadIdx.x; k < k1; k += 8u * blockDim.x) {
        uint32_t c[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint64_t kk = k + (uint64_t)j * blockDim.x;
            c[j] = kk < k1 ? (uint32_t)C[a.col_idx[kk]] : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int j = 0; j < 8; j++)
            if (c[j] != 0xFFFFFFFFu) atomicOr(&mask[c[j] >> 5], 1u << (c[j] & 31u));
    }
}

// A workgroup barrier for LDS hand-offs only: the walks' global loads and stores stay in flight
// across it (__syncthreads waits for every outstanding one: with the loaded latency of a sweep full of
// random gathers, each such wait costs microseconds).
__device__ __forceinline__ void walk_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Partitioned delta exchange (a.dcap > 0): this rank's vertex v takes colour c in sweep t (overflow
// events aside: every rank replays those), into its delta slot of the next-colour parity. One lane.
__device__ __forceinline__ void wide_delta_one(const SweepArgs& a, uint32_t t, uint32_t v, uint32_t c) {
    uint32_t* dl = (t & 1) ? a.dlt0 : a.dlt1;
    const uint32_t idx = atomicAdd(dl, 1u);
    if (idx < a.dcap) {
        dl[kDeltaHead + 2u * idx] = v;
        dl[kDeltaHead + 2u * idx + 1u] = c;
    }
}

// The resample of violator v (fill_p case (ii) / (i)) from its occupancy mask in LDS, by a whole
// 256-thread workgroup: word prefix counts, then one wave walks them. cv = C_t[v] and x = u_v's
// minstd state come in (loaded beside the task's first loads); deg = v's arcs. Overflow events go
// to the global list. All threads call it; it ends with an LDS barrier.
template <bool PART>
__device__ void walk_finish(const SweepArgs& a, uint32_t v, uint32_t t, uint32_t cv, uint32_t x, uint32_t deg,
                            uint16_t* __restrict__ Cs, const uint32_t* mask, uint32_t* pre, uint32_t* wsum,
                            uint32_t* islot, uint32_t* ic) {
    DevState* st = a.st;
    const uint32_t NWW = (a.nCol + 31u) >> 5;
    const uint32_t per = (NWW + kWideWalkThreads - 1u) / kWideWalkThreads;   // words per thread (prefix)
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t l = v - a.v_begin;
    // pre[w] = occupied colours in words < w: per-thread word runs, wave scan, workgroup offsets
    const uint32_t w0 = threadIdx.x * per;
    uint32_t s = 0;
    for (uint32_t w = w0; w < w0 + per && w < NWW; w++) s += __popc(mask[w]);
    uint32_t inc = s;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63u) wsum[wave] = inc;
    walk_sync();
    uint32_t run = inc - s;
    for (uint32_t k = 0; k < wave; k++) run += wsum[k];
    for (uint32_t w = w0; w < w0 + per && w < NWW; w++) {
        pre[w] = run;
        run += __popc(mask[w]);
    }
    if (threadIdx.x == 0) {
        uint32_t T = 0;
        for (uint32_t k = 0; k < kWideWalkThreads / 64; k++) T += wsum[k];
        pre[NWW] = T;
    }
    walk_sync();
    if (wave == 0) {   // the walk: one wave, all lanes in step (walk_mask_pre ballots)
        const uint32_t P = pre[NWW], Zvcomp = a.nCol - P;
        const float u = minstd_canonical(x);
        uint32_t nc;
        if (Zvcomp > 0) {   // case (ii)
            const float pf = (1.0f - a.eps * (float)P) / (float)Zvcomp;
            nc = walk_mask_pre(mask, pre, a.nCol, a.eps, pf, u, a.walk_tie != 0u);
        } else {            // case (i)
            nc = walk_own_tab(a.etab, a.nCol, cv, a.eps, a.hi, u);
        }
        if (lane == 0) {
            const bool event = nc == a.nCol;
            const uint32_t nv = event ? cv : nc;
            // an incremental sweep's C_t+1 buffer already holds C_t here (wide_inc_flags)
            if (nv != cv || a.inc == nullptr || a.inc[kIncMode]) {
                Cs[v] = (uint16_t)nv;
                if (a.fp_live) ((t & 1) ? a.wfp0 : a.wfp1)[v] = (uint8_t)nv;
            }
            if (islot != nullptr && nv != cv) atomicAdd(&ic[1], inc_list_deg(a, l, t, islot, a.inc_wslot_n, &ic[0], deg));
            if (PART && a.dcap && nv != cv) wide_delta_one(a, t, v, nv);
            if (a.taboo != nullptr && !event) a.taboo[l] = (nc == cv) ? a.tabooIteration : 0u;
            if (event) {
                const uint32_t idx = atomicAdd(&st->ev_count, 1u);
                if (idx < a.ev_cap) a.events[idx] = v;
                else atomicOr(&st->err, kDevErrEvents);
            }
        }
    }
    walk_sync();
}

// One wave's LDS hand-off: DS operations of a wave complete in order, so its lanes see each other's
// writes once they have completed (and the compiler may not move LDS accesses across it).
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// walk_gather for one wave: arcs [k0, k1) OR-ed into the wave's own LDS mask, 8 gathers per lane in flight.
__device__ __forceinline__ void walk_gather_wave(const SweepArgs& a, const uint16_t* __restrict__ C, uint32_t* mask,
                                                 uint64_t k0, uint64_t k1, uint32_t lane) {
    for (uint64_t k = k0 + lane; k < k1; k += 8u * 64u) {
        uint32_t c[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint64_t kk = k + (uint64_t)j * 64u;
            c[j] = kk < k1 ? (uint32_t)C[a.col_idx[kk]] : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int j = 0; j < 8; j++)
            if (c[j] != 0xFFFFFFFFu) atomicOr(&mask[c[j] >> 5], 1u << (c[j] & 31u));
    }
}

// walk_finish for one wave and its own mask set (a light walk): the word prefix counts by the
// wave's 64 lanes, then the same walk and stores. All 64 lanes call it.
template <bool PART>
__device__ void walk_finish_wave(const SweepArgs& a, uint32_t v, uint32_t t, uint32_t cv, uint32_t x, uint32_t deg,
                                 uint16_t* __restrict__ Cs, const uint32_t* mask, uint32_t* pre, uint32_t* islot,
                                 uint32_t* ic, uint32_t lane) {
    DevState* st = a.st;
    const uint32_t NWW = (a.nCol + 31u) >> 5;
    const uint32_t per = (NWW + 63u) >> 6;
    const uint32_t l = v - a.v_begin;
    const uint32_t w0 = lane * per;
    uint32_t s = 0;
    for (uint32_t w = w0; w < w0 + per && w < NWW; w++) s += __popc(mask[w]);
    uint32_t inc = s;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    uint32_t run = inc - s;
    for (uint32_t w = w0; w < w0 + per && w < NWW; w++) {
        pre[w] = run;
        run += __popc(mask[w]);
    }
    if (lane == 63u) pre[NWW] = inc;
    wave_lds_sync();
    const uint32_t P = pre[NWW], Zvcomp = a.nCol - P;
    const float u = minstd_canonical(x);
    uint32_t nc;
    if (Zvcomp > 0) {   // case (ii)
        const float pf = (1.0f - a.eps * (float)P) / (float)Zvcomp;
        nc = walk_mask_pre(mask, pre, a.nCol, a.eps, pf, u, a.walk_tie != 0u);
    } else {            // case (i)
        nc = walk_own_tab(a.etab, a.nCol, cv, a.eps, a.hi, u);
    }
    if (lane == 0) {
        const bool event = nc == a.nCol;
        const uint32_t nv = event ? cv : nc;
        if (nv != cv || a.inc == nullptr || a.inc[kIncMode]) {
            Cs[v] = (uint16_t)nv;
            if (a.fp_live) ((t & 1) ? a.wfp0 : a.wfp1)[v] = (uint8_t)nv;
        }
        if (islot != nullptr && nv != cv) atomicAdd(&ic[1], inc_list_deg(a, l, t, islot, a.inc_wslot_n, &ic[0], deg));
        if (PART && a.dcap && nv != cv) wide_delta_one(a, t, v, nv);
        if (a.taboo != nullptr && !event) a.taboo[l] = (nc == cv) ? a.tabooIteration : 0u;
        if (event) {
            const uint32_t idx = atomicAdd(&st->ev_count, 1u);
            if (idx < a.ev_cap) a.events[idx] = v;
            else atomicOr(&st->err, kDevErrEvents);
        }
    }
    wave_lds_sync();
}

// Diagnostics (MCMC_PHASE_DUMP): walk task k's gather and walk durations (wall-clock ticks, packed
// 32 | 32) and its arcs | kind << 32 (0 light, 1 heavy whole row, 2 split chunk, 3 split chunk + walk).
__device__ __forceinline__ void walk_task_stamp(const SweepArgs& a, uint32_t k, unsigned long long t0,
                                                unsigned long long t1, uint64_t deg, uint32_t kind) {
    if (k >= kPhaseTaskMax) return;
    const unsigned long long t2 = wall_clock64();
    a.phase_ts[kPhaseTaskBase + 2u * k] = (t1 - t0) | ((t2 - t1) << 32);
    a.phase_ts[kPhaseTaskBase + 2u * k + 1] = deg | ((unsigned long long)kind << 32);
}

// Light-walk mask sets: words of one (mask + prefix counts), and how many fit the LDS budget (the
// worker waves of a walk workgroup, at most its 4).
__host__ __device__ inline uint32_t walk_set_words(uint32_t nCol) {
    const uint32_t nww = (nCol + 31u) >> 5;
    return ((nww + 3u) & ~3u) + ((nww + 4u) & ~3u);
}
__host__ __device__ inline uint32_t walk_waves(uint32_t nCol) {
    const uint32_t g = kWalkLdsWords / walk_set_words(nCol);
    return g < 1u ? 1u : (g > 4u ? 4u : g);
}

// The walk workgroups of the evaluation launch. Heavy tasks first, b, b + nb, ... (push_violator). A one-task
// violator: its whole occupancy mask and walk here. A split violator (a hub, whose gathers would
// otherwise be one workgroup's serial latency chain): each task ORs its part of the occupancy into
// the slot's global mask, and the workgroup finishing the last task takes the mask back
// (atomicExch: read and clear for the next sweep) and walks. Software-pipelined: the next task's list
// entry is loaded beside this task's row offsets, own colour and first gathers, and LDS hand-offs
// use walk_sync, so a task costs its offsets, ids and colours round trips (~3), not ~7.
template <bool PART>
__device__ void walk_tasks(const SweepArgs& a, uint32_t b, uint32_t nb, uint32_t t, uint32_t x_t) {
    // the occupancy mask and its word prefix counts: dynamic LDS sized for nCol (wide_walk_lds), so
    // the evaluation launch's workgroups are not all sized for 65 536 colours
    extern __shared__ __attribute__((aligned(16))) uint32_t wlds[];
    const uint32_t nww = (a.nCol + 31u) >> 5;
    uint32_t* mask = wlds;
    uint32_t* pre = wlds + ((nww + 3u) & ~3u);
    __shared__ uint32_t wsum[kWideWalkThreads / 64];
    __shared__ uint32_t sh_last;
    __shared__ uint32_t ic[2];   // incremental counts: rows this workgroup changed, their arcs
    const uint32_t cnt = a.wcount[0], nh = a.wcount[1];   // light, heavy violators
    const uint32_t nx = a.wcount[2], ns = min(a.wcount[3], kSplitMax);
    const uint32_t T = nh + nx;   // heavy tasks
    // this workgroup's slot of changed rows (written every sweep, empty ones too)
    uint32_t* islot = a.inc ? a.inc_wslot + ((size_t)((t + 1u) & 1u) * kIncWalkSlots + b) * (2u + a.inc_wslot_n)
                            : nullptr;
    if (b >= T && b >= cnt) {
        if (islot != nullptr && threadIdx.x == 0) {
            islot[0] = islot[1] = 0;
            uint32_t* hd = a.inc_hdr + ((size_t)((t + 1u) & 1u) * (a.evnblk + kIncWalkSlots) + a.evnblk + b) * 2u;
            hd[0] = hd[1] = 0;
        }
        return;
    }
    __shared__ uint32_t sh_nt[2];   // diagnostics: tasks, split tasks
    if (threadIdx.x == 0) ic[0] = ic[1] = sh_nt[0] = sh_nt[1] = 0;   // (lane 0 of each wave uses them)
    walk_sync();
    const unsigned long long ts0 = a.phase_ts ? wall_clock64() : 0ull;   // diagnostics (MCMC_PHASE_DUMP)
    uint32_t ntask = 0, nsplit = 0;
    const uint16_t* __restrict__ C = reinterpret_cast<const uint16_t*>((t & 1) ? a.colors1 : a.colors0);
    uint16_t* __restrict__ Cs = reinterpret_cast<uint16_t*>((t & 1) ? a.colors0 : a.colors1);
    const uint32_t NWW = (a.nCol + 31u) >> 5;
    const uint32_t nloc = a.v_end - a.v_begin;
    const uint32_t* sidx = a.gdone + kSplitMax;
    const uint32_t* xbase = a.gdone + 2 * kSplitMax;
    const uint32_t SA = a.split_arcs;
    // task -> (list index, chunk); false past the last live split slot
    auto decode = [&](uint32_t task, uint32_t& idx, uint32_t& c) -> bool {
        c = 0;
        if (task < nh) {
            idx = nloc - 1u - task;
            return true;
        }
        const uint32_t j = task - nh;   // extra task j: the slot with the last xbase <= j
        if (ns == 0) return false;
        uint32_t lo = 0, hi = ns;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (xbase[mid] <= j) lo = mid;
            else hi = mid;
        }
        idx = sidx[lo];
        c = j - xbase[lo] + 1u;
        return true;
    };
    uint32_t idx = 0, c = 0;
    bool live = b < T && decode(b, idx, c);
    uint32_t v = live ? a.wlist[idx] : 0u, slot = live ? a.wlist[nloc + idx] : 0u;
    for (uint32_t task = b; live && task < T; task += nb) {
        const uint32_t l = v - a.v_begin;
        // this task's offsets, own colour and u_v; the next task's list entry (side by side)
        const uint64_t rb = a.row_off[l], re = a.row_off[l + 1];
        const uint32_t cv = C[v];
        const uint32_t x = minstd_mulmod(x_t, minstd_pow_tab_wave((uint64_t)v + 1));
        uint32_t nidx = 0, nc = 0;
        const bool nlive = task + nb < T && decode(task + nb, nidx, nc);
        const uint32_t nv = nlive ? a.wlist[nidx] : 0u, nslot = nlive ? a.wlist[nloc + nidx] : 0u;
        ntask++;
        const unsigned long long tt0 = a.phase_ts ? wall_clock64() : 0ull;
        if (slot == 0xFFFFFFFFu) {   // one task: the whole row
            for (uint32_t w = threadIdx.x; w < NWW; w += blockDim.x) mask[w] = 0;
            walk_sync();
            walk_gather(a, C, mask, rb, re);
            walk_sync();
            const unsigned long long tt1 = a.phase_ts ? wall_clock64() : 0ull;
            walk_finish<PART>(a, v, t, cv, x, (uint32_t)(re - rb), Cs, mask, pre, wsum, islot, ic);
            if (a.phase_ts && threadIdx.x == 0) walk_task_stamp(a, cnt + task, tt0, tt1, re - rb, 1u);
        } else {
            const uint32_t ntk = (uint32_t)((re - rb + SA - 1) / SA);
            nsplit++;
            if (c < ntk) {   // (else: an extra task of a slotless split violator)
                uint32_t* gm = a.gmask + (size_t)slot * kWideMaskWords;
                for (uint32_t w = threadIdx.x; w < NWW; w += blockDim.x) mask[w] = 0;
                walk_sync();
                walk_gather(a, C, mask, rb + (uint64_t)c * SA, min<uint64_t>(re, rb + (uint64_t)(c + 1) * SA));
                walk_sync();
                for (uint32_t w = threadIdx.x; w < NWW; w += blockDim.x)
                    if (mask[w]) atomicOr(&gm[w], mask[w]);
                __threadfence();
                __syncthreads();
                if (threadIdx.x == 0) {
                    const uint32_t done = atomicAdd(&a.gdone[slot], 1u) + 1u;
                    sh_last = done == ntk;
                    if (done == ntk) a.gdone[slot] = 0;   // every task of this sweep has counted
                }
                __syncthreads();
                const unsigned long long tt1 = a.phase_ts ? wall_clock64() : 0ull;
                if (sh_last) {
                    __threadfence();
                    for (uint32_t w = threadIdx.x; w < NWW; w += blockDim.x) mask[w] = atomicExch(&gm[w], 0u);
                    walk_sync();
                    walk_finish<PART>(a, v, t, cv, x, (uint32_t)(re - rb), Cs, mask, pre, wsum, islot, ic);
                }
                if (a.phase_ts && threadIdx.x == 0) walk_task_stamp(a, cnt + task, tt0, tt1, re - rb, sh_last ? 3u : 2u);
                walk_sync();   // sh_last and mask are reused by the next task
            }
        }
        live = nlive;
        idx = nidx;
        c = nc;
        v = nv;
        slot = nslot;
    }
    // light tasks: one wave each, worker b + nb w (w < the waves whose mask sets fit), own mask set
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u, G = walk_waves(a.nCol);
    uint32_t nlight = 0;
    if (wave < G) {
        uint32_t* wm = wlds + wave * walk_set_words(a.nCol);
        uint32_t* wp = wm + ((NWW + 3u) & ~3u);
        const uint32_t stride = nb * G;
        uint32_t k = b + nb * wave;
        uint32_t lv = k < cnt ? a.wlist[k] : 0u;
        for (; k < cnt; k += stride) {
            const uint32_t l = lv - a.v_begin;
            // this task's offsets, own colour and u_v; the next task's list entry (side by side)
            const uint64_t rb = a.row_off[l], re = a.row_off[l + 1];
            const uint32_t cv = C[lv];
            const uint32_t x = minstd_mulmod(x_t, minstd_pow_tab_wave((uint64_t)lv + 1));
            const uint32_t nv = k + stride < cnt ? a.wlist[k + stride] : 0u;
            const unsigned long long tt0 = a.phase_ts ? wall_clock64() : 0ull;
            for (uint32_t w = lane; w < NWW; w += 64u) wm[w] = 0;
            wave_lds_sync();
            walk_gather_wave(a, C, wm, rb, re, lane);
            wave_lds_sync();
            const unsigned long long tt1 = a.phase_ts ? wall_clock64() : 0ull;
            walk_finish_wave<PART>(a, lv, t, cv, x, (uint32_t)(re - rb), Cs, wm, wp, islot, ic, lane);
            if (a.phase_ts && lane == 0) walk_task_stamp(a, k, tt0, tt1, re - rb, 0u);
            nlight++;
            lv = nv;
        }
    }
    if (a.phase_ts && lane == 0) {
        atomicAdd(&sh_nt[0], nlight + (wave == 0 ? ntask : 0u));   // heavy tasks: counted by every wave
        if (wave == 0) atomicAdd(&sh_nt[1], nsplit);
    }
    __syncthreads();   // every wave's entries and counts are in
    if (a.phase_ts && threadIdx.x == 0) {   // walk workgroup b: start, end, tasks, split tasks
        a.phase_ts[b * 8u + 0] = ts0;
        a.phase_ts[b * 8u + 1] = wall_clock64();
        a.phase_ts[b * 8u + 2] = sh_nt[0];
        a.phase_ts[b * 8u + 3] = sh_nt[1];
    }
    if (islot != nullptr && threadIdx.x == 0) {   // lane 0 of the walking wave made every entry
        islot[0] = ic[0];
        islot[1] = ic[1];
        uint32_t* hd = a.inc_hdr + ((size_t)((t + 1u) & 1u) * (a.evnblk + kIncWalkSlots) + a.evnblk + b) * 2u;
        hd[0] = ic[0];
        hd[1] = ic[1];
    }
}

// Dynamic LDS of the evaluation launch: walk_waves mask sets, a walk's mask (nCol bits) and prefix
// counts each (a heavy walk uses the first).
inline size_t wide_walk_lds(uint32_t nCol) { return 4u * (size_t)walk_waves(nCol) * walk_set_words(nCol); }

// Grid: kWalkBlocks walk workgroups (walk_tasks; first, so that they start at once), then evnblk =
// ceil(nloc / (256 * kWideEvalPer)) evaluation workgroups of 256; lane `tid` of evaluation
// workgroup eb takes the vertices eb * 2048 + j * 256 + tid, j < 8 (coalesced per j).
// PART: a partitioned rank's sweep (the delta exchange's slot writes, a.dcap); the single-context
// instantiation carries none of that code.
template <bool PART>
__global__ __launch_bounds__(256) void wide_eval_kernel(SweepArgs a) {
    __shared__ uint32_t sh_viol, sh_nev;
    __shared__ uint32_t sh_ev[kEvSlot];   // this workgroup's overflow events (ordered at the end)
    __shared__ uint32_t sh_ic[3];         // incremental counts: changed rows, their arcs, violators listed
    DevState* st = a.st;
    if (a.check_done && st->done) return;
    if (blockIdx.x < kWalkBlocks) {   // the walks, beside the evaluation (dispatched first)
        walk_tasks<PART>(a, blockIdx.x, kWalkBlocks, st->t, st->x_t);
        return;
    }
    const uint32_t eb = blockIdx.x - kWalkBlocks;   // evaluation workgroup
    if (threadIdx.x == 0) {
        sh_viol = 0;
        sh_nev = 0;
        sh_ic[0] = sh_ic[1] = sh_ic[2] = 0;
    }
    __syncthreads();
    const uint32_t t = st->t, x_t = st->x_t;
    // incremental counts: this workgroup's slots -- rows it changes (C_t+1 parity) and violators of C_t
    uint32_t* islot = nullptr;
    uint32_t* vslot = nullptr;
    if (a.inc != nullptr) {
        islot = a.inc_eslot + ((size_t)((t + 1u) & 1u) * a.evnblk + eb) * (2u + a.inc_slot);
        vslot = a.inc_vslot + ((size_t)(t & 1u) * a.evnblk + eb) * (2u + a.inc_slot);
    }
    const uint16_t* __restrict__ C = reinterpret_cast<const uint16_t*>((t & 1) ? a.colors1 : a.colors0);
    uint16_t* __restrict__ Cs = reinterpret_cast<uint16_t*>((t & 1) ? a.colors0 : a.colors1);
    const uint32_t nloc = a.v_end - a.v_begin;
    const int lane = threadIdx.x & 63;
    const uint32_t l0 = eb * (256u * kWideEvalPer) + threadIdx.x;
    uint8_t* __restrict__ fpn = a.fp_live ? ((t & 1) ? a.wfp0 : a.wfp1) : nullptr;   // fingerprints of C_{t+1}
    uint32_t viol[kWideEvalPer], cv[kWideEvalPer], tab[kWideEvalPer];
#pragma unroll
    for (int j = 0; j < kWideEvalPer; j++) {
        const uint32_t l = l0 + 256u * j;
        viol[j] = 0;
        cv[j] = 0;
        tab[j] = 0;
        if (l < nloc) {
            viol[j] = a.wflag[l];
            cv[j] = C[(a.v_begin + l)];
            if (a.taboo != nullptr) tab[j] = a.taboo[l];
            if (a.vflags) a.vflags[(size_t)(t & 1u) * nloc + l] = (uint8_t)viol[j];   // Cviols of C_t (tail cut)
        }
    }
    // u_v: engine draw K_t + v + 1 (bulk draw in vertex order, coloringMCMC_CPU.cpp:139); the
    // lane's draw moves by 16807^256 from one j to the next
    const uint32_t a256 = a.a256;
    uint32_t x = minstd_mulmod(minstd_mulmod(x_t, a.evpow[4u * eb + (threadIdx.x >> 6)]), kMinstdLanePow[lane]);
    uint32_t xs[kWideEvalPer];
#pragma unroll
    for (int j = 0; j < kWideEvalPer; j++) {
        xs[j] = x;
        x = minstd_mulmod(x, a256);
    }
    // The own-colour walk (cases (i)/(iii)): for E[nCol-1] <= u < hi (all but about 2 (nCol-1) eps
    // of the draws) no eps prefix passes u and the own colour's step does -- the colour stays. For
    // u < E[nCol-1] the answer depends on u alone up to cv: F(u) = first k with E[k] > u, one load
    // of the host table ftab (indexed by x - 1, u = (x - 1) 2^-31 exactly); else the table walk.
    const bool tabled = a.eps > 0.0f;
    // an incremental sweep stores changes only: C_t+1's buffer already holds C_t (wide_inc_flag_kernel)
    const bool wall = a.inc == nullptr || a.inc[kIncMode] != 0u;
    uint32_t cviol = 0;
#pragma unroll
    for (int j = 0; j < kWideEvalPer; j++) {
        const uint32_t l = l0 + 256u * j;
        const bool valid = l < nloc;
        const uint32_t v = a.v_begin + l;
        const float u = minstd_canonical(xs[j]);
        cviol += viol[j];
        bool event = false;
        bool dch = false;   // a case (iii) change of colour (the delta slot's)
        uint32_t dnv = 0;
        if (valid) {
            if (viol[j]) {
                a.wflag[l] = 0;
                if (vslot != nullptr) {   // the next sweep's flag pass starts from the violators of C_t
                    const uint32_t k = atomicAdd(&sh_ic[2], 1u);
                    if (k < a.inc_slot) vslot[2 + k] = l;
                    else a.inc[kIncOvf + ((t + 1u) & 1u)] = 1u;
                }
            }
            if (tab[j] > 0) {   // :496-501
                if (wall) {
                    Cs[v] = (uint16_t)cv[j];
                    if (fpn) fpn[v] = (uint8_t)cv[j];
                }
                a.taboo[l] = tab[j] - 1;
            } else if (viol[j]) {
                // case (i) or (ii): a walk workgroup's (walk_tasks)
            } else {           // case (iii)
                uint32_t nc;
                if (tabled && a.emax <= u && u < a.hi) {
                    nc = cv[j];
                } else if (tabled && u < a.emax && xs[j] - 1u < a.ftab_n) {   // ftab_n > 0 only if emax < hi
                    const uint32_t F = a.ftab[xs[j] - 1u];
                    nc = F <= cv[j] ? F - 1u : cv[j];
                } else {
                    nc = walk_own_tab(a.etab, a.nCol, cv[j], a.eps, a.hi, u);
                }
                event = nc == a.nCol;
                const uint32_t nv = event ? cv[j] : nc;   // an event's colour is the commit's replay
                if (wall || nv != cv[j]) {
                    Cs[v] = (uint16_t)nv;
                    if (fpn) fpn[v] = (uint8_t)nv;
                }
                if (islot != nullptr && nv != cv[j]) atomicAdd(&sh_ic[1], inc_list(a, l, t, islot, a.inc_slot, &sh_ic[0]));
                if (a.taboo != nullptr && !event) a.taboo[l] = (nc == cv[j]) ? a.tabooIteration : 0u;
                dch = nv != cv[j];
                dnv = nv;
            }
        }
        if (PART && a.dcap) {   // partitioned delta exchange: one slot atomic per wave
            const uint64_t db = __ballot(dch);
            if (db) {
                uint32_t* dl = (t & 1) ? a.dlt0 : a.dlt1;
                const int lead = __ffsll((long long)db) - 1;
                uint32_t base = 0;
                if (lane == lead) base = atomicAdd(dl, (uint32_t)__popcll(db));
                base = __shfl(base, lead, 64);
                const uint32_t idx = base + (uint32_t)__popcll(db & ((1ull << lane) - 1ull));
                if (dch && idx < a.dcap) {
                    dl[kDeltaHead + 2u * idx] = v;
                    dl[kDeltaHead + 2u * idx + 1u] = dnv;
                }
            }
        }
        if (event) {   // into this workgroup's LDS list; past kEvSlot, the global list
            const uint32_t k = atomicAdd(&sh_nev, 1u);
            if (k < kEvSlot) {
                sh_ev[k] = v;
            } else {
                const uint32_t idx = atomicAdd(&st->ev_count, 1u);
                if (idx < a.ev_cap) a.events[idx] = v;
                else atomicOr(&st->err, kDevErrEvents);
            }
        }
    }
    __syncthreads();
    // this workgroup's list, ascending (rank of each event among at most kEvSlot), and its count
    const uint32_t ne = min(sh_nev, kEvSlot);
    if (threadIdx.x < ne) {
        const uint32_t v = sh_ev[threadIdx.x];
        uint32_t rk = 0;
        for (uint32_t k = 0; k < ne; k++) rk += sh_ev[k] < v ? 1u : 0u;
        a.evblk[(size_t)eb * kEvSlot + rk] = v;
    }
    if (threadIdx.x == 0) {
        a.evcnt[eb] = ne;
        if (islot != nullptr) {   // slot headers, written every sweep
            islot[0] = sh_ic[0];
            islot[1] = sh_ic[1];
            uint32_t* hd = a.inc_hdr + ((size_t)((t + 1u) & 1u) * (a.evnblk + kIncWalkSlots) + eb) * 2u;
            hd[0] = sh_ic[0];
            hd[1] = sh_ic[1];
            vslot[0] = sh_ic[2];
            vslot[1] = 0;
        }
    }
    for (int off = 32; off >= 1; off >>= 1) cviol += __shfl_xor(cviol, off, 64);
    if (lane == 0 && cviol) atomicAdd(&sh_viol, cviol);
    __syncthreads();
    if (threadIdx.x == 0 && sh_viol) atomicAdd(&st->viol, (unsigned long long)sh_viol);
}

// First local row of every 256-arc chunk (the row owning the chunk's first arc); entry nchunks =
// the last row.
__global__ void wide_chunk_row_kernel(const uint64_t* __restrict__ row_off, uint32_t nloc, uint64_t a0,
                                      uint64_t m, uint32_t nchunks, uint32_t* __restrict__ chunk_row) {
    for (uint32_t ch = blockIdx.x * blockDim.x + threadIdx.x; ch <= nchunks; ch += gridDim.x * blockDim.x) {
        if (ch == nchunks || nloc == 0) { chunk_row[ch] = nloc ? nloc - 1u : 0u; continue; }
        const uint64_t k = (uint64_t)ch * kWideChunk;
        uint32_t lo = 0, hi = nloc - 1u;   // largest r with row_off[r] - a0 <= k
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1u) >> 1;
            if (row_off[mid] - a0 <= k) lo = mid; else hi = mid - 1u;
        }
        chunk_row[ch] = lo;
    }
}

// ColoringMCMC_CPU ctor colouring (coloringMCMC_CPU.cpp:61) into a uint16 replica.
__global__ void init_coloring_wide_kernel(uint16_t* C, uint32_t n, uint32_t x0, UniformIntConst k, DevState* st) {
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        const uint32_t x = minstd_mulmod(x0, minstd_pow_tab((uint64_t)v + 1));
        const uint32_t r = x - 1u;
        if (r >= k.past) atomicAdd(&st->init_rejections, 1u);
        C[v] = (uint16_t)min(r / k.scaling, 65535u);
    }
}

// ---- slab edge layout (built once per graph, row range and mode; cached on the graph) ------------
// Local rows [vb, vb + nloc). Arc (i, j) of row i = vb + l is kept iff the layout is asymmetric
// (every arc, flags its row only), or j is another rank's row, or ((i + j) & 1) == (i < j): of the
// two arcs of a local edge exactly one survives.
__device__ __forceinline__ bool xs_keep(uint32_t i, uint32_t j, uint32_t vb, uint32_t nloc, uint32_t sym) {
    return !sym || j - vb >= nloc || ((i + j) & 1u) == (i < j ? 1u : 0u);
}

// *bad = 1 if a local row (ascending) lists a neighbour twice: the incremental counts need every
// edge exactly once in each end's row. One wave per row.
__global__ __launch_bounds__(256) void xs_dupcheck_kernel(const uint64_t* __restrict__ ro,
                                                          const uint32_t* __restrict__ col, uint32_t nloc,
                                                          uint32_t* __restrict__ bad) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t l = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; l < nloc; l += nw) {
        bool dup = false;
        for (uint64_t k = ro[l] + 1u + lane; k < ro[l + 1]; k += 64) dup = dup || col[k] == col[k - 1];
        if (__ballot(dup) && lane == 0) atomicOr(bad, 1u);
    }
}

// cnt[l] = kept arcs of local row l. One wave per row.
__global__ __launch_bounds__(256) void xs_rowcount_kernel(const uint64_t* __restrict__ ro,
                                                          const uint32_t* __restrict__ col, uint32_t nloc, uint32_t vb,
                                                          uint32_t sym, uint32_t* __restrict__ cnt) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t l = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; l < nloc; l += nw) {
        uint32_t k8 = 0;
        for (uint64_t k = ro[l] + lane; k < ro[l + 1]; k += 64) k8 += xs_keep(vb + l, col[k], vb, nloc, sym) ? 1u : 0u;
        for (int o = 32; o >= 1; o >>= 1) k8 += __shfl_xor(k8, o, 64);
        if (lane == 0) cnt[l] = k8;
    }
}

// key = slab << 32 | local row, val = slab-local column, for every kept arc in CSR order (pos = the
// exclusive scan of xs_rowcount_kernel). One wave per row, ballot ranks.
__global__ __launch_bounds__(256) void xs_keys_kernel(const uint64_t* __restrict__ ro, const uint32_t* __restrict__ col,
                                                      uint32_t nloc, uint32_t vb, uint32_t S, uint32_t sym,
                                                      const uint32_t* __restrict__ pos, uint64_t* __restrict__ key,
                                                      uint32_t* __restrict__ val) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (uint32_t l = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; l < nloc; l += nw) {
        uint32_t run = pos[l];
        const uint64_t e = ro[l + 1];
        for (uint64_t kb = ro[l]; kb < e; kb += 64) {
            const uint64_t k = kb + lane;
            const uint32_t j = k < e ? col[k] : 0u;
            const bool keep = k < e && xs_keep(vb + l, j, vb, nloc, sym);
            const uint64_t m = __ballot(keep);
            if (keep) {
                const uint32_t idx = run + (uint32_t)__popcll(m & lt);
                const uint32_t s = j / S;
                key[idx] = ((uint64_t)s << 32) | l;
                val[idx] = j - s * S;
            }
            run += (uint32_t)__popcll(m);
        }
    }
}

// start[s] = first sorted index whose slab is >= s, s = 0..nslabs.
__global__ void xs_slab_start_kernel(const uint64_t* __restrict__ key, uint32_t total, uint32_t nslabs,
                                     uint32_t* __restrict__ start) {
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s <= nslabs; s += gridDim.x * blockDim.x) {
        uint32_t lo = 0, hi = total;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((uint32_t)(key[mid] >> 32) < s) lo = mid + 1; else hi = mid;
        }
        start[s] = lo;
    }
}

// base[g] = local row of chunk g's first entry; ent = every sorted arc's entry.
__global__ void xs_base_kernel(const uint64_t* __restrict__ key, const uint32_t* __restrict__ start,
                               const uint32_t* __restrict__ chunk0, uint32_t nslabs, uint32_t chunks,
                               uint32_t* __restrict__ base) {
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < chunks; g += gridDim.x * blockDim.x) {
        uint32_t lo = 0, hi = nslabs - 1u;   // the slab s with chunk0[s] <= g < chunk0[s + 1]
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1u) >> 1;
            if (chunk0[mid] <= g) lo = mid; else hi = mid - 1u;
        }
        base[g] = (uint32_t)key[start[lo] + (g - chunk0[lo]) * kWideChunk];
    }
}

__global__ void xs_fill_kernel(const uint64_t* __restrict__ key, const uint32_t* __restrict__ val, uint32_t total,
                               const uint32_t* __restrict__ start, const uint32_t* __restrict__ chunk0,
                               const uint32_t* __restrict__ base, uint32_t cbits, uint32_t* __restrict__ ent,
                               uint32_t* err) {
    const uint32_t dmax = (1u << (32u - cbits)) - 2u;   // all-ones stays the padding value
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const uint64_t k = key[i];
        const uint32_t s = (uint32_t)(k >> 32), l = (uint32_t)k;
        const uint32_t rel = i - start[s];
        const uint32_t g = chunk0[s] + rel / kWideChunk;
        const uint32_t d = l - base[g];
        if (d > dmax) atomicOr(err, 1u);
        // lane-transposed chunk: lane l's 16-byte word holds entries l, 64 + l, 128 + l, 192 + l, so
        // each of a wave's four gathers covers 64 consecutive (row-ascending) entries
        const uint32_t q = rel % kWideChunk;
        ent[(size_t)g * kWideChunk + 4u * (q & 63u) + (q >> 6)] = (d << cbits) | val[i];
    }
}

XSlabLayout::~XSlabLayout() {
    (void)hipFree(ent);
    (void)hipFree(base);
    (void)hipFree(chunk0);
    (void)hipFree(pieces);
    (void)hipFree(wg_piece);
}

// LDS mode: cut every slab's chunks into pieces of about chunks / nwg (at least one per non-empty
// slab) and deal them to the nwg workgroups, largest first to the least loaded (LPT).
static void plan_pieces(const std::vector<uint32_t>& chunk0, uint32_t nwg, std::vector<uint32_t>& pieces,
                        std::vector<uint32_t>& wgp) {
    const uint32_t ns = (uint32_t)chunk0.size() - 1u;
    const double T = std::max(1.0, (double)chunk0[ns] / nwg);
    std::vector<std::array<uint32_t, 3>> pc;
    for (uint32_t s = 0; s < ns; s++) {
        const uint32_t c0 = chunk0[s], cs = chunk0[s + 1] - c0;
        if (!cs) continue;
        const uint32_t p = std::max<uint32_t>(1u, (uint32_t)std::llround(cs / T));
        for (uint32_t k = 0; k < p; k++) {
            const uint32_t a = c0 + (uint32_t)((uint64_t)cs * k / p), b = c0 + (uint32_t)((uint64_t)cs * (k + 1) / p);
            if (b > a) pc.push_back({s, a, b});
        }
    }
    std::stable_sort(pc.begin(), pc.end(), [](const std::array<uint32_t, 3>& x, const std::array<uint32_t, 3>& y) {
        return x[2] - x[1] > y[2] - y[1];
    });
    std::vector<std::vector<uint32_t>> per(nwg);
    std::vector<std::pair<uint64_t, uint32_t>> heap;   // (load, workgroup), min-heap
    for (uint32_t w = 0; w < nwg; w++) heap.push_back({0, w});
    auto cmp = [](const std::pair<uint64_t, uint32_t>& x, const std::pair<uint64_t, uint32_t>& y) { return x > y; };
    std::make_heap(heap.begin(), heap.end(), cmp);
    for (uint32_t i = 0; i < (uint32_t)pc.size(); i++) {
        std::pop_heap(heap.begin(), heap.end(), cmp);
        auto& h = heap.back();
        per[h.second].push_back(i);
        h.first += pc[i][2] - pc[i][1];
        std::push_heap(heap.begin(), heap.end(), cmp);
    }
    pieces.clear();
    wgp.assign(nwg + 1, 0);
    for (uint32_t w = 0; w < nwg; w++) {
        wgp[w] = (uint32_t)(pieces.size() / 3);
        for (uint32_t i : per[w]) pieces.insert(pieces.end(), pc[i].begin(), pc[i].end());
    }
    wgp[nwg] = (uint32_t)(pieces.size() / 3);
}

// XCD-aware variant (default when nwg is a multiple of kXSlabs): the row space is cut into kXSlabs
// ranges of equal chunk counts (quantiles of the chunks' base rows), and range x goes to the
// workgroups b with b % kXSlabs == x, which share one XCD under round-robin dispatch. A workgroup's
// row-fingerprint windows then stay inside its XCD's range (0.5 MiB of fingerprints at C5: resident
// in that XCD's 4 MiB L2 across all 32 slabs) instead of every XCD sweeping all n fingerprints once
// per slab. Inside an XCD, each slab's chunks of the range are cut into pieces of about the
// XCD's chunks / workgroups and dealt largest first (LPT) as plan_pieces does.
static void plan_pieces_xcd(const std::vector<uint32_t>& chunk0, const std::vector<uint32_t>& base, uint32_t nwg,
                            std::vector<uint32_t>& pieces, std::vector<uint32_t>& wgp) {
    const uint32_t ns = (uint32_t)chunk0.size() - 1u, C = chunk0[ns], X = kXSlabs, per_x = nwg / X;
    std::vector<uint32_t> sorted_base(base.begin(), base.begin() + C);
    std::sort(sorted_base.begin(), sorted_base.end());
    std::vector<uint32_t> bound(X + 1, 0u);   // row ranges [bound[x], bound[x+1])
    for (uint32_t x = 1; x < X; x++) bound[x] = sorted_base[(size_t)C * x / X];
    bound[X] = 0xFFFFFFFFu;
    std::vector<std::vector<uint32_t>> per(nwg);
    std::vector<std::array<uint32_t, 3>> all;
    for (uint32_t x = 0; x < X; x++) {
        std::vector<std::array<uint32_t, 3>> cells;   // (slab, lo, hi) of this row range
        uint64_t tot = 0;
        for (uint32_t s = 0; s < ns; s++) {
            const auto b0 = base.begin() + chunk0[s], b1 = base.begin() + chunk0[s + 1];
            // chunks of slab s ascend by base row: the range's chunks are one run
            const uint32_t lo = chunk0[s] + (uint32_t)(std::lower_bound(b0, b1, bound[x]) - b0);
            const uint32_t hi = x + 1 == X ? chunk0[s + 1] : chunk0[s] + (uint32_t)(std::lower_bound(b0, b1, bound[x + 1]) - b0);
            if (hi > lo) { cells.push_back({s, lo, hi}); tot += hi - lo; }
        }
        const double T = std::max(1.0, (double)tot / per_x);
        std::vector<std::array<uint32_t, 3>> pc;
        for (const auto& c : cells) {
            const uint32_t cs = c[2] - c[1];
            const uint32_t p = std::max<uint32_t>(1u, (uint32_t)std::llround(cs / T));
            for (uint32_t k = 0; k < p; k++) {
                const uint32_t a = c[1] + (uint32_t)((uint64_t)cs * k / p), b = c[1] + (uint32_t)((uint64_t)cs * (k + 1) / p);
                if (b > a) pc.push_back({c[0], a, b});
            }
        }
        std::stable_sort(pc.begin(), pc.end(), [](const std::array<uint32_t, 3>& p, const std::array<uint32_t, 3>& q) {
            return p[2] - p[1] > q[2] - q[1];
        });
        std::vector<std::pair<uint64_t, uint32_t>> heap;   // (load, workgroup), min-heap over the XCD's workgroups
        for (uint32_t k = 0; k < per_x; k++) heap.push_back({0, x + k * X});
        auto cmp = [](const std::pair<uint64_t, uint32_t>& p, const std::pair<uint64_t, uint32_t>& q) { return p > q; };
        std::make_heap(heap.begin(), heap.end(), cmp);
        for (const auto& p : pc) {
            std::pop_heap(heap.begin(), heap.end(), cmp);
            auto& h = heap.back();
            per[h.second].push_back((uint32_t)all.size());
            all.push_back(p);
            h.first += p[2] - p[1];
            std::push_heap(heap.begin(), heap.end(), cmp);
        }
    }
    pieces.clear();
    wgp.assign(nwg + 1, 0);
    for (uint32_t w = 0; w < nwg; w++) {
        wgp[w] = (uint32_t)(pieces.size() / 3);
        for (uint32_t i : per[w]) pieces.insert(pieces.end(), all[i].begin(), all[i].end());
    }
    wgp[nwg] = (uint32_t)(pieces.size() / 3);
}

// The slab layout of rows [vb, ve) in `mode` (0: 8 L2 slabs, 1: 2^17-vertex LDS tiles over `nwg`
// workgroups), built on first use and cached on the graph. *out stays nullptr (and MCMC_OK is
// returned) when the layout does not apply: no CSR, no arcs, uint32 entry positions or row deltas
// would overflow, or it does not fit in free device memory -- the sweep then scans the CSR.
int get_xslab(mcmc_graph* gh, uint32_t vb, uint32_t ve, uint32_t mode, uint32_t nwg, hipStream_t st,
              const XSlabLayout** out) {
    *out = nullptr;
    for (auto& x : gh->xslabs)
        if (x->v_begin == vb && x->v_end == ve && x->mode == mode && (mode == 0 || x->nwg == nwg)) {
            *out = x->ent ? x.get() : nullptr;
            return MCMC_OK;
        }
    GraphDev& gd = gh->g;
    const uint32_t nloc = ve - vb;
    if (!gd.row_off || nloc == 0) return MCMC_OK;
    uint64_t ends[2];
    MCMC_HIP_TRY(hipMemcpy(&ends[0], gd.row_off + vb, sizeof(uint64_t), hipMemcpyDeviceToHost));
    MCMC_HIP_TRY(hipMemcpy(&ends[1], gd.row_off + ve, sizeof(uint64_t), hipMemcpyDeviceToHost));
    const uint64_t mloc = ends[1] - ends[0];
    if (mloc == 0 || mloc >= 0x7FF00000ull) return MCMC_OK;
    const uint32_t S = mode == 1 ? (1u << kTsLog)
                                 : std::max<uint32_t>(1u, (uint32_t)(((uint64_t)gd.n + kXSlabs - 1) / kXSlabs));
    const uint32_t nslabs = (uint32_t)(((uint64_t)gd.n + S - 1) / S);
    uint32_t cbits = 1;
    while ((1ull << cbits) < S) cbits++;
    if (cbits > 26) return MCMC_OK;
    size_t fr = 0, tot = 0;
    MCMC_HIP_TRY(hipMemGetInfo(&fr, &tot));
    const uint64_t need = 28ull * mloc + 4ull * kWideChunk * nslabs + 8ull * nloc + (256ull << 20);
    if (need > fr) return MCMC_OK;
    if (!gd.sorted) {   // the symmetry check searches rows; neighbour order does not affect the sweep
        int rs = sort_rows_inplace(gd);
        if (rs) return rs;
    }
    std::unique_ptr<XSlabLayout> L(new XSlabLayout());
    L->v_begin = vb;
    L->v_end = ve;
    L->mode = mode;
    L->S = S;
    L->cbits = cbits;
    L->nslabs = nslabs;
    uint32_t *flag = nullptr, *cnt = nullptr, *pos = nullptr, *val = nullptr, *val2 = nullptr, *start = nullptr;
    uint64_t *key = nullptr, *key2 = nullptr;
    void* tmp = nullptr;
    auto cleanup = [&]() {
        (void)hipFree(flag);
        (void)hipFree(cnt);
        (void)hipFree(pos);
        (void)hipFree(val);
        (void)hipFree(val2);
        (void)hipFree(start);
        (void)hipFree(key);
        (void)hipFree(key2);
        (void)hipFree(tmp);
    };
#define XTRY(expr)                                                                                  \
    do {                                                                                            \
        hipError_t _e = (expr);                                                                     \
        if (_e != hipSuccess) {                                                                     \
            cleanup();                                                                              \
            return fail(MCMC_E_HIP, std::string("slab layout: " #expr ": ") + hipGetErrorString(_e)); \
        }                                                                                           \
    } while (0)
    const uint32_t wblocks = std::max<uint32_t>(1u, std::min<uint32_t>((nloc + 3u) / 4u, 65535u));   // 4 rows per block
    uint32_t h[2] = {0, 0};
    XTRY(hipMalloc(&flag, 2 * sizeof(uint32_t)));
    XTRY(hipMemsetAsync(flag, 0, 2 * sizeof(uint32_t), st));
    bool symmetric = false;   // the one-entry-per-edge layout needs every local arc's reverse
    if (int rs = csr_symmetric(gd, vb, nloc, st, &symmetric)) { cleanup(); return rs; }
    L->sym = symmetric ? 1u : 0u;
    if (symmetric) {   // rows are sorted (above): repeated arcs sit side by side
        xs_dupcheck_kernel<<<wblocks, 256, 0, st>>>(gd.row_off + vb, gd.col_idx, nloc, flag + 1);
        XTRY(hipGetLastError());
        XTRY(hipMemcpyAsync(&h[1], flag + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        XTRY(hipStreamSynchronize(st));
        L->simple = h[1] == 0 ? 1u : 0u;
        h[1] = 0;
        XTRY(hipMemsetAsync(flag + 1, 0, sizeof(uint32_t), st));
    }
    // kept arcs per row -> positions -> (slab, row) keys in CSR order -> stable sort by key
    XTRY(hipMalloc(&cnt, sizeof(uint32_t) * ((size_t)nloc + 1)));
    XTRY(hipMalloc(&pos, sizeof(uint32_t) * ((size_t)nloc + 1)));
    XTRY(hipMemsetAsync(cnt + nloc, 0, sizeof(uint32_t), st));
    xs_rowcount_kernel<<<wblocks, 256, 0, st>>>(gd.row_off + vb, gd.col_idx, nloc, vb, L->sym, cnt);
    XTRY(hipGetLastError());
    size_t tb = 0, tb2 = 0;
    XTRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, pos, (int)nloc + 1, st));
    XTRY(hipMalloc(&tmp, std::max<size_t>(tb, 1)));
    XTRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, pos, (int)nloc + 1, st));
    uint32_t total = 0;
    XTRY(hipMemcpyAsync(&total, pos + nloc, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    XTRY(hipStreamSynchronize(st));
    L->entries = total;
    if (total == 0) {
        cleanup();
        gh->xslabs.push_back(std::move(L));   // remembered as "not applicable"
        return MCMC_OK;
    }
    XTRY(hipMalloc(&key, sizeof(uint64_t) * total));
    XTRY(hipMalloc(&key2, sizeof(uint64_t) * total));
    XTRY(hipMalloc(&val, sizeof(uint32_t) * total));
    XTRY(hipMalloc(&val2, sizeof(uint32_t) * total));
    xs_keys_kernel<<<wblocks, 256, 0, st>>>(gd.row_off + vb, gd.col_idx, nloc, vb, S, L->sym, pos, key, val);
    XTRY(hipGetLastError());
    uint32_t kbits = 32;
    while ((1ull << (kbits - 32)) < nslabs) kbits++;
    XTRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, key, key2, val, val2, (int)total, 0, (int)kbits, st));
    if (tb2 > tb) {
        (void)hipFree(tmp);
        tmp = nullptr;
        XTRY(hipMalloc(&tmp, tb2));
        tb = tb2;
    }
    XTRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb2, key, key2, val, val2, (int)total, 0, (int)kbits, st));
    XTRY(hipMalloc(&start, sizeof(uint32_t) * ((size_t)nslabs + 1)));
    xs_slab_start_kernel<<<(nslabs + 256) / 256, 256, 0, st>>>(key2, total, nslabs, start);
    XTRY(hipGetLastError());
    std::vector<uint32_t> sh((size_t)nslabs + 1);
    XTRY(hipMemcpyAsync(sh.data(), start, sizeof(uint32_t) * sh.size(), hipMemcpyDeviceToHost, st));
    XTRY(hipStreamSynchronize(st));
    L->chunk0_h.assign((size_t)nslabs + 1, 0u);
    for (uint32_t s = 0; s < nslabs; s++)
        L->chunk0_h[s + 1] = L->chunk0_h[s] + (sh[s + 1] - sh[s] + kWideChunk - 1) / kWideChunk;
    L->chunks = L->chunk0_h[nslabs];
    XTRY(hipMalloc(&L->chunk0, sizeof(uint32_t) * L->chunk0_h.size()));
    XTRY(hipMemcpyAsync(L->chunk0, L->chunk0_h.data(), sizeof(uint32_t) * L->chunk0_h.size(), hipMemcpyHostToDevice, st));
    XTRY(hipMalloc(&L->ent, sizeof(uint32_t) * kWideChunk * (size_t)L->chunks));
    XTRY(hipMalloc(&L->base, sizeof(uint32_t) * (size_t)L->chunks));
    XTRY(hipMemsetAsync(L->ent, 0xFF, sizeof(uint32_t) * kWideChunk * (size_t)L->chunks, st));
    xs_base_kernel<<<std::max<uint32_t>(1u, std::min<uint32_t>((L->chunks + 255u) / 256u, 65535u)), 256, 0, st>>>(
        key2, start, L->chunk0, nslabs, L->chunks, L->base);
    XTRY(hipGetLastError());
    xs_fill_kernel<<<std::max<uint32_t>(1u, std::min<uint32_t>((total + 255u) / 256u, 65535u)), 256, 0, st>>>(
        key2, val2, total, start, L->chunk0, L->base, cbits, L->ent, flag + 1);
    XTRY(hipGetLastError());
    XTRY(hipMemcpyAsync(&h[1], flag + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    XTRY(hipStreamSynchronize(st));
    if (!h[1] && mode == 1) {
        std::vector<uint32_t> pc, wgp;
        const char* pe = getenv("MCMC_TSCAN_PLAN");   // "lpt": the XCD-blind plan (A/B)
        if (nwg % kXSlabs == 0 && !(pe && std::string(pe) == "lpt")) {
            std::vector<uint32_t> bh(L->chunks);
            XTRY(hipMemcpy(bh.data(), L->base, sizeof(uint32_t) * bh.size(), hipMemcpyDeviceToHost));
            plan_pieces_xcd(L->chunk0_h, bh, nwg, pc, wgp);
        } else {
            plan_pieces(L->chunk0_h, nwg, pc, wgp);
        }
        L->nwg = nwg;
        L->npieces = (uint32_t)(pc.size() / 3);
        XTRY(hipMalloc(&L->pieces, sizeof(uint32_t) * std::max<size_t>(pc.size(), 3)));
        XTRY(hipMalloc(&L->wg_piece, sizeof(uint32_t) * wgp.size()));
        if (!pc.empty())
            XTRY(hipMemcpy(L->pieces, pc.data(), sizeof(uint32_t) * pc.size(), hipMemcpyHostToDevice));
        XTRY(hipMemcpy(L->wg_piece, wgp.data(), sizeof(uint32_t) * wgp.size(), hipMemcpyHostToDevice));
        XTRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&wide_tscan_kernel),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTscanLds));
    }
#undef XTRY
    cleanup();
    if (h[1]) {   // a row delta beyond the entry's field: scan the CSR instead
        (void)hipFree(L->ent);
        L->ent = nullptr;
        gh->xslabs.push_back(std::move(L));
        return MCMC_OK;
    }
    *out = L.get();
    gh->xslabs.push_back(std::move(L));
    return MCMC_OK;
}
