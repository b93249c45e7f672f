// mcmc_colorer_amd/csrc/wide_solo.h -- the persistent wide sweep (ws_kernel): nCol > 256 once the
// colouring is nearly proper. Included by mcmc_sweep.hip inside namespace mcmc, after sweep_wide.h.
//
// The per-sweep wide launches (sweep_wide.h) evaluate all n rows every sweep, so a converged sweep
// at C5 (4.2e6 rows, ~1 200 of them changing) costs four launches and ~60 us of fixed work. Which
// rows can change is known before any row is read, as for the dense sweep (dense_sparse.h):
//   * a violator (its count of same-coloured neighbours is > 0) resamples from its occupancy mask
//     (fill_p cases (ii)/(i), coloringMCMC_CPU.cpp:414-420, 402-412);
//   * any other row is in case (iii) (own colour hi, others eps): it keeps its colour exactly when
//     its draw u_v lies in [E[nCol-1], hi) (sweep_wide.h wide_eval_kernel's range test), i.e. when
//     its minstd state lies outside the window W = [1, w_lo) U [w_hi, 2^31 - 1) -- C5 (eps 1e-8,
//     nCol 29 438): 1.26e6 of the 2^31 - 2 states. Vertex v draws state 16807^(lx_t + v + 1) in
//     sweep t (lx_t = log x_t), so the window's states sorted by logarithm L hand out sweep t's
//     candidate rows as the entries with L in [lx_t + 1, lx_t + 1 + n) mod (2^31 - 2): one or two
//     contiguous runs of the table (a bucket index finds them), ~n |W| / 2^31 rows (C5: ~2 500).
// The counts (SweepArgs::inc_vcnt, the incremental counts of sweep_wide.h) are kept exact across
// sweeps: each changed row moves both ends of its arcs by [C_t+1 equal] - [C_t equal]. So a sweep
// reads the candidates, the violators and the changed rows' arcs -- nothing else.
//
// One launch runs K sweeps, one 1024-thread workgroup per CU. Workgroup 0 (the leader) runs each
// sweep: loop control (:136, :259-269; Cviol_t = the violator list's length), its own small walks
// and the candidates' own-colour walks, the overflow events' glibc draws in ascending vertex order
// (:517-520) and the changed rows' writes (into BOTH colour buffers, which stay equal), and hands
// the grid-sized parts to the other workgroups as phases (posted through a flag word, completion
// counted on another): many violators' walks (a wave each, workgroups for heavy rows), count moves
// of many changed arcs, a full violator collection, the recount of a new colouring. Results come
// back through device-scope atomics and plain stores bracketed by release/acquire (the dense
// sweep's hand-off rules, dense_sparse.h).
// Entry from the per-sweep launches: a full recount pending (kIncMode) is run here; a pending
// change list of the last per-sweep commit is applied; the violator list is collected unless the
// last persistent launch left it valid for this t. Exit: the per-sweep path's next flag pass visits
// every row (kIncTchOvf) and its delta lists are empty -- both paths may alternate freely.

constexpr uint32_t kWsDone = 1, kWsAck = 2, kWsT = 3;
constexpr uint32_t kWsGen = 80;      // the phase flag the helpers poll: a cache line of its own
constexpr uint32_t kWsVn = 4;        // [2] violator-list lengths, by parity of t
constexpr uint32_t kWsResN = 6;      // results of the running sweep
constexpr uint32_t kWsTchN = 7, kWsTchOvf = 8;
constexpr uint32_t kWsHeavyN = 9, kWsChgN = 10, kWsArgT = 11, kWsArgP = 12;   // [13]: x_t of the sweep
constexpr uint32_t kWsCandN = 14, kWsArgL = 15;   // the next sweep's changing candidates, its minstd log
constexpr uint32_t kWsStat = 16;     // u64 [8]: solo sweeps, phases, leader walks, walk phases,
                                     // delta phases, collects, candidates, changed rows
constexpr uint32_t kWsErr = 32;      // watchdog: (phase sequence << 8) | where (a wait that never completed)
constexpr uint32_t kWsDbg = 33;      // [2] the leader's sweep of the launch and its step (diagnostics)
constexpr uint32_t kWsTime = 48;     // u64 [16]: wall-clock ticks (100 MHz) per step of the leader's sweeps,
                                     // then finer probes (diagnostics)
constexpr uint32_t kWsWords = 96;
// Watchdogs (wall clock, 100 MHz): a leader wait or an acknowledgement pending this long flags
// DevState::err and ends the launch instead of spinning forever; an idle helper leaves after kWsIdle.
constexpr unsigned long long kWsWaitTicks = 200000000ull;    // 2 s
constexpr unsigned long long kWsIdleTicks = 3000000000ull;   // 30 s
constexpr unsigned long long kWsPollFastTicks = 200ull;       // 2 us (wall_clock64 runs at 100 MHz)
constexpr uint32_t kWsBShift = 16;   // window buckets: L >> 16
constexpr uint32_t kWsNB = ((kMinstdN - 1u) >> kWsBShift) + 1u;
constexpr uint32_t kWsCandCap = 2048;      // changing candidate rows the leader holds (more: no prefetch)
constexpr uint32_t kWsResLds = 4096;       // results the leader keeps in LDS (more: the global list)
constexpr uint32_t kWsEvLds = 4096;        // overflow events sorted in LDS (more: in global memory)
constexpr uint32_t kWsRankMax = 1024;      // events ranked and drawn in parallel (more: bitonic + sequential)
constexpr uint32_t kWsLeadLight = 256;     // violator arcs the leader walks on one wave (more: the workgroup)
constexpr uint32_t kWsLeadSets = 6;        // the leader's walk mask sets at most (as many as fit the LDS)
constexpr uint32_t kWsLeadList = 16384;    // violator-list updates the leader does itself
constexpr uint32_t kWsVvLds = 32;          // violators held in LDS for the candidates' test (more: counts)
constexpr uint32_t kWsPreLds = 16384;      // delta phase: changed rows whose arc prefix sits in LDS
constexpr uint32_t kWsChgLds = 4096;       // and whose entries (16 B) sit there too, after the prefix
constexpr uint32_t kWsLds = 136u * 1024u;  // dynamic LDS
static_assert(4u * (kWsPreLds + 4u * kWsChgLds) <= kWsLds, "delta phase prefix + entries in LDS");
enum : uint32_t { kWsRecount = 1, kWsExit = 2, kWsDelta = 3, kWsWalkLight = 4, kWsWalkHeavy = 5, kWsCopy = 6,
                  kWsCollect = 7, kWsPending = 8, kWsZero = 9, kWsDeltaR = 10, kWsGo = 11 };
constexpr uint32_t kWsArcsOut = 36;  // a kWsDeltaR phase's changed arcs (workgroup 1 writes them)
constexpr uint32_t kWsLeadN = 16;    // results up to which the leader takes the rows' offsets itself

struct WsArgs {
    uint32_t* ctl;
    uint32_t* vl;          // [2][nloc] violator lists (parity of t)
    uint32_t* flag;        // [nloc] bytes: row in the current violator list
    uint32_t* res;         // [2 nloc] the sweep's results (l, cv | nc << 16; nc = nCol: an overflow)
    uint32_t* chg;         // [4 nloc] its changed rows (l, cov | cnv << 16, row start lo, hi)
    uint32_t* pre;         // [nloc + 1] their arcs' exclusive prefix
    uint32_t* tch;         // [nloc] rows whose count left 0
    uint32_t* heavy;       // [nloc] violators walked by a workgroup; then the events' drawn colours (by row)
    const uint32_t* wL;    // window logarithms, ascending
    const uint32_t* ww;    // the window states, same order
    const uint32_t* boff;  // [kWsNB + 1] first entry of each bucket
    uint32_t nw;           // window states
    uint32_t lead_arcs;    // changed arcs the leader moves itself (more: a delta phase)
    uint32_t light_arcs;   // violators of at most this many arcs walk on one wave
    uint32_t lead_heavy;   // heavier violators' arcs (in all) the leader walks itself, a workgroup each
    uint32_t sets;         // wave mask sets per workgroup
    uint32_t* dbg;         // diagnostics (MCMC_WS_DEBUG): host-visible progress words, or nullptr
    uint32_t poll;         // a helper's poll interval (s_sleep 2 units; MCMC_WS_POLL) for kWsPollFastTicks
    uint32_t poll_idle;    // after a phase, then this one (MCMC_WS_POLL_IDLE): fewer coherent loads while
                           // the leader runs its steps, ~0.4 us more wake-up latency on average
    uint32_t* gcand;       // [3 nloc] the next sweep's candidates that change colour in case (iii)
                           // (l, x, cv | nc << 16), found by the helpers during a delta phase
};

// The candidates of the sweep whose minstd log is lxv: window entries with L in [lxv + 1,
// lxv + 1 + n) mod (2^31 - 2) -- one or two runs of the table. Entry j (< *tot) of the runs: its
// row l (the vertex drawing state x) when it lies in them.
struct WsRuns {
    uint32_t lo, r1a, r1b, ea0, ea1, eb1, tot;
};
__device__ __forceinline__ WsRuns ws_runs(const WsArgs& w, uint32_t lxv, uint32_t nloc) {
    WsRuns r;
    r.lo = lxv + 1u >= kMinstdN ? lxv + 1u - kMinstdN : lxv + 1u;
    r.r1a = (uint32_t)min<uint64_t>((uint64_t)r.lo + nloc, kMinstdN);
    r.r1b = (uint64_t)r.lo + nloc > kMinstdN ? (uint32_t)((uint64_t)r.lo + nloc - kMinstdN) : 0u;
    r.ea0 = w.boff[r.lo >> kWsBShift];
    r.ea1 = w.boff[((r.r1a - 1u) >> kWsBShift) + 1u];
    r.eb1 = r.r1b ? w.boff[((r.r1b - 1u) >> kWsBShift) + 1u] : 0u;
    r.tot = (r.ea1 - r.ea0) + r.eb1;
    return r;
}
__device__ __forceinline__ bool ws_entry(const WsArgs& w, const WsRuns& r, uint32_t j0, uint32_t& l, uint32_t& x) {
    const bool ra = j0 < r.ea1 - r.ea0;
    const uint32_t j = ra ? r.ea0 + j0 : j0 - (r.ea1 - r.ea0);
    const uint32_t L = w.wL[j];
    x = w.ww[j];
    l = ra ? L - r.lo : L + (kMinstdN - r.lo);
    return ra ? (L >= r.lo && L < r.r1a) : (L < r.r1b);
}
// fill_p case (iii) (own colour hi, others eps) for a row of colour cv and state x: the new colour
// (nCol: an overflow).
__device__ __forceinline__ uint32_t ws_own_walk(const SweepArgs& a, uint32_t cv, uint32_t x) {
    const float u = minstd_canonical(x);
    if (u < a.emax && x - 1u < a.ftab_n) {
        const uint32_t F = a.ftab[x - 1u];
        return F <= cv ? F - 1u : cv;
    }
    return walk_own_tab(a.etab, a.nCol, cv, a.eps, a.hi, u);
}
// Progress words in host memory (MCMC_WS_DEBUG): readable while a launch runs.
__device__ __forceinline__ void ws_dbg(const WsArgs& w, uint32_t i, uint32_t v) {
    if (w.dbg != nullptr) __hip_atomic_store(&w.dbg[i], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A colour read coherently across workgroups without an acquire fence (a relaxed agent-scope load:
// no L2 invalidation, see ws_kernel's hand-off notes).
__device__ __forceinline__ uint32_t ld16c(const uint16_t* p) {
    return __hip_atomic_load(reinterpret_cast<const unsigned short*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// w[i] = the i-th state of the window [1, lo) U [hi, 2^31 - 1), L[i] = its logarithm; err |= 1 if a
// logarithm fails its check 16807^L = w.
__global__ __launch_bounds__(256) void ws_table_kernel(uint32_t* __restrict__ L, uint32_t* __restrict__ w, uint32_t lo,
                                                       uint32_t hi, uint32_t nw, uint32_t* __restrict__ err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nw) return;
    const uint32_t s = i < lo - 1u ? 1u + i : hi + (i - (lo - 1u));
    const uint32_t l = minstd_dlog(s);
    if (l == 0xFFFFFFFFu || minstd_pow(kMinstdA, l) != s) atomicOr(err, 1u);
    L[i] = l;
    w[i] = s;
}
// boff[b] = first i with L[i] >= b << kWsBShift (b <= kWsNB)
__global__ __launch_bounds__(256) void ws_bucket_kernel(const uint32_t* __restrict__ L, uint32_t nw,
                                                        uint32_t* __restrict__ boff) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b > kWsNB) return;
    const uint64_t key = (uint64_t)b << kWsBShift;
    uint32_t lo = 0, hi = nw;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((uint64_t)L[mid] < key) lo = mid + 1u; else hi = mid;
    }
    boff[b] = lo;
}

// Prefix counts of a mask (one wave: word runs per lane) and the walk of fill_p case (ii) / (i) --
// walk_finish_wave's selection without its writes. All 64 lanes call it; returns the new colour or
// nCol (an overflow), the same on every lane.
__device__ __forceinline__ uint32_t ws_mask_walk(const SweepArgs& a, const uint32_t* mask, uint32_t* pre, uint32_t cv,
                                                 float u, uint32_t lane) {
    const uint32_t NWW = (a.nCol + 31u) >> 5, per = (NWW + 63u) >> 6, w0 = lane * per;
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
    uint32_t nc;
    if (Zvcomp > 0) {   // case (ii)
        const float pf = (1.0f - a.eps * (float)P) / (float)Zvcomp;
        nc = walk_mask_pre(mask, pre, a.nCol, a.eps, pf, u, a.walk_tie != 0u);
    } else {            // case (i)
        nc = walk_own_tab(a.etab, a.nCol, cv, a.eps, a.hi, u);
    }
    wave_lds_sync();
    return __builtin_amdgcn_readfirstlane(nc);
}

// A result (lane's row l: colour cv -> nc), wave-aggregated into the global list.
__device__ __forceinline__ void ws_push(const WsArgs& w, bool want, uint32_t l, uint32_t cv, uint32_t nc, uint32_t lane) {
    const uint64_t m = __ballot(want);
    if (m == 0) return;
    const int lead = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if ((int)lane == lead) base = atomicAdd(&w.ctl[kWsResN], (uint32_t)__popcll(m));
    base = __shfl(base, lead, 64);
    if (want) {
        const uint32_t j = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        w.res[2u * j] = l;
        w.res[2u * j + 1u] = cv | (nc << 16);
    }
}
__device__ __forceinline__ void ws_touch(const SweepArgs& a, const WsArgs& w, uint32_t l) {
    const uint32_t idx = atomicAdd(&w.ctl[kWsTchN], 1u);
    if (idx < a.v_end - a.v_begin) w.tch[idx] = l;
    else atomicOr(&w.ctl[kWsTchOvf], 1u);
}

// One light violator on one wave: its occupancy mask in the wave's set, its walk, the result.
// Results go to (rcnt, rbuf): the global list (helpers) or the leader's LDS list. COH: colours read
// with coherent loads (a helper phase without an acquire).
template <bool COH>
__device__ __forceinline__ void ws_walk_light(const SweepArgs& a, const uint16_t* __restrict__ C, uint32_t x_t,
                                              uint32_t l, uint32_t* mask, uint32_t lane, uint32_t* rcnt, uint32_t* rbuf) {
    const uint32_t NWW = (a.nCol + 31u) >> 5;
    uint32_t* pre = mask + ((NWW + 3u) & ~3u);
    const uint32_t cv = COH ? ld16c(&C[l]) : C[l];
    const uint32_t x = minstd_mulmod(x_t, minstd_pow_tab_wave((uint64_t)l + 1ull));   // u_v (:139)
    for (uint32_t i = lane; i < NWW; i += 64u) mask[i] = 0u;
    wave_lds_sync();
    {   // walk_gather_wave with the colour loads COH
        const uint64_t k0 = a.row_off[l], k1 = a.row_off[l + 1];
        for (uint64_t k = k0 + lane; k < k1; k += 8u * 64u) {
            uint32_t c[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint64_t kk = k + (uint64_t)j * 64u;
                c[j] = kk < k1 ? (COH ? ld16c(&C[a.col_idx[kk]]) : (uint32_t)C[a.col_idx[kk]]) : 0xFFFFFFFFu;
            }
#pragma unroll
            for (int j = 0; j < 8; j++)
                if (c[j] != 0xFFFFFFFFu) atomicOr(&mask[c[j] >> 5], 1u << (c[j] & 31u));
        }
    }
    wave_lds_sync();
    const uint32_t nc = ws_mask_walk(a, mask, pre, cv, minstd_canonical(x), lane);
    if (lane == 0 && nc != cv) {
        const uint32_t j = atomicAdd(rcnt, 1u);
        rbuf[2u * j] = l;
        rbuf[2u * j + 1u] = cv | (nc << 16);
    }
}
// One heavy violator on the whole workgroup (mask set 0); all threads call it.
template <bool COH>
__device__ __forceinline__ void ws_walk_heavy(const SweepArgs& a, const uint16_t* __restrict__ C, uint32_t x_t,
                                              uint32_t l, uint32_t* mask, uint32_t* rcnt, uint32_t* rbuf) {
    const uint32_t NWW = (a.nCol + 31u) >> 5, lane = threadIdx.x & 63u;
    uint32_t* pre = mask + ((NWW + 3u) & ~3u);
    for (uint32_t i = threadIdx.x; i < NWW; i += blockDim.x) mask[i] = 0u;
    __syncthreads();
    {   // the row's occupancy: 16 gathers per thread in flight (a hub: ~2 rounds at C5)
        const uint64_t k0 = a.row_off[l], k1 = a.row_off[l + 1];
        for (uint64_t k = k0 + threadIdx.x; k < k1; k += 16u * blockDim.x) {
            uint32_t c[16];
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const uint64_t kk = k + (uint64_t)j * blockDim.x;
                c[j] = kk < k1 ? (COH ? ld16c(&C[a.col_idx[kk]]) : (uint32_t)C[a.col_idx[kk]]) : 0xFFFFFFFFu;
            }
#pragma unroll
            for (int j = 0; j < 16; j++)
                if (c[j] != 0xFFFFFFFFu) atomicOr(&mask[c[j] >> 5], 1u << (c[j] & 31u));
        }
    }
    __syncthreads();
    if (threadIdx.x < 64u) {
        const uint32_t cv = COH ? ld16c(&C[l]) : C[l];
        const uint32_t x = minstd_mulmod(x_t, minstd_pow_tab_wave((uint64_t)l + 1ull));
        const uint32_t nc = ws_mask_walk(a, mask, pre, cv, minstd_canonical(x), lane);
        if (lane == 0 && nc != cv) {
            const uint32_t j = atomicAdd(rcnt, 1u);
            rbuf[2u * j] = l;
            rbuf[2u * j + 1u] = cv | (nc << 16);
        }
    }
    __syncthreads();
}

// Arcs [k, k1) (step) of the flattened changed-row arcs: both ends' counts move by [Cn equal] -
// [Cp equal] (an arc whose other end changed too only from the smaller end; self-arcs never move).
// pre: the prefix (LDS or global), nch changed rows.
// chs: the changed-row entries in LDS (a helper that copied them), else nullptr; elate: their
// colours are not in chs (a kWsDeltaR phase built it before the events drew): read from the list.
// A listed row whose colour did not change (an overflow that drew its own) moves nothing: an arc to
// a changed row is counted from that row's side.
template <bool COH>   // COH: the list and the colours read with coherent loads (a helper, no acquire)
__device__ __forceinline__ void ws_delta_arcs(const SweepArgs& a, const WsArgs& w, const uint16_t* __restrict__ Cp,
                                              const uint16_t* __restrict__ Cn, const uint32_t* pre, uint32_t nch,
                                              uint32_t k, uint32_t k1, uint32_t step, const uint4* chs = nullptr,
                                              bool elate = false) {
    const uint32_t nloc = a.v_end - a.v_begin;
    for (; k < k1; k += step) {
        uint32_t lo = 0, hi = nch;   // the changed row i with pre[i] <= k < pre[i + 1]
        while (hi - lo > 1u) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pre[mid] <= k) lo = mid; else hi = mid;
        }
        uint4 ch;
        if (chs != nullptr) {
            ch = chs[lo];
            if (elate) ch.y = dc_ld(&w.chg[4u * lo + 1u]);
        } else if (COH) {
            ch.x = dc_ld(&w.chg[4u * lo]);
            ch.y = dc_ld(&w.chg[4u * lo + 1u]);
            ch.z = dc_ld(&w.chg[4u * lo + 2u]);
            ch.w = dc_ld(&w.chg[4u * lo + 3u]);
        } else {
            ch = reinterpret_cast<const uint4*>(w.chg)[lo];
        }
        const uint32_t v = ch.x, cov = ch.y & 0xFFFFu, cnv = ch.y >> 16;
        const uint32_t u = a.col_idx[(((uint64_t)ch.w << 32) | ch.z) + (k - pre[lo])];
        if (cov == cnv) continue;
        if (u == v) continue;
        const uint32_t ou = COH ? ld16c(&Cp[u]) : Cp[u], nu = COH ? ld16c(&Cn[u]) : Cn[u];
        if (ou != nu && u < v) continue;
        const int d = (int)(nu == cnv) - (int)(ou == cov);
        if (d == 0) continue;
        if (u < nloc) {
            const uint32_t old = atomicAdd(&a.inc_vcnt[u], (uint32_t)d);
            if (d > 0 && old == 0u) ws_touch(a, w, u);
        }
        const uint32_t old = atomicAdd(&a.inc_vcnt[v], (uint32_t)d);
        if (d > 0 && old == 0u) ws_touch(a, w, v);
    }
}

// Exclusive scan of one value per thread over the workgroup; *tot = the sum. All threads call it.
__device__ __forceinline__ uint32_t ws_scan(uint32_t v, uint32_t* wsum, uint32_t* tot) {
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    uint32_t inc = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63u) wsum[wv] = inc;
    dc_lbar();
    uint32_t off = 0, s = 0;
    for (uint32_t k = 0; k < nwv; k++) {
        if (k < wv) off += wsum[k];
        s += wsum[k];
    }
    *tot = s;
    dc_lbar();
    return off + inc - v;
}

// ---- helper phases (workgroups 1..G-1; h = blockIdx.x - 1 of H) ---------------------------------
// last: the phase word this workgroup has seen (a kWsDeltaR phase moves it on to its kWsGo post);
// gone: a kWsDeltaR phase whose go this workgroup saw first (its poll slept through the phase's
// own post), so it does the phase without waiting.
__device__ __forceinline__ void ws_help(const SweepArgs& a, const WsArgs& w, uint32_t kind, uint32_t* dyn, uint32_t& last,
                                        bool gone) {
    const uint32_t H = gridDim.x - 1u, h = blockIdx.x - 1u, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t gt = h * blockDim.x + threadIdx.x, GT = H * blockDim.x;
    const uint32_t nloc = a.v_end - a.v_begin;
    const uint32_t t = dc_ld(&w.ctl[kWsArgT]), P = dc_ld(&w.ctl[kWsArgP]);
    const uint16_t* __restrict__ C = reinterpret_cast<const uint16_t*>((t & 1) ? a.colors1 : a.colors0);   // C_t
    uint16_t* __restrict__ Cs = reinterpret_cast<uint16_t*>((t & 1) ? a.colors0 : a.colors1);
    if (kind == kWsZero) {   // counts to zero (a recount follows)
        for (uint32_t l = gt; l < nloc; l += GT) a.inc_vcnt[l] = 0u;
    } else if (kind == kWsCopy) {   // the other buffer = C_t (whole replica, 16 B at a time)
        const uint32_t n4 = (a.n * 2u + 15u) / 16u;
        const uint4* s = reinterpret_cast<const uint4*>(C);
        uint4* d = reinterpret_cast<uint4*>(Cs);
        for (uint32_t i = gt; i < n4; i += GT) d[i] = s[i];
    } else if (kind == kWsRecount) {   // every arc (r, u) with C_t[u] = C_t[r]: count of r (violation_count, :329-351)
        const uint64_t* __restrict__ ro = a.row_off;
        const uint64_t a0 = a.arc_begin, m = a.arc_count;
        const uint32_t gw = gt >> 6, nwv = GT >> 6;
        for (uint32_t ch = gw; ch < a.nchunks; ch += nwv) {
            const uint64_t k0 = (uint64_t)ch * kWideChunk + 4u * lane;
            if (k0 >= m) continue;
            const uint4 q = *reinterpret_cast<const uint4*>(a.col_idx + a0 + k0);
            uint32_t id[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int i = 1; i < 4; i++)
                if (k0 + i >= m) id[i] = 0u;
            uint32_t nc[4];
#pragma unroll
            for (int i = 0; i < 4; i++) nc[i] = C[id[i]];
            uint32_t lo = a.chunk_row[ch], hi = a.chunk_row[ch + 1];
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1u) >> 1;
                if (ro[mid] - a0 <= k0) lo = mid; else hi = mid - 1u;
            }
            uint32_t r = lo;
            uint64_t rend = ro[r + 1] - a0;
            uint32_t own = C[r];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint64_t k = k0 + i;
                if (k >= m) break;
                if (rend <= k) {
                    do { r++; rend = ro[r + 1] - a0; } while (rend <= k);
                    own = C[r];
                }
                if (nc[i] == own) atomicAdd(&a.inc_vcnt[r], 1u);
            }
        }
    } else if (kind == kWsCollect) {   // the violator list P and the flags, from the counts
        for (uint32_t q0 = gt & ~63u; q0 * 4u < nloc; q0 += GT) {
            const uint32_t q = q0 + lane, l0 = 4u * q;
            uint32_t f = 0, fl[4] = {0, 0, 0, 0};
            if (l0 < nloc) {
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    fl[i] = (l0 + i < nloc && a.inc_vcnt[l0 + i] > 0u) ? 1u : 0u;
                    f |= fl[i] << (8 * i);
                }
                w.flag[q] = f;
            }
            const uint32_t cnt = __popc(f);
            uint32_t inc = cnt;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(inc, o, 64);
                if (lane >= (uint32_t)o) inc += y;
            }
            uint32_t base = 0;
            const uint32_t tot = __shfl(inc, 63, 64);
            if (lane == 63u && tot) base = atomicAdd(&w.ctl[kWsVn + P], tot);
            base = __shfl(base, 63, 64) + inc - cnt;
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (fl[i]) w.vl[(size_t)P * nloc + base++] = l0 + i;
        }
    } else if (kind == kWsWalkLight) {
        // violator list P: entries h, h + H, ... of this workgroup; its waves walk the light ones
        // (one each), then the whole workgroup the heavy ones (listed in LDS)
        const uint32_t Vn = dc_ld(&w.ctl[kWsVn + P]), x_t = dc_ld(&w.ctl[kWsArgP + 1]);
        const uint32_t* vl = w.vl + (size_t)P * nloc;
        __shared__ uint32_t s_hn, s_hv[64];
        if (threadIdx.x == 0) s_hn = 0;
        __syncthreads();
        if (wv < w.sets) {
            uint32_t* mask = dyn + wv * walk_set_words(a.nCol);
            for (uint32_t i = h + H * wv; i < Vn; i += H * w.sets) {
                const uint32_t l = dc_ld(&vl[i]);
                if (a.row_off[l + 1] - a.row_off[l] > w.light_arcs) {
                    if (lane == 0) {
                        const uint32_t j = atomicAdd(&s_hn, 1u);
                        if (j < 64u) s_hv[j] = l;
                        else w.heavy[atomicAdd(&w.ctl[kWsHeavyN], 1u)] = l;
                    }
                    continue;
                }
                ws_walk_light<true>(a, C, x_t, l, mask, lane, &w.ctl[kWsResN], w.res);
            }
        }
        __syncthreads();
        const uint32_t hn = min(s_hn, 64u);
        for (uint32_t j = 0; j < hn; j++) ws_walk_heavy<true>(a, C, x_t, s_hv[j], dyn, &w.ctl[kWsResN], w.res);
    } else if (kind == kWsWalkHeavy) {
        const uint32_t hn = dc_ld(&w.ctl[kWsHeavyN]), x_t = dc_ld(&w.ctl[kWsArgP + 1]);
        for (uint32_t j = h; j < hn; j += H)
            ws_walk_heavy<true>(a, C, x_t, dc_ld(&w.heavy[j]), dyn, &w.ctl[kWsResN], w.res);
    } else if (kind == kWsDelta || kind == kWsDeltaR) {
        // the changed rows' arcs (prefix cached in LDS where it fits). This phase runs without an
        // acquire (no L2 invalidation on every XCD per sweep): what the leader wrote for it -- the
        // list, the prefix, the colours of C_t+1 -- is read with coherent loads
        const uint32_t nch = dc_ld(&w.ctl[kWsChgN]);
        const uint32_t* pre = w.pre;
        const uint4* chs = nullptr;
        if (kind == kWsDeltaR) {
            // kWsDeltaR: posted before the leader's event draws with the results' rows only (nch <=
            // kWsChgLds): every workgroup loads the rows' offsets and builds the entries and the
            // arcs' prefix in its LDS meanwhile; on the leader's kWsGo post (the colours out, the
            // events' draws in) the arcs run, each reading its row's colours from the list -- the
            // offsets' round trip and the scans leave the leader's critical path
            __shared__ uint32_t s_ds[16], s_go;
            uint32_t* const pl = dyn;
            uint4* const cs = reinterpret_cast<uint4*>(dyn + kWsPreLds);
            const uint32_t per = (nch + blockDim.x - 1u) / blockDim.x;   // (<= 4)
            const uint32_t i0 = min(nch, threadIdx.x * per), i1 = min(nch, i0 + per);
            uint32_t l[4], d[4], dsum = 0;
            uint64_t r0[4], r1[4];
#pragma unroll
            for (int u = 0; u < 4; u++) l[u] = i0 + (uint32_t)u < i1 ? dc_ld(&w.chg[4u * (i0 + u)]) : 0u;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const bool in = i0 + (uint32_t)u < i1;
                r0[u] = in ? a.row_off[l[u]] : 0ull;
                r1[u] = in ? a.row_off[l[u] + 1u] : 0ull;
            }
            // every listed row's arcs (an unchanged one's move nothing: ws_delta_arcs skips them), so
            // the prefix needs no colours and is ready before the go
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t i = i0 + (uint32_t)u;
                d[u] = (uint32_t)(r1[u] - r0[u]);
                dsum += d[u];
                if (i < i1) cs[i] = make_uint4(l[u], 0u, (uint32_t)r0[u], (uint32_t)(r0[u] >> 32));
            }
            uint32_t tot = 0;
            uint32_t run = ws_scan(dsum, s_ds, &tot);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (i0 + (uint32_t)u < i1) pl[i0 + u] = run;
                run += d[u];
            }
            if (threadIdx.x == 0) {
                pl[nch] = tot;
                if (h == 0u) w.ctl[kWsArcsOut] = tot;
            }
            if (threadIdx.x < 64u) {   // wave 0 waits for the go (wave-uniform; a watchdog as the leader's)
                const unsigned long long t0 = wall_clock64();
                uint32_t g2 = last;
                while (!gone && (g2 = __builtin_amdgcn_readfirstlane(dc_ld(&w.ctl[kWsGen]))) == last) {
                    if (wall_clock64() - t0 > kWsWaitTicks) {
                        if (threadIdx.x == 0) a.st->err |= kDevErrWatchdog;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (threadIdx.x == 0) s_go = g2;
            }
            __syncthreads();
            const uint32_t go = s_go;
            if ((go & 15u) != kWsGo) return;   // the leader left (its exit post): no moves
            last = go;
            pre = pl;
            chs = cs;
        } else if (nch + 1u <= kWsPreLds) {   // the entries too where they fit: one round trip for both, so an
            // arc's chain is prefix search (LDS) -> its id -> the colours -> the count atomics
            const bool cl = nch <= kWsChgLds;
            for (uint32_t i = threadIdx.x; i <= nch; i += blockDim.x) dyn[i] = dc_ld(&w.pre[i]);
            if (cl)
                for (uint32_t i = threadIdx.x; i < 4u * nch; i += blockDim.x) dyn[kWsPreLds + i] = dc_ld(&w.chg[i]);
            __syncthreads();
            pre = dyn;
            if (cl) chs = reinterpret_cast<const uint4*>(dyn + kWsPreLds);
        }
        // arcs dealt round-robin over the workgroups (h, h + H, ...): a few thousand random reads
        // spread over every CU rather than filling the first few
        const uint32_t tot = (kind == kWsDeltaR || nch + 1u <= kWsPreLds) ? pre[nch] : dc_ld(&w.pre[nch]);
        // the last wave of every workgroup takes the next sweep's candidates, the others the arcs:
        // the two dependent-load chains run side by side instead of one after the other
        const uint32_t na = blockDim.x - 64u;
        if (wv != (blockDim.x >> 6) - 1u) {
            ws_delta_arcs<true>(a, w, C, Cs, pre, nch, h + H * threadIdx.x, tot, H * na, chs, kind == kWsDeltaR);
            return;
        }
        // the next sweep's candidates (its colours: C_t+1, in Cs): those that change colour unless
        // they turn out violators, into gcand -- a slice of the entries per workgroup
        const WsRuns r = ws_runs(w, dc_ld(&w.ctl[kWsArgL]), nloc);
        const uint32_t per = (r.tot + H - 1u) / H, jb = min(r.tot, h * per), je = min(r.tot, jb + per);
        for (uint32_t j0 = jb; j0 < je; j0 += 64u) {   // (wave-uniform bounds)
            uint32_t l = 0, x = 1, cv = 0, nc = 0;
            bool in = j0 + lane < je && ws_entry(w, r, j0 + lane, l, x);
            if (in) {
                cv = ld16c(&Cs[l]);
                nc = ws_own_walk(a, cv, x);
                in = nc != cv;
            }
            const uint64_t m = __ballot(in);
            if (m == 0) continue;
            const int ld = __ffsll((long long)m) - 1;
            uint32_t b = 0;
            if ((int)lane == ld) b = atomicAdd(&w.ctl[kWsCandN], (uint32_t)__popcll(m));
            b = __shfl(b, ld, 64);
            if (in) {
                const uint32_t k = b + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                w.gcand[3u * k] = l;
                w.gcand[3u * k + 1u] = x;
                w.gcand[3u * k + 2u] = cv | (nc << 16);
            }
        }
    } else if (kind == kWsPending) {   // the last per-sweep commit's changed rows: C_t-1 (buffer of t-1) -> C_t
        const uint32_t p = t & 1u;
        const uint16_t* Cp = Cs;   // the buffer of C_t-1 (sweep t writes it next)
        const uint32_t nd = a.inc[kIncDenseN + p], nh = a.inc[kIncHubN + p];
        for (uint32_t i = h; i < nh; i += H) {   // hubs: a workgroup each
            const uint32_t v = a.inc_hub[(size_t)p * a.inc_lcap + i];
            int dv = inc_arcs(a, Cp, C, v, Cp[v], C[v], a.row_off_g[v] + threadIdx.x, a.row_off_g[v + 1], blockDim.x, t);
            for (int o = 32; o > 0; o >>= 1) dv += __shfl_xor(dv, o, 64);
            if (lane == 0 && dv != 0) {
                const uint32_t old = atomicAdd(&a.inc_vcnt[v], (uint32_t)dv);
                (void)old;
            }
        }
        const uint32_t gw = gt >> 6, nwv = GT >> 6;
        const uint32_t* dn = a.inc_dense + (size_t)p * a.inc_lcap;
        for (uint32_t i = gw; i < nd; i += nwv) {   // other rows: a wave each
            const uint32_t v = dn[i];
            int dv = inc_arcs(a, Cp, C, v, Cp[v], C[v], a.row_off_g[v] + lane, a.row_off_g[v + 1], 64u, t);
            for (int o = 32; o > 0; o >>= 1) dv += __shfl_xor(dv, o, 64);
            if (lane == 0 && dv != 0) atomicAdd(&a.inc_vcnt[v], (uint32_t)dv);
        }
    }
}

// The leader's loop state (LDS).
struct WsState {
    uint32_t t, x_t, lx, done, err, nres;
    uint32_t ring[31];
    unsigned long long draws;
    unsigned long long st[8];
    unsigned long long arcs;        // the changed rows' arcs (the incremental statistics)
    uint32_t recounts;
    unsigned long long tm[16], t0, ts, tp, tc;   // ticks per step: walks, candidates, walk wait, events, changes,
                                    // count moves, violator list, whole sweeps
};


__global__ __launch_bounds__(1024) void ws_kernel(SweepArgs a, WsArgs w, uint32_t K) {
    extern __shared__ uint4 ws_lds[];
    uint32_t* const dyn = reinterpret_cast<uint32_t*>(ws_lds);
    __shared__ uint32_t sh_g;
    DevState* __restrict__ st = a.st;
    const uint32_t nloc = a.v_end - a.v_begin, G = gridDim.x;
    if (blockIdx.x != 0) {   // helpers: phases until the exit post
        uint32_t last = 0;
        for (;;) {
            // the whole of wave 0 polls (a wave-uniform loop: a spin loop in one lane beside barriers
            // in the others lets the compiler's structurizer run the other lanes of the wave ahead)
            if (threadIdx.x < 64u) {
                uint32_t g;
                const unsigned long long t0 = wall_clock64();
                for (;;) {
                    g = __builtin_amdgcn_readfirstlane(dc_ld(&w.ctl[kWsGen]));
                    if (g != last) break;
                    const unsigned long long idle = wall_clock64() - t0;
                    if (idle > kWsIdleTicks) { g = kWsExit; break; }
                    const uint32_t zs = idle > kWsPollFastTicks ? w.poll_idle : w.poll;
                    for (uint32_t z = 0; z < zs; z++) __builtin_amdgcn_s_sleep(2);   // (0: spin)
                }
                if ((g & 15u) != kWsDelta && (g & 15u) != kWsDeltaR && (g & 15u) != kWsGo &&
                    (g & 15u) != kWsWalkLight && (g & 15u) != kWsWalkHeavy) {
                    // (the per-sweep phases read what the leader wrote coherently instead)
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                if (threadIdx.x == 0) sh_g = g;
            }
            __syncthreads();
            const uint32_t g = sh_g;
            last = g;
            __syncthreads();
            if ((g & 15u) == kWsExit) break;
            if (threadIdx.x == 0) ws_dbg(w, 64u + blockIdx.x, (g << 4) | 1u);
            ws_help(a, w, (g & 15u) == kWsGo ? kWsDeltaR : g & 15u, dyn, last, (g & 15u) == kWsGo);
            if (threadIdx.x == 0) ws_dbg(w, 64u + blockIdx.x, (g << 4) | 2u);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                atomicAdd(&w.ctl[kWsDone], 1u);
            }
        }
        if (threadIdx.x == 0) atomicAdd(&w.ctl[kWsAck], 1u);
        return;
    }
    // ---- the leader ----
    __shared__ WsState s;
    __shared__ uint32_t s_seq, s_exp, s_nc, s_ne, s_nr, s_wsum[16], s_nh, s_vq, s_w[4], s_pf, s_gn;
    __shared__ uint32_t s_ring[31], s_rawok, s_ha, s_hl[kWsLeadSets], s_vv[kWsVvLds];
    uint32_t* const cand = dyn;                              // [3 kWsCandCap] candidates (l, x, cv | nc << 16)
    uint32_t* const tmp = cand + 3u * kWsCandCap;            // [kWsResLds] raw draws, event vertices, degrees
    uint32_t* const lres = tmp + kWsResLds;                  // [2 kWsResLds] the sweep's results
    uint32_t* const evl = lres + 2u * kWsResLds;             // [kWsEvLds] overflow events (result indices)
    uint32_t* const sets = evl + kWsEvLds;                   // lead_sets mask sets
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    // a phase for the helpers: every wave's stores drained, release, the flag; then wait for all
    auto post = [&](uint32_t kind) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0 && (s.err == 0u || kind == kWsExit)) {
            s_seq++;
            s_exp += G - 1u;
            s.st[1]++;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(&w.ctl[kWsGen], (s_seq << 4) | kind, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
    };
    // the second post of a kWsDeltaR phase: its results' colours are out (no new phase: the
    // helpers already count it)
    auto post_go = [&]() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0 && s.err == 0u) {
            s_seq++;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(&w.ctl[kWsGen], (s_seq << 4) | kWsGo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
    };
    // acq: an acquire after the phase (L2 invalidation): the rare phases whose plain writes the
    // leader then reads plainly; the per-sweep ones are read back with coherent loads instead
    auto wait = [&](bool acq = true) {   // wave 0 waits (a wave-uniform loop, as the helpers poll)
        if (threadIdx.x < 64u && __builtin_amdgcn_readfirstlane(s.err) == 0u) {
            const unsigned long long t0 = wall_clock64();
            const uint32_t ex = __builtin_amdgcn_readfirstlane(s_exp);
            for (;;) {
                const uint32_t d = __builtin_amdgcn_readfirstlane(dc_ld(&w.ctl[kWsDone]));
                if (d >= ex) break;
                if (w.dbg != nullptr && threadIdx.x == 0) {
                    ws_dbg(w, 3, d);
                    ws_dbg(w, 4, ex);
                }
                if (wall_clock64() - t0 > kWsWaitTicks) {   // a phase that never completed: flag and leave
                    if (threadIdx.x == 0) {
                        w.ctl[kWsErr] = (s_seq << 8) | 1u;
                        st->err |= kDevErrWatchdog;
                        s.err = 1u;
                    }
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (acq) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __syncthreads();
    };
    auto probe = [&](uint32_t i) {   // tm[8 + i] += ticks since the last probe (i = 0: restart)
        if (threadIdx.x == 0) {
            const unsigned long long now = wall_clock64();
            if (i) s.tm[8 + i] += now - s.tp;
            s.tp = now;
        }
    };
    // The next kWsRankMax raw glibc draws from the window s.ring (draw r = sum_m T[m][r] ring[m], the
    // commit's table) into raw = evl + kWsRankMax, one per thread. They depend on the window only, so
    // the leader computes them while the helpers move the last sweep's counts (s_rawok: valid for
    // the current window), off the event step's critical path.
    auto draws = [&]() {
        // the lane's table column from one opaque base per call: hipcc otherwise hoists the 31
        // per-lane addresses out of the sweep loop, where they outlive the registers and spill
        const uint32_t* tp = kGlibcTab + threadIdx.x;
        asm volatile("" : "+v"(tp));
        uint32_t tv[31];
#pragma unroll
        for (int m = 0; m < 31; m++) tv[m] = tp[m * kGlibcTabK];
        uint32_t acc = 0;
#pragma unroll
        for (int m = 0; m < 31; m++) acc += tv[m] * s.ring[m];
        evl[kWsRankMax + threadIdx.x] = acc;
    };
    static_assert(kWsRankMax == 1024u && kWsEvLds >= 2u * kWsRankMax, "one draw per leader thread");
    auto mark = [&](uint32_t k, uint32_t step) {
        if (threadIdx.x == 0) {
            const unsigned long long now = wall_clock64();
            if (step >= 2u && step <= 8u) s.tm[step - 2u] += now - s.t0;
            if (step == 8u) {
                s.tm[7] += now - s.ts;
                s.tm[8] += __builtin_amdgcn_s_memtime() - s.tc;   // [8] shader clocks of the sweeps
            }
            if (step == 1u) {
                s.ts = now;
                s.tc = __builtin_amdgcn_s_memtime();
            }
            if (step >= 1u && step <= 8u) s.t0 = now;
            w.ctl[kWsDbg] = k;
            w.ctl[kWsDbg + 1] = step;
            ws_dbg(w, 0, k);
            ws_dbg(w, 1, step);
            ws_dbg(w, 2, s_seq);
        }
    };
    if (threadIdx.x == 0) {   // take over the loop state
        const uint32_t head = st->glibc_head;
        s.t = st->t;
        s.done = st->done;
        s.err = st->err;
        s.x_t = st->x_t;
        s.lx = st->lx;
        for (uint32_t i = 0; i < 31u; i++) s.ring[i] = st->glibc_ring[(head + i) % 31u];
        s.draws = st->glibc_draws;
        for (int i = 0; i < 8; i++) s.st[i] = 0;
        s.arcs = 0;
        s.recounts = 0;
        for (int i = 0; i < 16; i++) s.tm[i] = 0;
        s_seq = 0;
        s_exp = 0;
        s_rawok = 0;
    }
    __syncthreads();
    const bool go = !(s.done || s.err);
    mark(0xFFFFu, 100u);
    if (go) {
        const uint32_t t = s.t, p = t & 1u;
        if (threadIdx.x == 0) {
            s_w[0] = a.inc[kIncMode];
            s_w[1] = a.inc[kIncDenseN + p] + a.inc[kIncHubN + p];
            s_w[2] = w.ctl[kWsT] == t + 1u ? 1u : 0u;
            w.ctl[kWsArgT] = t;
            w.ctl[kWsArgP + 1] = s.x_t;
        }
        __syncthreads();
        const uint32_t mode = s_w[0], pend = s_w[1];
        bool valid = s_w[2] != 0u;
        __syncthreads();
        mark(0xFFFFu, 101u + (mode ? 10u : 0u) + (pend ? 20u : 0u) + (valid ? 40u : 0u));
        if (mode) {   // a new colouring: recount (both buffers = C_t first)
            post(kWsZero);
            wait();
            post(kWsCopy);
            wait();
            post(kWsRecount);
            wait();
            valid = false;
            if (threadIdx.x == 0) s.recounts = 1;
        } else if (pend) {   // the last per-sweep commit's changes: their counts, then both buffers = C_t
            post(kWsPending);
            wait();
            post(kWsCopy);
            wait();
            valid = false;
        }
        if (threadIdx.x == 0) {
            a.inc[kIncMode] = 0u;
            a.inc[kIncDenseN + p] = a.inc[kIncHubN + p] = 0u;
            w.ctl[kWsTchN] = 0u;
            w.ctl[kWsTchOvf] = 0u;
        }
        if (!valid) {
            if (threadIdx.x == 0) {
                w.ctl[kWsVn + p] = 0u;
                w.ctl[kWsArgP] = p;
                s.st[5]++;
            }
            post(kWsCollect);
            wait();
        }
    }
    const uint32_t SW = walk_set_words(a.nCol);
    // The candidates of the sweep whose minstd log is lxv: window entries with L in [lxv + 1,
    // lxv + 1 + n) mod N (one or two runs of the table), their colours in Cb and the colour a case
    // (iii) walk gives them (fill_p own colour hi, others eps) into cand; s_nc = their number, or
    // 0xFFFFFFFF if more than the LDS holds (the sweep then runs them in rounds, rounds()).
    auto fetch = [&](uint32_t lxv, const uint16_t* __restrict__ Cb) {
        probe(0);
        const uint32_t lo = lxv + 1u >= kMinstdN ? lxv + 1u - kMinstdN : lxv + 1u;
        const uint32_t r1a = (uint32_t)min<uint64_t>((uint64_t)lo + nloc, kMinstdN);
        const uint32_t r1b = (uint64_t)lo + nloc > kMinstdN ? (uint32_t)((uint64_t)lo + nloc - kMinstdN) : 0u;
        const uint32_t ea0 = w.boff[lo >> kWsBShift], ea1 = w.boff[((r1a - 1u) >> kWsBShift) + 1u];
        const uint32_t eb1 = r1b ? w.boff[((r1b - 1u) >> kWsBShift) + 1u] : 0u;
        if (threadIdx.x == 0) s_nc = 0u;
        dc_lbar();
        probe(1);   // [9] the bucket bounds
        // 4 entries per thread per round, every load of a stage issued before the next stage's
        // (table entries -> colours and F(u) -> the eps-prefix walks)
        const uint32_t tot = (ea1 - ea0) + eb1;
        for (uint32_t b0 = 0; b0 < tot; b0 += 4u * blockDim.x) {
            uint32_t L[4], x[4], l[4], cv[4], F[4];
            bool in[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t j0 = b0 + (uint32_t)q * blockDim.x + threadIdx.x;
                const bool ra = j0 < ea1 - ea0;
                const uint32_t j = ra ? ea0 + j0 : j0 - (ea1 - ea0);
                in[q] = j0 < tot;
                L[q] = in[q] ? w.wL[j] : 0u;
                x[q] = in[q] ? w.ww[j] : 1u;
                in[q] = in[q] && (ra ? (L[q] >= lo && L[q] < r1a) : (L[q] < r1b));
                l[q] = ra ? L[q] - lo : L[q] + (kMinstdN - lo);
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                cv[q] = in[q] ? (uint32_t)Cb[l[q]] : 0u;
                const bool tab = in[q] && minstd_canonical(x[q]) < a.emax && x[q] - 1u < a.ftab_n;
                F[q] = tab ? (uint32_t)a.ftab[x[q] - 1u] : 0xFFFFFFFFu;
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                uint32_t ncol = cv[q];
                if (!in[q]) continue;
                if (F[q] != 0xFFFFFFFFu) ncol = F[q] <= cv[q] ? F[q] - 1u : cv[q];
                else ncol = walk_own_tab(a.etab, a.nCol, cv[q], a.eps, a.hi, minstd_canonical(x[q]));
                in[q] = in[q] && ncol != cv[q];   // (candidates that keep their colour need nothing)
                cv[q] |= ncol << 16;
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {   // appends: one LDS atomic per wave
                const uint64_t m = __ballot(in[q]);
                if (m == 0) continue;
                const int lead = __ffsll((long long)m) - 1;
                uint32_t b = 0;
                if ((int)(threadIdx.x & 63u) == lead) b = atomicAdd(&s_nc, (uint32_t)__popcll(m));
                b = __shfl(b, lead, 64);
                const uint32_t kk = b + (uint32_t)__popcll(m & ((1ull << (threadIdx.x & 63u)) - 1ull));
                if (in[q] && kk < kWsCandCap) {
                    cand[3u * kk] = l[q];
                    cand[3u * kk + 1u] = x[q];
                    cand[3u * kk + 2u] = cv[q];
                }
            }
        }
        dc_lbar();
        probe(2);   // [10] the entries, colours, walks
        if (threadIdx.x == 0) {
            s.st[6] += (ea1 - ea0) + eb1;
            if (s_nc > kWsCandCap) s_nc = 0xFFFFFFFFu;
        }
        dc_lbar();
    };
    // a result of the leader into its LDS list (past it: the global one)
    auto push = [&](uint32_t l, uint32_t e) {
        const uint32_t j = atomicAdd(&s_nr, 1u);
        if (j < kWsResLds) {
            lres[2u * j] = l;
            lres[2u * j + 1u] = e;
        } else {
            const uint32_t g = atomicAdd(&w.ctl[kWsResN], 1u);
            w.res[2u * g] = l;
            w.res[2u * g + 1u] = e;
        }
    };
    if (threadIdx.x == 0) s_pf = 0xFFFFFFFFu;   // no prefetched candidates yet
    __syncthreads();
    for (uint32_t k = 0; go && k < K; k++) {
        if (s.done || s.err) break;
        const uint32_t t = s.t, p = t & 1u, q = p ^ 1u;
        const uint16_t* __restrict__ C = reinterpret_cast<const uint16_t*>(p ? a.colors1 : a.colors0);   // C_t
        uint16_t* __restrict__ Cs = reinterpret_cast<uint16_t*>(p ? a.colors0 : a.colors1);          // = C_t too
        mark(k, 1);
        if (threadIdx.x == 0) s_w[3] = dc_ld(&w.ctl[kWsVn + p]);
        dc_lbar();
        const uint32_t Vn = s_w[3];
        const uint32_t* vl = w.vl + (size_t)p * nloc;
        // loop control (:136, :259-269): Cviol_t = the violators
        const unsigned long long viol = Vn;
        const bool stop = t == a.maxRip + 1u || (!a.bench && viol <= a.z);
        if (threadIdx.x == 0) {
            if (t < a.traj_cap) a.traj[t] = viol;
            if (stop) {
                st->done = 1u;
                st->iter = t;
                st->maxIterReached = t == a.maxRip + 1u ? 1u : 0u;
                st->finalViol = viol;
                s.done = 1u;
            }
            w.ctl[kWsResN] = 0u;
            w.ctl[kWsHeavyN] = 0u;
            w.ctl[kWsArgT] = t;
            w.ctl[kWsArgP] = p;
            w.ctl[kWsArgP + 1] = s.x_t;
            s_nh = 0;
            s_nr = 0;
            s_ha = 0;
        }
        __syncthreads();
        if (stop) break;
        // violators: the leader's waves walk a few light ones (the workgroup the heavier), else a walk
        // phase (overlapping the candidates). The leader's results go to its LDS list.
        bool walking = false;
        const uint32_t lead_sets = min(kWsLeadSets, (kWsLds / 4u - (uint32_t)(sets - dyn)) / SW);
        bool lead = Vn > 0u && Vn <= lead_sets;
        if (lead) {   // the leader walks them if the heavy ones (a workgroup each) are few arcs in all
            bool heavy = false;
            uint32_t l = 0;
            if (wv < Vn) {
                l = vl[wv];
                const uint32_t d = (uint32_t)(a.row_off[l + 1] - a.row_off[l]);
                heavy = d > kWsLeadLight;
                if (heavy && lane == 0) {
                    s_hl[atomicAdd(&s_nh, 1u)] = l;
                    atomicAdd(&s_ha, d);
                }
            }
            dc_lbar();
            lead = s_nh == 0u || s_ha <= w.lead_heavy;
            if (lead) {
                if (wv < Vn && !heavy) ws_walk_light<false>(a, C, s.x_t, l, sets + wv * SW, lane, &s_nr, lres);
                __syncthreads();
                const uint32_t nh = s_nh;
                for (uint32_t j = 0; j < nh; j++) ws_walk_heavy<false>(a, C, s.x_t, s_hl[j], sets, &s_nr, lres);
            }
        }
        if (lead) {
            dc_lbar();
            if (threadIdx.x == 0) s.st[2] += Vn;
        } else if (Vn > 0u) {
            post(kWsWalkLight);
            walking = true;
            if (threadIdx.x == 0) s.st[3]++;
        }
        mark(k, 2);
        // the candidates (fetched while the last sweep's counts moved, where they fit): those that are
        // not violators keep the colour their case (iii) walk gave; more than the LDS holds: in rounds
        const bool pre_g = s_pf == s.lx;   // the helpers found them during the last delta phase
        if (!pre_g) fetch(s.lx, C);
        // a candidate is walked above if it is a violator of C_t, i.e. in the (exact) violator list:
        // a short list is tested in LDS instead of by a dependent load of the candidate's count
        const bool vv = Vn <= kWsVvLds;
        if (vv && threadIdx.x < Vn) s_vv[threadIdx.x] = vl[threadIdx.x];
        dc_lbar();
        if (pre_g || s_nc != 0xFFFFFFFFu) {
            const uint32_t nc = pre_g ? s_gn : s_nc;
            const uint32_t* cl = pre_g ? w.gcand : cand;
            for (uint32_t b0 = wv * 64u; b0 < nc; b0 += blockDim.x) {   // (wave-uniform bounds)
                const uint32_t kk = b0 + lane;
                const uint32_t l = kk < nc ? (pre_g ? dc_ld(&cl[3u * kk]) : cl[3u * kk]) : 0u;
                const uint32_t e = kk < nc ? (pre_g ? dc_ld(&cl[3u * kk + 2u]) : cl[3u * kk + 2u]) : 0u;
                bool keep = kk < nc;
                if (vv) {
                    for (uint32_t q2 = 0; q2 < Vn; q2++) keep = keep && s_vv[q2] != l;
                } else {
                    keep = keep && dc_ld(&a.inc_vcnt[l]) == 0u;   // a violator: walked above
                }
                const uint64_t m = __ballot(keep);
                if (m == 0) continue;
                const int ld = __ffsll((long long)m) - 1;
                uint32_t b = 0;
                if ((int)lane == ld) b = atomicAdd(&s_nr, (uint32_t)__popcll(m));
                b = __shfl(b, ld, 64);
                const uint32_t j = b + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                if (keep) {
                    if (j < kWsResLds) {
                        lres[2u * j] = l;
                        lres[2u * j + 1u] = e;
                    } else {
                        const uint32_t g = atomicAdd(&w.ctl[kWsResN], 1u);
                        w.res[2u * g] = l;
                        w.res[2u * g + 1u] = e;
                    }
                }
            }
        } else {
            const uint32_t lo = s.lx + 1u >= kMinstdN ? s.lx + 1u - kMinstdN : s.lx + 1u;
            for (uint32_t run = 0; run < 2u; run++) {
                uint32_t r0, r1;
                if (run == 0) { r0 = lo; r1 = (uint32_t)min<uint64_t>((uint64_t)lo + nloc, kMinstdN); }
                else { r0 = 0; r1 = (uint64_t)lo + nloc > kMinstdN ? (uint32_t)((uint64_t)lo + nloc - kMinstdN) : 0u; }
                if (r1 <= r0) continue;
                const uint32_t e0 = w.boff[r0 >> kWsBShift], e1 = w.boff[((r1 - 1u) >> kWsBShift) + 1u];
                const uint32_t base = run == 0 ? lo : lo - kMinstdN;   // v = L - base (mod 2^32)
                if (threadIdx.x == 0) s.st[6] += e1 - e0;
                for (uint32_t j = e0 + threadIdx.x; j < e1; j += blockDim.x) {
                    const uint32_t L = w.wL[j];
                    if (!(L >= r0 && L < r1)) continue;
                    const uint32_t l = L - base, x = w.ww[j];
                    const uint32_t cv = C[l];
                    if (dc_ld(&a.inc_vcnt[l]) != 0u) continue;   // a violator: walked above
                    const float u = minstd_canonical(x);
                    uint32_t ncol;
                    if (u < a.emax && x - 1u < a.ftab_n) {
                        const uint32_t F = a.ftab[x - 1u];
                        ncol = F <= cv ? F - 1u : cv;
                    } else {
                        ncol = walk_own_tab(a.etab, a.nCol, cv, a.eps, a.hi, u);
                    }
                    if (ncol != cv) push(l, cv | (ncol << 16));
                }
            }
        }
        mark(k, 3);
        if (walking) {   // (their results are read back coherently: no acquire)
            wait(false);
            if (threadIdx.x == 0) s_w[0] = dc_ld(&w.ctl[kWsHeavyN]);   // heavy rows past a workgroup's 64
            __syncthreads();
            if (s_w[0] > 0u) {
                post(kWsWalkHeavy);
                wait(false);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        mark(k, 4);
        // the results in one list: the global one (walk phases, LDS overflow) appended to the LDS one
        // where it fits, else the LDS one appended to the global one
        if (threadIdx.x == 0) {
            s_w[0] = dc_ld(&w.ctl[kWsResN]);
            s_ne = 0;
        }
        dc_lbar();
        probe(0);
        const uint32_t Ng = s_w[0], Nl = min(s_nr, kWsResLds);
        const bool inl = Nl + Ng <= kWsResLds;
        uint32_t* const R = inl ? lres : w.res;
        const uint32_t N = Nl + Ng;
        if (inl) {
            for (uint32_t i = threadIdx.x; i < 2u * Ng; i += blockDim.x) lres[2u * Nl + i] = dc_ld(&w.res[i]);
        } else {
            if (threadIdx.x == 0) {   // (the global list is read plainly from here: acquire)
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < 2u * Nl; i += blockDim.x) w.res[2u * Ng + i] = lres[i];
        }
        if (inl) dc_lbar(); else __syncthreads();
        // more than a few results: the delta phase goes out now with their rows (kWsDeltaR), its
        // workgroups load the rows' offsets while the events draw; the colours follow (post_go)
        const bool dr = N > kWsLeadN && N <= kWsChgLds && N <= 4u * blockDim.x;   // (a helper thread takes <= 4)
        const uint32_t lxn = s.lx + a.nmodN >= kMinstdN ? s.lx + a.nmodN - kMinstdN : s.lx + a.nmodN;
        if (dr) {
            for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) w.chg[4u * i] = R[2u * i];
            if (threadIdx.x == 0) {
                w.ctl[kWsChgN] = N;
                w.ctl[kWsArgL] = lxn;   // (the next sweep's candidates, found in the same phase)
                w.ctl[kWsCandN] = 0u;
            }
            post(kWsDeltaR);
        }
        probe(3);   // [11] merge
        // overflow events in ascending vertex order take the next glibc draws (:517-520): up to
        // kWsRankMax ranked and drawn in parallel (draw r = sum_m T[m][r] ring[m], the commit's table),
        // more sorted (bitonic) and drawn in sequence
        for (uint32_t i = threadIdx.x; i < N; i += blockDim.x)
            if ((R[2u * i + 1u] >> 16) == a.nCol) {
                const uint32_t j = atomicAdd(&s_ne, 1u);
                if (j < kWsEvLds) evl[j] = i;
                a.events[j] = R[2u * i];
            }
        if (threadIdx.x < 31u) s_ring[threadIdx.x] = s.ring[threadIdx.x];
        dc_lbar();
        probe(4);   // [12] the events' collection
        const uint32_t E = s_ne;

        if (E > 0u && E <= kWsRankMax) {
            // ranks by vertex: a counting sort over 1024 buckets of the row range (events are few
            // and spread: a bucket holds about one), then the order inside each bucket; beside it
            // the E raw draws, one per thread (glibc's r_i = r_i-31 + r_i-3 as a table of powers)
            uint32_t* const bc = tmp;               // [1024] events per bucket, then their offsets
            uint32_t* const bf = tmp + 1024u;       // [1024] fill counters
            uint32_t* const sl = tmp + 2048u;       // [E] the events' vertices, bucket by bucket
            uint32_t* const raw = evl + kWsRankMax; // [E] raw draws in order (rand() = raw >> 1)
            bc[threadIdx.x] = 0u;
            bf[threadIdx.x] = 0u;
            dc_lbar();
            uint32_t ii = 0, v = 0, bk = 0;
            if (threadIdx.x < E) {
                ii = evl[threadIdx.x];
                v = R[2u * ii];
                bk = (uint32_t)(((uint64_t)v * 1024u) / nloc);
                atomicAdd(&bc[bk], 1u);
            }
            if (!s_rawok) draws();   // (computed during the last count moves where there were any)
            dc_lbar();
            uint32_t tot = 0;
            const uint32_t off = ws_scan(bc[threadIdx.x], s_wsum, &tot);
            bc[threadIdx.x] = off;
            dc_lbar();
            if (threadIdx.x < E) sl[bc[bk] + atomicAdd(&bf[bk], 1u)] = v;
            dc_lbar();
            probe(6);   // [14] buckets
            if (threadIdx.x < E) {
                uint32_t rk = bc[bk];
                for (uint32_t j = bc[bk], je = bc[bk] + bf[bk]; j < je; j++) rk += sl[j] < v ? 1u : 0u;
                const uint32_t c = (raw[rk] >> 1) % (a.nCol - 1u);   // rand() % (nCol - 1), :518
                R[2u * ii + 1u] = (R[2u * ii + 1u] & 0xFFFFu) | (c << 16);
            }
            dc_lbar();
            probe(7);   // [15] ranks and colours
            if (threadIdx.x < 31u) {   // the window after E draws, oldest first
                const uint32_t nw = (E < 31u && threadIdx.x < 31u - E) ? s_ring[E + threadIdx.x] : raw[E + threadIdx.x - 31u];
                s.ring[threadIdx.x] = nw;
                st->glibc_ring[threadIdx.x] = nw;
            }
            if (threadIdx.x == 0) {
                st->glibc_head = 0u;
                s.draws += E;
                st->glibc_draws = s.draws;
                s_rawok = 0;
            }
            if (inl) dc_lbar(); else __syncthreads();
        } else if (E > 0u) {
            uint32_t P2 = 1;
            while (P2 < E) P2 <<= 1;
            uint32_t* sv = a.events;   // vertex ids
            for (uint32_t i = E + threadIdx.x; i < P2; i += blockDim.x) sv[i] = 0xFFFFFFFFu;
            __syncthreads();
            bitonic_sort_block(sv, P2);
            __syncthreads();
            if (threadIdx.x == 0) {
                uint32_t head = 0;
                for (uint32_t i = 0; i < E; i++) w.heavy[sv[i]] = glibc_next(s.ring, head) % (a.nCol - 1u);
                uint32_t r[31];
                for (uint32_t i = 0; i < 31u; i++) r[i] = s.ring[(head + i) % 31u];
                for (uint32_t i = 0; i < 31u; i++) {
                    s.ring[i] = r[i];
                    st->glibc_ring[i] = r[i];
                }
                st->glibc_head = 0u;
                s.draws += E;
                st->glibc_draws = s.draws;
                s_rawok = 0;
            }
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < N; i += blockDim.x)
                if ((R[2u * i + 1u] >> 16) == a.nCol)
                    R[2u * i + 1u] = (R[2u * i + 1u] & 0xFFFFu) | (w.heavy[R[2u * i]] << 16);
            __syncthreads();
        }
        mark(k, 5);
        // the changed rows: C_t+1 into the other buffer; every result listed (by result index) with
        // its row start and its arcs' prefix (an unchanged one -- an overflow that drew its own
        // colour -- with no arcs), per-thread runs of the results, workgroup scans. With the delta
        // phase posted early (dr) only the colours, then the go: the helpers have the rows' offsets
        uint32_t nch = 0, arcs = 0;
        probe(0);
        if (dr) {
            uint32_t mc = 0;
            for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) {
                const uint32_t l = R[2u * i], e = R[2u * i + 1u];
                if ((e >> 16) != (e & 0xFFFFu)) {
                    Cs[l] = (uint16_t)(e >> 16);
                    mc++;
                }
                w.chg[4u * i + 1u] = e;
            }
            (void)ws_scan(mc, s_wsum, &nch);
            if (threadIdx.x == 0) s.st[7] += nch;
            arcs = 0xFFFFFFFFu;   // (not known here: the delta phase)
            post_go();
            probe(1);
        } else {
            const uint32_t per = (N + blockDim.x - 1u) / blockDim.x, i0 = min(N, threadIdx.x * per), i1 = min(N, i0 + per);
            uint32_t* const dg = tmp;   // degrees by result index (LDS results only)
            uint32_t mc = 0, ma = 0;
            for (uint32_t ib = i0; ib < i1; ib += 4u) {   // 4 rows' offsets in flight per thread
                uint32_t l[4], e[4];
                uint64_t r0[4], r1[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t i = ib + (uint32_t)u;
                    l[u] = i < i1 ? R[2u * i] : 0u;
                    e[u] = i < i1 ? R[2u * i + 1u] : 0u;
                    const bool chg = i < i1 && (e[u] >> 16) != (e[u] & 0xFFFFu);
                    r0[u] = chg ? a.row_off[l[u]] : 0ull;
                    r1[u] = chg ? a.row_off[l[u] + 1u] : 0ull;
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t i = ib + (uint32_t)u;
                    if (i >= i1) break;
                    const uint32_t cv = e[u] & 0xFFFFu, nc = e[u] >> 16;
                    const uint32_t d = (uint32_t)(r1[u] - r0[u]);
                    if (nc != cv) {
                        Cs[l[u]] = (uint16_t)nc;
                        mc++;
                    }
                    reinterpret_cast<uint4*>(w.chg)[i] = make_uint4(l[u], e[u], (uint32_t)r0[u], (uint32_t)(r0[u] >> 32));
                    if (inl) dg[i] = d;
                    else w.pre[i] = d;
                    ma += d;
                }
            }
            probe(1);   // [9] rows' offsets
            (void)ws_scan(mc, s_wsum, &nch);
            uint32_t run = ws_scan(ma, s_wsum, &arcs);
            probe(2);   // [10] scans
            for (uint32_t i = i0; i < i1; i++) {
                const uint32_t d = inl ? dg[i] : w.pre[i];
                w.pre[i] = run;
                run += d;
            }
            if (threadIdx.x == 0) {
                w.pre[N] = arcs;
                w.ctl[kWsChgN] = N;
                s.st[7] += nch;
                s.arcs += arcs;
            }
            probe(5);   // [13] prefix stores
        }
        mark(k, 6);
        // the counts move: by the leader's threads when few arcs, else a delta phase
        if (nch || dr) {
            const uint32_t nl = N;   // listed results (changed or not)
            if (!dr && arcs <= w.lead_arcs) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                const uint32_t* pre = w.pre;
                if (nl + 1u <= 3u * kWsCandCap) {   // the prefix into LDS (the candidates' buffer: gone)
                    for (uint32_t i = threadIdx.x; i <= nl; i += blockDim.x) cand[i] = w.pre[i];
                    __syncthreads();
                    pre = cand;
                }
                ws_delta_arcs<false>(a, w, C, Cs, pre, nl, threadIdx.x, arcs, blockDim.x);
                if (threadIdx.x == 0) s_pf = 0xFFFFFFFFu;
            } else {
                // the helpers move the counts and find the next sweep's candidates (its log is lx + n,
                // its colours are C_t+1, in Cs); only those candidates' counts must wait
                if (!dr) {
                    if (threadIdx.x == 0) {
                        w.ctl[kWsArgL] = lxn;
                        w.ctl[kWsCandN] = 0u;
                    }
                    post(kWsDelta);
                }
                if (!s_rawok) {   // the next sweep's draws while the helpers work (E > kWsRankMax: the
                    draws();      // event list overwrote them; the window is that of sweep t + 1)
                    __syncthreads();
                    if (threadIdx.x == 0) s_rawok = 1;
                }
                wait(false);   // (candidates and touched rows read back coherently)
                if (threadIdx.x == 0) {
                    s.st[4]++;
                    s_pf = lxn;
                    s_gn = dc_ld(&w.ctl[kWsCandN]);
                    if (dr) s.arcs += dc_ld(&w.ctl[kWsArcsOut]);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            // both buffers = C_t+1
            for (uint32_t j = threadIdx.x; j < nl; j += blockDim.x) {
                const uint32_t e = w.chg[4u * j + 1u];
                if ((e >> 16) != (e & 0xFFFFu)) const_cast<uint16_t*>(C)[w.chg[4u * j]] = (uint16_t)(e >> 16);
            }
        }
        mark(k, 7);
        // the violators of C_t+1: those of C_t still counted and the touched rows (flags dedupe)
        {
            if (threadIdx.x == 0) {
                s_w[0] = dc_ld(&w.ctl[kWsTchN]);
                s_w[1] = dc_ld(&w.ctl[kWsTchOvf]);
                s_vq = 0;
            }
            dc_lbar();
            const uint32_t tn = s_w[0], tovf = s_w[1];
            if (threadIdx.x == 0) {
                w.ctl[kWsVn + q] = 0u;
                w.ctl[kWsTchN] = 0u;
                w.ctl[kWsTchOvf] = 0u;
            }
            if (!tovf && Vn + tn <= kWsLeadList) {
                uint32_t* vq = w.vl + (size_t)q * nloc;
                for (uint32_t i = threadIdx.x; i < Vn + tn; i += blockDim.x) {
                    const bool old = i < Vn;
                    const uint32_t l = old ? vl[i] : dc_ld(&w.tch[i - Vn]);
                    const bool on = dc_ld(&a.inc_vcnt[l]) > 0u;
                    const uint32_t bit = 1u << (8u * (l & 3u));
                    bool add = false;
                    if (old) {
                        if (on) add = true;
                        else atomicAnd(&w.flag[l >> 2], ~bit);
                    } else if (on) {
                        add = (atomicOr(&w.flag[l >> 2], bit) & bit) == 0u;
                    }
                    const uint64_t m = __ballot(add);
                    if (m) {
                        const int lead = __ffsll((long long)m) - 1;
                        uint32_t b = 0;
                        if ((int)lane == lead) b = atomicAdd(&s_vq, (uint32_t)__popcll(m));
                        b = __shfl(b, lead, 64);
                        if (add) vq[b + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = l;
                    }
                }
                dc_lbar();
                if (threadIdx.x == 0) w.ctl[kWsVn + q] = s_vq;
            } else {
                if (threadIdx.x == 0) {
                    w.ctl[kWsArgP] = q;
                    s.st[5]++;
                }
                post(kWsCollect);
                wait();
            }
        }
        mark(k, 8);
        // accept: the RNG advances by n draws (:139), lx with it
        if (threadIdx.x == 0) {
            s.t = t + 1u;
            s.x_t = minstd_mulmod(s.x_t, a.aN);
            const uint32_t lx = s.lx + a.nmodN;
            s.lx = lx >= kMinstdN ? lx - kMinstdN : lx;
            st->t = s.t;
            st->x_t = s.x_t;
            st->lx = s.lx;
            w.ctl[kWsT] = s.t + 1u;
            s.st[0]++;
        }
        __syncthreads();
    }
    // exit: the helpers leave; the per-sweep path finds its delta lists empty and visits every row
    mark(0xFFFFu, 200u);
    post(kWsExit);
    if (threadIdx.x < 64u) {   // (wave-uniform, as the waits)
        const unsigned long long t0 = wall_clock64();
        for (;;) {
            if (__builtin_amdgcn_readfirstlane(dc_ld(&w.ctl[kWsAck])) >= G - 1u) break;
            if (wall_clock64() - t0 > kWsWaitTicks) {
                if (threadIdx.x == 0) {
                    w.ctl[kWsErr] = (s_seq << 8) | 2u;
                    st->err |= kDevErrWatchdog;
                }
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        w.ctl[kWsGen] = 0u;
        w.ctl[kWsAck] = 0u;
        w.ctl[kWsDone] = 0u;
        const uint32_t p = s.t & 1u;
        if (go) {
            a.inc[kIncTchOvf + p] = 1u;
            a.inc[kIncDenseN + p] = 0u;
            a.inc[kIncHubN + p] = 0u;
            unsigned long long* is = reinterpret_cast<unsigned long long*>(a.inc + kIncStat);
            is[0] += s.st[0];
            is[1] += s.recounts;
            is[2] += s.st[7];
            is[3] += s.arcs;
        }
        unsigned long long* ss = reinterpret_cast<unsigned long long*>(w.ctl + kWsStat);
        for (int i = 0; i < 8; i++) ss[i] += s.st[i];
        unsigned long long* tt = reinterpret_cast<unsigned long long*>(w.ctl + kWsTime);
        for (int i = 0; i < 16; i++) tt[i] += s.tm[i];
    }
}
