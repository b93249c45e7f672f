// mcmc_colorer_amd/csrc/dense_sparse.h -- the persistent dense-count sweep (dc_multi_kernel).
// Included by mcmc_sweep.hip inside namespace mcmc, after dense_counts.h.
//
// The dense sweep (dense_counts.h) evaluates every row but writes only those that move. Which rows
// can move is known before any row is read:
//   * a row whose dense mask is full (no open bit) is in fill_p's case (i) (coloringMCMC_CPU.cpp:
//     402-412): own colour hi, every other eps; it keeps its colour exactly when its draw u_v lies
//     in [E[cv], S[cv]) (the closed-form walk, SweepArgs::ewalk), i.e. when its minstd state x_v
//     lies in [x_lo(cv), x_hi(cv)) (canonical is monotone in x);
//   * so a closed row whose state lies in [max_c x_lo(c), min_c x_hi(c)) keeps its colour whatever
//     its colour is. The states outside that interval form the candidate window W -- with the
//     reference's eps = 1e-8 (main.cu:160) a few thousand of the 2^31 - 2 states (C3: ~1.4e3);
//   * vertex v's state in sweep t is x_t 16807^(v+1) = 16807^(lx_t + v + 1), lx_t = log x_t (rng.h
//     minstd_dlog; 16807 is a primitive root). With L(w) the logarithm of a window state w, the
//     vertex that draws w in sweep t is v = L(w) - lx_t - 1 mod (2^31 - 2) -- ONE vertex per window
//     state, found with one subtraction. dl_tab holds {L(w), w} for every w in W (dl_table_kernel).
// A sweep therefore evaluates the candidate rows (C3: ~6 of 1e7), the open rows (none once S is
// large enough, setup_dense) and nothing else; every other row keeps its colour and is a violator
// (its full mask holds its own colour: violation_count, :329-351), so
//     Cviol_t = nloc - (rows evaluated) + (violators among them).
// The result is bit-identical to evaluating every row (tests/test_dense.py runs both).
//
// dc_multi_kernel runs K sweeps in one launch, one BS-thread workgroup per CU (BS = 512 by default:
// 256 VGPRs per lane, no scratch for NW <= 2; MCMC_DCM_BS=1024 doubles the waves). Workgroup 0 (the
// leader) plans each sweep from the control words:
//   solo  the update has at most a few moved vertices of S, the restore list was applied by the
//         last commit, few open mask words: the leader posts the moves to the helpers (a move
//         phase, dc_help_moves: ~2e4 random count atomics per moved vertex at C3 need the grid's
//         memory pipelines) and waits for them, evaluates the candidates and the open rows itself
//         and commits (dc_leader_solo) -- no grid-wide barrier;
//   full  anything else (the count rebuild of a new colouring, list overflows, many moves): the
//         leader posts the sweep (release + flag), every workgroup runs the dense sweep of
//         dense_counts.h (dc_full_body), the last to arrive commits and signals, the leader waits.
// The other workgroups poll the leader's flag between full sweeps (one lane, s_sleep) and leave on
// its exit post; the leader waits for their acknowledgements and resets the words before it
// returns, so the next launch starts from a clean flag. The loop state lives in DevState as for the
// per-sweep kernels; commit_control / commit_accept are the same code (loop control, the glibc
// replay, the lists' bookkeeping, the RNG advance incl. lx).
// Memory ordering (MI355X_MICROARCH.md "Workgroup dispatch ... visibility"): solo sweeps touch
// global memory from one CU only -- plain data is coherent through its L1, words changed by
// atomics are read with sc1 loads (dc_ld); full sweeps are bracketed by release/flag/acquire.

__device__ __forceinline__ uint32_t dc_ld(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long dc_ld(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// dl_tab[i] = {L(w), w} for the i-th state w of the window [1, lo) U [hi, 2^31 - 1); err[0] |= 1
// if a logarithm fails its check 16807^L = w.
__global__ __launch_bounds__(256) void dl_table_kernel(uint2* __restrict__ tab, uint32_t lo, uint32_t hi, uint32_t nw,
                                                       uint32_t* __restrict__ err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nw) return;
    const uint32_t nlo = lo - 1u;
    const uint32_t w = i < nlo ? 1u + i : hi + (i - nlo);
    const uint32_t L = minstd_dlog(w);
    if (L == 0xFFFFFFFFu || minstd_pow(kMinstdA, L) != w) atomicOr(err, 1u);
    tab[i] = make_uint2(L, w);
}

// Watchdogs of the persistent launch (wall_clock64 ticks, 100 MHz): the leader gives a phase of
// the helpers kDcWaitTicks to complete, then flags DevState::err (kDevErrWatchdog) and stops instead
// of waiting for workgroups that may not be resident; a helper that sees no post for kDcIdleTicks
// leaves (it would otherwise spin on words the leader has reset).
constexpr unsigned long long kDcWaitTicks = 200000000ull;    // 2 s
constexpr unsigned long long kDcIdleTicks = 3000000000ull;   // 30 s
constexpr uint32_t kDcSoloPairs = 4096;      // (moved vertex, column block) pairs a move phase takes
constexpr uint32_t kDcSoloMovesMax = 16;     // and moved vertices
constexpr uint32_t kDcSoloOpenWords = 32;    // nonzero open words a solo sweep evaluates itself
constexpr uint32_t kDcSoloOpenRows = 2048;   // (at most 64 rows each)
constexpr uint32_t kDcCandCap = 4096;        // candidate rows per round (LDS)
constexpr uint32_t kDcTabLds = 4096;         // window entries cached in LDS
// dynamic LDS of dc_multi_kernel: [the dense sweep's 64 KiB: stage, commit scratch][candidates:
// 2 x kDcCandCap words][window cache: 2 x kDcTabLds words][open rows: kDcSoloOpenRows words]
constexpr uint32_t kDcMultiLds = kDcEvalLds + 8u * kDcCandCap + 8u * kDcTabLds + 4u * kDcSoloOpenRows;

// fill_p + extract_new_color of one row from its occupancy mask and its draw u -- evaluate_lane's
// walk without its writes, no taboo (coloringMCMC_CPU.cpp:393-528): the new colour, or nCol for a
// CDF overflow (the glibc replay decides those).
template <int NW>
__device__ __forceinline__ uint32_t dc_walk(const SweepArgs& a, const uint32_t (&acc)[NW], uint32_t cv, float u,
                                            const float2* ew, bool& viol) {
    uint32_t pop = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) pop += __popc(acc[i]);
    viol = get_color_bit<NW>(acc, cv) != 0u;
    const uint32_t Zvcomp = a.nCol - pop;
    const bool ii = viol && Zvcomp > 0;   // case (ii): occupied eps, free pf; else own colour hi, others eps
    uint32_t sel[NW];
    float pA, pB;
    if (ii) {
#pragma unroll
        for (int i = 0; i < NW; i++) sel[i] = acc[i];
        pA = a.eps;
        pB = (1.0f - a.eps * (float)pop) / (float)Zvcomp;
    } else {
#pragma unroll
        for (int i = 0; i < NW; i++) sel[i] = 0;
        set_color_bit<NW>(sel, cv);
        pA = a.hi;
        pB = a.eps;
        if (ew != nullptr) {
            const float2 es = ew[cv];
            if (u >= es.x) return es.y > u ? cv : a.nCol;
        }
    }
    uint32_t newc = a.nCol;
    float cdf = 0.0f;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        const uint32_t bits = sel[i];
        const uint32_t cmax = min(32u, a.nCol > (uint32_t)(32 * i) ? a.nCol - 32u * i : 0u);
        for (uint32_t cc = 0; cc < cmax && newc == a.nCol; cc++) {
            cdf += ((bits >> cc) & 1u) ? pA : pB;
            if (cdf > u) newc = 32u * i + cc;
        }
    }
    return newc;
}

// A workgroup barrier for LDS only: this wave's LDS operations complete, then s_barrier. Unlike
// __syncthreads it does not wait for the wave's global stores (the solo sweep's writes drain while
// it goes on; where they must be complete it waits for them itself: s_waitcnt vmcnt(0) first).
__device__ __forceinline__ void dc_lbar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// The leader's loop state during solo sweeps (LDS). Read from DevState and the control words when
// the leader takes over (launch start, after a full sweep); every solo sweep writes what it changes
// back (plain stores nothing waits for), so a full sweep, the next launch or the host see it.
constexpr uint32_t kDcSoloRes = 4096;   // rows a solo sweep changes (more: that sweep runs full)
struct DcSolo {
    uint32_t t, x_t, lx, done, err, mode, ovf, chg, len;
    uint32_t ring[31];              // the glibc window, oldest first
    unsigned long long draws;       // glibc draws so far (DevState::glibc_draws)
    uint32_t nres, nev, neval, nviol, nmv;
    unsigned long long st_inc, st_listed, st_open, st_chg, st_eval;   // statistics, written back on leaving
};

// Evaluate rows (lane each, the whole wave calls): a candidate (closed row, state x) or an open row
// (its mask completed by dc_open_scan, x from skip-ahead). Rows whose colour changes (or that
// overflow) are appended to res (l, cv | newc << 16); neval / nviol counted.
template <int NW>
__device__ __forceinline__ void dc_solo_rows(const SweepArgs& a, const uint8_t* __restrict__ C, bool valid, uint32_t l,
                                             uint32_t cv, uint32_t x, bool open_row, uint32_t x_t, const float2* ew,
                                             DcSolo& sv, uint32_t* res, int lane) {
    uint32_t fullw[NW];
#pragma unroll
    for (int i = 0; i < NW; i++) fullw[i] = dc_fullw(a.nCol, (uint32_t)i);
    DcMask<NW> m, fw;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        m.w[i] = (valid && open_row) ? dc_ld(&a.dc_mask[(size_t)l * NW + i]) : fullw[i];
        fw.w[i] = fullw[i];
    }
    if (open_row && __ballot(valid)) {
        const DcScan ds{a.tseg, a.gbase, a.tcol, a.grp_rows, a.nblocks, a.block_log2, a.dc_s0, a.dc_s1};
        m = dc_open_scan<NW>(ds, C, l, valid, m, fw, lane);
    }
    if (open_row && valid) x = minstd_mulmod(x_t, minstd_pow_tab((uint64_t)a.v_begin + l + 1ull));
    uint32_t acc[NW];
#pragma unroll
    for (int i = 0; i < NW; i++) acc[i] = m.w[i];
    bool viol = false;
    const uint32_t newc = valid ? dc_walk<NW>(a, acc, cv, minstd_canonical(x), ew, viol) : cv;
    const bool chg = valid && newc != cv;
    const uint64_t cb = __ballot(chg);
    if (cb) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&sv.nres, (uint32_t)__popcll(cb));
        base = __shfl(base, 0, 64);
        const uint32_t j = base + (uint32_t)__popcll(cb & ((1ull << lane) - 1ull));
        if (chg && j < kDcSoloRes) {
            res[j] = l;
            res[kDcSoloRes + j] = cv | (newc << 16);
        }
        const uint32_t ne = (uint32_t)__popcll(__ballot(chg && newc == a.nCol));
        if (lane == 0 && ne) atomicAdd(&sv.nev, ne);
    }
    const uint32_t nv = (uint32_t)__popcll(__ballot(valid)), nvl = (uint32_t)__popcll(__ballot(valid && viol));
    if (lane == 0 && nv) {
        atomicAdd(&sv.neval, nv);
        atomicAdd(&sv.nviol, nvl);
    }
}

// The leader's solo sweeps, from the next one on, until a sweep needs the grid (returns 1), the
// launch's K sweeps are done or the loop stopped (returns 2). k: sweeps of this launch so far.
// Per sweep: [the counts moved by the last sweep's moves of S, dc_solo_moves] -> the candidates of
// the window and the open rows, one load round trip for their colours and open words -> their
// walks -> Cviol, loop control (coloringMCMC_CPU.cpp:136, :259-269) -> the overflow events' glibc
// draws in ascending vertex order from the window in LDS (:517-520) -> the changed rows written to
// BOTH colour buffers (so no restore list), moves of S listed for the next sweep.
// A move phase (persistent sweep, kind 3): the last sweep's moves of S (kDcMvN vertices, their
// (v, a << 16 | b) at kDcMvList) applied to the counts of every local row holding them, by the
// helpers: wave task j (vertex j / nbl, column block j % nbl) is u's segment in that block, the
// workgroup tasks (a wave task per wave) dealt statically to workgroups 1..G-1 -- no claim counter,
// so nothing to reset between phases. Each workgroup adds its completed tasks to kDcMvDone once
// its atomics have returned; the leader waits for the total. Everything it reads arrives by sc1
// loads (the list) or is read-only (the layout); the counts move by device-scope atomics.
template <int NW>
__device__ __forceinline__ void dc_help_moves(const SweepArgs& a) {
    __shared__ uint32_t s_len, s_mvl[2u * kDcSoloMovesMax];
    if (threadIdx.x < 2u * kDcSoloMovesMax + 1u) {
        if (threadIdx.x == 0) s_len = min(dc_ld(&a.dc_ctl[kDcMvN]), kDcSoloMovesMax);
        else s_mvl[threadIdx.x - 1u] = dc_ld(&a.dc_ctl[kDcMvList + threadIdx.x - 1u]);
    }
    __syncthreads();
    const uint32_t bl = a.block_log2, bl0 = a.v_begin >> bl, nbl = ((a.v_end - 1u) >> bl) - bl0 + 1u;
    const uint32_t nwv = blockDim.x >> 6;
    const uint32_t nloc = a.v_end - a.v_begin, T = s_len * nbl, J = (T + nwv - 1u) / nwv;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t mine = 0;
    for (uint32_t j = blockIdx.x - 1u; j < J; j += gridDim.x - 1u) {
        mine++;
        const uint32_t task = j * nwv + wv;
        if (task >= T) continue;
        const uint32_t i = task / nbl, b = bl0 + (task - i * nbl);
        const uint32_t u = s_mvl[2u * i], ab = s_mvl[2u * i + 1u], ca = ab >> 16, cb = ab & 0xFFFFu;
        uint32_t s0, s1;
        const uint16_t* gc;
        dc_segment(a, u - a.v_begin, b, s0, s1, gc);
        const uint32_t base = b << bl;
        for (uint32_t q0 = s0; q0 < s1; q0 += 256u) {   // 4 ids per lane in flight, then their atomics
            uint32_t lw[4], oa[4], ob[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const uint32_t qq = q0 + 64u * r + lane;
                lw[r] = qq < s1 ? (base | (uint32_t)gc[qq]) - a.v_begin : 0xFFFFFFFFu;
            }
#pragma unroll
            for (int r = 0; r < 4; r++) {
                oa[r] = 2u;
                ob[r] = 1u;
                if (lw[r] < nloc) {
                    uint32_t* cw = a.dc_cnt + (size_t)lw[r] * a.dc_cw;
                    oa[r] = atomicSub(&cw[ca], 1u);
                    ob[r] = atomicAdd(&cw[cb], 1u);
                }
            }
#pragma unroll
            for (int r = 0; r < 4; r++) {
                if (oa[r] == 1u) dc_flip<NW>(a, lw[r], ca);
                if (ob[r] == 0u) dc_flip<NW>(a, lw[r], cb);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && mine) atomicAdd(&a.dc_ctl[kDcMvDone], mine);
}

// tab: the window, the LDS copy at dyn + 96 KiB where it fits (reloaded on entry: a full sweep's
// count rebuild uses that LDS for its colour slices).
template <int NW>
__device__ __forceinline__ uint32_t dc_leader_solo(const SweepArgs& a, uint32_t K, uint32_t& k, DcTabs tb, uint32_t* dyn,
                                                   const uint2* tab, bool solo_ok, uint32_t moves_max,
                                                   unsigned long long& nsolo, uint32_t& seq, uint32_t& mvexp) {
    __shared__ DcSolo sv;
    __shared__ uint32_t s_mv[2 * kDcSoloMovesMax];
    __shared__ uint32_t s_ow;
    DevState* __restrict__ st = a.st;
    uint32_t* const cand = dyn + kDcEvalLds / 4u;               // [2 kDcCandCap]
    uint32_t* const orow = cand + 2u * kDcCandCap + 2u * kDcTabLds;   // [kDcSoloOpenRows]
    uint32_t* const res = dyn;                                   // [2 kDcSoloRes]
    uint32_t* const evs = dyn + 2u * kDcSoloRes;                 // [kDcSoloRes] events (ascending)
    const uint32_t nloc = a.v_end - a.v_begin, lane = threadIdx.x & 63u;
    const uint32_t wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    if (tab != a.dl_tab) {
        uint2* const tabl = const_cast<uint2*>(tab);
        for (uint32_t i = threadIdx.x; i < a.dl_n; i += blockDim.x) tabl[i] = a.dl_tab[i];
    }
    if (threadIdx.x == 0) {   // take over the loop state
        const uint32_t t = dc_ld(&st->t), p = t & 1u, head = dc_ld(&st->glibc_head);
        sv.t = t;
        sv.done = dc_ld(&st->done);
        sv.x_t = dc_ld(&st->x_t);
        sv.err = dc_ld(&st->err);
        sv.lx = dc_ld(&st->lx);
        for (uint32_t i = 0; i < 31u; i++) sv.ring[i] = dc_ld(&st->glibc_ring[(head + i) % 31u]);
        sv.draws = dc_ld(&st->glibc_draws);
        sv.mode = dc_ld(&a.dc_ctl[kDcMode]);
        sv.ovf = dc_ld(&a.dc_ctl[kDcChgOvf + p]) | dc_ld(&a.dc_ctl[kDcOvf + p]);
        sv.chg = dc_ld(&a.dc_ctl[kDcChgLen + p]);
        sv.len = dc_ld(&a.dc_ctl[kDcLen + p]);
        if (sv.len <= moves_max)
            for (uint32_t i = 0; i < 2u * sv.len; i++) s_mv[i] = dc_ld(&a.dc_list[2u * (size_t)p * a.dc_cap + i]);
        sv.st_inc = sv.st_listed = sv.st_open = sv.st_chg = sv.st_eval = 0;
    }
    __syncthreads();
    uint32_t ret = 2u;
    __shared__ uint32_t s_no, s_nc, s_e;
    // the open-summary word as last read (thread 0): only move phases and full sweeps change it, so
    // a sweep after neither reuses it instead of a round trip (C2: no candidates to hide it behind)
    bool ow_valid = false;
    uint32_t ow_cached = 0;
    for (; k < K; k++) {
        if (a.solo_ts && threadIdx.x == 0 && k < 4096u) a.solo_ts[8u * k] = wall_clock64();
        if (sv.done || sv.err) break;
        const uint32_t t = sv.t, p = t & 1u, q = p ^ 1u, len = sv.len;
        if (!(solo_ok && sv.mode == 0u && sv.ovf == 0u && sv.chg == 0u && len <= moves_max)) { ret = 1u; break; }
        const uint8_t* __restrict__ C = (t & 1) ? a.colors1 : a.colors0;   // C_t
        uint8_t* __restrict__ Cs = (t & 1) ? a.colors0 : a.colors1;        // C_t+1 (holds C_t on the local rows)
        if (len) {
            // the counts of C_t: the last sweep's moves of S (the list of parity p) applied by the
            // helpers (a move phase: one workgroup's 2 x 1e4 random count atomics at C3 take ~40 us,
            // the grid's a few), then its list is empty
            if (threadIdx.x == 0) {
                for (uint32_t i = 0; i < 2u * len; i++)
                    __hip_atomic_store(&a.dc_ctl[kDcMvList + i], s_mv[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&a.dc_ctl[kDcMvN], len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                seq++;
                __hip_atomic_store(&a.dc_ctl[kDcGen], (seq << 2) | 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t nbl = ((a.v_end - 1u) >> a.block_log2) - (a.v_begin >> a.block_log2) + 1u;
                mvexp += (len * nbl + nwv - 1u) / nwv;   // (dc_help_moves' workgroup tasks)
                a.dc_ctl[kDcLen + p] = 0u;
                sv.st_listed += len;
                sv.len = 0;
            }
            ow_valid = false;   // (the moves may open or close rows)
            if (threadIdx.x < 64u) {   // wave 0 waits (a wave-uniform spin loop: see dc_multi_kernel)
                const uint32_t ex = __builtin_amdgcn_readfirstlane(mvexp);
                const unsigned long long t0 = wall_clock64();
                while (__builtin_amdgcn_readfirstlane(dc_ld(&a.dc_ctl[kDcMvDone])) < ex) {
                    if (wall_clock64() - t0 > kDcWaitTicks) {   // helpers missing: flag, stop the loop
                        if (threadIdx.x == 0) {
                            atomicOr(&st->err, kDevErrWatchdog);
                            sv.err = kDevErrWatchdog;
                        }
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (threadIdx.x == 0 && a.solo_ts && k < 4096u) a.solo_ts[8u * k + 7u] = wall_clock64();
            }
            __syncthreads();
            if (sv.err) break;
        }
        if (threadIdx.x == 0) {
            sv.nres = sv.nev = sv.neval = sv.nviol = sv.nmv = 0;
            s_no = s_e = 0;
            if (a.solo_ts && k < 4096u) a.solo_ts[8u * k + 1u] = wall_clock64();
        }
        dc_lbar();
        // candidates of the window, kDcCandCap entries per round; a candidate that is open is left
        // to the open rows. The open summary word is read in the same round trip as the first
        // round's colours and open words (it decides only what comes after the candidates: the
        // open rows, or a full sweep -- nothing is written before that test)
        const uint32_t lxs = kMinstdN - 1u - sv.lx;
        uint32_t ow_r = 0xFFFFFFFFu;
        bool ow_issued = false;
        for (uint32_t c0 = 0; c0 < a.dl_n; c0 += kDcCandCap) {
            if (threadIdx.x == 0) s_nc = 0;
            dc_lbar();
            const uint32_t c1 = min(a.dl_n, c0 + kDcCandCap);
            for (uint32_t j = c0 + threadIdx.x; j < c1; j += blockDim.x) {
                const uint2 e = tab[j];
                uint32_t d = e.x + lxs;   // L(w) - lx - 1 mod N: the vertex drawing state w (both terms < N)
                if (d >= kMinstdN) d -= kMinstdN;
                const uint32_t l = d - a.v_begin;
                if (d >= a.v_begin && l < nloc) {
                    const uint32_t kk = atomicAdd(&s_nc, 1u);
                    cand[2u * kk] = l;
                    cand[2u * kk + 1u] = e.y;
                }
            }
            // the last sweep's colour writes are complete before any candidate's colour is read
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            dc_lbar();
            if (!ow_issued) {
                if (threadIdx.x == 0 && a.dc_osum && !ow_valid) ow_r = (uint32_t)dc_ld(a.dc_osum);
                ow_issued = true;
            }
            const uint32_t nc = s_nc;
            for (uint32_t b = wv * 64u; b < nc; b += nwv * 64u) {
                const uint32_t kk = b + lane;
                bool valid = kk < nc;
                const uint32_t l = valid ? cand[2u * kk] : 0u, x = valid ? cand[2u * kk + 1u] : 0u;
                unsigned long long o = 0;
                uint32_t cv = 0;
                if (valid) {   // its colour and open words in one round trip
                    cv = C[a.v_begin + l];
#pragma unroll
                    for (int i = 0; i < NW; i++) o |= dc_ld(&a.dc_open[(size_t)(l >> 6) * NW + i]);
                }
                valid = valid && ((o >> (l & 63u)) & 1ull) == 0ull;
                dc_solo_rows<NW>(a, C, valid, l, cv, x, false, sv.x_t, tb.ew, sv, res, (int)lane);
            }
            dc_lbar();
        }
        if (threadIdx.x == 0) {
            if (ow_valid) ow_r = ow_cached;
            else if (!ow_issued && a.dc_osum) ow_r = (uint32_t)dc_ld(a.dc_osum);
            ow_cached = ow_r;
            ow_valid = a.dc_osum != nullptr;
            s_ow = a.dc_osum ? ow_r : 0xFFFFFFFFu;
            if (a.solo_ts && k < 4096u) a.solo_ts[8u * k + 4u] = wall_clock64();
        }
        dc_lbar();
        const uint32_t ow = s_ow;
        if (ow > kDcSoloOpenWords) { ret = 1u; break; }   // (nothing written yet: the sweep runs full)
        // the open rows (the summary's set bits, one tile's NW bits together)
        if (ow != 0u) {
            const uint32_t ntiles = (nloc + 63u) >> 6, nsw = (ntiles * NW + 63u) >> 6;
            for (uint32_t w = threadIdx.x; w < nsw; w += blockDim.x) {
                unsigned long long sb = dc_ld(&a.dc_osum[1 + w]);
                while (sb) {
                    const uint32_t bit = (uint32_t)__ffsll((long long)sb) - 1u;
                    const uint32_t tile = (w * 64u + bit) / NW, b0 = (tile * NW) & 63u;
                    sb &= ~(((1ull << NW) - 1ull) << b0);
                    unsigned long long o = 0;
#pragma unroll
                    for (int i = 0; i < NW; i++) o |= dc_ld(&a.dc_open[(size_t)tile * NW + i]);
                    while (o) {
                        const uint32_t r = (uint32_t)__ffsll((long long)o) - 1u;
                        o &= o - 1ull;
                        const uint32_t kk = atomicAdd(&s_no, 1u);
                        if (kk < kDcSoloOpenRows) orow[kk] = tile * 64u + r;
                    }
                }
            }
            dc_lbar();
        }
        const uint32_t no = min(s_no, kDcSoloOpenRows);

        for (uint32_t b = wv * 64u; b < no; b += nwv * 64u) {
            const uint32_t kk = b + lane;
            const uint32_t l = kk < no ? orow[kk] : 0u;
            dc_solo_rows<NW>(a, C, kk < no, l, kk < no ? (uint32_t)C[a.v_begin + l] : 0u, 0u, true, sv.x_t, tb.ew, sv,
                             res, (int)lane);
        }
        dc_lbar();
        if (a.solo_ts && threadIdx.x == 0 && k < 4096u) a.solo_ts[8u * k + 2u] = wall_clock64();
        const uint32_t nres = sv.nres;
        if (nres > kDcSoloRes) { ret = 1u; break; }   // (nothing written yet: the sweep runs full)
        // loop control (coloringMCMC_CPU.cpp:136, :259-269): every row not evaluated keeps its colour
        // and violates (its full dense mask holds it)
        const unsigned long long viol = (unsigned long long)nloc - sv.neval + sv.nviol;
        const bool stop = t == a.maxRip + 1u || (!a.bench && viol <= a.z);
        if (threadIdx.x == 0) {
            if (t < a.traj_cap) a.traj[t] = viol;
            sv.st_open += no;
            sv.st_eval += sv.neval;
            if (stop) {
                st->done = 1u;
                st->iter = t;
                st->maxIterReached = t == a.maxRip + 1u ? 1u : 0u;
                st->finalViol = viol;
                sv.done = 1u;
            }
        }
        if (stop) {
            nsolo++;
            k++;
            break;
        }
        // accept: overflow events in ascending vertex order take the next glibc draws (rank sort)
        if (a.solo_ts && threadIdx.x == 0 && k < 4096u) a.solo_ts[8u * k + 5u] = wall_clock64();
        const uint32_t nev = sv.nev;
        if (nev) {
            for (uint32_t i = threadIdx.x; i < nres; i += blockDim.x)
                if ((res[kDcSoloRes + i] >> 16) == a.nCol) evs[atomicAdd(&s_e, 1u)] = i;
            dc_lbar();
            for (uint32_t i = threadIdx.x; i < nev; i += blockDim.x) {   // rank of event i among the events
                const uint32_t li = res[evs[i]];
                uint32_t r = 0;
                for (uint32_t j = 0; j < nev; j++) r += res[evs[j]] < li ? 1u : 0u;
                evs[nev + r] = evs[i];
            }
            dc_lbar();
            __shared__ uint32_t s_head;
            if (threadIdx.x == 0) {
                uint32_t head = 0;
                for (uint32_t i = 0; i < nev; i++) {
                    const uint32_t ri = evs[nev + i];
                    const uint32_t c = glibc_next(sv.ring, head) % (a.nCol - 1u);   // rand() % (nCol - 1), :518
                    res[kDcSoloRes + ri] = (res[kDcSoloRes + ri] & 0xFFFFu) | (c << 16);
                }
                s_head = head;
                st->glibc_head = 0u;
                sv.draws += nev;
                st->glibc_draws = sv.draws;
            }
            dc_lbar();
            // the window back to oldest-first order, a lane per entry (wave 0)
            uint32_t wr = 0;
            if (threadIdx.x < 31u) {
                const uint32_t j = s_head + threadIdx.x;
                wr = sv.ring[j >= 31u ? j - 31u : j];
            }
            dc_lbar();
            if (threadIdx.x < 31u) {
                sv.ring[threadIdx.x] = wr;
                st->glibc_ring[threadIdx.x] = wr;
            }
            dc_lbar();
        }
        // the changed rows into both buffers; moves of S listed for the next sweep (parity q)
        if (a.solo_ts && threadIdx.x == 0 && k < 4096u) a.solo_ts[8u * k + 6u] = wall_clock64();
        for (uint32_t i = threadIdx.x; i < nres; i += blockDim.x) {
            const uint32_t l = res[i], cn = res[kDcSoloRes + i];
            const uint32_t cv = cn & 0xFFFFu, nc = cn >> 16;
            if (nc == cv) continue;   // an overflow that drew the same colour
            const uint32_t v = a.v_begin + l;

            Cs[v] = (uint8_t)nc;
            const_cast<uint8_t*>(C)[v] = (uint8_t)nc;
            if (v - a.dc_s0 < a.dc_s1 - a.dc_s0) {
                const uint32_t j = atomicAdd(&sv.nmv, 1u);
                if (j < a.dc_cap) {
                    uint32_t* e = a.dc_list + 2u * ((size_t)q * a.dc_cap + j);
                    e[0] = v;
                    e[1] = (cv << 16) | nc;
                }
                if (j < kDcSoloMovesMax) {
                    s_mv[2u * j] = v;
                    s_mv[2u * j + 1u] = (cv << 16) | nc;
                }
            }
        }
        dc_lbar();
        if (threadIdx.x == 0) {
            const uint32_t nm = sv.nmv;
            const bool ovf = nm > a.dc_cap;
            const uint32_t mode = (ovf || nm > a.dc_max) ? 1u : 0u;
            a.dc_ctl[kDcLen + q] = min(nm, a.dc_cap);
            a.dc_ctl[kDcOvf + q] = ovf ? 1u : 0u;
            a.dc_ctl[kDcOvf + p] = 0u;
            a.dc_ctl[kDcMode] = mode;
            sv.mode = mode;
            sv.ovf = ovf ? 1u : 0u;
            sv.len = min(nm, a.dc_cap);
            sv.st_inc++;
            sv.st_chg += nres;
            sv.t = t + 1u;
            sv.x_t = minstd_mulmod(sv.x_t, a.aN);
            const uint32_t lx = sv.lx + a.nmodN;
            sv.lx = lx >= kMinstdN ? lx - kMinstdN : lx;
            st->t = sv.t;
            st->x_t = sv.x_t;
            st->lx = sv.lx;
            if (a.solo_ts && k < 4096u) a.solo_ts[8u * k + 3u] = wall_clock64();
        }
        dc_lbar();
        nsolo++;
    }
    // every wave's stores complete before the statistics / the caller's post
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {   // statistics (dc_commit's and the commit's counters)
        unsigned long long* s = reinterpret_cast<unsigned long long*>(a.dc_ctl + kDcStat);
        s[0] += sv.st_inc;
        s[2] += sv.st_listed;
        s[3] += sv.st_open;
        reinterpret_cast<unsigned long long*>(a.dc_ctl + kDcSoloEval)[0] += sv.st_eval;
        const uint32_t r = a.dc_ctl[kDcStat2] + (uint32_t)min(sv.st_chg, 0xFFFFFFFFull);
        a.dc_ctl[kDcStat2] = r < a.dc_ctl[kDcStat2] ? ~0u : r;
    }
    return ret;
}

// The leader's post of a phase: every wave's stores drained, then one release and the flag.
__device__ __forceinline__ void dc_post(const SweepArgs& a, uint32_t g) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&a.dc_ctl[kDcGen], g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <int NW, uint32_t BS>
__global__ __launch_bounds__(BS) void dc_multi_kernel(SweepArgs a, uint32_t K) {
    extern __shared__ uint4 dc_lds[];
    __shared__ float2 ewl[256];
    __shared__ uint2 xkeep[256];
    __shared__ uint32_t sh_g;
    uint32_t* const dyn = reinterpret_cast<uint32_t*>(dc_lds);
    const DcTabs tb = dc_tabs_load(a, ewl, xkeep);
    const bool leader = blockIdx.x == 0;
    const uint2* tab = a.dl_tab;   // the window, cached in LDS where it fits (dc_leader_solo loads it)
    if (a.dl_tab != nullptr && a.dl_n <= kDcTabLds) tab = reinterpret_cast<const uint2*>(dyn + kDcEvalLds / 4u + 2u * kDcCandCap);
    const uint32_t bl = a.block_log2, nbl = ((a.v_end - 1u) >> bl) - (a.v_begin >> bl) + 1u;
    const uint32_t moves_max = min(kDcSoloMovesMax, kDcSoloPairs / max(nbl, 1u));
    const bool solo_ok = a.dl_tab != nullptr && tb.ew != nullptr && a.taboo == nullptr && a.vflags == nullptr;
    uint32_t k = 0, last = 0, nfull = 0, mvexp = 0;
    __shared__ uint32_t s_seq;   // the leader's post count (its thread 0 posts the move phases)
    if (threadIdx.x == 0) s_seq = 0;
    unsigned long long nsolo = 0;
    __syncthreads();
    for (;;) {
        if (leader) {
            // solo sweeps (with move phases), then post what comes next: a full sweep or the exit
            uint32_t seq0 = s_seq;   // (thread 0's count is the one that moves: it posts)
            const uint32_t nxt = dc_leader_solo<NW>(a, K, k, tb, dyn, tab, solo_ok, moves_max, nsolo, seq0, mvexp);
            if (threadIdx.x == 0) s_seq = seq0 + 1u;
            __syncthreads();
            const uint32_t seq = s_seq;
            nfull += nxt == 1u ? 1u : 0u;
            dc_post(a, (seq << 2) | nxt);
            if (threadIdx.x == 0) {
                sh_g = (seq << 2) | nxt;
                if (nxt == 1u) {   // (its own L1: the last full sweep's data of other workgroups)
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            }
        } else if (threadIdx.x < 64u) {
            // wave 0 polls: a wave-uniform spin loop (a spin loop in one lane beside barriers in the
            // other waves lets the compiler's structurizer run the rest of the wave ahead of it)
            uint32_t g;
            const unsigned long long t0 = wall_clock64();
            while ((g = __builtin_amdgcn_readfirstlane(dc_ld(&a.dc_ctl[kDcGen]))) == last) {
                if (wall_clock64() - t0 > kDcIdleTicks) { g = 2u; break; }   // no leader: leave
                for (uint32_t z = 0; z < a.dc_poll; z++) __builtin_amdgcn_s_sleep(4);   // (>= 1)
            }
            if ((g & 3u) == 1u) {   // a full sweep reads plain data of the last phases: acquire
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            if (threadIdx.x == 0) sh_g = g;
        }
        __syncthreads();
        const uint32_t g = sh_g;
        last = g;
        __syncthreads();
        if ((g & 3u) == 2u) break;
        if ((g & 3u) == 3u) {   // a move phase (helpers only: the leader posts them from its solo loop)
            dc_help_moves<NW>(a);
            continue;
        }
        // a full sweep, every workgroup: the dense sweep of dense_counts.h; its committer signals
        const uint4 s4 = *reinterpret_cast<const uint4*>(a.st);
        const bool mine = dc_full_body<NW>(a, s4, tb, dyn);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0 && mine) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            atomicAdd(&a.dc_ctl[kDcCommitted], 1u);
        }
        if (leader && threadIdx.x < 64u) {   // the sweep is committed (its data released) before the leader plans the next
            const uint32_t nf = __builtin_amdgcn_readfirstlane(nfull);
            const unsigned long long t0 = wall_clock64();
            while (__builtin_amdgcn_readfirstlane(dc_ld(&a.dc_ctl[kDcCommitted])) < nf) {
                if (wall_clock64() - t0 > kDcWaitTicks) {   // the sweep never completed: flag (the solo loop stops)
                    if (threadIdx.x == 0) atomicOr(&a.st->err, kDevErrWatchdog);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        if (leader) k++;
    }
    if (leader) {
        if (threadIdx.x < 64u) {   // every helper saw the exit (wave 0 waits, wave-uniform)
            const unsigned long long t0 = wall_clock64();
            while (__builtin_amdgcn_readfirstlane(dc_ld(&a.dc_ctl[kDcAck])) < gridDim.x - 1u) {
                if (wall_clock64() - t0 > kDcWaitTicks) {
                    if (threadIdx.x == 0) atomicOr(&a.st->err, kDevErrWatchdog);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        if (threadIdx.x == 0) {   // the words are reset for the next launch
            a.dc_ctl[kDcGen] = 0u;
            a.dc_ctl[kDcAck] = 0u;
            a.dc_ctl[kDcCommitted] = 0u;
            a.dc_ctl[kDcMvDone] = 0u;
            if (nsolo) reinterpret_cast<unsigned long long*>(a.dc_ctl + kDcSoloStat)[0] += nsolo;
        }
    } else if (threadIdx.x == 0) {
        atomicAdd(&a.dc_ctl[kDcAck], 1u);
    }
}

template <int NW, uint32_t BS>
void launch_dcm(const SweepArgs& a, uint32_t K, dim3 g, hipStream_t s) {
    dc_multi_kernel<NW, BS><<<g, dim3(BS), kDcMultiLds, s>>>(a, K);
}
template <int NW, uint32_t BS>
hipError_t allow_lds_dcm() {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&dc_multi_kernel<NW, BS>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kDcMultiLds);
}
