// mcmc_colorer_amd/csrc/wide_tiled.h -- the wide sweep (nCol > 256, uint16 colours) over the tiled
// layout, for graphs that have no CSR: the build's generated G(n, p) at C3 size, where the
// reference's default colour count nCol = maxDeg (main.cu:162; about 10 500 at C3) applies and a
// CSR (4e11 B of uint32 ids) cannot exist beside the 2.2e11 B layout on one device. Included by
// mcmc_sweep.hip inside namespace mcmc, after sweep_wide.h.
//
// One wave per row, persistent (rows w, w + W, ... for the grid's W waves). The row's occupancy
// mask (count_free_colors, coloringMCMC_CPU.cpp:362-383: nCol bits) is built in the wave's own LDS
// words by scanning its segments of every column block of the layout (16-bit block-local ids; 4
// blocks per round, 16 lanes and 8 ids per lane in flight), the neighbours' colours gathered from
// the uint16 replica of C_t. Then, per the row's own colour and taboo counter:
//   taboo        the colour stays, the counter drops (:496-501);
//   violator     fill_p case (ii) or (i) and the exact CDF walk over the mask (walk_finish_wave:
//                word prefix counts, walk_mask_pre -- the wide sweep's violator walk);
//   otherwise    case (iii): own colour hi, others eps -- walk_own_tab over the eps prefix table.
// CDF overflows are appended to the event list; the stand-alone commit (commit_kernel<uint16_t>)
// replays them in ascending vertex order against glibc (:517-520) and runs the loop control.
// Every arc is read every sweep (the scan cannot stop early: a row without its own colour must
// see every neighbour), so a sweep moves the whole layout (2 B per arc) plus one 2-byte colour
// gather per arc from the replica (20 MB at C3: MALL-resident) -- exact, not fast: the dense and
// persistent sweeps of nCol <= 256 do not apply to masks of 10 000 colours.

// Waves per workgroup (8, or fewer when one wave's mask + prefix counts -- 2 NWW + 1 words -- make
// 8 of them exceed 144 KiB) and workgroups per CU: 24 waves per CU (the kernel's ~74 VGPRs allow 6
// per SIMD), as the LDS allows. Many waves in flight: a row's scan is a chain of dependent loads.
inline uint32_t wide_tiled_waves(uint32_t nCol) {
    const uint32_t nww = (nCol + 31u) >> 5;
    const uint32_t per = 4u * (2u * nww + 1u);
    uint32_t w = 8;
    while (w > 1 && (size_t)w * per > 144u * 1024u) w >>= 1;
    return w;
}
inline uint32_t wide_tiled_wgs_per_cu(uint32_t nCol) {
    const uint32_t W = wide_tiled_waves(nCol), per = 4u * (2u * ((nCol + 31u) >> 5) + 1u);
    return std::max<uint32_t>(1u, std::min<uint32_t>(24u / W, (uint32_t)((160u * 1024u) / ((size_t)W * per))));
}

// Incremental violation counts (r06): the scan above is needed for a row's mask only when the
// row violates (the walk of fill_p cases (i)/(ii) reads the mask); a non-violator's update is the
// own-colour walk of case (iii) (walk_own_tab), which needs nothing but its draw. So each row keeps
// vcnt = its neighbours of its own colour (violation_count, :329-351, is vcnt > 0) and a sweep in
// incremental mode runs
//   wt_eval_kernel   a lane per row: taboo rows keep their colour, non-violators take the own-colour
//                    walk, violators are listed;
//   wt_viol_kernel   a wave per listed violator: the scan and walk of the full sweep;
//   commit_kernel    as before (loop control, the glibc replay of the CDF overflows);
//   wt_diff_kernel   a lane per row: rows whose colour changed (C_t vs C_t+1, the replayed events
//                    included) listed, their arcs summed;
//   wt_delta_kernel  a wave per changed row u: for every arc (u, w) both counts move by
//                    [C_t+1 u == C_t+1 w] - [C_t u == C_t w] (an arc between two changed rows from the
//                    smaller end only).
// The full sweep (wide_tiled_kernel) counts vcnt in its scan. The delta kernel chooses the next
// sweep's mode: incremental while the changed rows' arcs are at most half the layout's (one gather
// per changed arc to an unchanged row against one per arc of a scan; the violators' walks cost the
// same either way), else full (the counts are then recounted by the scan). Exact: the
// counts are integers; tests/test_wide.py::test_wide_tiled_incremental* (against the oracle, the
// full mode, forced modes) and tests/test_c3_full.py.
constexpr uint32_t kWtMode = 0;   // the running sweep: 0 full (wide_tiled_kernel), 1 incremental
constexpr uint32_t kWtVN = 1;     // violators listed by wt_eval_kernel (zeroed by wt_diff_kernel)
constexpr uint32_t kWtCN = 2;     // changed rows listed by wt_diff_kernel (zeroed by the next sweep)
constexpr uint32_t kWtVDone = 3;  // listed violators walked by the calibration launch of wt_viol_kernel
constexpr uint32_t kWtArcs = 4;   // u64: their arcs
constexpr uint32_t kWtStat = 8;   // u64 [4]: full sweeps, incremental sweeps, changed rows, violator walks
constexpr uint32_t kWtWords = 16;

// Row l of the sweep: its mask from every column block of the layout (vcnt: its neighbours of its own
// colour, counted when FULL), then taboo / the violator walk / the own-colour walk. Returns viol.
template <bool FULL>
__device__ __forceinline__ uint32_t wt_row(const SweepArgs& a, uint32_t l, uint32_t t, uint32_t x_t,
                                           const uint16_t* __restrict__ C, uint16_t* __restrict__ Cs,
                                           uint32_t* mask, uint32_t* pre, unsigned long long tick) {
    DevState* st = a.st;
    const uint32_t NWW = (a.nCol + 31u) >> 5, lane = threadIdx.x & 63u;
    const uint32_t R = a.grp_rows, nb = a.nblocks, bl = a.block_log2;
    const uint32_t grp = lane >> 4, gl = lane & 15u;
    const uint32_t v = a.v_begin + l;
    const uint32_t cv = C[v];
    for (uint32_t i = lane; i < NWW; i += 64u) mask[i] = 0u;
    wave_lds_sync();
    const uint32_t g = l / R, r = l - g * R;
    const uint16_t* __restrict__ gc = a.tcol + a.gbase[g];
    uint64_t deg = 0;
    uint32_t same = 0;
    const uint32_t bs = tick ? (uint32_t)((wall_clock64() / tick) % nb) : 0u;
    for (uint32_t b0 = 0; b0 < nb; b0 += 4u) {
        const uint32_t bi = b0 + grp;
        const uint32_t b = bi + bs < nb ? bi + bs : bi + bs - nb;
        uint32_t s0 = 0, s1 = 0;
        if (bi < nb) {
            const uint32_t* ts = a.tseg + ((size_t)g * nb + b) * tseg_stride(R);
            const uint32_t raw = ts[r];
            s0 = raw & kTsegPos;
            s1 = (ts[r + 1] & kTsegPos) - (raw & 7u);
        }
        if (gl == 0 && s1 > s0) deg += s1 - s0;
        const uint32_t lo = b << bl;
        for (uint32_t k = s0 + gl; __ballot(k < s1); k += 128u) {
            uint32_t c[8];
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const uint32_t kk = k + 16u * q;
                c[q] = kk < s1 ? (uint32_t)C[lo | gc[kk]] : 0xFFFFFFFFu;
            }
#pragma unroll
            for (int q = 0; q < 8; q++)
                if (c[q] != 0xFFFFFFFFu) {
                    atomicOr(&mask[c[q] >> 5], 1u << (c[q] & 31u));
                    if (FULL) same += c[q] == cv ? 1u : 0u;
                }
        }
    }
    for (int o = 32; o > 0; o >>= 1) deg += __shfl_xor(deg, o, 64);
    if (FULL && a.wt_ctl != nullptr) {
        for (int o = 32; o > 0; o >>= 1) same += __shfl_xor(same, o, 64);
        if (lane == 0) {
            a.wt_vcnt[l] = same;
            a.wt_deg[l] = (uint32_t)min(deg, (uint64_t)0xFFFFFFFFu);
        }
    }
    wave_lds_sync();
    const uint32_t tab = a.taboo != nullptr ? a.taboo[l] : 0u;
    const uint32_t viol = (mask[cv >> 5] >> (cv & 31u)) & 1u;
    if (a.vflags != nullptr && lane == 0) a.vflags[(size_t)(t & 1u) * (a.v_end - a.v_begin) + l] = (uint8_t)viol;   // tail cut
    // u_v: engine draw K_t + v + 1 (coloringMCMC_CPU.cpp:139)
    const uint32_t x = minstd_mulmod(x_t, minstd_pow_tab_wave((uint64_t)v + 1ull));
    if (tab > 0) {   // :496-501
        if (lane == 0) {
            Cs[v] = (uint16_t)cv;
            a.taboo[l] = tab - 1u;
        }
    } else if (viol) {   // case (ii) / (i): the walk over the mask (writes Cs, taboo, the event)
        walk_finish_wave<false>(a, v, t, cv, x, (uint32_t)min(deg, (uint64_t)0xFFFFFFFFu), Cs, mask, pre, nullptr, nullptr,
                                lane);
    } else if (lane == 0) {   // case (iii)
        const uint32_t nc = walk_own_tab(a.etab, a.nCol, cv, a.eps, a.hi, minstd_canonical(x));
        const bool event = nc == a.nCol;
        Cs[v] = (uint16_t)(event ? cv : nc);
        if (a.taboo != nullptr && !event) a.taboo[l] = (nc == cv) ? a.tabooIteration : 0u;
        if (event) {
            const uint32_t idx = atomicAdd(&st->ev_count, 1u);
            if (idx < a.ev_cap) a.events[idx] = v;
            else atomicOr(&st->err, kDevErrEvents);
        }
    }
    wave_lds_sync();   // the walk's LDS reads are done before the next row clears the mask
    return viol;
}

__global__ __launch_bounds__(512) void wide_tiled_kernel(SweepArgs a) {
    extern __shared__ uint32_t wt_lds[];
    __shared__ uint32_t sh_viol;
    DevState* st = a.st;
    if (a.check_done && st->done) return;
    // an incremental sweep (wt_eval_kernel), or a full one run as recount + the incremental kernels
    if (a.wt_ctl != nullptr && (a.wt_ctl[kWtMode] != 0u || a.wt_rc)) return;
    if (threadIdx.x == 0) sh_viol = 0;
    if (a.wt_ctl != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {
        a.wt_ctl[kWtCN] = 0u;   // (the last sweep's delta has run)
        reinterpret_cast<unsigned long long*>(a.wt_ctl + kWtArcs)[0] = 0ull;
        reinterpret_cast<unsigned long long*>(a.wt_ctl + kWtStat)[0] += 1ull;
    }
    __syncthreads();
    const uint32_t t = st->t, x_t = st->x_t;
    const uint16_t* __restrict__ C = reinterpret_cast<const uint16_t*>((t & 1) ? a.colors1 : a.colors0);
    uint16_t* __restrict__ Cs = reinterpret_cast<uint16_t*>((t & 1) ? a.colors0 : a.colors1);
    const uint32_t nloc = a.v_end - a.v_begin, NWW = (a.nCol + 31u) >> 5;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    uint32_t* const mask = wt_lds + (size_t)wave * (2u * NWW + 1u);
    uint32_t* const pre = mask + NWW;
    const uint32_t nb = a.nblocks;
    uint32_t wave_viol = 0, nrows = 0;
    // Block rotation: a row's mask is an OR, so its blocks may be scanned in any cyclic order. Each
    // row starts at the block a common clock points to (one block per tick, the tick measured on
    // the previous sweep), so all waves gather from a narrow window of colour slices at any time --
    // one XCD's L2 holds it, where the 2 B x n replica (20 MB at C3) does not fit.
    const unsigned long long tick = a.wt_tick != nullptr ? *a.wt_tick : 0ull;
    const unsigned long long t_begin = wall_clock64();
    for (uint32_t l = blockIdx.x * nwv + wave; l < nloc; l += gridDim.x * nwv) {
        nrows++;
        wave_viol += wt_row<true>(a, l, t, x_t, C, Cs, mask, pre, tick);
    }
    if (lane == 0 && wave_viol) atomicAdd(&sh_viol, wave_viol);
    if (a.wt_tick != nullptr && blockIdx.x == 0 && threadIdx.x == 0 && nrows > 0) {   // next sweep's tick
        const unsigned long long d = (wall_clock64() - t_begin) / ((unsigned long long)nrows * nb);
        *a.wt_tick = d > 0 ? d : 1ull;
    }
    __syncthreads();
    if (threadIdx.x == 0 && sh_viol) atomicAdd(&st->viol, (unsigned long long)sh_viol);
}

// An incremental sweep, a lane per row: Cviol from the counts; taboo rows keep their colour (the
// counter drops); non-violators take the own-colour walk (case (iii), CDF overflows to the event
// list); violators are listed for wt_viol_kernel, which writes their colours.
__global__ __launch_bounds__(256) void wt_eval_kernel(SweepArgs a) {
    __shared__ uint32_t sh_viol;
    DevState* st = a.st;
    if (a.check_done && st->done) return;
    const bool inc = a.wt_ctl[kWtMode] != 0u;
    if (!inc && !a.wt_rc) return;   // a full sweep: wide_tiled_kernel (or wt_recount_kernel, then this)
    if (threadIdx.x == 0) sh_viol = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.wt_ctl[kWtCN] = 0u;
        reinterpret_cast<unsigned long long*>(a.wt_ctl + kWtArcs)[0] = 0ull;
        if (inc) reinterpret_cast<unsigned long long*>(a.wt_ctl + kWtStat)[1] += 1ull;
    }
    __syncthreads();
    const uint32_t t = st->t, x_t = st->x_t;
    const uint16_t* __restrict__ C = reinterpret_cast<const uint16_t*>((t & 1) ? a.colors1 : a.colors0);
    uint16_t* __restrict__ Cs = reinterpret_cast<uint16_t*>((t & 1) ? a.colors0 : a.colors1);
    const uint32_t nloc = a.v_end - a.v_begin, lane = threadIdx.x & 63u;
    uint32_t wave_viol = 0;
    // u_v's engine state x_t 16807^(v+1): the wave's first row's power on the scalar unit times
    // 16807^lane (a per-lane exponent would be a chain of ~22 dependent table loads and mulmods)
    const uint32_t lpow = kMinstdLanePow[lane];
    const uint32_t wstep = minstd_pow_tab_wave((uint64_t)gridDim.x * blockDim.x);
    uint32_t xw = minstd_mulmod(x_t, minstd_pow_tab_wave((uint64_t)a.v_begin + blockIdx.x * blockDim.x +
                                                         (threadIdx.x & ~63u) + 1ull));
    for (uint32_t base = blockIdx.x * blockDim.x; base < nloc; base += gridDim.x * blockDim.x) {
        const uint32_t l = base + threadIdx.x;
        const uint32_t xl = minstd_mulmod(xw, lpow);
        xw = __builtin_amdgcn_readfirstlane(minstd_mulmod(xw, wstep));
        const bool in = l < nloc;
        const uint32_t v = a.v_begin + l;
        const uint32_t cv = in ? (uint32_t)C[v] : 0u;
        const uint32_t viol = in && a.wt_vcnt[l] != 0u ? 1u : 0u;
        const uint32_t tab = (in && a.taboo != nullptr) ? a.taboo[l] : 0u;
        if (in && a.vflags != nullptr) a.vflags[(size_t)(t & 1u) * nloc + l] = (uint8_t)viol;   // tail cut
        wave_viol += (uint32_t)__popcll(__ballot(viol != 0u));
        const bool walk = in && tab == 0u && viol;
        const uint64_t wb = __ballot(walk);
        if (wb) {   // violators to the list (one reservation per wave)
            uint32_t b0 = 0;
            if (lane == 0) b0 = atomicAdd(&a.wt_ctl[kWtVN], (uint32_t)__popcll(wb));
            b0 = __shfl(b0, 0, 64);
            if (walk) a.wt_list[b0 + (uint32_t)__popcll(wb & ((1ull << lane) - 1ull))] = l;
        }
        bool event = false;
        if (in && tab > 0u) {   // :496-501
            Cs[v] = (uint16_t)cv;
            a.taboo[l] = tab - 1u;
        } else if (in && !viol) {   // case (iii)
            const uint32_t nc = walk_own_tab(a.etab, a.nCol, cv, a.eps, a.hi, minstd_canonical(xl));
            event = nc == a.nCol;
            Cs[v] = (uint16_t)(event ? cv : nc);
            if (a.taboo != nullptr && !event) a.taboo[l] = (nc == cv) ? a.tabooIteration : 0u;
        }
        const uint64_t eb = __ballot(event);
        if (eb) {
            uint32_t e0 = 0;
            if (lane == 0) e0 = atomicAdd(&st->ev_count, (uint32_t)__popcll(eb));
            e0 = __shfl(e0, 0, 64);
            if (event) {
                const uint32_t idx = e0 + (uint32_t)__popcll(eb & ((1ull << lane) - 1ull));
                if (idx < a.ev_cap) a.events[idx] = v;
                else atomicOr(&st->err, kDevErrEvents);
            }
        }
    }
    if (lane == 0 && wave_viol) atomicAdd(&sh_viol, wave_viol);
    __syncthreads();
    if (threadIdx.x == 0 && sh_viol) atomicAdd(&st->viol, (unsigned long long)sh_viol);
}

// The listed violators of an incremental sweep, a wave each: the full sweep's scan and walk.
// CAL (launched first, where the rotation has a clock): while no tick has been measured (the
// colouring's first sweep), one row a wave without rotation, timed -- the tick for the rest, which
// the main launch walks with rotation; otherwise returns at once and the main launch walks all.
template <bool CAL>
__global__ __launch_bounds__(512) void wt_viol_kernel(SweepArgs a) {
    extern __shared__ uint32_t wt_lds[];
    DevState* st = a.st;
    if (a.check_done && st->done) return;
    if (a.wt_ctl[kWtMode] == 0u && !a.wt_rc) return;
    const uint32_t nv = a.wt_ctl[kWtVN];
    const uint32_t t = st->t, x_t = st->x_t;
    const uint16_t* __restrict__ C = reinterpret_cast<const uint16_t*>((t & 1) ? a.colors1 : a.colors0);
    uint16_t* __restrict__ Cs = reinterpret_cast<uint16_t*>((t & 1) ? a.colors0 : a.colors1);
    const uint32_t NWW = (a.nCol + 31u) >> 5, wave = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    uint32_t* const mask = wt_lds + (size_t)wave * (2u * NWW + 1u);
    uint32_t* const pre = mask + NWW;
    const unsigned long long tick = a.wt_tick != nullptr ? *a.wt_tick : 0ull;
    const uint32_t nwg = gridDim.x * nwv;
    if (CAL) {
        const bool cal = tick == 0ull && nv >= 4u * nwg;   // (a short list: no rotation needed)
        if (blockIdx.x == 0 && threadIdx.x == 0) a.wt_ctl[kWtVDone] = cal ? nwg : 0u;
        if (!cal) return;
        const unsigned long long t0 = wall_clock64();
        (void)wt_row<false>(a, a.wt_list[blockIdx.x * nwv + wave], t, x_t, C, Cs, mask, pre, 0ull);
        if (blockIdx.x == 0 && threadIdx.x == 0) *a.wt_tick = max(1ull, (wall_clock64() - t0) / a.nblocks);
        return;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) reinterpret_cast<unsigned long long*>(a.wt_ctl + kWtStat)[3] += nv;
    const unsigned long long t_begin = wall_clock64();
    uint32_t nrows = 0;
    for (uint32_t i = (a.wt_tick != nullptr ? a.wt_ctl[kWtVDone] : 0u) + blockIdx.x * nwv + wave; i < nv; i += nwg) {
        nrows++;
        (void)wt_row<false>(a, a.wt_list[i], t, x_t, C, Cs, mask, pre, tick);
    }
    // the next sweep's block rotation tick (as wide_tiled_kernel measures it), from a walk of several
    // rows a wave (a full sweep's violators, the recount's sweeps)
    if (a.wt_tick != nullptr && blockIdx.x == 0 && threadIdx.x == 0 && nrows >= 4u) {
        const unsigned long long d = (wall_clock64() - t_begin) / ((unsigned long long)nrows * a.nblocks);
        *a.wt_tick = d > 0 ? d : 1ull;
    }
}

// A full sweep's counts from scratch (SweepArgs::wt_rc), then the incremental sweep's own kernels
// run the sweep (violators walked from the list). Block-major: a workgroup holds one column block's
// colours in LDS (loaded once) and streams a range of row groups' ids in that block (coalesced
// quads), kWtRcK groups' segment tables per round; a quad's row is a binary search of its table, an
// own-colour match a global atomic on the row's count (rare: a colour's share of the arcs). The ids
// are read once and no colour is gathered from the fabric (the mask scan of wide_tiled_kernel reads
// a fabric line per arc). vcnt = the row's neighbours of its own colour, deg = its neighbours (the
// layout's ids, as wt_row<true> counts them).
constexpr uint32_t kWtRcMaxK = 4;   // row groups' segment tables per round
inline uint32_t wt_rc_k(uint32_t block_log2, uint32_t R) {
    const size_t room = 160u * 1024u - 2ull * (1ull << block_log2) - 64u;
    return (uint32_t)std::min<size_t>(kWtRcMaxK, room / (6ull * R + 8u));   // 0: does not fit
}
inline size_t wt_recount_lds(uint32_t block_log2, uint32_t R, uint32_t k) {   // slice, tables, own colours
    return 2ull * (1ull << block_log2) + 4ull * k * (R + 1u) + 2ull * k * ((R + 1u) & ~1u);
}
// vcnt = 0 and deg = the row's ids over every block (a lane per row; the tables read row-coalesced).
__global__ __launch_bounds__(256) void wt_rc_zero_kernel(SweepArgs a) {
    if (a.check_done && a.st->done) return;
    if (a.wt_ctl[kWtMode] != 0u) return;
    const uint32_t nloc = a.v_end - a.v_begin, R = a.grp_rows, nb = a.nblocks;
    for (uint32_t l = blockIdx.x * blockDim.x + threadIdx.x; l < nloc; l += gridDim.x * blockDim.x) {
        const uint32_t g = l / R, r = l - g * R;
        uint64_t deg = 0;
        for (uint32_t b = 0; b < nb; b++) {
            const uint32_t* ts = a.tseg + ((size_t)g * nb + b) * tseg_stride(R);
            const uint32_t raw = ts[r];
            deg += (ts[r + 1] & kTsegPos) - (raw & 7u) - (raw & kTsegPos);
        }
        a.wt_vcnt[l] = 0u;
        a.wt_deg[l] = (uint32_t)min(deg, (uint64_t)0xFFFFFFFFu);
    }
}
// Grid: nblocks x S workgroups, workgroup (b, s) = block b over the s-th of S ranges of row groups.
__global__ __launch_bounds__(1024) void wt_recount_kernel(SweepArgs a, uint32_t S, uint32_t K) {
    extern __shared__ uint4 wt_rc_lds[];
    DevState* st = a.st;
    if (a.check_done && st->done) return;
    if (a.wt_ctl[kWtMode] != 0u) return;   // an incremental sweep: the counts are current
    const uint32_t t = st->t;
    const uint16_t* __restrict__ C = reinterpret_cast<const uint16_t*>((t & 1) ? a.colors1 : a.colors0);
    const uint32_t R = a.grp_rows, nb = a.nblocks, bl = a.block_log2, bsz = 1u << bl, ng = a.ngroups;
    const uint32_t nloc = a.v_end - a.v_begin, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    const uint32_t b = blockIdx.x / S, s = blockIdx.x - b * S;
    const uint32_t g0 = (uint32_t)((uint64_t)ng * s / S), g1 = (uint32_t)((uint64_t)ng * (s + 1u) / S);
    uint16_t* const sl = reinterpret_cast<uint16_t*>(wt_rc_lds);   // [bsz] block b's colours
    uint32_t* const tab = reinterpret_cast<uint32_t*>(sl + bsz);   // [K][R + 1] segment tables
    uint16_t* const own = reinterpret_cast<uint16_t*>(tab + K * (R + 1u));   // [K][R] their rows' colours
    __shared__ uint64_t sh_gb[kWtRcMaxK];
    if (blockIdx.x == 0 && threadIdx.x == 0) reinterpret_cast<unsigned long long*>(a.wt_ctl + kWtStat)[0] += 1ull;
    {   // block b's colours by LDS-DMA (1 KiB per wave-instruction; the replicas hold n + 256)
        const uint32_t blo = b << bl, npad = a.n + 256u;
        const uint32_t npc = (2u * min(bsz, npad - min(npad, blo)) + 15u) >> 4;
        const uint32_t lds0 = lds_addr(sl);
        for (uint32_t w = wv; w * 64u < npc; w += nwv) {
            const uint32_t pc = min(w * 64u + lane, npc - 1u);
            glds16(reinterpret_cast<const uint8_t*>(C + blo) + 16u * pc, __builtin_amdgcn_readfirstlane(lds0 + w * 1024u));
        }
    }
    for (uint32_t gb = g0; gb < g1; gb += K) {
        const uint32_t kk = min(K, g1 - gb);
        __syncthreads();   // the last round's readers of the tables are done
        for (uint32_t i = threadIdx.x; i < kk * (R + 1u); i += blockDim.x) {
            const uint32_t j = i / (R + 1u), r = i - j * (R + 1u), g = gb + j;
            const uint32_t rows = min(R, nloc - g * R);
            if (r <= rows) tab[i] = a.tseg[((size_t)g * nb + b) * tseg_stride(R) + r];
            if (r < rows) own[j * R + r] = C[a.v_begin + g * R + r];
        }
        if (threadIdx.x < kk) sh_gb[threadIdx.x] = a.gbase[gb + threadIdx.x];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (and the slice's DMA, the first round)
        __syncthreads();
        uint32_t pre[kWtRcMaxK + 1], p0[kWtRcMaxK];   // the round's quads: groups' ranges back to back
        pre[0] = 0u;
#pragma unroll
        for (uint32_t j = 0; j < kWtRcMaxK; j++) {
            uint32_t nq = 0;
            if (j < kk) {
                const uint32_t rows = min(R, nloc - (gb + j) * R);
                p0[j] = tab[j * (R + 1u)] & kTsegPos;
                nq = ((tab[j * (R + 1u) + rows] & kTsegPos) - p0[j]) >> 3;
            }
            pre[j + 1] = pre[j] + nq;
        }
        const uint32_t tot = pre[kWtRcMaxK];
        constexpr uint32_t kQ = 8;   // quads per thread in flight
        for (uint32_t q0 = 0; q0 < tot; q0 += kQ * blockDim.x) {
            uint4 v[kQ];
            uint32_t jq[kQ], pq[kQ];
#pragma unroll
            for (uint32_t u = 0; u < kQ; u++) {
                const uint32_t q = q0 + u * blockDim.x + threadIdx.x;
                uint32_t j = 0;
#pragma unroll
                for (uint32_t m = 1; m < kWtRcMaxK; m++) j += q >= pre[m] ? 1u : 0u;
                jq[u] = j;
                pq[u] = q < tot ? p0[j] + 8u * (q - pre[j]) : 0u;
                v[u] = q < tot ? *reinterpret_cast<const uint4*>(a.tcol + sh_gb[j] + pq[u]) : make_uint4(0u, 0u, 0u, 0u);
            }
#pragma unroll
            for (uint32_t u = 0; u < kQ; u++) {
                const uint32_t q = q0 + u * blockDim.x + threadIdx.x;
                if (q >= tot) continue;
                const uint32_t j = jq[u], pos = pq[u], g = gb + j;
                const uint32_t* tj = tab + j * (R + 1u);
                // the row holding pos (the last with start <= pos): a guess at the group's mean row
                // length, widened by doubling steps to a bracket, then halved
                const uint32_t rows = min(R, nloc - g * R), pe = tj[rows] & kTsegPos;
                uint32_t lo = min(rows - 1u, (uint32_t)((uint64_t)(pos - p0[j]) * rows / max(1u, pe - p0[j]))), hi;
                if ((tj[lo] & kTsegPos) <= pos) {
                    uint32_t st = 1;
                    while (lo + st < rows && (tj[lo + st] & kTsegPos) <= pos) { lo += st; st *= 2u; }
                    hi = min(lo + st, rows);
                } else {
                    uint32_t st = 1;
                    hi = lo;
                    while (hi >= st && (tj[hi - st] & kTsegPos) > pos) { hi -= st; st *= 2u; }
                    lo = hi >= st ? hi - st : 0u;
                }
                while (hi - lo > 1u) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if ((tj[mid] & kTsegPos) <= pos) lo = mid; else hi = mid;
                }
                const int nv = (int)((tj[lo + 1u] & kTsegPos) - (tj[lo] & 7u)) - (int)pos;   // its real ids here
                const uint32_t l = g * R + lo, cv = own[j * R + lo];
                const uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
                uint32_t same = 0;
#pragma unroll
                for (int k = 0; k < 8; k++)
                    if (k < nv) same += (uint32_t)sl[(w4[k >> 1] >> (16 * (k & 1))) & 0xFFFFu] == cv ? 1u : 0u;
                if (same) atomicAdd(&a.wt_vcnt[l], same);
            }
        }
    }
}

// After the commit of an accepted sweep (st->t = t + 1): the rows whose colour changed from C_t to
// C_t+1, listed (after the violators, which wt_viol_kernel has consumed: their count is reset here)
// and marked in wt_chg, their arcs summed. A lane per 8-row group (global v / 8): two 16-byte loads,
// one byte of wt_chg; the list reserved once per wave (a prefix sum of the lanes' changes).
__global__ __launch_bounds__(256) void wt_diff_kernel(SweepArgs a) {
    DevState* st = a.st;
    if (st->done) return;
    const uint32_t t1 = st->t;
    const uint16_t* __restrict__ Cn = reinterpret_cast<const uint16_t*>((t1 & 1) ? a.colors1 : a.colors0);
    const uint16_t* __restrict__ Co = reinterpret_cast<const uint16_t*>((t1 & 1) ? a.colors0 : a.colors1);
    const uint32_t nloc = a.v_end - a.v_begin, lane = threadIdx.x & 63u;
    uint32_t* const list = a.wt_list + nloc;
    if (blockIdx.x == 0 && threadIdx.x == 0) a.wt_ctl[kWtVN] = 0u;
    const uint32_t g0 = a.v_begin >> 3, ng = ((a.v_end + 7u) >> 3) - g0;
    unsigned long long arcs = 0;
    for (uint32_t base = blockIdx.x * blockDim.x; base < ng; base += gridDim.x * blockDim.x) {
        const uint32_t q = base + threadIdx.x, v0 = (g0 + q) << 3;
        uint32_t m = 0;
        if (q < ng && v0 >= a.v_begin && v0 + 8u <= a.v_end) {
            const uint4 xn = *reinterpret_cast<const uint4*>(Cn + v0), xo = *reinterpret_cast<const uint4*>(Co + v0);
            const uint32_t d[4] = {xn.x ^ xo.x, xn.y ^ xo.y, xn.z ^ xo.z, xn.w ^ xo.w};
#pragma unroll
            for (int i = 0; i < 4; i++) m |= ((d[i] & 0xFFFFu) ? 1u : 0u) << (2 * i) | ((d[i] >> 16) ? 2u : 0u) << (2 * i);
        } else if (q < ng) {   // the range's first and last group
            for (uint32_t i = 0; i < 8u; i++) {
                const uint32_t v = v0 + i;
                if (v >= a.v_begin && v < a.v_end && Cn[v] != Co[v]) m |= 1u << i;
            }
        }
        if (q < ng) a.wt_chg[q] = (uint8_t)m;
        const uint32_t k = (uint32_t)__builtin_popcount(m);
        uint32_t incl = k;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= (uint32_t)o) incl += y;
        }
        const uint32_t tot = __shfl(incl, 63, 64);
        if (tot == 0u) continue;
        uint32_t b0 = 0;
        if (lane == 63u) b0 = atomicAdd(&a.wt_ctl[kWtCN], tot);
        b0 = __shfl(b0, 63, 64) + incl - k;
        for (uint32_t mm = m; mm; mm &= mm - 1u) {
            const uint32_t l = v0 + (uint32_t)__builtin_ctz(mm) - a.v_begin;
            list[b0++] = l;
            arcs += a.wt_deg[l];
        }
    }
    for (int o = 32; o > 0; o >>= 1) arcs += __shfl_xor(arcs, o, 64);
    if (lane == 0 && arcs) atomicAdd(reinterpret_cast<unsigned long long*>(a.wt_ctl + kWtArcs), arcs);
}

// The counts of C_t+1 from those of C_t, a wave per changed row (the next sweep incremental), or
// the next sweep full when the changed arcs cost more than a scan (MCMC_WT_INC: 0 never incremental,
// 2 always). Every workgroup reads the same totals and takes the same decision.
__global__ __launch_bounds__(512) void wt_delta_kernel(SweepArgs a, uint64_t arcs_max) {
    DevState* st = a.st;
    if (st->done) return;
    const uint32_t nch = a.wt_ctl[kWtCN];
    const unsigned long long arcs = reinterpret_cast<const unsigned long long*>(a.wt_ctl + kWtArcs)[0];
    const bool inc = arcs <= arcs_max;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.wt_ctl[kWtMode] = inc ? 1u : 0u;
        reinterpret_cast<unsigned long long*>(a.wt_ctl + kWtStat)[2] += nch;
    }
    if (!inc) return;
    const uint32_t t1 = st->t;
    const uint16_t* __restrict__ Cn = reinterpret_cast<const uint16_t*>((t1 & 1) ? a.colors1 : a.colors0);
    const uint16_t* __restrict__ Co = reinterpret_cast<const uint16_t*>((t1 & 1) ? a.colors0 : a.colors1);
    const uint32_t nloc = a.v_end - a.v_begin, lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    const uint32_t R = a.grp_rows, nb = a.nblocks, bl = a.block_log2;
    const uint32_t grp = lane >> 4, gl = lane & 15u;
    const uint32_t* __restrict__ list = a.wt_list + nloc;
    const uint8_t* __restrict__ chg = a.wt_chg;
    const uint32_t g0 = a.v_begin >> 3;
    for (uint32_t i = blockIdx.x * nwv + wave; i < nch; i += gridDim.x * nwv) {
        const uint32_t l = list[i], u = a.v_begin + l;
        const uint32_t cu = Co[u], cu1 = Cn[u];
        const uint32_t g = l / R, r = l - g * R;
        const uint16_t* __restrict__ gc = a.tcol + a.gbase[g];
        int own = 0;
        for (uint32_t b0 = 0; b0 < nb; b0 += 4u) {
            const uint32_t b = b0 + grp;
            uint32_t s0 = 0, s1 = 0;
            if (b < nb) {
                const uint32_t* ts = a.tseg + ((size_t)g * nb + b) * tseg_stride(R);
                const uint32_t raw = ts[r];
                s0 = raw & kTsegPos;
                s1 = (ts[r + 1] & kTsegPos) - (raw & 7u);
            }
            const uint32_t lo = b << bl;
            for (uint32_t k = s0 + gl; __ballot(k < s1); k += 64u) {
                uint32_t w[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t kk = k + 16u * q;
                    w[q] = kk < s1 ? (lo | (uint32_t)gc[kk]) : 0xFFFFFFFFu;
                }
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    if (w[q] == 0xFFFFFFFFu) continue;
                    // C_t+1 w, and C_t w only where w changed (wt_chg: 1.25 MB at C3, L2-resident)
                    const uint32_t cw1 = Cn[w[q]], lw0 = w[q] - a.v_begin;
                    const bool wch = lw0 < nloc ? ((chg[(w[q] >> 3) - g0] >> (w[q] & 7u)) & 1u) != 0u : true;
                    const uint32_t cw = wch ? (uint32_t)Co[w[q]] : cw1;
                    const int d = (cu1 == cw1 ? 1 : 0) - (cu == cw ? 1 : 0);
                    if (d == 0 || (cw != cw1 && w[q] < u)) continue;   // (both changed: the smaller end)
                    own += d;
                    const uint32_t lw = w[q] - a.v_begin;
                    if (lw < nloc) atomicAdd(&a.wt_vcnt[lw], (uint32_t)d);
                }
            }
        }
        for (int o = 32; o > 0; o >>= 1) own += __shfl_xor(own, o, 64);
        if (lane == 0 && own) atomicAdd(&a.wt_vcnt[l], (uint32_t)own);
    }
}
void launch_wide_tiled(const SweepArgs& a, dim3 g, dim3 b, size_t lds, hipStream_t s) {
    wide_tiled_kernel<<<g, b, lds, s>>>(a);
}
