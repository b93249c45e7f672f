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
// So a sweep is three launches plus the commit (commit_kernel<uint16_t>):
//   wide_scan_kernel  arc-parallel pass over the CSR in 256-arc chunks (64 lanes x one dwordx4 of
//                     ids): neighbour colour == own colour -> viol flag of the row (plain byte
//                     store; conflicts are rare, so the flags cost almost no traffic). The row of
//                     an arc comes from a per-chunk first-row table and a short binary search.
//   wide_eval_kernel  lane per vertex: viol -> Cviol and, untaboo'd, the violator list;
//                     otherwise u_v, walk_own (cdf_walk.h), Cstar / taboo / overflow event.
//   wide_walk_kernel  one 256-thread workgroup per violator: occupancy mask of nCol bits in LDS
//                     (ds_or), Zvcomp by popcount, pf, walk_mask over runs of equal p.
// All three are persistent (grid-stride) and exit at once when the loop is done.

constexpr uint32_t kWideChunk = 256;      // arcs per wave chunk: 64 lanes x 4 ids
constexpr uint32_t kWideMaskWords = 2048; // nCol <= 65536
constexpr uint32_t kWideMaxCol = 65535;
constexpr int kWideWalkThreads = 256;

__global__ __launch_bounds__(256) void wide_scan_kernel(SweepArgs a) {
    DevState* st = a.st;
    if (a.check_done && st->done) return;
    const uint32_t t = st->t;
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.wcount = 0;   // the walk list of this sweep
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
        uint32_t own = C[a.v_begin + r];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint64_t k = k0 + i;
            if (k >= m) break;
            if (rend <= k) {
                do { r++; rend = ro[r + 1] - a0; } while (rend <= k);
                own = C[a.v_begin + r];
            }
            if (nc[i] == own) a.wflag[r] = 1;
        }
    }
}

__global__ __launch_bounds__(256) void wide_eval_kernel(SweepArgs a) {
    __shared__ uint32_t sh_viol;
    DevState* st = a.st;
    if (a.check_done && st->done) return;
    if (threadIdx.x == 0) sh_viol = 0;
    const uint32_t t = st->t, x_t = st->x_t;
    const uint16_t* __restrict__ C = reinterpret_cast<const uint16_t*>((t & 1) ? a.colors1 : a.colors0);
    uint16_t* __restrict__ Cs = reinterpret_cast<uint16_t*>((t & 1) ? a.colors0 : a.colors1);
    const uint32_t nloc = a.v_end - a.v_begin;
    const int lane = threadIdx.x & 63;
    uint32_t cviol = 0;
    // u_v: engine draw K_t + v + 1 (bulk draw in vertex order, coloringMCMC_CPU.cpp:139); the
    // grid-stride loop advances every lane's draw by 16807^stride, one mulmod per vertex
    const uint32_t stride = gridDim.x * blockDim.x;
    const uint32_t a_stride = minstd_pow_tab(stride);
    uint32_t x = minstd_mulmod(minstd_mulmod(x_t, minstd_pow_tab((uint64_t)a.v_begin + blockIdx.x * blockDim.x +
                                                                 (threadIdx.x & ~63u) + 1)),
                               kMinstdLanePow[lane]);
    for (uint32_t base = blockIdx.x * blockDim.x; base < nloc; base += stride, x = minstd_mulmod(x, a_stride)) {
        const uint32_t l = base + threadIdx.x;
        const bool valid = l < nloc;
        const uint32_t v = a.v_begin + l;
        const float u = minstd_canonical(x);
        uint32_t viol = 0, cv = 0, tab = 0;
        if (valid) {
            viol = a.wflag[l];
            if (viol) a.wflag[l] = 0;
            cv = C[v];
            if (a.taboo != nullptr) tab = a.taboo[l];
        }
        cviol += viol;
        bool event = false, walk = false;
        if (valid) {
            if (tab > 0) {   // :496-501
                Cs[v] = (uint16_t)cv;
                a.taboo[l] = tab - 1;
            } else if (viol) {
                walk = true;   // case (i) or (ii): needs the occupancy set
            } else {           // case (iii)
                const uint32_t nc = walk_own_tab(a.etab, a.nCol, cv, a.eps, a.hi, u);
                event = nc == a.nCol;
                Cs[v] = (uint16_t)(event ? cv : nc);   // an event's colour is the commit's replay
                if (a.taboo != nullptr && !event) a.taboo[l] = (nc == cv) ? a.tabooIteration : 0u;
            }
        }
        const uint64_t wb = __ballot(walk);
        if (wb) {
            uint32_t b = 0;
            if (lane == 0) b = atomicAdd(a.wcount, (uint32_t)__popcll(wb));
            b = __shfl(b, 0, 64);
            if (walk) a.wlist[b + (uint32_t)__popcll(wb & ((1ull << lane) - 1ull))] = v;
        }
        const uint64_t eb = __ballot(event);
        if (eb) {
            uint32_t b = 0;
            if (lane == 0) b = atomicAdd(&st->ev_count, (uint32_t)__popcll(eb));
            b = __shfl(b, 0, 64);
            if (event) {
                const uint32_t idx = b + (uint32_t)__popcll(eb & ((1ull << lane) - 1ull));
                if (idx < a.ev_cap) a.events[idx] = v;
                else atomicOr(&st->err, 1u);
            }
        }
    }
    __syncthreads();
    for (int off = 32; off >= 1; off >>= 1) cviol += __shfl_xor(cviol, off, 64);
    if (lane == 0 && cviol) atomicAdd(&sh_viol, cviol);
    __syncthreads();
    if (threadIdx.x == 0 && sh_viol) atomicAdd(&st->viol, (unsigned long long)sh_viol);
}

__global__ __launch_bounds__(kWideWalkThreads) void wide_walk_kernel(SweepArgs a) {
    __shared__ uint32_t mask[kWideMaskWords];
    __shared__ uint32_t sh_pop;
    DevState* st = a.st;
    if (a.check_done && st->done) return;
    const uint32_t t = st->t, x_t = st->x_t;
    const uint16_t* __restrict__ C = reinterpret_cast<const uint16_t*>((t & 1) ? a.colors1 : a.colors0);
    uint16_t* __restrict__ Cs = reinterpret_cast<uint16_t*>((t & 1) ? a.colors0 : a.colors1);
    const uint32_t cnt = *a.wcount;
    const uint32_t NWW = (a.nCol + 31u) >> 5;
    for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x) {
        const uint32_t v = a.wlist[i];
        const uint32_t l = v - a.v_begin;
        for (uint32_t w = threadIdx.x; w < NWW; w += blockDim.x) mask[w] = 0;
        if (threadIdx.x == 0) sh_pop = 0;
        __syncthreads();
        // count_free_colors (:362-383): occupancy of N(v), 4 independent gathers per thread in flight
        const uint64_t rb = a.row_off[l], re = a.row_off[l + 1];
        for (uint64_t k = rb + threadIdx.x; k < re; k += 4u * blockDim.x) {
            uint32_t c[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint64_t kk = k + (uint64_t)j * blockDim.x;
                c[j] = kk < re ? (uint32_t)C[a.col_idx[kk]] : 0xFFFFFFFFu;
            }
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (c[j] != 0xFFFFFFFFu) atomicOr(&mask[c[j] >> 5], 1u << (c[j] & 31u));
        }
        __syncthreads();
        uint32_t pop = 0;
        for (uint32_t w = threadIdx.x; w < NWW; w += blockDim.x) pop += __popc(mask[w]);
        for (int off = 32; off >= 1; off >>= 1) pop += __shfl_xor(pop, off, 64);
        if ((threadIdx.x & 63) == 0 && pop) atomicAdd(&sh_pop, pop);
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t P = sh_pop, Zvcomp = a.nCol - P;
            const uint32_t cv = C[v];
            const uint32_t x = minstd_mulmod(x_t, minstd_pow_tab((uint64_t)v + 1));
            const float u = minstd_canonical(x);
            uint32_t nc;
            if (Zvcomp > 0) {   // case (ii)
                const float pf = (1.0f - a.eps * (float)P) / (float)Zvcomp;
                nc = walk_mask(mask, a.nCol, a.eps, pf, u);
            } else {            // case (i)
                nc = walk_own_tab(a.etab, a.nCol, cv, a.eps, a.hi, u);
            }
            const bool event = nc == a.nCol;
            Cs[v] = (uint16_t)(event ? cv : nc);
            if (a.taboo != nullptr && !event) a.taboo[l] = (nc == cv) ? a.tabooIteration : 0u;
            if (event) {
                const uint32_t idx = atomicAdd(&st->ev_count, 1u);
                if (idx < a.ev_cap) a.events[idx] = v;
                else atomicOr(&st->err, 1u);
            }
        }
        __syncthreads();
    }
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
