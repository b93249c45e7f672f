// mcmc_colorer_amd/csrc/multi.hip -- the native multi-GPU path: RCCL
// communicators owned behind the C ABI and a driver that runs the vertex-partitioned colorer to the
// end of the reference loop inside one call, with no Python in the data path.
//
// Per sweep t (every local rank, on its own stream):
//   mcmc_part_sweep_async   the rank's rows -> its rows of colors[(t+1)&1] + its footer slot
//   exchange                colours: P2P send/recv of every rank's row range to every peer (xGMI is a
//                           full mesh of point-to-point links: each range travels once per link, in
//                           parallel; arc-balanced ranges have unequal sizes) -- or, MCMC_EXCHANGE=
//                           allgather, one in-place ncclAllGather for equal-stride plans; footers:
//                           one in-place ncclAllGather of world x 4 KiB
//   mcmc_part_commit_async  global Cviol, stop test, the rank-ordered glibc replay on every replica
// Every check_every sweeps the host reads the device state: done, a fatal error, or a spill pause
// (some rank's overflow-event list outgrew its footer): then the full sorted lists are all-gathered
// (stride = the longest) and the paused sweep is committed from them (mcmc_part_spill_commit_async).
//
// Without communicators (comm == NULL for every context) the same sequence runs over a loopback
// transport: all `world` ranks live in this process (one device or several), the exchange is
// hipMemcpyAsync between their buffers with events ordering the streams. It is what the tests use
// to run 2..8 ranks on one GPU through exactly this driver.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mcmc_common.h"

struct mcmc_comm {
    ncclComm_t comm = nullptr;
    int device = 0;
    uint32_t world = 1, rank = 0;
};

namespace {

using namespace mcmc;

#define MCMC_NCCL_TRY(expr)                                                                         \
    do {                                                                                            \
        ncclResult_t _r = (expr);                                                                   \
        if (_r != ncclSuccess) return fail(MCMC_E_HIP, std::string(#expr ": ") + ncclGetErrorString(_r)); \
    } while (0)

constexpr uint32_t kFootBytes = 4u * MCMC_FOOTER_WORDS;

// Equal-stride plan (every inner bound r * S): the colours can travel by one in-place all-gather.
uint32_t equal_stride(const PartDesc& d) {
    if (d.world < 2) return 0;
    const uint32_t S = d.bounds[1];
    for (uint32_t r = 1; r < d.world; r++)
        if (d.bounds[r] != std::min<uint64_t>((uint64_t)S * r, d.n)) return 0;
    return S;
}

// MCMC_EXCHANGE = p2p (default) | allgather. xGMI is a full mesh of point-to-point links: every
// rank's range goes to each peer over its own link, all links at once (7 x n/8 bytes per rank at
// 8 GPUs); the ring all-gather (equal-stride plans only) moves the same bytes through 7 hops.
int exchange_mode() {
    const char* e = getenv("MCMC_EXCHANGE");
    return (e && !strcmp(e, "allgather")) ? 2 : 1;
}

struct Driver {
    std::vector<mcmc_ctx*> ctx;
    std::vector<PartDesc> d;
    std::vector<hipEvent_t> ev;   // loopback: per rank, its copies of the step are enqueued
    bool rccl = false;
    uint32_t world = 1;
    int mode = 0;

    ~Driver() {
        for (size_t i = 0; i < ev.size(); i++)
            if (ev[i]) { (void)hipSetDevice(d[i].device); (void)hipEventDestroy(ev[i]); }
    }

    int setup(mcmc_ctx** cs, uint32_t k) {
        ctx.assign(cs, cs + k);
        d.resize(k);
        for (uint32_t i = 0; i < k; i++)
            if (int rc = part_desc(ctx[i], &d[i])) return rc;
        world = d[0].world;
        rccl = d[0].comm != nullptr;
        for (uint32_t i = 0; i < k; i++) {
            if (d[i].world != world) return fail(MCMC_E_ARG, "contexts of different partitions");
            if ((d[i].comm != nullptr) != rccl) return fail(MCMC_E_ARG, "mixed RCCL and loopback contexts");
            if (rccl && (d[i].comm->world != world || d[i].comm->rank != d[i].rank || d[i].comm->device != d[i].device))
                return fail(MCMC_E_ARG, "communicator does not match the context's rank/device");
        }
        if (!rccl) {
            if (k != world) return fail(MCMC_E_ARG, "loopback transport: all ranks must be passed");
            for (uint32_t i = 0; i < k; i++)
                if (d[i].rank != i) return fail(MCMC_E_ARG, "loopback transport: contexts in rank order");
            ev.assign(k, nullptr);
            for (uint32_t i = 0; i < k; i++) {
                MCMC_HIP_TRY(hipSetDevice(d[i].device));
                MCMC_HIP_TRY(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
            }
        }
        mode = exchange_mode();
        return MCMC_OK;
    }

    int exchange(uint32_t t) {
        const uint32_t nb = (t + 1) & 1u;
        if (rccl) {
            const uint32_t S = equal_stride(d[0]);
            const bool ag = S != 0 && mode == 2;   // equal-stride ranges may take one in-place all-gather
            if (world > 1) {
                MCMC_NCCL_TRY(ncclGroupStart());
                for (auto& x : d) {
                    uint8_t* C = x.colors[nb];
                    ncclComm_t cm = x.comm->comm;
                    if (ag) {
                        MCMC_NCCL_TRY(ncclAllGather(C + (size_t)x.rank * S * x.cbytes, C, (size_t)S * x.cbytes, ncclUint8,
                                                    cm, x.stream));
                        continue;
                    }
                    const size_t b0 = x.bounds[x.rank], len = x.bounds[x.rank + 1] - b0;
                    for (uint32_t q = 0; q < world; q++) {
                        if (q == x.rank) continue;
                        MCMC_NCCL_TRY(ncclSend(C + b0 * x.cbytes, len * x.cbytes, ncclUint8, (int)q, cm, x.stream));
                        const size_t c0 = x.bounds[q], clen = x.bounds[q + 1] - c0;
                        MCMC_NCCL_TRY(ncclRecv(C + c0 * x.cbytes, clen * x.cbytes, ncclUint8, (int)q, cm, x.stream));
                    }
                }
                MCMC_NCCL_TRY(ncclGroupEnd());
            }
            // footers: one in-place all-gather (also at world 1, where it is the only collective)
            MCMC_NCCL_TRY(ncclGroupStart());
            for (auto& x : d)
                MCMC_NCCL_TRY(ncclAllGather(x.foot[nb] + (size_t)x.rank * MCMC_FOOTER_WORDS, x.foot[nb], MCMC_FOOTER_WORDS,
                                            ncclUint32, x.comm->comm, x.stream));
            MCMC_NCCL_TRY(ncclGroupEnd());
            return MCMC_OK;
        }
        // loopback: rank r copies its rows and footer slot into every peer's buffers on its own
        // stream; every peer's commit waits for all of them
        for (uint32_t r = 0; r < world; r++) {
            const PartDesc& x = d[r];
            MCMC_HIP_TRY(hipSetDevice(x.device));
            const size_t b0 = x.bounds[r], len = x.bounds[r + 1] - b0;
            for (uint32_t q = 0; q < world; q++) {
                if (q == r) continue;
                if (len)
                    MCMC_HIP_TRY(hipMemcpyAsync(d[q].colors[nb] + b0 * x.cbytes, x.colors[nb] + b0 * x.cbytes,
                                                len * x.cbytes, hipMemcpyDefault, x.stream));
                MCMC_HIP_TRY(hipMemcpyAsync(d[q].foot[nb] + (size_t)r * MCMC_FOOTER_WORDS,
                                            x.foot[nb] + (size_t)r * MCMC_FOOTER_WORDS, kFootBytes, hipMemcpyDefault,
                                            x.stream));
            }
            MCMC_HIP_TRY(hipEventRecord(ev[r], x.stream));
        }
        for (uint32_t q = 0; q < world; q++) {
            MCMC_HIP_TRY(hipSetDevice(d[q].device));
            for (uint32_t r = 0; r < world; r++)
                if (r != q) MCMC_HIP_TRY(hipStreamWaitEvent(d[q].stream, ev[r], 0));
        }
        return MCMC_OK;
    }

    // The paused sweep's full lists: all-gathered with stride = the longest, then committed.
    int spill() {
        std::vector<uint32_t> cnt(world, 0);
        if (int rc = mcmc_part_spill_counts(ctx[0], cnt.data())) return rc;
        const uint32_t stride = std::max<uint32_t>(1u, *std::max_element(cnt.begin(), cnt.end()));
        std::vector<uint32_t*> buf(d.size());
        for (size_t i = 0; i < d.size(); i++) {
            MCMC_HIP_TRY(hipSetDevice(d[i].device));
            if (int rc = part_spill_buffer(ctx[i], stride, &buf[i])) return rc;
        }
        if (rccl) {
            MCMC_NCCL_TRY(ncclGroupStart());
            for (size_t i = 0; i < d.size(); i++)
                MCMC_NCCL_TRY(ncclAllGather(d[i].events, buf[i], stride, ncclUint32, d[i].comm->comm, d[i].stream));
            MCMC_NCCL_TRY(ncclGroupEnd());
        } else {
            for (uint32_t r = 0; r < world; r++) {   // rare: plain synchronous copies
                MCMC_HIP_TRY(hipSetDevice(d[r].device));
                MCMC_HIP_TRY(hipStreamSynchronize(d[r].stream));
            }
            for (uint32_t q = 0; q < world; q++)
                for (uint32_t r = 0; r < world; r++)
                    if (cnt[r])
                        MCMC_HIP_TRY(hipMemcpy(buf[q] + (size_t)r * stride, d[r].events, sizeof(uint32_t) * cnt[r],
                                               hipMemcpyDefault));
        }
        for (size_t i = 0; i < d.size(); i++)
            if (int rc = mcmc_part_spill_commit_async(ctx[i], buf[i], stride)) return rc;
        return MCMC_OK;
    }
};

}  // namespace

extern "C" {

int mcmc_comm_unique_id(uint8_t id[MCMC_COMM_ID_BYTES]) {
    if (!id) return fail(MCMC_E_ARG, "NULL id");
    static_assert(sizeof(ncclUniqueId) == MCMC_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    MCMC_NCCL_TRY(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return MCMC_OK;
}

int mcmc_comm_init_rank(const uint8_t id[MCMC_COMM_ID_BYTES], uint32_t world, uint32_t rank, int device,
                        mcmc_comm** out) {
    if (!id || !out) return fail(MCMC_E_ARG, "NULL argument");
    if (world == 0 || rank >= world) return fail(MCMC_E_ARG, "bad world/rank");
    *out = nullptr;
    MCMC_HIP_TRY(hipSetDevice(device));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    auto* c = new mcmc_comm();
    c->device = device;
    c->world = world;
    c->rank = rank;
    ncclResult_t r = ncclCommInitRank(&c->comm, (int)world, u, (int)rank);
    if (r != ncclSuccess) {
        delete c;
        return fail(MCMC_E_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    *out = c;
    return MCMC_OK;
}

int mcmc_comm_init_all(const int* devices, uint32_t ndev, mcmc_comm** out) {
    if (!devices || !out || ndev == 0) return fail(MCMC_E_ARG, "bad argument");
    std::vector<ncclComm_t> cs(ndev);
    std::vector<int> dv(devices, devices + ndev);
    MCMC_NCCL_TRY(ncclCommInitAll(cs.data(), (int)ndev, dv.data()));
    for (uint32_t i = 0; i < ndev; i++) {
        out[i] = new mcmc_comm();
        out[i]->comm = cs[i];
        out[i]->device = devices[i];
        out[i]->world = ndev;
        out[i]->rank = i;
    }
    return MCMC_OK;
}

void mcmc_comm_destroy(mcmc_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    delete c;
}

int mcmc_part_create(const mcmc_graph* g, const mcmc_params* p, uint32_t world, uint32_t rank, const uint32_t* bounds,
                     mcmc_comm* comm, mcmc_ctx** out) {
    if (!g || !p || !bounds || !out) return fail(MCMC_E_ARG, "NULL argument");
    if (rank >= world) return fail(MCMC_E_ARG, "rank >= world");
    *out = nullptr;
    uint32_t n = 0;
    uint64_t m = 0;
    uint32_t mx = 0, mn = 0;
    if (int rc = mcmc_graph_info(g, &n, &m, &mx, &mn)) return rc;
    const int device = g->g.device;
    if (comm && (comm->device != device || comm->world != world || comm->rank != rank))
        return fail(MCMC_E_ARG, "communicator does not match the graph's device or the rank");
    mcmc_ctx* c = nullptr;
    if (int rc = mcmc_create(g, p, bounds[rank], bounds[rank + 1], &c)) return rc;
    const size_t cb = mcmc_color_bytes(p->nCol);
    // room for an in-place all-gather of equal-stride ranges (world * S colours) and 256 of slack
    const size_t S = world > 1 ? bounds[1] : n;
    const size_t cols = (std::max<size_t>((size_t)n + 256, (size_t)world * S + 256) * cb + 255) & ~(size_t)255;
    const size_t foot = (size_t)world * 4u * MCMC_FOOTER_WORDS;
    void* mem = nullptr;
    hipStream_t st = nullptr;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipMalloc(&mem, 2 * cols + 2 * foot);
    if (e == hipSuccess) e = hipMemset(mem, 0, 2 * cols + 2 * foot);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (e != hipSuccess) {
        (void)hipFree(mem);
        mcmc_destroy(c);
        return fail(MCMC_E_NOMEM, std::string("partitioned buffers: ") + hipGetErrorString(e));
    }
    uint8_t* b = static_cast<uint8_t*>(mem);
    int rc = mcmc_part_attach(c, world, rank, bounds, b, b + cols, cols, b + 2 * cols, b + 2 * cols + foot, st);
    if (!rc) rc = part_adopt(c, mem, st, comm);
    if (rc) {
        (void)hipFree(mem);
        (void)hipStreamDestroy(st);
        mcmc_destroy(c);
        return rc;
    }
    *out = c;
    return MCMC_OK;
}

int mcmc_part_run(mcmc_ctx** ctxs, uint32_t k, uint32_t max_sweeps, mcmc_run_stats* stats) {
    if (!ctxs || k == 0) return fail(MCMC_E_ARG, "no contexts");
    Driver D;
    if (int rc = D.setup(ctxs, k)) return rc;
    const uint32_t limit = max_sweeps ? max_sweeps : D.d[0].maxRip + 2;   // + the final count pass (sweeps)
    const uint32_t check_every = 8;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    MCMC_HIP_TRY(hipSetDevice(D.d[0].device));
    MCMC_HIP_TRY(hipEventCreate(&e0));
    MCMC_HIP_TRY(hipEventCreate(&e1));
    MCMC_HIP_TRY(hipEventRecord(e0, D.d[0].stream));
    // the loop continues from the device's sweep counter (a second call resumes where the first
    // stopped: the exchange's buffer parity is the device's)
    int32_t dn0 = 0;
    uint32_t t = 0, err0 = 0;
    int rc = mcmc_part_state(D.ctx[0], &dn0, &t, &err0);
    if (rc) return rc;
    if (err0 & 2u) return fail(MCMC_E_STATE, "a spill exchange is pending");
    const uint32_t t_begin = t;
    bool done = dn0 != 0;
    while (!rc && !done && t - t_begin < limit) {
        const uint32_t kk = std::min(check_every, limit - (t - t_begin));
        for (uint32_t s = 0; s < kk && !rc; s++, t++) {
            for (auto* c : D.ctx)
                if ((rc = mcmc_part_sweep_async(c))) break;
            if (!rc) rc = D.exchange(t);
            for (auto* c : D.ctx)
                if (!rc && (rc = mcmc_part_commit_async(c))) break;
        }
        if (rc) break;
        int32_t dn = 0;
        uint32_t td = 0, err = 0;
        if ((rc = mcmc_part_state(D.ctx[0], &dn, &td, &err))) break;
        if (err & 1u) { rc = fail(MCMC_E_DEVICE, "partitioned sweep: device error flag"); break; }
        if (err & 2u) {   // spill pause at sweep td: resume from it
            if ((rc = D.spill())) break;
            if ((rc = mcmc_part_state(D.ctx[0], &dn, &td, &err))) break;
            t = td;
        }
        done = dn != 0;
    }
    if (!rc) {
        MCMC_HIP_TRY(hipSetDevice(D.d[0].device));
        MCMC_HIP_TRY(hipEventRecord(e1, D.d[0].stream));
        MCMC_HIP_TRY(hipEventSynchronize(e1));
    }
    float ms = 0;
    if (!rc) (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc) return rc;
    for (uint32_t i = 0; i < k; i++) {
        mcmc_run_stats s{};
        if ((rc = part_stats(D.ctx[i], &s))) return rc;
        s.loopMs = ms;
        if (stats) stats[i] = s;
    }
    return MCMC_OK;
}

}  // extern "C"
