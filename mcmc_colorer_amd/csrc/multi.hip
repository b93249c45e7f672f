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

// MCMC_EXCHANGE = delta (default) | p2p | allgather.
//   delta: a step sends only this rank's changed vertices (its delta slot, 16 KiB) and footer to
//          every peer; a slot that overflows pauses that sweep, which is then exchanged in full,
//          and the next kFullAfterOverflow steps run in full mode before delta mode resumes;
//   p2p:   every step sends this rank's whole row range to every peer (xGMI is a full mesh of
//          point-to-point links: each range rides its own link, all links at once);
//   allgather: equal-stride plans only, one in-place all-gather of the replica per step.
int exchange_mode() {
    const char* e = getenv("MCMC_EXCHANGE");
    if (e && !strcmp(e, "allgather")) return 2;
    if (e && !strcmp(e, "p2p")) return 1;
    return 0;
}
constexpr uint32_t kFullAfterOverflow = 16;
constexpr uint32_t kStepsPerPoll = 8;   // steps enqueued per batch; the host polls one batch behind
constexpr uint32_t kSoloStepsPerPoll = 64;   // world 1: one persistent launch per batch

struct Driver {
    std::vector<mcmc_ctx*> ctx;
    std::vector<PartDesc> d;
    std::vector<hipEvent_t> ev;   // loopback: per rank, its copies of the step are enqueued
    bool rccl = false;
    bool stub = false;            // mcmc_part_bench_rank: one rank's steps with the exchange left out
    uint32_t world = 1;
    int mode = 0;
    bool delta_ok = false;        // every local context can run delta-mode steps
    bool synced = false;          // delta invariant: both replicas hold the current colouring off the local rows
    PartRes* res0 = nullptr;      // ctx[0]'s resources: side stream reading the device state while steps
                                  // run, pinned copy of the state's first words {t, done, x_t, err}, events
    hipStream_t poll = nullptr;
    uint32_t* pinned = nullptr;

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
        if (stub) {
            if (k != 1 || rccl) return fail(MCMC_E_ARG, "rank bench: one loopback context");
        } else if (!rccl) {
            if (k != world) return fail(MCMC_E_ARG, "loopback transport: all ranks must be passed");
            for (uint32_t i = 0; i < k; i++)
                if (d[i].rank != i) return fail(MCMC_E_ARG, "loopback transport: contexts in rank order");
            ev.assign(k, nullptr);
            for (uint32_t i = 0; i < k; i++) {
                PartRes* r = nullptr;
                if (int rc = part_resources(ctx[i], &r)) return rc;
                ev[i] = r->ev[0];
            }
        }
        mode = exchange_mode();
        // delta mode needs the same decision on every rank: it depends only on the sweep kind
        // (uint8 tiled sweep), which every rank of a partition shares
        delta_ok = mode == 0 && world > 1;
        for (auto& x : d) delta_ok = delta_ok && x.delta_ok;
        if (int rc = part_resources(ctx[0], &res0)) return rc;
        poll = res0->poll;
        pinned = res0->pinned;
        for (auto* c : ctx)
            if (int rc = part_run_begin(c)) return rc;
        return MCMC_OK;
    }

    // Step t's exchange. delta: footers + delta slots; else footers + the row ranges.
    int exchange(uint32_t t, bool delta) {
        if (stub) return MCMC_OK;   // peers' footers and slots stay empty: no Cviol, events or changes
        const uint32_t nb = (t + 1) & 1u;
        if (rccl) {
            if (world == 1) return MCMC_OK;   // nothing leaves the rank
            const uint32_t S = equal_stride(d[0]);
            if (!delta && S != 0 && mode == 2) {   // equal-stride ranges: two in-place all-gathers
                MCMC_NCCL_TRY(ncclGroupStart());
                for (auto& x : d) {
                    uint8_t* C = x.colors[nb];
                    MCMC_NCCL_TRY(ncclAllGather(C + (size_t)x.rank * S * x.cbytes, C, (size_t)S * x.cbytes, ncclUint8,
                                                x.comm->comm, x.stream));
                    MCMC_NCCL_TRY(ncclAllGather(x.foot[nb] + (size_t)x.rank * MCMC_FOOTER_WORDS, x.foot[nb],
                                                MCMC_FOOTER_WORDS, ncclUint32, x.comm->comm, x.stream));
                }
                MCMC_NCCL_TRY(ncclGroupEnd());
                return MCMC_OK;
            }
            // one group of point-to-point transfers: to every peer this rank's footer slot and
            // either its delta slot or its row range; from every peer the same
            MCMC_NCCL_TRY(ncclGroupStart());
            for (auto& x : d) {
                ncclComm_t cm = x.comm->comm;
                const size_t b0 = x.bounds[x.rank], len = x.bounds[x.rank + 1] - b0;
                for (uint32_t q = 0; q < world; q++) {
                    if (q == x.rank) continue;
                    MCMC_NCCL_TRY(ncclSend(x.foot[nb] + (size_t)x.rank * MCMC_FOOTER_WORDS, MCMC_FOOTER_WORDS, ncclUint32,
                                           (int)q, cm, x.stream));
                    MCMC_NCCL_TRY(ncclRecv(x.foot[nb] + (size_t)q * MCMC_FOOTER_WORDS, MCMC_FOOTER_WORDS, ncclUint32,
                                           (int)q, cm, x.stream));
                    if (delta) {
                        MCMC_NCCL_TRY(ncclSend(x.dlt[nb] + (size_t)x.rank * kPartDeltaWords, kPartDeltaWords, ncclUint32,
                                               (int)q, cm, x.stream));
                        MCMC_NCCL_TRY(ncclRecv(x.dlt[nb] + (size_t)q * kPartDeltaWords, kPartDeltaWords, ncclUint32,
                                               (int)q, cm, x.stream));
                    } else {
                        uint8_t* C = x.colors[nb];
                        MCMC_NCCL_TRY(ncclSend(C + b0 * x.cbytes, len * x.cbytes, ncclUint8, (int)q, cm, x.stream));
                        const size_t c0 = x.bounds[q], clen = x.bounds[q + 1] - c0;
                        MCMC_NCCL_TRY(ncclRecv(C + c0 * x.cbytes, clen * x.cbytes, ncclUint8, (int)q, cm, x.stream));
                    }
                }
            }
            MCMC_NCCL_TRY(ncclGroupEnd());
            return MCMC_OK;
        }
        // loopback: rank r copies its footer slot and its delta slot or rows into every peer's
        // buffers on its own stream; every peer's commit waits for all of them
        for (uint32_t r = 0; r < world; r++) {
            const PartDesc& x = d[r];
            MCMC_HIP_TRY(hipSetDevice(x.device));
            const size_t b0 = x.bounds[r], len = x.bounds[r + 1] - b0;
            for (uint32_t q = 0; q < world; q++) {
                if (q == r) continue;
                if (delta) {
                    MCMC_HIP_TRY(hipMemcpyAsync(d[q].dlt[nb] + (size_t)r * kPartDeltaWords,
                                                x.dlt[nb] + (size_t)r * kPartDeltaWords, 4u * kPartDeltaWords,
                                                hipMemcpyDefault, x.stream));
                } else if (len) {
                    MCMC_HIP_TRY(hipMemcpyAsync(d[q].colors[nb] + b0 * x.cbytes, x.colors[nb] + b0 * x.cbytes,
                                                len * x.cbytes, hipMemcpyDefault, x.stream));
                }
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

    // bytes this rank sends per step in each mode (to world - 1 peers)
    uint64_t step_bytes(const PartDesc& x, bool delta) const {
        if (world < 2) return 0;
        const uint64_t rows = (uint64_t)x.bounds[x.rank + 1] - x.bounds[x.rank];
        const uint64_t per = 4ull * MCMC_FOOTER_WORDS + (delta ? 4ull * kPartDeltaWords : rows * x.cbytes);
        return per * (world - 1);
    }

    // One step: sweep (every local rank) -> exchange -> commit. A delta-mode step after full-mode
    // ones first makes both replicas equal off the local rows (part_sync_remote).
    int step(uint32_t t, bool delta) {
        for (size_t i = 0; i < d.size(); i++) part_add_xstats(ctx[i], delta ? 1 : 0, delta ? 0 : 1, 0, step_bytes(d[i], delta));
        if (delta && !synced) {
            for (auto* c : ctx)
                if (int rc = part_sync_remote(c)) return rc;
        }
        synced = delta;
        for (auto* c : ctx)
            if (int rc = part_sweep(c, delta)) return rc;
        if (int rc = exchange(t, delta)) return rc;
        for (auto* c : ctx)
            if (int rc = part_commit(c, delta ? 1 : 0, nullptr, 0u)) return rc;
        return MCMC_OK;
    }

    // The paused sweep's full lists: all-gathered with stride = the longest (rank order).
    int spill_gather(std::vector<uint32_t*>& buf, uint32_t* stride_out) {
        std::vector<uint32_t> cnt(world, 0);
        if (int rc = mcmc_part_spill_counts(ctx[0], cnt.data())) return rc;
        const uint32_t stride = std::max<uint32_t>(1u, *std::max_element(cnt.begin(), cnt.end()));
        buf.assign(d.size(), nullptr);
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
            for (uint32_t q = 0; q < world; q++)
                for (uint32_t r = 0; r < world; r++)
                    if (cnt[r])
                        MCMC_HIP_TRY(hipMemcpy(buf[q] + (size_t)r * stride, d[r].events, sizeof(uint32_t) * cnt[r],
                                               hipMemcpyDefault));
        }
        *stride_out = stride;
        return MCMC_OK;
    }

    int drain() {
        for (auto& x : d) {
            MCMC_HIP_TRY(hipSetDevice(x.device));
            MCMC_HIP_TRY(hipStreamSynchronize(x.stream));
        }
        return MCMC_OK;
    }

    // A sweep paused at td (err bits 2 spill, 4 delta overflow; the queue drained): the full event
    // lists and/or the sweep's row ranges, then its commit. delta_step: td ran in delta mode.
    int resume(uint32_t td, uint32_t err, bool delta_step) {
        std::vector<uint32_t*> buf;
        uint32_t stride = 0;
        if ((err & 2u) && (rc_ = spill_gather(buf, &stride))) return rc_;
        const bool full = (err & 4u) != 0;   // a delta slot overflowed: the rows travel in full
        if (full && (rc_ = exchange(td, false))) return rc_;
        if (full)
            for (size_t i = 0; i < d.size(); i++) part_add_xstats(ctx[i], 0, 0, 1, step_bytes(d[i], false));
        for (size_t i = 0; i < d.size(); i++) {
            const int m = full ? -1 : (delta_step ? 1 : 0);
            if (buf.empty() && m >= 0) return fail(MCMC_E_STATE, "nothing to resume");
            if ((rc_ = part_commit(ctx[i], m, buf.empty() ? nullptr : buf[i], stride))) return rc_;
        }
        synced = delta_step && !full;
        return MCMC_OK;
    }

    // ctx[0]'s {t, done, err} read on the side stream once `e` (end of a batch) has passed; the
    // steps enqueued after it keep the GPU busy meanwhile.
    int peek(hipEvent_t e, uint32_t* t, uint32_t* done, uint32_t* err) {
        MCMC_HIP_TRY(hipSetDevice(d[0].device));
        MCMC_HIP_TRY(hipStreamWaitEvent(poll, e, 0));
        MCMC_HIP_TRY(hipMemcpyAsync(pinned, part_state_ptr(ctx[0]), 16, hipMemcpyDeviceToHost, poll));
        MCMC_HIP_TRY(hipStreamSynchronize(poll));
        *t = pinned[0];
        *done = pinned[1];
        *err = pinned[3];
        return MCMC_OK;
    }

    // The corrected tail cut after the loop, rank by rank in ascending order (part_tail_*).
    int tailcut() {
        std::vector<uint64_t> cv(d.size());
        std::vector<uint32_t> tf(d.size());
        std::vector<uint8_t*> C(d.size());
        for (size_t i = 0; i < d.size(); i++)
            if ((rc_ = part_tail_init(ctx[i], &cv[i], &tf[i], &C[i]))) return rc_;
        uint64_t cviol = cv[0];
        uint32_t passes = 0;
        const uint32_t cap = d[0].tailcut_max;
        unsigned long long* hsum = reinterpret_cast<unsigned long long*>(pinned);
        while (cviol > 0 && passes < cap) {
            for (uint32_t r = 0; r < world; r++) {
                for (size_t i = 0; i < d.size(); i++)
                    if (d[i].rank == r && (rc_ = part_tail_repair(ctx[i], C[i], tf[i], passes == 0))) return rc_;
                // rank r's rows as repaired: to every other rank before the next rank's turn
                const size_t b0 = d[0].bounds[r], len = d[0].bounds[r + 1] - b0;
                if (world == 1 || len == 0) continue;
                if (rccl) {
                    MCMC_NCCL_TRY(ncclGroupStart());
                    for (size_t i = 0; i < d.size(); i++)
                        MCMC_NCCL_TRY(ncclBroadcast(C[i] + b0 * d[i].cbytes, C[i] + b0 * d[i].cbytes, len * d[i].cbytes,
                                                    ncclUint8, (int)r, d[i].comm->comm, d[i].stream));
                    MCMC_NCCL_TRY(ncclGroupEnd());
                } else {
                    if ((rc_ = drain())) return rc_;
                    for (uint32_t q = 0; q < world; q++)
                        if (q != r)
                            MCMC_HIP_TRY(hipMemcpy(C[q] + b0 * d[q].cbytes, C[r] + b0 * d[r].cbytes, len * d[r].cbytes,
                                                   hipMemcpyDefault));
                }
            }
            // recount (:308): every rank its rows, summed over the ranks
            uint64_t tot = 0;
            std::vector<unsigned long long*> cnt(d.size());
            for (size_t i = 0; i < d.size(); i++)
                if ((rc_ = part_tail_count(ctx[i], C[i], &cnt[i]))) return rc_;
            if (rccl) {
                if (world > 1) {
                    MCMC_NCCL_TRY(ncclGroupStart());
                    for (size_t i = 0; i < d.size(); i++)
                        MCMC_NCCL_TRY(ncclAllReduce(cnt[i], cnt[i], 1, ncclUint64, ncclSum, d[i].comm->comm, d[i].stream));
                    MCMC_NCCL_TRY(ncclGroupEnd());
                }
                MCMC_HIP_TRY(hipSetDevice(d[0].device));
                MCMC_HIP_TRY(hipMemcpyAsync(hsum, cnt[0], sizeof(unsigned long long), hipMemcpyDeviceToHost, d[0].stream));
                MCMC_HIP_TRY(hipStreamSynchronize(d[0].stream));
                tot = *hsum;
            } else {
                for (size_t i = 0; i < d.size(); i++) {
                    MCMC_HIP_TRY(hipSetDevice(d[i].device));
                    MCMC_HIP_TRY(hipMemcpyAsync(hsum, cnt[i], sizeof(unsigned long long), hipMemcpyDeviceToHost, d[i].stream));
                    MCMC_HIP_TRY(hipStreamSynchronize(d[i].stream));
                    tot += *hsum;
                }
            }
            cviol = tot;
            passes++;
        }
        for (auto* c : ctx) part_tail_done(c, cviol, passes);
        return MCMC_OK;
    }

    int rc_ = MCMC_OK;
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
    const size_t dlt = (size_t)world * 4u * kPartDeltaWords;   // delta slots (delta-mode exchange)
    void* mem = nullptr;
    hipStream_t st = nullptr;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipMalloc(&mem, 2 * cols + 2 * foot + 2 * dlt);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    // zeroed on the partition's own stream: a null-stream hipMemset does not order against a
    // non-blocking stream, and could land after mcmc_init_coloring wrote C_0 into these buffers
    if (e == hipSuccess) e = hipMemsetAsync(mem, 0, 2 * cols + 2 * foot + 2 * dlt, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        (void)hipFree(mem);
        mcmc_destroy(c);
        return fail(MCMC_E_NOMEM, std::string("partitioned buffers: ") + hipGetErrorString(e));
    }
    uint8_t* b = static_cast<uint8_t*>(mem);
    int rc = mcmc_part_attach(c, world, rank, bounds, b, b + cols, cols, b + 2 * cols, b + 2 * cols + foot, st);
    if (!rc) rc = part_adopt(c, mem, st, comm);
    if (!rc)
        rc = part_set_delta(c, reinterpret_cast<uint32_t*>(b + 2 * cols + 2 * foot),
                            reinterpret_cast<uint32_t*>(b + 2 * cols + 2 * foot + dlt));
    if (rc) {
        (void)hipFree(mem);
        (void)hipStreamDestroy(st);
        mcmc_destroy(c);
        return rc;
    }
    *out = c;
    return MCMC_OK;
}

}  // extern "C"

namespace {
int part_run_impl(mcmc_ctx** ctxs, uint32_t k, uint32_t max_sweeps, mcmc_run_stats* stats, bool stub) {
    if (!ctxs || k == 0) return fail(MCMC_E_ARG, "no contexts");
    Driver D;
    D.stub = stub;
    if (int rc = D.setup(ctxs, k)) return rc;
    const uint32_t limit = max_sweeps ? max_sweeps : D.d[0].maxRip + 2;   // + the final count pass (sweeps)
    struct Ev { hipEvent_t e; };   // the context's cached events (part_resources)
    Ev e0{D.res0->ev[1]}, e1{D.res0->ev[2]};
    Ev batch_ev[2] = {{D.res0->ev[3]}, {D.res0->ev[4]}};
    MCMC_HIP_TRY(hipSetDevice(D.d[0].device));
    // the loop continues from the device's sweep counter (a second call resumes where the first
    // stopped: the exchange's buffer parity is the device's)
    int32_t dn0 = 0;
    uint32_t t = 0, err0 = 0;
    if (int rc = mcmc_part_state(D.ctx[0], &dn0, &t, &err0)) return rc;
    if (err0 & 6u) return fail(MCMC_E_STATE, "an exchange of a paused sweep is pending");
    MCMC_HIP_TRY(hipSetDevice(D.d[0].device));
    MCMC_HIP_TRY(hipEventRecord(e0.e, D.d[0].stream));   // (after the state read: the loop's device time)
    const uint32_t t_begin = t;
    // host-side exchange policy, identical on every rank (it sees the same device decisions)
    uint32_t full_left = 0;                // steps to run in full mode after a delta overflow
    std::vector<uint8_t> was_delta;        // mode of every enqueued step (index t - t_begin)
    auto enqueue = [&](uint32_t steps) -> int {
        if (D.d.size() == 1 && D.world == 1 && !D.stub && !(D.delta_ok && full_left == 0)) {
            // world 1 in full mode: the steps are the one-GPU fused step, one cached graph per batch
            const int rc = part_solo_batch(D.ctx[0], steps);
            if (rc == MCMC_OK) {
                for (uint32_t s = 0; s < steps; s++, t++) {
                    if (full_left) full_left--;
                    was_delta.push_back(0);
                    part_add_xstats(D.ctx[0], 0, 1, 0, 0);
                }
                D.synced = false;
                return MCMC_OK;
            }
            if (rc != 1) return rc;
        }
        for (uint32_t s = 0; s < steps; s++, t++) {
            const bool delta = D.delta_ok && full_left == 0;
            if (full_left) full_left--;
            was_delta.push_back(delta ? 1 : 0);
            if (int rc = D.step(t, delta)) return rc;
        }
        return MCMC_OK;
    };
    // Batches of kStepsPerPoll steps; after enqueuing batch j + 1 the host waits for batch j's end
    // and reads ctx[0]'s state on a side stream, so the device never idles for the host's poll.
    bool done = dn0 != 0;
    uint32_t inflight = 0;                 // batches enqueued and not yet polled (0..2)
    uint32_t cur = 0;                      // batch_ev slot of the oldest unpolled batch
    while (!done) {
        const uint32_t left = limit - std::min(limit, t - t_begin);
        if (left && inflight < 2) {
            const bool solo1 = D.d.size() == 1 && D.world == 1 && !D.stub;
            if (int rc = enqueue(std::min(solo1 ? kSoloStepsPerPoll : kStepsPerPoll, left))) return rc;
            MCMC_HIP_TRY(hipSetDevice(D.d[0].device));
            MCMC_HIP_TRY(hipEventRecord(batch_ev[(cur + inflight) & 1].e, D.d[0].stream));
            inflight++;
            if (inflight < 2 && t - t_begin < limit) continue;   // keep one batch queued ahead
        }
        if (!inflight) break;   // the step limit is reached and every batch was polled
        uint32_t td = 0, dn = 0, err = 0;
        if (int rc = D.peek(batch_ev[cur].e, &td, &dn, &err)) return rc;
        cur ^= 1u;
        inflight--;
        if (err & 1u) return fail(MCMC_E_DEVICE, "partitioned sweep: device error flag");
        if (err & 6u) {   // paused at sweep td: drain the no-op steps behind it, exchange, resume
            if (int rc = D.drain()) return rc;
            int32_t dn2 = 0;
            uint32_t err2 = 0;
            if (int rc = mcmc_part_state(D.ctx[0], &dn2, &td, &err2)) return rc;
            // the steps enqueued behind the paused sweep were no-ops on the device: uncount them
            for (uint32_t s = td + 1; s < t; s++) {
                const bool dl = s - t_begin < was_delta.size() && was_delta[s - t_begin];
                for (size_t i = 0; i < D.d.size(); i++)
                    part_add_xstats(D.ctx[i], dl ? -1 : 0, dl ? 0 : -1, 0, -(int64_t)D.step_bytes(D.d[i], dl));
            }
            if (int rc = D.resume(td, err2, td - t_begin < was_delta.size() && was_delta[td - t_begin])) return rc;
            if (err2 & 4u) full_left = kFullAfterOverflow;
            t = td + 1;
            was_delta.resize(t - t_begin);
            inflight = 0;
            cur = 0;
            continue;
        }
        done = dn != 0;
    }
    if (int rc = D.drain()) return rc;
    int32_t dnf = 0;
    uint32_t tf = 0, errf = 0;
    if (int rc = mcmc_part_state(D.ctx[0], &dnf, &tf, &errf)) return rc;
    if (errf & 1u) return fail(MCMC_E_DEVICE, "partitioned sweep: device error flag");
    if (dnf && D.d[0].tailcut_max) {
        if (int rc = D.tailcut()) return rc;
    }
    MCMC_HIP_TRY(hipSetDevice(D.d[0].device));
    MCMC_HIP_TRY(hipEventRecord(e1.e, D.d[0].stream));
    MCMC_HIP_TRY(hipEventSynchronize(e1.e));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0.e, e1.e);
    for (uint32_t i = 0; i < k; i++) {
        mcmc_run_stats s{};
        if (int rc = part_stats(D.ctx[i], &s)) return rc;
        s.loopMs = ms;
        if (stats) stats[i] = s;
    }
    return MCMC_OK;
}
}  // namespace

extern "C" {

int mcmc_part_run(mcmc_ctx** ctxs, uint32_t k, uint32_t max_sweeps, mcmc_run_stats* stats) {
    return part_run_impl(ctxs, k, max_sweeps, stats, false);
}

int mcmc_part_bench_rank(mcmc_ctx* c, uint32_t steps, mcmc_run_stats* stats) {
    if (!c || steps == 0) return fail(MCMC_E_ARG, "a context and steps > 0");
    return part_run_impl(&c, 1, steps, stats, true);
}

}  // extern "C"
