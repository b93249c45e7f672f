// mcmc_colorer_amd/csrc/mcmc_common.h -- shared host-side plumbing of libmcmc_hip.so:
// error reporting (the C ABI returns codes, never aborts) and the opaque handle layouts.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

#include "../../include/mcmc_hip.h"

namespace mcmc {

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define MCMC_HIP_TRY(expr)                                                                          \
    do {                                                                                            \
        hipError_t _e = (expr);                                                                     \
        if (_e != hipSuccess)                                                                       \
            return ::mcmc::fail(MCMC_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e) +     \
                                                " (" __FILE__ ":" + std::to_string(__LINE__) + ")"); \
    } while (0)

// Reference counterpart: GraphStruct<nodeW,edgeW> (graph/graph.h:37-79) with uint64 offsets.
struct GraphDev {
    int device = 0;
    uint32_t n = 0;
    uint64_t m = 0;
    uint32_t maxDeg = 0, minDeg = 0;
    bool sorted = false;           // every neighbour list ascending
    int sym = -1;                  // whole CSR symmetric: 1 yes, 0 no, -1 not checked (csr_symmetric)
    int simple_sym = -1;           // every arc's reverse present and no arc repeated: 1 yes (the counter-based
                                   // G(n, p) by construction, or checked), 0 no, -1 not known
    bool partial_rows = false;     // generated for a row range only: rows outside it hold no arcs
    uint64_t* row_off = nullptr;   // [n+1]
    uint32_t* col_idx = nullptr;   // [m]
};

// Sorts every neighbour list ascending on the device, in place (graph.hip).
int sort_rows_inplace(GraphDev& g);
// *sym = every arc (i, j) of rows [vb, vb + nloc) with j in that range has its reverse (one wave per
// row, binary search of row j; sorts the rows first). The whole-graph answer is cached in g.sym.
int csr_symmetric(GraphDev& g, uint32_t vb, uint32_t nloc, hipStream_t s, bool* sym);

}  // namespace mcmc

struct mcmc_graph;

namespace mcmc {
// Row stride of a tiled layout's segment table: R + 1 entries rounded up to 4, so every
// (group, block) table row is 16-byte aligned for LDS-DMA.
__host__ __device__ inline uint32_t tseg_stride(uint32_t R) { return (R + 4u) & ~3u; }
// A segment-table entry: padded start (multiple of 8) | padding count of the segment (low 3 bits).
constexpr uint32_t kTsegPos = ~7u;

// Tiled copy of a row range of the CSR (sweep variant 3, mcmc_sweep.hip): rows in groups of
// grp_rows, per group the arcs block-major as 16-bit block-local ids, every (row, block) segment
// padded to a multiple of 8 ids. Cached on the graph, so contexts re-created per repetition reuse it.
struct TiledLayout {
    uint32_t v_begin = 0, v_end = 0, grp_rows = 0, block_log2 = 0, nblocks = 0, ngroups = 0;
    uint64_t ids = 0;              // padded length of tcol
    uint64_t arcs = 0;             // arcs of the rows (unpadded)
    uint16_t* tcol = nullptr;
    uint64_t* gbase = nullptr;     // [ngroups + 1]
    uint32_t* tseg = nullptr;      // [ngroups][nblocks][tseg_stride(grp_rows)] (entries 0..grp_rows used)
    ~TiledLayout();
};
}  // namespace mcmc

namespace mcmc {
// Builds (or finds in the graph's cache) the tiled layout of rows [v_begin, v_end) (tiled_layout.hip).
int get_tiled_layout(mcmc_graph* gh, uint32_t v_begin, uint32_t v_end, uint32_t R, uint32_t block_log2,
                     hipStream_t s, const TiledLayout** out);
// Default rows per group of a tiled layout on nloc rows (mcmc_create and the generator agree).
uint32_t tiled_default_rows(uint32_t nloc, uint32_t cus, uint32_t rmax);
constexpr uint32_t kTileRowsMax = 8191;      // tiled groups: dlist/claims are 16-bit row indices
constexpr uint32_t kTileGenRowsMax = 1792;   // generator layouts: fits the streaming LDS for nCol <= 64
// CSR (ascending rows) of a generated graph with a full-range layout.
int tiled_to_csr(const mcmc_graph* gh, uint64_t* row_off, uint32_t* col_idx);
}  // namespace mcmc

namespace mcmc {
// Row access for the tail cut (tailcut.hip): the CSR when the graph has one, else the tiled layout.
struct TailView {
    uint32_t n = 0;                // rows (a partitioned context: its local rows)
    uint32_t vb = 0;               // vertex of local row 0 (the replica's index of row l is vb + l)
    uint32_t csr_row0 = 0;         // CSR row of local row 0 (row_off is the whole graph's; tiled: local)
    const uint64_t* row_off = nullptr;
    const uint32_t* col_idx = nullptr;
    const uint16_t* tcol = nullptr;
    const uint64_t* gbase = nullptr;
    const uint32_t* tseg = nullptr;
    uint32_t R = 0, nb = 0, block_log2 = 0;
};
// flags[v] = colour of v used by a neighbour (violation_count, coloringMCMC_CPU.cpp:329-350); *count = sum.
// edges: the reference GPU colorer's conflictCounter (same-colour neighbours with a larger id, counted).
// C: the replica, cbytes = 1 (uint8) or 2 (uint16, the wide sweep).
int tail_count(const TailView& g, const void* C, uint32_t cbytes, uint8_t* flags, unsigned long long* count,
               hipStream_t s, bool edges);
// Ascending list of the flagged vertices; *list_len on the device. tmp: scratch, grown on demand.
int tail_select(const uint8_t* flags, uint32_t n, uint32_t* list, uint32_t* list_len, void** tmp, size_t* tmp_bytes,
                hipStream_t s);
// One corrected tail-cut pass (coloringMCMC_CPU.cpp:281-305, k++) over the listed vertices, in order.
// ref: the GPU colorer's tailCutting rule over at most `limit` listed vertices.
int tail_repair(const TailView& g, void* C, uint32_t cbytes, const uint32_t* list, const uint32_t* list_len,
                const uint32_t* colorIdx, uint32_t nCol, hipStream_t s, bool ref, unsigned long long limit);
}  // namespace mcmc

namespace mcmc {
constexpr uint32_t kXSlabs = 8;   // L2 mode: column slabs of the wide sweep's edge layout, one per XCD
// Slab edge layout of a row range for the wide sweep (sweep_wide.h, get_xslab): slab s holds the
// kept arcs whose column lies in [s S, (s+1) S), row-sorted, as 256-entry chunks of 32-bit entries
// (row delta from the chunk's base row << cbits | slab-local column), padded with 0xFFFFFFFF.
//   mode 0 (L2): 8 slabs, one per XCD, colours gathered through that XCD's L2;
//   mode 1 (LDS): slabs of 2^17 vertices whose colour fingerprints a workgroup stages in LDS, each
//                 slab's chunks cut into pieces, pieces assigned to workgroups on the host.
struct XSlabLayout {
    uint32_t v_begin = 0, v_end = 0;
    uint32_t mode = 0;
    uint32_t S = 0, cbits = 0;
    uint32_t sym = 0;                  // 1: one entry per local edge (symmetric CSR); 0: every arc
    uint32_t simple = 0;               // sym and no row lists a neighbour twice (incremental counts apply)
    uint32_t nslabs = 0, chunks = 0;
    std::vector<uint32_t> chunk0_h;    // first chunk of every slab (nslabs + 1)
    uint64_t entries = 0;              // kept arcs (unpadded)
    uint32_t* ent = nullptr;           // [chunks * 256]; nullptr: the layout does not apply
    uint32_t* base = nullptr;          // [chunks]
    uint32_t* chunk0 = nullptr;        // device copy of chunk0_h
    uint32_t nwg = 0, npieces = 0;     // LDS mode: workgroups, pieces
    uint32_t* pieces = nullptr;        // [npieces][3] {slab, first chunk, end chunk}, grouped by workgroup
    uint32_t* wg_piece = nullptr;      // [nwg + 1] first piece of every workgroup
    ~XSlabLayout();
};
}  // namespace mcmc

struct mcmc_ctx;
struct mcmc_comm;

namespace mcmc {
// A partitioned context's exchange buffers (mcmc_sweep.hip; used by the native driver, multi.hip).
struct PartDesc {
    uint8_t* colors[2];          // colour replicas (vertex order), C_t in colors[t & 1]
    uint32_t* foot[2];           // footer buffers, world x MCMC_FOOTER_WORDS; sweep t writes foot[(t+1) & 1]
    const uint32_t* bounds;      // [world + 1]
    uint32_t world, rank, cbytes, n;
    hipStream_t stream;
    int device;
    mcmc_comm* comm;             // nullptr: exchanged by the caller / the loopback transport
    uint32_t* events;            // the rank's sorted list of a paused (spill) sweep
    uint32_t maxRip;
    uint32_t* dlt[2];            // delta slots (world x kDeltaWords words), sweep t's at dlt[(t+1) & 1]
    bool delta_ok;               // the context can run delta-mode steps (tiled sweep with delta slots)
    uint32_t tailcut_max;        // mcmc_set_tailcut_repair pass cap (0: off)
};
constexpr uint32_t kPartDeltaWords = 4096;   // = kDeltaWords (mcmc_sweep.hip): one rank's delta slot
int part_desc(mcmc_ctx* c, PartDesc* d);
// Hands a native partitioned context its buffers (one allocation, freed by mcmc_destroy), its own
// stream (destroyed there too) and its communicator (borrowed).
int part_adopt(mcmc_ctx* c, void* mem, hipStream_t own_stream, mcmc_comm* comm);
// Device buffer of world x stride words for a spill exchange (grown on demand, owned by the context).
int part_spill_buffer(mcmc_ctx* c, uint32_t stride, uint32_t** buf);
// Refreshes and returns the context's run summary (mcmc_part_state + the stats of mcmc_run).
int part_stats(mcmc_ctx* c, mcmc_run_stats* s);
// Delta exchange (native driver): the context's delta slot buffers (world x kPartDeltaWords words
// each, owned by the caller's allocation); whether delta-mode steps are possible; a step's sweep
// (delta: append changed vertices), its commit (mode 1 delta, 0 full, -1 full-mode resumption of
// a paused sweep; spill: the gathered full event lists or nullptr), and the remote-range sync that
// precedes delta mode after full-mode steps.
int part_set_delta(mcmc_ctx* c, uint32_t* d0, uint32_t* d1);
bool part_delta_ok(const mcmc_ctx* c);
const void* part_state_ptr(const mcmc_ctx* c);   // device state: {t, done, x_t, err} in its first 16 bytes
int part_sweep(mcmc_ctx* c, bool delta);
// A world-1 partition's `steps` full-mode steps as one cached hipGraph launch (the one-GPU fused
// step each); returns 1 (nothing launched) when the context is not such a partition.
int part_solo_batch(mcmc_ctx* c, uint32_t steps);
int part_commit(mcmc_ctx* c, int mode, const uint32_t* spill, uint32_t stride);
int part_sync_remote(mcmc_ctx* c);
// Per-context driver resources, created on first use and kept until mcmc_destroy (a run then pays no
// stream / pinned-memory / event creation): a side stream, 16 pinned bytes, and events (0: the
// loopback transport's, 1-2: loop start/end, 3-4: batch ends).
struct PartRes {
    hipStream_t poll = nullptr;
    uint32_t* pinned = nullptr;
    hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
};
int part_resources(mcmc_ctx* c, PartRes** out);
int part_run_begin(mcmc_ctx* c);   // a run's start: this rank's delta slots empty, no tail-cut result, stats zero
void part_add_xstats(mcmc_ctx* c, int64_t delta_steps, int64_t full_steps, int64_t ovf, int64_t bytes);
// Partitioned tail cut (mcmc_sweep.hip): state and colorIdx at loop exit (global Cviol, the final t,
// the final colouring's buffer); one rank's repair of its flagged rows; its recount (device sum
// word); the result for the run summary.
int part_tail_init(mcmc_ctx* c, uint64_t* cviol, uint32_t* t_final, uint8_t** colors);
int part_tail_repair(mcmc_ctx* c, uint8_t* C, uint32_t t_final, bool first);
int part_tail_count(mcmc_ctx* c, const uint8_t* C, unsigned long long** count);
void part_tail_done(mcmc_ctx* c, uint64_t cviol, uint32_t passes);
}  // namespace mcmc

struct mcmc_graph {
    mcmc::GraphDev g;
    std::vector<std::unique_ptr<mcmc::TiledLayout>> tiles;   // freed with the graph
    std::vector<std::unique_ptr<mcmc::XSlabLayout>> xslabs;
};

// Per-vertex cuRAND XORWOW states of the reference-GPU-semantics mode (refmode.hip).
struct mcmc_gpurand {
    int device = 0;
    uint32_t n = 0;
    uint32_t seed = 0;
    uint32_t* states[2] = {nullptr, nullptr};   // SoA {v0..v4, d} x n words, double-buffered
    uint32_t cur = 0;                            // parity holding the current states
};
