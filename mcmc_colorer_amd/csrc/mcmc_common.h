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
    uint64_t* row_off = nullptr;   // [n+1]
    uint32_t* col_idx = nullptr;   // [m]
};

// Sorts every neighbour list ascending on the device, in place (graph.hip).
int sort_rows_inplace(GraphDev& g);

}  // namespace mcmc

namespace mcmc {
// Tiled copy of a row range of the CSR (sweep variant 3, mcmc_sweep.hip): rows in groups of
// grp_rows, per group the arcs block-major as 16-bit block-local ids, every (row, block) segment
// padded to a multiple of 8 ids. Cached on the graph, so contexts re-created per repetition reuse it.
struct TiledLayout {
    uint32_t v_begin = 0, v_end = 0, grp_rows = 0, block_log2 = 0, nblocks = 0, ngroups = 0;
    uint64_t ids = 0;              // padded length of tcol
    uint16_t* tcol = nullptr;
    uint64_t* gbase = nullptr;     // [ngroups + 1]
    uint32_t* tseg = nullptr;      // [ngroups][nblocks][grp_rows + 1]
    ~TiledLayout();
};
}  // namespace mcmc

struct mcmc_graph {
    mcmc::GraphDev g;
    std::vector<std::unique_ptr<mcmc::TiledLayout>> tiles;   // freed with the graph
};
