// mcmc_colorer_amd/csrc/mcmc_common.h -- shared host-side plumbing of libmcmc_hip.so:
// error reporting (the C ABI returns codes, never aborts) and the opaque handle layouts.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

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

struct mcmc_graph {
    mcmc::GraphDev g;
};
