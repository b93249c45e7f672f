// mcmc_colorer_amd/csrc/refmode.hip -- reference-GPU-semantics mode: the per-vertex cuRAND XORWOW
// states of the reference's GPURand (GPUutils/GPURandomizer.cu:8-13, 85-101).
//
// mcmc_gpurand: n XORWOW states, double-buffered (a sweep reads parity t & 1 and writes the other,
// so a sweep whose proposal is discarded leaves the states as they were). Layout: structure of
// arrays, 6 words x n per parity ({v0..v4, d}): a wave's 64 consecutive vertices read and write
// 256 contiguous bytes per word.
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <vector>

#include "mcmc_common.h"
#include "xorwow.h"

namespace mcmc {

// J_k = A^(2^(67+k)), column-major (column j = the state after one jump of e_j).
const uint32_t* xorwow_jump_tables() {
    static std::vector<uint32_t> T;
    static std::once_flag once;
    std::call_once(once, [] {
        using Col = std::vector<uint32_t>;   // kMatWords
        auto mul = [](const Col& A, const Col& B) {   // (A B) e_j = A (B e_j)
            Col out(xw::kMatWords);
            for (int j = 0; j < xw::kBits; j++) {
                uint32_t v[xw::kWords];
                std::memcpy(v, &B[(size_t)j * xw::kWords], sizeof(v));
                xw::matvec(A.data(), v);
                std::memcpy(&out[(size_t)j * xw::kWords], v, sizeof(v));
            }
            return out;
        };
        Col A(xw::kMatWords);
        for (int j = 0; j < xw::kBits; j++) {   // one step of e_j (d is not part of the linear state)
            xw::State s{};
            s.v[j >> 5] = 1u << (j & 31);
            xw::next(s);
            std::memcpy(&A[(size_t)j * xw::kWords], s.v, sizeof(s.v));
        }
        for (int i = 0; i < 67; i++) A = mul(A, A);
        T.resize((size_t)xw::kJumpTables * xw::kMatWords);
        for (int k = 0; k < xw::kJumpTables; k++) {
            std::memcpy(&T[(size_t)k * xw::kMatWords], A.data(), sizeof(uint32_t) * xw::kMatWords);
            A = mul(A, A);
        }
    });
    return T.data();
}

namespace {

__global__ void gpurand_init_kernel(uint32_t n, uint64_t seed, const uint32_t* __restrict__ tables,
                                    uint32_t* __restrict__ st) {
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        const xw::State s = xw::init(seed, v, xw::kCurand, tables);
        for (int k = 0; k < xw::kWords; k++) st[(size_t)k * n + v] = s.v[k];
        st[(size_t)xw::kWords * n + v] = s.d;
    }
}

}  // namespace

}  // namespace mcmc

using namespace mcmc;

extern "C" {

int mcmc_xorwow_state(uint64_t seed, uint64_t subsequence, int flavor, uint32_t out[6]) {
    if (!out || subsequence >> 32) return fail(MCMC_E_ARG, "bad argument (subsequence < 2^32)");
    const xw::State s = xw::init(seed, (uint32_t)subsequence, flavor, xorwow_jump_tables());
    std::memcpy(out, s.v, sizeof(s.v));
    out[5] = s.d;
    return MCMC_OK;
}

int mcmc_device_mem_info(int device, uint64_t* free_bytes, uint64_t* total_bytes) {
    if (!free_bytes || !total_bytes) return fail(MCMC_E_ARG, "NULL argument");
    MCMC_HIP_TRY(hipSetDevice(device));
    size_t f = 0, t = 0;
    MCMC_HIP_TRY(hipMemGetInfo(&f, &t));
    *free_bytes = f;
    *total_bytes = t;
    return MCMC_OK;
}

int mcmc_hip_versions(int* built, int* runtime) {
    if (!built || !runtime) return fail(MCMC_E_ARG, "NULL argument");
    *built = HIP_VERSION;
    *runtime = 0;
    MCMC_HIP_TRY(hipRuntimeGetVersion(runtime));
    return MCMC_OK;
}

int mcmc_gpurand_create(uint32_t n, uint32_t seed, int device, mcmc_gpurand** out) {
    if (!out || n == 0) return fail(MCMC_E_ARG, "bad argument");
    MCMC_HIP_TRY(hipSetDevice(device));
    auto* r = new mcmc_gpurand;
    r->device = device;
    r->n = n;
    r->seed = seed;
    const size_t bytes = sizeof(uint32_t) * 6ull * n;
    uint32_t* tab = nullptr;
    hipError_t e = hipMalloc(&r->states[0], bytes);
    if (e == hipSuccess) e = hipMalloc(&r->states[1], bytes);
    if (e == hipSuccess) e = hipMalloc(&tab, sizeof(uint32_t) * xw::kJumpTables * xw::kMatWords);
    if (e == hipSuccess)
        e = hipMemcpy(tab, xorwow_jump_tables(), sizeof(uint32_t) * xw::kJumpTables * xw::kMatWords,
                      hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        const uint32_t blocks = std::min<uint32_t>((n + 255) / 256, 8192u);
        gpurand_init_kernel<<<blocks, 256>>>(n, seed, tab, r->states[0]);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipDeviceSynchronize();
    }
    (void)hipFree(tab);
    if (e != hipSuccess) {
        mcmc_gpurand_destroy(r);
        return fail(MCMC_E_HIP, std::string("gpurand: ") + hipGetErrorString(e));
    }
    *out = r;
    return MCMC_OK;
}

int mcmc_gpurand_states(const mcmc_gpurand* r, uint32_t* out) {
    if (!r || !out) return fail(MCMC_E_ARG, "NULL argument");
    MCMC_HIP_TRY(hipSetDevice(r->device));
    std::vector<uint32_t> soa(6ull * r->n);
    MCMC_HIP_TRY(hipMemcpy(soa.data(), r->states[r->cur], sizeof(uint32_t) * soa.size(), hipMemcpyDeviceToHost));
    for (uint32_t v = 0; v < r->n; v++)
        for (int k = 0; k < 6; k++) out[6ull * v + k] = soa[(size_t)k * r->n + v];
    return MCMC_OK;
}

void mcmc_gpurand_destroy(mcmc_gpurand* r) {
    if (!r) return;
    (void)hipSetDevice(r->device);
    (void)hipFree(r->states[0]);
    (void)hipFree(r->states[1]);
    delete r;
}

}  // extern "C"
