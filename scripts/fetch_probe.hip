// FETCH_SIZE / WRITE_SIZE calibration on the access widths the sweep kernels use:
// known byte counts read (or written) in each pattern, run under
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_probe     (pass 1)
//   rocprofv3 --pmc WRITE_SIZE -- ./fetch_probe     (pass 2)
// and compared by scripts/fetch_calib.py with the bytes printed here. Patterns:
//   stream16 / stream4 / stream2  coalesced streaming reads, 16 / 4 / 2 B per lane, 1 GiB
//   gather2 / gather4 / gather16  random reads of 2 / 4 / 16 B (the walks' colour and id gathers)
//                                 over a 4 GiB buffer (past the 256 MiB Infinity Cache)
//   scatter2                      random 2 B stores (a changed row's uint16 colour)
// For the random patterns the expected bytes are the distinct 64 B and 128 B lines touched.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

template <typename T>
__device__ inline uint32_t fold(const T& v) {
    if constexpr (sizeof(T) == 16) {
        const uint4 u = *reinterpret_cast<const uint4*>(&v);
        return u.x ^ u.y ^ u.z ^ u.w;
    } else {
        return (uint32_t)v;
    }
}

// magic: a run-time value the zeroed input never produces (a compile-time one the compiler could
// prove unreachable for 16-bit data and drop the loads)
template <typename T>
__global__ void __launch_bounds__(256) stream_kernel(const T* __restrict__ p, size_t n, uint32_t* out, uint32_t magic) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256u) acc ^= fold(p[i]);
    if (acc == magic) out[blockIdx.x] = acc;   // (never true for the zeroed input: no stores)
}

__global__ void __launch_bounds__(256) flush_kernel(const uint4* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256u) acc ^= fold(p[i]);
    if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;
}

// the random slot of access i (computed on the device: no index array to stream)
__host__ __device__ inline uint64_t slot_of(uint64_t i, uint64_t salt, uint64_t slots) {
    uint64_t z = i * 0x9e3779b97f4a7c15ull + salt;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return (z ^ (z >> 31)) % slots;
}

template <typename T>
__global__ void __launch_bounds__(256) gather_kernel(const T* __restrict__ p, uint64_t salt, uint64_t slots, size_t m,
                                                     uint32_t* out, uint32_t magic) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < m; i += (size_t)gridDim.x * 256u)
        acc ^= fold(p[slot_of(i, salt, slots)]);
    if (acc == magic) out[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(256) scatter2_kernel(uint16_t* __restrict__ p, uint64_t salt, uint64_t slots, size_t m) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < m; i += (size_t)gridDim.x * 256u)
        p[slot_of(i, salt, slots)] = (uint16_t)i;
}

static void lines(const std::vector<uint64_t>& byte_off, uint64_t* l64, uint64_t* l128) {
    std::vector<uint64_t> a(byte_off);
    for (auto& x : a) x >>= 6;
    std::sort(a.begin(), a.end());
    *l64 = std::unique(a.begin(), a.end()) - a.begin();
    a.resize(*l64);
    for (auto& x : a) x >>= 1;
    *l128 = std::unique(a.begin(), a.end()) - a.begin();
}

int main() {
    const size_t SB = 1ull << 30, GB = 4ull << 30, M = 1ull << 24;
    void *s = nullptr, *g = nullptr;
    uint32_t* out = nullptr;
    CK(hipMalloc(&s, SB));
    CK(hipMalloc(&g, GB));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(s, 0, SB));
    CK(hipMemset(g, 0, GB));
    const int grid = 256 * 16;
    const uint32_t magic = 0x1234u;
    // streaming: every byte of the 1 GiB buffer once; a 512 MiB read of g between runs evicts the
    // Infinity Cache
    auto flush = [&]() -> int {
        flush_kernel<<<grid, 256>>>(reinterpret_cast<const uint4*>(g) + (GB / 2) / 16, (GB / 4) / 16, out);
        CK(hipDeviceSynchronize());
        return 0;
    };
    if (flush()) return 1;
    stream_kernel<uint4><<<grid, 256>>>(reinterpret_cast<const uint4*>(s), SB / 16, out, magic);
    CK(hipDeviceSynchronize());
    printf("stream16 bytes %zu\n", SB);
    if (flush()) return 1;
    stream_kernel<uint32_t><<<grid, 256>>>(reinterpret_cast<const uint32_t*>(s), SB / 4, out, magic);
    CK(hipDeviceSynchronize());
    printf("stream4 bytes %zu\n", SB);
    if (flush()) return 1;
    stream_kernel<uint16_t><<<grid, 256>>>(reinterpret_cast<const uint16_t*>(s), SB / 2, out, magic);
    CK(hipDeviceSynchronize());
    printf("stream2 bytes %zu\n", SB);
    std::vector<uint64_t> off(M);
    struct G { const char* name; uint32_t w; };
    uint64_t salt = 1;
    for (G pat : {G{"gather2", 2}, G{"gather4", 4}, G{"gather16", 16}, G{"scatter2", 2}}) {
        const uint64_t slots = GB / pat.w;
        salt += 0x1234567ull;
        for (size_t i = 0; i < M; i++) off[i] = slot_of(i, salt, slots) * pat.w;
        uint64_t l64 = 0, l128 = 0;
        lines(off, &l64, &l128);
        if (flush()) return 1;
        if (pat.w == 2 && pat.name[0] == 'g')
            gather_kernel<uint16_t><<<grid, 256>>>(reinterpret_cast<const uint16_t*>(g), salt, slots, M, out, magic);
        else if (pat.w == 4)
            gather_kernel<uint32_t><<<grid, 256>>>(reinterpret_cast<const uint32_t*>(g), salt, slots, M, out, magic);
        else if (pat.w == 16)
            gather_kernel<uint4><<<grid, 256>>>(reinterpret_cast<const uint4*>(g), salt, slots, M, out, magic);
        else
            scatter2_kernel<<<grid, 256>>>(reinterpret_cast<uint16_t*>(g), salt, slots, M);
        CK(hipDeviceSynchronize());
        printf("%s accesses %zu lines64 %llu lines128 %llu\n", pat.name, M, (unsigned long long)l64,
               (unsigned long long)l128);
    }
    CK(hipFree(s));
    CK(hipFree(g));
    CK(hipFree(out));
    return 0;
}
