// mcmc_colorer_amd/csrc/xorwow.h -- the cuRAND XORWOW generator of the reference's GPU colorer,
// host and device (reference-GPU-semantics mode).
//
// Reference call sites: GPURand_k::initCurand, curand_init(seed, tid, 0, &states[tid])
// (GPUutils/GPURandomizer.cu:8-13, one state per vertex, seed = the uint32 --seed); curand_uniform
// (coloringMCMC_utils.cu:29, coloringMCMC_balance.cu:120). cuRAND is not in this image; its
// published device header defines (restated here, parity unpinned against CUDA):
//   init:  s0 = seed_lo ^ 0xaad26b49, s1 = seed_hi ^ 0xf7dcefdd, t0 = 1099087573 * s0,
//          t1 = 2591861531 * s1; d = 6615241 + t1 + t0; v = {123456789 + t0, 362436069 ^ t0,
//          521288629 + t1, 88675123 ^ t1, 5783321 + t0}; then skip subsequence * 2^67 outputs
//          (d is unchanged: 362437 * 2^67 = 0 mod 2^32) and `offset` outputs (offset 0 here).
//   next:  t = v0 ^ (v0 >> 2); v0..v3 = v1..v4; v4 = (v4 ^ (v4 << 4)) ^ (t ^ (t << 1));
//          d += 362437; return v4 + d.           (Marsaglia's xorwow)
//   uniform: x * 2^-32 + 2^-33 in fp32, (0, 1]   (x -> float rounds to nearest; the product is
//          exact, so fused or not gives the same float).
// rocRAND ships the same transition and 2^67 subsequence jump with other salts
// (rocrand_xorwow.h:113-116): tests pin next() and the jump against rocRAND's engine (flavour
// kRocrand), so only the salts and the uniform map rest on the cuRAND header restated above.
//
// The subsequence jump: A is the 160x160 GF(2) matrix of one step on v; J_k = A^(2^(67+k)),
// k = 0..31, are computed once on the host (xorwow_jump_tables) and a state jumps by `sub`
// subsequences by applying J_k for every set bit k of sub.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define XW_HD __host__ __device__ __forceinline__
#else
#define XW_HD inline
#endif

namespace xw {

constexpr int kWords = 5;                 // v[0..4]
constexpr int kBits = 32 * kWords;        // 160
constexpr int kJumpTables = 32;           // subsequences < 2^32
constexpr uint32_t kMatWords = kBits * kWords;   // column-major: column j = A e_j, 5 words

enum Flavor : int { kCurand = 0, kRocrand = 1 };

struct State {
    uint32_t v[kWords];
    uint32_t d;
};

XW_HD State salted(uint64_t seed, int flavor) {
    State s;
    uint32_t t0, t1;
    if (flavor == kCurand) {
        t0 = 1099087573u * ((uint32_t)seed ^ 0xaad26b49u);
        t1 = 2591861531u * ((uint32_t)(seed >> 32) ^ 0xf7dcefddu);
    } else {
        t0 = 1228688033u * ((uint32_t)seed ^ 0x2c7f967fu);
        t1 = 2073658381u * ((uint32_t)(seed >> 32) ^ 0xa03697cbu);
    }
    s.d = 6615241u + t1 + t0;
    s.v[0] = 123456789u + t0;
    s.v[1] = 362436069u ^ t0;
    s.v[2] = 521288629u + t1;
    s.v[3] = 88675123u ^ t1;
    s.v[4] = 5783321u + t0;
    return s;
}

XW_HD uint32_t next(State& s) {
    const uint32_t t = s.v[0] ^ (s.v[0] >> 2);
    s.v[0] = s.v[1];
    s.v[1] = s.v[2];
    s.v[2] = s.v[3];
    s.v[3] = s.v[4];
    s.v[4] = (s.v[4] ^ (s.v[4] << 4)) ^ (t ^ (t << 1));
    s.d += 362437u;
    return s.v[4] + s.d;
}

// curand_uniform: (0, 1].
XW_HD float uniform(uint32_t x) {
    const float p = (float)x * 2.3283064365386963e-10f;   // exact (power-of-two scale)
    return p + 1.16415321826934814453125e-10f;           // + 2^-33, rounded once
}

// v <- M v (M column-major, kMatWords words).
XW_HD void matvec(const uint32_t* __restrict__ M, uint32_t (&v)[kWords]) {
    uint32_t r[kWords] = {0, 0, 0, 0, 0};
    for (int w = 0; w < kWords; w++) {
        uint32_t bits = v[w];
        while (bits) {
            const int b = __builtin_ctz(bits);
            bits &= bits - 1u;
            const uint32_t* col = M + (uint32_t)(32 * w + b) * kWords;
            for (int k = 0; k < kWords; k++) r[k] ^= col[k];
        }
    }
    for (int k = 0; k < kWords; k++) v[k] = r[k];
}

// State of subsequence `sub` (offset 0): J_k for every set bit k of sub (tables: kJumpTables
// matrices of kMatWords words, J_k = A^(2^(67+k))).
XW_HD State init(uint64_t seed, uint32_t sub, int flavor, const uint32_t* __restrict__ tables) {
    State s = salted(seed, flavor);
    for (int k = 0; sub; k++, sub >>= 1)
        if (sub & 1u) matvec(tables + (uint32_t)k * kMatWords, s.v);
    return s;
}

}  // namespace xw

// Host: the jump tables (computed once per process, csrc/refmode.hip).
namespace mcmc {
const uint32_t* xorwow_jump_tables();   // kJumpTables * kMatWords words
}
