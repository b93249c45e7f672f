// tests/probes/rocrand_xorwow_probe.cpp -- test helper: prints rocRAND's XORWOW engine state
// (seed, subsequence, offset 0) and its next 4 outputs, one line per "seed:subsequence" argument.
// rocRAND shares cuRAND's transition and 2^67 subsequence jump (other salts): the independent pin
// for the build's and the oracle's jump-ahead (tests/test_xorwow.py).
#include <rocrand/rocrand_xorwow.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

struct Probe : rocrand_device::xorwow_engine {
    using rocrand_device::xorwow_engine::xorwow_engine;
    const rocrand_device::xorwow_engine::xorwow_state& st() const { return m_state; }
};

int main(int argc, char** argv) {
    for (int i = 1; i < argc; i++) {
        unsigned long long seed = 0, sub = 0;
        if (std::sscanf(argv[i], "%llu:%llu", &seed, &sub) != 2) return 2;
        Probe e(seed, sub, 0);
        const auto& s = e.st();
        std::printf("%u %u %u %u %u %u", s.x[0], s.x[1], s.x[2], s.x[3], s.x[4], s.d);
        for (int k = 0; k < 4; k++) std::printf(" %u", e.next());
        std::printf("\n");
    }
    return 0;
}
