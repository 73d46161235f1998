// Generates tests/golden/rocrand_xorwow_kat.json from rocRAND's own XORWOW engine (the host side of its
// header-only device API, /opt/rocm/include/rocrand/rocrand_xorwow.h).  Test infrastructure: rocRAND
// implements the same published xorwow generator as cuRAND (Marsaglia's base state, Weyl step 362437,
// the five-word shift recurrence, the seed scrambled into the state by two xor constants and two
// multipliers) with its own four seeding constants, so the fixture pins everything of the oracle's
// cuRAND restatement (oracle/rt_oracle.c orc_xorwow_seed / orc_curand) except cuRAND's four constants,
// which the survey probe pins (tests/test_oracle.py).
//
//   hipcc -O1 -std=c++17 tests/golden/make_rocrand_xorwow_kat.cpp -o /tmp/make_rocrand_xorwow_kat
//   /tmp/make_rocrand_xorwow_kat > tests/golden/rocrand_xorwow_kat.json
#include <rocrand/rocrand_kernel.h>

#include <cstdio>

// the engine's state is protected: read it through a subclass
struct Peek : rocrand_device::xorwow_engine {
    Peek(unsigned long long seed) : rocrand_device::xorwow_engine(seed, 0ull, 0ull) {}
    unsigned d() const { return m_state.d; }
    unsigned x(int i) const { return m_state.x[i]; }
};

int main() {
    const unsigned long long seeds[] = {0ull, 1ull, 1984ull, 1985ull, 1984ull + 2073599ull, (1ull << 32) + 5ull,
                                        0xdeadbeefcafef00dull, 0xffffffffffffffffull};
    const int n = sizeof(seeds) / sizeof(seeds[0]);
    std::printf("{\n \"generator\": \"rocRAND xorwow_engine(seed, 0, 0): state (d, x[0..4]) after seeding, then next()\",\n");
    std::printf(" \"seeding_constants\": {\"xor0\": %u, \"xor1\": %u, \"mul0\": %u, \"mul1\": %u},\n", 0x2c7f967fu,
                0xa03697cbu, 1228688033u, 2073658381u);
    std::printf(" \"streams\": [\n");
    for (int c = 0; c < n; c++) {
        Peek s(seeds[c]);
        std::printf("  {\"seed\": %llu, \"init\": [%u, %u, %u, %u, %u, %u], \"raw\": [", seeds[c], s.d(), s.x(0), s.x(1),
                    s.x(2), s.x(3), s.x(4));
        for (int i = 0; i < 16; i++) std::printf("%s%u", i ? ", " : "", s.next());
        std::printf("]}%s\n", c + 1 < n ? "," : "");
    }
    std::printf(" ]\n}\n");
    return 0;
}
