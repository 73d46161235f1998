// Generates tests/golden/philox_kat.json from rocRAND's own Philox4x32-10 engine (the host side of its
// header-only device API, /opt/rocm/include/rocrand), the generator BASELINE.json's north_star names for
// the perf-mode RNG ("hiprand (Philox) per-pixel state").  Test infrastructure: the fixture pins the
// oracle's restatement (oracle/rt_oracle.c, orc_philox4x32_10) and, through the GPU parity tests, the
// kernel's.
//
//   hipcc -O1 -std=c++17 tests/golden/make_philox_kat.cpp -o /tmp/make_philox_kat
//   /tmp/make_philox_kat > tests/golden/philox_kat.json
//
// A pixel's stream is rocrand_init(seed, subsequence = global pixel index, offset = frame << 34, &s) followed
// by rocrand_uniform(&s) per draw.
#include <rocrand/rocrand_kernel.h>

#include <cstdio>
#include <cstring>

int main() {
    struct Case {
        unsigned long long seed, pixel, frame;
    };
    const Case cases[] = {{1984ull, 0ull, 0ull},       {1984ull, 1ull, 0ull},
                          {1984ull, 2073599ull, 0ull}, {1984ull, 123456ull, 7ull},
                          {0ull, 0ull, 0ull},          {0xdeadbeefcafef00dull, 4294967295ull, 65535ull},
                          {(1ull << 32) + 5ull, 99ull, 1ull}};
    const int n = sizeof(cases) / sizeof(cases[0]);
    std::printf("{\n \"generator\": \"rocRAND philox4x32_10 (rocrand_init(seed, pixel, frame << 34); rocrand / rocrand_uniform)\",\n");
    std::printf(" \"streams\": [\n");
    for (int c = 0; c < n; c++) {
        rocrand_state_philox4x32_10 s;
        rocrand_init(cases[c].seed, cases[c].pixel, cases[c].frame << 34, &s);
        rocrand_state_philox4x32_10 s2 = s;
        std::printf("  {\"seed\": %llu, \"pixel\": %llu, \"frame\": %llu, \"raw\": [", cases[c].seed, cases[c].pixel,
                    cases[c].frame);
        for (int i = 0; i < 11; i++) std::printf("%s%u", i ? ", " : "", rocrand(&s2));
        std::printf("], \"uniform_bits\": [");
        for (int i = 0; i < 11; i++) {
            const float f = rocrand_uniform(&s);
            unsigned u;
            std::memcpy(&u, &f, 4);
            std::printf("%s%u", i ? ", " : "", u);
        }
        std::printf("]}%s\n", c + 1 < n ? "," : "");
    }
    std::printf(" ]\n}\n");
    return 0;
}
