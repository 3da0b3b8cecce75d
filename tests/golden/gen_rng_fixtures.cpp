// Generates tests/golden/rng_fixtures.json from the C++ standard library (g++ / libstdc++), the same
// library the reference links: std::seed_seq (stage_prepare/prepare.cpp:549-562), std::mt19937_64
// (stage drivers' _random, e.g. stage_interphase/simulation_driver.cpp:19) and
// std::normal_distribution<double> (stage_anatelophase/simulation_driver.cpp:25-32).
// Build + run: tests/golden/make_fixtures.sh
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

int main()
{
    std::printf("{\n  \"seed_seq\": [\n");
    const std::uint32_t masters[] = {0u, 1u, 42u, 123456789u, 4294967295u};
    for (int m = 0; m < 5; ++m) {
        std::seed_seq seq = {masters[m]};
        std::uint32_t v[3];
        seq.generate(v, v + 3);
        std::printf("    {\"master\": %u, \"stage_seeds\": [%u, %u, %u]}%s\n", masters[m], v[0], v[1], v[2],
                    m < 4 ? "," : "");
    }
    std::printf("  ],\n  \"seed_seq_long\": {\"seeds\": [7, 11, 13], \"out\": [");
    {
        std::seed_seq seq = {7u, 11u, 13u};
        std::vector<std::uint32_t> v(10);
        seq.generate(v.begin(), v.end());
        for (int k = 0; k < 10; ++k) std::printf("%u%s", v[k], k < 9 ? ", " : "");
    }
    std::printf("]},\n  \"mt19937_64\": [\n");
    const std::uint64_t seeds[] = {0ull, 1ull, 5489ull, 2058941775ull};
    for (int s = 0; s < 4; ++s) {
        std::mt19937_64 g(seeds[s]);
        std::printf("    {\"seed\": %llu, \"draws\": [", (unsigned long long)seeds[s]);
        for (int k = 0; k < 5; ++k) std::printf("\"%llu\"%s", (unsigned long long)g(), k < 4 ? ", " : "");
        // the 1000th output, after a state regeneration
        for (int k = 5; k < 999; ++k) g();
        std::printf("], \"draw_1000\": \"%llu\"}%s\n", (unsigned long long)g(), s < 3 ? "," : "");
    }
    std::printf("  ],\n  \"normal_distribution\": [\n");
    for (int s = 0; s < 3; ++s) {
        std::mt19937_64 g(seeds[s + 1]);
        std::normal_distribution<double> normal;
        std::printf("    {\"seed\": %llu, \"values\": [", (unsigned long long)seeds[s + 1]);
        for (int k = 0; k < 12; ++k) std::printf("%.17g%s", normal(g), k < 11 ? ", " : "");
        std::printf("]}%s\n", s < 2 ? "," : "");
    }
    std::printf("  ]\n}\n");
    return 0;
}
