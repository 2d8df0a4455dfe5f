// The reference's random source, straight from the standard library it uses:
// std::mt19937 seeded (21 << 16) | rank (src/core/random.cpp:24-35) drawn through
// std::uniform_real_distribution (include/El/core/random/impl.hpp:134-139).
// Prints `count` draws of kind f64 or f32 on [lo, hi); pins oracle.mt_uniform.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
int main(int argc, char** argv) {
    if (argc != 6) return 2;
    const unsigned long seed = std::strtoul(argv[1], nullptr, 10);
    const int count = std::atoi(argv[2]);
    const double lo = std::atof(argv[3]), hi = std::atof(argv[4]);
    std::mt19937 g(static_cast<std::mt19937::result_type>(seed));
    if (std::strcmp(argv[5], "f64") == 0) {
        std::uniform_real_distribution<double> u(lo, hi);
        for (int i = 0; i < count; ++i) std::printf("%.17g\n", u(g));
    } else {
        std::uniform_real_distribution<float> u(static_cast<float>(lo), static_cast<float>(hi));
        for (int i = 0; i < count; ++i) std::printf("%.9g\n", static_cast<double>(u(g)));
    }
    return 0;
}
