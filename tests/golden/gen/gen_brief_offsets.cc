// Fixture generator: the reference's Brief::preComputeOffsets (/root/reference/src/BriefDescriptor.cc:4-20)
// algorithm -- std::mt19937 + std::uniform_int_distribution<int>(-8, 8), 256 x 4 draws -- with the
// std::random_device seed replaced by an explicit one so the table is reproducible.  Written from the
// reference's behaviour (not copied); built with this container's g++ 11 / libstdc++.
// Usage: gen_brief_offsets SEED OUT.bin   -> 1024 int8 values, row-major [256][4].
#include <cstdio>
#include <cstdlib>
#include <random>
int main(int argc, char** argv) {
    if (argc != 3) return 2;
    std::mt19937 gen((unsigned)std::strtoul(argv[1], nullptr, 10));
    std::uniform_int_distribution<int> dist(-8, 8);
    signed char buf[1024];
    for (int i = 0; i < 256; ++i)
        for (int j = 0; j < 4; ++j) buf[4 * i + j] = (signed char)dist(gen);
    FILE* f = std::fopen(argv[2], "wb");
    if (!f) return 1;
    std::fwrite(buf, 1, sizeof buf, f);
    std::fclose(f);
    return 0;
}
