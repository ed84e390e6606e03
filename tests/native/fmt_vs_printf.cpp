// Writer-format check (test infrastructure): the reference writes every spectrum column with
// std::format("{:10.5g} ", v) (harm_model.cpp:433-457); the product and the oracle write
// "%10.5g ".  This prints both for the values given on stdin (hex bit patterns, one per line) as
// "<fmt>|<printf>" so the test can compare them byte for byte.  fmt 12 (the library std::format
// was standardised from; header-only from torch's include tree) stands in for <format>, which
// libstdc++ 11 lacks.
#define FMT_HEADER_ONLY
#include <fmt/format.h>

#include <cinttypes>
#include <cstdio>
#include <cstring>

int main() {
    char line[64];
    while (std::fgets(line, sizeof line, stdin)) {
        uint64_t bits = std::strtoull(line, nullptr, 16);
        double v;
        std::memcpy(&v, &bits, sizeof v);
        const std::string a = fmt::format("{:10.5g} ", v);
        char b[64];
        std::snprintf(b, sizeof b, "%10.5g ", v);
        std::printf("%s|%s\n", a.c_str(), b);
    }
    return 0;
}
