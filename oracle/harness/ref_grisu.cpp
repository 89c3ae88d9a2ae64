// Number-formatting golden vectors: reads IEEE-754 doubles as 16-hex-digit bit
// patterns on stdin and prints how the reference's vendored JSON writer
// (/root/reference/src/json.hpp, nlohmann 3.5.0, dump()) renders each one.
// Development-container only; outputs committed as tests/golden/grisu2_vectors.tsv.
#include <cstdint>
#include <cstring>
#include <iostream>
#include <string>
#include "json.hpp"

int main() {
    std::string hex;
    while (std::cin >> hex) {
        uint64_t bits = std::stoull(hex, nullptr, 16);
        double d;
        std::memcpy(&d, &bits, sizeof d);
        jsn::json j = d;
        std::cout << hex << '\t' << j.dump() << '\n';
    }
    return 0;
}
