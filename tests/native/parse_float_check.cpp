// Test harness (CPU only, built by tests/test_parse_float_cpu.py with g++): reads one
// decimal literal per line and prints the bits of pytext.h's parse_float result as 16
// hex digits ("ERR" when it rejects the text).
#include <cstdio>
#include <cstring>
#include <iostream>
#include <string>

#include "../../improving-learned-index_amd/csrc/pytext.h"

int main() {
    std::string line;
    while (std::getline(std::cin, line)) {
        double v;
        if (!di::py::parse_float(line, &v)) {
            std::puts("ERR");
            continue;
        }
        unsigned long long b;
        std::memcpy(&b, &v, 8);
        std::printf("%016llx\n", b);
    }
    return 0;
}
