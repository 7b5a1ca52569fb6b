// Host sanitizer harness for the JS number formatter (mikmeans/csrc/jsnum.h).
// Built with -fsanitize=address,undefined by tests/test_native_host.py; reads
// doubles as hex bit patterns on stdin and prints one formatted number per line,
// which the test compares against the Python implementation (utils/jsjson.py).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "jsnum.h"

int main() {
  char line[64];
  while (std::fgets(line, sizeof line, stdin)) {
    unsigned long long bits = std::strtoull(line, nullptr, 16);
    double v;
    std::memcpy(&v, &bits, sizeof v);
    std::string s;
    mk::js_number(v, s);
    std::puts(s.c_str());
  }
  return 0;
}
