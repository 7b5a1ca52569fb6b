// mikmeans — host-side ECMAScript number formatting (header-only, no torch / HIP).
//
// ECMAScript Number::toString (what JSON.stringify emits for a finite number),
// from the shortest round-trip digits (std::to_chars).  NaN/Infinity -> "null" as
// in JSON.  Used by the binding (js_format / js_array) and by the host sanitizer
// harness tests/native/jsnum_fuzz.cpp (ASan + UBSan).
#pragma once
#include <charconv>
#include <cmath>
#include <cstdlib>
#include <string>

namespace mk {

inline void js_number(double v, std::string& out) {
  if (std::isnan(v) || std::isinf(v)) { out += "null"; return; }
  if (v == 0.0) { out += '0'; return; }
  if (v < 0) { out += '-'; v = -v; }
  char buf[64];
  auto res = std::to_chars(buf, buf + sizeof(buf) - 1, v, std::chars_format::scientific);
  *res.ptr = '\0';  // atoi below must stop at the exponent's last digit
  // buf = d[.ddd]e(+|-)XX
  std::string digits;
  char* p = buf;
  int e10 = 0;
  for (; p < res.ptr && *p != 'e'; ++p)
    if (*p != '.') digits += *p;
  if (p < res.ptr) e10 = std::atoi(p + 1);
  const int k = (int)digits.size();
  const int n = e10 + 1;  // value = 0.digits * 10^n
  if (k <= n && n <= 21) {
    out += digits;
    out.append(n - k, '0');
  } else if (0 < n && n <= 21) {
    out.append(digits, 0, n);
    out += '.';
    out.append(digits, n, std::string::npos);
  } else if (-6 < n && n <= 0) {
    out += "0.";
    out.append(-n, '0');
    out += digits;
  } else {
    out += digits[0];
    if (k > 1) { out += '.'; out.append(digits, 1, std::string::npos); }
    out += 'e';
    const int ee = n - 1;
    out += ee >= 0 ? '+' : '-';
    out += std::to_string(ee >= 0 ? ee : -ee);
  }
}

}  // namespace mk
