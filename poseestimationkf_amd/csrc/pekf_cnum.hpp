// pekf_cnum.hpp -- number parsing and printing of the host-side readers and writer (pekf_log.cpp,
// pekf_wire.cpp) in the "C" locale: the decimal point is '.' whatever LC_NUMERIC the process that loads
// libpekf has set, as Python's float() (ReadFile.py:14-21) and the server, a C++ program that never calls
// setlocale (its std::stod and std::to_string, KFS/Parser.cpp:23-25, KFS/KalmanFilter.cpp:28, then run in
// the "C" locale), read and write the same text.
#pragma once

#include <cstdlib>
#include <locale.h>

namespace pekf {

// the "C" locale object ((locale_t)0 if it cannot be made)
inline locale_t c_locale_obj() {
    static const locale_t c = newlocale(LC_ALL_MASK, "C", (locale_t)0);
    return c;
}

// for uselocale: the "C" locale, or the process's own if it cannot be made
inline locale_t c_locale() {
    const locale_t c = c_locale_obj();
    return c ? c : LC_GLOBAL_LOCALE;
}

inline double strtod_c(const char *s, char **end) {
    const locale_t c = c_locale_obj();
    return c ? strtod_l(s, end, c) : std::strtod(s, end);
}

}  // namespace pekf
