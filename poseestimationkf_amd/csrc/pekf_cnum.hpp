// pekf_cnum.hpp -- number parsing of the host-side readers (pekf_log.cpp, pekf_wire.cpp) in the "C"
// locale: the decimal point is '.' whatever LC_NUMERIC the process that loads libpekf has set, as Python's
// float() (ReadFile.py:14-21) and the server, a C++ program that never calls setlocale (its std::stod,
// KFS/Parser.cpp:23-25, then runs in the "C" locale), read the same text.
#pragma once

#include <cstdlib>
#include <locale.h>

namespace pekf {

inline double strtod_c(const char *s, char **end) {
    static const locale_t c_locale = newlocale(LC_ALL_MASK, "C", (locale_t)0);
    return c_locale ? strtod_l(s, end, c_locale) : std::strtod(s, end);
}

}  // namespace pekf
