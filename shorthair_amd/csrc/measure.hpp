// Measurement switches (A/B builds only).
//
// The shipped libcauchy256.so reads no environment variable and loads no code object: a drop-in
// codec must not change its kernels because of its caller's environment. The
// switches that select older kernels, launch splits or external code objects for same-box A/B
// runs exist only in libraries built with -DSH_MEASUREMENT_BUILD (tools/build_variant.sh); in the
// product build SH_MEASURE_ENV(name) is a null pointer and its argument text is dropped, so the
// switch names are not even present in the binary (tests/test_abi.py checks both).
#pragma once

#include <cstdlib>

#ifdef SH_MEASUREMENT_BUILD
#define SH_MEASURE_ENV(name) std::getenv(name)
#else
#define SH_MEASURE_ENV(name) (static_cast<const char *>(nullptr))
#endif

namespace sh {
// Integer value of a measurement switch (`e` from SH_MEASURE_ENV), or `dflt` when unset.
inline int measure_int(const char *e, int dflt) { return e ? std::atoi(e) : dflt; }
}  // namespace sh
