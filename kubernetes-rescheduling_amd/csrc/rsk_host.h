// rsk_host.h — host-only internals of librsk.so (no HIP): error reporting and
// the experiment-switch macros.  The host sources that take caller input
// (rsk_workmodel.cpp, rsk_snapshot.cpp, rsk_plan.cpp) include only this header,
// so `make asan` builds them with g++ -fsanitize=address,undefined into a
// CPU-only test driver (tests/test_asan.py).
#pragma once

#include <cstdint>

#include "rsk.h"

namespace rsk {

// Error reporting: thread-local last error, returned through rsk_last_error().
void set_error(const char *fmt, ...);
const char *last_error();

#define RSK_CHECK(cond, ...)                                                             \
    do {                                                                                 \
        if (!(cond)) {                                                                   \
            ::rsk::set_error(__VA_ARGS__);                                               \
            return RSK_EINVAL;                                                           \
        }                                                                                \
    } while (0)

#define RSK_TRY(expr)                                                                    \
    do {                                                                                 \
        int _rc = (expr);                                                                \
        if (_rc != RSK_OK) return _rc;                                                   \
    } while (0)

// Experiment switches.  The product librsk.so reads no environment variable:
// RSK_KNOB(NAME, dflt) is the compiled default (no product source keeps one
// after its experiment is decided).  `make variant NAME=x DEFS=-DRSK_ENV_KNOBS`
// builds librsk_x.so, whose knobs read getenv("NAME") (A/B runs through
// RSK_LIB=.../librsk_x.so).  The profiling ablations, which make results wrong
// on purpose, exist only with -DRSK_ABLATIONS: otherwise RSK_ABL(args) is the
// constant 0 and the kernels compile without them.
int env_int(const char *name, int dflt);
#if defined(RSK_ENV_KNOBS) || defined(RSK_ABLATIONS)
#define RSK_KNOB(name, dflt) ::rsk::env_int(#name, (dflt))
#else
#define RSK_KNOB(name, dflt) (dflt)
#endif
#ifdef RSK_ABLATIONS
#define RSK_ABLATION(name) ::rsk::env_int(#name, 0)
#define RSK_ABL(a) ((a).ablate)
#else
#define RSK_ABLATION(name) 0
#define RSK_ABL(a) 0
#endif

}  // namespace rsk
