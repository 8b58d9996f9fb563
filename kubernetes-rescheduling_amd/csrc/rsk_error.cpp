// rsk_error.cpp — librsk's thread-local last error and the experiment-switch
// reader (host only; also linked into the `make asan` test driver).
#include <cstdarg>
#include <cstdio>
#include <cstdlib>

#include "rsk_host.h"

namespace rsk {

static thread_local char g_err[1024] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

const char *last_error() { return g_err; }

int env_int(const char *name, int dflt) {  // RSK_KNOB in -DRSK_ENV_KNOBS variant builds only
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
}

}  // namespace rsk

extern "C" const char *rsk_last_error(void) { return rsk::last_error(); }
