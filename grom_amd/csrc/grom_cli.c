/* grom_cli.c -- the `grom` executable: a thin wrapper over grom_cli_main.
 * A fatal signal prints the host stack (addresses resolve with addr2line
 * against grom_amd/lib/libgrom_amd.so) before the process ends. */
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "../../include/grom_amd.h"

static void on_fatal(int sig) {
    void *fr[64];
    const int n = backtrace(fr, 64);
    static const char msg[] = "grom: fatal signal, host stack:\n";
    if (write(2, msg, sizeof(msg) - 1) < 0) { /* nothing more to do */ }
    backtrace_symbols_fd(fr, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

int main(int argc, char **argv) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_handler = on_fatal;
    sigaction(SIGBUS, &sa, NULL);
    sigaction(SIGSEGV, &sa, NULL);
    sigaction(SIGABRT, &sa, NULL);
    /* GROM_CLI_PROCESS=1 (opt-in): the library ends the process once the
     * outputs are written instead of freeing its device memory.  Not the
     * default: the driver then releases ~150 GB after the exit, and the next
     * run's large allocations wait for it (3.7 s per stage in back-to-back
     * runs) -- the freeing is only moved, not saved */
    const int rc = grom_cli_main(argc, argv);
    /* Every output is closed and the library has freed its device memory by
     * now; what is left of a normal exit is the runtime's own teardown in its
     * exit handlers (~0.1-0.2 s).  The process ends without it unless a tool
     * needs the handlers: a profiler that writes its records at exit
     * (GROM_EXIT_HANDLERS=1, e.g. rocprofv3) or the copy statistics
     * (GROM_COPY_STATS). */
    const char *eh = getenv("GROM_EXIT_HANDLERS");
    if (!(eh && atoi(eh) == 1) && !getenv("GROM_COPY_STATS")) {
        fflush(stdout);
        fflush(stderr);
        _exit(rc);
    }
    return rc;
}
