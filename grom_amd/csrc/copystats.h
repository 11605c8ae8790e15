// copystats.h -- GROM_COPY_STATS=1: how many runtime copies and fills each
// call site issues (printed at exit, most first).  A diagnostic for the
// blit counts of the whole-run trace; without the variable it
// costs one relaxed increment per call.
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

struct GromCopySite {
    const char *file;
    int line;
    std::atomic<long> n{0};
};

inline std::vector<GromCopySite *> &grom_copy_sites() {
    static std::vector<GromCopySite *> v;
    return v;
}

inline void grom_copy_report() {
    auto &v = grom_copy_sites();
    std::vector<GromCopySite *> s(v.begin(), v.end());
    std::sort(s.begin(), s.end(), [](GromCopySite *a, GromCopySite *b) { return a->n.load() > b->n.load(); });
    long tot = 0;
    for (auto *x : s) tot += x->n.load();
    fprintf(stderr, "copy stats: %ld runtime copies/fills\n", tot);
    for (auto *x : s)
        if (x->n.load()) fprintf(stderr, "  %6ld %s:%d\n", x->n.load(), x->file, x->line);
}

inline void grom_copy_register(GromCopySite *site) {
    static std::mutex mu;
    static bool armed = false;
    std::lock_guard<std::mutex> lk(mu);
    grom_copy_sites().push_back(site);
    if (!armed && getenv("GROM_COPY_STATS")) {
        armed = true;
        atexit(grom_copy_report);
    }
}

#define GROM_COPY_NOTE()                                                                                  \
    ([](const char *f, int l) {                                                                           \
        static GromCopySite site_{f, l};                                                                  \
        static std::once_flag once_;                                                                      \
        std::call_once(once_, [] { grom_copy_register(&site_); });                                        \
        site_.n.fetch_add(1, std::memory_order_relaxed);                                                  \
    }(__FILE__, __LINE__))
#define hipMemcpyAsync(...) (GROM_COPY_NOTE(), hipMemcpyAsync(__VA_ARGS__))
#define hipMemsetAsync(...) (GROM_COPY_NOTE(), hipMemsetAsync(__VA_ARGS__))
#define hipMemcpy(...) (GROM_COPY_NOTE(), hipMemcpy(__VA_ARGS__))
