// devmem.cpp -- the library's device allocations (devmem.h): accounting per
// buffer kind, and the reclaim / wait / retry path of an allocation that fails.
#include "devmem.h"

#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

namespace {

std::atomic<int64_t> g_now[GROM_DEVCAT_N + 1], g_peak[GROM_DEVCAT_N + 1];
std::atomic<int64_t> g_waits{0}, g_wait_ns{0}, g_slow{0}, g_slow_ns{0};
const char *cat_name(int cat) {
    static const char *n[] = {"scan", "breakpoint", "CNV", "stage", "decode", "phase arena", "other"};
    return cat >= 0 && cat < GROM_DEVCAT_N ? n[cat] : "other";
}

std::mutex g_mu;  // reclaim hooks, release epoch
std::condition_variable g_cv;
uint64_t g_epoch = 0;
struct Hook {
    grom_reclaim_fn fn;
    void *arg;
};
std::vector<Hook> g_hooks;
int g_reclaiming = 0;  // reclaim() calls running hooks (grom_dev_remove_reclaim waits for them)

double env_d(const char *name, double dflt) {
    const char *e = getenv(name);
    return e && *e ? atof(e) : dflt;
}

// The hooks run outside g_mu (they take their owners' locks and free device
// memory); g_reclaiming keeps a hook's owner alive meanwhile: removing a hook
// waits until no reclaim() is running one.
int64_t reclaim(int device, size_t want) {
    std::vector<Hook> hooks;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        hooks = g_hooks;
        g_reclaiming++;
    }
    int64_t got = 0;
    for (const Hook &h : hooks) {
        got += h.fn(h.arg, device, want);
        if (got >= (int64_t)want) break;
    }
    {
        std::lock_guard<std::mutex> lk(g_mu);
        g_reclaiming--;
    }
    g_cv.notify_all();
    return got;
}

}  // namespace

extern "C" void grom_dev_note(int cat, int64_t delta) {
    if (cat < 0 || cat >= GROM_DEVCAT_N) cat = GROM_DEVCAT_OTHER;
    const int64_t v = (g_now[cat] += delta), t = (g_now[GROM_DEVCAT_N] += delta);
    int64_t p = g_peak[cat].load();
    while (v > p && !g_peak[cat].compare_exchange_weak(p, v)) {}
    p = g_peak[GROM_DEVCAT_N].load();
    while (t > p && !g_peak[GROM_DEVCAT_N].compare_exchange_weak(p, t)) {}
}

extern "C" void grom_dev_peaks(int64_t *peak, int64_t *now) {
    for (int k = 0; k <= GROM_DEVCAT_N; k++) {
        if (peak) peak[k] = g_peak[k].load();
        if (now) now[k] = g_now[k].load();
    }
}

extern "C" void grom_dev_waits(int64_t *n, double *secs) {
    if (n) *n = g_waits.load();
    if (secs) *secs = (double)g_wait_ns.load() / 1e9;
}

extern "C" void grom_dev_slow(int64_t *n, double *secs) {
    if (n) *n = g_slow.load();
    if (secs) *secs = (double)g_slow_ns.load() / 1e9;
}

extern "C" void grom_dev_release_notify(void) {
    {
        std::lock_guard<std::mutex> lk(g_mu);
        g_epoch++;
    }
    g_cv.notify_all();
}

extern "C" void grom_dev_add_reclaim(grom_reclaim_fn fn, void *arg) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_hooks.push_back({fn, arg});
}

extern "C" void grom_dev_remove_reclaim(grom_reclaim_fn fn, void *arg) {
    std::unique_lock<std::mutex> lk(g_mu);
    for (size_t i = 0; i < g_hooks.size(); i++)
        if (g_hooks[i].fn == fn && g_hooks[i].arg == arg) {
            g_hooks.erase(g_hooks.begin() + (long)i);
            break;
        }
    // a reclaim() that copied the list before the erase may still call it
    g_cv.wait(lk, [] { return g_reclaiming == 0; });
}

extern "C" int grom_dev_malloc(void **p, size_t bytes, int cat) {
    *p = nullptr;
    if (bytes == 0) bytes = 16;
    // (read per call: in-process callers, e.g. the Python binding's cli_main,
    // set them per run)
    const double cap = env_d("GROM_TEST_HBM_CAP", 0.0);
    const double wait_s = env_d("GROM_ALLOC_WAIT_S", 60.0);
    const auto t0 = std::chrono::steady_clock::now();
    int device = 0;
    (void)hipGetDevice(&device);
    bool waited = false;
    for (;;) {
        const bool capped = cap > 0 && (double)(g_now[GROM_DEVCAT_N].load() + (int64_t)bytes) > cap;
        if (!capped) {
            const auto c0 = std::chrono::steady_clock::now();
            const hipError_t e = hipMalloc(p, bytes);
            const int64_t cns =
                std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - c0).count();
            if (cns > 100000000) {
                // one hipMalloc call that took long although the memory was
                // there: on a freshly started process, the driver still
                // clearing what an earlier process released
                g_slow++;
                g_slow_ns += cns;
                fprintf(stderr, "grom: hipMalloc of %.2f GB (%s) took %.1f ms\n", (double)bytes / 1e9, cat_name(cat),
                        cns / 1e6);
            }
            if (e == hipSuccess) {
                grom_dev_note(cat, (int64_t)bytes);
                if (waited) {
                    const int64_t ns =
                        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
                    g_waits++;
                    g_wait_ns += ns;
                    if (getenv("GROM_VERBOSE"))
                        fprintf(stderr, "grom: allocation of %.2f GB waited %.1f ms for device memory\n", (double)bytes / 1e9,
                                ns / 1e6);
                }
                return 0;
            }
            (void)hipGetLastError();  // the failure is handled here, not left sticky
            *p = nullptr;
            if (e != hipErrorOutOfMemory) {  // (a device fault, not memory: no reclaim, no wait)
                fprintf(stderr, "grom: hipMalloc of %.2f GB (%s) failed: %s\n", (double)bytes / 1e9, cat_name(cat),
                        hipGetErrorString(e));
                return -1;
            }
        }
        // idle memory of this process first (stages no chromosome holds)
        if (reclaim(device, bytes) > 0) continue;
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el > wait_s) return -1;
        waited = true;
        // then a release of this process, or 20 ms for another's
        std::unique_lock<std::mutex> lk(g_mu);
        const uint64_t e0 = g_epoch;
        g_cv.wait_for(lk, std::chrono::milliseconds(20), [&] { return g_epoch != e0; });
    }
}

extern "C" void grom_dev_free(void *p, size_t bytes, int cat) {
    if (!p) return;
    (void)hipFree(p);
    grom_dev_note(cat, -(int64_t)bytes);
    grom_dev_release_notify();
}

struct grom_arena {
    std::mutex mu;
    int cat = GROM_DEVCAT_OTHER;
    char *base = nullptr;
    size_t cap = 0, used = 0, over = 0, high = 0;
};

extern "C" grom_arena *grom_arena_new(int cat) {
    grom_arena *a = new grom_arena();
    a->cat = cat;
    return a;
}

extern "C" void grom_arena_free(grom_arena *a) {
    if (!a) return;
    if (a->base) grom_dev_free(a->base, a->cap, a->cat);
    delete a;
}

extern "C" int grom_arena_begin(grom_arena *a) {
    std::lock_guard<std::mutex> lk(a->mu);
    const size_t phase = a->used + a->over;
    if (phase > a->high) a->high = phase;
    a->used = 0;
    a->over = 0;
    if (a->high > a->cap) {  // an earlier phase overflowed: one block that holds it
        if (a->base) grom_dev_free(a->base, a->cap, a->cat);
        a->base = nullptr;
        a->cap = 0;
        const size_t want = a->high + a->high / 32 + ((size_t)1 << 20);
        void *p = nullptr;
        if (grom_dev_malloc(&p, want, a->cat)) return -1;
        a->base = (char *)p;
        a->cap = want;
    }
    return 0;
}

extern "C" void grom_arena_hint(grom_arena *a, size_t bytes) {
    std::lock_guard<std::mutex> lk(a->mu);
    if (bytes > a->high) a->high = bytes;
}

extern "C" void *grom_arena_take(grom_arena *a, size_t bytes) {
    std::lock_guard<std::mutex> lk(a->mu);
    const size_t b = (bytes + 255) & ~(size_t)255;
    if (a->base && a->used + b <= a->cap) {
        void *p = a->base + a->used;
        a->used += b;
        return p;
    }
    a->over += b;
    return nullptr;
}

extern "C" int64_t grom_arena_bytes(const grom_arena *a) { return a ? (int64_t)a->cap : 0; }
