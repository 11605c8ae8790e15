// tools/alloc_probe.hip -- how long hipMalloc takes in a process started
// right after another one released a lot of device memory.
//   alloc_probe hold GB     allocate GB in 10 GB blocks, touch them, free, exit
//   alloc_probe take GB...  time one hipMalloc (+ memset) per size, in order
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    const double t0 = now_ms();
    if (hipSetDevice(0) != hipSuccess) return 3;
    if (!strcmp(argv[1], "hold")) {
        const size_t gb = (size_t)atoll(argv[2]);
        std::vector<void *> v;
        for (size_t k = 0; k < gb; k += 10) {
            void *p = nullptr;
            const size_t b = (size_t)(gb - k < 10 ? gb - k : 10) << 30;
            if (hipMalloc(&p, b) != hipSuccess) return 4;
            (void)hipMemset(p, 1, b);
            v.push_back(p);
        }
        (void)hipDeviceSynchronize();
        const double t1 = now_ms();
        for (void *p : v) (void)hipFree(p);
        printf("hold %zu GB: allocated+touched %.1f ms, freed %.1f ms\n", gb, t1 - t0, now_ms() - t1);
        return 0;
    }
    printf("start-up %.1f ms\n", now_ms() - t0);
    for (int i = 2; i < argc; i++) {
        const size_t b = (size_t)(atof(argv[i]) * (double)(1ull << 30));
        void *p = nullptr;
        const double a = now_ms();
        const hipError_t e = hipMalloc(&p, b);
        const double m = now_ms();
        if (e == hipSuccess) (void)hipMemset(p, 0, b);
        (void)hipDeviceSynchronize();
        printf("take %.1f GB: hipMalloc %.1f ms (%s), memset %.1f ms\n", atof(argv[i]), m - a, hipGetErrorString(e),
               now_ms() - m);
    }
    return 0;
}
