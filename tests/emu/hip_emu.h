// hip_emu.h -- TEST INFRASTRUCTURE ONLY.
//
// Runs the unmodified HIP sources of grom_amd (scan.hip and the kernels it
// includes) on the host so kernels can be checked against the oracle -- and
// under AddressSanitizer -- without a GPU.  A launch executes its blocks one
// after another; each block runs blockDim host threads that meet at real
// barriers for __syncthreads, so LDS (`__shared__`, here a static) is shared by
// the block exactly as on the device.  Wave-level intrinsics assume the
// wave-uniform control flow the kernels already guarantee.  Never linked into
// the product library.
#pragma once
#include <algorithm>
#include <atomic>
#include <barrier>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#define __global__
#define __device__
#define __host__
#define __forceinline__ inline
#define __constant__ static const
#define __launch_bounds__(...)
#define __align__(n) alignas(n)
#define __shared__ static

struct dim3 {
    unsigned x, y, z;
    dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};
struct alignas(16) uint4 { unsigned x, y, z, w; };
struct alignas(8) uint2 { unsigned x, y; };
inline uint4 make_uint4(unsigned x, unsigned y, unsigned z, unsigned w) { return uint4{x, y, z, w}; }
struct emu_idx { unsigned x, y, z; };
extern thread_local emu_idx threadIdx, blockIdx;
extern emu_idx blockDim, gridDim;

using std::max;
using std::min;

// ---- synchronisation within the emulated block ----
struct emu_block_sync {
    std::barrier<> *bar = nullptr;
    std::vector<std::barrier<> *> wave_bar;  // one per 64-lane wave
    std::atomic<int> count{0};
    std::vector<unsigned long long> xch;
};
extern emu_block_sync *g_emu_sync;
inline void __syncthreads() { g_emu_sync->bar->arrive_and_wait(); }
inline int __syncthreads_count(int p) {
    if (p) g_emu_sync->count.fetch_add(1);
    g_emu_sync->bar->arrive_and_wait();
    int v = g_emu_sync->count.load();
    g_emu_sync->bar->arrive_and_wait();
    if (threadIdx.x == 0) g_emu_sync->count.store(0);
    g_emu_sync->bar->arrive_and_wait();
    return v;
}
// cross-lane operations exchange through xch under the wave's own barrier,
// so (as on the GPU) they need only the 64 lanes of one wave to be converged
inline unsigned long long emu_lane_xch(unsigned long long u, unsigned src) {
    const unsigned t = threadIdx.x;
    std::barrier<> *wb = g_emu_sync->wave_bar[t / 64];
    g_emu_sync->xch[t] = u;
    wb->arrive_and_wait();
    const unsigned long long r = g_emu_sync->xch[(t & ~63u) | (src & 63u)];
    wb->arrive_and_wait();
    return r;
}
template <typename T>
inline T __shfl_xor(T v, int off, int width = 64) {
    (void)width;
    unsigned long long u = 0;
    std::memcpy(&u, &v, sizeof(T));
    const unsigned long long r = emu_lane_xch(u, (threadIdx.x & 63u) ^ (unsigned)off);
    T out;
    std::memcpy(&out, &r, sizeof(T));
    return out;
}
template <typename T>
inline T __shfl_up(T v, unsigned d, int width = 64) {
    (void)width;
    unsigned long long u = 0;
    std::memcpy(&u, &v, sizeof(T));
    const unsigned l = threadIdx.x & 63u;
    const unsigned long long r = emu_lane_xch(u, l >= d ? l - d : l);
    T out;
    std::memcpy(&out, &r, sizeof(T));
    return out;
}
inline int __popcll(unsigned long long v) { return __builtin_popcountll(v); }
inline int __clzll(unsigned long long v) { return v ? __builtin_clzll(v) : 64; }
inline int __ffsll(long long v) { return __builtin_ffsll(v); }
template <typename T>
inline T __shfl(T v, int src, int width = 64) {
    (void)width;
    unsigned long long u = 0;
    std::memcpy(&u, &v, sizeof(T));
    const unsigned long long r = emu_lane_xch(u, (unsigned)src & 63u);
    T out;
    std::memcpy(&out, &r, sizeof(T));
    return out;
}
inline int __builtin_amdgcn_readlane(int v, int i) {
    return (int)(unsigned)emu_lane_xch((unsigned)v, (unsigned)i);
}
inline unsigned long long __ballot(int p) {
    const unsigned t = threadIdx.x;
    std::barrier<> *wb = g_emu_sync->wave_bar[t / 64];
    g_emu_sync->xch[t] = p ? 1 : 0;
    wb->arrive_and_wait();
    unsigned long long m = 0;
    for (unsigned k = 0; k < 64 && (t & ~63u) + k < g_emu_sync->xch.size(); k++)
        if (g_emu_sync->xch[(t & ~63u) + k]) m |= 1ull << k;
    wb->arrive_and_wait();
    return m;
}
inline int __builtin_amdgcn_readfirstlane(int v) { return v; }
inline long long __double_as_longlong(double d) { long long r; std::memcpy(&r, &d, 8); return r; }
inline double __longlong_as_double(long long v) { double r; std::memcpy(&r, &v, 8); return r; }

// ---- atomics ----
template <typename T, typename U>
inline T atomicAdd(T *p, U v) { return __atomic_fetch_add(p, (T)v, __ATOMIC_SEQ_CST); }
template <typename T, typename U>
inline T atomicSub(T *p, U v) { return __atomic_fetch_sub(p, (T)v, __ATOMIC_SEQ_CST); }
template <typename T, typename U>
inline T atomicMax(T *p, U v) {
    T old = __atomic_load_n(p, __ATOMIC_SEQ_CST);
    while (old < (T)v && !__atomic_compare_exchange_n(p, &old, (T)v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
    }
    return old;
}

// ---- runtime API subset used by scan.hip ----
typedef int hipError_t;
typedef void *hipStream_t;
typedef void *hipEvent_t;
enum { hipSuccess = 0, hipErrorInvalidValue = 1 };
enum hipMemcpyKind { hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice };
#define hipStreamNonBlocking 1
inline const char *hipGetErrorString(hipError_t) { return "emulated error"; }
inline hipError_t hipGetLastError() { return hipSuccess; }
inline hipError_t hipSetDevice(int) { return hipSuccess; }
inline hipError_t hipGetDevice(int *d) { *d = 0; return hipSuccess; }
inline hipError_t hipGetDeviceCount(int *n) { *n = 1; return hipSuccess; }
inline hipError_t hipMalloc(void **p, size_t n) {
    *p = std::malloc(n);
    return *p ? hipSuccess : hipErrorInvalidValue;
}
template <typename T>
inline hipError_t hipMalloc(T **p, size_t n) { return hipMalloc((void **)p, n); }
inline hipError_t hipFree(void *p) { std::free(p); return hipSuccess; }
inline hipError_t hipHostMalloc(void **p, size_t n, unsigned) {
    *p = std::malloc(n);
    return *p ? hipSuccess : hipErrorInvalidValue;
}
inline hipError_t hipHostFree(void *p) { std::free(p); return hipSuccess; }
inline hipError_t hipMemcpy(void *d, const void *s, size_t n, hipMemcpyKind) { std::memcpy(d, s, n); return hipSuccess; }
inline hipError_t hipMemcpyAsync(void *d, const void *s, size_t n, hipMemcpyKind k, hipStream_t) {
    return hipMemcpy(d, s, n, k);
}
inline hipError_t hipMemsetAsync(void *d, int v, size_t n, hipStream_t) { std::memset(d, v, n); return hipSuccess; }
inline hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned) { *s = (void *)1; return hipSuccess; }
inline hipError_t hipStreamCreateWithPriority(hipStream_t *s, unsigned, int) { *s = (void *)1; return hipSuccess; }
inline hipError_t hipDeviceGetStreamPriorityRange(int *lo, int *hi) { *lo = 0; *hi = 0; return hipSuccess; }
inline hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
inline hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }
inline hipError_t hipEventCreate(hipEvent_t *e) { *e = (void *)1; return hipSuccess; }
#define hipEventDisableTiming 2
inline hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned) { *e = (void *)1; return hipSuccess; }
// launches run synchronously here, so cross-stream waits are already satisfied
inline hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned) { return hipSuccess; }
inline hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
inline hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
inline hipError_t hipEventElapsedTime(float *ms, hipEvent_t, hipEvent_t) { *ms = 0.f; return hipSuccess; }
inline hipError_t hipEventDestroy(hipEvent_t) { return hipSuccess; }

void emu_run_grid(dim3 grid, dim3 block, const std::function<void()> &body);

#define hipLaunchKernelGGL(kernel, grid, block, shmem, stream, ...) \
    emu_run_grid(dim3(grid), dim3(block), [=]() { kernel(__VA_ARGS__); })
