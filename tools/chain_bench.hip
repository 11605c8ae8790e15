// tools/chain_bench.hip -- cycles per step of a serial f64 sum chain on one
// wave (the CNV slide's `tot`), in the forms the walk kernels could use:
// registers only, LDS broadcast, readlane into SGPRs, DPP lane shift.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/chain_bench.hip -o tools/chain_bench
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int N = 1 << 16;

__global__ __launch_bounds__(64) void k_reg(const double *in, double *out, long long *cyc) {
    double t = 0.0, a = in[threadIdx.x], b = in[threadIdx.x + 64];
    const long long c0 = clock64();
    for (int i = 0; i < N; i++) {
        t = t + a;
        t = t + b;
    }
    const long long c1 = clock64();
    out[threadIdx.x] = t;
    if (threadIdx.x == 0) cyc[0] = c1 - c0;
}

__global__ __launch_bounds__(64) void k_lds(const double *in, double *out, long long *cyc) {
    __shared__ double2 ad[64];
    const int lane = threadIdx.x;
    ad[lane] = make_double2(in[lane], in[lane + 64]);
    __syncthreads();
    double t = 0.0;
    const long long c0 = clock64();
    for (int r = 0; r < N / 64; r++) {
        double2 cur[8], nxt[8];
#pragma unroll
        for (int k = 0; k < 8; k++) cur[k] = ad[k];
#pragma unroll
        for (int g = 0; g < 8; g++) {
            if (g < 7) {
#pragma unroll
                for (int k = 0; k < 8; k++) nxt[k] = ad[(g + 1) * 8 + k];
            }
#pragma unroll
            for (int k = 0; k < 8; k++) {
                t = t + cur[k].x;
                t = t + cur[k].y;
            }
#pragma unroll
            for (int k = 0; k < 8; k++) cur[k] = nxt[k];
        }
        __syncthreads();
    }
    const long long c1 = clock64();
    out[threadIdx.x] = t;
    if (threadIdx.x == 0) cyc[0] = c1 - c0;
}

__device__ __forceinline__ double rl(double v, int k) {
    unsigned long long u;
    __builtin_memcpy(&u, &v, 8);
    const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)u, k), hi = __builtin_amdgcn_readlane((int)(unsigned)(u >> 32), k);
    const unsigned long long w = ((unsigned long long)hi << 32) | lo;
    double d;
    __builtin_memcpy(&d, &w, 8);
    return d;
}

__global__ __launch_bounds__(64) void k_readlane(const double *in, double *out, long long *cyc) {
    const double a = in[threadIdx.x], b = in[threadIdx.x + 64];
    double t = 0.0;
    const long long c0 = clock64();
    for (int r = 0; r < N / 64; r++) {
#pragma unroll
        for (int k = 0; k < 64; k++) {
            t = t + rl(a, k);
            t = t + rl(b, k);
        }
    }
    const long long c1 = clock64();
    out[threadIdx.x] = t;
    if (threadIdx.x == 0) cyc[0] = c1 - c0;
}

__device__ __forceinline__ double shr1(double v) {
    unsigned long long u;
    __builtin_memcpy(&u, &v, 8);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)u, 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), 0x138, 0xf, 0xf, true);
    const unsigned long long w = ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
    double d;
    __builtin_memcpy(&d, &w, 8);
    return d;
}

__global__ __launch_bounds__(64) void k_dpp(const double *in, double *out, long long *cyc) {
    const double a = in[threadIdx.x], b = in[threadIdx.x + 64];
    double t = 0.0;
    const long long c0 = clock64();
    for (int r = 0; r < N / 64; r++) {
        double x = threadIdx.x == 0 ? t + a : a;
        double y = x + b;
#pragma unroll
        for (int k = 1; k < 64; k++) y = (shr1(y) + x) + b;
        t = rl(y, 63);
    }
    const long long c1 = clock64();
    out[threadIdx.x] = t;
    if (threadIdx.x == 0) cyc[0] = c1 - c0;
}


// the walk's form: addends stored by the lanes, the chain run on the
// broadcast values, each step's sum handed back to its lane (lane-0 LDS
// stores, or a per-lane select)
template <int OUT>
__global__ __launch_bounds__(64) void k_lds_out(const double *in, double *out, long long *cyc) {
    __shared__ double2 ad[64];
    __shared__ double to[64];
    const int lane = threadIdx.x;
    double a = in[lane], b = in[lane + 64], acc = 0.0;
    double t = 0.0;
    const long long c0 = clock64();
    for (int r = 0; r < N / 64; r++) {
        ad[lane] = make_double2(a, b);
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        double2 cur[8], nxt[8];
        double mine = 0.0;
#pragma unroll
        for (int k = 0; k < 8; k++) cur[k] = ad[k];
#pragma unroll
        for (int g = 0; g < 8; g++) {
            if (g < 7) {
#pragma unroll
                for (int k = 0; k < 8; k++) nxt[k] = ad[(g + 1) * 8 + k];
            }
            double tt[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                t = t + cur[k].x;
                t = t + cur[k].y;
                tt[k] = t;
                if (OUT == 1) mine = lane == g * 8 + k ? t : mine;
            }
            if (OUT == 0 && lane == 0) {
#pragma unroll
                for (int k = 0; k < 8; k++) to[g * 8 + k] = tt[k];
            }
#pragma unroll
            for (int k = 0; k < 8; k++) cur[k] = nxt[k];
        }
        if (OUT == 0) {
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            mine = to[lane];
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
        }
        acc += mine;
        a = a * 0.5 + mine * 1e-30;  // the next round's addends depend on this round
    }
    const long long c1 = clock64();
    out[threadIdx.x] = t + acc;
    if (threadIdx.x == 0) cyc[0] = c1 - c0;
}

int main() {
    double h[128];
    for (int i = 0; i < 128; i++) h[i] = 1.0 / (i + 3);
    double *in, *out;
    long long *cyc, hc;
    (void)hipMalloc(&in, sizeof(h));
    (void)hipMalloc(&out, 64 * 8);
    (void)hipMalloc(&cyc, 8);
    (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    const char *names[] = {"registers", "lds broadcast", "readlane", "dpp shift", "lds, lane-0 out", "lds, select out"};
    void (*ks[])(const double *, double *, long long *) = {k_reg, k_lds, k_readlane, k_dpp, k_lds_out<0>, k_lds_out<1>};
    for (int k = 0; k < 6; k++) {
        for (int rep = 0; rep < 2; rep++) {
            hipLaunchKernelGGL(ks[k], dim3(1), dim3(64), 0, 0, in, out, cyc);
            (void)hipDeviceSynchronize();
        }
        (void)hipMemcpy(&hc, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-14s %.2f cycles per step (2 dependent f64 adds)\n", names[k], (double)hc / N);
    }
    return 0;
}
