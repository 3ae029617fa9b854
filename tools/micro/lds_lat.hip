// micro-benchmark: latency of LDS ops for a lone wave (development aid)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(64) void k(unsigned long long* out, int iters) {
    __shared__ unsigned long long a[4096];
    __shared__ unsigned int c32[64];
    const int ln = threadIdx.x;
    for (int e = ln; e < 4096; e += 64) a[e] = e;
    if (ln < 64) c32[ln] = 0;
    __syncthreads();
    unsigned long long t0, t1, x = ln;
    // 1) dependent ds_read_b64 chain
    t0 = clock64();
    for (int i = 0; i < iters; ++i) x = a[(x * 7 + 13) & 4095];
    t1 = clock64();
    if (ln == 0) out[0] = (t1 - t0) / iters;
    // 2) dependent CAS chain
    unsigned long long y = ln;
    t0 = clock64();
    for (int i = 0; i < iters; ++i) y = atomicCAS(&a[(y + ln) & 4095], 0ull, 5ull) & 4095;
    t1 = clock64();
    if (ln == 0) out[1] = (t1 - t0) / iters;
    // 3) ballot + popcount chain
    unsigned long long z = ln;
    t0 = clock64();
    for (int i = 0; i < iters; ++i) z += __popcll(__ballot((z & 1) == 0));
    t1 = clock64();
    if (ln == 0) out[2] = (t1 - t0) / iters;
    // 4) atomicXor no return
    t0 = clock64();
    for (int i = 0; i < iters; ++i) atomicXor(&a[(ln * 64 + i) & 4095], 1ull << 63);
    __syncthreads();
    t1 = clock64();
    if (ln == 0) out[3] = (t1 - t0) / iters;
    // 5) __syncthreads cost
    t0 = clock64();
    for (int i = 0; i < iters; ++i) __syncthreads();
    t1 = clock64();
    if (ln == 0) out[4] = (t1 - t0) / iters;
    // 6) 64-bit multiply-heavy ALU chain
    unsigned long long w = ln + 1;
    t0 = clock64();
    for (int i = 0; i < iters; ++i) w = w * 0x9E3779B97F4A7C15ull + (w >> 17);
    t1 = clock64();
    if (ln == 0) out[5] = (t1 - t0) / iters;
    if (ln == 0) out[6] = x + y + z + w;
    // 7) dependent flat load (generic pointer) chain on LDS
    unsigned long long* gp = a;
    unsigned long long v = ln;
    t0 = clock64();
    for (int i = 0; i < iters; ++i) v = gp[(v * 7 + 13) & 4095];
    t1 = clock64();
    if (ln == 0) out[7] = (t1 - t0) / iters + (v & 0);
}
int main() {
    unsigned long long* d; unsigned long long h[8];
    hipMalloc(&d, 64);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 1000);
        hipMemcpy(h, d, 64, hipMemcpyDeviceToHost);
    }
    printf("cycles/op: ds_read_b64 chain %llu, cas64 chain %llu, ballot chain %llu, xor-noret %llu, syncthreads %llu, mul64 chain %llu, flat chain %llu\n",
           h[0], h[1], h[2], h[3], h[4], h[5], h[7]);
    return 0;
}
