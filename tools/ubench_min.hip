// Micro-benchmark of k_reduce_par's front minimum (dev aid, r05): one
// 512-thread workgroup, a 4096-slot u64 toggle table in LDS with ~750 live
// keys and tombstones, one minimum per iteration behind a barrier (as in the
// step loop), a slot changed between iterations.  Prints s_memtime cycles per
// minimum for each variant:
//   0  per thread 8 slots (2 x u64 reads), DPP u64 wave minimum, per-wave LDS
//      slots, barrier, 8 reads (k_reduce_par's front_min)
//   1  as 0, wave minimum as two u32 passes (hi word, then lo among equal hi)
//   2  as 0, cross-wave minimum by an LDS u64 atomic min into a
//      double-buffered cell (one read after the barrier)
//   3  1 + 2
//   4  as 3, thread-local minimum on the hi words first
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o ubench_min tools/ubench_min.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../tda-multimodal_amd/csrc/rips_device.h"

using namespace tda;

constexpr int T = 512, W = T / 64, SLOTS = 4096, PER = SLOTS / T;
constexpr uint64_t EMPTY = ~0ull, TOMB = ~0ull - 1, DEAD = 1ull << 63;

struct Lds {
    uint64_t tab[SLOTS];
    uint64_t red[2][W];
    uint64_t cell[2];
};

__device__ __forceinline__ void bar() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ uint32_t now() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const uint32_t c = (uint32_t)__builtin_amdgcn_s_memtime();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    return c;
}
__device__ __forceinline__ uint64_t wave_min_2p(uint64_t v) {
    const uint32_t h = wave_min_u32((uint32_t)(v >> 32));
    const uint32_t l = wave_min_u32((uint32_t)(v >> 32) == h ? (uint32_t)v : ~0u);
    return ((uint64_t)h << 32) | l;
}

template <int V>
__device__ __forceinline__ uint64_t front_min(Lds& S, uint32_t& par) {
    uint64_t b = EMPTY;
    if (V == 4) {
        uint64_t x[PER];
#pragma unroll
        for (int q = 0; q < PER; q += 2) {
            const uint32_t e = q * T + 2 * threadIdx.x;
            x[q] = S.tab[e];
            x[q + 1] = S.tab[e + 1];
        }
        uint32_t h = ~0u;
#pragma unroll
        for (int q = 0; q < PER; ++q) h = min(h, (uint32_t)(x[q] >> 32));
        uint32_t lo = ~0u;
#pragma unroll
        for (int q = 0; q < PER; ++q) lo = (uint32_t)(x[q] >> 32) == h ? min(lo, (uint32_t)x[q]) : lo;
        b = ((uint64_t)h << 32) | lo;
    } else {
#pragma unroll
        for (int q = 0; q < PER; q += 2) {
            const uint32_t e = q * T + 2 * threadIdx.x;
            const uint64_t x = S.tab[e], y = S.tab[e + 1];
            b = x < b ? x : b;
            b = y < b ? y : b;
        }
    }
    b = b < DEAD ? b : EMPTY;
    const uint64_t w = (V == 1 || V == 3 || V == 4) ? wave_min_2p(b) : wave_min_u64(b);
    const uint32_t pb = par++ & 1;
    if (V >= 2) {
        if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_min((TDA_LDS unsigned long long*)&S.cell[pb], (unsigned long long)w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (threadIdx.x == 0) S.cell[pb ^ 1] = EMPTY;  // read two barriers ago; next written after the next barrier
        bar();
        return S.cell[pb];
    }
    if ((threadIdx.x & 63) == 0) S.red[pb][threadIdx.x >> 6] = w;
    bar();
    uint64_t m = S.red[pb][0];
#pragma unroll
    for (int i = 1; i < W; ++i) m = S.red[pb][i] < m ? S.red[pb][i] : m;
    return m;
}

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

template <int V>
__global__ __launch_bounds__(T) void k_bench(int iters, uint64_t* out, uint32_t* cyc) {
    __shared__ Lds S;
    const uint32_t t = threadIdx.x;
    for (uint32_t e = t; e < SLOTS; e += T) {
        const uint64_t r = mix(e * 7919ull + 1);
        const uint32_t u = (uint32_t)(r % 100);
        S.tab[e] = u < 18 ? ((r >> 8) & 0x3FFFFFFFFFFFull) : u < 33 ? TOMB : EMPTY;
    }
    if (t < 2) S.cell[t] = EMPTY;
    __syncthreads();
    uint32_t par = 0, acc = 0;
    uint64_t chk = 0;
    for (int it = 0; it < iters; ++it) {
        bar();
        const uint32_t t0 = now();
        const uint64_t m = front_min<V>(S, par);
        asm volatile("" : : "v"(m));
        const uint32_t t1 = now();
        acc += t1 - t0;
        chk += m;
        bar();
        if (t == 0) {  // remove one random live-ish slot, insert a key into another
            const uint64_t r = mix(it + 12345ull);
            S.tab[r & (SLOTS - 1)] = TOMB;
            S.tab[(r >> 12) & (SLOTS - 1)] = (r >> 20) & 0x3FFFFFFFFFFFull;
        }
    }
    if ((t & 63) == 0) cyc[t >> 6] = acc;
    if (t == 0) *out = chk;
}

template <int V>
void run(int iters, uint64_t* out, uint32_t* cyc) {
    hipLaunchKernelGGL(k_bench<V>, dim3(1), dim3(T), 0, 0, iters, out, cyc);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k_bench<V>, dim3(1), dim3(T), 0, 0, iters, out, cyc);
    uint32_t h[W];
    uint64_t c;
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    hipMemcpy(&c, out, 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < W; ++i) s += h[i];
    printf("variant %d: %.0f cycles per minimum (wave 0 %.0f), checksum %llx\n", V, s / W / iters, (double)h[0] / iters, (unsigned long long)c);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    uint64_t* out;
    uint32_t* cyc;
    hipMalloc(&out, 8);
    hipMalloc(&cyc, 4 * W);
    run<0>(iters, out, cyc);
    run<1>(iters, out, cyc);
    run<2>(iters, out, cyc);
    run<3>(iters, out, cyc);
    run<4>(iters, out, cyc);
    run<0>(iters, out, cyc);
    return 0;
}
