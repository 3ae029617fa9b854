// rips_device.h -- device-side helpers shared by the gfx950 Vietoris-Rips kernels.
//
// Simplex indexing follows the combinatorial number system that the
// reference's `ripser` core uses [upstream ripser.cpp: get_simplex_vertices /
// simplex_coboundary_enumerator]: a k-simplex with vertices v_k > ... > v_0
// has index sum_i C(v_i, i+1).  Filtration order (the total order that fixes
// every persistence pair) is (diameter asc, index desc); column order is its
// reverse (diameter desc, index asc).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tda {

constexpr uint64_t kEmpty64 = 0xFFFFFFFFFFFFFFFFull;

// ---------------------------------------------------------------- binomials
// C(n, k) for k <= 5 without 64-bit division: 32-bit exact-division steps
// (C(n,k) = C(n,k-1) * (n-k+1) / k, split so every quotient is exact) and one
// 32x32->64 multiply at the end.  Valid for n < 65536 (checked on the host).
__host__ __device__ __forceinline__ uint64_t binom(uint64_t n64, int k) {
    const uint32_t n = (uint32_t)n64;
    if (k == 0) return 1;
    if (n < (uint32_t)k) return 0;
    if (k == 1) return n;
    const uint32_t c2 = (n & 1) ? n * ((n - 1) >> 1) : (n >> 1) * (n - 1);  // < 2^31 for n < 65536
    if (k == 2) return c2;
    // C3 = c2 * (n-2) / 3, c2 = 3q + r
    const uint32_t q2 = c2 / 3u, r2 = c2 - 3u * q2;
    const uint64_t c3 = (uint64_t)q2 * (n - 2) + (r2 * (n - 2)) / 3u;
    if (k == 3) return c3;
    const uint64_t c4 = (c3 >> 2) * (n - 3) + ((uint32_t)(c3 & 3) * (n - 3)) / 4u;
    if (k == 4) return c4;
    const uint64_t q4 = c4 / 5u, r4 = c4 - 5u * q4;
    return q4 * (n - 4) + (r4 * (n - 4)) / 5u;
}

// largest v in [k-1, top] with C(v, k) <= idx.  The estimate is f32 hardware
// math (sqrt / exp2-log2 cube root, within a vertex or two of the answer);
// the integer walks below make the result exact.
__device__ __forceinline__ int max_vertex(uint64_t idx, int k, int top) {
    if (k == 1) return (int)(idx < (uint64_t)top ? idx : (uint64_t)top);
    float g;
    const float x = (float)idx;
    if (k == 2)
        g = 0.5f * (1.0f + __fsqrt_rn(1.0f + 8.0f * x));
    else if (k == 3)
        g = (x > 0.0f ? __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(6.0f * x) * (1.0f / 3.0f)) : 0.0f) + 1.0f;
    else
        g = __fsqrt_rn(__fsqrt_rn(24.0f * x)) + 1.5f;
    int v = (int)g;
    if (v > top) v = top;
    if (v < k - 1) v = k - 1;
    while (v > k - 1 && binom((uint64_t)v, k) > idx) --v;
    while (v < top && binom((uint64_t)(v + 1), k) <= idx) ++v;
    return v;
}

// 32-bit binomials for small vertex counts (N <= 64: C(N, 3) < 2^16)
__device__ __forceinline__ uint32_t c2u(uint32_t x) { return x * (x - 1) / 2; }
__device__ __forceinline__ uint32_t c3u(uint32_t x) { return x * (x - 1) * (x - 2) / 6; }

// index -> vertices, descending (vs[0] largest), DIM+1 vertices
template <int DIM>
__device__ __forceinline__ void decode(uint64_t idx, int n, int (&vs)[DIM + 1]) {
    int top = n - 1;
#pragma unroll
    for (int k = DIM + 1; k >= 1; --k) {
        int v = max_vertex(idx, k, top);
        vs[DIM + 1 - k] = v;
        idx -= binom((uint64_t)v, k);
        top = v - 1;
    }
}

template <int DIM>
__device__ __forceinline__ uint64_t encode(const int (&vs)[DIM + 1]) {
    uint64_t idx = 0;
#pragma unroll
    for (int i = 0; i <= DIM; ++i) idx += binom((uint64_t)vs[i], DIM + 1 - i);
    return idx;
}

// index of sigma u {v} (v not in sigma), sigma descending
template <int DIM>
__device__ __forceinline__ uint64_t cofacet_index(const int (&vs)[DIM + 1], int v) {
    uint64_t idx = 0;
    int pos = DIM + 2;  // binomial order of the next vertex written (descending)
    bool placed = false;
#pragma unroll
    for (int i = 0; i <= DIM; ++i) {
        if (!placed && v > vs[i]) {
            idx += binom((uint64_t)v, pos--);
            placed = true;
        }
        idx += binom((uint64_t)vs[i], pos--);
    }
    if (!placed) idx += binom((uint64_t)v, 1);
    return idx;
}

template <int DIM>
__device__ __forceinline__ float simplex_diam(const float* __restrict__ D, int n, const int (&vs)[DIM + 1]) {
    float d = 0.0f;
#pragma unroll
    for (int i = 0; i <= DIM; ++i)
#pragma unroll
        for (int j = i + 1; j <= DIM; ++j) d = fmaxf(d, D[(size_t)vs[i] * n + vs[j]]);
    return d;
}

// ---------------------------------------------------------------- sqrt
// Correctly rounded f32 sqrt, independent of the accuracy of the hardware
// sqrt: start from the f64 sqrt rounded to f32 (within 1 ulp) and fix the
// rounding with exact midpoint tests (a 25-bit midpoint squares exactly in
// f64; sqrt of a float never lands on a midpoint).  numpy's np.sqrt on f32
// (sklearn pairwise.py:441) is correctly rounded.
__device__ __forceinline__ float sqrt_rn_f32(float x) {
    if (!(x > 0.0f) || isinf(x)) return x == 0.0f ? 0.0f : (x > 0.0f ? x : __builtin_nanf(""));
    float f = (float)__builtin_sqrt((double)x);
    const double xd = (double)x;
    const float up = __uint_as_float(__float_as_uint(f) + 1u);  // f > 0 finite
    const double mu = 0.5 * ((double)f + (double)up);
    if (mu * mu <= xd) return up;
    const float dn = __uint_as_float(__float_as_uint(f) - 1u);
    const double md = 0.5 * ((double)f + (double)dn);
    if (md * md > xd) return dn;
    return f;
}

// ---------------------------------------------------------------- address spaces
// Pointers kept in structs lose their address space and become FLAT accesses
// (slower, and they tie up both vmcnt and lgkmcnt); hot loops re-type them.
#define TDA_LDS __attribute__((address_space(3)))
#define TDA_GLB __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ T ld_lds(const T* p, size_t i) { return ((const TDA_LDS T*)p)[i]; }
template <typename T>
__device__ __forceinline__ T ld_glb(const T* p, size_t i) { return ((const TDA_GLB T*)p)[i]; }
template <typename T>
__device__ __forceinline__ void st_lds(T* p, size_t i, T v) { ((TDA_LDS T*)p)[i] = v; }
template <typename T>
__device__ __forceinline__ void st_glb(T* p, size_t i, T v) { ((TDA_GLB T*)p)[i] = v; }
// address-space-typed access chosen at compile time (LDS = true: local)
template <bool LDS, typename T>
__device__ __forceinline__ T mld(const T* p, size_t i) {
    if constexpr (LDS) return ((const TDA_LDS T*)p)[i];
    else return ((const TDA_GLB T*)p)[i];
}
template <bool LDS, typename T>
__device__ __forceinline__ void mst(T* p, size_t i, T v) {
    if constexpr (LDS) ((TDA_LDS T*)p)[i] = v;
    else ((TDA_GLB T*)p)[i] = v;
}
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
template <bool LDS>
__device__ __forceinline__ u64x2 mld2(const uint64_t* p, size_t i) {  // 16-B load of p[i], p[i + 1]
    if constexpr (LDS) return *(const TDA_LDS u64x2*)((const TDA_LDS uint64_t*)p + i);
    else return *(const TDA_GLB u64x2*)((const TDA_GLB uint64_t*)p + i);
}
template <bool LDS, typename T>
__device__ __forceinline__ T matomic_add(T* p, T v) {
    if constexpr (LDS) return __hip_atomic_fetch_add((TDA_LDS T*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else return __hip_atomic_fetch_add((TDA_GLB T*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <bool LDS, typename T>
__device__ __forceinline__ void matomic_xor(T* p, T v) {
    if constexpr (LDS) __hip_atomic_fetch_xor((TDA_LDS T*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else __hip_atomic_fetch_xor((TDA_GLB T*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <bool LDS, typename T>
__device__ __forceinline__ T matomic_cas(T* p, T cmp, T v) {  // returns the old value
    if constexpr (LDS)
        __hip_atomic_compare_exchange_strong((TDA_LDS T*)p, &cmp, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else
        __hip_atomic_compare_exchange_strong((TDA_GLB T*)p, &cmp, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return cmp;
}
template <bool LDS, typename T>
__device__ __forceinline__ void matomic_min(T* p, T v) {
    if constexpr (LDS) __hip_atomic_fetch_min((TDA_LDS T*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else __hip_atomic_fetch_min((TDA_GLB T*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <bool LDS, typename T>
__device__ __forceinline__ void matomic_or(T* p, T v) {
    if constexpr (LDS) __hip_atomic_fetch_or((TDA_LDS T*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else __hip_atomic_fetch_or((TDA_GLB T*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- staging
// Copy nbytes (multiple of 4) global -> LDS with 16-B loads, 8 in flight per
// lane before the first LDS store (a single wave otherwise serialises one
// HBM/L2 round trip per 64 elements).
__device__ __forceinline__ void stage_to_lds(void* dst, const void* src, size_t nbytes, int t, int T) {
    // native vector type: HIP's uint4 class defeats register promotion and
    // sends the in-flight array through scratch
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const size_t n16 = (((uintptr_t)src | (uintptr_t)dst) & 15) ? 0 : nbytes / 16;
    const TDA_GLB v4u* s4 = (const TDA_GLB v4u*)src;
    TDA_LDS v4u* d4 = (TDA_LDS v4u*)dst;
    size_t e = t;
    for (; e + 7 * (size_t)T < n16; e += 8 * (size_t)T) {
        v4u r0 = s4[e], r1 = s4[e + T], r2 = s4[e + 2 * (size_t)T], r3 = s4[e + 3 * (size_t)T];
        v4u r4 = s4[e + 4 * (size_t)T], r5 = s4[e + 5 * (size_t)T], r6 = s4[e + 6 * (size_t)T], r7 = s4[e + 7 * (size_t)T];
        d4[e] = r0;
        d4[e + T] = r1;
        d4[e + 2 * (size_t)T] = r2;
        d4[e + 3 * (size_t)T] = r3;
        d4[e + 4 * (size_t)T] = r4;
        d4[e + 5 * (size_t)T] = r5;
        d4[e + 6 * (size_t)T] = r6;
        d4[e + 7 * (size_t)T] = r7;
    }
    for (; e < n16; e += T) d4[e] = s4[e];
    const TDA_GLB uint32_t* s1 = (const TDA_GLB uint32_t*)src;
    TDA_LDS uint32_t* d1 = (TDA_LDS uint32_t*)dst;
    size_t w = n16 * 4 + t;
    for (; w + 7 * (size_t)T < nbytes / 4; w += 8 * (size_t)T) {
        uint32_t r0 = s1[w], r1 = s1[w + T], r2 = s1[w + 2 * (size_t)T], r3 = s1[w + 3 * (size_t)T];
        uint32_t r4 = s1[w + 4 * (size_t)T], r5 = s1[w + 5 * (size_t)T], r6 = s1[w + 6 * (size_t)T], r7 = s1[w + 7 * (size_t)T];
        d1[w] = r0;
        d1[w + T] = r1;
        d1[w + 2 * (size_t)T] = r2;
        d1[w + 3 * (size_t)T] = r3;
        d1[w + 4 * (size_t)T] = r4;
        d1[w + 5 * (size_t)T] = r5;
        d1[w + 6 * (size_t)T] = r6;
        d1[w + 7 * (size_t)T] = r7;
    }
    for (; w < nbytes / 4; w += T) d1[w] = s1[w];
}

// ---------------------------------------------------------------- hashing
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}
// cheap 32-bit mixer for hash-table slots (keys' low 32 bits are unique)
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
// order-free pair hash; the CPU checker under oracle/ uses the same definition
__host__ __device__ __forceinline__ uint64_t pair_hash(uint64_t s, uint64_t t) {
    return mix64(s * 0x9E3779B97F4A7C15ull ^ mix64(t + 0x632BE59BD9B4E019ull));
}

// column key: ascending u64 order == column order (diam desc, idx asc)
__host__ __device__ __forceinline__ uint64_t col_key(float diam, uint64_t idx) {
    uint32_t b = __float_as_uint(diam + 0.0f);
    return ((uint64_t)(0xFFFFFFFFu - b) << 32) | (idx & 0xFFFFFFFFull);
}
__host__ __device__ __forceinline__ float key_diam(uint64_t key) { return __uint_as_float(0xFFFFFFFFu - (uint32_t)(key >> 32)); }
__host__ __device__ __forceinline__ uint64_t key_idx(uint64_t key) { return key & 0xFFFFFFFFull; }
// edge key in filtration order (diam asc, idx desc) for the H0 spanning forest
__host__ __device__ __forceinline__ uint64_t filt_key(float diam, uint64_t idx) {
    return ((uint64_t)__float_as_uint(diam + 0.0f) << 32) | (0xFFFFFFFFull - (idx & 0xFFFFFFFFull));
}

// ---------------------------------------------------------------- wave ops
// Synchronisation of ONE wave's lanes through memory (LDS and global): waits
// for the wave's outstanding memory operations and fences the compiler, but
// issues no s_barrier, so waves of one workgroup can run independent loops.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}
// compiler-only ordering of one wave's LDS traffic: LDS instructions of a
// wave execute in program order, so no wait is needed between steps
__device__ __forceinline__ void lds_order() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ int lane_id() { return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    uint32_t lo = __shfl_xor((unsigned)(uint32_t)v, m, 64);
    uint32_t hi = __shfl_xor((unsigned)(uint32_t)(v >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
    uint32_t lo = __shfl((unsigned)(uint32_t)v, src, 64);
    uint32_t hi = __shfl((unsigned)(uint32_t)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}
// Wave-64 reductions with DPP (row_shr 1/2/4/8 + row_bcast15/31, the
// GFX9 scan pattern) instead of ds_bpermute shuffles: ~6 VALU steps, no LDS
// round trips.  Call with the whole wave active; every lane gets the result.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp32(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROWMASK, 0xf, false);
}
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint64_t dpp64(uint64_t old, uint64_t v) {
    uint32_t lo = dpp32<CTRL, ROWMASK>((uint32_t)old, (uint32_t)v);
    uint32_t hi = dpp32<CTRL, ROWMASK>((uint32_t)(old >> 32), (uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t readlane63_u64(uint64_t v) {
    uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, 63);
    uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
    return ((uint64_t)hi << 32) | lo;
}
#define TDA_WAVE_REDUCE64(OP, ID)                     \
    v = OP(v, dpp64<0x111, 0xf>(ID, v));              \
    v = OP(v, dpp64<0x112, 0xf>(ID, v));              \
    v = OP(v, dpp64<0x114, 0xf>(ID, v));              \
    v = OP(v, dpp64<0x118, 0xf>(ID, v));              \
    v = OP(v, dpp64<0x142, 0xa>(ID, v));              \
    v = OP(v, dpp64<0x143, 0xc>(ID, v));              \
    return readlane63_u64(v);

__device__ __forceinline__ uint64_t op_min64(uint64_t a, uint64_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint64_t op_max64(uint64_t a, uint64_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint64_t op_add64(uint64_t a, uint64_t b) { return a + b; }
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) { TDA_WAVE_REDUCE64(op_add64, 0ull) }
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) { TDA_WAVE_REDUCE64(op_min64, ~0ull) }
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) { TDA_WAVE_REDUCE64(op_max64, 0ull) }
#undef TDA_WAVE_REDUCE64
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    v = max(v, dpp32<0x111, 0xf>(0u, v));
    v = max(v, dpp32<0x112, 0xf>(0u, v));
    v = max(v, dpp32<0x114, 0xf>(0u, v));
    v = max(v, dpp32<0x118, 0xf>(0u, v));
    v = max(v, dpp32<0x142, 0xa>(0u, v));
    v = max(v, dpp32<0x143, 0xc>(0u, v));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = min(v, dpp32<0x111, 0xf>(~0u, v));
    v = min(v, dpp32<0x112, 0xf>(~0u, v));
    v = min(v, dpp32<0x114, 0xf>(~0u, v));
    v = min(v, dpp32<0x118, 0xf>(~0u, v));
    v = min(v, dpp32<0x142, 0xa>(~0u, v));
    v = min(v, dpp32<0x143, 0xc>(~0u, v));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

}  // namespace tda
