// rips_reduce_big.h -- serial reduction for large N (one 1024-thread workgroup
// per layer, working tables in HBM).  H1 normally runs on k_reduce_par
// (rips_reduce_par.h, many columns in flight); this kernel reduces H2 above
// N = 256 and is the fallback when k_reduce_par aborts on a capacity limit.
//
// Same algorithm as rips_reduce.h (Ripser's compute_pairs over Z/2 with stored
// reduced columns and implicit apparent columns), but the working coboundary
// can hold millions of live entries (torus N = 1024: 5.1 M), so the pivot is
// never found by a full scan.  Within one column the pivot never decreases
// (every column added has the current pivot as its minimum), which is exactly
// the access pattern of a RADIX HEAP: entries are referenced from 33 buckets
// keyed by the highest bit in which their f32 diameter bits differ from the
// last extracted pivot's; extract-min scans only the lowest non-empty bucket
// and redistributes it when it is not bucket 0.  Cancelled entries are dropped
// lazily (parity = bit 63 of the key log entry, as in the small-N kernel).
#pragma once
#include "rips_reduce.h"

namespace tda {

constexpr int kBigT = 1024;    // threads per layer
constexpr int kBigW = kBigT / 64;
constexpr int kNB = 33;        // radix buckets (f32 diameter bits)

struct BigBufs {
    uint64_t* log;       // [L][cap] keys (| kDead)
    uint64_t* index;     // [L][2 cap] bucketed index, entry = lo32 << 32 | pos + 1
    uint32_t* fill;      // [L][2 cap / 8]
    uint32_t* bref;      // [L][kNB][bcap] log positions per radix bucket
    uint64_t cap, bcap;
    uint64_t step_limit;  // pivots per column before giving up (exit guarantee)
    // wide H2 keys (N > 568: tetrahedron indices need up to 42 bits): the
    // diameter is replaced by its edge code (rank of the first occurrence of
    // the value among the layer's sorted edge lengths, k_edge_codes)
    const uint32_t* dcode;  // [L][N][N] edge codes, kCodeInf above the threshold
    const uint64_t* dsort;  // [L][ecap] sorted edge-length bits: dsort[code] = bits of the value
    uint64_t ecap;
    int wide;
};

// wide key = code << 42 | (2^42 - 1 - idx): 21-bit edge code (C(2048, 2) <
// 2^21), 42-bit inverted index, bit 63 stays free for kDead
constexpr int kWideIdxBits = 42;
constexpr uint64_t kWideIdxMask = (1ull << kWideIdxBits) - 1;
constexpr uint32_t kCodeInf = (1u << 21) - 1;

// ---- wide H2 keys: per-layer edge codes
// The f32 bits of each layer's C(N,2) edge lengths (row-major strict upper
// triangle), sorted ascending over the whole GPU: k_edge_keys writes them,
// k_edge_chunks sorts 16384-key chunks in LDS (bitonic, one 1024-thread block
// per chunk), then log2(C(N,2) / 16384) k_edge_merge passes double the sorted
// runs (merge path: every thread finds its first output's split by binary
// search and merges 16 outputs).  (r04-: one workgroup per layer sorted and
// merged everything: 70.6 ms at N = 2048, L = 1.)
constexpr int kEdgeSortLog2 = 14;
constexpr size_t kEdgeSortLds = size_t(8) << kEdgeSortLog2;
constexpr uint32_t kMergePer = 16;                 // outputs per thread of a merge pass
constexpr uint32_t kMergeSeg = 256 * kMergePer;    // outputs per block
__global__ __launch_bounds__(256) void k_edge_keys(const float* __restrict__ dist, int n, uint64_t* __restrict__ keys, uint64_t ecap) {
    const int l = blockIdx.y;
    const float* D = dist + (size_t)l * n * n;
    uint64_t* K = keys + (size_t)l * ecap;
    const uint32_t nn = (uint32_t)n * (uint32_t)n;
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < nn; q += gridDim.x * blockDim.x) {
        const uint32_t i = q / (uint32_t)n, j = q - i * (uint32_t)n;
        if (j > i) st_glb(K, (size_t)i * (2 * (size_t)n - i - 1) / 2 + (j - i - 1), (uint64_t)__float_as_uint(ld_glb(D, q)));
    }
}
__global__ __launch_bounds__(1024) void k_edge_chunks(uint64_t* __restrict__ keys, uint64_t E, uint64_t ecap) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t* sk = (uint64_t*)smem;
    const uint32_t t = threadIdx.x, T = blockDim.x;
    const uint64_t c0 = (uint64_t)blockIdx.x << kEdgeSortLog2;
    if (c0 >= E) return;
    uint64_t* K = keys + (size_t)blockIdx.y * ecap + c0;
    const uint32_t m = (uint32_t)min((uint64_t)1 << kEdgeSortLog2, E - c0);
    uint32_t p2 = 1;
    while (p2 < m) p2 <<= 1;
    for (uint32_t e = t; e < p2; e += T) sk[e] = e < m ? ld_glb(K, e) : kEmpty64;
    __syncthreads();
    for (uint32_t k = 2; k <= p2; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t e = t; e < p2; e += T) {
                const uint32_t x = e ^ j;
                if (x > e) {
                    const bool up = (e & k) == 0;
                    const uint64_t a = sk[e], b = sk[x];
                    if ((a > b) == up) {
                        sk[e] = b;
                        sk[x] = a;
                    }
                }
            }
            __syncthreads();
        }
    for (uint32_t e = t; e < m; e += T) st_glb(K, e, sk[e]);
}
// runs of width w (a power of two >= kMergePer) -> 2 w; every thread's kMergePer outputs lie in one pair of runs
__global__ __launch_bounds__(256) void k_edge_merge(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst, uint64_t E, uint64_t ecap,
                                                    uint64_t w) {
    const uint64_t o0 = (uint64_t)blockIdx.x * kMergeSeg + (uint64_t)threadIdx.x * kMergePer;
    if (o0 >= E) return;
    const uint64_t* S = src + (size_t)blockIdx.y * ecap;
    uint64_t* O = dst + (size_t)blockIdx.y * ecap;
    const uint64_t o1 = min(o0 + kMergePer, E);
    const uint64_t a0 = o0 / (2 * w) * (2 * w), a1 = min(a0 + w, E), b1 = min(a0 + 2 * w, E);
    const uint64_t la = a1 - a0, lb = b1 - a1, d0 = o0 - a0;
    // merge path: the first output's split (i from run A, d0 - i from run B)
    uint64_t lo = d0 > lb ? d0 - lb : 0, hi = min(d0, la);
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (ld_glb(S, a0 + mid) <= ld_glb(S, a1 + d0 - mid - 1))
            lo = mid + 1;
        else
            hi = mid;
    }
    uint64_t ia = lo, ib = d0 - lo;
    for (uint64_t o = o0; o < o1; ++o) {
        const bool takeA = ib >= lb || (ia < la && ld_glb(S, a0 + ia) <= ld_glb(S, a1 + ib));
        st_glb(O, o, takeA ? ld_glb(S, a0 + ia) : ld_glb(S, a1 + ib));
        if (takeA)
            ++ia;
        else
            ++ib;
    }
}

// k_edge_codes: code(i, j) = position of the first occurrence of d(i, j) in
// the sorted lengths (monotone in the value, equal values share a code, and
// dsort[code] gives the value back); kCodeInf above the layer's threshold.
__global__ __launch_bounds__(256) void k_edge_codes(const float* __restrict__ dist, int n, const LayerStats* __restrict__ stats,
                                                    const uint64_t* __restrict__ dsort, uint64_t ecap, uint32_t* __restrict__ dcode) {
    const int l = blockIdx.y;
    const float r = stats[l].thresh;
    const float* D = dist + (size_t)l * n * n;
    const uint64_t* S = dsort + (size_t)l * ecap;
    const uint64_t E = binom((uint64_t)n, 2);
    const uint32_t nn = (uint32_t)n * (uint32_t)n;
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < nn; q += gridDim.x * blockDim.x) {
        const uint32_t i = q / (uint32_t)n, j = q - i * (uint32_t)n;
        const float d = ld_glb(D, q);
        uint32_t c = 0;
        if (i != j) {
            c = kCodeInf;
            if (d <= r) {
                const uint64_t b = __float_as_uint(d);
                uint64_t lo = 0, hi = E;
                while (lo < hi) {
                    const uint64_t mid = (lo + hi) >> 1;
                    if (ld_glb(S, mid) < b)
                        lo = mid + 1;
                    else
                        hi = mid;
                }
                c = (uint32_t)lo;
            }
        }
        st_glb(dcode, (size_t)l * nn + q, c);
    }
}

struct BigShared {  // block-uniform state in LDS
    uint32_t cnt;           // log length
    uint32_t last;          // diameter bits of the last extracted pivot
    uint32_t nb[kNB];       // references per radix bucket
    uint64_t red[kBigW];    // per-wave partials
    uint64_t bc[8];         // broadcast slots
    int32_t err;
};

__device__ __forceinline__ int radix_bucket(uint32_t dbits, uint32_t last) {
    const uint32_t x = dbits ^ last;
    return x ? 32 - __builtin_clz(x) : 0;
}

// block-wide reductions (all threads call; result in every thread)
__device__ __forceinline__ uint64_t block_min_u64(uint64_t v, BigShared& S) {
    v = wave_min_u64(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) S.red[threadIdx.x >> 6] = v;
    __syncthreads();
    uint64_t m = S.red[0];
#pragma unroll
    for (int w = 1; w < kBigW; ++w) m = S.red[w] < m ? S.red[w] : m;
    return m;
}
__device__ __forceinline__ uint64_t block_sum_u64(uint64_t v, BigShared& S) {
    v = wave_sum_u64(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) S.red[threadIdx.x >> 6] = v;
    __syncthreads();
    uint64_t m = 0;
#pragma unroll
    for (int w = 0; w < kBigW; ++w) m += S.red[w];
    return m;
}
// exclusive prefix of `flag` over the block; returns offset, total in *tot
__device__ __forceinline__ uint32_t block_prefix(bool flag, BigShared& S, uint32_t* tot) {
    const uint64_t m = __ballot(flag);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) S.red[threadIdx.x >> 6] = (uint64_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0, all = 0;
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < kBigW; ++q) {
        const uint32_t c = (uint32_t)S.red[q];
        before += q < w ? c : 0;
        all += c;
    }
    *tot = all;
    return before + lanes_below(m);
}

struct BigHeap {
    uint64_t* log;
    uint64_t* index;
    uint32_t* fill;
    uint32_t* bref;  // [kNB][bcap]
    uint64_t cap, bcap;
    uint32_t imask;
    bool wide;  // fingerprints (low 32 key bits) are not unique: verify hits against the log
    BigShared* S;

    // append log position pos (key k) to its radix bucket; wave-aggregated
    __device__ __forceinline__ void push_ref(bool act, uint32_t pos, uint64_t k) {
        int b = act ? radix_bucket((uint32_t)(k >> 32), S->last) : -1;
        uint64_t rem = __ballot(act);
        while (rem) {
            const int src = __builtin_ctzll(rem);
            const int bb = __shfl(b, src, 64);
            const uint64_t m = __ballot(act && b == bb);
            uint32_t base = 0;
            if ((threadIdx.x & 63) == src) base = atomicAdd(&S->nb[bb], (uint32_t)__popcll(m));
            base = __shfl(base, src, 64);
            if (act && b == bb) {
                const uint64_t slot = base + lanes_below(m);
                if (slot < bcap)
                    bref[(size_t)bb * bcap + slot] = pos;
                else
                    S->err = 1;
            }
            rem &= ~m;
        }
    }

    // slot of the key logged at position pos in the bucketed index (exact
    // entry match, so fingerprints need not be unique)
    __device__ __forceinline__ uint32_t slot_of(uint32_t fp, uint32_t pos) const {
        const uint64_t want = ((uint64_t)fp << 32) | (pos + 1);
        uint32_t h = (mix32(fp) & (imask >> 3)) * 8;
        for (;;) {
            const uint64_t cur = index[h];
            if (cur == 0 || cur == want) return h;
            h = (h + 1) & imask;
        }
    }

    // Drop cancelled keys from the log: unindex everything, compact the live
    // keys in place (stable), re-index them and rebuild the radix buckets
    // relative to the current `last` (all threads; the buckets' reference
    // arrays double as scratch for the index slots).
    __device__ void compact() {
        __syncthreads();
        const uint32_t c = S->cnt < cap ? S->cnt : (uint32_t)cap;
        for (uint32_t e = threadIdx.x; e < c; e += kBigT) bref[e] = slot_of((uint32_t)log[e], e);
        __syncthreads();
        for (uint32_t e = threadIdx.x; e < c; e += kBigT) {
            const uint32_t h = bref[e];
            index[h] = 0;
            fill[h >> 3] = 0;
        }
        uint32_t w = 0;
        for (uint32_t e0 = 0; e0 < c; e0 += kBigT) {
            const uint32_t e = e0 + threadIdx.x;
            const uint64_t k = e < c ? log[e] : kEmpty64;
            const bool lv = k < kDead;
            uint32_t tot;
            const uint32_t off = block_prefix(lv, *S, &tot);  // barriers: the chunk has been read
            if (lv) log[w + off] = k;                         // w + off <= e
            w += tot;
        }
        __syncthreads();
        const uint32_t bmask = imask >> 3;
        for (uint32_t e = threadIdx.x; e < w; e += kBigT) {
            const uint32_t fp = (uint32_t)log[e];
            uint32_t bkt = mix32(fp) & bmask;
            for (;;) {
                const uint32_t slot = atomicAdd(&fill[bkt], 1u);
                if (slot < 8) {
                    index[bkt * 8 + slot] = ((uint64_t)fp << 32) | (e + 1);
                    break;
                }
                bkt = (bkt + 1) & bmask;
            }
        }
        if (threadIdx.x == 0) {
            for (int q = 0; q < kNB; ++q) S->nb[q] = 0;
            S->cnt = w;
        }
        __syncthreads();
        for (uint32_t e0 = 0; e0 < w; e0 += kBigT) {
            const uint32_t e = e0 + threadIdx.x;
            push_ref(e < w, e, e < w ? log[e] : 0);
        }
        __syncthreads();
    }

    // toggle DISTINCT keys (all threads call)
    __device__ void toggle_pass(uint64_t k, bool valid) {
        __syncthreads();
        if (S->cnt + kBigT > cap) {  // a pass adds at most kBigT keys
            compact();
            if (2ull * S->cnt + kBigT > cap && threadIdx.x == 0) S->err = 1;  // live set too large: retry bigger
        }
        const uint32_t fp = (uint32_t)k;
        const uint32_t bmask = imask >> 3;
        uint32_t bkt = mix32(fp) & bmask;
        bool pending = valid;
        for (uint32_t iter = 0; __syncthreads_or(pending); ++iter) {
            if (iter > bmask + 1) {  // every bucket probed: cannot happen while cnt <= cap
                if (threadIdx.x == 0) S->err = 1;
                break;
            }
            bool isnew = false, relive = false;
            uint32_t target = 0, epos = 0;
            if (pending) {
                const ulonglong2* bp = (const ulonglong2*)&index[(size_t)bkt * 8];
                const ulonglong2 q0 = bp[0], q1 = bp[1], q2 = bp[2], q3 = bp[3];
                const uint64_t e[8] = {q0.x, q0.y, q1.x, q1.y, q2.x, q2.y, q3.x, q3.y};
                uint64_t eh = 0;
                bool full = true;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    if (e[u] != 0 && (uint32_t)(e[u] >> 32) == fp && (!wide || (log[(uint32_t)e[u] - 1] & ~kDead) == k)) eh = e[u];
                    full &= e[u] != 0;
                }
                if (eh) {
                    epos = (uint32_t)eh - 1;
                    const uint64_t old = atomicXor((unsigned long long*)&log[epos], (unsigned long long)kDead);
                    relive = (old & kDead) != 0;  // dead -> live: needs a bucket reference again
                    pending = false;
                } else if (!full) {
                    const uint32_t slot = atomicAdd(&fill[bkt], 1u);
                    if (slot < 8) {
                        isnew = true;
                        target = bkt * 8 + slot;
                    } else {
                        bkt = (bkt + 1) & bmask;
                    }
                } else {
                    bkt = (bkt + 1) & bmask;
                }
            }
            uint32_t nnew;
            const uint32_t off = block_prefix(isnew, *S, &nnew);
            const uint32_t base = S->cnt;
            if (isnew) {
                const uint32_t pos = base + off;
                if (pos < cap) {
                    log[pos] = k;
                    index[target] = ((uint64_t)fp << 32) | (pos + 1);
                    epos = pos;
                } else {
                    S->err = 1;
                    isnew = false;
                }
                pending = false;
            }
            __syncthreads();
            if (threadIdx.x == 0) S->cnt = base + nnew < cap ? base + nnew : (uint32_t)cap;
            push_ref(isnew || relive, epos, k);
            __syncthreads();
        }
    }

    // extract the minimum live key (block-uniform result, kEmpty64 if none)
    __device__ uint64_t pop_min() {
        for (;;) {
            __syncthreads();
            int b = -1;
            for (int q = 0; q < kNB; ++q)
                if (S->nb[q]) {
                    b = q;
                    break;
                }
            if (b < 0) return kEmpty64;
            const uint32_t nref = S->nb[b];
            const uint64_t bcapl = bcap;
            uint64_t mn = kEmpty64;
            for (uint32_t e = threadIdx.x; e < nref && e < bcapl; e += kBigT) {
                const uint64_t k = log[bref[(size_t)b * bcap + e]];
                mn = k < mn ? k : mn;
            }
            mn = mn < kDead ? mn : kEmpty64;
            const uint64_t m = block_min_u64(mn, *S);
            if (m == kEmpty64) {  // only cancelled references left
                __syncthreads();
                if (threadIdx.x == 0) S->nb[b] = 0;
                continue;
            }
            if (b == 0) return m;
            // new last: redistribute bucket b (its live references) below b
            __syncthreads();
            if (threadIdx.x == 0) {
                S->last = (uint32_t)(m >> 32);
                S->nb[b] = 0;
            }
            __syncthreads();
            for (uint32_t e0 = 0; e0 < nref && e0 < bcapl; e0 += kBigT) {
                const uint32_t e = e0 + threadIdx.x;
                bool act = false;
                uint32_t pos = 0;
                uint64_t k = 0;
                if (e < nref && e < bcapl) {
                    pos = bref[(size_t)b * bcap + e];
                    k = log[pos];
                    act = k < kDead;
                }
                push_ref(act, pos, k);
            }
            __syncthreads();
            return m;
        }
    }

    // zero the index for the logged keys, buckets and length (all threads)
    __device__ void reset() {
        const uint32_t c = S->cnt;
        for (uint32_t e = threadIdx.x; e < c; e += kBigT)
            log[e] = (uint64_t)slot_of((uint32_t)log[e], e);  // stash the slot (the log is rebuilt anyway)
        __syncthreads();
        for (uint32_t e = threadIdx.x; e < c; e += kBigT) {
            const uint32_t h = (uint32_t)log[e];
            index[h] = 0;
            fill[h >> 3] = 0;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            S->cnt = 0;
            for (int q = 0; q < kNB; ++q) S->nb[q] = 0;
        }
        __syncthreads();
    }
};

// the oldest facet of the apparent cofacet pidx (its apparent column), with diameter
template <int DIM>
__device__ __forceinline__ float apparent_facet(const float* __restrict__ D, int n, uint64_t pidx, int (&fv)[DIM + 1]) {
    constexpr int NV = DIM + 2;
    int t[NV];
    decode<DIM + 1>(pidx, n, t);
    float fd = -1.0f;
    int fu = 0;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
        float d = 0.0f;
#pragma unroll
        for (int i = 0; i < NV; ++i)
#pragma unroll
            for (int k = i + 1; k < NV; ++k)
                if (i != u && k != u) d = fmaxf(d, ld_glb(D, (size_t)t[i] * n + t[k]));
        if (d > fd) {
            fd = d;
            fu = u;
        }
    }
#pragma unroll
    for (int u = 0; u < NV; ++u) {
        if (u != fu) continue;
#pragma unroll
        for (int i = 0, q = 0; i < NV; ++i)
            if (i != u) fv[q++] = t[i];
    }
    return fd;
}

template <int DIM>
__device__ void big_reduce_dim(const float* __restrict__ D, int n, float r, LayerStats* st, int l, const DimBufs& b,
                               const Reduce2Bufs& rb, const BigBufs& gb, BigShared& S, PivMap& map, const PivMap* prev,
                               Pair* __restrict__ pairs, uint64_t pcap) {
    constexpr int NV = DIM + 2;
    const int tid = threadIdx.x, ln = tid & 63;
    uint64_t nres = (uint64_t)st->n_residual[DIM];
    if (nres > b.rcap) nres = b.rcap;
    const uint64_t* resid = b.resid + (size_t)l * b.rcap;
    uint32_t* pivg = b.pivbits + (size_t)l * b.piv_words;
    uint64_t rcap2 = 16;
    while (rcap2 < 2 * nres + 16) rcap2 <<= 1;
    if (rcap2 > rb.rmap_stride) rcap2 = rb.rmap_stride;
    map.k = rb.rmap_keys + ((size_t)l * 2 + (DIM - 1)) * rb.rmap_stride;  // cleared by k_sort_resid
    map.v = rb.rmap_vals + ((size_t)l * 2 + (DIM - 1)) * rb.rmap_stride;
    map.mask = rcap2 - 1;
    map.lds = false;

    BigHeap H;
    H.log = gb.log + (size_t)l * gb.cap;
    H.index = gb.index + (size_t)l * 2 * gb.cap;
    H.fill = gb.fill + (size_t)l * (2 * gb.cap / 8);
    H.bref = gb.bref + (size_t)l * kNB * gb.bcap;
    H.cap = gb.cap;
    H.bcap = gb.bcap;
    H.imask = (uint32_t)(2 * gb.cap - 1);
    const bool wide = DIM == 2 && gb.wide;
    H.wide = wide;
    H.S = &S;
    const uint32_t* dcode = wide ? gb.dcode + (size_t)l * n * n : nullptr;
    const uint64_t* dsort = wide ? gb.dsort + (size_t)l * gb.ecap : nullptr;
    // edge code of a simplex (max over its edges; codes are monotone in the diameter)
    auto scode = [&](const int (&vs)[DIM + 1]) -> uint32_t {
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i <= DIM; ++i)
#pragma unroll
            for (int k = i + 1; k <= DIM; ++k) c = max(c, ld_glb(dcode, (size_t)vs[i] * n + vs[k]));
        return c;
    };
    const uint32_t* mst = rb.mst + (size_t)l * rb.mst_words;
    uint64_t* roff = rb.roff + (size_t)l * b.rcap;
    uint32_t* rlen = rb.rlen + (size_t)l * b.rcap;
    uint64_t* rpool = rb.rpool + (size_t)l * rb.rpool_cap;
    uint64_t rused = 0;
    Pair* P = pairs + (size_t)l * pcap;
    uint64_t cs = 0, npairs = 0, nadds = 0, nskip = 0;
#ifdef TDA_PROFILE
    // cob0, pop_min, owner adds, apparent adds, store R_j, reset, (owner adds << 40 | owner entries), total
    uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint64_t t_all = clock64();
#endif
    if (tid == 0) {
        S.cnt = 0;
        S.err = 0;
        for (int q = 0; q < kNB; ++q) S.nb[q] = 0;
    }
    __syncthreads();

    // toggle the coboundary of vs (diam sd, wide: edge code sc) -- one thread per new vertex
    auto cob = [&](const int (&vs)[DIM + 1], float sd, uint32_t sc) {
        for (int v0 = 0; v0 < n; v0 += kBigT) {
            const int v = v0 + tid;
            bool ok = v < n;
#pragma unroll
            for (int i = 0; i <= DIM; ++i) ok &= (vs[i] != v);
            uint64_t key = 0;
            if (ok && wide) {
                uint32_t cc = sc;
#pragma unroll
                for (int i = 0; i <= DIM; ++i) cc = max(cc, ld_glb(dcode, (size_t)vs[i] * n + v));
                ok = cc < kCodeInf;
                key = ((uint64_t)cc << kWideIdxBits) | (kWideIdxMask - cofacet_index<DIM>(vs, v));
            } else if (ok) {
                float cd = sd;
#pragma unroll
                for (int i = 0; i <= DIM; ++i) cd = fmaxf(cd, ld_glb(D, (size_t)vs[i] * n + v));
                ok = cd <= r;
                key = filt_key(cd, cofacet_index<DIM>(vs, v));
            }
            H.toggle_pass(key, ok);
        }
    };

    for (uint64_t j = 0; j < nres; ++j) {
        __syncthreads();
        if (S.err) break;
        const uint64_t key = ld_glb(resid, j);
        const uint64_t sidx = key_idx(key);
        const float sdm = key_diam(key);
        int vs[DIM + 1];
        decode<DIM>(sidx, n, vs);
        bool cleared;
        if (DIM == 1) {
            cleared = (ld_glb(mst, sidx >> 5) >> (sidx & 31)) & 1u;
        } else {
            // every wave probes; the result is the same in all of them
            cleared = prev->find((uint32_t)encode<DIM>(vs), ln) >= 0;
        }
        if (cleared) {
            ++nskip;
            if (tid == 0) rlen[j] = 0;
            continue;
        }
        const uint32_t sc = wide ? scode(vs) : 0u;
        if (tid == 0) S.last = wide ? (uint32_t)(((uint64_t)sc << kWideIdxBits) >> 32) : __float_as_uint(sdm + 0.0f);
        __syncthreads();
        TDA_STAMP(t_c0);
        cob(vs, sdm, sc);
        TDA_ACC(0, t_c0);
        for (uint64_t step = 0;; ++step) {
            TDA_STAMP(t_p0);
            const uint64_t pk = H.pop_min();
            TDA_ACC(1, t_p0);
            if (step >= gb.step_limit) {
                if (tid == 0) {
                    printf("k_reduce_big: layer %d dim %d column %llu (idx %llu) step limit: pivot %016llx cnt %u last %08x\n", l,
                           DIM, (unsigned long long)j, (unsigned long long)sidx, (unsigned long long)pk, S.cnt, S.last);
                    S.err = 3;
                }
                __syncthreads();
            }
            if (S.err) break;
            if (pk == kEmpty64) {
                if (tid == 0) {
                    uint64_t pos = atomicAdd((unsigned long long*)&st->count[DIM], 1ull);
                    if (pos < pcap)
                        P[pos] = Pair{sdm, INFINITY, (int64_t)sidx, -1};
                    else
                        atomicOr(&st->err, ERR_PAIR_CAP);
                    rlen[j] = 0;
                }
                break;
            }
            const uint64_t pidx = wide ? kWideIdxMask - (pk & kWideIdxMask) : 0xFFFFFFFFull - (pk & 0xFFFFFFFFull);
            const float pd = wide ? __uint_as_float((uint32_t)ld_glb(dsort, pk >> kWideIdxBits)) : __uint_as_float((uint32_t)(pk >> 32));
            const bool app = (ld_glb((const uint32_t*)pivg, pidx >> 5) >> (pidx & 31)) & 1u;
            const int64_t owner = !app ? -1 : wide ? map.find64(pidx, ln) : map.find((uint32_t)pidx, ln);
            TDA_STAMP(t_a0);
            if (owner >= 0) {
                const uint64_t o0 = ld_glb((const uint64_t*)roff, owner);
                const uint32_t ol = ld_glb((const uint32_t*)rlen, owner);
                for (uint32_t e0 = 0; e0 < ol; e0 += kBigT) {
                    const uint32_t e = e0 + tid;
                    H.toggle_pass(e < ol ? ld_glb((const uint64_t*)rpool, o0 + e) : 0, e < ol);
                }
                ++nadds;
                TDA_ACC(2, t_a0);
#ifdef TDA_PROFILE
                prof[6] += (1ull << 40) + ol;
#endif
            } else if (app) {
                int fv[DIM + 1];
                const float fd = apparent_facet<DIM>(D, n, pidx, fv);
                cob(fv, fd, wide ? scode(fv) : 0u);
                ++nadds;
                TDA_ACC(3, t_a0);
            } else {
                __syncthreads();  // all waves decided before tid 0 publishes the pivot (a lagging wave would see its own column as the owner)
                if (tid == 0) {
                    if (pd > sdm) {
                        uint64_t pos = atomicAdd((unsigned long long*)&st->count[DIM], 1ull);
                        if (pos < pcap)
                            P[pos] = Pair{sdm, pd, (int64_t)sidx, (int64_t)pidx};
                        else
                            atomicOr(&st->err, ERR_PAIR_CAP);
                    }
                    if (wide)
                        map.insert64(pidx, (uint32_t)j);
                    else
                        map.insert((uint32_t)pidx, (uint32_t)j);
                    atomicOr(&pivg[pidx >> 5], 1u << (pidx & 31));
                }
                cs += pair_hash(sidx, pidx);
                npairs += 1;
                // R_j = live log entries
                const uint32_t c = S.cnt;
                uint64_t wr = 0;
                for (uint32_t e0 = 0; e0 < c; e0 += kBigT) {
                    const uint32_t e = e0 + tid;
                    const uint64_t k = e < c ? H.log[e] : kEmpty64;
                    const bool lv = k < kDead;
                    uint32_t tot;
                    const uint32_t off = block_prefix(lv, S, &tot);
                    if (lv && rused + wr + off < rb.rpool_cap) rpool[rused + wr + off] = k;
                    wr += tot;
                }
                if (rused + wr > rb.rpool_cap) {
                    if (tid == 0) S.err = 2;
                    wr = 0;
                }
                if (tid == 0) {
                    roff[j] = rused;
                    rlen[j] = (uint32_t)wr;
                }
                rused += wr;
                TDA_ACC(4, t_a0);
                break;
            }
        }
        __syncthreads();
        TDA_STAMP(t_r0);
        H.reset();
        TDA_ACC(5, t_r0);
    }
    __syncthreads();
    if (tid == 0) {
        if (S.err == 1) atomicOr(&st->err, ERR_WORK_CAP);
        if (S.err == 2) atomicOr(&st->err, ERR_VPOOL_CAP);
        if (S.err == 3) atomicOr(&st->err, ERR_STEP_LIMIT);
        atomicAdd((unsigned long long*)&st->checksum[DIM], (unsigned long long)cs);
        atomicAdd((unsigned long long*)&st->all_pairs[DIM], (unsigned long long)npairs);
        atomicAdd((unsigned long long*)&st->n_adds[DIM], (unsigned long long)nadds);
        atomicAdd((unsigned long long*)&st->n_columns[DIM], (unsigned long long)(0ull - nskip));
        st->nskip[DIM] = nskip;
#ifdef TDA_PROFILE
        prof[7] = clock64() - t_all;
        for (int i = 0; i < 8; ++i) st->prof[DIM][i] = prof[i];
#endif
    }
    __syncthreads();
}

// Large-N serial reductions: one 1024-thread workgroup per layer, H1 then H2.
// start_dim 2: H1 was reduced by k_reduce_par (rips_reduce_par.h), whose
// k_par_emit left the H1 residual pivots in the dim-1 map that H2 clears with.
__global__ __launch_bounds__(kBigT) void k_reduce_big(const float* __restrict__ dist, int n, int maxdim,
                                                       LayerStats* __restrict__ stats, DimBufs b1, DimBufs b2, Reduce2Bufs rb,
                                                       BigBufs gb, Pair* __restrict__ pairs1, Pair* __restrict__ pairs2,
                                                       uint64_t pcap1, uint64_t pcap2, int start_dim) {
    __shared__ BigShared S;
    const int l = blockIdx.x;
    LayerStats* st = stats + l;
    const float r = st->thresh;
    const float* D = dist + (size_t)l * n * n;
    PivMap m1, m2;
    if (start_dim <= 1) {
        big_reduce_dim<1>(D, n, r, st, l, b1, rb, gb, S, m1, nullptr, pairs1, pcap1);
    } else {  // the map k_par_emit filled (same region and mask rule as big_reduce_dim<1>)
        uint64_t nres = (uint64_t)st->n_residual[1];
        if (nres > b1.rcap) nres = b1.rcap;
        uint64_t rc2 = 16;
        while (rc2 < 2 * nres + 16) rc2 <<= 1;
        if (rc2 > rb.rmap_stride) rc2 = rb.rmap_stride;
        m1.k = rb.rmap_keys + ((size_t)l * 2 + 0) * rb.rmap_stride;
        m1.v = rb.rmap_vals + ((size_t)l * 2 + 0) * rb.rmap_stride;
        m1.mask = rc2 - 1;
        m1.lds = false;
    }
    if (maxdim >= 2) big_reduce_dim<2>(D, n, r, st, l, b2, rb, gb, S, m2, &m1, pairs2, pcap2);
}

}  // namespace tda
