// rips_reduce_small.h -- serial reductions for N <= 64 (the 48-point sweep),
// laid out around where the additions actually are.  A Python model of the
// reduction (tools/phase_sim.py) over the 32-layer sweep shows:
//   * H1: a layer has <= 8 residual columns, but ONE of them can need ~170
//     apparent additions in a row (layer 25: 168 of the layer's 173).  That
//     chain is the critical path of the whole batch, so its per-addition cost
//     is what matters.  The working column W is a dense LDS bitmap over the
//     triangles in FILTRATION order (k_h1_prep ranks them), so the pivot is
//     simply the first set bit: every lane tests its 32*K-bit slice, one
//     ballot picks the first non-empty slice.  A toggle is one fire-and-forget
//     ds_xor at the triangle's rank, a stored reduced column R_j is a copy of
//     the bitmap, and re-adding it is one XOR pass.
//   * H2: up to ~76 residual columns per layer with <= 13 additions each, and
//     over all 32 layers exactly one addition uses another RESIDUAL column;
//     every other addition is an apparent column, which does not depend on
//     any other column.  So H2 runs as phase 1 (apparent-only reduction,
//     column-parallel: kP1Blocks x kSmallW waves per layer pull columns from a
//     per-layer counter, concurrently with the H1 chain) and phase 2
//     (k_reduce_h2_finish: columns in order, O(1) each unless the phase-1
//     pivot is owned by an earlier residual column, in which case the stored
//     working column is reloaded and reduced further, exactly like Ripser
//     would have continued).
// Phase 1 of a column performs exactly the first steps Ripser's serial loop
// performs on it (the serial loop consults residual owners first, and a
// pivot owned by an apparent column is never a residual pivot), so the
// result is bit-identical to the serial order.
//
// Triangle ranks (k_h1_prep).  Every triangle t <= thresh is assigned to its
// youngest facet e(t) (longest edge, ties -> smallest edge index); that is the
// facet an apparent pair would pair it with.  Edges are sorted by length and
// edge e owns the rank block [off_e, off_e + |M_e|), M_e = bitmask of third
// vertices w of its triangles {a, b, w}, ordered by w DESCENDING -- the colex
// index of {a, b, w} grows with w, so inside a block rank order is Ripser's
// (diam asc, index desc).  Edges of equal length form a class whose blocks are
// contiguous; only inside such a tie class does rank order differ from
// filtration order, and the pivot search resolves it by index (rare path).
// Without a tie, t is an apparent pivot iff it is the FIRST triangle of its
// block (the oldest cofacet of e(t) whose youngest facet is e(t)).
#pragma once
#include "rips_reduce.h"

namespace tda {

constexpr int kDenseMaxN = 64;
constexpr int kChainT = 256;              // threads per k_h1_chain block (staging; the chain is wave 0)
constexpr int kP1Grid = 96;               // k_h2_phase1 blocks per layer (one wave each, strided columns)
constexpr uint32_t kP1WCap = 512;         // phase-1 toggle-set capacity
constexpr int kChainMaxCols = 512;        // non-cleared H1 residual columns / stored R_j per layer
constexpr int kMaxK = 21;                 // bitmap words per lane: ceil(C(64,3) / 32 / 64)

__device__ __forceinline__ uint32_t c2u(uint32_t x) { return x * (x - 1) / 2; }
__device__ __forceinline__ uint32_t c3u(uint32_t x) { return x * (x - 1) * (x - 2) / 6; }
__device__ __forceinline__ uint32_t edge_id(int a, int b) { return a > b ? c2u(a) + b : c2u(b) + a; }
__device__ __forceinline__ uint32_t tri_id(int a, int b, int c) {
    const int x = max(a, max(b, c)), z = min(a, min(b, c)), y = a + b + c - x - z;
    return c3u(x) + c2u(y) + z;
}
// edge index -> (a, b), a > b
__device__ __forceinline__ void edge_verts(uint32_t q, int& a, int& b) {
    int x = (int)((1.0f + sqrtf(1.0f + 8.0f * (float)q)) * 0.5f);
    while (c2u(x) > q) --x;
    while (c2u(x + 1) <= q) ++x;
    a = x;
    b = (int)(q - c2u(x));
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) { return (uint32_t)wave_max_u64((uint64_t)v); }
// set bits of M above bit v
__device__ __forceinline__ uint32_t bits_above(uint64_t M, int v) { return v >= 63 ? 0u : (uint32_t)__popcll(M >> (v + 1)); }
// bit position of the k-th highest set bit of M (k = 0: the highest), one lane
__device__ __forceinline__ int kth_highest(uint64_t M, uint32_t k) {
    for (uint32_t i = 0; i < k; ++i) M &= ~(1ull << (63 - __clzll(M)));
    return 63 - __clzll(M);
}
__device__ __forceinline__ void lds_xor(uint32_t* p, uint32_t v) {
    __hip_atomic_fetch_xor((TDA_LDS uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// per edge (colex index), 16 B: one ds_read_b128
struct EdgeRec {
    uint64_t M;        // third vertices w of the triangles {a, b, w} <= thresh whose youngest facet is this edge
    uint16_t off;      // first rank of the block
    uint16_t ab;       // a | b << 6 | tie << 12  (a > b; tie: the length class holds other edges)
    float len;         // edge length
};
static_assert(sizeof(EdgeRec) == 16, "EdgeRec is one 16-B load");
struct EdgeRecV {
    uint64_t M;
    uint32_t off;
    int a, b;
    bool tie;
    float len;
};
__device__ __forceinline__ EdgeRecV load_rec(const EdgeRec* R, uint32_t e) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 q = ((const TDA_LDS u32x4*)R)[e];
    EdgeRecV v;
    v.M = (uint64_t)q.x | ((uint64_t)q.y << 32);
    v.off = q.z & 0xFFFFu;
    v.a = (int)((q.z >> 16) & 63u);
    v.b = (int)((q.z >> 22) & 63u);
    v.tie = (q.z >> 28) & 1u;
    v.len = __uint_as_float(q.w);
    return v;
}

struct DenseBufs {
    EdgeRec* recs;      // [L][E]
    uint32_t* cls;      // [L][E] rank range of the edge's length class: cs | ce << 16 (tie path)
    uint16_t* inv;      // [L][inv_stride] rank -> edge (general path)
    uint32_t* inv32;    // [L][inv_stride] rank -> a | b << 6 | w << 12 | first << 18 | tie << 19 (FAST path)
    uint16_t* rank_of;  // [L][tri_stride] triangle colex index -> rank, 0xFFFF above thresh (FAST path)
    uint32_t tri_stride;
    uint16_t* cls2;     // [L][n2p] length-class rank of edge (u, v) at u * n + v; 0xFFFF above thresh (H2 phase 1)
    uint32_t n2p;
    uint32_t* res1;     // [L][piv_words1] colex bitmap of residual H1 pivots (H2 clearing; zeroed per call)
    uint32_t E, inv_stride;
    int K;              // bitmap words per lane (W = 64 K words)
};

// ---------------------------------------------------------------- ranks
// 2048 u64 keys in one 1024-thread block, ascending: two keys per thread in
// registers; compare-exchange distances below 128 are in-wave shuffles, only
// the 10 stages with distance >= 128 go through LDS (sk).
__device__ __forceinline__ void sort2048(uint64_t& k0, uint64_t& k1, uint64_t* sk) {
    const int t = threadIdx.x;
    for (int k = 2; k <= 2048; k <<= 1) {
        const bool up = ((2 * t) & k) == 0;
        int j = k >> 1;
        if (j >= 128) {
            sk[2 * t] = k0;
            sk[2 * t + 1] = k1;
            __syncthreads();
            for (; j >= 128; j >>= 1) {
                // element pairs (i, i ^ j) with i < i ^ j: one per thread
                const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
                const uint64_t x = sk[i], y = sk[i ^ j];
                const bool u = (i & k) == 0;
                if ((x > y) == u) {
                    sk[i] = y;
                    sk[i ^ j] = x;
                }
                __syncthreads();
            }
            k0 = sk[2 * t];
            k1 = sk[2 * t + 1];
            __syncthreads();
        }
        for (; j >= 2; j >>= 1) {
            const int m = j >> 1;  // partner thread t ^ m (same wave: m < 64)
            const uint64_t p0 = shfl_xor_u64(k0, m), p1 = shfl_xor_u64(k1, m);
            const bool lower = (t & m) == 0;
            const bool keep_min = lower == up;
            k0 = keep_min ? (k0 < p0 ? k0 : p0) : (k0 > p0 ? k0 : p0);
            k1 = keep_min ? (k1 < p1 ? k1 : p1) : (k1 > p1 ? k1 : p1);
        }
        {  // j == 1: inside the thread
            const uint64_t lo = k0 < k1 ? k0 : k1, hi = k0 < k1 ? k1 : k0;
            k0 = up ? lo : hi;
            k1 = up ? hi : lo;
        }
    }
}

// One 1024-thread block per layer: sort the edges <= thresh by length, build
// each edge's block mask, the exclusive scan of block sizes (= ranks), the
// class ranges and the rank tables:
//   recs[e], inv16[rank] = e           (general path)
//   rank_of[triangle] (0xFFFF: above thresh), inv32[rank] = a | b << 6 |
//   w << 12 | first-of-block << 18 | tie << 19      (FAST path, N <= ~51)
// Keys are (length bits << 32 | e << 12 | a << 6 | b): no index decode after
// the sort.  LDS: [16][D][keys 2048][counts 2048][masks 2048].
__global__ __launch_bounds__(1024) void k_h1_prep(const float* __restrict__ dist, int n, const uint32_t* __restrict__ rowmax,
                                                  float user_thresh, DenseBufs db, int fast, LayerStats* __restrict__ stats) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.x, t = threadIdx.x, T = blockDim.x, ln = t & 63, wv = t >> 6, nw = T >> 6;
#ifdef TDA_PROFILE
    uint64_t tp[8];
    tp[0] = clock64();
#define TDA_PREP_STAMP(i) tp[i] = clock64()
#else
#define TDA_PREP_STAMP(i)
#endif
    const float r = block_thresh(rowmax + (size_t)l * n, n, user_thresh, (uint32_t*)smem);
    float* D = (float*)(smem + 16);
    stage_to_lds(D, dist + (size_t)l * n * n, 4ull * n * n, t, T);
    uint64_t* sk = (uint64_t*)(smem + 16 + ((4ull * n * n + 15) & ~15ull));
    uint32_t* off = (uint32_t*)(sk + 2048);
    uint64_t* Ms = (uint64_t*)(off + 2048);
    uint32_t& s_ne = *(uint32_t*)(smem + 4);
    uint32_t& s_tot = *(uint32_t*)(smem + 8);
    const int E = n * (n - 1) / 2;
    if (t == 0) s_ne = 0;
    if (fast) {  // every triangle starts "above the threshold"
        uint32_t* ro = (uint32_t*)(db.rank_of + (size_t)l * db.tri_stride);
        for (uint32_t i = t; i < db.tri_stride / 2; i += T) st_glb(ro, i, 0xFFFFFFFFu);
    }
    __syncthreads();
    uint64_t k0 = kEmpty64, k1 = kEmpty64;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int q = 2 * t + c;
        uint64_t k = kEmpty64;
        if (q < E) {
            int a, b;
            edge_verts((uint32_t)q, a, b);
            const float d = D[a * n + b];
            if (d <= r) k = ((uint64_t)__float_as_uint(d + 0.0f) << 32) | ((uint32_t)q << 12) | ((uint32_t)a << 6) | (uint32_t)b;
        }
        (c == 0 ? k0 : k1) = k;
    }
    TDA_PREP_STAMP(1);
    sort2048(k0, k1, sk);
    sk[2 * t] = k0;
    sk[2 * t + 1] = k1;
    __syncthreads();
    // the thread holding the last real key publishes the edge count
    if (k0 != kEmpty64 && k1 == kEmpty64) s_ne = (uint32_t)(2 * t + 1);
    if (k1 != kEmpty64 && (t == T - 1 || sk[2 * t + 2] == kEmpty64)) s_ne = (uint32_t)(2 * t + 2);
    __syncthreads();
    TDA_PREP_STAMP(2);
    const int nE = (int)s_ne;
    // block masks: one wave per edge (4 edges in flight), lane = third vertex
    for (int q0 = wv; q0 < nE; q0 += 4 * nw) {
        uint64_t kk[4];
        float dav[4], dbv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int q = q0 + u * nw;
            kk[u] = q < nE ? sk[q] : kEmpty64;
            const int a = (int)((kk[u] >> 6) & 63u), b = (int)(kk[u] & 63u);
            dav[u] = ln < n ? D[a * n + ln] : 0.0f;
            dbv[u] = ln < n ? D[b * n + ln] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int q = q0 + u * nw;
            const uint32_t e = (uint32_t)(kk[u] >> 12) & 0xFFFFFu;
            const int a = (int)((kk[u] >> 6) & 63u), b = (int)(kk[u] & 63u), v = ln;
            const float le = __uint_as_float((uint32_t)(kk[u] >> 32));
            bool ok = q < nE && v < n && v != a && v != b && dav[u] <= le && dbv[u] <= le;
            if (ok && dav[u] == le && edge_id(a, v) < e) ok = false;  // (a, v) is the younger facet
            if (ok && dbv[u] == le && edge_id(b, v) < e) ok = false;
            const uint64_t m = __ballot(ok);
            if (ln == 0 && q < nE) {
                Ms[q] = m;
                off[q] = (uint32_t)__popcll(m);
            }
        }
    }
    __syncthreads();
    TDA_PREP_STAMP(3);
    if (wv == 0) {  // exclusive scan of the block sizes
        uint32_t carry = 0;
        for (int q0 = 0; q0 < nE; q0 += 64) {
            const int q = q0 + ln;
            const uint32_t c = q < nE ? off[q] : 0u;
            uint32_t x = c;
            for (int s = 1; s < 64; s <<= 1) {
                const uint32_t y = __shfl_up(x, s, 64);
                if (ln >= s) x += y;
            }
            if (q < nE) off[q] = carry + x - c;
            carry += __shfl(x, 63, 64);
        }
        if (ln == 0) s_tot = carry;
    }
    __syncthreads();
    TDA_PREP_STAMP(4);
    EdgeRec* R = db.recs + (size_t)l * db.E;
    for (int q = t; q < nE; q += T) {
        const uint32_t lb = (uint32_t)(sk[q] >> 32);
        int q0 = q, q1 = q;
        while (q0 > 0 && (uint32_t)(sk[q0 - 1] >> 32) == lb) --q0;
        while (q1 + 1 < nE && (uint32_t)(sk[q1 + 1] >> 32) == lb) ++q1;
        const uint32_t e = (uint32_t)(sk[q] >> 12) & 0xFFFFFu;
        const int a = (int)((sk[q] >> 6) & 63u), b = (int)(sk[q] & 63u);
        EdgeRec rec;
        rec.M = Ms[q];
        rec.off = (uint16_t)off[q];
        rec.ab = (uint16_t)(a | (b << 6) | ((q0 != q1) << 12));
        rec.len = __uint_as_float(lb);
        R[e] = rec;
        db.cls[(size_t)l * db.E + e] = off[q0] | ((off[q1] + (uint32_t)__popcll(Ms[q1])) << 16);
        uint16_t* c2 = db.cls2 + (size_t)l * db.n2p;
        st_glb(c2, (size_t)a * n + b, (uint16_t)q0);
        st_glb(c2, (size_t)b * n + a, (uint16_t)q0);
    }
    for (int e = t; e < E; e += T) {  // edges above the threshold own no triangles
        int a, b;
        edge_verts((uint32_t)e, a, b);
        const float d = D[a * n + b];
        if (!(d <= r)) {
            EdgeRec rec = {};
            rec.ab = (uint16_t)(a | (b << 6));
            rec.len = d;
            R[e] = rec;
            uint16_t* c2 = db.cls2 + (size_t)l * db.n2p;
            st_glb(c2, (size_t)a * n + b, (uint16_t)0xFFFFu);
            st_glb(c2, (size_t)b * n + a, (uint16_t)0xFFFFu);
        }
    }
    __syncthreads();
    TDA_PREP_STAMP(5);
    uint16_t* inv = db.inv + (size_t)l * db.inv_stride;
    uint32_t* inv32 = db.inv32 + (size_t)l * db.inv_stride;
    uint16_t* ro = db.rank_of + (size_t)l * db.tri_stride;
    for (int q0 = wv; q0 < nE; q0 += 4 * nw) {  // 4 edges in flight per wave
        uint64_t key[4], M[4], kp[4], kn[4];
        uint32_t o[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int q = q0 + u * nw;
            const bool in = q < nE;
            key[u] = in ? sk[q] : 0;
            M[u] = in ? Ms[q] : 0;
            o[u] = in ? off[q] : 0;
            kp[u] = in && q > 0 ? sk[q - 1] : kEmpty64;
            kn[u] = in && q + 1 < nE ? sk[q + 1] : kEmpty64;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t e = (uint32_t)(key[u] >> 12) & 0xFFFFFu;
            const int a = (int)((key[u] >> 6) & 63u), b = (int)(key[u] & 63u);
            const uint32_t lb = (uint32_t)(key[u] >> 32);
            const bool tie = (uint32_t)(kp[u] >> 32) == lb || (uint32_t)(kn[u] >> 32) == lb;
            if (!fast) {
                const uint32_t c = (uint32_t)__popcll(M[u]);
                if ((uint32_t)ln < c) inv[o[u] + ln] = (uint16_t)e;
            } else if (ln < n && ((M[u] >> ln) & 1ull)) {
                const uint32_t rk = o[u] + bits_above(M[u], ln);
                st_glb(inv32, rk, (uint32_t)a | ((uint32_t)b << 6) | ((uint32_t)ln << 12) | ((uint32_t)(rk == o[u]) << 18) |
                                      ((uint32_t)tie << 19));
                st_glb(ro, tri_id(a, b, ln), (uint16_t)rk);
            }
        }
    }
    if (t == 0) stats[l].ntri = s_tot;
#ifdef TDA_PROFILE
    TDA_PREP_STAMP(6);
    if (t == 0)
        for (int i = 1; i < 7; ++i) stats[l].prof[3][i] = tp[i] - tp[i - 1];
#endif
#undef TDA_PREP_STAMP
}

// ---------------------------------------------------------------- H1 chain
// H1 of one layer.  All kChainT threads stage the layer's tables and filter
// the residual columns; then wave 0 alone runs the serial reduction (waves
// 1..3 leave; no s_barrier is issued after that point).  K = bitmap words per
// lane (compile time: the pivot scan is K independent loads and a min tree).
// FAST (N <= ~51): a toggle is rank_of[triangle] -> ds_xor and the pivot's
// vertices are one inv32 load; otherwise edge records (recs, inv16).
// LDS: [16][D][recs E | rank_of][inv16 | inv32][W 64K][res 64K][piv][cols][own].
template <int K, bool FAST>
__global__ __launch_bounds__(kChainT) void k_h1_chain(const float* __restrict__ dist, int n, LayerStats* __restrict__ stats,
                                                      DimBufs b, Reduce2Bufs rb, DenseBufs db, uint64_t step_limit,
                                                      Pair* __restrict__ pairs, uint64_t pcap) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr uint32_t WP = 64u * K;
    const int l = blockIdx.x, t = threadIdx.x, ln = t & 63, wv = t >> 6;
    LayerStats* st = stats + l;
    const int E = n * (n - 1) / 2;
    unsigned char* p = smem + 16;
    auto take = [&](size_t bytes) {
        unsigned char* q = p;
        p += (bytes + 15) & ~(size_t)15;
        return q;
    };
    float* Dl = (float*)take(4ull * n * n);
    EdgeRec* R = FAST ? nullptr : (EdgeRec*)take(16ull * E);
    uint16_t* inv = FAST ? nullptr : (uint16_t*)take(2ull * db.inv_stride);
    uint16_t* rof = FAST ? (uint16_t*)take(2ull * db.tri_stride) : nullptr;
    uint32_t* inv32 = FAST ? (uint32_t*)take(4ull * db.inv_stride) : nullptr;
    uint32_t* W = (uint32_t*)take(4ull * WP);
    uint32_t* res = (uint32_t*)take(4ull * WP);  // ranks that are residual pivots
    uint32_t* piv = (uint32_t*)take(4ull * b.piv_words);  // colex bitmap of apparent pivots (tie classes)
    uint64_t* cols = (uint64_t*)take(8ull * kChainMaxCols);
    uint16_t* own = (uint16_t*)take(2ull * kChainMaxCols);
    uint32_t* hdr = (uint32_t*)smem;

    const uint32_t ntri = (uint32_t)st->ntri;
    stage_to_lds(Dl, dist + (size_t)l * n * n, 4ull * n * n, t, kChainT);
    if constexpr (FAST) {
        stage_to_lds(rof, db.rank_of + (size_t)l * db.tri_stride, 2ull * db.tri_stride, t, kChainT);
        stage_to_lds(inv32, db.inv32 + (size_t)l * db.inv_stride, 4ull * ntri, t, kChainT);
    } else {
        stage_to_lds(R, db.recs + (size_t)l * db.E, 16ull * E, t, kChainT);
        stage_to_lds(inv, db.inv + (size_t)l * db.inv_stride, 4ull * ((ntri + 1) / 2), t, kChainT);
    }
    const uint32_t* pivg = b.pivbits + (size_t)l * b.piv_words;
    uint32_t* res1 = db.res1 + (size_t)l * b.piv_words;
    stage_to_lds(piv, pivg, 4ull * b.piv_words, t, kChainT);
    for (uint32_t i = t; i < WP; i += kChainT) {
        st_lds(W, i, 0u);
        st_lds(res, i, 0u);
    }
    uint64_t nres = (uint64_t)st->n_residual[1];
    if (nres > b.rcap) nres = b.rcap;
    if (wv == 0) {  // drop H0 deaths (spanning-forest edges: cleared columns), keep column order
        const uint64_t* resid = b.resid + (size_t)l * b.rcap;
        const uint32_t* mst = rb.mst + (size_t)l * rb.mst_words;
        uint32_t nc = 0, nskip = 0;
        for (uint64_t j0 = 0; j0 < nres; j0 += 64) {
            const uint64_t j = j0 + ln;
            uint64_t key = 0;
            bool keep = false;
            if (j < nres) {
                key = ld_glb(resid, j);
                const uint32_t s = (uint32_t)key_idx(key);
                keep = !((ld_glb(mst, s >> 5) >> (s & 31)) & 1u);
            }
            const uint64_t m = __ballot(keep);
            const uint32_t pos = nc + lanes_below(m);
            if (keep && pos < (uint32_t)kChainMaxCols) st_lds(cols, pos, key);
            nc += (uint32_t)__popcll(m);
            nskip += (uint32_t)__popcll(__ballot(j < nres)) - (uint32_t)__popcll(m);
        }
        if (ln == 0) {
            hdr[0] = nc;
            hdr[1] = nskip;
        }
    }
    __syncthreads();
    if (wv != 0) return;

    const float r = st->thresh;
    const uint32_t nc = hdr[0], nskip = hdr[1];
    Pair* P = pairs + (size_t)l * pcap;
    uint32_t* pool = (uint32_t*)(rb.rpool + (size_t)l * rb.rpool_cap);
    const uint64_t pool_words = 2ull * rb.rpool_cap;
    const uint32_t* clsg = db.cls + (size_t)l * db.E;
    uint64_t ecnt = 0, cs = 0, npairs = 0, nadds = 0;
    uint32_t nown = 0;
    int err = nc > (uint32_t)kChainMaxCols ? 1 : 0;
#ifdef TDA_PROFILE
    uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // total, pivot, tie pivots, cob-app, add-owner, new pair, -, pivots
    const uint64_t t_all = clock64();
    uint64_t ties = 0;
#endif

    // toggle the coboundary of edge (a, b) (length le <= r): lane v -> {a, b, v}
    auto cob = [&](int a, int b, float le) {
        const int v = ln;
        if constexpr (FAST) {
            if (v < n && v != a && v != b) {
                const uint32_t rk = ld_lds(rof, tri_id(a, b, v));
                if (rk != 0xFFFFu) lds_xor(&W[rk >> 5], 1u << (rk & 31));
            }
            return;
        }
        bool ok = v < n && v != a && v != b;
        float dav = 0.0f, dbv = 0.0f;
        if (ok) {
            dav = ld_lds(Dl, (size_t)a * n + v);
            dbv = ld_lds(Dl, (size_t)b * n + v);
            ok = fmaxf(dav, dbv) <= r;
        }
        if (ok) {
            // youngest facet of {a, b, v}: longest edge, ties -> smallest index
            float bl = le;
            uint32_t be = edge_id(a, b);
            int third = v;
            const uint32_t eav = edge_id(a, v), ebv = edge_id(b, v);
            if (dav > bl || (dav == bl && eav < be)) {
                bl = dav;
                be = eav;
                third = b;
            }
            if (dbv > bl || (dbv == bl && ebv < be)) {
                bl = dbv;
                be = ebv;
                third = a;
            }
            const EdgeRecV q = load_rec(R, be);
            const uint32_t rk = q.off + bits_above(q.M, third);
            lds_xor(&W[rk >> 5], 1u << (rk & 31));
        }
    };
    // first set bit of W (wave-uniform), false if W is empty
    auto first_bit = [&](uint32_t& rk) -> bool {
        uint32_t w[K];
#pragma unroll
        for (int k = 0; k < K; ++k) w[k] = ld_lds(W, (size_t)ln * K + k);
        uint32_t pos[K];
#pragma unroll
        for (int k = 0; k < K; ++k) pos[k] = w[k] ? (uint32_t)k * 32u + (uint32_t)__builtin_ctz(w[k]) : 0xFFFFu;
#pragma unroll
        for (int s = 1; s < K; s <<= 1)
#pragma unroll
            for (int k = 0; k + s < K; k += 2 * s) pos[k] = min(pos[k], pos[k + s]);
        const uint64_t m = __ballot(pos[0] != 0xFFFFu);
        if (!m) return false;
        const int f = __builtin_ctzll(m);
        rk = (uint32_t)f * (32u * K) + (uint32_t)__builtin_amdgcn_readlane((int)pos[0], f);
        return true;
    };

    for (uint32_t j = 0; j < nc && !err; ++j) {
        const uint64_t key = ld_lds(cols, j);
        const uint32_t sidx = (uint32_t)key_idx(key);
        const float sdm = key_diam(key);
        int a0, b0;
        edge_verts(sidx, a0, b0);
        cob(a0, b0, sdm);
        lds_order();
        for (uint64_t step = 0;; ++step) {
            if (step >= step_limit) {
                if (ln == 0) printf("h1_chain: layer %d column %u step limit\n", l, j);
                err = 3;
                break;
            }
            TDA_STAMP(t1);
            uint32_t rk;
            const bool found = first_bit(rk);
#ifdef TDA_PROFILE
            prof[7] += 1;
#endif
            if (!found) {  // zero column: essential class
                if (ln == 0 && ecnt < pcap) store_pair(P, ecnt, sdm, INFINITY, (int64_t)sidx, -1);
                ++ecnt;
                TDA_ACC(1, t1);
                break;
            }
            uint32_t resw = ld_lds(res, rk >> 5);
            int a, b2, w;
            bool tie, first;
            if constexpr (FAST) {
                const uint32_t q = ld_lds(inv32, rk);
                a = (int)(q & 63u);
                b2 = (int)((q >> 6) & 63u);
                w = (int)((q >> 12) & 63u);
                first = (q >> 18) & 1u;
                tie = (q >> 19) & 1u;
            } else {
                const EdgeRecV q = load_rec(R, ld_lds(inv, rk));
                a = q.a;
                b2 = q.b;
                tie = q.tie;
                first = rk == q.off;
                const uint32_t k = rk - q.off;
                const int v = ln;
                w = __builtin_ctzll(__ballot(((q.M >> v) & 1ull) && bits_above(q.M, v) == k));
            }
            if (tie) {
                // tie class: the pivot is the set triangle of [cs, ce) with the largest index
#ifdef TDA_PROFILE
                ++ties;
#endif
                const uint32_t cc = ld_glb(clsg, edge_id(a, b2)), c0 = cc & 0xFFFFu, c1 = cc >> 16;
                uint32_t best = 0, brk = rk;
                for (uint32_t base = c0; base < c1; base += 64) {
                    const uint32_t rho = base + ln;
                    uint32_t cand = 0;
                    if (rho < c1 && ((ld_lds(W, rho >> 5) >> (rho & 31)) & 1u)) {
                        if constexpr (FAST) {
                            const uint32_t q2 = ld_lds(inv32, rho);
                            cand = tri_id((int)(q2 & 63u), (int)((q2 >> 6) & 63u), (int)((q2 >> 12) & 63u)) + 1;
                        } else {
                            const EdgeRecV q2 = load_rec(R, ld_lds(inv, rho));
                            cand = tri_id(q2.a, q2.b, kth_highest(q2.M, rho - q2.off)) + 1;
                        }
                    }
                    const uint32_t m = wave_max_u32(cand);
                    if (m > best) {
                        best = m;
                        brk = base + (uint32_t)__builtin_ctzll(__ballot(cand == m));
                    }
                }
                rk = brk;
                resw = ld_lds(res, rk >> 5);
                if constexpr (FAST) {
                    const uint32_t q = ld_lds(inv32, rk);
                    a = (int)(q & 63u);
                    b2 = (int)((q >> 6) & 63u);
                    w = (int)((q >> 12) & 63u);
                } else {
                    const EdgeRecV q = load_rec(R, ld_lds(inv, rk));
                    a = q.a;
                    b2 = q.b;
                    w = kth_highest(q.M, rk - q.off);
                }
            }
            const uint32_t tidx = tri_id(a, b2, w);
            TDA_ACC(1, t1);
            TDA_STAMP(t2);
            if ((resw >> (rk & 31)) & 1u) {
                // add the stored reduced column of the residual column that owns rk
                uint32_t s = 0;
                for (uint32_t s0 = 0; s0 < nown; s0 += 64) {
                    const uint32_t sl = s0 + ln;
                    const uint64_t m = __ballot(sl < nown && ld_lds(own, sl) == rk);
                    if (m) {
                        s = s0 + (uint32_t)__builtin_ctzll(m);
                        break;
                    }
                }
                const uint32_t* src = pool + (size_t)s * WP;
                uint32_t x[K];
#pragma unroll
                for (int k = 0; k < K; ++k) x[k] = ld_glb(src, (size_t)k * 64 + ln);
#pragma unroll
                for (int k = 0; k < K; ++k) st_lds(W, (size_t)ln * K + k, ld_lds(W, (size_t)ln * K + k) ^ x[k]);
                ++nadds;
                TDA_ACC(4, t2);
            } else if (tie ? ((ld_lds(piv, tidx >> 5) >> (tidx & 31)) & 1u) : first) {
                // apparent pair (e, t): add the coboundary of the youngest facet e
                cob(a, b2, FAST ? 0.0f : ld_lds(Dl, (size_t)a * n + b2));
                ++nadds;
                TDA_ACC(3, t2);
            } else {
                // new persistence pair (column, t); R_j = W
                const float pd = ld_lds(Dl, (size_t)a * n + b2);
                if (pd > sdm) {
                    if (ln == 0 && ecnt < pcap) store_pair(P, ecnt, sdm, pd, (int64_t)sidx, (int64_t)tidx);
                    ++ecnt;
                }
                cs += pair_hash(sidx, tidx);
                npairs += 1;
                if ((uint64_t)(nown + 1) * WP > pool_words || nown >= (uint32_t)kChainMaxCols) {
                    err = 2;
                    break;
                }
                uint32_t* dst = pool + (size_t)nown * WP;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    st_glb(dst, (size_t)k * 64 + ln, ld_lds(W, (size_t)ln * K + k));
                    st_lds(W, (size_t)ln * K + k, 0u);
                }
                if (ln == 0) {
                    st_lds(own, nown, (uint16_t)rk);
                    st_lds(res, rk >> 5, resw | (1u << (rk & 31)));
                    matomic_or<false>(&res1[tidx >> 5], 1u << (tidx & 31));  // H2 clearing reads this bitmap
                }
                ++nown;
                TDA_ACC(5, t2);
                break;
            }
            lds_order();
        }
        wave_sync();  // R_j stores reach memory before a later owner addition reads them
    }
    if (ln == 0) {
#ifdef TDA_PROFILE
        prof[0] = clock64() - t_all;
        prof[2] = ties;
        for (int i = 0; i < 8; ++i) st->prof[0][i] = prof[i];
#endif
        if (err == 1) atomicOr(&st->err, ERR_LDS_SPILL);
        if (err == 2) atomicOr(&st->err, ERR_VPOOL_CAP);
        if (err == 3) atomicOr(&st->err, ERR_STEP_LIMIT);
        if (ecnt > pcap) atomicOr(&st->err, ERR_PAIR_CAP);
        st->count[1] = (int64_t)ecnt;
        atomicAdd((unsigned long long*)&st->checksum[1], (unsigned long long)cs);
        atomicAdd((unsigned long long*)&st->all_pairs[1], (unsigned long long)npairs);
        atomicAdd((unsigned long long*)&st->n_adds[1], (unsigned long long)nadds);
        atomicAdd((unsigned long long*)&st->n_columns[1], (unsigned long long)(0ull - nskip));
        st->nskip[1] = nskip;
    }
}
// bitmap words per lane supported by k_h1_chain instantiations (FAST: up to 12)
constexpr int kChainKs[] = {1, 2, 3, 4, 6, 9, 12, 16, 21};
constexpr int kChainFastMaxK = 12;

// ---------------------------------------------------------------- H2 phase 1
// One wave per block; block (l, g) takes the layer's residual H2 columns
// g, g + gridDim.y, ... and reduces each with apparent columns only.  The
// whole step runs on 32-bit words:
//   * a tetrahedron's key is (class << 20) | (2^20 - 1 - colex index), where
//     class = rank of its longest edge's length among the sorted edges
//     (cls2, k_h1_prep): key order is Ripser's (diameter asc, index desc);
//   * membership is a bitmap over tetrahedron indices (a toggle is one
//     returning ds_xor), the keys live in an append-only log (+ packed
//     vertices) whose dead entries are dropped lazily by the bitmap test;
//   * apparency is tested on the fly from the classes the coboundary step
//     loads anyway (apparent pairs form a matching [upstream ripser.cpp
//     get_zero_apparent_facet], so this equals k_apparent's bitmap).
// Results go out in the u64 key format of the serial phase 2.
// LDS: [16][D][cls2][bitmap][log][log vertices].
constexpr uint32_t kP1LogCap = 1024;
// Phase-1 additions per column before handing the column to the serial phase
// 2.  The long phase-1 chains are H2 columns that turn out to be H1 deaths
// (cleared once the H1 chain pairs them); the kept columns of the 32-layer
// sweep need <= 44 additions in all.
constexpr uint32_t kP1MaxAdds = 32;
constexpr uint32_t kClsInvalid = 0xFFFFu;

__device__ __forceinline__ uint32_t c4u(uint32_t x) { return x < 4 ? 0u : x * (x - 1) * (x - 2) / 6 * (x - 3) / 4; }
__device__ __forceinline__ uint32_t c3s(uint32_t x) { return x < 3 ? 0u : x * (x - 1) * (x - 2) / 6; }
__device__ __forceinline__ uint32_t c2s(uint32_t x) { return x < 2 ? 0u : x * (x - 1) / 2; }

__global__ __launch_bounds__(64) void k_h2_phase1(const float* __restrict__ dist, int n, LayerStats* __restrict__ stats, DimBufs b,
                                                  SmallBufs sb, const uint16_t* __restrict__ cls2g, uint32_t n2p, uint32_t bm_words,
                                                  const uint32_t* __restrict__ res1g, uint32_t res1_words, uint64_t step_limit) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.x, ln = threadIdx.x;
    LayerStats* st = stats + l;
    uint64_t nres = (uint64_t)st->n_residual[2];
    if (nres > b.rcap) nres = b.rcap;
    if (blockIdx.y >= nres) return;
    const uint64_t* resid = b.resid + (size_t)l * b.rcap;
    unsigned char* p = smem + 16;
    auto take = [&](size_t bytes) {
        unsigned char* q = p;
        p += (bytes + 15) & ~(size_t)15;
        return q;
    };
    float* Dl = (float*)take(4ull * n * n);
    uint16_t* cls = (uint16_t*)take(2ull * n2p);
    uint32_t* bm = (uint32_t*)take(4ull * bm_words);
    uint32_t* lk = (uint32_t*)take(4ull * kP1LogCap);
    uint32_t* lv = (uint32_t*)take(4ull * kP1LogCap);
    stage_to_lds(Dl, dist + (size_t)l * n * n, 4ull * n * n, ln, 64);
    stage_to_lds(cls, cls2g + (size_t)l * n2p, 2ull * n2p, ln, 64);
    for (uint32_t i = ln; i < bm_words; i += 64) st_lds(bm, i, 0u);
    wave_sync();

    uint64_t* p1k = sb.p1_key + (size_t)l * b.rcap;
    uint32_t* p1i = sb.p1_info + (size_t)l * b.rcap;
    uint64_t* roff = sb.roff2 + (size_t)l * b.rcap;
    uint32_t* rlen = sb.rlen2 + (size_t)l * b.rcap;
    auto C = [&](int u, int v) -> uint32_t { return ld_lds(cls, (size_t)u * n + v); };
    uint32_t cnt = 0;  // log length (wave-uniform)

    // coboundary of facet f (f0 > f1 > f2, class fc) in lane v: key, vertices;
    // toggles it into the bitmap and appends new entries; returns the ballot
    // of lanes whose cofacet has class fc (apparent test)
    auto cob_entry = [&](int f0, int f1, int f2, uint32_t fc, uint32_t& key, uint32_t& pk, bool& ok) -> uint64_t {
        const int v = ln;
        ok = v < n && v != f0 && v != f1 && v != f2;
        uint32_t cc = kClsInvalid;
        if (ok) {
            const uint32_t a0 = C(v, f0), a1 = C(v, f1), a2 = C(v, f2);
            cc = max(fc, max(a0, max(a1, a2)));
            ok = cc != kClsInvalid;
        }
        const int x0 = max(v, f0), x1 = v > f0 ? f0 : max(v, f1), x2 = v > f1 ? f1 : max(v, f2), x3 = v > f2 ? f2 : v;
        const uint32_t tidx = c4u(x0) + c3s(x1) + c2s(x2) + (uint32_t)x3;
        key = (cc << 20) | (0xFFFFFu - tidx);
        pk = (uint32_t)x0 | ((uint32_t)x1 << 6) | ((uint32_t)x2 << 12) | ((uint32_t)x3 << 18);
        return __ballot(ok && cc == fc);
    };
    auto toggle = [&](uint32_t key, uint32_t pk, bool ok) {
        bool ins = false;
        if (ok) {
            const uint32_t tidx = 0xFFFFFu - (key & 0xFFFFFu), bit = 1u << (tidx & 31);
            const uint32_t old = __hip_atomic_fetch_xor((TDA_LDS uint32_t*)bm + (tidx >> 5), bit, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_WORKGROUP);
            ins = !(old & bit);
        }
        const uint64_t m = __ballot(ins);
        if (ins) {
            const uint32_t pos = cnt + lanes_below(m);
            st_lds(lk, pos, key);
            st_lds(lv, pos, pk);
        }
        cnt += (uint32_t)__popcll(m);
    };
    auto live = [&](uint32_t key) -> bool {
        const uint32_t tidx = 0xFFFFFu - (key & 0xFFFFFu);
        return (ld_lds(bm, tidx >> 5) >> (tidx & 31)) & 1u;
    };
    // rewrite the log with one entry per live key (in place, order kept);
    // `emit` sees every kept (key, vertices); returns the new length
    auto compact = [&](auto&& emit) -> uint32_t {
        uint32_t pos = 0;
        for (uint32_t e0 = 0; e0 < cnt; e0 += 64) {
            const uint32_t e = e0 + ln;
            uint32_t key = 0, pk = 0;
            bool keep = false;
            if (e < cnt) {
                key = ld_lds(lk, e);
                pk = ld_lds(lv, e);
                const uint32_t tidx = 0xFFFFFu - (key & 0xFFFFFu), bit = 1u << (tidx & 31);
                // first lane to clear a live bit keeps the key (duplicates drop)
                const uint32_t old = __hip_atomic_fetch_and((TDA_LDS uint32_t*)bm + (tidx >> 5), ~bit, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_WORKGROUP);
                keep = old & bit;
            }
            const uint64_t m = __ballot(keep);
            if (keep) {
                const uint32_t q = pos + lanes_below(m);
                st_lds(lk, q, key);
                st_lds(lv, q, pk);
                emit(q, key, pk);
            }
            pos += (uint32_t)__popcll(m);
        }
        // restore the bits of the kept keys
        for (uint32_t e = ln; e < pos; e += 64) {
            const uint32_t tidx = 0xFFFFFu - (ld_lds(lk, e) & 0xFFFFFu);
            __hip_atomic_fetch_or((TDA_LDS uint32_t*)bm + (tidx >> 5), 1u << (tidx & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        lds_order();
        return pos;
    };
    // packed vertices (6 bits each, descending) -> phase-2 key / diameter
    auto diam_of = [&](uint32_t pk) -> float {
        const int x0 = pk & 63, x1 = (pk >> 6) & 63, x2 = (pk >> 12) & 63, x3 = (pk >> 18) & 63;
        const float* r0 = Dl + (size_t)x0 * n;
        const float* r1 = Dl + (size_t)x1 * n;
        float d = fmaxf(fmaxf(ld_lds(r0, x1), ld_lds(r0, x2)), fmaxf(ld_lds(r0, x3), ld_lds(r1, x2)));
        return fmaxf(d, fmaxf(ld_lds(r1, x3), ld_lds(Dl, (size_t)x2 * n + x3)));
    };
    auto key64 = [&](uint32_t pk) -> uint64_t {
        const uint32_t p8 = (pk & 63) << 24 | ((pk >> 6) & 63) << 16 | ((pk >> 12) & 63) << 8 | ((pk >> 18) & 63);
        return ((uint64_t)__float_as_uint(diam_of(pk) + 0.0f) << 32) | (0xFFFFFFFFu - p8);
    };

#ifdef TDA_PROFILE
    const uint64_t t_p1 = clock64();
#endif
    for (uint64_t j = blockIdx.y; j < nres; j += gridDim.y) {
#ifdef TDA_PROFILE
        const uint64_t tcol = clock64();
#endif
        const uint64_t key = ld_glb(resid, j);
        const uint64_t sidx = key_idx(key);
        // an H1 death found by the concurrent H1 chain is cleared: no phase 1
        const TDA_GLB uint32_t* res1 = (const TDA_GLB uint32_t*)(res1g + (size_t)l * res1_words);
        auto cleared = [&]() -> bool {
            return (__hip_atomic_load(res1 + (sidx >> 5), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (sidx & 31)) & 1u;
        };
        if (cleared()) {
            if (ln == 0) {
                st_glb(p1k, j, kEmpty64);
                st_glb(p1i, j, kP1Overflow);
            }
            continue;
        }
        int vs[3];
        decode_wave<2>(sidx, n, vs, ln);
        const uint32_t scls = max(C(vs[0], vs[1]), max(C(vs[0], vs[2]), C(vs[1], vs[2])));
        {
            uint32_t k, pk;
            bool ok;
            (void)cob_entry(vs[0], vs[1], vs[2], scls, k, pk, ok);
            toggle(k, pk, ok);
        }
        lds_order();
        uint32_t adds = 0, flags = 0, out_idx = 0;
        uint64_t out_key = kEmpty64;
        for (uint64_t step = 0;; ++step) {
            if (step >= step_limit || adds >= kP1MaxAdds || ((step & 7) == 7 && cleared())) {
                flags = kP1Overflow;  // phase 2 skips it if cleared, else redoes it serially
                break;
            }
            // pivot: smallest live key (with its log position)
            uint32_t bk = 0xFFFFFFFFu, bp = 0;
            for (uint32_t e0 = 0; e0 < cnt; e0 += 256) {
                uint32_t k4[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t e = e0 + (uint32_t)u * 64 + ln;
                    k4[u] = e < cnt ? ld_lds(lk, e) : 0xFFFFFFFFu;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const bool lv4 = k4[u] != 0xFFFFFFFFu && live(k4[u]);
                    if (lv4 && k4[u] < bk) {
                        bk = k4[u];
                        bp = e0 + (uint32_t)u * 64 + ln;
                    }
                }
            }
            const uint32_t pk32 = wave_min_u32(bk);
            if (pk32 == 0xFFFFFFFFu) break;  // zero column: essential
            const int src = __builtin_ctzll(__ballot(bk == pk32));
            const uint32_t tpk = ld_lds(lv, (uint32_t)__builtin_amdgcn_readlane((int)bp, src));
            const uint32_t tcls = pk32 >> 20;
            int t[4] = {(int)(tpk & 63), (int)((tpk >> 6) & 63), (int)((tpk >> 12) & 63), (int)((tpk >> 18) & 63)};
            // youngest facet f of t: largest class, ties -> drop the larger vertex
            const uint32_t c01 = C(t[0], t[1]), c02 = C(t[0], t[2]), c03 = C(t[0], t[3]);
            const uint32_t c12 = C(t[1], t[2]), c13 = C(t[1], t[3]), c23 = C(t[2], t[3]);
            const uint32_t fc0 = max(c12, max(c13, c23)), fc1 = max(c02, max(c03, c23));
            const uint32_t fc2 = max(c01, max(c03, c13)), fc3 = max(c01, max(c02, c12));
            int fu = 0;
            uint32_t fc = fc0;
            if (fc1 > fc) { fc = fc1; fu = 1; }
            if (fc2 > fc) { fc = fc2; fu = 2; }
            if (fc3 > fc) { fc = fc3; fu = 3; }
            const int f0 = fu == 0 ? t[1] : t[0];
            const int f1 = fu <= 1 ? t[2] : t[1];
            const int f2 = fu <= 2 ? t[3] : t[2];
            const int tv = fu == 0 ? t[0] : fu == 1 ? t[1] : fu == 2 ? t[2] : t[3];
            uint32_t ck, cpk;
            bool cok;
            const uint64_t eq = cob_entry(f0, f1, f2, fc, ck, cpk, cok);
            const bool app = tcls == fc && eq && 63 - __clzll(eq) == tv;
            if (!app) {  // not apparent: phase 1 ends here
                out_key = key64(tpk);
                out_idx = 0xFFFFFu - (pk32 & 0xFFFFFu);
                unsigned long long base = 0;
                if (ln == 0) base = atomicAdd(&sb.p1_used[l], (unsigned long long)cnt);
                base = __shfl(base, 0, 64);
                if (base + cnt > sb.rpool2_cap) {
                    flags = kP1Overflow;
                    break;
                }
                uint64_t* out = sb.rpool2 + (size_t)l * sb.rpool2_cap + base;
                const uint32_t wr = compact([&](uint32_t q, uint32_t, uint32_t pk) { st_glb(out, q, key64(pk)); });
                cnt = wr;
                if (ln == 0) {
                    st_glb(roff, j, (uint64_t)base);
                    st_glb(rlen, j, wr);
                }
                break;
            }
            toggle(ck, cpk, cok);
            ++adds;
            if (cnt + 64 > kP1LogCap) {
                cnt = compact([](uint32_t, uint32_t, uint32_t) {});
                if (cnt + 64 > kP1LogCap) {
                    flags = kP1Overflow;
                    break;
                }
            }
            lds_order();
        }
        if (ln == 0) {
            st_glb(p1k, j, out_key);
            st_glb(p1i, j, adds | flags);
            st_glb(sb.p1_pidx + (size_t)l * b.rcap, j, out_idx);
#ifdef TDA_PROFILE
            const uint64_t tt = clock64() - tcol;
            atomicMax((unsigned long long*)&st->prof[1][2], (unsigned long long)tt);
            atomicMax((unsigned long long*)&st->prof[1][3], (unsigned long long)((tt << 16) | (adds & 0xFFFF)));
            atomicAdd((unsigned long long*)&st->prof[1][6], (unsigned long long)tt);
            atomicAdd((unsigned long long*)&st->prof[1][7], (unsigned long long)adds);
#endif
        }
        // clear the bitmap words this column touched
        for (uint32_t e = ln; e < cnt; e += 64) st_lds(bm, (0xFFFFFu - (ld_lds(lk, e) & 0xFFFFFu)) >> 5, 0u);
        cnt = 0;
        wave_sync();
    }
#ifdef TDA_PROFILE
    if (ln == 0) atomicMax((unsigned long long*)&st->prof[1][0], (unsigned long long)(clock64() - t_p1));
#endif
}

}  // namespace tda
