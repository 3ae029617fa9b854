// rips_dense.h -- the N <= 48 sweep in ONE launch (k_dense_fused): every
// stage of a layer's H0..H2 persistence runs inside the workgroups of that
// layer, with its tables in LDS, and the pairs go straight to the host-mapped
// result.  The reference runs this per layer in Python (debug_tda_pipeline.py
// :92-110, `ripser(cloud, maxdim)` at :109); the multi-kernel dense path
// (rips_reduce_small.h) needed ~10 dependent launches over four streams for
// the same work, whose boundaries and cross-queue waits were most of its time.
//
// Two workgroups of 1024 threads per layer (maxdim 2; one for maxdim 1):
//   A (blocks 0 .. L8-1):  distances staged to LDS, threshold; wave 15 runs
//       the one-wave Prim H0 (h0_wave_body) while waves 0..14 sort the edges
//       (LDS bitonic, group barrier of 15 waves); then the whole workgroup
//       builds the H1 tables: edge ranks, per-edge third-vertex masks
//       A_e = {v : d(a,v) <= d(a,b), d(b,v) <= d(a,b)} and M_e (the triangles
//       whose youngest facet is e), the apparent H1 pairs (e apparent iff the
//       highest vertex of A_e is in M_e: the zero-apparent cofacet test of
//       k_apparent<1>), triangle ranks (prefix of |M_e| in rank order),
//       inv32 / rank_of (the FAST tables of k_h1_chain); the residual H1
//       columns are the non-apparent, non-forest edges in descending rank,
//       so no residual sort is needed; wave 0 then runs the H1 chain
//       (h1_chain_wave<K, kChainFast>) and publishes the residual H1 pivots
//       (res1) and a done flag.
//   B (blocks L8 .. 2 L8 - 1, the same XCD as its A: block ids differ by a
//       multiple of 8): the same sort gives each edge its length class;
//       the same masks give the apparent H1 pivots (H2 clearing); per-vertex
//       sorted distance rows with prefix vertex masks give, for a triangle
//       {p, q, w} with longest edge (p, q), its zero-diameter cofacets as
//       A_pq & NB(w, d(p,q)) -- one binary search instead of a scan over N
//       (the k_apparent<2> test); the residual H2 columns are sorted in LDS;
//       phase 1 (apparent-only additions, as k_h2_phase1) runs on all 16
//       waves with a 32-bit key toggle set of 512 slots per wave; after A's
//       flag the serial phase 2 (as k_reduce_h2_finish) walks the columns in
//       order; then B emits dims 0..2 into the host-mapped output.
// The apparent-pair, tie and clearing rules are exactly those of the
// multi-kernel dense path (rips_reduce_small.h, rips_kernels.h k_apparent),
// which the parity tests pin against the CPU checker under oracle/.
//
// Cross-workgroup hand-off (MI355X_MICROARCH.md "inter-workgroup visibility"):
// A's stores drain (vmcnt(0)), the workgroup barrier precedes wave 0's chain,
// wave 0 ends with an agent release (buffer_wbl2), vmcnt(0), then a relaxed
// agent flag store; B polls the flag with relaxed agent loads, then ONE agent
// acquire, vmcnt(0), and reads A's data with plain loads.  A never waits for
// B, and B(l)'s block id is above A(l)'s; a spin limit aborts to the
// multi-kernel path (ERR_FUSED) if a flag never comes.
#pragma once
#include "rips_reduce_small.h"

namespace tda {

constexpr int kFT = 1024;             // threads per fused workgroup
constexpr int kFW = kFT / 64;         // waves
constexpr uint32_t kFCols = kChainMaxCols;  // non-cleared H1 residual columns per layer
constexpr uint32_t kF2Cap = 2048;     // H2 residual columns per layer (LDS sort / maps)
constexpr uint32_t kFSet = 512;       // phase-1 toggle-set slots per wave
constexpr uint32_t kFSet2 = 1024;     // phase-2 (serial) toggle-set slots
constexpr uint32_t kFSpin = 1u << 26; // polls of A's flag before B gives up (~seconds)
constexpr uint32_t kFEmpty = 0xFFFFFFFFu;
constexpr uint32_t kFDead = 0x80000000u;
enum : int32_t { ERR_FUSED = 512 };   // fused path gave up: the host re-runs the multi-kernel path
constexpr int kFusedKs[] = {1, 2, 3, 4, 6, 9};  // chain bitmap words per lane (N <= 48)

struct FusedBufs {
    const float* dist;        // [L][n][n]
    const uint32_t* rowmax;   // [L][n]
    float user_thresh;
    LayerStats* stats;
    Pair* pairs[3];
    uint64_t pcap[3];
    uint32_t* res1;           // [L][res1_words] residual H1 pivots (colex), A -> B
    uint64_t res1_words;
    uint32_t* clsg;           // [L][E] class triangle-rank range of each edge (chain tie path)
    uint32_t* pool1;          // [L][pool1_words] H1 reduced columns (chain)
    uint64_t pool1_words;
    uint32_t* done;           // [L] A finished (zeroed per call)
    uint32_t* p1_key;         // [L][kF2Cap] phase-1 pivot key (kFEmpty: zero column)
    uint32_t* p1_info;        // [L][kF2Cap] additions | kP1Overflow
    uint32_t* roff2;          // [L][kF2Cap] stored column: offset, length in rpool2
    uint32_t* rlen2;
    uint64_t* rpool2;         // [L][rpool2_cap] key | packed vertices << 32
    uint64_t rpool2_cap;
    unsigned long long* out_used;  // output cursor (zeroed per call)
    OutPair* hout;
    uint64_t hout_cap;
    int64_t* houtoff;
    LayerStats* hstats;
    uint64_t step_limit;
    uint32_t tri_stride, inv_stride, piv_words1;  // carve sizes (host mirrors)
    int stop;                 // dev aid (TDA_FUSED_STOP, test overrides only): role B gives up after that phase
};

// ---------------------------------------------------------------- LDS carves
// A: [hdr][D][rank_of][inv32][W][res][piv][mst][cols][own][scratch: keys, M, A, ep, fr, cse, app]
// B: [hdr][D][cls2][lenq][h1app][resk][union: prep (keys, Ae, srow, pm) | phase 1 sets | phase 2 maps + set]
struct FCarve {
    uint32_t D, rof, inv32, W, res, piv, mst, cols, own, keys, M, Ae, ep, fr, cse, app, endA;
    uint32_t cls2, lenq, h1app, resk, un, srow, pm, sets, map, tmap, wset, endB;
};
__host__ __device__ constexpr uint32_t fal16(uint64_t x) { return (uint32_t)((x + 15) & ~15ull); }
__host__ __device__ inline uint32_t fpow2(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}
__host__ __device__ inline FCarve fused_carve_b(int n, uint32_t piv_words1) {
    FCarve c{};
    const uint32_t E = (uint32_t)(n * (n - 1) / 2), P2 = fpow2(E < 2 ? 2 : E);
    uint32_t o = 128;  // header: 32 words (flags, counters, block_excl scratch at [8, 25))
    auto take = [&](uint64_t b) {
        const uint32_t r = o;
        o += fal16(b);
        return r;
    };
    c.D = take(4ull * n * n);
    c.cls2 = take(2ull * n * n);
    c.lenq = take(4ull * E);
    c.h1app = take(4ull * piv_words1);
    c.resk = take(4ull * kF2Cap);
    c.un = o;
    uint32_t end = o;
    // prep: sort keys, A_e, sorted rows, prefix masks
    c.keys = take(8ull * P2);
    c.Ae = take(8ull * E);
    c.srow = take(4ull * n * n);
    c.pm = take(8ull * n * (n + 1));
    end = end > o ? end : o;
    // phase 1: kFW sets of kFSet (key, packed vertices)
    o = c.un;
    c.sets = take(8ull * kFW * kFSet);
    end = end > o ? end : o;
    // phase 2: conflict table and pivot map (2 x u32 per slot each), serial set
    o = c.un;
    c.tmap = take(8ull * 2 * kF2Cap);
    c.map = take(8ull * 2 * kF2Cap);
    c.wset = take(8ull * kFSet2);
    end = end > o ? end : o;
    c.endB = end;
    return c;
}
__host__ __device__ inline FCarve fused_carve_a(int n, int K, uint32_t ts, uint32_t is, uint32_t pw) {
    FCarve c{};
    const uint32_t E = (uint32_t)(n * (n - 1) / 2), P2 = fpow2(E < 2 ? 2 : E);
    uint32_t o = 128;  // header: 32 words (flags, counters, block_excl scratch at [8, 25))
    auto take = [&](uint64_t b) {
        const uint32_t r = o;
        o += fal16(b);
        return r;
    };
    c.D = take(4ull * n * n);
    c.rof = take(2ull * ts);
    c.inv32 = take(4ull * is);
    c.W = take(4ull * 64 * K);
    c.res = take(4ull * 64 * K);
    c.piv = take(4ull * pw);
    c.mst = take(4ull * (E / 32 + 1));
    c.cols = take(8ull * kFCols);
    c.own = take(2ull * kFCols);
    c.keys = take(8ull * P2);
    c.M = take(8ull * E);
    c.Ae = 0;
    c.ep = take(2ull * E);
    c.fr = take(2ull * (E + 1));
    c.cse = take(4ull * E);
    c.app = take(4ull * (E / 32 + 1));
    c.endA = o;
    return c;
}

// ---------------------------------------------------------------- helpers
// barrier of the first nw waves of the workgroup through an LDS counter (the
// other waves run something else meanwhile, so s_barrier cannot be used)
__device__ __forceinline__ void grp_sync(uint32_t* ctr, uint32_t nw) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane_id() == 0) {
        const uint32_t old = __hip_atomic_fetch_add((TDA_LDS uint32_t*)ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t target = (old / nw + 1) * nw;
        while (__hip_atomic_load((TDA_LDS uint32_t*)ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target)
            __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// ascending bitonic sort of P2 (power of two) keys in LDS by threads t < T;
// sync() separates the stages
template <typename KT, typename Sync>
__device__ __forceinline__ void lds_bitonic(KT* a, uint32_t P2, int t, int T, Sync&& sync) {
    for (uint32_t k = 2; k <= P2; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = (uint32_t)t; i < P2 / 2; i += (uint32_t)T) {
                const uint32_t lo = ((i & ~(j - 1)) << 1) | (i & (j - 1)), hi = lo + j;
                const KT x = ld_lds(a, lo), y = ld_lds(a, hi);
                if ((x > y) == ((lo & k) == 0)) {
                    st_lds(a, lo, y);
                    st_lds(a, hi, x);
                }
            }
            sync();
        }
}

// exclusive prefix of c over the workgroup (all kFT threads, in thread order);
// *tot = total.  scratch: kFW + 1 words of LDS
__device__ __forceinline__ uint32_t block_excl(uint32_t c, uint32_t* tot, uint32_t* scratch) {
    const int t = threadIdx.x, ln = t & 63, w = t >> 6;
    uint32_t x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (ln >= o) x += y;
    }
    if (ln == 63) st_lds(scratch, (uint32_t)w, x);
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int q = 0; q < kFW; ++q) {
        const uint32_t s = ld_lds(scratch, (uint32_t)q);
        before += q < w ? s : 0u;
        all += s;
    }
    __syncthreads();
    *tot = all;
    return before + x - c;
}

__device__ __forceinline__ uint64_t shfl_up_u64(uint64_t v, int o) {
    const uint32_t lo = __shfl_up((unsigned)(uint32_t)v, o, 64), hi = __shfl_up((unsigned)(uint32_t)(v >> 32), o, 64);
    return ((uint64_t)hi << 32) | lo;
}

// stage the layer's matrix, resolve the threshold, build the edge keys (filtration
// order; edges above the threshold sort last); all threads
__device__ __forceinline__ float fused_stage(const FusedBufs& F, int l, int n, float* D, uint64_t* keys, uint32_t P2, uint32_t* hdr) {
    const int t = threadIdx.x;
    if (t < 32) st_lds(hdr, (uint32_t)t, t == 2 ? 0xFFFFFFFFu : 0u);  // [2]: threshold minimum
    stage_to_lds(D, F.dist + (size_t)l * n * n, 4ull * n * n, t, kFT);
    float thr = F.user_thresh;
    const bool enc = isinf(thr) || thr == 3.402823466e+38f;
    __syncthreads();
    if (enc) {
        if (t < n) __hip_atomic_fetch_min((TDA_LDS uint32_t*)hdr + 2, ld_glb(F.rowmax + (size_t)l * n, (size_t)t), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
        __syncthreads();
        thr = n == 1 ? 0.0f : __uint_as_float(ld_lds(hdr, 2u));
    }
    const uint32_t E = (uint32_t)(n * (n - 1) / 2);
    for (uint32_t e = t; e < P2; e += kFT) {
        uint64_t k = kEmpty64;
        if (e < E) {
            int a, b;
            edge_verts(e, a, b);
            const float le = ld_lds(D, (size_t)a * n + b);
            if (le <= thr) k = filt_key(le, e);
        }
        st_lds(keys, e, k);
    }
    return thr;
}

// Per-edge masks (wave per edge, lane = third vertex v): A_e (cofacets of
// diameter d(a,b)) and M_e (triangles whose youngest facet is e: longest edge,
// ties -> smallest index, as k_prep_edges); the edge is an apparent H1 column
// iff the highest vertex of A_e is in M_e.  fn(e, a, b, le, A, M) per edge <= thr
// (wave-uniform call).
template <typename Fn>
__device__ __forceinline__ void fused_masks(const float* D, int n, float thr, int wv, int nw, Fn&& fn) {
    const int ln = lane_id();
    const uint32_t E = (uint32_t)(n * (n - 1) / 2);
    for (uint32_t e0 = (uint32_t)wv * 4; e0 < E; e0 += (uint32_t)nw * 4) {
        float dav[4], dbv[4], le[4];
        int av[4], bv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t e = e0 + u;
            int a = 1, b = 0;
            if (e < E) edge_verts(e, a, b);
            av[u] = a;
            bv[u] = b;
            le[u] = e < E ? ld_lds(D, (size_t)a * n + b) : INFINITY;
            dav[u] = ln < n ? ld_lds(D, (size_t)a * n + ln) : INFINITY;
            dbv[u] = ln < n ? ld_lds(D, (size_t)b * n + ln) : INFINITY;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t e = e0 + u;
            if (e >= E || !(le[u] <= thr)) continue;
            const int a = av[u], b = bv[u], v = ln;
            const bool in = v < n && v != a && v != b && dav[u] <= le[u] && dbv[u] <= le[u];
            bool m = in;
            if (m && dav[u] == le[u] && edge_id(a, v) < e) m = false;  // (a, v) is the younger facet
            if (m && dbv[u] == le[u] && edge_id(b, v) < e) m = false;
            fn(e, a, b, le[u], __ballot(in), __ballot(m));
        }
    }
}

__device__ __forceinline__ uint32_t tet_colex(int v, int f0, int f1, int f2) {  // f0 > f1 > f2, v distinct
    const int x0 = max(v, f0), x1 = v > f0 ? f0 : max(v, f1), x2 = v > f1 ? f1 : max(v, f2), x3 = v > f2 ? f2 : v;
    return c4u((uint32_t)x0) + c3s((uint32_t)x1) + c2s((uint32_t)x2) + (uint32_t)x3;
}
__device__ __forceinline__ uint32_t tet_pack(int v, int f0, int f1, int f2) {
    const int x0 = max(v, f0), x1 = v > f0 ? f0 : max(v, f1), x2 = v > f1 ? f1 : max(v, f2), x3 = v > f2 ? f2 : v;
    return (uint32_t)x0 | ((uint32_t)x1 << 6) | ((uint32_t)x2 << 12) | ((uint32_t)x3 << 18);
}

// ---------------------------------------------------------------- 32-bit toggle set (one wave)
// Open addressing over u32 keys (key < 2^31; bit 31 = cancelled, kFEmpty =
// free), packed vertices beside each key.  Keys of one pass are distinct.
struct FSet {
    uint32_t* k;
    uint32_t* pk;
    uint32_t cap;   // power of two
    uint32_t used;  // occupied slots (wave-uniform)
    __device__ void clear() {
        for (uint32_t e = lane_id(); e < cap; e += 64) st_lds(k, e, kFEmpty);
        used = 0;
        lds_order();
    }
    // toggle key (if ok); returns false if the table is too full afterwards
    __device__ void toggle(uint32_t key, uint32_t p, bool ok) {
        bool ins = false;
        if (ok) {
            uint32_t h = mix32(key) & (cap - 1);
            for (uint32_t it = 0; it < cap; ++it, h = (h + 1) & (cap - 1)) {
                uint32_t cur = ld_lds(k, h);
                if (cur == kFEmpty) {
                    __hip_atomic_compare_exchange_strong((TDA_LDS uint32_t*)k + h, &cur, key, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (cur == kFEmpty) {  // claimed
                        st_lds(pk, h, p);
                        ins = true;
                        break;
                    }
                    // another lane of this pass took the slot: cur is its key
                }
                if ((cur & ~kFDead) == key) {  // present: flip its parity
                    __hip_atomic_fetch_xor((TDA_LDS uint32_t*)k + h, kFDead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
            }
        }
        used += (uint32_t)__popcll(__ballot(ins));
        lds_order();
    }
    // min live key (kFEmpty if none) and its packed vertices (wave-uniform)
    __device__ uint32_t pivot(uint32_t& pv) const {
        const int ln = lane_id();
        uint32_t best = kFDead, bs = 0;
        for (uint32_t e = ln; e < cap; e += 64) {
            const uint32_t x = ld_lds(k, e);
            if (x < best) best = x, bs = e;  // cancelled keys and kFEmpty have bit 31 set
        }
        const uint32_t m = wave_min_u32(best);
        if (m >= kFDead) return kFEmpty;
        const int src = __builtin_ctzll(__ballot(best == m));
        const uint32_t slot = (uint32_t)__builtin_amdgcn_readlane((int)bs, src);
        pv = (uint32_t)__builtin_amdgcn_readfirstlane((int)ld_lds(pk, slot));
        return m;
    }
    // live keys to out[] (u64: key | pk << 32), returns how many
    __device__ uint32_t gather(uint64_t* out, uint64_t lim) const {
        const int ln = lane_id();
        uint32_t pos = 0;
        for (uint32_t e0 = 0; e0 < cap; e0 += 64) {
            const uint32_t x = ld_lds(k, e0 + ln);
            const bool live = x < kFDead;
            const uint64_t m = __ballot(live);
            const uint32_t q = pos + lanes_below(m);
            if (live && q < lim) st_glb(out, q, (uint64_t)x | ((uint64_t)ld_lds(pk, e0 + ln) << 32));
            pos += (uint32_t)__popcll(m);
        }
        return pos;
    }
    // drop cancelled keys (re-insert the live ones); false if still too full
    __device__ bool compact(uint32_t limit) {
        const int ln = lane_id();
        constexpr int R = 16;  // cap <= 1024: up to 16 slots per lane
        uint32_t kk[R], pp[R];
        uint32_t nl = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t e = (uint32_t)r * 64 + ln;
            kk[r] = e < cap ? ld_lds(k, e) : kFEmpty;
            pp[r] = e < cap ? ld_lds(pk, e) : 0u;
            nl += kk[r] < kFDead;
        }
        lds_order();
        clear();
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if ((uint32_t)r * 64 >= cap) break;
            toggle(kk[r], pp[r], kk[r] < kFDead);
        }
        return used <= limit;
    }
};

// coboundary of triangle f (f0 > f1 > f2, class fc) in lane v: key, packed
// vertices, validity; returns the ballot of lanes whose cofacet has class fc
__device__ __forceinline__ uint64_t f_cob(const uint16_t* cls2, int n, int f0, int f1, int f2, uint32_t fc, uint32_t& key, uint32_t& pk,
                                          bool& ok) {
    const int v = lane_id();
    ok = v < n && v != f0 && v != f1 && v != f2;
    uint32_t cc = 0xFFFFu;
    if (ok) {
        const uint32_t a0 = ld_lds(cls2, (size_t)v * n + f0), a1 = ld_lds(cls2, (size_t)v * n + f1), a2 = ld_lds(cls2, (size_t)v * n + f2);
        cc = max(fc, max(a0, max(a1, a2)));
        ok = cc != 0xFFFFu;
    }
    key = (cc << 20) | (0xFFFFFu - tet_colex(v, f0, f1, f2));
    pk = tet_pack(v, f0, f1, f2);
    return __ballot(ok && cc == fc);
}

// apparent test of pivot t (packed vertices tp, class tc): its youngest facet
// (largest class, ties -> drop the larger vertex), and whether t is that
// facet's zero-apparent cofacet.  On true, key/pk/ok hold the facet's coboundary.
__device__ __forceinline__ bool f_apparent(const uint16_t* cls2, int n, uint32_t tp, uint32_t tc, uint32_t& key, uint32_t& pk, bool& ok) {
    const int t0 = (int)(tp & 63), t1 = (int)((tp >> 6) & 63), t2 = (int)((tp >> 12) & 63), t3 = (int)((tp >> 18) & 63);
    auto C = [&](int u, int v) -> uint32_t { return ld_lds(cls2, (size_t)u * n + v); };
    const uint32_t c01 = C(t0, t1), c02 = C(t0, t2), c03 = C(t0, t3), c12 = C(t1, t2), c13 = C(t1, t3), c23 = C(t2, t3);
    const uint32_t fc0 = max(c12, max(c13, c23)), fc1 = max(c02, max(c03, c23));
    const uint32_t fc2 = max(c01, max(c03, c13)), fc3 = max(c01, max(c02, c12));
    int fu = 0;
    uint32_t fc = fc0;
    if (fc1 > fc) fc = fc1, fu = 1;
    if (fc2 > fc) fc = fc2, fu = 2;
    if (fc3 > fc) fc = fc3, fu = 3;
    const int f0 = fu == 0 ? t1 : t0;
    const int f1 = fu <= 1 ? t2 : t1;
    const int f2 = fu <= 2 ? t3 : t2;
    const int tv = fu == 0 ? t0 : fu == 1 ? t1 : fu == 2 ? t2 : t3;
    const uint64_t eq = f_cob(cls2, n, f0, f1, f2, fc, key, pk, ok);
    return tc == fc && eq && 63 - __clzll(eq) == tv;
}

// emission of dims 0 .. nd-1 of layer l into the host-mapped output (one wave);
// every stat of the layer is final when this runs
__device__ __forceinline__ void fused_emit(const FusedBufs& F, int l, int nd, LayerStats* st) {
    const int ln = lane_id();
    uint64_t c[3] = {0, 0, 0}, total = 0;
    for (int d = 0; d < nd; ++d) {
        const uint64_t x = (uint64_t)st->count[d];
        c[d] = x < F.pcap[d] ? x : F.pcap[d];
        total += c[d];
    }
    uint64_t base = 0;
    if (ln == 0) base = atomicAdd(F.out_used, (unsigned long long)total);
    base = shfl_u64(base, 0);
    if (base + total > F.hout_cap) {
        if (ln == 0) atomicOr(&st->err, (int32_t)ERR_OUT_CAP);  // the host grows the output and runs k_emit
    } else {
        uint64_t o = base;
        for (int d = 0; d < nd; ++d) {
            const Pair* P = F.pairs[d] + (size_t)l * F.pcap[d];
            for (uint64_t e = ln; e < c[d]; e += 64) {
                const Pair q = P[e];
                F.hout[o + e] = OutPair{q.birth, q.death, q.birth_idx, q.death_idx};
            }
            if (ln == 0) F.houtoff[l * nd + d] = (int64_t)o;
            o += c[d];
        }
    }
    wave_sync();
    const uint64_t* src = (const uint64_t*)st;
    uint64_t* dst = (uint64_t*)(F.hstats + l);
    for (int i = ln; i < (int)(sizeof(LayerStats) / 8); i += 64) dst[i] = src[i];
}

// the fused path gave up on layer l (one wave): the error has to reach the
// host-mapped stats, which the host reads instead of the device copy (it then
// re-runs the batch on the multi-kernel path)
__device__ __forceinline__ void fused_fail(const FusedBufs& F, int l, LayerStats* st) {
    const int ln = lane_id();
    if (ln == 0) atomicOr(&st->err, (int32_t)ERR_FUSED);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    const uint64_t* src = (const uint64_t*)st;
    uint64_t* dst = (uint64_t*)(F.hstats + l);
    for (int i = ln; i < (int)(sizeof(LayerStats) / 8); i += 64) dst[i] = src[i];
}

// ---------------------------------------------------------------- role A: H0 + H1
template <int K>
__device__ void fused_role_a(const FusedBufs& F, int l, int n, int maxdim, unsigned char* smem) {
    const int t = threadIdx.x, ln = t & 63, wv = t >> 6;
    const FCarve cv = fused_carve_a(n, K, F.tri_stride, F.inv_stride, F.piv_words1);
    uint32_t* hdr = (uint32_t*)smem;  // [0] group barrier, [1] ncols, [2] threshold min, [3] nskip, [4] nres, [8..24] scratch
    float* D = (float*)(smem + cv.D);
    uint16_t* rof = (uint16_t*)(smem + cv.rof);
    uint32_t* inv32 = (uint32_t*)(smem + cv.inv32);
    uint32_t* W = (uint32_t*)(smem + cv.W);
    uint32_t* res = (uint32_t*)(smem + cv.res);
    uint32_t* piv = (uint32_t*)(smem + cv.piv);
    uint32_t* mst = (uint32_t*)(smem + cv.mst);
    uint64_t* cols = (uint64_t*)(smem + cv.cols);
    uint16_t* own = (uint16_t*)(smem + cv.own);
    uint64_t* keys = (uint64_t*)(smem + cv.keys);
    uint64_t* Ms = (uint64_t*)(smem + cv.M);
    uint16_t* ep = (uint16_t*)(smem + cv.ep);
    uint16_t* fr = (uint16_t*)(smem + cv.fr);
    uint32_t* cse = (uint32_t*)(smem + cv.cse);
    uint32_t* app = (uint32_t*)(smem + cv.app);
    LayerStats* st = F.stats + l;
    const uint32_t E = (uint32_t)(n * (n - 1) / 2), P2 = fpow2(E < 2 ? 2 : E);
    const uint32_t T3 = (uint32_t)(n * (n - 1) * (n - 2) / 6);
    constexpr uint32_t WP = 64u * K;
    // ---- A0: matrix, threshold, edge keys; clear the tables
    const float thr = fused_stage(F, l, n, D, keys, P2, hdr);
    for (uint32_t i = t; i < WP; i += kFT) {
        st_lds(W, i, 0u);
        st_lds(res, i, 0u);
    }
    for (uint32_t i = t; i < F.piv_words1; i += kFT) st_lds(piv, i, 0u);
    for (uint32_t i = t; i <= E / 32; i += kFT) {
        st_lds(mst, i, 0u);
        st_lds(app, i, 0u);
    }
    for (uint32_t i = t; i < (F.tri_stride + 1) / 2; i += kFT) st_lds((uint32_t*)rof, i, 0xFFFFFFFFu);
    __syncthreads();
    // ---- A1: wave 15 H0 (forest bits into LDS), waves 0..14 sort the edge keys
    if (wv == kFW - 1) {
        h0_wave_body<true>(D, n, thr, st, mst, F.pairs[0] + (size_t)l * F.pcap[0]);
    } else {
        lds_bitonic(keys, P2, t, (kFW - 1) * 64, [&]() { grp_sync(hdr, kFW - 1); });
    }
    __syncthreads();
    // ---- A2: ranks, classes
    uint32_t nE = 0;
    {
        uint32_t c = 0;
        for (uint32_t q = t; q < E; q += kFT) c += ld_lds(keys, q) != kEmpty64;
        uint32_t tot;
        (void)block_excl(c, &tot, hdr + 8);
        nE = tot;
    }
    for (uint32_t e = t; e < E; e += kFT) st_lds(ep, e, (uint16_t)0xFFFFu);
    __syncthreads();
    for (uint32_t q = t; q < nE; q += kFT) {
        const uint64_t k = ld_lds(keys, q);
        st_lds(ep, 0xFFFFFFFFu - (uint32_t)k, (uint16_t)q);
        const uint32_t len = (uint32_t)(k >> 32);
        uint32_t a = q, b = q;
        while (a > 0 && (uint32_t)(ld_lds(keys, a - 1) >> 32) == len) --a;
        while (b + 1 < nE && (uint32_t)(ld_lds(keys, b + 1) >> 32) == len) ++b;
        st_lds(cse, q, a | (b << 16));
    }
    // ---- masks: block sizes by rank, apparent H1 pairs (pivot bitmap, stats)
    uint64_t acs = 0, napp = 0;
    fused_masks(D, n, thr, wv, kFW, [&](uint32_t e, int a, int b, float le, uint64_t A, uint64_t M) {
        if (ln == 0) st_lds(Ms, e, M);
        const bool ap = A && ((M >> (63 - __clzll(A))) & 1ull);
        if (ap && ln == 0) {
            const int v = 63 - __clzll(A);
            const uint32_t tix = tri_id(a, b, v);
            __hip_atomic_fetch_or((TDA_LDS uint32_t*)piv + (tix >> 5), 1u << (tix & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_or((TDA_LDS uint32_t*)app + (e >> 5), 1u << (e & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            acs += pair_hash(e, tix);
            napp += 1;
        }
    });
    __syncthreads();
    // block sizes in rank order -> first triangle rank of each block (fr), triangles <= thr
    uint32_t ntri = 0;
    {
        // up to 2 ranks per thread (nE <= 1128 for N <= 48)
        const uint32_t q0 = 2 * t, q1 = 2 * t + 1;
        auto bsz = [&](uint32_t q) -> uint32_t {
            return q < nE ? (uint32_t)__popcll(ld_lds(Ms, 0xFFFFFFFFu - (uint32_t)ld_lds(keys, q))) : 0u;
        };
        const uint32_t s0 = bsz(q0), s1 = bsz(q1);
        uint32_t tot;
        const uint32_t ex = block_excl(s0 + s1, &tot, hdr + 8);
        if (q0 < nE) st_lds(fr, q0, (uint16_t)ex);
        if (q1 < nE) st_lds(fr, q1, (uint16_t)(ex + s0));
        if (t == 0) st_lds(fr, nE, (uint16_t)tot);
        ntri = tot;
    }
    __syncthreads();
    // ---- tables (wave per edge, lane = third vertex), class ranges, column list
    for (uint32_t e = wv; e < E; e += kFW) {
        const uint32_t q = ld_lds(ep, e);
        if (q == 0xFFFFu) continue;
        int a, b;
        edge_verts(e, a, b);
        const uint64_t M = ld_lds(Ms, e);
        const uint32_t off = ld_lds(fr, q), cs = ld_lds(cse, q), c0 = cs & 0xFFFFu, c1 = cs >> 16;
        const bool tie = c1 > c0;
        const int v = ln;
        if (v < n && ((M >> v) & 1ull)) {
            const uint32_t r2 = off + bits_above(M, v);
            st_lds(inv32, r2, (uint32_t)a | ((uint32_t)b << 6) | ((uint32_t)v << 12) | ((uint32_t)(r2 == off) << 18) | ((uint32_t)tie << 19));
            st_lds(rof, tri_id(a, b, v), (uint16_t)r2);
        }
        if (ln == 0) st_glb(F.clsg + (size_t)l * E, e, (uint32_t)ld_lds(fr, c0) | ((uint32_t)ld_lds(fr, c1 + 1) << 16));
    }
    // residual columns: non-apparent edges <= thr in column order (descending rank),
    // forest edges (H0 deaths) cleared
    uint32_t nc = 0, nskip = 0, nres = 0;
    for (uint32_t i0 = 0; i0 < nE; i0 += kFT) {
        const uint32_t i = i0 + t;
        bool keep = false, skip = false;
        uint64_t ck = 0;
        if (i < nE) {
            const uint32_t q = nE - 1 - i;
            const uint64_t k = ld_lds(keys, q);
            const uint32_t e = 0xFFFFFFFFu - (uint32_t)k;
            const bool ap = (ld_lds(app, e >> 5) >> (e & 31)) & 1u;
            const bool fo = (ld_lds(mst, e >> 5) >> (e & 31)) & 1u;
            keep = !ap && !fo;
            skip = !ap && fo;
            ck = col_key(__uint_as_float((uint32_t)(k >> 32)), e);
        }
        uint32_t tot, tsk, tre;
        const uint32_t pos = block_excl(keep ? 1u : 0u, &tot, hdr + 8);
        if (keep && nc + pos < kFCols) st_lds(cols, nc + pos, ck);
        (void)block_excl(skip ? 1u : 0u, &tsk, hdr + 8);
        nc += tot;
        nskip += tsk;
        nres += tot + tsk;
        (void)tre;
    }
    // apparent stats (one atomic per wave), the rest by the chain
    acs = wave_sum_u64(acs);
    napp = wave_sum_u64(napp);
    if (ln == 0 && napp) {
        atomicAdd((unsigned long long*)&st->checksum[1], (unsigned long long)acs);
        atomicAdd((unsigned long long*)&st->all_pairs[1], (unsigned long long)napp);
    }
    if (t == 0) {
        st->n_columns[1] = (int64_t)nE;
        st->n_residual[1] = (int64_t)nres;
        st->ntri = (int64_t)ntri;
    }
    (void)T3;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains before the barrier (A's release covers them)
    __syncthreads();  // tables, stats and the H0 stats (thresh) are complete
    if (wv != 0) return;
    // ---- A3: the H1 chain on wave 0
    ChainCtx c;
    c.Dl = D;
    c.R = nullptr;
    c.rof = rof;
    c.cobt = nullptr;
    c.inv = nullptr;
    c.inv32 = inv32;
    c.W = W;
    c.res = res;
    c.piv = piv;
    c.cols = cols;
    c.own = own;
    c.Dg = F.dist + (size_t)l * n * n;
    c.inv32g = nullptr;
    c.res1 = F.res1 + (size_t)l * F.res1_words;
    c.pool = F.pool1 + (size_t)l * F.pool1_words;
    c.pool_words = F.pool1_words;
    c.clsg = F.clsg + (size_t)l * E;
    c.P = F.pairs[1] + (size_t)l * F.pcap[1];
    c.pcap = F.pcap[1];
    c.st = st;
    c.n = n;
    c.l = l;
    c.nc = nc;
    c.nskip = nskip;
    c.step_limit = F.step_limit;
    c.t_entry = 0;
    h1_chain_wave<K, kChainFast>(c);
    wave_sync();
    if (maxdim < 2) {
        fused_emit(F, l, 2, st);
        return;
    }
    // publish: release (write back this XCD's L2), then the flag (agent scope)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (ln == 0) __hip_atomic_store(F.done + l, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- role B: H2
__device__ void fused_role_b(const FusedBufs& F, int l, int n, unsigned char* smem) {
    const int t = threadIdx.x, ln = t & 63, wv = t >> 6;
    const FCarve cv = fused_carve_b(n, F.piv_words1);
    uint32_t* hdr = (uint32_t*)smem;  // [0] barrier, [1] resid count, [2] thr min, [3] next column, [4] pool cursor, [5] flags, [8..24] scratch
    float* D = (float*)(smem + cv.D);
    uint16_t* cls2 = (uint16_t*)(smem + cv.cls2);
    uint32_t* lenq = (uint32_t*)(smem + cv.lenq);
    uint32_t* h1app = (uint32_t*)(smem + cv.h1app);
    uint32_t* resk = (uint32_t*)(smem + cv.resk);
    uint64_t* keys = (uint64_t*)(smem + cv.keys);
    uint64_t* Ae = (uint64_t*)(smem + cv.Ae);
    float* srow = (float*)(smem + cv.srow);
    uint64_t* pm = (uint64_t*)(smem + cv.pm);
    LayerStats* st = F.stats + l;
    const uint32_t E = (uint32_t)(n * (n - 1) / 2), P2 = fpow2(E < 2 ? 2 : E);
    const uint32_t T3 = (uint32_t)(n * (n - 1) * (n - 2) / 6);
    // ---- B0 / B1: matrix, threshold, edge keys, sort
    const float thr = fused_stage(F, l, n, D, keys, P2, hdr);
    for (uint32_t i = t; i < (uint32_t)(n * n + 1) / 2; i += kFT) st_lds((uint32_t*)cls2, i, 0xFFFFFFFFu);
    for (uint32_t i = t; i < F.piv_words1; i += kFT) st_lds(h1app, i, 0u);
    __syncthreads();
    lds_bitonic(keys, P2, t, kFT, []() { __syncthreads(); });
    if (F.stop == 1) {
        if (wv == 0) fused_fail(F, l, st);
        return;
    }
    // ---- B2: length class of every edge <= thr (rank of the first edge of its length)
    for (uint32_t q = t; q < E; q += kFT) {
        const uint64_t k = ld_lds(keys, q);
        if (k == kEmpty64) continue;
        const uint32_t len = (uint32_t)(k >> 32);
        uint32_t a = q;
        while (a > 0 && (uint32_t)(ld_lds(keys, a - 1) >> 32) == len) --a;
        const uint32_t e = 0xFFFFFFFFu - (uint32_t)k;
        int x, y;
        edge_verts(e, x, y);
        st_lds(cls2, (size_t)x * n + y, (uint16_t)a);
        st_lds(cls2, (size_t)y * n + x, (uint16_t)a);
        st_lds(lenq, q, len);
    }
    // ---- B3: A_e + apparent H1 pivots (H2 clearing); sorted rows + prefix masks
    fused_masks(D, n, thr, wv, kFW, [&](uint32_t e, int a, int b, float, uint64_t A, uint64_t M) {
        if (ln == 0) {
            st_lds(Ae, e, A);
            if (A && ((M >> (63 - __clzll(A))) & 1ull)) {
                const uint32_t tix = tri_id(a, b, 63 - __clzll(A));
                __hip_atomic_fetch_or((TDA_LDS uint32_t*)h1app + (tix >> 5), 1u << (tix & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    });
    for (int w = wv; w < n; w += kFW) {
        uint64_t k = ln < n ? (((uint64_t)__float_as_uint(ld_lds(D, (size_t)w * n + ln)) << 32) | (uint32_t)ln) : kEmpty64;
#pragma unroll
        for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                const uint64_t o = shfl_xor_u64(k, stride);
                const bool up = (ln & size) == 0, lower = (ln & stride) == 0;
                const uint64_t lo = o < k ? o : k, hi = o < k ? k : o;
                k = (lower == up) ? lo : hi;
            }
        uint64_t x = ln < n ? 1ull << (k & 63) : 0ull;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = shfl_up_u64(x, o);
            if (ln >= o) x |= y;
        }
        if (ln < n) {
            st_lds(srow, (size_t)w * n + ln, __uint_as_float((uint32_t)(k >> 32)));
            st_lds(pm, (size_t)w * (n + 1) + ln + 1, x);
        }
        if (ln == 0) st_lds(pm, (size_t)w * (n + 1), (uint64_t)0);
    }
    __syncthreads();
    if (F.stop == 2) {
        if (wv == 0) fused_fail(F, l, st);
        return;
    }
    // ---- B4: H2 columns (thread per triangle): cleared / apparent / residual
    uint64_t acs = 0, napp = 0, ncol = 0;
    for (uint32_t base = 0; base < T3; base += kFT) {
        const uint32_t tx = base + t;
        int kind = 0;
        uint32_t rkey = 0;
        if (tx < T3) {
            int vs[3];
            decode<2>(tx, n, vs);
            const int a = vs[0], b = vs[1], c = vs[2];
            const float dab = ld_lds(D, (size_t)a * n + b), dac = ld_lds(D, (size_t)a * n + c), dbc = ld_lds(D, (size_t)b * n + c);
            const float sd = fmaxf(dab, fmaxf(dac, dbc));
            if (sd <= thr && !((ld_lds(h1app, tx >> 5) >> (tx & 31)) & 1u)) {
                kind = 2;
                int p, q, w;
                if (dab == sd) p = a, q = b, w = c;
                else if (dac == sd) p = a, q = c, w = b;
                else p = b, q = c, w = a;
                // NB(w, sd): vertices within sd of w (sorted row, binary search)
                uint32_t lo = 0, hi = (uint32_t)n;
                const float* row = srow + (size_t)w * n;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (ld_lds(row, mid) <= sd) lo = mid + 1;
                    else hi = mid;
                }
                const uint64_t cand = ld_lds(Ae, (uint32_t)edge_id(p, q)) & ld_lds(pm, (size_t)w * (n + 1) + lo) & ~(1ull << w);
                if (cand) {
                    const int v = 63 - __clzll(cand);
                    const float dva = ld_lds(D, (size_t)v * n + a), dvb = ld_lds(D, (size_t)v * n + b), dvc = ld_lds(D, (size_t)v * n + c);
                    bool ap = true;
                    if (a > v) ap &= fmaxf(dbc, fmaxf(dvb, dvc)) < sd;
                    if (b > v) ap &= fmaxf(dac, fmaxf(dva, dvc)) < sd;
                    if (c > v) ap &= fmaxf(dab, fmaxf(dva, dvb)) < sd;
                    if (ap) {
                        kind = 1;
                        acs += pair_hash(tx, cofacet_index<2>(vs, v));
                        napp += 1;
                    }
                }
                if (kind == 2) rkey = ((2047u - (uint32_t)ld_lds(cls2, (size_t)p * n + q)) << 16) | tx;
            }
        }
        ncol += kind != 0;
        const uint64_t m = __ballot(kind == 2);
        if (m) {
            uint32_t b0 = 0;
            if (ln == __builtin_ctzll(m)) b0 = __hip_atomic_fetch_add((TDA_LDS uint32_t*)hdr + 1, (uint32_t)__popcll(m), __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
            b0 = (uint32_t)__shfl((int)b0, __builtin_ctzll(m), 64);
            const uint32_t pos = b0 + lanes_below(m);
            if (kind == 2 && pos < kF2Cap) st_lds(resk, pos, rkey);
        }
    }
    acs = wave_sum_u64(acs);
    napp = wave_sum_u64(napp);
    ncol = wave_sum_u64(ncol);
    if (ln == 0) {
        if (napp) {
            atomicAdd((unsigned long long*)&st->checksum[2], (unsigned long long)acs);
            atomicAdd((unsigned long long*)&st->all_pairs[2], (unsigned long long)napp);
        }
        if (ncol) atomicAdd((unsigned long long*)&st->n_columns[2], (unsigned long long)ncol);
    }
    __syncthreads();
    const uint32_t nres = ld_lds(hdr, 1u);
    if (nres > kF2Cap) {  // too many H2 columns for the LDS lists: the multi-kernel path takes the batch
        if (wv == 0) fused_fail(F, l, st);
        return;
    }
    if (F.stop == 3) {
        if (wv == 0) fused_fail(F, l, st);
        return;
    }
    // ---- B5: residual columns in column order (diam desc, idx asc)
    {
        const uint32_t P = fpow2(nres < 2 ? 2 : nres);
        for (uint32_t i = nres + t; i < P; i += kFT) st_lds(resk, i, 0xFFFFFFFFu);
        __syncthreads();
        lds_bitonic(resk, P, t, kFT, []() { __syncthreads(); });
    }
    if (t == 0) st->n_residual[2] = (int64_t)nres;
    if (F.stop == 4) {
        if (wv == 0) fused_fail(F, l, st);
        return;
    }
    // ---- B6: phase 1 on every wave: apparent-only additions per column
    const uint32_t* res1 = F.res1 + (size_t)l * F.res1_words;
    auto cleared = [&](uint32_t tx) -> bool {
        return (__hip_atomic_load(res1 + (tx >> 5), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (tx & 31)) & 1u;
    };
    uint32_t* p1k = F.p1_key + (size_t)l * kF2Cap;
    uint32_t* p1i = F.p1_info + (size_t)l * kF2Cap;
    uint32_t* roff = F.roff2 + (size_t)l * kF2Cap;
    uint32_t* rlen = F.rlen2 + (size_t)l * kF2Cap;
    uint64_t* pool = F.rpool2 + (size_t)l * F.rpool2_cap;
    {
        FSet S;
        S.k = (uint32_t*)(smem + cv.sets) + (size_t)wv * 2 * kFSet;
        S.pk = S.k + kFSet;
        S.cap = kFSet;
        S.clear();
#ifdef TDA_FUSED_DEBUG
        uint32_t dbg_it = 0;
#endif
        for (uint32_t it = 0; it <= nres; ++it) {  // a wave takes at most nres columns
            uint32_t j = 0;
            if (ln == 0) j = __hip_atomic_fetch_add((TDA_LDS uint32_t*)hdr + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            j = (uint32_t)__builtin_amdgcn_readlane((int)j, 0);  // lane 0's counter, whatever the exec mask
            if (j >= nres) break;
            const uint32_t rk = ld_lds(resk, j), tx = rk & 0xFFFFu, sc = 2047u - (rk >> 16);
            uint32_t out_key = kFEmpty, info = 0;
            if (cleared(tx)) {
                info = kP1Overflow;  // an H1 death: phase 2 skips it
            } else {
                int vs[3];
                decode<2>(tx, n, vs);
                uint32_t key, pk;
                bool ok;
                (void)f_cob(cls2, n, vs[0], vs[1], vs[2], sc, key, pk, ok);
                S.toggle(key, pk, ok);
                uint32_t adds = 0;
                for (uint32_t step = 0; step <= kP1MaxAdds + 1; ++step) {  // every pass either ends or adds
#ifdef TDA_FUSED_DEBUG
                    if (++dbg_it > 100000u) {
                        if (ln == 0) printf("[fused dbg] layer %d wave %d phase1 stuck: col %u/%u step %u adds %u used %u\n", l, wv, j, nres, step, adds, S.used);
                        info = kP1Overflow;
                        break;
                    }
#endif
                    if (adds >= kP1MaxAdds || ((step & 7) == 7 && cleared(tx))) {
                        info = kP1Overflow;
                        break;
                    }
                    uint32_t tp = 0;
                    const uint32_t pvk = S.pivot(tp);
                    if (pvk == kFEmpty) {  // zero column: essential
                        info = adds;
                        break;
                    }
                    uint32_t ck, cpk;
                    bool cok;
                    if (f_apparent(cls2, n, tp, pvk >> 20, ck, cpk, cok)) {
                        S.toggle(ck, cpk, cok);
                        ++adds;
                        if (S.used > kFSet / 2 && !S.compact(kFSet / 2 - 64)) {
                            info = kP1Overflow;
                            break;
                        }
                        continue;
                    }
                    // not apparent: phase 1 ends; store the working column
                    uint32_t nlive = 0;
                    for (uint32_t e = ln; e < kFSet; e += 64) nlive += ld_lds(S.k, e) < kFDead;
                    nlive = (uint32_t)wave_sum_u64(nlive);
                    uint32_t o = 0;
                    if (ln == 0) o = __hip_atomic_fetch_add((TDA_LDS uint32_t*)hdr + 4, nlive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    o = (uint32_t)__builtin_amdgcn_readlane((int)o, 0);
                    if ((uint64_t)o + nlive > F.rpool2_cap) {
                        info = kP1Overflow;
                        break;
                    }
                    (void)S.gather(pool + o, nlive);
                    if (ln == 0) {
                        st_glb(roff, j, o);
                        st_glb(rlen, j, nlive);
                    }
                    out_key = pvk;
                    info = adds;
                    break;
                }
                S.clear();
            }
            if (ln == 0) {
                st_glb(p1k, j, out_key);
                st_glb(p1i, j, info);
            }
        }
    }
    __syncthreads();  // phase-1 results (HBM) are complete for wave 0
    if (F.stop == 5) {
        if (wv == 0) fused_fail(F, l, st);
        return;
    }
    if (wv != 0) return;
    // ---- B7: wait for A (H1 residual pivots, dims 0-1 stats and pairs)
    if (ln == 0) {
        uint32_t s = 0;
        while (__hip_atomic_load(F.done + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u && ++s < kFSpin) __builtin_amdgcn_s_sleep(2);
        if (s >= kFSpin) st_lds(hdr, 5u, 1u);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    if (ld_lds(hdr, 5u)) {
        fused_fail(F, l, st);
        return;
    }
    if (F.stop == 6) {
        fused_fail(F, l, st);
        return;
    }
    // ---- B8: phase 2 (serial, column order) on wave 0
    Pair* P2p = F.pairs[2] + (size_t)l * F.pcap[2];
    uint32_t* tk = (uint32_t*)(smem + cv.tmap);   // pivot -> smallest column (conflict detection)
    uint32_t* tv = tk + 2 * kF2Cap;
    uint32_t* mk = (uint32_t*)(smem + cv.map);    // final pivot -> column
    uint32_t* mv = mk + 2 * kF2Cap;
    const uint32_t mcap = fpow2(2 * nres + 16) < 2 * kF2Cap ? fpow2(2 * nres + 16) : 2 * kF2Cap;
    for (uint32_t e = ln; e < mcap; e += 64) {
        st_lds(tk, e, kFEmpty);
        st_lds(tv, e, kFEmpty);
        st_lds(mk, e, kFEmpty);
    }
    wave_sync();
    auto col_cleared = [&](uint32_t j) -> bool {
        const uint32_t tx = ld_lds(resk, j) & 0xFFFFu;
        return (ld_glb(res1, tx >> 5) >> (tx & 31)) & 1u;
    };
    // prologue: columns before the first conflict pair with their phase-1 pivot
    for (uint32_t j = ln; j < nres; j += 64) {
        const uint32_t info = ld_glb(p1i, j), pk = ld_glb(p1k, j);
        if (!(info & kP1Overflow) && pk != kFEmpty && !col_cleared(j)) {
            uint32_t h = mix32(pk) & (mcap - 1);
            for (;;) {
                uint32_t cmp = kFEmpty;
                __hip_atomic_compare_exchange_strong((TDA_LDS uint32_t*)tk + h, &cmp, pk, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP);
                if (cmp == kFEmpty || cmp == pk) {
                    __hip_atomic_fetch_min((TDA_LDS uint32_t*)tv + h, j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
                h = (h + 1) & (mcap - 1);
            }
        }
    }
    wave_sync();
    uint32_t jc = nres;
    for (uint32_t j = ln; j < nres; j += 64) {
        const uint32_t info = ld_glb(p1i, j), pk = ld_glb(p1k, j);
        if (col_cleared(j)) continue;
        bool serial = (info & kP1Overflow) != 0;
        if (!serial && pk != kFEmpty) {
            uint32_t h = mix32(pk) & (mcap - 1);
            while (ld_lds(tk, h) != pk) h = (h + 1) & (mcap - 1);
            serial = ld_lds(tv, h) != j;
        }
        if (serial) jc = min(jc, j);
    }
    jc = wave_min_u32(jc);
    uint64_t cs = 0, npairs = 0, nadds = 0, nskip = 0, ecnt = 0;
    auto map_insert = [&](uint32_t key, uint32_t j) {  // one lane
        uint32_t h = mix32(key) & (mcap - 1);
        for (;;) {
            uint32_t cmp = kFEmpty;
            __hip_atomic_compare_exchange_strong((TDA_LDS uint32_t*)mk + h, &cmp, key, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
            if (cmp == kFEmpty) break;
            h = (h + 1) & (mcap - 1);
        }
        st_lds(mv, h, j);
    };
    auto map_find = [&](uint32_t key) -> uint32_t {  // wave-parallel probe
        for (uint32_t h0 = mix32(key);; h0 += 64) {
            const uint32_t kk = ld_lds(mk, (h0 + ln) & (mcap - 1));
            const uint64_t mhit = __ballot(kk == key), mend = __ballot(kk == kFEmpty);
            const uint64_t below_end = mend ? ((mend & (~mend + 1)) - 1) : ~0ull;
            if (mhit & below_end) return ld_lds(mv, (h0 + __builtin_ctzll(mhit & below_end)) & (mcap - 1));
            if (mend) return kFEmpty;
        }
    };
    auto lenof = [&](uint32_t key) -> float { return __uint_as_float(ld_lds(lenq, key >> 20)); };
    for (uint32_t j0 = 0; j0 < jc; j0 += 64) {
        const uint32_t j = j0 + ln;
        const bool act = j < jc;
        uint32_t info = 0, pk = kFEmpty, tx = 0, sc = 0;
        bool cl = false;
        if (act) {
            info = ld_glb(p1i, j);
            pk = ld_glb(p1k, j);
            const uint32_t rk = ld_lds(resk, j);
            tx = rk & 0xFFFFu;
            sc = 2047u - (rk >> 16);
            cl = col_cleared(j);
        }
        const float sd = __uint_as_float(ld_lds(lenq, sc));
        const bool ess = act && !cl && pk == kFEmpty;
        const bool pr = act && !cl && pk != kFEmpty;
        const float pd = pr ? lenof(pk) : 0.0f;
        const uint32_t pidx = 0xFFFFFu - (pk & 0xFFFFFu);
        const bool emit = ess || (pr && pd > sd);
        const uint64_t m = __ballot(emit);
        const uint64_t pos = ecnt + lanes_below(m);
        if (emit && pos < F.pcap[2]) store_pair(P2p, pos, sd, ess ? INFINITY : pd, (int64_t)tx, ess ? -1 : (int64_t)pidx);
        ecnt += (uint64_t)__popcll(m);
        if (pr) {
            cs += pair_hash(tx, pidx);
            ++npairs;
            map_insert(pk, j);
        }
        if (act && !cl) nadds += info;
        nskip += cl;
    }
    wave_sync();
    // serial walk from the first conflict (a pivot owned by an earlier column, or an overflow)
    FSet Wf;
    Wf.k = (uint32_t*)(smem + cv.wset);
    Wf.pk = Wf.k + kFSet2;
    Wf.cap = kFSet2;
    Wf.clear();
    uint64_t rused = ld_lds(hdr, 4u);
    int err = 0;
    // keep W below half full between 64-key passes (a pass adds at most 64 slots)
    auto room = [&]() -> bool { return Wf.used <= kFSet2 / 2 || Wf.compact(kFSet2 / 2 - 64); };
    auto add_stored = [&](uint32_t off, uint32_t len) -> bool {
        for (uint32_t e0 = 0; e0 < len; e0 += 64) {
            if (!room()) return false;
            const uint32_t e = e0 + ln;
            const uint64_t x = e < len ? ld_glb(pool, (size_t)off + e) : 0ull;
            Wf.toggle((uint32_t)x, (uint32_t)(x >> 32), e < len);
        }
        return true;
    };
    uint64_t tsteps = 0;  // every column's steps together: a non-cancelling pivot ends in ERR_FUSED, not a hang
    for (uint32_t j = jc; j < nres && !err; ++j) {
        const uint32_t rk = ld_lds(resk, j), tx = rk & 0xFFFFu, sc = 2047u - (rk >> 16);
        const float sd = __uint_as_float(ld_lds(lenq, sc));
        if (col_cleared(j)) {
            ++nskip;
            continue;
        }
        const uint32_t info = ld_glb(p1i, j), pk1 = ld_glb(p1k, j);
        if (!(info & kP1Overflow)) {
            nadds += info;
            if (pk1 == kFEmpty) {
                if (ln == 0 && ecnt < F.pcap[2]) store_pair(P2p, ecnt, sd, INFINITY, (int64_t)tx, -1);
                ++ecnt;
                continue;
            }
            const uint32_t own = map_find(pk1);
            if (own == kFEmpty) {  // new pair; R_j is the stored phase-1 column
                const float pd = lenof(pk1);
                const uint32_t pidx = 0xFFFFFu - (pk1 & 0xFFFFFu);
                if (pd > sd) {
                    if (ln == 0 && ecnt < F.pcap[2]) store_pair(P2p, ecnt, sd, pd, (int64_t)tx, (int64_t)pidx);
                    ++ecnt;
                }
                cs += pair_hash(tx, pidx);
                ++npairs;
                if (ln == 0) map_insert(pk1, j);
                wave_sync();
                continue;
            }
            if (!add_stored(ld_glb(roff, j), ld_glb(rlen, j))) {  // continue from the stored working column
                err = 1;
                break;
            }
        } else {
            int vs[3];
            decode<2>(tx, n, vs);
            uint32_t key, pk;
            bool ok;
            (void)f_cob(cls2, n, vs[0], vs[1], vs[2], sc, key, pk, ok);
            Wf.toggle(key, pk, ok);
        }
        for (uint64_t step = 0;; ++step) {
            if (step >= F.step_limit || ++tsteps >= F.step_limit || !room()) {
                err = 1;
                break;
            }
            uint32_t tp = 0;
            const uint32_t pvk = Wf.pivot(tp);
            if (pvk == kFEmpty) {  // zero column: essential
                if (ln == 0 && ecnt < F.pcap[2]) store_pair(P2p, ecnt, sd, INFINITY, (int64_t)tx, -1);
                ++ecnt;
                break;
            }
            const uint32_t own = map_find(pvk);
            if (own != kFEmpty) {  // add the stored reduced column of the owner
                if (!add_stored(ld_glb(roff, own), ld_glb(rlen, own))) {
                    err = 1;
                    break;
                }
                ++nadds;
                continue;
            }
            uint32_t ck, cpk;
            bool cok;
            if (f_apparent(cls2, n, tp, pvk >> 20, ck, cpk, cok)) {
                Wf.toggle(ck, cpk, cok);
                ++nadds;
                continue;
            }
            // new pair (column j, pvk); R_j = live keys of W
            const float pd = lenof(pvk);
            const uint32_t pidx = 0xFFFFFu - (pvk & 0xFFFFFu);
            if (pd > sd) {
                if (ln == 0 && ecnt < F.pcap[2]) store_pair(P2p, ecnt, sd, pd, (int64_t)tx, (int64_t)pidx);
                ++ecnt;
            }
            cs += pair_hash(tx, pidx);
            ++npairs;
            uint32_t nlive = 0;
            for (uint32_t e = ln; e < kFSet2; e += 64) nlive += ld_lds(Wf.k, e) < kFDead;
            nlive = (uint32_t)wave_sum_u64(nlive);
            if (rused + nlive > F.rpool2_cap) {
                err = 1;
                break;
            }
            (void)Wf.gather(pool + rused, nlive);
            if (ln == 0) {
                st_glb(roff, j, (uint32_t)rused);
                st_glb(rlen, j, nlive);
                map_insert(pvk, j);
            }
            rused += nlive;
            wave_sync();
            break;
        }
        Wf.clear();
    }
    if (ln == 0) {
        if (ecnt > F.pcap[2]) atomicOr(&st->err, ERR_PAIR_CAP);
        st->count[2] = (int64_t)ecnt;
        atomicAdd((unsigned long long*)&st->checksum[2], (unsigned long long)cs);
        atomicAdd((unsigned long long*)&st->all_pairs[2], (unsigned long long)npairs);
        atomicAdd((unsigned long long*)&st->n_adds[2], (unsigned long long)nadds);
        atomicAdd((unsigned long long*)&st->n_columns[2], (unsigned long long)(0ull - nskip));
        st->nskip[2] = (int64_t)nskip;
    }
    wave_sync();
    if (F.stop == 7) err = 1;
    if (err) fused_fail(F, l, st);
    else fused_emit(F, l, 3, st);
}

// grid: maxdim 2: [0, L8) role A of layer l0 + b, [L8, 2 L8) role B; maxdim 1: role A only
template <int K>
__global__ __launch_bounds__(kFT) void k_dense_fused(FusedBufs F, int n, int maxdim, int l0, int Lc, int L8) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int b = blockIdx.x;
    if (b < L8) {
        if (b < Lc) fused_role_a<K>(F, l0 + b, n, maxdim, smem);
    } else if (b - L8 < Lc) {
        fused_role_b(F, l0 + b - L8, n, smem);
    }
}

}  // namespace tda
