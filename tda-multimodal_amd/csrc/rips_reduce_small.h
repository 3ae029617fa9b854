// rips_reduce_small.h -- serial reductions for N <= 64 (the 48-point sweep),
// laid out around where the additions actually are.  A Python model of the
// reduction (tools/phase_sim.py) over the 32-layer sweep shows:
//   * H1: a layer has <= 8 residual columns, but ONE of them can need ~170
//     apparent additions in a row (layer 25: 168 of the layer's 173).  That
//     chain is the critical path of the whole batch, so its per-addition cost
//     is what matters.  The working column W is a dense LDS bitmap over the
//     triangles in FILTRATION order (k_prep_* rank them), so the pivot is
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
// Triangle ranks (k_prep_*).  Every triangle t <= thresh is assigned to its
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
constexpr int kChainT = 1024;             // threads per k_h1_chain block (staging; the chain is wave 0)
constexpr int kP1Grid = 96;               // k_h2_phase1 blocks per layer at most (one wave each, strided columns; rips.hip sizes it by L)
constexpr uint32_t kP1WCap = 512;         // phase-1 toggle-set capacity
constexpr int kChainMaxCols = 512;        // non-cleared H1 residual columns / stored R_j per layer
constexpr int kMaxK = 21;                 // bitmap words per lane: ceil(C(64,3) / 32 / 64)

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
typedef unsigned int rec_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ EdgeRecV rec_fields(rec_u32x4 q) {
    EdgeRecV v;
    v.M = (uint64_t)q.x | ((uint64_t)q.y << 32);
    v.off = q.z & 0xFFFFu;
    v.a = (int)((q.z >> 16) & 63u);
    v.b = (int)((q.z >> 22) & 63u);
    v.tie = (q.z >> 28) & 1u;
    v.len = __uint_as_float(q.w);
    return v;
}
__device__ __forceinline__ EdgeRecV load_rec(const EdgeRec* R, uint32_t e) { return rec_fields(((const TDA_LDS rec_u32x4*)R)[e]); }
__device__ __forceinline__ EdgeRecV load_rec_glb(const EdgeRec* R, uint32_t e) { return rec_fields(((const TDA_GLB rec_u32x4*)R)[e]); }

struct DenseBufs {
    EdgeRec* recs;      // [L][E]
    uint32_t* cls;      // [L][E] rank range of the edge's length class: cs | ce << 16 (tie path)
    uint16_t* inv;      // [L][inv_stride] rank -> edge | kInvFirst | kInvTie (kInvRes set by the TABLE chain in LDS)
    uint32_t* inv32;    // [L][inv_stride] rank -> a | b << 6 | w << 12 | first << 18 | tie << 19 (FAST path)
    uint16_t* rank_of;  // [L][tri_stride] triangle colex index -> rank, 0xFFFF above thresh (FAST path)
    uint32_t tri_stride;
    uint16_t* cls2;     // [L][n2p] length-class rank of edge (u, v) at u * n + v; 0xFFFF above thresh (H2 phase 1)
    uint32_t n2p;
    uint32_t* res1;     // [L][piv_words1] colex bitmap of residual H1 pivots (H2 clearing; zeroed per call)
    uint32_t* epos;     // [L][E] rank of the edge among edges <= thresh (kNoRank above)
    uint64_t* eM;       // [L][E] block masks
    uint32_t* necnt;    // [L] edges <= thresh (zeroed per call)
    uint16_t* cobt;     // [L][cob_stride] TABLE chain: rank of {a, b, v} at e * n + v
    uint32_t cob_stride;
    uint32_t E, inv_stride;
    int K;              // bitmap words per lane (W = 64 K words)
};

// ---------------------------------------------------------------- ranks
// Triangle ranks in three launches, spread over kPrepEdges-edge blocks so a
// layer's edge work is not serialised on one CU:
//   k_prep_edges   rank of each edge <= thresh in (length, index) order by
//                  counting smaller 64-bit keys; its block mask M_e; by rank:
//                  the block size and the length bits
//   k_prep_tables  recs / cls / cls2 and the rank tables: inv16[rank] = edge
//                  | first | tie; FAST: inv32[rank] = a | b << 6 |
//                  w << 12 | first << 18 | tie << 19 and rank_of[triangle]
//                  (0xFFFF above thresh); TABLE: cobt[e][v] = rank of
//                  {a, b, v} from its youngest facet's block
constexpr int kPrepEdges = 256;  // edges per k_prep_edges mask block (16 per wave)
constexpr uint32_t kNoRank = 0xFFFFFFFFu;
// inv16[rank] = edge | flags (edge < 2048 for N <= 64)
constexpr uint32_t kInvEdge = 0x7FFu, kInvFirst = 1u << 11, kInvTie = 1u << 12, kInvRes = 1u << 13;
// k_h1_chain variants (template MODE)
constexpr int kChainGeneral = 0, kChainFast = 1, kChainTable = 2;

// Grid (L, nb + 1), nb = ceil(E / kPrepEdges), kPrepT threads.  Blocks
// y >= 1: the block masks M_e of their kPrepEdges edges (wave per edge, lane
// = third vertex).  Block y == 0: the ranks -- one bitonic sort of the
// layer's (length bits, edge index) keys in LDS; rank = position among the
// edges <= thresh (they sort first; keys are unique, so this equals the count
// of smaller keys that r03 computed with E x E comparisons in every block).
// Sort stages with j <= 64 stay inside one wave's 128 keys: register
// shuffles, no LDS and no block barrier (TDA_PROFILE, a 36-point layer: the
// network takes 14 of the kernel's 17 us; r06: counting smaller keys instead,
// in this block or in every block, was slower or no shorter).  k_prep_tables
// derives the per-rank block sizes and lengths from M_e and the ranks.
constexpr int kPrepT = 1024;
__global__ __launch_bounds__(kPrepT) void k_prep_edges(const float* __restrict__ dist, int n, const uint32_t* __restrict__ rowmax,
                                                       float user_thresh, DenseBufs db, int cmode, LayerStats* __restrict__ stats) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int NW = kPrepT / 64, EPW = kPrepEdges / NW;  // waves, edges per wave
    const int l = blockIdx.x, t = threadIdx.x, ln = t & 63, wv = t >> 6;
#ifdef TDA_PROFILE  // wall-clock ticks (100 MHz) from the block's entry: the sort block [0..3], the mask blocks' max [4..6]
    const uint64_t pe0 = wall_clock64();
#define PE_STAMP(i) do { if (t == 0) atomicMax((unsigned long long*)&stats[l].prof[4][i], (unsigned long long)(wall_clock64() - pe0)); } while (0)
#else
#define PE_STAMP(i) (void)stats
#endif
    const int E = n * (n - 1) / 2;
    const int nb = (E + kPrepEdges - 1) / kPrepEdges;
    const float r = block_thresh(rowmax + (size_t)l * n, n, user_thresh, (uint32_t*)smem);
    PE_STAMP(blockIdx.y == 0 ? 0 : 4);
    float* D = (float*)(smem + 16);
    stage_to_lds(D, dist + (size_t)l * n * n, 4ull * n * n, t, kPrepT);
    __syncthreads();
    PE_STAMP(blockIdx.y == 0 ? 1 : 5);
    if (blockIdx.y == 0) {  // ranks (y = 0: dispatched first, the long pole overlaps the mask blocks)
        TDA_LDS uint64_t* keys = (TDA_LDS uint64_t*)(D + ((n * n + 3) & ~3));  // [P]
        int P = 2;
        while (P < E) P <<= 1;
        // thread t holds keys 2t and 2t + 1 in registers; a stage's partner is
        // in the same thread (j = 1), in lane t ^ j/2 of the same wave (j <= 64:
        // a wave holds 128 consecutive keys) or, for j >= 128, read through LDS
        auto key_of = [&](int i) -> uint64_t {
            if (i >= E) return ~0ull;
            int a, b;
            edge_verts((uint32_t)i, a, b);
            return ((uint64_t)__float_as_uint(D[a * n + b]) << 32) | (uint32_t)i;
        };
        const int i0 = 2 * t;
        const bool mine = i0 < P;
        uint64_t x0 = key_of(i0), x1 = key_of(i0 + 1);
        for (int k = 2; k <= P; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                uint64_t y0, y1;
                if (j >= 128) {
                    if (mine) {
                        keys[i0] = x0;
                        keys[i0 + 1] = x1;
                    }
                    __syncthreads();
                    y0 = mine ? keys[i0 ^ j] : ~0ull;
                    y1 = mine ? keys[(i0 + 1) ^ j] : ~0ull;
                    __syncthreads();  // every read done before the next stage's writes
                } else if (j >= 2) {
                    y0 = shfl_xor_u64(x0, j >> 1);
                    y1 = shfl_xor_u64(x1, j >> 1);
                } else {
                    y0 = x1;
                    y1 = x0;
                }
                const bool asc = (i0 & k) == 0;                   // the same for i0 and i0 + 1 (k >= 2)
                const bool lo0 = (i0 & j) == 0, lo1 = ((i0 + 1) & j) == 0;
                x0 = (lo0 == asc) ? (x0 < y0 ? x0 : y0) : (x0 < y0 ? y0 : x0);
                x1 = (lo1 == asc) ? (x1 < y1 ? x1 : y1) : (x1 < y1 ? y1 : x1);
            }
        if (mine) {
            keys[i0] = x0;
            keys[i0 + 1] = x1;
        }
        __syncthreads();
        PE_STAMP(2);
        uint32_t* ep = db.epos + (size_t)l * db.E;
        for (int q = t; q < E; q += kPrepT) {
            const uint64_t k = keys[q];
            const bool in = __uint_as_float((uint32_t)(k >> 32)) <= r;
            st_glb(ep, (size_t)(uint32_t)k, in ? (uint32_t)q : kNoRank);
            // edges <= thresh sort first: the last of them writes their count
            if (in && (q + 1 == E || !(__uint_as_float((uint32_t)(keys[q + 1] >> 32)) <= r))) st_glb(db.necnt, (size_t)l, (uint32_t)(q + 1));
        }
        PE_STAMP(3);
        return;
    }
    const int mb = blockIdx.y - 1;  // mask block 0 .. nb-1
    const int e0 = mb * kPrepEdges;
    if (cmode == kChainFast) {  // this block's share of "every triangle above the threshold"
        uint32_t* ro = (uint32_t*)(db.rank_of + (size_t)l * db.tri_stride);
        const uint32_t words = db.tri_stride / 2, per = (words + nb - 1) / nb;
        const uint32_t w0 = mb * per, w1 = min(words, w0 + per);
        for (uint32_t i = w0 + t; i < w1; i += kPrepT) st_glb(ro, i, 0xFFFFFFFFu);
    }
    // block masks: wave per edge (4 in flight), lane = third vertex
    for (int i0 = 0; i0 < EPW; i0 += 4) {
        float dav[4], dbv[4], lev[4];
        int av[4], bv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = e0 + wv * EPW + i0 + u;
            int a = 0, b = 0;
            if (e < E) edge_verts((uint32_t)e, a, b);
            av[u] = a;
            bv[u] = b;
            lev[u] = e < E ? D[a * n + b] : INFINITY;
            dav[u] = ln < n ? D[a * n + ln] : 0.0f;
            dbv[u] = ln < n ? D[b * n + ln] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = e0 + wv * EPW + i0 + u;
            const int a = av[u], b = bv[u], v = ln;
            const float le = lev[u];
            bool ok = e < E && le <= r && v < n && v != a && v != b && dav[u] <= le && dbv[u] <= le;
            if (ok && dav[u] == le && edge_id(a, v) < (uint32_t)e) ok = false;  // (a, v) is the younger facet
            if (ok && dbv[u] == le && edge_id(b, v) < (uint32_t)e) ok = false;
            const uint64_t m = __ballot(ok);
            if (ln == 0 && e < E) st_glb(db.eM + (size_t)l * db.E, (size_t)e, m);
        }
    }
    PE_STAMP(6);
#undef PE_STAMP
}

// tables: kPrepTabBlocks blocks of 1024 threads per layer.  Every block
// stages the layer's per-edge words (rank, block mask) and per-rank words
// (first triangle rank, class range, class start) in LDS, so the
// coboundary rows' youngest-facet lookups are LDS gathers; then one wave per
// edge writes its record, class words and rank-table entries, and (TABLE)
// its coboundary row, lane v -> rank of {a, b, v}.
constexpr int kPrepTabBlocks = 4;
constexpr int kPrepTabT = 1024;
__host__ __device__ constexpr size_t prep_tables_lds(int n) {
    return 16 + (((size_t)4 * n * n + 15) & ~(size_t)15) + (size_t)(n * (n - 1) / 2 + 8) * (8 + 4 + 4 + 4 + 4 + 4) + 64;
}
// The per-layer scan (block sizes in rank order -> first triangle rank of
// every block, and each rank's length class) is folded in: every block of the
// layer redoes it in LDS from k_prep_edges' raw sizes and lengths (at most
// C(64,2) = 2016 ranks), which takes one launch and one dependency hop off the
// critical path (it was k_prep_scan).
__global__ __launch_bounds__(kPrepTabT) void k_prep_tables(const float* __restrict__ dist, int n, DenseBufs db, int cmode,
                                                           LayerStats* __restrict__ stats) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.x, t = threadIdx.x, ln = t & 63, wv = t >> 6;
    constexpr int NW = kPrepTabT / 64;
    const int E = n * (n - 1) / 2;
    const int ES = E + 8;
    float* D = (float*)(smem + 16);
    uint64_t* Ms = (uint64_t*)(smem + 16 + (((size_t)4 * n * n + 15) & ~(size_t)15));  // [E] by edge
    uint32_t* ep = (uint32_t*)(Ms + ES);                                             // [E] edge -> rank
    uint32_t* fr = ep + ES;                                                          // [nE + 1] rank -> first triangle rank
    uint32_t* cl = fr + ES;                                                          // [nE] rank -> class triangle range
    uint32_t* qt = cl + ES;                                                          // [nE] rank -> class start | tie << 16
    uint32_t* lens = qt + ES;                                                        // [nE] rank -> length bits
    uint32_t* wsum = lens + ES;                                                      // [NW]
    const size_t lE = (size_t)l * db.E;
    stage_to_lds(D, dist + (size_t)l * n * n, 4ull * n * n, t, kPrepTabT);
    const uint32_t nE = ld_glb(db.necnt, (size_t)l);
    for (int e = t; e < E; e += kPrepTabT) {
        Ms[e] = ld_glb(db.eM + lE, (size_t)e);
        ep[e] = ld_glb(db.epos + lE, (size_t)e);
    }
    __syncthreads();
    // by rank: block size |M_e| and length bits of the ranked edges
    for (int e = t; e < E; e += kPrepTabT) {
        const uint32_t rk = ep[e];
        if (rk != kNoRank) {
            int a, b;
            edge_verts((uint32_t)e, a, b);
            fr[rk] = (uint32_t)__popcll(Ms[e]);
            lens[rk] = __float_as_uint(D[a * n + b]);
        }
    }
    __syncthreads();
    // scan: block sizes by rank -> exclusive prefix (fr[nE] = triangles <= thresh)
    const uint32_t per = (nE + kPrepTabT - 1) / kPrepTabT, q0 = t * per, q1 = min(nE, q0 + per);
    uint32_t loc = 0;
    for (uint32_t q = q0; q < q1; ++q) loc += fr[q];
    uint32_t x = loc;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (ln >= o) x += y;
    }
    if (ln == 63) wsum[wv] = x;
    __syncthreads();
    uint32_t run = x - loc, tot = 0;
    for (int w = 0; w < NW; ++w) {
        run += w < wv ? wsum[w] : 0u;
        tot += wsum[w];
    }
    for (uint32_t q = q0; q < q1; ++q) {
        const uint32_t v = fr[q];
        fr[q] = run;
        run += v;
    }
    if (t == 0) {
        fr[nE] = tot;
        if (blockIdx.y == 0) stats[l].ntri = tot;
    }
    __syncthreads();
    for (uint32_t q = t; q < nE; q += kPrepTabT) {  // length classes (short except on lattice-like inputs)
        const uint32_t len = lens[q];
        uint32_t a = q, b = q;
        while (a > 0 && lens[a - 1] == len) --a;
        while (b + 1 < nE && lens[b + 1] == len) ++b;
        cl[q] = fr[a] | (fr[b + 1] << 16);
        qt[q] = a | ((uint32_t)(b > a) << 16);
    }
    __syncthreads();
    EdgeRec* R = db.recs + lE;
    uint16_t* c2 = db.cls2 + (size_t)l * db.n2p;
    uint16_t* inv = db.inv + (size_t)l * db.inv_stride;
    uint32_t* inv32 = db.inv32 + (size_t)l * db.inv_stride;
    uint16_t* ro = db.rank_of + (size_t)l * db.tri_stride;
    uint16_t* ct = db.cobt + (size_t)l * db.cob_stride;
    for (int e = blockIdx.y * NW + wv; e < E; e += gridDim.y * NW) {
        int a, b;
        edge_verts((uint32_t)e, a, b);
        const uint32_t rk = ep[e];
        const float len = D[a * n + b];
        if (rk == kNoRank) {  // above the threshold: owns no triangles, no coboundary
            if (ln == 0) {
                EdgeRec rec = {};
                rec.ab = (uint16_t)(a | (b << 6));
                rec.len = len;
                R[e] = rec;
                st_glb(c2, (size_t)a * n + b, (uint16_t)0xFFFFu);
                st_glb(c2, (size_t)b * n + a, (uint16_t)0xFFFFu);
            }
            if (cmode == kChainTable && ln < n) st_glb(ct, (size_t)e * n + ln, (uint16_t)0xFFFFu);
            continue;
        }
        const uint64_t M = Ms[e];
        const uint32_t off = fr[rk], q = qt[rk];
        const bool tie = (q >> 16) & 1u;
        if (ln == 0) {
            EdgeRec rec;
            rec.M = M;
            rec.off = (uint16_t)off;
            rec.ab = (uint16_t)(a | (b << 6) | ((uint32_t)tie << 12));
            rec.len = len;
            R[e] = rec;
            st_glb(db.cls + lE, (size_t)e, cl[rk]);
            st_glb(c2, (size_t)a * n + b, (uint16_t)(q & 0xFFFFu));
            st_glb(c2, (size_t)b * n + a, (uint16_t)(q & 0xFFFFu));
        }
        if ((uint32_t)ln < (uint32_t)__popcll(M))
            st_glb(inv, off + ln, (uint16_t)(e | (ln == 0 ? kInvFirst : 0u) | (tie ? kInvTie : 0u)));
        if (cmode == kChainFast && ln < n && ((M >> ln) & 1ull)) {  // (TABLE decodes its rare steps from recs: r06)
            const uint32_t r2 = off + bits_above(M, ln);
            st_glb(inv32, r2, (uint32_t)a | ((uint32_t)b << 6) | ((uint32_t)ln << 12) | ((uint32_t)(r2 == off) << 18) | ((uint32_t)tie << 19));
            st_glb(ro, tri_id(a, b, ln), (uint16_t)r2);
        }
        if (cmode == kChainTable && ln < n) {
            // lane v: youngest facet e' of {a, b, v} (longest edge, ties ->
            // smallest index); the triangle is <= thresh iff e' is
            const int v = ln;
            uint16_t out = 0xFFFFu;
            if (v != a && v != b) {
                const float dav = D[a * n + v], dbv = D[b * n + v];
                float bl = len;
                uint32_t be = (uint32_t)e;
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
                const uint32_t rb = ep[be];
                if (rb != kNoRank) out = (uint16_t)(fr[rb] + bits_above(Ms[be], third));
            }
            st_glb(ct, (size_t)e * n + v, out);
        }
    }
}

// ---------------------------------------------------------------- H1 chain
// H1 of one layer.  All kChainT threads stage the layer's tables and filter
// the residual columns; then wave 0 alone runs the serial reduction (waves
// 1..15 leave; no s_barrier is issued after that point).  K = bitmap words per
// lane; the bitmap is word-major (word i = k * 64 + lane holds ranks
// [32 i, 32 i + 32)), so the pivot is the first lane of the first non-empty
// ballot over k.  MODE picks how a step finds the triangles:
//   kChainTable (N <= 48): cobt[e][v] is the coboundary of edge e by rank and
//     inv16[rank] carries edge | first | tie | residual, so an apparent step is
//     three dependent LDS reads (bitmap, inv16, cobt) and a ds_xor; the
//     rare new-pair / tie steps decode the triangle from its youngest facet's
//     HBM record (r06: no inv32 table -- 69 KB of writes per 48-point layer).
//   kChainFast (N <= ~51): rank_of[triangle] + inv32 in LDS.
//   kChainGeneral: edge records (youngest facet, block mask) + inv16.
// LDS: [16][D][recs E | rank_of | cobt][inv16 | inv32][W 64K][res 64K][piv][cols][own].
// The serial chain of k_h1_chain (wave 0 after the staging): every table
// pointer is the layer's (LDS
// where the MODE reads it from LDS), cols holds the nc non-cleared residual
// columns in column order, nskip the cleared ones (stats only).
struct ChainCtx {
    const float* Dl;
    const EdgeRec* R;
    const uint16_t* rof;
    const uint16_t* cobt;
    uint16_t* inv;
    const uint32_t* inv32;
    uint32_t* W;
    uint32_t* res;
    const uint32_t* piv;
    const uint64_t* cols;
    uint16_t* own;
    const float* Dg;
    const uint32_t* inv32g;
    const EdgeRec* Rg;  // the layer's edge records in HBM (TABLE: the rare steps' triangle decode)
    uint32_t* res1;
    uint32_t* pool;
    uint64_t pool_words;
    const uint32_t* clsg;
    Pair* P;
    uint64_t pcap;
    LayerStats* st;
    int n, l;
    uint32_t nc, nskip;
    uint64_t step_limit;
    uint64_t t_entry;
};
template <int K, int MODE>
__device__ __forceinline__ void h1_chain_wave(const ChainCtx& c) {
    constexpr bool FAST = MODE == kChainFast, TABLE = MODE == kChainTable, GEN = MODE == kChainGeneral;
    constexpr uint32_t WP = 64u * K;
    const float* Dl = c.Dl;
    const EdgeRec* R = c.R;
    const uint16_t* rof = c.rof;
    const uint16_t* cobt = c.cobt;
    uint16_t* inv = c.inv;
    const uint32_t* inv32 = c.inv32;
    uint32_t* W = c.W;
    uint32_t* res = c.res;
    const uint32_t* piv = c.piv;
    const uint64_t* cols = c.cols;
    uint16_t* own = c.own;
    const float* Dg = c.Dg;
    const uint32_t* inv32g = c.inv32g;
    const EdgeRec* Rg = c.Rg;
    uint32_t* res1 = c.res1;
    LayerStats* st = c.st;
    const int n = c.n, l = c.l, ln = lane_id();
    const uint32_t nc = c.nc, nskip = c.nskip;
    const uint64_t step_limit = c.step_limit, pcap = c.pcap;
#ifdef TDA_PROFILE
    const uint64_t t_entry = c.t_entry;
#endif
    (void)Dl, (void)R, (void)rof, (void)cobt, (void)inv32, (void)res, (void)Dg, (void)inv32g, (void)Rg, (void)l;
    const float r = st->thresh;
    Pair* P = c.P;
    uint32_t* pool = c.pool;
    const uint64_t pool_words = c.pool_words;
    const uint32_t* clsg = c.clsg;
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
        if constexpr (TABLE) {
            if (v < n) {
                const uint32_t rk = ld_lds(cobt, (size_t)edge_id(a, b) * n + v);
                if (rk != 0xFFFFu) lds_xor(&W[rk >> 5], 1u << (rk & 31));
            }
            return;
        }
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
    // the TABLE coboundary of edge e
    auto cob_e = [&](uint32_t e) {
        if (ln < n) {
            const uint32_t rk = ld_lds(cobt, (size_t)e * n + ln);
            if (rk != 0xFFFFu) lds_xor(&W[rk >> 5], 1u << (rk & 31));
        }
    };
    // first set bit of W (wave-uniform), false if W is empty; TABLE: also
    // inv16 of it, loaded per lane for the lane's own first bit while the
    // ballots run
    auto first_bit = [&](uint32_t& rk, uint32_t& qv) -> bool {
        uint32_t w[K];
#pragma unroll
        for (int k = 0; k < K; ++k) w[k] = ld_lds(W, (size_t)k * 64 + ln);
        uint32_t ws = 0, kk = 0;
#pragma unroll
        for (int k = K - 1; k >= 0; --k)
            if (w[k]) {
                ws = w[k];
                kk = (uint32_t)k;
            }
        const uint32_t rl = ((kk * 64u + (uint32_t)ln) << 5) + (uint32_t)__builtin_ctz(ws | 0x80000000u);
        uint32_t ql = 0;
        if constexpr (TABLE) ql = ld_lds(inv, ws ? rl : 0u);
        uint64_t m = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            m = __ballot(w[k] != 0u);
            if (m) break;
        }
        if (!m) return false;
        const int f = __builtin_ctzll(m);
        rk = (uint32_t)__builtin_amdgcn_readlane((int)rl, f);
        if constexpr (TABLE) qv = (uint32_t)__builtin_amdgcn_readlane((int)ql, f);
        return true;
    };
    // first set bit at rank >= lo, where every bit below lo is known to be
    // clear: one read of the 64 words from lo on (a column's pivot only moves
    // forward, and usually not far), the full scan when those are empty
    auto first_bit_from = [&](uint32_t lo, uint32_t& rk, uint32_t& qv) -> bool {
        const uint32_t wi = (lo >> 5) + (uint32_t)ln;
        uint32_t x = wi < WP ? ld_lds(W, wi) : 0u;
        if (ln == 0) x &= ~0u << (lo & 31);
        const uint32_t rl = (wi << 5) + (uint32_t)__builtin_ctz(x | 0x80000000u);
        uint32_t ql = 0;
        if constexpr (TABLE) ql = ld_lds(inv, x ? rl : 0u);
        const uint64_t m = __ballot(x != 0u);
        if (!m) return first_bit(rk, qv);
        const int f = __builtin_ctzll(m);
        rk = (uint32_t)__builtin_amdgcn_readlane((int)rl, f);
        if constexpr (TABLE) qv = (uint32_t)__builtin_amdgcn_readlane((int)ql, f);
        return true;
    };
    // vertices of the triangle at rank rk (a > b: its youngest facet, w: third vertex)
    auto decode = [&](uint32_t rk, int& a, int& b2, int& w) {
        if constexpr (GEN) {
            const EdgeRecV q = load_rec(R, ld_lds(inv, rk) & kInvEdge);
            a = q.a;
            b2 = q.b;
            w = kth_highest(q.M, rk - q.off);
        } else if constexpr (FAST) {
            const uint32_t q = ld_lds(inv32, rk);
            a = (int)(q & 63u);
            b2 = (int)((q >> 6) & 63u);
            w = (int)((q >> 12) & 63u);
        } else {  // TABLE: the youngest facet from inv16, its block from the HBM record (no inv32 table)
            const EdgeRecV q = load_rec_glb(Rg, ld_lds(inv, rk) & kInvEdge);
            a = q.a;
            b2 = q.b;
            w = kth_highest(q.M, rk - q.off);
        }
    };

    for (uint32_t j = 0; j < nc && !err; ++j) {
        const uint64_t key = ld_lds(cols, j);
        const uint32_t sidx = (uint32_t)key_idx(key);
        const float sdm = key_diam(key);
        if constexpr (TABLE) {
            cob_e(sidx);
        } else {
            int a0, b0;
            edge_verts(sidx, a0, b0);
            cob(a0, b0, sdm);
        }
        lds_order();
        uint32_t lo = 0;  // every bit of W below rank lo is clear
        for (uint64_t step = 0;; ++step) {
            if (step >= step_limit) {
                if (ln == 0) printf("h1_chain: layer %d column %u step limit\n", l, j);
                err = 3;
                break;
            }
            TDA_STAMP(t1);
            uint32_t rk = 0, qv = 0;
            bool found;
            if constexpr (TABLE) {
                // apparent run: window pivot -> inv16 -> coboundary row, for
                // as long as the pivot is the first triangle of a non-tie,
                // non-residual block (one ballot, two scalar reads per step)
                found = false;
                bool win = true;
                while (step < step_limit) {
                    const uint32_t w0 = lo >> 5, wi = w0 + (uint32_t)ln;
                    uint32_t x = wi < WP ? ld_lds(W, wi) : 0u;
                    if (ln == 0) x &= ~0u << (lo & 31);
                    const uint64_t m = __ballot(x != 0u);
                    if (!m) {
                        win = false;
                        break;
                    }
                    const int f = __builtin_ctzll(m);
                    const uint32_t wd = (uint32_t)__builtin_amdgcn_readlane((int)x, f);
                    rk = ((w0 + (uint32_t)f) << 5) + (uint32_t)__builtin_ctz(wd);
                    qv = (uint32_t)__builtin_amdgcn_readfirstlane((int)ld_lds(inv, rk));
                    if ((qv & (kInvFirst | kInvTie | kInvRes)) != kInvFirst) {
                        found = true;
                        break;
                    }
                    lo = rk + 1;  // the added column starts at rk, which cancels
                    cob_e(qv & kInvEdge);
                    ++nadds;
                    ++step;
                    lds_order();
                }
                if (step >= step_limit) continue;  // the loop head reports it
                if (!win) found = first_bit(rk, qv);
            } else {
                found = first_bit_from(lo, rk, qv);
            }
#ifdef TDA_PROFILE
            prof[7] += 1;
#endif
            if (!found) {  // zero column: essential class
                if (ln == 0 && ecnt < pcap) store_pair(P, ecnt, sdm, INFINITY, (int64_t)sidx, -1);
                ++ecnt;
                TDA_ACC(1, t1);
                break;
            }
            if constexpr (TABLE) {
                if ((qv & (kInvFirst | kInvTie | kInvRes)) == kInvFirst) {
                    // apparent pair (e, t): add the coboundary of the youngest facet e
                    TDA_ACC(1, t1);
                    TDA_STAMP(t2);
                    lo = rk + 1;  // the added column starts at rk, which cancels
                    cob_e(qv & kInvEdge);
                    ++nadds;
                    TDA_ACC(3, t2);
                    lds_order();
                    continue;
                }
            }
            bool isres, tie, first;
            int a = 0, b2 = 0, w = 0;
            uint32_t lo_next = rk + 1;
            if constexpr (TABLE) {
                isres = (qv & kInvRes) != 0;
                tie = (qv & kInvTie) != 0;
                first = (qv & kInvFirst) != 0;
                if (!isres && !tie) decode(rk, a, b2, w);
            } else {
                isres = (ld_lds(res, rk >> 5) >> (rk & 31)) & 1u;
                if constexpr (FAST) {
                    const uint32_t q = ld_lds(inv32, rk);
                    a = (int)(q & 63u);
                    b2 = (int)((q >> 6) & 63u);
                    w = (int)((q >> 12) & 63u);
                    first = (q >> 18) & 1u;
                    tie = (q >> 19) & 1u;
                } else {
                    const uint32_t qi = ld_lds(inv, rk);
                    const EdgeRecV q = load_rec(R, qi & kInvEdge);
                    a = q.a;
                    b2 = q.b;
                    tie = q.tie;
                    first = rk == q.off;
                    const uint32_t k = rk - q.off;
                    const int v = ln;
                    w = __builtin_ctzll(__ballot(((q.M >> v) & 1ull) && bits_above(q.M, v) == k));
                }
            }
            if (tie) {
                // tie class: the pivot is the set triangle of [cs, ce) with the largest index
#ifdef TDA_PROFILE
                ++ties;
#endif
                const uint32_t cc = ld_glb(clsg, TABLE ? (qv & kInvEdge) : edge_id(a, b2)), c0 = cc & 0xFFFFu, c1 = cc >> 16;
                lo_next = c0;  // inside the class rank order is not filtration order
                uint32_t best = 0, brk = rk;
                for (uint32_t base = c0; base < c1; base += 64) {
                    const uint32_t rho = base + ln;
                    uint32_t cand = 0;
                    if (rho < c1 && ((ld_lds(W, rho >> 5) >> (rho & 31)) & 1u)) {
                        int x, y, z;
                        decode(rho, x, y, z);
                        cand = tri_id(x, y, z) + 1;
                    }
                    const uint32_t m = wave_max_u32(cand);
                    if (m > best) {
                        best = m;
                        brk = base + (uint32_t)__builtin_ctzll(__ballot(cand == m));
                    }
                }
                rk = brk;
                if constexpr (TABLE) {
                    qv = ld_lds(inv, rk);
                    isres = (qv & kInvRes) != 0;
                } else {
                    isres = (ld_lds(res, rk >> 5) >> (rk & 31)) & 1u;
                }
                decode(rk, a, b2, w);
            }
            TDA_ACC(1, t1);
            TDA_STAMP(t2);
            if (isres) {
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
                for (int k = 0; k < K; ++k) st_lds(W, (size_t)k * 64 + ln, ld_lds(W, (size_t)k * 64 + ln) ^ x[k]);
                ++nadds;
                TDA_ACC(4, t2);
                lo = lo_next;
                lds_order();
                continue;
            }
            const uint32_t tidx = tri_id(a, b2, w);
            if (tie ? ((ld_lds(piv, tidx >> 5) >> (tidx & 31)) & 1u) : first) {
                // apparent pair (e, t): add the coboundary of the youngest facet e
                if constexpr (TABLE)
                    cob_e(edge_id(a, b2));
                else
                    cob(a, b2, FAST ? 0.0f : ld_lds(Dl, (size_t)a * n + b2));
                ++nadds;
                lo = lo_next;
                TDA_ACC(3, t2);
            } else {
                // new persistence pair (column, t); R_j = W
                const float pd = TABLE ? ld_glb(Dg, (size_t)a * n + b2) : ld_lds(Dl, (size_t)a * n + b2);
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
                    st_glb(dst, (size_t)k * 64 + ln, ld_lds(W, (size_t)k * 64 + ln));
                    st_lds(W, (size_t)k * 64 + ln, 0u);
                }
                if (ln == 0) {
                    st_lds(own, nown, (uint16_t)rk);
                    if constexpr (TABLE)
                        st_lds(inv, rk, (uint16_t)(ld_lds(inv, rk) | kInvRes));
                    else
                        st_lds(res, rk >> 5, ld_lds(res, rk >> 5) | (1u << (rk & 31)));
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
        prof[6] = t_all - t_entry;  // staging + column filter
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

template <int K, int MODE>
__global__ __launch_bounds__(kChainT) void k_h1_chain(const float* __restrict__ dist, int n, LayerStats* __restrict__ stats,
                                                      DimBufs b, Reduce2Bufs rb, DenseBufs db, uint64_t step_limit,
                                                      Pair* __restrict__ pairs, uint64_t pcap) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr bool FAST = MODE == kChainFast, TABLE = MODE == kChainTable, GEN = MODE == kChainGeneral;
    constexpr uint32_t WP = 64u * K;
#ifdef TDA_PROFILE
    const uint64_t t_entry = clock64();
#endif
    const int l = blockIdx.x, t = threadIdx.x, ln = t & 63, wv = t >> 6;
    LayerStats* st = stats + l;
    const int E = n * (n - 1) / 2;
    unsigned char* p = smem + 16;
    auto take = [&](size_t bytes) {
        unsigned char* q = p;
        p += (bytes + 15) & ~(size_t)15;
        return q;
    };
    float* Dl = TABLE ? nullptr : (float*)take(4ull * n * n);
    EdgeRec* R = GEN ? (EdgeRec*)take(16ull * E) : nullptr;
    uint16_t* rof = FAST ? (uint16_t*)take(2ull * db.tri_stride) : nullptr;
    uint16_t* cobt = TABLE ? (uint16_t*)take(2ull * db.cob_stride) : nullptr;
    uint16_t* inv = FAST ? nullptr : (uint16_t*)take(2ull * db.inv_stride);
    uint32_t* inv32 = FAST ? (uint32_t*)take(4ull * db.inv_stride) : nullptr;
    uint32_t* W = (uint32_t*)take(4ull * WP);
    uint32_t* res = TABLE ? nullptr : (uint32_t*)take(4ull * WP);  // ranks that are residual pivots
    uint32_t* piv = (uint32_t*)take(4ull * b.piv_words);  // colex bitmap of apparent pivots (tie classes)
    uint64_t* cols = (uint64_t*)take(8ull * kChainMaxCols);
    uint16_t* own = (uint16_t*)take(2ull * kChainMaxCols);

    const uint32_t ntri = (uint32_t)st->ntri;
    const float* Dg = dist + (size_t)l * n * n;
    const uint32_t* inv32g = db.inv32 + (size_t)l * db.inv_stride;
    if constexpr (!TABLE) stage_to_lds(Dl, Dg, 4ull * n * n, t, kChainT);
    if constexpr (FAST) {
        stage_to_lds(rof, db.rank_of + (size_t)l * db.tri_stride, 2ull * db.tri_stride, t, kChainT);
        stage_to_lds(inv32, inv32g, 4ull * ntri, t, kChainT);
    } else {
        if constexpr (GEN) stage_to_lds(R, db.recs + (size_t)l * db.E, 16ull * E, t, kChainT);
        if constexpr (TABLE) stage_to_lds(cobt, db.cobt + (size_t)l * db.cob_stride, 2ull * db.cob_stride, t, kChainT);  // whole words
        stage_to_lds(inv, db.inv + (size_t)l * db.inv_stride, 4ull * ((ntri + 1) / 2), t, kChainT);
    }
    const uint32_t* pivg = b.pivbits + (size_t)l * b.piv_words;
    uint32_t* res1 = db.res1 + (size_t)l * b.piv_words;
    stage_to_lds(piv, pivg, 4ull * b.piv_words, t, kChainT);
    for (uint32_t i = t; i < WP; i += kChainT) {
        st_lds(W, i, 0u);
        if constexpr (!TABLE) st_lds(res, i, 0u);
    }
    uint64_t nres = (uint64_t)st->n_residual[1];
    if (nres > b.rcap) nres = b.rcap;
    // drop H0 deaths (spanning-forest edges: cleared columns), keep column
    // order: ordered compaction over the whole block, kChainT columns a round
    uint32_t* wcnt = (uint32_t*)own;  // per-wave counts (own is unused until the chain)
    uint32_t nc = 0, nskip = 0;
    {
        const uint64_t* resid = b.resid + (size_t)l * b.rcap;
        const uint32_t* mst = rb.mst + (size_t)l * rb.mst_words;
        for (uint64_t j0 = 0; j0 < nres; j0 += kChainT) {
            const uint64_t j = j0 + t;
            uint64_t key = 0;
            bool keep = false;
            if (j < nres) {
                key = ld_glb(resid, j);
                const uint32_t s = (uint32_t)key_idx(key);
                keep = !((ld_glb(mst, s >> 5) >> (s & 31)) & 1u);
            }
            const uint64_t m = __ballot(keep);
            if (ln == 0) wcnt[wv] = (uint32_t)__popcll(m);
            __syncthreads();
            uint32_t below = 0, tot = 0;
            for (int q = 0; q < kChainT / 64; ++q) {
                const uint32_t c = wcnt[q];
                below += q < wv ? c : 0u;
                tot += c;
            }
            const uint32_t pos = nc + below + lanes_below(m);
            if (keep && pos < (uint32_t)kChainMaxCols) st_lds(cols, pos, key);
            const uint32_t valid = (uint32_t)min<uint64_t>(kChainT, nres - j0);
            nc += tot;
            nskip += valid - tot;
            __syncthreads();
        }
    }
    __syncthreads();  // staging done (also when there are no columns)
    if (wv != 0) return;
    ChainCtx c;
    c.Dl = Dl;
    c.R = R;
    c.rof = rof;
    c.cobt = cobt;
    c.inv = inv;
    c.inv32 = inv32;
    c.W = W;
    c.res = res;
    c.piv = piv;
    c.cols = cols;
    c.own = own;
    c.Dg = Dg;
    c.inv32g = inv32g;
    c.Rg = db.recs + (size_t)l * db.E;
    c.res1 = res1;
    c.pool = (uint32_t*)(rb.rpool + (size_t)l * rb.rpool_cap);
    c.pool_words = 2ull * rb.rpool_cap;
    c.clsg = db.cls + (size_t)l * db.E;
    c.P = pairs + (size_t)l * pcap;
    c.pcap = pcap;
    c.st = st;
    c.n = n;
    c.l = l;
    c.nc = nc;
    c.nskip = nskip;
    c.step_limit = step_limit;
#ifdef TDA_PROFILE
    c.t_entry = t_entry;
#endif
    h1_chain_wave<K, MODE>(c);
}
// bitmap words per lane supported by k_h1_chain instantiations (FAST / TABLE: up to 12)
constexpr int kChainKs[] = {1, 2, 3, 4, 6, 9, 12, 16, 21};
constexpr int kChainFastMaxK = 12;

// ---------------------------------------------------------------- H2 phase 1
// One wave per block; block (l, g) takes the layer's residual H2 columns
// g, g + gridDim.y, ... and reduces each with apparent columns only.  The
// whole step runs on 32-bit words:
//   * a tetrahedron's key is (class << 20) | (2^20 - 1 - colex index), where
//     class = rank of its longest edge's length among the sorted edges
//     (cls2, k_prep_tables): key order is Ripser's (diameter asc, index desc);
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

// Blocks of kP1MaxWaves (or 1, when two waves' bitmaps do not fit the LDS)
// independent waves: the layer's matrix and class table are staged once per
// block and shared; each wave has its own bitmap and log and takes its own
// columns (virtual one-wave block blockIdx.y * waves + wave).
constexpr int kP1MaxWaves = 2;
__global__ __launch_bounds__(64 * kP1MaxWaves) void k_h2_phase1(const float* __restrict__ dist, int n, LayerStats* __restrict__ stats,
                                                                DimBufs b, SmallBufs sb, const uint16_t* __restrict__ cls2g, uint32_t n2p,
                                                                uint32_t bm_words, const uint32_t* __restrict__ res1g, uint32_t res1_words,
                                                                uint64_t step_limit) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.x, ln = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint64_t vb = (uint64_t)blockIdx.y * nw + wv, vstride = (uint64_t)gridDim.y * nw;
    LayerStats* st = stats + l;
    uint64_t nres = (uint64_t)st->n_residual[2];
    if (nres > b.rcap) nres = b.rcap;
    if ((uint64_t)blockIdx.y * nw >= nres) return;  // the whole block is idle (uniform exit)
    const uint64_t* resid = b.resid + (size_t)l * b.rcap;
    unsigned char* p = smem + 16;
    auto take = [&](size_t bytes) {
        unsigned char* q = p;
        p += (bytes + 15) & ~(size_t)15;
        return q;
    };
    float* Dl = (float*)take(4ull * n * n);
    uint16_t* cls = (uint16_t*)take(2ull * n2p);
    for (int w = 0; w < wv; ++w) {  // the earlier waves' private regions
        (void)take(4ull * bm_words);
        (void)take(4ull * kP1LogCap);
        (void)take(4ull * kP1LogCap);
    }
    uint32_t* bm = (uint32_t*)take(4ull * bm_words);
    uint32_t* lk = (uint32_t*)take(4ull * kP1LogCap);
    uint32_t* lv = (uint32_t*)take(4ull * kP1LogCap);
    stage_to_lds(Dl, dist + (size_t)l * n * n, 4ull * n * n, threadIdx.x, blockDim.x);
    stage_to_lds(cls, cls2g + (size_t)l * n2p, 2ull * n2p, threadIdx.x, blockDim.x);
    for (uint32_t i = ln; i < bm_words; i += 64) st_lds(bm, i, 0u);
    __syncthreads();  // the shared matrix and class table; below, every wave works alone

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
    for (uint64_t j = vb; j < nres; j += vstride) {
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
