// rips_reduce_small.h -- serial reductions for N <= 64 (the 48-point sweep),
// laid out around where the additions actually are.  A Python model of the
// reduction (tools/phase_sim.py) over the 32-layer sweep shows:
//   * H1: a layer has <= 8 residual columns, but ONE of them can need ~170
//     apparent additions in a row (layer 25: 168 of the layer's 173).  That
//     chain is the critical path of the whole batch, so its per-addition cost
//     is what matters.  The working column W becomes a dense LDS bitmap over
//     all C(N,3) triangles (17,296 bits at N=48): a toggle is one ds_xor, no
//     hashing, no log, no capacity.  The pivot (min diam, then max index) is
//     found through per-diameter-class live counts: class = rank of the first
//     edge of that length in the sorted edge list (k_edge_class), so the
//     lowest non-empty class is one ballot over a 63-word summary, and its
//     live triangles {a, b, v} (max edge (a, b)) are one lane per v.
//   * H2: up to ~76 residual columns per layer with <= 13 additions each, and
//     over all 32 layers exactly one addition uses another RESIDUAL column;
//     every other addition is an apparent column, which does not depend on
//     any other column.  So H2 runs as phase 1 (apparent-only reduction,
//     column-parallel: K waves per layer, concurrently with the H1 chain) and
//     phase 2 (k_reduce_h2_finish: columns in order, O(1) each unless the
//     phase-1 pivot is owned by an earlier residual column, in which case the
//     stored working column is reloaded and reduced further, exactly like
//     Ripser would have continued).
// Phase 1 of a column performs exactly the first steps Ripser's serial loop
// performs on it (the serial loop consults residual owners first, and a
// pivot owned by an apparent column is never a residual pivot), so the
// result is bit-identical to the serial order.
#pragma once
#include "rips_reduce.h"

namespace tda {

constexpr int kDenseMaxN = 64;
constexpr int kP1Waves = 8;                 // H2 phase-1 waves per layer

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

// ---------------------------------------------------------------- edge classes
// Per layer: edges sorted by (length, a, b); cls[e] = position of the first
// edge with e's length (tied lengths share a class), srt[q] = a << 8 | b of
// the q-th edge.  One 256-thread block per layer, bitonic sort in LDS.
__global__ __launch_bounds__(256) void k_edge_class(const float* __restrict__ dist, int n, uint16_t* __restrict__ cls,
                                                   uint16_t* __restrict__ srt, int E2) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t* s = (uint64_t*)smem;
    const int l = blockIdx.x, t = threadIdx.x;
    const float* D = dist + (size_t)l * n * n;
    const int E = n * (n - 1) / 2;
    for (int q = t; q < E2; q += 256) {
        uint64_t k = kEmpty64;
        if (q < E) {
            int a, b;
            edge_verts((uint32_t)q, a, b);
            k = ((uint64_t)__float_as_uint(D[(size_t)a * n + b] + 0.0f) << 32) | ((uint32_t)a << 8) | (uint32_t)b;
        }
        s[q] = k;
    }
    __syncthreads();
    for (int k = 2; k <= E2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = t; i < E2; i += 256) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t x = s[i], y = s[ixj];
                    if ((x > y) == ((i & k) == 0)) {
                        s[i] = y;
                        s[ixj] = x;
                    }
                }
            }
            __syncthreads();
        }
    uint16_t* C = cls + (size_t)l * E2;
    uint16_t* S = srt + (size_t)l * E2;
    for (int q = t; q < E; q += 256) {
        const uint64_t k = s[q];
        const uint32_t len = (uint32_t)(k >> 32);
        int lo = 0, hi = q;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((uint32_t)(s[mid] >> 32) < len)
                lo = mid + 1;
            else
                hi = mid;
        }
        const int a = (int)((k >> 8) & 0xFF), b = (int)(k & 0xFF);
        C[c2u(a) + b] = (uint16_t)lo;
        S[q] = (uint16_t)((a << 8) | b);
    }
}

// ---------------------------------------------------------------- dense H1
struct DenseW {
    const float* D;      // LDS distance matrix
    uint32_t* W;         // LDS bitmap over triangles
    uint32_t* cnt;       // LDS live triangles per class [E]
    uint32_t* sum;       // LDS "class may be non-empty" bits [64]
    const uint16_t* cls; // LDS class of edge [E]
    const uint16_t* srt; // LDS sorted edges [E]
    int n, E, wwords, swords;
    float r;

    // toggle the coboundary of edge (x, y) (length fd, class cf): lane v -> {x, y, v}
    __device__ __forceinline__ void cob(int x, int y, float fd, uint32_t cf, int ln) const {
        const int v = ln;
        bool ok = v < n && v != x && v != y;
        float dx = 0.0f, dy = 0.0f;
        if (ok) {
            dx = ld_lds(D, (size_t)x * n + v);
            dy = ld_lds(D, (size_t)y * n + v);
        }
        const float cd = fmaxf(fd, fmaxf(dx, dy));
        ok = ok && cd <= r;
        const bool same = cd == fd;  // max edge has length fd: class cf
        uint32_t c = cf;
        if (ok && !same) c = ld_lds(cls, dx >= dy ? edge_id(x, v) : edge_id(y, v));
        bool was = false;
        if (ok) {
            const uint32_t idx = tri_id(x, y, v);
            const uint32_t bit = 1u << (idx & 31);
            was = (atomicXor(&W[idx >> 5], bit) & bit) != 0;
        }
        // class cf: one aggregated update (many lanes share it)
        const uint64_t mp = __ballot(ok && same && !was), mm = __ballot(ok && same && was);
        if (ln == 0 && (mp | mm)) {
            atomicAdd(&cnt[cf], (uint32_t)(__popcll(mp) - __popcll(mm)));
            if (mp) atomicOr(&sum[cf >> 5], 1u << (cf & 31));
        }
        if (ok && !same) toggle_count(c, was);
    }
    __device__ __forceinline__ void toggle_count(uint32_t c, bool was) const {
        if (was) {
            atomicSub(&cnt[c], 1u);
        } else {
            atomicAdd(&cnt[c], 1u);
            atomicOr(&sum[c >> 5], 1u << (c & 31));
        }
    }
    // toggle stored keys (class << 32 | triangle index), distinct
    __device__ __forceinline__ void toggle_keys(uint64_t k, bool ok) const {
        if (!ok) return;
        const uint32_t idx = (uint32_t)k, c = (uint32_t)(k >> 32);
        const uint32_t bit = 1u << (idx & 31);
        const bool was = (atomicXor(&W[idx >> 5], bit) & bit) != 0;
        toggle_count(c, was);
    }
    // pivot = live triangle of min (diam, -idx).  Returns false if W is empty.
    // Out: idx, vertices (a, b) = a max edge (a > b), v, the class and the
    // lengths |av|, |bv|.
    __device__ bool pivot(int ln, uint32_t& pidx, int& pa, int& pb, int& pv, uint32_t& pc, float& len, float& dav,
                          float& dbv) const {
        for (;;) {
            const uint32_t sw = ln < swords ? ld_lds(sum, ln) : 0u;
            const uint64_t nz = __ballot(sw != 0);
            if (!nz) return false;
            const int f = __builtin_ctzll(nz);
            const uint32_t w = __builtin_amdgcn_readlane(sw, f);
            const uint32_t c = (uint32_t)f * 32 + __builtin_ctz(w);
            if (ld_lds(cnt, c) == 0) {  // lazily cleared summary bit
                if (ln == 0) sum[c >> 5] = w & ~(1u << (c & 31));
                continue;
            }
            uint32_t best = 0;
            float lc = 0.0f;
            for (int q = (int)c; q < E; ++q) {
                const uint32_t e = ld_lds(srt, q);
                const int a = (int)(e >> 8), b = (int)(e & 0xFF);
                const float le = ld_lds(D, (size_t)a * n + b);
                if (q == (int)c)
                    lc = le;
                else if (le != lc)
                    break;
                const int v = ln;
                bool ok = v < n && v != a && v != b;
                float x = 0.0f, y = 0.0f;
                if (ok) {
                    x = ld_lds(D, (size_t)a * n + v);
                    y = ld_lds(D, (size_t)b * n + v);
                    ok = x <= lc && y <= lc;
                }
                const uint32_t idx = tri_id(a, b, v);
                ok = ok && ((ld_lds(W, idx >> 5) >> (idx & 31)) & 1u);
                const uint32_t cand = ok ? idx + 1 : 0u;
                const uint32_t m = wave_max_u32(cand);
                if (m > best) {
                    best = m;
                    const int lane = __builtin_ctzll(__ballot(cand == m));
                    pa = a;
                    pb = b;
                    pv = lane;
                    dav = __shfl(x, lane, 64);
                    dbv = __shfl(y, lane, 64);
                }
            }
            if (best == 0) {  // counts and bitmap disagree: cannot happen
                if (ln == 0) sum[c >> 5] = w & ~(1u << (c & 31));
                continue;
            }
            pidx = best - 1;
            pc = c;
            len = lc;
            return true;
        }
    }
    // append (class << 32 | idx) of every live triangle to out; returns count
    __device__ uint32_t gather(int ln, uint64_t* out) const {
        uint32_t pos = 0;
        for (int w0 = 0; w0 < wwords; w0 += 64) {
            const int wi = w0 + ln;
            uint32_t bits = wi < wwords ? ld_lds(W, wi) : 0u;
            while (__ballot(bits != 0)) {
                const bool has = bits != 0;
                uint64_t key = 0;
                if (has) {
                    const uint32_t idx = (uint32_t)wi * 32 + __builtin_ctz(bits);
                    bits &= bits - 1;
                    int t[3];
                    decode<2>(idx, n, t);
                    const float d01 = ld_lds(D, (size_t)t[0] * n + t[1]), d02 = ld_lds(D, (size_t)t[0] * n + t[2]),
                                d12 = ld_lds(D, (size_t)t[1] * n + t[2]);
                    const uint32_t e = (d01 >= d02 && d01 >= d12) ? edge_id(t[0], t[1]) : (d02 >= d12 ? edge_id(t[0], t[2]) : edge_id(t[1], t[2]));
                    key = ((uint64_t)ld_lds(cls, e) << 32) | idx;
                }
                const uint64_t m = __ballot(has);
                if (has) out[pos + lanes_below(m)] = key;
                pos += (uint32_t)__popcll(m);
            }
        }
        return pos;
    }
    __device__ void reset(int ln) const {
        for (int i = ln; i < wwords; i += 64) W[i] = 0;
        for (int i = ln; i < E; i += 64) cnt[i] = 0;
        for (int i = ln; i < swords; i += 64) sum[i] = 0;
    }
};


// H1 of one layer with the dense working column (one wave).
__device__ void reduce_h1_dense(const float* Dl, int n, float r, LayerStats* st, int l, const DimBufs& b, const Reduce2Bufs& rb,
                                const SmallBufs& sb, unsigned char* lds, uint64_t step_limit, Pair* __restrict__ pairs,
                                uint64_t pcap) {
    const int ln = threadIdx.x;
    const int E = n * (n - 1) / 2;
    uint64_t nres = (uint64_t)st->n_residual[1];
    if (nres > b.rcap) nres = b.rcap;
    const uint64_t* resid = b.resid + (size_t)l * b.rcap;
    uint32_t* pivg = b.pivbits + (size_t)l * b.piv_words;

    unsigned char* p = lds;
    auto take = [&](size_t bytes) {
        unsigned char* q = p;
        p += (bytes + 15) & ~(size_t)15;
        return q;
    };
    DenseW S;
    S.D = Dl;
    S.n = n;
    S.E = E;
    S.r = r;
    S.wwords = (int)((binom((uint64_t)n, 3) + 31) / 32);
    S.swords = (E + 31) / 32;
    S.W = (uint32_t*)take(4ull * S.wwords);
    S.cnt = (uint32_t*)take(4ull * E);
    S.sum = (uint32_t*)take(4ull * 64);
    uint16_t* cl = (uint16_t*)take(2ull * E);
    uint16_t* sr = (uint16_t*)take(2ull * E);
    uint32_t* piv = (uint32_t*)take(4ull * b.piv_words);
    // residual pivot map: LDS copy for probes, mirrored to HBM for H2 clearing
    uint64_t rcap2 = 16;
    while (rcap2 < 2 * nres + 16) rcap2 <<= 1;
    if (rcap2 > rb.rmap_stride) rcap2 = rb.rmap_stride;
    PivMap mg;
    mg.k = rb.rmap_keys + ((size_t)l * 2) * rb.rmap_stride;  // cleared by k_sort_resid
    mg.v = rb.rmap_vals + ((size_t)l * 2) * rb.rmap_stride;
    mg.mask = rcap2 - 1;
    PivMap ml = mg;
    const bool map_lds = rcap2 <= 1024;
    if (map_lds) {
        ml.k = (uint64_t*)take(8ull * rcap2);
        ml.v = (uint32_t*)take(4ull * rcap2);
        for (uint64_t e = ln; e < rcap2; e += 64) ml.k[e] = kEmpty64;
    }
    for (int i = ln; i < E; i += 64) {
        cl[i] = sb.cls[(size_t)l * sb.E2 + i];
        sr[i] = sb.srt[(size_t)l * sb.E2 + i];
    }
    stage_to_lds(piv, pivg, 4ull * b.piv_words, ln, 64);
    S.cls = cl;
    S.srt = sr;
    S.reset(ln);
    __syncthreads();

    const uint32_t* mst = rb.mst + (size_t)l * rb.mst_words;
    uint64_t* roff = rb.roff + (size_t)l * b.rcap;
    uint32_t* rlen = rb.rlen + (size_t)l * b.rcap;
    uint64_t* rpool = rb.rpool + (size_t)l * rb.rpool_cap;
    uint64_t rused = 0;
    Pair* P = pairs + (size_t)l * pcap;
    uint64_t cs = 0, npairs = 0, nadds = 0, nskip = 0;
    int err = 0;

    for (uint64_t j = 0; j < nres && !err; ++j) {
        const uint64_t key = ld_glb(resid, j);
        const uint32_t sidx = (uint32_t)key_idx(key);
        const float sdm = key_diam(key);
        if ((ld_glb(mst, sidx >> 5) >> (sidx & 31)) & 1u) {  // H0 death: cleared
            ++nskip;
            if (ln == 0) rlen[j] = 0;
            continue;
        }
        int a0, b0;
        edge_verts(sidx, a0, b0);
        S.cob(a0, b0, sdm, ld_lds(cl, sidx), ln);
        __syncthreads();
        for (uint64_t step = 0;; ++step) {
            if (step >= step_limit) {
                if (ln == 0) printf("reduce_h1_dense: layer %d column %llu step limit\n", l, (unsigned long long)j);
                err = 3;
                break;
            }
            uint32_t pidx, pc;
            int pa, pb, pv;
            float pd, dav, dbv;
            if (!S.pivot(ln, pidx, pa, pb, pv, pc, pd, dav, dbv)) {
                if (ln == 0) {  // essential class
                    const uint64_t pos = atomicAdd((unsigned long long*)&st->count[1], 1ull);
                    if (pos < pcap)
                        P[pos] = Pair{sdm, INFINITY, (int64_t)sidx, -1};
                    else
                        atomicOr(&st->err, ERR_PAIR_CAP);
                    rlen[j] = 0;
                }
                break;
            }
            int t[3] = {pa, pb, pv};  // descending for the packed payload
            if (t[1] < t[2]) { const int x = t[1]; t[1] = t[2]; t[2] = x; }
            if (t[0] < t[1]) { const int x = t[0]; t[0] = t[1]; t[1] = x; }
            if (t[1] < t[2]) { const int x = t[1]; t[1] = t[2]; t[2] = x; }
            const uint32_t plo = RowLo<3>::pack(t);
            const bool app = (ld_lds(piv, pidx >> 5) >> (pidx & 31)) & 1u;
            const int64_t owner = app ? ml.find(plo, ln) : -1;
            if (owner >= 0) {
                const uint64_t o0 = ld_glb((const uint64_t*)roff, owner);
                const uint32_t ol = ld_glb((const uint32_t*)rlen, owner);
                for (uint32_t e0 = 0; e0 < ol; e0 += 64) {
                    const uint32_t e = e0 + ln;
                    S.toggle_keys(e < ol ? ld_glb((const uint64_t*)rpool, o0 + e) : 0, e < ol);
                }
                ++nadds;
            } else if (app) {
                // youngest facet: max length (= pd), ties -> smallest edge index
                uint32_t fe = edge_id(pa, pb);
                int fx = pa, fy = pb;
                if (dav == pd && edge_id(pa, pv) < fe) {
                    fe = edge_id(pa, pv);
                    fx = pa;
                    fy = pv;
                }
                if (dbv == pd && edge_id(pb, pv) < fe) {
                    fe = edge_id(pb, pv);
                    fx = pb;
                    fy = pv;
                }
                S.cob(fx, fy, pd, pc, ln);
                ++nadds;
            } else {
                if (ln == 0) {
                    if (pd > sdm) {
                        const uint64_t pos = atomicAdd((unsigned long long*)&st->count[1], 1ull);
                        if (pos < pcap)
                            P[pos] = Pair{sdm, pd, (int64_t)sidx, (int64_t)pidx};
                        else
                            atomicOr(&st->err, ERR_PAIR_CAP);
                    }
                    if (map_lds) ml.insert(plo, (uint32_t)j);
                    mg.insert(plo, (uint32_t)j);
                    atomicOr(&piv[pidx >> 5], 1u << (pidx & 31));
                    atomicOr(&pivg[pidx >> 5], 1u << (pidx & 31));
                }
                cs += pair_hash(sidx, pidx);
                npairs += 1;
                // R_j = live triangles (bounded by C(N,3))
                const uint64_t room = rb.rpool_cap - rused;
                if (room < binom((uint64_t)n, 3)) {
                    err = 2;
                    break;
                }
                const uint32_t wr = S.gather(ln, rpool + rused);
                if (ln == 0) {
                    roff[j] = rused;
                    rlen[j] = wr;
                }
                rused += wr;
                break;
            }
            __syncthreads();
        }
        __syncthreads();
        S.reset(ln);
        __syncthreads();
    }
    if (ln == 0) {
        if (err == 2) atomicOr(&st->err, ERR_VPOOL_CAP);
        if (err == 3) atomicOr(&st->err, ERR_STEP_LIMIT);
        atomicAdd((unsigned long long*)&st->checksum[1], (unsigned long long)cs);
        atomicAdd((unsigned long long*)&st->all_pairs[1], (unsigned long long)npairs);
        atomicAdd((unsigned long long*)&st->n_adds[1], (unsigned long long)nadds);
        atomicAdd((unsigned long long*)&st->n_columns[1], (unsigned long long)(0ull - nskip));
        st->rmask[1] = rcap2 - 1;  // H2 clearing probes the HBM mirror with this mask
        st->nskip[1] = nskip;
    }
}

// H2 phase 1 of one layer: wave w of kP1Waves takes residual columns w, w+K, ...
// and reduces each with apparent columns only.
template <bool PACKED>
__device__ void h2_phase1(const float* Dl, int n, float r, LayerStats* st, int l, int w, const DimBufs& b, const SmallBufs& sb,
                          unsigned char* lds, uint64_t step_limit) {
    constexpr int DIM = 2, NV = 4;
    using Lo = RowLo<NV>;
    const int ln = threadIdx.x;
    uint64_t nres = (uint64_t)st->n_residual[2];
    if (nres > b.rcap) nres = b.rcap;
    if ((uint64_t)w >= nres) return;
    const uint64_t* resid = b.resid + (size_t)l * b.rcap;
    const uint32_t* pivg = b.pivbits + (size_t)l * b.piv_words;

    unsigned char* p = lds;
    auto take = [&](size_t bytes) {
        unsigned char* q = p;
        p += (bytes + 15) & ~(size_t)15;
        return q;
    };
    KeySet W;
    const uint32_t wcap = sb.p1_wcap;
    W.log = (uint64_t*)take(8ull * wcap);
    W.index = (uint64_t*)take(16ull * wcap);
    W.fill = (uint32_t*)take(4ull * (2 * wcap / 8));
    W.tmp = (uint64_t*)take(8ull * 2 * wcap);
    W.imask = 2 * wcap - 1;
    W.cnt = 0;
    const uint32_t* piv = pivg;
    if (sb.p1_piv_lds) {
        uint32_t* pl = (uint32_t*)take(4ull * b.piv_words);
        stage_to_lds(pl, pivg, 4ull * b.piv_words, ln, 64);
        piv = pl;
    }
    for (uint32_t e = ln; e <= W.imask; e += 64) W.index[e] = 0;
    for (uint32_t e = ln; e <= (W.imask >> 3); e += 64) W.fill[e] = 0;
    __syncthreads();
    const uint32_t wlim = (wcap >> 1) + (wcap >> 2);

    uint64_t* p1k = sb.p1_key + (size_t)l * b.rcap;
    uint32_t* p1i = sb.p1_info + (size_t)l * b.rcap;
    uint64_t* roff = sb.roff2 + (size_t)l * b.rcap;
    uint32_t* rlen = sb.rlen2 + (size_t)l * b.rcap;

    auto cob = [&](const int (&vs)[DIM + 1], float sd) {
        const int v = ln;
        bool ok = v < n;
#pragma unroll
        for (int i = 0; i <= DIM; ++i) ok &= (vs[i] != v);
        float cd = sd;
        uint64_t key = 0;
        if (ok) {
#pragma unroll
            for (int i = 0; i <= DIM; ++i) cd = fmaxf(cd, ld_lds(Dl, (size_t)vs[i] * n + v));
            ok = cd <= r;
            uint32_t lo;
            if (PACKED) {
                int t[NV];
                int q = 0;
                bool placed = false;
#pragma unroll
                for (int i = 0; i <= DIM; ++i) {
                    if (!placed && v > vs[i]) {
                        t[q++] = v;
                        placed = true;
                    }
                    t[q++] = vs[i];
                }
                if (!placed) t[NV - 1] = v;
                lo = Lo::pack(t);
            } else {
                lo = (uint32_t)cofacet_index<DIM>(vs, v);
            }
            key = ((uint64_t)__float_as_uint(cd + 0.0f) << 32) | (0xFFFFFFFFu - lo);
        }
        W.toggle_pass(key, ok, ln);
    };

    for (uint64_t j = (uint64_t)w; j < nres; j += kP1Waves) {
        const uint64_t key = ld_glb(resid, j);
        const uint64_t sidx = key_idx(key);
        const float sdm = key_diam(key);
        int vs[DIM + 1];
        decode_wave<DIM>(sidx, n, vs, ln);
        cob(vs, sdm);
        __syncthreads();
        uint32_t adds = 0, flags = 0;
        uint64_t out_key = kEmpty64;
        for (uint64_t step = 0;; ++step) {
            uint64_t pk;
            uint32_t nlive;
            W.scan(ln, pk, nlive);
            if (step >= step_limit) {
                flags = kP1Overflow;  // phase 2 redoes it from scratch (and enforces the limit)
                break;
            }
            if (W.cnt > 2 * nlive + 256) W.compact(ln);
            if (pk == kEmpty64) break;
            const uint32_t plo = 0xFFFFFFFFu - (uint32_t)pk;
            int t[NV];
            uint64_t pidx;
            if (PACKED) {
                Lo::unpack(plo, t);
                pidx = encode<DIM + 1>(t);
            } else {
                pidx = plo;
                decode_wave<DIM + 1>(pidx, n, t, ln);
            }
            const uint32_t pw = sb.p1_piv_lds ? ld_lds(piv, pidx >> 5) : ld_glb(piv, pidx >> 5);
            if (!((pw >> (pidx & 31)) & 1u)) {  // not apparent: phase 1 ends here
                out_key = pk;
                const uint32_t nl = nlive;
                unsigned long long base = 0;
                if (ln == 0) base = atomicAdd(&sb.p1_used[l], (unsigned long long)nl);
                base = __shfl(base, 0, 64);
                if (base + nl > sb.rpool2_cap) {
                    flags = kP1Overflow;
                    break;
                }
                const uint32_t wr = W.gather_live(ln, sb.rpool2 + (size_t)l * sb.rpool2_cap + base);
                if (ln == 0) {
                    roff[j] = base;
                    rlen[j] = wr;
                }
                break;
            }
            // apparent column: youngest facet's coboundary
            float dd[NV][NV];
#pragma unroll
            for (int i = 0; i < NV; ++i)
#pragma unroll
                for (int k = i + 1; k < NV; ++k) dd[i][k] = ld_lds(Dl, (size_t)t[i] * n + t[k]);
            float fd = -1.0f;
            int fu = 0;
#pragma unroll
            for (int u = 0; u < NV; ++u) {
                float d = 0.0f;
#pragma unroll
                for (int i = 0; i < NV; ++i)
#pragma unroll
                    for (int k = i + 1; k < NV; ++k)
                        if (i != u && k != u) d = fmaxf(d, dd[i][k]);
                if (d > fd) {
                    fd = d;
                    fu = u;
                }
            }
            int fv[DIM + 1];
#pragma unroll
            for (int u = 0; u < NV; ++u) {
                if (u != fu) continue;
#pragma unroll
                for (int i = 0, q = 0; i < NV; ++i)
                    if (i != u) fv[q++] = t[i];
            }
            if (W.cnt + (uint32_t)n > wlim) {
                W.compact(ln);
                if (W.cnt + (uint32_t)n > wlim) {
                    flags = kP1Overflow;
                    break;
                }
            }
            cob(fv, fd);
            ++adds;
            __syncthreads();
        }
        if (ln == 0) {
            p1k[j] = out_key;
            p1i[j] = adds | flags;
        }
        __syncthreads();
        W.reset(ln);
    }
}

// One launch, two roles: blockIdx.y == 0 runs the H1 chain of layer
// blockIdx.x (dense working column), blockIdx.y = 1..kP1Waves run H2 phase 1.
template <bool P2>
__global__ __launch_bounds__(64) void k_reduce_small(const float* __restrict__ dist, int n, int maxdim,
                                                     LayerStats* __restrict__ stats, DimBufs b1, DimBufs b2, Reduce2Bufs rb,
                                                     SmallBufs sb, uint64_t step_limit, Pair* __restrict__ pairs1, uint64_t pcap1) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.x, role = blockIdx.y, ln = threadIdx.x;
    LayerStats* st = stats + l;
    const float r = st->thresh;
    float* Dl = (float*)(smem + 16);
    stage_to_lds(Dl, dist + (size_t)l * n * n, 4ull * n * n, ln, 64);
    unsigned char* p = smem + 16 + ((4ull * n * n + 15) & ~15ull);
    __syncthreads();
    if (role == 0)
        reduce_h1_dense(Dl, n, r, st, l, b1, rb, sb, p, step_limit, pairs1, pcap1);
    else if (maxdim >= 2)
        h2_phase1<P2>(Dl, n, r, st, l, role - 1, b2, sb, p, step_limit);
}

}  // namespace tda
