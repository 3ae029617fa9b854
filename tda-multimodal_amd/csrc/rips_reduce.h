// rips_reduce.h -- serial part of the cohomology reduction on gfx950.
//
// [upstream ripser.cpp compute_pairs / add_coboundary / get_pivot]: the
// residual (non-apparent) columns of one layer are reduced in column order by
// ONE wave (64 lanes, no cross-wave barriers).  The run time is a dependency
// chain of pivot steps (one column addition each), so every step is built to
// issue few dependent LDS round trips:
//   * working coboundary W: Z/2 toggle-set of u64 filtration keys
//     (diam_bits << 32 | ~lo32), pivot = plain u64 wave-min (DPP).  lo32 is
//     the row simplex's PACKED vertex tuple when it fits 32 bits (colex order
//     == lexicographic order of descending vertex tuples, so the key order is
//     Ripser's (diam asc, index desc)); the pivot's vertices are then shifts,
//     not a combinatorial decode.  Otherwise lo32 is the index itself.
//   * W layout: insertion-ordered key log (parity = bit 63 of the entry) +
//     64-bit index (lo32 << 32 | log pos + 1): a pivot scan is a bare u64 min
//     over the log with 16-B loads, a toggle is one index read + one CAS (or
//     one 64-bit XOR); the log length lives in a wave-uniform register, so
//     reservations need no LDS atomics;
//   * a residual column's reduced coboundary R_j is stored explicitly (HBM
//     pool) when it pairs; re-adding it is one toggle pass over |R_j| keys
//     (Ripser keeps V_j instead and re-enumerates every coboundary);
//   * apparent columns are re-added implicitly: the owner of an apparent pivot
//     is its youngest facet (pivot bitmap from k_apparent), whose coboundary
//     is enumerated wave-parallel (one lane per new vertex, reading the
//     symmetric distance matrix column-wise: conflict-free LDS access);
//   * distance matrix, pivot bitmap and the residual pivot map live in LDS.
#pragma once
#include "rips_kernels.h"

namespace tda {

#ifdef TDA_PROFILE
#define TDA_STAMP(var) const uint64_t var = clock64()
#define TDA_ACC(i, t0) prof[i] += clock64() - (t0)
#else
#define TDA_STAMP(var)
#define TDA_ACC(i, t0)
#endif

// wave-parallel decode: all 64 lanes cooperate, every lane gets the result
template <int DIM>
__device__ __forceinline__ void decode_wave(uint64_t idx, int n, int (&vs)[DIM + 1], int ln) {
    int top = n - 1;
#pragma unroll
    for (int k = DIM + 1; k >= 1; --k) {
        int v = k - 1;
        for (int base = top;; base -= 64) {
            int cand = base - ln;
            bool ok = cand >= k - 1 && binom((uint64_t)cand, k) <= idx;
            uint64_t m = __ballot(ok);
            if (m) {
                v = base - __builtin_ctzll(m);
                break;
            }
            if (base - 63 <= k - 1) break;
        }
        vs[DIM + 1 - k] = v;
        idx -= binom((uint64_t)v, k);
        top = v - 1;
    }
}

// row-simplex key payload: packed descending vertices
template <int NV>
struct RowLo {
    static constexpr int B = NV == 3 ? 10 : 8;  // triangles: N <= 1024, tetrahedra: N <= 256
    __device__ static uint32_t pack(const int (&t)[NV]) {
        uint32_t h = 0;
#pragma unroll
        for (int i = 0; i < NV; ++i) h = (h << B) | (uint32_t)t[i];
        return h;
    }
    __device__ static void unpack(uint32_t h, int (&t)[NV]) {
#pragma unroll
        for (int i = NV - 1; i >= 0; --i) {
            t[i] = (int)(h & ((1u << B) - 1));
            h >>= B;
        }
    }
};

// ---------------------------------------------------------------- toggle set
// Z/2 set of u64 keys for ONE wave: key log (insertion order) + open-
// addressing index (entry = lo32 << 32 | pos + 1).  A key's parity lives in
// bit 63 of its log entry (keys have bit 63 clear: non-negative f32 diameter
// bits), set = dead, so a dead entry is never the minimum and a pivot scan is
// a bare u64 min over the log (16-B loads, no side table).  toggle_pass()
// toggles one set of DISTINCT keys with the whole wave; new keys take
// consecutive log positions [cnt, cnt + new) from the wave-uniform counter.
constexpr uint64_t kDead = 1ull << 63;
// LDS: log / index / fill live in LDS (else HBM); TLDS: the scratch `tmp` does.
// Every access is address-space typed (no FLAT), so LDS round trips never
// wait on the wave's outstanding HBM traffic.
template <bool LDS, bool TLDS = LDS>
struct KeySet {
    uint64_t* index;  // icap entries, 0 = free
    uint32_t* fill;   // per-bucket fill count (icap / 8)
    uint64_t* log;    // cap keys (| kDead when cancelled)
    uint64_t* tmp;    // scratch >= 2 * cap keys
    uint32_t imask;   // icap - 1
    uint32_t cnt;     // log length (wave-uniform register)

    // index lookup of one key: 8-slot buckets (64 B, four 16-B reads in
    // flight) with a per-bucket fill counter, so a probe is one LDS round trip
    // and an insert takes its slot with one atomicAdd (no CAS retry loop when
    // several lanes of the pass land in the same bucket).
    __device__ __forceinline__ void toggle_pass(uint64_t k, bool valid, int ln) {
        const uint32_t fp = (uint32_t)k;
        const uint32_t bmask = imask >> 3;
        uint32_t bkt = mix32(fp) & bmask;
        uint32_t mine = 0;  // reserved log position + 1
        bool pending = valid;
        while (__ballot(pending)) {
            bool want = false;
            uint32_t target = 0;
            if (pending) {
                const size_t bo = (size_t)bkt * 8;
                const u64x2 q0 = mld2<LDS>(index, bo), q1 = mld2<LDS>(index, bo + 2), q2 = mld2<LDS>(index, bo + 4),
                            q3 = mld2<LDS>(index, bo + 6);
                const uint64_t e[8] = {q0.x, q0.y, q1.x, q1.y, q2.x, q2.y, q3.x, q3.y};
                uint64_t eh = 0;
                bool full = true;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    if (e[u] != 0 && (uint32_t)(e[u] >> 32) == fp) eh = e[u];
                    full &= e[u] != 0;
                }
                if (eh) {
                    matomic_xor<LDS>(&log[(uint32_t)eh - 1], kDead);  // flip parity
                    pending = false;
                } else if (!full) {
                    const uint32_t slot = matomic_add<LDS>(&fill[bkt], 1u);
                    if (slot < 8) {
                        want = true;
                        target = bkt * 8 + slot;
                    } else {
                        bkt = (bkt + 1) & bmask;  // filled up by other lanes of this pass
                    }
                } else {
                    bkt = (bkt + 1) & bmask;  // bucket full: next one
                }
            }
            const uint64_t need = __ballot(want);
            if (want) {
                mine = cnt + lanes_below(need) + 1;
                mst<LDS>(log, mine - 1, k);  // new entry: live
                mst<LDS>(index, target, ((uint64_t)fp << 32) | mine);
                pending = false;
            }
            cnt += (uint32_t)__popcll(need);
        }
    }
    // zero the index, cnt = 0 (whole wave)
    __device__ void reset(int ln) {
        const uint32_t c = cnt;
        if (c * 4 >= imask) {
            for (uint32_t e = ln; e <= (imask >> 3); e += 64) mst<LDS>(fill, e, 0u);
            for (uint32_t e = ln; e <= imask; e += 64) mst<LDS>(index, e, (uint64_t)0);
        } else {
            // probe each logged key's slot, then zero (two phases)
            uint32_t* slots = (uint32_t*)tmp;
            const uint32_t bmask = imask >> 3;
            for (uint32_t e = ln; e < c; e += 64) {
                const uint32_t fp = (uint32_t)mld<LDS>(log, e);
                uint32_t h = (mix32(fp) & bmask) * 8;
                for (;;) {
                    const uint64_t cur = mld<LDS>(index, h);
                    if (cur == 0 || (uint32_t)(cur >> 32) == fp) break;
                    h = (h + 1) & imask;  // buckets are filled in slot order
                }
                mst<TLDS>(slots, e, h);
            }
            wave_sync();
            for (uint32_t e = ln; e < c; e += 64) {
                const uint32_t h = mld<TLDS>(slots, e);
                mst<LDS>(index, h, (uint64_t)0);
                mst<LDS>(fill, h >> 3, 0u);
            }
        }
        cnt = 0;
        wave_sync();
    }
    // min live key + live count (wave-uniform)
    __device__ void scan(int ln, uint64_t& best, uint32_t& nlive) const {
        const uint32_t c = cnt;
        uint64_t b = kEmpty64;
        uint32_t nl = 0;
        uint32_t e = 2 * ln;
        for (; e + 384 + 1 < c; e += 512) {  // 4 x 16-B loads in flight
            const u64x2 a0 = mld2<LDS>(log, e), a1 = mld2<LDS>(log, e + 128);
            const u64x2 a2 = mld2<LDS>(log, e + 256), a3 = mld2<LDS>(log, e + 384);
            nl += (a0.x < kDead) + (a0.y < kDead) + (a1.x < kDead) + (a1.y < kDead) + (a2.x < kDead) + (a2.y < kDead) +
                  (a3.x < kDead) + (a3.y < kDead);
            uint64_t m0 = a0.x < a0.y ? a0.x : a0.y, m1 = a1.x < a1.y ? a1.x : a1.y;
            uint64_t m2 = a2.x < a2.y ? a2.x : a2.y, m3 = a3.x < a3.y ? a3.x : a3.y;
            m0 = m0 < m1 ? m0 : m1;
            m2 = m2 < m3 ? m2 : m3;
            m0 = m0 < m2 ? m0 : m2;
            b = m0 < b ? m0 : b;
        }
        for (; e < c; e += 128) {
            const uint64_t k0 = mld<LDS>(log, e);
            const uint64_t k1 = e + 1 < c ? mld<LDS>(log, e + 1) : kEmpty64;
            nl += (k0 < kDead) + (k1 < kDead);
            const uint64_t m = k0 < k1 ? k0 : k1;
            b = m < b ? m : b;
        }
        b = b < kDead ? b : kEmpty64;
        best = wave_min_u64(b);
        nlive = (uint32_t)wave_sum_u64(nl);
    }
    // min live key only (wave-uniform)
    __device__ uint64_t scan_min(int ln) const {
        const uint32_t c = cnt;
        uint64_t b = kEmpty64;
        uint32_t e = 2 * ln;
        for (; e + 384 + 1 < c; e += 512) {
            const u64x2 a0 = mld2<LDS>(log, e), a1 = mld2<LDS>(log, e + 128);
            const u64x2 a2 = mld2<LDS>(log, e + 256), a3 = mld2<LDS>(log, e + 384);
            uint64_t m0 = a0.x < a0.y ? a0.x : a0.y, m1 = a1.x < a1.y ? a1.x : a1.y;
            uint64_t m2 = a2.x < a2.y ? a2.x : a2.y, m3 = a3.x < a3.y ? a3.x : a3.y;
            m0 = m0 < m1 ? m0 : m1;
            m2 = m2 < m3 ? m2 : m3;
            m0 = m0 < m2 ? m0 : m2;
            b = m0 < b ? m0 : b;
        }
        for (; e < c; e += 128) {
            const uint64_t k0 = mld<LDS>(log, e);
            const uint64_t k1 = e + 1 < c ? mld<LDS>(log, e + 1) : kEmpty64;
            const uint64_t m = k0 < k1 ? k0 : k1;
            b = m < b ? m : b;
        }
        b = b < kDead ? b : kEmpty64;
        return wave_min_u64(b);
    }
    __device__ uint32_t count_live(int ln) const {
        uint32_t nl = 0;
        for (uint32_t e = ln; e < cnt; e += 64) nl += mld<LDS>(log, e) < kDead;
        return (uint32_t)wave_sum_u64(nl);
    }
    // write the live keys to out[] (whole wave), returns how many
    template <bool OLDS = false>
    __device__ uint32_t gather_live(int ln, uint64_t* out) const {
        const uint32_t c = cnt;
        uint32_t pos = 0;
        for (uint32_t e0 = 0; e0 < c; e0 += 64) {
            uint32_t e = e0 + ln;
            const uint64_t k = e < c ? mld<LDS>(log, e) : kEmpty64;
            const bool lv = k < kDead;
            uint64_t m = __ballot(lv);
            if (lv) mst<OLDS>(out, pos + lanes_below(m), k);
            pos += (uint32_t)__popcll(m);
        }
        return pos;
    }
    // keep only live keys (whole wave)
    __device__ void compact(int ln) {
        uint64_t* kept = tmp + (imask + 1) / 2;  // after the slot scratch
        const uint32_t pos = gather_live<TLDS>(ln, kept);
        wave_sync();
        reset(ln);
        for (uint32_t e0 = 0; e0 < pos; e0 += 64) {
            const uint32_t e = e0 + ln;
            toggle_pass(e < pos ? mld<TLDS>(kept, e) : 0, e < pos, ln);
        }
        wave_sync();
    }
};

struct Reduce2Bufs {
    uint64_t* rmap_keys;  // [L][2][rmap_stride] per-dim maps that do not fit LDS
    uint32_t* rmap_vals;
    uint64_t rmap_stride;
    uint64_t* roff;       // [L][rcap] offset of R_j in rpool
    uint32_t* rlen;       // [L][rcap]
    uint64_t* rpool;      // [L][rpool_cap] reduced coboundary keys
    uint64_t rpool_cap;
    uint64_t* wtmp;       // [L][wtmp_stride] scratch
    uint64_t wtmp_stride;
    // global working tables (global mode)
    uint64_t* windex;  // [L][2 wcap]
    uint32_t* wfill;   // [L][2 wcap / 8]
    uint64_t* wlog;    // [L][wcap]
    uint64_t wcap;
    const uint32_t* mst;  // [L][mst_words] H0 forest edges (dim-1 columns to skip)
    uint64_t mst_words;
};

// H2 phase 1 -> phase 2 hand-off (rips_reduce_small.h)
struct SmallBufs {
    uint32_t* p1_next;    // [L] next H2 column for a phase-1 wave (zeroed per call)
    uint64_t* p1_key;     // [L][rcap2] pivot key after phase 1 (kEmpty64: zero column)
    uint32_t* p1_info;    // [L][rcap2] additions | kP1Overflow
    uint32_t* p1_pidx;    // [L][rcap2] index of the phase-1 pivot (when p1_key is a pivot)
    uint64_t* roff2;      // [L][rcap2] phase-1 working column, then R_j, in rpool2
    uint32_t* rlen2;
    uint64_t* rpool2;     // [L][rpool2_cap]
    uint64_t rpool2_cap;
    unsigned long long* p1_used;  // [L] rpool2 entries taken by phase 1 (zeroed per call)
    uint32_t p1_wcap;     // phase-1 LDS toggle-set capacity per wave
};
constexpr uint32_t kP1Overflow = 1u << 31;  // phase-1 column outgrew its LDS table
constexpr uint32_t kP1Cleared = 1u << 30;   // phase 2: the column is an H1 death (prefetched flag)

struct Reduce2Cfg {  // per-dim LDS carve, decided on the host
    uint32_t wcap, rmap_lds_cap;  // rmap_lds_cap = 0 -> global map
    int piv_lds;
};
struct ReduceAllCfg {
    Reduce2Cfg dim[3];
    uint64_t step_limit;  // pivots per column before giving up (exit guarantee)
    int dist_lds;
    uint32_t bytes;  // dynamic LDS of the launch
};

enum : int32_t { ERR_LDS_SPILL = 32, ERR_STEP_LIMIT = 64 };  // STEP_LIMIT: a column exceeded the pivot budget

// residual pivot map of one dim: open addressing, key = row payload lo32.
// lds: the table lives in LDS (typed accesses), else in HBM.
struct PivMap {
    uint64_t* k;
    uint32_t* v;
    uint64_t mask;
    bool lds;
    template <bool L>
    __device__ int64_t find_t(uint32_t lo, int ln) const {  // wave-parallel probe
        for (uint64_t h0 = mix32(lo);; h0 += 64) {
            const uint64_t kk = mld<L>(k, (h0 + ln) & mask);
            const uint64_t mhit = __ballot(kk == lo), mend = __ballot(kk == kEmpty64);
            const uint64_t below_end = mend ? ((mend & (~mend + 1)) - 1) : ~0ull;
            if (mhit & below_end) return (int64_t)mld<L>(v, (h0 + __builtin_ctzll(mhit & below_end)) & mask);
            if (mend) return -1;
        }
    }
    template <bool L>
    __device__ void insert_t(uint32_t lo, uint32_t val) const {  // one lane
        uint64_t h = mix32(lo) & mask;
        while (mld<L>(k, h) != kEmpty64) h = (h + 1) & mask;
        mst<L>(k, h, (uint64_t)lo);
        mst<L>(v, h, val);
    }
    __device__ int64_t find(uint32_t lo, int ln) const { return lds ? find_t<true>(lo, ln) : find_t<false>(lo, ln); }
    // any number of lanes at once; keys must be distinct and absent
    template <bool L>
    __device__ void insert_par_t(uint32_t lo, uint32_t val) const {
        uint64_t h = mix32(lo) & mask;
        while (matomic_cas<L>(&k[h], kEmpty64, (uint64_t)lo) != kEmpty64) h = (h + 1) & mask;
        mst<L>(v, h, val);
    }
    __device__ void insert_par(uint32_t lo, uint32_t val) const {
        if (lds)
            insert_par_t<true>(lo, val);
        else
            insert_par_t<false>(lo, val);
    }
    __device__ void insert(uint32_t lo, uint32_t val) const {
        if (lds)
            insert_t<true>(lo, val);
        else
            insert_t<false>(lo, val);
    }
    // full 64-bit row keys (H2 above N = 568: tetrahedron indices exceed 32
    // bits); HBM tables only.  A key never equals kEmpty64 (indices < 2^42).
    __device__ int64_t find64(uint64_t key, int ln) const {
        for (uint64_t h0 = mix64(key);; h0 += 64) {
            const uint64_t kk = ld_glb(k, (h0 + ln) & mask);
            const uint64_t mhit = __ballot(kk == key), mend = __ballot(kk == kEmpty64);
            const uint64_t below_end = mend ? ((mend & (~mend + 1)) - 1) : ~0ull;
            if (mhit & below_end) return (int64_t)ld_glb(v, (h0 + __builtin_ctzll(mhit & below_end)) & mask);
            if (mend) return -1;
        }
    }
    __device__ void insert64(uint64_t key, uint32_t val) const {  // one lane
        uint64_t h = mix64(key) & mask;
        while (ld_glb(k, h) != kEmpty64) h = (h + 1) & mask;
        st_glb(k, h, key);
        st_glb(v, h, val);
    }
};

struct ReduceCtx {
    const float* D;  // distance matrix (LDS or HBM)
    int n;
    float r;
    LayerStats* st;
    unsigned char* lds;  // start of the per-dim LDS region
    int l, ln;
    uint64_t step_limit;
};

// payload (lo32) of a d-simplex with descending vertices, as the dim-(d-1)
// reduction keyed its rows
template <int NVTX, bool PACKED>
__device__ __forceinline__ uint32_t row_payload(const int (&t)[NVTX]) {
    if (PACKED) return RowLo<NVTX>::pack(t);
    return (uint32_t)encode<NVTX - 1>(t);
}

// Reduce the residual columns of dimension DIM of one layer (one wave).
// prev: residual pivot map of DIM-1 (DIM == 2), used to skip columns that are
// H_{DIM-1} deaths found by the serial reduction (clearing; k_apparent only
// knew the apparent ones).  Returns this dim's map (valid until the kernel ends
// if it lives in a persistent region).
// PH2: phase 2 of the split H2 reduction (rips_reduce_small.h): every column
// starts from its phase-1 result in `sb` instead of its coboundary.
template <int DIM, bool LDSW, bool PACKED, bool PREV_PACKED, bool PH2 = false>
__device__ void reduce_dim(const ReduceCtx& c, const DimBufs& b, const Reduce2Bufs& rb, const Reduce2Cfg& cfg, PivMap& map,
                           const PivMap* prev, unsigned char* map_lds, Pair* __restrict__ pairs, uint64_t pcap,
                           const SmallBufs* sb = nullptr, const uint32_t* clr = nullptr, unsigned char* pre_lds = nullptr,
                           uint32_t pre_cap = 0) {
    constexpr int NV = DIM + 2;  // vertices of a row simplex
    using Lo = RowLo<NV>;
    const int l = c.l, ln = c.ln, n = c.n;
    const float r = c.r;
    const float* D = c.D;
    // distance matrix: LDS in LDS mode, HBM otherwise (typed loads, no FLAT)
    auto dist_at = [&](size_t i) -> float { return LDSW ? ld_lds(D, i) : ld_glb(D, i); };
    LayerStats* st = c.st;
    uint64_t nres = (uint64_t)st->n_residual[DIM];
    if (nres > b.rcap) nres = b.rcap;
    const uint64_t* resid = b.resid + (size_t)l * b.rcap;
    uint32_t* pivg = b.pivbits + (size_t)l * b.piv_words;

    // ---- residual pivot map of this dim (LDS when it fits)
    uint64_t rcap2 = 16;
    while (rcap2 < 2 * nres + 16) rcap2 <<= 1;
    if (cfg.rmap_lds_cap && rcap2 <= cfg.rmap_lds_cap) {
        rcap2 = cfg.rmap_lds_cap;
        map.k = (uint64_t*)map_lds;
        map.v = (uint32_t*)(map_lds + 8ull * rcap2);
        map.lds = true;
        for (uint64_t e = ln; e < rcap2; e += 64) map.k[e] = kEmpty64;
    } else {
        if (rcap2 > rb.rmap_stride) rcap2 = rb.rmap_stride;
        map.k = rb.rmap_keys + ((size_t)l * 2 + (DIM - 1)) * rb.rmap_stride;  // cleared by k_sort_resid
        map.v = rb.rmap_vals + ((size_t)l * 2 + (DIM - 1)) * rb.rmap_stride;
        map.lds = false;
    }
    map.mask = rcap2 - 1;
    if (nres == 0) {
        __syncthreads();
        return;
    }

    // ---- LDS carve of the per-dim region (16-B aligned pieces)
    unsigned char* p = c.lds;
    auto take = [&](size_t bytes) {
        unsigned char* q = p;
        p += (bytes + 15) & ~(size_t)15;
        return q;
    };
    KeySet<LDSW, false> W;
    uint32_t wcap;
    if (LDSW) {
        wcap = cfg.wcap;
        W.log = (uint64_t*)take(8ull * wcap);
        W.index = (uint64_t*)take(16ull * wcap);
        W.fill = (uint32_t*)take(4ull * (2 * wcap / 8));
    } else {
        wcap = (uint32_t)rb.wcap;
        W.log = rb.wlog + (size_t)l * wcap;
        W.index = rb.windex + (size_t)l * 2 * wcap;
        W.fill = rb.wfill + (size_t)l * (2 * wcap / 8);
    }
    W.tmp = rb.wtmp + (size_t)l * rb.wtmp_stride;
    W.imask = 2 * wcap - 1;
    W.cnt = 0;
    uint32_t* piv = pivg;
    if (cfg.piv_lds) {
        uint32_t* pl = (uint32_t*)take(4ull * b.piv_words);
        stage_to_lds(pl, pivg, 4ull * b.piv_words, ln, 64);
        piv = pl;
    }
    if (LDSW) {  // global-mode index: zeroed by the host, left clean by reset()
        for (uint32_t e = ln; e <= W.imask; e += 64) W.index[e] = 0;
        for (uint32_t e = ln; e <= (W.imask >> 3); e += 64) W.fill[e] = 0;
    }
    __syncthreads();
    const uint32_t* mst = rb.mst + (size_t)l * rb.mst_words;

    uint64_t* roff = PH2 ? sb->roff2 + (size_t)l * b.rcap : rb.roff + (size_t)l * b.rcap;
    uint32_t* rlen = PH2 ? sb->rlen2 + (size_t)l * b.rcap : rb.rlen + (size_t)l * b.rcap;
    const uint64_t pool_cap = PH2 ? sb->rpool2_cap : rb.rpool_cap;
    uint64_t* rpool = PH2 ? sb->rpool2 + (size_t)l * sb->rpool2_cap : rb.rpool + (size_t)l * rb.rpool_cap;
    uint64_t rused = 0;
    if (PH2) {
        rused = (uint64_t)sb->p1_used[l];
        if (rused > pool_cap) rused = pool_cap;
    }
    Pair* P = pairs + (size_t)l * pcap;
    uint64_t cs = 0, npairs = 0, nadds = 0, nskip = 0;
    uint64_t ecnt = (uint64_t)st->count[DIM];  // emitted pairs: one wave owns this dim's count
    int err = 0;  // wave-uniform
    // PH2: per-column inputs prefetched into LDS in parallel (key, phase-1
    // pivot, phase-1 info | kP1Cleared), so the serial walk issues no
    // dependent HBM loads on its common path
    uint64_t* pre_k = (uint64_t*)pre_lds;
    uint64_t* pre_p = pre_k + pre_cap;
    uint32_t* pre_i = (uint32_t*)(pre_p + pre_cap);
    uint32_t* pre_x = pre_i + pre_cap;
    const uint64_t npre = PH2 ? (nres < pre_cap ? nres : pre_cap) : 0;
    const uint64_t* p1k_g = PH2 ? sb->p1_key + (size_t)l * b.rcap : nullptr;
    const uint32_t* p1i_g = PH2 ? sb->p1_info + (size_t)l * b.rcap : nullptr;
    const uint32_t* clr_l = PH2 ? clr + (size_t)l * b.cleared_words : nullptr;
    auto ph2_load = [&](uint64_t j, uint64_t& key, uint64_t& pk1, uint32_t& info) {
        key = ld_glb(resid, j);
        const uint64_t si = key_idx(key);
        pk1 = ld_glb(p1k_g, j);
        info = ld_glb(p1i_g, j) | (((ld_glb(clr_l, si >> 5) >> (si & 31)) & 1u) ? kP1Cleared : 0u);
    };
    if (PH2) {
        for (uint64_t j = ln; j < npre; j += 64) {
            uint64_t key, pk1;
            uint32_t info;
            ph2_load(j, key, pk1, info);
            st_lds(pre_k, j, key);
            st_lds(pre_p, j, pk1);
            st_lds(pre_i, j, info);
            st_lds(pre_x, j, ld_glb(sb->p1_pidx + (size_t)l * b.rcap, j));
        }
        __syncthreads();
    }
    // PH2 prologue: column j pairs with its phase-1 pivot unless an earlier
    // column already owns that pivot (or phase 1 overflowed).  Every column
    // before the first such conflict is final, so they are emitted in
    // parallel; the serial walk starts at the conflict.
    uint64_t jstart = 0;
    if (PH2 && LDSW && npre == nres) {
        uint32_t tcap = 16;
        while (tcap < 2 * nres + 16) tcap <<= 1;
        if ((uint64_t)tcap * 8 <= 16ull * wcap) {
            uint32_t* tk = (uint32_t*)W.index;  // temp table over the (still unused) W index
            uint32_t* tv = tk + tcap;
            for (uint32_t e = ln; e < tcap; e += 64) {
                st_lds(tk, e, 0xFFFFFFFFu);
                st_lds(tv, e, 0xFFFFFFFFu);
            }
            wave_sync();
            for (uint64_t j = ln; j < nres; j += 64) {
                const uint32_t info = ld_lds(pre_i, j);
                const uint64_t pk1 = ld_lds(pre_p, j);
                if (!(info & (kP1Cleared | kP1Overflow)) && pk1 != kEmpty64) {
                    const uint32_t plo = 0xFFFFFFFFu - (uint32_t)pk1;
                    uint32_t h = mix32(plo) & (tcap - 1);
                    for (;;) {
                        const uint32_t old = matomic_cas<true>(&tk[h], 0xFFFFFFFFu, plo);
                        if (old == 0xFFFFFFFFu || old == plo) {
                            matomic_min<true>(&tv[h], (uint32_t)j);
                            break;
                        }
                        h = (h + 1) & (tcap - 1);
                    }
                }
            }
            wave_sync();
            uint32_t jc = (uint32_t)nres;
            for (uint64_t j = ln; j < nres; j += 64) {
                const uint32_t info = ld_lds(pre_i, j);
                const uint64_t pk1 = ld_lds(pre_p, j);
                bool serial = false;
                if (!(info & kP1Cleared)) {
                    if (info & kP1Overflow) {
                        serial = true;
                    } else if (pk1 != kEmpty64) {
                        const uint32_t plo = 0xFFFFFFFFu - (uint32_t)pk1;
                        uint32_t h = mix32(plo) & (tcap - 1);
                        while (ld_lds(tk, h) != plo) h = (h + 1) & (tcap - 1);
                        serial = ld_lds(tv, h) != (uint32_t)j;
                    }
                }
                if (serial) jc = min(jc, (uint32_t)j);
            }
            jc = wave_min_u32(jc);
            uint64_t pcs = 0, pnp = 0, pad = 0, psk = 0;
            for (uint32_t j0 = 0; j0 < jc; j0 += 64) {
                const uint32_t j = j0 + ln;
                const bool act = j < jc;
                uint32_t info = 0;
                uint64_t pk1 = kEmpty64, key = 0;
                uint32_t pidx1 = 0;
                if (act) {
                    info = ld_lds(pre_i, j);
                    pk1 = ld_lds(pre_p, j);
                    key = ld_lds(pre_k, j);
                    pidx1 = ld_lds(pre_x, j);
                }
                const bool cl = act && (info & kP1Cleared);
                const bool ess = act && !cl && pk1 == kEmpty64;
                const bool pr = act && !cl && pk1 != kEmpty64;
                const float sdm = key_diam(key), pd = __uint_as_float((uint32_t)(pk1 >> 32));
                const uint64_t sidx = key_idx(key);
                const bool emit = ess || (pr && pd > sdm);
                const uint64_t m = __ballot(emit);
                const uint64_t pos = ecnt + lanes_below(m);
                if (emit && pos < pcap) store_pair(P, pos, sdm, ess ? INFINITY : pd, (int64_t)sidx, ess ? -1 : (int64_t)pidx1);
                ecnt += (uint64_t)__popcll(m);
                if (pr) {
                    pcs += pair_hash(sidx, pidx1);
                    ++pnp;
                    map.insert_par(0xFFFFFFFFu - (uint32_t)pk1, j);
                    if (cfg.piv_lds) matomic_or<true>(&piv[pidx1 >> 5], 1u << (pidx1 & 31));
                    matomic_or<false>(&pivg[pidx1 >> 5], 1u << (pidx1 & 31));
                }
                if (act && !cl) pad += info & ~kP1Overflow;
                psk += cl;
            }
            cs += wave_sum_u64(pcs);
            npairs += wave_sum_u64(pnp);
            nadds += wave_sum_u64(pad);
            nskip += wave_sum_u64(psk);
            jstart = jc;
            for (uint32_t e = ln; e <= W.imask; e += 64) st_lds(W.index, e, (uint64_t)0);
            wave_sync();
        }
    }
#ifdef TDA_PROFILE
    uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // scan, lookup, facet, cob-app, cob-res, reset, compact, total
    const uint64_t t_all = clock64();
#endif
    const uint32_t wlim = (wcap >> 1) + (wcap >> 2);

    // make room for `need` new log entries; false on overflow
    auto room = [&](uint32_t need) -> bool {
        if (W.cnt + need <= wlim) return true;
        W.compact(ln);
        if (W.cnt + need <= wlim) return true;
        err = 1;
        return false;
    };
    // toggle the coboundary of the simplex with vertices vs (diam sd) into W
    auto cob = [&](const int (&vs)[DIM + 1], float sd) {
        for (int v0 = 0; v0 < n; v0 += 64) {
            const int v = v0 + ln;
            bool ok = v < n;
#pragma unroll
            for (int i = 0; i <= DIM; ++i) ok &= (vs[i] != v);
            float cd = sd;
            uint64_t key = 0;
            if (ok) {
#pragma unroll
                for (int i = 0; i <= DIM; ++i) cd = fmaxf(cd, dist_at((size_t)vs[i] * n + v));  // D symmetric: column read
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
            TDA_STAMP(tq);
            W.toggle_pass(key, ok, ln);
            TDA_ACC(4, tq);
        }
    };

    auto emit_essential = [&](uint64_t j, float sdm, uint64_t sidx) {
        if (ln == 0) {
            if (ecnt < pcap) store_pair(P, ecnt, sdm, INFINITY, (int64_t)sidx, -1);
            rlen[j] = 0;
        }
        ++ecnt;
    };
    auto emit_pair = [&](uint64_t j, float sdm, uint64_t sidx, float pd, uint64_t pidx, uint32_t plo) {
        if (pd > sdm) {
            if (ln == 0 && ecnt < pcap) store_pair(P, ecnt, sdm, pd, (int64_t)sidx, (int64_t)pidx);
            ++ecnt;
        }
        if (ln == 0) {
            map.insert(plo, (uint32_t)j);
            if (cfg.piv_lds) matomic_or<true>(&piv[pidx >> 5], 1u << (pidx & 31));
            matomic_or<false>(&pivg[pidx >> 5], 1u << (pidx & 31));
        }
        cs += pair_hash(sidx, pidx);
        npairs += 1;
    };

    for (uint64_t j = jstart; j < nres && !err; ++j) {
        TDA_STAMP(tA);
        uint64_t key, pk1 = 0;
        uint32_t info = 0;
        if (PH2) {
            if (j < npre) {
                key = ld_lds(pre_k, j);
                pk1 = ld_lds(pre_p, j);
                info = ld_lds(pre_i, j);
            } else {
                ph2_load(j, key, pk1, info);
            }
        } else {
            key = ld_glb(resid, j);
        }
        const uint64_t sidx = key_idx(key);
        const float sdm = key_diam(key);
        int vs[DIM + 1];
        // clearing: skip columns that are H_{DIM-1} deaths (PH2: a set bit in
        // the H_{DIM-1} pivot bitmap -- apparent pivots were never columns)
        bool cleared;
        if (PH2) {
            cleared = (info & kP1Cleared) != 0;
            info &= ~kP1Cleared;
        } else {
            decode_wave<DIM>(sidx, n, vs, ln);
            if (DIM == 1)
                cleared = (ld_glb(mst, sidx >> 5) >> (sidx & 31)) & 1u;
            else
                cleared = prev->find(row_payload<DIM + 1, PREV_PACKED>(vs), ln) >= 0;
        }
        if (cleared) {
            ++nskip;
            if (ln == 0) rlen[j] = 0;
            continue;
        }
        if (PH2 && !(info & kP1Overflow)) {
            nadds += info;
            if (pk1 == kEmpty64) {
                emit_essential(j, sdm, sidx);
                continue;
            }
            const uint32_t plo1 = 0xFFFFFFFFu - (uint32_t)pk1;
            uint64_t pidx1;
            if (PACKED) {
                int t1[NV];
                Lo::unpack(plo1, t1);
                pidx1 = encode<DIM + 1>(t1);
            } else {
                pidx1 = plo1;
            }
            // not apparent (phase 1 stopped there): a set bit is an earlier residual pivot
            TDA_ACC(1, tA);
            TDA_STAMP(tB);
            const uint32_t pw1 = cfg.piv_lds ? ld_lds(piv, pidx1 >> 5) : ld_glb((const uint32_t*)pivg, pidx1 >> 5);
            const int64_t own1 = ((pw1 >> (pidx1 & 31)) & 1u) ? map.find(plo1, ln) : -1;
            TDA_ACC(2, tB);
            if (own1 < 0) {  // new pair; R_j is the stored phase-1 column
                TDA_STAMP(tC);
                emit_pair(j, sdm, sidx, __uint_as_float((uint32_t)(pk1 >> 32)), pidx1, plo1);
                TDA_ACC(3, tC);
                continue;
            }
            // continue Ripser's loop from the stored working column
            const uint64_t o0 = roff[j];
            const uint32_t ol = rlen[j];
            if (!room(ol)) break;
            for (uint32_t e0 = 0; e0 < ol; e0 += 64) {
                const uint32_t e = e0 + ln;
                W.toggle_pass(e < ol ? ld_glb((const uint64_t*)rpool, o0 + e) : 0, e < ol, ln);
            }
        } else {
            if (PH2) decode_wave<DIM>(sidx, n, vs, ln);
            if (!room((uint32_t)n)) break;
            cob(vs, sdm);
        }
        __syncthreads();
        for (uint64_t step = 0;; ++step) {
            uint64_t pk;
            uint32_t nlive;
            TDA_STAMP(t0);
            W.scan(ln, pk, nlive);
            TDA_ACC(0, t0);
            if (step >= c.step_limit) {
                if (ln == 0)
                    printf("k_reduce_all: layer %d dim %d column %llu (idx %llu) step limit: pivot %016llx cnt %u live %u\n", l,
                           DIM, (unsigned long long)j, (unsigned long long)sidx, (unsigned long long)pk, W.cnt, nlive);
                err = 3;
                break;
            }
            if (W.cnt > 2 * nlive + 256) {
                TDA_STAMP(t6);
                W.compact(ln);
                TDA_ACC(6, t6);
            }
            if (pk == kEmpty64) {
                emit_essential(j, sdm, sidx);  // zero column: essential class (birth = diam sigma_j)
                break;
            }
            TDA_STAMP(t1);
            const uint32_t plo = 0xFFFFFFFFu - (uint32_t)pk;
            const float pd = __uint_as_float((uint32_t)(pk >> 32));
            int t[NV];
            uint64_t pidx;
            if (PACKED) {
                Lo::unpack(plo, t);
                pidx = encode<DIM + 1>(t);
            } else {
                pidx = plo;
                decode_wave<DIM + 1>(pidx, n, t, ln);
            }
            const uint32_t pw = cfg.piv_lds ? ld_lds(piv, pidx >> 5) : ld_glb((const uint32_t*)pivg, pidx >> 5);
            const bool app = (pw >> (pidx & 31)) & 1u;
            // the pivot bitmap marks apparent AND residual pivots: a clear bit
            // is a new pair without probing the residual map
            const int64_t owner = app ? map.find(plo, ln) : -1;
            TDA_ACC(1, t1);
            TDA_STAMP(t2);
            if (owner >= 0) {
                // add the stored reduced column R_owner
                const uint64_t o0 = ld_glb((const uint64_t*)roff, owner);
                const uint32_t ol = ld_glb((const uint32_t*)rlen, owner);
                if (!room(ol)) break;
                for (uint32_t e0 = 0; e0 < ol; e0 += 8 * 64) {
                    uint64_t rk8[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const uint32_t e = e0 + u * 64 + ln;
                        rk8[u] = e < ol ? ld_glb((const uint64_t*)rpool, o0 + e) : 0;
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        if (e0 + u * 64 >= ol) break;
                        W.toggle_pass(rk8[u], e0 + u * 64 + ln < ol, ln);
                    }
                }
                ++nadds;
                TDA_ACC(4, t2);
            } else if (app) {
                // apparent pair (phi, pivot): phi = youngest facet of the pivot,
                // i.e. max diameter, ties -> smallest index = smallest u (the
                // facet dropping t[u] grows in colex order with u)
                float dd[NV][NV];
#pragma unroll
                for (int i = 0; i < NV; ++i)
#pragma unroll
                    for (int k = i + 1; k < NV; ++k) dd[i][k] = dist_at((size_t)t[i] * n + t[k]);
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
                TDA_ACC(2, t2);
                TDA_STAMP(t3);
                if (!room((uint32_t)n)) break;
                cob(fv, fd);
                ++nadds;
                TDA_ACC(3, t3);
            } else {
                // new persistence pair (sigma_j, pivot); R_j = live keys of W
                emit_pair(j, sdm, sidx, pd, pidx, plo);
                if (rused + nlive > pool_cap) {
                    err = 2;
                    break;
                }
                const uint32_t wr = W.gather_live(ln, rpool + rused);
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
        TDA_STAMP(t5);
        W.reset(ln);
        TDA_ACC(5, t5);
    }
    if (ln == 0) {
        if (err == 1) atomicOr(&st->err, LDSW ? (int32_t)ERR_LDS_SPILL : (int32_t)ERR_WORK_CAP);
        if (err == 2) atomicOr(&st->err, ERR_VPOOL_CAP);
        if (err == 3) atomicOr(&st->err, ERR_STEP_LIMIT);
        if (ecnt > pcap) atomicOr(&st->err, ERR_PAIR_CAP);
        st->count[DIM] = (int64_t)ecnt;
        atomicAdd((unsigned long long*)&st->checksum[DIM], (unsigned long long)cs);
        atomicAdd((unsigned long long*)&st->all_pairs[DIM], (unsigned long long)npairs);
        atomicAdd((unsigned long long*)&st->n_adds[DIM], (unsigned long long)nadds);
        // cleared columns were counted as columns by k_apparent
        atomicAdd((unsigned long long*)&st->n_columns[DIM], (unsigned long long)(0ull - nskip));
        st->nskip[DIM] = nskip;
#ifdef TDA_PROFILE
        prof[7] = clock64() - t_all;
        for (int i = 0; i < 8; ++i) st->prof[DIM][i] = prof[i];
#endif
    }
    __syncthreads();
}

// All serial reductions of one layer in ONE launch (one wave per layer):
// H1 then H2, so a layer's H2 chain starts as soon as its own H1 chain ends
// (the batch time is the max over layers of the sum, not the sum of maxes).
// LDS: [16 B][distance matrix][H1 residual-pivot map][per-dim region].
template <bool LDSW, bool P1, bool P2>
__global__ __launch_bounds__(64) void k_reduce_all(const float* __restrict__ dist, int n, int maxdim, LayerStats* __restrict__ stats,
                                                   DimBufs b1, DimBufs b2, Reduce2Bufs rb, ReduceAllCfg cfg, Pair* __restrict__ pairs1,
                                                   Pair* __restrict__ pairs2, uint64_t pcap1, uint64_t pcap2) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.x, ln = threadIdx.x;
    LayerStats* st = stats + l;
    unsigned char* p = smem + 16;
    ReduceCtx c;
    c.n = n;
    c.l = l;
    c.ln = ln;
    c.st = st;
    c.r = st->thresh;
    c.step_limit = cfg.step_limit;
    c.D = dist + (size_t)l * n * n;
    if (LDSW) {  // LDS mode (N <= 64): the matrix always fits
        float* dl = (float*)p;
        stage_to_lds(dl, c.D, 4ull * n * n, ln, 64);
        p += (4ull * n * n + 15) & ~15ull;
        c.D = dl;
    }
    unsigned char* map1_lds = p;
    p += 12ull * cfg.dim[1].rmap_lds_cap;
    __syncthreads();
    PivMap m1, m2;
    c.lds = p;
    reduce_dim<1, LDSW, P1, P1>(c, b1, rb, cfg.dim[1], m1, nullptr, map1_lds, pairs1, pcap1);
    if (maxdim >= 2) {
        unsigned char* map2_lds = p;
        c.lds = p + 12ull * cfg.dim[2].rmap_lds_cap;
        reduce_dim<2, LDSW, P2, P1>(c, b2, rb, cfg.dim[2], m2, &m1, map2_lds, pairs2, pcap2);
    }
}

// Phase 2 of the split H2 reduction (N <= 64): one wave per layer walks the
// H2 columns in order on top of k_reduce_small's phase-1 results.  Clearing
// reads the H1 pivot bitmap (k_apparent<1> + the H1 chain).  LDS: [16 B]
// [distance matrix][per-column prefetch][H2 map + W + pivot bitmap], the
// k_reduce_all carve with the H1-map area holding the prefetch.
__global__ __launch_bounds__(64) void k_reduce_h2_finish(const float* __restrict__ dist, int n, LayerStats* __restrict__ stats,
                                                         DimBufs b1, DimBufs b2, Reduce2Bufs rb, ReduceAllCfg cfg, SmallBufs sb,
                                                         const uint32_t* __restrict__ res1, Pair* __restrict__ pairs2, uint64_t pcap2) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.x, ln = threadIdx.x;
    LayerStats* st = stats + l;
    unsigned char* p = smem + 16;
    ReduceCtx c;
    c.n = n;
    c.l = l;
    c.ln = ln;
    c.st = st;
    c.r = st->thresh;
    c.step_limit = cfg.step_limit;
    float* dl = (float*)p;
    stage_to_lds(dl, dist + (size_t)l * n * n, 4ull * n * n, ln, 64);
    p += (4ull * n * n + 15) & ~15ull;
    c.D = dl;
    unsigned char* pre = p;
    const uint32_t pre_cap = (uint32_t)(12ull * cfg.dim[1].rmap_lds_cap / 24);
    p += 12ull * cfg.dim[1].rmap_lds_cap;
    __syncthreads();
    PivMap m2;
    DimBufs b = b2;
    b.cleared_words = b1.piv_words;  // stride of the clearing bitmap below
    c.lds = p + 12ull * cfg.dim[2].rmap_lds_cap;
    reduce_dim<2, true, true, true, true>(c, b, rb, cfg.dim[2], m2, nullptr, p, pairs2, pcap2, &sb, res1, pre, pre_cap);
}

}  // namespace tda
