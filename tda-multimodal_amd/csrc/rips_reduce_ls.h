// rips_reduce_ls.h -- the parallel column reduction (k_reduce_ls) with a
// LEADER wave: the same lock-free owner-map scheme as k_reduce_par
// (rips_reduce_par.h: every residual column in flight, pivot -> owner map by
// CAS, records, requeues; [upstream ripser.cpp compute_pairs] order-free
// pairing), with a different column engine.
//
// Why: k_reduce_par's column step (r03 profile, torus1024's longest column:
// 9,207 steps of ~13.7 K cycles) spent a block-wide min scan + reduction
// barrier (1.3 K), hashed LDS toggles (1.8 K for ~24 front keys), refills
// (3 K amortised) and ~3 K at the step barrier per step -- almost all of it
// latency of a chain in which one step's pivot needs every wave's keys.
//
// Here the smallest keys of the working column live in ONE wave's registers:
//   * LS ("low set"), wave 0: up to 64 keys, sorted across the lanes, with a
//     bound B such that every live key < B is in LS (Z/2: a key present twice
//     cancels).  The pivot is LS[0]: no scan, no reduction.
//   * front: a RAW multiset of keys >= B in LDS (F[0, fc), appended without
//     deduplication; pulled entries are tombstoned).  It holds the radix
//     levels 0..kf relative to `last` (rips_reduce_par.h's radix heap).
//   * back: the HBM radix buckets of k_reduce_par (levels > kf).
// An apparent step: wave 0 loads the pivot's bitmap word and the facet's FULL
// rows, finds the coboundary's keys < B (the "low" keys: typically a few) and
// toggles them into LS; waves 1..7 compute the coboundary's other keys for
// their vertex ranges and append them (front or back) during the NEXT step,
// under that step's row loads, once wave 0 has said the step was apparent.
// One workgroup barrier per step (which also carries a room check); the
// block-wide work happens only at sync points: pulls of the next smallest
// front keys into LS (a radix select by level relative to B), front refills
// from HBM buckets, spills, and the owner path.
//
// Invariants (I1) every live key < B is in LS, LS holds only keys < B;
// (I2) front keys are >= B and at levels <= kf relative to `last`;
// (I3) back keys are at levels > kf; `last` <= every key of the column.
// Records stay raw multisets (rips_reduce_par.h), so k_par_emit and the
// record readers are shared.
#pragma once
#include "rips_reduce_par.h"

namespace tda {

constexpr int kLsT = 512;                   // threads: wave 0 leader, waves 1..7 workers
constexpr int kLsW = kLsT / 64;
constexpr int kLsWorkers = kLsW - 1;
// front keys (raw, tombstones included): 96 KB, so a 32-KB sort chunk of the
// H2 columns still fits beside a reducer workgroup on its CU (rips.hip)
constexpr uint32_t kLsFCap = 12288;
#ifndef TDA_LS_FILL                         // build-time A/B knob: keys a bucket refill keeps in the front
#define TDA_LS_FILL 3072
#endif
constexpr uint32_t kLsFill = TDA_LS_FILL;
constexpr uint32_t kLsPull = 256;           // raw front keys one pull hands to the leader
constexpr uint32_t kLsH = 512;              // leader hash slots: key | kDead (cancelled) | kEmpty64 (free)
constexpr uint32_t kLsHLive = 320;          // live leader keys before it flushes its set back out
constexpr uint32_t kLsCand = 256;           // compacted low-key candidates per round
constexpr int kLsLV = 16;                   // leader: vertices per lane per chunk (1024)
constexpr uint64_t kLsTomb = kEmpty64;      // pulled front entry
enum : uint32_t { LS_STEP = 0, LS_REFILL = 1, LS_OWNER = 2 };

struct LsLds {
    uint64_t F[kLsFCap];
    uint64_t pull[kLsPull];
    uint64_t H[kLsH];          // the leader's set (wave 0 only)
    int32_t cv[kLsCand];       // candidate vertex and its row values (wave 0 only)
    float ca[kLsCand], cb[kLsCand], cc[kLsCand];
    uint32_t npull;
    uint32_t bcnt[kParLv];
    uint32_t cptr[kParLv][kParChunks];
    uint32_t hist[kParLv];
    uint64_t red[2][kLsW];
    uint32_t wsum[2][kLsW];
    uint32_t anyf[2][kLsW];
    uint64_t bc[8];
    // mailbox: the leader writes step s + 1's entry during step s (parity s + 1)
    uint64_t mb_p[2], mb_B[2], mb_pidx[2];
    int32_t mb_fv[2][4];
    uint32_t mb_kind[2], mb_prev[2], mb_fsc[2];
    float mb_pd[2];
    uint64_t last;  // radix reference
    uint64_t B;     // LS bound (published at sync points)
    uint32_t kf;    // front holds levels 0..kf
    uint32_t fc;    // front length
    uint32_t lsc;   // LS count (published at sync points)
    int32_t err;
    uint32_t wide;
};
extern __shared__ LsLds ls_smem[];
#define LSS (ls_smem[0])

// ------------------------------------------------------------------ block helpers
struct LsRed {  // double-buffered block reductions, one barrier each (as ParRed)
    uint32_t par = 0;
    __device__ __forceinline__ bool any(bool p) {
        const uint64_t m = __ballot(p);
        const uint32_t b = par++ & 1;
        if ((threadIdx.x & 63) == 0) LSS.anyf[b][threadIdx.x >> 6] = m != 0;
        lds_sync();
        uint32_t r = 0;
#pragma unroll
        for (int w = 0; w < kLsW; ++w) r |= LSS.anyf[b][w];
        return r != 0;
    }
    // block-wide OR of 2 flag bits (one barrier)
    __device__ __forceinline__ uint32_t or2(uint32_t f) {
        const uint32_t m = (__ballot(f & 1u) ? 1u : 0u) | (__ballot(f & 2u) ? 2u : 0u);
        const uint32_t b = par++ & 1;
        if ((threadIdx.x & 63) == 0) LSS.anyf[b][threadIdx.x >> 6] = m;
        lds_sync();
        uint32_t r = 0;
#pragma unroll
        for (int w = 0; w < kLsW; ++w) r |= LSS.anyf[b][w];
        return r;
    }
    __device__ __forceinline__ uint64_t min(uint64_t v) {
        v = wave_min_u64(v);
        const uint32_t b = par++ & 1;
        if ((threadIdx.x & 63) == 0) LSS.red[b][threadIdx.x >> 6] = v;
        lds_sync();
        uint64_t m = LSS.red[b][0];
#pragma unroll
        for (int w = 1; w < kLsW; ++w) m = LSS.red[b][w] < m ? LSS.red[b][w] : m;
        return m;
    }
    __device__ __forceinline__ uint64_t sum(uint64_t v) {
        v = wave_sum_u64(v);
        const uint32_t b = par++ & 1;
        if ((threadIdx.x & 63) == 0) LSS.red[b][threadIdx.x >> 6] = v;
        lds_sync();
        uint64_t m = 0;
#pragma unroll
        for (int w = 0; w < kLsW; ++w) m += LSS.red[b][w];
        return m;
    }
    __device__ __forceinline__ uint32_t prefix(uint32_t c, uint32_t* tot) {
        const int ln = threadIdx.x & 63, w = threadIdx.x >> 6;
        uint32_t x = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (ln >= o) x += y;
        }
        const uint32_t b = par++ & 1;
        if (ln == 63) LSS.wsum[b][w] = x;
        lds_sync();
        uint32_t before = 0, all = 0;
#pragma unroll
        for (int q = 0; q < kLsW; ++q) {
            const uint32_t s = LSS.wsum[b][q];
            before += q < w ? s : 0;
            all += s;
        }
        *tot = all;
        return before + x - c;
    }
};

__device__ __forceinline__ int ls_first_bucket(uint32_t from) {
    const uint32_t ln = threadIdx.x & 63;
    const uint64_t m = __ballot(ln >= from && LSS.bcnt[ln] != 0);
    if (m) return (int)__builtin_ctzll(m);
    return (from <= 64u && LSS.bcnt[64]) ? 64 : -1;
}

// Append key k[r] to HBM bucket bb[r] (bit r of vmask): k_reduce_par's
// bucket_append on this kernel's LDS (chunks 0..3 preallocated, the key that
// opens chunk c allocates chunk c + 2).
template <int R>
__device__ __forceinline__ void ls_bucket_append(const uint64_t (&k)[R], const uint32_t (&bb)[R], uint32_t vmask, const ParBufs& P) {
    uint32_t slot[R];
#pragma unroll
    for (int r = 0; r < R; ++r) slot[r] = ((vmask >> r) & 1u) ? atomicAdd(&LSS.bcnt[bb[r]], 1u) : 0u;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!((vmask >> r) & 1u)) continue;
        const uint32_t kc = chunk_of(slot[r]);
        if (slot[r] == chunk_start(kc) && kc + 2 < (uint32_t)kParChunks && LSS.cptr[bb[r]][kc + 2] == kNoChunk) {
            const uint64_t sz = 256ull << (kc + 2);
            const uint64_t o = aadd(&P.ctl->bpool_used, sz);
            if (o + sz <= P.bpool_cap) LSS.cptr[bb[r]][kc + 2] = (uint32_t)(o >> 8);
            else LSS.err = 22;
        }
        const uint32_t cp = kc < (uint32_t)kParChunks ? LSS.cptr[bb[r]][kc] : kNoChunk;
        if (cp == kNoChunk) {
            LSS.err = 21;
            continue;
        }
        st_glb(P.bpool, (uint64_t)cp * 256 + (slot[r] - chunk_start(kc)), k[r]);
    }
}

__device__ __forceinline__ uint64_t ls_bucket_at(const ParBufs& P, uint32_t b, uint32_t e) {
    const uint32_t kc = chunk_of(e);
    return ld_glb(P.bpool, (uint64_t)LSS.cptr[b][kc] * 256 + (e - chunk_start(kc)));
}

// Route keys (bit r of vmask; all >= B) out of the leader's reach: levels
// <= kf (relative to last) to the front (wave-aggregated tail append), the
// rest to their HBM buckets.  No barrier; the caller made room in the front.
template <int R>
__device__ __forceinline__ void ls_route_p(const uint64_t (&k)[R], uint32_t vmask, const ParBufs& P) {
    const uint64_t last = LSS.last;
    const uint32_t kf = LSS.kf;
    uint32_t fm = 0, bm = 0, bb[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        bb[r] = par_bucket(k[r], last);
#ifdef TDA_LS_CHECK
        if (((vmask >> r) & 1u) && k[r] < last) LSS.err = 92;  // below the radix reference
#endif
        if ((vmask >> r) & 1u) {
            if (bb[r] <= kf) fm |= 1u << r;
            else bm |= 1u << r;
        }
    }
    uint64_t m[R];
    uint32_t wtot = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        m[r] = __ballot((fm >> r) & 1u);
        wtot += (uint32_t)__popcll(m[r]);
    }
    if (wtot) {
        const int ln = threadIdx.x & 63;
        const uint32_t lead = (uint32_t)__builtin_ctzll(__ballot(1));
        uint32_t base = 0;
        if ((uint32_t)ln == lead) base = atomicAdd(&LSS.fc, wtot);
        base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)lead);
        uint32_t off = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t pos = base + off + lanes_below(m[r]);
            off += (uint32_t)__popcll(m[r]);
            if ((fm >> r) & 1u) {
                if (pos < kLsFCap) LSS.F[pos] = k[r];
                else LSS.err = 13;  // the room check failed to make room (cannot happen)
            }
        }
    }
    if (bm) ls_bucket_append<R>(k, bb, bm, P);
}

// ------------------------------------------------------------------ coboundary keys
// Key of the cofacet of edge (a > b) (diameter sd) with vertex v, as
// k_reduce_par's col_cob: (diam bits << 32) | tri_lo (packed vertex triple +
// apparent facet f for N <= 1024, else ~colex index).
template <bool PACKED>
__device__ __forceinline__ bool ls_key1(int v, int n, int a, int b, float sd, float r, float da, float db, uint64_t& key) {
    if (v >= n || v == a || v == b) return false;
    const float cd = fmaxf(sd, fmaxf(da, db));
    if (!(cd <= r)) return false;
    int x, y, z;
    float ex, ey, ez;
    if (v > a) {
        x = v, y = a, z = b;
        ex = sd, ey = db, ez = da;
    } else if (v > b) {
        x = a, y = v, z = b;
        ex = db, ey = sd, ez = da;
    } else {
        x = a, y = b, z = v;
        ex = db, ey = da, ez = sd;
    }
    int f = 0;
    float fd = ex;
    if (ey > fd) f = 1, fd = ey;
    if (ez > fd) f = 2;
    key = ((uint64_t)__float_as_uint(cd + 0.0f) << 32) | tri_lo<PACKED>(x, y, z, f);
    return true;
}
// High part of that key (every key of vertex v is in [hi, hi + 2^32)), or
// kEmpty64 if v has no cofacet <= r.
__device__ __forceinline__ uint64_t ls_hi1(int v, int n, int a, int b, float sd, float r, float da, float db) {
    if (v >= n || v == a || v == b) return kEmpty64;
    const float cd = fmaxf(sd, fmaxf(da, db));
    if (!(cd <= r)) return kEmpty64;
    return (uint64_t)__float_as_uint(cd + 0.0f) << 32;
}

// Cofacet of triangle (a > b > c) with vertex v, as col_cob2: PACKED (N <=
// 400) lo32 = ~(tetrahedron index << 2 | f), unpacked ~index, WIDE (N > 568)
// code << 42 | (2^42 - 1 - index) with the rows holding edge codes.
template <bool PACKED, bool WIDE>
__device__ __forceinline__ bool ls_key2(int v, int n, const int (&vs)[3], float sd, float r, float da, float db, float dc,
                                        float eab, float eac, float ebc, uint64_t& key) {
    const int a = vs[0], b = vs[1], c = vs[2];
    if (v >= n || v == a || v == b || v == c) return false;
    if constexpr (WIDE) {
        const uint32_t cc = max(max(__float_as_uint(sd), __float_as_uint(da)), max(__float_as_uint(db), __float_as_uint(dc)));
        if (cc >= kCodeInf) return false;
        key = ((uint64_t)cc << kWideIdxBits) | (kWideIdxMask - cofacet_index<2>(vs, v));
        return true;
    } else {
        const float cd = fmaxf(fmaxf(sd, da), fmaxf(db, dc));
        if (!(cd <= r)) return false;
        const float oa = fmaxf(ebc, fmaxf(db, dc));
        const float ob = fmaxf(eac, fmaxf(da, dc));
        const float oc = fmaxf(eab, fmaxf(da, db));
        const int pv = v > a ? 0 : v > b ? 1 : v > c ? 2 : 3;
        float ex[4];
        ex[0] = pv == 0 ? sd : oa;
        ex[1] = pv == 0 ? oa : pv == 1 ? sd : ob;
        ex[2] = pv <= 1 ? ob : pv == 2 ? sd : oc;
        ex[3] = pv <= 2 ? oc : sd;
        int f = 0;
        float fd = ex[0];
#pragma unroll
        for (int u = 1; u < 4; ++u)
            if (ex[u] > fd) f = u, fd = ex[u];
        key = ((uint64_t)__float_as_uint(cd + 0.0f) << 32) | tet_lo<PACKED>(cofacet_index<2>(vs, v), f);
        return true;
    }
}
template <bool WIDE>
__device__ __forceinline__ uint64_t ls_hi2(int v, int n, const int (&vs)[3], float sd, float r, float da, float db, float dc) {
    if (v >= n || v == vs[0] || v == vs[1] || v == vs[2]) return kEmpty64;
    if constexpr (WIDE) {
        const uint32_t cc = max(max(__float_as_uint(sd), __float_as_uint(da)), max(__float_as_uint(db), __float_as_uint(dc)));
        return cc >= kCodeInf ? kEmpty64 : (uint64_t)cc << kWideIdxBits;
    } else {
        const float cd = fmaxf(fmaxf(sd, da), fmaxf(db, dc));
        return cd <= r ? (uint64_t)__float_as_uint(cd + 0.0f) << 32 : kEmpty64;
    }
}

// ------------------------------------------------------------------ the leader's set
// A wave-private open-addressing set in LDS (kLsH slots): a key toggles by
// one probe chain per lane, all of a round's keys at once; the pivot is a
// 512-slot min scan by the one wave.  (A sorted register set measured slower:
// torus1024's longest column toggles ~26 keys below B per step, nearly all of
// them cancellations, so serial sorted inserts and frequent pulls dominated.)
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

struct LsLeader {    // wave 0 (wave-uniform values)
    uint32_t c = 0;     // live keys in the set
    uint32_t used = 0;  // occupied slots (live + cancelled)
    uint64_t B = 0;     // bound
};

__device__ __forceinline__ void lh_reset(LsLeader& S) {
    const int ln = threadIdx.x & 63;
    for (uint32_t e = ln; e < kLsH; e += 64) LSS.H[e] = kEmpty64;
    S.c = 0;
    S.used = 0;
    wave_sync();
}

// Toggle each lane's key x (act) into the set: present (live or cancelled)
// -> its parity flips; absent -> inserted.  The keys of one call are
// distinct.  Keys >= B (none, by construction) would go out to the front.
__device__ __forceinline__ void lh_toggle(LsLeader& S, uint64_t x, bool act, const ParBufs& P) {
    const bool out = act && x >= S.B;
    if (__ballot(out)) {
        const uint64_t k1[1] = {x};
        ls_route_p<1>(k1, out ? 1u : 0u, P);
    }
    bool pend = act && !out;
    int dl = 0, du = 0;
    uint32_t h = (uint32_t)mix64(x) & (kLsH - 1);
    for (uint32_t it = 0; it < 4 * kLsH && __ballot(pend); ++it) {
        if (pend) {
            const uint64_t cur = LSS.H[h];
            if (cur == kEmpty64) {
                const uint64_t old = atomicCAS((unsigned long long*)&LSS.H[h], (unsigned long long)kEmpty64, (unsigned long long)x);
                if (old == kEmpty64) {
                    dl += 1;
                    du += 1;
                    pend = false;
                }  // else: another lane took the slot: look at it again
            } else if ((cur & ~kDead) == x) {
                const uint64_t old = __hip_atomic_fetch_xor(&LSS.H[h], kDead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                dl += (old & kDead) ? 1 : -1;
                pend = false;
            } else {
                h = (h + 1) & (kLsH - 1);
            }
        }
    }
    if (__ballot(pend) && (threadIdx.x & 63) == 0) LSS.err = 36;  // the set is full (the caller keeps it below half)
    S.c += (uint32_t)(int)wave_sum_u64((uint64_t)(int64_t)dl);
    S.used += (uint32_t)wave_sum_u64((uint64_t)du);
    wave_sync();
}

// smallest live key of the set (kEmpty64 if none)
__device__ __forceinline__ uint64_t lh_min() {
    const int ln = threadIdx.x & 63;
    uint64_t b = kEmpty64;
#pragma unroll
    for (uint32_t e = 0; e < kLsH; e += 64) {
        const uint64_t x = LSS.H[e + ln];
        b = x < b ? x : b;  // cancelled entries and free slots have bit 63 set
    }
    b = wave_min_u64(b);
    return b < kDead ? b : kEmpty64;
}

// every live key of the set out to the front / back; B drops to the smallest
__device__ __forceinline__ void lh_flush(LsLeader& S, const ParBufs& P) {
    const int ln = threadIdx.x & 63;
    if (S.c) {
        S.B = lh_min();
        for (uint32_t e = 0; e < kLsH; e += 64) {
            const uint64_t x = LSS.H[e + ln];
            const uint64_t k1[1] = {x};
            ls_route_p<1>(k1, x < kDead ? 1u : 0u, P);
        }
    }
    lh_reset(S);
    if (ln == 0) {
        LSS.B = S.B;
        LSS.lsc = 0;
    }
}

// rebuild the set without its cancelled entries (slots fill up with them)
__device__ __forceinline__ void lh_rebuild(LsLeader& S, const ParBufs& P) {
    const int ln = threadIdx.x & 63;
    uint64_t x[kLsH / 64];
#pragma unroll
    for (uint32_t r = 0; r < kLsH / 64; ++r) x[r] = LSS.H[r * 64 + ln];
    wave_sync();
    lh_reset(S);
#pragma unroll
    for (uint32_t r = 0; r < kLsH / 64; ++r) lh_toggle(S, x[r], x[r] < kDead, P);
}

// ------------------------------------------------------------------ column state
struct LsCol {
    LsRed rd;
    uint64_t adds = 0;
#ifdef TDA_PROFILE
    uint64_t q[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // pulls, pull cycles, bucket refills, refill cycles, room syncs, room cycles, candidates, evictions
#endif
};

// Block-wide: drop tombstones from the front; if it is still too full for
// `need` more keys, spill its highest levels to HBM (kf drops).
__device__ __forceinline__ void ls_room(LsCol& C, const ParBufs& P, uint32_t need) {
    __syncthreads();
    // compaction (in place, order kept: each chunk is read before the barrier in prefix)
    const uint32_t c = LSS.fc;
    uint32_t w = 0;
    for (uint32_t e0 = 0; e0 < c; e0 += kLsT) {
        const uint32_t e = e0 + threadIdx.x;
        const uint64_t x = e < c ? LSS.F[e] : kLsTomb;
        const bool lv = x != kLsTomb;
        uint32_t tot;
        const uint32_t o = C.rd.prefix(lv ? 1u : 0u, &tot);
        if (lv) LSS.F[w + o] = x;  // w + o <= e
        w += tot;
    }
    __syncthreads();
    if (threadIdx.x == 0) LSS.fc = w;
    __syncthreads();
    if (w + need <= kLsFCap) return;
    // spill: keep the lowest levels (relative to last) holding at most kLsFill keys
    for (uint32_t q = threadIdx.x; q < kParLv; q += kLsT) LSS.hist[q] = 0;
    __syncthreads();
    const uint64_t last = LSS.last;
    for (uint32_t e = threadIdx.x; e < w; e += kLsT) atomicAdd(&LSS.hist[par_bucket(LSS.F[e], last)], 1u);
    __syncthreads();
    int keep = par_keep_level(LSS.hist, (int)min(LSS.kf + 1u, 64u), kLsFill);
    if (keep < 0) {
        if (LSS.hist[0] + need <= kLsFCap) keep = 0;
        else if (threadIdx.x == 0) LSS.err = 31;
    }
    __syncthreads();
    if (LSS.err) return;
    uint32_t w2 = 0;
    for (uint32_t e0 = 0; e0 < w; e0 += kLsT) {
        const uint32_t e = e0 + threadIdx.x;
        const uint64_t x = e < w ? LSS.F[e] : 0ull;
        const uint32_t b = e < w ? par_bucket(x, last) : 0u;
        const bool out = e < w && b > (uint32_t)keep;
        uint64_t k1[1] = {x};
        uint32_t b1[1] = {b};
        ls_bucket_append<1>(k1, b1, out ? 1u : 0u, P);
        uint32_t tot;
        const uint32_t o = C.rd.prefix((e < w && !out) ? 1u : 0u, &tot);  // barrier: the chunk has been read
        if (e < w && !out) LSS.F[w2 + o] = x;
        w2 += tot;
        __syncthreads();  // chunk pointers opened by this pass
    }
    if (threadIdx.x == 0) {
        LSS.fc = w2;
        LSS.kf = (uint32_t)keep;
    }
    __syncthreads();
}

// Block-wide: the front is empty -- redistribute the lowest non-empty HBM
// bucket relative to its minimum (k_reduce_par's col_refill, with the front
// keys appended raw).  Returns false when no bucket is left (zero column).
__device__ __forceinline__ bool ls_bucket_refill(LsCol& C, const ParBufs& P) {
    __syncthreads();
    const int b = ls_first_bucket(LSS.kf + 1);
    if (b < 0) return false;
    const uint32_t c = LSS.bcnt[b];
    constexpr uint32_t kPass = kLsT * kParRegs;
    for (uint32_t q = threadIdx.x; q < kParLv; q += kLsT) LSS.hist[q] = 0;
    if (threadIdx.x == 0) LSS.fc = 0;
    auto batch = [&](uint32_t e0, uint64_t (&x)[kParRegs]) -> uint32_t {
        uint32_t vm = 0;
#pragma unroll
        for (int r = 0; r < kParRegs; ++r) {
            const uint32_t e = e0 + threadIdx.x + r * kLsT;
            x[r] = e < c ? ls_bucket_at(P, (uint32_t)b, e) : kEmpty64;
            if (e < c) vm |= 1u << r;
        }
        return vm;
    };
    uint64_t mn = kEmpty64;
    for (uint32_t e0 = 0; e0 < c; e0 += kPass) {
        uint64_t y[kParRegs];
        (void)batch(e0, y);
#pragma unroll
        for (int r = 0; r < kParRegs; ++r) mn = y[r] < mn ? y[r] : mn;
    }
    mn = C.rd.min(mn);
    const uint64_t nl = mn;
#ifdef TDA_LS_CHECK
    if (threadIdx.x == 0 && nl < LSS.B) LSS.err = 91;  // a back key below B
#endif
    for (uint32_t e0 = 0; e0 < c; e0 += kPass) {
        uint64_t y[kParRegs];
        const uint32_t ym = batch(e0, y);
#pragma unroll
        for (int r = 0; r < kParRegs; ++r)
            if ((ym >> r) & 1u) atomicAdd(&LSS.hist[par_bucket(y[r], nl)], 1u);
    }
    __syncthreads();
    int keep = par_keep_level(LSS.hist, b, kLsFill);
    if (keep < 0) {
        if (LSS.hist[0] <= kLsFCap / 2) keep = 0;
        else {
            if (threadIdx.x == 0) LSS.err = 32;
            __syncthreads();
            return false;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        LSS.bcnt[b] = 0;
        LSS.last = nl;
        LSS.kf = (uint32_t)keep;
        LSS.B = nl;
    }
    __syncthreads();
    for (uint32_t e0 = 0; e0 < c; e0 += kPass) {
        uint64_t y[kParRegs];
        const uint32_t ym = batch(e0, y);
        __syncthreads();  // chunk pointers opened by the previous pass
        ls_route_p<kParRegs>(y, ym, P);  // level <= keep: front; below b: lower buckets
    }
    __syncthreads();
    return LSS.err == 0;
}

// Block-wide: move the smallest front keys (levels 0..q relative to B, at
// most kLsPull raw keys) to the leader.  Returns false when the front is
// empty.  LS is empty on entry.
__device__ __forceinline__ bool ls_pull(LsCol& C, LsLeader& S, const ParBufs& P) {
    const int wv = threadIdx.x >> 6;
    for (int pass = 0; pass < 130; ++pass) {
        __syncthreads();
        const uint64_t lo = LSS.B;
        const uint32_t fc = LSS.fc;
        for (uint32_t q = threadIdx.x; q < kParLv; q += kLsT) LSS.hist[q] = 0;
        __syncthreads();
        for (uint32_t e = threadIdx.x; e < fc; e += kLsT) {
            const uint64_t x = LSS.F[e];
            if (x != kLsTomb) atomicAdd(&LSS.hist[par_bucket(x, lo)], 1u);
#ifdef TDA_LS_CHECK
            if (x != kLsTomb && x < lo) LSS.err = 90;  // (I2): a front key below B
            if (x != kLsTomb && x < LSS.last) LSS.err = 93;
#endif
        }
        __syncthreads();
        // every wave: total, the level q to pull up to, its cumulative count
        const int ln = threadIdx.x & 63;
        uint32_t hx = ln < 64 ? LSS.hist[ln] : 0u;
        uint32_t cum = hx;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)cum, o, 64);
            if (ln >= o) cum += y;
        }
        const uint32_t h64 = LSS.hist[64];
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)cum, 63) + h64;
        if (total == 0) return false;
        const uint64_t okm = __ballot(cum <= kLsPull);
        int q = okm ? 63 - __builtin_clzll(okm) : -1;  // largest level <= 63 with cum <= kLsPull
        uint32_t cq = q >= 0 ? (uint32_t)__builtin_amdgcn_readlane((int)cum, q) : 0u;
        if (q == 63 && total <= kLsPull) {
            q = 64;
            cq = total;
        }
        if (cq == 0) {
            if (q < 0) {
                // level 0 alone exceeds the pull: all its keys equal lo -- parity decides
                const uint32_t h0 = LSS.hist[0];
                for (uint32_t e = threadIdx.x; e < fc; e += kLsT)
                    if (LSS.F[e] == lo) LSS.F[e] = kLsTomb;
                __syncthreads();
                if (wv == 0) {
                    lh_reset(S);
                    S.B = lo + 1;  // before the toggle: keys >= B would be routed back out
                    lh_toggle(S, lo, (h0 & 1u) && ln == 0, P);
                    if (ln == 0) {
                        LSS.B = S.B;
                        LSS.lsc = S.c;
                    }
                }
                __syncthreads();
                if (LSS.lsc) return true;
                continue;
            }
            // levels 0..q are empty: every key is in level q + 1 or above, whose
            // range starts at lo's bits above q, then bit q set
            if (q >= 63) {
                if (threadIdx.x == 0) LSS.err = 35;
                return false;
            }
            if (threadIdx.x == 0) LSS.B = ((lo >> (q + 1)) << (q + 1)) | (1ull << q);
            continue;
        }
        // keys < T: exactly levels 0..q; capped at the front's upper radix bound,
        // above which the HBM buckets start (B must stay <= every back key: I1)
        const uint32_t kf = LSS.kf;
        const uint64_t fu = kf >= 64 ? kEmpty64 : ((LSS.last >> kf) + 1) << kf;
        uint64_t T = q >= 64 ? kEmpty64 : (q == 0 ? lo + 1 : ((lo >> q) + 1) << q);
        T = T < fu ? T : fu;
        // gather keys < T into pull (any order: the set does not care), tombstone them
        if (threadIdx.x == 0) LSS.npull = 0;
        __syncthreads();
        for (uint32_t e0 = 0; e0 < fc; e0 += kLsT) {
            const uint32_t e = e0 + threadIdx.x;
            const uint64_t x = e < fc ? LSS.F[e] : kLsTomb;
            const bool tk = x < T;
            const uint64_t m = __ballot(tk);
            if (m) {
                const uint32_t lead = (uint32_t)__builtin_ctzll(m);
                uint32_t base = 0;
                if ((uint32_t)ln == lead) base = atomicAdd(&LSS.npull, (uint32_t)__popcll(m));
                base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)lead);
                if (tk) {
                    const uint32_t pos = base + lanes_below(m);
                    if (pos < kLsPull) LSS.pull[pos] = x;
                    LSS.F[e] = kLsTomb;
                }
            }
        }
        __syncthreads();
        const uint32_t got = LSS.npull < kLsPull ? LSS.npull : kLsPull;
        if (wv == 0) {
            lh_reset(S);
            S.B = T;  // before the toggles: keys >= B would be routed back out
            for (uint32_t r0 = 0; r0 < got; r0 += 64) {
                const uint32_t i = r0 + (uint32_t)ln;
                lh_toggle(S, i < got ? LSS.pull[i] : 0ull, i < got, P);
            }
#ifdef TDA_PROFILE
            C.q[4] += S.c;
            C.q[5] += got;
#endif
            if (ln == 0) {
                LSS.B = S.B;
                LSS.lsc = S.c;
            }
        }
        __syncthreads();
        if (LSS.lsc) return true;
        // everything cancelled: pull again above T
    }
    if (threadIdx.x == 0) LSS.err = 33;
    return false;
}

// Block-wide: LS is empty -- next keys from the front, or from HBM buckets.
__device__ __forceinline__ bool ls_refill(LsCol& C, LsLeader& S, const ParBufs& P) {
    for (int it = 0; it < 200; ++it) {
#ifdef TDA_PROFILE
        const uint64_t t0 = clock64();
#endif
        const bool got = ls_pull(C, S, P);
#ifdef TDA_PROFILE
        C.q[0] += 1;
        C.q[1] += clock64() - t0;
#endif
        if (got) return true;
        if (LSS.err) return false;
#ifdef TDA_PROFILE
        const uint64_t t1 = clock64();
#endif
        const bool more = ls_bucket_refill(C, P);
#ifdef TDA_PROFILE
        C.q[2] += 1;
        C.q[3] += clock64() - t1;
#endif
        if (!more) return false;
    }
    if (threadIdx.x == 0) LSS.err = 34;
    return false;
}

// Block-wide: add len keys src[0, len) (plain loads: the caller acquired) to
// the column; LS is empty and every key is >= B.
__device__ __forceinline__ void ls_add_keys(LsCol& C, const ParBufs& P, const uint64_t* src, uint64_t len) {
    for (uint64_t e0 = 0; e0 < len; e0 += kLsT * kParRegs) {
        uint64_t x[kParRegs];
        uint32_t vm = 0;
#pragma unroll
        for (int q = 0; q < kParRegs; ++q) {
            const uint64_t e = e0 + threadIdx.x + (uint64_t)q * kLsT;
            x[q] = e < len ? ld_glb(src, e) : 0;
            if (e < len) vm |= 1u << q;
        }
        __syncthreads();
        if (LSS.fc + kLsT * kParRegs > kLsFCap) ls_room(C, P, kLsT * kParRegs);
        if (LSS.err) return;
        ls_route_p<kParRegs>(x, vm, P);
    }
    __syncthreads();
}

__device__ __forceinline__ void ls_add_record(LsCol& C, const ParBufs& P, uint64_t id) {
    if (threadIdx.x == 0) {
        LSS.bc[2] = ald(P.rec + id * 4 + 0);
        LSS.bc[3] = ald(P.rec + id * 4 + 1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        drain_vm();
    }
    __syncthreads();
    const uint64_t h0 = LSS.bc[2], h1 = LSS.bc[3];
    __syncthreads();
    const uint64_t off = h0 & ~kParSegBit;
    if (!(h0 & kParSegBit)) {
        ls_add_keys(C, P, P.rpool + off, h1);
    } else {
        const uint64_t nfront = h1 & 0xFFFFFFFFull, ns = h1 >> 32;
        const uint64_t* tab = P.rpool + off + nfront;
        ls_add_keys(C, P, P.rpool + off, nfront);
        for (uint64_t g = 0; g < ns && !LSS.err; ++g) ls_add_keys(C, P, P.bpool + ld_glb(tab, 2 * g), ld_glb(tab, 2 * g + 1));
    }
    __syncthreads();
}

// Block-wide: publish the column (LS flushed: front + buckets) as an
// immutable record, as col_save (copy, or zero-copy segments above kParSegMin).
__device__ __forceinline__ int64_t ls_save(LsCol& C, const ParBufs& P, uint64_t pkey, uint64_t item, bool* seg) {
    drain_vm();
    __syncthreads();
    const uint32_t c = LSS.fc;
    uint32_t lv = 0;
    for (uint32_t e = threadIdx.x; e < c; e += kLsT) lv += LSS.F[e] != kLsTomb;
    const uint64_t nfront = C.rd.sum(lv);
    uint64_t nback = 0;
    for (int q = 0; q < kParLv; ++q) nback += LSS.bcnt[q];
    const uint64_t total = nfront + nback;
    const bool segd = total > kParSegMin;
    constexpr uint32_t kSegs = (uint32_t)kParLv * kParChunks;
    const uint64_t words = segd ? nfront + 2ull * kSegs : total;
    if (threadIdx.x == 0) {
        const uint64_t o = aadd(&P.ctl->rpool_used, (words + 15) & ~15ull);
        const uint64_t id = aadd(&P.ctl->rec_used, 1ull);
        LSS.bc[0] = (o + words <= P.rpool_cap && id < P.rec_cap) ? o : kEmpty64;
        LSS.bc[1] = id;
    }
    __syncthreads();
    const uint64_t off = LSS.bc[0], id = LSS.bc[1];
    if (off == kEmpty64) {
        if (threadIdx.x == 0) LSS.err = 41;
        __syncthreads();
        return -1;
    }
    uint64_t* out = P.rpool + off;
    uint32_t w = 0;
    for (uint32_t e0 = 0; e0 < c; e0 += kLsT) {
        const uint32_t e = e0 + threadIdx.x;
        const uint64_t x = e < c ? LSS.F[e] : kLsTomb;
        const bool live = x != kLsTomb;
        uint32_t tot;
        const uint32_t o = C.rd.prefix(live ? 1u : 0u, &tot);
        if (live) ast(out + w + o, x);
        w += tot;
    }
    uint64_t hdr1 = total;
    if (segd) {
        uint32_t ns = 0;
        for (uint32_t e0 = 0; e0 < kSegs; e0 += kLsT) {
            const uint32_t e = e0 + threadIdx.x;
            const uint32_t q = e / kParChunks, kc = e % kParChunks;
            uint32_t cnt = 0;
            if (e < kSegs) {
                const uint32_t cq = LSS.bcnt[q], lo = chunk_start(kc);
                if (lo < cq) cnt = min(cq, chunk_start(kc + 1)) - lo;
            }
            uint32_t tot;
            const uint32_t o = C.rd.prefix(cnt ? 1u : 0u, &tot);
            if (cnt) {
                ast(out + nfront + 2 * (ns + o), (uint64_t)LSS.cptr[q][kc] * 256);
                ast(out + nfront + 2 * (ns + o) + 1, (uint64_t)cnt);
            }
            ns += tot;
        }
        hdr1 = nfront | ((uint64_t)ns << 32);
    } else {
        uint64_t pos = nfront;
        for (int q = 0; q < kParLv; ++q) {
            const uint32_t cq = LSS.bcnt[q];
            for (uint32_t e0 = 0; e0 < cq; e0 += kLsT * kParRegs) {
#pragma unroll
                for (int r = 0; r < kParRegs; ++r) {
                    const uint32_t e = e0 + threadIdx.x + r * kLsT;
                    if (e < cq) ast(out + pos + e, ls_bucket_at(P, (uint32_t)q, e));
                }
            }
            pos += cq;
        }
    }
    drain_vm();
    __syncthreads();
    if (threadIdx.x == 0) {
        if (segd) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        uint64_t* rh = P.rec + id * 4;
        ast(rh + 0, off | (segd ? kParSegBit : 0ull));
        ast(rh + 1, hdr1);
        ast(rh + 2, pkey);
        ast(rh + 3, item);
    }
    drain_vm();
    __syncthreads();
    *seg = segd;
    return (int64_t)id;
}

// ------------------------------------------------------------------ pivot decode (leader)
// facet of pivot key pk whose coboundary eliminates it, the pivot's diameter
// (or the facet's code), its index.  PACKED keys decode with shifts; the
// others read distances (apparent_facet).
template <int DIM, bool PACKED, bool WIDE>
__device__ __forceinline__ void ls_decode(uint64_t pk, const float* D, const uint32_t* Dc, int n, const uint64_t* dsort_l, int (&fv)[3],
                                          float& pd, uint32_t& fsc, uint64_t& pidx) {
    const uint32_t plo = 0xFFFFFFFFu - (uint32_t)pk;
    fsc = 0;
    pd = WIDE ? 0.0f : __uint_as_float((uint32_t)(pk >> 32));
    fv[2] = 0;
    if constexpr (DIM == 1) {
        int t[3];
        if (PACKED) {
            t[0] = (int)(plo >> 22);
            t[1] = (int)((plo >> 12) & 1023u);
            t[2] = (int)((plo >> 2) & 1023u);
            const int f = (int)(plo & 3u);
            fv[0] = f == 0 ? t[1] : t[0];
            fv[1] = f == 2 ? t[1] : t[2];
            pidx = encode<2>(t);
        } else {
            pidx = plo;
            int f2[2];
            (void)apparent_facet<1>(D, n, pidx, f2);
            fv[0] = f2[0];
            fv[1] = f2[1];
        }
    } else if constexpr (WIDE) {
        pidx = kWideIdxMask - (pk & kWideIdxMask);
        (void)apparent_facet<2>(D, n, pidx, fv);
        fsc = max(ld_glb(Dc, (size_t)fv[0] * n + fv[1]), max(ld_glb(Dc, (size_t)fv[0] * n + fv[2]), ld_glb(Dc, (size_t)fv[1] * n + fv[2])));
        pd = __uint_as_float((uint32_t)ld_glb(dsort_l, pk >> kWideIdxBits));
    } else {
        if (PACKED) {
            pidx = plo >> 2;
            const int f = (int)(plo & 3u);
            int t[4];
            decode<3>(pidx, n, t);
#pragma unroll
            for (int u = 0, q = 0; u < 4; ++u)
                if (u != f) fv[q++] = t[u];
        } else {
            pidx = plo;
            (void)apparent_facet<2>(D, n, pidx, fv);
        }
    }
}

// ------------------------------------------------------------------ kernel
// RV: coboundary vertices per worker lane per step (workers cover 448 * RV
// vertices: RV = 3 up to N = 1344, 7 up to N = 3136).
template <int DIM, bool PACKED, bool WIDE, int RV>
__global__ __launch_bounds__(kLsT) void k_reduce_ls(const float* __restrict__ dist, int n, int L, LayerStats* __restrict__ stats,
                                                    DimBufs b1, const uint32_t* __restrict__ clr, uint64_t clr_words, Reduce2Bufs rb,
                                                    ParBufs P, const uint32_t* __restrict__ dcode, const uint64_t* __restrict__ dsort,
                                                    uint64_t ecap) {
    static_assert(!WIDE || (DIM == 2 && !PACKED), "wide keys: unpacked H2 rows only");
    LsCol C;
    const int tid = threadIdx.x, ln = tid & 63, wv = tid >> 6;
    for (uint32_t e = tid; e < (uint32_t)kParLv * kParChunks; e += kLsT) (&LSS.cptr[0][0])[e] = kNoChunk;
    if (tid == 0) {
        LSS.err = 0;
        LSS.wide = WIDE ? 1u : 0u;
    }
    __syncthreads();
    const uint64_t total = ald(&P.ctl->total);
    bool prealloc = false;
    LsLeader S;
    // worker stash: the keys of the last step, appended once it is known to be apparent
    uint64_t sk[RV];
    uint32_t sm = 0;
    for (;;) {
        // ---------------- work: requeued columns first, then fresh ones (as k_reduce_par)
        if (tid == 0) {
            uint64_t got = kEmpty64;
            for (uint32_t spin = 0; spin < kParSpin; ++spin) {
                if (ald(&P.ctl->abort)) break;
                const uint64_t h = ald(&P.ctl->rq_head), t = ald(&P.ctl->rq_tail);
                if (h < t && h < P.rq_cap) {
                    if (acas((uint64_t*)&P.ctl->rq_head, h, h + 1) != h) continue;
                    uint64_t v = 0;
                    for (uint32_t q = 0; q < kParSpin && !(v = ald(P.rq + h)); ++q) __builtin_amdgcn_s_sleep(1);
                    if (!v) {
                        aadd(&P.ctl->abort, 1);
                        acas((uint64_t*)&P.ctl->err, 0, 51);
                        break;
                    }
                    ast(P.rq + h, 0);
                    got = v;
                    break;
                }
                if (ald(&P.ctl->next) < total) {
                    const uint64_t c = aadd(&P.ctl->next, 1);
                    if (c < total) got = c << 32;
                }
                break;
            }
            LSS.bc[4] = got;
        }
        __syncthreads();
        const uint64_t got = LSS.bc[4];
        __syncthreads();
        if (got == kEmpty64) break;
        const uint64_t item = got >> 32;
        const uint64_t rec0 = got & 0xFFFFFFFFull;
        int l = 0;
        while (l + 1 < L && ld_glb(P.item_base, l + 1) <= item) ++l;
        const uint64_t j = item - ld_glb(P.item_base, l);
        LayerStats* st = stats + l;
        const float r = st->thresh;
        const float* D = dist + (size_t)l * n * n;
        const float* Dr = WIDE ? (const float*)(dcode + (size_t)l * n * n) : D;
        const uint32_t* Dc = (const uint32_t*)Dr;
        const uint64_t* dsort_l = WIDE ? dsort + (size_t)l * ecap : nullptr;
        const uint64_t* resid = b1.resid + (size_t)l * b1.rcap;
        const uint32_t* pivg = b1.pivbits + (size_t)l * b1.piv_words;
        const uint32_t* mst = rb.mst + (size_t)l * rb.mst_words;
        uint64_t* okey = P.okey + (size_t)l * P.ostride;
        uint64_t* oval = P.oval + (size_t)l * P.ostride;
        const uint64_t nres_l = ld_glb(P.item_base, l + 1) - ld_glb(P.item_base, l);
        const uint64_t omask = par_omask(nres_l, P.ostride);
        uint64_t* colpiv = P.colpiv + (size_t)l * b1.rcap;
        const uint64_t ckey = ld_glb(resid, j);
        const uint64_t sidx = key_idx(ckey);
        const float sdm = key_diam(ckey);
        int sv[DIM + 1];
        decode<DIM>(sidx, n, sv);
        const uint32_t* cbits = DIM == 1 ? mst : clr + (size_t)l * clr_words;
        if (!rec0 && ((ld_glb(cbits, sidx >> 5) >> (sidx & 31)) & 1u)) {  // cleared: an H_{DIM-1} death
            if (tid == 0) ast(colpiv + j, kParSkip);
            continue;
        }
        if (!prealloc) {  // chunks 0..3 of every bucket
            if (tid == 0) {
                constexpr uint64_t per = (uint64_t)kParLv * chunk_start(4);
                const uint64_t o = aadd(&P.ctl->bpool_used, per);
                LSS.bc[5] = o + per <= P.bpool_cap ? o : kEmpty64;
            }
            __syncthreads();
            const uint64_t o = LSS.bc[5];
            if (o == kEmpty64) {
                if (tid == 0) {
                    acas((uint64_t*)&P.ctl->err, 0, ((uint64_t)item << 16) | 22u);
                    aadd(&P.ctl->abort, 1);
                }
                break;
            }
            for (uint32_t e = tid; e < (uint32_t)kParLv * 4u; e += kLsT)
                LSS.cptr[e / 4][e % 4] = (uint32_t)((o + (e / 4) * chunk_start(4) + chunk_start(e % 4)) >> 8);
            prealloc = true;
        }
        // ---------------- column state: empty LS, empty front, empty buckets
        for (uint32_t q = tid; q < kParLv; q += kLsT) LSS.bcnt[q] = 0;
        uint32_t sc = 0;  // WIDE: the column's edge code
        if constexpr (WIDE)
            sc = max(ld_glb(Dc, (size_t)sv[0] * n + sv[1]), max(ld_glb(Dc, (size_t)sv[0] * n + sv[2]), ld_glb(Dc, (size_t)sv[1] * n + sv[2])));
        const uint64_t base_key = WIDE ? (uint64_t)sc << kWideIdxBits : (uint64_t)__float_as_uint(sdm + 0.0f) << 32;
        if (tid == 0) {
            LSS.kf = kParLv - 1;  // everything in the front until a spill
            LSS.fc = 0;
            LSS.lsc = 0;
            LSS.last = base_key;
            LSS.B = base_key;
            if (rec0) {
                const uint64_t pk = ald(P.rec + (rec0 - 1) * 4 + 2);  // the record's pivot: its smallest key
                LSS.last = pk;
                LSS.B = pk;
            }
            LSS.mb_kind[0] = LS_REFILL;
            LSS.mb_prev[0] = 0;
        }
        if (wv == 0) lh_reset(S);
        sm = 0;
        __syncthreads();
        S.B = LSS.B;
        if (!rec0) {  // the column's coboundary: every key to the front (kf = 64)
            float eab = 0.0f, eac = 0.0f, ebc = 0.0f;
            if constexpr (DIM == 2 && !WIDE) {
                eab = ld_glb(D, (size_t)sv[0] * n + sv[1]);
                eac = ld_glb(D, (size_t)sv[0] * n + sv[2]);
                ebc = ld_glb(D, (size_t)sv[1] * n + sv[2]);
            }
            const float sdk = WIDE ? __uint_as_float(sc) : sdm;
            for (int v0 = 0; v0 < n; v0 += kLsT * kParRegs) {
                uint64_t k[kParRegs];
                uint32_t vm = 0;
#pragma unroll
                for (int q = 0; q < kParRegs; ++q) {
                    const int v = v0 + tid + q * kLsT;
                    k[q] = 0;
                    bool ok = false;
                    if (v < n) {
                        if constexpr (DIM == 1)
                            ok = ls_key1<PACKED>(v, n, sv[0], sv[1], sdk, r, ld_glb(Dr, (size_t)sv[0] * n + v), ld_glb(Dr, (size_t)sv[1] * n + v), k[q]);
                        else {
                            const int vs3[3] = {sv[0], sv[1], DIM == 2 ? sv[DIM] : 0};
                            ok = ls_key2<PACKED, WIDE>(v, n, vs3, sdk, r, ld_glb(Dr, (size_t)sv[0] * n + v), ld_glb(Dr, (size_t)sv[1] * n + v),
                                                       ld_glb(Dr, (size_t)vs3[2] * n + v), eab, eac, ebc, k[q]);
                        }
                    }
                    if (ok) vm |= 1u << q;
                }
                __syncthreads();
                if (LSS.fc + kLsT * kParRegs > kLsFCap) ls_room(C, P, kLsT * kParRegs);
                ls_route_p<kParRegs>(k, vm, P);
            }
            __syncthreads();
        } else {
            ls_add_record(C, P, rec0 - 1);
        }
        int64_t my_rec = -1;
        bool my_seg = false;
        uint64_t adds = 0;
        bool done = false;
#ifdef TDA_PROFILE
        uint64_t pf[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // total, -, leader step, -, refill syncs, owner path, steps, -
        const uint64_t t_col = clock64();
        for (int q = 0; q < 8; ++q) C.q[q] = 0;
#endif
        // front keys one step can add: the workers' previous keys (<= n), the leader's keys >= B
        // and a flushed set (<= n + kLsH)
        const uint32_t margin = 2u * (uint32_t)n + kLsH + 64u;
        uint64_t step = 0;
        for (; !done; ++step) {
            if (step > P.step_limit) {
                if (tid == 0) LSS.err = 61;
                __syncthreads();
                break;
            }
            // the step barrier; every wave's view of the front length and the error flag
            const uint32_t fl = C.rd.or2((LSS.fc + margin > kLsFCap ? 1u : 0u) | (LSS.err ? 2u : 0u));
            if (fl & 2u) break;
            const bool need_room = (fl & 1u) != 0;
            const uint32_t mb = (uint32_t)(step & 1);
            const uint32_t kind = LSS.mb_kind[mb];
            const bool prev_app = LSS.mb_prev[mb] != 0;
            if (need_room || kind != LS_STEP) {
#ifdef TDA_PROFILE
                const uint64_t ts0 = clock64();
#endif
                if (wv != 0 && prev_app) ls_route_p<RV>(sk, sm, P);
                sm = 0;
                __syncthreads();
                if (need_room) {
                    ls_room(C, P, margin);
                    if (LSS.err) break;
                }
                if (kind == LS_REFILL) {
                    const bool more = ls_refill(C, S, P);
                    if (!more) {
                        if (LSS.err) break;
                        if (tid == 0) ast(colpiv + j, kParEss);  // zero column: essential
                        done = true;
                        break;
                    }
                    if (wv == 0) {  // the pivot's facet for the next step
                        const uint64_t pk = lh_min();
                        int fv[3];
                        float pd;
                        uint32_t fsc;
                        uint64_t pidx;
                        ls_decode<DIM, PACKED, WIDE>(pk, D, Dc, n, dsort_l, fv, pd, fsc, pidx);
                        if (ln == 0) {
                            const uint32_t nb = (uint32_t)((step + 1) & 1);
                            LSS.mb_p[nb] = pk;
                            LSS.mb_pidx[nb] = pidx;
                            LSS.mb_B[nb] = S.B;
                            LSS.mb_fv[nb][0] = fv[0];
                            LSS.mb_fv[nb][1] = fv[1];
                            LSS.mb_fv[nb][2] = fv[2];
                            LSS.mb_pd[nb] = pd;
                            LSS.mb_fsc[nb] = fsc;
                            LSS.mb_kind[nb] = LS_STEP;
                            LSS.mb_prev[nb] = 0;
                        }
                    }
#ifdef TDA_PROFILE
                    pf[4] += clock64() - ts0;
#endif
                    continue;
                }
                if (kind == LS_OWNER) {
#ifdef TDA_PROFILE
                    const uint64_t to0 = clock64();
#endif
                    // ---------------- residual pivot p = LS[0]: owner map (as k_reduce_par)
                    const uint64_t pk = LSS.mb_p[mb];
                    const uint64_t pix = LSS.mb_pidx[mb];
                    const float pd = LSS.mb_pd[mb];
                    const uint64_t fkey = WIDE ? pk : filt_key(pd, pix);
                    bool added = false;
                    for (uint32_t round = 0;; ++round) {
                        if (tid == 0) {
                            uint64_t slot = 0;
                            bool found = false;
                            const uint64_t v = round > 64 ? kEmpty64 : omap_find(P, okey, oval, omask, pix, &slot, &found);
                            LSS.bc[6] = v;
                            LSS.bc[7] = slot;
                        }
                        __syncthreads();
                        const uint64_t v = LSS.bc[6];
                        const uint64_t slot = LSS.bc[7];
                        __syncthreads();
                        if (v == kEmpty64) {
                            if (tid == 0) LSS.err = 71;
                            break;
                        }
                        const uint64_t oi = v >> 32;
                        if (v != 0 && oi == j) {
                            if (tid == 0) LSS.err = 72;
                            break;
                        }
                        if (v != 0 && oi < j) {  // earlier owner: add its record
                            if (wv == 0) lh_flush(S, P);
                            __syncthreads();
                            ls_add_record(C, P, (v & 0xFFFFFFFFull) - 1);
                            ++adds;
                            added = true;
                            break;
                        }
                        // free, or owned by a later column: publish R_j, then claim
                        if (my_rec < 0) {
                            if (wv == 0) lh_flush(S, P);
                            __syncthreads();
                            my_rec = ls_save(C, P, pk, item, &my_seg);
                            if (my_rec < 0) break;
                        }
                        const uint64_t mine = (j << 32) | (uint64_t)(my_rec + 1);
                        if (tid == 0) {
                            bool ok;
                            if (v == 0) {
                                const uint64_t old = acas(okey + slot, 0, pix + 1);
                                ok = old == 0;
                                if (ok) ast(oval + slot, mine);
                            } else {
                                ok = acas(oval + slot, v, mine) == v;
                                if (ok) {
                                    const uint64_t qt = aadd(&P.ctl->rq_tail, 1);
                                    if (qt >= P.rq_cap) {
                                        aadd(&P.ctl->abort, 1);
                                        acas((uint64_t*)&P.ctl->err, 0, 53);
                                    } else {
                                        const uint64_t oitem = ld_glb(P.item_base, l) + oi;
                                        ast(P.rq + qt, (oitem << 32) | (v & 0xFFFFFFFFull));
                                    }
                                    aadd(&P.ctl->evictions, 1);
                                }
                            }
                            if (ok) ast(colpiv + j, fkey);
                            LSS.bc[6] = ok;
                        }
                        __syncthreads();
                        const bool ok = LSS.bc[6] != 0;
                        __syncthreads();
                        if (ok) {
                            done = true;
                            break;
                        }
                    }
                    if (added) my_rec = -1;  // the column changed: a saved record is stale
#ifdef TDA_PROFILE
                    pf[5] += clock64() - to0;
#endif
                    if (LSS.err || done) break;
                    // next: the smallest keys again (LS was flushed)
                    if (tid == 0) {
                        const uint32_t nb = (uint32_t)((step + 1) & 1);
                        LSS.mb_kind[nb] = LS_REFILL;
                        LSS.mb_prev[nb] = 0;
                    }
                    continue;
                }
                // LS_STEP after a room sync: go on with the step
                __syncthreads();
            }
            // ---------------- apparent step candidate: pivot p = LS[0], facet fv
            const uint64_t Bs = LSS.mb_B[mb];
            const int fa = LSS.mb_fv[mb][0], fb = LSS.mb_fv[mb][1], fcx = LSS.mb_fv[mb][2];
            const float pd = LSS.mb_pd[mb];
            const float sdk = WIDE ? __uint_as_float(LSS.mb_fsc[mb]) : pd;
            const int fvs[3] = {fa, fb, DIM == 2 ? fcx : 0};
            if (wv == 0) {
#ifdef TDA_PROFILE
                const uint64_t tl0 = clock64();
#endif
                // ---- leader: the pivot's bitmap word + the facet's full rows; the low keys into LS
                const uint64_t pk = LSS.mb_p[mb];
                const uint64_t pidx = LSS.mb_pidx[mb];
                const uint32_t pw = ld_glb(pivg, pidx >> 5);
                float eab = 0.0f, eac = 0.0f, ebc = 0.0f;
                if constexpr (DIM == 2 && !WIDE) {
                    eab = ld_glb(D, (size_t)fa * n + fb);
                    eac = ld_glb(D, (size_t)fa * n + fcx);
                    ebc = ld_glb(D, (size_t)fb * n + fcx);
                }
                const bool app = (pw >> (pidx & 31)) & 1u;
                uint32_t ncand = 0;
#ifdef TDA_PROFILE
                uint64_t tw = 0, tt = 0;
#endif
                if (app) {
                    for (int v0 = 0; v0 < n; v0 += 64 * kLsLV) {
                        float za[kLsLV], zb[kLsLV], zc[kLsLV];
#pragma unroll
                        for (int q = 0; q < kLsLV; ++q) {
                            const int v = v0 + ln + 64 * q;
                            za[q] = v < n ? ld_glb(Dr, (size_t)fa * n + v) : 0.0f;
                            zb[q] = v < n ? ld_glb(Dr, (size_t)fb * n + v) : 0.0f;
                            zc[q] = (DIM == 2 && v < n) ? ld_glb(Dr, (size_t)fcx * n + v) : 0.0f;
                        }
#ifdef TDA_PROFILE
                        const uint64_t tw0 = clock64();
                        float zs = 0.0f;
#pragma unroll
                        for (int q = 0; q < kLsLV; ++q) zs += za[q] + zb[q] + zc[q];
                        if (zs == -1.0f) C.q[7] += 1;  // forces the loads to complete here
                        tw += clock64() - tw0;
#endif
                        // vertices whose cofacet may be below B: compacted (vertex + rows) into
                        // LDS, then the full keys one per lane and one batch of set toggles
                        const uint64_t Bl = Bs;  // the workers took the keys >= Bs
                        uint32_t nc = 0;
#ifdef TDA_PROFILE
                        uint64_t tt0 = 0;
#endif
                        auto drain = [&]() {  // full keys of the buffered candidates, one batch of toggles per 64
#ifdef TDA_PROFILE
                            tt0 = clock64();
#endif
                            wave_sync();
                            for (uint32_t r0 = 0; r0 < nc; r0 += 64) {
                                if (S.used > kLsH / 2) {  // keep the probe chains short and the set below capacity
                                    if (S.c > kLsH / 4) lh_flush(S, P);
                                    else lh_rebuild(S, P);
                                }
                                const uint32_t i = r0 + (uint32_t)ln;
                                uint64_t key = 0;
                                bool ok = false;
                                if (i < nc) {
                                    const int v = LSS.cv[i];
                                    if constexpr (DIM == 1) ok = ls_key1<PACKED>(v, n, fa, fb, sdk, r, LSS.ca[i], LSS.cb[i], key);
                                    else ok = ls_key2<PACKED, WIDE>(v, n, fvs, sdk, r, LSS.ca[i], LSS.cb[i], LSS.cc[i], eab, eac, ebc, key);
                                    ok = ok && key < Bl;
                                }
                                lh_toggle(S, key, ok, P);
                                ncand += (uint32_t)__popcll(__ballot(ok));
                            }
                            nc = 0;
                            wave_sync();
#ifdef TDA_PROFILE
                            tt += clock64() - tt0;
#endif
                        };
#pragma unroll
                        for (int q = 0; q < kLsLV; ++q) {
                            const int v = v0 + ln + 64 * q;
                            uint64_t hi;
                            if constexpr (DIM == 1) hi = ls_hi1(v, n, fa, fb, sdk, r, za[q], zb[q]);
                            else hi = ls_hi2<WIDE>(v, n, fvs, sdk, r, za[q], zb[q], zc[q]);
                            const bool cand = hi < Bl;
                            const uint64_t m = __ballot(cand);
                            if (cand) {
                                const uint32_t pos = nc + lanes_below(m);
                                LSS.cv[pos] = v;
                                LSS.ca[pos] = za[q];
                                LSS.cb[pos] = zb[q];
                                LSS.cc[pos] = zc[q];
                            }
                            nc += (uint32_t)__popcll(m);
                            if (nc > kLsCand - 64) drain();
                        }
                        drain();
                    }
                }
#ifdef TDA_PROFILE
                C.q[6] += ncand;
                pf[2] += clock64() - tl0;
                pf[1] += tt;
                pf[3] += tw;
                pf[7] += S.c;
#endif
                (void)ncand;
                const uint32_t nb = (uint32_t)((step + 1) & 1);
                if (app) {
                    ++adds;
                    if (S.c > kLsHLive) lh_flush(S, P);                // too many low keys: back out, pull again
                    else if (S.used > kLsH * 3 / 4) lh_rebuild(S, P);  // cancelled entries fill the slots
                    const uint64_t pk2 = S.c ? lh_min() : kEmpty64;
                    if (S.c) {
                        int fv[3];
                        float pd2;
                        uint32_t fsc2;
                        uint64_t pidx2;
                        ls_decode<DIM, PACKED, WIDE>(pk2, D, Dc, n, dsort_l, fv, pd2, fsc2, pidx2);
                        if (ln == 0) {
                            LSS.mb_p[nb] = pk2;
                            LSS.mb_pidx[nb] = pidx2;
                            LSS.mb_B[nb] = S.B;
                            LSS.mb_fv[nb][0] = fv[0];
                            LSS.mb_fv[nb][1] = fv[1];
                            LSS.mb_fv[nb][2] = fv[2];
                            LSS.mb_pd[nb] = pd2;
                            LSS.mb_fsc[nb] = fsc2;
                            LSS.mb_kind[nb] = LS_STEP;
                            LSS.mb_prev[nb] = 1;
                        }
                    } else if (ln == 0) {
                        LSS.B = S.B;
                        LSS.lsc = 0;
                        LSS.mb_kind[nb] = LS_REFILL;
                        LSS.mb_prev[nb] = 1;
                    }
                } else if (ln == 0) {  // not apparent: the owner path for p (still LS[0])
                    LSS.mb_p[nb] = pk;
                    LSS.mb_pidx[nb] = pidx;
                    LSS.mb_pd[nb] = pd;
                    LSS.mb_kind[nb] = LS_OWNER;
                    LSS.mb_prev[nb] = 0;
                }
            } else {
                // ---- workers: the coboundary's keys >= B of their vertices, stashed
                const int wb = (wv - 1) * 64 + ln;
                float za[RV], zb[RV], zc[RV];
#pragma unroll
                for (int q = 0; q < RV; ++q) {
                    const int v = wb + q * (64 * kLsWorkers);
                    za[q] = v < n ? ld_glb(Dr, (size_t)fa * n + v) : 0.0f;
                    zb[q] = v < n ? ld_glb(Dr, (size_t)fb * n + v) : 0.0f;
                    zc[q] = (DIM == 2 && v < n) ? ld_glb(Dr, (size_t)fcx * n + v) : 0.0f;
                }
                float eab = 0.0f, eac = 0.0f, ebc = 0.0f;
                if constexpr (DIM == 2 && !WIDE) {
                    eab = ld_glb(D, (size_t)fa * n + fb);
                    eac = ld_glb(D, (size_t)fa * n + fcx);
                    ebc = ld_glb(D, (size_t)fb * n + fcx);
                }
                // the previous step's keys, under this step's loads
                if (prev_app) ls_route_p<RV>(sk, sm, P);
                sm = 0;
#pragma unroll
                for (int q = 0; q < RV; ++q) {
                    const int v = wb + q * (64 * kLsWorkers);
                    uint64_t key = 0;
                    bool ok;
                    if constexpr (DIM == 1) ok = ls_key1<PACKED>(v, n, fa, fb, sdk, r, za[q], zb[q], key);
                    else ok = ls_key2<PACKED, WIDE>(v, n, fvs, sdk, r, za[q], zb[q], zc[q], eab, eac, ebc, key);
                    sk[q] = key;
                    if (ok && key >= Bs) sm |= 1u << q;
                }
            }
        }
#ifdef TDA_PROFILE
        if (tid == 0 && step > stats[0].prof[2][6]) {
            pf[0] = clock64() - t_col;
            pf[6] = step;
            for (int q = 0; q < 8; ++q) stats[0].prof[2][q] = pf[q];
            for (int q = 0; q < 8; ++q) stats[0].prof[3][q] = C.q[q];
        }
#endif
        if (tid == 0 && adds) atomicAdd((unsigned long long*)&st->n_adds[DIM], (unsigned long long)adds);
        sm = 0;
        if (done && my_rec >= 0 && my_seg) {  // the claimed record references this workgroup's chunks
            for (uint32_t e = tid; e < (uint32_t)kParLv * kParChunks; e += kLsT) (&LSS.cptr[0][0])[e] = kNoChunk;
            prealloc = false;
        }
        __syncthreads();
        if (LSS.err) {
            if (tid == 0) {
                acas((uint64_t*)&P.ctl->err, 0, ((uint64_t)item << 16) | (uint64_t)LSS.err);
                aadd(&P.ctl->abort, 1);
            }
            break;
        }
    }
}

#undef LSS

}  // namespace tda
