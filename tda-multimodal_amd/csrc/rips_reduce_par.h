// rips_reduce_par.h -- large-N H1 reduction with many residual columns in
// flight at once (k_reduce_par), one 512-thread workgroup per column.
//
// [upstream ripser.cpp compute_pairs] reduces the residual columns one after
// the other.  The persistence PAIRING does not depend on that order: any
// reduction R = D V with V upper triangular and pairwise distinct pivots gives
// the same pairs.  So every residual column is reduced concurrently, lock-free
// (the scheme of Morozov & Nigmetov, "Towards lockfree persistent homology",
// SPAA 2020), with a per-layer pivot -> owner map in HBM:
//   * pivot p apparent (k_apparent's bitmap): add the implicit apparent column;
//   * p free: publish R_j as an immutable record, then claim p (CAS);
//   * p owned by i < j: add R_i (its record) and go on;
//   * p owned by i > j: publish R_j, CAS the owner from i to j and requeue i,
//     which resumes from its own record and adds R_j.
// Every addition is of an EARLIER column, so V stays upper triangular; the
// owner of every pivot only ever moves to a smaller column, so the process
// terminates.  Pairs are read from the final owners by k_par_emit.
//
// One column's working coboundary (torus N=1024: two columns need 8,632 and
// 6,644 additions and grow to millions of raw entries) is a RADIX HEAP over
// the f32 diameter bits whose low levels live in LDS:
//   * the FRONT (levels 0..kf relative to `last`) is an LDS Z/2 toggle set:
//     key log (parity = bit 63) + 8-slot hashed index; the pivot is a min scan
//     of the log;
//   * levels kf+1..32 are append-only HBM buckets (chunks of 256 << k keys,
//     addressed from LDS, reused across the columns of one workgroup);
//     duplicates cancel when a bucket is pulled into the front;
//   * when the front empties, the lowest non-empty bucket is redistributed
//     relative to its minimum: the part that fits goes to the front, the rest
//     one level down.
// An apparent addition is then one dependent global round trip: the pivot's
// bitmap word and the two distance rows of its apparent facet are loaded
// together (for N <= 1024 the facet is encoded in the key's low bits, next to
// the packed vertex triple), everything else is LDS work.
//
// Cross-workgroup hand-offs follow MI355X_MICROARCH.md "inter-workgroup
// visibility": record payloads are written with sc1 (agent-scope relaxed)
// stores, every storing wave drains with s_waitcnt vmcnt(0) before the
// workgroup barrier that precedes the publishing CAS, and every load of a
// record header is an sc1 load, followed by one agent-scope acquire before
// the payload's plain loads (cdna_hip_programming.md Guideline 16, R1); map
// words and queue words are agent-scope atomics.
// Any capacity overflow, step limit or spin limit aborts the launch and the
// host re-runs the layer batch on k_reduce_big (the serial radix-heap kernel).
#pragma once
#include "rips_reduce_big.h"

namespace tda {

#ifndef TDA_PAR_T  // build-time A/B knob (tools/): threads per column workgroup
#define TDA_PAR_T 512
#endif
constexpr int kParT = TDA_PAR_T;
constexpr int kParW = kParT / 64;
// Sizes (build-time constants; tools/build_variants.py times other values).  Variants that
// were measured and dropped (the r02-r04 key log + hashed index front, deferred back-key
// appends, exact-minimum refills, sc1 bucket stores, read-then-CAS probing, one-pass block
// minima) are described in DESIGN.md §6.8 and no longer in the source.
#ifndef TDA_PAR_FILL  // refill / spill target (front keys)
#define TDA_PAR_FILL 768
#endif
#ifndef TDA_PAR_TAB  // toggle-table slots
#define TDA_PAR_TAB 4096
#endif
constexpr uint32_t kFrontLog = TDA_PAR_TAB;          // toggle-table slots
constexpr uint32_t kFrontLive = kFrontLog * 7 / 16;  // live front keys that trigger a spill (1792 at 4096)
constexpr uint32_t kFrontFill = TDA_PAR_FILL;        // refill / spill target
constexpr int kParChunks = 22;         // chunk k of an HBM bucket holds 256 << k keys
constexpr int kParRegs = 2048 / kParT;  // keys per thread per pass of refills and record adds (2048 per pass)
#ifndef TDA_PAR_REFILL  // refill passes kept in registers
#define TDA_PAR_REFILL 2
#endif
constexpr int kParRefill = TDA_PAR_REFILL;          // a refill keeps up to kParRefill passes (4096 keys) in registers
constexpr int kParRV = 1024 / kParT;   // coboundary vertices per thread per round (1024 per round)
// vertex of thread t in slot q of the coboundary round starting at v0.  (r05: the odd slots
// mirrored -- wave w taking 64-vertex blocks w and 2 W - 1 - w, to spread the waves' unequal key
// counts -- measured no faster: torus1024 34.3 ms either way)
__device__ __forceinline__ int par_vert(int v0, int q) { return v0 + q * kParT + (int)threadIdx.x; }
constexpr uint32_t kNoChunk = 0xFFFFFFFFu;
constexpr uint64_t kParEss = kEmpty64;        // colpiv: essential (zero column)
constexpr uint64_t kParSkip = kEmpty64 - 1;   // colpiv: cleared column (H0 death)
constexpr uint32_t kParSpin = 1u << 22;       // polls before a wait on another workgroup is declared hung

// k_reduce_par aborted: the host re-runs the call with k_reduce_big (ERR_PAR:
// the H1 launch aborted, both dimensions go serial; ERR_PAR2: the H2 launch
// aborted, H1 stays parallel and H2 goes serial).  ERR_CAP_MISS (per layer): a
// capped column ran empty below its cap; the layer's remaining columns are
// dropped and the host re-runs that layer alone without caps.
enum : int32_t { ERR_PAR = 128, ERR_PAR2 = 256, ERR_CAP_MISS = 512 };


struct ParCtl {  // zeroed by k_par_init
    unsigned long long next;     // next fresh item
    unsigned long long rq_head, rq_tail;
    unsigned long long bpool_used, rpool_used, rec_used;
    unsigned long long abort;
    unsigned long long err;      // first error code (diagnostics)
    unsigned long long total;    // items over all layers
    unsigned long long evictions;
    unsigned long long pad[6];
};

struct ParBufs {
    ParCtl* ctl;
    uint64_t* item_base;  // [L + 1] prefix of per-layer residual counts
    uint64_t* okey;       // [L][ostride] owner map keys: pivot index + 1 (0 = empty)
    uint64_t* oval;       // [L][ostride] owner map values: column << 32 | record + 1
    uint64_t ostride;
    uint64_t* colpiv;     // [L][rcap] final pivot (filt_key form) | kParEss | kParSkip
    uint64_t* rec;        // [rec_cap][4]: offset, length, pivot key, column
    uint64_t rec_cap;
    uint64_t* rpool;      // record payloads
    uint64_t rpool_cap;
    uint64_t* bpool;      // bucket chunks (per-workgroup, reused)
    uint64_t bpool_cap;   // in keys, multiple of 256
    uint64_t* rq;         // requeue slots (used once per launch, zero = not yet written): item << 32 | record + 1
    uint64_t rq_cap;
    uint64_t step_limit;
    float capf;           // column caps: keys above birth + capf * thresh are dropped (0 = off); see k_reduce_par
    uint64_t* dbg;        // -DTDA_PROFILE: [kParDbgCap][4] long-column timeline (layer << 40 | column, start, end, steps)
};
constexpr uint32_t kParDbgCap = 4096;
constexpr uint32_t kParP2Words = 12;       // -DTDA_PROF2 record: layer << 40 | column, wave, steps, 8 phase cycle sums, spare
constexpr uint64_t kParP2MinSteps = 1000;
constexpr uint64_t kParDbgMinSteps = 256;  // columns with at least this many steps are logged

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ uint64_t ald(const uint64_t* p) {  // sc1 load (agent scope)
    return __hip_atomic_load((uint64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ald(const unsigned long long* p) {
    return __hip_atomic_load((unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ast(uint64_t* p, uint64_t v) {  // sc1 store (write-through)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t acas(uint64_t* p, uint64_t cmp, uint64_t v) {  // returns old
    __hip_atomic_compare_exchange_strong(p, &cmp, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return cmp;
}
__device__ __forceinline__ uint64_t aadd(unsigned long long* p, unsigned long long v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Radix levels over the WHOLE 64-bit key (r03): level of key k relative to
// the reference `last` (a lower bound of every key in the column) is the
// position of the highest differing bit, 0 .. 64.  With levels on the high
// word only (r02), every key of one diameter (or, for the wide H2 keys, one
// edge code) shared level 0, which the front had to hold at once: torus1024's
// H2 columns exceeded it and fell back to the serial reducer.  Level 0 now
// means equal keys, which cancel in the front.
constexpr int kParLv = 65;
__device__ __forceinline__ uint32_t par_bucket(uint64_t key, uint64_t last) {
    const uint64_t x = key ^ last;
    return x ? 64u - (uint32_t)__builtin_clzll(x) : 0u;
}
// smallest key of bucket b >= 1 relative to `last`: bits above b - 1 as last, bit b - 1 set.
// (r05: two levels per bit -- 1 + 2 p + the key's bit p - 1 -- to halve the keys a refill moves,
// is wrong as a radix heap: a refill of a sub-level-0 bucket re-references the column, and its
// sibling bucket (same p, sub-level 1) then no longer holds keys of its own level; it failed the
// torus256 H1 parity test.  It would need the two siblings refilled together.)
__device__ __forceinline__ uint64_t par_bucket_floor(uint64_t last, uint32_t b) {
    return b >= 64u ? (1ull << 63) : (((last >> b) << b) | (1ull << (b - 1)));
}
__device__ __forceinline__ uint32_t chunk_of(uint32_t s) { return 31u - (uint32_t)__builtin_clz((s >> 8) + 1u); }
__host__ __device__ constexpr uint32_t chunk_start(uint32_t k) { return ((1u << k) - 1u) << 8; }

// triangle keys.  PACKED (N <= 1024): lo32 = ~(x << 22 | y << 12 | z << 2 | f)
// with x > y > z the vertices and f the apparent facet (the vertex t[f] it
// omits: the longest edge, first in (x, y, z) order on ties -- the facet
// apparent_facet<1> picks).  Colex order == order of the descending triples,
// so the key order is Ripser's (diam asc, index desc).  Otherwise lo32 = ~index.
template <bool PACKED>
__device__ __forceinline__ uint32_t tri_lo(int x, int y, int z, int f) {
    if (PACKED) return 0xFFFFFFFFu - (((uint32_t)x << 22) | ((uint32_t)y << 12) | ((uint32_t)z << 2) | (uint32_t)f);
    const int vs[3] = {x, y, z};
    return 0xFFFFFFFFu - (uint32_t)encode<2>(vs);
}

// ------------------------------------------------------------------ LDS
// The front: `log` is an open-addressing table of kFrontLog slots holding the
// live front keys; kTabEmpty / kTabTomb (a removed key) are above every key
// (keys < kDead), so the front minimum is the plain minimum of all slots.
// fcnt counts the slots ever filled since the last rebuild (live + tombstones).
constexpr uint64_t kTabEmpty = kEmpty64;
constexpr uint64_t kTabTomb = kEmpty64 - 1;
constexpr uint32_t kTabMax = kFrontLog * 3 / 4;  // filled slots allowed before a rebuild
constexpr uint32_t kTabPer = kFrontLog / kParT;  // slots per thread in scans
constexpr uint32_t kStageW = 64 * (kParRegs > 4 ? kParRegs : 4);           // per-wave staging of the keys one toggle pass hands to the table

struct ParLds {
    uint64_t log[kFrontLog];
    uint64_t stage[kParW][kStageW];
    uint32_t bcnt[kParLv];
    uint32_t cptr[kParLv][kParChunks];
    uint32_t hist[kParLv];
    uint64_t red[2][kParW];
    uint64_t redm[3];  // block minimum cells (triple-buffered LDS u64 atomic min)
    uint32_t wsum[2][kParW];
    uint32_t anyf[2][kParW];
    uint64_t bc[8];
    uint64_t last;  // radix reference: a lower bound of every key of the column
    uint32_t fcnt;  // front slots filled since the last rebuild
    uint32_t kf;    // front holds levels 0..kf
    int32_t err;
    uint32_t wide;  // wide H2 keys: the low 32 bits (index fingerprint) are not unique -> verify hits
    uint64_t ccol[3];  // the current column's layer, index in the layer, item
};
extern __shared__ ParLds par_smem[];
#define PS (par_smem[0])

// Level bookkeeping: one wave does what a serial loop over the 65 levels did
// (r03 profile, torus1024: those LDS loops cost ~7.5 K cycles per refill).
// Lowest non-empty HBM bucket at level >= from (-1 if none).  Block-uniform:
// every wave computes it from the same LDS counters (no barrier).
__device__ __forceinline__ int par_first_bucket(uint32_t from) {
    const uint32_t ln = threadIdx.x & 63;
    const uint64_t m = __ballot(ln >= from && PS.bcnt[ln] != 0);
    if (m) return (int)__builtin_ctzll(m);
    return (from <= 64u && PS.bcnt[64]) ? 64 : -1;
}

// Largest level q < lim (lim <= 64) whose cumulative count hist[0..q] is
// <= fill, or -1.  Counts are non-negative, so the levels that qualify are a
// prefix: a wave scan and one ballot.  Block-uniform.
__device__ __forceinline__ int par_keep_level(const uint32_t* hist, int lim, uint32_t fill) {
    const int ln = threadIdx.x & 63;
    uint32_t x = ln < lim ? hist[ln] : 0u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (ln >= o) x += y;
    }
    const uint64_t m = __ballot(ln < lim && x <= fill);
    return m ? 63 - (int)__builtin_clzll(m) : -1;
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a workgroup
// release/acquire, which waits for ALL of the wave's outstanding global
// memory operations (s_waitcnt vmcnt(0)) -- here the previous step's ~1000
// scattered bucket stores and any row loads in flight.  The step loop only
// exchanges LDS data across waves, so it waits for LDS (lgkmcnt) and leaves
// global traffic in flight.  HBM bucket data written by other waves is read
// only behind a full __syncthreads() (col_refill, col_save).
__device__ __forceinline__ void lds_sync() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Block minimum: the wave minimum as two u32 passes, then the cross-wave step as an LDS atomic
// min into a triple-buffered cell (r05, torus1024: 36.9 -> 34.7 ms against one u64 wave pass +
// a per-wave LDS array; tools/ubench_min: 1.41 K -> 1.12 K cycles per minimum)
__device__ __forceinline__ uint64_t wave_min_2p(uint64_t v) {  // u64 wave minimum: the hi words, then the lo words of the lanes that hold it
    const uint32_t h = wave_min_u32((uint32_t)(v >> 32));
    const uint32_t l = wave_min_u32((uint32_t)(v >> 32) == h ? (uint32_t)v : ~0u);
    return ((uint64_t)h << 32) | l;
}
struct ParRed {  // double-buffered block reductions: one barrier each
    uint32_t par = 0;
    uint32_t parm = 0;  // the minimum cell of this reduction (mod 3)
    // block-wide OR of p (HIP's OR-barrier builtin lowers to three barriers)
    __device__ __forceinline__ bool any(bool p) {
        const uint64_t m = __ballot(p);
        const uint32_t b = par++ & 1;
        if ((threadIdx.x & 63) == 0) PS.anyf[b][threadIdx.x >> 6] = m != 0;
        lds_sync();
        uint32_t r = 0;
#pragma unroll
        for (int w = 0; w < kParW; ++w) r |= PS.anyf[b][w];
        return r != 0;
    }
    __device__ __forceinline__ uint64_t min(uint64_t v) {
        v = wave_min_2p(v);
        // cell parm was reset two reductions ago; the next one's cell was last read before the
        // previous barrier, so it is reset here for the reduction after this one
        const uint32_t c = parm, cn = c == 2 ? 0 : c + 1;
        parm = cn;
        if ((threadIdx.x & 63) == 0)
            __hip_atomic_fetch_min((TDA_LDS unsigned long long*)&PS.redm[c], (unsigned long long)v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        if (threadIdx.x == 0) PS.redm[cn] = kEmpty64;
        lds_sync();
        return PS.redm[c];
    }
    __device__ __forceinline__ uint64_t sum(uint64_t v) {
        v = wave_sum_u64(v);
        const uint32_t b = par++ & 1;
        if ((threadIdx.x & 63) == 0) PS.red[b][threadIdx.x >> 6] = v;
        lds_sync();
        uint64_t m = 0;
#pragma unroll
        for (int w = 0; w < kParW; ++w) m += PS.red[b][w];
        return m;
    }
    // exclusive block prefix of per-thread counts c; *tot = block total
    __device__ __forceinline__ uint32_t prefix(uint32_t c, uint32_t* tot) {
        // wave-inclusive scan with shuffles (c small)
        const int ln = threadIdx.x & 63, w = threadIdx.x >> 6;
        uint32_t x = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (ln >= o) x += y;
        }
        const uint32_t b = par++ & 1;
        if (ln == 63) PS.wsum[b][w] = x;
        lds_sync();
        uint32_t before = 0, all = 0;
#pragma unroll
        for (int q = 0; q < kParW; ++q) {
            const uint32_t s = PS.wsum[b][q];
            before += q < w ? s : 0;
            all += s;
        }
        *tot = all;
        return before + x - c;
    }
};

// ------------------------------------------------------------------ front
// One open-addressing Z/2 toggle table.
// A toggle flips the presence of its key with ONE successful CAS on the key's
// probe chain: EMPTY -> key (insert) or key -> TOMB (remove); a failed CAS
// re-reads the same slot.  Slots never return to EMPTY between rebuilds, so a
// present key is always reached before any EMPTY slot of its chain, and
// concurrent toggles of one key (raw multisets from refills and records) net
// out to the right parity in every interleaving.  Against the r04 log + index:
// no per-wave log allocation (an LDS atomic whose result the wave waited on),
// no index entry to publish, no fingerprint to verify.
__device__ __forceinline__ uint32_t tab_hash(uint64_t k) { return (uint32_t)mix64(k) & (kFrontLog - 1); }

__device__ __forceinline__ void front_clear() {  // no barrier
    for (uint32_t e = threadIdx.x; e < kFrontLog; e += kParT) PS.log[e] = kTabEmpty;
    if (threadIdx.x == 0) PS.fcnt = 0;
}
__device__ __forceinline__ void front_reset() {
    front_clear();
    __syncthreads();
}

// toggle one key (the lane's own); returns 1 if it filled an EMPTY slot
// Probing with the inserting CAS itself: one LDS round trip per empty slot (r05: torus1024 32.5 ->
// 31.8 ms, grid144 5.38 -> 5.31 ms against a read, then a CAS).  Also measured and dropped: the
// second wave of each SIMD at a higher issue priority, s_setprio 1 / 3: torus1024 32.1 -> 33.5-33.8 ms.
__device__ __forceinline__ uint32_t tab_toggle(uint64_t key) {
    uint32_t h = tab_hash(key);
    for (uint32_t it = 0; it < 4 * kFrontLog; ++it) {
        // the CAS that inserts into an EMPTY slot also reads the slot: a present key
        // comes back as itself (remove it), a tombstone or another key moves the probe on
        const uint64_t v = atomicCAS((unsigned long long*)&PS.log[h], (unsigned long long)kTabEmpty, (unsigned long long)key);
        if (v == kTabEmpty) return 1;
        if (v == key) {
            if (atomicCAS((unsigned long long*)&PS.log[h], (unsigned long long)key, (unsigned long long)kTabTomb) == key) return 0;
            continue;  // another toggle of this key won: look at the slot again
        }
        h = (h + 1) & (kFrontLog - 1);
    }
    PS.err = 13;  // table full (front_room keeps it below kTabMax)
    return 0;
}

// Toggle up to R keys per thread (bit r of vmask) with NO workgroup barrier:
// the wave's keys are packed into its lanes through a wave-private LDS stage
// (no atomics), then each lane toggles ceil(n / 64) of them.  Callers put a
// barrier between this and the next read of the front; the caller made room
// (fcnt + R * kParT <= kTabMax).
template <int R>
__device__ __forceinline__ void front_toggle(const uint64_t (&k)[R], uint32_t vmask) {
    static_assert(R * 64 <= (int)kStageW, "stage");
    const int ln = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t m[R];
    uint32_t wtot = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        m[r] = __ballot((vmask >> r) & 1u);
        wtot += (uint32_t)__popcll(m[r]);
    }
    if (!wtot) return;
    uint32_t ins = 0;
    // (r06: lanes with at most one key toggling it in place, skipping the stage, measured no faster:
    // torus1024 33.45 vs 33.43 ms)
    if (wtot <= 64 && R == 1) {  // one key per lane already
        if (vmask & 1u) ins = tab_toggle(k[0]);
    } else {
        uint32_t off = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if ((vmask >> r) & 1u) PS.stage[w][off + lanes_below(m[r])] = k[r];
            off += (uint32_t)__popcll(m[r]);
        }
        // a wave's LDS operations complete in order: the stage is visible to every lane
        for (uint32_t pos = (uint32_t)ln; pos < wtot; pos += 64) ins += tab_toggle(PS.stage[w][pos]);
    }
    const uint64_t mi = __ballot(ins != 0);
    uint32_t n = ins;
    if (__popcll(mi) > 0) {
        n = (uint32_t)wave_sum_u64(ins);
        if (ln == 0) atomicAdd(&PS.fcnt, n);  // no return: nobody waits on it
    }
}

// min live front key (block-uniform; kEmpty64 if none): every slot, 16-B
// reads.  (r05, measured slower: group minima kept by the toggles -- ds_min on
// insert, a dirty bit on removal, only dirty groups rescanned: the front
// minimum 1.9 K -> 4.2 K cycles a step, torus1024 41.9 -> 49.2 ms; a minimum
// cache listing the slots of every live key below a bound taken from the scan
// (the smallest second-smallest key over the threads' slot sets, ~28 keys):
// 1.9 K -> 3.0 K cycles, 37.4 -> 42.2 ms -- an addition cancels the keys just
// above its pivot, so the cache empties within ~1.5 steps (a replay of the
// longest column's key trace: 33 % of the minima served; 80 % would need the
// 128 smallest keys, which no longer avoids a block-wide reduction).)
__device__ __forceinline__ uint64_t front_scan() {  // this thread's share of the front minimum
    uint64_t b = kEmpty64;
#pragma unroll
    for (uint32_t q = 0; q < kTabPer; q += 2) {  // slots 2 t, 2 t + 1 of each 2 kParT block
        const u64x2 v = *(const TDA_LDS u64x2*)&PS.log[q * kParT + 2 * threadIdx.x];
        b = v.x < b ? v.x : b;
        b = v.y < b ? v.y : b;
    }
    return b < kDead ? b : kEmpty64;
}
__device__ __forceinline__ uint64_t front_min(ParRed& rd) { return rd.min(front_scan()); }

// Rebuild the table with the live keys of level <= keep (relative to
// PS.last): read every slot, clear, re-insert.  Returns the live count kept
// (block-uniform).
__device__ __forceinline__ uint32_t front_compact(ParRed& rd, uint32_t keep) {
    __syncthreads();
    const uint64_t last = PS.last;
    uint64_t mine[kTabPer];
    uint32_t nl = 0;
#pragma unroll
    for (uint32_t q = 0; q < kTabPer; ++q) {
        const uint64_t x = PS.log[q * kParT + threadIdx.x];
        const bool lv = x < kDead && par_bucket(x, last) <= keep;
        mine[q] = lv ? x : kTabEmpty;
        nl += lv;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kTabPer; ++q) PS.log[q * kParT + threadIdx.x] = kTabEmpty;
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kTabPer; ++q) {
        if (mine[q] == kTabEmpty) continue;
        uint32_t h = tab_hash(mine[q]);  // distinct keys: the first EMPTY slot of the chain
        for (uint32_t it = 0; it < kFrontLog; ++it, h = (h + 1) & (kFrontLog - 1))
            if (PS.log[h] == kTabEmpty &&
                atomicCAS((unsigned long long*)&PS.log[h], (unsigned long long)kTabEmpty, (unsigned long long)mine[q]) == kTabEmpty)
                break;
    }
    const uint32_t w = (uint32_t)rd.sum(nl);  // barrier: the inserts are done
    if (threadIdx.x == 0) PS.fcnt = w;
    __syncthreads();
    return w;
}

// ------------------------------------------------------------------ HBM buckets
// (r05: the slot's chunk pointer read from a per-bucket "current chunk" cache
// beside the slot atomic -- one LDS round trip instead of two -- measured no
// faster: torus1024 49.2 vs 49.4 ms; dropped)
// Append key k[r] to bucket bb[r] (bit r of vmask); chunks that start in this
// pass and were never allocated by this workgroup are taken from the pool.
// Append key k[r] to HBM bucket bb[r] (bit r of vmask), with NO workgroup
// barrier: slots come from one LDS atomic per key; every bucket's chunks 0..3
// are allocated when the workgroup starts, and the key that opens chunk c
// allocates chunk c + 2, so a pass of up to 3072 keys per bucket never needs a
// chunk that is not there yet (chunks c and c + 1 hold >= 3072 keys from c = 2
// on).  Callers put a barrier between passes that may open new chunks.
// (r05: slot allocation and the refill histogram aggregated per (wave, level) by
// ballots -- one LDS atomic per distinct level instead of per key -- measured
// slower: torus1024 45.2 -> 50.1 ms, torus1024x32 108 -> 114 ms; the native
// same-address LDS atomics stay)
template <int R>
__device__ __forceinline__ void bucket_append(const uint64_t (&k)[R], const uint32_t (&bb)[R], uint32_t vmask, const ParBufs& P) {
    uint32_t slot[R];
#pragma unroll
    for (int r = 0; r < R; ++r) slot[r] = ((vmask >> r) & 1u) ? atomicAdd(&PS.bcnt[bb[r]], 1u) : 0u;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!((vmask >> r) & 1u)) continue;
        const uint32_t kc = chunk_of(slot[r]);
        if (slot[r] == chunk_start(kc) && kc + 2 < (uint32_t)kParChunks && PS.cptr[bb[r]][kc + 2] == kNoChunk) {
            const uint64_t sz = 256ull << (kc + 2);
            const uint64_t o = aadd(&P.ctl->bpool_used, sz);
            if (o + sz <= P.bpool_cap) PS.cptr[bb[r]][kc + 2] = (uint32_t)(o >> 8);
            else PS.err = 22;
        }
        const uint32_t cp = kc < (uint32_t)kParChunks ? PS.cptr[bb[r]][kc] : kNoChunk;
        if (cp == kNoChunk) {
            PS.err = 21;
            continue;
        }
        // (r05: sc1 write-through stores that drop the line from this XCD's L2, measured within noise)
        st_glb(P.bpool, (uint64_t)cp * 256 + (slot[r] - chunk_start(kc)), k[r]);
    }
}

__device__ __forceinline__ uint64_t bucket_at(const ParBufs& P, uint32_t b, uint32_t e) {
    const uint32_t kc = chunk_of(e);
    return ld_glb(P.bpool, (uint64_t)PS.cptr[b][kc] * 256 + (e - chunk_start(kc)));
}

// ------------------------------------------------------------------ column
struct ParCol {
    ParRed rd;
    uint64_t steps = 0, adds = 0;
    uint32_t capbits = 0xFFFFFFFFu;  // the column's cap (f32 bits of the largest kept diameter); record keys above it are dropped
#ifdef TDA_PROF2
    // per-wave phase cycles of the current column (s_memtime deltas):
    // room + step barrier, front min, pivot + row loads, keys, bucket appends, front toggles, refills, owner path / records
    uint32_t tp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
#ifdef TDA_PROFILE
    uint64_t ncompact = 0, nspill = 0;
    uint64_t q[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // keys, front toggle, bucket append, capacity, R adds, R entries, refill keys, load wait
    uint64_t q2[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // record: room, add, front keys, back keys; refill: passes 1-2, pass 3
    uint64_t q3[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // refill: search, pass 1 (loads + min), pass 2 (histogram), level choice, toggles, appends, compactions, keys kept in front
#endif
};
#ifdef TDA_PROF2
// gfx950 has no HW_REG_SHADER_CYCLES: s_memtime (an SMEM read of the shader
// clock; its use waits lgkmcnt, so a phase is charged with the LDS work it
// issued)
__device__ __forceinline__ uint32_t p2_now() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const uint32_t c = (uint32_t)__builtin_amdgcn_s_memtime();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    return c;
}
#define P2_T(v) const uint32_t v = p2_now()
#define P2_ACC(i, v) C.tp[i] += p2_now() - (v)
#define P2_DEP(x) asm volatile("" : : "v"(x))
#else
#define P2_T(v)
#define P2_ACC(i, v)
#define P2_DEP(x)
#endif
#ifdef TDA_PROFILE
#define PAR_T0(v) const uint64_t v = clock64()
#define PAR_ACC(i, v) C.q[i] += clock64() - (v)
#else
#define PAR_T0(v)
#define PAR_ACC(i, v)
#endif

// Barrier, then room in the front for `need` more log entries: compact, and
// spill the highest front levels to HBM if too many keys are live.
constexpr uint32_t kFrontRoom = kTabMax;
__device__ __forceinline__ void front_room_slow(ParCol& C, const ParBufs& P, uint32_t need);
__device__ __forceinline__ void front_room(ParCol& C, const ParBufs& P, uint32_t need) {
    lds_sync();
    if (PS.fcnt + need <= kFrontRoom) return;
    front_room_slow(C, P, need);
}
// compact the front, and spill its highest levels to HBM if too many keys are live
__device__ __forceinline__ void front_room_slow(ParCol& C, const ParBufs& P, uint32_t need) {
    PAR_T0(tc0);
    uint32_t w = front_compact(C.rd, kParLv);
#ifdef TDA_PROFILE
    ++C.ncompact;
#endif
    if (w > kFrontLive || w + need > kFrontRoom) {
#ifdef TDA_PROFILE
        ++C.nspill;
#endif
        // histogram of the live front by level, keep the lowest levels up to kFrontFill
        for (uint32_t q = threadIdx.x; q < kParLv; q += kParT) PS.hist[q] = 0;
        __syncthreads();
        const uint64_t last = PS.last;
        for (uint32_t e = threadIdx.x; e < kFrontLog; e += kParT)
            if (PS.log[e] < kDead) atomicAdd(&PS.hist[par_bucket(PS.log[e], last)], 1u);
        __syncthreads();
        int keep = par_keep_level(PS.hist, (int)min(PS.kf + 1u, 64u), kFrontFill);
        if (keep < 0) {  // the exact-diameter level alone is too large for the front
            if (PS.hist[0] + need <= kFrontRoom) keep = 0;
            else if (threadIdx.x == 0) PS.err = 31;
        }
        __syncthreads();
        if (PS.err) return;
        // move the levels above `keep` out to their HBM buckets, then drop them from the front
        const uint32_t ns = kFrontLog;  // every slot (tombstones and EMPTY are skipped)
        for (uint32_t e0 = 0; e0 < ns; e0 += kParT) {
            const uint32_t e = e0 + threadIdx.x;
            uint64_t x[1] = {e < ns ? PS.log[e] : kEmpty64};
            uint32_t b[1] = {x[0] < kDead ? par_bucket(x[0], last) : 0};
            bucket_append<1>(x, b, (x[0] < kDead && b[0] > (uint32_t)keep) ? 1u : 0u, P);
            __syncthreads();  // chunk pointers opened by this pass
        }
        if (threadIdx.x == 0) PS.kf = (uint32_t)keep;
        front_compact(C.rd, (uint32_t)keep);
    }
    PAR_ACC(3, tc0);
}

// Insert keys (bit r of vmask; all >= the current pivot) into the working
// column: front levels toggle in LDS, the rest append to HBM buckets.  No
// barrier: the caller made room (front_room) for every key of the pass.
// (r06: the kernel's arguments copied to LDS and read from there outside the step loop -- SGPR
// spills 159 -> 119 but 13 VGPRs spilled to scratch: torus1024 31.9 -> 34.3 ms, measured and dropped.)
// (r06: a coboundary round's two LDS dependency chains -- back keys: slot atomic -> chunk pointer ->
// store; front keys: stage write -> stage read -> CAS -- issued side by side instead of one after the
// other, measured no faster: torus1024 33.8 vs 33.7 ms)
template <int R>
__device__ __forceinline__ void col_add(ParCol& C, const ParBufs& P, const uint64_t (&k)[R], uint32_t vmask) {
    const uint64_t last = PS.last;
    const uint32_t kf = PS.kf;
    uint32_t fm = 0, bm = 0, bb[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        bb[r] = par_bucket(k[r], last);
        if ((vmask >> r) & 1u) {
            if (bb[r] <= kf) fm |= 1u << r;
            else bm |= 1u << r;
        }
    }
#ifdef TDA_PROFILE
    C.q[7] += (wave_sum_u64((uint64_t)__builtin_popcount(fm)) << 32) | wave_sum_u64((uint64_t)__builtin_popcount(bm));  // wave 0's front / back keys
#endif
    // back keys first: their stores are issued as early as possible, so they are
    // acknowledged before the next step waits for its row loads (gfx950 has no
    // separate store counter: a load's s_waitcnt vmcnt also waits for every
    // store issued before it -- with the r04 deferred appends, the previous step's
    // ~600 bucket stores went out right after the row loads and sat in their wait)
    PAR_T0(tb0);
    P2_T(pb0);
    // (r05: back keys staged per wave in LDS and appended in bulk, 256 or 128 per wave -- one
    // slot-atomic / chunk / store chain per flush instead of per step -- measured slower:
    // torus1024 32.2-32.6 -> 33.2 ms)
    bucket_append<R>(k, bb, bm, P);
    P2_ACC(4, pb0);
    PAR_ACC(2, tb0);
    PAR_T0(tf0);
    P2_T(pf0);
    front_toggle<R>(k, fm);
    P2_ACC(5, pf0);
    PAR_ACC(1, tf0);
}

// kParRegs keys per thread of bucket b at [e0, c), loads all in flight
__device__ __forceinline__ uint32_t bucket_batch(const ParBufs& P, uint32_t b, uint32_t e0, uint32_t c, uint64_t (&x)[kParRegs]) {
    uint32_t vm = 0;
#pragma unroll
    for (int r = 0; r < kParRegs; ++r) {
        const uint32_t e = e0 + threadIdx.x + r * kParT;
        x[r] = e < c ? bucket_at(P, b, e) : kEmpty64;
        if (e < c) vm |= 1u << r;
    }
    return vm;
}

// Front empty: redistribute the lowest non-empty bucket relative to its
// lower bound.  Returns false when the working column is zero.  A bucket of up
// to kParRefill * kParT * kParRegs keys is read once into registers; larger
// ones stream twice (level histogram, distribution), kParRegs loads in flight
// per thread.  (r05: relative to the bucket's exact minimum, one more pass and
// a block reduction: torus1024 34.4 vs 32.6 ms.)
__device__ __forceinline__ bool col_refill(ParCol& C, const ParBufs& P) {
    __syncthreads();
#ifdef TDA_PROFILE
    uint64_t tq = clock64();
#define PAR_Q3(i) do { __syncthreads(); const uint64_t tn = clock64(); C.q3[i] += tn - tq; tq = tn; } while (0)
#else
#define PAR_Q3(i)
#endif
    const int b = par_first_bucket(PS.kf + 1);
    PAR_Q3(0);
    if (b < 0) return false;
    const uint32_t c = PS.bcnt[b];
    constexpr uint32_t kPass = kParT * kParRegs;
    const bool inreg = c <= kParRefill * kPass;
#ifdef TDA_PROFILE
    C.q[6] += c;
#endif
    front_clear();
    for (uint32_t q = threadIdx.x; q < kParLv; q += kParT) PS.hist[q] = 0;
    uint64_t x[kParRefill][kParRegs];
    uint32_t vm[kParRefill] = {};
    // no minimum pass: the new reference is the smallest key with bucket b's common high bits
    // (bits above b - 1 as `last`, bit b - 1 set), a lower bound of every key in the bucket, so
    // the bucket's keys fall in levels < b and the higher buckets keep theirs.  (The exact
    // minimum puts at least one key in the front; with the bound a refill may place none and
    // the next one refines the lower buckets.)
    const uint64_t nl = par_bucket_floor(PS.last, (uint32_t)b);
    if (inreg) {
#pragma unroll
        for (int h = 0; h < kParRefill; ++h) vm[h] = bucket_batch(P, (uint32_t)b, h * kPass, c, x[h]);
    }
    __syncthreads();  // the resets above are done
    PAR_Q3(1);
    // pass 2: histogram of the new levels (all < b); the front keeps the lowest
    // levels that hold at most kFrontFill keys.  (A binary search on the level
    // with block counts instead of the atomics measured slower: 7.1 vs 4.3 M
    // cycles over torus1024's refills.)
#define PAR_HIST_ADD(key, valid) do { if (valid) atomicAdd(&PS.hist[par_bucket((key), nl)], 1u); } while (0)
    if (inreg) {
#pragma unroll
        for (int h = 0; h < kParRefill; ++h)
#pragma unroll
            for (int r = 0; r < kParRegs; ++r) PAR_HIST_ADD(x[h][r], (vm[h] >> r) & 1u);
    } else {
        for (uint32_t e0 = 0; e0 < c; e0 += kPass) {
            uint64_t y[kParRegs];
            const uint32_t ym = bucket_batch(P, (uint32_t)b, e0, c, y);
#pragma unroll
            for (int r = 0; r < kParRegs; ++r) PAR_HIST_ADD(y[r], (ym >> r) & 1u);
        }
    }
#undef PAR_HIST_ADD
    __syncthreads();
    int keep = par_keep_level(PS.hist, b, kFrontFill);
    const uint32_t cnt0 = PS.hist[0];  // keys equal to nl (level 0)
    PAR_Q3(2);
    if (keep < 0) {
        if (cnt0 <= kFrontLive) keep = 0;
        else {
            if (threadIdx.x == 0) PS.err = 32;
            __syncthreads();
            return false;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        PS.bcnt[b] = 0;  // consumed (its chunks stay with this workgroup)
        PS.last = nl;
        PS.kf = (uint32_t)keep;
    }
    __syncthreads();
    PAR_Q3(3);
#ifdef TDA_PROFILE
    const uint64_t t3 = clock64();
#endif
    // pass 3: distribute (front: toggles; below b: appends to empty lower buckets)
    auto distribute = [&](const uint64_t (&y)[kParRegs], uint32_t ym) {
        // the front takes at most kFrontLive keys in all: compaction keeps room
        __syncthreads();  // chunk pointers opened by the previous pass
        if (PS.fcnt + kParRegs * kParT > kFrontRoom) front_compact(C.rd, kParLv);
        PAR_Q3(6);
        uint32_t fm = 0, bm = 0, bb[kParRegs];
#pragma unroll
        for (int r = 0; r < kParRegs; ++r) {
            bb[r] = par_bucket(y[r], nl);
            if ((ym >> r) & 1u) {
                if (bb[r] <= (uint32_t)keep) fm |= 1u << r;
                else bm |= 1u << r;
            }
        }
        front_toggle<kParRegs>(y, fm);
        PAR_Q3(4);
#ifdef TDA_PROFILE
        C.q3[7] += C.rd.sum((uint32_t)__builtin_popcount(fm));
        tq = clock64();
#endif
        bucket_append<kParRegs>(y, bb, bm, P);
        PAR_Q3(5);
    };
    if (inreg) {
#pragma unroll
        for (int h = 0; h < kParRefill; ++h) {
            if (h * kPass >= c) break;
            distribute(x[h], vm[h]);
        }
    } else {
        for (uint32_t e0 = 0; e0 < c; e0 += kPass) {
            uint64_t y[kParRegs];
            const uint32_t ym = bucket_batch(P, (uint32_t)b, e0, c, y);
            distribute(y, ym);
        }
    }
    __syncthreads();
#ifdef TDA_PROFILE
    C.q2[5] += clock64() - t3;
#endif
    return PS.err == 0;
#undef PAR_Q3
}

// toggle the coboundary of edge (a > b), diameter sd, into the column (no
// barrier; the caller made room for n front keys: front_room(C, P, par_need(n))).
// Round 0's rows may already be in registers (da0 / db0, prefetched with the pivot).
template <bool PACKED>
__device__ __forceinline__ void col_cob(ParCol& C, const ParBufs& P, const float* __restrict__ D, int n, float r, int a, int b, float sd,
                        const float (&da0)[kParRV], const float (&db0)[kParRV]) {
    for (int v0 = 0; v0 < n; v0 += kParT * kParRV) {
        float da[kParRV], db[kParRV];
#pragma unroll
        for (int q = 0; q < kParRV; ++q) {
            const int v = par_vert(v0, q);
            if (v0 == 0) {
                da[q] = da0[q];
                db[q] = db0[q];
            } else {
                da[q] = v < n ? ld_glb(D, (size_t)a * n + v) : 0.0f;
                db[q] = v < n ? ld_glb(D, (size_t)b * n + v) : 0.0f;
            }
        }
        PAR_T0(tk0);
        P2_T(pk0);
        uint64_t key[kParRV];
        uint32_t vm = 0;
#pragma unroll
        for (int q = 0; q < kParRV; ++q) {
            const int v = par_vert(v0, q);
            key[q] = 0;
            if (v >= n || v == a || v == b) continue;
            const float cd = fmaxf(sd, fmaxf(da[q], db[q]));
            if (!(cd <= r)) continue;
            // vertices descending; the edge omitting vertex u has length excl(u):
            // excl(v) = sd, excl(a) = |bv| = db, excl(b) = |av| = da
            int x, y, z;
            float ex, ey, ez;
            if (v > a) {
                x = v, y = a, z = b;
                ex = sd, ey = db[q], ez = da[q];
            } else if (v > b) {
                x = a, y = v, z = b;
                ex = db[q], ey = sd, ez = da[q];
            } else {
                x = a, y = b, z = v;
                ex = db[q], ey = da[q], ez = sd;
            }
            int f = 0;
            float fd = ex;
            if (ey > fd) f = 1, fd = ey;
            if (ez > fd) f = 2;
            key[q] = ((uint64_t)__float_as_uint(cd + 0.0f) << 32) | tri_lo<PACKED>(x, y, z, f);
            vm |= 1u << q;
        }
        P2_DEP(vm);
        P2_ACC(3, pk0);
        PAR_ACC(0, tk0);
        col_add<kParRV>(C, P, key, vm);  // no barrier: the caller made room for all n keys
    }
}

// tetrahedron keys (H2 columns' cofacets).  PACKED (N <= 400, C(N,4) < 2^30):
// lo32 = ~(index << 2 | f), f the position (in descending vertex order) of the
// vertex its apparent facet omits -- the facet apparent_facet<2> picks: max
// diameter, first on ties.  Otherwise (N <= 568) lo32 = ~index.
constexpr int kPar2PackedMaxN = 400;
template <bool PACKED>
__device__ __forceinline__ uint32_t tet_lo(uint64_t idx, int f) {
    if (PACKED) return 0xFFFFFFFFu - (((uint32_t)idx << 2) | (uint32_t)f);
    return 0xFFFFFFFFu - (uint32_t)idx;
}

// toggle the coboundary of triangle (a > b > c), diameter sd, into the column
// (no barrier; the caller made room).  Round 0's rows may be prefetched (r0).
// WIDE (N > 568): D holds the layer's edge CODES (bit patterns in float
// slots), sd is the triangle's code, keys are code << 42 | (2^42 - 1 - index).
template <bool PACKED, bool WIDE = false>
__device__ __forceinline__ void col_cob2(ParCol& C, const ParBufs& P, const float* __restrict__ D, int n, float r, int a, int b, int c,
                                         float sd, const float (&r0)[3][kParRV]) {
    // the triangle's own edges (facet diameters of its cofacets)
    const float eab = WIDE ? 0.0f : ld_glb(D, (size_t)a * n + b), eac = WIDE ? 0.0f : ld_glb(D, (size_t)a * n + c),
                ebc = WIDE ? 0.0f : ld_glb(D, (size_t)b * n + c);
    const int vs[3] = {a, b, c};
    for (int v0 = 0; v0 < n; v0 += kParT * kParRV) {
        float da[kParRV], db[kParRV], dc[kParRV];
#pragma unroll
        for (int q = 0; q < kParRV; ++q) {
            const int v = par_vert(v0, q);
            if (v0 == 0) {
                da[q] = r0[0][q];
                db[q] = r0[1][q];
                dc[q] = r0[2][q];
            } else {
                da[q] = v < n ? ld_glb(D, (size_t)a * n + v) : 0.0f;
                db[q] = v < n ? ld_glb(D, (size_t)b * n + v) : 0.0f;
                dc[q] = v < n ? ld_glb(D, (size_t)c * n + v) : 0.0f;
            }
        }
        PAR_T0(tk0);
        uint64_t key[kParRV];
        uint32_t vm = 0;
#pragma unroll
        for (int q = 0; q < kParRV; ++q) {
            const int v = par_vert(v0, q);
            key[q] = 0;
            if (v >= n || v == a || v == b || v == c) continue;
            if constexpr (WIDE) {
                const uint32_t cc = max(max(__float_as_uint(sd), __float_as_uint(da[q])), max(__float_as_uint(db[q]), __float_as_uint(dc[q])));
                if (cc >= kCodeInf) continue;
                key[q] = ((uint64_t)cc << kWideIdxBits) | (kWideIdxMask - cofacet_index<2>(vs, v));
                vm |= 1u << q;
                continue;
            }
            const float cd = fmaxf(fmaxf(sd, da[q]), fmaxf(db[q], dc[q]));
            if (!(cd <= r)) continue;
            // facet diameters: omitting v -> sd; a -> (b,c,v); b -> (a,c,v); c -> (a,b,v)
            const float oa = fmaxf(ebc, fmaxf(db[q], dc[q]));
            const float ob = fmaxf(eac, fmaxf(da[q], dc[q]));
            const float oc = fmaxf(eab, fmaxf(da[q], db[q]));
            // in descending vertex order of the cofacet
            const int pv = v > a ? 0 : v > b ? 1 : v > c ? 2 : 3;  // position of v
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
            key[q] = ((uint64_t)__float_as_uint(cd + 0.0f) << 32) | tet_lo<PACKED>(cofacet_index<2>(vs, v), f);
            vm |= 1u << q;
        }
        PAR_ACC(0, tk0);
        col_add<kParRV>(C, P, key, vm);
    }
}

__host__ __device__ __forceinline__ uint32_t par_need(int n) {  // log entries one coboundary can add
    return (uint32_t)((n + kParT * kParRV - 1) / (kParT * kParRV)) * kParT * kParRV;
}

// Publish the working column as an immutable record (sc1 stores, drained).
// Returns the record id (block-uniform), or -1 on overflow.
// Small columns are copied (front + every HBM bucket).  A column with more
// than kParSegMin keys is published ZERO-COPY: the record holds its live
// front keys and a table of (bpool offset, count) segments that point at the
// workgroup's own bucket chunks (*seg = true).  The caller then gives those
// chunks up once the record is referenced (a successful claim) and takes
// fresh ones for its next column.  (r03 profile, torus1024: the longest
// column's final save copied 5.3 M raw bucket keys, ~10 ms of one workgroup's
// bandwidth, on the critical path.)
constexpr uint64_t kParSegMin = 1ull << 16;
constexpr uint64_t kParSegBit = 1ull << 63;  // record header word 0: segmented payload
__device__ __forceinline__ int64_t col_save(ParCol& C, const ParBufs& P, uint64_t pkey, uint64_t item, bool* seg) {
    drain_vm();       // this wave's bucket stores have reached L2
    __syncthreads();  // full barrier: every wave's bucket stores are visible to the copy below
#ifdef TDA_PROFILE
    const uint64_t tsv = clock64();
#endif
    const uint32_t c = kFrontLog;  // every slot (only live keys are < kDead)
    uint32_t lv = 0;
    for (uint32_t e = threadIdx.x; e < c; e += kParT) lv += PS.log[e] < kDead;
    const uint64_t nfront = C.rd.sum(lv);
    uint64_t nback = 0;
    for (int q = 0; q < kParLv; ++q) nback += PS.bcnt[q];
    const uint64_t total = nfront + nback;
    const bool segd = total > kParSegMin;
    constexpr uint32_t kSegs = (uint32_t)kParLv * kParChunks;
    const uint64_t words = segd ? nfront + 2ull * kSegs : total;
    if (threadIdx.x == 0) {
        const uint64_t o = aadd(&P.ctl->rpool_used, (words + 15) & ~15ull);  // 128-B aligned records
        const uint64_t id = aadd(&P.ctl->rec_used, 1ull);
        PS.bc[0] = (o + words <= P.rpool_cap && id < P.rec_cap) ? o : kEmpty64;
        PS.bc[1] = id;
    }
    __syncthreads();
    const uint64_t off = PS.bc[0], id = PS.bc[1];
    if (off == kEmpty64) {
        if (threadIdx.x == 0) PS.err = 41;
        __syncthreads();
        return -1;
    }
    uint64_t* out = P.rpool + off;
    uint32_t w = 0;
    for (uint32_t e0 = 0; e0 < c; e0 += kParT) {
        const uint32_t e = e0 + threadIdx.x;
        const uint64_t x = e < c ? PS.log[e] : kEmpty64;
        const bool live = x < kDead;
        uint32_t tot;
        const uint32_t o = C.rd.prefix(live ? 1u : 0u, &tot);
        if (live) ast(out + w + o, x);
        w += tot;
    }
    uint64_t hdr1 = total;
    if (segd) {
        // compacted segment table: one (offset, count) per non-empty (bucket, chunk)
        uint32_t ns = 0;
        for (uint32_t e0 = 0; e0 < kSegs; e0 += kParT) {
            const uint32_t e = e0 + threadIdx.x;
            const uint32_t q = e / kParChunks, kc = e % kParChunks;
            uint32_t cnt = 0;
            if (e < kSegs) {
                const uint32_t cq = PS.bcnt[q], lo = chunk_start(kc);
                if (lo < cq) cnt = min(cq, chunk_start(kc + 1)) - lo;
            }
            uint32_t tot;
            const uint32_t o = C.rd.prefix(cnt ? 1u : 0u, &tot);
            if (cnt) {
                ast(out + nfront + 2 * (ns + o), (uint64_t)PS.cptr[q][kc] * 256);
                ast(out + nfront + 2 * (ns + o) + 1, (uint64_t)cnt);
            }
            ns += tot;
        }
        hdr1 = nfront | ((uint64_t)ns << 32);
    } else {
        uint64_t pos = nfront;
        for (int q = 0; q < kParLv; ++q) {  // kParRegs bucket loads in flight per thread
            const uint32_t cq = PS.bcnt[q];
            for (uint32_t e0 = 0; e0 < cq; e0 += kParT * kParRegs) {
                uint64_t x[kParRegs];
                const uint32_t vm = bucket_batch(P, (uint32_t)q, e0, cq, x);
#pragma unroll
                for (int r = 0; r < kParRegs; ++r)
                    if ((vm >> r) & 1u) ast(out + pos + e0 + threadIdx.x + r * kParT, x[r]);
            }
            pos += cq;
        }
    }
#ifdef TDA_PROFILE
    C.q2[6] += 1;
    C.q2[7] += total;
    C.q2[4] += clock64() - tsv;
#endif
    drain_vm();
    __syncthreads();
    if (threadIdx.x == 0) {
        // the bucket chunks were written with plain stores: write this XCD's L2 back before
        // the header (and the CAS after it) can be seen by a reader on another XCD
        if (segd) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        uint64_t* rh = P.rec + id * 4;
        ast(rh + 0, off | (segd ? kParSegBit : 0ull));
        ast(rh + 1, hdr1);
        ast(rh + 2, pkey);
        ast(rh + 3, item);
    }
    drain_vm();  // every storing wave, before the barrier that precedes the publishing CAS
    __syncthreads();
    *seg = segd;
    return (int64_t)id;
}

// add len keys src[0 .. len) (plain loads: the caller acquired) to the working column
__device__ __forceinline__ void col_add_keys(ParCol& C, const ParBufs& P, const uint64_t* src, uint64_t len) {
    for (uint64_t e0 = 0; e0 < len; e0 += kParT * kParRegs) {
        uint64_t x[kParRegs];
        uint32_t vm = 0;
#pragma unroll
        for (int q = 0; q < kParRegs; ++q) {
            const uint64_t e = e0 + threadIdx.x + (uint64_t)q * kParT;
            x[q] = e < len ? ld_glb(src, e) : 0;
            if (e < len && (uint32_t)(x[q] >> 32) <= C.capbits) vm |= 1u << q;  // keys above the column's cap: dropped
        }
        PAR_T0(tr0);
        front_room(C, P, kParT * kParRegs);
#ifdef TDA_PROFILE
        C.q2[0] += clock64() - tr0;
        {
            uint32_t nf = 0;
#pragma unroll
            for (int q = 0; q < kParRegs; ++q)
                nf += ((vm >> q) & 1u) && par_bucket(x[q], PS.last) <= PS.kf;
            C.q2[2] += C.rd.sum(nf);
            C.q2[3] += C.rd.sum((uint32_t)__builtin_popcount(vm)) ;
        }
        const uint64_t ta0 = clock64();
#endif
        if (PS.err) return;
        col_add<kParRegs>(C, P, x, vm);
#ifdef TDA_PROFILE
        C.q2[1] += clock64() - ta0;
#endif
    }
}

// add record `id` (sc1 loads) to the working column
__device__ __forceinline__ void col_add_record(ParCol& C, const ParBufs& P, uint64_t id) {
    if (threadIdx.x == 0) {  // header by sc1 loads, then ONE agent acquire: the payload reads are plain loads
        PS.bc[2] = ald(P.rec + id * 4 + 0);
        PS.bc[3] = ald(P.rec + id * 4 + 1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        drain_vm();
    }
    __syncthreads();
    const uint64_t h0 = PS.bc[2], h1 = PS.bc[3];
    __syncthreads();
    const uint64_t off = h0 & ~kParSegBit;
    if (!(h0 & kParSegBit)) {
#ifdef TDA_PROFILE
        C.q[4] += 1;
        C.q[5] += h1;
#endif
        col_add_keys(C, P, P.rpool + off, h1);
    } else {  // segmented: front keys, then every (offset, count) segment of bucket chunks
        const uint64_t nfront = h1 & 0xFFFFFFFFull, ns = h1 >> 32;
        const uint64_t* tab = P.rpool + off + nfront;
#ifdef TDA_PROFILE
        C.q[4] += 1;
        C.q[5] += nfront;
#endif
        col_add_keys(C, P, P.rpool + off, nfront);
        uint64_t so = ns ? ld_glb(tab, 0) : 0, sc = ns ? ld_glb(tab, 1) : 0;
        for (uint64_t g = 0; g < ns && !PS.err; ++g) {
            // the next descriptor is in flight while this segment is added
            const uint64_t no = g + 1 < ns ? ld_glb(tab, 2 * (g + 1)) : 0, nc = g + 1 < ns ? ld_glb(tab, 2 * (g + 1) + 1) : 0;
#ifdef TDA_PROFILE
            C.q[5] += sc;
#endif
            col_add_keys(C, P, P.bpool + so, sc);
            so = no;
            sc = nc;
        }
    }
    __syncthreads();
}

// owner-map probe (one lane): slot of pivot pidx, and its value (0 if absent: *slot = first empty)
__device__ __forceinline__ uint64_t omap_find(const ParBufs& P, uint64_t* okey, uint64_t* oval, uint64_t mask, uint64_t pidx, uint64_t* slot,
                              bool* found) {
    uint64_t h = mix64(pidx) & mask;
    for (uint64_t it = 0; it <= mask; ++it, h = (h + 1) & mask) {
        const uint64_t k = ald(okey + h);
        if (k == pidx + 1) {
            *slot = h;
            *found = true;
            for (uint32_t s = 0; s < kParSpin; ++s) {  // the inserter stores the value right after its key CAS
                const uint64_t v = ald(oval + h);
                if (v) return v;
                __builtin_amdgcn_s_sleep(1);
            }
            return kEmpty64;  // hung
        }
        if (k == 0) {
            *slot = h;
            *found = false;
            return 0;
        }
    }
    *found = false;
    return kEmpty64;  // map full
}

__device__ __forceinline__ uint64_t par_omask(uint64_t nres, uint64_t ostride) {
    uint64_t m = 16;
    while (m < 2 * nres + 16) m <<= 1;
    return (m > ostride ? ostride : m) - 1;
}

// DIM 1: edge columns, triangle rows (PACKED: N <= 1024).  DIM 2: triangle
// columns, tetrahedron rows (PACKED: N <= 400); a triangle is cleared when it
// is any H1 pivot: `clr` is the dim-1 pivot bitmap, which k_par_emit<1> has
// completed with the residual H1 pivots.
// WIDE (DIM 2, N > 568): rows keyed by edge codes (see rips_reduce_big.h):
// dcode / dsort / ecap from k_edge_sort / k_edge_codes.
template <int DIM, bool PACKED, bool WIDE = false>
__global__ __launch_bounds__(kParT) void k_reduce_par(const float* __restrict__ dist, int n, int L, LayerStats* __restrict__ stats,
                                                      DimBufs b1, const uint32_t* __restrict__ clr, uint64_t clr_words, Reduce2Bufs rb,
                                                      ParBufs P, const uint32_t* __restrict__ dcode, const uint64_t* __restrict__ dsort,
                                                      uint64_t ecap) {
    static_assert(!WIDE || (DIM == 2 && !PACKED), "wide keys: unpacked H2 rows only");
    ParCol C;
    const int tid = threadIdx.x;
    for (uint32_t e = tid; e < (uint32_t)kParLv * kParChunks; e += kParT) (&PS.cptr[0][0])[e] = kNoChunk;
    if (tid == 0) {
        PS.err = 0;
        PS.wide = WIDE ? 1u : 0u;
        PS.redm[0] = PS.redm[1] = PS.redm[2] = kEmpty64;
    }
    __syncthreads();
    const uint64_t total = ald(&P.ctl->total);
#ifdef TDA_PROFILE
    if (tid == 0) atomicMin((unsigned long long*)&P.ctl->pad[0], (unsigned long long)wall_clock64());
#endif
    bool prealloc = false;
    for (;;) {
        // ---------------- get work (lane 0): requeued columns first, then fresh ones.
        // A worker with nothing to take exits: every requeue push is made by a
        // worker that dequeues again right after, so no item is ever stranded
        // and nobody spins idle next to the columns still being reduced.
        if (tid == 0) {
            uint64_t got = kEmpty64;  // item << 32 | (record + 1)
            for (uint32_t spin = 0; spin < kParSpin; ++spin) {
                if (ald(&P.ctl->abort)) break;
                const uint64_t h = ald(&P.ctl->rq_head), t = ald(&P.ctl->rq_tail);
                if (h < t && h < P.rq_cap) {
                    if (acas((uint64_t*)&P.ctl->rq_head, h, h + 1) != h) continue;
                    uint64_t v = 0;
                    for (uint32_t q = 0; q < kParSpin && !(v = ald(P.rq + h)); ++q) __builtin_amdgcn_s_sleep(1);
                    if (!v) {  // the pusher never wrote its slot
                        aadd(&P.ctl->abort, 1);
                        acas((uint64_t*)&P.ctl->err, 0, 51);
                        break;
                    }
                    ast(P.rq + h, 0);  // slots are used once per launch; leave the ring zeroed
                    got = v;
                    break;
                }
                if (ald(&P.ctl->next) < total) {
                    const uint64_t c = aadd(&P.ctl->next, 1);
                    if (c < total) got = c << 32;
                }
                break;
            }
            PS.bc[4] = got;
        }
        __syncthreads();
        const uint64_t got = PS.bc[4];
        __syncthreads();
        if (got == kEmpty64) break;
        const uint64_t item = got >> 32;
        const uint64_t rec0 = got & 0xFFFFFFFFull;  // 0: fresh column, else resume from record rec0 - 1
        // ---------------- layer / column
        int l = 0;
        while (l + 1 < L && ld_glb(P.item_base, l + 1) <= item) ++l;
        const uint64_t j = item - ld_glb(P.item_base, l);
        LayerStats* st = stats + l;
        const float r = st->thresh;
        const float* D = dist + (size_t)l * n * n;
        // rows the coboundaries read: distances, or (WIDE) edge codes in float slots
        const float* Dr = WIDE ? (const float*)(dcode + (size_t)l * n * n) : D;
        const uint64_t* resid = b1.resid + (size_t)l * b1.rcap;
        const uint32_t* pivg = b1.pivbits + (size_t)l * b1.piv_words;
        const uint32_t* mst = rb.mst + (size_t)l * rb.mst_words;
        // the column's layer / index / item, read back from LDS where the owner path and the column's
        // end need them, so they are not live in scalar registers through the step loop (r06: SGPR
        // spills 167 -> 159, torus1024 32.3 -> 32.0 ms, torus2048 657 -> 655 ms)
        if (tid == 0) {  // published by the working column's reset barrier below
            PS.ccol[0] = (uint64_t)l;
            PS.ccol[1] = j;
            PS.ccol[2] = item;
        }
#define PAR_CL ((int)PS.ccol[0])
#define PAR_CJ (PS.ccol[1])
#define PAR_CITEM (PS.ccol[2])
        const uint64_t ckey = ld_glb(resid, j);
        const uint64_t sidx = key_idx(ckey);
        const float sdm = key_diam(ckey);
        // Column cap (r05).  With ripser's default threshold (the enclosing radius) the complex at r
        // is a cone, so no H1 / H2 class is essential: every residual column has a finite pivot
        // <= r.  Column j keeps only the keys <= rc = birth_j + capf * r (the rest are never stored):
        // the reduction restricted to rows <= rc is exact for every column whose pivot is <= rc,
        // because pivots only grow along a column's reduction.  The records j adds come from
        // EARLIER columns (larger births, so larger caps: they hold every key j keeps), and an
        // evicted column re-adds the record of an earlier one (the same order).  A column that
        // runs empty below its cap has its pivot above it: its layer is flagged (ERR_CAP_MISS) and the
        // host re-runs that layer alone without caps -- the other layers of the launch are unaffected
        // (a missed column never claims a pivot, and a column of another layer never reads this
        // layer's records); the flagged layer's other H1 columns still run, its H2 columns do not.  90 % of the keys the longest
        // torus1024 column generates lie above its final pivot (tools/front_sim.py).
        float rc = r;
        bool capped = false;
        if (!WIDE && P.capf > 0.0f) {
            const float capd = sdm + P.capf * r;
            if (capd < r) {
                rc = capd;
                capped = true;
            }
        }
        C.capbits = capped ? __float_as_uint(rc) : 0xFFFFFFFFu;
        int sv[DIM + 1];
        decode<DIM>(sidx, n, sv);
        const uint32_t* cbits = DIM == 1 ? mst : clr + (size_t)l * clr_words;
        if (!rec0 && ((ld_glb(cbits, sidx >> 5) >> (sidx & 31)) & 1u)) {  // cleared: an H_{DIM-1} death
            if (tid == 0) ast(P.colpiv + (size_t)l * b1.rcap + j, kParSkip);
            continue;
        }
        // ---------------- working column: reset (chunks stay), then the coboundary or the record
        if (!prealloc) {  // chunks 0..3 of every bucket (bucket_append opens chunk c + 2 from chunk c)
            if (tid == 0) {
                constexpr uint64_t per = (uint64_t)kParLv * chunk_start(4);
                const uint64_t o = aadd(&P.ctl->bpool_used, per);
                PS.bc[5] = o + per <= P.bpool_cap ? o : kEmpty64;
            }
            __syncthreads();
            const uint64_t o = PS.bc[5];
            if (o == kEmpty64) {
                if (tid == 0) {
                    acas((uint64_t*)&P.ctl->err, 0, ((uint64_t)item << 16) | 22u);
                    aadd(&P.ctl->abort, 1);
                }
                break;
            }
            for (uint32_t e = tid; e < (uint32_t)kParLv * 4u; e += kParT)
                PS.cptr[e / 4][e % 4] = (uint32_t)((o + (e / 4) * chunk_start(4) + chunk_start(e % 4)) >> 8);
            prealloc = true;
        }
        for (uint32_t q = tid; q < kParLv; q += kParT) PS.bcnt[q] = 0;
        uint32_t sc = 0;  // WIDE: the column's edge code
        if constexpr (WIDE) {
            const uint32_t* Dc = (const uint32_t*)Dr;
            sc = max(ld_glb(Dc, (size_t)sv[0] * n + sv[1]), max(ld_glb(Dc, (size_t)sv[0] * n + sv[2]), ld_glb(Dc, (size_t)sv[1] * n + sv[2])));
        }
        if (tid == 0) {
            PS.kf = kParLv - 1;
            PS.last = WIDE ? (uint64_t)sc << kWideIdxBits : (uint64_t)__float_as_uint(sdm + 0.0f) << 32;
        }
        front_reset();
        if (!rec0) {
            float z[DIM + 1][kParRV];
#pragma unroll
            for (int q = 0; q < kParRV; ++q) {
                const int v = par_vert(0, q);
#pragma unroll
                for (int i = 0; i <= DIM; ++i) z[i][q] = v < n ? ld_glb(Dr, (size_t)sv[i] * n + v) : 0.0f;
            }
            if constexpr (DIM == 1)
                col_cob<PACKED>(C, P, D, n, rc, sv[0], sv[1], sdm, z[0], z[1]);
            else
                col_cob2<PACKED, WIDE>(C, P, Dr, n, rc, sv[0], sv[1], sv[2], WIDE ? __uint_as_float(sc) : sdm, z);
        } else {
            if (tid == 0) PS.last = ald(P.rec + (rec0 - 1) * 4 + 2);  // the record's pivot: its smallest key
            __syncthreads();
            col_add_record(C, P, rec0 - 1);
        }
        int64_t my_rec = -1;
        bool my_seg = false;  // my_rec is zero-copy: it owns this workgroup's bucket chunks
        uint64_t adds = 0;
        bool done = false;
#ifdef TDA_PROFILE
        uint64_t pf[8] = {0, 0, 0, 0, 0, 0, 0, 0}, nref = 0, fsum = 0;
        const uint64_t t_col = clock64(), w_col = wall_clock64();
        C.ncompact = C.nspill = 0;
        for (int q = 0; q < 8; ++q) C.q[q] = C.q2[q] = C.q3[q] = 0;
#endif
        uint64_t step = 0;
        const uint32_t need = par_need(n);
#ifdef TDA_PROF2
        for (int q = 0; q < 8; ++q) C.tp[q] = 0;
#endif
        for (; !done; ++step) {
            P2_T(ps0);
            front_room(C, P, need);  // barrier: the previous step's toggles and appends are done
            P2_ACC(0, ps0);
            if (PS.err) break;
            if (step > P.step_limit) {
                if (tid == 0) PS.err = 61;
                break;
            }
#ifdef TDA_PROFILE
            fsum += PS.fcnt;
            uint64_t t0 = clock64();
#endif
            P2_T(ps1);
            uint64_t pk = front_min(C.rd);
            P2_ACC(1, ps1);
#ifdef TDA_PROFILE
            pf[1] += clock64() - t0;
            t0 = clock64();
#endif
            if (pk == kEmpty64) {
#ifdef TDA_PROFILE
                ++nref;
#endif
                P2_T(ps6);
                const bool more = col_refill(C, P);
                P2_ACC(6, ps6);
#ifdef TDA_PROFILE
                pf[4] += clock64() - t0;
#endif
                if (!more) {
                    if (PS.err) break;
                    if (capped) {  // empty below the cap: the pivot lies above it -> this layer re-runs uncapped
                        if (tid == 0) PS.err = 81;
                        break;
                    }
                    if (tid == 0) ast(P.colpiv + (size_t)PAR_CL * b1.rcap + PAR_CJ, kParEss);  // zero column: essential
                    done = true;
                }
                continue;
            }
            // pivot: vertices, index, apparent facet fv
            P2_T(ps2);
            int fv[DIM + 1];
            uint64_t pidx;
            const uint32_t plo = 0xFFFFFFFFu - (uint32_t)pk;
            const float pd = WIDE ? __uint_as_float((uint32_t)ld_glb(dsort + (size_t)l * ecap, pk >> kWideIdxBits))
                                  : __uint_as_float((uint32_t)(pk >> 32));
            uint32_t fsc = 0;  // WIDE: the facet's edge code
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
                    (void)apparent_facet<1>(D, n, pidx, fv);
                }
            } else if constexpr (WIDE) {
                pidx = kWideIdxMask - (pk & kWideIdxMask);
                (void)apparent_facet<2>(D, n, pidx, fv);
                const uint32_t* Dc = (const uint32_t*)Dr;
                fsc = max(ld_glb(Dc, (size_t)fv[0] * n + fv[1]), max(ld_glb(Dc, (size_t)fv[0] * n + fv[2]), ld_glb(Dc, (size_t)fv[1] * n + fv[2])));
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
            // one round trip: the pivot's bitmap word and the facet's rows
            float z[DIM + 1][kParRV];
#pragma unroll
            for (int q = 0; q < kParRV; ++q) {
                const int v = par_vert(0, q);
#pragma unroll
                for (int i = 0; i <= DIM; ++i) z[i][q] = v < n ? ld_glb(Dr, (size_t)fv[i] * n + v) : 0.0f;
            }
            // every thread reads the pivot's bitmap word (one address per wave): no barrier.  (r05: a
            // per-edge apparent-partner table, 2 B per edge -- 1 MB per layer at N = 1024 against the
            // 22 MB triangle bitmap -- measured no faster: torus1024 37.0 vs 36.7 ms, dropped)
            const uint32_t pw = ld_glb(pivg, pidx >> 5);
            const bool app = (pw >> (pidx & 31)) & 1u;
            P2_DEP(pw);
            P2_ACC(2, ps2);
#ifdef TDA_PROFILE
            pf[2] += clock64() - t0;
            t0 = clock64();
#endif
            if (app) {
                if constexpr (DIM == 1)
                    col_cob<PACKED>(C, P, D, n, rc, fv[0], fv[1], pd, z[0], z[1]);
                else
                    col_cob2<PACKED, WIDE>(C, P, Dr, n, rc, fv[0], fv[1], fv[2], WIDE ? __uint_as_float(fsc) : pd, z);
                ++adds;
#ifdef TDA_PROFILE
                pf[3] += clock64() - t0;
#endif
                continue;
            }
            // ---------------- residual pivot: owner map
            P2_T(ps7);
            const uint64_t fkey = WIDE ? pk : filt_key(pd, pidx);  // colpiv: k_par_emit decodes it
            const int lc = PAR_CL;
            const uint64_t jc = PAR_CJ;
            uint64_t* okey = P.okey + (size_t)lc * P.ostride;
            uint64_t* oval = P.oval + (size_t)lc * P.ostride;
            const uint64_t omask = par_omask(ld_glb(P.item_base, lc + 1) - ld_glb(P.item_base, lc), P.ostride);
            for (uint32_t round = 0;; ++round) {
                if (tid == 0) {
                    uint64_t slot = 0;
                    bool found = false;
                    const uint64_t v = round > 64 ? kEmpty64 : omap_find(P, okey, oval, omask, pidx, &slot, &found);
                    PS.bc[6] = v;
                    PS.bc[7] = slot | (found ? 1ull << 63 : 0);
                }
                __syncthreads();
                const uint64_t v = PS.bc[6];
                const uint64_t slot = PS.bc[7] & ~(1ull << 63);
                __syncthreads();
                if (v == kEmpty64) {
                    if (tid == 0) PS.err = 71;
                    break;
                }
                const uint64_t oi = v >> 32;
                if (v != 0 && oi < jc) {  // earlier owner: add its record
                    col_add_record(C, P, (v & 0xFFFFFFFFull) - 1);
                    ++adds;
                    break;
                }
                if (v != 0 && oi == jc) {
                    if (tid == 0) PS.err = 72;
                    break;
                }
                // free, or owned by a later column: publish R_j, then claim
                if (my_rec < 0) {
                    my_rec = col_save(C, P, pk, PAR_CITEM, &my_seg);
                    if (my_rec < 0) break;
                }
                const uint64_t mine = (jc << 32) | (uint64_t)(my_rec + 1);
                if (tid == 0) {
                    bool ok;
                    if (v == 0) {
                        const uint64_t old = acas(okey + slot, 0, pidx + 1);
                        ok = old == 0;
                        if (ok) ast(oval + slot, mine);
                        // lost the key race (same pivot) or the slot (another pivot): look again
                    } else {
                        ok = acas(oval + slot, v, mine) == v;
                        if (ok) {  // evict the later owner: it resumes from its record
                            const uint64_t qt = aadd(&P.ctl->rq_tail, 1);
                            if (qt >= P.rq_cap) {
                                aadd(&P.ctl->abort, 1);
                                acas((uint64_t*)&P.ctl->err, 0, 53);
                            } else {
                                const uint64_t oitem = ld_glb(P.item_base, lc) + oi;
                                ast(P.rq + qt, (oitem << 32) | (v & 0xFFFFFFFFull));
                            }
                            aadd(&P.ctl->evictions, 1);
                        }
                    }
                    if (ok) ast(P.colpiv + (size_t)lc * b1.rcap + jc, fkey);
                    PS.bc[6] = ok;
                }
                __syncthreads();
                const bool ok = PS.bc[6] != 0;
                __syncthreads();
                if (ok) {
                    done = true;
                    break;
                }
            }
            // a record added above changes the column: any saved record is stale
            if (!done) my_rec = -1;
            P2_ACC(7, ps7);
#ifdef TDA_PROFILE
            pf[5] += clock64() - t0;
#endif
        }
#ifdef TDA_PROFILE
        // the column with the most steps so far publishes its profile (layer 0 slot, racy by design)
        if (tid == 0 && step > stats[0].prof[2][6]) {
            pf[0] = clock64() - t_col;
            pf[6] = step;
            pf[7] = (fsum / (step ? step : 1)) | (nref << 16) | (C.ncompact << 32) | (C.nspill << 48);
            for (int q = 0; q < 8; ++q) stats[0].prof[2][q] = pf[q];
            for (int q = 0; q < 8; ++q) stats[0].prof[3][q] = C.q[q];
            for (int q = 0; q < 8; ++q) stats[0].prof[4][q] = C.q2[q];
            for (int q = 0; q < 8; ++q) stats[0].prof[1][q] = C.q3[q];
        }
#endif
#ifdef TDA_PROF2
        if ((tid & 63) == 0 && step >= kParP2MinSteps && P.dbg) {  // every wave's phase cycles of a long column
            const uint64_t q = aadd(&P.ctl->pad[2], 1ull);
            if (q < kParDbgCap) {
                uint64_t* o = P.dbg + (uint64_t)kParDbgCap * 4 + q * kParP2Words;
                o[0] = ((uint64_t)l << 40) | j;
                o[1] = (uint64_t)(tid >> 6);
                o[2] = step;
                for (int u = 0; u < 8; ++u) o[3 + u] = C.tp[u];
            }
        }
#endif
#ifdef TDA_PROFILE
        if (tid == 0 && step >= kParDbgMinSteps && P.dbg) {  // the long columns' timeline (wall clock, 100 MHz)
            const uint64_t q = aadd(&P.ctl->pad[1], 1ull);
            if (q < kParDbgCap) {
                P.dbg[q * 4 + 0] = ((uint64_t)l << 40) | j;
                P.dbg[q * 4 + 1] = w_col;
                P.dbg[q * 4 + 2] = wall_clock64();
                P.dbg[q * 4 + 3] = step | (rec0 ? 1ull << 63 : 0ull);
            }
        }
#endif
        if (tid == 0 && adds) atomicAdd((unsigned long long*)&stats[PAR_CL].n_adds[DIM], (unsigned long long)adds);
        if (done && my_rec >= 0 && my_seg) {  // the claimed record references this workgroup's chunks: fresh ones next
            for (uint32_t e = tid; e < (uint32_t)kParLv * kParChunks; e += kParT) (&PS.cptr[0][0])[e] = kNoChunk;
                    prealloc = false;
            __syncthreads();
        }
        if (PS.err) {
            if (PS.err == 81) {
                // a capped column ran empty below its cap: its layer is flagged (ERR_CAP_MISS) and re-run
                // alone, uncapped, by the host; this worker goes on with the next column.  (Handled here,
                // off the step loop: a flag check in the pickup or in the step loop raised k_reduce_par's
                // SGPR spills 164 -> 180 and cost torus1024 ~2 ms, r06.)
                __syncthreads();  // every thread has read PS.err
                if (tid == 0) {
                    atomicOr(&stats[PAR_CL].err, ERR_CAP_MISS);
                    ast(P.colpiv + (size_t)PAR_CL * b1.rcap + PAR_CJ, kParSkip);
                    PS.err = 0;
                }
                continue;  // the pickup's barrier publishes PS.err = 0
            }
            if (tid == 0) {
                acas((uint64_t*)&P.ctl->err, 0, ((uint64_t)PAR_CITEM << 16) | (uint64_t)PS.err);  // first error: item, code
                aadd(&P.ctl->abort, 1);
            }
            break;
        }
    }
}

#undef PAR_CL
#undef PAR_CJ
#undef PAR_CITEM

// per-layer residual counts -> item prefix, control block, owner maps cleared
__global__ __launch_bounds__(256) void k_par_init(LayerStats* __restrict__ stats, int L, uint64_t rcap, ParBufs P, int dim) {
    const int l = blockIdx.y;
    uint64_t nres = (uint64_t)stats[l].n_residual[dim];
    if (nres > rcap) nres = rcap;
    const uint64_t m = par_omask(nres, P.ostride) + 1;
    uint64_t* ok = P.okey + (size_t)l * P.ostride;
    uint64_t* ov = P.oval + (size_t)l * P.ostride;
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (uint64_t)gridDim.x * blockDim.x) {
        ok[e] = 0;
        ov[e] = 0;
    }
    if (blockIdx.x == 0 && l == 0 && threadIdx.x == 0) {
        if (dim > 1 && P.ctl->abort) {  // the H1 launch aborted: keep its flag and error, run nothing
            P.ctl->total = 0;
            return;
        }
        uint64_t s = 0;
        for (int q = 0; q < L; ++q) {
            P.item_base[q] = s;
            uint64_t c = (uint64_t)stats[q].n_residual[dim];
            // H2 of a layer whose H1 missed a column cap: nothing (the host re-runs the layer; its H1
            // pivots, H2's clearing test, are incomplete)
            if (dim > 1 && (stats[q].err & ERR_CAP_MISS)) c = 0;
            s += c > rcap ? rcap : c;
        }
        P.item_base[L] = s;
        unsigned long long* c = (unsigned long long*)P.ctl;
        for (int q = 0; q < (int)(sizeof(ParCtl) / 8); ++q) c[q] = 0;
        P.ctl->total = s;
        P.ctl->pad[0] = ~0ull;  // -DTDA_PROFILE: earliest workgroup start (atomicMin)
    }
}

// Pairs from the final owners (one block per layer): emission buffer, stats,
// and (DIM 1, H2 next) the residual H1 pivots that the H2 reduction clears
// with: fill_map 1 -> the dim-1 pivot map (k_reduce_big), 2 -> OR'ed into the
// dim-1 pivot bitmap (k_reduce_par<2>).
template <int DIM>
__global__ __launch_bounds__(1024) void k_par_emit(LayerStats* __restrict__ stats, DimBufs b1, Reduce2Bufs rb, ParBufs P,
                                                   Pair* __restrict__ pairs, uint64_t pcap, int fill_map,
                                                   const uint64_t* __restrict__ dsort = nullptr, uint64_t ecap = 0) {
    __shared__ uint64_t red[3][16];
    const int l = blockIdx.x, tid = threadIdx.x;
    LayerStats* st = stats + l;
    const uint64_t nres = P.item_base[l + 1] - P.item_base[l];
    const uint64_t* resid = b1.resid + (size_t)l * b1.rcap;
    const uint64_t* colpiv = P.colpiv + (size_t)l * b1.rcap;
    Pair* Pp = pairs + (size_t)l * pcap;
    PivMap map;
    map.k = rb.rmap_keys + ((size_t)l * 2 + 0) * rb.rmap_stride;  // cleared by k_sort_resid
    map.v = rb.rmap_vals + ((size_t)l * 2 + 0) * rb.rmap_stride;
    {
        uint64_t rc2 = 16;
        while (rc2 < 2 * nres + 16) rc2 <<= 1;
        if (rc2 > rb.rmap_stride) rc2 = rb.rmap_stride;
        map.mask = rc2 - 1;
    }
    map.lds = false;
    const bool failed = P.ctl->abort != 0;
    const bool missed = (st->err & ERR_CAP_MISS) != 0;  // the host re-runs this layer without caps
    uint64_t cs = 0, np = 0, nskip = 0;
    if (!failed && !missed) {
        for (uint64_t j = tid; j < nres; j += blockDim.x) {
            const uint64_t cp = colpiv[j];
            const uint64_t key = resid[j];
            const uint64_t sidx = key_idx(key);
            const float sdm = key_diam(key);
            if (cp == kParSkip) {
                ++nskip;
                continue;
            }
            if (cp == kParEss) {
                const uint64_t pos = atomicAdd((unsigned long long*)&st->count[DIM], 1ull);
                if (pos < pcap) store_pair(Pp, pos, sdm, INFINITY, (int64_t)sidx, -1);
                else atomicOr(&st->err, ERR_PAIR_CAP);
                continue;
            }
            // colpiv: filtration key, or (dsort given) a wide code key
            const uint64_t pidx = dsort ? kWideIdxMask - (cp & kWideIdxMask) : 0xFFFFFFFFull - (cp & 0xFFFFFFFFull);
            const float pd = dsort ? __uint_as_float((uint32_t)dsort[(size_t)l * ecap + (cp >> kWideIdxBits)]) : __uint_as_float((uint32_t)(cp >> 32));
            if (pd > sdm) {
                const uint64_t pos = atomicAdd((unsigned long long*)&st->count[DIM], 1ull);
                if (pos < pcap) store_pair(Pp, pos, sdm, pd, (int64_t)sidx, (int64_t)pidx);
                else atomicOr(&st->err, ERR_PAIR_CAP);
            }
            cs += pair_hash(sidx, pidx);
            ++np;
            if (fill_map == 1) map.insert_par_t<false>((uint32_t)pidx, (uint32_t)j);
            if (fill_map == 2) atomicOr(&b1.pivbits[(size_t)l * b1.piv_words + (pidx >> 5)], 1u << (pidx & 31));
        }
    }
    cs = wave_sum_u64(cs);
    np = wave_sum_u64(np);
    nskip = wave_sum_u64(nskip);
    if ((tid & 63) == 0) {
        red[0][tid >> 6] = cs;
        red[1][tid >> 6] = np;
        red[2][tid >> 6] = nskip;
    }
    __syncthreads();
    if (tid == 0) {
        uint64_t a = 0, b = 0, c = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) a += red[0][w], b += red[1][w], c += red[2][w];
        if (failed) {
            atomicOr(&st->err, DIM == 1 ? ERR_PAR : ERR_PAR2);
        } else if (!missed) {
            atomicAdd((unsigned long long*)&st->checksum[DIM], (unsigned long long)a);
            atomicAdd((unsigned long long*)&st->all_pairs[DIM], (unsigned long long)b);
            atomicAdd((unsigned long long*)&st->n_columns[DIM], (unsigned long long)(0ull - c));
            st->nskip[DIM] = c;
        }
    }
}

#undef PS

}  // namespace tda
