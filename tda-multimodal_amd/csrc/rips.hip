// rips.hip -- host orchestration + C ABI (include/tda_rips.h) of the MI355X
// Vietoris-Rips persistence engine.  Built for gfx950 only:
//     hipcc --offload-arch=gfx950 -O3 -shared -fPIC rips.hip -o libtda_rips.so
//
// One call processes a batch of L layers (the reference's 32-layer sweep,
// debug_tda_pipeline.py:92-150) with ~8 + 3*maxdim kernel launches on one
// stream and a single host synchronisation at the end.
#include <hip/hip_runtime.h>
#include <execinfo.h>
#include <link.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../../include/tda_rips.h"
#include "rips_kernels.h"
#include "rips_reduce_big.h"
#include "rips_reduce_par.h"
#include "rips_reduce_small.h"

using namespace tda;

namespace {

thread_local std::string g_err;

// TDA_SEGV_TRACE=1 (diagnostics): a host segfault prints the faulting thread's native frames
// (backtrace_symbols_fd: module + offset) before the default action
void segv_trace(int sig, siginfo_t* si, void*) {
    void* fr[64];
    const int nf = backtrace(fr, 64);
    char msg[128];
    const int m = snprintf(msg, sizeof msg, "[tda-segv] signal %d, address %p, thread %ld\n", sig, si ? si->si_addr : nullptr,
                           (long)syscall(SYS_gettid));
    if (m > 0) (void)!write(2, msg, (size_t)m);
    backtrace_symbols_fd(fr, nf, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}
__attribute__((constructor)) void install_segv_trace() {
    const char* e = getenv("TDA_SEGV_TRACE");
    if (!e || e[0] != '1') return;
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = segv_trace;
    sa.sa_flags = SA_SIGINFO;
    sigaction(SIGSEGV, &sa, nullptr);
}

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPC(x)                                                                                   \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) return fail(TDA_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

inline uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}
inline uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }
inline int ilog2(uint64_t x) {
    int r = 0;
    while ((1ull << (r + 1)) <= x) ++r;
    return r;
}

// Test / A-B knobs (TDA_REDUCE, TDA_PAR, TDA_CHAIN, TDA_DIST, TDA_ORDER, ...)
// force a kernel variant or a launch shape.  The library honours them only
// when TDA_TEST_OVERRIDES=1 is set as well, so a stray variable in a user's
// environment cannot change the reducer (tests/conftest.py sets the gate).
const char* test_env(const char* name) {
    const char* g = getenv("TDA_TEST_OVERRIDES");
    return (g && g[0] == '1' && !g[1]) ? getenv(name) : nullptr;
}
bool test_env_is(const char* name, const char* val) {
    const char* m = test_env(name);
    return m && !strcmp(m, val);
}

constexpr uint64_t kRCapMax = 1ull << 22;    // residual columns per layer and dim
constexpr uint64_t kPCapMax = 1ull << 16;    // emitted pairs per layer and dim (H>=1)
constexpr int kLdsMax = 160 * 1024;
constexpr int kSmallN = 64;                  // one-wave H0 + LDS-resident reduction up to here
constexpr int kAppLdsMaxN = 128;             // k_apparent stages the distance matrix in LDS up to here
constexpr int kBigMinN = 256;                // large-N reducer above this N (global mode)
constexpr int64_t kDistMfmaMinD = 32;        // k_distance_mfma (FP64 MFMA Gram tiles) from this D up
constexpr unsigned kParGrid = 512;           // k_reduce_par workgroups at most (pool sizing): two 72-KB-LDS workgroups per CU
// default: one per CU -- the longest column is the critical path and runs
// faster without a second workgroup on its CU (r02, tools/ab_pargrid.sh:
// grid144 10.5 -> 8.5 ms, torus1024 61 -> 58.5 ms at 256 vs 512)
constexpr unsigned kParGridDefault = 256;
// column cap of k_reduce_par: keys above birth + f * thresh are never stored.  f = 0.5 keeps
// 35 % of the keys of torus1024's longest column (whose pivot is at birth + 0.35 thresh; the
// largest H1 persistence of the torus seeds, grid144 and the sweep clouds is <= 0.38 thresh); a
// cap that is too small costs one uncapped re-run of the call, remembered for the shape.
// TDA_PAR_CAPF (tests) overrides it (0 = off).
float par_capf() {
    const char* e = test_env("TDA_PAR_CAPF");
    return e ? (float)atof(e) : 0.5f;
}
unsigned par_grid_size() {
    const char* g = test_env("TDA_PAR_GRID");
    const unsigned v = g ? (unsigned)atoi(g) : kParGridDefault;
    return v < 1 ? 1 : (v > kParGrid ? kParGrid : v);
}

// ------------------------------------------------------------------ plan
struct Plan {
    int64_t L = 0, N = 0, D = 0;
    int maxdim = 0, dtype = 0, is_dist = 0;
    bool want64 = false;  // TDA_FLAG_DIST64: f64 distances of f64 points as well (dperm2all)
    uint64_t ncand[4] = {0}, piv_words[4] = {0}, rcap[4] = {0}, pcap[4] = {0};
    uint64_t mst_words = 0, max_rcap = 0, rmap_stride = 0, vpool_cap = 0, wcap_g = 0, vcap_g = 0, sstride = 0;
    bool lds_mode = false;
    bool big = false;  // k_reduce_big (1024-thread radix-heap reduction) instead of one wave per layer
    bool par = false;  // H1 on k_reduce_par (many columns in flight), k_reduce_big for H2 / fallback
    bool par2 = false;    // H2 on k_reduce_par as well (N <= 568: 32-bit tetrahedron indices)
    bool packed = false;  // k_reduce_par keys carry packed vertices + apparent facet (N <= 1024)
    bool wide = false;    // H2 on k_reduce_big with edge-code keys (tetrahedron indices > 32 bits)
    uint64_t ecap = 0;    // per-layer stride of the sorted edge lengths
    size_t o_dsort = 0, o_dtmp = 0, o_dcode = 0;
    int dsplit = 1;       // K slices of k_distance_mfma (1: no split)
    bool gram_layer = false;  // N <= 144, f32: k_gram_layer (whole upper triangle per workgroup) + combine
    size_t o_gpart = 0, o_npart = 0, o_d64 = 0;
    size_t o_bcomp = 0, o_bcheap = 0, o_bctl = 0;  // Borůvka H0 state (N > kH0WaveMaxN)
    bool serial_tables = false;  // HBM working tables of k_reduce_all (global mode) / k_reduce_big
    uint64_t ostride = 0, rec_cap = 0, rpool_cap = 0, bpool_cap = 0, rq_cap = 0;
    size_t o_pctl = 0, o_pitem = 0, o_pokey = 0, o_poval = 0, o_colpiv = 0, o_prec = 0, o_prpool = 0, o_pbpool = 0, o_prq = 0, o_pdbg = 0;
    bool dense = false;  // N <= 64: dense-bitmap H1 chain + column-parallel H2 phase 1 (rips_reduce_small.h)
    int dK = 0;          // dense H1 bitmap words per lane (a k_h1_chain instantiation)
    uint32_t inv_stride = 0;  // rank -> edge table stride (C(N,3) rounded up)
    uint32_t tri_stride = 0;  // triangle -> rank table stride (C(N,3) rounded up)
    bool fast = false;        // rank_of + inv32 tables exist (k_h1_chain FAST / TABLE)
    int cmode = 0;            // k_h1_chain MODE: kChainGeneral / kChainFast / kChainTable
    uint32_t cob_stride = 0;  // per-layer coboundary table (TABLE): E * N rounded up
    uint32_t chain_lds = 0;   // dynamic LDS of k_h1_chain
    uint32_t p1_lds = 0;      // dynamic LDS of k_h2_phase1
    int p1_waves = 1;         // waves per k_h2_phase1 block
    uint32_t n2p = 0;         // stride of the per-layer edge-class table (N * N rounded up)
    uint32_t bm_words = 0;    // tetrahedron membership bitmap of k_h2_phase1 (words)
    uint32_t prep_lds = 0;    // dynamic LDS of k_prep_edges
    ReduceAllCfg rcfg = {};
    // byte offsets in the device workspace
    size_t o_x = 0, o_dist = 0, o_stats = 0, o_mst = 0, o_piv[4] = {0}, o_resid[4] = {0}, o_tmp = 0, o_rmk = 0, o_rmv = 0,
           o_voff = 0, o_vlen = 0, o_vpool = 0, o_wk = 0, o_wt = 0, o_wp = 0, o_wl = 0, o_vk = 0, o_vt = 0, o_vp = 0, o_vl = 0, o_bref = 0, o_recs = 0, o_cls2 = 0, o_cls = 0, o_res1 = 0, o_inv32 = 0, o_rof = 0, o_inv = 0, o_epos = 0, o_cobt = 0, o_eM = 0, o_necnt = 0, o_p1next = 0, o_p1k = 0, o_p1i = 0, o_p1x = 0, o_roff2 = 0, o_rlen2 = 0, o_rpool2 = 0, o_p1used = 0,
           o_hsig = 0, o_rowmax = 0, o_pairs[4] = {0}, o_h0s = 0,
           o_fk = 0, o_fv = 0, o_pptr = 0, o_pcap = 0, o_outoff = 0, total = 0;
    size_t memset_lo = 0, memset_hi = 0;  // zeroed every call: stats .. pivbits
    // H2 pivot bitmap too large to memset every call (>= 2 GB: C(N, 4) / 8 B per layer, 91 GB at
    // N = 2048): kept zero between calls by k_clear_words over the words k_apparent<2> lists
    bool piv2_sparse = false;
    uint64_t clr_cap = 0;
    size_t o_clr2 = 0;
};

bool getenv_is(const char* name, const char* val) {
    const char* m = getenv(name);
    return m && !strcmp(m, val);
}


// pivots per column before a reduction kernel gives up (ERR_STEP_LIMIT): an
// exit guarantee, far above any real column (torus1024: < 2^15)
uint64_t step_limit() {
    const char* sl = test_env("TDA_STEP_LIMIT");
    return sl ? strtoull(sl, nullptr, 10) : (1ull << 26);
}

// LDS carve of k_reduce_all (mirrors the kernel): [16][dist][map H1][per-dim:
// map H2 (dim 2 only) + W (log 8 B + index 16 B per entry) + pivot bitmap]
ReduceAllCfg reduce_cfg(int n, int maxdim, const uint64_t* piv_words, bool lds_mode) {
    ReduceAllCfg c{};
    auto al = [](uint64_t x) { return (x + 15) & ~15ull; };
    const uint32_t mapcap = 1024;
    c.dist_lds = lds_mode ? 1 : 0;
    const uint64_t prefix = 16 + (c.dist_lds ? al(4ull * n * n) : 0) + 12ull * mapcap;
    uint64_t need = prefix;
    for (int d = 1; d <= maxdim; ++d) {
        Reduce2Cfg& r = c.dim[d];
        r.rmap_lds_cap = mapcap;
        const uint64_t map = d == 2 ? 12ull * mapcap : 0;
        const uint64_t piv = al(4ull * piv_words[d]);
        if (!lds_mode) {
            r.wcap = 0;
            r.piv_lds = 0;
            need = std::max<uint64_t>(need, prefix + map);
            continue;
        }
        r.wcap = 4096;
        r.piv_lds = 1;
        auto bytes = [&]() { return prefix + map + 24ull * r.wcap + r.wcap + (r.piv_lds ? piv : 0); };
        if (bytes() > (uint64_t)kLdsMax) r.piv_lds = 0;
        while (r.wcap > 1024 && bytes() > (uint64_t)kLdsMax) r.wcap >>= 1;
        need = std::max<uint64_t>(need, bytes());
    }
    c.bytes = (uint32_t)need;
    c.step_limit = step_limit();
    return c;
}

constexpr int kMaxParScale = 4;  // k_reduce_par capacity retries: pools up to 16x
// no_par: 0 = k_reduce_par for H1 and H2, 1 = H1 only (an H2 launch aborted), 2 = none
int make_plan(Plan& p, bool force_global, int scale, bool force_big, int no_par) {
    const uint64_t N = (uint64_t)p.N, L = (uint64_t)p.L;
    p.mst_words = (binom(N, 2) + 31) / 32 + 1;
    for (int d = 1; d <= p.maxdim; ++d) {
        p.ncand[d] = binom(N, d + 1);
        p.piv_words[d] = (binom(N, d + 2) + 31) / 32 + 1;
        p.rcap[d] = std::max<uint64_t>(1, std::min(p.ncand[d], kRCapMax));
        p.pcap[d] = std::max<uint64_t>(16, std::min(p.ncand[d], kPCapMax));
        p.max_rcap = std::max(p.max_rcap, p.rcap[d]);
    }
    p.pcap[0] = N + 1;
    p.max_rcap = std::max<uint64_t>(p.max_rcap, 1);
    p.rmap_stride = next_pow2(2 * p.max_rcap + 16);
    // capacity retries: `scale` grows the parallel reducer's pools up to 16x (kMaxParScale); the
    // other work buffers (serial reducers) grow up to 4x
    const int s2 = std::min(scale, 2);
    p.vpool_cap = std::min<uint64_t>(std::max<uint64_t>(1ull << 16, 32 * p.max_rcap), 1ull << 27) << s2;
    p.lds_mode = p.N <= kSmallN && !force_global;
    p.rcfg = reduce_cfg((int)N, p.maxdim, p.piv_words, p.lds_mode);
    p.wcap_g = (N <= 256 ? 1ull << 17 : (N <= 640 ? 1ull << 21 : 1ull << 23)) << (2 * s2);
    {
        const char* m = test_env("TDA_REDUCE");
        // measured (r01): one wave per layer beats the serial radix heap up to
        // N = 256 (grid144 md2 20.6 vs 26.8 ms); measured (r02): the parallel
        // reducer k_reduce_par beats both at every N > 64, H1 and H2, L = 1 and
        // 32 (tools/ab_reduce.py: grid144 md2 L=32 24.1 -> 6.8 ms, torus256
        // md2 L=32 926 -> 50 ms).  After a parallel abort (no_par) the old rule.
        const bool want_wave = m && !strcmp(m, "wave"), want_big = m && !strcmp(m, "big"), want_par = m && !strcmp(m, "par");
        const bool par_ok = no_par < 2 && p.maxdim >= 1 && !test_env_is("TDA_PAR", "0");
        p.big = !p.lds_mode && (force_big || want_big || want_par || (!want_wave && (p.N > kBigMinN || par_ok)));
        // TDA_PAR=0: H1 on the serial k_reduce_big as well (comparison / debugging)
        p.par = p.big && p.maxdim >= 1 && no_par < 2 && !test_env_is("TDA_PAR", "0");
        p.packed = p.N <= 1024;
        // C(N, 4) >= 2^32 (N > 568): the 32-bit index word of the H2 pivot keys
        // overflows; TDA_H2_WIDE=1 forces the wide keys on any big-path N (tests)
        p.wide = p.big && p.maxdim >= 2 && (binom(N, 4) >= (1ull << 32) || test_env_is("TDA_H2_WIDE", "1"));
        // TDA_PAR2=0: H2 on the serial radix-heap kernel after a parallel H1
        p.par2 = p.par && p.maxdim >= 2 && no_par < 1 && !test_env_is("TDA_PAR2", "0");
        p.dense = p.lds_mode && p.maxdim >= 1 && p.N <= kDenseMaxN && p.N >= 3 && !want_wave;
    }
    if (p.dense) {  // carve of rips_reduce_small.h (h1_chain / h2_phase1), mirrored here
        const uint64_t E = binom(N, 2), T3 = binom(N, 3);
        const int kneed = (int)std::max<uint64_t>(1, (((T3 + 31) / 32) + 63) / 64);
        p.dK = 0;
        for (int k : kChainKs)
            if (k >= kneed) {
                p.dK = k;
                break;
            }
        p.inv_stride = (uint32_t)align_up(T3, 8);
        auto al = [](uint64_t x) { return (x + 15) & ~15ull; };
        const uint64_t pre = 16 + al(4 * N * N);
        const uint64_t WP = 64ull * p.dK;
        p.tri_stride = (uint32_t)align_up(T3, 8);
        const uint64_t tail = 2 * al(4 * WP) + al(4 * p.piv_words[1]) + al(8ull * kChainMaxCols) + al(2ull * kChainMaxCols);
        const uint64_t fast_lds = pre + al(2ull * p.tri_stride) + al(4ull * p.inv_stride) + tail;
        p.cob_stride = (uint32_t)align_up(E * N, 8);
        const uint64_t table_lds = 16 + al(2ull * p.cob_stride) + al(2ull * p.inv_stride) + al(4 * WP) + al(4 * p.piv_words[1]) +
                                   al(8ull * kChainMaxCols) + al(2ull * kChainMaxCols);
        // TDA_CHAIN=general|fast forces a slower variant (tests)
        const bool want_gen = test_env_is("TDA_CHAIN", "general"), want_fast = test_env_is("TDA_CHAIN", "fast");
        p.cmode = kChainGeneral;
        if (!want_gen && p.dK <= kChainFastMaxK) {
            if (!want_fast && table_lds <= (uint64_t)kLdsMax)
                p.cmode = kChainTable;
            else if (fast_lds <= (uint64_t)kLdsMax)
                p.cmode = kChainFast;
        }
        p.fast = p.cmode != kChainGeneral;
        p.chain_lds = (uint32_t)(p.cmode == kChainTable  ? table_lds
                                 : p.cmode == kChainFast ? fast_lds
                                                         : pre + al(16 * E) + al(2ull * p.inv_stride) + tail);
        p.n2p = (uint32_t)align_up(N * N, 8);
        p.bm_words = (uint32_t)((binom(N, 4) + 31) / 32 + 1);
        // k_h2_phase1: shared matrix + class table, then one bitmap + log per wave (2 waves when they fit)
        const uint64_t p1_wave = al(4ull * p.bm_words) + 2 * al(4ull * kP1LogCap);
        p.p1_waves = (pre + al(2ull * p.n2p) + kP1MaxWaves * p1_wave <= (uint64_t)kLdsMax && !test_env_is("TDA_P1_WAVES", "1"))
                         ? kP1MaxWaves : 1;
        p.p1_lds = (uint32_t)(pre + al(2ull * p.n2p) + p.p1_waves * p1_wave);
        p.prep_lds = (uint32_t)(pre + al(8 * std::max<uint64_t>(2, next_pow2(E))));  // k_prep_edges' rank sort keys
        if (p.chain_lds > (uint32_t)kLdsMax || p.prep_lds > (uint32_t)kLdsMax || p.p1_lds > (uint32_t)kLdsMax || p.dK == 0)
            p.dense = false;
    }
    uint64_t maxp = 16;
    for (int d = 1; d <= p.maxdim; ++d) maxp = std::max(maxp, p.pcap[d]);
    p.sstride = 3 * maxp;

    size_t o = 0;
    auto take = [&](size_t bytes) {
        size_t r = o;
        o = align_up(o + bytes, 256);
        return r;
    };
    const size_t esz = p.dtype == TDA_F64 ? 8 : 4;
    p.o_x = take(L * N * (p.is_dist ? N : (uint64_t)std::max<int64_t>(p.D, 1)) * esz);
    {   // split-K for the MFMA distance when its tiles leave CUs idle: aim at ~3 workgroups per CU,
        // at least 4 K chunks per slice (TDA_DIST_SPLIT=n forces n).  The slice count fixes the f64
        // summation order, so it depends on (N, D) only -- sized for the reference's 32-layer sweep
        // (debug_tda_pipeline.py:92), never on this call's L: a layer's distances (and so its
        // diagram) are the same in a single call, a batch and every multi-GPU shard.
        const bool mfma = !p.is_dist && (test_env_is("TDA_DIST", "mfma") || (p.D >= kDistMfmaMinD && !test_env_is("TDA_DIST", "scalar")));
        if (mfma && p.dtype == TDA_F32 && N <= (uint64_t)kGlMaxN && !test_env_is("TDA_DIST", "tiles")) {
            // whole-layer Gram (k_gram_layer): K slices so that a 32-layer sweep runs two
            // workgroups per CU (512), at least 8 chunks each -- again from (N, D) only.
            // raw4096: 16 slices 94 us + combine 26 us; 8: 130 + 15; 32: 101 + 35 (r03)
            const uint64_t chunks = ((uint64_t)p.D + kDmKC - 1) / kDmKC;
            uint64_t sp = std::min<uint64_t>(16, std::max<uint64_t>(1, chunks / 8));
            if (const char* e = test_env("TDA_DIST_SPLIT")) sp = std::max(1, atoi(e));
            p.dsplit = (int)sp;
            p.gram_layer = true;
            p.o_gpart = take(L * sp * N * N * 8);
            p.o_npart = take(L * sp * N * 8);
        } else if (mfma) {
            constexpr uint64_t kSplitRefL = 32;
            const uint64_t nt = (N + kDmT - 1) / kDmT, tiles = nt * (nt + 1) / 2 * kSplitRefL, chunks = ((uint64_t)p.D + kDmKC - 1) / kDmKC;
            uint64_t sp = std::min<uint64_t>(8, std::max<uint64_t>(1, (768 + tiles - 1) / tiles));
            sp = std::min<uint64_t>(sp, std::max<uint64_t>(1, chunks / 4));
            if (const char* e = test_env("TDA_DIST_SPLIT")) sp = std::max(1, atoi(e));
            p.dsplit = (int)sp;
            if (p.dsplit > 1) {
                p.o_gpart = take(L * sp * N * N * 8);
                p.o_npart = take(L * sp * N * 8);
            }
        }
    }
    p.o_dist = take(L * N * N * 4);
    if (p.want64) p.o_d64 = take(L * N * N * 8);
    p.memset_lo = o;
    p.o_stats = take(L * sizeof(LayerStats));
    p.o_mst = take(L * p.mst_words * 4);
    // (TDA_PIV2_SPARSE=1 forces the sparse-clear bitmap at any size: the stale-bit tests at N = 300)
    p.piv2_sparse = p.maxdim >= 2 && ((L * p.piv_words[2] * 4 >= (2ull << 30) && !test_env_is("TDA_PIV2_SPARSE", "0")) ||
                                      test_env_is("TDA_PIV2_SPARSE", "1"));
    for (int d = 1; d <= p.maxdim; ++d)
        if (!(d == 2 && p.piv2_sparse)) p.o_piv[d] = take(L * p.piv_words[d] * 4);
    p.o_rowmax = take(L * N * 4);
    p.o_p1used = take(L * 8);
    p.o_p1next = take(L * 4);
    if (p.dense) {
        p.o_res1 = take(L * p.piv_words[1] * 4);
        p.o_necnt = take(L * 4);
    }
    p.memset_hi = o;
    if (p.piv2_sparse) {
        p.o_piv[2] = take(L * p.piv_words[2] * 4);
        // one entry per apparent H2 pair (at most one per triangle); an overflow only costs a memset
        p.clr_cap = std::min<uint64_t>(std::max<uint64_t>(p.ncand[2], 1), 1ull << 28);
        p.o_clr2 = take(L * p.clr_cap * 8);
    }
    for (int d = 1; d <= p.maxdim; ++d) p.o_resid[d] = take(L * p.rcap[d] * 8);
    p.o_tmp = take(L * 2 * p.max_rcap * 8);
    if (p.maxdim >= 1) {
        p.o_rmk = take(L * 2 * p.rmap_stride * 8);
        p.o_rmv = take(L * 2 * p.rmap_stride * 4);
        p.o_vlen = take(L * p.max_rcap * 4);
        p.o_vpool = take(L * p.vpool_cap * 8);
        p.o_voff = take(L * p.max_rcap * 8);
        uint64_t wmax = p.lds_mode ? 8192 : p.wcap_g;
        if (!p.big) p.o_wt = take(L * wmax * 8 * 2);  // slot scratch + compaction keys
        // global working tables of the one-wave / serial radix-heap kernels (not needed when
        // k_reduce_par takes H1 and there is no H2)
        p.serial_tables = !p.lds_mode && !(p.par && (p.maxdim < 2 || p.par2));
        if (p.serial_tables) {
            p.o_wk = take(L * p.wcap_g * 8);       // key log
            p.o_wl = take(L * p.wcap_g * 2 * 8);   // u64 index, 2 * wcap slots
            p.o_wp = take(L * p.wcap_g / 4 * 4);   // bucket fill counters
            if (p.big) p.o_bref = take(L * kNB * p.wcap_g * 4);  // radix-heap bucket references
        }
        if (p.wide) {
            p.ecap = align_up(std::max<uint64_t>(binom(N, 2), 1), 32);
            p.o_dsort = take(L * p.ecap * 8);
            p.o_dtmp = take(L * p.ecap * 8);
            p.o_dcode = take(L * N * N * 4);
        }
        if (p.par) {
            // k_reduce_par: owner maps, final pivots, records, bucket chunks, requeue slots
            const uint64_t prc = p.par2 ? std::max(p.rcap[1], p.rcap[2]) : p.rcap[1];
            p.ostride = next_pow2(2 * prc + 16);
            p.rec_cap = (2 * (uint64_t)L * prc + 4096) << scale;  // a capacity retry (scale) grows every pool
            // bucket chunks: every workgroup keeps its peak bucket sizes (torus N=1024 needs ~2^26 keys
            // in all, N=2048 ~2^28); records: raw copies of the paired columns.  HBM is 288 GB.
            auto clampp = [](uint64_t x, int lo, int hi) { return std::min<uint64_t>(std::max<uint64_t>(next_pow2(x), 1ull << lo), 1ull << hi); };
            // + chunks 0..3 of the kParLv buckets of every k_reduce_par workgroup
            // above N = 1024 start at 4x (torus N=2048 overflows 2x: measured r02, 3 attempts per call).
            // Per layer in the batch: every layer's long columns hold their bucket chunks at the same
            // time, and zero-copy records keep theirs (r03: 32 torus1024 layers per call overflowed a
            // per-call pool and fell back to the serial reducer)
            const int big4 = N > 1024 ? 2 : 0;
            // (at most 2^33 keys = 64 GiB of the 288 GiB; torus1024 x 32 layers draws ~2.5 G keys)
            p.bpool_cap = std::min<uint64_t>(clampp(N * N * 128 * L, 24, 32) << (scale + big4), 1ull << 33) +
                          (uint64_t)kParGrid * kParLv * 3840;
            // H2 records as well: grid144 (32 layers) stores ~4.4 M keys of reduced H2 columns
            p.rpool_cap = clampp(std::max<uint64_t>(N * N * 64 * std::min<uint64_t>(L, 8), p.par2 ? L * N * N * 8 : 0), 22, 29)
                          << (scale + big4);
            p.rq_cap = 1ull << (16 + scale);  // memset per launch: 0.5 MB at scale 0
            p.o_pctl = take(sizeof(ParCtl));
            p.o_pitem = take((L + 1) * 8);
            p.o_pokey = take(L * p.ostride * 8);
            p.o_poval = take(L * p.ostride * 8);
            p.o_colpiv = take(L * prc * 8);
            p.o_prec = take(p.rec_cap * 32);
            p.o_prpool = take(p.rpool_cap * 8);
            p.o_pbpool = take(p.bpool_cap * 8);
            p.o_prq = take(p.rq_cap * 8);
#if defined(TDA_PROFILE) || defined(TDA_PROF2)
            p.o_pdbg = take((size_t)kParDbgCap * 32 + (size_t)kParDbgCap * kParP2Words * 8);
#endif
        }
        if (p.dense) {
            p.o_recs = take(L * binom(N, 2) * 16);
            p.o_cls2 = take(L * (uint64_t)p.n2p * 2);
            p.o_cls = take(L * binom(N, 2) * 4);
            p.o_inv = take(L * (uint64_t)p.inv_stride * 2);
            p.o_epos = take(L * binom(N, 2) * 4);
            p.o_eM = take(L * binom(N, 2) * 8);
            if (p.fast) {
                p.o_inv32 = take(L * (uint64_t)p.inv_stride * 4);
                p.o_rof = take(L * (uint64_t)p.tri_stride * 2);
            }
            if (p.cmode == kChainTable) p.o_cobt = take(L * (uint64_t)p.cob_stride * 2);
            if (p.maxdim >= 2) {
                p.o_p1k = take(L * p.rcap[2] * 8);
                p.o_p1i = take(L * p.rcap[2] * 4);
                p.o_p1x = take(L * p.rcap[2] * 4);
                p.o_roff2 = take(L * p.rcap[2] * 8);
                p.o_rlen2 = take(L * p.rcap[2] * 4);
                p.o_rpool2 = take(L * p.vpool_cap * 8);
            }
        }
    }
    for (int d = 0; d <= p.maxdim; ++d) p.o_pairs[d] = take(L * p.pcap[d] * sizeof(Pair));
    p.o_h0s = take(L * 2 * N * 8 + 64);
    if (N > (uint64_t)kSmallN) {
        p.o_bcomp = take(L * N * 4);
        p.o_bcheap = take(L * N * 8);
        p.o_bctl = take(L * sizeof(BorCtl));
    }
    p.o_fk = take(L * 2 * p.sstride * 8);
    p.o_fv = take(L * 2 * p.sstride * 4);
    p.o_pptr = take(4 * sizeof(void*));
    p.o_pcap = take(4 * 8);
    p.o_outoff = take(L * 4 * 8);
    p.total = o;
    return 0;
}

// ------------------------------------------------------------------ workspace
struct Workspace {
    int device = -1;
    int slot = 0;
    bool init = false;
    hipStream_t stream = nullptr, stream2 = nullptr, stream3 = nullptr, stream4 = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, evf = nullptr, evj = nullptr, evs = nullptr, evp = nullptr, evh = nullptr, evsil = nullptr;
    char* dbuf = nullptr;
    size_t dcap = 0;
    OutPair* hout = nullptr;  // host-mapped
    OutPair* hout_dev = nullptr;
    size_t hout_cap = 0;      // in pairs
    LayerStats* hstats = nullptr;  // host-mapped: k_emit writes it
    // sparse-cleared H2 pivot bitmap (Plan::piv2_sparse): the region known to be zero
    bool piv2_dirty = true;
    char* piv2_ptr = nullptr;
    size_t piv2_bytes = 0;
    char* hsil = nullptr;          // host-mapped: silhouette labels [S][N] i32, then scores [L][S] f64
    char* hsil_dev = nullptr;
    size_t hsil_cap = 0;
    float* htn = nullptr;          // host-mapped: TwoNN estimates [L] (k_twonn writes them)
    float* htn_dev = nullptr;
    size_t htn_cap = 0;
    LayerStats* hstats_dev = nullptr;
    int64_t* houtoff_dev = nullptr;
    size_t hstats_cap = 0;
    int64_t* houtoff = nullptr;
    size_t houtoff_cap = 0;
    std::vector<hipEvent_t> stage_ev;  // stage-time events (TDA_FLAG_STAGE_TIMES)
    std::vector<hipEvent_t> stage_ev2; // ... on the side stream
    std::vector<hipEvent_t> stage_ev3; // ... on the third stream
    std::vector<hipEvent_t> stage_ev4; // ... on the fourth stream
    hipEvent_t evin = nullptr;         // caller's stream -> library stream
    char* hin = nullptr;               // pinned staging of host inputs (stable graph source)
    size_t hin_cap = 0;
    char* hdist = nullptr;             // pinned landing of the distance matrices (want_dist: f32, then f64)
    size_t hdist_cap = 0;
    void* xin = nullptr;  // gathered device input parts (ABI 6 x_parts)
    size_t xin_cap = 0;
    uint64_t gen = 0;                  // bumped whenever a buffer baked into graphs moves
    std::vector<struct GraphEntry> graphs;
    // the configuration a retry ended on (larger pools / another reducer), per
    // (N, maxdim, input kind): later calls of that shape start there instead of
    // failing the same way first
    struct Retry {
        int64_t N;
        int maxdim, input_kind;
        bool force_global, force_big;
        int no_par;
        int scale;
    };
    std::vector<Retry> retry;
    std::mutex mu;
};

// one captured launch sequence (everything between ev0 and ev1), replayed with
// a single hipGraphLaunch when the same plan, input address and flags recur
struct GraphKey {
    int64_t L, N, D;
    int maxdim, dtype, input_kind, x_on_device, flags, force_global, scale, force_big, variant, n_label_sets, sil_K, no_par, twonn, no_cap;
    float thresh, tn_eps, capf;
    double tn_discard;
    const void* x;
    uint64_t gen;
    bool operator==(const GraphKey& o) const { return std::memcmp(this, &o, sizeof(GraphKey)) == 0; }
};
struct GraphEntry {
    GraphKey key;
    hipGraphExec_t exec;
    hipGraph_t graph;  // kept as long as its exec (r06: see the capture below)
};

// records an event after each stage when stage timing is on
struct StageTimer {
    std::vector<hipEvent_t>& ev;
    hipStream_t s;
    bool on;
    std::vector<const char*> names;
    StageTimer* fwd = nullptr;  // serial stage timing: marks go to the main stream's timer
    hipError_t rec(hipEvent_t e) { return hipEventRecord(e, s); }
    int mark(const char* name) {
        if (fwd) return fwd->mark(name);
        if (!on) return 0;
        size_t i = names.size() + 1;
        while (ev.size() <= i) {
            hipEvent_t e;
            HIPC(hipEventCreate(&e));
            ev.push_back(e);
        }
        HIPC(rec(ev[i]));
        names.push_back(name);
        return 0;
    }
    int begin() {
        if (!on || fwd) return 0;
        while (ev.empty()) {
            hipEvent_t e;
            HIPC(hipEventCreate(&e));
            ev.push_back(e);
        }
        HIPC(rec(ev[0]));
        return 0;
    }
};

// ------------------------------------------------------------------ caller streams
// Device input is read after the work the caller queued on its stream.  A NULL
// handle is the null (legacy default) stream -- what torch's default stream is
// on ROCm (raw handle 0).  Before r05 NULL meant "no ordering": a tensor that a
// torch kernel had just written on the default stream (r04's torch.cat of the
// coalesced sweeps) could be read by the library's non-blocking stream before
// that kernel ran, i.e. as stale / uninitialised memory.
//
// Distinct HIP runtimes (libamdhip64 objects, by inode) mapped in the process.
// The torch wheel ships its own copy with the same soname, so the dynamic linker
// normally maps ONE of the two; a second one (a dlmopen'ed namespace,
// RTLD_DEEPBIND) would own streams this library's runtime cannot use.
int hip_runtimes_loaded() {
    struct Acc {
        dev_t dev[8];
        ino_t ino[8];
        int n;
    } acc{};
    dl_iterate_phdr(
        [](struct dl_phdr_info* info, size_t, void* data) -> int {
            auto* a = (Acc*)data;
            const char* nm = info->dlpi_name;
            const char* base = nm ? strrchr(nm, '/') : nullptr;
            base = base ? base + 1 : nm;
            if (!base || strncmp(base, "libamdhip64", 11) != 0) return 0;
            struct stat st;
            if (stat(nm, &st) != 0) return 0;
            for (int i = 0; i < a->n; ++i)
                if (a->dev[i] == st.st_dev && a->ino[i] == st.st_ino) return 0;
            if (a->n < 8) a->dev[a->n] = st.st_dev, a->ino[a->n] = st.st_ino, ++a->n;
            return 0;
        },
        &acc);
    return acc.n;
}

// Order `lib` after the caller's stream (NULL = the null stream) with `ev`.  A
// non-NULL handle must be a stream of THIS library's HIP runtime on `dev`:
// hipStreamGetDevice validates it against the runtime's own stream set, so a
// handle from another runtime, a destroyed stream or garbage is refused with
// TDA_E_HIP instead of being dereferenced by hipEventRecord.
int order_after_caller(hipStream_t lib, hipEvent_t ev, void* caller, int dev) {
    // counted once per process (dl_iterate_phdr + stat per call cost ~10 us).  With
    // a second runtime mapped, NULL would be THIS runtime's null stream, not the caller's default
    // stream, so neither a handle nor NULL orders anything: the caller must pass the input ready
    static const int n_rt = hip_runtimes_loaded();
    if (n_rt > 1)
        return fail(TDA_E_HIP, "two HIP runtimes are loaded in this process: the caller's stream (a handle or NULL) cannot "
                               "be ordered against (pass the input ready instead, TDA_FLAG_INPUT_READY)");
    if (caller) {
        hipDevice_t d = -1;
        const hipError_t e = hipStreamGetDevice((hipStream_t)caller, &d);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return fail(TDA_E_HIP, std::string("caller stream is not a stream of this library's HIP runtime: ") + hipGetErrorString(e));
        }
        if ((int)d != dev)
            return fail(TDA_E_INVALID, "caller stream is on device " + std::to_string((int)d) + ", the call on " + std::to_string(dev));
    }
    HIPC(hipEventRecord(ev, (hipStream_t)caller));
    HIPC(hipStreamWaitEvent(lib, ev, 0));
    return 0;
}

std::mutex g_ws_mu;
// Graph capture + instantiation AND every workspace (re)allocation / free, across
// all slots of the process.  r03 saw a host segfault inside the first calls of
// two slots that ran concurrently; the cause was not isolated then.  The HIP
// calls those first calls made at the same time were: hipFuncSetAttribute
// (one-time, now under g_attr_mu), stream capture + hipGraphInstantiate on
// the two slots' streams, and hipMalloc / hipHostMalloc of the workspaces --
// and on growth hipFree / hipHostFree / hipGraphExecDestroy.  ThreadLocal
// capture only restricts the CAPTURING thread, and HIP's hipFree synchronises
// the whole device (all streams, a capturing one included) while another
// thread captures; it is the one call whose contract does not cover running
// beside a capture.  So no (re)allocation, free or graph destruction runs
// while any slot captures: they take this lock too (first call / growth only;
// replays never take it).
std::mutex g_capture_mu;
// Graph launches: replays (and direct launches) share it; a capture with its instantiation and
// first launch holds it alone.  r06 (tools/concurrency_stress.py: 8 slots, calls of mixed shapes
// at once): a freshly instantiated graph's first hipGraphLaunch faulted inside the HIP runtime
// (a null dereference) while other slots replayed theirs; one slot at a time never did.
std::shared_mutex g_launch_mu;
std::vector<Workspace*> g_ws;

Workspace* get_ws(int dev, int slot) {
    std::lock_guard<std::mutex> g(g_ws_mu);
    for (auto* w : g_ws)
        if (w->device == dev && w->slot == slot) return w;
    auto* w = new Workspace();
    w->device = dev;
    w->slot = slot;
    g_ws.push_back(w);
    return w;
}

void drop_graphs(Workspace& w) {
    for (auto& g : w.graphs) {
        (void)hipGraphExecDestroy(g.exec);
        (void)hipGraphDestroy(g.graph);
    }
    w.graphs.clear();
    ++w.gen;
}

// ------------------------------------------------------------------ build consistency
// hipcc compiles this file twice (device pass, then host pass minutes later) and both read the
// headers; an edit in between once gave a library whose host side packed kernel arguments
// differently from what the device side read.  The first workspace of the
// process checks the sizes of every structure that crosses the host/device boundary, as the
// device code sees them, against the host's: a skewed build fails loudly instead of faulting.
#define TDA_LAYOUT_STRUCTS(X)                                                                                     \
    X(LayerStats) X(DimBufs) X(Pair) X(PairSet) X(OutPair) X(AppBlock) X(PartList) X(SortArgs) X(Reduce2Bufs)  \
    X(Reduce2Cfg) X(ReduceAllCfg) X(SmallBufs) X(BigBufs) X(DenseBufs) X(ParCtl) X(ParBufs) X(ParLds)
#define TDA_LAYOUT_COUNT(T) +1
constexpr int kLayoutN = 0 TDA_LAYOUT_STRUCTS(TDA_LAYOUT_COUNT);
__global__ void k_layout_probe(uint32_t* out) {
    if (threadIdx.x != 0) return;
    int i = 0;
#define TDA_LAYOUT_DEV(T) out[i++] = (uint32_t)sizeof(T);
    TDA_LAYOUT_STRUCTS(TDA_LAYOUT_DEV)
#undef TDA_LAYOUT_DEV
}
int check_layout(hipStream_t s) {
    static std::mutex mu;
    static bool done = false;
    std::lock_guard<std::mutex> g(mu);
    if (done) return 0;
    uint32_t* d = nullptr;
    uint32_t h[kLayoutN] = {};
    HIPC(hipMalloc(&d, sizeof(h)));
    hipLaunchKernelGGL(k_layout_probe, dim3(1), dim3(64), 0, s, d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(TDA_E_HIP, std::string("layout probe: ") + hipGetErrorString(e));
    static const char* names[kLayoutN] = {
#define TDA_LAYOUT_NAME(T) #T,
        TDA_LAYOUT_STRUCTS(TDA_LAYOUT_NAME)
#undef TDA_LAYOUT_NAME
    };
    const uint32_t host[kLayoutN] = {
#define TDA_LAYOUT_HOST(T) (uint32_t)sizeof(T),
        TDA_LAYOUT_STRUCTS(TDA_LAYOUT_HOST)
#undef TDA_LAYOUT_HOST
    };
    for (int i = 0; i < kLayoutN; ++i)
        if (h[i] != host[i])
            return fail(TDA_E_HIP, std::string("library build is inconsistent: sizeof(") + names[i] + ") is " + std::to_string(host[i]) +
                                       " on the host and " + std::to_string(h[i]) + " on the device (rebuild from one source tree)");
    done = true;
    return 0;
}

int ws_side_streams(Workspace& w) {
    if (w.stream2) return 0;
    HIPC(hipStreamCreateWithFlags(&w.stream2, hipStreamNonBlocking));
    HIPC(hipStreamCreateWithFlags(&w.stream3, hipStreamNonBlocking));
    HIPC(hipStreamCreateWithFlags(&w.stream4, hipStreamNonBlocking));
    return 0;
}

int ws_prepare(Workspace& w, const Plan& p) {
    if (!w.init) {
        // the side streams are created on the first multi-stream call (ws_side_streams):
        // a slot that only runs TDA_FLAG_ONE_STREAM calls holds one hardware queue
        HIPC(hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking));
        HIPC(hipEventCreateWithFlags(&w.evh, hipEventDisableTiming));
        HIPC(hipEventCreateWithFlags(&w.evs, hipEventDisableTiming));
        HIPC(hipEventCreateWithFlags(&w.evp, hipEventDisableTiming));
        HIPC(hipEventCreateWithFlags(&w.evsil, hipEventDisableTiming));
        HIPC(hipEventCreate(&w.ev0));
        HIPC(hipEventCreate(&w.ev1));
        HIPC(hipEventCreateWithFlags(&w.evf, hipEventDisableTiming));
        HIPC(hipEventCreateWithFlags(&w.evj, hipEventDisableTiming));
        HIPC(hipEventCreateWithFlags(&w.evin, hipEventDisableTiming));
        if (int rc = check_layout(w.stream)) return rc;
        w.init = true;
    }
    if (w.dcap < p.total) {
        drop_graphs(w);
        w.piv2_dirty = true;
        if (w.dbuf) HIPC(hipFree(w.dbuf));
        w.dbuf = nullptr;
        size_t cap = std::max<size_t>(p.total, w.dcap + w.dcap / 2);
        if (hipMalloc(&w.dbuf, cap) != hipSuccess) {
            (void)hipGetLastError();
            size_t fr = 0, tot = 0;
            (void)hipMemGetInfo(&fr, &tot);
            w.dbuf = nullptr;
            w.dcap = 0;
            return fail(TDA_E_HIP, "device workspace of " + std::to_string(cap >> 20) + " MiB does not fit (free " +
                                       std::to_string(fr >> 20) + " of " + std::to_string(tot >> 20) + " MiB)");
        }
        w.dcap = cap;
    }
    if (w.hstats_cap < (size_t)p.L) {
        drop_graphs(w);
        if (w.hstats) HIPC(hipHostFree(w.hstats));
        HIPC(hipHostMalloc((void**)&w.hstats, sizeof(LayerStats) * p.L, hipHostMallocMapped));
        HIPC(hipHostGetDevicePointer((void**)&w.hstats_dev, w.hstats, 0));
        w.hstats_cap = p.L;
    }
    if (w.houtoff_cap < (size_t)p.L * 4) {
        drop_graphs(w);
        if (w.houtoff) HIPC(hipHostFree(w.houtoff));
        HIPC(hipHostMalloc((void**)&w.houtoff, sizeof(int64_t) * p.L * 4, hipHostMallocMapped));
        HIPC(hipHostGetDevicePointer((void**)&w.houtoff_dev, w.houtoff, 0));
        w.houtoff_cap = p.L * 4;
    }
    size_t want = std::max<size_t>(1 << 16, (size_t)p.L * 256);
    if (w.hout_cap < want) {
        drop_graphs(w);
        if (w.hout) HIPC(hipHostFree(w.hout));
        HIPC(hipHostMalloc((void**)&w.hout, sizeof(OutPair) * want, hipHostMallocMapped));
        HIPC(hipHostGetDevicePointer((void**)&w.hout_dev, w.hout, 0));
        w.hout_cap = want;
    }
    return 0;
}

int grow_hout(Workspace& w, size_t need) {
    drop_graphs(w);
    if (w.hout) HIPC(hipHostFree(w.hout));
    w.hout = nullptr;
    size_t cap = std::max(need, 2 * w.hout_cap);
    HIPC(hipHostMalloc((void**)&w.hout, sizeof(OutPair) * cap, hipHostMallocMapped));
    HIPC(hipHostGetDevicePointer((void**)&w.hout_dev, w.hout, 0));
    w.hout_cap = cap;
    return 0;
}

bool g_attr_done[64] = {false};
std::mutex g_attr_mu;
int set_lds_attrs(int dev) {
    std::lock_guard<std::mutex> lk(g_attr_mu);  // first calls on several workspace slots at once
    if (dev < 64 && g_attr_done[dev]) return 0;
    HIPC(hipFuncSetAttribute((const void*)k_h0<0, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
    HIPC(hipFuncSetAttribute((const void*)k_h0<kH0BorWQ, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
    HIPC(hipFuncSetAttribute((const void*)k_h0<kH0WaveQ, true>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
    HIPC(hipFuncSetAttribute((const void*)k_bor_hook, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
    HIPC(hipFuncSetAttribute((const void*)k_sort_resid, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
    HIPC(hipFuncSetAttribute((const void*)k_emit, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kEmitLds));
#define TDA_ATTR_RED(LW, P1, P2) \
    HIPC(hipFuncSetAttribute((const void*)k_reduce_all<LW, P1, P2>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax))
    TDA_ATTR_RED(true, true, true);
    TDA_ATTR_RED(true, true, false);
    TDA_ATTR_RED(true, false, false);
    TDA_ATTR_RED(false, true, true);
    TDA_ATTR_RED(false, true, false);
    TDA_ATTR_RED(false, false, false);
#undef TDA_ATTR_RED
    HIPC(hipFuncSetAttribute((const void*)k_reduce_par<1, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(ParLds)));
    HIPC(hipFuncSetAttribute((const void*)k_reduce_par<1, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(ParLds)));
    HIPC(hipFuncSetAttribute((const void*)k_reduce_par<2, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(ParLds)));
    HIPC(hipFuncSetAttribute((const void*)k_reduce_par<2, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(ParLds)));
    HIPC(hipFuncSetAttribute((const void*)k_reduce_par<2, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(ParLds)));

    HIPC(hipFuncSetAttribute((const void*)k_h2_phase1, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
    HIPC(hipFuncSetAttribute((const void*)k_edge_chunks, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kEdgeSortLds));
    HIPC(hipFuncSetAttribute((const void*)k_silhouette, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
    HIPC(hipFuncSetAttribute((const void*)k_twonn, hipFuncAttributeMaxDynamicSharedMemorySize, 8192 * 4));
#define TDA_ATTR_CHAIN(K, F) HIPC(hipFuncSetAttribute((const void*)k_h1_chain<K, F>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
    TDA_ATTR_CHAIN(1, 0) TDA_ATTR_CHAIN(2, 0) TDA_ATTR_CHAIN(3, 0) TDA_ATTR_CHAIN(4, 0) TDA_ATTR_CHAIN(6, 0)
    TDA_ATTR_CHAIN(9, 0) TDA_ATTR_CHAIN(12, 0) TDA_ATTR_CHAIN(16, 0) TDA_ATTR_CHAIN(21, 0)
    TDA_ATTR_CHAIN(1, 1) TDA_ATTR_CHAIN(2, 1) TDA_ATTR_CHAIN(3, 1) TDA_ATTR_CHAIN(4, 1) TDA_ATTR_CHAIN(6, 1)
    TDA_ATTR_CHAIN(9, 1) TDA_ATTR_CHAIN(12, 1)
    TDA_ATTR_CHAIN(1, 2) TDA_ATTR_CHAIN(2, 2) TDA_ATTR_CHAIN(3, 2) TDA_ATTR_CHAIN(4, 2) TDA_ATTR_CHAIN(6, 2)
    TDA_ATTR_CHAIN(9, 2) TDA_ATTR_CHAIN(12, 2)
#undef TDA_ATTR_CHAIN
    HIPC(hipFuncSetAttribute((const void*)k_prep_edges, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
    HIPC(hipFuncSetAttribute((const void*)k_prep_tables, hipFuncAttributeMaxDynamicSharedMemorySize, (int)prep_tables_lds(kDenseMaxN)));
    HIPC(hipFuncSetAttribute((const void*)k_reduce_h2_finish, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
    HIPC(hipFuncSetAttribute((const void*)k_apparent<1, false>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
    HIPC(hipFuncSetAttribute((const void*)k_apparent<2, false>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
    HIPC(hipFuncSetAttribute((const void*)k_apparent<1, true>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
    HIPC(hipFuncSetAttribute((const void*)k_apparent<2, true>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax));
    if (dev < 64) g_attr_done[dev] = true;
    return 0;
}

// result owned by the library
// The per-(layer, dim) arrays are one allocation, in the order count,
// offset, checksum, n_all_pairs, n_columns, n_residual, n_adds; birth/death
// and birth_idx/death_idx are each one allocation too (tda_rips.h).
struct ResultImpl {
    tda_rips_result pub;
    std::vector<uint64_t> blob;  // meta | num_edges | birth_idx, death_idx | thresh (padded) | birth, death
    std::vector<float> dist, stage_ms, tn;
    std::vector<double> dist64;
    std::vector<double> sil;
    std::vector<const char*> stage_name;
};

std::string err_flags(int e) {
    std::string s;
    if (e & ERR_RESID_CAP) s += " residual-column-capacity";
    if (e & ERR_PAIR_CAP) s += " pair-capacity";
    if (e & ERR_WORK_CAP) s += " working-column-capacity";
    if (e & ERR_VPOOL_CAP) s += " reduction-pool-capacity";
    if (e & ERR_OUT_CAP) s += " output-capacity";
    if (e & ERR_STEP_LIMIT) s += " reduction-step-limit";
    if (e & ERR_PAR2) s += " parallel-h2-reduction-abort";
    if (e & ERR_PAR) s += " parallel-reduction-abort";
    return s;
}

// ------------------------------------------------------------------ pipeline
// (re)point the public result at its one-allocation blob (tda_rips.h layout)
void point_result(ResultImpl& R, size_t total) {
    tda_rips_result& o = R.pub;
    const size_t S = (size_t)o.L * (o.maxdim + 1);
    const size_t o_ne = 7 * S, o_idx = o_ne + o.L, o_thr = o_idx + 2 * total, o_bd = o_thr + (o.L + 1) / 2;
    int64_t* m = (int64_t*)R.blob.data();
    o.count = m;
    o.offset = m + S;
    o.checksum = (const uint64_t*)(m + 2 * S);
    o.n_all_pairs = m + 3 * S;
    o.n_columns = m + 4 * S;
    o.n_residual = m + 5 * S;
    o.n_adds = m + 6 * S;
    o.num_edges = (const int64_t*)(R.blob.data() + o_ne);
    o.birth_idx = (const int64_t*)(R.blob.data() + o_idx);
    o.death_idx = o.birth_idx + total;
    o.thresh = (const float*)(R.blob.data() + o_thr);
    o.birth = (const float*)(R.blob.data() + o_bd);
    o.death = o.birth + total;
    o.blob = R.blob.data();
    o.blob_bytes = (int64_t)(R.blob.size() * 8);
    o.n_pairs = (int64_t)total;
}

// Layers ls[i] of R replaced by the one-layer results subs[i] (same N and maxdim): every
// per-layer block of the blob is rebuilt in layer order.  Distances, silhouettes and TwoNN
// stay R's (they do not depend on the reduction).
void splice_layers(ResultImpl& R, const std::vector<int>& ls, const std::vector<tda_rips_result*>& subs) {
    const tda_rips_result& o = R.pub;
    const int L = (int)o.L, nd = (int)o.maxdim + 1;
    std::vector<const tda_rips_result*> src((size_t)L, &o);
    std::vector<int> sl((size_t)L);
    for (int l = 0; l < L; ++l) sl[l] = l;
    for (size_t i = 0; i < ls.size(); ++i) src[ls[i]] = subs[i], sl[ls[i]] = 0;
    size_t total = 0;
    for (int l = 0; l < L; ++l)
        for (int d = 0; d < nd; ++d) total += (size_t)src[l]->count[sl[l] * nd + d];
    const size_t S = (size_t)L * nd;
    const size_t o_ne = 7 * S, o_idx = o_ne + L, o_thr = o_idx + 2 * total, o_bd = o_thr + (L + 1) / 2;
    std::vector<uint64_t> blob(o_bd + total, 0);
    int64_t* m = (int64_t*)blob.data();
    float* thr = (float*)(blob.data() + o_thr);
    int64_t* ne = (int64_t*)(blob.data() + o_ne);
    int64_t* idx = (int64_t*)(blob.data() + o_idx);
    float* bd = (float*)(blob.data() + o_bd);
    size_t e = 0;
    for (int l = 0; l < L; ++l) {
        const tda_rips_result& q = *src[l];
        const int k = sl[l];
        thr[l] = q.thresh[k];
        ne[l] = q.num_edges[k];
        for (int d = 0; d < nd; ++d) {
            const size_t a = (size_t)l * nd + d, b = (size_t)k * nd + d;
            const int64_t c = q.count[b];
            m[a] = c;
            m[S + a] = (int64_t)e;
            ((uint64_t*)m)[2 * S + a] = q.checksum[b];
            m[3 * S + a] = q.n_all_pairs[b];
            m[4 * S + a] = q.n_columns[b];
            m[5 * S + a] = q.n_residual[b];
            m[6 * S + a] = q.n_adds[b];
            const int64_t f = q.offset[b];
            for (int64_t i = 0; i < c; ++i, ++e) {
                bd[e] = q.birth[f + i];
                bd[total + e] = q.death[f + i];
                idx[e] = q.birth_idx[f + i];
                idx[total + e] = q.death_idx[f + i];
            }
        }
    }
    R.blob.swap(blob);
    point_result(R, total);
}

int run_pipeline(const tda_rips_args& a, int input_kind, const void* host_or_dev, tda_rips_result** out,
                 bool force_global, int scale, bool force_big, int no_par, bool no_cap);

// Column caps missed on some layers (ERR_CAP_MISS: a column's pivot lies above its cap -- a
// class that lives longer than capf * thresh, e.g. the one loop of a circle): each such layer is
// re-run ALONE without caps and spliced into the batch's result; the other layers keep their
// capped (exact) reductions.  A one-layer call simply re-runs without caps.
int rerun_cap_missed(const tda_rips_args& a, int input_kind, const void* host_or_dev, tda_rips_result** out, ResultImpl* R,
                     const std::vector<int>& ls, bool force_global, int scale, bool force_big, int no_par) {
    std::unique_ptr<ResultImpl> own(R);
    if (getenv("TDA_DEBUG")) fprintf(stderr, "[tda] column cap missed on %zu of %lld layers: re-run without caps\n", ls.size(), (long long)a.L);
    if (a.L == 1 || input_kind == 2) {
        const double dms = R->pub.device_ms;
        if (int rc = run_pipeline(a, input_kind, host_or_dev, out, force_global, scale, force_big, no_par, true)) return rc;
        (*out)->n_cap_reruns = a.L;
        (*out)->device_ms += dms;
        return 0;
    }
    const size_t esz = a.dtype == TDA_F64 ? 8 : 4;
    const size_t lb = (size_t)a.N * (input_kind == 1 ? (size_t)a.N : (size_t)a.D) * esz;  // bytes per layer
    const int64_t per = a.n_parts > 0 ? a.L / a.n_parts : a.L;
    std::vector<tda_rips_result*> subs;
    struct Free {
        std::vector<tda_rips_result*>& v;
        ~Free() {
            for (auto* r : v) delete reinterpret_cast<ResultImpl*>(r);
        }
    } free_subs{subs};
    double dms = R->pub.device_ms;
    for (int l : ls) {
        tda_rips_args b = a;
        const char* base = (const char*)(a.n_parts > 0 ? a.x_parts[l / per] : host_or_dev);
        b.x = base + (size_t)(a.n_parts > 0 ? l % per : l) * lb;
        b.L = 1;
        b.n_parts = 0;
        b.x_parts = nullptr;
        b.flags = (a.flags | TDA_FLAG_INPUT_READY) & ~TDA_FLAG_DIST64;  // the batch's call ordered and read it already
        b.want_dist = 0;
        b.labels = nullptr;
        b.n_label_sets = 0;
        b.want_twonn = 0;
        tda_rips_result* sub = nullptr;
        if (int rc = run_pipeline(b, input_kind, b.x, &sub, force_global, scale, force_big, no_par, true)) return rc;
        subs.push_back(sub);
        dms += sub->device_ms;
    }
    splice_layers(*R, ls, subs);
    R->pub.n_cap_reruns = (int64_t)ls.size();
    R->pub.device_ms = dms;
    *out = &own.release()->pub;
    return 0;
}

// input_kind: 0 = points (dtype), 1 = square distance (dtype), 2 = condensed f32
// no_cap: k_reduce_par without column caps (a capped column ran empty below its cap: code 81)
int run_pipeline(const tda_rips_args& a, int input_kind, const void* host_or_dev, tda_rips_result** out,
                 bool force_global, int scale, bool force_big, int no_par, bool no_cap) {
    const auto h_entry = std::chrono::steady_clock::now();
    Plan p;
    p.L = a.L;
    p.N = a.N;
    p.D = a.D;
    p.maxdim = a.maxdim;
    p.dtype = a.dtype;
    p.is_dist = input_kind != 0;
    p.want64 = input_kind == 0 && a.dtype == TDA_F64 && a.want_dist && (a.flags & TDA_FLAG_DIST64);
    make_plan(p, force_global, scale, force_big, no_par);
    const int dev = a.device;
    HIPC(hipSetDevice(dev));
    Workspace& w = *get_ws(dev, a.slot);
    std::unique_lock<std::mutex> guard(w.mu);  // released before any retry (which re-enters)
    // allocations, frees and graph drops (first call / growth) never overlap another slot's
    // capture: g_capture_mu is held from here through the buffer growth below, and released
    // before the input copies (the host-input memcpy serialised pipelined slots)
    std::unique_lock<std::mutex> rt_lock(g_capture_mu);
    if (int rc = ws_prepare(w, p)) return rc;
    if (int rc = set_lds_attrs(dev)) return rc;
    // all work runs on the library stream, ordered after the caller's stream
    hipStream_t s = w.stream;
    char* B = w.dbuf;
    const int n = (int)p.N, L = (int)p.L;
    float* dist = (float*)(B + p.o_dist);
    LayerStats* stats = (LayerStats*)(B + p.o_stats);
    const size_t esz = p.dtype == TDA_F64 ? 8 : 4;
    PairSet ps = {};
    for (int d = 0; d <= p.maxdim; ++d) {
        ps.p[d] = (Pair*)(B + p.o_pairs[d]);
        ps.cap[d] = p.pcap[d];
    }

    // host inputs go through a pinned staging buffer: a stable graph source
    // (grown here, filled after the lock is released)
    const void* xsrc = host_or_dev;
    const int nparts = input_kind == 2 ? 0 : a.n_parts;
    const bool host_in = !a.x_on_device || input_kind == 2;
    const bool dev_parts = !host_in && nparts > 0;
    const size_t xbytes = input_kind == 2 ? binom((uint64_t)n, 2) * 4
                                          : (size_t)L * n * (input_kind == 1 ? (size_t)n : (size_t)p.D) * esz;
    // want_dist: the matrices come back by an async copy queued behind the call's work (one
    // stream sync for both; r06: a blocking hipMemcpy after the sync cost ~20 us per small call)
    const size_t dbytes = a.want_dist ? (size_t)L * n * n * (4 + (p.want64 ? 8 : 0)) : 0;
    if (dbytes > w.hdist_cap) {
        if (w.hdist) HIPC(hipHostFree(w.hdist));
        w.hdist = nullptr;
        w.hdist_cap = 0;
        HIPC(hipHostMalloc((void**)&w.hdist, std::max<size_t>(dbytes, 1 << 16), hipHostMallocDefault));
        w.hdist_cap = std::max<size_t>(dbytes, 1 << 16);
    }
    if (host_in) {
        if (w.hin_cap < xbytes) {
            drop_graphs(w);
            if (w.hin) HIPC(hipHostFree(w.hin));
            w.hin = nullptr;
            HIPC(hipHostMalloc((void**)&w.hin, std::max<size_t>(xbytes, 1 << 16), hipHostMallocDefault));
            w.hin_cap = std::max<size_t>(xbytes, 1 << 16);
        }
        xsrc = w.hin;
    } else if (dev_parts) {
        if (w.xin_cap < xbytes) {
            drop_graphs(w);
            if (w.xin) HIPC(hipFree(w.xin));
            w.xin = nullptr;
            HIPC(hipMalloc(&w.xin, xbytes));
            w.xin_cap = xbytes;
        }
        xsrc = w.xin;
    }

    // silhouette labels -> host-mapped buffer (stable address: a graph source)
    const int nls = (a.labels && a.n_label_sets > 0) ? (int)a.n_label_sets : 0;
    int sil_K = 0;
    size_t sil_out_off = 0;
    if (nls) {
        for (int q = 0; q < nls; ++q) {
            int K = 0;
            std::vector<int> f(kSilMaxK, 0);
            for (int i = 0; i < n; ++i) {
                const int32_t c = a.labels[(size_t)q * n + i];
                if (c < 0 || c >= kSilMaxK) return fail(TDA_E_INVALID, "silhouette labels must be codes 0..K-1 with K <= 32");
                ++f[c];
                K = std::max(K, c + 1);
            }
            for (int c = 0; c < K; ++c)
                if (!f[c]) return fail(TDA_E_INVALID, "silhouette labels must be contiguous codes 0..K-1 (LabelEncoder)");
            if (K < 2 || K > n - 1)
                return fail(TDA_E_INVALID, "Number of labels is " + std::to_string(K) + ". Valid values are 2 to n_samples - 1 (inclusive)");
            sil_K = std::max(sil_K, K);
        }
        sil_out_off = align_up((size_t)nls * n * 4, 16);
        const size_t need = sil_out_off + (size_t)L * nls * 8;
        if (w.hsil_cap < need) {
            drop_graphs(w);
            if (w.hsil) HIPC(hipHostFree(w.hsil));
            w.hsil = nullptr;
            HIPC(hipHostMalloc((void**)&w.hsil, std::max<size_t>(need, 1 << 12), hipHostMallocMapped));
            HIPC(hipHostGetDevicePointer((void**)&w.hsil_dev, w.hsil, 0));
            w.hsil_cap = std::max<size_t>(need, 1 << 12);
        }
    }

    // TwoNN estimates -> host-mapped buffer (stable address: a graph source)
    const bool want_tn = a.want_twonn != 0;
    const bool no_ph = (a.flags & TDA_FLAG_NO_PERSISTENCE) != 0;  // distances + side metrics only
    if (want_tn && w.htn_cap < (size_t)L) {
        drop_graphs(w);
        if (w.htn) HIPC(hipHostFree(w.htn));
        w.htn = nullptr;
        HIPC(hipHostMalloc((void**)&w.htn, sizeof(float) * std::max(L, 64), hipHostMallocMapped));
        HIPC(hipHostGetDevicePointer((void**)&w.htn_dev, w.htn, 0));
        w.htn_cap = std::max(L, 64);
    }

    // TDA_FLAG_STAGE_SERIAL (with stage times) or TDA_FLAG_ONE_STREAM: every
    // stage on the main stream -- each pair of stage events then brackets one
    // kernel only, and a slot keeps to one hardware queue (several slots in
    // flight each get their own: SweepPipeline)
    const bool serial_stages = ((a.flags & TDA_FLAG_STAGE_TIMES) && (a.flags & TDA_FLAG_STAGE_SERIAL)) || (a.flags & TDA_FLAG_ONE_STREAM);
    if (!serial_stages)
        if (int rc = ws_side_streams(w)) return rc;

    rt_lock.unlock();  // buffers are in place; the capture below re-takes it

    // input copies and ordering, outside the lock
    if (a.x_on_device && input_kind != 2 && !(a.flags & TDA_FLAG_INPUT_READY))
        if (int rc = order_after_caller(s, w.evin, a.stream, dev)) return rc;
    if (host_in) {
        if (nparts > 0) {  // parts: one after the other into the staging buffer
            const size_t pb = xbytes / nparts;
            for (int i = 0; i < nparts; ++i) std::memcpy((char*)w.hin + i * pb, a.x_parts[i], pb);
        } else if (xbytes) {
            std::memcpy(w.hin, host_or_dev, xbytes);
        }
    } else if (dev_parts) {
        // device parts: gathered into the workspace's own input buffer by one kernel on the
        // library stream (ordered after the caller's stream above, outside any captured graph)
        PartList pl = {};
        for (int i = 0; i < nparts; ++i) pl.p[i] = a.x_parts[i];
        const uint64_t words = xbytes / nparts / 4;
        const unsigned gx = (unsigned)std::min<uint64_t>(64, (words + 255) / 256);
        hipLaunchKernelGGL(k_gather_parts, dim3(std::max(1u, gx), nparts), dim3(256), 0, s, pl, words, (uint32_t*)w.xin);
        HIPC(hipGetLastError());
    }
    if (nls) std::memcpy(w.hsil, a.labels, (size_t)nls * n * 4);

    // serial_stages: the side streams are aliased to the main one here and restored on return
    struct StreamSwap {
        Workspace& w;
        hipStream_t s2, s3, s4;
        bool on;
        ~StreamSwap() {
            if (on) w.stream2 = s2, w.stream3 = s3, w.stream4 = s4;
        }
    } swap_guard{w, w.stream2, w.stream3, w.stream4, serial_stages};
    if (serial_stages) w.stream2 = w.stream3 = w.stream4 = s;
    StageTimer tm{w.stage_ev, s, (a.flags & TDA_FLAG_STAGE_TIMES) != 0, {}};
    StageTimer tm2{w.stage_ev2, w.stream2, tm.on, {}};
    StageTimer tm3{w.stage_ev3, w.stream3, tm.on, {}};
    StageTimer tm4{w.stage_ev4, w.stream4, tm.on, {}};
    if (serial_stages) tm2.fwd = tm3.fwd = tm4.fwd = &tm;
    // D >= 32 (raw activations): Gram tiles on the FP64 matrix cores; TDA_DIST=scalar|mfma forces one (tests)
    const bool dist_mfma = input_kind == 0 && (test_env_is("TDA_DIST", "mfma") || (p.D >= kDistMfmaMinD && !test_env_is("TDA_DIST", "scalar")));
    GraphKey gk;
    std::memset(&gk, 0, sizeof(gk));
    gk.L = p.L;
    gk.N = p.N;
    gk.D = p.D;
    gk.maxdim = p.maxdim;
    gk.dtype = p.dtype;
    gk.input_kind = input_kind;
    gk.x_on_device = a.x_on_device;
    gk.flags = a.flags;
    gk.force_global = force_global;
    gk.scale = scale;
    gk.force_big = force_big;
    gk.no_par = no_par;
    gk.no_cap = no_cap;
    // column caps only with ripser's default threshold (the enclosing radius: no essential
    // H1 / H2 class); a finite user threshold can leave classes essential (k_reduce_par)
    // caps also off when H2 runs on the serial k_reduce_big after a parallel H1 (TDA_PAR2=0, or an H2
    // abort): that kernel reads every layer's H1 pivots, so no layer's H1 may be left unfinished
    const bool h2_serial = p.par && p.maxdim >= 2 && !p.par2;
    const float capf = (no_cap || h2_serial || !(std::isinf(a.thresh) || a.thresh == 3.402823466e+38f)) ? 0.0f : par_capf();
    gk.capf = capf;
    gk.variant = (p.dense ? 1 : 0) | (p.big ? 2 : 0) | (p.fast ? 4 : 0) | (p.lds_mode ? 8 : 0) | (p.cmode << 4) | (p.par ? 1 << 8 : 0) | (dist_mfma ? 1 << 9 : 0) |
                 (p.wide ? 1 << 10 : 0) | (p.want64 ? 1 << 11 : 0) | (p.par2 ? 1 << 12 : 0) | (p.piv2_sparse ? 1 << 13 : 0);
    gk.thresh = a.thresh;
    gk.n_label_sets = nls;
    gk.sil_K = sil_K;  // baked into the k_silhouette launch (argument K and its LDS size)
    gk.twonn = want_tn;
    gk.tn_discard = want_tn ? a.twonn_discard : 0.0;
    gk.tn_eps = want_tn ? a.twonn_eps : 0.0f;
    gk.x = xsrc;
    gk.gen = w.gen;
    GraphEntry* ge = nullptr;
    // stage-timed calls run eagerly: timing events inside a capture need
    // external event nodes, which torch's bundled HIP runtime rejects
    const bool use_graph = !test_env_is("TDA_GRAPH", "0") && !tm.on;
    if (use_graph)
        for (auto& g : w.graphs)
            if (g.key == gk) ge = &g;
    const bool capture = use_graph && !ge;
    // ev0 / ev1 bracket the whole sequence; a graph replay records them around the launch
    auto rec_t = [&](hipEvent_t e) { return capture ? hipSuccess : hipEventRecord(e, s); };
#define MARK(name) \
    do {           \
        if (int rc_ = tm.mark(name)) return rc_; \
    } while (0)
    auto enqueue = [&]() -> int {
    HIPC(rec_t(w.ev0));
    if (int rc = tm.begin()) return rc;
    MARK("event_gap");  // an empty interval: what two back-to-back events measure with no kernel between (bench.py subtracts it)
    HIPC(hipMemsetAsync(B + p.memset_lo, 0, p.memset_hi - p.memset_lo, s));
    MARK("memset");

    // ---- distances (+ row maxima for the enclosing radius)
    uint32_t* rowmax = (uint32_t*)(B + p.o_rowmax);
    if (input_kind == 0) {
        const void* x = xsrc;
        if (!a.x_on_device) {
            HIPC(hipMemcpyAsync(B + p.o_x, x, (size_t)L * n * p.D * esz, hipMemcpyHostToDevice, s));
            x = B + p.o_x;
        }
        dim3 grid((n + 15) / 16, (n + 15) / 16, L);
        const bool mfma = dist_mfma;
        const unsigned nt = (unsigned)((n + kDmT - 1) / kDmT);
        double* gpart = (double*)(B + p.o_gpart);
        double* npart = (double*)(B + p.o_npart);
        double* d64 = p.want64 ? (double*)(B + p.o_d64) : nullptr;
        const dim3 gsplit(nt * (nt + 1) / 2, L, (unsigned)p.dsplit);
        const dim3 gcomb((unsigned)std::min<uint64_t>(1024, ((uint64_t)n * n + 255) / 256), L);
        if (mfma && p.dsplit > 1 && p.dtype == TDA_F64) {
            hipLaunchKernelGGL((k_distance_mfma<double, 0, true>), gsplit, dim3(256), 0, s, (const double*)x, n, (int)p.D, dist, rowmax,
                               gpart, npart, (double*)nullptr);
            hipLaunchKernelGGL((k_distance_combine<double, 0>), gcomb, dim3(256), 0, s, gpart, npart, p.dsplit, n, dist, rowmax, d64);
            hipLaunchKernelGGL(k_rowmax, dim3((n + 3) / 4, L), dim3(256), 0, s, dist, n, rowmax);
        } else if (mfma && (p.dsplit > 1 || p.gram_layer)) {
            if (p.gram_layer)
                hipLaunchKernelGGL(k_gram_layer, dim3((unsigned)p.dsplit, L), dim3(256), 0, s, (const float*)x, n, (int)p.D, gpart, npart);
            else
                hipLaunchKernelGGL((k_distance_mfma<float, 0, true>), gsplit, dim3(256), 0, s, (const float*)x, n, (int)p.D, dist, rowmax,
                                   gpart, npart);
            MARK(p.gram_layer ? "k_gram_layer" : "k_distance_mfma");  // the Gram kernel alone (bench roofline): combine, row maxima: own stages
            hipLaunchKernelGGL((k_distance_combine<float, 0>), gcomb, dim3(256), 0, s, gpart, npart, p.dsplit, n, dist, rowmax);
            MARK("k_distance_combine");
            hipLaunchKernelGGL(k_rowmax, dim3((n + 3) / 4, L), dim3(256), 0, s, dist, n, rowmax);
        } else if (mfma && p.dtype == TDA_F64)
            hipLaunchKernelGGL((k_distance_mfma<double>), dim3(nt * (nt + 1) / 2, L), dim3(256), 0, s, (const double*)x, n, (int)p.D,
                               dist, rowmax, (double*)nullptr, (double*)nullptr, d64);
        else if (mfma)
            hipLaunchKernelGGL((k_distance_mfma<float>), dim3(nt * (nt + 1) / 2, L), dim3(256), 0, s, (const float*)x, n, (int)p.D,
                               dist, rowmax, (double*)nullptr, (double*)nullptr);
        else if (p.dtype == TDA_F64)
            hipLaunchKernelGGL(k_distance<double>, grid, dim3(256), 0, s, (const double*)x, n, (int)p.D, dist, rowmax, d64);
        else
            hipLaunchKernelGGL(k_distance<float>, grid, dim3(256), 0, s, (const float*)x, n, (int)p.D, dist, rowmax);
    } else {
        const void* x = xsrc;
        unsigned gx = (unsigned)std::min<uint64_t>(1024, ((uint64_t)n * n + 255) / 256);
        if (input_kind == 1) {
            if (!a.x_on_device) {
                HIPC(hipMemcpyAsync(B + p.o_x, x, (size_t)L * n * n * esz, hipMemcpyHostToDevice, s));
                x = B + p.o_x;
            }
            if (p.dtype == TDA_F64)
                hipLaunchKernelGGL(k_square_dist<double>, dim3(gx, L), dim3(256), 0, s, (const double*)x, n, dist);
            else
                hipLaunchKernelGGL(k_square_dist<float>, dim3(gx, L), dim3(256), 0, s, (const float*)x, n, dist);
        } else {
            const uint64_t ne = binom((uint64_t)n, 2);
            if (ne) HIPC(hipMemcpyAsync(B + p.o_x, x, ne * 4, hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(k_square_from_condensed, dim3(gx), dim3(256), 0, s, (const float*)(B + p.o_x), n, dist);
        }
        HIPC(hipGetLastError());
        hipLaunchKernelGGL(k_rowmax, dim3((n + 3) / 4, L), dim3(256), 0, s, dist, n, rowmax);
    }
    HIPC(hipGetLastError());
    MARK(input_kind != 0 ? "k_square_dist" : dist_mfma ? ((p.dsplit > 1 || p.gram_layer) && p.dtype == TDA_F32 ? "k_rowmax" : "k_distance_mfma") : "k_distance");
    HIPC(hipEventRecord(w.evf, s));  // fork point of the side streams

    DenseBufs dnb = {};

    // ---- H0 on its own stream: it overlaps the apparent-pair kernels, which
    // do not need the spanning forest (a forest edge is an H0 death, never an
    // apparent column; the reductions skip forest edges among the residuals).
    // The triangle ranks of the dense H1 chain go on a second side stream.
    // Enqueued after apparent<1>, so the critical path's kernels are queued first.
    auto launch_side = [&]() -> int {
        hipStream_t s2 = w.stream2, s4 = w.stream4;
        HIPC(hipStreamWaitEvent(s2, w.evf, 0));
        HIPC(hipStreamWaitEvent(s4, w.evf, 0));
        if (int rc = tm2.begin()) return rc;
        if (int rc = tm4.begin()) return rc;
        if (no_ph) {
            // TDA_FLAG_NO_PERSISTENCE: no spanning forest, no H0 pairs
        } else if (n <= kSmallN) {
            hipLaunchKernelGGL(k_h0_wave, dim3(L), dim3(64), 64 * 64 * 4 + 64 * 4 + 64 * 8, s4, dist, n, rowmax, a.thresh, stats,
                               (uint32_t*)(B + p.o_mst), p.mst_words, (Pair*)(B + p.o_pairs[0]), p.pcap[0]);
        } else {
            int T = n <= 256 ? 256 : 1024;
            if (n <= kH0WaveMaxN && !test_env_is("TDA_H0_WAVE", "0")) T = 1024;  // LDS Borůvka: a wave per vertex
            // best | par | red | sort chunk | (LDS rows) | Borůvka hooks
            size_t base = 16 + (size_t)n * 8 + (size_t)((n + 1) & ~1) * 4 + 40 * 8 + (size_t)n * 4;
            base = align_up(base, 16);
            // n <= kH0WaveMaxN: one-wave Prim on the LDS-staged matrix (sort chunk just covers the forest)
            const bool wave_ok = !test_env_is("TDA_H0_WAVE", "0");
            const bool dlds = n <= kH0WaveMaxN && wave_ok;
            size_t avail = kLdsMax - base - (dlds ? (size_t)4 * n * n : 0);
            uint64_t ch = 1;
            if (dlds)
                ch = next_pow2((uint64_t)n);
            else
                while (ch * 2 * 8 <= avail && ch * 2 <= 16384) ch *= 2;
            size_t lds = base + ch * 8 + (dlds ? (size_t)4 * n * n : 0);
            if (dlds) {
                hipLaunchKernelGGL((k_h0<kH0WaveQ, true>), dim3(L), dim3(T), lds, s4, dist, n, a.thresh, stats, (uint32_t*)(B + p.o_mst),
                                   p.mst_words, (Pair*)(B + p.o_pairs[0]), p.pcap[0], (uint64_t*)(B + p.o_h0s), ilog2(ch),
                                   (const BorCtl*)nullptr);
            } else {  // Borůvka over the whole GPU: ceil(log2 N) rounds of (cheapest edges, hooking)
                int32_t* bcomp = (int32_t*)(B + p.o_bcomp);
                uint64_t* bcheap = (uint64_t*)(B + p.o_bcheap);
                BorCtl* bctl = (BorCtl*)(B + p.o_bctl);
                hipLaunchKernelGGL(k_bor_init, dim3(L), dim3(256), 0, s4, rowmax, n, a.thresh, stats, bcomp, bcheap, bctl);
                const size_t hl = (size_t)((n + 3) & ~3) * 8 + (size_t)n * 8;
                const int rounds = std::max(1, ilog2(next_pow2((uint64_t)n)));
                for (int r = 0; r < rounds; ++r) {
                    hipLaunchKernelGGL(k_bor_min, dim3((unsigned)((n + 3) / 4), L), dim3(256), 0, s4, dist, n, stats, bcomp, bcheap, bctl,
                                       r == 0 ? 1 : 0);
                    if (r == 0)
                        if (int rc = tm4.mark("k_bor_min")) return rc;
                    hipLaunchKernelGGL(k_bor_hook, dim3(L), dim3(1024), hl, s4, n, bcomp, bcheap, bctl, (uint64_t*)(B + p.o_h0s));
                    if (r == 0)
                        if (int rc = tm4.mark("k_bor_hook")) return rc;
                }
                HIPC(hipGetLastError());
                if (int rc = tm4.mark("k_bor_rounds")) return rc;
                // elder rule: one wave with register labels up to N = 64 * kH0BorWQ, thread 0 above
                if (n <= 64 * kH0BorWQ)
                    hipLaunchKernelGGL((k_h0<kH0BorWQ, false, true>), dim3(L), dim3(T), lds, s4, dist, n, a.thresh, stats,
                                       (uint32_t*)(B + p.o_mst), p.mst_words, (Pair*)(B + p.o_pairs[0]), p.pcap[0], (uint64_t*)(B + p.o_h0s),
                                       ilog2(ch), (const BorCtl*)bctl);
                else
                    hipLaunchKernelGGL((k_h0<0, false, true>), dim3(L), dim3(T), lds, s4, dist, n, a.thresh, stats, (uint32_t*)(B + p.o_mst),
                                       p.mst_words, (Pair*)(B + p.o_pairs[0]), p.pcap[0], (uint64_t*)(B + p.o_h0s), ilog2(ch),
                                       (const BorCtl*)bctl);
            }
        }
        HIPC(hipGetLastError());
        if (!no_ph)
            if (int rc = tm4.mark("k_h0")) return rc;
        HIPC(hipEventRecord(w.evh, s4));
        if (nls) {  // silhouette scores on the same distance matrices (sklearn semantics), after the H0 join
            const size_t lds = (size_t)sil_K * kSilT * 8 + (size_t)n * 4;
            hipLaunchKernelGGL(k_silhouette, dim3(L, nls), dim3(kSilT), lds, s4, dist, n, (const int32_t*)w.hsil_dev, sil_K,
                               (double*)(w.hsil_dev + sil_out_off));
            HIPC(hipGetLastError());
            if (int rc = tm4.mark("k_silhouette")) return rc;
        }
        if (want_tn) {  // TwoNN intrinsic dimension on the same distance matrices
            // beside H0 on the ranks stream when there are no ranks (the raw-activation sweeps:
            // H0 and TwoNN only read the distances; r03 raw4096: they ran back to back on s4)
            // (only without H1: with H1 the main stream joins s2 before the reduction, and
            // TwoNN there would sit on the critical path -- ADVICE r03)
            const bool tn_s2 = !p.dense && p.maxdim == 0;
            const int pw2 = (int)next_pow2((uint64_t)std::max(n, 64));
            hipLaunchKernelGGL(k_twonn, dim3(L), dim3(kTnT), (size_t)pw2 * 4, tn_s2 ? s2 : s4, dist, n, a.twonn_discard, a.twonn_eps, pw2,
                               w.htn_dev);
            HIPC(hipGetLastError());
            if (int rc = (tn_s2 ? tm2 : tm4).mark("k_twonn")) return rc;
        }
        if (nls || want_tn) HIPC(hipEventRecord(w.evsil, s4));
        if (p.dense) {  // triangle ranks for the dense H1 chain, off the critical path
            dnb.recs = (EdgeRec*)(B + p.o_recs);
            dnb.cls = (uint32_t*)(B + p.o_cls);
            dnb.res1 = (uint32_t*)(B + p.o_res1);
            dnb.inv32 = (uint32_t*)(B + p.o_inv32);
            dnb.rank_of = (uint16_t*)(B + p.o_rof);
            dnb.tri_stride = p.tri_stride;
            dnb.cls2 = (uint16_t*)(B + p.o_cls2);
            dnb.n2p = p.n2p;
            dnb.inv = (uint16_t*)(B + p.o_inv);
            dnb.E = (uint32_t)binom((uint64_t)n, 2);
            dnb.inv_stride = p.inv_stride;
            dnb.K = p.dK;
            dnb.epos = (uint32_t*)(B + p.o_epos);
            dnb.cobt = (uint16_t*)(B + p.o_cobt);
            dnb.cob_stride = p.cob_stride;
            dnb.eM = (uint64_t*)(B + p.o_eM);
            dnb.necnt = (uint32_t*)(B + p.o_necnt);
            const dim3 pg((unsigned)L, (unsigned)((dnb.E + kPrepEdges - 1) / kPrepEdges + 1));  // + the rank-sort block
            hipLaunchKernelGGL(k_prep_edges, pg, dim3(kPrepT), p.prep_lds, s2, dist, n, rowmax, a.thresh, dnb, p.cmode, stats);
            HIPC(hipGetLastError());
            if (int rc = tm2.mark("k_prep_edges")) return rc;
            // blocks per layer: 8 up to 64 layers (sweep48, 32 layers: 27 -> 18 us), 4 above (256 layers:
            // 83 us with 4, 96 with 8 -- the per-block staging and scan then cost more than the spread saves)
            const int ptb = test_env("TDA_PREP_TAB_BLOCKS") ? std::max(1, atoi(test_env("TDA_PREP_TAB_BLOCKS")))
                                                           : (L <= 64 ? 2 * kPrepTabBlocks : kPrepTabBlocks);
            hipLaunchKernelGGL(k_prep_tables, dim3(L, ptb), dim3(kPrepTabT), prep_tables_lds(n), s2, dist, n, dnb, p.cmode, stats);
            HIPC(hipGetLastError());
            if (int rc = tm2.mark("k_prep_tables")) return rc;
        }
        HIPC(hipEventRecord(w.evj, s2));
        return 0;
    };

    // ---- H1 .. Hmaxdim: apparent pairs (parallel), residual sort, serial reduction
    DimBufs db[3] = {};
    for (int d = 1; d <= p.maxdim; ++d) {
        db[d].cleared = d == 1 ? nullptr : (const uint32_t*)(B + p.o_piv[d - 1]);
        db[d].cleared_words = d == 1 ? 0 : p.piv_words[d - 1];
        db[d].pivbits = (uint32_t*)(B + p.o_piv[d]);
        db[d].piv_words = p.piv_words[d];
        db[d].resid = (uint64_t*)(B + p.o_resid[d]);
        db[d].rcap = p.rcap[d];
        db[d].ncand = p.ncand[d];
        db[d].clr = d == 2 && p.piv2_sparse ? (uint64_t*)(B + p.o_clr2) : nullptr;
        db[d].clr_cap = d == 2 && p.piv2_sparse ? p.clr_cap : 0;
    }
    // N <= 64 with H2: the H2 columns (apparent<2>, their sort, phase 1) run
    // on a third stream beside the H1 chain; they only need apparent<1>'s
    // pivot bitmap, and the chain records its residual pivots separately
    const bool split2 = p.dense && p.maxdim >= 2;
    auto launch_apparent = [&](int d, hipStream_t st, uint64_t total_override = 0) {
        uint64_t blocks = (p.ncand[d] + 255) / 256;
        // total blocks over all layers: measured (r01, sweep48) 1024 beats 4096,
        // whose grid holds every CU while the critical small kernels wait; off
        // the dense path the apparent kernels run alone: 4096 (r02, grid144:
        // apparent<2> 1.08 -> 0.87 ms; staging the 83-KB matrix in LDS: 2.25 ms)
        const char* app_env = test_env("TDA_APP_GRID");
        const uint64_t app_total = app_env ? strtoull(app_env, nullptr, 10) : total_override ? total_override : (p.dense ? 1024 : 4096);
        unsigned gx = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(blocks, std::max<uint64_t>(1, app_total / L)));
        const int app_lds_max = test_env("TDA_APP_LDS_MAXN") ? atoi(test_env("TDA_APP_LDS_MAXN")) : kAppLdsMaxN;
        const bool dl = n <= app_lds_max && 16 + (size_t)n * n * 4 <= (size_t)kLdsMax;
        const size_t alds = 16 + (dl ? (size_t)n * n * 4 : 0);
        // N <= 64: the small-N pass (32-bit decode, 4 vertices per LDS read); TDA_APP_SMALL=0 -> k_apparent
        if (n <= 64 && dl && !test_env_is("TDA_APP_SMALL", "0")) {
            // the pivot bitmap copied in LDS when it fits and a block's simplices outnumber a quarter
            // of its words (every block flushes the whole copy): r06, 160 layers per call,
            // apparent<1> 24.7 -> 19.3 us, apparent<2> 73.7 -> 57.0 us; at 32 layers per call (540
            // triangles per block) the flushes cost more than the atomics saved: call 0.171 -> 0.177 ms.
            // TDA_APP_PIV_LDS=0 / 1: never / always.
            const uint64_t per_block = (p.ncand[d] + gx - 1) / gx;
            const bool pl_fit = db[d].piv_words * 4 <= kSmallPivLdsMax;
            const bool pl_on = test_env_is("TDA_APP_PIV_LDS", "1") ? pl_fit
                               : test_env_is("TDA_APP_PIV_LDS", "0") ? false
                                                                    : pl_fit && per_block * 4 >= db[d].piv_words;
            const uint32_t pl_words = pl_on ? (uint32_t)db[d].piv_words : 0u;
            const size_t slds = 16 + small_piv_offset(n) + 4ull * pl_words;
            if (d == 1)
                hipLaunchKernelGGL((k_apparent_small<1>), dim3(gx, L), dim3(256), slds, st, dist, n, stats, db[d], rowmax, a.thresh, pl_words);
            else
                hipLaunchKernelGGL((k_apparent_small<2>), dim3(gx, L), dim3(256), slds, st, dist, n, stats, db[d], rowmax, a.thresh, pl_words);
        } else {
            // L a multiple of 8: a 1-D grid whose blocks take their layers XCD by XCD (app_block)
            const int xl = (L % 8 == 0 && !test_env_is("TDA_APP_XCD", "0")) ? L : 0;
            const dim3 ag = xl ? dim3(gx * (unsigned)L) : dim3(gx, L);
            // H1 above the LDS-matrix range: 16 x 16 edge tiles over LDS-staged v-tiles (TDA_APP_TILE=0: one edge per thread)
            const bool tiled = d == 1 && !dl && !test_env_is("TDA_APP_TILE", "0");
            if (tiled) {
                const uint64_t nt = ((uint64_t)n + kAppTS - 1) / kAppTS, tiles = nt * (nt + 1) / 2;
                const unsigned tx = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(tiles, std::max<uint64_t>(1, app_total / L)));
                const dim3 tg = xl ? dim3(tx * (unsigned)L) : dim3(tx, L);
                hipLaunchKernelGGL(k_apparent_tile, tg, dim3(256), 0, st, dist, n, stats, db[d], rowmax, a.thresh, xl);
            } else if (d == 1 && dl)
                hipLaunchKernelGGL((k_apparent<1, true>), ag, dim3(256), alds, st, dist, n, stats, db[d], rowmax, a.thresh, xl);
            else if (d == 1)
                hipLaunchKernelGGL((k_apparent<1, false>), ag, dim3(256), alds, st, dist, n, stats, db[d], rowmax, a.thresh, xl);
            else if (dl)
                hipLaunchKernelGGL((k_apparent<2, true>), ag, dim3(256), alds, st, dist, n, stats, db[d], rowmax, a.thresh, xl);
            else
                hipLaunchKernelGGL((k_apparent<2, false>), ag, dim3(256), alds, st, dist, n, stats, db[d], rowmax, a.thresh, xl);
        }
    };
    Reduce2Bufs rb;
    rb.rmap_keys = (uint64_t*)(B + p.o_rmk);
    rb.rmap_vals = (uint32_t*)(B + p.o_rmv);
    rb.rmap_stride = p.rmap_stride;
    rb.roff = (uint64_t*)(B + p.o_voff);
    rb.rlen = (uint32_t*)(B + p.o_vlen);
    rb.rpool = (uint64_t*)(B + p.o_vpool);
    rb.rpool_cap = p.vpool_cap;
    rb.wtmp = (uint64_t*)(B + p.o_wt);
    rb.wtmp_stride = 2 * (p.lds_mode ? 8192 : p.wcap_g);
    rb.wlog = (uint64_t*)(B + p.o_wk);
    rb.windex = (uint64_t*)(B + p.o_wl);
    rb.wfill = (uint32_t*)(B + p.o_wp);
    rb.wcap = p.wcap_g;
    rb.mst = (const uint32_t*)(B + p.o_mst);
    rb.mst_words = p.mst_words;
    SortArgs sa = {};
    for (int d = 1; d <= p.maxdim; ++d) {
        sa.resid[d] = db[d].resid;
        sa.rcap[d] = db[d].rcap;
    }
    auto launch_sort = [&](int d0, int nd, hipStream_t st, uint64_t max_chunk = 16384) {
        // LDS chunk: the largest residual list of these dims, at most max_chunk keys
        uint64_t cap = 64;
        for (int d = d0; d < d0 + nd; ++d) cap = std::max<uint64_t>(cap, std::min<uint64_t>(next_pow2(p.rcap[d]), max_chunk));
        hipLaunchKernelGGL(k_sort_resid, dim3(L, nd), dim3(1024), cap * 8, st, stats, sa, (uint64_t*)(B + p.o_tmp), p.max_rcap,
                           rb.rmap_keys, rb.rmap_stride, ilog2(cap), d0);
    };
    SmallBufs sb = {};
    if (p.dense) {
        sb.p1_next = (uint32_t*)(B + p.o_p1next);
        sb.p1_key = (uint64_t*)(B + p.o_p1k);
        sb.p1_info = (uint32_t*)(B + p.o_p1i);
        sb.p1_pidx = (uint32_t*)(B + p.o_p1x);
        sb.roff2 = (uint64_t*)(B + p.o_roff2);
        sb.rlen2 = (uint32_t*)(B + p.o_rlen2);
        sb.rpool2 = (uint64_t*)(B + p.o_rpool2);
        sb.rpool2_cap = p.vpool_cap;
        sb.p1_used = (unsigned long long*)(B + p.o_p1used);
        sb.p1_wcap = kP1WCap;
    }
    // H2 phase 1 (its early exits read the chain's residual H1 pivots as they
    // appear); in the one-stream timing mode it runs right after the chain,
    // so it sees what it sees when it runs beside it
    auto launch_phase1 = [&](hipStream_t st) -> int {
        // blocks per layer: each holds ~46 KB of LDS (one wave), so the whole grid is occupancy-bound:
        // ~1 K blocks over all layers (r04, sweep48 serial stage: L = 32: 96 -> 32 blocks 35 -> 28 us;
        // L = 128: 96 -> 16 blocks 108 -> 73 us); small batches keep up to kP1Grid
        const int p1g = test_env("TDA_P1_GRID") ? std::max(1, atoi(test_env("TDA_P1_GRID")))
                                                : std::min(kP1Grid, std::max(16, 1024 / std::max(1, L)));
        hipLaunchKernelGGL(k_h2_phase1, dim3(L, (p1g + p.p1_waves - 1) / p.p1_waves), dim3(64 * p.p1_waves), p.p1_lds, st, dist, n, stats, db[2], sb, (const uint16_t*)dnb.cls2,
                           p.n2p, p.bm_words, (const uint32_t*)dnb.res1, (uint32_t)p.piv_words[1], step_limit());
        HIPC(hipGetLastError());
        if (int rc = (st == s ? tm : tm3).mark("k_h2_phase1")) return rc;
        HIPC(hipEventRecord(w.evp, st));
        return 0;
    };
    // capture order of the launches (the graph executor dispatches in it):
    // TDA_ORDER=0 apparent<1> first; 1 side streams first; 2 side streams
    // first and the H2 branch after the triangle ranks; 3 side streams first,
    // sort<1> enqueued before the H2 branch; 5 (N <= 64 with H2) as 3, with
    // apparent<1> at the head of the H2 branch's stream: sweep48 0.182 ->
    // 0.175 ms device, L = 4 0.136 -> 0.131 ms (replayed graph; eager slower)
    // 5 up to 64 layers per call; 3 above (sweep48x4, 128 layers: 0.42 vs 0.48 ms with 5)
    // r04 (after the §6.4-6.5 kernel changes, graph replay, one call at a time): L = 32 order 2 0.167 ms
    // device vs 0.174 with 5; L = 4 order 5 0.124 ms vs 0.138 with 2
    const int order = test_env("TDA_ORDER") ? atoi(test_env("TDA_ORDER")) : (L <= 16 ? 5 : L <= 64 ? 2 : 3);
    if (p.maxdim < 1 || order >= 1)
        if (int rc = launch_side()) return rc;
    const bool h2_side = !p.dense && p.par && p.par2 && p.maxdim >= 2;
    // the H2 branch forks once k_reduce_par<1> is about to start (after k_par_init), not after
    // apparent<1>: launched together with the H1 prerequisites, the GPU-filling apparent<2> pass
    // slowed them (torus2048_h2 trace: sort<1> 0.06 -> 7 ms, the edge chunk sort 0.5 -> 15 ms, the
    // H1 reduction starting at 26.6 ms); after k_par_init it fills the CUs the H1 workers leave.
    // The wide edge codes (H2 keys only) move onto the branch too.  TDA_H2_LATE=0: the r04 fork.
    const bool h2_late = h2_side && !test_env_is("TDA_H2_LATE", "0");
    // A k_reduce_par worker fills a CU (two 256-VGPR waves per SIMD), so apparent<2> blocks
    // dispatched before the H1 workers keep them off every CU they hold (torus2048_h2: the H1
    // reduction 124 -> 154 ms); on a small grid the pass itself crawls (128 blocks: 30 -> 194 ms).
    // The branch starts after a short device-side delay instead, so the H1 workers are resident
    // first and apparent<2> fills the CUs they leave as the column queue drains.
    const uint64_t h2_late_grid = test_env("TDA_H2_LATE_GRID") ? strtoull(test_env("TDA_H2_LATE_GRID"), nullptr, 10) : 0;
    const uint32_t h2_late_delay_us = test_env("TDA_H2_LATE_DELAY") ? (uint32_t)atoi(test_env("TDA_H2_LATE_DELAY")) : 50;
    auto launch_h2_columns = [&]() -> int {  // apparent<2> + their sort on the third stream
        if (int rc = tm3.begin()) return rc;
        launch_apparent(2, w.stream3, h2_late ? h2_late_grid : 0);
        HIPC(hipGetLastError());
        if (int rc = tm3.mark("k_apparent<2>")) return rc;
        // beside k_reduce_par<1> (one 72-KB workgroup per CU) the sort's LDS chunk must fit next to
        // it: 4096 keys (32 KB); a 128-KB chunk waited for the H1 reduction (grid144: 0.85 ms)
        launch_sort(2, 1, w.stream3, h2_side ? 4096 : 16384);
        HIPC(hipGetLastError());
        if (int rc = tm3.mark("k_sort_resid<2>")) return rc;
        return 0;
    };
    Pair* const pairs1 = (Pair*)(B + p.o_pairs[1]);
    Pair* const pairs2 = p.maxdim >= 2 ? (Pair*)(B + p.o_pairs[2]) : pairs1;
    auto launch_chain = [&](hipStream_t st) -> int {  // dense H1 (N <= 64): one k_h1_chain instantiation per (words, mode)
        switch (p.dK * 3 + p.cmode) {
#define TDA_CHAIN(K, F)                                                                                                          \
    case K * 3 + F:                                                                                                              \
        hipLaunchKernelGGL((k_h1_chain<K, F>), dim3(L), dim3(kChainT), p.chain_lds, st, dist, n, stats, db[1], rb, dnb, step_limit(), \
                           pairs1, p.pcap[1]);                                                                                   \
        break;
            TDA_CHAIN(1, 0) TDA_CHAIN(2, 0) TDA_CHAIN(3, 0) TDA_CHAIN(4, 0) TDA_CHAIN(6, 0) TDA_CHAIN(9, 0) TDA_CHAIN(12, 0)
            TDA_CHAIN(16, 0) TDA_CHAIN(21, 0)
            TDA_CHAIN(1, 1) TDA_CHAIN(2, 1) TDA_CHAIN(3, 1) TDA_CHAIN(4, 1) TDA_CHAIN(6, 1) TDA_CHAIN(9, 1) TDA_CHAIN(12, 1)
            TDA_CHAIN(1, 2) TDA_CHAIN(2, 2) TDA_CHAIN(3, 2) TDA_CHAIN(4, 2) TDA_CHAIN(6, 2) TDA_CHAIN(9, 2) TDA_CHAIN(12, 2)
#undef TDA_CHAIN
            default:
                return fail(TDA_E_INVALID, "no k_h1_chain instantiation for this N");
        }
        HIPC(hipGetLastError());
        return 0;
    };
    auto launch_h2_finish = [&](hipStream_t st) -> int {
        hipLaunchKernelGGL(k_reduce_h2_finish, dim3(L), dim3(64), p.rcfg.bytes, st, dist, n, stats, db[1], db[2], rb, p.rcfg, sb,
                           (const uint32_t*)dnb.res1, pairs2, p.pcap[2]);
        HIPC(hipGetLastError());
        return 0;
    };
    // order 5 (N <= 64, H0-H2): apparent<1> opens the H2 branch's stream (its pivot
    // bitmap is apparent<2>'s clearing test), so the branch runs on one queue up to
    // phase 1; the main stream picks up apparent<1>'s residuals for sort<1> and the chain
    const bool app1_side = split2 && order == 5 && !serial_stages;
    if (p.maxdim >= 1 && app1_side) {
        HIPC(hipStreamWaitEvent(w.stream3, w.evf, 0));
        if (int rc = tm3.begin()) return rc;
        launch_apparent(1, w.stream3);
        HIPC(hipGetLastError());
        if (int rc = tm3.mark("k_apparent<1>")) return rc;
        HIPC(hipEventRecord(w.evs, w.stream3));
        launch_apparent(2, w.stream3);
        HIPC(hipGetLastError());
        if (int rc = tm3.mark("k_apparent<2>")) return rc;
        launch_sort(2, 1, w.stream3, 16384);
        HIPC(hipGetLastError());
        if (int rc = tm3.mark("k_sort_resid<2>")) return rc;
        HIPC(hipStreamWaitEvent(w.stream3, w.evj, 0));  // edge classes (k_prep_*)
        if (int rc = launch_phase1(w.stream3)) return rc;
        HIPC(hipStreamWaitEvent(s, w.evs, 0));
        launch_sort(1, 1, s);
        HIPC(hipGetLastError());
        MARK("k_sort_resid<1>");
    }
    if (p.maxdim >= 1) {
        if (!app1_side) {
            launch_apparent(1, s);
            HIPC(hipGetLastError());
            MARK("k_apparent<1>");
        }
        if (order == 0)
            if (int rc = launch_side()) return rc;
        if (app1_side) {
            // enqueued above
        } else if (split2) {
            HIPC(hipEventRecord(w.evs, s));
            if (order == 3) {
                launch_sort(1, 1, s);
                HIPC(hipGetLastError());
                MARK("k_sort_resid<1>");
            }
            HIPC(hipStreamWaitEvent(w.stream3, w.evs, 0));
            if (order == 2) HIPC(hipStreamWaitEvent(w.stream3, w.evj, 0));
            if (int rc = launch_h2_columns()) return rc;
            HIPC(hipStreamWaitEvent(w.stream3, w.evj, 0));  // edge classes (k_prep_*)
            if (!serial_stages)
                if (int rc = launch_phase1(w.stream3)) return rc;
            if (order != 3) {
                launch_sort(1, 1, s);
                HIPC(hipGetLastError());
                MARK("k_sort_resid<1>");
            }
        } else if (h2_side && h2_late) {
            // (fork after k_par_init below)
            launch_sort(1, 1, s);
            HIPC(hipGetLastError());
            MARK("k_sort_resid<1>");
        } else if (h2_side) {
            // parallel H1 and H2: the H2 columns' apparent pass and sort run on
            // the third stream beside the H1 reduction (k_reduce_par<2> joins
            // them).  k_par_emit<1> may OR residual H1 pivots into the bitmap
            // k_apparent<2> reads as its clearing test while it runs: a triangle
            // seen cleared is skipped there, otherwise it becomes a residual
            // column that k_reduce_par<2> skips -- never an apparent pair (a
            // cleared triangle is an H1 death, and apparent pairs are
            // persistence pairs), so pairs and checksums do not depend on the race.
            HIPC(hipEventRecord(w.evs, s));
            HIPC(hipStreamWaitEvent(w.stream3, w.evs, 0));
            if (int rc = launch_h2_columns()) return rc;
            HIPC(hipEventRecord(w.evp, w.stream3));
            launch_sort(1, 1, s);
            HIPC(hipGetLastError());
            MARK("k_sort_resid<1>");
        } else {
            for (int d = 2; d <= p.maxdim; ++d) {
                launch_apparent(d, s);
                HIPC(hipGetLastError());
                MARK("k_apparent<2>");
            }
            launch_sort(1, p.maxdim, s);
            HIPC(hipGetLastError());
            MARK("k_sort_resid");
        }
        if (p.serial_tables) {
            HIPC(hipMemsetAsync(rb.windex, 0, (size_t)L * p.wcap_g * 2 * 8, s));
            HIPC(hipMemsetAsync(rb.wfill, 0, (size_t)L * p.wcap_g / 4 * 4, s));
        }
        HIPC(hipStreamWaitEvent(s, w.evh, 0));  // join: forest edges (clearing of H1 columns)
        HIPC(hipStreamWaitEvent(s, w.evj, 0));  // join: triangle ranks
        MARK("wait:join");  // keeps the side streams' time out of the next kernel's stage
        const bool p1 = n <= 1024, p2 = n <= 256;
        const ReduceAllCfg& rc = p.rcfg;
#define TDA_LAUNCH_RED(LW, P1, P2)                                                                                        \
    hipLaunchKernelGGL((k_reduce_all<LW, P1, P2>), dim3(L), dim3(64), rc.bytes, s, dist, n, p.maxdim, stats, db[1], db[2], rb, rc, \
                       pairs1, pairs2, p.pcap[1], p.maxdim >= 2 ? p.pcap[2] : 0)
        if (p.dense) {
            if (int rc = launch_chain(s)) return rc;
            MARK("k_h1_chain");
            if (p.maxdim >= 2) {
                if (serial_stages)
                    if (int rc = launch_phase1(s)) return rc;
                HIPC(hipStreamWaitEvent(s, w.evp, 0));  // phase-1 results
                MARK("wait:phase1");
                if (int rc = launch_h2_finish(s)) return rc;
                MARK("k_reduce_h2_finish");
            }
        } else if (p.big) {
            BigBufs gb;
            gb.log = rb.wlog;
            gb.index = rb.windex;
            gb.fill = rb.wfill;
            gb.bref = (uint32_t*)(B + p.o_bref);
            gb.cap = p.wcap_g;
            gb.bcap = p.wcap_g;
            gb.step_limit = step_limit();
            gb.wide = p.wide ? 1 : 0;
            gb.dcode = (const uint32_t*)(B + p.o_dcode);
            gb.dsort = (const uint64_t*)(B + p.o_dsort);
            gb.ecap = p.ecap;
            // edge codes of the wide H2 keys (thresholds are known: after the H0 join)
            auto launch_edge_codes = [&](hipStream_t es, StageTimer& et) -> int {
                // the sorted lengths end in dsort: with an odd number of merge passes the keys start in dtmp
                const uint64_t E = binom((uint64_t)n, 2), CH = 1ull << kEdgeSortLog2;
                int passes = 0;
                for (uint64_t w = CH; w < E; w <<= 1) ++passes;
                uint64_t* ka = (uint64_t*)(B + ((passes & 1) ? p.o_dtmp : p.o_dsort));
                uint64_t* kb = (uint64_t*)(B + ((passes & 1) ? p.o_dsort : p.o_dtmp));
                const unsigned gk = (unsigned)std::min<uint64_t>(1024, ((uint64_t)n * n + 255) / 256);
                hipLaunchKernelGGL(k_edge_keys, dim3(gk, L), dim3(256), 0, es, dist, n, ka, p.ecap);
                hipLaunchKernelGGL(k_edge_chunks, dim3((unsigned)((E + CH - 1) / CH), L), dim3(1024), kEdgeSortLds, es, ka, E, p.ecap);
                for (uint64_t w = CH; w < E; w <<= 1) {
                    hipLaunchKernelGGL(k_edge_merge, dim3((unsigned)((E + kMergeSeg - 1) / kMergeSeg), L), dim3(256), 0, es, ka, kb, E,
                                       p.ecap, w);
                    std::swap(ka, kb);
                }
                HIPC(hipGetLastError());
                if (int rc = et.mark("k_edge_sort")) return rc;
                const unsigned gx = (unsigned)std::min<uint64_t>(1024, ((uint64_t)n * n + 255) / 256);
                hipLaunchKernelGGL(k_edge_codes, dim3(gx, L), dim3(256), 0, es, dist, n, stats, (const uint64_t*)(B + p.o_dsort), p.ecap,
                                   (uint32_t*)(B + p.o_dcode));
                HIPC(hipGetLastError());
                return et.mark("k_edge_codes");
            };
            if (p.wide && !h2_late)
                if (int rc = launch_edge_codes(s, tm)) return rc;
            int start_dim = 1;
            if (p.par) {
                ParBufs pb;
                pb.ctl = (ParCtl*)(B + p.o_pctl);
                pb.item_base = (uint64_t*)(B + p.o_pitem);
                pb.okey = (uint64_t*)(B + p.o_pokey);
                pb.oval = (uint64_t*)(B + p.o_poval);
                pb.ostride = p.ostride;
                pb.colpiv = (uint64_t*)(B + p.o_colpiv);
                pb.rec = (uint64_t*)(B + p.o_prec);
                pb.rec_cap = p.rec_cap;
                pb.rpool = (uint64_t*)(B + p.o_prpool);
                pb.rpool_cap = p.rpool_cap;
                pb.bpool = (uint64_t*)(B + p.o_pbpool);
                pb.bpool_cap = p.bpool_cap;
                pb.rq = (uint64_t*)(B + p.o_prq);
                pb.rq_cap = p.rq_cap;
                pb.step_limit = step_limit();
                pb.capf = capf;
                pb.dbg = p.o_pdbg ? (uint64_t*)(B + p.o_pdbg) : nullptr;  // profile builds only
                HIPC(hipMemsetAsync(pb.rq, 0, p.rq_cap * 8, s));
                hipLaunchKernelGGL(k_par_init, dim3(64, L), dim3(256), 0, s, stats, L, p.rcap[1], pb, 1);
                HIPC(hipGetLastError());
                MARK("k_par_init");
                if (h2_late) {  // the H2 branch (and the wide edge codes) beside the H1 reduction
                    HIPC(hipEventRecord(w.evs, s));
                    HIPC(hipStreamWaitEvent(w.stream3, w.evs, 0));
                    if (h2_late_delay_us && !serial_stages)
                        hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, w.stream3, h2_late_delay_us);
                    if (int rc = launch_h2_columns()) return rc;
                    if (p.wide)
                        if (int rc = launch_edge_codes(w.stream3, tm3)) return rc;
                    HIPC(hipEventRecord(w.evp, w.stream3));
                }
                // persistent workers (one 71-KB-LDS workgroup per CU by default); the surplus exits at once
                const unsigned par_grid = par_grid_size();
                const uint32_t* no_clr = nullptr;
                if (p.packed)
                    hipLaunchKernelGGL((k_reduce_par<1, true>), dim3(par_grid), dim3(kParT), sizeof(ParLds), s, dist, n, L, stats, db[1], no_clr,
                                       (uint64_t)0, rb, pb, gb.dcode, gb.dsort, gb.ecap);
                else
                    hipLaunchKernelGGL((k_reduce_par<1, false>), dim3(par_grid), dim3(kParT), sizeof(ParLds), s, dist, n, L, stats, db[1], no_clr,
                                       (uint64_t)0, rb, pb, gb.dcode, gb.dsort, gb.ecap);
                HIPC(hipGetLastError());
                MARK("k_reduce_par");
                // H2 next: residual H1 pivots into the dim-1 bitmap (k_reduce_par<2>) or map (k_reduce_big)
                hipLaunchKernelGGL(k_par_emit<1>, dim3(L), dim3(1024), 0, s, stats, db[1], rb, pb, pairs1, p.pcap[1],
                                   p.maxdim < 2 ? 0 : p.par2 ? 2 : 1, (const uint64_t*)nullptr, (uint64_t)0);
                HIPC(hipGetLastError());
                MARK("k_par_emit");
                start_dim = 2;
                if (p.par2) {  // H2 columns on the same workers (an H1 abort skips it: k_par_init keeps the flag)
                    if (h2_side) HIPC(hipStreamWaitEvent(s, w.evp, 0));  // join: H2 columns (third stream)
                    HIPC(hipMemsetAsync(pb.rq, 0, p.rq_cap * 8, s));
                    hipLaunchKernelGGL(k_par_init, dim3(64, L), dim3(256), 0, s, stats, L, p.rcap[2], pb, 2);
                    HIPC(hipGetLastError());
                    if (p.wide)  // N > 568: edge-code keys (k_edge_codes ran above)
                        hipLaunchKernelGGL((k_reduce_par<2, false, true>), dim3(par_grid), dim3(kParT), sizeof(ParLds), s, dist, n, L, stats,
                                           db[2], (const uint32_t*)db[1].pivbits, db[1].piv_words, rb, pb, gb.dcode, gb.dsort, gb.ecap);
                    else if (n <= kPar2PackedMaxN)
                        hipLaunchKernelGGL((k_reduce_par<2, true>), dim3(par_grid), dim3(kParT), sizeof(ParLds), s, dist, n, L, stats, db[2],
                                           (const uint32_t*)db[1].pivbits, db[1].piv_words, rb, pb, gb.dcode, gb.dsort, gb.ecap);
                    else
                        hipLaunchKernelGGL((k_reduce_par<2, false>), dim3(par_grid), dim3(kParT), sizeof(ParLds), s, dist, n, L, stats, db[2],
                                           (const uint32_t*)db[1].pivbits, db[1].piv_words, rb, pb, gb.dcode, gb.dsort, gb.ecap);
                    HIPC(hipGetLastError());
                    MARK("k_reduce_par<2>");
                    hipLaunchKernelGGL(k_par_emit<2>, dim3(L), dim3(1024), 0, s, stats, db[2], rb, pb, pairs2, p.pcap[2], 0,
                                       p.wide ? gb.dsort : (const uint64_t*)nullptr, p.ecap);
                    HIPC(hipGetLastError());
                    MARK("k_par_emit<2>");
                    start_dim = 3;
                }
            }
            if (start_dim <= p.maxdim)
                hipLaunchKernelGGL(k_reduce_big, dim3(L), dim3(kBigT), 0, s, dist, n, p.maxdim, stats, db[1], db[2], rb, gb, pairs1,
                                   pairs2, p.pcap[1], p.maxdim >= 2 ? p.pcap[2] : 0, start_dim);
        } else if (p.lds_mode) {
            if (p2) TDA_LAUNCH_RED(true, true, true); else if (p1) TDA_LAUNCH_RED(true, true, false); else TDA_LAUNCH_RED(true, false, false);
        } else {
            if (p2) TDA_LAUNCH_RED(false, true, true); else if (p1) TDA_LAUNCH_RED(false, true, false); else TDA_LAUNCH_RED(false, false, false);
        }
#undef TDA_LAUNCH_RED
        HIPC(hipGetLastError());
        if (!p.dense && !(p.par && (p.maxdim < 2 || p.par2))) MARK(p.big ? "k_reduce_big" : "k_reduce_all");
    } else {
        HIPC(hipStreamWaitEvent(s, w.evh, 0));
        HIPC(hipStreamWaitEvent(s, w.evj, 0));
    }

    if (nls || want_tn) HIPC(hipStreamWaitEvent(s, w.evsil, 0));  // join: silhouette scores, TwoNN on s4
    if (want_tn) HIPC(hipStreamWaitEvent(s, w.evj, 0));          // join: TwoNN on s2
    // ---- emission order, straight into host-mapped memory
    hipLaunchKernelGGL(k_emit, dim3(L), dim3(1024), kEmitLds, s, stats, L, p.maxdim, ps, (uint64_t*)(B + p.o_fk),
                       (uint32_t*)(B + p.o_fv), p.sstride, w.houtoff_dev, w.hout_dev, (uint64_t)w.hout_cap, w.hstats_dev);
    HIPC(hipGetLastError());
    MARK("k_emit");
    if (p.piv2_sparse) {  // the H2 pivot bitmap back to zero: only the words this call set
        hipLaunchKernelGGL(k_clear_words, dim3(1024, L), dim3(256), 0, s, stats, (const uint64_t*)(B + p.o_clr2), p.clr_cap,
                           (uint32_t*)(B + p.o_piv[2]), p.piv_words[2]);
        HIPC(hipGetLastError());
        MARK("k_clear_words");
    }
    HIPC(rec_t(w.ev1));
    return 0;
    };  // enqueue
    // TDA_HOST_PROF=1: host-side time of the call's parts (stderr, every 200 calls)
    static const bool host_prof = getenv_is("TDA_HOST_PROF", "1");
    using hclk = std::chrono::steady_clock;
    const auto h0 = hclk::now();
    if (p.piv2_sparse) {  // first use of the region, or the last call left it dirty: one full memset
        char* pv2 = B + p.o_piv[2];
        const size_t bytes = (size_t)L * p.piv_words[2] * 4;
        if (w.piv2_dirty || w.piv2_ptr != pv2 || w.piv2_bytes < bytes) {
            HIPC(hipMemsetAsync(pv2, 0, bytes, s));
            w.piv2_ptr = pv2;
            w.piv2_bytes = bytes;
        }
        w.piv2_dirty = true;  // until this call has cleared the words it set
    }
    if (ge) {
        std::shared_lock<std::shared_mutex> launch_lock(g_launch_mu);
        HIPC(hipEventRecord(w.ev0, s));
        HIPC(hipGraphLaunch(ge->exec, s));
        HIPC(hipEventRecord(w.ev1, s));
    } else if (capture) {
        // capture + instantiate one graph at a time across the process: concurrent
        // captures from several slot threads crashed the HIP runtime once (r03, host
        // segfault inside a first call of two slots); replays run concurrently with each
        // other, but not with a capture and its first launch (g_launch_mu)
        std::lock_guard<std::mutex> cap_lock(g_capture_mu);
        std::unique_lock<std::shared_mutex> launch_lock(g_launch_mu);
        HIPC(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        const int rc = enqueue();
        hipGraph_t graph = nullptr;
        const hipError_t ce = hipStreamEndCapture(s, &graph);
        if (rc) {
            if (graph) (void)hipGraphDestroy(graph);
            return rc;
        }
        if (ce != hipSuccess) return fail(TDA_E_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ce));
        GraphEntry e;
        e.key = gk;
        e.graph = graph;
        // the captured graph lives as long as its executable instance: destroying it right after
        // hipGraphInstantiate (legal by the API) faulted in the instance's first hipGraphLaunch
        // when other slots' threads were calling at the same time (r06, tools/concurrency_stress.py)
        const hipError_t ie = hipGraphInstantiate(&e.exec, graph, nullptr, nullptr, 0);
        if (ie != hipSuccess) {
            (void)hipGraphDestroy(graph);
            return fail(TDA_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ie));
        }
        if (w.graphs.size() >= 16) drop_graphs(w), e.key.gen = w.gen;
        w.graphs.push_back(e);
        HIPC(hipEventRecord(w.ev0, s));
        HIPC(hipGraphLaunch(w.graphs.back().exec, s));
        HIPC(hipEventRecord(w.ev1, s));
    } else {
        std::shared_lock<std::shared_mutex> launch_lock(g_launch_mu);
        if (int rc = enqueue()) return rc;
    }
    if (a.want_dist) {
        HIPC(hipMemcpyAsync(w.hdist, dist, sizeof(float) * L * n * n, hipMemcpyDeviceToHost, s));
        if (p.want64) HIPC(hipMemcpyAsync(w.hdist + sizeof(float) * L * n * n, B + p.o_d64, sizeof(double) * L * n * n, hipMemcpyDeviceToHost, s));
    }
    const auto h1 = hclk::now();
    // (an event sync or a busy-polled end event measured the same for one call at a time, r02; and
    // for six pipelined slots, hipStreamQuery polled in a loop: 697-701 vs 540-727 K layers/s, r06)
    HIPC(hipStreamSynchronize(s));
    const auto h2 = hclk::now();

    int errs = 0;
    for (int l = 0; l < L; ++l) errs |= w.hstats[l].err & ~ERR_CAP_MISS;
    if (p.piv2_sparse) {  // clean again unless a layer's word list overflowed
        bool over = false;
        for (int l = 0; l < L; ++l) over |= (uint64_t)w.hstats[l].n_clr2 > p.clr_cap;
        // only k_apparent<2> lists the words it sets: when H2 was reduced by k_reduce_big<2>
        // (TDA_PAR2=0, or no_par >= 1 after a k_reduce_par abort) that kernel also set residual-pivot
        // bits nobody listed, so the next call must start from a full memset
        w.piv2_dirty = over || !p.par2;
    }
    if (errs == ERR_OUT_CAP) {
        size_t need = 0;
        for (int l = 0; l < L; ++l)
            for (int d = 0; d <= p.maxdim; ++d) need += (size_t)std::min<uint64_t>(w.hstats[l].count[d], p.pcap[d]);
        {
            std::lock_guard<std::mutex> g(g_capture_mu);
            if (int rc = grow_hout(w, need + 16)) return rc;
        }
        for (int l = 0; l < L; ++l) w.hstats[l].err = 0;
        HIPC(hipMemcpyAsync(stats, w.hstats, sizeof(LayerStats) * L, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_emit, dim3(L), dim3(1024), kEmitLds, s, stats, L, p.maxdim, ps, (uint64_t*)(B + p.o_fk),
                           (uint32_t*)(B + p.o_fv), p.sstride, w.houtoff_dev, w.hout_dev, (uint64_t)w.hout_cap, w.hstats_dev);
        HIPC(hipGetLastError());
        HIPC(hipStreamSynchronize(s));
        errs = 0;
        for (int l = 0; l < L; ++l) errs |= w.hstats[l].err & ~ERR_CAP_MISS;
    }
    if (errs && getenv("TDA_DEBUG"))
        fprintf(stderr, "[tda] N=%d L=%d errs=%s force_global=%d scale=%d\n", n, L, err_flags(errs).c_str(), (int)force_global, scale);
    if (errs & (ERR_PAR | ERR_PAR2)) {
        // k_reduce_par gave up (a capacity or spin limit): the whole call is re-run (distances,
        // H0, apparent pairs included) with the reduction on the serial radix-heap kernel -- both
        // dimensions after an H1 abort (ERR_PAR); after an H2 abort alone (ERR_PAR2) H1 stays on
        // k_reduce_par and only H2 moves to k_reduce_big.  An abort costs the first call of a
        // shape about twice its time; the retry memo skips the failing attempt on later calls.
        const int np_next = (errs & ERR_PAR) ? 2 : std::max(no_par, 1);
        ParCtl c;
        HIPC(hipMemcpy(&c, B + p.o_pctl, sizeof(c), hipMemcpyDeviceToHost));
        if (getenv("TDA_DEBUG"))
            fprintf(stderr, "[tda] k_reduce_par aborted: code %llu, evictions %llu, records %llu, pools %llu / %llu keys\n", c.err,
                    c.evictions, c.rec_used, c.rpool_used, c.bpool_used);
        const unsigned code = (unsigned)(c.err & 0xFFFF);
        const bool capacity = code == 21 || code == 22 || code == 41 || code == 53;  // pools / requeue slots
        // (a noisy circle at N = 1024 needs ~450 M bucket keys for its one long column, 4x the
        // first pool; a sphere's H2 at N = 1024 more: tools/cap_miss.py)
        if (capacity && scale < kMaxParScale) {  // the same parallel reduction with larger pools
            guard.unlock();
            return run_pipeline(a, input_kind, host_or_dev, out, force_global, scale + 1, force_big, no_par, no_cap);
        }
        if (test_env_is("TDA_PAR_STRICT", "1"))  // tests: the parallel path itself must succeed
            return fail(TDA_E_CAPACITY, "k_reduce_par aborted: item " + std::to_string(c.err >> 16) + " code " +
                                            std::to_string(code));
        guard.unlock();
        return run_pipeline(a, input_kind, host_or_dev, out, force_global, scale, force_big, np_next, no_cap);
    }
    if ((errs & ERR_LDS_SPILL) && !force_global) {
        // a working column outgrew LDS: redo the batch with global-memory tables
        guard.unlock();
        return run_pipeline(a, input_kind, host_or_dev, out, true, scale, false, no_par, no_cap);
    }
    if ((errs & ERR_WORK_CAP) && !p.big && !test_env_is("TDA_REDUCE", "wave")) {
        // a working column outgrew the one-wave HBM tables: full scans of a
        // large column are the slow case, so switch to the radix-heap kernel
        guard.unlock();
        return run_pipeline(a, input_kind, host_or_dev, out, true, 0, true, no_par, no_cap);
    }
    if ((errs & ~(ERR_LDS_SPILL)) == (errs & (ERR_WORK_CAP | ERR_VPOOL_CAP)) && errs && scale < 2) {
        // working column / reduced-column pool too small: retry with larger buffers
        guard.unlock();
        return run_pipeline(a, input_kind, host_or_dev, out, force_global, scale + 1, p.big, no_par, no_cap);
    }
    if (errs) return fail(TDA_E_CAPACITY, "device work buffer overflow:" + err_flags(errs));
#ifdef TDA_PROF2
    if (p.par) {  // per-wave phase cycles of the long columns (k_reduce_par, the last launch)
        ParCtl c;
        HIPC(hipMemcpy(&c, B + p.o_pctl, sizeof(c), hipMemcpyDeviceToHost));
        const uint64_t nrec = std::min<uint64_t>(c.pad[2], kParDbgCap);
        std::vector<uint64_t> d(nrec * kParP2Words);
        if (nrec) HIPC(hipMemcpy(d.data(), B + p.o_pdbg + (size_t)kParDbgCap * 32, nrec * kParP2Words * 8, hipMemcpyDeviceToHost));
        static const char* nm[8] = {"room+barrier", "min", "pivot+loads", "keys", "appends", "toggles", "refills", "owner"};
        uint64_t best = ~0ull, bsteps = 0;
        for (uint64_t i = 0; i < nrec; ++i)
            if (d[i * kParP2Words + 2] > bsteps) bsteps = d[i * kParP2Words + 2], best = d[i * kParP2Words];
        for (uint64_t i = 0; i < nrec; ++i) {
            const uint64_t* r = &d[i * kParP2Words];
            if (r[0] != best) continue;
            uint64_t tot = 0;
            for (int u = 0; u < 8; ++u) tot += r[3 + u];
            fprintf(stderr, "[tda-prof2] layer %llu column %llu wave %llu: %llu steps, %.0f cycles/step:", (unsigned long long)(r[0] >> 40),
                    (unsigned long long)(r[0] & ((1ull << 40) - 1)), (unsigned long long)r[1], (unsigned long long)r[2], (double)tot / (double)r[2]);
            for (int u = 0; u < 8; ++u) fprintf(stderr, " %s %.0f", nm[u], (double)r[3 + u] / (double)r[2]);
            fprintf(stderr, "\n");
        }
    }
#endif
#ifdef TDA_PROFILE
    if (p.dense && !p.par) {
        int arg = 0;
        uint64_t p1max = 0;
        for (int l = 0; l < L; ++l) {
            if (w.hstats[l].prof[0][0] > w.hstats[arg].prof[0][0]) arg = l;
            p1max = std::max<uint64_t>(p1max, w.hstats[l].prof[1][0]);
        }
        const uint64_t* q = w.hstats[arg].prof[0];
        fprintf(stderr, "[tda-prof] dense H1 slowest layer %d adds %lld: total %llu pivot %llu (calls %llu ties %llu) cob_app %llu add_owner %llu new_pair %llu cycles; H2 phase-1 slowest wave %llu cycles\n",
                arg, (long long)w.hstats[arg].n_adds[1], (unsigned long long)q[0], (unsigned long long)q[1], (unsigned long long)q[7],
                (unsigned long long)q[2], (unsigned long long)q[3], (unsigned long long)q[4], (unsigned long long)q[5],
                (unsigned long long)p1max);
        uint64_t sc = 0, cb = 0, tt = 0, ad = 0, mx = 0, mxa = 0;
        for (int l = 0; l < L; ++l) {
            sc += w.hstats[l].prof[1][4];
            cb += w.hstats[l].prof[1][5];
            tt += w.hstats[l].prof[1][6];
            ad += w.hstats[l].prof[1][7];
            if (w.hstats[l].prof[1][2] > mx) {
                mx = w.hstats[l].prof[1][2];
                mxa = w.hstats[l].prof[1][3] & 0xFFFF;
            }
        }
        {
            const uint64_t* e = w.hstats[0].prof[4];
            fprintf(stderr, "[tda-prof] k_prep_edges layer 0 (us from block entry): sort block thresh %.2f staged %.2f sorted %.2f end %.2f; mask blocks (max) thresh %.2f staged %.2f end %.2f\n",
                    e[0] * 0.01, e[1] * 0.01, e[2] * 0.01, e[3] * 0.01, e[4] * 0.01, e[5] * 0.01, e[6] * 0.01);
        }
        {
            const uint64_t* h = w.hstats[0].prof[3];
            fprintf(stderr, "[tda-prof] k_h0_wave layer 0 (cycles from entry): thresh %llu prim %llu sort %llu unionfind %llu end %llu; chain staging (slowest layer) %llu\n",
                    (unsigned long long)h[1], (unsigned long long)h[2], (unsigned long long)h[3], (unsigned long long)h[4],
                    (unsigned long long)h[5], (unsigned long long)q[6]);
        }
        fprintf(stderr, "[tda-prof] H2 phase 1: all columns %llu cycles (scan %llu cob %llu), %llu adds; slowest column %llu cycles (%llu adds)\n",
                (unsigned long long)tt, (unsigned long long)sc, (unsigned long long)cb, (unsigned long long)ad, (unsigned long long)mx,
                (unsigned long long)mxa);
    }
    if (n > kSmallN) {
        const uint64_t* h = w.hstats[0].prof[0];
        fprintf(stderr, "[tda-prof] k_h0 layer 0 (cycles from entry): staged %llu, thresh+edges %llu, forest %llu, sort %llu, end %llu\n",
                (unsigned long long)h[0], (unsigned long long)h[1], (unsigned long long)h[2], (unsigned long long)h[3],
                (unsigned long long)h[4]);
    }
    if (p.par) {
        {   // long-column timeline of the last k_reduce_par launch (H2's when it ran, else H1's)
            ParCtl c;
            HIPC(hipMemcpy(&c, B + p.o_pctl, sizeof(c), hipMemcpyDeviceToHost));
            const uint64_t nlog = std::min<uint64_t>(c.pad[1], kParDbgCap);
            std::vector<uint64_t> d(nlog * 4);
            if (nlog) HIPC(hipMemcpy(d.data(), B + p.o_pdbg, nlog * 32, hipMemcpyDeviceToHost));
            std::vector<uint64_t> order(nlog);
            for (uint64_t i = 0; i < nlog; ++i) order[i] = i;
            std::sort(order.begin(), order.end(), [&](uint64_t x, uint64_t y) { return d[x * 4 + 2] - d[x * 4 + 1] > d[y * 4 + 2] - d[y * 4 + 1]; });
            uint64_t tend = 0;
            for (uint64_t i = 0; i < nlog; ++i) tend = std::max(tend, d[i * 4 + 2]);
            fprintf(stderr, "[tda-prof] k_reduce_par timeline: %llu columns of >= %llu steps; last one ends %.3f ms after the first workgroup started\n",
                    (unsigned long long)nlog, (unsigned long long)kParDbgMinSteps, nlog ? (tend - c.pad[0]) * 1e-5 : 0.0);
            for (uint64_t k = 0; k < std::min<uint64_t>(nlog, 12); ++k) {
                const uint64_t i = order[k];
                fprintf(stderr, "[tda-prof]   layer %llu column %llu: start %.3f ms, %.3f ms, %llu steps%s\n",
                        (unsigned long long)(d[i * 4] >> 40), (unsigned long long)(d[i * 4] & ((1ull << 40) - 1)),
                        (d[i * 4 + 1] - c.pad[0]) * 1e-5, (d[i * 4 + 2] - d[i * 4 + 1]) * 1e-5,
                        (unsigned long long)(d[i * 4 + 3] & ~(1ull << 63)), (d[i * 4 + 3] >> 63) ? " (resumed)" : "");
            }
        }
        const uint64_t* q = w.hstats[0].prof[2];
        fprintf(stderr, "[tda-prof] k_reduce_par longest column: %llu steps, %llu cycles: front_min %llu, pivot+rows %llu, apparent adds %llu, refills %llu (%llu), owner path %llu; avg front log %llu, compactions %llu, spills %llu\n",
                (unsigned long long)q[6], (unsigned long long)q[0], (unsigned long long)q[1], (unsigned long long)q[2], (unsigned long long)q[3],
                (unsigned long long)q[4], (unsigned long long)((q[7] >> 16) & 0xFFFF), (unsigned long long)q[5], (unsigned long long)(q[7] & 0xFFFF),
                (unsigned long long)((q[7] >> 32) & 0xFFFF), (unsigned long long)(q[7] >> 48));
        const uint64_t* u = w.hstats[0].prof[3];
        fprintf(stderr, "[tda-prof]   inside adds: keys %llu, capacity %llu, front toggles %llu, bucket appends %llu cycles; %llu record adds (%llu keys); refills moved %llu keys; wave 0 toggled %llu front / %llu back keys\n",
                (unsigned long long)u[0], (unsigned long long)u[3], (unsigned long long)u[1], (unsigned long long)u[2],
                (unsigned long long)u[4], (unsigned long long)u[5], (unsigned long long)u[6], (unsigned long long)(u[7] >> 32),
                (unsigned long long)(u[7] & 0xFFFFFFFFull));
        const uint64_t* v = w.hstats[0].prof[4];
        fprintf(stderr, "[tda-prof]   record adds: room %llu, col_add %llu cycles, keys front %llu / all %llu; refill pass 3 %llu cycles; %llu saves (%llu keys) %llu cycles\n",
                (unsigned long long)v[0], (unsigned long long)v[1], (unsigned long long)v[2], (unsigned long long)v[3], (unsigned long long)v[5],
                (unsigned long long)v[6], (unsigned long long)v[7], (unsigned long long)v[4]);
        const uint64_t* y = w.hstats[0].prof[1];
        fprintf(stderr, "[tda-prof]   refill phases: search %llu, loads+min %llu, histogram %llu, level choice %llu, toggles %llu, appends %llu, compactions %llu cycles; %llu keys kept in front\n",
                (unsigned long long)y[0], (unsigned long long)y[1], (unsigned long long)y[2], (unsigned long long)y[3],
                (unsigned long long)y[4], (unsigned long long)y[5], (unsigned long long)y[6], (unsigned long long)y[7]);
    }
    if (p.big && !p.par)
        for (int d = 1; d <= p.maxdim; ++d) {
            const uint64_t* q = w.hstats[0].prof[d];
            fprintf(stderr, "[tda-prof] big dim %d layer 0: cob0 %llu pop %llu owner_add %llu app_add %llu store %llu reset %llu total %llu cycles; owner adds %llu entries %llu, all adds %lld\n",
                    d, (unsigned long long)q[0], (unsigned long long)q[1], (unsigned long long)q[2], (unsigned long long)q[3],
                    (unsigned long long)q[4], (unsigned long long)q[5], (unsigned long long)q[7], (unsigned long long)(q[6] >> 40),
                    (unsigned long long)(q[6] & ((1ull << 40) - 1)), (long long)w.hstats[0].n_adds[d]);
        }
    for (int d = 1; d <= p.maxdim; ++d) {
        uint64_t mx[8] = {0};
        int arg = 0;
        for (int l = 0; l < L; ++l)
            if (w.hstats[l].prof[d][7] > mx[7]) {
                arg = l;
                for (int i = 0; i < 8; ++i) mx[i] = w.hstats[l].prof[d][i];
            }
        fprintf(stderr, "[tda-prof] dim %d slowest layer %d adds %lld: scan %llu lookup %llu dec+facet %llu cob_app %llu toggles %llu reset %llu compact %llu total %llu cycles\n",
                d, arg, (long long)w.hstats[arg].n_adds[d], (unsigned long long)mx[0], (unsigned long long)mx[1], (unsigned long long)mx[2],
                (unsigned long long)mx[3], (unsigned long long)mx[4], (unsigned long long)mx[5], (unsigned long long)mx[6], (unsigned long long)mx[7]);
    }
#endif

    // remember what this shape needed (capacity / reducer retries; column caps are not
    // remembered: a cap miss re-runs only its own layers, below, and every call starts capped)
    if (force_global || scale || force_big || no_par) {
        bool seen = false;
        for (auto& m : w.retry)
            if (m.N == p.N && m.maxdim == p.maxdim && m.input_kind == input_kind) {
                m.force_global = m.force_global || force_global;
                m.force_big = m.force_big || force_big;
                m.no_par = std::max(m.no_par, no_par);
                m.scale = std::max(m.scale, scale);
                seen = true;
            }
        if (!seen) w.retry.push_back({p.N, p.maxdim, input_kind, force_global, force_big, no_par, scale});
    }
    std::vector<int> cap_miss;  // layers whose capped reduction missed (ERR_CAP_MISS): re-run below without caps
    for (int l = 0; l < L; ++l)
        if (w.hstats[l].err & ERR_CAP_MISS) cap_miss.push_back(l);

    // ---- result
    auto* R = new ResultImpl();
    const int nd = p.maxdim + 1;
    const size_t S = (size_t)L * nd;
    size_t total = 0;
    for (int l = 0; l < L; ++l)
        for (int d = 0; d < nd; ++d) total += (size_t)std::min<int64_t>(w.hstats[l].count[d], (int64_t)p.pcap[d]);
    // one allocation (tda_rips.h layout guarantee): a binding copies it in one read
    const size_t o_ne = 7 * S, o_idx = o_ne + L, o_thr = o_idx + 2 * total, o_bd = o_thr + (L + 1) / 2;
    R->blob.assign(o_bd + total, 0);
    int64_t* m_count = (int64_t*)R->blob.data();
    int64_t* m_off = m_count + S;
    uint64_t* m_cs = (uint64_t*)(m_count + 2 * S);
    int64_t* m_all = m_count + 3 * S;
    int64_t* m_cols = m_count + 4 * S;
    int64_t* m_res = m_count + 5 * S;
    int64_t* m_add = m_count + 6 * S;
    float* r_thr = (float*)(R->blob.data() + o_thr);
    int64_t* r_ne = (int64_t*)(R->blob.data() + o_ne);
    int64_t* r_idx = (int64_t*)(R->blob.data() + o_idx);
    float* r_bd = (float*)(R->blob.data() + o_bd);
    for (int l = 0; l < L; ++l) {
        const LayerStats& st = w.hstats[l];
        r_thr[l] = st.thresh;
        r_ne[l] = st.num_edges;
        for (int d = 0; d < nd; ++d) {
            int64_t c = std::min<int64_t>(st.count[d], (int64_t)p.pcap[d]);
            m_count[l * nd + d] = c;
            m_off[l * nd + d] = w.houtoff[l * nd + d];
            m_cs[l * nd + d] = st.checksum[d];
            m_all[l * nd + d] = st.all_pairs[d];
            m_cols[l * nd + d] = st.n_columns[d];
            m_res[l * nd + d] = st.n_residual[d] - st.nskip[d];
            m_add[l * nd + d] = st.n_adds[d];
        }
    }
    // layer-major result (tda_rips.h); the device wrote each (layer, dim) segment
    // at houtoff, in layer order (k_emit)
    {
        size_t e = 0;
        for (int l = 0; l < L; ++l)
            for (int d = 0; d < nd; ++d) {
                const size_t src = (size_t)w.houtoff[l * nd + d];
                const size_t c = (size_t)m_count[l * nd + d];
                m_off[l * nd + d] = (int64_t)e;
                for (size_t i = 0; i < c; ++i, ++e) {
                    const OutPair q = w.hout[src + i];
                    r_bd[e] = q.birth;
                    r_bd[total + e] = q.death;
                    r_idx[e] = q.birth_idx;
                    r_idx[total + e] = q.death_idx;
                }
            }
    }
    if (a.want_dist) {  // landed by the async copies behind the call (synchronised above)
        R->dist.resize((size_t)L * n * n);
        std::memcpy(R->dist.data(), w.hdist, sizeof(float) * L * n * n);
    }
    if (p.want64) {
        R->dist64.resize((size_t)L * n * n);
        std::memcpy(R->dist64.data(), w.hdist + sizeof(float) * L * n * n, sizeof(double) * L * n * n);
    }
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, w.ev0, w.ev1);
    tda_rips_result& o = R->pub;
    o.L = L;
    o.maxdim = p.maxdim;
    o.N = n;
    o.count = m_count;
    o.offset = m_off;
    o.birth = r_bd;
    o.death = r_bd + total;
    o.birth_idx = r_idx;
    o.death_idx = r_idx + total;
    o.thresh = r_thr;
    o.num_edges = r_ne;
    o.blob = R->blob.data();
    o.blob_bytes = (int64_t)(R->blob.size() * 8);
    o.n_pairs = (int64_t)total;
    o.checksum = m_cs;
    o.n_all_pairs = m_all;
    o.n_columns = m_cols;
    o.n_residual = m_res;
    o.n_adds = m_add;
    o.dist = a.want_dist ? R->dist.data() : nullptr;
    o.dist64 = p.want64 ? R->dist64.data() : nullptr;
    if (nls) {
        R->sil.assign((const double*)(w.hsil + sil_out_off), (const double*)(w.hsil + sil_out_off) + (size_t)L * nls);
        o.silhouette = R->sil.data();
    } else {
        o.silhouette = nullptr;
    }
    if (want_tn) {
        R->tn.assign(w.htn, w.htn + L);
        o.twonn = R->tn.data();
    } else {
        o.twonn = nullptr;
    }
    o.device_ms = ms;
    for (size_t i = 0; i < tm.names.size(); ++i) {
        float t = 0.0f;
        (void)hipEventElapsedTime(&t, w.stage_ev[i], w.stage_ev[i + 1]);
        R->stage_ms.push_back(t);
        R->stage_name.push_back(tm.names[i]);
    }
    for (size_t i = 0; i < tm2.names.size(); ++i) {  // side stream: H0, edge classes
        float t = 0.0f;
        (void)hipEventElapsedTime(&t, w.stage_ev2[i], w.stage_ev2[i + 1]);
        R->stage_ms.push_back(t);
        R->stage_name.push_back(tm2.names[i]);
    }
    for (size_t i = 0; i < tm4.names.size(); ++i) {  // fourth stream: H0
        float t = 0.0f;
        (void)hipEventElapsedTime(&t, w.stage_ev4[i], w.stage_ev4[i + 1]);
        R->stage_ms.push_back(t);
        R->stage_name.push_back(tm4.names[i]);
    }
    for (size_t i = 0; i < tm3.names.size(); ++i) {  // third stream: H2 phase 1
        float t = 0.0f;
        (void)hipEventElapsedTime(&t, w.stage_ev3[i], w.stage_ev3[i + 1]);
        R->stage_ms.push_back(t);
        R->stage_name.push_back(tm3.names[i]);
    }
    o.n_stages = (int32_t)R->stage_name.size();
    if (host_prof) {
        static double acc[5] = {0, 0, 0, 0, 0};
        static int calls = 0;
        const auto h3 = hclk::now();
        auto us = [](hclk::duration d) { return std::chrono::duration<double, std::micro>(d).count(); };
        acc[0] += us(h1 - h0);
        acc[1] += us(h2 - h1);
        acc[2] += us(h3 - h2);
        acc[3] += ms * 1e3;
        acc[4] += us(h0 - h_entry);
        if (++calls % 200 == 0) {
            fprintf(stderr, "[tda-host] per call: setup %.1f us, launch %.1f us, sync %.1f us (device %.1f us), result %.1f us\n",
                    acc[4] / 200, acc[0] / 200, acc[1] / 200, acc[3] / 200, acc[2] / 200);
            acc[0] = acc[1] = acc[2] = acc[3] = acc[4] = 0;
        }
    }
    o.stage_name = R->stage_name.data();
    o.stage_ms = R->stage_ms.data();
    o.n_cap_reruns = 0;
    if (!cap_miss.empty()) {
        guard.unlock();
        return rerun_cap_missed(a, input_kind, host_or_dev, out, R, cap_miss, force_global, scale, force_big, no_par);
    }
    *out = &R->pub;
    return 0;
}

// entry: start from the configuration an earlier call of this shape ended on
int run_entry(const tda_rips_args& a, int input_kind, const void* src, tda_rips_result** out) {
    bool fg = false, fb = false;
    int np = 0;
    int sc = 0;
    // not when a test forces a reducer (the memo would override what it asks for)
    if (!test_env_is("TDA_RETRY_MEMO", "0") && !test_env("TDA_REDUCE") && !test_env("TDA_PAR") && !test_env("TDA_PAR_STRICT") &&
        !test_env("TDA_CHAIN")) {
        Workspace& w = *get_ws(a.device, a.slot);
        std::lock_guard<std::mutex> g(w.mu);
        for (const auto& m : w.retry)
            if (m.N == a.N && m.maxdim == a.maxdim && m.input_kind == input_kind) {
                fg = m.force_global;
                fb = m.force_big;
                np = m.no_par;
                sc = m.scale;
            }
    }
    return run_pipeline(a, input_kind, src, out, fg, sc, fb, np, false);
}

int validate(const tda_rips_args* a) {
    if (!a) return fail(TDA_E_INVALID, "args is NULL");
    if (a->n_parts < 0 || a->n_parts > TDA_MAX_PARTS) return fail(TDA_E_INVALID, "n_parts must be in [0, TDA_MAX_PARTS]");
    if (a->n_parts > 0) {
        if (!a->x_parts) return fail(TDA_E_INVALID, "x_parts is NULL");
        for (int i = 0; i < a->n_parts; ++i)
            if (!a->x_parts[i]) return fail(TDA_E_INVALID, "x_parts[" + std::to_string(i) + "] is NULL");
        if (a->L % a->n_parts) return fail(TDA_E_INVALID, "L must be a multiple of n_parts");
    } else if (!a->x && a->L * a->N > 0) {
        return fail(TDA_E_INVALID, "x is NULL");
    }
    if (a->L < 1) return fail(TDA_E_INVALID, "L must be >= 1");
    if (a->N < 1) return fail(TDA_E_INVALID, "N must be >= 1");
    if (!a->is_dist && a->D < 1) return fail(TDA_E_INVALID, "D must be >= 1");
    if (a->dtype != TDA_F32 && a->dtype != TDA_F64) return fail(TDA_E_INVALID, "dtype must be TDA_F32 or TDA_F64");
    if (a->modulus != 2) return fail(TDA_E_UNSUPPORTED, "only coeff=2 (Z/2) is supported");
    if (a->maxdim < 0 || a->maxdim > 2) return fail(TDA_E_UNSUPPORTED, "maxdim must be 0, 1 or 2");
    if (a->N > 8192) return fail(TDA_E_UNSUPPORTED, "N > 8192 is not supported");
    if (a->slot < 0 || a->slot >= TDA_MAX_SLOTS) return fail(TDA_E_INVALID, "slot must be in [0, TDA_MAX_SLOTS)");
    // H1 filtration keys pack a 32-bit row-simplex index: C(N, 3) < 2^32.  H2
    // above N = 568 uses edge-code keys (21-bit code + 42-bit index): C(N, 2) < 2^21
    if (a->maxdim == 1 && a->N > 2900) return fail(TDA_E_UNSUPPORTED, "maxdim=1 requires N <= 2900");
    if (a->maxdim == 2 && a->N > 2048) return fail(TDA_E_UNSUPPORTED, "maxdim=2 requires N <= 2048");
    if (std::isnan(a->thresh)) return fail(TDA_E_INVALID, "thresh is NaN");
    if ((a->flags & TDA_FLAG_NO_PERSISTENCE) && a->maxdim != 0) return fail(TDA_E_INVALID, "TDA_FLAG_NO_PERSISTENCE needs maxdim 0");
    if (a->want_twonn && !(a->twonn_discard >= 0.0 && a->twonn_discard < 1.0 && a->twonn_eps >= 0.0f))
        return fail(TDA_E_INVALID, "TwoNN needs 0 <= discard_fraction < 1 and eps >= 0");
    return 0;
}

}  // namespace

extern "C" {

int tda_rips_batch(const tda_rips_args* args, tda_rips_result** out) {
    if (!out) return fail(TDA_E_INVALID, "out is NULL");
    *out = nullptr;
    if (int rc = validate(args)) return rc;
    if (!tda_device_ok(args->device)) return fail(TDA_E_NODEVICE, "no gfx950 device at ordinal " + std::to_string(args->device));
    return run_entry(*args, args->is_dist ? 1 : 0, args->x, out);
}

int tda_rips_dm(const float* D, int64_t n_entries, int32_t modulus, int32_t dim_max, float threshold, int32_t do_cocycles,
                tda_rips_result** out) {
    if (!out) return fail(TDA_E_INVALID, "out is NULL");
    *out = nullptr;
    if (do_cocycles) return fail(TDA_E_UNSUPPORTED, "do_cocycles is not supported");
    if (n_entries < 0 || (n_entries > 0 && !D)) return fail(TDA_E_INVALID, "bad condensed distance vector");
    // ripser.cpp compressed_distance_matrix: rows = (1 + sqrt(1 + 8 n)) / 2
    int64_t N = (int64_t)((1.0 + std::sqrt(1.0 + 8.0 * (double)n_entries)) / 2.0);
    if (N * (N - 1) / 2 != n_entries) return fail(TDA_E_INVALID, "n_entries is not N(N-1)/2");
    tda_rips_args a;
    std::memset(&a, 0, sizeof(a));
    a.x = D;
    a.dtype = TDA_F32;
    a.L = 1;
    a.N = N;
    a.D = 0;
    a.is_dist = 1;
    a.maxdim = dim_max;
    a.thresh = threshold;
    a.modulus = modulus;
    a.device = 0;
    if (int rc = validate(&a)) return rc;
    if (!tda_device_ok(0)) return fail(TDA_E_NODEVICE, "no gfx950 device");
    return run_entry(a, 2, D, out);
}

void tda_rips_free(tda_rips_result* r) {
    if (!r) return;
    delete reinterpret_cast<ResultImpl*>(r);  // pub is the first member
}

const char* tda_last_error(void) { return g_err.c_str(); }

int tda_version(void) { return TDA_RIPS_ABI_VERSION; }

int tda_device_ok(int32_t device) {
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess || device < 0 || device >= cnt) return 0;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 0;
    return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

}  // extern "C"

// UMAP embedding (include/tda_umap.h): same library, same error state
#include "umap_host.h"
// effective dimensionality (include/tda_rips.h tda_effective_dim)
#include "ed_host.h"
