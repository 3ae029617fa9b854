// rips_kernels.h -- gfx950 kernels of the batched Vietoris-Rips pipeline.
//
// One launch of each kernel covers every layer of a batch (blockIdx.y or
// blockIdx.x = layer), so the reference's per-layer Python loop
// (debug_tda_pipeline.py:92-150) becomes a handful of launches per sweep.
//
//   k_distance      pairwise L2 in FP64, sklearn-f32 rounding   
//   k_square_dist   condensed/square distance input             (a2' / is_dist)
//   k_h0 / k_h0_wave enclosing radius, num_edges, spanning forest, H0 pairs (a3, a4)
//   k_apparent<d>   column enumeration + apparent-pair test     (a5, parallel part)
//   k_sort_resid    per-layer sort of the residual columns
//   k_emit          per-layer emission order of the pairs, packed into the
//                   host-mapped result                           (a6)
//   k_silhouette    sklearn silhouette_score on the same distances (8f row 1)
// The residual reductions are in rips_reduce.h (one wave per layer),
// rips_reduce_small.h (N <= 64 dense chain), rips_reduce_par.h (large N,
// many columns in flight) and rips_reduce_big.h (its fallback).
#pragma once
#include "rips_device.h"

namespace tda {

// ------------------------------------------------------------------ layout
struct Pair {
    float birth, death;
    int64_t birth_idx, death_idx;
};
// typed (non-FLAT) store of one pair to HBM
__device__ __forceinline__ void store_pair(Pair* P, uint64_t i, float b, float d, int64_t bi, int64_t di) {
    uint64_t* q = (uint64_t*)(P + i);
    st_glb(q, 0, (uint64_t)__float_as_uint(b) | ((uint64_t)__float_as_uint(d) << 32));
    st_glb(q, 1, (uint64_t)bi);
    st_glb(q, 2, (uint64_t)di);
}

struct LayerStats {  // zeroed every call; copied to the host result
    float thresh;
    int32_t err;  // bit flags, see ERR_*
    int64_t num_edges;
    int64_t count[4];      // emitted pairs per dim
    uint64_t checksum[4];  // sum of pair_hash over all pairs
    int64_t all_pairs[4];
    int64_t n_columns[4];
    int64_t n_residual[4];
    int64_t n_adds[4];     // column additions in the serial reduction
    int64_t nskip[4];      // residual columns cleared by the serial reduction (host: n_residual - nskip)
    uint64_t rmask[4];     // residual pivot map mask used by the dim's reducer (HBM map consumers)
    int64_t ntri;          // N <= 64: triangles <= thresh (k_prep_tables)
    int64_t n_clr2;        // sparse-cleared H2 pivot bitmap: words k_apparent<2> listed for the end-of-call clear
    uint64_t prof[5][8];   // -DTDA_PROFILE builds: cycle counters (per dim; [3]: k_h0_wave, [4]: k_prep_layer)
};
enum : int32_t { ERR_RESID_CAP = 1, ERR_PAIR_CAP = 2, ERR_WORK_CAP = 4, ERR_VPOOL_CAP = 8, ERR_OUT_CAP = 16 };

struct DimBufs {              // per reduction dim d (columns = d-simplices)
    const uint32_t* cleared;  // bitmap over d-simplices (per layer stride)
    uint64_t cleared_words;
    uint32_t* pivbits;        // bitmap over (d+1)-simplices
    uint64_t piv_words;
    uint64_t* resid;          // residual column keys [L][rcap]
    uint64_t rcap;
    uint64_t ncand;           // C(N, d+1)
    // d = 2 with a bitmap too large to memset every call (C(N, 4) / 8 B: 91 GB at N = 2048): the
    // word of every bit k_apparent<2> sets, [L][clr_cap]; k_clear_words zeroes them at the end
    uint64_t* clr;
    uint64_t clr_cap;
};

// ------------------------------------------------------------------ distance
// sklearn/metrics/pairwise.py:582-653: X chunk upcast to f64,
// d = (-2 <x_i,x_j> + |x_i|^2) + |x_j|^2 (i < j, i is the "X" row as ripser.py
// reads dm[I > J]), cast to f32 (:651), clamp (:429), diag 0 (:436), sqrt (:441).
// The dot products and norms accumulate in increasing k with FMA, exact for
// f32 inputs (products are exact in f64).
// Row maxima for the enclosing radius (ripser.py rips_dm: thresh = min_i
// max_j d(i,j)) are folded into the distance pass: per-tile row/column maxima,
// then one atomicMax per row on the f32 bit pattern (non-negative floats order
// like unsigned ints).  rowmax must be zeroed before the launch.
template <typename T>
__global__ __launch_bounds__(256) void k_distance(const T* __restrict__ X, int n, int D, float* __restrict__ dist,
                                                  uint32_t* __restrict__ rowmax, double* __restrict__ dist64 = nullptr) {
    constexpr int TS = 16, KC = 32;
    __shared__ double xi[TS][KC + 1], xj[TS][KC + 1];
    __shared__ uint32_t rmax_i[TS], rmax_j[TS];
    const int l = blockIdx.z;
    const int bi = blockIdx.y, bj = blockIdx.x;
    if (bj < bi) return;
    const T* Xl = X + (size_t)l * n * D;
    float* Dl = dist + (size_t)l * n * n;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int i = bi * TS + ty, j = bj * TS + tx;
    double dot = 0.0, ni = 0.0, nj = 0.0;
    for (int k0 = 0; k0 < D; k0 += KC) {
        const int kc = min(KC, D - k0);
        for (int e = threadIdx.x; e < TS * KC; e += 256) {
            int r = e / KC, c = e % KC;
            int gi = bi * TS + r, gj = bj * TS + r;
            xi[r][c] = (gi < n && c < kc) ? (double)Xl[(size_t)gi * D + k0 + c] : 0.0;
            xj[r][c] = (gj < n && c < kc) ? (double)Xl[(size_t)gj * D + k0 + c] : 0.0;
        }
        __syncthreads();
        for (int c = 0; c < kc; ++c) {
            double a = xi[ty][c], b = xj[tx][c];
            dot = fma(a, b, dot);
            ni = fma(a, a, ni);
            nj = fma(b, b, nj);
        }
        __syncthreads();
    }
    if (threadIdx.x < TS) {
        rmax_i[threadIdx.x] = 0;
        rmax_j[threadIdx.x] = 0;
    }
    __syncthreads();
    if (i < n && j < n && j >= i) {
        if (i == j) {
            Dl[(size_t)i * n + i] = 0.0f;
            if (dist64) dist64[((size_t)l * n + i) * n + i] = 0.0;
        } else {
            double d = (-2.0 * dot + ni) + nj;
            float f;
            if constexpr (sizeof(T) == 4) {
                f = (float)d;
                f = (f != f) ? f : fmaxf(f, 0.0f);
                f = sqrt_rn_f32(f);
            } else {
                d = (d != d) ? d : fmax(d, 0.0);
                const double r = __dsqrt_rn(d);
                f = (float)r;
                if (dist64) dist64[((size_t)l * n + i) * n + j] = dist64[((size_t)l * n + j) * n + i] = r + 0.0;
            }
            f = f + 0.0f;
            Dl[(size_t)i * n + j] = f;
            Dl[(size_t)j * n + i] = f;
            atomicMax(&rmax_i[ty], __float_as_uint(f));
            atomicMax(&rmax_j[tx], __float_as_uint(f));
        }
    }
    __syncthreads();
    uint32_t* rm = rowmax + (size_t)l * n;
    if (threadIdx.x < TS && bi * TS + threadIdx.x < n && rmax_i[threadIdx.x]) atomicMax(&rm[bi * TS + threadIdx.x], rmax_i[threadIdx.x]);
    if (threadIdx.x >= 64 && threadIdx.x < 64 + TS && bj * TS + threadIdx.x - 64 < n && rmax_j[threadIdx.x - 64])
        atomicMax(&rm[bj * TS + threadIdx.x - 64], rmax_j[threadIdx.x - 64]);
}

// ------------------------------------------------------------------ distance, D >= 32: FP64 MFMA Gram tiles
// Same arithmetic as k_distance (sklearn pairwise.py:582-653: f64 Gram
// products of the upcast rows, d = (-2 g_ij + |x_i|^2) + |x_j|^2 for i < j,
// round to f32, clamp, sqrt), with the dot products on the matrix cores:
// v_mfma_f64_16x16x4_f64.  Products of upcast f32 values are exact in f64, so
// only the summation order differs from the scalar kernel (and from sklearn's
// BLAS dgemm, whose order is its own): the f32 results agree within the
// north_star bound, and almost always bit for bit.
//
// One workgroup = one 64x64 tile of one layer's matrix, upper-triangle tile
// pairs only (bi <= bj, enumerated linearly: no idle lower-triangle blocks).
// 4 waves, each a 32x32 quadrant as 2x2 MFMA tiles (4 independent f64x4
// accumulators hide the MFMA latency).  K is staged through LDS in chunks of
// kDmKC in the input type (widened to f64 at the operand read), row-major with a row stride of kDmS = kDmKC + 2
// doubles: an MFMA operand read (lane -> row lane & 15, k = lane >> 4) maps
// each half-wave's 32 lanes to 32 distinct 8-byte bank pairs (row r, k:
// slot 2r + k mod 32), so the ds_read_b64 is conflict-free; each thread
// stages 4 consecutive k of one row (coalesced global reads, 16-B aligned
// LDS writes).
// The squared norms accumulate in the same pass from the LDS tiles, in a
// fixed but NOT sequential order: each row's K chunks are split into two k
// halves summed by different threads in a lane-rotated k order, then added
// (k_gram_layer, N <= 144: sequential k within each K slice, slices added in
// slice order by k_distance_combine).  So at D >= 32 a few distances differ
// from the oracle's sequential-k f32 rounding (and between the N <= 144 and
// N > 144 kernels) by an ulp: parity there is tolerance-based (1e-5, the
// north_star bound; tests/test_gpu_parity.py test_distance_high_dim_vs_sklearn),
// pair indices are exact only where no two distances swap order.
#ifndef TDA_DM_KC  // build-time A/B knob (tools/): K chunk of k_distance_mfma
#define TDA_DM_KC 32
#endif
constexpr int kDmT = 64, kDmKC = TDA_DM_KC, kDmS = kDmKC + 2;
typedef double dm_d4 __attribute__((ext_vector_type(4)));

// METRIC 1: cosine distance instead (UMAP input, umap.distances.cosine:
// 1 - <x,y> / sqrt(|x|^2 |y|^2), 0 for two zero rows, 1 for one), from the
// same Gram tiles; clamped at 0.  METRIC 2: the raw f64 Gram matrix X X^T
// (both triangles) into gpart (ed_kernels.h: effective dimensionality).
// SPLIT (gridDim.z = S > 1 K slices, chosen on the host when the tiles alone
// leave CUs idle -- raw4096: 6 tiles x 32 layers on 256 CUs): slice z sums
// its K range and stores the tile's partial Gram and (diagonal tiles) the
// partial norms in f64; k_distance_combine adds the slices in a fixed order
// and runs the epilogue.
template <typename T, int METRIC = 0, bool SPLIT = false>
__global__ __launch_bounds__(256) void k_distance_mfma(const T* __restrict__ X, int n, int D, float* __restrict__ dist,
                                                       uint32_t* __restrict__ rowmax, double* __restrict__ gpart = nullptr,
                                                       double* __restrict__ npart = nullptr, double* __restrict__ dist64 = nullptr) {
    // K chunks staged in LDS in the INPUT type (r03: f32 for the raw activations, half the LDS
    // bytes of the f64 staging it replaces -- LDS traffic, not the MFMA pipe, bounded the kernel)
    // and widened to f64 at the operand read; row stride kDmS = kDmKC + 2 elements keeps the
    // operand reads conflict-free for 4-byte and 8-byte elements alike
    __shared__ T xs[2][2][kDmT][kDmS];  // [buffer][i/j tile][row][k]: chunk c + 1 is written while chunk c feeds the MFMAs
    __shared__ double nrm[2][kDmT];
    __shared__ double nrp[2][2][kDmT];  // norm partials: [k half][tile][row]
    __shared__ uint32_t rmx[2][kDmT];
    const int l = blockIdx.y;
    const int nt = (n + kDmT - 1) / kDmT;
    // linear upper-triangle tile index -> (bi, bj), bi <= bj
    int p = blockIdx.x, bi = 0;
    while (p >= nt - bi) p -= nt - bi, ++bi;
    const int bj = bi + p;
    const T* Xl = X + (size_t)l * n * D;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    dm_d4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = dm_d4{0.0, 0.0, 0.0, 0.0};
    // squared norms: thread t sums row (t & 63) of tile ((t >> 6) & 1) over k half t >> 7 of every
    // chunk (all four waves share the work; lane-rotated k order spreads the LDS banks; the order
    // is fixed per row, so a layer's norms do not depend on the launch)
    double nacc = 0.0;
    const int nt_r = tid & 63, nt_t = (tid >> 6) & 1, nt_h = tid >> 7;
    if (tid < 2 * kDmT) rmx[tid >> 6][tid & 63] = 0;
    // register prefetch two chunks deep (r03): chunks c + 1 and c + 2 are in flight while chunk
    // c feeds the MFMAs (one chunk ahead left the kernel waiting on MALL/HBM latency, not on the
    // MFMA pipe).  A diagonal tile (bi == bj) loads and stages its row panel once and reads the
    // B operand from the A panel.
    constexpr int kDmG = kDmKC / 4, kDmU = 2 * kDmT * kDmG / 256;  // 4-element groups per row, per thread
    const bool diag = bi == bj;
    int kbeg = 0, kend = D;  // this slice's K range (whole chunks)
    if (SPLIT) {
        const int C = (D + kDmKC - 1) / kDmKC, S = (int)gridDim.z, z = (int)blockIdx.z;
        kbeg = (int)((int64_t)C * z / S) * kDmKC;
        kend = min(D, (int)((int64_t)C * (z + 1) / S) * kDmKC);
    }
    const bool vec4 = (D & 3) == 0;  // rows 16-B aligned: one 4-element load per group
    auto load = [&](T (&pr)[kDmU][4], int k0) {
        const int kc = min(kDmKC, kend - k0);
#pragma unroll
        for (int u = 0; u < kDmU; ++u) {  // 2 tiles x 64 rows x kDmKC / 4 groups of 4 consecutive k
            const int e = tid + 256 * u, t = e / (kDmT * kDmG), r = (e / kDmG) % kDmT, c0 = (e % kDmG) * 4;
            const int g = (t ? bj : bi) * kDmT + r;
            const T* src = Xl + (size_t)g * D + k0 + c0;
            const bool live = g < n && !(diag && t);
            if (live && vec4 && c0 + 4 <= kc) {
                if constexpr (sizeof(T) == 4) {
                    const float4 v = *(const float4*)src;
                    pr[u][0] = v.x, pr[u][1] = v.y, pr[u][2] = v.z, pr[u][3] = v.w;
                } else {
                    const double2 v0 = *(const double2*)src, v1 = *(const double2*)(src + 2);
                    pr[u][0] = v0.x, pr[u][1] = v0.y, pr[u][2] = v1.x, pr[u][3] = v1.y;
                }
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) pr[u][q] = (live && c0 + q < kc) ? src[q] : (T)0;
            }
        }
    };
    auto stage = [&](const T (&pr)[kDmU][4], int buf) {
#pragma unroll
        for (int u = 0; u < kDmU; ++u) {
            const int e = tid + 256 * u, t = e / (kDmT * kDmG), r = (e / kDmG) % kDmT, c0 = (e % kDmG) * 4;
            if (diag && t) continue;
#pragma unroll
            for (int q = 0; q < 4; ++q) xs[buf][t][r][c0 + q] = pr[u][q];
        }
    };
    // 16x16 blocks of this wave's 32x32 quadrant that hold an output entry
    // (i <= j, both < n): the padding rows of the last tile row/column and the
    // blocks below a diagonal tile's diagonal are skipped (wave-uniform).  At
    // N = 144 that is 45 of the 96 blocks of the six upper tiles (r03).
    bool need[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int ri0 = bi * kDmT + wr * 32 + a * 16, cj0 = bj * kDmT + wc * 32 + b * 16;
            need[a][b] = ri0 < n && cj0 < n && ri0 <= cj0 + 15;
        }
    const int tb = diag ? 0 : 1;    // panel of the B operand
    const int tn = diag ? 0 : nt_t;  // panel of this thread's norm rows
    auto compute = [&](int buf) {
#pragma unroll 8
        for (int cc = 0; cc < kDmKC / 2; ++cc) {  // zero padding adds exact zeros
            const double v = (double)xs[buf][tn][nt_r][nt_h * (kDmKC / 2) + ((cc + nt_r) & (kDmKC / 2 - 1))];
            nacc = fma(v, v, nacc);
        }
#pragma unroll
        for (int ks = 0; ks < kDmKC; ks += 4) {
            const int k = ks + (lane >> 4);
            double av[2], bv[2];
#pragma unroll
            for (int a = 0; a < 2; ++a) av[a] = (double)xs[buf][0][wr * 32 + a * 16 + (lane & 15)][k];
#pragma unroll
            for (int b = 0; b < 2; ++b) bv[b] = (double)xs[buf][tb][wc * 32 + b * 16 + (lane & 15)][k];
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    if (need[a][b]) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
        }
    };
    T pa[kDmU][4], pb[kDmU][4];
    const int nch = (kend - kbeg + kDmKC - 1) / kDmKC;
    load(pa, kbeg);
    if (nch > 1) load(pb, kbeg + kDmKC);
    stage(pa, 0);
    __syncthreads();
    // two chunks per trip: chunk c (buffer 0, pb holds c + 1), then c + 1 (buffer 1, pa holds c + 2);
    // a buffer is restaged only after the barrier that its last readers passed
    for (int c = 0; c < nch; c += 2) {
        if (c + 2 < nch) load(pa, kbeg + (c + 2) * kDmKC);
        compute(0);
        if (c + 1 < nch) stage(pb, 1);
        __syncthreads();
        if (c + 1 >= nch) break;
        if (c + 3 < nch) load(pb, kbeg + (c + 3) * kDmKC);
        compute(1);
        if (c + 2 < nch) stage(pa, 0);
        __syncthreads();
    }
    nrp[nt_h][nt_t][nt_r] = nacc;
    __syncthreads();
    if (tid < 2 * kDmT) nrm[tid >> 6][tid & 63] = nrp[0][tid >> 6][tid & 63] + nrp[1][tid >> 6][tid & 63];
    __syncthreads();
    if constexpr (SPLIT) {
        const size_t zo = ((size_t)l * gridDim.z + blockIdx.z);
        double* G = gpart + zo * n * n;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = bi * kDmT + wr * 32 + a * 16 + (lane >> 4) + 4 * r, j = bj * kDmT + wc * 32 + b * 16 + (lane & 15);
                    if (i < n && j < n && i < j) G[(size_t)i * n + j] = acc[a][b][r];
                }
        if (bi == bj && tid < kDmT && bi * kDmT + tid < n) npart[zo * n + bi * kDmT + tid] = nrm[0][tid];
        return;
    }
    if constexpr (METRIC == 2) {  // raw f64 Gram matrix into gpart [L][n][n] (effective dimensionality)
        double* G = gpart + (size_t)l * n * n;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = bi * kDmT + wr * 32 + a * 16 + (lane >> 4) + 4 * r, j = bj * kDmT + wc * 32 + b * 16 + (lane & 15);
                    if (i >= n || j >= n || j < i) continue;
                    G[(size_t)i * n + j] = acc[a][b][r];
                    G[(size_t)j * n + i] = acc[a][b][r];
                }
        return;
    }
    float* Dl = dist + (size_t)l * n * n;
    // C/D map of v_mfma_f64_16x16x4_f64: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ri = wr * 32 + a * 16 + (lane >> 4) + 4 * r, cj = wc * 32 + b * 16 + (lane & 15);
                const int i = bi * kDmT + ri, j = bj * kDmT + cj;
                if (i >= n || j >= n || j < i) continue;
                if (i == j) {
                    Dl[(size_t)i * n + i] = 0.0f;
                    if (dist64) dist64[((size_t)l * n + i) * n + i] = 0.0;
                    continue;
                }
                double d = (-2.0 * acc[a][b][r] + nrm[0][ri]) + nrm[1][cj];
                float f;
                if constexpr (METRIC == 1) {
                    const double ni = nrm[0][ri], nj = nrm[1][cj];
                    d = (ni == 0.0 && nj == 0.0) ? 0.0 : (ni == 0.0 || nj == 0.0) ? 1.0 : 1.0 - acc[a][b][r] / sqrt(ni * nj);
                    f = fmaxf((float)d, 0.0f);
                } else if constexpr (sizeof(T) == 4) {
                    f = (float)d;
                    f = (f != f) ? f : fmaxf(f, 0.0f);
                    f = sqrt_rn_f32(f);
                } else {
                    d = (d != d) ? d : fmax(d, 0.0);
                    const double r64 = __dsqrt_rn(d);
                    f = (float)r64;
                    if (dist64) dist64[((size_t)l * n + i) * n + j] = dist64[((size_t)l * n + j) * n + i] = r64 + 0.0;
                }
                f = f + 0.0f;
                Dl[(size_t)i * n + j] = f;
                Dl[(size_t)j * n + i] = f;
                atomicMax(&rmx[0][ri], __float_as_uint(f));
                atomicMax(&rmx[1][cj], __float_as_uint(f));
            }
    __syncthreads();
    uint32_t* rm = rowmax + (size_t)l * n;
    if (tid < 2 * kDmT) {
        const int t = tid >> 6, r = tid & 63, g = (t ? bj : bi) * kDmT + r;
        if (g < n && rmx[t][r]) atomicMax(&rm[g], rmx[t][r]);
    }
}

// N <= 144 (r03): the whole upper triangle of a layer's Gram matrix in one
// workgroup per (K slice, layer).  The layer's rows of a K chunk are staged in
// LDS once and every one of the nb(nb+1)/2 16x16 blocks (45 at N = 144) is an
// accumulator of one of the four waves (block q -> wave q % 4, <= 12 each), so
// every row is read from HBM once per slice (k_distance_mfma's 64-row tiles
// read each panel once per tile of its row and column: 3.1x the input at
// N = 144) and the MFMA work is spread evenly over the waves.  Partial Gram
// entries (i < j) and row norms per slice go to k_distance_combine, the same
// fixed-order combine as the tiled split.  f32 input, Euclidean.
constexpr int kGlMaxNB = 9, kGlMaxN = 16 * kGlMaxNB, kGlMB = (kGlMaxNB * (kGlMaxNB + 1) / 2 + 3) / 4;
__global__ __launch_bounds__(256) void k_gram_layer(const float* __restrict__ X, int n, int D, double* __restrict__ gpart,
                                                    double* __restrict__ npart) {
    __shared__ float xs[2][kGlMaxN][kDmS];
    const int l = blockIdx.y, z = blockIdx.x, S = gridDim.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int nb = (n + 15) >> 4, np = nb * 16, nblk = nb * (nb + 1) / 2;
    const float* Xl = X + (size_t)l * n * D;
    const int C = (D + kDmKC - 1) / kDmKC;
    const int kbeg = (int)((int64_t)C * z / S) * kDmKC, kend = min(D, (int)((int64_t)C * (z + 1) / S) * kDmKC);
    // this wave's blocks: q = wv, wv + 4, ... of the row-major upper triangle
    int bi[kGlMB], bj[kGlMB];
    int nw = 0;
#pragma unroll
    for (int u = 0; u < kGlMB; ++u) {
        int q = wv + 4 * u, r = 0;
        bi[u] = bj[u] = 0;
        if (q < nblk) {
            while (q >= nb - r) q -= nb - r, ++r;
            bi[u] = r, bj[u] = r + q;
            nw = u + 1;
        }
    }
    dm_d4 acc[kGlMB];
#pragma unroll
    for (int u = 0; u < kGlMB; ++u) acc[u] = dm_d4{0.0, 0.0, 0.0, 0.0};
    double nacc = 0.0;  // row tid's squared norm over this slice, k in order
    constexpr int kG = kDmKC / 4;                         // 4-element groups per row
    constexpr int kU = (kGlMaxN * kG + 255) / 256;        // groups per thread per chunk
    float pre[kU][4];
    const bool vec4 = (D & 3) == 0;
    auto load = [&](int k0) {
        const int kc = min(kDmKC, kend - k0);
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int e = tid + 256 * u, r = e / kG, c0 = (e % kG) * 4;
            const float* src = Xl + (size_t)r * D + k0 + c0;
            const bool live = r < n && e < np * kG;
            if (live && vec4 && c0 + 4 <= kc) {
                const float4 v = *(const float4*)src;
                pre[u][0] = v.x, pre[u][1] = v.y, pre[u][2] = v.z, pre[u][3] = v.w;
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) pre[u][q] = (live && c0 + q < kc) ? src[q] : 0.0f;
            }
        }
    };
    auto stage = [&](int buf) {
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int e = tid + 256 * u, r = e / kG, c0 = (e % kG) * 4;
            if (e < np * kG)
#pragma unroll
                for (int q = 0; q < 4; ++q) xs[buf][r][c0 + q] = pre[u][q];
        }
    };
    load(kbeg);
    stage(0);
    __syncthreads();
    int buf = 0;
    for (int k0 = kbeg; k0 < kend; k0 += kDmKC, buf ^= 1) {
        const bool more = k0 + kDmKC < kend;
        if (more) load(k0 + kDmKC);  // global loads in flight under this chunk's MFMAs
        if (tid < n) {
#pragma unroll 8
            for (int c = 0; c < kDmKC; ++c) {  // zero padding adds exact zeros
                const double v = (double)xs[buf][tid][c];
                nacc = fma(v, v, nacc);
            }
        }
#pragma unroll
        for (int ks = 0; ks < kDmKC; ks += 4) {
            const int k = ks + (lane >> 4);
#pragma unroll
            for (int u = 0; u < kGlMB; ++u)
                if (u < nw) {
                    const double av = (double)xs[buf][bi[u] * 16 + (lane & 15)][k];
                    const double bv = (double)xs[buf][bj[u] * 16 + (lane & 15)][k];
                    acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[u], 0, 0, 0);
                }
        }
        if (more) stage(buf ^ 1);  // the other buffer: its last readers passed the previous barrier
        __syncthreads();
    }
    const size_t zo = (size_t)l * S + z;
    double* G = gpart + zo * n * n;
    // C/D map of v_mfma_f64_16x16x4_f64: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
    for (int u = 0; u < kGlMB; ++u)
        if (u < nw)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = bi[u] * 16 + (lane >> 4) + 4 * r, j = bj[u] * 16 + (lane & 15);
                if (i < n && j < n && i < j) G[(size_t)i * n + j] = acc[u][r];
            }
    if (tid < n) npart[zo * n + tid] = nacc;
}

// the K slices of k_distance_mfma<..., SPLIT>: fixed-order sums, then the same epilogue
template <typename T, int METRIC = 0>
__global__ __launch_bounds__(256) void k_distance_combine(const double* __restrict__ gpart, const double* __restrict__ npart, int S, int n,
                                                          float* __restrict__ dist, uint32_t* __restrict__ rowmax,
                                                          double* __restrict__ dist64 = nullptr) {
    const int l = blockIdx.y;
    const size_t nn = (size_t)n * n;
    float* Dl = dist + (size_t)l * nn;
    uint32_t* rm = rowmax + (size_t)l * n;
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < nn; q += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(q / n), j = (int)(q - (size_t)i * n);
        if (i == j) {
            Dl[q] = 0.0f;
            if (dist64) dist64[(size_t)l * nn + q] = 0.0;
        }
        if (i >= j) continue;
        double g = 0.0, ni = 0.0, nj = 0.0;
        for (int z = 0; z < S; ++z) {
            const size_t zo = (size_t)l * S + z;
            g += gpart[zo * nn + q];
            ni += npart[zo * n + i];
            nj += npart[zo * n + j];
        }
        float f;
        if constexpr (METRIC == 1) {
            const double d = (ni == 0.0 && nj == 0.0) ? 0.0 : (ni == 0.0 || nj == 0.0) ? 1.0 : 1.0 - g / sqrt(ni * nj);
            f = fmaxf((float)d, 0.0f);
        } else if constexpr (sizeof(T) == 4) {
            f = (float)((-2.0 * g + ni) + nj);
            f = (f != f) ? f : fmaxf(f, 0.0f);
            f = sqrt_rn_f32(f);
        } else {
            double d = (-2.0 * g + ni) + nj;
            d = (d != d) ? d : fmax(d, 0.0);
            const double r64 = __dsqrt_rn(d);
            f = (float)r64;
            if (dist64) dist64[(size_t)l * nn + q] = dist64[(size_t)l * nn + (size_t)j * n + i] = r64 + 0.0;
        }
        f = f + 0.0f;
        Dl[q] = f;
        Dl[(size_t)j * n + i] = f;
    }
    (void)rm;  // row maxima: k_rowmax after this kernel (per-element atomics on N row words serialised: r03 89 us)
}

// row maxima of a square distance matrix (distance-matrix inputs): one wave per row
__global__ __launch_bounds__(256) void k_rowmax(const float* __restrict__ dist, int n, uint32_t* __restrict__ rowmax) {
    const int l = blockIdx.y, w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, ln = threadIdx.x & 63;
    if (w >= n) return;
    const float* row = dist + ((size_t)l * n + w) * n;
    float m = 0.0f;
    for (int j = ln; j < n; j += 64) m = fmaxf(m, row[j]);
    for (int k = 32; k >= 1; k >>= 1) m = fmaxf(m, __shfl_xor(m, k, 64));
    if (ln == 0) rowmax[(size_t)l * n + w] = __float_as_uint(m);
}

// threshold of layer l: the user's, or the enclosing radius min_i rowmax[i]
__device__ __forceinline__ float block_thresh(const uint32_t* __restrict__ rowmax, int n, float user_thresh, uint32_t* s_min) {
    if (!(isinf(user_thresh) || user_thresh == 3.402823466e+38f)) return user_thresh;
    if (threadIdx.x == 0) *s_min = 0xFFFFFFFFu;
    __syncthreads();
    uint32_t m = 0xFFFFFFFFu;
    for (int i = threadIdx.x; i < n; i += blockDim.x) m = min(m, rowmax[i]);
    if (threadIdx.x < n) atomicMin(s_min, m);  // only lanes that read a row (1024-thread blocks: no 1024-way LDS conflict)
    __syncthreads();
    const float r = __uint_as_float(*s_min);
    __syncthreads();
    return n == 1 ? 0.0f : r;
}

// distance-matrix input: ripser.py condenses dm[I > J] (upper triangle,
// row-major) to float32; we symmetrise from the upper triangle.
template <typename T>
__global__ __launch_bounds__(256) void k_square_dist(const T* __restrict__ M, int n, float* __restrict__ dist) {
    const int l = blockIdx.y;
    const T* Ml = M + (size_t)l * n * n;
    float* Dl = dist + (size_t)l * n * n;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < (size_t)n * n; e += (size_t)gridDim.x * blockDim.x) {
        int i = (int)(e / n), j = (int)(e % n);
        float v;
        if (i == j)
            v = 0.0f;
        else if (i < j)
            v = (float)Ml[(size_t)i * n + j];
        else
            v = (float)Ml[(size_t)j * n + i];
        Dl[e] = v + 0.0f;
    }
}

// condensed vector (i<j row-major) -> square
__global__ __launch_bounds__(256) void k_square_from_condensed(const float* __restrict__ c, int n, float* __restrict__ dist) {
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < (size_t)n * n; e += (size_t)gridDim.x * blockDim.x) {
        int i = (int)(e / n), j = (int)(e % n);
        float v = 0.0f;
        if (i != j) {
            int a = i < j ? i : j, b = i < j ? j : i;
            // offset of (a,b), a<b, in row-major strict upper triangle
            size_t off = (size_t)a * (2 * (size_t)n - a - 1) / 2 + (b - a - 1);
            v = c[off];
        }
        dist[e] = v + 0.0f;
    }
}

// ------------------------------------------------------------------ block sort
// Ascending sort of n u64 keys (with optional u32 payload) by ONE workgroup.
// n <= LDS chunk: bitonic in LDS.  Larger: chunk-sort + merge-path merges in
// global memory (ping-pong with tmp).  Result ends in `keys`.
template <bool KV>
__device__ void block_sort(uint64_t* keys, uint32_t* vals, uint64_t n, uint64_t* tkeys, uint32_t* tvals, uint64_t* sk,
                           uint32_t* sv, int chunk_log2) {
    const int T = blockDim.x, t = threadIdx.x;
    const uint64_t CH = 1ull << chunk_log2;
    // 1) chunk sorts in LDS
    for (uint64_t c0 = 0; c0 < n; c0 += CH) {
        uint64_t m = min(CH, n - c0);
        uint32_t p2 = 1;
        while (p2 < m) p2 <<= 1;
        for (uint32_t e = t; e < p2; e += T) {
            sk[e] = e < m ? keys[c0 + e] : kEmpty64;
            if (KV) sv[e] = e < m ? vals[c0 + e] : 0u;
        }
        __syncthreads();
        for (uint32_t k = 2; k <= p2; k <<= 1) {
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t e = t; e < p2; e += T) {
                    uint32_t x = e ^ j;
                    if (x > e) {
                        bool up = (e & k) == 0;
                        uint64_t a = sk[e], b = sk[x];
                        if ((a > b) == up) {
                            sk[e] = b;
                            sk[x] = a;
                            if (KV) {
                                uint32_t va = sv[e];
                                sv[e] = sv[x];
                                sv[x] = va;
                            }
                        }
                    }
                }
                __syncthreads();
            }
        }
        for (uint32_t e = t; e < m; e += T) {
            keys[c0 + e] = sk[e];
            if (KV) vals[c0 + e] = sv[e];
        }
        __syncthreads();
    }
    if (n <= CH) return;
    // 2) merge passes, ping-pong keys <-> tkeys
    uint64_t* src = keys;
    uint64_t* dst = tkeys;
    uint32_t* vsrc = vals;
    uint32_t* vdst = tvals;
    for (uint64_t w = CH; w < n; w <<= 1) {
        for (uint64_t a0 = 0; a0 < n; a0 += 2 * w) {
            uint64_t a1 = min(a0 + w, n), b1 = min(a0 + 2 * w, n);
            uint64_t la = a1 - a0, lb = b1 - a1, m = la + lb;
            uint64_t per = (m + T - 1) / T;
            uint64_t d0 = min(per * t, m), d1 = min(per * (t + 1), m);
            // merge path split for diagonal d: i from A, d-i from B
            auto split = [&](uint64_t d) {
                uint64_t lo = d > lb ? d - lb : 0, hi = min(d, la);
                while (lo < hi) {
                    uint64_t mid = (lo + hi) >> 1;
                    // take A[mid] before B[d-mid-1]?
                    if (src[a0 + mid] <= src[a1 + d - mid - 1])
                        lo = mid + 1;
                    else
                        hi = mid;
                }
                return lo;
            };
            uint64_t ia = split(d0), ib = d0 - ia;
            for (uint64_t o = d0; o < d1; ++o) {
                bool takeA = ib >= lb || (ia < la && src[a0 + ia] <= src[a1 + ib]);
                if (takeA) {
                    dst[a0 + o] = src[a0 + ia];
                    if (KV) vdst[a0 + o] = vsrc[a0 + ia];
                    ++ia;
                } else {
                    dst[a0 + o] = src[a1 + ib];
                    if (KV) vdst[a0 + o] = vsrc[a1 + ib];
                    ++ib;
                }
            }
        }
        __syncthreads();
        uint64_t* tk = src;
        src = dst;
        dst = tk;
        uint32_t* tv = vsrc;
        vsrc = vdst;
        vdst = tv;
    }
    if (src != keys) {
        for (uint64_t e = t; e < n; e += T) {
            keys[e] = src[e];
            if (KV) vals[e] = vsrc[e];
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ H0
// Threshold (ripser.py rips_dm: enclosing radius when thresh is inf/FLT_MAX),
// num_edges, minimum spanning forest under the total order (diam asc, idx
// desc) by Prim (one wave, N <= 190) or Borůvka (block) -- the unique forest,
// i.e. Kruskal's -- then Kruskal-order emission and
// elder-rule union-find [upstream compute_dim_0_pairs], consumed at
// debug_tda_pipeline.py:112, :126.
// LDS: best[N] u64, intree[N] u8 ... par[N] int  (N <= 8192)
//
// n <= kH0WaveMaxN (64 < n, the dense path has k_h0_wave below): the layer's
// matrix is staged in LDS after the sort chunk and Prim runs on wave 0 alone
// -- lane l owns vertices l, l + 64, l + 128; the frontier keys live in
// registers and a step is an LDS row read + a DPP wave minimum, no block
// barriers; the threshold and edge count read the LDS copy too (r02:
// 32 x N=144 layers 0.47 -> 0.30 ms; the sequential thread-0 elder-rule
// pass that follows is not parallelised yet).
// Template: WQ = vertices per lane of the one-wave path (0: the block path
// above), LROWS = rows staged in LDS.  The one-wave path with rows read from
// global memory (WQ = 16, N = 1024) measured slower than the block path
// (torus1024: 3.95 vs 3.57 ms, latency-bound row loads), so above N = 190 the
// block path stays.
// ------------------------------------------------------------------ H0 above N = kH0WaveMaxN: Borůvka over the GPU
// (r03; replaces a block-wide Prim of N - 1 dependent steps, torus1024 3.6 ms).
// k_bor_init: threshold (enclosing radius = min row maximum) and per-layer
// state; then ceil(log2 N) rounds of k_bor_min (one wave per vertex: its
// cheapest edge <= thresh to another component under the total order (diam
// asc, idx desc) -> atomicMin on its component's slot; round 0 also counts
// num_edges) and k_bor_hook (one workgroup per layer, in LDS: every root
// hooks to the other endpoint's root -- keys are unique, so the only cycles
// are mutual pairs, whose smaller root stays -- the hooking edges are the
// new forest edges, pointer jumping flattens the components).  The forest is
// the unique minimum spanning forest of the total order, i.e. Kruskal's;
// k_h0<0, false> then sorts it and runs the elder rule.
struct BorCtl {
    unsigned long long nmst;  // forest edges found
    uint32_t done, pad;
};

__global__ __launch_bounds__(256) void k_bor_init(const uint32_t* __restrict__ rowmax, int n, float user_thresh,
                                                  LayerStats* __restrict__ stats, int32_t* __restrict__ comp,
                                                  uint64_t* __restrict__ cheap, BorCtl* __restrict__ ctl) {
    __shared__ uint32_t s_min;
    const int l = blockIdx.x;
    const float thr = block_thresh(rowmax + (size_t)l * n, n, user_thresh, &s_min);
    for (int v = threadIdx.x; v < n; v += blockDim.x) {
        comp[(size_t)l * n + v] = v;
        cheap[(size_t)l * n + v] = kEmpty64;
    }
    if (threadIdx.x == 0) {
        stats[l].thresh = thr;
        stats[l].num_edges = 0;
        ctl[l].nmst = 0;
        ctl[l].done = 0;
    }
}

constexpr int kBorLoads = 8;  // row loads in flight per lane
__global__ __launch_bounds__(256) void k_bor_min(const float* __restrict__ dist, int n, LayerStats* __restrict__ stats,
                                                 const int32_t* __restrict__ comp, uint64_t* __restrict__ cheap,
                                                 const BorCtl* __restrict__ ctl, int first) {
    const int l = blockIdx.y, u = blockIdx.x * 4 + (threadIdx.x >> 6), ln = threadIdx.x & 63;
    if (u >= n || ctl[l].done) return;
    const float thr = stats[l].thresh;
    const float* row = dist + ((size_t)l * n + u) * n;
    const int32_t* cl = comp + (size_t)l * n;
    const int cu = cl[u];
    uint64_t mk = kEmpty64;
    unsigned long long cnt = 0;
    for (int v0 = 0; v0 < n; v0 += 64 * kBorLoads) {
        float d[kBorLoads];
        int32_t c[kBorLoads];
#pragma unroll
        for (int q = 0; q < kBorLoads; ++q) {
            const int v = v0 + ln + 64 * q;
            d[q] = v < n ? row[v] : INFINITY;
            c[q] = v < n ? cl[v] : cu;
        }
#pragma unroll
        for (int q = 0; q < kBorLoads; ++q) {
            const int v = v0 + ln + 64 * q;
            if (!(d[q] <= thr)) continue;
            cnt += v > u;
            if (c[q] == cu) continue;
            const int a = u > v ? u : v, b = u > v ? v : u;
            const uint64_t k = filt_key(d[q], binom((uint64_t)a, 2) + b);
            mk = k < mk ? k : mk;
        }
    }
    mk = wave_min_u64(mk);
    if (ln == 0 && mk != kEmpty64) atomicMin((unsigned long long*)&cheap[(size_t)l * n + cu], (unsigned long long)mk);
    if (first) {
        cnt = wave_sum_u64(cnt);
        if (ln == 0 && cnt) atomicAdd((unsigned long long*)&stats[l].num_edges, cnt);
    }
}

// LDS: comp n x i32 | hook n x i32 | cheap n x u64
__global__ __launch_bounds__(1024) void k_bor_hook(int n, int32_t* __restrict__ comp, uint64_t* __restrict__ cheap,
                                                   BorCtl* __restrict__ ctl, uint64_t* __restrict__ scratch /* [L][2n] */) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ uint32_t flag[2], s_any;
    const int l = blockIdx.x, t = threadIdx.x, T = blockDim.x;
    if (ctl[l].done) return;
    int32_t* cs = (int32_t*)smem;
    int32_t* hook = cs + ((n + 3) & ~3);
    uint64_t* ch = (uint64_t*)(hook + ((n + 3) & ~3));
    int32_t* cg = comp + (size_t)l * n;
    uint64_t* chg = cheap + (size_t)l * n;
    uint64_t* mst = scratch + (size_t)l * 2 * n;
    for (int v = t; v < n; v += T) {
        cs[v] = cg[v];
        ch[v] = chg[v];
        chg[v] = kEmpty64;  // ready for the next round
    }
    if (t < 2) flag[t] = 0;
    if (t == 0) s_any = 0;
    __syncthreads();
    for (int r = t; r < n; r += T) {
        hook[r] = r;
        if (cs[r] != r || ch[r] == kEmpty64) continue;
        s_any = 1;
        const uint64_t eidx = 0xFFFFFFFFull - (ch[r] & 0xFFFFFFFFull);
        const int a = max_vertex(eidx, 2, n - 1), b = (int)(eidx - binom((uint64_t)a, 2));
        const int ca = cs[a], cb = cs[b];
        const int other = ca == r ? cb : ca;
        if (ch[other] == ch[r] && r < other) continue;  // the smaller root of a mutual pair stays a root
        hook[r] = other;
        const unsigned long long pos = atomicAdd(&ctl[l].nmst, 1ull);
        if (pos < (unsigned long long)n) mst[pos] = ch[r];  // every forest edge once: a mutual edge by its larger root
    }
    __syncthreads();
    if (!s_any) {  // no component has an edge <= thresh to another: the forest is complete
        if (t == 0) ctl[l].done = 1;
        return;
    }
    for (int it = 0; it < 32; ++it) {  // pointer jumping on the hook forest (depth < n)
        bool ch2 = false;
        for (int r = t; r < n; r += T) {
            const int h = hook[r], hh = hook[h];
            if (h != hh) {
                hook[r] = hh;
                ch2 = true;
            }
        }
        if (ch2) flag[it & 1] = 1;
        __syncthreads();
        const bool again = flag[it & 1] != 0;
        __syncthreads();
        if (t == 0) flag[it & 1] = 0;
        if (!again) break;
    }
    for (int v = t; v < n; v += T) cg[v] = hook[cs[v]];
}

constexpr int kH0WaveMaxN = 190;  // 4 n^2 B of LDS staging
constexpr int kH0WaveQ = (kH0WaveMaxN + 63) / 64;
constexpr int kH0BorWQ = 16;  // Borůvka path: one-wave elder rule with register labels up to N = 1024
template <int WQ, bool LROWS, bool BOR = false>
__global__ __launch_bounds__(1024) void k_h0(const float* __restrict__ dist, int n, float user_thresh,
                                             LayerStats* __restrict__ stats, uint32_t* __restrict__ mst_bits,
                                             uint64_t mst_words, Pair* __restrict__ pairs0, uint64_t pcap0,
                                             uint64_t* __restrict__ scratch /* [L][2n] */, int sort_log2,
                                             const BorCtl* __restrict__ bctl = nullptr) {
    constexpr bool dlds = LROWS;   // the layer's matrix is staged in LDS
    // BOR: the forest, threshold and num_edges come from k_bor_* (N > kH0WaveMaxN); WQ > 0
    // then sizes the one-wave elder rule's register labels (N <= 64 WQ), else thread 0 runs it
    constexpr bool wave = WQ > 0 && !BOR;  // one-wave Prim (+ threshold / num_edges here)
    constexpr bool welder = WQ > 0;        // one-wave elder rule
    constexpr int QA = WQ > 0 ? WQ : 1;  // register-array extent (unused when !wave)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.x, T = blockDim.x, t = threadIdx.x;
    const float* Dl = dist + (size_t)l * n * n;
    LayerStats* st = stats + l;
    // dynamic LDS (16-B aligned carve, no static __shared__: Guideline 17)
    unsigned long long& s_cnt = *(unsigned long long*)smem;
    float& s_thresh = *(float*)(smem + 8);
    int& s_cur = *(int*)(smem + 12);
    uint64_t* best = (uint64_t*)(smem + 16);              // n
    int* par = (int*)(best + n);                          // n
    uint64_t* red = (uint64_t*)(par + ((n + 1) & ~1));    // 32 wave partials + 8
    uint64_t* sk = red + 40;                              // sort chunk
    const int nw = T >> 6, w = t >> 6, ln = t & 63;
    float* Ds = (float*)(sk + (1ull << sort_log2));       // dlds: the layer's matrix
#ifdef TDA_PROFILE
    const uint64_t h0t0 = clock64();
#define H0M(i) if (t == 0 && l == 0) st->prof[0][i] = clock64() - h0t0;
#else
#define H0M(i)
#endif
    if (dlds) {
        stage_to_lds(Ds, Dl, 4ull * n * n, t, T);
        __syncthreads();
    }
    H0M(0)

    uint64_t* mst = scratch + (size_t)l * 2 * n;  // MST edge keys
    int nmst = 0;
    float thr = user_thresh;
    if constexpr (wave) {
        // -- threshold
        if (isinf(user_thresh) || user_thresh == 3.402823466e+38f) {
            float local = INFINITY;
            for (int i = w; i < n; i += nw) {
                float r = 0.0f;  // distances are >= 0 (the diagonal is 0): the bits order like the values
                for (int j = ln; j < n; j += 64) r = fmaxf(r, dlds ? ld_lds(Ds, (size_t)i * n + j) : Dl[(size_t)i * n + j]);
                local = fminf(local, __uint_as_float(wave_max_u32(__float_as_uint(r))));  // DPP, no LDS round trips
            }
            if (ln == 0) ((float*)red)[w] = local;
            __syncthreads();
            if (t == 0) {
                float e = INFINITY;
                for (int q = 0; q < nw; ++q) e = fminf(e, ((float*)red)[q]);
                s_thresh = e;
            }
            __syncthreads();
            thr = s_thresh;
        }
        // -- num_edges
        if (t == 0) s_cnt = 0;
        __syncthreads();
        {
            unsigned long long c = 0;
            for (int i = w; i < n; i += nw)
                for (int j = i + 1 + ln; j < n; j += 64) c += (dlds ? ld_lds(Ds, (size_t)i * n + j) : Dl[(size_t)i * n + j]) <= thr;
            c = wave_sum_u64(c);  // one LDS atomic per wave, not per thread
            if (ln == 0) atomicAdd(&s_cnt, c);
        }
        __syncthreads();
        if (t == 0) {
            st->thresh = thr;
            st->num_edges = (int64_t)s_cnt;
        }
    } else {
        // the forest, threshold and num_edges come from k_bor_* (one pass per Borůvka round over the whole GPU)
        nmst = (int)min(bctl[l].nmst, (unsigned long long)n);
        thr = st->thresh;
    }
    (void)s_cur;
    (void)best;
    (void)thr;
    H0M(1)
    if constexpr (wave && LROWS) {
        // Borůvka on the whole workgroup over the LDS-staged rows (r03; the
        // one-wave Prim it replaces took N - 1 dependent steps: 32 x N=144
        // 0.16 ms): every round each vertex's cheapest edge to another
        // component (one wave per vertex), component minima by LDS
        // atomicMin, roots hook to the other endpoint's root (unique keys:
        // only mutual pairs form cycles, the smaller root stays), pointer
        // jumping.  The unique minimum spanning forest, as k_bor_* and Prim.
        int* comp = par;                         // n
        int* hook = (int*)(Ds + (size_t)n * n);  // n (carved by the host after the rows)
        uint64_t* cheap = best;                  // n
        int orp = 0;
        auto block_or = [&](bool p) {  // via red[36 + parity]: no static LDS in this kernel
            uint64_t* f = red + 36 + (orp++ & 1);
            if (p) *f = 1;
            __syncthreads();
            const bool r = *f != 0;
            __syncthreads();
            if (t == 0) *f = 0;
            return r;
        };
        for (int v = t; v < n; v += T) comp[v] = v;
        if (t == 0) red[35] = red[36] = red[37] = 0;
        __syncthreads();
        for (int round = 0; round < 64; ++round) {
            for (int v = t; v < n; v += T) cheap[v] = kEmpty64;
            __syncthreads();
            for (int u = w; u < n; u += nw) {
                const int cu = comp[u];
                uint64_t mk = kEmpty64;
                for (int v = ln; v < n; v += 64) {
                    const float d = ld_lds(Ds, (size_t)u * n + v);
                    if (d <= thr && comp[v] != cu) {
                        const int a = u > v ? u : v, b = u > v ? v : u;
                        const uint64_t k = filt_key(d, binom((uint64_t)a, 2) + b);
                        mk = k < mk ? k : mk;
                    }
                }
                mk = wave_min_u64(mk);
                if (ln == 0 && mk != kEmpty64) atomicMin((unsigned long long*)&cheap[cu], (unsigned long long)mk);
            }
            __syncthreads();
            bool any = false;
            for (int r = t; r < n; r += T) {
                hook[r] = r;
                if (comp[r] != r || cheap[r] == kEmpty64) continue;
                any = true;
                const uint64_t eidx = 0xFFFFFFFFull - (cheap[r] & 0xFFFFFFFFull);
                const int a = max_vertex(eidx, 2, n - 1), b = (int)(eidx - binom((uint64_t)a, 2));
                const int ca = comp[a], cb = comp[b];
                const int other = ca == r ? cb : ca;
                if (cheap[other] == cheap[r] && r < other) continue;  // the smaller root of a mutual pair stays
                hook[r] = other;
                mst[atomicAdd((unsigned long long*)&red[35], 1ull)] = cheap[r];
            }
            if (!block_or(any)) break;
            for (int it = 0; it < 32; ++it) {
                bool ch = false;
                for (int r = t; r < n; r += T) {
                    const int h = hook[r], hh = hook[h];
                    if (h != hh) {
                        hook[r] = hh;
                        ch = true;
                    }
                }
                if (!block_or(ch)) break;
            }
            for (int v = t; v < n; v += T) comp[v] = hook[comp[v]];
            __syncthreads();
        }
        nmst = (int)red[35];
        __syncthreads();
    } else if constexpr (wave) {  // one-wave Prim on rows from global memory
        if (w == 0) {
            uint64_t bst[QA];
            bool in[QA];
#pragma unroll
            for (int q = 0; q < WQ; ++q) {
                bst[q] = kEmpty64;
                in[q] = ln + 64 * q >= n || (ln == 0 && q == 0);  // vertex 0 starts the tree
            }
            int cur = 0;
            for (int it = 1; it < n; ++it) {
                uint64_t mk = kEmpty64;
#pragma unroll
                for (int q = 0; q < WQ; ++q) {
                    const int v = ln + 64 * q;
                    if (in[q]) continue;
                    const float d = LROWS ? ld_lds(Ds, (size_t)cur * n + v) : ld_glb(Dl, (size_t)cur * n + v);
                    if (d <= thr) {
                        const int a = cur > v ? cur : v, b = cur > v ? v : cur;
                        const uint64_t k = filt_key(d, binom((uint64_t)a, 2) + b);
                        bst[q] = k < bst[q] ? k : bst[q];
                    }
                    mk = bst[q] < mk ? bst[q] : mk;
                }
                const uint64_t gmin = wave_min_u64(mk);
                if (gmin == kEmpty64) {  // new component: the smallest vertex not in the forest
                    uint32_t sv = 0xFFFFFFFFu;
#pragma unroll
                    for (int q = WQ - 1; q >= 0; --q)
                        if (!in[q]) sv = (uint32_t)(ln + 64 * q);
                    cur = (int)wave_min_u32(sv);
                } else {  // the owner of the minimum key joins (keys are unique)
                    int nv = 0x7FFFFFFF;
#pragma unroll
                    for (int q = 0; q < WQ; ++q)
                        if (!in[q] && bst[q] == gmin) nv = ln + 64 * q;
                    cur = (int)wave_min_u32((uint32_t)nv);
                    if (ln == 0) mst[nmst] = gmin;
                    ++nmst;
                }
#pragma unroll
                for (int q = 0; q < WQ; ++q)
                    if (ln + 64 * q == cur) in[q] = true;
            }
        }
        if (w == 0 && ln == 0) red[34] = (uint64_t)nmst;
        __syncthreads();
        nmst = (int)red[34];
    }
    H0M(2)
    // -- Kruskal order of the forest edges
    block_sort<false>(mst, nullptr, (uint64_t)nmst, mst + n, nullptr, sk, nullptr, sort_log2);
    H0M(3)
    for (int e = t; e < nmst; e += T) {
        uint64_t eidx = 0xFFFFFFFFull - (mst[e] & 0xFFFFFFFFull);
        atomicOr(&mst_bits[(size_t)l * mst_words + (eidx >> 5)], 1u << (eidx & 31));
    }
    if constexpr (welder) {  // elder rule on wave 0: lane l holds the component labels (= max vertex) of vertices l, l + 64, ...
        if (w == 0) {
            int label[QA];
#pragma unroll
            for (int q = 0; q < WQ; ++q) label[q] = ln + 64 * q;
            auto lab_of = [&](int v) -> int {  // v wave-uniform
                int x = label[0];
#pragma unroll
                for (int q = 1; q < WQ; ++q)
                    if ((v >> 6) == q) x = label[q];
                return __builtin_amdgcn_readlane(x, v & 63);
            };
            Pair* P = pairs0 + (size_t)l * pcap0;
            uint64_t cs = 0;
            uint64_t cnt = 0;
            for (int e0 = 0; e0 < nmst; e0 += 64) {
                const int e = e0 + ln;
                const bool valid = e < nmst;
                const uint64_t k = valid ? mst[e] : 0;
                const uint64_t eidx = 0xFFFFFFFFull - (k & 0xFFFFFFFFull);
                const float d = __uint_as_float((uint32_t)(k >> 32));
                int a = 0, b = 0;
                if (valid) {
                    a = max_vertex(eidx, 2, n - 1);
                    b = (int)(eidx - binom((uint64_t)a, 2));
                }
                int my_young = 0;
                const int ne = min(64, nmst - e0);
                for (int j = 0; j < ne; ++j) {  // merges in Kruskal order
                    const int aj = __builtin_amdgcn_readlane(a, j), bj = __builtin_amdgcn_readlane(b, j);
                    const int ra = lab_of(aj), rb = lab_of(bj);
                    const int young = ra < rb ? ra : rb, old = ra < rb ? rb : ra;
#pragma unroll
                    for (int q = 0; q < WQ; ++q)
                        if (label[q] == young) label[q] = old;
                    if (ln == j) my_young = young;
                }
                if (valid) cs += pair_hash((uint64_t)my_young, eidx);
                const bool fin = valid && d > 0.0f;  // finite bars in Kruskal order
                const uint64_t m = __ballot(fin);
                const uint64_t pos = cnt + lanes_below(m);
                if (fin && pos < pcap0) P[pos] = Pair{0.0f, d, (int64_t)my_young, (int64_t)eidx};
                cnt += (uint64_t)__popcll(m);
            }
#pragma unroll
            for (int q = 0; q < WQ; ++q) {  // one [0, inf) bar per component, vertex order
                const int v = ln + 64 * q;
                const bool root = v < n && label[q] == v;
                const uint64_t m = __ballot(root);
                const uint64_t pos = cnt + lanes_below(m);
                if (root && pos < pcap0) P[pos] = Pair{0.0f, INFINITY, (int64_t)v, -1};
                cnt += (uint64_t)__popcll(m);
            }
            cs = wave_sum_u64(cs);
            if (ln == 0) {
                if (cnt > pcap0) {
                    st->err |= ERR_PAIR_CAP;
                    cnt = pcap0;
                }
                st->count[0] = (int64_t)cnt;
                st->checksum[0] = cs;
                st->all_pairs[0] = nmst;
                st->n_columns[0] = n;
            }
        }
        return;
    }
    for (int v = t; v < n; v += T) par[v] = v;
    __syncthreads();
    if (t == 0) {
        Pair* P = pairs0 + (size_t)l * pcap0;
        int64_t cnt = 0;
        uint64_t cs = 0;
        for (int e = 0; e < nmst; ++e) {
            uint64_t k = mst[e];
            uint64_t eidx = 0xFFFFFFFFull - (k & 0xFFFFFFFFull);
            float d = __uint_as_float((uint32_t)(k >> 32));
            int a = max_vertex(eidx, 2, n - 1), b = (int)(eidx - binom((uint64_t)a, 2));
            int u = a, v = b;
            while (par[u] != u) { par[u] = par[par[u]]; u = par[u]; }
            while (par[v] != v) { par[v] = par[par[v]]; v = par[v]; }
            int young = u < v ? u : v, old = u < v ? v : u;
            par[young] = old;
            cs += pair_hash((uint64_t)young, eidx);
            if (d > 0.0f) {
                if ((uint64_t)cnt < pcap0) P[cnt] = Pair{0.0f, d, (int64_t)young, (int64_t)eidx};
                ++cnt;
            }
        }
        red[38] = (uint64_t)cnt;
        red[39] = cs;
    }
    __syncthreads();
    // one [0, inf) bar per component in vertex order: the roots (a component's root is its
    // largest vertex: the younger root always hooks under the older), block prefix per chunk
    {
        Pair* P = pairs0 + (size_t)l * pcap0;
        uint64_t base = red[38];
        for (int v0 = 0; v0 < n; v0 += T) {
            const int v = v0 + t;
            const bool root = v < n && par[v] == v;
            const uint64_t m = __ballot(root);
            if (ln == 0) red[w] = (uint64_t)__popcll(m);
            __syncthreads();
            uint64_t before = 0, tot = 0;
            for (int q = 0; q < nw; ++q) {
                before += q < w ? red[q] : 0;
                tot += red[q];
            }
            const uint64_t pos = base + before + lanes_below(m);
            if (root && pos < pcap0) P[pos] = Pair{0.0f, INFINITY, (int64_t)v, -1};
            base += tot;
            __syncthreads();
        }
        if (t == 0) red[38] = base;
    }
    __syncthreads();
    if (t == 0) {
        uint64_t cnt = red[38];
        const uint64_t cs = red[39];
        if ((uint64_t)cnt > pcap0) {
            st->err |= ERR_PAIR_CAP;
            cnt = (int64_t)pcap0;
        }
        st->count[0] = cnt;
        st->checksum[0] = cs;
        st->all_pairs[0] = nmst;
        st->n_columns[0] = n;
    }
    H0M(4)
#undef H0M
}

// Small-N H0 (N <= 64): one wave per layer, distance matrix in LDS, lane v
// owns vertex v; Prim's frontier keys live in registers, the arg-min vertex is
// found by ballot (no index decode); the <= 63 forest edges are sorted with an
// in-register bitonic network.  Same results as k_h0.
// Body: D is the layer's matrix in LDS, thr the resolved threshold; forest
// edges go to mst_bits (LDS when MST_LDS, else HBM, per-layer pointer), H0
// pairs to P, the H0 stats to st.
template <bool MST_LDS>
__device__ __forceinline__ void h0_wave_body(const float* D, int n, float thr, LayerStats* st, uint32_t* mst_bits, Pair* P) {
    const int v = lane_id();
    const bool real = v < n;
#ifdef TDA_PROFILE
    const uint64_t tp0 = clock64();
#define TDA_H0_MARK(i) \
    if (v == 0) st->prof[3][i] = clock64() - tp0;
#else
#define TDA_H0_MARK(i)
#endif
    TDA_H0_MARK(0)
    // D is symmetric: lane v counts column v below the diagonal, 8 loads in flight
    uint64_t ne = 0;
    if (real)
        for (int j0 = v + 1; j0 < n; j0 += 8) {
            float x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = j0 + u < n ? D[(j0 + u) * n + v] : INFINITY;
#pragma unroll
            for (int u = 0; u < 8; ++u) ne += x[u] <= thr;
        }
    ne = wave_sum_u64(ne);
    TDA_H0_MARK(1)
    // Prim: lane v keeps its best tree edge as a filtration key (diam, then
    // index desc); the arg-min is a 32-bit min over the diameter bits, and a
    // second one over the index word only when diameters tie
    bool intree = v == 0;
    uint64_t best = kEmpty64;
    int cur = 0;
    uint64_t mykey = kEmpty64;  // forest edge discovered at step == lane
    int nmst = 0;
    for (int it = 1; it < n; ++it) {
        if (real && !intree) {
            const float d = D[cur * n + v];
            if (d <= thr) {
                const uint32_t a = (uint32_t)max(cur, v), bb = (uint32_t)min(cur, v);
                const uint64_t k = filt_key(d, (uint64_t)(a * (a - 1) / 2 + bb));
                best = k < best ? k : best;
            }
        }
        const bool live = real && !intree;
        const uint32_t hi = live ? (uint32_t)(best >> 32) : 0xFFFFFFFFu;
        const uint32_t mh = wave_min_u32(hi);
        int nv;
        if (mh == 0xFFFFFFFFu) {
            nv = __builtin_ctzll(__ballot(live));  // new component
        } else {
            uint64_t cm = __ballot(live && hi == mh);
            if (__popcll(cm) > 1) {  // equal diameters: smallest index word = largest edge index
                const uint32_t lo = (live && hi == mh) ? (uint32_t)best : 0xFFFFFFFFu;
                const uint32_t ml = wave_min_u32(lo);
                cm = __ballot(live && hi == mh && (uint32_t)best == ml);
            }
            nv = __builtin_ctzll(cm);
            const uint64_t m = ((uint64_t)mh << 32) | (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)best, nv);
            if (v == nmst) mykey = m;
            ++nmst;
        }
        if (v == nv) intree = true;
        cur = nv;
    }
    TDA_H0_MARK(2)
    // bitonic sort of the forest keys (one per lane, EMPTY padding)
    uint64_t k = mykey;
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            uint64_t o = shfl_xor_u64(k, stride);
            bool up = (v & size) == 0;
            bool lower = (v & stride) == 0;
            uint64_t lo = o < k ? o : k, hi = o < k ? k : o;
            k = (lower == up) ? lo : hi;
        }
    }
    TDA_H0_MARK(3)
    // lane e now holds the e-th forest edge in Kruskal order (diam asc, idx desc)
    const bool has = v < nmst;
    const uint64_t eidx = has ? 0xFFFFFFFFull - (k & 0xFFFFFFFFull) : 0;
    const float d = has ? __uint_as_float((uint32_t)(k >> 32)) : 0.0f;
    int ea = 0, eb = 0;
    if (has) {
        ea = max_vertex(eidx, 2, n - 1);
        eb = (int)(eidx - binom((uint64_t)ea, 2));
        matomic_or<MST_LDS>(&mst_bits[eidx >> 5], 1u << (eidx & 31));
    }
    // elder-rule union-find in registers: lane u holds the label (= max
    // vertex) of its component; each merge is two readlanes + a select.
    int label = v;
    int young_e = -1;
    for (int e = 0; e < nmst; ++e) {
        const int a = __builtin_amdgcn_readlane(ea, e), bb = __builtin_amdgcn_readlane(eb, e);
        const int ra = __builtin_amdgcn_readlane(label, a), rb = __builtin_amdgcn_readlane(label, bb);
        const int young = ra < rb ? ra : rb, old = ra < rb ? rb : ra;
        if (label == young) label = old;
        if (v == e) young_e = young;
    }
    TDA_H0_MARK(4)
    // emission: finite bars (d > 0) in Kruskal order, then [0, inf) per root
    const uint64_t posm = __ballot(has && d > 0.0f);
    const int nfin = __popcll(posm);
    if (has && d > 0.0f) P[lanes_below(posm)] = Pair{0.0f, d, (int64_t)young_e, (int64_t)eidx};
    const uint64_t rootm = __ballot(real && label == v);
    if (real && label == v) P[nfin + lanes_below(rootm)] = Pair{0.0f, INFINITY, (int64_t)v, -1};
    const uint64_t cs = wave_sum_u64(has ? pair_hash((uint64_t)young_e, eidx) : 0ull);
    if (v == 0) {
        st->thresh = thr;
        st->num_edges = (int64_t)ne;
        st->count[0] = nfin + __popcll(rootm);
        st->checksum[0] = cs;
        st->all_pairs[0] = nmst;
        st->n_columns[0] = n;
    }
    TDA_H0_MARK(5)
#undef TDA_H0_MARK
}

__global__ __launch_bounds__(64) void k_h0_wave(const float* __restrict__ dist, int n, const uint32_t* __restrict__ rowmax,
                                                float user_thresh, LayerStats* __restrict__ stats, uint32_t* __restrict__ mst_bits,
                                                uint64_t mst_words, Pair* __restrict__ pairs0, uint64_t pcap0) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.x, v = threadIdx.x;
    // enclosing radius = min over rows of the row maxima k_distance folded in
    const uint32_t rmv = v < n ? ld_glb(rowmax + (size_t)l * n, (size_t)v) : 0xFFFFFFFFu;
    float* D = (float*)smem;              // n*n
    const float* Dg = dist + (size_t)l * n * n;
    stage_to_lds(D, Dg, sizeof(float) * n * n, v, 64);
    __syncthreads();
    float thr = user_thresh;
    if (isinf(user_thresh) || user_thresh == 3.402823466e+38f) thr = n == 1 ? 0.0f : __uint_as_float(wave_min_u32(rmv));
    h0_wave_body<false>(D, n, thr, stats + l, mst_bits + (size_t)l * mst_words, pairs0 + (size_t)l * pcap0);
}

// ------------------------------------------------------------------ apparent
// Parallel part of compute_pairs [upstream]: every d-simplex s <= thresh that
// is not cleared (an H_{d-1} death) is a column.  Its coboundary pivot (the
// oldest cofacet: min diam, then max index) is found by scanning vertices in
// decreasing order with an early exit at diam == diam(s).  (s, t) is an
// apparent pair iff t is also the pivot-from-below, i.e. s is t's youngest
// facet (max diam, then min index); for VR this forces diam(t) == diam(s) and
// reduces to: every facet t\{u} with u > v has diam < diam(s).  Apparent
// pairs are persistence pairs (zero persistence: never emitted), columns with
// an empty coboundary are essential (emitted here), the rest go to k_reduce.
// (layer, block within the layer, blocks per layer) of an apparent-pass block.  A 2-D grid is
// (blocks per layer, L).  A 1-D grid of L x G blocks (L a multiple of 8, rips.hip) is XCD-aware:
// blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, for speed only), so block b
// takes layer (b mod 8) + 8 j and every XCD's L2 serves its own layers' distance matrices instead
// of a slice of all of them (torus1024x32: 11.4 GB of HBM reads per 32-layer launch, 356 MB per
// 4-MB matrix)
struct AppBlock {
    int l;
    uint32_t bx, nbx;
};
__device__ __forceinline__ AppBlock app_block(int xcd_layers) {
    if (xcd_layers <= 0) return {(int)blockIdx.y, blockIdx.x, gridDim.x};
    const uint32_t G = gridDim.x / (uint32_t)xcd_layers, b = blockIdx.x, r = b >> 3;
    return {(int)((b & 7u) + 8u * (r / G)), r % G, G};
}

// Classify simplex s (vertices vs descending, diameter sd <= r) from its oldest cofacet (vertex
// bv, diameter bcd; bv < 0: empty coboundary): 1 = apparent (pivot bit set, pair counted), 2 =
// residual (an empty coboundary too: essential unless cleared, decided by the reduction).
template <int DIM, typename Dat>
__device__ __forceinline__ int apparent_kind(uint64_t s, const int (&vs)[DIM + 1], float sd, int bv, float bcd, Dat dat, int n,
                                             uint32_t* piv, uint64_t& tixv, uint64_t& acc_cs, uint64_t& acc_app) {
    if (bv < 0 || bcd != sd) return 2;
    bool app = true;
#pragma unroll
    for (int u = 0; u <= DIM; ++u) {
        if (vs[u] < bv) continue;
        // diam of (s u {bv}) \ {vs[u]}
        float fd = 0.0f;
#pragma unroll
        for (int i = 0; i <= DIM; ++i) {
            if (i == u) continue;
            fd = fmaxf(fd, dat((size_t)bv * n + vs[i]));
#pragma unroll
            for (int j = i + 1; j <= DIM; ++j)
                if (j != u) fd = fmaxf(fd, dat((size_t)vs[i] * n + vs[j]));
        }
        app &= fd < sd;
    }
    if (!app) return 2;
    const uint64_t tix = cofacet_index<DIM>(vs, bv);
    matomic_or<false>(&piv[tix >> 5], 1u << (tix & 31));  // no return: fire and forget
    tixv = tix;
    acc_cs += pair_hash(s, tix);
    acc_app += 1;
    return 1;
}

// One simplex per lane (kind 0: none): the words of set H2 pivot bits (sparse-cleared bitmap) and
// the residual columns, each wave aggregated.
template <int DIM>
__device__ __forceinline__ void apparent_append(int kind, uint64_t s, float sd, uint64_t tixv, const DimBufs& b, LayerStats* st, int l,
                                                uint64_t* resid) {
    if (DIM == 2 && b.clr) {  // sparse-cleared bitmap: list the words set (wave aggregated)
        const uint64_t mc = __ballot(kind == 1);
        if (mc) {
            uint64_t cb = 0;
            if (lane_id() == __builtin_ctzll(mc)) cb = atomicAdd((unsigned long long*)&st->n_clr2, (unsigned long long)__popcll(mc));
            cb = shfl_u64(cb, __builtin_ctzll(mc)) + lanes_below(mc);
            if (kind == 1 && cb < b.clr_cap) st_glb(b.clr + (size_t)l * b.clr_cap, cb, tixv >> 5);
        }
    }
    // residual append (wave aggregated)
    const uint64_t m = __ballot(kind == 2);
    if (m) {
        uint64_t basepos = 0;
        if (lane_id() == __builtin_ctzll(m))
            basepos = atomicAdd((unsigned long long*)&st->n_residual[DIM], (unsigned long long)__popcll(m));
        basepos = shfl_u64(basepos, __builtin_ctzll(m));
        if (kind == 2) {
            uint64_t pos = basepos + lanes_below(m);
            if (pos < b.rcap)
                st_glb(resid, pos, col_key(sd, s));
            else
                atomicOr(&st->err, ERR_RESID_CAP);
        }
    }
}

__device__ __forceinline__ void apparent_stats(LayerStats* st, int dim, uint64_t acc_cs, uint64_t acc_app, uint64_t acc_cols) {
    acc_cs = wave_sum_u64(acc_cs);
    acc_app = wave_sum_u64(acc_app);
    acc_cols = wave_sum_u64(acc_cols);
    if (lane_id() == 0) {
        if (acc_app) {
            atomicAdd((unsigned long long*)&st->checksum[dim], (unsigned long long)acc_cs);
            atomicAdd((unsigned long long*)&st->all_pairs[dim], (unsigned long long)acc_app);
        }
        if (acc_cols) atomicAdd((unsigned long long*)&st->n_columns[dim], (unsigned long long)acc_cols);
    }
}

template <int DIM, bool DLDS>
__global__ __launch_bounds__(256) void k_apparent(const float* __restrict__ dist, int n, LayerStats* __restrict__ stats,
                                                  DimBufs b, const uint32_t* __restrict__ rowmax, float user_thresh,
                                                  int xcd_layers) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const AppBlock ab = app_block(xcd_layers);  // 0: 2-D grid (blocks per layer, L)
    const int l = ab.l;
    const float* Dg = dist + (size_t)l * n * n;
    const float r = block_thresh(rowmax + (size_t)l * n, n, user_thresh, (uint32_t*)smem);
    float* Dsh = (float*)(smem + 16);
    if (DLDS) {  // stage this layer's distance matrix in LDS (N <= 128: <= 64 KB)
        stage_to_lds(Dsh, Dg, sizeof(float) * n * n, threadIdx.x, blockDim.x);
        __syncthreads();
    }
    // typed distance reads (LDS or HBM, never FLAT)
    auto dat = [&](size_t i) -> float { return DLDS ? ld_lds(Dsh, i) : ld_glb(Dg, i); };
    LayerStats* st = stats + l;
    const uint32_t* cleared = b.cleared ? b.cleared + (size_t)l * b.cleared_words : nullptr;
    uint32_t* piv = b.pivbits + (size_t)l * b.piv_words;
    uint64_t* resid = b.resid + (size_t)l * b.rcap;
    const uint64_t stride = (uint64_t)ab.nbx * blockDim.x;
    uint64_t acc_cs = 0, acc_app = 0, acc_cols = 0;
    for (uint64_t base = (uint64_t)ab.bx * blockDim.x; base < b.ncand; base += stride) {
        const uint64_t s = base + threadIdx.x;
        int kind = 0;  // 0 skip, 1 apparent, 2 residual (incl. empty coboundary)
        uint64_t tixv = 0;
        int vs[DIM + 1];
        float sd = 0.0f;
        if (s < b.ncand && !(cleared && ((ld_glb(cleared, s >> 5) >> (s & 31)) & 1u))) {
            decode<DIM>(s, n, vs);
#pragma unroll
            for (int i = 0; i <= DIM; ++i)
#pragma unroll
                for (int j = i + 1; j <= DIM; ++j) sd = fmaxf(sd, dat((size_t)vs[i] * n + vs[j]));
            if (sd <= r) {
                // oldest cofacet, vertices descending
                float bcd = INFINITY;
                int bv = -1;
                for (int v = n - 1; v >= 0; --v) {
                    bool mem = false;
#pragma unroll
                    for (int i = 0; i <= DIM; ++i) mem |= (vs[i] == v);
                    if (mem) continue;
                    float cd = sd;
#pragma unroll
                    for (int i = 0; i <= DIM; ++i) cd = fmaxf(cd, dat((size_t)v * n + vs[i]));
                    if (cd <= r && cd < bcd) {
                        bcd = cd;
                        bv = v;
                        if (cd == sd) break;
                    }
                }
                kind = apparent_kind<DIM>(s, vs, sd, bv, bcd, dat, n, piv, tixv, acc_cs, acc_app);
            }
        }
        acc_cols += (kind != 0);
        apparent_append<DIM>(kind, s, sd, tixv, b, st, l, resid);
    }
    apparent_stats(st, DIM, acc_cs, acc_app, acc_cols);
}

// H1 apparent pass at large N (r06): the edge columns in 16 x 16 tiles (a in one block of 16
// vertices, b in another, a > b), the oldest-cofacet scan over v-tiles of kAppTV rows whose
// columns a and b are staged in LDS -- 2 x 64 B of every row per tile of 256 edges, where the
// one-edge-per-thread pass read a 1-KB row segment per 256 edges of one a and every tile's rows
// from L2 again (torus1024x32: 3.2 GB of fabric reads per 32-layer launch for 128 MB of
// matrices).  The next v-tile's loads are in flight while the current one is scanned.  Each edge's
// scan, early exit, apparent test and outputs are k_apparent<1, false>'s.
constexpr int kAppTS = 16;   // tile side (vertices)
constexpr int kAppTV = 64;   // rows per v-tile
__global__ __launch_bounds__(256) void k_apparent_tile(const float* __restrict__ dist, int n, LayerStats* __restrict__ stats,
                                                       DimBufs b, const uint32_t* __restrict__ rowmax, float user_thresh,
                                                       int xcd_layers) {
    __shared__ float Ta[2][kAppTV][kAppTS + 1], Tb[2][kAppTV][kAppTS + 1];
    __shared__ uint32_t s_min;
    __shared__ int s_any[3];  // "a lane is still scanning", one cell per v-tile mod 3 (a slow reader of cell j
                              // is past barrier j + 1 before anyone clears it again)
    const AppBlock ab = app_block(xcd_layers);
    const int l = ab.l;
    const float* Dg = dist + (size_t)l * n * n;
    const float r = block_thresh(rowmax + (size_t)l * n, n, user_thresh, &s_min);
    auto dat = [&](size_t i) -> float { return ld_glb(Dg, i); };
    LayerStats* st = stats + l;
    const uint32_t* cleared = b.cleared ? b.cleared + (size_t)l * b.cleared_words : nullptr;
    uint32_t* piv = b.pivbits + (size_t)l * b.piv_words;
    uint64_t* resid = b.resid + (size_t)l * b.rcap;
    const int nt = (n + kAppTS - 1) / kAppTS;
    uint64_t acc_cs = 0, acc_app = 0, acc_cols = 0;
    const int t = threadIdx.x, ti = t / kAppTS, tj = t % kAppTS;
    // staging: thread t loads rows (t / 16) + 16 q, q < 4, column t % 16, of both column blocks
    const int sr = t / kAppTS, sc = t % kAppTS;
    for (uint32_t tile = ab.bx; tile < (uint32_t)(nt * (nt + 1) / 2); tile += ab.nbx) {
        // tile -> (ta >= tb): row ta holds tiles ta (ta + 1) / 2 .. + ta
        int ta = (int)((sqrtf(8.0f * (float)tile + 1.0f) - 1.0f) * 0.5f);
        while ((ta + 1) * (ta + 2) / 2 <= (int)tile) ++ta;
        while (ta * (ta + 1) / 2 > (int)tile) --ta;
        const int tb = (int)tile - ta * (ta + 1) / 2;
        const int a = ta * kAppTS + ti, bb = tb * kAppTS + tj;
        const int A0 = ta * kAppTS, B0 = tb * kAppTS;
        int kind = 0;
        uint64_t tixv = 0;
        int vs[2] = {a, bb};
        float sd = 0.0f;
        uint64_t s = 0;
        bool live = false;  // still scanning
        if (a < n && bb < a) {
            s = (uint64_t)a * (a - 1) / 2 + (uint64_t)bb;
            if (!(cleared && ((ld_glb(cleared, s >> 5) >> (s & 31)) & 1u))) {
                sd = dat((size_t)a * n + bb);
                live = sd <= r;
                kind = live ? 2 : 0;  // decided below
            }
        }
        float bcd = INFINITY;
        int bv = -1;
        // v-tiles from the top (vertices descending)
        const int nv = (n + kAppTV - 1) / kAppTV;
        float ra[kAppTV / 16], rb[kAppTV / 16];
        auto load = [&](int vt) {
#pragma unroll
            for (int q = 0; q < kAppTV / 16; ++q) {
                const int v = vt * kAppTV + sr + 16 * q;
                const bool ok = v < n;
                ra[q] = ok && A0 + sc < n ? ld_glb(Dg, (size_t)v * n + A0 + sc) : 0.0f;
                rb[q] = ok && B0 + sc < n ? ld_glb(Dg, (size_t)v * n + B0 + sc) : 0.0f;
            }
        };
        auto store = [&](int buf) {
#pragma unroll
            for (int q = 0; q < kAppTV / 16; ++q) {
                Ta[buf][sr + 16 * q][sc] = ra[q];
                Tb[buf][sr + 16 * q][sc] = rb[q];
            }
        };
        int buf = 0, cell = 0;
        load(nv - 1);
        store(0);
        if (t == 0) s_any[0] = 0;
        __syncthreads();
        for (int vt = nv - 1; vt >= 0; --vt) {
            if (vt > 0) load(vt - 1);  // in flight during the scan below
            if (live) {
                for (int k = kAppTV - 1; k >= 0; --k) {
                    const int v = vt * kAppTV + k;
                    if (v >= n || v == a || v == bb) continue;
                    const float cd = fmaxf(sd, fmaxf(Ta[buf][k][ti], Tb[buf][k][tj]));
                    if (cd <= r && cd < bcd) {
                        bcd = cd;
                        bv = v;
                        if (cd == sd) {
                            live = false;
                            break;
                        }
                    }
                }
            }
            const int next = cell == 2 ? 0 : cell + 1;
            if (live) s_any[cell] = 1;  // every writer writes 1
            if (vt > 0) store(buf ^ 1);
            if (t == 0) s_any[next] = 0;
            __syncthreads();
            const bool more = s_any[cell] != 0;
            buf ^= 1;
            cell = next;
            if (!more) break;
        }
        if (kind == 2) kind = apparent_kind<1>(s, vs, sd, bv, bcd, dat, n, piv, tixv, acc_cs, acc_app);
        acc_cols += (kind != 0);
        apparent_append<1>(kind, s, sd, tixv, b, st, l, resid);
        __syncthreads();  // the staging buffers are rewritten by the next tile
    }
    apparent_stats(st, 1, acc_cs, acc_app, acc_cols);
}

// Small-N apparent pass (N <= 64, the reference's clouds): same columns,
// pairs and residual lists as k_apparent<DIM, true>, with the per-simplex
// instruction count cut ~3x (PMC r04: k_apparent<2> issued 2.1 K VALU per wave
// and was VALU-bound): 32-bit index decode (every binomial < 2^18), the
// matrix staged with rows padded to a multiple of 4 (+inf pads), and the
// oldest-cofacet scan reading four vertices per ds_read_b128 from the rows of
// the simplex's own vertices (D symmetric), branch-free inside a group.  Scan
// order and tie rule are k_apparent's: vertices descending, a strictly smaller
// diameter wins (so the largest vertex among equal minima), stop at
// diam == diam(s) -- no later vertex can beat it, as every cofacet diameter is
// >= diam(s).  With pl_words > 0 the apparent pivots collect in an LDS copy of
// the layer's pivot bitmap, OR-ed into HBM once per non-zero word at the end
// (r06: one scattered HBM atomic per pair was a quarter of the pass).
template <int DIM>
__device__ __forceinline__ void decode_small(uint32_t s, int n, int (&vs)[DIM + 1]) {
    uint32_t rem = s;
    int top = n - 1;
    if (DIM == 2) {  // largest a <= n - 1 with C(a, 3) <= s
        const float x = 6.0f * (float)rem;
        int a = (x > 0.0f ? (int)__builtin_amdgcn_exp2f(__builtin_amdgcn_logf(x) * (1.0f / 3.0f)) : 0) + 1;
        a = min(max(a, 2), top);
        while (a > 2 && c3u((uint32_t)a) > rem) --a;
        while (a < top && c3u((uint32_t)a + 1u) <= rem) ++a;
        vs[0] = a;
        rem -= c3u((uint32_t)a);
        top = a - 1;
    }
    {  // largest b <= top with C(b, 2) <= rem
        int b = (int)(0.5f * (1.0f + __fsqrt_rn(1.0f + 8.0f * (float)rem)));
        b = min(max(b, 1), top);
        while (b > 1 && c2u((uint32_t)b) > rem) --b;
        while (b < top && c2u((uint32_t)b + 1u) <= rem) ++b;
        vs[DIM - 1] = b;
        rem -= c2u((uint32_t)b);
        vs[DIM] = (int)min(rem, (uint32_t)(b - 1));
    }
}

// LDS of k_apparent_small: 16 | the matrix, rows padded to 4 | the pivot bitmap copy (pl_words)
__host__ __device__ constexpr size_t small_piv_offset(int n) { return (size_t)n * ((n + 3) & ~3) * 4; }
constexpr uint32_t kSmallPivLdsMax = 32 * 1024;  // largest LDS bitmap copy (bytes): C(48, 4) bits take 24 KB

template <int DIM>
__global__ __launch_bounds__(256) void k_apparent_small(const float* __restrict__ dist, int n, LayerStats* __restrict__ stats,
                                                        DimBufs b, const uint32_t* __restrict__ rowmax, float user_thresh,
                                                        uint32_t pl_words) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.y;
    const float* Dg = dist + (size_t)l * n * n;
    const float r = block_thresh(rowmax + (size_t)l * n, n, user_thresh, (uint32_t*)smem);
    const int ns = (n + 3) & ~3;  // padded row stride (16-B rows)
    TDA_LDS float* Dsh = (TDA_LDS float*)(smem + 16);
    if (ns == n) {
        stage_to_lds((float*)Dsh, Dg, sizeof(float) * n * n, threadIdx.x, blockDim.x);
    } else {  // padded rows: (i, j) advanced incrementally (no division per element)
        const int T = blockDim.x, di = T / ns, dj = T - di * ns;
        int i = threadIdx.x / ns, j = threadIdx.x - i * ns;
        for (int e = threadIdx.x; e < n * ns; e += T) {
            Dsh[e] = j < n ? ld_glb(Dg, (size_t)i * n + j) : INFINITY;
            i += di;
            j += dj;
            if (j >= ns) j -= ns, ++i;
        }
    }
    // the block's apparent pivots collect in an LDS copy of the pivot bitmap when it fits
    // (pl_words > 0: the launch sized the LDS for it) and reach HBM as one OR per non-zero word
    // at the end, instead of one scattered HBM atomic per pair
    TDA_LDS uint32_t* pl = (TDA_LDS uint32_t*)(smem + 16 + small_piv_offset(n));
    if (pl_words)
        for (uint32_t w = threadIdx.x; w < pl_words; w += blockDim.x) pl[w] = 0u;
    __syncthreads();
    LayerStats* st = stats + l;
    const uint32_t* cleared = b.cleared ? b.cleared + (size_t)l * b.cleared_words : nullptr;
    uint32_t* piv = b.pivbits + (size_t)l * b.piv_words;
    uint64_t* resid = b.resid + (size_t)l * b.rcap;
    const uint32_t stride = gridDim.x * blockDim.x;
    const uint32_t ncand = (uint32_t)b.ncand;
    uint64_t acc_cs = 0, acc_app = 0, acc_cols = 0;
    for (uint32_t base = blockIdx.x * blockDim.x; base < ncand; base += stride) {
        const uint32_t s = base + threadIdx.x;
        int kind = 0;  // 0 skip, 1 apparent, 2 residual (incl. empty coboundary)
        int vs[DIM + 1];
        float sd = 0.0f;
        if (s < ncand && !(cleared && ((ld_glb(cleared, (size_t)(s >> 5)) >> (s & 31)) & 1u))) {
            decode_small<DIM>(s, n, vs);
            float pd[DIM + 1][DIM + 1];  // the simplex's edge lengths (registers after unrolling)
#pragma unroll
            for (int i = 0; i <= DIM; ++i)
#pragma unroll
                for (int j = i + 1; j <= DIM; ++j) {
                    pd[i][j] = pd[j][i] = Dsh[vs[i] * ns + vs[j]];
                    sd = fmaxf(sd, pd[i][j]);
                }
            if (sd <= r) {
                uint64_t mm = 0;
#pragma unroll
                for (int i = 0; i <= DIM; ++i) mm |= 1ull << vs[i];
                float bcd = INFINITY;
                int bv = -1;
                // eight vertices per iteration: both groups' reads are in flight together
                for (int g = ns - 4; g >= 0; g -= 8) {
                    const int g2 = max(g - 4, 0);
                    v4f x[2][DIM + 1];
#pragma unroll
                    for (int i = 0; i <= DIM; ++i) {
                        x[0][i] = *(const TDA_LDS v4f*)(Dsh + vs[i] * ns + g);
                        x[1][i] = *(const TDA_LDS v4f*)(Dsh + vs[i] * ns + g2);
                    }
                    // the second group is void past vertex 0 (all four marked as members)
                    const uint32_t mb = ((uint32_t)(mm >> g) & 0xFu) | (((g >= 4 ? (uint32_t)(mm >> g2) : 0xFu) & 0xFu) << 4);
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int q = 3; q >= 0; --q) {
                            float cd = sd;
#pragma unroll
                            for (int i = 0; i <= DIM; ++i) cd = fmaxf(cd, x[h][i][q]);
                            const bool ok = !((mb >> (4 * h + q)) & 1u) && cd <= r && cd < bcd;
                            bcd = ok ? cd : bcd;
                            bv = ok ? (h ? g2 : g) + q : bv;
                        }
                    if (bcd == sd) break;
                }
                kind = 2;  // residual unless apparent (an empty coboundary is decided by the reduction)
                if (bv >= 0 && bcd == sd) {
                    float dv[DIM + 1];
#pragma unroll
                    for (int i = 0; i <= DIM; ++i) dv[i] = Dsh[bv * ns + vs[i]];
                    bool app = true;
#pragma unroll
                    for (int u = 0; u <= DIM; ++u) {
                        if (vs[u] < bv) continue;
                        // diam of (s u {bv}) \ {vs[u]}
                        float fd = 0.0f;
#pragma unroll
                        for (int i = 0; i <= DIM; ++i) {
                            if (i == u) continue;
                            fd = fmaxf(fd, dv[i]);
#pragma unroll
                            for (int j = i + 1; j <= DIM; ++j)
                                if (j != u) fd = fmaxf(fd, pd[i][j]);
                        }
                        app &= fd < sd;
                    }
                    if (app) {
                        kind = 1;
                        const uint64_t tix = cofacet_index<DIM>(vs, bv);
                        if (pl_words)
                            __hip_atomic_fetch_or(pl + (tix >> 5), 1u << (tix & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        else
                            matomic_or<false>(&piv[tix >> 5], 1u << (tix & 31));  // no return: fire and forget
                        acc_cs += pair_hash(s, tix);
                        acc_app += 1;
                    }
                }
            }
        }
        acc_cols += (kind != 0);
        // residual append (wave aggregated)
        const uint64_t m = __ballot(kind == 2);
        if (m) {
            uint64_t basepos = 0;
            if (lane_id() == __builtin_ctzll(m))
                basepos = atomicAdd((unsigned long long*)&st->n_residual[DIM], (unsigned long long)__popcll(m));
            basepos = shfl_u64(basepos, __builtin_ctzll(m));
            if (kind == 2) {
                const uint64_t pos = basepos + lanes_below(m);
                if (pos < b.rcap)
                    st_glb(resid, pos, col_key(sd, s));
                else
                    atomicOr(&st->err, ERR_RESID_CAP);
            }
        }
    }
    if (pl_words) {
        __syncthreads();
        for (uint32_t w = threadIdx.x; w < pl_words; w += blockDim.x) {
            const uint32_t v = pl[w];
            if (v) matomic_or<false>(&piv[w], v);
        }
    }
    acc_cs = wave_sum_u64(acc_cs);
    acc_app = wave_sum_u64(acc_app);
    acc_cols = wave_sum_u64(acc_cols);
    if (lane_id() == 0) {
        if (acc_app) {
            atomicAdd((unsigned long long*)&st->checksum[DIM], (unsigned long long)acc_cs);
            atomicAdd((unsigned long long*)&st->all_pairs[DIM], (unsigned long long)acc_app);
        }
        if (acc_cols) atomicAdd((unsigned long long*)&st->n_columns[DIM], (unsigned long long)acc_cols);
    }
}

// ------------------------------------------------------------------ input parts
// ABI 6 x_parts: the parts of a dynamically batched call, gathered into the
// workspace's input buffer (part k -> words [k * part_words, (k + 1) * part_words))
struct PartList {
    const void* p[TDA_MAX_PARTS];
};
// one wave that returns after `us` microseconds (s_memrealtime: 100 MHz), sleeping between
// reads: orders a side stream's next launch after work the main stream dispatches meanwhile
__global__ __launch_bounds__(64) void k_delay(uint32_t us) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime(), ticks = (uint64_t)us * 100;
    for (uint32_t i = 0; i < (1u << 20) && __builtin_amdgcn_s_memrealtime() - t0 < ticks; ++i) __builtin_amdgcn_s_sleep(8);  // capped
}

// end of a call with a sparse-cleared H2 pivot bitmap: zero the words k_apparent<2> listed
// (a layer whose list overflowed leaves the bitmap dirty: the host memsets it before the next call)
__global__ __launch_bounds__(256) void k_clear_words(const LayerStats* __restrict__ stats, const uint64_t* __restrict__ clr, uint64_t cap,
                                                     uint32_t* __restrict__ pivbits, uint64_t piv_words) {
    const int l = blockIdx.y;
    const uint64_t cnt = min((uint64_t)stats[l].n_clr2, cap);
    const uint64_t* c = clr + (size_t)l * cap;
    uint32_t* pv = pivbits + (size_t)l * piv_words;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (uint64_t)gridDim.x * blockDim.x) st_glb(pv, ld_glb(c, i), 0u);
}

__global__ __launch_bounds__(256) void k_gather_parts(PartList pl, uint64_t part_words, uint32_t* __restrict__ dst) {
    const int k = blockIdx.y;
    const uint32_t* src = (const uint32_t*)pl.p[k];
    uint32_t* d = dst + (size_t)k * part_words;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < part_words; i += (uint64_t)gridDim.x * blockDim.x)
        st_glb(d, i, ld_glb(src, i));
}

// ------------------------------------------------------------------ sort residual
struct SortArgs {
    uint64_t* resid[3];
    uint64_t rcap[3];
};
__global__ __launch_bounds__(1024) void k_sort_resid(LayerStats* __restrict__ stats, SortArgs sa, uint64_t* __restrict__ tmp,
                                                     uint64_t tmp_stride, uint64_t* __restrict__ rmap_keys, uint64_t rmap_stride,
                                                     int sort_log2, int dim0) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.x, dim = blockIdx.y + dim0;
    uint64_t* resid = sa.resid[dim];
    const uint64_t rcap = sa.rcap[dim];
    uint64_t cnt = (uint64_t)stats[l].n_residual[dim];
    if (cnt > rcap) cnt = rcap;
    block_sort<false>(resid + (size_t)l * rcap, nullptr, cnt, tmp + ((size_t)l * 2 + dim - 1) * tmp_stride, nullptr, (uint64_t*)smem,
                      nullptr, sort_log2);
    // clear the residual pivot map region this layer will use
    uint64_t cap = 16;
    while (cap < 2 * cnt + 16) cap <<= 1;
    if (cap > rmap_stride) cap = rmap_stride;
    uint64_t* rk = rmap_keys + ((size_t)l * 2 + dim - 1) * rmap_stride;
    for (uint64_t e = threadIdx.x; e < cap; e += blockDim.x) rk[e] = kEmpty64;
}

// per-dim pair buffers, passed by value (no host-side pointer tables)
struct PairSet {
    Pair* p[4];
    uint64_t cap[4];
};

// ------------------------------------------------------------------ output
struct OutPair {
    float birth, death;
    int64_t birth_idx, death_idx;
};

// ------------------------------------------------------------------ emit
// Emission order of dims >= 1 (reference: births_and_deaths_by_dim filled in
// column order, i.e. birth desc / column index asc; pinned 32/32 by
// summary_stats.json all_h1_persistence_values).  Block l sorts its layer's
// dims >= 1 into emission order and writes every segment straight into the host-mapped
// output at its global offset (a prefix over the stats' counts, recomputed
// per block), then its LayerStats.  LDS: the sort chunk (8 KiB keys * 12 B)
// and 16 x 2 words of reduction scratch behind it.
constexpr int kEmitSortLog2 = 13;
constexpr size_t kEmitLds = (size_t(12) << kEmitSortLog2) + 16 * 2 * 8;
__global__ __launch_bounds__(1024) void k_emit(LayerStats* __restrict__ stats, int L, int maxdim, PairSet ps, uint64_t* __restrict__ skeys,
                                               uint32_t* __restrict__ svals, uint64_t sstride, int64_t* __restrict__ out_off,
                                               OutPair* __restrict__ out, uint64_t out_cap, LayerStats* __restrict__ stats_host) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.x, t = threadIdx.x, nd = maxdim + 1;
    constexpr uint64_t CH = 1ull << kEmitSortLog2;
    uint64_t* sk = (uint64_t*)smem;
    uint32_t* sv = (uint32_t*)(sk + CH);
    uint64_t* red = (uint64_t*)(smem + CH * 12);  // [16][2]
    auto cnt_of = [&](int ll, int d) -> uint64_t {
        const uint64_t c = (uint64_t)stats[ll].count[d];
        return c > ps.cap[d] ? ps.cap[d] : c;
    };
    uint64_t before = 0, total = 0;
    for (int i = t; i < L * nd; i += blockDim.x) {
        const uint64_t c = cnt_of(i / nd, i % nd);
        total += c;
        before += i < l * nd ? c : 0;
    }
    before = wave_sum_u64(before);
    total = wave_sum_u64(total);
    if ((t & 63) == 0) {
        red[(t >> 6) * 2] = before;
        red[(t >> 6) * 2 + 1] = total;
    }
    __syncthreads();
    before = 0;
    total = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        before += red[w * 2];
        total += red[w * 2 + 1];
    }
    const bool over = total > out_cap;
    uint64_t o = before;
    for (int d = 0; d < nd; ++d) {
        const uint64_t cnt = cnt_of(l, d);
        if (t == 0) out_off[l * nd + d] = (int64_t)o;
        if (!over) {
            const Pair* P = ps.p[d] + (size_t)l * ps.cap[d];
            OutPair* dst = out + o;
            if (d == 0 || cnt < 2) {
                for (uint64_t e = t; e < cnt; e += blockDim.x) dst[e] = OutPair{P[e].birth, P[e].death, P[e].birth_idx, P[e].death_idx};
            } else {
                uint64_t* k = skeys + (size_t)l * sstride * 2;
                uint32_t* v = svals + (size_t)l * sstride * 2;
                for (uint64_t e = t; e < cnt; e += blockDim.x) {
                    k[e] = col_key(P[e].birth, (uint64_t)P[e].birth_idx);
                    v[e] = (uint32_t)e;
                }
                __syncthreads();
                block_sort<true>(k, v, cnt, k + sstride, v + sstride, sk, sv, kEmitSortLog2);
                for (uint64_t e = t; e < cnt; e += blockDim.x) {
                    const Pair q = P[v[e]];
                    dst[e] = OutPair{q.birth, q.death, q.birth_idx, q.death_idx};
                }
                __syncthreads();  // k / v are reused by the next dim
            }
        }
        o += cnt;
    }
    if (over && t == 0) stats[l].err |= ERR_OUT_CAP;
    __syncthreads();
    static_assert(sizeof(LayerStats) % 8 == 0, "LayerStats copies as u64 words");
    const uint64_t* src = (const uint64_t*)(stats + l);
    uint64_t* dstS = (uint64_t*)(stats_host + l);
    for (int i = t; i < (int)(sizeof(LayerStats) / 8); i += blockDim.x) dstS[i] = src[i];
}

// ---------------------------------------------------------------- silhouette
// Silhouette coefficient of each label set on the layer's f32 distance matrix:
// sklearn.metrics.silhouette_score(X, labels) (metric='euclidean'), which the
// reference calls next to ripser on the same cloud (debug_tda_pipeline.py:117-118,
// analyze_adversarial_tda.py:108-111).  Follows sklearn's _silhouette_reduce /
// silhouette_samples arithmetic: per-(point, cluster) distance sums in f64
// rounded to f32, intra / (|C|-1) and inter = min_k sum_k / |C_k| computed in
// f64 and rounded to f32, s = (b - a) / max(a, b) in f32, NaN (singleton
// cluster) -> 0; the mean is accumulated in f64.
// One block per (layer, label set); thread per point i, j-major loop over
// column i of the symmetric matrix (D[j][i]), so a wave's loads are coalesced.
// labels: [S][N] codes 0..K-1, every code present (checked on the host).
constexpr int kSilT = 256;
constexpr int kSilMaxK = 32;
__global__ __launch_bounds__(kSilT) void k_silhouette(const float* __restrict__ dist, int n, const int32_t* __restrict__ labels,
                                                      int K, double* __restrict__ out) {
    extern __shared__ __align__(16) unsigned char sil_lds[];
    const int l = blockIdx.x, s = blockIdx.y, S = gridDim.y, t = threadIdx.x;
    double* acc = (double*)sil_lds;                        // [K][kSilT]
    int32_t* lab = (int32_t*)(acc + (size_t)K * kSilT);    // [n]
    __shared__ int32_t freq[kSilMaxK];
    __shared__ double part[kSilT / 64];
    const float* D = dist + (size_t)l * n * n;
    if (t < kSilMaxK) freq[t] = 0;
    __syncthreads();
    for (int j = t; j < n; j += kSilT) {
        const int32_t c = labels[(size_t)s * n + j];
        lab[j] = c;
        atomicAdd(&freq[c], 1);
    }
    __syncthreads();
    double tot = 0.0;
    for (int i0 = 0; i0 < n; i0 += kSilT) {
        const int i = i0 + t;
        const bool on = i < n;
        for (int k = 0; k < K; ++k) acc[k * kSilT + t] = 0.0;
        if (on)
            for (int j = 0; j < n; ++j) acc[lab[j] * kSilT + t] += (double)D[(size_t)j * n + i];
        if (on) {
            const int li = lab[i];
            float inter = INFINITY;
            for (int k = 0; k < K; ++k) {
                if (k == li) continue;
                const float c = (float)((double)(float)acc[k * kSilT + t] / (double)freq[k]);
                inter = c < inter ? c : inter;
            }
            const int den = freq[li] - 1;
            float sv = 0.0f;
            if (den > 0) {
                const float a = (float)((double)(float)acc[li * kSilT + t] / (double)den);
                const float m = fmaxf(a, inter);
                sv = m > 0.0f ? (inter - a) / m : 0.0f;  // 0/0 -> NaN -> 0 (nan_to_num)
            }
            tot += (double)sv;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
    if ((t & 63) == 0) part[t >> 6] = tot;
    __syncthreads();
    if (t == 0) {
        double m = 0.0;
        for (int w = 0; w < kSilT / 64; ++w) m += part[w];
        out[(size_t)l * S + s] = m / (double)n;
    }
}

// ---------------------------------------------------------------- TwoNN
// Intrinsic dimension of each layer's cloud on its distance matrix: the
// reference's compute_intrinsic_dimensionality (metrics.py:113-208), which
// runs torch.cdist (:143), diagonal -> inf (:146), topk(2, smallest) (:149),
// mu = r2 / r1 where both exceed eps (:154-155), keeps the finite mu (:163),
// sorts them and drops the largest discard fraction (:169-172,
// n_keep = max(int(len * (1 - discard)), 5)), F_emp = i / n_samples over ALL
// samples (:180-181), x = log(mu + eps), y = -log(1 - F + eps) (:184-187),
// rejects var(x) or var(y) < eps (:190), slope = sum(xy) / sum(xx) (:195-201)
// and returns it iff finite and in (0, 1000) (:204), else NaN.
// Elementwise steps are f32 as in the reference; the sums and variances
// accumulate in f64 and round to f32 (the reference's f32 reductions have
// their own order), which is where the test tolerance comes from.
// One 1024-thread block per layer: a wave per row finds the two smallest
// off-diagonal distances (lane-strided, coalesced, DPP top-2 merge), the
// finite ratios go to LDS, a bitonic sort orders them, block reductions do
// the regression.  LDS: next_pow2(n) floats (n <= 8192).
constexpr int kTnT = 1024;
__device__ __forceinline__ void top2_insert(float v, float& a, float& b) {
    if (v < a) {
        b = a;
        a = v;
    } else if (v < b) {
        b = v;
    }
}
__device__ __forceinline__ double block_sum_f64(double v, double* part) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += part[w];
    return s;
}
__global__ __launch_bounds__(kTnT) void k_twonn(const float* __restrict__ dist, int n, double discard, float eps, int pw2,
                                                float* __restrict__ out) {
    extern __shared__ __align__(16) unsigned char tn_lds[];
    float* mu = (float*)tn_lds;  // [pw2]
    __shared__ int cnt;
    __shared__ double part[kTnT / 64];
    const int l = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const float* D = dist + (size_t)l * n * n;
    if (n <= 5) {  // metrics.py:136-137
        if (t == 0) out[l] = __int_as_float(0x7fc00000);
        return;
    }
    if (t == 0) cnt = 0;
    __syncthreads();
    for (int i = wv; i < n; i += kTnT / 64) {
        float a = INFINITY, b = INFINITY;
        const float* row = D + (size_t)i * n;
        for (int j = lane; j < n; j += 64)
            if (j != i) top2_insert(row[j], a, b);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float oa = __shfl_xor(a, o, 64), ob = __shfl_xor(b, o, 64);
            top2_insert(oa, a, b);
            top2_insert(ob, a, b);
        }
        if (lane == 0) {
            const float m = (a > eps && b > eps) ? b / a : INFINITY;
            if (isfinite(m)) mu[atomicAdd(&cnt, 1)] = m;
        }
    }
    __syncthreads();
    const int v = cnt;
    if (v < 5) {  // :165-166
        if (t == 0) out[l] = __int_as_float(0x7fc00000);
        return;
    }
    for (int i = v + t; i < pw2; i += kTnT) mu[i] = INFINITY;
    __syncthreads();
    // bitonic sort, ascending
    for (int k = 2; k <= pw2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = t; i < pw2; i += kTnT) {
                const int p = i ^ j;
                if (p > i) {
                    const float x = mu[i], y = mu[p];
                    if (((i & k) == 0) == (x > y)) {
                        mu[i] = y;
                        mu[p] = x;
                    }
                }
            }
            __syncthreads();
        }
    int keep = (int)((double)v * (1.0 - discard));  // Python float arithmetic (:170)
    keep = keep < 5 ? 5 : (keep > v ? v : keep);
    const float fn = (float)n;
    double sx = 0.0, sy = 0.0;
    for (int i = t; i < keep; i += kTnT) {
        const float x = logf(mu[i] + eps);
        const float f = (float)(i + 1) / fn;
        const float y = -logf((1.0f - f) + eps);
        sx += (double)x;
        sy += (double)y;
    }
    const double mx = block_sum_f64(sx, part) / keep, my = block_sum_f64(sy, part) / keep;
    double vx = 0.0, vy = 0.0, sxy = 0.0, sxx = 0.0;
    for (int i = t; i < keep; i += kTnT) {
        const float x = logf(mu[i] + eps);
        const float f = (float)(i + 1) / fn;
        const float y = -logf((1.0f - f) + eps);
        vx += ((double)x - mx) * ((double)x - mx);
        vy += ((double)y - my) * ((double)y - my);
        sxy += (double)(x * y);
        sxx += (double)(x * x);
    }
    const float varx = (float)(block_sum_f64(vx, part) / (keep - 1));
    const float vary = (float)(block_sum_f64(vy, part) / (keep - 1));
    const float num = (float)block_sum_f64(sxy, part);
    const float den = (float)block_sum_f64(sxx, part);
    if (t == 0) {
        float r = __int_as_float(0x7fc00000);
        if (!(varx < eps || vary < eps) && !(fabsf(den) < eps)) {
            const float slope = num / den;
            if (isfinite(slope) && slope > 0.0f && slope < 1000.0f) r = slope;
        }
        out[l] = r;
    }
}

}  // namespace tda
