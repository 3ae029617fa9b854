// rips_kernels.h -- gfx950 kernels of the batched Vietoris-Rips pipeline.
//
// One launch of each kernel covers every layer of a batch (blockIdx.y or
// blockIdx.x = layer), so the reference's per-layer Python loop
// (debug_tda_pipeline.py:92-150) becomes a handful of launches per sweep.
//
//   k_distance      pairwise L2 in FP64, sklearn-f32 rounding   
//   k_square_dist   condensed/square distance input             (a2' / is_dist)
//   k_h0            enclosing radius, num_edges, spanning forest, H0 pairs (a3, a4)
//   k_apparent<d>   column enumeration + apparent-pair test     (a5, parallel part)
//   k_sort_resid    per-layer sort of the residual columns
//   k_reduce<d>     Z/2 cohomology reduction of residual columns (a5, serial part)
//   k_finalize      per-layer emission order of the pairs        (a6)
//   k_compact       pack all layers' pairs into the host-mapped result
#pragma once
#include "rips_device.h"

namespace tda {

// ------------------------------------------------------------------ layout
struct Pair {
    float birth, death;
    int64_t birth_idx, death_idx;
};

struct LayerStats {  // zeroed every call; copied to the host result
    float thresh;
    int32_t err;  // bit flags, see ERR_*
    int64_t num_edges;
    int64_t count[4];      // emitted pairs per dim
    uint64_t checksum[4];  // sum of pair_hash over all pairs
    int64_t all_pairs[4];
    int64_t n_columns[4];
    int64_t n_residual[4];
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
};

// ------------------------------------------------------------------ distance
// sklearn/metrics/pairwise.py:582-653: X chunk upcast to f64,
// d = (-2 <x_i,x_j> + |x_i|^2) + |x_j|^2 (i < j, i is the "X" row as ripser.py
// reads dm[I > J]), cast to f32 (:651), clamp (:429), diag 0 (:436), sqrt (:441).
// The dot products and norms accumulate in increasing k with FMA, exact for
// f32 inputs (products are exact in f64).
template <typename T>
__global__ __launch_bounds__(256) void k_distance(const T* __restrict__ X, int n, int D, float* __restrict__ dist) {
    constexpr int TS = 16, KC = 32;
    __shared__ double xi[TS][KC + 1], xj[TS][KC + 1];
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
    if (i >= n || j >= n || j < i) return;
    if (i == j) {
        Dl[(size_t)i * n + i] = 0.0f;
        return;
    }
    double d = (-2.0 * dot + ni) + nj;
    float f;
    if constexpr (sizeof(T) == 4) {
        f = (float)d;
        f = (f != f) ? f : fmaxf(f, 0.0f);
        f = sqrt_rn_f32(f);
    } else {
        d = (d != d) ? d : fmax(d, 0.0);
        f = (float)__dsqrt_rn(d);
    }
    f = f + 0.0f;
    Dl[(size_t)i * n + j] = f;
    Dl[(size_t)j * n + i] = f;
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
// desc) by Prim (unique forest == Kruskal's), then Kruskal-order emission and
// elder-rule union-find [upstream compute_dim_0_pairs], consumed at
// debug_tda_pipeline.py:112, :126.
// LDS: best[N] u64, intree[N] u8 ... par[N] int  (N <= 8192)
__global__ __launch_bounds__(1024) void k_h0(const float* __restrict__ dist, int n, float user_thresh,
                                             LayerStats* __restrict__ stats, uint32_t* __restrict__ mst_bits,
                                             uint64_t mst_words, Pair* __restrict__ pairs0, uint64_t pcap0,
                                             uint64_t* __restrict__ scratch /* [L][2n] */, int sort_log2) {
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

    // -- threshold
    float thr = user_thresh;
    if (isinf(user_thresh) || user_thresh == 3.402823466e+38f) {
        float local = INFINITY;
        for (int i = w; i < n; i += nw) {
            float r = -INFINITY;
            for (int j = ln; j < n; j += 64) r = fmaxf(r, Dl[(size_t)i * n + j]);
            for (int m = 32; m >= 1; m >>= 1) r = fmaxf(r, __shfl_xor(r, m, 64));
            local = fminf(local, r);
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
            for (int j = i + 1 + ln; j < n; j += 64) c += Dl[(size_t)i * n + j] <= thr;
        atomicAdd(&s_cnt, c);
    }
    // -- Prim
    for (int v = t; v < n; v += T) {
        best[v] = kEmpty64;
        par[v] = 0;  // par doubles as in-tree flag during Prim
    }
    __syncthreads();
    if (t == 0) {
        st->thresh = thr;
        st->num_edges = (int64_t)s_cnt;
        s_cur = 0;
        par[0] = 1;
    }
    __syncthreads();
    uint64_t* mst = scratch + (size_t)l * 2 * n;  // MST edge keys
    int nmst = 0;
    for (int it = 1; it < n; ++it) {
        const int cur = s_cur;
        uint64_t mk = kEmpty64;
        for (int v = t; v < n; v += T) {
            if (par[v]) continue;
            float d = Dl[(size_t)cur * n + v];
            if (d <= thr) {
                int a = cur > v ? cur : v, b = cur > v ? v : cur;
                uint64_t k = filt_key(d, binom((uint64_t)a, 2) + b);
                if (k < best[v]) best[v] = k;
            }
            // candidate: (key, v) packed; key unique per edge, ties impossible
            uint64_t bk = best[v];
            if (bk < mk) mk = bk;
        }
        // find min key (and the vertex that owns it) across the block
        uint64_t wm = wave_min_u64(mk);
        if (ln == 0) red[w] = wm;
        __syncthreads();
        if (t == 0) {
            uint64_t m = kEmpty64;
            for (int q = 0; q < nw; ++q) m = red[q] < m ? red[q] : m;
            red[32] = m;
        }
        __syncthreads();
        const uint64_t gmin = red[32];
        if (gmin == kEmpty64) {
            // new component: smallest vertex not in the forest
            if (t == 0) red[33] = (uint64_t)n;
            __syncthreads();
            for (int v = t; v < n; v += T)
                if (!par[v]) atomicMin((unsigned long long*)&red[33], (unsigned long long)v);
            __syncthreads();
            if (t == 0) {
                s_cur = (int)red[33];
                par[s_cur] = 1;
            }
        } else {
            // the new vertex is the non-tree endpoint of edge gmin
            if (t == 0) {
                uint64_t eidx = 0xFFFFFFFFull - (gmin & 0xFFFFFFFFull);
                int a = max_vertex(eidx, 2, n - 1), b = (int)(eidx - binom((uint64_t)a, 2));
                int nv = par[a] ? b : a;
                par[nv] = 1;
                s_cur = nv;
                mst[nmst] = gmin;
            }
            ++nmst;
        }
        __syncthreads();
    }
    // -- Kruskal order of the forest edges
    block_sort<false>(mst, nullptr, (uint64_t)nmst, mst + n, nullptr, sk, nullptr, sort_log2);
    for (int e = t; e < nmst; e += T) {
        uint64_t eidx = 0xFFFFFFFFull - (mst[e] & 0xFFFFFFFFull);
        atomicOr(&mst_bits[(size_t)l * mst_words + (eidx >> 5)], 1u << (eidx & 31));
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
        for (int i = 0; i < n; ++i) {
            int u = i;
            while (par[u] != u) u = par[u];
            if (u == i) {
                if ((uint64_t)cnt < pcap0) P[cnt] = Pair{0.0f, INFINITY, (int64_t)i, -1};
                ++cnt;
            }
        }
        if ((uint64_t)cnt > pcap0) {
            st->err |= ERR_PAIR_CAP;
            cnt = (int64_t)pcap0;
        }
        st->count[0] = cnt;
        st->checksum[0] = cs;
        st->all_pairs[0] = nmst;
        st->n_columns[0] = n;
    }
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
template <int DIM>
__global__ __launch_bounds__(256) void k_apparent(const float* __restrict__ dist, int n, LayerStats* __restrict__ stats,
                                                  DimBufs b, Pair* __restrict__ pairs, uint64_t pcap) {
    const int l = blockIdx.y;
    const float* Dl = dist + (size_t)l * n * n;
    LayerStats* st = stats + l;
    const float r = st->thresh;
    const uint32_t* cleared = b.cleared + (size_t)l * b.cleared_words;
    uint32_t* piv = b.pivbits + (size_t)l * b.piv_words;
    uint64_t* resid = b.resid + (size_t)l * b.rcap;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t acc_cs = 0, acc_app = 0, acc_cols = 0;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < b.ncand; base += stride) {
        const uint64_t s = base + threadIdx.x;
        int kind = 0;  // 0 skip, 1 apparent, 2 residual, 3 essential
        int vs[DIM + 1];
        float sd = 0.0f;
        if (s < b.ncand && !((cleared[s >> 5] >> (s & 31)) & 1u)) {
            decode<DIM>(s, n, vs);
            sd = simplex_diam<DIM>(Dl, n, vs);
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
                    const float* row = Dl + (size_t)v * n;
#pragma unroll
                    for (int i = 0; i <= DIM; ++i) cd = fmaxf(cd, row[vs[i]]);
                    if (cd <= r && cd < bcd) {
                        bcd = cd;
                        bv = v;
                        if (cd == sd) break;
                    }
                }
                if (bv < 0) {
                    kind = 3;
                } else {
                    kind = 2;
                    if (bcd == sd) {
                        bool app = true;
                        const float* row = Dl + (size_t)bv * n;
#pragma unroll
                        for (int u = 0; u <= DIM; ++u) {
                            if (vs[u] < bv) continue;
                            // diam of (s u {bv}) \ {vs[u]}
                            float fd = 0.0f;
#pragma unroll
                            for (int i = 0; i <= DIM; ++i) {
                                if (i == u) continue;
                                fd = fmaxf(fd, row[vs[i]]);
#pragma unroll
                                for (int j = i + 1; j <= DIM; ++j)
                                    if (j != u) fd = fmaxf(fd, Dl[(size_t)vs[i] * n + vs[j]]);
                            }
                            app &= fd < sd;
                        }
                        if (app) {
                            kind = 1;
                            uint64_t tix = cofacet_index<DIM>(vs, bv);
                            atomicOr(&piv[tix >> 5], 1u << (tix & 31));
                            acc_cs += pair_hash(s, tix);
                            acc_app += 1;
                        }
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
                uint64_t pos = basepos + lanes_below(m);
                if (pos < b.rcap)
                    resid[pos] = col_key(sd, s);
                else
                    atomicOr(&st->err, ERR_RESID_CAP);
            }
        }
        if (kind == 3) {
            uint64_t pos = atomicAdd((unsigned long long*)&st->count[DIM], 1ull);
            if (pos < pcap)
                pairs[(size_t)l * pcap + pos] = Pair{sd, INFINITY, (int64_t)s, -1};
            else
                atomicOr(&st->err, ERR_PAIR_CAP);
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

// ------------------------------------------------------------------ sort residual
__global__ __launch_bounds__(1024) void k_sort_resid(LayerStats* __restrict__ stats, int dim, uint64_t* __restrict__ resid,
                                                     uint64_t rcap, uint64_t* __restrict__ tmp, uint64_t* __restrict__ rmap_keys,
                                                     uint64_t rmap_stride, int sort_log2) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.x;
    uint64_t cnt = (uint64_t)stats[l].n_residual[dim];
    if (cnt > rcap) cnt = rcap;
    block_sort<false>(resid + (size_t)l * rcap, nullptr, cnt, tmp + (size_t)l * rcap, nullptr, (uint64_t*)smem, nullptr,
                      sort_log2);
    // clear the residual pivot map region this layer will use
    uint64_t cap = 16;
    while (cap < 2 * cnt + 16) cap <<= 1;
    if (cap > rmap_stride) cap = rmap_stride;
    uint64_t* rk = rmap_keys + (size_t)l * rmap_stride;
    for (uint64_t e = threadIdx.x; e < cap; e += blockDim.x) rk[e] = kEmpty64;
}

// ------------------------------------------------------------------ reduce
// Serial part of compute_pairs [upstream ripser.cpp compute_pairs /
// add_coboundary]: the residual columns of one layer, in column order, reduced
// by ONE wave.  The working coboundary W and the working reduction column V are
// Z/2 toggle-sets (open addressing, parity bit per slot); the coboundary of a
// simplex is enumerated wave-parallel (one lane per new vertex); the pivot is a
// wave min over the live slots.  Pivot owners: residual columns in a global
// hash map (written by this kernel), apparent columns via the pivot bitmap
// (owner = youngest facet of the pivot, no lookup table needed).
struct ReduceBufs {
    uint64_t* rmap_keys;  // [L][rmap_stride]
    uint32_t* rmap_vals;
    uint64_t rmap_stride;
    uint32_t* voff;       // [L][rcap] offset of V_j in vpool
    uint32_t* vlen;
    uint64_t* vpool;      // [L][vpool_cap]
    uint64_t vpool_cap;
    // global working tables (used when not in LDS mode)
    uint64_t* wkeys;
    float* wdiam;
    uint32_t* wpar;
    uint32_t* wlist;
    uint64_t wcap;        // per layer, pow2
};

template <bool LDS>
struct ToggleSet {
    uint64_t* keys;
    float* diam;
    uint32_t* par;
    uint32_t* list;
    uint32_t* count;  // LDS scalar
    uint32_t mask;

    __device__ void clear_all(int t, int T) {
        for (uint32_t e = t; e <= mask; e += T) {
            keys[e] = kEmpty64;
            par[e] = 0;
        }
    }
    // clear only the touched slots (call with all lanes, then sync)
    __device__ void reset(int t, int T, uint32_t cnt) {
        for (uint32_t e = t; e < cnt; e += T) {
            uint32_t s = list[e];
            keys[s] = kEmpty64;
            par[s] = 0;
        }
    }
    // toggle key (unique among concurrent callers)
    __device__ void toggle(uint64_t k, float d) {
        uint32_t h = (uint32_t)mix64(k) & mask;
        for (;;) {
            uint64_t cur = keys[h];
            if (cur == k) break;
            if (cur == kEmpty64) {
                unsigned long long old = atomicCAS((unsigned long long*)&keys[h], (unsigned long long)kEmpty64, (unsigned long long)k);
                if (old == kEmpty64) {
                    diam[h] = d;
                    uint32_t pos = atomicAdd(count, 1u);
                    list[pos] = h;
                    break;
                }
                if (old == k) break;
            }
            h = (h + 1) & mask;
        }
        par[h] ^= 1u;
    }
};

template <int DIM>
__device__ __forceinline__ void youngest_facet(const float* __restrict__ D, int n, uint64_t tidx, uint64_t& fidx, float& fd) {
    int tv[DIM + 2];
    decode<DIM + 1>(tidx, n, tv);
    fd = -1.0f;
    fidx = 0;
#pragma unroll
    for (int u = 0; u <= DIM + 1; ++u) {
        int fv[DIM + 1];
        int q = 0;
#pragma unroll
        for (int i = 0; i <= DIM + 1; ++i)
            if (i != u) fv[q++] = tv[i];
        float d = simplex_diam<DIM>(D, n, fv);
        uint64_t ix = encode<DIM>(fv);
        if (d > fd || (d == fd && ix < fidx)) {
            fd = d;
            fidx = ix;
        }
    }
}

template <int DIM, bool LDS>
__global__ __launch_bounds__(64) void k_reduce(const float* __restrict__ dist, int n, LayerStats* __restrict__ stats, DimBufs b,
                                               ReduceBufs rb, Pair* __restrict__ pairs, uint64_t pcap, uint32_t wcap_lds,
                                               uint32_t vcap_lds, int dist_in_lds) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.x, ln = threadIdx.x;
    LayerStats* st = stats + l;
    const float r = st->thresh;
    uint64_t nres = (uint64_t)st->n_residual[DIM];
    if (nres > b.rcap) nres = b.rcap;
    if (nres == 0) return;
    const uint64_t* resid = b.resid + (size_t)l * b.rcap;
    uint32_t* piv = b.pivbits + (size_t)l * b.piv_words;

    // carve LDS (all scratch in the dynamic region, 16-B aligned)
    uint32_t& wcount = *(uint32_t*)smem;
    uint32_t& vcount = *(uint32_t*)(smem + 4);
    uint32_t& s_err = *(uint32_t*)(smem + 8);
    unsigned char* p = smem + 16;
    ToggleSet<LDS> W, V;
    uint32_t wcap, vcap;
    if (LDS) {
        wcap = wcap_lds;
        vcap = vcap_lds;
        W.keys = (uint64_t*)p; p += sizeof(uint64_t) * wcap;
        V.keys = (uint64_t*)p; p += sizeof(uint64_t) * vcap;
        W.diam = (float*)p; p += sizeof(float) * wcap;
        W.par = (uint32_t*)p; p += sizeof(uint32_t) * wcap;
        W.list = (uint32_t*)p; p += sizeof(uint32_t) * wcap;
        V.diam = (float*)p; p += sizeof(float) * vcap;
        V.par = (uint32_t*)p; p += sizeof(uint32_t) * vcap;
        V.list = (uint32_t*)p; p += sizeof(uint32_t) * vcap;
    } else {
        wcap = (uint32_t)rb.wcap;
        vcap = vcap_lds;
        W.keys = rb.wkeys + (size_t)l * wcap;
        W.diam = rb.wdiam + (size_t)l * wcap;
        W.par = rb.wpar + (size_t)l * wcap;
        W.list = rb.wlist + (size_t)l * wcap;
        V.keys = (uint64_t*)p; p += sizeof(uint64_t) * vcap;
        V.diam = (float*)p; p += sizeof(float) * vcap;
        V.par = (uint32_t*)p; p += sizeof(uint32_t) * vcap;
        V.list = (uint32_t*)p; p += sizeof(uint32_t) * vcap;
    }
    const float* D = dist + (size_t)l * n * n;
    if (dist_in_lds) {
        float* dl = (float*)p;
        for (int e = ln; e < n * n; e += 64) dl[e] = D[e];
        D = dl;
    }
    W.mask = wcap - 1;
    V.mask = vcap - 1;
    W.count = &wcount;
    V.count = &vcount;
    W.clear_all(ln, 64);
    V.clear_all(ln, 64);
    if (ln == 0) {
        wcount = 0;
        vcount = 0;
        s_err = 0;
    }
    __syncthreads();

    uint64_t* rk = rb.rmap_keys + (size_t)l * rb.rmap_stride;
    uint32_t* rvl = rb.rmap_vals + (size_t)l * rb.rmap_stride;
    uint64_t rcap2 = 16;
    while (rcap2 < 2 * nres + 16) rcap2 <<= 1;
    if (rcap2 > rb.rmap_stride) rcap2 = rb.rmap_stride;
    const uint64_t rmask = rcap2 - 1;
    uint32_t* voff = rb.voff + (size_t)l * b.rcap;
    uint32_t* vlen = rb.vlen + (size_t)l * b.rcap;
    uint64_t* vpool = rb.vpool + (size_t)l * rb.vpool_cap;
    uint64_t vused = 0;  // uniform
    Pair* P = pairs + (size_t)l * pcap;
    uint64_t cs = 0, npairs = 0;

    // toggle the coboundary of simplex s (diam sd) into W: one pass
    auto add_cob = [&](uint64_t s, float sd) {
        if (wcount + (uint32_t)n > (wcap >> 1) + (wcap >> 2)) {
            __syncthreads();
            if (ln == 0) s_err = 1;
            __syncthreads();
            return;
        }
        int vs[DIM + 1];
        decode<DIM>(s, n, vs);
        for (int v = ln; v < n; v += 64) {
            bool mem = false;
#pragma unroll
            for (int i = 0; i <= DIM; ++i) mem |= (vs[i] == v);
            if (mem) continue;
            float cd = sd;
            const float* row = D + (size_t)v * n;
#pragma unroll
            for (int i = 0; i <= DIM; ++i) cd = fmaxf(cd, row[vs[i]]);
            if (cd <= r) W.toggle(cofacet_index<DIM>(vs, v), cd);
        }
        __syncthreads();
    };
    auto vtoggle = [&](uint64_t s) {
        if (vcount + 2 > (vcap >> 1) + (vcap >> 2)) {
            __syncthreads();
            if (ln == 0) s_err = 1;
            __syncthreads();
            return;
        }
        if (ln == 0) V.toggle(s, 0.0f);
        __syncthreads();
    };

    for (uint64_t j = 0; j < nres; ++j) {
        const uint64_t key = resid[j];
        const uint64_t sidx = key_idx(key);
        const float sdm = key_diam(key);
        add_cob(sidx, sdm);
        bool done = false;
        while (!done) {
            if (s_err) break;
            // pivot: min diam, then max index, over live slots
            const uint32_t cnt = wcount;
            float bd = INFINITY;
            uint64_t bi = 0;
            bool has = false;
            for (uint32_t e = ln; e < cnt; e += 64) {
                uint32_t sl = W.list[e];
                if (W.par[sl]) {
                    float d = W.diam[sl];
                    uint64_t k = W.keys[sl];
                    if (!has || d < bd || (d == bd && k > bi)) {
                        bd = d;
                        bi = k;
                        has = true;
                    }
                }
            }
            uint32_t db = has ? __float_as_uint(bd) : 0xFFFFFFFFu;
            uint32_t dmin = wave_min_u32(db);
            uint64_t cand = (has && db == dmin) ? bi : 0;
            uint64_t imax = wave_max_u64(cand);
            bool anyw = dmin != 0xFFFFFFFFu;
            if (!anyw) {
                // zero column: essential class
                if (ln == 0) {
                    uint64_t pos = atomicAdd((unsigned long long*)&st->count[DIM], 1ull);
                    if (pos < pcap) P[pos] = Pair{sdm, INFINITY, (int64_t)sidx, -1};
                    else atomicOr(&st->err, ERR_PAIR_CAP);
                    voff[j] = 0;
                    vlen[j] = 0;
                }
                done = true;
                break;
            }
            const float pd = __uint_as_float(dmin);
            const uint64_t pidx = imax;
            // owner lookup (lane 0)
            int64_t owner = -1;
            if (ln == 0) {
                uint64_t h = mix64(pidx) & rmask;
                while (rk[h] != kEmpty64) {
                    if (rk[h] == pidx) {
                        owner = rvl[h];
                        break;
                    }
                    h = (h + 1) & rmask;
                }
            }
            owner = (int64_t)shfl_u64((uint64_t)owner, 0);
            if (owner >= 0) {
                const uint64_t ok = resid[owner];
                add_cob(key_idx(ok), key_diam(ok));
                vtoggle(key_idx(ok));
                const uint32_t o0 = voff[owner], ol = vlen[owner];
                for (uint32_t q = 0; q < ol; ++q) {
                    uint64_t s = vpool[o0 + q];
                    int vs[DIM + 1];
                    decode<DIM>(s, n, vs);
                    add_cob(s, simplex_diam<DIM>(D, n, vs));
                    vtoggle(s);
                }
            } else if ((piv[pidx >> 5] >> (pidx & 31)) & 1u) {
                uint64_t fidx;
                float fd;
                youngest_facet<DIM>(D, n, pidx, fidx, fd);
                add_cob(fidx, fd);
                vtoggle(fidx);
            } else {
                // new pair (sigma_j, pivot)
                if (ln == 0) {
                    if (pd > sdm) {
                        uint64_t pos = atomicAdd((unsigned long long*)&st->count[DIM], 1ull);
                        if (pos < pcap) P[pos] = Pair{sdm, pd, (int64_t)sidx, (int64_t)pidx};
                        else atomicOr(&st->err, ERR_PAIR_CAP);
                    }
                    uint64_t h = mix64(pidx) & rmask;
                    while (rk[h] != kEmpty64) h = (h + 1) & rmask;
                    rk[h] = pidx;
                    rvl[h] = (uint32_t)j;
                    atomicOr(&piv[pidx >> 5], 1u << (pidx & 31));
                }
                cs += pair_hash(sidx, pidx);
                npairs += 1;
                // store V_j (live entries of V)
                const uint32_t vc = vcount;
                uint64_t wr = 0;
                for (uint32_t e0 = 0; e0 < vc; e0 += 64) {
                    uint32_t e = e0 + ln;
                    bool live = false;
                    uint64_t k = 0;
                    if (e < vc) {
                        uint32_t sl = V.list[e];
                        live = V.par[sl] != 0;
                        k = V.keys[sl];
                    }
                    uint64_t m = __ballot(live);
                    if (live) {
                        uint64_t pos = vused + wr + lanes_below(m);
                        if (pos < rb.vpool_cap) vpool[pos] = k;
                    }
                    wr += __popcll(m);
                }
                if (vused + wr > rb.vpool_cap) {
                    if (ln == 0) s_err = 2;
                    wr = 0;
                }
                if (ln == 0) {
                    voff[j] = (uint32_t)vused;
                    vlen[j] = (uint32_t)wr;
                }
                vused += wr;
                done = true;
            }
        }
        __syncthreads();
        if (s_err) break;
        // reset the tables for the next column
        W.reset(ln, 64, wcount);
        V.reset(ln, 64, vcount);
        __syncthreads();
        if (ln == 0) {
            wcount = 0;
            vcount = 0;
        }
        __syncthreads();
    }
    if (ln == 0) {
        if (s_err == 1) atomicOr(&st->err, ERR_WORK_CAP);
        if (s_err == 2) atomicOr(&st->err, ERR_VPOOL_CAP);
        atomicAdd((unsigned long long*)&st->checksum[DIM], (unsigned long long)cs);
        atomicAdd((unsigned long long*)&st->all_pairs[DIM], (unsigned long long)npairs);
    }
}

// ------------------------------------------------------------------ finalize
// Emission order of dims >= 1 (reference: births_and_deaths_by_dim filled in
// column order, i.e. birth desc / column index asc; pinned 32/32 by
// summary_stats.json all_h1_persistence_values).
__global__ __launch_bounds__(1024) void k_finalize(LayerStats* __restrict__ stats, int maxdim, Pair* const* __restrict__ pairs,
                                                   const uint64_t* __restrict__ pcap, uint64_t* __restrict__ skeys,
                                                   uint32_t* __restrict__ svals, uint64_t sstride, int sort_log2) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.x;
    const uint64_t CH = 1ull << sort_log2;
    uint64_t* sk = (uint64_t*)smem;
    uint32_t* sv = (uint32_t*)(sk + CH);
    for (int d = 1; d <= maxdim; ++d) {
        uint64_t cnt = (uint64_t)stats[l].count[d];
        if (cnt > pcap[d]) cnt = pcap[d];
        if (cnt < 2) continue;
        Pair* P = pairs[d] + (size_t)l * pcap[d];
        uint64_t* k = skeys + (size_t)l * sstride * 2;
        uint32_t* v = svals + (size_t)l * sstride * 2;
        for (uint64_t e = threadIdx.x; e < cnt; e += blockDim.x) {
            k[e] = col_key(P[e].birth, (uint64_t)P[e].birth_idx);
            v[e] = (uint32_t)e;
        }
        __syncthreads();
        block_sort<true>(k, v, cnt, k + sstride, v + sstride, sk, sv, sort_log2);
        // permute through the scratch (pairs -> scratch bytes -> pairs)
        Pair* tmpP = (Pair*)(k + sstride);  // sstride*8 bytes >= cnt*24? ensured by host (sstride >= 3*pcap)
        for (uint64_t e = threadIdx.x; e < cnt; e += blockDim.x) tmpP[e] = P[v[e]];
        __syncthreads();
        for (uint64_t e = threadIdx.x; e < cnt; e += blockDim.x) P[e] = tmpP[e];
        __syncthreads();
    }
}

// ------------------------------------------------------------------ compact
// Pack every (layer, dim) segment into the host-mapped output.
struct OutPair {
    float birth, death;
    int64_t birth_idx, death_idx;
};
__global__ __launch_bounds__(1024) void k_compact(LayerStats* __restrict__ stats, int L, int maxdim, Pair* const* __restrict__ pairs,
                                                  const uint64_t* __restrict__ pcap, int64_t* __restrict__ out_off,
                                                  OutPair* __restrict__ out, uint64_t out_cap) {
    __shared__ int64_t s_total;
    const int nd = maxdim + 1;
    if (threadIdx.x == 0) {
        int64_t acc = 0;
        for (int l = 0; l < L; ++l)
            for (int d = 0; d < nd; ++d) {
                int64_t c = stats[l].count[d];
                if ((uint64_t)c > pcap[d]) c = (int64_t)pcap[d];
                out_off[l * nd + d] = acc;
                acc += c;
            }
        s_total = acc;
        if ((uint64_t)acc > out_cap)
            for (int l = 0; l < L; ++l) stats[l].err |= ERR_OUT_CAP;
    }
    __syncthreads();
    if ((uint64_t)s_total > out_cap) return;
    for (int l = 0; l < L; ++l)
        for (int d = 0; d < nd; ++d) {
            int64_t c = stats[l].count[d];
            if ((uint64_t)c > pcap[d]) c = (int64_t)pcap[d];
            const Pair* P = pairs[d] + (size_t)l * pcap[d];
            OutPair* o = out + out_off[l * nd + d];
            for (int64_t e = threadIdx.x; e < c; e += blockDim.x) o[e] = OutPair{P[e].birth, P[e].death, P[e].birth_idx, P[e].death_idx};
        }
}

}  // namespace tda
