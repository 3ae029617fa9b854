// umap_kernels.h -- gfx950 kernels of the per-layer UMAP embedding that the
// reference runs right before ripser (debug_tda_pipeline.py:96-104:
// umap.UMAP(n_neighbors=6, n_components=3, min_dist=0.1, random_state=42,
// metric='cosine').fit_transform(cloud_high_dim); analyze_tda_over_layers.py:
// 38-44, :67-72; analyze_adversarial_tda.py).  umap-learn is not vendored in
// the reference and not installed here; these kernels restate its published
// algorithm for the reference's regime (N < 4096: exact pairwise distances):
//
//   k_umap_knn      k nearest neighbours of every point from its distance row
//                   (self included, (distance, index) order) -- umap
//                   nearest_neighbors / fast_knn_indices on the full matrix
//   k_umap_smooth   smooth_knn_dist (rho = nearest non-zero distance, sigma by
//                   64-step bisection on sum exp(-(d - rho) / sigma) =
//                   log2(k), MIN_K_DIST_SCALE floor) and
//                   compute_membership_strengths -> directed weights P (dense)
//   k_umap_sym      fuzzy union S = (P + P^T) - P o P^T (set_op_mix_ratio 1)
//   k_umap_edges    prune S < max(S) / n_epochs, edge list in row-major (CSR)
//                   order, epochs_per_sample = n_epochs / (n_epochs w / w_max),
//                   degrees for the spectral layout
//   k_umap_spectral spectral_layout: the c eigenvectors of the normalised
//                   Laplacian I - D^-1/2 S D^-1/2 after the trivial one, by
//                   block subspace iteration on (M + I) / 2 with Gram-Schmidt
//                   and a final Rayleigh-Ritz step; then umap's scaling
//                   (10 / max|.|, N(0, 1e-4) noise, min-max to [0, 10])
//   k_umap_sgd      optimize_layout_euclidean: 1/(1 + a d^2b) attraction along
//                   edges (both ends move), negative_sample_rate repulsive
//                   samples per edge sample, clip 4, alpha = lr (1 - n/epochs).
//                   MI355X-specific: epoch-synchronous updates -- every edge of
//                   an epoch reads the epoch-start layout and its moves are
//                   summed in LDS as 2^-40 fixed-point int64 atomics, so the
//                   result is deterministic for a seed whatever the thread
//                   schedule (umap-learn's numba loop is sequential with a
//                   seed and Hogwild-parallel without one).  The random
//                   streams depend on the seed only, not on the layer, so a
//                   layer embeds the same alone or in a batch (the reference
//                   passes random_state=42 for every layer).
#pragma once
#include "rips_device.h"

namespace tda {

constexpr int kUmapMaxK = 64;        // n_neighbors
constexpr int kUmapMaxC = 8;         // n_components
constexpr int kUmapKnnT = 64;        // k_umap_knn threads per block (LDS lists of kUmapMaxK per thread)
constexpr int kUmapT = 1024;         // one workgroup per layer: smooth / edges / spectral / sgd
constexpr int kUmapSpecMaxN = 2048;  // spectral layout up to here (V, W in LDS); random init above
constexpr double kUmapFix = 1099511627776.0;  // 2^40: fixed-point scale of the SGD move sums

struct UmapBufs {
    const float* dist;      // [L][N][N]
    float* kd;              // [L][N][k] neighbour distances
    int32_t* ki;            // [L][N][k] neighbour indices
    float* P;               // [L][N][N] directed memberships (zeroed per call)
    float* S;               // [L][N][N] fuzzy union
    uint32_t* smax;         // [L] max S (float bits; zeroed per call)
    int32_t* head;          // [L][ecap]
    int32_t* tail;          // [L][ecap]
    double* eps;            // [L][ecap] epochs per sample
    double* nxt;            // [L][ecap] epoch of next sample
    double* nxn;            // [L][ecap] epoch of next negative sample
    float* deg;             // [L][N] row sums of the pruned S
    uint32_t* nedge;        // [L] edge count (zeroed per call)
    float* emb;             // [L][N][c] layout (init, then the result)
    uint64_t ecap;
    int n, k, c, n_epochs;
    // kNN rows: queries qrow0 .. qrow0 + nq - 1 of a layer's distance matrix
    // (row length `stride`, `lstride` floats per layer) against its first
    // `ncand` columns.  Fit: all n rows against all n points; transform: the
    // M new points (rows N..N+M-1 of [train; new]) against the N training points.
    size_t lstride;
    int stride, qrow0, nq, ncand;
};

__device__ __forceinline__ uint64_t umap_hash(uint64_t a, uint64_t b) { return mix64(a * 0x9E3779B97F4A7C15ull ^ mix64(b + 0x632BE59BD9B4E019ull)); }

// block-wide sum of a double (all threads call)
__device__ __forceinline__ double umap_block_sum(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
    return s;
}

// ---------------------------------------------------------------- kNN
// thread per point: the k smallest (distance, index) of its row, by insertion
// into an LDS list (insertions are rare once the list is warm)
__global__ __launch_bounds__(kUmapKnnT) void k_umap_knn(UmapBufs u) {
    __shared__ float ld[kUmapKnnT][kUmapMaxK];
    __shared__ int32_t li[kUmapKnnT][kUmapMaxK];
    const int l = blockIdx.y, t = threadIdx.x, i = blockIdx.x * kUmapKnnT + t, nq = u.nq, k = u.k;
    if (i >= nq) return;
    const float* row = u.dist + (size_t)l * u.lstride + (size_t)(u.qrow0 + i) * u.stride;
    int cnt = 0;
    for (int j = 0; j < u.ncand; ++j) {
        const float d = ld_glb(row, j);
        if (cnt == k && !(d < ld[t][k - 1])) continue;  // ties keep the smaller index (already in)
        int p = cnt < k ? cnt++ : k - 1;
        while (p > 0 && ld[t][p - 1] > d) {
            ld[t][p] = ld[t][p - 1];
            li[t][p] = li[t][p - 1];
            --p;
        }
        ld[t][p] = d;
        li[t][p] = j;
    }
    float* kd = u.kd + ((size_t)l * nq + i) * k;
    int32_t* ki = u.ki + ((size_t)l * nq + i) * k;
    for (int q = 0; q < k; ++q) {
        kd[q] = ld[t][q];
        ki[q] = li[t][q];
    }
}

// ---------------------------------------------------------------- smooth kNN + memberships
// umap smooth_knn_dist (local_connectivity 1, bandwidth 1, n_iter 64) in f64
// on the f32 neighbour distances, then compute_membership_strengths
__global__ __launch_bounds__(kUmapT) void k_umap_smooth(UmapBufs u) {
    __shared__ double red[kUmapT / 64];
    const int l = blockIdx.x, n = u.n, k = u.k;
    const float* kd = u.kd + (size_t)l * n * k;
    const int32_t* ki = u.ki + (size_t)l * n * k;
    double s = 0.0;
    for (int e = threadIdx.x; e < n * k; e += kUmapT) s += (double)kd[e];
    const double mean_all = umap_block_sum(s, red) / (double)(n * k);
    const double target = log2((double)k);
    float* P = u.P + (size_t)l * n * n;
    for (int i = threadIdx.x; i < n; i += kUmapT) {
        const float* d = kd + (size_t)i * k;
        double rho = 0.0, mean_i = 0.0;
        bool nz = false;
        for (int j = 0; j < k; ++j) {
            mean_i += (double)d[j];
            if (d[j] > 0.0f && !nz) {  // local_connectivity 1: rho = the smallest non-zero distance
                rho = (double)d[j];
                nz = true;
            }
        }
        mean_i /= (double)k;
        double lo = 0.0, hi = INFINITY, mid = 1.0;
        for (int it = 0; it < 64; ++it) {
            double psum = 0.0;
            for (int j = 1; j < k; ++j) {
                const double dd = (double)d[j] - rho;
                psum += dd > 0.0 ? exp(-(dd / mid)) : 1.0;
            }
            if (fabs(psum - target) < 1e-5) break;
            if (psum > target) {
                hi = mid;
                mid = (lo + hi) / 2.0;
            } else {
                lo = mid;
                mid = isinf(hi) ? mid * 2.0 : (lo + hi) / 2.0;
            }
        }
        double sigma = mid;
        if (rho > 0.0) {
            if (sigma < 1e-3 * mean_i) sigma = 1e-3 * mean_i;
        } else if (sigma < 1e-3 * mean_all) {
            sigma = 1e-3 * mean_all;
        }
        for (int j = 0; j < k; ++j) {
            const int c = ki[(size_t)i * k + j];
            float val;
            if (c == i)
                val = 0.0f;
            else if ((double)d[j] - rho <= 0.0 || sigma == 0.0)
                val = 1.0f;
            else
                val = (float)exp(-(((double)d[j] - rho) / sigma));
            P[(size_t)i * n + c] = val;
        }
    }
}

// ---------------------------------------------------------------- fuzzy union
__global__ __launch_bounds__(256) void k_umap_sym(UmapBufs u) {
    const int l = blockIdx.y, n = u.n;
    const size_t nn = (size_t)n * n;
    const float* P = u.P + (size_t)l * nn;
    float* S = u.S + (size_t)l * nn;
    uint32_t mx = 0;
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < nn; q += (size_t)gridDim.x * blockDim.x) {
        const size_t i = q / n, j = q - i * n;
        const float p = P[q], pt = P[j * n + i];
        // scipy float32 ops: (P + P^T) - (P o P^T), no contraction
        const float v = __fsub_rn(__fadd_rn(p, pt), __fmul_rn(p, pt));
        S[q] = v;
        mx = max(mx, __float_as_uint(v));  // v >= 0
    }
    mx = (uint32_t)wave_max_u64(mx);
    if ((threadIdx.x & 63) == 0 && mx) atomicMax(&u.smax[l], mx);
}

// ---------------------------------------------------------------- edges
// one workgroup per layer: rows in order, each row's surviving entries
// compacted in column order (CSR / COO order of the symmetric graph)
__global__ __launch_bounds__(kUmapT) void k_umap_edges(UmapBufs u) {
    __shared__ uint32_t wsum[kUmapT / 64];
    __shared__ double red[kUmapT / 64];
    __shared__ uint32_t base_sh;
    const int l = blockIdx.x, n = u.n, t = threadIdx.x;
    const float smax = __uint_as_float(u.smax[l]);
    const double thr = (double)smax / (double)u.n_epochs;
    float* S = u.S + (size_t)l * n * n;
    if (t == 0) base_sh = 0;
    __syncthreads();
    for (int i = 0; i < n; ++i) {
        float* row = S + (size_t)i * n;
        double rs = 0.0;
        for (int j0 = 0; j0 < n; j0 += kUmapT) {
            const int j = j0 + t;
            float w = j < n ? row[j] : 0.0f;
            if (w > 0.0f && (double)w < thr) {  // pruned (graph.data < max / n_epochs)
                w = 0.0f;
                row[j] = 0.0f;
            }
            const bool e = w > 0.0f;
            rs += (double)w;
            const uint64_t m = __ballot(e);
            if ((t & 63) == 0) wsum[t >> 6] = (uint32_t)__popcll(m);
            __syncthreads();
            uint32_t before = 0, tot = 0;
            for (int q = 0; q < kUmapT / 64; ++q) {
                before += q < (t >> 6) ? wsum[q] : 0;
                tot += wsum[q];
            }
            const uint32_t pos = base_sh + before + lanes_below(m);
            if (e && pos < u.ecap) {
                const size_t o = (size_t)l * u.ecap + pos;
                u.head[o] = i;
                u.tail[o] = j;
                // make_epochs_per_sample: n_samples = n_epochs * (w / w_max) in f32, eps = n_epochs / n_samples (f64)
                const float ns = __fmul_rn((float)u.n_epochs, __fdiv_rn(w, smax));
                const double eps = (double)u.n_epochs / (double)ns;
                u.eps[o] = eps;
                u.nxt[o] = eps;
                u.nxn[o] = eps;  // k_umap_sgd divides by negative_sample_rate
            }
            __syncthreads();
            if (t == 0) base_sh += tot;
            __syncthreads();
        }
        const double r = umap_block_sum(rs, red);
        if (t == 0) u.deg[(size_t)l * n + i] = (float)r;
        __syncthreads();
    }
    if (t == 0) u.nedge[l] = base_sh;
}

// ---------------------------------------------------------------- spectral layout
// top B = c + 3 eigenvectors of (M + I) / 2, M = D^-1/2 S D^-1/2, by block
// subspace iteration (V, W in LDS as f32), Gram-Schmidt every step, then a
// Rayleigh-Ritz rotation; column 0 (eigenvalue 1, the trivial D^1/2 1) is
// dropped.  Then umap's init scaling and noise.
__global__ __launch_bounds__(kUmapT) void k_umap_spectral(UmapBufs u, int iters, uint64_t seed, int random_init) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ double red[kUmapT / 64];
    __shared__ double H[kUmapMaxC + 3][kUmapMaxC + 3], Q[kUmapMaxC + 3][kUmapMaxC + 3];
    __shared__ int order[kUmapMaxC + 3];
    __shared__ float colmin[kUmapMaxC], colmax[kUmapMaxC];
    const int l = blockIdx.x, n = u.n, c = u.c, t = threadIdx.x;
    const int B = c + 3;
    float* V = (float*)smem;         // [B][n]
    float* W = V + (size_t)B * n;    // [B][n]
    float* dis = W + (size_t)B * n;  // [n] D^-1/2
    const float* S = u.S + (size_t)l * n * n;
    float* emb = u.emb + (size_t)l * n * c;
    auto rnd_unit = [&](uint64_t a, uint64_t b) {  // uniform in [0, 1)
        return (double)(umap_hash(seed, a * 1000003ull + b) >> 11) * (1.0 / 9007199254740992.0);
    };
    if (!random_init) {
        for (int i = t; i < n; i += kUmapT) {
            const float d = u.deg[(size_t)l * n + i];
            dis[i] = d > 0.0f ? 1.0f / sqrtf(d) : 0.0f;
        }
        for (int e = t; e < B * n; e += kUmapT) V[e] = (float)(rnd_unit(1, e) - 0.5);
        __syncthreads();
        auto orthonormalize = [&](float* X) {
            for (int a = 0; a < B; ++a) {
                for (int b = 0; b < a; ++b) {
                    double s = 0.0;
                    for (int i = t; i < n; i += kUmapT) s += (double)X[a * n + i] * X[b * n + i];
                    s = umap_block_sum(s, red);
                    for (int i = t; i < n; i += kUmapT) X[a * n + i] -= (float)s * X[b * n + i];
                    __syncthreads();
                }
                double s = 0.0;
                for (int i = t; i < n; i += kUmapT) s += (double)X[a * n + i] * X[a * n + i];
                s = umap_block_sum(s, red);
                const float inv = s > 0.0 ? (float)(1.0 / sqrt(s)) : 0.0f;
                for (int i = t; i < n; i += kUmapT) X[a * n + i] *= inv;
                __syncthreads();
            }
        };
        orthonormalize(V);
        // (M x)_i = dis_i sum_j S_ji dis_j x_j (S symmetric: column reads coalesce over i)
        auto apply = [&](const float* X, float* Y, bool shift) {
            for (int i = t; i < n; i += kUmapT) {
                float acc[kUmapMaxC + 3];
                for (int a = 0; a < B; ++a) acc[a] = 0.0f;
                for (int j = 0; j < n; ++j) {
                    const float s = ld_glb(S, (size_t)j * n + i) * dis[j];
                    if (s != 0.0f)
                        for (int a = 0; a < B; ++a) acc[a] = fmaf(s, X[a * n + j], acc[a]);
                }
                for (int a = 0; a < B; ++a) Y[a * n + i] = shift ? 0.5f * (dis[i] * acc[a] + X[a * n + i]) : dis[i] * acc[a];
            }
            __syncthreads();
        };
        for (int it = 0; it < iters; ++it) {
            apply(V, W, true);
            orthonormalize(W);
            float* tmp = V;
            V = W;
            W = tmp;
        }
        // Rayleigh-Ritz: H = V^T M V, eigenvectors by cyclic Jacobi (thread 0, f64)
        apply(V, W, false);
        for (int a = 0; a < B; ++a)
            for (int b = 0; b < B; ++b) {
                double s = 0.0;
                for (int i = t; i < n; i += kUmapT) s += (double)V[a * n + i] * W[b * n + i];
                s = umap_block_sum(s, red);
                if (t == 0) H[a][b] = s;
            }
        __syncthreads();
        if (t == 0) {
            for (int a = 0; a < B; ++a)
                for (int b = 0; b < B; ++b) Q[a][b] = a == b ? 1.0 : 0.0;
            for (int a = 0; a < B; ++a)
                for (int b = a + 1; b < B; ++b) H[a][b] = H[b][a] = 0.5 * (H[a][b] + H[b][a]);
            for (int sweep = 0; sweep < 60; ++sweep) {
                double off = 0.0;
                for (int p = 0; p < B; ++p)
                    for (int q = p + 1; q < B; ++q) off += H[p][q] * H[p][q];
                if (off < 1e-30) break;
                for (int p = 0; p < B; ++p)
                    for (int q = p + 1; q < B; ++q) {
                        if (fabs(H[p][q]) < 1e-300) continue;
                        const double th = (H[q][q] - H[p][p]) / (2.0 * H[p][q]);
                        const double tt = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
                        const double cs = 1.0 / sqrt(tt * tt + 1.0), sn = tt * cs;
                        for (int r = 0; r < B; ++r) {  // H <- J^T H J, Q <- Q J
                            const double hp = H[r][p], hq = H[r][q];
                            H[r][p] = cs * hp - sn * hq;
                            H[r][q] = sn * hp + cs * hq;
                        }
                        for (int r = 0; r < B; ++r) {
                            const double hp = H[p][r], hq = H[q][r];
                            H[p][r] = cs * hp - sn * hq;
                            H[q][r] = sn * hp + cs * hq;
                        }
                        for (int r = 0; r < B; ++r) {
                            const double qp = Q[r][p], qq = Q[r][q];
                            Q[r][p] = cs * qp - sn * qq;
                            Q[r][q] = sn * qp + cs * qq;
                        }
                    }
            }
            for (int a = 0; a < B; ++a) order[a] = a;
            for (int a = 0; a < B; ++a)  // eigenvalues of M descending (L = I - M ascending)
                for (int b = a + 1; b < B; ++b)
                    if (H[order[b]][order[b]] > H[order[a]][order[a]]) {
                        const int x = order[a];
                        order[a] = order[b];
                        order[b] = x;
                    }
        }
        __syncthreads();
        // eigenvectors 1..c (after the trivial one) into W[0..c)
        for (int i = t; i < n; i += kUmapT)
            for (int d = 0; d < c; ++d) {
                const int col = order[d + 1];
                double s = 0.0;
                for (int a = 0; a < B; ++a) s += Q[a][col] * (double)V[a * n + i];
                W[d * n + i] = (float)s;
            }
        __syncthreads();
        // expansion = 10 / max|init|; init * expansion + N(0, 1e-4) (umap simplicial_set_embedding)
        double m = 0.0;
        for (int e = t; e < c * n; e += kUmapT) m = fmax(m, fabs((double)W[e]));
        for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
        __syncthreads();
        if ((t & 63) == 0) red[t >> 6] = m;
        __syncthreads();
        m = 0.0;
        for (int w = 0; w < kUmapT / 64; ++w) m = fmax(m, red[w]);
        const double expn = m > 0.0 ? 10.0 / m : 1.0;
        for (int e = t; e < c * n; e += kUmapT) {
            const int i = e / c, d = e - i * c;
            const double u1 = fmax(rnd_unit(2, e), 1e-300), u2 = rnd_unit(3, e);
            const double g = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
            emb[e] = (float)(W[d * n + i] * expn) + (float)(1e-4 * g);
        }
    } else {  // random init: uniform in [-10, 10] (umap init='random')
        for (int e = t; e < c * n; e += kUmapT) emb[e] = (float)(20.0 * rnd_unit(4, e) - 10.0);
    }
    __syncthreads();
    // min-max scale every column to [0, 10]
    if (t < c) {
        float lo = INFINITY, hi = -INFINITY;
        for (int i = 0; i < n; ++i) {
            lo = fminf(lo, emb[i * c + t]);
            hi = fmaxf(hi, emb[i * c + t]);
        }
        colmin[t] = lo;
        colmax[t] = hi;
    }
    __syncthreads();
    for (int e = t; e < c * n; e += kUmapT) {
        const int d = e % c;
        const float span = colmax[d] - colmin[d];
        emb[e] = span > 0.0f ? 10.0f * (emb[e] - colmin[d]) / span : 0.0f;
    }
}

// ---------------------------------------------------------------- SGD
__device__ __forceinline__ double umap_clip(double v) { return v > 4.0 ? 4.0 : (v < -4.0 ? -4.0 : v); }

__global__ __launch_bounds__(kUmapT) void k_umap_sgd(UmapBufs u, double a, double b, double lr, double gamma, int neg_rate,
                                                     uint64_t seed) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int l = blockIdx.x, n = u.n, c = u.c, t = threadIdx.x;
    float* E = (float*)smem;                                                  // [n][c]
    long long* acc = (long long*)(smem + (((size_t)4 * n * c + 15) & ~(size_t)15));  // [n][c]
    float* emb = u.emb + (size_t)l * n * c;
    for (int e = t; e < n * c; e += kUmapT) {
        E[e] = emb[e];
        acc[e] = 0;
    }
    const uint32_t ne = min((uint64_t)u.nedge[l], u.ecap);
    const size_t o = (size_t)l * u.ecap;
    const double negr = (double)neg_rate;
    for (uint32_t e = t; e < ne; e += kUmapT) u.nxn[o + e] = u.eps[o + e] / negr;  // epochs_per_negative_sample
    __syncthreads();
    auto add = [&](int p, int d, double v) {
        __hip_atomic_fetch_add((TDA_LDS long long*)&acc[p * c + d], (long long)llrint(v * kUmapFix), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    for (int ep = 0; ep < u.n_epochs; ++ep) {
        const double alpha = lr * (1.0 - (double)ep / (double)u.n_epochs);
        for (uint32_t e = t; e < ne; e += kUmapT) {
            double nx = u.nxt[o + e];
            if (nx > (double)ep) continue;
            const double eps = u.eps[o + e], epsn = eps / negr;
            const int j = u.head[o + e], k = u.tail[o + e];
            float cur[kUmapMaxC];
            double d2 = 0.0;
            for (int d = 0; d < c; ++d) {
                cur[d] = E[j * c + d];
                const double df = (double)cur[d] - (double)E[k * c + d];
                d2 += df * df;
            }
            const float d2f = (float)d2;  // rdist in f32
            double gc = 0.0;
            if (d2f > 0.0f) {
                gc = -2.0 * a * b * pow((double)d2f, b - 1.0);
                gc /= a * pow((double)d2f, b) + 1.0;
            }
            for (int d = 0; d < c; ++d) {
                const double gd = umap_clip(gc * ((double)cur[d] - (double)E[k * c + d]));
                add(j, d, gd * alpha);
                add(k, d, -gd * alpha);  // move_other (fit: head and tail embeddings are one)
            }
            u.nxt[o + e] = nx + eps;
            double nn = u.nxn[o + e];
            const int nneg = (int)(((double)ep - nn) / epsn);
            for (int p = 0; p < nneg; ++p) {
                const int q = (int)(umap_hash(seed, ((uint64_t)ep << 32) ^ ((uint64_t)e << 8) ^ (uint64_t)p) % (uint64_t)n);
                double r2 = 0.0;
                for (int d = 0; d < c; ++d) {
                    const double df = (double)cur[d] - (double)E[q * c + d];
                    r2 += df * df;
                }
                const float r2f = (float)r2;
                double g2;
                if (r2f > 0.0f) {
                    g2 = 2.0 * gamma * b;
                    g2 /= (0.001 + (double)r2f) * (a * pow((double)r2f, b) + 1.0);
                } else if (j == q) {
                    continue;
                } else {
                    g2 = 0.0;
                }
                for (int d = 0; d < c; ++d) {
                    const double gd = g2 > 0.0 ? umap_clip(g2 * ((double)cur[d] - (double)E[q * c + d])) : 4.0;
                    add(j, d, gd * alpha);
                }
            }
            u.nxn[o + e] = nn + (double)nneg * epsn;
        }
        __syncthreads();
        for (int e = t; e < n * c; e += kUmapT) {
            E[e] = (float)((double)E[e] + (double)acc[e] * (1.0 / kUmapFix));
            acc[e] = 0;
        }
        __syncthreads();
    }
    for (int e = t; e < n * c; e += kUmapT) emb[e] = E[e];
}

// ---------------------------------------------------------------- transform
// [train; new] -> one layer's M x c transform embedding, one workgroup per
// layer (umap-learn UMAP.transform, small-data regime).  u.kd / u.ki hold the
// M new points' n_neighbors nearest training points (k_umap_knn with qrow0 =
// N); `temb` is the fitted N x c embedding; `vals` [L][M * k] the bipartite
// memberships.  Edges are the (point, neighbour) slots in row-major kNN
// order (umap's coo graph after eliminate_zeros); a dropped or pruned slot
// has epochs_per_sample -1.
__global__ __launch_bounds__(kUmapT) void k_umap_transform(UmapBufs u, const float* __restrict__ temb, int N, float* __restrict__ vals,
                                                           double a, double b, double lr, double gamma, int neg_rate, uint64_t seed,
                                                           float disc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ double red[kUmapT / 64];
    __shared__ uint32_t vmax_sh;
    const int l = blockIdx.x, M = u.nq, k = u.k, c = u.c, t = threadIdx.x;
    float* E = (float*)smem;                                                          // [M][c] new points
    long long* acc = (long long*)(smem + (((size_t)4 * M * c + 15) & ~(size_t)15));  // [M][c] epoch move sums
    float* T = (float*)(acc + (size_t)M * c);                                         // [N][c] training embedding (fixed)
    const float* kd = u.kd + (size_t)l * M * k;
    const int32_t* ki = u.ki + (size_t)l * M * k;
    float* V = vals + (size_t)l * M * k;
    const size_t o = (size_t)l * u.ecap;
    for (int e = t; e < N * c; e += kUmapT) T[e] = temb[e];
    for (int e = t; e < M * c; e += kUmapT) acc[e] = 0;
    if (t == 0) vmax_sh = 0;
    // smooth_knn_dist(dists, k, local_connectivity = max(0, 1 - 1) = 0): rho = 0;
    // mean_distances over every transform distance (dropped neighbours included, as umap)
    double s = 0.0;
    for (int e = t; e < M * k; e += kUmapT) s += (double)kd[e];
    const double mean_all = umap_block_sum(s, red) / (double)(M * k);
    const double target = log2((double)k);
    uint32_t vmax = 0;
    for (int i = t; i < M; i += kUmapT) {
        const float* d = kd + (size_t)i * k;
        double lo = 0.0, hi = INFINITY, mid = 1.0;
        for (int it = 0; it < 64; ++it) {
            double psum = 0.0;
            for (int j = 1; j < k; ++j) {  // umap skips slot 0 (the fit's self neighbour) here too
                const double dd = (double)d[j];
                psum += dd > 0.0 ? exp(-(dd / mid)) : 1.0;
            }
            if (fabs(psum - target) < 1e-5) break;
            if (psum > target) {
                hi = mid;
                mid = (lo + hi) / 2.0;
            } else {
                lo = mid;
                mid = isinf(hi) ? mid * 2.0 : (lo + hi) / 2.0;
            }
        }
        double sigma = mid;
        if (sigma < 1e-3 * mean_all) sigma = 1e-3 * mean_all;  // rho == 0 branch (MIN_K_DIST_SCALE)
        // compute_membership_strengths(bipartite=True); index -1 (d >= disconnection) -> no entry
        for (int j = 0; j < k; ++j) {
            float val;
            if (!(d[j] < disc))
                val = 0.0f;
            else if ((double)d[j] <= 0.0 || sigma == 0.0)
                val = 1.0f;
            else
                val = (float)exp(-((double)d[j] / sigma));
            V[(size_t)i * k + j] = val;
            vmax = max(vmax, __float_as_uint(val));
        }
    }
    vmax = (uint32_t)wave_max_u64(vmax);
    if ((t & 63) == 0 && vmax) atomicMax(&vmax_sh, vmax);
    __syncthreads();
    // init_graph_transform on the unpruned graph (zeros eliminated): the
    // membership-weighted mean of the neighbours' embeddings in f32 -- or a
    // neighbour's own embedding when its membership is exactly 1 -- NaN without
    // neighbours.  umap-learn walks graph.tocsr() rows, whose entries are in
    // ascending column (training index) order: the row sum, the weighted sum
    // and which membership-1 entry wins all follow that order (the k neighbour
    // slots are visited by ascending index, O(k^2) selection: k <= 64)
    auto next_col = [&](int i, int prev) -> int {  // slot of the smallest training index > prev, -1 if none
        int best = 0x7FFFFFFF, bj = -1;
        for (int j = 0; j < k; ++j) {
            const int col = ki[(size_t)i * k + j];
            if (col > prev && col < best) best = col, bj = j;
        }
        return bj;
    };
    for (int i = t; i < M; i += kUmapT) {
        float rs = 0.0f;
        int nnz = 0;
        for (int j = next_col(i, -1); j >= 0; j = next_col(i, ki[(size_t)i * k + j])) {
            const float v = V[(size_t)i * k + j];
            if (v != 0.0f) rs += v, ++nnz;
        }
        float r[kUmapMaxC];
        for (int dd = 0; dd < c; ++dd) r[dd] = nnz ? 0.0f : __builtin_nanf("");
        for (int j = nnz ? next_col(i, -1) : -1; j >= 0; j = next_col(i, ki[(size_t)i * k + j])) {
            const float v = V[(size_t)i * k + j];
            if (v == 0.0f) continue;
            const int col = ki[(size_t)i * k + j];
            if (v == 1.0f) {
                for (int dd = 0; dd < c; ++dd) r[dd] = T[col * c + dd];
                break;
            }
            const float wgt = __fdiv_rn(v, rs);
            for (int dd = 0; dd < c; ++dd) r[dd] = __fadd_rn(r[dd], __fmul_rn(wgt, T[col * c + dd]));
        }
        for (int dd = 0; dd < c; ++dd) E[i * c + dd] = r[dd];
    }
    // prune below max / n_epochs, make_epochs_per_sample on the survivors
    const float vm = __uint_as_float(vmax_sh);
    const double thr = (double)vm / (double)u.n_epochs, negr = (double)neg_rate;
    for (int e = t; e < M * k; e += kUmapT) {
        const float w = V[e];
        double eps = -1.0;
        if (w != 0.0f && !((double)w < thr)) {
            const float ns = __fmul_rn((float)u.n_epochs, __fdiv_rn(w, vm));
            if (ns > 0.0f) eps = (double)u.n_epochs / (double)ns;
        }
        u.eps[o + e] = eps;
        u.nxt[o + e] = eps;
        u.nxn[o + e] = eps / negr;
    }
    __syncthreads();
    auto add = [&](int p, int dd, double v) {
        __hip_atomic_fetch_add((TDA_LDS long long*)&acc[p * c + dd], (long long)llrint(v * kUmapFix), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    // optimize_layout_euclidean(move_other=False): the new points move, the training embedding stays
    for (int ep = 0; ep < u.n_epochs; ++ep) {
        const double alpha = lr * (1.0 - (double)ep / (double)u.n_epochs);
        for (int e = t; e < M * k; e += kUmapT) {
            const double eps = u.eps[o + e];
            if (eps < 0.0) continue;
            const double nx = u.nxt[o + e];
            if (nx > (double)ep) continue;
            const double epsn = eps / negr;
            const int j = e / k, kk = ki[e];
            float cur[kUmapMaxC];
            double d2 = 0.0;
            for (int dd = 0; dd < c; ++dd) {
                cur[dd] = E[j * c + dd];
                const double df = (double)cur[dd] - (double)T[kk * c + dd];
                d2 += df * df;
            }
            const float d2f = (float)d2;
            double gc = 0.0;
            if (d2f > 0.0f) {
                gc = -2.0 * a * b * pow((double)d2f, b - 1.0);
                gc /= a * pow((double)d2f, b) + 1.0;
            }
            for (int dd = 0; dd < c; ++dd) add(j, dd, umap_clip(gc * ((double)cur[dd] - (double)T[kk * c + dd])) * alpha);
            u.nxt[o + e] = nx + eps;
            const double nn = u.nxn[o + e];
            const int nneg = (int)(((double)ep - nn) / epsn);
            for (int p = 0; p < nneg; ++p) {
                const int q = (int)(umap_hash(seed, ((uint64_t)ep << 32) ^ ((uint64_t)e << 8) ^ (uint64_t)p) % (uint64_t)N);
                double r2 = 0.0;
                for (int dd = 0; dd < c; ++dd) {
                    const double df = (double)cur[dd] - (double)T[q * c + dd];
                    r2 += df * df;
                }
                const float r2f = (float)r2;
                double g2;
                if (r2f > 0.0f) {
                    g2 = 2.0 * gamma * b;
                    g2 /= (0.001 + (double)r2f) * (a * pow((double)r2f, b) + 1.0);
                } else if (j == q) {  // umap compares the head index with the sample's (different sets here, as there)
                    continue;
                } else {
                    g2 = 0.0;
                }
                for (int dd = 0; dd < c; ++dd) {
                    const double gd = g2 > 0.0 ? umap_clip(g2 * ((double)cur[dd] - (double)T[q * c + dd])) : 4.0;
                    add(j, dd, gd * alpha);
                }
            }
            u.nxn[o + e] = nn + (double)nneg * epsn;
        }
        __syncthreads();
        for (int e = t; e < M * c; e += kUmapT) {
            E[e] = (float)((double)E[e] + (double)acc[e] * (1.0 / kUmapFix));
            acc[e] = 0;
        }
        __syncthreads();
    }
    float* emb = u.emb + (size_t)l * M * c;
    for (int e = t; e < M * c; e += kUmapT) emb[e] = E[e];
}

// [x_train; y_l] per layer (the transform's distance input), 4-byte words
__global__ __launch_bounds__(256) void k_umap_concat(const uint32_t* __restrict__ xt, const uint32_t* __restrict__ y, uint32_t* __restrict__ z,
                                                     uint64_t train_words, uint64_t layer_words) {
    const int l = blockIdx.y;
    uint32_t* zl = z + (size_t)l * (train_words + layer_words);
    const uint32_t* yl = y + (size_t)l * layer_words;
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < train_words + layer_words; e += (uint64_t)gridDim.x * blockDim.x)
        zl[e] = e < train_words ? xt[e] : yl[e - train_words];
}

}  // namespace tda
