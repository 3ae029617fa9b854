// ed_kernels.h -- normalised effective dimensionality of activation batches
// on gfx950: the reference's compute_effective_dimensionality
// (metrics.py:5-44): S = svdvals(X) for every (n_samples, embed_dim) item,
// ED = (sum S)^2 / max(sum S^2, 1e-10) / max(min(n, d), 1).
//
// MI355X formulation: the squared singular values are the eigenvalues of the
// m x m Gram matrix, m = min(n, d) -- X X^T (n <= d: the FP64 MFMA Gram tiles
// of k_distance_mfma<T, 2>, or k_gram_rows below D = 32) or X^T X (n > d:
// k_gram_cols) -- accumulated in f64 from the f32/f64 inputs (products of f32
// values are exact in f64).  k_ed_jacobi diagonalises each Gram matrix with
// the parallel cyclic Jacobi method (one workgroup per item, round-robin pair
// schedule: m/2 disjoint rotations per step, applied as independent 2 x 2
// blocks J_i^T A J_j), in LDS up to m = kEdLdsMaxM and in an HBM scratch
// above, until the off-diagonal mass is below 1e-30 of the diagonal's.
#pragma once
#include "rips_device.h"

namespace tda {

constexpr int kEdT = 1024;
constexpr int kEdLdsMaxM = 128;  // m x m f64 in LDS (128 KB)
constexpr int kEdMaxM = 1024;    // the HBM path's bound (pairs and rotations live in LDS)

// G[l] = X_l X_l^T (n x n, f64) for small D: thread per (i, j >= i), sequential k
template <typename T>
__global__ __launch_bounds__(256) void k_gram_rows(const T* __restrict__ X, int n, int d, double* __restrict__ G) {
    const int l = blockIdx.y;
    const T* Xl = X + (size_t)l * n * d;
    double* Gl = G + (size_t)l * n * n;
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < (size_t)n * n; q += (size_t)gridDim.x * blockDim.x) {
        const int i = (int)(q / n), j = (int)(q - (size_t)i * n);
        if (j < i) continue;
        double s = 0.0;
        for (int k = 0; k < d; ++k) s = fma((double)Xl[(size_t)i * d + k], (double)Xl[(size_t)j * d + k], s);
        Gl[(size_t)i * n + j] = s;
        Gl[(size_t)j * n + i] = s;
    }
}

// G[l] = X_l^T X_l (d x d, f64) when n > d: thread per (a, b >= a), sequential over the samples
template <typename T>
__global__ __launch_bounds__(256) void k_gram_cols(const T* __restrict__ X, int n, int d, double* __restrict__ G) {
    const int l = blockIdx.y;
    const T* Xl = X + (size_t)l * n * d;
    double* Gl = G + (size_t)l * d * d;
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < (size_t)d * d; q += (size_t)gridDim.x * blockDim.x) {
        const int a = (int)(q / d), b = (int)(q - (size_t)a * d);
        if (b < a) continue;
        double s = 0.0;
        for (int i = 0; i < n; ++i) s = fma((double)Xl[(size_t)i * d + a], (double)Xl[(size_t)i * d + b], s);
        Gl[(size_t)a * d + b] = s;
        Gl[(size_t)b * d + a] = s;
    }
}

// round-robin schedule: step s of a sweep over M (even) indices pairs index 0
// with 1 + s mod (M - 1) and, for k = 1 .. M/2 - 1, 1 + (s + k) mod (M - 1)
// with 1 + (s - k) mod (M - 1): every pair exactly once per M - 1 steps
__device__ __forceinline__ void ed_pair(int s, int k, int M, int* p, int* q) {
    const int r = M - 1;
    int a, b;
    if (k == 0) {
        a = 0;
        b = 1 + s % r;
    } else {
        a = 1 + (s + k) % r;
        b = 1 + ((s - k) % r + r) % r;
    }
    *p = a < b ? a : b;
    *q = a < b ? b : a;
}

// one workgroup per item: Jacobi eigenvalues of the m x m Gram matrix Gin[l]
// (LDS: copied into dynamic LDS; else updated in place), then the normalised
// participation ratio of the singular values sqrt(max(lambda, 0)) -> out[l]
template <bool LDS>
__global__ __launch_bounds__(kEdT) void k_ed_jacobi(double* __restrict__ Gin, int m, int min_dim, float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ double cs[kEdMaxM / 2], sn[kEdMaxM / 2];
    __shared__ int pp[kEdMaxM / 2], qq[kEdMaxM / 2];
    __shared__ double red[kEdT / 64];
    const int l = blockIdx.x, t = threadIdx.x;
    double* A = LDS ? (double*)smem : Gin + (size_t)l * m * m;
    if (LDS) {
        const double* src = Gin + (size_t)l * m * m;
        for (int e = t; e < m * m; e += kEdT) A[e] = src[e];
    }
    auto block_sum = [&](double v) {
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        __syncthreads();
        if ((t & 63) == 0) red[t >> 6] = v;
        __syncthreads();
        double s = 0.0;
        for (int w = 0; w < kEdT / 64; ++w) s += red[w];
        return s;
    };
    const int M = (m + 1) & ~1, H = M / 2;  // odd m: index m is a dummy (identity rotations)
    __syncthreads();
    for (int sweep = 0; sweep < 60 && m > 1; ++sweep) {
        double off = 0.0, dia = 0.0;
        for (int e = t; e < m * m; e += kEdT) {
            const double v = mld<LDS>(A, e);
            const int i = e / m, j = e - (e / m) * m;
            if (i == j) dia += v * v;
            else off += v * v;
        }
        off = block_sum(off);
        dia = block_sum(dia);
        if (!(off > 1e-30 * dia)) break;
        for (int s = 0; s < M - 1; ++s) {
            for (int k = t; k < H; k += kEdT) {  // rotation of pair k (NR jacobi: theta, t, c, s)
                int p, q;
                ed_pair(s, k, M, &p, &q);
                double c = 1.0, sv = 0.0;
                if (q < m) {
                    const double apq = mld<LDS>(A, (size_t)p * m + q);
                    if (apq != 0.0) {
                        const double app = mld<LDS>(A, (size_t)p * m + p), aqq = mld<LDS>(A, (size_t)q * m + q);
                        const double th = (aqq - app) / (2.0 * apq);
                        const double tt = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
                        c = 1.0 / sqrt(tt * tt + 1.0);
                        sv = tt * c;
                    }
                }
                cs[k] = c;
                sn[k] = sv;
                pp[k] = p;
                qq[k] = q;
            }
            __syncthreads();
            // A <- J^T A J as independent 2 x 2 blocks (rows of pair ki) x (columns of pair kj), kj >= ki
            const int nb = H * (H + 1) / 2;
            for (int e = t; e < nb; e += kEdT) {
                int ki = 0, rem = e;
                while (rem >= H - ki) rem -= H - ki, ++ki;
                const int kj = ki + rem;
                const int p = pp[ki], q = qq[ki], p2 = pp[kj], q2 = qq[kj];
                const double ci = cs[ki], si = sn[ki], cj = cs[kj], sj = sn[kj];
                const bool qv = q < m, q2v = q2 < m;
                const double x00 = mld<LDS>(A, (size_t)p * m + p2), x01 = q2v ? mld<LDS>(A, (size_t)p * m + q2) : 0.0;
                const double x10 = qv ? mld<LDS>(A, (size_t)q * m + p2) : 0.0, x11 = (qv && q2v) ? mld<LDS>(A, (size_t)q * m + q2) : 0.0;
                // columns (pair kj), then rows (pair ki)
                const double y00 = cj * x00 - sj * x01, y01 = sj * x00 + cj * x01;
                const double y10 = cj * x10 - sj * x11, y11 = sj * x10 + cj * x11;
                double z00 = ci * y00 - si * y10, z01 = ci * y01 - si * y11;
                const double z10 = si * y00 + ci * y10;
                double z11 = si * y01 + ci * y11;
                double z10w = z10;
                if (ki == kj) z01 = z10w = 0.0;  // the pair's own off-diagonal entry is annihilated
                mst<LDS>(A, (size_t)p * m + p2, z00);
                if (q2v) mst<LDS>(A, (size_t)p * m + q2, z01);
                if (qv) mst<LDS>(A, (size_t)q * m + p2, z10w);
                if (qv && q2v) mst<LDS>(A, (size_t)q * m + q2, z11);
                if (ki != kj) {  // the symmetric block
                    mst<LDS>(A, (size_t)p2 * m + p, z00);
                    if (qv) mst<LDS>(A, (size_t)p2 * m + q, z10);
                    if (q2v) mst<LDS>(A, (size_t)q2 * m + p, z01);
                    if (qv && q2v) mst<LDS>(A, (size_t)q2 * m + q, z11);
                }
            }
            __syncthreads();
        }
    }
    double s1 = 0.0, s2 = 0.0;
    for (int i = t; i < m; i += kEdT) {
        const double lam = fmax(mld<LDS>(A, (size_t)i * m + i), 0.0);
        s1 += sqrt(lam);
        s2 += lam;
    }
    s1 = block_sum(s1);
    s2 = block_sum(s2);
    if (t == 0) {
        const double pr = (s1 * s1) / fmax(s2, 1e-10);
        out[l] = (float)(pr / fmax((double)min_dim, 1.0));
    }
}

}  // namespace tda
