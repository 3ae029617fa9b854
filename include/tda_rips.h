/*
 * tda_rips.h -- C ABI of the MI355X (gfx950) Vietoris-Rips persistence engine.
 *
 * Drop-in boundary for the reference's hot path: the third-party call
 *     result = ripser(cloud_low_dim, maxdim=MAX_DIM); dgms = result['dgms']
 * at debug_tda_pipeline.py:109-110, analyze_tda_over_layers.py:76 and
 * experiments/adversarial_compositional_binding/analyze_adversarial_tda.py:100.
 * The reference binds ripser's C++ core through Cython (package `ripser`,
 * unpinned, README.md:28; not vendored in the reference) with two entry points,
 *     rips_dm(float* D, int N, int modulus, int dim_max, float threshold,
 *             int do_cocycles)                                   [upstream]
 *     rips_dm_sparse(int* I, int* J, float* V, int NEdges, int N, int modulus,
 *             int dim_max, float threshold, int do_cocycles)     [upstream]
 * returning {births_and_deaths_by_dim, cocycles_by_dim, num_edges}.
 * `tda_rips_dm` below replaces `rips_dm` one-for-one (same argument meaning:
 * D is the condensed strict-upper-triangle distance vector in row-major (i<j)
 * order, exactly what ripser.py passes after `dm[I > J]`).  `tda_rips_batch`
 * is the layer-loop entry (point clouds in, distance + persistence on the
 * GPU) that the reference's per-layer loop (debug_tda_pipeline.py:92-150)
 * calls once per sweep instead of once per layer.
 *
 * Conventions
 *  - All functions return 0 on success or a negative TDA_E* code; the message
 *    is kept in thread-local storage and returned by tda_last_error().
 *  - Inputs are never owned by the library.  Results are library-owned until
 *    tda_rips_free().
 *  - coeff/modulus must be 2 (the reference never overrides ripser's default);
 *    other values return TDA_E_UNSUPPORTED.  do_cocycles != 0 likewise.
 *  - No torch types cross this boundary: plain pointers and sizes.
 */
#ifndef TDA_RIPS_H
#define TDA_RIPS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TDA_RIPS_ABI_VERSION 8

/* error codes */
#define TDA_OK 0
#define TDA_E_INVALID (-1)      /* bad shape / argument / non-finite input   */
#define TDA_E_UNSUPPORTED (-2)  /* coeff != 2, cocycles, maxdim > 2, ...     */
#define TDA_E_HIP (-3)          /* HIP runtime error (message has details)   */
#define TDA_E_CAPACITY (-4)     /* a device work buffer overflowed           */
#define TDA_E_NODEVICE (-5)     /* no gfx950 device visible                  */

/* dtype of the point-cloud input */
#define TDA_F32 0
#define TDA_F64 1

/* arguments of one batched call: L layers of N points in R^D */
typedef struct tda_rips_args {
    const void *x;      /* (L, N, D) row-major points, or (L, N, N) distances   */
    int32_t dtype;      /* TDA_F32 | TDA_F64                                    */
    int32_t x_on_device;/* 1: x is a device pointer on `device`; 0: host memory */
    int64_t L, N, D;    /* D ignored when is_dist                               */
    int32_t is_dist;    /* 1: x holds (L, N, N) distance matrices (upper used)  */
    int32_t maxdim;     /* 0, 1 or 2                                            */
    float thresh;       /* +inf -> enclosing radius (ripser.py default)         */
    int32_t modulus;    /* must be 2                                            */
    int32_t device;     /* HIP device ordinal                                   */
    void *stream;       /* device input (x_on_device) is read after the work queued
                           on this hipStream_t so far; NULL = the null (legacy
                           default) stream, which is torch's default stream.  ABI 7:
                           before, NULL meant no ordering.  A handle that is not a
                           stream of the library's HIP runtime on `device` is
                           refused (TDA_E_HIP).  Ignored with TDA_FLAG_INPUT_READY
                           and for host input.                                   */
    int32_t want_dist;  /* 1: also return the (L, N, N) f32 distance matrices   */
    int32_t flags;      /* TDA_FLAG_* bits (0 = none)                           */
    /* optional silhouette scores on the same distance matrices (ABI >= 2):
     * sklearn.metrics.silhouette_score(cloud, labels), called by the reference
     * beside ripser at debug_tda_pipeline.py:117-118 (shape / color labels) and
     * analyze_adversarial_tda.py:108-111.  `labels` is host memory [n_label_sets][N]
     * of LabelEncoder codes 0..K-1 (every code present, 2 <= K <= min(N-1, 32)),
     * shared by all L layers.  NULL / 0 = none. */
    const int32_t *labels;
    int32_t n_label_sets;
    /* optional TwoNN intrinsic dimension per layer on the same distance
     * matrices (ABI >= 3): the reference's compute_intrinsic_dimensionality
     * (metrics.py:113-208: two nearest neighbours per point, mu = r2/r1,
     * discard the largest `twonn_discard` fraction, slope of -log(1-F) on
     * log(mu) through the origin).  0 = off. */
    int32_t want_twonn;
    float twonn_eps;       /* eps (reference default 1e-10; compared in f32)   */
    double twonn_discard;  /* discard_fraction (reference default 0.1; f64 as
                              in int(len * (1.0 - discard_fraction)))          */
    /* ABI >= 5: workspace slot 0 .. TDA_MAX_SLOTS-1 on `device`.  Each slot has
     * its own streams, device buffers, host-mapped outputs and captured
     * graphs, so calls on different slots (from different host threads) run
     * concurrently on the GPU -- e.g. consecutive sweeps of a layer loop in
     * flight at once; calls on one slot are serialised. */
    int32_t slot;
    /* ABI >= 6: input in parts (dynamic batching of consecutive sweeps).  When
     * n_parts > 0, x is ignored and the L layers are the concatenation of the
     * n_parts arrays x_parts[0 .. n_parts-1], each (L / n_parts, N, D) (or
     * (L / n_parts, N, N) with is_dist), all in host memory or all on `device`
     * as x_on_device says.  The library gathers them into its own buffer (one
     * copy kernel on its stream, after the caller's stream), so the captured
     * graph reads one stable address whatever the parts' addresses are. */
    const void *const *x_parts;
    int32_t n_parts;
} tda_rips_args;

#define TDA_MAX_SLOTS 8
#define TDA_MAX_PARTS 16

/* per (layer, dim) emitted persistence pairs, in the reference's emission
 * order: H0 = Kruskal order of the finite deaths then one [0, inf) per
 * component; Hk = columns in (birth desc, birth-simplex index asc) order.
 * birth_idx/death_idx are combinatorial-number-system simplex indices
 * (H0: birth vertex, death edge; essential classes: death_idx = -1). */
typedef struct tda_rips_result {
    int64_t L, maxdim, N;
    const int64_t *count;     /* [L][maxdim+1] pairs per layer and dim          */
    const int64_t *offset;    /* [L][maxdim+1] offset into the pair arrays      */
    const float *birth;       /* [total] */
    const float *death;       /* [total] (+inf for essential)                   */
    const int64_t *birth_idx; /* [total] */
    const int64_t *death_idx; /* [total] */
    const float *thresh;      /* [L] threshold actually used (enclosing radius) */
    const int64_t *num_edges; /* [L] condensed distances <= thresh              */
    const uint64_t *checksum; /* [L][maxdim+1] order-free hash of ALL pairs     */
    const int64_t *n_all_pairs;/* [L][maxdim+1] all pairs incl. zero-persistence*/
    const int64_t *n_columns; /* [L][maxdim+1] columns considered per dim       */
    const int64_t *n_residual;/* [L][maxdim+1] columns needing reduction        */
    const int64_t *n_adds;    /* [L][maxdim+1] column additions (serial part)   */
    const float *dist;        /* [L][N][N] when want_dist, else NULL            */
    /* Layout guarantee (lets a binding copy them in three reads): count,
     * offset, checksum, n_all_pairs, n_columns, n_residual and n_adds are
     * consecutive [L][maxdim+1] blocks of one allocation, in that order
     * (count + k * L * (maxdim+1) is the k-th); death = birth + total and
     * death_idx = birth_idx + total. */
    double device_ms;         /* device time of the call (HIP events)           */
    /* per-stage device times, filled when args.flags & TDA_FLAG_STAGE_TIMES:
     * stage_ms[i] is the time between consecutive stream events bracketing
     * stage i (one kernel, memset or copy), named by stage_name[i]. */
    int32_t n_stages;
    const char *const *stage_name;
    const float *stage_ms;
    /* [L][n_label_sets] silhouette scores when args.labels was given, else NULL */
    const double *silhouette;
    /* [L] TwoNN intrinsic dimension when args.want_twonn (NaN where the
     * reference returns NaN), else NULL (ABI >= 3) */
    const float *twonn;
    /* ABI >= 3: count .. n_adds, num_edges, birth_idx / death_idx, thresh
     * (padded to 8 bytes) and birth / death, in this order, are ONE
     * allocation of blob_bytes bytes starting at blob (8-byte aligned
     * blocks), so a binding copies every per-pair array in one read;
     * n_pairs = total pairs over all layers and dims. */
    const void *blob;
    int64_t blob_bytes;
    int64_t n_pairs;
    /* ABI >= 4: [L][N][N] float64 distances (sqrt in f64 before any rounding:
     * what sklearn's pairwise_distances returns for float64 points and
     * ripser.py hands back as dperm2all) when args.flags & TDA_FLAG_DIST64,
     * want_dist and float64 point clouds, else NULL */
    const double *dist64;
    /* ABI >= 8: layers of this call re-run without column caps.  With the
     * default threshold (enclosing radius) the parallel reducer stores only
     * the keys of a column up to birth + 0.5 * thresh; a column whose pivot
     * lies above that (a class living longer than half the radius) flags its
     * layer, and the library re-runs that layer alone, uncapped, and splices
     * it in.  Results are exact either way; this only reports the cost. */
    int64_t n_cap_reruns;
} tda_rips_result;

#define TDA_FLAG_STAGE_TIMES 1
/* with TDA_FLAG_STAGE_TIMES: run every stage on one stream so each stage time
 * is one kernel's duration (no overlap with, or queueing behind, the side
 * streams); for per-kernel measurement only */
#define TDA_FLAG_STAGE_SERIAL 2
/* with want_dist and float64 point clouds: also return result->dist64 */
#define TDA_FLAG_DIST64 4
/* distances and the side metrics asked for (want_twonn, labels) only: no
 * persistence at all (maxdim must be 0); every diagram is empty and thresh /
 * num_edges are 0.  What metrics.compute_intrinsic_dimensionality needs
 * (reference metrics.py:113-208 computes no persistence). */
#define TDA_FLAG_NO_PERSISTENCE 8
/* every kernel of the call on the slot's one stream (no side streams): the
 * call's own latency grows, but a slot that only runs such calls holds one
 * hardware queue, so several slots driven from their own host threads
 * (args.slot) run their batches side by side (ripser.SweepPipeline) */
#define TDA_FLAG_ONE_STREAM 16
/* ABI >= 7: device input is complete (the caller synchronised after producing
 * it): no ordering after args.stream at all */
#define TDA_FLAG_INPUT_READY 32

/* Batched point clouds (or distance matrices) -> persistence diagrams. */
int tda_rips_batch(const tda_rips_args *args, tda_rips_result **out);

/* One condensed distance vector (length N(N-1)/2, i<j row-major) -> diagrams.
 * Replaces ripser.py's rips_dm (see header comment). */
int tda_rips_dm(const float *D, int64_t n_entries, int32_t modulus, int32_t dim_max, float threshold,
                int32_t do_cocycles, tda_rips_result **out);

void tda_rips_free(tda_rips_result *r);
const char *tda_last_error(void);
int tda_version(void);
/* 1 if a gfx950 device is visible, 0 otherwise (never aborts). */
int tda_device_ok(int32_t device);

/*
 * Normalised effective dimensionality of B activation matrices (B, N, D):
 * replaces the reference's TorchScript compute_effective_dimensionality
 * (metrics.py:5-44): S = svdvals(X_b), ED_b = (sum S)^2 /
 * max(sum S^2, 1e-10) / max(min(N, D), 1), as float32 into out[B] (host).
 * The squared singular values are the eigenvalues of the f64 Gram matrix
 * (X X^T on the FP64 matrix cores when N <= D, X^T X otherwise), found by
 * parallel Jacobi on the GPU (csrc/ed_kernels.h).  min(N, D) <= 1024.
 */
typedef struct tda_ed_args {
    const void *x;          /* (B, N, D) row-major, host or device               */
    int32_t dtype;          /* TDA_F32 | TDA_F64                                 */
    int32_t x_on_device;    /* 1: x is a device pointer on `device`              */
    int64_t B, N, D;
    int32_t device;
    void *stream;           /* device input is read after it; NULL = null stream  */
} tda_ed_args;

int tda_effective_dim(const tda_ed_args *args, float *out);

#ifdef __cplusplus
}
#endif
#endif /* TDA_RIPS_H */
