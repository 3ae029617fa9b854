/*
 * tda_umap.h -- C ABI of the MI355X UMAP embedding (same library as
 * tda_rips.h: libtda_rips.so).
 *
 * Replaces the step right before the hot path in the reference's layer loop:
 *     reducer = umap.UMAP(n_neighbors=6, n_components=3, min_dist=0.1,
 *                         random_state=42, metric='cosine')
 *     cloud_low_dim = reducer.fit_transform(cloud_high_dim)
 * (debug_tda_pipeline.py:96-104; analyze_tda_over_layers.py:38-44, :67-72),
 * for L layers at once.  umap-learn is a third-party package (unpinned,
 * absent from the reference and this image); the kernels restate its
 * published algorithm in the small-data regime (exact pairwise distances,
 * N < 4096): kNN -> smooth_knn_dist -> fuzzy union -> spectral layout ->
 * negative-sampling SGD.  a, b are umap's find_ab_params(spread, min_dist)
 * (the Python binding fits them as umap does).  SGD epochs are synchronous
 * and the result is deterministic for a seed (see csrc/umap_kernels.h).
 * Returns 0 or a negative TDA_E* code (tda_last_error()).
 */
#ifndef TDA_UMAP_H
#define TDA_UMAP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TDA_UMAP_EUCLIDEAN 0
#define TDA_UMAP_COSINE 1
#define TDA_UMAP_INIT_SPECTRAL 0
#define TDA_UMAP_INIT_RANDOM 1

typedef struct tda_umap_args {
    const void *x;          /* (L, N, D) row-major points, host or device           */
    int32_t dtype;          /* TDA_F32 | TDA_F64                                    */
    int32_t x_on_device;    /* 1: x is a device pointer on `device`                 */
    int64_t L, N, D;
    int32_t metric;         /* TDA_UMAP_EUCLIDEAN | TDA_UMAP_COSINE                 */
    int32_t n_neighbors;    /* 2 .. min(64, N)                                      */
    int32_t n_components;   /* 1 .. 8                                               */
    int32_t n_epochs;       /* >= 1 (umap default: 500 for N <= 10000)               */
    int32_t init;           /* TDA_UMAP_INIT_SPECTRAL | TDA_UMAP_INIT_RANDOM         */
    int32_t negative_sample_rate;
    float a, b;             /* curve parameters (find_ab_params)                    */
    float learning_rate, repulsion_strength;
    uint64_t seed;          /* random_state                                         */
    int32_t device;
    float *out;             /* host (L, N, n_components) f32: the embedding          */
    float *graph_out;       /* optional host (L, N, N) f32: the pruned fuzzy graph   */
    void *stream;           /* device inputs are read after the work queued on this
                               hipStream_t so far (e.g. torch's current stream);
                               NULL = the null (legacy default) stream            */
} tda_umap_args;

int tda_umap_batch(const tda_umap_args *args);

/*
 * UMAP.transform of a fitted model, for L batches of new points at once:
 * replaces `reducer.transform(cloud_high_dim)` in the reference's second
 * driver, which fits one reducer on layer 31 and transforms every layer with
 * it (analyze_tda_over_layers.py:38-44, :67-72).  umap-learn's transform in
 * the small-data regime: exact distances to the training points, the
 * n_neighbors nearest (ties: smaller index), smooth_knn_dist with
 * local_connectivity - 1 = 0, bipartite memberships (neighbours at or beyond
 * the metric's disconnection distance dropped), the weighted-mean
 * initialisation (init_graph_transform), pruning below max / n_epochs, and
 * n_epochs of SGD in which only the new points move (move_other = False),
 * attracted to and repelled from the fixed training embedding, at
 * learning_rate (umap passes its initial alpha / 4).  Same epoch-synchronous
 * deterministic SGD as tda_umap_batch.  Returns 0 or a negative TDA_E* code.
 */
typedef struct tda_umap_transform_args {
    const void *x_train;      /* (N, D) row-major points the model was fitted on   */
    const float *emb_train;   /* host (N, n_components) f32: the fitted embedding  */
    const void *y;            /* (L, M, D) row-major new points                    */
    int32_t dtype;            /* TDA_F32 | TDA_F64 (x_train and y)                 */
    int32_t x_on_device;      /* 1: x_train and y are device pointers on `device`  */
    int64_t L, M, N, D;
    int32_t metric;           /* TDA_UMAP_EUCLIDEAN | TDA_UMAP_COSINE              */
    int32_t n_neighbors;      /* the fitted model's, 2 .. min(64, N)                */
    int32_t n_components;     /* 1 .. 8                                            */
    int32_t n_epochs;         /* umap: 100 (M <= 10000) or the fit's n_epochs // 3  */
    int32_t negative_sample_rate;
    float a, b;               /* the fitted curve parameters                       */
    float learning_rate;      /* initial alpha (umap: fit learning_rate / 4)       */
    float repulsion_strength;
    float disconnection;      /* neighbours at >= this distance are dropped (inf: none) */
    uint64_t seed;
    int32_t device;
    float *out;               /* host (L, M, n_components) f32                     */
    void *stream;             /* hipStream_t (or NULL), as in tda_umap_args        */
} tda_umap_transform_args;

int tda_umap_transform(const tda_umap_transform_args *args);

#ifdef __cplusplus
}
#endif

#endif /* TDA_UMAP_H */
