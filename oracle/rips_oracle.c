/*
 * rips_oracle.c -- CPU ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity checker and the CPU baseline ("kind": "port") for the
 * MI355X hot path.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product path (tda-multimodal_amd) never
 * links, loads or calls anything under oracle/.
 *
 * What it restates (the reference's hot path is the third-party call
 * `ripser(cloud, maxdim)` at debug_tda_pipeline.py:109,
 * analyze_tda_over_layers.py:76, analyze_adversarial_tda.py:100; the package
 * is `ripser` (scikit-tda ripser.py, wrapping U. Bauer's Ripser C++), installed
 * unpinned by README.md:28 and absent from /root/reference and this image):
 *
 *   1. distance  : scikit-learn euclidean_distances for float32 input
 *                  (sklearn/metrics/pairwise.py:582-653 upcast path, :429 clamp,
 *                  :436 zero diagonal, :441 sqrt) -> f32 square matrix; only the
 *                  strict upper triangle is used (ripser.py condenses dm[I > J]).
 *   2. threshold : thresh = inf -> enclosing radius min_i max_j d(i,j)
 *                  (ripser.py rips_dm); num_edges = #{d <= thresh}.
 *   3. H0        : Kruskal over edges sorted by (diam asc, index desc), union
 *                  find, emit [0,d) for d > 0, then one [0,inf) per component.
 *   4. Hk, k>=1  : cohomology column reduction over Z/2 with clearing and the
 *                  emergent-pair shortcut; columns in (diam desc, index asc)
 *                  order; pivot = min cofacet by (diam asc, index desc); emit
 *                  (birth, death) iff death > birth, (birth, inf) for zero
 *                  columns.  Simplex indices use the combinatorial number
 *                  system (colex): idx{v_k>...>v_0} = sum_i C(v_i, i+1).
 *
 * The emission order (decreasing birth, ties by increasing column index) is
 * pinned by tests/golden/summary_stats.json (all_h1_persistence_values).
 *
 * Parity anchors: tests/golden/ (32 reference clouds + summary_stats.json from
 * /root/reference/tda-output, sklearn distance goldens, naive-reduction
 * goldens) -- see tests/golden/make_golden.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

#define OR_MAXDIM 3

typedef struct {
    float diam;
    uint64_t idx;
} splx_t;

/* ---------- result ---------------------------------------------------- */
typedef struct {
    int64_t n_pairs[OR_MAXDIM + 1];     /* emitted pairs per dim                */
    float *births[OR_MAXDIM + 1];
    float *deaths[OR_MAXDIM + 1];
    int64_t *birth_idx[OR_MAXDIM + 1];  /* column simplex index (H0: vertex)    */
    int64_t *death_idx[OR_MAXDIM + 1];  /* pivot simplex index, -1 = essential  */
    int64_t n_all_pairs[OR_MAXDIM + 1]; /* all pairs incl. zero persistence     */
    uint64_t checksum[OR_MAXDIM + 1];   /* order-free hash over all pairs       */
    int64_t n_columns[OR_MAXDIM + 1];   /* columns reduced per dim              */
    int64_t n_apparent[OR_MAXDIM + 1];  /* columns that are apparent pairs      */
    int64_t n_adds[OR_MAXDIM + 1];      /* column additions performed           */
    int64_t max_heap[OR_MAXDIM + 1];    /* largest working heap (entries)       */
    int64_t max_live[OR_MAXDIM + 1];    /* largest reduced column |R_j| (debug) */
    int64_t sum_live[OR_MAXDIM + 1];
    int64_t sum_heap_steps[OR_MAXDIM + 1]; /* sum over pivot steps of heap size */
    int64_t num_edges;
    float thresh;
} oracle_result;

/* ---------- small helpers ---------------------------------------------- */
typedef struct {
    int64_t n;
    int kmax;
    uint64_t *t; /* (kmax+1) x (n+2) */
} binom_t;

static void binom_init(binom_t *b, int64_t n, int kmax) {
    b->n = n;
    b->kmax = kmax;
    b->t = (uint64_t *)calloc((size_t)(kmax + 1) * (size_t)(n + 2), sizeof(uint64_t));
    for (int64_t i = 0; i <= n + 1; ++i) {
        b->t[0 * (n + 2) + i] = 1;
        for (int k = 1; k <= kmax; ++k) {
            if (i == 0)
                b->t[k * (n + 2) + i] = 0;
            else
                b->t[k * (n + 2) + i] = b->t[(k - 1) * (n + 2) + i - 1] + b->t[k * (n + 2) + i - 1];
        }
    }
}
static inline uint64_t C(const binom_t *b, int64_t n, int k) {
    if (k < 0 || n < k) return 0;
    return b->t[k * (b->n + 2) + n];
}

/* decode simplex index -> vertices (descending), dim+1 vertices */
static void decode(const binom_t *b, uint64_t idx, int dim, int64_t n, int64_t *v) {
    int64_t top = n - 1;
    for (int k = dim + 1; k >= 1; --k) {
        /* largest x <= top with C(x,k) <= idx */
        int64_t lo = k - 1, hi = top;
        while (lo < hi) {
            int64_t mid = (lo + hi + 1) >> 1;
            if (C(b, mid, k) <= idx)
                lo = mid;
            else
                hi = mid - 1;
        }
        v[dim + 1 - k] = lo;
        idx -= C(b, lo, k);
        top = lo - 1;
    }
}

static inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}
/* order-independent pair hash: shared definition with the HIP path
   (tda-multimodal_amd/csrc/rips.hip pair_hash) */
static inline uint64_t pair_hash(uint64_t s, uint64_t t) { return mix64(s * 0x9E3779B97F4A7C15ULL ^ mix64(t + 0x632BE59BD9B4E019ULL)); }

/* filtration-order comparator for qsort: column order = diam desc, idx asc */
static int cmp_col_order(const void *a, const void *b) {
    const splx_t *x = (const splx_t *)a, *y = (const splx_t *)b;
    if (x->diam > y->diam) return -1;
    if (x->diam < y->diam) return 1;
    return (x->idx < y->idx) ? -1 : (x->idx > y->idx);
}
/* Kruskal order = diam asc, idx desc */
static int cmp_filt_order(const void *a, const void *b) { return cmp_col_order(b, a); }

/* ---------- distances (sklearn restatement) ------------------------------ */
/* sklearn/metrics/pairwise.py:582-653 (_euclidean_distances_upcast): chunk
 * upcast to f64, d = (-2 x.y + |x|^2) + |y|^2, cast to f32 (:651), clamp at 0
 * (:429), zero diagonal (:436), f32 sqrt (:441).  The dot and the norms are
 * summed in increasing k (bit-identical to OpenBLAS/einsum for D <= 8,
 * verified in tests/golden/make_golden.py).  ripser.py reads dm[r,c] for
 * r < c, so pair (i<j) is always evaluated with i as the "X" row. */
void oracle_distances_f32(const float *X, int64_t n, int64_t D, float *out) {
    double *xx = (double *)malloc(sizeof(double) * (size_t)(n ? n : 1));
    for (int64_t i = 0; i < n; ++i) {
        double s = 0.0;
        for (int64_t k = 0; k < D; ++k) {
            double a = (double)X[i * D + k];
            s = fma(a, a, s);
        }
        xx[i] = s;
    }
    for (int64_t i = 0; i < n; ++i) {
        out[i * n + i] = 0.0f;
        for (int64_t j = i + 1; j < n; ++j) {
            double dot = 0.0;
            for (int64_t k = 0; k < D; ++k) dot = fma((double)X[i * D + k], (double)X[j * D + k], dot);
            double d = (-2.0 * dot + xx[i]) + xx[j];
            float f = (float)d;
            if (!(f >= 0.0f)) f = (f != f) ? f : 0.0f;
            f = sqrtf(f);
            out[i * n + j] = f;
            out[j * n + i] = f;
        }
    }
    free(xx);
}

/* float64 input: pairwise.py:423-441 keeps f64, sqrt in f64; ripser.py then
   casts the condensed values to float32 (a2' in SURVEY 8a). */
void oracle_distances_f64(const double *X, int64_t n, int64_t D, float *out) {
    double *xx = (double *)malloc(sizeof(double) * (size_t)(n ? n : 1));
    for (int64_t i = 0; i < n; ++i) {
        double s = 0.0;
        for (int64_t k = 0; k < D; ++k) s = fma(X[i * D + k], X[i * D + k], s);
        xx[i] = s;
    }
    for (int64_t i = 0; i < n; ++i) {
        out[i * n + i] = 0.0f;
        for (int64_t j = i + 1; j < n; ++j) {
            double dot = 0.0;
            for (int64_t k = 0; k < D; ++k) dot = fma(X[i * D + k], X[j * D + k], dot);
            double d = (-2.0 * dot + xx[i]) + xx[j];
            if (!(d >= 0.0)) d = (d != d) ? d : 0.0;
            float f = (float)sqrt(d);
            out[i * n + j] = f;
            out[j * n + i] = f;
        }
    }
    free(xx);
}

/* ---------- pivot hash map: uint64 simplex idx -> int64 column -------------- */
typedef struct {
    uint64_t *keys;
    int64_t *vals;
    uint64_t mask;
    int64_t count;
} hmap_t;
#define HM_EMPTY 0xFFFFFFFFFFFFFFFFULL

static void hm_init(hmap_t *h, int64_t expect) {
    uint64_t cap = 16;
    while (cap < (uint64_t)(expect * 2 + 16)) cap <<= 1;
    h->keys = (uint64_t *)malloc(cap * sizeof(uint64_t));
    h->vals = (int64_t *)malloc(cap * sizeof(int64_t));
    memset(h->keys, 0xFF, cap * sizeof(uint64_t));
    h->mask = cap - 1;
    h->count = 0;
}
static void hm_free(hmap_t *h) {
    free(h->keys);
    free(h->vals);
}
static void hm_grow(hmap_t *h);
static void hm_put(hmap_t *h, uint64_t k, int64_t v) {
    if ((uint64_t)(h->count + 1) * 2 > h->mask + 1) hm_grow(h);
    uint64_t i = mix64(k) & h->mask;
    while (h->keys[i] != HM_EMPTY && h->keys[i] != k) i = (i + 1) & h->mask;
    if (h->keys[i] == HM_EMPTY) h->count++;
    h->keys[i] = k;
    h->vals[i] = v;
}
static int64_t hm_get(const hmap_t *h, uint64_t k) {
    uint64_t i = mix64(k) & h->mask;
    while (h->keys[i] != HM_EMPTY) {
        if (h->keys[i] == k) return h->vals[i];
        i = (i + 1) & h->mask;
    }
    return -1;
}
static void hm_grow(hmap_t *h) {
    hmap_t g;
    hm_init(&g, (int64_t)(h->mask + 1));
    for (uint64_t i = 0; i <= h->mask; ++i)
        if (h->keys[i] != HM_EMPTY) hm_put(&g, h->keys[i], h->vals[i]);
    hm_free(h);
    *h = g;
}

/* ---------- binary heap with Ripser priority (min diam, then max idx) ------ */
typedef struct {
    splx_t *a;
    int64_t n, cap;
} heap_t;
static inline int heap_before(splx_t x, splx_t y) { /* x has higher priority */
    return x.diam < y.diam || (x.diam == y.diam && x.idx > y.idx);
}
static void heap_push(heap_t *h, splx_t e) {
    if (h->n == h->cap) {
        h->cap = h->cap ? h->cap * 2 : 256;
        h->a = (splx_t *)realloc(h->a, (size_t)h->cap * sizeof(splx_t));
    }
    int64_t i = h->n++;
    while (i > 0) {
        int64_t p = (i - 1) >> 1;
        if (!heap_before(e, h->a[p])) break;
        h->a[i] = h->a[p];
        i = p;
    }
    h->a[i] = e;
}
static splx_t heap_pop(heap_t *h) {
    splx_t top = h->a[0];
    splx_t last = h->a[--h->n];
    int64_t i = 0;
    for (;;) {
        int64_t l = 2 * i + 1, r = l + 1, m = i;
        splx_t best = last;
        if (l < h->n && heap_before(h->a[l], best)) { m = l; best = h->a[l]; }
        if (r < h->n && heap_before(h->a[r], best)) { m = r; }
        if (m == i) break;
        h->a[i] = h->a[m];
        i = m;
    }
    if (h->n > 0) h->a[i] = last;
    return top;
}
/* Z/2 pivot: pop equal pairs (they cancel); returns idx = HM_EMPTY if empty.
   Leaves the pivot in the heap. */
static splx_t heap_get_pivot(heap_t *h) {
    splx_t none = {0.0f, HM_EMPTY};
    while (h->n > 0) {
        splx_t p = heap_pop(h);
        if (h->n > 0 && h->a[0].idx == p.idx) {
            heap_pop(h); /* cancel pair */
            continue;
        }
        heap_push(h, p);
        return p;
    }
    return none;
}

int cmpu(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

/* ---------- the complex ------------------------------------------------ */
typedef struct {
    int64_t n;
    const float *dist; /* n x n */
    float thresh;
    binom_t B;
} cx_t;

static inline float dd(const cx_t *c, int64_t i, int64_t j) { return c->dist[i * c->n + j]; }

/* enumerate cofacets of sigma (vertices vs[0..dim], descending) in decreasing
   cofacet-index order; calls back only cofacets with diam <= thresh.  */
typedef struct {
    uint64_t idx;
    float diam;
} cof_t;

static int64_t cofacets(const cx_t *c, const int64_t *vs, int dim, float sdiam, uint64_t sidx, cof_t *out) {
    int64_t m = 0;
    uint64_t idx_below = sidx, idx_above = 0;
    int k = dim + 1; /* vertices of sigma below current v */
    int pos = 0;     /* next sigma vertex (descending) */
    for (int64_t v = c->n - 1; v >= 0; --v) {
        if (pos <= dim && vs[pos] == v) {
            idx_below -= C(&c->B, v, k);
            idx_above += C(&c->B, v, k + 1);
            --k;
            ++pos;
            continue;
        }
        float d = sdiam;
        for (int i = 0; i <= dim; ++i) {
            float x = dd(c, v, vs[i]);
            if (x > d) d = x;
        }
        if (d <= c->thresh) {
            out[m].idx = idx_above + C(&c->B, v, k + 1) + idx_below;
            out[m].diam = d;
            ++m;
        }
    }
    return m;
}

/* the first (largest-index) cofacet with diameter == sdiam, if any: the
   emergent-pair probe of Ripser's compute_pairs, which stops at it instead of
   enumerating the whole coboundary.  Returns 0 if none. */
static int first_equal_cofacet(const cx_t *c, const int64_t *vs, int dim, float sdiam, uint64_t sidx, uint64_t *out_idx) {
    uint64_t idx_below = sidx, idx_above = 0;
    int k = dim + 1, pos = 0;
    for (int64_t v = c->n - 1; v >= 0; --v) {
        if (pos <= dim && vs[pos] == v) {
            idx_below -= C(&c->B, v, k);
            idx_above += C(&c->B, v, k + 1);
            --k;
            ++pos;
            continue;
        }
        float d = sdiam;
        for (int i = 0; i <= dim; ++i) {
            float x = dd(c, v, vs[i]);
            if (x > d) d = x;
        }
        if (d == sdiam && d <= c->thresh) {
            *out_idx = idx_above + C(&c->B, v, k + 1) + idx_below;
            return 1;
        }
    }
    return 0;
}

static float simplex_diam(const cx_t *c, const int64_t *vs, int dim) {
    float d = 0.0f;
    for (int i = 0; i <= dim; ++i)
        for (int j = i + 1; j <= dim; ++j) {
            float x = dd(c, vs[i], vs[j]);
            if (x > d) d = x;
        }
    return d;
}

/* growable output buffer for emitted pairs of one dim */
typedef struct {
    float *b, *d;
    int64_t *bi, *di;
    int64_t n, cap;
} pairs_t;
static void pairs_push(pairs_t *p, float b, float d, int64_t bi, int64_t di) {
    if (p->n == p->cap) {
        p->cap = p->cap ? p->cap * 2 : 16;
        p->b = (float *)realloc(p->b, p->cap * sizeof(float));
        p->d = (float *)realloc(p->d, p->cap * sizeof(float));
        p->bi = (int64_t *)realloc(p->bi, p->cap * sizeof(int64_t));
        p->di = (int64_t *)realloc(p->di, p->cap * sizeof(int64_t));
    }
    p->b[p->n] = b;
    p->d[p->n] = d;
    p->bi[p->n] = bi;
    p->di[p->n] = di;
    p->n++;
}

/* union-find with elder rule under the vertex order (all births 0, ties ->
   larger vertex index is older): representative = max vertex of component. */
static int64_t uf_find(int64_t *par, int64_t x) {
    while (par[x] != x) {
        par[x] = par[par[x]];
        x = par[x];
    }
    return x;
}

/* ---------- main entry ---------------------------------------------------- */
/* dist: n x n float32 symmetric (only i<j used), zero diagonal.
   thresh: +inf -> enclosing radius. */
int oracle_rips_dm(const float *dist, int64_t n, int maxdim, float thresh, oracle_result *res) {
    memset(res, 0, sizeof(*res));
    if (maxdim < 0 || maxdim > OR_MAXDIM - 1) return -1;
    cx_t c;
    c.n = n;
    c.dist = dist;
    /* ORACLE_STATS=1: debug statistics (apparent pairs, heap sizes); off by
       default so the CPU baseline does only the work the result needs */
    const int stats = getenv("ORACLE_STATS") != NULL;
    /* ORACLE_COLSTATS=1: print the columns with more than 500 additions (dev aid) */
    const int colstats = getenv("ORACLE_COLSTATS") != NULL;
    /* ORACLE_TRACE=<file> ORACLE_TRACE_COL=<j> (dim 1): every key the column's reduction pushes and
       every pivot it pops, as u64 filtration keys diam_bits << 32 | ~idx (a pivot follows a ~0 marker);
       dev aid for modelling the GPU reducer's working-column structure (tools/front_sim.py) */
    FILE *trace = NULL;
    int64_t trace_col = getenv("ORACLE_TRACE_COL") ? atoll(getenv("ORACLE_TRACE_COL")) : -1;
    if (getenv("ORACLE_TRACE") && trace_col >= 0) trace = fopen(getenv("ORACLE_TRACE"), "wb");
    /* threshold (ripser.py rips_dm): enclosing radius when thresh is inf/max */
    if (isinf(thresh) || thresh == 3.402823466e+38f) {
        float enc = INFINITY;
        for (int64_t i = 0; i < n; ++i) {
            float r = -INFINITY;
            for (int64_t j = 0; j < n; ++j) {
                float x = (i == j) ? 0.0f : dd(&c, i < j ? i : j, i < j ? j : i);
                if (x > r) r = x;
            }
            if (r < enc) enc = r;
        }
        thresh = enc;
    }
    c.thresh = thresh;
    res->thresh = thresh;
    binom_init(&c.B, n, maxdim + 3);

    /* edges <= thresh */
    int64_t ne_all = n * (n - 1) / 2;
    splx_t *edges = (splx_t *)malloc(sizeof(splx_t) * (size_t)(ne_all ? ne_all : 1));
    int64_t ne = 0;
    for (int64_t i = 1; i < n; ++i)
        for (int64_t j = 0; j < i; ++j) {
            float d = dd(&c, j, i); /* upper triangle value (r=j < c=i) */
            if (d <= thresh) {
                edges[ne].diam = d;
                edges[ne].idx = C(&c.B, i, 2) + (uint64_t)j;
                ++ne;
            }
        }
    res->num_edges = ne;

    /* ---- H0 ---- */
    qsort(edges, (size_t)ne, sizeof(splx_t), cmp_filt_order);
    int64_t *par = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n ? n : 1));
    for (int64_t i = 0; i < n; ++i) par[i] = i;
    pairs_t P[OR_MAXDIM + 1];
    memset(P, 0, sizeof(P));
    splx_t *cols = (splx_t *)malloc(sizeof(splx_t) * (size_t)(ne ? ne : 1));
    int64_t ncols = 0;
    for (int64_t e = 0; e < ne; ++e) {
        int64_t vs[2];
        decode(&c.B, edges[e].idx, 1, n, vs);
        int64_t u = uf_find(par, vs[0]), v = uf_find(par, vs[1]);
        if (u != v) {
            /* elder rule: younger component = smaller representative */
            int64_t young = u < v ? u : v, old = u < v ? v : u;
            par[young] = old;
            res->n_all_pairs[0]++;
            res->checksum[0] += pair_hash((uint64_t)young, edges[e].idx);
            if (edges[e].diam > 0.0f) pairs_push(&P[0], 0.0f, edges[e].diam, young, (int64_t)edges[e].idx);
        } else {
            cols[ncols++] = edges[e];
        }
    }
    for (int64_t i = 0; i < n; ++i)
        if (uf_find(par, i) == i) pairs_push(&P[0], 0.0f, INFINITY, i, -1);
    /* columns for dim 1 in (diam desc, idx asc): reverse of Kruskal order */
    for (int64_t a = 0, b = ncols - 1; a < b; ++a, --b) {
        splx_t t = cols[a];
        cols[a] = cols[b];
        cols[b] = t;
    }
    free(par);

    /* simplices of current dim (for assembling next columns) */
    splx_t *simp = edges;
    int64_t nsimp = ne;

    heap_t work = {0}, vwork = {0};
    cof_t *cbuf = (cof_t *)malloc(sizeof(cof_t) * (size_t)(n + 1));
    int64_t vsig[OR_MAXDIM + 2], vtmp[OR_MAXDIM + 2];

    for (int dim = 1; dim <= maxdim; ++dim) {
        hmap_t piv;
        hm_init(&piv, ncols);
        /* reduction matrix V (extra entries per column) */
        int64_t *voff = (int64_t *)malloc(sizeof(int64_t) * (size_t)(ncols + 1));
        int64_t vcap = 1024, vn = 0;
        uint64_t *vdat = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)vcap);
        voff[0] = 0;
        res->n_columns[dim] = ncols;

        for (int64_t j = 0; j < ncols; ++j) {
            splx_t sg = cols[j];
            decode(&c.B, sg.idx, dim, n, vsig);
            /* emergent pair shortcut: the first cofacet (largest idx) with
               equal diameter is the pivot; if unclaimed it pairs immediately
               (found without enumerating the rest of the coboundary). */
            if (!stats) {
                uint64_t e_idx;
                if (first_equal_cofacet(&c, vsig, dim, sg.diam, sg.idx, &e_idx) && hm_get(&piv, e_idx) < 0) {
                    hm_put(&piv, e_idx, j);
                    res->n_all_pairs[dim]++;
                    res->checksum[dim] += pair_hash(sg.idx, e_idx);
                    voff[j + 1] = vn;
                    continue;
                }
            }
            int64_t m = cofacets(&c, vsig, dim, sg.diam, sg.idx, cbuf);
            /* apparent-pair statistic (ORACLE_STATS=1 only; not used for the result) */
            if (stats) {
                int64_t best = -1;
                for (int64_t q = 0; q < m; ++q)
                    if (best < 0 || cbuf[q].diam < cbuf[best].diam) best = q; /* decreasing idx: first min = max idx */
                if (best >= 0 && cbuf[best].diam == sg.diam) {
                    /* sigma is youngest facet of tau iff no facet with larger
                       vertex removed... computed generically: */
                    int64_t tv[OR_MAXDIM + 2];
                    decode(&c.B, cbuf[best].idx, dim + 1, n, tv);
                    int ok = 1;
                    for (int r = 0; r <= dim + 1 && ok; ++r) {
                        int64_t fv[OR_MAXDIM + 2];
                        int q = 0;
                        uint64_t fidx = 0;
                        for (int s = 0; s <= dim + 1; ++s)
                            if (s != r) fv[q++] = tv[s];
                        for (int s = 0; s <= dim; ++s) fidx += C(&c.B, fv[s], dim + 1 - s);
                        if (fidx == sg.idx) continue;
                        float fd = simplex_diam(&c, fv, dim);
                        if (fd > sg.diam || (fd == sg.diam && fidx < sg.idx)) ok = 0;
                    }
                    if (ok) res->n_apparent[dim]++;
                }
            }
            /* emergent pair shortcut: first cofacet (largest idx) with equal
               diameter is the pivot; if unclaimed it pairs immediately. */
            int emergent_done = 0;
            for (int64_t q = 0; q < m; ++q) {
                if (cbuf[q].diam == sg.diam) {
                    if (hm_get(&piv, cbuf[q].idx) < 0) {
                        hm_put(&piv, cbuf[q].idx, j);
                        res->n_all_pairs[dim]++;
                        res->checksum[dim] += pair_hash(sg.idx, cbuf[q].idx);
                        emergent_done = 1;
                    }
                    break;
                }
            }
            if (emergent_done) {
                voff[j + 1] = vn;
                continue;
            }
            work.n = 0;
            vwork.n = 0;
            int64_t adds0 = res->n_adds[dim];
            const int tr = trace && dim == 1 && j == trace_col;
            for (int64_t q = 0; q < m; ++q) {
                splx_t e = {cbuf[q].diam, cbuf[q].idx};
                heap_push(&work, e);
                if (tr) {
                    uint32_t db;
                    memcpy(&db, &cbuf[q].diam, 4);
                    const uint64_t key = ((uint64_t)db << 32) | (0xFFFFFFFFull - (cbuf[q].idx & 0xFFFFFFFFull));
                    fwrite(&key, 8, 1, trace);
                }
            }
            for (;;) {
                splx_t p = heap_get_pivot(&work);
                if (stats) {
                    if (work.n > res->max_heap[dim]) res->max_heap[dim] = work.n;
                    res->sum_heap_steps[dim] += work.n;
                }
                if ((p.idx == HM_EMPTY || hm_get(&piv, p.idx) < 0) && colstats && res->n_adds[dim] - adds0 > 500)
                    fprintf(stderr, "[oracle-col] dim %d col %lld of %lld adds %lld birth %.6f death %.6f heap %lld\n", dim,
                            (long long)j, (long long)ncols, (long long)(res->n_adds[dim] - adds0), sg.diam,
                            p.idx == HM_EMPTY ? INFINITY : p.diam, (long long)work.n);
                if (p.idx == HM_EMPTY) {
                    pairs_push(&P[dim], sg.diam, INFINITY, (int64_t)sg.idx, -1);
                    voff[j + 1] = vn;
                    break;
                }
                int64_t o = hm_get(&piv, p.idx);
                if (tr && p.idx != HM_EMPTY) {
                    uint32_t db;
                    memcpy(&db, &p.diam, 4);
                    const uint64_t mk = ~0ull, key = ((uint64_t)db << 32) | (0xFFFFFFFFull - (p.idx & 0xFFFFFFFFull));
                    fwrite(&mk, 8, 1, trace);
                    fwrite(&key, 8, 1, trace);
                }
                if (o >= 0) {
                    res->n_adds[dim]++;
                    /* add column o: its simplex plus its V entries */
                    int64_t cnt = 1 + (voff[o + 1] - voff[o]);
                    for (int64_t t = 0; t < cnt; ++t) {
                        uint64_t s = (t == 0) ? cols[o].idx : vdat[voff[o] + t - 1];
                        decode(&c.B, s, dim, n, vtmp);
                        float sd = (t == 0) ? cols[o].diam : simplex_diam(&c, vtmp, dim);
                        int64_t mm = cofacets(&c, vtmp, dim, sd, s, cbuf);
                        for (int64_t q = 0; q < mm; ++q) {
                            splx_t e = {cbuf[q].diam, cbuf[q].idx};
                            heap_push(&work, e);
                            if (tr) {
                                uint32_t db;
                                memcpy(&db, &cbuf[q].diam, 4);
                                const uint64_t key = ((uint64_t)db << 32) | (0xFFFFFFFFull - (cbuf[q].idx & 0xFFFFFFFFull));
                                fwrite(&key, 8, 1, trace);
                            }
                        }
                        splx_t ve = {0.0f, s};
                        heap_push(&vwork, ve);
                    }
                } else {
                    if (getenv("ORACLE_DEBUG_LIVE")) {
                        uint64_t *tmpk = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(work.n + 1));
                        for (int64_t q = 0; q < work.n; ++q) tmpk[q] = work.a[q].idx;
                        int cmpu(const void *a, const void *b);
                        qsort(tmpk, (size_t)work.n, sizeof(uint64_t), cmpu);
                        int64_t live = 0;
                        for (int64_t q = 0; q < work.n;) {
                            int64_t r = q;
                            while (r < work.n && tmpk[r] == tmpk[q]) ++r;
                            live += (r - q) & 1;
                            q = r;
                        }
                        free(tmpk);
                        if (live > res->max_live[dim]) res->max_live[dim] = live;
                        res->sum_live[dim] += live;
                    }
                    if (p.diam > sg.diam) pairs_push(&P[dim], sg.diam, p.diam, (int64_t)sg.idx, (int64_t)p.idx);
                    hm_put(&piv, p.idx, j);
                    res->n_all_pairs[dim]++;
                    res->checksum[dim] += pair_hash(sg.idx, p.idx);
                    /* store V_j = Z/2-reduced vwork */
                    for (;;) {
                        splx_t v = heap_get_pivot(&vwork);
                        if (v.idx == HM_EMPTY) break;
                        heap_pop(&vwork);
                        if (vn == vcap) {
                            vcap *= 2;
                            vdat = (uint64_t *)realloc(vdat, sizeof(uint64_t) * (size_t)vcap);
                        }
                        vdat[vn++] = v.idx;
                    }
                    voff[j + 1] = vn;
                    break;
                }
            }
        }
        free(voff);
        free(vdat);
        if (trace && dim == 1) {
            fclose(trace);
            trace = NULL;
        }

        if (dim < maxdim) {
            /* assemble (dim+1)-simplices: add a vertex above the max vertex of
               each dim-simplex; skip pivots (clearing) */
            int64_t cap = 1024, nn = 0, nc = 0;
            splx_t *next = (splx_t *)malloc(sizeof(splx_t) * (size_t)cap);
            free(cols);
            int64_t ccap = 1024;
            cols = (splx_t *)malloc(sizeof(splx_t) * (size_t)ccap);
            for (int64_t s = 0; s < nsimp; ++s) {
                decode(&c.B, simp[s].idx, dim, n, vsig);
                uint64_t base = simp[s].idx;
                for (int64_t v = vsig[0] + 1; v < n; ++v) {
                    float d = simp[s].diam;
                    for (int i = 0; i <= dim; ++i) {
                        float x = dd(&c, v, vsig[i]);
                        if (x > d) d = x;
                    }
                    if (d > thresh) continue;
                    uint64_t idx = C(&c.B, v, dim + 2) + base;
                    if (nn == cap) {
                        cap *= 2;
                        next = (splx_t *)realloc(next, sizeof(splx_t) * (size_t)cap);
                    }
                    next[nn].diam = d;
                    next[nn].idx = idx;
                    ++nn;
                    if (hm_get(&piv, idx) < 0) {
                        if (nc == ccap) {
                            ccap *= 2;
                            cols = (splx_t *)realloc(cols, sizeof(splx_t) * (size_t)ccap);
                        }
                        cols[nc].diam = d;
                        cols[nc].idx = idx;
                        ++nc;
                    }
                }
            }
            free(simp);
            simp = next;
            nsimp = nn;
            ncols = nc;
            qsort(cols, (size_t)ncols, sizeof(splx_t), cmp_col_order);
        }
        hm_free(&piv);
    }
    free(simp);
    free(cols);
    free(cbuf);
    free(work.a);
    free(vwork.a);
    free(c.B.t);
    for (int d = 0; d <= maxdim; ++d) {
        res->n_pairs[d] = P[d].n;
        res->births[d] = P[d].b;
        res->deaths[d] = P[d].d;
        res->birth_idx[d] = P[d].bi;
        res->death_idx[d] = P[d].di;
    }
    return 0;
}

void oracle_free(oracle_result *r) {
    for (int d = 0; d <= OR_MAXDIM; ++d) {
        free(r->births[d]);
        free(r->deaths[d]);
        free(r->birth_idx[d]);
        free(r->death_idx[d]);
        r->births[d] = r->deaths[d] = NULL;
        r->birth_idx[d] = r->death_idx[d] = NULL;
    }
}

/* batch helper used by the CPU baseline: L layers of (n, D) f32 clouds. */
int oracle_rips_batch_f32(const float *X, int64_t L, int64_t n, int64_t D, int maxdim, float thresh,
                          oracle_result *res) {
    float *dist = (float *)malloc(sizeof(float) * (size_t)(n > 0 ? n * n : 1));
    for (int64_t l = 0; l < L; ++l) {
        oracle_distances_f32(X + l * n * D, n, D, dist);
        int rc = oracle_rips_dm(dist, n, maxdim, thresh, &res[l]);
        if (rc) {
            free(dist);
            return rc;
        }
    }
    free(dist);
    return 0;
}

int oracle_version(void) { return 1; }
