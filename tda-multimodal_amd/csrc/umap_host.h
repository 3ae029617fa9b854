// umap_host.h -- host side of tda_umap_batch (include/tda_umap.h), part of
// rips.hip's translation unit (shares its error state and device checks).
#pragma once
#include "../../include/tda_umap.h"
#include "umap_kernels.h"

namespace {

struct UmapWs {
    int device = -1;
    hipStream_t stream = nullptr;
    hipEvent_t evin = nullptr;
    char* buf = nullptr;
    size_t cap = 0;
    std::mutex mu;
};
std::mutex g_umap_mu;
std::vector<UmapWs*> g_umap_ws;

UmapWs& umap_ws(int dev) {
    std::lock_guard<std::mutex> g(g_umap_mu);
    for (auto* w : g_umap_ws)
        if (w->device == dev) return *w;
    auto* w = new UmapWs();
    w->device = dev;
    g_umap_ws.push_back(w);
    return *w;
}

int umap_validate(const tda_umap_args* a) {
    if (!a) return fail(TDA_E_INVALID, "args is NULL");
    if (!a->x || !a->out) return fail(TDA_E_INVALID, "x and out are required");
    if (a->L < 1 || a->N < 2 || a->D < 1) return fail(TDA_E_INVALID, "need L >= 1, N >= 2, D >= 1");
    if (a->dtype != TDA_F32 && a->dtype != TDA_F64) return fail(TDA_E_INVALID, "dtype must be TDA_F32 or TDA_F64");
    if (a->metric != TDA_UMAP_EUCLIDEAN && a->metric != TDA_UMAP_COSINE)
        return fail(TDA_E_UNSUPPORTED, "metric must be 'euclidean' or 'cosine'");
    if (a->N >= 4096) return fail(TDA_E_UNSUPPORTED, "UMAP: N < 4096 (umap-learn's exact small-data regime) is supported");
    if (a->n_neighbors < 2 || a->n_neighbors > kUmapMaxK || a->n_neighbors > a->N)
        return fail(TDA_E_INVALID, "n_neighbors must be in [2, min(64, N)]");
    if (a->n_components < 1 || a->n_components > kUmapMaxC) return fail(TDA_E_INVALID, "n_components must be in [1, 8]");
    if ((size_t)a->N * a->n_components * 12 > 150 * 1024) return fail(TDA_E_UNSUPPORTED, "UMAP: N * n_components too large for LDS");
    if (a->n_epochs < 1 || a->negative_sample_rate < 0) return fail(TDA_E_INVALID, "n_epochs >= 1, negative_sample_rate >= 0");
    if (!(a->a > 0.0f) || !(a->b > 0.0f)) return fail(TDA_E_INVALID, "a, b must be positive");
    return 0;
}

// the UMAP input distances of L clouds of n points (cosine always on the FP64
// matrix cores; euclidean from D >= 32 there too, else the scalar kernel)
void umap_distances(const void* x, int dtype, int metric, int64_t L, int64_t N, int64_t D, float* dist, uint32_t* rmax, hipStream_t s) {
    const unsigned nt = (unsigned)((N + kDmT - 1) / kDmT);
    const dim3 gm(nt * (nt + 1) / 2, (unsigned)L);
    if (metric == TDA_UMAP_COSINE) {
        if (dtype == TDA_F64)
            hipLaunchKernelGGL((k_distance_mfma<double, 1>), gm, dim3(256), 0, s, (const double*)x, (int)N, (int)D, dist, rmax, (double*)nullptr, (double*)nullptr);
        else
            hipLaunchKernelGGL((k_distance_mfma<float, 1>), gm, dim3(256), 0, s, (const float*)x, (int)N, (int)D, dist, rmax, (double*)nullptr, (double*)nullptr);
    } else if (D >= kDistMfmaMinD) {
        if (dtype == TDA_F64)
            hipLaunchKernelGGL((k_distance_mfma<double, 0>), gm, dim3(256), 0, s, (const double*)x, (int)N, (int)D, dist, rmax, (double*)nullptr, (double*)nullptr);
        else
            hipLaunchKernelGGL((k_distance_mfma<float, 0>), gm, dim3(256), 0, s, (const float*)x, (int)N, (int)D, dist, rmax, (double*)nullptr, (double*)nullptr);
    } else {
        const dim3 g((unsigned)((N + 15) / 16), (unsigned)((N + 15) / 16), (unsigned)L);
        if (dtype == TDA_F64)
            hipLaunchKernelGGL(k_distance<double>, g, dim3(256), 0, s, (const double*)x, (int)N, (int)D, dist, rmax);
        else
            hipLaunchKernelGGL(k_distance<float>, g, dim3(256), 0, s, (const float*)x, (int)N, (int)D, dist, rmax);
    }
}

}  // namespace

extern "C" int tda_umap_batch(const tda_umap_args* a) {
    if (int rc = umap_validate(a)) return rc;
    if (!tda_device_ok(a->device)) return fail(TDA_E_NODEVICE, "no gfx950 device at ordinal " + std::to_string(a->device));
    HIPC(hipSetDevice(a->device));
    UmapWs& w = umap_ws(a->device);
    std::lock_guard<std::mutex> guard(w.mu);
    if (!w.stream) HIPC(hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking));
    const int64_t L = a->L, N = a->N, D = a->D, k = a->n_neighbors, c = a->n_components;
    const size_t esz = a->dtype == TDA_F64 ? 8 : 4;
    const uint64_t ecap = (uint64_t)align_up((uint64_t)(2 * N * k), 64);
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t r = o;
        o = align_up(o + bytes, 256);
        return r;
    };
    const size_t o_x = take(a->x_on_device ? 0 : L * N * D * esz), o_dist = take(L * N * N * 4), o_rmax = take(L * N * 4),
                 o_kd = take(L * N * k * 4), o_ki = take(L * N * k * 4), o_P = take(L * N * N * 4), o_S = take(L * N * N * 4),
                 o_smax = take(L * 4), o_ne = take(L * 4), o_head = take(L * ecap * 4), o_tail = take(L * ecap * 4),
                 o_eps = take(L * ecap * 8), o_nxt = take(L * ecap * 8), o_nxn = take(L * ecap * 8), o_deg = take(L * N * 4),
                 o_emb = take(L * N * c * 4);
    if (w.cap < o) {
        if (w.buf) HIPC(hipFree(w.buf));
        w.buf = nullptr;
        HIPC(hipMalloc(&w.buf, o));
        w.cap = o;
    }
    char* B = w.buf;
    hipStream_t s = w.stream;
    if (a->x_on_device) {  // device inputs: read after the caller's queued work (NULL = the null stream)
        if (!w.evin) HIPC(hipEventCreateWithFlags(&w.evin, hipEventDisableTiming));
        if (int rc = order_after_caller(s, w.evin, a->stream, a->device)) return rc;
    }
    const void* x = a->x;
    if (!a->x_on_device) {
        HIPC(hipMemcpyAsync(B + o_x, a->x, (size_t)L * N * D * esz, hipMemcpyHostToDevice, s));
        x = B + o_x;
    }
    UmapBufs u;
    u.dist = (const float*)(B + o_dist);
    u.kd = (float*)(B + o_kd);
    u.ki = (int32_t*)(B + o_ki);
    u.P = (float*)(B + o_P);
    u.S = (float*)(B + o_S);
    u.smax = (uint32_t*)(B + o_smax);
    u.head = (int32_t*)(B + o_head);
    u.tail = (int32_t*)(B + o_tail);
    u.eps = (double*)(B + o_eps);
    u.nxt = (double*)(B + o_nxt);
    u.nxn = (double*)(B + o_nxn);
    u.deg = (float*)(B + o_deg);
    u.nedge = (uint32_t*)(B + o_ne);
    u.emb = (float*)(B + o_emb);
    u.ecap = ecap;
    u.n = (int)N;
    u.k = (int)k;
    u.c = (int)c;
    u.n_epochs = a->n_epochs;
    u.lstride = (size_t)N * N;
    u.stride = (int)N;
    u.qrow0 = 0;
    u.nq = (int)N;
    u.ncand = (int)N;
    HIPC(hipMemsetAsync(u.P, 0, (size_t)L * N * N * 4, s));
    HIPC(hipMemsetAsync(u.smax, 0, (size_t)L * 4, s));
    HIPC(hipMemsetAsync(u.nedge, 0, (size_t)L * 4, s));
    // distances: Gram tiles on the FP64 matrix cores (cosine always; euclidean from D >= 32, else the scalar kernel)
    float* dist = (float*)(B + o_dist);
    uint32_t* rmax = (uint32_t*)(B + o_rmax);
    umap_distances(x, a->dtype, a->metric, L, N, D, dist, rmax, s);
    HIPC(hipGetLastError());
    hipLaunchKernelGGL(k_umap_knn, dim3((unsigned)((N + kUmapKnnT - 1) / kUmapKnnT), (unsigned)L), dim3(kUmapKnnT), 0, s, u);
    HIPC(hipGetLastError());
    hipLaunchKernelGGL(k_umap_smooth, dim3((unsigned)L), dim3(kUmapT), 0, s, u);
    HIPC(hipGetLastError());
    const unsigned gs = (unsigned)std::min<uint64_t>(1024, ((uint64_t)N * N + 255) / 256);
    hipLaunchKernelGGL(k_umap_sym, dim3(gs, (unsigned)L), dim3(256), 0, s, u);
    HIPC(hipGetLastError());
    hipLaunchKernelGGL(k_umap_edges, dim3((unsigned)L), dim3(kUmapT), 0, s, u);
    HIPC(hipGetLastError());
    const int B2 = (int)c + 3;
    const size_t spec_lds = ((size_t)2 * B2 + 1) * N * 4;
    const bool spectral = a->init == TDA_UMAP_INIT_SPECTRAL && N <= kUmapSpecMaxN && spec_lds <= 150 * 1024;
    HIPC(hipFuncSetAttribute((const void*)k_umap_spectral, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
    HIPC(hipFuncSetAttribute((const void*)k_umap_sgd, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
    const int spec_iters = test_env("TDA_UMAP_SPEC_ITERS") ? atoi(test_env("TDA_UMAP_SPEC_ITERS")) : 300;
    hipLaunchKernelGGL(k_umap_spectral, dim3((unsigned)L), dim3(kUmapT), spectral ? spec_lds : 0, s, u, spec_iters, a->seed,
                       spectral ? 0 : 1);
    HIPC(hipGetLastError());
    const size_t sgd_lds = align_up((size_t)4 * N * c, 16) + (size_t)8 * N * c;
    hipLaunchKernelGGL(k_umap_sgd, dim3((unsigned)L), dim3(kUmapT), sgd_lds, s, u, (double)a->a, (double)a->b,
                       (double)a->learning_rate, (double)a->repulsion_strength, a->negative_sample_rate, a->seed);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(a->out, u.emb, (size_t)L * N * c * 4, hipMemcpyDeviceToHost, s));
    if (a->graph_out) HIPC(hipMemcpyAsync(a->graph_out, u.S, (size_t)L * N * N * 4, hipMemcpyDeviceToHost, s));
    std::vector<uint32_t> ne(L);
    HIPC(hipMemcpyAsync(ne.data(), u.nedge, (size_t)L * 4, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    for (int64_t l = 0; l < L; ++l)
        if (ne[l] > ecap) return fail(TDA_E_CAPACITY, "UMAP edge list overflow");
    return 0;
}

extern "C" int tda_umap_transform(const tda_umap_transform_args* a) {
    if (!a) return fail(TDA_E_INVALID, "args is NULL");
    if (!a->x_train || !a->emb_train || !a->y || !a->out) return fail(TDA_E_INVALID, "x_train, emb_train, y and out are required");
    if (a->L < 1 || a->M < 1 || a->N < 2 || a->D < 1) return fail(TDA_E_INVALID, "need L >= 1, M >= 1, N >= 2, D >= 1");
    if (a->dtype != TDA_F32 && a->dtype != TDA_F64) return fail(TDA_E_INVALID, "dtype must be TDA_F32 or TDA_F64");
    if (a->metric != TDA_UMAP_EUCLIDEAN && a->metric != TDA_UMAP_COSINE)
        return fail(TDA_E_UNSUPPORTED, "metric must be 'euclidean' or 'cosine'");
    if (a->N + a->M > 8192) return fail(TDA_E_UNSUPPORTED, "UMAP transform: N + M <= 8192 (exact small-data regime) is supported");
    if (a->n_neighbors < 2 || a->n_neighbors > kUmapMaxK || a->n_neighbors > a->N)
        return fail(TDA_E_INVALID, "n_neighbors must be in [2, min(64, N)]");
    if (a->n_components < 1 || a->n_components > kUmapMaxC) return fail(TDA_E_INVALID, "n_components must be in [1, 8]");
    const int64_t L = a->L, M = a->M, N = a->N, D = a->D, k = a->n_neighbors, c = a->n_components, NM = N + M;
    const size_t lds = (((size_t)4 * M * c + 15) & ~(size_t)15) + (size_t)8 * M * c + (size_t)4 * N * c;
    if (lds > 150 * 1024) return fail(TDA_E_UNSUPPORTED, "UMAP transform: (M, N) * n_components too large for LDS");
    if (a->n_epochs < 1 || a->negative_sample_rate < 0) return fail(TDA_E_INVALID, "n_epochs >= 1, negative_sample_rate >= 0");
    if (!(a->a > 0.0f) || !(a->b > 0.0f)) return fail(TDA_E_INVALID, "a, b must be positive");
    if (!tda_device_ok(a->device)) return fail(TDA_E_NODEVICE, "no gfx950 device at ordinal " + std::to_string(a->device));
    HIPC(hipSetDevice(a->device));
    UmapWs& w = umap_ws(a->device);
    std::lock_guard<std::mutex> guard(w.mu);
    if (!w.stream) HIPC(hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking));
    hipStream_t s = w.stream;
    if (a->x_on_device) {  // device inputs: read after the caller's queued work (NULL = the null stream)
        if (!w.evin) HIPC(hipEventCreateWithFlags(&w.evin, hipEventDisableTiming));
        if (int rc = order_after_caller(s, w.evin, a->stream, a->device)) return rc;
    }
    const size_t esz = a->dtype == TDA_F64 ? 8 : 4;
    const uint64_t ecap = (uint64_t)M * k;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t r = o;
        o = align_up(o + bytes, 256);
        return r;
    };
    const size_t o_xt = take(a->x_on_device ? 0 : N * D * esz), o_y = take(a->x_on_device ? 0 : L * M * D * esz),
                 o_z = take(L * NM * D * esz), o_dist = take(L * NM * NM * 4), o_rmax = take(L * NM * 4), o_kd = take(L * M * k * 4),
                 o_ki = take(L * M * k * 4), o_val = take(L * M * k * 4), o_eps = take(L * ecap * 8), o_nxt = take(L * ecap * 8),
                 o_nxn = take(L * ecap * 8), o_temb = take(N * c * 4), o_emb = take(L * M * c * 4);
    if (w.cap < o) {
        if (w.buf) HIPC(hipFree(w.buf));
        w.buf = nullptr;
        HIPC(hipMalloc(&w.buf, o));
        w.cap = o;
    }
    char* B = w.buf;
    const void* xt = a->x_train;
    const void* y = a->y;
    if (!a->x_on_device) {
        HIPC(hipMemcpyAsync(B + o_xt, xt, (size_t)N * D * esz, hipMemcpyHostToDevice, s));
        HIPC(hipMemcpyAsync(B + o_y, y, (size_t)L * M * D * esz, hipMemcpyHostToDevice, s));
        xt = B + o_xt;
        y = B + o_y;
    }
    HIPC(hipMemcpyAsync(B + o_temb, a->emb_train, (size_t)N * c * 4, hipMemcpyHostToDevice, s));
    const uint64_t tw = (uint64_t)N * D * esz / 4, lw = (uint64_t)M * D * esz / 4;
    hipLaunchKernelGGL(k_umap_concat, dim3((unsigned)std::min<uint64_t>(1024, (tw + lw + 255) / 256), (unsigned)L), dim3(256), 0, s,
                       (const uint32_t*)xt, (const uint32_t*)y, (uint32_t*)(B + o_z), tw, lw);
    HIPC(hipGetLastError());
    umap_distances(B + o_z, a->dtype, a->metric, L, NM, D, (float*)(B + o_dist), (uint32_t*)(B + o_rmax), s);
    HIPC(hipGetLastError());
    UmapBufs u = {};
    u.dist = (const float*)(B + o_dist);
    u.kd = (float*)(B + o_kd);
    u.ki = (int32_t*)(B + o_ki);
    u.eps = (double*)(B + o_eps);
    u.nxt = (double*)(B + o_nxt);
    u.nxn = (double*)(B + o_nxn);
    u.emb = (float*)(B + o_emb);
    u.ecap = ecap;
    u.n = (int)NM;
    u.k = (int)k;
    u.c = (int)c;
    u.n_epochs = a->n_epochs;
    u.lstride = (size_t)NM * NM;
    u.stride = (int)NM;
    u.qrow0 = (int)N;
    u.nq = (int)M;
    u.ncand = (int)N;
    hipLaunchKernelGGL(k_umap_knn, dim3((unsigned)((M + kUmapKnnT - 1) / kUmapKnnT), (unsigned)L), dim3(kUmapKnnT), 0, s, u);
    HIPC(hipGetLastError());
    HIPC(hipFuncSetAttribute((const void*)k_umap_transform, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
    hipLaunchKernelGGL(k_umap_transform, dim3((unsigned)L), dim3(kUmapT), lds, s, u, (const float*)(B + o_temb), (int)N,
                       (float*)(B + o_val), (double)a->a, (double)a->b, (double)a->learning_rate, (double)a->repulsion_strength,
                       a->negative_sample_rate, a->seed, a->disconnection);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(a->out, u.emb, (size_t)L * M * c * 4, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    return 0;
}
