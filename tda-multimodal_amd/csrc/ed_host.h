// ed_host.h -- host side of tda_effective_dim (include/tda_rips.h), part of
// rips.hip's translation unit (shares its error state and device checks).
#pragma once
#include "ed_kernels.h"

namespace {

struct EdWs {
    int device = -1;
    hipStream_t stream = nullptr;
    hipEvent_t evin = nullptr;
    char* buf = nullptr;
    size_t cap = 0;
    float* hout = nullptr;  // pinned result
    size_t hcap = 0;
    std::mutex mu;
};
std::mutex g_ed_mu;
std::vector<EdWs*> g_ed_ws;

EdWs& ed_ws(int dev) {
    std::lock_guard<std::mutex> g(g_ed_mu);
    for (auto* w : g_ed_ws)
        if (w->device == dev) return *w;
    auto* w = new EdWs();
    w->device = dev;
    g_ed_ws.push_back(w);
    return *w;
}

}  // namespace

extern "C" int tda_effective_dim(const tda_ed_args* a, float* out) {
    if (!a || !out) return fail(TDA_E_INVALID, "args and out are required");
    if (a->B < 1 || a->N < 1 || a->D < 1) return fail(TDA_E_INVALID, "need B, N, D >= 1");
    if (!a->x) return fail(TDA_E_INVALID, "x is NULL");
    if (a->dtype != TDA_F32 && a->dtype != TDA_F64) return fail(TDA_E_INVALID, "dtype must be TDA_F32 or TDA_F64");
    const int64_t B = a->B, N = a->N, D = a->D, m = std::min(N, D);
    if (m > kEdMaxM) return fail(TDA_E_UNSUPPORTED, "effective dimensionality: min(N, D) <= 1024 is supported");
    if (N > 8192 && N <= D) return fail(TDA_E_UNSUPPORTED, "effective dimensionality: N <= 8192");
    if (!tda_device_ok(a->device)) return fail(TDA_E_NODEVICE, "no gfx950 device at ordinal " + std::to_string(a->device));
    HIPC(hipSetDevice(a->device));
    EdWs& w = ed_ws(a->device);
    std::lock_guard<std::mutex> guard(w.mu);
    if (!w.stream) HIPC(hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking));
    hipStream_t s = w.stream;
    if (a->x_on_device) {  // device inputs: read after the caller's queued work (NULL = the null stream)
        if (!w.evin) HIPC(hipEventCreateWithFlags(&w.evin, hipEventDisableTiming));
        if (int rc = order_after_caller(s, w.evin, a->stream, a->device)) return rc;
    }
    const size_t esz = a->dtype == TDA_F64 ? 8 : 4;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t r = o;
        o = align_up(o + bytes, 256);
        return r;
    };
    const size_t o_x = take(a->x_on_device ? 0 : (size_t)B * N * D * esz), o_g = take((size_t)B * m * m * 8);
    if (w.cap < o) {
        if (w.buf) HIPC(hipFree(w.buf));
        w.buf = nullptr;
        HIPC(hipMalloc(&w.buf, o));
        w.cap = o;
    }
    if (w.hcap < (size_t)B) {
        if (w.hout) HIPC(hipHostFree(w.hout));
        w.hout = nullptr;
        HIPC(hipHostMalloc((void**)&w.hout, sizeof(float) * B, hipHostMallocMapped));
        w.hcap = (size_t)B;
    }
    const void* x = a->x;
    if (!a->x_on_device) {
        HIPC(hipMemcpyAsync(w.buf + o_x, x, (size_t)B * N * D * esz, hipMemcpyHostToDevice, s));
        x = w.buf + o_x;
    }
    double* G = (double*)(w.buf + o_g);
    const bool f64 = a->dtype == TDA_F64;
    if (N <= D && D >= kDistMfmaMinD) {  // X X^T on the FP64 matrix cores
        const unsigned nt = (unsigned)((N + kDmT - 1) / kDmT);
        const dim3 gm(nt * (nt + 1) / 2, (unsigned)B);
        if (f64)
            hipLaunchKernelGGL((k_distance_mfma<double, 2>), gm, dim3(256), 0, s, (const double*)x, (int)N, (int)D, (float*)nullptr,
                               (uint32_t*)nullptr, G, (double*)nullptr);
        else
            hipLaunchKernelGGL((k_distance_mfma<float, 2>), gm, dim3(256), 0, s, (const float*)x, (int)N, (int)D, (float*)nullptr,
                               (uint32_t*)nullptr, G, (double*)nullptr);
    } else {
        const unsigned gx = (unsigned)std::min<uint64_t>(1024, ((uint64_t)m * m + 255) / 256);
        if (N <= D) {
            if (f64) hipLaunchKernelGGL(k_gram_rows<double>, dim3(gx, (unsigned)B), dim3(256), 0, s, (const double*)x, (int)N, (int)D, G);
            else hipLaunchKernelGGL(k_gram_rows<float>, dim3(gx, (unsigned)B), dim3(256), 0, s, (const float*)x, (int)N, (int)D, G);
        } else {
            if (f64) hipLaunchKernelGGL(k_gram_cols<double>, dim3(gx, (unsigned)B), dim3(256), 0, s, (const double*)x, (int)N, (int)D, G);
            else hipLaunchKernelGGL(k_gram_cols<float>, dim3(gx, (unsigned)B), dim3(256), 0, s, (const float*)x, (int)N, (int)D, G);
        }
    }
    HIPC(hipGetLastError());
    float* dout = nullptr;
    HIPC(hipHostGetDevicePointer((void**)&dout, w.hout, 0));
    if (m <= kEdLdsMaxM) {
        HIPC(hipFuncSetAttribute((const void*)k_ed_jacobi<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * kEdLdsMaxM * kEdLdsMaxM));
        hipLaunchKernelGGL(k_ed_jacobi<true>, dim3((unsigned)B), dim3(kEdT), (size_t)8 * m * m, s, G, (int)m, (int)m, dout);
    } else {
        hipLaunchKernelGGL(k_ed_jacobi<false>, dim3((unsigned)B), dim3(kEdT), 0, s, G, (int)m, (int)m, dout);
    }
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(s));
    std::memcpy(out, w.hout, sizeof(float) * B);
    return 0;
}
