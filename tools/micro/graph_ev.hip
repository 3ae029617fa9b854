// probe: can a timing event be recorded inside a stream capture (external event node)?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k_spin(int* x, int n) {
    for (int i = 0; i < n; ++i) atomicAdd(x, 1);
}
int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    int* x;
    hipMalloc(&x, 4);
    hipStreamCaptureMode modes[3] = {hipStreamCaptureModeGlobal, hipStreamCaptureModeThreadLocal, hipStreamCaptureModeRelaxed};
    for (int m = 0; m < 3; ++m)
        for (int f = 0; f < 2; ++f) {
            hipEvent_t e0, e1;
            if (f == 0) { hipEventCreate(&e0); hipEventCreate(&e1); }
            else { hipEventCreateWithFlags(&e0, hipEventDefault); hipEventCreateWithFlags(&e1, hipEventBlockingSync); }
            hipStreamBeginCapture(s, modes[m]);
            hipError_t r0 = hipEventRecordWithFlags(e0, s, hipEventRecordExternal);
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(1), 0, s, x, 100000);
            hipError_t r1 = hipEventRecordWithFlags(e1, s, hipEventRecordExternal);
            hipGraph_t g = nullptr;
            hipError_t re = hipStreamEndCapture(s, &g);
            hipGraphExec_t ex = nullptr;
            hipError_t ri = g ? hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) : hipErrorInvalidValue;
            hipError_t rl = ex ? hipGraphLaunch(ex, s) : hipErrorInvalidValue;
            hipStreamSynchronize(s);
            float ms = -1;
            hipError_t rt = hipEventElapsedTime(&ms, e0, e1);
            printf("mode %d flags %d: rec0 %s rec1 %s end %s inst %s launch %s elapsed %s %.3f ms\n", m, f, hipGetErrorName(r0),
                   hipGetErrorName(r1), hipGetErrorName(re), hipGetErrorName(ri), hipGetErrorName(rl), hipGetErrorName(rt), ms);
            (void)hipGetLastError();
        }
    return 0;
}
