// api_probe.hip — host cost of the HIP calls a band cycle makes (gfx950, one GPU): kernel launch
// (<<<>>> and hipExtLaunchKernelGGL with a stop event), hipEventRecord, hipStreamWaitEvent and a
// small hipMemcpyAsync D2D, each timed on the host over N calls while the GPU is kept busy, so that
// submission never waits for completion.  Build: hipcc --offload-arch=gfx950 -O2 -o scripts/bin/api_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void tiny(int* p) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && p) p[0] += 1;
}
__global__ void busy(long spin) {
    const long t0 = clock64();
    while (clock64() - t0 < spin) {
    }
}

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            return 1;                                                      \
        }                                                                  \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const int N = 2000;
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t ev[8];
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
    int* d = nullptr;
    char *a = nullptr, *b = nullptr;
    CK(hipMalloc(&d, 64));
    CK(hipMalloc(&a, 1 << 20));
    CK(hipMalloc(&b, 1 << 20));
    for (int rep = 0; rep < 2; ++rep) {
        // keep the GPU busy (~50 ms) so that every call below is pure submission
        busy<<<1, 64, 0, s>>>(100000000L);
        double t = now();
        for (int i = 0; i < N; ++i) tiny<<<64, 256, 0, s>>>(d);
        const double launch = (now() - t) / N;
        t = now();
        for (int i = 0; i < N; ++i) hipExtLaunchKernelGGL(tiny, dim3(64), dim3(256), 0, s, nullptr, ev[i & 7], 0, d);
        const double ext = (now() - t) / N;
        t = now();
        for (int i = 0; i < N; ++i) CK(hipEventRecord(ev[i & 7], s));
        const double rec = (now() - t) / N;
        t = now();
        for (int i = 0; i < N; ++i) CK(hipStreamWaitEvent(s2, ev[i & 7], 0));
        const double wait = (now() - t) / N;
        t = now();
        for (int i = 0; i < N; ++i) CK(hipMemcpyAsync(b, a, 65536, hipMemcpyDeviceToDevice, s));
        const double cpy = (now() - t) / N;
        CK(hipDeviceSynchronize());
        printf("rep %d: launch %.2f us, ext launch + stop event %.2f us, event record %.2f us, stream wait %.2f us, "
               "memcpy D2D 64 KiB %.2f us\n",
               rep, launch * 1e6, ext * 1e6, rec * 1e6, wait * 1e6, cpy * 1e6);
    }
    return 0;
}
