// wait_probe.hip — what the slab hand-off's bounded device waits rely on (round 6):
//  1. wall_clock64() (s_memrealtime) ticks per second against hipDeviceAttributeWallClockRate and the
//     host clock, across a host-timed hold;
//  2. a one-wave kernel that polls a host-coherent word which a host thread sets after `ms`
//     (the test hold of ctx_step.hip:exchange), bounded by a wall-clock deadline;
//  3. hipStreamWaitValue32 on the same kind of word (a queue-level hold, no wave).
// Build: hipcc -O2 --offload-arch=gfx950 -o scripts/bin/wait_probe scripts/wait_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                      \
            return 1;                                                                \
        }                                                                            \
    } while (0)

__global__ void hold_kernel(const unsigned* word, unsigned long long limit, unsigned long long* out) {
    const unsigned long long t0 = wall_clock64();
    unsigned long long t = t0;
    unsigned polls = 0;
    for (;;) {
        const unsigned w = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        t = wall_clock64();
        ++polls;
        if (w != 0 || t - t0 > limit) break;
        __builtin_amdgcn_s_sleep(127);
    }
    if (threadIdx.x == 0) {
        out[0] = t0;
        out[1] = t;
        out[2] = polls;
    }
}

int main(int argc, char** argv) {
    const int ms = argc > 1 ? std::atoi(argv[1]) : 500;
    int rate_khz = 0;
    CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
    unsigned* word = nullptr;
    CK(hipHostMalloc((void**)&word, 64, hipHostMallocCoherent));
    unsigned long long* out = nullptr;
    CK(hipHostMalloc((void**)&out, 64, hipHostMallocCoherent));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

    // 1 + 2: the wave hold
    *word = 0;
    const unsigned long long limit = (unsigned long long)rate_khz * 1000ull * 10ull;  // 10 s
    auto h0 = std::chrono::steady_clock::now();
    hold_kernel<<<1, 64, 0, s>>>(word, limit, out);
    std::thread rel([&] {
        std::this_thread::sleep_for(std::chrono::milliseconds(ms));
        __atomic_store_n(word, 1u, __ATOMIC_RELEASE);
    });
    CK(hipStreamSynchronize(s));
    const double host_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - h0).count();
    rel.join();
    const double dev_ticks = (double)(out[1] - out[0]);
    std::printf("{\"probe\": \"wave_hold\", \"ms\": %d, \"wall_clock_rate_khz\": %d, \"host_s\": %.4f, "
                "\"dev_ticks\": %.0f, \"ticks_per_host_s\": %.4e, \"polls\": %llu}\n",
                ms, rate_khz, host_s, dev_ticks, dev_ticks / host_s, out[2]);

    // 3: the queue hold
    *word = 0;
    void* dword = nullptr;
    CK(hipHostGetDevicePointer(&dword, word, 0));
    h0 = std::chrono::steady_clock::now();
    hipError_t e = hipStreamWaitValue32(s, dword, 1, hipStreamWaitValueGte, 0xffffffffu);
    std::printf("{\"probe\": \"queue_hold_submit\", \"err\": \"%s\"}\n", hipGetErrorString(e));
    hold_kernel<<<1, 64, 0, s>>>(word, limit, out);  // returns at once once the wait is released
    std::thread rel2([&] {
        std::this_thread::sleep_for(std::chrono::milliseconds(ms));
        __atomic_store_n(word, 1u, __ATOMIC_RELEASE);
    });
    CK(hipStreamSynchronize(s));
    rel2.join();
    std::printf("{\"probe\": \"queue_hold\", \"host_s\": %.4f}\n",
                std::chrono::duration<double>(std::chrono::steady_clock::now() - h0).count());
    return 0;
}
