// xcc_probe.hip — which XCD (XCC) and CU run the workgroups of a CU-masked stream.
//
// Checks how hipExtStreamCreateWithCUMask's bit i maps to the hardware: bit i -> XCC i / 32
// (contiguous) or bit i -> XCC i % 8 (round-robin).  Each workgroup records HW_REG_XCC_ID and
// HW_REG_HW_ID (SE / SH / CU) with s_getreg; the host prints, per mask, the workgroups per XCC and
// the distinct CUs used per XCC.  Build: hipcc --offload-arch=gfx950 -O2 -o xcc_probe xcc_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdint>
#include <set>
#include <string>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void probe(uint32_t* out, int spin) {
    if (threadIdx.x == 0) {
        const uint32_t xcc = __builtin_amdgcn_s_getreg(0xF814);  // hwreg(HW_REG_XCC_ID, 0, 32)
        const uint32_t hw = __builtin_amdgcn_s_getreg(0xF804);   // hwreg(HW_REG_HW_ID, 0, 32)
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
    // keep the workgroup resident a little so the dispatcher spreads the grid
    long long t0 = clock64();
    while (clock64() - t0 < spin) {}
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int ncu = p.multiProcessorCount, words = (ncu + 31) / 32, nb = 16384;
    std::printf("device %s, %d CUs\n", p.gcnArchName, ncu);
    uint32_t* d = nullptr;
    CHECK(hipMalloc(&d, sizeof(uint32_t) * 2 * nb));
    std::vector<uint32_t> h(2 * nb);

    struct Case { std::string name; std::vector<uint32_t> mask; };
    std::vector<Case> cases;
    auto make = [&](const std::string& n, auto pick) {
        std::vector<uint32_t> m(words, 0u);
        for (int i = 0; i < ncu; ++i)
            if (pick(i)) m[i / 32] |= 1u << (i % 32);
        cases.push_back({n, m});
    };
    make("all", [&](int) { return true; });
    make("top32 (bits 224-255)", [&](int i) { return i >= ncu - 32; });
    make("bottom224 (bits 0-223)", [&](int i) { return i < ncu - 32; });
    make("bits = 7 mod 8", [&](int i) { return i % 8 == 7; });
    make("bits != 7 mod 8", [&](int i) { return i % 8 != 7; });
    make("bits 0-31", [&](int i) { return i < 32; });
    make("bit 0", [&](int i) { return i == 0; });
    make("bit 1", [&](int i) { return i == 1; });
    make("bit 8", [&](int i) { return i == 8; });

    for (const Case& cs : cases) {
        hipStream_t s;
        CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)cs.mask.size(), cs.mask.data()));
        CHECK(hipMemsetAsync(d, 0xff, sizeof(uint32_t) * 2 * nb, s));
        hipLaunchKernelGGL(probe, dim3(nb), dim3(64), 0, s, d, 20000);
        CHECK(hipGetLastError());
        CHECK(hipStreamSynchronize(s));
        CHECK(hipMemcpy(h.data(), d, sizeof(uint32_t) * 2 * nb, hipMemcpyDeviceToHost));
        CHECK(hipStreamDestroy(s));
        std::vector<long> per(16, 0);
        std::vector<std::set<uint32_t>> cus(16);
        for (int b = 0; b < nb; ++b) {
            const uint32_t x = h[2 * b] & 0xf, hw = h[2 * b + 1];
            const uint32_t cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
            per[x]++;
            cus[x].insert(se * 32 + sh * 16 + cu);
        }
        std::printf("%-24s wg/xcc:", cs.name.c_str());
        for (int x = 0; x < 8; ++x) std::printf(" %5ld", per[x]);
        std::printf("   cus/xcc:");
        for (int x = 0; x < 8; ++x) std::printf(" %2zu", cus[x].size());
        std::printf("\n");
    }
    CHECK(hipFree(d));
    return 0;
}
