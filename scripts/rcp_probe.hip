// Accuracy of 1/x on gfx950: v_rcp_f64 alone, + one Newton step, + two (the collide's recip),
// against the correctly rounded quotient, over x in the LBM density range and beyond.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
__global__ void k(const double* x, double* r0, double* r1, double* r2, double* q, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double v = x[i];
    double r = __builtin_amdgcn_rcp(v);
    r0[i] = r;
    double a = __builtin_fma(r, __builtin_fma(-v, r, 1.0), r);
    r1[i] = a;
    r2[i] = __builtin_fma(a, __builtin_fma(-v, a, 1.0), a);
    q[i] = 1.0 / v;
}
int main() {
    const int n = 1 << 22;
    std::vector<double> x(n);
    unsigned long long s = 12345;
    for (int i = 0; i < n; ++i) {
        s = s * 6364136223846793005ULL + 1442695040888963407ULL;
        double u = (double)(s >> 11) / 9007199254740992.0;
        x[i] = i < n / 2 ? 0.98 + 0.04 * u : std::ldexp(1.0 + u, (int)(u * 40) - 20);
    }
    double *dx, *d0, *d1, *d2, *dq;
    hipMalloc(&dx, n * 8); hipMalloc(&d0, n * 8); hipMalloc(&d1, n * 8); hipMalloc(&d2, n * 8); hipMalloc(&dq, n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dx, d0, d1, d2, dq, n);
    std::vector<double> r0(n), r1(n), r2(n), q(n);
    hipMemcpy(r0.data(), d0, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(r1.data(), d1, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(r2.data(), d2, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(q.data(), dq, n * 8, hipMemcpyDeviceToHost);
    double e[3] = {0, 0, 0};
    long ne[3] = {0, 0, 0};
    for (int i = 0; i < n; ++i) {
        const double ref = 1.0 / x[i];  // host IEEE division
        const double* rr[3] = {&r0[i], &r1[i], &r2[i]};
        for (int j = 0; j < 3; ++j) {
            const double ulp = std::nextafter(std::fabs(ref), INFINITY) - std::fabs(ref);
            const double eu = std::fabs(*rr[j] - ref) / ulp;
            if (eu > e[j]) e[j] = eu;
            if (*rr[j] != ref) ne[j]++;
        }
    }
    printf("rcp only: max %.3g ulp, %ld of %d differ\n", e[0], ne[0], n);
    printf("1 Newton: max %.3g ulp, %ld of %d differ\n", e[1], ne[1], n);
    printf("2 Newton: max %.3g ulp, %ld of %d differ\n", e[2], ne[2], n);
    return 0;
}
