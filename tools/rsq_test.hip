#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
__device__ __forceinline__ double rsqrt_nr(double x) {
    double y = __builtin_amdgcn_rsq(x);
    const double h = 0.5 * x;
    y = fma(y, fma(-h * y, y, 0.5), y);
    y = fma(y, fma(-h * y, y, 0.5), y);
    return y;
}
__device__ __forceinline__ double rsqrt_nr1(double x) {
    double y = __builtin_amdgcn_rsq(x);
    const double h = 0.5 * x;
    return fma(y, fma(-h * y, y, 0.5), y);
}
__global__ void k(const double* x, double* a, double* b, double* c, double* d, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { a[i] = rsqrt_nr(x[i]); b[i] = 1.0 / sqrt(x[i]); c[i] = __builtin_amdgcn_rsq(x[i]); d[i] = rsqrt_nr1(x[i]); }
}
int main() {
    const int n = 1 << 20;
    double *x, *a, *b, *c, *d1;
    hipMallocManaged(&x, n * 8); hipMallocManaged(&a, n * 8); hipMallocManaged(&b, n * 8); hipMallocManaged(&c, n * 8);
    hipMallocManaged(&d1, n * 8);
    unsigned long long s = 88172645463325252ull;
    for (int i = 0; i < n; ++i) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; double u = (s >> 11) * (1.0 / 9007199254740992.0);
        x[i] = std::ldexp(0.5 + u, (int)(s % 200) - 100); }
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, x, a, b, c, d1, n);
    hipDeviceSynchronize();
    double ea = 0, ec = 0, ed = 0; long ulpa = 0, ulpd = 0;
    for (int i = 0; i < n; ++i) {
        double r = b[i];
        ea = fmax(ea, fabs(a[i] - r) / r); ec = fmax(ec, fabs(c[i] - r) / r);
        long d = std::llabs(*(long*)&a[i] - *(long*)&r); if (d > ulpa) ulpa = d;
        ed = fmax(ed, fabs(d1[i] - r) / r);
        long dd = std::llabs(*(long*)&d1[i] - *(long*)&r); if (dd > ulpd) ulpd = dd;
    }
    printf("rsqrt_nr max rel err %.3e (max ulps %ld), raw v_rsq %.3e, one Newton step %.3e (max ulps %ld)\n", ea, ulpa, ec, ed, ulpd);
    return 0;
}
