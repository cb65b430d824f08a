// Unit check of the V_MFMA_F64_16X16X4F64 lane maps gram_mfma relies on
// (csrc/ntm_device.h): lane l supplies A(l & 15, l >> 4) and B(l >> 4, l & 15);
// D(row (l >> 4) + 4 i, col l & 15) comes back in element i.  Exact integer data,
// so the product must match bit for bit.   hipcc --offload-arch=gfx950 -o /tmp/mc tools/mfma_f64_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(const double* A, const double* B, double* D) {
    const int l = threadIdx.x;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) * 4 + (l >> 4)], B[(l >> 4) * 16 + (l & 15)], acc, 0, 0, 0);
    for (int i = 0; i < 4; ++i) D[((l >> 4) + 4 * i) * 16 + (l & 15)] = acc[i];
}
int main() {
    double A[64], B[64], D[256], R[256];
    for (int i = 0; i < 64; ++i) { A[i] = (i * 7) % 13 - 6; B[i] = (i * 5) % 11 - 5; }
    for (int m = 0; m < 16; ++m)
        for (int n = 0; n < 16; ++n) {
            double s = 0;
            for (int kk = 0; kk < 4; ++kk) s += A[m * 4 + kk] * B[kk * 16 + n];
            R[m * 16 + n] = s;
        }
    double *dA, *dB, *dD;
    if (hipMalloc(&dA, sizeof A) || hipMalloc(&dB, sizeof B) || hipMalloc(&dD, sizeof D)) return 2;
    hipMemcpy(dA, A, sizeof A, hipMemcpyHostToDevice);
    hipMemcpy(dB, B, sizeof B, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    hipMemcpy(D, dD, sizeof D, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += D[i] != R[i];
    printf("mfma_f64_16x16x4 lane map: %s (%d of 256 entries differ)\n", bad ? "WRONG" : "ok", bad);
    return bad ? 1 : 0;
}
