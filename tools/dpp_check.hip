#include <hip/hip_runtime.h>
__device__ __forceinline__ double dpp_d(double v, int ctrl_dummy);
template <int CTRL>
__device__ __forceinline__ double dppx(double v) {
  int2 a = __builtin_bit_cast(int2, v);
  a.x = __builtin_amdgcn_update_dpp(0, a.x, CTRL, 0xF, 0xF, false);
  a.y = __builtin_amdgcn_update_dpp(0, a.y, CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, a);
}
__device__ __forceinline__ double swap16(double v) {
  int2 a = __builtin_bit_cast(int2, v);
  auto r0 = __builtin_amdgcn_permlane16_swap(a.x, a.x, false, false);
  auto r1 = __builtin_amdgcn_permlane16_swap(a.y, a.y, false, false);
  int2 o; o.x = r0[0]; o.y = r1[0];   // which half? test
  return __builtin_bit_cast(double, o);
}
__device__ __forceinline__ double swap32(double v) {
  int2 a = __builtin_bit_cast(int2, v);
  auto r0 = __builtin_amdgcn_permlane32_swap(a.x, a.x, false, false);
  auto r1 = __builtin_amdgcn_permlane32_swap(a.y, a.y, false, false);
  int2 o; o.x = r0[0]; o.y = r1[0];
  return __builtin_bit_cast(double, o);
}
__global__ void k(const double* in, double* out) {
  int l = threadIdx.x;
  double v = in[l];
  out[l] = dppx<0xB1>(v);
  out[64 + l] = dppx<0x4E>(v);
  out[128 + l] = dppx<0x141>(v);
  out[192 + l] = dppx<0x140>(v);
  out[256 + l] = swap16(v);
  out[320 + l] = swap32(v);
}
int main() {
  double *d_in, *d_out, h[64], o[384];
  for (int i = 0; i < 64; ++i) h[i] = i;
  hipMalloc(&d_in, 512); hipMalloc(&d_out, 384*8);
  hipMemcpy(d_in, h, 512, hipMemcpyHostToDevice);
  k<<<1,64>>>(d_in, d_out);
  hipMemcpy(o, d_out, 384*8, hipMemcpyDeviceToHost);
  const char* nm[] = {"xor1","xor2","halfmirror","mirror","swap16","swap32"};
  for (int t = 0; t < 6; ++t) { printf("%s:", nm[t]); for (int i = 0; i < 64; ++i) printf(" %d", (int)o[t*64+i]); printf("\n"); }
  return 0;
}
