// Probe: semantics of v_permlane16/32_swap builtins and DPP row_newbcast on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
template<int K> __device__ __forceinline__ void fmac_nb(float& acc, float x, float w){
  asm volatile("s_nop 4\n\tv_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(x), "v"(w), "i"(K));
}
__global__ void k(float* out){
  int j = threadIdx.x;
  float x = (float)j;
  auto a = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(int,x), __builtin_bit_cast(int,x + 1000.f), false, false);
  auto p0 = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(int,x), __builtin_bit_cast(int,x + 1000.f), false, false);
  out[j] = __builtin_bit_cast(float,a[0]); out[64+j] = __builtin_bit_cast(float,a[1]);
  out[128+j] = __builtin_bit_cast(float,p0[0]); out[192+j] = __builtin_bit_cast(float,p0[1]);
  float acc = 0.f; fmac_nb<5>(acc, x, 1.0f); out[256+j] = acc;
  float acc2 = 0.f; fmac_nb<15>(acc2, x, 2.0f); out[320+j] = acc2;
}
int main(){
  float* d; hipMalloc(&d, 384*4); hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  float h[384]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[6] = {"p32.vdst(x, x+1000)", "p32.src", "p16.vdst(x,x+1000)", "p16.src", "newbcast5*1", "newbcast15*2"};
  for (int r=0;r<6;r++){ printf("%s:", names[r]); for(int i=0;i<64;i++) printf(" %g", h[r*64+i]); printf("\n"); }
  return 0;
}
