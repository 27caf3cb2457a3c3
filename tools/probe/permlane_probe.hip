#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* p, int* q){
  int a = threadIdx.x, b = 1000 + threadIdx.x;
  auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  p[threadIdx.x] = r[0]; q[threadIdx.x] = r[1];
}
int main(){ int *p,*q; hipMalloc(&p,256); hipMalloc(&q,256); k<<<1,64>>>(p,q); int hp[64],hq[64]; hipMemcpy(hp,p,256,hipMemcpyDeviceToHost); hipMemcpy(hq,q,256,hipMemcpyDeviceToHost);
 for(int i=0;i<64;i++) printf("%d:%d,%d ", i,hp[i],hq[i]); printf("\n"); return 0; }
