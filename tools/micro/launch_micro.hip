// Launch-overhead / grid-sync microbenchmark (dev tool).
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <cstdio>
namespace cg = cooperative_groups;
__global__ void empty_kernel(int *p) { if (p && threadIdx.x == 9999) p[0] = 1; }
__global__ void dep_kernel(int *p) {  // one dependent global round trip
  int v = p[blockIdx.x];
  if (threadIdx.x == 0) p[blockIdx.x] = v + 1;
}
__global__ void coop_kernel(int *p, int iters) {
  cg::grid_group g = cg::this_grid();
  for (int i = 0; i < iters; ++i) {
    if (threadIdx.x == 0) p[blockIdx.x] += 1;
    g.sync();
  }
}
int main() {
  int *p; (void)hipMalloc(&p, 1 << 20); (void)hipMemset(p, 0, 1 << 20);
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  float ms;
  for (int grid : {1, 32, 256}) {
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipEventRecord(a);
      for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, 0, p);
      (void)hipEventRecord(b); (void)hipEventSynchronize(b); (void)hipEventElapsedTime(&ms, a, b);
      printf("empty grid=%d: %.2f us/kernel\n", grid, ms * 1000 / 200);
      (void)hipEventRecord(a);
      for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(dep_kernel, dim3(grid), dim3(256), 0, 0, p);
      (void)hipEventRecord(b); (void)hipEventSynchronize(b); (void)hipEventElapsedTime(&ms, a, b);
      printf("dep   grid=%d: %.2f us/kernel\n", grid, ms * 1000 / 200);
    }
  }
  for (int grid : {32, 256}) {
    for (int iters : {1, 101}) {
      void *args[] = {&p, &iters};
      for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(a);
        for (int i = 0; i < 20; ++i)
          (void)hipLaunchCooperativeKernel((void *)coop_kernel, dim3(grid), dim3(256), args, 0, 0);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b); (void)hipEventElapsedTime(&ms, a, b);
        printf("coop grid=%d iters=%d: %.2f us/launch\n", grid, iters, ms * 1000 / 20);
      }
    }
  }
  printf("err %s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
