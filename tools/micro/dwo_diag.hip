// kl_dwo_kernel and kl_dwo2_kernel alone at the full-mode shape (rows = 22,016, d = 256, V = 22,000), built with one
// DWO_DIAG mask (decreg.hip: 1 no MFMA, 2 no B reads, 4 no dZ loads, 8 no A loads) to split its time
// between its streams, and DW2_DIAG the same for kl_dwo2_kernel (2 no MFMA, 4 no dZ DMA, 8 no A
// loads; its halves' sum kernel timed apart) (dev tool; the outputs of a masked build are meaningless).
// for m in 0 1 2 4 8 3 12; do hipcc -O3 -std=c++17 --offload-arch=gfx950 -DDWO_DIAG=$m -I include \
//   -I cubecobrarecommender_amd/csrc tools/micro/dwo_diag.hip cubecobrarecommender_amd/csrc/api.cpp \
//   cubecobrarecommender_amd/csrc/host_util.cpp -o tools/micro/gpubin/dwo_diag_$m; done
#include "decreg.hip"

#include <cstdio>

int main() {
  const int V = 22000, d = 256, rows = 22016, B = 512, R = B + rows;
  void *D3tp, *dZ, *gW, *part;
  (void)hipMalloc(&part, (size_t)d * V * 4);
  (void)hipMalloc(&D3tp, (size_t)R * d * 2);
  (void)hipMalloc(&dZ, (size_t)rows * V * 2);
  (void)hipMalloc(&gW, (size_t)d * V * 4);
  (void)hipMemset(D3tp, 0x3c, (size_t)R * d * 2);
  (void)hipMemset(dZ, 0x3c, (size_t)rows * V * 2);   // finite nonzero bf16
  KlP p{};
  p.d = d; p.V = V; p.rows = rows; p.ldt = R; p.row0 = B;
  p.D3tp = (const bf16_t *)D3tp; p.dZ = (bf16_t *)dZ; p.gW = (float *)gW;
  p.dw_part = (float *)part;
  (void)hipFuncSetAttribute((const void *)kl_dwo2_kernel<256>, hipFuncAttributeMaxDynamicSharedMemorySize, DW2_LDS);
  const dim3 gd((unsigned)((V + DW_NB - 1) / DW_NB), 1);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int k = 0; k < 3; ++k) {
  float best = 1e9f, sum = 0.f;
  for (int rep = 0; rep < 12; ++rep) {
    (void)hipEventRecord(e0);
    if (k == 0)
      hipLaunchKernelGGL((kl_dwo_kernel<256, true>), gd, dim3(NTH), 0, nullptr, p);
    else if (k == 1)
      hipLaunchKernelGGL((kl_dwo2_kernel<256>), dim3((V + DW2_NB - 1) / DW2_NB, DW2_SPLIT), dim3(DW2_NT), DW2_LDS, nullptr, p);
    else
      hipLaunchKernelGGL(kl_dwo2_sum_kernel, dim3(1024), dim3(256), 0, nullptr, (const float4 *)part, (float4 *)gW,
                         (int64_t)d * V / 4);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep >= 2) { best = ms < best ? ms : best; sum += ms; }
  }
  printf("DWO_DIAG %d DW2_DIAG %d: %s best %.1f us, mean %.1f us (%s)\n", DWO_DIAG, DW2_DIAG,
         k == 2 ? "kl_dwo2_sum_kernel" : k ? "kl_dwo2_kernel" : "kl_dwo_kernel", best * 1e3, sum * 1e2, hipGetErrorString(hipGetLastError()));
  }
  return 0;
}
