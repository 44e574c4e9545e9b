// dx_wide_kernel alone at the full-mode shape (dX = dZ Wo^T: M = 22,016 rows, N = d = 256,
// K = |V| = 22,000, 4 splits), built with one DXW_DIAG mask (dxgemm.hip: 1 no Wo copies, 2 no dZ
// copies, 4 no MFMA) to split its time between its streams (dev tool; masked outputs are meaningless).
// hipcc -O3 -std=c++17 --offload-arch=gfx950 -DDXW_DIAG=0 -I include -I cubecobrarecommender_amd/csrc \
//   tools/micro/dx_diag.hip cubecobrarecommender_amd/csrc/api.cpp cubecobrarecommender_amd/csrc/host_util.cpp -o tools/micro/gpubin/dx_diag_0
#include "dxgemm.hip"

#include <cstdio>

int main(int argc, char **argv) {
  const int M = 22016, N = 256, K = 22000, splits = argc > 1 ? atoi(argv[1]) : 4;
  const bool pk = argc > 2 && atoi(argv[2]) != 0;   // B from its packed fragment image (cc_gemm_dx_splitk_pk)
  void *A, *B, *P, *Bp;
  (void)hipMalloc(&Bp, cc_pack_frag_b_size(N, K));
  (void)hipMalloc(&A, (size_t)M * K * 2);
  (void)hipMalloc(&B, (size_t)N * K * 2);
  (void)hipMalloc(&P, (size_t)splits * M * N * 4);
  (void)hipMemset(A, 0x3c, (size_t)M * K * 2);   // finite nonzero bf16
  (void)hipMemset(B, 0x3c, (size_t)N * K * 2);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e9f, sum = 0.f;
  for (int rep = 0; rep < 12; ++rep) {
    (void)hipEventRecord(e0);
    if (pk && rep == 0) (void)cc_pack_frag_b(B, N, K, K, Bp, nullptr);
    const int rc = pk ? cc_gemm_dx_splitk_pk(A, K, Bp, M, N, K, splits, (float *)P, nullptr)
                      : cc_gemm_dx_splitk(A, K, B, K, M, N, K, splits, (float *)P, nullptr);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rc != 0) printf("rc %d\n", rc);
    if (rep >= 2) { best = ms < best ? ms : best; sum += ms; }
  }
  printf("DXW_DIAG %d splits %d packed %d: dx_wide best %.1f us, mean %.1f us (%s)\n", DXW_DIAG, splits, (int)pk, best * 1e3, sum * 1e2,
         hipGetErrorString(hipGetLastError()));
  return 0;
}
