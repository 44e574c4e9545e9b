// Microbenchmark for cc_topn (dev tool; not part of the library).
// Build: hipcc -O3 --offload-arch=gfx950 -Iinclude -Icubecobrarecommender_amd/csrc tools/micro/topn_micro.hip -o tools/micro/topn_micro
#include "../../cubecobrarecommender_amd/csrc/topn.hip"
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
namespace cc {
void set_error(const std::string &) {}
int fail(int code, const std::string &m) { fprintf(stderr, "%s\n", m.c_str()); return code; }
}  // namespace cc
int main(int argc, char **argv) {
  int V = argc > 1 ? atoi(argv[1]) : 20884;
  int amount = argc > 2 ? atoi(argv[2]) : 30000;
  std::mt19937 g(1);
  std::vector<float> p(V);
  for (auto &x : p) x = std::ldexp((float)(g() % 100000) / 100000.f + 0.5f, -(int)(g() % 14));
  std::vector<int> cube;
  for (int i = 0; i < 360; ++i) cube.push_back((int)(g() % V));
  std::sort(cube.begin(), cube.end());
  cube.erase(std::unique(cube.begin(), cube.end()), cube.end());
  float *dp, *av, *cv; int *ci, *ad, *na, *ord; void *ws;
  (void)hipMalloc(&dp, V * 4); (void)hipMalloc(&av, V * 4); (void)hipMalloc(&cv, V * 4);
  (void)hipMalloc(&ci, V * 4); (void)hipMalloc(&ad, V * 4); (void)hipMalloc(&na, 4);
  (void)hipMalloc(&ord, V * 4); (void)hipMalloc(&ws, cc_topn_workspace_size(V));
  (void)hipMemcpy(dp, p.data(), V * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(ci, cube.data(), cube.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  for (int variant = 0; variant < 2; ++variant) {
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(a);
      for (int i = 0; i < 20; ++i)
        cc_topn(dp, V, ci, (int)cube.size(), amount, ad, na, av, cv, variant ? ord : nullptr, ws, nullptr);
      (void)hipEventRecord(b); (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b);
      printf("V=%d amount=%d path=%s avg %.1f us\n", V, amount, variant ? "full" : "tiled", ms * 1000 / 20);
    }
  }
  int k; (void)hipMemcpy(&k, na, 4, hipMemcpyDeviceToHost);
  printf("n_add %d err %s\n", k, hipGetErrorString(hipGetLastError()));
  return 0;
}
