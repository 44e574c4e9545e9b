// Phase timestamps of F (noise_block, csrc/noise.hip) per block, thread 0 (dev tool).
// Built by tools/micro/noise_micro.py into tools/micro/libnoise_probe.so (links libccrec_hip.so
// for cc::fail); noise_probe_fwd / noise_probe_adam run this copy of the kernels.
#include <hip/hip_runtime.h>
__device__ unsigned long long g_nprobe[1024 * 8];
#define NOISE_PROBE(b, k)                                                              \
  do {                                                                                 \
    if (threadIdx.x == 0 && (b) < 1024) g_nprobe[(b) * 8 + (k)] = wall_clock64();    \
  } while (0)
#include "noise.hip"

extern "C" int noise_probe_read(unsigned long long *host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_nprobe), (size_t)n * 8);
}
extern "C" int noise_probe_fwd(const cc_noise_args *a, void *stream) { return cc_noise_fwd(a, stream); }
