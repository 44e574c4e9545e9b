// HBM read rate of the full-mode dZ stream shapes (dev tool): a [rows][V] bf16 matrix read by
//   slice  — block b owns columns [96 b, 96 b + 96) and walks every row (192-B pieces 2V B apart),
//            kl_dwo_kernel's pattern;
//   panel  — block b owns rows [128 b, ..) and walks 64-column k tiles (128-B pieces), dx_wide's;
//   tiled  — the same bytes laid out slice-major ([slice][rows][96]): block b streams one
//            contiguous region.
// Each thread loads 16 B per access with 4 loads in flight and folds them into one word.
// hipcc -O3 --offload-arch=gfx950 tools/micro/stride_bw.hip -o tools/micro/gpubin/stride_bw
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __attribute__((ext_vector_type(4))) unsigned int v4u;

__global__ __launch_bounds__(512) void slice_read(const char *z, int rows, int V, unsigned *out) {
  const int n0 = blockIdx.x * 96, tid = threadIdx.x;
  const int per_row = 12;                          // 16-B pieces per 192-B row piece
  const int rpi = 512 / per_row;                   // 42 rows per sweep (504 threads)
  unsigned acc = 0;
  if (tid < rpi * per_row) {
    const int r0 = tid / per_row, e = tid % per_row;
    for (int r = r0; r < rows; r += 4 * rpi) {
      v4u x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int rr = min(r + u * rpi, rows - 1);
        x[u] = *reinterpret_cast<const v4u *>(z + ((size_t)rr * V + n0) * 2 + e * 16);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc ^= x[u][0] ^ x[u][1] ^ x[u][2] ^ x[u][3];
    }
  }
  out[blockIdx.x * 512 + tid] = acc;
}

__global__ __launch_bounds__(512) void panel_read(const char *z, int rows, int V, unsigned *out) {
  const int m0 = blockIdx.x * 128, tid = threadIdx.x;   // 128 rows x 64 columns per k tile: 8 pieces per row
  const int r = tid / 8 + 0, e = tid % 8;               // 64 rows per sweep
  unsigned acc = 0;
  for (int k = 0; k < V; k += 64 * 4) {
    v4u x[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int kk = min(k + 64 * u, V - 64), rr = min(m0 + r + 64 * h, rows - 1);
        x[u][h] = *reinterpret_cast<const v4u *>(z + ((size_t)rr * V + kk) * 2 + e * 16);
      }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int h = 0; h < 2; ++h) acc ^= x[u][h][0] ^ x[u][h][1] ^ x[u][h][2] ^ x[u][h][3];
  }
  out[blockIdx.x * 512 + tid] = acc;
}

__global__ __launch_bounds__(512) void tiled_read(const char *z, size_t bytes_per_block, unsigned *out) {
  const char *base = z + (size_t)blockIdx.x * bytes_per_block;
  unsigned acc = 0;
  for (size_t o = (size_t)threadIdx.x * 16; o < bytes_per_block; o += 512 * 16 * 4) {
    v4u x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t oo = min(o + (size_t)u * 512 * 16, bytes_per_block - 16);
      x[u] = *reinterpret_cast<const v4u *>(base + oo);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc ^= x[u][0] ^ x[u][1] ^ x[u][2] ^ x[u][3];
  }
  out[blockIdx.x * 512 + threadIdx.x] = acc;
}

int main() {
  const int rows = 22016, V = 22000;
  const size_t bytes = (size_t)rows * V * 2;
  char *z;
  unsigned *out;
  (void)hipMalloc(&z, bytes + 4096);
  (void)hipMalloc(&out, 4096 * 512 * 4);
  (void)hipMemset(z, 1, bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    float ms;
    const int nsl = (V + 95) / 96;
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(slice_read, dim3(nsl), dim3(512), 0, nullptr, z, rows, V, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("slice (%d blocks, 192-B pieces): %.1f us, %.2f TB/s\n", nsl, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(panel_read, dim3(rows / 128), dim3(512), 0, nullptr, z, rows, V, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("panel (%d blocks, 128-B pieces): %.1f us, %.2f TB/s\n", rows / 128, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    for (int nb : {230, 256, 1024}) {
      const size_t per = bytes / nb / 16 * 16;
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(tiled_read, dim3(nb), dim3(512), 0, nullptr, z, per, out);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("tiled (%d blocks, contiguous): %.1f us, %.2f TB/s\n", nb, ms * 1e3, per * nb / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
