// C-ABI plumbing of libccrec_hip.so: version, thread-local error strings, parameter layout.
#include <hip/hip_runtime.h>

#include <string>

#include "common.hpp"

namespace cc {
static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }
int fail(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}

// Flat layout in Keras creation order (model.py:27-33 encoder, :58-64 decoder, :92-98 the two
// decoders).  Every tensor starts on a 64-element (256 B) boundary so kernels can use 16-byte
// vector accesses on any slice.
int param_offsets(int V, int d, int64_t *off, int64_t *size, int64_t *total, int64_t *main_total) {
  if (V <= 0 || d <= 0) return fail(CC_ERR_ARG, "cc_param_layout: V and d must be positive");
  const int64_t shapes[12][2] = {
      {V, d},   {d, 256}, {256, 128}, {128, 64},  // encoder e1, e2, e3, bottleneck
      {64, 128}, {128, 256}, {256, d}, {d, V},    // decoder (D1) d1, d2, d3, reconstruct
      {64, 128}, {128, 256}, {256, d}, {d, V}};   // decoder_for_reg (D2)
  int64_t o = 0;
  for (int l = 0; l < 12; ++l) {
    const int64_t kn = shapes[l][0] * shapes[l][1], bn = shapes[l][1];
    off[2 * l] = o;
    size[2 * l] = kn;
    o += (kn + 63) / 64 * 64;
    off[2 * l + 1] = o;
    size[2 * l + 1] = bn;
    o += (bn + 63) / 64 * 64;
    if (l == 7) *main_total = o;
  }
  *total = o;
  return CC_OK;
}
}  // namespace cc

extern "C" int cc_abi_version(void) { return CC_ABI_VERSION; }

// SHA-256 prefix of the sources this library was compiled from (build.py -> buildid.py); the
// Python side refuses a library whose id differs from the tree's sources.
#ifndef CC_BUILD_ID
#define CC_BUILD_ID "unknown"
#endif
extern "C" const char *cc_build_id(void) { return CC_BUILD_ID; }

extern "C" const char *cc_last_error_string(void) { return cc::g_last_error.c_str(); }

extern "C" int cc_param_layout(int32_t V, int32_t d, int64_t *offsets, int64_t *sizes,
                               int64_t *total, int64_t *main_total) {
  if (!offsets || !sizes || !total || !main_total)
    return cc::fail(CC_ERR_ARG, "cc_param_layout: null pointer");
  return cc::param_offsets(V, d, offsets, sizes, total, main_total);
}
