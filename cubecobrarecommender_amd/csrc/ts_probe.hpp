// Wall-clock launch probe (dev builds only, -DCCREC_TS_PROBE=1; compiled out by default): the
// first block's start / the last block's end of a kernel, per training step, from s_memrealtime
// (100 MHz), so that the idle time between two launches of a replayed graph can be read without a
// profiler attached (tools/micro/gap_probe.py).  Slots are the device step counter mod 1024.
#pragma once
#ifndef CCREC_TS_PROBE
#define CCREC_TS_PROBE 0
#endif
#if CCREC_TS_PROBE
#define TS_PROBE_DEFINE(tag)                                                                          \
  __device__ unsigned long long ts_first_##tag[1024];                                                 \
  __device__ unsigned long long ts_last_##tag[1024];                                                  \
  extern "C" int cc_ts_dump_##tag(unsigned long long *first, unsigned long long *last) {              \
    if (hipMemcpyFromSymbol(first, HIP_SYMBOL(ts_first_##tag), sizeof(ts_first_##tag)) != hipSuccess) \
      return 1;                                                                                       \
    if (hipMemcpyFromSymbol(last, HIP_SYMBOL(ts_last_##tag), sizeof(ts_last_##tag)) != hipSuccess)    \
      return 1;                                                                                       \
    return 0;                                                                                         \
  }
#define TS_PROBE_FIRST(tag, slot) \
  if (blockIdx.x == 0 && threadIdx.x == 0) ts_first_##tag[(slot) & 1023] = wall_clock64()
#define TS_PROBE_LAST(tag, slot) \
  if (threadIdx.x == 0) atomicMax(&ts_last_##tag[(slot) & 1023], (unsigned long long)wall_clock64())
#else
#define TS_PROBE_DEFINE(tag)
#define TS_PROBE_FIRST(tag, slot)
#define TS_PROBE_LAST(tag, slot)
#endif
