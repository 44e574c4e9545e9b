"""Time the transposing MX-FP8 quantiser alone on config 5's decoder weight (d x V bf16 -> V x d
fp8 + scales) and on the D3 transpose (dev tool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from cubecobrarecommender_amd import _lib as L  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    s = L.stream_ptr()
    for rows, cols, ld in ((1024, 22000, 1024), (2048, 1024, 2048), (256, 22000, 256)):
        src = torch.randn(rows, cols, device='cuda').to(torch.bfloat16)
        dst = torch.zeros(cols, ld, device='cuda', dtype=torch.uint8)
        sc = torch.zeros(cols, ld // 32, device='cuda', dtype=torch.uint8)
        us = timeit(lambda: L.call('cc_quant_mx8', L.CC_BF16, L.ptr(src), rows, cols, cols, 1, L.ptr(dst), ld,
                                   L.ptr(sc), None, s))
        mb = (rows * cols * 2 + cols * ld * 33 / 32) / 1e6
        print(f'quant_t {rows}x{cols} -> ld {ld}: {us:.1f} us  {mb / us:.2f} TB/s', flush=True)


if __name__ == '__main__':
    main()
