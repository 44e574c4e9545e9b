"""A/B of cc_dec_bce_dw between two library builds (dev tool).

  python tools/micro/d1_ab.py dump OUT.npz      # with CCREC_LIB=<lib>: outputs of every path
  python tools/micro/d1_ab.py cmp A.npz B.npz   # bit-identity of two dumps
  python tools/micro/d1_ab.py time              # with CCREC_LIB=<lib>: the bench shape, alone

Paths per shape: the Wo^T copy, the packed operand images, Wo read in place (LDS-DMA slices)."""
import os
import sys

import numpy as np

SHAPES = [(512, 256, 22000), (512, 256, 2504), (128, 128, 712), (256, 128, 22000), (512, 512, 2500),
          (128, 512, 700), (256, 256, 64), (512, 256, 2500)]


def _setup():
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
    from cubecobrarecommender_amd import _lib as L
    return torch, L


def _case(torch, L, B, d, V, seed=0):
    g = torch.Generator(device='cuda').manual_seed(seed + B + d + V)
    D3 = (torch.randn(B, d, device='cuda', generator=g) * 0.5).to(torch.bfloat16)
    D3t = D3.t().contiguous()
    WoT = (torch.randn(V, d, device='cuda', generator=g) * 0.1).to(torch.bfloat16)
    bo = torch.randn(V, device='cuda', generator=g) * 0.1
    VW = (V + 31) // 32
    yb = torch.randint(-2**31, 2**31 - 1, (B, VW), device='cuda', dtype=torch.int32, generator=g)
    D3p = D3.view(B // 32, 32, d // 16, 2, 8).permute(0, 2, 3, 1, 4).contiguous()
    D3tp = D3t.view(d // 32, 32, B // 16, 2, 8).permute(0, 2, 3, 1, 4).contiguous()
    Wo = WoT.t().contiguous()
    return dict(D3=D3, D3t=D3t, WoT=WoT, bo=bo, yb=yb, D3p=D3p, D3tp=D3tp, Wo=Wo, yimg=y_image(torch, yb))


def y_image(torch, yb):
    """cc_tower_args.y_img from y_bits [B][VW]: word-column major, rows of every 32-row block in
    accumulator-register order (dword 2r + h = row (r & 3) + 8 (r >> 2) + 4h)."""
    B = yb.shape[0]
    pos = torch.arange(32)
    row = 8 * (pos >> 3) + 4 * (pos & 1) + ((pos >> 1) & 3)
    idx = (torch.arange(B // 32)[:, None] * 32 + row[None, :]).reshape(-1).to(yb.device)
    return yb[idx].t().contiguous()


def _run(torch, L, c, B, d, V, mode, bufs=None):
    bf = dict(device='cuda', dtype=torch.bfloat16)
    if bufs is None:
        nblk = L.lib().cc_dec_bce_dw_blocks(V)
        bufs = dict(dZ=torch.zeros(B, V, **bf), gW=torch.full((d, V), 7.0, device='cuda'),
                    gb=torch.full((V,), 7.0, device='cuda'),
                    part=torch.zeros(nblk, device='cuda', dtype=torch.float64),
                    loss=torch.zeros(1, device='cuda', dtype=torch.float64),
                    tick=torch.zeros(1, device='cuda', dtype=torch.int32))
    pk = (None, None) if mode == 0 else (L.ptr(c['D3p']), L.ptr(c['D3tp']))
    wot, wo = (L.ptr(c['WoT']), None) if mode < 2 else (None, L.ptr(c['Wo']))
    if mode == 3:   # Wo in place + the target-mask image (the trainer's call)
        L.call('cc_dec_bce_dw_img', L.ptr(c['D3']), L.ptr(c['D3t']), B, pk[0], pk[1], wot, wo, L.ptr(c['bo']), B, d,
               V, L.ptr(c['yb']), L.ptr(c['yimg']), L.ptr(bufs['dZ']), V, L.ptr(bufs['gW']), L.ptr(bufs['gb']),
               L.ptr(bufs['part']), L.ptr(bufs['loss']), 1.0 / (B * V), L.ptr(bufs['tick']), L.stream_ptr())
        return bufs
    L.call('cc_dec_bce_dw', L.ptr(c['D3']), L.ptr(c['D3t']), B, pk[0], pk[1], wot, wo, L.ptr(c['bo']), B, d, V,
           L.ptr(c['yb']), L.ptr(bufs['dZ']), L.ptr(bufs['gW']), L.ptr(bufs['gb']), L.ptr(bufs['part']),
           L.ptr(bufs['loss']), 1.0 / (B * V), L.ptr(bufs['tick']), L.stream_ptr())
    return bufs


def dump(out):
    torch, L = _setup()
    res = {}
    for (B, d, V) in SHAPES:
        c = _case(torch, L, B, d, V)
        for mode in (0, 1, 2, 3):
            b = _run(torch, L, c, B, d, V, mode)
            torch.cuda.synchronize()
            k = f'{B}_{d}_{V}_{mode}'
            res[k + '_dZ'] = b['dZ'].view(torch.int16).cpu().numpy()
            res[k + '_gW'] = b['gW'].cpu().numpy()
            res[k + '_gb'] = b['gb'].cpu().numpy()
            res[k + '_loss'] = b['loss'].cpu().numpy()
    np.savez(out, **res)
    print('dumped', len(res), 'arrays to', out)


def cmp(a, b=None):
    """Two dumps, or (b None) every path of one dump against its mode-0 path."""
    A = np.load(a)
    Bz = np.load(b) if b else None
    bad = 0
    for k in A.files:
        if Bz is not None:
            x, y = A[k], Bz[k]
        else:
            base = k.split('_')
            base[3] = '0'
            x, y = A[k], A['_'.join(base)]
        if not np.array_equal(x, y):
            bad += 1
            xf, yf = x.astype(np.float64), y.astype(np.float64)
            print('DIFF', k, 'n=', int((x != y).sum()), 'max abs', float(np.max(np.abs(xf - yf))))
    print('compared', len(A.files), 'arrays,', bad, 'differ')
    return bad


def time_it():
    torch, L = _setup()
    B, d, V = 512, 256, 22000
    c = _case(torch, L, B, d, V)
    n = int(os.environ.get('N', '200'))
    for mode in (1, 2, 3):
        bufs = _run(torch, L, c, B, d, V, mode)
        for _ in range(5):
            _run(torch, L, c, B, d, V, mode, bufs)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            _run(torch, L, c, B, d, V, mode, bufs)
        e1.record()
        torch.cuda.synchronize()
        print(f'dec_bce_dw mode={mode} {e0.elapsed_time(e1) / n * 1000:.2f} us ({os.path.basename(L.LIB_PATH)})')


if __name__ == '__main__':
    if sys.argv[1] == 'dump':
        dump(sys.argv[2])
    elif sys.argv[1] == 'cmp':
        sys.exit(1 if cmp(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None) else 0)
    else:
        time_it()
