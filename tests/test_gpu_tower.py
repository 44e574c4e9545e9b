"""GPU: fused tower kernels (tower.hip) vs a numpy restatement of the same layer chain."""
import ctypes

import numpy as np
import pytest
import torch

from cubecobrarecommender_amd import _lib as L
from tests.gpu_helpers import rel_err

pytestmark = pytest.mark.gpu


def _dims(d):
    return [(d, 256), (256, 128), (128, 64), (64, 128), (128, 256), (256, d)]


@pytest.mark.parametrize('dtype', [L.CC_F32, L.CC_BF16])
@pytest.mark.parametrize('d,B,R', [(64, 32, 64), (256, 64, 128), (256, 64, 64), (64, 32, 32), (512, 64, 128),
                                   (1024, 64, 128)])
def test_tower_fwd_bwd_vs_numpy(dtype, d, B, R):
    if dtype == L.CC_F32 and d > 256:
        pytest.skip('fp32 fused towers cover d <= 256')
    rng = np.random.default_rng(d + R)
    tdt = torch.bfloat16 if dtype == L.CC_BF16 else torch.float32
    rnd = lambda *s: torch.from_numpy((rng.standard_normal(s) * 0.2).astype(np.float32)).to('cuda', tdt)
    dims = _dims(d)
    W = [rnd(*dims[l if l < 6 else l - 3]) for l in range(9)]
    Wt = [torch.zeros(w.shape[1], w.shape[0], device='cuda', dtype=tdt) for w in W]
    bias = [torch.from_numpy(rng.standard_normal(w.shape[1]).astype(np.float32) * 0.1).cuda() for w in W]
    widths = [d, 256, 128, 64, 128, 256, d]
    act = [rnd(R, widths[0])] + [torch.zeros(R, w, device='cuda', dtype=tdt) for w in widths[1:]]
    gD3 = rnd(R, d)
    gact = [torch.zeros(R, w, device='cuda', dtype=tdt) for w in (256, 128, 64, 128, 256)]
    gpre1 = torch.zeros(R, d, device='cuda')
    slab = torch.zeros((R // 32) * int(L.lib().cc_tower_slab_elems(d)), device='cuda')
    gw = [torch.zeros(w.shape, device='cuda') for w in W]
    gb = [torch.zeros(w.shape[1], device='cuda') for w in W]
    t = L.TowerArgs(dtype=dtype, d=d, B=B, R=R)
    for l in range(9):
        t.w[l], t.wt[l], t.b[l] = W[l].data_ptr(), Wt[l].data_ptr(), bias[l].data_ptr()
        t.gw[l], t.gb[l] = gw[l].data_ptr(), gb[l].data_ptr()
    for a in range(7):
        t.act[a] = act[a].data_ptr()
    t.gD3, t.gpre1, t.slab = gD3.data_ptr(), gpre1.data_ptr(), slab.data_ptr()
    for a in range(5):
        t.gact[a] = gact[a].data_ptr()
    s = L.stream_ptr()
    for fn in ('cc_tower_transpose', 'cc_tower_fwd', 'cc_tower_bwd', 'cc_tower_reduce'):
        L.call(fn, ctypes.byref(t), s)
    torch.cuda.synchronize()
    f = lambda x: x.double().cpu().numpy()
    q = (lambda a: torch.from_numpy(np.asarray(a, np.float32)).to(tdt).double().numpy())
    for l in range(9 if R > B else 6):
        assert np.array_equal(f(Wt[l]), f(W[l]).T), f'transpose {l}'
    # forward
    h = f(act[0])
    errs = {}
    acts = [h]
    for i in range(6):
        rows_l = [(np.arange(R) < B), (np.arange(R) >= B)]
        out = np.zeros((R, widths[i + 1]))
        for br, rows in enumerate(rows_l):
            l = i if i < 3 else i + 3 * br
            if rows.any():
                out[rows] = q(np.maximum(h[rows] @ f(W[l]) + f(bias[l]), 0))
        errs[f'act{i + 1}'] = rel_err(f(act[i + 1]), out)
        h = f(act[i + 1])          # continue from the GPU's own activations
        acts.append(h)
    # backward
    g = f(gD3)
    gW = [np.zeros(w.shape) for w in W]
    gB = [np.zeros(w.shape[1]) for w in W]
    for i in range(5, -1, -1):
        H = acts[i]
        dX = np.zeros((R, widths[i]))
        for br, rows in enumerate([(np.arange(R) < B), (np.arange(R) >= B)]):
            l = i if i < 3 else i + 3 * br
            if not rows.any():
                continue
            gW[l] += H[rows].T @ g[rows]
            gB[l] += g[rows].sum(0)
            dX[rows] = (g[rows] @ f(W[l]).T) * (H[rows] > 0)
        g = dX if i == 0 else q(dX)
    errs['gpre1'] = rel_err(f(gpre1), g)
    for l in range(9):
        if l >= 6 and R == B:
            continue
        errs[f'gw{l}'] = rel_err(f(gw[l]), gW[l])
        errs[f'gb{l}'] = rel_err(f(gb[l]), gB[l])
    tol = 1e-5 if dtype == L.CC_F32 else 2e-2
    bad = {k: v for k, v in errs.items() if not v < tol}
    assert not bad, bad


def test_device_lds_limits():
    p = torch.cuda.get_device_properties(0)
    print('LDS per block', getattr(p, 'shared_memory_per_block', None),
          'optin', getattr(p, 'shared_memory_per_block_optin', None),
          'per CU', getattr(p, 'shared_memory_per_multiprocessor', None))



def test_fused_towers_match_generic_gemm_path():
    """The fused tower kernels and the per-layer cc_gemm path give the same step (bf16 & fp32)."""
    from tests.test_gpu_train import _setup
    for dtype in ('fp32', 'bf16'):
        res = {}
        for fused in (True, False):
            tr, *_ = _setup(700, 64, 32, 128, 0.1, dtype, fused_tower=fused)
            tr.forward_backward()
            torch.cuda.synchronize()
            res[fused] = tr.layout.unpack(tr.grads.cpu().numpy())
        tol = 1e-5 if dtype == 'fp32' else 1e-2
        bad = {k: rel_err(res[True][k], res[False][k]) for k in res[True]
               if not rel_err(res[True][k], res[False][k]) < tol}
        assert not bad, (dtype, bad)


@pytest.mark.parametrize('d,B,R', [(256, 64, 128), (256, 512, 512), (128, 32, 64), (64, 32, 32),
                                   (512, 64, 128), (1024, 64, 128), (1024, 128, 256), (768, 32, 96)])
def test_packed_weight_images_bit_exact(d, B, R):
    """The fragment-packed weight images (cc_tower_args.wpf/wpb, written by cc_tower_transpose)
    feed the fast bf16 kernels the same fragments as the row-strided reads: identical outputs,
    and the images hold exactly the documented element order.  At d > 256 the packed images
    select the wide item-stream kernels (several tiles / reduction chunks per wave), the unpacked
    arm the generic 4-wave kernels: the two must agree bit for bit."""
    rng = np.random.default_rng(d * 7 + R)
    tdt = torch.bfloat16
    rnd = lambda *s: torch.from_numpy((rng.standard_normal(s) * 0.2).astype(np.float32)).to('cuda', tdt)
    dims = _dims(d)
    W = [rnd(*dims[l if l < 6 else l - 3]) for l in range(9)]
    bias = [torch.from_numpy(rng.standard_normal(w.shape[1]).astype(np.float32) * 0.1).cuda() for w in W]
    widths = [d, 256, 128, 64, 128, 256, d]
    x0, gD3 = rnd(R, d), rnd(R, d)
    outs = {}
    for packed in (False, True):
        Wt = [torch.zeros(w.shape[1], w.shape[0], device='cuda', dtype=tdt) for w in W]
        wpf = [torch.zeros(w.numel(), device='cuda', dtype=tdt) for w in W]
        wpb = [torch.zeros(w.numel(), device='cuda', dtype=tdt) for w in W]
        act = [x0.clone()] + [torch.zeros(R, w, device='cuda', dtype=tdt) for w in widths[1:]]
        act6t = torch.zeros(d, R, device='cuda', dtype=tdt)
        gact = [torch.zeros(R, w, device='cuda', dtype=tdt) for w in (256, 128, 64, 128, 256)]
        gpre1 = torch.zeros(R, d, device='cuda')
        gpre1t = torch.zeros(d, (R + 63) // 64 * 64, device='cuda', dtype=tdt)
        slab = torch.zeros((R // 32) * int(L.lib().cc_tower_slab_elems(d)), device='cuda')
        t = L.TowerArgs(dtype=L.CC_BF16, d=d, B=B, R=R)
        t.slab = slab.data_ptr()
        for l in range(9):
            t.w[l], t.wt[l], t.b[l] = W[l].data_ptr(), Wt[l].data_ptr(), bias[l].data_ptr()
            if packed:
                t.wpf[l], t.wpb[l] = wpf[l].data_ptr(), wpb[l].data_ptr()
        for a in range(7):
            t.act[a] = act[a].data_ptr()
        t.act6t, t.gD3, t.gpre1, t.gpre1t = act6t.data_ptr(), gD3.data_ptr(), gpre1.data_ptr(), gpre1t.data_ptr()
        act6p, act6tp = torch.zeros(R * d, device='cuda', dtype=tdt), torch.zeros(R * d, device='cuda', dtype=tdt)
        t.act6p, t.act6tp = act6p.data_ptr(), act6tp.data_ptr()
        for a in range(5):
            t.gact[a] = gact[a].data_ptr()
        s = L.stream_ptr()
        for fn in ('cc_tower_transpose', 'cc_tower_fwd', 'cc_tower_bwd_chain'):
            L.call(fn, ctypes.byref(t), s)
        torch.cuda.synchronize()
        outs[packed] = [a.cpu() for a in act[1:]] + [act6t.cpu()] + [g.cpu() for g in gact] + [gpre1.cpu(), gpre1t.cpu()]
        D3 = act[6].cpu()
        if d <= 256:   # the fused D1/D2 kernels' packed D3 operands (d <= 256 only)
            assert torch.equal(act6p.cpu(), D3.view(R // 32, 32, d // 16, 2, 8).permute(0, 2, 3, 1, 4).reshape(-1))
            assert torch.equal(act6tp.cpu(), D3.t().contiguous().view(d // 32, 32, R // 16, 2, 8)
                               .permute(0, 2, 3, 1, 4).reshape(-1))
        if packed:
            for l in range(9 if R > B else 6):
                w = W[l].cpu().view(torch.int16).numpy()
                K, N = w.shape
                f = wpf[l].cpu().view(torch.int16).numpy().reshape(N // 32, K // 16, 2, 32, 8)
                assert np.array_equal(f, w.T.reshape(N // 32, 32, K // 16, 2, 8).transpose(0, 2, 3, 1, 4)), l
                b = wpb[l].cpu().view(torch.int16).numpy().reshape(K // 32, N // 16, 2, 32, 8)
                assert np.array_equal(b, w.reshape(K // 32, 32, N // 16, 2, 8).transpose(0, 2, 3, 1, 4)), l
    for i, (a, b) in enumerate(zip(outs[False], outs[True])):
        assert torch.equal(a, b), i


@pytest.mark.parametrize('d,B,R', [(256, 64, 128), (256, 512, 512), (128, 32, 64), (1024, 64, 128), (512, 128, 256)])
def test_packed_dw_matches_tiled(d, B, R):
    """cc_tower_bwd_dw_direct from the packed transposed H_i / G_i images (written by the fast
    forward / backward chains) equals the LDS-staged tiled kernel up to fp32 summation order, and
    the images hold the documented element order."""
    rng = np.random.default_rng(d + 3 * R)
    tdt = torch.bfloat16
    rnd = lambda *s: torch.from_numpy((rng.standard_normal(s) * 0.2).astype(np.float32)).to('cuda', tdt)
    dims = _dims(d)
    W = [rnd(*dims[l if l < 6 else l - 3]) for l in range(9)]
    bias = [torch.from_numpy(rng.standard_normal(w.shape[1]).astype(np.float32) * 0.1).cuda() for w in W]
    widths = [d, 256, 128, 64, 128, 256, d]
    x0, gD3 = rnd(R, d), rnd(R, d)
    outs = {}
    for packed in (False, True):
        t = L.TowerArgs(dtype=L.CC_BF16, d=d, B=B, R=R)
        keep = []
        def buf(n, dt=tdt):
            b = torch.zeros(n, device='cuda', dtype=dt)
            keep.append(b)
            return b
        act = [x0.clone()] + [buf(R * w) for w in widths[1:]]
        gact = [buf(R * w) for w in (256, 128, 64, 128, 256)]
        gw = [buf(w.numel(), torch.float32) for w in W]
        gb = [buf(w.shape[1], torch.float32) for w in W]
        hpt = [buf(R * w) for w in (d, 256, 128, 64, 128, 256)]
        gpt = [buf(R * w) for w in (256, 128, 64, 128, 256, d)]
        for l in range(9):
            t.w[l], t.wt[l], t.b[l] = W[l].data_ptr(), buf(W[l].numel()).data_ptr(), bias[l].data_ptr()
            t.wpf[l], t.wpb[l] = buf(W[l].numel()).data_ptr(), buf(W[l].numel()).data_ptr()
            t.gw[l], t.gb[l] = gw[l].data_ptr(), gb[l].data_ptr()
        for a in range(7):
            t.act[a] = act[a].data_ptr()
        for a in range(5):
            t.gact[a] = gact[a].data_ptr()
        t.gD3, t.gpre1 = gD3.data_ptr(), buf(R * d, torch.float32).data_ptr()
        t.gpre1t = buf(d * ((R + 63) // 64 * 64)).data_ptr()
        t.slab = buf((R // 32) * int(L.lib().cc_tower_slab_elems(d)), torch.float32).data_ptr()
        if packed:
            for a in range(6):
                t.hpt[a], t.gpt[a] = hpt[a].data_ptr(), gpt[a].data_ptr()
        s = L.stream_ptr()
        for fn in ('cc_tower_transpose', 'cc_tower_fwd', 'cc_tower_bwd_chain', 'cc_tower_bwd_dw_direct'):
            L.call(fn, ctypes.byref(t), s)
        torch.cuda.synchronize()
        outs[packed] = ([g.cpu().numpy() for g in gw], [g.cpu().numpy() for g in gb])
        if packed:
            pt = lambda X, w: X.view(R // 16, 2, 8, w // 32, 32).permute(3, 0, 1, 4, 2).reshape(-1)
            Hs = [x0.cpu()] + [act[a].cpu().view(R, widths[a]) for a in range(1, 6)]
            Gs = [gact[a].cpu().view(R, w) for a, w in enumerate((256, 128, 64, 128, 256))] + [gD3.cpu()]
            for a in range(6):
                assert torch.equal(hpt[a].cpu(), pt(Hs[a], Hs[a].shape[1])), a
                assert torch.equal(gpt[a].cpu(), pt(Gs[a], Gs[a].shape[1])), a
    for l in range(9 if R > B else 6):
        assert rel_err(outs[True][0][l], outs[False][0][l]) < 1e-5, l
        assert rel_err(outs[True][1][l], outs[False][1][l]) < 1e-5, l
