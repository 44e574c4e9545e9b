"""GPU parity tests of the individual kernels against the CPU oracle (run on an MI355X)."""
import ctypes

import numpy as np
import pytest
import torch

from cubecobrarecommender_amd import _lib as L
from oracle import noise_ref
from tests.gpu_helpers import problem, rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def _gpu():
    assert torch.cuda.is_available(), 'GPU tests need a GPU'
    L.lib()


def _run_noise(lists, V, B, ns, seed, step, with_reg=True, slot_rank=0, guide_log2=0, x_bits=None):
    dev = 'cuda'
    lens = np.array([len(c) for c in lists])
    indptr = np.zeros(len(lists) + 1, np.int64)
    indptr[1:] = np.cumsum(lens)
    idx = np.concatenate(lists).astype(np.int32)
    cdf = noise_ref.cdf_of(ns)
    max_n = int(lens.max())
    x_cap = max_n + int(max_n * 0.8) + 1
    R = 2 * B if with_reg else B
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)
    cube_ptr, cube_idx = t(indptr, torch.int64), t(idx, torch.int32)
    perm = t(np.arange(len(lists), dtype=np.int32), torch.int32)
    cdf_d, ns_d = t(cdf, torch.float64), t(ns, torch.float64)
    guide = t(np.searchsorted(cdf, np.arange((1 << guide_log2) + 1) / float(1 << guide_log2),
                              side='right').astype(np.int32), torch.int32) if guide_log2 else None
    state = t(np.array([step, 0, 0, 0], np.int64), torch.int64)
    x_cnt = torch.zeros(R, device=dev, dtype=torch.int32)
    x_idx = torch.zeros(R, x_cap, device=dev, dtype=torch.int32)
    VW = (V + 31) // 32
    y_bits = torch.zeros(B, VW, device=dev, dtype=torch.int32)
    xt = torch.zeros(V, (R + 31) // 32, device=dev, dtype=torch.int32)
    reg = torch.zeros(B, device=dev, dtype=torch.int32)
    status = torch.zeros(1, device=dev, dtype=torch.int32)
    a = L.NoiseArgs(V=V, B=B, x_cap=x_cap, with_reg=int(with_reg), seed=seed, slot_base=slot_rank * B,
                    batch_stride=B, batch_offset=0, num_perms=1, num_cubes=len(lists), noise_mean=0.2, noise_std=0.1,
                    cube_ptr=cube_ptr.data_ptr(), cube_idx=cube_idx.data_ptr(), perm=perm.data_ptr(),
                    cdf=cdf_d.data_ptr(), neg_sampler=ns_d.data_ptr(), state=state.data_ptr(),
                    guide=guide.data_ptr() if guide is not None else None, guide_log2=guide_log2,
                    x_cnt=x_cnt.data_ptr(), x_idx=x_idx.data_ptr(), y_bits=y_bits.data_ptr(),
                    xt_bits=xt.data_ptr() if x_bits is None else None, reg_idx=reg.data_ptr(),
                    status=status.data_ptr(), xt_rows=R, x_bits=x_bits.data_ptr() if x_bits is not None else None)
    L.call('cc_noise_fwd', ctypes.byref(a), L.stream_ptr())
    torch.cuda.synchronize()
    assert int(status.item()) == 0
    cnt = x_cnt.cpu().numpy()
    xi = x_idx.cpu().numpy()
    xs = [xi[r, :cnt[r]] for r in range(R)]
    yb = y_bits.cpu().numpy().view(np.uint32)
    ys = [np.nonzero(np.unpackbits(yb[b].view(np.uint8), bitorder='little')[:V])[0] for b in range(B)]
    xtb = xt.cpu().numpy().view(np.uint32)
    return xs, ys, reg.cpu().numpy(), xtb, cdf


@pytest.mark.parametrize('V,B,sizes,seed,step,glog2', [
    (300, 16, (5, 30, 60), 1, 0, 0),
    (1500, 64, (40, 200, 400), 2, 7, 0),
    (1500, 64, (40, 200, 400), 2, 7, 12),
    (22000, 64, (180, 360, 450, 540, 720), 20250301, 123456, 0),
    (22000, 64, (180, 360, 450, 540, 720), 20250301, 123456, 12),
    (22000, 64, (180, 360, 450, 540, 720), 20250301, 123456, 16),
    (300, 16, (5, 30, 60), 1, 0, 16),
])
def test_noise_bit_exact_vs_oracle(V, B, sizes, seed, step, glog2):
    lists, Mt, ns = problem(seed, B, V, sizes)
    xs, ys, reg, xt, cdf = _run_noise(lists, V, B, ns, seed, step, guide_log2=glog2)
    oxs, oys, oreg, ks = noise_ref.philox_noise_batch(lists, cdf, ns, seed, step, slot_base=0)
    assert np.array_equal(reg, oreg)
    for b in range(B):
        assert np.array_equal(xs[b], oxs[b]), f'x row {b}'
        assert np.array_equal(ys[b], oys[b]), f'y row {b}'
        assert list(xs[B + b]) == [oreg[b]]
    # transposed bitmask == x rows
    R = 2 * B
    for r in range(0, R, max(1, R // 7)):
        col = (xt[:, r // 32] >> np.uint32(r % 32)) & 1
        assert np.array_equal(np.nonzero(col)[0], xs[r])


@pytest.mark.parametrize('V,B,d,sizes,rows', [(22000, 64, 256, (180, 360, 720), 'R'), (1500, 64, 256, (40, 200, 400), 'R'),
                                               (1500, 64, 64, (40, 200, 400), 'R'), (300, 48, 256, (5, 30, 60), 'B'),
                                               (1000, 40, 128, (5, 30, 60), 'B'), (22000, 64, 1024, (180, 360, 720), 'R'),
                                               (1500, 48, 512, (40, 200, 400), 'B')])
def test_gather_xt_transpose(V, B, d, sizes, rows):
    """F with x_bits (row bitmasks, no xt atomics) + cc_embed_gather_fwd_xt's bit transpose (fused
    into the bf16 d = 256 gather, a separate kernel otherwise) == the xt bits F's atomics set, and
    the gathered rows are unchanged."""
    lists, Mt, ns = problem(11, B, V, sizes)
    xs, ys, reg, xt_ref, cdf = _run_noise(lists, V, B, ns, 11, 3)
    R, VW = 2 * B, (V + 31) // 32
    xb = torch.zeros(R, VW, device='cuda', dtype=torch.int32)
    xs2, ys2, _, xt_none, _ = _run_noise(lists, V, B, ns, 11, 3, x_bits=xb)
    assert not xt_none.any()
    for r in range(R):
        assert np.array_equal(xs2[r], xs[r])
        bits = np.nonzero(np.unpackbits(xb[r].cpu().numpy().view(np.uint8), bitorder='little')[:V])[0]
        assert np.array_equal(bits, xs[r]), f'x_bits row {r}'
    xt_rows = R if rows == 'R' else B
    XW = (xt_rows + 31) // 32
    exp = np.zeros((V, XW), np.uint32)
    for r in range(xt_rows):
        exp[xs[r], r // 32] |= np.uint32(1 << (r % 32))
    if rows == 'R':
        assert np.array_equal(exp, xt_ref)
    cap = max(len(x) for x in xs) + 1
    x_cnt = torch.tensor([len(x) for x in xs], dtype=torch.int32, device='cuda')
    x_idx = torch.zeros(R, cap, dtype=torch.int32)
    for r, x in enumerate(xs):
        x_idx[r, :len(x)] = torch.from_numpy(x.astype(np.int32))
    x_idx = x_idx.cuda()
    table = (torch.randn(V, d, device='cuda') * 0.1).to(torch.bfloat16)
    bias = torch.randn(d, device='cuda') * 0.1
    outs = []
    for xt_on in (False, True):
        out = torch.zeros(R, d, device='cuda', dtype=torch.bfloat16)
        xt = torch.full((V, XW), -1, device='cuda', dtype=torch.int32)   # every word is written
        L.call('cc_embed_gather_fwd_xt', L.CC_BF16, L.ptr(table), L.ptr(bias), V, d, R, L.ptr(x_cnt), L.ptr(x_idx),
               cap, L.ptr(out), None, 0, None, 1, L.ptr(xb) if xt_on else None, L.ptr(xt) if xt_on else None,
               xt_rows, L.stream_ptr())
        torch.cuda.synchronize()
        outs.append(out)
    # bf16 d = 256: without xt the XCD column-sliced gather runs (another fp32 summation order than
    # the transposing gather2): equal to one bf16 ulp
    o0, o1 = outs[0].float(), outs[1].float()
    assert torch.all((o0 - o1).abs() <= o1.abs() * 2 ** -7 + 1e-30)
    if d != 256:
        assert torch.equal(outs[0], outs[1])
    assert np.array_equal(xt.cpu().numpy().view(np.uint32), exp)


def test_noise_edge_cases():
    V, B = 200, 8
    rng = np.random.default_rng(5)
    ns = rng.dirichlet(np.ones(V))
    ns[190:] = 1e-6          # cube 2 holds ~all the mass: forces the exact fallback path
    ns[20] = 0.0             # a zero-probability card is never added
    ns /= ns.sum()
    lists = [np.zeros(0, np.int64), np.array([3]), np.arange(0, 190),  # empty, 1 card, nearly all mass
             np.array([0, 199]), np.arange(50, 60), np.arange(100, 150), np.array([7, 8]), np.arange(0, 200, 2)]
    xs, ys, reg, xt, cdf = _run_noise(lists, V, B, ns, seed=9, step=1)
    oxs, oys, oreg, _ = noise_ref.philox_noise_batch(lists, cdf, ns, 9, 1)
    for b in range(B):
        assert np.array_equal(xs[b], oxs[b]) and np.array_equal(ys[b], oys[b])
    assert len(xs[0]) == 0 and len(ys[0]) == 0


def _gemm_case(dtype, ta, tb, M, N, K, epi, rng):
    tdt = torch.bfloat16 if dtype == L.CC_BF16 else torch.float32
    A = torch.from_numpy(rng.standard_normal((K, M) if ta else (M, K)).astype(np.float32)).to('cuda', tdt)
    Bm = torch.from_numpy(rng.standard_normal((N, K) if tb else (K, N)).astype(np.float32)).to('cuda', tdt)
    Ad = A.double().cpu().numpy()
    Bd = Bm.double().cpu().numpy()
    ref = (Ad.T if ta else Ad) @ (Bd.T if tb else Bd)
    bias = torch.from_numpy(rng.standard_normal(N).astype(np.float32)).cuda()
    Cf = torch.zeros(M, N, device='cuda')
    g = L.GemmArgs(dtype=dtype, ta=ta, tb=tb, epilogue=epi, M=M, N=N, K=K, lda=M if ta else K,
                   ldb=K if tb else N, ldc=N, splits=1, relu=0, A=A.data_ptr(), B=Bm.data_ptr())
    return A, Bm, ref, bias, Cf, g


@pytest.mark.parametrize('dtype', [L.CC_F32, L.CC_BF16])
@pytest.mark.parametrize('ta,tb', [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize('M,N,K', [(64, 64, 32), (100, 72, 50), (512, 256, 256), (37, 130, 1000)])
def test_gemm_store_vs_fp64(dtype, ta, tb, M, N, K):
    rng = np.random.default_rng(M * 7 + N + K)
    A, Bm, ref, bias, Cf, g = _gemm_case(dtype, ta, tb, M, N, K, L.CC_EPI_STORE, rng)
    g.bias = bias.data_ptr()
    g.relu = 1
    g.Cf = Cf.data_ptr()
    cs = torch.zeros(N, device='cuda')
    g.colsum = cs.data_ptr()
    L.call('cc_gemm', ctypes.byref(g), L.stream_ptr())
    torch.cuda.synchronize()
    want = np.maximum(ref + bias.double().cpu().numpy(), 0)
    assert rel_err(Cf.cpu().numpy(), want) < 2e-6
    Bd = Bm.double().cpu().numpy()
    assert rel_err(cs.cpu().numpy(), (Bd.T if tb else Bd).sum(0)) < 2e-6   # fused bias gradient


@pytest.mark.parametrize('dtype', [L.CC_F32, L.CC_BF16])
def test_gemm_splitk_and_mask(dtype):
    rng = np.random.default_rng(11)
    M, N, K, S = 96, 80, 3000, 7
    A, Bm, ref, bias, Cf, g = _gemm_case(dtype, 0, 1, M, N, K, L.CC_EPI_SPLITK, rng)
    part = torch.zeros(S, M, N, device='cuda')
    cs_part = torch.zeros(S, N, device='cuda')
    cs = torch.zeros(N, device='cuda')
    g.splits = S
    g.Cf = part.data_ptr()
    g.colsum = cs_part.data_ptr()
    L.call('cc_gemm', ctypes.byref(g), L.stream_ptr())
    tdt = torch.bfloat16 if dtype == L.CC_BF16 else torch.float32
    H = torch.from_numpy(rng.standard_normal((M, N)).astype(np.float32)).to('cuda', tdt)
    out = torch.zeros(M, N, device='cuda', dtype=tdt)
    L.call('cc_splitk_reduce', dtype, L.ptr(part), S, M, N, L.ptr(H), L.ptr(out), L.ptr(Cf),
           L.ptr(cs_part), L.ptr(cs), L.stream_ptr())
    torch.cuda.synchronize()
    want = ref * (H.double().cpu().numpy() > 0)
    assert rel_err(Cf.cpu().numpy(), want) < 2e-6
    assert rel_err(cs.cpu().numpy(), Bm.double().cpu().numpy().T.sum(0)) < 2e-6
    # MASK epilogue directly (no split)
    g2 = L.GemmArgs(dtype=dtype, ta=0, tb=1, epilogue=L.CC_EPI_MASK, M=M, N=N, K=K, lda=K, ldb=K, ldc=N,
                    splits=1, A=A.data_ptr(), B=Bm.data_ptr(), H=H.data_ptr(), Cf=Cf.data_ptr())
    Cf.zero_()
    L.call('cc_gemm', ctypes.byref(g2), L.stream_ptr())
    torch.cuda.synchronize()
    assert rel_err(Cf.cpu().numpy(), want) < 2e-6


@pytest.mark.parametrize('dtype', [L.CC_F32, L.CC_BF16])
def test_bce_epilogue(dtype):
    rng = np.random.default_rng(3)
    B, d, V = 70, 64, 333
    tdt = torch.bfloat16 if dtype == L.CC_BF16 else torch.float32
    H = torch.from_numpy(rng.standard_normal((B, d)).astype(np.float32)).to('cuda', tdt)
    W = torch.from_numpy(rng.standard_normal((d, V)).astype(np.float32) * 0.3).to('cuda', tdt)
    bo = torch.from_numpy(rng.standard_normal(V).astype(np.float32)).cuda()
    Y = (rng.random((B, V)) < 0.1)
    VW = (V + 31) // 32
    yb = np.zeros((B, VW * 32), np.uint8)
    yb[:, :V] = Y
    ybits = torch.from_numpy(np.packbits(yb, axis=1, bitorder='little').view(np.int32).copy()).cuda()
    dZ = torch.zeros(B, V, device='cuda', dtype=torch.float32)
    tiles = ((B + 63) // 64) * ((V + 63) // 64)
    part = torch.zeros(tiles, device='cuda', dtype=torch.float64)
    loss = torch.zeros(1, device='cuda', dtype=torch.float64)
    n = ctypes.c_int32()
    L.call('cc_dec_bce_fused', dtype, L.ptr(H), L.ptr(W), L.ptr(bo), B, d, V, L.ptr(ybits), None,
           L.ptr(part), ctypes.byref(n), L.stream_ptr())
    L.call('cc_reduce_loss', L.ptr(part), n.value, 1.0 / (B * V), L.ptr(loss), L.stream_ptr())
    g = L.GemmArgs(dtype=dtype, ta=0, tb=0, epilogue=L.CC_EPI_BCE, M=B, N=V, K=d, lda=d, ldb=V, ldc=V,
                   A=H.data_ptr(), B=W.data_ptr(), bias=bo.data_ptr(), Cf=dZ.data_ptr(),
                   y_bits=ybits.data_ptr(), scale=1.0 / (B * V), loss_partials=part.data_ptr())
    L.call('cc_gemm', ctypes.byref(g), L.stream_ptr())
    torch.cuda.synchronize()
    z = H.double().cpu().numpy() @ W.double().cpu().numpy() + bo.double().cpu().numpy()
    l = np.maximum(z, 0) - z * Y + np.log1p(np.exp(-np.abs(z)))
    assert abs(loss.item() - l.mean()) / l.mean() < 1e-6
    want = (1 / (1 + np.exp(-z)) - Y) / (B * V)
    assert rel_err(dZ.cpu().numpy(), want) < 1e-5


@pytest.mark.parametrize('dtype', [L.CC_F32, L.CC_BF16])
@pytest.mark.parametrize('d', [64, 256, 512])
def test_gather_and_scatter(dtype, d):
    rng = np.random.default_rng(d)
    V, R, cap = 3000, 50, 120
    tdt = torch.bfloat16 if dtype == L.CC_BF16 else torch.float32
    W = torch.from_numpy(rng.standard_normal((V, d)).astype(np.float32)).to('cuda', tdt)
    b = torch.from_numpy(rng.standard_normal(d).astype(np.float32)).cuda()
    lists = [np.sort(rng.choice(V, int(rng.integers(0, cap)), replace=False)) for _ in range(R)]
    xi = np.zeros((R, cap), np.int32)
    for r, l in enumerate(lists):
        xi[r, :len(l)] = l
    cnt = torch.from_numpy(np.array([len(l) for l in lists], np.int32)).cuda()
    xid = torch.from_numpy(xi).cuda()
    out = torch.zeros(R, d, device='cuda', dtype=tdt)
    L.call('cc_embed_gather_fwd', dtype, L.ptr(W), L.ptr(b), V, d, R, L.ptr(cnt), L.ptr(xid), cap, L.ptr(out),
           L.stream_ptr())
    Wd = W.double().cpu().numpy()
    want = np.stack([np.maximum(Wd[l].sum(0) + b.double().cpu().numpy(), 0) for l in lists])
    torch.cuda.synchronize()
    tol = 1e-2 if dtype == L.CC_BF16 else 1e-6
    assert rel_err(out.double().cpu().numpy(), want) < tol
    # backward: dW[r] = sum_{b: r in x_b} dpre[b]
    dpre = torch.from_numpy(rng.standard_normal((R, d)).astype(np.float32)).cuda()
    XW = (R + 31) // 32
    xt = np.zeros((V, XW), np.uint32)
    for r, l in enumerate(lists):
        xt[l, r // 32] |= np.uint32(1 << (r % 32))
    xtd = torch.from_numpy(xt.view(np.int32)).cuda()
    grad = torch.full((V, d), 7.0, device='cuda')
    bgrad = torch.full((d,), 7.0, device='cuda')
    L.call('cc_embed_scatter_bwd', L.ptr(dpre), V, d, R, L.ptr(xtd), L.ptr(grad), L.ptr(bgrad), L.stream_ptr())
    torch.cuda.synchronize()
    assert rel_err(bgrad.cpu().numpy(), dpre.double().cpu().numpy().sum(0)) < 1e-6
    gw = np.zeros((V, d))
    dp = dpre.double().cpu().numpy()
    for r, l in enumerate(lists):
        gw[l] += dp[r]
    assert rel_err(grad.cpu().numpy(), gw) < 1e-6


@pytest.mark.parametrize('d', [256, 512, 1024])
@pytest.mark.parametrize('R', [51, 64])
def test_gather_xcd_slices_edge_rows(R, d):
    """The bf16 E1 gathers by XCD column slices (d = 256: 4 slices x 2 row parities per 8 blocks;
    d = 512 / 1024: 8 slices of one row, gather_xcdw_kernel): odd R (the last block pair half
    empty), empty rows, one card, a row longer than the LDS index stage (2,100 > 2,048: read from
    global), list tails that are not whole card groups; every output element within bf16 rounding
    of the fp64 sum, the counters advanced once (inside the gather launch)."""
    rng = np.random.default_rng(R)
    V, cap = 3000, 2112
    W = torch.from_numpy(rng.standard_normal((V, d)).astype(np.float32)).to('cuda', torch.bfloat16)
    b = torch.from_numpy(rng.standard_normal(d).astype(np.float32)).cuda()
    sizes = [0, 1, 2100, 7, 9, 63, 65] + [int(rng.integers(0, 800)) for _ in range(R - 7)]
    lists = [np.sort(rng.choice(V, n, replace=False)) for n in sizes]
    xi = np.zeros((R, cap), np.int32)
    for r, l in enumerate(lists):
        xi[r, :len(l)] = l
    cnt = torch.from_numpy(np.array(sizes, np.int32)).cuda()
    xid = torch.from_numpy(xi).cuda()
    out = torch.full((R + 1, d), 3.0, device='cuda', dtype=torch.bfloat16)   # row R must stay untouched
    state = torch.tensor([5, 2, 0], dtype=torch.int64, device='cuda')
    L.call('cc_embed_gather_fwd_warm', L.CC_BF16, L.ptr(W), L.ptr(b), V, d, R, L.ptr(cnt), L.ptr(xid), cap,
           L.ptr(out), None, 0, L.ptr(state), 3, L.stream_ptr())
    torch.cuda.synchronize()
    Wd = W.double().cpu().numpy()
    want = np.stack([np.maximum(Wd[l].sum(0) + b.double().cpu().numpy(), 0) for l in lists])
    got = out.double().cpu().numpy()
    assert np.all(got[R] == 3.0)
    err = np.abs(got[:R] - want) / np.maximum(np.abs(want), 1.0)
    assert err.max() < 2 ** -7, err.max()
    assert state.tolist() == [6, 0, 1]


@pytest.mark.parametrize('rows,cols', [(256, 22000), (64, 700), (256, 20884), (13, 7), (24, 40)])
def test_transpose_bf16_and_fp32(rows, cols):
    """cc_transpose (the Wo^T refresh): vector bf16 path (rows, cols % 8 == 0) and scalar paths."""
    from cubecobrarecommender_amd import _lib as L
    for dt, tdt in ((L.CC_BF16, torch.bfloat16), (L.CC_F32, torch.float32)):
        src = torch.randn(rows, cols, device='cuda').to(tdt)
        dst = torch.zeros(cols, rows, device='cuda', dtype=tdt)
        L.call('cc_transpose', dt, L.ptr(src), rows, cols, L.ptr(dst), L.stream_ptr())
        torch.cuda.synchronize()
        assert torch.equal(dst, src.t().contiguous())


@pytest.mark.parametrize('B,d,V,splits', [(128, 64, 700, 4), (512, 256, 2500, 8)])
def test_gemm_pair_equals_two_launches(B, d, V, splits):
    """cc_gemm_pair (grouped dX split-K + dW with colsum) == the two cc_gemm launches, bitwise."""
    bf = dict(device='cuda', dtype=torch.bfloat16)
    dZ = (torch.randn(B, V, device='cuda') * 1e-3).to(torch.bfloat16)
    Wo = torch.randn(d, V, **bf)
    D3t = torch.randn(d, B, **bf)
    dZt = dZ.t().contiguous()

    def args(out_split, gW, gb):
        gx = L.GemmArgs(dtype=L.CC_BF16, ta=0, tb=1, epilogue=L.CC_EPI_SPLITK, M=B, N=d, K=V, lda=V, ldb=V,
                        ldc=d, splits=splits, A=dZ.data_ptr(), B=Wo.data_ptr(), Cf=out_split.data_ptr())
        gw = L.GemmArgs(dtype=L.CC_BF16, ta=0, tb=1, epilogue=L.CC_EPI_STORE, M=d, N=V, K=B, lda=B, ldb=B,
                        ldc=V, splits=1, A=D3t.data_ptr(), B=dZt.data_ptr(), Cf=gW.data_ptr(), colsum=gb.data_ptr())
        return gx, gw

    outs = []
    for pair in (False, True):
        sp = torch.zeros(splits * B * d, device='cuda')
        gW = torch.zeros(d, V, device='cuda')
        gb = torch.zeros(V, device='cuda')
        gx, gw = args(sp, gW, gb)
        if pair:
            L.call('cc_gemm_pair', ctypes.byref(gx), ctypes.byref(gw), L.stream_ptr())
        else:
            L.call('cc_gemm', ctypes.byref(gx), L.stream_ptr())
            L.call('cc_gemm', ctypes.byref(gw), L.stream_ptr())
        torch.cuda.synchronize()
        outs.append((sp.cpu(), gW.cpu(), gb.cpu()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    ref = (D3t.float() @ dZt.float().t())
    assert rel_err(outs[1][1].numpy(), ref.cpu().numpy()) < 1e-5


def _softmax_kl_ref(Z, T, reg, B):
    """fp64 statement of the KL term: loss rows and dZ = reg/B p (g - <p,g>)."""
    Z = Z.astype(np.float64)
    p = np.exp(Z - Z.max(1, keepdims=True))
    p /= p.sum(1, keepdims=True)
    t = np.clip(T.astype(np.float64), 1e-7, 1.0)
    q = np.clip(p, 1e-7, 1.0)
    kl = (t * np.log(t / q)).sum(1)
    live = p >= 1e-7
    S = (t * live).sum(1, keepdims=True)
    dz = reg / B * (np.where(live, -t, 0.0) + p * S)
    return kl, dz


@pytest.mark.parametrize('V', [701, 2500, 22000, 33000])
@pytest.mark.parametrize('dtype', ['fp32', 'bf16'])
def test_softmax_kl_rows(V, dtype):
    """cc_dec_softmax_kl_fused: register-resident rows (V % 4 == 0, V <= 32768) and the generic
    row kernel (V = 701, 33000) against fp64; rows with very negative logits exercise the
    p < 1e-7 clip."""
    rng = np.random.default_rng(V)
    B, reg = 24, 0.1
    Z = (rng.standard_normal((B, V)) * 3).astype(np.float32)
    Z[::5, : V // 3] -= 40.0                    # p below the 1e-7 clip on a third of the row
    Mt = rng.random((B + 3, V)).astype(np.float32) ** 8
    Mt /= Mt.sum(1, keepdims=True)
    Mt[:, ::7] = 0.0
    ridx = rng.integers(0, B + 3, B).astype(np.int32)
    ridx[7] = -1                                # a masked padding row (owner-computes capacity)
    dt = L.CC_BF16 if dtype == 'bf16' else L.CC_F32
    tdt = torch.bfloat16 if dtype == 'bf16' else torch.float32
    Zd = torch.from_numpy(Z).cuda()
    Md = torch.from_numpy(Mt).cuda()
    rd = torch.from_numpy(ridx).cuda()
    dZ = torch.zeros(B, V, device='cuda', dtype=tdt)
    part = torch.zeros(B, device='cuda', dtype=torch.float64)
    L.call('cc_dec_softmax_kl_fused', dt, L.ptr(Zd), B, V, L.ptr(Md), L.ptr(rd), reg / B, L.ptr(dZ),
           L.ptr(part), L.stream_ptr())
    torch.cuda.synchronize()
    kl, dz = _softmax_kl_ref(Z, Mt[np.maximum(ridx, 0)], reg, B)
    kl[7], dz[7] = 0.0, 0.0
    np.testing.assert_allclose(part.cpu().numpy(), kl, rtol=1e-4)
    assert rel_err(dZ.float().cpu().numpy(), dz) < (1e-5 if dtype == 'fp32' else 4e-3)


@pytest.mark.parametrize('V,R,d,heavy', [(3000, 512, 256, True), (1000, 96, 128, False),
                                         (777, 1024, 512, True), (64, 40, 256, False)])
def test_embed_grad_mfma(V, R, d, heavy):
    """cc_embed_grad_mfma: dW1 = X^T dPre1 on bf16 MFMA with the x^T bitmask as the A operand.
    Against the fp64 product of the bits and the bf16-rounded dPre1 (the only rounding), the bias
    row (all-ones) = colsum, bit words zeroed after the call, R not a multiple of 64."""
    rng = np.random.default_rng(V + R + d)
    XW = (R + 31) // 32
    RP = (R + 63) // 64 * 64
    p = np.full(V, 0.02)
    if heavy:
        p[:8] = 0.97      # Zipf-heavy rows: a bit for nearly every batch row
    X = rng.random((R, V)) < p
    xt = np.zeros((V, XW), np.uint32)
    for r in range(R):
        cols = np.nonzero(X[r])[0]
        xt[cols, r // 32] |= np.uint32(1 << (r % 32))
    dpre = rng.standard_normal((R, d)).astype(np.float32)
    dT = torch.zeros(d, RP, dtype=torch.bfloat16)
    dT[:, :R] = torch.from_numpy(dpre.T.copy()).to(torch.bfloat16)
    dTd = dT.cuda()                                # columns R..RP-1 zero (the contract)
    xtd = torch.from_numpy(xt.view(np.int32)).cuda()
    grad = torch.full((V, d), 7.0, device='cuda')
    bgrad = torch.full((d,), 7.0, device='cuda')
    L.call('cc_embed_grad_mfma', L.ptr(dTd), V, d, R, RP, L.ptr(xtd), L.ptr(grad), L.ptr(bgrad),
           L.stream_ptr())
    torch.cuda.synchronize()
    dq = dT[:, :R].double().numpy().T            # bf16-rounded dPre1 [R, d]
    want = X.T.astype(np.float64) @ dq
    got = grad.cpu().numpy()
    assert rel_err(got, want) < 1e-6
    assert np.all(got[~X.any(0)] == 0.0)           # rows absent from the batch: exact zero
    assert rel_err(bgrad.cpu().numpy(), dq.sum(0)) < 1e-6
    assert int(xtd.abs().sum()) == 0               # consumed
    # no bias row
    xtd = torch.from_numpy(xt.view(np.int32)).cuda()
    grad2 = torch.zeros(V, d, device='cuda')
    L.call('cc_embed_grad_mfma', L.ptr(dTd), V, d, R, RP, L.ptr(xtd), L.ptr(grad2), None, L.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(grad2, grad)


def _nt_gemm(M, N, K, A, lda, Bm, ldb, epi, **kw):
    g = L.GemmArgs()
    g.dtype, g.ta, g.tb, g.epilogue = L.CC_BF16, 0, 1, epi
    g.M, g.N, g.K, g.lda, g.ldb, g.ldc, g.splits, g.relu = M, N, K, lda, ldb, kw.get('ldc', N), 1, 0
    g.A, g.B = A.data_ptr(), Bm.data_ptr()
    for k in ('bias', 'C', 'Cf', 'y_bits', 'loss_partials', 'colsum', 'Ct'):
        v = kw.get(k)
        setattr(g, k, v.data_ptr() if v is not None else None)
    g.scale = kw.get('scale', 1.0)
    g.ldct = kw.get('ldct', 0)
    L.call('cc_gemm', ctypes.byref(g), L.stream_ptr())


@pytest.mark.parametrize('B,d,V', [(512, 256, 2500), (128, 128, 700), (256, 256, 64), (512, 512, 2500),
                                   (128, 512, 700), (512, 256, 2504), (128, 128, 712), (256, 128, 22000),
                                   (512, 256, 22000)])
def test_dec_bce_dw_matches_unfused(B, d, V):
    """cc_dec_bce_dw (logits + BCE + dZ + dWo/dbo in one pass) vs the unfused NT-GEMM path (BCE
    epilogue writing dZ and dZ^T, then dW = D3^T dZ^T with the colsum bias gradient): dZ and dWo
    to a bf16 ulp, dbo (fused: the fp32 dz summed; unfused: the rounded dZ) to the same level; the
    fp64 oracle of the same bf16 operands bounds both.  With Wo read in place at d <= 256 and
    V % 8 == 0 the kernel stages its slice by LDS-DMA (tr-read B fragments, dWo from the swapped
    product): bit-identical to the Wo^T-copy kernel."""
    torch.manual_seed(B + d + V)
    bf = dict(device='cuda', dtype=torch.bfloat16)
    D3 = (torch.randn(B, d, device='cuda') * 0.5).to(torch.bfloat16)
    D3t = D3.t().contiguous()
    WoT = (torch.randn(V, d, device='cuda') * 0.1).to(torch.bfloat16)
    bo = torch.randn(V, device='cuda') * 0.1
    VW = (V + 31) // 32
    ybits = torch.randint(-2**31, 2**31 - 1, (B, VW), device='cuda', dtype=torch.int32)
    scale = 1.0 / (B * V)
    # fused
    dZ = torch.zeros(B, V, **bf)
    gW = torch.full((d, V), 7.0, device='cuda')
    gb = torch.full((V,), 7.0, device='cuda')
    nblk = L.lib().cc_dec_bce_dw_blocks(V)
    part = torch.zeros(nblk, device='cuda', dtype=torch.float64)
    loss = torch.zeros(1, device='cuda', dtype=torch.float64)
    tick = torch.zeros(1, device='cuda', dtype=torch.int32)
    L.call('cc_dec_bce_dw', L.ptr(D3), L.ptr(D3t), B, None, None, L.ptr(WoT), None, L.ptr(bo), B, d, V, L.ptr(ybits),
           L.ptr(dZ), L.ptr(gW), L.ptr(gb), L.ptr(part), L.ptr(loss), scale, L.ptr(tick), L.stream_ptr())
    # the fragment-packed operand images (cc_tower_args.act6p / act6tp) give identical results
    D3p = D3.view(B // 32, 32, d // 16, 2, 8).permute(0, 2, 3, 1, 4).contiguous()
    D3tp = D3t.view(d // 32, 32, B // 16, 2, 8).permute(0, 2, 3, 1, 4).contiguous()
    dZp, gWp, gbp = torch.zeros_like(dZ), torch.zeros_like(gW), torch.zeros_like(gb)
    lossp = torch.zeros_like(loss)
    L.call('cc_dec_bce_dw', L.ptr(D3), L.ptr(D3t), B, L.ptr(D3p), L.ptr(D3tp), L.ptr(WoT), None, L.ptr(bo), B, d, V,
           L.ptr(ybits), L.ptr(dZp), L.ptr(gWp), L.ptr(gbp), L.ptr(part), L.ptr(lossp), scale, L.ptr(tick),
           L.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dZ, dZp) and torch.equal(gW, gWp) and torch.equal(gb, gbp) and torch.equal(loss, lossp)
    # ... and so does reading Wo [d][V] itself (slice transposed in LDS) instead of the Wo^T copy
    Wo = WoT.t().contiguous()
    dZw, gWw, gbw, lossw = torch.zeros_like(dZ), torch.zeros_like(gW), torch.zeros_like(gb), torch.zeros_like(loss)
    L.call('cc_dec_bce_dw', L.ptr(D3), L.ptr(D3t), B, L.ptr(D3p), L.ptr(D3tp), None, L.ptr(Wo), L.ptr(bo), B, d, V,
           L.ptr(ybits), L.ptr(dZw), L.ptr(gWw), L.ptr(gbw), L.ptr(part), L.ptr(lossw), scale, L.ptr(tick),
           L.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dZ, dZw) and torch.equal(gW, gWw) and torch.equal(gb, gbw) and torch.equal(loss, lossw)
    # ... and so does the target-mask image (cc_tower_args.y_img; the trainer's call): the epilogue's
    # lane masks from two scalar loads per tile instead of 32 scattered target words
    pos = torch.arange(32)
    row = 8 * (pos >> 3) + 4 * (pos & 1) + ((pos >> 1) & 3)
    yimg = ybits[(torch.arange(B // 32)[:, None] * 32 + row[None, :]).reshape(-1).cuda()].t().contiguous()
    dZi, gWi, gbi, lossi = torch.zeros_like(dZ), torch.zeros_like(gW), torch.zeros_like(gb), torch.zeros_like(loss)
    L.call('cc_dec_bce_dw_img', L.ptr(D3), L.ptr(D3t), B, L.ptr(D3p), L.ptr(D3tp), None, L.ptr(Wo), L.ptr(bo), B, d,
           V, L.ptr(ybits), L.ptr(yimg), L.ptr(dZi), V, L.ptr(gWi), L.ptr(gbi), L.ptr(part), L.ptr(lossi), scale,
           L.ptr(tick), L.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dZ, dZi) and torch.equal(gW, gWi) and torch.equal(gb, gbi) and torch.equal(loss, lossi)
    # unfused
    dZ2 = torch.zeros(B, V, **bf)
    dZt = torch.zeros(V, B, **bf)
    part2 = torch.zeros(4096, device='cuda', dtype=torch.float64)
    _nt_gemm(B, V, d, D3, d, WoT, d, L.CC_EPI_BCE, bias=bo, C=dZ2, y_bits=ybits, loss_partials=part2,
             scale=scale, Ct=dZt, ldct=B)
    gW2 = torch.zeros(d, V, device='cuda')
    gb2 = torch.zeros(V, device='cuda')
    _nt_gemm(d, V, B, D3t, B, dZt, B, L.CC_EPI_STORE, Cf=gW2, colsum=gb2)
    torch.cuda.synchronize()
    # both round dz to bf16 (the fused kernel forms (sigmoid - y) * scale with one fma): equal up
    # to a bf16 ulp, and the products built on them agree to that level
    assert rel_err(dZ.float().cpu().numpy(), dZ2.float().cpu().numpy()) < 4e-3
    assert rel_err(gW.cpu().numpy(), gW2.cpu().numpy()) < 4e-3
    assert rel_err(gb.cpu().numpy(), gb2.cpu().numpy()) < 4e-3
    assert int(tick.item()) == 0
    # fp64 references of dZ (to bf16 rounding), dWo / dbo on the kernel's own rounded dZ, the loss
    y = np.unpackbits(ybits.cpu().numpy().view(np.uint8), axis=1, bitorder='little')[:, :V].astype(np.float64)
    z = D3.double().cpu().numpy() @ WoT.double().cpu().numpy().T + bo.double().cpu().numpy()
    dz_ref = (1.0 / (1.0 + np.exp(-z)) - y) * scale
    dzk = dZ.double().cpu().numpy()
    assert np.max(np.abs(dzk - dz_ref) / np.maximum(np.abs(dz_ref), 1e-30)) < 2 ** -8 + 1e-5
    assert rel_err(gW.cpu().numpy(), D3.double().cpu().numpy().T @ dzk) < 1e-5
    # dbo sums the fp32 dz (before the bf16 rounding of the dZ operand): against the fp64 dz
    assert rel_err(gb.cpu().numpy(), dz_ref.sum(0)) < 2e-5
    want = (np.maximum(z, 0) - z * y + np.log1p(np.exp(-np.abs(z)))).mean()
    assert abs(loss.item() - want) < 1e-5 * abs(want)
    assert abs(part.sum().item() * scale - want) < 1e-5 * abs(want)


@pytest.mark.parametrize('V,R', [(3000, 512), (777, 96), (22000, 1024)])
def test_embed_grad_packed_bit_exact(V, R):
    """cc_embed_grad_packed (B fragments streamed from the packed transposed dPre1) equals
    cc_embed_grad_mfma (LDS-staged dPre1^T) bit for bit: same MFMA k order; both zero xt_bits."""
    d = 256
    RP = (R + 63) // 64 * 64
    rng = np.random.default_rng(V + R)
    X = rng.random((R, V)) < 0.02
    xt = np.zeros((V, (R + 31) // 32), np.uint32)
    rr, cc = np.nonzero(X)
    np.bitwise_or.at(xt, (cc, rr // 32), (np.uint32(1) << (rr % 32).astype(np.uint32)))
    g = (torch.randn(R, d, device='cuda') * 0.1).to(torch.bfloat16)
    gpad = torch.zeros(RP, d, device='cuda', dtype=torch.bfloat16)
    gpad[:R] = g
    gT = gpad.t().contiguous()
    gP = gpad.view(RP // 16, 2, 8, d // 32, 32).permute(3, 0, 1, 4, 2).contiguous()
    outs = []
    for fn, src in (('cc_embed_grad_mfma', gT), ('cc_embed_grad_packed', gP)):
        xtd = torch.from_numpy(xt.view(np.int32)).cuda()
        grad = torch.full((V, d), 7.0, device='cuda')
        bg = torch.full((d,), 7.0, device='cuda')
        L.call(fn, L.ptr(src), V, d, R, RP, L.ptr(xtd), L.ptr(grad), L.ptr(bg), L.stream_ptr())
        torch.cuda.synchronize()
        assert int(xtd.abs().sum().item()) == 0
        outs.append((grad.cpu(), bg.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    want = X.T.astype(np.float64) @ g.double().cpu().numpy()
    assert rel_err(outs[1][0].numpy(), want) < 1e-5


@pytest.mark.parametrize('V,R,d', [(22000, 512, 256), (3000, 512, 256), (777, 96, 256), (22000, 1024, 256),
                                   (5000, 1024, 1024), (1500, 200, 128), (64, 32, 32)])
def test_embed_grad_cs_bit_exact(V, R, d):
    """cc_embed_grad_cs (column slices: the dPre1 slice and the chunk's bit words staged in LDS
    once, A fragments from a nibble LUT) equals cc_embed_grad_mfma bit for bit (same MFMA k order),
    from the packed image and from dPre1^T; it zeroes xt_bits and leaves its tickets zero, so a
    second call (the next step) works the same."""
    RP = (R + 63) // 64 * 64
    rng = np.random.default_rng(V + R + d)
    g = (torch.randn(R, d, device='cuda') * 0.1).to(torch.bfloat16)
    gpad = torch.zeros(RP, d, device='cuda', dtype=torch.bfloat16)
    gpad[:R] = g
    gT = gpad.t().contiguous()
    gP = gpad.view(RP // 16, 2, 8, d // 32, 32).permute(3, 0, 1, 4, 2).contiguous()
    nt = int(L.lib().cc_embed_grad_cs_tickets(V, d, R))
    assert nt >= 1
    tickets = torch.zeros(nt, device='cuda', dtype=torch.int32)
    for rep in range(2):
        X = rng.random((R, V)) < (0.02 if rep == 0 else 0.3)
        xt = np.zeros((V, (R + 31) // 32), np.uint32)
        rr, cc = np.nonzero(X)
        np.bitwise_or.at(xt, (cc, rr // 32), (np.uint32(1) << (rr % 32).astype(np.uint32)))
        outs = []
        runs = [('cs', 1, gP), ('cs', 0, gT)]
        if d % 128 == 0:
            runs.insert(0, ('mfma', None, gT))
        for kind, pk, src in runs:
            xtd = torch.from_numpy(xt.view(np.int32)).cuda()
            grad = torch.full((V, d), 7.0, device='cuda')
            bg = torch.full((d,), 7.0, device='cuda')
            if kind == 'mfma':
                L.call('cc_embed_grad_mfma', L.ptr(src), V, d, R, RP, L.ptr(xtd), L.ptr(grad), L.ptr(bg), L.stream_ptr())
            else:
                L.call('cc_embed_grad_cs', L.ptr(src), pk, V, d, R, RP, L.ptr(xtd), L.ptr(grad), L.ptr(bg),
                       L.ptr(tickets), L.stream_ptr())
            torch.cuda.synchronize()
            assert int(xtd.abs().sum().item()) == 0, kind
            assert int(tickets.abs().sum().item()) == 0, kind
            outs.append((grad.cpu(), bg.cpu()))
        for o in outs[1:]:
            assert torch.equal(outs[0][0], o[0]) and torch.equal(outs[0][1], o[1])
        want = X.T.astype(np.float64) @ g.double().cpu().numpy()
        assert rel_err(outs[-1][0].numpy(), want) < 1e-5
        assert rel_err(outs[-1][1].numpy(), g.double().cpu().numpy().sum(0)) < 1e-5


@pytest.mark.parametrize('M,N,K,splits', [(512, 256, 22000, 32), (640, 128, 1000, 7), (128, 256, 64, 1),
                                          (256, 256, 5008, 3), (4096, 256, 3000, 4), (4224, 512, 2008, 3)])
def test_dx_splitk_glds_matches_nt_gemm(M, N, K, splits):
    """cc_gemm_dx_splitk (LDS-DMA pipeline, dxgemm.hip) == cc_gemm's register-staged NT split-K path:
    the same split boundaries and the same MFMA chain order, so the fp32 partials agree bit for bit;
    ragged K (a K-tile past the end is zero-filled by the buffer range check) included; M >= 4096
    with N % 256 == 0 runs the 128 x 256-tile kernel (the full-mode regulariser's dX)."""
    rng = np.random.default_rng(M + K)
    A = torch.from_numpy(rng.standard_normal((M, K)).astype(np.float32)).to(torch.bfloat16).cuda()
    Bm = torch.from_numpy(rng.standard_normal((N, K)).astype(np.float32)).to(torch.bfloat16).cuda()
    p1 = torch.full((splits, M, N), 7.0, device='cuda')
    p0 = torch.zeros(splits, M, N, device='cuda')
    g = L.GemmArgs(dtype=L.CC_BF16, ta=0, tb=1, epilogue=L.CC_EPI_SPLITK, M=M, N=N, K=K, lda=K, ldb=K, ldc=N,
                   splits=splits, A=L.ptr(A), B=L.ptr(Bm), Cf=L.ptr(p0))
    L.call('cc_gemm', ctypes.byref(g), L.stream_ptr())
    L.call('cc_gemm_dx_splitk', L.ptr(A), K, L.ptr(Bm), K, M, N, K, splits, L.ptr(p1), L.stream_ptr())
    torch.cuda.synchronize()
    want = (A.float() @ Bm.float().t()).cpu().numpy()
    assert rel_err(p1.sum(0).cpu().numpy(), want) < 1e-5
    np.testing.assert_array_equal(p1.cpu().numpy(), p0.cpu().numpy())


@pytest.mark.parametrize('M,N,K,splits', [(4096, 256, 3000, 4), (512, 512, 2008, 3), (128, 256, 64, 1),
                                          (1024, 256, 22000, 5)])
def test_dx_splitk_packed_b_matches(M, N, K, splits):
    """cc_pack_frag_b's fragment image (checked element by element against its layout) and
    cc_gemm_dx_splitk_pk (Wo fragments straight into registers) == cc_gemm_dx_splitk bit for bit,
    ragged last K-tile and K % 16 != 0 (zero-padded last k step) included."""
    rng = np.random.default_rng(M + K + 1)
    A = torch.from_numpy(rng.standard_normal((M, K)).astype(np.float32)).to(torch.bfloat16).cuda()
    Bm = torch.from_numpy(rng.standard_normal((N, K)).astype(np.float32)).to(torch.bfloat16).cuda()
    nks = (K + 15) // 16
    assert L.lib().cc_pack_frag_b_size(N, K) == (N // 32) * nks * 1024
    Bp = torch.full(((N // 32) * nks * 512,), 3.0, dtype=torch.bfloat16, device='cuda')
    L.call('cc_pack_frag_b', L.ptr(Bm), N, K, K, L.ptr(Bp), L.stream_ptr())
    p0 = torch.zeros(splits, M, N, device='cuda')
    p1 = torch.full((splits, M, N), 7.0, device='cuda')
    L.call('cc_gemm_dx_splitk', L.ptr(A), K, L.ptr(Bm), K, M, N, K, splits, L.ptr(p0), L.stream_ptr())
    L.call('cc_gemm_dx_splitk_pk', L.ptr(A), K, L.ptr(Bp), M, N, K, splits, L.ptr(p1), L.stream_ptr())
    torch.cuda.synchronize()
    img = Bp.view(N // 32, nks, 2, 32, 8).cpu().float().numpy()   # [band][k step][lane >> 5][lane & 31][8]
    Bpad = np.zeros((N, nks * 16), np.float32)
    Bpad[:, :K] = Bm.cpu().float().numpy()
    want = Bpad.reshape(N // 32, 32, nks, 2, 8).transpose(0, 2, 3, 1, 4)
    np.testing.assert_array_equal(img, want)
    np.testing.assert_array_equal(p1.cpu().numpy(), p0.cpu().numpy())
