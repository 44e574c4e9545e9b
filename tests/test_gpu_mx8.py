"""MX-FP8 path (config 5): the quantiser bit-exact against oracle/mx8_ref.py and the
block-scaled MFMA GEMM against fp64 products of the dequantised operands."""
import numpy as np
import pytest
import torch

from cubecobrarecommender_amd import _lib as L
from oracle import mx8_ref
from tests.gpu_helpers import rel_err

pytestmark = pytest.mark.gpu
MFMA_TOL = 5e-4


@pytest.fixture(scope='module', autouse=True)
def _gpu():
    assert torch.cuda.is_available(), 'GPU tests need a GPU'
    L.lib()


def _bf16(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(torch.bfloat16)


def _data(rng, rows, cols):
    """Rows of very different magnitudes, exact zeros, a zero block and tiny values."""
    X = rng.standard_normal((rows, cols)).astype(np.float32)
    X *= np.exp2(rng.integers(-40, 20, rows))[:, None].astype(np.float32)
    X[rng.random((rows, cols)) < 0.1] = 0.0
    X[0, :min(cols, 40)] = 0.0
    if rows > 2:
        X[2] *= 1e-20
    return X


def _quant_gpu(X, dt, ld_dst, transpose=False, rowsum=False):
    rows, cols = X.shape
    src = (_bf16(X) if dt == L.CC_BF16 else torch.from_numpy(X)).cuda()
    out_rows = cols if transpose else rows
    dst = torch.zeros(out_rows, ld_dst, device='cuda', dtype=torch.uint8)
    sc = torch.zeros(out_rows, ld_dst // 32, device='cuda', dtype=torch.uint8)
    rs = torch.zeros(rows, device='cuda', dtype=torch.float32) if rowsum else None
    L.call('cc_quant_mx8', dt, L.ptr(src), rows, cols, cols, int(transpose), L.ptr(dst), ld_dst,
           L.ptr(sc), L.ptr(rs), L.stream_ptr())
    torch.cuda.synchronize()
    Xv = src.float().cpu().numpy()
    return Xv, dst.cpu().numpy(), sc.cpu().numpy(), (rs.cpu().numpy() if rowsum else None)


@pytest.mark.parametrize('dtype', ['bf16', 'fp32'])
@pytest.mark.parametrize('rows,cols,ld', [(7, 100, 128), (64, 512, 512), (33, 2049, 2176), (5, 22000, 22016)])
def test_quant_rows_bit_exact(dtype, rows, cols, ld):
    rng = np.random.default_rng(rows * 7 + cols)
    dt = L.CC_BF16 if dtype == 'bf16' else L.CC_F32
    X = _data(rng, rows, cols)
    Xv, q, s, _ = _quant_gpu(X, dt, ld)
    qr, sr = mx8_ref.quantize_rows(Xv, ld)
    assert np.array_equal(s, sr)
    assert np.array_equal(q, qr)


@pytest.mark.parametrize('dtype', ['bf16', 'fp32'])
@pytest.mark.parametrize('rows,cols,ld', [(64, 300, 128), (512, 1000, 512), (100, 257, 128), (1000, 1024, 1024),
                                          (130, 2112, 256)])
def test_quant_transposed_bit_exact(dtype, rows, cols, ld):
    rng = np.random.default_rng(rows + cols)
    X = _data(rng, rows, cols)
    Xv, q, s, _ = _quant_gpu(X, L.CC_BF16 if dtype == 'bf16' else L.CC_F32, ld, transpose=True)
    qr, sr = mx8_ref.quantize_rows(np.ascontiguousarray(Xv.T), ld)
    assert np.array_equal(s, sr)
    assert np.array_equal(q, qr)


def test_quant_rowsum():
    rng = np.random.default_rng(5)
    X = rng.standard_normal((300, 512)).astype(np.float32) * 1e-4
    Xv, q, s, rs = _quant_gpu(X, L.CC_BF16, 512, rowsum=True)
    np.testing.assert_allclose(rs, Xv.astype(np.float64).sum(1), rtol=1e-5, atol=1e-9)


def _mx8_operand(X, ld):
    q, s = mx8_ref.quantize_rows(X, ld)
    return (torch.from_numpy(q).cuda(), torch.from_numpy(s).cuda(), mx8_ref.dequantize_rows(q, s))


@pytest.mark.parametrize('M,N,K', [(128, 128, 128), (300, 260, 384), (512, 1000, 1024), (37, 129, 256)])
def test_mx8_gemm_store(M, N, K):
    rng = np.random.default_rng(M + N + K)
    A = _data(rng, M, K)
    B = _data(rng, N, K)
    qa, sa, Ad = _mx8_operand(A, K)
    qb, sb, Bd = _mx8_operand(B, K)
    bias = torch.from_numpy(rng.standard_normal(N).astype(np.float32)).cuda()
    Cf = torch.zeros(M, N, device='cuda', dtype=torch.float32)
    g = L.GemmArgs(dtype=L.CC_MX8, ta=0, tb=1, epilogue=L.CC_EPI_STORE, M=M, N=N, K=K, lda=K, ldb=K, ldc=N,
                   splits=1, A=qa.data_ptr(), B=qb.data_ptr(), bias=bias.data_ptr(), Cf=Cf.data_ptr(),
                   a_scale=sa.data_ptr(), b_scale=sb.data_ptr())
    L.call('cc_gemm', L.C.byref(g), L.stream_ptr())
    torch.cuda.synchronize()
    ref = Ad[:, :K] @ Bd[:, :K].T + bias.cpu().numpy()[None, :]
    got = Cf.cpu().numpy()
    # per-row relative error (rows span 60 binades).  The block-scaled MFMA does not accumulate as
    # an IEEE fp32 fmac chain: measured up to 1.1e-4 of the row's magnitude at K = 1024 (vs 6 % for
    # one e4m3 element), hence the bound.
    err = np.abs(got - ref).max(1) / np.maximum(np.abs(ref).max(1), 1e-300)
    assert (err < MFMA_TOL).all(), err.max()


def test_mx8_gemm_splitk_and_pair():
    """dX-shaped split-K (K = padded V) and the grouped dX + dW launch equal separate launches."""
    rng = np.random.default_rng(11)
    B_, d, V = 256, 256, 1000
    Vp = 1024
    dZ = rng.standard_normal((B_, V)).astype(np.float32) * 1e-6
    Wo = rng.standard_normal((d, V)).astype(np.float32) * 0.02
    D3t = np.abs(rng.standard_normal((d, B_))).astype(np.float32)
    qz, sz, Zd = _mx8_operand(dZ, Vp)
    qw, sw, Wd = _mx8_operand(Wo, Vp)
    qd, sd, Dd = _mx8_operand(D3t, B_)
    qzt, szt, Ztd = _mx8_operand(np.ascontiguousarray(dZ.T), B_)
    S = 4
    part = torch.zeros(S, B_, d, device='cuda', dtype=torch.float32)
    gW = torch.zeros(d, V, device='cuda', dtype=torch.float32)
    gx = L.GemmArgs(dtype=L.CC_MX8, ta=0, tb=1, epilogue=L.CC_EPI_SPLITK, M=B_, N=d, K=Vp, lda=Vp, ldb=Vp,
                    ldc=d, splits=S, A=qz.data_ptr(), B=qw.data_ptr(), Cf=part.data_ptr(),
                    a_scale=sz.data_ptr(), b_scale=sw.data_ptr())
    gw = L.GemmArgs(dtype=L.CC_MX8, ta=0, tb=1, epilogue=L.CC_EPI_STORE, M=d, N=V, K=B_, lda=B_, ldb=B_,
                    ldc=V, splits=1, A=qd.data_ptr(), B=qzt.data_ptr(), Cf=gW.data_ptr(),
                    a_scale=sd.data_ptr(), b_scale=szt.data_ptr())
    L.call('cc_gemm_pair', L.C.byref(gx), L.C.byref(gw), L.stream_ptr())
    torch.cuda.synchronize()
    ref_x = Zd @ Wd.T
    ref_w = Dd @ Ztd.T
    assert rel_err(part.sum(0).cpu().numpy(), ref_x) < MFMA_TOL
    assert rel_err(gW.cpu().numpy(), ref_w) < MFMA_TOL
    part2 = torch.zeros_like(part)
    gx.Cf = part2.data_ptr()
    L.call('cc_gemm', L.C.byref(gx), L.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(part, part2)


def test_mx8_bce_epilogue():
    rng = np.random.default_rng(3)
    Bn, d, V = 128, 256, 700
    D3 = np.abs(rng.standard_normal((Bn, d))).astype(np.float32)
    WoT = rng.standard_normal((V, d)).astype(np.float32) * 0.05
    qa, sa, Ad = _mx8_operand(D3, d)
    qb, sb, Bd = _mx8_operand(WoT, d)
    bias = rng.standard_normal(V).astype(np.float32) * 0.01
    y = rng.random((Bn, V)) < 0.05
    VW = (V + 31) // 32
    bits = np.zeros((Bn, VW), np.uint32)
    for b in range(Bn):
        for j in np.nonzero(y[b])[0]:
            bits[b, j >> 5] |= np.uint32(1 << (j & 31))
    yb = torch.from_numpy(bits.view(np.int32)).cuda()
    bias_d = torch.from_numpy(bias).cuda()
    dZ = torch.zeros(Bn, V, device='cuda', dtype=torch.bfloat16)
    dZt = torch.zeros(V, Bn, device='cuda', dtype=torch.bfloat16)
    tiles = np.zeros(1, np.int32)
    L.call('cc_gemm_grid', Bn, V, tiles.ctypes.data_as(L.C.c_void_p))
    part = torch.zeros(int(tiles[0]) * 4, device='cuda', dtype=torch.float64)
    loss = torch.zeros(1, device='cuda', dtype=torch.float64)
    ticket = torch.zeros(1, device='cuda', dtype=torch.int32)
    g = L.GemmArgs(dtype=L.CC_MX8, ta=0, tb=1, epilogue=L.CC_EPI_BCE, M=Bn, N=V, K=d, lda=d, ldb=d, ldc=V,
                   splits=1, A=qa.data_ptr(), B=qb.data_ptr(), bias=bias_d.data_ptr(), C=dZ.data_ptr(),
                   y_bits=yb.data_ptr(), scale=1.0 / (Bn * V), loss_partials=part.data_ptr(),
                   Ct=dZt.data_ptr(), ldct=Bn, loss_out=loss.data_ptr(), loss_scale=1.0 / (Bn * V),
                   ticket=ticket.data_ptr(), a_scale=sa.data_ptr(), b_scale=sb.data_ptr())
    L.call('cc_gemm', L.C.byref(g), L.stream_ptr())
    torch.cuda.synchronize()
    z = Ad @ Bd.T + bias[None, :]
    yy = y.astype(np.float64)
    ref_loss = (np.maximum(z, 0) - z * yy + np.log1p(np.exp(-np.abs(z)))).mean()
    ref_dz = (1 / (1 + np.exp(-z)) - yy) / (Bn * V)
    assert abs(loss.item() - ref_loss) / ref_loss < MFMA_TOL
    assert rel_err(dZ.float().cpu().numpy(), ref_dz) < 5e-3
    assert torch.equal(dZt.t().contiguous(), dZ)


@pytest.mark.parametrize('M,N,K,epi,splits', [(512, 1000, 1024, 'store', 1), (300, 260, 384, 'store', 1),
                                               (37, 129, 256, 'store', 1), (1024, 2100, 512, 'store', 1),
                                               (512, 1024, 2944, 'splitk', 8), (512, 256, 1024, 'splitk', 32),
                                               (512, 1000, 1024, 'bce', 1), (300, 700, 256, 'bce', 1)])
def test_mx8_wide_bit_identical_to_128_kernel(M, N, K, epi, splits):
    """The 256 x 256 LDS-DMA kernel (mx8gemm.hip, cc_gemm's MX8 STORE / SPLITK / BCE path) runs the
    same MFMA sequence per output as the 128 x 128 kernel: bitwise equal products, ragged edges
    included, empty K splits written as zeros; BCE outputs to the rounding of its epilogue math."""
    rng = np.random.default_rng(M * 3 + N + K)
    qa, sa, _ = _mx8_operand(_data(rng, M, K), K)
    qb, sb, _ = _mx8_operand(_data(rng, N, K), K)
    bias = torch.from_numpy(rng.standard_normal(N).astype(np.float32)).cuda()
    bits = torch.from_numpy(rng.integers(0, 2**31, (M, (N + 31) // 32), dtype=np.int64).astype(np.int32)).cuda()
    outs = []
    for kern in ('cc_gemm_tile128', 'cc_gemm'):
        if epi == 'store':
            Cf = torch.full((M, N), 7.0, device='cuda')
            Cb = torch.zeros(M, N, device='cuda', dtype=torch.bfloat16)
            g = L.GemmArgs(dtype=L.CC_MX8, ta=0, tb=1, epilogue=L.CC_EPI_STORE, M=M, N=N, K=K, lda=K, ldb=K,
                           ldc=N, splits=1, A=qa.data_ptr(), B=qb.data_ptr(), bias=bias.data_ptr(),
                           Cf=Cf.data_ptr(), C=Cb.data_ptr(), a_scale=sa.data_ptr(), b_scale=sb.data_ptr())
            L.call(kern, L.C.byref(g), L.stream_ptr())
            outs.append((Cf, Cb))
        elif epi == 'bce':
            dZ = torch.zeros(M, N, device='cuda', dtype=torch.bfloat16)
            dZt = torch.zeros(N, M + 4, device='cuda', dtype=torch.bfloat16)
            part = torch.zeros(4096, device='cuda', dtype=torch.float64)
            loss = torch.zeros(1, device='cuda', dtype=torch.float64)
            ticket = torch.zeros(1, device='cuda', dtype=torch.int32)
            g = L.GemmArgs(dtype=L.CC_MX8, ta=0, tb=1, epilogue=L.CC_EPI_BCE, M=M, N=N, K=K, lda=K, ldb=K, ldc=N,
                           splits=1, A=qa.data_ptr(), B=qb.data_ptr(), bias=bias.data_ptr(), C=dZ.data_ptr(),
                           y_bits=bits.data_ptr(), scale=1.0 / (M * N), loss_partials=part.data_ptr(),
                           Ct=dZt.data_ptr(), ldct=M + 4, loss_out=loss.data_ptr(), loss_scale=1.0 / (M * N),
                           ticket=ticket.data_ptr(), a_scale=sa.data_ptr(), b_scale=sb.data_ptr())
            L.call(kern, L.C.byref(g), L.stream_ptr())
            torch.cuda.synchronize()
            outs.append((dZ, dZt[:, :M], ticket))
            losses = locals().get('losses', []) + [loss.item()]
        else:
            P = torch.full((splits, M, N), 7.0, device='cuda')
            g = L.GemmArgs(dtype=L.CC_MX8, ta=0, tb=1, epilogue=L.CC_EPI_SPLITK, M=M, N=N, K=K, lda=K, ldb=K,
                           ldc=N, splits=splits, A=qa.data_ptr(), B=qb.data_ptr(), Cf=P.data_ptr(),
                           a_scale=sa.data_ptr(), b_scale=sb.data_ptr())
            L.call(kern, L.C.byref(g), L.stream_ptr())
            outs.append((P,))
    torch.cuda.synchronize()
    if epi == 'bce':
        # the 256 x 256 kernel's BCE math is decout.hip's (hardware exp2 / rcp, one log2 per 4
        # factors): dz within a bf16 ulp, the loss to float rounding; dZ^T is its own dZ transposed
        (z0, zt0, t0), (z1, zt1, t1) = outs
        assert torch.equal(zt1.t(), z1) and torch.equal(zt0.t(), z0)
        assert ((z1.float() - z0.float()).abs() <= z0.float().abs() * 2.0 ** -7 + 1e-30).all()
        assert abs(losses[0] - losses[1]) <= 1e-5 * abs(losses[0])
        assert t0.item() == 0 and t1.item() == 0
        return
    for x, y in zip(*outs):
        assert torch.equal(x, y)


@pytest.mark.parametrize('M,N,K', [(512, 1000, 1024), (256, 22000, 256), (128, 300, 128)])
def test_mx8_bce_q_matches_quantiser(M, N, K):
    """cc_gemm_mx8_bce_q (config 5's BCE product making dZ's MX-FP8 images in its epilogue) ==
    the same product's bf16 dZ / dZ^T run through cc_quant_mx8: codes and scales bit for bit
    (padded columns [N, ldzq) included), the bias gradient to fp32 rounding, the same loss."""
    rng = np.random.default_rng(M + N)
    qa, sa, _ = _mx8_operand(rng.standard_normal((M, K)).astype(np.float32), K)
    qb, sb, _ = _mx8_operand(rng.standard_normal((N, K)).astype(np.float32) * 0.05, K)
    bias = torch.from_numpy(rng.standard_normal(N).astype(np.float32) * 0.1).cuda()
    bits = torch.from_numpy(rng.integers(0, 2**31, (M, (N + 31) // 32), dtype=np.int64).astype(np.int32)).cuda()
    Np = (N + 127) // 128 * 128

    def run(fused):
        dZ = torch.zeros(M, N, device='cuda', dtype=torch.bfloat16)
        dZt = torch.zeros(N, M, device='cuda', dtype=torch.bfloat16)
        part = torch.zeros(4096, device='cuda', dtype=torch.float64)
        loss = torch.zeros(1, device='cuda', dtype=torch.float64)
        ticket = torch.zeros(1, device='cuda', dtype=torch.int32)
        zq = torch.full((M, Np), 0x55, device='cuda', dtype=torch.uint8)
        zqs = torch.full((M, Np // 32), 0x55, device='cuda', dtype=torch.uint8)
        ztq = torch.full((N, M), 0x55, device='cuda', dtype=torch.uint8)
        ztqs = torch.full((N, M // 32), 0x55, device='cuda', dtype=torch.uint8)
        gb = torch.full((N,), 3.0, device='cuda')
        g = L.GemmArgs(dtype=L.CC_MX8, ta=0, tb=1, epilogue=L.CC_EPI_BCE, M=M, N=N, K=K, lda=K, ldb=K, ldc=N,
                       splits=1, A=qa.data_ptr(), B=qb.data_ptr(), bias=bias.data_ptr(),
                       C=None if fused else dZ.data_ptr(), y_bits=bits.data_ptr(), scale=1.0 / (M * N),
                       loss_partials=part.data_ptr(), Ct=None if fused else dZt.data_ptr(), ldct=M,
                       loss_out=loss.data_ptr(), loss_scale=1.0 / (M * N), ticket=ticket.data_ptr(),
                       a_scale=sa.data_ptr(), b_scale=sb.data_ptr())
        if fused:
            L.call('cc_gemm_mx8_bce_q', L.C.byref(g), L.ptr(zq), Np, L.ptr(zqs), L.ptr(ztq), M, L.ptr(ztqs),
                   L.ptr(gb), L.stream_ptr())
        else:
            L.call('cc_gemm', L.C.byref(g), L.stream_ptr())
            L.call('cc_quant_mx8', L.CC_BF16, L.ptr(dZ), M, N, N, 0, L.ptr(zq), Np, L.ptr(zqs), None, L.stream_ptr())
            L.call('cc_quant_mx8', L.CC_BF16, L.ptr(dZt), N, M, M, 0, L.ptr(ztq), M, L.ptr(ztqs), L.ptr(gb),
                   L.stream_ptr())
        torch.cuda.synchronize()
        return zq, zqs, ztq, ztqs, gb, loss.item()

    ref, got = run(False), run(True)
    for a, b in zip(ref[:4], got[:4]):
        assert torch.equal(a, b)
    torch.testing.assert_close(got[4], ref[4], rtol=1e-5, atol=1e-12)
    assert abs(got[5] - ref[5]) <= 1e-9 * abs(ref[5])


@pytest.mark.parametrize('M,N,K', [(512, 1000, 1024), (128, 700, 256)])
def test_mx8_bce_q2_pair_equals_separate_launches(M, N, K):
    """cc_gemm_mx8_bce_q2 (config 5: the BCE product with the regulariser's logits as extra blocks of
    the same launch) == cc_gemm_mx8_bce_q and a separate cc_gemm of the second product, bit for bit;
    M = 512 spans two 256-row tiles (bias gradient added onto a zeroing kernel's zeros), M = 128 one
    (stored)."""
    rng = np.random.default_rng(M * 5 + N)
    qa, sa, _ = _mx8_operand(rng.standard_normal((M, K)).astype(np.float32), K)
    qb, sb, _ = _mx8_operand(rng.standard_normal((N, K)).astype(np.float32) * 0.05, K)
    qa2, sa2, _ = _mx8_operand(rng.standard_normal((M, K)).astype(np.float32), K)
    qb2, sb2, _ = _mx8_operand(rng.standard_normal((N, K)).astype(np.float32) * 0.05, K)
    bias = torch.from_numpy(rng.standard_normal(N).astype(np.float32) * 0.1).cuda()
    bias2 = torch.from_numpy(rng.standard_normal(N).astype(np.float32) * 0.1).cuda()
    bits = torch.from_numpy(rng.integers(0, 2**31, (M, (N + 31) // 32), dtype=np.int64).astype(np.int32)).cuda()
    Np = (N + 127) // 128 * 128

    def run(paired):
        u8 = dict(device='cuda', dtype=torch.uint8)
        part = torch.zeros(4096, device='cuda', dtype=torch.float64)
        loss = torch.zeros(1, device='cuda', dtype=torch.float64)
        ticket = torch.zeros(1, device='cuda', dtype=torch.int32)
        zq, zqs = torch.full((M, Np), 0x55, **u8), torch.full((M, Np // 32), 0x55, **u8)
        ztq, ztqs = torch.full((N, M), 0x55, **u8), torch.full((N, M // 32), 0x55, **u8)
        gb = torch.full((N,), 3.0, device='cuda')
        Z2 = torch.full((M, N), 7.0, device='cuda')
        g = L.GemmArgs(dtype=L.CC_MX8, ta=0, tb=1, epilogue=L.CC_EPI_BCE, M=M, N=N, K=K, lda=K, ldb=K, ldc=N,
                       splits=1, A=qa.data_ptr(), B=qb.data_ptr(), bias=bias.data_ptr(), y_bits=bits.data_ptr(),
                       scale=1.0 / (M * N), loss_partials=part.data_ptr(), ldct=M, loss_out=loss.data_ptr(),
                       loss_scale=1.0 / (M * N), ticket=ticket.data_ptr(), a_scale=sa.data_ptr(),
                       b_scale=sb.data_ptr())
        g2 = L.GemmArgs(dtype=L.CC_MX8, ta=0, tb=1, epilogue=L.CC_EPI_STORE, M=M, N=N, K=K, lda=K, ldb=K, ldc=N,
                        splits=1, A=qa2.data_ptr(), B=qb2.data_ptr(), bias=bias2.data_ptr(), Cf=Z2.data_ptr(),
                        a_scale=sa2.data_ptr(), b_scale=sb2.data_ptr())
        if paired:
            L.call('cc_gemm_mx8_bce_q2', L.C.byref(g), L.ptr(zq), Np, L.ptr(zqs), L.ptr(ztq), M, L.ptr(ztqs),
                   L.ptr(gb), L.C.byref(g2), L.stream_ptr())
        else:
            L.call('cc_gemm_mx8_bce_q', L.C.byref(g), L.ptr(zq), Np, L.ptr(zqs), L.ptr(ztq), M, L.ptr(ztqs),
                   L.ptr(gb), L.stream_ptr())
            L.call('cc_gemm', L.C.byref(g2), L.stream_ptr())
        torch.cuda.synchronize()
        assert int(ticket.item()) == 0
        return zq, zqs, ztq, ztqs, gb, loss, Z2

    for a, b in zip(run(False), run(True)):
        assert torch.equal(a, b)


@pytest.mark.parametrize('dtype', ['bf16', 'fp32'])
@pytest.mark.parametrize('rows,cols,ld_t,ld_r', [(1024, 2200, 1024, 2304), (256, 1000, 256, 1024),
                                                 (100, 257, 128, 384), (130, 64, 256, 128)])
def test_quant_both_images_bit_exact(dtype, rows, cols, ld_t, ld_r):
    """cc_quant_mx8_both (config 5's Wo images after Adam, one read) == cc_quant_mx8 transposed and
    by rows, codes and scales bit for bit, padding included."""
    rng = np.random.default_rng(rows + 3 * cols)
    dt = L.CC_BF16 if dtype == 'bf16' else L.CC_F32
    X = _data(rng, rows, cols)
    src = (_bf16(X) if dt == L.CC_BF16 else torch.from_numpy(X)).cuda()
    u8 = dict(device='cuda', dtype=torch.uint8)
    imgs = []
    for both in (False, True):
        qt, st = torch.full((cols, ld_t), 0x5A, **u8), torch.full((cols, ld_t // 32), 0x5A, **u8)
        qr, sr = torch.full((rows, ld_r), 0x5A, **u8), torch.full((rows, ld_r // 32), 0x5A, **u8)
        if both:
            L.call('cc_quant_mx8_both', dt, L.ptr(src), rows, cols, cols, L.ptr(qt), ld_t, L.ptr(st),
                   L.ptr(qr), ld_r, L.ptr(sr), L.stream_ptr())
        else:
            L.call('cc_quant_mx8', dt, L.ptr(src), rows, cols, cols, 1, L.ptr(qt), ld_t, L.ptr(st), None, L.stream_ptr())
            L.call('cc_quant_mx8', dt, L.ptr(src), rows, cols, cols, 0, L.ptr(qr), ld_r, L.ptr(sr), None, L.stream_ptr())
        imgs.append((qt, st, qr, sr))
    torch.cuda.synchronize()
    for a, b in zip(*imgs):
        assert torch.equal(a, b)


def test_softmax_kl_q_matches_quantiser():
    """cc_dec_softmax_kl_q (config 5's regulariser branch) == cc_dec_softmax_kl_fused + cc_quant_mx8
    of its bf16 dZ: dZ, the KL partials, codes and scales bit for bit, a padding row included."""
    rng = np.random.default_rng(7)
    B_, V = 64, 3000
    Vp = (V + 127) // 128 * 128
    Z2 = torch.from_numpy(rng.standard_normal((B_, V)).astype(np.float32) * 3).cuda()
    Mt = rng.random((50, V)).astype(np.float32)
    Mt /= Mt.sum(1, keepdims=True)
    Mt = torch.from_numpy(Mt).cuda()
    idx = torch.from_numpy(rng.integers(0, 50, B_).astype(np.int32)).cuda()
    idx[5] = -1
    outs = []
    for fused in (False, True):
        dZ = torch.zeros(B_, V, device='cuda', dtype=torch.bfloat16)
        part = torch.zeros(B_, device='cuda', dtype=torch.float64)
        zq = torch.full((B_, Vp), 0x5A, device='cuda', dtype=torch.uint8)
        zqs = torch.full((B_, Vp // 32), 0x5A, device='cuda', dtype=torch.uint8)
        if fused:
            L.call('cc_dec_softmax_kl_q', L.ptr(Z2), B_, V, L.ptr(Mt), L.ptr(idx), 0.1 / B_, L.ptr(dZ), L.ptr(part),
                   L.ptr(zq), Vp, L.ptr(zqs), L.stream_ptr())
        else:
            L.call('cc_dec_softmax_kl_fused', L.CC_BF16, L.ptr(Z2), B_, V, L.ptr(Mt), L.ptr(idx), 0.1 / B_,
                   L.ptr(dZ), L.ptr(part), L.stream_ptr())
            L.call('cc_quant_mx8', L.CC_BF16, L.ptr(dZ), B_, V, V, 0, L.ptr(zq), Vp, L.ptr(zqs), None, L.stream_ptr())
        outs.append((dZ, part, zq, zqs))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
