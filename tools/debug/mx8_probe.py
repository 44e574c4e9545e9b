"""Probe the block-scaled MFMA scale/element mapping and the fp8 quantiser on the GPU."""
import numpy as np
import torch
from cubecobrarecommender_amd import _lib as L
from oracle import mx8_ref

L.lib()


def gemm(qa, sa, qb, sb, M, N, K):
    Cf = torch.zeros(M, N, device='cuda')
    A, SA, B, SB = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (qa, sa, qb, sb)]
    g = L.GemmArgs(dtype=L.CC_MX8, ta=0, tb=1, epilogue=L.CC_EPI_STORE, M=M, N=N, K=K, lda=K, ldb=K, ldc=N,
                   splits=1, A=A.data_ptr(), B=B.data_ptr(), Cf=Cf.data_ptr(), a_scale=SA.data_ptr(),
                   b_scale=SB.data_ptr())
    L.call('cc_gemm', L.C.byref(g), L.stream_ptr())
    torch.cuda.synchronize()
    return Cf.cpu().numpy()


M = N = 64
K = 128
one = 0x38
qa = np.full((M, K), one, np.uint8)
qb = np.full((N, K), one, np.uint8)
sa = np.full((M, K // 32), 127, np.uint8)
sb = np.full((N, K // 32), 127, np.uint8)
C = gemm(qa, sa, qb, sb, M, N, K)
print('unit', np.unique(C))
for (m, b) in [(3, 0), (3, 1), (3, 2), (3, 3), (40, 1)]:
    s2 = sa.copy()
    s2[m, b] = 131
    C = gemm(qa, s2, qb, sb, M, N, K)
    dev = np.argwhere(C != 128)
    rows = sorted(set(dev[:, 0].tolist()))
    print('A scale', (m, b), 'rows hit', rows[:10], 'vals', np.unique(C[C != 128])[:5], 'n', len(dev))
for (n, b) in [(5, 0), (5, 1), (37, 3)]:
    s2 = sb.copy()
    s2[n, b] = 131
    C = gemm(qa, sa, qb, s2, M, N, K)
    dev = np.argwhere(C != 128)
    cols = sorted(set(dev[:, 1].tolist()))
    print('B scale', (n, b), 'cols hit', cols[:10], 'vals', np.unique(C[C != 128])[:5], 'n', len(dev))
# element mapping: one element = 2.0 (0x40)
for (m, k) in [(3, 0), (3, 31), (3, 32), (3, 64), (3, 100)]:
    q2 = qa.copy()
    q2[m, k] = 0x40
    C = gemm(q2, sa, qb, sb, M, N, K)
    dev = np.argwhere(C != 128)
    print('A elem', (m, k), 'rows', sorted(set(dev[:, 0].tolist()))[:5], 'vals', np.unique(C[C != 128])[:3])
# scale on a block with a distinct element pattern: A row 3 block 1 elements = 2.0, scale x16
q2 = qa.copy(); q2[3, 32:64] = 0x40
s2 = sa.copy(); s2[3, 1] = 131
C = gemm(q2, s2, qb, sb, M, N, K)
print('block1 x2 elems x16 scale ->', np.unique(C[3]), 'expect', 96 + 32 * 2 * 16)

# quantiser codes
rng = np.random.default_rng(0)
X = (rng.standard_normal((4, 256)) * 0.01).astype(np.float32)
src = torch.from_numpy(X).cuda()
dst = torch.zeros(4, 256, device='cuda', dtype=torch.uint8)
sc = torch.zeros(4, 8, device='cuda', dtype=torch.uint8)
L.call('cc_quant_mx8', L.CC_F32, L.ptr(src), 4, 256, 256, 0, L.ptr(dst), 256, L.ptr(sc), None, L.stream_ptr())
torch.cuda.synchronize()
q, s = mx8_ref.quantize_rows(X, 256)
g = dst.cpu().numpy()
print('scales equal', np.array_equal(s, sc.cpu().numpy()))
bad = np.argwhere(g != q)
print('code mismatches', len(bad))
for r, c in bad[:12]:
    e = int(s[r, c // 32]) - 127
    print(r, c, X[r, c], X[r, c] * 2.0 ** -e, 'gpu', hex(g[r, c]), mx8_ref.e4m3_decode(g[r, c]), 'ref', hex(q[r, c]),
          mx8_ref.e4m3_decode(q[r, c]))
