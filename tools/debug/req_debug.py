"""Debug: run cc_recommend_fp32 once and inspect the top-N sort workspace."""
import numpy as np
import torch
import sys
sys.path.insert(0, '.')
from cubecobrarecommender_amd import _lib as L
from cubecobrarecommender_amd.layout import Layout
from oracle import model_ref, infer_ref

V, d = 20884, 512
P = model_ref.init_params(V, d, seed=20250301, bias_std=0.01)
params = torch.from_numpy(Layout(V, d).pack(P)).cuda()
ws = torch.zeros(int(L.lib().cc_recommend_ws_size(V, d)) // 4 + 64, dtype=torch.int32, device='cuda')
probs = torch.zeros(V, device='cuda')
res = torch.zeros(1 + 3 * V, dtype=torch.int32, device='cuda')
cube = np.sort(np.random.default_rng(5).choice(V, 45, replace=False)).astype(np.int32)
req = torch.from_numpy(np.concatenate([[len(cube), 100], cube]).astype(np.int32)).cuda()
torch.cuda.synchronize()
L.call('cc_recommend_fp32', L.ptr(params), V, d, L.ptr(req), len(cube), L.ptr(ws), L.ptr(probs), L.ptr(res),
       L.stream_ptr())
torch.cuda.synchronize()
p = probs.cpu().numpy()
want_p = infer_ref.recommend_probs(P, cube)
print('probs exact', np.array_equal(p, want_p))
cap = -(-V // 32)
fpart = ((cap * d + 64 + d) * 4 + 255) // 256 * 256
w = ws.cpu().numpy().view(np.uint8)[fpart:]
v = (V * 4 + 255) // 256 * 256
kA = w[:V * 4].view(np.uint32)
iA = w[v:v + V * 4].view(np.uint32)
nt = -(-V // 1024)
H = w[4 * v:4 * v + 3 * nt * 1024 * 4].view(np.uint32).reshape(3, nt, 1024)
bits = w[4 * v + ((3 * nt * 1024 * 4 + 255) // 256 * 256):][:(V + 31) // 32 * 4].view(np.uint32)
print('bits set', int(np.unpackbits(bits.view(np.uint8)).sum()), 'expected', len(cube))
inc = np.zeros(V, bool); inc[cube] = True
exp_keys = np.where(inc, 0, p.view(np.uint32) + 1).astype(np.uint32)
print('H0 total', H[0].sum(), 'per tile', H[0].sum(1)[:3], H[0].sum(1)[-1])
print('H1 total', H[1].sum(), 'H2 total', H[2].sum())
exp_h0 = np.zeros((nt, 1024), np.int64)
np.add.at(exp_h0, (np.arange(V) // 1024, exp_keys & 1023), 1)
print('H0 matches', np.array_equal(H[0], exp_h0))
r = res.cpu().numpy()
print('n_add', r[0], 'adds', r[1:6], 'expected', infer_ref.top_n(want_p, cube, 100)[0][:5])
