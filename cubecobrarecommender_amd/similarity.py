"""Card similarity (src/scripts/similarity.py:19-31) on the GPU: the encoder on
the identity (cc_infer_encode_fp32 on one-card rows, the same kernel as model.encoder) gives the
[V, 64] card embeddings, cached per model; cc_similar_cards scores every card against the query
with Keras CosineSimilarity and returns the N smallest distances (argsort order, ties -> lower
index first)."""
import numpy as np
import torch

from . import _lib as L


def card_embeddings(model):
    """model.encoder(I[V, V]) -> [V, 64] fp32 on the device (cached on the model object)."""
    rec = model.recommender() if hasattr(model, 'recommender') else model
    emb = getattr(rec, '_card_emb', None)
    if emb is None:
        emb = rec.encode_lists([[i] for i in range(rec.V)])
        rec._card_emb = emb
    return emb


SIM_NMAX = 4096   # cc_similar_cards' in-LDS selection limit (csrc/similarity.hip)


def similar(emb, idx, N):
    """(indices [N] int64, dists [N] float32) of the N cards closest to card idx (idx itself first
    unless another card ties at -1).  N <= 0 gives empty arrays (the reference's loop prints
    nothing); N is capped at V.  Up to SIM_NMAX the selection runs in cc_similar_cards' one-workgroup
    radix select; beyond it the same kernel's distance vector is fully sorted on the device
    (stable, ties -> lower index, as numpy's argsort(kind='stable'))."""
    emb = emb.contiguous()
    V, K = emb.shape
    N = min(int(N), V)
    if N <= 0:
        return np.zeros(0, np.int64), np.zeros(0, np.float32)
    dev = emb.device
    ws = torch.empty(int(L.lib().cc_similar_ws_size(V)) // 8 + 1, device=dev, dtype=torch.int64)
    n_sel = min(N, SIM_NMAX)
    out_idx = torch.empty(n_sel, device=dev, dtype=torch.int32)
    out_d = torch.empty(n_sel, device=dev, dtype=torch.float32)
    dist_all = torch.empty(V, device=dev, dtype=torch.float32)
    L.call('cc_similar_cards', L.ptr(emb), V, K, int(idx), n_sel, L.ptr(out_idx), L.ptr(out_d),
           L.ptr(dist_all), L.ptr(ws), L.stream_ptr())
    if N > SIM_NMAX:
        order = torch.sort(dist_all, stable=True).indices[:N]
        out_idx, out_d = order, dist_all[order]
    torch.cuda.current_stream().synchronize()
    return out_idx.cpu().numpy().astype(np.int64), out_d.cpu().numpy()


def similar_cards(model, name, N, int_to_card, card_to_int):
    """similarity.py:19-31 for one card name: [(rank, name, dist)] for ranks 1..N."""
    emb = card_embeddings(model)
    idx, dists = similar(emb, card_to_int[name], N)
    return [(i + 1, int_to_card[int(j)], float(dv)) for i, (j, dv) in enumerate(zip(idx, dists))]
