"""The recommend call surface of ``src/scripts/ml_recommend.py`` and ``web/ml_recommend_web.py``,
with the model resident (the reference reloads the ~390 MB SavedModel per web request,
ml_recommend_web.py:37) and the forward + ranking on the GPU (cc_infer_*_fp32 + cc_topn)."""
import json
import os
import threading
import urllib.request

import numpy as np

from .names import normalize

ROOT = 'https://cubecobra.com'
_models = {}
_lock = threading.Lock()


def load_id_map(path='ml_files/recommender_id_map.json'):
    """ml_recommend.py:34-36: {"<int>": "<name>"} -> (int_to_card, card_to_int)."""
    int_to_card = {int(k): v for k, v in json.load(open(path, 'r')).items()}
    return int_to_card, {v: k for k, v in int_to_card.items()}


def fetch_cube_list(cube_name, root=ROOT):
    """ml_recommend.py:22-30: GET <root>/cube/api/cubelist/<cube_name> -> list of names.
    A local directory (or file://) root reads <root>/cube/api/cubelist/<cube_name> from disk."""
    if root.startswith('file://'):
        root = root[len('file://'):]
    if os.path.isdir(root):
        with open(os.path.join(root, 'cube', 'api', 'cubelist', cube_name), 'rb') as fh:
            return fh.read().decode('utf8').split('\n')
    with urllib.request.urlopen(root + '/cube/api/cubelist/' + cube_name) as fp:
        return fp.read().decode('utf8').split('\n')


def cube_indices_of(card_names, card_to_int):
    """ml_recommend.py:42-47: unknown names (custom cards) are skipped; duplicates kept in order."""
    out = []
    for name in card_names:
        idx = card_to_int.get(normalize(name))
        if idx is not None:
            out.append(idx)
    return out


def get_model(path):
    """Resident model per checkpoint directory (thread-safe; Flask runs threaded)."""
    from .model import load_model
    with _lock:
        if path not in _models:
            _models[path] = load_model(path)
        return _models[path]


def recommend(model, cube_indices, amount, int_to_card, non_json=False, print_fn=print, print_cuts=True):
    """ml_recommend.py:78-116 / ml_recommend_web.py:39-67 on the GPU.  Returns
    {"additions": {name: p}, "cuts": {name: p}} (additions empty in non_json mode, as the reference
    prints instead of storing them).  print_cuts: in non_json mode also print the lowest-scoring
    cuts — the CLI does (ml_recommend.py:110-116), the web function does not
    (ml_recommend_web.py:50-67 prints only the additions)."""
    out = model.recommender().recommend(cube_indices, amount)
    output = {'additions': {}, 'cuts': {}}
    for idx, p in zip(out['additions'].tolist(), out['add_vals'].tolist()):
        card = int_to_card[idx]
        if non_json:
            print_fn(card)
        else:
            output['additions'][card] = p
    for idx, p in zip(list(cube_indices), out['cut_vals'].tolist()):
        output['cuts'][int_to_card[idx]] = p
    if non_json and print_cuts:   # ml_recommend.py:110-116: lowest-scoring cuts
        cards = list(output['cuts'].keys())
        vals = list(output['cuts'].values())
        rank_cuts = np.argsort(np.array(vals), kind='stable')
        print_fn('\n')
        for i in range(min(int(amount), len(cards))):
            print_fn(cards[rank_cuts[i]], vals[rank_cuts[i]])
    return output
