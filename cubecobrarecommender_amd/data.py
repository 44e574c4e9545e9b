"""Host-side data plumbing for the training CLI (outside the hot path; SURVEY §2 row 4 marks the
JSON loaders out of scope — restated here only so scripts/train.py can run on real data):
card maps (src/non_ml/utils.py:27-47), cube lists (:49-73) and M / M~ (utils.py:75-91,
train.py:69-71, computed on the GPU by cubecobrarecommender_amd.adjacency)."""
import json
import os

import numpy as np


def get_card_maps(map_file):
    """utils.py:27-47 (the exclusion hook is dead code in the reference and is not restated)."""
    names = json.load(open(map_file, 'rb'))
    name_lookup, card_to_int = {}, {}
    for n, (name, ids) in enumerate(names.items()):
        card_to_int[name] = n
        for idx in ids:
            name_lookup[idx] = name
    int_to_card = {v: k for k, v in card_to_int.items()}
    return len(card_to_int), name_lookup, card_to_int, int_to_card


def build_cube_lists(cube_folder, name_lookup, card_to_int):
    """utils.py:49-73 as card-index lists (the reference builds a dense f64 [C, V] matrix)."""
    lists = []
    for f in sorted(os.listdir(cube_folder)):
        for cube in json.load(open(os.path.join(cube_folder, f), 'rb')):
            ids = []
            for card in cube['cards']:
                name = name_lookup.get(card['cardID'])
                if name is not None and card_to_int.get(name) is not None:
                    ids.append(card_to_int[name])
            lists.append(np.unique(np.asarray(ids, np.int64)))
    return lists


def lists_to_csr(lists):
    indptr = np.zeros(len(lists) + 1, np.int64)
    indptr[1:] = np.cumsum([len(l) for l in lists])
    idx = np.concatenate(lists).astype(np.int32) if lists else np.zeros(0, np.int32)
    return indptr, idx
