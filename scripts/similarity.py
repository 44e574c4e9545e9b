#!/usr/bin/env python3
"""Drop-in for src/scripts/similarity.py: `similarity.py card_name N`.

Same arguments and output lines as the reference (similarity.py:7-34: underscores in the name
become spaces; prints "<rank>: <card> <dist>" for the N most similar cards, the card itself
first).  Model ml_files/high_req (:15) unless --model-dir; --id-map as ml_recommend.py."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cubecobrarecommender_amd import api  # noqa: E402
from cubecobrarecommender_amd.similarity import similar_cards  # noqa: E402


def main(argv=None, print_fn=print):
    ap = argparse.ArgumentParser()
    ap.add_argument('name')
    ap.add_argument('N', type=int)
    ap.add_argument('--model-dir', default='ml_files/high_req')
    ap.add_argument('--id-map', default='ml_files/recommender_id_map.json')
    a = ap.parse_args(argv)
    name = a.name.replace('_', ' ')
    int_to_card, card_to_int = api.load_id_map(a.id_map)
    model = api.get_model(a.model_dir)
    rows = similar_cards(model, name, a.N, int_to_card, card_to_int)
    for rank, card, dist in rows:
        print_fn(str(rank) + ':', card, dist)
    if a.N > len(int_to_card):   # the reference's ranked[i] runs past the end (similarity.py:32-34)
        raise IndexError(f'index {len(int_to_card)} is out of bounds for axis 0 with size {len(int_to_card)}')
    return rows


if __name__ == '__main__':
    main()
