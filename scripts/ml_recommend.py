#!/usr/bin/env python3
"""Drop-in for src/scripts/ml_recommend.py: `ml_recommend.py cube_name [amount [root]]`.

Same arguments and output as the reference (ml_recommend.py:8-18, 94-116): with a root given the
reference switches to JSON mode and prints nothing (:12-16, :110); kept.  Extra optional flags:
--model-dir (default ml_files/neg, as :54) and --id-map."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cubecobrarecommender_amd import api  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('cube_name')
    ap.add_argument('amount', nargs='?', type=int, default=100)
    ap.add_argument('root', nargs='?', default=None)
    ap.add_argument('--model-dir', default='ml_files/neg')
    ap.add_argument('--id-map', default='ml_files/recommender_id_map.json')
    a = ap.parse_args(argv)
    non_json = a.root is None
    root = a.root or 'https://cubecobra.com'
    print('Getting Cube List . . . \n')
    names = api.fetch_cube_list(a.cube_name, root)
    print('Loading Card Name Lookup . . . \n')
    int_to_card, card_to_int = api.load_id_map(a.id_map)
    print('Creating Cube Vector . . . \n')
    cube_indices = api.cube_indices_of(names, card_to_int)
    print('Loading Model . . . \n')
    model = api.get_model(a.model_dir)
    print('Generating Recommendations . . . \n')
    return api.recommend(model, cube_indices, a.amount, int_to_card, non_json=non_json)


if __name__ == '__main__':
    main()
