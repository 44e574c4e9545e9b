"""Drop-in for the reference's web/ml_recommend_web.py:get_ml_recommend (same signature/result).

The model is loaded once per process and stays resident in HBM (the reference reloads it on every
request, ml_recommend_web.py:37); forward and ranking run on the GPU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cubecobrarecommender_amd import api  # noqa: E402

ROOT = "https://cubecobra.com"


def get_ml_recommend(cube_name, amount, root=ROOT, non_json=False,
                     model_dir='./ml_files/recommender', id_map='./ml_files/recommender_id_map.json'):
    card_names = api.fetch_cube_list(cube_name, root)                  # :11-19
    int_to_card, card_to_int = api.load_id_map(id_map)                  # :21-23
    cube_indices = api.cube_indices_of(card_names, card_to_int)         # :27-32
    model = api.get_model(model_dir)                                    # :37 (resident here)
    output = api.recommend(model, cube_indices, amount, int_to_card, non_json=non_json,
                           print_cuts=False)                           # :50-64 (additions only)
    if not non_json:
        return output
