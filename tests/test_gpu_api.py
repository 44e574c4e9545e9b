"""GPU: the drop-in call surface — DataGenerator, CC_Recommender.compile/fit/save, load_model,
model.encoder/decoder, get_ml_recommend / ml_recommend.py — against the CPU oracle."""
import json
import os

import numpy as np
import pytest
import torch

from cubecobrarecommender_amd import api
from cubecobrarecommender_amd.generator import DataGenerator
from cubecobrarecommender_amd.model import CC_Recommender, load_model
from oracle import infer_ref, noise_ref
from tests.gpu_helpers import problem

pytestmark = pytest.mark.gpu


def test_datagenerator_batches_match_oracle():
    V, C, B = 600, 128, 16
    lists, Mt, ns = problem(7, C, V, (10, 30, 60))
    gen = DataGenerator(Mt.astype(np.float32), lists, batch_size=B, noise=0.2, seed=5)
    assert len(gen) == C // B
    assert np.allclose(gen.neg_sampler, noise_ref.neg_sampler_of(Mt.astype(np.float32)), rtol=1e-6)
    cdf = noise_ref.cdf_of(gen.neg_sampler)
    for i in (0, 3):
        batch = gen[i]
        cubes = [lists[c] for c in gen.indices[i * B:(i + 1) * B]]
        oxs, oys, oreg, _ = noise_ref.philox_noise_batch(cubes, cdf, gen.neg_sampler, 5, i)
        xl = batch.x_lists()
        assert all(np.array_equal(xl[b], oxs[b]) for b in range(B))
        assert np.array_equal(batch.reg_idx.cpu().numpy(), oreg)
        assert np.array_equal(batch.y_reg.cpu().numpy(), Mt.astype(np.float32)[oreg])


def test_fit_save_load_recommend(tmp_path):
    V, d, C = 800, 64, 256
    lists, Mt, ns = problem(11, C, V, (15, 40, 90))
    gen = DataGenerator(Mt.astype(np.float32), lists, batch_size=32, noise=0.2, seed=1)
    model = CC_Recommender(V, d=d, dtype='bf16', seed=2)
    model.compile(optimizer='adam', loss=['binary_crossentropy', 'kullback_leibler_divergence'],
                  loss_weights=[1.0, 0.1], metrics=['accuracy'])
    model.fit(gen, epochs=4, verbose=0)
    h = [x['loss'] for x in model.history]
    assert h[-1] < h[0], h
    dest = str(tmp_path / 'ml_files' / 'recommender')
    model.save(dest, save_format='tf')
    m2 = load_model(dest)
    P = m2.layout.unpack(m2._current_flat())
    assert np.array_equal(P['encoder/encoded_1/kernel'], model.layout.unpack(model._current_flat())['encoder/encoded_1/kernel'])
    cube = lists[0]
    x = np.zeros((1, V))
    x[0, cube] = 1
    probs = m2.decoder(m2.encoder(x, training=False), training=False)[0].numpy()   # ml_recommend.py:78-85
    want = infer_ref.recommend_probs(P, cube)
    assert np.array_equal(probs, want)
    # get_ml_recommend over a local "root" and id map (web/ml_recommend_web.py surface)
    root = tmp_path / 'site'
    (root / 'cube' / 'api' / 'cubelist').mkdir(parents=True)
    names = {i: f'card {i}' for i in range(V)}
    names[int(cube[0])] = 'aether vial'      # id maps hold unidecoded lower-case names
    (root / 'cube' / 'api' / 'cubelist' / 'mycube').write_text('\n'.join(['Æther Vial'] + [names[int(c)] for c in cube[1:]] + ['custom card']))
    idmap = tmp_path / 'id_map.json'
    idmap.write_text(json.dumps({str(k): v for k, v in names.items()}))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from web.ml_recommend_web import get_ml_recommend
    out = get_ml_recommend('mycube', 25, root=str(root), model_dir=dest, id_map=str(idmap))
    adds, _ = infer_ref.top_n(want, cube, 25)
    assert list(out['additions'].keys()) == [names[int(i)] for i in adds]
    assert list(out['additions'].values()) == [float(want[i]) for i in adds]
    assert list(out['cuts'].keys()) == [names[int(c)] for c in cube]
    assert list(out['cuts'].values()) == [float(want[c]) for c in cube]
