#!/usr/bin/env python3
"""Drop-in for src/ml/train.py: `train.py epochs batch_size name reg noise [seed]` (train.py:28-38).

Loads data/maps/nameToId.json + data/cube/*.json (train.py:40-51) and output/full_adj_mtx.npy
(:55; computed on the GPU when absent), builds M~ (:69-71), trains CC_Recommender with Adam on
BCE + reg*KL (:82-102) on the GPU and saves ml_files/<name>/ (:112-115).  Optional flags:
--d (E/D width, reference 512), --dtype fp32|bf16|fp8 (fp32 = the reference's precision), --synthetic C V (no data/ needed),
data-parallel over all GPUs when launched with torch.distributed.run."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('epochs', type=int)
    ap.add_argument('batch_size', type=int)
    ap.add_argument('name')
    ap.add_argument('reg', type=float)
    ap.add_argument('noise', type=float)
    ap.add_argument('seed', nargs='?', type=int, default=0)
    ap.add_argument('--d', type=int, default=512)
    ap.add_argument('--dtype', default='fp32')
    ap.add_argument('--synthetic', nargs=2, type=int, metavar=('C', 'V'))
    ap.add_argument('--data-dir', default='./data')
    ap.add_argument('--adj', default='./output/full_adj_mtx.npy')
    ap.add_argument('--out-dir', default='./ml_files')
    a = ap.parse_args(argv)
    from cubecobrarecommender_amd import adjacency, data as D, distributed
    from cubecobrarecommender_amd.generator import DataGenerator
    from cubecobrarecommender_amd.model import CC_Recommender
    from cubecobrarecommender_amd.synthetic import synthetic_cubes
    world, rank, dev = distributed.init()
    print('Loading Cube Data . . .\n')
    if a.synthetic:
        C, V = a.synthetic
        indptr, idx = synthetic_cubes(C, V, seed=a.seed, device=dev)
    else:
        V, name_lookup, card_to_int, _ = D.get_card_maps(os.path.join(a.data_dir, 'maps', 'nameToId.json'))
        indptr, idx = D.lists_to_csr(D.build_cube_lists(os.path.join(a.data_dir, 'cube'), name_lookup, card_to_int))
    print('Creating Graph for Regularization . . . \n')
    from cubecobrarecommender_amd.synthetic import neg_sampler_from_csr
    if os.path.exists(a.adj) and not a.synthetic:
        M = torch.from_numpy(np.load(a.adj)).to(dev, torch.float64)
        M.fill_diagonal_(1.0)
        M /= M.sum(1, keepdim=True)                  # train.py:69-71, in float64 like the reference
        neg_sampler = (M.sum(0) / M.sum()).cpu().numpy()                    # generator.py:30
        y_mtx = M.to(torch.float32)
        del M
    else:
        y_mtx = adjacency.adjacency_normalised_gpu(indptr, idx, V, device=dev)
        neg_sampler = neg_sampler_from_csr(indptr, idx, V)   # the float64 closed form of :30
    print('Setting Up Model . . . \n')
    model = CC_Recommender(V, d=a.d, dtype=a.dtype, seed=a.seed)
    model.compile(optimizer='adam', loss=['binary_crossentropy', 'kullback_leibler_divergence'],
                  loss_weights=[1.0, a.reg], metrics=['accuracy'])
    gen = DataGenerator(y_mtx, (indptr, idx), batch_size=a.batch_size, noise=a.noise, seed=a.seed, device=dev,
                        neg_sampler=neg_sampler)
    model.fit(gen, epochs=a.epochs, rank=rank, world=world)
    if rank == 0:
        model.save(os.path.join(a.out_dir, a.name), save_format='tf')
    distributed.finish()
    return model


if __name__ == '__main__':
    main()
