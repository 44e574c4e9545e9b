"""Data parallelism over the GPUs of one node: one process per GPU,
torch.distributed with backend "nccl" (= RCCL over xGMI on ROCm), gloo for CPU tests.

Each rank takes its own B cubes of every global batch (disjoint slices of the shared epoch
permutation: cubes perm[g*B*W + r*B : g*B*W + (r+1)*B]) and draws F with Philox slots r*B..r*B+B-1,
so the W ranks together process exactly the batch a single process with batch W*B would
(tests/test_gpu_train.py::test_data_parallel_equivalence, tests/test_gpu_dp.py).  The exchange is
the gradient reduction (zero.py: bucketed reduce-scatter, Adam on the rank's shard, all-gather of the
parameters); every rank ends the step with the same weights.  With reg > 0 the regulariser is
row-sharded over M~ (owner computes; trainer.reg_row_shards and DESIGN.md §5): each
rank holds only its rows of M~ and computes the KL terms of the regulariser rows it owns.

Backend: "nccl" (= RCCL over xGMI) with one GPU per rank; gloo on CPU, or when several ranks share
one GPU (tests), or when CCREC_DIST_BACKEND says so."""
import os

import numpy as np
import torch


def init(backend=None):
    """Read RANK/LOCAL_RANK/WORLD_SIZE; init the process group when WORLD_SIZE > 1.
    Returns (world, rank, device)."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    cuda = torch.cuda.is_available()
    dev = torch.device('cuda', local % torch.cuda.device_count()) if cuda else torch.device('cpu')
    if cuda:
        torch.cuda.set_device(dev)
    if world > 1 and not torch.distributed.is_initialized():
        backend = backend or os.environ.get('CCREC_DIST_BACKEND')
        if backend is None:
            # one GPU per rank OF THIS NODE (LOCAL_WORLD_SIZE; a multi-node launch has world >
            # GPUs per node and still one GPU per rank)
            per_node = int(os.environ.get('LOCAL_WORLD_SIZE', str(world)))
            backend = 'nccl' if cuda and torch.cuda.device_count() >= per_node else 'gloo'
            if backend == 'gloo':
                import sys
                print(f'cubecobrarecommender_amd.distributed: {per_node} ranks per node on '
                      f'{torch.cuda.device_count() if cuda else 0} GPU(s): gloo collectives instead of RCCL',
                      file=sys.stderr)
        kw = {'device_id': dev} if backend == 'nccl' else {}
        torch.distributed.init_process_group(backend, **kw)
    return world, rank, dev


def finish():
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


def rank_cubes(perm, batch_in_epoch, B, rank, world):
    """Host mirror of the cube selection in cc_noise_fwd: this rank's cube ids for a global batch."""
    base = batch_in_epoch * B * world + rank * B
    return np.asarray(perm)[base:base + B]


def allreduce_grads(grads, n=None, world=None):
    """Average the first n gradient entries over ranks (gradient of the mean loss over W*B cubes)."""
    world = world or (torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1)
    if world == 1:
        return grads
    g = grads[:n] if n is not None else grads
    if g.is_cuda:
        torch.distributed.all_reduce(g, op=torch.distributed.ReduceOp.AVG)
    else:  # gloo has no AVG
        torch.distributed.all_reduce(g, op=torch.distributed.ReduceOp.SUM)
        g.div_(world)
    return grads
