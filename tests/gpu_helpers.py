"""Shared helpers for the GPU parity tests (synthetic data, oracle plumbing)."""
import numpy as np

from oracle import adjacency_ref, noise_ref


def synthetic_lists(rng, C, V, sizes=(20, 40, 60), never_seen=3):
    live = V - never_seen
    pop = 1.0 / (1.0 + rng.permutation(live))
    out = []
    for _ in range(C):
        n = int(rng.choice(sizes))
        g = np.log(pop) + rng.gumbel(size=live)
        out.append(np.sort(np.argsort(-g)[:n]))
    return out


def problem(seed, C, V, sizes):
    rng = np.random.default_rng(seed)
    lists = synthetic_lists(rng, C, V, sizes)
    M = adjacency_ref.adjacency_from_lists(lists, V)
    Mt = adjacency_ref.normalise(M)
    ns = noise_ref.neg_sampler_of(Mt)
    return lists, Mt, ns


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def progress(msg):
    """A progress line for multi-process GPU tests: printed (pytest shows a failing test's captured
    output) and appended to progress.log beside $CCREC_PARITY_LOG (if set), so a stuck child leaves
    its last completed stage in gpurun_out/ even when the session is cut before the test's own
    time limits fire (the r04j stall: DESIGN.md §5)."""
    import os
    import time
    print(msg, flush=True)
    path = os.environ.get('CCREC_PARITY_LOG')
    if path:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(os.path.join(os.path.dirname(os.path.abspath(path)), 'progress.log'), 'a') as fh:
            fh.write(f'{time.strftime("%H:%M:%S")} pid {os.getpid()} {msg}\n')


def record_errors(test, step, errs):
    """Append observed parity errors as a JSON line to $CCREC_PARITY_LOG (if set): the tolerances
    in the tests are set from these observations (about 3x the largest one seen)."""
    import json
    import os
    path = os.environ.get('CCREC_PARITY_LOG')
    if path:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, 'a') as fh:
            fh.write(json.dumps({'test': test, 'step': step,
                                 'errs': {k: float(v) for k, v in errs.items()}}) + '\n')
