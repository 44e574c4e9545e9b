#!/usr/bin/env python3
"""Headline benchmark: DAE training cubes/s at |V|=22,000, d=256, B=512/GPU, BCE only, bf16
(BASELINE.json configs[1]) on synthetic cubes, plus the recommend p50/p99 latency (configs[0]
architecture: |V|=20,884, d=512, fp32, model resident).

    python bench.py [--gpus N] [--steps K] [--warmup W]
N>1 is launched by torch.distributed.run (one rank per GPU, RCCL); cubes shard data-parallel
(weak scaling: B=512 per rank), gradients are all-reduced.  Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BF16_PEAK_TFLOPS = 2500.0   # dense bf16 MFMA (spec, no sparsity)
MX8_PEAK_TFLOPS = 5000.0    # dense (MX-)FP8 MFMA (spec, no sparsity)
F32_PEAK_TFLOPS = 157.3     # f32 MFMA (exact f32 in / acc; no xf32 on gfx950): 1/16 of bf16


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--wo-tower-frac', type=float, default=-1.0,
                    help="the trailing fraction of Wo's Adam run in the tower backward launch (-1: TrainConfig's default)")
    ap.add_argument('--f-in-tower', type=int, default=0,
                    help='one process: the next step\'s F in the tower backward launch (1) or the Adam launch (0)')
    ap.add_argument('--dx-packed-wo', type=int, default=1,
                    help="full mode: the regulariser's dX from Wo's fragment image (1) or the row-major Wo (0)")
    ap.add_argument('--prespin-ms', type=float, default=300.0,
                    help='untimed non-training GPU work (a memory-bound scale + a bf16 matmul loop) before '
                         'warmup: the GPU out of its idle clocks, so that a short --warmup already times the '
                         'steady state (DESIGN.md: the timed bracket)')
    ap.add_argument('--prespin-kind', default='both', choices=('mem', 'mfma', 'both'))
    ap.add_argument('--graph-steps', type=int, default=0,
                    help='steps per multi-step graph replay (0: the largest of 8, 7, ..., 1 that divides '
                         '--steps and is <= --warmup, so warmup has replayed every graph the timed region '
                         'replays: a graph\'s first replay costs extra)')
    ap.add_argument('--V', type=int, default=22000)
    ap.add_argument('--d', '--dim', dest='d', type=int, default=256)
    ap.add_argument('--batch', type=int, default=512)
    ap.add_argument('--cubes', type=int, default=65536)
    ap.add_argument('--reg', type=float, default=0.0)
    ap.add_argument('--dtype', default='bf16')
    ap.add_argument('--reg-shard', type=int, default=1,
                    help='with --reg > 0 on N > 1 ranks: M~ row-sharded at equal neg_sampler mass, '
                         'owner computes over the global reg draws (SURVEY 8(e)); 0 = every rank '
                         'holds all of M~ and draws its own B reg rows')
    ap.add_argument('--reg-mode', default='sampled', choices=('sampled', 'full'),
                    help="sampled: B reg rows per step drawn from neg_sampler (generator.py:47-51); "
                         "full: all |V| identity rows every step (README.md:27, the |V|x|V| MFMA path)")
    ap.add_argument('--dz-pad', type=int, default=1,
                    help='the fused D1 kernel\'s dZ rows at a 64-element pitch (TrainConfig.dz_pad)')
    ap.add_argument('--force-dp', action='store_true',
                    help='one GPU driving the data-parallel step through a 1-rank RCCL process group '
                         '(the per-rank kernel and exchange sequence the N-GPU run executes)')
    ap.add_argument('--dp-graph', type=int, default=1, choices=(0, 1),
                    help='data parallel over RCCL: 1 = the whole step (collectives included) as one captured '
                         'hipGraph; 0 = graph replays of the step\'s parts with eager RCCL collectives between '
                         'them (the fallback if multi-rank capture misbehaves; same arithmetic, bit-identical)')
    ap.add_argument('--reg-by-index', type=int, default=1, choices=(0, 1),
                    help='sampled regulariser: its one-card rows enter the W1 gradient by index (1, '
                         'TrainConfig.reg_by_index) or as bits of a 2B-row bit matrix (0); bit-identical')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-steps', type=int, default=16)
    ap.add_argument('--no-recommend', action='store_true')
    ap.add_argument('--backend', default='nccl',
                    help="collective backend for --gpus > 1 (nccl = RCCL; gloo only to rehearse the "
                         "data-parallel path with several ranks on one GPU)")
    ap.add_argument('--traffic-json', default=os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                           'profiles', 'traffic_r06.json'))
    return ap.parse_args()


def child_argv(argv):
    """bench.py's arguments as the ranks receive them through torch.distributed.run, whose parser
    rejects an option that abbreviates several of its own before handing the rest to the script
    (`--d` would abbreviate --duplicate-stdout-filters / --duplicate-stderr-filters): `--d` is
    passed as its long form `--dim`."""
    out = []
    for a in argv:
        if a == '--d':
            a = '--dim'
        elif a.startswith('--d='):
            a = '--dim=' + a[4:]
        out.append(a)
    return out


def launch_ranks(args):
    """--gpus N > 1 without a torch.distributed.run environment: start one rank per GPU as CHILD
    processes (torch.distributed.run, rendezvous on 127.0.0.1) and exit with their status.  This
    parent never touches the GPU (no HIP call before the children start, no exec)."""
    if args.gpus <= 1 or 'WORLD_SIZE' in os.environ:
        return
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={args.gpus}',
           '--master-addr', '127.0.0.1', f'--master-port={port}', os.path.abspath(__file__),
           *child_argv(sys.argv[1:])]
    sys.exit(subprocess.run(cmd, env=env).returncode)


def setup_dist(args):
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        import torch.distributed as dist
        ndev = torch.cuda.device_count()
        local = local % ndev
        torch.cuda.set_device(local)
        per_node = int(os.environ.get('LOCAL_WORLD_SIZE', str(world)))
        if args.backend == 'nccl' and ndev < per_node:   # RCCL needs one GPU per rank
            print(f'bench.py: {per_node} ranks on {ndev} GPU(s): gloo collectives instead of RCCL',
                  file=sys.stderr)
            args.backend = 'gloo'
        if args.backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(args.backend)
    elif args.force_dp:   # a 1-rank RCCL group: zero.py's collectives on device tensors
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', store=dist.HashStore(), rank=0, world_size=1,
                                device_id=torch.device('cuda', local))
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


PEAKS = {'hbm': (HBM_PEAK_GBS, 'GB/s'), 'mfma': (BF16_PEAK_TFLOPS, 'TFLOP/s'),
         'mfma_mx8': (MX8_PEAK_TFLOPS, 'TFLOP/s'), 'mfma_f32': (F32_PEAK_TFLOPS, 'TFLOP/s')}


def mfma_kind(tr):
    """The MFMA peak a product of this trainer is priced against: its operand dtype."""
    return 'mfma_f32' if tr.cfg.dtype == 'fp32' else 'mfma'


def roofline_for(name, ms, tr):
    """Algorithmic bytes (HBM-bound kernels) or flops (MFMA products) per launch of an
    instrumented kernel, and the achieved rate at the measured duration `ms`."""
    cfg = tr.cfg
    V, d, B = cfg.V, cfg.d, cfg.batch_size
    fl = byt = None
    kind = mfma_kind(tr)
    if name == 'cc_adam_dense':
        n = tr.layout.total if tr.use_reg else tr.layout.main_total
        if getattr(tr, 'fuse_w1', False):     # W1's Adam runs in its gradient kernel
            n -= tr.w1_off
        for lo, hi in (getattr(tr, 'wo_ranges', None) or ()):   # (the output layers' tails: in the
            n -= hi - lo                                          # tower backward launch)
        byt = n * (16 + 12 + 2)                    # read p,m,v,g; write p,m,v; write bf16 shadow
        what = ('adam_noise_kernel (TF Adam over the parameters not updated elsewhere + F of the next step; '
                'bytes counted are Adam\'s only, F adds <2%)' if getattr(tr, 'prefetch', False)
                else 'adam_kernel (cc_adam_dense)')
    elif name == 'dec_bce_fwd':
        if getattr(tr, 'fused_out', False):  # logits + dWo = D3^T dZ in one pass (dX: its own launch)
            fl = 2 * 2.0 * B * d * V
            what = 'dec_bce_dw_kernel (fused D1: logits + sigmoid/BCE + dZ + dWo/dbo; flops = logits + dWo)'
        else:
            fl = 2.0 * B * d * V
            what = ('mx8_wide_kernel (MX-FP8 logits + BCE epilogue)' if tr.mx8 else 'gemm (D1 logits + BCE epilogue)')
        if tr.mx8:
            kind = 'mfma_mx8'
    elif name == 'dec_softmax_kl' and getattr(tr, 'fused_reg', False):
        fl = 3 * 2.0 * tr.Breg * d * V      # logits twice (stats, main) + dWo
        what = 'kl_stats + kl_main (fused D2: logits twice, softmax/KL, dZ, dWo/dbo)'
    elif name == 'dec_dX':
        fl = 2.0 * B * d * V
        what = 'dX split-K (dD3 = dZ Wo^T) + reduce'
        if tr.mx8:
            kind = 'mfma_mx8'
    elif name == 'cc_embed_scatter_bwd' and getattr(tr, 'fuse_w1', False):
        # W1 [V][d]: p, m, v read + written (24 B), bf16 shadow written (2 B); the row bit matrix
        # (V x ceil(rows/32) words) and the packed dPre1 image (rows x d bf16) read; b1's gradient row
        rows = getattr(tr, 'xt_rows', tr.R)
        byt = V * d * 26 + V * ((rows + 31) // 32) * 4 + ((rows + 63) // 64 * 64) * d * 2 + d * 4
        what = ('embed_grad_cs_kernel<.., ADAM> (cc_embed_grad_cs_adam: the W1 gradient X^T dPre1 from the '
                'bit-transposed batch on MFMA, TF Adam on W1 in its epilogue; bytes: W1 p/m/v read + write, '
                'the bf16 shadow, the bit matrix and the dPre1 image)')
    elif name == 'cc_embed_scatter_bwd':
        byt = V * d * 4 + V * ((tr.R + 31) // 32) * 4
        what = 'embed_grad (the W1 gradient X^T dPre1, stored fp32)'
    else:
        return None
    if byt is not None:
        kind, work = 'hbm', byt
        rate = byt / (ms * 1e-3) / 1e9
    else:
        work = fl
        rate = fl / (ms * 1e-3) / 1e12
    peak, unit = PEAKS[kind]
    return {'bound': 'hbm' if kind == 'hbm' else 'mfma', 'achieved': rate, 'peak': peak, 'unit': unit,
            'frac': rate / peak, ('bytes_per_launch' if byt is not None else 'flops_per_launch'): work,
            'avg_us': ms * 1e3, 'kernel': what, 'tick': name}


# rocprofv3 kernel-name keys of the PMC traffic table (profiles/traffic_*.json) per instrumented tick
TRAFFIC_KEYS = {'cc_embed_scatter_bwd': 'embed_grad_cs_kernel', 'cc_adam_dense': 'adam_noise_kernel',
                'dec_bce_fwd': 'dec_bce_dw_kernel'}


def kernel_rooflines(tr, kt, traffic_json):
    """Roofline entries of the step's instrumented kernels, longest first.  kt: steady-state
    per-kernel durations (us) from kernel_profile (HIP events on the launching stream)."""
    tj = json.load(open(traffic_json)) if traffic_json and os.path.exists(traffic_json) else {}
    out = []
    for name, us in sorted(kt.items(), key=lambda kv: -kv[1]):
        r = roofline_for(name, us * 1e-3, tr)
        if r is None:
            continue
        r['traffic'] = None
        t = tj.get(TRAFFIC_KEYS.get(name, ''), {})
        tb = t.get('bytes_per_launch')
        ref = r.get('bytes_per_launch') or t.get('algorithmic_bytes')
        # PMC bytes were collected on one build / configuration: attach only to the same launch
        if tb and ref and (r['bound'] == 'mfma' or abs(tb - ref) <= 0.10 * ref):
            r['traffic'] = tb
            r['traffic_detail'] = t
        out.append(r)
    return out


def workload_label(args, world):
    """Which BASELINE.json config this line measures (configs[0] is the CPU recommend case)."""
    what = 'DAE training step (F noise + E + D1/BCE' + (
        (' + D2/KL over all |V| identity rows' if args.reg_mode == 'full' else ' + D2/KL') if args.reg > 0 else '') + \
        ' + backward + Adam)'
    if args.dtype == 'fp8':
        idx = 4
    elif world > 1 or args.force_dp:
        idx = 3
    else:
        idx = 2 if args.reg > 0 else 1
    note = '' if (idx != 4 or world == 8) else f' on {world} of its 8 GPUs'
    if idx == 3 and args.reg == 0:
        note = ' with reg=0 (BCE only, configs[1] per GPU)'
    return f'{what}, BASELINE configs[{idx}]{note}'


def kernel_profile(tr, step, samples=8):
    """Steady-state per-kernel durations (us) for the step-level report: HIP events around each
    kernel of an eager step launched while the GPU is still busy with three queued whole-step graph
    replays, so every interval is the kernel's own duration (not launch latency or first-launch
    module loads).  Run after the timed region; it does not touch the headline number."""
    tr.events = {}
    for i in range(samples + 1):
        for _ in range(3):
            step(True)
        tr.timing = True
        step(False)
        tr.timing = False
        if i == 0:                 # first eager step after graph replays: discard
            torch.cuda.synchronize()
            tr.events = {}
    return {k: 1e3 * v for k, v in tr.kernel_times_ms().items()}


def dp_profile(tr, step, samples=8, replays=40):
    """Data-parallel per-rank report (after the timed region): per gradient bucket the collectives'
    and the sharded Adam's durations (HIP events on the comm stream, eager steps queued behind graph
    replays), and the whole-step graph replayed with and without its collectives — the difference is
    the exchange time the step does not hide behind compute."""
    import torch.distributed as dist
    sh = tr.sharded
    sh.adam_events, sh.comm_events = [], {}
    for i in range(samples + 1):
        for _ in range(3):
            step(True)
        step(False, timed=True)
        if i == 0:
            torch.cuda.synchronize()
            sh.adam_events, sh.comm_events = [], {}
    torch.cuda.synchronize()
    rep = {'buckets': {}}
    for (bname, what), evs in sorted(sh.comm_events.items()):
        rep['buckets'].setdefault(bname, {})[what + '_us'] = 1e3 * float(np.mean([a.elapsed_time(b) for a, b in evs]))
    for b in sh.buckets:
        ent = rep['buckets'].setdefault(b['name'], {})
        ent['elements'] = b['hi'] - b['lo']
        ent['shard'] = b['chunk']
    n_sh = sum(n for _, _, n in sh.adam_events) / samples
    adam_us = 1e3 * sum(a.elapsed_time(b) for a, b, _ in sh.adam_events) / samples
    byt = n_sh * (16 + 12 + 2)
    rep['_adam'] = {'tick': 'sharded_adam', 'kernel': 'adam_kernel (cc_adam_dense on this rank\'s 1/world shard '
                    'of every bucket; sum over the buckets per step)', 'bound': 'hbm',
                    'achieved': byt / (adam_us * 1e-6) / 1e9, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                    'frac': byt / (adam_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 'bytes_per_launch': byt,
                    'avg_us': adam_us, 'traffic': None}
    if tr.g_dp is not None:
        times = {}
        for key, g in (('step_us', tr.g_dp), ('step_without_exchange_us', tr.g_dp_nocomm),
                       ('step_us_again', tr.g_dp)):
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(replays):
                g.replay()
            torch.cuda.synchronize()
            dt = torch.tensor([(time.perf_counter() - t0) / replays], device=tr.params.device, dtype=torch.float64)
            if dist.get_world_size() > 1:
                dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            times[key] = 1e6 * float(dt.item())
        rep.update(times)
        rep['exposed_exchange_us'] = 0.5 * (times['step_us'] + times['step_us_again']) - times['step_without_exchange_us']
        rep['graph'] = 'whole'
        rep['graph_path'] = 'whole DP step as one hipGraph (RCCL collectives captured on the comm stream)'
    else:
        rep['graph'] = 'parts'
        rep['graph_path'] = ('graph replays of forward_backward_a / forward_backward_b / counters with eager '
                             'collectives and sharded Adam between them (' +
                             ('--dp-graph 0' if not tr.cfg.dp_graph else 'gloo backend') + ')')
    rep['backend'] = dist.get_backend()
    rep['world'] = dist.get_world_size()
    return rep


def step_roofline(tr, ms_per_step, kt):
    """Whole-step HBM roofline: algorithmic bytes per step =
    B*n*d*e (E1 gather) + 34*P (fp32 grad write+read, Adam p/m/v read+write, low-precision shadow)
    + 2*e*d*V*n_dec (decoder output weights, forward + dX) + B*(4n + V/8) (x CSR + y bits)
    [+ 4*B*V with reg (M~ rows)], n = mean noised cube size of the step's batch; plus the decoder
    output layer's MFMA rate."""
    cfg = tr.cfg
    V, d, B = cfg.V, cfg.d, cfg.batch_size
    e = 1 if tr.mx8 else 2 if tr.dtype == 1 else 4
    n = float(tr.x_cnt[:B].float().mean().item())
    P = tr.layout.total if tr.use_reg else tr.layout.main_total
    ndec = 2 if tr.use_reg else 1
    byt = B * n * d * e + 34 * P + 2 * e * d * V * ndec + B * (4 * n + V / 8) + (4 * tr.Breg * V if tr.use_reg else 0)
    if getattr(tr, 'fuse_w1', False):   # W1's fp32 gradient is never written nor read back
        byt -= 8 * tr.w1_off
    out = {'bound': 'hbm', 'bytes_per_step': byt, 'achieved': byt / (ms_per_step * 1e-3) / 1e9,
           'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'mean_cube_n': n}
    out['frac'] = out['achieved'] / out['peak']
    if tr.full_reg:   # the |V| x |V| regulariser product dominates: MFMA-bound
        T = 512 * d + 81920
        fl = 6.0 * (d * V + T) * (B + tr.Breg) + 4.0 * n * d * B   # SURVEY 8(d) FLOP/row
        pk = PEAKS[mfma_kind(tr)][0]
        out.update({'bound': 'mfma', 'flops_per_step': fl, 'achieved_tflops': fl / (ms_per_step * 1e-3) / 1e12,
                    'peak_tflops': pk, 'frac_mfma': fl / (ms_per_step * 1e-3) / 1e12 / pk})
    if kt and 'dec_bce_fwd' in kt and getattr(tr, 'fused_out', False):
        fl = 2 * 2.0 * B * d * V            # logits + dWo (dX runs in its own GEMM)
        us = kt['dec_bce_fwd']
        out['decoder_mfma'] = {'kernel': 'dec_bce_dw_kernel (fused D1: logits + sigmoid/BCE + dZ + dWo/dbo)',
                               'flops_per_launch': fl, 'avg_us': us, 'achieved': fl / (us * 1e-6) / 1e12,
                               'peak': BF16_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                               'frac': fl / (us * 1e-6) / 1e12 / BF16_PEAK_TFLOPS}
    elif kt and 'dec_bce_fwd' in kt:   # (the unfused logits product: fp32 / MX-FP8 / other shapes)
        fl = 2.0 * B * d * V
        us = kt['dec_bce_fwd']
        peak = PEAKS['mfma_mx8' if tr.mx8 else mfma_kind(tr)][0]
        out['decoder_mfma'] = {'kernel': 'D1 logits product + BCE epilogue', 'flops_per_launch': fl, 'avg_us': us,
                               'achieved': fl / (us * 1e-6) / 1e12, 'peak': peak, 'unit': 'TFLOP/s',
                               'frac': fl / (us * 1e-6) / 1e12 / peak}
    if kt and 'dec_dX' in kt:
        out['decoder_dx_mfma'] = {'flops_per_launch': 2.0 * B * d * V, 'avg_us': kt['dec_dX'],
                                  'achieved': 2.0 * B * d * V / (kt['dec_dX'] * 1e-6) / 1e12,
                                  'peak': PEAKS['mfma_mx8' if tr.mx8 else mfma_kind(tr)][0], 'unit': 'TFLOP/s'}
    if kt and 'cc_embed_gather_fwd' in kt:
        gb = tr.R * n * d * e
        out['gather'] = {'bytes_per_launch': gb, 'avg_us': kt['cc_embed_gather_fwd'],
                         'achieved_GBs': gb / (kt['cc_embed_gather_fwd'] * 1e-6) / 1e9,
                         'note': 'row bytes gathered (mostly L2/MALL hits: W1 is 11 MB)'}
    return out


def cpu_baseline(args, seconds_cap=30.0):
    """The CPU oracle (numpy restatement of generator.py + model.py/train.py) on a bounded sample
    of the same workload: a few B=512 steps at |V|=22k, d=256 (oracle is test infra; used here
    only as the timed CPU baseline)."""
    from threadpoolctl import threadpool_info
    from oracle import model_ref, noise_ref
    from cubecobrarecommender_amd.synthetic import synthetic_cubes, neg_sampler_from_csr
    V, d, B = args.V, args.d, args.batch
    C = max(B * args.cpu_steps, 1024)
    indptr, indices = synthetic_cubes(C, V, seed=7, device='cuda' if torch.cuda.is_available() else 'cpu')
    ns = neg_sampler_from_csr(indptr, indices, V)
    lists = [indices[indptr[c]:indptr[c + 1]] for c in range(C)]
    P = model_ref.init_params(V, d, seed=1)
    Mo = {k: np.zeros_like(v) for k, v in P.items()}
    Vo = {k: np.zeros_like(v) for k, v in P.items()}
    rs = np.random.RandomState(0)
    mt = noise_ref.MTNoise(rs, ns, V)
    t0 = time.perf_counter()
    done = 0
    for s in range(args.cpu_steps):
        xs, ys, _ = mt.batch(lists[s * B:(s + 1) * B])            # generator.py F (MT19937 replay)
        _, G = model_ref.train_forward_backward(P, xs, ys, V, d, reg=0.0, mode='fp32')
        P, Mo, Vo = model_ref.adam_tf(P, Mo, Vo, G, t=s + 1)
        done += B
        if time.perf_counter() - t0 > seconds_cap:
            break
    dt = time.perf_counter() - t0
    threads = max([i.get('num_threads', 1) for i in threadpool_info()] + [1])
    return {'value': done / dt, 'unit': 'cubes/s', 'cores': int(threads), 'kind': 'port',
            'sample': f'{done} cubes ({done // B} steps of B={B}) at V={V}, d={d}: oracle numpy '
                      f'generator (MT19937 replay of generator.py) + fp32 numpy fwd/bwd + TF-Adam'}


def recommend_latency(n_req=1000):
    from cubecobrarecommender_amd.layout import Layout
    from cubecobrarecommender_amd.recommender import Recommender
    V, d = 20884, 512
    rng = np.random.default_rng(0)
    lay = Layout(V, d)
    flat = (rng.standard_normal(lay.total).astype(np.float32) * 0.02)
    rec = Recommender(flat, V, d)
    out = {}
    for amount in (100, 30000):
        lat = []
        for i in range(n_req // 2 + 20):
            cube = rng.choice(V, 360, replace=False)
            t0 = time.perf_counter()
            rec.recommend(cube, amount)
            lat.append(time.perf_counter() - t0)
        lat = np.array(lat[20:]) * 1e3
        out[f'amount_{amount}'] = {'p50_ms': float(np.percentile(lat, 50)),
                                   'p99_ms': float(np.percentile(lat, 99)), 'requests': len(lat)}
    out['config'] = 'V=20884 d=512 fp32 resident model, cube n=360, index list in -> top-N indices out'
    out['cold_load'] = cold_load(flat, lay, V, d, rng)
    return out


def cold_load(flat, lay, V, d, rng):
    """BASELINE configs[0]'s cold path (ml_recommend.py:54-108: load_model on ml_files/<name>, then
    one single-cube recommend): a checkpoint of the reference architecture is written in the
    ml_files layout (TF tensor bundle, checkpoint.py), then load_model + the first recommend are
    timed in this process (torch and the HIP library already loaded; the reference's own
    interpreter start and TF import are not part of either side)."""
    import shutil
    import tempfile
    from cubecobrarecommender_amd import checkpoint
    from cubecobrarecommender_amd.model import load_model
    tmp = tempfile.mkdtemp(prefix='ccrec_cold_')
    try:
        path = os.path.join(tmp, 'recommender')
        checkpoint.save_model(path, V, d, lay.unpack(flat))
        size = sum(os.path.getsize(os.path.join(dp, f)) for dp, _, fs in os.walk(path) for f in fs)
        cube = rng.choice(V, 360, replace=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        model = load_model(path)
        t1 = time.perf_counter()
        model.recommender().recommend(cube, 100)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        return {'load_model_s': t1 - t0, 'first_recommend_s': t2 - t1, 'total_s': t2 - t0,
                'checkpoint_bytes': size}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    args = parse()
    launch_ranks(args)
    world, rank, local = setup_dist(args)
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    from cubecobrarecommender_amd.synthetic import synthetic_cubes, neg_sampler_from_csr
    from cubecobrarecommender_amd.trainer import DeviceDataset, TrainConfig, Trainer
    from cubecobrarecommender_amd.layout import Layout, glorot_flat
    V, d, B = args.V, args.d, args.batch
    t_setup = time.perf_counter()
    indptr, indices = synthetic_cubes(args.cubes, V, seed=20250301, device=dev)
    ns = neg_sampler_from_csr(indptr, indices, V)
    y_mtx, reg_rows = None, None
    reg_shard = bool(args.reg_shard) and (world > 1 or args.force_dp) and args.reg > 0
    if args.reg > 0:
        from cubecobrarecommender_amd.adjacency import adjacency_normalised_gpu
        y_mtx = adjacency_normalised_gpu(indptr, indices, V, device=dev)
        if (world > 1 or args.force_dp) and (reg_shard or args.reg_mode == 'full'):   # this rank's rows of M~
            from cubecobrarecommender_amd.trainer import reg_rows_for
            reg_rows = reg_rows_for(ns, world, rank, args.reg_mode)
            y_mtx = y_mtx[reg_rows[0]:reg_rows[1]].clone()
            torch.cuda.empty_cache()
    data = DeviceDataset(csr=(indptr, indices), num_cards=V, neg_sampler=ns, y_mtx=y_mtx, device=dev,
                         reg_rows=reg_rows)
    del y_mtx
    graph_steps = args.graph_steps or next(g for g in range(8, 0, -1)
                                           if args.steps % g == 0 and (g <= args.warmup or g == 1))
    cfg = TrainConfig(V=V, d=d, batch_size=B, reg=args.reg, dtype=args.dtype, seed=1234,
                      rank=rank, world=world, reg_shard=reg_shard, reg_mode=args.reg_mode,
                      force_dp=args.force_dp, dp_graph=bool(args.dp_graph), reg_by_index=bool(args.reg_by_index),
                      dz_pad=bool(args.dz_pad), graph_steps=graph_steps, wo_tower_frac=args.wo_tower_frac,
                      fuse_w1_adam=True,   # one process: W1's Adam in its gradient kernel, and (BCE
                      wo_adam_in_tower=True,   # only) Wo's in the tower backward launch, with the next
                      f_in_tower=bool(args.f_in_tower),   # step's F (parity:
                      dx_packed_wo=bool(args.dx_packed_wo))
    #                                        tests/test_gpu_train.py::test_fused_w1_adam_matches_unfused)
    tr = Trainer(cfg, data, params_flat=glorot_flat(V, d, seed=42), device=dev)
    rng = np.random.default_rng(99)      # same permutations on every rank
    tr.set_epoch_permutations(np.stack([rng.permutation(args.cubes) for _ in range(4)]))
    setup_s = time.perf_counter() - t_setup

    dp = tr.dp

    def step(graphed, timed=False):
        if dp:   # bucketed reduce-scatter + sharded Adam + all-gather (zero.py)
            if graphed:
                tr.step_dp()
            else:             # eager parts (kernel_profile's HIP events need eager launches)
                tr._dp_call(None, timing=timed)
            return
        saved, tr.graphs = tr.graphs, (tr.graphs if graphed else None)
        tr.step()
        tr.graphs = saved

    def steps(n):
        """n steady-state steps: one process replays tr.step_many's multi-step graph (cfg.graph_steps
        whole steps per replay, single-step graphs for the remainder); data parallel replays the
        whole DP step graph (RCCL collectives inside) step by step.  Nothing else runs in the timed
        region: the per-kernel durations come from kernel_profile after it."""
        if dp:
            for _ in range(n):
                step(True)
            return
        tr.step_many(n)

    for _ in range(3):          # eager steps: module loads, lazy allocations
        step(False)
    tr.capture()
    if args.prespin_ms > 0:     # untimed non-training GPU work: the clocks out of idle before warmup
        big = torch.empty(256 << 20, device=dev, dtype=torch.float32)
        spin = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
        t_end = time.perf_counter() + args.prespin_ms / 1e3
        while time.perf_counter() < t_end:
            for _ in range(4):
                if args.prespin_kind in ('mem', 'both'):
                    big.mul_(1.0)
                if args.prespin_kind in ('mfma', 'both'):
                    spin = torch.tanh(spin @ spin)
            torch.cuda.synchronize()
        del big, spin

    steps(args.warmup)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps(args.steps)
    barrier(world)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    tr.check_status()
    losses = tr.losses()
    # per-kernel steady-state times (HIP events; with DP the collectives and the sharded Adam run
    # between the ticked kernels and are not in them): every rank runs the same extra steps
    ktimes = kernel_profile(tr, step)
    dp_report = dp_profile(tr, step) if dp else None
    if rank != 0:
        if dp:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    value = B * world * args.steps / dt
    kr = kernel_rooflines(tr, ktimes, args.traffic_json)
    if dp:   # the sharded Adam: this rank's 1/world shard of every bucket, per step
        ev = dp_report.pop('_adam')
        kr.append(ev)
        kr.sort(key=lambda r: -r['avg_us'])
    roof = dict(kr[0]) if kr else {'bound': 'hbm', 'achieved': None, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                                   'frac': None, 'traffic': None}
    roof['measured'] = ('the step\'s longest kernel with a stated algorithmic cost; its average duration from '
                        'HIP events on its stream around the kernels of eager steps queued behind whole-step '
                        'graph replays, after the timed region (bench.kernel_profile); the timed region '
                        'replays graphs only')
    roof['others'] = [{k: r[k] for k in ('tick', 'kernel', 'bound', 'achieved', 'unit', 'frac', 'avg_us', 'traffic')}
                      for r in kr[1:]]
    out = {
        'metric': 'training cubes/sec at |V|~22k d=256; top-N recommend p50 latency',
        'value': value, 'unit': 'cubes/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': dt / args.steps * 1e3, 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': args.dtype,
        'data': 'synthetic cubes (SURVEY §8(d): Zipf popularity, sizes 180-720, C=65536), random-init weights',
        'config': {'workload': workload_label(args, world),
                   'V': V, 'd': d, 'batch_per_gpu': B, 'global_batch': B * world, 'reg': args.reg,
                   'reg_mode': args.reg_mode, 'reg_rows_per_gpu': tr.Breg,
                   'reg_shard': 'owner computes' if tr.owner else ('full rows' if tr.full_reg and world > 1 else 'replicated'),
                   'cubes': args.cubes,
                   'parallelism': f'dp{world}' + (' (1-rank RCCL group driving the data-parallel step)'
                                                  if args.force_dp and world == 1 else ''),
                   'graph_steps': tr.multi_n if not dp else 1,
                   'prespin_ms': args.prespin_ms, 'prespin_kind': args.prespin_kind},
        'roofline': roof,
        'step_roofline': step_roofline(tr, dt / args.steps * 1e3, ktimes),
        'kernel_us': ktimes,
        'final_loss': losses,
        'setup_s': setup_s,
    }
    if dp:
        out['dp'] = dp_report
    if not args.no_recommend and world == 1:
        out['recommend'] = recommend_latency()
    if not args.no_cpu_baseline and world == 1:
        out['cpu_baseline'] = cpu_baseline(args)
    print(json.dumps(out), flush=True)
    if dp:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
