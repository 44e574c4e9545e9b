#!/usr/bin/env python3
"""Per-kernel roofline table from one profiling session (tools/gpu_prof.sh): rocprofv3 kernel stats
(average duration) joined with the PMC passes of the same bench command:

  HW FLOP / launch  = SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 (the counter's unit: 512 FLOP per count;
                      checked against the decoder kernels' algorithmic 2*B*d*V*2 = 11.53 GFLOP)
  HBM B / launch    = 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024; MI355X_MICROARCH.md §HBM: FETCH_SIZE
                      counts half the bytes of wide coalesced reads on gfx950), separate passes

python tools/prof_report.py DIR TAG TITLE CMD > profiles/<TAG>_<name>_roofline.md
"""
import csv
import json
import os
import sys

BF16_PEAK = 2500.0   # TFLOP/s dense (MI355X_MICROARCH.md)
HBM_PEAK = 8000.0    # GB/s
SKIP = ('at::', 'rocclr', 'rocprim', 'mbtopk', 'cooccur', 'xt_scatter', 'card_stats', 'kl_tsum',
        'to_bf16', 'tower_transpose', 'state_advance', 'normalise', 'adjacency', 'csr_')


def short(name):
    n = name.replace('(anonymous namespace)::', '')
    return n.split('(')[0][:48]


def load(path):
    return json.load(open(path)) if os.path.exists(path) else {}


def main():
    d, tag, title, cmd = sys.argv[1:5]
    stats = list(csv.DictReader(open(os.path.join(d, f'stats_{tag}.csv'))))
    pre = '' if tag == 'base' else tag
    mf = load(os.path.join(d, f'pmc_{pre}mfma.json'))
    fe = load(os.path.join(d, f'pmc_{pre}fetch.json'))
    wr = load(os.path.join(d, f'pmc_{pre}write.json'))
    print(f'# {title}\n')
    print(f'Kernel stats: `{cmd}` under `rocprofv3 --kernel-trace --stats`; counters: the same bench '
          f'command (16 timed steps) under `rocprofv3 --pmc`, one pass per counter group '
          f'(tools/gpu_prof.sh, reduced on the box by tools/prof_collect.py).\n')
    print('HW FLOP = SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512; HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE '
          '(gfx950 FETCH_SIZE correction; the write pass is absent for some sessions).  Fractions '
          f'against {BF16_PEAK:.0f} TFLOP/s dense bf16 and {HBM_PEAK:.0f} GB/s.\n')
    print('| kernel | calls | avg us | % time | HW GFLOP | TFLOP/s | MFMA frac | HBM MB | GB/s | HBM frac |')
    print('|---|---|---|---|---|---|---|---|---|---|')
    for r in stats:
        name = r['Name']
        if any(s in name for s in SKIP):
            continue
        us = float(r['AverageNs']) / 1e3
        m = mf.get(name, {}).get('SQ_INSTS_VALU_MFMA_MOPS_BF16')
        f = fe.get(name, {}).get('FETCH_SIZE')
        w = wr.get(name, {}).get('WRITE_SIZE')
        fl = m * 512 / 1e9 if m is not None else None
        byt = ((2 * f if f is not None else 0) + (w or 0)) * 1024 / 1e6 if f is not None else None
        cells = [f'`{short(name)}`', r['Calls'], f'{us:.1f}', f"{float(r['Percentage']):.1f}"]
        if fl:
            tf = fl / (us * 1e-6) / 1e3
            cells += [f'{fl:.2f}', f'{tf:.0f}', f'{tf / BF16_PEAK:.3f}']
        else:
            cells += ['-', '-', '-']
        if byt is not None:
            gbs = byt / (us * 1e-6) / 1e3
            cells += [f'{byt:.1f}' + ('' if w is not None else ' (read)'), f'{gbs:.0f}', f'{gbs / HBM_PEAK:.3f}']
        else:
            cells += ['-', '-', '-']
        print('| ' + ' | '.join(cells) + ' |')


if __name__ == '__main__':
    main()
