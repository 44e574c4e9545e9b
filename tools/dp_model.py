"""Modelled exposed gradient exchange of the data-parallel step at W ranks.

Not a measurement: a timeline of one rank's comm stream against its compute, from
  * the buckets' sizes (layout.Layout, the bf16 / fp8 grouped layout: fp32 reduce-scatter, bf16
    all-gather of the kernels, fp32 all-reduce of the biases),
  * per-rank compute segments measured on one GPU (the 1-rank RCCL profile, profiles/r04ak_dp_*,
    and the one-process kernel stats): when each bucket's gradient is final, when backward ends,
  * a link model: a reduce-scatter / all-gather of S bytes moves S (W-1)/W per rank at an
    effective bus bandwidth `bus` (7 xGMI links x ~153 GB/s per direction if every link carries a
    share; one link if a single ring does), plus a fixed latency `lat` per collective,
  * the sharded Adam at `adam_bw` over 26 B per element of the shard.
The comm stream runs its work in issue order (zero.py: one communicator, one stream); the
exposed time is when it finishes minus when the rank's backward ends.

  * defer_out (zero.py's default where the decoder reads Wo straight from the shadow): the output
    layers' all-gather leaves this step's comm timeline and runs at the next step's head, beside
    its E1 gather and tower forward (`t_head`); only what outlasts that window is exposed there.

  python tools/dp_model.py [--world 8] [--bus 1.07e12] [--lat 8e-6] [--chunks 1 2 4] [--defer-out 0 1]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cubecobrarecommender_amd.layout import Layout


def model(V=22000, d=256, reg=True, world=8, chunks=4, bus=1.07e12, lat=8e-6, adam_bw=5.0e12,
          t_out=0.0, t_dx_done=40e-6, t_towers=67e-6, t_w1=14e-6, defer_out=False, t_head=32e-6):
    """Times in seconds from the moment the output layers' gradients are final (the D2 kernel's
    end).  t_dx_done: both dX products done (the output bucket's Adam may start); t_towers: the
    towers' gradient final; t_w1: the W1-gradient kernel's duration (split evenly over chunks)."""
    lay = Layout(V, d, align=world * 64, group_biases=True, w1_chunks=chunks)
    f = (world - 1) / world
    comm = 0.0
    log = []

    def coll(name, nbytes, ready):
        nonlocal comm
        start = max(comm, ready)
        comm = start + lat + nbytes * f / bus
        log.append((name, start, comm))

    def adam(name, n, ready):
        nonlocal comm
        start = max(comm, ready)
        comm = start + n / world * 26 / adam_bw
        log.append((name, start, comm))
    backward_end = t_towers + t_w1
    head = 0.0   # exposed at the next step's head (defer_out)
    for name, lo, hi in lay.buckets(reg):
        n = hi - lo
        if name == 'output_layers':
            coll('rs ' + name, 4 * n, t_out)
            adam('adam ' + name, n, t_dx_done)
            if defer_out:
                head = max(0.0, lat + 2 * n * f / bus - t_head)
            else:
                coll('ag ' + name, 2 * n, 0)
        elif name.startswith('w1_'):   # (the last chunk's bucket also holds the towers)
            i = int(name[3:])
            ready = t_towers + t_w1 * (i + 1) / len(lay.w1_chunks)
            coll('rs ' + name, 4 * n, ready)
            adam('adam ' + name, n, 0)
            coll('ag ' + name, 2 * n, 0)
        else:   # biases: all-reduce = reduce-scatter + all-gather of the fp32 values
            coll('ar ' + name, 2 * 4 * n, backward_end)
    return max(0.0, comm - backward_end) + head, comm, backward_end, log


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--world', type=int, default=8)
    ap.add_argument('--d', type=int, default=256)
    ap.add_argument('--reg', type=int, default=1)
    ap.add_argument('--bus', type=float, nargs='+', default=[1.07e12, 0.6e12, 0.153e12])
    ap.add_argument('--lat', type=float, nargs='+', default=[3e-6, 8e-6])
    ap.add_argument('--chunks', type=int, nargs='+', default=[1, 2, 4])
    ap.add_argument('--defer-out', type=int, nargs='+', default=[0, 1])
    ap.add_argument('--verbose', action='store_true')
    a = ap.parse_args()
    seg = (dict(t_dx_done=40e-6, t_towers=67e-6, t_w1=14e-6) if a.d <= 256 else
           dict(t_dx_done=190e-6, t_towers=280e-6, t_w1=81e-6))
    for dfr in a.defer_out:
        for bus in a.bus:
            for lat in a.lat:
                row = []
                for c in a.chunks:
                    exp, end, be, log = model(d=a.d, reg=bool(a.reg), world=a.world, chunks=c, bus=bus, lat=lat,
                                              defer_out=bool(dfr), **seg)
                    row.append(f'chunks {c}: exposed {exp * 1e6:6.1f} us')
                    if a.verbose:
                        for nm, s, e in log:
                            print(f'    {nm:22s} {s * 1e6:7.1f} -> {e * 1e6:7.1f} us')
                print(f'W={a.world} d={a.d} reg={a.reg} defer_out={dfr} bus {bus / 1e9:6.0f} GB/s '
                      f'lat {lat * 1e6:3.0f} us | ' + ' | '.join(row))


if __name__ == '__main__':
    main()
