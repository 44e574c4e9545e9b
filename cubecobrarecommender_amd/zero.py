"""Data-parallel optimizer step: bucketed reduce-scatter, Adam on the rank's shard, all-gather.

The reference trains on one host (train.py:99-102); SURVEY §8(e) shards the cube batches over
the GPUs of one node with one exchange step, the gradient reduction.  A plain all-reduce of the
46 MB fp32 gradient followed by a full Adam on every rank repeats the optimizer's ~34 B/param of
HBM traffic world times over.  Here (ZeRO-1):

  * the flat buffers are split into gradient buckets in the order backward finishes them
    (Layout.buckets: the decoder output layer first — final after forward_backward_a —, then
    the towers + E1, then decoder_for_reg), each padded to a multiple of world*64;
  * each bucket is reduce-scattered (SUM, then 1/world: the mean over the global batch, exactly
    the single-process gradient of world*B cubes) as soon as it is final, on a side stream, so
    the decoder-output bucket's exchange overlaps the towers' backward;
  * every rank runs TF Adam (cc_adam_dense) on its 1/world shard only and all-gathers the
    updated fp32 parameters in place; the bf16 operand shadow is refreshed locally.

Every rank ends the step with identical parameters; m and v are only kept current on the owning
rank's shard (the checkpoint writer gathers them, model.py).  Every backend runs the same two
collectives RCCL runs (reduce_scatter_tensor, in-place all_gather_into_tensor): gloo takes them on
CPU tensors, so with gloo and device buffers (several ranks rehearsed on one GPU) each bucket is
staged through a host copy around the identical call.
"""
import torch
import torch.distributed as dist


class ShardedStep:
    def __init__(self, trainer, group=None):
        self.tr = trainer
        self.group = group
        self.world = trainer.cfg.world
        self.rank = trainer.cfg.rank
        self.nccl = dist.get_backend(group) == 'nccl'
        # gloo + device buffers: host staging around the same collective calls
        self.stage = (not self.nccl) and trainer.params.is_cuda
        self.buckets = []
        for name, lo, hi in trainer.layout.buckets(trainer.use_reg):
            size = hi - lo
            assert size % (self.world * 64) == 0, (name, size)
            chunk = size // self.world
            self.buckets.append({
                'name': name, 'lo': lo, 'hi': hi, 'chunk': chunk, 's0': lo + self.rank * chunk,
                'gshard': torch.zeros(chunk, device=trainer.params.device, dtype=torch.float32)})
        self.comm = torch.cuda.Stream(device=trainer.params.device) if trainer.params.is_cuda else None
        self.adam_events = []          # (e0, e1, n) around each shard's Adam when timing

    def bucket(self, name):
        return next(b for b in self.buckets if b['name'] == name)

    # ------------------------------------------------------------------ collectives
    def reduce_scatter(self, b, grads):
        src = grads[b['lo']:b['hi']]
        if self.stage:
            out = torch.empty(b['chunk'], dtype=torch.float32)
            dist.reduce_scatter_tensor(out, src.cpu(), op=dist.ReduceOp.SUM, group=self.group)
            b['gshard'].copy_(out)
        else:
            dist.reduce_scatter_tensor(b['gshard'], src, op=dist.ReduceOp.SUM, group=self.group)
        b['gshard'].mul_(1.0 / self.world)

    def all_gather(self, b, buf):
        full = buf[b['lo']:b['hi']]
        off = b['s0'] - b['lo']
        if self.stage:
            host = full.cpu()
            dist.all_gather_into_tensor(host, host[off:off + b['chunk']], group=self.group)
            full.copy_(host)
        else:           # in place: my shard already sits at rank * chunk inside the output
            dist.all_gather_into_tensor(full, full[off:off + b['chunk']], group=self.group)

    def update(self, b, adam_fn, timing=False):
        """Reduce-scatter bucket b, Adam on this rank's shard, all-gather the parameters."""
        self.reduce_scatter(b, self.tr.grads)
        if timing:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        adam_fn(b['s0'], b['chunk'], b['gshard'])
        if timing:
            e1.record()
            self.adam_events.append((e0, e1, b['chunk']))
        self.all_gather(b, self.tr.params)

    def gather_state(self):
        """Make m and v complete on every rank (checkpointing): all-gather each bucket's shards."""
        for b in self.buckets:
            self.all_gather(b, self.tr.m)
            self.all_gather(b, self.tr.v)

    # ------------------------------------------------------------------ one training step
    def step(self, phase_a, phase_b, rest, adam_fn, refresh_fn, timing=False):
        """phase_a / phase_b: the two halves of forward_backward (graph replays or eager);
        rest: counters + transposed operand copies; adam_fn(lo, n, g) / refresh_fn(lo, hi)."""
        first, later = self.buckets[0], self.buckets[1:]
        if self.comm is None:          # CPU (gloo tests): no streams
            phase_a()
            phase_b()
            for b in self.buckets:
                self.update(b, adam_fn)
                refresh_fn(b['lo'], b['hi'])
            rest()
            return
        main = torch.cuda.current_stream()
        phase_a()
        ev = torch.cuda.Event()
        ev.record(main)
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(ev)
            self.update(first, adam_fn, timing)
            refresh_fn(first['lo'], first['hi'])
        phase_b()
        ev2 = torch.cuda.Event()
        ev2.record(main)
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(ev2)
            for b in later:
                self.update(b, adam_fn, timing)
                refresh_fn(b['lo'], b['hi'])
        main.wait_stream(self.comm)
        rest()
