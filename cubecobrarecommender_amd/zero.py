"""Data-parallel optimizer step: bucketed reduce-scatter, Adam on the rank's shard, all-gather.

The reference trains on one host (train.py:99-102); SURVEY §8(e) shards the cube batches over
the GPUs of one node with one exchange step, the gradient reduction.  A plain all-reduce of the
46 MB fp32 gradient followed by a full Adam on every rank repeats the optimizer's ~34 B/param of
HBM traffic world times over.  Here (ZeRO-1):

  * the flat buffers are split into gradient buckets in the order backward finishes them
    (Layout.buckets, bf16 / fp8: both output layers first — final after forward_backward_a —,
    then the towers, then W1 in row chunks; fp32: the decoder output layer, the towers + E1,
    decoder_for_reg), each padded to a multiple of world*64;
  * each bucket's exchange is issued on the comm stream the moment its gradient is final: the
    output layers' at the trainer's hook inside forward_backward_a, the towers' and every W1 row
    chunk's at the trainer's bucket hooks inside forward_backward_b (chunk i's reduce-scatter then
    runs beside chunk i+1's gradient launch);
  * each bucket is reduce-scattered (SUM, then 1/world: the mean over the global batch, exactly
    the single-process gradient of world*B cubes) as soon as it is final, on a side stream, so
    the decoder-output bucket's exchange overlaps the towers' backward;
  * every rank runs TF Adam (cc_adam_dense) on its 1/world shard only and all-gathers the
    updated fp32 parameters in place; the bf16 operand shadow is refreshed locally.

With a bf16 operand shadow (the bf16 / fp8 paths) and the grouped-bias layout (Layout(group_biases=
True)), the kernels' parameters are all-gathered as the bf16 shadow the Adam launch wrote for the
shard — half the bytes of the fp32 values, and exactly what every kernel reads — while the fp32
biases (read in fp32 by the kernels) stay exact everywhere: their one small bucket is all-reduced
and every rank runs its Adam.  The fp32 master values of the other ranks' kernel shards are then
only brought in by gather_state() (checkpoints, tests).

Every rank ends the step with identical operands (shadow and biases); m and v are only kept current
on the owning rank's shard (the checkpoint writer gathers them, model.py).  Every backend runs the same two
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
        # bf16 shadow + grouped biases: gather the shadow, all-reduce the biases (module docstring)
        self.shadow_gather = (getattr(trainer, 'shadow', None) is not None
                              and getattr(trainer.layout, 'group_biases', False))
        if self.shadow_gather:
            bb = self.bucket('biases')
            bb['gfull'] = torch.zeros(bb['hi'] - bb['lo'], device=trainer.params.device, dtype=torch.float32)
        self.comm = torch.cuda.Stream(device=trainer.params.device) if trainer.params.is_cuda else None
        self.adam_events = []          # (e0, e1, n) around each shard's Adam when timing
        self.comm_events = {}          # (bucket, collective) -> [(e0, e1)] when timing
        self.timing = False
        self.no_comm = False           # capture a timing reference of the step without the exchange
        # the output layers' all-gather deferred to the head of the next step, beside its F / E1
        # gather / tower forward, its D1 launch waiting for it (trainer.hook_d1): nothing reads the
        # output layers' shadow between this step's Adam and the next D1 when the decoder operands
        # are read straight from the shadow (no Wo^T / MX-FP8 / fragment images refreshed from it)
        self.defer_out = (self.shadow_gather and self.comm is not None and bool(self.buckets)
                          and self.buckets[0]['name'] == 'output_layers' and trainer.dp_defer_out_ok())
        self.out_pending = False       # a deferred output-layer all-gather not yet issued

    def bucket(self, name):
        return next(b for b in self.buckets if b['name'] == name)

    # ------------------------------------------------------------------ collectives
    def _ev(self, b, what):
        """Record a timing event on the comm stream (timing mode); returns a closer."""
        if not self.timing:
            return lambda: None
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()

        def close():
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self.comm_events.setdefault((b['name'], what), []).append((e0, e1))
        return close

    def reduce_scatter(self, b, grads):
        src = grads[b['lo']:b['hi']]
        t = self._ev(b, 'reduce_scatter')
        if self.no_comm:      # (timing reference: the same step without the exchange)
            off = b['s0'] - b['lo']
            b['gshard'].copy_(src[off:off + b['chunk']])
        elif self.stage:
            out = torch.empty(b['chunk'], dtype=torch.float32)
            dist.reduce_scatter_tensor(out, src.cpu(), op=dist.ReduceOp.SUM, group=self.group)
            b['gshard'].copy_(out)
        else:
            dist.reduce_scatter_tensor(b['gshard'], src, op=dist.ReduceOp.SUM, group=self.group)
        if self.world > 1:
            b['gshard'].mul_(1.0 / self.world)
        t()

    def all_gather(self, b, buf):
        full = buf[b['lo']:b['hi']]
        off = b['s0'] - b['lo']
        if self.no_comm:
            return
        t = self._ev(b, 'all_gather')
        if self.stage:
            host = full.cpu()
            dist.all_gather_into_tensor(host, host[off:off + b['chunk']], group=self.group)
            full.copy_(host)
        else:           # in place: my shard already sits at rank * chunk inside the output
            dist.all_gather_into_tensor(full, full[off:off + b['chunk']], group=self.group)
        t()

    def all_reduce_mean(self, b, grads):
        """The biases bucket: the full mean gradient on every rank (b['gfull'])."""
        src = grads[b['lo']:b['hi']]
        t = self._ev(b, 'all_reduce')
        if self.stage:
            host = src.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=self.group)
            b['gfull'].copy_(host)
        else:
            b['gfull'].copy_(src)
            if not self.no_comm:
                dist.all_reduce(b['gfull'], op=dist.ReduceOp.SUM, group=self.group)
        if self.world > 1:
            b['gfull'].mul_(1.0 / self.world)
        t()

    def update(self, b, adam_fn, gate=None, gather=True):
        """Reduce-scatter bucket b, Adam on this rank's shard, all-gather the parameters (the
        bf16 shadow in shadow_gather mode; gather=False: left to the caller); the biases bucket:
        all-reduce, Adam on every rank.  gate: an event the Adam waits for (the step's last reader
        of the bucket's old shadow)."""
        full = self.shadow_gather and b['name'] == 'biases'
        if full:
            self.all_reduce_mean(b, self.tr.grads)
        else:
            self.reduce_scatter(b, self.tr.grads)
        if gate is not None:
            torch.cuda.current_stream().wait_event(gate)
        if self.timing:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        if full:
            adam_fn(b['lo'], b['hi'] - b['lo'], b['gfull'])
        else:
            adam_fn(b['s0'], b['chunk'], b['gshard'])
        if self.timing:
            e1.record()
            self.adam_events.append((e0, e1, b['hi'] - b['lo'] if full else b['chunk']))
        if full or not gather:
            return
        self.all_gather(b, self.tr.shadow if self.shadow_gather else self.tr.params)

    def flush_out(self):
        """Issue a deferred output-layer all-gather now (every rank: a collective) and make the
        current stream wait for it — before the shadow is read outside a step."""
        if not self.out_pending:
            return
        self.out_pending = False
        main = torch.cuda.current_stream()
        e = torch.cuda.Event()
        e.record(main)
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(e)
            self.all_gather(self.buckets[0], self.tr.shadow)
        main.wait_stream(self.comm)

    def warm(self):
        """Run every collective of the step once on scratch tensors of the buckets' sizes, so the
        communicator's lazy set-up happens before a step is captured into a graph."""
        if self.stage:
            return
        for b in self.buckets:
            src = torch.zeros(b['hi'] - b['lo'], device=self.tr.params.device, dtype=torch.float32)
            if self.shadow_gather and b['name'] == 'biases':
                dist.all_reduce(src, op=dist.ReduceOp.SUM, group=self.group)
                continue
            out = torch.empty(b['chunk'], device=src.device, dtype=torch.float32)
            dist.reduce_scatter_tensor(out, src, op=dist.ReduceOp.SUM, group=self.group)
            g = src.to(torch.bfloat16) if self.shadow_gather else src
            off = b['s0'] - b['lo']
            dist.all_gather_into_tensor(g, g[off:off + b['chunk']], group=self.group)
        torch.cuda.synchronize()

    def gather_state(self):
        """Make m and v (and, in shadow_gather mode, the fp32 kernel parameters) complete on every
        rank (checkpointing): all-gather each sharded bucket."""
        self.flush_out()
        for b in self.buckets:
            if self.shadow_gather and b['name'] == 'biases':
                continue      # replicated
            self.all_gather(b, self.tr.m)
            self.all_gather(b, self.tr.v)
            if self.shadow_gather:
                self.all_gather(b, self.tr.params)

    # ------------------------------------------------------------------ one training step
    def step(self, phase_a, phase_b, rest, adam_fn, refresh_fn, timing=False, after_b=None, hooks=False):
        """phase_a / phase_b: the two halves of forward_backward (graph replays or eager);
        rest: counters + transposed operand copies; adam_fn(lo, n, g) / refresh_fn(lo, hi);
        after_b: main-stream work that needs phase_b's consumers of the batch buffers done but not
        the exchange (the next step's F), issued beside the later buckets' exchange.  The whole
        call can be captured into one graph (RCCL: the collectives run on the comm stream, which
        forks from and joins the capturing stream).  hooks (phase_a launched eagerly or captured in
        the same graph, not a separate graph replay): the first bucket's reduce-scatter starts at
        the trainer's hook_out and its Adam / all-gather wait for hook_dx."""
        self.timing = timing
        first, later = self.buckets[0], self.buckets[1:]
        refresh = (lambda lo, hi: None) if self.shadow_gather else refresh_fn   # (shadow gathered)
        if self.comm is None:          # CPU (gloo tests): no streams
            phase_a()
            phase_b()
            if after_b is not None:
                after_b()
            for b in self.buckets:
                self.update(b, adam_fn)
                refresh(b['lo'], b['hi'])
            rest()
            self.timing = False
            return
        main = torch.cuda.current_stream()
        ev, gate = torch.cuda.Event(), None
        if self.defer_out:   # the previous step's output-layer all-gather (idempotent at the first)
            self.out_pending = False
            e0 = torch.cuda.Event()
            e0.record(main)
            ag = torch.cuda.Event()
            with torch.cuda.stream(self.comm):
                self.comm.wait_event(e0)
                self.all_gather(first, self.tr.shadow)
                ag.record(self.comm)
            if hooks:      # the forward's D1 launch waits for it (trainer.hook_d1)
                self.tr.hook_d1 = lambda: main.wait_event(ag)
            else:
                main.wait_event(ag)
        early = []   # later buckets started from the trainer's bucket hooks inside phase_b
        if hooks:   # the first bucket's reduce-scatter as soon as its gradient is final (before dX)
            gate = torch.cuda.Event()
            self.tr.hook_out = lambda: ev.record(main)
            self.tr.hook_dx = lambda: gate.record(main)
            names = set(self.tr.bucket_hook_names()) if hasattr(self.tr, 'bucket_hook_names') else set()
            early = [b for b in later if b['name'] in names]

            def launch(b):   # on the comm stream after everything issued so far on main
                e = torch.cuda.Event()
                e.record(main)
                with torch.cuda.stream(self.comm):
                    self.comm.wait_event(e)
                    self.update(b, adam_fn)
                    refresh(b['lo'], b['hi'])
            self.tr.bucket_hooks = {b['name']: (lambda b=b: launch(b)) for b in early}
        phase_a()
        if hooks:
            assert self.tr.hook_out is None and self.tr.hook_dx is None, 'forward_backward_a fired no hooks'
            assert getattr(self.tr, 'hook_d1', None) is None, 'forward_backward_a fired no hook_d1'
        else:
            ev.record(main)
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(ev)
            self.update(first, adam_fn, gate, gather=not self.defer_out)
            refresh(first['lo'], first['hi'])
        self.out_pending = self.defer_out
        phase_b()
        if hooks:
            assert not self.tr.bucket_hooks, f'forward_backward_b left bucket hooks {list(self.tr.bucket_hooks)}'
        ev2 = torch.cuda.Event()
        ev2.record(main)
        if after_b is not None:
            after_b()
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(ev2)
            for b in later:
                if any(b is e for e in early):
                    continue
                self.update(b, adam_fn)
                refresh(b['lo'], b['hi'])
        main.wait_stream(self.comm)
        rest()
        self.timing = False
