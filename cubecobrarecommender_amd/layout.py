"""Flat parameter layout shared by the kernels, Adam, the bf16 shadow and checkpoints.

Tensor order is the Keras creation order of ``src/ml/model.py`` (:27-33 encoder, :58-64 decoder,
:92-98 ``decoder`` then ``decoder_for_reg``).  Mirrors ``cc_param_layout`` (api.cpp); a CPU test
checks the two agree.
"""
import numpy as np

LAYERS = ('encoder/encoded_1', 'encoder/encoded_2', 'encoder/encoded_3', 'encoder/bottleneck',
          'decoder/decoded_1', 'decoder/decoded_2', 'decoder/decoded_3', 'decoder/reconstruct',
          'decoder_for_reg/decoded_1', 'decoder_for_reg/decoded_2', 'decoder_for_reg/decoded_3',
          'decoder_for_reg/reconstruct')
NAMES = tuple(n for l in LAYERS for n in (l + '/kernel', l + '/bias'))


def layer_shapes(V, d):
    return ((V, d), (d, 256), (256, 128), (128, 64),
            (64, 128), (128, 256), (256, d), (d, V),
            (64, 128), (128, 256), (256, d), (d, V))


def _round_up(x, a):
    return (x + a - 1) // a * a


class Layout:
    """name -> (offset, shape) in the flat fp32 buffer; 64-element aligned tensors.

    align > 1 (data-parallel training, align = world * 64) additionally starts the decoder output
    layer and the decoder_for_reg block on multiples of `align` and pads every block to one, so the
    three gradient buckets (towers + E1 | decoder output layer | decoder_for_reg) split into equal
    per-rank shards (zero.py).  align == 1 is exactly cc_param_layout.

    group_biases (data parallel with a bf16 shadow): every bias moves into one trailing 'biases'
    block, and the kernels are ordered by their gradients' exchange buckets (each bucket a
    multiple of `align`):
      W1 (row chunks: w1_chunks buckets, exchanged chunk by chunk as the W1-gradient kernel runs
      them; the towers, final just before W1's gradient, ride in the last chunk's bucket) | the
      encoder / decoder towers | the decoder_for_reg towers | the decoder output layer | the
      decoder_for_reg output layer | biases.
    The two output layers are one early bucket (final after the output-layer kernels, exchanged
    beside the towers' backward); without the regulariser the decoder_for_reg tensors sit outside
    every bucket (never updated, as the one-process Adam range skips them).  zero.py then
    all-gathers the kernels' bf16 shadow (half the bytes of the fp32 parameters) and keeps the
    fp32 biases — which the kernels read in fp32 — exact on every rank by all-reducing their
    gradients and running their Adam on every rank."""

    def __init__(self, V, d, align=1, group_biases=False, w1_chunks=1):
        self.V, self.d, self.align = int(V), int(d), int(align)
        self.group_biases = bool(group_biases)
        self.entries = {}
        shapes = layer_shapes(V, d)
        if self.group_biases:
            self._init_grouped(shapes, max(1, int(w1_chunks)))
            return
        o = 0
        for li, (fi, fo) in enumerate(shapes):
            if li in (7, 8):
                o = _round_up(o, self.align)
            parts = ((LAYERS[li] + '/kernel', (fi, fo)),) if self.group_biases else \
                ((LAYERS[li] + '/kernel', (fi, fo)), (LAYERS[li] + '/bias', (fo,)))
            for name, shape in parts:
                self.entries[name] = (o, shape)
                o += (int(np.prod(shape)) + 63) // 64 * 64
            if li == 7:
                o = _round_up(o, self.align)
                self.main_total = o
        self.total = _round_up(o, self.align)

    def _init_grouped(self, shapes, nchunks):
        """The data-parallel bf16 / fp8 layout (class docstring): kernels in bucket order, biases last."""
        a = self.align
        o = 0
        marks = {}

        def put(li, name, shape):
            nonlocal o
            self.entries[LAYERS[li] + name] = (o, shape)
            o += (int(np.prod(shape)) + 63) // 64 * 64
        put(0, '/kernel', shapes[0])
        w1 = self.V * self.d
        # W1 row chunks: boundaries at multiples of q rows — q a multiple of 64 (the gradient
        # kernel's row tiles) with q * d a multiple of align, so every chunk is whole bucket shards
        # for any world (align = 64 * world need not divide 64 * d when world is not a power of
        # two); the last chunk padded with the block, chunks that round away dropped
        q = int(np.lcm(64, a // int(np.gcd(a, self.d))))
        rows = [min(self.V, (self.V * c // nchunks + q - 1) // q * q) for c in range(nchunks + 1)]
        rows[0], rows[-1] = 0, self.V
        o = _round_up(o, a)
        self.w1_chunks = [(r0, r1) for r0, r1 in zip(rows[:-1], rows[1:]) if r1 > r0]
        self.w1_bounds = [r0 * self.d for r0, _ in self.w1_chunks] + [o]
        assert all(b % a == 0 for b in self.w1_bounds), ('W1 chunk boundaries off the bucket alignment', a)
        assert w1 <= o
        marks['towers_lo'] = o
        for li in (1, 2, 3, 4, 5, 6):
            put(li, '/kernel', shapes[li])
        o = _round_up(o, a)
        marks['towers_hi'] = o
        for li in (8, 9, 10):
            put(li, '/kernel', shapes[li])
        o = _round_up(o, a)
        marks['reg_towers_hi'] = o
        put(7, '/kernel', shapes[7])
        o = _round_up(o, a)
        marks['out_hi'] = o
        put(11, '/kernel', shapes[11])
        o = _round_up(o, a)
        marks['reg_out_hi'] = o
        self.bias_lo = o
        for li, (fi, fo) in enumerate(shapes):
            self.entries[LAYERS[li] + '/bias'] = (o, (fo,))
            o += (fo + 63) // 64 * 64
        self.total = self.main_total = _round_up(o, a)   # (the main model is no longer a prefix)
        self.marks = marks

    def buckets(self, with_reg):
        """Gradient buckets in the order backward produces them: (name, lo, hi)."""
        if self.group_biases:
            m = self.marks
            out = [('output_layers', m['reg_towers_hi'], m['reg_out_hi'] if with_reg else m['out_hi'])]
            b = list(self.w1_bounds)
            b[-1] = m['reg_towers_hi'] if with_reg else m['towers_hi']   # the towers ride in the last chunk
            out += [(f'w1_{i}', b[i], b[i + 1]) for i in range(len(b) - 1)]
            out.append(('biases', self.bias_lo, self.total))
            return out
        out = [('decoder_output', self.offset('decoder/reconstruct/kernel'), self.main_total),
               ('towers_e1', 0, self.offset('decoder/reconstruct/kernel'))]
        if with_reg:
            out.append(('decoder_for_reg', self.main_total, self.total))
        return out

    def convert(self, flat, other):
        """Re-lay a flat buffer written in layout `other` into this layout (numpy)."""
        return self.pack(other.unpack(flat))

    def offset(self, name):
        return self.entries[name][0]

    def shape(self, name):
        return self.entries[name][1]

    def view(self, flat, name):
        o, shape = self.entries[name]
        n = int(np.prod(shape))
        return flat[o:o + n].reshape(shape)

    def pack(self, params, out=None):
        """dict name -> array  ->  flat float32 numpy buffer (padding zero)."""
        flat = np.zeros(self.total, np.float32) if out is None else out
        for name in NAMES:
            if name in params:
                o, shape = self.entries[name]
                flat[o:o + int(np.prod(shape))] = np.asarray(params[name], np.float32).reshape(-1)
        return flat

    def unpack(self, flat):
        flat = np.asarray(flat)
        return {name: self.view(flat, name).copy() for name in NAMES}


def glorot_flat(V, d, seed=0):
    """Keras Dense defaults: glorot_uniform kernels, zero biases — as one flat float32 buffer."""
    lay = Layout(V, d)
    rng = np.random.default_rng(seed)
    flat = np.zeros(lay.total, np.float32)
    for li, (fi, fo) in enumerate(layer_shapes(V, d)):
        o, shape = lay.entries[LAYERS[li] + '/kernel']
        lim = np.sqrt(6.0 / (fi + fo))
        flat[o:o + fi * fo] = rng.uniform(-lim, lim, fi * fo).astype(np.float32)
    return flat
