"""Codec program builder: DenseNet config -> list of gpi_conv_desc.

The reference composes its encoder / decoder from nn.Sequential blocks
(bottleneck/codec.py:150-298, Encoder.py:133-196, Decoder.py:163-305) and lets
autograd + cuDNN run them layer by layer.  Here the same structure is
compiled once, per batch layout, into a flat *program* of fused conv
operators that libgpi_hip.so executes:

  * every tensor of the network is a workspace *buffer* [B, C, H, W] of raw
    (pre-BatchNorm) values; a dense block is ONE buffer whose layers append
    their growth channels in place, so torch.cat never happens;
  * a BatchNorm+ReLU is never materialised: the consumer conv applies it on
    load, from the per-channel fp64 sums the producer's epilogue wrote
    (BN-statistics slots are allocated per buffer channel and group);
  * backward wiring: every BN-consumed buffer gets an S buffer (sum over its
    BN consumers of gamma * dL/d(bn)); the first consumer in backward order
    overwrites it, later ones accumulate.

Sizes are element offsets; the engine owns the tensors.
"""
import ctypes as C

from . import _lib as L


class Arena(object):
    """Bump allocator of element offsets (64-element aligned)."""

    def __init__(self, align=64):
        self.size = 0
        self.align = align

    def alloc(self, n):
        off = self.size
        self.size += (int(n) + self.align - 1) // self.align * self.align
        return off


class Buffer(object):
    def __init__(self, name, C_, H, W):
        self.name, self.C, self.H, self.W = name, C_, H, W
        self.off = None          # forward values (per-call workspace offset)
        self.stat = None         # stat slot of channel 0
        self.s_off = None        # S / gradient buffer
        self.bn_consumed = False
        self.external = False

    @property
    def per_sample(self):
        return self.C * self.H * self.W


class Op(object):
    """Python-side mirror of gpi_conv_desc before offsets are resolved."""

    def __init__(self, name, src, c0, cin, dst, d0, cout, k, stride, pad, upsample, w, bn=None, epilogue=None,
                 drop=False):
        self.name = name
        self.drop = bool(drop)   # nn.Dropout2d on this conv's output (codec.py:177-178,218-282)
        self.drop_off = None
        self.src, self.c0, self.cin = src, c0, cin
        self.dst, self.d0, self.cout = dst, d0, cout
        self.k, self.stride, self.pad, self.upsample = k, stride, pad, upsample
        self.w = w               # param name of the weight
        self.bn = bn             # param prefix of the input BatchNorm (None: identity)
        self.epilogue = epilogue
        self.gin_accumulate = 0
        self.desc = None


class CodecProgram(object):
    """Ordered conv ops + buffers of one encoder or decoder."""

    def __init__(self, kind, drop_rate=0.0):
        self.kind = kind
        self.drop_rate = float(drop_rate)
        if not 0.0 <= self.drop_rate < 1.0:
            raise ValueError('drop_rate must be in [0, 1)')
        self.ops = []
        self.buffers = []
        self.input = None       # Buffer fed from outside (image / latent map)
        self.output = None      # Buffer read by the outside (features / (mu, logsigma))

    def buf(self, name, C_, H, W):
        b = Buffer(name, C_, H, W)
        self.buffers.append(b)
        return b

    def conv(self, *a, **k):
        if k.pop('dropout', False) and self.drop_rate > 0:
            k['drop'] = True
        op = Op(*a, **k)
        if op.bn is not None:
            op.src.bn_consumed = True
        self.ops.append(op)
        return op

    # ------------------------------------------------------------ lowering
    def layout(self, B, ws, stats, parts, groups, param_offset, grad=True):
        """Assign workspace / stat / partial-slab offsets for batch B."""
        for b in self.buffers:
            if b.external:
                continue
            b.off = ws.alloc(B * b.per_sample)
            if b.bn_consumed:
                b.stat = stats.alloc(b.C) if isinstance(stats, Arena) else None
        # Dropout2d channel scales [B][cout] of every dropout op, one contiguous region
        self.drop_off = ws.size
        for op in self.ops:
            if op.drop:
                op.drop_off = ws.alloc(B * op.cout)
        self.drop_numel = ws.size - self.drop_off
        # backward buffers
        if grad:
            for b in self.buffers:
                if b.bn_consumed or b in (self.output, self.input) and not b.external:
                    b.s_off = ws.alloc(B * b.per_sample)
        # gin_accumulate: first writer in backward order overwrites
        seen = {}
        for op in reversed(self.ops):
            chans = set(range(op.c0, op.c0 + op.cin))
            done = seen.setdefault(id(op.src), set())
            inter = chans & done
            if inter and inter != chans:
                raise RuntimeError('mixed gradient initialisation in %s' % op.name)
            op.gin_accumulate = 1 if inter else 0
            done |= chans
        descs = []
        for op in self.ops:
            d = L.ConvDesc()
            d.cin, d.cout, d.k, d.stride, d.pad, d.upsample = op.cin, op.cout, op.k, op.stride, op.pad, op.upsample
            d.h_in, d.w_in = op.src.H, op.src.W
            d.h_out, d.w_out = op.dst.H, op.dst.W
            d.in_off = -1 if op.src.external else op.src.off
            d.in_ctot, d.in_c0 = op.src.C, op.c0
            d.in_bn = 1 if op.bn is not None else 0
            d.gin_accumulate = op.gin_accumulate
            if op.bn is not None:
                d.gamma_off = param_offset(op.bn + '.weight')
                d.beta_off = param_offset(op.bn + '.bias')
                d.in_stat = op.src.stat + op.c0
            else:
                d.gamma_off = d.beta_off = d.in_stat = -1
            d.w_off = param_offset(op.w)
            d.out_off = op.dst.off
            d.out_ctot, d.out_c0 = op.dst.C, op.d0
            d.out_stat = (op.dst.stat + op.d0) if op.dst.bn_consumed else -1
            if op.epilogue is not None:
                d.epilogue = op.epilogue
            else:
                d.epilogue = L.EPI_STORE_STATS if op.dst.bn_consumed else L.EPI_STORE
            d.gout_mode = 0 if op.dst.bn_consumed else 1
            d.gout_off = op.dst.s_off if op.dst.s_off is not None else -1
            if op.bn is not None or (not op.src.external and op.src.s_off is not None):
                d.gin_off = op.src.s_off if op.src.s_off is not None else -1
            else:
                d.gin_off = -1
            nb = C.c_int32(0)
            L.check(L.lib().gpi_conv_blocks(C.byref(d), C.byref(groups), C.byref(nb)), 'gpi_conv_blocks(%s)' % op.name)
            op.blocks = nb.value
            op.numel = op.cout * op.cin * op.k * op.k
            op.rowlen = op.numel + (2 * op.cin if op.bn is not None else 0)
            d.wpart_off = parts.alloc(op.blocks * op.rowlen) if grad else -1
            d.drop_off = op.drop_off if op.drop else -1
            op.desc = d
            descs.append(d)
        arr = (L.ConvDesc * len(descs))(*descs)
        return arr

    def drop_ops(self):
        """[(op name, workspace offset, cout)] of the Dropout2d ops (batch-major [B][cout] each)."""
        return [(op.name, op.drop_off, op.cout) for op in self.ops if op.drop]

    def reduce_items(self, param_offset):
        """Slab reductions: the conv weight, then the input BN's (dgamma, dbeta) that
        follow it in every slab row (one item when gamma/beta are adjacent parameters)."""
        items = []

        def item(part, dst, numel, stride, blocks):
            it = L.ReduceItem()
            it.part_off, it.w_off, it.numel, it.row_stride, it.blocks = part, dst, numel, stride, blocks
            items.append(it)

        for op in self.ops:
            base = op.desc.wpart_off
            item(base, param_offset(op.w), op.numel, op.rowlen, op.blocks)
            if op.bn is not None:
                g, b = param_offset(op.bn + '.weight'), param_offset(op.bn + '.bias')
                if b == g + op.cin:
                    item(base + op.numel, g, 2 * op.cin, op.rowlen, op.blocks)
                else:
                    item(base + op.numel, g, op.cin, op.rowlen, op.blocks)
                    item(base + op.numel + op.cin, b, op.cin, op.rowlen, op.blocks)
        return items

    def reduce_counts(self, param_offset):
        """Number of reduce_items() entries each op contributes, in op order."""
        out = []
        for op in self.ops:
            n = 1
            if op.bn is not None:
                g, b = param_offset(op.bn + '.weight'), param_offset(op.bn + '.bias')
                n += 1 if b == g + op.cin else 2
            out.append(n)
        return out


# --------------------------------------------------------------------------
def encoder_program(imsize, blocks, growth, init_features, bn_size=8, bottleneck=True, drop_rate=0.0):
    """CNNEncoder (Encoder.py:133-196) -> program; output buffer = flattened features.
    drop_rate > 0: Dropout2d after every dense-layer conv and both transition convs
    (codec.py:177-178,218-219,226-227), as the reference's _DenseLayer / _Transition(down) place it."""
    P = CodecProgram('encoder', drop_rate)
    x = P.buf('input', 1, imsize, imsize)
    x.external = True
    P.input = x
    pad = 3 if imsize % 2 == 0 else 2
    h = imsize // 2
    nf = init_features
    D = P.buf('EncBlock1', nf + blocks[0] * growth, h, h)
    P.conv('features.In_conv', x, 0, 1, D, 0, nf, 7, 2, pad, 0, 'features.In_conv.weight')
    for i, nl in enumerate(blocks):
        for l in range(nl):
            cin = nf + l * growth
            name = 'features.EncBlock%d.denselayer%d' % (i + 1, l + 1)
            _dense_layer(P, name, D, cin, growth, bn_size, bottleneck, h)
        nf += nl * growth
        t = 'features.TransDown%d' % (i + 1)
        T = P.buf(t, nf // 2, h, h)
        P.conv(t + '.conv1', D, 0, nf, T, 0, nf // 2, 1, 1, 0, 0, t + '.conv1.weight', bn=t + '.norm1', dropout=True)
        nf //= 2
        h //= 2
        if i < len(blocks) - 1:
            Dn = P.buf('EncBlock%d' % (i + 2), nf + blocks[i + 1] * growth, h, h)
        else:
            Dn = P.buf('features', nf, h, h)
            P.output = Dn
        P.conv(t + '.conv2', T, 0, nf, Dn, 0, nf, 3, 2, 1, 0, t + '.conv2.weight', bn=t + '.norm2', dropout=True)
        D = Dn
    P.d_feat = nf * h * h
    return P


def _dense_layer(P, name, D, cin, growth, bn_size, bottleneck, h):
    """_DenseLayer (codec.py:150-182)."""
    if bottleneck and cin > bn_size * growth:
        Bt = P.buf(name + '.bottleneck', bn_size * growth, h, h)
        P.conv(name + '.conv1', D, 0, cin, Bt, 0, bn_size * growth, 1, 1, 0, 0, name + '.conv1.weight',
               bn=name + '.norm1')
        P.conv(name + '.conv2', Bt, 0, bn_size * growth, D, cin, growth, 3, 1, 1, 0, name + '.conv2.weight',
               bn=name + '.norm2', dropout=True)
    else:
        P.conv(name + '.conv1', D, 0, cin, D, cin, growth, 3, 1, 1, 0, name + '.conv1.weight', bn=name + '.norm1',
               dropout=True)


def decoder_program(latent_img_size, latent_img_features, init_features, blocks, growth, out_channels=2,
                    drop_rate=0.0, final_epilogue=None):
    """CNNDecoder (Decoder.py:163-305) -> program; input buffer = latent map image.
    drop_rate > 0: Dropout2d after every dense-layer conv, both transition-up convs and the first
    conv of last_decoding (codec.py:177-178,231-232,239-240,259-260), not after conv0 / conv2 / conv3."""
    P = CodecProgram('decoder', drop_rate)
    h = latent_img_size
    z = P.buf('latent', latent_img_features, h, h)
    P.input = z
    nf = init_features
    D = P.buf('DecBlock1', nf + blocks[0] * growth, h, h)
    P.conv('features.conv0', z, 0, latent_img_features, D, 0, nf, 3, 1, 1, 0, 'features.conv0.weight')
    for i, nl in enumerate(blocks):
        for l in range(nl):
            cin = nf + l * growth
            _dense_layer(P, 'features.DecBlock%d.denselayer%d' % (i + 1, l + 1), D, cin, growth, 4, False, h)
        nf += nl * growth
        if i < len(blocks) - 1:
            t = 'features.TransUp%d' % (i + 1)
            U = P.buf(t, nf // 2, h, h)
            P.conv(t + '.conv1', D, 0, nf, U, 0, nf // 2, 1, 1, 0, 0, t + '.conv1.weight', bn=t + '.norm1',
                   dropout=True)
            nf //= 2
            h *= 2
            D2 = P.buf('DecBlock%d' % (i + 2), nf + blocks[i + 1] * growth, h, h)
            P.conv(t + '.conv2', U, 0, nf, D2, 0, nf, 3, 1, 1, 1, t + '.conv2.weight', bn=t + '.norm2',
                   dropout=True)
            D = D2
    t = 'features.LastTransUp'
    L1 = P.buf(t + '.1', nf // 2, h, h)
    P.conv(t + '.conv1', D, 0, nf, L1, 0, nf // 2, 3, 1, 1, 0, t + '.conv1.weight', bn=t + '.norm1', dropout=True)
    L2 = P.buf(t + '.2', nf // 4, 2 * h, 2 * h)
    P.conv(t + '.conv2', L1, 0, nf // 2, L2, 0, nf // 4, 3, 1, 1, 1, t + '.conv2.weight', bn=t + '.norm2')
    out = P.buf('output', out_channels, 2 * h, 2 * h)
    P.conv(t + '.conv3', L2, 0, nf // 4, out, 0, out_channels, 5, 1, 2, 0, t + '.conv3.weight', bn=t + '.norm3',
           epilogue=final_epilogue)
    P.output = out
    return P
