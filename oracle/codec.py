"""torch.nn.functional restatement of the DenseNet conv codec (CPU reference).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Follows the reference's module structure and parameter names so that a
reference ``state_dict`` drives it directly:
  * CNNEncoder   bottleneck/Encoder.py:133-196
  * CNNDecoder   bottleneck/Decoder.py:163-305
  * blocks       bottleneck/codec.py:131-298, 484-504
BatchNorm is always in training mode (nothing in the reference calls
``.eval()``), eps 1e-5.

``masks`` (optional, every function): {BN / FC layer name: 0/1 tensor of the shape of that
layer's ReLU input}.  A ReLU listed there takes the given branch decisions instead of its own
sign test: the GPU parity tests pass the masks the fp32 kernels took, so that activations
within rounding of 0 (a few tens among the ~10^7 of a C64 batch) do not flip one implementation's
gradient against the other's.  Off the ties the given mask and the sign test agree (checked by
the tests), so the oracle stays an independent fp64 computation.
"""
import torch
import torch.nn.functional as F

BN_EPS = 1e-5


# (layer, elements whose given mask disagrees with the sign of the oracle's own input, largest
# |input| among them, elements): filled when masks are given, read by the tests
MASK_AUDIT = []


def _relu(x, masks, name):
    if masks is not None and name in masks:
        m = masks[name].to(torch.bool)
        assert m.shape == x.shape, (name, tuple(m.shape), tuple(x.shape))
        dis = m != (x.detach() > 0)
        MASK_AUDIT.append((name, int(dis.sum()), float(x.detach().abs()[dis].max()) if dis.any() else 0.0,
                           x.numel()))
        return x * m.to(x.dtype)
    return torch.relu(x)


def _bn_relu(x, p, name, masks=None):
    x = F.batch_norm(x, None, None, p[name + '.weight'], p[name + '.bias'],
                     training=True, momentum=0.0, eps=BN_EPS)
    return _relu(x, masks, name)


def _conv(x, p, name, stride=1, padding=0, drops=None):
    """Conv; ``drops`` {conv name: [B, C] channel scales} applies the Dropout2d that follows it
    (codec.py:177-178,218-219,226-227,231-232,239-240,259-260) with an injected mask."""
    w = p[name + '.weight']
    b = p.get(name + '.bias')
    y = F.conv2d(x, w, b, stride=stride, padding=padding)
    if drops is not None and name in drops:
        y = y * drops[name].to(y.dtype)[:, :, None, None]
    return y


def _up(x):
    return F.interpolate(x, scale_factor=2.0, mode='nearest')


def _dense_layer(x, p, name, in_features, growth, bn_size, bottleneck, masks=None, drops=None):
    """codec.py:150-182 (cat [x, y] on channels)."""
    if bottleneck and in_features > bn_size * growth:
        y = _conv(_bn_relu(x, p, name + '.norm1', masks), p, name + '.conv1')
        y = _conv(_bn_relu(y, p, name + '.norm2', masks), p, name + '.conv2', padding=1, drops=drops)
    else:
        y = _conv(_bn_relu(x, p, name + '.norm1', masks), p, name + '.conv1', padding=1, drops=drops)
    return torch.cat([x, y], 1)


def _dense_block(x, p, name, num_layers, in_features, growth, bn_size, bottleneck, masks=None, drops=None):
    for i in range(num_layers):
        x = _dense_layer(x, p, '%s.denselayer%d' % (name, i + 1), in_features + i * growth,
                         growth, bn_size, bottleneck, masks, drops)
    return x


def encoder_forward(p, x, imsize, blocks, growth, init_features, masks=None, drops=None):
    """CNNEncoder.forward -> (mean, logsigma)  (Encoder.py:147-196)."""
    if x.dim() < 4:
        x = x.unsqueeze(1)
    pad = 3 if imsize % 2 == 0 else 2
    h = _conv(x, p, 'features.In_conv', stride=2, padding=pad)
    nf = init_features
    for i, L in enumerate(blocks):
        h = _dense_block(h, p, 'features.EncBlock%d' % (i + 1), L, nf, growth, 8, True, masks, drops)
        nf = nf + L * growth
        t = 'features.TransDown%d' % (i + 1)
        h = _conv(_bn_relu(h, p, t + '.norm1', masks), p, t + '.conv1', drops=drops)
        h = _conv(_bn_relu(h, p, t + '.norm2', masks), p, t + '.conv2', stride=2, padding=1, drops=drops)
        nf = nf // 2
    h = h.reshape(h.shape[0], -1)
    h = _relu(F.linear(h, p['features.FC.weight'], p['features.FC.bias']), masks, 'features.FC')
    mean = F.linear(h, p['features.SplitDense.fc_mean.weight'], p['features.SplitDense.fc_mean.bias'])
    logsig = F.linear(h, p['features.SplitDense.fc_logvar.weight'], p['features.SplitDense.fc_logvar.bias'])
    return mean, logsig


def decoder_forward(p, z, latent_img_size, blocks, growth, init_features, masks=None, drops=None):
    """CNNDecoder.forward -> (mean, logsigma) [B, H, W]  (Decoder.py:288-305)."""
    h = F.linear(z, p['latent_map.weight'], p['latent_map.bias'])
    h = h.reshape(h.shape[0], -1, latent_img_size, latent_img_size)
    h = _conv(h, p, 'features.conv0', padding=1)
    nf = init_features
    for i, L in enumerate(blocks):
        h = _dense_block(h, p, 'features.DecBlock%d' % (i + 1), L, nf, growth, 4, False, masks, drops)
        nf += L * growth
        if i < len(blocks) - 1:
            t = 'features.TransUp%d' % (i + 1)
            h = _conv(_bn_relu(h, p, t + '.norm1', masks), p, t + '.conv1', drops=drops)
            h = _conv(_up(_bn_relu(h, p, t + '.norm2', masks)), p, t + '.conv2', padding=1, drops=drops)
            nf = nf // 2
    t = 'features.LastTransUp'
    h = _conv(_bn_relu(h, p, t + '.norm1', masks), p, t + '.conv1', padding=1, drops=drops)
    h = _conv(_up(_bn_relu(h, p, t + '.norm2', masks)), p, t + '.conv2', padding=1)
    h = _conv(_bn_relu(h, p, t + '.norm3', masks), p, t + '.conv3', padding=2)
    return h[:, 0], h[:, 1]
