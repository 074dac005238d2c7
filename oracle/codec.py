"""torch.nn.functional restatement of the DenseNet conv codec (CPU reference).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Follows the reference's module structure and parameter names so that a
reference ``state_dict`` drives it directly:
  * CNNEncoder   bottleneck/Encoder.py:133-196
  * CNNDecoder   bottleneck/Decoder.py:163-305
  * blocks       bottleneck/codec.py:131-298, 484-504
BatchNorm is always in training mode (nothing in the reference calls
``.eval()``), eps 1e-5; Dropout2d is supported with an injected channel mask.
"""
import torch
import torch.nn.functional as F

BN_EPS = 1e-5


def _bn_relu(x, p, name):
    x = F.batch_norm(x, None, None, p[name + '.weight'], p[name + '.bias'],
                     training=True, momentum=0.0, eps=BN_EPS)
    return torch.relu(x)


def _conv(x, p, name, stride=1, padding=0):
    w = p[name + '.weight']
    b = p.get(name + '.bias')
    return F.conv2d(x, w, b, stride=stride, padding=padding)


def _up(x):
    return F.interpolate(x, scale_factor=2.0, mode='nearest')


def _dense_layer(x, p, name, in_features, growth, bn_size, bottleneck):
    """codec.py:150-182 (cat [x, y] on channels)."""
    if bottleneck and in_features > bn_size * growth:
        y = _conv(_bn_relu(x, p, name + '.norm1'), p, name + '.conv1')
        y = _conv(_bn_relu(y, p, name + '.norm2'), p, name + '.conv2', padding=1)
    else:
        y = _conv(_bn_relu(x, p, name + '.norm1'), p, name + '.conv1', padding=1)
    return torch.cat([x, y], 1)


def _dense_block(x, p, name, num_layers, in_features, growth, bn_size, bottleneck):
    for i in range(num_layers):
        x = _dense_layer(x, p, '%s.denselayer%d' % (name, i + 1), in_features + i * growth,
                         growth, bn_size, bottleneck)
    return x


def encoder_forward(p, x, imsize, blocks, growth, init_features):
    """CNNEncoder.forward -> (mean, logsigma)  (Encoder.py:147-196)."""
    if x.dim() < 4:
        x = x.unsqueeze(1)
    pad = 3 if imsize % 2 == 0 else 2
    h = _conv(x, p, 'features.In_conv', stride=2, padding=pad)
    nf = init_features
    for i, L in enumerate(blocks):
        h = _dense_block(h, p, 'features.EncBlock%d' % (i + 1), L, nf, growth, 8, True)
        nf = nf + L * growth
        t = 'features.TransDown%d' % (i + 1)
        h = _conv(_bn_relu(h, p, t + '.norm1'), p, t + '.conv1')
        h = _conv(_bn_relu(h, p, t + '.norm2'), p, t + '.conv2', stride=2, padding=1)
        nf = nf // 2
    h = h.reshape(h.shape[0], -1)
    h = torch.relu(F.linear(h, p['features.FC.weight'], p['features.FC.bias']))
    mean = F.linear(h, p['features.SplitDense.fc_mean.weight'], p['features.SplitDense.fc_mean.bias'])
    logsig = F.linear(h, p['features.SplitDense.fc_logvar.weight'], p['features.SplitDense.fc_logvar.bias'])
    return mean, logsig


def decoder_forward(p, z, latent_img_size, blocks, growth, init_features):
    """CNNDecoder.forward -> (mean, logsigma) [B, H, W]  (Decoder.py:288-305)."""
    h = F.linear(z, p['latent_map.weight'], p['latent_map.bias'])
    h = h.reshape(h.shape[0], -1, latent_img_size, latent_img_size)
    h = _conv(h, p, 'features.conv0', padding=1)
    nf = init_features
    for i, L in enumerate(blocks):
        h = _dense_block(h, p, 'features.DecBlock%d' % (i + 1), L, nf, growth, 4, False)
        nf += L * growth
        if i < len(blocks) - 1:
            t = 'features.TransUp%d' % (i + 1)
            h = _conv(_bn_relu(h, p, t + '.norm1'), p, t + '.conv1')
            h = _conv(_up(_bn_relu(h, p, t + '.norm2')), p, t + '.conv2', padding=1)
            nf = nf // 2
    t = 'features.LastTransUp'
    h = _conv(_bn_relu(h, p, t + '.norm1'), p, t + '.conv1', padding=1)
    h = _conv(_up(_bn_relu(h, p, t + '.norm2')), p, t + '.conv2', padding=1)
    h = _conv(_bn_relu(h, p, t + '.norm3'), p, t + '.conv3', padding=2)
    return h[:, 0], h[:, 1]
