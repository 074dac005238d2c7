"""DenseNet codec building blocks (reference bottleneck/codec.py:131-298, 484-504).

These modules are parameter containers with the reference's exact module
names and construction order, so that ``state_dict`` keys
(e.g. ``features.EncBlock1.denselayer1.conv1.weight``) and seeded default
initialisation are interchangeable with the reference.  They are never
executed layer by layer: CNNEncoder / CNNDecoder compile the whole tree into
one native conv program (gpi/plan.py) run by libgpi_hip.so.
"""
import torch
import torch.nn as nn


class _NativeOnly(object):
    def forward(self, *args, **kwargs):
        raise NotImplementedError('%s is executed by the native codec program (CNNEncoder / CNNDecoder)'
                                  % type(self).__name__)


class FlattenImage(nn.Module):
    def forward(self, x):
        return x.view(x.shape[0], -1)


class UnflattenLatentDimension(nn.Module):
    def __init__(self, hidden_img_size):
        super().__init__()
        self._hidden_img_size = hidden_img_size

    def forward(self, x):
        return x.view(x.size(0), -1, self._hidden_img_size, self._hidden_img_size)


class UpsamplingNearest2d(nn.Module):
    def __init__(self, scale_factor=2.):
        super().__init__()
        self.scale_factor = scale_factor

    def forward(self, x):
        return torch.nn.functional.interpolate(x, scale_factor=self.scale_factor, mode='nearest')


class SplitModule(nn.Module):
    """Two linear heads (mean, log-sigma) on the same features (codec.py:495-504)."""

    def __init__(self, dim_in, dim_out):
        super().__init__()
        self.fc_mean = nn.Linear(dim_in, dim_out)
        self.fc_logvar = nn.Linear(dim_in, dim_out)

    def forward(self, x):
        return self.fc_mean(x), self.fc_logvar(x)


def _bn_relu_conv(seq, idx, cin, cout, k, stride, pad, drop_rate, bias=False, upsample=False, relu_name=None):
    seq.add_module('norm%d' % idx, nn.BatchNorm2d(cin))
    seq.add_module(relu_name or 'relu%d' % idx, nn.ReLU(inplace=True))
    if upsample:
        seq.add_module('upsample', UpsamplingNearest2d(scale_factor=2))
    seq.add_module('conv%d' % idx, nn.Conv2d(cin, cout, kernel_size=k, stride=stride, padding=pad, bias=bias))
    if drop_rate > 0:
        seq.add_module('dropout' if relu_name == 'single' else 'dropout%d' % idx, nn.Dropout2d(p=drop_rate))


class _DenseLayer(_NativeOnly, nn.Sequential):
    """BN -> ReLU -> conv3x3 (or the 1x1 bottleneck pair), output concatenated to the input."""

    def __init__(self, in_features, growth_rate, drop_rate=0., bn_size=8, bottleneck=False):
        super().__init__()
        if bottleneck and in_features > bn_size * growth_rate:
            _bn_relu_conv(self, 1, in_features, bn_size * growth_rate, 1, 1, 0, 0)
            _bn_relu_conv(self, 2, bn_size * growth_rate, growth_rate, 3, 1, 1, 0)
        else:
            _bn_relu_conv(self, 1, in_features, growth_rate, 3, 1, 1, 0)
        if drop_rate > 0:
            self.add_module('dropout', nn.Dropout2d(p=drop_rate))


class _DenseBlock(_NativeOnly, nn.Sequential):
    def __init__(self, num_layers, in_features, growth_rate, drop_rate, bn_size=4, bottleneck=False):
        super().__init__()
        for i in range(num_layers):
            self.add_module('denselayer%d' % (i + 1),
                            _DenseLayer(in_features + i * growth_rate, growth_rate, drop_rate=drop_rate,
                                        bn_size=bn_size, bottleneck=bottleneck))


class _Transition(_NativeOnly, nn.Sequential):
    """Bottleneck transition: BN-ReLU-1x1 (C -> C/2), BN-ReLU-[up]-3x3 (/2 stride when down)."""

    def __init__(self, in_features, out_features, down, bottleneck=True, drop_rate=0, upsample='nearest'):
        super().__init__()
        if not bottleneck:
            raise NotImplementedError('only the bottleneck transition of the reference codec is supported')
        if not down and upsample != 'nearest':
            raise NotImplementedError('only nearest upsampling is supported')
        _bn_relu_conv(self, 1, in_features, out_features, 1, 1, 0, drop_rate)
        _bn_relu_conv(self, 2, out_features, out_features, 3, 2 if down else 1, 1, drop_rate, upsample=not down)


def last_decoding(in_features, out_channels, bias=False, drop_rate=0., upsample='nearest'):
    """BN-ReLU-3x3 (C->C/2), BN-ReLU-up-3x3 (C/2->C/4), BN-ReLU-5x5 (C/4->out)."""
    seq = nn.Sequential()
    seq.add_module('norm1', nn.BatchNorm2d(in_features))
    seq.add_module('relu1', nn.ReLU(True))
    seq.add_module('conv1', nn.Conv2d(in_features, in_features // 2, 3, 1, 1, bias=False))
    if drop_rate > 0.:
        seq.add_module('dropout1', nn.Dropout2d(p=drop_rate))
    seq.add_module('norm2', nn.BatchNorm2d(in_features // 2))
    seq.add_module('relu2', nn.ReLU(True))
    seq.add_module('upsample', UpsamplingNearest2d(scale_factor=2))
    seq.add_module('conv2', nn.Conv2d(in_features // 2, in_features // 4, 3, 1, 1, bias=bias))
    seq.add_module('norm3', nn.BatchNorm2d(in_features // 4))
    seq.add_module('relu3', nn.ReLU(True))
    seq.add_module('conv3', nn.Conv2d(in_features // 4, out_channels, 5, 1, 2, bias=bias))
    if bias:
        raise NotImplementedError('biased last decoding is not used by the reference codec')
    return seq


def module_size(module):
    n_params = sum(p.numel() for p in module.parameters())
    n_conv = sum(1 for n, _ in module.named_parameters() if 'conv' in n)
    return n_params, n_conv
