"""CNNEncoder (reference bottleneck/Encoder.py:133-222) on the native codec.

Module tree and construction order follow the reference so that state_dict
keys and seeded initialisation match; ``forward`` runs the whole encoder as
one native conv program + the dense-head kernel (no per-layer autograd).
"""
import torch
import torch.nn as nn

import lamp.modules
from bottleneck.codec import _DenseBlock, _Transition, FlattenImage, SplitModule, module_size


class BaseEncoder(lamp.modules.BaseModule):

    @property
    def dim_in(self):
        raise NotImplementedError

    @property
    def dim_out(self):
        raise NotImplementedError


class CNNEncoder(BaseEncoder):
    """7x7/s2 conv -> [DenseBlock -> TransitionDown] x L -> flatten -> FC -> ReLU -> (mean, logsigma)."""

    def __init__(self, imsize, latent_dim, blocks=[3, 5, 3], growth_rate=8, init_features=32, drop_rate=0,
                 makedeterministic=False):
        super().__init__()
        if makedeterministic:
            raise NotImplementedError('the deterministic encoder head is not on the ELBO path')
        self._cfg = dict(imsize=int(imsize), blocks=list(blocks), growth=int(growth_rate),
                         init_features=int(init_features), bn_size=8, bottleneck=True, drop_rate=float(drop_rate))
        self.latent_dim = latent_dim
        self.features = nn.Sequential()
        pad = 3 if imsize % 2 == 0 else 2
        self.features.add_module('In_conv', nn.Conv2d(1, init_features, kernel_size=7, stride=2, padding=pad,
                                                      bias=False))
        nf = init_features
        for i, nl in enumerate(blocks):
            self.features.add_module('EncBlock%d' % (i + 1), _DenseBlock(nl, nf, growth_rate, drop_rate, bn_size=8,
                                                                         bottleneck=True))
            nf += nl * growth_rate
            self.features.add_module('TransDown%d' % (i + 1), _Transition(nf, nf // 2, down=True,
                                                                          drop_rate=drop_rate))
            nf //= 2
        side = int(imsize / (2 ** (len(blocks) + 1)))
        q = nf * side * side
        self._dim_feat = q
        self.features.add_module('FlattenImage', FlattenImage())
        self.features.add_module('FC', nn.Linear(q, q))
        self.features.add_module('ActivRelu', nn.ReLU())
        self.features.add_module('SplitDense', SplitModule(q, latent_dim))

    def native_config(self):
        return dict(self._cfg)

    @property
    def dim_in(self):
        return self._cfg['imsize'] ** 2

    @property
    def dim_out(self):
        return self.latent_dim

    @property
    def model_size(self):
        return module_size(self)

    def forward(self, x):
        from gpi.native import encoder_forward
        return encoder_forward(self, x)

    def reset_parameters(self, verbose=False):
        for m in self.modules():
            if m is not self and hasattr(m, 'reset_parameters'):
                m.reset_parameters()
