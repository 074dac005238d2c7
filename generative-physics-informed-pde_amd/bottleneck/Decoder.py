"""CNNDecoder (reference bottleneck/Decoder.py:163-325) on the native codec.

Linear latent map -> 1 x 8 x 8 image -> conv0 -> [DenseBlock -> TransitionUp]
-> last decoding -> 2 channels (mean, logsigma).  Module tree / order as in
the reference; ``forward`` runs the latent map and the whole conv stack as
native kernels.
"""
import torch
import torch.nn as nn

import lamp.modules
from bottleneck.codec import _DenseBlock, _Transition, last_decoding, UnflattenLatentDimension, module_size


class BaseDecoder(lamp.modules.BaseModule):

    @property
    def dim_in(self):
        raise NotImplementedError

    @property
    def dim_out(self):
        raise NotImplementedError

    def propagate_samples(self, Z):
        """Decoder.py:29-37: a sample of the decoder's Gaussian for each z."""
        means, logsigmas = self.forward(Z)
        if means.shape != logsigmas.shape:
            raise RuntimeError('Implementation assumes that full logsigmas matrix is given; check for broadcasting')
        return means + torch.exp(logsigmas) * torch.randn_like(logsigmas)


class CNNDecoder(BaseDecoder):

    def __init__(self, target_img_size, dim_latent, latent_img_size=(4, 4), latent_img_features=16,
                 init_features=32, blocks=[3, 5, 3], binary=False, growth_rate=8, drop_rate=0., upsample='nearest',
                 force_single_output=False, homoscedastic=False):
        super().__init__()
        if isinstance(target_img_size, tuple):
            assert all(e == target_img_size[0] for e in target_img_size)
            target_img_size = target_img_size[0]
        if isinstance(latent_img_size, tuple):
            assert all(e == latent_img_size[0] for e in latent_img_size)
            latent_img_size = latent_img_size[0]
        out_size = int(latent_img_size * 2 ** len(blocks))
        if out_size != target_img_size:
            raise ValueError('Latent image size {0}x{0} with {1} blocks yields a {2}x{2} output, target is {3}x{3}'
                             .format(latent_img_size, len(blocks), out_size, target_img_size))
        if binary or force_single_output or homoscedastic:
            raise NotImplementedError('the native decoder implements the heteroscedastic Gaussian head '
                                      '(binary / homoscedastic variants are not on the ELBO path)')
        if upsample != 'nearest':
            raise NotImplementedError('only nearest upsampling is supported')
        self._output_shape = (target_img_size, target_img_size)
        self._dim_in = dim_latent
        self._dim_out = target_img_size ** 2
        self._binary = False
        self._homoscedastic = False
        self._latent_img_dimension = latent_img_size ** 2 * latent_img_features
        self._cfg = dict(latent_img_size=latent_img_size, latent_img_features=latent_img_features,
                         init_features=init_features, blocks=list(blocks), growth=growth_rate, out_channels=2,
                         drop_rate=float(drop_rate))
        self.latent_map = nn.Linear(dim_latent, self._latent_img_dimension)
        self.features = nn.Sequential()
        self.features.add_module('unflatten_latent', UnflattenLatentDimension(latent_img_size))
        self.features.add_module('conv0', nn.Conv2d(latent_img_features, init_features, 3, 1, 1, bias=False))
        nf = init_features
        for i, nl in enumerate(blocks):
            self.features.add_module('DecBlock%d' % (i + 1), _DenseBlock(nl, nf, growth_rate, drop_rate))
            nf += nl * growth_rate
            if i < len(blocks) - 1:
                self.features.add_module('TransUp%d' % (i + 1), _Transition(nf, nf // 2, down=False,
                                                                            drop_rate=drop_rate,
                                                                            upsample=upsample))
                nf //= 2
        self.features.add_module('LastTransUp', last_decoding(nf, 2, drop_rate=drop_rate, upsample=upsample))

    def native_config(self):
        return dict(self._cfg)

    @property
    def dim_latent_img(self):
        return self._latent_img_dimension

    @property
    def dim_latent(self):
        return self._dim_in

    @property
    def dim_in(self):
        return self._dim_in

    @property
    def dim_out(self):
        return self._dim_out

    @property
    def model_size(self):
        return module_size(self)

    def forward(self, x, flatten=False):
        from gpi.native import decoder_forward
        out = decoder_forward(self, x)
        mean, logsigmas = out[:, 0], out[:, 1]
        if flatten:
            mean = mean.reshape(mean.shape[0], -1)
            logsigmas = logsigmas.reshape(logsigmas.shape[0], -1)
        return mean, logsigmas
