"""Model factories (reference factories/model.py:12-258): identifier -> physics + model.

``ModelFactory.FromIdentifier('highres32' | 'highres' | 'highres128')``,
``.set(key, value)``, ``.setup()`` -> (physics, model, discriminative_model,
encoder, dtype, device), with the reference's codec hyper-parameters.
"""
import torch

from physics.LinearElliptic import LinearEllipticPhysics
from bottleneck.Decoder import CNNDecoder
from bottleneck.Encoder import CNNEncoder
from bottleneck.components import EffectivePropertyMap, ReducedOrderModelOperator, PhysicsResolutionInterpolator
from bottleneck.generative import GenerativeModel


def fetch_dtype_device(dtype, device):
    s = dtype.lower()
    if s == 'float32':
        dt = torch.float32
    elif s in ('float64', 'double'):
        dt = torch.double
    else:
        raise ValueError('dtype option not recognized. options are: float32, float64 (double)')
    d = device.lower()
    if d == 'cpu':
        dev = torch.device('cpu')
    elif d in ('cuda', 'cuda:0', 'gpu'):
        dev = torch.device('cuda:0')
    elif d == 'best':
        dev = torch.device('cuda:0') if torch.cuda.is_available() else torch.device('cpu')
    else:
        raise ValueError('device option not recognized. options are: cpu, cuda, best')
    return dt, dev


class ModelFactory(object):

    CODEC = None   # dict(latent_img_size, latent_img_features, init_features_decoder, init_features_encoder, blocks, growth)

    def __init__(self, **kwargs):
        self.params = dict(independent_X=True, ptype=None, dim_latent=None, binary_field=False, dtype=None,
                           device=None, nx_rom=None, ny_rom=None, eff_property_map_hidden_layers=None,
                           num_refines=None, make_scalar_effective_property_map=False, droprate=0.0,
                           homoscedastic=False)
        self._identifier = None

    @classmethod
    def FromIdentifier(cls, identifier, *args, **kwargs):
        classes = {c.__name__: c for c in (highres, highres32, highres128, highres256)}
        return classes[identifier](*args, **kwargs)

    @property
    def identifier(self):
        return self._identifier or type(self).__name__

    @property
    def dtype(self):
        return fetch_dtype_device(self.params['dtype'], self.params['device'])[0]

    @property
    def device(self):
        return fetch_dtype_device(self.params['dtype'], self.params['device'])[1]

    def set(self, *args):
        if len(args) == 1 and isinstance(args[0], dict):
            items = args[0].items()
        elif len(args) == 2 and isinstance(args[0], str):
            items = [args]
        else:
            raise ValueError
        for k, v in items:
            if k not in self.params:
                raise KeyError(k)
            self.params[k] = v

    def _physics(self):
        p = self.params
        if p['nx_rom'] != p['ny_rom']:
            raise NotImplementedError('square ROM meshes only')
        r = 2 ** p['num_refines']
        physics = {'fom': LinearEllipticPhysics('fom', p['ptype'], p['nx_rom'] * r),
                   'rom': LinearEllipticPhysics('rom', p['ptype'], p['nx_rom'], refine_to_fom=r)}
        physics['W'] = physics['fom'].grid.prolongation_from(physics['rom'].grid)    # [d_y, n_c]
        return physics

    def setup(self):
        p = self.params
        dtype, device = fetch_dtype_device(p['dtype'], p['device'])
        physics = self._physics()
        c = self.CODEC
        n = p['nx_rom'] * 2 ** p['num_refines']
        decoder = CNNDecoder(n, p['dim_latent'], (c['latent'], c['latent']), c['latent_features'], c['f_dec'],
                             c['blocks'], p['binary_field'], c['growth'], drop_rate=p['droprate'],
                             upsample='nearest', force_single_output=False, homoscedastic=p['homoscedastic'])
        encoder = CNNEncoder(n, p['dim_latent'], c['blocks'], c['growth'], c['f_enc'], drop_rate=p['droprate'])
        encoder = encoder.to(dtype=dtype, device=device)
        f = decoder.to(dtype=dtype, device=device)
        g = ReducedOrderModelOperator.FromPhysics(physics, dtype=dtype, device=device)
        gp = EffectivePropertyMap(f.dim_latent, g.dim_effective_property,
                                  num_hidden_layers=p['eff_property_map_hidden_layers'],
                                  independent_X=p['independent_X'], dtype=dtype, device=device)
        model = GenerativeModel(f=f, g=g, gp=gp, dtype=dtype, device=device)
        disc = model.extract_discriminative_model(FromLatentEncoding=False, duplicate=True, encoder=encoder)
        return physics, model, disc, encoder, dtype, device

    @property
    def physics(self):
        return self._physics()


class highres(ModelFactory):
    """64 x 64 (factories/model.py:172-213), droprate 0.2 as the reference (:187): Dropout2d in train
    mode on the native codec.  The reference sets ptype 'ND', which is unreachable;
    'NDP' here."""
    CODEC = dict(latent=8, latent_features=1, f_dec=6, f_enc=6, blocks=[1, 2, 1], growth=4)

    def __init__(self, **kwargs):
        super().__init__()
        self.params.update(ptype='NDP', dim_latent=64, dtype='float32', device='best', nx_rom=8, ny_rom=8,
                           eff_property_map_hidden_layers=0, num_refines=3, droprate=0.2)
        self._identifier = 'highres'
        self.set(kwargs)


class highres32(ModelFactory):
    """32 x 32, the published notebook configuration (factories/model.py:215-257)."""
    CODEC = dict(latent=8, latent_features=1, f_dec=4, f_enc=4, blocks=[1, 1], growth=4)

    def __init__(self, **kwargs):
        super().__init__()
        self.params.update(ptype='NDP', dim_latent=16, dtype='float32', device='best', nx_rom=4, ny_rom=4,
                           eff_property_map_hidden_layers=0, num_refines=3, droprate=0.0)
        self._identifier = 'highres32'
        self.set(kwargs)


class highres128(ModelFactory):
    """128 x 128 scale-up (BASELINE config 4): deeper codec, ROM 8x8 with 4 refinements, droprate 0.2
    as the 64 x 64 factory it extends."""
    CODEC = dict(latent=8, latent_features=1, f_dec=6, f_enc=6, blocks=[1, 2, 2, 1], growth=4)

    def __init__(self, **kwargs):
        super().__init__()
        self.params.update(ptype='NDP', dim_latent=64, dtype='float32', device='best', nx_rom=8, ny_rom=8,
                           eff_property_map_hidden_layers=0, num_refines=4, droprate=0.2)
        self._identifier = 'highres128'
        self.set(kwargs)


class highres256(ModelFactory):
    """256 x 256 scale-up (BASELINE config 5): blocks [1, 2, 2, 2, 1], ROM 8x8 with 5 refinements,
    droprate 0.2."""
    CODEC = dict(latent=8, latent_features=1, f_dec=6, f_enc=6, blocks=[1, 2, 2, 2, 1], growth=4)

    def __init__(self, **kwargs):
        super().__init__()
        self.params.update(ptype='NDP', dim_latent=64, dtype='float32', device='best', nx_rom=8, ny_rom=8,
                           eff_property_map_hidden_layers=0, num_refines=5, droprate=0.2)
        self._identifier = 'highres256'
        self.set(kwargs)
