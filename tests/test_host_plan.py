"""CPU tests of the host side: module trees vs the reference's state_dict,
planner wiring (interpreted on CPU against the oracle codec), layouts."""
import os

import numpy as np
import pytest
import torch

from oracle import codec as ocodec
from bottleneck.Encoder import CNNEncoder
from bottleneck.Decoder import CNNDecoder
from gpi.plan import encoder_program, decoder_program, Arena
from program_interp import run_program

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


def gold(tag):
    return dict(np.load(os.path.join(GOLD, 'codec_%s.npz' % tag), allow_pickle=False))


def build(tag):
    d = gold(tag)
    imsize, dz, latent, growth, f_enc, f_dec = [int(v) for v in d['cfg'][:6]]
    blocks = [int(v) for v in d['cfg'][6:]]
    torch.manual_seed(0)
    enc = CNNEncoder(imsize, dz, blocks, growth, f_enc, drop_rate=0)
    dec = CNNDecoder(imsize, dz, (latent, latent), 1, f_dec, blocks, False, growth, drop_rate=0.)
    return d, enc, dec, imsize, dz, latent, growth, f_enc, f_dec, blocks


@pytest.mark.parametrize('tag', ['c32', 'c64'])
def test_state_dict_keys_and_seeded_init_match_reference(tag):
    d, enc, dec = build(tag)[:3]
    for prefix, mod in (('enc.', enc), ('dec.', dec)):
        ref_keys = sorted(k[len(prefix):] for k in d if k.startswith(prefix) and not k.startswith(prefix + 'grad.'))
        assert sorted(mod.state_dict().keys()) == ref_keys
        for k, v in mod.state_dict().items():
            if 'conv' in k or 'FC' in k or 'fc_' in k or 'latent_map' in k or 'In_conv' in k:
                np.testing.assert_array_equal(v.numpy(), d[prefix + k], err_msg=k)


@pytest.mark.parametrize('tag', ['c32', 'c64'])
def test_planned_program_matches_oracle(tag):
    d, enc, dec, imsize, dz, latent, growth, f_enc, f_dec, blocks = build(tag)
    pe = {k[4:]: torch.tensor(v, dtype=torch.float64) for k, v in d.items() if k.startswith('enc.') and
          not k.startswith('enc.grad.')}
    pd = {k[4:]: torch.tensor(v, dtype=torch.float64) for k, v in d.items() if k.startswith('dec.') and
          not k.startswith('dec.grad.')}
    X = torch.tensor(d['X'], dtype=torch.float64).unsqueeze(1)
    prog = encoder_program(**enc.native_config())
    feat = run_program(prog, pe, X).reshape(X.shape[0], -1)
    h = torch.relu(torch.nn.functional.linear(feat, pe['features.FC.weight'], pe['features.FC.bias']))
    mu = torch.nn.functional.linear(h, pe['features.SplitDense.fc_mean.weight'], pe['features.SplitDense.fc_mean.bias'])
    np.testing.assert_allclose(mu.numpy(), d['enc_mu'], rtol=1e-4, atol=1e-5)
    assert prog.d_feat == feat.shape[1]

    Z = torch.tensor(d['Z'], dtype=torch.float64)
    lat = torch.nn.functional.linear(Z, pd['latent_map.weight'], pd['latent_map.bias']).reshape(Z.shape[0], 1,
                                                                                                latent, latent)
    prog = decoder_program(**dec.native_config())
    out = run_program(prog, pd, lat)
    np.testing.assert_allclose(out[:, 0].numpy(), d['dec_mu'], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out[:, 1].numpy(), d['dec_ls'], rtol=1e-4, atol=1e-5)
    # the oracle agrees with the same parameters
    mo, lo = ocodec.decoder_forward(pd, Z, latent, blocks, growth, f_dec)
    np.testing.assert_allclose(out[:, 0].numpy(), mo.numpy(), atol=1e-10)


def test_program_shapes_c64():
    enc = CNNEncoder(64, 64, [1, 2, 1], 4, 6)
    p = encoder_program(**enc.native_config())
    assert len(p.ops) == 11 and p.d_feat == 80
    dec = CNNDecoder(64, 64, (8, 8), 1, 6, [1, 2, 1], False, 4)
    q = decoder_program(**dec.native_config())
    assert len(q.ops) == 12
    assert (q.output.C, q.output.H) == (2, 64)
