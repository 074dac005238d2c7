"""lamp.modules -- BaseModule with the reference's helper API (lamp/modules.py:4-64)."""
import torch

from lamp.utils import get_default_device, get_default_dtype, get_device, get_dtype


class BaseModule(torch.nn.Module):
    """torch.nn.Module + state()/load()/_to() helpers used across the reference."""

    @property
    def num_parameters(self):
        return sum(p.numel() for p in self.parameters())

    @property
    def num_trainable_parameters(self):
        return sum(p.numel() for p in self.parameters() if p.requires_grad)

    def gradient_norm(self):
        norms = [p.grad.norm() for p in self.parameters() if p.grad is not None]
        return torch.stack(norms).mean()

    def freeze(self):
        for p in self.parameters():
            p.requires_grad = False

    def unfreeze(self):
        for p in self.parameters():
            p.requires_grad = True

    def state(self, *args, **kwargs):
        return self.state_dict(*args, **kwargs)

    def load(self, *args, **kwargs):
        self.load_state_dict(*args, **kwargs)

    def copy_values_from(self, module):
        res = self.load_state_dict(module.state_dict())
        if res.missing_keys or res.unexpected_keys:
            raise RuntimeError('state mismatch: %s' % (res,))

    def _to(self, **kwargs):
        dtype = kwargs.get('dtype')
        device = kwargs.get('device')
        dtype = get_dtype(dtype) if dtype is not None else get_default_dtype()
        device = get_device(device) if device is not None else get_default_device()
        self.to(dtype=dtype, device=device)
