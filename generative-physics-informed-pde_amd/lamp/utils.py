"""lamp.utils -- dtype / device helpers (lamp/utils.py) and R^2 (coefficient_of_determination)."""
import torch

_DEFAULT_DTYPE = torch.float32


def get_default_dtype():
    return _DEFAULT_DTYPE


def get_default_device():
    return torch.device('cuda:0') if torch.cuda.is_available() else torch.device('cpu')


def get_dtype(dtype):
    if isinstance(dtype, torch.dtype):
        return dtype
    s = str(dtype).lower()
    if s in ('float32', 'float', 'single'):
        return torch.float32
    if s in ('float64', 'double'):
        return torch.float64
    raise ValueError('unknown dtype %s' % dtype)


def get_device(device):
    if isinstance(device, torch.device):
        return device
    s = str(device).lower()
    if s in ('gpu', 'cuda', 'best'):
        return get_default_device()
    return torch.device(s)


def coefficient_of_determination(y_pred, y_true, global_average=False):
    """R^2 = 1 - SS_res / SS_tot, averaged over samples (lamp/utils.py:5-20)."""
    if global_average:
        mu = torch.mean(y_true)
        return 1 - torch.sum((y_pred - y_true) ** 2) / torch.sum((y_true - mu) ** 2)
    mu = torch.mean(y_true, 0, keepdim=True)
    return 1 - torch.sum((y_pred - y_true) ** 2) / torch.sum((y_true - mu) ** 2)
