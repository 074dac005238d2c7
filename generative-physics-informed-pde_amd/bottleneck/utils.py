"""Gaussian helpers (reference bottleneck/utils.py:216-248).

Tensor-level utilities kept with the reference's names and signatures for
callers outside the fused step (e.g. monitoring); the training step computes
the same quantities inside the native kernels (head.hip, conv.hip, rom.hip).
"""
import torch

LOG2PI = 1.8378770664093453


def reparametrize(mean, logsigma):
    return mean + torch.exp(logsigma) * torch.randn_like(logsigma)


def DiagonalGaussianLogLikelihood(target, mean, logvars, target_logvars=None, reduce=torch.sum):
    if target_logvars is not None:
        raise DeprecationWarning
    L = -0.5 * (logvars + (target - mean) ** 2 * torch.exp(-logvars) + LOG2PI)
    return reduce(L) if reduce is not None else L


def UnitGaussianKullbackLeiblerDivergence(mean, logvars):
    return -0.5 * torch.sum(1 + logvars - mean.pow(2) - logvars.exp())


def relative_error(y, y_true):
    return (torch.norm(y - y_true) / torch.norm(y_true)).item()


def relative_error_batched(Y_mean, Y_true):
    return torch.mean(torch.norm(Y_mean - Y_true, dim=1) / torch.norm(Y_true, dim=1)).item()
