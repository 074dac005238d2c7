"""Restatement of the reference's ELBO algebra (torch CPU, any dtype).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Every function cites the reference lines it follows.  Random draws are
always *injected* (eps tensors) so results are comparable across
implementations whose RNG streams differ.
"""
import math
import numpy as np
import torch

LOG2PI = 1.8378770664093453


def dgll(target, mean, logvars):
    """DiagonalGaussianLogLikelihood, reduce=sum (bottleneck/utils.py:231-243)."""
    sigma = torch.exp(0.5 * logvars)
    return torch.sum(-0.5 * (logvars + ((target - mean) / sigma) ** 2 + LOG2PI))


def field_loglik(X, mx, lsx, log_field=True):
    """GenerativeModel.random_field_likelihood (generative.py:232-239): Gaussian on the log-property
    (reconstruct_log_eff_property=True, the default) or on the exponentiated field."""
    if log_field:
        return dgll(X, mx, 2 * lsx)
    return dgll(torch.exp(X), torch.exp(mx), 2 * lsx)


def kl_unit(mean, logvars):
    """UnitGaussianKullbackLeiblerDivergence (bottleneck/utils.py:246-248)."""
    return -0.5 * torch.sum(1 + logvars - mean.pow(2) - logvars.exp())


def reparam(mean, logsigma, eps):
    """reparametrize with injected eps (bottleneck/utils.py:216-219)."""
    return mean + torch.exp(logsigma) * eps


def entropy(logsigma):
    """VariationalApproximation.entropy (components.py:195-197); the constant
    uses N (rows), not N*dim -- reference quirk kept."""
    N = logsigma.shape[0]
    return torch.sum(logsigma) + N * 0.5 * (np.log(2 * np.pi) + 1)


def rom_solve(M, kappa, F, bc_dofs):
    """ROM.__call__ (bottleneck/ROM.py:65-100): K = M x^T, Dirichlet rows
    zeroed with 1 on the diagonal (columns kept), batched solve.
    torch.solve (removed in torch>=2) -> torch.linalg.solve (same math)."""
    if (kappa <= 1e-12).any():
        raise ValueError('kappa <= 1e-12')
    K = torch.matmul(M, kappa.t())                     # [n, n, N]
    K[bc_dofs] = 0
    K[bc_dofs, bc_dofs] = 1
    return torch.linalg.solve(K.permute(2, 0, 1), F.unsqueeze(2)).squeeze(2)


def rom_operator(W, M, bc_dofs, effprop, F, logsigmas_y):
    """ReducedOrderModelOperator.forward (components.py:296-298)."""
    yc = rom_solve(M, torch.exp(effprop) + 1e-8, F, bc_dofs)
    mu = torch.einsum('sk,nk->ns', W, yc)
    return mu, logsigmas_y.repeat(effprop.shape[0], 1)


def elbo_unsupervised_armortized(encoder, decoder, X, eps, log_field=True):
    """generative.py:546-585 (normalize=False)."""
    mean, logsigma = encoder(X)
    Z = reparam(mean, logsigma, eps)
    mx, lsx = decoder(Z)
    logL_x = field_loglik(X, mx, lsx, log_field)
    DKL = kl_unit(mean, 2 * logsigma)
    return logL_x - DKL, dict(logL_x=logL_x, DKL=DKL)


def elbo_supervised_freeX(decoder, gp_linear, logsigmas_X_gp, rom, qz, qX, X, Y, F, eps_z, eps_X, log_field=True):
    """generative.py:461-500 with independent_X=True.

    qz / qX : (mean, logsigma) parameter pairs [N, d]
    gp_linear(Z) -> mu_X; logsigmas_X_gp the EffectivePropertyMap's logsigmas_X
    rom(X_sample, F) -> (mu_y, logsigma_y)
    """
    Z = reparam(qz[0], qz[1], eps_z)
    Xs = reparam(qX[0], qX[1], eps_X)
    mx, lsx = decoder(Z)
    logL_x = field_loglik(X, mx, lsx, log_field)
    mu_X = gp_linear(Z)
    logL_X = dgll(Xs, mu_X, 2 * logsigmas_X_gp.expand(Z.shape[0], -1))
    mu_y, ls_y = rom(Xs, F)
    logL_y = dgll(Y, mu_y, 2 * ls_y)
    DKL = kl_unit(qz[0], 2 * qz[1])
    ent = entropy(qX[1])
    terms = dict(logL_x=logL_x, logL_X=logL_X, logL_y=logL_y, DKL=DKL, entropy=ent)
    return logL_x + logL_y + logL_X + ent - DKL, terms



def elbo_supervised_lockX(decoder, gp_linear, rom, qz, X, Y, F, eps_z):
    """generative.py:429-459 with independent_X=False: X~ = gp(z) (EffectivePropertyMap.forward
    components.py:224-229 returns fc(z) only), no q_X, no logL_X / entropy.  The VO term
    _elbo_virtual_observables_lockX (generative.py:300-339) is the same algebra with Y drawn
    from the VO posterior."""
    Z = reparam(qz[0], qz[1], eps_z)
    mx, lsx = decoder(Z)
    logL_x = dgll(X, mx, 2 * lsx)
    mu_y, ls_y = rom(gp_linear(Z), F)
    logL_y = dgll(Y, mu_y, 2 * ls_y)
    DKL = kl_unit(qz[0], 2 * qz[1])
    return logL_x + logL_y - DKL, dict(logL_x=logL_x, logL_y=logL_y, DKL=DKL)

# --------------------------------------------------------------------------
# virtual observables (VirtualObservables.py:642-669, 960-998)
# --------------------------------------------------------------------------
def vo_condition(Gamma, alpha, g, prec, vo_variances):
    """VirtualObservable.update: condition N(g, diag(1/prec)) on
    Gamma y = alpha + N(0, diag(vo_variances)).  Gamma [m, d]; fp64."""
    g = g.double()
    prec = prec.double()
    cov = 1 / prec
    Lam = torch.einsum('im,m,sm->is', Gamma, cov, Gamma) + torch.diag(vo_variances)
    L = torch.linalg.cholesky(Lam)
    LamInv = torch.cholesky_inverse(L)
    solvec = LamInv @ (Gamma @ g - alpha)
    mean = g - torch.einsum('i,mi,m->i', cov, Gamma, solvec)
    A = Gamma * cov
    sub = torch.einsum('si,sm,mi->i', A, LamInv, A)
    return mean, cov - sub


def vo_precision_beta(Gammas, alphas, means, vars_, beta0=1e-6):
    """update_vo_precision: prec_beta = 0.5 sum_n [(G mu - a)^2 + G^2 var] + beta0."""
    beta = 0
    for G, a, mu, v in zip(Gammas, alphas, means, vars_):
        beta = beta + (G @ mu - a) ** 2 + (G ** 2) @ v
    return 0.5 * beta + beta0


def vo_mean_variances(prec_beta, N, infinite_mask, alpha0=1e-6):
    """_get_mean_vo_variances (VirtualObservables.py:960-964)."""
    prec_alpha = 0.5 * N + alpha0
    v = prec_beta / (prec_alpha + 1)
    v = v.clone()
    v[infinite_mask] = 0
    return v


def vo_predictive(W, M, bc_dofs, qx_mean, qx_logsigma, F, logsigmas_y, eps_X, eps_y, gp_linear=None):
    """update_virtual_observables' MC predictive (generative.py:191-207): per VO sample n,
    X_s = q_X mean + exp(logsigma) eps_X (components.py:174-180), y_s = rom mean(X_s) +
    exp(logsigmas_y) eps_y (components.py:304-311); returns torch.mean / torch.std (unbiased).
    eps_X [N, N_mc, dx], eps_y [N, N_mc, d_y].  lockX (generative.py:202-204): pass q_z's
    mean / logsigma, eps_Z and gp_linear; X_s = gp(z_s) (components.py:238-249)."""
    means, stds = [], []
    for n in range(qx_mean.shape[0]):
        X = qx_mean[n] + torch.exp(qx_logsigma[n]) * eps_X[n]
        if gp_linear is not None:
            X = gp_linear(X)
        mu, ls = rom_operator(W, M, bc_dofs, X, F[n].expand(X.shape[0], -1), logsigmas_y)
        y = mu + torch.exp(ls) * eps_y[n]
        means.append(torch.mean(y, 0))
        stds.append(torch.std(y, 0))
    return torch.stack(means), torch.stack(stds)
