"""Flat parameter / gradient storage.

All parameters of a model live in ONE fp32 device buffer (each nn.Parameter's
``.data`` becomes a view of it), gradients land in ONE fp32 buffer (each
``.grad`` a view), and kernels accumulate gradients in a parallel fp64
buffer.  One flat buffer gives: single-offset parameter addressing in the
kernels, one all-reduce for data parallelism, one Adam launch.
The Parameter objects themselves are unchanged, so optimizers built on
``model.parameters()`` and ``state_dict()`` / ``load_state_dict()`` keep working.
"""
import torch

# Every matrix parameter (nn.Linear weights, per-sample variational rows) starts on a 16-byte boundary
# of the flat buffers, so the dense-layer kernels (head.hip) read weight rows as aligned float4; vectors
# and conv kernels stay packed (a BN layer's gamma and beta adjacent: one slab-reduction item).  The
# padding floats are zero in P, G and gacc and stay zero under Adam (zero gradient, zero moments).
ALIGN = 4


class FlatParameters(object):

    def __init__(self, named_params, device, shared_prefixes=None, err_slot=False):
        """err_slot: reserve one float at the end of the shared prefix (inside the data-parallel all-reduce,
        no parameter): FusedElboStep's hand-off error flag, summed over the ranks (gpi_step_epilogue_desc)."""
        named = [(n, p) for n, p in named_params]
        # shared parameters first, rank-local ones (per-sample variational params) last
        if shared_prefixes is not None:
            named.sort(key=lambda np_: 0 if any(np_[0].startswith(s) for s in shared_prefixes) else 1)
        self.names = [n for n, _ in named]
        self.params = [p for _, p in named]
        self.offsets = {}
        self.name_offsets = {}
        total = 0
        self.err_slot = -1
        for n, p in named:
            if err_slot and self.err_slot < 0 and shared_prefixes is not None and \
                    not any(n.startswith(s) for s in shared_prefixes):
                self.err_slot = total
                total += 1
            if p.dim() == 2:
                total = (total + ALIGN - 1) // ALIGN * ALIGN
            self.offsets[id(p)] = total
            self.name_offsets[n] = total
            total += p.numel()
        if err_slot and self.err_slot < 0:
            self.err_slot = total
            total += 1
        self.numel = total
        self.P = torch.zeros(total, dtype=torch.float32, device=device)
        self.G = torch.zeros(total, dtype=torch.float32, device=device)
        self.gacc = torch.zeros(total, dtype=torch.float64, device=device)
        for n, p in named:
            o = self.offsets[id(p)]
            self.P[o:o + p.numel()].copy_(p.detach().reshape(-1))
            p.data = self.P[o:o + p.numel()].view(p.shape)
        self.n_shared = total
        if shared_prefixes is not None:
            local = [n for n in self.names if not any(n.startswith(s) for s in shared_prefixes)]
            self.n_shared = self.name_offsets[local[0]] if local else total
            if self.err_slot >= 0:
                assert self.err_slot < self.n_shared

    def offset(self, p):
        return self.offsets[id(p)]

    def owns(self, p):
        return id(p) in self.offsets and p.data.data_ptr() == self.P.data_ptr() + 4 * self.offsets[id(p)]

    def grad_view(self, p):
        o = self.offsets[id(p)]
        return self.G[o:o + p.numel()].view(p.shape)

    def deliver(self, tmp):
        """Hand the flat gradient ``tmp`` to the parameters with torch
        accumulation semantics (None -> assign a view, existing -> add)."""
        grads = [p.grad for p in self.params]
        if all(g is None for g in grads):
            self.G.copy_(tmp)
            for p in self.params:
                p.grad = self.grad_view(p)
        elif all(g is not None and g.data_ptr() == self.G.data_ptr() + 4 * self.offsets[id(p)]
                 for g, p in zip(grads, self.params)):
            self.G.add_(tmp)
        else:
            for p in self.params:
                o = self.offsets[id(p)]
                v = tmp[o:o + p.numel()].view(p.shape)
                p.grad = v.clone() if p.grad is None else p.grad + v
