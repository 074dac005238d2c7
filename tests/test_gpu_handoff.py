"""A timed-out cross-stream hand-off fails loudly and never moves the parameters (VERDICT r04 item 5,
ADVICE r04): the fused step's side stream hands its last reductions to the epilogue + Adam launch by a
device counter with a bounded spin (gpi_stream_wait); on a timeout the error word is set, the update of
that step (and of every later one: the word is sticky) leaves parameters and Adam moments untouched, and
the host raises (check_handoff at once, step() / run() lazily from an async copy of the word)."""
import ctypes as C

import pytest
import torch

from test_gpu_parity import load, build_golden_model, cuda

pytestmark = pytest.mark.gpu


def test_adam_skips_update_while_wait_error_is_set(device):
    """gpi_adam (the DP form, after gpi_stream_wait on the main stream): error word set -> p, m, v unchanged
    (the RNG offset still advances); word clear -> the normal update."""
    from gpi import _lib as L
    torch.manual_seed(0)
    p = torch.randn(5000, device='cuda')
    g = torch.randn(5000, device='cuda')
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    lr = torch.tensor([1e-2], device='cuda')
    step = torch.ones(1, dtype=torch.int64, device='cuda')
    err = torch.ones(1, dtype=torch.int32, device='cuda')
    off = torch.zeros(1, dtype=torch.int64, device='cuda')
    p0 = p.clone()
    dsc = L.AdamDesc(p=p.data_ptr(), g=g.data_ptr(), m=m.data_ptr(), v=v.data_ptr(), n=p.numel(),
                     lr=lr.data_ptr(), step=step.data_ptr(), beta1=0.9, beta2=0.999, eps=1e-8,
                     rng_offset=off.data_ptr(), rng_advance=7, wait_err=err.data_ptr())
    L.check(L.lib().gpi_adam(C.byref(dsc), L.stream_handle()), 'adam')
    torch.cuda.synchronize()
    assert torch.equal(p, p0) and int(m.abs().max()) == 0 and int(v.abs().max()) == 0
    assert int(off.item()) == 7
    err.zero_()
    L.check(L.lib().gpi_adam(C.byref(dsc), L.stream_handle()), 'adam')
    torch.cuda.synchronize()
    assert not torch.equal(p, p0) and int(off.item()) == 14


def test_fused_step_wait_timeout_skips_update_and_raises(device):
    """One eager fused step whose side-stream flag can never reach its target (the word set 2^30 below it):
    the epilogue's wait times out (~10 s), the gradient is still delivered, but parameters, Adam moments
    and the Adam step's effect are absent; check_handoff() raises, and so does the next step() once the
    posted copy of the error word has landed."""
    from gpi.train import FusedElboStep
    d = load('elbo_c32.npz')
    model, bs = build_golden_model(d)
    Xu, Xs, Y, F = cuda(d['Xu']), cuda(d['Xs']), cuda(d['Y']), cuda(d['F'])
    st = FusedElboStep(model, Xu, bs, Xs, Y, F, lr=1e-3, seed=3)
    if st.handoff != 'flags' or not st.fuse_adam:
        pytest.skip('no flag hand-off into the fused epilogue in this configuration')
    st.step()                                    # one good step first: the machinery works
    torch.cuda.synchronize()
    st.check_handoff()
    P0, m0, v0 = st.flat.P.clone(), st.m.clone(), st.v.clone()
    st.handoff_flags[3] -= (1 << 30)             # flag 3 (side stream done) can no longer reach step + 1
    st.step()
    torch.cuda.synchronize()
    assert int(st.handoff_flags[4].item()) == 1
    assert torch.equal(st.flat.P, P0) and torch.equal(st.m, m0) and torch.equal(st.v, v0)
    assert float(st.flat.G.abs().max()) > 0      # the (possibly incomplete) gradient was still delivered
    with pytest.raises(RuntimeError, match='timed out'):
        st.check_handoff()
    st.run(0)                                    # posts the async copy of the error word
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match='timed out'):
        st.step()
