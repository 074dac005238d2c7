"""A timed-out cross-stream hand-off fails loudly and never moves the parameters (VERDICT r04 item 5,
ADVICE r04): the fused step's side stream hands its last reductions to the epilogue + Adam launch by a
device counter with a bounded spin (gpi_stream_wait); on a timeout the error word is set, the update of
that step (and of every later one: the word is sticky) leaves parameters and Adam moments untouched, and
the host raises (check_handoff at once, step() / run() lazily from an async copy of the word)."""
import ctypes as C

import numpy as np
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


def _c256_step(seed):
    """FusedElboStep at BASELINE config 5's per-GPU shape (256^2, B_u = 128 of 256, N_s = 32, droprate 0.2):
    the largest flat vector the fused epilogue + Adam launch covers."""
    from factories.model import ModelFactory
    from gpi.train import FusedElboStep
    from test_gpu_c64 import _DS
    n, Nu, bs, Ns = 256, 256, 128, 32
    torch.manual_seed(seed)
    fac = ModelFactory.FromIdentifier('highres256')
    fac.set('device', 'cuda')
    physics_, model, _, encoder, _, _ = fac.setup()
    model.encoder = encoder.cuda()
    nc = physics_['rom'].grid.n
    rng = np.random.default_rng(n)
    Xu = torch.tensor(rng.normal(0.3, 0.6, (Nu, n, n)), dtype=torch.float32, device='cuda')
    Xs = torch.tensor(rng.normal(0.3, 0.6, (Ns, n, n)), dtype=torch.float32, device='cuda')
    Y = torch.tensor(rng.normal(0.0, 0.3, (Ns, (n + 1) * (n - 1))), dtype=torch.float32, device='cuda')
    F = np.zeros((Ns, (nc + 1) ** 2), dtype=np.float32)
    F[:, [e for e in range((nc + 1) ** 2) if e % (nc + 1) in (0, nc)]] = rng.uniform(-0.5, 0.5, (Ns, 2 * (nc + 1)))
    F = torch.tensor(F, device='cuda')
    model.register_datasets({'supervised': _DS(X=Xs, Y=Y, F_ROM_BC=F),
                             'unsupervised': _DS(perm=torch.arange(Nu, device='cuda'), X=Xu)}, None,
                            create_unsupervised_variational_approximation=False)
    model.cuda()
    return FusedElboStep(model, Xu, bs, Xs, Y, F, lr=1e-3, seed=5)


def test_fused_epilogue_progresses_with_a_delayed_side_stream(device):
    """the fused epilogue + Adam launch spins on the side stream's flag in every
    workgroup, so it must never hold enough workgroups to keep the side stream's kernels off the CUs.  At
    config 5's per-GPU shape (the largest flat vector) the side stream is held back ~0.1 s by a sleep
    kernel ahead of its work, so the main stream reaches the epilogue first and spins there: the step still
    completes without a wait timeout, and its parameters match an undelayed step's (atomic-order rounding
    of the BN statistics aside: 1e-6 of the largest parameter)."""
    a = _c256_step(11)
    if a.handoff != 'flags' or not a.fuse_adam:
        pytest.skip('no flag hand-off into the fused epilogue in this configuration')
    a.step()
    torch.cuda.synchronize()
    a.check_handoff()
    b = _c256_step(11)
    side = b.engine._side_stream()
    with torch.cuda.stream(side):
        torch.cuda._sleep(int(2.5e8))           # ~0.1 s at the shader clock
    import time
    t0 = time.perf_counter()
    b.step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    e = b.epi
    m = max(e.n, e.n_scratch, e.n_idx, (e.drop_n + 3) // 4)
    print('epilogue items %d (%d workgroups uncapped), delayed step %.3f s' % (m, (m + 255) // 256, dt))
    b.check_handoff()                           # raises on a wait timeout
    scale = float(a.flat.P.abs().max())
    assert float((a.flat.P - b.flat.P).abs().max()) <= 1e-6 * scale


def _separate_side_stream():
    """A stream on another hardware queue than the current one (as FusedElboStep._queues_separate)."""
    from gpi import _lib as L
    pr = torch.zeros(2, dtype=torch.int32, device='cuda')
    ctr = torch.zeros(1, dtype=torch.int64, device='cuda')
    for _ in range(4):
        side = torch.cuda.Stream()
        pr.zero_()
        torch.cuda.synchronize()
        L.check(L.lib().gpi_queue_probe(L.ptr(pr), L.ptr(pr[1:]), C.c_void_p(side.cuda_stream)), 'queue probe')
        L.check(L.lib().gpi_stream_signal(L.ptr(pr), L.ptr(ctr), L.stream_handle()), 'queue probe signal')
        torch.cuda.synchronize()
        if int(pr[1].item()) == 1:
            return side
    pytest.skip('no stream on a separate hardware queue')


def test_epilogue_grid_leaves_room_for_the_signalling_stream(device):
    """ADVICE r04 (high), at the ABI: gpi_step_epilogue_adam over 2^23 elements (32 768 workgroups if one
    element per thread -- far more than the chip holds) whose every workgroup spins on a flag that another
    stream signals only after a ~20 ms sleep kernel.  The grid-stride launch of <= GPI_EPILOGUE_MAX_WG
    workgroups leaves CU slots for the signal kernel: no wait timeout, the update done, the accumulator
    delivered and zeroed.  (A one-element-per-thread grid fills every slot with spinning workgroups: the
    signal cannot run until they time out, and the error word is set -- checked with the cap lifted.)"""
    from gpi import _lib as L
    n = 1 << 23
    torch.manual_seed(1)
    gacc = torch.randn(n, dtype=torch.float64, device='cuda')
    g0 = gacc.float()
    grad = torch.empty(n, device='cuda')
    p = torch.randn(n, device='cuda')
    p0 = p.clone()
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    lr = torch.tensor([1e-3], device='cuda')
    step = torch.zeros(1, dtype=torch.int64, device='cuda')
    flag, err, done = (torch.zeros(1, dtype=torch.int32, device='cuda') for _ in range(3))
    side = _separate_side_stream()
    d = L.StepEpilogueDesc(gacc=gacc.data_ptr(), grad=grad.data_ptr(), n=n, flags=2, wait_flag=flag.data_ptr(),
                           wait_err=err.data_ptr())
    a = L.AdamDesc(p=p.data_ptr(), g=grad.data_ptr(), m=m.data_ptr(), v=v.data_ptr(), n=n, lr=lr.data_ptr(),
                   step=step.data_ptr(), beta1=0.9, beta2=0.999, eps=1e-8, wait_err=err.data_ptr())
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        torch.cuda._sleep(int(5e7))
    L.check(L.lib().gpi_step_epilogue_adam(C.byref(d), C.byref(a), L.ptr(done), L.stream_handle()), 'epilogue')
    L.check(L.lib().gpi_stream_signal(L.ptr(flag), L.ptr(step), C.c_void_p(side.cuda_stream)), 'signal')
    torch.cuda.synchronize()
    assert int(err.item()) == 0, 'the epilogue wait timed out: its workgroups kept the signal off the CUs'
    assert int(step.item()) == 1 and int(done.item()) == 0
    assert torch.equal(grad, g0) and int(gacc.abs().max().item() == 0) == 1
    assert not torch.equal(p, p0)
