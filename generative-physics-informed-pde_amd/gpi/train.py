"""Fused native training step: Trainer.run's loop body (training.py:403-417)
without Python/autograd glue, for production runs and the benchmark.

One step = random armortized subset (utils/data.py:444) + reparametrisation
noise (device Philox) + ELBO forward/backward (ElboEngine) + gradient
finalisation + [one SUM all-reduce of the shared-parameter gradients over
RCCL] + flat Adam (training.py:254,417).  Per-sample variational parameters
(q_z / q_X rows of this rank's labeled samples) are rank-local and never
communicated.  Every launch is stream-ordered with no host synchronisation,
so the whole step can be captured once into a HIP graph and replayed.
"""
import ctypes as C
import os

import torch
import torch.distributed as dist

from . import _lib as L
from .engine import ElboEngine


def allreduce_shared(flat, group=None):
    """Data-parallel gradient exchange: ONE SUM all-reduce
    (the ELBO is a sum over samples, normalize=False) of the shared-parameter
    prefix G[:n_shared] of the flat gradient; the per-sample variational rows
    that follow it are rank-owned and never communicated."""
    n = flat.n_shared
    if n > 0:
        dist.all_reduce(flat.G[:n], op=dist.ReduceOp.SUM, group=group)


class FusedAdamSchedule(torch.optim.Optimizer):
    """The learning-rate handle of a FusedElboStep as a torch Optimizer, so that torch LR schedulers
    (and lamp.optimization.LearningScheduleWrapper, lamp/optimization.py:71-93, training.py:452,615)
    drive the fused step's device-resident Adam exactly as they drive torch.optim.Adam: the
    scheduler edits ``param_groups[0]['lr']``; FusedElboStep copies a changed value into the
    device learning rate before its next step (an async fill, no host synchronisation)."""

    def __init__(self, lr, betas, eps):
        super().__init__([torch.zeros(1)], dict(lr=lr, betas=betas, eps=eps))

    def step(self, closure=None):     # the update itself runs inside the fused step
        return None


class FusedElboStep(object):
    """rank / world: data-parallel position.  Every rank holds the same global unlabeled pool and
    draws the same global permutation (``subset_seed``, shared) of which it takes its B_u-slice
    (SURVEY.md section 8e); labeled samples and their q rows are rank-owned; the
    reparametrisation noise uses ``seed`` (per rank)."""

    def __init__(self, model, X_pool, B_u, X_s=None, Y=None, F=None, lr=1e-2, betas=(0.9, 0.999), eps=1e-8,
                 seed=0, normalize=False, process_group=None, distributed=False, rank=0, world=1, subset_seed=None,
                 graph_allreduce=True, sync_bn=False, bn_exchange='collective'):
        self.model = model
        self.flat = model.native_flat()
        self.N_s = 0 if X_s is None else int(X_s.shape[0])
        self.B_u = int(B_u)
        self.rank, self.world = int(rank), int(world)
        assert 0 <= self.rank < self.world
        if subset_seed is None and self.world > 1 and self.B_u > 0:
            # every rank must draw the SAME global permutation (its B_u-slice of it); the per-rank
            # noise seed would give overlapping / duplicated slices without any error
            raise ValueError('FusedElboStep: world > 1 needs an explicit subset_seed shared by all ranks')
        self.engine = ElboEngine(model, self.B_u, self.N_s, normalize=normalize)
        # SyncBN: every codec call's BN statistics over the union of the ranks' batches (ElboEngine.set_sync_bn);
        # default replica-BN (per-rank batch statistics, no collective in the codec).  Any distributed world
        # size, 1 included: a one-rank NCCL job runs (and captures) the same per-conv collectives as the
        # 8-GPU one (tools/dist_capture_probe.py --sync-bn)
        # bn_exchange: 'collective' (each seam's message all-reduced over the process group: RCCL in the graph)
        # or 'peer' (the one-shot exchange through the ranks' IPC-mapped buffers, gpi.peer: one launch per
        # seam, any backend, capturable)
        self.sync_bn = bool(sync_bn) and bool(distributed)
        self.bn_exchange = bn_exchange if self.sync_bn else None
        self.handoff_flags = torch.zeros(8, dtype=torch.int32, device=self.flat.P.device)   # [0..3] flags, [4] error
        self._peer = None
        if self.sync_bn:
            pg = process_group
            if bn_exchange not in ('collective', 'peer'):
                raise ValueError("bn_exchange: 'collective' or 'peer'")
            if bn_exchange == 'peer':
                from .peer import PeerExchange
                self._peer = PeerExchange(pg, err=self.handoff_flags[4:5])
            self.engine.set_sync_bn(lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM, group=pg), self.world,
                                    exchange=self._peer)
        dev = self.flat.P.device
        self.X_pool = X_pool.contiguous().float() if X_pool is not None else None
        self.X_s, self.Y, self.F = X_s, Y, F
        # global subset of world * B_u pool indices; this rank's slice [rank * B_u, (rank + 1) * B_u)
        self.n_sub = self.world * self.B_u
        self.idx = torch.zeros(max(self.n_sub, 1), dtype=torch.int32, device=dev)
        self.rng_off = torch.zeros(1, dtype=torch.int64, device=dev)
        self.step_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        self.lr = torch.tensor([lr], dtype=torch.float32, device=dev)
        self.optimizer = FusedAdamSchedule(lr, betas, eps)
        self._lr_host = float(lr)
        self.m = torch.zeros_like(self.flat.P)
        self.v = torch.zeros_like(self.flat.P)
        self.seed = int(seed)
        self.subset_seed = int(seed if subset_seed is None else subset_seed)
        self.distributed = distributed
        self.pg = process_group
        # RCCL all-reduce captured inside the step's graph (one replay per step, no host hop between
        # the gradient and the update); host-side between two graphs for gloo
        self.graph_allreduce = bool(graph_allreduce)
        self.adam = L.AdamDesc(p=self.flat.P.data_ptr(), g=self.flat.G.data_ptr(), m=self.m.data_ptr(),
                               v=self.v.data_ptr(), n=self.flat.numel, lr=self.lr.data_ptr(),
                               step=self.step_ctr.data_ptr(), beta1=betas[0], beta2=betas[1], eps=eps)
        self.idx_next = torch.zeros_like(self.idx)
        # A/B switch (tools/critpath_probe.py): draw the next step's subset on the side stream ahead of the ROM
        self.subset_early = False
        # captured form: 'streams' (one graph per stream, ordered only by device counters, _capture_streams:
        # no event edge between the streams at all -- 0.5816 / 0.5827 vs 0.5901 / 0.5904 ms per step with
        # 'single', interleaved on one box, r04g), 'single' (one graph spanning both streams, forked and
        # joined by events at its ends) or 'segments' (single-stream graphs joined by events,
        # _capture_segments: each graph boundary leaves the GPU idle ~15 us: 0.673 vs 0.629 ms, r03).
        # The split DP form (host-side all-reduce between two graphs) keeps 'single'.
        # GPI_GRAPH_MODE overrides (A/B runs)
        self.graph_mode = os.environ.get('GPI_GRAPH_MODE', 'streams')
        if self.graph_mode == 'streams' and self.distributed and not (
                self.graph_allreduce and dist.get_backend(self.pg) == dist.Backend.NCCL):
            self.graph_mode = 'single'
        my_idx = self.idx[self.rank * self.B_u:(self.rank + 1) * self.B_u] if self.B_u else None
        self.engine.bind(X_u=self.X_pool, u_index=my_idx, X_s=X_s, Y=Y, F=F)
        n_pool = self.X_pool.shape[0] if self.X_pool is not None else 0
        if self.B_u and self.n_sub > n_pool:
            raise ValueError('the pool (%d) is smaller than the global armortized batch (%d)' % (n_pool, self.n_sub))
        self.n_pool = n_pool
        self._subset_ws = None
        if self.B_u and n_pool > 16384:
            nb = C.c_int64(0)
            L.check(L.lib().gpi_random_subset_workspace(n_pool, C.byref(nb)), 'random subset workspace')
            self._subset_ws = torch.zeros(nb.value, dtype=torch.uint8, device=dev)
        drop_span = max([(p.drop_numel + 3) // 4 + 1 for p in (self.engine.ep, self.engine.dp)
                         if p is not None and p.drop_numel] or [0])
        self.rng_span = max(n_pool, (self.engine.B * self.engine.dz + 3) // 4 + 1,
                            (self.N_s * self.engine.d_x + 3) // 4 + 1, drop_span)
        self.adam.rng_offset = self.rng_off.data_ptr()
        self.adam.rng_advance = self.rng_span
        ws = self.engine.ws
        self.last_terms = torch.zeros(L.GPI_REPLICAS * 16, dtype=torch.float64, device=dev)
        self.epi = L.StepEpilogueDesc(gacc=self.flat.gacc.data_ptr(), grad=self.flat.G.data_ptr(), n=self.flat.numel,
                                      flags=L.FINALIZE_ZERO, n_terms=self.last_terms.numel(),
                                      step=self.step_ctr.data_ptr(), scratch=ws.t_scr.data_ptr(),
                                      n_scratch=ws.t_scr.numel(), terms_dst=self.last_terms.data_ptr(),
                                      idx_src=self.idx_next.data_ptr(), idx_dst=self.idx.data_ptr(),
                                      n_idx=self.n_sub if self.B_u else 0)
        # the next step's encoder Dropout2d masks: drawn by the epilogue (after the encoder backward,
        # which reads this step's), Philox sub id 4 as _launch_noise(sub0=0) would
        ep = self.engine.ep
        if ep is not None and ep.drop_numel > 0:
            self.epi.drop_out = self.engine.ws.fptr(ep.drop_off).value
            self.epi.drop_n = ep.drop_numel
            self.epi.drop_p = ep.drop_rate
            self.epi.drop_seed = self.seed
            self.epi.drop_offset = self.rng_off.data_ptr()
            self.epi.drop_sub = 4
        # single-process steps: the epilogue and Adam in one launch (gpi_step_epilogue_adam; nothing
        # runs between the gradient delivery and the update); GPI_FUSED_ADAM=0 keeps two launches
        self.fuse_adam = not self.distributed and os.environ.get('GPI_FUSED_ADAM', '1') != '0'
        self.epi_adam = L.StepEpilogueDesc.from_buffer_copy(self.epi)
        self.epi_adam.step = None                  # Adam's counter: incremented once by the fused launch
        self.done_ctr = torch.zeros(1, dtype=torch.int32, device=dev)
        # side-stream hand-offs by device flags (gpi_stream_signal / gpi_stream_wait) instead of graph
        # events between the streams; GPI_HANDOFF=events keeps the events (A/B)
        self.handoff = os.environ.get('GPI_HANDOFF', 'flags') if self.graph_mode in ('single', 'streams') \
            else 'events'
        if self.graph_mode == 'streams' and self.handoff != 'flags':
            self.graph_mode = 'single'
        # 'streams': the side stream is gated per step by this counter (no event between the streams), so
        # each stream's part of the step is captured as a graph of its own
        self.side_done = torch.zeros(1, dtype=torch.int64, device=dev)
        self._probed_stream = None
        self.unroll = 1
        self.g_fb_k = self.g_side_k = None
        if self.handoff == 'flags':
            self._configure_handoff()
            if self.fuse_adam:
                # the join with the side stream's last reduction inside the fused epilogue + Adam launch
                self.epi_adam.wait_flag = self.handoff_flags.data_ptr() + 4 * 3
                self.epi_adam.wait_err = self.handoff_flags.data_ptr() + 4 * 4
            # a timed-out hand-off (sticky error word) stops every later parameter update: the gradient of
            # such a step may be incomplete, so no step after it may move the parameters
            self.adam.wait_err = self.handoff_flags.data_ptr() + 4 * 4
            if self.distributed and self.flat.err_slot >= 0:
                # data parallel: the epilogue writes the word into the flat gradient's error slot (inside the
                # all-reduced prefix) and Adam reads the SUM, so one rank's timeout stops every rank's update
                # (and sets every rank's word: all of them raise) -- no rank applies a gradient averaged with
                # an incomplete one
                self.epi.wait_err = self.handoff_flags.data_ptr() + 4 * 4
                self.epi.err_slot = self.flat.err_slot
                self.adam.skip_if = self.flat.G.data_ptr() + 4 * self.flat.err_slot
        # lazy surfacing of that error word without a host sync: an async copy to pinned memory after
        # a replay, read once its event has completed (at the next step() / run() / check_handoff())
        self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True) if dev.type == 'cuda' else None
        self._err_ev = None
        self._err_every = int(os.environ.get('GPI_ERR_CHECK_EVERY', '16'))
        self._n_steps = 0
        self._fb_pending = False
        self.graph = None
        self._one_draw = os.environ.get('GPI_ONE_DRAW', '1') != '0'
        # the first step's noise; every step then draws the next step's during its backward
        self._launch_noise(L.stream_handle(), self.idx, sub0=100)

    # ------------------------------------------------------------------
    def _launch_subset(self, st, idx, sub0=0):
        if not self.B_u:
            return
        if self._subset_ws is None:       # pools up to 16384: one launch, the keys in LDS
            L.check(L.lib().gpi_random_subset(L.ptr(idx), self.n_pool, self.n_sub, self.subset_seed,
                                              L.ptr(self.rng_off), sub0 + 1, st), 'random subset')
        else:                             # any pool (the reference's randperm(N) has no cap)
            L.check(L.lib().gpi_random_subset_ws(L.ptr(idx), self.n_pool, self.n_sub, self.subset_seed,
                                                 L.ptr(self.rng_off), sub0 + 1, L.ptr(self._subset_ws),
                                                 self._subset_ws.numel(), st), 'random subset')

    def _launch_noise(self, st, idx, sub0=0, codecs=('enc', 'dec'), subset=True):
        """Random subset into ``idx`` and the reparametrisation noise into the engine's eps
        buffers.  Philox streams: the step's offset (advanced by Adam at the end of every step)
        and sub ids sub0 + {1, 2, 3}; the noise drawn during step k (for step k+1) therefore
        differs from step k's own, which was drawn during step k-1 or by the prologue (sub0 = 100).
        All of it in ONE launch (gpi_draws: the same draws as the separate entry points, bit for bit)
        unless the pool needs the multi-launch subset form or GPI_ONE_DRAW=0."""
        lib = L.lib()
        if self._one_draw and (not subset or not self.B_u or self._subset_ws is None):
            items = []
            e = self.engine
            if e.has_dropout and codecs:
                for k, (c, prog) in enumerate((('enc', e.ep), ('dec', e.dp))):
                    if c in codecs and prog is not None and prog.drop_numel:
                        items.append(L.DrawItem(kind=L.DRAW_DROPOUT, p=prog.drop_rate, out=e.ws.fptr(prog.drop_off).value,
                                                n=prog.drop_numel, sub=sub0 + 4 + k, seed=self.seed))
            if subset and self.B_u:     # (the subset's key: the seed every rank shares)
                items.append(L.DrawItem(kind=L.DRAW_SUBSET, out=idx.data_ptr(), n=self.n_pool, k=self.n_sub,
                                        sub=sub0 + 1, seed=self.subset_seed))
            ez = e.eps_z()
            items.append(L.DrawItem(kind=L.DRAW_RANDN, out=ez.data_ptr(), n=ez.numel(), sub=sub0 + 2, seed=self.seed))
            if e.N_ex:
                ex = e.eps_x()
                items.append(L.DrawItem(kind=L.DRAW_RANDN, out=ex.data_ptr(), n=ex.numel(), sub=sub0 + 3,
                                        seed=self.seed))
            arr = (L.DrawItem * len(items))(*items)
            L.check(lib.gpi_draws(arr, len(items), L.ptr(self.rng_off), st), 'step draws')
            return
        if self.engine.has_dropout and codecs:   # Dropout2d channel scales (sub ids sub0 + 4 enc, + 5 dec)
            self.engine.draw_dropout(st, self.seed, L.ptr(self.rng_off), sub0 + 4, codecs=codecs)
        if subset:
            self._launch_subset(st, idx, sub0)
        ez = self.engine.eps_z()
        L.check(lib.gpi_randn(L.ptr(ez), ez.numel(), self.seed, L.ptr(self.rng_off), sub0 + 2, st), 'randn z')
        if self.engine.N_ex:
            ex = self.engine.eps_x()
            L.check(lib.gpi_randn(L.ptr(ex), ex.numel(), self.seed, L.ptr(self.rng_off), sub0 + 3, st), 'randn x')

    def forward_backward(self, stream=None):
        """One step without the parameter update (gradient in flat.G and the ELBO terms delivered;
        update() then applies Adam).  Every forward_backward() must be followed by update() before the
        next one: the cross-stream flags count one signal per step, and the step counter that their waits
        compare against advances only in the update (an unpaired pass would leave the flags ahead and every
        later wait would pass at once)."""
        if self._fb_pending:
            raise RuntimeError('FusedElboStep.forward_backward() called twice without update() in between')
        self._forward_backward(stream, epilogue=True)
        self.engine.rejoin()
        self._fb_pending = True

    def _forward_backward(self, stream=None, epilogue=True):
        """One step without the parameter update.  The step's noise and subset were drawn by the
        previous step (off the critical path); the next step's are drawn on the side stream once
        the head backward has consumed this step's; the epilogue (gradient finalisation, scratch
        reset, subset hand-over) is one launch."""
        st = stream if stream is not None else L.stream_handle()
        # subset_early: the next step's subset (it writes only idx_next) ahead of the ROM on the side stream
        early = self.subset_early and bool(self.engine.roms)
        self.engine.side_pre = (lambda sst: self._launch_subset(sst, self.idx_next)) if early else None
        self.engine.forward(st, compute_value=False, zero_gacc=False, zero_scratch=False, running='defer')
        # next step's subset / noise / decoder masks concurrently with the encoder backward; the
        # encoder's masks by the epilogue below (the encoder backward reads this step's)
        # the fused epilogue + Adam launch (update(fused=True)) waits for the side stream itself; every
        # other continuation needs the main stream to wait here
        self.engine.backward(st, side_extra=lambda sst: self._launch_noise(sst, self.idx_next, codecs=('dec',),
                                                                           subset=not early),
                             main_wait=epilogue or not self.fuse_adam)
        if epilogue:                  # (else: launched by update(fused=True), with Adam)
            L.check(L.lib().gpi_step_epilogue(C.byref(self.epi), st), 'step epilogue')

    def allreduce(self):
        if self.distributed:
            allreduce_shared(self.flat, self.pg)

    def sync_lr(self):
        """Copy a scheduler-changed learning rate (optimizer.param_groups[0]['lr']) to the device."""
        lr = float(self.optimizer.param_groups[0]['lr'])
        if lr != self._lr_host:
            self.lr.fill_(lr)
            self._lr_host = lr

    def update(self, stream=None, fused=False):
        """Adam (+ RNG offset advance).  fused: the step epilogue and Adam in one launch -- after
        _forward_backward(epilogue=False), single-process steps only."""
        st = stream if stream is not None else L.stream_handle()
        self._fb_pending = False
        if fused:
            L.check(L.lib().gpi_step_epilogue_adam(C.byref(self.epi_adam), C.byref(self.adam),
                                                   L.ptr(self.done_ctr), st), 'step epilogue + adam')
        else:
            L.check(L.lib().gpi_adam(C.byref(self.adam), st), 'adam (+ rng offset advance)')

    def _mark_optimizer_step(self):
        """Tell torch LR schedulers that an optimizer step happened (their hook wraps
        optimizer.step() to set this flag; calling the wrapped no-op through torch's profiling
        hooks costs ~0.2 ms of host time per step, as much as a third of the step)."""
        self.optimizer._opt_called = True

    def step_eager(self):
        self._check_stream_pair()
        fused = self.fuse_adam
        self._forward_backward(epilogue=not fused)
        self.allreduce()
        self.update(fused=fused)
        self.engine.rejoin()
        self._mark_optimizer_step()

    def check_handoff(self):
        """Raise if a side-stream flag wait timed out (host sync).  The step that timed out and every step
        after it have left the parameters and Adam moments untouched (the error word is sticky)."""
        if int(self.handoff_flags[4].item()) != 0:
            raise RuntimeError('FusedElboStep: a cross-stream flag wait timed out (gpi_stream_wait); '
                               'parameter updates were skipped from that step on')

    def _poll_error(self):
        """Raise if the last posted copy of the error word (see _post_error_copy) shows a timed-out wait;
        never blocks (an unfinished copy is read at a later call)."""
        ev = self._err_ev
        if ev is not None and ev.query():
            self._err_ev = None
            if int(self._err_host[0]) != 0:
                raise RuntimeError('FusedElboStep: a cross-stream flag wait timed out (gpi_stream_wait); '
                                   'parameter updates were skipped from that step on')

    def _post_error_copy(self):
        if self._err_host is None or self.handoff != 'flags' or self._err_ev is not None:
            return
        self._err_host.copy_(self.handoff_flags[4:5], non_blocking=True)
        self._err_ev = torch.cuda.Event()
        self._err_ev.record()

    # ------------------------------------------------------------------
    def _mutable_state(self):
        """Every device buffer a step writes: parameters, Adam moments and counter, Philox offset,
        subsets, accumulators, gradient, the workspace (incl. the pre-drawn noise) and the term /
        statistics scratch."""
        ws = self.engine.ws
        return [self.flat.P, self.m, self.v, self.step_ctr, self.rng_off, self.idx, self.idx_next, self.done_ctr,
                self.handoff_flags, self.side_done,
                self.flat.gacc, self.flat.G, ws.t_ws, ws.t_scr, ws.t_parts, ws.t_flag, self.last_terms] + \
            self.engine.running.buffers

    def capture(self, unroll=1):
        """Capture the step into HIP graph(s); the all-reduce stays outside the graph.
        The two warm-up steps run on snapshots: capture() leaves parameters, optimizer state,
        step counter, random stream and the pre-drawn subset / noise exactly as it found them, so
        the first replayed step is the step an eager loop would take next.
        unroll > 1 ('streams' mode): also capture `unroll` consecutive steps as one pair of graphs, which
        run(n) replays (one graph-launch boundary per `unroll` steps; every step still reads its counters,
        subset, noise and learning rate from device memory, so the steps are the ones step() would take --
        a learning-rate change reaches the device at the next replay)."""
        self.unroll = 1
        self.g_fb_k = self.g_side_k = None
        if self.sync_bn and self.bn_exchange != 'peer' and dist.get_backend(self.pg) != dist.Backend.NCCL:
            raise RuntimeError('FusedElboStep.capture: SyncBN over a host-side backend (gloo) runs eagerly only '
                               "(bn_exchange='peer' captures with any backend)")
        torch.cuda.synchronize()
        saved = [t.clone() for t in self._mutable_state()]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):          # warm up allocator / kernels on the side stream
                self.step_eager()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.check_handoff()            # (the restore below would erase a warm-up step's timeout)
        for t, v in zip(self._mutable_state(), saved):
            t.copy_(v)
        del saved
        torch.cuda.synchronize()
        self.g_fb = torch.cuda.CUDAGraph()
        self.g_up = None
        self.g_side = None
        self.segs = None
        self.split_graph = self.distributed and not (self.graph_allreduce and
                                                      dist.get_backend(self.pg) == dist.Backend.NCCL)
        if not self.split_graph and self.graph_mode == 'segments':
            self._capture_segments()
        elif not self.split_graph and self.graph_mode == 'streams':
            self._capture_streams()
            if unroll > 1:
                self.g_fb_k, self.g_side_k = self._capture_streams(unroll)
                self.unroll = int(unroll)
        elif self.split_graph:
            with torch.cuda.graph(self.g_fb):
                self.forward_backward()
                self.engine.rejoin()
            self.g_up = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_up):
                self.update()
        else:
            fused = self.fuse_adam
            with torch.cuda.graph(self.g_fb):
                self._forward_backward(epilogue=not fused)
                self.allreduce()        # RCCL: captured as a graph node
                self.update(fused=fused)
                self.engine.rejoin()
        self.graph = True

    def _queues_separate(self):
        """True iff a kernel on the current stream runs while a kernel of the side stream spins
        (gpi_queue_probe): the two are on different hardware queues.  HIP maps streams to its
        GPU_MAX_HW_QUEUES queues round-robin, so in a process with many streams two can share one, and
        a flag wait ahead of its signal on a shared queue blocks it (tools/queue_stress.py: 3 of 18
        steps timed out with 6 step objects in 'streams' mode, none in 'single', whose graph
        branches the runtime places itself)."""
        e = self.engine
        pr = torch.zeros(2, dtype=torch.int32, device=self.flat.P.device)
        # up to four side-stream candidates (HIP deals new streams round-robin over its queues, so one of
        # four consecutive ones sits on another queue than the current stream); a replaced candidate is
        # dropped before any work or capture used it
        for attempt in range(4):
            side = e._side_stream()
            pr.zero_()
            torch.cuda.synchronize()
            L.check(L.lib().gpi_queue_probe(L.ptr(pr), L.ptr(pr[1:]), C.c_void_p(side.cuda_stream)), 'queue probe')
            L.check(L.lib().gpi_stream_signal(L.ptr(pr), L.ptr(self.step_ctr), L.stream_handle()),
                    'queue probe signal')
            torch.cuda.synchronize()
            self._probed_stream = torch.cuda.current_stream()
            if int(pr[1].item()) == 1:
                return True
            if getattr(self, 'graph', None) is not None:
                return False        # the captured graphs hold this side stream
            e._side = None          # next candidate
        return False

    def _configure_handoff(self):
        """Flag hand-offs between the streams; graph mode 'streams' (no event between the streams at all)
        only on a verified pair of hardware queues, else 'single' (one graph whose event fork / join at
        its ends the runtime orders)."""
        if self.graph_mode == 'streams' and not self._queues_separate():
            self.graph_mode = 'single'
        self.engine.set_flag_handoff(self.handoff_flags[:4], self.step_ctr, self.handoff_flags[4:5],
                                     side_done=self.side_done if self.graph_mode == 'streams' else None)

    def _check_stream_pair(self):
        """'streams' mode, before a step: the probe was made against another current stream -- probe this
        one; on a shared queue fall back to 'single' (and capture again if the step was captured)."""
        if self.graph_mode != 'streams' or torch.cuda.current_stream() == self._probed_stream:
            return
        if self._queues_separate():
            return
        self.graph_mode = 'single'
        self._configure_handoff()
        if self.graph is not None:
            self.capture()          # ('single': no unrolled graphs; run() replays single steps)

    def _capture_streams(self, steps=1):
        """The step as TWO graphs, one per stream, captured at once: the main stream's (encoder, head,
        decoder, their backward, the epilogue + Adam) and the side stream's (ROM, the variational samples'
        head backward, the slab reductions, the next step's noise), ordered only by the device counters
        of the flag hand-offs and the side stream's step gate -- no graph edge between the streams.
        steps > 1: that many consecutive steps in the pair, returned as (main, side) graphs."""
        fused = self.fuse_adam
        side = self.engine._side_stream()
        cap = torch.cuda.Stream()
        cap.wait_stream(torch.cuda.current_stream())
        side.wait_stream(torch.cuda.current_stream())
        g_fb = self.g_fb if steps == 1 else torch.cuda.CUDAGraph()
        g_side = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            g_side.capture_begin(capture_error_mode='relaxed')
        try:
            with torch.cuda.stream(cap):
                g_fb.capture_begin(capture_error_mode='relaxed')
                try:
                    for _ in range(steps):
                        self._forward_backward(epilogue=not fused)
                        self.allreduce()        # RCCL: captured as a graph node
                        self.update(fused=fused)
                finally:
                    g_fb.capture_end()
        finally:
            with torch.cuda.stream(side):
                g_side.capture_end()
        torch.cuda.current_stream().wait_stream(cap)
        if steps == 1:
            self.g_side = g_side
        return g_fb, g_side

    def _capture_segments(self):
        """The step as single-stream graphs, one per stretch of a stream between two cross-stream
        dependencies, replayed with events between them (_replay_segments).  A HIP graph whose
        nodes span two streams costs the host ~4-8 us per node to launch (tools/graph_launch_probe.py:
        64 nodes 211-245 us on two streams vs 50-58 us on one); with the step's ~70 nodes in one
        two-stream graph the host walk (~0.59 ms) paced the GPU and the side stream's kernels were
        submitted late, so the step waited at the join for them."""
        e = self.engine
        e.handoff = None                     # the segments are joined by events between the graphs
        self.epi_adam.wait_flag = None
        self.epi_adam.wait_err = None
        side = e._side_stream()
        rom = bool(e.roms)
        early = self.subset_early and rom
        e.side_pre = (lambda sst: self._launch_subset(sst, self.idx_next)) if early else None
        n_enc = len(e.enc_descs) if e.ep is not None else 0
        enc_split = bool(n_enc) and e.enc_reduce == 'split'

        def cap(fn):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fn(L.stream_handle())
            return g

        def m2(st):
            e.forward_b(st)
            e._running_pending = True            # running statistics deferred to the side stream
            e.backward_a(st, rom)

        def m5(st):
            fused = self.fuse_adam
            if not fused:
                L.check(L.lib().gpi_step_epilogue(C.byref(self.epi), st), 'step epilogue')
            self.allreduce()                     # RCCL: captured as a graph node
            self.update(st, fused=fused)

        noise = (lambda sst: self._launch_noise(sst, self.idx_next, codecs=('dec',), subset=not early))
        segs = {'m1': cap(lambda st: e.forward_a(st, zero_gacc=False, zero_scratch=False))}
        if rom:
            segs['s1'] = cap(e.rom_side)
        segs['m2'] = cap(m2)
        segs['s2'] = cap(lambda st: e.backward_side_a(st, rom, noise))
        if n_enc:
            segs['m3'] = cap(e.backward_b)
        if enc_split:
            segs['s3'] = cap(e.backward_side_b)
        if n_enc:
            segs['m4'] = cap(lambda st: e.backward_c(st, enc_split))
        segs['m5'] = cap(m5)
        self.segs = segs
        self._seg_ev = [torch.cuda.Event() for _ in range(4)]
        self._seg_side = side

    def _replay_segments(self):
        g, ev, side = self.segs, self._seg_ev, self._seg_side
        main = torch.cuda.current_stream()
        g['m1'].replay()
        if 's1' in g:
            ev[0].record(main)
            with torch.cuda.stream(side):
                side.wait_event(ev[0])
                g['s1'].replay()
        g['m2'].replay()
        ev[1].record(main)
        with torch.cuda.stream(side):
            side.wait_event(ev[1])
            g['s2'].replay()
        if 'm3' in g:
            g['m3'].replay()
        if 's3' in g:
            ev[2].record(main)
            with torch.cuda.stream(side):
                side.wait_event(ev[2])
                g['s3'].replay()
        ev[3].record(side)
        if 'm4' in g:
            g['m4'].replay()
        main.wait_event(ev[3])
        g['m5'].replay()

    def step(self):
        """One training step (graph replay once captured).  A timed-out cross-stream wait raises at a
        later step() (its error word is copied back every GPI_ERR_CHECK_EVERY steps, no host sync)."""
        self._poll_error()
        self._step()
        self._n_steps += 1
        if self._err_every > 0 and self._n_steps % self._err_every == 0:
            self._post_error_copy()

    def _step(self):
        self.sync_lr()
        if self.graph is None:
            return self.step_eager()
        if self.segs is not None:
            self._replay_segments()
            self._mark_optimizer_step()
            return
        if self.g_side is not None:
            self._check_stream_pair()
        if self.g_side is not None:
            # (the side graph launched first instead: 0.5772-0.5774 vs 0.5767-0.5769 ms, r04k)
            self.g_fb.replay()
            with torch.cuda.stream(self.engine._side):
                self.g_side.replay()
            self._mark_optimizer_step()
            return
        self.g_fb.replay()
        if self.split_graph:
            self.allreduce()
            self.g_up.replay()
        self._mark_optimizer_step()

    def run(self, n):
        """n steps: with capture(unroll=k), n // k replays of the k-step graphs, then single steps."""
        n = int(n)
        self._poll_error()
        if self.graph is not None and self.unroll > 1 and self.g_fb_k is not None:
            self.sync_lr()
            self._check_stream_pair()
            if self.graph_mode == 'streams' and self.g_fb_k is not None:
                for _ in range(n // self.unroll):
                    self.g_fb_k.replay()
                    with torch.cuda.stream(self.engine._side):
                        self.g_side_k.replay()
                    self._mark_optimizer_step()
                n %= self.unroll
        for _ in range(n):
            self._step()
        self._post_error_copy()

    def elbo(self):
        """ELBO value of the last completed step (0-d tensor)."""
        return self.engine.elbo_value(self.last_terms)
