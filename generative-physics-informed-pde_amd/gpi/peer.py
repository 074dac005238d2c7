"""One-shot peer exchange for the SyncBN seams (SURVEY.md sections 2.3 / 8e): each rank's process owns a
small device buffer [2 message slots | flag word]; every rank maps every other rank's buffer through HIP IPC
(gpi_peer_alloc / gpi_peer_open, handles exchanged once over the process group), and gpi_bn_exchange
(GPI_BNX_PEER) all-reduces one BN seam's sums through them in ONE 64-thread launch: no collective library
call, no host involvement, capturable in the step graph.  The RCCL form of the same seam is three launches
(fold, all-reduce, unfold: ElboEngine._sync_stats)."""
import ctypes as C

import torch
import torch.distributed as dist

from . import _lib as L

FLAG_OFF = 2 * L.GPI_BNX_MSG * 8          # bytes: two message slots, then the flag word
BYTES = FLAG_OFF + 256


class PeerExchange(object):
    def __init__(self, group=None, err=None):
        """group: the ranks' process group (any backend; used once, for the IPC handles).  err: a device
        uint32 error word set on a wait timeout (FusedElboStep's hand-off error word)."""
        lib = L.lib()
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if self.world > L.GPI_MAX_RANKS:
            raise ValueError('PeerExchange: at most %d ranks' % L.GPI_MAX_RANKS)
        own = C.c_void_p()
        handle = (C.c_char * 64)()
        L.check(lib.gpi_peer_alloc(BYTES, C.byref(own), handle), 'peer buffer')
        self._own = own
        handles = [bytes(handle)]
        if self.world > 1:
            handles = [None] * self.world
            dist.all_gather_object(handles, bytes(handle), group=group)
        self.bufs = []
        self._opened = []
        for p in range(self.world):
            if p == self.rank:
                self.bufs.append(own.value)
                continue
            ptr = C.c_void_p()
            h = (C.c_char * 64).from_buffer_copy(handles[p])
            L.check(lib.gpi_peer_open(h, C.byref(ptr)), 'peer buffer of rank %d' % p)
            self.bufs.append(ptr.value)
            self._opened.append(ptr)
        self.seq = torch.zeros(1, dtype=torch.int32, device=torch.device('cuda', torch.cuda.current_device()))
        self.err = err
        if self.world > 1:
            dist.barrier(group)

    def fill(self, d):
        """Point a BnExchangeDesc at the exchange (mode GPI_BNX_PEER)."""
        d.mode = L.BNX_PEER
        d.rank, d.world = self.rank, self.world
        for p, b in enumerate(self.bufs):
            d.peer_buf[p] = b
            d.peer_flag[p] = b + FLAG_OFF
        d.seq = self.seq.data_ptr()
        d.err = self.err.data_ptr() if self.err is not None else None
        return d

    def close(self):
        lib = L.lib()
        for p in self._opened:
            lib.gpi_peer_close(p, 0)
        self._opened = []
        if self._own is not None:
            lib.gpi_peer_close(self._own, 1)
            self._own = None
