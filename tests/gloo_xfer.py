"""The owner's tagged transport over torch.distributed gloo, for the
multi-process tests of peer-transfer domains (tests/test_coll_host.py,
tests/test_coll_peer_gpu.py): it stands in for the owner provider's
fi_tsendmsg / fi_trecvmsg(FI_PEER_TRANSFER) (coll_coll.c:770-814).  Host
memory only — device buffers reach it through the provider's staging."""
import ctypes

import torch
import torch.distributed as dist


class GlooXfer:
    """The owner's tagged transport, over gloo.  prov/coll's tag
    (cid | sender << 32, cid = group_id << 16 | seq, group_id <= 256) is
    folded into gloo's 31-bit tag space: 6 bits of sender, 9 of group id, 16
    of seq."""

    def __init__(self):
        self.reqs, self.next = {}, 1
        self.sent = self.received = 0

    @staticmethod
    def _tag(tag):
        return ((tag >> 32) & 0x3F) << 25 | ((tag >> 16) & 0x1FF) << 16 | (tag & 0xFFFF)

    def _put(self, v):
        h = self.next
        self.next += 1
        self.reqs[h] = v
        return h

    def send(self, peer, ptr, nbytes, tag):
        # a zero-byte message (a barrier arrival) travels as one byte
        t = (torch.frombuffer(bytearray(ctypes.string_at(ptr, nbytes)), dtype=torch.uint8)
             if nbytes else torch.zeros(1, dtype=torch.uint8))
        self.sent += nbytes
        return self._put((dist.isend(t, peer, tag=self._tag(tag)), t, None, 0))

    def recv(self, peer, ptr, nbytes, tag):
        t = torch.empty(max(nbytes, 1), dtype=torch.uint8)
        return self._put((dist.irecv(t, peer, tag=self._tag(tag)), t, ptr, nbytes))

    def test(self, h):
        # gloo's send/recv Work objects only report completion through
        # wait(); every transfer of a group is posted before the executor
        # tests any, so waiting here cannot deadlock the schedule
        w, t, ptr, n = self.reqs[h]
        w.wait()
        if ptr and n:
            ctypes.memmove(ptr, t.data_ptr(), n)
            self.received += n
        del self.reqs[h]
        return 1
