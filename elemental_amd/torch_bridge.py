"""Host collective bridge: implements the library's host-backend collectives
(elx_host_coll_fn / elx_host_split_fn) with torch.distributed process groups
(gloo).  This plays the role the reference gives plain MPI for host buffers
(src/core/imports/mpi/*.hpp) and is what the CPU multi-rank tests run on;
device data on a host-backed grid is staged through pinned memory by the
library itself.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L

_NP = {L.F32: np.float32, L.F64: np.float64, L.F16: np.float16, L.BF16: np.int16, L.I32: np.int32,
       L.I64: np.int64, L.U8: np.uint8}
_ES = {L.F32: 4, L.F64: 8, L.F16: 2, L.BF16: 2, L.I32: 4, L.I64: 8, L.U8: 1}


def _arr(ptr: int, count: int, dtype: int) -> torch.Tensor:
    """Tensor view over `count` elements at raw host address `ptr`."""
    if count == 0 or not ptr:
        t = torch.empty(0, dtype=torch.float32)
        return t
    nbytes = count * _ES[dtype]
    buf = (ctypes.c_char * nbytes).from_address(ptr)
    a = np.frombuffer(buf, dtype=_NP[dtype], count=count)
    t = torch.from_numpy(a)
    if dtype == L.BF16:
        t = t.view(torch.bfloat16)
    return t


class GlooBridge:
    """Collectives for an already initialised torch.distributed world (gloo)."""

    def __init__(self):
        assert dist.is_initialized(), "init torch.distributed (gloo) first"
        self.rank = dist.get_rank()
        self.size = dist.get_world_size()
        self.groups = {0: (None, list(range(self.size)))}  # id -> (pg, ranks by group rank)
        self.coll_fn = L.HOST_COLL_FN(self._coll)
        self.split_fn = L.HOST_SPLIT_FN(self._split)

    def _coll(self, ctx, op, group, dtype, send, recv, count, peer, peer2):
        try:
            pg, ranks = self.groups[group]
            n = len(ranks)
            me = ranks.index(self.rank)
            if op == L.COLL_BARRIER:
                dist.barrier(group=pg)
            elif op == L.COLL_ALLGATHER:
                s = _arr(send, count, dtype).clone()
                r = _arr(recv, count * n, dtype)
                outs = self._gather(s, pg, ranks)
                if count:
                    r.copy_(torch.cat(outs))
            elif op == L.COLL_REDUCE_SCATTER:  # gloo has no reduce_scatter: all-reduce, keep my slice
                s = _arr(send, count * n, dtype).clone()
                acc = s.double() if s.dtype in (torch.float16, torch.bfloat16) else s
                dist.all_reduce(acc, group=pg)
                r = _arr(recv, count, dtype)
                if count:
                    r.copy_(acc[me * count:(me + 1) * count].to(r.dtype))
            elif op == L.COLL_ALLREDUCE:
                s = _arr(send, count, dtype).clone()
                acc = s.double() if s.dtype in (torch.float16, torch.bfloat16) else s
                dist.all_reduce(acc, group=pg)
                if count:
                    _arr(recv, count, dtype).copy_(acc.to(s.dtype))
            elif op == L.COLL_ALLTOALL:  # gloo has no all_to_all: gather everything, keep my column
                s = _arr(send, count * n, dtype).clone()
                outs = self._gather(s, pg, ranks)
                r = _arr(recv, count * n, dtype)
                if count:
                    r.copy_(torch.cat([o[me * count:(me + 1) * count] for o in outs]))
            elif op == L.COLL_SENDRECV:  # send -> group rank peer, recv <- group rank peer2
                s = _arr(send, count, dtype).clone()
                r = _arr(recv, count, dtype)
                if peer == me and peer2 == me:
                    r.copy_(s)
                elif count:
                    tmp = torch.empty_like(s)
                    req = dist.isend(s, dst=ranks[peer], group=pg)
                    dist.recv(tmp, src=ranks[peer2], group=pg)
                    req.wait()
                    r.copy_(tmp)
            elif op == L.COLL_BCAST:
                t = _arr(send, count, dtype)
                tmp = t.clone()
                dist.broadcast(tmp, src=ranks[peer], group=pg)
                if count:
                    t.copy_(tmp)
            else:
                return 1
            return 0
        except Exception as e:  # never let an exception unwind through C
            import sys
            print(f"GlooBridge op {op} failed: {e!r}", file=sys.stderr)
            return 1

    @staticmethod
    def _gather(s: torch.Tensor, pg, ranks):
        """all_gather in THIS group's rank order: torch numbers a new_group's
        members in ascending global rank, a Split orders them by key."""
        outs = [torch.empty_like(s) for _ in ranks]
        dist.all_gather(outs, s, group=pg)
        by_global = dict(zip(sorted(ranks), outs))
        return [by_global[g] for g in ranks]

    def _split(self, ctx, group, color, key, out_group, out_rank, out_size):
        try:
            assert group == 0, "only the world is split"
            pairs = [None] * self.size
            dist.all_gather_object(pairs, (color, key, self.rank))
            colors = sorted({c for c, _, _ in pairs})
            mine = None
            for c in colors:  # every rank creates every group in the same order
                members = sorted([(k, r) for cc, k, r in pairs if cc == c])
                ranks = [r for _, r in members]
                pg = dist.new_group(ranks=ranks)
                if c == color:
                    mine = (pg, ranks)
            gid = len(self.groups)
            self.groups[gid] = mine
            out_group[0] = gid
            out_rank[0] = mine[1].index(self.rank)
            out_size[0] = len(mine[1])
            return 0
        except Exception as e:
            import sys
            print(f"GlooBridge split failed: {e!r}", file=sys.stderr)
            return 1
