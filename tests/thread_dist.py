"""In-process stand-in for the torch.distributed collectives the ledger router uses
(all_gather, all_gather_object, all_to_all_single, all_reduce), with one thread per rank.

It lets the device-resident routed step run with several ranks on ONE GPU and with
CUDA tensors -- the path `bench.py --gpus N` takes over RCCL -- where a real RCCL
group needs one GPU per rank.  Test infrastructure only.
"""
from __future__ import annotations

import copy
import threading


class ThreadGroup:
    def __init__(self, world: int):
        self.world = world
        self.barrier = threading.Barrier(world)
        self.slots = [None] * world


class ThreadDist:
    class ReduceOp:
        SUM, MAX = "sum", "max"

    def __init__(self, group: ThreadGroup, rank: int):
        self.g, self.rank, self.world = group, rank, group.world

    def _exchange(self, obj):
        self.g.slots[self.rank] = obj
        self.g.barrier.wait()
        out = list(self.g.slots)
        self.g.barrier.wait()
        return out

    @staticmethod
    def _sync(t):
        import torch
        if t.is_cuda:
            torch.cuda.current_stream(t.device).synchronize()

    def all_gather(self, tensor_list, tensor, group=None):
        self._sync(tensor)
        got = self._exchange(tensor.clone())
        for dst, src in zip(tensor_list, got):
            dst.copy_(src)
        self._sync(tensor)

    def all_gather_object(self, out, obj, group=None):
        got = self._exchange(copy.deepcopy(obj))
        out[:] = got

    def all_to_all_single(self, output, input, output_split_sizes=None, input_split_sizes=None, group=None):
        import torch
        w = self.world
        ins = list(input_split_sizes) if input_split_sizes is not None else [input.shape[0] // w] * w
        self._sync(input)
        parts = [p.clone() for p in torch.split(input, ins)]
        allparts = self._exchange(parts)
        mine = [allparts[src][self.rank] for src in range(w)]
        if output.numel():
            output.copy_(torch.cat(mine))
        self._sync(output)

    def all_reduce(self, tensor, op="sum", group=None):
        import torch
        self._sync(tensor)
        got = self._exchange(tensor.clone())
        out = got[0].clone()
        for t in got[1:]:
            out = torch.maximum(out, t) if op == "max" else out + t
        tensor.copy_(out)
        self._sync(tensor)
