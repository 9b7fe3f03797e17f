"""Data parallelism for the train step: one process per GPU, windows sharded by
rows, weights/Adam state replicated, ONE exchange per step = sum all-reduce of
the flat fp32 gradient buffer over RCCL (torch.distributed 'nccl' backend is
RCCL on ROCm; xGMI between the GPUs of a node).  Sum, not mean: the reference
loss is sum-reduced (model_builder.py:42), so the global gradient of the
concatenated batch is the sum of the shard gradients.  BatchNorm statistics
stay per shard (DDP semantics).  The grad buffer is one
contiguous tensor, so the whole exchange is a single large all-reduce (the
shape xGMI rings like)."""
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's env vars.
    Returns (rank, world_size, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend)
    return rank, world, local


class DataParallel:
    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1

    def all_reduce_grads(self, flat_grads):
        if self.world > 1:
            dist.all_reduce(flat_grads, op=dist.ReduceOp.SUM, group=self.group)

    def all_reduce_loss(self, loss):
        if self.world > 1:
            dist.all_reduce(loss, op=dist.ReduceOp.SUM, group=self.group)

    def broadcast_params(self, model, src=0):
        if self.world > 1:
            dist.broadcast(model._native.params, src=src, group=self.group)


def attach_data_parallel(model, group=None):
    """Replicate rank-0 weights and make AutoEncoder.step all-reduce grads."""
    dp = DataParallel(group)
    dp.broadcast_params(model)
    if dp.world > 1:
        model._native.sync_shadow(force=True)
    model.dist = dp if dp.world > 1 else None
    return model
