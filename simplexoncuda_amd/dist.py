"""Multi-GPU plumbing: one process per GPU, RCCL communicator owned by the HIP library.

torch.distributed is used only to rendezvous (broadcast the RCCL unique id from rank 0);
every per-pivot collective (tile-winner allgather, pivot-row allreduce) is enqueued by the
library itself on its own stream, with no host synchronisation.
"""
import ctypes

from . import _lib


def init_from_torch(local_rank, force_rccl=False):
    """force_rccl: build the RCCL communicator (and the exchange path) even at world size 1."""
    import torch.distributed as dist

    lib = _lib.load()
    if force_rccl:
        lib.simplex_set_force_exchange(1)
    rank, world = dist.get_rank(), dist.get_world_size()
    size = lib.simplex_dist_unique_id_size()
    uid = b""
    if world > 1 or force_rccl:
        if rank == 0:
            buf = ctypes.create_string_buffer(size)
            lib.simplex_dist_get_unique_id(buf)
            uid = bytes(buf.raw[:size])
        obj = [uid]
        dist.broadcast_object_list(obj, src=0)
        uid = obj[0]
    else:
        uid = bytes(size)
    lib.simplex_dist_init(rank, world, uid, local_rank)
    return rank, world


def finalize():
    _lib.load().simplex_dist_finalize()
