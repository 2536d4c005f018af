"""Parallelism: synchronous RCCL data parallel (allreduce) and async parameter server (ps)."""
from .allreduce import GradAllReduce, broadcast_variables
from .launch import init_distributed, local_rank, rank, world_size

__all__ = ["GradAllReduce", "broadcast_variables", "init_distributed", "local_rank", "rank", "world_size"]
