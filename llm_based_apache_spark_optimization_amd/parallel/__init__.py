"""Parallelism: tensor parallel (RCCL over xGMI) and data-parallel replica dispatch."""
from .tp import TPGroup, init_distributed, make_replica_groups  # noqa: F401
