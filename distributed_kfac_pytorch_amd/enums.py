"""Option enums (API parity with reference ``kfac/enums.py:7-53``)."""
from __future__ import annotations

import enum


class AllreduceMethod(enum.Enum):
    """How factor all-reduces are issued.

    ALLREDUCE issues one collective per factor; ALLREDUCE_BUCKETED packs
    factors into flat buckets of at most ``allreduce_bucket_cap_mb``.
    """

    ALLREDUCE = 1
    ALLREDUCE_BUCKETED = 2


class AssignmentStrategy(enum.Enum):
    """Cost model used to load-balance second-order work across ranks.

    COMPUTE prices a factor of dimension n at n**3 (eigendecomposition /
    inversion flops); MEMORY at n**2 (bytes held by the inverse worker).
    """

    COMPUTE = 1
    MEMORY = 2


class ComputeMethod(enum.Enum):
    """Second-order method: eigendecomposition or damped explicit inverse."""

    EIGEN = 1
    INVERSE = 2


class DistributedStrategy(enum.Enum):
    """KAISA presets for the gradient worker fraction.

    COMM_OPT: every rank preconditions every layer (fraction 1).
    MEM_OPT: one grad worker per layer (fraction 1/world).
    HYBRID_OPT: half of the ranks per layer (fraction 0.5).
    """

    COMM_OPT = 1
    MEM_OPT = 2
    HYBRID_OPT = 3
