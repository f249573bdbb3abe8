"""Reference-path alias: ``kfac.assignment`` -> ``parallel.assignment``."""
from distributed_kfac_pytorch_amd.parallel.assignment import KAISAAssignment  # noqa: F401
from distributed_kfac_pytorch_amd.parallel.assignment import WorkAssignment  # noqa: F401
