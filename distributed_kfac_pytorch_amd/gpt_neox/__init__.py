"""Reference-path alias: ``kfac.gpt_neox`` -> ``distributed_kfac_pytorch_amd.neox``."""
from distributed_kfac_pytorch_amd.neox import *  # noqa: F401,F403
from distributed_kfac_pytorch_amd.neox import assignment  # noqa: F401
from distributed_kfac_pytorch_amd.neox import layer  # noqa: F401
from distributed_kfac_pytorch_amd.neox import modules  # noqa: F401
from distributed_kfac_pytorch_amd.neox import mpu  # noqa: F401
from distributed_kfac_pytorch_amd.neox import preconditioner  # noqa: F401
