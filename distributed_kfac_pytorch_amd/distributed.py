"""Reference-path alias: ``kfac.distributed`` -> ``parallel.comm``."""
from distributed_kfac_pytorch_amd.parallel.comm import *  # noqa: F401,F403
from distributed_kfac_pytorch_amd.parallel.comm import AllreduceTensorBucket  # noqa: F401
from distributed_kfac_pytorch_amd.parallel.comm import AsyncTensor  # noqa: F401
from distributed_kfac_pytorch_amd.parallel.comm import fill_triu  # noqa: F401
from distributed_kfac_pytorch_amd.parallel.comm import Future  # noqa: F401
from distributed_kfac_pytorch_amd.parallel.comm import FutureType  # noqa: F401
from distributed_kfac_pytorch_amd.parallel.comm import get_rank  # noqa: F401
from distributed_kfac_pytorch_amd.parallel.comm import get_triu  # noqa: F401
from distributed_kfac_pytorch_amd.parallel.comm import get_world_size  # noqa: F401
from distributed_kfac_pytorch_amd.parallel.comm import NonSquareTensorError  # noqa: F401
from distributed_kfac_pytorch_amd.parallel.comm import TorchDistributedCommunicator  # noqa: F401
