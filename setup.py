"""Install ``distributed_kfac_pytorch_amd`` (reference ``setup.py`` /
``setup.cfg``).

The HIP extension is compiled for gfx950 by ``tools/build_native.py``
(hipcc directly, no JIT) as part of ``build_py``, so both
``pip install .`` and ``python setup.py build_ext --inplace`` /
``python tools/build_native.py`` produce ``distributed_kfac_pytorch_amd/_C*.so``.
Set ``KFAC_SKIP_NATIVE_BUILD=1`` to install the pure-Python parts only
(CPU / gloo use).
"""
from __future__ import annotations

import os
import shutil
import sys

from setuptools import Command
from setuptools import find_packages
from setuptools import setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))


def _build_native() -> str | None:
    if os.environ.get('KFAC_SKIP_NATIVE_BUILD') == '1':
        return None
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import build_native  # type: ignore[import-not-found]
    return build_native.build(jobs=int(os.environ.get('MAX_JOBS', '8')))


class BuildPyWithNative(build_py):
    def run(self) -> None:
        so = _build_native()
        super().run()
        if so is not None and not self.dry_run:
            dst = os.path.join(self.build_lib, 'distributed_kfac_pytorch_amd')
            os.makedirs(dst, exist_ok=True)
            shutil.copy2(so, dst)


class BuildExtInplace(Command):
    """``python setup.py build_ext --inplace``: build the in-tree .so."""

    user_options = [('inplace', 'i', 'ignored (always in place)')]

    def initialize_options(self) -> None:
        self.inplace = True

    def finalize_options(self) -> None:
        pass

    def run(self) -> None:
        print(_build_native())


setup(
    name='distributed-kfac-pytorch-amd',
    version='0.4.1+mi355x.1',
    description='MI355X-native distributed K-FAC / KAISA preconditioner for PyTorch-ROCm',
    long_description=open(os.path.join(ROOT, 'README.md'), encoding='utf-8').read(),
    long_description_content_type='text/markdown',
    python_requires='>=3.9',
    packages=find_packages(include=['distributed_kfac_pytorch_amd*']),
    install_requires=['torch>=2.1', 'numpy'],
    extras_require={'examples': ['tqdm', 'pillow'], 'dev': ['pytest', 'pytest-timeout']},
    package_data={'distributed_kfac_pytorch_amd': ['*.so', 'py.typed']},
    cmdclass={'build_py': BuildPyWithNative, 'build_ext': BuildExtInplace},
    zip_safe=False,
)
