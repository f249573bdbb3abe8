"""Build the in-tree HIP extension ``distributed_kfac_pytorch_amd/_C*.so``.

Drives ``hipcc --offload-arch=gfx950`` directly (no hipify, no JIT cache):
every ``csrc/*.hip`` kernel file is compiled to an object, the
``csrc/*.cpp`` host files (bindings, rocSOLVER tier -- the only torch-aware
translation units) are compiled against the installed PyTorch-ROCm headers,
and everything is linked into one shared object next to the Python package
so it travels with the repo snapshot to the GPU box.

Usage:  python tools/build_native.py [--force] [--jobs N] [--verbose]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'csrc')
PKG = os.path.join(ROOT, 'distributed_kfac_pytorch_amd')
BUILD = os.path.join(ROOT, 'build', 'native')
ARCH = os.environ.get('KFAC_OFFLOAD_ARCH', 'gfx950')


def _hipcc() -> str:
    rocm = os.environ.get('ROCM_PATH', '/opt/rocm')
    return os.path.join(rocm, 'bin', 'hipcc')


def _torch_paths() -> tuple[list[str], list[str], bool]:
    import torch
    from torch.utils import cpp_extension

    incs = cpp_extension.include_paths(device_type='cuda')
    libdir = os.path.join(os.path.dirname(torch.__file__), 'lib')
    abi = bool(torch._C._GLIBCXX_USE_CXX11_ABI)
    return incs, [libdir], abi


def ext_suffix() -> str:
    return sysconfig.get_config_var('EXT_SUFFIX') or '.so'


def target_path() -> str:
    return os.path.join(PKG, '_C' + ext_suffix())


def _newer(src_files: list[str], out: str) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in src_files)


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(' '.join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f'command failed: {" ".join(cmd[:3])} ...')
    if verbose and (r.stdout or r.stderr):
        sys.stderr.write(r.stdout + r.stderr)


def build(force: bool = False, jobs: int = 8, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    hipcc = _hipcc()
    incs, libdirs, abi = _torch_paths()
    header_deps = [
        os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith('.h')
    ]
    common = [
        f'--offload-arch={ARCH}',
        '-O3',
        '-fPIC',
        '-std=c++17',
        '-D__HIP_PLATFORM_AMD__=1',
        '-DUSE_ROCM=1',
        f'-D_GLIBCXX_USE_CXX11_ABI={int(abi)}',
        f'-I{CSRC}',
    ]
    kernel_srcs = sorted(
        os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith('.hip')
    )
    jobs_list = []
    objs = []
    for src in kernel_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + '.o')
        objs.append(obj)
        if force or _newer([src] + header_deps, obj):
            jobs_list.append([hipcc, *common, '-c', src, '-o', obj])
    py_inc = sysconfig.get_paths()['include']
    torch_srcs = sorted(
        os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith('.cpp')
    )
    for src in torch_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + '.o')
        objs.append(obj)
        if force or _newer([src] + header_deps, obj):
            jobs_list.append(
                [
                    hipcc,
                    *common,
                    '-DTORCH_EXTENSION_NAME=_C',
                    '-DTORCH_API_INCLUDE_EXTENSION_H',
                    '-Wno-unused-result',
                    '-Wno-deprecated-declarations',
                    *[f'-I{p}' for p in incs],
                    f'-I{py_inc}',
                    '-c',
                    src,
                    '-o',
                    obj,
                ],
            )
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = [ex.submit(_run, cmd, verbose) for cmd in jobs_list]
        for f in futs:
            f.result()
    out = target_path()
    if force or jobs_list or not os.path.exists(out):
        link = [
            hipcc,
            f'--offload-arch={ARCH}',
            '-shared',
            '-fPIC',
            *objs,
            '-o',
            out,
            *[f'-L{d}' for d in libdirs],
            *[f'-Wl,-rpath,{d}' for d in libdirs],
            '-lc10',
            '-lc10_hip',
            '-ltorch',
            '-ltorch_cpu',
            '-ltorch_hip',
            '-ltorch_python',
            '-lamdhip64',
            '-L/opt/rocm/lib',
            '-Wl,-rpath,/opt/rocm/lib',
            '-lrocsolver',
            '-lrocblas',
        ]
        _run(link, verbose)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--force', action='store_true')
    ap.add_argument('--jobs', type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument('--verbose', action='store_true')
    args = ap.parse_args()
    print(build(args.force, args.jobs, args.verbose))


if __name__ == '__main__':
    main()
