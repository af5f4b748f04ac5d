"""Build libmdsx.so for gfx950 in-tree (``python -m streaming_amd.build``).

One hipcc invocation over the HIP kernels and the host plan builder; the output lands in
``streaming_amd/lib/`` so it travels with the repository snapshot to the GPU box.
"""

from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SOURCES = [
    os.path.join(HERE, 'csrc', name)
    for name in ('mdsx_kernels.hip', 'mdsx_stage.hip', 'mdsx_run.hip', 'mdsx_rows.hip', 'mdsx_encode.hip', 'mdsx_hash.hip',
                 'mdsx_plan.cpp')
]
HEADERS = [os.path.join(HERE, 'csrc', name)
           for name in ('mdsx_internal.h', 'mdsx_device.h', 'mdsx_decode.h')]
OUTPUT = os.path.join(HERE, 'lib', 'libmdsx.so')
ARCH = os.environ.get('MDSX_OFFLOAD_ARCH', 'gfx950')


def hipcc() -> str:
    rocm = os.environ.get('ROCM_PATH', '/opt/rocm')
    path = os.path.join(rocm, 'bin', 'hipcc')
    return path if os.path.exists(path) else 'hipcc'


FLAGS = ['-O3', '-std=c++17', '-fPIC', '-Wall', '-Wno-unused-function', '--no-offload-compress']


def command(output: str = OUTPUT, extra: tuple = ()) -> list[str]:
    """One hipcc invocation building the whole library (compile + link)."""
    return [
        hipcc(), f'--offload-arch={ARCH}', *FLAGS, '-shared', '-I', os.path.join(ROOT, 'include'),
        '-o', output, *extra, *SOURCES
    ]


def _compile(src: str, obj: str, verbose: bool) -> None:
    cmd = [hipcc(), f'--offload-arch={ARCH}', *FLAGS, '-I', os.path.join(ROOT, 'include'), '-c',
           src, '-o', obj]
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile every source to an object in parallel, then link libmdsx.so (in-tree)."""
    os.makedirs(os.path.dirname(OUTPUT), exist_ok=True)
    if not force and os.path.exists(OUTPUT):
        newest = max(os.path.getmtime(p) for p in SOURCES + HEADERS + [
            os.path.join(ROOT, 'include', 'mdsx.h')
        ])
        if os.path.getmtime(OUTPUT) >= newest:
            return OUTPUT
    objdir = os.path.join(HERE, 'build')
    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, os.path.basename(s) + '.o') for s in SOURCES]
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=max(1, min(len(SOURCES), os.cpu_count() or 1))) as pool:
        for f in [pool.submit(_compile, s, o, verbose) for s, o in zip(SOURCES, objs)]:
            f.result()
    tmp = OUTPUT + '.tmp'
    cmd = [hipcc(), f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', tmp, *objs]
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUTPUT)
    return OUTPUT


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose=True))
