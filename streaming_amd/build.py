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
    for name in ('mdsx_kernels.hip', 'mdsx_encode.hip', 'mdsx_hash.hip', 'mdsx_plan.cpp')
]
HEADERS = [os.path.join(HERE, 'csrc', name) for name in ('mdsx_internal.h', 'mdsx_device.h')]
OUTPUT = os.path.join(HERE, 'lib', 'libmdsx.so')
ARCH = os.environ.get('MDSX_OFFLOAD_ARCH', 'gfx950')


def hipcc() -> str:
    rocm = os.environ.get('ROCM_PATH', '/opt/rocm')
    path = os.path.join(rocm, 'bin', 'hipcc')
    return path if os.path.exists(path) else 'hipcc'


def command(output: str = OUTPUT, extra: tuple = ()) -> list[str]:
    return [
        hipcc(), f'--offload-arch={ARCH}', '-O3', '-std=c++17', '-fPIC', '-shared',
        '-Wall', '-Wno-unused-function', '--no-offload-compress',
        '-I', os.path.join(ROOT, 'include'), '-o', output, *extra, *SOURCES
    ]


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(os.path.dirname(OUTPUT), exist_ok=True)
    if not force and os.path.exists(OUTPUT):
        newest = max(os.path.getmtime(p) for p in SOURCES + HEADERS + [
            os.path.join(ROOT, 'include', 'mdsx.h')
        ])
        if os.path.getmtime(OUTPUT) >= newest:
            return OUTPUT
    tmp = OUTPUT + '.tmp'
    cmd = command(tmp)
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUTPUT)
    return OUTPUT


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose=True))
