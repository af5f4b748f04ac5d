"""Build libmdsx.so for gfx950 in-tree (``python -m streaming_amd.build``).

One hipcc invocation over the HIP kernels and the host plan builder; the output lands in
``streaming_amd/lib/`` so it travels with the repository snapshot to the GPU box.
"""

from __future__ import annotations

import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SOURCES = [
    os.path.join(HERE, 'csrc', name)
    for name in ('mdsx_kernels.hip', 'mdsx_stage.hip', 'mdsx_run.hip', 'mdsx_rows.hip', 'mdsx_swave.hip',
                 'mdsx_sample.hip', 'mdsx_encode.hip', 'mdsx_hash.hip', 'mdsx_plan.cpp')
]
HEADERS = [os.path.join(HERE, 'csrc', name)
           for name in ('mdsx_internal.h', 'mdsx_device.h', 'mdsx_decode.h', 'mdsx_ring.h',
                        'mdsx_run_body.h')]
OUTPUT = os.path.join(HERE, 'lib', 'libmdsx.so')
ARCH = os.environ.get('MDSX_OFFLOAD_ARCH', 'gfx950')


def hipcc() -> str:
    rocm = os.environ.get('ROCM_PATH', '/opt/rocm')
    path = os.path.join(rocm, 'bin', 'hipcc')
    return path if os.path.exists(path) else 'hipcc'


FLAGS = ['-O3', '-std=c++17', '-fPIC', '-Wall', '-Wno-unused-function', '--no-offload-compress']


def source_sha() -> str:
    """sha256 (16 hex digits) of every source, header, the target and the flags of the library.

    Compiled into the library (``mdsx_version()``), so a measurement names the code it ran: two
    links of the same sources need not give identical bytes, the same sources give the same code.
    """
    h = hashlib.sha256()
    for path in SOURCES + HEADERS + [os.path.join(ROOT, 'include', 'mdsx.h')]:
        h.update(os.path.basename(path).encode() + b'\0')
        with open(path, 'rb') as f:
            h.update(f.read())
    h.update(' '.join([ARCH, *FLAGS]).encode())
    return h.hexdigest()[:16]


def _defines() -> list[str]:
    return [f'-DMDSX_SOURCE_SHA="{source_sha()}"']


def command(output: str = OUTPUT, extra: tuple = ()) -> list[str]:
    """One hipcc invocation building the whole library (compile + link)."""
    return [
        hipcc(), f'--offload-arch={ARCH}', *FLAGS, *_defines(), '-shared', '-I',
        os.path.join(ROOT, 'include'), '-o', output, *extra, *SOURCES
    ]


def _compile(src: str, obj: str, verbose: bool) -> None:
    defs = _defines() if src.endswith('mdsx_plan.cpp') else []
    cmd = [hipcc(), f'--offload-arch={ARCH}', *FLAGS, *defs, '-I', os.path.join(ROOT, 'include'),
           '-c', src, '-o', obj]
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)


def _compile_device(src: str, obj: str, verbose: bool) -> None:
    """The device code alone (for the ISA check below)."""
    cmd = [hipcc(), f'--offload-arch={ARCH}', *FLAGS, '-I', os.path.join(ROOT, 'include'),
           '--cuda-device-only', '--no-gpu-bundle-output', '-c', src, '-o', obj]
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)


# Kernels whose cross-lane reads the ISA check covers, per source: the row-parallel decode, the
# one-row-per-wave decode of all-fixed plans and the one-sample-per-wave decode of ragged plans
# (each reads registers of a lane chosen at run time: v_readlane with an SGPR lane).
ISA_CHECKED = {
    'mdsx_rows.hip': ('rows_decode_kernel',),
    'mdsx_kernels.hip': ('rowwave_decode_kernel',),
    'mdsx_swave.hip': ('swave_decode_kernel',),
}


def _check_cross_lane_reads(obj: str, want: tuple = ('rows_decode_kernel',)) -> None:
    """Refuse a build whose listed kernels read a register across lanes where the exec mask may
    be partial (streaming_amd/isa_check.py)."""
    from streaming_amd import isa_check
    rocm = os.environ.get('ROCM_PATH', '/opt/rocm')
    text = subprocess.run([os.path.join(rocm, 'lib', 'llvm', 'bin', 'llvm-objdump'), '-d', obj],
                          capture_output=True, text=True, check=True).stdout
    bad = [hit for w in want for hit in isa_check.check(text, w)]
    missing = [w for w in want if not any(w in name for name, _ in isa_check.kernels(text))]
    if missing:
        raise RuntimeError(f'mdsx build: no kernel named {missing} in {obj} for the ISA check')
    if bad:
        raise RuntimeError('mdsx build: cross-lane reads under a possibly partial exec mask in ' +
                           '; '.join(f'{name} (at {", ".join(hex(a) for a in addrs)})'
                                     for name, addrs in bad))


# Kernels that must not spill at all: a VGPR reloaded from scratch under a partial exec mask holds
# stale bits in its inactive lanes, which a later cross-lane read with every lane active returns.
NO_SCRATCH = {'mdsx_swave.hip': ('swave_decode_kernel',)}


def _check_no_scratch(obj: str, want: tuple) -> None:
    rocm = os.environ.get('ROCM_PATH', '/opt/rocm')
    text = subprocess.run([os.path.join(rocm, 'lib', 'llvm', 'bin', 'llvm-readelf'), '--notes',
                           obj], capture_output=True, text=True, check=True).stdout
    name, bad = None, []
    for line in text.splitlines():
        line = line.strip()
        if line.startswith('.name:'):
            name = line.split(':', 1)[1].strip()
        elif line.startswith('.private_segment_fixed_size:') and name and \
                any(w in name for w in want) and int(line.split(':', 1)[1]) != 0:
            bad.append(name)
    if bad:
        raise RuntimeError(f'mdsx build: kernels that must not spill use scratch: {bad}')


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
    devs = {src: os.path.join(objdir, src.replace('.hip', '.device.o')) for src in ISA_CHECKED}
    with ThreadPoolExecutor(max_workers=max(1, min(len(SOURCES) + len(devs),
                                                   os.cpu_count() or 1))) as pool:
        jobs = [pool.submit(_compile, s, o, verbose) for s, o in zip(SOURCES, objs)]
        jobs += [pool.submit(_compile_device, os.path.join(HERE, 'csrc', src), obj, verbose)
                 for src, obj in devs.items()]
        for f in jobs:
            f.result()
    for src, obj in devs.items():
        _check_cross_lane_reads(obj, ISA_CHECKED[src])
        if src in NO_SCRATCH:
            _check_no_scratch(obj, NO_SCRATCH[src])
    tmp = OUTPUT + '.tmp'
    cmd = [hipcc(), f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', tmp, *objs]
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUTPUT)
    return OUTPUT


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose=True))
