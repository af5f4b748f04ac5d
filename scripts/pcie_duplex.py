"""PCIe H2D and D2H rates alone and concurrently (two streams, pinned host buffers): whether the
host hand-off can overlap the next batch's upload. Prints one JSON object."""
import json
import time

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    n = 512 << 20
    h_in = torch.empty(n, dtype=torch.uint8, pin_memory=True).fill_(1)
    h_out = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d_in = torch.empty(n, dtype=torch.uint8, device='cuda')
    d_out = torch.ones(n, dtype=torch.uint8, device='cuda')
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def h2d():
        with torch.cuda.stream(s1):
            d_in.copy_(h_in, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h_out.copy_(d_out, non_blocking=True)

    def both():
        h2d()
        d2h()

    # D2H by a kernel storing straight into the pinned host buffer (mdsx_copy_probe: 16-byte
    # loads and stores, the destination mapped over PCIe), next to the DMA-engine H2D
    from streaming_amd import _native
    lib = _native.lib()

    def d2h_kernel():
        lib.mdsx_copy_probe(d_out.data_ptr(), h_out.data_ptr(), n, s2.cuda_stream)

    def both_kernel():
        h2d()
        d2h_kernel()

    for f in (h2d, d2h, both, d2h_kernel, both_kernel):
        timed(f, 2)
    t_h2d, t_d2h, t_both = timed(h2d), timed(d2h), timed(both)
    t_kd2h, t_kboth = timed(d2h_kernel), timed(both_kernel)
    assert bool((h_out == 1).all())
    print(json.dumps({'bytes': n, 'h2d_GBps': n / t_h2d / 1e9, 'd2h_GBps': n / t_d2h / 1e9,
                      'both_GBps_each': n / t_both / 1e9,
                      'overlap': (t_h2d + t_d2h) / t_both,
                      'd2h_kernel_GBps': n / t_kd2h / 1e9,
                      'both_kernel_d2h_GBps_each': n / t_kboth / 1e9,
                      'overlap_kernel_d2h': (t_h2d + t_kd2h) / t_kboth}))


if __name__ == '__main__':
    main()
