"""One decode of the full-size config-C workload (bench.py's) per MDSX_TUNE variant, checked
against its sources -- run as its own process per variant (a fault names its variant).

    python scripts/swave_check.py "swave=1"
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    tune = sys.argv[1] if len(sys.argv) > 1 else ''
    os.environ['MDSX_TUNE'] = tune
    import torch
    import bench
    from streaming_amd import _native
    from streaming_amd.decoder import BatchDecoder
    torch.cuda.set_device(0)
    synth, _ = bench.build_workload('C', list(range(bench.SHARDS_PER_GPU['C'])))
    dec = BatchDecoder(synth.plan, synth.batch)
    for _ in range(2):
        out = dec.run()
        dec.check()
        bench.verify('C', out, synth.sources)
    print(f'swave_check {tune!r}: OK ({_native.last_kernel()})', flush=True)


if __name__ == '__main__':
    main()
