"""Measurement: the next step's scan pass on a few reserved CUs beside this step's decode on the
others (HIP CU-masked streams, hipExtStreamCreateWithCUMask), against the one-stream step and the
unmasked scan-ahead (ScanAheadDecoder), config C and short rows. The side-stream scan without
masks waits for the decode's workgroups to retire (profiles/r05/scan_ahead/); with its own CUs it
should run beside the decode, at the cost of those CUs for the decode.

    python scripts/cu_mask_ahead.py [--config C|short] [--cus 8,16,32]
"""

import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from streaming_amd.decoder import BatchDecoder, Plan, RaggedColumn, ScanAheadDecoder  # noqa: E402
from streaming_amd.synth import var_c_batch_on_device  # noqa: E402


def masked_stream(hip, cus, ncu):
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in cus:
        mask[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise RuntimeError(f'hipExtStreamCreateWithCUMask: {rc}')
    return torch.cuda.ExternalStream(s.value)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='C')
    ap.add_argument('--cus', default='8,16,32')
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--rounds', type=int, default=3)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    hip = ctypes.CDLL('libamdhip64.so')
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    if args.config == 'C':
        synth = var_c_batch_on_device(list(range(64)), seed=4)
    else:
        synth = var_c_batch_on_device(list(range(16)), seed=4, str_chars=(8, 64),
                                      blob_bytes=(32, 256))
    plan = Plan(['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None])
    base = BatchDecoder(plan, synth.batch)
    want = base.run()
    base.check()
    want = {k: (v.values.clone(), v.offsets.clone()) if isinstance(v, RaggedColumn) else v.clone()
            for k, v in want.columns.items()}
    caps = base.capacities

    def same(out):
        for k, v in want.items():
            got = out.columns[k]
            if isinstance(v, tuple):
                if not (torch.equal(got.values, v[0]) and torch.equal(got.offsets, v[1])):
                    return False
            elif not torch.equal(got, v):
                return False
        return True

    variants = {'one_stream': None, 'ahead': None}
    for k in [int(x) for x in args.cus.split(',')]:
        variants[f'ahead_cu{k}'] = k
        variants[f'decode_only_cu{k}'] = k
    variants['decode_only'] = 0
    decs, streams = {}, {}
    for name, k in variants.items():
        if name == 'one_stream':
            decs[name] = base
        elif name.startswith('ahead'):
            sad = ScanAheadDecoder(plan, synth.batch, capacities=caps)
            if k:
                # the scan's CUs spread over the XCDs: every (ncu / k)-th CU
                step = ncu // k
                scan_cus = list(range(0, ncu, step))[:k]
                rest = [c for c in range(ncu) if c not in set(scan_cus)]
                sad._side = masked_stream(hip, scan_cus, ncu)
                streams[name] = masked_stream(hip, rest, ncu)
            decs[name] = sad
        else:
            decs[name] = base
            if k:
                step = ncu // k
                scan_cus = set(list(range(0, ncu, step))[:k])
                streams[name] = masked_stream(hip, [c for c in range(ncu) if c not in scan_cus], ncu)
    times = {n: [] for n in variants}
    ok = {}
    for _ in range(args.rounds):
        for name, dec in decs.items():
            st = streams.get(name, torch.cuda.current_stream())
            with torch.cuda.stream(st):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                if name.startswith('decode_only'):
                    dec._scan(st.cuda_stream)
                    s.record()
                    for _ in range(args.iters):
                        dec._decode(st.cuda_stream)
                    e.record()
                elif isinstance(dec, ScanAheadDecoder):
                    dec.run(ahead=True)
                    s.record()
                    for k in range(args.iters):
                        out = dec.run(ahead=k + 1 < args.iters)
                    e.record()
                else:
                    s.record()
                    for _ in range(args.iters):
                        out = dec.run()
                    e.record()
                torch.cuda.synchronize()
                times[name].append(s.elapsed_time(e) / args.iters)
                if not name.startswith('decode_only'):
                    dec.check()
                    ok[name] = same(dec.result())
    res = {n: round(float(np.median(t)), 4) for n, t in times.items()}
    print(json.dumps({'config': args.config, 'cus': ncu, 'ms_per_step': res, 'outputs_equal': ok},
                     indent=1))


if __name__ == '__main__':
    main()
