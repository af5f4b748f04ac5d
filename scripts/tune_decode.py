"""A/B the decode kernel's tuning knobs in ONE process on one GPU (interleaved rounds).

    python scripts/tune_decode.py --config B --variants "tile=256" "tile=64" "unroll=8,nt=1"

Each variant builds its own plan (MDSX_TUNE is read at plan creation) over the SAME resident
shard batch (tile tables rebuilt for its tile size), is verified bit-exact, then all variants are
timed round-robin for --rounds rounds with HIP events around the scan + decode kernels (a
variant holding 'single' runs the single-pass decode). Also times a
torch device-to-device copy of the shard bytes (the measured HBM copy ceiling on this box).
"""

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from streaming_amd.decoder import (BatchDecoder, DeviceBatch, Plan, ScanAheadDecoder,  # noqa
                                   _tables, output_bytes)
from streaming_amd.synth import fixed_b_batch_on_device, var_c_batch_on_device  # noqa


def retile(batch: DeviceBatch, plan: Plan) -> DeviceBatch:
    tr = plan.tile_rows_for(int(batch.buffer.numel()), batch.total_rows)
    raw, tile_shard, row0, rows, tiles = _tables(batch.sizes, batch.samples, batch.offsets, tr)
    dev = batch.device
    return DeviceBatch(batch.buffer, torch.from_numpy(raw).to(dev),
                       torch.from_numpy(tile_shard).to(dev), batch.offsets, batch.sizes,
                       batch.samples, row0, tiles, rows, tr)


def src_abs_offset(nvar: int, ntiles: int, nbytes: int) -> int:
    """Workspace byte offset of the src_abs region (mdsx_kernels.hip workspace_layout)."""
    r256 = lambda x: (x + 255) // 256 * 256  # noqa: E731
    tile_prefix = 256 + r256(nvar * ntiles * 8)
    chunk_sum = tile_prefix + r256(nvar * ntiles * 8)
    tile_run = chunk_sum + r256(nvar * (ntiles // (256 * 16) + 1) * 8)
    return tile_run + r256(ntiles * 48 if nvar else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='B')
    ap.add_argument('--samples', type=int, default=1_000_000, help='config B samples')
    ap.add_argument('--shards', type=int, default=64, help='config C: full 64 MiB shards')
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--variants', nargs='+', default=['tile=256'])
    ap.add_argument('--blob', default='3072,5120', help="config C 'b' byte-length range")
    ap.add_argument('--chars', default='16,256', help="config C 's' code-point range")
    ap.add_argument('--str-widths', type=int, default=4,
                    help="config C 's': code points of 1..N UTF-8 bytes (1: ASCII text)")
    ap.add_argument('--own-outputs', action='store_true',
                    help='each variant allocates its own outputs (the round-2 harness)')
    args = ap.parse_args()
    torch.cuda.set_device(0)
    if args.config == 'B':
        synth = fixed_b_batch_on_device(args.samples, seed=3)
        base_batch, names = synth.batch, (['id', 'x'], ['int32', 'ndarray:float32:1024'],
                                           [4, 4096])
        src = synth.sources
    else:
        blob = tuple(int(x) for x in args.blob.split(','))
        chars = tuple(int(x) for x in args.chars.split(','))
        synth = var_c_batch_on_device(list(range(args.shards)), seed=4, str_chars=chars,
                                      blob_bytes=blob, str_widths=args.str_widths)
        names = (['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None])
        base_batch, src = synth.batch, synth.sources
    decs = {}
    shared = None  # the output buffers every two-pass variant writes (placement held fixed)
    for v in args.variants:
        # 'enc=a|b|c' overrides the column encodings (e.g. read a str column as bytes)
        # 'single' runs the single-pass decode (mdsx_decode_shards_single) for that variant
        # '#tag' makes a repeated variant distinct (an identical control)
        spec = v.split('#')[0].split(',')
        knobs = [kv for kv in spec if kv and not kv.startswith('enc=') and kv not in
                 ('single', 'nocheck', 'ahead', 'ahead_hi')]
        encs = [kv[4:].split('|') for kv in spec if kv.startswith('enc=')]
        os.environ['MDSX_TUNE'] = ','.join(knobs)
        plan = Plan(names[0], encs[0] if encs else names[1], names[2])
        single = 'single' in spec
        dec = BatchDecoder(plan, retile(base_batch, plan), single=single)
        if not single and not encs and not args.own_outputs:
            # identical decoders with their own outputs measured ~5 % apart (output placement):
            # every variant writes the same buffers, so only the kernels differ
            if shared is None:
                shared = (dec.outputs, dec._fixed_raw)
            else:
                dec.outputs, dec._fixed_raw = shared
        decs[v] = dec
        if 'ahead' in spec or 'ahead_hi' in spec:  # the next step's scan on a side stream
            dec.run()
            dec.check()
            sad = ScanAheadDecoder(plan, dec.batch, capacities=dec.capacities,
                                   priority=-1 if 'ahead_hi' in spec else 0)
            sad.outputs_owner = dec  # (keeps the sizing decoder's buffers alive)
            decs[v] = sad
        if 'nocheck' in spec:  # measurement-only variants (e.g. parts skipped)
            dec.run()
            continue
        # the first run (scan + sizing) and a re-run (known totals) against the sources
        for _ in range(2):
            dec = decs[v]
            out = dec.run(ahead=False) if isinstance(dec, ScanAheadDecoder) else dec.run()
            dec.check()
            if args.config == 'B':
                assert torch.equal(out['x'].view(torch.int32), src['x'].view(torch.int32)), v
                assert torch.equal(out['id'], src['id']), v
            else:
                for name in ('b', 's'):
                    assert torch.equal(out[name].values, src[name].values), (v, name)
                    assert torch.equal(out[name].offsets, src[name].offsets), (v, name)
                if out['s'].flags is not None:
                    assert int(out['s'].flags.sum()) == 0, v
                assert torch.equal(out['n'], src['n']), v
    R = base_batch.shard_bytes
    W = output_bytes(decs[args.variants[0]].plan, decs[args.variants[0]].result())
    copy_dst = torch.empty_like(base_batch.buffer)
    times = {v: [] for v in args.variants}
    dtimes = {v: [] for v in args.variants}  # the decode launch alone (after the scan pass)
    times['torch_copy'] = []
    pe = os.environ.get('MDSX_PROBES', '')  # '1': shapes 0-4; or a list of shapes, '1,5,7,8'
    probes = [int(x) for x in pe.split(',')] if ',' in pe else [0, 1, 2, 3, 4] if pe else []
    times['mdsx_copy_probe'] = []
    for pv in probes:
        times[f'probe{pv}'] = []
    from streaming_amd import _native
    lib = _native.lib()
    nprobe = (base_batch.buffer.numel() // 16) * 16
    for rnd in range(args.rounds):
        # the variants' order rotates every round: a variant's rate depends on its position in a
        # round (the GPU's state after the previous one), so each one takes every position
        order = list(decs.items())
        order = order[rnd % len(order):] + order[:rnd % len(order)]
        for v, dec in order:
            if isinstance(dec, ScanAheadDecoder):  # whole-span time of the pipelined steps
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for k in range(args.iters):
                    dec.run(ahead=k + 1 < args.iters)
                e.record()
                torch.cuda.synchronize()
                times[v].append(s.elapsed_time(e) / args.iters)
                continue
            evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)]
                   for _ in range(args.iters)]
            for e in evs:
                dec.run(e)
            torch.cuda.synchronize()
            times[v].extend(e[0].elapsed_time(e[2]) for e in evs)  # scan (if any) + decode
            dtimes[v].extend(e[1].elapsed_time(e[2]) for e in evs)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(args.iters):
            copy_dst.copy_(base_batch.buffer)
        e.record()
        torch.cuda.synchronize()
        times['torch_copy'].append(s.elapsed_time(e) / args.iters)
        stream = torch.cuda.current_stream().cuda_stream
        s.record()
        for _ in range(args.iters):
            lib.mdsx_copy_probe(base_batch.buffer.data_ptr(), copy_dst.data_ptr(), nprobe, stream)
        e.record()
        torch.cuda.synchronize()
        times['mdsx_copy_probe'].append(s.elapsed_time(e) / args.iters)
        for pv in probes:
            s.record()
            for _ in range(args.iters):
                lib.mdsx_copy_probe_variant(base_batch.buffer.data_ptr(), copy_dst.data_ptr(),
                                            nprobe, pv, stream)
            e.record()
            torch.cuda.synchronize()
            times[f'probe{pv}'].append(s.elapsed_time(e) / args.iters)
    phases = {}
    for v, dec in decs.items():  # sdbg bit 16: the staged decode's cycles per phase, per tile
        dbg = [int(kv[5:], 0) for kv in v.split('#')[0].split(',') if kv.startswith('sdbg=')]
        swx = [int(kv[4:], 0) for kv in v.split('#')[0].split(',') if kv.startswith('swx=')]
        if swx and swx[0] & 8:  # one sample per wave: per-wave stamps (mdsx_swave.hip kX 8)
            dec.run()
            torch.cuda.synchronize()
            ntile = int(dec.batch.tile_shard.numel())
            rows = dec.batch.total_rows
            off = src_abs_offset(dec.plan.num_var, ntile, int(dec.batch.buffer.numel()))
            raw = dec.workspace[off:off + 16 * rows].cpu().view(torch.int32).view(rows, 4)
            raw = raw.double()
            names = ['offsets_pair_in', 'loads_landed', 'stores_issued', 'wave_end']
            phases[v] = dict(zip(names, [round(x) for x in raw.mean(dim=0).tolist()]))
            phases[v]['median'] = [round(x) for x in raw.median(dim=0).values.tolist()]
            phases[v]['p90'] = [round(x) for x in raw.quantile(0.9, dim=0).tolist()]
            phases[v]['waves'] = rows
        elif dbg and dbg[0] & 64 and 'run=' in v:  # the lean streaming decode's wave stamps
            dec.run()
            torch.cuda.synchronize()
            ntile = int(dec.batch.tile_shard.numel())
            off = src_abs_offset(dec.plan.num_var, ntile, int(dec.batch.buffer.numel()))
            raw = dec.workspace[off:off + 24 * ntile].cpu().view(torch.int64).view(ntile, 3)
            raw = raw.double()
            phases[v] = dict(zip(['first_sample_landed', 'later_ring_waits', 'wave_total'],
                                 [round(x) for x in raw.mean(dim=0).tolist()]))
            phases[v]['median'] = [round(x) for x in raw.median(dim=0).values.tolist()]
            phases[v]['waves'] = ntile
        elif dbg and dbg[0] & 64:  # the row-parallel decode's phase stamps (mdsx_rows.hip)
            dec.run()
            torch.cuda.synchronize()
            ntile = int(dec.batch.tile_shard.numel())
            off = src_abs_offset(dec.plan.num_var, ntile, int(dec.batch.buffer.numel()))
            raw = dec.workspace[off:off + 64 * ntile].cpu().view(torch.int64).view(ntile, 8)[:, :7]
            med = raw.double().median(dim=0).values.tolist()
            phases[v] = dict(zip(['dma_wait', 'heads_bounds', 'value_records',
                                  'scan_offsets_maps', 'geometry_barrier', 'write', 'flags'],
                                 [round(x) for x in raw.double().mean(dim=0).tolist()]))
            phases[v]['median'] = [round(x) for x in med]
            phases[v]['tiles'] = ntile
            phases[v]['rows_per_tile'] = dec.batch.tile_rows
        elif dbg and dbg[0] & 16:
            dec.run()
            torch.cuda.synchronize()
            raw = dec.workspace[200:256].cpu().view(torch.int64).tolist()
            nt = int(dec.batch.tile_shard.numel())
            if 'run=' in v:  # streaming decode: per-wave (tile) ring-wait and total cycles
                phases[v] = {'ring_wait': round(raw[0] / max(raw[2], 1)),
                             'total': round(raw[1] / max(raw[2], 1)), 'waves': raw[2],
                             'rows_per_tile': dec.batch.tile_rows}
            else:
                phases[v] = dict(zip(['loader_wait', 'rows', 'offsets', 'place', 'write', 'utf8',
                                      'end_barrier'], [round(x / nt) for x in raw]))
    res = {}
    for v, ts in times.items():
        ms = float(np.median(ts))
        nbytes = 2 * base_batch.buffer.numel() if v in ('torch_copy', 'mdsx_copy_probe') or \
            v.startswith('probe') else R + W
        res[v] = {'median_ms': ms, 'min_ms': float(np.min(ts)), 'GBps': nbytes / ms / 1e6}
        if dtimes.get(v):
            dms = float(np.median(dtimes[v]))
            res[v].update(decode_ms=dms, decode_GBps=nbytes / dms / 1e6)
    print(json.dumps({'config': args.config, 'blob': args.blob, 'chars': args.chars, 'R': R,
                      'W': W, 'rows': base_batch.total_rows, 'results': res,
                      'phase_cycles_per_tile': phases}, indent=1))


if __name__ == '__main__':
    main()
