"""Malformed-shard fixtures: what the REAL reference's per-sample reader returns, sample by
sample, on MDS shards that break its layout (run in the build container, offline, against
/root/reference; the outputs under tests/golden/malformed/ are committed, the reference is not).

The reference reads a sample as ``data = fp.read(end - begin)`` from its offsets pair
(streaming/base/format/mds/reader.py:128-149) and slices every column out of ``data``
(mds/reader.py:103-126): it never checks a size head against the sample, so a head larger than the
sample, a sample shorter than its fixed columns, or a last offset past the end of the file give
shorter slices -- values or the column decoder's exception -- never a layout error. Cases (shards
written by the reference MDSWriter, then edited):

* ``head_over``       -- a bytes column's u32 head set far past its sample;
* ``head_over_last``  -- the last ragged column's head a few bytes past its sample;
* ``cut_str``         -- a sample's end moved 1 byte back (a 2-byte UTF-8 sequence cut; the next
                         sample starts 1 byte early);
* ``junk_after``      -- 7 junk bytes between two samples (later offsets moved);
* ``last_past_file``  -- the last offset 100 bytes past the end of the file;
* ``file_cut``        -- the file's last 3 bytes cut off (the last offset unchanged);
* ``short_heads``     -- a 6-byte sample (its second size head cut short);
* ``empty``           -- an empty sample (end == begin);
* ``end_before_begin``-- an offsets pair with end < begin (read(end - begin) wraps: to EOF);
* ``fixed_short``     -- an all-fixed schema, a sample two bytes short (a static ndarray cut);
* ``scalar_short``    -- {uint16, int}: samples cut to 1, 2 and 8 bytes.

Output: tests/golden/malformed/<case>/ (index.json + the edited shard) and outcomes.json:
{case: [per sample: {"value": {column: value record}} or {"exc": type name, "msg": text}]}.

    python tests/golden/make_malformed.py [--reference /root/reference]
"""

import argparse
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, 'malformed')
sys.path.insert(0, HERE)

from make_golden import boot_reference, value_record  # noqa: E402


def _offsets(raw: bytes) -> np.ndarray:
    n = int(np.frombuffer(raw[:4], np.uint32)[0])
    return np.frombuffer(raw[4:4 + 4 * (n + 1)], np.uint32).astype(np.int64)


def _with_offsets(raw: bytes, offs) -> bytes:
    n = int(np.frombuffer(raw[:4], np.uint32)[0])
    return raw[:4] + np.asarray(offs, np.uint32).tobytes() + raw[4 + 4 * (n + 1):]


def _insert(raw: bytes, at: int, junk: bytes, after_sample: int) -> bytes:
    offs = _offsets(raw)
    offs[after_sample + 1:] += len(junk)
    body = raw[:at] + junk + raw[at:]
    return _with_offsets(body, offs)


def _set_u32(raw: bytes, at: int, value: int) -> bytes:
    return raw[:at] + np.uint32(value).tobytes() + raw[at + 4:]


SCHEMA_A = {'a': 'bytes', 'n': 'int', 's': 'str'}  # columns a, n, s; heads of a and s


def _samples_a():
    return [{'a': bytes(range(i, i + 5 + 3 * i)), 'n': 1000 * i - 7, 's': 'zé€' * (i + 1)}
            for i in range(6)]


def _edits():
    """case -> (schema, samples, edit(raw bytes) -> edited raw bytes)."""

    def head_over(raw):
        return _set_u32(raw, int(_offsets(raw)[1]), 0x7FFFFFFF)  # sample 1, head of `a`

    def head_over_last(raw):
        b = int(_offsets(raw)[2])
        s_len = int(np.frombuffer(raw[b + 4:b + 8], np.uint32)[0])
        return _set_u32(raw, b + 4, s_len + 5)  # sample 2, head of `s`

    def cut_str(raw):
        offs = _offsets(raw)
        offs[3] -= 1  # sample 2 ends inside its last euro sign
        return _with_offsets(raw, offs)

    def junk_after(raw):
        offs = _offsets(raw)
        return _insert(raw, int(offs[4]), b'JUNK!!!', 3)

    def last_past_file(raw):
        offs = _offsets(raw)
        offs[-1] += 100
        return _with_offsets(raw, offs)

    def file_cut(raw):
        return raw[:-3]

    def short_heads(raw):
        offs = _offsets(raw)
        offs[5] = offs[4] + 6  # sample 4: 6 bytes (the `s` head cut short)
        return _with_offsets(raw, offs)

    def empty(raw):
        offs = _offsets(raw)
        offs[2] = offs[1]  # sample 1 empty; sample 2 spans samples 1 and 2
        return _with_offsets(raw, offs)

    def end_before_begin(raw):
        offs = _offsets(raw)
        offs[3] = offs[2] - 10  # sample 2: end < begin; sample 3 starts 10 bytes early
        return _with_offsets(raw, offs)

    def fixed_short(raw):
        offs = _offsets(raw)
        offs[2] -= 2  # sample 1: 18 of its 20 bytes
        return _with_offsets(raw, offs)

    def scalar_short(raw):
        offs = _offsets(raw)
        offs[2] = offs[1] + 1  # sample 1: 1 byte (the uint16 cut)
        offs[4] = offs[3] + 2  # sample 3: 2 bytes (the int empty)
        offs[6] = offs[5] + 8  # sample 5: 8 bytes (the int cut to 6)
        return _with_offsets(raw, offs)

    fixed = {'id': 'int32', 'x': 'ndarray:float32:4'}
    fixed_rows = [{'id': np.int32(i * 3 - 1), 'x': np.arange(4, dtype=np.float32) * (i + 0.5)}
                  for i in range(5)]
    scal = {'a': 'uint16', 'b': 'int'}
    scal_rows = [{'a': np.uint16(i * 1000 + 1), 'b': -(10**12) * i + 5} for i in range(8)]
    a = (SCHEMA_A, _samples_a)
    return {
        'head_over': (*a, head_over),
        'head_over_last': (*a, head_over_last),
        'cut_str': (*a, cut_str),
        'junk_after': (*a, junk_after),
        'last_past_file': (*a, last_past_file),
        'file_cut': (*a, file_cut),
        'short_heads': (*a, short_heads),
        'empty': (*a, empty),
        'end_before_begin': (*a, end_before_begin),
        'fixed_short': (fixed, lambda: fixed_rows, fixed_short),
        'scalar_short': (scal, lambda: scal_rows, scalar_short),
    }


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--reference', default='/root/reference')
    args = ap.parse_args()
    MDSWriter, reader_from_json, _ = boot_reference(args.reference)
    import warnings
    warnings.simplefilter('ignore')  # numpy's uint32 wrap in end - begin (end_before_begin)
    shutil.rmtree(OUT, ignore_errors=True)
    outcomes = {}
    for case, (cols, rows, edit) in _edits().items():
        d = os.path.join(OUT, case)
        with MDSWriter(columns=cols, out=d) as w:
            for r in rows():
                w.write(r)
        index = json.load(open(os.path.join(d, 'index.json')))
        assert len(index['shards']) == 1
        info = index['shards'][0]
        path = os.path.join(d, info['raw_data']['basename'])
        raw = edit(open(path, 'rb').read())
        with open(path, 'wb') as f:
            f.write(raw)
        info['raw_data']['bytes'] = len(raw)
        with open(os.path.join(d, 'index.json'), 'w') as f:
            json.dump(index, f, indent=1, sort_keys=True)
        reader = reader_from_json(d, None, info)
        per = []
        for i in range(info['samples']):
            try:
                sample = reader[i]
                per.append({'value': {k: value_record(v) for k, v in sample.items()}})
            except Exception as e:  # noqa: BLE001 -- the outcome IS the exception
                per.append({'exc': type(e).__name__, 'msg': str(e)})
        del reader
        outcomes[case] = per
        print(case, [p.get('exc', 'value') for p in per], flush=True)
    with open(os.path.join(OUT, 'outcomes.json'), 'w') as f:
        json.dump(outcomes, f, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
