"""Debug: decode a config-A shard whose sample 5 was made empty, per copy mode, and compare every
other row with the oracle (the reference's algorithm on the same corrupt file)."""
import os
import shutil
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import mds_oracle  # noqa: E402
from tests import golden_util as gu  # noqa: E402

MODES = {'default': '', 'gather': 'gmin=1000000000', 'group': 'gmin=0,gmax=1000000000',
         'wave': 'gmin=0,gmax=0,ring=0', 'run': 'run=8'}

d = tempfile.mkdtemp()
shutil.copytree(os.path.join(gu.GOLDEN, 'config_a'), d + '/a')
info = gu.index('config_a')['shards'][0]
path = os.path.join(d, 'a', info['raw_data']['basename'])
k = 5
with open(path, 'r+b') as f:
    f.seek(4 * (1 + k))
    begin = f.read(4)
    f.seek(4 * (2 + k))
    f.write(begin)
data = open(path, 'rb').read()
orc = mds_oracle.OracleMDSReader(os.path.join(d, 'a'), None, info)
want = {}
for i in range(info['samples']):
    try:
        want[i] = orc.get_item(i)
    except IndexError:
        pass
for mode, tune in MODES.items():
    os.environ['MDSX_TUNE'] = tune
    from streaming_amd.decoder import Plan, decode_batch, stage_shards
    plan = Plan(info['column_names'], info['column_encodings'], info['column_sizes'])
    dec = decode_batch(plan, stage_shards([data], [info['samples']], plan), check=False)
    nums = dec['number'].cpu().numpy()
    col = dec['words']
    vals, offs = col.values.cpu().numpy(), col.offsets.cpu().numpy()
    bad = []
    for i, w in want.items():
        got = vals[offs[i]:offs[i + 1]].tobytes()
        if int(nums[i]) != w['number'] or got != w['words'].encode():
            bad.append(i)
    print(mode, 'bad rows', bad[:10], len(bad), 'offs[:10]', offs[:10].tolist(),
          'want lens', [len(want[i]['words'].encode()) if i in want else 0 for i in range(10)],
          flush=True)
