cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r02o && export TMPDIR=/tmp
V="tile=16 run=8 run=8,sdbg=16 run=8,sdbg=1,nocheck run=8,sdbg=2,nocheck run=8,sdbg=3,nocheck run=8,sdbg=4,nocheck run=8,sdbg=8,nocheck run=8,sdbg=12,nocheck"
for cfg in "C" "C --blob 32,256 --chars 8,64"; do
timeout -k 10 300 python3 scripts/tune_decode.py --config $cfg --shards 16 --rounds 3 --variants $V > gpurun_out/r02o/t.json 2> gpurun_out/r02o/t.err || { tail -30 gpurun_out/r02o/t.err; exit 1; }
python3 -c "
import json; d = json.load(open('gpurun_out/r02o/t.json'))
for k, v in d['results'].items(): print('%-28s %8.3f ms %6d GB/s' % (k, v['median_ms'], v['GBps']))
print(d['phase_cycles_per_tile'])"
done
