"""Build check (no GPU, run by streaming_amd.build): in the row-parallel decode kernels, no VGPR
read across lanes by `v_readlane_b32 sX, vN, sY` (a lane chosen at run time) comes straight from a
scratch reload. A reload runs under the exec mask of its point in the program and restores only
the active lanes, so a cross-lane read of a spilled register inside divergent code can return
stale bits -- a 64-VGPR build of the row decode faulted that way.
usage: python -m streaming_amd.isa_check <device object or objdump text> [kernel substring]"""
import re
import subprocess
import sys


def kernels(text):
    cur, body = None, []
    for line in text.splitlines():
        m = re.match(r'^[0-9a-f]+ <(.+)>:$', line)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
        elif cur:
            body.append(line.split('//')[0].strip())
    if cur:
        yield cur, body


def vregs(op):
    m = re.match(r'v\[(\d+):(\d+)\]', op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r'v(\d+)$', op)
    return {int(m.group(1))} if m else set()


def check(text, want='rows_decode_kernel'):
    """Variable-lane readlanes whose source VGPR was last written (in program order) by a scratch
    reload."""
    bad = []
    for name, body in kernels(text):
        if want not in name:
            continue
        last = {}  # VGPR -> mnemonic of its most recent writer
        hits = set()
        for ins in body:
            parts = ins.replace(',', ' ').split()
            if not parts:
                continue
            op = parts[0]
            if op == 'v_readlane_b32' and len(parts) >= 4 and parts[3].startswith('s'):
                for r in vregs(parts[2]):
                    if last.get(r, '').startswith(('scratch_load', 'buffer_load')):
                        hits.add(r)
            # writers: vector ALU / loads name their destination first (stores and v_readlane
            # / v_cmp write no VGPR)
            if len(parts) > 1 and (op.startswith(('v_', 'scratch_load', 'buffer_load',
                                                  'global_load', 'ds_read', 'flat_load')) and
                                   not op.startswith(('v_readlane', 'v_readfirstlane', 'v_cmp'))):
                for r in vregs(parts[1]):
                    last[r] = op
        if hits:
            bad.append((name, sorted(hits)))
    return bad


if __name__ == '__main__':
    src = sys.argv[1]
    text = open(src).read() if src.endswith('.s') else subprocess.run(
        ['/opt/rocm/lib/llvm/bin/llvm-objdump', '-d', src], capture_output=True, text=True,
        check=True).stdout
    bad = check(text, sys.argv[2] if len(sys.argv) > 2 else 'rows_decode_kernel')
    for name, regs in bad:
        print(f'{name}: cross-lane source VGPRs reloaded from scratch: {regs}')
    sys.exit(1 if bad else 0)
