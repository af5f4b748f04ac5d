"""Build check (no GPU, run by streaming_amd.build): in the row-parallel decode kernels, no VGPR is
read across lanes by `v_readlane_b32 sX, vN, sY` (a lane chosen at run time) where the exec mask
may be partial.

A VGPR's inactive lanes are not preserved by the compiler: a spill reload, a copy or a reuse of the
register under a partial exec mask writes the active lanes only, so a cross-lane read of a lane
that is inactive there can return stale bits (a 64-VGPR build of the row decode faulted that way,
DESIGN.md §9). The kernels read every cross-lane value where all lanes are active (or from SGPRs /
LDS); this check keeps it so.

The analysis is a forward data flow over the kernel's basic blocks (branch targets from the SOPP
offsets) that tracks exec and the 64-bit masks in SGPR pairs symbolically, as conjunctions of
literals over the full mask (the empty conjunction is the full mask):
  * `s_and_saveexec_b64 sX, cond` saves exec in sX and narrows exec by a literal of that
    instruction; the structurizer's if / else / join forms (`s_xor_b64`, `s_or_saveexec_b64`,
    `s_or_b64 exec, exec, sX`) combine a literal and its negation back into the mask they split;
  * a loop's `s_andn2_b64 exec, exec, sX` narrows exec by an opaque literal (the loop header's
    meet then holds it: later trips are partial) and marks sX as the loop's exit accumulator:
    `s_or_b64 exec, exec, sX` after the loop restores exec to its value before the loop;
  * masks spilled to VGPR lanes (`v_writelane` / `v_readlane` with a constant lane) keep their
    value; every other write of an SGPR forgets it; a taken `s_cbranch_execz` carries an empty
    exec (its target restores exec first);
  * at a join, masks that differ are combined as their conjunction (may be smaller).
A readlane is flagged unless exec is certainly full there. Exempt: a readlane whose lane comes
from `s_ff1_i32_b64` in the same block (the compiler's loop over the active lanes of a wave
reduction: that lane is active).

Second rule (reload taint): a VGPR reloaded from scratch (`scratch_load_*`) where exec may be
partial holds stale bits in the lanes that were inactive, until the next write of the register;
any cross-lane read of it meanwhile -- readlane / readfirstlane, a DPP move, ds_(b)permute's data,
permlane -- is flagged, whatever exec is at the read (a readfirstlane under a partial mask and the
s_ff1 readlane read a lane active now: exempt).
usage: python -m streaming_amd.isa_check <device object or objdump text> [kernel substring]"""
import re
import subprocess
import sys

EMPTY = 'empty'  # exec with no lane (a taken s_cbranch_execz)


def kernels(text):
    cur, body = None, []
    for line in text.splitlines():
        m = re.match(r'^[0-9a-f]+ <(.+)>:$', line)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
        elif cur:
            body.append(line)
    if cur:
        yield cur, body


def parse(body):
    """(address, mnemonic, operands) per instruction; the address from objdump's comment."""
    out = []
    for line in body:
        code, _, comment = line.partition('//')
        parts = code.replace(',', ' ').split()
        if not parts:
            continue
        m = re.match(r'\s*([0-9A-Fa-f]+):', comment)
        addr = int(m.group(1), 16) if m else (out[-1][0] + 4 if out else 0)
        out.append((addr, parts[0], parts[1:]))
    return out


def branch_target(addr, op, args):
    """Target address of a SOPP branch (simm16 words after the next instruction)."""
    if not (op == 's_branch' or op.startswith('s_cbranch')) or not args:
        return None
    try:
        imm = int(args[0], 0)
    except ValueError:
        return None
    if imm >= 0x8000:
        imm -= 0x10000
    return addr + 4 + 4 * imm


def sregs(op_str):
    """The SGPR numbers an operand names (s7, s[8:9]), or None."""
    m = re.match(r's\[(\d+):(\d+)\]$', op_str)
    if m:
        return tuple(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r's(\d+)$', op_str)
    return (int(m.group(1)),) if m else None


def blocks(ins):
    """Basic blocks [(start, end)] and their successors [(block, edge kind)]."""
    starts = {0}
    addr_ix = {a: i for i, (a, _, _) in enumerate(ins)}
    for i, (addr, op, args) in enumerate(ins):
        tgt = branch_target(addr, op, args)
        if tgt is not None:
            if tgt in addr_ix:
                starts.add(addr_ix[tgt])
            starts.add(i + 1)
        elif op in ('s_endpgm', 's_setpc_b64'):
            starts.add(i + 1)
    starts = sorted(s for s in starts if s < len(ins))
    bl = [(s, (starts[k + 1] if k + 1 < len(starts) else len(ins))) for k, s in enumerate(starts)]
    first = {s: k for k, (s, _) in enumerate(bl)}
    succ = []
    for s, e in bl:
        addr, op, args = ins[e - 1]
        out = []
        tgt = branch_target(addr, op, args)
        if tgt is not None and tgt in addr_ix and addr_ix[tgt] in first:
            out.append((first[addr_ix[tgt]], 'taken'))
        if op not in ('s_branch', 's_endpgm', 's_setpc_b64') and e in first:
            out.append((first[e], 'fall'))
        succ.append(out)
    return bl, succ


# ---- masks: frozensets of literals (conjunctions), EMPTY, or None (unknown)
FULL = frozenset()


def neg(lit):
    return (lit[0], lit[1], 1 - lit[2]) if lit[0] == 'c' else None


def m_or(a, b):
    if a == EMPTY:
        return b
    if b == EMPTY:
        return a
    if a == FULL or b == FULL:
        return FULL
    if a is None or b is None:
        return None
    if a <= b:
        return a  # fewer literals: the larger mask
    if b <= a:
        return b
    da, db = a - b, b - a
    if len(da) == 1 and len(db) == 1 and neg(next(iter(da))) == next(iter(db)):
        return a & b
    return None


def m_and(a, b):
    if a == EMPTY or b == EMPTY:
        return EMPTY
    if a is None or b is None:
        return None
    return a | b


def m_xor(a, b):
    if a is None or b is None:
        return None
    if a == EMPTY:
        return b
    if b == EMPTY:
        return a
    if a == b:
        return EMPTY
    if a <= b or b <= a:
        big, small = (a, b) if a <= b else (b, a)  # big: the larger mask (fewer literals)
        extra = small - big
        if len(extra) == 1 and neg(next(iter(extra))):
            return big | {neg(next(iter(extra)))}
        return None
    da, db = a - b, b - a
    if len(da) == 1 and len(db) == 1 and neg(next(iter(da))) == next(iter(db)):
        return a & b
    return None


def is_acc(m):
    return isinstance(m, tuple) and m[0] == 'acc'


def m_meet(a, b):
    if is_acc(a) or is_acc(b):
        return ('acc', a[1] | b[1]) if is_acc(a) and is_acc(b) else None
    if a == EMPTY:
        return b
    if b == EMPTY:
        return a
    if a is None or b is None:
        return None
    return a | b


class State:
    """exec, SGPR halves ({sgpr: (mask, half)}), spill slots ({(vgpr, lane): (mask, half)}), and
    the VGPRs reloaded from scratch where exec may have been partial (``taint``: their inactive
    lanes hold stale bits until a full-exec write). A loop's exit accumulator holds ('acc', exec
    before the loop)."""

    def __init__(self, ex=FULL, sg=None, slots=None, taint=frozenset()):
        self.ex, self.sg = ex, dict(sg or {})
        self.slots = dict(slots or {})
        self.taint = frozenset(taint)

    def key(self):
        return (self.ex, tuple(sorted(self.sg.items(), key=str)),
                tuple(sorted(self.slots.items(), key=str)), tuple(sorted(self.taint)))

    def copy(self):
        return State(self.ex, self.sg, self.slots, self.taint)

    def val(self, op_str):
        if op_str == 'exec':
            return self.ex
        if op_str == '-1':
            return FULL
        if op_str == '0':
            return EMPTY
        r = sregs(op_str)
        if not r or len(r) != 2:
            return None
        lo, hi = self.sg.get(r[0]), self.sg.get(r[1])
        if lo and hi and lo[1] == 0 and hi[1] == 1 and lo[0] == hi[0]:
            return lo[0]
        return None

    def kill(self, regs):
        for r in regs:
            self.sg.pop(r, None)

    def put(self, op_str, m):
        if op_str == 'exec':
            self.ex = m
            return
        r = sregs(op_str)
        if not r:
            return
        self.kill(r)
        if m is not None and len(r) == 2:
            self.sg[r[0]] = (m, 0)
            self.sg[r[1]] = (m, 1)


def _meet_halves(x, y):
    """Saved masks that differ between two paths: their conjunction (the restore they feed may
    then look smaller than it is, never larger)."""
    out = {}
    for k, v in x.items():
        w = y.get(k)
        if w is not None and w[1] == v[1]:
            m = m_meet(v[0], w[0])
            if m is not None:
                out[k] = (m, v[1])
    return out


def meet_states(a, b):
    if a is None:
        return b.copy()
    out = State(m_meet(a.ex, b.ex), taint=a.taint | b.taint)
    out.sg = _meet_halves(a.sg, b.sg)
    out.slots = _meet_halves(a.slots, b.slots)
    return out


def vregs(op_str):
    """The VGPR numbers an operand names (v7, v[8:9]), or ()."""
    m = re.match(r'v\[(\d+):(\d+)\]$', op_str)
    if m:
        return tuple(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r'v(\d+)$', op_str)
    return (int(m.group(1)),) if m else ()


_DPP = ('row_shr', 'row_shl', 'row_ror', 'wave_shl', 'wave_shr', 'wave_rol', 'wave_ror',
        'row_bcast', 'quad_perm', 'row_mirror', 'row_half_mirror', 'row_share', 'row_xmask')


def cross_lane_sources(op, args):
    """The VGPRs an instruction reads from lanes other than the lane it writes (or from one
    chosen lane): readlane / readfirstlane, DPP moves, ds_(b)permute's data, permlane."""
    if op.startswith(('v_readlane', 'v_readfirstlane')) and len(args) >= 2:
        return vregs(args[1])
    if op.startswith(('ds_bpermute', 'ds_permute')) and len(args) >= 3:
        return vregs(args[2])
    if op.startswith('v_permlane'):
        return tuple(r for a in args for r in vregs(a))
    if op.startswith('v_') and any(a.startswith(_DPP) for a in args):
        return tuple(r for a in args[1:] for r in vregs(a))
    return ()


def taint_step(st, op, args):
    """The reload taint of one instruction: a scratch load under a possibly partial exec taints
    the VGPRs it writes; any write with every lane active clears them."""
    if not args:
        return
    dest = vregs(args[0])
    if not dest or op.startswith(('v_cmp', 'v_readlane', 'v_readfirstlane', 'v_writelane')):
        return
    if op.startswith('scratch_load') or (op.startswith('buffer_load') and 'off' in args):
        st.taint = (st.taint - set(dest)) if st.ex == FULL else (st.taint | set(dest))
    elif op.startswith(('v_', 'global_load', 'flat_load', 'ds_read', 'ds_bpermute', 'ds_permute',
                        'buffer_load')):
        # a new value of the register (defined in the lanes active now, as the source defines it)
        st.taint = st.taint - set(dest)


_NO_DEST = ('s_cmp', 's_bitcmp', 's_cbranch', 's_branch', 's_store', 's_buffer_store', 's_waitcnt',
            's_nop', 's_barrier', 's_sleep', 's_setprio', 's_endpgm', 's_dcache', 's_sendmsg',
            's_trap', 's_setpc', 's_set_gpr_idx', 'v_writelane', 's_memrealtime')


def step(st, addr, op, args):
    """Transfer of one instruction (st updated in place)."""
    if not args:
        return
    d = args[0]
    if op in ('s_and_saveexec_b64', 's_or_saveexec_b64', 's_andn2_saveexec_b64',
              's_xor_saveexec_b64'):
        old, src = st.ex, st.val(args[1])
        if op == 's_and_saveexec_b64':
            if src is not None:
                new = m_and(old, src)
            else:  # a condition: narrow by this instruction's literal
                new = old | {('c', addr, 1)} if old not in (None, EMPTY) else old
        elif op == 's_or_saveexec_b64':
            new = m_or(old, src)
        elif op == 's_andn2_saveexec_b64':
            new = m_and(m_xor(FULL, src), old) if src is not None else None
        else:
            new = m_xor(old, src) if src is not None else None
        st.put(d, old)
        st.ex = new
        return
    if op == 's_andn2_b64' and args[:2] == ['exec', 'exec']:
        if st.ex not in (None, EMPTY):
            before = frozenset(x for x in st.ex if x != ('u', addr, 0))
            st.put(args[2], ('acc', before))
            st.ex = st.ex | {('u', addr, 0)}
        return
    if op == 's_or_b64' and d == 'exec' and args[1] == 'exec':
        v = st.val(args[2])
        if is_acc(v):  # a loop's exit: every lane that entered it
            st.ex = v[1] if st.ex == EMPTY or (st.ex is not None and v[1] <= st.ex) else None
            return
        st.ex = m_or(st.ex, v)
        return
    if op in ('s_or_b64', 's_and_b64', 's_xor_b64', 's_andn2_b64', 's_mov_b64') and \
            (d == 'exec' or (sregs(d) and len(sregs(d)) == 2)):
        if op == 's_mov_b64':
            m = st.val(args[1])
        else:
            a, b = st.val(args[1]), st.val(args[2])
            if op == 's_or_b64' and sregs(d) and (is_acc(a) or is_acc(b)) and \
                    sregs(d) in (sregs(args[1]), sregs(args[2])):
                st.put(d, a if is_acc(a) else b)  # a loop's exit accumulator grows
                return
            a = None if is_acc(a) else a
            b = None if is_acc(b) else b
            if op == 's_or_b64':
                m = m_or(a, b)
            elif op == 's_and_b64':
                m = m_and(a, b)
            elif op == 's_xor_b64':
                m = m_xor(a, b)
            else:
                m = m_and(a, m_xor(FULL, b)) if b is not None else None
        st.put(d, m)
        return
    if op == 's_mov_b32' and sregs(d):
        src = sregs(args[1])
        v = st.sg.get(src[0]) if src else None
        st.kill(sregs(d))
        if v is not None:
            st.sg[sregs(d)[0]] = v
        return
    if op == 'v_writelane_b32' and len(args) >= 3:
        m = re.match(r'v(\d+)$', d)
        src = sregs(args[1])
        if m:
            slot = (int(m.group(1)), args[2])
            v = st.sg.get(src[0]) if src else None
            if v is not None:
                st.slots[slot] = v
            else:
                st.slots.pop(slot, None)
        return
    if op == 'v_readlane_b32' and len(args) >= 3 and sregs(d):
        m = re.match(r'v(\d+)$', args[1])
        st.kill(sregs(d))
        v = st.slots.get((int(m.group(1)), args[2])) if m else None
        if v is not None:
            st.sg[sregs(d)[0]] = v
        return
    if d in ('exec', 'exec_lo', 'exec_hi'):
        st.ex = None
        return
    r = sregs(d)
    if r and not op.startswith(_NO_DEST):
        st.kill(r)
        return
    m = re.match(r'v(\d+)$', d)
    if m and op.startswith('v_') and not op.startswith(('v_cmp', 'v_readfirstlane')):
        n = int(m.group(1))  # a VALU write of a spill VGPR ends the slots it held
        st.slots = {k: v for k, v in st.slots.items() if k[0] != n}


def check(text, want='rows_decode_kernel'):
    """[(kernel, [addresses of variable-lane readlanes where exec may be partial])]"""
    bad = []
    for name, body in kernels(text):
        if want not in name:
            continue
        ins = parse(body)
        if not ins:
            continue
        bl, succ = blocks(ins)
        entry = [None] * len(bl)
        entry[0] = State()
        work = [0]
        while work:
            k = work.pop()
            st = entry[k].copy()
            s, e = bl[k]
            for addr, op, args in ins[s:e]:
                step(st, addr, op, args)
                taint_step(st, op, args)
            last_op = ins[e - 1][1]
            for n, kind in succ[k]:
                out = st
                if (kind == 'taken' and last_op == 's_cbranch_execz') or \
                        (kind == 'fall' and last_op == 's_cbranch_execnz'):
                    out = st.copy()
                    out.ex = EMPTY
                m = meet_states(entry[n], out)
                if entry[n] is None or m.key() != entry[n].key():
                    entry[n] = m
                    work.append(n)
        hits = []
        for k, (s, e) in enumerate(bl):
            if entry[k] is None:
                continue  # unreachable
            st = entry[k].copy()
            ff1 = set()  # SGPRs holding an active lane's index (s_ff1 of exec's copy)
            for addr, op, args in ins[s:e]:
                if op == 'v_readlane_b32' and len(args) >= 3 and re.match(r's\d+$', args[2]):
                    if st.ex != FULL and st.ex != EMPTY and args[2] not in ff1:
                        hits.append(addr)
                # a lane of a register reloaded under a partial mask (readfirstlane under a partial
                # mask, and readlane of the s_ff1 lane, read a lane active now, which was active at
                # the nested reload)
                active_lane = (op.startswith('v_readfirstlane') and st.ex != FULL) or (
                    op == 'v_readlane_b32' and len(args) >= 3 and args[2] in ff1)
                if st.taint and set(cross_lane_sources(op, args)) & st.taint and not active_lane:
                    hits.append(addr)
                dest = args[0] if args else None
                if op.startswith('s_ff1_i32'):
                    ff1.add(dest)
                elif dest in ff1 and not op.startswith(_NO_DEST):
                    ff1.discard(dest)
                step(st, addr, op, args)
                taint_step(st, op, args)
        if hits:
            bad.append((name, sorted(set(hits))))
    return bad


if __name__ == '__main__':
    src = sys.argv[1]
    text = open(src).read() if src.endswith('.s') else subprocess.run(
        ['/opt/rocm/lib/llvm/bin/llvm-objdump', '-d', src], capture_output=True, text=True,
        check=True).stdout
    bad = check(text, sys.argv[2] if len(sys.argv) > 2 else 'rows_decode_kernel')
    for name, addrs in bad:
        print(f'{name}: variable-lane v_readlane where exec may be partial at ' +
              ', '.join(hex(a) for a in addrs))
    sys.exit(1 if bad else 0)
