"""The build's ISA check (streaming_amd/isa_check.py): a cross-lane read (`v_readlane` with a
run-time lane) where the exec mask may be partial is refused -- inside a divergent loop (the
round-4 fault's shape: the column ends read inside the row decode's chunk loop), inside an if,
and after a reload fed through the loop's back edge -- and passes where every lane is active:
straight-line code, after an if / if-else join, after a divergent loop's exit, the compiler's own
active-lane loop (s_ff1). CPU only (objdump-format text)."""
import os

from streaming_amd import isa_check

NAME = '_ZN12mdsx_kernels12rows_decode_kernelILi6EEEvv'


def asm(lines, name=NAME):
    """objdump-style text: one instruction per line at 0x1000 + 4 i (every instruction one word
    here); `@label` operands become SOPP branch offsets, `label:` lines mark targets."""
    labels, ins = {}, []
    for ln in lines:
        if ln.endswith(':'):
            labels[ln[:-1]] = 0x1000 + 4 * len(ins)
        else:
            ins.append(ln)
    out = [f'0000000000001000 <{name}>:']
    for i, ln in enumerate(ins):
        addr = 0x1000 + 4 * i
        if '@' in ln:
            op, lab = ln.split('@')
            off = ((labels[lab] - (addr + 4)) // 4) & 0xffff
            ln = f'{op}{off}'
        out.append(f'\t{ln:<58}// {addr:012X}: 00000000')
    return '\n'.join(out) + '\n'


def flagged(lines, **kw):
    bad = isa_check.check(asm(lines, **kw))
    return [a for _, addrs in bad for a in addrs]


def test_flags_readlane_inside_divergent_loop():
    # for (k = t; k < n; k += 256) { ... readlane(ends, j) ... }: lanes leave one by one
    lines = [
        's_mov_b64 s[84:85], 0',
        'loop:',
        'v_readlane_b32 s3, v45, s2',  # the column ends, read on every trip
        'v_add_u32_e32 v70, 0x100, v70',
        'v_cmp_le_u32_e32 vcc, s36, v70',
        's_or_b64 s[84:85], vcc, s[84:85]',
        's_andn2_b64 exec, exec, s[84:85]',
        's_cbranch_execnz @loop',
        's_or_b64 exec, exec, s[84:85]',
        's_endpgm',
    ]
    assert flagged(lines) == [0x1004]


def test_flags_reload_through_back_edge():
    # the reload comes later in the text than the readlane: reached through the back edge
    lines = [
        's_mov_b64 s[84:85], 0',
        'loop:',
        'v_readlane_b32 s3, v3, s10',
        'v_cmp_le_u32_e32 vcc, s36, v70',
        's_or_b64 s[84:85], vcc, s[84:85]',
        's_andn2_b64 exec, exec, s[84:85]',
        'scratch_load_dwordx2 v[2:3], off, off offset:8',
        's_waitcnt vmcnt(0)',
        's_cbranch_execnz @loop',
        's_or_b64 exec, exec, s[84:85]',
        's_endpgm',
    ]
    assert flagged(lines) == [0x1004]


def test_flags_readlane_inside_if():
    lines = [
        'v_cmp_gt_u32_e32 vcc, s36, v0',
        's_and_saveexec_b64 s[2:3], vcc',
        's_cbranch_execz @join',
        'v_readlane_b32 s3, v3, s10',
        'join:',
        's_or_b64 exec, exec, s[2:3]',
        's_endpgm',
    ]
    assert flagged(lines) == [0x100c]


def test_passes_after_joins():
    lines = [
        'v_readlane_b32 s4, v2, s9',  # straight-line, every lane active
        # an if
        'v_cmp_gt_u32_e32 vcc, s36, v0',
        's_and_saveexec_b64 s[2:3], vcc',
        's_cbranch_execz @j1',
        'v_add_u32_e32 v3, 1, v3',
        'j1:',
        's_or_b64 exec, exec, s[2:3]',
        'v_readlane_b32 s5, v3, s10',
        # an if-else (the structurizer's form)
        'v_cmp_gt_u32_e32 vcc, s37, v0',
        's_and_saveexec_b64 s[6:7], vcc',
        's_xor_b64 s[6:7], exec, s[6:7]',
        'v_add_u32_e32 v4, 1, v4',
        's_or_saveexec_b64 s[6:7], s[6:7]',
        's_xor_b64 exec, exec, s[6:7]',
        's_cbranch_execz @j2',
        'v_add_u32_e32 v4, 2, v4',
        'j2:',
        's_or_b64 exec, exec, s[6:7]',
        'v_readlane_b32 s6, v4, s10',
        # a divergent loop, then its exit (its saved mask spilled and reloaded on the way)
        's_mov_b64 s[84:85], 0',
        'loop:',
        'v_add_u32_e32 v70, 0x100, v70',
        'v_cmp_le_u32_e32 vcc, s36, v70',
        's_or_b64 s[84:85], vcc, s[84:85]',
        's_andn2_b64 exec, exec, s[84:85]',
        's_cbranch_execnz @loop',
        'v_writelane_b32 v79, s84, 3',
        'v_writelane_b32 v79, s85, 4',
        's_mov_b64 s[84:85], -1',
        'v_readlane_b32 s84, v79, 3',
        'v_readlane_b32 s85, v79, 4',
        's_or_b64 exec, exec, s[84:85]',
        'v_readlane_b32 s7, v70, s10',
        # the compiler's loop over the active lanes (a wave reduction)
        's_and_saveexec_b64 s[2:3], vcc',
        's_mov_b64 s[4:5], exec',
        'red:',
        's_ff1_i32_b64 s36, s[4:5]',
        'v_readlane_b32 s43, v32, s36',
        's_lshl_b64 s[54:55], 1, s36',
        's_andn2_b64 s[4:5], s[4:5], s[54:55]',
        's_cmp_lg_u64 s[4:5], 0',
        's_cbranch_scc1 @red',
        's_or_b64 exec, exec, s[2:3]',
        's_endpgm',
    ]
    assert flagged(lines) == []


def test_other_kernels_ignored():
    lines = ['s_and_saveexec_b64 s[2:3], vcc', 'v_readlane_b32 s1, v7, s2', 's_endpgm']
    assert flagged(lines, name=NAME.replace('rows_decode_kernel', 'seg_decode_kernel')) == []
    assert flagged(lines) == [0x1004]


def test_built_row_decode_passes():
    obj = os.path.join(os.path.dirname(isa_check.__file__), 'build', 'mdsx_rows.device.o')
    if not os.path.exists(obj):
        import pytest
        pytest.skip('library not built here')
    import subprocess
    text = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-objdump', '-d', obj], capture_output=True,
                          text=True, check=True).stdout
    assert 'rows_decode_kernel' in text
    assert isa_check.check(text) == []


def test_checked_kernels_by_name():
    """The build checks the one-row-per-wave and one-sample-per-wave decodes too:
    the same flow refuses their variable-lane reads under a partial exec mask."""
    lines = ['v_cmp_gt_u32_e32 vcc, s36, v0', 's_and_saveexec_b64 s[2:3], vcc',
             'v_readlane_b32 s1, v7, s2', 's_or_b64 exec, exec, s[2:3]',
             'v_readlane_b32 s3, v7, s2', 's_endpgm']
    for kernel in ('rowwave_decode_kernel', 'swave_decode_kernel'):
        name = NAME.replace('rows_decode_kernel', kernel)
        bad = isa_check.check(asm(lines, name=name), kernel)
        assert [a for _, addrs in bad for a in addrs] == [0x1008], kernel


def test_built_checked_kernels_pass():
    from streaming_amd import build
    import subprocess
    for src, want in build.ISA_CHECKED.items():
        obj = os.path.join(os.path.dirname(isa_check.__file__), 'build',
                           src.replace('.hip', '.device.o'))
        if not os.path.exists(obj):
            import pytest
            pytest.skip('library not built here')
        text = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-objdump', '-d', obj],
                              capture_output=True, text=True, check=True).stdout
        for w in want:
            assert w in text, (src, w)
            assert isa_check.check(text, w) == [], (src, w)


def test_flags_cross_lane_read_of_a_partial_reload():
    """A VGPR reloaded from scratch under a partial exec mask holds stale bits in its inactive
    lanes: a later cross-lane read of it -- readlane, DPP, ds_bpermute -- is flagged even with
    every lane active; a full-exec write (or a new value) clears it."""
    def body(read):
        return ['v_cmp_gt_u32_e32 vcc, s36, v0', 's_and_saveexec_b64 s[2:3], vcc',
                'scratch_load_dwordx2 v[6:7], off, off offset:4', 's_or_b64 exec, exec, s[2:3]',
                read, 's_endpgm']
    assert flagged(body('v_readlane_b32 s1, v6, 5')) == [0x1010]
    assert flagged(body('v_mov_b32_dpp v9, v7 row_shr:1 row_mask:0xf bank_mask:0xf')) == [0x1010]
    assert flagged(body('ds_bpermute_b32 v9, v8, v6')) == [0x1010]
    assert flagged(body('v_readlane_b32 s1, v8, 5')) == []  # another register
    cleared = body('v_readlane_b32 s1, v6, 5')
    cleared.insert(4, 'v_mov_b32_e32 v6, 0')  # a full-exec write
    assert flagged(cleared) == []
    full = ['v_cmp_gt_u32_e32 vcc, s36, v0', 's_and_saveexec_b64 s[2:3], vcc', 's_nop 0',
            's_or_b64 exec, exec, s[2:3]',  # the reload after the join sees every lane
            'scratch_load_dwordx2 v[6:7], off, off offset:4', 'v_readlane_b32 s1, v6, 5',
            's_endpgm']
    assert flagged(full) == []
