"""The build's ISA check (streaming_amd/isa_check.py): a cross-lane read (`v_readlane` with a
run-time lane) of a register that was just reloaded from scratch is refused; the same read of a
register computed in place passes. CPU only (objdump text)."""
import os

from streaming_amd import isa_check

HEAD = '0000000000001000 <_ZN12mdsx_kernels12rows_decode_kernelILi6EEEvv>:\n'


def test_flags_readlane_of_reloaded_register():
    text = HEAD + '\n'.join([
        '\ts_and_saveexec_b64 s[2:3], vcc',
        '\tscratch_load_dwordx2 v[2:3], off, off offset:8   // 0000',
        '\ts_waitcnt vmcnt(0)',
        '\tv_readlane_b32 s3, v3, s10',
        '\ts_endpgm',
    ])
    assert isa_check.check(text) == [(HEAD.split('<')[1].split('>')[0], [3])]


def test_passes_readlane_of_computed_register():
    text = HEAD + '\n'.join([
        '\tscratch_load_dwordx2 v[2:3], off, off offset:8',
        '\tv_add_u32_e32 v3, 1, v3',
        '\tv_readlane_b32 s3, v3, s10',
        '\tv_readlane_b32 s4, v2, 5',  # (a constant lane: not a run-time choice)
        '\ts_endpgm',
    ])
    assert isa_check.check(text) == []


def test_other_kernels_ignored():
    text = HEAD.replace('rows_decode_kernel', 'seg_decode_kernel') + \
        '\tscratch_load_dword v7, off, off\n\tv_readlane_b32 s1, v7, s2\n'
    assert isa_check.check(text) == []


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
