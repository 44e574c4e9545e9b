"""The ctypes mirrors of include/ccrec.h's argument structs (cubecobrarecommender_amd/_lib.py) against
the C layout: every field's offset and every struct's size as gcc lays them out from the header.
A mirror that drifts from the header (a field added on one side only) would hand the kernels
shifted arguments without any error; this pins them on the CPU (no GPU, no library load)."""
import os
import subprocess

import pytest

from cubecobrarecommender_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ctypes mirror -> C typedef
PAIRS = [(L.NoiseArgs, 'cc_noise_args'), (L.GemmArgs, 'cc_gemm_args'), (L.AdamTRegion, 'cc_adam_tregion'),
         (L.TowerArgs, 'cc_tower_args'), (L.DecKlArgs, 'cc_dec_kl_args'), (L.AdamPack, 'cc_adam_pack')]


def _c_layout(tmp_path):
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "ccrec.h"', 'int main(void) {']
    for cls, cname in PAIRS:
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for name, _ in cls._fields_:
            lines.append(f'  printf("{cname} {name} %zu\\n", offsetof({cname}, {name}));')
    lines += ['  return 0;', '}']
    src = tmp_path / 'layout.c'
    src.write_text('\n'.join(lines) + '\n')
    exe = tmp_path / 'layout'
    subprocess.run(['gcc', '-std=c11', '-I', os.path.join(ROOT, 'include'), str(src), '-o', str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    lay = {}
    for ln in out.splitlines():
        cname, field, val = ln.split()
        lay[(cname, field)] = int(val)
    return lay


@pytest.mark.skipif(subprocess.run(['which', 'gcc'], capture_output=True).returncode != 0, reason='gcc absent')
def test_ctypes_mirrors_match_the_header(tmp_path):
    lay = _c_layout(tmp_path)
    for cls, cname in PAIRS:
        assert lay[(cname, 'size')] == L.C.sizeof(cls), (cname, lay[(cname, 'size')], L.C.sizeof(cls))
        for name, _ in cls._fields_:
            assert lay[(cname, name)] == getattr(cls, name).offset, (cname, name)
