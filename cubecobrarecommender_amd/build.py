"""Build libccrec_hip.so in-tree for gfx950 with hipcc (no CUDA, no hipify, no JIT cache).

Usage: python -m cubecobrarecommender_amd.build [--force]
The .so lands next to this file so gpurun snapshots carry it to the GPU box.
"""
import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, 'csrc')
INC = os.path.join(ROOT, 'include')
# dev experiments: CCREC_BUILD_TAG=x builds libccrec_hip_x.so from build_obj_x with CCREC_EXTRA_FLAGS
# (load it with CCREC_LIB=...); the product library is the untagged one
_TAG = os.environ.get('CCREC_BUILD_TAG', '')
OBJ = os.path.join(PKG, 'build_obj' + (f'_{_TAG}' if _TAG else ''))
LIB = os.path.join(PKG, 'libccrec_hip' + (f'_{_TAG}' if _TAG else '') + '.so')
ARCH = os.environ.get('CCREC_ARCH', 'gfx950')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
FLAGS = ['-O3', '-fPIC', '-std=c++17', f'--offload-arch={ARCH}', '-I', INC, '-I', CSRC,
         '-Wall', '-Wno-unused-function', '-Wno-unused-variable'] + os.environ.get('CCREC_EXTRA_FLAGS', '').split()


# per-file flags: the fused output-layer kernels' inputs are finite (logits, M~ rows, row stats;
# the KL's clipped targets never meet an infinite log); without NaN semantics their min / max need
# no canonicalising v_max (one VALU op per logit in VALU-bound epilogues; decreg.hip: the sampled
# main pass's scratch spill goes too)
FILE_FLAGS = {'decout.hip': ['-fno-honor-nans'], 'decreg.hip': ['-fno-honor-nans']}


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(('.hip', '.cpp')))


def _headers_mtime():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(('.hpp', '.h'))]
    hs.append(os.path.join(INC, 'ccrec.h'))
    return max(os.path.getmtime(h) for h in hs)


def _compile(src, force, build_id):
    obj = os.path.join(OBJ, os.path.basename(src) + '.o')
    extra = []
    if os.path.basename(src) == 'api.cpp':   # the source identity (buildid.py) lives in api.cpp
        extra = [f'-DCC_BUILD_ID="{build_id}"']
        stamp = os.path.join(OBJ, 'build_id.txt')
        if not os.path.exists(stamp) or open(stamp).read() != build_id:
            force = True
    if not force and os.path.exists(obj) and os.path.getmtime(obj) > max(os.path.getmtime(src), _headers_mtime()):
        return obj
    cmd = [HIPCC, *FLAGS, *FILE_FLAGS.get(os.path.basename(src), []), *extra, '-c', src, '-o', obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'hipcc failed for {src}:\n{r.stderr}')
    if extra:
        with open(os.path.join(OBJ, 'build_id.txt'), 'w') as fh:
            fh.write(build_id)
    return obj


def build(force=False, jobs=8):
    from .buildid import tree_build_id
    os.makedirs(OBJ, exist_ok=True)
    bid = tree_build_id()
    try:
        with cf.ThreadPoolExecutor(jobs) as ex:
            objs = list(ex.map(lambda s: _compile(s, force, bid), sources()))
    except RuntimeError:
        if os.path.exists(LIB):
            os.remove(LIB)        # never leave a stale library behind a failed build
        raise
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, '-shared', '-fPIC', f'--offload-arch={ARCH}', *objs, '-o', LIB]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'link failed:\n{r.stderr}')
    return LIB


if __name__ == '__main__':
    print(build(force='--force' in sys.argv))
