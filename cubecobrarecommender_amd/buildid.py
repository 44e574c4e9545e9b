"""Source identity of libccrec_hip.so: a SHA-256 over every file the library is compiled from
(csrc/*.hip, *.cpp, *.hpp, *.h and include/ccrec.h, in sorted name order, each prefixed by its
name and length).  build.py compiles the digest into the library (cc_build_id()); _lib.check_build_id
compares it with the digest of the sources in the tree, so a test run or smoke() on a stale
binary fails instead of testing something other than HEAD.  No torch / HIP import here."""
import hashlib
import os

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, 'csrc')
INC = os.path.join(os.path.dirname(PKG), 'include')


def source_files():
    fs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(('.hip', '.cpp', '.hpp', '.h'))]
    fs += [os.path.join(INC, f) for f in os.listdir(INC) if f.endswith('.h')]
    return sorted(fs, key=os.path.basename)


def tree_build_id(extra=''):
    """Hex digest (first 32 chars) of the library's sources; `extra` = build flags."""
    h = hashlib.sha256()
    for f in source_files():
        data = open(f, 'rb').read()
        h.update(f'{os.path.basename(f)}:{len(data)}:'.encode())
        h.update(data)
    h.update(extra.encode())
    return h.hexdigest()[:32]
