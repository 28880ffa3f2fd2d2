"""Build identity of libtkv_crc32.so: a hash of the sources and build flags it is made from.

The Makefile (tinykvpp_amd/csrc/Makefile) runs this module at build time and bakes the hash into
the library (`tkv_build_id()`); the GPU test session and bench.py compare it with the hash of the
tree they run in, so a library left over from other sources cannot pass unnoticed.

    python3 tinykvpp_amd/build_id.py [ROOT]   # prints the tree's hash
"""
import glob
import hashlib
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_files(root=_ROOT):
    """Every input of the product library: csrc sources, headers and Makefile, and the public headers."""
    csrc = os.path.join(root, "tinykvpp_amd", "csrc")
    files = []
    for pat in ("*.hip", "*.cpp", "*.h", "Makefile"):
        files += glob.glob(os.path.join(csrc, pat))
    files += glob.glob(os.path.join(root, "include", "*.h"))
    return sorted(os.path.relpath(f, root) for f in files)


def source_hash(root=_ROOT):
    """First 16 hex digits of sha256 over (relative path, NUL, contents, NUL) of every source file."""
    h = hashlib.sha256()
    for rel in source_files(root):
        h.update(rel.encode() + b"\0")
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def library_build_id():
    """The hash baked into the loaded libtkv_crc32.so."""
    from ._lib import load_library
    return load_library().tkv_build_id().decode()


def check():
    """(library id, tree hash, equal)."""
    lib, tree = library_build_id(), source_hash()
    return lib, tree, lib == tree


if __name__ == "__main__":
    print(source_hash(os.path.abspath(sys.argv[1]) if len(sys.argv) > 1 else _ROOT))
