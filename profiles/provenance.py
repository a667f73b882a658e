"""Which engine build a measurement belongs to, without git (the GPU box gets the tree minus .git):
a SHA-256 over the sources libplacement.so is built from.  profiles/summarize.py stamps it into a
profile's summary.json and bench.py compares it with the tree it runs from, so a committed profile
is only used for the bench line of the same kernels."""
import hashlib
import os

SOURCES = ("training-operator_amd/csrc", "include")
EXTS = (".hip", ".cpp", ".h", "Makefile")


def source_hash(root: str) -> str:
    h = hashlib.sha256()
    for sub in SOURCES:
        d = os.path.join(root, sub)
        for name in sorted(os.listdir(d)):
            if name.endswith(EXTS):
                with open(os.path.join(d, name), "rb") as f:
                    h.update(name.encode() + b"\0" + f.read() + b"\0")
    return h.hexdigest()[:16]
