"""Hash of the native sources: every file of aioquic_amd/csrc/ and the C ABI
header include/quic_pp.h.

build.py compiles the hash into libquicpp.so (``qpp_source_hash()``) and into
the _crypto extension; the extension refuses to import when the two differ or
when the tree's sources no longer hash to what it was built from, so a
snapshot whose file times are skewed cannot silently run old kernels (the
reference rebuilds its extension from source every time, setup.py:33-39).
Plain Python with no package imports: _crypto's module init calls it.
"""

import hashlib
import os
from typing import Optional

_PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(_PKG, "csrc")
HEADER = os.path.join(os.path.dirname(_PKG), "include", "quic_pp.h")
_EXTS = (".hip", ".h", ".c", ".cc", ".cpp")


def source_files() -> list:
    # (dot files are scratch copies, e.g. tools/build_variant.py's)
    names = sorted(f for f in os.listdir(CSRC) if f.endswith(_EXTS) and not f.startswith("."))
    return [os.path.join(CSRC, f) for f in names] + [HEADER]


def tree_hash() -> Optional[str]:
    """16 hex digits over (name, bytes) of every source file; None when the
    sources are not present (nothing to compare against)."""
    if not os.path.isdir(CSRC) or not os.path.exists(HEADER):
        return None
    h = hashlib.sha256()
    for path in source_files():
        h.update(os.path.basename(path).encode() + b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]
