"""Source hash of the engine library: sha256 over the engine's sources (taxi2_amd/csrc/*.hip,
*.hpp, the Makefile and include/*.h), each as "<relative path>\\0<bytes>\\0", in sorted path order.

The Makefile bakes it into the library (-DTAXI2_SRC_HASH, returned by taxi2_version()), and
bench.py / smoke() print it next to the same hash computed from the tree they run in, so a record
shows whether the measured binary was built from the sources beside it.  Standard library only
(the Makefile runs it before anything is built): ``python3 srchash.py`` prints the 16-hex prefix.
"""

from __future__ import annotations

import hashlib
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def src_files(root: Path = ROOT) -> list[Path]:
    c = root / "taxi2_amd" / "csrc"
    files = [*c.glob("*.hip"), *c.glob("*.hpp"), c / "Makefile", *(root / "include").glob("*.h")]
    return sorted((f for f in files if f.is_file()), key=lambda f: f.relative_to(root).as_posix())


def src_hash(root: Path = ROOT) -> str:
    h = hashlib.sha256()
    for f in src_files(root):
        h.update(f.relative_to(root).as_posix().encode() + b"\0")
        h.update(f.read_bytes() + b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(src_hash())
