#!/usr/bin/env python3
"""sha256 of the gfx950 code object (one per translation unit) that holds a given kernel.

libldpc_amd.so embeds one uncompressed clang offload bundle per .hip translation unit; the
gfx950 entry of each is an ELF code object.  A PMC count (VALU instructions, bytes) describes the
machine code of the profiled kernel, so bench.py accepts a PMC summary whose stamp matches either
the whole library's sha256 or the sha256 of the code object that contains the benched kernel:
rebuilding the library after a change in an unrelated translation unit leaves the latter alone.

    python3 tools/code_object_sha.py <lib.so> <kernel-name-substring>
    python3 tools/code_object_sha.py --all <lib.so>      (one sha256 per code object)
"""
import hashlib
import re
import struct
import sys

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib_path):
    """[(offset, bytes)] of the gfx950 code objects in the library's offload bundles."""
    d = open(lib_path, "rb").read()
    out = []
    for m in re.finditer(re.escape(MAGIC), d):
        o = m.start()
        n = struct.unpack_from("<Q", d, o + 24)[0]
        p = o + 32
        for _ in range(n):
            off, size, ts = struct.unpack_from("<QQQ", d, p)
            p += 24
            triple = d[p:p + ts]
            p += ts
            if b"gfx950" in triple:
                out.append((o + off, d[o + off:o + off + size]))
    return out


def kernel_code_sha(lib_path, needle):
    """sha256 of the one code object whose symbols include `needle` (bytes or str), else None."""
    if isinstance(needle, str):
        needle = needle.encode()
    hits = [blob for _, blob in code_objects(lib_path) if needle in blob]
    if len(hits) != 1:
        return None
    return hashlib.sha256(hits[0]).hexdigest()


if __name__ == "__main__":
    if sys.argv[1] == "--all":
        for _, blob in code_objects(sys.argv[2]):
            print(hashlib.sha256(blob).hexdigest())
        sys.exit(0)
    sha = kernel_code_sha(sys.argv[1], sys.argv[2])
    if sha is None:
        sys.exit(f"no unique gfx950 code object holds {sys.argv[2]!r}")
    print(sha)
