"""Identity of the libfugu build a committed rocprof profile measured: sha1 of
the sources that decide the device path's memory traffic (the kernels, the
shared layout header, the host planner/builder and the compile flags).  Host-
only code (host.cpp: parser, registry, JSON) does not change it, and a rebuild
of the same sources keeps it, so bench.py quotes `roofline.traffic` exactly for
the build it was counted on."""
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = ("kernels.hip", "fg_internal.h", "fugu.cpp", "Makefile")


def lib_id(csrc=None):
    csrc = csrc or os.path.join(ROOT, "fugu_amd", "csrc")
    h = hashlib.sha1()
    for name in SOURCES:
        with open(os.path.join(csrc, name), "rb") as f:
            h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(lib_id())
