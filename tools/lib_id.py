"""Identity of the built libfugu.so (sha1 of its device code object section
and host code) so a committed rocprof profile is only quoted for the build it
measured."""
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def lib_id(path=None):
    path = path or os.environ.get("FUGU_LIB") or os.path.join(ROOT, "fugu_amd", "libfugu.so")
    with open(path, "rb") as f:
        return hashlib.sha1(f.read()).hexdigest()[:16]
