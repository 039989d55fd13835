"""ngt_amd -- MI355X-native NGT distance hot path (Python side).

The product is ``ngt_amd/libngt_amd.so`` (HIP kernels for gfx950 + the C ABI of
include/ngt_amd.h and the drop-in ``ngt_*`` API of include/NGT/Capi.h).  This
package only loads it with ctypes: there is no Python or CPU compute path, and
importing the bindings fails loudly when the library is missing.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NGT_AMD_LIB") or os.path.join(HERE, "libngt_amd.so")
_LIB = None


class NativeError(Exception):
    pass


def build(verbose=False):
    """Compile libngt_amd.so for gfx950 in-tree (hipcc)."""
    import subprocess
    cmd = ["make", "-j8", "-C", HERE]
    r = subprocess.run(cmd, capture_output=not verbose, text=True)
    if r.returncode != 0:
        raise NativeError("building libngt_amd.so failed:\n%s\n%s" % (r.stdout, r.stderr))
    return LIB_PATH


def lib():
    """The loaded libngt_amd.so (raises if it has not been built)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError("%s is missing: run ngt_amd.build() (or `make -C ngt_amd`)" % LIB_PATH)
        # One HIP runtime per process: torch bundles its own libamdhip64 (found
        # by file name, not SONAME).  Loading torch first lets our library bind
        # to that same runtime (SONAME libamdhip64.so.7); loading ours first would
        # leave torch a second runtime that cannot see the device.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        _LIB = ctypes.CDLL(LIB_PATH)
        from . import _sigs
        _sigs.declare(_LIB)
    return _LIB


def last_error():
    return lib().ngt_amd_last_error().decode()


def device_count():
    return int(lib().ngt_amd_device_count())
