"""aioquic_amd -- MI355X-native QUIC packet protection.

Drop-in for aioquic's packet-protection path (``aioquic._crypto`` and
``aioquic.quic.crypto``): the same AEAD / HeaderProtection / CryptoError object
API and CryptoContext / CryptoPair semantics, executed by HIP kernels on a
gfx950 GPU, plus a batch engine (``aioquic_amd.batch``) that protects and
unprotects many packets per launch.
"""

import ctypes as _ctypes
import importlib.util as _ilu
import os as _os

__version__ = "0.1.0"


def _share_hip_runtime_with_torch() -> None:
    """PyTorch wheels bundle their own libamdhip64 (same soname as /opt/rocm's).
    Two HIP runtimes in one process break whichever initialises second, so when
    torch is installed load ITS runtime first: libquicpp's NEEDED entry then
    binds to the same copy whatever the import order."""
    try:
        spec = _ilu.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is None or not spec.origin:
        return
    lib = _os.path.join(_os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if _os.path.exists(lib):
        try:
            _ctypes.CDLL(lib, mode=_ctypes.RTLD_GLOBAL)
        except OSError:
            pass


_share_hip_runtime_with_torch()
