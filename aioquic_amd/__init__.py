"""aioquic_amd -- MI355X-native QUIC packet protection.

Drop-in for aioquic's packet-protection path (``aioquic._crypto`` and
``aioquic.quic.crypto``): the same AEAD / HeaderProtection / CryptoError object
API and CryptoContext / CryptoPair semantics, executed by HIP kernels on a
gfx950 GPU, plus a batch engine (``aioquic_amd.batch``) that protects and
unprotects many packets per launch.
"""

__version__ = "0.1.0"
