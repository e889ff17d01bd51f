"""aioquic tests/test_crypto_v2.py against aioquic_amd (RFC 9369 App. A)."""
from tests.crypto_cases import V2, make_tests

globals().update(make_tests(V2))
