"""aioquic tests/test_crypto_v1.py against aioquic_amd (RFC 9001 App. A)."""
from tests.crypto_cases import V1, make_tests

globals().update(make_tests(V1))
