"""Runs last (file order): after the GPU suite, no GCM launch hit the table
entry watchdog (qpp_watchdog_count: a kernel that waited ~1 s for a GHASH
table entry and skipped that slot's packets without results)."""

import pytest


@pytest.mark.gpu
def test_no_watchdog_events():
    from aioquic_amd import _crypto

    assert _crypto.watchdog_count() == 0
