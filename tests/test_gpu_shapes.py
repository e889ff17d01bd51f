"""GCM launch shapes (qpp_engine.hip launch_packets / gcm_two_wg): a key table
holding one key of the suite and a launch of at most one 16-packet item per
wave runs as two 512-thread workgroups per CU (one GHASH table entry each);
everything else as one 1024-thread workgroup per CU.  Both shapes against the
oracle, byte for byte, on either side of the boundary."""

import numpy as np
import pytest

from tests.test_gpu_parity import _keys, _random_batch

pytestmark = pytest.mark.gpu


def _check(oracle, recs, n, seed, max_payload=1400):
    from aioquic_amd import layout as L
    from aioquic_amd.batch import PacketEngine, layout_packets

    rng = np.random.default_rng(seed)
    eng = PacketEngine(len(recs))
    eng.set_key_records(recs)
    headers, payloads, pns, slots = _random_batch(rng, n, len(recs), recs, max_payload=max_payload)
    inbuf, desc, size = layout_packets(headers, payloads, pns, slots)
    out_g, res_g = eng.protect_host(desc, inbuf.tobytes(), size)
    out_o, res_o = oracle.protect_batch(recs, desc, inbuf, size)
    assert (res_g == res_o).all()
    assert np.array_equal(out_g, out_o)
    ud = desc.copy()
    ud["len"] = res_g["out_len"]
    ud["hdr_len"] = [len(h) - ((h[0] & 3) + 1) for h in headers]
    u_g, r_g = eng.unprotect_host(ud, out_g.tobytes(), size)
    u_o, r_o = oracle.unprotect_batch(recs, ud, out_g, size)
    assert (r_g == r_o).all()
    ok = r_g["status"] == L.S_OK
    assert ok.mean() > 0.75  # the rest: the reference's signed-pn quirk (test_random_batch_vs_oracle)
    for i in np.nonzero(ok)[0]:
        o, ln = int(ud[i]["out_off"]), int(r_g[i]["out_len"])
        assert np.array_equal(u_g[o : o + ln], u_o[o : o + ln]), i


@pytest.mark.parametrize("suite", [0, 1], ids=["aes128", "aes256"])
def test_two_workgroups_single_key(oracle, suite):
    """One key of the suite, 3000 ragged packets (188 items): two 512-thread
    workgroups per CU."""
    recs = _keys(np.random.default_rng(11 + suite), 1, suites=(suite,))
    _check(oracle, recs, 3000, 21 + suite)


@pytest.mark.parametrize("suite", [0, 1], ids=["aes128", "aes256"])
def test_one_workgroup_two_keys(oracle, suite):
    """Two keys of the suite, same batch shape: one 1024-thread workgroup per CU."""
    recs = _keys(np.random.default_rng(31 + suite), 2, suites=(suite,))
    _check(oracle, recs, 3000, 41 + suite)


def test_shape_boundary_one_key(oracle):
    """One key, 4096 x 16 + 16 small packets (4097 items: past one item per
    wave on a 256-CU part, so one 1024-thread workgroup per CU) and 4096 x 16
    (two of 512): both against the oracle."""
    recs = _keys(np.random.default_rng(51), 1, suites=(0,))
    _check(oracle, recs, 4096 * 16 + 16, 61, max_payload=64)
    _check(oracle, recs, 4096 * 16, 62, max_payload=64)



def test_one_key_many_items(oracle):
    """One key, 12,300 items of small packets (about 3 items per wave on a
    256-CU part, one 1024-thread workgroup per CU) with a ragged last item."""
    recs = _keys(np.random.default_rng(71), 1, suites=(0,))
    _check(oracle, recs, 12300 * 16 - 5, 72, max_payload=48)
