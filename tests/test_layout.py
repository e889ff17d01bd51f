"""Host-side batch layout (aioquic_amd.batch.layout_packets): packet and payload
alignment, no overlaps, bytes where the descriptors say.  CPU only."""

import numpy as np
import pytest


@pytest.mark.parametrize("align,payload_align", [(1, 1), (16, 1), (1, 16), (1, 64)])
def test_layout_packets_offsets(align, payload_align):
    from aioquic_amd.batch import layout_packets

    rng = np.random.default_rng(7 + align + payload_align)
    headers = [bytes(rng.integers(0, 256, int(rng.integers(1, 60)), dtype=np.uint8)) for _ in range(200)]
    payloads = [bytes(rng.integers(0, 256, int(rng.integers(0, 1400)), dtype=np.uint8)) for _ in range(200)]
    buf, desc, size = layout_packets(headers, payloads, list(range(200)), [0] * 200, align=align,
                                     payload_align=payload_align)
    end = 0
    for i, (h, p) in enumerate(zip(headers, payloads)):
        o = int(desc[i]["in_off"])
        assert o >= end  # in order, no overlap (room for the tag included)
        assert int(desc[i]["out_off"]) == o
        if payload_align > 1:
            assert (o + len(h)) % payload_align == 0
        else:
            assert o % align == 0
        assert bytes(buf[o : o + len(h)]) == h
        assert bytes(buf[o + len(h) : o + len(h) + len(p)]) == p
        assert int(desc[i]["hdr_len"]) == len(h) and int(desc[i]["len"]) == len(p)
        end = o + len(h) + len(p) + 16
    assert size >= end and len(buf) == size
