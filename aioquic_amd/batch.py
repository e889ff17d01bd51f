"""Batch engine: protect / unprotect many packets per launch.

The per-packet API (aioquic_amd.crypto) issues one launch per packet to stay
call-compatible with aioquic.  Real throughput comes from handing the GPU a
whole batch -- every datagram of a ``datagrams_to_send`` call, or every
datagram a server socket read -- as one descriptor array.  This module is that
interface over device-resident buffers (torch tensors on ``cuda``), plus host
helpers that lay out synthetic or real packets into the descriptor format.

Layout (include/quic_pp.h):
  desc     n x 40 B  (in_off, out_off, len, hdr_len, flags, pn, slot)
  results  n x 16 B  (pn, status, hdr_len, out_len)
  keys     one device table of expanded key slots (KeyTable)
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import layout as L
from . import _crypto

__all__ = ["PacketEngine", "MultiDeviceEngine", "KeySpec", "layout_packets"]


@dataclass
class KeySpec:
    slot: int
    suite: int
    key: bytes
    iv: bytes
    hp: bytes
    key_phase: int = 0


def _ptr(t) -> int:
    return int(t.data_ptr())


class PacketEngine:
    """Device key table + launches on device buffers.

    Buffers are torch.uint8 CUDA tensors (or anything with ``data_ptr()``).
    Calls are asynchronous on ``stream`` (default: torch's current stream).

    ``bucket(desc, n)`` sorts a batch by (suite, key slot) on the device
    (qpp_plan_build); launches given ``plan=`` then run each suite over its
    own bucket and write results in the caller's order.  A server batch that
    interleaves connections wants this; a batch already grouped by key does
    not need it.
    """

    def __init__(self, capacity: int):
        self.table = _crypto.KeyTable(int(capacity))
        self._plan = None
        self._plan_cap = 0

    @property
    def capacity(self) -> int:
        return self.table.capacity

    def set_keys(self, specs) -> None:
        recs = np.concatenate(
            [L.key_material(s.slot, s.suite, s.key, s.iv, s.hp, s.key_phase) for s in specs]
        )
        self.table.set(recs.tobytes())

    def derive_keys(self, secrets: np.ndarray) -> np.ndarray:
        """Batched CryptoContext.setup on the device (qpp_keytab_derive):
        `secrets` are layout.SECRET records; returns the derived KEY_MATERIAL."""
        assert secrets.dtype == L.SECRET
        km = self.table.derive(np.ascontiguousarray(secrets).tobytes())
        return np.frombuffer(km, dtype=L.KEY_MATERIAL).copy()

    def set_key_records(self, recs: np.ndarray) -> None:
        assert recs.dtype == L.KEY_MATERIAL
        self.table.set(np.ascontiguousarray(recs).tobytes())

    @staticmethod
    def _stream(stream) -> int:
        if stream is None:
            import torch

            return int(torch.cuda.current_stream().cuda_stream)
        if isinstance(stream, int):
            return stream
        return int(stream.cuda_stream)

    def plan(self, n: int):
        """The engine's bucketing scratch for batches of up to n packets."""
        if self._plan is None or self._plan_cap < n:
            self._plan = _crypto.Plan(max(int(n), 1))
            self._plan_cap = max(int(n), 1)
        return self._plan

    def bucket(self, desc, n: int, stream=None):
        """Sort a device descriptor batch by (suite, slot); returns the plan
        to pass to protect / unprotect of descriptors with the same slots."""
        plan = self.plan(n)
        _crypto.plan_build(plan, self.table, _ptr(desc), int(n), self._stream(stream))
        return plan

    def protect(self, desc, n: int, inbuf, outbuf, results, stream=None, plan=None) -> None:
        _crypto.protect(self.table, _ptr(desc), int(n), _ptr(inbuf), _ptr(outbuf),
                        _ptr(results), self._stream(stream), plan)

    def unprotect(self, desc, n: int, inbuf, outbuf, results, stream=None, plan=None) -> None:
        _crypto.unprotect(self.table, _ptr(desc), int(n), _ptr(inbuf), _ptr(outbuf),
                          _ptr(results), self._stream(stream), plan)

    # ----------------------------------------------- host-buffer forms ----

    def protect_host(self, desc: np.ndarray, data, out_len: int):
        out, res = _crypto.protect_host(self.table, np.ascontiguousarray(desc).tobytes(),
                                        bytes(data), int(out_len))
        return np.frombuffer(out, dtype=np.uint8), np.frombuffer(res, dtype=L.RESULT)

    def unprotect_host(self, desc: np.ndarray, data, out_len: int):
        out, res = _crypto.unprotect_host(self.table, np.ascontiguousarray(desc).tobytes(),
                                          bytes(data), int(out_len))
        return np.frombuffer(out, dtype=np.uint8), np.frombuffer(res, dtype=L.RESULT)


    def protect_into(self, desc: np.ndarray, data, out: np.ndarray, results: np.ndarray) -> None:
        """protect_host into caller-owned buffers (out: uint8, results: RESULT
        array of len(desc)), reusable across batches."""
        self._into(_crypto.protect_into, desc, data, out, results)

    def unprotect_into(self, desc: np.ndarray, data, out: np.ndarray, results: np.ndarray) -> None:
        self._into(_crypto.unprotect_into, desc, data, out, results)

    def _into(self, fn, desc, data, out, results) -> None:
        desc = np.ascontiguousarray(desc, dtype=L.DESC)
        data = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8)
                                    if not isinstance(data, np.ndarray) else data.view(np.uint8).ravel())
        if not (out.flags.c_contiguous and out.flags.writeable):
            raise ValueError("out must be a writable contiguous array")
        if not (results.flags.c_contiguous and results.flags.writeable) or \
                results.nbytes < len(desc) * L.RESULT.itemsize:
            raise ValueError("results must be a writable contiguous array of len(desc) records")
        # the arrays stay referenced here for the whole call
        fn(self.table, desc.ctypes.data, len(desc), data.ctypes.data, data.nbytes,
           out.ctypes.data, out.nbytes, results.ctypes.data)


class MultiDeviceEngine:
    """Host-buffer batches split over several GPUs of the node (qpp_multi):
    the batch's descriptors are cut into contiguous ranges, one per device,
    each device holds its own replica of the key table and its own pinned
    staging, and the results come back in the caller's order -- the bytes of
    PacketEngine.protect_host on one device.  `devices` defaults to every
    visible GPU; a device may be listed twice (two sessions on one GPU)."""

    def __init__(self, capacity: int, devices=None):
        if devices is None:
            import torch

            devices = list(range(torch.cuda.device_count()))
        self.devices = list(devices)
        self.multi = _crypto.MultiSession(self.devices, int(capacity))

    def set_key_records(self, recs: np.ndarray) -> None:
        assert recs.dtype == L.KEY_MATERIAL
        self.multi.set_keys(np.ascontiguousarray(recs).tobytes())

    def protect_host(self, desc: np.ndarray, data, out_len: int):
        out, res = self.multi.protect(np.ascontiguousarray(desc).tobytes(), bytes(data), int(out_len))
        return np.frombuffer(out, dtype=np.uint8), np.frombuffer(res, dtype=L.RESULT)

    def unprotect_host(self, desc: np.ndarray, data, out_len: int):
        out, res = self.multi.unprotect(np.ascontiguousarray(desc).tobytes(), bytes(data), int(out_len))
        return np.frombuffer(out, dtype=np.uint8), np.frombuffer(res, dtype=L.RESULT)

    def protect_into(self, desc: np.ndarray, data: np.ndarray, out: np.ndarray, results: np.ndarray) -> None:
        """protect_host into caller-owned arrays, reusable across batches."""
        _into_arrays(self.multi.protect_into, desc, data, out, results)

    def unprotect_into(self, desc: np.ndarray, data: np.ndarray, out: np.ndarray, results: np.ndarray) -> None:
        _into_arrays(self.multi.unprotect_into, desc, data, out, results)

    def trace(self, enable=None) -> list:
        """Per device, the host-copy / PCIe / kernel phases of its session's
        last traced pipelined call (qpp_multi_trace); enable=True / False turns
        tracing on / off for the following calls."""
        return self.multi.trace(-1 if enable is None else int(bool(enable)))


def _into_arrays(fn, desc, data, out, results) -> None:
    desc = np.ascontiguousarray(desc, dtype=L.DESC)
    data = np.ascontiguousarray(data).view(np.uint8).ravel()
    if not (out.flags.c_contiguous and out.flags.writeable):
        raise ValueError("out must be a writable contiguous array")
    if not (results.flags.c_contiguous and results.flags.writeable) or \
            results.nbytes < len(desc) * L.RESULT.itemsize:
        raise ValueError("results must be a writable contiguous array of len(desc) records")
    fn(desc.ctypes.data, len(desc), data.ctypes.data, data.nbytes, out.ctypes.data, out.nbytes,
       results.ctypes.data)


def layout_packets(headers, payloads, pns, slots, *, align: int = 1, tag_room: bool = True,
                   flags: int = 0, payload_align: int = 1):
    """Pack (header, payload) pairs into one input buffer and build protect
    descriptors whose outputs go to the same offsets of an output buffer.

    align: each packet starts on a multiple of it.  payload_align: each
    packet is placed so that its payload (after the header) starts on a
    multiple of it instead -- 16 saves the kernels' 16-byte loads and stores
    a second segment each (Payload alignment).

    Returns (inbuf uint8 array, desc array, out_size)."""
    n = len(headers)
    desc = np.zeros(n, dtype=L.DESC)
    sizes = [len(h) + len(p) + (L.TAG_LEN if tag_room else 0) for h, p in zip(headers, payloads)]
    offs = np.zeros(n, dtype=np.int64)
    pos = 0
    for i, s in enumerate(sizes):
        if payload_align > 1:
            hl = len(headers[i])
            pos = (pos + hl + payload_align - 1) // payload_align * payload_align - hl
        else:
            pos = (pos + align - 1) // align * align
        offs[i] = pos
        pos += s
    buf = np.zeros(pos + 16, dtype=np.uint8)
    for i, (h, p) in enumerate(zip(headers, payloads)):
        o = int(offs[i])
        buf[o : o + len(h)] = np.frombuffer(h, dtype=np.uint8)
        buf[o + len(h) : o + len(h) + len(p)] = np.frombuffer(p, dtype=np.uint8)
    desc["in_off"] = offs
    desc["out_off"] = offs
    desc["len"] = [len(p) for p in payloads]
    desc["hdr_len"] = [len(h) for h in headers]
    desc["pn"] = np.asarray(pns, dtype=np.uint64)
    desc["slot"] = np.asarray(slots, dtype=np.uint32)
    desc["flags"] = flags
    return buf, desc, pos + 16
