"""Batched send / receive: the callers of the packet-protection path
(SURVEY.md sec. 8(f) rows 1-2), one device launch per batch instead of one per packet.

SendBatch is the deferred form of the builder's encryption.
  In aioquic, QuicPacketBuilder._end_packet encrypts each packet the moment it is
  closed (quic/packet_builder.py:341-350, CryptoPair.encrypt_packet,
  quic/crypto.py:194-199).  A SendBatch collects (crypto, plain_header,
  plain_payload, packet_number) for every packet of a datagrams_to_send call,
  across connections, and flush() protects them all in ONE launch.  It returns
  exactly the bytes each encrypt_packet call would have returned.

ReceiveBatch is the batched form of QuicConnection.receive_datagram's decrypt
step (quic/connection.py:905-947, CryptoPair.decrypt_packet, crypto.py:184-192).
  Items are (crypto pair, packet, encrypted_offset, expected packet number or a
  packet-number space).  run() unprotects them in one launch, and in a second
  launch only for packets whose key-phase bit flipped (crypto.py:91-96).  The
  result is the same per-packet outcome as calling pair.decrypt_packet item by
  item, in order:
    * a successful key-phase flip rolls the pair's keys (crypto.py:190-191,
      _update_key "remote_update") before later packets of the same pair;
    * with a space, expected_packet_number advances as connection.py:984-985
      does, and a later packet's truncated number is decoded against it.
  A later packet whose outcome could depend on such an update is relaunched.
  A packet decoded under the earlier expected number whose decoded value is
  unchanged used the same nonce, so its result stands.  Each round resolves at
  least the first pending packet of every pair, so run() ends after at most
  1 + (state changes) rounds.
  Outcomes are (plain_header, payload, packet_number) tuples or the exception
  the reference raises: KeyUnavailableError -> "key_unavailable" drop,
  CryptoError -> "payload_decrypt_error" drop (connection.py:911-947).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Union

import numpy as np

from . import layout as L
from ._crypto import CryptoError, KeyTable, protect_host, unprotect_host
from .crypto import CryptoContext, CryptoPair, KeyUnavailableError, next_key_phase
from .packet import decode_packet_number

__all__ = ["SendBatch", "ReceiveBatch", "KeySlots"]


class KeySlots:
    """One device key table shared by every context in a batch.

    A slot is keyed by the identity of a context's (AEAD, HeaderProtection,
    key phase).  Those objects are immutable once built, so a slot never goes
    stale.  Objects are kept alive while slotted, so their ids stay unique.
    When the table is full it is cleared and refilled; that happens only
    between launches."""

    def __init__(self, capacity: int = 1024) -> None:
        self.capacity = int(capacity)
        self.table = KeyTable(self.capacity)
        self._slot: dict = {}
        self._keep: list = []
        self._pending: list = []

    def slot_for(self, aead, hp, key_phase: int) -> int:
        ident = (id(aead), id(hp), int(key_phase))
        s = self._slot.get(ident)
        if s is not None:
            return s
        if len(self._slot) >= self.capacity:
            raise OverflowError("key table full")
        s = len(self._slot)
        self._slot[ident] = s
        self._keep.append((aead, hp))
        suite, key, iv = aead._material()
        _, hp_key = hp._material()
        self._pending.append(L.key_material(s, suite, key, iv, hp_key, key_phase))
        return s

    def reset(self) -> None:
        self._slot.clear()
        self._keep.clear()
        self._pending.clear()

    def commit(self) -> None:
        """Install the slots added since the last commit (one launch)."""
        if self._pending:
            self.table.set(np.concatenate(self._pending).tobytes())
            self._pending.clear()

    def assign(self, triples) -> list:
        """Slots for a list of (aead, hp, key_phase), refilling the table if it overflows."""
        try:
            slots = [self.slot_for(*t) for t in triples]
        except OverflowError:
            self.reset()
            uniq = {(id(a), id(h), int(k)) for a, h, k in triples}
            if len(uniq) > self.capacity:
                raise
            slots = [self.slot_for(*t) for t in triples]
        self.commit()
        return slots


def _raise_status(status: int) -> Exception:
    if status == L.S_DECRYPT:
        return CryptoError("Payload decryption failed")
    if status == L.S_NO_KEY:
        return KeyUnavailableError("Decryption key is not available")
    return CryptoError("Invalid payload length")


def _context_of(crypto) -> CryptoContext:
    return crypto.send if isinstance(crypto, CryptoPair) else crypto


# ------------------------------------------------------------------ send --


@dataclass
class _SendItem:
    aead: object
    hp: object
    key_phase: int
    header: bytes
    payload: bytes
    pn: int


class SendBatch:
    """Deferred packet encryption for QuicPacketBuilder (packet_builder.py:341-350)."""

    def __init__(self, slots: Optional[KeySlots] = None, capacity: int = 1024) -> None:
        self.slots = slots or KeySlots(capacity)
        self._items: list[_SendItem] = []

    def __len__(self) -> int:
        return len(self._items)

    def add(self, crypto: Union[CryptoPair, CryptoContext], plain_header: bytes,
            plain_payload: bytes, packet_number: int) -> int:
        """Queue one packet; returns its index in flush()'s result.

        The context's state is captured NOW, as CryptoPair.encrypt_packet would
        use it at this point (including a pending local key update,
        crypto.py:194-199)."""
        if isinstance(crypto, CryptoPair) and crypto._update_key_requested:
            crypto._update_key("local_update")
        ctx = _context_of(crypto)
        assert ctx.is_valid(), "Encryption key is not available"
        self._items.append(_SendItem(ctx.aead, ctx.hp, ctx.key_phase, bytes(plain_header),
                                     bytes(plain_payload), int(packet_number)))
        return len(self._items) - 1

    def flush(self) -> list[bytes]:
        """Protect every queued packet in one launch; returns the wire bytes in
        add() order.  Raises CryptoError("Invalid payload length") for the
        first packet that the reference would reject."""
        items, self._items = self._items, []
        if not items:
            return []
        n = len(items)
        slots = self.slots.assign([(it.aead, it.hp, it.key_phase) for it in items])
        hl = np.fromiter((len(it.header) for it in items), np.int64, n)
        pl = np.fromiter((len(it.payload) for it in items), np.int64, n)
        out_sz = hl + pl + L.TAG_LEN
        offs = np.zeros(n, np.int64)
        np.cumsum(out_sz[:-1], out=offs[1:])
        desc = np.zeros(n, dtype=L.DESC)
        desc["in_off"] = offs
        desc["out_off"] = offs
        desc["len"] = pl
        desc["hdr_len"] = np.minimum(hl, 0xFFFF)
        desc["pn"] = np.fromiter((it.pn & 0xFFFFFFFFFFFFFFFF for it in items), np.uint64, n)
        desc["slot"] = slots
        # each packet occupies its output-sized region of the input (spare tag room)
        data = b"".join(it.header + it.payload + bytes(L.TAG_LEN) for it in items)
        total = int(offs[-1] + out_sz[-1])
        for i, it in enumerate(items):
            if len(it.header) > L.MAX_HDR:
                raise CryptoError("Invalid payload length")
        out, res = protect_host(self.slots.table, desc.tobytes(), data, total)
        r = np.frombuffer(res, dtype=L.RESULT)
        bad = np.nonzero(r["status"] != L.S_OK)[0]
        if len(bad):
            raise _raise_status(int(r["status"][bad[0]]))
        mv = memoryview(out)
        return [bytes(mv[o : o + s]) for o, s in zip(offs.tolist(), out_sz.tolist())]


# --------------------------------------------------------------- receive --


class _Space:
    """Holder for an explicit expected packet number (no tracking)."""

    __slots__ = ("expected_packet_number",)

    def __init__(self, v: int) -> None:
        self.expected_packet_number = v


@dataclass
class _RecvItem:
    pair: CryptoPair
    packet: bytes
    pn_off: int
    space: object
    track: bool


def _signed_trunc(pn: int, pn_len: int) -> int:
    t = pn & ((1 << (8 * pn_len)) - 1)
    # HeaderProtection.remove hands the truncated number over as a C int
    # (_crypto.c:349): a 4-byte value >= 2^31 arrives negative
    if pn_len == 4 and t >= 1 << 31:
        t -= 1 << 32
    return t


class ReceiveBatch:
    """Batched CryptoPair.decrypt_packet for QuicConnection.receive_datagram."""

    def __init__(self, slots: Optional[KeySlots] = None, capacity: int = 1024) -> None:
        self.slots = slots or KeySlots(capacity)
        self._items: list[_RecvItem] = []
        self.launches = 0

    def __len__(self) -> int:
        return len(self._items)

    def add(self, pair: CryptoPair, packet: bytes, encrypted_offset: int,
            expected_packet_number: Optional[int] = None, space=None) -> int:
        """Queue one packet.  Give either an explicit expected packet number or
        a packet-number space (any object with .expected_packet_number), which
        run() then advances as connection.py:984-985 does."""
        if (expected_packet_number is None) == (space is None):
            raise ValueError("give exactly one of expected_packet_number / space")
        track = space is not None
        sp = space if track else _Space(int(expected_packet_number))
        self._items.append(_RecvItem(pair, bytes(packet), int(encrypted_offset), sp, track))
        return len(self._items) - 1

    def _launch(self, idx, keys, expected):
        """One unprotect launch over items idx with (aead, hp, key_phase) keys;
        returns (out bytes, results, offsets)."""
        items = [self._items[i] for i in idx]
        n = len(items)
        slots = self.slots.assign(keys)
        lens = np.fromiter((len(it.packet) for it in items), np.int64, n)
        offs = np.zeros(n, np.int64)
        np.cumsum(lens[:-1], out=offs[1:])
        desc = np.zeros(n, dtype=L.DESC)
        desc["in_off"] = offs
        desc["out_off"] = offs
        desc["len"] = lens
        desc["hdr_len"] = [min(it.pn_off, 0xFFFF) for it in items]
        desc["pn"] = np.asarray([e & 0xFFFFFFFFFFFFFFFF for e in expected], dtype=np.uint64)
        desc["slot"] = slots
        data = b"".join(it.packet for it in items)
        out, res = unprotect_host(self.slots.table, desc.tobytes(), data, len(data))
        self.launches += 1
        return out, np.frombuffer(res, dtype=L.RESULT), offs

    def run(self) -> list:
        items, n = self._items, len(self._items)
        outcome: list = [None] * n
        todo = list(range(n))
        while todo:
            # items whose pair has no receive key fail up front (crypto.py:78-79)
            launch = []
            for i in todo:
                if items[i].pair.recv.aead is None:
                    continue
                launch.append(i)
            # snapshot of each pair's receive keys at launch time; _update_key
            # mutates the context in place (apply_key_phase, crypto.py:148-154)
            ctx = {i: items[i].pair.recv for i in launch}
            cur = {i: (ctx[i].aead, ctx[i].hp, ctx[i].key_phase) for i in launch}
            exp_at = {i: items[i].space.expected_packet_number for i in launch}
            resA = {}
            for i in launch:
                if items[i].pn_off > L.MAX_HDR:
                    resA[i] = None  # Invalid payload length, host-side
            run_a = [i for i in launch if i not in resA]
            if run_a:
                out, r, offs = self._launch(run_a, [cur[i] for i in run_a], [exp_at[i] for i in run_a])
                for k, i in enumerate(run_a):
                    resA[i] = (out, r[k], int(offs[k]))
            # second launch: short-header packets whose key phase bit flipped,
            # on the next-phase key (same HP key), crypto.py:91-96
            flip = [i for i in run_a if int(resA[i][1]["status"]) == L.S_KEY_PHASE]
            nxt_ctx = {}
            resB = {}
            if flip:
                keys = []
                for i in flip:
                    k = id(cur[i][0])
                    if k not in nxt_ctx:
                        nxt = next_key_phase(ctx[i])
                        nxt_ctx[k] = (nxt.aead, ctx[i].hp, nxt.key_phase)
                    keys.append(nxt_ctx[k])
                out, r, offs = self._launch(flip, keys, [exp_at[i] for i in flip])
                for k, i in enumerate(flip):
                    resB[i] = (out, r[k], int(offs[k]))
            # walk in order, applying each packet's effect on its pair
            blocked: set = set()
            stale = []
            for i in todo:
                it = items[i]
                pid = id(it.pair)
                if pid in blocked:
                    stale.append(i)
                    continue
                if it.pair.recv.aead is None:
                    outcome[i] = KeyUnavailableError("Decryption key is not available")
                    continue
                rc = it.pair.recv
                if i not in cur or (rc.aead, rc.hp, rc.key_phase) != cur[i]:
                    blocked.add(pid)
                    stale.append(i)
                    continue
                got = resA[i]
                if got is None:
                    outcome[i] = CryptoError("Invalid payload length")
                    continue
                rolled = False
                if int(got[1]["status"]) == L.S_KEY_PHASE:
                    got = resB[i]
                    rolled = True
                out, r, off = got
                st = int(r["status"])
                exp_now = it.space.expected_packet_number
                if exp_now != exp_at[i] and st != L.S_OK:
                    # decoded under an expected number an earlier packet has
                    # since raised: the packet number, hence the nonce, may
                    # differ now, so a failure is not final -- relaunch
                    blocked.add(pid)
                    stale.append(i)
                    continue
                if st == L.S_OK:
                    hl, ln, pn = int(r["hdr_len"]), int(r["out_len"]), int(r["pn"])
                    if exp_now != exp_at[i]:
                        pn_len = hl - it.pn_off
                        again = decode_packet_number(_signed_trunc(pn, pn_len), pn_len * 8, exp_now)
                        if again != pn:  # decoded under a stale expected number
                            blocked.add(pid)
                            stale.append(i)
                            continue
                    outcome[i] = (bytes(out[off : off + hl]), bytes(out[off + hl : off + ln]), pn)
                    if rolled:
                        it.pair._update_key("remote_update")
                        blocked.add(pid)
                    if it.track and pn > it.space.expected_packet_number:
                        it.space.expected_packet_number = pn + 1
                else:
                    outcome[i] = _raise_status(st)
            todo = stale
        self._items = []
        return outcome
