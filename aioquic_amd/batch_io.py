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
  unchanged used the same nonce, so its result stands -- a failed one too
  (forged or corrupt packets cost no extra launch).  Each round resolves at
  least the first pending packet of every pair, so run() ends after at most
  1 + (state changes) rounds.
  Outcomes are (plain_header, payload, packet_number) tuples or the exception
  the reference raises: KeyUnavailableError -> "key_unavailable" drop,
  CryptoError -> "payload_decrypt_error" drop (connection.py:911-947).
  Items may name their connection and its reserved-bit mask (receive_datagram's
  check after the decrypt, connection.py:949-960): a packet that authenticates
  with a reserved bit set gives ReservedBitsError, closes its connection and
  leaves the expected number alone; every later packet of a closed connection
  gives ConnectionClosedError without touching any state (:756-757).
"""

from __future__ import annotations

import threading
import weakref
from typing import Optional, Union

import numpy as np

from . import crypto as crypto_mod
from . import layout as L
from ._crypto import CryptoError, KeyTable, protect_list, unprotect_list, unprotect_walk
from .crypto import CryptoContext, CryptoPair, KeyUnavailableError, next_key_phase
from .packet import decode_packet_number

__all__ = ["SendBatch", "ReceiveBatch", "KeySlots", "ReservedBitsError", "ConnectionClosedError"]

# host-side statuses of the C receive walks (_crypto_ext.c WALK_S_*)
_S_RESERVED, _S_CLOSED = 0x101, 0x102
_NO_CONN = 0xFFFFFFFF


class ReservedBitsError(Exception):
    """The packet authenticated but carries a reserved header bit: the
    reference closes the connection (PROTOCOL_VIOLATION, connection.py:949-960)."""


class ConnectionClosedError(Exception):
    """The packet's connection was closed by an earlier packet of the batch;
    the reference ignores it (connection.py:756-757)."""


class KeySlots:
    """One device key table shared by every context in a batch.

    A slot is keyed by the identity of a context's (AEAD, HeaderProtection,
    key phase).  Those objects are immutable once built, so a slot never goes
    stale.  Objects are kept alive while slotted, so their ids stay unique,
    until their context lets them go: CryptoContext.teardown and a key update
    (apply_key_phase) release them here (``release``), which frees the slot
    and clears its device entry, as the reference drops its EVP contexts.
    When the table is full it is cleared and refilled; that happens only
    between launches.

    Like the reference's AEAD objects, a KeySlots is not meant to be shared
    by threads; the batched callers' default table is one per thread.  A
    release that another thread triggers (a context torn down there) is
    queued and applied by the table's own thread at its next assign(),
    commit(), release() or close(), so no thread changes another's table
    (close() lets an owner that stops assigning apply the queue and free every
    slot at once)."""

    def __init__(self, capacity: int = 1024) -> None:
        self.capacity = int(capacity)
        self.table = KeyTable(self.capacity)
        self._slot: dict = {}
        self._keep: dict = {}  # slot -> (aead, hp)
        self._free: list = []
        self._by_obj: dict = {}  # id(aead or hp) -> idents using it
        self._pending: list = []
        self._owner = threading.get_ident()
        self._inbox: list = []  # releases queued by other threads
        self._inbox_lock = threading.Lock()
        with _holders_lock:
            _holders.add(self)

    def slot_for(self, aead, hp, key_phase: int) -> int:
        ident = (id(aead), id(hp), int(key_phase))
        s = self._slot.get(ident)
        if s is not None:
            return s
        if self._free:
            s = self._free.pop()
        elif len(self._keep) < self.capacity:
            s = len(self._keep)
        else:
            raise OverflowError("key table full")
        self._slot[ident] = s
        self._keep[s] = (aead, hp)
        self._by_obj.setdefault(ident[0], []).append(ident)
        self._by_obj.setdefault(ident[1], []).append(ident)
        suite, key, iv = aead._material()
        _, hp_key = hp._material()
        self._pending.append(L.key_material(s, suite, key, iv, hp_key, key_phase))
        return s

    def reset(self) -> None:
        self._slot.clear()
        self._keep.clear()
        self._free.clear()
        self._by_obj.clear()
        self._pending.clear()

    def commit(self) -> None:
        """Install the slots added since the last commit (one launch)."""
        if self._inbox:
            self._drain()
        if self._pending:
            self.table.set(np.concatenate(self._pending).tobytes())
            self._pending.clear()

    def assign(self, triples) -> list:
        """Slots for a list of (aead, hp, key_phase), refilling the table if it overflows."""
        if self._inbox:
            self._drain()
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

    def release(self, objs) -> None:
        """Forget every slot built from one of `objs` (AEAD or HP objects)
        and clear those device entries."""
        if self._inbox:
            self._drain()
        dropped = set()
        for o in objs:
            for k in self._by_obj.pop(id(o), ()) if o is not None else ():
                s = self._slot.pop(k, None)
                if s is None:
                    continue  # already gone through its other object
                self._keep.pop(s, None)
                self._free.append(s)
                dropped.add(s)
                # the ident leaves the other object's list too
                for other in (k[0], k[1]):
                    lst = self._by_obj.get(other)
                    if lst is not None and other != id(o):
                        try:
                            lst.remove(k)
                        except ValueError:
                            pass
                        if not lst:
                            del self._by_obj[other]
        if not dropped:
            return
        self._pending = [m for m in self._pending if int(m["slot"][0]) not in dropped]
        self.table.clear(np.asarray(sorted(dropped), np.uint32).tobytes())

    def _queue_release(self, objs) -> None:
        with self._inbox_lock:
            self._inbox.append(objs)

    def _drain(self) -> None:
        with self._inbox_lock:
            todo, self._inbox = self._inbox, []
        for objs in todo:
            self.release(objs)

    def close(self) -> None:
        """The owner is done with the table: apply queued releases, then
        clear every device entry still held and drop the held objects."""
        self._drain()
        held = sorted(self._keep)
        if held:
            self.table.clear(np.asarray(held, np.uint32).tobytes())
        self.reset()


# every live KeySlots, so that a context's teardown can release its keys;
# registration and the snapshot below under one lock (a WeakSet's iterator
# fails if another thread adds to it meanwhile)
_holders: "weakref.WeakSet[KeySlots]" = weakref.WeakSet()
_holders_lock = threading.Lock()


def _release_keys(*objs) -> None:
    me = threading.get_ident()
    with _holders_lock:
        holders = list(_holders)
    for h in holders:
        if h._owner == me:
            h.release(objs)
        else:
            h._queue_release(objs)  # applied by the table's own thread


crypto_mod._KEY_RELEASE_HOOKS.append(_release_keys)

_per_thread = threading.local()


def default_slots() -> KeySlots:
    """The batched callers' default key table (the builders' flush and
    receive_datagrams): one per OS thread, so concurrent batches on different
    threads never assign or reset each other's slots (the C extension gives
    each thread its own staging the same way)."""
    t = getattr(_per_thread, "slots", None)
    if t is None:
        t = _per_thread.slots = KeySlots(4096)
    return t


def _raise_status(status: int) -> Exception:
    if status == _S_RESERVED:
        return ReservedBitsError("Reserved bits must be zero")
    if status == _S_CLOSED:
        return ConnectionClosedError("Connection is closed")
    if status == L.S_DECRYPT:
        return CryptoError("Payload decryption failed")
    if status == L.S_NO_KEY:
        return KeyUnavailableError("Decryption key is not available")
    if status == L.S_INTERNAL:
        return CryptoError(L.INTERNAL_ERROR)
    return CryptoError("Invalid payload length")


def _context_of(crypto) -> CryptoContext:
    return crypto.send if isinstance(crypto, CryptoPair) else crypto


# ------------------------------------------------------------------ send --


class _KeyRefs:
    """Distinct (aead, hp, key_phase) triples of a batch, by identity, so a
    batch resolves key slots once per connection rather than per packet
    (with the context each came from, when given)."""

    __slots__ = ("index", "triples", "ctxs")

    def __init__(self) -> None:
        self.index: dict = {}
        self.triples: list = []
        self.ctxs: list = []

    def ref(self, aead, hp, key_phase: int, ctx=None) -> int:
        k = (id(aead), id(hp), key_phase)
        r = self.index.get(k)
        if r is None:
            r = self.index[k] = len(self.triples)
            self.triples.append((aead, hp, key_phase))
            self.ctxs.append(ctx)
        return r

    def superseded(self) -> list:
        """AEADs whose context moved on (a key update) since they were added:
        their release already ran, so a slot made for them now is stale."""
        return [t[0] for t, c in zip(self.triples, self.ctxs) if c is not None and c.aead is not t[0]]

    def slots(self, table: KeySlots, refs: list) -> bytes:
        per = np.asarray(table.assign(self.triples), dtype=np.uint32)
        return per[np.asarray(refs, dtype=np.int64)].tobytes()


class SendBatch:
    """Deferred packet encryption for QuicPacketBuilder (packet_builder.py:341-350)."""

    def __init__(self, slots: Optional[KeySlots] = None, capacity: int = 1024) -> None:
        self.slots = slots or KeySlots(capacity)
        self._reset()

    def _reset(self) -> None:
        self._keys = _KeyRefs()
        self._refs: list = []
        self._headers: list = []
        self._payloads: list = []
        self._pns: list = []

    def __len__(self) -> int:
        return len(self._refs)

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
        self._refs.append(self._keys.ref(ctx.aead, ctx.hp, ctx.key_phase, ctx))
        self._headers.append(bytes(plain_header))
        self._payloads.append(bytes(plain_payload))
        self._pns.append(packet_number & 0xFFFFFFFFFFFFFFFF)
        return len(self._refs) - 1

    def flush(self) -> list:
        """Protect every queued packet in one launch; returns the wire bytes in
        add() order.  Raises CryptoError("Invalid payload length") for the
        first packet that the reference would reject."""
        keys, refs, headers, payloads, pns = self._keys, self._refs, self._headers, self._payloads, self._pns
        self._reset()
        if not refs:
            return []
        if max(map(len, headers)) > L.MAX_HDR:
            raise CryptoError("Invalid payload length")
        slots = keys.slots(self.slots, refs)
        wires, res = protect_list(self.slots.table, slots, np.asarray(pns, np.uint64).tobytes(),
                                  headers, payloads)
        old = keys.superseded()
        if old:
            self.slots.release(old)
        status = np.frombuffer(res, dtype=L.RESULT)["status"]
        bad = np.flatnonzero(status != L.S_OK)
        if len(bad):
            raise _raise_status(int(status[bad[0]]))
        return wires


# --------------------------------------------------------------- receive --


class _Space:
    """Holder for an explicit expected packet number (no tracking)."""

    __slots__ = ("expected_packet_number",)

    def __init__(self, v: int) -> None:
        self.expected_packet_number = v


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
        self._pairs: list = []
        self._packets: list = []
        self._offs: list = []
        self._spaces: list = []
        self._track: list = []
        self._conns: list = []  # connection key per item (None: none)
        self._rsv: list = []    # reserved-bit mask per item (0: no check)
        self._closed: set = set()  # connections closed by the walk so far
        self.launches = 0

    def __len__(self) -> int:
        return len(self._pairs)

    def add(self, pair: CryptoPair, packet: bytes, encrypted_offset: int,
            expected_packet_number: Optional[int] = None, space=None, conn=None, reserved_mask: int = 0) -> int:
        """Queue one packet.  Give either an explicit expected packet number or
        a packet-number space (any object with .expected_packet_number), which
        run() then advances as connection.py:984-985 does.  `conn` (any
        object, by identity) and `reserved_mask` (0x18 for a short header,
        0x0C for a long one) add receive_datagram's reserved-bit close."""
        if (expected_packet_number is None) == (space is None):
            raise ValueError("give exactly one of expected_packet_number / space")
        track = space is not None
        self._pairs.append(pair)
        self._packets.append(bytes(packet))
        self._offs.append(int(encrypted_offset))
        self._spaces.append(space if track else _Space(int(expected_packet_number)))
        self._track.append(track)
        self._conns.append(conn)
        self._rsv.append(int(reserved_mask) & 0xFF)
        return len(self._pairs) - 1

    def _extend(self, pairs: list, packets: list, offs: list, spaces: list, conns: Optional[list] = None,
                rsv: int = 0) -> None:
        """add() for many packets at once, each with a tracked space (the
        batched receive walk's form: packets are bytes, no copies)."""
        self._pairs += pairs
        self._packets += packets
        self._offs += offs
        self._spaces += spaces
        self._track += [True] * len(pairs)
        self._conns += conns if conns is not None else [None] * len(pairs)
        self._rsv += [rsv] * len(pairs)

    def _fast_round(self, outcome: list) -> list:
        """The first round in C (_crypto.unprotect_walk): one launch and the
        in-order walk for every packet whose outcome no state change of this
        round can alter; returns the deferred items (in order) for the
        general rounds of run().  Every item goes to the walk, those without a
        receive key or with a packet-number offset past the header limit too
        (the walk fails them by their slot and offset), so a closed
        connection's packets come back closed in order."""
        pairs, spaces, offs, track, conns = self._pairs, self._spaces, self._offs, self._track, self._conns
        n = len(pairs)
        if not n:
            return []
        # pairs, spaces and connections by identity, each resolved once
        pix: dict = {}
        six: dict = {}
        cix: dict = {}
        p_of = [pix.setdefault(id(p), len(pix)) for p in pairs]
        s_of = [six.setdefault(id(sp), len(six)) for sp in spaces]
        c_of = [_NO_CONN if c is None else cix.setdefault(id(c), len(cix)) for c in conns]
        upairs = [None] * len(pix)
        for p, k in zip(pairs, p_of):
            upairs[k] = p
        uspaces = [None] * len(six)
        for sp, k in zip(spaces, s_of):
            uspaces[k] = sp
        keyed = [k for k, p in enumerate(upairs) if p.recv.aead is not None]
        pslot = np.full(len(upairs), 0xFFFFFFFF, np.uint32)
        if keyed:
            keys = _KeyRefs()
            prefs = [keys.ref(upairs[k].recv.aead, upairs[k].recv.hp, upairs[k].recv.key_phase) for k in keyed]
            pslot[keyed] = np.asarray(self.slots.assign(keys.triples), dtype=np.uint32)[np.asarray(prefs, np.int64)]
        p_arr = np.asarray(p_of, dtype=np.uint32)
        s_arr = np.asarray(s_of, dtype=np.uint32)
        sexp = np.asarray([sp.expected_packet_number & 0xFFFFFFFFFFFFFFFF for sp in uspaces], dtype=np.uint64)
        outs, res, deferred, sexp2, closed = unprotect_walk(
            self.slots.table, pslot[p_arr].tobytes(), sexp[s_arr].tobytes(), self._packets,
            np.asarray([min(o, 0xFFFF) for o in offs], np.uint32).tobytes(),
            p_arr.tobytes(), s_arr.tobytes(), np.asarray(track, np.uint8).tobytes(),
            sexp.tobytes(), len(upairs), np.asarray(c_of, np.uint32).tobytes(),
            np.asarray(self._rsv, np.uint8).tobytes(), bytes(len(cix)))
        self.launches += 1
        # outcomes: successes come as (header, payload, pn); failures by status
        st = np.frombuffer(res, dtype=L.RESULT)["status"]
        fail = np.flatnonzero(st != L.S_OK)
        dset = set(deferred)
        for k in fail.tolist():
            if k not in dset:
                outs[k] = _raise_status(int(st[k]))
        outcome[:] = outs
        # the spaces' expected numbers after the walk (only tracked spaces move)
        new = np.frombuffer(sexp2, dtype=np.uint64)
        for k in np.flatnonzero(new != sexp).tolist():
            uspaces[k].expected_packet_number = int(new[k])
        if cix:
            ckeys = [None] * len(cix)
            for c in conns:
                if c is not None:
                    ckeys[cix[id(c)]] = c
            self._closed.update(id(ckeys[k]) for k, f in enumerate(closed) if f)
        return list(deferred)

    def _launch(self, idx: list, triples: list, expected: list):
        """One unprotect launch over items idx with per-item (aead, hp,
        key_phase); returns (list of (header, payload) | None, status list,
        pn list, hdr_len list)."""
        keys = _KeyRefs()
        refs = [keys.ref(*t) for t in triples]
        slots = keys.slots(self.slots, refs)
        outs, res = unprotect_list(self.slots.table, slots,
                                   np.asarray([e & 0xFFFFFFFFFFFFFFFF for e in expected], np.uint64).tobytes(),
                                   [self._packets[i] for i in idx],
                                   np.asarray([min(self._offs[i], 0xFFFF) for i in idx], np.uint32).tobytes())
        self.launches += 1
        r = np.frombuffer(res, dtype=L.RESULT)
        return outs, r["status"].tolist(), r["pn"].tolist(), r["hdr_len"].tolist()

    def _walk(self, todo, speculate, r_out, r_st, r_pn, r_hl, exp_at, rolled_at):
        """One round's in-order walk over the launch results, with every state
        change deferred: returns (outcomes by item, stale items, speculated
        items [(item, expected number)], pairs to roll, {space: (space, new
        expected number)}, connections closed).  Keys change only at a roll,
        which blocks its pair for the rest of the round, so every unblocked
        pair still has its launch-time keys.  A stale item blocks its
        connection as well: whether it closes the connection is not known.

        A packet decoded under an expected number an earlier packet has since
        raised needs another launch only if its number (hence nonce) decodes
        differently now.  A failed tag check reports its number too; length
        and missing-key failures do not depend on the expected number.  With
        `speculate`, such a failed packet is taken to fail again (a corrupt
        or forged packet does, whatever its number) and listed for one
        confirming launch instead of blocking its pair."""
        pairs, spaces, track, offs = self._pairs, self._spaces, self._track, self._offs
        conns, rsv, closed = self._conns, self._rsv, self._closed
        got: dict = {}
        stale, spec, rolls = [], [], []
        blocked: set = set()
        bconn: set = set()
        closing: set = set()
        exp: dict = {}
        for i in todo:
            pair = pairs[i]
            cid = None if conns[i] is None else id(conns[i])
            if (blocked and id(pair) in blocked) or (bconn and cid in bconn):
                stale.append(i)
                if cid is not None:
                    bconn.add(cid)
                continue
            if cid is not None and (cid in closed or cid in closing):
                got[i] = ConnectionClosedError("Connection is closed")  # connection.py:756-757
                continue
            if pair.recv.aead is None:
                got[i] = KeyUnavailableError("Decryption key is not available")
                continue
            status = r_st[i]
            if status is None:  # the offset check failed
                got[i] = CryptoError("Invalid payload length")
                continue
            space = spaces[i]
            held = exp.get(id(space))
            exp_now = held[1] if held else space.expected_packet_number
            pn = r_pn[i]
            if exp_now != exp_at[i] and status in (L.S_OK, L.S_DECRYPT):
                pn_len = r_hl[i] - offs[i]
                if decode_packet_number(_signed_trunc(pn, pn_len), pn_len * 8, exp_now) != pn:
                    if speculate and status == L.S_DECRYPT:
                        spec.append((i, exp_now))
                        got[i] = _raise_status(status)
                        continue
                    blocked.add(id(pair))
                    stale.append(i)
                    if cid is not None:
                        bconn.add(cid)
                    continue
            if status != L.S_OK:
                got[i] = _raise_status(status)
                continue
            out = r_out[i]
            if i in rolled_at:
                # the key update inside decrypt_packet stands (crypto.py:184-192)
                rolls.append(pair)
                blocked.add(id(pair))
            if rsv[i] and out[0] and out[0][0] & rsv[i]:
                # connection.py:949-960: close before :984-985 raises the number
                got[i] = ReservedBitsError("Reserved bits must be zero")
                if cid is not None:
                    closing.add(cid)
                continue
            got[i] = (out[0], out[1], pn)
            if track[i] and pn > exp_now:
                exp[id(space)] = (space, pn + 1)
        return got, stale, spec, rolls, exp, closing

    def run(self) -> list:
        pairs, spaces, offs = self._pairs, self._spaces, self._offs
        n = len(pairs)
        outcome: list = [None] * n
        # the first round in C; the general rounds below take what it defers
        todo = self._fast_round(outcome)
        # per item of the current round, by item index
        r_out: list = [None] * n
        r_st: list = [None] * n
        r_pn: list = [0] * n
        r_hl: list = [0] * n
        exp_at: list = [0] * n
        while todo:
            # items whose pair has no receive key fail up front (crypto.py:78-79);
            # a pn offset beyond the header limit fails host-side (length)
            launch = [i for i in todo if pairs[i].recv.aead is not None and offs[i] <= L.MAX_HDR]
            keys = []
            used: dict = {}  # item -> the (aead, hp, key_phase) it was decrypted with
            for i in launch:
                rc = pairs[i].recv
                keys.append((rc.aead, rc.hp, rc.key_phase))
                used[i] = keys[-1]
                exp_at[i] = spaces[i].expected_packet_number
            flip = []
            if launch:
                outs, st, pn, hl = self._launch(launch, keys, [exp_at[i] for i in launch])
                for k, i in enumerate(launch):
                    r_out[i], r_st[i], r_pn[i], r_hl[i] = outs[k], st[k], pn[k], hl[k]
                    if st[k] == L.S_KEY_PHASE:
                        flip.append((i, keys[k]))
            # second launch: short-header packets whose key phase bit flipped,
            # on the next-phase key (same HP key), crypto.py:91-96
            rolled_at = set()
            if flip:
                nxt_keys: dict = {}
                triples = []
                for i, cur in flip:
                    k = id(cur[0])
                    if k not in nxt_keys:
                        nxt = next_key_phase(pairs[i].recv)
                        nxt_keys[k] = (nxt.aead, cur[1], nxt.key_phase)
                    triples.append(nxt_keys[k])
                idx = [i for i, _ in flip]
                outs, st, pn, hl = self._launch(idx, triples, [exp_at[i] for i in idx])
                for k, i in enumerate(idx):
                    r_out[i], r_st[i], r_pn[i], r_hl[i] = outs[k], st[k], pn[k], hl[k]
                    rolled_at.add(i)
                    used[i] = triples[k]
            # walk in order, applying each packet's effect on its pair
            got, stale, spec, rolls, exp, closing = self._walk(todo, True, r_out, r_st, r_pn, r_hl, exp_at,
                                                               rolled_at)
            if spec:
                # failed packets whose number now decodes differently were
                # assumed to fail again: check them all in one launch, each
                # with the keys it was tried with (no roll is applied yet)
                idx = [i for i, _ in spec]
                _, st, _, _ = self._launch(idx, [used[i] for i in idx], [e for _, e in spec])
                if any(x == L.S_OK for x in st):
                    # a packet the walk took for a failure authenticates now:
                    # walk the round again without assuming (rare)
                    got, stale, spec, rolls, exp, closing = self._walk(todo, False, r_out, r_st, r_pn, r_hl,
                                                                       exp_at, rolled_at)
                else:
                    for i, x in zip(idx, st):
                        got[i] = _raise_status(x)
            # commit the round: outcomes, expected packet numbers, key rolls
            for i, o in got.items():
                outcome[i] = o
            for space, v in exp.values():
                space.expected_packet_number = v
            for pair in rolls:
                pair._update_key("remote_update")
            if flip:
                # the retry keys were this round's own: a roll builds the
                # pair's next phase afresh
                self.slots.release([t[0] for t in nxt_keys.values()])
            self._closed |= closing
            for i in stale:
                r_st[i] = None
            todo = stale
        self._pairs, self._packets, self._offs, self._spaces, self._track = [], [], [], [], []
        self._conns, self._rsv, self._closed = [], [], set()
        return outcome
