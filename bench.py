"""Benchmark: device-resident QUIC packet protect + unprotect on MI355X.

Metric (BASELINE.json): GiB/s of device-resident AEAD protect+unprotect on
1200 B packets = packets * 1200 B / (t_protect + t_unprotect), summed over all
ranks (weak scaling: every rank owns its own shard of packets, no collective
on the data path).  One "step" = protect the batch, then unprotect it.

Default workload = the north-star configuration (BASELINE.json north_star):
AES-128-GCM protect+unprotect of 1Mi x 1200 B packets, one key, per GPU.
--config 2/3/4/5 run the other BASELINE configs.  Configs 4 and 5 arrive in
random key order (a server socket's view of many connections), so every
step buckets each batch by (suite, key) on the device (qpp_plan_build)
inside the timed region, once for the protect batch and once for the
unprotect batch.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config ns] [--no-e2e]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

After the timed region rank 0 also times the path the north star says
starts and ends in host memory (UDP socket buffers): pinned H2D -> protect ->
unprotect -> D2H on its own 1Mi-packet workload, reported as "e2e" beside
`value` and never as `value` (--no-e2e skips it).

--gpus N without a launcher (WORLD_SIZE unset) starts N rank processes
itself, one per visible GPU, before anything touches a GPU; with fewer than N
visible GPUs it refuses unless --rehearse is given (ranks then share devices
round-robin, a rehearsal of the launch path, not a scaling number).  Under a
launcher WORLD_SIZE must equal N.
"""

import argparse
import ctypes
import glob
import importlib.util
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
BYTES_PER_PKT_KERNEL = 1184 + 1200 + 40 + 16  # algorithmic HBM bytes per packet per kernel
# The GCM kernels' binding resource is the LDS array, not HBM:
# LDS-array cycles per 1200 B packet per kernel from the instruction mix
# (ds_read_b32 = 2 cycles, ds_read_b64 = 2 cycles per wave instruction,
# MI355X_MICROARCH.md sec. LDS; 5-bit GHASH windows), at 256 CUs and 2.4 GHz.
# SQ_LDS_IDX_ACTIVE measures 471 per packet for AES-128-GCM.
LDS_CYCLES_PER_PKT = {0: 478.0, 1: 638.0}  # AES-128-GCM, AES-256-GCM
N_CU, CLOCK_GHZ = 256, 2.4

CONFIGS = {
    "ns": dict(name="aes-128-gcm 1Mi x 1200B, 1 key", n=1 << 20, suite=0, n_keys=1, version=1),
    "2": dict(name="aes-128-gcm 64Ki x 1200B, 1 key", n=65536, suite=0, n_keys=1, version=1),
    "3": dict(name="chacha20-poly1305 64Ki x 1200B, 1 key, QUIC v2", n=65536, suite=2, n_keys=1,
              version=0x6B3343CF),
    "4": dict(name="aes-256-gcm 1Mi x 1200B, 4096 keys, random arrival order", n=1 << 20, suite=1,
              n_keys=4096, version=1, order="random"),
    "5": dict(name="mixed aes-128-gcm/chacha20-poly1305 2Mi x 1200B per GPU, 1024 keys, "
                   "random arrival order", n=1 << 21, suite=0, n_keys=1024, version=1,
              mixed=(0, 2), order="random"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10,
                    help="untimed steps first (the GPU clock needs ~20 ms of work to ramp)")
    ap.add_argument("--config", default="ns", choices=sorted(CONFIGS))
    ap.add_argument("--packets", type=int, default=0, help="override packets per GPU")
    ap.add_argument("--order", choices=("grouped", "round_robin", "random"), default=None,
                    help="override the config's arrival order (non-grouped orders are bucketed)")
    ap.add_argument("--keys", type=int, default=0, help="study knob: override the config's key count")
    ap.add_argument("--layout", choices=("arrival", "by_key"), default="arrival",
                    help="study knob: by_key stores each key's packets contiguously")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-all-cores", type=int, default=1,
                    help="also time the reference on every host core of this GPU's share")
    ap.add_argument("--event-every", type=int, default=1,
                    help="bracket the kernels of every N-th timed step (steps N-1, 2N-1, ...) with HIP "
                         "events (1 = all, the default: the kernels' event intervals then lie inside the "
                         "timed steps, so they sum to at most ms_per_step)")
    ap.add_argument("--sustain-seconds", type=float, default=4.0,
                    help="after the timed region (N = 1, rank 0): the same step back to back for about this "
                         "long, reported as `sustained` (steady-state clocks; never `value`; 0 = skip)")
    ap.add_argument("--e2e", dest="e2e", action="store_true", default=True,
                    help="time pinned H2D->kernels->D2H after the timed region (the default)")
    ap.add_argument("--no-e2e", dest="e2e", action="store_false", help="skip the end-to-end leg")
    ap.add_argument("--e2e-packets", type=int, default=1 << 20,
                    help="packets of the end-to-end run (the north star's 1Mi)")
    ap.add_argument("--e2e-chunks", type=int, default=32)
    ap.add_argument("--e2e-streams", type=int, default=4)
    ap.add_argument("--e2e-mode", choices=("staged", "per-chunk"), default="staged",
                    help="staged: one H2D, one compute and one D2H stream chained by events; "
                         "per-chunk: each chunk's copy/kernels/copy on one of --e2e-streams streams")
    ap.add_argument("--no-check", dest="check", action="store_false",
                    help="skip the round-trip comparison after timing (default: every byte compared)")
    ap.add_argument("--rehearse", action="store_true",
                    help="allow more ranks than visible GPUs (devices shared round-robin)")
    ap.add_argument("--master-port", type=int, default=0, help="rendezvous port of self-launched ranks")
    return ap.parse_args()


# ------------------------------------------------------------ CPU baseline --


def _load_reference():
    """oracle/_ref: the reference's own _crypto.c, built from /root/reference."""
    so = glob.glob(os.path.join(ROOT, "oracle", "_ref", "aioquic_ref", "_crypto*.so"))
    if not so:
        return None
    try:
        spec = importlib.util.spec_from_file_location("_crypto", so[0])
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        return mod
    except Exception:
        return None


_NAMES = {0: (b"aes-128-gcm", b"aes-128-ecb", 16), 1: (b"aes-256-gcm", b"aes-256-ecb", 32),
          2: (b"chacha20-poly1305", b"chacha20", 32)}


class _RefContext:
    """The call sequence of the reference's CryptoContext.encrypt_packet /
    decrypt_packet (quic/crypto.py:75-116) over its own AEAD / HeaderProtection
    objects: attribute lookups, the key-phase test and the decode of
    quic/packet.py:118-132 included (the reference's crypto.py itself cannot
    travel to the GPU box; this restates its method bodies)."""

    def __init__(self, aead, hp, key_phase=0):
        self.aead, self.hp, self.key_phase = aead, hp, key_phase

    def encrypt_packet(self, plain_header, plain_payload, packet_number):
        protected_payload = self.aead.encrypt(plain_payload, plain_header, packet_number)
        return self.hp.apply(plain_header, protected_payload)

    def decrypt_packet(self, packet, encrypted_offset, expected_packet_number):
        from aioquic_amd.packet import decode_packet_number

        plain_header, packet_number = self.hp.remove(packet, encrypted_offset)
        first_byte = plain_header[0]
        pn_length = (first_byte & 0x03) + 1
        packet_number = decode_packet_number(packet_number, pn_length * 8, expected_packet_number)
        crypto = self
        if not first_byte & 0x80:
            key_phase = (first_byte & 4) >> 2
            assert key_phase == self.key_phase  # the bench's packets never change phase
        payload = crypto.aead.decrypt(packet[len(plain_header):], plain_header, packet_number)
        return plain_header, payload, packet_number, crypto != self


def _cpu_loop(w, seconds: float, part: int = 0, parts: int = 1, samples: int = 1, mode: str = "objects"):
    """aioquic's own per-packet path over a bounded sample of the workload's
    packets, `samples` timed slices of seconds / samples each; returns
    (packets, seconds, kind, per-slice GiB/s).
    mode "objects": the AEAD / HeaderProtection calls of
    CryptoContext.encrypt_packet (AEAD.encrypt + HeaderProtection.apply) and
    decrypt_packet (remove + decode_packet_number + AEAD.decrypt) made
    directly; mode "context": through _RefContext, the methods' own bodies
    (quic/crypto.py:75-116)."""
    from aioquic_amd.packet import decode_packet_number

    ref = _load_reference()
    kind = "reference" if ref is not None else "port"
    if ref is None:
        sys.path.insert(0, ROOT)
        from oracle import oracle as orc
    m = min(w.n // parts, 20000)
    base = part * m
    pk = [bytes(w.plain[(base + i) * 1200 : (base + i) * 1200 + 1184]) for i in range(m)]
    pns = [int(x) for x in w.desc["pn"][base : base + m]]
    slots = [int(x) for x in w.desc["slot"][base : base + m]]
    # each sampled packet under its own connection's key (per-connection
    # objects, built before timing, as aioquic builds them at key install)
    objs = {}
    for sl in set(slots):
        k = w.keys[sl]
        suite = int(k["suite"])
        an, hn, kl = _NAMES[suite]
        key, iv, hp = bytes(k["key"][:kl]), bytes(k["iv"]), bytes(k["hp"][:kl])
        if ref is not None:
            objs[sl] = (ref.AEAD(an, key, iv), ref.HeaderProtection(hn, hp))
            if mode == "context":
                objs[sl] = _RefContext(*objs[sl])
        else:
            objs[sl] = (suite, key, iv, hp)
    ko = [objs[sl] for sl in slots]
    done = 0
    t_all = 0.0
    rates = []
    for _ in range(max(1, samples)):
        t_end = time.perf_counter() + seconds / max(1, samples)
        n0, t_s = done, 0.0
        while time.perf_counter() < t_end:
            t0 = time.perf_counter()
            if ref is not None and mode == "context":
                wire = [o.encrypt_packet(p[:11], p[11:], pn) for p, pn, o in zip(pk, pns, ko)]
                for x, pn, o in zip(wire, pns, ko):
                    o.decrypt_packet(x, 9, pn)
            elif ref is not None:
                wire = [o[1].apply(p[:11], o[0].encrypt(p[11:], p[:11], pn)) for p, pn, o in zip(pk, pns, ko)]
                for x, pn, o in zip(wire, pns, ko):
                    hdr, trunc = o[1].remove(x, 9)
                    pnd = decode_packet_number(trunc, ((hdr[0] & 3) + 1) * 8, pn)
                    o[0].decrypt(x[len(hdr):], hdr, pnd)
            else:
                wire = [orc.protect(o[0], o[1], o[2], o[3], p[:11], p[11:], pn) for p, pn, o in zip(pk, pns, ko)]
                for x, pn, o in zip(wire, pns, ko):
                    orc.unprotect(o[0], o[1], o[2], o[3], x, 9, pn)
            t_s += time.perf_counter() - t0
            done += m
        t_all += t_s
        rates.append((done - n0) * 1200 / t_s / GIB)
    return done, t_all, kind, rates


def _cpu_worker(args):
    w, seconds, part, parts = args
    return _cpu_loop(w, seconds, part, parts)[:3]


def cpu_share() -> int:
    """Host cores this process may use, capped at the GPU box's share (16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 16))


def host_identity():
    """(CPU model, OpenSSL_version() of the libcrypto the reference's _crypto
    links) for the baseline's line."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    ssl = None
    if _load_reference() is not None:
        try:
            paths = {ln.split()[-1] for ln in open("/proc/self/maps") if "libcrypto" in ln}
            for path in sorted(paths):
                lib = ctypes.CDLL(path)
                lib.OpenSSL_version.restype = ctypes.c_char_p
                lib.OpenSSL_version.argtypes = [ctypes.c_int]
                ssl = {"version": lib.OpenSSL_version(0).decode(), "path": path}
                break
        except (OSError, AttributeError):
            pass
    return model, ssl


def cpu_baseline(w, seconds: float, cfg, procs: int = 1, samples: int = 5):
    """The reference's CPU path timed on `procs` host cores (one process per
    core, each with its own AEAD/HP objects and packets, like one aioquic
    connection per core).  Runs BEFORE the GPU is initialised (fork).  On one
    core: the median of `samples` slices of the objects-only sequence, then
    the same through the CryptoContext method bodies."""
    extra = {}
    if procs <= 1:
        half = seconds / 2
        done, t, kind, rates = _cpu_loop(w, half, samples=samples)
        value = float(np.median(rates))
        if kind == "reference":
            _, _, _, crates = _cpu_loop(w, half, samples=samples, mode="context")
            extra = {"samples_gib_s": [round(r, 4) for r in rates], "median_of": len(rates),
                     "context_value": round(float(np.median(crates)), 4),
                     "context_samples_gib_s": [round(r, 4) for r in crates]}
        else:
            extra = {"samples_gib_s": [round(r, 4) for r in rates], "median_of": len(rates)}
    else:
        import multiprocessing as mp

        with mp.get_context("fork").Pool(procs) as pool:
            res = pool.map(_cpu_worker, [(w, seconds, i, procs) for i in range(procs)])
        done = sum(r[0] for r in res)
        kind = res[0][2]
        value = sum(r[0] * 1200 / r[1] for r in res) / GIB
    model, ssl = host_identity()
    an = "/".join(sorted({_NAMES[int(s)][0].decode() for s in w.suites[: min(w.n, 20000)]}))
    what = ("AEAD/HP objects only: AEAD.encrypt + HeaderProtection.apply, then remove + decode_packet_number + "
            "AEAD.decrypt per packet, no CryptoContext wrapper (context_value: through the bodies of "
            "CryptoContext.encrypt_packet/decrypt_packet, quic/crypto.py:75-116)"
            if kind == "reference" else "C oracle protect/unprotect per packet")
    out = {"value": round(value, 4), "unit": "GiB/s", "cores": procs, "kind": kind,
           "sample": f"{done} packets of the bench workload ({cfg['name']}), suites {an}; {what}; "
                     f"~{seconds:.0f} s on {procs} core(s) of the GPU host"
                     + (f", median of {samples} slices" if procs <= 1 else ", one slice per core, summed"),
           "cpu_model": model, "libcrypto": ssl}
    out.update(extra)
    return out


# --------------------------------------------------------------------- main --


class HipEvents:
    """Timing-only HIP events on torch's HIP runtime, created with
    hipEventReleaseToDevice (or hipEventDisableSystemFence; hip_runtime_api.h)
    so that recording one does not write back and invalidate the caches the
    way a default event does (each default event costs ~15 us of stream time
    here).  `flags` records which one the runtime accepted."""

    # preferred first; the runtime may refuse a combination
    FLAG_CHOICES = (0x40000000, 0x20000000, 0x0)  # ReleaseToDevice, DisableSystemFence, default

    def __init__(self, torch):
        lib = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
        self.hip = hip = ctypes.CDLL(lib)  # the copy torch already loaded
        vp = ctypes.c_void_p
        hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
        hip.hipEventRecord.argtypes = [vp, vp]
        hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), vp, vp]
        hip.hipEventDestroy.argtypes = [vp]
        self.events = []
        self.flags = None
        for f in self.FLAG_CHOICES:
            e = ctypes.c_void_p()
            if hip.hipEventCreateWithFlags(ctypes.byref(e), f) == 0:
                hip.hipEventDestroy(e)
                self.flags = f
                break
        if self.flags is None:
            raise RuntimeError("hipEventCreateWithFlags failed")

    def new(self):
        e = ctypes.c_void_p()
        if self.hip.hipEventCreateWithFlags(ctypes.byref(e), self.flags) != 0:
            raise RuntimeError("hipEventCreateWithFlags failed")
        self.events.append(e)
        return e

    def record(self, e, stream) -> None:
        if self.hip.hipEventRecord(e, ctypes.c_void_p(int(stream.cuda_stream))) != 0:
            raise RuntimeError("hipEventRecord failed")

    def ms(self, a, b) -> float:
        out = ctypes.c_float()
        if self.hip.hipEventElapsedTime(ctypes.byref(out), a, b) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return float(out.value)

    def close(self) -> None:
        for e in self.events:
            self.hip.hipEventDestroy(e)
        self.events = []


def hbm_copy_gbs(dev, nbytes=1 << 30, reps=10):
    """Attainable HBM bandwidth on this box: a device-to-device copy of 1 GiB
    (read + write bytes / time), the practical ceiling beside the 8 TB/s spec."""
    import torch

    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    e1.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / reps
    del a, b
    return round(2 * nbytes / t / 1e9, 1)


def measured_traffic(workload, n, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    passes (profiles/traffic.json, tools/traffic.py), when they were taken on
    this workload at this packet count."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        entry = json.load(open(path))[workload]
    except (OSError, KeyError, ValueError):
        return {}
    if entry.get("packets") != n or kernel not in entry:
        return {}
    return {"bytes": entry[kernel]["bytes"], "source": entry["source"]}


def key_schedule(eng_cls, n_keys, suite, version):
    """Batched CryptoContext.setup for n_keys connections: the device path
    (qpp_keytab_derive: HKDF + slot expansion, synchronous) against the host
    HKDF of derive_key_iv_hp (quic/crypto.py:34-56, stdlib hmac) alone."""
    from aioquic_amd import layout as L
    from aioquic_amd.crypto import derive_key_iv_hp
    from aioquic_amd.bench_data import _SUITE_TO_CS

    rng = np.random.default_rng(0x5EC)
    sl = 48 if suite == L.AES_256_GCM else 32
    secrets = [rng.bytes(sl) for _ in range(n_keys)]
    recs = np.concatenate([L.secret_record(i, suite, sc, v2=version != 1)
                           for i, sc in enumerate(secrets)])
    eng = eng_cls(n_keys)
    eng.derive_keys(recs)  # warm-up (module load, allocation)
    t0 = time.perf_counter()
    eng.derive_keys(recs)
    dev_ms = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    for sc in secrets:
        derive_key_iv_hp(cipher_suite=_SUITE_TO_CS[suite], secret=sc, version=version)
    host_ms = (time.perf_counter() - t0) * 1e3
    return {"keys": n_keys, "device_ms": round(dev_ms, 3), "host_hkdf_ms": round(host_ms, 3),
            "note": "device = HKDF-Expand-Label x3 + AES key schedule + GHASH tables per key; "
                    "host = HKDF only, 1 thread"}


METRIC = "GiB/s device-resident AEAD protect+unprotect, 1200B packets, 1/2/4/8 MI355X"


def plan_ranks(gpus: int, env: dict, visible: int, rehearse: bool):
    """How this invocation runs: ("run", None) -- this process is one rank
    (launched by torch.distributed.run, or N = 1); ("spawn", n) -- start n
    rank processes; ("refuse", reason)."""
    if gpus < 1:
        return "refuse", f"--gpus {gpus}: need at least one GPU"
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            return "refuse", f"WORLD_SIZE={world} but --gpus {gpus}: the launcher and the flag disagree"
        return "run", None
    if gpus == 1:
        return "run", None
    if visible < gpus and not rehearse:
        return "refuse", (f"--gpus {gpus} but {visible} GPU(s) visible; "
                          "pass --rehearse to share devices (not a scaling number)")
    return "spawn", gpus


def _free_port() -> int:
    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(n: int, port: int) -> int:
    """Start ranks 0..n-1 of this command as child processes (this process
    has not touched a GPU) and wait for them; returns the worst exit code."""
    import subprocess

    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    codes = [p.wait() for p in procs]
    return max(codes, key=abs)


def main():
    args = parse()
    import torch

    # device_count() does not initialise the GPU on this image: safe before a spawn
    mode, what = plan_ranks(args.gpus, os.environ, torch.cuda.device_count(), args.rehearse)
    if mode == "refuse":
        print(f"bench.py: {what}", file=sys.stderr, flush=True)
        sys.exit(2)
    if mode == "spawn":
        sys.exit(spawn_ranks(what, args.master_port or _free_port()))
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # gloo reports its connections on the C++ side's stdout: keep them out
        # of the one JSON line (fd 1 -> fd 2 while the group forms)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
        finally:
            os.dup2(saved, 1)
            os.close(saved)
    cfg = dict(CONFIGS[args.config])
    if args.keys:
        cfg["n_keys"] = args.keys
        cfg["name"] = cfg["name"].replace(f"{CONFIGS[args.config]['n_keys']} key", f"{args.keys} key")
    if args.order:
        cfg["order"] = args.order
        cfg["name"] += f" [{args.order} order]"
    n = args.packets or cfg["n"]
    from aioquic_amd.bench_data import make_workload
    from aioquic_amd.shard import shard_range

    # shard: rank r owns packets [r*n, (r+1)*n) of the global stream
    first, n = shard_range(rank, world, n)
    seed = 0x9001 + (int(args.config) if args.config.isdigit() else 0)
    w = make_workload(n, suite=cfg["suite"], n_keys=cfg["n_keys"], seed=seed,
                      version=cfg["version"], mixed=cfg.get("mixed"), first_packet=first,
                      order=cfg.get("order", "grouped"), layout=args.layout)
    if args.layout != "arrival":
        cfg["name"] += f" [{args.layout} layout]"
    bucketed = cfg.get("order", "grouped") != "grouped"
    # the CPU baselines run before anything touches the GPU (they fork), on
    # rank 0 of an N = 1 run only (the same host and sample at every N; a
    # scaling run's line carries null)
    cpu = cpu_all = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(w, args.cpu_seconds, cfg, 1)
        if args.cpu_all_cores:
            cpu_all = cpu_baseline(w, max(2.0, args.cpu_seconds / 2), cfg, cpu_share())

    # one rank per GPU; more ranks than GPUs (a rehearsal on a smaller box)
    # share devices round-robin
    ndev = torch.cuda.device_count()
    local = local % ndev if ndev else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from aioquic_amd import layout as L
    from aioquic_amd.batch import PacketEngine
    eng = PacketEngine(w.n_keys)
    eng.set_key_records(w.keys)

    d_plain = torch.from_numpy(w.plain).to(dev)
    d_desc = torch.from_numpy(w.desc.view(np.uint8)).to(dev)
    d_udesc = torch.from_numpy(w.udesc.view(np.uint8)).to(dev)
    d_wire = torch.zeros(w.wire_size, dtype=torch.uint8, device=dev)
    d_back = torch.zeros(w.plain_size, dtype=torch.uint8, device=dev)
    d_r1 = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    d_r2 = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    hev = HipEvents(torch)

    def step(ev=None):
        # bucketed configs: each batch is sorted by (suite, key) on the device
        # first -- the protect batch and the unprotect batch each get their own
        # plan build, as two independent batches of a server would.  Unbucketed
        # steps record 3 events (ev[1] / ev[3] alias ev[0] / ev[2] then).
        if ev:
            hev.record(ev[0], stream)
        plan = eng.bucket(d_desc, n, stream) if bucketed else None
        if ev and bucketed:
            hev.record(ev[1], stream)
        eng.protect(d_desc, n, d_plain, d_wire, d_r1, stream, plan)
        if ev:
            hev.record(ev[2], stream)
        plan = eng.bucket(d_udesc, n, stream) if bucketed else None
        if ev and bucketed:
            hev.record(ev[3], stream)
        eng.unprotect(d_udesc, n, d_wire, d_back, d_r2, stream, plan)
        if ev:
            hev.record(ev[4], stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    # the timed region: K steps on one stream; in every `--event-every`-th step
    # (by default every step, since round 4) each kernel sits between two
    # timing-only HIP events (its launch duration for the roofline).  The
    # records' own stream time (~6 us per step: 0.25 % of a north-star step,
    # ~3 % of config 2's) is inside `value`; --event-every 10 keeps it out of
    # 9 steps in 10, as rounds 1-3 measured.
    every = max(1, args.event_every)
    # (sampled: not the first timed step, which follows the barrier, the
    # others follow a step)
    def new_evs():
        e = [hev.new() for _ in range(5 if bucketed else 3)]
        return e if bucketed else [e[0], e[0], e[1], e[1], e[2]]

    evs = [new_evs() if k % every == every - 1 else None for k in range(args.steps)]
    if not any(evs):
        evs[-1] = new_evs()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize(dev)
    elapsed_own = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    evs = [e for e in evs if e]
    t_plan = float(np.mean([hev.ms(e[0], e[1]) + hev.ms(e[2], e[3]) for e in evs])) / 1e3
    t_prot = float(np.mean([hev.ms(e[1], e[2]) for e in evs])) / 1e3
    t_unp = float(np.mean([hev.ms(e[3], e[4]) for e in evs])) / 1e3
    hev_flags = hev.flags
    hev.close()

    # sustained: the same step back to back for a few seconds after the timed
    # region, no events (the clocks' steady state; reported beside `value`,
    # never as it); its last step's results are checked below like the
    # timed region's
    sustained = None
    if world == 1 and args.sustain_seconds > 0:
        k_s = max(1, int(args.sustain_seconds / max(elapsed / args.steps, 1e-6)))
        torch.cuda.synchronize(dev)
        t_s = time.perf_counter()
        for _ in range(k_s):
            step()
        torch.cuda.synchronize(dev)
        dt_s = time.perf_counter() - t_s
        sustained = {"steps": k_s, "seconds": round(dt_s, 3),
                     "gib_s": round(float(n) * 1200 * k_s / dt_s / GIB, 3),
                     "ms_per_step": round(dt_s / k_s * 1e3, 4),
                     "note": "the timed region's step repeated back to back after it, without timing events"}

    # after timing: every packet of the last step authenticated, and (unless
    # --no-check) the unprotected bytes equal the plaintext, every byte
    r1 = d_r1.cpu().numpy().view(L.RESULT)
    r2 = d_r2.cpu().numpy().view(L.RESULT)
    tags_ok = bool((r1["status"] == 0).all() and (r2["status"] == 0).all())
    rt_ok = bool(torch.equal(d_back, d_plain)) if args.check else None
    ok = tags_ok and rt_ok is not False
    mine = {"rank": rank, "device": local, "packets": n, "status_ok": ok, "tags_ok": tags_ok,
            "round_trip_ok": rt_ok, "seconds": round(float(elapsed_own), 6),
            "kernels_ms": {"protect": round(t_prot * 1e3, 4), "unprotect": round(t_unp * 1e3, 4)}}
    per_rank = [mine]
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    ok = all(r["status_ok"] for r in per_rank)

    total_bytes = float(n) * 1200 * args.steps * world
    value = total_bytes / elapsed / GIB
    copy_gbs = hbm_copy_gbs(dev) if rank == 0 else None
    kern_t = max(t_prot, t_unp)
    dom = "protect" if t_prot >= t_unp else "unprotect"
    achieved = BYTES_PER_PKT_KERNEL * n / kern_t / 1e9
    traffic = measured_traffic(cfg["name"], n, dom)
    floor = None
    if not cfg.get("mixed") and cfg["suite"] in LDS_CYCLES_PER_PKT:
        cyc = LDS_CYCLES_PER_PKT[cfg["suite"]]
        floor_us = cyc * n / N_CU / (CLOCK_GHZ * 1e3)
        floor = {"resource": "LDS array", "cycles_per_packet": cyc, "clock_ghz": CLOCK_GHZ,
                 "floor_us": round(floor_us, 2), "kernel_us": round(kern_t * 1e6, 2),
                 "frac": round(floor_us / (kern_t * 1e6), 4)}

    out = None
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded 1-RTT packets, 11 B header + 1173 B payload + 16 B tag)",
            "config": {"workload": _workload_name(cfg, n), "packets_per_gpu": n, "packet_bytes": 1200,
                       "keys": w.n_keys, "arrival": cfg.get("order", "grouped"),
                       "bucketed_in_timed_region": bucketed,
                       "parallelism": f"packet shards x{world}"},
            "kernels_ms": {"protect": round(t_prot * 1e3, 4), "unprotect": round(t_unp * 1e3, 4),
                           "bucketing": round(t_plan * 1e3, 4) if bucketed else None},
            "kernel_gib_s": round(n * 1200 / (t_prot + t_unp) / GIB, 3),
            "event_flags": hex(hev_flags), "event_steps": len(evs),
            "roofline": {"bound": "hbm", "kernel": dom, "launch_us": round(kern_t * 1e6, 2),
                         "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic.get("bytes"),
                         "traffic_source": traffic.get("source"),
                         "algorithmic_bytes": BYTES_PER_PKT_KERNEL * n,
                         "attainable_copy": copy_gbs,
                         "frac_of_attainable": round(achieved / copy_gbs, 4) if copy_gbs else None,
                         "compute_floor": floor},
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_all,
            "sustained": sustained,
            "status_ok": ok,
            "round_trip_checked": bool(args.check),
            "ranks": per_rank,
            "devices_visible": torch.cuda.device_count(),
            "rehearsal_shared_devices": world > torch.cuda.device_count(),
        }
        if w.n_keys >= 64:
            out["key_schedule"] = key_schedule(PacketEngine, w.n_keys, cfg["suite"], cfg["version"])
        if args.e2e:
            # the PCIe legs start from a clean host and device: the timed
            # region's buffers go first (host and device memory they held
            # otherwise sits beside the legs' own multi-GiB buffers)
            del d_plain, d_desc, d_udesc, d_wire, d_back, d_r1, d_r2, w
            torch.cuda.synchronize(dev)
            torch.cuda.empty_cache()
            # (PCIe-inclusive legs, never `value`: a failure is reported in
            # the line instead of losing it)
            if world == 1:
                try:
                    out["e2e_host_devices"] = e2e_host_devices(cfg, seed, args.e2e_packets)
                except Exception as exc:
                    out["e2e_host_devices"] = {"error": f"{type(exc).__name__}: {exc}"}
            try:
                out["e2e"] = e2e(PacketEngine, cfg, seed, dev, args.e2e_packets,
                                 chunks=args.e2e_chunks, n_streams=args.e2e_streams,
                                 mode=args.e2e_mode)
            except Exception as exc:
                out["e2e"] = {"error": f"{type(exc).__name__}: {exc}"}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _workload_name(cfg, n):
    """cfg's name, with the packet count replaced when --packets overrides it."""
    if n == cfg["n"]:
        return cfg["name"]
    def ki(x):
        return f"{x >> 20}Mi" if x % (1 << 20) == 0 else f"{x >> 10}Ki" if x % 1024 == 0 else str(x)
    return cfg["name"].replace(ki(cfg["n"]), ki(n), 1)


def L_RESULT():
    from aioquic_amd import layout as L

    return L.RESULT


def e2e_host_devices(cfg, seed, n, reps=5):
    """The library's own host-buffer path over every visible GPU
    (MultiDeviceEngine / qpp_multi: one host batch cut into contiguous ranges,
    one session and key-table replica per device, host threads in parallel):
    host memory -> protect -> host, then host -> unprotect -> host, per device
    count 1..D, from and into caller-owned pageable arrays.  PCIe-inclusive;
    never the bench value.  After the timed round trips, one more round trip
    runs with the sessions' tracing on (qpp_multi_trace: host copies in and
    out of pinned staging, H2D, kernels, D2H per call), reported as `phases`
    beside that round trip's own rate."""
    import torch
    from aioquic_amd.batch import MultiDeviceEngine
    from aioquic_amd.bench_data import make_workload

    w = make_workload(n, suite=cfg["suite"], n_keys=cfg["n_keys"], seed=seed, version=cfg["version"],
                      mixed=cfg.get("mixed"))
    out = {}
    plain = np.ascontiguousarray(w.plain)
    wire = np.empty(w.wire_size, np.uint8)
    back = np.empty(w.plain_size, np.uint8)
    r1 = np.empty(n, L_RESULT())
    r2 = np.empty(n, L_RESULT())

    def rnd(t):
        return {k: (round(v, 3) if isinstance(v, float) else v) for k, v in t.items()}

    ndev = torch.cuda.device_count()
    counts = sorted({d for d in (1, 2, 4, 8) if d <= ndev} | {ndev})
    t_start = time.perf_counter()
    for d in counts:
        if d > 1 and time.perf_counter() - t_start > 120:
            out[str(d)] = {"skipped": "the device counts before it took over 120 s"}
            continue
        try:
            out[str(d)] = _host_devices_leg(MultiDeviceEngine, w, d, plain, wire, back, r1, r2, n, reps, rnd)
        except Exception as exc:  # a leg's failure is reported in the line, not fatal to the bench
            out[str(d)] = {"error": f"{type(exc).__name__}: {exc}"}
    return {"per_device_count": out, "packets": n,
            "note": "caller-owned pageable host arrays: qpp_multi protect_into, then unprotect_into (two "
                    "synchronous calls; each a chunked pipeline: host copy into pinned staging by the library's "
                    "copy threads, H2D, kernels, D2H, copy out); median of the timed round trips; `phases` per "
                    "device session from one more, traced round trip (copy_in/copy_out: host copies, "
                    "h2d/kernel/d2h: sums of the chunks' GPU durations, submit/wait: the calling thread)"}


def _host_devices_leg(MultiDeviceEngine, w, d, plain, wire, back, r1, r2, n, reps, rnd):
    """One device count of e2e_host_devices: devices 0..d-1."""
    eng = MultiDeviceEngine(w.n_keys, devices=list(range(d)))
    eng.set_key_records(w.keys)
    eng.protect_into(w.desc, plain, wire, r1)  # warm-up (staging allocation, first touch)
    eng.unprotect_into(w.udesc, wire, back, r2)
    times = []
    for _ in range(reps):
        back[:1] ^= 1  # the round trip below must rewrite it
        t0 = time.perf_counter()
        eng.protect_into(w.desc, plain, wire, r1)
        eng.unprotect_into(w.udesc, wire, back, r2)
        times.append(time.perf_counter() - t0)
    ok = bool((r1["status"] == 0).all() and (r2["status"] == 0).all() and np.array_equal(back, plain))
    # the traced round trip (timing events on every chunk: not in `times`)
    eng.trace(True)
    t0 = time.perf_counter()
    eng.protect_into(w.desc, plain, wire, r1)
    t_p = eng.trace()
    eng.unprotect_into(w.udesc, wire, back, r2)
    t_u = eng.trace()
    t_traced = time.perf_counter() - t0
    eng.trace(False)
    res = {"gib_s": round(n * 1200 / float(np.median(times)) / GIB, 3), "round_trip_ok": ok,
           "samples_gib_s": [round(n * 1200 / t / GIB, 3) for t in times],
           "phases": {"traced_gib_s": round(n * 1200 / t_traced / GIB, 3),
                      "protect": [rnd(t) for t in t_p], "unprotect": [rnd(t) for t in t_u]}}
    del eng
    return res


def e2e(eng_cls, cfg, seed, dev, n, chunks=16, n_streams=4, reps=5, mode="staged"):
    """Pinned host -> H2D -> protect -> unprotect -> D2H in `chunks` slices
    (the path starts and ends in UDP socket buffers), on its own workload of
    `n` packets (the north star's 1Mi x 1200 B by default).  Verifies the
    round trip.

    mode "staged": a three-stage pipeline -- every H2D on one copy stream,
    every kernel pair on one compute stream, every D2H on a second copy
    stream, each chunk handed on by an event -- so the two PCIe directions
    and the kernels of three different chunks run at once.
    mode "per-chunk": chunk c's four steps in order on stream c % n_streams."""
    import torch
    from aioquic_amd.bench_data import make_workload

    w = make_workload(n, suite=cfg["suite"], n_keys=cfg["n_keys"], seed=seed,
                      version=cfg["version"], mixed=cfg.get("mixed"))
    eng = eng_cls(w.n_keys)
    eng.set_key_records(w.keys)

    h_in = torch.from_numpy(w.plain).pin_memory()
    h_out = torch.empty_like(h_in).pin_memory()
    d_in = torch.empty(w.plain_size, dtype=torch.uint8, device=dev)
    d_wire = torch.empty(w.wire_size, dtype=torch.uint8, device=dev)
    d_out = torch.empty(w.plain_size, dtype=torch.uint8, device=dev)
    per = n // chunks
    streams = [torch.cuda.Stream(dev) for _ in range(n_streams)]
    descs, udescs, res = [], [], []
    for c in range(chunks):
        d = w.desc[c * per : (c + 1) * per].copy()
        u = w.udesc[c * per : (c + 1) * per].copy()
        descs.append(torch.from_numpy(d.view(np.uint8)).to(dev))
        udescs.append(torch.from_numpy(u.view(np.uint8)).to(dev))
        res.append(torch.empty(per * 16, dtype=torch.uint8, device=dev))
    span = per * 1200
    stages = [torch.cuda.Stream(dev) for _ in range(3)]
    ev_in = [torch.cuda.Event() for _ in range(chunks)]
    ev_k = [torch.cuda.Event() for _ in range(chunks)]
    times = []
    for _ in range(reps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if mode == "staged":
            s_in, s_k, s_out = stages
            for c in range(chunks):
                lo, hi = c * span, (c + 1) * span
                with torch.cuda.stream(s_in):
                    d_in[lo:hi].copy_(h_in[lo:hi], non_blocking=True)
                    ev_in[c].record(s_in)
                s_k.wait_event(ev_in[c])
                eng.protect(descs[c], per, d_in, d_wire, res[c], s_k)
                eng.unprotect(udescs[c], per, d_wire, d_out, res[c], s_k)
                ev_k[c].record(s_k)
                s_out.wait_event(ev_k[c])
                with torch.cuda.stream(s_out):
                    h_out[lo:hi].copy_(d_out[lo:hi], non_blocking=True)
        else:
            for c in range(chunks):
                s = streams[c % n_streams]
                with torch.cuda.stream(s):
                    lo, hi = c * span, (c + 1) * span
                    d_in[lo:hi].copy_(h_in[lo:hi], non_blocking=True)
                    eng.protect(descs[c], per, d_in, d_wire, res[c], s)
                    eng.unprotect(udescs[c], per, d_wire, d_out, res[c], s)
                    h_out[lo:hi].copy_(d_out[lo:hi], non_blocking=True)
        torch.cuda.synchronize(dev)
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    # the PCIe legs alone, same buffers (what bounds the host-resident rate)
    leg = {}
    for name, dst, src in (("h2d", d_in, h_in), ("d2h", h_out, d_out)):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize(dev)
        leg[name] = round(reps * src.numel() / (time.perf_counter() - t0) / GIB, 3)
    # both directions at once on two streams (the duplex bound of the link)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        with torch.cuda.stream(streams[0]):
            d_in.copy_(h_in, non_blocking=True)
        with torch.cuda.stream(streams[1 % n_streams]):
            h_out.copy_(d_out, non_blocking=True)
    torch.cuda.synchronize(dev)
    leg["duplex"] = round(reps * h_in.numel() / (time.perf_counter() - t0) / GIB, 3)
    ok = bool(np.array_equal(h_out.numpy()[: per * chunks * 1200], w.plain[: per * chunks * 1200]))
    return {"gib_s": round(per * chunks * 1200 / t / GIB, 3), "packets": per * chunks,
            "round_trip_ok": ok, "chunks": chunks,
            "streams": 3 if mode == "staged" else n_streams, "mode": mode, "h2d_gib_s": leg["h2d"], "d2h_gib_s": leg["d2h"],
            "duplex_gib_s_each_way": leg["duplex"],
            "note": ("pinned H2D + protect + unprotect + D2H, "
                     + ("3-stage pipeline (H2D / kernels / D2H streams)" if mode == "staged"
                        else f"{n_streams} streams, one chunk per stream"))}


if __name__ == "__main__":
    main()
