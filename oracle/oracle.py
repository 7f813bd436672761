"""ctypes binding of the CPU oracle (oracle/cl_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- never by the product package.  See cl_oracle.c's header for the
reference map (file:line) and the parity pin (21 golden snapshots + Go RNG KATs).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

OK, FATAL_INSUFFICIENT_TOKENS, FATAL_UNKNOWN_DEST, HANG, DELAY_EXHAUSTED = 0, 1, 2, 4, 5
COUNTER_NAMES = ("push", "peek", "pop_tok", "pop_mk", "recorded", "draws", "completed")
REFERENCE_SEED = 8053172852482175523 + 1  # snapshot_test.go:9,20
MAX_DRAIN_TICKS = 1_000_000

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, i64, i32, cp = C.c_void_p, C.c_int64, C.c_int32, C.c_char_p
        sig = {
            "orc_new": (vp, []),
            "orc_free": (None, [vp]),
            "orc_seed_go": (None, [vp, i64]),
            "orc_use_schedule": (None, [vp, vp, i64]),
            "orc_status": (C.c_int, [vp]),
            "orc_time": (i64, [vp]),
            "orc_num_nodes": (C.c_int, [vp]),
            "orc_num_snapshots": (C.c_int, [vp]),
            "orc_counters_get": (None, [vp, vp]),
            "orc_add_node": (C.c_int, [vp, cp, i64]),
            "orc_add_link": (C.c_int, [vp, cp, cp]),
            "orc_tick": (C.c_int, [vp]),
            "orc_send_tokens": (C.c_int, [vp, cp, cp, i64]),
            "orc_start_snapshot": (C.c_int, [vp, cp, vp]),
            "orc_snapshot_complete": (C.c_int, [vp, C.c_int]),
            "orc_completion_tick": (i64, [vp, C.c_int]),
            "orc_node_tokens": (None, [vp, vp]),
            "orc_node_id": (cp, [vp, C.c_int]),
            "orc_collect": (i64, [vp, C.c_int, vp, vp, vp, vp, i64]),
            "orc_snapshot_hash": (C.c_uint64, [vp, C.c_int]),
            "orc_read_topology": (C.c_int, [vp, cp]),
            "orc_read_events": (C.c_int, [vp, cp, i64]),
            "orc_read_topology_text": (C.c_int, [vp, vp]),
            "orc_read_events_text": (C.c_int, [vp, vp, i64]),
            "orc_go_int63_seq": (None, [i64, i64, vp]),
            "orc_go_intn_seq": (None, [i64, i32, i64, vp]),
            "orc_run_batch": (C.c_double, [cp, cp, i64, vp, i64, i64, i64, C.c_int,
                                           vp, vp, vp, vp]),
            "orc_run_batch_prepared": (C.c_double, [cp, cp, i64, i64, i64, C.c_int, vp, vp, vp, vp]),
            "orc_counter_hash": (C.c_uint64, [C.c_uint64, C.c_uint64, C.c_uint64]),
            "orc_counter_delay": (C.c_int, [C.c_uint64, C.c_uint64]),
            "orc_use_counter_hash": (None, [vp, C.c_uint64]),
            "orc_build_graph": (C.c_int, [vp, C.c_int, vp, i64, vp, vp, C.c_int]),
            "orc_traffic_sends": (C.c_int, [vp, C.c_uint64, C.c_uint32, i64]),
            "orc_run_program": (C.c_int, [vp, i64, C.c_uint64, C.c_uint32, i64, C.c_int, vp, vp]),
            "orc_collect_channels": (i64, [vp, C.c_int, vp, vp, vp, i64]),
            "orc_drain": (C.c_int, [vp, i64]),
            "orc_num_links": (C.c_int, [vp]),
            "orc_queue_depths": (None, [vp, vp]),
            "orc_log_enable": (None, [vp, C.c_int]),
            "orc_log_count": (i64, [vp]),
            "orc_log_get": (None, [vp, vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def go_int63(seed, n):
    out = np.zeros(n, dtype=np.int64)
    lib().orc_go_int63_seq(seed, n, _ptr(out))
    return out


def go_intn(seed, bound, n):
    out = np.zeros(n, dtype=np.int32)
    lib().orc_go_intn_seq(seed, bound, n, _ptr(out))
    return out


class Snapshot:
    """GlobalSnapshot (common.go:13-17): id, tokenMap, messages [(src, dest, amount)]."""

    def __init__(self, sid, tokens, messages):
        self.id, self.tokens, self.messages = sid, tokens, messages

    def per_channel(self):
        out = {}
        for s, d, a in self.messages:
            out.setdefault((s, d), []).append(a)
        return out


class OracleSim:
    """One reference simulator (sim.go ChandyLamportSim), restated on the CPU."""

    def __init__(self):
        self._L = lib()
        self._h = self._L.orc_new()
        self._sched = None

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.orc_free(self._h)
            self._h = None

    def seed_go(self, seed):
        self._L.orc_seed_go(self._h, seed)

    def use_schedule(self, delays):
        self._sched = np.ascontiguousarray(delays, dtype=np.uint8)
        self._L.orc_use_schedule(self._h, _ptr(self._sched), self._sched.size)

    def add_node(self, nid, tokens):
        return self._L.orc_add_node(self._h, nid.encode(), tokens)

    def add_link(self, src, dest):
        return self._L.orc_add_link(self._h, src.encode(), dest.encode())

    def send_tokens(self, src, dest, n):
        return self._L.orc_send_tokens(self._h, src.encode(), dest.encode(), n)

    def start_snapshot(self, node):
        sid = C.c_int(-1)
        rc = self._L.orc_start_snapshot(self._h, node.encode(), C.byref(sid))
        return rc, sid.value

    def tick(self):
        return self._L.orc_tick(self._h)

    def read_topology(self, path):
        return self._L.orc_read_topology(self._h, path.encode())

    def read_events(self, path, max_drain=MAX_DRAIN_TICKS):
        return self._L.orc_read_events(self._h, path.encode(), max_drain)

    def read_topology_text(self, text):
        buf = C.create_string_buffer(text.encode())   # the C parser tokenizes in place
        return self._L.orc_read_topology_text(self._h, buf)

    def read_events_text(self, text, max_drain=MAX_DRAIN_TICKS):
        buf = C.create_string_buffer(text.encode())
        return self._L.orc_read_events_text(self._h, buf, max_drain)

    @property
    def status(self):
        return self._L.orc_status(self._h)

    @property
    def time(self):
        return self._L.orc_time(self._h)

    @property
    def num_snapshots(self):
        return self._L.orc_num_snapshots(self._h)

    def node_ids(self):
        return [self._L.orc_node_id(self._h, i).decode() for i in range(self._L.orc_num_nodes(self._h))]

    def node_tokens(self):
        n = self._L.orc_num_nodes(self._h)
        out = np.zeros(n, dtype=np.int64)
        self._L.orc_node_tokens(self._h, _ptr(out))
        return dict(zip(self.node_ids(), out.tolist()))

    def counters(self):
        out = np.zeros(7, dtype=np.int64)
        self._L.orc_counters_get(self._h, _ptr(out))
        return dict(zip(COUNTER_NAMES, out.tolist()))

    def complete(self, sid):
        return bool(self._L.orc_snapshot_complete(self._h, sid))

    def completion_tick(self, sid):
        return self._L.orc_completion_tick(self._h, sid)

    def snapshot_hash(self, sid):
        return self._L.orc_snapshot_hash(self._h, sid)

    # ---- Logger (logger.go:12-76) ----------------------------------------------
    def log_enable(self, on=True):
        self._L.orc_log_enable(self._h, 1 if on else 0)

    def log(self):
        """LogEvents in Logger order: (epoch, kind, node rank, other rank | -1, data,
        nodeTokens), kinds as CL_LOG_* (include/clsnap.h)."""
        n = self._L.orc_log_count(self._h)
        out = np.zeros((max(n, 1), 6), dtype=np.int64)
        if n:
            self._L.orc_log_get(self._h, _ptr(out))
        return [tuple(int(x) for x in r) for r in out[:n]]

    # ---- synthetic large-graph workloads ----------------------
    def use_counter_hash(self, seed):
        self._L.orc_use_counter_hash(self._h, seed)

    def build_graph(self, tokens, src, dst, width):
        """Nodes "N%0{width}d" % r with tokens[r]; AddLink(src[i], dst[i]) (ranks)."""
        tok = np.ascontiguousarray(tokens, dtype=np.int64)
        s = np.ascontiguousarray(src, dtype=np.int32)
        d = np.ascontiguousarray(dst, dtype=np.int32)
        return self._L.orc_build_graph(self._h, tok.size, _ptr(tok), s.size, _ptr(s), _ptr(d), width)

    def run_program(self, steps, traffic_seed, thresh, traffic_steps, snap_step=(), snap_rank=()):
        ss = np.ascontiguousarray(snap_step, dtype=np.int32)
        sr = np.ascontiguousarray(snap_rank, dtype=np.int32)
        return self._L.orc_run_program(self._h, steps, traffic_seed, thresh, traffic_steps, ss.size,
                                       _ptr(ss), _ptr(sr))

    def drain(self, max_drain=MAX_DRAIN_TICKS):
        """readEventsFile's drain (test_common.go:123-137) after a program run."""
        return self._L.orc_drain(self._h, max_drain)

    @property
    def num_links(self):
        return self._L.orc_num_links(self._h)

    def queue_depths(self):
        out = np.zeros(self.num_links, dtype=np.int64)
        self._L.orc_queue_depths(self._h, _ptr(out))
        return out

    def collect_channels(self, sid):
        """(tokens[N] rank order (-1: no local snapshot), offsets[E+1], values) with
        channels in (src rank, dest rank) order."""
        n, e = self._L.orc_num_nodes(self._h), self.num_links
        tok = np.zeros(n, dtype=np.int64)
        off = np.zeros(e + 1, dtype=np.int64)
        m = self._L.orc_collect_channels(self._h, sid, _ptr(tok), _ptr(off), None, 0)
        vals = np.zeros(max(m, 1), dtype=np.int64)
        self._L.orc_collect_channels(self._h, sid, _ptr(tok), _ptr(off), _ptr(vals), m)
        return tok, off, vals[:m]

    def collect(self, sid):
        n = self._L.orc_num_nodes(self._h)
        tok = np.zeros(n, dtype=np.int64)
        m = self._L.orc_collect(self._h, sid, _ptr(tok), None, None, None, 0)
        if m < 0:
            return None
        src = np.zeros(max(m, 1), dtype=np.int32)
        dst = np.zeros(max(m, 1), dtype=np.int32)
        amt = np.zeros(max(m, 1), dtype=np.int64)
        self._L.orc_collect(self._h, sid, _ptr(tok), _ptr(src), _ptr(dst), _ptr(amt), m)
        ids = self.node_ids()
        msgs = [(ids[src[i]], ids[dst[i]], int(amt[i])) for i in range(m)]
        return Snapshot(sid, dict(zip(ids, tok.tolist())), msgs)


def counter_hash(seed, a, b):
    return lib().orc_counter_hash(seed, a, b)


def counter_delay(seed, k):
    return lib().orc_counter_delay(seed, k)


def run_batch(top_text, events_text, n, sched=None, draws=0, seed_base=REFERENCE_SEED,
              threads=1, max_drain=MAX_DRAIN_TICKS):
    """Independent simulations of one scenario (cpu_baseline / parity sampling).

    Returns (seconds, status[n], ticks[n], counters[n,7], hash[n])."""
    status = np.zeros(n, dtype=np.int32)
    ticks = np.zeros(n, dtype=np.int64)
    counters = np.zeros((n, 7), dtype=np.int64)
    hashes = np.zeros(n, dtype=np.uint64)
    sp = None
    if sched is not None:
        sched = np.ascontiguousarray(sched, dtype=np.uint8)
        sp = _ptr(sched)
    secs = lib().orc_run_batch(top_text.encode(), events_text.encode(), n, sp, draws, seed_base,
                               max_drain, threads, _ptr(status), _ptr(ticks), _ptr(counters),
                               _ptr(hashes))
    if secs < 0:
        raise RuntimeError("oracle batch failed (parse/API error)")
    return secs, status, ticks, counters, hashes


def run_batch_prepared(top_text, events_text, n, seed_base=REFERENCE_SEED, threads=1,
                       max_drain=MAX_DRAIN_TICKS, want_hash=True):
    """Like run_batch with Go seeds, but the topology and events are parsed once and
    each thread resets one simulator per instance; the returned seconds cover the
    simulations only (bench.py cpu_baseline).  hash is None unless want_hash."""
    status = np.zeros(n, dtype=np.int32)
    ticks = np.zeros(n, dtype=np.int64)
    counters = np.zeros((n, 7), dtype=np.int64)
    hashes = np.zeros(n, dtype=np.uint64) if want_hash else None
    secs = lib().orc_run_batch_prepared(top_text.encode(), events_text.encode(), n, seed_base, max_drain,
                                        threads, _ptr(status), _ptr(ticks), _ptr(counters),
                                        _ptr(hashes) if want_hash else None)
    if secs < 0:
        raise RuntimeError("oracle batch failed (parse/API error)")
    return secs, status, ticks, counters, hashes
