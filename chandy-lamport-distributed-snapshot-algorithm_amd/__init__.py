"""MI355X-native batch engine for the reference's Chandy-Lamport simulator hot path.

The reference (Go package ``chandy_lamport``) simulates one run: ``ChandyLamportSim``
(sim.go) with ``AddNode/AddLink/ProcessEvent/Tick/StartSnapshot/CollectSnapshot`` and
nodes exchanging tokens and markers over FIFO channels (node.go, queue.go).  This
package runs ``n_instances`` such simulations at once on one gfx950 GPU through the C
ABI in ``include/clsnap.h`` (library ``lib/libclsnap.so``, built in-tree).  Each
instance is the reference run under its own delay stream; by default instance ``i``
uses Go's ``rand.Seed(seed_base + i)`` stream, so instance 0 with the reference seed
reproduces the reference's golden snapshots.

The Python layer is a thin mirror of the reference API (same method names and argument
meaning); there is no CPU fallback: if the library or a gfx950 GPU is missing, calls
that need them raise ``ClSnapError``.
"""
import ctypes as C
import os

import numpy as np

__all__ = ["ChandyLamportSim", "GlobalSnapshot", "MsgSnapshot", "PassTokenEvent", "SnapshotEvent",
           "ClSnapError", "lib", "go_delay_schedule", "go_int63", "go_intn", "REFERENCE_SEED",
           "INST_OK", "INST_FATAL_INSUFFICIENT_TOKENS", "INST_FATAL_UNKNOWN_DEST",
           "INST_FIFO_OVERFLOW", "INST_HANG", "INST_DELAY_EXHAUSTED", "COUNTER_NAMES",
           "SUM_NAMES", "MAX_DELAY", "E_INVALID", "E_UNKNOWN_NODE", "E_DUPLICATE_NODE", "E_PARSE",
           "E_IO", "E_DEVICE", "E_LIMIT", "E_STATE", "E_NOT_COMPLETE"]

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libclsnap.so")
if os.environ.get("CLSNAP_VARIANT"):  # diagnostic ablation builds (Makefile `variant`)
    LIB_PATH = os.path.join(HERE, "lib", f"libclsnap_{os.environ['CLSNAP_VARIANT']}.so")

REFERENCE_SEED = 8053172852482175523 + 1  # snapshot_test.go:9,20 rand.Seed(seed + 1)
MAX_DELAY = 5                              # sim.go:10

(INST_OK, INST_FATAL_INSUFFICIENT_TOKENS, INST_FATAL_UNKNOWN_DEST, INST_FIFO_OVERFLOW,
 INST_HANG, INST_DELAY_EXHAUSTED) = range(6)
COUNTER_NAMES = ("push", "peek", "pop_tok", "pop_mk", "recorded", "completed", "instances", "ticks")
SUM_NAMES = ("instances", "ok", "fatal", "other", "delivered", "snapshot_hash", "cut_residual",
             "final_residual", "completed", "in_flight")

# the C ABI's return codes (include/clsnap.h CL_E_*)
(E_INVALID, E_UNKNOWN_NODE, E_DUPLICATE_NODE, E_PARSE, E_IO, E_DEVICE, E_LIMIT, E_STATE,
 E_NOT_COMPLETE) = range(-1, -10, -1)
_ERRORS = {E_INVALID: "invalid", E_UNKNOWN_NODE: "unknown node", E_DUPLICATE_NODE: "duplicate node",
           E_PARSE: "parse", E_IO: "io", E_DEVICE: "device", E_LIMIT: "limit", E_STATE: "state",
           E_NOT_COMPLETE: "not complete"}


class ClSnapError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{_ERRORS.get(code, code)}] {msg}")
        self.code = code


_lib = None


def lib():
    """Load lib/libclsnap.so (build it with __graft_entry__.build() or `make`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ClSnapError(-6, f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(LIB_PATH)
    vp, i64, i32, cp, pp = C.c_void_p, C.c_int64, C.c_int32, C.c_char_p, C.POINTER(C.c_void_p)
    sig = {
        "cl_sim_create": [i64, pp],
        "cl_sim_destroy": [vp],
        "cl_add_node": [vp, cp, i64],
        "cl_add_link": [vp, cp, cp],
        "cl_read_topology_file": [vp, cp],
        "cl_read_topology_text": [vp, cp],
        "cl_set_device": [vp, i32],
        "cl_set_limits": [vp, i32, i64],
        "cl_set_delay_go_seeds": [vp, i64],
        "cl_set_delay_schedule": [vp, vp, i64],
        "cl_send_tokens": [vp, cp, cp, i64],
        "cl_start_snapshot": [vp, cp, vp],
        "cl_tick": [vp, i32],
        "cl_drain": [vp],
        "cl_read_events_file": [vp, cp, vp],
        "cl_read_events_text": [vp, cp, vp],
        "cl_flush": [vp],
        "cl_rerun": [vp],
        "cl_synchronize": [vp],
        "cl_last_kernel_ms": [vp, vp],
        "cl_kernel_time": [vp, vp, vp],
        "cl_replay_spill_free": [vp, vp],
        "cl_replay_mapped": [vp, vp],
        "cl_debug_poison_outputs": [vp],
        "cl_replay_split": [vp, vp, vp],
        "cl_num_nodes": [vp, vp],
        "cl_node_id": [vp, i32, vp],
        "cl_num_channels": [vp, vp],
        "cl_channel": [vp, i32, vp, vp],
        "cl_num_snapshots": [vp, vp],
        "cl_num_instances": [vp, vp],
        "cl_delay_draws_needed": [vp, vp],
        "cl_device_bytes": [vp, vp],
        "cl_get_status": [vp, vp],
        "cl_get_time": [vp, vp],
        "cl_node_tokens": [vp, i64, vp],
        "cl_snapshot_tick": [vp, i32, i64, vp],
        "cl_collect_snapshot": [vp, i32, i64, vp, vp, vp, i64],
        "cl_poll_snapshot": [vp, i32, i64, i64, vp],
        "cl_wait_snapshot": [vp, i32, i64, i64, i64, vp],
        "cl_collect_snapshot_range": [vp, i32, i64, i64, vp, vp, vp, vp, i64],
        "cl_collect_snapshot_packed": [vp, i32, i64, i64, vp, vp, vp, vp, i64, vp],
        "cl_collect_time": [vp, vp],
        "cl_get_counters": [vp, i32, vp],
        "cl_get_checksums": [vp, vp],
        "cl_go_delay_schedule": [i64, i64, i64, vp],
        "cl_go_int63": [i64, i64, vp],
        "cl_go_intn": [i64, i32, i64, vp],
        "cl_trace_enable": [vp, i64, i32, i32],
        "cl_trace_read": [vp, i64, vp, i32, vp],
        "cl_set_exec_engine": [vp, i32],
        "cl_exec_engine": [vp, vp],
        "cl_jit_stats": [vp, vp],
        "cl_lanes_compile_check": [vp, vp, vp, i64],
    }
    for name, args in sig.items():
        if os.environ.get("CLSNAP_VARIANT") and not hasattr(L, name):
            continue  # (an older diagnostic build: entry points added since are absent)
        f = getattr(L, name)
        f.restype, f.argtypes = C.c_int, args
    L.cl_status_string.restype, L.cl_status_string.argtypes = cp, [i32]
    L.cl_last_error.restype, L.cl_last_error.argtypes = cp, []
    _lib = L
    return L


# Logger record kinds (include/clsnap.h CL_LOG_*)
LOG_SENT_TOKEN, LOG_SENT_MARKER, LOG_RECV_TOKEN, LOG_RECV_MARKER, LOG_START, LOG_END = range(6)


def jit_stats():
    """Run-time kernel compilations of this process: (total ms, count)."""
    ms, n = C.c_double(), C.c_int64()
    _check(lib().cl_jit_stats(C.byref(ms), C.byref(n)))
    return ms.value, n.value


def format_log(ids, records):
    """Logger.PrettyPrint (logger.go:55-64) of (epoch, kind, node, other, data, tokens)
    records: LogEvent.String / the record String methods (logger.go:25-50,
    common.go:75-122)."""
    name = lambda r: ids[r] if r >= 0 else "?"  # noqa: E731  (no link: the dest string is not kept)
    lines, epoch = [], None
    for ep, kind, node, other, data, tokens in records:
        if ep != epoch:
            lines.append(f"Time {ep}:")
            epoch = ep
        if kind == LOG_SENT_TOKEN:
            rec, pre = f"{ids[node]} sent {data} tokens to {name(other)}", True
        elif kind == LOG_SENT_MARKER:
            rec, pre = f"{ids[node]} sent marker({data}) to {name(other)}", False
        elif kind == LOG_RECV_TOKEN:
            rec, pre = f"{ids[node]} received {data} tokens from {name(other)}", True
        elif kind == LOG_RECV_MARKER:
            rec, pre = f"{ids[node]} received marker({data}) from {name(other)}", False
        elif kind == LOG_START:
            rec, pre = f"{ids[node]} startSnapshot({data})", True
        else:
            rec, pre = f"{ids[node]} endSnapshot({data})", False
        lines.append(f"\t{ids[node]} has {tokens} token(s)\n\t{rec}" if pre else f"\t{rec}")
    return "\n".join(lines) + ("\n" if lines else "")


def _check(rc):
    if rc != 0:
        raise ClSnapError(rc, lib().cl_last_error().decode())
    return rc


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def go_delay_schedule(seed_base, n, draws):
    """uint8[n, draws]: rand.Intn(5) draws of rand.Seed(seed_base + i) (sim.go:101)."""
    out = np.empty((n, draws), dtype=np.uint8)
    _check(lib().cl_go_delay_schedule(seed_base, n, draws, _p(out)))
    return out


def go_int63(seed, n):
    out = np.empty(n, dtype=np.int64)
    _check(lib().cl_go_int63(seed, n, _p(out)))
    return out


def go_intn(seed, bound, n):
    out = np.empty(n, dtype=np.int32)
    _check(lib().cl_go_intn(seed, bound, n, _p(out)))
    return out


class PassTokenEvent:  # common.go:61-65
    def __init__(self, src, dest, tokens):
        self.src, self.dest, self.tokens = src, dest, tokens


class SnapshotEvent:  # common.go:67-70
    def __init__(self, node_id):
        self.nodeId = node_id


class MsgSnapshot:  # common.go:20-24
    __slots__ = ("src", "dest", "tokens")

    def __init__(self, src, dest, tokens):
        self.src, self.dest, self.tokens = src, dest, tokens

    def __repr__(self):
        return f"{self.src} -> {self.dest}: token({self.tokens})"

    def astuple(self):
        return (self.src, self.dest, self.tokens)


class GlobalSnapshot:  # common.go:13-17
    def __init__(self, sid, token_map, messages):
        self.id, self.tokenMap, self.messages = sid, token_map, messages


class ChandyLamportSim:
    """A batch of ``n_instances`` reference simulators (sim.go ChandyLamportSim).

    Events (``AddNode``, ``AddLink``, ``ProcessEvent``, ``Tick``, ``StartSnapshot``) are
    broadcast to every instance; results are read per instance.
    """

    def __init__(self, n_instances=1, device=0, seed_base=REFERENCE_SEED, fifo_lds_slots=None,
                 max_drain_ticks=None):
        self._L = lib()
        h = C.c_void_p()
        _check(self._L.cl_sim_create(n_instances, C.byref(h)))
        self._h = h
        self.n_instances = n_instances
        _check(self._L.cl_set_device(self._h, device))
        _check(self._L.cl_set_delay_go_seeds(self._h, seed_base))
        if fifo_lds_slots is not None or max_drain_ticks is not None:
            _check(self._L.cl_set_limits(self._h, fifo_lds_slots or 0,
                                         10000 if max_drain_ticks is None else max_drain_ticks))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.cl_sim_destroy(h)
            self._h = None

    # ---- reference API (sim.go) ---------------------------------------------
    def AddNode(self, node_id, tokens):           # sim.go:40
        _check(self._L.cl_add_node(self._h, node_id.encode(), tokens))

    def AddLink(self, src, dest):                 # sim.go:46
        _check(self._L.cl_add_link(self._h, src.encode(), dest.encode()))

    def ProcessEvent(self, event):                # sim.go:58
        if isinstance(event, PassTokenEvent):
            _check(self._L.cl_send_tokens(self._h, event.src.encode(), event.dest.encode(), event.tokens))
        elif isinstance(event, SnapshotEvent):
            self.StartSnapshot(event.nodeId)
        else:
            raise ClSnapError(-1, f"Error unknown event: {event!r}")

    def Tick(self, n=1):                          # sim.go:71
        _check(self._L.cl_tick(self._h, n))

    def StartSnapshot(self, node_id):             # sim.go:105
        sid = C.c_int32(-1)
        _check(self._L.cl_start_snapshot(self._h, node_id.encode(), C.byref(sid)))
        return sid.value

    def CollectSnapshot(self, snapshot_id, instance=0, timeout_ms=0):   # sim.go:134
        """GlobalSnapshot of one instance, messages in (dest, src, delivery) order.

        The reference blocks until the snapshot completes (sim.go:137-140): pass
        timeout_ms=-1 for that (from a collector thread while another thread drives
        the ticks), or a bound in ms; the default 0 raises ClSnapError(-9) at once if
        the snapshot has not completed."""
        if timeout_ms:
            self.wait_snapshot(snapshot_id, instance, instance + 1, timeout_ms)
        n, ch = self.num_nodes, self.num_channels
        tok = np.zeros(n, dtype=np.int64)
        off = np.zeros(ch + 1, dtype=np.int64)
        cap = 1024
        while True:
            msg = np.zeros(cap, dtype=np.int64)
            rc = self._L.cl_collect_snapshot(self._h, snapshot_id, instance, _p(tok), _p(off), _p(msg), cap)
            if rc == -7 and off[ch] > cap:
                cap = int(off[ch])
                continue
            _check(rc)
            break
        ids = self.node_ids()
        chans = self.channels()
        token_map = {ids[r]: int(tok[r]) for r in range(n)}
        order = sorted(range(ch), key=lambda c: (chans[c][1], chans[c][0]))
        msgs = [MsgSnapshot(ids[chans[c][0]], ids[chans[c][1]], int(msg[k]))
                for c in order for k in range(off[c], off[c + 1])]
        return GlobalSnapshot(snapshot_id, token_map, msgs)

    def poll_snapshot(self, snapshot_id, inst_lo=0, inst_hi=None):
        """Instances of [inst_lo, inst_hi) in which the snapshot has completed (the
        per-instance WaitGroup of sim.go:116-131); executes issued events, never ticks."""
        hi = self.n_instances if inst_hi is None else inst_hi
        v = C.c_int64(0)
        _check(self._L.cl_poll_snapshot(self._h, snapshot_id, inst_lo, hi, C.byref(v)))
        return v.value

    def wait_snapshot(self, snapshot_id, inst_lo=0, inst_hi=None, timeout_ms=-1):
        """Block until the snapshot has completed in every instance of [inst_lo,
        inst_hi); woken by the driver thread's executions.  Raises ClSnapError(-9) on
        timeout (timeout_ms >= 0)."""
        hi = self.n_instances if inst_hi is None else inst_hi
        v = C.c_int64(0)
        _check(self._L.cl_wait_snapshot(self._h, snapshot_id, inst_lo, hi, timeout_ms, C.byref(v)))
        return v.value

    def collect_snapshot_range(self, snapshot_id, inst_lo=0, inst_hi=None):
        """CollectSnapshot of many instances: (tokens[n, N] rank order, -1 where not
        complete; complete[n]; offsets[n * C + 1]; messages) -- one CSR over
        (instance, channel) with channels in (src rank, dest rank) order."""
        hi = self.n_instances if inst_hi is None else inst_hi
        k, n, ch = hi - inst_lo, self.num_nodes, self.num_channels
        tok = np.zeros((k, n), dtype=np.int64)
        done = np.zeros(k, dtype=np.int32)
        off = np.zeros(k * ch + 1, dtype=np.int64)
        cap = max(1024, 4 * k)
        while True:
            msg = np.zeros(cap, dtype=np.int64)
            rc = self._L.cl_collect_snapshot_range(self._h, snapshot_id, inst_lo, hi, _p(tok), _p(done), _p(off),
                                                   _p(msg), cap)
            if rc == -7 and off[-1] > cap:
                cap = int(off[-1])
                continue
            _check(rc)
            return tok, done.astype(bool), off, msg[:off[-1]]

    def collect_snapshot_packed(self, snapshot_id, inst_lo=0, inst_hi=None, out=None):
        """CollectSnapshot of many instances packed on the GPU (cl_collect_snapshot_packed):
        (tokens int32[n, N], complete bool[n], offsets int64[n * C + 1], messages int32).
        `out` = (tokens, complete, offsets, messages) arrays to fill (reused across calls; the
        message array is grown when too small: the returned messages are a view of the array
        actually filled, so pass that base array back in `out` to reuse it)."""
        hi = self.n_instances if inst_hi is None else inst_hi
        k, n, ch = hi - inst_lo, self.num_nodes, self.num_channels
        if out is None:
            out = (np.zeros((k, n), dtype=np.int32), np.zeros(k, dtype=np.int32),
                   np.zeros(k * ch + 1, dtype=np.int64), np.zeros(max(1024, 4 * k), dtype=np.int32))
        tok, done, off, msg = out
        # the C side writes k * N tokens, k flags, k * C + 1 offsets: a buffer sized for another
        # range would be overrun
        for name, a, shape, dt in (("tokens", tok, (k, n), np.int32), ("complete", done, (k,), np.int32),
                                   ("offsets", off, (k * ch + 1,), np.int64)):
            if not isinstance(a, np.ndarray) or a.shape != shape or a.dtype != dt or not a.flags.c_contiguous:
                raise ValueError(f"collect_snapshot_packed: out {name} must be a C-contiguous {np.dtype(dt)} array "
                                 f"of shape {shape}")
        if not isinstance(msg, np.ndarray) or msg.dtype != np.int32 or msg.ndim != 1 or not msg.flags.c_contiguous:
            raise ValueError("collect_snapshot_packed: out messages must be a C-contiguous 1-d int32 array")
        m = C.c_int64(0)
        rc = self._L.cl_collect_snapshot_packed(self._h, snapshot_id, inst_lo, hi, _p(tok), _p(done), _p(off),
                                                _p(msg), msg.size, C.byref(m))
        if rc == -7 and m.value > msg.size:
            msg = np.zeros(m.value, dtype=np.int32)
            rc = self._L.cl_collect_snapshot_packed(self._h, snapshot_id, inst_lo, hi, _p(tok), _p(done), _p(off),
                                                    _p(msg), msg.size, C.byref(m))
        _check(rc)
        return tok, done.astype(bool), off, msg[:m.value]

    def collect_time(self):
        """Device ms of the latest packed collect's kernels."""
        ms = C.c_double(0)
        _check(self._L.cl_collect_time(self._h, C.byref(ms)))
        return ms.value

    # ---- drivers (test_common.go) -------------------------------------------
    def read_topology_file(self, path):           # test_common.go:29
        _check(self._L.cl_read_topology_file(self._h, path.encode()))

    def read_topology_text(self, text):
        _check(self._L.cl_read_topology_text(self._h, text.encode()))

    def read_events_file(self, path):             # test_common.go:79 (incl. drain)
        n = C.c_int32(0)
        _check(self._L.cl_read_events_file(self._h, path.encode(), C.byref(n)))
        return n.value

    def read_events_text(self, text):
        n = C.c_int32(0)
        _check(self._L.cl_read_events_text(self._h, text.encode(), C.byref(n)))
        return n.value

    def drain(self):                               # test_common.go:123-137
        _check(self._L.cl_drain(self._h))

    # ---- engine control -----------------------------------------------------
    def set_delay_schedule(self, delays):
        d = np.ascontiguousarray(delays, dtype=np.uint8)
        if d.ndim != 2 or d.shape[0] != self.n_instances:
            raise ClSnapError(-1, "schedule must be uint8[n_instances, draws]")
        _check(self._L.cl_set_delay_schedule(self._h, _p(d), d.shape[1]))

    def set_delay_go_seeds(self, seed_base):
        _check(self._L.cl_set_delay_go_seeds(self._h, seed_base))

    def set_limits(self, fifo_lds_slots=0, max_drain_ticks=10000):
        _check(self._L.cl_set_limits(self._h, fifo_lds_slots, max_drain_ticks))

    def flush(self):
        _check(self._L.cl_flush(self._h))

    def rerun(self):
        _check(self._L.cl_rerun(self._h))

    def synchronize(self):
        _check(self._L.cl_synchronize(self._h))

    def poison_outputs(self):
        """Overwrite every result plane with 0xA5 bytes (cl_debug_poison_outputs): results
        read after the next rerun() can only come from that launch."""
        _check(self._L.cl_debug_poison_outputs(self._h))

    def last_kernel_ms(self):
        ms = C.c_double(0)
        _check(self._L.cl_last_kernel_ms(self._h, C.byref(ms)))
        return ms.value

    def replay_split(self):
        """(instances that spilled in the probe run, -1 before it; first slot of the
        spill-capable part of split replays, 0 = no split) -- cl_replay_split."""
        a, b = C.c_int64(0), C.c_int64(0)
        _check(self._L.cl_replay_split(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def spill_free_replays(self):
        """True when the next rerun() runs wholly on the spill-free kernel (cl_replay_spill_free)."""
        v = C.c_int32(0)
        _check(self._L.cl_replay_spill_free(self._h, C.byref(v)))
        return bool(v.value)

    def mapped_replays(self):
        """True when the next rerun() launches through the length-ordered slot map."""
        v = C.c_int32(0)
        _check(self._L.cl_replay_mapped(self._h, C.byref(v)))
        return bool(v.value)

    # exec kernel choice (include/clsnap.h CL_ENGINE_*): results are identical on either kernel
    ENGINE_AUTO, ENGINE_NODES, ENGINE_LANES = 0, 1, 2

    def set_exec_engine(self, engine):
        _check(self._L.cl_set_exec_engine(self._h, int(engine)))

    def exec_engine(self):
        """The exec kernel the most recent launch used (ENGINE_NODES / ENGINE_LANES; 0 before any)."""
        return self._i32(self._L.cl_exec_engine)

    def lanes_compile_check(self):
        """Compile the instance-per-lane kernels for this topology without a device:
        (compile ms, compiler log); raises ClSnapError when they do not fit or fail to compile."""
        ms = C.c_double()
        buf = C.create_string_buffer(16384)
        _check(self._L.cl_lanes_compile_check(self._h, C.byref(ms), buf, len(buf)))
        return ms.value, buf.value.decode(errors="replace")

    def kernel_time(self):
        """(total exec-kernel ms, launches) since the previous call (HIP events)."""
        ms, n = C.c_double(0), C.c_int64(0)
        _check(self._L.cl_kernel_time(self._h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    # ---- queries ------------------------------------------------------------
    def _i32(self, fn, *args):
        v = C.c_int32(0)
        _check(fn(self._h, *args, C.byref(v)))
        return v.value

    def _i64(self, fn):
        v = C.c_int64(0)
        _check(fn(self._h, C.byref(v)))
        return v.value

    @property
    def num_nodes(self):
        return self._i32(self._L.cl_num_nodes)

    @property
    def num_channels(self):
        return self._i32(self._L.cl_num_channels)

    @property
    def num_snapshots(self):
        return self._i32(self._L.cl_num_snapshots)

    @property
    def draws_needed(self):
        return self._i64(self._L.cl_delay_draws_needed)

    @property
    def device_bytes(self):
        return self._i64(self._L.cl_device_bytes)

    def node_ids(self):
        out = []
        for r in range(self.num_nodes):
            s = C.c_char_p()
            _check(self._L.cl_node_id(self._h, r, C.byref(s)))
            out.append(s.value.decode())
        return out

    def channels(self):
        out = []
        for c in range(self.num_channels):
            a, b = C.c_int32(), C.c_int32()
            _check(self._L.cl_channel(self._h, c, C.byref(a), C.byref(b)))
            out.append((a.value, b.value))
        return out

    def status(self):
        out = np.zeros(self.n_instances, dtype=np.int32)
        _check(self._L.cl_get_status(self._h, _p(out)))
        return out

    def time(self):
        out = np.zeros(self.n_instances, dtype=np.int32)
        _check(self._L.cl_get_time(self._h, _p(out)))
        return out

    def node_tokens(self, instance=0):
        out = np.zeros(self.num_nodes, dtype=np.int64)
        _check(self._L.cl_node_tokens(self._h, instance, _p(out)))
        return dict(zip(self.node_ids(), out.tolist()))

    def snapshot_tick(self, snapshot_id, instance=0):
        return self._i32(self._L.cl_snapshot_tick, snapshot_id, instance)

    def counters(self, only_ok=False):
        out = np.zeros(len(COUNTER_NAMES), dtype=np.int64)
        _check(self._L.cl_get_counters(self._h, 1 if only_ok else 0, _p(out)))
        return dict(zip(COUNTER_NAMES, out.tolist()))

    def checksums(self):
        out = np.zeros(len(SUM_NAMES), dtype=np.int64)
        _check(self._L.cl_get_checksums(self._h, _p(out)))
        return out

    # ---- device event trace: the reference's debug Logger (logger.go:12-76) ------
    def trace_enable(self, instance_lo=0, n_instances=1, capacity=4096):
        """Record the Logger of instances [instance_lo, instance_lo + n_instances); the
        next flush replays the event program with the trace build of the kernel."""
        _check(self._L.cl_trace_enable(self._h, instance_lo, n_instances, capacity))

    def trace(self, instance=0):
        """LogEvents of one traced instance in Logger order: (epoch, kind, node rank,
        other rank | -1, data, nodeTokens); kinds LOG_* (include/clsnap.h CL_LOG_*)."""
        n = C.c_int32(0)
        _check(self._L.cl_trace_read(self._h, instance, None, 0, C.byref(n)))
        out = np.zeros((max(n.value, 1), 6), dtype=np.int32)
        _check(self._L.cl_trace_read(self._h, instance, _p(out), n.value, C.byref(n)))
        return [tuple(int(x) for x in r) for r in out[:n.value]]

    def pretty_print(self, instance=0):
        """Logger.PrettyPrint (logger.go:55-64) of a traced instance, as text."""
        return format_log(self.node_ids(), self.trace(instance))

    @staticmethod
    def status_string(code):
        return lib().cl_status_string(code).decode()
