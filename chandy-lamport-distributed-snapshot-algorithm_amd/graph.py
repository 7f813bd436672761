"""Graph engine: ONE reference simulation over a large topology (include/clgraph.h).

``GraphSim`` mirrors the reference simulator API (sim.go ``ChandyLamportSim``:
``AddNode``, ``AddLink``, ``ProcessEvent``, ``Tick``, ``StartSnapshot``,
``CollectSnapshot``) for a single run whose nodes and channels span the whole GPU --
BASELINE configs 4 (2^20-node random regular digraph under continuous token traffic)
and 5 (100k-node power-law graph with 4,096 overlapping snapshots) -- and runs the
reference's own test_data scenarios as well.  There is no CPU fallback: without the
HIP library or a gfx950 GPU, calls that need them raise ``ClSnapError``.
"""
import ctypes as C

import numpy as np

from . import (ClSnapError, GlobalSnapshot, MsgSnapshot, PassTokenEvent, SnapshotEvent, _check, _p, format_log,
               COUNTER_NAMES, lib)

GSUM_NAMES = ("ok", "delivered", "completed", "cut_residual", "final_residual", "digest", "in_flight")

_SIGS = None


def glib():
    """The engine library with the cl_graph_* signatures bound."""
    global _SIGS
    L = lib()
    if _SIGS is None:
        vp, i64, i32, u64, u32, cp = C.c_void_p, C.c_int64, C.c_int32, C.c_uint64, C.c_uint32, C.c_char_p
        sig = {
            "cl_graph_create": [C.POINTER(C.c_void_p)],
            "cl_graph_destroy": [vp],
            "cl_graph_set_device": [vp, i32],
            "cl_graph_add_node": [vp, cp, i64],
            "cl_graph_add_link": [vp, cp, cp],
            "cl_graph_read_topology_text": [vp, cp],
            "cl_graph_read_topology_file": [vp, cp],
            "cl_graph_set_topology": [vp, i32, i32, vp, i64, vp, vp],
            "cl_graph_generate_regular": [vp, i32, i32, i64, u64],
            "cl_graph_generate_powerlaw": [vp, i32, i32, C.c_double, i32, i64, u64],
            "cl_graph_num_nodes": [vp, vp],
            "cl_graph_num_channels": [vp, vp],
            "cl_graph_channels": [vp, vp, vp],
            "cl_graph_node_id": [vp, i32, vp, i32],
            "cl_graph_node_id_length": [vp, i32, vp],
            "cl_graph_set_push_lanes": [vp, i32],
            "cl_graph_trace_enable": [vp, i32],
            "cl_graph_trace_read": [vp, vp, i32, vp],
            "cl_graph_set_limits": [vp, i32, i32, i64],
            "cl_graph_set_delay_hash": [vp, u64],
            "cl_graph_set_delay_go_seed": [vp, i64],
            "cl_graph_set_delay_schedule": [vp, vp, i64],
            "cl_graph_set_traffic": [vp, u64, u32, i64],
            "cl_graph_send_tokens": [vp, cp, cp, i64],
            "cl_graph_send_tokens_rank": [vp, i32, i32, i64],
            "cl_graph_start_snapshot": [vp, cp, vp],
            "cl_graph_start_snapshot_rank": [vp, i32, vp],
            "cl_graph_tick": [vp, i32],
            "cl_graph_drain": [vp],
            "cl_graph_read_events_text": [vp, cp, vp],
            "cl_graph_read_events_file": [vp, cp, vp],
            "cl_graph_flush": [vp],
            "cl_graph_rerun": [vp],
            "cl_graph_synchronize": [vp],
            "cl_graph_run_time": [vp, vp, vp, vp],
            "cl_graph_phase_time": [vp, vp, vp],
            "cl_graph_debug_poison_outputs": [vp],
            "cl_graph_device_bytes": [vp, vp],
            "cl_graph_get_status": [vp, vp],
            "cl_graph_get_time": [vp, vp],
            "cl_graph_num_snapshots": [vp, vp],
            "cl_graph_node_tokens": [vp, vp],
            "cl_graph_snapshot_tick": [vp, i32, vp],
            "cl_graph_collect_snapshot": [vp, i32, vp, vp, vp, i64],
            "cl_graph_get_counters": [vp, vp],
            "cl_graph_get_checksums": [vp, vp],
            "cl_graph_part_begin": [vp, i32, i32],
            "cl_graph_part_snapshot": [vp, i32, vp],
            "cl_graph_part_pick": [vp, vp, i64, vp],
            "cl_graph_part_receive": [vp, vp, i64, vp, i64, vp],
            "cl_graph_part_tally": [vp, i32, vp, i64, vp],
            "cl_graph_part_bases": [vp, vp, vp, i64, vp],
            "cl_graph_part_push": [vp, i32, vp, i64],
            "cl_graph_part_freeze": [vp, i32],
            "cl_graph_part_dev_bind": [vp, i32, i32, i32, i64, vp, vp, vp, vp],
            "cl_graph_part_dev_seal": [vp],
            "cl_graph_part_dev_pick": [vp],
            "cl_graph_part_dev_receive": [vp],
            "cl_graph_part_dev_tally": [vp, i32],
            "cl_graph_part_dev_bases": [vp],
            "cl_graph_part_dev_push": [vp, i32],
            "cl_graph_set_stream": [vp, vp],
        }
        for name, args in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = C.c_int, args
        L.cl_counter_hash.restype, L.cl_counter_hash.argtypes = u64, [u64, u64, u64]
        _SIGS = sig
    return L


def counter_hash(seed, a, b):
    """The synthetic workloads' counter hash (cg_hash, cg_engine.h)."""
    return glib().cl_counter_hash(seed, a, b)


class GraphSim:
    """One reference simulator (sim.go ChandyLamportSim) on the GPU, state in HBM."""

    def __init__(self, device=0, fifo_slots=16, max_snapshots=0, max_drain_ticks=10000):
        self._L = glib()
        h = C.c_void_p()
        _check(self._L.cl_graph_create(C.byref(h)))
        self._h = h
        self.device = device
        _check(self._L.cl_graph_set_device(self._h, device))
        _check(self._L.cl_graph_set_limits(self._h, fifo_slots, max_snapshots, max_drain_ticks))
        self._ids = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.cl_graph_destroy(h)
            self._h = None

    # ---- topology -----------------------------------------------------------------
    def AddNode(self, node_id, tokens):             # sim.go:40
        _check(self._L.cl_graph_add_node(self._h, node_id.encode(), tokens))

    def AddLink(self, src, dest):                   # sim.go:46
        _check(self._L.cl_graph_add_link(self._h, src.encode(), dest.encode()))

    def read_topology_file(self, path):             # test_common.go:29
        _check(self._L.cl_graph_read_topology_file(self._h, path.encode()))

    def read_topology_text(self, text):
        _check(self._L.cl_graph_read_topology_text(self._h, text.encode()))

    def set_topology(self, tokens, src, dst, id_width=0):
        tok = np.ascontiguousarray(tokens, dtype=np.int64)
        s = np.ascontiguousarray(src, dtype=np.int32)
        d = np.ascontiguousarray(dst, dtype=np.int32)
        _check(self._L.cl_graph_set_topology(self._h, tok.size, id_width, _p(tok), s.size, _p(s), _p(d)))

    def generate_regular(self, n_nodes, degree=8, tokens=100, seed=0):
        _check(self._L.cl_graph_generate_regular(self._h, n_nodes, degree, tokens, seed))

    def generate_powerlaw(self, n_nodes, targets=8, exponent=0.9, ring=True, tokens=100, seed=0):
        _check(self._L.cl_graph_generate_powerlaw(self._h, n_nodes, targets, exponent, 1 if ring else 0,
                                                  tokens, seed))

    # ---- configuration --------------------------------------------------------------
    def set_limits(self, fifo_slots=16, max_snapshots=0, max_drain_ticks=10000):
        _check(self._L.cl_graph_set_limits(self._h, fifo_slots, max_snapshots, max_drain_ticks))

    def set_delay_hash(self, seed):
        _check(self._L.cl_graph_set_delay_hash(self._h, seed))

    def set_delay_go_seed(self, seed):
        _check(self._L.cl_graph_set_delay_go_seed(self._h, seed))

    def set_delay_schedule(self, delays):
        d = np.ascontiguousarray(delays, dtype=np.uint8).ravel()
        _check(self._L.cl_graph_set_delay_schedule(self._h, _p(d), d.size))

    def set_traffic(self, seed, threshold, steps):
        _check(self._L.cl_graph_set_traffic(self._h, seed, threshold, steps))

    def set_push_lanes(self, lanes):
        """Force the push kernel's lanes per node (0 automatic, 1 or 4): diagnostics and
        tests -- results are identical on either path."""
        _check(self._L.cl_graph_set_push_lanes(self._h, lanes))

    # ---- events -------------------------------------------------------------------------
    def ProcessEvent(self, event):                  # sim.go:58
        if isinstance(event, PassTokenEvent):
            _check(self._L.cl_graph_send_tokens(self._h, event.src.encode(), event.dest.encode(), event.tokens))
        elif isinstance(event, SnapshotEvent):
            self.StartSnapshot(event.nodeId)
        else:
            raise ClSnapError(-1, f"Error unknown event: {event!r}")

    def send_tokens_rank(self, src, dest, n):
        _check(self._L.cl_graph_send_tokens_rank(self._h, src, dest, n))

    def Tick(self, n=1):                            # sim.go:71
        _check(self._L.cl_graph_tick(self._h, n))

    def StartSnapshot(self, node_id):               # sim.go:105
        sid = C.c_int32(-1)
        _check(self._L.cl_graph_start_snapshot(self._h, node_id.encode(), C.byref(sid)))
        return sid.value

    def start_snapshot_rank(self, rank):
        sid = C.c_int32(-1)
        _check(self._L.cl_graph_start_snapshot_rank(self._h, rank, C.byref(sid)))
        return sid.value

    def drain(self):                                # test_common.go:123-137
        _check(self._L.cl_graph_drain(self._h))

    def read_events_file(self, path):               # test_common.go:79 (incl. drain)
        n = C.c_int32(0)
        _check(self._L.cl_graph_read_events_file(self._h, path.encode(), C.byref(n)))
        return n.value

    def read_events_text(self, text):
        n = C.c_int32(0)
        _check(self._L.cl_graph_read_events_text(self._h, text.encode(), C.byref(n)))
        return n.value

    # ---- execution ----------------------------------------------------------------------
    def flush(self):
        _check(self._L.cl_graph_flush(self._h))

    def rerun(self):
        _check(self._L.cl_graph_rerun(self._h))

    def synchronize(self):
        _check(self._L.cl_graph_synchronize(self._h))

    def run_time(self):
        """(device ms of the runs since the previous call, runs, ticks) -- HIP events."""
        ms, r, t = C.c_double(0), C.c_int64(0), C.c_int64(0)
        _check(self._L.cl_graph_run_time(self._h, C.byref(ms), C.byref(r), C.byref(t)))
        return ms.value, r.value, t.value

    def poison_outputs(self):
        """Overwrite the result planes with 0xA5 bytes (cl_graph_debug_poison_outputs)."""
        _check(self._L.cl_graph_debug_poison_outputs(self._h))

    def phase_time(self):
        """Latest run: ((ms, ticks) before the first drain, (ms, ticks) of the drains)."""
        ms = np.zeros(2, dtype=np.float64)
        t = np.zeros(2, dtype=np.int64)
        _check(self._L.cl_graph_phase_time(self._h, _p(ms), _p(t)))
        return (float(ms[0]), int(t[0])), (float(ms[1]), int(t[1]))

    # ---- queries ------------------------------------------------------------------------
    def _get(self, fn, ctype, *args):
        v = ctype(0)
        _check(fn(self._h, *args, C.byref(v)))
        return v.value

    @property
    def num_nodes(self):
        return self._get(self._L.cl_graph_num_nodes, C.c_int32)

    @property
    def num_channels(self):
        return self._get(self._L.cl_graph_num_channels, C.c_int64)

    @property
    def num_snapshots(self):
        return self._get(self._L.cl_graph_num_snapshots, C.c_int32)

    @property
    def device_bytes(self):
        return self._get(self._L.cl_graph_device_bytes, C.c_int64)

    def channels(self):
        e = self.num_channels
        s = np.zeros(e, dtype=np.int32)
        d = np.zeros(e, dtype=np.int32)
        _check(self._L.cl_graph_channels(self._h, _p(s), _p(d)))
        return s, d

    def node_ids(self):
        if self._ids is None:
            cap = 64
            buf = C.create_string_buffer(cap)
            out = []
            for r in range(self.num_nodes):
                rc = self._L.cl_graph_node_id(self._h, r, buf, cap)
                if rc == -7:                             # longer id: size the buffer to it
                    cap = self._get(self._L.cl_graph_node_id_length, C.c_int32, r) + 1
                    buf = C.create_string_buffer(cap)
                    rc = self._L.cl_graph_node_id(self._h, r, buf, cap)
                _check(rc)
                out.append(buf.value.decode())
            self._ids = out
        return self._ids

    def status(self):
        return self._get(self._L.cl_graph_get_status, C.c_int32)

    def time(self):
        return self._get(self._L.cl_graph_get_time, C.c_int64)

    def node_tokens_array(self):
        out = np.zeros(self.num_nodes, dtype=np.int64)
        _check(self._L.cl_graph_node_tokens(self._h, _p(out)))
        return out

    def node_tokens(self):
        return dict(zip(self.node_ids(), self.node_tokens_array().tolist()))

    def snapshot_tick(self, sid):
        return self._get(self._L.cl_graph_snapshot_tick, C.c_int32, sid)

    def collect_arrays(self, sid):
        """(tokens[N] rank order, offsets[E+1], messages) with channels in (src, dest)
        rank order; raises ClSnapError(-9) if the snapshot has not completed."""
        n, e = self.num_nodes, self.num_channels
        tok = np.zeros(n, dtype=np.int64)
        off = np.zeros(e + 1, dtype=np.int64)
        cap = 1 << 16
        while True:
            msg = np.zeros(cap, dtype=np.int64)
            rc = self._L.cl_graph_collect_snapshot(self._h, sid, _p(tok), _p(off), _p(msg), cap)
            if rc == -7 and off[e] > cap:
                cap = int(off[e])
                continue
            _check(rc)
            return tok, off, msg[:off[e]]

    def CollectSnapshot(self, snapshot_id):         # sim.go:134
        """GlobalSnapshot, messages in (dest, src, delivery) order."""
        tok, off, msg = self.collect_arrays(snapshot_id)
        ids = self.node_ids()
        src, dst = self.channels()
        order = np.lexsort((src, dst))
        msgs = [MsgSnapshot(ids[src[c]], ids[dst[c]], int(msg[k]))
                for c in order for k in range(off[c], off[c + 1])]
        return GlobalSnapshot(snapshot_id, dict(zip(ids, tok.tolist())), msgs)

    def counters(self):
        out = np.zeros(len(COUNTER_NAMES), dtype=np.int64)
        _check(self._L.cl_graph_get_counters(self._h, _p(out)))
        return dict(zip(COUNTER_NAMES, out.tolist()))

    def checksums(self):
        out = np.zeros(len(GSUM_NAMES), dtype=np.int64)
        _check(self._L.cl_graph_get_checksums(self._h, _p(out)))
        return dict(zip(GSUM_NAMES, out.tolist()))

    # ---- device event trace: the reference's debug Logger (logger.go:12-76) ------------
    def trace_enable(self, capacity=1 << 16):
        """Record the Logger from the next run on (capacity records; 0 = off)."""
        _check(self._L.cl_graph_trace_enable(self._h, capacity))

    def trace(self):
        """LogEvents in Logger order: (epoch, kind, node rank, other rank | -1, data,
        nodeTokens); kinds LOG_* (include/clsnap.h CL_LOG_*)."""
        n = C.c_int32(0)
        _check(self._L.cl_graph_trace_read(self._h, None, 0, C.byref(n)))
        out = np.zeros((max(n.value, 1), 6), dtype=np.int32)
        _check(self._L.cl_graph_trace_read(self._h, _p(out), n.value, C.byref(n)))
        return [tuple(int(x) for x in r) for r in out[:n.value]]

    def pretty_print(self):
        """Logger.PrettyPrint (logger.go:55-64) as text."""
        return format_log(self.node_ids(), self.trace())


def bucket_capacity(src, dst, span, world):
    """Rows per device-exchange bucket of the partitioned mode: the most nodes of one rank
    with a channel into another rank's nodes (rank r owns node ranks [r * span, (r + 1) *
    span)).  Each sender delivers at most one packet per tick (sim.go:90), so this bounds
    the deliveries from r to q, the broadcast reports q sends r about r's senders, and r's
    replies to them."""
    w = world
    key = np.unique(np.asarray(src, dtype=np.int64) * w + np.asarray(dst, dtype=np.int64) // span)
    pair = (key // w) // span * w + key % w
    cnt = np.bincount(pair, minlength=w * w).reshape(w, w)
    np.fill_diagonal(cnt, 0)
    return max(int(cnt.max()), 1)


class PartitionedGraphSim:
    """ONE simulation over a graph split into contiguous node-rank ranges, one range per
    process / GPU (graph-partitioned mode, DESIGN.md §11, include/clgraph.h
    cl_graph_part_*).  Every rank builds the same topology and program; per tick the
    ranks exchange deliveries, broadcast-trigger reports, trigger totals and draw replies
    with dist.exchange_rows / allgather_ints (RCCL over xGMI with exchange_device="cuda",
    gloo on host tensors).  Results are gathered on every rank: the run equals the
    whole-graph engine's and the oracle's bit for bit (tests/test_partition_gpu.py).

    There is no reference counterpart (the reference runs one process); the exchange
    steps restate the tick of sim.go:71-95 across ranks (tests/partition_model.py is the
    same protocol on the CPU)."""

    def __init__(self, sim, rank, world, exchange_device="cpu", transport="host"):
        from . import dist as D
        if transport not in ("host", "device"):
            raise ValueError(f"transport {transport!r}: 'host' or 'device'")
        self.D, self.g, self.rank, self.world = D, sim, rank, world
        self.dev = exchange_device
        self.transport = transport
        n = sim.num_nodes
        blocks = -(-n // 256)
        per = -(-blocks // world)
        self.span = per * 256                    # node ranks per rank, block-aligned
        self.lo, self.hi = min(n, rank * self.span), min(n, (rank + 1) * self.span)
        if self.lo >= self.hi:
            raise ValueError(f"{world} ranks over {blocks} node blocks of 256: rank {rank} would own no nodes")
        self.n = n
        self._L = sim._L
        _check(self._L.cl_graph_part_begin(sim._h, self.lo, self.hi))
        self.time = 0
        self.n_sids = 0
        self._frozen = 0
        if transport == "device":
            self._dev_setup()

    @property
    def frozen(self):
        """Nonzero once the run stopped (every rank stops at the same step).  The device
        transport decides it on the device (cl_graph_part_dev_bases): read back here."""
        return self.g.status() if self.transport == "device" else self._frozen

    # ---- device-resident exchange (clgraph.h cl_graph_part_dev_*) ----------------------
    def bucket_capacity(self):
        """Rows per exchange bucket for this graph and rank split (bucket_capacity below)."""
        src, dst = self.g.channels()
        return bucket_capacity(src, dst, self.span, self.world)

    def _dev_setup(self):
        import torch
        dev = torch.device("cuda", self.g.device)
        self.cap = self.bucket_capacity()
        rows = self.world * (self.cap + 1)
        self._send = torch.zeros(2 * rows, dtype=torch.int64, device=dev)    # 16-B rows
        self._recv = torch.zeros_like(self._send)
        self._tsend = torch.zeros(4, dtype=torch.int64, device=dev)
        self._trecv = torch.zeros(4 * self.world, dtype=torch.int64, device=dev)
        self._stream = torch.cuda.Stream(device=dev)
        self.g._stream_ref = self._stream          # (outlives the engine's use of it)
        _check(self._L.cl_graph_set_stream(self.g._h, C.c_void_p(self._stream.cuda_stream)))
        _check(self._L.cl_graph_part_dev_bind(self.g._h, self.world, self.rank, self.span, self.cap,
                                              C.c_void_p(self._send.data_ptr()), C.c_void_p(self._recv.data_ptr()),
                                              C.c_void_p(self._tsend.data_ptr()), C.c_void_p(self._trecv.data_ptr())))

    def _a2a(self):
        """Bucket q of send to rank q, rank q's bucket for this rank into recv bucket q (RCCL
        on the device buffers; gloo rehearsals stage them through host memory)."""
        import torch
        import torch.distributed as dist
        with torch.cuda.stream(self._stream):
            if self.dev == "cuda":
                dist.all_to_all_single(self._recv, self._send)
            else:
                h = self._send.cpu()                # (after the engine's launches on this stream)
                r = torch.empty_like(h)
                dist.all_to_all_single(r, h)
                self._recv.copy_(r)

    def _gather(self):
        import torch
        import torch.distributed as dist
        with torch.cuda.stream(self._stream):
            if self.dev == "cuda":
                dist.all_gather_into_tensor(self._trecv, self._tsend)
            else:
                h = self._tsend.cpu()
                out = [torch.empty_like(h) for _ in range(self.world)]
                dist.all_gather(out, h)
                self._trecv.copy_(torch.cat(out))

    def _dev_finish(self, step):
        """reports -> tally -> totals -> bases + replies -> push, all on the device."""
        L, h = self._L, self.g._h
        self._a2a()
        _check(L.cl_graph_part_dev_tally(h, step))
        self._gather()
        _check(L.cl_graph_part_dev_bases(h))
        self._a2a()
        _check(L.cl_graph_part_dev_push(h, step))

    def owner(self, v):
        return np.asarray(v) // self.span

    def _by_owner(self, rows, col):
        if len(rows) == 0:
            return [np.zeros((0, rows.shape[1] if rows.ndim == 2 else 1), dtype=np.int64)] * self.world
        own = self.owner(rows[:, col])
        return [rows[own == r].astype(np.int64) for r in range(self.world)]

    def _finish_step(self, step, reports_by_src):
        """tally -> allgather totals -> bases -> replies -> push (the end of a tick, and the
        step-0 traffic with no reports)."""
        mine = np.concatenate([r for r in reports_by_src if len(r)] or [np.zeros((0, 2), dtype=np.int64)])
        rep = np.ascontiguousarray(mine, dtype=np.int32)
        tot = np.zeros(3, dtype=np.int64)
        _check(self._L.cl_graph_part_tally(self.g._h, step, _p(rep), len(rep), _p(tot)))
        allt = self.D.allgather_ints(tot.tolist(), self.dev)
        frozen = int(allt[:, 2].max())
        if frozen:                  # a device froze (its totals are stale): every device stops here
            if not tot[2]:
                _check(self._L.cl_graph_part_freeze(self.g._h, frozen))
            self._frozen = frozen
            return
        r = self.rank
        bases = np.array([allt[:r, 0].sum(), allt[:, 0].sum(), allt[:r, 1].sum(), allt[:, 1].sum()], dtype=np.int64)
        s0 = np.ascontiguousarray(rep[:, 0]) if len(rep) else np.zeros(0, dtype=np.int32)
        draw0 = np.zeros(max(len(s0), 1), dtype=np.int64)
        _check(self._L.cl_graph_part_bases(self.g._h, _p(bases), _p(s0), len(s0), _p(draw0)))
        replies, o = [], 0
        for src_rows in reports_by_src:            # back to the ranks that reported them
            k = len(src_rows)
            replies.append(np.stack([s0[o:o + k].astype(np.int64), draw0[o:o + k]], axis=1) if k
                           else np.zeros((0, 2), dtype=np.int64))
            o += k
        back = self.D.exchange_rows(replies, 2, self.dev)
        rows = np.ascontiguousarray(np.concatenate([b for b in back if len(b)] or [np.zeros((0, 2), dtype=np.int64)]),
                                    dtype=np.int64)
        _check(self._L.cl_graph_part_push(self.g._h, step, _p(rows), len(rows)))

    def start(self):
        """The step-0 traffic (the whole-graph engine runs it at reset)."""
        if self.transport == "device":
            _check(self._L.cl_graph_part_dev_seal(self.g._h))      # no reports
            self._dev_finish(0)
            return
        self._finish_step(0, [np.zeros((0, 2), dtype=np.int64)] * self.world)

    def start_snapshot_rank(self, node):            # sim.go:105 (called on every rank)
        sid = C.c_int32(-1)
        _check(self._L.cl_graph_part_snapshot(self.g._h, node, C.byref(sid)))
        self.n_sids += 1
        return sid.value

    def tick(self):                                 # sim.go:71-95 across the ranks
        h = self.g._h
        if self.transport == "device":              # no host round trip (a frozen run's kernels return)
            _check(self._L.cl_graph_part_dev_pick(h))
            self.time += 1
            self._a2a()
            _check(self._L.cl_graph_part_dev_receive(h))
            self._dev_finish(self.time)
            return
        if self._frozen:                            # (the run stopped on every rank)
            return
        out = np.zeros((max(self.hi - self.lo, 1), 4), dtype=np.int32)
        m = C.c_int64(0)
        _check(self._L.cl_graph_part_pick(h, _p(out), out.shape[0], C.byref(m)))
        self.time += 1
        inbox = self.D.exchange_rows(self._by_owner(out[:m.value], 1), 4, self.dev)
        rows = np.ascontiguousarray(np.concatenate([b for b in inbox if len(b)] or [np.zeros((0, 4), dtype=np.int64)]),
                                    dtype=np.int32)
        reps = np.zeros((max(len(rows), 1), 2), dtype=np.int32)
        q = C.c_int64(0)
        _check(self._L.cl_graph_part_receive(h, _p(rows), len(rows), _p(reps), reps.shape[0], C.byref(q)))
        got = self.D.exchange_rows(self._by_owner(reps[:q.value], 0), 2, self.dev)
        self._finish_step(self.time, got)

    def run_program(self, steps, snap_step=(), snap_rank=()):
        """The synthetic program: for step k, snapshots scheduled at k,
        one tick (whose end pushes the traffic of step k + 1)."""
        self.start()
        si = 0
        for k in range(steps):
            while si < len(snap_step) and snap_step[si] == k:
                self.start_snapshot_rank(int(snap_rank[si]))
                si += 1
            self.tick()

    def completion_ticks(self):
        """Global completion tick of each snapshot (-1 if some rank's nodes are not all done):
        the latest of the ranks' local completion ticks."""
        loc = [self.g.snapshot_tick(s) for s in range(self.n_sids)]
        allc = self.D.allgather_ints(loc or [0], self.dev)[:, :len(loc)]
        return [int(allc[:, s].max()) if (allc[:, s] >= 0).all() else -1 for s in range(len(loc))]

    def drain(self, max_ticks=10000):
        """test_common.go:123-137 across the ranks: tick until every snapshot started so far
        has completed on every rank, then maxDelay + 1 more ticks."""
        for _ in range(max_ticks + 1):
            if self.frozen:
                return False
            if all(x >= 0 for x in self.completion_ticks()):
                for _ in range(6):
                    self.tick()
                return True
            self.tick()
        return False

    def results(self):
        """(status, final tokens[n], completion ticks, counters, {sid: (tokens[n], offsets,
        payloads)} for completed snapshots), gathered on every rank."""
        import torch.distributed as dist
        g = self.g
        cnt = g.counters()
        st = g.status()
        tok = g.node_tokens_array()[self.lo:self.hi]
        ct = self.completion_ticks()
        src, dst = g.channels()
        mine = (dst >= self.lo) & (dst < self.hi)
        snaps = {}
        for sid, c in enumerate(ct):
            if c < 0:
                continue
            t, off, msg = g.collect_arrays(sid)
            per = [msg[off[k]:off[k + 1]] for k in np.nonzero(mine)[0]]
            snaps[sid] = (t[self.lo:self.hi], np.nonzero(mine)[0], per)
        allr = [None] * self.world
        dist.all_gather_object(allr, (st, tok, cnt, snaps))
        status = max(r[0] for r in allr)
        tokens = np.concatenate([r[1] for r in allr])
        counters = {k: sum(r[2][k] for r in allr) for k in ("push", "peek", "pop_tok", "pop_mk", "recorded")}
        counters["completed"] = sum(1 for x in ct if x >= 0)
        out = {}
        e = len(src)
        for sid in snaps:
            stok = np.concatenate([r[3][sid][0] for r in allr])
            lists = [None] * e
            for r in allr:
                for c, m in zip(r[3][sid][1], r[3][sid][2]):
                    lists[c] = m
            off = np.zeros(e + 1, dtype=np.int64)
            off[1:] = np.cumsum([len(x) for x in lists])
            vals = np.concatenate(lists) if e else np.zeros(0, dtype=np.int64)
            out[sid] = (stok, off, vals)
        return status, tokens, ct, counters, out
