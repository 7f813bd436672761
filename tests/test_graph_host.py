"""CPU tests of the graph engine's host side (no GPU): the C ABI exports, the counter
hash against the oracle and the numpy restatement, the synthetic graph generators
against tests/graphgen.py, topology freezing, argument validation, and that the
product fails loudly (CL_E_DEVICE) when no gfx950 GPU is present.

The oracle's graph driver is checked here too: its bulk builder must equal the
reference's own readTopologyFile path, and its runs must conserve tokens and produce
consistent cuts.
"""
import os
import re

import numpy as np
import pytest

import graphgen as G
import oracle as O
from graphcheck import clg, cl, oracle_program, powerlaw_program, regular_program, digest_from_oracle
from snapcheck import ROOT, TEST_DATA

HEADER = os.path.join(ROOT, "include", "clgraph.h")


def test_exports_every_declared_symbol():
    names = re.findall(r"^(?:int|uint64_t)\s+(cl_\w+)\(", open(HEADER).read(), re.M)
    assert len(names) >= 40
    L = clg.glib()
    for n in names:
        assert hasattr(L, n), n


def test_counter_hash_three_ways():
    rng = np.random.default_rng(5)
    for _ in range(200):
        s, a, b = (int(x) for x in rng.integers(0, 2**63, size=3, dtype=np.uint64))
        want = G.counter_hash(s, a, b)
        assert clg.counter_hash(s, a, b) == want
        assert O.counter_hash(s, a, b) == want
    a = np.arange(1000, dtype=np.uint64)
    np.testing.assert_array_equal(G.counter_hash_np(7, a, a * 3),
                                  [G.counter_hash(7, int(x), int(x) * 3) for x in a])
    for k in range(100):
        assert O.counter_delay(99, k) == (G.counter_hash(99, k, 0) >> 32) % 5


def _edges(g):
    s, d = g.channels()
    return s.astype(np.int64), d.astype(np.int64)


@pytest.mark.parametrize("n", [1, 2, 7, 1000, 4096])
def test_regular_generator_matches_restatement(n):
    g = clg.GraphSim()
    g.generate_regular(n, 8, 100, seed=1234)
    s, d = _edges(g)
    ws, wd = G.regular_graph(n, 8, 1234)
    np.testing.assert_array_equal(s, ws)
    np.testing.assert_array_equal(d, wd)
    assert g.num_nodes == n
    assert g.node_ids()[0] == "N" + "0" * len(str(n - 1))


@pytest.mark.parametrize("n", [3, 100, 2000, 20000])
def test_powerlaw_generator_matches_restatement(n):
    g = clg.GraphSim()
    g.generate_powerlaw(n, 8, 0.9, True, 100, seed=77)
    s, d = _edges(g)
    ws, wd = G.powerlaw_graph(n, 8, 0.9, True, 77)
    np.testing.assert_array_equal(s, ws)
    np.testing.assert_array_equal(d, wd)
    indeg = np.bincount(d, minlength=n)
    if n >= 2000:
        assert indeg[0] > 20 * np.median(indeg)   # skewed in-degree: rank 0 is the hub
    assert np.bincount(s, minlength=n).max() <= 10  # bounded out-degree


def test_topology_from_top_file_is_rank_ordered():
    g = clg.GraphSim()
    g.read_topology_file(os.path.join(TEST_DATA, "10nodes.top"))
    ids = g.node_ids()
    assert ids == sorted(ids) and ids[:3] == ["N1", "N10", "N2"]   # getSortedKeys: N10 < N2
    s, d = g.channels()
    pairs = list(zip(s.tolist(), d.tolist()))
    assert pairs == sorted(pairs)
    o = O.OracleSim()
    o.read_topology(os.path.join(TEST_DATA, "10nodes.top"))
    assert o.node_ids() == ids


def test_validation_errors():
    g = clg.GraphSim()
    g.AddNode("A", 5)
    with pytest.raises(cl.ClSnapError) as e:
        g.AddNode("A", 1)
    assert e.value.code == -3
    with pytest.raises(cl.ClSnapError) as e:
        g.AddLink("A", "B")
    assert e.value.code == -2
    g.AddNode("B", 0)
    g.AddLink("A", "B")
    with pytest.raises(cl.ClSnapError) as e:
        g.StartSnapshot("C")
    assert e.value.code == -2
    g.Tick(1)
    with pytest.raises(cl.ClSnapError) as e:
        g.AddNode("C", 1)
    assert e.value.code == -8
    with pytest.raises(cl.ClSnapError):
        g.set_limits(fifo_slots=3)
    star = clg.GraphSim()
    with pytest.raises(cl.ClSnapError) as e:   # out-degree above the 64-bit channel mask
        star.set_topology(np.full(100, 1), np.zeros(99, dtype=np.int32), np.arange(1, 100, dtype=np.int32))
    assert e.value.code == -7


def test_no_gpu_fails_loudly():
    """The product never falls back to the CPU: without a gfx950 device it raises."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    g = clg.GraphSim()
    g.read_topology_file(os.path.join(TEST_DATA, "2nodes.top"))
    g.Tick(1)
    with pytest.raises(cl.ClSnapError) as e:
        g.flush()
    assert e.value.code == -6


# ---- the oracle's graph driver ------------------------------------------------------

def test_oracle_bulk_builder_equals_reference_parser():
    """orc_build_graph + traffic must equal the reference's AddNode/AddLink path."""
    n = 40
    src, dst = G.regular_graph(n, 3, 5)
    text = f"{n}\n" + "".join(f"N{r:02d} {100 + r}\n" for r in range(n)) + \
        "".join(f"N{a:02d} N{b:02d}\n" for a, b in zip(src, dst))
    a = O.OracleSim()
    a.read_topology_text(text)
    b = O.OracleSim()
    b.build_graph(100 + np.arange(n), src, dst, 2)
    for s in (a, b):
        s.use_counter_hash(3)
        s.run_program(60, 9, 1 << 30, 60, [4, 9], [3, 17])
    assert a.counters() == b.counters()
    assert a.node_tokens() == b.node_tokens()
    for sid in range(2):
        ta, oa, va = a.collect_channels(sid)
        tb, ob, vb = b.collect_channels(sid)
        np.testing.assert_array_equal(ta, tb)
        np.testing.assert_array_equal(oa, ob)
        np.testing.assert_array_equal(va, vb)


@pytest.mark.parametrize("kind", ["regular", "powerlaw"])
def test_oracle_program_conserves_tokens(kind):
    p = regular_program(512, steps=70) if kind == "regular" else powerlaw_program(300, 300, 8)
    o = oracle_program(p)
    assert o.status == 0
    total = int(p.tokens.sum())
    done = 0
    for sid in range(o.num_snapshots):
        if not o.complete(sid):
            continue
        done += 1
        tok, off, vals = o.collect_channels(sid)
        assert tok.sum() + vals.sum() == total     # consistent cut
    assert done >= 1
    assert o.counters()["draws"] == o.counters()["push"]
    assert isinstance(digest_from_oracle(o), int)


def _topology_text(n, src, dst, tokens=100, comments=False):
    w = len(str(n - 1))
    lines = [f"{n}"] + [f"N{r:0{w}d} {tokens}" for r in range(n)]
    for i, (a, b) in enumerate(zip(src, dst)):
        if comments and i % 100000 == 7:
            lines.append("# a comment inside the link section")
        lines.append(f"N{a:0{w}d} N{b:0{w}d}")
    return "\n".join(lines) + "\n"


def test_streaming_topology_parse_matches_bulk_topology():
    """readTopologyFile over a C4-shaped text (2^17 nodes, ~1M link lines, comments,
    self links and duplicate links): the streaming parser (parallel link section) builds
    the same channels and ids as the bulk rank API."""
    n = 1 << 17
    ws, wd = G.regular_graph(n, 8, 99)
    src = np.concatenate([ws, [5, 6, int(ws[0])]]).astype(np.int64)
    dst = np.concatenate([wd, [5, 6, int(wd[0])]]).astype(np.int64)   # self links + a duplicate
    g = clg.GraphSim()
    g.read_topology_text(_topology_text(n, src, dst, comments=True))
    b = clg.GraphSim()
    b.set_topology(np.full(n, 100), src.astype(np.int32), dst.astype(np.int32), id_width=len(str(n - 1)))
    gs, gd = _edges(g)
    bs, bd = _edges(b)
    np.testing.assert_array_equal(gs, bs)
    np.testing.assert_array_equal(gd, bd)
    assert g.node_ids()[:3] == b.node_ids()[:3] and g.node_ids()[-1] == b.node_ids()[-1]


def test_streaming_topology_parse_reports_first_error_in_file_order():
    """Errors in different parallel chunks: the one earlier in the file is reported,
    with the reference's message (sim.go:49-54, test_common.go:51-53)."""
    n = 1 << 16
    ws, wd = G.regular_graph(n, 8, 3)
    text = _topology_text(n, ws, wd)
    lines = text.split("\n")
    k1, k2 = int(len(lines) * 0.4), int(len(lines) * 0.8)
    a = list(lines)
    a[k1] = "N00001 Nxyz"          # unknown node, earlier
    a[k2] = "N00001 N00002 N00003"  # three fields, later
    g = clg.GraphSim()
    with pytest.raises(cl.ClSnapError) as e:
        g.read_topology_text("\n".join(a))
    assert e.value.code == -2 and "Nxyz does not exist" in str(e.value)
    b = list(lines)
    b[k1] = "N00001 N00002 N00003"
    b[k2] = "N00001 Nxyz"
    g = clg.GraphSim()
    with pytest.raises(cl.ClSnapError) as e:
        g.read_topology_text("\n".join(b))
    assert e.value.code == -4 and "Expected 2 tokens" in str(e.value)


def test_partitioned_mode_argument_checks():
    """cl_graph_part_begin validates the node range and the run before touching a device;
    PartitionedGraphSim refuses ranks that would own no node block."""
    import ctypes as C
    src, dst = G.regular_graph(1000, 4, 1)
    L = clg.glib()

    def fresh(**kw):
        g = clg.GraphSim()
        g.set_topology(np.full(1000, 5), src, dst)
        return g
    g = fresh()
    for lo, hi in ((0, 300), (100, 1000), (512, 256), (-256, 0), (0, 1024)):
        assert L.cl_graph_part_begin(g._h, lo, hi) == -1, (lo, hi)   # CL_E_INVALID
    g.Tick(1)
    assert L.cl_graph_part_begin(g._h, 0, 1000) == -8                # a program exists: CL_E_STATE
    g = fresh()
    g.set_delay_go_seed(7)
    assert L.cl_graph_part_begin(g._h, 0, 1000) == -8                # Go streams are per-process
    g = fresh()
    g.trace_enable(16)
    assert L.cl_graph_part_begin(g._h, 0, 512) == -8
    g = fresh()
    assert L.cl_graph_part_pick(g._h, None, 0, C.byref(C.c_int64())) == -8   # not partitioned
    with pytest.raises(cl.ClSnapError):
        clg.PartitionedGraphSim(fresh(), 3, 4)        # a valid range: fails loudly without a GPU
    with pytest.raises(ValueError):
        clg.PartitionedGraphSim(fresh(), 2, 3)        # 4 blocks over 3 ranks: 2 + 2 + 0
