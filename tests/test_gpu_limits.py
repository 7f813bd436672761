"""Edge sizes of the node-parallel kernel against the oracle: a full 64-lane wave of
nodes (one instance per wave), the 32-snapshot limit, and high-degree nodes that select
the runtime-loop kernels (D = 16, 64: in-link words in LDS instead of registers)."""
import numpy as np
import pytest

import oracle as O
from enginecheck import compare_instance, engine_run, oracle_run


def _scenario(rng, ids, edges, n_events, n_snaps, tok_range=(5, 40)):
    top = f"{len(ids)}\n" + "".join(f"{i} {int(rng.integers(*tok_range))}\n" for i in ids)
    top += "".join(f"{a} {b}\n" for a, b in sorted(edges))
    out = {}
    for a, b in edges:
        out.setdefault(a, []).append(b)
    snap_at = set(rng.choice(n_events, n_snaps, replace=False).tolist())
    ev = []
    for k in range(n_events):
        if k in snap_at:
            ev.append(f"snapshot {rng.choice(ids)}")
        elif rng.random() < 0.7:
            a = str(rng.choice(ids))
            ev.append(f"send {a} {rng.choice(out[a])} {int(rng.integers(0, 3))}")
        else:
            ev.append(f"tick {int(rng.integers(1, 3))}")
    return top, "\n".join(ev) + "\n"


def _compare_all(top, events, n, **kw):
    sim = engine_run(top, events, n, **kw)
    status, times = sim.status(), sim.time()
    for i in range(n):
        compare_instance(sim, i, oracle_run(top, events, seed=O.REFERENCE_SEED + i), status=status, times=times)
    return status


@pytest.mark.gpu
def test_full_wave_64_nodes_32_snapshots():
    """N = 64: one instance fills a wave (segment mask = all lanes); 32 snapshot ids."""
    rng = np.random.default_rng(7)
    ids = [f"N{k:02d}" for k in range(64)]
    edges = {(ids[k], ids[(k + 1) % 64]) for k in range(64)} | {(ids[k], ids[(k - 1) % 64]) for k in range(64)}
    for _ in range(64):
        a, b = rng.choice(64, 2, replace=False)
        edges.add((ids[a], ids[b]))
    top, events = _scenario(rng, ids, edges, 160, 32)
    status = _compare_all(top, events, 64)
    assert (status == 0).any()


@pytest.mark.gpu
@pytest.mark.parametrize("n_nodes,seed", [(17, 1), (17, 2)])
def test_complete_digraph_degree_16(n_nodes, seed):
    """Every node linked to every other (degree 16: the D = 16 runtime-loop kernel), with
    many same-tick deliveries into one receiver from up to 16 senders."""
    rng = np.random.default_rng(seed)
    ids = [f"N{k}" for k in range(1, n_nodes + 1)]     # N10 < N2: rank != numeric order
    edges = {(a, b) for a in ids for b in ids if a != b}
    top, events = _scenario(rng, ids, edges, 80, 12)
    _compare_all(top, events, 128, fifo_lds_slots=2)


@pytest.mark.gpu
@pytest.mark.parametrize("n_nodes", [40, 64])
def test_hub_degree(n_nodes):
    """A hub linked both ways to every other node (degree 39 / 63: the D = 64 kernel) on
    a ring.  One wave's state then needs up to ~100 KB of LDS: the host launches fewer
    waves per workgroup instead of refusing the topology."""
    rng = np.random.default_rng(11 + n_nodes)
    ids = [f"N{k:02d}" for k in range(n_nodes)]
    edges = {(ids[k], ids[(k + 1) % n_nodes]) for k in range(n_nodes)}
    edges |= {(ids[0], b) for b in ids[1:]} | {(b, ids[0]) for b in ids[1:]}
    top, events = _scenario(rng, ids, edges, 120, 8)
    _compare_all(top, events, 64 if n_nodes < 64 else 32, fifo_lds_slots=2)
