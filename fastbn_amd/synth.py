"""Seeded synthetic workloads for benches and parity tests (numpy, host side).

* ``read_xmlbif`` -- XMLBIF -> (names, dims, parents in GIVEN order, CPTs) using the reference's CPT
  convention: count = int(p*10000) (src/XMLBIFParser.cpp:176), P = (count+1)/(sum+|dom|)
  (src/DiscreteNode.cpp:152-161), TABLE node-major (src/common.cpp:193-232).
* ``forward_sample`` -- ancestral sampling of complete cases (column store uint8 [var][sample]).
* ``evidence_cases`` -- JT test cases in the reference's format: var 0 is the query, k evidence
  variables drawn without replacement from 1..V-1 and set to their sampled values.
* ``random_network`` -- "Munin-like"/synthetic DAGs: parents drawn from a sliding window of
  earlier nodes, Dirichlet(1) CPT rows rounded to 4 decimals, written as XMLBIF in the reference's
  node-major TABLE layout.
The reference's own generator (src/SampleSetGenerator.cpp) is wall-clock seeded and unreachable
from its CLI, so these generators are new; all randomness comes from numpy's PCG64 with the seed.
"""
import xml.etree.ElementTree as ET

import numpy as np


def read_xmlbif(path):
    root = ET.parse(path).getroot()
    net = root.find("NETWORK")
    names, dims = [], []
    for v in net.findall("VARIABLE"):
        if v.find("TYPE").text.strip() != "discrete":
            continue
        names.append(v.find("NAME").text.strip())
        dims.append(len(v.findall("VALUE")))
    idx = {n: i for i, n in enumerate(names)}
    parents = [[] for _ in names]
    cpts = [None] * len(names)
    for p in net.findall("PROBABILITY"):
        v = idx[p.find("FOR").text.strip()]
        given = [idx[g.text.strip()] for g in p.findall("GIVEN")]
        vals = [float(t) for t in p.find("TABLE").text.strip().split(" ")]
        shape = [dims[v]] + [dims[g] for g in given]
        # int(p*10000): truncation of the double product, as the C++ int conversion does
        counts = np.array([int(x * 10000) for x in vals], np.int64).reshape(shape)
        tot = counts.sum(axis=0, keepdims=True)
        prob = (counts + 1.0) / (tot + 1.0 * dims[v])
        parents[v] = given
        cpts[v] = prob  # [node value, given...]
    return names, np.array(dims, np.int32), parents, cpts


def _topo(parents):
    n = len(parents)
    indeg = [len(set(p)) for p in parents]
    children = [[] for _ in range(n)]
    for c, ps in enumerate(parents):
        for p in set(ps):
            children[p].append(c)
    order, stack = [], [i for i in range(n) if indeg[i] == 0][::-1]
    while stack:
        u = stack.pop()
        order.append(u)
        for c in children[u]:
            indeg[c] -= 1
            if indeg[c] == 0:
                stack.append(c)
    if len(order) != n:
        raise ValueError("network has a cycle")
    return order


def forward_sample(net, n, seed):
    """net = read_xmlbif(...) tuple; returns uint8 [V][n]."""
    names, dims, parents, cpts = net
    rng = np.random.Generator(np.random.PCG64(seed))
    V = len(names)
    out = np.zeros((V, n), np.uint8)
    for v in _topo(parents):
        prob = cpts[v]
        if parents[v]:
            rows = prob.reshape(dims[v], -1)  # [value][parent config], GIVEN order, last fastest
            pc = np.zeros(n, np.int64)
            for g in parents[v]:
                pc = pc * dims[g] + out[g]
            cdf = np.cumsum(rows[:, pc], axis=0)  # [value][n]
        else:
            cdf = np.cumsum(prob.reshape(dims[v], 1), axis=0) * np.ones((1, n))
        u = rng.random(n) * cdf[-1]
        out[v] = np.minimum((u[None, :] >= cdf).sum(axis=0), dims[v] - 1).astype(np.uint8)
    return out


def evidence_cases(net, n, k, seed, query=0):
    """int8 [n][V]: k observed variables per case (never the query), -1 elsewhere."""
    names, dims, parents, cpts = net
    V = len(names)
    full = forward_sample(net, n, seed)
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    cand = np.array([v for v in range(V) if v != query])
    k = max(0, min(k, cand.size))
    keys = rng.random((n, cand.size))
    # k distinct candidates per case: the k smallest keys (argpartition: same set as a full sort)
    pick = cand[np.argpartition(keys, k - 1, axis=1)[:, :k]] if 0 < k < cand.size else cand[np.argsort(keys, axis=1)[:, :k]]
    ev = np.full((n, V), -1, np.int8)
    rows = np.repeat(np.arange(n), k)
    cols = pick.reshape(-1)
    ev[rows, cols] = full[cols, rows].astype(np.int8)
    return ev


def random_network(n_nodes, seed, window=12, parent_probs=(0.8, 0.15, 0.05), dom=(2, 5), path=None,
                   name="synthetic", k_min=1, fan_in=None):
    """Random DAG over nodes 0..n-1: node i > 0 draws k parents from the previous `window` nodes,
    P(k = k_min, k_min + 1, ...) = parent_probs (default: k >= 1, mean 1.25 parents per node, i.e.
    ~1300 arcs at 1041 nodes like Munin3).  k_min = 1 keeps the DAG connected, which the JT path
    needs: the reference's Prim step has no junction-forest support
    (src/JunctionTreeStructure.cpp:262-281); the PC datasets use k_min = 0.
    fan_in = {node: k}: those nodes draw exactly k parents (wide cliques for tests; every other
    node's draw is unchanged)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    dims = rng.integers(dom[0], dom[1] + 1, size=n_nodes)
    pp = np.asarray(parent_probs, float) / np.sum(parent_probs)
    parents = []
    for i in range(n_nodes):
        lo = max(0, i - window)
        k = min(int(rng.choice(np.arange(k_min, k_min + pp.size), p=pp)), i - lo) if i > 0 else 0
        if fan_in and i in fan_in:
            k = min(int(fan_in[i]), i - lo)
        ps = sorted(rng.choice(np.arange(lo, i), size=k, replace=False).tolist()) if k else []
        parents.append(ps)
    cpts = []
    for i in range(n_nodes):
        ncfg = int(np.prod([dims[p] for p in parents[i]])) if parents[i] else 1
        rows = rng.dirichlet(np.ones(dims[i]), size=ncfg)  # [cfg][value]
        rows = np.round(rows, 4)
        cpts.append(rows)
    if path is not None:
        with open(path, "w") as f:
            f.write('<?xml version="1.0" encoding="UTF-8"?>\n<BIF>\n<NETWORK>\n<NAME>%s</NAME>\n' % name)
            for i in range(n_nodes):
                f.write("<VARIABLE>\n<NAME>X%d</NAME>\n<TYPE>discrete</TYPE>\n" % i)
                for s in range(dims[i]):
                    f.write("<VALUE>s%d</VALUE>\n" % s)
                f.write("</VARIABLE>\n")
            for i in range(n_nodes):
                f.write("<PROBABILITY>\n<FOR>X%d</FOR>\n" % i)
                for p in parents[i]:
                    f.write("<GIVEN>X%d</GIVEN>\n" % p)
                # node-major: node value most significant, then parents (last fastest)
                vals = cpts[i].T.reshape(-1)
                f.write("<TABLE>%s </TABLE>\n</PROBABILITY>\n" % " ".join("%.4f" % x for x in vals))
            f.write("</NETWORK>\n</BIF>\n")
    return dims, parents, cpts


def config5_dataset(nvars=1000, nsamples=100_000, seed=1000):
    """SURVEY §8(d) config 5 dataset: node i draws k ~ U{0..2} parents from the previous 50,
    domains U{2..4}, Dirichlet(1) CPTs (4 decimals, XMLBIF round trip), forward sampling, seed 1000.
    Returns (uint8 columns [nvars][nsamples], dims = observed state counts)."""
    import os
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "pc_c5.xml")
        random_network(nvars, seed=seed, window=50, parent_probs=(1, 1, 1), dom=(2, 4), path=path, k_min=0)
        cols = forward_sample(read_xmlbif(path), nsamples, seed=seed)
    return cols, (cols.max(axis=1).astype(np.int32) + 1)
