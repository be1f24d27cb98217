"""TEST INFRASTRUCTURE ONLY (never imported by the product): pure-Python restatement of the
reference's PC-stable orientation, used to check libfastbn's `pc_orient.cpp` edge for edge.

Follows src/PCStable.cpp:576-843 (OrientVStructure, OrientImplied, Direct, Rule1-3/R3Helper) on top
of the reference's Network edge-list semantics (src/Network.cpp:229-399: AddDirectedEdge with the
cycle roll-back, DeleteDirectedEdge / DeleteUndirectedEdge erase the first match, AddUndirectedEdge
appends (min, max)).  Small graphs only (pure-Python loops).
"""

TAIL, ARROW = "T", "A"


class _Net:
    def __init__(self, n, skeleton):
        self.n = n
        self.edges = [(min(a, b), max(a, b), TAIL, TAIL) for a, b in skeleton]  # vec_edges
        self.adj = [set() for _ in range(n)]
        for a, b in skeleton:
            self.adj[a].add(b)
            self.adj[b].add(a)
        self.par = [set() for _ in range(n)]

    def _cyclic(self):
        indeg = [0] * self.n
        for c in range(self.n):
            indeg[c] = len(self.par[c])
        children = [[] for _ in range(self.n)]
        for c in range(self.n):
            for p in self.par[c]:
                children[p].append(c)
        stack = [i for i in range(self.n) if indeg[i] == 0]
        seen = 0
        while stack:
            u = stack.pop()
            seen += 1
            for c in children[u]:
                indeg[c] -= 1
                if indeg[c] == 0:
                    stack.append(c)
        return seen != self.n

    def add_directed(self, p, c):
        self.par[c].add(p)
        self.edges.append((p, c, TAIL, ARROW))
        if self._cyclic():
            self.del_directed(p, c)
            return False
        return True

    def del_directed(self, p, c):
        e = (p, c, TAIL, ARROW)
        if e not in self.edges:
            return False
        self.edges.remove(e)  # first match
        self.par[c].discard(p)
        return True

    def add_undirected(self, a, b):
        self.edges.append((min(a, b), max(a, b), TAIL, TAIL))

    def del_undirected(self, a, b):
        e = (min(a, b), max(a, b), TAIL, TAIL)
        if e not in self.edges:
            return False
        self.edges.remove(e)
        return True

    def adjacent(self, a, b):
        return 0 <= a < self.n and b in self.adj[a]

    def directed(self, a, b):
        return a in self.par[b]

    def undirected(self, a, b):
        return self.adjacent(a, b) and not self.directed(a, b) and not self.directed(b, a)


def orient(n, skeleton, sepset):
    """skeleton: [(x, y)] in vec_edges order; sepset: {(x, y): Z} for x < y.
    Returns [(from, to, 1)] arcs and [(min, max, 0)] undirected edges in final vec_edges order."""
    g = _Net(n, skeleton)
    for b in range(n):  # OrientVStructure
        nb = sorted(g.adj[b])
        for i in range(len(nb)):
            for j in range(i + 1, len(nb)):
                a, c = nb[i], nb[j]
                if g.adjacent(a, c) or b in sepset.get((a, c), ()):
                    continue
                dd1 = g.del_directed(b, a)
                du1 = False if dd1 else g.del_undirected(a, b)
                dd2 = g.del_directed(b, c)
                du2 = False if dd2 else g.del_undirected(c, b)
                ok1 = g.add_directed(a, b) if (dd1 or du1) else False
                ok2 = g.add_directed(c, b) if (dd2 or du2) else False
                if (dd1 or du1) and not ok1:
                    g.add_directed(b, a) if dd1 else g.add_undirected(a, b)
                if (dd2 or du2) and not ok2:
                    g.add_directed(b, c) if dd2 else g.add_undirected(c, b)

    def direct(a, c):
        g.del_undirected(a, c)
        ok = g.add_directed(a, c)
        if not ok:
            g.add_undirected(a, c)
        return ok

    def common(x, y):
        return sorted(g.adj[x] & g.adj[y])

    def rule1(b, c):
        for a in sorted(g.par[b]):
            if g.adjacent(c, a):
                continue
            if direct(b, c):
                return True
        return False

    def rule2(a, c):
        for b in common(a, c):
            if g.directed(a, b) and g.directed(b, c) and direct(a, c):
                return True
        return False

    def rule3(d, a):
        cm = common(a, d)
        if len(cm) < 2:
            return False
        for b in range(len(cm)):  # positions used as node ids (reference behaviour)
            for c in range(b + 1, len(cm)):
                if not g.adjacent(b, c):
                    if g.undirected(d, b) and g.undirected(d, c) and g.directed(b, a) and g.directed(c, a):
                        if direct(d, a):
                            return True
        return False

    changed = True
    while changed:  # OrientImplied
        changed = False
        i = 0
        while i < len(g.edges):
            x, y = g.edges[i][0], g.edges[i][1]
            if g.undirected(x, y):
                if rule1(x, y) or rule1(y, x) or rule2(x, y) or rule2(y, x) or rule3(x, y) or rule3(y, x):
                    changed = True
                else:
                    i += 1
            else:
                i += 1
    out = []
    for a, b, e1, e2 in g.edges:
        if e1 == TAIL and e2 == TAIL:
            out.append((a, b, 0))
        elif e1 == TAIL:
            out.append((a, b, 1))
        else:
            out.append((b, a, 1))
    return out
