"""Independent pure-Python restatement of DistributeOctTree
(R/src/ORBextractor.cpp:571-817) with literal std::list semantics, used only to
cross-check the C oracle on small inputs (TEST INFRASTRUCTURE).  Equal-size
nodes are ordered by creation sequence (the pinned stand-in for the
reference's pointer order)."""
import math


class Node:
    __slots__ = ("ul", "ur", "bl", "br", "keys", "nomore", "seq")

    def __init__(self, seq):
        self.keys = []
        self.nomore = False
        self.seq = seq


def _divide(n, kx, ky, mk):
    halfX = int(math.ceil(float(n.ur[0] - n.ul[0]) / 2))
    halfY = int(math.ceil(float(n.br[1] - n.ul[1]) / 2))
    c = [mk() for _ in range(4)]
    c[0].ul = n.ul; c[0].ur = (n.ul[0] + halfX, n.ul[1]); c[0].bl = (n.ul[0], n.ul[1] + halfY)
    c[0].br = (n.ul[0] + halfX, n.ul[1] + halfY)
    c[1].ul = c[0].ur; c[1].ur = n.ur; c[1].bl = c[0].br; c[1].br = (n.ur[0], n.ul[1] + halfY)
    c[2].ul = c[0].bl; c[2].ur = c[0].br; c[2].bl = n.bl; c[2].br = (c[0].br[0], n.bl[1])
    c[3].ul = c[2].ur; c[3].ur = c[1].br; c[3].bl = c[2].br; c[3].br = n.br
    for k in n.keys:
        if kx[k] < c[0].ur[0]:
            (c[0] if ky[k] < c[0].br[1] else c[2]).keys.append(k)
        elif ky[k] < c[0].br[1]:
            c[1].keys.append(k)
        else:
            c[3].keys.append(k)
    for q in c:
        if len(q.keys) == 1:
            q.nomore = True
    return c


def distribute_octree(kx, ky, kr, minX, maxX, minY, maxY, N):
    import numpy as np
    kx = np.asarray(kx, np.float32)
    ky = np.asarray(ky, np.float32)
    seq = [0]

    def fresh():          # child objects are only "allocated" when pushed (see push)
        return Node(-1)

    def push_front(lst, c):
        c.seq = seq[0]
        seq[0] += 1
        lst.insert(0, c)

    nIni = int(np.round(np.float32(maxX - minX) / np.float32(maxY - minY)))
    hX = np.float32(maxX - minX) / np.float32(nIni)
    lst = []
    for i in range(nIni):
        n = Node(seq[0]); seq[0] += 1
        n.ul = (int(hX * np.float32(i)), 0); n.ur = (int(hX * np.float32(i + 1)), 0)
        n.bl = (n.ul[0], maxY - minY); n.br = (n.ur[0], maxY - minY)
        lst.append(n)
    for i in range(len(kx)):
        lst[int(kx[i] / hX)].keys.append(i)
    lst = [n for n in lst if n.keys]
    for n in lst:
        if len(n.keys) == 1:
            n.nomore = True
    finish = False
    while not finish:
        prev = len(lst)
        vsize = []
        nexp = 0
        idx = 0
        while idx < len(lst):
            n = lst[idx]
            if n.nomore:
                idx += 1
                continue
            for c in _divide(n, kx, ky, fresh):
                if c.keys:
                    push_front(lst, c)
                    idx += 1
                    if len(c.keys) > 1:
                        nexp += 1
                        vsize.append(c)
            lst.pop(idx)
        if len(lst) >= N or len(lst) == prev:
            finish = True
        elif len(lst) + nexp * 3 > N:
            while not finish:
                prev = len(lst)
                vprev = sorted(vsize, key=lambda n: (len(n.keys), n.seq))
                vsize = []
                for j in range(len(vprev) - 1, -1, -1):
                    for c in _divide(vprev[j], kx, ky, fresh):
                        if c.keys:
                            push_front(lst, c)
                            if len(c.keys) > 1:
                                vsize.append(c)
                    lst.remove(vprev[j])
                    if len(lst) >= N:
                        break
                if len(lst) >= N or len(lst) == prev:
                    finish = True
    out = []
    for n in lst:
        best = n.keys[0]
        for k in n.keys[1:]:
            if kr[k] > kr[best]:
                best = k
        out.append(best)
    return out
