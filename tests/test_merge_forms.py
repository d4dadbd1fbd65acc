"""The three forms k_tree uses for the reference's Huffman merge (fcx_entropy.hip), checked on the
CPU against the oracle's restatement of the reference's sorted-list re-insertion
(oracle/fcx_oracle.c orc_huffman_tree, my_compress.cpp:570-611; pinned to the reference by the
huffman_tree KATs in test_oracle.py):

  serial      the two-queue merge (sorted leaves, internal nodes in creation order, a leaf first
              on a tie), one thread
  closed      when the two lightest leaves outweigh the heaviest: step k takes S[2k], S[2k+1] of
              S = sorted leaves ++ internal nodes
  fixed point P = the sorted merge of the leaves L and the internal weights I, I[k] = P[2k] +
              P[2k+1]; from I = infinity, rank everything into P and recompute I until it settles

Each model returns the children (left, right) of every internal node as ("L", symbol) or
("I", creation index); the oracle's node ids are mapped the same way."""
import bisect
import ctypes
import random

import oracle

INF = 2**32 - 1


def sorted_leaves(w):
    """(weight, symbol) of the symbols with weight > 0, stably sorted by weight (458-498)"""
    return sorted(((x, s) for s, x in enumerate(w) if x > 0), key=lambda t: (t[0], t[1]))


def serial(leaves):
    L = [x for x, _ in leaves]
    n = len(L)
    I, kids = [], []
    lq = iq = 0
    for k in range(n - 1):
        pick = []
        for _ in range(2):
            if lq < n and (iq >= len(I) or L[lq] <= I[iq]):
                pick.append((L[lq], ("L", leaves[lq][1])))
                lq += 1
            else:
                pick.append((I[iq], ("I", iq)))
                iq += 1
        I.append(pick[0][0] + pick[1][0])
        kids.append((pick[0][1], pick[1][1]))
    return kids


def closed(leaves):
    n = len(leaves)
    L = [x for x, _ in leaves]
    if n < 2 or not L[0] + L[1] > L[-1]:
        return None
    ident = lambda i: ("L", leaves[i][1]) if i < n else ("I", i - n)
    return [(ident(2 * k), ident(2 * k + 1)) for k in range(n - 1)]


def fixed_point(leaves, max_rounds=400):
    n = len(leaves)
    L = [x for x, _ in leaves]
    I = [INF] * (n - 1)
    for rounds in range(1, max_rounds + 1):
        P = [None] * (2 * n - 1)
        for t, x in enumerate(L):   # a leaf after the internal nodes lighter than it
            P[t + bisect.bisect_left(I, x)] = (x, ("L", leaves[t][1]))
        for j, x in enumerate(I):   # an internal node after the leaves no heavier than it
            P[j + bisect.bisect_right(L, x)] = (x, ("I", j))
        nI = [INF if INF in (P[2 * k][0], P[2 * k + 1][0]) else P[2 * k][0] + P[2 * k + 1][0] for k in range(n - 1)]
        if nI == I:
            return [(P[2 * k][1], P[2 * k + 1][1]) for k in range(n - 1)], rounds
        I = nI
    return None, max_rounds


def reference(w):
    nodes = (ctypes.c_uint32 * (4 * 511))()
    real = oracle.orc().orc_huffman_tree((ctypes.c_uint32 * 256)(*w), 256, nodes)
    base = 256 + (256 - real)   # the oracle's first internal node id
    ident = lambda c: ("L", c) if c < 256 else ("I", c - base)
    return [(ident(nodes[4 * node + 2]), ident(nodes[4 * node + 3])) for node in range(base, base + real - 1)]


def histograms(count=600, seed=7):
    rng = random.Random(seed)
    for i in range(count):
        n = rng.choice([2, 3, 5, 17, 64, 65, 100, 200, 256])
        syms = rng.sample(range(256), n)
        kind = i % 5
        w = [0] * 256
        for s in syms:
            if kind == 0:
                w[s] = rng.randint(200, 300)                        # random bytes: balanced
            elif kind == 1:
                w[s] = int(50 * rng.paretovariate(1.1)) + 1         # heavy tail (text chars)
            elif kind == 2:
                w[s] = rng.choice([1, 2, 3, 5, 8])                 # many ties
            elif kind == 3:
                w[s] = rng.randint(1, 1 << 16)
            else:
                w[s] = 1 << rng.randint(0, 12)                    # powers of two: ties between leaves and nodes
        yield w


def test_serial_form_is_the_reference():
    for w in histograms():
        assert serial(sorted_leaves(w)) == reference(w)


def test_closed_form_where_it_applies():
    applied = 0
    for w in histograms():
        c = closed(sorted_leaves(w))
        if c is not None:
            applied += 1
            assert c == reference(w)
    assert applied > 100


def test_fixed_point_matches_and_settles():
    worst = 0
    for w in histograms():
        kids, rounds = fixed_point(sorted_leaves(w))
        assert kids == reference(w)
        worst = max(worst, rounds)
    assert worst <= 40   # k_tree's kJacobiMax: beyond it the kernel runs the serial merge
