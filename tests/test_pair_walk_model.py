"""A Python model of the sibling-pair walk's state machine (crt_device.hip walk_pairs: tokens,
skip kinds, the far token pushed or continued, the speculative round that records the first leaf
and parks at the second as a re-test token) against the reference's DFS (bvh.h:617-712). Random
trees whose node test is monotone in t_max and in containment (a child is entered only where its
parent is, at any t_max where the parent is: the property the f32 / f64 node test has, walk_pairs'
header), random primitive hits: the sequence of (leaf, t_max at its primitive tests) must be the
reference's, including rounds the wave ends before the lane parks. CPU only; the GPU parity tests
run the kernel itself."""
import random

import pytest


def make_tree(rng, depth, near, hit):
    hit = hit and rng.random() < 0.85
    if depth > 8 or (depth > 1 and rng.random() < 0.25):
        prims = [rng.uniform(near, near + 10) if rng.random() < 0.6 else None for _ in range(rng.randint(1, 3))]
        return {"leaf": True, "near": near, "hit": hit, "prims": prims}
    ch = [make_tree(rng, depth + 1, near + rng.choice([0.0, rng.uniform(0, 3)]), hit) for _ in range(2)]
    return {"leaf": False, "near": near, "hit": hit, "ch": ch, "sw": rng.random() < 0.5}


def enter(n, tmax):
    return n["hit"] and n["near"] < tmax


def reference(root):
    """BVH::hit_by's loop: pop, test at the current t_max, leaf primitives shrink t_max, near child
    first."""
    log, tmax, stack = [], float("inf"), [root]
    while stack:
        n = stack.pop()
        if not enter(n, tmax):
            continue
        if n["leaf"]:
            log.append((id(n), tmax))
            for t in n["prims"]:
                if t is not None and t < tmax:
                    tmax = t
        else:
            a, b = n["ch"]
            near, far = (b, a) if n["sw"] else (a, b)
            stack.append(far)
            stack.append(near)
    return log


def pair_walk(root, stop):
    """walk_pairs + leaf_step, one lane: token = (pair, kind), kind 0 / 1 both children (1: right
    first), 2 the left child alone, 3 the right one alone."""
    sentinel = {"leaf": True, "near": float("-inf"), "hit": True, "prims": []}
    pad = {"leaf": True, "near": 0.0, "hit": False, "prims": []}
    pairs = {"root": [root, pad], "sent": [sentinel, None]}

    def reg(n):
        if not n["leaf"]:
            pairs[id(n)] = n["ch"]
            for c in n["ch"]:
                reg(c)
    reg(root)

    def tok_of(x, pair, is_r):
        if x["leaf"]:
            return (pair, 3 if is_r else 2)
        return (id(x), 1 if x["sw"] else 0)

    log, tmax, stack, cur = [], float("inf"), [], ("root", 2)
    while True:
        pref, run = None, True
        while run:
            if pref is not None and stop.random() < 0.3:
                break  # the wave's loop ends before this lane parks
            pair, kind = cur
            L, R = pairs[pair]
            ml, mr, sw = kind != 3, kind != 2, kind == 1
            el = ml and enter(L, tmax)
            er = mr and R is not None and enter(R, tmax)
            tl = tok_of(L, pair, False)
            tr = tok_of(R, pair, True) if R is not None else None
            xr = er and (sw or not el)
            both, anyc = el and er, el or er
            X = R if xr else L
            xi = anyc and not X["leaf"]
            leaf = anyc and X["leaf"]
            park = leaf and (pref is not None or ((not xr) and L is sentinel))
            tf = tl if sw else tr
            tx = tr if xr else tl
            if leaf and pref is None:
                pref = tx
            if xi or park:
                cur = tx
                if both:
                    stack.append(tf)
            elif both:
                cur = tf
            else:
                cur = stack.pop() if stack else ("sent", 2)  # the guard level
            run = not park
        pair, kind = pref
        node = pairs[pair][1 if kind == 3 else 0]
        if node is sentinel:
            return log
        log.append((id(node), tmax))
        for t in node["prims"]:
            if t is not None and t < tmax:
                tmax = t


@pytest.mark.parametrize("seed", range(4))
def test_pair_walk_tests_the_reference_leaves_in_order(seed):
    rng, stop = random.Random(seed), random.Random(100 + seed)
    total = 0
    for _ in range(2500):
        root = make_tree(rng, 0, 0.0, True)
        want = reference(root)
        assert pair_walk(root, stop) == want
        total += len(want)
    assert total > 10000
