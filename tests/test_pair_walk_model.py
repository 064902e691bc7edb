"""A Python model of the sibling-pair walk's state machine (crt_device.hip walk_pairs: tokens of
a first node and its sibling or of one node alone, the sibling's token pushed or continued, the speculative round that records the first leaf
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
    """walk_pairs + leaf_step, one lane: token = (first node, alone). Without `alone` the step tests
    the first node and its sibling (the first one is the near child of their parent); an entered
    interior node continues as its near child's token, a leaf not processed now as (itself, alone):
    a re-test of its box."""
    sentinel = {"leaf": True, "near": float("-inf"), "hit": True, "prims": []}
    sibling = {}

    def reg(n):
        if not n["leaf"]:
            a, b = n["ch"]
            sibling[id(a)], sibling[id(b)] = b, a
            for c in n["ch"]:
                reg(c)
    reg(root)

    def tok_of(x):
        if x["leaf"]:
            return (x, True)
        a, b = x["ch"]
        return ((b if x["sw"] else a), False)  # the near child, with its sibling

    log, tmax, stack, cur = [], float("inf"), [], (root, True)
    while True:
        pref, run = None, True
        while run:
            if pref is not None and stop.random() < 0.3:
                break  # the wave's loop ends before this lane parks
            first, alone = cur
            second = None if alone else sibling[id(first)]
            e1 = enter(first, tmax)
            e2 = second is not None and enter(second, tmax)
            t1 = tok_of(first) if not first["leaf"] else (first, True)
            t2 = tok_of(second) if second is not None else None
            both, anyc = e1 and e2, e1 or e2
            X = first if e1 else second
            xi = anyc and not X["leaf"]
            leaf = anyc and X["leaf"]
            park = leaf and (pref is not None or (e1 and first is sentinel))
            tx = t1 if e1 else t2
            if leaf and pref is None:
                pref = tx
            if xi or park:
                cur = tx
                if both:
                    stack.append(t2)
            elif both:
                cur = t2
            else:
                cur = stack.pop() if stack else (sentinel, True)  # the guard level
            run = not park
        node = pref[0]
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
