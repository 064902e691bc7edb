"""The device node order of crt_stage_gpu.hip (node_positions) restated in numpy and checked against
the host staging's own algorithm (crt_host.cpp stage(): a breadth-first top of kTopBfs nodes, then
each unexpanded node's subtree depth-first with the two children of a node side by side) on the
preorder arrays of real scenes, built on the host here (no GPU needed). The GPU tests
(test_gpu_stage.py) then compare the device-staged image with the host-staged one byte for byte."""
import numpy as np
import pytest

TOP_BFS = 1024


def host_positions(nodes):
    """stage()'s order, transcribed: device position of every preorder node."""
    nn = len(nodes)
    count, index = nodes["count"], nodes["index"]

    def interior(i):
        return count[i] == 0 and i + 1 < nn

    bfs, q = [0], 0
    while q < len(bfs) and len(bfs) < TOP_BFS:
        i = bfs[q]
        if interior(i):
            bfs += [i + 1, int(index[i])]
        q += 1
    todo = [bfs[r] for r in range(len(bfs) - 1, q - 1, -1)]
    while todo:
        i = todo.pop()
        if not interior(i):
            continue
        l, r = i + 1, int(index[i])
        bfs += [l, r]
        todo += [r, l]
    pos = np.zeros(nn, np.int64)
    for k, i in enumerate(bfs):
        pos[i] = 0 if k == 0 else k + 1
    return pos


def path_positions(nodes):
    """node_positions' rule: the top table from the breadth-first top, then for every other node
    the walk from its frontier ancestor (children at c, c + 1; the left subtree from c + 2; the
    right subtree from c + 1 + size(left), size(left) = right - left)."""
    nn = len(nodes)
    count, index = nodes["count"], nodes["index"].astype(np.int64)

    def interior(i):
        return count[i] == 0 and i + 1 < nn

    bfs, q = [0], 0
    while q < len(bfs) and len(bfs) < TOP_BFS:
        if interior(bfs[q]):
            bfs += [bfs[q] + 1, int(index[bfs[q]])]
        q += 1
    tpos, tbase = {}, {}
    c = len(bfs)
    for k, i in enumerate(bfs):
        tpos[i] = 0 if k == 0 else k + 1
        if k >= q and interior(i):
            tbase[i] = c
            e = i
            while interior(e):
                e = int(index[e])
            c += e - i
    pos = np.zeros(nn, np.int64)
    for i in range(nn):
        if i in tpos:
            pos[i] = tpos[i]
            continue
        p = 0
        while True:
            ch = p + 1 if i < index[p] else int(index[p])
            if ch not in tpos:
                break
            p = ch
        base = tbase[p]
        while True:
            l, r = p + 1, int(index[p])
            if i == l or i == r:
                pos[i] = (base + 1 if i == r else base) + 1
                break
            if i < r:
                p, base = l, base + 2
            else:
                p, base = r, base + 1 + (r - l)
    return pos


@pytest.mark.parametrize("name,seed,ml", [("rtow_final", 42, 12), ("rtow_final", 7, 1), ("cornell", None, 12),
                                          ("christmas_tree", None, 12), ("dance_floor", None, 4),
                                          ("bvh_pathological", None, 12), ("config1", None, 12)])
def test_path_rule_equals_stage_order(crt, name, seed, ml):
    nodes, _ = crt.GpuScene(crt.SceneData.named(name, seed), max_prims_in_node=ml).export_bvh()
    want = host_positions(nodes)
    assert np.array_equal(path_positions(nodes), want)
    # a permutation of [0, nn + 1) without position 1 (the pad), pairs of siblings side by side
    assert sorted(want.tolist()) == [0] + list(range(2, len(nodes) + 1))
