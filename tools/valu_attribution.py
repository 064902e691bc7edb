"""Per-phase VALU instruction attribution of one render-kernel instance.

Static opcode mix per basic block of a `hipcc -S` listing (blocks split at labels and after branches;
the loop each block belongs to from LLVM's "in Loop: Header=" comments), times the dynamic
frequency of each phase's loop body from the instrumented pass (bench.py's `instrumented_counts`:
wave iterations of the walk, of the leaf filter, of the candidates' exact tests, of shading).
The phase loops are found by their loop header and by content:
  walk      the loop (ds_read_b128 / global_load of nodes) with v_fma_f32 and v_min3_f32, without its
            f64 fallback sub-blocks: x wave_iters_walk; the fallback: x wave_iters_slow
  pass1     the loop with v_pk_fma_f32 (the packed sphere filter): x wave_iters_leaf / 2
  pass2     the loop with v_rsq_f64 and v_ffbh_u32 (hit_sphere on the next candidate): x wave_iters_candidates
  rest      everything else (shade, path start, traversal set-up, draws): SQ_INSTS_VALU minus the above
Classes: f64, f32 (arith and transcendental), pk_f32, int (add/sub/mul/mad/cvt/mbcnt), cmp/cndmask,
min/max/med3, bit/shift (and/or/xor/bfe/lshl/lshr/bitop3/perm), mov/lane (mov, readlane, writelane).
The SQ_INSTS_VALU_* hardware classes count f32 / f64 add, mul, fma, trans, INT32, INT64, CVT; the rest
(cmp/cndmask, min/max, bit ops, movs, packed f32) is the counters' unclassified "other".
usage: python tools/valu_attribution.py listing.s kernel_substring bench.json [pmc.json]"""
import collections
import json
import re
import sys

CLASSES = ["f64", "f32", "pk_f32", "int", "cmp/cndmask", "min/max", "bit/shift", "mov/lane"]


def cls(op):
    if not op.startswith("v_"):
        return None
    if "f64" in op:
        return "f64"
    if op.startswith("v_pk_"):
        return "pk_f32"
    if op.startswith(("v_cmp", "v_cndmask")):
        return "cmp/cndmask"
    if op.startswith(("v_min", "v_max", "v_med")):
        return "min/max"
    if op.startswith(("v_bfe", "v_lshl", "v_lshr", "v_ashr", "v_alignbit", "v_bfi", "v_perm", "v_bitop",
                      "v_and", "v_or", "v_xor", "v_not", "v_bfrev")):
        return "bit/shift"
    if op.startswith(("v_mov", "v_readlane", "v_writelane", "v_readfirstlane", "v_accvgpr", "v_swap")):
        return "mov/lane"
    if "f32" in op or "f16" in op:
        return "f32"
    return "int"


def blocks_of(path, name):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and name in l and ":" in l.split(";")[0])
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur, header = [], None, None
    for l in lines[start + 1:end]:
        m = re.match(r"^(\.LBB\d+_\d+):(.*)", l)
        if m:
            h = re.search(r"Header=(BB\d+_\d+)", m.group(2))
            header = h.group(1) if h else ("BB" + m.group(1)[4:] if "Loop Header" in m.group(2) or "Parent Loop" in m.group(2) else None)
            cur = {"label": m.group(1), "loop": header, "ins": []}
            blocks.append(cur)
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        if cur is None:
            cur = {"label": "entry", "loop": None, "ins": []}
            blocks.append(cur)
        ins = s.split(";")[0].strip()
        cur["ins"].append(ins)
        if ins.startswith(("s_cbranch", "s_branch")):  # a new basic block after a branch
            cur = {"label": cur["label"] + "+", "loop": cur["loop"], "ins": []}
            blocks.append(cur)
    return blocks


def mix(ins_list):
    c = collections.Counter()
    for x in ins_list:
        k = cls(x.split()[0])
        if k:
            c[k] += 1
    return c


def main():
    path, name, bench = sys.argv[1], sys.argv[2], json.load(open(sys.argv[3]))
    pmc = json.load(open(sys.argv[4])) if len(sys.argv) > 4 else None
    cnt = bench["instrumented_counts"]["timed_walk"]
    blocks = blocks_of(path, name)
    loops = collections.defaultdict(list)
    for b in blocks:
        if b["loop"]:
            loops[b["loop"]].append(b)

    def has(bs, *ops):
        text = " ".join(x.split()[0] for b in bs for x in b["ins"])
        return all(o in text for o in ops)

    walk = next(bs for bs in loops.values() if has(bs, "v_fma_f32", "v_min3_f32") and not has(bs, "v_pk_fma_f32"))
    pass1 = next(bs for bs in loops.values() if has(bs, "v_pk_fma_f32"))
    pass2 = next(bs for bs in loops.values() if has(bs, "v_rsq_f64", "v_ffbh_u32"))  # 31 - clz(candidates)
    walk_main = [b for b in walk if not any("f64" in x.split()[0] for x in b["ins"])]
    walk_f64 = [b for b in walk if any("f64" in x.split()[0] for x in b["ins"])]
    # pass 2: every block of the loop, the root's divisions included (an upper bound: they run
    # where the discriminant admits a root in range, most candidates)
    pass2_main = pass2
    rows = [
        ("walk step", walk_main, cnt["wave_iters_walk"]),
        ("walk f64 fallback", walk_f64, cnt["wave_iters_slow"]),
        ("leaf pass 1 (pair)", pass1, cnt["wave_iters_leaf"] / 2),
        ("leaf pass 2 (candidate)", pass2_main, cnt["wave_iters_candidates"]),
    ]
    out, total = [], collections.Counter()
    print(f"{'phase':26s} {'iters':>10s} {'VALU/it':>8s} " + " ".join(f"{c:>11s}" for c in CLASSES) + f" {'dynamic':>10s}")
    for label, bs, it in rows:
        m = mix(x for b in bs for x in b["ins"])
        n = sum(m.values())
        dyn = {c: m[c] * it for c in CLASSES}
        total.update(dyn)
        out.append({"phase": label, "wave_iterations": it, "valu_per_iteration": n, "per_iteration": dict(m),
                    "dynamic": dyn})
        print(f"{label:26s} {it:10.3e} {n:8d} " + " ".join(f"{m[c]:11d}" for c in CLASSES) + f" {n * it:10.3e}")
    acc = sum(total.values())
    print(f"{'sum of the four':26s} {'':10s} {'':8s} " + " ".join(f"{total[c]:11.3e}" for c in CLASSES) + f" {acc:10.3e}")
    if pmc:
        insts = pmc["SQ_INSTS_VALU"]
        print(f"SQ_INSTS_VALU {insts:.3e}; the rest (shade, path start, traversal set-up, draws): {insts - acc:.3e}")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
