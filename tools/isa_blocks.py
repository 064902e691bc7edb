"""Basic-block instruction counts of one kernel in a hipcc -S listing (loops marked by back edges).
usage: python tools/isa_blocks.py file.s kernel_symbol_substring"""
import re
import sys

path, name = sys.argv[1], sys.argv[2]
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and name in l and l.rstrip().endswith(name) is False and ":" in l)
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.section") or lines[i].startswith(".Lfunc_end"))
blocks, cur = [], None
for l in lines[start:end]:
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        cur = {"label": m.group(1), "ins": []}
        blocks.append(cur)
        continue
    s = l.strip()
    if not s or s.startswith(";") or s.startswith("."):
        continue
    if cur is None:
        cur = {"label": "entry", "ins": []}
        blocks.append(cur)
    cur["ins"].append(s.split(";")[0].strip())
pos = {b["label"]: i for i, b in enumerate(blocks)}
for i, b in enumerate(blocks):
    ins = b["ins"]
    v = sum(1 for x in ins if x.startswith("v_"))
    f64 = sum(1 for x in ins if x.startswith("v_") and "f64" in x.split()[0])
    s_ = sum(1 for x in ins if x.startswith("s_"))
    ds = sum(1 for x in ins if x.startswith("ds_"))
    gl = sum(1 for x in ins if x.startswith(("global_", "buffer_", "flat_", "scratch_")))
    back = [x.split()[-1] for x in ins if x.startswith("s_cbranch") or x.startswith("s_branch")]
    back = [t for t in back if t in pos and pos[t] <= i]
    print(f"{i:4d} {b['label']:14s} n={len(ins):4d} v={v:4d} f64={f64:3d} s={s_:3d} ds={ds:2d} mem={gl:2d} {'BACK->' + ','.join(back) if back else ''}")
