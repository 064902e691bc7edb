"""Summarise tools/gpu_pmc.sh output (gpurun_out/pmc/p*/run_counter_collection.csv) into the
per-launch counter JSON bench.py reads (profiles/pmc_latest.json).

Per the MI355X_MICROARCH guide's HBM section: FETCH_SIZE (KB) under-reads wide coalesced reads on
gfx950 by 2x, so HBM read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE (KB) is taken as is. Each
counter group ran in its own rocprofv3 --pmc pass. Values are averaged over the timed launches of
the product render kernel (the non-instrumented variant: template COUNT = false).

usage: python tools/pmc_summary.py <pmc dir> <workload key> <out.json>
The workload key is bench.py's config.workload string; the summary also records the hash of the
kernel sources (bench.kernel_source_sha), so bench.py only reports `traffic` measured on the
kernel it is timing.
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from bench import kernel_source_sha  # noqa: E402

# the timed pass of an LDS-scene kernel (template: stack entry, GSTACK, LSCENE, COUNT = false, then the
# primitive-mix and wave-count instance flags, which vary with the scene)
KERNEL = "crt::dev::render_kernel<unsigned short, false, true, false,"


def main():
    src, workload, out = Path(sys.argv[1]), sys.argv[2], Path(sys.argv[3])
    vals = defaultdict(list)
    names = set()
    for f in sorted(src.glob("p*/run_counter_collection.csv")):
        for r in csv.DictReader(f.open()):
            name = r["Kernel_Name"].removeprefix("void ")
            if name.startswith(KERNEL):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                names.add(name.split("(")[0])
    if len(names) > 1:
        raise SystemExit(f"several timed kernel instances under {src}: {sorted(names)}")
    if not vals:
        raise SystemExit(f"no {KERNEL} rows under {src}")
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    res = {"workload": workload, "kernel": names.pop(), "kernel_source_sha": kernel_source_sha(),
           "launches": {k: len(v) for k, v in vals.items()}}
    res.update({k: avg[k] for k in sorted(avg)})
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        res["FETCH_SIZE_KB"] = avg["FETCH_SIZE"]
        res["WRITE_SIZE_KB"] = avg["WRITE_SIZE"]
        res["hbm_bytes_per_launch"] = int(round(2 * avg["FETCH_SIZE"] * 1024 + avg["WRITE_SIZE"] * 1024))
        res["correction"] = ("MI355X_MICROARCH.md HBM: FETCH_SIZE reads 1/2 of wide coalesced reads on "
                             "gfx950 -> x2; WRITE_SIZE taken as is; separate --pmc passes (tools/gpu_pmc.sh)")
    f64 = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")
    if "SQ_INSTS_VALU" in avg and "SQ_BUSY_CYCLES" in avg and all(k in avg for k in f64):
        # VALU issue utilization: a wave64 VALU instruction occupies a SIMD32 for 2 cycles, an f64
        # one for 4 (the f64 vector rate is half the f32 rate); SQ_BUSY_CYCLES counts cycles per SQ
        # (one per shader engine of 32 SIMDs), so the chip's SIMD-cycles are 32 x SQ_BUSY_CYCLES
        n64 = sum(avg[k] for k in f64)
        res["valu_issue_cycles"] = 2 * avg["SQ_INSTS_VALU"] + 2 * n64
        res["valu_issue_frac"] = res["valu_issue_cycles"] / (32 * avg["SQ_BUSY_CYCLES"])
    if "SQ_THREAD_CYCLES_VALU" in avg and "SQ_ACTIVE_INST_VALU" in avg:
        res["valu_lane_utilization"] = avg["SQ_THREAD_CYCLES_VALU"] / (64 * avg["SQ_ACTIVE_INST_VALU"])
    out.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
